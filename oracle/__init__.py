"""ORACLE -- test infrastructure only.

CPU restatements of the reference's hot path (see the headers of
actdist_ref.c / mstep_ref.c for the reference file:line each follows).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package; the product (igm_amd) never does.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, 'liboracle.so')

pair_dtype = np.dtype([('i', '<i4'), ('j', '<i4'), ('pwish', '<f8'), ('plast', '<f8')])
row_dtype = np.dtype([('row', '<i4'), ('col', '<i4'), ('dist', '<f4'), ('prob', '<f4')])
result_dtype = np.dtype([('ad', '<f8'), ('p', '<f8'), ('pnow', '<f8'), ('o', '<i4'), ('nrows', '<i4')])

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.check_call(['make', '-C', HERE, '-s'])
        _lib = ctypes.CDLL(LIB)
        _lib.oracle_actdist.restype = ctypes.c_int64
        _lib.oracle_actdist.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]
    return _lib


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def actdist(xyz, radii, copy_ptr, copy_idx, chrom, pairs, contact_range=2.0, it_corr=1, nthreads=1):
    """Reference-semantics A-step on the CPU.  Returns (rows, per_pair)."""
    xyz = _c(xyz, np.float32)
    radii = _c(radii, np.float32)
    copy_ptr = _c(copy_ptr, np.int32)
    copy_idx = _c(copy_idx, np.int32)
    chrom = _c(chrom, np.int32)
    pairs = np.ascontiguousarray(pairs, dtype=pair_dtype)
    nbead, S = xyz.shape[0], xyz.shape[1]
    res = np.zeros(len(pairs), result_dtype)
    L = lib()
    args = [xyz.ctypes.data, nbead, S, radii.ctypes.data, copy_ptr.ctypes.data, copy_idx.ctypes.data,
            len(copy_ptr) - 1, chrom.ctypes.data, pairs.ctypes.data, len(pairs), float(contact_range),
            int(it_corr), res.ctypes.data]
    total = L.oracle_actdist(*(args + [None, 0, int(nthreads)]))
    rows = np.zeros(total, row_dtype)
    L.oracle_actdist(*(args + [rows.ctypes.data, total, int(nthreads)]))
    return rows, res
