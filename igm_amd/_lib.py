"""ctypes binding of libigmhip.so (include/igm_hip.h).

This is the Python side of the drop-in boundary: the exact stub a maintainer
would add to the reference.  There is no fallback: if the
HIP library is missing or the GPU call fails, the error propagates as
RuntimeError, like a failed LAMMPS run in the reference (lammps.py:453-457).
"""
import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('IGM_HIP_LIB', os.path.join(HERE, 'lib', 'libigmhip.so'))

IGM_OK = 0
IGM_E_INVALID = -1
IGM_E_HIP = -2
IGM_E_NOMEM = -3
IGM_E_OVERFLOW = -4
IGM_E_UNSUPPORTED = -5
IGM_DEVICE_PTRS = 0x1
IGM_ASYNC = 0x2
IGM_F32_PATH = 0x4
IGM_MSTEP_FORCE_GLOBAL = 0x1  # igm_mstep_params.flags: HBM-resident kernels even when LDS fits
IGM_MSTEP_STRUCT_FLAGS = 0x2  # igm_mstep_params.flags: atom_flags is (nstruct, natom)

IGM_MAX_STAGES = 16
IGM_MAX_ENVELOPES = 4

IGM_ATOM_BEAD = 0x1
IGM_ATOM_FIXED = 0x2
IGM_ATOM_ENV0 = 0x10
IGM_ENV_ELLIPSOID = 0
IGM_ENV_VOLUME = 1

# numpy views of the ABI structs (packed exactly like the C layouts)
pair_dtype = np.dtype([('i', '<i4'), ('j', '<i4'), ('pwish', '<f8'), ('plast', '<f8')])
row_dtype = np.dtype([('row', '<i4'), ('col', '<i4'), ('dist', '<f4'), ('prob', '<f4')])
damid_row_dtype = np.dtype([('loc', '<i4'), ('dist', '<f4'), ('prob', '<f4')])
result_dtype = np.dtype([('ad', '<f8'), ('p', '<f8'), ('pnow', '<f8'), ('o', '<i4'), ('nrows', '<i4')])
bond_dtype = np.dtype([('i', '<u4'), ('j', '<u4'), ('r0', '<f4'), ('k', '<f4')])
optinfo_dtype = np.dtype([('final_energy', '<f8'), ('pair_energy', '<f8'), ('bond_energy', '<f8'),
                          ('env_energy', '<f8', (IGM_MAX_ENVELOPES,)), ('temp', '<f8'),
                          ('einitial', '<f8'), ('fnorm_final', '<f8'),
                          ('cg_iters', '<i4'), ('cg_evals', '<i4'), ('stop_reason', '<i4'), ('nrebuild', '<i4')])
assert pair_dtype.itemsize == 24 and row_dtype.itemsize == 16 and result_dtype.itemsize == 32
assert bond_dtype.itemsize == 16

LOWER_BOUND_BIT = np.uint32(1 << 31)


class MStepParams(ctypes.Structure):
    _fields_ = [
        ('nstages', ctypes.c_int32),
        ('mdsteps', ctypes.c_int32 * IGM_MAX_STAGES),
        ('tstart', ctypes.c_double * IGM_MAX_STAGES),
        ('tstop', ctypes.c_double * IGM_MAX_STAGES),
        ('evfactor', ctypes.c_double * IGM_MAX_STAGES),
        ('envfactor', ctypes.c_double * IGM_MAX_STAGES),
        ('relax_steps', ctypes.c_int32),
        ('relax_temperature', ctypes.c_double),
        ('relax_max_velocity', ctypes.c_double),
        ('timestep', ctypes.c_double),
        ('max_velocity', ctypes.c_double),
        ('t_window', ctypes.c_double),
        ('t_fraction', ctypes.c_double),
        ('etol', ctypes.c_double),
        ('ftol', ctypes.c_double),
        ('max_cg_iter', ctypes.c_int32),
        ('max_cg_eval', ctypes.c_int32),
        ('dmax', ctypes.c_double),
        ('evfactor_base', ctypes.c_double),
        ('skin', ctypes.c_double),
        ('nenvelopes', ctypes.c_int32),
        ('env_semiaxes', (ctypes.c_double * 3) * IGM_MAX_ENVELOPES),
        ('env_k', ctypes.c_double * IGM_MAX_ENVELOPES),
        ('neigh_capacity', ctypes.c_int32),
        ('flags', ctypes.c_int32),
        ('env_kind', ctypes.c_int32 * IGM_MAX_ENVELOPES),
    ]


class VolumeMap(ctypes.Structure):
    _fields_ = [
        ('body_idx', ctypes.c_int32),
        ('nvoxel', ctypes.c_int32 * 3),
        ('center', ctypes.c_float * 3),
        ('origin', ctypes.c_float * 3),
        ('grid', ctypes.c_float * 3),
        ('voxels', ctypes.c_void_p),
    ]


_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_f64 = ctypes.c_double

# name -> (restype, argtypes): every symbol declared in include/igm_hip.h
SIGNATURES = {
    'igm_ctx_create': (_i32, [_i32, ctypes.POINTER(_vp)]),
    'igm_ctx_destroy': (None, [_vp]),
    'igm_last_error': (ctypes.c_char_p, [_vp]),
    'igm_ctx_set_stream': (_i32, [_vp, _vp]),
    'igm_ctx_synchronize': (_i32, [_vp]),
    'igm_last_kernel_ms': (_f64, [_vp, ctypes.c_char_p]),
    'igm_mstep_last_profile': (_i32, [_vp, _vp]),
    'igm_version': (ctypes.c_char_p, []),
    'igm_astep_actdist': (_i32, [_vp, _u32, _vp, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _i64, _f64, _i32,
                                 _vp, _vp, _i64, ctypes.POINTER(_i64)]),
    'igm_astep_update_plast': (_i32, [_vp, _u32, _vp, _i64, _vp]),
    'igm_damid_actdist': (_i32, [_vp, _u32, _vp, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i32, _i32, _f64,
                                 _i32, _vp, _vp, _vp, _i64, ctypes.POINTER(_i64)]),
    'igm_damid_select': (_i32, [_vp, _u32, _i32, _i32, _vp, _vp, _vp, _i64, _vp, _f64, _u32, _vp, _vp, _vp]),
    'igm_fish_assign': (_i32, [_vp, _u32, _vp, _i32, _i32, _vp, _vp, _i32, _i32, _vp, _i32, _vp, _vp, _vp, _vp,
                               _vp, _vp]),
    'igm_contact_map': (_i32, [_vp, _u32, _vp, _i32, _i32, _vp, _f64, _vp]),
    'igm_contact_map_haploid': (_i32, [_vp, _u32, _vp, _i32, _i32, _vp, _f64, _vp, _vp, _i32, _vp]),
    'igm_polymer_assign': (_i32, [_vp, _u32, _vp, _i32, _i32, _vp, _i32, _vp, _i32, _vp, _vp, _vp, _vp]),
    'igm_sprite_assign': (_i32, [_vp, _u32, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _i32,
                                 _vp, _vp, _vp, _vp]),
    'igm_mstep_run': (_i32, [_vp, _u32, ctypes.POINTER(MStepParams), _i32, _i32, _vp, _vp, _vp, _vp, _i64,
                             _vp, _vp, _vp, _vp]),
    'igm_mstep_forces': (_i32, [_vp, _u32, ctypes.POINTER(MStepParams), _i32, _i32, _vp, _vp, _vp, _vp, _i64,
                                _vp, _vp, _f64, _f64, _vp, _vp]),
    'igm_mstep_md': (_i32, [_vp, _u32, ctypes.POINTER(MStepParams), _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i64,
                            _vp, _vp, _f64, _f64, _f64, _f64, _f64, _i32]),
    'igm_velocity_create': (_i32, [_vp, _u32, _i32, _i32, _vp, _vp, _f64, _vp]),
    'igm_hic_select': (_i32, [_vp, _u32, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _f64, _f64,
                              _i32, _i32, _vp, _vp, _vp, ctypes.POINTER(_i64)]),
    'igm_population_transpose': (_i32, [_vp, _u32, _i32, _i32, _i32, _vp, _vp, _i32]),
    'igm_mstep_set_volumes': (_i32, [_vp, _i32, _vp, _vp, _i32]),
    'igm_mstep_violations': (_i32, [_vp, _u32, ctypes.POINTER(MStepParams), _i32, _i32, _vp, _vp, _vp,
                                    _vp, _vp, _i64, _vp, _vp, _vp, _i32, _vp, _vp, _f64, _vp]),
}

_lib = None
_lock = threading.Lock()


def load():
    """Load libigmhip.so (raises ImportError if it was not built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError('libigmhip.so not found at %s -- build it with `python -m igm_amd.build` '
                                  '(the HIP path has no CPU fallback)' % LIB_PATH)
            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in SIGNATURES.items():
                try:
                    f = getattr(lib, name)
                except AttributeError:
                    continue  # tests/test_capi.py asserts that every declared symbol is exported
                f.restype = res
                f.argtypes = args
            _lib = lib
    return _lib


def ptr(a):
    """Address of a numpy array / torch tensor / None."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags['C_CONTIGUOUS'], 'arrays passed to libigmhip must be C-contiguous'
        return a.ctypes.data
    if hasattr(a, 'data_ptr'):
        return a.data_ptr()
    raise TypeError('cannot take the address of %r' % type(a))


class Context(object):
    """One igm_ctx (one GPU, one host thread)."""

    def __init__(self, device=0):
        self.lib = load()
        h = _vp()
        rc = self.lib.igm_ctx_create(int(device), ctypes.byref(h))
        if rc != IGM_OK:
            raise RuntimeError('igm_ctx_create(device=%d) failed with code %d (no HIP device?)' % (device, rc))
        self.h = h
        self.device = device

    def check(self, rc, what):
        if rc != IGM_OK:
            msg = self.lib.igm_last_error(self.h)
            raise RuntimeError('%s failed (code %d): %s' % (what, rc, msg.decode() if msg else ''))

    def set_stream(self, stream_handle):
        self.check(self.lib.igm_ctx_set_stream(self.h, stream_handle), 'igm_ctx_set_stream')

    def synchronize(self):
        self.check(self.lib.igm_ctx_synchronize(self.h), 'igm_ctx_synchronize')

    def kernel_ms(self, name):
        return self.lib.igm_last_kernel_ms(self.h, name.encode())

    def mstep_profile(self):
        """cycle counters of the last anneal launch (IGM_PROF=1): dict of sums."""
        out = (ctypes.c_ulonglong * 6)()
        self.check(self.lib.igm_mstep_last_profile(self.h, out), 'igm_mstep_last_profile')
        return dict(zip(('build_cycles', 'force_cycles', 'rest_cycles', 'evaluations', 'builds', 'walk_cycles'),
                        list(out)))

    def close(self):
        if getattr(self, 'h', None):
            self.lib.igm_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_contexts = {}


def context(device=0):
    """Process-wide context per device (lazily created)."""
    c = _contexts.get(device)
    if c is None:
        c = _contexts[device] = Context(device)
    return c
