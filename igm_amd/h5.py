"""ctypes binding of the native HDF5-subset reader/writer (include/igm_io.h,
csrc/h5io.cpp, linked into libigmhip.so): the h5py calls IGM's steps make on its
population files, without h5py/libhdf5 (not importable here).

    with File(path) as f:          # h5py.File(path, 'r')
        f.keys('index')            # list(f['index'].keys())
        f.read('coordinates')      # f['coordinates'][:]
        f.read('summary')          # f['summary'][()] of a vlen str -> str
        f.attrs('/')               # dict(f.attrs)
    write(path, {'coordinates': arr, 'index': {'chrom': a}, '@nstruct': np.int64(S),
                 'summary': 'json text'})   # h5py create_dataset / create_group / attrs

Keys starting with '@' are attributes of the enclosing group; str values are
variable-length strings (h5py's str), numpy 'S<n>' arrays fixed-length strings.
Errors raise OSError with the library's message, like h5py.
"""
import ctypes

import numpy as np

from . import _lib

INT, FLOAT, STRING, VLSTR = 0, 1, 3, 9
MAXRANK = 8


class Info(ctypes.Structure):
    _fields_ = [('cls', ctypes.c_int32), ('size', ctypes.c_int32), ('is_signed', ctypes.c_int32),
                ('rank', ctypes.c_int32), ('dims', ctypes.c_int64 * MAXRANK), ('nelem', ctypes.c_int64),
                ('layout', ctypes.c_int32), ('nfilter', ctypes.c_int32), ('data_offset', ctypes.c_int64)]


_vp, _cp, _i32, _i64, _sz = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
# every function declared in include/igm_io.h
SIGNATURES = {
    'igm_io_last_error': (_cp, []),
    'igm_h5_open': (_i32, [_cp, ctypes.POINTER(_vp)]),
    'igm_h5_close': (_i32, [_vp]),
    'igm_h5_list': (_i32, [_vp, _cp, _vp, _sz, ctypes.POINTER(_sz)]),
    'igm_h5_attr_names': (_i32, [_vp, _cp, _vp, _sz, ctypes.POINTER(_sz)]),
    'igm_h5_info_of': (_i32, [_vp, _cp, _cp, ctypes.POINTER(Info)]),
    'igm_h5_read': (_i32, [_vp, _cp, _cp, _vp, _sz]),
    'igm_h5_read_vlstr': (_i32, [_vp, _cp, _cp, _i64, _vp, _sz, ctypes.POINTER(_sz)]),
    'igm_h5w_create': (_i32, [_cp, ctypes.POINTER(_vp)]),
    'igm_h5w_group': (_i32, [_vp, _cp]),
    'igm_h5w_dataset': (_i32, [_vp, _cp, _i32, _i32, _i32, _i32, _vp, _vp]),
    'igm_h5w_vlstr': (_i32, [_vp, _cp, _cp, _cp, _sz]),
    'igm_h5w_attr': (_i32, [_vp, _cp, _cp, _i32, _i32, _i32, _i32, _vp, _vp]),
    'igm_h5w_close': (_i32, [_vp]),
    'igm_h5w_abort': (_i32, [_vp]),
}
_io = None


def lib():
    global _io
    if _io is None:
        L = _lib.load()
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _io = L
    return _io


def _check(rc, what):
    if rc != 0:
        raise OSError('%s: %s' % (what, lib().igm_io_last_error().decode(errors='replace')))


def _b(s):
    return None if s is None else s.encode()


def _numpy_dtype(info):
    if info.cls == INT:
        return np.dtype('<%s%d' % ('i' if info.is_signed else 'u', info.size))
    if info.cls == FLOAT:
        return np.dtype('<f%d' % info.size)
    if info.cls == STRING:
        return np.dtype('S%d' % info.size)
    return None


class File(object):
    """Read access to an HDF5 file (h5py.File(path, 'r') for the calls IGM makes)."""

    def __init__(self, path):
        h = _vp()
        _check(lib().igm_h5_open(_b(str(path)), ctypes.byref(h)), 'open %s' % path)
        self.h, self.path = h, str(path)

    def close(self):
        if self.h:
            lib().igm_h5_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _names(self, fn, path):
        need = _sz()
        _check(fn(self.h, _b(path), None, 0, ctypes.byref(need)), 'list %s' % path)
        buf = ctypes.create_string_buffer(need.value)
        _check(fn(self.h, _b(path), buf, need.value, ctypes.byref(need)), 'list %s' % path)
        s = buf.value.decode()
        return s.split('\n') if s else []

    def keys(self, group='/'):
        """member names; groups end with '/'"""
        return self._names(lib().igm_h5_list, group)

    def info(self, path, attr=None):
        inf = Info()
        _check(lib().igm_h5_info_of(self.h, _b(path), _b(attr), ctypes.byref(inf)), 'info %s' % path)
        return inf

    def shape(self, path):
        inf = self.info(path)
        return tuple(inf.dims[d] for d in range(inf.rank))

    def read(self, path, attr=None):
        """the whole dataset (or attribute) as a numpy array / scalar; vlen strings as str"""
        inf = self.info(path, attr)
        shape = tuple(inf.dims[d] for d in range(inf.rank))
        if inf.cls == VLSTR:
            out = []
            for k in range(inf.nelem):
                n = _sz()
                _check(lib().igm_h5_read_vlstr(self.h, _b(path), _b(attr), k, None, 0, ctypes.byref(n)),
                       'read %s' % path)
                buf = ctypes.create_string_buffer(max(n.value, 1))
                _check(lib().igm_h5_read_vlstr(self.h, _b(path), _b(attr), k, buf, n.value, ctypes.byref(n)),
                       'read %s' % path)
                out.append(buf.raw[:n.value].decode())
            return out[0] if inf.rank == 0 else np.array(out, dtype=object).reshape(shape)
        try:
            a = np.empty(shape, _numpy_dtype(inf))
        except MemoryError:
            raise OSError('read %s: %d elements cannot be allocated (corrupt extent?)' % (path, inf.nelem))
        _check(lib().igm_h5_read(self.h, _b(path), _b(attr), a.ctypes.data if a.size else None, a.nbytes),
               'read %s' % path)
        return a[()] if inf.rank == 0 else a

    def attrs(self, path='/'):
        return {n: self.read(path, n) for n in self._names(lib().igm_h5_attr_names, path)}

    def data_offset(self, path):
        """file offset of a contiguous, unfiltered dataset's raw data (for an in-place
        np.memmap), or None"""
        off = self.info(path).data_offset
        return None if off < 0 else int(off)


def _put(w, path, name, value, attr):
    full = (path.rstrip('/') + '/' + name) if not attr else path
    if isinstance(value, str):
        _check(lib().igm_h5w_vlstr(w, _b(full), _b(name) if attr else None, _b(value), len(value.encode())),
               'write %s' % full)
        return
    a = np.asarray(value)
    a = a if a.flags['C_CONTIGUOUS'] else a.copy(order='C')  # (ascontiguousarray would make 0-d arrays 1-d)
    if a.dtype.kind in 'iub':
        if a.dtype.kind == 'b':
            a = a.astype(np.int8)
        cls, signed = INT, int(a.dtype.kind == 'i')
    elif a.dtype.kind == 'f':
        cls, signed = FLOAT, 0
    elif a.dtype.kind == 'S':
        cls, signed = STRING, 0
    else:
        raise TypeError('cannot write %s of dtype %s' % (full, a.dtype))
    a = a.astype(a.dtype.newbyteorder('<'), copy=False)
    dims = (ctypes.c_int64 * max(a.ndim, 1))(*a.shape)
    data = a.ctypes.data if a.size else None
    if attr:
        _check(lib().igm_h5w_attr(w, _b(path), _b(name), cls, a.dtype.itemsize, signed, a.ndim, dims, data),
               'write %s@%s' % (path, name))
    else:
        _check(lib().igm_h5w_dataset(w, _b(full), cls, a.dtype.itemsize, signed, a.ndim, dims, data),
               'write %s' % full)


def _write_group(w, path, tree):
    if path != '/':
        _check(lib().igm_h5w_group(w, _b(path)), 'group %s' % path)
    for k, v in tree.items():
        if k.startswith('@'):
            continue
        if isinstance(v, dict):
            _write_group(w, path.rstrip('/') + '/' + k, v)
        else:
            _put(w, path, k, v, False)
    for k, v in tree.items():
        if k.startswith('@'):
            _put(w, path, k[1:], v, True)


def write(path, tree):
    """Write a new file (replacing any) from a nested dict (see the module doc)."""
    w = _vp()
    _check(lib().igm_h5w_create(_b(str(path)), ctypes.byref(w)), 'create %s' % path)
    try:
        _write_group(w, '/', tree)
    except Exception:
        lib().igm_h5w_abort(w)
        raise
    _check(lib().igm_h5w_close(w), 'write %s' % path)
