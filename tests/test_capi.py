"""The C-ABI library loads and exports every symbol include/igm_hip.h declares
(no compute calls: runs without a GPU)."""
import ctypes
import os
import re

from conftest import ROOT


def declared_functions(header='igm_hip.h'):
    src = open(os.path.join(ROOT, 'include', header)).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    names = re.findall(r'^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_ ]*[\s\*]+(igm_[a-z0-9_]+)\s*\(', src, flags=re.M)
    return sorted(set(names))


def test_header_declares_entry_points():
    names = declared_functions()
    for n in ('igm_ctx_create', 'igm_astep_actdist', 'igm_mstep_run', 'igm_hic_select',
              'igm_mstep_violations', 'igm_mstep_forces', 'igm_mstep_md'):
        assert n in names


def test_library_exports_all_declared_symbols():
    from igm_amd import _lib
    lib = _lib.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, 'libigmhip.so is missing %s' % missing
    assert set(declared_functions()) == set(_lib.SIGNATURES), 'ctypes signature table out of sync with header'
    assert lib.igm_version().decode().startswith('igm_amd')


def test_abi_struct_sizes():
    from igm_amd import _lib
    assert _lib.pair_dtype.itemsize == 24
    assert _lib.row_dtype.itemsize == 16
    assert _lib.result_dtype.itemsize == 32
    assert _lib.bond_dtype.itemsize == 16
    assert ctypes.sizeof(_lib.MStepParams) > 0


def test_no_gpu_means_loud_failure():
    """Without a HIP device the context cannot be created: the product raises
    instead of falling back to a CPU path."""
    import pytest
    import torch
    from igm_amd import _lib
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(RuntimeError):
        _lib.Context(0)


def test_io_library_exports_all_declared_symbols():
    """include/igm_io.h (the native .hss / actdist.hdf5 I/O) is exported by the same
    library and bound symbol for symbol in igm_amd.h5"""
    from igm_amd import _lib, h5
    lib = _lib.load()
    names = declared_functions('igm_io.h')
    assert 'igm_h5_open' in names and 'igm_h5w_close' in names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, 'libigmhip.so is missing %s' % missing
    assert set(names) == set(h5.SIGNATURES)
    h5.lib()
