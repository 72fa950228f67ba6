"""The native HDF5 writer pinned by libhdf5 itself.

This image has h5py 3.3.0 over libhdf5 1.10.6 under /opt/conda/bin/python3.9 (the
interpreter tests/golden/make_golden*.py use).  Each test writes IGM files with this
package -- the .hss a ModelingStep reduce leaves behind (coordinates updated in place
through the memory map, then the summary/violation rewrite of update_hss), the
actdist.hdf5 of ActivationDistanceStep.reduce (ActivationDistanceStep.py:285-289), and
a file holding every type/shape the writer supports -- then opens them with h5py in a
child process and compares every dataset and attribute, value and type, with what this
package meant to write.  The reverse direction: h5py writes a population the way
ModelingStep.reduce's h5repack leaves it (coordinates gzip-chunked
CHUNK = min(1e6/S/3, N) x S x 3, ModelingStep.py:753-762) and the native reader and
the Step layer's memory map read it.

Skipped where /opt/conda/bin/python3.9 or its h5py is absent (the GPU box)."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN
from igm_amd import h5, hss
from igm_amd import steps as ST

PY39 = '/opt/conda/bin/python3.9'


def _have_h5py():
    if not os.path.exists(PY39):
        return False
    return subprocess.run([PY39, '-c', 'import h5py'], stdout=subprocess.DEVNULL,
                          stderr=subprocess.DEVNULL).returncode == 0


pytestmark = pytest.mark.skipif(not _have_h5py(), reason='no h5py interpreter in this image')

# Child: every dataset and attribute of a file as {path: {'kind', 'dtype', 'shape', ...}}
# plus the raw values in an .npz (numeric / fixed strings) or the JSON (vlen strings).
DUMP = r'''
import json, sys
import h5py, numpy as np
src, out = sys.argv[1], sys.argv[2]
meta, arrays = {}, {}
def put(key, v, where, dt=None):
    if isinstance(v, (bytes, str)) and not isinstance(v, np.ndarray):
        sd = h5py.check_string_dtype(dt) if dt is not None else None
        meta[key] = {'kind': where, 'str': v.decode() if isinstance(v, bytes) else v,
                     'vlen': sd is not None and sd.length is None}
        return
    a = np.asarray(v)
    if a.dtype.kind == 'O':
        meta[key] = {'kind': where, 'str': a[()].decode() if isinstance(a[()], bytes) else str(a[()]), 'vlen': True}
        return
    meta[key] = {'kind': where, 'dtype': a.dtype.str, 'shape': list(a.shape)}
    arrays[key.replace('/', '|')] = a
def visit(name, obj):
    if isinstance(obj, h5py.Dataset):
        dt = obj.dtype
        if h5py.check_string_dtype(dt) is not None and dt.kind == 'O':
            meta['/' + name] = {'kind': 'dataset', 'str': obj.asstr()[()], 'vlen': True,
                                'chunks': obj.chunks}
        else:
            put('/' + name, obj[()], 'dataset')
            meta['/' + name]['chunks'] = obj.chunks
    else:
        meta['/' + name] = {'kind': 'group'}
    for k, v in obj.attrs.items():
        put('/' + name + '@' + k, v, 'attr', obj.attrs.get_id(k).dtype)
with h5py.File(src, 'r') as f:
    for k, v in f.attrs.items():
        put('@' + k, v, 'attr', f.attrs.get_id(k).dtype)
    f.visititems(visit)
np.savez(out + '.npz', **arrays)
json.dump(meta, open(out + '.json', 'w'))
'''


def h5py_dump(path, tmp_path):
    out = str(tmp_path / (os.path.basename(path) + '.dump'))
    r = subprocess.run([PY39, '-c', DUMP, path, out], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    meta = json.load(open(out + '.json'))
    arr = dict(np.load(out + '.npz'))
    return meta, {k.replace('|', '/'): v for k, v in arr.items()}


def flatten(tree, prefix=''):
    """the write() tree as {h5py path: value}: '/g/d' datasets, '/g@a' attributes"""
    out = {}
    for k, v in tree.items():
        if k.startswith('@'):
            out[(prefix if prefix else '') + k] = v
        elif isinstance(v, dict):
            out[prefix + '/' + k] = {}
            out.update(flatten(v, prefix + '/' + k))
        else:
            out[prefix + '/' + k] = v
    return out


def compare(tree, meta, arr):
    want = flatten(tree)
    assert set(want) == set(meta), (sorted(set(want) ^ set(meta)))
    for key, v in want.items():
        m = meta[key]
        if isinstance(v, dict):
            assert m['kind'] == 'group', key
            continue
        if isinstance(v, str):
            assert m.get('vlen') and m['str'] == v, key
            continue
        a = np.asarray(v)
        got = arr[key]
        assert np.dtype(m['dtype']) == a.dtype.newbyteorder('<'), (key, m['dtype'], a.dtype)
        assert tuple(m['shape']) == a.shape, key
        assert got.tobytes() == a.astype(a.dtype.newbyteorder('<')).tobytes(), key


def test_h5py_reads_every_type_the_writer_emits(tmp_path):
    from test_h5io import _tree
    tree = _tree(np.random.default_rng(5))
    p = str(tmp_path / 'types.h5')
    h5.write(p, tree)
    meta, arr = h5py_dump(p, tmp_path)
    compare(tree, meta, arr)


def test_h5py_reads_the_population_after_mstep_reduce_and_the_actdist_file(tmp_path):
    """The files the Step layer leaves: a .hss created by PopulationStore.create, its
    coordinates rewritten in place through the memory map (ModelingStep.reduce's
    set_structure), then summary + violation written by update_hss; and the
    actdist.hdf5 of the A-step reduce."""
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    path = str(tmp_path / 'igm-model.hss')
    st = ST.PopulationStore.create(path, pop['coordinates'][:, :6], pop['radii'], pop['chrom'], pop['copy'],
                                   pop['copy_ptr'], pop['copy_idx'])
    crd = st.coordinates('r+')
    new = np.random.default_rng(1).normal(0, 2000, (crd.shape[0], 3)).astype(np.float32)
    crd[:, 4, :] = new
    crd.flush()
    del crd
    summary = json.dumps({'n_imposed': 1234, 'n_violations': 5, 'histogram': {'counts': [1, 2, 3]}})
    st.write_summary(summary, 5.0 / 1234.0)
    meta, arr = h5py_dump(path, tmp_path)
    with h5.File(path) as f:
        tree = hss.read_tree(f)
    compare(tree, meta, arr)
    # what the reference's HssFile reads: float32 bead-major coordinates with the
    # in-place update, the attributes with their alabtools types
    c = arr['/coordinates']
    assert c.dtype == np.float32 and c.shape == (3008, 6, 3)
    assert np.array_equal(c[:, 4], new) and np.array_equal(c[:, 3], pop['coordinates'][:, 3])
    assert meta['@nstruct']['dtype'] == '<i8' and meta['@nbead']['dtype'] == '<i8'
    assert meta['@version']['dtype'] == '<i4' and meta['@violation']['dtype'] == '<f8'
    assert float(arr['@violation']) == 5.0 / 1234.0 and meta['/summary']['str'] == summary
    assert json.loads(meta['/index/copy_index']['str']) == json.loads(
        hss.copy_index_json(pop['copy_ptr'], pop['copy_idx']))
    assert meta['/coordinates']['chunks'] is None  # contiguous: h5py reads it like the chunked original
    # actdist.hdf5
    rows = np.zeros(5, ST.row_dtype)
    rows['row'], rows['col'] = [0, 1, 2, 3, 4], [9, 8, 7, 6, 5]
    rows['dist'], rows['prob'] = np.float32([1.5, 2.25, 3.0, 4.0, 1e4]), np.float32([.1, .2, .3, .4, 1.0])
    ap = str(tmp_path / 'actdist.hdf5')
    hss.write_actdist(ap, rows)
    meta, arr = h5py_dump(ap, tmp_path)
    assert sorted(k for k in meta if meta[k]['kind'] == 'dataset') == ['/col', '/dist', '/prob', '/row']
    for k, dt in (('row', '<i4'), ('col', '<i4'), ('dist', '<f4'), ('prob', '<f4')):
        assert meta['/' + k]['dtype'] == dt and arr['/' + k].tobytes() == np.ascontiguousarray(rows[k]).tobytes()


WRITE_REPACKED = r'''
import sys, h5py, numpy as np
path, n, s = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rng = np.random.default_rng(4)
crd = rng.normal(0, 3000, (n, s, 3)).astype('f4')
chunk = (min(int(1e6 / s / 3), n), s, 3)   # ModelingStep.py:753-762 repack
with h5py.File(path, 'w') as f:
    f.create_dataset('coordinates', data=crd, chunks=chunk, compression='gzip', compression_opts=4)
    f.create_dataset('radii', data=np.full(n, 130.6, 'f4'))
    f['summary'] = '{"n_imposed": 7}'
    f.attrs['nstruct'] = np.int64(s)
    f.attrs['nbead'] = np.int64(n)
    f.attrs['version'] = np.int32(2)
    f.attrs['violation'] = np.float64(0.125)
np.save(path + '.npy', crd)
'''


def test_native_reader_on_an_h5py_repacked_population(tmp_path):
    """ModelingStep.reduce's h5repack layout written by libhdf5 (gzip chunks of
    min(1e6/S/3, N) beads x S x 3): the native reader returns the same bytes, and the
    read-write memory map the M-step reduce uses rewrites it contiguous with the data
    intact."""
    path = str(tmp_path / 'repacked.hss')
    r = subprocess.run([PY39, '-c', WRITE_REPACKED, path, '2000', '300'], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    ref = np.load(path + '.npy')
    with h5.File(path) as f:
        assert f.info('coordinates').layout == 2 and f.info('coordinates').nfilter == 1
        assert f.read('coordinates').tobytes() == ref.tobytes()
        assert f.read('summary') == '{"n_imposed": 7}' and f.attrs('/')['violation'] == 0.125
    m = hss.coordinates_memmap(path, 'r+')
    assert np.array_equal(np.asarray(m), ref)
    m[:, 0, :] = 1.0
    m.flush()
    del m
    meta, arr = h5py_dump(path, tmp_path)
    want = ref.copy()
    want[:, 0, :] = 1.0
    assert arr['/coordinates'].tobytes() == want.tobytes()
    assert meta['/summary']['str'] == '{"n_imposed": 7}' and float(arr['@violation']) == 0.125
