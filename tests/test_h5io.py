"""Native .hss / .hcs / actdist.hdf5 I/O (include/igm_io.h, csrc/h5io.cpp, igm_amd.h5,
igm_amd.hss), CPU only.

Reader parity is pinned on the reference's OWN HDF5 files (written by h5py/alabtools):
the demo .hss.T / .hss.randomInit / .hcs under /root/reference/demo are read natively
(chunked + deflate datasets, vlen strings in the global heap, attributes) and
compared with the arrays tests/golden/make_golden.py extracted from the same files
with h5py, and the .hcs read natively feeds select_pairs to reproduce the reference
setup()'s pair batches.  (Those tests skip where /root/reference is absent.)
Writer: round trips of every type / shape the IGM files use, the demo .hss rewritten
member for member, and an independent structural walk (tests/h5_inspect.py).  libhdf5
itself opening the written files (h5py 3.3.0 / libhdf5 1.10.6 under the build image's
/opt/conda/bin/python3.9) is pinned in tests/test_h5py_pin.py; the datasets are
contiguous instead of chunked, which h5py reads like the chunked originals."""
import json
import os

import numpy as np
import pytest

import h5_inspect
from conftest import GOLDEN
from igm_amd import h5, hss
from igm_amd import astep
from igm_amd import steps as ST

DEMO = '/root/reference/demo'
HSS_T = os.path.join(DEMO, 'demo_sample_outputs', 'igm-model.hss.T')
HSS_R = os.path.join(DEMO, 'demo_sample_outputs', 'igm-model.hss.randomInit')
HCS = os.path.join(DEMO, 'WTC11_HiC_2Mb.hcs')
need_ref = pytest.mark.skipif(not os.path.exists(HSS_T), reason='reference demo files absent')


@need_ref
def test_reader_on_the_reference_hss_matches_h5py():
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    with h5.File(HSS_T) as f:
        assert f.keys('/') == ['config_data', 'coordinates', 'envelope/', 'genome/', 'index/', 'radii', 'summary']
        a = f.attrs('/')
        assert a['nstruct'] == 100 and a['nbead'] == 3008 and a['version'] == 2
        assert a['violation'] == 3.0 / 1443907.0  # the demo summary's violation fraction
        assert f.info('coordinates').layout == 2  # chunked in the reference file
        assert f.read('coordinates').tobytes() == pop['coordinates'].tobytes()
        assert f.read('radii').tobytes() == pop['radii'].tobytes()
        assert f.read('index/chrom').tobytes() == pop['chrom'].tobytes()
        assert f.read('index/copy').tobytes() == pop['copy'].tobytes()
        assert f.read('index/chrom_sizes').tobytes() == pop['chrom_sizes'].astype(np.int32).tobytes()
        assert f.read('summary') == str(pop['summary_json'])
        assert f.read('genome/assembly') == 'hg38' and f.read('envelope/shape') == 'sphere'
        assert list(f.read('genome/chroms')[:2]) == [b'chr1', b'chr2']
    h = hss.Hss(HSS_T)
    assert h.copy_ptr.tobytes() == pop['copy_ptr'].astype(np.int32).tobytes()
    assert h.copy_idx.tobytes() == pop['copy_idx'].astype(np.int32).tobytes()
    store = ST.PopulationStore.__new__(ST.PopulationStore)
    assert np.array_equal(h.chrom[h.copy_idx[h.copy_ptr[:-1]]], pop['hap_chrom'])
    del store


@need_ref
def test_reader_on_the_reference_randominit_and_hcs_drives_setup():
    with h5.File(HSS_R) as f:
        assert f.read('coordinates').shape == (3008, 100, 3) and np.isnan(f.attrs('/')['violation'])
    hic = hss.read_hcs(HCS)
    assert hic['nbin'] == 1558 and len(hic['indptr']) == 1559 and len(hic['data']) == 1047862
    # the reference setup()'s pair batches (ActivationDistanceStep.py:124-191, recorded by
    # tests/golden/make_golden_init.py) from the natively read .hcs: same pairs, same
    # CSR order, same probabilities
    gold = np.load(os.path.join(GOLDEN, 'init_golden.npz'))
    for case in ('c0', 'c2'):
        intra, inter = gold['a2_%s_sigma' % case]
        inter = False if inter < 0 else float(inter)
        pairs = astep.select_pairs(hic['indptr'], hic['indices'], hic['data'], hic['chrom'], float(intra), inter)
        ref = gold['a2_%s_pairs' % case]
        assert len(pairs) == len(ref)
        assert np.array_equal(pairs['i'], ref[:, 0]) and np.array_equal(pairs['j'], ref[:, 1])
        assert np.array_equal(pairs['pwish'], ref[:, 2])


@need_ref
def test_demo_hss_rewritten_member_for_member(tmp_path):
    with h5.File(HSS_T) as f:
        tree = hss.read_tree(f)
    out = str(tmp_path / 'demo.hss')
    h5.write(out, tree)
    h5_inspect.inspect(out)
    with h5.File(out) as f:
        back = hss.read_tree(f)
        assert f.info('coordinates').layout == 1 and f.data_offset('coordinates') is not None

    def same(a, b):
        assert set(a) == set(b)
        for k in a:
            if isinstance(a[k], dict):
                same(a[k], b[k])
            elif isinstance(a[k], str):
                assert a[k] == b[k]
            else:
                x, y = np.asarray(a[k]), np.asarray(b[k])
                assert x.dtype == y.dtype and x.shape == y.shape and x.tobytes() == y.tobytes(), k
    same(tree, back)


def _tree(rng):
    return {
        '@i8': np.int64(-7), '@u2': np.uint16(65535), '@f8': np.float64(1.0 / 3.0), '@f4v': np.arange(5, dtype=np.float32),
        '@name': 'root attr', '@empty': '',
        'ints': {'i1': np.arange(-5, 5, dtype=np.int8), 'i2': np.arange(7, dtype=np.int16).reshape(7, 1),
                 'i4': rng.integers(-2**31, 2**31 - 1, (3, 4, 5), dtype=np.int64).astype(np.int32),
                 'i8': rng.integers(-2**62, 2**62, 11), 'u1': np.arange(256, dtype=np.uint8),
                 'u4': np.array([0, 2**32 - 1], np.uint32), 'u8': np.array([2**64 - 1], np.uint64)},
        'floats': {'f4': rng.standard_normal((13, 3)).astype(np.float32), 'f8': rng.standard_normal(17),
                   'scalar': np.float64(np.pi), 'nan': np.array([np.nan, np.inf, -0.0])},
        'strings': {'s10': np.array([b'chr1', b'chrX', b'', b'0123456789'], 'S10'),
                    'vlen': 'x' * 100000 + 'é', '@note': 'attribute string'},
        'empty': np.zeros((0, 3), np.float32),
        # more members than one symbol-table node holds (8): several SNODs under one B-tree
        'many': {'d%02d' % k: np.full(k + 1, k, np.int32) for k in range(40)},
        'nested': {'a': {'b': {'c': np.arange(3, dtype=np.float32), '@depth': np.int32(3)}}},
        'emptygroup': {},
    }


def test_writer_round_trip_every_type(tmp_path):
    rng = np.random.default_rng(7)
    tree = _tree(rng)
    p = str(tmp_path / 't.h5')
    h5.write(p, tree)
    walk = h5_inspect.inspect(p)
    assert '/many/d39' in walk and walk['/emptygroup']['kind'] == 'group'
    with h5.File(p) as f:
        back = hss.read_tree(f)
        assert f.keys('emptygroup') == []

    def same(a, b, path='/'):
        assert set(a) == set(b), path
        for k, v in a.items():
            if isinstance(v, dict):
                same(v, b[k], path + k + '/')
            elif isinstance(v, str):
                assert b[k] == v
            else:
                x, y = np.asarray(v), np.asarray(b[k])
                assert x.dtype.newbyteorder('<') == y.dtype and x.shape == y.shape, path + k
                assert x.tobytes() == y.tobytes(), path + k
    same(tree, back)


def test_hss_store_memmap_and_summary(tmp_path):
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    path = str(tmp_path / 'pop.hss')
    st = ST.PopulationStore.create(path, pop['coordinates'][:, :5], pop['radii'], pop['chrom'], pop['copy'],
                                   pop['copy_ptr'], pop['copy_idx'])
    h5_inspect.inspect(path)
    assert np.array_equal(st.hap_chrom, pop['hap_chrom']) and st.nstruct == 5
    crd = st.coordinates('r+')
    crd[:, 2, :] = 1.5
    crd.flush()
    del crd
    with h5.File(path) as f:
        x = f.read('coordinates')
    assert np.all(x[:, 2] == 1.5) and np.array_equal(x[:, 1], pop['coordinates'][:, 1])
    st.write_summary(json.dumps({'n_imposed': 3}), 0.25)
    h = hss.Hss(path)
    assert json.loads(h.summary) == {'n_imposed': 3} and h.violation == 0.25
    assert np.all(h.get_struct_crd(2) == 1.5)
    rows = np.zeros(4, ST.row_dtype)
    rows['row'], rows['col'], rows['dist'], rows['prob'] = [0, 1, 2, 3], [5, 6, 7, 8], [1.5, 2, 3, 4], [.1, .2, .3, .4]
    ap = str(tmp_path / 'actdist.hdf5')
    hss.write_actdist(ap, rows)
    assert hss.read_actdist(ap).tobytes() == rows.tobytes()
    with h5.File(ap) as f:
        assert f.keys('/') == ['col', 'dist', 'prob', 'row']


def test_errors_are_loud(tmp_path):
    bad = tmp_path / 'x.hss'
    bad.write_bytes(b'not hdf5 at all' * 100)
    with pytest.raises(OSError, match='not an HDF5 file'):
        h5.File(str(bad))
    p = str(tmp_path / 'ok.h5')
    h5.write(p, {'a': np.arange(3)})
    with h5.File(p) as f:
        with pytest.raises(OSError, match="no object 'b'"):
            f.read('b')
        with pytest.raises(OSError, match='no attribute'):
            f.read('a', 'nope')
    with pytest.raises(TypeError):
        h5.write(p, {'obj': np.array([object()])})
    # a truncated file fails with a range error instead of reading past the end
    data = open(p, 'rb').read()
    open(p, 'wb').write(data[:200])
    with pytest.raises(OSError):
        with h5.File(p) as f:
            f.read('a')


FUZZ = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from igm_amd import h5, hss
src, n, seed = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
data = open(src, 'rb').read()
rng = np.random.default_rng(seed)
ok = bad = 0
for it in range(n):
    b = bytearray(data)
    if it % 3 == 0:
        b = b[:int(rng.integers(0, len(b)))]
    else:
        hi = min(len(b), 1 << 16)  # the metadata (superblock, headers, B-trees) sits in front
        for _ in range(int(rng.integers(1, 8))):
            b[int(rng.integers(0, hi))] = int(rng.integers(0, 256))
    p = src + '.fuzz'
    open(p, 'wb').write(bytes(b))
    try:
        with h5.File(p) as f:
            hss.read_tree(f)
        ok += 1
    except (OSError, ValueError, UnicodeDecodeError):
        bad += 1
print(ok, bad)
'''


@pytest.mark.parametrize('which', ['written', 'reference'])
def test_corrupted_files_fail_cleanly(tmp_path, which):
    """Truncated files and files with random bytes changed in their metadata either
    read or raise; the reader never reads past the mapping or writes out of bounds
    (a crash would kill the child process, so the loop runs in one)."""
    import subprocess
    import sys
    if which == 'reference':
        if not os.path.exists(HSS_T):
            pytest.skip('reference demo files absent')
        src = str(tmp_path / 'ref.hss')
        open(src, 'wb').write(open(HSS_T, 'rb').read())
    else:
        src = str(tmp_path / 'own.h5')
        h5.write(src, _tree(np.random.default_rng(3)))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, '-c', FUZZ, root, src, '150', '11'], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    ok, bad = map(int, r.stdout.split()[-2:])
    assert ok + bad == 150 and bad > 0
