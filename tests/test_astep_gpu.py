"""A-step on the MI355X through the C ABI, against the reference's golden vectors
(bit-exact) and against the CPU oracle at full population size."""
import numpy as np
import pytest

from conftest import make_pairs

import oracle

pytestmark = pytest.mark.gpu

SIGMAS = [1.0, 0.2, 0.05, 0.02]


@pytest.fixture(scope='module')
def astep():
    from igm_amd import astep as a
    return a


@pytest.mark.parametrize('it_corr', [0, 1])
@pytest.mark.parametrize('sig', SIGMAS)
def test_gpu_demo_golden(astep, demo_pop, demo_pairs, g1, sig, it_corr):
    keep = demo_pairs['p'] >= sig
    tag = 's%g_c%d' % (sig, it_corr)
    pairs = make_pairs(demo_pairs['i'][keep], demo_pairs['j'][keep],
                       demo_pairs['p'][keep].astype(np.float64), g1[tag + '_plast'])
    rows, res = astep.compute_actdist(demo_pop['coordinates'], demo_pop['radii'], demo_pop['copy_ptr'],
                                      demo_pop['copy_idx'], demo_pop['chrom'], pairs, 2.0, it_corr,
                                      return_per_pair=True)
    nr = g1[tag + '_nrows'].astype(np.int32)
    assert np.array_equal(res['nrows'], nr)
    has = nr > 0
    assert np.array_equal(res['ad'][has], g1[tag + '_ad64'][has])
    assert np.array_equal(res['p'][has], g1[tag + '_p64'][has])
    first = np.concatenate([[0], np.cumsum(res['nrows'])[:-1]])
    assert np.array_equal(rows['dist'][first[has]].view(np.uint32), g1[tag + '_dist'][has].view(np.uint32))
    assert np.array_equal(rows['prob'][first[has]].view(np.uint32), g1[tag + '_prob'][has].view(np.uint32))
    assert len(rows) == int(g1[tag + '_nrows_total'])
    if tag + '_rows_row' in g1:
        for k in ('row', 'col', 'dist', 'prob'):
            assert np.array_equal(rows[k], g1[tag + '_rows_' + k])


def test_gpu_sigma001_subset(astep, demo_pop, demo_pairs, g1):
    pairs = make_pairs(demo_pairs['i01'], demo_pairs['j01'], demo_pairs['p01'].astype(np.float64),
                       g1['s0.01sub_c1_plast'])
    rows, res = astep.compute_actdist(demo_pop['coordinates'], demo_pop['radii'], demo_pop['copy_ptr'],
                                      demo_pop['copy_idx'], demo_pop['chrom'], pairs, 2.0, 1,
                                      return_per_pair=True)
    nr = g1['s0.01sub_c1_nrows'].astype(np.int32)
    assert np.array_equal(res['nrows'], nr)
    has = nr > 0
    first = np.concatenate([[0], np.cumsum(res['nrows'])[:-1]])
    assert np.array_equal(rows['dist'][first[has]], g1['s0.01sub_c1_dist'][has])
    assert np.array_equal(rows['prob'][first[has]], g1['s0.01sub_c1_prob'][has])


@pytest.mark.parametrize('ci,it_corr', [(c, i) for c in range(4) for i in (0, 1)])
def test_gpu_edge_cases(astep, g2, ci, it_corr):
    tag = 'c%d_i%d' % (ci, it_corr)
    pairs = make_pairs(g2[tag + '_pi'], g2[tag + '_pj'], g2[tag + '_pwish'], g2[tag + '_plast'])
    rows, res = astep.compute_actdist(g2['c%d_crd' % ci], g2['c%d_radii' % ci], g2['c%d_copy_ptr' % ci],
                                      g2['c%d_copy_idx' % ci], g2['c%d_chrom' % ci], pairs, 2.0, it_corr,
                                      return_per_pair=True)
    assert np.array_equal(res['nrows'], g2[tag + '_nrows'])
    has = res['nrows'] > 0
    assert np.array_equal(res['ad'][has], g2[tag + '_ad64'][has])
    assert np.array_equal(res['p'][has], g2[tag + '_p64'][has])
    for k in ('row', 'col', 'dist', 'prob'):
        assert np.array_equal(rows[k], g2[tag + '_' + k])


def test_gpu_vs_oracle_population_1000(astep, demo_pop, demo_pairs):
    """Config B size (S=1000, diploid 2 Mb): the demo population tiled x10 with a
    seeded perturbation; GPU rows must equal the oracle's rows bit for bit."""
    import oracle
    rng = np.random.default_rng(11)
    base = demo_pop['coordinates']
    xyz = np.concatenate([base + rng.normal(0, 50.0, base.shape).astype(np.float32) for _ in range(10)], axis=1)
    xyz = np.ascontiguousarray(xyz, np.float32)
    keep = demo_pairs['p'] >= 0.05
    sub = np.where(keep)[0][::5]
    pairs = make_pairs(demo_pairs['i'][sub], demo_pairs['j'][sub], demo_pairs['p'][sub].astype(np.float64),
                       rng.uniform(0, 0.5, len(sub)))
    for it_corr in (0, 1):
        rows, res = astep.compute_actdist(xyz, demo_pop['radii'], demo_pop['copy_ptr'], demo_pop['copy_idx'],
                                          demo_pop['chrom'], pairs, 2.0, it_corr, return_per_pair=True)
        orows, ores = oracle.actdist(xyz, demo_pop['radii'], demo_pop['copy_ptr'], demo_pop['copy_idx'],
                                     demo_pop['chrom'], pairs, 2.0, it_corr, nthreads=16)
        assert np.array_equal(res['nrows'], ores['nrows'])
        assert np.array_equal(res['o'], ores['o'])
        has = res['nrows'] > 0
        assert np.array_equal(res['ad'][has], ores['ad'][has])
        assert rows.tobytes() == orows.tobytes()


@pytest.mark.parametrize('reps', [11, 80])
def test_gpu_vs_oracle_large_population(astep, demo_pop, demo_pairs, reps):
    """Populations past one wave's registers (S = 1100: inter pairs need the
    workgroup kernel; S = 8000: the 8-GPU weak-scaling population, every pair
    on the workgroup kernel): rows bit-identical to the oracle."""
    import oracle
    rng = np.random.default_rng(12 + reps)
    base = demo_pop['coordinates']
    xyz = np.concatenate([base + rng.normal(0, 50.0, base.shape).astype(np.float32) for _ in range(reps)], axis=1)
    xyz = np.ascontiguousarray(xyz, np.float32)
    keep = np.where(demo_pairs['p'] >= 0.02)[0]
    sub = keep[rng.choice(len(keep), 400, replace=False)]
    sub.sort()
    pairs = make_pairs(demo_pairs['i'][sub], demo_pairs['j'][sub], demo_pairs['p'][sub].astype(np.float64),
                       rng.uniform(0, 0.5, len(sub)))
    for it_corr in (0, 1):
        rows, res = astep.compute_actdist(xyz, demo_pop['radii'], demo_pop['copy_ptr'], demo_pop['copy_idx'],
                                          demo_pop['chrom'], pairs, 2.0, it_corr, return_per_pair=True)
        orows, ores = oracle.actdist(xyz, demo_pop['radii'], demo_pop['copy_ptr'], demo_pop['copy_idx'],
                                     demo_pop['chrom'], pairs, 2.0, it_corr, nthreads=16)
        assert np.array_equal(res['nrows'], ores['nrows'])
        assert np.array_equal(res['o'], ores['o'])
        assert np.array_equal(res['pnow'], ores['pnow'])
        has = res['nrows'] > 0
        assert np.array_equal(res['ad'][has], ores['ad'][has])
        assert rows.tobytes() == orows.tobytes()


def test_gpu_device_pointer_path(astep, demo_pop, demo_pairs, g1):
    """Inputs already resident in HBM (torch tensors): same rows as the host path."""
    import torch
    keep = demo_pairs['p'] >= 0.02
    tag = 's0.02_c0'
    pairs = make_pairs(demo_pairs['i'][keep], demo_pairs['j'][keep],
                       demo_pairs['p'][keep].astype(np.float64), g1[tag + '_plast'])
    dev = torch.device('cuda:0')
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    rows_t, n = astep.compute_actdist(t(demo_pop['coordinates']), t(demo_pop['radii']), t(demo_pop['copy_ptr']),
                                      t(demo_pop['copy_idx']), t(demo_pop['chrom']),
                                      torch.from_numpy(pairs.view(np.uint8)).to(dev), 2.0, 0)
    torch.cuda.synchronize()
    rows = rows_t[:n * 16].cpu().numpy().view(astep.row_dtype)
    ref = astep.compute_actdist(demo_pop['coordinates'], demo_pop['radii'], demo_pop['copy_ptr'],
                                demo_pop['copy_idx'], demo_pop['chrom'], pairs, 2.0, 0)
    assert rows.tobytes() == ref.tobytes()
    assert n == int(g1[tag + '_nrows_total'])


def test_gpu_get_actdist_signature(astep, demo_pop):
    """The reference's per-pair function signature on a duck-typed hss."""
    class Idx:
        pass

    class Hss:
        def __init__(self, p):
            self.p = p
            self.idx = Idx()
            ptr, ci = p['copy_ptr'], p['copy_idx']
            self.idx.copy_index = {h: list(ci[ptr[h]:ptr[h + 1]]) for h in range(len(ptr) - 1)}
            self.idx.chrom = p['chrom']

        def get_nstruct(self):
            return self.p['coordinates'].shape[1]

        def get_index(self):
            return self.idx

        def get_radii(self):
            return self.p['radii']

        def get_bead_crd(self, k):
            return self.p['coordinates'][k]

    p = demo_pop
    for (i, j, pw, it_corr) in [(0, 5, 0.3, 0), (0, 5, 0.3, 1), (2, 40, 0.05, 0), (0, 1500, 0.02, 0)]:
        res = astep.get_actdist(i, j, pw, 0.0, Hss(p), it_corr, contactRange=2.0)
        _, ores = oracle.actdist(p['coordinates'], p['radii'], p['copy_ptr'], p['copy_idx'], p['chrom'],
                                 make_pairs([i], [j], [pw], [0.0]), 2.0, it_corr)
        if ores['nrows'][0] == 0:
            assert res == []
            continue
        ci = [list(p['copy_idx'][p['copy_ptr'][h]:p['copy_ptr'][h + 1]]) for h in (i, j)]
        combos = list(zip(*ci)) if p['chrom'][i] == p['chrom'][j] else [(a, b) for a in ci[0] for b in ci[1]]
        assert [(r[0], r[1]) for r in res] == combos
        assert all(r[2] == ores['ad'][0] and r[3] == ores['p'][0] for r in res)
    assert astep.get_actdist(3, 3, 0.3, 0.0, Hss(p), 1) == []
