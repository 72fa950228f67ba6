"""Polymer-distance A-step (PolymerAssignmentStep) and PolymerDistrib restraint.

Golden vectors: tests/golden/make_golden_polymer.py ran the reference's task() and
PolymerDistrib._apply on the demo population (np.random seeded).  The reference ranks
with argsort(argsort(d)) under NumPy's default (unstable) sort, so structures whose
distances tie exactly may swap their targets; those tie groups are compared as sets.
Everything else is bit-exact.
"""
import os

import numpy as np
import pytest

import oracle.asteps as OA
from igm_amd import polymer as PL
from igm_amd._lib import bond_dtype
from igm_amd.model import LOWER_BOUND_BIT

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.fixture(scope='module')
def data():
    return (np.load(os.path.join(GOLD, 'demo_population.npz')), np.load(os.path.join(GOLD, 'polymer_golden.npz')))


def assert_equal_up_to_ties(crd, loci, got, ref):
    bad = np.argwhere(got != ref)
    for q in np.unique(bad[:, 0]):
        i = loci[q]
        d = np.linalg.norm(crd[i] - crd[i + 1], axis=1)
        rows = bad[bad[:, 0] == q, 1]
        for s in rows:  # every differing entry belongs to a group of exactly tied distances
            grp = np.where(d == d[s])[0]
            assert len(grp) > 1, (q, s)
            assert np.array_equal(np.sort(got[q, grp]), np.sort(ref[q, grp])), (q, s)
    return len(bad)


def test_batches_follow_setup():
    b = PL.batches(3008)
    assert [x[0] for x in b] == [0, 1, 2, 3]
    assert list(b[0][1]) == list(range(0, 1000)) and list(b[-1][1]) == list(range(3000, 3007))
    assert sum(len(r) for _, r in b) == 3007
    assert list(PL.batches(2001)[-1][1]) == list(range(1000, 2000))
    # nbead a multiple of the batch size: setup() puts locus nbead-1 in the last batch,
    # whose x_(i+1) does not exist (the reference raises IndexError in task(); so does assign)
    assert list(PL.batches(2000)[-1][1]) == list(range(1000, 2000))


@pytest.mark.parametrize('case', ['a', 'b'])
def test_oracle_matches_reference(data, case):
    pop, g = data
    crd = pop['coordinates']
    o = OA.polymer_assign(crd, g[case + '_loci'], g[case + '_edges'], g[case + '_prob'],
                          np.random.RandomState(int(g[case + '_seed'])))
    n = assert_equal_up_to_ties(crd, g[case + '_loci'], o, g[case + '_nn_dist'])
    assert n < 10


def test_distribution_checks_mirror_choice():
    e = np.arange(4.0)
    with pytest.raises(ValueError, match='same size'):
        PL._check_distribution(e, [0.5, 0.5])
    with pytest.raises(ValueError, match='non-negative'):
        PL._check_distribution(e, [0.5, 0.6, -0.1, 0.0])
    with pytest.raises(ValueError, match='sum to 1'):
        PL._check_distribution(e, [0.5, 0.5, 0.5, 0.0])


@pytest.mark.parametrize('sid', [0, 7, 42])
def test_polymer_distrib_bonds_match_reference(data, sid):
    pop, g = data
    b = PL.polymer_distrib_bonds(g['a_loci'], g['a_nn_dist'], pop['chrom'], [sid], float(g['tolerance']),
                                 float(g['kspring']))[0]
    assert b.dtype == bond_dtype
    lower = (b['j'] & LOWER_BOUND_BIT) != 0
    assert np.array_equal(b['i'], g['bonds_%d_i' % sid])
    assert np.array_equal(b['j'] & ~LOWER_BOUND_BIT, g['bonds_%d_j' % sid])
    assert np.array_equal(lower, g['bonds_%d_lower' % sid])
    assert np.array_equal(b['r0'], g['bonds_%d_d' % sid].astype(np.float32))
    assert np.all(b['k'] == np.float32(g['bonds_%d_k' % sid]))


@pytest.mark.gpu
@pytest.mark.parametrize('case', ['a', 'b'])
def test_gpu_polymer_assign_matches_reference(data, case):
    pop, g = data
    crd = pop['coordinates']
    loci, nn, dist = PL.assign(crd, g[case + '_edges'], g[case + '_prob'],
                               np.random.RandomState(int(g[case + '_seed'])), return_dists=True)
    assert np.array_equal(loci, g[case + '_loci'])
    # bit-exact against the oracle (same tie order) ...
    o = OA.polymer_assign(crd, loci, g[case + '_edges'], g[case + '_prob'],
                          np.random.RandomState(int(g[case + '_seed'])))
    assert nn.tobytes() == o.tobytes()
    ref_d = np.linalg.norm(crd[loci] - crd[loci + 1], axis=2)
    assert dist.tobytes() == ref_d.astype(np.float32).tobytes()
    # ... and equal to the reference's own output up to exactly tied distances
    assert assert_equal_up_to_ties(crd, loci, nn, g[case + '_nn_dist']) < 10


@pytest.mark.gpu
def test_gpu_polymer_assign_edge_cases(data):
    pop, _ = data
    crd = pop['coordinates'][:, :37]  # S not a multiple of the workgroup or the unroll
    rng = np.random.RandomState(3)
    e = np.array([500.0])  # a single bin: every target is that edge
    loci, nn = PL.assign(crd, e, [1.0], rng, loci=[0, 5, 3006])
    assert np.all(nn == np.float32(500.0))
    # many bins, ragged subset of loci, duplicated locus, f32-unrepresentable edges
    e = np.linspace(100.0, 1200.0, 3001) + 1e-9
    p = np.random.RandomState(4).rand(3001)
    p /= p.sum()
    lo = np.array([3006, 0, 17, 17, 1500], np.int32)
    _, nn = PL.assign(crd, e, p, np.random.RandomState(9), loci=lo)
    o = OA.polymer_assign(crd, lo, e, p, np.random.RandomState(9))
    assert nn.tobytes() == o.tobytes()
    with pytest.raises(Exception):
        PL.assign(crd, e, p, np.random.RandomState(9), loci=[3007])  # i + 1 out of range
    _, nn = PL.assign(crd, e, p, np.random.RandomState(9), loci=np.zeros(0, np.int32))
    assert nn.shape == (0, 37)


@pytest.mark.gpu
@pytest.mark.parametrize('S', [5000, 10000])
def test_gpu_polymer_assign_large_populations(S):
    """Populations past the LDS-resident kernel's rank sort (S = 10000: distances and bin
    histograms in HBM, ranks counted per structure) and just inside it (S = 5000): a
    lattice population where many distances tie, bit-exact against the oracle."""
    rng = np.random.default_rng(S)
    crd = np.round(rng.normal(0.0, 3.0, (6, S, 3))).astype(np.float32)
    e = np.linspace(1.0, 12.0, 40)
    p = np.random.RandomState(2).rand(40)
    p /= p.sum()
    loci, nn, dist = PL.assign(crd, e, p, np.random.RandomState(11), loci=np.arange(5, dtype=np.int32),
                               return_dists=True)
    o = OA.polymer_assign(crd, loci, e, p, np.random.RandomState(11))
    assert len(np.unique(dist[0])) < S // 4  # ties decided by structure order
    assert nn.tobytes() == o.tobytes()
