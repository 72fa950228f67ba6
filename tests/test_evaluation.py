"""Hi-C evaluation (HicEvaluationStep.reduce, igm/steps/HicEvaluationStep.py:96-179):
the GPU population contact map against the oracle (bit-exact counts), and the score
arithmetic against a literal restatement of reduce()'s dict/coo loop.  buildContactMap
and sumCopies are alabtools' (absent here): their parity is unpinned, see
igm_amd/evaluation.py."""
import os

import numpy as np
import pytest

import oracle.asteps as OA
from igm_amd import evaluation as EV

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.fixture(scope='module')
def pop():
    return np.load(os.path.join(GOLD, 'demo_population.npz'))


def test_oracle_counts_match_scalar_loop():
    rng = np.random.default_rng(3)
    crd = (rng.standard_normal((9, 5, 3)) * 300).astype(np.float32)
    r = rng.uniform(80, 160, 9).astype(np.float32)
    o = OA.contact_counts(crd, r, 2.0)
    for i in range(9):
        for j in range(9):
            n = 0
            for s in range(5):
                d = crd[i, s] - crd[j, s]
                dd = np.sqrt(np.float32(np.float32(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]))
                n += int(dd <= np.float32(2.0) * np.float32(r[i] + r[j]))
            assert o[i, j] == n
    assert (np.diag(o) == 5).all() and (o == o.T).all()


def test_sum_copies_and_score_follow_reduce():
    full = np.arange(16, dtype=np.float64).reshape(4, 4) / 40
    full = full + full.T
    copy_ptr = np.array([0, 2, 4])
    copy_idx = np.array([0, 2, 1, 3])  # haploid 0 = beads 0, 2; haploid 1 = beads 1, 3
    h = EV.sum_copies(full, copy_ptr, copy_idx)
    assert h[0, 1] == full[0, 1] + full[0, 3] + full[2, 1] + full[2, 3]
    assert h[1, 1] == full[1, 1] + full[1, 3] + full[3, 1] + full[3, 3]
    rng = np.random.default_rng(5)
    inp = np.triu(rng.uniform(0, 0.5, (12, 12)))
    out = np.clip(inp + rng.normal(0, 0.05, (12, 12)), 0, 1) * (rng.uniform(size=(12, 12)) > 0.2)
    sigma = 0.1
    # reduce(): dict of input pairs i != j with p >= sigma; loop over stored output entries
    want = {(i, j): inp[i, j] for i in range(12) for j in range(i, 12) if inp[i, j] >= sigma and i != j}
    diffs, rel = [], []
    for i in range(12):
        for j in range(i, 12):
            if out[i, j] != 0 and (i, j) in want:
                diffs.append(out[i, j] - want[i, j])
                rel.append((out[i, j] - want[i, j]) / want[i, j])
    score, ad, ar, n = EV.hic_evaluation(inp, out, sigma)
    assert n == len(diffs)
    assert score == np.abs(np.array(rel)).mean()
    assert ad == np.average(diffs) and ar == np.average(rel)


@pytest.mark.gpu
@pytest.mark.parametrize('nbead,S', [(1, 1), (130, 37), (600, 100)])
def test_gpu_contact_counts_match_oracle(pop, nbead, S):
    crd = np.ascontiguousarray(pop['coordinates'][:nbead, :S])
    r = pop['radii'][:nbead]
    got = EV.contact_counts(crd, r, 2.0 * (1 + EV.EPS))
    assert got.tobytes() == OA.contact_counts(crd, r, 2.0 * (1 + EV.EPS)).tobytes()


@pytest.mark.gpu
def test_gpu_contact_map_full_population(pop):
    crd, r = pop['coordinates'], pop['radii']
    S = crd.shape[1]
    got = EV.contact_counts(crd, r, 2.0)
    assert (got == got.T).all() and (np.diag(got) == S).all() and got.min() >= 0 and got.max() <= S
    rows = np.array([0, 1, 777, 1503, 1504, 3007])  # the whole oracle is 3008^2 x 100: check rows
    for i in rows:
        x = crd[i][None]  # (1, S, 3)
        d = x - crd
        dd = np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])
        ref = (dd <= np.float32(2.0) * (r[i] + r)[:, None]).sum(axis=1)
        assert np.array_equal(got[i], ref.astype(np.int32))
    m = EV.contact_map(crd, r, 2.0, pop['copy_ptr'], pop['copy_idx'])
    nhap = len(pop['copy_ptr']) - 1
    assert m.shape == (nhap, nhap) and m.min() >= 0 and m.max() <= 1
    # neighbouring beads of a chain are in contact in (nearly) every structure
    assert np.median(np.diag(m, 1)) == 1.0


@pytest.mark.gpu
def test_gpu_contact_counts_near_ties():
    """Pairs within a few ulp of the contact threshold: the squared-norm bound of the
    kernel must decide exactly as the float32 sqrt compare of the oracle."""
    rng = np.random.default_rng(11)
    S, nb = 256, 8
    r = np.full(nb, 50.0, np.float32)
    crd = np.zeros((nb, S, 3), np.float32)
    base = rng.uniform(-3000, 3000, (S, 3)).astype(np.float32)
    for b in range(nb):
        u = rng.standard_normal((S, 3))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        scale = 200.0 * (1 + rng.integers(-40, 40, S) * 6e-8) * (b > 0)
        crd[b] = (base + u * scale[:, None]).astype(np.float32)
    got = EV.contact_counts(crd, r, 2.0)
    ref = OA.contact_counts(crd, r, 2.0)
    assert got.tobytes() == ref.tobytes()
    assert 0 < ref[0, 1:].min() and ref[0, 1:].max() < S  # genuinely split decisions


@pytest.mark.gpu
def test_gpu_haploid_counts_equal_summed_copies(pop):
    """igm_contact_map_haploid (copies summed on the device) equals the diploid counts
    summed over copy pairs on the host, exactly (integer sums), on the demo population;
    reduce()'s matrix then follows by one division."""
    crd, r = pop['coordinates'], pop['radii']
    cp, ci = pop['copy_ptr'], pop['copy_idx']
    full = EV.contact_counts(crd, r, 2.0 * (1 + EV.EPS))
    want = EV.sum_copies(full.astype(np.float64), cp, ci)
    got = EV.haploid_counts(crd, r, 2.0 * (1 + EV.EPS), cp, ci)
    assert np.array_equal(got.astype(np.float64), want)
    m = EV.contact_map(crd, r, 2.0, cp, ci)
    ref = np.clip(EV.sum_copies(full / np.float64(crd.shape[1]), cp, ci), 0, 1)
    assert np.allclose(m, ref, rtol=1e-14, atol=0)


@pytest.mark.gpu
def test_gpu_haploid_counts_rejects_bad_copy_index(pop):
    crd, r = pop['coordinates'][:4, :3], pop['radii'][:4]
    with pytest.raises((ValueError, RuntimeError)):
        EV.haploid_counts(crd, r, 2.0, np.array([0, 2, 3]), np.array([0, 1, 1]))  # bead 1 twice, 2 and 3 missing
    with pytest.raises(RuntimeError):  # passes the host checks, the library finds the repeat
        EV.haploid_counts(crd, r, 2.0, np.array([0, 2, 4]), np.array([0, 1, 1, 3]))


def test_haploid_counts_rejects_inconsistent_copy_ptr_on_the_host():
    """copy_ptr past copy_idx or decreasing is refused before any library call (the
    C entry point reads copy_idx[k] for k < copy_ptr[nhap])."""
    crd = np.zeros((4, 2, 3), np.float32)
    r = np.ones(4, np.float32)
    for cp, ci in (([0, 2, 9], [0, 1, 2, 3]), ([0, 3, 2, 4], [0, 1, 2, 3]), ([1, 2, 4], [0, 1, 2, 3]),
                   ([0, 2, 3], [0, 1, 2])):
        with pytest.raises(ValueError):
            EV.haploid_counts(crd, r, 2.0, np.array(cp), np.array(ci))
