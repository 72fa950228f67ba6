"""CPU: host-side logic of the configuration D/E A-steps (no GPU calls): locus
selection of DamidActivationDistanceStep.setup, the SPRITE cluster tables
(compute_gyration_radius bookkeeping) and the reduce() Gibbs assignment."""
import numpy as np

from conftest import load_golden


class Recorded(object):
    def __init__(self, values):
        self.values = list(values)

    def choice(self, x):
        v = self.values.pop(0)
        assert v in x
        return v


def test_damid_select_loci():
    from igm_amd import damid
    prof = np.array([0.1, 0.5, 0.45, 0.9, 0.44999], np.float32)
    last = np.zeros(3, [('loc', 'i4'), ('dist', 'f4'), ('prob', 'f4')])
    last['loc'] = [1, 3, 3]
    last['prob'] = [0.25, 0.5, 0.75]  # later rows win in the reference's dict (py:188-189)
    ii, pe, pl = damid.select_loci(prof, 0.45, last)
    assert list(ii) == [1, 2, 3]
    assert pe.dtype == np.float32 and pl.dtype == np.float32
    assert list(pl) == [0.25, 0.0, 0.75]


def test_sprite_tables_match_reference_grouping():
    """Segments grouped by chromosome in np.unique order, one representative per
    chromosome drawn in that order (sprite.pyx:214-231), single-chromosome clusters
    in sorted order with no representatives."""
    from igm_amd import sprite
    pop = load_golden('demo_population.npz')
    g = load_golden('sprite_cluster_golden.npz')
    hc = pop['hap_chrom']
    cl = [g['cl_loci'][g['cl_ptr'][c]:g['cl_ptr'][c + 1]] for c in range(len(g['cl_ptr']) - 1)]
    t = sprite.cluster_tables(cl, hc, pop['copy_ptr'], max_chrom_in_cluster=100, rng=Recorded(g['reps']))
    assert len(t['kept']) == len(cl)
    for c, x in enumerate(cl):
        x = np.sort(x)
        segs = t['seg_region'][t['seg_ptr'][c]:t['seg_ptr'][c + 1]]
        reps = t['rep_region'][t['rep_ptr'][c]:t['rep_ptr'][c + 1]]
        u = np.unique(hc[x])
        if len(u) == 1:
            assert np.array_equal(segs, x) and len(reps) == 0
        else:
            assert np.array_equal(segs, np.concatenate([x[hc[x] == ch] for ch in u]))
            assert np.array_equal(hc[reps], u)
            slots = t['seg_rep'][t['seg_ptr'][c]:t['seg_ptr'][c + 1]]
            assert np.array_equal(hc[reps][slots], hc[segs])
        assert np.array_equal(reps, g['reps'][g['rep_ptr'][c]:g['rep_ptr'][c + 1]])


def test_sprite_tables_skip_over_max_chrom():
    from igm_amd import sprite
    hc = np.repeat(np.arange(10), 5)
    clusters = [np.arange(0, 50, 5), np.arange(3), np.array([0, 5, 10])]
    t = sprite.cluster_tables(clusters, hc, np.arange(51, dtype=np.int32), max_chrom_in_cluster=6,
                              rng=np.random.RandomState(0))
    assert list(t['kept']) == [1, 2]
    assert list(t['seg_ptr']) == [0, 3, 6]


def test_sprite_gibbs_assign():
    """reduce(): every assigned structure is one of the cluster's keep_best
    candidates, skipped clusters get -1, occupancy penalises reuse."""
    from igm_amd import sprite
    rng = np.random.RandomState(1)
    ncl, S, kb = 400, 40, 10
    idx = [rng.choice(S, kb, replace=False) for _ in range(ncl)]
    val = [np.sort(rng.random(kb)).astype(np.float32) * 100 for _ in range(ncl)]
    sel = [np.arange(kb * 3).reshape(kb, 3) for _ in range(ncl)]
    val[7] = np.array([-1] * kb)
    a, chosen = sprite.assign(val, idx, sel, S, kT=50.0, rng=np.random.RandomState(3))
    assert a[7] == -1 and np.array_equal(chosen[7], sel[7][0])
    for c in range(ncl):
        if c != 7:
            assert a[c] in idx[c]
    counts = np.bincount(a[a >= 0], minlength=S)
    assert counts.max() <= 4 * (ncl / S)
    a2, _ = sprite.assign(val, idx, sel, S, kT=50.0, rng=np.random.RandomState(3))
    assert np.array_equal(a, a2)
