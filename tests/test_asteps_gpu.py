"""Configuration D/E A-steps (DamID, FISH, SPRITE) on the MI355X through the C ABI:
bit-exact against the golden vectors of the reference functions, against the CPU
oracle at full 200 kb population size, and the edge cases."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import asteps as A

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def pop():
    return load_golden('demo_population.npz')


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope='module')
def pop200():
    """Config C/D/E population: 200 kb diploid, 1000 structures, bead-major."""
    from igm_amd import synthetic
    p = synthetic.population_200kb(1000)
    p['xyz'] = np.ascontiguousarray(p['xyz'].transpose(1, 0, 2))
    return p


class DuckHss(object):
    """The hss duck type get_damid_actdist_I reads (get_nstruct, get_index().copy_index,
    get_radii, get_bead_crd)."""

    def __init__(self, pop):
        self.pop = pop
        ptr, idx = pop['copy_ptr'], pop['copy_idx']
        self.copy_index = {h: [int(x) for x in idx[ptr[h]:ptr[h + 1]]] for h in range(len(ptr) - 1)}

    def get_nstruct(self):
        return self.pop['coordinates'].shape[1]

    def get_index(self):
        return self

    def get_radii(self):
        return self.pop['radii']

    def get_bead_crd(self, b):
        return self.pop['coordinates'][b]


class Recorded(object):
    """np.random stand-in that replays the recorded representative draws."""

    def __init__(self, values):
        self.values = list(values)

    def choice(self, x):
        v = self.values.pop(0)
        assert v in x
        return v


# ---------------------------------------------------------------- DamID
@pytest.mark.parametrize('shape', ['sphere', 'ellipsoid'])
@pytest.mark.parametrize('it_corr', [0, 1])
@pytest.mark.parametrize('sigma', [0.45, 0.2])
def test_damid_golden(pop, shape, it_corr, sigma):
    from igm_amd import damid
    g = load_golden('damid_golden.npz')
    tag = '%s_c%d_s%g' % (shape, it_corr, sigma)
    loci = g[tag + '_loci']
    param = float(g['sphere_radius']) if shape == 'sphere' else g['ellipsoid_semiaxes']
    rows, res = damid.compute_damid_actdist(pop['coordinates'], pop['radii'], pop['copy_ptr'], pop['copy_idx'], loci,
                                            g['profile'][loci], g['plast'][loci], it_corr, 0.05, shape, param,
                                            return_per_locus=True)
    assert np.array_equal(rows['loc'], g[tag + '_loc'])
    assert np.array_equal(bits(rows['dist']), bits(g[tag + '_dist']))
    assert np.array_equal(bits(rows['prob']), bits(g[tag + '_prob']))
    assert np.array_equal(res['nrows'], np.diff(pop['copy_ptr'])[loci])


def test_damid_edges(pop):
    from igm_amd import damid
    crd, radii, cp, ci = pop['coordinates'], pop['radii'], pop['copy_ptr'], pop['copy_idx']
    rows = damid.compute_damid_actdist(crd, radii, cp, ci, [], [], [], 1)
    assert len(rows) == 0
    # p_exp = 0 -> no quantile: the row carries dist 2 (py:460); plast >= 1 keeps p_exp
    loci = np.array([0, 1, 2, 3], np.int32)
    pe = np.array([0.0, 0.3, 1.0, 0.5], np.float32)
    pl = np.array([0.0, 1.0, 0.2, 0.99], np.float32)
    for it in (0, 1):
        rows = damid.compute_damid_actdist(crd, radii, cp, ci, loci, pe, pl, it, 0.05, 'sphere', 5500.0)
        ref = A.damid_actdist(crd, radii, cp, ci, loci, pe, pl, it, 0.05, 'sphere', 5500.0)
        assert np.array_equal(rows['loc'], ref['loc'])
        assert np.array_equal(bits(rows['dist']), bits(ref['dist']))
        assert np.array_equal(bits(rows['prob']), bits(ref['prob']))
    assert rows['dist'][0] == 2.0
    with pytest.raises(RuntimeError):
        damid.compute_damid_actdist(crd, radii, cp, ci, [len(cp) - 1], [0.5], [0.0], 1)
    with pytest.raises(NotImplementedError):
        damid.compute_damid_actdist(crd, radii, cp, ci, [0], [0.5], [0.0], 1, shape='cylinder')


def test_damid_per_locus_signature(pop):
    """get_damid_actdist_I (py:376) returns the float64 ad/p of the oracle."""
    from igm_amd import damid
    hss = DuckHss(pop)
    for I in (0, 5, 300):
        out = damid.get_damid_actdist_I(I, np.float32(0.4), np.float32(0.1), hss, 1, 0.05, 'sphere', 5500.0)
        nhap = len(pop['copy_ptr']) - 1
        ref = A.damid_actdist(pop['coordinates'], pop['radii'], pop['copy_ptr'], pop['copy_idx'], [I],
                              np.full(nhap, 0.4, np.float32), np.full(nhap, 0.1, np.float32), 1, 0.05, 'sphere',
                              5500.0)
        assert [o[0] for o in out] == list(ref['loc'])
        assert np.float32(float('%.5f' % out[0][1])) == ref['dist'][0]


@pytest.mark.parametrize('shape', ['sphere', 'ellipsoid'])
def test_damid_full_size_200kb(pop200, shape):
    """Config D sizes (200 kb diploid, 1000 structures, sigma 0.45): every row the GPU
    emits for a sample of loci equals the oracle's, and the row count is exact."""
    from igm_amd import damid, synthetic
    p = pop200
    xyz = p['xyz']
    prof = synthetic.damid_profile_200kb()
    loci, pe, pl = damid.select_loci(prof, 0.45)
    pl[::3] = np.float32(0.2)
    param = 5500.0 if shape == 'sphere' else synthetic.ELLIPSOID_D
    rows, res = damid.compute_damid_actdist(xyz, p['radii'], p['copy_ptr'], p['copy_idx'], loci, pe, pl, 1, 0.05,
                                            shape, param, return_per_locus=True)
    assert len(rows) == int(np.diff(p['copy_ptr'])[loci].sum())
    off = np.concatenate([[0], np.cumsum(res['nrows'])])
    plfull = np.zeros(len(prof), np.float32)
    plfull[loci] = pl
    for q in np.random.default_rng(0).choice(len(loci), 40, replace=False):
        ref = A.damid_actdist(xyz, p['radii'], p['copy_ptr'], p['copy_idx'], [loci[q]], prof, plfull, 1, 0.05,
                              shape, param)
        got = rows[off[q]:off[q + 1]]
        assert np.array_equal(got['loc'], ref['loc'])
        assert np.array_equal(bits(got['dist']), bits(ref['dist'])), q
        assert np.array_equal(bits(got['prob']), bits(ref['prob'])), q


# ---------------------------------------------------------------- FISH
def test_fish_radial_golden(pop):
    from igm_amd import fish
    g = load_golden('fish_golden.npz')
    omin, omax, dmin, dmax = fish.assign(pop['coordinates'], pop['copy_ptr'], pop['copy_idx'], 'probe', g['probes'],
                                         g['radial_min_targets'], g['radial_max_targets'], return_dists=True)
    assert np.array_equal(dmin.astype(np.float64), g['rad_min'])
    assert np.array_equal(dmax.astype(np.float64), g['rad_max'])
    assert np.array_equal(bits(omin), bits(g['radial_min']))
    assert np.array_equal(bits(omax), bits(g['radial_max']))


def test_fish_pair_golden(pop):
    from igm_amd import fish
    g = load_golden('fish_golden.npz')
    omin, omax, dmin, dmax = fish.assign(pop['coordinates'], pop['copy_ptr'], pop['copy_idx'], 'pair', g['pairs'],
                                         g['pair_min_targets'], g['pair_max_targets'], return_dists=True)
    assert np.array_equal(dmin.astype(np.float64), g['pair_dmin'])
    assert np.array_equal(dmax.astype(np.float64), g['pair_dmax'])
    assert np.array_equal(bits(omin), bits(g['pair_min']))
    assert np.array_equal(bits(omax), bits(g['pair_max']))


def test_fish_task_dict_and_ties(pop):
    """task()'s fish_restr layout; duplicate pairs report the first matching row
    (py:211); ties rank in structure order."""
    from igm_amd import fish
    g = load_golden('fish_golden.npz')
    pairs = np.concatenate([g['pairs'][:5], g['pairs'][:1]])
    inp = {'pairs': pairs, 'pair_min': g['pair_min_targets'][:6], 'probes': g['probes'][:4],
           'radial_max': g['radial_max_targets'][:4]}
    out = fish.task(pop['coordinates'], pop['copy_ptr'], pop['copy_idx'], inp)
    assert [q for q, _ in out['pair_min']] == [0, 1, 2, 3, 4, 0]
    assert np.array_equal(out['pair_min'][5][1], out['pair_min'][0][1])
    assert len(out['radial_max']) == 4 and out['radial_min'] == [] and out['pair_max'] == []
    # a probe whose two copies coincide in every structure (ties everywhere)
    crd = np.zeros((2, 50, 3), np.float32)
    crd[:, :, 0] = 7.0
    t = np.sort(np.random.default_rng(0).random((1, 50))).astype(np.float32)
    omin, _ = fish.assign(crd, np.array([0, 2], np.int32), np.array([0, 1], np.int32), 'probe', [0], t, None)
    assert np.array_equal(omin[0], t[0])


@pytest.mark.parametrize('S', [50, 200, 256, 300, 512, 700, 1024, 1500, 2048, 2100, 4096, 5000, 10000])
def test_fish_rank_widths_with_ties(S):
    """The rank sort at every width it takes (registers for npad = 256, 512, 1024, 2048;
    LDS otherwise; past one CU's LDS, S = 5000 and 10000, the columns in HBM and counted
    ranks): radial distances rounded to a few values, so most ranks are decided by
    structure order, against the oracle's argsort(argsort(kind='stable'))."""
    from igm_amd import fish
    rng = np.random.default_rng(S)
    xyz = np.round(rng.normal(0.0, 2.0, (4, S, 3))).astype(np.float32)  # integer lattice: many equal norms
    cptr = np.array([0, 2, 3], np.int32)
    cidx = np.array([0, 1, 2], np.int32)
    probes = np.array([0, 1], np.int32)
    tmin = np.sort(rng.random((2, S)), axis=1).astype(np.float32)
    tmax = np.sort(rng.random((2, S)), axis=1).astype(np.float32)
    omin, omax = fish.assign(xyz, cptr, cidx, 'probe', probes, tmin, tmax)
    rmin, rmax, _, _ = A.fish_radial(xyz, cptr, cidx, probes, tmin, tmax)
    assert np.array_equal(bits(omin), bits(rmin))
    assert np.array_equal(bits(omax), bits(rmax))


def test_fish_full_size_200kb(pop200):
    from igm_amd import fish, synthetic
    p = pop200
    xyz = p['xyz']
    f = synthetic.fish_inputs_200kb(1000)
    for kind, key, pre, fn in (('probe', 'probes', 'radial', A.fish_radial), ('pair', 'pairs', 'pair', A.fish_pair)):
        omin, omax = fish.assign(xyz, p['copy_ptr'], p['copy_idx'], kind, f[key], f[pre + '_min'], f[pre + '_max'])
        sel = np.arange(0, len(f[key]), 25)
        rmin, rmax, _, _ = fn(xyz, p['copy_ptr'], p['copy_idx'], f[key][sel], f[pre + '_min'][sel],
                              f[pre + '_max'][sel])
        assert np.array_equal(bits(omin[sel]), bits(rmin))
        assert np.array_equal(bits(omax[sel]), bits(rmax))
        # rank matching is a permutation of the targets
        assert np.array_equal(np.sort(omin, axis=1), f[pre + '_min'])


# ---------------------------------------------------------------- SPRITE
def golden_tables(pop, g):
    from igm_amd import sprite
    cl = [g['cl_loci'][g['cl_ptr'][c]:g['cl_ptr'][c + 1]] for c in range(len(g['cl_ptr']) - 1)]
    t = sprite.cluster_tables(cl, pop['hap_chrom'], pop['copy_ptr'], max_chrom_in_cluster=100,
                              rng=Recorded(g['reps']))
    return cl, t


def test_sprite_golden_rg2_and_selection(pop):
    from igm_amd import sprite
    g = load_golden('sprite_cluster_golden.npz')
    cl, t = golden_tables(pop, g)
    S = pop['coordinates'].shape[1]
    kb = int(g['keep_best'])
    bi, bv, bs, rg2 = sprite.rg2_select(pop['coordinates'], pop['copy_ptr'], pop['copy_idx'], t, kb, return_rg2=True)
    assert np.array_equal(bits(rg2), bits(g['rg2s']))
    assert np.array_equal(bi, g['best_idx'])
    assert np.array_equal(bits(bv), bits(np.take_along_axis(g['rg2s'], g['best_idx'].astype(np.int64), 1)))
    # selected beads of the kept structures == the reference's selected rows
    for c in range(len(cl)):
        g0, g1 = int(t['seg_ptr'][c]), int(t['seg_ptr'][c + 1])
        got = bs[g0 * kb:g1 * kb].reshape(kb, g1 - g0)
        ref = g['selected'][:, g0:g1][g['best_idx'][c]]
        assert np.array_equal(got, ref), c
    # every structure's selection (keep_best = S - 1 keeps all but the worst)
    bi2, _, bs2 = sprite.rg2_select(pop['coordinates'], pop['copy_ptr'], pop['copy_idx'], t, S - 1)
    for c in range(0, len(cl), 13):
        g0, g1 = int(t['seg_ptr'][c]), int(t['seg_ptr'][c + 1])
        got = bs2[g0 * (S - 1):g1 * (S - 1)].reshape(S - 1, g1 - g0)
        assert np.array_equal(got, g['selected'][:, g0:g1][bi2[c]]), c


def test_sprite_table_path_equals_index_path(pop, monkeypatch):
    """The kernel's table path (bead ids of every segment and representative copy in flat
    host-built tables, representatives' copies in registers) and its per-bead index path
    (IGM_SPRITE_TABLES=0) give the same bits: Rg^2 of every (cluster, structure), kept
    structures and selected beads."""
    from igm_amd import sprite
    g = load_golden('sprite_cluster_golden.npz')
    cl, t = golden_tables(pop, g)
    out = []
    for mode in ('1', '0'):
        monkeypatch.setenv('IGM_SPRITE_TABLES', mode)
        out.append(sprite.rg2_select(pop['coordinates'], pop['copy_ptr'], pop['copy_idx'], t, 5, return_rg2=True))
    for a, b in zip(*out):
        assert np.array_equal(bits(a) if a.dtype == np.float32 else a, bits(b) if b.dtype == np.float32 else b)


def test_sprite_table_path_mixed_copies(monkeypatch):
    """A 2-copy segment under a 1-copy representative (and a 2-copy one under a 2-copy
    representative): the table path must pick the copies the index path picks."""
    from igm_amd import sprite
    rng = np.random.default_rng(3)
    S = 300
    xyz = rng.normal(0.0, 1.0, (7, S, 3)).astype(np.float32)
    copy_ptr = np.array([0, 1, 3, 5, 7], np.int32)  # region 0: 1 copy, regions 1-3: 2 copies
    copy_idx = np.arange(7, dtype=np.int32)
    i32 = lambda a: np.asarray(a, np.int32)
    # cluster 0: region 1 (2 copies) under the 1-copy representative region 0, regions 2 and 3
    # under region 2; cluster 1: every segment with its representative's copies
    t = dict(seg_ptr=i32([0, 3, 5]), seg_region=i32([1, 2, 3, 0, 1]), seg_rep=i32([0, 1, 1, 0, 1]),
             rep_ptr=i32([0, 2, 4]), rep_region=i32([0, 2, 0, 2]), kept=np.arange(2))
    out = []
    for mode in ('1', '0'):
        monkeypatch.setenv('IGM_SPRITE_TABLES', mode)
        out.append(sprite.rg2_select(xyz, copy_ptr, copy_idx, t, 7, return_rg2=True))
    for a, b in zip(*out):
        assert np.array_equal(bits(a) if a.dtype == np.float32 else a, bits(b) if b.dtype == np.float32 else b)


def test_sprite_task_skip_and_errors(pop):
    from igm_amd import sprite
    hc = pop['hap_chrom']
    many = [int(np.where(hc == ch)[0][0]) for ch in range(8)]  # 8 chromosomes > 6
    clusters = [np.array(many), np.where(hc == 3)[0][:5]]
    idx, val, sel = sprite.task(pop['coordinates'], clusters, hc, pop['copy_ptr'], pop['copy_idx'], keep_best=10,
                                max_chrom_in_cluster=6)
    assert list(idx[0]) == [-1] * 10 and sel[0].shape == (10, 8) and (sel[0] == -1).all()
    assert sel[1].shape == (10, 5) and (idx[1] >= 0).all()
    assert np.all(np.diff(val[1]) >= 0)
    with pytest.raises(RuntimeError):  # keep_best must be < nstruct (np.argpartition)
        sprite.task(pop['coordinates'], clusters, hc, pop['copy_ptr'], pop['copy_idx'],
                    keep_best=pop['coordinates'].shape[1])


@pytest.mark.parametrize('S', [50, 256, 700, 1024, 2048, 2100, 9000])
def test_sprite_keep_best_widths_and_ties(S):
    """keep_best at every width of the rank sort (and the counting kernel past the sort's
    LDS, S = 9000): a lattice population where many structures share an Rg^2, so the order
    of the kept structures is decided by structure index -- a stable argsort of the column."""
    from igm_amd import sprite
    rng = np.random.default_rng(S)
    nbead = 6
    xyz = np.round(rng.normal(0.0, 1.0, (nbead, S, 3))).astype(np.float32)
    copy_ptr = np.arange(nbead + 1, dtype=np.int32)
    copy_idx = np.arange(nbead, dtype=np.int32)
    chrom = np.zeros(nbead, np.int64)
    t = sprite.cluster_tables([np.array([0, 1, 2]), np.array([2, 3, 4, 5]), np.array([1, 5])], chrom, copy_ptr)
    kb = min(50, S - 1)
    bi, bv, bs, rg2 = sprite.rg2_select(xyz, copy_ptr, copy_idx, t, kb, return_rg2=True)
    for c in range(3):
        order = np.argsort(rg2[c], kind='stable')[:kb]
        assert len(np.unique(rg2[c])) < S  # ties are the point
        assert np.array_equal(bi[c], order)
        assert np.array_equal(bits(bv[c]), bits(rg2[c][order]))


def test_sprite_full_size_200kb(pop200):
    """Config E sizes: 200 kb population, 1000 structures, clusters of 2..20 loci;
    a sample of (cluster, structure) Rg^2 and selections against the oracle."""
    from igm_amd import sprite, synthetic
    p = pop200
    xyz = p['xyz']
    ptr, data = synthetic.sprite_clusters_200kb(3000)
    cl = [data[ptr[c]:ptr[c + 1]] for c in range(len(ptr) - 1)]
    rng = np.random.RandomState(5)
    t = sprite.cluster_tables(cl, p['hap_chrom'], p['copy_ptr'], rng=rng)
    bi, bv, bs, rg2 = sprite.rg2_select(xyz, p['copy_ptr'], p['copy_idx'], t, 50, return_rg2=True)
    # the representatives drawn are recoverable from the tables
    for k in range(0, len(t['kept']), 97):
        c = int(t['kept'][k])
        reps = t['rep_region'][t['rep_ptr'][k]:t['rep_ptr'][k + 1]]
        rg, sel = A.sprite_cluster_rg2(xyz, p['hap_chrom'], p['copy_ptr'], p['copy_idx'], cl[c], reps,
                                       structs=range(0, 1000, 111))
        for s in range(0, 1000, 111):
            assert rg2[k, s] == rg[s], (c, s)
        assert np.array_equal(bi[k], A.keep_best(rg2[k], 50))


@pytest.mark.parametrize('it_corr', [0, 1])
def test_damid_exp_map_golden(pop, it_corr):
    """exp_map DamID (get_damid_actdist_exp, py:475-577) on two maps assigned per
    structure: rows bit-exact against the reference's."""
    from igm_amd import damid
    g = load_golden('damid_exp_golden.npz')
    maps = [dict(body_idx=0, nvoxel=g['m%d_nvoxel' % m], center=g['m%d_center' % m], origin=g['m%d_origin' % m],
                 grid=g['m%d_grid' % m], matrice=g['m%d_matrice' % m]) for m in (0, 1)]
    rows = damid.compute_damid_actdist(pop['coordinates'], pop['radii'], pop['copy_ptr'], pop['copy_idx'], g['loci'],
                                       g['pexp'], g['plast'], it_corr, 0.05, 'exp_map', volumes=maps,
                                       struct_map=g['volumes_idx'])
    assert np.array_equal(rows['loc'], g['c%d_loc' % it_corr])
    assert np.array_equal(bits(rows['dist']), bits(g['c%d_dist' % it_corr]))
    assert np.array_equal(bits(rows['prob']), bits(g['c%d_prob' % it_corr]))
