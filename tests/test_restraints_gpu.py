"""Configuration D/E M-step restraints on the MI355X: DamID lamina-envelope membership
(bit-exact against the reference's arithmetic), per-structure atom flags (SPRITE
centroid slots, DamID envelope) through the anneal/CG/violation kernels, forces
against the fp64 oracle structure by structure."""
import numpy as np
import pytest

import oracle
import mstep_fixtures as F
from conftest import load_golden
from igm_amd import model as M
from test_mstep_gpu import _bonds_for, short_protocol

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def demo():
    return F.load()


@pytest.fixture(scope='module')
def ms():
    from igm_amd import mstep
    return mstep


def damid_rows():
    g = load_golden('damid_golden.npz')
    r = np.zeros(len(g['sphere_c1_s0.2_loc']), [('loc', 'i4'), ('dist', 'f4'), ('prob', 'f4')])
    r['loc'], r['dist'], r['prob'] = g['sphere_c1_s0.2_loc'], g['sphere_c1_s0.2_dist'], g['sphere_c1_s0.2_prob']
    return r


def select_restatement(x, radii, rows, abc, cr):
    """Damid._apply_envelope membership (damid.py:112-126) with NumPy 1.x scalar
    promotion written out: f32 squares / f64 (abc*cutoff - r)^2, f64 sums, >= f64(d)^2."""
    sel = np.zeros(x.shape[0], bool)
    A = np.asarray(abc, np.float64) * (1 - cr)
    for loc, d in zip(rows['loc'], rows['dist']):
        r = np.float64(radii[loc])
        a, b, c = A - r
        sq = np.square(x[loc]).astype(np.float64)
        v = (sq[0] / (a * a) + sq[1] / (b * b)) + sq[2] / (c * c)
        if v >= np.float64(d) * np.float64(d):
            sel[loc] = True
    return sel


@pytest.mark.parametrize('abc', [(5500.0,) * 3, (5488.0, 5499.5, 5390.0)])
def test_damid_select_bitexact(demo, abc):
    from igm_amd import restraints as R
    pop, _ = demo
    atoms = M.Atoms(pop['radii'])
    sids = list(range(40))
    x = F.struct_major(pop, sids, atoms.n)
    rows = damid_rows()
    flags, nsel = R.damid_envelope_flags(x, atoms.radii, rows, abc, 0.05, 1, atoms.flags)
    bit = np.uint32(M.IGM_ATOM_ENV0 << 1)
    for s in range(len(sids)):
        sel = select_restatement(x[s], atoms.radii, rows, abc, 0.05)
        assert np.array_equal((flags[s] & bit) != 0, sel), s
        assert np.array_equal(flags[s] & ~bit, atoms.flags)
        assert nsel[s] == int(sel.sum())
    assert 0 < nsel.sum() < len(rows) * len(sids)


def test_struct_flags_identical_rows_bitwise(demo, ms):
    """(S, N) flags whose rows all equal the shared flags reproduce the shared-flag
    run bit for bit (LDS anneal + CG)."""
    pop, _ = demo
    sids = list(range(4))
    atoms, poly, prm, ptr, sb = _bonds_for(demo, sids)
    p = M.params_from_cfg({'optimization': {'optimizer_options': short_protocol((100, 100, 100, 100), 50)}},
                          [((5500.0,) * 3, 1.0)])
    x = F.struct_major(pop, sids, atoms.n)
    seeds = M.lammps_seeds(6535, sids, 11)
    x1, i1 = ms.run(p, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    fl = np.repeat(atoms.flags[None, :], len(sids), axis=0)
    x2, i2 = ms.run(p, x, atoms.radii, fl, poly, ptr, sb, seeds)
    assert np.array_equal(x1, x2)
    assert np.array_equal(i1['final_energy'], i2['final_energy'])


def de_model(demo, sids, nslot=3):
    """Beads + centre dummy + nslot SPRITE centroid slots; envelopes: nucleus (k=1,
    all beads) and DamID lamina (k=-1, per structure); per-structure flags."""
    from igm_amd import restraints as R
    pop, g3 = demo
    atoms0, poly, _, ptr, sb = _bonds_for(demo, sids)
    nb = atoms0.nbead
    first = atoms0.n
    n = first + nslot
    radii = np.concatenate([atoms0.radii, np.zeros(nslot, np.float32)])
    base = np.concatenate([atoms0.flags, np.zeros(nslot, np.uint32)])
    x = F.struct_major(pop, sids, n)
    # SPRITE: clusters of 4 consecutive beads assigned round-robin to the structures
    rng = np.random.default_rng(7)
    ncl = 2 * len(sids)
    indptr = np.arange(ncl + 1) * 4
    selected = np.concatenate([np.arange(st, st + 4) for st in rng.integers(0, nb - 4, ncl)]).astype(np.int32)
    assignment = np.array([c % len(sids) if c < ncl - 1 else -1 for c in range(ncl)], np.int32)
    k, pos, active, sbonds = R.sprite_centroids(assignment, indptr, selected, x, range(len(sids)), radii, 0.3, 1.0,
                                                first)
    assert k <= nslot
    x[:, first:first + k] = pos
    flags = R.centroid_flags(base, active, first, nslot)
    rows = damid_rows()
    dflags, nsel = R.damid_envelope_flags(x, radii, rows, (5500.0,) * 3, 0.05, 1, base)
    flags |= dflags & np.uint32(M.IGM_ATOM_ENV0 << 1)
    # FISH: radial min/max bonds to the centre dummy for 10 probes
    g = load_golden('fish_golden.npz')
    fish = {'probes': g['probes'][:10], 'radial_min': g['radial_min_targets'][:10],
            'radial_max': g['radial_max_targets'][:10]}
    fb = R.fish_bonds(fish, pop['copy_ptr'], pop['copy_idx'], x, sids, 'rR', nb, tol=50.0, kspring=1.0)
    per = [np.concatenate([sb[ptr[s]:ptr[s + 1]], sbonds[s], fb[s]]) for s in range(len(sids))]
    ptr2, sb2 = M.concat_bonds(per)
    prm = M.params_from_cfg({'optimization': {'optimizer_options': short_protocol((120, 120, 120, 120), 40)}},
                            [((5500.0,) * 3, 1.0), ((5500.0 * 0.95,) * 3, -1.0)])
    return dict(x=x, radii=radii, flags=flags, poly=poly, ptr=ptr2, sb=sb2, prm=prm, active=active, first=first,
                nslot=nslot, nsel=nsel)


@pytest.mark.parametrize('evf,envf', [(0.5, 1.2), (1.0, 1.0)])
def test_de_forces_match_oracle(demo, ms, evf, envf):
    """Per-structure flags (lamina envelope k<0, centroid slots) and SPRITE/FISH bonds:
    GPU f64 forces and energies = the fp64 oracle run structure by structure."""
    sids = list(range(5))
    d = de_model(demo, sids)
    x = d['x'].copy()
    x[:, :3008] += np.random.default_rng(9).normal(0, 80.0, (len(sids), 3008, 3)).astype(np.float32)
    fg, eg = ms.forces(d['prm'], x, d['radii'], d['flags'], d['poly'], d['ptr'], d['sb'], evf, envf)
    for s in range(len(sids)):
        sp = np.array([0, d['ptr'][s + 1] - d['ptr'][s]], np.int64)
        fo, eo = oracle.mstep_forces(d['prm'], x[s:s + 1], d['radii'], d['flags'][s], d['poly'], sp,
                                     d['sb'][d['ptr'][s]:d['ptr'][s + 1]], evf, envf)
        scale = np.abs(fo).max()
        assert np.abs(fg[s] - fo[0]).max() <= 1e-6 * scale + 1e-6, s
        assert np.allclose(eg[s, :5], eo[0, :5], rtol=1e-9, atol=1e-9), s
    assert np.any(eg[:, 4] > 0)  # the lamina envelope is active somewhere


def test_de_short_protocol(demo, ms):
    """The whole protocol with the D/E restraints: deterministic, finite, inactive
    centroid slots stay put, violation records count the per-structure envelope."""
    sids = list(range(5))
    d = de_model(demo, sids)
    seeds = M.lammps_seeds(6535, sids, 11)
    x1, i1 = ms.run(d['prm'], d['x'], d['radii'], d['flags'], d['poly'], d['ptr'], d['sb'], seeds)
    x2, _ = ms.run(d['prm'], d['x'], d['radii'], d['flags'], d['poly'], d['ptr'], d['sb'], seeds)
    assert np.array_equal(x1, x2) and np.all(np.isfinite(x1))
    f, n = d['first'], d['nslot']
    for s in range(len(sids)):
        a = d['active'][s]
        assert np.array_equal(x1[s, f + a:f + n], d['x'][s, f + a:f + n])  # inert padding
        if a:
            assert np.abs(x1[s, f:f + a] - d['x'][s, f:f + a]).max() > 0  # centroids move
    stats = ms.violations(d['prm'], x1, d['radii'], d['flags'], d['poly'], None, d['ptr'], d['sb'], None,
                          [0.0], None, 0.05)
    env1 = stats[:, 2, 103]  # n_imposed of the lamina envelope class
    assert np.array_equal(env1, ((d['flags'] & np.uint32(M.IGM_ATOM_ENV0 << 1)) != 0).sum(1))
    assert np.array_equal(env1, d['nsel'])


def test_de_hbm_path_matches_lds_path(demo, ms):
    """The HBM-resident population engine with per-structure flags: f32 forces equal
    the LDS path's to f32 rounding; a short protocol keeps inactive slots inert, and
    over 16 structures the two engines' final populations are not separated by the KS
    statistic of tests/mstep_stats.py (energies per bead incl. both envelopes, final
    Temp, Verlet rebuilds: same skin on both engines)."""
    import mstep_stats as MS
    from igm_amd._lib import MStepParams, IGM_MSTEP_FORCE_GLOBAL
    sids = list(range(16))
    d = de_model(demo, sids)
    pg = MStepParams.from_buffer_copy(d['prm'])
    pg.flags = IGM_MSTEP_FORCE_GLOBAL
    x = d['x'].copy()
    x[:, :3008] += np.random.default_rng(10).normal(0, 80.0, (len(sids), 3008, 3)).astype(np.float32)
    f_lds, _ = ms.forces(d['prm'], x, d['radii'], d['flags'], d['poly'], d['ptr'], d['sb'], 0.5, 1.2, f32=True)
    f_hbm, _ = ms.forces(pg, x, d['radii'], d['flags'], d['poly'], d['ptr'], d['sb'], 0.5, 1.2, f32=True)
    assert np.abs(f_lds - f_hbm).max() <= 1e-5 * np.abs(f_lds).max()
    seeds = M.lammps_seeds(6535, sids, 11)
    x1, i1 = ms.run(d['prm'], d['x'], d['radii'], d['flags'], d['poly'], d['ptr'], d['sb'], seeds)
    x2, i2 = ms.run(pg, d['x'], d['radii'], d['flags'], d['poly'], d['ptr'], d['sb'], seeds)
    assert np.all(np.isfinite(x2))
    f, n = d['first'], d['nslot']
    for s in range(len(sids)):
        a = d['active'][s]
        assert np.array_equal(x2[s, f + a:f + n], d['x'][s, f + a:f + n])

    def st(info):
        return {'pair': info['pair_energy'] / 3008, 'bond': info['bond_energy'] / 3008,
                'total': info['final_energy'] / 3008, 'env0': info['env_energy'][:, 0] / 3008,
                'env1': info['env_energy'][:, 1] / 3008, 'temp': info['temp'].astype(np.float64),
                'rebuilds': info['nrebuild'].astype(np.float64)}
    ok, pv = MS.same_population(st(i1), st(i2), keys=('pair', 'bond', 'total', 'env0', 'env1', 'temp', 'rebuilds'))
    assert ok, pv
