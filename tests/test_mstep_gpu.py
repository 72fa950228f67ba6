"""M-step on the MI355X through the C ABI, against the fp64 CPU oracle (same
algorithm) and the reference's own restraint selection / violation records."""
import json
import os

import numpy as np
import pytest

import oracle
import mstep_fixtures as F
from igm_amd import model as M

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def demo():
    return F.load()


@pytest.fixture(scope='module')
def ms():
    from igm_amd import mstep
    return mstep


def short_protocol(steps=(300, 300, 300, 300), relax=100):
    p = json.loads(json.dumps(F.DEMO_PROTOCOL))
    p['custom_annealing_protocol']['mdsteps'] = list(steps)
    p['custom_annealing_protocol']['relax']['mdsteps'] = relax
    return p


def test_gpu_hic_select_equals_reference(demo, ms):
    """interHiC + intraHiC selection (G4) and bond parameters (G3), bit-exact."""
    pop, g3 = demo
    atoms, poly, prm, chrom = F.demo_model(pop)
    xyz = F.struct_major(pop, list(range(10)), atoms.n)
    ptr, bonds, cls = ms.hic_select(xyz, atoms.radii, chrom, g3['act_row'], g3['act_col'], g3['act_dist'], 2.0, 1.0)
    for s in range(10):
        b = bonds[ptr[s]:ptr[s + 1]]
        c = cls[ptr[s]:ptr[s + 1]]
        ref, rcls = F.hic_bonds_from_golden(g3, atoms.radii, s)
        assert np.array_equal(b['i'], ref['i']) and np.array_equal(b['j'], ref['j'])
        assert np.array_equal(b['r0'], ref['r0']) and np.array_equal(b['k'], ref['k'])
        assert np.array_equal(c, rcls)
    # the assembled list equals the reference LammpsModel bonds of structures 0 and 1
    for s in (0, 1):
        full = np.concatenate([poly, bonds[ptr[s]:ptr[s + 1]]])
        ref = F.golden_bonds(g3, s)
        assert np.array_equal(full['i'], ref['i']) and np.array_equal(full['j'], ref['j'])
        assert np.array_equal(full['r0'], ref['r0'].astype(np.float32))


def test_gpu_velocity_create_matches_oracle(demo, ms):
    """RNG-stream parity of 'velocity nonfixed create' (RanPark, loop all, mom yes)."""
    pop, _ = demo
    atoms, _, _, _ = F.demo_model(pop)
    seeds = np.array([1, 84956, 84959, 9190037], np.int32)
    v = ms.velocity_create(atoms.flags, seeds, 5000.0)
    for k, sd in enumerate(seeds):
        ref = oracle.velocity_create(atoms.flags, 5000.0, int(sd))
        assert np.allclose(v[k], ref, rtol=2e-6, atol=1e-5)
        assert np.all(v[k][atoms.flags & M.IGM_ATOM_FIXED != 0] == 0)


def _bonds_for(demo, sids):
    pop, g3 = demo
    atoms, poly, prm, chrom = F.demo_model(pop)
    per = []
    for s in sids:
        b, _ = F.hic_bonds_from_golden(g3, atoms.radii, s % 10)
        per.append(b)
    ptr, sb = M.concat_bonds(per)
    return atoms, poly, prm, ptr, sb


@pytest.mark.parametrize('evf,envf', [(0.5, 1.2), (1.0, 1.0)])
def test_gpu_forces_f64_match_oracle(demo, ms, evf, envf):
    pop, g3 = demo
    sids = list(range(10))
    atoms, poly, prm, ptr, sb = _bonds_for(demo, sids)
    x = F.struct_major(pop, sids, atoms.n)
    rng = np.random.default_rng(3)
    x[:, :3008] += rng.normal(0, 120.0, (10, 3008, 3)).astype(np.float32)  # overlaps + stretched bonds
    x[:, :50] *= np.float32(1.5)  # some beads outside the envelope
    fg, eg = ms.forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, evf, envf)
    fo, eo = oracle.mstep_forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, evf, envf)
    scale = np.abs(fo).max()
    assert np.abs(fg - fo).max() <= 1e-6 * scale + 1e-6  # f64 path, rounded to f32 on output
    assert np.allclose(eg[:, :4], eo[:, :4], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize('evf,envf', [(0.5, 1.2), (1.0, 1.0)])
def test_gpu_forces_f32_match_oracle(demo, ms, evf, envf):
    """The f32 MD force path vs the fp64 oracle: <= 1e-5 of the force scale."""
    pop, g3 = demo
    sids = list(range(10))
    atoms, poly, prm, ptr, sb = _bonds_for(demo, sids)
    x = F.struct_major(pop, sids, atoms.n)
    rng = np.random.default_rng(4)
    x[:, :3008] += rng.normal(0, 120.0, (10, 3008, 3)).astype(np.float32)
    x[:, :50] *= np.float32(1.5)
    fg, _ = ms.forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, evf, envf, f32=True)
    fo, _ = oracle.mstep_forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, evf, envf)
    err = np.linalg.norm(fg - fo, axis=2)
    ref = np.linalg.norm(fo, axis=2)
    assert np.linalg.norm(err) <= 1e-5 * np.linalg.norm(ref)
    assert np.all(err <= 2e-4 * ref + 1e-2 * max(1.0, np.median(ref)))


def test_gpu_md_segment_tracks_oracle(demo, ms):
    """20 steps of nve/limit + temp/rescale from identical x, v: the f32 GPU trajectory
    stays within 1e-3 nm of the fp64 oracle (chaos has not amplified rounding yet)."""
    pop, g3 = demo
    sids = [0, 1, 2]
    atoms, poly, prm, ptr, sb = _bonds_for(demo, sids)
    x = F.struct_major(pop, sids, atoms.n)
    v = np.stack([oracle.velocity_create(atoms.flags, 50.0, 11 + s) for s in sids]).astype(np.float32)
    xg, vg = ms.md(prm, x, v, atoms.radii, atoms.flags, poly, ptr, sb, 1.0, 1.0, 50.0, 40.0, 1000.0, 20)
    xo, vo = oracle.mstep_md(prm, x.astype(np.float64), v.astype(np.float64), atoms.radii, atoms.flags, poly, ptr,
                             sb, 1.0, 1.0, 50.0, 40.0, 1000.0, 20)
    moved = np.abs(xo - x).max()
    assert moved > 1.0  # it did move
    assert np.abs(xg - xo).max() < 1e-3 * max(1.0, moved)
    assert np.allclose(vg, vo, rtol=1e-3, atol=1e-3 * np.abs(vo).max())


def test_gpu_cg_matches_oracle(demo, ms):
    """CG only (no annealing stages): same algorithm in f64 on both sides."""
    pop, g3 = demo
    sids = [0, 1, 2, 3]
    atoms, poly, prm, ptr, sb = _bonds_for(demo, sids)
    prm.nstages = 0
    x = F.struct_major(pop, sids, atoms.n)
    rng = np.random.default_rng(5)
    x[:, :3008] += rng.normal(0, 60.0, (len(sids), 3008, 3)).astype(np.float32)
    seeds = M.lammps_seeds(6535, sids, 11)
    xg, ig = ms.run(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    xo, io, x64 = oracle.mstep_run(prm, x.copy(), atoms.radii, atoms.flags, poly, ptr, sb, seeds, nthreads=4)
    assert np.allclose(ig['einitial'], io['einitial'], rtol=1e-10)
    assert np.allclose(ig['final_energy'], io['final_energy'], rtol=1e-5)
    assert np.all(ig['final_energy'] < ig['einitial'])
    # identical arithmetic up to summation order: the iteration paths agree for a while
    assert np.all(np.abs(ig['cg_iters'] - io['cg_iters']) <= max(5, 0.1 * io['cg_iters'].max()))


def test_gpu_full_protocol_short(demo, ms):
    """Whole protocol (4 stages, relax, velocity create, CG) on a shortened schedule
    (300 MD steps per stage): runs, is bitwise deterministic, and -- 16 structures of
    the demo model with frustrated restraints -- is not separated from the fp64
    oracle's population by the KS statistic of tests/mstep_stats.py (energies per
    bead, envelope energy, violation fraction, final Temp, rebuilds at the same skin)."""
    import mstep_stats as MS
    from test_mstep_stats import _inputs
    sids = list(range(16))
    atoms, poly, ptr, sb, x = _inputs(sids, 1000, 1000)
    p = M.params_from_cfg({'optimization': {'optimizer_options': short_protocol()}}, [((5500.0,) * 3, 1.0)])
    p.skin = 280.7308  # LAMMPS 'neighbor maxrad bin' on both sides, so rebuild counts compare
    seeds = M.lammps_seeds(6535, sids, 11)
    xg, ig = ms.run(p, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    xg2, ig2 = ms.run(p, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    assert np.array_equal(xg, xg2)  # bitwise reproducible
    assert np.all(np.isfinite(xg))
    xo, io, _ = oracle.mstep_run(p, x.copy(), atoms.radii, atoms.flags, poly, ptr, sb, seeds, nthreads=16)
    sg = MS.population_stats(ig, xg, poly, ptr, sb, atoms.nbead)
    so = MS.population_stats(io, xo, poly, ptr, sb, atoms.nbead)
    sg['env'], so['env'] = ig['env_energy'][:, 0] / atoms.nbead, io['env_energy'][:, 0] / atoms.nbead
    ok, pv = MS.same_population(sg, so, keys=('pair', 'bond', 'env', 'total', 'viol_frac', 'temp', 'rebuilds'))
    assert ok, pv
    assert np.all(ig['temp'] < 0.2)


def test_gpu_violations_equal_reference(demo, ms):
    """The ModelingStep violation record (G6) of the demo final coordinates, exactly."""
    pop, g3 = demo
    sids = list(range(10))
    atoms, poly, prm, chrom = F.demo_model(pop)
    per, pcls = [], []
    for s in sids:
        b, c = F.hic_bonds_from_golden(g3, atoms.radii, s)
        per.append(b)
        pcls.append(c)
    ptr, sb = M.concat_bonds(per)
    scls = np.concatenate(pcls)
    x = F.struct_major(pop, sids, atoms.n)
    shared_cls = np.full(len(poly), M.CLASS_POLYMER, np.int32)
    class_cr = np.array([2.0, 2.0, 2.0])
    stats = ms.violations(prm, x, atoms.radii, atoms.flags, poly, shared_cls, ptr, sb, scls, class_cr, [550.0], 0.05)
    names = {0: 'Polymer', 1: 'interHiC', 2: 'intraHiC', 3: 'Envelope[shape=sphere,k=1.0,a=5500,b=5500,c=5500]'}
    for s in sids:
        vstat = json.loads(str(g3['vstat_%d' % s]))
        for c, name in names.items():
            rec = vstat[name]
            assert stats[s, c, :101].tolist() == rec['counts'], (s, name)
            assert stats[s, c, 101] == rec['violated_restr']
            assert stats[s, c, 102] == rec['n_violations']
            assert stats[s, c, 103] == rec['n_imposed']


def test_gpu_bond_pruning_is_bitwise_exact(demo, ms, monkeypatch):
    """The LDS anneal kernel's bond pruning (bond_candidates: at each list build, the
    bonds that cannot act before the next build are skipped) changes no bit: the same
    config B batch (frustrated demo restraints, the whole protocol shape at 300 MD steps
    per stage, default skins) with IGM_BOND_PRUNE=0 and with pruning on ends in the
    same coordinates, energies, temperatures and rebuild counts."""
    from test_mstep_stats import _inputs
    sids = list(range(16))
    atoms, poly, ptr, sb, x = _inputs(sids, 1000, 1000)
    p = M.params_from_cfg({'optimization': {'optimizer_options': short_protocol()}}, [((5500.0,) * 3, 1.0)])
    seeds = M.lammps_seeds(6535, sids, 7)
    monkeypatch.setenv('IGM_BOND_PRUNE', '0')
    x0, i0 = ms.run(p, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    monkeypatch.delenv('IGM_BOND_PRUNE')
    x1, i1 = ms.run(p, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    assert np.array_equal(x0, x1) and i0.tobytes() == i1.tobytes()
    assert np.all(i1['nrebuild'] > 10) and np.all(np.isfinite(x1))
