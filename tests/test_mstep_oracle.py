"""M-step oracle (fp64 CPU restatement) and host-side restraint assembly, pinned
against the reference's own outputs: the LAMMPS inputs the reference writes (G3),
its Hi-C selection (G4), its violation records (G6) and the per-structure energies
of the demo run summary (G7)."""
import json

import numpy as np
import pytest

import oracle
import mstep_fixtures as F
from igm_amd import model as M


@pytest.fixture(scope='module')
def demo():
    return F.load()


def test_polymer_and_hic_bonds_equal_reference_lammps_model(demo):
    """Our polymer bonds + the reference Hi-C selection == the .data bond list of the
    reference LammpsModel (lammps_model.py:277-301), bond by bond, in order."""
    pop, g3 = demo
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    for sid in (0, 1):
        hic, _ = F.hic_bonds_from_golden(g3, pop['radii'], sid)
        ours = np.concatenate([poly, hic])
        ref = F.golden_bonds(g3, sid)
        # the reference order is: polymer (forces added first), inter, intra
        assert len(ours) == len(ref)
        assert np.array_equal(ours['i'], ref['i']) and np.array_equal(ours['j'], ref['j'])
        assert np.array_equal(ours['r0'], ref['r0'].astype(np.float32))
        assert np.array_equal(ours['k'], ref['k'])


def test_pairij_and_seed_match_reference_script(demo):
    """PairIJ A = ((ri+rj)/pi)^2 * evfactor and the velocity seeds of the .lam file."""
    pop, g3 = demo
    data = str(g3['data_text_0'])
    line = data[data.index('PairIJ Coeffs'):].split('\n')[2].split()
    r = np.float32(pop['radii'][0])
    dc = np.float32(r + r)
    assert float(line[2]) == (float(dc) / np.pi) ** 2 * 1.0
    lam = str(g3['lam_text_1'])
    seeds = M.lammps_seeds(6535, [1], 11)
    assert 'velocity nonfixed create 5000.0 %d' % seeds[0] in lam
    assert 'velocity nonfixed create 1.0 %d' % (seeds[0] + 3) in lam
    assert M.lammps_seeds(6535, [0], 11)[0] == 1  # D6: struct 0 always gets seed 1


def test_protocol_params_from_reference_script(demo):
    pop, g3 = demo
    atoms, poly, prm, chrom = F.demo_model(pop)
    lam = str(g3['lam_text_0'])
    assert prm.nstages == 4 and list(prm.mdsteps[:4]) == [5000, 15000, 15000, 10000]
    for k, (t0, t1) in enumerate(zip(prm.tstart[:4], prm.tstop[:4])):
        assert 'temp/rescale 1  %s %s 0.1 1' % (t0, t1) in lam
    assert 'ellipsoidalenvelope 6600.0 6600.0 6600.0 1.0' in lam  # 5500 * envf 1.2
    assert 'minimize 0.0001 1e-06 500 500' in lam
    assert prm.relax_steps == 500 and prm.relax_max_velocity == 10.0


def test_oracle_hic_selection_equals_reference(demo):
    pop, g3 = demo
    xyz = F.struct_major(pop, list(range(10)), 3008)
    sel = oracle.hic_select(xyz, pop['chrom'], g3['act_row'], g3['act_col'], g3['act_dist'])
    for s in range(10):
        for code, key in ((1, 'sel_inter_%d'), (2, 'sel_intra_%d')):
            got = np.stack([g3['act_row'][sel[s] == code], g3['act_col'][sel[s] == code]], 1)
            assert np.array_equal(got, g3[key % s])


def test_oracle_pair_energy_pinned_by_demo_summary(demo):
    """E_pair of the final demo coordinates == summary.bystructure.pair_energies to the
    %g quantization of the dumped coordinates, on the CG-final frames (D13)."""
    pop, _ = demo
    atoms, poly, prm, chrom = F.demo_model(pop)
    x = F.struct_major(pop, list(range(100)), atoms.n)
    f, e = oracle.mstep_forces(prm, x, atoms.radii, atoms.flags, None, None, None, 1.0, 1.0)
    pe = pop['pin_pair_energies']
    rel = np.abs(e[:, 1] - pe) / np.maximum(np.abs(pe), 1e-9)
    good = rel < 1e-3
    assert good.sum() >= 45
    assert np.median(rel[good]) < 3e-5
    # ellipsoidal envelope energy (k > 0) pinned by thermo f_envelope0
    fe = pop['pin_f_envelope0']
    assert np.corrcoef(e[:, 3], fe)[0, 1] > 0.9999
    assert abs(e[:, 3].mean() - fe.mean()) / fe.mean() < 0.01


def test_oracle_forces_are_energy_gradients(demo):
    """Central differences of the oracle energy == oracle forces (pair, bond, envelope)."""
    pop, g3 = demo
    atoms, poly, prm, chrom = F.demo_model(pop)
    x = F.struct_major(pop, [0], atoms.n).astype(np.float64)
    rng = np.random.default_rng(0)
    x[0, :3008] += rng.normal(0, 150.0, (3008, 3))  # stretch bonds, overlap beads, leave envelope
    x[0, :20] *= 1.6
    bonds = F.golden_bonds(g3, 0)
    f, e = oracle.mstep_forces(prm, x.astype(np.float32), atoms.radii, atoms.flags, bonds, None, None, 0.5, 1.0)
    x32 = x.astype(np.float32)
    for a in [0, 5, 17, 100, 1557, 2000]:
        for d in range(3):
            h = np.float32(0.05)
            xp = x32.copy()
            xm = x32.copy()
            xp[0, a, d] += h
            xm[0, a, d] -= h
            _, ep = oracle.mstep_forces(prm, xp, atoms.radii, atoms.flags, bonds, None, None, 0.5, 1.0)
            _, em = oracle.mstep_forces(prm, xm, atoms.radii, atoms.flags, bonds, None, None, 0.5, 1.0)
            num = -(ep[0, 0] - em[0, 0]) / (float(xp[0, a, d]) - float(xm[0, a, d]))
            assert abs(num - f[0, a, d]) <= 1e-3 * max(1.0, abs(f[0, a, d])), (a, d, num, f[0, a, d])


def test_oracle_violations_equal_reference(demo):
    """Violation histograms / counts of the reference (G6) from a numpy restatement."""
    pop, g3 = demo
    viol = np.load(F.os.path.join(F.GOLDEN, 'violations_golden.npz'))
    for sid in range(10):
        vstat = json.loads(str(g3['vstat_%d' % sid]))
        for key, rec in vstat.items():
            name = key.split('[')[0]
            mine = oracle.violations(viol['vs_%s_%d' % (name, sid)], 0.05)
            assert mine['counts'] == rec['counts']
            assert mine['violated_restr'] == rec['violated_restr']
            assert mine['n_violations'] == rec['n_violations']


def test_ranpark_known_answer():
    """Park & Miller (1988) minimal standard: seed 1, after 10000 draws -> 1043618065."""
    assert oracle.ranpark_state(1, 10000) == 1043618065


def test_oracle_md_segment_conserves_energy_at_small_dt(demo):
    """nve without limit/rescale (huge window) conserves E_kin + E_pot in the oracle."""
    pop, g3 = demo
    atoms, poly, prm, chrom = F.demo_model(pop)
    prm.timestep = 0.01
    prm.t_window = 1e30
    x = F.struct_major(pop, [3], atoms.n).astype(np.float64)
    v = oracle.velocity_create(atoms.flags, 1.0, 77)[None]
    bonds = F.golden_bonds(g3, 0)
    f0, e0 = oracle.mstep_forces(prm, x.astype(np.float32), atoms.radii, atoms.flags, bonds, None, None, 1.0, 1.0)
    x1, v1 = oracle.mstep_md(prm, x, v, atoms.radii, atoms.flags, bonds, None, None, 1.0, 1.0, 1.0, 1.0, 1e9, 200)
    # energies from the f64 positions: evaluate through the f32 interface is lossy; use kinetic drift bound
    ek0 = 0.5 * (v ** 2).sum()
    ek1 = 0.5 * (v1 ** 2).sum()
    _, e1 = oracle.mstep_forces(prm, x1.astype(np.float32), atoms.radii, atoms.flags, bonds, None, None, 1.0, 1.0)
    drift = abs((ek1 + e1[0, 0]) - (ek0 + e0[0, 0]))
    assert drift < 1e-3 * (abs(e0[0, 0]) + ek0) + 5.0
