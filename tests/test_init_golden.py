"""The A-step setup and the init steps (8(f)1) against outputs of the
REFERENCE itself (tests/golden/make_golden_init.py -> init_golden.npz):

  * select_pairs / plast_from_rows == the '<b>.in.npy' batches ActivationDistanceStep.setup
    (ActivationDistanceStep.py:111-194) writes for the demo .hcs: CSR (coo_generator)
    order, the intra / inter sigma filter (inter disabled included), plast read from a
    previous actdist file through coo -> lil with row, col < n -- all four columns exact;
  * generate_territories == RandomInit.generate_territories (RandomInit.py:207-240)
    after np.random.seed, draw for draw;
  * the RelaxInit model (RelaxInit.py:93-258: Steric, Polymer, Envelope) == the
    reference LammpsModel's bond list, atoms, PairIJ, seeds and protocol;
  * GPU: the batched relax against the fp64 oracle as populations.
"""
import os

import numpy as np
import pytest

import oracle
import mstep_fixtures as F
import mstep_stats as MS
from conftest import GOLDEN
from igm_amd import astep, init as I, model as M
from igm_amd._lib import row_dtype


@pytest.fixture(scope='module')
def gold():
    return np.load(os.path.join(GOLDEN, 'init_golden.npz'))


@pytest.mark.parametrize('case', ['c0', 'c1', 'c2'])
def test_select_pairs_equals_reference_setup(gold, case):
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    hic = np.load(os.path.join(GOLDEN, 'demo_hic_pairs.npz'))
    nhap = int(hic['nhap'])
    # the .hcs upper triangle restricted to p >= 0.02 (every case's sigmas are >= 0.02)
    indptr = np.concatenate([[0], np.cumsum(np.bincount(hic['i'], minlength=nhap))])
    intra, inter = gold['a2_%s_sigma' % case]
    inter = False if inter < 0 else float(inter)
    last = None
    if case == 'c1':
        g1 = np.load(os.path.join(GOLDEN, 'actdist_golden.npz'))
        last = np.zeros(len(g1['s0.2_c1_rows_row']), row_dtype)
        for k in ('row', 'col', 'dist', 'prob'):
            last[k] = g1['s0.2_c1_rows_' + k]
    pairs = astep.select_pairs(indptr, hic['j'], hic['p'], pop['hap_chrom'], float(intra), inter, last_rows=last)
    ref = gold['a2_%s_pairs' % case]
    assert len(pairs) == len(ref)
    assert np.array_equal(pairs['i'], ref[:, 0].astype(np.int32))
    assert np.array_equal(pairs['j'], ref[:, 1].astype(np.int32))
    assert np.array_equal(pairs['pwish'], ref[:, 2])
    assert np.array_equal(pairs['plast'], ref[:, 3])
    if case == 'c1':
        assert np.count_nonzero(ref[:, 3]) > 1000  # the previous probabilities were picked up


@pytest.mark.parametrize('seed,R', [(0, 5000), (0, 7000), (5, 5000), (5, 7000)])
def test_generate_territories_equals_reference(gold, seed, R):
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    got = I.generate_territories(pop['chrom_sizes'], float(R), np.random.RandomState(seed))
    ref = gold['terr_s%d_R%d' % (seed, R)]
    assert got.shape == ref.shape
    # the same draws; numpy's vectorised sin/cos/arccos vs the reference's math.* differ by ulps
    assert np.allclose(got, ref, rtol=0, atol=1e-9 * R)


def test_relax_model_equals_reference_lammps_model(gold):
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    radii = pop['radii']
    atoms = M.Atoms(radii)
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], radii, 2.0, 1.0)
    for sid in (0, 1):
        ref = gold['relax_bonds_%d' % sid]
        bt = gold['relax_bond_types_%d' % sid]
        assert int(gold['relax_natoms_%d' % sid]) == atoms.n  # beads + the envelope's static centre
        assert np.array_equal(poly['i'], ref[:, 0]) and np.array_equal(poly['j'], ref[:, 1])
        assert np.array_equal(poly['r0'], bt[ref[:, 2], 2].astype(np.float32))
        assert np.array_equal(poly['k'], bt[ref[:, 2], 1].astype(np.float32))
        lam = str(gold['relax_lam_text_%d' % sid])
        seed = M.lammps_seeds(6535, [sid], 1)[0]  # runtime/step_no defaults to 1 (lammps.py:435)
        assert 'velocity nonfixed create 5000.0 %d' % seed in lam
        cfg = {'optimization': {'optimizer_options': F.DEMO_PROTOCOL}}
        prm = M.params_from_cfg(cfg, [((5500.0,) * 3, 1.0)])
        for k in range(prm.nstages):
            assert 'temp/rescale 1  %s %s 0.1 1' % (prm.tstart[k], prm.tstop[k]) in lam
        assert 'ellipsoidalenvelope 6600.0 6600.0 6600.0 1.0' in lam
        data = str(gold['relax_data_text_%d' % sid])
        line = data[data.index('PairIJ Coeffs'):].split('\n')[2].split()
        dc = np.float32(np.float32(radii[0]) + np.float32(radii[0]))
        assert float(line[2]) == (float(dc) / np.pi) ** 2


@pytest.mark.gpu
def test_gpu_relax_population_matches_oracle():
    """RelaxInit on the batched engine vs the fp64 oracle of the same model (steric,
    polymer, sphere envelope), 16 reference-drawn territories, protocol steps x0.1."""
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    S = 16
    xyz = np.stack([I.generate_territories(pop['chrom_sizes'], 7000.0, np.random.RandomState(s))
                    for s in range(S)]).astype(np.float32)
    prot = MS.scaled_protocol(F.DEMO_PROTOCOL, 0.1)
    cfg = {'model': {'restraints': {'excluded': {'evfactor': 1.0},
                                    'polymer': {'contact_range': 2.0, 'polymer_kspring': 1.0},
                                    'envelope': {'nucleus_shape': 'sphere', 'nucleus_radius': 5500.0,
                                                 'nucleus_kspring': 1.0}}},
           'optimization': {'optimizer_options': prot}, 'runtime': {'step_no': 1}}
    sids = list(range(S))
    xg, ig = I.relax_population(cfg, xyz, pop['radii'], pop['chrom'], pop['copy'], sids)
    atoms = M.Atoms(pop['radii'])
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    prm = M.params_from_cfg(cfg, [((5500.0,) * 3, 1.0)], evfactor=1.0)
    x = np.zeros((S, atoms.n, 3), np.float32)
    x[:, :atoms.nbead] = xyz
    xo, io, _ = oracle.mstep_run(prm, x, atoms.radii, atoms.flags, poly, None, None,
                                 M.lammps_seeds(6535, sids, 1), nthreads=16)
    sg = MS.population_stats(ig, xg, poly, None, None, atoms.nbead)
    so = MS.population_stats(io, xo[:, :atoms.nbead], poly, None, None, atoms.nbead)
    ok, pv = MS.same_population(sg, so, keys=('pair', 'bond', 'total', 'viol_frac'))
    assert ok, pv
    assert np.all(np.isfinite(xg)) and np.all(ig['final_energy'] <= ig['einitial'])  # CG may stop at once
