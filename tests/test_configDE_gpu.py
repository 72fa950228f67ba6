"""Configurations D and E (BASELINE.json configs[3], configs[4]) through the M-step at
their workload size: 200 kb diploid structures (29 838 beads, the population engine)
with the D/E restraints assembled exactly as the Step layer assembles them
(igm_amd.assemble, tests/de200.py), the whole demo protocol shape (4 stages + relax +
CG, MD step counts x0.02), against the fp64 oracle as populations.

  D  per-structure DamID membership (igm_damid_select on the batch's own A-step rows)
     + the k < 0 lamina envelope on the shrunk ellipsoid + the ellipsoid nucleus.
  E  SPRITE centroid slots (inert past each structure's own clusters) and their bounds,
     FISH radial and pair lower/upper bounds, the imaged nucleus map (volumetric
     restraint, VolumeFile EDT sphere).

Statistic (tests/mstep_stats.same_population, the one that rejects a 2x bond K or a
2x evfactor in tests/test_mstep_stats.py): two-sample KS at alpha = 1e-3 over 16 vs 16
structures on E_pair, E_bond, every envelope energy, E_total per bead, the violation
fraction of every monitored restraint (violation records of both final populations
scored by the same bit-exact kernel) and the final Temp.  The same run without bond
pruning (IGM_POP_BOND_PRUNE=0) is bitwise the same: SPRITE centroids (not watched by the
list-build trigger) keep their bonds, DamID and FISH bounds prune like Hi-C's.  Verlet rebuild counts are
not compared: the GPU's default skin is 0.7 maxrad, the oracle's LAMMPS maxrad.
Parity of the DamID k < 0 envelope form and of the volumetric force stays UNPINNED
(no reference output exists): both sides implement the documented
forms, and this test shows the GPU engine reproduces its own oracle at 200 kb.
"""
import os

import numpy as np
import pytest

import de200
import mstep_stats as MS
import oracle
from igm_amd import model as M

pytestmark = pytest.mark.gpu

N = 16
SCALE = 0.02


def _run(config):
    from igm_amd import _lib, assemble as A, mstep, volume as V
    ctx = _lib.context(0)
    pop = de200.population(config, N, first_sid=700)
    vol = None
    if config == 'D':
        spec = de200.spec_D(pop, N, SCALE, ctx)
    else:
        vol = V.sphere_map(5500.0, 100.0)
        spec = de200.spec_E(pop, N, SCALE, ctx, vol)
    sids = np.arange(N)
    b = A.build(pop['xyz'], sids, de200.index_of(pop), spec, ctx)
    assert b.natom > 3072  # past one CU's LDS: the population engine
    seeds = M.lammps_seeds(6535, 700 + sids, 3)
    try:
        xg, ig, sg = A.run(b, seeds, 0.05, ctx)
        xg2, ig2, _ = A.run(b, seeds, 0.05, ctx)
        os.environ['IGM_POP_BOND_PRUNE'] = '0'  # every bond at every step: bitwise the same
        try:
            xg3, ig3, _ = A.run(b, seeds, 0.05, ctx)
        finally:
            del os.environ['IGM_POP_BOND_PRUNE']
        assert np.array_equal(xg, xg3) and ig.tobytes() == ig3.tobytes(), 'bond pruning changed the run'
        if vol is not None:
            oracle.set_volume(vol)
        xo, io, _ = oracle.mstep_run(b.prm, b.x.copy(), b.radii, b.flags, b.poly, b.ptr, b.bonds, seeds, nthreads=16)
        so = mstep.violations(b.prm, xo, b.radii, b.flags, b.poly, b.poly_cls, b.ptr, b.bonds, b.bcls, b.class_cr,
                              b.env_scale, 0.05, ctx=ctx)
    finally:
        if vol is not None:
            oracle.set_volume(None)
            V.stage(ctx, [])
    return b, (xg, ig, sg), (xg2, ig2), (xo, io, so)


@pytest.mark.parametrize('config', ['D', 'E'])
def test_gpu_200kb_protocol_population_matches_oracle(config):
    b, (xg, ig, sg), (xg2, ig2), (xo, io, so) = _run(config)
    assert np.array_equal(xg, xg2) and ig.tobytes() == ig2.tobytes()  # bitwise reproducible
    assert np.all(np.isfinite(xg)) and np.all(np.isfinite(xo))
    assert np.all(ig['final_energy'] < ig['einitial'])
    a, o = de200.run_stats(b, ig, xg, sg), de200.run_stats(b, io, xo, so)
    keys = ('pair', 'bond', 'total', 'viol_frac', 'temp') + tuple('env%d' % e for e in range(b.prm.nenvelopes))
    ok, pv = MS.same_population(a, o, keys=keys)
    assert ok, pv
    names = b.vstat_names(0)
    if config == 'D':
        # the lamina envelope class counts each structure's own DamID members, and the
        # k < 0 term is active in both engines
        d = names.index('Damid')
        members = ((np.atleast_2d(b.flags) & np.uint32(M.IGM_ATOM_ENV0 << 1)) != 0).sum(1)
        assert np.array_equal(sg[:, d, 103], members) and members.min() > 0
        assert np.any(ig['env_energy'][:, 1] != 0) or np.any(io['env_energy'][:, 1] != 0)
    else:
        f, n = b.nbead + 1, b.nslot
        for s in range(N):
            k = b.active[s]
            assert np.array_equal(xg[s, f + k:f + n], b.x[s, f + k:f + n])  # inert slots stay put
            sp, fi = names.index('Sprite'), names.index('Fish')
            cls = b.bcls[b.ptr[s]:b.ptr[s + 1]]
            assert sg[s, sp, 103] == np.count_nonzero(cls == 3) and sg[s, fi, 103] == np.count_nonzero(cls == 4)
        assert b.active.min() > 0 and np.all(sg[:, names.index('Fish'), 103] > 0)
        # the map restraint is active in the initial (1.27x oversized) territories
        assert np.all(ig['einitial'] > ig['final_energy'])


@pytest.mark.parametrize('config', ['D', 'E'])
def test_gpu_200kb_stagewise_matches_oracle(config, heartbeat):
    """Configurations D and E stage by stage (tests/stagewise.py, the design of config C's
    full-protocol test): 16 structures, the demo protocol's MD steps x0.1 in the suite (4 700
    per structure: the oracle's ~120 s per configuration fits the round-end GPU tier next to
    the rest; IGM_DE_STAGEWISE_SCALE=0.2 for the recorded x0.2 run,
    profiles/r06_parity/config{D,E}_stagewise_x0.2.json), each stage's energies -- pair, bond, every envelope (D: the nucleus ellipsoid
    and the k < 0 lamina DamID envelope; E: the volumetric map) -- and temperatures against
    the fp64 oracle from the same coordinates and velocities, the final CG state and the
    product path's whole-protocol igm_mstep_run against the oracle's final state; restraints
    frustrated (16.5k Hi-C-like contacts per structure, 1 500 of them long-range), so the
    final energies stay >= 1e-2 per bead.  Protocol: lammps.py:285-356; restraints:
    ModelingStep.py:402-503."""
    import stagewise as SW
    from igm_amd import _lib, assemble as A, volume as V
    n, scale = 16, float(os.environ.get('IGM_DE_STAGEWISE_SCALE', '0.1'))
    ctx = _lib.context(0)
    pop = de200.population(config, n, first_sid=900)
    vol = None
    if config == 'D':
        spec = de200.spec_D(pop, n, scale, ctx)
    else:
        vol = V.sphere_map(5500.0, 100.0)
        spec = de200.spec_E(pop, n, scale, ctx, vol)
    sids = np.arange(n)
    b = A.build(pop['xyz'], sids, de200.index_of(pop), spec, ctx)
    seeds = M.lammps_seeds(6535, 900 + sids, 2)
    try:
        if vol is not None:
            oracle.set_volume(vol)
        ok, out, (sg, so, sp) = SW.run(b.prm, spec['protocol'], b.x, b.radii, b.flags, b.poly, b.ptr, b.bonds, seeds,
                                       b.nbead, 'config%s_stagewise' % config, ctx=ctx)
    finally:
        if vol is not None:
            oracle.set_volume(None)
            V.stage(ctx, [])
    assert ok, out
    assert len(out['stages'][0]) == 4 + b.prm.nenvelopes  # T1, pair, bond, temp + every envelope
    assert np.median(so['total']) > 1e-2 and np.median(sg['total']) > 1e-2 and np.median(sp['total']) > 1e-2
