"""Volumetric nuclear-body map restraint (configuration E):
VolumeFile round trip, the violation score oracle pinned against the reference's
ExpEnvelope.getScores goldens (CPU), and on the MI355X the violation records
(bit-exact vs the goldens), forces vs the fp64 oracle, and a confining run."""
import os
import tempfile

import numpy as np
import pytest

import oracle
from conftest import load_golden
from igm_amd import model as M
from igm_amd import volume as V
from oracle import volume as OV


def golden_vol(g, b):
    return dict(body_idx=b, nvoxel=g['b%d_nvoxel' % b], center=g['b%d_center' % b], origin=g['b%d_origin' % b],
                grid=g['b%d_grid' % b], matrice=g['b%d_matrice' % b])


@pytest.mark.parametrize('body', [0, 1])
@pytest.mark.parametrize('k', [1.0, -1.0])
def test_oracle_scores_equal_reference(body, k):
    g = load_golden('volume_golden.npz')
    s = OV.exp_envelope_scores(g['b%d_pos' % body], golden_vol(g, body), k)
    assert np.array_equal(s, g['b%d_k%+d_scores' % (body, int(k))])


def test_volume_file_round_trip_and_sphere_map():
    vol = V.sphere_map(1000.0, 100.0, 2)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, 'm.bin')
        V.write_volume(p, vol)
        assert os.path.getsize(p) == 4 + 12 * 4 + 4 * int(np.prod(vol['nvoxel'])) * 4
        back = V.read_volume(p)
    for key in ('nvoxel', 'center', 'origin', 'grid', 'matrice'):
        assert np.array_equal(back[key], vol[key])
    m = vol['matrice']
    lam = m[..., 3].astype(bool)
    # lamina voxels point to themselves; every EDT target is an inside voxel
    ii = np.indices(m.shape[:3]).transpose(1, 2, 3, 0)
    self_t = np.all(m[..., :3] == ii, axis=3)
    t = m[..., :3].reshape(-1, 3)
    assert np.all(lam[t[:, 0], t[:, 1], t[:, 2]])
    assert self_t.sum() > 0 and np.all(lam[self_t])


def test_model_translation_of_exp_envelope():
    class P(object):
        def __init__(self, pos, r, t):
            self.pos, self.r, self.ptype = np.asarray(pos, np.float32), np.float32(r), t

    class Exp(object):
        ftype = 4
        shape = 'exp_map'

        def __init__(self):
            self.particle_ids, self.volume_file, self.k = [0, 1], 'nucleus_3.bin', 1.0

    class Mdl(object):
        id = 0
        particles = [P([0, 0, 0], 10, 0), P([1, 0, 0], 10, 0)]
        forces = [Exp()]

    lm = M.from_igm_model(Mdl())
    assert lm.envelopes == [('volume', 1.0)] and lm.volume_files == ['nucleus_3.bin']
    prm = M.params_from_cfg({'optimization': {'optimizer_options': {'mdsteps': 10, 'tstart': 1, 'tstop': 1}}},
                            lm.envelopes)
    assert prm.env_kind[0] == 1 and prm.nenvelopes == 1


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize('body', [0, 1])
@pytest.mark.parametrize('k', [1.0, -1.0])
def test_gpu_volume_violation_records_equal_reference(body, k):
    from igm_amd import _lib, mstep
    g = load_golden('volume_golden.npz')
    ctx = _lib.context(0)
    V.stage(ctx, [golden_vol(g, body)])
    pos = g['b%d_pos' % body]
    n = len(pos)
    prm = M.params_from_cfg({'optimization': {'optimizer_options': {'mdsteps': 10, 'tstart': 1, 'tstop': 1}}},
                            [('volume', k)])
    flags = np.full(n, M.IGM_ATOM_BEAD | M.IGM_ATOM_ENV0, np.uint32)
    stats = mstep.violations(prm, pos[None], np.full(n, 10.0, np.float32), flags, None, None, None, None, None,
                             [0.0], [0.95], 0.05, ctx=ctx)
    ref = oracle.violations(g['b%d_k%+d_scores' % (body, int(k))], 0.05)
    rec = stats[0, 1]
    assert list(rec[:101]) == ref['counts']
    assert rec[101] == ref['violated_restr'] and rec[102] == ref['n_violations'] and rec[103] == n
    V.stage(ctx, [])


def _demo_volume_case(sids):
    import mstep_fixtures as F
    pop, g3 = F.load()
    atoms = M.Atoms(pop['radii'], envelope_members=[np.arange(len(pop['radii']))])
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    x = F.struct_major(pop, sids, atoms.n)
    x[:, :3008] *= np.float32(1.25)  # push part of the population outside the map
    return atoms, poly, x


@pytest.mark.gpu
@pytest.mark.parametrize('f32', [False, True])
def test_gpu_volume_forces_match_oracle(f32):
    from igm_amd import _lib, mstep
    g = load_golden('volume_golden.npz')
    vol = golden_vol(g, 0)
    ctx = _lib.context(0)
    V.stage(ctx, [vol])
    oracle.set_volume(vol)
    sids = [0, 1, 2]
    atoms, poly, x = _demo_volume_case(sids)
    prm = M.params_from_cfg({'optimization': {'optimizer_options': {'mdsteps': 10, 'tstart': 1, 'tstop': 1}}},
                            [('volume', 1.0)])
    fg, eg = mstep.forces(prm, x, atoms.radii, atoms.flags, poly, None, None, 1.0, 1.1, f32=f32, ctx=ctx)
    fo, eo = oracle.mstep_forces(prm, x, atoms.radii, atoms.flags, poly, None, None, 1.0, 1.1)
    oracle.set_volume(None)
    V.stage(ctx, [])
    assert np.all(eo[:, 3] > 0)  # the map restraint is active
    if f32:
        assert np.linalg.norm(fg - fo) <= 1e-5 * np.linalg.norm(fo)
    else:
        assert np.abs(fg - fo).max() <= 1e-6 * np.abs(fo).max() + 1e-6
        assert np.allclose(eg[:, 3], eo[:, 3], rtol=1e-9)


@pytest.mark.gpu
def test_gpu_volume_confines_short_protocol():
    """A short protocol with only the map restraint (per-structure map index) pulls
    the beads that start outside the nucleus map back inside."""
    import json
    from igm_amd import _lib, mstep
    from igm_amd.synthetic import DEMO_PROTOCOL
    g = load_golden('volume_golden.npz')
    vol = golden_vol(g, 0)
    ctx = _lib.context(0)
    sids = [0, 1, 2, 3]
    V.stage(ctx, [vol, vol], struct_map=[0, 1, 0, 1])
    atoms, poly, x = _demo_volume_case(sids)
    p = json.loads(json.dumps(DEMO_PROTOCOL))
    p['custom_annealing_protocol']['mdsteps'] = [200, 200, 200, 200]
    p['custom_annealing_protocol']['relax']['mdsteps'] = 50
    prm = M.params_from_cfg({'optimization': {'optimizer_options': p}}, [('volume', 1.0)])
    seeds = M.lammps_seeds(6535, sids, 11)
    xo, info = mstep.run(prm, x, atoms.radii, atoms.flags, poly, None, None, seeds, ctx=ctx)
    V.stage(ctx, [])

    def outside(xx):
        ix = np.rint((xx[:, :3008] - vol['origin']) / vol['grid']).astype(int)
        ix = np.clip(ix, 0, vol['nvoxel'] - 1)
        return (vol['matrice'][ix[..., 0], ix[..., 1], ix[..., 2], 3] == 0).mean()

    assert np.all(np.isfinite(xo))
    assert outside(x) > 0.05 and outside(xo) < 0.5 * outside(x)
