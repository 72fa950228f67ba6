"""The two M-step kernel families against each other and against the fp64 oracle:
the LDS-resident path (structures of <= 3072 atoms, 2 Mb) and the HBM-resident path
(any size; the 200 kb model with 29 838 beads), through the C ABI."""
import json

import numpy as np
import pytest

import oracle
import mstep_fixtures as F
from igm_amd import model as M
from igm_amd import synthetic as syn
from igm_amd import _lib
from igm_amd._lib import IGM_MSTEP_FORCE_GLOBAL

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def demo():
    return F.load()


@pytest.fixture(scope='module')
def ms():
    from igm_amd import mstep
    return mstep


def _demo_inputs(demo, sids):
    pop, g3 = demo
    atoms, poly, prm, chrom = F.demo_model(pop)
    per = [F.hic_bonds_from_golden(g3, atoms.radii, s % 10)[0] for s in sids]
    ptr, sb = M.concat_bonds(per)
    x = F.struct_major(pop, sids, atoms.n)
    return atoms, poly, prm, ptr, sb, x


def _global(prm):
    prm.flags = IGM_MSTEP_FORCE_GLOBAL
    return prm


def test_gpu_hbm_path_f32_forces_equal_lds_path(demo, ms):
    """Same arithmetic on both paths; the summation order follows each path's cell
    grid (the LDS grid is capped at 4096 cells), so equal to f32 rounding."""
    atoms, poly, prm, ptr, sb, x = _demo_inputs(demo, list(range(6)))
    rng = np.random.default_rng(7)
    x[:, :3008] += rng.normal(0, 120.0, (6, 3008, 3)).astype(np.float32)
    f_lds, _ = ms.forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, f32=True)
    f_hbm, _ = ms.forces(_global(prm), x, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, f32=True)
    assert np.abs(f_lds - f_hbm).max() <= 1e-5 * np.abs(f_lds).max()


def test_gpu_hbm_path_f64_forces_match_oracle(demo, ms):
    atoms, poly, prm, ptr, sb, x = _demo_inputs(demo, list(range(4)))
    rng = np.random.default_rng(8)
    x[:, :3008] += rng.normal(0, 120.0, (4, 3008, 3)).astype(np.float32)
    fg, eg = ms.forces(_global(prm), x, atoms.radii, atoms.flags, poly, ptr, sb, 1.0, 1.0)
    fo, eo = oracle.mstep_forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, 1.0, 1.0)
    assert np.abs(fg - fo).max() <= 1e-6 * np.abs(fo).max() + 1e-6
    assert np.allclose(eg[:, :4], eo[:, :4], rtol=1e-9, atol=1e-9)


def _few_bonds(demo, sids, nhic=1500):
    """polymer + the first nhic Hi-C bonds: small enough for the LDS-staged bond path"""
    atoms, poly, prm, ptr, sb, x = _demo_inputs(demo, sids)
    per = [sb[ptr[k]:ptr[k + 1]][:nhic] for k in range(len(sids))]
    ptr, sb = M.concat_bonds(per)
    return atoms, poly, prm, ptr, sb, x


@pytest.mark.parametrize('nhic', [1500, None])
def test_gpu_f32_forces_lds_bonds_match_oracle(demo, ms, nhic):
    """nhic=1500: the structure's bonds are staged in LDS; None: all demo Hi-C bonds
    (too many for LDS, read from HBM)."""
    sids = list(range(4))
    atoms, poly, prm, ptr, sb, x = _few_bonds(demo, sids, nhic) if nhic else _demo_inputs(demo, sids)
    rng = np.random.default_rng(12)
    x[:, :3008] += rng.normal(0, 120.0, (4, 3008, 3)).astype(np.float32)
    fg, _ = ms.forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, f32=True)
    fo, _ = oracle.mstep_forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2)
    err = np.linalg.norm(fg - fo, axis=2)
    assert np.linalg.norm(err) <= 1e-5 * np.linalg.norm(np.linalg.norm(fo, axis=2))


@pytest.mark.parametrize('path', ['lds', 'hbm', 'lds_bonds'])
def test_gpu_md_segment_both_paths_track_oracle(demo, ms, path):
    if path == 'lds_bonds':
        atoms, poly, prm, ptr, sb, x = _few_bonds(demo, [0, 1, 2])
    else:
        atoms, poly, prm, ptr, sb, x = _demo_inputs(demo, [0, 1, 2])
    if path == 'hbm':
        _global(prm)
    v = np.stack([oracle.velocity_create(atoms.flags, 50.0, 11 + s) for s in range(3)]).astype(np.float32)
    xg, vg = ms.md(prm, x, v, atoms.radii, atoms.flags, poly, ptr, sb, 1.0, 1.0, 50.0, 40.0, 1000.0, 20)
    xo, vo = oracle.mstep_md(prm, x.astype(np.float64), v.astype(np.float64), atoms.radii, atoms.flags, poly, ptr,
                             sb, 1.0, 1.0, 50.0, 40.0, 1000.0, 20)
    moved = np.abs(xo - x).max()
    assert moved > 1.0
    assert np.abs(xg - xo).max() < 1e-3 * max(1.0, moved)


def test_gpu_hbm_path_protocol_short(demo, ms):
    atoms, poly, prm, ptr, sb, x = _demo_inputs(demo, list(range(4)))
    p = json.loads(json.dumps(F.DEMO_PROTOCOL))
    p['custom_annealing_protocol']['mdsteps'] = [200, 200, 200, 200]
    p['custom_annealing_protocol']['relax']['mdsteps'] = 50
    prm = _global(M.params_from_cfg({'optimization': {'optimizer_options': p}}, [((5500.0,) * 3, 1.0)]))
    seeds = M.lammps_seeds(6535, list(range(4)), 3)
    xg, ig = ms.run(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    xg2, _ = ms.run(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    assert np.array_equal(xg, xg2)
    assert np.all(np.isfinite(xg)) and np.all(ig['final_energy'] < ig['einitial'])
    assert np.all(ig['final_energy'] / 3008 < 50.0)


# ------------------------------------------------------------------ 200 kb
@pytest.fixture(scope='module')
def model200():
    pop = syn.population_200kb(2)
    atoms = M.Atoms(pop['radii'])
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    prm = M.params_from_cfg({'optimization': {'optimizer_options': F.DEMO_PROTOCOL}}, [((5500.0,) * 3, 1.0)])
    x = np.zeros((2, atoms.n, 3), np.float32)
    x[:, :atoms.nbead] = pop['xyz']
    # a few thousand random contacts per structure (Hi-C-like bonds)
    rng = np.random.default_rng(9)
    per = []
    for s in range(2):
        i = rng.integers(0, atoms.nbead, 4000)
        j = (i + rng.integers(2, 60, 4000)) % atoms.nbead
        b = np.zeros(4000, poly.dtype)
        b['i'], b['j'] = i, j
        b['r0'] = M.r0_contact(2.0, atoms.radii[i], atoms.radii[j]).astype(np.float32)
        b['k'] = 1.0
        per.append(b)
    ptr, sb = M.concat_bonds(per)
    return atoms, poly, prm, ptr, sb, x


def test_gpu_200kb_forces_match_oracle(ms, model200):
    atoms, poly, prm, ptr, sb, x = model200
    assert atoms.nbead == 29838
    fg, eg = ms.forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2)
    fo, eo = oracle.mstep_forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2)
    assert np.abs(fg - fo).max() <= 1e-6 * np.abs(fo).max() + 1e-6
    assert np.allclose(eg[:, :4], eo[:, :4], rtol=1e-9, atol=1e-9)
    # the f32 MD force path of the population engine
    f32, _ = ms.forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, f32=True)
    err = np.linalg.norm(f32 - fo, axis=2)
    assert np.linalg.norm(err) <= 1e-5 * np.linalg.norm(np.linalg.norm(fo, axis=2))


def test_gpu_200kb_md_segment_tracks_oracle(ms, model200):
    atoms, poly, prm, ptr, sb, x = model200
    v = np.stack([oracle.velocity_create(atoms.flags, 50.0, 21 + s) for s in range(2)]).astype(np.float32)
    xg, vg = ms.md(prm, x, v, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, 50.0, 40.0, 1000.0, 10)
    xo, vo = oracle.mstep_md(prm, x.astype(np.float64), v.astype(np.float64), atoms.radii, atoms.flags, poly, ptr,
                             sb, 0.5, 1.2, 50.0, 40.0, 1000.0, 10)
    moved = np.abs(xo - x).max()
    assert moved > 1.0
    assert np.abs(xg - xo).max() < 1e-3 * max(1.0, moved)


@pytest.mark.parametrize('scale', [0.6, 0.4])
def test_gpu_200kb_dense_lists_forces_match_oracle(ms, model200, scale):
    """A compressed 200 kb structure: Verlet lists far longer than the list build's LDS row
    (40 entries, stored a block of quads at a time) and, at 0.4, past the list capacity
    (256: those slots take the cell walk).  f32 MD forces against the fp64 oracle."""
    from scipy.spatial import cKDTree
    atoms, poly, prm, ptr, sb, x = model200
    xc = x.copy()
    xc[:, :atoms.nbead] *= scale
    rmax = float(atoms.radii[:atoms.nbead].max())
    counts = cKDTree(xc[0, :atoms.nbead]).query_ball_point(xc[0, :atoms.nbead], 2.7 * rmax, return_length=True)
    assert counts.max() > 60  # the row is flushed
    if scale == 0.4:  # past the 256-entry list capacity (at 2.7 rmax, below any cut_list): the cell walk
        assert (counts - 1).max() > 256
    f32, _ = ms.forces(prm, xc, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, f32=True)
    fo, _ = oracle.mstep_forces(prm, xc, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2)
    err = np.linalg.norm(f32 - fo, axis=2)
    assert np.linalg.norm(err) <= 1e-5 * np.linalg.norm(np.linalg.norm(fo, axis=2))


def test_gpu_200kb_small_list_capacity_forces_match_oracle(ms, model200):
    """neigh_capacity below most list lengths: the population engine's slots past it take
    their pairs from the cell walk; forces unchanged against the fp64 oracle."""
    atoms, poly, prm, ptr, sb, x = model200
    prm16 = M.params_from_cfg({'optimization': {'optimizer_options': F.DEMO_PROTOCOL}}, [((5500.0,) * 3, 1.0)])
    prm16.neigh_capacity = 8
    f32, _ = ms.forces(prm16, x, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, f32=True)
    fo, _ = oracle.mstep_forces(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2)
    err = np.linalg.norm(f32 - fo, axis=2)
    assert np.linalg.norm(err) <= 1e-5 * np.linalg.norm(np.linalg.norm(fo, axis=2))


def _with_env(env, fn):
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_gpu_200kb_build_variants_bitwise_equal(ms, model200):
    """The population engine's list builds sort the slots by cell, ids ascending inside a
    cell.  The single-workgroup LDS sort (the default) and the split sort (IGM_POP_SORT=1:
    pop_count/scan/scatter/rank, several workgroups per flagged structure, counts in HBM)
    give the same slot order, so a protocol run is bitwise the same on both; so is the
    split sort with one structure slot in the build grids (IGM_POP_BUILD_SLOTS=1: every
    block loops over the flagged structures), with 3 structure groups, and its rerun; and so
    is the engine with the forces of the structures not rebuilt at a step running ahead of
    the list builds on a second stream (IGM_POP_EARLY=1), and the engine without bond
    pruning (IGM_POP_BOND_PRUNE=0: every bond visited at every step, the pruned ones adding
    exactly 0) or pruning at every build (IGM_POP_PRUNE_AGE=0; default: builds whose lists
    served >= 6 steps)."""
    atoms, poly, prm, ptr, sb, x = model200
    n = 6
    x6 = np.concatenate([x] * 3)
    rng = np.random.default_rng(77)
    x6[:, :atoms.nbead] += rng.normal(0, 30.0, (n, atoms.nbead, 3)).astype(np.float32)
    per = [sb[ptr[s % 2]:ptr[s % 2 + 1]] for s in range(n)]
    ptr6, sb6 = M.concat_bonds(per)
    p = json.loads(json.dumps(F.DEMO_PROTOCOL))
    p['custom_annealing_protocol']['mdsteps'] = [60, 80, 80, 60]
    p['custom_annealing_protocol']['relax']['mdsteps'] = 20
    prm6 = M.params_from_cfg({'optimization': {'optimizer_options': p}}, [((5500.0,) * 3, 1.0)])
    seeds = M.lammps_seeds(6535, list(range(n)), 3)

    def run():
        return ms.run(prm6, x6, atoms.radii, atoms.flags, poly, ptr6, sb6, seeds)
    xs, is_ = _with_env({'IGM_POP_SORT': '1'}, run)
    xl, il = run()
    x1, i1 = _with_env({'IGM_POP_SORT': '1', 'IGM_POP_BUILD_SLOTS': '1', 'IGM_POP_GROUPS': '3'}, run)
    xr, ir = _with_env({'IGM_POP_SORT': '1'}, run)
    xe, ie = _with_env({'IGM_POP_EARLY': '1'}, run)
    xp, ip = _with_env({'IGM_POP_BOND_PRUNE': '0'}, run)
    xa, ia = _with_env({'IGM_POP_PRUNE_AGE': '0'}, run)
    assert np.all(is_['nrebuild'] > 10)  # many list builds
    runs = {'lds sort': (xl, il), 'split sort, 1 build slot, 3 groups': (x1, i1), 'split sort rerun': (xr, ir),
            'early forces': (xe, ie), 'no bond pruning': (xp, ip), 'pruning at every build': (xa, ia)}
    bad = [k for k, (xo, io) in runs.items() if not (np.array_equal(xs, xo) and is_.tobytes() == io.tobytes())]
    assert not bad, bad


@pytest.mark.parametrize('engine', ['lds', 'hbm'])
def test_gpu_retired_engine_flag_is_rejected(demo, ms, engine):
    """params flag 0x4 (round 3's domain-decomposed engine) is retired: igm_mstep_run returns
    IGM_E_UNSUPPORTED on the LDS engine as on the population engine (include/igm_hip.h)."""
    atoms, poly, prm, ptr, sb, x = _demo_inputs(demo, [0, 1])
    if engine == 'hbm':
        _global(prm)
    prm.flags |= 0x4
    seeds = M.lammps_seeds(6535, [0, 1], 3)
    with pytest.raises(RuntimeError, match=r'code %d\).*retired' % _lib.IGM_E_UNSUPPORTED):
        ms.run(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
