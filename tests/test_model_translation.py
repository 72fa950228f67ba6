"""CPU: model.from_igm_model (LammpsModel.from_model semantics, lammps_model.py:244-312)
on a reference-shaped igm Model built from the demo structure and the reference's
own restraint selection; the bond list must equal the reference LammpsModel's."""
import numpy as np
import pytest

import mstep_fixtures as F
from igm_amd import model as M
from igm_amd._lib import IGM_ATOM_BEAD, IGM_ATOM_ENV0, IGM_ATOM_FIXED, LOWER_BOUND_BIT


class P(object):  # igm.model.particle.Particle (particle.py:16-20)
    def __init__(self, pos, r, t):
        self.pos = np.array(pos).astype(np.float32)
        self.r = np.float32(r)
        self.ptype = t


class Bound(object):  # HarmonicUpperBound / HarmonicLowerBound (forces.py:93-140)
    def __init__(self, i, j, d, k, lower=False):
        self.ftype = 2 if lower else 1
        self.i, self.j, self.d, self.k = i, j, d, k


class Env(object):  # EllipticEnvelope (forces.py:189-205)
    ftype = 3
    shape = 'ellipsoid'

    def __init__(self, ids, semiaxes, k):
        self.particle_ids, self.semiaxes, self.k = ids, semiaxes, k


class EV(object):  # ExcludedVolume (forces.py:44-55)
    ftype = 0

    def __init__(self, k):
        self.k = k


class Model(object):
    def __init__(self, uid):
        self.id = uid
        self.particles, self.forces = [], []


def demo_igm_model(pop, g3, sid):
    """ModelingStep.task's restraint order (ModelingStep.py:216-397): Steric, Polymer,
    Envelope (adds the centre dummy), inter Hi-C, intra Hi-C."""
    m = Model(sid)
    crd = pop['coordinates'][:, sid, :]
    for i in range(len(pop['radii'])):
        m.particles.append(P(crd[i], pop['radii'][i], 0))
    m.forces.append(EV(1.0))
    for b in M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0):
        m.forces.append(Bound(int(b['i']), int(b['j']), float(b['r0']), float(b['k'])))
    m.particles.append(P([0, 0, 0], 0, 1))
    m.forces.append(Env(list(range(len(pop['radii']))), np.array([5500.0] * 3), 1.0))
    hic, _ = F.hic_bonds_from_golden(g3, pop['radii'], sid)
    for b in hic:
        m.forces.append(Bound(int(b['i']), int(b['j']), float(b['r0']), float(b['k'])))
    return m


@pytest.mark.parametrize('sid', [0, 1])
def test_from_igm_model_equals_reference_lammps_model(sid):
    pop, g3 = F.load()
    lm = M.from_igm_model(demo_igm_model(pop, g3, sid))
    nb = len(pop['radii'])
    assert lm.id == sid and len(lm.radii) == nb + 1
    assert np.all(lm.flags[:nb] == (IGM_ATOM_BEAD | IGM_ATOM_ENV0)) and lm.flags[nb] == IGM_ATOM_FIXED
    assert lm.envelopes == [((5500.0,) * 3, 1.0)] and lm.evfactor == 1.0
    ref = F.golden_bonds(g3, sid)
    assert np.array_equal(lm.bonds['i'], ref['i']) and np.array_equal(lm.bonds['j'], ref['j'])
    assert np.array_equal(lm.bonds['r0'], ref['r0'].astype(np.float32))
    assert np.array_equal(lm.bonds['k'], ref['k'].astype(np.float32))
    assert np.array_equal(lm.xyz[:nb], pop['coordinates'][:, sid, :])


def test_from_igm_model_dummies_and_lower_bounds():
    m = Model(3)
    for q in range(4):
        m.particles.append(P([q, 0, 0], 10.0, 0))
    m.particles.append(P([0, 0, 0], 0, 1))   # static dummy
    m.particles.append(P([0, 0, 0], 0, 1))   # same position, consecutive: merged (get_next_dummy)
    m.particles.append(P([1, 2, 3], 0, 2))   # dynamic centroid
    m.particles.append(P([0, 0, 0], 0, 1))   # not consecutive to a dummy: a new atom
    m.forces += [Bound(0, 5, 100.0, 2.0, lower=True), Bound(1, 4, 50.0, 1.0), Bound(6, 7, 5.0, 1.0),
                 Env([], np.array([1.0, 1.0, 1.0]), 1.0), Env([0, 1], np.array([9.0, 8.0, 7.0]), -1.0), EV(0.5)]
    lm = M.from_igm_model(m)
    assert list(lm.imap) == [0, 1, 2, 3, 4, 4, 5, 6]
    assert list(lm.flags) == [IGM_ATOM_BEAD | IGM_ATOM_ENV0] * 2 + [IGM_ATOM_BEAD] * 2 + [IGM_ATOM_FIXED, 0,
                                                                                          IGM_ATOM_FIXED]
    assert list(lm.bonds['i']) == [0, 1, 5]
    assert list(lm.bonds['j']) == [4 | int(LOWER_BOUND_BIT), 4, 6]
    assert lm.envelopes == [((9.0, 8.0, 7.0), -1.0)]  # the empty envelope gets no group (lammps.py:231-233)
    assert lm.evfactor == 0.5


@pytest.mark.gpu
def test_kernel_hip_optimize_contract():
    """kernel_hip.optimize keeps lammps.optimize's contract (lammps.py:361-492): the
    particles move in place, the info dict carries the parsed LAMMPS fields."""
    from igm_amd import kernel_hip
    from test_mstep_gpu import short_protocol
    pop, g3 = F.load()
    m = demo_igm_model(pop, g3, 1)
    before = np.stack([p.pos for p in m.particles])
    info = kernel_hip.optimize(m, {'optimization': {'optimizer_options': short_protocol((200, 200, 200, 200), 50)}})
    after = np.stack([p.pos for p in m.particles])
    assert after.dtype == np.float32 and np.all(np.isfinite(after))
    assert np.abs(after[:-1] - before[:-1]).max() > 1.0
    assert np.array_equal(after[-1], before[-1])  # the frozen centre dummy
    assert set(info) == {'final-energy', 'pair-energy', 'bond-energy', 'md-time', 'thermo'}
    assert set(info['thermo']) == {'Temp', 'E_pair', 'E_bond', 'f_envelope0'}
    assert np.isfinite(info['final-energy']) and info['final-energy'] >= 0
