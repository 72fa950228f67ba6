"""Population initialisation: RandomInit territories (CPU, against
a literal restatement of RandomInit.generate_territories) and RelaxInit on the batched
engine (GPU: identical to the per-structure 'hip' kernel on the reference-shaped model)."""
import json
import math

import numpy as np
import pytest

import mstep_fixtures as F
from igm_amd import init as I


def territories_loop(chrom_sizes, R, rs):
    """RandomInit.generate_territories / uniform_sphere (RandomInit.py:182-240), point by point."""
    def uniform_sphere(R):
        phi = rs.uniform(0, 2 * math.pi)
        costheta = rs.uniform(-1, 1)
        u = rs.uniform(0, 1)
        theta = math.acos(costheta)
        r = R * (u ** (1. / 3.))
        return np.array([r * math.sin(theta) * math.cos(phi), r * math.sin(theta) * math.sin(phi),
                         r * math.cos(theta)])
    n_tot = int(sum(chrom_sizes))
    chr_radii = [0.75 * R * (float(nb) / n_tot) ** (1. / 3) for nb in chrom_sizes]
    crad = np.average(chr_radii)
    crds = np.empty((n_tot, 3))
    k = 0
    for nb in chrom_sizes:
        center = uniform_sphere(R - crad)
        for _ in range(nb):
            crds[k] = uniform_sphere(crad) + center
            k += 1
    return crds


def test_generate_territories_matches_reference_draws():
    pop, _ = F.load()
    cs = pop['chrom_sizes']
    a = I.generate_territories(cs, 5000.0, np.random.RandomState(17))
    b = territories_loop(cs, 5000.0, np.random.RandomState(17))
    assert a.shape == b.shape
    assert np.allclose(a, b, rtol=0, atol=1e-9 * 5000.0)  # same draws; numpy vs libm trig differ by ulps
    assert np.linalg.norm(a, axis=1).max() <= 5000.0 + 1e-6


@pytest.mark.gpu
def test_relax_population_equals_per_structure_kernel():
    """RelaxInit batched (one igm_mstep_run) == kernel_hip.optimize on each structure's
    reference-shaped Model (Steric, Polymer, Envelope in RelaxInit's order), bitwise."""
    from igm_amd import kernel_hip
    from test_model_translation import Model, P, Bound, Env, EV
    from test_mstep_gpu import short_protocol
    from igm_amd import model as M
    pop, _ = F.load()
    sids = [3, 4, 5]
    prot = short_protocol((150, 150, 150, 150), 40)
    cfg = {'model': {'restraints': {'excluded': {'evfactor': 1.0},
                                    'polymer': {'contact_range': 2.0, 'polymer_kspring': 1.0},
                                    'envelope': {'nucleus_shape': 'sphere', 'nucleus_radius': 5500.0,
                                                 'nucleus_kspring': 1.0}}},
           'optimization': {'optimizer_options': prot}, 'runtime': {'step_no': 0}}
    xyz = pop['coordinates'][:, sids, :].transpose(1, 0, 2)
    xr, info = I.relax_population(cfg, xyz, pop['radii'], pop['chrom'], pop['copy'], sids)
    assert np.all(np.isfinite(xr)) and np.all(info['final_energy'] < info['einitial'])
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    for q, sid in enumerate(sids):
        m = Model(sid)
        for i in range(len(pop['radii'])):
            m.particles.append(P(xyz[q, i], pop['radii'][i], 0))
        m.forces.append(EV(1.0))
        for b in poly:
            m.forces.append(Bound(int(b['i']), int(b['j']), float(b['r0']), float(b['k'])))
        m.particles.append(P([0, 0, 0], 0, 1))
        m.forces.append(Env(list(range(len(pop['radii']))), np.array([5500.0] * 3), 1.0))
        out = kernel_hip.optimize(m, cfg)
        got = np.stack([p.pos for p in m.particles[:-1]])
        assert np.array_equal(got, xr[q]), sid
        assert out['final-energy'] == info['final_energy'][q]
