"""Configurations D and E at their workload size: 200 kb hg38 male
diploid (29 838 beads) with the restraints of ModelingStep.task assembled by
igm_amd.assemble -- the same code the Step layer runs (test helper).

  D  ellipsoid nucleus (7840, 6470, 2450), r = 118.5 nm; lamina DamID: the A-step
     (igm_damid_actdist, ellipsoid) on the batch's own population at sigma 0.45 of
     the synthetic Beta(2, 5) profile, then Damid._apply_envelope's per-structure
     membership (igm_damid_select) and the k < 0 envelope on the shrunk ellipsoid.
  E  sphere nucleus as an imaged map (VolumeFile, 100 nm EDT sphere, GenEnvelope /
     fix volumetricrestraint); SPRITE: the A-step (Rg^2 keep_best + Gibbs assignment)
     over synthetic clusters, centroid slots and bead->centroid bounds; FISH: the
     A-step's rank-matched radial and pair targets, lower/upper bounds to the centre
     and between copies.
Both carry frustrated Hi-C-like contacts (tests/mstep_stats.random_contacts, as rows
whose activation distance admits every structure), so the final energies balance
every term and respond to each of them.
"""
import json
import types

import numpy as np

from igm_amd import synthetic as syn
from igm_amd.workloads import (DAMID_CR, DAMID_SIGMA, hic_rows, population, spec_D, spec_E,  # noqa: F401
                               scaled_protocol)


def index_of(pop):
    return types.SimpleNamespace(radii=pop['radii'], chrom=pop['chrom'], copy=pop['copy'],
                                 copy_ptr=pop['copy_ptr'], copy_idx=pop['copy_idx'])


def protocol(scale):
    return scaled_protocol(syn.DEMO_PROTOCOL, scale)


def run_stats(batch, info, x, stats):
    """per-structure summary: energies per bead, every envelope's energy, the violation
    fraction over all monitored classes (violation records), final Temp."""
    nb = batch.nbead
    out = {'pair': info['pair_energy'] / nb, 'bond': info['bond_energy'] / nb, 'total': info['final_energy'] / nb,
           'temp': info['temp'].astype(np.float64), 'rebuilds': info['nrebuild'].astype(np.float64)}
    for e in range(batch.prm.nenvelopes):
        out['env%d' % e] = info['env_energy'][:, e] / nb
    nv = stats[:, :, 102].sum(1).astype(np.float64)
    ni = stats[:, :, 103].sum(1).astype(np.float64)
    out['viol_frac'] = nv / np.maximum(ni, 1)
    return out


def dumps(spec):
    return json.dumps({k: v for k, v in spec.items() if k == 'protocol'})
