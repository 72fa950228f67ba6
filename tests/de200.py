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

import mstep_stats as MS
from igm_amd import model as M
from igm_amd import synthetic as syn
from igm_amd._lib import row_dtype

DAMID_SIGMA = 0.45
DAMID_CR = 0.05


def index_of(pop):
    return types.SimpleNamespace(radii=pop['radii'], chrom=pop['chrom'], copy=pop['copy'],
                                 copy_ptr=pop['copy_ptr'], copy_idx=pop['copy_idx'])


def hic_rows(radii, nbead, nlocal, nlong, seed):
    """random_contacts as actdist rows that every structure selects (dist >= any d)."""
    b = MS.random_contacts(radii, nbead, nlocal, nlong, seed)
    rows = np.zeros(len(b), row_dtype)
    rows['row'], rows['col'] = b['i'], b['j'] & 0x7fffffff
    rows['dist'] = np.float32(1e9)
    rows['prob'] = np.float32(1.0)
    return rows


def protocol(scale):
    return MS.scaled_protocol(syn.DEMO_PROTOCOL, scale)


def spec_D(pop, n, scale, ctx, nlocal=15000, nlong=1500, seed=41):
    from igm_amd import assemble as A
    from igm_amd import damid
    xyz_bm = np.ascontiguousarray(pop['xyz'].transpose(1, 0, 2))
    loci, pe, pl = damid.select_loci(syn.damid_profile_200kb(), DAMID_SIGMA)
    drows = damid.compute_damid_actdist(xyz_bm, pop['radii'], pop['copy_ptr'], pop['copy_idx'], loci, pe, pl, 1,
                                        DAMID_CR, 'ellipsoid', syn.ELLIPSOID_D, ctx=ctx)
    nb = len(pop['radii'])
    return {'evfactor': 1.0, 'protocol': protocol(scale),
            'polymer': {'contact_range': 2.0, 'kspring': 1.0},
            'envelope': A.envelope_spec('ellipsoid', semiaxes=syn.ELLIPSOID_D, k=1.0),
            'hic': {'rows': hic_rows(pop['radii'], nb, nlocal, nlong, seed), 'contact_range': 2.0, 'k': 1.0},
            'damid': {'rows': drows, 'contact_range': DAMID_CR, 'k': 1.0}}


def spec_E(pop, n, scale, ctx, vol, nclusters=2000, keep_best=4, nprobe=50, npair=50, nlocal=15000, nlong=1500,
           seed=43):
    from igm_amd import fish, sprite
    xyz_bm = np.ascontiguousarray(pop['xyz'].transpose(1, 0, 2))
    cp, ci = pop['copy_ptr'], pop['copy_idx']
    # SPRITE A-step: keep_best by Rg^2 on the GPU, Gibbs assignment on the host
    ptr, data = syn.sprite_clusters_200kb(nclusters, seed=2)
    cl = [data[ptr[c]:ptr[c + 1]] for c in range(len(ptr) - 1)]
    idx, val, sel = sprite.task(xyz_bm, cl, pop['hap_chrom'], cp, ci, keep_best=keep_best, ctx=ctx,
                                rng=np.random.RandomState(5))
    assignment, chosen = sprite.assign(val, idx, sel, n, kT=50.0, rng=np.random.RandomState(6))
    indptr = np.concatenate([[0], np.cumsum([len(c) for c in chosen])]).astype(np.int64)
    selected = np.concatenate(chosen).astype(np.int32)
    # FISH A-step: rank-matched targets
    f = syn.fish_inputs_200kb(n, nprobe=nprobe, npair=npair)
    fr = fish.task(xyz_bm, cp, ci, f, ctx=ctx)
    fd = {'probes': f['probes'], 'pairs': f['pairs']}
    for key in ('radial_min', 'radial_max', 'pair_min', 'pair_max'):
        fd[key] = np.stack([v for _, v in sorted(fr[key], key=lambda t: t[0])])
    nb = len(pop['radii'])
    return {'evfactor': 1.0, 'protocol': protocol(scale),
            'polymer': {'contact_range': 2.0, 'kspring': 1.0},
            'envelope': {'shape': 'exp_map', 'k': 1.0, 'volumes': [vol], 'struct_map': None,
                         'files': ['nucleus_sphere.bin']},
            'hic': {'rows': hic_rows(pop['radii'], nb, nlocal, nlong, seed), 'contact_range': 2.0, 'k': 1.0},
            'sprite': {'assignment': assignment, 'indptr': indptr, 'selected': selected, 'volume_fraction': 0.2,
                       'k': 1.0},
            'fish': {'data': fd, 'rtype': 'rRpP', 'tol': 50.0, 'k': 1.0}}


def population(config, n, first_sid):
    if config == 'D':
        return syn.population_200kb(n, first_sid=first_sid, semiaxes=syn.ELLIPSOID_D)
    pop = syn.population_200kb(n, first_sid=first_sid)
    return pop


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
