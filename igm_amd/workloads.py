"""Synthetic restraint specs of configurations D and E (BASELINE.json configs[3],
configs[4]) for igm_amd.assemble.build -- what ModelingStep.task
(igm/steps/ModelingStep.py:200-503) assembles for one structure, built for a batch, on
the synthetic 200 kb population (igm_amd.synthetic: no network, no real data).  The
bench times these workloads and tests/de200.py checks them against the oracle.

  D  ellipsoid nucleus (7840, 6470, 2450), r = 118.5 nm; lamina DamID: the A-step
     (igm_damid_actdist, ellipsoid) on the batch's own population at sigma 0.45 of
     the synthetic Beta(2, 5) profile, then Damid._apply_envelope's per-structure
     membership (igm_damid_select) and the k < 0 envelope on the shrunk ellipsoid
     (ModelingStep.py:402-440).
  E  sphere nucleus as an imaged map (VolumeFile, 100 nm EDT sphere, GenEnvelope /
     fix volumetricrestraint); SPRITE: the A-step (Rg^2 keep_best + Gibbs assignment)
     over synthetic clusters, centroid slots and bead->centroid bounds
     (ModelingStep.py:456-480); FISH: the A-step's rank-matched radial and pair
     targets, lower/upper bounds to the centre and between copies (:482-503).
The parity tests give both frustrated Hi-C-like contacts (random_contacts, as actdist rows
whose activation distance admits every structure), so the final energies balance every
term and respond to each of them; the bench gives them the Hi-C A-step's rows
(hic_actdist_rows), the satisfiable restraint set of igm-run's loop.
"""
import json

import numpy as np

from . import model as M
from . import synthetic as syn
from ._lib import bond_dtype, row_dtype

DAMID_SIGMA = 0.45
DAMID_CR = 0.05


def scaled_protocol(protocol, scale):
    """The protocol with every MD step count scaled (all stages, relax and CG kept)."""
    p = json.loads(json.dumps(protocol))
    cap = p['custom_annealing_protocol']
    cap['mdsteps'] = [max(1, int(round(n * scale))) for n in cap['mdsteps']]
    cap['relax']['mdsteps'] = max(1, int(round(cap['relax']['mdsteps'] * scale)))
    return p


def random_contacts(radii, nbead, nlocal, nlong, seed, cr=2.0, k=1.0):
    """Hi-C-like bonds (harmonic upper bound, r0 = cr (r_i + r_j)): nlocal pairs at
    genomic separations 2..60 beads, nlong between random beads."""
    rng = np.random.default_rng(seed)
    i1 = rng.integers(0, nbead - 61, nlocal)
    j1 = i1 + rng.integers(2, 61, nlocal)
    i2 = rng.integers(0, nbead, nlong)
    j2 = rng.integers(0, nbead, nlong)
    i = np.concatenate([i1, i2])
    j = np.concatenate([j1, j2])
    keep = i != j
    b = np.zeros(int(keep.sum()), bond_dtype)
    b['i'], b['j'] = i[keep], j[keep]
    b['r0'] = M.r0_contact(cr, radii[b['i']], radii[b['j']]).astype(np.float32)
    b['k'] = k
    return b


def hic_rows(radii, nbead, nlocal, nlong, seed):
    """random_contacts as actdist rows that every structure selects (dist >= any d)."""
    b = random_contacts(radii, nbead, nlocal, nlong, seed)
    rows = np.zeros(len(b), row_dtype)
    rows['row'], rows['col'] = b['i'], b['j'] & 0x7fffffff
    rows['dist'] = np.float32(1e9)
    rows['prob'] = np.float32(1.0)
    return rows


def population(config, n, first_sid):
    """the synthetic 200 kb population of configuration D (ellipsoid nucleus) or E"""
    if config == 'D':
        return syn.population_200kb(n, first_sid=first_sid, semiaxes=syn.ELLIPSOID_D)
    return syn.population_200kb(n, first_sid=first_sid)


def hic_actdist_rows(pop, sigma=0.01, contact_range=2.0):
    """the Hi-C A-step (get_actdist over the synthetic 200 kb .hcs at `sigma`, it_corr 1) on
    this population: the activated rows ModelingStep's Hi-C restraints select from (a
    satisfiable restraint set, as in igm-run's loop, where the frustrated random_contacts
    are the parity tests' choice)"""
    from . import astep
    from ._lib import pair_dtype
    i, j, p = syn.hic_pairs_200kb(sigma)
    pairs = np.zeros(len(i), pair_dtype)
    pairs['i'], pairs['j'], pairs['pwish'] = i, j, p
    xyz_bm = np.ascontiguousarray(pop['xyz'].transpose(1, 0, 2))
    return astep.compute_actdist(xyz_bm, pop['radii'], pop['copy_ptr'], pop['copy_idx'], pop['chrom'], pairs,
                                 contact_range, 1)


def spec_D(pop, n, scale, ctx, nlocal=15000, nlong=1500, seed=41, hic=None):
    from . import assemble as A
    from . import damid
    xyz_bm = np.ascontiguousarray(pop['xyz'].transpose(1, 0, 2))
    loci, pe, pl = damid.select_loci(syn.damid_profile_200kb(), DAMID_SIGMA)
    drows = damid.compute_damid_actdist(xyz_bm, pop['radii'], pop['copy_ptr'], pop['copy_idx'], loci, pe, pl, 1,
                                        DAMID_CR, 'ellipsoid', syn.ELLIPSOID_D, ctx=ctx)
    nb = len(pop['radii'])
    return {'evfactor': 1.0, 'protocol': scaled_protocol(syn.DEMO_PROTOCOL, scale),
            'polymer': {'contact_range': 2.0, 'kspring': 1.0},
            'envelope': A.envelope_spec('ellipsoid', semiaxes=syn.ELLIPSOID_D, k=1.0),
            'hic': {'rows': hic_rows(pop['radii'], nb, nlocal, nlong, seed) if hic is None else hic,
                    'contact_range': 2.0, 'k': 1.0},
            'damid': {'rows': drows, 'contact_range': DAMID_CR, 'k': 1.0}}


def spec_E(pop, n, scale, ctx, vol, nclusters=2000, keep_best=4, nprobe=50, npair=50, nlocal=15000, nlong=1500,
           seed=43, hic=None):
    from . import fish, sprite
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
    return {'evfactor': 1.0, 'protocol': scaled_protocol(syn.DEMO_PROTOCOL, scale),
            'polymer': {'contact_range': 2.0, 'kspring': 1.0},
            'envelope': {'shape': 'exp_map', 'k': 1.0, 'volumes': [vol], 'struct_map': None,
                         'files': ['nucleus_sphere.bin']},
            'hic': {'rows': hic_rows(pop['radii'], nb, nlocal, nlong, seed) if hic is None else hic,
                    'contact_range': 2.0, 'k': 1.0},
            'sprite': {'assignment': assignment, 'indptr': indptr, 'selected': selected, 'volume_fraction': 0.2,
                       'k': 1.0},
            'fish': {'data': fd, 'rtype': 'rRpP', 'tol': 50.0, 'k': 1.0}}
