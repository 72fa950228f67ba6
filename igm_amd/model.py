"""Vectorised M-step model assembly (replaces the per-structure Python object
model of the reference for the hot path).

The reference builds, per structure, a `Model` of `Particle` objects and
`Force` objects (igm/model/model.py:9-159, particle.py, forces.py) from the
`Restraint` plugins (restraints/*.py) and converts it to a LammpsModel
(model/kernel/lammps_model.py:244-301).  Here the same quantities are produced
as flat arrays shared by the whole population:

  atoms      beads (NORMAL particles) then the static envelope centre
             (Envelope._apply_sphere_envelop adds a DUMMY_STATIC at the origin,
             restraints/envelope.py:36-62; LAMMPS freezes it with setforce 0)
  bonds      polymer bonds (restraints/polymer.py:31-58) shared by all
             structures; Hi-C bonds per structure (igm_hic_select on the GPU)
  envelopes  fix ellipsoidalenvelope a b c k (lammps.py:292-303)
  seeds      create_lammps_script's seed formula (lammps.py:159-165)
"""
import numpy as np

from ._lib import (IGM_ATOM_BEAD, IGM_ATOM_ENV0, IGM_ATOM_FIXED, IGM_ENV_VOLUME, IGM_MAX_ENVELOPES, IGM_MAX_STAGES,
                   LOWER_BOUND_BIT, MStepParams, bond_dtype)

# restraint classes used for violation statistics (ModelingStep.py:511-557)
CLASS_POLYMER = 0
CLASS_INTER_HIC = 1
CLASS_INTRA_HIC = 2
NCLASS_BONDS = 3


def r0_contact(cr, ri, rj):
    """dij = contactRange * (r_i + r_j): the radii are np.float32 so their sum is
    f32, the product with the Python float is f64 (NumPy 1.x), restraints/*.py."""
    s = (np.asarray(ri, np.float32) + np.asarray(rj, np.float32)).astype(np.float32)
    return float(cr) * s.astype(np.float64)


def polymer_bonds(chrom, copy, radii, contact_range=2.0, k=1.0, contact_probabilities=None):
    """Polymer._apply (restraints/polymer.py:159-183): bond (i, i+1) when both are in
    the same chromosome AND copy; r0 = cr*(ri+rj) or the cube-root formula when
    consecutive contact probabilities are given."""
    chrom = np.asarray(chrom)
    copy = np.asarray(copy)
    radii = np.asarray(radii, np.float32)
    n = len(chrom)
    i = np.arange(n - 1)
    m = (chrom[:-1] == chrom[1:]) & (copy[:-1] == copy[1:])
    i = i[m]
    if contact_probabilities is None:
        r0 = r0_contact(contact_range, radii[i], radii[i + 1])
    else:
        cp = np.asarray(contact_probabilities, np.float64)
        d0 = (radii[i] + radii[i + 1]).astype(np.float32).astype(np.float64)
        d1 = contact_range * d0
        f = cp[i].copy()
        f[(f < 0.5) | (f > 1)] = 0.5  # MIN_CONSECUTIVE (polymer.py:35,176-177)
        x3 = (d1 ** 3 + (f - 1) * d0 ** 3) / f
        r0 = x3 ** (1.0 / 3)
    b = np.zeros(len(i), bond_dtype)
    b['i'] = i
    b['j'] = i + 1
    b['r0'] = r0.astype(np.float32)
    b['k'] = np.float32(k)
    return b


def lammps_seeds(seed, struct_ids, step_no):
    """((seed * model.id * step_no) % 9190037) + 1 with step_no = runtime step_no + 2
    (lammps.py:159-165, :435)."""
    sid = np.asarray(struct_ids, np.int64)
    return (((int(seed) * sid * (int(step_no) + 2)) % 9190037) + 1).astype(np.int32)


class Atoms(object):
    """Per-atom arrays shared by all structures of a batch."""

    def __init__(self, radii, envelope_members=None, n_static_dummies=1):
        radii = np.asarray(radii, np.float32)
        self.nbead = len(radii)
        self.n = self.nbead + n_static_dummies
        self.radii = np.zeros(self.n, np.float32)
        self.radii[:self.nbead] = radii
        self.flags = np.zeros(self.n, np.uint32)
        self.flags[:self.nbead] = IGM_ATOM_BEAD
        self.flags[self.nbead:] = IGM_ATOM_FIXED
        if envelope_members is None:
            envelope_members = [np.arange(self.nbead)]
        for e, mem in enumerate(envelope_members):
            self.flags[np.asarray(mem, np.int64)] |= np.uint32(IGM_ATOM_ENV0 << e)


def params_from_cfg(cfg, envelopes, evfactor=1.0, skin=None):
    """MStepParams from the reference config sections
    optimization/optimizer_options (+ custom_annealing_protocol) and
    model/restraints (lammps.py:149-358 reads the same keys)."""
    opt = cfg['optimization']['optimizer_options'] if 'optimization' in cfg else cfg
    p = MStepParams()
    prot = opt.get('custom_annealing_protocol', None)
    if prot is None:
        prot = {'num_steps': 1, 'mdsteps': [opt['mdsteps']], 'tstarts': [opt['tstart']],
                'tstops': [opt['tstop']], 'evfactors': [1], 'envelope_factors': [1]}
    ns = int(prot.get('num_steps'))
    if ns > IGM_MAX_STAGES:
        raise ValueError('at most %d annealing stages' % IGM_MAX_STAGES)
    mdsteps = prot.get('mdsteps', [opt['mdsteps']] * ns)
    tstarts = prot.get('tstarts', [opt['tstart']] * ns)
    tstops = prot.get('tstops', tstarts)
    evfs = prot.get('evfactors', [1] * ns)
    envfs = prot.get('envelope_factors', [1] * ns)
    assert len(mdsteps) == len(tstarts) == len(tstops) == len(evfs) == len(envfs) == ns
    p.nstages = ns
    for k in range(ns):
        p.mdsteps[k] = int(mdsteps[k])
        p.tstart[k] = float(tstarts[k])
        p.tstop[k] = float(tstops[k])
        p.evfactor[k] = float(evfs[k])
        p.envfactor[k] = float(envfs[k])
    relax = prot.get('relax', None)
    if relax is not None:
        p.relax_steps = int(relax['mdsteps'])
        p.relax_temperature = float(relax['temperature'])
        p.relax_max_velocity = float(relax['max_velocity'])
    p.timestep = float(opt.get('timestep', 0.25))
    p.max_velocity = float(opt.get('max_velocity', 1000.0))
    p.t_window = 0.1
    p.t_fraction = 1.0
    p.etol = float(opt.get('etol', 1e-4))
    p.ftol = float(opt.get('ftol', 1e-6))
    p.max_cg_iter = int(opt.get('max_cg_iter', 500))
    p.max_cg_eval = int(opt.get('max_cg_eval', 500))
    p.dmax = 0.1
    p.evfactor_base = float(evfactor)
    p.skin = float(skin) if skin is not None else 0.0
    if len(envelopes) > IGM_MAX_ENVELOPES:
        raise ValueError('at most %d envelopes' % IGM_MAX_ENVELOPES)
    p.nenvelopes = len(envelopes)
    for e, (abc, k) in enumerate(envelopes):
        if isinstance(abc, str):  # ('volume', k): fix volumetricrestraint (lammps.py:305-310)
            if abc != 'volume':
                raise ValueError('unknown envelope kind %r' % abc)
            p.env_kind[e] = IGM_ENV_VOLUME
        else:
            for d in range(3):
                p.env_semiaxes[e][d] = float(abc[d])
        p.env_k[e] = float(k)
    p.neigh_capacity = 0
    return p


def lower_bound(b):
    """mark bonds as harmonic_lower_bound (bit 31 of j)."""
    b = b.copy()
    b['j'] |= LOWER_BOUND_BIT
    return b


def concat_bonds(per_struct):
    """list of bond arrays (one per structure) -> CSR (ptr, bonds)."""
    ptr = np.zeros(len(per_struct) + 1, np.int64)
    ptr[1:] = np.cumsum([len(b) for b in per_struct])
    bonds = np.concatenate(per_struct) if len(per_struct) else np.zeros(0, bond_dtype)
    return ptr, np.ascontiguousarray(bonds, bond_dtype)


# ---- LammpsModel.from_model for a reference igm Model object --------------------
class LammpsLikeModel(object):
    """The arrays LammpsModel.from_model (igm/model/kernel/lammps_model.py:244-301)
    derives from an igm Model: atoms (radii, flags, xyz), bonds, envelopes, evfactor,
    and imap (particle index -> atom index)."""

    def __init__(self, radii, flags, xyz, bonds, envelopes, evfactor, imap, uid):
        self.radii, self.flags, self.xyz, self.bonds = radii, flags, xyz, bonds
        self.envelopes, self.evfactor, self.imap, self.id = envelopes, evfactor, imap, uid


# Force.ftype codes (igm/model/forces.py:14-18) and Particle.ptype codes (particle.py:11-13)
_EXCLUDED_VOLUME, _UPPER, _LOWER, _ENVELOPE, _GENERAL_ENVELOPE = 0, 1, 2, 3, 4
_NORMAL, _DUMMY_STATIC, _DUMMY_DYNAMIC = 0, 1, 2
_DUMMY_MAX_BONDS = 20  # FrozenPhantomBead.MAX_BONDS (lammps_model.py:177)


def from_igm_model(model):
    """LammpsModel.from_model semantics on a reference `igm.model.Model` (duck typed:
    .id, .particles[.pos, .r, .ptype], .forces[.ftype, .i, .j, .d, .k | .particle_ids,
    .semiaxes, .shape]):
      NORMAL -> bead atom; DUMMY_STATIC -> frozen dummy, merged into the previous atom
      when that is a dummy at the same position (get_next_dummy, :303-312);
      DUMMY_DYNAMIC -> mobile centroid without pair interactions;
      HARMONIC_UPPER/LOWER_BOUND -> bonds in force order; EXCLUDED_VOLUME -> evfactor;
      ENVELOPE -> envelope (only those with particles get a LAMMPS group, lammps.py:231-233).
    ExpEnvelope (exp_map) -> ('volume', k) envelope; its map file in lm.volume_files."""
    radii, flags, xyz, imap = [], [], [], []
    for p in model.particles:
        pos = np.asarray(p.pos, np.float32)
        if p.ptype == _NORMAL:
            radii.append(np.float32(p.r))
            flags.append(IGM_ATOM_BEAD)
            xyz.append(pos)
        elif p.ptype == _DUMMY_STATIC:
            if flags and flags[-1] == IGM_ATOM_FIXED and np.all(xyz[-1] == pos):
                imap.append(len(flags) - 1)
                continue
            radii.append(np.float32(0.0))
            flags.append(IGM_ATOM_FIXED)
            xyz.append(pos)
        elif p.ptype == _DUMMY_DYNAMIC:
            radii.append(np.float32(0.0))
            flags.append(0)
            xyz.append(pos)
        else:
            raise ValueError('Unknown particle type')
        imap.append(len(flags) - 1)
    flags = np.asarray(flags, np.uint32)
    imap = np.asarray(imap, np.int64)
    bi, bj, br, bk, lower, envelopes, evfactor = [], [], [], [], [], [], 1.0
    volume_files = []
    for f in model.forces:
        if f.ftype in (_ENVELOPE, _GENERAL_ENVELOPE):
            shape = getattr(f, 'shape', 'ellipsoid')
            if shape not in ('ellipsoid', 'exp_map'):
                raise NotImplementedError('Envelope (%s) not implemented' % shape)  # lammps.py:313-315
            if len(f.particle_ids):
                e = len(envelopes)
                if e >= IGM_MAX_ENVELOPES:
                    raise ValueError('at most %d envelopes' % IGM_MAX_ENVELOPES)
                flags[imap[np.asarray(f.particle_ids, np.int64)]] |= np.uint32(IGM_ATOM_ENV0 << e)
                if shape == 'exp_map':  # ExpEnvelope -> fix volumetricrestraint (lammps.py:305-310)
                    envelopes.append(('volume', float(f.k)))
                    volume_files.append(f.volume_file)
                else:
                    envelopes.append((tuple(float(v) for v in f.semiaxes), float(f.k)))
        elif f.ftype == _EXCLUDED_VOLUME:
            evfactor = float(f.k)
        elif f.ftype in (_UPPER, _LOWER):
            bi.append(imap[f.i])
            bj.append(imap[f.j])
            br.append(f.d)
            bk.append(f.k)
            lower.append(f.ftype == _LOWER)
        else:
            raise ValueError('Unknown force type %r' % f.ftype)
    bonds = np.zeros(len(bi), bond_dtype)
    if len(bi):
        bonds['i'] = bi
        bonds['j'] = np.asarray(bj, np.uint32) | np.where(lower, LOWER_BOUND_BIT, np.uint32(0)).astype(np.uint32)
        bonds['r0'] = br
        bonds['k'] = bk
    lm = LammpsLikeModel(np.asarray(radii, np.float32), flags, np.stack(xyz).astype(np.float32), bonds,
                         envelopes, evfactor, imap, getattr(model, 'id', 0))
    lm.volume_files = volume_files
    return lm
