"""ModelingStep.task's restraint assembly for a BATCH of structures (SURVEY 8(a) M1-M3,
configurations A-E): everything ModelingStep.task (igm/steps/ModelingStep.py:200-503)
adds to one structure's Model before model.optimize, built once for many structures
as the flat arrays the batched engine consumes.

  restraint (reference, order of ModelingStep.task)   here
  Steric            steric.py:23-31                     evfactor (params)
  Polymer           polymer.py:31-58 (:221-233)         shared bonds, class POLYMER
  PolymerDistrib    polymer_bis.py:50-90 (:236-249)     per-structure bonds, class POLYMER
  Envelope          envelope.py:36-62 (:252-262)        envelope 0 (ellipsoid, all beads)
  GenEnvelope       genenvelope.py:37-58 (:263-274)     envelope 0 ('volume': per-structure map)
  interHiC/intraHiC inter_hic.py / intra_hic.py (:376)  per-structure bonds (igm_hic_select)
  Damid             damid.py:112-143 (:402-440)         envelope 1 (k < 0) on per-structure
                                                        atom flags (igm_damid_select)
  Sprite            sprite.py:36-71 (:456-480)          centroid slots + per-structure bonds
  Fish              fish.py:85-266 (:482-503)           per-structure bonds to the centre

Atom layout shared by the batch: the beads, ONE static centre dummy at the origin
(the Envelope/Damid/Fish centres are the same frozen point; LammpsModel merges the
consecutive ones, lammps_model.py:303-312), then `nslot` SPRITE centroid slots (a
structure's unused slots are inert: IGM_ATOM_FIXED, no bonds).  A restraint section
this module does not implement raises -- nothing in the config is dropped silently.

Violation classes (the kernel's record index -> the reference's vstat key,
repr(restraint), in ModelingStep's monitored_restraints order): bond classes
POLYMER, INTER_HIC, INTRA_HIC, SPRITE, FISH, then one class per envelope.
"""
import numpy as np

from . import model as M
from ._lib import IGM_ATOM_BEAD, IGM_ATOM_ENV0, IGM_ATOM_FIXED, bond_dtype

CLASS_SPRITE = 3
CLASS_FISH = 4
NCLASS = 5


class Batch(object):
    """Inputs of igm_mstep_run / igm_mstep_violations for one batch of structures."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def vstat_names(self, q):
        """vstat key per record class for the batch's structure q (None: a class the
        config does not monitor)."""
        return [n[q] if isinstance(n, list) else n for n in self.names]


def envelope_spec(shape, radius=None, semiaxes=None, k=1.0):
    """The nucleus envelope of model/restraints/envelope; the raw config values are
    kept for the vstat key (Envelope.__repr__ formats them as written, envelope.py:65)."""
    if shape == 'sphere':
        return {'shape': 'sphere', 'abc': (float(radius),) * 3, 'k': float(k), 'repr_abc': (radius,) * 3,
                'repr_k': k}
    if shape == 'ellipsoid':
        return {'shape': 'ellipsoid', 'abc': tuple(float(v) for v in semiaxes), 'k': float(k),
                'repr_abc': tuple(semiaxes), 'repr_k': k}
    raise NotImplementedError('Envelope (%s) not implemented' % shape)


class DeviceSelect(object):
    """The per-structure selections of the assembly on the GPU (the product path):
    interHiC/intraHiC (igm_hic_select), Damid._apply_envelope membership
    (igm_damid_select), the staging of the volumetric maps."""

    def __init__(self, ctx):
        self.ctx = ctx

    def hic(self, x, radii, chrom, rows, contact_range, k):
        from . import mstep
        return mstep.hic_select(x, radii, chrom, rows['row'], rows['col'], rows['dist'], contact_range, k,
                                ctx=self.ctx)

    def damid(self, x, radii, rows, abc, contact_range, env_index, base):
        from . import restraints as R
        return R.damid_envelope_flags(x, radii, rows, abc, contact_range, env_index, base, ctx=self.ctx)[0]

    def volumes(self, vols, struct_map):
        from . import volume as V
        V.stage(self.ctx, vols, struct_map)


def build(xyz, sids, index, spec, ctx, select=None):
    """xyz: (S, nbead, 3) float32 bead coordinates of the batch (struct-major);
    sids: their structure ids; index: radii, chrom, copy, copy_ptr, copy_idx (e.g. a
    steps.PopulationStore); spec: dict with
      evfactor, protocol (the optimization/optimizer_options dict),
      polymer   {contact_range, kspring, monitored[, contact_probabilities]} or
                {distrib: (loci, nn_dist), tolerance, kspring, monitored} or None,
      envelope  envelope_spec(...) or {'shape': 'exp_map', 'k', 'volumes' [maps],
                'struct_map' (S,) map index per structure, 'files' [names]},
      hic       {rows, contact_range, k} or None,
      damid     {rows, contact_range, k} or None,
      sprite    {assignment, indptr, selected, volume_fraction, k} or None,
      fish      {data (fish_assignment dict), rtype, tol, k} or None.
    ctx: the igm context of the device; select: the selection backend (default
    DeviceSelect(ctx); the CPU tests pass the oracle's)."""
    from . import restraints as R
    sel = select or DeviceSelect(ctx)
    xyz = np.ascontiguousarray(xyz, np.float32)
    S, nbead = xyz.shape[0], xyz.shape[1]
    sids = np.asarray(sids, np.int64)
    radii_b = np.asarray(index.radii, np.float32)
    chrom_b = np.asarray(index.chrom, np.int32)
    assert radii_b.shape == (nbead,) and len(sids) == S
    centre = nbead
    first_slot = nbead + 1
    # ---- SPRITE centroids first: they set the atom count
    sp = spec.get('sprite')
    sbonds = [np.zeros(0, bond_dtype)] * S
    nslot, active = 0, np.zeros(S, np.int32)
    cpos = None
    if sp is not None:
        nslot, cpos, active, sbonds = R.sprite_centroids(sp['assignment'], sp['indptr'], sp['selected'], xyz, sids,
                                                         radii_b, float(sp['volume_fraction']), float(sp['k']),
                                                         first_slot)
    natom = first_slot + nslot
    radii = np.zeros(natom, np.float32)
    radii[:nbead] = radii_b
    base = np.zeros(natom, np.uint32)
    base[:nbead] = IGM_ATOM_BEAD | IGM_ATOM_ENV0  # the nucleus envelope holds every bead
    base[centre] = IGM_ATOM_FIXED
    x = np.zeros((S, natom, 3), np.float32)
    x[:, :nbead] = xyz
    if nslot:
        x[:, first_slot:] = cpos
    # ---- envelopes
    env = spec['envelope']
    envelopes, env_scale, env_names = [], [], []
    volumes = None
    if env['shape'] == 'exp_map':
        volumes = env['volumes']
        sel.volumes(volumes, env.get('struct_map'))
        envelopes.append(('volume', float(env['k'])))
        env_scale.append(0.95)  # ExpEnvelope contact_range (genenvelope.py:49)
        files = env.get('files') or ['map%d' % m for m in range(len(volumes))]
        smap = env.get('struct_map')
        # GenEnvelope.__repr__ names the structure's own map file (genenvelope.py:60-61)
        env_names.append(['ExpEnvelope[shape=exp_map,map={},k={}]'.format(
            files[int(smap[q]) if smap is not None else 0], env.get('repr_k', env['k'])) for q in range(S)])
    else:
        abc = env['abc']
        envelopes.append((abc, float(env['k'])))
        env_scale.append(0.1 * float(np.mean(abc)))  # envelope.py:51
        env_names.append('Envelope[shape={},k={},a={},b={},c={}]'.format(
            env['shape'], env.get('repr_k', env['k']), *env.get('repr_abc', abc)))
    flags = base
    dm = spec.get('damid')
    if dm is not None:
        if env['shape'] not in ('sphere', 'ellipsoid'):
            raise NotImplementedError('DamID with a %s envelope (GenDamid) is not implemented' % env['shape'])
        cut = 1.0 - float(dm['contact_range'])
        abc = np.asarray(env['abc'], np.float64)
        e = len(envelopes)
        flags = sel.damid(x, radii, dm['rows'], abc, float(dm['contact_range']), e, base)
        envelopes.append((tuple(abc * cut), -float(dm['k'])))
        env_scale.append(cut * float(np.mean(abc)))  # damid.py:134
        env_names.append('Damid')
    if nslot:
        cf = R.centroid_flags(base, active, first_slot, nslot)
        flags = cf if flags.ndim == 1 else (flags & ~np.uint32(IGM_ATOM_FIXED)) | (cf & np.uint32(IGM_ATOM_FIXED))
    prm = M.params_from_cfg({'optimization': {'optimizer_options': spec['protocol']}}, envelopes,
                            evfactor=float(spec.get('evfactor', 1.0)))
    if spec.get('skin'):
        prm.skin = float(spec['skin'])
    # ---- bonds: polymer (shared or per structure), Hi-C, SPRITE, FISH
    names = [None] * NCLASS
    class_cr = np.zeros(NCLASS)
    pol = spec.get('polymer')
    poly = np.zeros(0, bond_dtype)
    pbonds = [np.zeros(0, bond_dtype)] * S
    if pol is not None and 'distrib' in pol:
        from . import polymer as P
        loci, nn = pol['distrib']
        pbonds = P.polymer_distrib_bonds(loci, nn, chrom_b, sids, pol.get('tolerance', 10.0), pol.get('kspring', 2.0))
        if pol.get('monitored', True):
            names[M.CLASS_POLYMER] = 'PolymerDistrib'
    elif pol is not None:
        poly = M.polymer_bonds(chrom_b, index.copy, radii_b, pol['contact_range'], pol['kspring'],
                               pol.get('contact_probabilities'))
        class_cr[M.CLASS_POLYMER] = 0.0 if pol.get('contact_probabilities') is not None else float(pol['contact_range'])
        if pol.get('monitored', True):
            names[M.CLASS_POLYMER] = 'Polymer'
    hic = spec.get('hic')
    chrom_all = np.concatenate([chrom_b, np.full(natom - nbead, -1, np.int32)]).astype(np.int32)
    if hic is not None:
        rows = hic['rows']
        hptr, hb, hc = sel.hic(x, radii, chrom_all, rows, float(hic['contact_range']), float(hic['k']))
        names[M.CLASS_INTER_HIC], names[M.CLASS_INTRA_HIC] = 'interHiC', 'intraHiC'
        class_cr[M.CLASS_INTER_HIC] = class_cr[M.CLASS_INTRA_HIC] = float(hic['contact_range'])
    else:
        hptr, hb, hc = np.zeros(S + 1, np.int64), np.zeros(0, bond_dtype), np.zeros(0, np.int32)
    if sp is not None:
        names[CLASS_SPRITE] = 'Sprite'
    fb = [np.zeros(0, bond_dtype)] * S
    fi = spec.get('fish')
    if fi is not None:
        fb = R.fish_bonds(fi['data'], index.copy_ptr, index.copy_idx, xyz, sids, fi['rtype'], centre,
                          tol=float(fi['tol']), kspring=float(fi['k']))
        names[CLASS_FISH] = 'Fish'
    per, pcls = [], []
    for s in range(S):
        parts = [(pbonds[s], M.CLASS_POLYMER), (hb[hptr[s]:hptr[s + 1]], None), (sbonds[s], CLASS_SPRITE),
                 (fb[s], CLASS_FISH)]
        per.append(np.concatenate([p for p, _ in parts]))
        pcls.append(np.concatenate([hc[hptr[s]:hptr[s + 1]] if c is None else np.full(len(p), c, np.int32)
                                    for p, c in parts]).astype(np.int32))
    ptr, bonds = M.concat_bonds(per)
    bcls = np.concatenate(pcls) if pcls else np.zeros(0, np.int32)
    return Batch(x=x, radii=radii, flags=flags, prm=prm, poly=poly,
                 poly_cls=np.full(len(poly), M.CLASS_POLYMER, np.int32), ptr=ptr, bonds=bonds, bcls=bcls,
                 class_cr=class_cr, env_scale=np.asarray(env_scale, np.float64), names=names + env_names,
                 nbead=nbead, natom=natom, nslot=nslot, active=active, centre=centre, volumes=volumes)


def run(batch, seeds, tol, ctx):
    """model.optimize + the violation records of a Batch: (x (S, natom, 3), info,
    stats (S, ncls, 104))."""
    from . import mstep
    xo, info = mstep.run(batch.prm, batch.x, batch.radii, batch.flags, batch.poly, batch.ptr, batch.bonds, seeds,
                         ctx=ctx)
    stats = mstep.violations(batch.prm, xo, batch.radii, batch.flags, batch.poly, batch.poly_cls, batch.ptr,
                             batch.bonds, batch.bcls, batch.class_cr, batch.env_scale, float(tol), ctx=ctx)
    return xo, info, stats
