"""Population initialisation on the same batched engine.

  generate_territories -- RandomInit.generate_territories (igm/steps/RandomInit.py:207-240):
                          chromosome territories as spheres of 0.75 R (n_c / n)^(1/3),
                          centres uniform in R - <crad>, beads uniform in the territory;
                          drawn with a numpy RandomState in the reference's order (three
                          uniforms per point: phi, cos(theta), u), so a seeded run
                          reproduces the reference's draws.
  relax_population     -- RelaxInit.task (igm/steps/RelaxInit.py:93-258) for a whole batch:
                          steric + polymer + nucleus envelope (sphere / ellipsoid /
                          volumetric map), the optimizer protocol of the config, one
                          igm_mstep_run call instead of one LAMMPS process per structure.
"""
import numpy as np

from . import model as M
from . import mstep


def uniform_sphere(rng, R, n):
    """uniform_sphere (RandomInit.py:182-203) for n points, same draw order."""
    u = rng.random_sample((n, 3))
    phi = 0.0 + (2 * np.pi - 0.0) * u[:, 0]
    costheta = -1.0 + 2.0 * u[:, 1]
    theta = np.arccos(costheta)
    r = R * (u[:, 2] ** (1. / 3.))
    return np.stack([r * np.sin(theta) * np.cos(phi), r * np.sin(theta) * np.sin(phi), r * np.cos(theta)], 1)


def generate_territories(chrom_sizes, R=5000.0, rng=None):
    """One structure (n, 3) float64; chrom_sizes = index.chrom_sizes."""
    rng = np.random.mtrand._rand if rng is None else rng
    sizes = np.asarray(chrom_sizes, np.int64)
    n_tot = int(sizes.sum())
    chr_radii = [0.75 * R * (float(nb) / n_tot) ** (1. / 3) for nb in sizes]
    crad = np.average(chr_radii)
    out = np.empty((n_tot, 3))
    k = 0
    for nb in sizes:
        center = uniform_sphere(rng, R - crad, 1)[0]
        out[k:k + nb] = uniform_sphere(rng, crad, int(nb)) + center
        k += nb
    return out


def relax_population(cfg, xyz, radii, chrom, copy, struct_ids, volumes=None, volume_struct_map=None, ctx=None,
                     device=0):
    """RelaxInit.task for structures struct_ids: xyz (S, nbead, 3) -> relaxed (S, nbead, 3)
    float32 and the per-structure info.  cfg is the igm config dict (model/restraints/
    {excluded, polymer, envelope}, optimization/optimizer_options, runtime/step_no)."""
    from . import _lib
    c = ctx or _lib.context(device)
    rs = cfg['model']['restraints']
    radii = np.asarray(radii, np.float32)
    nb = len(radii)
    poly_cfg = rs['polymer']
    poly = M.polymer_bonds(chrom, copy, radii, poly_cfg['contact_range'], poly_cfg['polymer_kspring'],
                           cfg.get('runtime', {}).get('consecutive_contact_probabilities', None))
    env = rs['envelope']
    shape = env['nucleus_shape']
    if shape == 'sphere':
        envelope = ((float(env['nucleus_radius']),) * 3, float(env['nucleus_kspring']))
    elif shape == 'ellipsoid':
        envelope = (tuple(float(v) for v in env['nucleus_semiaxes']), float(env['nucleus_kspring']))
    elif shape == 'exp_map':
        from . import volume as V
        if volumes is None:
            raise ValueError('exp_map relax needs the volume maps')
        V.stage(c, volumes, volume_struct_map)
        envelope = ('volume', float(env['nucleus_kspring']))
    else:
        raise NotImplementedError('Envelope (%s) not implemented' % shape)
    atoms = M.Atoms(radii)  # beads (all in the envelope group) + the static centre dummy
    prm = M.params_from_cfg(cfg, [envelope], evfactor=float(rs['excluded']['evfactor']))
    x = np.zeros((len(struct_ids), atoms.n, 3), np.float32)
    x[:, :nb] = xyz
    opt = cfg['optimization']['optimizer_options']
    seeds = M.lammps_seeds(opt.get('seed', 6535), struct_ids, cfg.get('runtime', {}).get('step_no', 1))  # lammps.py:435
    xo, info = mstep.run(prm, x, atoms.radii, atoms.flags, poly, None, None, seeds, ctx=c)
    return xo[:, :nb], info
