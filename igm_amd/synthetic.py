"""Seeded synthetic inputs for the benchmark configurations of BASELINE.json
(SURVEY.md section 8(d)).  Inputs only -- nothing here is on the measured path.

  config B  2 Mb diploid (the demo index, 3008 beads), S structures, Hi-C pairs of
            the demo .hcs (tests/golden/demo_hic_pairs.npz), demo protocol.
  initial   RandomInit.generate_territories semantics (steps/RandomInit.py:207-240),
            R = init_radius, numpy.random.default_rng(1000 + sid) per structure.
"""
import os

import numpy as np

# demo/config_file.json optimizer_options of the reference (data), the protocol of
# every benchmark configuration
DEMO_PROTOCOL = {
    "mdsteps": 45000, "timestep": 0.25, "tstart": 500.0, "tstop": 0.01,
    "custom_annealing_protocol": {
        "num_steps": 4, "mdsteps": [5000, 15000, 15000, 10000],
        "tstarts": [5000.0, 500.0, 50.0, 1.0], "tstops": [500.0, 50.0, 1.0, 0.0],
        "evfactors": [0.5, 1.0, 1.0, 1.0], "envelope_factors": [1.2, 1.0, 1.0, 1.0],
        "relax": {"mdsteps": 500, "temperature": 1.0, "max_velocity": 10.0}},
    "damp": 50.0, "max_velocity": 1000.0, "etol": 0.0001, "ftol": 1e-06,
    "max_cg_iter": 500, "max_cg_eval": 500, "thermo": 1000, "write": -1,
}

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def uniform_sphere(rng, R, n):
    """RandomInit.uniform_sphere (py:182-203) vectorised."""
    phi = rng.uniform(0, 2 * np.pi, n)
    costheta = rng.uniform(-1, 1, n)
    u = rng.uniform(0, 1, n)
    theta = np.arccos(costheta)
    r = R * u ** (1.0 / 3.0)
    return np.stack([r * np.sin(theta) * np.cos(phi), r * np.sin(theta) * np.sin(phi), r * np.cos(theta)], 1)


def territories(chrom_sizes, R, seed):
    """RandomInit.generate_territories (py:207-240) with a seeded generator."""
    rng = np.random.default_rng(seed)
    chrom_sizes = np.asarray(chrom_sizes, np.int64)
    n_tot = int(chrom_sizes.sum())
    chr_radii = 0.75 * R * (chrom_sizes / n_tot) ** (1.0 / 3)
    crad = float(np.average(chr_radii))
    centers = uniform_sphere(rng, R - crad, len(chrom_sizes))
    crds = uniform_sphere(rng, crad, n_tot) + np.repeat(centers, chrom_sizes, axis=0)
    return crds.astype(np.float32)


def population_2mb(nstruct, first_sid=0, init_radius=7000.0):
    """Config B: the demo 2 Mb male diploid index with synthetic territories.
    Returns dict(xyz (S, N, 3) f32 struct-major, radii, chrom, copy, copy_ptr,
    copy_idx, chrom_sizes)."""
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    cs = pop['chrom_sizes']
    xyz = np.stack([territories(cs, init_radius, 1000 + first_sid + s) for s in range(nstruct)])
    return {'xyz': xyz, 'radii': pop['radii'], 'chrom': pop['chrom'], 'copy': pop['copy'],
            'copy_ptr': pop['copy_ptr'], 'copy_idx': pop['copy_idx'], 'chrom_sizes': cs}


def hic_pairs_2mb(sigma):
    """Upper-triangle demo .hcs entries with p >= sigma, in CSR order."""
    d = np.load(os.path.join(GOLDEN, 'demo_hic_pairs.npz'))
    if sigma < 0.02:
        raise ValueError('the committed demo pairs cover sigma >= 0.02')
    m = d['p'] >= sigma
    return d['i'][m], d['j'][m], d['p'][m]
