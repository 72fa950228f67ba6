"""Seeded synthetic inputs for the benchmark configurations of BASELINE.json
(SURVEY.md section 8(d)).  Inputs only -- nothing here is on the measured path.

  config B  2 Mb diploid (the demo index, 3008 beads), S structures, Hi-C pairs of
            the demo .hcs (tests/golden/demo_hic_pairs.npz), demo protocol.
  config C  200 kb hg38 male diploid (15 453 haploid bins, 29 838 beads), radii from
            occupancy 0.4 in a 5500 nm sphere (_preprocess.py:153-162), synthetic .hcs:
            intra p = min(1, 0.9 |i-j|^-1) for |i-j| <= 200, inter density 1e-4 with
            p ~ LogUniform(1e-3, 5e-2), default_rng(0).
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


# hg38 chromosome lengths (bp), chr1..chr22, chrX, chrY: the genome of the demo .hcs
HG38_LENGTHS = [248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973, 145138636,
                138394717, 133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345,
                83257441, 80373285, 58617616, 64444167, 46709983, 50818468, 156040895, 57227415]


def male_diploid_index(resolution, lengths=HG38_LENGTHS):
    """alabtools make_diploid layout of a male genome (as in the demo index): copy 0
    of chr1..chrY, then copy 1 of chr1..chr22; copy_index[h] = [h, h + nhap] for
    autosomes, [h] for X and Y.  Returns dict(chrom, copy, start, end, chrom_sizes,
    copy_ptr, copy_idx, nhap)."""
    nb = [-(-L // resolution) for L in lengths]
    hap_chrom = np.repeat(np.arange(len(lengths), dtype=np.int32), nb)
    hap_start = np.concatenate([np.arange(n, dtype=np.int64) * resolution for n in nb])
    hap_end = np.concatenate([np.minimum((np.arange(n, dtype=np.int64) + 1) * resolution, L)
                              for n, L in zip(nb, lengths)])
    nhap = len(hap_chrom)
    auto = hap_chrom < 22
    chrom = np.concatenate([hap_chrom, hap_chrom[auto]]).astype(np.int32)
    copy = np.concatenate([np.zeros(nhap, np.int32), np.ones(int(auto.sum()), np.int32)])
    start = np.concatenate([hap_start, hap_start[auto]])
    end = np.concatenate([hap_end, hap_end[auto]])
    second = np.full(nhap, -1, np.int64)
    second[auto] = nhap + np.arange(int(auto.sum()))
    ptr = np.zeros(nhap + 1, np.int32)
    ptr[1:] = np.cumsum(1 + auto.astype(np.int32))
    idx = np.empty(ptr[-1], np.int32)
    idx[ptr[:-1]] = np.arange(nhap)
    idx[ptr[:-1][auto] + 1] = second[auto]
    chrom_sizes = np.concatenate([nb, nb[:22]]).astype(np.int64)
    return dict(chrom=chrom, copy=copy, start=start, end=end, chrom_sizes=chrom_sizes, copy_ptr=ptr,
                copy_idx=idx, nhap=nhap, hap_chrom=hap_chrom)


def occupancy_radii(start, end, occupancy=0.4, nucleus_radius=5500.0):
    """_preprocess.py:153-162: bead volume proportional to its bp size."""
    vol = 4.0 / 3.0 * np.pi * nucleus_radius ** 3
    bp = (end - start).astype(np.float64)
    rho = occupancy * vol / bp.sum()
    return ((rho * bp) / (4.0 / 3.0 * np.pi)) ** (1.0 / 3.0)


def population_200kb(nstruct, first_sid=0, init_radius=7000.0, semiaxes=None):
    """Config C: 200 kb hg38 male diploid, synthetic territories (same recipe as
    population_2mb).  Same keys as population_2mb.  With `semiaxes` (config D's
    ellipsoid) the radii follow the occupancy of the ellipsoid's volume
    (_preprocess.py:153-162 with the volume-equivalent radius: 118.5 nm for
    ELLIPSOID_D) and the territories are stretched by semiaxes / 5500."""
    ix = male_diploid_index(200000)
    req = 5500.0 if semiaxes is None else float(np.prod(semiaxes)) ** (1.0 / 3.0)
    radii = occupancy_radii(ix['start'], ix['end'], nucleus_radius=req).astype(np.float32)
    xyz = np.stack([territories(ix['chrom_sizes'], init_radius, 1000 + first_sid + s) for s in range(nstruct)])
    if semiaxes is not None:
        xyz = (xyz * (np.asarray(semiaxes, np.float64) / 5500.0)).astype(np.float32)
    return {'xyz': xyz, 'radii': radii, 'chrom': ix['chrom'], 'copy': ix['copy'], 'copy_ptr': ix['copy_ptr'],
            'copy_idx': ix['copy_idx'], 'chrom_sizes': ix['chrom_sizes'], 'hap_chrom': ix['hap_chrom']}


def hic_pairs_200kb(sigma, max_sep=200, inter_density=1e-4, seed=0):
    """Synthetic 200 kb .hcs, upper triangle in CSR order,
    entries with p >= sigma: (i, j, p) arrays."""
    ix = male_diploid_index(200000)
    hc = ix['hap_chrom']
    n = ix['nhap']
    rng = np.random.default_rng(seed)
    ii, jj, pp = [], [], []
    for d in range(1, max_sep + 1):
        i = np.arange(n - d)
        ok = hc[i] == hc[i + d]
        ii.append(i[ok])
        jj.append(i[ok] + d)
        pp.append(np.full(int(ok.sum()), min(1.0, 0.9 / d), np.float32))
    # inter-chromosomal entries: density inter_density of the inter pairs
    sizes = np.bincount(hc)
    n_inter = (n * n - int((sizes.astype(np.int64) ** 2).sum())) // 2
    k = int(round(inter_density * n_inter))
    a = rng.integers(0, n, 4 * k)
    b = rng.integers(0, n, 4 * k)
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    keep = hc[lo] != hc[hi]
    key = np.unique(lo[keep].astype(np.int64) * n + hi[keep])[:k]
    ii.append((key // n).astype(np.int64))
    jj.append((key % n).astype(np.int64))
    pp.append(np.exp(rng.uniform(np.log(1e-3), np.log(5e-2), len(key))).astype(np.float32))
    i = np.concatenate(ii).astype(np.int32)
    j = np.concatenate(jj).astype(np.int32)
    p = np.concatenate(pp)
    m = p >= sigma
    order = np.lexsort((j[m], i[m]))
    return i[m][order], j[m][order], p[m][order]


# ---- configurations D/E A-step inputs ----------------------
ELLIPSOID_D = (7840.0, 6470.0, 2450.0)


def damid_profile_200kb(seed=1):
    """Config D: DamID lamina-contact profile over the 15 453 haploid 200 kb loci,
    p ~ Beta(2, 5) with rng(seed), float32 (the reference loads it as float32 text)."""
    nhap = male_diploid_index(200000)['nhap']
    return np.random.default_rng(seed).beta(2.0, 5.0, nhap).astype(np.float32)


def sprite_clusters_200kb(nclusters=100000, seed=2, lo=2, hi=20):
    """Config E: SPRITE clusters of lo..hi haploid loci.  Half are runs on one
    chromosome, half draw from 2..6 chromosomes (each a short run) -- the mix of
    single- and multi-chromosome clusters the reference handles.  Returns
    (indptr, data) like the clusters h5 (SpriteAssignmentStep.py:84-99)."""
    ix = male_diploid_index(200000)
    hc = ix['hap_chrom']
    starts = np.concatenate([[0], np.cumsum(np.bincount(hc))])
    rng = np.random.default_rng(seed)
    ptr, data = [0], []
    for c in range(nclusters):
        n = int(rng.integers(lo, hi + 1))
        nch = 1 if c % 2 == 0 else int(rng.integers(2, 7))
        chroms = rng.choice(24, size=nch, replace=False)
        parts = np.array_split(np.arange(n), nch)
        cl = []
        for ch, part in zip(chroms, parts):
            if len(part) == 0:
                continue
            size = starts[ch + 1] - starts[ch]
            st = int(rng.integers(0, size - len(part)))
            cl.extend(range(starts[ch] + st, starts[ch] + st + len(part)))
        cl = np.unique(cl)
        data.extend(cl.tolist())
        ptr.append(len(data))
    return np.asarray(ptr, np.int64), np.asarray(data, np.int32)


def fish_inputs_200kb(nstruct, nprobe=500, npair=500, seed=3):
    """Config E: FISH probes and pairs over the 200 kb loci with sorted LogNormal
    target distributions x S (nm)."""
    nhap = male_diploid_index(200000)['nhap']
    rng = np.random.default_rng(seed)
    probes = np.sort(rng.choice(nhap, nprobe, replace=False)).astype(np.int32)
    pi = rng.choice(nhap, npair)
    pj = rng.choice(nhap, npair)
    pj = np.where(pj == pi, (pj + 1) % nhap, pj)
    pairs = np.stack([pi, pj], 1).astype(np.int32)
    srt = lambda m, s, n: np.sort(rng.lognormal(m, s, (n, nstruct)), axis=1).astype(np.float32)
    return {'probes': probes, 'radial_min': srt(7.5, 0.4, nprobe), 'radial_max': srt(8.0, 0.3, nprobe),
            'pairs': pairs, 'pair_min': srt(7.0, 0.5, npair), 'pair_max': srt(7.6, 0.4, npair)}
