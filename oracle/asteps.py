"""ORACLE (test infrastructure only -- never imported by the product path):
NumPy restatements of the configuration D/E A-steps of the reference, operation by
operation with NumPy-1.x promotion, pinned against the golden vectors that
tests/golden/make_golden_asteps.py produced by running the reference itself.

  damid_actdist          steps/DamidActivationDistanceStep.py:39-76,362-471 (+ the
                         "%6d %.5f %.5f" text round trip of task()/reduce(), :35,:286,:308)
  fish_radial/fish_pair  steps/FishAssignmentStep.py:23-77,188-242
  sprite_cluster_rg2     cython_compiled/sprite.pyx:104-283 with get_rg2s_cpp
                         (cpp_sprite_assignment.cpp:49-143)
  keep_best              steps/SpriteAssignmentStep.py:138-143
  contact_counts         steps/HicEvaluationStep.py:109 (buildContactMap; parity unpinned)
  polymer_assign         steps/PolymerAssignmentStep.py:24-32,84-129 (golden vectors:
                         tests/golden/make_golden_polymer.py, the reference run here)
"""
import numpy as np

f32 = np.float32


def _clean(pij, pexist):
    """cleanProbability (DamidActivationDistanceStep.py:362-372).  Under NumPy 1.x an
    np.float32 scalar combined with a Python float or int promotes to float64 (NumPy 2
    would stay in float32, so the casts are explicit); max(0, x) returns 0 if x <= 0."""
    pij, pexist = float(pij), float(pexist)
    if pexist < 1:
        pclean = (pij - pexist) / (1.0 - pexist)
    else:
        pclean = pij
    return max(0, pclean)


def damid_d2(x, r, contact_range, shape, param):
    """snormsq_sphere / snormsq_ellipse (py:39-76) as get_damid_actdist_I calls them
    (R = param * (1 - contact_range), :436-438): x (S, 3) f32 -> (S,) f32 values.
    NumPy 1.x value-based casting: the float64 scalar divisor is cast to float32 and
    the division runs in float32 (written out explicitly for NumPy 2)."""
    x = np.asarray(x, np.float32)
    R = np.array(param, np.float64) * (1 - contact_range)
    sq = np.square(x)
    if shape == 'sphere':
        D = f32((float(R) - float(r)) ** 2)
        return ((sq[:, 0] + sq[:, 1]) + sq[:, 2]) / D
    a, b, c = (float(v) - float(r) for v in R)
    return (sq[:, 0] / f32(a * a) + sq[:, 1] / f32(b * b)) + sq[:, 2] / f32(c * c)


def damid_actdist(crd, radii, copy_ptr, copy_idx, loci, profile, plast, it_corr, contact_range=0.05,
                  shape='sphere', param=5000.0):
    """Rows {loc, dist, prob} task() writes for the loci (in order), after the text
    round trip.  crd: bead-major (N, S, 3) f32."""
    rows = []
    S = crd.shape[1]
    for I in loci:
        ii = [int(v) for v in copy_idx[copy_ptr[I]:copy_ptr[I + 1]]]
        nc = len(ii)
        p_exp, pl = f32(profile[I]), f32(plast[I])  # setup() stores (I, p_exp, plast) as float32 (:211-217)
        r = radii[ii[0]]
        d_sq = np.empty(nc * S)
        for i in range(nc):
            d_sq[i * S:(i + 1) * S] = damid_d2(crd[ii[i]], r, contact_range, shape, param)
        d_sq[::-1].sort()  # descending (:444)
        if it_corr == 1:
            pnow = float(np.count_nonzero(d_sq >= 1.0)) / (S * nc)
            p = _clean(p_exp, _clean(pnow, pl))
        else:
            p = float(p_exp)
        ad = 2
        if p > 0:
            o = min(nc * S - 1, int(np.round(np.float64(nc * S) * p)))  # round half to even
            ad = float(np.sqrt(d_sq[o]))
        for i in ii:
            line = '%6d %.5f %.5f' % (i, ad, p)
            a, b, c = line.split()
            rows.append((int(a), f32(float(b)), f32(float(c))))
    out = np.zeros(len(rows), [('loc', 'i4'), ('dist', 'f4'), ('prob', 'f4')])
    if rows:
        out['loc'], out['dist'], out['prob'] = zip(*rows)
    return out


def _rank(v):
    """argsort(argsort(v)) (FishAssignmentStep.py:74-75) with ties in index order."""
    order = np.argsort(v, kind='stable')
    r = np.empty(len(v), np.int64)
    r[order] = np.arange(len(v))
    return r


def fish_radial(crd, copy_ptr, copy_idx, probes, tmin, tmax):
    """get_rad_dists + get_min_max_and_idx + target[idx] (py:44-77, 218-242) for every
    probe; every copy of the probe (the reference reads ii[0], ii[1] only)."""
    S = crd.shape[1]
    out_min = np.zeros((len(probes), S), np.float32)
    out_max = np.zeros((len(probes), S), np.float32)
    dmin = np.zeros((len(probes), S))
    dmax = np.zeros((len(probes), S))
    for q, pr in enumerate(probes):
        ii = copy_idx[copy_ptr[pr]:copy_ptr[pr + 1]]
        d = np.stack([np.linalg.norm(crd[i], axis=1) for i in ii]).astype(np.float64)
        dmin[q], dmax[q] = d.min(0), d.max(0)
        out_min[q] = tmin[q][_rank(dmin[q])]
        out_max[q] = tmax[q][_rank(dmax[q])]
    return out_min, out_max, dmin, dmax


def fish_pair(crd, copy_ptr, copy_idx, pairs, tmin, tmax):
    """The pair path with every copy pair's distance (get_pair_dists' documented
    intent; the reference never advances its row counter, defect D4)."""
    S = crd.shape[1]
    out_min = np.zeros((len(pairs), S), np.float32)
    out_max = np.zeros((len(pairs), S), np.float32)
    dmin = np.zeros((len(pairs), S))
    dmax = np.zeros((len(pairs), S))
    for q, (i, j) in enumerate(pairs):
        ii = copy_idx[copy_ptr[i]:copy_ptr[i + 1]]
        jj = copy_idx[copy_ptr[j]:copy_ptr[j + 1]]
        d = np.stack([np.linalg.norm(crd[a] - crd[b], axis=1) for a in ii for b in jj]).astype(np.float64)
        dmin[q], dmax[q] = d.min(0), d.max(0)
        out_min[q] = tmin[q][_rank(dmin[q])]
        out_max[q] = tmax[q][_rank(dmax[q])]
    return out_min, out_max, dmin, dmax


def rg2_f32(pts):
    """gyration_radius_sq (cpp_sprite_assignment.cpp:49-61) in float32, left to right."""
    n = len(pts)
    m = [f32(0), f32(0), f32(0)]
    for p in pts:
        m = [f32(m[d] + p[d]) for d in range(3)]
    m = [f32(m[d] / f32(n)) for d in range(3)]
    rg = f32(0)
    for p in pts:
        dx, dy, dz = f32(p[0] - m[0]), f32(p[1] - m[1]), f32(p[2] - m[2])
        rg = f32(rg + f32(f32(f32(dx * dx) + f32(dy * dy)) + f32(dz * dz)))
    return f32(rg / f32(n))


def sprite_cluster_rg2(crd, hap_chrom, copy_ptr, copy_idx, cluster, reps, structs=None):
    """compute_gyration_radius (sprite.pyx:104-283) with the per-chromosome
    representatives given (they are np.random.choice draws in the reference, D9).
    Returns rg2s (S,) f32 and selected beads (S, len(cluster))."""
    cluster = np.sort(np.asarray(cluster))
    S = crd.shape[1]
    structs = range(S) if structs is None else structs
    ci = lambda h: [int(v) for v in copy_idx[copy_ptr[h]:copy_ptr[h + 1]]]
    cchroms = hap_chrom[cluster]
    rg = np.zeros(S, np.float32)
    sel = np.zeros((S, len(cluster)), np.int32)
    if len(np.unique(cchroms)) == 1:
        nc = len(ci(cluster[0]))
        groups = [[ci(i)[k] for i in cluster] for k in range(nc)]
        for s in structs:
            vals = [rg2_f32([crd[b, s] for b in g]) for g in groups]
            k = int(np.argmin(vals))  # first minimum
            rg[s], sel[s] = vals[k], groups[k]
        return rg, sel
    chroms = list(np.unique(cchroms))
    by_chrom = [cluster[cchroms == c] for c in chroms]
    all_segments = np.concatenate(by_chrom)
    for s in structs:
        # get_rg2s_cpp on the representatives: mixed-radix combinations, strict <, first found
        alts = [[crd[b, s] for b in ci(r)] for r in reps]
        ncomb = int(np.prod([len(a) for a in alts]))
        best, bestc = f32(1e8), None
        for k in range(ncomb):
            kk, comb = k, []
            for a in alts:
                comb.append(kk % len(a))
                kk //= len(a)
            v = rg2_f32([alts[i][comb[i]] for i in range(len(alts))])
            if v < best:
                best, bestc = v, comb
        choice = {hap_chrom[r]: bestc[i] for i, r in enumerate(reps)}
        beads = [ci(seg)[choice[hap_chrom[seg]]] for seg in all_segments]
        rg[s] = rg2_f32([crd[b, s] for b in beads])
        sel[s] = beads
    return rg, sel


def keep_best(rg2s, k):
    """argpartition + argsort of SpriteAssignmentStep.task (py:138-139), ties by index."""
    return np.argsort(rg2s, kind='stable')[:k]


def _snormsq_exp(x, vol):
    """snormsq_exp (DamidActivationDistanceStep.py:79-115): float64 arithmetic on the
    f32 coordinates, np.round half to even, np.dot as the reference BLAS sums it,
    (t0^2 + t2^2) + t1^2."""
    origin = np.array([float(v) for v in vol['origin']])
    grid = np.array([float(v) for v in vol['grid']])
    center = np.array([float(v) for v in vol['center']])
    n = np.asarray(vol['nvoxel'])
    mat = vol['matrice']
    vox = np.round(np.array((np.asarray(x, np.float32) - origin) / grid)).astype(int)
    out = []
    for k in range(vox.shape[0]):
        if (vox[k] >= 0).all() and (vox[k] < n).all():
            t = x[k] - (mat[tuple(vox[k])][0:3] * grid + origin)
        else:
            t = (vox[k] - center) * grid
        t = [float(v) for v in t]
        out.append((t[0] * t[0] + t[2] * t[2]) + t[1] * t[1])
    return out


def damid_actdist_exp(crd, copy_ptr, copy_idx, loci, pexp, plast, it_corr, contact_range, maps, volumes_idx):
    """get_damid_actdist_exp (py:475-577) + the text round trip: rows {loc, dist, prob}.
    pexp/plast are per listed locus (the batch params); maps[m] is volume_idx m."""
    S = crd.shape[1]
    vidx = np.asarray(volumes_idx)
    rows = []
    for q, I in enumerate(loci):
        ii = [int(v) for v in copy_idx[copy_ptr[I]:copy_ptr[I + 1]]]
        nc = len(ii)
        d = []
        for m in sorted(set(vidx.tolist())):
            where = np.where(vidx == m)[0]
            for b in ii:
                d += _snormsq_exp(crd[b][where], maps[m])
        d = np.sort(np.array(d))
        if it_corr == 1:
            pnow = float(np.count_nonzero(d >= contact_range)) / (S * nc)
            p = _clean(pexp[q], _clean(pnow, plast[q]))
        else:
            p = float(pexp[q])
        ad = 1e-9
        if p > 0:
            o = min(nc * S - 1, int(np.round(np.float64(nc * S) * p)))
            ad = float(np.sqrt(d[o]))
        for i in ii:
            a, b, c = ('%6d %.5f %.5f' % (i, ad, p)).split()
            rows.append((int(a), f32(float(b)), f32(float(c))))
    out = np.zeros(len(rows), [('loc', 'i4'), ('dist', 'f4'), ('prob', 'f4')])
    if rows:
        out['loc'], out['dist'], out['prob'] = zip(*rows)
    return out


def polymer_assign(crd, loci, edges, prob, rng):
    """PolymerAssignmentStep.task for `loci` in order, drawing from `rng` (a RandomState)
    as the reference draws from np.random: per locus np.sort(choice(edges, S, p)), the
    float32 norms |x_i - x_(i+1)| ranked (argsort(argsort), ties in structure order --
    the reference's default quicksort leaves exact ties unspecified) and the sorted
    draws indexed by rank; returned as the reduce() 'f4' dataset."""
    S = crd.shape[1]
    out = np.zeros((len(loci), S), np.float32)
    for q, i in enumerate(loci):
        sampled = np.sort(rng.choice(edges, S, p=prob))
        d = np.linalg.norm(crd[i, :, :] - crd[i + 1, :, :], axis=1)
        idx = np.argsort(np.argsort(d, kind='stable'), kind='stable')
        out[q] = sampled[idx]
    return out


def contact_counts(crd, radii, contact_range):
    """Population contact counts behind HicEvaluationStep.reduce's buildContactMap
    (steps/HicEvaluationStep.py:109; alabtools, absent: parity unpinned) with IGM's
    own contact test -- float32 norm (restraints/inter_hic.py:47) <= fl32(cr * fl32(ri + rj))
    (restraints/hic.py r0).  crd (nbead, S, 3) float32.  Returns (nbead, nbead) int32."""
    crd = np.asarray(crd, f32)
    r = np.asarray(radii, f32)
    thr = f32(contact_range) * (r[:, None] + r[None, :])
    n = crd.shape[0]
    out = np.zeros((n, n), np.int32)
    for s in range(crd.shape[1]):
        x = crd[:, s, :]
        d = x[:, None, :] - x[None, :, :]
        dd = np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])
        out += dd <= thr
    return out
