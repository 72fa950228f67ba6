#!/opt/conda/bin/python3.9
"""Golden vectors for the configuration D/E A-steps, produced by running the
REFERENCE functions in this container (build container only, like make_golden.py):

    /opt/conda/bin/python3.9 tests/golden/make_golden_asteps.py

Inputs are the committed demo fixture (tests/golden/demo_population.npz: the demo
.hss.T coordinates, radii, copy index) plus seeded synthetic profiles/targets; the
outputs are what the reference computes from them.  Nothing of the reference is
written here except these numbers.

  damid_golden.npz   DamidActivationDistanceStep.get_damid_actdist_I
                     (steps/DamidActivationDistanceStep.py:376-471) for every demo
                     locus, shape 'sphere' (R=5500) and 'ellipsoid' (7840, 6470, 2450
                     scaled to the demo nucleus), it_corr 0/1, contact_range 0.05,
                     after the "%6d %.5f %.5f" text round trip of task()/reduce()
                     (:35, :286, :308).  The ellipsoid rows are the function's own
                     output: the step itself never calls it for an ellipsoid
                     (defect D3, :258).
  fish_golden.npz    FishAssignmentStep.get_rad_dists / get_min_max_and_idx
                     (steps/FishAssignmentStep.py:44-77) for 300 two-copy probes and
                     the target assignment target[idx] of task() (:218-242); pairs
                     through get_min_max_and_idx on all copy-pair distances (the
                     reference get_pair_dists never advances its row counter, defect
                     D4, so the pair distances are formed here as its docstring says)
  sprite_cluster_golden.npz
                     cython_compiled/sprite.pyx compute_gyration_radius
                     (:104-283) on 400 demo clusters (single- and multi-chromosome;
                     the per-chromosome representative drawn by np.random.choice is
                     recorded) and SpriteAssignmentStep.task's keep_best selection
                     (steps/SpriteAssignmentStep.py:138-143)
"""
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden  # noqa: E402  (builds the reference environment: stub alabtools + Cython SPRITE)
import numpy as np  # noqa: E402
import importlib  # noqa: E402
# the step modules (igm.steps re-exports the classes under the same names)
damid_mod = importlib.import_module('igm.steps.DamidActivationDistanceStep')
fish_mod = importlib.import_module('igm.steps.FishAssignmentStep')
sprite_mod = sys.modules['igm.cython_compiled.sprite']

assert np.__version__.startswith('1.')


def load_demo():
    d = np.load(os.path.join(HERE, 'demo_population.npz'))
    ptr, idx = d['copy_ptr'], d['copy_idx']
    copy_index = {h: [int(x) for x in idx[ptr[h]:ptr[h + 1]]] for h in range(len(ptr) - 1)}
    return d, copy_index


def damid_roundtrip(rows):
    fmt = damid_mod.damid_actdist_fmt_str
    with tempfile.NamedTemporaryFile('w+', suffix='.tmp', delete=False) as f:
        f.write('\n'.join([fmt % x for x in rows]))
        name = f.name
    a = np.genfromtxt(name, dtype=damid_mod.damid_actdist_shape)
    os.unlink(name)
    return np.atleast_1d(a)


def make_damid(d, copy_index):
    crd, radii, chrom = d['coordinates'], d['radii'], d['chrom']
    hss = make_golden.DuckHss(crd, radii, copy_index, chrom)
    nhap = len(d['copy_ptr']) - 1
    rng = np.random.RandomState(11)
    # a DamID profile over the haploid loci (p ~ Beta(2, 5)) and plast
    profile = rng.beta(2.0, 5.0, nhap).astype(np.float32)
    plast = np.where(rng.rand(nhap) < 0.5, rng.beta(2.0, 5.0, nhap), 0.0).astype(np.float32)
    plast[:5] = 1.0  # cleanProbability's pexist >= 1 branch
    g = {'profile': profile, 'plast': plast}
    shapes = {'sphere': 5500.0, 'ellipsoid': [7840.0 * 0.7, 6470.0 * 0.85, 2450.0 * 2.2]}
    for shape, param in shapes.items():
        for it_corr in (0, 1):
            for sigma in (0.45, 0.2):
                sel = np.where(profile >= sigma)[0]
                # the rows task() writes for these loci (params are f32: setup() :211-217)
                params = np.array([(i, profile[i], plast[i]) for i in sel], dtype=np.float32)
                rows = []
                for I, p_exp, pl in params:
                    rows += damid_mod.get_damid_actdist_I(int(I), p_exp, pl, hss, it_corr, contact_range=0.05,
                                                          shape=shape, nucleus_param=param)
                rt = damid_roundtrip(rows)
                tag = '%s_c%d_s%g' % (shape, it_corr, sigma)
                g[tag + '_loci'] = sel.astype(np.int32)
                g[tag + '_loc'] = rt['loc']
                g[tag + '_dist'] = rt['dist']
                g[tag + '_prob'] = rt['prob']
    g['ellipsoid_semiaxes'] = np.array(shapes['ellipsoid'], np.float64)
    g['sphere_radius'] = np.float64(shapes['sphere'])
    return g


def make_fish(d, copy_index):
    crd = d['coordinates']
    S = crd.shape[1]
    nhap = len(d['copy_ptr']) - 1
    rng = np.random.RandomState(12)
    two = [h for h in range(nhap) if len(copy_index[h]) == 2]
    probes = np.array(sorted(rng.choice(two, 300, replace=False)), np.int32)
    g = {'probes': probes}
    # per-probe target distributions (sorted LogNormal x S)
    rmin = np.sort(rng.lognormal(7.5, 0.4, (len(probes), S)), axis=1).astype(np.float32)
    rmax = np.sort(rng.lognormal(8.0, 0.3, (len(probes), S)), axis=1).astype(np.float32)
    mins, maxs, imin, imax, amin, amax = [], [], [], [], [], []
    for q, probe in enumerate(probes):
        ii = copy_index[int(probe)]
        dists = fish_mod.get_rad_dists(ii, crd.shape[0], S, crd)
        mn, mx, i1, i2 = fish_mod.get_min_max_and_idx(dists)
        mins.append(mn)
        maxs.append(mx)
        imin.append(i1)
        imax.append(i2)
        amin.append(rmin[q][i1])  # task(): target_min[idxmin]
        amax.append(rmax[q][i2])
    g.update(radial_min_targets=rmin, radial_max_targets=rmax, rad_min=np.array(mins), rad_max=np.array(maxs),
             rad_idxmin=np.array(imin), rad_idxmax=np.array(imax), radial_min=np.array(amin, np.float32),
             radial_max=np.array(amax, np.float32))
    # pairs: all copy-pair distances as get_pair_dists documents them (np.linalg.norm, f32)
    pi = rng.choice(nhap, 300)
    pj = rng.choice(nhap, 300)
    keep = pi != pj
    pairs = np.stack([pi[keep], pj[keep]], 1).astype(np.int32)
    pmin = np.sort(rng.lognormal(7.0, 0.5, (len(pairs), S)), axis=1).astype(np.float32)
    pmax = np.sort(rng.lognormal(7.6, 0.4, (len(pairs), S)), axis=1).astype(np.float32)
    amin, amax, dmn, dmx = [], [], [], []
    for q, (i, j) in enumerate(pairs):
        ii, jj = copy_index[int(i)], copy_index[int(j)]
        dists = np.empty((len(ii) * len(jj), S))
        c = 0
        for a in ii:
            for b in jj:
                dists[c] = np.linalg.norm(crd[a, :, :] - crd[b, :, :], axis=1)
                c += 1
        mn, mx, i1, i2 = fish_mod.get_min_max_and_idx(dists)
        dmn.append(mn)
        dmx.append(mx)
        amin.append(pmin[q][i1])
        amax.append(pmax[q][i2])
    g.update(pairs=pairs, pair_min_targets=pmin, pair_max_targets=pmax, pair_dmin=np.array(dmn),
             pair_dmax=np.array(dmx), pair_min=np.array(amin, np.float32), pair_max=np.array(amax, np.float32))
    return g


class _Ix(object):
    def __init__(self, chrom):
        self.chrom = chrom


def make_sprite_clusters(d, copy_index):
    crd = np.ascontiguousarray(d['coordinates'])  # bead-major (N, S, 3): the .hss layout
    hap_chrom = d['hap_chrom']
    index = _Ix(hap_chrom)
    nhap = len(hap_chrom)
    rng = np.random.RandomState(13)
    # representatives drawn by compute_gyration_radius are recorded by wrapping np.random.choice
    drawn = []
    real_choice = np.random.choice

    def recording_choice(x, *a, **k):
        v = real_choice(x, *a, **k)
        drawn.append(int(v))
        return v

    np.random.seed(2024)
    np.random.choice = recording_choice
    g = {}
    ptr, loci, reps, rptr = [0], [], [], [0]
    rg2s, sel, best = [], [], []
    try:
        for c in range(400):
            if c % 2 == 0:  # single chromosome: a run of loci on one chromosome
                ch = rng.randint(0, 22)
                cand = np.where(hap_chrom == ch)[0]
                n = rng.randint(2, 12)
                start = rng.randint(0, len(cand) - n)
                cl = cand[start:start + n]
            else:  # 2..5 chromosomes
                cl = np.unique(rng.choice(nhap, rng.randint(2, 16), replace=False))
            cl = np.sort(cl).astype(np.int64)
            drawn.clear()
            r, b, s = sprite_mod.compute_gyration_radius(crd, cl, index, copy_index)
            loci += cl.tolist()
            ptr.append(len(loci))
            reps += drawn
            rptr.append(len(reps))
            rg2s.append(np.asarray(r, np.float32))
            sel.append(np.asarray(s, np.int32))  # (S, len(cluster)) diploid bead ids
            best.append(int(b))
    finally:
        np.random.choice = real_choice
    S = crd.shape[1]
    keep_best = 50
    ind = []
    for r in rg2s:
        i = np.argpartition(r, keep_best)[:keep_best]  # SpriteAssignmentStep.py:138-139
        ind.append(i[np.argsort(r[i])])
    g.update(cl_ptr=np.array(ptr, np.int32), cl_loci=np.array(loci, np.int32), rep_ptr=np.array(rptr, np.int32),
             reps=np.array(reps, np.int32), rg2s=np.stack(rg2s), best=np.array(best, np.int32),
             selected=np.concatenate([x.reshape(S, -1) for x in sel], axis=1), keep_best=np.int32(keep_best),
             best_idx=np.stack(ind).astype(np.int32))
    return g


def main():
    d, copy_index = load_demo()
    np.savez_compressed(os.path.join(HERE, 'damid_golden.npz'), **make_damid(d, copy_index))
    np.savez_compressed(os.path.join(HERE, 'fish_golden.npz'), **make_fish(d, copy_index))
    np.savez_compressed(os.path.join(HERE, 'sprite_cluster_golden.npz'), **make_sprite_clusters(d, copy_index))
    for f in ('damid_golden.npz', 'fish_golden.npz', 'sprite_cluster_golden.npz'):
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == '__main__':
    main()
