#!/opt/conda/bin/python3.9
"""Golden vectors for the volumetric map restraint's violation scores, produced by
running the REFERENCE ExpEnvelope.getScores (igm/model/forces.py:306-417) on maps
written in the VolumeFile format and read back by the reference VolumeFile
(igm/utils/files.py:137-166).  Build container only, like make_golden.py:

    /opt/conda/bin/python3.9 tests/golden/make_golden_volume.py

volume_golden.npz: for body 0 (nucleus sphere R=5500, 100 nm grid) and body 1
(nucleolus sphere R=1500 centred off-origin), k = +1 and -1, contact_range 0.95:
the map (nvoxel, center, origin, grid, matrice), 4000 particle positions (f32, some
outside the grid) and the reference's per-particle scores.
"""
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import make_golden  # noqa: E402,F401  (builds the reference environment)
import importlib  # noqa: E402
import numpy as np  # noqa: E402
from igm_amd import volume as V  # noqa: E402  (map construction and .bin writer only)

forces = importlib.import_module('igm.model.forces')
assert np.__version__.startswith('1.')


class P(object):
    def __init__(self, pos):
        self.pos = np.asarray(pos, np.float32)


def main():
    rng = np.random.RandomState(21)
    out = {}
    maps = {0: V.sphere_map(5500.0, 100.0, 3, body_idx=0),
            1: V.sphere_map(1500.0, 100.0, 3, body_idx=1, center=(1000.0, 0.0, 500.0))}
    for body, vol in maps.items():
        span = 7000.0 if body == 0 else 2500.0
        c = np.asarray(vol['center'], np.float64)
        pos = (c + rng.uniform(-span, span, (4600, 3))).astype(np.float32)
        # the reference raises IndexError when round(idx) == nvoxel (idx in [n - 0.5, n));
        # such positions are dropped here (the GPU restatement clamps them)
        n = np.asarray(vol['nvoxel'])
        bad = np.zeros(len(pos), bool)
        for k in (1.0, -1.0):
            o = np.array(vol['origin'], np.float64)
            g = np.array(vol['grid'], np.float64)
            if k < 0:
                o, g = (o * 0.95, g * 0.95) if body == 0 else (o / 0.95, g / 0.95)
            ix = (pos - o) / g
            bad |= np.any((ix >= n - 0.5) & (ix < n), axis=1)
        pos = pos[~bad][:4000]
        parts = [P(x) for x in pos]
        with tempfile.NamedTemporaryFile(suffix='.bin', delete=False) as f:
            name = f.name
        V.write_volume(name, vol)
        for k in (1.0, -1.0):
            f = forces.ExpEnvelope(list(range(len(parts))), volume_file=name, k=k, contact_range=0.95)
            s = f.getScores(parts)
            out['b%d_k%+d_scores' % (body, int(k))] = np.asarray(s, np.float64)
        os.unlink(name)
        for key in ('nvoxel', 'center', 'origin', 'grid', 'matrice'):
            out['b%d_%s' % (body, key)] = vol[key]
        out['b%d_pos' % body] = pos
    np.savez_compressed(os.path.join(HERE, 'volume_golden.npz'), **out)
    print('volume_golden.npz', os.path.getsize(os.path.join(HERE, 'volume_golden.npz')))
    np.savez_compressed(os.path.join(HERE, 'damid_exp_golden.npz'), **make_damid_exp())
    print('damid_exp_golden.npz', os.path.getsize(os.path.join(HERE, 'damid_exp_golden.npz')))


def make_damid_exp():
    """get_damid_actdist_exp (DamidActivationDistanceStep.py:475-577) on the demo
    population with two nucleus maps (R 5500 and 5200, 100 nm grid) assigned
    alternately through volumes_idx (one entry per structure), it_corr 0/1, after the
    '%6d %.5f %.5f' text round trip.  Only two-copy loci: a batch that mixes copy
    counts makes the reference's np.array(d_sq).sort(axis=1) fail."""
    damid_mod = importlib.import_module('igm.steps.DamidActivationDistanceStep')
    d = np.load(os.path.join(HERE, 'demo_population.npz'))
    ptr, idx = d['copy_ptr'], d['copy_idx']
    copy_index = {h: [int(x) for x in idx[ptr[h]:ptr[h + 1]]] for h in range(len(ptr) - 1)}
    hss = make_golden.DuckHss(d['coordinates'], d['radii'], copy_index, d['chrom'])
    S = d['coordinates'].shape[1]
    rng = np.random.RandomState(31)
    two = np.array([h for h in range(len(ptr) - 1) if len(copy_index[h]) == 2])
    loci = np.sort(rng.choice(two, 300, replace=False)).astype(np.int32)
    pexp = rng.beta(2.0, 5.0, len(loci)).astype(np.float32)
    pexp[:5] = 0.0
    plast = np.where(rng.rand(len(loci)) < 0.5, rng.beta(2.0, 5.0, len(loci)), 0.0).astype(np.float32)
    volumes_idx = [s % 2 for s in range(S)]
    maps = [V.sphere_map(5500.0, 100.0, 3), V.sphere_map(5200.0, 100.0, 3)]
    out = {'loci': loci, 'pexp': pexp, 'plast': plast, 'volumes_idx': np.array(volumes_idx, np.int32)}
    with tempfile.TemporaryDirectory() as tmp:
        prefix = os.path.join(tmp, 'nucleus_')
        for m, vol in enumerate(maps):
            V.write_volume(prefix + str(m) + '.bin', vol)
            for key in ('nvoxel', 'center', 'origin', 'grid', 'matrice'):
                out['m%d_%s' % (m, key)] = vol[key]
        params = np.array([(i, p, q) for i, p, q in zip(loci, pexp, plast)], dtype=np.float32)
        params = [(int(I), pe, pl) for I, pe, pl in params]
        for it_corr in (0, 1):
            rows = damid_mod.get_damid_actdist_exp(params, hss, S, copy_index, it_corr, contact_range=0.05,
                                                   volumes_idx=volumes_idx, volume_prefix=prefix)
            fmt = damid_mod.damid_actdist_fmt_str
            name = os.path.join(tmp, 'rows.tmp')
            with open(name, 'w') as f:
                f.write('\n'.join([fmt % x for x in rows]))
            rt = np.atleast_1d(np.genfromtxt(name, dtype=damid_mod.damid_actdist_shape))
            out['c%d_loc' % it_corr] = rt['loc']
            out['c%d_dist' % it_corr] = rt['dist']
            out['c%d_prob' % it_corr] = rt['prob']
    return out


if __name__ == '__main__':
    main()
