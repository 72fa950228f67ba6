#!/opt/conda/bin/python3.9
"""Golden vectors for the polymer-distance A-step and its M-step restraint, produced by
running the REFERENCE code in this container (build container only, like make_golden.py):

    /opt/conda/bin/python3.9 tests/golden/make_golden_polymer.py

  polymer_golden.npz
    PolymerAssignmentStep.task (steps/PolymerAssignmentStep.py:84-129) over every
    (i, i+1) locus of the demo population, batched as setup() does (:55-79), after
    np.random.seed(seed): the sampled, sorted distance of each structure's rank
    (nn_dist, the task's npz), for two distributions:
      'a'  float64 ascending bin edges, smooth probabilities
      'b'  float32 edges in shuffled order with zero-probability bins
    and PolymerDistrib._apply (restraints/polymer_bis.py:50-90) for structures
    0, 7 and 42 of case 'a': the (i, j, d, k, lower/upper) of every force added, in order.

The reference reads the population through alabtools.HssFile and the distribution
through h5py; both are given the committed demo coordinates here.  Only the numbers
are written.
"""
import importlib
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402  (reference environment: stub alabtools)
import h5py  # noqa: E402
import numpy as np  # noqa: E402

poly_step = importlib.import_module('igm.steps.PolymerAssignmentStep')
poly_bis = importlib.import_module('igm.restraints.polymer_bis')
from igm.model import Model  # noqa: E402
from igm.model.forces import HarmonicLowerBound  # noqa: E402


class Cfg(dict):
    def get(self, key, default=None):
        d = self
        for k in key.split('/'):
            if not isinstance(d, dict) or k not in d:
                return default
            d = d[k]
        return d


class Hss(object):
    def __init__(self, crd, copy_index, chrom):
        self.crd = crd
        self.index = make_golden._Index(copy_index, chrom)

    def __getitem__(self, key):
        assert key == 'coordinates'
        return self.crd


def run_case(crd, hss, edges, prob, seed, tmp):
    pfile = os.path.join(tmp, 'polymer_%d.h5' % seed)
    with h5py.File(pfile, 'w') as f:
        f.create_dataset('bin_edges', data=edges)
        f.create_dataset('probability', data=prob)
    poly_step.HssFile = lambda *a, **k: hss
    cfg = Cfg({'optimization': {'structure_output': 'unused.hss'},
               'restraints': {'polymer': {'polymer_file': pfile}}})
    # setup()'s batches of 1000 loci over range(0, nbead - 1)
    batches = []
    for i in range(0, crd.shape[0] - 1, 1000):
        stop = crd.shape[0] - 1 if i + 1000 > crd.shape[0] else i + 1000
        batches.append((len(batches), range(i, stop)))
    np.random.seed(seed)
    out = []
    for b in batches:
        poly_step.PolymerAssignmentStep.task(b, cfg, tmp)
        out.append(np.load(os.path.join(tmp, 'tmp.%d.polymer.npz' % b[0]))['nn_dist'])
    loci = np.concatenate([np.asarray(list(r), np.int32) for _, r in batches])
    return loci, np.concatenate(out).astype(np.float32)


def main():
    d = np.load(os.path.join(HERE, 'demo_population.npz'))
    crd = d['coordinates']  # (nbead, S, 3) float32, the .hss layout
    chrom = d['chrom']
    ptr, idx = d['copy_ptr'], d['copy_idx']
    copy_index = {h: [int(x) for x in idx[ptr[h]:ptr[h + 1]]] for h in range(len(ptr) - 1)}
    hss = Hss(crd, copy_index, chrom)
    g = {}
    rng = np.random.RandomState(21)
    ea = np.linspace(300.0, 900.0, 61)
    pa = np.exp(-0.5 * ((ea - 560.0) / 90.0) ** 2)
    pa = pa / pa.sum()
    eb = rng.permutation(np.linspace(250.0, 1000.0, 40)).astype(np.float32)
    pb = rng.gamma(2.0, 1.0, 40)
    pb[rng.choice(40, 8, replace=False)] = 0.0
    pb = pb / pb.sum()
    with tempfile.TemporaryDirectory() as tmp:
        for tag, e, p, seed in (('a', ea, pa, 5), ('b', eb, pb, 6)):
            loci, nn = run_case(crd, hss, e, p, seed, tmp)
            g[tag + '_edges'], g[tag + '_prob'], g[tag + '_seed'] = e, p, np.int64(seed)
            g[tag + '_loci'], g[tag + '_nn_dist'] = loci, nn
        # PolymerDistrib._apply on case 'a'
        afile = os.path.join(tmp, 'assign.h5')
        with h5py.File(afile, 'w') as f:
            f.create_dataset('loci', data=g['a_loci'], dtype='i4')
            f.create_dataset('nn_dist', data=g['a_nn_dist'], dtype='f4')
        tol, ck = 25.0, 2.0
        for sid in (0, 7, 42):
            pd = poly_bis.PolymerDistrib(afile, sid, make_golden._Index(copy_index, chrom), tolerance=tol, kspring=ck)
            m = Model()
            pd._apply(m)
            fs = [m.forces[k] for k in pd.forceID]
            g['bonds_%d_i' % sid] = np.array([f.i for f in fs], np.int64)
            g['bonds_%d_j' % sid] = np.array([f.j for f in fs], np.int64)
            g['bonds_%d_d' % sid] = np.array([f.d for f in fs], np.float64)
            g['bonds_%d_k' % sid] = np.array([f.k for f in fs], np.float64)
            g['bonds_%d_lower' % sid] = np.array([isinstance(f, HarmonicLowerBound) for f in fs])
        g['tolerance'], g['kspring'] = np.float64(tol), np.float64(ck)
    np.savez_compressed(os.path.join(HERE, 'polymer_golden.npz'), **g)
    print('polymer_golden.npz:', {k: v.shape for k, v in g.items()})


if __name__ == '__main__':
    main()
