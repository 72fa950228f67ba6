#!/opt/conda/bin/python3.9
"""Golden vectors for the A-step setup and the init steps (8(f)1), from
the REFERENCE run in this container (same environment as make_golden.py: NumPy 1.26,
an alabtools stub that only satisfies imports, the reference imported from
/root/reference).  Run ONLY in the build container:

    /opt/conda/bin/python3.9 tests/golden/make_golden_init.py

Writes tests/golden/init_golden.npz (numerical data only):

  a2_<case>_pairs     ActivationDistanceStep.setup (ActivationDistanceStep.py:111-194)
                      run as is on the demo .hcs: the concatenated '<b>.in.npy' batches
                      (i, j, pwish, plast) float64, for
                        c0  intra 0.02, inter 0.02, no previous actdist
                        c1  intra 0.05, inter 0.02, previous actdist = the G1 rows of
                            sigma 0.2 / it_corr 1 (actdist_golden.npz s0.2_c1_rows_*)
                        c2  intra 1.0, inter disabled (False)
                      The .hcs reader is a duck for alabtools.Contactmatrix: matrix.shape,
                      matrix.coo_generator() = the stored upper triangle in CSR row-major
                      order (the order SURVEY 8 A2 measured), index.chrom.
  terr_s<seed>_R<R>   RandomInit.generate_territories (RandomInit.py:207-240) of the
                      demo index after np.random.seed(seed), float64 (nbead, 3)
  relax_*             RelaxInit.task's model (RelaxInit.py:93-258) for randomInit
                      structures 0 and 1: Steric(1.0), Polymer(index, 2.0, 1.0),
                      Envelope('sphere', 5500, 1.0) -> LammpsModel -> the .data / .lam
                      text, bond list and bond types the reference would hand to LAMMPS
"""
import os
import sys
import glob
import json
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as G  # noqa: E402  (builds the reference environment on import)
import numpy as np  # noqa: E402
import h5py  # noqa: E402
import igm.steps.ActivationDistanceStep  # noqa: E402,F401
import igm.steps.RandomInit  # noqa: E402,F401
from igm.model import Model, Particle  # noqa: E402
from igm.restraints import Polymer, Envelope, Steric  # noqa: E402
from igm.model.kernel import lammps as reflammps  # noqa: E402
from igm.model.kernel.lammps_model import LammpsModel  # noqa: E402

RANDOM_INIT = os.path.join(G.DEMO, 'demo_sample_outputs', 'igm-model.hss.randomInit')
# the module (igm.steps re-exports the class under the same name)
ADS = sys.modules['igm.steps.ActivationDistanceStep']
RI = sys.modules['igm.steps.RandomInit']


class _DuckMatrix(object):
    def __init__(self, indptr, indices, data):
        self.indptr, self.indices, self.data = indptr, indices, data
        self.shape = (len(indptr) - 1, len(indptr) - 1)

    def coo_generator(self):
        for i in range(len(self.indptr) - 1):
            for k in range(self.indptr[i], self.indptr[i + 1]):
                yield i, int(self.indices[k]), self.data[k]


class _DuckContactmatrix(object):
    def __init__(self, path):
        with h5py.File(path, 'r') as g:
            self.matrix = _DuckMatrix(g['matrix/indptr'][()], g['matrix/indices'][()], g['matrix/data'][()])

            class _I(object):
                pass
            self.index = _I()
            self.index.chrom = g['index/chrom'][()]


class _Cfg(dict):
    """keypath get of igm.core.config.Config (config.py:98-127), enough for setup()."""

    def get(self, key, default=None):
        d = self
        for k in key.split('/'):
            if not isinstance(d, dict) or k not in d:
                return default
            d = d[k]
        return d


def run_setup(tmp, intra, inter, last_file):
    ADS.Contactmatrix = _DuckContactmatrix
    step = ADS.ActivationDistanceStep.__new__(ADS.ActivationDistanceStep)
    tdir = tempfile.mkdtemp(dir=tmp)
    hic_rt = {'inter_sigma': inter, 'intra_sigma': intra}
    if last_file is not None:
        hic_rt['actdist_file'] = last_file
    step.cfg = _Cfg({'restraints': {'Hi-C': {'input_matrix': G.HCS, 'batch_size': 1000, 'tmp_dir': tdir}},
                     'runtime': {'Hi-C': hic_rt}, 'parameters': {'tmp_dir': tdir}})
    step.setup()
    parts = [np.load(os.path.join(tdir, '%d.in.npy' % b)) for b in step.argument_list]
    parts = [p.reshape(-1, 4) for p in parts if p.size]
    return np.concatenate(parts).astype(np.float64)


class _TerrIndex(object):
    def __init__(self, chrom_sizes):
        self.chrom_sizes = [int(x) for x in chrom_sizes]

    def __len__(self):
        return int(sum(self.chrom_sizes))


def main():
    out = {}
    tmp = tempfile.mkdtemp()
    g1 = np.load(os.path.join(HERE, 'actdist_golden.npz'))
    last = os.path.join(tmp, 'actdist_prev.hdf5')
    with h5py.File(last, 'w') as h5f:
        for k in ('row', 'col', 'dist', 'prob'):
            h5f.create_dataset(k, data=g1['s0.2_c1_rows_' + k])
    for case, (intra, inter, lf) in {'c0': (0.02, 0.02, None), 'c1': (0.05, 0.02, last),
                                     'c2': (1.0, False, None)}.items():
        out['a2_%s_pairs' % case] = run_setup(tmp, intra, inter, lf)
        out['a2_%s_sigma' % case] = np.array([intra, -1.0 if inter is False else inter])
        print('A2', case, out['a2_%s_pairs' % case].shape, flush=True)

    with h5py.File(G.HSS_T, 'r') as f:
        chrom_sizes = f['index/chrom_sizes'][()]
        radii = f['radii'][()]
        ci_json = json.loads(f['index/copy_index'][()])
        chrom = f['index/chrom'][()]
        copy = f['index/copy'][()]
    for seed in (0, 5):
        for R in (5000.0, 7000.0):
            np.random.seed(seed)
            out['terr_s%d_R%d' % (seed, int(R))] = RI.generate_territories(_TerrIndex(chrom_sizes), R=R)
    print('territories', flush=True)

    with h5py.File(RANDOM_INIT, 'r') as f:
        crd0 = f['coordinates'][()]
    out['relax_crd'] = crd0[:, :2, :].astype(np.float32)
    copy_index = {int(k): [int(x) for x in v] for k, v in ci_json.items()}
    idx = G._Index(copy_index, chrom, copy)
    with open(os.path.join(G.DEMO, 'config_file.json')) as fcfg:
        dcfg = json.load(fcfg)
    opt = dict(dcfg['optimization']['optimizer_options'])
    opt['write'] = opt['mdsteps']
    opt['ev_step'] = 0
    for sid in (0, 1):
        model = Model(uid=sid)
        for i in range(crd0.shape[0]):
            model.addParticle(crd0[i, sid], radii[i], Particle.NORMAL)
        model.addRestraint(Steric(1.0))
        model.addRestraint(Polymer(idx, 2.0, 1.0, contact_probabilities=None))
        model.addRestraint(Envelope('sphere', 5500, 1.0))
        m = LammpsModel(model)
        run_opts = dict(opt)
        run_opts.update(dcfg['optimization']['kernel_opts']['lammps'])
        run_opts.update({'out': os.path.join(tmp, 'o.lammpstrj'), 'data': os.path.join(tmp, 'r.data'),
                         'lmp': os.path.join(tmp, 'r.lam'), 'step_no': 1 + 2})
        reflammps.create_lammps_data(m, run_opts)
        reflammps.create_lammps_script(m, run_opts)
        with open(run_opts['data']) as fd:
            out['relax_data_text_%d' % sid] = np.array(fd.read())
        with open(run_opts['lmp']) as fl:
            out['relax_lam_text_%d' % sid] = np.array(fl.read())
        out['relax_bonds_%d' % sid] = np.array([(b.i.id, b.j.id, b.bond_type.id) for b in m.bonds], np.int32)
        bts = [(bt.style_id, bt.k, bt.r0) for bt in sorted(m.bond_types.values(), key=lambda x: x.id)]
        out['relax_bond_types_%d' % sid] = np.array(bts, np.float64).reshape(-1, 3)
        out['relax_natoms_%d' % sid] = np.int64(len(m.atoms))
        print('relax', sid, len(m.bonds), 'bonds', flush=True)
    np.savez_compressed(os.path.join(HERE, 'init_golden.npz'), **out)
    print('done')


if __name__ == '__main__':
    main()
