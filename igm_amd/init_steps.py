"""Population start-up as drop-in Steps (bin/igm-run:63-82):

  RandomInit  igm/steps/RandomInit.py:19-171 -- chromosome territories per structure
              (generate_territories, :207-240) written into the population; the
              intermediate copy '<structure_output>.randomInit'.
  RelaxInit   igm/steps/RelaxInit.py:21-325 -- the relax M-step (steric + polymer or
              PolymerDistrib + nucleus envelope / map) of every structure on the
              batched engine; the intermediate copy '<structure_output>.relaxInit.hss'.

The reference draws the territories from the unseeded global np.random (D9); here
structure s draws from RandomState(model/init_seed (default 0) * 1000003 + s), so a
restarted batch reproduces its structures, and the draw order inside a structure is
the reference's (igm_amd.init.generate_territories).
"""
import os
import shutil

import numpy as np

from .steps import PopulationStore, Step, _kernel, cget, rget


def _batches(S, bs):
    return [list(range(s0, min(s0 + bs, S))) for s0 in range(0, S, bs)]


class RandomInit(Step):

    def setup(self):
        S = int(self.cfg['model']['population_size'])
        bs = int(cget(self.cfg, 'optimization/kernel_opts/hip/batch_size', 1000))
        self.argument_list = [{'batch': b, 'sids': sids} for b, sids in enumerate(_batches(S, bs))]

    def task(self, batch, device):
        """generate_territories for the batch's structures straight into the population
        file's coordinates (disjoint columns per batch: batches run concurrently)"""
        from . import init
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        R = float(rget(self.cfg, 'model/init_radius'))
        seed = int(cget(self.cfg, 'model/init_seed', 0))
        crd = store.coordinates('r+')
        for sid in batch['sids']:
            rng = np.random.RandomState((seed * 1000003 + sid) % 2**32)  # (a valid RandomState seed for any init_seed)
            crd[:, sid, :] = init.generate_territories(store.chrom_sizes, R, rng).astype(np.float32)
        crd.flush()
        del crd

    def reduce(self):
        """the population's violation is NaN (no restraints yet, RandomInit.py:145-148)"""
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        store.write_violation(float('nan'))
        if rget(self.cfg, 'optimization/keep_intermediate_structures'):
            shutil.copyfile(store.path + ('' if store.is_hss else '.npy'),
                            self.cfg['optimization']['structure_output'] + '.randomInit')


def _hip_relax(store, sids, cfg, device):
    """RelaxInit.task for a batch (RelaxInit.py:93-258): (xyz (S, nbead, 3), info)."""
    from . import _lib, init
    from .steps import batch_coordinates, envelope_section
    ctx = _lib.context(device)
    rs = cfg['model']['restraints']
    if 'polymer' not in rs:
        raise NotImplementedError('RelaxInit with PolymerDistrib restraints is not implemented on the hip kernel')
    kw = {}
    if rget(cfg, 'model/restraints/envelope/nucleus_shape') == 'exp_map':
        env = envelope_section(cfg, sids)
        kw = {'volumes': env['volumes'], 'volume_struct_map': env['struct_map']}
    return init.relax_population(cfg, batch_coordinates(store, sids), store.radii, store.chrom, store.copy, sids,
                                 ctx=ctx, **kw)


class RelaxInit(Step):

    def setup(self):
        S = int(self.cfg['model']['population_size'])
        bs = int(cget(self.cfg, 'optimization/kernel_opts/hip/batch_size', 1000))
        self.argument_list = [{'batch': b, 'sids': sids,
                               'out': os.path.join(self.tmp_dir, '%s.%d.relax.npy' % (self.uid, b))}
                              for b, sids in enumerate(_batches(S, bs))]
        self.tmp_extensions = ['.npy']

    def task(self, batch, device):
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        xo, _ = _kernel(self.cfg, 'relax')(store, np.asarray(batch['sids']), self.cfg, device)
        tmp = batch['out'] + '.part.npy'
        np.save(tmp, np.asarray(xo, np.float32))
        os.replace(tmp, batch['out'])

    def reduce(self):
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        crd = store.coordinates('r+')
        for b in self.argument_list:
            x = np.load(b['out'])
            for q, sid in enumerate(b['sids']):
                crd[:, sid, :] = x[q]
        crd.flush()
        del crd
        if rget(self.cfg, 'optimization/keep_intermediate_structures'):
            shutil.copyfile(store.path + ('' if store.is_hss else '.npy'),
                            self.cfg['optimization']['structure_output'] + '.relaxInit.hss')


KERNELS_HIP = {'relax': _hip_relax}
