"""The assignment steps of configurations D/E and of the polymer-distribution model as
drop-in Steps: DamidActivationDistanceStep, FishAssignmentStep,
SpriteAssignmentStep and PolymerAssignmentStep with the reference's Step contract,
config keys, runtime entries and output files, their per-locus / per-cluster loops on
the GPU kernels of this package (igm_amd.damid, .fish, .sprite, .polymer).

  DamidActivationDistanceStep  igm/steps/DamidActivationDistanceStep.py:125-346
  FishAssignmentStep           igm/steps/FishAssignmentStep.py:82-389
  SpriteAssignmentStep         igm/steps/SpriteAssignmentStep.py:20-263
  PolymerAssignmentStep        igm/steps/PolymerAssignmentStep.py:35-206

Batches are GPU-sized (kernel_opts/hip: one launch covers thousands of loci or
clusters) instead of one process per 100 loci.  The reference draws its SPRITE
representatives, its SPRITE Gibbs picks and its polymer samples from the unseeded
global np.random (D9); here every batch draws from a RandomState seeded by
(restraints/<section>/seed, default 0) and the batch, so a restarted step reproduces
the batches it redoes.
"""
import os
import shutil

import numpy as np

from .steps import (Step, PopulationStore, _kernel, _h5_tree, _write_h5, cget, cset, envelope_section,
                    make_absolute_path, read_damid_rows, rget, sprite_assignment_path)


def _rng(seed, k):
    """the RandomState of batch k of a section seeded `seed` (wrapped to a valid 32-bit
    seed, so any configured seed works)"""
    return np.random.RandomState((int(seed) * 1000003 + int(k)) % 2**32)


def _rotate(last, current, suffix):
    """the previous result file is kept as '<file>.<suffix...>' (the reduce()s' swapfile)"""
    if last is not None and os.path.isfile(last):
        swap = os.path.realpath('.'.join([current] + suffix))
        if os.path.abspath(last) != os.path.abspath(swap):
            shutil.move(last, swap)


def _runtime(cfg, section):
    return cfg.setdefault('runtime', {}).setdefault(section, {})


# ------------------------------------------------------------------ kernels (hip)
def _hip_damid(store, loci, pexp, plast, cfg, device):
    from . import _lib, damid
    shape = rget(cfg, 'model/restraints/envelope/nucleus_shape')
    xyz = np.ascontiguousarray(store.coordinates())
    it_corr = int(cget(cfg, 'runtime/DamID/iter_corr_knob', 1))
    kw = {}
    if shape == 'sphere':
        param = rget(cfg, 'model/restraints/envelope/nucleus_radius')
        cr = rget(cfg, 'restraints/DamID/contact_range', 0.05)
    elif shape == 'ellipsoid':
        param = rget(cfg, 'model/restraints/envelope/nucleus_semiaxes')
        cr = rget(cfg, 'restraints/DamID/contact_range', 0.05)
    elif shape == 'exp_map':  # get_damid_actdist_exp over the per-structure maps (py:270-279)
        env = envelope_section(cfg, range(xyz.shape[1]))
        param, cr = None, rget(cfg, 'restraints/DamID/contact_range', 0.95)
        kw = {'volumes': env['volumes'], 'struct_map': env['struct_map']}
    else:
        raise NotImplementedError('DamID restraint for shape %s has not been implemented yet.' % shape)
    return damid.compute_damid_actdist(xyz, store.radii, store.copy_ptr, store.copy_idx, loci, pexp, plast, it_corr,
                                       float(cr), shape, param, ctx=_lib.context(device), **kw)


def _hip_fish(store, kind, items, tmin, tmax, device):
    from . import _lib, fish
    xyz = np.ascontiguousarray(store.coordinates())
    return fish.assign(xyz, store.copy_ptr, store.copy_idx, kind, items, tmin, tmax, ctx=_lib.context(device))


def _hip_sprite(store, clusters, keep_best, max_chrom, rng, device):
    from . import _lib, sprite
    xyz = np.ascontiguousarray(store.coordinates())
    return sprite.task(xyz, clusters, store.hap_chrom, store.copy_ptr, store.copy_idx, keep_best=keep_best,
                       max_chrom_in_cluster=max_chrom, ctx=_lib.context(device), rng=rng)


def _hip_polymer(store, loci, edges, prob, rng, device):
    from . import _lib, polymer
    xyz = np.ascontiguousarray(store.coordinates())
    return polymer.assign(xyz, edges, prob, rng, loci=loci, ctx=_lib.context(device))[1]


# ------------------------------------------------------------------ DamID
class DamidActivationDistanceStep(Step):
    """Lamina-DamID activation distances (DamidActivationDistanceStep.py:125-346)."""

    def __init__(self, cfg):
        rt = _runtime(cfg, 'DamID')
        if 'sigma_list' not in rt:
            rt['sigma_list'] = list(cfg['restraints']['DamID']['sigma_list'])
        if 'sigma' not in rt:
            rt['sigma'] = rt['sigma_list'].pop(0)
        if 'iter_corr_knob' not in rt:  # D1: optimization/iter_corr_knob is not in the schema, default 1
            rt['iter_corr_knob'] = cget(cfg, 'optimization/iter_corr_knob', 1)
        super(DamidActivationDistanceStep, self).__init__(cfg)

    def name(self):
        return 'DamidActivationDistanceStep (sigma={:.2f}%, iter={:s})'.format(
            cget(self.cfg, 'runtime/DamID/sigma', -1) * 100.0, str(cget(self.cfg, 'runtime/opt_iter', 'N/A')))

    def _dir(self):
        d = make_absolute_path(cget(self.cfg, 'restraints/DamID/tmp_dir', 'damid_actdist'),
                               cget(self.cfg, 'parameters/tmp_dir', 'tmp'))
        os.makedirs(d, exist_ok=True)
        return d

    def setup(self):
        from . import damid
        sigma = cget(self.cfg, 'runtime/DamID/sigma')
        profile = np.loadtxt(self.cfg['restraints']['DamID']['input_profile'], dtype='float32')
        last = cget(self.cfg, 'runtime/DamID/damid_actdist_file', None)
        last_rows = read_damid_rows(last) if last is not None and os.path.isfile(last) else None
        loci, pexp, plast = damid.select_loci(profile, sigma, last_rows)  # py:185-217
        bs = int(cget(self.cfg, 'optimization/kernel_opts/hip/locus_batch', 1 << 20))
        self.argument_list = []
        for b, q0 in enumerate(range(0, max(len(loci), 1), bs)):
            fn = os.path.join(self.tmp_dir, '%s.%d.damid.in.npz' % (self.uid, b))
            np.savez(fn, loci=loci[q0:q0 + bs], pexp=pexp[q0:q0 + bs], plast=plast[q0:q0 + bs])
            self.argument_list.append({'batch': b, 'in': fn,
                                       'out': os.path.join(self.tmp_dir, '%s.%d.damid.out.npy' % (self.uid, b))})
        self.tmp_extensions = ['.npz', '.npy']

    def task(self, batch, device):
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        d = np.load(batch['in'])
        rows = _kernel(self.cfg, 'damid')(store, d['loci'], d['pexp'], d['plast'], self.cfg, device)
        tmp = batch['out'] + '.part.npy'
        np.save(tmp, rows)
        os.replace(tmp, batch['out'])

    def reduce(self):
        """concatenate -> damid_actdist.hdf5 {loc, dist, prob}; the previous file kept as
        damid_actdist.hdf5.DamID_<sigma>.iter_<n> (py:289-345)"""
        from ._lib import damid_row_dtype
        rows = np.concatenate([np.load(b['out']) for b in self.argument_list]) if self.argument_list else \
            np.zeros(0, damid_row_dtype)
        out = os.path.join(self._dir(), 'damid_actdist.hdf5')
        suffix = ['DamID_{:.4f}'.format(cget(self.cfg, 'runtime/DamID/sigma'))]
        if 'opt_iter' in self.cfg['runtime']:
            suffix.append('iter_{}'.format(self.cfg['runtime']['opt_iter'] - 1))
        _rotate(cget(self.cfg, 'runtime/DamID/damid_actdist_file', None), out, suffix)
        _write_h5(out, {'loc': np.ascontiguousarray(rows['loc'], np.int32),
                        'dist': np.ascontiguousarray(rows['dist'], np.float32),
                        'prob': np.ascontiguousarray(rows['prob'], np.float32)})
        cset(self.cfg, 'runtime/DamID/damid_actdist_file', out)

    def skip(self):
        cset(self.cfg, 'runtime/DamID/damid_actdist_file', os.path.join(self._dir(), 'damid_actdist.hdf5'))


# ------------------------------------------------------------------ FISH
class FishAssignmentStep(Step):
    """FISH target assignment (FishAssignmentStep.py:82-389)."""

    KEYS = ('pairs', 'pair_min', 'pair_max', 'probes', 'radial_min', 'radial_max')

    def __init__(self, cfg):
        rt = _runtime(cfg, 'FISH')
        if 'tol_list' not in rt:
            rt['tol_list'] = list(cfg['restraints']['FISH']['tol_list'])
        if 'tol' not in rt:
            rt['tol'] = rt['tol_list'].pop(0)
        super(FishAssignmentStep, self).__init__(cfg)

    def name(self):
        return 'FishAssignmentStep (tol={:.2f}, iter={:s})'.format(
            cget(self.cfg, 'runtime/FISH/tol', -1), str(cget(self.cfg, 'runtime/opt_iter', 'N/A')))

    def _dir(self):
        d = self.cfg['restraints']['FISH'].get('fish_dir', 'fish_actdist')  # set_tmp_path (py:376-387)
        if not os.path.isabs(d):
            d = os.path.abspath(os.path.join(cget(self.cfg, 'parameters/tmp_dir', 'tmp'), d))
        os.makedirs(d, exist_ok=True)
        return d

    def _input(self):
        return _h5_tree(self.cfg['restraints']['FISH']['input_fish'])

    def setup(self):
        """batches of pairs, then of probes (py:129-153); each item carries the row of
        the input its targets come from: the first row equal to the pair (py:203) and the
        one row equal to the probe, which must be unique (py:230-235)"""
        f = self._input()
        bs = int(cget(self.cfg, 'optimization/kernel_opts/hip/fish_batch', 1 << 20))
        self.argument_list = []
        for kind, key in (('pair', 'pairs'), ('probe', 'probes')):
            if key not in f:
                continue
            items = np.asarray(f[key])
            if kind == 'pair':
                _, idx, inv = np.unique(items, axis=0, return_index=True, return_inverse=True)
                first = idx[np.ravel(inv)]
            else:
                u, cnt = np.unique(items, return_counts=True)
                if np.any(cnt != 1):
                    raise ValueError('Cannot find probe: %s' % u[cnt != 1][0])
                first = np.arange(len(items))
            for q0 in range(0, len(items), bs):
                b = len(self.argument_list)
                fn = os.path.join(self.tmp_dir, '%s.%d.fish.in.npz' % (self.uid, b))
                np.savez(fn, items=items[q0:q0 + bs], first=first[q0:q0 + bs])
                self.argument_list.append({'batch': b, 'kind': kind, 'in': fn,
                                           'out': os.path.join(self.tmp_dir, '%s.%d.fish.out.npz' % (self.uid, b))})
        self.tmp_extensions = ['.npz']

    def task(self, batch, device):
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        f = self._input()
        d = np.load(batch['in'])
        pre = 'pair' if batch['kind'] == 'pair' else 'radial'
        tmin = np.asarray(f[pre + '_min'])[d['first']] if pre + '_min' in f else None
        tmax = np.asarray(f[pre + '_max'])[d['first']] if pre + '_max' in f else None
        omin, omax = _kernel(self.cfg, 'fish')(store, batch['kind'], d['items'], tmin, tmax, device)
        res = {'first': d['first']}
        if omin is not None:
            res['min'] = omin
        if omax is not None:
            res['max'] = omax
        tmp = batch['out'] + '.part.npz'
        np.savez(tmp, **res)
        os.replace(tmp, batch['out'])

    def reduce(self):
        """fish_assignment.h5 with the input's pairs/probes and the assigned (n, S)
        targets of every key the input has (py:259-362)"""
        f = self._input()
        S = PopulationStore(self.cfg['optimization']['structure_output']).nstruct
        out = {}
        for key, pre in (('pairs', 'pair'), ('probes', 'radial')):
            if key not in f:
                continue
            out[key] = np.ascontiguousarray(f[key], np.int32)
            for kk in ('min', 'max'):
                if pre + '_' + kk in f:
                    out[pre + '_' + kk] = np.zeros((len(f[key]), S), np.float32)
        for b in self.argument_list:
            r = np.load(b['out'])
            pre = 'pair' if b['kind'] == 'pair' else 'radial'
            for kk in ('min', 'max'):
                if kk in r:
                    out[pre + '_' + kk][r['first']] = r[kk]
        path = os.path.join(self._dir(), 'fish_assignment.h5')
        suffix = ['tol_{:.4f}'.format(cget(self.cfg, 'runtime/FISH/tol'))]
        if 'opt_iter' in self.cfg['runtime']:
            suffix.append('iter_{}'.format(self.cfg['runtime']['opt_iter']))
        _rotate(cget(self.cfg, 'runtime/FISH/fish_assignment_file', None), path, suffix)
        _write_h5(path, out)
        cset(self.cfg, 'runtime/FISH/fish_assignment_file', path)

    def skip(self):
        cset(self.cfg, 'runtime/FISH/fish_assignment_file', os.path.join(self._dir(), 'fish_assignment.h5'))


# ------------------------------------------------------------------ SPRITE
class SpriteAssignmentStep(Step):
    """SPRITE cluster assignment (SpriteAssignmentStep.py:20-263): Rg^2 keep_best on the
    GPU, the sequential Gibbs assignment with the occupancy penalty on the host."""

    def __init__(self, cfg):
        rt = _runtime(cfg, 'sprite')
        if 'volume_fraction_list' not in rt:
            rt['volume_fraction_list'] = list(cfg['restraints']['sprite']['volume_fraction_list'])
        if 'volume_fraction' not in rt:
            rt['volume_fraction'] = rt['volume_fraction_list'].pop(0)
        super(SpriteAssignmentStep, self).__init__(cfg)

    def name(self):
        return 'SpriteAssignmentStep (volume_fraction={:.1f}%, iter={:s})'.format(
            cget(self.cfg, 'runtime/sprite/volume_fraction', -1), str(cget(self.cfg, 'runtime/opt_iter', 'N/A')))

    def _clusters(self):
        c = _h5_tree(self.cfg['restraints']['sprite']['clusters'])
        return np.asarray(c['indptr'], np.int64), np.asarray(c['data'])

    def setup(self):
        indptr, _ = self._clusters()
        self.n_clusters = len(indptr) - 1
        bs = int(cget(self.cfg, 'optimization/kernel_opts/hip/cluster_batch', 1 << 20))
        self.argument_list = [{'batch': b, 'c0': c0, 'c1': min(c0 + bs, self.n_clusters),
                               'out': os.path.join(self.tmp_dir, '%s.%d.sprite.npz' % (self.uid, b))}
                              for b, c0 in enumerate(range(0, self.n_clusters, bs))]
        self.tmp_extensions = ['.npz']

    def task(self, batch, device):
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        indptr, data = self._clusters()
        clusters = [data[indptr[c]:indptr[c + 1]] for c in range(batch['c0'], batch['c1'])]
        kb = int(rget(self.cfg, 'restraints/sprite/keep_best', 50))
        rng = _rng(cget(self.cfg, 'restraints/sprite/seed', 0), batch['batch'])
        idx, val, sel = _kernel(self.cfg, 'sprite')(store, clusters, kb,
                                                    int(rget(self.cfg, 'restraints/sprite/max_chrom_in_cluster', 6)),
                                                    rng, device)
        sizes = np.array([s.shape[1] for s in sel], np.int64)
        tmp = batch['out'] + '.part.npz'
        np.savez(tmp, idx=np.asarray(idx, np.int32).reshape(len(clusters), kb),
                 val=np.asarray(val, np.float32).reshape(len(clusters), kb), sizes=sizes,
                 sel=np.concatenate([np.asarray(s, np.int32).ravel() for s in sel]) if sel else np.zeros(0, np.int32))
        os.replace(tmp, batch['out'])

    def reduce(self):
        """Gibbs assignment over the clusters in the reference's order (its batches of
        restraints/sprite/batch_size in a random permutation, py:166-262) ->
        assignment.h5 {assignment, selected, indptr}"""
        from . import sprite
        S = PopulationStore(self.cfg['optimization']['structure_output']).nstruct
        indptr, _ = self._clusters()
        kb = int(rget(self.cfg, 'restraints/sprite/keep_best', 50))
        idx, val, sel = [], [], []
        for b in self.argument_list:
            r = np.load(b['out'])
            o = 0
            for q in range(b['c1'] - b['c0']):
                n = int(r['sizes'][q])
                idx.append(r['idx'][q])
                val.append(r['val'][q])
                sel.append(r['sel'][o:o + kb * n].reshape(kb, n))
                o += kb * n
        rng = _rng(cget(self.cfg, 'restraints/sprite/seed', 0), 999983)
        rbs = int(cget(self.cfg, 'restraints/sprite/batch_size', 10))  # SpriteAssignmentStep.py:71,171
        nb = -(-self.n_clusters // rbs)
        order = [c for b in rng.permutation(nb) for c in range(b * rbs, min((b + 1) * rbs, self.n_clusters))]
        assignment, chosen = sprite.assign(val, idx, sel, S, kT=float(rget(self.cfg, 'restraints/sprite/radius_kt')),
                                           order=order, rng=rng)
        selected = np.concatenate(chosen).astype(np.int32) if chosen else np.zeros(0, np.int32)
        path = sprite_assignment_path(self.cfg)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        _write_h5(path, {'assignment': assignment.astype(np.int32), 'selected': selected,
                         'indptr': indptr})


# ------------------------------------------------------------------ polymer distances
class PolymerAssignmentStep(Step):
    """Consecutive-bead distance targets (PolymerAssignmentStep.py:35-206)."""

    def name(self):
        return 'PolymerAssignmentStep (iter={:s})'.format(str(cget(self.cfg, 'runtime/opt_iter', 'N/A')))

    def _dir(self):
        d = _runtime(self.cfg, 'polymer').get('tmp_dir', 'poly_actdist')  # set_tmp_path (py:193-206)
        if not os.path.isabs(d):
            d = os.path.abspath(os.path.join(cget(self.cfg, 'parameters/tmp_dir', 'tmp'), d))
        os.makedirs(d, exist_ok=True)
        return d

    def setup(self):
        from . import polymer
        nbead = PopulationStore(self.cfg['optimization']['structure_output']).nbead
        bs = int(cget(self.cfg, 'optimization/kernel_opts/hip/locus_batch', polymer.BATCH_SIZE))
        self.argument_list = [{'batch': b, 'loci': list(r),
                               'out': os.path.join(self.tmp_dir, '%s.%d.polymer.npy' % (self.uid, b))}
                              for b, r in polymer.batches(nbead, bs)]
        self.tmp_extensions = ['.npy']

    def task(self, batch, device):
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        d = _h5_tree(self.cfg['restraints']['polymer']['polymer_file'])
        rng = _rng(cget(self.cfg, 'restraints/polymer/seed', 0), batch['batch'])
        nn = _kernel(self.cfg, 'polymer')(store, np.asarray(batch['loci'], np.int32), d['bin_edges'],
                                          d['probability'], rng, device)
        tmp = batch['out'] + '.part.npy'
        np.save(tmp, np.asarray(nn, np.float32))
        os.replace(tmp, batch['out'])

    def reduce(self):
        """<tmp>/<restraints/polymer/assignment_file> {loci i4, nn_dist f4 (nloci, S)}"""
        loci = np.concatenate([np.asarray(b['loci'], np.int32) for b in self.argument_list])
        nn = np.concatenate([np.load(b['out']) for b in self.argument_list])
        path = os.path.join(self._dir(), self.cfg['restraints']['polymer']['assignment_file'])
        suffix = ['iter_{}'.format(self.cfg['runtime']['opt_iter'])] if 'opt_iter' in self.cfg['runtime'] else []
        _rotate(cget(self.cfg, 'runtime/polymer/assignment_file', None), path, suffix)
        _write_h5(path, {'loci': loci, 'nn_dist': nn})
        cset(self.cfg, 'runtime/polymer/assignment_file', path)

    def skip(self):
        cset(self.cfg, 'runtime/polymer/assignment_file',
             os.path.join(self._dir(), self.cfg['restraints']['polymer']['assignment_file']))


KERNELS_HIP = {'damid': _hip_damid, 'fish': _hip_fish, 'sprite': _hip_sprite, 'polymer': _hip_polymer}
