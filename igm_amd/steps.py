"""Drop-in Step layer for igm-run: ActivationDistanceStep and
ModelingStep with the reference's Step plugin contract, run by a per-GPU batch
scheduler instead of ipyparallel, restartable at batch granularity.

  StepDB          igm/core/job_tracking.py:9-123 -- the same sqlite file and schema
                  (table `steps`: uid, name, cfg, time, status, data), so igm-run's
                  restart logic reads our records unchanged.
  Step            igm/core/step.py:23-328 -- the same lifecycle and status rows
                  (entry, setup, map, mapped, reduced, cleanup, completed, failed),
                  uid = md5('<name>:<step_no>'), a completed step is skipped, a
                  failure is recorded with its traceback and re-raised.
  BatchScheduler  replaces Controller.map (parallel/ipyparallel_controller.py:61-109):
                  argument_list entries are BATCHES (thousands of structures or pairs
                  per GPU call, not one structure per process); one worker thread per
                  GPU, each with its own igm_ctx; a batch's completion is recorded
                  (<uid>.batch<k>.done, written by atomic rename after the batch's
                  outputs) in place of the per-structure '<uid>.<sid>.ready' files
                  (ModelingStep.py:178-183), and a restarted map skips every batch
                  that has one.
  ActivationDistanceStep / ModelingStep
                  the A-step (ActivationDistanceStep.py:42-298) and M-step
                  (ModelingStep.py:105-783) on the GPU kernels of this package.

Storage.  The population, the Hi-C input and the A-step rows are the reference's own
HDF5 files, read and written by the native reader/writer of this package (igm_amd.h5
over csrc/h5io.cpp; no libhdf5 in the product path, the files are checked with h5py in
tests/test_h5py_pin.py): `<structure_output>` ending in
.hss is an alabtools HssFile (coordinates (nbead, nstruct, 3) float32 bead-major,
index, radii, summary), `input_matrix` a .hcs Contactmatrix, `actdist_file` an
actdist.hdf5 {row, col, dist, prob}.  Files this package writes are contiguous, so
the coordinates are memory-mapped and the M-step's reduce updates them in place.
Other extensions keep the same arrays in numpy files (`<out>.npy` + `<out>.index.npz`,
`.npz` rows / CSR).  The kernels behind the steps are looked up by name in KERNELS
(cfg optimization/kernel, default 'hip'); the product registers only the GPU kernels.
"""
import hashlib
import json
import os
import sqlite3
import threading
import time
import traceback
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import model as M
from ._lib import pair_dtype, row_dtype


# ------------------------------------------------------------------ config helpers
def cget(cfg, key, default=None):
    """Config.get keypath semantics (core/config.py:98-127) on a plain dict."""
    d = cfg
    for k in key.split('/'):
        if not isinstance(d, dict) or k not in d:
            return default
        d = d[k]
    return d


def cset(cfg, key, value):
    ks = key.split('/')
    d = cfg
    for k in ks[:-1]:
        d = d.setdefault(k, {})
    d[ks[-1]] = value


def _json_default(o):
    if isinstance(o, np.generic):
        return o.item()
    if isinstance(o, np.ndarray):
        return o.tolist()
    raise TypeError(type(o))


# ------------------------------------------------------------------ StepDB
class StepDB(object):
    """igm.core.job_tracking.StepDB: sqlite table `steps`, json columns cfg / data."""
    SCHEMA = [('uid', 'TEXT'), ('name', 'TEXT'), ('cfg', 'TEXT'), ('time', 'INT'), ('status', 'TEXT'),
              ('data', 'TEXT')]
    JSONCOLS = ('cfg', 'data')
    COLUMNS = [x[0] for x in SCHEMA]

    def __init__(self, cfg):
        self.db = cfg if isinstance(cfg, str) else cget(cfg, 'parameters/step_db', None)
        if self.db and not os.path.isfile(self.db):
            with sqlite3.connect(self.db) as conn:
                conn.execute('CREATE TABLE steps (' + ','.join(' '.join(x) for x in self.SCHEMA) + ')')
        elif self.db:
            with sqlite3.connect(self.db) as conn:
                s = conn.execute('PRAGMA table_info(steps)').fetchall()
            for i, (n, t) in enumerate(self.SCHEMA):
                if i >= len(s) or s[i][1] != n or s[i][2] != t:
                    raise AssertionError('Invalid database file %s (column %d)' % (self.db, i))

    def record(self, **kw):
        if not self.db:
            return
        row = []
        for c, _ in self.SCHEMA:
            if c == 'time':
                row.append(kw.get('time', time.time()))
            elif c in self.JSONCOLS:
                row.append(json.dumps(kw.get(c, None), default=_json_default))
            else:
                row.append(kw.get(c, ''))
        with sqlite3.connect(self.db) as conn:
            conn.execute('INSERT INTO steps (%s) VALUES (%s)' % (','.join(self.COLUMNS), ','.join('?' * len(row))),
                         tuple(row))

    def get_history(self, uid=None):
        if not self.db:
            return []
        with sqlite3.connect(self.db) as conn:
            if uid is None:
                r = conn.execute('SELECT * FROM steps ORDER BY time').fetchall()
            else:
                r = conn.execute('SELECT * FROM steps WHERE uid=? ORDER BY time', (uid,)).fetchall()
        return [{c: (json.loads(v) if c in self.JSONCOLS else v) for c, v in zip(self.COLUMNS, x)} for x in r]


# ------------------------------------------------------------------ scheduler
class BatchScheduler(object):
    """Per-GPU batch scheduler: map(task, batches) runs task(batch, device) for every
    batch not yet recorded as done, one worker thread per device (each thread owns
    its device's igm_ctx: _lib.context(device)).  A batch is done once task returned
    and its record was renamed into place; the first failing batch stops the map and
    re-raises (the reference's remote-failure abort, ipyparallel_controller.py:92-97),
    after the batches already running have finished and been recorded."""

    def __init__(self, devices=(0,), record_dir='.', uid='step', clean_restart=False):
        self.devices = list(devices) or [0]
        self.record_dir = record_dir
        self.uid = uid
        if clean_restart:
            for f in os.listdir(record_dir):
                if f.startswith(uid + '.batch') and f.endswith('.done'):
                    os.remove(os.path.join(record_dir, f))

    def record_path(self, k):
        return os.path.join(self.record_dir, '%s.batch%d.done' % (self.uid, k))

    def done(self, k):
        return os.path.isfile(self.record_path(k))

    def _record(self, k, info):
        tmp = self.record_path(k) + '.tmp'
        with open(tmp, 'w') as f:
            json.dump(info, f, default=_json_default)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self.record_path(k))

    def map(self, task, batches):
        pending = [k for k in range(len(batches)) if not self.done(k)]
        lock = threading.Lock()
        queue = list(pending)
        errors = []
        ran = []

        def worker(dev):
            while True:
                with lock:
                    if errors or not queue:
                        return
                    k = queue.pop(0)
                t0 = time.time()
                try:
                    task(batches[k], dev)
                except BaseException as e:  # noqa: B902 -- recorded, then re-raised by map()
                    with lock:
                        errors.append((k, e, traceback.format_exc()))
                    return
                self._record(k, {'batch': k, 'device': dev, 'seconds': time.time() - t0})
                with lock:
                    ran.append(k)

        with ThreadPoolExecutor(max_workers=len(self.devices)) as ex:
            list(ex.map(worker, self.devices))
        if errors:
            k, e, tb = min(errors, key=lambda x: x[0])
            raise RuntimeError('batch %d failed: %s\n%s' % (k, e, tb))
        return sorted(ran)


# ------------------------------------------------------------------ Step
class Step(object):
    """igm.core.step.Step with the same run() semantics; argument_list holds batches."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.tmp_extensions = []
        workdir = cget(cfg, 'parameters/workdir', '.')
        tmp = cget(cfg, 'parameters/tmp_dir', 'tmp/')
        self.tmp_dir = tmp if os.path.isabs(tmp) else os.path.join(workdir, tmp)
        self.keep_temporary_files = True
        os.makedirs(self.tmp_dir, exist_ok=True)
        rt = cfg.setdefault('runtime', {})
        if 'current_iteration_name' not in rt:
            rt['current_iteration_name'] = self.name()
        if rt.get('step_no') is None:
            rt['step_no'] = -1
        rt['step_no'] += 1
        self._db = StepDB(cfg)
        self.uid = hashlib.md5('{:s}:{:d}'.format(self.name(), rt['step_no']).encode()).hexdigest()
        rt['step_hash'] = self.uid
        self.argument_list = []
        self.mapped_batches = []

    # overridables
    def setup(self):
        self.argument_list = []

    def before_map(self):
        return

    def task(self, batch, device):
        raise NotImplementedError

    def before_reduce(self):
        return

    def reduce(self):
        return

    def cleanup(self):
        if not self.keep_temporary_files:
            for f in os.listdir(self.tmp_dir):
                if os.path.splitext(f)[1] in self.tmp_extensions:
                    os.remove(os.path.join(self.tmp_dir, f))

    def skip(self):
        return None

    def name(self):
        return self.__class__.__name__

    def scheduler(self):
        hip = cget(self.cfg, 'optimization/kernel_opts/hip', {}) or {}
        return BatchScheduler(hip.get('devices', [0]), self.tmp_dir, self.uid,
                              clean_restart=bool(cget(self.cfg, 'optimization/clean_restart', False)))

    def run(self):
        """core/step.py:226-322, DO NOT OVERLOAD."""
        dbdata = {'uid': self.uid, 'name': self.name(), 'cfg': self.cfg}
        past = {x['status']: x['cfg'] for x in self._db.get_history(self.uid)}
        if 'completed' in past:
            self.cfg['runtime'].update(past['completed']['runtime'])
            self.skip()
            return
        try:
            dbdata['status'] = 'entry'
            self._db.record(**dbdata)
            self.setup()
            dbdata['status'] = 'setup'
            self._db.record(**dbdata)
            if 'mapped' not in past:
                self.before_map()
                dbdata['status'] = 'map'
                self._db.record(**dbdata)
                self.mapped_batches = self.scheduler().map(self.task, self.argument_list)
                dbdata['status'] = 'mapped'
                self._db.record(**dbdata)
            else:
                self.cfg['runtime'].update(past['mapped']['runtime'])
            if 'reduced' not in past:
                self.before_reduce()
                self.reduce()
                dbdata['status'] = 'reduced'
                self._db.record(**dbdata)
            else:
                self.cfg['runtime'].update(past['reduced']['runtime'])
            if 'cleanup' not in past:
                self.cleanup()
                dbdata['status'] = 'cleanup'
                self._db.record(**dbdata)
            else:
                self.cfg['runtime'].update(past['cleanup']['runtime'])
            dbdata['status'] = 'completed'
            self.cfg['runtime'].pop('step_hash', None)
            self._db.record(**dbdata)
        except BaseException:
            dbdata['status'] = 'failed'
            dbdata['data'] = {'exception': traceback.format_exc()}
            self._db.record(**dbdata)
            raise


# ------------------------------------------------------------------ population store
class PopulationStore(object):
    """The .hss arrays the steps read and write: coordinates (nbead, nstruct, 3) float32
    bead-major (core/step.py:373, _preprocess.py:103-105) and the index (radii, chrom,
    copy, copy_ptr/copy_idx of index.copy_index, the haploid chrom).  A path ending in
    .hss is the HDF5 HssFile itself (igm_amd.hss); otherwise numpy files."""

    def __init__(self, path):
        self.path = path
        self.is_hss = path.endswith('.hss')
        if self.is_hss:
            from . import hss
            h = hss.Hss(path)
            self.radii, self.chrom, self.copy = h.radii, h.chrom, h.copy
            self.copy_ptr, self.copy_idx = h.copy_ptr, h.copy_idx
            self.hap_chrom = self.chrom[self.copy_idx[self.copy_ptr[:-1]]]
            self.chrom_sizes = h.chrom_sizes
        else:
            meta = np.load(path + '.index.npz')
            self.radii = meta['radii'].astype(np.float32)
            self.chrom = meta['chrom'].astype(np.int32)
            self.copy = meta['copy'].astype(np.int32)
            self.copy_ptr = meta['copy_ptr'].astype(np.int32)
            self.copy_idx = meta['copy_idx'].astype(np.int32)
            self.hap_chrom = meta['hap_chrom'].astype(np.int32) if 'hap_chrom' in meta else self.chrom
            self.chrom_sizes = meta['chrom_sizes'].astype(np.int64) if 'chrom_sizes' in meta else None
        if self.chrom_sizes is None:  # index.chrom_sizes: the beads of every (chromosome, copy) run in order
            key = self.chrom.astype(np.int64) * 64 + self.copy
            starts = np.concatenate([[0], np.nonzero(np.diff(key))[0] + 1, [len(key)]])
            self.chrom_sizes = np.diff(starts).astype(np.int64)
        self.nbead = len(self.radii)

    @staticmethod
    def create(path, coordinates, radii, chrom, copy, copy_ptr, copy_idx, hap_chrom=None):
        if path.endswith('.hss'):
            from . import hss
            hss.write_hss(path, coordinates, radii, hss.index_tree(chrom, copy, copy_ptr, copy_idx))
            return PopulationStore(path)
        np.savez(path + '.index.npz', radii=radii, chrom=chrom, copy=copy, copy_ptr=copy_ptr, copy_idx=copy_idx,
                 hap_chrom=chrom if hap_chrom is None else hap_chrom)
        np.save(path + '.npy', np.ascontiguousarray(coordinates, np.float32))
        return PopulationStore(path)

    def coordinates(self, mode='r'):
        if self.is_hss:
            from . import hss
            return hss.coordinates_memmap(self.path, mode)
        return np.load(self.path + '.npy', mmap_mode=mode)

    @property
    def nstruct(self):
        return self.coordinates().shape[1]

    def write_summary(self, text, violation):
        """the population summary (ModelingStep.py:700-726: hss 'summary' + 'violation')"""
        if self.is_hss:
            from . import hss
            hss.update_hss(self.path, summary=text, violation=violation)
        else:
            with open(self.path + '.summary.json', 'w') as f:
                f.write(text)

    def write_violation(self, violation):
        """the population's 'violation' attribute (HssFile.set_violation)"""
        if self.is_hss:
            from . import hss
            hss.update_hss(self.path, violation=violation)

    def read_summary(self):
        if self.is_hss:
            from . import hss
            return hss.Hss(self.path).summary
        with open(self.path + '.summary.json') as f:
            return f.read()


def read_rows(path):
    """the A-step rows of an actdist file (actdist.hdf5, or the .npz form)"""
    if path.endswith('.npz'):
        d = np.load(path)
        rows = np.zeros(len(d['row']), row_dtype)
        for k in ('row', 'col', 'dist', 'prob'):
            rows[k] = d[k]
        return rows
    from . import hss
    return hss.read_actdist(path)


def read_input_matrix(path):
    """the .hcs CSR arrays (indptr, indices, data, chrom) of restraints/Hi-C/input_matrix"""
    if path.endswith('.npz'):
        return dict(np.load(path))
    from . import hss
    return hss.read_hcs(path)


# ------------------------------------------------------------------ config semantics
_RAISE = object()
# the defaults of igm/core/defaults/config_schema.json this layer reads (Config.get
# falls back to them when the key is absent and no explicit default is given,
# core/config.py:98-115)
SCHEMA_DEFAULTS = {
    'model/init_radius': 5000, 'model/restraints/excluded/evfactor': 1.0,
    'model/restraints/envelope/nucleus_shape': 'sphere', 'model/restraints/envelope/nucleus_radius': 5000.0,
    'model/restraints/envelope/nucleus_semiaxes': [5000.0, 5000.0, 5000.0],
    'model/restraints/envelope/volumes_idx': [0], 'model/restraints/envelope/volume_prefix': '',
    'model/restraints/envelope/nucleus_kspring': 1, 'model/restraints/polymer/contact_range': 2.0,
    'model/restraints/polymer/polymer_bonds_style': 'simple', 'model/restraints/polymer/polymer_kspring': 1.0,
    'restraints/Hi-C/contact_range': 2.0, 'restraints/Hi-C/contact_kspring': 1.0,
    'restraints/DamID/contact_range': 0.05, 'restraints/DamID/contact_kspring': 1.0,
    'restraints/sprite/kspring': 1.0, 'restraints/sprite/radius_kt': 100.0,
    'restraints/sprite/assignment_file': 'assignment.h5', 'restraints/sprite/tmp_dir': 'tmp_opt',
    'restraints/sprite/max_chrom_in_cluster': 6, 'restraints/sprite/batch_size': 150,
    'restraints/sprite/keep_best': 50, 'restraints/FISH/rtype': 'rRpP', 'restraints/FISH/kspring': 1.0,
    'restraints/FISH/batch_size': 200, 'restraints/FISH/tmp_dir': 'tmp_opt',
    'optimization/violation_tolerance': 0.05, 'optimization/keep_intermediate_structures': True,
    'optimization/clean_restart': False,
}


def rget(cfg, key, default=_RAISE):
    """igm Config.get: the value, else the explicit default, else the schema default."""
    v = cget(cfg, key, _RAISE)
    if v is not _RAISE:
        return v
    if default is not _RAISE:
        return default
    if key in SCHEMA_DEFAULTS:
        return SCHEMA_DEFAULTS[key]
    raise KeyError('%s does not exist' % key)


def make_absolute_path(path, basedir='.'):
    """igm.utils.files.make_absolute_path"""
    if os.path.isabs(path):
        return path
    return os.path.abspath(os.path.join(basedir, path))


def _h5_tree(path):
    from . import h5
    with h5.File(path) as f:
        return {k.rstrip('/'): f.read(k) for k in f.keys('/') if not k.endswith('/')}


def _write_h5(path, tree):
    """a small result file (written beside, then renamed into place)"""
    from . import h5
    tmp = path + '.tmp'
    h5.write(tmp, tree)
    os.replace(tmp, path)


def read_damid_rows(path):
    """damid_actdist.hdf5 {loc i4, dist f4, prob f4} (DamidActivationDistanceStep.py:332-335)"""
    from ._lib import damid_row_dtype
    if path.endswith('.npz'):
        d = np.load(path)
    else:
        d = _h5_tree(path)
    rows = np.zeros(len(d['loc']), damid_row_dtype)
    for k in ('loc', 'dist', 'prob'):
        rows[k] = d[k]
    return rows


def sprite_assignment_path(cfg):
    """where SpriteAssignmentStep.reduce writes and ModelingStep.task reads the SPRITE
    assignment (SpriteAssignmentStep.py:53-56,183-186; ModelingStep.py:459-466)"""
    tmp = make_absolute_path(rget(cfg, 'restraints/sprite/tmp_dir', 'sprite'),
                             cget(cfg, 'parameters/tmp_dir', 'tmp'))
    return make_absolute_path(rget(cfg, 'restraints/sprite/assignment_file', 'assignment.h5'), tmp)


def fish_assignment_path(cfg):
    """the FISH assignment ModelingStep.task reads: the file the last FishAssignmentStep
    recorded in runtime/FISH/fish_assignment_file; without one, ModelingStep's own
    formula (ModelingStep.py:485-492 -- the reference's A-step writes under
    restraints/FISH/fish_dir instead, FishAssignmentStep.py:376-387, so a config relies
    on the runtime entry)"""
    rt = cget(cfg, 'runtime/FISH/fish_assignment_file', None)
    if rt:
        return rt
    tmp = make_absolute_path(rget(cfg, 'restraints/FISH/tmp_dir', 'FISH'), cget(cfg, 'parameters/tmp_dir', 'tmp'))
    return make_absolute_path(rget(cfg, 'restraints/FISH/fish_file', 'fish_assignment.h5'), tmp)


_VOLUMES = {}


def _volume(path):
    from . import volume as V
    key = (path, os.path.getmtime(path))
    if key not in _VOLUMES:
        _VOLUMES.clear()
        _VOLUMES[key] = V.read_volume(path)
    return _VOLUMES[key]


def envelope_section(cfg, sids):
    """model/restraints/envelope as an assemble envelope spec (ModelingStep.py:252-277)"""
    from . import assemble as A
    shape = rget(cfg, 'model/restraints/envelope/nucleus_shape')
    k = rget(cfg, 'model/restraints/envelope/nucleus_kspring')
    if shape == 'sphere':
        return A.envelope_spec('sphere', radius=rget(cfg, 'model/restraints/envelope/nucleus_radius'), k=k)
    if shape == 'ellipsoid':
        return A.envelope_spec('ellipsoid', semiaxes=rget(cfg, 'model/restraints/envelope/nucleus_semiaxes'), k=k)
    if shape == 'exp_map':
        prefix = rget(cfg, 'model/restraints/envelope/volume_prefix')
        idx = rget(cfg, 'model/restraints/envelope/volumes_idx')
        files = [prefix + str(idx[int(s) % len(idx)]) + '.bin' for s in sids]  # ModelingStep.py:265-270
        uniq = sorted(set(files))
        return {'shape': 'exp_map', 'k': float(k), 'repr_k': k, 'files': uniq,
                'volumes': [_volume(f) for f in uniq], 'struct_map': np.array([uniq.index(f) for f in files], np.int32)}
    raise NotImplementedError('Envelope (%s) not implemented' % shape)


def modeling_spec(cfg, sids):
    """Everything ModelingStep.task adds to a structure (ModelingStep.py:213-503) for the
    structures `sids`, as an igm_amd.assemble spec.  Sections this layer does not
    implement raise NotImplementedError -- none is dropped silently."""
    rs = cget(cfg, 'model/restraints', {}) or {}
    R = cfg.get('restraints', {}) or {}
    for key in ('tracing', 'nuclDamID'):
        if key in R:
            raise NotImplementedError('restraints/%s is not implemented on the hip kernel' % key)
    if 'nucleolus' in rs:
        # ModelingStep.py:306-327: GenEnvelope of a second map; the reference logs an
        # undefined name unless the envelope is exp_map (D8), and one structure would need
        # two maps -- not supported by igm_mstep_set_volumes
        raise NotImplementedError('model/restraints/nucleolus is not implemented on the hip kernel')
    spec = {'evfactor': float(rget(cfg, 'model/restraints/excluded/evfactor')),
            'protocol': cfg['optimization']['optimizer_options']}
    if 'polymer' in rs:
        if rget(cfg, 'model/restraints/polymer/polymer_bonds_style') != 'none':
            spec['polymer'] = {'contact_range': float(rs['polymer'].get('contact_range', 2.0)),
                               'kspring': float(rs['polymer'].get('polymer_kspring', 1.0)),
                               'monitored': rs['polymer'].get('violations', 'true') == 'true',  # D2
                               'contact_probabilities': cget(cfg, 'runtime/consecutive_contact_probabilities')}
    else:  # PolymerDistrib on the PolymerAssignmentStep targets (ModelingStep.py:236-249)
        pr = R['polymer']
        d = _h5_tree(cget(cfg, 'runtime/polymer/assignment_file'))
        spec['polymer'] = {'distrib': (d['loci'], d['nn_dist']), 'tolerance': float(pr['tolerance']),
                           'kspring': float(pr['polymer_kspring']),
                           'monitored': pr.get('violations', 'true') == 'true'}
    spec['envelope'] = envelope_section(cfg, sids)
    if 'Hi-C' in R:
        act = cget(cfg, 'runtime/Hi-C/actdist_file', None)
        spec['hic'] = {'rows': read_rows(act) if act else np.zeros(0, row_dtype),
                       'contact_range': float(rget(cfg, 'restraints/Hi-C/contact_range', 2.0)),
                       'k': float(rget(cfg, 'restraints/Hi-C/contact_kspring', 0.05))}
    if 'DamID' in R:
        spec['damid'] = {'rows': read_damid_rows(cget(cfg, 'runtime/DamID/damid_actdist_file')),
                         'contact_range': float(rget(cfg, 'restraints/DamID/contact_range', 2.0)),
                         'k': float(rget(cfg, 'restraints/DamID/contact_kspring', 0.05))}
    if 'sprite' in R:
        a = _h5_tree(sprite_assignment_path(cfg))
        spec['sprite'] = {'assignment': a['assignment'], 'indptr': a['indptr'], 'selected': a['selected'],
                          'volume_fraction': float(cfg['runtime']['sprite']['volume_fraction']),
                          'k': float(R['sprite']['kspring'])}
    if 'FISH' in R:
        spec['fish'] = {'data': _h5_tree(fish_assignment_path(cfg)), 'rtype': R['FISH']['rtype'],
                        'tol': float(cfg['runtime']['FISH']['tol']), 'k': float(R['FISH']['kspring'])}
    return spec


# ------------------------------------------------------------------ kernels
def _hip_actdist(store, pairs, cfg, device):
    from . import astep, _lib
    xyz = np.ascontiguousarray(store.coordinates())
    return astep.compute_actdist(xyz, store.radii, store.copy_ptr, store.copy_idx, store.hap_chrom, pairs,
                                 float(cget(cfg, 'restraints/Hi-C/contact_range', 2.0)),
                                 int(cget(cfg, 'runtime/Hi-C/iter_corr_knob', 1)), ctx=_lib.context(device))


def batch_coordinates(store, sids):
    """(S, nbead, 3) float32 struct-major coordinates of the structures sids"""
    crd = store.coordinates()
    return np.ascontiguousarray(np.asarray(crd[:, sids, :]).transpose(1, 0, 2), np.float32)


def _hip_mstep(store, sids, cfg, device):
    """ModelingStep.task for a batch of structures on one GPU: the restraints of
    modeling_spec assembled on the device (Hi-C and DamID selections), the annealing
    protocol + CG, violation records.  Returns dict(xyz (S, nbead, 3) f32, info (S)
    optinfo, stats (S, ncls, 104), names [per structure: vstat key per class])."""
    from . import _lib, assemble as A
    ctx = _lib.context(device)
    spec = modeling_spec(cfg, sids)
    b = A.build(batch_coordinates(store, sids), sids, store, spec, ctx)
    seeds = M.lammps_seeds(cget(cfg, 'optimization/optimizer_options/seed', 6535), sids,
                           cget(cfg, 'runtime/step_no', 1))
    xo, info, stats = A.run(b, seeds, float(rget(cfg, 'optimization/violation_tolerance')), ctx)
    return {'xyz': xo[:, :b.nbead], 'info': info, 'stats': stats,
            'names': [b.vstat_names(q) for q in range(len(sids))]}


KERNELS = {'hip': {'actdist': _hip_actdist, 'mstep': _hip_mstep}}


def modeling_inputs(store, cfg):
    """The Hi-C configuration's shared model pieces (steric + polymer + nucleus envelope,
    params of optimization/optimizer_options): prm, atoms, poly, chrom, Hi-C contact
    range and k, envelope violation scale."""
    rs = cget(cfg, 'model/restraints', {})
    env = rs.get('envelope', {'nucleus_shape': 'sphere', 'nucleus_radius': 5500.0, 'nucleus_kspring': 1.0})
    if env['nucleus_shape'] == 'sphere':
        abc = (float(env['nucleus_radius']),) * 3
    else:
        abc = tuple(float(v) for v in env['nucleus_semiaxes'])
    kenv = float(env.get('nucleus_kspring', 1.0))
    poly_cfg = rs.get('polymer', {'contact_range': 2.0, 'polymer_kspring': 1.0})
    poly = M.polymer_bonds(store.chrom, store.copy, store.radii, poly_cfg['contact_range'],
                           poly_cfg['polymer_kspring'])
    atoms = M.Atoms(store.radii)
    prm = M.params_from_cfg(cfg, [(abc, kenv)], evfactor=float(rs.get('excluded', {}).get('evfactor', 1.0)))
    chrom = np.concatenate([store.chrom, [-1]]).astype(np.int32)
    hic = cget(cfg, 'restraints/Hi-C', {})
    return (prm, atoms, poly, chrom, float(hic.get('contact_range', 2.0)), float(hic.get('contact_kspring', 1.0)),
            [0.1 * float(np.mean(abc))])


def _kernel(cfg, what):
    name = cget(cfg, 'optimization/kernel', 'hip')
    if name not in KERNELS:
        raise ValueError('optimization/kernel %r is not registered (have %s)' % (name, sorted(KERNELS)))
    return KERNELS[name][what]


# ------------------------------------------------------------------ the steps
class ActivationDistanceStep(Step):
    """ActivationDistanceStep.py:42-298 with the pair batches on the GPUs."""

    def __init__(self, cfg):
        rt = cfg.setdefault('runtime', {}).setdefault('Hi-C', {})
        hic = cfg['restraints']['Hi-C']
        rt.setdefault('intra_sigma_list', list(hic['intra_sigma_list']))
        rt.setdefault('inter_sigma_list', list(hic['inter_sigma_list']))
        if 'iter_corr_knob' not in rt:  # D1: absent from the schema, default 1
            rt['iter_corr_knob'] = cget(cfg, 'optimization/iter_corr_knob', 1)
        if 'inter_sigma' not in rt and 'intra_sigma' not in rt:
            if len(rt['inter_sigma_list']) and len(rt['intra_sigma_list']):
                rt['inter_sigma'] = rt['inter_sigma_list'].pop(0)
                rt['intra_sigma'] = rt['intra_sigma_list'].pop(0)
        super(ActivationDistanceStep, self).__init__(cfg)

    def name(self):
        return 'ActivationDistanceStep (INTER sigma={:.2f}%, INTRA sigma={:.2f}%, iter={:s})'.format(
            cget(self.cfg, 'runtime/Hi-C/inter_sigma') * 100.0, cget(self.cfg, 'runtime/Hi-C/intra_sigma') * 100.0,
            str(cget(self.cfg, 'runtime/opt_iter', 'NA')))

    def setup(self):
        from . import astep
        hic = read_input_matrix(self.cfg['restraints']['Hi-C']['input_matrix'])  # indptr, indices, data, chrom
        last = cget(self.cfg, 'runtime/Hi-C/actdist_file', None)
        last_rows = read_rows(last) if last is not None and os.path.isfile(last) else None
        pairs = astep.select_pairs(hic['indptr'], hic['indices'], hic['data'], hic['chrom'],
                                   cget(self.cfg, 'runtime/Hi-C/intra_sigma', False),
                                   cget(self.cfg, 'runtime/Hi-C/inter_sigma', False), last_rows=last_rows)
        bs = int(cget(self.cfg, 'optimization/kernel_opts/hip/pair_batch', 1 << 20))
        self.argument_list = []
        for b, q0 in enumerate(range(0, max(len(pairs), 1), bs)):
            fn = os.path.join(self.tmp_dir, '%s.%d.in.npy' % (self.uid, b))
            np.save(fn, pairs[q0:q0 + bs])
            self.argument_list.append({'batch': b, 'pairs': fn,
                                       'out': os.path.join(self.tmp_dir, '%s.%d.rows.npy' % (self.uid, b))})
        self.tmp_extensions = ['.npy']

    def task(self, batch, device):
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        pairs = np.load(batch['pairs'])
        rows = _kernel(self.cfg, 'actdist')(store, pairs, self.cfg, device)
        tmp = batch['out'] + '.part.npy'
        np.save(tmp, rows)
        os.replace(tmp, batch['out'])

    def reduce(self):
        """concatenate in batch order (= CSR pair order) -> actdist.hdf5 (:285-289); the
        previous file is rotated like ActivationDistanceStep.py:292-295."""
        rows = np.concatenate([np.load(b['out']) for b in self.argument_list]) if self.argument_list else \
            np.zeros(0, row_dtype)
        out = os.path.join(cget(self.cfg, 'parameters/workdir', '.'),
                           cget(self.cfg, 'restraints/Hi-C/actdist_file', 'actdist.hdf5'))
        last = cget(self.cfg, 'runtime/Hi-C/actdist_file', None)
        if last is not None and os.path.isfile(last) and os.path.abspath(last) == os.path.abspath(out):
            os.replace(last, '%s.INTERsigma_%.4f_INTRAsigma_%.4f_iter_%s' % (
                out, cget(self.cfg, 'runtime/Hi-C/inter_sigma'), cget(self.cfg, 'runtime/Hi-C/intra_sigma'),
                str(cget(self.cfg, 'runtime/opt_iter', 0))))
        if out.endswith('.npz'):
            tmp = out + '.part.npz'
            np.savez(tmp, row=rows['row'], col=rows['col'], dist=rows['dist'], prob=rows['prob'])
            os.replace(tmp, out)
        else:
            from . import hss
            hss.write_actdist(out, rows)
        cset(self.cfg, 'runtime/Hi-C/actdist_file', out)


class ModelingStep(Step):
    """ModelingStep.py:105-783 with batches of structures on the GPUs; the per-batch
    records replace the '.ready' files and the FilePoller."""

    def setup(self):
        S = int(self.cfg['model']['population_size'])
        bs = int(cget(self.cfg, 'optimization/kernel_opts/hip/batch_size', 1000))
        self.argument_list = [{'batch': b, 'sids': list(range(s0, min(s0 + bs, S))),
                               'out': os.path.join(self.tmp_dir, '%s.%d.mstep.npz' % (self.uid, b))}
                              for b, s0 in enumerate(range(0, S, bs))]
        self.tmp_extensions = ['.npz']

    def task(self, batch, device):
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        res = _kernel(self.cfg, 'mstep')(store, np.asarray(batch['sids']), self.cfg, device)
        tmp = batch['out'] + '.part.npz'
        np.savez(tmp, xyz=res['xyz'], info=res['info'].view(np.uint8), stats=res['stats'],
                 names=json.dumps(res['names']))
        os.replace(tmp, batch['out'])

    def reduce(self):
        """set_structure for every structure + teardown_poller + log_stats
        (ModelingStep.py:612-746): coordinates into the population, the summary JSON,
        runtime/violation_score."""
        from ._lib import optinfo_dtype
        from .summary import PopulationSummary, vstat_from_record
        store = PopulationStore(self.cfg['optimization']['structure_output'])
        crd = store.coordinates('r+')
        summ = PopulationSummary(crd.shape[1])
        for b in self.argument_list:
            res = np.load(b['out'])
            info = res['info'].view(optinfo_dtype)
            names = json.loads(str(res['names']))  # vstat key per class (repr() of the restraints)
            for q, sid in enumerate(b['sids']):
                crd[:, sid, :] = res['xyz'][q]
                opt = {'final-energy': float(info['final_energy'][q]), 'pair-energy': float(info['pair_energy'][q]),
                       'bond-energy': float(info['bond_energy'][q]),
                       'thermo': {'Temp': float(info['temp'][q])}}
                summ.set_structure(sid, vstat_from_record(res['stats'][q], names[q]), opt)
        crd.flush()
        del crd
        score = float(summ.violation_score())
        store.write_summary(summ.to_json(), score)
        cset(self.cfg, 'runtime/violation_score', score)


# ------------------------------------------------------------------ the other steps
from .assign_steps import (DamidActivationDistanceStep, FishAssignmentStep, PolymerAssignmentStep,  # noqa: E402
                           SpriteAssignmentStep, KERNELS_HIP as _A_HIP)
from .init_steps import RandomInit, RelaxInit, KERNELS_HIP as _I_HIP  # noqa: E402

KERNELS['hip'].update(_A_HIP)
KERNELS['hip'].update(_I_HIP)
