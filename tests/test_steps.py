"""The drop-in Step layer (igm_amd.steps) on CPU: StepDB rows with
the reference's schema and statuses (core/job_tracking.py, core/step.py:226-322), the
A-step -> M-step chain of one igm-run iteration through the per-GPU batch scheduler,
and the batch-granular restart: a run killed in the middle of the M-step resumes
without redoing the batches it had finished, and ends where an uninterrupted run
ends.  The kernels are the CPU oracle registered under a test-only kernel name (the
GPU kernels, which the gpu tests pin to the same oracle, are the product's 'hip')."""
import copy
import json
import os
import sqlite3

import numpy as np
import pytest

import oracle
import mstep_fixtures as F
import mstep_stats as MS
from conftest import GOLDEN
from igm_amd import steps as ST
from igm_amd import model as M

import cpu_kernels as CK  # registers optimization/kernel 'cpu_oracle_test'

CALLS = CK.CALLS
FAIL_AT = CK.FAIL_AT


def _oracle_actdist(store, pairs, cfg, device):
    return CK.actdist(store, pairs, cfg, device)


def _setup(tmp, S=9, fmt='hdf5'):
    """fmt 'hdf5': the reference's own files (.hcs input, .hss population, actdist.hdf5)
    through the native HDF5 reader/writer; 'npy': the numpy-file form"""
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    hic = np.load(os.path.join(GOLDEN, 'demo_hic_pairs.npz'))
    nhap = int(hic['nhap'])
    indptr = np.concatenate([[0], np.cumsum(np.bincount(hic['i'], minlength=nhap))])
    if fmt == 'hdf5':
        from igm_amd import h5
        hcs = os.path.join(tmp, 'input.hcs')
        h5.write(hcs, {'@nbin': np.int64(nhap), '@version': '0.0.4',
                       'matrix': {'indptr': indptr.astype(np.int32), 'indices': hic['j'].astype(np.int32),
                                  'data': hic['p'].astype(np.float32)},
                       'index': {'chrom': pop['hap_chrom'].astype(np.int32)}})
        out, act = os.path.join(tmp, 'igm-model.hss'), 'actdist.hdf5'
    else:
        hcs = os.path.join(tmp, 'input.hcs.npz')
        np.savez(hcs, indptr=indptr, indices=hic['j'], data=hic['p'], chrom=pop['hap_chrom'])
        out, act = os.path.join(tmp, 'igm-model'), 'actdist.npz'
    ST.PopulationStore.create(out, pop['coordinates'][:, :S], pop['radii'], pop['chrom'], pop['copy'],
                              pop['copy_ptr'], pop['copy_idx'])
    cfg = {'parameters': {'workdir': tmp, 'tmp_dir': 'tmp', 'step_db': os.path.join(tmp, 'stepdb.sqlite')},
           'model': {'population_size': S,
                     'restraints': {'excluded': {'evfactor': 1.0},
                                    'polymer': {'contact_range': 2.0, 'polymer_kspring': 1.0},
                                    'envelope': {'nucleus_shape': 'sphere', 'nucleus_radius': 5500,
                                                 'nucleus_kspring': 1.0}}},
           'restraints': {'Hi-C': {'input_matrix': hcs, 'intra_sigma_list': [1.0, 0.2], 'inter_sigma_list': [1.0, 0.2],
                                   'contact_range': 2.0, 'contact_kspring': 1.0, 'actdist_file': act}},
           'optimization': {'structure_output': out, 'kernel': 'cpu_oracle_test', 'iter_corr_knob': 1,
                            'kernel_opts': {'hip': {'batch_size': 3, 'pair_batch': 500, 'devices': [0]}},
                            'optimizer_options': MS.scaled_protocol(F.DEMO_PROTOCOL, 0.002)},
           'runtime': {}}
    return cfg


def _statuses(db, uid):
    return [x['status'] for x in ST.StepDB(db).get_history(uid)]


@pytest.mark.parametrize('fmt', ['hdf5', 'npy'])
def test_iteration_chain_and_stepdb(tmp_path, fmt):
    tmp = str(tmp_path)
    cfg = _setup(tmp, fmt=fmt)
    del CALLS[:]
    a = ST.ActivationDistanceStep(cfg)
    a.run()
    db = cfg['parameters']['step_db']
    assert _statuses(db, a.uid) == ['entry', 'setup', 'map', 'mapped', 'reduced', 'cleanup', 'completed']
    assert cfg['runtime']['Hi-C']['intra_sigma'] == 1.0 and cfg['runtime']['Hi-C']['intra_sigma_list'] == [0.2]
    # the rows: the pair batches in order == one oracle pass over every selected pair
    act = ST.read_rows(cfg['runtime']['Hi-C']['actdist_file'])
    assert len(a.argument_list) > 1
    pairs = np.concatenate([np.load(b['pairs']) for b in a.argument_list])
    store = ST.PopulationStore(cfg['optimization']['structure_output'])
    ref = _oracle_actdist(store, pairs, cfg, 0)
    assert np.array_equal(act['row'], ref['row']) and np.array_equal(act['dist'], ref['dist'])
    x0 = np.array(store.coordinates())
    m = ST.ModelingStep(cfg)
    m.run()
    assert _statuses(db, m.uid)[-1] == 'completed'
    assert sorted(CALLS) == [0, 3, 6]  # three batches of three structures
    x1 = np.array(store.coordinates())
    assert not np.array_equal(x0, x1) and np.all(np.isfinite(x1))
    assert 'violation_score' in cfg['runtime']
    summ = json.loads(store.read_summary())
    assert len(summ['bystructure']['total_energies']) == 9
    if fmt == 'hdf5':  # the population file carries the score like the reference's .hss
        from igm_amd import hss
        h = hss.Hss(cfg['optimization']['structure_output'])
        assert h.violation == cfg['runtime']['violation_score'] and h.nstruct == 9
    # the StepDB file has the reference schema: igm-run's restart code reads it
    with sqlite3.connect(db) as conn:
        cols = [(r[1], r[2]) for r in conn.execute('PRAGMA table_info(steps)')]
    assert cols == ST.StepDB.SCHEMA
    # a completed step is skipped on a rerun: no kernel call, runtime restored
    del CALLS[:]
    cfg2 = copy.deepcopy(cfg)
    cfg2['runtime']['step_no'] = cfg['runtime']['step_no'] - 1
    ST.ModelingStep(cfg2).run()
    assert CALLS == []


@pytest.mark.parametrize('fmt', ['hdf5', 'npy'])
def test_killed_mstep_resumes_without_redoing_batches(tmp_path, fmt):
    # reference result: an uninterrupted A-step + M-step in its own directory
    ref_dir = tmp_path / 'ref'
    ref_dir.mkdir()
    cfg_r = _setup(str(ref_dir), fmt=fmt)
    ST.ActivationDistanceStep(cfg_r).run()
    ST.ModelingStep(cfg_r).run()
    x_ref = np.array(ST.PopulationStore(cfg_r['optimization']['structure_output']).coordinates())

    run_dir = tmp_path / 'run'
    run_dir.mkdir()
    cfg = _setup(str(run_dir), fmt=fmt)
    ST.ActivationDistanceStep(cfg).run()
    before = copy.deepcopy(cfg)  # igm-run restores this runtime section from the StepDB on restart
    del CALLS[:]
    FAIL_AT['batch'] = 6  # the third batch dies
    try:
        with pytest.raises(RuntimeError, match='injected failure'):
            ST.ModelingStep(cfg).run()
    finally:
        FAIL_AT['batch'] = None
    m = ST.ModelingStep(copy.deepcopy(before))
    db = before['parameters']['step_db']
    assert _statuses(db, m.uid)[-1] == 'failed'
    hist = ST.StepDB(db).get_history(m.uid)
    assert 'injected failure' in hist[-1]['data']['exception']
    assert CALLS == [0, 3]  # batches 0 and 1 finished and were recorded
    del CALLS[:]
    cfg3 = copy.deepcopy(before)
    m = ST.ModelingStep(cfg3)
    m.run()
    assert CALLS == [6]  # the restart ran only the unfinished batch
    assert _statuses(db, m.uid)[-1] == 'completed'
    x = np.array(ST.PopulationStore(cfg3['optimization']['structure_output']).coordinates())
    assert np.array_equal(x, x_ref)
    assert cfg3['runtime']['violation_score'] == cfg_r['runtime']['violation_score']


def test_scheduler_spreads_batches_over_devices(tmp_path):
    seen = []

    def task(b, dev):
        seen.append((b, dev))

    s = ST.BatchScheduler([0, 1, 2], str(tmp_path), 'u')
    assert s.map(task, list(range(7))) == list(range(7))
    assert sorted(b for b, _ in seen) == list(range(7)) and {d for _, d in seen} <= {0, 1, 2}
    assert s.map(task, list(range(7))) == []  # all recorded: nothing reruns
    s2 = ST.BatchScheduler([0], str(tmp_path), 'u', clean_restart=True)
    assert s2.map(task, list(range(7))) == list(range(7))


@pytest.mark.gpu
def test_gpu_iteration_chain_with_hip_kernels(tmp_path):
    """The same igm-run iteration with optimization/kernel = 'hip' (the product
    kernels): rows equal the oracle's, the M-step batches run on the GPU."""
    tmp = str(tmp_path)
    cfg = _setup(tmp)
    cfg['optimization']['kernel'] = 'hip'
    ST.ActivationDistanceStep(cfg).run()
    act = ST.read_rows(cfg['runtime']['Hi-C']['actdist_file'])
    store = ST.PopulationStore(cfg['optimization']['structure_output'])
    a_pairs = [f for f in os.listdir(os.path.join(tmp, 'tmp')) if f.endswith('.in.npy')]
    assert a_pairs
    m = ST.ModelingStep(cfg)
    x0 = np.array(store.coordinates())
    m.run()
    x1 = np.array(store.coordinates())
    assert np.all(np.isfinite(x1)) and not np.array_equal(x0, x1)
    assert 0.0 <= cfg['runtime']['violation_score'] < 0.5
    summ = json.loads(store.read_summary())
    assert 'Envelope[shape=sphere,k=1.0,a=5500,b=5500,c=5500]' in summ['byrestraint']
    assert len(act['row']) > 100
