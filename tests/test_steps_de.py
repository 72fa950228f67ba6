"""Configurations D and E through the drop-in Step layer on CPU:
the steps igm-run appends for them (bin/igm-run:138-156) -- ActivationDistanceStep,
FishAssignmentStep, SpriteAssignmentStep, DamidActivationDistanceStep -- then a
ModelingStep whose restraint assembly (igm_amd.assemble via steps.modeling_spec) picks
up every file those steps wrote; StepDB rows and batch-granular restart; the start-up
steps (RandomInit, PolymerAssignmentStep, RelaxInit) and the whole igm-run loop
(igm_amd.igm_run.run_pipeline).  Kernels: the CPU oracle (tests/cpu_kernels.py), the
same host code as the product's 'hip' kernels."""
import copy
import json
import os

import numpy as np
import pytest

import cpu_kernels as CK
import mstep_fixtures as F
import mstep_stats as MS
from conftest import GOLDEN
from igm_amd import assemble as A
from igm_amd import h5
from igm_amd import igm_run as RUN
from igm_amd import steps as ST

S = 6


def _base(tmp, envelope, S=S):
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    hic = np.load(os.path.join(GOLDEN, 'demo_hic_pairs.npz'))
    nhap = int(hic['nhap'])
    indptr = np.concatenate([[0], np.cumsum(np.bincount(hic['i'], minlength=nhap))])
    hcs = os.path.join(tmp, 'input.hcs')
    h5.write(hcs, {'@nbin': np.int64(nhap), 'matrix': {'indptr': indptr.astype(np.int32),
                                                       'indices': hic['j'].astype(np.int32),
                                                       'data': hic['p'].astype(np.float32)},
                   'index': {'chrom': pop['hap_chrom'].astype(np.int32)}})
    out = os.path.join(tmp, 'igm-model.hss')
    ST.PopulationStore.create(out, pop['coordinates'][:, :S], pop['radii'], pop['chrom'], pop['copy'],
                              pop['copy_ptr'], pop['copy_idx'])
    cfg = {'parameters': {'workdir': tmp, 'tmp_dir': os.path.join(tmp, 'tmp'),
                          'step_db': os.path.join(tmp, 'stepdb.sqlite')},
           'model': {'population_size': S, 'init_radius': 7000.0, 'starting_coordinates': out,
                     'restraints': {'excluded': {'evfactor': 1.0},
                                    'polymer': {'contact_range': 2.0, 'polymer_kspring': 1.0},
                                    'envelope': envelope}},
           'restraints': {'Hi-C': {'input_matrix': hcs, 'intra_sigma_list': [1.0, 0.2], 'inter_sigma_list': [1.0, 0.2],
                                   'contact_range': 2.0, 'contact_kspring': 1.0, 'actdist_file': 'actdist.hdf5'}},
           'optimization': {'structure_output': out, 'kernel': 'cpu_oracle_test', 'iter_corr_knob': 1,
                            'keep_intermediate_structures': False,
                            'kernel_opts': {'hip': {'batch_size': 3, 'pair_batch': 5000, 'devices': [0]}},
                            'optimizer_options': MS.scaled_protocol(F.DEMO_PROTOCOL, 0.002)},
           'runtime': {}}
    return cfg, pop


def _config_D(tmp):
    cfg, pop = _base(tmp, {'nucleus_shape': 'ellipsoid', 'nucleus_semiaxes': [5600.0, 5500.0, 5400.0],
                           'nucleus_kspring': 1.0})
    prof = os.path.join(tmp, 'damid_profile.txt')
    np.savetxt(prof, np.random.default_rng(1).beta(2.0, 5.0, len(pop['copy_ptr']) - 1).astype(np.float32))
    cfg['restraints']['DamID'] = {'input_profile': prof, 'sigma_list': [0.6, 0.45], 'contact_range': 0.05,
                                  'contact_kspring': 1.0, 'tmp_dir': 'damid'}
    return cfg, pop


def _config_E(tmp):
    from igm_amd import volume as V
    V.write_volume(os.path.join(tmp, 'nuc_0.bin'), V.sphere_map(5500.0, 250.0))
    cfg, pop = _base(tmp, {'nucleus_shape': 'exp_map', 'volume_prefix': os.path.join(tmp, 'nuc_'),
                           'volumes_idx': [0], 'nucleus_kspring': 1.0})
    nhap = len(pop['copy_ptr']) - 1
    rng = np.random.default_rng(3)
    probes = np.sort(rng.choice(nhap, 12, replace=False)).astype(np.int32)
    pairs = np.stack([rng.choice(nhap, 10), rng.choice(nhap, 10)], 1).astype(np.int32)
    pairs[:, 1] = np.where(pairs[:, 1] == pairs[:, 0], (pairs[:, 1] + 1) % nhap, pairs[:, 1])
    srt = lambda m, n: np.sort(rng.lognormal(m, 0.3, (n, S)), axis=1).astype(np.float32)
    fin = os.path.join(tmp, 'fish_input.h5')
    h5.write(fin, {'probes': probes, 'radial_min': srt(7.5, 12), 'radial_max': srt(8.0, 12), 'pairs': pairs,
                   'pair_min': srt(7.0, 10), 'pair_max': srt(7.6, 10)})
    cfg['restraints']['FISH'] = {'input_fish': fin, 'tol_list': [50.0, 25.0], 'rtype': 'rRpP', 'kspring': 1.0,
                                 'batch_size': 200}
    # SPRITE clusters of 2..6 consecutive haploid loci on one or two chromosomes
    ptr, data = [0], []
    hc = pop['hap_chrom']
    for c in range(40):
        st = int(rng.integers(0, nhap - 8))
        cl = list(range(st, st + int(rng.integers(2, 7))))
        if c % 3 == 0:
            cl.append(int(rng.integers(0, nhap)))
        data.extend(sorted(set(cl)))
        ptr.append(len(data))
    cl_file = os.path.join(tmp, 'clusters.h5')
    h5.write(cl_file, {'indptr': np.asarray(ptr, np.int64), 'data': np.asarray(data, np.int32)})
    cfg['restraints']['sprite'] = {'clusters': cl_file, 'volume_fraction_list': [0.2, 0.1], 'kspring': 1.0,
                                   'keep_best': 2, 'batch_size': 10, 'radius_kt': 50.0, 'tmp_dir': 'sprite'}
    del hc
    return cfg, pop


def _iteration(cfg):
    ran = []
    for Step in RUN.iteration_steps(cfg):
        st = Step(cfg)
        st.run()
        ran.append(st)
    return ran


def test_iteration_steps_follow_igm_run():
    cfg = {'restraints': {'Hi-C': {}, 'FISH': {}, 'sprite': {}, 'DamID': {}, 'polymer': {}}}
    names = [s.__name__ for s in RUN.iteration_steps(cfg)]
    assert names == ['PolymerAssignmentStep', 'ActivationDistanceStep', 'FishAssignmentStep', 'SpriteAssignmentStep',
                     'DamidActivationDistanceStep', 'ModelingStep']
    with pytest.raises(NotImplementedError):
        RUN.iteration_steps({'restraints': {'tracing': {}}})


def test_unsupported_sections_raise_instead_of_being_dropped(tmp_path):
    cfg, _ = _config_D(str(tmp_path))
    for where, key in (('restraints', 'tracing'), ('restraints', 'nuclDamID')):
        c = copy.deepcopy(cfg)
        c[where][key] = {}
        with pytest.raises(NotImplementedError):
            ST.modeling_spec(c, [0])
    c = copy.deepcopy(cfg)
    c['model']['restraints']['nucleolus'] = {}
    with pytest.raises(NotImplementedError):
        ST.modeling_spec(c, [0])


def test_config_D_iteration_chain_and_restart(tmp_path):
    tmp = str(tmp_path)
    cfg, pop = _config_D(tmp)
    del CK.CALLS[:]
    ran = _iteration(cfg)
    assert [type(s).__name__ for s in ran] == ['ActivationDistanceStep', 'DamidActivationDistanceStep', 'ModelingStep']
    db = cfg['parameters']['step_db']
    for s in ran:
        assert [x['status'] for x in ST.StepDB(db).get_history(s.uid)][-1] == 'completed'
    # the DamID rows: the oracle's get_damid_actdist_I over every selected locus
    dfile = cfg['runtime']['DamID']['damid_actdist_file']
    assert dfile.endswith('damid/damid_actdist.hdf5') and cfg['runtime']['DamID']['sigma'] == 0.6
    rows = ST.read_damid_rows(dfile)
    assert len(rows) > 0 and np.all(rows['prob'] > 0)
    # the M-step assembled the DamID envelope from them: per-structure members, k < 0
    store = ST.PopulationStore(cfg['optimization']['structure_output'])
    spec = ST.modeling_spec(cfg, np.arange(3))
    b = A.build(ST.batch_coordinates(store, np.arange(3)), np.arange(3), store, spec, None,
                select=CK.OracleSelect())
    assert b.prm.nenvelopes == 2 and b.prm.env_k[1] == -1.0
    assert np.allclose([b.prm.env_semiaxes[1][d] for d in range(3)], np.array([5600.0, 5500.0, 5400.0]) * 0.95)
    assert b.flags.ndim == 2 and ((b.flags & np.uint32(ST.M.IGM_ATOM_ENV0 << 1)) != 0).sum() > 0
    summ = json.loads(store.read_summary())
    assert 'Damid' in summ['byrestraint'] and 'Envelope[shape=ellipsoid,k=1.0,a=5600.0,b=5500.0,c=5400.0]' in \
        summ['byrestraint']
    # a second iteration at the same sigma reads the first's rows as plast, rotates the file
    x1 = np.array(store.coordinates())
    cfg['runtime']['opt_iter'] = 1
    del cfg['runtime']['DamID']['sigma']  # next sigma, as igm-run does after an acceptable iteration
    ran2 = _iteration(cfg)
    assert cfg['runtime']['DamID']['sigma'] == 0.45 and len(ran2) == 3
    assert os.path.isfile(dfile + '.DamID_0.4500.iter_0')  # the reference names it by the new sigma (py:317-341)
    assert not np.array_equal(x1, np.array(store.coordinates()))
    # a killed M-step resumes without redoing finished batches (StepDB + batch records)
    before = copy.deepcopy(cfg)
    CK.FAIL_AT['batch'] = 3
    del CK.CALLS[:]
    try:
        with pytest.raises(RuntimeError, match='injected failure'):
            ST.ModelingStep(cfg).run()
    finally:
        CK.FAIL_AT['batch'] = None
    assert CK.CALLS == [0]
    del CK.CALLS[:]
    m = ST.ModelingStep(copy.deepcopy(before))
    m.run()
    assert CK.CALLS == [3]


def test_config_E_iteration_chain(tmp_path):
    tmp = str(tmp_path)
    cfg, pop = _config_E(tmp)
    ran = _iteration(cfg)
    assert [type(s).__name__ for s in ran] == ['ActivationDistanceStep', 'FishAssignmentStep', 'SpriteAssignmentStep',
                                               'ModelingStep']
    # FISH: every probe/pair row of the input assigned, rank-matched per structure
    fa = ST._h5_tree(cfg['runtime']['FISH']['fish_assignment_file'])
    fin = ST._h5_tree(cfg['restraints']['FISH']['input_fish'])
    assert fa['radial_min'].shape == (12, S) and fa['pair_max'].shape == (10, S)
    assert np.array_equal(np.sort(fa['radial_min'], axis=1), fin['radial_min'])  # a permutation of the targets
    # SPRITE: one structure (or -1) per cluster, the selected beads laid out like the clusters
    sa = ST._h5_tree(ST.sprite_assignment_path(cfg))
    assert len(sa['assignment']) == 40 and sa['assignment'].min() >= -1 and sa['assignment'].max() < S
    assert len(sa['selected']) == sa['indptr'][-1]
    # the M-step assembly: map envelope, centroid slots with their bonds, FISH bonds
    store = ST.PopulationStore(cfg['optimization']['structure_output'])
    sids = np.arange(S)
    spec = ST.modeling_spec(cfg, sids)
    b = A.build(ST.batch_coordinates(store, sids), sids, store, spec, None, select=CK.OracleSelect())
    CK.oracle.set_volume(None)
    assert b.prm.env_kind[0] == ST.M.IGM_ENV_VOLUME
    per = np.bincount(sa['assignment'][sa['assignment'] >= 0], minlength=S)
    assert np.array_equal(b.active, per) and b.nslot == per.max()
    cls = b.bcls
    assert np.count_nonzero(cls == A.CLASS_SPRITE) == int(np.diff(sa['indptr'])[sa['assignment'] >= 0].sum())
    # FISH bonds: radial r and R give 3 bonds per probe, pairs 'p' ncomb + 1 and 'P' ncomb + 1
    assert np.count_nonzero(cls == A.CLASS_FISH) > 0
    summ = json.loads(store.read_summary())
    for key in ('Sprite', 'Fish', 'interHiC', 'Polymer',
                'ExpEnvelope[shape=exp_map,map={},k=1.0]'.format(os.path.join(tmp, 'nuc_0.bin'))):
        assert key in summ['byrestraint'], key


def test_startup_steps_and_the_igm_run_loop(tmp_path):
    """run_pipeline from scratch: RandomInit + RelaxInit, then A/M iterations until the
    Hi-C and DamID threshold lists are used up (max_violations 1: every iteration is
    acceptable), 'completed' marker, every step completed in the StepDB."""
    tmp = str(tmp_path)
    cfg, pop = _config_D(tmp)
    cfg['model']['starting_coordinates'] = ''
    cfg['restraints']['Hi-C']['intra_sigma_list'] = [1.0]
    cfg['restraints']['Hi-C']['inter_sigma_list'] = [1.0]
    cfg['restraints']['DamID']['sigma_list'] = [0.6]
    cfg['optimization'].update({'max_violations': 1.0, 'min_iterations': 1, 'max_iterations': 3})
    seen = []
    state = RUN.run_pipeline(cfg, on_iteration=lambda c, it, steps: seen.append((it, [s.__name__ for s in steps])))
    assert state == 'completed' and os.path.isfile(os.path.join(tmp, 'completed'))
    assert seen == [(0, ['ActivationDistanceStep', 'DamidActivationDistanceStep', 'ModelingStep'])]
    rows = ST.StepDB(cfg['parameters']['step_db']).get_history()
    names = [r['name'] for r in rows if r['status'] == 'completed']
    assert names[:2] == ['RandomInit', 'RelaxInit'] and names[-1] == 'ModelingStep'
    x = np.array(ST.PopulationStore(cfg['optimization']['structure_output']).coordinates())
    assert np.all(np.isfinite(x)) and np.abs(x).max() < 8000.0


def test_random_init_reproduces_the_reference_draw_order(tmp_path):
    """RandomInit writes generate_territories(index.chrom_sizes, init_radius) drawn from
    RandomState(init_seed * 1000003 + sid) -- igm_amd.init.generate_territories follows
    RandomInit.py:207-240's draw order (pinned against the reference in
    tests/test_init_golden.py)."""
    from igm_amd import init
    tmp = str(tmp_path)
    cfg, pop = _config_D(tmp)
    ST.RandomInit(cfg).run()
    store = ST.PopulationStore(cfg['optimization']['structure_output'])
    x = np.array(store.coordinates())
    for sid in (0, 4):
        want = init.generate_territories(pop['chrom_sizes'], 7000.0, np.random.RandomState(sid)).astype(np.float32)
        assert np.array_equal(x[:, sid], want)
    from igm_amd import hss
    assert np.isnan(hss.Hss(store.path).violation)


@pytest.mark.gpu
@pytest.mark.parametrize('config', ['D', 'E'])
def test_gpu_config_chain_with_hip_kernels(tmp_path, config):
    """The configuration D / E iteration of igm-run with optimization/kernel = 'hip'
    (the product's HIP kernels behind every Step class igm-run instantiates for them,
    bin/igm-run:139-167) beside the same chain on the CPU oracle kernels, from the same
    files: the same steps and StepDB status rows; the A-step outputs (Hi-C actdist rows,
    DamID rows, FISH and SPRITE assignments) byte-identical; the M-step ran on the GPU
    (coordinates updated in place, the summary carries every restraint class)."""
    make = _config_D if config == 'D' else _config_E
    out = {}
    for kind in ('oracle', 'hip'):
        d = tmp_path / kind
        d.mkdir()
        cfg, _ = make(str(d))
        if kind == 'hip':
            cfg['optimization']['kernel'] = 'hip'
        store = ST.PopulationStore(cfg['optimization']['structure_output'])
        x0 = np.array(store.coordinates())
        ran = _iteration(cfg)
        db = ST.StepDB(cfg['parameters']['step_db'])
        out[kind] = dict(cfg=cfg, names=[type(s).__name__ for s in ran], x0=x0, x1=np.array(store.coordinates()),
                         status=[[r['status'] for r in db.get_history(s.uid)] for s in ran],
                         summary=json.loads(store.read_summary()))
        if config == 'E':
            CK.oracle.set_volume(None)
    o, h = out['oracle'], out['hip']
    assert h['names'] == o['names'] and h['status'] == o['status']
    assert all(st[-1] == 'completed' for st in h['status'])
    ro = ST.read_rows(o['cfg']['runtime']['Hi-C']['actdist_file'])
    rh = ST.read_rows(h['cfg']['runtime']['Hi-C']['actdist_file'])
    assert len(rh) > 100 and rh.tobytes() == ro.tobytes()
    if config == 'D':
        do = ST.read_damid_rows(o['cfg']['runtime']['DamID']['damid_actdist_file'])
        dh = ST.read_damid_rows(h['cfg']['runtime']['DamID']['damid_actdist_file'])
        assert len(dh) > 0 and dh.tobytes() == do.tobytes()
    else:
        fo = ST._h5_tree(o['cfg']['runtime']['FISH']['fish_assignment_file'])
        fh = ST._h5_tree(h['cfg']['runtime']['FISH']['fish_assignment_file'])
        for k in ('radial_min', 'radial_max', 'pair_min', 'pair_max'):
            assert np.array_equal(fh[k], fo[k]), k
        so, sh = ST._h5_tree(ST.sprite_assignment_path(o['cfg'])), ST._h5_tree(ST.sprite_assignment_path(h['cfg']))
        for k in ('assignment', 'selected', 'indptr'):
            assert np.array_equal(sh[k], so[k]), k
    assert np.all(np.isfinite(h['x1'])) and not np.array_equal(h['x0'], h['x1'])
    keys = lambda kind: {k.replace(str(tmp_path / kind), '<dir>') for k in out[kind]['summary']['byrestraint']}
    assert keys('hip') == keys('oracle')
    assert 0.0 <= h['cfg']['runtime']['violation_score'] < 0.5


def test_every_step_class_igm_run_instantiates_has_a_dropin():
    """INTEGRATION.md 1b swaps every Step class bin/igm-run instantiates (:66-82 start-up,
    :105-167 iteration) for igm_amd.steps' class of the same name: each exists, is a Step
    with the reference's run() lifecycle, and igm_run's step lists use exactly them."""
    names = ('RandomInit', 'PolymerAssignmentStep', 'RelaxInit', 'ActivationDistanceStep', 'FishAssignmentStep',
             'SpriteAssignmentStep', 'DamidActivationDistanceStep', 'ModelingStep')
    for n in names:
        cls = getattr(ST, n)
        assert issubclass(cls, ST.Step) and cls.__name__ == n and cls.run is ST.Step.run
    used = {c.__name__ for c in RUN.iteration_steps({'restraints': {'Hi-C': {}, 'FISH': {}, 'sprite': {},
                                                                    'DamID': {}, 'polymer': {}}})}
    used |= {c.__name__ for c in RUN.startup_steps({'model': {'restraints': {}}})}
    assert used == set(names)
