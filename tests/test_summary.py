"""CPU: the population summary / violation_score of the M-step (ModelingStep.py:519-557,
578-725) from the reference's own per-structure violation records (G6) against the
demo .hss summary the reference wrote."""
import json

import numpy as np

from conftest import load_golden
from igm_amd import summary as SM


def test_summary_bystructure_equals_reference_demo_summary():
    g = load_golden('mstep_inputs.npz')
    ref = json.loads(str(load_golden('demo_population.npz')['summary_json']))
    S = len(ref['bystructure']['n_imposed'])
    ps = SM.PopulationSummary(S)
    sids = [i for i in range(10) if 'vstat_%d' % i in g.files]
    for i in sids:  # G6 keeps counts flat; the .hms vstat nests them under 'histogram' (py:546-553)
        v = json.loads(str(g['vstat_%d' % i]))
        ps.set_structure(i, {k: {'histogram': {'counts': c['counts']}, 'violated_restr': c['violated_restr'],
                                 'n_violations': c['n_violations'], 'n_imposed': c['n_imposed']}
                             for k, c in v.items()})
    bs = ps.data['bystructure']
    # G6 re-scored the demo coordinates with a reconstructed Hi-C selection, so the
    # per-structure totals are checked against the records themselves; the schema,
    # keys and histogram edges against the reference's own demo summary
    for i in sids:
        v = json.loads(str(g['vstat_%d' % i]))
        for key in ('n_imposed', 'n_violations', 'violated_restr'):
            assert bs[key][i] == sum(c[key] for c in v.values()), (key, i)
    assert set(ps.data['byrestraint']) == set(ref['byrestraint'])
    assert set(ps.data) == set(ref) and set(ps.data['bystructure']) == set(ref['bystructure'])
    assert ps.data['n_imposed'] == sum(bs['n_imposed'][i] for i in sids)
    assert len(ps.data['histogram']['edges']) == len(ref['histogram']['edges'])
    assert np.allclose(ps.data['histogram']['edges'][:-1], ref['histogram']['edges'][:-1])
    js = json.loads(ps.to_json())
    assert js['bystructure']['n_imposed'][sids[0]] == float(bs['n_imposed'][sids[0]])


def test_vstat_from_record_and_keys():
    rec = np.zeros((2, 104), np.int64)
    rec[0, 0], rec[0, 101:104] = 5, (0, 0, 5)
    rec[1, 3], rec[1, 100], rec[1, 101:104] = 2, 1, (3, 1, 3)
    names = ['Polymer', SM.restraint_key('Envelope', shape='sphere', k=1.0, a=5500, b=5500, c=5500)]
    v = SM.vstat_from_record(rec, names)
    assert names[1] == 'Envelope[shape=sphere,k=1.0,a=5500,b=5500,c=5500]'
    assert v['Polymer']['n_imposed'] == 5 and v[names[1]]['n_violations'] == 1
    assert len(v['Polymer']['histogram']['edges']) == 102 and v[names[1]]['histogram']['counts'][100] == 1
    ps = SM.PopulationSummary(3)
    ps.set_structure(1, v, {'final-energy': 2.0, 'pair-energy': 1.0, 'bond-energy': 1.0, 'thermo': {'Temp': 0.1}})
    assert ps.violation_score() == 1 / 8
    assert ps.data['bystructure']['thermo']['Temp'][1] == 0.1
