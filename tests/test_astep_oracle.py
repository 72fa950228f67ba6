"""The CPU oracle of the A-step against the reference's own outputs (golden
vectors made by tests/golden/make_golden.py from the reference get_actdist)."""
import numpy as np
import pytest

import oracle
from conftest import make_pairs

SIGMAS = [1.0, 0.2, 0.05, 0.02]


def demo_case(demo_pop, demo_pairs, g1, sig, it_corr):
    keep = demo_pairs['p'] >= sig
    tag = 's%g_c%d' % (sig, it_corr)
    pairs = make_pairs(demo_pairs['i'][keep], demo_pairs['j'][keep],
                       demo_pairs['p'][keep].astype(np.float64), g1[tag + '_plast'])
    return tag, pairs


@pytest.mark.parametrize('it_corr', [0, 1])
@pytest.mark.parametrize('sig', SIGMAS)
def test_oracle_demo(demo_pop, demo_pairs, g1, sig, it_corr):
    tag, pairs = demo_case(demo_pop, demo_pairs, g1, sig, it_corr)
    rows, res = oracle.actdist(demo_pop['coordinates'], demo_pop['radii'], demo_pop['copy_ptr'],
                               demo_pop['copy_idx'], demo_pop['chrom'], pairs, 2.0, it_corr, nthreads=8)
    nr = g1[tag + '_nrows'].astype(np.int32)
    assert np.array_equal(res['nrows'], nr)
    has = nr > 0
    # f64 values before the text round trip: exact
    assert np.array_equal(res['ad'][has], g1[tag + '_ad64'][has])
    assert np.array_equal(res['p'][has], g1[tag + '_p64'][has])
    # rows after the '%10.4f %.4f' round trip: bit-exact f32
    first = np.concatenate([[0], np.cumsum(res['nrows'])[:-1]])
    assert np.array_equal(rows['dist'][first[has]].view(np.uint32), g1[tag + '_dist'][has].view(np.uint32))
    assert np.array_equal(rows['prob'][first[has]].view(np.uint32), g1[tag + '_prob'][has].view(np.uint32))
    assert len(rows) == int(g1[tag + '_nrows_total'])
    if tag + '_rows_row' in g1:
        assert np.array_equal(rows['row'], g1[tag + '_rows_row'])
        assert np.array_equal(rows['col'], g1[tag + '_rows_col'])
        assert np.array_equal(rows['dist'], g1[tag + '_rows_dist'])
        assert np.array_equal(rows['prob'], g1[tag + '_rows_prob'])


def test_oracle_sigma001_subset(demo_pop, demo_pairs, g1):
    pairs = make_pairs(demo_pairs['i01'], demo_pairs['j01'], demo_pairs['p01'].astype(np.float64),
                       g1['s0.01sub_c1_plast'])
    rows, res = oracle.actdist(demo_pop['coordinates'], demo_pop['radii'], demo_pop['copy_ptr'],
                               demo_pop['copy_idx'], demo_pop['chrom'], pairs, 2.0, 1, nthreads=8)
    nr = g1['s0.01sub_c1_nrows'].astype(np.int32)
    assert np.array_equal(res['nrows'], nr)
    has = nr > 0
    first = np.concatenate([[0], np.cumsum(res['nrows'])[:-1]])
    assert np.array_equal(rows['dist'][first[has]], g1['s0.01sub_c1_dist'][has])
    assert np.array_equal(rows['prob'][first[has]], g1['s0.01sub_c1_prob'][has])


def edge_cases(g2):
    for ci in range(int(g2['ncases'])):
        for it_corr in (0, 1):
            yield ci, it_corr


@pytest.mark.parametrize('ci,it_corr', [(c, i) for c in range(4) for i in (0, 1)])
def test_oracle_edge_cases(g2, ci, it_corr):
    tag = 'c%d_i%d' % (ci, it_corr)
    pairs = make_pairs(g2[tag + '_pi'], g2[tag + '_pj'], g2[tag + '_pwish'], g2[tag + '_plast'])
    rows, res = oracle.actdist(g2['c%d_crd' % ci], g2['c%d_radii' % ci], g2['c%d_copy_ptr' % ci],
                               g2['c%d_copy_idx' % ci], g2['c%d_chrom' % ci], pairs, 2.0, it_corr)
    assert np.array_equal(res['nrows'], g2[tag + '_nrows'])
    has = res['nrows'] > 0
    assert np.array_equal(res['ad'][has], g2[tag + '_ad64'][has])
    assert np.array_equal(res['p'][has], g2[tag + '_p64'][has])
    assert np.array_equal(rows['row'], g2[tag + '_row'])
    assert np.array_equal(rows['col'], g2[tag + '_col'])
    assert np.array_equal(rows['dist'], g2[tag + '_dist'])
    assert np.array_equal(rows['prob'], g2[tag + '_prob'])
