"""CPU: the configuration D/E A-step oracle (oracle/asteps.py) against the golden
vectors of the reference functions (tests/golden/make_golden_asteps.py)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import load_golden
from oracle import asteps as A


@pytest.fixture(scope='module')
def pop():
    return load_golden('demo_population.npz')


@pytest.mark.parametrize('shape', ['sphere', 'ellipsoid'])
@pytest.mark.parametrize('it_corr', [0, 1])
@pytest.mark.parametrize('sigma', [0.45, 0.2])
def test_damid_oracle_equals_reference(pop, shape, it_corr, sigma):
    g = load_golden('damid_golden.npz')
    tag = '%s_c%d_s%g' % (shape, it_corr, sigma)
    param = float(g['sphere_radius']) if shape == 'sphere' else list(g['ellipsoid_semiaxes'])
    rows = A.damid_actdist(pop['coordinates'], pop['radii'], pop['copy_ptr'], pop['copy_idx'], g[tag + '_loci'],
                           g['profile'], g['plast'], it_corr, 0.05, shape, param)
    assert np.array_equal(rows['loc'], g[tag + '_loc'])
    assert np.array_equal(rows['dist'].view(np.uint32), g[tag + '_dist'].view(np.uint32))
    assert np.array_equal(rows['prob'].view(np.uint32), g[tag + '_prob'].view(np.uint32))


def test_fish_radial_oracle_equals_reference(pop):
    g = load_golden('fish_golden.npz')
    omin, omax, dmin, dmax = A.fish_radial(pop['coordinates'], pop['copy_ptr'], pop['copy_idx'], g['probes'],
                                           g['radial_min_targets'], g['radial_max_targets'])
    assert np.array_equal(dmin, g['rad_min']) and np.array_equal(dmax, g['rad_max'])
    assert np.array_equal(omin, g['radial_min']) and np.array_equal(omax, g['radial_max'])


def test_fish_pair_oracle_equals_reference(pop):
    g = load_golden('fish_golden.npz')
    omin, omax, dmin, dmax = A.fish_pair(pop['coordinates'], pop['copy_ptr'], pop['copy_idx'], g['pairs'],
                                         g['pair_min_targets'], g['pair_max_targets'])
    assert np.array_equal(dmin, g['pair_dmin']) and np.array_equal(dmax, g['pair_dmax'])
    assert np.array_equal(omin, g['pair_min']) and np.array_equal(omax, g['pair_max'])


def test_sprite_cluster_oracle_equals_reference(pop):
    g = load_golden('sprite_cluster_golden.npz')
    crd = pop['coordinates']
    S = crd.shape[1]
    col = 0
    for c in range(0, len(g['cl_ptr']) - 1, 7):  # a subset: the restatement is a slow Python loop
        cl = g['cl_loci'][g['cl_ptr'][c]:g['cl_ptr'][c + 1]]
        reps = g['reps'][g['rep_ptr'][c]:g['rep_ptr'][c + 1]]
        rg, sel = A.sprite_cluster_rg2(crd, pop['hap_chrom'], pop['copy_ptr'], pop['copy_idx'], cl, reps,
                                       structs=range(0, S, 9))
        c0 = int(np.sum(np.diff(g['cl_ptr'])[:c]))
        ref_sel = g['selected'][:, c0:c0 + len(cl)]
        for s in range(0, S, 9):
            assert rg[s].view(np.uint32) == g['rg2s'][c][s].view(np.uint32), (c, s)
            assert np.array_equal(sel[s], ref_sel[s]), (c, s)
        col += 1
    assert col > 50


def test_sprite_keep_best_equals_reference():
    g = load_golden('sprite_cluster_golden.npz')
    for c in range(len(g['rg2s'])):
        assert np.array_equal(A.keep_best(g['rg2s'][c], int(g['keep_best'])), g['best_idx'][c])


def test_sprite_get_rgs2_known_answers():
    """The reference's own known-answer cases (igm/cython_compiled/tests.py) through
    the f32 restatement of gyration_radius_sq."""
    g = load_golden('sprite_golden.npz')
    for q in range(int(g['nkat'])):
        crd, cn = g['kat%d_crd' % q], g['kat%d_ncopies' % q]
        S = crd.shape[1]
        for s in range(S):
            alts, k0 = [], 0
            for n in cn:
                alts.append([crd[k0 + t, s] for t in range(n)])
                k0 += n
            best = np.float32(1e8)
            ncomb = int(np.prod(cn))
            for k in range(ncomb):
                kk, comb = k, []
                for a in alts:
                    comb.append(kk % len(a))
                    kk //= len(a)
                v = A.rg2_f32([alts[i][comb[i]] for i in range(len(alts))])
                best = min(best, v) if v < best else best
            assert best == g['kat%d_rg2s' % q][s]


REF_SPRITE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle', '_ref',
                          'libsprite_ref.so')


@pytest.mark.skipif(not os.path.exists(REF_SPRITE), reason='oracle/_ref not built (make -C oracle ref)')
def test_compiled_reference_sprite_kernel_reproduces_goldens(pop):
    """oracle/_ref/libsprite_ref.so -- the reference's cpp_sprite_assignment.cpp compiled
    from /root/reference by oracle/Makefile -- against the goldens its Cython build wrote
    (make_golden.py:450-489): the demo cases and the known-answer cases, bit for bit."""
    lib = ctypes.CDLL(REF_SPRITE)
    g = load_golden('sprite_golden.npz')
    P = np.ctypeslib.ndpointer
    lib.sprite_ref_get_rg2s.argtypes = [P(np.float32, flags='C'), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        P(np.int32, flags='C'), P(np.float32, flags='C'), P(np.int32, flags='C'),
                                        ctypes.POINTER(ctypes.c_int)]
    cases = [('s%d' % c, pop['coordinates'][g['s%d_beads' % c]]) for c in range(int(g['ncases']))]
    cases += [('kat%d' % q, g['kat%d_crd' % q]) for q in range(int(g['nkat']))]
    for tag, crd in cases:
        crd = np.ascontiguousarray(crd, np.float32)
        cn = np.ascontiguousarray(g[tag + '_ncopies'], np.int32)
        S = crd.shape[1]
        rg2s = np.zeros(S, np.float32)
        cidx = np.zeros((S, len(cn)), np.int32)
        best = ctypes.c_int(-1)
        lib.sprite_ref_get_rg2s(crd, S, crd.shape[0], len(cn), cn, rg2s, cidx, ctypes.byref(best))
        assert np.array_equal(rg2s.view(np.uint32), g[tag + '_rg2s'].view(np.uint32)), tag
        assert np.array_equal(cidx, g[tag + '_copy_idxs']), tag
        assert best.value == int(g[tag + '_best']), tag


def exp_maps(g):
    return [dict(body_idx=0, nvoxel=g['m%d_nvoxel' % m], center=g['m%d_center' % m], origin=g['m%d_origin' % m],
                 grid=g['m%d_grid' % m], matrice=g['m%d_matrice' % m]) for m in (0, 1)]


@pytest.mark.parametrize('it_corr', [0, 1])
def test_damid_exp_oracle_equals_reference(pop, it_corr):
    g = load_golden('damid_exp_golden.npz')
    rows = A.damid_actdist_exp(pop['coordinates'], pop['copy_ptr'], pop['copy_idx'], g['loci'], g['pexp'],
                               g['plast'], it_corr, 0.05, exp_maps(g), g['volumes_idx'])
    assert np.array_equal(rows['loc'], g['c%d_loc' % it_corr])
    assert np.array_equal(rows['dist'].view(np.uint32), g['c%d_dist' % it_corr].view(np.uint32))
    assert np.array_equal(rows['prob'].view(np.uint32), g['c%d_prob' % it_corr].view(np.uint32))
