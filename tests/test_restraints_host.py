"""CPU: the batched restraint assembly of configurations D/E (igm_amd/restraints.py)
against per-structure loops that restate the reference's Restraint._apply
(igm/restraints/fish.py:85-266, sprite.py:36-71) literally."""
import numpy as np
from numpy.linalg import norm

from conftest import load_golden
from igm_amd import restraints as R
from igm_amd.model import LOWER_BOUND_BIT


def decode(b):
    j = b['j'] & ~LOWER_BOUND_BIT
    return [(int(x), int(y), float(r), bool(lw)) for x, y, r, lw in
            zip(b['i'], j, b['r0'], (b['j'] & LOWER_BOUND_BIT) != 0)]


def fish_loop(fish, copy_index, crd, sid, rtype, center, tol, k):
    """Fish._apply of one structure, force by force (fish.py:101-266)."""
    out = []
    lo = lambda i, j, d: out.append((int(i), int(j), float(np.float32(d)), True))
    up = lambda i, j, d: out.append((int(i), int(j), float(np.float32(d)), False))

    def sort_radially(ii):
        ii = np.array(ii)
        return ii[np.argsort([norm(crd[i]) for i in ii], kind='stable')]

    def sort_pairs(ii, jj):
        d, p = [], []
        for m in ii:
            for n in jj:
                d.append(norm(crd[m] - crd[n]))
                p.append((m, n))
        return np.array(p)[np.argsort(d, kind='stable')]

    if 'r' in rtype:
        for q, i in enumerate(fish['probes']):
            t = fish['radial_min'][q][sid]
            srt = sort_radially(copy_index[i])
            lo(center, srt[0], max(0, t - tol))
            up(center, srt[0], t + tol)
            lo(center, srt[-1], t + tol)
    if 'R' in rtype:
        for q, i in enumerate(fish['probes']):
            t = fish['radial_max'][q][sid]
            srt = sort_radially(copy_index[i])
            lo(center, srt[-1], max(0, t - tol))
            up(center, srt[-1], t + tol)
            up(center, srt[0], t - tol)
    if 'p' in rtype:
        for q, (i, j) in enumerate(fish['pairs']):
            t = fish['pair_min'][q][sid]
            sp = sort_pairs(copy_index[i], copy_index[j])
            for m, n in sp:
                lo(m, n, max(0, t - tol))
            up(sp[0][0], sp[0][1], t + tol)
    if 'P' in rtype:
        for q, (i, j) in enumerate(fish['pairs']):
            t = fish['pair_max'][q][sid]
            sp = sort_pairs(copy_index[i], copy_index[j])
            for m, n in sp:
                up(m, n, t + tol)
            lo(sp[-1][0], sp[-1][1], max(0, t - tol))
    return out


def test_fish_bonds_match_reference_loop():
    pop = load_golden('demo_population.npz')
    g = load_golden('fish_golden.npz')
    ptr, idx = pop['copy_ptr'], pop['copy_idx']
    copy_index = {h: [int(x) for x in idx[ptr[h]:ptr[h + 1]]] for h in range(len(ptr) - 1)}
    xyz = np.ascontiguousarray(pop['coordinates'].transpose(1, 0, 2))[:6]  # 6 structures, struct-major
    sids = np.array([0, 1, 2, 3, 4, 5])
    fish = {'probes': g['probes'][:20], 'radial_min': g['radial_min_targets'][:20],
            'radial_max': g['radial_max_targets'][:20], 'pairs': g['pairs'][:20],
            'pair_min': g['pair_min_targets'][:20], 'pair_max': g['pair_max_targets'][:20]}
    center = xyz.shape[1]
    for rtype in ('rRpP', 'rp', 'P'):
        got = R.fish_bonds(fish, ptr, idx, xyz, sids, rtype, center, tol=10.0, kspring=2.0)
        for s in range(len(sids)):
            ref = fish_loop(fish, copy_index, xyz[s], sids[s], rtype, center, 10.0, 2.0)
            assert sorted(decode(got[s])) == sorted(ref), (rtype, s)
            assert np.all(got[s]['k'] == np.float32(2.0))


def test_sprite_centroids_match_reference_loop():
    rng = np.random.default_rng(4)
    S, N = 5, 60
    xyz = rng.normal(0, 500, (S, N, 3)).astype(np.float32)
    radii = rng.uniform(100, 200, N).astype(np.float32)
    ncl = 12
    sizes = rng.integers(2, 6, ncl)
    indptr = np.concatenate([[0], np.cumsum(sizes)])
    selected = np.concatenate([rng.choice(N, n, replace=False) for n in sizes]).astype(np.int32)
    assignment = rng.integers(-1, S, ncl).astype(np.int32)
    vf, k, first = 0.2, 1.5, N + 1
    nslot, pos, active, bonds = R.sprite_centroids(assignment, indptr, selected, xyz, range(S), radii, vf, k, first)
    assert nslot == max(np.bincount(assignment[assignment >= 0], minlength=S))
    for s in range(S):
        cids = np.where(assignment == s)[0]
        assert active[s] == len(cids)
        ref = []
        for slot, ci in enumerate(cids):
            beads = selected[indptr[ci]:indptr[ci + 1]]
            assert np.array_equal(pos[s, slot], np.mean(xyz[s][beads], axis=0))
            csize = (np.sum(radii[beads] ** 3) / vf) ** (1. / 3.)  # get_cluster_size (sprite.py:73-79)
            for b in beads:
                ref.append((int(b), first + slot, float(np.float32(float(csize - radii[b]))), False))
        assert decode(bonds[s]) == ref
    f = R.centroid_flags(np.zeros(first + nslot, np.uint32), active, first, nslot)
    for s in range(S):
        assert np.all(f[s, first:first + active[s]] == 0)
        assert np.all(f[s, first + active[s]:] == 2)
