"""The N>1 data path of igm_amd.pipeline on CPU (gloo, world_size 2 and 4): structure
shards -> population all-gather -> pair-sharded A-step -> rows gathered in CSR
order must equal one rank doing everything.  The per-shard A-step
compute here is the CPU oracle standing in for the HIP kernel (which the gpu
tests check against the same oracle)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from conftest import GOLDEN, make_pairs
from igm_amd import pipeline
from igm_amd._lib import row_dtype


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _inputs(nstruct=32):
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    hic = np.load(os.path.join(GOLDEN, 'demo_hic_pairs.npz'))
    keep = np.where(hic['p'] >= 0.05)[0][:3001]
    pairs = make_pairs(hic['i'][keep], hic['j'][keep], hic['p'][keep].astype(np.float64), np.zeros(len(keep)))
    xyz_sm = np.ascontiguousarray(pop['coordinates'][:, :nstruct].transpose(1, 0, 2))  # (S, nbead, 3) struct-major
    return pop, pairs, xyz_sm


def _worker(rank, world, port, out, nstruct=32):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        pop, pairs, xyz_sm = _inputs(nstruct)
        S = xyz_sm.shape[0]
        s0, s1 = pipeline.shard(S, rank, world)
        local = torch.from_numpy(xyz_sm[s0:s1].copy())
        counts = [b - a for a, b in (pipeline.shard(S, r, world) for r in range(world))]
        full = pipeline.gather_population(local, counts=counts).numpy()
        assert np.array_equal(full, xyz_sm)
        bead_major = np.ascontiguousarray(full.transpose(1, 0, 2))
        combos = pipeline.pair_combos(pairs, pop['copy_ptr'], pop['chrom'][:len(pop['copy_ptr']) - 1])
        spans = [pipeline.shard_weighted(combos, r, world) for r in range(world)]
        lo, hi = spans[rank]
        rows, _ = oracle.actdist(bead_major, pop['radii'], pop['copy_ptr'], pop['copy_idx'], pop['chrom'],
                                 pairs[lo:hi], 2.0, 1)
        u8 = torch.from_numpy(rows.view(np.uint8).copy())
        cap = max(int(combos[a:b].sum()) for a, b in spans)
        allrows, n = pipeline.gather_rows(u8, len(rows), row_dtype.itemsize, cap)
        tot = pipeline.reduce_sum_f64([float(rank + 1), 2.0], torch.device('cpu'))
        if rank == 0:
            np.save(out, allrows.numpy())
            assert n * row_dtype.itemsize == allrows.numel()
            assert tot.tolist() == [world * (world + 1) / 2.0, 2.0 * world]
    finally:
        dist.destroy_process_group()


def test_shard_covers_everything():
    for n in (0, 1, 7, 1000, 45123):
        for world in (1, 2, 3, 8):
            spans = [pipeline.shard(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[k][1] == spans[k + 1][0] for k in range(world - 1))


def test_weighted_pair_shards_balance_combinations():
    """contiguous pair shards of (nearly) equal distance combinations --
    an inter pair of diploid loci is 4 combinations, an intra pair 2 -- covering every
    pair once in CSR order."""
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    hic = np.load(os.path.join(GOLDEN, 'demo_hic_pairs.npz'))
    pairs = make_pairs(hic['i'], hic['j'], hic['p'].astype(np.float64), np.zeros(len(hic['i'])))
    hap = pop['chrom'][:len(pop['copy_ptr']) - 1]
    w = pipeline.pair_combos(pairs, pop['copy_ptr'], hap)
    nc = np.diff(pop['copy_ptr'])
    assert set(np.unique(w)) <= {1, 2, 4}
    assert np.all(w[hap[pairs['i']] != hap[pairs['j']]] == (nc[pairs['i']] * nc[pairs['j']])[hap[pairs['i']] != hap[pairs['j']]])
    for world in (1, 2, 3, 4, 8):
        spans = [pipeline.shard_weighted(w, r, world) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == len(w)
        assert all(spans[k][1] == spans[k + 1][0] for k in range(world - 1))
        loads = [int(w[a:b].sum()) for a, b in spans]
        assert max(loads) - min(loads) <= 2 * w.max(), loads
    assert pipeline.shard_weighted(np.zeros(0, np.int64), 0, 4) == (0, 0)
    assert [pipeline.shard_weighted([4], r, 2) for r in range(2)] == [(0, 1), (1, 1)]


@pytest.mark.parametrize('world,nstruct', [(2, 32), (4, 32), (3, 10)])
def test_multi_rank_astep_rows_equal_single_rank(tmp_path, world, nstruct):
    """(3, 10): a population that does not split evenly (4/3/3 structures per rank): the
    padded all-gather gives the same population, and the rows equal one rank's."""
    out = str(tmp_path / 'rows.npy')
    mp.spawn(_worker, args=(world, _free_port(), out, nstruct), nprocs=world, join=True)
    got = np.load(out)
    pop, pairs, xyz_sm = _inputs(nstruct)
    ref, _ = oracle.actdist(np.ascontiguousarray(xyz_sm.transpose(1, 0, 2)), pop['radii'], pop['copy_ptr'],
                            pop['copy_idx'], pop['chrom'], pairs, 2.0, 1)
    assert got.tobytes() == ref.tobytes()
    assert len(ref) > 500


def _de_worker(rank, world, port, out):
    """Configuration D/E A-steps over the gathered population: DamID loci and FISH
    probes sharded in contiguous ranges, results gathered in rank order (the oracle
    standing in for the HIP kernels, which the gpu tests pin to the same oracle)."""
    from oracle import asteps as A
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        pop, _, xyz_sm = _inputs()
        S = xyz_sm.shape[0]
        s0, s1 = pipeline.shard(S, rank, world)
        full = pipeline.gather_population(torch.from_numpy(xyz_sm[s0:s1].copy())).numpy()
        bm = np.ascontiguousarray(full.transpose(1, 0, 2))
        nhap = len(pop['copy_ptr']) - 1
        prof = np.random.default_rng(1).beta(2.0, 5.0, nhap).astype(np.float32)
        loci = np.where(prof >= 0.3)[0].astype(np.int32)
        lo, hi = pipeline.shard(len(loci), rank, world)
        rows = A.damid_actdist(bm, pop['radii'], pop['copy_ptr'], pop['copy_idx'], loci[lo:hi], prof,
                               np.zeros(nhap, np.float32), 1, 0.05, 'sphere', 5500.0)
        allrows, n = pipeline.gather_rows(torch.from_numpy(rows.view(np.uint8).copy()), len(rows), 12,
                                          max(b - a for a, b in (pipeline.shard(len(loci), r, world)
                                                                  for r in range(world))) * 2 * S)
        probes = loci[:40]
        t = np.sort(np.random.default_rng(2).lognormal(7.5, 0.4, (len(probes), S)), axis=1).astype(np.float32)
        plo, phi = pipeline.shard(len(probes), rank, world)
        omin, _, _, _ = A.fish_radial(bm, pop['copy_ptr'], pop['copy_idx'], probes[plo:phi], t[plo:phi], t[plo:phi])
        allf, nf = pipeline.gather_rows(torch.from_numpy(omin.view(np.uint8).ravel().copy()), len(omin), 4 * S,
                                        max(b - a for a, b in (pipeline.shard(len(probes), r, world)
                                                                for r in range(world))))
        if rank == 0:
            np.savez(out, damid=allrows.numpy(), fish=allf.numpy())
    finally:
        dist.destroy_process_group()


def test_two_rank_de_asteps_equal_single_rank(tmp_path):
    from oracle import asteps as A
    out = str(tmp_path / 'de.npz')
    mp.spawn(_de_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    pop, _, xyz_sm = _inputs()
    bm = np.ascontiguousarray(xyz_sm.transpose(1, 0, 2))
    S = xyz_sm.shape[0]
    nhap = len(pop['copy_ptr']) - 1
    prof = np.random.default_rng(1).beta(2.0, 5.0, nhap).astype(np.float32)
    loci = np.where(prof >= 0.3)[0].astype(np.int32)
    ref = A.damid_actdist(bm, pop['radii'], pop['copy_ptr'], pop['copy_idx'], loci, prof, np.zeros(nhap, np.float32),
                          1, 0.05, 'sphere', 5500.0)
    assert got['damid'].tobytes() == ref.tobytes() and len(ref) > 100
    probes = loci[:40]
    t = np.sort(np.random.default_rng(2).lognormal(7.5, 0.4, (len(probes), S)), axis=1).astype(np.float32)
    omin, _, _, _ = A.fish_radial(bm, pop['copy_ptr'], pop['copy_idx'], probes, t, t)
    assert got['fish'].tobytes() == omin.tobytes()


def _rows_worker(rank, world, port, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        # 12-byte rows (the DamID layout) and a capacity whose byte size is not a multiple of 8:
        # the count word of each buffer still sits at an aligned offset
        itemsize, cap = 12, 7
        n = 3 + 2 * rank
        rows = (np.arange(n * itemsize, dtype=np.uint8) + 50 * rank).astype(np.uint8)
        got, total = pipeline.gather_rows(torch.from_numpy(rows), n, itemsize, cap)
        if rank == 0:
            want = np.concatenate([(np.arange((3 + 2 * r) * itemsize, dtype=np.uint8) + 50 * r).astype(np.uint8)
                                   for r in range(world)])
            np.save(out, got.numpy())
            assert total == sum(3 + 2 * r for r in range(world))
            assert np.array_equal(got.numpy(), want)
    finally:
        dist.destroy_process_group()


def test_gather_rows_unaligned_capacity(tmp_path):
    """gather_rows with a row size and capacity whose product is not 8-byte aligned (12-byte
    DamID rows, capacity 7): the ranks' rows in rank order and their total (world 2, gloo)."""
    out = str(tmp_path / 'rows.npy')
    mp.spawn(_rows_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert os.path.exists(out)
