"""Device-resident A/M iteration (the loop body of bin/igm-run:105-167 for the
Hi-C hot path) on one GPU per process.

  A-step  ActivationDistanceStep (steps/ActivationDistanceStep.py:111-298)
  M-step  ModelingStep (steps/ModelingStep.py:105-783) with the LAMMPS kernel
          replaced by igm_mstep_run

The population never leaves HBM between the steps: the structures of this rank
are struct-major (S_local, natom, 3) for the M-step; the A-step needs every
structure of the population, so with several ranks one all_gather (RCCL over
xGMI) assembles it before the A-step, whose pair list is split into contiguous
shards; the rows come back in pair order with a second all_gather.  Nothing is
exchanged during the M-step: structures are independent (ModelingStep.py:164-573
only touches its own struct_id).

torch is used for device memory, streams and torch.distributed only; every
computation is a libigmhip.so kernel.
"""
import ctypes
import time

import numpy as np

from . import _lib
from . import model as M
from ._lib import IGM_DEVICE_PTRS, bond_dtype, optinfo_dtype, pair_dtype, result_dtype, row_dtype

REC = 104


# ------------------------------------------------------------------ sharding
def shard(n, rank, world):
    """Contiguous block [lo, hi) of n units owned by `rank`: structures
    for the M-step, CSR-ordered pairs for the A-step."""
    return n * rank // world, n * (rank + 1) // world


def pair_combos(pairs, copy_ptr, hap_chrom):
    """Distance combinations get_actdist evaluates per pair (ActivationDistanceStep.py:
    405-436): min(|ii|, |jj|) for an intra-chromosome pair (copies zipped), |ii|.|jj|
    for an inter pair (every combination) -- each one an (S,)-column distance and a
    row of output."""
    cp = np.asarray(copy_ptr, np.int64)
    nc = np.diff(cp)
    hc = np.asarray(hap_chrom)
    i, j = np.asarray(pairs['i'], np.int64), np.asarray(pairs['j'], np.int64)
    ni, nj = nc[i], nc[j]
    return np.where(hc[i] == hc[j], np.minimum(ni, nj), ni * nj).astype(np.int64)


def shard_weighted(weights, rank, world):
    """Contiguous block [lo, hi) of the units whose weights sum to this rank's equal
    share (A-step pairs balanced by distance combinations -- an inter
    pair of two diploid loci costs 4, an intra pair 2).  Contiguous, so the rows in
    rank order are still the CSR order of one rank."""
    w = np.asarray(weights, np.int64)
    if len(w) == 0:
        return 0, 0
    cum = np.concatenate([[0], np.cumsum(w)])
    tot = int(cum[-1])
    lo = int(np.searchsorted(cum, tot * rank // world, side='left')) if rank > 0 else 0
    hi = int(np.searchsorted(cum, tot * (rank + 1) // world, side='left')) if rank + 1 < world else len(w)
    return lo, hi


def _staged(t, group):
    """gloo moves host tensors only: device tensors go through host memory (the
    functional multi-process path on one GPU and the CPU tests); RCCL ('nccl') keeps
    them in HBM."""
    import torch.distributed as dist
    return t.is_cuda and dist.get_backend(group) == 'gloo'


def gather_population(xyz_local, group=None, counts=None):
    """Every rank's (S_local, natom, 3) block -> the (S_total, natom, 3) population
    in rank order (one all-gather; RCCL over xGMI on the GPUs).  counts: the structures
    of every rank (pipeline.shard of any population size -- ModelingStep.py:111 runs
    range(population_size), any size); unequal blocks travel padded to the largest
    and are cut back to their counts."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    host = _staged(xyz_local, group)
    src = xyz_local.contiguous().cpu() if host else xyz_local.contiguous()
    n = src.shape[0]
    if counts is None:
        counts = [n] * world
    if counts.count(counts[0]) != len(counts):  # uneven shards: pad to the largest block
        big = max(counts)
        pad = src.new_zeros((big,) + tuple(src.shape[1:]))
        pad[:n] = src
        src = pad
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    out = torch.cat([p[:c] for p, c in zip(parts, counts)], 0)
    return out.to(xyz_local.device) if host else out


def gather_rows(rows_u8, nrows, itemsize, cap, group=None):
    """Concatenate the ranks' A-step rows in rank order, i.e. in CSR pair order
    (task() appends pair after pair, ActivationDistanceStep.py:228-230): the result
    is byte-identical to one rank processing every pair.  `cap` = the largest row
    count any rank can emit (every rank knows every shard), so one all-gather of
    fixed-size buffers carries the rows and, in each buffer's last 8 bytes, the
    count; the host reads the counts once (one sync) to compact."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    host = _staged(rows_u8, group)
    dev = rows_u8.device
    cdev = torch.device('cpu') if host else dev
    cap = max(int(cap), 1)
    off = (cap * itemsize + 7) & ~7  # the count at an 8-byte-aligned offset (an int64 view needs it)
    buf = torch.zeros(off + 8, dtype=torch.uint8, device=cdev)
    buf[:nrows * itemsize] = rows_u8[:nrows * itemsize].to(cdev)
    buf[off:].view(torch.int64).fill_(int(nrows))
    out = torch.empty(world * buf.numel(), dtype=torch.uint8, device=cdev)
    dist.all_gather_into_tensor(out, buf, group=group)
    out = out.view(world, -1)
    allc = out[:, off:].contiguous().view(torch.int64).view(-1).tolist()  # the one host sync
    rows = torch.cat([out[r, :c * itemsize] for r, c in enumerate(allc)])
    return (rows.to(dev) if host else rows), sum(allc)


def reduce_sum_f64(values, device, group=None):
    """Sum a few host numbers over the ranks (violation counts of log_stats)."""
    import torch
    import torch.distributed as dist
    dev = torch.device(device)
    if dev.type == 'cuda' and dist.get_backend(group) == 'gloo':
        dev = torch.device('cpu')
    v = torch.tensor(values, dtype=torch.float64, device=dev)
    dist.all_reduce(v, group=group)
    return v.cpu().numpy()


class AMIteration(object):
    """One GPU's share of a population and the state of the A/M loop."""

    def __init__(self, device, xyz_local, atoms, chrom, copy_ptr, copy_idx, pairs, params, polymer,
                 seed=6535, contact_range=2.0, kspring=1.0, it_corr=1, tol=0.05, env_scale=(550.0,),
                 first_sid=0, rank=0, world=1, group=None, collective=None):
        """collective: run the N > 1 exchange (population all-gather, row gather, score
        all-reduce) through torch.distributed; default world > 1.  True at world 1 puts a
        single rank through the same collectives (the one-GPU RCCL test)."""
        import torch
        self.torch = torch
        self.dev = torch.device(device)
        self.rank, self.world, self.group = rank, world, group
        self.coll = world > 1 if collective is None else bool(collective)
        self.ctx = _lib.context(self.dev.index or 0)
        T = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a if dt is None else a.astype(dt))).to(self.dev)
        xyz_local = np.ascontiguousarray(xyz_local, np.float32)
        self.S_local, self.natom = xyz_local.shape[0], xyz_local.shape[1]
        self.nbead = int(atoms.nbead)
        # every rank's structure count (shards of any population size may differ by one;
        # gather_population pads them), this rank's first column in the population
        self.counts = self._all_counts(self.S_local) if self.coll else [self.S_local] * world
        self.s_off = sum(self.counts[:rank])
        self.S_total = sum(self.counts)
        self.xyz = T(xyz_local)                                  # (S_local, natom, 3) M-step layout
        self.radii = T(atoms.radii)
        self.flags = T(atoms.flags)
        self.chrom = T(np.asarray(chrom, np.int32))              # (natom) diploid chrom
        self.bead_radii = T(atoms.radii[:self.nbead])
        self.copy_ptr = T(np.asarray(copy_ptr, np.int32))
        self.copy_idx = T(np.asarray(copy_idx, np.int32))
        self.hap_chrom = T(np.asarray(chrom, np.int32)[:len(copy_ptr) - 1])
        # contiguous pair shard of this rank (CSR order is kept across ranks), balanced
        # by distance combinations; every rank knows every shard (the row capacity)
        P = len(pairs)
        combos = pair_combos(pairs, copy_ptr, np.asarray(chrom, np.int32)[:len(copy_ptr) - 1])
        spans = [shard_weighted(combos, r, world) for r in range(world)]
        self.pair_lo, self.pair_hi = spans[rank]
        self.row_cap = max(int(combos[lo:hi].sum()) for lo, hi in spans)
        self._combos = combos
        self.npairs_total = P
        self.pairs = T(np.ascontiguousarray(pairs[self.pair_lo:self.pair_hi], pair_dtype).view(np.uint8))
        self.npairs = self.pair_hi - self.pair_lo
        self.per_pair = torch.empty(max(self.npairs, 1) * result_dtype.itemsize, dtype=torch.uint8, device=self.dev)
        self.params = params
        self.poly = T(np.ascontiguousarray(polymer, bond_dtype).view(np.uint8))
        self.npoly = len(polymer)
        self.poly_cls = T(np.full(len(polymer), M.CLASS_POLYMER, np.int32))
        self.class_cr = np.array([contact_range, contact_range, contact_range], np.float64)
        self.env_scale = np.asarray(env_scale, np.float64)
        self.seed, self.cr, self.kspring, self.it_corr, self.tol = seed, contact_range, kspring, it_corr, tol
        self.sids = np.arange(first_sid, first_sid + self.S_local)
        self.step_no = 0
        self.times = {}
        # bead-major full population for the A-step
        self.pop_bm = torch.empty((self.nbead, self.S_total, 3), dtype=torch.float32, device=self.dev)

    # ------------------------------------------------------------------ helpers
    def _all_counts(self, n):
        import torch.distributed as dist
        t = self.torch.tensor([int(n)], dtype=self.torch.int64,
                              device=self.dev if dist.get_backend(self.group) == 'nccl' else 'cpu')
        parts = [self.torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t, group=self.group)
        return [int(p.item()) for p in parts]

    def _call(self, fn, *args):
        c = self.ctx
        c.set_stream(self.torch.cuda.current_stream(self.dev).cuda_stream)
        try:
            c.check(getattr(c.lib, fn)(c.h, *args), fn)
        finally:
            c.set_stream(None)

    def _sync(self):
        self.torch.cuda.synchronize(self.dev)

    # ------------------------------------------------------------------ A-step
    def astep(self):
        torch = self.torch
        P = _lib.ptr
        if self.coll:
            src = gather_population(self.xyz, self.group, self.counts)
        else:
            src = self.xyz
        # (S_total, natom, 3) -> (nbead, S_total, 3): the .hss / A-step layout
        self._call('igm_population_transpose', IGM_DEVICE_PTRS, self.nbead, self.S_total, self.natom, P(src),
                   P(self.pop_bm), 1)
        cap = 4 * max(self.npairs, 1)
        rows = torch.empty(cap * row_dtype.itemsize, dtype=torch.uint8, device=self.dev)
        n = ctypes.c_int64(0)
        if self.npairs > 0:
            self._call('igm_astep_actdist', IGM_DEVICE_PTRS, P(self.pop_bm), self.nbead, self.S_total,
                       P(self.bead_radii), P(self.copy_ptr), P(self.copy_idx), int(self.copy_ptr.shape[0]) - 1,
                       P(self.hap_chrom), P(self.pairs), self.npairs, float(self.cr), int(self.it_corr),
                       P(self.per_pair), P(rows), cap, ctypes.byref(n))
        nrows = n.value
        if self.coll:
            rows, nrows = gather_rows(rows, nrows, row_dtype.itemsize, self.row_cap, self.group)
        self.rows, self.nrows = rows, nrows
        if self.it_corr == 1 and self.npairs > 0:  # plast of the next iteration (same sigma)
            self._call('igm_astep_update_plast', IGM_DEVICE_PTRS, P(self.pairs), self.npairs, P(self.per_pair))
        return nrows

    # ------------------------------------------------------------------ M-step
    def select(self):
        """interHiC/intraHiC restraint selection of every local structure from the
        A-step rows (restraints/inter_hic.py:294-312): per-structure CSR on device."""
        torch = self.torch
        P = _lib.ptr
        S, N = self.S_local, self.natom
        ptr = torch.empty(S + 1, dtype=torch.int64, device=self.dev)
        tot = ctypes.c_int64(0)
        args = [IGM_DEVICE_PTRS, S, N, P(self.xyz), P(self.radii), P(self.chrom), P(self.rows), self.nrows,
                float(self.cr), float(self.kspring), M.CLASS_INTER_HIC, M.CLASS_INTRA_HIC, P(ptr)]
        self._call('igm_hic_select', *(args + [None, None, ctypes.byref(tot)]))
        nb = tot.value
        bonds = torch.empty(max(nb, 1) * bond_dtype.itemsize, dtype=torch.uint8, device=self.dev)
        bcls = torch.empty(max(nb, 1), dtype=torch.int32, device=self.dev)
        self._call('igm_hic_select', *(args + [P(bonds), P(bcls), ctypes.byref(tot)]))
        self.hic_ptr, self.hic_bonds, self.hic_cls, self.nbonds = ptr, bonds, bcls, nb
        return ptr, bonds, bcls

    def mstep(self):
        torch = self.torch
        P = _lib.ptr
        S, N = self.S_local, self.natom
        ptr, bonds, bcls = self.select()
        seeds = torch.from_numpy(M.lammps_seeds(self.seed, self.sids, self.step_no)).to(self.dev)
        info = torch.empty(S * optinfo_dtype.itemsize, dtype=torch.uint8, device=self.dev)
        self._call('igm_mstep_run', IGM_DEVICE_PTRS, ctypes.byref(self.params), S, N, P(self.xyz), P(self.radii),
                   P(self.flags), P(self.poly), self.npoly, P(ptr), P(bonds), P(seeds), P(info))
        ncls = len(self.class_cr) + self.params.nenvelopes
        stats = torch.empty((S, ncls, REC), dtype=torch.int64, device=self.dev)
        self._call('igm_mstep_violations', IGM_DEVICE_PTRS, ctypes.byref(self.params), S, N, P(self.xyz),
                   P(self.radii), P(self.flags), P(self.poly), P(self.poly_cls), self.npoly, P(ptr), P(bonds),
                   P(bcls), len(self.class_cr), self.class_cr.ctypes.data, self.env_scale.ctypes.data,
                   float(self.tol), P(stats))
        self.info, self.stats = info, stats
        self.step_no += 1
        return stats

    def violation_score(self):
        """ModelingStep.log_stats: sum n_violations / sum n_imposed (all ranks)."""
        nv, ni = float(self.stats[:, :, 102].sum()), float(self.stats[:, :, 103].sum())
        if self.coll:
            nv, ni = reduce_sum_f64([nv, ni], self.dev, self.group)
        return nv / ni if ni > 0 else 0.0

    def step(self):
        t0 = time.perf_counter()
        self.astep()
        self._sync()
        t1 = time.perf_counter()
        self.mstep()
        self._sync()
        t2 = time.perf_counter()
        self.times = {'astep_s': t1 - t0, 'mstep_s': t2 - t1}
        return self.times

    # ------------------------------------------------------------------ checkpoint
    def checkpoint(self, path):
        """Write the loop state to a .hss (igm_amd.hss layout; collective when world > 1,
        rank 0 writes): the population bead-major like the reference's .hss after a
        ModelingStep (ModelingStep.py:578-610), and under 'igm_amd/' what the next
        iteration needs -- step_no (the LAMMPS seeds), every pair with its plast (the
        it_corr state of ActivationDistanceStep), the non-bead atoms' coordinates."""
        from . import hss
        P = _lib.ptr
        src = gather_population(self.xyz, self.group, self.counts) if self.coll else self.xyz
        self._call('igm_population_transpose', IGM_DEVICE_PTRS, self.nbead, self.S_total, self.natom, P(src),
                   P(self.pop_bm), 1)
        pairs_u8 = self.pairs[:self.npairs * pair_dtype.itemsize]
        if self.coll:
            cap = max(hi - lo for lo, hi in (shard_weighted(self._combos, r, self.world) for r in range(self.world)))
            pairs_u8, np_tot = gather_rows(pairs_u8, self.npairs, pair_dtype.itemsize, cap, self.group)
            pairs_u8 = pairs_u8[:np_tot * pair_dtype.itemsize]
        # the score is a collective (all_reduce over the ranks): every rank computes it
        # before the non-writers leave
        score = self.violation_score() if hasattr(self, 'stats') else np.nan
        self._sync()
        if self.rank != 0:
            return
        crd = self.pop_bm.cpu().numpy()
        extra = src[:, self.nbead:, :].cpu().numpy()
        pairs = pairs_u8.cpu().numpy().view(pair_dtype)
        cp, ci = self.copy_ptr.cpu().numpy(), self.copy_idx.cpu().numpy()
        chrom = self.chrom.cpu().numpy()[:self.nbead]
        copy = np.zeros(self.nbead, np.int32)
        for h in range(len(cp) - 1):
            copy[ci[cp[h]:cp[h + 1]]] = np.arange(cp[h + 1] - cp[h], dtype=np.int32)
        from . import h5
        tree = {'@version': np.int32(2), '@violation': np.float64(score),
                '@nstruct': np.int64(self.S_total), '@nbead': np.int64(self.nbead),
                'coordinates': crd, 'radii': self.bead_radii.cpu().numpy(),
                'index': hss.index_tree(chrom, copy, cp, ci),
                'igm_amd': {'@step_no': np.int64(self.step_no), 'extra_atoms': extra,
                            'pair_i': pairs['i'], 'pair_j': pairs['j'], 'pwish': pairs['pwish'],
                            'plast': pairs['plast']}}
        h5.write(path, tree)

    def restore(self, path):
        """Load a checkpoint() of the same population and pair list (this rank's
        structures and pair shard): the next step() continues the interrupted run."""
        from . import h5
        torch = self.torch
        with h5.File(path) as f:
            if int(f.attrs('/')['nstruct']) != self.S_total or int(f.attrs('/')['nbead']) != self.nbead:
                raise ValueError('checkpoint %s holds a different population' % path)
            crd = f.read('coordinates')
            extra = f.read('igm_amd/extra_atoms')
            step_no = int(f.attrs('igm_amd')['step_no'])
            pi, pj, plast = f.read('igm_amd/pair_i'), f.read('igm_amd/pair_j'), f.read('igm_amd/plast')
        if len(pi) != self.npairs_total:
            raise ValueError('checkpoint %s holds a different pair list' % path)
        # checkpoint() wrote the ranks' blocks in rank order: this rank's structures are
        # columns s_off .. s_off + S_local (whatever its first structure id is)
        s0 = self.s_off
        x = np.zeros((self.S_local, self.natom, 3), np.float32)
        x[:, :self.nbead] = crd[:, s0:s0 + self.S_local].transpose(1, 0, 2)
        x[:, self.nbead:] = extra[s0:s0 + self.S_local]
        self.xyz.copy_(torch.from_numpy(x))
        pairs = self.pairs[:self.npairs * pair_dtype.itemsize].cpu().numpy().view(pair_dtype).copy()
        lo, hi = self.pair_lo, self.pair_hi
        if not (np.array_equal(pairs['i'], pi[lo:hi]) and np.array_equal(pairs['j'], pj[lo:hi])):
            raise ValueError('checkpoint %s holds a different pair list' % path)
        pairs['plast'] = plast[lo:hi]
        if self.npairs:
            self.pairs[:self.npairs * pair_dtype.itemsize].copy_(torch.from_numpy(pairs.view(np.uint8)))
        self.step_no = step_no

    # ------------------------------------------------------------------ snapshots
    def snapshot(self):
        """the loop state one step starts from (device copies): structures, pair list
        with its plast, step counter"""
        return {'xyz': self.xyz.clone(), 'pairs': self.pairs.clone(), 'step_no': self.step_no}

    def load_snapshot(self, snap):
        self.xyz.copy_(snap['xyz'])
        self.pairs.copy_(snap['pairs'])
        self.step_no = snap['step_no']

    def info_host(self):
        return self.info.cpu().numpy().view(optinfo_dtype)

    def anneal_evaluations(self):
        """Force evaluations of one anneal launch per structure: every 'run n' of the
        protocol (relax + main run per stage, lammps.py:285-351) is n steps plus the
        Verlet setup evaluation."""
        p = self.params
        n = 0
        for k in range(p.nstages):
            if p.relax_steps > 0:
                n += p.relax_steps + 1
            n += p.mdsteps[k] + 1
        return n

    def algorithmic_anneal_bytes(self):
        """B_eval = 72 N + 4 N + 16 B_bonds bytes per force evaluation
        per structure (x, v, f f32x3 read+write; radius/flags; bond records), times
        the evaluations of one anneal launch, summed over this rank's structures."""
        ptr = self.hic_ptr.cpu().numpy()
        bonds_per = np.diff(ptr) + self.npoly
        return float(np.sum(76.0 * self.natom + 16.0 * bonds_per) * self.anneal_evaluations())
