"""Benchmark of the IGM hot path on MI355X: one A/M iteration per step.

Metric (BASELINE.json): "M-step structures/sec + A/M iteration wall-time".
  step      = one igm-run loop body (bin/igm-run:105-167) at fixed sigma: the Hi-C
              A-step (actdist over the whole population) + the M-step (restraint
              selection, full anneal + CG protocol, violation records) of every
              structure of this rank, everything resident in HBM.
  value     = structures completed by all ranks / wall time of a step (structures/s)
  ms_per_step = the A/M iteration wall-time.
Workload at N=1: BASELINE configs[1] = SURVEY 8(d) config B: 2 Mb diploid (the demo
index, 3008 beads + 1 static dummy), 1000 structures per GPU (weak scaling: each
rank owns its own block of 1000 structure ids), Hi-C pairs of the demo .hcs at
sigma = 0.02, the demo annealing protocol (47 000 MD steps + CG), synthetic
territory initial coordinates (RandomInit semantics, seeded).

config_C block (the metric's own workload, BASELINE.json "200kb diploid pop=1000"):
200 kb diploid, pop = --c-total (default 1000) structures STRONG-split over the ranks
(all 1000 on one GPU; at 8 GPUs the 125-structure shards, the north-star run), Hi-C
sigma 0.01, full protocol, the A-step over the whole population after one RCCL
all-gather; c_warmup warmup A/M iterations at protocol x c_warmup_scale (0.1: RandomInit
to annealed structures), then c_steps timed full-protocol A/M iterations between barriers,
max over ranks.
N=1 only, beside it: the 125-structure shard of config C on frustrated restraints (A-step
bonds + 700 random long-range contacts per structure), and configurations D and E
(BASELINE.json configs[3], configs[4]) through one M-step of the 125-structure shard
(mstep_DE: DamID / SPRITE / FISH / volumetric-map restraints assembled by
igm_amd.assemble, after a warmup iteration).
CPU baselines (rank 0, N=1): the fp64 C port on the state of the first TIMED step
(snapshot after the warmup: same coordinates, restraints, seeds), one structure per
thread on every CPU the process may use (the affinity mask capped by the cgroup CPU
quota: 16 of the 256 visible CPUs on the GPU box), with the per-core rate and its
linear extrapolation to every visible CPU.

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 under
torch.distributed.run (one process per GPU, RCCL).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', choices=['B', 'C'], default='B',
                    help='B: 2 Mb diploid (the N=1 metric workload); C: 200 kb diploid (29 838 beads)')
    ap.add_argument('--nstruct', type=int, default=None, help='structures per GPU (B: 1000, C: 125)')
    ap.add_argument('--sigma', type=float, default=None, help='Hi-C sigma (B: 0.02, C: 0.01)')
    ap.add_argument('--cpu-sample', type=int, default=-1,
                    help='structures in the CPU baseline sample (-1: one per host thread; 0: skip)')
    ap.add_argument('--cpu-threads', type=int, default=0,
                    help='at most this many host threads (0: every CPU the affinity mask and cgroup quota grant)')
    ap.add_argument('--no-de', action='store_true', help='skip the configuration D/E A-step measurement')
    ap.add_argument('--sprite-clusters', type=int, default=20000, help='SPRITE clusters in the D/E measurement')
    ap.add_argument('--protocol-scale', type=float, default=1.0,
                    help='scale the MD step counts (only for smoke tests; the metric needs 1.0)')
    ap.add_argument('--no-c', action='store_true', help='skip the config C (200 kb) block of the N=1 line')
    ap.add_argument('--no-mstep-de', action='store_true',
                    help='skip the N=1 line\'s configuration D/E M-step blocks and the frustrated shard')
    ap.add_argument('--c-steps', type=int, default=1, help='timed A/M iterations of the config C block')
    ap.add_argument('--c-total', type=int, default=None,
                    help='config C population split over the ranks (default 1000: the metric\'s workload)')
    ap.add_argument('--c-warmup', type=int, default=1, help='warmup A/M iterations of the config C block')
    ap.add_argument('--c-warmup-scale', type=float, default=0.1,
                    help='MD steps of the config C warmup iterations x this (they take RandomInit to annealed '
                         'structures; the timed iterations run the full protocol)')
    ap.add_argument('--c-cpu-scale', type=float, default=0.02,
                    help='protocol scale of the config C CPU-baseline sample (0: skip it)')
    ap.add_argument('--c-shard', type=int, default=125,
                    help='N=1 only: structures of the per-GPU shard sub-block of config C (the north-star run '
                         'splits pop=1000 over 8 GPUs: 125 per GPU; 0: skip)')
    a = ap.parse_args()
    if a.nstruct is None:
        a.nstruct = 1000 if a.config == 'B' else 125
    if a.sigma is None:
        a.sigma = 0.02 if a.config == 'B' else 0.01
    if a.c_total is None:
        a.c_total = 1000
    return a


def build_inputs(args, rank, first=None):
    from igm_amd import model as M
    from igm_amd import synthetic as syn
    from igm_amd._lib import pair_dtype
    first = rank * args.nstruct if first is None else first
    pop = (syn.population_2mb if args.config == 'B' else syn.population_200kb)(args.nstruct, first_sid=first)
    atoms = M.Atoms(pop['radii'])
    natom = atoms.n
    xyz = np.zeros((args.nstruct, natom, 3), np.float32)
    xyz[:, :pop['xyz'].shape[1]] = pop['xyz']
    chrom = np.concatenate([pop['chrom'], [-1]]).astype(np.int32)
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    proto = json.loads(json.dumps(syn.DEMO_PROTOCOL))
    if args.protocol_scale != 1.0:
        cap = proto['custom_annealing_protocol']
        cap['mdsteps'] = [max(1, int(round(n * args.protocol_scale))) for n in cap['mdsteps']]
        cap['relax']['mdsteps'] = max(1, int(round(cap['relax']['mdsteps'] * args.protocol_scale)))
    prm = M.params_from_cfg({'optimization': {'optimizer_options': proto}}, [((5500.0,) * 3, 1.0)])
    i, j, p = (syn.hic_pairs_2mb if args.config == 'B' else syn.hic_pairs_200kb)(args.sigma)
    pairs = np.zeros(len(i), pair_dtype)
    pairs['i'], pairs['j'], pairs['pwish'], pairs['plast'] = i, j, p, 0.0
    return dict(pop=pop, atoms=atoms, xyz=xyz, chrom=chrom, poly=poly, prm=prm, pairs=pairs, first=first)


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cgroup v2 cpu.max, v1
    cfs_quota/period), or None when unlimited.  On the GPU box the affinity mask shows
    every CPU of the machine (256) but cpu.max grants 16 (scripts/probe_cpu.py:
    16 threads 30.3 structures/s, 256 threads 20.3 -- oversubscribed)."""
    try:
        with open('/sys/fs/cgroup/cpu.max') as fh:
            q, per = fh.read().split()[:2]
        return None if q == 'max' else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as fh:
            q = float(fh.read())
        with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as fh:
            per = float(fh.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def host_threads(args):
    """threads for the CPU baselines: every CPU this process may use -- the affinity
    mask, capped by the cgroup's CPU quota (more threads than the quota only time-slice
    the same CPU time) -- and at most --cpu-threads when given.  Returns (threads,
    affinity CPUs, quota or None)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    n = avail if quota is None else max(1, min(avail, int(quota)))
    if args.cpu_threads > 0:
        n = min(n, args.cpu_threads)
    return n, avail, quota


def host_fields(nth, avail, quota, rate):
    """the host-CPU fields every CPU baseline carries: threads used, the CPUs visible,
    the cgroup quota, the per-core rate and its linear extrapolation to every visible
    CPU (an upper bound for the CPU side: no SMT or memory-bandwidth loss assumed)"""
    return {'cores': nth, 'host_cpus_visible': avail, 'cgroup_cpu_quota': quota, 'per_core': rate / nth,
            'all_host_cpus_linear': rate / nth * avail}


def step_restraints(it, snap):
    """The Hi-C restraints the M-step of the step starting from `snap` uses: the A-step
    and the selection of that step, recomputed on the GPU from the snapshot (the state
    after the warmup = the first timed step's input)."""
    import torch
    it.load_snapshot(snap)
    it.astep()
    it.select()
    torch.cuda.synchronize(it.dev)
    return it.hic_ptr.cpu().numpy(), it.hic_bonds.cpu().numpy(), snap['xyz'].cpu().numpy(), snap['step_no']


def cpu_baseline(args, it, inp, snap):
    """The fp64 C restatement of the LAMMPS protocol (oracle/mstep_ref.c, kind 'port'),
    one structure per thread, on a bounded sample of the SAME work as the first timed
    GPU step: the first `cpu_sample` structures of rank 0 at the state after the
    warmup, with the Hi-C restraints and LAMMPS seeds of that step."""
    import oracle
    from igm_amd import model as M
    from igm_amd._lib import bond_dtype
    nth, avail, quota = host_threads(args)
    ptr, bonds, xall, step_no = step_restraints(it, snap)
    bonds = bonds.view(bond_dtype)
    n = min(nth if args.cpu_sample < 0 else args.cpu_sample, it.S_local)
    sptr = ptr[:n + 1].copy()
    sb = bonds[:sptr[-1]].copy()
    x = np.ascontiguousarray(xall[:n])
    seeds = M.lammps_seeds(it.seed, it.sids[:n], step_no)
    t0 = time.perf_counter()
    oracle.mstep_run(inp['prm'], x, inp['atoms'].radii, inp['atoms'].flags, inp['poly'], sptr, sb, seeds,
                     nthreads=min(nth, n))
    dt = time.perf_counter() - t0
    out = {'value': n / dt, 'unit': 'structures/s', 'kind': 'port'}
    out.update(host_fields(min(nth, n), avail, quota, n / dt))
    out['sample'] = ('%d structures of config B at the state of the first timed step (after %d warmup A/M '
                     'iterations: same coordinates, Hi-C restraints and seeds as that GPU step), full demo protocol, '
                     'fp64 C restatement, one structure per thread on %d threads (affinity %d CPUs, cgroup quota %s '
                     'CPUs), %.1f s' % (n, args.warmup, min(nth, n), avail, quota, dt))
    return out


def cpu_baseline_c(args, it, inp, snap, warmup):
    """The fp64 C restatement (oracle/mstep_ref.c, kind 'port') on a bounded sample of
    config C: one 200 kb structure per thread at the state of the first timed step
    (coordinates, Hi-C restraints, seeds), the demo protocol with every MD step count
    scaled by args.c_cpu_scale (the stage mix kept), timed once with and once without
    the MD stages; the MD part is extrapolated to the full protocol and the CG part
    added as measured: t = (t_sample - t_cg) / scale + t_cg per structure."""
    import oracle
    from igm_amd import model as M
    from igm_amd._lib import bond_dtype
    nth, avail, quota = host_threads(args)
    ptr, bonds, xall, step_no = step_restraints(it, snap)
    bonds = bonds.view(bond_dtype)
    n = min(nth, it.S_local)
    sptr = ptr[:n + 1].copy()
    sb = bonds[:sptr[-1]].copy()
    x = np.ascontiguousarray(xall[:n])
    seeds = M.lammps_seeds(it.seed, it.sids[:n], step_no)
    proto = json.loads(json.dumps(syn_protocol()))
    cap = proto['custom_annealing_protocol']
    sc = args.c_cpu_scale
    cap['mdsteps'] = [max(1, int(round(k * sc))) for k in cap['mdsteps']]
    cap['relax']['mdsteps'] = max(1, int(round(cap['relax']['mdsteps'] * sc)))
    prm = M.params_from_cfg({'optimization': {'optimizer_options': proto}}, [((5500.0,) * 3, 1.0)])
    t0 = time.perf_counter()
    oracle.mstep_run(prm, x.copy(), inp['atoms'].radii, inp['atoms'].flags, inp['poly'], sptr, sb, seeds, nthreads=n)
    t_sample = time.perf_counter() - t0
    prm.nstages = 0  # CG only
    t0 = time.perf_counter()
    oracle.mstep_run(prm, x.copy(), inp['atoms'].radii, inp['atoms'].flags, inp['poly'], sptr, sb, seeds, nthreads=n)
    t_cg = time.perf_counter() - t0
    t_full = max(t_sample - t_cg, 0.0) / sc + t_cg
    out = {'value': n / t_full, 'unit': 'structures/s', 'kind': 'port', 'extrapolated': True}
    out.update(host_fields(n, avail, quota, n / t_full))
    out['sample'] = ('%d structures of config C at the state of the first timed step (after %d warmup A/M '
                     'iterations: same coordinates, Hi-C restraints and seeds), fp64 C restatement, one structure '
                     'per thread on %d threads (affinity %d CPUs, cgroup quota %s CPUs); demo protocol MD steps x%g: '
                     '%.1f s, CG alone %.1f s, extrapolated to the full protocol %.0f s per %d structures (a '
                     'full-protocol measurement of the same kind: profiles/r04_parity/configC_full_protocol.json)' % (n, warmup, n, avail, quota, sc, t_sample,
                                                                          t_cg, t_full, n))
    return out


def syn_protocol():
    from igm_amd import synthetic as syn
    return syn.DEMO_PROTOCOL


def cpu_baseline_astep(args, it, nthreads, npairs=4000):
    """The bit-exact C restatement of get_actdist (oracle/actdist_ref.c, kind 'port'),
    OpenMP over pairs on `nthreads` host threads, on a seeded sample of the same pair
    list and population as the GPU A-step; pairs/s."""
    import oracle
    from igm_amd._lib import pair_dtype
    rng = np.random.default_rng(0)
    P = it.npairs
    sub = np.sort(rng.choice(P, min(npairs, P), replace=False))
    pairs = it.pairs.cpu().numpy().view(pair_dtype)[sub]
    xyz = it.pop_bm.cpu().numpy()
    t0 = time.perf_counter()
    oracle.actdist(xyz, it.bead_radii.cpu().numpy(), it.copy_ptr.cpu().numpy(), it.copy_idx.cpu().numpy(),
                   it.hap_chrom.cpu().numpy(), pairs, float(it.cr), int(it.it_corr), nthreads=nthreads)
    dt = time.perf_counter() - t0
    return {'value': len(sub) / dt, 'unit': 'pairs/s', 'cores': nthreads, 'kind': 'port',
            'per_core': len(sub) / dt / nthreads,
            'sample': '%d seeded pairs of the same list, %d structures, %.2f s' % (len(sub), it.S_total, dt)}


def max_over_ranks(dt, world, dev):
    """the slowest rank's time (the contract's max over ranks)"""
    if world == 1:
        return dt
    import torch
    import torch.distributed as dist
    t = torch.tensor([dt], dtype=torch.float64, device=dev if dist.get_backend() == 'nccl' else 'cpu')
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bench_config_c(args, dev, world, rank, local, backend='nccl'):
    """SURVEY 8(d) config C (BASELINE.json configs[2], the metric's workload): 200 kb
    diploid, Hi-C sigma 0.01, full demo protocol, inputs resident in HBM.  The
    population of args.c_total structures is split over the ranks (STRONG scaling:
    c_total / world structures per GPU; at 8 GPUs the 125-structure shards of
    pop=1000), the A-step over the whole population through the RCCL all-gather;
    c_warmup + c_steps A/M iterations, timed between barriers, max over ranks.
    Roofline of the population engine: SURVEY 8(d)'s algorithmic bytes per force
    evaluation per structure (76 N + 16 B) times the evaluations of the anneal, over
    the anneal's HIP-event time (the pop_* kernels of every MD step)."""
    import torch
    import torch.distributed as dist
    from igm_amd.pipeline import AMIteration
    from igm_amd.pipeline import shard
    total = args.c_total
    lo, hi = shard(total, rank, world)  # any population over any N (shards differ by at most one)
    per = hi - lo
    ca = argparse.Namespace(**vars(args))
    ca.config, ca.nstruct, ca.sigma = 'C', per, 0.01  # protocol_scale: 1.0 for the metric
    inp = build_inputs(ca, rank, first=lo)
    pop = inp['pop']
    it = AMIteration(dev, inp['xyz'], inp['atoms'], inp['chrom'], pop['copy_ptr'], pop['copy_idx'], inp['pairs'],
                     inp['prm'], inp['poly'], first_sid=inp['first'], rank=rank, world=world)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier(device_ids=[local]) if backend == 'nccl' else dist.barrier()
        torch.cuda.synchronize(dev)

    it.params = _scaled_prm(inp['prm'], args.c_warmup_scale)
    for w in range(args.c_warmup):
        progress('config C (pop=%d) warmup %d/%d' % (total, w + 1, args.c_warmup))
        it.step()
    it.params = inp['prm']
    barrier()
    want_cpu = args.c_cpu_scale > 0 and world == 1 and rank == 0
    snap = it.snapshot() if want_cpu else None
    anneal_ms, bytes_launch, steps = [], [], []
    t0 = time.perf_counter()
    for k in range(args.c_steps):
        progress('config C (pop=%d) timed step %d/%d' % (total, k + 1, args.c_steps))
        steps.append(it.step())
        anneal_ms.append(it.ctx.kernel_ms('anneal'))
        bytes_launch.append(it.algorithmic_anneal_bytes())
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0, world, dev)
    kms = {k: it.ctx.kernel_ms(k) for k in ('cg', 'actdist', 'actdist_select', 'hic_select', 'violations')}
    score = it.violation_score()
    info = it.info_host()
    nrows, nbonds, S_local = int(it.nrows), it.nbonds, it.S_local
    progress('config C CPU baseline')
    cpu = cpu_baseline_c(args, it, inp, snap, args.c_warmup) if want_cpu else None
    a_ms = float(np.mean(anneal_ms))
    achieved = float(np.mean(bytes_launch)) / (a_ms * 1e-3) / 1e9
    traffic, traffic_src = measured_traffic('C')
    tm = steps[-1]
    out = {
        'metric': 'M-step structures/sec + A/M iteration wall-time, 200 kb diploid pop=%d (configs[2]) on %d GPU%s'
                  % (total, world, 's' if world > 1 else ''),
        'value': total * args.c_steps / dt, 'unit': 'structures/s', 'n_gpus': world, 'steps': args.c_steps,
        'warmup': args.c_warmup, 'warmup_protocol_scale': args.c_warmup_scale,
        'ms_per_step': 1000.0 * dt / args.c_steps, 'scaling': 'strong',
        'config': {'workload': 'C: 200 kb diploid (29 838 beads), Hi-C only, pop=%d, %d structures per GPU, demo '
                               'protocol%s' % (total, per, '' if args.protocol_scale == 1.0 else
                                               ' x%g (NOT the metric)' % args.protocol_scale),
                   'nstruct_total': total, 'nstruct_per_gpu': per, 'sigma': 0.01, 'npairs': int(it.npairs_total),
                   'parallelism': 'structures sharded over %d ranks, A-step pair-sharded after an all-gather (%s)'
                                  % (world, 'RCCL' if backend == 'nccl' else backend + ' rehearsal, not a measurement')
                                  if world > 1 else 'one GPU'},
        'roofline': {'bound': 'hbm', 'kernel': 'population engine (pop_* kernels of every MD step)',
                     'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS,
                     'traffic': traffic, 'traffic_source': traffic_src,
                     'algorithmic_bytes_per_launch': float(np.mean(bytes_launch)), 'avg_launch_ms': a_ms},
        'cpu_baseline': cpu,
        'breakdown': {'astep_ms': 1000 * tm['astep_s'], 'mstep_ms': 1000 * tm['mstep_s'], 'anneal_ms': a_ms,
                      'cg_ms': kms['cg'], 'actdist_ms': kms['actdist'], 'actdist_select_ms': kms['actdist_select'],
                      'hic_select_ms': kms['hic_select'], 'violations_ms': kms['violations'],
                      'violation_score': score,
                      'median_final_energy_per_bead': float(np.median(info['final_energy'])) / inp['atoms'].nbead,
                      'rows': nrows, 'hic_bonds_per_struct': nbonds / S_local,
                      'mean_rebuilds': float(np.mean(info['nrebuild']))},
        'excludes': 'host pair enumeration (select_pairs) and file I/O: inputs resident in HBM',
    }
    del it
    torch.cuda.empty_cache()
    return out


def bench_shard(args, dev):
    """The per-GPU share of the north-star run (BASELINE.json configs[2] at 8 GPUs: pop=1000
    split 125 per GPU): one warmup and c_steps timed A/M iterations of a args.c_shard-structure
    200 kb population on this GPU, full protocol.  Its M-step time is what each of the 8 GPUs
    spends; the A-step there runs over all 1000 structures, 1/8 of the pairs per rank (7.6 ms
    for all of them at N=1, the config C block's actdist_ms), so the A-step of this shard's own
    population stands in for it."""
    sa = argparse.Namespace(**vars(args))
    sa.c_total, sa.c_cpu_scale, sa.c_warmup = args.c_shard, 0.0, 1
    progress('config C shard of %d structures' % args.c_shard)
    r = bench_config_c(sa, dev, 1, 0, 0)
    b = r['breakdown']
    return {'value': r['value'], 'unit': 'structures/s', 'nstruct': args.c_shard, 'steps': r['steps'],
            'ms_per_step': r['ms_per_step'], 'anneal_ms': b['anneal_ms'], 'cg_ms': b['cg_ms'],
            'astep_ms': b['astep_ms'], 'mstep_ms': b['mstep_ms'], 'mean_rebuilds': b['mean_rebuilds'],
            'median_final_energy_per_bead': b['median_final_energy_per_bead'], 'roofline_frac': r['roofline']['frac'],
            'mstep_bound_projection_8gpu_structures_per_s': 8.0 * args.c_shard * 1000.0 / r['ms_per_step'],
            'note': 'one GPU running the %d-structure shard each of 8 GPUs owns in the pop=1000 north-star run; '
                    'mstep_bound_projection = 8 x shard / its A/M iteration time: an M-step-bound projection, NOT a '
                    'measurement -- it leaves out the population all-gather and counts the shard\'s own A-step in '
                    'place of 1/8 of the pop=1000 A-step (both ms-scale against the ~%.0f s M-step)'
                    % (args.c_shard, b['mstep_ms'] / 1000.0)}


def _evaluations(prm):
    """force evaluations of one anneal per structure (AMIteration.anneal_evaluations)"""
    n = 0
    for k in range(prm.nstages):
        if prm.relax_steps > 0:
            n += prm.relax_steps + 1
        n += prm.mdsteps[k] + 1
    return n


def _mstep_timed(run, ctx):
    """run() = one M-step launch sequence (anneal + CG [+ violation records]) with host
    inputs/outputs, after a device sync; its wall time and the engine's HIP-event times"""
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return out, dt, {k: ctx.kernel_ms(k) for k in ('anneal', 'cg', 'violations')}


def _scaled_prm(prm, scale):
    """a copy of the M-step parameters with every MD step count x scale (stages and relax runs
    kept, at least one step each; CG unchanged)"""
    p = type(prm).from_buffer_copy(prm)
    if scale != 1.0:
        for k in range(p.nstages):
            p.mdsteps[k] = max(1, int(round(p.mdsteps[k] * scale)))
        if p.relax_steps > 0:
            p.relax_steps = max(1, int(round(p.relax_steps * scale)))
    return p


def _warm_prm(args, scale=0.1):
    """the demo protocol with the MD steps x scale (x args.protocol_scale): the warmup A/M
    iteration that takes a RandomInit population to annealed structures before the timed
    one (the steady state of igm-run's loop, where each M-step starts from the last)"""
    from igm_amd import model as M, workloads as W
    proto = W.scaled_protocol(syn_protocol(), scale * args.protocol_scale)
    return M.params_from_cfg({'optimization': {'optimizer_options': proto}}, [((5500.0,) * 3, 1.0)])


def bench_mstep_de(args, dev, config, n):
    """Configurations D and E (BASELINE.json configs[3], configs[4]) through the M-step on
    the n-structure per-GPU shard of the pop=1000 8-GPU run: 200 kb diploid (the population
    engine), the restraints of ModelingStep.task (ModelingStep.py:402-503) assembled by
    igm_amd.assemble from igm_amd.workloads' specs -- D: lamina DamID (its A-step,
    igm_damid_select membership, the k < 0 envelope, lammps.py:292-310) on the ellipsoidal
    nucleus; E: SPRITE centroid slots + bounds, FISH radial/pair bounds (their A-steps) and
    the imaged nucleus map (per-bead volume lookups) -- both with the Hi-C restraints of the
    Hi-C A-step (actdist over the synthetic 200 kb .hcs at sigma 0.01, as config C); full
    demo protocol.  A warmup A/M iteration (protocol x0.1) takes
    the RandomInit territories to annealed structures; the next A/M iteration is timed in its
    parts: A-steps (the spec's GPU A-steps and host reductions, on the warmed population),
    assembly (host), M-step (anneal + CG + violation records, host arrays in and out: PCIe
    included)."""
    import types
    from igm_amd import _lib, assemble as A, model as M, volume as V, workloads as W
    ctx = _lib.context(dev.index or 0)
    progress('config %s M-step (%d structures)' % (config, n))
    pop = W.population(config, n, first_sid=0)
    sids = np.arange(n)
    vol = V.sphere_map(5500.0, 100.0) if config == 'E' else None
    idx = types.SimpleNamespace(radii=pop['radii'], chrom=pop['chrom'], copy=pop['copy'], copy_ptr=pop['copy_ptr'],
                                copy_idx=pop['copy_idx'])

    def spec_of(scale):  # the A-steps of the configuration on the current population
        hic = W.hic_actdist_rows(pop)
        return (W.spec_D(pop, n, scale, ctx, hic=hic) if config == 'D' else
                W.spec_E(pop, n, scale, ctx, vol, hic=hic))
    try:
        # warmup A/M iteration (protocol x0.1) from RandomInit
        b = A.build(pop['xyz'], sids, idx, spec_of(0.1 * args.protocol_scale), ctx)
        xw, _, _ = A.run(b, M.lammps_seeds(6535, sids, 0), 0.05, ctx)
        pop = dict(pop, xyz=np.ascontiguousarray(xw[:, :b.nbead]))
        # the timed A/M iteration
        t0 = time.perf_counter()
        spec = spec_of(args.protocol_scale)
        t1 = time.perf_counter()
        b = A.build(pop['xyz'], sids, idx, spec, ctx)
        t2 = time.perf_counter()
        seeds = M.lammps_seeds(6535, sids, 1)
        (xg, info, st), dt, kms = _mstep_timed(lambda: A.run(b, seeds, 0.05, ctx), ctx)
    finally:
        if vol is not None:
            V.stage(ctx, [])
    nbonds = np.diff(b.ptr) + len(b.poly)
    per_eval = float(np.sum(76.0 * b.natom + 16.0 * nbonds))
    abytes = per_eval * _evaluations(b.prm)
    achieved = abytes / (kms['anneal'] * 1e-3) / 1e9
    mix = {}
    for c in range(len(b.names)):
        nm = b.names[c] if isinstance(b.names[c], str) or b.names[c] is None else b.names[c][0]
        if nm is None:
            continue
        if c < 5:
            cnt = int(np.count_nonzero(b.bcls == c)) + (len(b.poly) * n if c == M.CLASS_POLYMER else 0)
            mix[nm] = cnt / n
    if b.flags.ndim == 2 and config == 'D':
        mix['Damid lamina members'] = float(np.count_nonzero(b.flags[:, :b.nbead] & (_lib.IGM_ATOM_ENV0 << 1))) / n
    if config == 'E':
        mix['SPRITE centroid slots (active mean)'] = float(np.mean(b.active))
    out = {
        'workload': '%s: 200 kb diploid (29 838 beads), %d structures (the per-GPU shard of pop=1000 at 8 GPUs), %s, '
                    'demo protocol%s' % (config, n, 'Hi-C (A-step rows, sigma 0.01) + lamina DamID (k<0 envelope) + '
                                         'ellipsoidal nucleus' if config == 'D' else 'Hi-C (A-step rows, sigma 0.01) + '
                                         'SPRITE + FISH + imaged nuclear-body map (volumetric restraint)',
                                         '' if args.protocol_scale == 1.0 else ' x%g (NOT the metric)'
                                         % args.protocol_scale),
        'value': n / dt, 'unit': 'structures/s (M-step)', 'nstruct': n, 'natom': int(b.natom),
        'mstep_s': dt, 'astep_s': t1 - t0, 'assemble_s': t2 - t1, 'iteration_s': t1 - t0 + (t2 - t1) + dt,
        'anneal_ms': kms['anneal'], 'cg_ms': kms['cg'], 'violations_ms': kms['violations'],
        'restraints_per_structure': mix,
        'roofline': {'bound': 'hbm', 'kernel': 'population engine (anneal)', 'achieved': achieved,
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS,
                     'algorithmic_bytes_per_launch': abytes, 'avg_launch_ms': kms['anneal']},
        'median_final_energy_per_bead': float(np.median(info['final_energy'])) / b.nbead,
        'mean_rebuilds': float(np.mean(info['nrebuild'])),
        'note': 'value = structures / M-step wall time (anneal + CG + violation records, host arrays over PCIe); '
                'iteration_s adds the A-steps and the host assembly of this configuration; timed after a warmup '
                'A/M iteration (protocol x0.1) from RandomInit',
    }
    del xg, st, b
    return out


def bench_frustrated(args, dev, n, ncontacts=700):
    """The north-star shard on FRUSTRATED restraints (tests/test_configC_gpu.py's stage-wise
    recipe): a 200 kb population's A-step bonds after one warmup A/M iteration plus
    `ncontacts` random long-range contacts per structure that cannot all be met, so the final
    energies stay far from zero (the satisfiable synthetic .hcs anneals to ~1e-11 per bead).
    Times the M-step (anneal + CG) of those n structures, full protocol."""
    import torch
    from igm_amd import model as M, mstep, workloads as W
    from igm_amd._lib import bond_dtype
    from igm_amd.pipeline import AMIteration
    progress('config C frustrated shard (%d structures)' % n)
    ca = argparse.Namespace(**vars(args))
    ca.config, ca.nstruct, ca.sigma = 'C', n, 0.01
    inp = build_inputs(ca, 0, first=0)
    pop = inp['pop']
    it = AMIteration(dev, inp['xyz'], inp['atoms'], inp['chrom'], pop['copy_ptr'], pop['copy_idx'], inp['pairs'],
                     _warm_prm(args), inp['poly'], first_sid=0)
    it.step()  # the first A/M iteration from RandomInit (protocol x0.1: relaxes the territories)
    it.params = inp['prm']
    it.astep()
    it.select()
    torch.cuda.synchronize(dev)
    ptr = it.hic_ptr.cpu().numpy()
    hic = it.hic_bonds.cpu().numpy().view(bond_dtype)[:ptr[-1]]
    x0 = it.xyz.cpu().numpy()
    atoms = inp['atoms']
    per = [np.concatenate([hic[ptr[s]:ptr[s + 1]], W.random_contacts(atoms.radii, atoms.nbead, 0, ncontacts, 7000 + s)])
           for s in range(n)]
    sptr, sb = M.concat_bonds(per)
    seeds = M.lammps_seeds(it.seed, it.sids, it.step_no)
    ctx = it.ctx
    del it
    torch.cuda.empty_cache()
    (xg, info), dt, kms = _mstep_timed(lambda: mstep.run(inp['prm'], x0, atoms.radii, atoms.flags, inp['poly'], sptr,
                                                         sb, seeds, ctx=ctx), ctx)
    return {'value': n / dt, 'unit': 'structures/s (M-step)', 'nstruct': n, 'mstep_s': dt,
            'anneal_ms': kms['anneal'], 'cg_ms': kms['cg'],
            'bonds_per_structure': float(sptr[-1]) / n, 'extra_contacts_per_structure': ncontacts,
            'median_final_energy_per_bead': float(np.median(info['final_energy'])) / atoms.nbead,
            'mean_rebuilds': float(np.mean(info['nrebuild'])),
            'note': 'A-step bonds + %d random long-range contacts per structure (frustrated); M-step = anneal + CG, '
                    'host arrays over PCIe' % ncontacts}


def bench_asteps_de(args, ctx):
    """Configuration D/E A-steps at full population size (200 kb diploid, 1000
    structures, bead-major .hss layout resident in HBM), timed with HIP events around
    each kernel family: DamID (ellipsoid, sigma 0.45), FISH (500 probes + 500 pairs),
    SPRITE (Rg^2 of every (cluster, structure) + keep_best 50), polymer distances
    (every (i, i+1) locus, PolymerAssignmentStep).  Outside the timed
    A/M region; reported beside it.  Algorithmic bytes: the unique coordinate columns
    each unit reads (12 B per bead per structure) plus its inputs/outputs."""
    import torch
    from igm_amd import damid, fish, sprite, synthetic as syn
    S = 1000
    pop = syn.population_200kb(S)
    xyz = np.ascontiguousarray(pop['xyz'].transpose(1, 0, 2))
    cp, ci = pop['copy_ptr'], pop['copy_idx']
    nc = np.diff(cp)
    out = {}
    loci, pe, pl = damid.select_loci(syn.damid_profile_200kb(), 0.45)
    pl[::2] = np.float32(0.3)
    for _ in range(2):  # first call stages the population; time the second
        damid.compute_damid_actdist(xyz, pop['radii'], cp, ci, loci, pe, pl, 1, 0.05, 'ellipsoid',
                                    syn.ELLIPSOID_D, ctx=ctx)
    ms = ctx.kernel_ms('damid')
    b = float((12.0 * S * nc[loci] + 12.0 * nc[loci] + 8).sum())

    def uniq(beads):  # the distinct coordinate columns a launch reads, once each (12 B x S per bead)
        return 12.0 * S * len(np.unique(np.asarray(beads)))
    u = uniq(np.concatenate([ci[cp[h]:cp[h + 1]] for h in loci]))
    out['damid'] = {'units': int(len(loci)), 'unit': 'loci', 'ms': ms, 'algorithmic_bytes': b,
                    'achieved_GBps': b / (ms * 1e-3) / 1e9, 'unique_bytes': u, 'unique_GBps': u / (ms * 1e-3) / 1e9}
    f = syn.fish_inputs_200kb(S)
    tot_ms, tot_b = 0.0, 0.0
    fb = np.concatenate([np.ravel(f['probes']), np.ravel(f['pairs'])])
    u_fish = uniq(np.concatenate([ci[cp[h]:cp[h + 1]] for h in fb]))
    for kind, key, pre in (('probe', 'probes', 'radial'), ('pair', 'pairs', 'pair')):
        for _ in range(2):
            fish.assign(xyz, cp, ci, kind, f[key], f[pre + '_min'], f[pre + '_max'], ctx=ctx)
        tot_ms += ctx.kernel_ms('fish')
        cols = nc[f[key]] if kind == 'probe' else nc[f[key][:, 0]] + nc[f[key][:, 1]]
        tot_b += float((12.0 * S * cols + 16.0 * S).sum())
    out['fish'] = {'units': int(len(f['probes']) + len(f['pairs'])), 'unit': 'probes+pairs', 'ms': tot_ms,
                   'algorithmic_bytes': tot_b, 'achieved_GBps': tot_b / (tot_ms * 1e-3) / 1e9,
                   'unique_bytes': u_fish, 'unique_GBps': u_fish / (tot_ms * 1e-3) / 1e9}
    ptr, data = syn.sprite_clusters_200kb(args.sprite_clusters)
    cl = [data[ptr[c]:ptr[c + 1]] for c in range(len(ptr) - 1)]
    t = sprite.cluster_tables(cl, pop['hap_chrom'], cp, rng=np.random.RandomState(0))
    for _ in range(2):
        sprite.rg2_select(xyz, cp, ci, t, 50, ctx=ctx)
    ms = ctx.kernel_ms('sprite')
    alts = nc[t['seg_region']].sum() + (nc[t['rep_region']].sum() if len(t['rep_region']) else 0)
    b = float(12.0 * S * alts + 4.0 * S * len(t['kept']) * 2 + 4.0 * S * len(t['seg_region']) +
              (4 + 4) * 50 * len(t['kept']) + 4 * 50 * len(t['seg_region']))
    regs = np.concatenate([t['seg_region'], t['rep_region']]) if len(t['rep_region']) else t['seg_region']
    u = uniq(np.concatenate([ci[cp[h]:cp[h + 1]] for h in np.unique(regs)]))
    out['sprite'] = {'units': int(len(t['kept'])), 'unit': 'clusters x 1000 structures', 'ms': ms,
                     'algorithmic_bytes': b, 'achieved_GBps': b / (ms * 1e-3) / 1e9, 'unique_bytes': u,
                     'unique_GBps': u / (ms * 1e-3) / 1e9,
                     'note': 'algorithmic_bytes counts every cluster\'s columns (clusters share loci: re-reads, '
                             'served by L2); unique_bytes each column once'}
    # polymer distances: every (i, i+1) locus, 60-bin distribution, one launch
    from igm_amd import polymer
    nb = xyz.shape[0]
    edges = np.linspace(200.0, 900.0, 60)
    prob = np.exp(-0.5 * ((edges - 500.0) / 120.0) ** 2)
    prob /= prob.sum()
    for _ in range(2):
        polymer.assign(xyz, edges, prob, np.random.RandomState(1), chunk=nb, ctx=ctx)
    ms = ctx.kernel_ms('polymer')
    b = float((nb - 1) * S * (24.0 + 8.0 + 4.0))
    out['polymer'] = {'units': int(nb - 1), 'unit': 'loci x 1000 structures', 'ms': ms, 'algorithmic_bytes': b,
                      'achieved_GBps': b / (ms * 1e-3) / 1e9, 'unique_bytes': 12.0 * S * nb,
                      'unique_GBps': 12.0 * S * nb / (ms * 1e-3) / 1e9}
    out['workload'] = '200 kb diploid (29 838 beads), 1000 structures, bead-major f32 in HBM'
    del torch
    return out


def measured_traffic(config):
    """HBM bytes per anneal launch from the committed PMC passes (FETCH_SIZE x 2 gfx950
    correction + WRITE_SIZE, scripts/gpu_bench.sh -> profiles/<round>/hbm_traffic.txt),
    kept in bench_traffic.json beside this file; None when not measured."""
    path = os.path.join(ROOT, 'bench_traffic.json')
    if not os.path.exists(path):
        return None, None
    with open(path) as fh:
        d = json.load(fh).get(config)
    if not d:
        return None, None
    return float(d['fetch_bytes_per_launch']) + float(d['write_bytes_per_launch']), d['source']


def measured_issue(config):
    """VALU-pipe fraction of the anneal kernel from the committed SQ counter passes
    (scripts/make_issue.py over profiles/<round>/sq*.txt), kept in bench_issue.json:
    the fraction of each SIMD-32's cycles its VALU pipe is busy (2 cycles per wave64
    VALU instruction; SQ_WAVE_CYCLES in quad-cycles), beside the wait and LDS
    bank-conflict shares.  The anneal kernel keeps its structure in LDS, so these --
    not HBM bytes -- say what binds it."""
    path = os.path.join(ROOT, 'bench_issue.json')
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        return json.load(fh).get(config)


class Progress(object):
    """A stderr line every 30 s with the phase the bench is in (the run is minutes long and
    its one JSON line comes at the end; runners that take a silent process for a hung one
    see it alive).  Never on stdout."""

    def __init__(self, rank):
        import threading
        self.phase, self.t0, self.rank = 'start', time.time(), rank
        self.stop = threading.Event()
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    def _run(self):
        while not self.stop.wait(30.0):
            print('[bench rank %d] %.0f s: %s' % (self.rank, time.time() - self.t0, self.phase), file=sys.stderr,
                  flush=True)

    def set(self, phase):
        self.phase = phase

    def close(self):
        self.stop.set()


PROGRESS = None


def progress(phase):
    if PROGRESS is not None:
        PROGRESS.set(phase)


def main():
    global PROGRESS
    args = parse()
    PROGRESS = Progress(int(os.environ.get('RANK', '0')))
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # RCCL ('nccl') is the product path; IGM_BENCH_BACKEND=gloo rehearses the N > 1 code on
    # one GPU (every rank on cuda:0, collectives host-staged) -- never a measurement
    backend = os.environ.get('IGM_BENCH_BACKEND', 'nccl')
    if backend != 'nccl':
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    from igm_amd.pipeline import AMIteration
    inp = build_inputs(args, rank)
    pop = inp['pop']
    it = AMIteration(dev, inp['xyz'], inp['atoms'], inp['chrom'], pop['copy_ptr'], pop['copy_idx'], inp['pairs'],
                     inp['prm'], inp['poly'], first_sid=inp['first'], rank=rank, world=world)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier(device_ids=[local]) if backend == 'nccl' else dist.barrier()
        torch.cuda.synchronize(dev)

    for w in range(args.warmup):
        progress('config %s warmup %d/%d' % (args.config, w + 1, args.warmup))
        it.step()
    barrier()
    want_cpu = args.cpu_sample != 0 and world == 1 and rank == 0
    snap = it.snapshot() if want_cpu else None  # the first timed step's input state
    anneal_ms, bytes_launch, astep_s, mstep_s = [], [], [], []
    t0 = time.perf_counter()
    for k in range(args.steps):
        progress('config %s timed step %d/%d' % (args.config, k + 1, args.steps))
        tm = it.step()
        anneal_ms.append(it.ctx.kernel_ms('anneal'))
        if os.environ.get('IGM_PROF'):  # tuning: the LDS anneal kernel's cycle profile (perturbs the timing)
            print('[prof]', json.dumps(it.ctx.mstep_profile()), file=sys.stderr, flush=True)
        bytes_launch.append(it.algorithmic_anneal_bytes())
        astep_s.append(tm['astep_s'])
        mstep_s.append(tm['mstep_s'])
    barrier()
    dt = time.perf_counter() - t0
    kms = {k: it.ctx.kernel_ms(k) for k in ('cg', 'actdist', 'actdist_select', 'hic_select', 'violations')}
    dt = max_over_ranks(dt, world, dev)
    score = it.violation_score()
    info = it.info_host()
    nrows, nbonds, S_local, npairs, npairs_total = int(it.nrows), it.nbonds, it.S_local, it.npairs, it.npairs_total
    de = cblock = astep_cpu = cpu = mde = None
    if want_cpu:
        progress('CPU baselines of config %s' % args.config)
        nth, _, _ = host_threads(args)
        astep_cpu = cpu_baseline_astep(args, it, nth, npairs=2000 * nth)
        cpu = cpu_baseline(args, it, inp, snap)
    if rank == 0 and world == 1 and not args.no_de:  # the N=1 line carries it; scaling runs stay lean
        progress('configuration D/E A-steps')
        de = bench_asteps_de(args, it.ctx)
    del it, snap
    torch.cuda.empty_cache()
    if args.config == 'B' and not args.no_c:  # every rank: the 200 kb pop=c_total population, strong split
        cblock = bench_config_c(args, dev, world, rank, local, backend)
        if world == 1 and args.c_shard > 0 and args.c_shard != args.c_total:
            cblock['shard%d' % args.c_shard] = bench_shard(args, dev)
            if not args.no_mstep_de:
                cblock['shard%d_frustrated' % args.c_shard] = bench_frustrated(args, dev, args.c_shard)
                torch.cuda.empty_cache()
    if rank == 0 and world == 1 and args.config == 'B' and not args.no_mstep_de:
        n = args.c_shard if args.c_shard > 0 else 125
        mde = {}
        for cfg in ('D', 'E'):
            mde['config_%s' % cfg] = bench_mstep_de(args, dev, cfg, n)
            torch.cuda.empty_cache()
    ms_per_step = 1000.0 * dt / max(args.steps, 1)
    total = S_local * world
    value = total * args.steps / dt
    a_ms = float(np.mean(anneal_ms)) if anneal_ms else float('nan')
    achieved = float(np.mean(bytes_launch)) / (a_ms * 1e-3) / 1e9 if anneal_ms else 0.0
    traffic, traffic_src = measured_traffic(args.config)
    if rank == 0:
        line = {
            'metric': 'M-step structures/sec + A/M iteration wall-time (BASELINE.json), %s' % (
                '2 Mb diploid pop=1000 per GPU (configs[1])' if args.config == 'B' else
                '200 kb diploid pop=%d per GPU (configs[2] shard)' % args.nstruct),
            'value': value, 'unit': 'structures/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': ms_per_step, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'f32 (MD), f64 (CG, reductions)',
            'data': 'synthetic: RandomInit territories default_rng(1000+sid), %s pairs sigma>=%g' % (
                'demo .hcs' if args.config == 'B' else 'synthetic 200 kb .hcs (SURVEY 8d)', args.sigma),
            'config': {'workload': '%s, Hi-C only, %d structures per GPU, demo protocol%s' % (
                           'B: 2 Mb diploid (3008 beads)' if args.config == 'B' else 'C: 200 kb diploid (29 838 beads)',
                           args.nstruct, '' if args.protocol_scale == 1.0 else
                           ' x%g (NOT the metric)' % args.protocol_scale),
                       'nstruct_per_gpu': S_local, 'nstruct_total': total, 'sigma': args.sigma,
                       'npairs': int(npairs_total), 'parallelism': 'structures sharded, A-step pair-sharded'},
            'roofline': {'bound': 'hbm', 'kernel': 'anneal_kernel' if args.config == 'B' else
                         'population engine (pop_integrate, pop_sort, pop_permute, pop_fill, pop_force per MD step)',
                         'achieved': achieved, 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'traffic_source': traffic_src,
                         'algorithmic_bytes_per_launch': float(np.mean(bytes_launch)),
                         'avg_launch_ms': a_ms},
            'roofline_issue': measured_issue(args.config),
            'cpu_baseline': cpu,
            'cpu_baseline_astep': astep_cpu,
            'astep_pairs_per_s': float(npairs) / (kms['actdist'] * 1e-3),
            'config_C': cblock,
            'asteps_DE': de,
            'mstep_DE': mde,
            'breakdown': {'astep_ms': 1000 * float(np.mean(astep_s)), 'mstep_ms': 1000 * float(np.mean(mstep_s)),
                          'anneal_ms': a_ms, 'cg_ms': kms['cg'],
                          'actdist_ms': kms['actdist'], 'actdist_select_ms': kms['actdist_select'],
                          'hic_select_ms': kms['hic_select'], 'violations_ms': kms['violations'],
                          'violation_score': score, 'median_final_energy_per_bead':
                              float(np.median(info['final_energy'])) / inp['atoms'].nbead,
                          'rows': nrows, 'hic_bonds_per_struct': nbonds / S_local,
                          'mean_rebuilds': float(np.mean(info['nrebuild']))},
            'excludes': 'host pair enumeration (select_pairs) and file I/O: inputs resident in HBM',
        }
        print(json.dumps(line), flush=True)
    PROGRESS.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
