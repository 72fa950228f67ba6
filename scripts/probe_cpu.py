"""Probe the GPU box's host CPUs for the cpu_baseline leg: affinity, cgroup quota,
and the fp64 oracle's throughput at 16 / 64 / 128 / all threads (one config B
structure per thread, protocol x0.01).  Not a test; run under gpurun."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def read(p):
    try:
        with open(p) as fh:
            return fh.read().strip()
    except OSError as e:
        return 'n/a (%s)' % e.__class__.__name__


def main():
    import oracle
    from igm_amd import model as M, synthetic as syn
    aff = len(os.sched_getaffinity(0))
    print(json.dumps({'affinity': aff, 'cpu_count': os.cpu_count(), 'cpu.max': read('/sys/fs/cgroup/cpu.max'),
                      'cpuset': read('/sys/fs/cgroup/cpuset.cpus.effective'),
                      'pids.max': read('/sys/fs/cgroup/pids.max'),
                      'cgroup': read('/proc/self/cgroup'),
                      'cfs_quota': read('/sys/fs/cgroup/cpu/cpu.cfs_quota_us'),
                      'cfs_period': read('/sys/fs/cgroup/cpu/cpu.cfs_period_us'),
                      'model': [l for l in read('/proc/cpuinfo').splitlines() if l.startswith('model name')][:1],
                      'OMP_NUM_THREADS': os.environ.get('OMP_NUM_THREADS')}), flush=True)
    nmax = aff
    pop = syn.population_2mb(nmax)
    atoms = M.Atoms(pop['radii'])
    x = np.zeros((nmax, atoms.n, 3), np.float32)
    x[:, :pop['xyz'].shape[1]] = pop['xyz']
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    proto = json.loads(json.dumps(syn.DEMO_PROTOCOL))
    cap = proto['custom_annealing_protocol']
    sc = float(os.environ.get('PROBE_SCALE', '0.01'))
    cap['mdsteps'] = [max(1, int(round(n * sc))) for n in cap['mdsteps']]
    cap['relax']['mdsteps'] = max(1, int(round(cap['relax']['mdsteps'] * sc)))
    prm = M.params_from_cfg({'optimization': {'optimizer_options': proto}}, [((5500.0,) * 3, 1.0)])
    seeds = M.lammps_seeds(6535, np.arange(nmax), 0)
    for n in sorted({1, 16, 64, 128, nmax}):
        if n > nmax:
            continue
        t0 = time.perf_counter()
        oracle.mstep_run(prm, x[:n].copy(), atoms.radii, atoms.flags, poly, None, None, seeds[:n], nthreads=n)
        dt = time.perf_counter() - t0
        print(json.dumps({'threads': n, 'structures': n, 's': round(dt, 3), 'per_s': n / dt}), flush=True)


if __name__ == '__main__':
    main()
