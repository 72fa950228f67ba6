"""Stage-resolved full-protocol comparison of the GPU population engine with the fp64
oracle (test helper for tests/test_configC_gpu.py and tests/test_configDE_gpu.py).

The protocol of create_lammps_script (igm/model/kernel/lammps.py:285-356): per stage a
relax run and an annealing run, each after its own 'velocity create', then 'min cg'.
Both engines run every segment from the same coordinates with the same velocities --
RanPark 'velocity create' with the seed the product path derives for that stage
(igm_mstep_run: the structure's LAMMPS seed + the stage index) -- the GPU through
igm_mstep_md, the oracle through its fp64 MD; after each stage's annealing run the
energies (E_pair, E_bond, every envelope's E per bead, each engine's state evaluated by its
own force routine) and the temperature are recorded (the per-run thermo the reference
reads back, lammps_io.py:6-37); the final CG follows (igm_mstep_run / the oracle with no
MD stage).  Besides, the PRODUCT path -- one igm_mstep_run over the whole protocol, the
velocities created in-engine -- runs from the same start and seeds, and its final state
is compared with the oracle's.

Criteria (alpha = 1e-3 throughout):
  * energies of every stage and of the final states: two-sample KS and the paired
    Wilcoxon signed-rank test over the n structures (the pairing removes the
    structure-to-structure spread, so a systematic difference of a few per cent shows);
  * temperature: |T_gpu - T_oracle| <= min(2 window, 0.1 + 0.05 T1) for every structure
    (temp/rescale holds T within its window of the target T1; the bound tightens as T1
    falls), and in the stages whose target is below 10 windows (T1 = 1, 0: there the
    dynamics, not the rescale, set T) also KS and Wilcoxon.
Per-structure atom flags (DamID membership, SPRITE centroid slots) go to the oracle one
structure at a time on a thread pool (its MD and force entry points take shared flags).
"""
import json
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import mstep_stats as MS
import oracle
from igm_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALPHA = 1e-3


def paired(a, b):
    """Wilcoxon signed-rank p-value of a - b and the median relative difference"""
    from scipy import stats
    d = a - b
    p = float(stats.wilcoxon(d).pvalue) if np.any(d != 0) else 1.0
    return p, float(np.median(d / np.maximum(np.abs(b), 1e-30)))


class Oracle(object):
    """the fp64 oracle's MD / forces / velocities with shared (N,) or per-structure (S, N)
    flags; per-structure flags run one structure per pool thread"""

    def __init__(self, prm, radii, flags, poly, ptr, sb, nthreads=16):
        self.prm, self.radii, self.flags, self.poly, self.ptr, self.sb = prm, radii, flags, poly, ptr, sb
        self.nth = nthreads
        self.per = flags.ndim == 2

    def _one(self, s):
        a, b = int(self.ptr[s]), int(self.ptr[s + 1])
        return self.flags[s], np.array([0, b - a], np.int64), self.sb[a:b]

    def velocities(self, n, t, seeds):
        return np.stack([oracle.velocity_create(self.flags[s] if self.per else self.flags, t, int(seeds[s]))
                         for s in range(n)])

    def md(self, x, v, evf, envf, t0, t1, xmax, nst):
        if not self.per:
            return oracle.mstep_md(self.prm, x, v, self.radii, self.flags, self.poly, self.ptr, self.sb, evf, envf,
                                   t0, t1, xmax, nst, nthreads=self.nth)

        def job(s):
            fl, p, b = self._one(s)
            return oracle.mstep_md(self.prm, x[s:s + 1], v[s:s + 1], self.radii, fl, self.poly, p, b, evf, envf, t0,
                                   t1, xmax, nst, nthreads=1)
        with ThreadPoolExecutor(self.nth) as ex:
            res = list(ex.map(job, range(x.shape[0])))
        return np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])

    def forces(self, x, evf, envf):
        if not self.per:
            return oracle.mstep_forces(self.prm, x, self.radii, self.flags, self.poly, self.ptr, self.sb, evf, envf)
        res = []
        for s in range(x.shape[0]):
            fl, p, b = self._one(s)
            res.append(oracle.mstep_forces(self.prm, x[s:s + 1], self.radii, fl, self.poly, p, b, evf, envf))
        return np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])


def run(prm, proto, x0, radii, flags, poly, ptr, sb, seeds, nbead, name, nthreads=16, ctx=None):
    """The stage-wise comparison (module docstring) of n = len(seeds) structures; returns
    (ok, record).  The record also goes to gpurun_out/<name>.json."""
    from scipy import stats as st
    from igm_amd import mstep
    n = len(seeds)
    cap = proto['custom_annealing_protocol']
    rlx = cap['relax']
    flags = np.asarray(flags, np.uint32)
    O = Oracle(prm, radii, flags, poly, ptr, sb, nthreads)
    fl_mob = flags if flags.ndim == 2 else flags[None, :]
    dof = 3.0 * np.count_nonzero((fl_mob & _lib.IGM_ATOM_FIXED) == 0, axis=1) - 3.0
    nenv = prm.nenvelopes
    xg, xo = x0.copy(), x0.astype(np.float64)
    stages, t_oracle = [], 0.0
    for k in range(cap['num_steps']):
        evf = prm.evfactor_base * cap['evfactors'][k]
        envf = cap['envelope_factors'][k]
        segs = [(rlx['temperature'], rlx['temperature'], rlx['max_velocity'], rlx['mdsteps']),
                (cap['tstarts'][k], cap['tstops'][k], proto['max_velocity'], cap['mdsteps'][k])]
        for (t0, t1, xmax, nst) in segs:
            v = O.velocities(n, t0, seeds + k)  # igm_mstep_run's seed of stage k
            xg, vg = mstep.md(prm, xg, v.astype(np.float32), radii, flags, poly, ptr, sb, evf, envf, t0, t1, xmax,
                              nst, ctx=ctx)
            t = time.perf_counter()
            xo, vo = O.md(xo, v, evf, envf, t0, t1, xmax, nst)
            t_oracle += time.perf_counter() - t
        _, eg = mstep.forces(prm, xg, radii, flags, poly, ptr, sb, evf, envf, ctx=ctx)
        _, eo = O.forces(xo.astype(np.float32), evf, envf)
        rec = {}
        for key, col in [('pair', 1), ('bond', 2)] + [('env%d' % e, 3 + e) for e in range(nenv)]:
            rec[key] = (eg[:, col] / nbead, eo[:, col] / nbead)
        rec['temp'] = ((vg.astype(np.float64) ** 2).sum(axis=(1, 2)) / dof, (vo ** 2).sum(axis=(1, 2)) / dof)
        stages.append((cap['tstops'][k], rec))
    prm0 = _lib.MStepParams.from_buffer_copy(prm)
    prm0.nstages = 0  # the final min cg alone
    cg_seeds = np.arange(n, dtype=np.int32) + 1
    xg, ig = mstep.run(prm0, xg, radii, flags, poly, ptr, sb, cg_seeds, ctx=ctx)
    t = time.perf_counter()
    xof, io, _ = oracle.mstep_run(prm0, xo.astype(np.float32), radii, flags, poly, ptr, sb, cg_seeds,
                                  nthreads=nthreads)
    t_oracle += time.perf_counter() - t
    # the product path: one igm_mstep_run of the whole protocol from the same start and seeds
    xp, ip = mstep.run(prm, x0, radii, flags, poly, ptr, sb, seeds, ctx=ctx)
    shared = poly
    sg = MS.population_stats(ig, xg, shared, ptr, sb, nbead)
    so = MS.population_stats(io, xof, shared, ptr, sb, nbead)
    sp = MS.population_stats(ip, xp, shared, ptr, sb, nbead)
    out = {'test': name, 'structures': n, 'oracle_threads': nthreads, 'oracle_s': t_oracle,
           'bonds_per_structure': float(ptr[-1]) / n, 'alpha': ALPHA, 'stages': []}
    ok = True
    window = prm.t_window
    for t1, rec in stages:
        row = {'T1': t1}
        for key, (a, b) in rec.items():
            ks = float(st.ks_2samp(a, b).pvalue)
            pw, rel = paired(a, b)
            row[key] = {'gpu_median': float(np.median(a)), 'oracle_median': float(np.median(b)), 'ks_p': ks,
                        'wilcoxon_p': pw, 'median_rel_diff': rel}
            if key == 'temp':
                bound = min(2.0 * window, 0.1 + 0.05 * t1)
                row[key]['max_abs_diff'] = float(np.abs(a - b).max())
                row[key]['bound'] = bound
                ok = ok and np.abs(a - b).max() <= bound + 1e-6
                if t1 < 10.0 * window:  # the dynamics set T here: compared as the energies are
                    ok = ok and ks > ALPHA and pw > ALPHA
            else:
                ok = ok and ks > ALPHA and pw > ALPHA
        out['stages'].append(row)
    for label, s_gpu in (('final', sg), ('product_final', sp)):
        blk = {}
        for key in ('pair', 'bond', 'total', 'viol_frac'):
            ks = float(st.ks_2samp(s_gpu[key], so[key]).pvalue)
            pw, rel = paired(s_gpu[key], so[key])
            blk[key] = {'gpu_median': float(np.median(s_gpu[key])), 'oracle_median': float(np.median(so[key])),
                        'ks_p': ks, 'wilcoxon_p': pw, 'median_rel_diff': rel}
            ok = ok and ks > ALPHA and pw > ALPHA
        out[label] = blk
    out['final_total_median'] = {'gpu': float(np.median(sg['total'])), 'oracle': float(np.median(so['total'])),
                                 'product': float(np.median(sp['total']))}
    print('[stagewise]', json.dumps(out))
    d = os.path.join(os.environ.get('GRAFT_REPO_ROOT', ROOT), 'gpurun_out')
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, name + '.json'), 'w') as fh:
        json.dump(out, fh, indent=1)
    return ok, out, (sg, so, sp)
