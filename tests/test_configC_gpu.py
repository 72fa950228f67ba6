"""The metric's workload (BASELINE.json configs[2], SURVEY 8(d) config C: 200 kb hg38
male diploid, 29 838 beads, 1000 structures, synthetic .hcs at sigma 0.01) through the
C ABI on the MI355X:

  * the Hi-C A-step (ActivationDistanceStep.get_actdist, igm/steps/
    ActivationDistanceStep.py:336-485) on the WHOLE 1.3 M-pair list: per-pair row
    counts and the CSR row layout checked for every pair, and a seeded sample of
    20 000 pairs bit-exact against the C oracle (rows, o, pnow, ad, p);
  * the population engine (the HBM-resident M-step for structures past one CU's LDS)
    running the whole demo protocol shape (4 stages + relax + CG, step counts scaled)
    on 200 kb structures with frustrated Hi-C-like restraints, against the fp64
    oracle (population statistics) and bitwise against its own rerun.
"""
import json
import os

import numpy as np
import pytest

import oracle
import mstep_stats as MS
import stagewise as SW
from igm_amd import model as M
from igm_amd import synthetic as syn
from igm_amd._lib import pair_dtype

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def popC():
    pop = syn.population_200kb(1000)
    xyz = np.ascontiguousarray(pop['xyz'].transpose(1, 0, 2))  # (nbead, S, 3), the .hss layout
    i, j, p = syn.hic_pairs_200kb(0.01)
    return pop, xyz, i, j, p


def test_gpu_configC_actdist_every_pair(popC):
    from igm_amd import astep
    pop, xyz, i, j, p = popC
    assert xyz.shape == (29838, 1000, 3) and len(i) > 1_290_000
    rng = np.random.default_rng(2024)
    pairs = np.zeros(len(i), pair_dtype)
    pairs['i'], pairs['j'], pairs['pwish'] = i, j, p.astype(np.float64)
    pairs['plast'] = np.where(rng.uniform(size=len(i)) < 0.5, rng.uniform(0, 0.6, len(i)), 0.0)
    cp, ci, chrom = pop['copy_ptr'], pop['copy_idx'], pop['chrom']
    rows, res = astep.compute_actdist(xyz, pop['radii'], cp, ci, chrom, pairs, 2.0, 1, return_per_pair=True)
    # every pair: rows only when p > 0, then one per copy combination (zip for intra, all
    # copy pairs for inter), in CSR pair order
    nc = np.diff(cp)
    intra = chrom[i] == chrom[j]  # the reference indexes index.chrom with the haploid ids (py:398-400)
    ncomb = np.where(intra, np.minimum(nc[i], nc[j]), nc[i] * nc[j])
    want = np.where(res['p'] > 0, ncomb, 0)
    assert np.array_equal(res['nrows'], want.astype(np.int32))
    assert len(rows) == int(want.sum())
    first = np.concatenate([[0], np.cumsum(want)[:-1]])
    has = want > 0
    assert np.array_equal(rows['row'][first[has]], ci[cp[i[has]]])  # first combination: copy 0 x copy 0
    assert np.array_equal(rows['col'][first[has]], ci[cp[j[has]]])
    # ('%.4f' % p can print a p < 5e-5 as 0.0000)
    assert np.all(rows['dist'] > 0) and np.all((rows['prob'] >= 0) & (rows['prob'] <= 1))
    # a seeded 20 000-pair sample bit for bit against the oracle
    sub = np.sort(rng.choice(len(i), 20000, replace=False))
    orows, ores = oracle.actdist(xyz, pop['radii'], cp, ci, chrom, pairs[sub], 2.0, 1, nthreads=16)
    for k in ('nrows', 'o', 'pnow', 'ad', 'p'):
        a, b = res[k][sub], ores[k]
        if k in ('ad', 'p'):
            a, b = a[ores['nrows'] > 0], b[ores['nrows'] > 0]
        assert np.array_equal(a, b), k
    mine = np.concatenate([rows[first[q]:first[q] + want[q]] for q in sub if want[q] > 0])
    assert mine.tobytes() == orows.tobytes()


# ------------------------------------------------------------------ 200 kb protocol
def _model200(n, nlocal=15000, nlong=1500, seed=31):
    pop = syn.population_200kb(n, first_sid=500)
    atoms = M.Atoms(pop['radii'])
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    x = np.zeros((n, atoms.n, 3), np.float32)
    x[:, :atoms.nbead] = pop['xyz']
    per = [MS.random_contacts(atoms.radii, atoms.nbead, nlocal, nlong, seed + s) for s in range(n)]
    ptr, sb = M.concat_bonds(per)
    return atoms, poly, ptr, sb, x


def test_gpu_200kb_protocol_matches_oracle_and_reruns_bitwise():
    """16 structures of the metric's 200 kb model with frustrated Hi-C-like restraints,
    the whole demo protocol shape at x0.02 (940 MD steps + CG), the engines' DEFAULT
    Verlet skins (GPU 0.7 maxrad, oracle LAMMPS maxrad): the KS statistic of
    tests/mstep_stats.py (it rejects a 2x bond K or a 2x evfactor) does not separate
    the GPU population from the fp64 oracle's on E_pair, E_bond, E_env, E_total per
    bead, the violation fraction and the final Temp; the rerun is bitwise identical.
    (Rebuild counts differ by construction of the skins and are not compared.)"""
    from igm_amd import mstep
    n = 16
    atoms, poly, ptr, sb, x = _model200(n)
    proto = MS.scaled_protocol(syn.DEMO_PROTOCOL, 0.02)  # 4 stages + relax + CG, 940 MD steps
    prm = M.params_from_cfg({'optimization': {'optimizer_options': proto}}, [((5500.0,) * 3, 1.0)])
    seeds = M.lammps_seeds(6535, np.arange(500, 500 + n), 3)
    xg, ig = mstep.run(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    xg2, ig2 = mstep.run(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    assert np.array_equal(xg, xg2) and ig.tobytes() == ig2.tobytes()  # bitwise reproducible
    assert np.all(np.isfinite(xg)) and np.all(ig['final_energy'] < ig['einitial'])
    xo, io, _ = oracle.mstep_run(prm, x.copy(), atoms.radii, atoms.flags, poly, ptr, sb, seeds, nthreads=16)
    so = MS.population_stats(io, xo, poly, ptr, sb, atoms.nbead)
    so['env'] = io['env_energy'][:, 0] / atoms.nbead
    sg = MS.population_stats(ig, xg, poly, ptr, sb, atoms.nbead)
    sg['env'] = ig['env_energy'][:, 0] / atoms.nbead
    ok, pv = MS.same_population(sg, so, keys=('pair', 'bond', 'env', 'total', 'viol_frac', 'temp'))
    assert ok, pv
    assert np.all(ig['temp'] < 1.0)
    assert np.all(io['temp'] < 1.0)


def test_gpu_200kb_full_protocol_stagewise_matches_oracle(heartbeat):
    """The bench's own workload at the FULL protocol (lammps.py:285-356: 4 stages, each a
    relax run and an annealing run after its own 'velocity create', 47 008 MD steps, then
    min cg), on frustrated restraints, compared stage by stage with the fp64 oracle, and the
    product path's one igm_mstep_run over the whole protocol against the oracle's final
    state (tests/stagewise.py: criteria and record).

    A 200 kb population runs one warmup A/M iteration on the GPU (AMIteration); from that
    state the next iteration's A-step and selection give 16 (IGM_STAGEWISE_N) structures
    ~34 000 Hi-C bonds each, and 700 random long-range contacts per structure are added on
    top (restraints that cannot all be met: the final energies stay far from zero instead of
    reaching ~1e-11 per bead on the self-consistent synthetic .hcs alone).  Recorded in
    gpurun_out/configC_stagewise.json beside the oracle's wall time."""
    import torch
    from igm_amd.pipeline import AMIteration
    from igm_amd._lib import bond_dtype
    # 16 structures in the suite (the oracle runs one per thread on the box's 16 CPUs: 32 would
    # double its ~260 s and crowd the round-end GPU tier's 900 s); IGM_STAGEWISE_N=32 for the
    # recorded 32-structure run (profiles/r05_parity/configC_stagewise.json)
    S = 32
    n = int(os.environ.get('IGM_STAGEWISE_N', '16'))
    assert 2 <= n <= S
    pop = syn.population_200kb(S, first_sid=0)
    atoms = M.Atoms(pop['radii'])
    x = np.zeros((S, atoms.n, 3), np.float32)
    x[:, :atoms.nbead] = pop['xyz']
    chrom = np.concatenate([pop['chrom'], [-1]]).astype(np.int32)
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    proto = json.loads(json.dumps(syn.DEMO_PROTOCOL))
    prm = M.params_from_cfg({'optimization': {'optimizer_options': proto}}, [((5500.0,) * 3, 1.0)])
    i, j, p = syn.hic_pairs_200kb(0.01)
    pairs = np.zeros(len(i), pair_dtype)
    pairs['i'], pairs['j'], pairs['pwish'] = i, j, p
    dev = torch.device('cuda', 0)
    it = AMIteration(dev, x, atoms, chrom, pop['copy_ptr'], pop['copy_idx'], pairs, prm, poly)
    it.step()  # the warmup A/M iteration
    snap = it.snapshot()
    it.load_snapshot(snap)
    it.astep()
    it.select()
    torch.cuda.synchronize(dev)
    ptr = it.hic_ptr.cpu().numpy()[:n + 1].copy()
    hic = it.hic_bonds.cpu().numpy().view(bond_dtype)[:ptr[-1]].copy()
    x0 = np.ascontiguousarray(snap['xyz'].cpu().numpy()[:n])
    del it, snap
    torch.cuda.empty_cache()
    assert ptr[-1] > 1000 * n  # thousands of A-step-selected Hi-C bonds per structure
    per = [np.concatenate([hic[ptr[s]:ptr[s + 1]], MS.random_contacts(atoms.radii, atoms.nbead, 0, 700, 7000 + s)])
           for s in range(n)]
    ptr, sb = M.concat_bonds(per)
    seeds = M.lammps_seeds(6535, np.arange(n), 1)
    ok, out, (sg, so, sp) = SW.run(prm, proto, x0, atoms.radii, atoms.flags, poly, ptr, sb, seeds, atoms.nbead,
                                   'configC_stagewise')
    assert ok, out
    # frustrated: the compared final energies are far from zero (~40 per bead)
    assert np.median(so['total']) > 1e-2 and np.median(sg['total']) > 1e-2
