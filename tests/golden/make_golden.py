#!/opt/conda/bin/python3.9
"""Generate golden vectors by running the REFERENCE (bonimba87/igm) in this container.

Run ONLY in the build container (the reference is not on the GPU box):

    /opt/conda/bin/python3.9 tests/golden/make_golden.py

It needs /opt/conda/bin/python3.9 (numpy 1.26 -- the reference's NumPy-1.x
promotion rules -- plus h5py and Cython 0.29) and /root/reference.  The
reference is imported exactly as SURVEY.md section 8(c) describes: a stub
`alabtools` package that only satisfies imports (no alabtools arithmetic is
used: get_actdist receives a duck-typed hss) and the reference's own Cython
SPRITE extension compiled from /root/reference/igm/cython_compiled into
/tmp.  Nothing from the reference is written into the repository except the
numerical inputs/outputs below (fixtures = data).

Fixtures written to tests/golden/:
  demo_population.npz   demo .hss.T coordinates (3008,100,3) f32, radii, index,
                        copy_index CSR, hcs haploid chrom, summary energy pins (G7)
  demo_hic_pairs.npz    upper-triangle .hcs entries with p >= 0.02 in CSR order,
                        plus a 20k-entry subset of 0.01 <= p < 0.02
  actdist_golden.npz    G1: reference get_actdist on the demo population
                        (sigma 1.0/0.2/0.05/0.02 x it_corr 0/1, plast chained;
                        sigma 0.01 on the 20k subset), after the "%10.4f %.4f"
                        text round trip exactly as ActivationDistanceStep.reduce
  actdist_edge.npz      G2: synthetic edge cases (ties, coincident beads,
                        single-copy loci, banker's rounding at .5, plast>=1, ...)
  mstep_inputs.npz      G3/G4: reference LammpsModel for demo structures 0..9
                        at sigma=0.02 (bond lists, bond types, PairIJ, seeds)
                        and the .lam protocol script text of structure 0
  violations_golden.npz G6: reference violation ratios / histograms (M9)
  sprite_golden.npz     G5: reference get_rgs2 (Cython+C++) on demo coordinates
"""
import os
import sys
import json
import importlib.util
import tempfile
import subprocess
import shutil

# never write anything (bytecode, generated C++) under the read-only reference
sys.dont_write_bytecode = True

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'
ORACLE_TMP = '/tmp/igm_ref_oracle'


def _build_reference_env():
    """Stub alabtools + build the reference Cython extension into /tmp."""
    stubs = os.path.join(ORACLE_TMP, 'stubs', 'alabtools')
    build = os.path.join(ORACLE_TMP, 'build')
    os.makedirs(stubs, exist_ok=True)
    os.makedirs(build, exist_ok=True)
    files = {
        '__init__.py': 'class Contactmatrix(object):\n    pass\n',
        'analysis.py': ('import numpy as np\nCOORD_DTYPE = np.float32\n'
                        'class HssFile(object):\n    pass\n'
                        'def get_simulated_hic(*a, **k):\n    raise NotImplementedError\n'),
        'utils.py': 'Genome = Index = make_diploid = make_multiploid = natural_sort = None\n',
        'plots.py': 'plot_comparison = red = plot_by_chromosome = None\n',
    }
    for k, v in files.items():
        with open(os.path.join(stubs, k), 'w') as f:
            f.write(v)
    so = [f for f in os.listdir(build) if f.startswith('sprite') and f.endswith('.so')]
    if not so:
        # Cython writes the generated .cpp next to the .pyx: work on copies in /tmp
        src = os.path.join(build, 'src')
        os.makedirs(src, exist_ok=True)
        for fn in ('sprite.pyx', 'cpp_sprite_assignment.cpp', 'cpp_sprite_assignment.h'):
            shutil.copy(os.path.join(REF, 'igm', 'cython_compiled', fn), src)
        setup_py = os.path.join(build, 'setup_ref.py')
        with open(setup_py, 'w') as f:
            f.write(
                'import numpy\n'
                'from setuptools import setup, Extension\n'
                'from Cython.Build import cythonize\n'
                'src = %r\n'
                'ext = Extension("sprite", [src + "/sprite.pyx", src + "/cpp_sprite_assignment.cpp"],\n'
                '                language="c++", include_dirs=[numpy.get_include(), src])\n'
                'setup(ext_modules=cythonize([ext], language_level=3, build_dir=%r))\n' % (src, build))
        subprocess.check_call([sys.executable, '-B', setup_py, 'build_ext', '--inplace'], cwd=build,
                              stdout=subprocess.DEVNULL, env=dict(os.environ, PYTHONDONTWRITEBYTECODE='1'))
        so = [f for f in os.listdir(build) if f.startswith('sprite') and f.endswith('.so')]
    sys.path[:0] = [os.path.dirname(stubs), REF]
    spec = importlib.util.spec_from_file_location('igm.cython_compiled.sprite', os.path.join(build, so[0]))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    sys.modules['igm.cython_compiled.sprite'] = m
    return m


sprite_mod = _build_reference_env()

import numpy as np  # noqa: E402
import h5py  # noqa: E402
import igm  # noqa: E402,F401
from igm.steps.ActivationDistanceStep import get_actdist, actdist_fmt_str, actdist_shape  # noqa: E402
from igm.model import Model, Particle  # noqa: E402
from igm.restraints import Polymer, Envelope, Steric, intraHiC, interHiC  # noqa: E402
from igm.model.kernel import lammps as reflammps  # noqa: E402
from igm.model.kernel.lammps_model import LammpsModel  # noqa: E402
from igm.steps.ModelingStep import get_violation_histogram  # noqa: E402

assert np.__version__.startswith('1.'), 'golden vectors need NumPy 1.x promotion rules'

DEMO = os.path.join(REF, 'demo')
HSS_T = os.path.join(DEMO, 'demo_sample_outputs', 'igm-model.hss.T')
HCS = os.path.join(DEMO, 'WTC11_HiC_2Mb.hcs')


class _Index(object):
    def __init__(self, copy_index, chrom, copy=None):
        self.copy_index = copy_index
        self.chrom = chrom
        self.copy = copy

    def __len__(self):
        return len(self.chrom)


class DuckHss(object):
    """The four accessors get_actdist uses (ActivationDistanceStep.py:382-392,415-432)."""

    def __init__(self, crd, radii, copy_index, chrom):
        self.crd = crd
        self.radii = radii
        self.index = _Index(copy_index, chrom)

    def get_nstruct(self):
        return self.crd.shape[1]

    def get_index(self):
        return self.index

    def get_radii(self):
        return self.radii

    def get_bead_crd(self, k):
        return self.crd[k]


def text_roundtrip(rows):
    """ActivationDistanceStep.task writes '%6d %6d %10.4f %.4f'; reduce() reads it
    back with np.genfromtxt(dtype=actdist_shape)."""
    if len(rows) == 0:
        return np.zeros(0, dtype=actdist_shape)
    with tempfile.NamedTemporaryFile('w+', suffix='.tmp', delete=False) as f:
        f.write('\n'.join([actdist_fmt_str % x for x in rows]))
        name = f.name
    a = np.genfromtxt(name, dtype=actdist_shape)
    os.unlink(name)
    if a.ndim == 0:
        a = np.array([a], dtype=actdist_shape)
    return a


def run_pairs(hss, pairs_i, pairs_j, pwish, plast, it_corr, cr=2.0):
    """Apply the reference get_actdist to every pair; return per-pair summary and rows."""
    P = len(pairs_i)
    nrows = np.zeros(P, np.int32)
    ad64 = np.full(P, np.nan)
    p64 = np.full(P, np.nan)
    allrows = []
    for q in range(P):
        res = get_actdist(int(pairs_i[q]), int(pairs_j[q]), float(pwish[q]), float(plast[q]),
                          hss, it_corr, contactRange=cr)
        nrows[q] = len(res)
        if len(res):
            ad64[q] = float(res[0][2])
            p64[q] = float(res[0][3])
        allrows += res
    rt = text_roundtrip(allrows)
    return nrows, ad64, p64, rt


def plast_lookup(rows, n, pi, pj):
    """ActivationDistanceStep.setup:144-160 (coo -> lil, duplicates summed in f32)."""
    import scipy.sparse
    row, col, prob = rows['row'], rows['col'], rows['prob']
    ii = np.logical_and(row < n, col < n)
    m = scipy.sparse.coo_matrix((prob[ii], (row[ii], col[ii])), shape=(n, n)).tolil()
    return np.array([m[int(a), int(b)] for a, b in zip(pi, pj)], dtype=np.float64)


def main():
    out = {}
    with h5py.File(HSS_T, 'r') as f:
        crd = f['coordinates'][()]
        radii = f['radii'][()]
        chrom = f['index/chrom'][()]
        copy = f['index/copy'][()]
        chrom_sizes = f['index/chrom_sizes'][()]
        ci_json = json.loads(f['index/copy_index'][()])
        summary = json.loads(f['summary'][()])
        cfg_data = json.loads(f['config_data'][()])
    with h5py.File(HCS, 'r') as g:
        data = g['matrix/data'][()]
        indices = g['matrix/indices'][()]
        indptr = g['matrix/indptr'][()]
        hap_chrom = g['index/chrom'][()]
    nhap = len(indptr) - 1
    copy_index = {int(k): [int(x) for x in v] for k, v in ci_json.items()}
    ci_ptr = np.zeros(nhap + 1, np.int32)
    ci_idx = []
    for h in range(nhap):
        ci_idx += copy_index[h]
        ci_ptr[h + 1] = len(ci_idx)
    ci_idx = np.array(ci_idx, np.int32)
    S = crd.shape[1]
    bs = summary['bystructure']
    np.savez_compressed(
        os.path.join(HERE, 'demo_population.npz'),
        coordinates=crd, radii=radii, chrom=chrom, copy=copy, chrom_sizes=chrom_sizes,
        copy_ptr=ci_ptr, copy_idx=ci_idx, hap_chrom=hap_chrom,
        pin_pair_energies=np.array(bs['pair_energies'], np.float64),
        pin_total_energies=np.array(bs['total_energies'], np.float64),
        pin_bond_energies=np.array(bs['bond_energies'], np.float64),
        pin_f_envelope0=np.array(bs['thermo']['f_envelope0'], np.float64),
        pin_E_pair=np.array(bs['thermo']['E_pair'], np.float64),
        pin_Temp=np.array(bs['thermo']['Temp'], np.float64),
        pin_n_imposed=np.array(bs['n_imposed'], np.float64),
        pin_n_violations=np.array(bs['n_violations'], np.float64),
        summary_json=np.array(json.dumps(summary)),
        step_no=np.int64(cfg_data['runtime']['step_no']),
    )

    # ---- hcs entries, CSR (coo_generator) order ------------------------------
    ent_i = np.repeat(np.arange(nhap, dtype=np.int32), np.diff(indptr))
    ent_j = indices.astype(np.int32)
    ent_p = data.astype(np.float32)
    keep = ent_p >= 0.02
    sub01 = np.where((ent_p >= 0.01) & (ent_p < 0.02))[0]
    rng = np.random.RandomState(7)
    sub01 = np.sort(rng.choice(sub01, 20000, replace=False))
    np.savez_compressed(os.path.join(HERE, 'demo_hic_pairs.npz'),
                        i=ent_i[keep], j=ent_j[keep], p=ent_p[keep],
                        i01=ent_i[sub01], j01=ent_j[sub01], p01=ent_p[sub01],
                        diagonal=np.array([], np.float32), nhap=np.int64(nhap))

    hss = DuckHss(crd, radii, copy_index, chrom)

    def select(sig):
        m = keep & (ent_p >= sig)  # intra and inter sigma identical in the demo
        return ent_i[m], ent_j[m], ent_p[m].astype(np.float64)

    # ---- G1 ------------------------------------------------------------------
    sigmas = [1.0, 0.2, 0.05, 0.02]
    g1 = {}
    for it_corr in (0, 1):
        prev_rows = None
        for sig in sigmas:
            pi, pj, pw = select(sig)
            pl = np.zeros(len(pi)) if prev_rows is None else plast_lookup(prev_rows, nhap, pi, pj)
            nrows, ad64, p64, rt = run_pairs(hss, pi, pj, pw, pl, it_corr)
            tag = 's%g_c%d' % (sig, it_corr)
            # per-pair f32 outputs, in row order
            first = np.concatenate([[0], np.cumsum(nrows)[:-1]])
            has = nrows > 0
            d32 = np.full(len(pi), np.nan, np.float32)
            p32 = np.full(len(pi), np.nan, np.float32)
            d32[has] = rt['dist'][first[has]]
            p32[has] = rt['prob'][first[has]]
            g1[tag + '_sigma'] = np.float64(sig)
            g1[tag + '_plast'] = pl
            g1[tag + '_nrows'] = nrows.astype(np.uint8)
            g1[tag + '_dist'] = d32
            g1[tag + '_prob'] = p32
            g1[tag + '_ad64'] = ad64
            g1[tag + '_p64'] = p64
            g1[tag + '_nrows_total'] = np.int64(len(rt))
            if sig == 0.2 and it_corr == 1:
                g1[tag + '_rows_row'] = rt['row']
                g1[tag + '_rows_col'] = rt['col']
                g1[tag + '_rows_dist'] = rt['dist']
                g1[tag + '_rows_prob'] = rt['prob']
            prev_rows = rt
            print('G1', tag, len(pi), 'pairs', len(rt), 'rows', flush=True)
            if sig == 0.02 and it_corr == 0:
                rows002 = rt
    # sigma = 0.01 subset, it_corr = 1 with plast from the sigma=0.02 chain
    pi, pj, pw = ent_i[sub01], ent_j[sub01], ent_p[sub01].astype(np.float64)
    pl = plast_lookup(prev_rows, nhap, pi, pj)
    nrows, ad64, p64, rt = run_pairs(hss, pi, pj, pw, pl, 1)
    first = np.concatenate([[0], np.cumsum(nrows)[:-1]])
    has = nrows > 0
    d32 = np.full(len(pi), np.nan, np.float32)
    p32 = np.full(len(pi), np.nan, np.float32)
    d32[has] = rt['dist'][first[has]]
    p32[has] = rt['prob'][first[has]]
    g1.update({'s0.01sub_c1_plast': pl, 's0.01sub_c1_nrows': nrows.astype(np.uint8),
               's0.01sub_c1_dist': d32, 's0.01sub_c1_prob': p32,
               's0.01sub_c1_ad64': ad64, 's0.01sub_c1_p64': p64})
    print('G1 s0.01sub', len(pi), 'pairs', len(rt), 'rows', flush=True)
    np.savez_compressed(os.path.join(HERE, 'actdist_golden.npz'), **g1)

    # ---- G2: synthetic edge cases ----------------------------------------------
    g2 = make_edge_cases()
    np.savez_compressed(os.path.join(HERE, 'actdist_edge.npz'), **g2)

    # ---- G3/G4/G6: restraint assembly + LAMMPS inputs + violations -------------
    tmpd = tempfile.mkdtemp()
    actfile = os.path.join(tmpd, 'actdist.hdf5')
    with h5py.File(actfile, 'w') as h5f:
        for k in ('row', 'col', 'dist', 'prob'):
            h5f.create_dataset(k, data=rows002[k])
    with open(os.path.join(DEMO, 'config_file.json')) as fcfg:
        dcfg = json.load(fcfg)
    opt = dict(dcfg['optimization']['optimizer_options'])
    opt['write'] = opt['mdsteps']
    opt['ev_step'] = 0
    g3 = {'act_row': rows002['row'], 'act_col': rows002['col'],
          'act_dist': rows002['dist'], 'act_prob': rows002['prob']}
    idx = _Index(copy_index, chrom, copy)
    chain_ids = np.concatenate([[i] * s for i, s in enumerate(chrom_sizes)])
    vs_all = {}
    for sid in range(10):
        model = Model(uid=sid)
        for i in range(crd.shape[0]):
            model.addParticle(crd[i, sid], radii[i], Particle.NORMAL, chainID=chain_ids[i])
        ex = Steric(1.0)
        model.addRestraint(ex)
        pp = Polymer(idx, 2.0, 1.0, contact_probabilities=None)
        model.addRestraint(pp)
        ev = Envelope('sphere', 5500, 1.0)
        model.addRestraint(ev)
        inter = interHiC(actfile, chrom, 2.0, 1.0)
        model.addRestraint(inter)
        intra = intraHiC(actfile, chrom, 2.0, 1.0)
        model.addRestraint(intra)
        # G4: selected actdist rows (the reference iterates the file in order)
        sel_inter = [(model.forces[f].i, model.forces[f].j) for f in inter.forceID]
        sel_intra = [(model.forces[f].i, model.forces[f].j) for f in intra.forceID]
        g3['sel_inter_%d' % sid] = np.array(sel_inter, np.int32).reshape(-1, 2)
        g3['sel_intra_%d' % sid] = np.array(sel_intra, np.int32).reshape(-1, 2)
        # G6: violation statistics exactly as ModelingStep.task:520-554 (tol = 0.05)
        vstat = {}
        for r in [pp, ev, inter, intra]:
            vs = []
            n_imposed = 0
            for fid in r.forceID:
                f = model.forces[fid]
                n_imposed += f.rnum
                if f.rnum > 1:
                    vs += f.getViolationRatios(model.particles).tolist()
                else:
                    vs.append(f.getViolationRatio(model.particles))
            vs = np.array(vs)
            H, edges = get_violation_histogram(vs)
            vstat[repr(r)] = {'counts': H.tolist(), 'violated_restr': int(np.count_nonzero(vs)),
                              'n_violations': int(np.count_nonzero(vs > 0.05)), 'n_imposed': int(n_imposed)}
            vs_all['vs_%s_%d' % (repr(r).split('[')[0], sid)] = vs.astype(np.float64)
        g3['vstat_%d' % sid] = np.array(json.dumps(vstat))
        if sid < 2:
            # G3: the LAMMPS .data / .lam the reference would hand to lmp_serial
            m = LammpsModel(model)
            run_opts = dict(opt)
            run_opts.update(dcfg['optimization']['kernel_opts']['lammps'])
            run_opts.update({'out': os.path.join(tmpd, 'o.lammpstrj'),
                             'data': os.path.join(tmpd, 'm.data'),
                             'lmp': os.path.join(tmpd, 'm.lam'),
                             'step_no': 11 + 2})
            reflammps.create_lammps_data(m, run_opts)
            reflammps.create_lammps_script(m, run_opts)
            with open(run_opts['data']) as fd:
                g3['data_text_%d' % sid] = np.array(fd.read())
            with open(run_opts['lmp']) as fl:
                g3['lam_text_%d' % sid] = np.array(fl.read())
            bonds = np.array([(b.i.id, b.j.id, b.bond_type.id) for b in m.bonds], np.int32)
            btypes = [(bt.style_id, bt.k, bt.r0) for bt in sorted(m.bond_types.values(), key=lambda x: x.id)]
            g3['bonds_%d' % sid] = bonds
            g3['bond_types_%d' % sid] = np.array(btypes, np.float64).reshape(-1, 3)
        print('G3/G4/G6 structure', sid, len(sel_inter), len(sel_intra), flush=True)
    np.savez_compressed(os.path.join(HERE, 'mstep_inputs.npz'), **g3)
    np.savez_compressed(os.path.join(HERE, 'violations_golden.npz'), **vs_all)

    # ---- G5: SPRITE get_rgs2 ---------------------------------------------------
    g5 = make_sprite_cases(crd, copy_index)
    np.savez_compressed(os.path.join(HERE, 'sprite_golden.npz'), **g5)
    print('done')


def make_edge_cases():
    """G2 -- synthetic populations exercising every branch of get_actdist."""
    g = {}
    rng = np.random.RandomState(1234)
    cases = []
    # case A: S=5, diploid intra + inter, random coordinates
    for S in (5, 16, 64, 1000):
        nb = 8  # haploid loci 0..3 chrom 0, 4..7 chrom 1; copies at +8
        copy_index = {h: [h, h + nb] for h in range(nb)}
        for h in range(4, 8):  # chromosome 1 is single-copy, like chrX in a male genome
            copy_index[h] = [h]  # (the reference reads uninitialised memory for an intra
                                 #  pair whose loci have different copy numbers)
        chrom = np.array([0, 0, 0, 0, 1, 1, 1, 1] * 2, np.int32)
        crd = (rng.rand(2 * nb, S, 3).astype(np.float32) * 2000.0).astype(np.float32)
        if S == 16:
            crd[1] = crd[0]  # coincident beads: d2 == 0
            crd[9] = crd[8]
            crd[2, :, :] = crd[0, :, :] + np.float32(100.0)  # exact ties across structures
        radii = np.full(2 * nb, 100.0, np.float32)
        cases.append((S, crd, radii, copy_index, chrom))
    pairs = [(0, 1), (0, 2), (1, 3), (0, 4), (2, 7), (6, 7), (3, 5), (0, 0)]
    for ci, (S, crd, radii, copy_index, chrom) in enumerate(cases):
        hss = DuckHss(crd, radii, copy_index, chrom)
        for it_corr in (0, 1):
            pw_list, pl_list, pi_list, pj_list = [], [], [], []
            for (a, b) in pairs:
                for pw, pl in ((0.5, 0.0), (0.25, 0.1), (1.0, 1.0), (0.3, 1.5), (0.05, 0.9), (0.7, 0.2)):
                    pi_list.append(a)
                    pj_list.append(b)
                    pw_list.append(np.float64(np.float32(pw)))
                    pl_list.append(np.float64(np.float32(pl)))
            # banker's rounding: n*p*S == k + 0.5 exactly (n=2, S=5 -> p = 0.45 gives 4.5)
            if S == 5:
                for (a, b, pw) in ((0, 1, 0.45), (0, 1, 0.25), (0, 1, 0.35), (0, 4, 0.125), (0, 4, 0.375)):
                    pi_list.append(a)
                    pj_list.append(b)
                    pw_list.append(pw)  # exact doubles, not via f32
                    pl_list.append(0.0)
            nrows, ad64, p64, rt = run_pairs(hss, pi_list, pj_list, pw_list, pl_list, it_corr)
            tag = 'c%d_i%d' % (ci, it_corr)
            g[tag + '_pi'] = np.array(pi_list, np.int32)
            g[tag + '_pj'] = np.array(pj_list, np.int32)
            g[tag + '_pwish'] = np.array(pw_list, np.float64)
            g[tag + '_plast'] = np.array(pl_list, np.float64)
            g[tag + '_nrows'] = nrows
            g[tag + '_ad64'] = ad64
            g[tag + '_p64'] = p64
            g[tag + '_row'] = rt['row']
            g[tag + '_col'] = rt['col']
            g[tag + '_dist'] = rt['dist']
            g[tag + '_prob'] = rt['prob']
        g['c%d_crd' % ci] = crd
        g['c%d_radii' % ci] = radii
        g['c%d_chrom' % ci] = chrom
        ptr = [0]
        idx = []
        for h in range(8):
            idx += copy_index[h]
            ptr.append(len(idx))
        g['c%d_copy_ptr' % ci] = np.array(ptr, np.int32)
        g['c%d_copy_idx' % ci] = np.array(idx, np.int32)
    g['ncases'] = np.int64(len(cases))
    return g


def make_sprite_cases(crd, copy_index):
    """G5 -- the reference Cython/C++ get_rgs2 (sprite.pyx:36-101 -> cpp:79-143)."""
    g = {}
    get_rgs2 = sprite_mod.get_rgs2
    # the reference's own known-answer tests (igm/cython_compiled/tests.py)
    rng = np.random.RandomState(5)
    cases = []
    for ci, loci in enumerate([[0, 1, 2], [10, 11], [100, 200, 300, 400], [1556, 1557], [5, 6, 7, 8, 9, 10]]):
        nloc = len(loci)
        copies = [copy_index[h] for h in loci]
        beads = [b for c in copies for b in c]
        sub = crd[beads][:, :, :].astype(np.float32)  # (B_alt, S, 3) bead-major
        ncopies = np.array([len(c) for c in copies], np.int32)
        rg2s, best_struct, copy_idxs = get_rgs2(np.ascontiguousarray(sub), ncopies)
        g['s%d_loci' % ci] = np.array(loci, np.int32)
        g['s%d_beads' % ci] = np.array(beads, np.int32)
        g['s%d_ncopies' % ci] = ncopies
        g['s%d_rg2s' % ci] = np.asarray(rg2s)
        g['s%d_best' % ci] = np.int64(best_struct)
        g['s%d_copy_idxs' % ci] = np.asarray(copy_idxs)
        cases.append(ci)
    g['ncases'] = np.int64(len(cases))
    # the three cases of igm/cython_compiled/tests.py (their expected values are
    # written there as comments; the reference output is stored, not the comments)
    kat = [
        (np.array([[[1, 0, 0]], [[-1, 0, 0]], [[0, -1, 0]], [[0, 1, 0]]], np.float32), [1, 1, 1, 1]),
        (np.array([[[1, 0, 0]], [[0.5, 0, 0]], [[0, -0.5, 0]], [[0, 0.5, 0]]], np.float32), [2, 2]),
        (np.array([[[1, 0, 0], [0.1, 0, 0]], [[0.5, 0, 0], [1, 0, 0]], [[0, -0.5, 0], [-1, 0, 0]],
                   [[0, 0.5, 0], [-0.1, 0, 0]]], np.float32), [2, 2]),
    ]
    for q, (c, cn) in enumerate(kat):
        cn = np.array(cn, np.int32)
        rg2s, best, cidx = get_rgs2(c, cn)
        g['kat%d_crd' % q] = c
        g['kat%d_ncopies' % q] = cn
        g['kat%d_rg2s' % q] = np.asarray(rg2s)
        g['kat%d_best' % q] = np.int64(best)
        g['kat%d_copy_idxs' % q] = np.asarray(cidx)
    g['nkat'] = np.int64(len(kat))
    return g


if __name__ == '__main__':
    main()
