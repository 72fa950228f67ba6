"""The M-step on the demo, against the summary the reference wrote for it
(demo/demo_sample_outputs/igm-model.hss.T -> summary): the
100 demo structures, the reference's sigma = 0.02 Hi-C rows (G3), the demo protocol,
polymer + sphere envelope + Hi-C, through the GPU selection, anneal/CG and violation
kernels.

The reference's M-step that wrote the summary started from the sigma = 0.05 population
(not shipped), in which the newly imposed sigma = 0.02 contacts were still far apart:
47 of its 100 structures ended trapped at E > 1 (up to 5e5).  This one starts from the
final structures, which already satisfy them, so the trapped fraction is not comparable
and only bounded; what is compared, with the tolerances stated here:

  * n_imposed per structure: mean within 2 % of the summary's (14 439), spread within
    a factor 2 (206);
  * violation fraction (ModelingStep tolerance 0.05) <= 1e-4 (the summary: 3 of
    1 443 907 = 2.1e-6);
  * the converged structures' total energies (E < 1: the CG end state, etol 1e-4 /
    ftol 1e-6): two-sample KS test against the summary's converged structures at
    alpha = 1e-3 (the summary: 53 structures, quantiles 10/50/90 % = 4.3e-9 / 1.6e-3 /
    2.5e-2);
  * the trapped fraction no larger than the summary's 0.47 (+0.1).
"""
import json

import numpy as np
import pytest
from scipy import stats

import mstep_fixtures as F
from igm_amd import model as M

pytestmark = pytest.mark.gpu


def test_gpu_demo_population_matches_reference_summary():
    from igm_amd import mstep as ms
    pop, g3 = F.load()
    ref = json.loads(str(pop['summary_json']))['bystructure']
    S = pop['coordinates'].shape[1]
    sids = list(range(S))
    atoms, poly, prm, chrom = F.demo_model(pop)
    x = F.struct_major(pop, sids, atoms.n)
    ptr, sb, scls = ms.hic_select(x, atoms.radii, chrom, g3['act_row'], g3['act_col'], g3['act_dist'])
    seeds = M.lammps_seeds(6535, sids, int(pop['step_no']))
    xg, ig = ms.run(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    assert np.all(np.isfinite(xg))
    shared_cls = np.full(len(poly), M.CLASS_POLYMER, np.int32)
    st = ms.violations(prm, xg, atoms.radii, atoms.flags, poly, shared_cls, ptr, sb, scls,
                       np.array([2.0, 2.0, 2.0]), [550.0], 0.05)
    n_imposed = st[:, :, 103].sum(axis=1).astype(np.float64)  # every class, as the summary counts
    ref_imp = np.asarray(ref['n_imposed'], np.float64)
    assert abs(n_imposed.mean() / ref_imp.mean() - 1.0) < 0.02, (n_imposed.mean(), ref_imp.mean())
    assert 0.5 < n_imposed.std() / ref_imp.std() < 2.0, (n_imposed.std(), ref_imp.std())
    viol = st[:, :, 102].sum() / max(1, st[:, :, 103].sum())
    assert viol <= 1e-4, viol
    e = ig['final_energy']
    e_ref = np.asarray(ref['total_energies'], np.float64)
    lo, lo_ref = e[e < 1.0], e_ref[e_ref < 1.0]
    assert len(lo) >= 20
    p = stats.ks_2samp(lo, lo_ref).pvalue
    assert p > 1e-3, (p, np.percentile(lo, [10, 50, 90]), np.percentile(lo_ref, [10, 50, 90]))
    assert (e >= 1.0).mean() <= (e_ref >= 1.0).mean() + 0.1, ((e >= 1.0).mean(), (e_ref >= 1.0).mean())
