/*
 * ORACLE -- test infrastructure only.  Never linked into libigmhip.so; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * CPU restatement (C99, OpenMP over pairs) of the reference A-step:
 *   get_actdist           igm/steps/ActivationDistanceStep.py:336-485
 *   cleanProbability      igm/steps/ActivationDistanceStep.py:314-332
 *   task() text rows      igm/steps/ActivationDistanceStep.py:38,228-230  ("%6d %6d %10.4f %.4f")
 *   reduce() parse        igm/steps/ActivationDistanceStep.py:249        (np.genfromtxt -> f32)
 *
 * Pinned by tests/golden/actdist_golden.npz and actdist_edge.npz, which were
 * produced by running the reference itself (tests/golden/make_golden.py).
 * Unlike the GPU kernel it does the text round trip literally (snprintf/strtod)
 * and the order statistic by an explicit selection, so it is an independent
 * check of both the bisection selection and the exact decimal rounding.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int32_t i, j;
    double pwish, plast;
} o_pair;

typedef struct {
    int32_t row, col;
    float dist, prob;
} o_row;

typedef struct {
    double ad, p, pnow;
    int32_t o, nrows;
} o_result;

static double clean_probability(double pij, double pexist) {
    double pclean = (pexist < 1.0) ? (pij - pexist) / (1.0 - pexist) : pij;
    /* Python max(0, pclean) returns the int 0 unless pclean > 0 */
    return (pclean > 0.0) ? pclean : 0.0;
}

/* k-th smallest (0-based) of a[0..n): Hoare quickselect on a scratch copy */
static double select_kth(double* a, int64_t n, int64_t k) {
    int64_t lo = 0, hi = n - 1;
    while (lo < hi) {
        double pivot = a[lo + (hi - lo) / 2];
        int64_t i = lo, j = hi;
        while (i <= j) {
            while (a[i] < pivot) i++;
            while (a[j] > pivot) j--;
            if (i <= j) {
                double t = a[i];
                a[i] = a[j];
                a[j] = t;
                i++;
                j--;
            }
        }
        if (k <= j)
            hi = j;
        else if (k >= i)
            lo = i;
        else
            return a[k];
    }
    return a[k];
}

static float text_roundtrip(double x, const char* fmt) {
    char buf[64];
    snprintf(buf, sizeof(buf), fmt, x);
    return (float)strtod(buf, NULL); /* genfromtxt: float(s) then astype(f4) */
}

static void one_pair(const float* xyz, int S, const float* radii, const int32_t* copy_ptr, const int32_t* copy_idx,
                     int nhap, const int32_t* chrom, const o_pair* pr, double cr, int it_corr, double* scratch,
                     o_result* res) {
    const int i = pr->i, j = pr->j;
    res->ad = NAN;
    res->p = NAN;
    res->pnow = NAN;
    res->o = -1;
    res->nrows = 0;
    if (i == j || i < 0 || j < 0 || i >= nhap || j >= nhap) return; /* py:379-380 */
    const int a0 = copy_ptr[i], na = copy_ptr[i + 1] - a0;
    const int b0 = copy_ptr[j], nb = copy_ptr[j + 1] - b0;
    const int intra = chrom[i] == chrom[j];
    const int n = intra ? (na < nb ? na : nb) : na * nb;
    if (n <= 0) return;
    /* d_sq rows: intra zip(ii, jj); inter for k in ii: for m in jj  (py:405-436) */
    int64_t cnt = 0;
    const float rs = radii[copy_idx[a0]] + radii[copy_idx[b0]]; /* np.float32 + np.float32 */
    const double rc = cr * (double)rs;                          /* python float * f32 -> f64 (NumPy 1.x) */
    const double rcutsq = rc * rc;                              /* np.square */
    for (int c = 0; c < n; ++c) {
        const int k = intra ? copy_idx[a0 + c] : copy_idx[a0 + c / nb];
        const int m = intra ? copy_idx[b0 + c] : copy_idx[b0 + c % nb];
        for (int s = 0; s < S; ++s) {
            const float* x = xyz + ((size_t)k * S + s) * 3;
            const float* y = xyz + ((size_t)m * S + s) * 3;
            /* built with -ffp-contract=off: no FMA, left-to-right f32 as NumPy */
            const float dx = x[0] - y[0], dy = x[1] - y[1], dz = x[2] - y[2];
            const float d2 = (dx * dx + dy * dy) + dz * dz; /* np.sum(np.square(x - y), axis=1) */
            const double v = (double)d2; /* stored into the float64 d_sq array */
            scratch[(int64_t)c * S + s] = v;
            cnt += (v <= rcutsq);
        }
    }
    const int64_t nS = (int64_t)n * S;
    const double pnow = (double)cnt / (double)nS;
    double p;
    if (it_corr == 1) {
        double t = clean_probability(pnow, pr->plast);
        p = clean_probability(pr->pwish, t);
    } else {
        p = pr->pwish;
    }
    res->pnow = pnow;
    res->p = p;
    if (!(p > 0.0)) return;
    const double ox = nearbyint((double)n * p * (double)S); /* Python round(): half to even */
    const int64_t o = (ox >= (double)(nS - 1)) ? nS - 1 : (int64_t)ox;
    res->o = (int32_t)o;
    res->ad = sqrt(select_kth(scratch, nS, o));
    res->nrows = n;
}

/* returns total rows; rows written when rows != NULL and total <= cap */
int64_t oracle_actdist(const float* xyz, int32_t nbead, int32_t S, const float* radii, const int32_t* copy_ptr,
                       const int32_t* copy_idx, int32_t nhap, const int32_t* chrom, const o_pair* pairs,
                       int64_t npairs, double cr, int32_t it_corr, o_result* res, o_row* rows, int64_t cap,
                       int32_t nthreads) {
    (void)nbead;
    int maxc = 1;
    for (int h = 0; h < nhap; ++h) {
        int d = copy_ptr[h + 1] - copy_ptr[h];
        if (d > maxc) maxc = d;
    }
    const int64_t scratch_len = (int64_t)maxc * maxc * S;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
    {
        double* scratch = (double*)malloc(sizeof(double) * (size_t)scratch_len);
#pragma omp for schedule(dynamic, 64)
        for (int64_t q = 0; q < npairs; ++q)
            one_pair(xyz, S, radii, copy_ptr, copy_idx, nhap, chrom, &pairs[q], cr, it_corr, scratch, &res[q]);
        free(scratch);
    }
    int64_t total = 0;
    for (int64_t q = 0; q < npairs; ++q) total += res[q].nrows;
    if (!rows || total > cap) return total;
    int64_t w = 0;
    for (int64_t q = 0; q < npairs; ++q) {
        if (res[q].nrows <= 0) continue;
        const int i = pairs[q].i, j = pairs[q].j;
        const int a0 = copy_ptr[i], b0 = copy_ptr[j], nb = copy_ptr[j + 1] - b0;
        const int intra = chrom[i] == chrom[j];
        const float dist = text_roundtrip(res[q].ad, "%10.4f");
        const float prob = text_roundtrip(res[q].p, "%.4f");
        for (int c = 0; c < res[q].nrows; ++c) {
            rows[w].row = intra ? copy_idx[a0 + c] : copy_idx[a0 + c / nb];
            rows[w].col = intra ? copy_idx[b0 + c] : copy_idx[b0 + c % nb];
            rows[w].dist = dist;
            rows[w].prob = prob;
            ++w;
        }
    }
    return total;
}
