// A-step: activation distances for every kept haploid pair, bit-exact with the
// reference get_actdist (igm/steps/ActivationDistanceStep.py:336-485) followed
// by the '%10.4f %.4f' text round trip of task()/reduce() (py:38,228-230,249).
//
// Layout: xyz is the .hss 'coordinates' dataset, bead-major (nbead, nstruct, 3)
// f32 (core/step.py:373, _preprocess.py:103-105), so the S structures of one
// bead are one contiguous 12*S-byte column: a wave reads a column coalesced.
//
// One 64-lane wavefront per pair.  Lane l owns structures s = l, l+64, ...; the
// n*S squared distances (n = copy combinations) stay in VGPRs (VPL per lane).
// count(d2 <= rcut2) and the o-th order statistic are wave-wide ballot+popcount
// reductions: the o-th smallest d2 is found by bisection on the IEEE bit
// pattern (d2 >= 0, so uint order == float order), which is exact and needs no
// sort.  This file is compiled with -ffp-contract=off: every f32/f64 operation
// rounds exactly like the NumPy/CPython expressions it restates.
#include <hipcub/hipcub.hpp>

#include "exact_math.h"
#include "igm_ctx.h"

namespace {

constexpr int kWavesPerBlock = 4;
// buckets: 0..6 one wave per pair with VPL 1..64 keys per lane; 7 unsupported;
// 8 no combination; 9..12 one 1024-thread workgroup per pair with VPL 8..64
// keys per thread (populations too large for one wave's registers).
constexpr int kBuckets = 13;
constexpr int kBlockThreads = 1024;

__device__ __forceinline__ int pair_ncomb(const int* copy_ptr, const int* chrom, int i, int j, int nhap, int* na,
                                          int* nb, bool* intra) {
    if (i < 0 || j < 0 || i >= nhap || j >= nhap || i == j) return 0;
    *na = copy_ptr[i + 1] - copy_ptr[i];
    *nb = copy_ptr[j + 1] - copy_ptr[j];
    *intra = chrom[i] == chrom[j];
    // ActivationDistanceStep.py:405-436: intra = zip(ii, jj); inter = all |ii|*|jj|
    return *intra ? min(*na, *nb) : (*na) * (*nb);
}

__global__ void classify_kernel(const igm_pair* __restrict__ pairs, int64_t npairs, const int* __restrict__ copy_ptr,
                                const int* __restrict__ chrom, int nhap, int S, int* __restrict__ counts,
                                int* __restrict__ lists) {
    int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npairs) return;
    int na = 0, nb = 0;
    bool intra = false;
    int n = pair_ncomb(copy_ptr, chrom, pairs[q].i, pairs[q].j, nhap, &na, &nb, &intra);
    int b;
    if (n <= 0) {
        b = 8;
    } else {
        const int64_t need = (int64_t)n * ((S + 63) / 64);
        const int64_t keys = (int64_t)n * S;
        b = 7;
        for (int k = 0, v = 1; k < 7; ++k, v <<= 1)
            if (need <= v) {
                b = k;
                break;
            }
        if (b == 7)
            for (int k = 0, v = 8; k < 4; ++k, v <<= 1)
                if (keys <= (int64_t)kBlockThreads * v) {
                    b = 9 + k;
                    break;
                }
    }
    // Wave-aggregated append: the lanes of a wave that share a bucket take one
    // atomicAdd per bucket (the wave's leader adds their count) and their ranks from
    // mbcnt, instead of one atomic per pair -- with 1.3 M pairs over 13 counters the
    // per-thread atomics serialised in L2 (14.7 of the 16.3 ms config C A-step).
    // The order inside a bucket list does not matter: results are stored by pair index.
    uint64_t todo = __ballot(1);
    while (todo) {
        const int lead = __ffsll((unsigned long long)todo) - 1;
        const int lb = __shfl(b, lead);
        const uint64_t mask = __ballot(b == lb);
        int base = 0;
        if ((int)(threadIdx.x & 63) == lead) base = atomicAdd(&counts[lb], __popcll(mask));
        base = __shfl(base, lead);
        if (b == lb) {
            const int rank = __popcll(mask & ((1ull << (threadIdx.x & 63)) - 1ull));
            lists[(int64_t)lb * npairs + base + rank] = (int)q;
        }
        todo &= ~mask;
    }
}

using igm::sqrt_rn;

// CPython '%.4f' % x (exact decimal rounding of the binary value, ties to even)
// then float('...') -> nearest double of k/10^4, which IEEE division gives.
__device__ __forceinline__ double round_dec4(double x) {
    if (!isfinite(x)) return x;
    const double hi = x * 10000.0;
    const double lo = fma(x, 10000.0, -hi);  // exact product error
    double r = rint(hi);
    const double t = hi - r;  // exact
    const double u = (t - 0.5) + lo;
    const double w = (t + 0.5) + lo;
    if (u > 0.0) {
        r += 1.0;
    } else if (u == 0.0) {
        if (fmod(r, 2.0) != 0.0) r += 1.0;
    } else if (w < 0.0) {
        r -= 1.0;
    } else if (w == 0.0) {
        if (fmod(r, 2.0) != 0.0) r -= 1.0;
    }
    return r / 10000.0;
}

// cleanProbability (ActivationDistanceStep.py:314-332)
__device__ __forceinline__ double clean_prob(double pij, double pexist) {
    double pc = (pexist < 1.0) ? (pij - pexist) / (1.0 - pexist) : pij;
    return pc > 0.0 ? pc : 0.0;  // Python max(0, pc): 0 when pc <= 0 (or NaN)
}

// rcutsq = (cr*(ri+rj))^2: ri+rj in f32, the rest in f64 (NumPy 1.x scalar
// promotion, py:393-396); returns the largest float key f with (double)f <= rcutsq,
// so that  d2 <= f  <=>  (double)d2 <= rcutsq.
__device__ __forceinline__ uint32_t cut_key(const float* radii, const int* copy_idx, int a0, int b0, double cr) {
    const float rsum = __fadd_rn(radii[copy_idx[a0]], radii[copy_idx[b0]]);
    const double rc = cr * (double)rsum;
    const double rcutsq = rc * rc;
    float fthr = (float)rcutsq;
    if ((double)fthr > rcutsq) fthr = nextafterf(fthr, 0.0f);
    return __float_as_uint(fthr);
}

// pnow, the corrected probability and the order index o (py:445-476); returns o,
// or -1 when the pair emits nothing (r filled completely then)
__device__ __forceinline__ int64_t pair_order(int cnt, int n, int S, const igm_pair& pr, int it_corr,
                                              igm_pair_result* r) {
    const int64_t nS = (int64_t)n * S;
    const double pnow = (double)cnt / (double)nS;  // py:445
    double p;
    if (it_corr == 1) {  // py:452-459
        const double tcorr = clean_prob(pnow, pr.plast);
        p = clean_prob(pr.pwish, tcorr);
    } else {
        p = pr.pwish;
    }
    r->p = p;
    r->pnow = pnow;
    if (!(p > 0.0)) {
        r->ad = __longlong_as_double(0x7ff8000000000000LL);
        r->o = -1;
        r->nrows = 0;
        return -1;
    }
    // o = min(nS - 1, int(round(n * p * S)))   (py:469-470, banker's rounding)
    const double ox = rint((double)n * p * (double)S);
    const int64_t o = (ox >= (double)(nS - 1)) ? nS - 1 : (int64_t)ox;
    r->o = (int)o;
    r->nrows = n;  // py:476-483: zip(ii,jj) or the ii x jj product
    return o;
}

template <int VPL>
__global__ void __launch_bounds__(64 * kWavesPerBlock)
    actdist_kernel(const float* __restrict__ xyz, int S, const float* __restrict__ radii,
                   const int* __restrict__ copy_ptr, const int* __restrict__ copy_idx, const int* __restrict__ chrom,
                   int nhap, const igm_pair* __restrict__ pairs, const int* __restrict__ list, int nlist, double cr,
                   int it_corr, igm_pair_result* __restrict__ res) {
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (w >= nlist) return;  // wave-uniform exit
    const int q = list[w];
    const igm_pair pr = pairs[q];
    int na = 0, nb = 0;
    bool intra = false;
    const int n = pair_ncomb(copy_ptr, chrom, pr.i, pr.j, nhap, &na, &nb, &intra);
    const int a0 = copy_ptr[pr.i], b0 = copy_ptr[pr.j];
    const int SP = (S + 63) / 64;

    // ---- d2[c][s] = sum((x - y)^2) in f32, left to right, no FMA (py:418,435)
    uint32_t key[VPL];
    int c = 0, sl = 0;
#pragma unroll
    for (int t = 0; t < VPL; ++t) {
        key[t] = 0xFFFFFFFFu;  // padding sorts after every real value (NaN incl.)
        const int s = sl * 64 + lane;
        if (c < n && s < S) {
            int k, m;
            if (intra) {
                k = copy_idx[a0 + c];
                m = copy_idx[b0 + c];
            } else {
                k = copy_idx[a0 + c / nb];
                m = copy_idx[b0 + c % nb];
            }
            const float* xk = xyz + ((size_t)k * S + s) * 3;
            const float* xm = xyz + ((size_t)m * S + s) * 3;
            const float dx = __fsub_rn(xk[0], xm[0]);
            const float dy = __fsub_rn(xk[1], xm[1]);
            const float dz = __fsub_rn(xk[2], xm[2]);
            const float d2 = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
            key[t] = __float_as_uint(d2);
        }
        if (++sl == SP) {
            sl = 0;
            ++c;
        }
    }

    const uint32_t thr = cut_key(radii, copy_idx, a0, b0, cr);
    int cnt = 0;
#pragma unroll
    for (int t = 0; t < VPL; ++t) cnt += __popcll(__ballot(key[t] <= thr));
    igm_pair_result r;
    const int64_t o = pair_order(cnt, n, S, pr, it_corr, &r);
    if (o >= 0) {
        // o-th smallest key by bisection on the bit pattern
        uint32_t lo = 0u, hi = 0xFFFFFFFEu;
        const int target = (int)o + 1;
        while (lo < hi) {
            const uint32_t mid = lo + ((hi - lo) >> 1);
            int cm = 0;
#pragma unroll
            for (int t = 0; t < VPL; ++t) cm += __popcll(__ballot(key[t] <= mid));
            if (cm >= target)
                hi = mid;
            else
                lo = mid + 1u;
        }
        r.ad = sqrt_rn((double)__uint_as_float(lo));  // py:473
    }
    if (lane == 0) res[q] = r;
}

// Same contract for populations whose n*S keys exceed one wave's registers: a
// 1024-thread workgroup per pair, key e = t + k*1024 over the flattened
// (combination, structure) range, block-wide counts through LDS.
template <int VPL>
__global__ void __launch_bounds__(kBlockThreads)
    actdist_block_kernel(const float* __restrict__ xyz, int S, const float* __restrict__ radii,
                         const int* __restrict__ copy_ptr, const int* __restrict__ copy_idx,
                         const int* __restrict__ chrom, int nhap, const igm_pair* __restrict__ pairs,
                         const int* __restrict__ list, int nlist, double cr, int it_corr,
                         igm_pair_result* __restrict__ res) {
    __shared__ int part[2][kBlockThreads / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int q = list[blockIdx.x];
    const igm_pair pr = pairs[q];
    int na = 0, nb = 0;
    bool intra = false;
    const int n = pair_ncomb(copy_ptr, chrom, pr.i, pr.j, nhap, &na, &nb, &intra);
    const int a0 = copy_ptr[pr.i], b0 = copy_ptr[pr.j];
    const int nk = n * S;
    uint32_t key[VPL];
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
        key[k] = 0xFFFFFFFFu;
        const int e = k * kBlockThreads + t;
        if (e < nk) {
            const int c = e / S, s = e - c * S;
            int ka, m;
            if (intra) {
                ka = copy_idx[a0 + c];
                m = copy_idx[b0 + c];
            } else {
                ka = copy_idx[a0 + c / nb];
                m = copy_idx[b0 + c % nb];
            }
            const float* xk = xyz + ((size_t)ka * S + s) * 3;
            const float* xm = xyz + ((size_t)m * S + s) * 3;
            const float dx = __fsub_rn(xk[0], xm[0]);
            const float dy = __fsub_rn(xk[1], xm[1]);
            const float dz = __fsub_rn(xk[2], xm[2]);
            key[k] = __float_as_uint(__fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
        }
    }
    int it = 0;
    // block-wide count of keys <= v (alternating LDS buffers: one barrier per count)
    auto count_le = [&](uint32_t v) {
        int cm = 0;
#pragma unroll
        for (int k = 0; k < VPL; ++k) cm += key[k] <= v;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) cm += __shfl_xor(cm, off);
        int* buf = part[it & 1];
        ++it;
        if (lane == 0) buf[w] = cm;
        __syncthreads();
        int tot = 0;
#pragma unroll
        for (int i = 0; i < kBlockThreads / 64; ++i) tot += buf[i];
        return tot;
    };
    const int cnt = count_le(cut_key(radii, copy_idx, a0, b0, cr));
    igm_pair_result r;
    const int64_t o = pair_order(cnt, n, S, pr, it_corr, &r);
    if (o >= 0) {
        uint32_t lo = 0u, hi = 0xFFFFFFFEu;
        const int target = (int)o + 1;
        while (lo < hi) {
            const uint32_t mid = lo + ((hi - lo) >> 1);
            if (count_le(mid) >= target)
                hi = mid;
            else
                lo = mid + 1u;
        }
        r.ad = sqrt_rn((double)__uint_as_float(lo));  // py:473
    }
    if (t == 0) res[q] = r;
}

__global__ void nrows_kernel(const igm_pair_result* __restrict__ res, int64_t npairs, int64_t* __restrict__ nr) {
    int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < npairs) nr[q] = res[q].nrows;
}

__global__ void mark_unprocessed(igm_pair_result* __restrict__ res, const int* __restrict__ list, int nlist) {
    int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nlist) return;
    igm_pair_result r;
    r.ad = __longlong_as_double(0x7ff8000000000000LL);
    r.p = __longlong_as_double(0x7ff8000000000000LL);
    r.pnow = __longlong_as_double(0x7ff8000000000000LL);
    r.o = -1;
    r.nrows = 0;
    res[list[w]] = r;
}

__global__ void emit_kernel(const igm_pair* __restrict__ pairs, int64_t npairs, const int* __restrict__ copy_ptr,
                            const int* __restrict__ copy_idx, const int* __restrict__ chrom,
                            const igm_pair_result* __restrict__ res, const int64_t* __restrict__ off,
                            igm_actdist_row* __restrict__ rows, int64_t cap) {
    int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npairs) return;
    const igm_pair_result r = res[q];
    if (r.nrows <= 0) return;
    const int64_t o = off[q];
    if (o + r.nrows > cap) return;
    const int i = pairs[q].i, j = pairs[q].j;
    const int a0 = copy_ptr[i], b0 = copy_ptr[j];
    const int nb = copy_ptr[j + 1] - b0;
    const bool intra = chrom[i] == chrom[j];
    const float dist = (float)round_dec4(r.ad);
    const float prob = (float)round_dec4(r.p);
    for (int c = 0; c < r.nrows; ++c) {
        igm_actdist_row w;
        if (intra) {
            w.row = copy_idx[a0 + c];
            w.col = copy_idx[b0 + c];
        } else {
            w.row = copy_idx[a0 + c / nb];
            w.col = copy_idx[b0 + c % nb];
        }
        w.dist = dist;
        w.prob = prob;
        rows[o + c] = w;
    }
}

template <int VPL>
int launch_bucket(igm_ctx* c, const float* xyz, int S, const float* radii, const int* cptr, const int* cidx,
                  const int* chrom, int nhap, const igm_pair* pairs, const int* list, int nlist, double cr,
                  int it_corr, igm_pair_result* res) {
    if (nlist <= 0) return IGM_OK;
    dim3 grid((unsigned)igm::ceil_div(nlist, kWavesPerBlock));
    hipLaunchKernelGGL(actdist_kernel<VPL>, grid, dim3(64 * kWavesPerBlock), 0, c->stream, xyz, S, radii, cptr, cidx,
                       chrom, nhap, pairs, list, nlist, cr, it_corr, res);
    IGM_HIP_CHECK(c, hipGetLastError());
    return IGM_OK;
}

template <int VPL>
int launch_block_bucket(igm_ctx* c, const float* xyz, int S, const float* radii, const int* cptr, const int* cidx,
                        const int* chrom, int nhap, const igm_pair* pairs, const int* list, int nlist, double cr,
                        int it_corr, igm_pair_result* res) {
    if (nlist <= 0) return IGM_OK;
    hipLaunchKernelGGL(actdist_block_kernel<VPL>, dim3((unsigned)nlist), dim3(kBlockThreads), 0, c->stream, xyz, S,
                       radii, cptr, cidx, chrom, nhap, pairs, list, nlist, cr, it_corr, res);
    IGM_HIP_CHECK(c, hipGetLastError());
    return IGM_OK;
}

}  // namespace

extern "C" int igm_astep_actdist(igm_ctx* c, uint32_t flags, const float* xyz, int32_t nbead, int32_t nstruct,
                                 const float* radii, const int32_t* copy_ptr, const int32_t* copy_idx, int32_t nhap,
                                 const int32_t* chrom, const igm_pair* pairs, int64_t npairs, double contact_range,
                                 int32_t it_corr, igm_pair_result* per_pair, igm_actdist_row* rows,
                                 int64_t row_capacity, int64_t* nrows_out) {
    using namespace igm;
    if (!c) return IGM_E_INVALID;
    if (nbead <= 0 || nstruct <= 0 || nhap <= 0 || npairs < 0 || !xyz || !radii || !copy_ptr || !copy_idx || !chrom ||
        (npairs > 0 && !pairs) || !nrows_out)
        return fail(c, IGM_E_INVALID, "igm_astep_actdist: invalid arguments");
    if (npairs > 0x7fffffff) return fail(c, IGM_E_UNSUPPORTED, "igm_astep_actdist: more than 2^31 pairs per call");
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    *nrows_out = 0;
    if (npairs == 0) return IGM_OK;

    // copy_idx length is copy_ptr[nhap]; in device mode we read it back once
    int32_t ncopy = 0;
    if (flags & IGM_DEVICE_PTRS) {
        IGM_HIP_CHECK(c, hipMemcpyAsync(&ncopy, copy_ptr + nhap, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    } else {
        ncopy = copy_ptr[nhap];
    }
    const float* d_xyz;
    const float* d_radii;
    const int32_t *d_cptr, *d_cidx, *d_chrom;
    const igm_pair* d_pairs;
    IGM_TRY(to_device(c, flags, "ad_xyz", xyz, (size_t)nbead * nstruct * 3, &d_xyz));
    IGM_TRY(to_device(c, flags, "ad_radii", radii, (size_t)nbead, &d_radii));
    IGM_TRY(to_device(c, flags, "ad_cptr", copy_ptr, (size_t)nhap + 1, &d_cptr));
    IGM_TRY(to_device(c, flags, "ad_cidx", copy_idx, (size_t)ncopy, &d_cidx));
    IGM_TRY(to_device(c, flags, "ad_chrom", chrom, (size_t)nhap, &d_chrom));
    IGM_TRY(to_device(c, flags, "ad_pairs", pairs, (size_t)npairs, &d_pairs));

    igm_pair_result* d_res;
    if (per_pair && (flags & IGM_DEVICE_PTRS)) {
        d_res = per_pair;
    } else {
        void* p;
        IGM_TRY(workspace(c, "ad_res", (size_t)npairs * sizeof(igm_pair_result), &p));
        d_res = (igm_pair_result*)p;
    }
    void *p_counts, *p_lists, *p_nr, *p_off;
    IGM_TRY(workspace(c, "ad_counts", kBuckets * sizeof(int), &p_counts));
    IGM_TRY(workspace(c, "ad_lists", (size_t)kBuckets * npairs * sizeof(int), &p_lists));
    IGM_TRY(workspace(c, "ad_nr", (size_t)npairs * sizeof(int64_t), &p_nr));
    IGM_TRY(workspace(c, "ad_off", (size_t)npairs * sizeof(int64_t), &p_off));
    int* d_counts = (int*)p_counts;
    int* d_lists = (int*)p_lists;
    // "actdist": the whole device A-step (classification, selection, row scan and emit,
    // with the host reads of the bucket counts and row total in between);
    // "actdist_select": the selection kernels alone
    Timed tm_all(c, "actdist");
    IGM_HIP_CHECK(c, hipMemsetAsync(d_counts, 0, kBuckets * sizeof(int), c->stream));
    {
        dim3 g1((unsigned)ceil_div(npairs, 256));
        hipLaunchKernelGGL(classify_kernel, g1, dim3(256), 0, c->stream, d_pairs, npairs, d_cptr, d_chrom, nhap,
                           nstruct, d_counts, d_lists);
        IGM_HIP_CHECK(c, hipGetLastError());
        int h_counts[kBuckets];
        IGM_HIP_CHECK(c, hipMemcpyAsync(h_counts, d_counts, sizeof(h_counts), hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        if (h_counts[7] > 0)
            return fail(c, IGM_E_UNSUPPORTED,
                        "igm_astep_actdist: %d pairs need n_combinations*S > %d keys (S=%d); "
                        "population too large for the register-resident selection kernels",
                        h_counts[7], 64 * kBlockThreads, nstruct);
        const int* L = d_lists;
        Timed tm(c, "actdist_select");  // the selection kernels only (inputs resident)
        IGM_TRY(launch_bucket<1>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs, L + 0 * npairs,
                                 h_counts[0], contact_range, it_corr, d_res));
        IGM_TRY(launch_bucket<2>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs, L + 1 * npairs,
                                 h_counts[1], contact_range, it_corr, d_res));
        IGM_TRY(launch_bucket<4>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs, L + 2 * npairs,
                                 h_counts[2], contact_range, it_corr, d_res));
        IGM_TRY(launch_bucket<8>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs, L + 3 * npairs,
                                 h_counts[3], contact_range, it_corr, d_res));
        IGM_TRY(launch_bucket<16>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs, L + 4 * npairs,
                                  h_counts[4], contact_range, it_corr, d_res));
        IGM_TRY(launch_bucket<32>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs, L + 5 * npairs,
                                  h_counts[5], contact_range, it_corr, d_res));
        IGM_TRY(launch_bucket<64>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs, L + 6 * npairs,
                                  h_counts[6], contact_range, it_corr, d_res));
        IGM_TRY(launch_block_bucket<8>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs,
                                       L + 9 * npairs, h_counts[9], contact_range, it_corr, d_res));
        IGM_TRY(launch_block_bucket<16>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs,
                                        L + 10 * npairs, h_counts[10], contact_range, it_corr, d_res));
        IGM_TRY(launch_block_bucket<32>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs,
                                        L + 11 * npairs, h_counts[11], contact_range, it_corr, d_res));
        IGM_TRY(launch_block_bucket<64>(c, d_xyz, nstruct, d_radii, d_cptr, d_cidx, d_chrom, nhap, d_pairs,
                                        L + 12 * npairs, h_counts[12], contact_range, it_corr, d_res));
        if (h_counts[8] > 0) {
            hipLaunchKernelGGL(mark_unprocessed, dim3((unsigned)ceil_div(h_counts[8], 256)), dim3(256), 0, c->stream,
                               d_res, L + 8 * npairs, h_counts[8]);
            IGM_HIP_CHECK(c, hipGetLastError());
        }
    }
    // ---- CSR-order compaction of the rows (task() appends pair after pair)
    int64_t* d_nr = (int64_t*)p_nr;
    int64_t* d_off = (int64_t*)p_off;
    hipLaunchKernelGGL(nrows_kernel, dim3((unsigned)ceil_div(npairs, 256)), dim3(256), 0, c->stream, d_res, npairs,
                       d_nr);
    size_t tmp_bytes = 0;
    IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, d_nr, d_off, (int)npairs, c->stream));
    void* d_tmp;
    IGM_TRY(workspace(c, "ad_scan_tmp", tmp_bytes, &d_tmp));
    IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_bytes, d_nr, d_off, (int)npairs, c->stream));
    int64_t last_off = 0, last_n = 0;
    IGM_HIP_CHECK(c, hipMemcpyAsync(&last_off, d_off + npairs - 1, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipMemcpyAsync(&last_n, d_nr + npairs - 1, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    const int64_t total = last_off + last_n;
    *nrows_out = total;
    if (per_pair && !(flags & IGM_DEVICE_PTRS)) IGM_TRY(to_host(c, flags, per_pair, d_res, (size_t)npairs));
    if (total > row_capacity || (total > 0 && !rows)) {
        IGM_TRY(finish(c, flags & ~IGM_ASYNC));
        return fail(c, IGM_E_OVERFLOW, "igm_astep_actdist: %lld rows exceed capacity %lld", (long long)total,
                    (long long)row_capacity);
    }
    igm_actdist_row* d_rows;
    IGM_TRY(out_device(c, flags, "ad_rows", rows, (size_t)total, &d_rows));
    if (total > 0) {
        hipLaunchKernelGGL(emit_kernel, dim3((unsigned)ceil_div(npairs, 256)), dim3(256), 0, c->stream, d_pairs,
                           npairs, d_cptr, d_cidx, d_chrom, d_res, d_off, d_rows, total);
        IGM_HIP_CHECK(c, hipGetLastError());
        IGM_TRY(to_host(c, flags, rows, d_rows, (size_t)total));
    }
    return finish(c, flags);
}

namespace {
__global__ void plast_kernel(igm_pair* __restrict__ pairs, int64_t npairs, const igm_pair_result* __restrict__ res) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npairs) return;
    const igm_pair_result r = res[q];
    pairs[q].plast = r.nrows > 0 ? (double)(float)round_dec4(r.p) : 0.0;
}
}  // namespace

extern "C" int igm_astep_update_plast(igm_ctx* c, uint32_t flags, igm_pair* pairs, int64_t npairs,
                                      const igm_pair_result* per_pair) {
    using namespace igm;
    if (!c || npairs < 0 || (npairs > 0 && (!pairs || !per_pair)))
        return fail(c, IGM_E_INVALID, "igm_astep_update_plast: invalid arguments");
    if (npairs == 0) return IGM_OK;
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    igm_pair* d_pairs;
    const igm_pair_result* d_res;
    if (flags & IGM_DEVICE_PTRS) {
        d_pairs = pairs;
    } else {
        void* p;
        IGM_TRY(workspace(c, "up_pairs", sizeof(igm_pair) * npairs, &p));
        d_pairs = (igm_pair*)p;
        IGM_HIP_CHECK(c, hipMemcpyAsync(d_pairs, pairs, sizeof(igm_pair) * npairs, hipMemcpyHostToDevice, c->stream));
    }
    IGM_TRY(to_device(c, flags, "up_res", per_pair, (size_t)npairs, &d_res));
    hipLaunchKernelGGL(plast_kernel, dim3((unsigned)ceil_div(npairs, 256)), dim3(256), 0, c->stream, d_pairs, npairs,
                       d_res);
    IGM_HIP_CHECK(c, hipGetLastError());
    IGM_TRY(to_host(c, flags, pairs, (const igm_pair*)d_pairs, (size_t)npairs));
    return finish(c, flags);
}
