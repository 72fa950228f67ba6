// A-steps of configurations D/E on the MI355X:
//
//   DamID   DamidActivationDistanceStep.task over all loci at once
//           (igm/steps/DamidActivationDistanceStep.py:223-287, get_damid_actdist_I :376-471)
//           plus the "%6d %.5f %.5f" text round trip of task()/reduce() (:35, :286, :308).
//   FISH    FishAssignmentStep.task (igm/steps/FishAssignmentStep.py:188-242):
//           per-structure min/max radial or pair distance over the copies, ranks,
//           target[rank] for every probe/pair at once.
//   SPRITE  SpriteAssignmentStep.task (igm/steps/SpriteAssignmentStep.py:105-160):
//           compute_gyration_radius (igm/cython_compiled/sprite.pyx:104-283, with
//           get_rg2s_cpp, cpp_sprite_assignment.cpp:49-143) for every (cluster,
//           structure), then the keep_best selection (:138-143).
//
// All three are HBM/L2-bound gathers over the bead-major (nbead, nstruct, 3) .hss
// coordinate array; the arithmetic restates NumPy 1.x / the reference C++ operation
// by operation (no FMA contraction: built with -ffp-contract=off), so the outputs are
// bit-identical to the reference's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "exact_math.h"
#include "igm_ctx.h"
#include "mstep_common.h"

namespace {
using namespace igm;

constexpr int kBT = 256;  // threads per workgroup (4 waves of 64)

__device__ __forceinline__ int block_sum(int v, int* sh) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    int t = 0;
    for (int i = 0; i < kBT / 64; ++i) t += sh[i];
    return t;
}

__device__ __forceinline__ void load3(const float* __restrict__ xyz, int S, int bead, int s, float& x, float& y,
                                      float& z) {
    const float* p = xyz + ((size_t)bead * S + s) * 3;
    x = p[0];
    y = p[1];
    z = p[2];
}

// rank[t] = the position of element t in the stable ascending order of v[0..n): the
// argsort(argsort(v)) NumPy computes (ties in index order), i.e. #{u : v[u] < v[t]} +
// #{u < t : v[u] == v[t]}.  A bitonic sort of the (value, index) pairs in LDS -- npad (a power
// of two >= n) keys sk and indices si, every thread of the block taking part -- in place of
// counting every rank against the whole column (O(n^2): 1 M comparisons per FISH item at
// n = 1000, against ~28 k compare-exchanges here).  The pad sorts after every value (+inf,
// index >= n).
__device__ void block_stable_rank(const float* v, int n, int npad, float* sk, int* si, int* rank) {
    for (int p = threadIdx.x; p < npad; p += kBT) {
        sk[p] = p < n ? v[p] : INFINITY;
        si[p] = p;
    }
    __syncthreads();
    for (int k = 2; k <= npad; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int p = threadIdx.x; p < npad; p += kBT) {
                const int q = p ^ j;
                if (q > p) {
                    const float a = sk[p], b = sk[q];
                    const int ia = si[p], ib = si[q];
                    const bool gt = a > b || (a == b && ia > ib);
                    if (gt == ((p & k) == 0)) {
                        sk[p] = b;
                        sk[q] = a;
                        si[p] = ib;
                        si[q] = ia;
                    }
                }
            }
            __syncthreads();
        }
    for (int p = threadIdx.x; p < n; p += kBT) rank[si[p]] = p;
    __syncthreads();
}

// block_stable_rank for npad = E * kBT (E <= 8): thread t holds the E consecutive keys
// t E .. t E + E - 1 in registers as u64 (the value's order-preserving bits above its index,
// so equal values order by index -- the same stable order as above).  A bitonic stage with partner distance j < E
// swaps inside a thread, E <= j < 64 E exchanges through a wave shuffle, and only the
// stages with j >= 64 E (3 of the 55 at npad = 1024) go through LDS (hi and lo words in the
// sk / si arrays) with a barrier.
template <int E, int C>
__device__ void block_stable_rank_reg(const float* const (&v)[C], int n, uint32_t* kh, uint32_t* kl,
                                      int* const (&rank)[C]) {
    const int t = threadIdx.x;
    constexpr int NP = E * kBT;
    uint64_t key[C][E];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int p = t * E + e;
            // IEEE bits made order-preserving for every sign (negative: all bits flipped); the
            // pad is +inf with an index >= n.  (-0 would sort before +0 where the float compare
            // ties them: the columns ranked here are norms, never -0.)
            const uint32_t bits = p < n ? __float_as_uint(v[c][p]) : 0x7f800000u;
            const uint32_t ord = bits ^ ((bits >> 31) ? 0xffffffffu : 0x80000000u);
            key[c][e] = ((uint64_t)ord << 32) | (uint32_t)p;
        }
#pragma unroll
    for (int k = 2; k <= NP; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j < E) {
#pragma unroll
                for (int c = 0; c < C; ++c)
#pragma unroll
                    for (int e = 0; e < E; ++e)
                        if ((e & j) == 0) {
                            const int p = t * E + e;
                            const uint64_t a = key[c][e], b = key[c][e | j];
                            const bool up = (p & k) == 0;
                            key[c][e] = up ? (a < b ? a : b) : (a < b ? b : a);
                            key[c][e | j] = up ? (a < b ? b : a) : (a < b ? a : b);
                        }
            } else {
                uint64_t o[C][E];
                if (j < 64 * E) {
                    const int d = j / E;  // lane distance of the partner
#pragma unroll
                    for (int c = 0; c < C; ++c)
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const uint32_t h = __shfl_xor((int)(uint32_t)(key[c][e] >> 32), d, 64),
                                           l = __shfl_xor((int)(uint32_t)key[c][e], d, 64);
                            o[c][e] = ((uint64_t)h << 32) | l;
                        }
                } else {
#pragma unroll
                    for (int c = 0; c < C; ++c)
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            kh[c * NP + t * E + e] = (uint32_t)(key[c][e] >> 32);
                            kl[c * NP + t * E + e] = (uint32_t)key[c][e];
                        }
                    __syncthreads();
#pragma unroll
                    for (int c = 0; c < C; ++c)
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const int q = c * NP + ((t * E + e) ^ j);
                            o[c][e] = ((uint64_t)kh[q] << 32) | kl[q];
                        }
                    __syncthreads();
                }
#pragma unroll
                for (int c = 0; c < C; ++c)
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const int p = t * E + e;
                        const bool up = (p & k) == 0, lower = (p & j) == 0;
                        const uint64_t a = key[c][e], b = o[c][e];
                        key[c][e] = (up == lower) ? (a < b ? a : b) : (a < b ? b : a);
                    }
            }
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int p = t * E + e;
            if (p < n) rank[c][(uint32_t)key[c][e]] = p;
        }
    __syncthreads();
}

// the stable ranks of C columns v[c][0..n): the register sort (all C columns through one
// network) when npad = E kBT, E <= 8, else the LDS sort column by column.  Scratch: sk and
// si of C npad words each.
template <int C>
__device__ void stable_rank(const float* const (&v)[C], int n, int npad, float* sk, int* si, int* const (&rank)[C]) {
    __syncthreads();  // (v complete)
    uint32_t* kh = reinterpret_cast<uint32_t*>(sk);
    uint32_t* kl = reinterpret_cast<uint32_t*>(si);
    if (npad == kBT) block_stable_rank_reg<1, C>(v, n, kh, kl, rank);
    else if (npad == 2 * kBT) block_stable_rank_reg<2, C>(v, n, kh, kl, rank);
    else if (npad == 4 * kBT) block_stable_rank_reg<4, C>(v, n, kh, kl, rank);
    else if (npad == 8 * kBT) block_stable_rank_reg<8, C>(v, n, kh, kl, rank);
    else
        for (int c = 0; c < C; ++c) block_stable_rank(v[c], n, npad, sk, si, rank[c]);
}

__host__ __device__ inline int pow2_at_least(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

// ============================================================================ DamID
struct DamidArgs {
    const float* xyz;
    int S;
    const float* radii;
    const int* cptr;
    const int* cidx;
    const int* loci;
    const float* pexp;
    const float* plast;
    int nloci;
    int it_corr;
    int shape;         // 0 sphere, 1 ellipsoid
    double R[3];       // nucleus_param * (1 - contact_range), f64 (py:436)
    igm_pair_result* res;
    const int64_t* rowoff;
    igm_damid_row* rows;
};

// snormsq_sphere / snormsq_ellipse (py:39-76): float32 squares, the float64 divisor
// cast to float32 (NumPy 1.x value-based casting), float32 divisions and sums
__device__ __forceinline__ float damid_key(const DamidArgs& A, int bead, int s, float D0, float D1, float D2) {
    float x, y, z;
    load3(A.xyz, A.S, bead, s, x, y, z);
    const float q0 = __fmul_rn(x, x), q1 = __fmul_rn(y, y), q2 = __fmul_rn(z, z);
    if (A.shape == 0) return __fdiv_rn(__fadd_rn(__fadd_rn(q0, q1), q2), D0);
    return __fadd_rn(__fadd_rn(__fdiv_rn(q0, D0), __fdiv_rn(q1, D1)), __fdiv_rn(q2, D2));
}

// cleanProbability (DamidActivationDistanceStep.py:362-372) in float64
__device__ __forceinline__ double damid_clean(double pij, double pexist) {
    const double pc = (pexist < 1.0) ? (pij - pexist) / (1.0 - pexist) : pij;
    return pc > 0.0 ? pc : 0.0;
}

// One workgroup per locus.  The o-th entry of d^2 sorted in decreasing order is the
// (nS-1-o)-th smallest: found by a 4-pass 8-bit radix select over the float bits
// (non-negative floats order like their bit patterns; NaN sorts last ascending, first
// descending, like numpy's sort).  Keys are recomputed from the L2-resident
// coordinates each pass instead of being staged (nc*S can exceed LDS).
__global__ void __launch_bounds__(kBT) damid_kernel(DamidArgs A) {
    const int q = blockIdx.x;
    if (q >= A.nloci) return;
    __shared__ int sh_red[kBT / 64];
    __shared__ unsigned hist[256];
    __shared__ long long sh_m;
    __shared__ unsigned sh_prefix, sh_mask;
    __shared__ double sh_p;
    __shared__ int sh_o;
    const int I = A.loci[q];
    const int c0 = A.cptr[I], nc = A.cptr[I + 1] - c0;
    const int S = A.S;
    if (nc <= 0) {
        if (threadIdx.x == 0) {
            igm_pair_result r;
            r.ad = __longlong_as_double(0x7ff8000000000000LL);
            r.p = 0.0;
            r.pnow = 0.0;
            r.o = -1;
            r.nrows = 0;
            A.res[q] = r;
        }
        return;
    }
    const float rad = A.radii[A.cidx[c0]];  // r = radii[ii[0]] (py:429)
    float D0, D1 = 1.0f, D2 = 1.0f;
    if (A.shape == 0) {
        const double t = A.R[0] - (double)rad;
        D0 = (float)(t * t);
    } else {
        const double a = A.R[0] - (double)rad, b = A.R[1] - (double)rad, c = A.R[2] - (double)rad;
        D0 = (float)(a * a);
        D1 = (float)(b * b);
        D2 = (float)(c * c);
    }
    // contact count: d_sq >= rcutsq = 1.0 (py:449-450)
    int cnt = 0;
    for (int ci = 0; ci < nc; ++ci) {
        const int bead = A.cidx[c0 + ci];
        for (int s = threadIdx.x; s < S; s += kBT) cnt += damid_key(A, bead, s, D0, D1, D2) >= 1.0f;
    }
    cnt = block_sum(cnt, sh_red);
    const int64_t nS = (int64_t)nc * S;
    if (threadIdx.x == 0) {
        const double pnow = (double)cnt / (double)nS;
        const double pexp = (double)A.pexp[q];
        double p;
        if (A.it_corr == 1) {
            p = damid_clean(pexp, damid_clean(pnow, (double)A.plast[q]));
        } else {
            p = pexp;
        }
        int o = -1;
        if (p > 0.0) {  // o = min(nS - 1, int(round(nS * p)))  (py:464-466, half to even)
            const double ox = rint((double)nS * p);
            o = (ox >= (double)(nS - 1)) ? (int)(nS - 1) : (int)ox;
        }
        sh_p = p;
        sh_o = o;
        sh_m = o >= 0 ? nS - 1 - o : 0;
        sh_prefix = 0u;
        sh_mask = 0u;
        igm_pair_result r;
        r.p = p;
        r.pnow = pnow;
        r.o = o;
        r.nrows = nc;
        r.ad = __longlong_as_double(0x7ff8000000000000LL);
        A.res[q] = r;
    }
    __syncthreads();
    const int o = sh_o;
    double ad = 2.0;  // py:460
    if (o >= 0) {
        for (int shift = 24; shift >= 0; shift -= 8) {
            hist[threadIdx.x] = 0u;
            __syncthreads();
            const unsigned prefix = sh_prefix, mask = sh_mask;
            for (int ci = 0; ci < nc; ++ci) {
                const int bead = A.cidx[c0 + ci];
                for (int s = threadIdx.x; s < S; s += kBT) {
                    const unsigned u = __float_as_uint(damid_key(A, bead, s, D0, D1, D2));
                    if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255u], 1u);
                }
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                long long m = sh_m;
                int b = 0;
                for (; b < 255; ++b) {
                    if (m < (long long)hist[b]) break;
                    m -= hist[b];
                }
                sh_m = m;
                sh_prefix = prefix | ((unsigned)b << shift);
                sh_mask = mask | (255u << shift);
            }
            __syncthreads();
        }
        ad = sqrt_rn((double)__uint_as_float(sh_prefix));  // np.sqrt(d_sq[o]) in float64 (py:470)
        if (threadIdx.x == 0) A.res[q].ad = ad;
    }
    // rows (i, ad, p) for i in ii (py:473) through '%.5f' and genfromtxt(float32)
    const float dist = (float)round_dec(ad, 1e5);
    const float prob = (float)round_dec(sh_p, 1e5);
    const int64_t base = A.rowoff[q];
    for (int ci = threadIdx.x; ci < nc; ci += kBT) {
        igm_damid_row w;
        w.loc = A.cidx[c0 + ci];
        w.dist = dist;
        w.prob = prob;
        A.rows[base + ci] = w;
    }
}

// ---------------------------------------------------------------- DamID, exp_map
// get_damid_actdist_exp (DamidActivationDistanceStep.py:475-577) with snormsq_exp
// (:79-115): the squared distance of a bead to its voxel's nearest lamina voxel
// (inside the grid) or, outside, |(voxel - center) * grid|^2 in the reference's mixed
// units; all float64 (f32 coordinate minus float64 map geometry), np.round half to
// even, np.dot summing (t0^2 + t2^2) + t1^2 like the reference BLAS.  Distances are
// sorted ASCENDING here (d_sq.sort(axis=1)); pnow counts d_sq >= contact_range.
struct DamidExpArgs {
    const float* xyz;
    int S;
    const int* cptr;
    const int* cidx;
    const int* loci;
    const float* pexp;
    const float* plast;
    int nloci;
    int it_corr;
    double cr;
    const igm::ms::VolMapDev* maps;
    const int4* vox;
    const int* smap;  // (S) map of each structure
    igm_pair_result* res;
    const int64_t* rowoff;
    igm_damid_row* rows;
};

__device__ __forceinline__ double damid_exp_key(const DamidExpArgs& A, int bead, int s) {
    const igm::ms::VolMapDev m = A.maps[A.smap[s]];
    float p[3];
    load3(A.xyz, A.S, bead, s, p[0], p[1], p[2]);
    long long v[3];
    bool in = true;
    for (int d = 0; d < 3; ++d) {
        v[d] = (long long)rint(((double)p[d] - (double)m.origin[d]) / (double)m.grid[d]);
        in = in && v[d] >= 0 && v[d] < m.n[d];
    }
    double t[3];
    if (in) {
        const int4 r = A.vox[m.off + (v[0] * m.n[1] + v[1]) * m.n[2] + v[2]];
        const int e[3] = {r.x, r.y, r.z};
        for (int d = 0; d < 3; ++d) t[d] = (double)p[d] - ((double)e[d] * (double)m.grid[d] + (double)m.origin[d]);
    } else {
        for (int d = 0; d < 3; ++d) t[d] = ((double)v[d] - (double)m.center[d]) * (double)m.grid[d];
    }
    return (t[0] * t[0] + t[2] * t[2]) + t[1] * t[1];
}

__global__ void __launch_bounds__(kBT) damid_exp_kernel(DamidExpArgs A) {
    const int q = blockIdx.x;
    if (q >= A.nloci) return;
    __shared__ int sh_red[kBT / 64];
    __shared__ unsigned hist[256];
    __shared__ long long sh_m;
    __shared__ unsigned long long sh_prefix, sh_mask;
    __shared__ double sh_p;
    __shared__ int sh_o;
    const int I = A.loci[q];
    const int c0 = A.cptr[I], nc = A.cptr[I + 1] - c0;
    const int S = A.S;
    int cnt = 0;
    for (int ci = 0; ci < nc; ++ci) {
        const int bead = A.cidx[c0 + ci];
        for (int s = threadIdx.x; s < S; s += kBT) cnt += damid_exp_key(A, bead, s) >= A.cr;
    }
    cnt = block_sum(cnt, sh_red);
    const int64_t nS = (int64_t)nc * S;
    if (threadIdx.x == 0) {
        const double pnow = nS > 0 ? (double)cnt / (double)nS : 0.0;
        const double pexp = (double)A.pexp[q];
        const double p = (A.it_corr == 1) ? damid_clean(pexp, damid_clean(pnow, (double)A.plast[q])) : pexp;
        int o = -1;
        if (p > 0.0 && nS > 0) {
            const double ox = rint((double)nS * p);
            o = (ox >= (double)(nS - 1)) ? (int)(nS - 1) : (int)ox;
        }
        sh_p = p;
        sh_o = o;
        sh_m = o;  // ascending: the o-th smallest
        sh_prefix = 0ull;
        sh_mask = 0ull;
        igm_pair_result r;
        r.p = p;
        r.pnow = pnow;
        r.o = o;
        r.nrows = nc;
        r.ad = __longlong_as_double(0x7ff8000000000000LL);
        A.res[q] = r;
    }
    __syncthreads();
    double ad = 1e-9;  // py:540
    if (sh_o >= 0) {
        for (int shift = 56; shift >= 0; shift -= 8) {
            hist[threadIdx.x] = 0u;
            __syncthreads();
            const unsigned long long prefix = sh_prefix, mask = sh_mask;
            for (int ci = 0; ci < nc; ++ci) {
                const int bead = A.cidx[c0 + ci];
                for (int s = threadIdx.x; s < S; s += kBT) {
                    const unsigned long long u = (unsigned long long)__double_as_longlong(damid_exp_key(A, bead, s));
                    if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255ull], 1u);
                }
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                long long m = sh_m;
                int b = 0;
                for (; b < 255; ++b) {
                    if (m < (long long)hist[b]) break;
                    m -= hist[b];
                }
                sh_m = m;
                sh_prefix = prefix | ((unsigned long long)b << shift);
                sh_mask = mask | (255ull << shift);
            }
            __syncthreads();
        }
        ad = sqrt_rn(__longlong_as_double((long long)sh_prefix));
        if (threadIdx.x == 0) A.res[q].ad = ad;
    }
    const float dist = (float)round_dec(ad, 1e5);
    const float prob = (float)round_dec(sh_p, 1e5);
    const int64_t base = A.rowoff[q];
    for (int ci = threadIdx.x; ci < nc; ci += kBT) {
        igm_damid_row w;
        w.loc = A.cidx[c0 + ci];
        w.dist = dist;
        w.prob = prob;
        A.rows[base + ci] = w;
    }
}

__global__ void damid_nrows_kernel(const int* __restrict__ loci, int nloci, const int* __restrict__ cptr,
                                   int64_t* __restrict__ nr) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nloci) nr[q] = cptr[loci[q] + 1] - cptr[loci[q]];
}

__global__ void check_loci_kernel(const int* __restrict__ loci, int n, int nhap, int* __restrict__ bad) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n && (loci[q] < 0 || loci[q] >= nhap)) atomicOr(bad, 1);
}

// ============================================================================ FISH
struct FishArgs {
    const float* xyz;
    int S;
    const int* cptr;
    const int* cidx;
    int kind;  // 0 radial (items[q]), 1 pair (items[2q], items[2q+1])
    const int* items;
    int nitems;
    const float* tmin;
    const float* tmax;
    float* omin;
    float* omax;
    float* dmin;
    float* dmax;
};

// np.linalg.norm(x, axis=1) in float32: sqrt(((x0^2 + x1^2) + x2^2)), correctly rounded
__device__ __forceinline__ float norm3(float x, float y, float z) {
    return sqrtf_rn(__fadd_rn(__fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y)), __fmul_rn(z, z)));
}

// One workgroup per probe/pair: the per-structure min and max over the copies
// (get_rad_dists / get_pair_dists + get_min_max_and_idx, py:23-77) are staged in
// LDS, then every structure's rank -- argsort(argsort(.)), ties in index order -- is
// counted against the whole column, and target[rank] is written (py:221-242).
__global__ void __launch_bounds__(kBT) fish_kernel(FishArgs A) {
    extern __shared__ float fsm[];
    const int q = blockIdx.x;
    if (q >= A.nitems) return;
    const int S = A.S;
    float* vmin = fsm;
    float* vmax = fsm + S;
    int a0, na, b0 = 0, nb = 0;
    if (A.kind == 0) {
        const int h = A.items[q];
        a0 = A.cptr[h];
        na = A.cptr[h + 1] - a0;
    } else {
        const int h = A.items[2 * q], g = A.items[2 * q + 1];
        a0 = A.cptr[h];
        na = A.cptr[h + 1] - a0;
        b0 = A.cptr[g];
        nb = A.cptr[g + 1] - b0;
    }
    if (na <= 2 && nb <= 2 && na > 0 && (A.kind == 0 || nb > 0)) {
        // <= 2 copies a side (every diploid locus): a thread's U structures and all their
        // copies' positions are loaded together, one memory round trip (the min / max do
        // not depend on the order the distances are taken in)
        constexpr int U = 4;
        const int ia0 = A.cidx[a0], ia1 = A.cidx[a0 + na - 1];
        const int ib0 = nb > 0 ? A.cidx[b0] : 0, ib1 = nb > 0 ? A.cidx[b0 + nb - 1] : 0;
        for (int s0 = threadIdx.x; s0 < S; s0 += U * kBT) {
            float p[4][U][3];  // copies a0, a1, b0, b1
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int s = min(s0 + u * kBT, S - 1);
                load3(A.xyz, S, ia0, s, p[0][u][0], p[0][u][1], p[0][u][2]);
                load3(A.xyz, S, ia1, s, p[1][u][0], p[1][u][1], p[1][u][2]);
                if (A.kind != 0) {
                    load3(A.xyz, S, ib0, s, p[2][u][0], p[2][u][1], p[2][u][2]);
                    load3(A.xyz, S, ib1, s, p[3][u][0], p[3][u][1], p[3][u][2]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int s = s0 + u * kBT;
                if (s >= S) break;
                float mn = INFINITY, mx = -INFINITY;
                auto take = [&](float d) {
                    mn = d < mn ? d : mn;
                    mx = d > mx ? d : mx;
                };
                if (A.kind == 0) {
                    take(norm3(p[0][u][0], p[0][u][1], p[0][u][2]));
                    take(norm3(p[1][u][0], p[1][u][1], p[1][u][2]));
                } else {
#pragma unroll
                    for (int a = 0; a < 2; ++a)
#pragma unroll
                        for (int b = 2; b < 4; ++b)
                            take(norm3(__fsub_rn(p[a][u][0], p[b][u][0]), __fsub_rn(p[a][u][1], p[b][u][1]),
                                       __fsub_rn(p[a][u][2], p[b][u][2])));
                }
                vmin[s] = mn;
                vmax[s] = mx;
            }
        }
    } else
    for (int s = threadIdx.x; s < S; s += kBT) {
        float mn = INFINITY, mx = -INFINITY;
        for (int a = 0; a < na; ++a) {
            float x, y, z;
            load3(A.xyz, S, A.cidx[a0 + a], s, x, y, z);
            if (A.kind == 0) {
                const float d = norm3(x, y, z);
                mn = d < mn ? d : mn;
                mx = d > mx ? d : mx;
            } else {
                for (int b = 0; b < nb; ++b) {
                    float u, v, w;
                    load3(A.xyz, S, A.cidx[b0 + b], s, u, v, w);
                    const float d = norm3(__fsub_rn(x, u), __fsub_rn(y, v), __fsub_rn(z, w));
                    mn = d < mn ? d : mn;
                    mx = d > mx ? d : mx;
                }
            }
        }
        vmin[s] = mn;
        vmax[s] = mx;
    }
    __syncthreads();
    // the ranks of the column (block_stable_rank), min then max
    const int npad = pow2_at_least(S);
    float* sk = fsm + 2 * S;
    int* si = reinterpret_cast<int*>(sk + 2 * npad);
    int* rmin = si + 2 * npad;
    int* rmax = rmin + S;
    const float* const cols[2] = {vmin, vmax};
    int* const ranks[2] = {rmin, rmax};
    stable_rank<2>(cols, S, npad, sk, si, ranks);
    const size_t row = (size_t)q * S;
    for (int s = threadIdx.x; s < S; s += kBT) {
        if (A.omin) A.omin[row + s] = A.tmin[row + rmin[s]];
        if (A.omax) A.omax[row + s] = A.tmax[row + rmax[s]];
        if (A.dmin) A.dmin[row + s] = vmin[s];
        if (A.dmax) A.dmax[row + s] = vmax[s];
    }
}

// LDS of fish_kernel: the min and max columns, the sort's keys and indices (both columns), two rank columns
inline size_t fish_lds(int S) { return sizeof(float) * (4 * (size_t)S + 4 * (size_t)pow2_at_least(S)); }

// ============================================================================ SPRITE
struct SpriteArgs {
    const float* xyz;
    int S;
    int ncl;
    int nsb;  // structure blocks per cluster
    const int* seg_ptr;
    const int* seg_region;
    const int* seg_rep;
    const int* rep_ptr;
    const int* rep_region;
    const int* alt_ptr;
    const int* alt_bead;
    float* rg2;  // (ncl, S)
    int* sel;    // (nseg, S): the selected bead of every cluster segment
    // flat tables of the clusters whose regions all have 1 or 2 copies (two[c]), built on the
    // host: each segment's / representative's copy 0 and copy 1 (copy 0 again for one copy,
    // which is then also the last copy that -1 selects) and the bit of its representative's
    // digit in a combination index (0 for one copy: both entries are the same bead)
    const int* ncomb2;  // 2^(2-copy representatives) of a two[c] cluster, 0 otherwise
    const int2* seg_b2;
    const unsigned char* seg_bit;
    const int2* rep_b2;
    const unsigned char* rep_bit;
};

constexpr float kSpriteInf = 100000000.0f;  // INF of cpp_sprite_assignment.cpp:4
constexpr int kMaxReps = 16;
// representatives whose copies a SPRITE thread keeps in registers: 6, the reference's default
// max_chrom_in_cluster (SpriteAssignmentStep.py:114: clusters with more chromosomes are
// skipped), so every computed cluster of a default configuration fits; 8 kept the kernel at 70
// VGPRs against 61, SPRITE 2.98 / 3.00 ms against 2.81 / 2.83 (profiles/r05_de)
constexpr int kRegReps = 6;

// gyration_radius_sq (cpp_sprite_assignment.cpp:49-61): float mean accumulated in
// order and divided by float(n), then the sum of X0*X0 + X1*X1 + X2*X2 in order / n
template <class Bead>
__device__ __forceinline__ float rg2_of(const float* __restrict__ xyz, int S, int s, int n, Bead bead) {
    float mx = 0.0f, my = 0.0f, mz = 0.0f;
    for (int i = 0; i < n; ++i) {
        float x, y, z;
        load3(xyz, S, bead(i), s, x, y, z);
        mx = __fadd_rn(mx, x);
        my = __fadd_rn(my, y);
        mz = __fadd_rn(mz, z);
    }
    const float fn = (float)n;
    mx = __fdiv_rn(mx, fn);
    my = __fdiv_rn(my, fn);
    mz = __fdiv_rn(mz, fn);
    float rg = 0.0f;
    for (int i = 0; i < n; ++i) {
        float x, y, z;
        load3(xyz, S, bead(i), s, x, y, z);
        const float dx = __fsub_rn(x, mx), dy = __fsub_rn(y, my), dz = __fsub_rn(z, mz);
        rg = __fadd_rn(rg, __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
    }
    return __fdiv_rn(rg, fn);
}

// rg2_of with the n <= kRegBeads positions loaded into registers first (all in flight
// together, each read once): the same sums in the same order, bit for bit
#ifndef IGM_SPRITE_REG_BEADS
// segments whose positions the final Rg^2 pass keeps in registers (more: two passes of loads).
// 20 needed 146 VGPRs (3 waves per SIMD): SPRITE 3.95 ms; 12 (86 VGPRs) 3.45 ms; 10 3.02 ms;
// 8 (70 VGPRs) 3.07 ms (200 kb x 1000, 20 000 clusters of <= 20 segments, profiles/r05_de)
#define IGM_SPRITE_REG_BEADS 10
#endif
constexpr int kRegBeads = IGM_SPRITE_REG_BEADS;
template <class Bead>
__device__ __forceinline__ float rg2_regs(const float* __restrict__ xyz, int S, int s, int n, Bead bead) {
    if (n > kRegBeads) return rg2_of(xyz, S, s, n, bead);
    float px[kRegBeads], py[kRegBeads], pz[kRegBeads];
#pragma unroll
    for (int i = 0; i < kRegBeads; ++i)
        if (i < n) load3(xyz, S, bead(i), s, px[i], py[i], pz[i]);
    float mx = 0.0f, my = 0.0f, mz = 0.0f;
#pragma unroll
    for (int i = 0; i < kRegBeads; ++i)
        if (i < n) {
            mx = __fadd_rn(mx, px[i]);
            my = __fadd_rn(my, py[i]);
            mz = __fadd_rn(mz, pz[i]);
        }
    const float fn = (float)n;
    mx = __fdiv_rn(mx, fn);
    my = __fdiv_rn(my, fn);
    mz = __fdiv_rn(mz, fn);
    float rg = 0.0f;
#pragma unroll
    for (int i = 0; i < kRegBeads; ++i)
        if (i < n) {
            const float dx = __fsub_rn(px[i], mx), dy = __fsub_rn(py[i], my), dz = __fsub_rn(pz[i], mz);
            rg = __fadd_rn(rg, __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
        }
    return __fdiv_rn(rg, fn);
}

// Python indexing of a copy list by the selected copy: -1 (no combination below INF)
// wraps to the last copy, as curr_beads[sel] does in sprite.pyx:268
__device__ __forceinline__ int alt_of(const SpriteArgs& A, int region, int k) {
    const int a0 = A.alt_ptr[region], n = A.alt_ptr[region + 1] - a0;
    return A.alt_bead[a0 + (k < 0 ? n + k : k)];
}

// One thread per (cluster, structure), consecutive structures across the wave so the
// coordinate gathers of a bead are contiguous.
//  single-chromosome clusters (no representatives): every copy k of the segments is a
//    group; the group with the smallest Rg^2 (first on ties, sprite.pyx:184-200) wins;
//  multi-chromosome clusters: get_rg2s_cpp over the representatives' copy
//    combinations (mixed radix, first representative fastest; strict <, first found),
//    then Rg^2 of all segments with each chromosome's selected copy (sprite.pyx:231-283).
// Every Rg^2 goes through get_rg2s_cpp in the reference, so a value not below INF
// reads as INF.
__global__ void __launch_bounds__(kBT) sprite_rg2_kernel(SpriteArgs A) {
    const int c = blockIdx.x / A.nsb;
    const int s = (blockIdx.x - c * A.nsb) * kBT + threadIdx.x;
    if (c >= A.ncl || s >= A.S) return;
    const int g0 = A.seg_ptr[c], ng = A.seg_ptr[c + 1] - g0;
    const int r0 = A.rep_ptr[c], nr = A.rep_ptr[c + 1] - r0;
    const int S = A.S;
    float best;
    const int nc2 = A.ncomb2[c];
    if (nc2 > 0 && nr <= kRegReps) {
        // the tables: every bead id one uniform load, no chain of index loads per bead
        const int2* sb = A.seg_b2 + g0;
        if (nr == 0) {
            const int nalt = sb[0].x != sb[0].y ? 2 : 1;
            best = kSpriteInf;
            int bk = 0;
            for (int k = 0; k < nalt; ++k) {
                float v = rg2_regs(A.xyz, S, s, ng, [&](int i) { return k ? sb[i].y : sb[i].x; });
                v = v < kSpriteInf ? v : kSpriteInf;
                if (k == 0 || v < best) {
                    best = v;
                    bk = k;
                }
            }
            for (int i = 0; i < ng; ++i) A.sel[(size_t)(g0 + i) * S + s] = bk ? sb[i].y : sb[i].x;
        } else {
            const int2* rb = A.rep_b2 + r0;
            const unsigned char* rbit = A.rep_bit + r0;
            float px[kRegReps][2], py[kRegReps][2], pz[kRegReps][2];
            int sh[kRegReps];
#pragma unroll
            for (int i = 0; i < kRegReps; ++i)
                if (i < nr) {
                    load3(A.xyz, S, rb[i].x, s, px[i][0], py[i][0], pz[i][0]);
                    load3(A.xyz, S, rb[i].y, s, px[i][1], py[i][1], pz[i][1]);
                    sh[i] = rbit[i];
                }
            float bv = kSpriteInf;
            int bcomb = -1;
            const float fn = (float)nr;
            for (int k = 0; k < nc2; ++k) {  // mixed radix, representative 0 fastest
                float mx = 0.0f, my = 0.0f, mz = 0.0f;
#pragma unroll
                for (int i = 0; i < kRegReps; ++i)
                    if (i < nr) {
                        const int ci = (k >> sh[i]) & 1;
                        mx = __fadd_rn(mx, ci ? px[i][1] : px[i][0]);
                        my = __fadd_rn(my, ci ? py[i][1] : py[i][0]);
                        mz = __fadd_rn(mz, ci ? pz[i][1] : pz[i][0]);
                    }
                mx = __fdiv_rn(mx, fn);
                my = __fdiv_rn(my, fn);
                mz = __fdiv_rn(mz, fn);
                float rg = 0.0f;
#pragma unroll
                for (int i = 0; i < kRegReps; ++i)
                    if (i < nr) {
                        const int ci = (k >> sh[i]) & 1;
                        const float dx = __fsub_rn(ci ? px[i][1] : px[i][0], mx),
                                    dy = __fsub_rn(ci ? py[i][1] : py[i][0], my),
                                    dz = __fsub_rn(ci ? pz[i][1] : pz[i][0], mz);
                        rg = __fadd_rn(rg, __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
                    }
                const float v = __fdiv_rn(rg, fn);
                if (v < bv) {
                    bv = v;
                    bcomb = k;
                }
            }
            // each segment with its chromosome's selected copy; no combination below INF
            // (bcomb -1, all bits set) selects the last copy, .y
            const unsigned char* sbit = A.seg_bit + g0;
            const unsigned m = (unsigned)bcomb;
            auto bead = [=](int i) { return (m >> sbit[i]) & 1u ? sb[i].y : sb[i].x; };
            for (int i = 0; i < ng; ++i) A.sel[(size_t)(g0 + i) * S + s] = bead(i);
            best = rg2_regs(A.xyz, S, s, ng, bead);
            best = best < kSpriteInf ? best : kSpriteInf;
        }
    } else if (nr == 0) {
        const int nalt = A.alt_ptr[A.seg_region[g0] + 1] - A.alt_ptr[A.seg_region[g0]];
        best = kSpriteInf;
        int bk = 0;
        for (int k = 0; k < nalt; ++k) {
            float v = rg2_regs(A.xyz, S, s, ng, [&](int i) { return alt_of(A, A.seg_region[g0 + i], k); });
            v = v < kSpriteInf ? v : kSpriteInf;
            if (k == 0 || v < best) {
                best = v;
                bk = k;
            }
        }
        for (int i = 0; i < ng; ++i) A.sel[(size_t)(g0 + i) * S + s] = alt_of(A, A.seg_region[g0 + i], bk);
    } else {
        int ncomb = 1, two = 1;
        int nalt[kMaxReps], bit[kMaxReps];  // bit: position of representative i's copy digit (copies <= 2)
        for (int i = 0; i < nr; ++i) {
            const int rg = A.rep_region[r0 + i];
            nalt[i] = A.alt_ptr[rg + 1] - A.alt_ptr[rg];
            bit[i] = 0;
            two &= nalt[i] >= 1 && nalt[i] <= 2;
            ncomb *= nalt[i];
        }
        float bv = kSpriteInf;
        int bcomb = -1;
        if (two && nr <= kRegReps) {
            // Every combination reads the same 2 nr bead columns: load them once (all in
            // flight together) and form the combinations from registers, in the reference's
            // order and arithmetic (mixed radix with copies <= 2: digit i is bit bit[i] of k).
            float px[kRegReps][2], py[kRegReps][2], pz[kRegReps][2];
            int b = 0;
#pragma unroll
            for (int i = 0; i < kRegReps; ++i) {
                if (i < nr) {
                    const int rg = A.rep_region[r0 + i];
                    load3(A.xyz, S, alt_of(A, rg, 0), s, px[i][0], py[i][0], pz[i][0]);
                    load3(A.xyz, S, alt_of(A, rg, nalt[i] - 1), s, px[i][1], py[i][1], pz[i][1]);
                    bit[i] = b;
                    b += nalt[i] - 1;
                }
            }
            const float fn = (float)nr;
            for (int k = 0; k < ncomb; ++k) {
                float mx = 0.0f, my = 0.0f, mz = 0.0f;
#pragma unroll
                for (int i = 0; i < kRegReps; ++i)
                    if (i < nr) {
                        const int ci = (k >> bit[i]) & (nalt[i] - 1);
                        mx = __fadd_rn(mx, ci ? px[i][1] : px[i][0]);
                        my = __fadd_rn(my, ci ? py[i][1] : py[i][0]);
                        mz = __fadd_rn(mz, ci ? pz[i][1] : pz[i][0]);
                    }
                mx = __fdiv_rn(mx, fn);
                my = __fdiv_rn(my, fn);
                mz = __fdiv_rn(mz, fn);
                float rg = 0.0f;
#pragma unroll
                for (int i = 0; i < kRegReps; ++i)
                    if (i < nr) {
                        const int ci = (k >> bit[i]) & (nalt[i] - 1);
                        const float dx = __fsub_rn(ci ? px[i][1] : px[i][0], mx),
                                    dy = __fsub_rn(ci ? py[i][1] : py[i][0], my),
                                    dz = __fsub_rn(ci ? pz[i][1] : pz[i][0], mz);
                        rg = __fadd_rn(rg, __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
                    }
                const float v = __fdiv_rn(rg, fn);
                if (v < bv) {
                    bv = v;
                    bcomb = k;
                }
            }
        } else {
            for (int k = 0; k < ncomb; ++k) {
                const float v = rg2_of(A.xyz, S, s, nr, [&](int i) {
                    int kk = k, ci = 0;
                    for (int j = 0; j <= i; ++j) {
                        ci = kk % nalt[j];
                        kk /= nalt[j];
                    }
                    return alt_of(A, A.rep_region[r0 + i], ci);
                });
                if (v < bv) {
                    bv = v;
                    bcomb = k;
                }
            }
        }
        // the chosen copy of representative i (-1 when no combination was below INF)
        auto choice = [&](int i) {
            if (bcomb < 0) return -1;
            int kk = bcomb, ci = 0;
            for (int j = 0; j <= i; ++j) {
                ci = kk % nalt[j];
                kk /= nalt[j];
            }
            return ci;
        };
        // the segments with each chromosome's selected copy: the beads from the tables (no
        // re-read of the selection just stored)
        for (int i = 0; i < ng; ++i)
            A.sel[(size_t)(g0 + i) * S + s] = alt_of(A, A.seg_region[g0 + i], choice(A.seg_rep[g0 + i]));
        best = rg2_regs(A.xyz, S, s, ng, [&](int i) { return alt_of(A, A.seg_region[g0 + i], choice(A.seg_rep[g0 + i])); });
        best = best < kSpriteInf ? best : kSpriteInf;
    }
    A.rg2[(size_t)c * S + s] = best;
}

// keep_best (SpriteAssignmentStep.py:138-143): the keep_best smallest Rg^2 of a
// cluster in increasing order (ties by structure index), their values and the
// selected beads of those structures, row-major (keep_best, len(cluster)).  The rank of
// every structure comes from the block's stable sort of the column (stable_rank), where
// counting each rank against the whole column was O(S^2) per cluster (7.7 of the 11 ms
// of config D/E's SPRITE step).
__global__ void __launch_bounds__(kBT) sprite_keep_best_kernel(const float* __restrict__ rg2, const int* __restrict__ sel,
                                                               const int* __restrict__ seg_ptr, int S, int kb,
                                                               int* __restrict__ best_idx, float* __restrict__ best_val,
                                                               int* __restrict__ best_sel) {
    extern __shared__ float ksm[];
    const int c = blockIdx.x;
    const int npad = pow2_at_least(S);
    float* sk = ksm + S;
    int* si = reinterpret_cast<int*>(sk + npad);
    int* rk = si + npad;
    const float* v = rg2 + (size_t)c * S;
    for (int s = threadIdx.x; s < S; s += kBT) ksm[s] = v[s];
    const float* const cols[1] = {ksm};
    int* const ranks[1] = {rk};
    stable_rank<1>(cols, S, npad, sk, si, ranks);
    const int g0 = seg_ptr[c], ng = seg_ptr[c + 1] - g0;
    for (int s = threadIdx.x; s < S; s += kBT) {
        const int r = rk[s];
        if (r < kb) {
            best_idx[(size_t)c * kb + r] = s;
            best_val[(size_t)c * kb + r] = ksm[s];
            int* out = best_sel + (size_t)g0 * kb + (size_t)r * ng;
            for (int i = 0; i < ng; ++i) out[i] = sel[(size_t)(g0 + i) * S + s];
        }
    }
}

// keep_best by counting every rank against the column: the fallback for populations
// whose sort scratch does not fit (S > ~9 000), LDS of the column only
__global__ void __launch_bounds__(kBT) sprite_keep_best_count_kernel(const float* __restrict__ rg2,
                                                                     const int* __restrict__ sel,
                                                                     const int* __restrict__ seg_ptr, int S, int kb,
                                                                     int* __restrict__ best_idx,
                                                                     float* __restrict__ best_val,
                                                                     int* __restrict__ best_sel) {
    extern __shared__ float ksm[];
    const int c = blockIdx.x;
    const float* v = rg2 + (size_t)c * S;
    for (int s = threadIdx.x; s < S; s += kBT) ksm[s] = v[s];
    __syncthreads();
    const int g0 = seg_ptr[c], ng = seg_ptr[c + 1] - g0;
    for (int s = threadIdx.x; s < S; s += kBT) {
        const float x = ksm[s];
        int r = 0;
        for (int t = 0; t < S && r < kb; ++t) {
            const float y = ksm[t];
            r += (y < x) | ((y == x) & (t < s));
        }
        if (r < kb) {
            best_idx[(size_t)c * kb + r] = s;
            best_val[(size_t)c * kb + r] = x;
            int* out = best_sel + (size_t)g0 * kb + (size_t)r * ng;
            for (int i = 0; i < ng; ++i) out[i] = sel[(size_t)(g0 + i) * S + s];
        }
    }
}

// LDS of sprite_keep_best_kernel: the column, the sort's keys and indices, the ranks
constexpr size_t kSortLdsMax = (size_t)160 * 1024 - 1024;  // one CU's LDS, less the static part
inline size_t keep_best_lds(int S) { return sizeof(float) * (2 * (size_t)S + 2 * (size_t)pow2_at_least(S)); }

// ============================================================================ polymer
// PolymerAssignmentStep.task (igm/steps/PolymerAssignmentStep.py:84-129): for locus i,
// the S distances |x_i - x_(i+1)| (get_polymer_dists, :24-32, float32 norms) are
// ranked -- argsort(argsort(d)), ties in structure order -- and structure s receives
// the rank-th smallest of S distances drawn from the bin distribution
// (np.sort(np.random.choice(edges, S, p=prob)), :113).  The draws arrive as the
// uniforms random_sample() produced for that choice; the bin of a draw is
// cdf.searchsorted(u, side='right') as RandomState.choice computes it.  The sorted
// draws are never materialised: a per-locus histogram over the bins in VALUE order,
// prefix-summed, answers "rank-th smallest" by binary search.
struct PolymerArgs {
    const float* xyz;    // (nbead, S, 3)
    int S;
    const int* loci;
    int nloci;
    const double* u;     // (nloci, S)
    int nbins;
    const double* cdf;   // (nbins) p.cumsum() / last
    const int* vpos;     // (nbins) position of each bin in value order
    const double* vsort; // (nbins) bin values in value order
    float* out;          // (nloci, S)
    float* dist;         // (nloci, S) or null
};

__global__ void __launch_bounds__(kBT) polymer_kernel(PolymerArgs A) {
    extern __shared__ __attribute__((aligned(16))) float psm[];
    const int q = blockIdx.x;
    if (q >= A.nloci) return;
    const int S = A.S, nb = A.nbins, t = threadIdx.x;
    float* d = psm;
    int* cnt = reinterpret_cast<int*>(psm + S);  // nb counts, then the inclusive prefix
    // the bin tables staged in LDS (after the sort's scratch and the ranks): every structure's
    // cdf search and rank lookup then costs LDS round trips instead of global ones
    const int npad = pow2_at_least(S);
    double* lcdf = reinterpret_cast<double*>(psm + ((S + nb + 2 * npad + S + 1) & ~1));
    double* lvs = lcdf + nb;
    int* lvp = reinterpret_cast<int*>(lvs + nb);
    for (int b = t; b < nb; b += kBT) {
        cnt[b] = 0;
        lcdf[b] = A.cdf[b];
        lvs[b] = A.vsort[b];
        lvp[b] = A.vpos[b];
    }
    __syncthreads();
    const int i = A.loci[q];
    const double* u = A.u + (size_t)q * S;
    for (int s = t; s < S; s += kBT) {
        float x, y, z, a, b, c;
        load3(A.xyz, S, i, s, x, y, z);
        load3(A.xyz, S, i + 1, s, a, b, c);
        d[s] = norm3(__fsub_rn(x, a), __fsub_rn(y, b), __fsub_rn(z, c));
        const double uv = u[s];
        int lo = 0, hi = nb;  // first k with cdf[k] > u
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (lcdf[mid] <= uv) lo = mid + 1;
            else hi = mid;
        }
        atomicAdd(&cnt[lvp[lo < nb ? lo : nb - 1]], 1);
    }
    __syncthreads();
    if (t < 64) {  // inclusive prefix over the bins: one wave, a chunk per lane
        const int per = (nb + 63) / 64, b0 = t * per, b1 = min(nb, b0 + per);
        int run = 0;
        for (int b = b0; b < b1; ++b) run += cnt[b];
        int incl = run;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (t >= o) incl += v;
        }
        run = incl - run;
        for (int b = b0; b < b1; ++b) {
            run += cnt[b];
            cnt[b] = run;
        }
    }
    __syncthreads();
    // the ranks of the distances (block_stable_rank)
    float* sk = reinterpret_cast<float*>(cnt + nb);
    int* si = reinterpret_cast<int*>(sk + npad);
    int* rk = si + npad;
    const float* const cols[1] = {d};
    int* const ranks[1] = {rk};
    stable_rank<1>(cols, S, npad, sk, si, ranks);
    const size_t row = (size_t)q * S;
    for (int s = t; s < S; s += kBT) {
        const float ds = d[s];
        const int r = rk[s];
        int lo = 0, hi = nb - 1;  // first value position whose prefix count exceeds r
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (cnt[mid] > r) hi = mid;
            else lo = mid + 1;
        }
        A.out[row + s] = __double2float_rn(lvs[lo]);
        if (A.dist) A.dist[row + s] = ds;
    }
}

// ---- Populations past the LDS-resident rank kernels (fish_lds / polymer LDS > one CU's
// LDS: about 4 000 / 8 000 structures).  The population size is unbounded in the reference
// (ModelingStep.py:111, FishAssignmentStep.py:221-242, PolymerAssignmentStep.py:84-129), so
// these take any S: the columns go to HBM scratch (kernel 1, one thread per (item,
// structure)), and every structure's rank is counted against its whole column (kernel 2,
// the column read in the same order by every lane: one broadcast load per step).  O(S^2)
// compares per item, the same ranks as the sort (ties by structure index).
__global__ void __launch_bounds__(kBT) fish_columns_kernel(FishArgs A, float* col) {
    const int q = blockIdx.y, s = blockIdx.x * kBT + threadIdx.x;
    if (q >= A.nitems || s >= A.S) return;
    const int S = A.S;
    int a0, na, b0 = 0, nb = 0;
    if (A.kind == 0) {
        const int h = A.items[q];
        a0 = A.cptr[h];
        na = A.cptr[h + 1] - a0;
    } else {
        const int h = A.items[2 * q], g = A.items[2 * q + 1];
        a0 = A.cptr[h];
        na = A.cptr[h + 1] - a0;
        b0 = A.cptr[g];
        nb = A.cptr[g + 1] - b0;
    }
    float mn = INFINITY, mx = -INFINITY;
    for (int a = 0; a < na; ++a) {
        float x, y, z;
        load3(A.xyz, S, A.cidx[a0 + a], s, x, y, z);
        if (A.kind == 0) {
            const float d = norm3(x, y, z);
            mn = d < mn ? d : mn;
            mx = d > mx ? d : mx;
        } else {
            for (int b = 0; b < nb; ++b) {
                float u, v, w;
                load3(A.xyz, S, A.cidx[b0 + b], s, u, v, w);
                const float d = norm3(__fsub_rn(x, u), __fsub_rn(y, v), __fsub_rn(z, w));
                mn = d < mn ? d : mn;
                mx = d > mx ? d : mx;
            }
        }
    }
    col[(size_t)q * 2 * S + s] = mn;
    col[(size_t)q * 2 * S + S + s] = mx;
}

__global__ void __launch_bounds__(kBT) fish_count_kernel(FishArgs A, const float* col) {
    const int q = blockIdx.y, s = blockIdx.x * kBT + threadIdx.x, S = A.S;
    if (q >= A.nitems) return;
    const float* vmin = col + (size_t)q * 2 * S;
    const float* vmax = vmin + S;
    const int ss = s < S ? s : S - 1;  // (lanes past S count along, store nothing)
    const float mn = vmin[ss], mx = vmax[ss];
    int rmin = 0, rmax = 0;
    for (int t = 0; t < S; ++t) {
        const float a = vmin[t], b = vmax[t];
        rmin += (a < mn) | ((a == mn) & (t < ss));
        rmax += (b < mx) | ((b == mx) & (t < ss));
    }
    if (s >= S) return;
    const size_t row = (size_t)q * S;
    if (A.omin) A.omin[row + s] = A.tmin[row + rmin];
    if (A.omax) A.omax[row + s] = A.tmax[row + rmax];
    if (A.dmin) A.dmin[row + s] = mn;
    if (A.dmax) A.dmax[row + s] = mx;
}

// polymer past the LDS kernel: distances to HBM scratch and the per-locus bin histogram by
// integer atomics (the same counts in any order), then ranks counted per structure and the
// histogram's prefix (in the block's LDS, nb bins) searched as polymer_kernel does
__global__ void __launch_bounds__(kBT) polymer_columns_kernel(PolymerArgs A, float* col, int* hist) {
    const int q = blockIdx.y, s = blockIdx.x * kBT + threadIdx.x, S = A.S, nb = A.nbins;
    if (q >= A.nloci || s >= S) return;
    const int i = A.loci[q];
    float x, y, z, a, b, c;
    load3(A.xyz, S, i, s, x, y, z);
    load3(A.xyz, S, i + 1, s, a, b, c);
    col[(size_t)q * S + s] = norm3(__fsub_rn(x, a), __fsub_rn(y, b), __fsub_rn(z, c));
    const double uv = A.u[(size_t)q * S + s];
    int lo = 0, hi = nb;  // first k with cdf[k] > u
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (A.cdf[mid] <= uv) lo = mid + 1;
        else hi = mid;
    }
    atomicAdd(&hist[(size_t)q * nb + A.vpos[lo < nb ? lo : nb - 1]], 1);
}

__global__ void __launch_bounds__(kBT) polymer_count_kernel(PolymerArgs A, const float* col, const int* hist) {
    extern __shared__ int pcnt[];  // nb: the inclusive prefix of the locus' histogram
    const int q = blockIdx.y, t = threadIdx.x, s = blockIdx.x * kBT + t, S = A.S, nb = A.nbins;
    if (q >= A.nloci) return;
    if (t < 64) {  // one wave, a chunk of bins per lane
        const int* h = hist + (size_t)q * nb;
        const int per = (nb + 63) / 64, b0 = t * per, b1 = min(nb, b0 + per);
        int run = 0;
        for (int b = b0; b < b1; ++b) run += h[b];
        int incl = run;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (t >= o) incl += v;
        }
        run = incl - run;
        for (int b = b0; b < b1; ++b) {
            run += h[b];
            pcnt[b] = run;
        }
    }
    __syncthreads();
    const float* d = col + (size_t)q * S;
    const int ss = s < S ? s : S - 1;
    const float ds = d[ss];
    int r = 0;
    for (int k = 0; k < S; ++k) {
        const float e = d[k];
        r += (e < ds) | ((e == ds) & (k < ss));
    }
    if (s >= S) return;
    int lo = 0, hi = nb - 1;  // first value position whose prefix count exceeds r
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (pcnt[mid] > r) hi = mid;
        else lo = mid + 1;
    }
    const size_t row = (size_t)q * S;
    A.out[row + s] = __double2float_rn(A.vsort[lo]);
    if (A.dist) A.dist[row + s] = ds;
}

}  // namespace

// ============================================================================ C ABI
extern "C" int igm_damid_actdist(igm_ctx* c, uint32_t flags, const float* xyz, int32_t nbead, int32_t nstruct,
                                 const float* radii, const int32_t* copy_ptr, const int32_t* copy_idx, int32_t nhap,
                                 const int32_t* loci, const float* p_exp, const float* plast, int32_t nloci,
                                 int32_t it_corr, double contact_range, int32_t shape, const double* nucleus_param,
                                 igm_pair_result* per_locus, igm_damid_row* rows, int64_t row_capacity,
                                 int64_t* nrows_out) {
    if (!c) return IGM_E_INVALID;
    if (nbead <= 0 || nstruct <= 0 || nhap <= 0 || nloci < 0 || !xyz || !radii || !copy_ptr || !copy_idx ||
        (nloci > 0 && (!loci || !p_exp || !plast)) || !nrows_out || (shape < 0 || shape > IGM_DAMID_EXP_MAP) ||
        (shape != IGM_DAMID_EXP_MAP && !nucleus_param))
        return fail(c, IGM_E_INVALID, "igm_damid_actdist: invalid arguments");
    if (shape == IGM_DAMID_EXP_MAP && (c->vol_nmap <= 0 || (c->vol_nsmap > 0 && c->vol_nsmap != nstruct)))
        return fail(c, IGM_E_INVALID,
                    "igm_damid_actdist: exp_map needs maps staged by igm_mstep_set_volumes with one map index per "
                    "structure (%d staged, %d structures)", c->vol_nsmap, nstruct);
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    *nrows_out = 0;
    if (nloci == 0) return IGM_OK;
    int32_t ncopy = 0;
    if (flags & IGM_DEVICE_PTRS) {
        IGM_HIP_CHECK(c, hipMemcpyAsync(&ncopy, copy_ptr + nhap, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    } else {
        ncopy = copy_ptr[nhap];
    }
    const float *d_xyz, *d_radii, *d_pexp, *d_plast;
    const int32_t *d_cptr, *d_cidx, *d_loci;
    IGM_TRY(to_device(c, flags, "dm_xyz", xyz, (size_t)nbead * nstruct * 3, &d_xyz));
    IGM_TRY(to_device(c, flags, "dm_radii", radii, (size_t)nbead, &d_radii));
    IGM_TRY(to_device(c, flags, "dm_cptr", copy_ptr, (size_t)nhap + 1, &d_cptr));
    IGM_TRY(to_device(c, flags, "dm_cidx", copy_idx, (size_t)ncopy, &d_cidx));
    IGM_TRY(to_device(c, flags, "dm_loci", loci, (size_t)nloci, &d_loci));
    IGM_TRY(to_device(c, flags, "dm_pexp", p_exp, (size_t)nloci, &d_pexp));
    IGM_TRY(to_device(c, flags, "dm_plast", plast, (size_t)nloci, &d_plast));
    void *p_bad, *p_nr, *p_off;
    IGM_TRY(workspace(c, "dm_bad", sizeof(int), &p_bad));
    IGM_TRY(workspace(c, "dm_nr", (size_t)nloci * sizeof(int64_t), &p_nr));
    IGM_TRY(workspace(c, "dm_off", (size_t)nloci * sizeof(int64_t), &p_off));
    const unsigned g1 = (unsigned)ceil_div(nloci, 256);
    IGM_HIP_CHECK(c, hipMemsetAsync(p_bad, 0, sizeof(int), c->stream));
    hipLaunchKernelGGL(check_loci_kernel, dim3(g1), dim3(256), 0, c->stream, d_loci, nloci, nhap, (int*)p_bad);
    IGM_HIP_CHECK(c, hipGetLastError());
    int bad = 0;
    IGM_HIP_CHECK(c, hipMemcpyAsync(&bad, p_bad, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    if (bad) return fail(c, IGM_E_INVALID, "igm_damid_actdist: locus index outside [0, %d)", nhap);
    int64_t* d_nr = (int64_t*)p_nr;
    int64_t* d_off = (int64_t*)p_off;
    hipLaunchKernelGGL(damid_nrows_kernel, dim3(g1), dim3(256), 0, c->stream, d_loci, nloci, d_cptr, d_nr);
    IGM_HIP_CHECK(c, hipGetLastError());
    size_t tmp_bytes = 0;
    IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, d_nr, d_off, (int)nloci, c->stream));
    void* d_tmp;
    IGM_TRY(workspace(c, "dm_scan_tmp", tmp_bytes, &d_tmp));
    IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_bytes, d_nr, d_off, (int)nloci, c->stream));
    int64_t last_off = 0, last_n = 0;
    IGM_HIP_CHECK(c, hipMemcpyAsync(&last_off, d_off + nloci - 1, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipMemcpyAsync(&last_n, d_nr + nloci - 1, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    const int64_t total = last_off + last_n;
    *nrows_out = total;
    if (total > row_capacity || (total > 0 && !rows))
        return fail(c, IGM_E_OVERFLOW, "igm_damid_actdist: %lld rows exceed capacity %lld", (long long)total,
                    (long long)row_capacity);
    igm_pair_result* d_res;
    if (per_locus && (flags & IGM_DEVICE_PTRS)) {
        d_res = per_locus;
    } else {
        void* p;
        IGM_TRY(workspace(c, "dm_res", (size_t)nloci * sizeof(igm_pair_result), &p));
        d_res = (igm_pair_result*)p;
    }
    igm_damid_row* d_rows;
    IGM_TRY(out_device(c, flags, "dm_rows", rows, (size_t)total, &d_rows));
    if (shape == IGM_DAMID_EXP_MAP) {
        DamidExpArgs E;
        E.xyz = d_xyz;
        E.S = nstruct;
        E.cptr = d_cptr;
        E.cidx = d_cidx;
        E.loci = d_loci;
        E.pexp = d_pexp;
        E.plast = d_plast;
        E.nloci = nloci;
        E.it_corr = it_corr;
        E.cr = contact_range;
        void *pm, *pv, *ps;
        IGM_TRY(workspace(c, "vol_maps", 1, &pm));
        IGM_TRY(workspace(c, "vol_vox", 1, &pv));
        E.maps = (const igm::ms::VolMapDev*)pm;
        E.vox = (const int4*)pv;
        if (c->vol_nsmap > 0) {
            IGM_TRY(workspace(c, "vol_smap", 1, &ps));
        } else {  // every structure uses map 0
            IGM_TRY(workspace(c, "dm_smap0", sizeof(int) * nstruct, &ps));
            IGM_HIP_CHECK(c, hipMemsetAsync(ps, 0, sizeof(int) * nstruct, c->stream));
        }
        E.smap = (const int*)ps;
        E.res = d_res;
        E.rowoff = d_off;
        E.rows = d_rows;
        {
            Timed tm(c, "damid");
            hipLaunchKernelGGL(damid_exp_kernel, dim3((unsigned)nloci), dim3(kBT), 0, c->stream, E);
            IGM_HIP_CHECK(c, hipGetLastError());
        }
        IGM_TRY(to_host(c, flags, rows, d_rows, (size_t)total));
        if (per_locus && !(flags & IGM_DEVICE_PTRS)) IGM_TRY(to_host(c, flags, per_locus, d_res, (size_t)nloci));
        return finish(c, flags);
    }
    DamidArgs A;
    A.xyz = d_xyz;
    A.S = nstruct;
    A.radii = d_radii;
    A.cptr = d_cptr;
    A.cidx = d_cidx;
    A.loci = d_loci;
    A.pexp = d_pexp;
    A.plast = d_plast;
    A.nloci = nloci;
    A.it_corr = it_corr;
    A.shape = shape;
    for (int k = 0; k < 3; ++k) A.R[k] = nucleus_param[shape == 0 ? 0 : k] * (1.0 - contact_range);
    A.res = d_res;
    A.rowoff = d_off;
    A.rows = d_rows;
    {
        Timed tm(c, "damid");
        hipLaunchKernelGGL(damid_kernel, dim3((unsigned)nloci), dim3(kBT), 0, c->stream, A);
        IGM_HIP_CHECK(c, hipGetLastError());
    }
    IGM_TRY(to_host(c, flags, rows, d_rows, (size_t)total));
    if (per_locus && !(flags & IGM_DEVICE_PTRS)) IGM_TRY(to_host(c, flags, per_locus, d_res, (size_t)nloci));
    return finish(c, flags);
}

extern "C" int igm_fish_assign(igm_ctx* c, uint32_t flags, const float* xyz, int32_t nbead, int32_t nstruct,
                               const int32_t* copy_ptr, const int32_t* copy_idx, int32_t nhap, int32_t kind,
                               const int32_t* items, int32_t nitems, const float* target_min,
                               const float* target_max, float* out_min, float* out_max, float* dist_min,
                               float* dist_max) {
    if (!c) return IGM_E_INVALID;
    if (nbead <= 0 || nstruct <= 0 || nhap <= 0 || nitems < 0 || !xyz || !copy_ptr || !copy_idx ||
        (kind != 0 && kind != 1) || (nitems > 0 && !items) || (out_min && !target_min) || (out_max && !target_max))
        return fail(c, IGM_E_INVALID, "igm_fish_assign: invalid arguments");
    const size_t lds = fish_lds(nstruct);
    const bool big = lds > kSortLdsMax;  // past the LDS-resident rank kernel: columns in HBM, counted ranks
    if (big && nitems > 65535)
        return fail(c, IGM_E_UNSUPPORTED, "igm_fish_assign: %d items at %d structures exceed the grid", nitems,
                    nstruct);
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    if (nitems == 0) return IGM_OK;
    int32_t ncopy = 0;
    if (flags & IGM_DEVICE_PTRS) {
        IGM_HIP_CHECK(c, hipMemcpyAsync(&ncopy, copy_ptr + nhap, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    } else {
        ncopy = copy_ptr[nhap];
        const int per = kind == 0 ? 1 : 2;
        for (int64_t k = 0; k < (int64_t)nitems * per; ++k)
            if (items[k] < 0 || items[k] >= nhap)
                return fail(c, IGM_E_INVALID, "igm_fish_assign: item locus %d outside [0, %d)", items[k], nhap);
    }
    const float *d_xyz, *d_tmin, *d_tmax;
    const int32_t *d_cptr, *d_cidx, *d_items;
    const size_t nout = (size_t)nitems * nstruct;
    IGM_TRY(to_device(c, flags, "fi_xyz", xyz, (size_t)nbead * nstruct * 3, &d_xyz));
    IGM_TRY(to_device(c, flags, "fi_cptr", copy_ptr, (size_t)nhap + 1, &d_cptr));
    IGM_TRY(to_device(c, flags, "fi_cidx", copy_idx, (size_t)ncopy, &d_cidx));
    IGM_TRY(to_device(c, flags, "fi_items", items, (size_t)nitems * (kind == 0 ? 1 : 2), &d_items));
    IGM_TRY(to_device(c, flags, "fi_tmin", out_min ? target_min : nullptr, nout, &d_tmin));
    IGM_TRY(to_device(c, flags, "fi_tmax", out_max ? target_max : nullptr, nout, &d_tmax));
    float *d_omin, *d_omax, *d_dmin, *d_dmax;
    IGM_TRY(out_device(c, flags, "fi_omin", out_min, nout, &d_omin));
    IGM_TRY(out_device(c, flags, "fi_omax", out_max, nout, &d_omax));
    IGM_TRY(out_device(c, flags, "fi_dmin", dist_min, nout, &d_dmin));
    IGM_TRY(out_device(c, flags, "fi_dmax", dist_max, nout, &d_dmax));
    FishArgs A{d_xyz, nstruct, d_cptr, d_cidx, kind, d_items, nitems, d_tmin, d_tmax, d_omin, d_omax, d_dmin, d_dmax};
    if (big) {
        void* col;
        IGM_TRY(workspace(c, "fi_col", sizeof(float) * 2 * nout, &col));
        Timed tm(c, "fish");
        const dim3 g((unsigned)((nstruct + kBT - 1) / kBT), (unsigned)nitems);
        hipLaunchKernelGGL(fish_columns_kernel, g, dim3(kBT), 0, c->stream, A, (float*)col);
        hipLaunchKernelGGL(fish_count_kernel, g, dim3(kBT), 0, c->stream, A, (const float*)col);
        IGM_HIP_CHECK(c, hipGetLastError());
    } else {
        Timed tm(c, "fish");
        if (lds > 65536)
            IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)fish_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)lds));
        hipLaunchKernelGGL(fish_kernel, dim3((unsigned)nitems), dim3(kBT), lds, c->stream, A);
        IGM_HIP_CHECK(c, hipGetLastError());
    }
    IGM_TRY(to_host(c, flags, out_min, d_omin, nout));
    IGM_TRY(to_host(c, flags, out_max, d_omax, nout));
    IGM_TRY(to_host(c, flags, dist_min, d_dmin, nout));
    IGM_TRY(to_host(c, flags, dist_max, d_dmax, nout));
    return finish(c, flags);
}

extern "C" int igm_sprite_assign(igm_ctx* c, uint32_t flags, const float* xyz, int32_t nbead, int32_t nstruct,
                                 int32_t ncluster, const int32_t* seg_ptr, const int32_t* seg_region,
                                 const int32_t* seg_rep, const int32_t* rep_ptr, const int32_t* rep_region,
                                 int32_t nregion, const int32_t* alt_ptr, const int32_t* alt_bead, int32_t keep_best,
                                 float* rg2_out, int32_t* best_idx, float* best_rg2, int32_t* best_sel) {
    if (!c) return IGM_E_INVALID;
    if (nbead <= 0 || nstruct <= 0 || ncluster < 0 || nregion < 0 || !xyz || !seg_ptr || !rep_ptr || !alt_ptr ||
        keep_best < 0 || (keep_best > 0 && (!best_idx || !best_rg2 || !best_sel)))
        return fail(c, IGM_E_INVALID, "igm_sprite_assign: invalid arguments");
    if (keep_best >= nstruct && keep_best > 0)
        return fail(c, IGM_E_INVALID, "igm_sprite_assign: keep_best %d must be < nstruct %d (np.argpartition)",
                    keep_best, nstruct);
    if ((size_t)nstruct * sizeof(float) > (size_t)64 * 1024)
        return fail(c, IGM_E_UNSUPPORTED, "igm_sprite_assign: %d structures exceed the LDS-resident selection",
                    nstruct);
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    if (ncluster == 0) return IGM_OK;
    if (flags & IGM_DEVICE_PTRS)
        return fail(c, IGM_E_UNSUPPORTED, "igm_sprite_assign: host CSR arrays expected (validated on the host)");
    // host validation of the CSR description (the kernels trust it)
    const int nseg = seg_ptr[ncluster], nrep = rep_ptr[ncluster], nalt = alt_ptr[nregion];
    if (seg_ptr[0] != 0 || rep_ptr[0] != 0 || alt_ptr[0] != 0 || nseg < 0 || nrep < 0 || nalt < 0 ||
        (nseg > 0 && (!seg_region || !seg_rep)) || (nrep > 0 && !rep_region) || (nalt > 0 && !alt_bead))
        return fail(c, IGM_E_INVALID, "igm_sprite_assign: malformed CSR arrays");
    for (int r = 0; r < nregion; ++r)
        if (alt_ptr[r + 1] <= alt_ptr[r]) return fail(c, IGM_E_INVALID, "igm_sprite_assign: region %d has no copies", r);
    for (int k = 0; k < nalt; ++k)
        if (alt_bead[k] < 0 || alt_bead[k] >= nbead)
            return fail(c, IGM_E_INVALID, "igm_sprite_assign: bead %d outside [0, %d)", alt_bead[k], nbead);
    for (int q = 0; q < ncluster; ++q) {
        const int g0 = seg_ptr[q], ng = seg_ptr[q + 1] - g0, r0 = rep_ptr[q], nr = rep_ptr[q + 1] - r0;
        if (ng <= 0 || nr < 0 || nr > kMaxReps)
            return fail(c, IGM_E_INVALID, "igm_sprite_assign: cluster %d has %d segments, %d representatives", q, ng,
                        nr);
        long long ncomb = 1;
        for (int i = 0; i < nr; ++i) {
            const int rg = rep_region[r0 + i];
            if (rg < 0 || rg >= nregion) return fail(c, IGM_E_INVALID, "igm_sprite_assign: bad region id");
            ncomb *= alt_ptr[rg + 1] - alt_ptr[rg];
            if (ncomb > (1 << 20)) return fail(c, IGM_E_UNSUPPORTED, "igm_sprite_assign: too many copy combinations");
        }
        int nalt0 = -1;
        for (int i = 0; i < ng; ++i) {
            const int rg = seg_region[g0 + i];
            if (rg < 0 || rg >= nregion) return fail(c, IGM_E_INVALID, "igm_sprite_assign: bad region id");
            const int na = alt_ptr[rg + 1] - alt_ptr[rg];
            if (nr == 0) {
                if (nalt0 >= 0 && na < nalt0)
                    return fail(c, IGM_E_INVALID, "igm_sprite_assign: cluster %d segments differ in copy count", q);
                if (nalt0 < 0) nalt0 = na;
            } else {
                const int rp = seg_rep[g0 + i];
                if (rp < 0 || rp >= nr) return fail(c, IGM_E_INVALID, "igm_sprite_assign: bad representative slot");
                if (alt_ptr[rep_region[r0 + rp] + 1] - alt_ptr[rep_region[r0 + rp]] > na)
                    return fail(c, IGM_E_INVALID, "igm_sprite_assign: segment has fewer copies than its chromosome");
            }
        }
    }
    const float* d_xyz;
    const int32_t *d_sp, *d_sr, *d_srep, *d_rp, *d_rr, *d_ap, *d_ab;
    IGM_TRY(to_device(c, flags, "sp_xyz", xyz, (size_t)nbead * nstruct * 3, &d_xyz));
    IGM_TRY(to_device(c, flags, "sp_sp", seg_ptr, (size_t)ncluster + 1, &d_sp));
    IGM_TRY(to_device(c, flags, "sp_sr", seg_region, (size_t)nseg, &d_sr));
    IGM_TRY(to_device(c, flags, "sp_srep", seg_rep, (size_t)nseg, &d_srep));
    IGM_TRY(to_device(c, flags, "sp_rp", rep_ptr, (size_t)ncluster + 1, &d_rp));
    IGM_TRY(to_device(c, flags, "sp_rr", rep_region, (size_t)nrep, &d_rr));
    IGM_TRY(to_device(c, flags, "sp_ap", alt_ptr, (size_t)nregion + 1, &d_ap));
    IGM_TRY(to_device(c, flags, "sp_ab", alt_bead, (size_t)nalt, &d_ab));
    void *p_rg, *p_sel;
    IGM_TRY(workspace(c, "sp_rg2", (size_t)ncluster * nstruct * sizeof(float), &p_rg));
    IGM_TRY(workspace(c, "sp_sel", (size_t)nseg * nstruct * sizeof(int32_t), &p_sel));
    SpriteArgs A;
    A.xyz = d_xyz;
    A.S = nstruct;
    A.ncl = ncluster;
    A.nsb = (int)ceil_div(nstruct, kBT);
    A.seg_ptr = d_sp;
    A.seg_region = d_sr;
    A.seg_rep = d_srep;
    A.rep_ptr = d_rp;
    A.rep_region = d_rr;
    A.alt_ptr = d_ap;
    A.alt_bead = d_ab;
    A.rg2 = (float*)p_rg;
    A.sel = (int*)p_sel;
    {  // the flat bead tables of the clusters whose regions have 1 or 2 copies
        const char* et = getenv("IGM_SPRITE_TABLES");  // 0: the per-bead index path for every cluster (tests)
        const bool no_tables = et && atoi(et) == 0;
        std::vector<int> nc2(ncluster);
        std::vector<int2> sb2(nseg > 0 ? nseg : 1), rb2(nrep > 0 ? nrep : 1);
        std::vector<unsigned char> sbit(nseg > 0 ? nseg : 1), rbit(nrep > 0 ? nrep : 1);
        auto b2 = [&](int rg) {
            const int a0 = alt_ptr[rg], na = alt_ptr[rg + 1] - a0;
            return make_int2(alt_bead[a0], alt_bead[a0 + (na > 1 ? 1 : 0)]);
        };
        auto ncopy = [&](int rg) { return alt_ptr[rg + 1] - alt_ptr[rg]; };
        for (int q = 0; q < ncluster; ++q) {
            const int g0 = seg_ptr[q], ng = seg_ptr[q + 1] - g0, r0 = rep_ptr[q], nr = rep_ptr[q + 1] - r0;
            bool ok = true;
            int b = 0;
            for (int i = 0; i < nr; ++i) {
                const int rg = rep_region[r0 + i];
                ok = ok && ncopy(rg) <= 2;
                rb2[r0 + i] = b2(rg);
                rbit[r0 + i] = (unsigned char)(ncopy(rg) == 2 ? b : 0);
                b += ncopy(rg) == 2 ? 1 : 0;
            }
            for (int i = 0; i < ng; ++i) {
                const int rg = seg_region[g0 + i];
                // a segment takes its representative's copy bit: only when both have the same
                // copies (a 2-copy segment under a 1-copy representative takes copy 0 in the
                // index path, choice() = 0, but would read another representative's bit here)
                ok = ok && ncopy(rg) <= 2 && (nr == 0 || ncopy(rg) == ncopy(rep_region[r0 + seg_rep[g0 + i]]));
                sb2[g0 + i] = b2(rg);
                sbit[g0 + i] = nr > 0 ? rbit[r0 + seg_rep[g0 + i]] : 0;
            }
            nc2[q] = ok && !no_tables ? 1 << b : 0;
        }
        const int* d_nc2;
        const int2 *d_sb2, *d_rb2;
        const unsigned char *d_sbit, *d_rbit;
        // host-built, so copied whatever IGM_DEVICE_PTRS says about the caller's arrays
        const uint32_t hf = flags & ~(uint32_t)IGM_DEVICE_PTRS;
        IGM_TRY(to_device(c, hf, "sp_nc2", nc2.data(), nc2.size(), &d_nc2));
        IGM_TRY(to_device(c, hf, "sp_sb2", sb2.data(), sb2.size(), &d_sb2));
        IGM_TRY(to_device(c, hf, "sp_sbit", sbit.data(), sbit.size(), &d_sbit));
        IGM_TRY(to_device(c, hf, "sp_rb2", rb2.data(), rb2.size(), &d_rb2));
        IGM_TRY(to_device(c, hf, "sp_rbit", rbit.data(), rbit.size(), &d_rbit));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));  // (the host tables are freed at the end of this scope)
        A.ncomb2 = d_nc2;
        A.seg_b2 = d_sb2;
        A.seg_bit = d_sbit;
        A.rep_b2 = d_rb2;
        A.rep_bit = d_rbit;
    }
    if ((int64_t)ncluster * A.nsb > 0x7fffffff) return fail(c, IGM_E_UNSUPPORTED, "igm_sprite_assign: grid too large");
    int32_t *d_bi = nullptr, *d_bs = nullptr;
    float* d_bv = nullptr;
    const size_t nb = (size_t)ncluster * keep_best, nbs = (size_t)nseg * keep_best;
    IGM_TRY(out_device(c, flags, "sp_bi", best_idx, nb, &d_bi));
    IGM_TRY(out_device(c, flags, "sp_bv", best_rg2, nb, &d_bv));
    IGM_TRY(out_device(c, flags, "sp_bs", best_sel, nbs, &d_bs));
    {
        Timed tm(c, "sprite");
        hipLaunchKernelGGL(sprite_rg2_kernel, dim3((unsigned)(ncluster * A.nsb)), dim3(kBT), 0, c->stream, A);
        IGM_HIP_CHECK(c, hipGetLastError());
        if (keep_best > 0) {
            const size_t klds = keep_best_lds(nstruct);
            if (klds <= kSortLdsMax) {
                if (klds > 65536)
                    IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)sprite_keep_best_kernel,
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)klds));
                hipLaunchKernelGGL(sprite_keep_best_kernel, dim3((unsigned)ncluster), dim3(kBT), klds, c->stream,
                                   (const float*)p_rg, (const int*)p_sel, d_sp, nstruct, keep_best, d_bi, d_bv, d_bs);
            } else {
                hipLaunchKernelGGL(sprite_keep_best_count_kernel, dim3((unsigned)ncluster), dim3(kBT),
                                   (size_t)nstruct * sizeof(float), c->stream, (const float*)p_rg, (const int*)p_sel,
                                   d_sp, nstruct, keep_best, d_bi, d_bv, d_bs);
            }
            IGM_HIP_CHECK(c, hipGetLastError());
        }
    }
    IGM_TRY(to_host(c, flags, rg2_out, (const float*)p_rg, (size_t)ncluster * nstruct));
    if (keep_best > 0) {
        IGM_TRY(to_host(c, flags, best_idx, d_bi, nb));
        IGM_TRY(to_host(c, flags, best_rg2, d_bv, nb));
        IGM_TRY(to_host(c, flags, best_sel, d_bs, nbs));
    }
    return finish(c, flags);
}

extern "C" int igm_polymer_assign(igm_ctx* c, uint32_t flags, const float* xyz, int32_t nbead, int32_t nstruct,
                                  const int32_t* loci, int32_t nloci, const double* uniforms, int32_t nbins,
                                  const double* edges, const double* prob, float* nn_dist, float* dist) {
    if (!c) return IGM_E_INVALID;
    if (nbead < 2 || nstruct <= 0 || nloci < 0 || nbins <= 0 || !xyz || !edges || !prob ||
        (nloci > 0 && (!loci || !uniforms || !nn_dist)))
        return fail(c, IGM_E_INVALID, "igm_polymer_assign: invalid arguments");
    // the distances, the bin counts, the sort's scratch, the ranks (8-byte aligned after), then
    // the bin tables: cdf and values (double), value positions (int)
    const size_t lds = (((size_t)nstruct + nbins + 2 * (size_t)pow2_at_least(nstruct) + nstruct + 1) & ~(size_t)1) *
                           sizeof(float) + (size_t)nbins * (2 * sizeof(double) + sizeof(int));
    // past the LDS-resident kernel: distances and histograms in HBM, counted ranks (the
    // prefix of one locus' histogram in LDS)
    const bool big = lds > kSortLdsMax;
    if (big && ((size_t)nbins * sizeof(int) > kSortLdsMax || nloci > 65535))
        return fail(c, IGM_E_UNSUPPORTED, "igm_polymer_assign: %d loci x %d bins at %d structures exceed the kernels",
                    nloci, nbins, nstruct);
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    if (nloci == 0) return IGM_OK;
    if (flags & IGM_DEVICE_PTRS)
        return fail(c, IGM_E_UNSUPPORTED, "igm_polymer_assign: host distribution arrays expected");
    for (int32_t k = 0; k < nloci; ++k)
        if (loci[k] < 0 || loci[k] >= nbead - 1)
            return fail(c, IGM_E_INVALID, "igm_polymer_assign: locus %d outside [0, %d)", loci[k], nbead - 1);
    // RandomState.choice: cdf = p.cumsum(); cdf /= cdf[-1] (sequential float64 sums)
    std::vector<double> cdf(nbins);
    double run = 0.0;
    for (int b = 0; b < nbins; ++b) cdf[b] = run += prob[b];
    const double last = cdf[nbins - 1];
    for (int b = 0; b < nbins; ++b) cdf[b] /= last;
    // the bins in value order (np.sort of the drawn values)
    std::vector<int> order(nbins), vpos(nbins);
    for (int b = 0; b < nbins; ++b) order[b] = b;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return edges[x] < edges[y]; });
    std::vector<double> vsort(nbins);
    for (int k = 0; k < nbins; ++k) {
        vpos[order[k]] = k;
        vsort[k] = edges[order[k]];
    }
    const size_t nout = (size_t)nloci * nstruct;
    const float* d_xyz;
    const int32_t *d_loci, *d_vpos;
    const double *d_u, *d_cdf, *d_vsort;
    IGM_TRY(to_device(c, flags, "po_xyz", xyz, (size_t)nbead * nstruct * 3, &d_xyz));
    IGM_TRY(to_device(c, flags, "po_loci", loci, (size_t)nloci, &d_loci));
    IGM_TRY(to_device(c, flags, "po_u", uniforms, nout, &d_u));
    IGM_TRY(to_device(c, flags, "po_cdf", (const double*)cdf.data(), (size_t)nbins, &d_cdf));
    IGM_TRY(to_device(c, flags, "po_vpos", (const int32_t*)vpos.data(), (size_t)nbins, &d_vpos));
    IGM_TRY(to_device(c, flags, "po_vsort", (const double*)vsort.data(), (size_t)nbins, &d_vsort));
    float *d_out, *d_dist;
    IGM_TRY(out_device(c, flags, "po_out", nn_dist, nout, &d_out));
    IGM_TRY(out_device(c, flags, "po_dist", dist, nout, &d_dist));
    PolymerArgs A{d_xyz, nstruct, d_loci, nloci, d_u, nbins, d_cdf, d_vpos, d_vsort, d_out, d_dist};
    if (big) {
        void *col, *hist;
        IGM_TRY(workspace(c, "po_col", sizeof(float) * nout, &col));
        IGM_TRY(workspace(c, "po_hist", sizeof(int) * (size_t)nloci * nbins, &hist));
        IGM_HIP_CHECK(c, hipMemsetAsync(hist, 0, sizeof(int) * (size_t)nloci * nbins, c->stream));
        const size_t hl = sizeof(int) * (size_t)nbins;
        if (hl > 65536)
            IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)polymer_count_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)hl));
        Timed tm(c, "polymer");
        const dim3 g((unsigned)((nstruct + kBT - 1) / kBT), (unsigned)nloci);
        hipLaunchKernelGGL(polymer_columns_kernel, g, dim3(kBT), 0, c->stream, A, (float*)col, (int*)hist);
        hipLaunchKernelGGL(polymer_count_kernel, g, dim3(kBT), hl, c->stream, A, (const float*)col,
                           (const int*)hist);
        IGM_HIP_CHECK(c, hipGetLastError());
    } else {
        if (lds > 65536)
            IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)polymer_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        Timed tm(c, "polymer");
        hipLaunchKernelGGL(polymer_kernel, dim3((unsigned)nloci), dim3(kBT), lds, c->stream, A);
        IGM_HIP_CHECK(c, hipGetLastError());
    }
    IGM_TRY(to_host(c, flags, nn_dist, d_out, nout));
    IGM_TRY(to_host(c, flags, dist, d_dist, nout));
    return finish(c, flags);
}

// ============================================================================ contact map
// HicEvaluationStep.reduce (igm/steps/HicEvaluationStep.py:96-179) builds the simulated
// Hi-C map of the population with alabtools' HssFile.buildContactMap(contactRange) (:109)
// before summing the copies.  counts[i, j] = the number of structures with
// |x_i - x_j| <= fl32(contact_range * fl32(r_i + r_j)), the float32 norm of the A/M
// contact test (inter_hic.py:47) against the Hi-C restraint's r0 (hic.py), decided
// exactly on the squared norm (sq_bound).  One
// workgroup per 64x64 bead tile (upper triangle, mirrored on store); the structures
// stream through LDS in chunks of kCS, each thread keeps a 4x4 block of counters.
namespace {
constexpr int kCT = 64;  // beads per tile side
constexpr int kCS = 32;  // structures per LDS chunk
constexpr int kCRow = kCS * 3 + 1;  // padded LDS row (floats)

// The largest float T with  RN(sqrt(d2)) <= dist  <=>  d2 <= T  for every float d2 >= 0
// (sqrt_le's exact bound (dist + ulp/2)^2, rounded down to the float strictly below it):
// the per-structure test is then the float32 squared norm and one compare, no sqrt.
__device__ __forceinline__ float sq_bound(float dist) {
    if (!(dist >= 0.0f)) return -1.0f;
    if (isinf(dist)) return INFINITY;
    const double m = (double)dist + 0.5 * ((double)nextafterf(dist, INFINITY) - (double)dist);
    const double M = m * m;  // exact (m has <= 25 significant bits)
    float t = (float)M;
    if ((double)t >= M) t = nextafterf(t, -INFINITY);
    return t;
}

// HAP: the copies are summed on the device -- counts is (nhap, nhap) and every pair
// (i, j) adds its count to (hap_of[i], hap_of[j]) and (hap_of[j], hap_of[i]) (integer
// atomics: the sum is exact and order-independent); diagonal tiles take each unordered
// pair once.
template <bool HAP>
__global__ void __launch_bounds__(kBT) contact_map_kernel(const float* __restrict__ xyz, int n, int S,
                                                          const float* __restrict__ radii, float cr,
                                                          int* __restrict__ counts, const int* __restrict__ hap_of,
                                                          int nhap) {
    const int bi = blockIdx.y, bj = blockIdx.x;
    if (bj < bi) return;  // upper-triangle tiles only (whole workgroup exits together)
    __shared__ float li[kCT * kCRow];
    __shared__ float lj[kCT * kCRow];
    const int t = threadIdx.x, ti = t >> 4, tj = t & 15;
    const int i0 = bi * kCT, j0 = bj * kCT;
    float thr[4][4];
    int cnt[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const int i = min(i0 + ti * 4 + a, n - 1);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int j = min(j0 + tj * 4 + b, n - 1);
            thr[a][b] = sq_bound(__fmul_rn(cr, __fadd_rn(radii[i], radii[j])));
            cnt[a][b] = 0;
        }
    }
    for (int s0 = 0; s0 < S; s0 += kCS) {
        const int ns = min(kCS, S - s0), w = ns * 3;
        __syncthreads();
        for (int e = t; e < kCT * kCS * 3; e += kBT) {  // stage both bead blocks' chunk rows
            const int r = e / (kCS * 3), c = e - r * (kCS * 3);
            float vi = 0.f, vj = 0.f;
            if (c < w) {
                if (i0 + r < n) vi = xyz[((size_t)(i0 + r) * S + s0) * 3 + c];
                if (j0 + r < n) vj = xyz[((size_t)(j0 + r) * S + s0) * 3 + c];
            }
            li[r * kCRow + c] = vi;
            lj[r * kCRow + c] = vj;
        }
        __syncthreads();
#pragma unroll 1
        for (int s = 0; s < ns; ++s) {
            float xi[4][3], xj[4][3];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    xi[a][k] = li[(ti * 4 + a) * kCRow + s * 3 + k];
                    xj[a][k] = lj[(tj * 4 + a) * kCRow + s * 3 + k];
                }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const float dx = __fsub_rn(xi[a][0], xj[b][0]), dy = __fsub_rn(xi[a][1], xj[b][1]),
                                dz = __fsub_rn(xi[a][2], xj[b][2]);
                    const float d2 = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
                    cnt[a][b] += d2 <= thr[a][b];
                }
        }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const int i = i0 + ti * 4 + a;
        if (i >= n) continue;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int j = j0 + tj * 4 + b;
            if (j >= n) continue;
            if (HAP) {
                if (j < i || cnt[a][b] == 0) continue;  // diagonal tiles: each unordered pair once
                const size_t ha = (size_t)hap_of[i], hb = (size_t)hap_of[j];
                atomicAdd(&counts[ha * nhap + hb], cnt[a][b]);
                if (i != j) atomicAdd(&counts[hb * nhap + ha], cnt[a][b]);
                continue;
            }
            counts[(size_t)i * n + j] = cnt[a][b];
            counts[(size_t)j * n + i] = cnt[a][b];
        }
    }
}
}  // namespace

extern "C" int igm_contact_map(igm_ctx* c, uint32_t flags, const float* xyz, int32_t nbead, int32_t nstruct,
                               const float* radii, double contact_range, int32_t* counts) {
    if (!c) return IGM_E_INVALID;
    if (nbead <= 0 || nstruct <= 0 || !xyz || !radii || !counts || !(contact_range >= 0.0))
        return fail(c, IGM_E_INVALID, "igm_contact_map: invalid arguments");
    const int nt = (int)ceil_div(nbead, kCT);
    if (nt > 65535) return fail(c, IGM_E_UNSUPPORTED, "igm_contact_map: %d beads exceed the tile grid", nbead);
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    const float* d_xyz;
    const float* d_radii;
    IGM_TRY(to_device(c, flags, "cm_xyz", xyz, (size_t)nbead * nstruct * 3, &d_xyz));
    IGM_TRY(to_device(c, flags, "cm_radii", radii, (size_t)nbead, &d_radii));
    int32_t* d_cnt;
    IGM_TRY(out_device(c, flags, "cm_counts", counts, (size_t)nbead * nbead, &d_cnt));
    {
        Timed tm(c, "contact_map");
        hipLaunchKernelGGL(contact_map_kernel<false>, dim3((unsigned)nt, (unsigned)nt), dim3(kBT), 0, c->stream,
                           d_xyz, (int)nbead, (int)nstruct, d_radii, (float)contact_range, (int*)d_cnt,
                           (const int*)nullptr, 0);
        IGM_HIP_CHECK(c, hipGetLastError());
    }
    IGM_TRY(to_host(c, flags, counts, d_cnt, (size_t)nbead * nbead));
    return finish(c, flags);
}

extern "C" int igm_contact_map_haploid(igm_ctx* c, uint32_t flags, const float* xyz, int32_t nbead, int32_t nstruct,
                                       const float* radii, double contact_range, const int32_t* copy_ptr,
                                       const int32_t* copy_idx, int32_t nhap, int32_t* counts) {
    if (!c) return IGM_E_INVALID;
    if (nbead <= 0 || nstruct <= 0 || nhap <= 0 || !xyz || !radii || !copy_ptr || !copy_idx || !counts ||
        !(contact_range >= 0.0))
        return fail(c, IGM_E_INVALID, "igm_contact_map_haploid: invalid arguments");
    const int nt = (int)ceil_div(nbead, kCT);
    if (nt > 65535) return fail(c, IGM_E_UNSUPPORTED, "igm_contact_map_haploid: %d beads exceed the tile grid", nbead);
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    // the haploid locus of every bead from the CSR copy index (host pointers)
    std::vector<int32_t> hap(nbead, -1);
    if (copy_ptr[0] != 0) return fail(c, IGM_E_INVALID, "igm_contact_map_haploid: copy_ptr[0] != 0");
    // every bead belongs to exactly one haploid locus, so copy_idx holds nbead entries:
    // a non-decreasing copy_ptr ending at nbead keeps every read inside it
    for (int a = 0; a < nhap; ++a)
        if (copy_ptr[a + 1] < copy_ptr[a] || copy_ptr[a + 1] > nbead)
            return fail(c, IGM_E_INVALID, "igm_contact_map_haploid: copy_ptr not non-decreasing within [0, %d]", nbead);
    if (copy_ptr[nhap] != nbead)
        return fail(c, IGM_E_INVALID, "igm_contact_map_haploid: copy_ptr[%d] = %d, expected nbead = %d", nhap,
                    copy_ptr[nhap], nbead);
    for (int a = 0; a < nhap; ++a)
        for (int k = copy_ptr[a]; k < copy_ptr[a + 1]; ++k) {
            const int b = copy_idx[k];
            if (b < 0 || b >= nbead || hap[b] >= 0)
                return fail(c, IGM_E_INVALID, "igm_contact_map_haploid: copy index entry %d invalid or repeated", b);
            hap[b] = a;
        }
    for (int b = 0; b < nbead; ++b)
        if (hap[b] < 0) return fail(c, IGM_E_INVALID, "igm_contact_map_haploid: bead %d has no haploid locus", b);
    const float* d_xyz;
    const float* d_radii;
    const int32_t* d_hap;
    IGM_TRY(to_device(c, flags, "cm_xyz", xyz, (size_t)nbead * nstruct * 3, &d_xyz));
    IGM_TRY(to_device(c, flags, "cm_radii", radii, (size_t)nbead, &d_radii));
    IGM_TRY(to_device(c, 0u, "cm_hap", hap.data(), (size_t)nbead, &d_hap));
    int32_t* d_cnt;
    IGM_TRY(out_device(c, flags, "cm_counts", counts, (size_t)nhap * nhap, &d_cnt));
    IGM_HIP_CHECK(c, hipMemsetAsync(d_cnt, 0, sizeof(int32_t) * (size_t)nhap * nhap, c->stream));
    {
        Timed tm(c, "contact_map");
        hipLaunchKernelGGL(contact_map_kernel<true>, dim3((unsigned)nt, (unsigned)nt), dim3(kBT), 0, c->stream,
                           d_xyz, (int)nbead, (int)nstruct, d_radii, (float)contact_range, (int*)d_cnt, d_hap,
                           (int)nhap);
        IGM_HIP_CHECK(c, hipGetLastError());
    }
    IGM_TRY(to_host(c, flags, counts, d_cnt, (size_t)nhap * nhap));
    return finish(c, flags);
}
