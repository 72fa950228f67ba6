// Device building blocks of the M-step engine (mstep.hip): block reductions,
// the cell-list Verlet neighbour build, and the force field of the reference's
// LAMMPS run (lammps.py:63-358):
//   pair soft      E = A [1 + cos(pi r / rc)],  rc = r_i + r_j,  A = evf (rc/pi)^2
//   bond upper/lower bound   E = K (r - r0)^2 beyond the bound (LAMMPS bond_harmonic form)
//   ellipsoidal envelope     E = k/2 t^2, t = (1 - k2^-1/2) |x|, k2 = sum x_d^2/(s_d)^2,
//                            s_d = envf*abc_d - r_i   (k>0: active outside; k<0: inside)
// Every atom's force is GATHERED by the thread that owns the atom (full
// neighbour list, both bond ends): no atomics, fixed summation order, so a run
// is bitwise reproducible.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "igm_ctx.h"

namespace igm {
namespace ms {

constexpr int kCellCap = 4096;  // cells of the per-structure binning grid
constexpr int kMaxWaves = 16;   // 1024 threads

template <typename T>
using vec4_t = typename std::conditional<std::is_same<T, float>::value, float4, double4>::type;

// one volumetric map on the device (igm_volume_map; voxels at vvox + off)
struct VolMapDev {
    int n[3];
    int body;
    float center[3], origin[3], grid[3];
    long long off;
};

// protocol constants shared by every structure of a launch
struct DevParams {
    int nenv;
    int env_kind[IGM_MAX_ENVELOPES];  // IGM_ENV_ELLIPSOID / IGM_ENV_VOLUME
    const VolMapDev* vmaps;           // volume maps (igm_mstep_set_volumes)
    const int4* vvox;
    const int* vsmap;                 // map of structure s (NULL: map 0)
    float env_abc[IGM_MAX_ENVELOPES][3];
    float env_k[IGM_MAX_ENVELOPES];
    double env_abc_d[IGM_MAX_ENVELOPES][3];
    double env_k_d[IGM_MAX_ENVELOPES];
    float cut_list;  // rc_max + skin
    float skin;
    int kcap;        // neighbour capacity per atom
    int natom;
    int nslice;
    // f64 path: the reference's LAMMPS atom types (one per distinct radius,
    // lammps.py:114-146).  pair_tab[ti*ntype+tj] = {dc = f32(ri + rj), rc = the
    // PairIJ cutoff LAMMPS parses from repr(dc)}; rtype = repr(radius) as the
    // 'User' data line is read.
    int ntype;
    const double2* pair_tab;
    const double* rtype;
};

// ------------------------------------------------------------- reductions
#ifndef IGM_DPP_REDUCE
#define IGM_DPP_REDUCE 1
#endif
// a double moved across lanes by one DPP control (both halves, full row/bank masks)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Sum of a double over the 64 lanes, the same bits in every lane.  DPP inside each
// 16-lane row (quad xor 1, quad xor 2, half-row mirror, row mirror: every lane of a
// row then holds the row sum, addition being commutative), then the four row sums
// through readlane -- no LDS-crossbar round trips (ds_bpermute) on the chain.
__device__ __forceinline__ double wave_sum_f64(double v) {
#if IGM_DPP_REDUCE
    v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_f64<0x141>(v);  // row_half_mirror
    v += dpp_f64<0x140>(v);  // row_mirror
    return ((readlane_f64(v, 0) + readlane_f64(v, 16)) + readlane_f64(v, 32)) + readlane_f64(v, 48);
#else
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
#endif
}

// max of a float over the 64 lanes, every lane (exact: the same bits in any order)
__device__ __forceinline__ float wave_max_f32(float v) {
#if IGM_DPP_REDUCE
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xf, 0xf, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xf, 0xf, false)));
    const float a = fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)),
                          __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16)));
    const float b = fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)),
                          __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
    return fmaxf(a, b);
#else
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
#endif
}

// Sum K doubles over the block.  Only lane 0 of each wave publishes; every
// thread then adds the per-wave partials in the same order, so all threads get
// the bitwise identical result (uniform control flow afterwards).  `red` must
// not be rewritten by any thread before all threads have read it: callers
// alternate two buffers or place a barrier.
template <int NT, int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double* red) {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = wave_sum_f64(v[k]);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[w * K + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NT / 64; ++i) s += red[i * K + k];
        v[k] = s;
    }
}

template <int NT, int K>
__device__ __forceinline__ void block_max(double (&v)[K], double* red) {
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v[k] = fmax(v[k], __shfl_xor(v[k], off));
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[w * K + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double s = red[k];
#pragma unroll
        for (int i = 1; i < NT / 64; ++i) s = fmax(s, red[i * K + k]);
        v[k] = s;
    }
}

// ------------------------------------------------------------- RanPark
// LAMMPS RanPark (Park-Miller minimal standard, Schrage): seed_n = seed*16807^n
// mod (2^31-1).  Jump-ahead lets every thread draw its own atoms' numbers.
__device__ __forceinline__ uint32_t mulmod_m31(uint32_t a, uint32_t b) {
    const uint64_t x = (uint64_t)a * (uint64_t)b;  // < 2^62
    uint64_t r = (x & 0x7fffffffull) + (x >> 31);  // Mersenne reduction
    r = (r & 0x7fffffffull) + (r >> 31);
    return (uint32_t)(r >= 0x7fffffffull ? r - 0x7fffffffull : r);
}
__device__ __forceinline__ uint32_t powmod_m31(uint32_t base, uint64_t e) {
    uint32_t r = 1;
    while (e) {
        if (e & 1) r = mulmod_m31(r, base);
        base = mulmod_m31(base, base);
        e >>= 1;
    }
    return r;
}
// uniform() number `n` (1-based) of a RanPark seeded with `seed`
__device__ __forceinline__ double ranpark_nth(uint32_t seed, uint64_t n) {
    const uint32_t s = mulmod_m31(seed % 0x7fffffffu, powmod_m31(16807u, n));
    return (1.0 / 2147483647.0) * (double)s;
}

// ------------------------------------------------------------- force field
// one pair (soft), returns the scalar f/r multiplier; energy added if EN
template <typename T, bool EN>
__device__ __forceinline__ T soft_pair(T r2, T rc, T evf, double& e) {
    if (!(r2 < rc * rc)) return T(0);
    const T r = sqrt(r2);
    const T inv_pi = T(0.318309886183790671537767526745);
    const T pref = evf * rc * inv_pi;  // A * pi / rc
    T s, c;
    if constexpr (std::is_same<T, float>::value) {
        // arg = pi r / rc = 2 pi * (r / (2 rc)): v_sin_f32 / v_cos_f32 take revolutions
        const float rev = 0.5f * r / rc;
        s = __builtin_amdgcn_sinf(rev);
        c = __builtin_amdgcn_cosf(rev);
    } else {
        sincospi(r / rc, &s, &c);
    }
    if (EN) e += (double)(pref * rc * inv_pi) * (1.0 + (double)c);
    return (r > T(0)) ? pref * s / r : T(0);
}

// f64 soft pair exactly as LAMMPS evaluates the printed coefficients:
// A = evf (dc/pi)^2 at full precision, cutoff and argument from the parsed rc
__device__ __forceinline__ double soft_pair_typed(double r2, double dc, double rc, double evf, double& e) {
    if (!(r2 < rc * rc)) return 0.0;
    const double kPi = 3.14159265358979323846;
    const double A = (dc / kPi) * (dc / kPi) * evf;
    const double r = sqrt(r2);
    const double arg = kPi * r / rc;
    double s, c;
    sincos(arg, &s, &c);
    e += A * (1.0 + c);
    return (r > 0.0) ? A * s * kPi / rc / r : 0.0;
}

// bond (harmonic upper/lower bound); returns f/r multiplier
template <typename T, bool EN>
__device__ __forceinline__ T bond_term(T r2, T r0, T k, bool lower, double& e) {
    const T r = sqrt(r2);
    const T dr = r - r0;
    const bool active = lower ? (dr < T(0)) : (dr > T(0));
    if (!active) return T(0);
    const T rk = k * dr;
    if (EN) e += (double)rk * (double)dr;
    return (r > T(0)) ? T(-2) * rk / r : T(0);
}

// branch-free f32 soft pair (the MD kernels): f/r multiplier, 0 outside the cutoff
// or for coincident atoms; all candidates of a batch evaluate together.  evfpi =
// evf / pi; the hardware v_rsq / v_rcp (1 ulp) stand in for the correctly rounded
// forms, whose denormal-safe expansions cost 5 VALU ops each on gfx950.
__device__ __forceinline__ float soft_pair_bf(float r2, float rc, float evfpi) {
    const float rinv = __builtin_amdgcn_rsqf(fmaxf(r2, 1.0e-30f));
    const float r = r2 * rinv;
    const float s = __builtin_amdgcn_sinf(r * (0.5f * __builtin_amdgcn_rcpf(rc)));  // sin(pi r / rc), in revolutions
    const float f = (evfpi * rc) * s * rinv;
    return (r2 < rc * rc && r2 > 0.0f) ? f : 0.0f;
}

// branch-free harmonic upper/lower bound (f/r multiplier)
template <typename T, bool EN>
__device__ __forceinline__ T bond_term_bf(T r2, T r0, T k, bool lower, double& e) {
    const T r = sqrt(r2);
    const T dr = r - r0;
    const bool active = lower ? (dr < T(0)) : (dr > T(0));
    const T rk = k * dr;
    if (EN && active) e += (double)rk * (double)dr;
    return (active && r > T(0)) ? T(-2) * rk / r : T(0);
}

// ellipsoidal envelope on one atom; adds force, returns energy (if EN)
template <typename T, bool EN>
__device__ __forceinline__ void envelope_term(T x, T y, T z, T rad, T a, T b, T c, T k, T& fx, T& fy, T& fz,
                                              double& e) {
    const T sx = a - rad, sy = b - rad, sz = c - rad;
    const T ix = T(1) / (sx * sx), iy = T(1) / (sy * sy), iz = T(1) / (sz * sz);
    const T k2 = x * x * ix + y * y * iy + z * z * iz;
    const bool active = (k > T(0)) ? (k2 > T(1)) : (k2 < T(1) && k2 > T(0));
    if (!active) return;
    const T rn = sqrt(x * x + y * y + z * z);
    const T sk = sqrt(k2);
    const T t = (T(1) - T(1) / sk) * rn;
    const T ka = fabs(k);
    const T A = (T(1) - T(1) / sk) / rn;
    const T B = rn / (k2 * sk);
    fx -= ka * t * (A * x + B * x * ix);
    fy -= ka * t * (A * y + B * y * iy);
    fz -= ka * t * (A * z + B * z * iz);
    if (EN) e += 0.5 * (double)ka * (double)t * (double)t;
}

// volumetric map restraint (IGM_ENV_VOLUME; form documented in igm_hip.h): pulls a
// member atom whose voxel violates the map to its nearest lamina voxel centre
template <typename T, bool EN>
__device__ __forceinline__ void volume_term(T x, T y, T z, const VolMapDev& m, const int4* __restrict__ vox,
                                            T envf, T k, T& fx, T& fy, T& fz, double& e) {
    const T p[3] = {x, y, z};
    T o[3], g[3];
    int v[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        o[d] = (T)m.origin[d] * envf;
        g[d] = (T)m.grid[d] * envf;
        int iv = (int)rint((p[d] - o[d]) / g[d]);
        iv = iv < 0 ? 0 : (iv >= m.n[d] ? m.n[d] - 1 : iv);
        v[d] = iv;
    }
    const int4 r = vox[m.off + ((long long)v[0] * m.n[1] + v[1]) * m.n[2] + v[2]];
    const bool outside_ok = (m.body == 0) == (k > T(0));  // violation = outside (else inside)
    const bool viol = outside_ok ? (r.w == 0) : (r.w != 0);
    if (!viol) return;
    const T dx = x - (o[0] + g[0] * (T)r.x), dy = y - (o[1] + g[1] * (T)r.y), dz = z - (o[2] + g[2] * (T)r.z);
    const T ka = fabs(k);
    fx -= ka * dx;
    fy -= ka * dy;
    fz -= ka * dz;
    if (EN) e += 0.5 * (double)ka * ((double)dx * dx + (double)dy * dy + (double)dz * dz);
}

}  // namespace ms
}  // namespace igm
