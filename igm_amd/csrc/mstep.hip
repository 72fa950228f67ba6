// M-step engine: batched replacement of the per-structure serial LAMMPS run
// (igm/model/kernel/lammps.py:361-492 via ModelingStep.task, ModelingStep.py:508-509).
//
// Design (MI355X-first):
//  * one workgroup = one structure, persistent: it pulls structure ids from an
//    atomic work counter and runs the WHOLE protocol for that structure inside
//    one launch (47 000 MD steps for the demo protocol) -- no per-step launches.
//  * positions live in LDS (float4 x,y,z,radius); each thread owns BPT atoms
//    (a = b*NT + tid) and keeps their velocity, force and last-build position in
//    VGPRs.  Per MD step: one barrier after the position update (fused with the
//    neighbour-displacement vote, __syncthreads_or) and one for the temperature
//    reduction of fix temp/rescale.
//  * neighbours: Verlet list with skin (LAMMPS 'neighbor maxrad bin', 'check yes'),
//    rebuilt in-kernel from an LDS cell grid (count / scan / scatter / per-cell
//    sort -> deterministic order) into a sliced-ELLPACK list in HBM
//    ([slice][k][64 lanes], coalesced per k).
//  * bonds: per-structure sliced-ELLPACK adjacency (both ends) built once by
//    adj_count/adj_fill, sorted per atom for a fixed summation order.
//  * anneal (MD) in f32 with f64 reductions; the CG minimisation (LAMMPS
//    min_style cg, quadratic line search) runs in a second kernel in f64 with
//    f64 positions in LDS, because its energy tests (EMACH = 1e-8) need it.
#include <hipcub/hipcub.hpp>

#include <cstdlib>
#include <unordered_map>

#include "mstep_common.h"

namespace igm {
namespace ms {

constexpr uint32_t kLowerBit = 0x80000000u;
// nnb value of an atom with more list candidates than the capacity: its pair
// forces are taken by walking the 27 cells of the build-time grid, which
// visits a superset of its list in the same order (so no overflow error).
constexpr int kNnbWalk = 0xFFFF;
constexpr int kMaxTypes = 2048;  // distinct radii (LAMMPS atom types); the pair table is kMaxTypes^2

struct Bonds {
    const int4* ent;     // all structures' SELL entries
    const int64_t* base; // (B) entry offset of structure s
    const int* soff;     // (B, nslice+1) slice offsets (entries)
    const int* deg;      // (B, natom)
};

struct Common {
    int nstruct, natom, nslice, kcap;
    const float* radii;
    const int* atype;  // per atom: index into DevParams::pair_tab / rtype
    const uint32_t* aflags;
    Bonds bonds;
    int* work_counter;  // dynamic structure scheduler
    int* error;         // overflow flag (per launch)
};

// ------------------------------------------------------------------ LDS carve
// MD kernel (f32):  pos f4[npad] | frc f4[npad] | cell i32[kCellCap+4] | red 3x | wsum | misc |
//                   nnb u16[npad] | sorted u16[npad] | slot u16[npad] | cellid u16[npad]
// CG kernel (f64):  pos d4[npad] | ... same tail, forces live in HBM scratch.
template <typename T>
struct Smem {
    vec4_t<T>* pos;
    float4* frc;      // MD only
    int* cell;        // kCellCap + 4
    double* red0;     // kMaxWaves*8
    double* red1;
    double* redb;
    int* wsum;        // kMaxWaves
    int* misc;        // 16 ints
    uint16_t* nnb;    // npad
    uint16_t* sorted; // npad
    uint16_t* slot;   // npad
    uint16_t* cellid; // npad
};

template <typename T>
__host__ __device__ inline size_t smem_bytes(int npad) {
    size_t b = sizeof(vec4_t<T>) * (size_t)npad;
    if (sizeof(T) == 4) b += sizeof(float4) * (size_t)npad;
    b += sizeof(int) * (kCellCap + 4);
    b += 3 * sizeof(double) * kMaxWaves * 8;
    b += sizeof(int) * (kMaxWaves + 16);
    b += 4 * ((sizeof(uint16_t) * (size_t)npad + 15) / 16) * 16;
    return b;
}

template <typename T>
__device__ inline Smem<T> carve(unsigned char* smem, int npad) {
    Smem<T> s;
    size_t o = 0;
    s.pos = reinterpret_cast<vec4_t<T>*>(smem + o);
    o += sizeof(vec4_t<T>) * (size_t)npad;
    s.frc = nullptr;
    if (sizeof(T) == 4) {
        s.frc = reinterpret_cast<float4*>(smem + o);
        o += sizeof(float4) * (size_t)npad;
    }
    s.red0 = reinterpret_cast<double*>(smem + o);
    o += sizeof(double) * kMaxWaves * 8;
    s.red1 = reinterpret_cast<double*>(smem + o);
    o += sizeof(double) * kMaxWaves * 8;
    s.redb = reinterpret_cast<double*>(smem + o);
    o += sizeof(double) * kMaxWaves * 8;
    s.cell = reinterpret_cast<int*>(smem + o);
    o += sizeof(int) * (kCellCap + 4);
    s.wsum = reinterpret_cast<int*>(smem + o);
    o += sizeof(int) * kMaxWaves;
    s.misc = reinterpret_cast<int*>(smem + o);
    o += sizeof(int) * 16;
    const size_t u16b = ((sizeof(uint16_t) * (size_t)npad + 15) / 16) * 16;
    s.nnb = reinterpret_cast<uint16_t*>(smem + o);
    o += u16b;
    s.sorted = reinterpret_cast<uint16_t*>(smem + o);
    o += u16b;
    s.slot = reinterpret_cast<uint16_t*>(smem + o);
    o += u16b;
    s.cellid = reinterpret_cast<uint16_t*>(smem + o);
    return s;
}

// --------------------------------------------------------- neighbour build
template <int NT>
__device__ __forceinline__ void block_exclusive_scan(int* a, int n, int* wsum) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int cpt = (n + NT - 1) / NT;
    const int beg = t * cpt;
    int s = 0;
    for (int i = 0; i < cpt; ++i) {
        const int idx = beg + i;
        if (idx < n) {
            const int v = a[idx];
            a[idx] = s;
            s += v;
        }
    }
    int incl = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int woff = 0, total = 0;
    for (int i = 0; i < NT / 64; ++i) {
        if (i < w) woff += wsum[i];
        total += wsum[i];
    }
    const int toff = woff + incl - s;
    for (int i = 0; i < cpt; ++i) {
        const int idx = beg + i;
        if (idx < n) a[idx] += toff;
    }
    if (t == 0) a[n] = total;
    __syncthreads();
}

// Verlet list with skin from an LDS cell grid.  Positions are read from sm.pos
// (all writers have passed a barrier).  The bead mask is pos.w >= 0.
template <typename T, int NT, int BPT>
__device__ __noinline__ void build_nlist(int natom, Smem<T> sm, uint16_t* nbr, int kcap, T cut_list, int* error) {
    const int t = threadIdx.x;
    const int lane = t & 63;
    float mm[6];
#pragma unroll
    for (int d = 0; d < 6; ++d) mm[d] = -3.0e38f;
    for (int b = 0; b < BPT; ++b) {
        const int a = b * NT + t;
        if (a >= natom) break;
        const vec4_t<T> p = sm.pos[a];
        if (!(p.w >= T(0))) continue;
        mm[0] = fmaxf(mm[0], -(float)p.x);
        mm[1] = fmaxf(mm[1], -(float)p.y);
        mm[2] = fmaxf(mm[2], -(float)p.z);
        mm[3] = fmaxf(mm[3], (float)p.x);
        mm[4] = fmaxf(mm[4], (float)p.y);
        mm[5] = fmaxf(mm[5], (float)p.z);
    }
    {
        double md[6];
#pragma unroll
        for (int d = 0; d < 6; ++d) md[d] = mm[d];
        block_max<NT, 6>(md, sm.redb);
#pragma unroll
        for (int d = 0; d < 6; ++d) mm[d] = (float)md[d];
    }
    // grid (identical in every thread): cells of side >= cut_list, at most kCellCap
    T lo[3], inv[3];
    int nb[3];
    {
        float ext[3], vol = 1.0f;
        const float cut = (float)cut_list;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            // bounding box with a 1 ulp-safe margin (f32 min/max of f64 positions)
            ext[d] = mm[3 + d] + mm[d];
            if (!(ext[d] >= 0.0f)) ext[d] = 0.0f;
            vol *= fmaxf(ext[d], cut);
        }
        float cs = cut;
        if (vol / (cs * cs * cs) > (float)kCellCap) cs = cbrtf(vol / (float)kCellCap) * 1.0001f;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = (T)(-mm[d]);
            nb[d] = (int)floorf(ext[d] / cs);
            if (nb[d] < 1) nb[d] = 1;
            inv[d] = ext[d] > 0.0f ? (T)((float)nb[d] / ext[d]) : T(0);
        }
    }
    const int ncell = nb[0] * nb[1] * nb[2];
    if (t == 0) {  // for the cell walk of atoms past the list capacity (before the barrier below)
        sm.misc[4] = nb[0];
        sm.misc[5] = nb[1];
        sm.misc[6] = nb[2];
    }
    for (int c = t; c <= ncell; c += NT) sm.cell[c] = 0;
    __syncthreads();
    for (int b = 0; b < BPT; ++b) {
        const int a = b * NT + t;
        if (a >= natom) break;
        const vec4_t<T> p = sm.pos[a];
        if (!(p.w >= T(0))) continue;
        const T pp[3] = {p.x, p.y, p.z};
        int ci[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const int v = (int)((pp[d] - lo[d]) * inv[d]);
            ci[d] = v < 0 ? 0 : (v >= nb[d] ? nb[d] - 1 : v);
        }
        const int c = (ci[2] * nb[1] + ci[1]) * nb[0] + ci[0];
        sm.cellid[a] = (uint16_t)c;
        sm.slot[a] = (uint16_t)atomicAdd(&sm.cell[c], 1);
    }
    __syncthreads();
    block_exclusive_scan<NT>(sm.cell, ncell, sm.wsum);
    for (int b = 0; b < BPT; ++b) {
        const int a = b * NT + t;
        if (a >= natom) break;
        if (!(sm.pos[a].w >= T(0))) continue;
        sm.sorted[sm.cell[sm.cellid[a]] + sm.slot[a]] = (uint16_t)a;
    }
    __syncthreads();
    for (int c = t; c < ncell; c += NT) {  // deterministic order inside each cell
        const int beg = sm.cell[c], end = sm.cell[c + 1];
        for (int i = beg + 1; i < end; ++i) {
            const uint16_t v = sm.sorted[i];
            int k = i - 1;
            while (k >= beg && sm.sorted[k] > v) {
                sm.sorted[k + 1] = sm.sorted[k];
                --k;
            }
            sm.sorted[k + 1] = v;
        }
    }
    __syncthreads();
    (void)error;
    const T cut2 = cut_list * cut_list;
    for (int b = 0; b < BPT; ++b) {
        const int a = b * NT + t;
        if (a >= natom) break;
        const vec4_t<T> p0 = sm.pos[a];
        int cnt = 0;
        if (p0.w >= T(0)) {
            uint16_t* out = nbr + (size_t)(a >> 6) * kcap * 64 + lane;
            const int c = sm.cellid[a];
            const int cx = c % nb[0], cy = (c / nb[0]) % nb[1], cz = c / (nb[0] * nb[1]);
            for (int dz = -1; dz <= 1; ++dz) {
                const int z0 = cz + dz;
                if (z0 < 0 || z0 >= nb[2]) continue;
                for (int dy = -1; dy <= 1; ++dy) {
                    const int y0 = cy + dy;
                    if (y0 < 0 || y0 >= nb[1]) continue;
                    const int row = (z0 * nb[1] + y0) * nb[0];
                    const int xlo = cx > 0 ? cx - 1 : 0, xhi = cx + 1 < nb[0] ? cx + 1 : nb[0] - 1;
                    const int beg = sm.cell[row + xlo], end = sm.cell[row + xhi + 1];  // contiguous x-run
                    for (int q = beg; q < end; ++q) {
                        const int j = sm.sorted[q];
                        if (j == a) continue;
                        const vec4_t<T> p = sm.pos[j];
                        const T ddx = p0.x - p.x, ddy = p0.y - p.y, ddz = p0.z - p.z;
                        if (ddx * ddx + ddy * ddy + ddz * ddz < cut2) {
                            if (cnt < kcap) out[(size_t)cnt * 64] = (uint16_t)j;
                            ++cnt;
                        }
                    }
                }
            }
            if (cnt > kcap) cnt = kNnbWalk;  // the force routine walks the cells instead
        }
        sm.nnb[a] = (uint16_t)cnt;
    }
}

// ------------------------------------------------------------- forces
// force (and energy if EN) on atom a; position p0 (w: f32 radius / f64 atom type, <0: no pair)
template <typename T, bool EN>
__device__ __forceinline__ void pair_one(int j, T xi, T yi, T zi, T ri, const vec4_t<T>* pos, const DevParams& P,
                                         T evf, T& fx, T& fy, T& fz, double& ep) {
    const vec4_t<T> p = pos[j];
    const T dx = xi - p.x, dy = yi - p.y, dz = zi - p.z;
    double e = 0.0;
    T fp;
    if constexpr (std::is_same<T, float>::value) {
        fp = soft_pair<T, EN>(dx * dx + dy * dy + dz * dz, ri + (T)p.w, evf, e);
    } else {
        const double2 pc = P.pair_tab[(int)ri * P.ntype + (int)p.w];
        fp = soft_pair_typed(dx * dx + dy * dy + dz * dz, pc.x, pc.y, evf, e);
    }
    fx += fp * dx;
    fy += fp * dy;
    fz += fp * dz;
    if (EN) ep += 0.5 * e;
}

// the build-time cell grid (LDS), used for atoms past the list capacity
struct CellGrid {
    const int* cell;
    const uint16_t* sorted;
    const uint16_t* cellid;
    const int* dims;  // sm.misc + 4
};

template <typename T, bool EN>
__device__ __noinline__ void pair_walk(int a, T xi, T yi, T zi, T ri, const vec4_t<T>* pos, CellGrid g,
                                       const DevParams& P, T evf, T* f, double* ep) {
    const int nx = g.dims[0], ny = g.dims[1], nz = g.dims[2];
    const int c = g.cellid[a];
    const int cx = c % nx, cy = (c / nx) % ny, cz = c / (nx * ny);
    T fx = f[0], fy = f[1], fz = f[2];
    double e = *ep;
    for (int dz = -1; dz <= 1; ++dz) {
        const int z0 = cz + dz;
        if (z0 < 0 || z0 >= nz) continue;
        for (int dy = -1; dy <= 1; ++dy) {
            const int y0 = cy + dy;
            if (y0 < 0 || y0 >= ny) continue;
            const int row = (z0 * ny + y0) * nx;
            const int xlo = cx > 0 ? cx - 1 : 0, xhi = cx + 1 < nx ? cx + 1 : nx - 1;
            const int beg = g.cell[row + xlo], end = g.cell[row + xhi + 1];
            for (int q = beg; q < end; ++q) {
                const int j = g.sorted[q];
                if (j != a) pair_one<T, EN>(j, xi, yi, zi, ri, pos, P, evf, fx, fy, fz, e);
            }
        }
    }
    f[0] = fx;
    f[1] = fy;
    f[2] = fz;
    *ep = e;
}

template <typename T, bool EN>
__device__ __forceinline__ void atom_force(int a, const vec4_t<T>& p0, uint32_t fl, const vec4_t<T>* pos,
                                           const uint16_t* nl, int nn, const int4* al, int nd, const DevParams& P,
                                           CellGrid grid, T evf, T envf, T& fx, T& fy, T& fz, double& ep,
                                           double& eb, double (&ee)[IGM_MAX_ENVELOPES]) {
    fx = fy = fz = T(0);
    const T xi = p0.x, yi = p0.y, zi = p0.z;
    const T ri = (T)p0.w;
    constexpr int U = 8;  // neighbour indices fetched per batch: one memory wait per U pairs
    if (ri >= T(0) && nn == kNnbWalk) {
        T f3[3] = {T(0), T(0), T(0)};
        double e = 0.0;
        pair_walk<T, EN>(a, xi, yi, zi, ri, pos, grid, P, evf, f3, &e);
        fx = f3[0];
        fy = f3[1];
        fz = f3[2];
        if (EN) ep += e;
    } else if (ri >= T(0)) {
        for (int k0 = 0; k0 < nn; k0 += U) {
            int jv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) jv[u] = (k0 + u < nn) ? (int)nl[(size_t)(k0 + u) * 64] : -1;
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (jv[u] >= 0) pair_one<T, EN>(jv[u], xi, yi, zi, ri, pos, P, evf, fx, fy, fz, ep);
        }
    }
    constexpr int UB = 4;  // bond entries (16 B) per batch
    for (int k0 = 0; k0 < nd; k0 += UB) {
        int4 ev[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) ev[u] = (k0 + u < nd) ? al[(size_t)(k0 + u) * 64] : make_int4(-1, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            if (k0 + u >= nd) continue;
            const uint32_t jj = (uint32_t)ev[u].x;
            const vec4_t<T> p = pos[jj & 0x7fffffffu];
            const T dx = xi - p.x, dy = yi - p.y, dz = zi - p.z;
            double e = 0.0;
            const T fb = bond_term<T, EN>(dx * dx + dy * dy + dz * dz, (T)__int_as_float(ev[u].y),
                                          (T)__int_as_float(ev[u].z), (jj & kLowerBit) != 0u, e);
            fx += fb * dx;
            fy += fb * dy;
            fz += fb * dz;
            if (EN) eb += 0.5 * e;
        }
    }
    // non-bead atoms carry -(w + 1); f32: w = radius, f64: w = atom type
    T rad;
    if constexpr (std::is_same<T, float>::value)
        rad = ri >= T(0) ? ri : -ri - T(1);
    else
        rad = P.rtype[ri >= T(0) ? (int)ri : (int)(-ri - T(1))];
    for (int e = 0; e < P.nenv; ++e) {
        if (!(fl & (IGM_ATOM_ENV0 << e))) continue;
        double en = 0.0;
        if constexpr (std::is_same<T, float>::value)
            envelope_term<T, EN>(xi, yi, zi, rad, P.env_abc[e][0] * envf, P.env_abc[e][1] * envf,
                                 P.env_abc[e][2] * envf, P.env_k[e], fx, fy, fz, en);
        else
            envelope_term<T, EN>(xi, yi, zi, rad, P.env_abc_d[e][0] * envf, P.env_abc_d[e][1] * envf,
                                 P.env_abc_d[e][2] * envf, P.env_k_d[e], fx, fy, fz, en);
        if (EN) ee[e] += en;
    }
    if (fl & IGM_ATOM_FIXED) fx = fy = fz = T(0);  // fix setforce 0 (lammps.py:222-223)
}

// ------------------------------------------------------------- anneal
struct AnnealArgs {
    Common cm;
    DevParams P;
    float* xyz;          // (B, natom, 3)
    float* vel;          // (B, natom, 3): out (mode 0) / in-out (mode 1)
    const float* vinit;  // mode 0: (B, nseg, natom, 3) velocities of each 'velocity create'
    uint16_t* nbr_ws;    // per resident workgroup
    size_t nbr_stride;
    int* nrebuild;       // (B)
    float* forces_out;   // forces at the end (B, natom, 3), may be null
    int mode;            // 0: full protocol, 1: one MD segment from vel
    int nseg;
    // per segment (mode 0) or the single segment (mode 1)
    int seg_steps[2 * IGM_MAX_STAGES];
    float seg_evf[2 * IGM_MAX_STAGES], seg_envf[2 * IGM_MAX_STAGES], seg_t0[2 * IGM_MAX_STAGES],
        seg_t1[2 * IGM_MAX_STAGES], seg_xmax[2 * IGM_MAX_STAGES];
    float dt, t_window, t_fraction;
};

template <int NT, int BPT>
__global__ void __launch_bounds__(NT) anneal_kernel(AnnealArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int npad = NT * BPT;
    Smem<float> sm = carve<float>(smem, npad);
    const int t = threadIdx.x, lane = t & 63;
    const int natom = A.cm.natom;
    uint16_t* nbr = A.nbr_ws + (size_t)blockIdx.x * A.nbr_stride;
    float v[BPT][3], xb[BPT][3];
    for (;;) {
        if (t == 0) sm.misc[0] = atomicAdd(A.cm.work_counter, 1);
        __syncthreads();
        const int s = sm.misc[0];
        __syncthreads();
        if (s >= A.cm.nstruct) break;
        const float* xs = A.xyz + (size_t)s * natom * 3;
        uint32_t mobile = 0u;  // bit b: atom b*NT+t is integrated
        int nmob = 0;
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const int a = b * NT + t;
            const bool in = a < natom;
            const uint32_t fl = in ? A.cm.aflags[a] : 0u;
            const bool bead = in && (fl & IGM_ATOM_BEAD);
            if (in && !(fl & IGM_ATOM_FIXED)) {
                mobile |= 1u << b;
                ++nmob;
            }
            const float r = in ? A.cm.radii[a] : 0.0f;
            sm.pos[a] = make_float4(in ? xs[(size_t)a * 3] : 0.f, in ? xs[(size_t)a * 3 + 1] : 0.f,
                                    in ? xs[(size_t)a * 3 + 2] : 0.f, bead ? r : -(r + 1.0f));
            sm.frc[a] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                v[b][d] = 0.0f;
                xb[b][d] = __int_as_float(0x7f800000);  // +inf: forces the first neighbour build
            }
        }
        double cnt[1] = {(double)nmob};
        block_sum<NT, 1>(cnt, sm.red0);
        const double dof = 3.0 * cnt[0] - 3.0;  // compute temp of group nonfixed
        __syncthreads();
        const int4* adj = A.cm.bonds.ent + A.cm.bonds.base[s];
        const int* soff = A.cm.bonds.soff + (size_t)s * (A.cm.nslice + 1);
        const int* deg = A.cm.bonds.deg + (size_t)s * natom;
        int nbuild = 0;
        for (int seg = 0; seg < A.nseg; ++seg) {
            const float* vsrc = A.mode == 1 ? A.vel + (size_t)s * natom * 3
                                            : A.vinit + ((size_t)s * A.nseg + seg) * natom * 3;
#pragma unroll
            for (int b = 0; b < BPT; ++b) {
                const int a = b * NT + t;
#pragma unroll
                for (int d = 0; d < 3; ++d) v[b][d] = (mobile >> b & 1u) ? vsrc[(size_t)a * 3 + d] : 0.0f;
            }
            const int nsteps = A.seg_steps[seg];
            const float evf = A.seg_evf[seg], envf = A.seg_envf[seg];
            const float t0 = A.seg_t0[seg], t1 = A.seg_t1[seg];
            const float dtv = A.dt, dtf = 0.5f * A.dt;
            const float vlim = A.seg_xmax[seg] / dtv;
            const float vlimsq = vlim * vlim;
            const float trig = 0.25f * A.P.skin * A.P.skin;
            // ---- run nsteps: step 0 is Verlet::setup (forces only)
            for (int step = 0; step <= nsteps; ++step) {
                int moved = 0;
#pragma unroll
                for (int b = 0; b < BPT; ++b) {
                    const int a = b * NT + t;
                    float4 p = sm.pos[a];
                    if (step > 0 && (mobile >> b & 1u)) {  // fix nve/limit: initial_integrate
                        const float4 fo = sm.frc[a];
                        v[b][0] += dtf * fo.x;
                        v[b][1] += dtf * fo.y;
                        v[b][2] += dtf * fo.z;
                        const float vsq = v[b][0] * v[b][0] + v[b][1] * v[b][1] + v[b][2] * v[b][2];
                        if (vsq > vlimsq) {
                            const float sc = vlim * __frsqrt_rn(vsq);
#pragma unroll
                            for (int d = 0; d < 3; ++d) v[b][d] *= sc;
                        }
                        p.x += dtv * v[b][0];
                        p.y += dtv * v[b][1];
                        p.z += dtv * v[b][2];
                        sm.pos[a] = p;
                    }
                    if (p.w >= 0.0f) {
                        const float ddx = p.x - xb[b][0], ddy = p.y - xb[b][1], ddz = p.z - xb[b][2];
                        moved |= !(ddx * ddx + ddy * ddy + ddz * ddz <= trig);
                    }
                }
                if (__syncthreads_or(moved)) {  // neigh_modify every 1 check yes
                    build_nlist<float, NT, BPT>(natom, sm, nbr, A.cm.kcap, A.P.cut_list, A.cm.error);
                    ++nbuild;
#pragma unroll
                    for (int b = 0; b < BPT; ++b) {
                        const float4 p = sm.pos[b * NT + t];
                        xb[b][0] = p.x;
                        xb[b][1] = p.y;
                        xb[b][2] = p.z;
                    }
                }
                // forces: the owner thread gathers every contribution of its atoms
                for (int b = 0; b < BPT; ++b) {
                    const int a = b * NT + t;
                    if (a >= natom) break;
                    double ep = 0, eb = 0, ee[IGM_MAX_ENVELOPES] = {0, 0, 0, 0};
                    float fx, fy, fz;
                    atom_force<float, false>(a, sm.pos[a], A.cm.aflags[a], sm.pos,
                                             nbr + (size_t)(a >> 6) * A.cm.kcap * 64 + lane, sm.nnb[a],
                                             adj + soff[a >> 6] + lane, deg[a], A.P,
                                             CellGrid{sm.cell, sm.sorted, sm.cellid, sm.misc + 4}, evf, envf, fx,
                                             fy, fz, ep, eb,
                                             ee);
                    sm.frc[a] = make_float4(fx, fy, fz, 0.f);
                }
                if (step == 0) {
                    __syncthreads();  // setup forces read sm.pos: no update before every wave is done
                    continue;
                }
                double ts[1] = {0.0};
#pragma unroll
                for (int b = 0; b < BPT; ++b) {  // final_integrate
                    if (!(mobile >> b & 1u)) continue;
                    const float4 fo = sm.frc[b * NT + t];
                    v[b][0] += dtf * fo.x;
                    v[b][1] += dtf * fo.y;
                    v[b][2] += dtf * fo.z;
                    const float vsq = v[b][0] * v[b][0] + v[b][1] * v[b][1] + v[b][2] * v[b][2];
                    if (vsq > vlimsq) {
                        const float sc = vlim * __frsqrt_rn(vsq);
#pragma unroll
                        for (int d = 0; d < 3; ++d) v[b][d] *= sc;
                    }
#pragma unroll
                    for (int d = 0; d < 3; ++d) ts[0] += (double)(v[b][d] * v[b][d]);
                }
                block_sum<NT, 1>(ts, (step & 1) ? sm.red1 : sm.red0);
                // fix temp/rescale 1 t0 t1 window fraction: end_of_step
                const double tcur = dof > 0 ? ts[0] / dof : 0.0;
                if (tcur > 0.0) {
                    const double delta = (double)step / (double)nsteps;
                    double tt = (double)t0 + delta * ((double)t1 - (double)t0);
                    if (fabs(tcur - tt) > (double)A.t_window) {
                        tt = tcur - (double)A.t_fraction * (tcur - tt);
                        const float factor = (float)sqrt(tt / tcur);
#pragma unroll
                        for (int b = 0; b < BPT; ++b)
#pragma unroll
                            for (int d = 0; d < 3; ++d) v[b][d] *= factor;
                    }
                }
            }
        }
        __syncthreads();
        float* xo = A.xyz + (size_t)s * natom * 3;
        float* vo = A.vel + (size_t)s * natom * 3;
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const int a = b * NT + t;
            if (a >= natom) continue;
            const float4 p = sm.pos[a];
            const float4 fo = sm.frc[a];
            xo[(size_t)a * 3] = p.x;
            xo[(size_t)a * 3 + 1] = p.y;
            xo[(size_t)a * 3 + 2] = p.z;
#pragma unroll
            for (int d = 0; d < 3; ++d) vo[(size_t)a * 3 + d] = v[b][d];
            if (A.forces_out) {
                float* fo3 = A.forces_out + ((size_t)s * natom + a) * 3;
                fo3[0] = fo.x;
                fo3[1] = fo.y;
                fo3[2] = fo.z;
            }
        }
        if (t == 0 && A.nrebuild) A.nrebuild[s] = nbuild;
        __syncthreads();
    }
}

// 'velocity nonfixed create T seed' (dist uniform, loop all, mom yes) for every
// structure and segment: RanPark draws in atom-id order, momentum zeroed, scaled
// to T with the group's dof.  grid (nseg, B), one workgroup each.
struct VelArgs {
    int nstruct, natom, nseg;
    const uint32_t* aflags;
    const int* seeds;              // (B) stage-0 seed
    int seg_stage[2 * IGM_MAX_STAGES];
    float seg_temp[2 * IGM_MAX_STAGES];
    float* vinit;                  // (B, nseg, natom, 3)
};

__global__ void __launch_bounds__(256) velocity_kernel(VelArgs V) {
    __shared__ double red[4 * 8 * 4];
    const int seg = blockIdx.x, s = blockIdx.y, t = threadIdx.x;
    const uint32_t seed = (uint32_t)(V.seeds[s] + V.seg_stage[seg]);
    float* out = V.vinit + ((size_t)s * V.nseg + seg) * V.natom * 3;
    double s4[4] = {0, 0, 0, 0};
    for (int a = t; a < V.natom; a += 256) {
        if (V.aflags[a] & IGM_ATOM_FIXED) continue;
#pragma unroll
        for (int d = 0; d < 3; ++d) s4[d] += ranpark_nth(seed, 3ull * a + d + 1) - 0.5;
        s4[3] += 1.0;
    }
    block_sum<256, 4>(s4, red);
    __syncthreads();
    const double nmob = s4[3];
    double t2[1] = {0.0};
    for (int a = t; a < V.natom; a += 256) {
        if (V.aflags[a] & IGM_ATOM_FIXED) continue;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const double vd = (ranpark_nth(seed, 3ull * a + d + 1) - 0.5) - s4[d] / nmob;
            t2[0] += vd * vd;
        }
    }
    block_sum<256, 1>(t2, red + 64);
    const double dof = 3.0 * nmob - 3.0;
    const double tc = dof > 0 ? t2[0] / dof : 0.0;
    const double factor = tc > 0.0 ? sqrt((double)V.seg_temp[seg] / tc) : 0.0;
    for (int a = t; a < V.natom; a += 256) {
        const bool fixed = V.aflags[a] & IGM_ATOM_FIXED;
#pragma unroll
        for (int d = 0; d < 3; ++d)
            out[(size_t)a * 3 + d] =
                fixed ? 0.0f : (float)(((ranpark_nth(seed, 3ull * a + d + 1) - 0.5) - s4[d] / nmob) * factor);
    }
}

// ------------------------------------------------------------- CG (f64)
struct CGArgs {
    Common cm;
    DevParams P;
    float* xyz;          // (B, natom, 3) in/out
    const float* vel;    // (B, natom, 3) velocities after MD (thermo Temp), may be null
    uint16_t* nbr_ws;
    size_t nbr_stride;
    double* vec_ws;      // per resident workgroup: F, X0, G, H as [4][3][npad] doubles
    size_t vec_stride;
    igm_opt_info* info;  // (B)
    const int* nrebuild_md;
    double evf, envf, etol, ftol, dmax;
    int max_iter, max_eval;
    int mode;            // 0: minimize, 1: energy/forces only
    float* forces_out;   // (B, natom, 3) or null
    double* energies_out;// (B, 3 + IGM_MAX_ENVELOPES) or null
};

enum { MAXITER = 1, MAXEVAL, ETOL, FTOL, DOWNHILL, ZEROALPHA, ZEROFORCE, ZEROQUAD };
// phases of the flattened MinCG::iterate + MinLineSearch::linemin_quadratic
enum { PH_SETUP, PH_BT, PH_QUAD, PH_RET_ZEROQUAD, PH_RET_ZEROALPHA };

template <int NT, int BPT>
__global__ void __launch_bounds__(NT) cg_kernel(CGArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int npad = NT * BPT;
    Smem<double> sm = carve<double>(smem, npad);
    const int t = threadIdx.x, lane = t & 63;
    const int natom = A.cm.natom;
    uint16_t* nbr = A.nbr_ws + (size_t)blockIdx.x * A.nbr_stride;
    double* F = A.vec_ws + (size_t)blockIdx.x * A.vec_stride;
    double* X0 = F + 3 * (size_t)npad;
    double* G = X0 + 3 * (size_t)npad;
    double* H = G + 3 * (size_t)npad;
    double xb[BPT][3];
    const double ALPHA_MAX = 1.0, ALPHA_REDUCE = 0.5, BACKTRACK_SLOPE = 0.4, QUADRATIC_TOL = 0.1, EMACH = 1.0e-8,
                 EPS_QUAD = 1.0e-28;
    for (;;) {
        if (t == 0) sm.misc[0] = atomicAdd(A.cm.work_counter, 1);
        __syncthreads();
        const int s = sm.misc[0];
        __syncthreads();
        if (s >= A.cm.nstruct) break;
        const float* xs = A.xyz + (size_t)s * natom * 3;
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const int a = b * NT + t;
            const bool in = a < natom;
            const uint32_t fl = in ? A.cm.aflags[a] : 0u;
            const double r = in ? (double)A.cm.atype[a] : 0.0;
            sm.pos[a] = make_double4(in ? (double)xs[(size_t)a * 3] : 0.0, in ? (double)xs[(size_t)a * 3 + 1] : 0.0,
                                     in ? (double)xs[(size_t)a * 3 + 2] : 0.0,
                                     (in && (fl & IGM_ATOM_BEAD)) ? r : -(r + 1.0));
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                xb[b][d] = __longlong_as_double(0x7ff0000000000000LL);
                F[d * npad + a] = 0.0;
            }
        }
        __syncthreads();
        const int4* adj = A.cm.bonds.ent + A.cm.bonds.base[s];
        const int* soff = A.cm.bonds.soff + (size_t)s * (A.cm.nslice + 1);
        const int* deg = A.cm.bonds.deg + (size_t)s * natom;
        const double trig = 0.25 * (double)A.P.skin * (double)A.P.skin;
        int neval = 0, nbuild = 0, niter = 0, stop = MAXITER;
        double ecurrent = 0, einitial = 0, eoriginal = 0, eprevious = 0;
        double ep = 0, eb = 0, ee[IGM_MAX_ENVELOPES] = {0, 0, 0, 0};
        double alpha = 0, alphamax = 0, alpha0 = 0, alphaprev = 0, engprev = 0, fhprev = 0, fdothall = 0, ggv = 0;
        int phase = PH_SETUP;
        double a_eval = -1.0;  // < 0: evaluate at x as is (setup)
        for (;;) {
            // ---------- the single energy/force evaluation site
            int moved = 0;
#pragma unroll
            for (int b = 0; b < BPT; ++b) {
                const int a = b * NT + t;
                double4 p = sm.pos[a];
                if (a_eval >= 0.0 && a < natom) {  // alpha_step: x = x0 + alpha h
                    p.x = X0[a] + (a_eval > 0.0 ? a_eval * H[a] : 0.0);
                    p.y = X0[npad + a] + (a_eval > 0.0 ? a_eval * H[npad + a] : 0.0);
                    p.z = X0[2 * npad + a] + (a_eval > 0.0 ? a_eval * H[2 * npad + a] : 0.0);
                    sm.pos[a] = p;
                }
                if (p.w >= 0.0) {
                    const double dx = p.x - xb[b][0], dy = p.y - xb[b][1], dz = p.z - xb[b][2];
                    moved |= !(dx * dx + dy * dy + dz * dz <= trig);
                }
            }
            if (a_eval >= 0.0) ++neval;
            if (__syncthreads_or(moved)) {
                build_nlist<double, NT, BPT>(natom, sm, nbr, A.cm.kcap, (double)A.P.cut_list, A.cm.error);
                ++nbuild;
#pragma unroll
                for (int b = 0; b < BPT; ++b) {
                    const double4 p = sm.pos[b * NT + t];
                    xb[b][0] = p.x;
                    xb[b][1] = p.y;
                    xb[b][2] = p.z;
                }
            }
            double vv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int b = 0; b < BPT; ++b) {
                const int a = b * NT + t;
                if (a >= natom) break;
                double e_e[IGM_MAX_ENVELOPES] = {0, 0, 0, 0};
                double fx, fy, fz;
                atom_force<double, true>(a, sm.pos[a], A.cm.aflags[a], sm.pos,
                                         nbr + (size_t)(a >> 6) * A.cm.kcap * 64 + lane, sm.nnb[a],
                                         adj + soff[a >> 6] + lane, deg[a], A.P,
                                         CellGrid{sm.cell, sm.sorted, sm.cellid, sm.misc + 4}, A.evf, A.envf, fx,
                                         fy, fz, vv[0],
                                         vv[1], e_e);
                for (int e = 0; e < IGM_MAX_ENVELOPES; ++e) vv[2 + e] += e_e[e];
                F[a] = fx;
                F[npad + a] = fy;
                F[2 * npad + a] = fz;
                vv[6] += fx * fx + fy * fy + fz * fz;
                if (phase != PH_SETUP) vv[7] += fx * H[a] + fy * H[npad + a] + fz * H[2 * npad + a];
            }
            block_sum<NT, 8>(vv, sm.red0);
            __syncthreads();
            ep = vv[0];
            eb = vv[1];
            for (int e = 0; e < IGM_MAX_ENVELOPES; ++e) ee[e] = vv[2 + e];
            ecurrent = vv[0] + vv[1] + vv[2] + vv[3] + vv[4] + vv[5];
            const double ff = vv[6], fh = vv[7];
            // ---------- what the evaluation was for
            bool linemin_done = false;  // linemin_quadratic returned 0
            int fail = 0;
            bool start_iter = false;
            if (phase == PH_SETUP) {  // Min::setup, then the MinCG::iterate prologue
                einitial = ecurrent;
                if (A.mode == 1) break;
                for (int b = 0; b < BPT; ++b) {
                    const int a = b * NT + t;
                    if (a >= natom) break;
#pragma unroll
                    for (int d = 0; d < 3; ++d) G[d * npad + a] = H[d * npad + a] = F[d * npad + a];
                }
                ggv = ff;
                start_iter = true;
            } else if (phase == PH_RET_ZEROQUAD) {
                fail = ZEROQUAD;
            } else if (phase == PH_RET_ZEROALPHA) {
                fail = ZEROALPHA;
            } else {
                bool de_check = false;
                if (phase == PH_BT) {
                    const double delfh = fh - fhprev;
                    if (fabs(fh) < EPS_QUAD || fabs(delfh) < EPS_QUAD) {
                        phase = PH_RET_ZEROQUAD;
                        a_eval = 0.0;
                        continue;
                    }
                    const double relerr = fabs(1.0 - (0.5 * (alpha - alphaprev) * (fh + fhprev) + ecurrent) / engprev);
                    alpha0 = alpha - (alpha - alphaprev) * fh / delfh;
                    fhprev = fh;  // LAMMPS saves it after the tests; fh of the quadratic eval is never used
                    if (relerr <= QUADRATIC_TOL && alpha0 > 0.0 && alpha0 < alphamax) {
                        phase = PH_QUAD;
                        a_eval = alpha0;
                        continue;
                    }
                    de_check = true;
                } else {  // PH_QUAD
                    if (ecurrent - eoriginal < EMACH)
                        linemin_done = true;
                    else
                        de_check = true;
                }
                if (de_check) {
                    const double de_ideal = -BACKTRACK_SLOPE * alpha * fdothall;
                    if (ecurrent - eoriginal <= de_ideal) {
                        linemin_done = true;
                    } else {
                        engprev = ecurrent;
                        alphaprev = alpha;
                        alpha *= ALPHA_REDUCE;
                        if (alpha <= 0.0 || de_ideal >= -EMACH) {
                            phase = PH_RET_ZEROALPHA;
                            a_eval = 0.0;
                            continue;
                        }
                        phase = PH_BT;
                        a_eval = alpha;
                        continue;
                    }
                }
            }
            if (fail) {
                stop = fail;
                break;
            }
            if (linemin_done) {  // the rest of one MinCG::iterate iteration
                if (neval >= A.max_eval) {
                    stop = MAXEVAL;
                    break;
                }
                if (fabs(ecurrent - eprevious) < A.etol * 0.5 * (fabs(ecurrent) + fabs(eprevious) + 1.0e-8)) {
                    stop = ETOL;
                    break;
                }
                if (A.ftol > 0.0 && ff < A.ftol * A.ftol) {
                    stop = FTOL;
                    break;
                }
                double dd[1] = {0.0};
                for (int b = 0; b < BPT; ++b) {
                    const int a = b * NT + t;
                    if (a >= natom) break;
#pragma unroll
                    for (int d = 0; d < 3; ++d) dd[0] += F[d * npad + a] * G[d * npad + a];
                }
                block_sum<NT, 1>(dd, sm.red1);
                __syncthreads();
                double beta = fmax(0.0, (ff - dd[0]) / ggv);
                if ((long)(niter + 1) % (3L * natom) == 0) beta = 0.0;
                ggv = ff;
                double gh[1] = {0.0};
                for (int b = 0; b < BPT; ++b) {
                    const int a = b * NT + t;
                    if (a >= natom) break;
#pragma unroll
                    for (int d = 0; d < 3; ++d) {
                        const double fv = F[d * npad + a];
                        const double hv = fv + beta * H[d * npad + a];
                        G[d * npad + a] = fv;
                        H[d * npad + a] = hv;
                        gh[0] += fv * hv;
                    }
                }
                block_sum<NT, 1>(gh, sm.red1);
                __syncthreads();
                if (gh[0] <= 0.0)
                    for (int b = 0; b < BPT; ++b) {
                        const int a = b * NT + t;
                        if (a >= natom) break;
#pragma unroll
                        for (int d = 0; d < 3; ++d) H[d * npad + a] = G[d * npad + a];
                    }
                start_iter = true;
            }
            if (!start_iter) break;  // unreachable
            // ---------- next CG iteration: linemin_quadratic prologue
            if (niter >= A.max_iter) {
                stop = MAXITER;
                break;
            }
            ++niter;
            eprevious = ecurrent;
            eoriginal = ecurrent;
            double pr[1] = {0.0}, hm[1] = {0.0};
            for (int b = 0; b < BPT; ++b) {
                const int a = b * NT + t;
                if (a >= natom) break;
                const double4 p = sm.pos[a];
                X0[a] = p.x;
                X0[npad + a] = p.y;
                X0[2 * npad + a] = p.z;
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    const double hv = H[d * npad + a];
                    pr[0] += F[d * npad + a] * hv;
                    hm[0] = fmax(hm[0], fabs(hv));
                }
            }
            block_sum<NT, 1>(pr, sm.red1);
            __syncthreads();
            block_max<NT, 1>(hm, sm.red0);
            __syncthreads();
            fdothall = pr[0];
            if (fdothall <= 0.0) {
                stop = DOWNHILL;
                break;
            }
            if (hm[0] == 0.0) {
                stop = ZEROFORCE;
                break;
            }
            alphamax = fmin(ALPHA_MAX, A.dmax / hm[0]);
            alpha = alphamax;
            engprev = eoriginal;
            alphaprev = 0.0;
            fhprev = fdothall;
            phase = PH_BT;
            a_eval = alpha;
        }
        // ---------- outputs
        double fn[2] = {0.0, 0.0};
        for (int b = 0; b < BPT; ++b) {
            const int a = b * NT + t;
            if (a >= natom) break;
#pragma unroll
            for (int d = 0; d < 3; ++d) fn[0] += F[d * npad + a] * F[d * npad + a];
            if (A.vel) {
                const float* vs = A.vel + ((size_t)s * natom + a) * 3;
#pragma unroll
                for (int d = 0; d < 3; ++d) fn[1] += (double)vs[d] * (double)vs[d];
            }
        }
        block_sum<NT, 2>(fn, sm.red1);
        float* xo = A.xyz + (size_t)s * natom * 3;
        for (int b = 0; b < BPT; ++b) {
            const int a = b * NT + t;
            if (a >= natom) break;
            const double4 p = sm.pos[a];
            if (A.mode == 0) {
                xo[(size_t)a * 3] = (float)p.x;
                xo[(size_t)a * 3 + 1] = (float)p.y;
                xo[(size_t)a * 3 + 2] = (float)p.z;
            }
            if (A.forces_out)
#pragma unroll
                for (int d = 0; d < 3; ++d) A.forces_out[((size_t)s * natom + a) * 3 + d] = (float)F[d * npad + a];
        }
        if (t == 0) {
            if (A.info) {
                igm_opt_info I;
                I.final_energy = ecurrent;
                I.pair_energy = ep;
                I.bond_energy = eb;
                for (int e = 0; e < IGM_MAX_ENVELOPES; ++e) I.env_energy[e] = ee[e];
                const double dof_all = 3.0 * natom - 3.0;  // thermo temp: group all
                I.temp = dof_all > 0 ? fn[1] / dof_all : 0.0;
                I.einitial = einitial;
                I.fnorm_final = sqrt(fn[0]);
                I.cg_iters = niter;
                I.cg_evals = neval;
                I.stop_reason = stop;
                I.nrebuild = nbuild + (A.nrebuild_md ? A.nrebuild_md[s] : 0);
                A.info[s] = I;
            }
            if (A.energies_out) {
                double* en = A.energies_out + (size_t)s * (3 + IGM_MAX_ENVELOPES);
                en[0] = ecurrent;
                en[1] = ep;
                en[2] = eb;
                for (int e = 0; e < IGM_MAX_ENVELOPES; ++e) en[3 + e] = ee[e];
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------- adjacency
__device__ __forceinline__ const igm_bond& bond_at(const igm_bond* shared, int64_t nshared, const igm_bond* own,
                                                   int64_t q) {
    return q < nshared ? shared[q] : own[q - nshared];
}

__global__ void adj_count_kernel(int nstruct, int natom, int nslice, const igm_bond* shared, int64_t nshared,
                                 const int64_t* sptr, const igm_bond* sbonds, int* deg, int* soff, int64_t* size,
                                 int* error) {
    extern __shared__ int cnt[];
    const int s = blockIdx.x;
    const int t = threadIdx.x;
    for (int a = t; a < nslice * 64; a += blockDim.x) cnt[a] = 0;
    __syncthreads();
    const int64_t b0 = sptr ? sptr[s] : 0, b1 = sptr ? sptr[s + 1] : 0;
    const igm_bond* own = sbonds ? sbonds + b0 : nullptr;
    const int64_t nb = nshared + (b1 - b0);
    for (int64_t q = t; q < nb; q += blockDim.x) {
        const igm_bond& bd = bond_at(shared, nshared, own, q);
        const uint32_t i = bd.i, j = bd.j & 0x7fffffffu;
        if (i >= (uint32_t)natom || j >= (uint32_t)natom) {
            atomicOr(error, 2);
            continue;
        }
        atomicAdd(&cnt[i], 1);
        atomicAdd(&cnt[j], 1);
    }
    __syncthreads();
    for (int a = t; a < natom; a += blockDim.x) deg[(size_t)s * natom + a] = cnt[a];
    __syncthreads();
    // per-slice max degree (thread per slice), stored back into cnt[slice*64]
    for (int sl = t; sl < nslice; sl += blockDim.x) {
        int m = 0;
        for (int l = 0; l < 64; ++l) m = max(m, cnt[sl * 64 + l]);
        cnt[sl * 64] = m;
    }
    __syncthreads();
    if (t == 0) {
        int acc = 0;
        int* so = soff + (size_t)s * (nslice + 1);
        for (int sl = 0; sl < nslice; ++sl) {
            so[sl] = acc;
            acc += cnt[sl * 64] * 64;
        }
        so[nslice] = acc;
        size[s] = acc;
    }
}

__global__ void adj_fill_kernel(int nstruct, int natom, int nslice, const igm_bond* shared, int64_t nshared,
                                const int64_t* sptr, const igm_bond* sbonds, const int* deg, const int* soff,
                                const int64_t* base, int4* ent) {
    extern __shared__ int fill[];
    const int s = blockIdx.x;
    const int t = threadIdx.x;
    for (int a = t; a < natom; a += blockDim.x) fill[a] = 0;
    __syncthreads();
    const int64_t b0 = sptr ? sptr[s] : 0, b1 = sptr ? sptr[s + 1] : 0;
    const igm_bond* own = sbonds ? sbonds + b0 : nullptr;
    const int64_t nb = nshared + (b1 - b0);
    const int* so = soff + (size_t)s * (nslice + 1);
    int4* E = ent + base[s];
    for (int64_t q = t; q < nb; q += blockDim.x) {
        const igm_bond& bd = bond_at(shared, nshared, own, q);
        const uint32_t i = bd.i, j = bd.j & 0x7fffffffu, low = bd.j & kLowerBit;
        if (i >= (uint32_t)natom || j >= (uint32_t)natom) continue;
        const int si = atomicAdd(&fill[i], 1);
        const int sj = atomicAdd(&fill[j], 1);
        E[so[i >> 6] + si * 64 + (i & 63)] = make_int4((int)(j | low), __float_as_int(bd.r0), __float_as_int(bd.k), 0);
        E[so[j >> 6] + sj * 64 + (j & 63)] = make_int4((int)(i | low), __float_as_int(bd.r0), __float_as_int(bd.k), 0);
    }
    __syncthreads();
    __threadfence_block();
    // fixed order per atom: sort entries by (partner|style, r0, k)
    for (int a = t; a < natom; a += blockDim.x) {
        const int n = deg[(size_t)s * natom + a];
        int4* L = E + so[a >> 6] + (a & 63);
        for (int i = 1; i < n; ++i) {
            const int4 v = L[(size_t)i * 64];
            int k = i - 1;
            while (k >= 0) {
                const int4 u = L[(size_t)k * 64];
                const bool gt = ((uint32_t)u.x > (uint32_t)v.x) ||
                                ((uint32_t)u.x == (uint32_t)v.x &&
                                 ((uint32_t)u.y > (uint32_t)v.y ||
                                  ((uint32_t)u.y == (uint32_t)v.y && (uint32_t)u.z > (uint32_t)v.z)));
                if (!gt) break;
                L[(size_t)(k + 1) * 64] = u;
                --k;
            }
            L[(size_t)(k + 1) * 64] = v;
        }
    }
}

}  // namespace ms
}  // namespace igm

// =================================================================== host side
using namespace igm;
using namespace igm::ms;

namespace {

struct Prepared {
    Common cm;
    DevParams P;
    int npad_needed;
    int64_t total_ent;
};

// The reference writes np.float32 values with Python's shortest round-trip repr
// (PairIJ cutoff and 'User' radius, lammps.py:128-146) and LAMMPS parses them as
// doubles: the shortest %.{p}g that reads back as the same float, read as double.
static double f32_as_printed(float f) {
    char buf[48];
    for (int p = 1; p <= 9; ++p) {
        snprintf(buf, sizeof(buf), "%.*g", p, (double)f);
        if (strtof(buf, nullptr) == f) return strtod(buf, nullptr);
    }
    return (double)f;
}

int make_devparams(igm_ctx* c, const igm_mstep_params* prm, int natom, const float* d_radii,
                   const uint32_t* d_flags, DevParams* P, const int** d_atype) {
    // host copies of radii/flags: max bead radius and the atom types
    std::vector<float> r(natom);
    std::vector<uint32_t> fl(natom);
    IGM_HIP_CHECK(c, hipMemcpyAsync(r.data(), d_radii, sizeof(float) * natom, hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipMemcpyAsync(fl.data(), d_flags, sizeof(uint32_t) * natom, hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    float rmax = 0.f;
    for (int i = 0; i < natom; ++i)
        if ((fl[i] & IGM_ATOM_BEAD) && r[i] > rmax) rmax = r[i];
    memset(P, 0, sizeof(*P));
    P->nenv = prm->nenvelopes;
    if (P->nenv < 0 || P->nenv > IGM_MAX_ENVELOPES) return fail(c, IGM_E_INVALID, "nenvelopes out of range");
    for (int e = 0; e < P->nenv; ++e) {
        for (int d = 0; d < 3; ++d) {
            P->env_abc[e][d] = (float)prm->env_semiaxes[e][d];
            P->env_abc_d[e][d] = prm->env_semiaxes[e][d];
        }
        P->env_k[e] = (float)prm->env_k[e];
        P->env_k_d[e] = prm->env_k[e];
    }
    P->skin = prm->skin > 0 ? (float)prm->skin : rmax;  // LAMMPS 'neighbor maxrad bin'
    P->cut_list = 2.0f * rmax + P->skin;
    P->kcap = prm->neigh_capacity > 0 ? prm->neigh_capacity : 128;
    if (P->kcap >= kNnbWalk) return fail(c, IGM_E_INVALID, "neigh_capacity must be < %d", kNnbWalk);
    P->natom = natom;
    P->nslice = (natom + 63) / 64;
    // atom types: one per distinct f32 radius, in order of first appearance
    std::vector<int> type(natom);
    std::vector<float> tr;
    std::unordered_map<uint32_t, int> seen;
    for (int i = 0; i < natom; ++i) {
        uint32_t key;
        memcpy(&key, &r[i], 4);
        auto it = seen.find(key);
        if (it == seen.end()) {
            it = seen.emplace(key, (int)tr.size()).first;
            tr.push_back(r[i]);
        }
        type[i] = it->second;
    }
    const int nt = (int)tr.size();
    if (nt > kMaxTypes) return fail(c, IGM_E_UNSUPPORTED, "%d distinct radii (> %d atom types)", nt, kMaxTypes);
    std::vector<double2> tab((size_t)nt * nt);
    std::vector<double> rt(nt);
    for (int a = 0; a < nt; ++a) {
        rt[a] = f32_as_printed(tr[a]);
        for (int b = 0; b < nt; ++b) {
            const float dc = tr[a] + tr[b];
            tab[(size_t)a * nt + b] = make_double2((double)dc, f32_as_printed(dc));
        }
    }
    void *p_t, *p_tab, *p_rt;
    IGM_TRY(workspace(c, "ms_atype", sizeof(int) * (size_t)natom, &p_t));
    IGM_TRY(workspace(c, "ms_ptab", sizeof(double2) * tab.size(), &p_tab));
    IGM_TRY(workspace(c, "ms_rtype", sizeof(double) * (size_t)nt, &p_rt));
    IGM_HIP_CHECK(c, hipMemcpyAsync(p_t, type.data(), sizeof(int) * natom, hipMemcpyHostToDevice, c->stream));
    IGM_HIP_CHECK(c, hipMemcpyAsync(p_tab, tab.data(), sizeof(double2) * tab.size(), hipMemcpyHostToDevice, c->stream));
    IGM_HIP_CHECK(c, hipMemcpyAsync(p_rt, rt.data(), sizeof(double) * nt, hipMemcpyHostToDevice, c->stream));
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));  // host vectors die here
    P->ntype = nt;
    P->pair_tab = (const double2*)p_tab;
    P->rtype = (const double*)p_rt;
    *d_atype = (const int*)p_t;
    return IGM_OK;
}

// stage inputs + build the bond adjacency for all structures
int prepare(igm_ctx* c, uint32_t flags, const igm_mstep_params* prm, int32_t nstruct, int32_t natom,
            const float* radii, const uint32_t* atom_flags, const igm_bond* shared_bonds, int64_t nshared,
            const int64_t* sbond_ptr, const igm_bond* sbonds, Prepared* out) {
    if (natom <= 0 || natom > 65535) return fail(c, IGM_E_UNSUPPORTED, "natom=%d outside [1, 65535]", natom);
    const float* d_radii;
    const uint32_t* d_flags;
    const igm_bond* d_shared;
    const int64_t* d_sptr;
    const igm_bond* d_sb;
    IGM_TRY(to_device(c, flags, "ms_radii", radii, (size_t)natom, &d_radii));
    IGM_TRY(to_device(c, flags, "ms_flags", atom_flags, (size_t)natom, &d_flags));
    IGM_TRY(to_device(c, flags, "ms_shared", shared_bonds, (size_t)nshared, &d_shared));
    int64_t nsb = 0;
    if (sbond_ptr) {
        if (flags & IGM_DEVICE_PTRS) {
            IGM_HIP_CHECK(c, hipMemcpyAsync(&nsb, sbond_ptr + nstruct, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
            IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        } else {
            nsb = sbond_ptr[nstruct];
        }
    }
    IGM_TRY(to_device(c, flags, "ms_sptr", sbond_ptr, sbond_ptr ? (size_t)nstruct + 1 : 0, &d_sptr));
    IGM_TRY(to_device(c, flags, "ms_sbonds", sbonds, (size_t)nsb, &d_sb));
    if (nsb == 0) d_sb = nullptr;
    if (!sbond_ptr) d_sptr = nullptr;
    DevParams P;
    const int* d_atype;
    IGM_TRY(make_devparams(c, prm, natom, d_radii, d_flags, &P, &d_atype));
    const int nslice = P.nslice;
    void *p_deg, *p_soff, *p_size, *p_base, *p_err, *p_wc;
    IGM_TRY(workspace(c, "ms_deg", sizeof(int) * (size_t)nstruct * natom, &p_deg));
    IGM_TRY(workspace(c, "ms_soff", sizeof(int) * (size_t)nstruct * (nslice + 1), &p_soff));
    IGM_TRY(workspace(c, "ms_size", sizeof(int64_t) * (size_t)nstruct, &p_size));
    IGM_TRY(workspace(c, "ms_base", sizeof(int64_t) * (size_t)nstruct, &p_base));
    IGM_TRY(workspace(c, "ms_err", sizeof(int) * 4, &p_err));
    IGM_TRY(workspace(c, "ms_wc", sizeof(int) * 4, &p_wc));
    int* d_err = (int*)p_err;
    IGM_HIP_CHECK(c, hipMemsetAsync(d_err, 0, sizeof(int) * 4, c->stream));
    const size_t lds_cnt = sizeof(int) * (size_t)nslice * 64;
    if (lds_cnt > 160 * 1024) return fail(c, IGM_E_UNSUPPORTED, "natom too large for the adjacency builder");
    {
        Timed tm(c, "adjacency");
        hipLaunchKernelGGL(adj_count_kernel, dim3(nstruct), dim3(256), lds_cnt, c->stream, nstruct, natom, nslice,
                           d_shared, nshared, d_sptr, d_sb, (int*)p_deg, (int*)p_soff, (int64_t*)p_size, d_err);
        IGM_HIP_CHECK(c, hipGetLastError());
        size_t tmp_bytes = 0;
        IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, (int64_t*)p_size, (int64_t*)p_base,
                                                          nstruct, c->stream));
        void* d_tmp;
        IGM_TRY(workspace(c, "ms_scan_tmp", tmp_bytes, &d_tmp));
        IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_bytes, (int64_t*)p_size, (int64_t*)p_base,
                                                          nstruct, c->stream));
        int64_t last_base = 0, last_size = 0;
        int herr = 0;
        IGM_HIP_CHECK(c, hipMemcpyAsync(&last_base, (int64_t*)p_base + nstruct - 1, sizeof(int64_t),
                                        hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipMemcpyAsync(&last_size, (int64_t*)p_size + nstruct - 1, sizeof(int64_t),
                                        hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipMemcpyAsync(&herr, d_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        if (herr & 2) return fail(c, IGM_E_INVALID, "bond atom index out of range");
        const int64_t total = last_base + last_size;
        void* p_ent;
        IGM_TRY(workspace(c, "ms_ent", sizeof(int4) * (size_t)(total > 0 ? total : 1), &p_ent));
        const size_t lds_fill = sizeof(int) * (size_t)natom;
        hipLaunchKernelGGL(adj_fill_kernel, dim3(nstruct), dim3(256), lds_fill, c->stream, nstruct, natom, nslice,
                           d_shared, nshared, d_sptr, d_sb, (const int*)p_deg, (const int*)p_soff,
                           (const int64_t*)p_base, (int4*)p_ent);
        IGM_HIP_CHECK(c, hipGetLastError());
        out->total_ent = total;
        out->cm.bonds.ent = (const int4*)p_ent;
    }
    out->cm.nstruct = nstruct;
    out->cm.natom = natom;
    out->cm.nslice = nslice;
    out->cm.kcap = P.kcap;
    out->cm.radii = d_radii;
    out->cm.atype = d_atype;
    out->cm.aflags = d_flags;
    out->cm.bonds.base = (const int64_t*)p_base;
    out->cm.bonds.soff = (const int*)p_soff;
    out->cm.bonds.deg = (const int*)p_deg;
    out->cm.work_counter = (int*)p_wc;
    out->cm.error = d_err;
    out->P = P;
    return IGM_OK;
}

// launch configuration: NT threads, BPT atoms per thread
struct LaunchCfg {
    int nt, bpt;
};

int pick_cfg(igm_ctx* c, int natom, LaunchCfg* cfg) {
    static const int opts[][2] = {{256, 1}, {512, 1}, {1024, 1}, {1024, 2}, {1024, 3}};
    for (auto& o : opts)
        if (o[0] * o[1] >= natom) {
            cfg->nt = o[0];
            cfg->bpt = o[1];
            return IGM_OK;
        }
    return fail(c, IGM_E_UNSUPPORTED,
                "natom=%d exceeds the LDS-resident M-step kernel (max 3072 atoms per structure)", natom);
}

#define IGM_DISPATCH_CFG(NTV, BPTV, ...)                           \
    if (cfg.nt == NTV && cfg.bpt == BPTV) {                        \
        constexpr int NT = NTV, BPT = BPTV;                        \
        __VA_ARGS__;                                               \
        done = true;                                               \
    }

#define IGM_DISPATCH_ALL(...)                                      \
    bool done = false;                                             \
    IGM_DISPATCH_CFG(256, 1, __VA_ARGS__)                          \
    else IGM_DISPATCH_CFG(512, 1, __VA_ARGS__)                     \
    else IGM_DISPATCH_CFG(1024, 1, __VA_ARGS__)                    \
    else IGM_DISPATCH_CFG(1024, 2, __VA_ARGS__)                    \
    else IGM_DISPATCH_CFG(1024, 3, __VA_ARGS__)                    \
    if (!done) return fail(c, IGM_E_UNSUPPORTED, "no kernel configuration");

template <typename KernelT>
int resident_grid(igm_ctx* c, KernelT kernel, int nt, size_t lds, int nstruct, int* grid) {
    int per_cu = 0;
    IGM_HIP_CHECK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, nt, lds));
    if (per_cu < 1) return fail(c, IGM_E_UNSUPPORTED, "kernel does not fit a CU (lds=%zu)", lds);
    int g = per_cu * c->num_cus;
    *grid = g < nstruct ? g : nstruct;
    return IGM_OK;
}

int run_anneal(igm_ctx* c, const Prepared& pr, const igm_mstep_params* prm, float* d_xyz, float* d_vel,
               const int* d_seeds, int* d_nreb, int mode, double seg_evf, double seg_envf, double t0, double t1,
               double xmax, int nsteps, float* d_forces = nullptr) {
    LaunchCfg cfg;
    IGM_TRY(pick_cfg(c, pr.cm.natom, &cfg));
    AnnealArgs A;
    memset(&A, 0, sizeof(A));
    A.cm = pr.cm;
    A.P = pr.P;
    A.xyz = d_xyz;
    A.vel = d_vel;
    A.nrebuild = d_nreb;
    A.forces_out = d_forces;
    A.mode = mode;
    A.dt = (float)prm->timestep;
    A.t_window = (float)(prm->t_window > 0 ? prm->t_window : 0.1);
    A.t_fraction = (float)(prm->t_fraction > 0 ? prm->t_fraction : 1.0);
    VelArgs V;
    memset(&V, 0, sizeof(V));
    if (mode == 1) {
        A.nseg = 1;
        A.seg_steps[0] = nsteps;
        A.seg_evf[0] = (float)seg_evf;
        A.seg_envf[0] = (float)seg_envf;
        A.seg_t0[0] = (float)t0;
        A.seg_t1[0] = (float)t1;
        A.seg_xmax[0] = (float)xmax;
    } else {
        // the runs of create_lammps_script (lammps.py:285-351): per stage an optional
        // relax run then the main run, each preceded by 'velocity create'
        int n = 0;
        for (int k = 0; k < prm->nstages; ++k) {
            const float evf = (float)(prm->evfactor_base * prm->evfactor[k]);  // fix adapt scale yes
            const float envf = (float)prm->envfactor[k];
            if (prm->relax_steps > 0) {
                A.seg_steps[n] = prm->relax_steps;
                A.seg_evf[n] = evf;
                A.seg_envf[n] = envf;
                A.seg_t0[n] = A.seg_t1[n] = (float)prm->relax_temperature;
                A.seg_xmax[n] = (float)prm->relax_max_velocity;
                V.seg_stage[n] = k;
                V.seg_temp[n] = (float)prm->relax_temperature;
                ++n;
            }
            A.seg_steps[n] = prm->mdsteps[k];
            A.seg_evf[n] = evf;
            A.seg_envf[n] = envf;
            A.seg_t0[n] = (float)prm->tstart[k];
            A.seg_t1[n] = (float)prm->tstop[k];
            A.seg_xmax[n] = (float)prm->max_velocity;
            V.seg_stage[n] = k;
            V.seg_temp[n] = (float)prm->tstart[k];
            ++n;
        }
        A.nseg = n;
        if (n > 0) {
            void* pv;
            IGM_TRY(workspace(c, "ms_vinit", sizeof(float) * (size_t)n * pr.cm.nstruct * pr.cm.natom * 3, &pv));
            V.nstruct = pr.cm.nstruct;
            V.natom = pr.cm.natom;
            V.nseg = n;
            V.aflags = pr.cm.aflags;
            V.seeds = d_seeds;
            V.vinit = (float*)pv;
            Timed tm(c, "velocity");
            hipLaunchKernelGGL(velocity_kernel, dim3(n, pr.cm.nstruct), dim3(256), 0, c->stream, V);
            IGM_HIP_CHECK(c, hipGetLastError());
            A.vinit = (const float*)pv;
        }
    }
    A.nbr_stride = (size_t)pr.cm.nslice * pr.cm.kcap * 64;
    IGM_HIP_CHECK(c, hipMemsetAsync(pr.cm.work_counter, 0, sizeof(int), c->stream));
    IGM_DISPATCH_ALL({
        const size_t lds = smem_bytes<float>(NT * BPT);
        auto kern = anneal_kernel<NT, BPT>;
        IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        int grid = 0;
        IGM_TRY(resident_grid(c, kern, NT, lds, pr.cm.nstruct, &grid));
        void* ws;
        IGM_TRY(workspace(c, "ms_nbr", sizeof(uint16_t) * A.nbr_stride * (size_t)grid, &ws));
        A.nbr_ws = (uint16_t*)ws;
        Timed tm(c, "anneal");
        hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, c->stream, A);
        IGM_HIP_CHECK(c, hipGetLastError());
    })
    return IGM_OK;
}

int run_cg(igm_ctx* c, const Prepared& pr, const igm_mstep_params* prm, float* d_xyz, const float* d_vel,
           igm_opt_info* d_info, const int* d_nreb, int mode, double evf, double envf, float* d_forces,
           double* d_energies) {
    LaunchCfg cfg;
    IGM_TRY(pick_cfg(c, pr.cm.natom, &cfg));
    CGArgs A;
    memset(&A, 0, sizeof(A));
    A.cm = pr.cm;
    A.P = pr.P;
    A.xyz = d_xyz;
    A.vel = d_vel;
    A.info = d_info;
    A.nrebuild_md = d_nreb;
    A.evf = evf;
    A.envf = envf;
    A.etol = prm->etol;
    A.ftol = prm->ftol;
    A.dmax = prm->dmax > 0 ? prm->dmax : 0.1;
    A.max_iter = prm->max_cg_iter;
    A.max_eval = prm->max_cg_eval;
    A.mode = mode;
    A.forces_out = d_forces;
    A.energies_out = d_energies;
    A.nbr_stride = (size_t)pr.cm.nslice * pr.cm.kcap * 64;
    IGM_HIP_CHECK(c, hipMemsetAsync(pr.cm.work_counter, 0, sizeof(int), c->stream));
    IGM_DISPATCH_ALL({
        const size_t lds = smem_bytes<double>(NT * BPT);
        auto kern = cg_kernel<NT, BPT>;
        IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        int grid = 0;
        IGM_TRY(resident_grid(c, kern, NT, lds, pr.cm.nstruct, &grid));
        void* ws;
        IGM_TRY(workspace(c, "ms_nbr", sizeof(uint16_t) * A.nbr_stride * (size_t)grid, &ws));
        A.nbr_ws = (uint16_t*)ws;
        void* vw;
        A.vec_stride = 12 * (size_t)(NT * BPT);
        IGM_TRY(workspace(c, "ms_cgvec", sizeof(double) * A.vec_stride * (size_t)grid, &vw));
        A.vec_ws = (double*)vw;
        Timed tm(c, mode == 0 ? "cg" : "forces");
        hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, c->stream, A);
        IGM_HIP_CHECK(c, hipGetLastError());
    })
    return IGM_OK;
}

int check_error(igm_ctx* c, const Prepared& pr) {
    int herr = 0;
    IGM_HIP_CHECK(c, hipMemcpyAsync(&herr, pr.cm.error, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    if (herr & 1)
        return fail(c, IGM_E_OVERFLOW,
                    "neighbour list overflow: an atom has more than %d neighbours within cutoff+skin; raise "
                    "igm_mstep_params.neigh_capacity",
                    pr.cm.kcap);
    return IGM_OK;
}

}  // namespace

extern "C" int igm_mstep_run(igm_ctx* c, uint32_t flags, const igm_mstep_params* prm, int32_t nstruct, int32_t natom,
                             float* xyz, const float* radii, const uint32_t* atom_flags,
                             const igm_bond* shared_bonds, int64_t nshared, const int64_t* sbond_ptr,
                             const igm_bond* sbonds, const int32_t* seeds, igm_opt_info* info) {
    if (!c || !prm || !xyz || !radii || !atom_flags || !seeds || nstruct <= 0)
        return fail(c, IGM_E_INVALID, "igm_mstep_run: invalid arguments");
    if (prm->nstages < 0 || prm->nstages > IGM_MAX_STAGES) return fail(c, IGM_E_INVALID, "nstages out of range");
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    Prepared pr;
    IGM_TRY(prepare(c, flags, prm, nstruct, natom, radii, atom_flags, shared_bonds, nshared, sbond_ptr, sbonds, &pr));
    float* d_xyz;
    const int* d_seeds;
    if (flags & IGM_DEVICE_PTRS) {
        d_xyz = xyz;
    } else {
        void* p;
        IGM_TRY(workspace(c, "ms_xyz", sizeof(float) * (size_t)nstruct * natom * 3, &p));
        d_xyz = (float*)p;
        IGM_HIP_CHECK(c, hipMemcpyAsync(d_xyz, xyz, sizeof(float) * (size_t)nstruct * natom * 3,
                                        hipMemcpyHostToDevice, c->stream));
    }
    IGM_TRY(to_device(c, flags, "ms_seeds", seeds, (size_t)nstruct, &d_seeds));
    void *p_vel, *p_reb, *p_info;
    IGM_TRY(workspace(c, "ms_vel", sizeof(float) * (size_t)nstruct * natom * 3, &p_vel));
    IGM_TRY(workspace(c, "ms_reb", sizeof(int) * (size_t)nstruct, &p_reb));
    igm_opt_info* d_info;
    if (info && (flags & IGM_DEVICE_PTRS)) {
        d_info = info;
    } else {
        IGM_TRY(workspace(c, "ms_info", sizeof(igm_opt_info) * (size_t)nstruct, &p_info));
        d_info = (igm_opt_info*)p_info;
    }
    IGM_TRY(run_anneal(c, pr, prm, d_xyz, (float*)p_vel, d_seeds, (int*)p_reb, 0, 0, 0, 0, 0, 0, 0));
    const double envf_last = prm->nstages > 0 ? prm->envfactor[prm->nstages - 1] : 1.0;
    IGM_TRY(run_cg(c, pr, prm, d_xyz, (const float*)p_vel, d_info, (const int*)p_reb, 0, prm->evfactor_base,
                   envf_last, nullptr, nullptr));
    IGM_TRY(check_error(c, pr));
    if (!(flags & IGM_DEVICE_PTRS)) {
        IGM_HIP_CHECK(c, hipMemcpyAsync(xyz, d_xyz, sizeof(float) * (size_t)nstruct * natom * 3,
                                        hipMemcpyDeviceToHost, c->stream));
        if (info) IGM_TRY(to_host(c, flags, info, d_info, (size_t)nstruct));
    }
    return finish(c, flags);
}

extern "C" int igm_mstep_forces(igm_ctx* c, uint32_t flags, const igm_mstep_params* prm, int32_t nstruct,
                                int32_t natom, const float* xyz, const float* radii, const uint32_t* atom_flags,
                                const igm_bond* shared_bonds, int64_t nshared, const int64_t* sbond_ptr,
                                const igm_bond* sbonds, double evf, double envf, float* forces, double* energies) {
    if (!c || !prm || !xyz || !radii || !atom_flags || nstruct <= 0)
        return fail(c, IGM_E_INVALID, "igm_mstep_forces: invalid arguments");
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    Prepared pr;
    IGM_TRY(prepare(c, flags, prm, nstruct, natom, radii, atom_flags, shared_bonds, nshared, sbond_ptr, sbonds, &pr));
    const float* d_xyz_c;
    IGM_TRY(to_device(c, flags, "mf_xyz", xyz, (size_t)nstruct * natom * 3, &d_xyz_c));
    float* d_forces;
    double* d_en;
    IGM_TRY(out_device(c, flags, "mf_forces", forces, (size_t)nstruct * natom * 3, &d_forces));
    IGM_TRY(out_device(c, flags, "mf_en", energies, (size_t)nstruct * (3 + IGM_MAX_ENVELOPES), &d_en));
    if (flags & IGM_F32_PATH) {
        // the f32 MD force path (anneal kernel, 0-step segment): forces only
        void *px, *pv;
        const size_t n3 = (size_t)nstruct * natom * 3;
        IGM_TRY(workspace(c, "mf_x32", sizeof(float) * n3, &px));
        IGM_TRY(workspace(c, "mf_v32", sizeof(float) * n3, &pv));
        IGM_HIP_CHECK(c, hipMemcpyAsync(px, d_xyz_c, sizeof(float) * n3, hipMemcpyDeviceToDevice, c->stream));
        IGM_HIP_CHECK(c, hipMemsetAsync(pv, 0, sizeof(float) * n3, c->stream));
        IGM_TRY(run_anneal(c, pr, prm, (float*)px, (float*)pv, nullptr, nullptr, 1, evf, envf, 0, 0, 1e30, 0,
                           d_forces));
        IGM_HIP_CHECK(c, hipMemsetAsync(d_en, 0xff, sizeof(double) * nstruct * (3 + IGM_MAX_ENVELOPES), c->stream));
    } else {
        IGM_TRY(run_cg(c, pr, prm, const_cast<float*>(d_xyz_c), nullptr, nullptr, nullptr, 1, evf, envf, d_forces,
                       d_en));
    }
    IGM_TRY(check_error(c, pr));
    IGM_TRY(to_host(c, flags, forces, d_forces, (size_t)nstruct * natom * 3));
    IGM_TRY(to_host(c, flags, energies, d_en, (size_t)nstruct * (3 + IGM_MAX_ENVELOPES)));
    return finish(c, flags);
}

extern "C" int igm_mstep_md(igm_ctx* c, uint32_t flags, const igm_mstep_params* prm, int32_t nstruct, int32_t natom,
                            float* xyz, float* v, const float* radii, const uint32_t* atom_flags,
                            const igm_bond* shared_bonds, int64_t nshared, const int64_t* sbond_ptr,
                            const igm_bond* sbonds, double evf, double envf, double t0, double t1,
                            double max_velocity, int32_t nsteps) {
    if (!c || !prm || !xyz || !v || !radii || !atom_flags || nstruct <= 0 || nsteps < 0)
        return fail(c, IGM_E_INVALID, "igm_mstep_md: invalid arguments");
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    Prepared pr;
    IGM_TRY(prepare(c, flags, prm, nstruct, natom, radii, atom_flags, shared_bonds, nshared, sbond_ptr, sbonds, &pr));
    float *d_xyz, *d_v;
    const size_t n3 = (size_t)nstruct * natom * 3;
    if (flags & IGM_DEVICE_PTRS) {
        d_xyz = xyz;
        d_v = v;
    } else {
        void *px, *pv;
        IGM_TRY(workspace(c, "md_xyz", sizeof(float) * n3, &px));
        IGM_TRY(workspace(c, "md_v", sizeof(float) * n3, &pv));
        d_xyz = (float*)px;
        d_v = (float*)pv;
        IGM_HIP_CHECK(c, hipMemcpyAsync(d_xyz, xyz, sizeof(float) * n3, hipMemcpyHostToDevice, c->stream));
        IGM_HIP_CHECK(c, hipMemcpyAsync(d_v, v, sizeof(float) * n3, hipMemcpyHostToDevice, c->stream));
    }
    IGM_TRY(run_anneal(c, pr, prm, d_xyz, d_v, nullptr, nullptr, 1, evf, envf, t0, t1, max_velocity, nsteps));
    IGM_TRY(check_error(c, pr));
    if (!(flags & IGM_DEVICE_PTRS)) {
        IGM_HIP_CHECK(c, hipMemcpyAsync(xyz, d_xyz, sizeof(float) * n3, hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipMemcpyAsync(v, d_v, sizeof(float) * n3, hipMemcpyDeviceToHost, c->stream));
    }
    return finish(c, flags);
}

extern "C" int igm_velocity_create(igm_ctx* c, uint32_t flags, int32_t nseed, int32_t natom,
                                   const uint32_t* atom_flags, const int32_t* seeds, double temperature, float* v) {
    if (!c || nseed <= 0 || natom <= 0 || !atom_flags || !seeds || !v)
        return fail(c, IGM_E_INVALID, "igm_velocity_create: invalid arguments");
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    VelArgs V;
    memset(&V, 0, sizeof(V));
    const int32_t* d_seeds;
    IGM_TRY(to_device(c, flags, "vc_flags", atom_flags, (size_t)natom, &V.aflags));
    IGM_TRY(to_device(c, flags, "vc_seeds", seeds, (size_t)nseed, &d_seeds));
    float* d_v;
    IGM_TRY(out_device(c, flags, "vc_v", v, (size_t)nseed * natom * 3, &d_v));
    V.nstruct = nseed;
    V.natom = natom;
    V.nseg = 1;
    V.seeds = d_seeds;
    V.seg_stage[0] = 0;
    V.seg_temp[0] = (float)temperature;
    V.vinit = d_v;
    hipLaunchKernelGGL(velocity_kernel, dim3(1, nseed), dim3(256), 0, c->stream, V);
    IGM_HIP_CHECK(c, hipGetLastError());
    IGM_TRY(to_host(c, flags, v, (const float*)d_v, (size_t)nseed * natom * 3));
    return finish(c, flags);
}
