// M-step engine: batched replacement of the per-structure serial LAMMPS run
// (igm/model/kernel/lammps.py:361-492 via ModelingStep.task, ModelingStep.py:508-509).
//
// Design (MI355X-first):
//  * one workgroup = one structure, persistent: it pulls structure ids from an
//    atomic work counter and runs the WHOLE protocol for that structure inside
//    one launch (47 000 MD steps for the demo protocol) -- no per-step launches.
//  * LDS path (natom <= 3072, the 2 Mb diploid model): float4 positions
//    (x, y, z, radius) AND the Verlet list live in LDS; each thread owns BPT atoms
//    (a = b*NT + t) and keeps their velocity, force and last-build position in
//    VGPRs.  Per MD step: one barrier after the position update (fused with the
//    neighbour-displacement vote, __syncthreads_or) and one for the temperature
//    sum of fix temp/rescale.  The only per-step HBM/L2 traffic left is the
//    compact bond adjacency (4 B per bond end).
//  * HBM path (larger structures, the 200 kb model with 29 838 beads): the same
//    algorithm with positions, Verlet list, cell grid and per-atom state in a
//    per-workgroup HBM workspace (L2/MALL-resident working set).
//  * neighbours: Verlet list with skin (LAMMPS 'neighbor maxrad bin', 'check
//    yes'), rebuilt in-kernel from a cell grid (count / scan / scatter / per-cell
//    sort -> deterministic order) into a compact CSR list (u16 entries).  Atoms
//    past the list capacity take their pair forces by walking the 27 cells of the
//    build-time grid, a superset of their list visited in the same order.
//  * bonds: per-structure sliced-ELLPACK adjacency (both ends, per-atom sorted
//    for a fixed summation order) of 4-byte entries j | type << 16 | lower << 31;
//    (r0, k) come from the structure's bond-type table -- the bond types LAMMPS
//    itself dedupes (lammps_model.py:314-329).
//  * anneal (MD) in f32 with f64 reductions; the CG minimisation (LAMMPS
//    min_style cg, quadratic line search) runs in a second kernel in f64,
//    because its energy tests (EMACH = 1e-8) need it.
#include <hipcub/hipcub.hpp>

#include <cstdlib>
#include <unordered_map>

#include "mstep_common.h"

namespace igm {
namespace ms {

constexpr uint32_t kLowerBit = 0x80000000u;
constexpr int kNnbWalk = 0xFFFF;          // nnb of an atom whose pair forces come from a cell walk
constexpr int kMaxTypes = 2048;           // distinct radii (LAMMPS atom types); the pair table is kMaxTypes^2
constexpr int kTypeHash = 8192;           // LDS hash slots of the bond-type builder
constexpr int kMaxBondTypes = 4096;       // distinct (r0, k) per structure
constexpr int kCellCapBig = 32768;        // cell grid of an HBM-resident structure
constexpr size_t kLdsBytes = 160 * 1024 - 1024;  // dynamic LDS per workgroup: 160 KB per CU (gfx950) less a static reserve
constexpr int kNeighBudget = 64;          // default Verlet-list slots per atom
constexpr int kLdsListSlots = 8;          // LDS path: the first slots of every atom's list live in LDS
#ifndef IGM_BOND_PRUNE
#define IGM_BOND_PRUNE 1  // LDS anneal: bonds that cannot act before the next list build are skipped
#endif
constexpr bool kBondPrune = IGM_BOND_PRUNE != 0;
#ifndef IGM_BOND_BATCH
#define IGM_BOND_BATCH 1  // LDS bonds per batch (config B anneal, with bond pruning: 1 is 0.8 % faster than 2, 2.7 % than 4)
#endif
#ifndef IGM_PAIR_BATCH
#define IGM_PAIR_BATCH 4
#endif
#ifndef IGM_POP_PAIR_BATCH
#define IGM_POP_PAIR_BATCH 1  // list quads (4 neighbours each) per batch of the population engine
#endif
constexpr int kPopPairBatch = IGM_POP_PAIR_BATCH;  // population engine: list quads whose loads are in flight together
#ifndef IGM_POP_FORCE_OCC
#define IGM_POP_FORCE_OCC 7  // waves per SIMD the force kernel's registers must allow (7: -1.0 % anneal against 6, which beat 4, 5 and 8)
#endif

// LDS anneal kernel: neighbours per batch.  LDS latency is short and lists are short, so
// the masked tail of a wide batch costs more than the extra loads in flight win
// (measured config B, anneal: batch 2 1700 ms, 1 1761 ms, 4 1779 ms, 8 1907 ms)
#ifndef IGM_LDS_PAIR_BATCH
#define IGM_LDS_PAIR_BATCH 2
#endif
constexpr int kLdsPairBatch = IGM_LDS_PAIR_BATCH;

// ------------------------------------------------------------------ carving
struct Carver {
    unsigned char* base;
    size_t o;
    __host__ __device__ explicit Carver(void* b) : base(static_cast<unsigned char*>(b)), o(0) {}
    template <typename T>
    __host__ __device__ T* take(size_t n) {
        o = (o + 15) & ~size_t(15);
        T* p = reinterpret_cast<T*>(base + o);
        o += n * sizeof(T);
        return p;
    }
};

struct Bonds {
    const uint32_t* ent;   // compact entries, sliced ELLPACK [slice][k][64 lanes]
    const int64_t* base;   // (B) first entry of structure s
    const int* soff;       // (B, nslice+1) slice offsets (entries)
    const int* deg;        // (B, natom)
    const float2* types;   // (r0, k) of every structure's bond types
    const int64_t* tbase;  // (B) first type of structure s
    const int64_t* ntype;  // (B) bond types of structure s
};

// The bonds of one atom: either the HBM adjacency (g: ELLPACK entries, stride 64,
// types gt) or, when the structure's bonds were staged in LDS, a CSR row l of u16
// entries j | (2*type + lower) << 12 with the type table lt.
struct BondView {
    const uint32_t* g;
    const float2* gt;
    const uint16_t* l;
    const float4* lt;  // LDS bond types {r0^2, 2 k r0, -2 k, k}
    int n;
};

struct Common {
    int nstruct, natom, nslice, ldn;  // ldn: SoA stride of per-atom HBM arrays (natom rounded to 64)
    const float* radii;
    const int* atype;  // per atom: index into DevParams::pair_tab / rtype
    const uint32_t* aflags;  // (natom), or (nstruct, natom) when afs == natom
    size_t afs;              // aflags stride between structures (0: shared by all)
    Bonds bonds;
    int* work_counter;  // dynamic structure scheduler
    int* error;         // error bits (per launch)
    int kcap;           // Verlet-list slots per atom (LDS + HBM)
};

// the neighbour structure of one workgroup (pointers into LDS or HBM).  The Verlet
// list is a fixed-capacity ELLPACK built in ONE pass: slot k < kl of atom a lives at
// lell[k * lstride + a] (LDS, bank-conflict free), slot k >= kl at
// gell[((a >> 6) * kg + k - kl) * 64 + (a & 63)] (HBM, one coalesced line per wave);
// an atom with more than kl + kg neighbours takes its pair forces from a cell walk.
template <typename T, typename OffT>
struct NList {
    OffT* cell;        // ncell+1 offsets into sorted (build-time cell grid)
    uint16_t* sorted;  // bead ids by cell, ascending inside a cell
    uint16_t* nnb;     // per atom: list length, or kNnbWalk
    uint16_t* lell;
    int lstride, kl;
    uint16_t* gell;
    int kg;
    int* scratch;      // the build's int scratch: (ncell + 1) + natom ints (aliases a list region)
    int cellcap;
    T* gp;             // lo[3], inv[3] of the grid (LDS)
    int* gn;           // nb[3] (LDS)
    __device__ __forceinline__ uint16_t* slot(int a, int k) const {
        return k < kl ? lell + (size_t)k * lstride + a : gell + ((size_t)(a >> 6) * kg + (k - kl)) * 64 + (a & 63);
    }
};

// small LDS block shared by every kernel variant
struct Red {
    double* red0;  // kMaxWaves*8
    double* red1;
    double* redb;
    int* wsum;     // kMaxWaves
    int* misc;     // 16
};

template <typename T>
__host__ __device__ inline Red carve_red(Carver& cv, T** gp, int** gn) {
    Red r;
    r.red0 = cv.take<double>(kMaxWaves * 8);
    r.red1 = cv.take<double>(kMaxWaves * 8);
    r.redb = cv.take<double>(kMaxWaves * 8);
    r.wsum = cv.take<int>(kMaxWaves);
    r.misc = cv.take<int>(16);
    *gp = cv.take<T>(8);
    *gn = cv.take<int>(8);
    return r;
}

// LDS layout of the MD kernel (LDS path).  `rest` holds the structure's bond CSR
// (when it fits) followed by the Verlet list; the list also serves as the build's
// int scratch.
constexpr int kLdsBondTypes = 8;  // 3-bit type field of an LDS bond entry (x2 for the lower-bound bit)

struct MdLds {
    Red r;
    float4* pos;
    uint16_t* boff;  // npad+8 bond CSR offsets
    float4* btab;    // kLdsBondTypes {r0^2, 2 k r0, -2 k, k}
    uint16_t* rest;  // the structure's bond CSR, when it fits
    int rest_cap;    // u16 entries
    NList<float, uint16_t> L;
};

__host__ __device__ inline MdLds carve_md_lds(void* smem, int npad) {
    Carver cv(smem);
    MdLds m;
    m.r = carve_red<float>(cv, &m.L.gp, &m.L.gn);
    m.pos = cv.take<float4>(npad);
    m.L.cell = cv.take<uint16_t>(kCellCap + 8);
    m.L.nnb = cv.take<uint16_t>(npad);
    m.L.sorted = cv.take<uint16_t>(npad);
    m.boff = cv.take<uint16_t>(npad + 8);
    m.btab = cv.take<float4>(kLdsBondTypes);
    m.L.lell = cv.take<uint16_t>((size_t)kLdsListSlots * npad);
    m.L.lstride = npad;
    m.L.kl = kLdsListSlots;
    m.L.scratch = reinterpret_cast<int*>(m.L.lell);
    m.L.gell = nullptr;
    m.L.kg = 0;
    m.L.cellcap = kCellCap;
    m.rest = cv.take<uint16_t>(0);
    const long rest = (long)kLdsBytes - (long)cv.o;
    m.rest_cap = rest > 0 ? (int)(rest / 2) : 0;
    return m;
}

// ints of the build's scratch: (ncell + 1) counts + natom slots
__host__ __device__ inline size_t build_scratch_bytes(int cellcap, int natom) {
    return sizeof(int) * (size_t)(cellcap + 2 + natom);
}

// HBM workspace of one workgroup: the neighbour structure (both kernels) and,
// for the MD kernel of the HBM path, positions + per-atom state
template <typename T>
struct BigWs {
    vec4_t<T>* pos;
    T* v;   // [3][ldn]
    T* f;   // [3][ldn]
    T* xb;  // [3][ldn]
};

template <typename T>
__host__ __device__ inline size_t carve_ws(void* base, int natom, int ldn, int kg, int cellcap, bool with_pos,
                                           bool with_state, NList<T, int>* L, BigWs<T>* W) {
    Carver cv(base);
    L->cell = cv.take<int>(cellcap + 8);
    L->nnb = cv.take<uint16_t>(ldn);
    L->sorted = cv.take<uint16_t>(ldn);
    L->gell = cv.take<uint16_t>((size_t)ldn * kg + 64 * IGM_PAIR_BATCH);  // slack for the batched reads
    L->kg = kg;
    L->lell = nullptr;
    L->lstride = 0;
    L->kl = 0;
    L->scratch = reinterpret_cast<int*>(L->gell);
    L->cellcap = cellcap;
    W->pos = with_pos ? cv.take<vec4_t<T>>(ldn) : nullptr;
    W->v = with_state ? cv.take<T>(3 * (size_t)ldn) : nullptr;
    W->f = with_state ? cv.take<T>(3 * (size_t)ldn) : nullptr;
    W->xb = with_state ? cv.take<T>(3 * (size_t)ldn) : nullptr;
    return (cv.o + 255) & ~size_t(255);
}

// --------------------------------------------------------- block scans
// out[i] = sum_{k<i} in[k] (i < n), out[n] = total; in may alias out.  Stored
// values saturate at the range of OutT (u16 offsets past the LDS list capacity
// only need to compare >= it).
template <int NT, typename InT, typename OutT>
__device__ __forceinline__ void block_scan(const InT* in, OutT* out, int n, int* wsum) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int cpt = (n + NT - 1) / NT;
    const int beg = t * cpt;
    constexpr long kMax = sizeof(OutT) == 2 ? 0xFFFF : 0x7FFFFFFF;
    long s = 0;
    for (int i = 0; i < cpt; ++i) {
        const int idx = beg + i;
        if (idx < n) s += (long)in[idx];
    }
    long incl = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const long y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[w] = (int)(incl > 0x7FFFFFFF ? 0x7FFFFFFF : incl);
    __syncthreads();
    long woff = 0, total = 0;
    for (int i = 0; i < NT / 64; ++i) {
        if (i < w) woff += wsum[i];
        total += wsum[i];
    }
    long run = woff + incl - s;
    for (int i = 0; i < cpt; ++i) {
        const int idx = beg + i;
        if (idx < n) {
            const long v = (long)in[idx];
            out[idx] = (OutT)(run < kMax ? run : kMax);
            run += v;
        }
    }
    if (t == 0) out[n] = (OutT)(total < kMax ? total : kMax);
    __syncthreads();
}

// --------------------------------------------------------- neighbour build
template <typename T>
__device__ __forceinline__ int cell_index(T x, T y, T z, const T* lo, const T* inv, const int* nb) {
    const T pp[3] = {x, y, z};
    int ci[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const int v = (int)((pp[d] - lo[d]) * inv[d]);
        ci[d] = v < 0 ? 0 : (v >= nb[d] ? nb[d] - 1 : v);
    }
    return (ci[2] * nb[1] + ci[1]) * nb[0] + ci[0];
}

// visit the beads of the 27 cells around cell c (x-runs are contiguous in `sorted`):
// f(j, valid) in batches of WB -- the bead ids of a batch are loaded together so the
// dependent LDS reads overlap; an invalid slot carries a valid id (masked by caller)
#ifndef IGM_WALK_BATCH
#define IGM_WALK_BATCH 4
#endif
#ifndef IGM_LDS_WALK_BATCH
// the LDS list build's walk: candidates per batch (cell-ordered lanes walk similar runs;
// measured on config B: 2 is 1.3 % faster than 4, 8 is 4.8 % slower)
#define IGM_LDS_WALK_BATCH 2
#endif
#ifndef IGM_WALK_SORTED
#define IGM_WALK_SORTED 1  // LDS list build: threads walk the beads in cell order
#endif
template <int WB = IGM_WALK_BATCH, typename OffT, typename F>
__device__ __forceinline__ void walk27(int c, const OffT* cell, const uint16_t* sorted, const int* gn, F&& f) {
    const int nx = gn[0], ny = gn[1], nz = gn[2];
    const int cx = c % nx, cy = (c / nx) % ny, cz = c / (nx * ny);
    for (int dz = -1; dz <= 1; ++dz) {
        const int z0 = cz + dz;
        if (z0 < 0 || z0 >= nz) continue;
        for (int dy = -1; dy <= 1; ++dy) {
            const int y0 = cy + dy;
            if (y0 < 0 || y0 >= ny) continue;
            const int row = (z0 * ny + y0) * nx;
            const int xlo = cx > 0 ? cx - 1 : 0, xhi = cx + 1 < nx ? cx + 1 : nx - 1;
            const int beg = (int)cell[row + xlo], end = (int)cell[row + xhi + 1];
            for (int q = beg; q < end; q += WB) {
                int jj[WB];
#pragma unroll
                for (int u = 0; u < WB; ++u) {
                    const int qq = q + u < end ? q + u : beg;
                    jj[u] = sorted ? (int)sorted[qq] : qq;  // no `sorted`: the runs hold the ids themselves
                }
#pragma unroll
                for (int u = 0; u < WB; ++u) f(jj[u], q + u < end);
            }
        }
    }
}

// Verlet list with skin from a cell grid.  Positions are read from `pos` (all
// writers have passed a barrier).  The bead mask is pos.w >= 0.  Ends with a
// barrier.  Returns the clock cycles of the list-fill walk (profiling).
template <typename T, int NT, typename OffT>
__device__ __noinline__ unsigned long long build_nlist(int natom, const vec4_t<T>* pos, NList<T, OffT> L, T cut_list, Red R) {
    const int t = threadIdx.x;
    float mm[6];
#pragma unroll
    for (int d = 0; d < 6; ++d) mm[d] = -3.0e38f;
    for (int a = t; a < natom; a += NT) {
        const vec4_t<T> p = pos[a];
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
        block_max<NT, 6>(md, R.redb);
#pragma unroll
        for (int d = 0; d < 6; ++d) mm[d] = (float)md[d];
    }
    // grid (identical in every thread): cells of side >= cut_list, at most cellcap
    T lo[3], inv[3];
    int nb[3];
    {
        float ext[3], vol = 1.0f;
        const float cut = (float)cut_list;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            ext[d] = mm[3 + d] + mm[d];
            if (!(ext[d] >= 0.0f)) ext[d] = 0.0f;
            vol *= fmaxf(ext[d], cut);
        }
        float cs = cut;
        if (vol / (cs * cs * cs) > (float)L.cellcap) cs = cbrtf(vol / (float)L.cellcap) * 1.0001f;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = (T)(-mm[d]);
            nb[d] = (int)floorf(ext[d] / cs);
            if (nb[d] < 1) nb[d] = 1;
            inv[d] = ext[d] > 0.0f ? (T)((float)nb[d] / ext[d]) : T(0);
        }
    }
    const int ncell = nb[0] * nb[1] * nb[2];
    if (t == 0) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            L.gp[d] = lo[d];
            L.gp[3 + d] = inv[d];
            L.gn[d] = nb[d];
        }
    }
    int* cnt = L.scratch;  // ncell+1 counts, then natom slots
    int* slot = cnt + ncell + 1;
    for (int c = t; c <= ncell; c += NT) cnt[c] = 0;
    __syncthreads();
    for (int a = t; a < natom; a += NT) {
        const vec4_t<T> p = pos[a];
        if (!(p.w >= T(0))) continue;
        slot[a] = atomicAdd(&cnt[cell_index<T>(p.x, p.y, p.z, lo, inv, nb)], 1);
    }
    __syncthreads();
    block_scan<NT, int, int>(cnt, cnt, ncell, R.wsum);
    for (int c = t; c <= ncell; c += NT) L.cell[c] = (OffT)cnt[c];
    for (int a = t; a < natom; a += NT) {
        const vec4_t<T> p = pos[a];
        if (!(p.w >= T(0))) continue;
        L.sorted[cnt[cell_index<T>(p.x, p.y, p.z, lo, inv, nb)] + slot[a]] = (uint16_t)a;
    }
    __syncthreads();
    for (int c = t; c < ncell; c += NT) {  // deterministic order inside each cell
        const int beg = (int)L.cell[c], end = (int)L.cell[c + 1];
        for (int i = beg + 1; i < end; ++i) {
            const uint16_t v = L.sorted[i];
            int k = i - 1;
            while (k >= beg && L.sorted[k] > v) {
                L.sorted[k + 1] = L.sorted[k];
                --k;
            }
            L.sorted[k + 1] = v;
        }
    }
    __syncthreads();
    const T cut2 = cut_list * cut_list;
    const unsigned long long c_walk = clock64();
    // one pass: walk the 27 cells, write the list slots (the scratch above is dead)
    const int cap = L.kl + L.kg;
    for (int a = t; a < natom; a += NT) {
        const vec4_t<T> p0 = pos[a];
        int k = 0;
        if (p0.w >= T(0)) {
            walk27(cell_index<T>(p0.x, p0.y, p0.z, lo, inv, nb), L.cell, L.sorted, nb, [&](int j, bool ok) {
                const vec4_t<T> p = pos[j];
                const T ddx = p0.x - p.x, ddy = p0.y - p.y, ddz = p0.z - p.z;
                const bool in = ok && j != a && ddx * ddx + ddy * ddy + ddz * ddz < cut2;
                if (in && k < L.kl) L.lell[(size_t)k * L.lstride + a] = (uint16_t)j;
                if (in && k >= L.kl && k < cap) L.gell[((size_t)(a >> 6) * L.kg + (k - L.kl)) * 64 + (a & 63)] = (uint16_t)j;
                k += in ? 1 : 0;
            });
        }
        L.nnb[a] = (uint16_t)(k <= cap ? k : kNnbWalk);
    }
    __syncthreads();
    return clock64() - c_walk;
}

// LDS-path Verlet-list build of the anneal kernel: the algorithm and the list of
// build_nlist (same grid, same cell order, ascending ids inside a cell, same slot
// order -> bitwise the same list), written against address-space-qualified
// pointers.  As a separate (non-inlined) function the generic pointers of NList
// would compile to FLAT memory operations with full vmcnt+lgkmcnt waits and 64-bit
// address arithmetic; here every scratch, grid and list access is a ds_* op and
// the overflow slots are global stores.
#if defined(__HIP_DEVICE_COMPILE__)
#define IGM_LDS __attribute__((address_space(3)))
#define IGM_GLB __attribute__((address_space(1)))
#else  // host pass: the kernels' bodies are not compiled for the host
#define IGM_LDS
#define IGM_GLB
#endif
typedef float igm_f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 lds_f4(const IGM_LDS igm_f4v* p, int i) {
    const igm_f4v v = p[i];
    return make_float4(v.x, v.y, v.z, v.w);
}

template <int NT>
__device__ __noinline__ unsigned long long build_nlist_lds(int natom, int nwalk, const float4* pos_g,
                                                           NList<float, uint16_t> Lg, float cut_list, Red R) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    constexpr int NW = NT / 64;
    const IGM_LDS igm_f4v* pos = (const IGM_LDS igm_f4v*)pos_g;
    IGM_LDS uint16_t* cell = (IGM_LDS uint16_t*)Lg.cell;
    IGM_LDS uint16_t* sorted = (IGM_LDS uint16_t*)Lg.sorted;
    IGM_LDS uint16_t* nnb = (IGM_LDS uint16_t*)Lg.nnb;
    IGM_LDS uint16_t* lell = (IGM_LDS uint16_t*)Lg.lell;
    IGM_GLB uint16_t* gell = (IGM_GLB uint16_t*)Lg.gell;
    IGM_LDS int* cnt = (IGM_LDS int*)Lg.scratch;
    IGM_LDS float* redf = (IGM_LDS float*)R.redb;  // NW * 6 floats
    IGM_LDS int* wsum = (IGM_LDS int*)R.wsum;
    IGM_LDS float* gp = (IGM_LDS float*)Lg.gp;
    IGM_LDS int* gn = (IGM_LDS int*)Lg.gn;
    const int lstride = Lg.lstride, kl = Lg.kl, kg = Lg.kg, cap = kl + kg;
    // bounding box of the beads (max of -x and x: exact in f32)
    float mm[6];
#pragma unroll
    for (int d = 0; d < 6; ++d) mm[d] = -3.0e38f;
    for (int a = t; a < natom; a += NT) {
        const float4 p = lds_f4(pos, a);
        if (!(p.w >= 0.0f)) continue;
        mm[0] = fmaxf(mm[0], -p.x);
        mm[1] = fmaxf(mm[1], -p.y);
        mm[2] = fmaxf(mm[2], -p.z);
        mm[3] = fmaxf(mm[3], p.x);
        mm[4] = fmaxf(mm[4], p.y);
        mm[5] = fmaxf(mm[5], p.z);
    }
#pragma unroll
    for (int d = 0; d < 6; ++d)
        mm[d] = wave_max_f32(mm[d]);
    if (lane == 0)
#pragma unroll
        for (int d = 0; d < 6; ++d) redf[w * 6 + d] = mm[d];
    __syncthreads();
#pragma unroll
    for (int d = 0; d < 6; ++d) {
        float v = redf[d];
#pragma unroll
        for (int i = 1; i < NW; ++i) v = fmaxf(v, redf[i * 6 + d]);
        mm[d] = v;
    }
    // grid (identical in every thread and to build_nlist): cells of side >= cut_list
    float lo[3], inv[3];
    int nb[3];
    {
        float ext[3], vol = 1.0f;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            ext[d] = mm[3 + d] + mm[d];
            if (!(ext[d] >= 0.0f)) ext[d] = 0.0f;
            vol *= fmaxf(ext[d], cut_list);
        }
        float cs = cut_list;
        if (vol / (cs * cs * cs) > (float)Lg.cellcap) cs = cbrtf(vol / (float)Lg.cellcap) * 1.0001f;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = -mm[d];
            nb[d] = (int)floorf(ext[d] / cs);
            if (nb[d] < 1) nb[d] = 1;
            inv[d] = ext[d] > 0.0f ? (float)nb[d] / ext[d] : 0.0f;
        }
    }
    const int ncell = nb[0] * nb[1] * nb[2];
    if (t == 0) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            gp[d] = lo[d];
            gp[3 + d] = inv[d];
            gn[d] = nb[d];
        }
    }
    auto cell_of = [&](const float4& p) {
        int ci[3];
        const float pp[3] = {p.x, p.y, p.z};
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const int v = (int)((pp[d] - lo[d]) * inv[d]);
            ci[d] = v < 0 ? 0 : (v >= nb[d] ? nb[d] - 1 : v);
        }
        return (ci[2] * nb[1] + ci[1]) * nb[0] + ci[0];
    };
    IGM_LDS int* slot = cnt + ncell + 1;
    for (int c = t; c <= ncell; c += NT) cnt[c] = 0;
    __syncthreads();
    for (int a = t; a < natom; a += NT) {
        const float4 p = lds_f4(pos, a);
        if (!(p.w >= 0.0f)) continue;
        slot[a] = __hip_atomic_fetch_add(&cnt[cell_of(p)], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    {  // exclusive scan of the counts: cell[c] = sum_{c' < c} cnt[c'], cell[ncell] = total
        const int cpt = (ncell + NT - 1) / NT, beg = t * cpt;
        int s = 0;
        for (int i = 0; i < cpt; ++i)
            if (beg + i < ncell) s += cnt[beg + i];
        int incl = s;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        int woff = 0, total = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int v = wsum[i];
            woff += i < w ? v : 0;
            total += v;
        }
        int run = woff + incl - s;
        for (int i = 0; i < cpt; ++i) {
            const int idx = beg + i;
            if (idx < ncell) {
                const int v = cnt[idx];
                cnt[idx] = run;
                cell[idx] = (uint16_t)run;
                run += v;
            }
        }
        if (t == 0) {
            cnt[ncell] = total;
            cell[ncell] = (uint16_t)total;
        }
        __syncthreads();
    }
    for (int a = t; a < natom; a += NT) {
        const float4 p = lds_f4(pos, a);
        if (!(p.w >= 0.0f)) continue;
        sorted[cnt[cell_of(p)] + slot[a]] = (uint16_t)a;
    }
    __syncthreads();
    for (int c = t; c < ncell; c += NT) {  // deterministic order inside each cell
        const int beg = (int)cell[c], end = (int)cell[c + 1];
        for (int i = beg + 1; i < end; ++i) {
            const uint16_t v = sorted[i];
            int k = i - 1;
            while (k >= beg && sorted[k] > v) {
                sorted[k + 1] = sorted[k];
                --k;
            }
            sorted[k + 1] = v;
        }
    }
    __syncthreads();
    const float cut2 = cut_list * cut_list;
    const unsigned long long c_walk = clock64();
    // one pass: walk the 27 cells (9 x-runs of consecutive sorted slots), write the
    // list slots (the count scratch above is dead)
    const int nx = nb[0], ny = nb[1], nz = nb[2];
#if IGM_WALK_SORTED
    // threads take the beads in cell order (lanes of a wave = neighbouring cells: their
    // 27-cell walks have similar run lengths and read neighbouring positions); the
    // non-bead atoms have empty lists
    // (a domain of the domain-decomposed engine, nwalk < natom, walks its owned atoms in
    // id order -- chain order, also spatially coherent -- so no lane idles on a halo atom)
    const bool by_cell = nwalk == natom;
    if (by_cell)
        for (int a = t; a < nwalk; a += NT)
            if (!(lds_f4(pos, a).w >= 0.0f)) nnb[a] = 0;
    const int nq = by_cell ? (int)cell[ncell] : nwalk;
    for (int qa = t; qa < nq; qa += NT) {
        const int a = by_cell ? (int)sorted[qa] : qa;
#else
    for (int a = t; a < nwalk; a += NT) {
#endif
        const float4 p0 = lds_f4(pos, a);
        int k = 0;
        if (p0.w >= 0.0f) {
            const int c = cell_of(p0);
            const int cx = c % nx, cy = (c / nx) % ny, cz = c / (nx * ny);
            const int xlo = cx > 0 ? cx - 1 : 0, xhi = cx + 1 < nx ? cx + 1 : nx - 1;
            for (int dz = -1; dz <= 1; ++dz) {
                const int z0 = cz + dz;
                if (z0 < 0 || z0 >= nz) continue;
                for (int dy = -1; dy <= 1; ++dy) {
                    const int y0 = cy + dy;
                    if (y0 < 0 || y0 >= ny) continue;
                    const int row = (z0 * ny + y0) * nx;
                    const int beg = (int)cell[row + xlo], end = (int)cell[row + xhi + 1];
                    for (int q = beg; q < end; q += IGM_LDS_WALK_BATCH) {
                        int jj[IGM_LDS_WALK_BATCH];
#pragma unroll
                        for (int u = 0; u < IGM_LDS_WALK_BATCH; ++u) jj[u] = (int)sorted[q + u < end ? q + u : beg];
                        float4 pj[IGM_LDS_WALK_BATCH];
#pragma unroll
                        for (int u = 0; u < IGM_LDS_WALK_BATCH; ++u) pj[u] = lds_f4(pos, jj[u]);
#pragma unroll
                        for (int u = 0; u < IGM_LDS_WALK_BATCH; ++u) {
                            const float ddx = p0.x - pj[u].x, ddy = p0.y - pj[u].y, ddz = p0.z - pj[u].z;
                            const bool in = q + u < end && jj[u] != a && ddx * ddx + ddy * ddy + ddz * ddz < cut2;
                            if (in) {
                                if (k < kl)
                                    lell[k * lstride + a] = (uint16_t)jj[u];
                                else if (k < cap)
                                    gell[((a >> 6) * kg + (k - kl)) * 64 + (a & 63)] = (uint16_t)jj[u];
                            }
                            k += in ? 1 : 0;
                        }
                    }
                }
            }
        }
        nnb[a] = (uint16_t)(k <= cap ? k : kNnbWalk);
    }
    __syncthreads();
    return clock64() - c_walk;
}

// ------------------------------------------------------------- forces
// pair force (and energy if EN) of atom i (xi, yi, zi, radius/type ri) from atom j
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

// pair forces of an atom past the list capacity: walk the 27 cells around its
// build-time position (a superset of its list, visited in the same order)
template <typename T, bool EN, typename OffT>
__device__ __noinline__ void pair_walk(int a, T xi, T yi, T zi, T ri, const vec4_t<T>* pos, const NList<T, OffT>& L,
                                       T bx, T by, T bz, const DevParams& P, T evf, T& fx, T& fy, T& fz,
                                       double& ep) {
    T gx = 0, gy = 0, gz = 0;
    double e = 0.0;
    walk27(cell_index<T>(bx, by, bz, L.gp, L.gp + 3, L.gn), L.cell, L.sorted, L.gn, [&](int j, bool ok) {
        if (ok && j != a) pair_one<T, EN>(j, xi, yi, zi, ri, pos, P, evf, gx, gy, gz, e);
    });
    fx = gx;
    fy = gy;
    fz = gz;
    if (EN) ep += e;
}

// the same for the f32 MD force path, returning the force by value: a reference to
// the caller's accumulators would make them escape into this out-of-line call and
// live in scratch memory for the whole force routine (every bond's `fx +=` a scratch
// load and store)
__device__ __noinline__ float4 pair_walk_md(int a, float4 p0, const float4* pos, NList<float, uint16_t> L, float bx,
                                            float by, float bz, const DevParams& P, float evf) {
    float gx = 0.0f, gy = 0.0f, gz = 0.0f;
    double e = 0.0;
    walk27(cell_index<float>(bx, by, bz, L.gp, L.gp + 3, L.gn), L.cell, L.sorted, L.gn, [&](int j, bool ok) {
        if (ok && j != a) pair_one<float, false>(j, p0.x, p0.y, p0.z, p0.w, pos, P, evf, gx, gy, gz, e);
    });
    return make_float4(gx, gy, gz, 0.0f);
}

// the bonds of one atom from the HBM adjacency (B.g, B.gt; B.n entries)
template <typename T, bool EN>
__device__ __forceinline__ void hbm_bonds(T xi, T yi, T zi, const vec4_t<T>* pos, const BondView& B, T& fx, T& fy,
                                          T& fz, double& eb) {
    constexpr int UB = 4;  // HBM bond entries per batch
    for (int k0 = 0; k0 < B.n; k0 += UB) {
        uint32_t ev[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) ev[u] = (k0 + u < B.n) ? B.g[(size_t)(k0 + u) * 64] : 0u;
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            if (k0 + u >= B.n) continue;
            const uint32_t e32 = ev[u];
            const float2 rk = B.gt[(e32 >> 16) & 0x7fffu];
            const vec4_t<T> p = pos[e32 & 0xffffu];
            const T dx = xi - p.x, dy = yi - p.y, dz = zi - p.z;
            double e = 0.0;
            const T fb = bond_term<T, EN>(dx * dx + dy * dy + dz * dz, (T)rk.x, (T)rk.y, (e32 & kLowerBit) != 0u, e);
            fx += fb * dx;
            fy += fb * dy;
            fz += fb * dz;
            if (EN) eb += 0.5 * e;
        }
    }
}

// envelope terms and fix setforce of one atom (radius/type ri as stored in pos.w)
template <typename T, bool EN>
__device__ __forceinline__ void env_terms(int s, T xi, T yi, T zi, T ri, uint32_t fl, const DevParams& P, T envf,
                                          T& fx, T& fy, T& fz, double (&ee)[IGM_MAX_ENVELOPES]) {
    // non-bead atoms carry -(w + 1); f32: w = radius, f64: w = atom type
    T rad;
    if constexpr (std::is_same<T, float>::value)
        rad = ri >= T(0) ? ri : -ri - T(1);
    else
        rad = P.rtype[ri >= T(0) ? (int)ri : (int)(-ri - T(1))];
    for (int e = 0; e < P.nenv; ++e) {
        if (!(fl & (IGM_ATOM_ENV0 << e))) continue;
        double en = 0.0;
        if (P.env_kind[e] == IGM_ENV_VOLUME) {
            const T kk = std::is_same<T, float>::value ? (T)P.env_k[e] : (T)P.env_k_d[e];
            volume_term<T, EN>(xi, yi, zi, P.vmaps[P.vsmap ? P.vsmap[s] : 0], P.vvox, envf, kk, fx, fy, fz, en);
        } else if constexpr (std::is_same<T, float>::value)
            envelope_term<T, EN>(xi, yi, zi, rad, P.env_abc[e][0] * envf, P.env_abc[e][1] * envf,
                                 P.env_abc[e][2] * envf, P.env_k[e], fx, fy, fz, en);
        else
            envelope_term<T, EN>(xi, yi, zi, rad, P.env_abc_d[e][0] * envf, P.env_abc_d[e][1] * envf,
                                 P.env_abc_d[e][2] * envf, P.env_k_d[e], fx, fy, fz, en);
        if (EN) ee[e] += en;
    }
    if (fl & IGM_ATOM_FIXED) fx = fy = fz = T(0);  // fix setforce 0 (lammps.py:222-223)
}

// Total force on atom a, gathered by its owner thread: pairs from the Verlet
// list (or the cell walk around the build-time position b*), bonds B, envelopes
// (the CG kernel; the f32 MD kernel uses atom_force_md).
template <typename T, bool EN, typename OffT, int PB = IGM_PAIR_BATCH>
__device__ __forceinline__ void atom_force(int s, int a, const vec4_t<T>& p0, uint32_t fl, const vec4_t<T>* pos,
                                           const NList<T, OffT>& L, T bx, T by, T bz, const BondView& B,
                                           const DevParams& P, T evf, T envf, T& fx, T& fy,
                                           T& fz, double& ep, double& eb, double (&ee)[IGM_MAX_ENVELOPES]) {
    fx = fy = fz = T(0);
    const T xi = p0.x, yi = p0.y, zi = p0.z;
    const T ri = (T)p0.w;
    if (ri >= T(0)) {
        const int nn = L.nnb[a];
        if (nn == kNnbWalk) {
            pair_walk<T, EN, OffT>(a, xi, yi, zi, ri, pos, L, bx, by, bz, P, evf, fx, fy, fz, ep);
        } else if (nn > 0) {
            constexpr int U = PB;  // neighbours whose loads are in flight together
            const int n1 = nn < L.kl ? nn : L.kl;
            const uint16_t* gl = L.gell + (size_t)(a >> 6) * L.kg * 64 + (a & 63);
            for (int k0 = 0; k0 < nn; k0 += U) {
                int jv[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int k = k0 + u;
                    jv[u] = k >= nn ? -1 : (k < n1 ? (int)L.lell[(size_t)k * L.lstride + a] : (int)gl[(size_t)(k - n1) * 64]);
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (jv[u] >= 0) pair_one<T, EN>(jv[u], xi, yi, zi, ri, pos, P, evf, fx, fy, fz, ep);
            }
        }
    }
    hbm_bonds<T, EN>(xi, yi, zi, pos, B, fx, fy, fz, eb);
    env_terms<T, EN>(s, xi, yi, zi, ri, fl, P, envf, fx, fy, fz, ee);
}

// soft-pair f/r of one flagged pair, without the evf/pi factor (applied once per
// atom): ONE v_rsq, t = 1/(r rc): sin(pi r/rc) = sin_rev(r^2 t / 2),
// f/r = evf/pi rc sin / r = evf/pi * rc^2 t sin.  Coincident atoms: 0.
__device__ __forceinline__ float soft_pair_t(float r2, float rc) {
    const float rc2 = rc * rc;
    const float t = __builtin_amdgcn_rsqf(fmaxf(r2 * rc2, 1.0e-30f));
    const float s = __builtin_amdgcn_sinf(0.5f * (r2 * t));
    return r2 > 0.0f ? rc2 * t * s : 0.0f;
}

// LDS bond entries 0..31 of an atom at p that may act before the next Verlet-list
// build (bit k: entry k).  Between builds every bead moves at most skin/2 (the
// `check yes` trigger), so a bead-bead distance changes by less than skin: an upper
// bound whose build distance is below r0 - skin (a lower bound: above r0 + skin)
// contributes exactly 0 until then.  Non-bead atoms are not watched by the trigger,
// so their bonds stay candidates.  1 % of the skin covers the f32 rounding.
__device__ __forceinline__ uint32_t bond_candidates(const float4& p, const uint16_t* l, int n, const float4* btab,
                                                    const float4* pos, float skin) {
    if (!(p.w >= 0.0f)) return 0xffffffffu;
    const float d = 1.01f * skin;
    uint32_t m = 0u;
    const int n32 = n < 32 ? n : 32;
    for (int k = 0; k < n32; ++k) {
        const uint32_t ev = l[k];
        const float4 pj = pos[ev & 0xfffu];
        const float r0 = __builtin_sqrtf(btab[ev >> 13].x);
        const float dx = p.x - pj.x, dy = p.y - pj.y, dz = p.z - pj.z;
        const float r = __builtin_sqrtf(dx * dx + dy * dy + dz * dz);
        const bool idle = pj.w >= 0.0f && (((ev >> 12) & 1u) ? r - d > r0 : r + d < r0);
        m |= idle ? 0u : 1u << k;
    }
    return m;
}

// f32 MD force of atom a in the LDS anneal kernel.  Pairs in two passes over
// the Verlet list: a distance filter over every entry (one bit per entry inside
// r_i + r_j) and the soft-pair force of the flagged entries only.  In a relaxed
// structure ~2% of the list interacts (the list reaches cut_list = rc_max + skin),
// so the rsq/sin work runs once or twice per atom instead of once per entry, and
// the filter pass is a gather, 6 FMA-class ops and a compare.  Entries are
// visited in slot order in both passes (fixed summation order).  LDS bonds take
// one rsq each from the type table {r0^2, 2 k r0, -2 k}: f/r = 2 k r0/r - 2 k.
template <int U>
__device__ __forceinline__ void atom_force_md(int s, int a, const float4& p0, uint32_t fl, const float4* pos,
                                              const NList<float, uint16_t>& L, float bx, float by, float bz,
                                              const BondView& B, const DevParams& P, float evf,
                                              float envf, float& fx, float& fy, float& fz, int amax,
                                              uint32_t bmask = 0xffffffffu) {
    fx = fy = fz = 0.0f;
    const float xi = p0.x, yi = p0.y, zi = p0.z, ri = p0.w;
    double unused = 0.0;
    if (ri >= 0.0f) {
        const int nn = L.nnb[a];
        if (nn == kNnbWalk) {
            const float4 w = pair_walk_md(a, p0, pos, L, bx, by, bz, P, evf);
            fx = w.x;
            fy = w.y;
            fz = w.z;
        } else if (nn > 0) {
            // slots k0..k0+U-1 are always readable (LDS: kl is a multiple of U; HBM: the
            // overflow regions carry U-1 slack slots); a slot past n holds a stale or
            // scratch value, clamped to a valid atom, its bit cleared after the pass
            const int n1 = nn < L.kl ? nn : L.kl;
            const uint16_t* ll = L.lell + a;
            const int ls = __builtin_amdgcn_readfirstlane(L.lstride);  // uniform: scalar slot offsets
            const uint16_t* gl = L.gell + (size_t)(a >> 6) * L.kg * 64 + (a & 63);
            float gx = 0.0f, gy = 0.0f, gz = 0.0f;
            auto filter = [&](int k0, int n, auto idx) {  // bits of the entries k0 .. k0+31 inside r_i + r_j
                uint32_t m = 0u;
                for (int k = 0; k < 32 && k0 + k < n; k += U) {
                    int jv[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) jv[u] = min((int)idx(k0 + k + u), amax);
                    float4 pj[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) pj[u] = pos[jv[u]];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const float dx = xi - pj[u].x, dy = yi - pj[u].y, dz = zi - pj[u].z;
                        const float rc = ri + pj[u].w;
                        m |= (dx * dx + dy * dy + dz * dz < rc * rc) ? (1u << (k + u)) : 0u;
                    }
                }
                const int left = n - k0;
                return left >= 32 ? m : m & ((1u << left) - 1u);
            };
            auto force = [&](int j) {
                const float4 pj = pos[j];
                const float dx = xi - pj.x, dy = yi - pj.y, dz = zi - pj.z;
                const float f = soft_pair_t(dx * dx + dy * dy + dz * dz, ri + pj.w);
                gx += f * dx;
                gy += f * dy;
                gz += f * dz;
            };
            {
                uint32_t m = filter(0, n1, [&](int k) { return ll[(size_t)k * ls]; });  // kl <= 32
                while (m) {
                    const int k = __builtin_ctz(m);
                    m &= m - 1u;
                    force(ll[(size_t)k * ls]);
                }
            }
            const int n2 = nn - n1;
            for (int w0 = 0; w0 < n2; w0 += 32) {
                uint32_t m = filter(w0, n2, [&](int k) { return gl[(size_t)k * 64]; });
                while (m) {
                    const int k = __builtin_ctz(m);
                    m &= m - 1u;
                    force(gl[(size_t)(w0 + k) * 64]);
                }
            }
            const float evfpi = evf * 0.318309886183790671537767526745f;
            fx = evfpi * gx;
            fy = evfpi * gy;
            fz = evfpi * gz;
        }
    }
    if (B.l) {
        // entries 0..31 whose bit in bmask is clear cannot act before the next list
        // build (bond_candidates); the rest are visited in entry order as before
        constexpr int UL = IGM_BOND_BATCH;  // LDS bond entries per batch, branch-free
        uint32_t bm = bmask;
        int kh = 32;
        for (;;) {
            int ku[UL];
#pragma unroll
            for (int u = 0; u < UL; ++u) {
                if (bm) {
                    ku[u] = __builtin_ctz(bm);
                    bm &= bm - 1u;
                } else {
                    ku[u] = kh++;
                }
            }
            if (ku[0] >= B.n) break;
            uint32_t ev[UL];
#pragma unroll
            for (int u = 0; u < UL; ++u) ev[u] = (uint32_t)B.l[ku[u] < B.n ? ku[u] : B.n - 1];
            float4 q[UL];
            float4 pj[UL];
#pragma unroll
            for (int u = 0; u < UL; ++u) {
                q[u] = B.lt[ev[u] >> 13];
                pj[u] = pos[ev[u] & 0xfffu];
            }
#pragma unroll
            for (int u = 0; u < UL; ++u) {
                const float dx = xi - pj[u].x, dy = yi - pj[u].y, dz = zi - pj[u].z;
                const float r2 = dx * dx + dy * dy + dz * dz;
                // upper bound active beyond r0, lower bound inside it
                const bool act = (r2 > q[u].x) != (((ev[u] >> 12) & 1u) != 0u);
                const float fb = q[u].y * __builtin_amdgcn_rsqf(fmaxf(r2, 1.0e-30f)) + q[u].z;
                const float m = (act && ku[u] < B.n) ? fb : 0.0f;
                fx += m * dx;
                fy += m * dy;
                fz += m * dz;
            }
        }
    } else {
        hbm_bonds<float, false>(xi, yi, zi, pos, B, fx, fy, fz, unused);
    }
    double ee[IGM_MAX_ENVELOPES];
    env_terms<float, false>(s, xi, yi, zi, ri, fl, P, envf, fx, fy, fz, ee);
}

// ------------------------------------------------------------- anneal
struct AnnealArgs {
    Common cm;
    DevParams P;
    float* xyz;          // (B, natom, 3)
    float* vel;          // (B, natom, 3): out (mode 0) / in-out (mode 1)
    const float* vinit;  // mode 0: (B, nseg, natom, 3) velocities of each 'velocity create'
    unsigned char* ws;   // HBM path: per resident workgroup
    size_t ws_stride;
    int* nrebuild;       // (B)
    unsigned long long* prof;  // optional: cycles {build, force, rest, steps, builds} summed over structures
    float* forces_out;   // forces at the end (B, natom, 3), may be null
    int mode;            // 0: full protocol, 1: one MD segment from vel
    int prune;           // LDS kernel: bond pruning on (IGM_BOND_PRUNE=0 turns it off: a test switch)
    int nseg;
    // per segment (mode 0) or the single segment (mode 1)
    int seg_steps[2 * IGM_MAX_STAGES];
    float seg_evf[2 * IGM_MAX_STAGES], seg_envf[2 * IGM_MAX_STAGES], seg_t0[2 * IGM_MAX_STAGES],
        seg_t1[2 * IGM_MAX_STAGES], seg_xmax[2 * IGM_MAX_STAGES];
    float seg_skin[2 * IGM_MAX_STAGES];  // Verlet skin of every run (equal forces for any skin; see run_anneal)
    float dt, t_window, t_fraction;
};

// next structure id of this workgroup (uniform), or >= nstruct when done
__device__ __forceinline__ int next_structure(const Common& cm, int* misc) {
    if (threadIdx.x == 0) misc[0] = atomicAdd(cm.work_counter, 1);
    __syncthreads();
    const int s = __builtin_amdgcn_readfirstlane(misc[0]);  // uniform: keeps derived pointers in SGPRs
    __syncthreads();
    return s;
}

// fix temp/rescale 1 t0 t1 window fraction at the end of step `step` of nsteps:
// the factor applied to every velocity (1 if no rescale)
__device__ __forceinline__ float temp_rescale_factor(double ke2, double dof, int step, int nsteps, float t0, float t1,
                                                     float window, float fraction) {
    const double tcur = dof > 0 ? ke2 / dof : 0.0;
    if (!(tcur > 0.0)) return 1.0f;
    const double delta = (double)step / (double)nsteps;
    double tt = (double)t0 + delta * ((double)t1 - (double)t0);
    if (!(fabs(tcur - tt) > (double)window)) return 1.0f;
    tt = tcur - (double)fraction * (tcur - tt);
    return (float)sqrt(tt / tcur);
}

// fix nve/limit half-kick with the velocity cap
__device__ __forceinline__ void kick_limit(float& vx, float& vy, float& vz, float fx, float fy, float fz, float dtf,
                                           float vlim, float vlimsq) {
    vx += dtf * fx;
    vy += dtf * fy;
    vz += dtf * fz;
    const float vsq = vx * vx + vy * vy + vz * vz;
    if (vsq > vlimsq) {
        const float sc = vlim * __frsqrt_rn(vsq);
        vx *= sc;
        vy *= sc;
        vz *= sc;
    }
}

// element b (runtime, uniform per loop trip) of a per-thread register array.  Each
// element passes through an empty asm first: a select of plain loads would be folded
// into ONE load from a selected address, i.e. a dynamically indexed array, which
// the compiler then keeps in scratch memory (it did: xb and the bond masks of
// anneal_kernel lived in scratch, read every step of the force loop).
template <typename X>
__device__ __forceinline__ X opaque(X x) {
    uint32_t u = __builtin_bit_cast(uint32_t, x);
    asm("" : "+v"(u));
    return __builtin_bit_cast(X, u);
}
template <int BPT, typename X>
__device__ __forceinline__ X pick(const X (&arr)[BPT], int b) {
    X r = opaque(arr[0]);
#pragma unroll
    for (int i = 1; i < BPT; ++i) r = b == i ? opaque(arr[i]) : r;
    return r;
}
template <int BPT>
__device__ __forceinline__ float pick(const float (&arr)[BPT][3], int b, int d) {
    float r = opaque(arr[0][d]);
#pragma unroll
    for (int i = 1; i < BPT; ++i) r = b == i ? opaque(arr[i][d]) : r;
    return r;
}

template <int NT, int BPT>
__global__ void __launch_bounds__(NT) anneal_kernel(AnnealArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int npad = NT * BPT;
    MdLds sm = carve_md_lds(smem, npad);
    sm.L.gell = reinterpret_cast<uint16_t*>(A.ws + (size_t)blockIdx.x * A.ws_stride);  // list overflow (HBM)
    sm.L.kg = A.cm.kcap - kLdsListSlots;
    const int t = threadIdx.x, lane = t & 63;
    const int natom = A.cm.natom;
    float v[BPT][3], f[BPT][3], xb[BPT][3];
    uint32_t bmk[BPT];  // LDS bond entries 0..31 that may act before the next list build
    for (;;) {
        const int s = next_structure(A.cm, sm.r.misc);
        if (s >= A.cm.nstruct) break;
        const float* xs = A.xyz + (size_t)s * natom * 3;
        uint32_t mobile = 0u;  // bit b: atom b*NT+t is integrated
        uint32_t flk = 0u;     // 5 bits per atom b: FIXED, ENV0..ENV3 (the flags the force reads)
        int nmob = 0;
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const int a = b * NT + t;
            const bool in = a < natom;
            const uint32_t fl = in ? A.cm.aflags[(size_t)s * A.cm.afs + a] : 0u;
            const bool bead = in && (fl & IGM_ATOM_BEAD);
            flk |= (((fl & IGM_ATOM_FIXED) ? 1u : 0u) | (((fl >> 4) & 0xfu) << 1)) << (5 * b);
            if (in && !(fl & IGM_ATOM_FIXED)) {
                mobile |= 1u << b;
                ++nmob;
            }
            const float r = in ? A.cm.radii[a] : 0.0f;
            sm.pos[a] = make_float4(in ? xs[(size_t)a * 3] : 0.f, in ? xs[(size_t)a * 3 + 1] : 0.f,
                                    in ? xs[(size_t)a * 3 + 2] : 0.f, bead ? r : -(r + 1.0f));
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                v[b][d] = 0.0f;
                f[b][d] = 0.0f;
                xb[b][d] = __int_as_float(0x7f800000);  // +inf: forces the first neighbour build
            }
            bmk[b] = 0xffffffffu;
        }
        double cnt[1] = {(double)nmob};
        block_sum<NT, 1>(cnt, sm.r.red0);
        const double dof = 3.0 * cnt[0] - 3.0;  // compute temp of group nonfixed
        __syncthreads();
        const uint32_t* adj = A.cm.bonds.ent + A.cm.bonds.base[s];
        const int* soff = A.cm.bonds.soff + (size_t)s * (A.cm.nslice + 1);
        const int* deg = A.cm.bonds.deg + (size_t)s * natom;
        const float2* bt = A.cm.bonds.types + A.cm.bonds.tbase[s];
        // stage the bonds in LDS when the structure's types and entries fit: CSR of
        // u16 entries j | (2*type + lower) << 12 ahead of the Verlet list
        block_scan<NT, int, uint16_t>(deg, sm.boff, natom, sm.r.wsum);
        const int nbent = __builtin_amdgcn_readfirstlane((int)sm.boff[natom]);
        const int bond_u16 = (nbent + 7) & ~7;
        const bool lds_bonds = A.cm.bonds.ntype[s] <= kLdsBondTypes && nbent < 0xFFFF && bond_u16 <= sm.rest_cap;
        if (lds_bonds) {
            for (int i = t; i < (int)A.cm.bonds.ntype[s]; i += NT) {
                const float2 rk = bt[i];
                sm.btab[i] = make_float4(rk.x * rk.x, 2.0f * rk.y * rk.x, -2.0f * rk.y, rk.y);
            }
            for (int a = t; a < natom; a += NT) {
                const uint32_t* g = adj + soff[a >> 6] + (a & 63);
                uint16_t* o = sm.rest + sm.boff[a];
                const int n = deg[a];
                for (int k = 0; k < n; ++k) {
                    const uint32_t e = g[(size_t)k * 64];
                    o[k] = (uint16_t)((e & 0xfffu) | ((((e >> 16) & 0x7fffu) * 2u + (e >> 31)) << 12));
                }
            }
        }
        __syncthreads();
        int nbuild = 0;
        unsigned long long c_build = 0, c_force = 0, c_all = 0, nstep_total = 0, c_walk = 0;
        const unsigned long long c_begin = A.prof ? clock64() : 0;
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
            const float skin = A.seg_skin[seg];
            const float trig = 0.25f * skin * skin;
            const float cut_list = A.P.cut_list - A.P.skin + skin;
            if (seg > 0 && skin != A.seg_skin[seg - 1])  // a new cut: rebuild at the run's setup step
#pragma unroll
                for (int b = 0; b < BPT; ++b) xb[b][0] = xb[b][1] = xb[b][2] = __int_as_float(0x7f800000);
            // ---- run nsteps: step 0 is Verlet::setup (forces only)
            for (int step = 0; step <= nsteps; ++step) {
                int moved = 0;
#pragma unroll
                for (int b = 0; b < BPT; ++b) {
                    const int a = b * NT + t;
                    float4 p = sm.pos[a];
                    if (step > 0 && (mobile >> b & 1u)) {  // fix nve/limit: initial_integrate
                        kick_limit(v[b][0], v[b][1], v[b][2], f[b][0], f[b][1], f[b][2], dtf, vlim, vlimsq);
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
                    const unsigned long long c0 = A.prof ? clock64() : 0;
                    const unsigned long long cw = build_nlist_lds<NT>(natom, natom, sm.pos, sm.L, cut_list, sm.r);
                    if (A.prof) {
                        c_build += clock64() - c0;
                        c_walk += cw;
                    }
                    ++nbuild;
#pragma unroll
                    for (int b = 0; b < BPT; ++b) {
                        const int a = b * NT + t;
                        const float4 p = sm.pos[a];
                        xb[b][0] = p.x;
                        xb[b][1] = p.y;
                        xb[b][2] = p.z;
                        bmk[b] = 0xffffffffu;
                        if (kBondPrune && A.prune && lds_bonds && a < natom)
                            bmk[b] = bond_candidates(p, sm.rest + sm.boff[a], (int)sm.boff[a + 1] - (int)sm.boff[a],
                                                     sm.btab, sm.pos, skin);
                    }
                }
                // forces: the owner thread gathers every contribution of its atoms (one
                // copy of the force code; per-atom registers picked by conditional moves)
                const unsigned long long cf0 = A.prof ? clock64() : 0;
#pragma unroll 1
                for (int b = 0; b < BPT; ++b) {
                    const int a = b * NT + t;
                    if (a < natom) {
                        float fx, fy, fz;
                        const BondView B = lds_bonds ? BondView{nullptr, nullptr, sm.rest + sm.boff[a], sm.btab,
                                                                (int)sm.boff[a + 1] - (int)sm.boff[a]}
                                                     : BondView{adj + soff[a >> 6] + lane, bt, nullptr, nullptr, deg[a]};
                        const uint32_t f5 = (flk >> (5 * b)) & 31u;
                        const uint32_t fla = ((f5 & 1u) ? IGM_ATOM_FIXED : 0u) | ((f5 >> 1) << 4);
                        atom_force_md<kLdsPairBatch>(s, a, sm.pos[a], fla, sm.pos,
                                                     sm.L, pick<BPT>(xb, b, 0), pick<BPT>(xb, b, 1),
                                                     pick<BPT>(xb, b, 2), B, A.P, evf, envf, fx, fy, fz,
                                                     natom - 1, pick<BPT>(bmk, b));
#pragma unroll
                        for (int i = 0; i < BPT; ++i) {  // (unconditional selects: no store to a selected address)
                            f[i][0] = b == i ? fx : f[i][0];
                            f[i][1] = b == i ? fy : f[i][1];
                            f[i][2] = b == i ? fz : f[i][2];
                        }
                    }
                }
                if (A.prof) {
                    __syncthreads();  // profiling only: the force phase of every wave
                    c_force += clock64() - cf0;
                    ++nstep_total;
                }
                if (step == 0) {
                    __syncthreads();  // setup forces read sm.pos: no update before every wave is done
                    continue;
                }
                double ts[1] = {0.0};
#pragma unroll
                for (int b = 0; b < BPT; ++b) {  // final_integrate
                    if (!(mobile >> b & 1u)) continue;
                    kick_limit(v[b][0], v[b][1], v[b][2], f[b][0], f[b][1], f[b][2], dtf, vlim, vlimsq);
#pragma unroll
                    for (int d = 0; d < 3; ++d) ts[0] += (double)(v[b][d] * v[b][d]);
                }
                block_sum<NT, 1>(ts, (step & 1) ? sm.r.red1 : sm.r.red0);
                const float factor = temp_rescale_factor(ts[0], dof, step, nsteps, t0, t1, A.t_window, A.t_fraction);
                if (factor != 1.0f)
#pragma unroll
                    for (int b = 0; b < BPT; ++b)
#pragma unroll
                        for (int d = 0; d < 3; ++d) v[b][d] *= factor;
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
            xo[(size_t)a * 3] = p.x;
            xo[(size_t)a * 3 + 1] = p.y;
            xo[(size_t)a * 3 + 2] = p.z;
#pragma unroll
            for (int d = 0; d < 3; ++d) vo[(size_t)a * 3 + d] = v[b][d];
            if (A.forces_out) {
                float* fo3 = A.forces_out + ((size_t)s * natom + a) * 3;
#pragma unroll
                for (int d = 0; d < 3; ++d) fo3[d] = f[b][d];
            }
        }
        if (t == 0 && A.nrebuild) A.nrebuild[s] = nbuild;
        if (t == 0 && A.prof) {
            c_all = clock64() - c_begin;
            atomicAdd(&A.prof[0], c_build);
            atomicAdd(&A.prof[1], c_force);
            atomicAdd(&A.prof[2], c_all - c_build - c_force);
            atomicAdd(&A.prof[3], nstep_total);
            atomicAdd(&A.prof[4], (unsigned long long)nbuild);
            atomicAdd(&A.prof[5], c_walk);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------- population engine
// Structures too large for one CU's LDS (the 200 kb model, 29 838 beads) run as ONE
// system: a step is a few launches over all atoms of all structures.  Every
// structure keeps its per-atom state in SLOT order -- the order of its atoms in the
// cell grid of its last Verlet-list build (cells x-fastest, ascending atom ids inside
// a cell, non-bead atoms last) -- so the 27-cell walk of a build reads contiguous
// position runs, and the neighbour and bond-partner gathers of a wave of 64
// consecutive slots fall on a few nearby cache lines.  At every build the state is
// permuted into the new slot order (two buffers) and the structure's bonds are
// re-indexed into slot space.  Per MD step:
//   pop_integrate  rescale of the previous step, kick, drift, displacement check, bbox
//   pop_sort       flagged structures, one workgroup each: counting sort into the cell
//                  grid in LDS, ids sorted inside each cell (deterministic), slot map
//   pop_permute    flagged structures: state and bonds into the new slot order
//   pop_fill       flagged structures: Verlet list (slot ids) from the cell runs
//   pop_force      forces, final kick, per-block kinetic-energy partial
// The three build kernels exit at once when no structure is flagged.  Per-structure
// sums go through per-block partials added in a fixed order, so a run is bitwise
// reproducible.
constexpr int kPopBS = 256;
constexpr int kPopSortNT = 1024;
constexpr int kPopMaxGroups = 64;  // structure groups (streams) of one run: build counters nflag[g], nflag2[g]
#ifndef IGM_POP_CELL_CAP
#define IGM_POP_CELL_CAP 32768
#endif
// cells of a structure's grid in the population engine: the sort keeps their u16 counts
// and the structure's u16 atom ids in one CU's LDS (32 768 cells + 29 838 ids: 124 KB).
// The cap trades the cold runs' cell size (0.475 rmax skin: ~39 000 cells of side cut_list
// over a 200 kb nucleus; at 32 768 they grow ~6 % past cut_list) against the sort's LDS
// footprint: at 124 KB a sort workgroup shares its CU with a fill workgroup of the other
// structure group (21.5 KB), at 158 KB (cap 49 152) with nothing.  Measured on config C
// (pop = 1000, protocol x0.05, two groups, same box, profiles/r05_ab): 49 152 5 451 / 5 456
// ms anneal, 32 768 5 366 / 5 363 / 5 308 ms, 24 576 5 551 ms.  (Round 3, one group in
// effect at protocol x0.1, had measured 49 152 0.8 % faster than 32 768.)
constexpr int kPopCellCap = IGM_POP_CELL_CAP;
constexpr int kPopCells = kPopCellCap + 2;  // cell offsets of a structure: real cells, non-bead run, end
constexpr int kPopCntStride = (kPopCells + 3) & ~3;  // cell counts of a structure (16-byte rows)
#ifndef IGM_POP_FILL_W
#define IGM_POP_FILL_W 2
#endif
constexpr int kFillW = IGM_POP_FILL_W;  // list build: slots per x-run loaded in one batch
#ifndef IGM_POP_FILL_TAIL
#define IGM_POP_FILL_TAIL 4
#endif
constexpr int kFillTail = IGM_POP_FILL_TAIL;  // list build: slots past the batch loaded at a time
#ifndef IGM_POP_LIST_CAP
#define IGM_POP_LIST_CAP 256
#endif
constexpr int kPopListCap = IGM_POP_LIST_CAP;  // Verlet-list entries per slot (more: the cell walk)
#ifndef IGM_POP_ROW_CAP
#define IGM_POP_ROW_CAP 40
#endif
// entries of the list build's LDS row per thread: the list collects there and is stored a
// block of quads at a time, so the list capacity is not bound by the row (the row sets
// the fill kernel's occupancy: 40 entries + 2 of stride, 84 B per thread, 7 workgroups per CU)
constexpr int kPopRowCap = IGM_POP_ROW_CAP;
#ifndef IGM_POP_PREFETCH
#define IGM_POP_PREFETCH 1  // force kernel: software-pipelined list quads, bond entries with the slot's loads
#endif
#ifndef IGM_POP_QDEPTH
#define IGM_POP_QDEPTH 2  // list quads in flight ahead of the one being gathered (2: -0.7 %, profiles/r04_ab)
#endif
#ifndef IGM_POP_BOND_BATCH
#define IGM_POP_BOND_BATCH 4  // force kernel: bond entries (and partner gathers) per batch
#endif
#ifndef IGM_POP_FUSED
// 1: list build + bond re-index inside the force kernel of a rebuild step.  Measured
// on config C (protocol x0.1, same box): fused -1.8 % anneal alone, but with the
// prefetching force kernel its 80 VGPRs spill and the pair is +2.4 %; the unfused
// engine with the prefetch is -2 %, so 0 is the default.
#define IGM_POP_FUSED 0
#endif
constexpr bool kPopFused = IGM_POP_FUSED != 0;
#ifndef IGM_POP_OUTER_CAP
#define IGM_POP_OUTER_CAP 80
#endif
constexpr int kPopOuterCap = IGM_POP_OUTER_CAP;  // outer-list entries per slot (two-level lists)
#ifndef IGM_POP_TYPE_STAGE
#define IGM_POP_TYPE_STAGE 512  // bond types a force block stages in LDS (4 KB); 0: always gathered
#endif
constexpr int kPopTypeStage = IGM_POP_TYPE_STAGE > 0 ? IGM_POP_TYPE_STAGE : 1;
#ifndef IGM_POP_QX
#define IGM_POP_QX 1
#endif
// x cells of the build grid per cut_list.  2 (half-width x cells, 5-cell runs) was 1 % faster
// in one-group kernel traces (fill -1 %, force -1.3 %) but 1 % slower in the bench's two-group
// anneal (profiles/r05_ab), so cubic cells stay the default.
constexpr int kPopQx = IGM_POP_QX;
constexpr int kPopListRow = kPopRowCap + 2;  // u16 per LDS list row of the build (odd word stride)
// index of cell (cx, cy, cz) in the slot order of a grid of nb[3] cells: x-fastest.
// (Measured on config C, pop=1000: bricks of 2^3 or 4^3 cells -- 64 or 256 consecutive
// slots a compact blob instead of a rod along x -- were 12 % and 13 % SLOWER, profiles/history_r01_r04.md.)
__device__ __forceinline__ int pop_cell_of(int cx, int cy, int cz, const int* nb) {
    return (cz * nb[1] + cy) * nb[0] + cx;
}
__host__ __device__ __forceinline__ int pop_ncell(const int* nb) { return nb[0] * nb[1] * nb[2]; }
// the cell coordinates of a position (clamped into the grid, as cell_index)
__device__ __forceinline__ void pop_cell_xyz(float x, float y, float z, const float* lo, const float* inv,
                                             const int* nb, int& cx, int& cy, int& cz) {
    const float pp[3] = {x, y, z};
    int ci[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const int v = (int)((pp[d] - lo[d]) * inv[d]);
        ci[d] = v < 0 ? 0 : (v >= nb[d] ? nb[d] - 1 : v);
    }
    cx = ci[0];
    cy = ci[1];
    cz = ci[2];
}
__device__ __forceinline__ int pop_cell_index(float x, float y, float z, const float* lo, const float* inv,
                                              const int* nb) {
    int cx, cy, cz;
    pop_cell_xyz(x, y, z, lo, inv, nb, cx, cy, cz);
    return pop_cell_of(cx, cy, cz, nb);
}
// The slot runs of the cells around (cx, cy, cz) that can hold a slot within cut_list:
// per (y, z) row of the 3 x 3 rows the x-run of cells cx - reach .. cx + reach (nb[3]:
// the x cells span cut_list / qx, so reach <= qx), one contiguous slot range (rows
// outside the grid are empty).  cell[] holds the first slot of every cell (and the end
// of the last one).
__device__ __forceinline__ void pop_runs(int cx, int cy, int cz, const int* cell, const int* nb, int (&rb)[9],
                                         int (&re)[9]) {
    const int nx = nb[0], ny = nb[1], nz = nb[2], R = nb[3];
    const int xlo = cx > R ? cx - R : 0, xhi = cx + R < nx ? cx + R : nx - 1;
#pragma unroll
    for (int r = 0; r < 9; ++r) {
        const int z0 = cz + r / 3 - 1, y0 = cy + r % 3 - 1;
        const bool ok = z0 >= 0 && z0 < nz && y0 >= 0 && y0 < ny;
        const int rw = ok ? (z0 * ny + y0) * nx : 0;
        rb[r] = ok ? cell[rw + xlo] : 0;
        re[r] = ok ? cell[rw + xhi + 1] : 0;
    }
}

// a packed f32 triple (12 bytes, 4-byte aligned: one dwordx3 access per lane; a wave's
// 64 consecutive triples are 768 contiguous bytes) -- the per-slot state nobody gathers
// (forces, build positions) carries no fourth word to stream
struct __attribute__((aligned(4))) pop_f3 {
    float x, y, z;
};

struct PopBuf {
    float4* pos;   // (B, ldn): x, y, z, w = radius (bead) or -(radius + 1)
    pop_f3* vel;   // (B, ldn)
    pop_f3* frc;   // (B, ldn)
    int* aid;      // (B, ldn) atom id of a slot
    int* slot;     // (B, ldn) slot of an atom id
    uint8_t* flg;  // (B, ldn) the atom flags (every IGM_ATOM_* bit is below 0x100)
};

struct PopArgs {
    Common cm;
    DevParams P;
    PopBuf buf[2];
    int* par;            // (B) buffer holding the current slot order
    pop_f3* xb;          // (B, ldn) position of the slot at its list build
    uint2* nl;           // (B, nslice, kq, 64) Verlet list: quads of u16 slot ids, padded with the own slot
    uint16_t* nnb;       // (B, ldn) list length, or kNnbWalk
    int* cell;           // (B, kPopCells) first slot of every cell of the build grid
    int ccap;            // cells per grid of this run (<= kPopCellCap; pop_sort_cells)
    float* gp;           // (B, 8) grid lo[3], inv[3]
    int* gn;             // (B, 8) grid nb[3], x reach in cells of cut_list
    int qx;              // x cells per cut_list: x cells of >= cut_list / qx (runs reach gn[3] x cells each way)
    // bonds of a slot, by buffer parity (as the state): partner slot | type << 16 | lower << 31
    uint32_t* bentb[2];  // (B, nslice, bdmax, 64)
    uint16_t* bdegb[2];  // (B, ldn)
    // bond pruning (null: off): the slot's bonds that may act before the next list build, in
    // the same layout and order, and their count -- written by the permute at every build
    uint32_t* bc;        // (B, nslice, bdmax, 64)
    uint16_t* bcn;       // (B, ldn)
    int* bpr;            // (B) the structure's last build pruned (1) or kept every bond (0)
    int* bage;           // (B) steps its lists have served since their build (the force kernel counts)
    int prune_age;       // a build prunes when the lists it replaces served at least this many steps
    // the slot order change of a list build (the sort writes both): new slot -> old slot,
    // old slot -> new slot; the permute moves a slot's state and bonds by them, bond
    // partners re-indexed old slot -> new slot (slot-space reads near the slot, instead
    // of the atom-space adjacency rows, which lie scattered by atom id)
    int* inv;            // (B, ldn)
    int* remap;          // (B, ldn)
    int bdmax;
    int kq;              // list quads per slot (4 kq >= the Verlet-list capacity)
    int* flag[2];        // (B) list rebuild needed, by step parity (the force kernel clears the next step's)
    int* flist;          // (B) the flagged structures of this step, compacted
    int* nflag;          // (1)
    int* nrebuild;       // (B)
    double* kep;         // (B, nbs) per-block kinetic-energy partials (2x KE, mass 1)
    float* bbp;          // (B, nbs, 6) per-block bounding boxes {max -x, -y, -z, max x, y, z}
    const double* dofs;  // (B) dof of group nonfixed
    int nbs;
    // the bonds of every atom as contiguous rows (CSR, the sliced ELLPACK of prepare()
    // re-laid out once per run): the rebuild's re-index gathers atoms in slot order,
    // where one row is one cache line instead of one line per entry
    const uint32_t* csr;  // entries: partner atom | type << 16 | lower << 31
    const int* coff;      // (B, natom + 1) row offsets within the structure
    const int64_t* cbase;  // (B) first entry of the structure
    // Two-level lists (two != 0): the cell grid, the slot order and the OUTER list
    // (cut_list = cut_in + the outer margin) are rebuilt only when an atom moved past
    // half the margin since the last outer build; the inner list (cut_in, the list
    // the force kernel reads) is re-filtered from the outer one at every other rebuild.
    int two;
    float cut_in;        // inner list cut (two-level), P.cut_list is then the outer one
    float4* xo;          // (B, ldn) position of the slot at the last outer build
    uint2* nlo;          // (B, nslice, kqo, 64) outer list quads
    uint16_t* nnbo;      // (B, ldn) outer list length, or kNnbWalk
    int kqo;
    int* oflag[2];       // (B) outer margin exceeded, by step parity
    int* flist2;         // (B) the structures whose inner list is rebuilt this step
    int* nflag2;         // (1)
    unsigned long long* sprof;  // optional (8): the sort kernel's phase cycles, summed (profiling)
    // The split sort (pop_grid .. pop_rank, several 256-thread workgroups per flagged
    // structure instead of one 1024-thread workgroup holding the grid in LDS):
    int* ccnt;           // (B, kPopCntStride) cell counts; zero between builds (the scan clears them)
    int* tid;            // (B, ldn) atom ids scattered into their cells (before the in-cell rank)
    int* ctot;           // (B, 8) cells counted per scan chunk (zero between builds: the scatter clears them)
};

// one Verlet list of the engine (the inner one, or the outer one of two-level lists)
struct PopList {
    uint2* nl;
    uint16_t* nnb;
    int kq;
};

// XCD-aware block order for the kernels over every structure: the grid (padded to a
// multiple of 8) is dealt round-robin over the 8 XCDs, so logical block
// (x % 8) * (grid / 8) + x / 8 keeps the blocks of a structure on one XCD and its
// positions and lists in that XCD's L2.
__device__ __forceinline__ int pop_block() {
    const int x = blockIdx.x, per = gridDim.x >> 3;
    return (x & 7) * per + (x >> 3);
}

// CSR row offsets of every structure's bonds (one workgroup per structure): the
// exclusive scan of the atom degrees, the structure's total at coff[natom]
__global__ void __launch_bounds__(1024) pop_csr_scan_kernel(const int* deg, int natom, int* coff) {
    __shared__ int wsum[1024 / 64];
    const int s = blockIdx.x;
    block_scan<1024, int, int>(deg + (size_t)s * natom, coff + (size_t)s * (natom + 1), natom, wsum);
}

// the entries of every atom's row from the sliced ELLPACK adjacency
__global__ void __launch_bounds__(256) pop_csr_fill_kernel(Bonds Bd, int nstruct, int natom, int nslice,
                                                            const int* coff, const int64_t* cbase, uint32_t* csr) {
    const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (x >= (int64_t)nstruct * natom) return;
    const int s = (int)(x / natom), a = (int)(x - (int64_t)s * natom);
    const int deg = Bd.deg[x];
    const uint32_t* g = Bd.ent + Bd.base[s] + Bd.soff[(size_t)s * (nslice + 1) + (a >> 6)] + (a & 63);
    uint32_t* o = csr + cbase[s] + coff[(size_t)s * (natom + 1) + a];
    for (int e = 0; e < deg; ++e) o[e] = g[(size_t)e * 64];
}

__global__ void __launch_bounds__(kPopBS) pop_load_kernel(PopArgs A, const float* xyz) {
    const int lb = pop_block(), s = lb / A.nbs, a = (lb % A.nbs) * kPopBS + threadIdx.x;
    if (s >= A.cm.nstruct) return;
    if (lb == 0 && threadIdx.x == 0) {
        *A.nflag = 0;
        if (A.two) *A.nflag2 = 0;
    }
    if (a == 0) {
        A.flag[0][s] = 1;  // the first step builds
        A.flag[1][s] = 0;
        A.oflag[0][s] = 1;
        A.oflag[1][s] = 0;
        A.nrebuild[s] = 0;
        A.par[s] = 0;
    }
    if (a >= A.cm.natom) return;
    const size_t i = (size_t)s * A.cm.ldn + a;
    const float* x = xyz + ((size_t)s * A.cm.natom + a) * 3;
    const uint32_t fl = A.cm.aflags[(size_t)s * A.cm.afs + a];
    const float r = A.cm.radii[a];
    const PopBuf& B = A.buf[0];
    {  // the bonds in the identity slot order (parity 0): the sliced adjacency of prepare()
        const int deg = A.cm.bonds.deg[(size_t)s * A.cm.natom + a];
        const uint32_t* g = A.cm.bonds.ent + A.cm.bonds.base[s] +
                            A.cm.bonds.soff[(size_t)s * (A.cm.nslice + 1) + (a >> 6)] + (a & 63);
        uint32_t* d = A.bentb[0] + ((size_t)s * A.cm.nslice + (a >> 6)) * A.bdmax * 64 + (a & 63);
        for (int e = 0; e < deg; ++e) d[(size_t)e * 64] = g[(size_t)e * 64];
        A.bdegb[0][i] = (uint16_t)deg;
    }
    B.pos[i] = make_float4(x[0], x[1], x[2], (fl & IGM_ATOM_BEAD) ? r : -(r + 1.0f));
    B.vel[i] = pop_f3{0.f, 0.f, 0.f};
    B.flg[i] = (uint8_t)fl;
    B.frc[i] = pop_f3{0.f, 0.f, 0.f};
    B.aid[i] = a;
    B.slot[i] = a;
    const float inf = __int_as_float(0x7f800000);
    A.xb[i] = pop_f3{inf, inf, inf};
    if (A.two) A.xo[i] = make_float4(inf, inf, inf, 0.f);
}

// velocities of a run: 'velocity create' of segment seg (vsrc = vinit + seg stride) or
// given, in atom order
__global__ void __launch_bounds__(kPopBS) pop_setvel_kernel(PopArgs A, const float* vsrc, size_t sstride) {
    const int lb = pop_block(), s = lb / A.nbs, i = (lb % A.nbs) * kPopBS + threadIdx.x;
    if (s >= A.cm.nstruct || i >= A.cm.natom) return;
    const PopBuf& B = A.buf[A.par[s]];
    const size_t k = (size_t)s * A.cm.ldn + i;
    const float* v = vsrc + (size_t)s * sstride + (size_t)B.aid[k] * 3;
    B.vel[k] = (B.flg[k] & IGM_ATOM_FIXED) ? pop_f3{0.f, 0.f, 0.f} : pop_f3{v[0], v[1], v[2]};
}

struct PopStep {
    float dtv, dtf, vlim, vlimsq, trig;
    float trig_out;   // two-level lists: (outer margin / 2)^2
    int integrate;    // 0: neighbour check only (run setup)
    int rescale;      // apply the temp/rescale of step `prev` first
    int prev, nsteps;
    float t0, t1, window, fraction;
    int fp;           // parity of this step's rebuild flags
    int part;         // force kernel: 0 every structure, 1 those not rebuilt this step, 2 those rebuilt
};

// temp/rescale factor of structure s at the end of step P.prev (fixed-order sum of partials)
// (wave 0 loads the partials in parallel and adds them in a fixed tree: every block
// gets the same bits, and no block waits on a serial chain of nbs loads)
__device__ __forceinline__ float pop_factor(const PopArgs& A, const PopStep& S, int s, float* shared) {
    if (threadIdx.x < 64) {
        const double* kp = A.kep + (size_t)s * A.nbs;
        double ke = 0.0;
        for (int i = threadIdx.x; i < A.nbs; i += 64) ke += kp[i];
        ke = wave_sum_f64(ke);
        if (threadIdx.x == 0)
            *shared = temp_rescale_factor(ke, A.dofs[s], S.prev, S.nsteps, S.t0, S.t1, S.window, S.fraction);
    }
    __syncthreads();
    return *shared;
}

// [end_of_step rescale of the previous step] + initial_integrate + the displacement check
__global__ void __launch_bounds__(kPopBS) pop_integrate_kernel(PopArgs A, PopStep S) {
    __shared__ float fac;
    __shared__ float red[kPopBS / 64 * 6];
    const int lb = pop_block(), s = lb / A.nbs, i = (lb % A.nbs) * kPopBS + threadIdx.x;
    if (s >= A.cm.nstruct) return;
    const PopBuf& B = A.buf[A.par[s]];
    // the slot's state is loaded before the rescale factor's block reduction, so the
    // loads are in flight while wave 0 sums the KE partials
    const bool live = i < A.cm.natom;
    const size_t k = (size_t)s * A.cm.ldn + (live ? i : 0);
    float4 p = B.pos[k];
    pop_f3 v = B.vel[k];
    const uint32_t fl = B.flg[k];
    const pop_f3 f = B.frc[k];
    const pop_f3 b = A.xb[k];
    const float4 bo = A.two ? A.xo[k] : make_float4(b.x, b.y, b.z, 0.f);
    const float factor = S.rescale ? pop_factor(A, S, s, &fac) : 1.0f;
    int moved = 0, moved_o = 0;
    float mm[6] = {-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f};
    if (live) {
        if (S.integrate && !(fl & IGM_ATOM_FIXED)) {
            // the final_integrate half-kick of the previous step: the force kernel only
            // stores the force (its kinetic-energy partial used the same kicked velocity),
            // so the kick is redone here, bit for bit, instead of storing v in between
            if (S.rescale) kick_limit(v.x, v.y, v.z, f.x, f.y, f.z, S.dtf, S.vlim, S.vlimsq);
            v.x *= factor;
            v.y *= factor;
            v.z *= factor;
            kick_limit(v.x, v.y, v.z, f.x, f.y, f.z, S.dtf, S.vlim, S.vlimsq);
            p.x += S.dtv * v.x;
            p.y += S.dtv * v.y;
            p.z += S.dtv * v.z;
            B.vel[k] = v;
            B.pos[k] = p;
        }
        if (p.w >= 0.0f) {
            const float dx = p.x - b.x, dy = p.y - b.y, dz = p.z - b.z;
            moved = !(dx * dx + dy * dy + dz * dz <= S.trig);
            const float ox = p.x - bo.x, oy = p.y - bo.y, oz = p.z - bo.z;
            moved_o = !(ox * ox + oy * oy + oz * oz <= S.trig_out);
            mm[0] = -p.x;
            mm[1] = -p.y;
            mm[2] = -p.z;
            mm[3] = p.x;
            mm[4] = p.y;
            mm[5] = p.z;
        }
    }
    // this block's bounding box of the beads (for a list build of the structure)
#pragma unroll
    for (int d = 0; d < 6; ++d)
        mm[d] = wave_max_f32(mm[d]);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int d = 0; d < 6; ++d) red[(threadIdx.x >> 6) * 6 + d] = mm[d];
    if (__syncthreads_or(moved) && threadIdx.x == 0) atomicOr(&A.flag[S.fp][s], 1);
    if (A.two && __syncthreads_or(moved_o) && threadIdx.x == 0) atomicOr(&A.oflag[S.fp][s], 1);
    if (threadIdx.x < 6) {
        float m = red[threadIdx.x];
#pragma unroll
        for (int w = 1; w < kPopBS / 64; ++w) m = fmaxf(m, red[w * 6 + threadIdx.x]);
        A.bbp[((size_t)s * A.nbs + lb % A.nbs) * 6 + threadIdx.x] = m;
    }
}

// The cell grid of build_nlist for structure s from its bead bounding box mm = {max -x,
// -y, -z, max x, y, z}: cells of side cs >= cut_list in y and z, cs / qx in x (the sort
// order is x-fastest, so an x run of cells stays one slot range, and a slot's list build
// visits only the x cells its cut_list sphere meets in each row), at most A.ccap cells.
// Stored to gp (lo[3], inv[3]) and gn (nb[3], x reach); sg/sn get lo, inv and nb.
__device__ __forceinline__ void pop_grid_of(const PopArgs& A, int s, const float (&mm)[6], float* sg, int* sn,
                                            bool store = true) {
    float ext[3], vol = 1.0f;
    const float cut = A.P.cut_list;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        ext[d] = mm[3 + d] + mm[d];
        if (!(ext[d] >= 0.0f)) ext[d] = 0.0f;
        vol *= fmaxf(ext[d], cut);
    }
    float cs = cut;
    const float cap = (float)A.ccap, qx = (float)A.qx;
    if (vol * qx / (cs * cs * cs) > cap) cs = cbrtf(vol * qx / cap) * 1.0001f;
    float* gp = A.gp + (size_t)s * 8;
    int* gn = A.gn + (size_t)s * 8;
    int nbv[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        nbv[d] = (int)floorf(d == 0 ? ext[d] * qx / cs : ext[d] / cs);
        if (nbv[d] < 1) nbv[d] = 1;
    }
    // x cells a pair within cut_list can be apart (the cell walk's x reach)
    if (store) gn[3] = ext[0] > 0.0f ? max(1, (int)ceilf(cut * (float)nbv[0] / ext[0] * 1.00001f)) : 1;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const int nbd = nbv[d];
        sg[d] = -mm[d];
        sg[3 + d] = ext[d] > 0.0f ? (float)nbd / ext[d] : 0.0f;
        sn[d] = nbd;
        if (store) {
            gp[d] = sg[d];
            gp[3 + d] = sg[3 + d];
            gn[d] = nbd;
        }
    }
}

// One workgroup per flagged structure: the cell grid of build_nlist (cells of side >=
// cut_list, at most kPopCellCap) from the bbox partials, then a counting sort of the
// slots into it -- cell counts as packed u16 pairs in LDS, and with IDS_LDS the new
// order of atom ids too (u16), so the ranks, the scan and the per-cell insertion
// sort (ascending ids: deterministic) never leave the CU.  Non-bead atoms form a last
// run after the real cells.  Writes the new slot order (aid, slot) and the cell
// offsets, and flips the structure's parity.
//   APT > 0: every thread keeps the (cell, rank) of its APT atoms (t + u * kPopSortNT,
// N <= APT * kPopSortNT) in registers, and all their loads are in flight together --
// the sort is one workgroup's chain of dependent memory round trips, so fewer and
// wider trips are what makes it faster.
#ifndef IGM_POP_SORT_PROF
#define IGM_POP_SORT_PROF 0  // 1: per-phase cycle counters of the sort (with IGM_POP_SORT_PROF set at run time)
#endif
template <bool IDS_LDS, int APT>
__global__ void __launch_bounds__(kPopSortNT) pop_sort_kernel(PopArgs A, int fp) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cw[];  // (kPopCells + 1) / 2 words, then ids
    __shared__ int wsum[kMaxWaves];
    __shared__ float sg[6];
    __shared__ int sn[3];
    const int s = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (!A.flag[fp][s]) return;
#if IGM_POP_SORT_PROF
    unsigned long long tp = A.sprof ? clock64() : 0;
    auto phase = [&](int k) {  // profiling builds: thread 0 charges the cycles since the last mark
        if (A.sprof && t == 0) {
            const unsigned long long now = clock64();
            atomicAdd(&A.sprof[k], now - tp);
            tp = now;
        }
    };
#else
    auto phase = [](int) {};
#endif
    if (A.two) {  // every rebuild re-filters the inner list; the outer one waits for its margin
        if (t == 0) A.flist2[atomicAdd(A.nflag2, 1)] = s;
        if (!A.oflag[fp][s]) return;
    }
    const int N = A.cm.natom;
    const size_t base = (size_t)s * A.cm.ldn;
    const int p = A.par[s], q = p ^ 1;
    const float4* pos = A.buf[p].pos + base;
    const int* aido = A.buf[p].aid + base;
    int* aidn = A.buf[q].aid + base;
    int* slotn = A.buf[q].slot + base;  // first the packed (cell, rank) of every old slot
    __shared__ float smm[6];
    if (w < 6) {  // the structure's bbox from the blocks' partials, one wave per component
        const float* bp = A.bbp + (size_t)s * A.nbs * 6;
        float m = -3.0e38f;
        for (int b = lane; b < A.nbs; b += 64) m = fmaxf(m, bp[b * 6 + w]);
        m = wave_max_f32(m);
        if (lane == 0) smm[w] = m;
    }
    __syncthreads();
    if (t == 0) {
        A.flist[atomicAdd(A.nflag, 1)] = s;
        float mm[6];
#pragma unroll
        for (int d = 0; d < 6; ++d) mm[d] = smm[d];
        pop_grid_of(A, s, mm, sg, sn);
    }
    __syncthreads();
    const float lo[3] = {sg[0], sg[1], sg[2]}, inv[3] = {sg[3], sg[4], sg[5]};
    const int nb[3] = {sn[0], sn[1], sn[2]};
    const int ncell = pop_ncell(nb);
    const int nw = (ncell + 3) >> 1;  // words holding the cells 0..ncell+1
    uint16_t* ids = reinterpret_cast<uint16_t*>(cw + ((A.ccap + 3) >> 1));
    for (int k = t; k < nw; k += kPopSortNT) cw[k] = 0u;
    __syncthreads();
    phase(0);  // grid from the bbox partials, counts cleared
    constexpr int U = 4;  // independent loads in flight per thread
    uint32_t cr[APT > 0 ? APT : 1];
    if constexpr (APT > 0) {
#pragma unroll
        for (int u0 = 0; u0 < APT; u0 += 8) {
            float4 pp[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = t + (u0 + u) * kPopSortNT;
                pp[u] = pos[i < N ? i : 0];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = t + (u0 + u) * kPopSortNT;
                if (u0 + u < APT && i < N) {
                    const int c = pp[u].w >= 0.0f ? pop_cell_index(pp[u].x, pp[u].y, pp[u].z, lo, inv, nb) : ncell;
                    const uint32_t sh = (uint32_t)(c & 1) << 4;
                    const uint32_t old = atomicAdd(&cw[c >> 1], 1u << sh);
                    cr[u0 + u] = ((uint32_t)c << 16) | ((old >> sh) & 0xffffu);
                }
            }
        }
    } else
    for (int i0 = t; i0 < N; i0 += U * kPopSortNT) {
        float4 pp[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * kPopSortNT;
            pp[u] = pos[i < N ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * kPopSortNT;
            if (i >= N) break;
            const int c = pp[u].w >= 0.0f ? pop_cell_index(pp[u].x, pp[u].y, pp[u].z, lo, inv, nb) : ncell;
            const uint32_t sh = (uint32_t)(c & 1) << 4;
            const uint32_t old = atomicAdd(&cw[c >> 1], 1u << sh);
            slotn[i] = (int)(((uint32_t)c << 16) | ((old >> sh) & 0xffffu));
        }
    }
    __syncthreads();
    phase(1);  // positions loaded, cells counted
    // exclusive scan of the u16 counts in place (offsets <= N < 65536 fit the halves)
    {
        const int cpt = (nw + kPopSortNT - 1) / kPopSortNT, k0 = t * cpt;
        uint32_t sum = 0;
        for (int k = k0; k < k0 + cpt && k < nw; ++k) sum += (cw[k] & 0xffffu) + (cw[k] >> 16);
        uint32_t incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[w] = (int)incl;
        __syncthreads();
        uint32_t run = incl - sum;
        for (int i = 0; i < w; ++i) run += (uint32_t)wsum[i];
        for (int k = k0; k < k0 + cpt && k < nw; ++k) {
            const uint32_t v = cw[k], lo16 = run, hi16 = run + (v & 0xffffu);
            run = hi16 + (v >> 16);
            cw[k] = lo16 | (hi16 << 16);
        }
    }
    __syncthreads();
    phase(2);  // scan
    auto off = [&](int c) -> int { return (int)((cw[c >> 1] >> ((c & 1) << 4)) & 0xffffu); };
    auto put = [&](int k, int v) {
        if (IDS_LDS)
            ids[k] = (uint16_t)v;
        else
            aidn[k] = v;
    };
    auto get = [&](int k) -> int { return IDS_LDS ? (int)ids[k] : aidn[k]; };
    if constexpr (APT > 0) {
#pragma unroll
        for (int u0 = 0; u0 < APT; u0 += 16) {
            int aa[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int i = t + (u0 + u) * kPopSortNT;
                aa[u] = aido[i < N ? i : 0];
            }
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (u0 + u < APT && t + (u0 + u) * kPopSortNT < N)
                    put(off((int)(cr[u0 + u] >> 16)) + (int)(cr[u0 + u] & 0xffffu), aa[u]);
        }
    } else
    for (int i0 = t; i0 < N; i0 += U * kPopSortNT) {
        uint32_t uu[U];
        int aa[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * kPopSortNT < N ? i0 + u * kPopSortNT : 0;
            uu[u] = (uint32_t)slotn[i];
            aa[u] = aido[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * kPopSortNT < N) put(off((int)(uu[u] >> 16)) + (int)(uu[u] & 0xffffu), aa[u]);
    }
    __syncthreads();
    phase(3);  // ids scattered into their cells
    if constexpr (APT > 0) {
        // deterministic order inside a cell: an atom's slot is its cell's first slot plus
        // the number of the cell's atoms with a smaller id (independent LDS reads per
        // atom, where an insertion sort per cell is a serial chain of them).  (Measured,
        // IGM_POP_SORT_PROF: this phase is ~half of the kernel; keeping slot and id in
        // registers for coalesced stores after a barrier was 2.5 % slower on the anneal.)
#pragma unroll
        for (int u = 0; u < APT; ++u) {
            if (t + u * kPopSortNT >= N) continue;
            const int c = (int)(cr[u] >> 16), beg = off(c), end = off(c + 1);
            const int a = get(beg + (int)(cr[u] & 0xffffu));
            int r = 0;
            for (int k = beg; k < end; ++k) r += get(k) < a ? 1 : 0;
            aidn[beg + r] = a;
            slotn[a] = beg + r;
            A.remap[base + t + u * kPopSortNT] = beg + r;  // (old slot t + u * kPopSortNT)
            A.inv[base + beg + r] = t + u * kPopSortNT;
        }
    } else {
        for (int c = t; c <= ncell; c += kPopSortNT) {  // deterministic order inside a cell
            const int beg = off(c), end = off(c + 1);
            for (int i = beg + 1; i < end; ++i) {
                const int v = get(i);
                int k = i - 1;
                while (k >= beg && get(k) > v) {
                    put(k + 1, get(k));
                    --k;
                }
                put(k + 1, v);
            }
        }
        __syncthreads();
        const int* slot_old = A.buf[p].slot + base;
        for (int i = t; i < N; i += kPopSortNT) {
            const int a = get(i);
            if (IDS_LDS) aidn[i] = a;
            slotn[a] = i;
            const int o = slot_old[a];
            A.remap[base + o] = i;
            A.inv[base + i] = o;
        }
    }
    phase(4);  // ranks inside the cells, new slot order stored
    int* cg = A.cell + (size_t)s * kPopCells;
    for (int c = t; c <= ncell + 1; c += kPopSortNT) cg[c] = off(c);
    if (t == 0) A.par[s] = q;
#if IGM_POP_SORT_PROF
    if (A.sprof) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (profiling: this wave's stores done)
        phase(5);  // cell offsets stored
        if (t == 0) atomicAdd(&A.sprof[6], 1ull);
    }
#endif
}

// LDS bytes of pop_sort_kernel<IDS_LDS> over grids of at most ccap cells
__host__ __device__ inline size_t pop_sort_lds(bool ids_lds, int natom, int ccap) {
    return sizeof(uint32_t) * ((ccap + 3) / 2) + (ids_lds ? sizeof(uint16_t) * (size_t)natom : 0);
}

// the grid cap of a run: kPopCellCap when the ids fit beside its counts in LDS, else the
// largest cap (>= kCellCapBig) that keeps them there, else kPopCellCap with HBM ids
inline int pop_sort_cells(int natom) {
    if (pop_sort_lds(true, natom, kPopCellCap) <= kLdsBytes) return kPopCellCap;
    const long long room = ((long long)kLdsBytes - 2LL * natom) / 2 - 4;
    if (room >= kCellCapBig) return (int)(room & ~63LL);
    return kPopCellCap;
}
static_assert(kPopCells < 65536, "cell ids are packed in 16 bits");

// ---- The split sort: the same slot order as pop_sort_kernel (same grid, same cells, ids
// ascending inside a cell), built by several workgroups per flagged structure with the
// counts and ids in HBM/L2 instead of one CU's LDS (pop_sort_kernel holds 124 KB of LDS
// for ~200 us per flagged structure, which keeps the other structure group's kernels off
// that CU, profiles/r05_ab).
//   pop_count    every slot of every flagged structure: the grid (each block from the bbox
//                partials; block 0 stores it and the flist entry), the slot's cell, its
//                arrival rank there (global atomic), key = c << 16 | rank; chunk totals
//   pop_scan     per flagged structure and chunk of kScanChunk cells: cell offsets
//                (exclusive scan from the chunk totals before it), counts cleared, parity flipped
//   pop_scatter  per slot: its atom id at its cell's first slot + arrival rank
//   pop_rank     per slot: new slot = cell's first slot + ids of the cell below its own
// The arrival ranks differ run to run; the in-cell order (ascending ids) does not.
// The kernels after pop_count run a grid of `per` structure slots x nbs blocks, and block
// b takes flagged structures b / nbs, + per, ... (*nflag of them).
constexpr int kScanLog = 13, kScanChunk = 1 << kScanLog, kScanChunks = 8;  // 8 x 8192 >= kPopCells
static_assert(kScanChunk * kScanChunks >= kPopCells, "the scan chunks cover every cell");

__global__ void __launch_bounds__(kPopBS) pop_count_kernel(PopArgs A, int fp) {
    __shared__ float sgl[6];
    __shared__ int snb[3], scc[kScanChunks];
    const int s = blockIdx.x / A.nbs, blk = blockIdx.x % A.nbs, t = threadIdx.x, i = blk * kPopBS + t;
    if (s >= A.cm.nstruct || !A.flag[fp][s]) return;  // (block-uniform)
    if (t < kScanChunks) scc[t] = 0;
    if (t < 64) {  // the structure's bead bbox from the blocks' partials (max: exact in any order)
        const float* bp = A.bbp + (size_t)s * A.nbs * 6;
        float mm[6];
#pragma unroll
        for (int d = 0; d < 6; ++d) mm[d] = -3.0e38f;
        for (int b = t; b < A.nbs; b += 64)
#pragma unroll
            for (int d = 0; d < 6; ++d) mm[d] = fmaxf(mm[d], bp[b * 6 + d]);
#pragma unroll
        for (int d = 0; d < 6; ++d) mm[d] = wave_max_f32(mm[d]);
        if (t == 0) {
            float sg[6];
            int sn[3];
            pop_grid_of(A, s, mm, sg, sn, blk == 0);
            if (blk == 0) A.flist[atomicAdd(A.nflag, 1)] = s;
#pragma unroll
            for (int d = 0; d < 6; ++d) sgl[d] = sg[d];
#pragma unroll
            for (int d = 0; d < 3; ++d) snb[d] = sn[d];
        }
    }
    __syncthreads();
    if (i < A.cm.natom) {
        const float lo[3] = {sgl[0], sgl[1], sgl[2]}, inv[3] = {sgl[3], sgl[4], sgl[5]};
        const int nb[3] = {snb[0], snb[1], snb[2]};
        const size_t base = (size_t)s * A.cm.ldn;
        const float4 p = A.buf[A.par[s]].pos[base + i];
        const int c = p.w >= 0.0f ? pop_cell_index(p.x, p.y, p.z, lo, inv, nb) : pop_ncell(nb);
        const int r = atomicAdd(A.ccnt + (size_t)s * kPopCntStride + c, 1);
        atomicAdd(&scc[c >> kScanLog], 1);  // (the chunk totals: one global add per block and chunk,
        A.remap[base + i] = (c << 16) | r;   // not per slot -- a few words take every slot's add)
    }
    __syncthreads();
    if (t < kScanChunks && scc[t]) atomicAdd(A.ctot + (size_t)s * kScanChunks + t, scc[t]);
}

// exclusive scan of the counts of cells 0..ncell (the last one the non-bead run) into the
// cell offsets (cell[ncell + 1] = N): one workgroup per (flagged structure, chunk of
// kScanChunk cells), 8 cells per thread, the chunk's base from the chunk totals before it;
// the counts cleared behind
template <int NT>
__global__ void __launch_bounds__(NT) pop_scan_kernel(PopArgs A) {
    static_assert(8 * NT == kScanChunk, "one tile per chunk");
    __shared__ int wsum[NT / 64];
    const int nf = *A.nflag, t = threadIdx.x, lane = t & 63, w = t >> 6, ch = blockIdx.x % kScanChunks;
    for (int k = blockIdx.x / kScanChunks; k < nf; k += gridDim.x / kScanChunks) {
        const int s = A.flist[k];
        const int* gn = A.gn + (size_t)s * 8;
        const int n = gn[0] * gn[1] * gn[2] + 1;  // cells and the non-bead run
        const int c0 = ch * kScanChunk;
        if (c0 >= n) continue;  // (block-uniform)
        const int* ct = A.ctot + (size_t)s * kScanChunks;
        int run = 0;
        for (int q = 0; q < ch; ++q) run += ct[q];
        int4* cnt = reinterpret_cast<int4*>(A.ccnt + (size_t)s * kPopCntStride);
        int* cg = A.cell + (size_t)s * kPopCells;
        const int c = c0 + 8 * t;
        int4 a = make_int4(0, 0, 0, 0), b = make_int4(0, 0, 0, 0);
        if (c < n) {  // (the stride rounds the rows to 4: c + 4 < kPopCntStride)
            a = cnt[c >> 2];
            b = c + 4 < n ? cnt[(c >> 2) + 1] : make_int4(0, 0, 0, 0);
        }
        const int v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        int sum = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) sum += v[u];
        int incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        int ex = run + incl - sum, tile = 0;
        for (int q = 0; q < NT / 64; ++q) {
            ex += q < w ? wsum[q] : 0;
            tile += wsum[q];
        }
        if (c < n) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (c + u < n) cg[c + u] = ex;
                ex += v[u];
            }
            const int4 z = make_int4(0, 0, 0, 0);
            cnt[c >> 2] = z;
            if (c + 4 < n) cnt[(c >> 2) + 1] = z;
        }
        if (t == 0) {
            if (c0 + kScanChunk >= n) cg[n] = run + tile;  // = N (the chunk holding the last cell)
            if (ch == 0) A.par[s] ^= 1;  // the slot order being built is the other buffer's
        }
        __syncthreads();  // (wsum reused by the next structure)
    }
}

__global__ void __launch_bounds__(kPopBS) pop_scatter_kernel(PopArgs A) {
    const int nf = *A.nflag, per = gridDim.x / A.nbs, i = (blockIdx.x % A.nbs) * kPopBS + threadIdx.x;
    if (i >= A.cm.natom) return;
    for (int k = blockIdx.x / A.nbs; k < nf; k += per) {
        const int s = A.flist[k];
        if (i < kScanChunks) A.ctot[(size_t)s * kScanChunks + i] = 0;  // (read by the scan launch before)
        const size_t base = (size_t)s * A.cm.ldn;
        const uint32_t key = (uint32_t)A.remap[base + i];
        const int* cg = A.cell + (size_t)s * kPopCells;
        A.tid[base + cg[key >> 16] + (key & 0xffffu)] = A.buf[A.par[s] ^ 1].aid[base + i];
    }
}

__global__ void __launch_bounds__(kPopBS) pop_rank_kernel(PopArgs A) {
    const int nf = *A.nflag, per = gridDim.x / A.nbs, i = (blockIdx.x % A.nbs) * kPopBS + threadIdx.x;
    if (i >= A.cm.natom) return;
    for (int k = blockIdx.x / A.nbs; k < nf; k += per) {
        const int s = A.flist[k];
        const size_t base = (size_t)s * A.cm.ldn;
        const uint32_t key = (uint32_t)A.remap[base + i];
        const int c = (int)(key >> 16);
        const int* cg = A.cell + (size_t)s * kPopCells;
        const int beg = cg[c], end = cg[c + 1];
        const int q = A.par[s], a = A.buf[q ^ 1].aid[base + i];
        const int* id = A.tid + base;
        int r = 0;
        for (int j = beg; j < end; ++j) r += id[j] < a ? 1 : 0;
        const int n = beg + r;
        A.buf[q].aid[base + n] = a;
        A.buf[q].slot[base + a] = n;
        A.remap[base + i] = n;  // (old slot i -> new slot)
        A.inv[base + n] = i;
    }
}

// state (and with BONDS the bonds; the fused force kernel re-indexes them itself) of
// every slot of a flagged structure into its new slot order: block b works on flagged
// structure b / nbs (plain order: the working blocks are dealt over all XCDs)
template <bool BONDS>
__device__ __forceinline__ void pop_permute_slot(const PopArgs& A, int s, int i);
template <bool BONDS>
__global__ void __launch_bounds__(kPopBS) pop_permute_kernel(PopArgs A) {
    const int k = blockIdx.x / A.nbs, i = (blockIdx.x % A.nbs) * kPopBS + threadIdx.x;
    if (k >= *A.nflag || i >= A.cm.natom) return;  // (idle blocks: the structure was not flagged)
    pop_permute_slot<BONDS>(A, A.flist[k], i);
}
template <bool BONDS>
__device__ __forceinline__ void pop_permute_slot(const PopArgs& A, int s, int i) {
    const size_t base = (size_t)s * A.cm.ldn, k = base + i;
    const int q = A.par[s], p = q ^ 1;
    const PopBuf &O = A.buf[p], &B = A.buf[q];
    const int o = A.inv[k];  // the slot's old slot
    const float4 x = O.pos[base + o];
    B.pos[k] = x;
    B.vel[k] = O.vel[base + o];
    B.flg[k] = O.flg[base + o];
    // (no force: the force kernel of this step rewrites every slot's before any read)
    A.xb[k] = pop_f3{x.x, x.y, x.z};
    if (A.two) A.xo[k] = make_float4(x.x, x.y, x.z, 0.f);
    if (!BONDS) return;
    // the old slot's bonds, partners re-indexed old slot -> new slot
    const int nsl = A.cm.nslice;
    const int deg = A.bdegb[p][base + o];
    const uint32_t* g = A.bentb[p] + ((size_t)s * nsl + (o >> 6)) * A.bdmax * 64 + (o & 63);
    uint32_t* d = A.bentb[q] + ((size_t)s * nsl + (i >> 6)) * A.bdmax * 64 + (i & 63);
    const int* rm = A.remap + base;
    const bool prune = A.bc && A.bage[s] >= A.prune_age;
    if (A.bc && i == 0) A.bpr[s] = prune ? 1 : 0;
    if (prune) {
        // Bond pruning: between builds every bead stays within skin/2 of its build position
        // (the integrate's trigger), so a bead-bead distance moves by less than skin.  An
        // upper bound whose build distance is below r0 - skin (a lower bound: above r0 + skin)
        // adds exactly 0 until the next build; the candidates keep the entry order, so the
        // force sums are bitwise those of the whole list.  1 % of the skin covers the f32
        // rounding; bonds of non-bead atoms (not watched by the trigger) stay candidates.
        uint32_t* dc = A.bc + ((size_t)s * nsl + (i >> 6)) * A.bdmax * 64 + (i & 63);
        const float2* bt = A.cm.bonds.types + A.cm.bonds.tbase[s];
        const float dsk = 1.01f * A.P.skin;
        int nc = 0;
        for (int e0 = 0; e0 < deg; e0 += 4) {  // 4 entries, then their new slots and old positions
            uint32_t v[4];
            int t[4];
            float4 pj[4];
            float2 ct[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = g[(size_t)min(e0 + u, deg - 1) * 64];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                t[u] = rm[v[u] & 0xffffu];
                pj[u] = O.pos[base + (v[u] & 0xffffu)];
                ct[u] = bt[(v[u] >> 16) & 0x7fffu];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (e0 + u >= deg) continue;
                const uint32_t e = (v[u] & 0xffff0000u) | (uint32_t)t[u];
                d[(size_t)(e0 + u) * 64] = e;
                const float dx = x.x - pj[u].x, dy = x.y - pj[u].y, dz = x.z - pj[u].z;
                const float r = __builtin_sqrtf(dx * dx + dy * dy + dz * dz);
                const bool idle = x.w >= 0.0f && pj[u].w >= 0.0f &&
                                  ((v[u] & kLowerBit) ? r - dsk > ct[u].x : r + dsk < ct[u].x);
                if (!idle) dc[(size_t)nc++ * 64] = e;
            }
        }
        A.bcn[k] = (uint16_t)nc;
    } else {
        for (int e0 = 0; e0 < deg; e0 += 4) {  // 4 entries, then their 4 new slots, in flight together
            uint32_t v[4];
            int t[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = g[(size_t)min(e0 + u, deg - 1) * 64];
#pragma unroll
            for (int u = 0; u < 4; ++u) t[u] = rm[v[u] & 0xffffu];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (e0 + u < deg) d[(size_t)(e0 + u) * 64] = (v[u] & 0xffff0000u) | (uint32_t)t[u];
        }
    }
    A.bdegb[q][k] = (uint16_t)deg;
}


typedef float pop_f2 __attribute__((ext_vector_type(2)));

// slot j of a structure's float4 array through a buffer resource: a 32-bit offset and
// no 64-bit address arithmetic per gather.  The array is the same for the whole wave
// (one structure per block); readfirstlane says so, or every load becomes a waterfall.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pop_rsrc(const float4* p, int n) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* u = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(u, (short)0, __builtin_amdgcn_readfirstlane(n * 16), 0x00020000);
}
__device__ __forceinline__ float3 pop_ld3(__amdgpu_buffer_rsrc_t r, uint32_t j) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, j * 16u, 0, 0);
    return make_float3(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]));
}
__device__ __forceinline__ float4 pop_ld(__amdgpu_buffer_rsrc_t r, uint32_t j) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, j * 16u, 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}

// The Verlet list of bead slot i of structure s (p0 its position): collected in the
// thread's LDS row `row` (kPopListRow u16), padded to whole quads with the slot itself,
// stored as quads to the global list and its length (or kNnbWalk) to nnb.  Returns
// the number of entries (> kcap: the slot takes its pairs from the cell walk).
//   FLUSH: the row (rowcap entries) is stored and emptied whenever it holds flush_at
// entries, so the list may be longer than the row (the fused force kernel reads its
// list from the row: no flush, the list capacity capped at the row's).
template <bool FLUSH>
__device__ __forceinline__ int pop_fill_slot(const PopArgs& A, const PopList& T, int s, int i, size_t base,
                                             const float4* pos, float4 p0, uint32_t* row, int rowcap) {
    const float* gp = A.gp + (size_t)s * 8;
    const int* gn = A.gn + (size_t)s * 8;
    const int* cell = A.cell + (size_t)s * kPopCells;
    const int kcap = FLUSH ? 4 * T.kq : min(4 * T.kq, rowcap & ~3);
    uint16_t* lst = reinterpret_cast<uint16_t*>(row);
    uint64_t* out = reinterpret_cast<uint64_t*>(T.nl + ((size_t)s * A.cm.nslice + (i >> 6)) * T.kq * 64 + (i & 63));
    const float cut2 = A.P.cut_list * A.P.cut_list;
    // k: entries found; kr: entries in the row; qo: quads stored.  A flush check follows
    // every group of at most 8 tests, so the row never holds more than flush_at + 7.
    static_assert(kFillW <= 8 && kFillTail <= 8, "a test group must fit the row's slack");
    const int flush_at = (rowcap - 8) & ~3;
    int k = 0, kr = 0, qo = 0;
    auto flush = [&]() {
        if (FLUSH && kr >= flush_at) {
#pragma unroll 1
            for (int q = 0; q < (flush_at >> 2); ++q)
                out[(size_t)(qo + q) * 64] = ((uint64_t)row[2 * q + 1] << 32) | row[2 * q];
            qo += flush_at >> 2;
#pragma unroll 1
            for (int e = flush_at; e < kr; ++e) lst[e - flush_at] = lst[e];
            kr -= flush_at;
        }
    };
    // The 3 x 3 rows' x-runs of cells (cx - reach .. cx + reach, pop_runs) are 9 slot
    // ranges.  All 18 run bounds are loaded together,
    // then each z-layer's 3 runs a batch of kFillW slots per run at once, the rest of a
    // longer run kFillTail slots at a time (the hot runs' lists reach 3.4 rmax: ~10
    // candidates per run; one dependent load per candidate there was +2 % anneal).
    int cx, cy, cz;
    pop_cell_xyz(p0.x, p0.y, p0.z, gp, gp + 3, gn, cx, cy, cz);
    constexpr int RL = 3, FW = kFillW;  // runs per z-layer, slots per run and batch
    int rb[9], re[9];
    pop_runs(cx, cy, cz, cell, gn, rb, re);
    const __amdgpu_buffer_rsrc_t rp = pop_rsrc(pos, A.cm.natom);
    auto test = [&](int j, const float3& p) {
        const float ddx = p0.x - p.x, ddy = p0.y - p.y, ddz = p0.z - p.z;
        const bool in = j != i && ddx * ddx + ddy * ddy + ddz * ddz < cut2;
        if (in && k < kcap) lst[kr++] = (uint16_t)j;
        k += in ? 1 : 0;
    };
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        float3 pp[RL][FW];
        int jj[RL][FW];
#pragma unroll
        for (int r = 0; r < RL; ++r)
#pragma unroll
            for (int u = 0; u < FW; ++u) {
                const int j = rb[RL * g + r] + u;
                jj[r][u] = j < re[RL * g + r] ? j : i;  // past the run: the slot itself (never listed)
                pp[r][u] = pop_ld3(rp, jj[r][u]);
            }
#pragma unroll
        for (int r = 0; r < RL; ++r) {
#pragma unroll
            for (int u = 0; u < FW; ++u) test(jj[r][u], pp[r][u]);
            flush();
            // the rest of a longer run, kFillTail loads in flight at a time (the slot itself
            // past the run's end: never listed)
            const int e = re[RL * g + r];
            for (int j0 = rb[RL * g + r] + FW; j0 < e; j0 += kFillTail) {
                float3 pt[kFillTail];
                int jt[kFillTail];
#pragma unroll
                for (int u = 0; u < kFillTail; ++u) {
                    jt[u] = j0 + u < e ? j0 + u : i;
                    pt[u] = pop_ld3(rp, jt[u]);
                }
#pragma unroll
                for (int u = 0; u < kFillTail; ++u) test(jt[u], pt[u]);
                flush();
            }
        }
    }
    // the last quad padded with the slot itself: a zero-distance entry adds no force
    if (k <= kcap) {
        for (int kk = kr; kk & 3; ++kk) lst[kk] = (uint16_t)i;
#pragma unroll 1
        for (int q = 0; q < (kr + 3) >> 2; ++q)
            out[(size_t)(qo + q) * 64] = ((uint64_t)row[2 * q + 1] << 32) | row[2 * q];
    }
    T.nnb[base + i] = (uint16_t)(k <= kcap ? k : kNnbWalk);
    return k;
}

// Verlet list of every bead slot of a flagged structure (the unfused engine): the 27
// cells around its cell, each x-run of cells one contiguous slot range.  Measured on
// config C (kernel traces, scripts/gpu_profab.sh): collecting the list in an LDS row
// and storing it a quad at a time is 13 % faster than one global u16 store per entry;
// batches of 4 slots per run beat 2 and 6.  Staging positions in LDS does not pay,
// neither the block's whole neighbourhood range (~50 KB, 18 % slower) nor the union of
// the slots its lists use (lists rewritten to union indices: this kernel +58 %, the
// force kernel +9 %).
//   One block per (flagged structure, slot block): the grid covers every structure of the
// group and the blocks past *nflag exit (a loop over the flagged structures in a smaller grid
// costs the kernel 8 VGPRs: 74, 6 waves per SIMD instead of 7, profiles/r06_ab).
template <int ROW>
__global__ void __launch_bounds__(kPopBS) pop_fill_kernel(PopArgs A) {
    __shared__ uint32_t lrow[kPopBS * ROW / 2];
    const int kb = blockIdx.x / A.nbs;
    if (kb >= *A.nflag) return;  // an idle block (the structure was not flagged)
    const int s = A.flist[kb], blk = blockIdx.x % A.nbs, t = threadIdx.x, i = blk * kPopBS + t;
    const size_t base = (size_t)s * A.cm.ldn;
    const float4* pos = A.buf[A.par[s]].pos + base;
    if (i >= A.cm.natom) return;
    const float4 p0 = pos[i];
    const PopList T = A.two ? PopList{A.nlo, A.nnbo, A.kqo} : PopList{A.nl, A.nnb, A.kq};
    if (p0.w >= 0.0f)
        pop_fill_slot<true>(A, T, s, i, base, pos, p0, lrow + t * (ROW / 2), ROW - 2);
    else
        T.nnb[base + i] = 0;
}

// Two-level lists: the inner Verlet list (cut_in) of every slot of a structure whose
// inner list is rebuilt this step, filtered from its outer list (no cell walk, no new
// slot order); a slot whose outer list overflowed keeps the cell walk.  Same output
// format as pop_fill_slot (quads of slot ids in the list's order, the last one padded
// with the slot itself).
__global__ void __launch_bounds__(kPopBS) pop_refilter_kernel(PopArgs A) {
    __shared__ uint32_t lrow[kPopBS * kPopListRow / 2];
    const int kb = blockIdx.x / A.nbs;
    if (kb >= *A.nflag2) return;
    const int s = A.flist2[kb], t = threadIdx.x, i = (blockIdx.x % A.nbs) * kPopBS + t;
    if (i >= A.cm.natom) return;
    const size_t base = (size_t)s * A.cm.ldn;
    const float4* pos = A.buf[A.par[s]].pos + base;
    const float4 p0 = pos[i];
    A.xb[base + i] = pop_f3{p0.x, p0.y, p0.z};  // the inner build position
    if (!(p0.w >= 0.0f)) {
        A.nnb[base + i] = 0;
        return;
    }
    const int no = A.nnbo[base + i];
    if (no == kNnbWalk) {
        A.nnb[base + i] = kNnbWalk;
        return;
    }
    uint32_t* row = lrow + t * (kPopListRow / 2);
    uint16_t* lst = reinterpret_cast<uint16_t*>(row);
    const int kcap = min(4 * A.kq, kPopRowCap & ~3);  // (the list collects in the LDS row)
    const float cut2 = A.cut_in * A.cut_in;
    const __amdgpu_buffer_rsrc_t rp = pop_rsrc(pos, A.cm.natom);
    const uint2* go = A.nlo + ((size_t)s * A.cm.nslice + (i >> 6)) * A.kqo * 64 + (i & 63);
    int k = 0;
    auto test = [&](uint32_t j) {
        const float3 p = pop_ld3(rp, j);
        const float dx = p0.x - p.x, dy = p0.y - p.y, dz = p0.z - p.z;
        const bool in = j != (uint32_t)i && dx * dx + dy * dy + dz * dz < cut2;  // (the padding is the slot)
        if (in && k < kcap) lst[k] = (uint16_t)j;
        k += in ? 1 : 0;
    };
    const int nq = (no + 3) >> 2;
    for (int q0 = 0; q0 < nq; q0 += 2) {  // two quads (8 candidates) in flight
        const uint2 e0 = go[(size_t)q0 * 64];
        const uint2 e1 = q0 + 1 < nq ? go[(size_t)(q0 + 1) * 64] : make_uint2(i * 0x10001u, i * 0x10001u);
        test(e0.x & 0xffffu);
        test(e0.x >> 16);
        test(e0.y & 0xffffu);
        test(e0.y >> 16);
        test(e1.x & 0xffffu);
        test(e1.x >> 16);
        test(e1.y & 0xffffu);
        test(e1.y >> 16);
    }
    for (int kk = k; kk < kcap && (kk & 3); ++kk) lst[kk] = (uint16_t)i;
    const int nlist = k <= kcap ? ((k + 3) & ~3) : 0;
    if (nlist > 0) {
        uint64_t* out = reinterpret_cast<uint64_t*>(A.nl + ((size_t)s * A.cm.nslice + (i >> 6)) * A.kq * 64 + (i & 63));
#pragma unroll 1
        for (int q = 0; q < nlist >> 2; ++q) out[(size_t)q * 64] = ((uint64_t)row[2 * q + 1] << 32) | row[2 * q];
    }
    A.nnb[base + i] = (uint16_t)(k <= kcap ? k : kNnbWalk);
}

// pair forces of a slot past the Verlet-list capacity: the 27 cells of the build-time
// grid (a superset of its list, visited in slot order).  Out of line, with plain
// arguments, so the rare path costs the hot force kernel no registers.
__device__ __noinline__ float4 pop_walk_pairs(const float4* pos, const int* cell, const float* gp, const int* gn,
                                              float bx, float by, float bz, int i, float4 p0, float evfpi) {
    float fx = 0.0f, fy = 0.0f, fz = 0.0f;
    int cx, cy, cz;
    pop_cell_xyz(bx, by, bz, gp, gp + 3, gn, cx, cy, cz);
    int rb[9], re[9];
    pop_runs(cx, cy, cz, cell, gn, rb, re);
    constexpr int W = 4;  // candidates in flight (the slot itself past a run's end: no force)
    for (int r = 0; r < 9; ++r)
        for (int j0 = rb[r]; j0 < re[r]; j0 += W) {
            float4 pw[W];
            int jw[W];
#pragma unroll
            for (int u = 0; u < W; ++u) {
                jw[u] = j0 + u < re[r] ? j0 + u : i;
                pw[u] = pos[jw[u]];
            }
#pragma unroll
            for (int u = 0; u < W; ++u) {
                const float dx = p0.x - pw[u].x, dy = p0.y - pw[u].y, dz = p0.z - pw[u].z;
                const float f = soft_pair_bf(dx * dx + dy * dy + dz * dz, p0.w + pw[u].w, evfpi);
                const float m = jw[u] != i ? f : 0.0f;
                fx += m * dx;
                fy += m * dy;
                fz += m * dz;
            }
        }
    return make_float4(fx, fy, fz, 0.0f);
}

// f32 force on slot i of structure s: the MD force path of atom_force specialised
// for the population engine -- slot-space Verlet list and bonds, hardware rsq/rcp in
// place of the IEEE sqrt/divide expansions, no calls (a call would put the kernel
// arguments in scratch).  Neighbours and bond partners are loaded a batch at a time
// so their gathers are in flight together; a masked tail keeps the batch branch-free.
//   Fused rebuild step (lrow != null): the slot's list was just built into its LDS row
// (nn_built entries) and is read from there; the slot's bonds are re-indexed from the
// atom-space adjacency into the new slot order here (written to bent/bdeg for the
// following steps) and used directly.
__device__ __forceinline__ void pop_slot_force(const PopArgs& A, int s, int i, size_t base, const float4* pos,
                                               uint32_t fl, float evf, float envf, float& fx, float& fy,
                                               float& fz, const IGM_LDS float2* sbt, bool lds_types,
                                               const uint32_t* lrow = nullptr, int nn_built = 0) {
    constexpr int U = kPopPairBatch;  // list quads per batch
    const int nsl = A.cm.nslice;
    const uint2* gl = A.nl + ((size_t)s * nsl + (i >> 6)) * A.kq * 64 + (i & 63);
    // the bonds: the pruned candidates of the last build when the engine keeps them
    const bool pruned = A.bc && A.bpr[s];
    uint32_t* g = (pruned ? A.bc : A.bentb[A.par[s]]) + ((size_t)s * nsl + (i >> 6)) * A.bdmax * 64 + (i & 63);
    const float2* bt = A.cm.bonds.types + A.cm.bonds.tbase[s];
    const __amdgpu_buffer_rsrc_t rp = pop_rsrc(pos, A.cm.natom);
    const float4 p0 = pos[i];
    const float xi = p0.x, yi = p0.y, zi = p0.z, ri = p0.w;
    fx = fy = fz = 0.0f;
    const float evfpi = evf * 0.318309886183790671537767526745f;
    const bool rebuilt = lrow != nullptr;
    const int nn = rebuilt ? (nn_built <= min(4 * A.kq, (kPopListRow - 2) & ~3) ? nn_built : kNnbWalk)
                           : A.nnb[base + i];
    const int* sl = A.buf[A.par[s]].slot + base;
    int a_id = 0;
    const uint32_t* ga = nullptr;  // atom-space adjacency (rebuilt step)
    int deg;
    if (rebuilt) {
        a_id = A.buf[A.par[s]].aid[base + i];
        const int* co = A.coff + (size_t)s * (A.cm.natom + 1);
        const int r0 = co[a_id];
        deg = co[a_id + 1] - r0;
        ga = A.csr + A.cbase[s] + r0;
        A.bdegb[A.par[s]][base + i] = (uint16_t)deg;
    } else {
        deg = pruned ? A.bcn[base + i] : A.bdegb[A.par[s]][base + i];
    }
#if IGM_POP_PREFETCH
    // Latency: the slot's loads, its first list quad and first bond entries go out in
    // one memory round trip (their addresses depend on (s, i) only; slots past the
    // atom's own are clamped into the allocated region and never used).
    uint2 qnext = make_uint2(i * 0x10001u, i * 0x10001u);
    if (!rebuilt) qnext = gl[0];
    constexpr int UB = IGM_POP_BOND_BATCH;
    uint32_t et0[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) et0[u] = rebuilt ? 0u : g[(size_t)min(u, A.bdmax - 1) * 64];
#else
    constexpr int UB = IGM_POP_BOND_BATCH;
#endif
    // Two list entries per packed-f32 op.  With t = 1/(r rc) from ONE rsq,
    //   sin(pi r / rc) = sin_rev(r2 t / 2)   and   evf rc sin / (pi r) = evfpi rc2 t sin,
    // the soft_pair_bf force without the rcp; the 1e-20 keeps a zero distance (the
    // padding entries, which are the slot itself) finite, and it is below one ulp of
    // every r2 that is not zero.
    pop_f2 ax = {0.0f, 0.0f}, ay = {0.0f, 0.0f}, az = {0.0f, 0.0f};
    float bfx = 0.0f, bfy = 0.0f, bfz = 0.0f;  // the bonds' sum
    auto pair2 = [&](const float4& a, const float4& b) {
        const pop_f2 dx = pop_f2{xi, xi} - pop_f2{a.x, b.x}, dy = pop_f2{yi, yi} - pop_f2{a.y, b.y},
                     dz = pop_f2{zi, zi} - pop_f2{a.z, b.z};
        const pop_f2 r2 = dx * dx + dy * dy + dz * dz;
        const pop_f2 rc = pop_f2{ri, ri} + pop_f2{a.w, b.w};
        const pop_f2 rc2 = rc * rc;
        const pop_f2 q = (r2 + 1.0e-20f) * rc2;
        const pop_f2 t = {__builtin_amdgcn_rsqf(q.x), __builtin_amdgcn_rsqf(q.y)};
        const pop_f2 h = (0.5f * r2) * t;
        const pop_f2 sn = {__builtin_amdgcn_sinf(h.x), __builtin_amdgcn_sinf(h.y)};
        const pop_f2 f = (evfpi * rc2) * (sn * t);
        const pop_f2 m = {r2.x < rc2.x ? f.x : 0.0f, r2.y < rc2.y ? f.y : 0.0f};
        ax += m * dx;
        ay += m * dy;
        az += m * dz;
    };
    auto bond = [&](const float4& p, float2 c, uint32_t e, bool on) {
        const float dx = xi - p.x, dy = yi - p.y, dz = zi - p.z;
        const float r2 = dx * dx + dy * dy + dz * dz;
        const float rinv = __builtin_amdgcn_rsqf(fmaxf(r2, 1.0e-30f));
        const float dr = r2 * rinv - c.x;
        const bool active = (e & kLowerBit) ? (dr < 0.0f) : (dr > 0.0f);
        const float m = (on && active && r2 > 0.0f) ? -2.0f * c.y * dr * rinv : 0.0f;
        bfx += m * dx;
        bfy += m * dy;
        bfz += m * dz;
    };
    if (ri >= 0.0f) {
        if (nn == kNnbWalk) {
            // the walk covers the cells around the position of the grid's build (with
            // two-level lists the outer build: the cells hold the slots of that build)
            const float4 b = A.two ? A.xo[base + i]
                                   : make_float4(A.xb[base + i].x, A.xb[base + i].y, A.xb[base + i].z, 0.f);
            const float4 f = pop_walk_pairs(pos, A.cell + (size_t)s * kPopCells, A.gp + (size_t)s * 8,
                                            A.gn + (size_t)s * 8, b.x, b.y, b.z, i, p0, evfpi);
            fx = f.x;
            fy = f.y;
            fz = f.z;
        } else {
            const int nq = (nn + 3) >> 2;
            auto pairs = [&](auto fetch) {
#if IGM_POP_PREFETCH
                // one quad at a time, the next QD quads' loads in flight with this one's gathers
                constexpr int QD = IGM_POP_QDEPTH;
                uint2 qb[QD];
                qb[0] = qnext;
#pragma unroll
                for (int d = 1; d < QD; ++d) {
                    qb[d] = make_uint2(i * 0x10001u, i * 0x10001u);
                    if (!rebuilt && nq > d) qb[d] = gl[(size_t)d * 64];
                }
                for (int q = 0; q < nq; ++q) {
                    const uint2 e = rebuilt ? make_uint2(lrow[2 * q], lrow[2 * q + 1]) : qb[0];
#pragma unroll
                    for (int d = 0; d + 1 < QD; ++d) qb[d] = qb[d + 1];
                    if (!rebuilt && q + QD < nq) qb[QD - 1] = gl[(size_t)(q + QD) * 64];
                    const float4 a0 = fetch(e.x & 0xffffu), a1 = fetch(e.x >> 16), a2 = fetch(e.y & 0xffffu),
                                 a3 = fetch(e.y >> 16);
                    pair2(a0, a1);
                    pair2(a2, a3);
                }
                return;
#endif
                for (int q0 = 0; q0 < nq; q0 += U) {
                    uint2 e[U];  // a quad past the list: the slot itself 4 times (no force)
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        e[u] = q0 + u >= nq ? make_uint2(i * 0x10001u, i * 0x10001u)
                               : rebuilt    ? make_uint2(lrow[2 * (q0 + u)], lrow[2 * (q0 + u) + 1])
                                            : gl[(size_t)(q0 + u) * 64];
                    float4 pt[4 * U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        pt[4 * u + 0] = fetch(e[u].x & 0xffffu);
                        pt[4 * u + 1] = fetch(e[u].x >> 16);
                        pt[4 * u + 2] = fetch(e[u].y & 0xffffu);
                        pt[4 * u + 3] = fetch(e[u].y >> 16);
                    }
#pragma unroll
                    for (int u = 0; u < 2 * U; ++u) pair2(pt[2 * u], pt[2 * u + 1]);
                }
            };
            pairs([&](uint32_t j) { return pop_ld(rp, j); });
            fx = ax.x + ax.y;
            fy = ay.x + ay.y;
            fz = az.x + az.y;
        }
    }
    for (int k0 = 0; k0 < deg; k0 += UB) {
        uint32_t et[UB];
        if (rebuilt) {  // atom-space entries -> slot-space (the permute of the unfused engine)
#pragma unroll
            for (int u = 0; u < UB; ++u) et[u] = ga[min(k0 + u, deg - 1)];
            int sv[UB];
#pragma unroll
            for (int u = 0; u < UB; ++u) sv[u] = sl[et[u] & 0xffffu];
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                et[u] = (et[u] & 0xffff0000u) | (uint32_t)sv[u];
                if (k0 + u < deg) g[(size_t)(k0 + u) * 64] = et[u];
            }
        } else {
#if IGM_POP_PREFETCH
            if (k0 == 0) {
#pragma unroll
                for (int u = 0; u < UB; ++u) et[u] = u < deg ? et0[u] : et0[0];  // (past deg: a valid entry)
            } else
#endif
#pragma unroll
            for (int u = 0; u < UB; ++u) et[u] = g[(size_t)min(k0 + u, deg - 1) * 64];
        }
        float4 pt[UB];
        float2 ct[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            pt[u] = pop_ld(rp, et[u] & 0xffffu);
            ct[u] = lds_types ? sbt[(et[u] >> 16) & 0x7fffu] : bt[(et[u] >> 16) & 0x7fffu];
        }
#pragma unroll
        for (int u = 0; u < UB; ++u) bond(pt[u], ct[u], et[u], k0 + u < deg);
    }
    fx += bfx;
    fy += bfy;
    fz += bfz;
    // envelopes (non-bead atoms carry -(radius + 1))
    const float rad = ri >= 0.0f ? ri : -ri - 1.0f;
    for (int e = 0; e < A.P.nenv; ++e) {
        if (!(fl & (IGM_ATOM_ENV0 << e))) continue;
        if (A.P.env_kind[e] == IGM_ENV_VOLUME) {
            double en = 0.0;
            volume_term<float, false>(xi, yi, zi, A.P.vmaps[A.P.vsmap ? A.P.vsmap[s] : 0], A.P.vvox, envf,
                                      A.P.env_k[e], fx, fy, fz, en);
            continue;
        }
        const float k = A.P.env_k[e];
        const float sx = A.P.env_abc[e][0] * envf - rad, sy = A.P.env_abc[e][1] * envf - rad,
                    sz = A.P.env_abc[e][2] * envf - rad;
        const float ix = __builtin_amdgcn_rcpf(sx * sx), iy = __builtin_amdgcn_rcpf(sy * sy),
                    iz = __builtin_amdgcn_rcpf(sz * sz);
        const float k2 = xi * xi * ix + yi * yi * iy + zi * zi * iz;
        const bool active = (k > 0.0f) ? (k2 > 1.0f) : (k2 < 1.0f && k2 > 0.0f);
        if (!active) continue;
        const float r2 = xi * xi + yi * yi + zi * zi;
        const float rinv = __builtin_amdgcn_rsqf(r2), rsk = __builtin_amdgcn_rsqf(k2);
        const float rn = r2 * rinv;
        const float t = (1.0f - rsk) * rn;
        const float ca = (1.0f - rsk) * rinv, cb = rn * rsk * __builtin_amdgcn_rcpf(k2);
        const float ka = fabsf(k);
        fx -= ka * t * (ca * xi + cb * xi * ix);
        fy -= ka * t * (ca * yi + cb * yi * iy);
        fz -= ka * t * (ca * zi + cb * zi * iz);
    }
    if (fl & IGM_ATOM_FIXED) fx = fy = fz = 0.0f;  // fix setforce 0 (lammps.py:222-223)
}

// forces of every slot (+ final_integrate and this block's kinetic-energy partial
// when S.integrate; the run's setup evaluation otherwise).  (Measured on config C: a
// block running the pairs and the bonds of its slots in separate waves at the same
// time is 6 % slower than one thread per slot doing both.)
//   FUSED: a structure whose list is rebuilt this step builds it here, a slot per
// thread (pop_fill_slot into the thread's LDS row), and takes this step's pairs from
// that row and its bonds from the atom-space adjacency (pop_slot_force's rebuilt
// path): no fill launch, no list or bond re-read on rebuild steps.  Every cross-slot
// input (the new slot order, cell offsets and positions) was written by the sort and
// permute kernels before this launch.
//   (Block windows staged in LDS, every neighbour inside them an LDS read instead of a
// gather: round 5 with window-form lists, round 6 with the slot -> window mapping in this
// kernel -- both slower on config C, profiles/r05_ab and profiles/r06_ab.)
template <bool FUSED>
__global__ void __launch_bounds__(kPopBS, IGM_POP_FORCE_OCC) pop_force_kernel(PopArgs A, float evf, float envf, PopStep S) {
    __shared__ double red[kPopBS / 64];
    __shared__ uint32_t lrow[FUSED ? kPopBS * kPopListRow / 2 : 1];
    const int lb = pop_block(), s = lb / A.nbs, blk = lb % A.nbs, i = blk * kPopBS + threadIdx.x;
    if (s >= A.cm.nstruct) return;
    // the build kernels of this step are done (part 1 runs beside them: it leaves the counters)
    if (S.part != 1 && blockIdx.x == 0 && threadIdx.x == 0) {
        *A.nflag = 0;
        if (A.two) *A.nflag2 = 0;
    }
    const int rebuilt = A.flag[S.fp][s];  // the structure's list is (was) rebuilt this step
    if ((S.part == 1 && rebuilt) || (S.part == 2 && !rebuilt)) return;  // (block-uniform)
    if (i == 0) {
        A.nrebuild[s] += rebuilt ? 1 : 0;
        if (A.bc) A.bage[s] = rebuilt ? 0 : A.bage[s] + 1;
        A.flag[S.fp ^ 1][s] = 0;  // the next step's flags start clear
        A.oflag[S.fp ^ 1][s] = 0;
    }
    const size_t base = (size_t)s * A.cm.ldn, k = base + i;
    const PopBuf& B = A.buf[A.par[s]];
    // the structure's bond types (r0, k) staged in LDS when they fit: a bond's type is then an
    // LDS read, not one more gather through the texture path (which bounds this kernel)
    __shared__ float2 sbt[kPopTypeStage];
    const int64_t ntyp = A.cm.bonds.ntype[s];
    const bool lds_types = IGM_POP_TYPE_STAGE > 0 && ntyp <= kPopTypeStage;
    if (lds_types) {
        const float2* bt = A.cm.bonds.types + A.cm.bonds.tbase[s];
        for (int q = threadIdx.x; q < (int)ntyp; q += kPopBS) sbt[q] = bt[q];
    }
    __syncthreads();
    double ke = 0.0;
    if (i < A.cm.natom) {
        pop_f3 v = B.vel[k];
        const uint32_t fl = B.flg[k];
        float fx, fy, fz;
        if (FUSED && rebuilt) {
            uint32_t* row = lrow + threadIdx.x * (kPopListRow / 2);
            const float4 p0 = B.pos[k];
            int nb = 0;
            if (p0.w >= 0.0f)
                nb = pop_fill_slot<false>(A, PopList{A.nl, A.nnb, A.kq}, s, i, base, B.pos + base, p0, row,
                                          kPopListRow - 2);
            else
                A.nnb[k] = 0;
            pop_slot_force(A, s, i, base, B.pos + base, fl, evf, envf, fx, fy, fz, (const IGM_LDS float2*)sbt, lds_types, row, nb);
        } else {
            pop_slot_force(A, s, i, base, B.pos + base, fl, evf, envf, fx, fy, fz, (const IGM_LDS float2*)sbt, lds_types);
        }
        B.frc[k] = pop_f3{fx, fy, fz};
        if (S.integrate && !(fl & IGM_ATOM_FIXED)) {
            // final_integrate for the temperature only: the kicked velocity is not stored
            // (the next integrate, or the run's finish, redoes the kick from v and f)
            kick_limit(v.x, v.y, v.z, fx, fy, fz, S.dtf, S.vlim, S.vlimsq);
            ke = (double)(v.x * v.x) + (double)(v.y * v.y) + (double)(v.z * v.z);
        }
    }
    if (!S.integrate) return;
    ke = wave_sum_f64(ke);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ke;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < kPopBS / 64; ++w) t += red[w];
        A.kep[(size_t)s * A.nbs + blk] = t;
    }
}

// end of a run: the last step's rescale, then (optionally) the outputs in atom order
__global__ void __launch_bounds__(kPopBS) pop_finish_kernel(PopArgs A, PopStep S, float* xyz, float* vel,
                                                            float* forces_out) {
    __shared__ float fac;
    const int lb = pop_block(), s = lb / A.nbs, i = (lb % A.nbs) * kPopBS + threadIdx.x;
    if (s >= A.cm.nstruct) return;
    const float factor = S.rescale ? pop_factor(A, S, s, &fac) : 1.0f;
    if (i >= A.cm.natom) return;
    const PopBuf& B = A.buf[A.par[s]];
    const size_t k = (size_t)s * A.cm.ldn + i;
    pop_f3 v = B.vel[k];
    if (S.rescale && !(B.flg[k] & IGM_ATOM_FIXED)) {  // the last step's final_integrate
        const pop_f3 f = B.frc[k];
        kick_limit(v.x, v.y, v.z, f.x, f.y, f.z, S.dtf, S.vlim, S.vlimsq);
    }
    v.x *= factor;
    v.y *= factor;
    v.z *= factor;
    B.vel[k] = v;
    if (!xyz) return;  // more runs follow
    const size_t a = (size_t)s * A.cm.natom + B.aid[k];
    const float4 p = B.pos[k];
    xyz[a * 3] = p.x;
    xyz[a * 3 + 1] = p.y;
    xyz[a * 3 + 2] = p.z;
    vel[a * 3] = v.x;
    vel[a * 3 + 1] = v.y;
    vel[a * 3 + 2] = v.z;
    if (forces_out) {
        const pop_f3 f = B.frc[k];
        forces_out[a * 3] = f.x;
        forces_out[a * 3 + 1] = f.y;
        forces_out[a * 3 + 2] = f.z;
    }
}

// Tuning diagnostic (IGM_POP_STATS): per run, the Verlet-list and bond-degree shape the
// force kernel sees after a step -- slots, sum of list lengths (and squares), sum over
// waves of the wave's longest list in quads (a wave runs to its longest list), walks,
// bond degrees (the pruned candidates when the engine prunes) and the waves' longest.  Never launched in a measured run.
__global__ void __launch_bounds__(kPopBS) pop_stats_kernel(PopArgs A, unsigned long long* st) {
    const int lb = pop_block(), s = lb / A.nbs, i = (lb % A.nbs) * kPopBS + threadIdx.x;
    if (s >= A.cm.nstruct) return;
    const size_t base = (size_t)s * A.cm.ldn;
    const bool live = i < A.cm.natom && A.buf[A.par[s]].pos[base + (i < A.cm.natom ? i : 0)].w >= 0.0f;
    int nn = live ? A.nnb[base + i] : 0;
    const int walk = nn == kNnbWalk ? 1 : 0;
    if (walk) nn = 0;
    const bool pruned = A.bc && A.bpr[s];
    const int deg = live ? (pruned ? A.bcn[base + i] : A.bdegb[A.par[s]][base + i]) : 0;  // (the bonds visited)
    int mq = (nn + 3) >> 2, md = deg;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        mq = max(mq, __shfl_xor(mq, off));
        md = max(md, __shfl_xor(md, off));
    }
    unsigned long long v[8] = {live ? 1ull : 0ull, (unsigned long long)nn, (unsigned long long)(nn * nn),
                               (unsigned long long)walk, (unsigned long long)deg, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
    if ((threadIdx.x & 63) == 0) {
        for (int k = 0; k < 5; ++k) atomicAdd(&st[k], v[k]);
        atomicAdd(&st[5], (unsigned long long)mq);
        atomicAdd(&st[6], (unsigned long long)md);
        atomicAdd(&st[7], 1ull);
    }
    if (live && !walk) atomicMax(&st[8], (unsigned long long)nn);
    // the slot window of the block: every list entry of its slots (and the slots)
    __shared__ int wlo, whi, nin;
    if (threadIdx.x == 0) {
        wlo = 1 << 30;
        whi = -1;
        nin = 0;
    }
    __syncthreads();
    int lo = i < A.cm.natom ? i : (1 << 30), hi = i < A.cm.natom ? i : -1;
    const uint2* gl = A.nl + ((size_t)s * A.cm.nslice + (i >> 6)) * A.kq * 64 + (i & 63);
    for (int q = 0; q < (nn + 3) >> 2; ++q) {
        const uint2 e = gl[(size_t)q * 64];
        const int j4[4] = {(int)(e.x & 0xffffu), (int)(e.x >> 16), (int)(e.y & 0xffffu), (int)(e.y >> 16)};
        for (int u = 0; u < 4; ++u) {
            lo = min(lo, j4[u]);
            hi = max(hi, j4[u]);
        }
    }
    atomicMin(&wlo, lo);
    atomicMax(&whi, hi);
    __syncthreads();
    const uint32_t* g = (pruned ? A.bc : A.bentb[A.par[s]]) + ((size_t)s * A.cm.nslice + (i >> 6)) * A.bdmax * 64 +
                        (i & 63);
    int in = 0;
    for (int e = 0; e < deg; ++e) {
        const int j = (int)(g[(size_t)e * 64] & 0xffffu);
        in += (j >= wlo && j <= whi) ? 1 : 0;
    }
    atomicAdd(&nin, in);
    __syncthreads();
    if (threadIdx.x == 0 && whi >= 0) {
        const int span = whi - wlo + 1;
        atomicAdd(&st[9], (unsigned long long)span);
        atomicAdd(&st[10], 1ull);
        atomicMax(&st[11], (unsigned long long)span);
        atomicAdd(&st[12], span > 2048 ? 1ull : 0ull);
        atomicAdd(&st[13], span > 3072 ? 1ull : 0ull);
        atomicAdd(&st[14], span > 4096 ? 1ull : 0ull);
        atomicAdd(&st[15], (unsigned long long)nin);
    }
}

// every structure of the engine rebuilds its list at the next step (a run whose Verlet
// skin differs from the last build's)
__global__ void pop_flag_all_kernel(PopArgs A, int fp) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < A.cm.nstruct) {
        A.flag[fp][s] = 1;
        A.oflag[fp][s] = 1;
    }
}

__global__ void deg_max_kernel(const int* deg, size_t n, int* out) {
    int m = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        m = max(m, deg[i]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
    if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}


// 'velocity nonfixed create T seed' (dist uniform, loop all, mom yes) for every
// structure and segment: RanPark draws in atom-id order, momentum zeroed, scaled
// to T with the group's dof.  grid (nseg, B), one workgroup each.
struct VelArgs {
    int nstruct, natom, nseg;
    const uint32_t* aflags;
    size_t afs;                    // aflags stride between structures (0: shared)
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
    const uint32_t* vfl = V.aflags + (size_t)s * V.afs;
    double s4[4] = {0, 0, 0, 0};
    for (int a = t; a < V.natom; a += 256) {
        if (vfl[a] & IGM_ATOM_FIXED) continue;
#pragma unroll
        for (int d = 0; d < 3; ++d) s4[d] += ranpark_nth(seed, 3ull * a + d + 1) - 0.5;
        s4[3] += 1.0;
    }
    block_sum<256, 4>(s4, red);
    __syncthreads();
    const double nmob = s4[3];
    double t2[1] = {0.0};
    for (int a = t; a < V.natom; a += 256) {
        if (vfl[a] & IGM_ATOM_FIXED) continue;
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
        const bool fixed = vfl[a] & IGM_ATOM_FIXED;
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
    unsigned char* ws;   // per resident workgroup: neighbour structure (+ positions on the HBM path)
    size_t ws_stride;
    double* vec_ws;      // per resident workgroup: F, X0, G, H, XB as [5][3][ldn] doubles
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

// LDS layout of the CG kernel: f64 positions + the cell grid / list index in LDS
// on the LDS path; only the reduction block on the HBM path.
struct CgLds {
    Red r;
    double4* pos;
    int* cell;
    uint16_t* nnb;
    uint16_t* sorted;
    double* gp;
    int* gn;
};

__host__ __device__ inline size_t carve_cg_lds(void* smem, int npad, bool big, CgLds* m) {
    Carver cv(smem);
    m->r = carve_red<double>(cv, &m->gp, &m->gn);
    if (!big) {
        m->pos = cv.take<double4>(npad);
        m->cell = cv.take<int>(kCellCap + 8);
        m->nnb = cv.take<uint16_t>(npad);
        m->sorted = cv.take<uint16_t>(npad);
    }
    return cv.o;
}

template <int NT, bool BIG>
__global__ void __launch_bounds__(NT) cg_kernel(CGArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int t = threadIdx.x, lane = t & 63;
    const int natom = A.cm.natom, ldn = A.cm.ldn;
    CgLds sm;
    carve_cg_lds(smem, ldn, BIG, &sm);
    NList<double, int> L;
    BigWs<double> W;
    carve_ws<double>(A.ws + (size_t)blockIdx.x * A.ws_stride, natom, ldn, A.cm.kcap,
                     BIG ? kCellCapBig : kCellCap, BIG, false, &L, &W);
    L.gp = sm.gp;
    L.gn = sm.gn;
    double4* pos = W.pos;
    if (!BIG) {
        pos = sm.pos;
        L.cell = sm.cell;
        L.nnb = sm.nnb;
        L.sorted = sm.sorted;
    }
    const Red R = sm.r;
    double* F = A.vec_ws + (size_t)blockIdx.x * A.vec_stride;
    double* X0 = F + 3 * (size_t)ldn;
    double* G = X0 + 3 * (size_t)ldn;
    double* H = G + 3 * (size_t)ldn;
    double* XB = H + 3 * (size_t)ldn;
    const double ALPHA_MAX = 1.0, ALPHA_REDUCE = 0.5, BACKTRACK_SLOPE = 0.4, QUADRATIC_TOL = 0.1, EMACH = 1.0e-8,
                 EPS_QUAD = 1.0e-28;
    for (;;) {
        const int s = next_structure(A.cm, R.misc);
        if (s >= A.cm.nstruct) break;
        const float* xs = A.xyz + (size_t)s * natom * 3;
        for (int a = t; a < natom; a += NT) {
            const uint32_t fl = A.cm.aflags[(size_t)s * A.cm.afs + a];
            const double r = (double)A.cm.atype[a];
            pos[a] = make_double4((double)xs[(size_t)a * 3], (double)xs[(size_t)a * 3 + 1],
                                  (double)xs[(size_t)a * 3 + 2], (fl & IGM_ATOM_BEAD) ? r : -(r + 1.0));
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                XB[d * ldn + a] = __longlong_as_double(0x7ff0000000000000LL);
                F[d * ldn + a] = 0.0;
            }
        }
        __syncthreads();
        const uint32_t* adj = A.cm.bonds.ent + A.cm.bonds.base[s];
        const int* soff = A.cm.bonds.soff + (size_t)s * (A.cm.nslice + 1);
        const int* deg = A.cm.bonds.deg + (size_t)s * natom;
        const float2* bt = A.cm.bonds.types + A.cm.bonds.tbase[s];
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
            for (int a = t; a < natom; a += NT) {
                double4 p = pos[a];
                if (a_eval >= 0.0) {  // alpha_step: x = x0 + alpha h
                    p.x = X0[a] + (a_eval > 0.0 ? a_eval * H[a] : 0.0);
                    p.y = X0[ldn + a] + (a_eval > 0.0 ? a_eval * H[ldn + a] : 0.0);
                    p.z = X0[2 * ldn + a] + (a_eval > 0.0 ? a_eval * H[2 * ldn + a] : 0.0);
                    pos[a] = p;
                }
                if (p.w >= 0.0) {
                    const double dx = p.x - XB[a], dy = p.y - XB[ldn + a], dz = p.z - XB[2 * ldn + a];
                    moved |= !(dx * dx + dy * dy + dz * dz <= trig);
                }
            }
            if (a_eval >= 0.0) ++neval;
            if (__syncthreads_or(moved)) {
                build_nlist<double, NT, int>(natom, pos, L, (double)A.P.cut_list, R);
                ++nbuild;
                for (int a = t; a < natom; a += NT) {
                    const double4 p = pos[a];
                    XB[a] = p.x;
                    XB[ldn + a] = p.y;
                    XB[2 * ldn + a] = p.z;
                }
            }
            double vv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int a = t; a < natom; a += NT) {
                double e_e[IGM_MAX_ENVELOPES] = {0, 0, 0, 0};
                double fx, fy, fz;
                const BondView B{adj + soff[a >> 6] + lane, bt, nullptr, nullptr, deg[a]};
                atom_force<double, true, int>(s, a, pos[a], A.cm.aflags[(size_t)s * A.cm.afs + a], pos, L, XB[a], XB[ldn + a],
                                              XB[2 * ldn + a], B, A.P, A.evf, A.envf, fx, fy, fz, vv[0], vv[1], e_e);
                for (int e = 0; e < IGM_MAX_ENVELOPES; ++e) vv[2 + e] += e_e[e];
                F[a] = fx;
                F[ldn + a] = fy;
                F[2 * ldn + a] = fz;
                vv[6] += fx * fx + fy * fy + fz * fz;
                if (phase != PH_SETUP) vv[7] += fx * H[a] + fy * H[ldn + a] + fz * H[2 * ldn + a];
            }
            block_sum<NT, 8>(vv, R.red0);
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
                for (int a = t; a < natom; a += NT)
#pragma unroll
                    for (int d = 0; d < 3; ++d) G[d * ldn + a] = H[d * ldn + a] = F[d * ldn + a];
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
                for (int a = t; a < natom; a += NT)
#pragma unroll
                    for (int d = 0; d < 3; ++d) dd[0] += F[d * ldn + a] * G[d * ldn + a];
                block_sum<NT, 1>(dd, R.red1);
                __syncthreads();
                double beta = fmax(0.0, (ff - dd[0]) / ggv);
                if ((long)(niter + 1) % (3L * natom) == 0) beta = 0.0;
                ggv = ff;
                double gh[1] = {0.0};
                for (int a = t; a < natom; a += NT)
#pragma unroll
                    for (int d = 0; d < 3; ++d) {
                        const double fv = F[d * ldn + a];
                        const double hv = fv + beta * H[d * ldn + a];
                        G[d * ldn + a] = fv;
                        H[d * ldn + a] = hv;
                        gh[0] += fv * hv;
                    }
                block_sum<NT, 1>(gh, R.red1);
                __syncthreads();
                if (gh[0] <= 0.0)
                    for (int a = t; a < natom; a += NT)
#pragma unroll
                        for (int d = 0; d < 3; ++d) H[d * ldn + a] = G[d * ldn + a];
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
            for (int a = t; a < natom; a += NT) {
                const double4 p = pos[a];
                X0[a] = p.x;
                X0[ldn + a] = p.y;
                X0[2 * ldn + a] = p.z;
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    const double hv = H[d * ldn + a];
                    pr[0] += F[d * ldn + a] * hv;
                    hm[0] = fmax(hm[0], fabs(hv));
                }
            }
            block_sum<NT, 1>(pr, R.red1);
            __syncthreads();
            block_max<NT, 1>(hm, R.red0);
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
        for (int a = t; a < natom; a += NT) {
#pragma unroll
            for (int d = 0; d < 3; ++d) fn[0] += F[d * ldn + a] * F[d * ldn + a];
            if (A.vel) {
                const float* vs = A.vel + ((size_t)s * natom + a) * 3;
#pragma unroll
                for (int d = 0; d < 3; ++d) fn[1] += (double)vs[d] * (double)vs[d];
            }
        }
        block_sum<NT, 2>(fn, R.red1);
        float* xo = A.xyz + (size_t)s * natom * 3;
        for (int a = t; a < natom; a += NT) {
            const double4 p = pos[a];
            if (A.mode == 0) {
                xo[(size_t)a * 3] = (float)p.x;
                xo[(size_t)a * 3 + 1] = (float)p.y;
                xo[(size_t)a * 3 + 2] = (float)p.z;
            }
            if (A.forces_out)
#pragma unroll
                for (int d = 0; d < 3; ++d) A.forces_out[((size_t)s * natom + a) * 3 + d] = (float)F[d * ldn + a];
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
// Per structure: degrees, bond types (distinct (r0, k), sorted by their bit
// pattern -> deterministic ids) and the compact sliced-ELLPACK entries.
__device__ __forceinline__ const igm_bond& bond_at(const igm_bond* shared, int64_t nshared, const igm_bond* own,
                                                   int64_t q) {
    return q < nshared ? shared[q] : own[q - nshared];
}

__device__ __forceinline__ uint64_t bond_key(const igm_bond& b) {
    return ((uint64_t)__float_as_uint(b.r0) << 32) | (uint64_t)__float_as_uint(b.k);
}

__device__ __forceinline__ uint32_t key_hash(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    return (uint32_t)k & (kTypeHash - 1);
}

constexpr uint64_t kEmptyKey = ~0ull;

// insert every bond key of structure s into the LDS hash; returns (uniform) the
// number of distinct keys, or > kMaxBondTypes if the structure has too many
__device__ int hash_bond_types(uint64_t* hash, const igm_bond* shared, int64_t nshared, const igm_bond* own,
                               int64_t nb, int* nuniq) {
    const int t = threadIdx.x;
    for (int i = t; i < kTypeHash; i += blockDim.x) hash[i] = kEmptyKey;
    if (t == 0) *nuniq = 0;
    __syncthreads();
    for (int64_t q = t; q < nb; q += blockDim.x) {
        const uint64_t key = bond_key(bond_at(shared, nshared, own, q));
        uint32_t h = key_hash(key);
        for (int probe = 0; probe < kTypeHash; ++probe) {
            const uint64_t prev = atomicCAS((unsigned long long*)&hash[h], (unsigned long long)kEmptyKey,
                                            (unsigned long long)key);
            if (prev == kEmptyKey) {
                atomicAdd(nuniq, 1);
                break;
            }
            if (prev == key) break;
            h = (h + 1) & (kTypeHash - 1);
        }
    }
    __syncthreads();
    const int n = *nuniq;
    __syncthreads();
    return n;
}

__global__ void adj_degree_kernel(int natom, const igm_bond* shared, int64_t nshared, const int64_t* sptr,
                                  const igm_bond* sbonds, int* deg, int64_t* ntype, int* error) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_adj[];
    uint64_t* hash = reinterpret_cast<uint64_t*>(smem_adj);
    int* nuniq = reinterpret_cast<int*>(hash + kTypeHash);
    const int s = blockIdx.x;
    const int64_t b0 = sptr ? sptr[s] : 0, b1 = sptr ? sptr[s + 1] : 0;
    const igm_bond* own = sbonds ? sbonds + b0 : nullptr;
    const int64_t nb = nshared + (b1 - b0);
    int* dg = deg + (size_t)s * natom;
    for (int64_t q = threadIdx.x; q < nb; q += blockDim.x) {
        const igm_bond& bd = bond_at(shared, nshared, own, q);
        const uint32_t i = bd.i, j = bd.j & 0x7fffffffu;
        if (i >= (uint32_t)natom || j >= (uint32_t)natom) {
            atomicOr(error, 2);
            continue;
        }
        atomicAdd(&dg[i], 1);
        atomicAdd(&dg[j], 1);
    }
    const int n = hash_bond_types(hash, shared, nshared, own, nb, nuniq);
    if (threadIdx.x == 0) {
        ntype[s] = n;
        if (n > kMaxBondTypes) atomicOr(error, 4);
    }
}

// per-slice max degree -> slice offsets (runs after adj_degree_kernel completed)
__global__ void adj_slices_kernel(int natom, int nslice, const int* deg, int* soff, int64_t* size) {
    __shared__ int smax[1024];
    const int s = blockIdx.x;
    const int* dg = deg + (size_t)s * natom;
    for (int sl0 = 0; sl0 < nslice; sl0 += 1024) {
        const int sl = sl0 + (int)threadIdx.x;
        __syncthreads();
        if (threadIdx.x < 1024) {
            int m = 0;
            if (sl < nslice)
                for (int l = 0; l < 64; ++l) {
                    const int a = sl * 64 + l;
                    if (a < natom) m = max(m, dg[a]);
                }
            smax[threadIdx.x] = m;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t acc = sl0 == 0 ? 0 : (int64_t)soff[(size_t)s * (nslice + 1) + sl0];
            int* so = soff + (size_t)s * (nslice + 1);
            for (int i = 0; i < 1024 && sl0 + i < nslice; ++i) {
                so[sl0 + i] = (int)acc;
                acc += (int64_t)smax[i] * 64;
            }
            so[min(sl0 + 1024, nslice)] = (int)acc;
            if (sl0 + 1024 >= nslice) size[s] = acc;
        }
    }
}

__global__ void adj_fill_kernel(int natom, int nslice, const igm_bond* shared, int64_t nshared, const int64_t* sptr,
                                const igm_bond* sbonds, const int* deg, const int* soff, const int64_t* base,
                                const int64_t* tbase, int* fillc, uint32_t* ent, float2* types) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_adj[];
    uint64_t* hash = reinterpret_cast<uint64_t*>(smem_adj);
    int* nuniq = reinterpret_cast<int*>(hash + kTypeHash);
    uint64_t* uniq = hash + kTypeHash + 2;  // kMaxBondTypes sorted keys
    __shared__ int ncomp;
    const int s = blockIdx.x;
    const int t = threadIdx.x;
    const int64_t b0 = sptr ? sptr[s] : 0, b1 = sptr ? sptr[s + 1] : 0;
    const igm_bond* own = sbonds ? sbonds + b0 : nullptr;
    const int64_t nb = nshared + (b1 - b0);
    const int n = hash_bond_types(hash, shared, nshared, own, nb, nuniq);
    if (n > kMaxBondTypes) return;  // reported by adj_degree_kernel
    // compact the keys, then rank them: id = #keys below (deterministic)
    if (t == 0) ncomp = 0;
    __syncthreads();
    for (int i = t; i < kTypeHash; i += blockDim.x)
        if (hash[i] != kEmptyKey) uniq[atomicAdd(&ncomp, 1)] = hash[i];
    __syncthreads();
    float2* tt = types + tbase[s];
    for (int i = t; i < n; i += blockDim.x) {
        const uint64_t k = uniq[i];
        int r = 0;
        for (int q = 0; q < n; ++q) r += uniq[q] < k ? 1 : 0;
        hash[r] = k;  // the hash is dead: reuse it as the sorted table
    }
    __syncthreads();
    for (int i = t; i < n; i += blockDim.x) {
        const uint64_t k = hash[i];
        tt[i] = make_float2(__uint_as_float((uint32_t)(k >> 32)), __uint_as_float((uint32_t)k));
    }
    const int* so = soff + (size_t)s * (nslice + 1);
    uint32_t* E = ent + base[s];
    int* fc = fillc + (size_t)s * natom;
    for (int64_t q = t; q < nb; q += blockDim.x) {
        const igm_bond& bd = bond_at(shared, nshared, own, q);
        const uint32_t i = bd.i, j = bd.j & 0x7fffffffu, low = bd.j & kLowerBit;
        if (i >= (uint32_t)natom || j >= (uint32_t)natom) continue;
        const uint64_t key = bond_key(bd);
        int lo = 0, hi = n - 1;
        while (lo < hi) {  // lower_bound in the sorted table
            const int mid = (lo + hi) >> 1;
            if (hash[mid] < key)
                lo = mid + 1;
            else
                hi = mid;
        }
        const uint32_t tid = (uint32_t)lo << 16;
        const int si = atomicAdd(&fc[i], 1);
        const int sj = atomicAdd(&fc[j], 1);
        E[so[i >> 6] + (size_t)si * 64 + (i & 63)] = j | tid | low;
        E[so[j >> 6] + (size_t)sj * 64 + (j & 63)] = i | tid | low;
    }
    __syncthreads();
    // fixed order per atom: sort the entries
    const int* dg = deg + (size_t)s * natom;
    for (int a = t; a < natom; a += blockDim.x) {
        const int m = dg[a];
        uint32_t* Lp = E + so[a >> 6] + (a & 63);
        for (int i = 1; i < m; ++i) {
            const uint32_t v = Lp[(size_t)i * 64];
            int k = i - 1;
            while (k >= 0 && Lp[(size_t)k * 64] > v) {
                Lp[(size_t)(k + 1) * 64] = Lp[(size_t)k * 64];
                --k;
            }
            Lp[(size_t)(k + 1) * 64] = v;
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
    int64_t total_ent;
    bool big;  // HBM-resident kernels
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
        P->env_kind[e] = prm->env_kind[e];
        if (P->env_kind[e] != IGM_ENV_ELLIPSOID && P->env_kind[e] != IGM_ENV_VOLUME)
            return fail(c, IGM_E_INVALID, "env_kind[%d] = %d", e, P->env_kind[e]);
        if (P->env_kind[e] == IGM_ENV_VOLUME) {
            if (c->vol_nmap <= 0)
                return fail(c, IGM_E_INVALID, "envelope %d is volumetric but no map was staged (igm_mstep_set_volumes)",
                            e);
            void *pm, *pv, *ps;
            IGM_TRY(workspace(c, "vol_maps", 1, &pm));
            IGM_TRY(workspace(c, "vol_vox", 1, &pv));
            P->vmaps = (const VolMapDev*)pm;
            P->vvox = (const int4*)pv;
            P->vsmap = nullptr;
            if (c->vol_nsmap > 0) {
                IGM_TRY(workspace(c, "vol_smap", 1, &ps));
                P->vsmap = (const int*)ps;
            }
        }
    }
    // Verlet skin: LAMMPS 'neighbor maxrad bin' uses skin = maxrad.  The skin only sets
    // how often the (always complete) list is rebuilt, not the forces; 0.7 maxrad is the
    // measured optimum on MI355X (scripts/gpu_skin.sh: fewer list entries per force
    // evaluation vs more rebuilds).  prm->skin > 0 overrides.
    P->skin = prm->skin > 0 ? (float)prm->skin : 0.7f * rmax;
    if (const char* e = getenv("IGM_SKIN_FACTOR")) P->skin = (float)(atof(e) * rmax);  // tuning only
    P->cut_list = 2.0f * rmax + P->skin;
    P->kcap = prm->neigh_capacity > 0 ? prm->neigh_capacity : kNeighBudget;
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

// LDS path launch configuration: NT threads, BPT atoms per thread
struct LaunchCfg {
    int nt, bpt;
};

// 1024 threads x 3 atoms measured fastest for 2 Mb structures (profiles/); the
// choice can be overridden with IGM_MD_CFG=<threads>x<atoms per thread> (tuning).
bool lds_fits(int natom, LaunchCfg* cfg) {
    static const int opts[][2] = {{256, 1}, {512, 1}, {768, 1}, {1024, 1}, {1024, 2}, {1024, 3},
                                  {768, 4}, {512, 6}};
    int want_nt = 0, want_bpt = 0;
    if (const char* e = getenv("IGM_MD_CFG")) sscanf(e, "%dx%d", &want_nt, &want_bpt);
    for (auto& o : opts)
        if (o[0] * o[1] >= natom && (!want_nt || (o[0] == want_nt && o[1] == want_bpt))) {
            const int npad = o[0] * o[1];
            const MdLds m = carve_md_lds(nullptr, npad);
            // the list region doubles as the build's int scratch
            if ((size_t)kLdsListSlots * npad * 2 < build_scratch_bytes(kCellCap, npad) || m.rest_cap < 0) return false;
            CgLds cg;
            if (carve_cg_lds(nullptr, npad, false, &cg) > kLdsBytes) return false;
            cfg->nt = o[0];
            cfg->bpt = o[1];
            return true;
        }
    return false;
}

// ------------------------------------------------------------- volume maps
int set_volumes(igm_ctx* c, int32_t nmap, const igm_volume_map* maps, const int32_t* struct_map, int32_t nstruct) {
    if (nmap < 0 || (nmap > 0 && !maps) || (struct_map && nstruct <= 0))
        return fail(c, IGM_E_INVALID, "igm_mstep_set_volumes: invalid arguments");
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    c->vol_nmap = 0;
    c->vol_nsmap = 0;
    if (nmap == 0) return IGM_OK;
    std::vector<VolMapDev> hm(nmap);
    long long tot = 0;
    for (int m = 0; m < nmap; ++m) {
        const igm_volume_map& v = maps[m];
        if (!v.voxels || v.nvoxel[0] <= 0 || v.nvoxel[1] <= 0 || v.nvoxel[2] <= 0 || (v.body_idx != 0 && v.body_idx != 1))
            return fail(c, IGM_E_INVALID, "igm_mstep_set_volumes: map %d malformed", m);
        for (int d = 0; d < 3; ++d) {
            if (!(v.grid[d] > 0.0f)) return fail(c, IGM_E_INVALID, "igm_mstep_set_volumes: map %d grid <= 0", m);
            hm[m].n[d] = v.nvoxel[d];
            hm[m].center[d] = v.center[d];
            hm[m].origin[d] = v.origin[d];
            hm[m].grid[d] = v.grid[d];
        }
        hm[m].body = v.body_idx;
        hm[m].off = tot;
        const long long nv = (long long)v.nvoxel[0] * v.nvoxel[1] * v.nvoxel[2];
        for (long long q = 0; q < nv; ++q)
            for (int d = 0; d < 3; ++d)
                if (v.voxels[4 * q + d] < 0 || v.voxels[4 * q + d] >= v.nvoxel[d])
                    return fail(c, IGM_E_INVALID, "igm_mstep_set_volumes: map %d voxel %lld: EDT index out of range",
                                m, q);
        tot += nv;
    }
    if (struct_map)
        for (int s = 0; s < nstruct; ++s)
            if (struct_map[s] < 0 || struct_map[s] >= nmap)
                return fail(c, IGM_E_INVALID, "igm_mstep_set_volumes: struct_map[%d] = %d", s, struct_map[s]);
    void *pm, *pv;
    IGM_TRY(workspace(c, "vol_maps", sizeof(VolMapDev) * nmap, &pm));
    IGM_TRY(workspace(c, "vol_vox", sizeof(int4) * (size_t)tot, &pv));
    IGM_HIP_CHECK(c, hipMemcpyAsync(pm, hm.data(), sizeof(VolMapDev) * nmap, hipMemcpyHostToDevice, c->stream));
    for (int m = 0; m < nmap; ++m) {
        const long long nv = (long long)maps[m].nvoxel[0] * maps[m].nvoxel[1] * maps[m].nvoxel[2];
        IGM_HIP_CHECK(c, hipMemcpyAsync((int4*)pv + hm[m].off, maps[m].voxels, sizeof(int4) * (size_t)nv,
                                        hipMemcpyHostToDevice, c->stream));
    }
    if (struct_map) {
        void* ps;
        IGM_TRY(workspace(c, "vol_smap", sizeof(int) * nstruct, &ps));
        IGM_HIP_CHECK(c, hipMemcpyAsync(ps, struct_map, sizeof(int) * nstruct, hipMemcpyHostToDevice, c->stream));
        c->vol_nsmap = nstruct;
    }
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    c->vol_nmap = nmap;
    return IGM_OK;
}

// stage inputs + build the bond adjacency for all structures
int prepare(igm_ctx* c, uint32_t flags, const igm_mstep_params* prm, int32_t nstruct, int32_t natom,
            const float* radii, const uint32_t* atom_flags, const igm_bond* shared_bonds, int64_t nshared,
            const int64_t* sbond_ptr, const igm_bond* sbonds, Prepared* out) {
    if (natom <= 0 || natom > 65535) return fail(c, IGM_E_UNSUPPORTED, "natom=%d outside [1, 65535]", natom);
    for (int e = 0; e < prm->nenvelopes && e < IGM_MAX_ENVELOPES; ++e)
        if (prm->env_kind[e] == IGM_ENV_VOLUME && c->vol_nsmap > 0 && c->vol_nsmap < nstruct)
            return fail(c, IGM_E_INVALID, "volume map index staged for %d structures, batch has %d", c->vol_nsmap,
                        nstruct);
    const float* d_radii;
    const uint32_t* d_flags;
    const igm_bond* d_shared;
    const int64_t* d_sptr;
    const igm_bond* d_sb;
    IGM_TRY(to_device(c, flags, "ms_radii", radii, (size_t)natom, &d_radii));
    // IGM_MSTEP_STRUCT_FLAGS: one flag row per structure (DamID envelope membership,
    // SPRITE centroid slots); the BEAD bit must agree between structures
    const bool per_struct = (prm->flags & IGM_MSTEP_STRUCT_FLAGS) != 0;
    const size_t nfl = per_struct ? (size_t)nstruct * natom : (size_t)natom;
    IGM_TRY(to_device(c, flags, "ms_flags", atom_flags, nfl, &d_flags));
    if (per_struct) {
        std::vector<uint32_t> fl(nfl);
        IGM_HIP_CHECK(c, hipMemcpyAsync(fl.data(), d_flags, sizeof(uint32_t) * nfl, hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        for (size_t k = natom; k < nfl; ++k)
            if ((fl[k] ^ fl[k % natom]) & IGM_ATOM_BEAD)
                return fail(c, IGM_E_INVALID, "per-structure atom flags: atom %d is a bead in one structure only",
                            (int)(k % natom));
    }
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
    void *p_deg, *p_fill, *p_soff, *p_size, *p_base, *p_nt, *p_tb, *p_err, *p_wc;
    IGM_TRY(workspace(c, "ms_deg", sizeof(int) * (size_t)nstruct * natom, &p_deg));
    IGM_TRY(workspace(c, "ms_fill", sizeof(int) * (size_t)nstruct * natom, &p_fill));
    IGM_TRY(workspace(c, "ms_soff", sizeof(int) * (size_t)nstruct * (nslice + 1), &p_soff));
    IGM_TRY(workspace(c, "ms_size", sizeof(int64_t) * (size_t)nstruct, &p_size));
    IGM_TRY(workspace(c, "ms_base", sizeof(int64_t) * (size_t)nstruct, &p_base));
    IGM_TRY(workspace(c, "ms_ntype", sizeof(int64_t) * (size_t)nstruct, &p_nt));
    IGM_TRY(workspace(c, "ms_tbase", sizeof(int64_t) * (size_t)nstruct, &p_tb));
    IGM_TRY(workspace(c, "ms_err", sizeof(int) * 4, &p_err));
    IGM_TRY(workspace(c, "ms_wc", sizeof(int) * 4, &p_wc));
    int* d_err = (int*)p_err;
    IGM_HIP_CHECK(c, hipMemsetAsync(d_err, 0, sizeof(int) * 4, c->stream));
    IGM_HIP_CHECK(c, hipMemsetAsync(p_deg, 0, sizeof(int) * (size_t)nstruct * natom, c->stream));
    IGM_HIP_CHECK(c, hipMemsetAsync(p_fill, 0, sizeof(int) * (size_t)nstruct * natom, c->stream));
    const size_t lds_deg = sizeof(uint64_t) * kTypeHash + 16;
    const size_t lds_fill = lds_deg + sizeof(uint64_t) * kMaxBondTypes;
    {
        Timed tm(c, "adjacency");
        IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)adj_degree_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_deg));
        IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)adj_fill_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds_fill));
        hipLaunchKernelGGL(adj_degree_kernel, dim3(nstruct), dim3(256), lds_deg, c->stream, natom, d_shared, nshared,
                           d_sptr, d_sb, (int*)p_deg, (int64_t*)p_nt, d_err);
        IGM_HIP_CHECK(c, hipGetLastError());
        hipLaunchKernelGGL(adj_slices_kernel, dim3(nstruct), dim3(1024), 0, c->stream, natom, nslice,
                           (const int*)p_deg, (int*)p_soff, (int64_t*)p_size);
        IGM_HIP_CHECK(c, hipGetLastError());
        size_t tmp_bytes = 0;
        IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, (int64_t*)p_size, (int64_t*)p_base,
                                                          nstruct, c->stream));
        void* d_tmp;
        IGM_TRY(workspace(c, "ms_scan_tmp", tmp_bytes, &d_tmp));
        IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_bytes, (int64_t*)p_size, (int64_t*)p_base,
                                                          nstruct, c->stream));
        IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_bytes, (int64_t*)p_nt, (int64_t*)p_tb, nstruct,
                                                          c->stream));
        int64_t last[4] = {0, 0, 0, 0};
        int herr = 0;
        IGM_HIP_CHECK(c, hipMemcpyAsync(&last[0], (int64_t*)p_base + nstruct - 1, sizeof(int64_t),
                                        hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipMemcpyAsync(&last[1], (int64_t*)p_size + nstruct - 1, sizeof(int64_t),
                                        hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipMemcpyAsync(&last[2], (int64_t*)p_tb + nstruct - 1, sizeof(int64_t),
                                        hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipMemcpyAsync(&last[3], (int64_t*)p_nt + nstruct - 1, sizeof(int64_t),
                                        hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipMemcpyAsync(&herr, d_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        if (herr & 2) return fail(c, IGM_E_INVALID, "bond atom index out of range");
        if (herr & 4)
            return fail(c, IGM_E_UNSUPPORTED, "a structure has more than %d distinct bond (r0, k) types",
                        kMaxBondTypes);
        const int64_t total = last[0] + last[1], ntypes = last[2] + last[3];
        void *p_ent, *p_types;
        IGM_TRY(workspace(c, "ms_ent", sizeof(uint32_t) * (size_t)(total > 0 ? total : 1), &p_ent));
        IGM_TRY(workspace(c, "ms_types", sizeof(float2) * (size_t)(ntypes > 0 ? ntypes : 1), &p_types));
        hipLaunchKernelGGL(adj_fill_kernel, dim3(nstruct), dim3(256), lds_fill, c->stream, natom, nslice, d_shared,
                           nshared, d_sptr, d_sb, (const int*)p_deg, (const int*)p_soff, (const int64_t*)p_base,
                           (const int64_t*)p_tb, (int*)p_fill, (uint32_t*)p_ent, (float2*)p_types);
        IGM_HIP_CHECK(c, hipGetLastError());
        out->total_ent = total;
        out->cm.bonds.ent = (const uint32_t*)p_ent;
        out->cm.bonds.types = (const float2*)p_types;
    }
    out->cm.nstruct = nstruct;
    out->cm.natom = natom;
    out->cm.nslice = nslice;
    out->cm.ldn = nslice * 64;
    out->cm.radii = d_radii;
    out->cm.atype = d_atype;
    out->cm.aflags = d_flags;
    out->cm.afs = per_struct ? (size_t)natom : 0;
    out->cm.bonds.base = (const int64_t*)p_base;
    out->cm.bonds.soff = (const int*)p_soff;
    out->cm.bonds.deg = (const int*)p_deg;
    out->cm.bonds.tbase = (const int64_t*)p_tb;
    out->cm.bonds.ntype = (const int64_t*)p_nt;
    out->cm.work_counter = (int*)p_wc;
    out->cm.error = d_err;
    // Verlet-list slots per atom; the HBM part must also hold the build's int scratch
    int kcap = P.kcap;
    while ((size_t)out->cm.ldn * kcap * 2 < build_scratch_bytes(kCellCapBig, out->cm.ldn)) ++kcap;
    out->cm.kcap = kcap;
    LaunchCfg cfg;
    out->big = (prm->flags & IGM_MSTEP_FORCE_GLOBAL) || getenv("IGM_FORCE_POP") || !lds_fits(natom, &cfg);
    // (the population engine's skin optimum is also 0.7 maxrad: config C, protocol x0.2,
    //  0.45 / 0.55 / 0.7 / 0.85 / 1.0 maxrad -> 5.59 / 5.45 / 5.31 / 5.32 / 5.37 s anneal)
    out->P = P;
    return IGM_OK;
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
    else IGM_DISPATCH_CFG(768, 1, __VA_ARGS__)                     \
    else IGM_DISPATCH_CFG(1024, 1, __VA_ARGS__)                    \
    else IGM_DISPATCH_CFG(1024, 2, __VA_ARGS__)                    \
    else IGM_DISPATCH_CFG(768, 4, __VA_ARGS__)                     \
    else IGM_DISPATCH_CFG(512, 6, __VA_ARGS__)                     \
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


// the structures [s0, s0 + ns) of a population engine as an engine of their own
// (per-structure pointers offset; flag counter g)
PopArgs pop_view(const PopArgs& Q, int s0, int ns, int g) {
    PopArgs V = Q;
    const size_t ldn = Q.cm.ldn, nsl = Q.cm.nslice, o = (size_t)s0 * ldn;
    V.cm.nstruct = ns;
    V.cm.aflags = Q.cm.aflags + (size_t)s0 * Q.cm.afs;
    V.cm.bonds.base = Q.cm.bonds.base + s0;
    V.cm.bonds.soff = Q.cm.bonds.soff + (size_t)s0 * (nsl + 1);
    V.cm.bonds.deg = Q.cm.bonds.deg + (size_t)s0 * Q.cm.natom;
    V.cm.bonds.tbase = Q.cm.bonds.tbase + s0;
    V.cm.bonds.ntype = Q.cm.bonds.ntype + s0;
    if (V.P.vsmap) V.P.vsmap = Q.P.vsmap + s0;
    for (int b = 0; b < 2; ++b)
        V.buf[b] = PopBuf{Q.buf[b].pos + o, Q.buf[b].vel + o, Q.buf[b].frc + o, Q.buf[b].aid + o, Q.buf[b].slot + o,
                        Q.buf[b].flg + o};
    V.par = Q.par + s0;
    V.xb = Q.xb + o;
    V.nl = Q.nl + (size_t)s0 * nsl * Q.kq * 64;
    V.nnb = Q.nnb + o;
    V.cell = Q.cell + (size_t)s0 * kPopCells;
    V.gp = Q.gp + (size_t)s0 * 8;
    V.gn = Q.gn + (size_t)s0 * 8;
    for (int b = 0; b < 2; ++b) {
        V.bentb[b] = Q.bentb[b] + (size_t)s0 * nsl * Q.bdmax * 64;
        V.bdegb[b] = Q.bdegb[b] + o;
    }
    if (Q.bc) {
        V.bc = Q.bc + (size_t)s0 * nsl * Q.bdmax * 64;
        V.bcn = Q.bcn + o;
        V.bpr = Q.bpr + s0;
        V.bage = Q.bage + s0;
    }
    V.inv = Q.inv + o;
    V.remap = Q.remap + o;
    if (Q.ccnt) {
        V.ccnt = Q.ccnt + (size_t)s0 * kPopCntStride;
        V.tid = Q.tid + o;
        V.ctot = Q.ctot + (size_t)s0 * 8;
    }
    V.flag[0] = Q.flag[0] + s0;
    V.flag[1] = Q.flag[1] + s0;
    V.oflag[0] = Q.oflag[0] + s0;
    V.oflag[1] = Q.oflag[1] + s0;
    V.flist = Q.flist + s0;
    V.flist2 = Q.flist2 + s0;
    V.nflag = Q.nflag + g;  // one build counter per group, each on its own stream
    V.nflag2 = Q.nflag2 + g;
    if (Q.two) {
        V.xo = Q.xo + o;
        V.nlo = Q.nlo + (size_t)s0 * nsl * Q.kqo * 64;
        V.nnbo = Q.nnbo + o;
    }
    V.nrebuild = Q.nrebuild + s0;
    V.kep = Q.kep + (size_t)s0 * Q.nbs;
    V.bbp = Q.bbp + (size_t)s0 * Q.nbs * 6;
    V.dofs = Q.dofs + s0;
    V.coff = Q.coff + (size_t)s0 * (Q.cm.natom + 1);
    V.cbase = Q.cbase + s0;
    return V;
}

// The population engine (HBM path): per step  integrate | [sort | permute | fill of the
// flagged structures] | forces + final kick, over every slot of every structure.
int run_anneal_pop(igm_ctx* c, const Prepared& pr, const AnnealArgs& A) {
    const int S = pr.cm.nstruct, N = pr.cm.natom, ldn = pr.cm.ldn, nsl = pr.cm.nslice;
    PopArgs Q;
    memset(&Q, 0, sizeof(Q));
    Q.cm = pr.cm;
    Q.P = pr.P;
    Q.nbs = (N + kPopBS - 1) / kPopBS;
    const size_t SL = (size_t)S * ldn;
    // the largest bond degree sizes the slot-ordered bond ELL
    void* pdm;
    IGM_TRY(workspace(c, "pop_dmax", sizeof(int), &pdm));
    IGM_HIP_CHECK(c, hipMemsetAsync(pdm, 0, sizeof(int), c->stream));
    hipLaunchKernelGGL(deg_max_kernel, dim3(1024), dim3(256), 0, c->stream, pr.cm.bonds.deg, (size_t)S * N, (int*)pdm);
    int dmax = 0;
    IGM_HIP_CHECK(c, hipMemcpyAsync(&dmax, pdm, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    if (dmax > 0xFFFF) return fail(c, IGM_E_UNSUPPORTED, "an atom has %d bonds", dmax);
    Q.bdmax = dmax > 0 ? dmax : 1;
    Q.kq = ((pr.P.kcap == kNeighBudget ? kPopListCap : std::min(pr.P.kcap, kPopListCap)) + 3) / 4;
    {
        // HBM of the engine's state, per slot: two parity buffers of (position 16, velocity
        // 12, force 12, atom id 4, slot 4, flags 1), build position 12, Verlet list 8 kq (512
        // B at the default 256 entries -- most of it), list length 2, bonds 2 x 4 bdmax, degree
        // 2 x 2, slot remaps 8, pruned bonds 4 bdmax + 2; per structure the cell offsets.  At
        // config C (1000 x 29 839 slots) the lists alone are 15.3 GB.  Checked against the free
        // HBM (plus what this context's population workspace already holds) before anything
        // is allocated.
        const size_t per_slot = 2 * (16 + 12 + 12 + 4 + 4 + 1) + 12 + 8 * (size_t)Q.kq + 2 + 12 * (size_t)Q.bdmax + 6 +
                                8 + 4;
        const size_t need = per_slot * SL + sizeof(int) * (size_t)S * (kPopCells + kPopCntStride);
        size_t held = 0;
        for (const auto& kv : c->ws)
            if (kv.first.compare(0, 4, "pop_") == 0) held += kv.second.second;
        size_t fre = 0, tot = 0;
        if (hipMemGetInfo(&fre, &tot) == hipSuccess && need > fre + held)
            return fail(c, IGM_E_NOMEM,
                        "population engine: %zu structures x %d slots need %.1f GB of HBM (%.1f MB per structure, "
                        "%.1f of it the %d-entry Verlet lists), %.1f GB free: pass fewer structures per call or a "
                        "smaller neigh_capacity", (size_t)S, ldn, need / 1e9, need / 1e6 / S,
                        8.0 * Q.kq * ldn / 1e6, 4 * Q.kq, (fre + held) / 1e9);
        (void)hipGetLastError();
    }
    for (int b = 0; b < 2; ++b) {
        char nm[6][16];
        const char* what[6] = {"pos", "vel", "frc", "aid", "slot", "flg"};
        void* p[6];
        const size_t sz[6] = {sizeof(float4), sizeof(pop_f3), sizeof(pop_f3), sizeof(int), sizeof(int), 1};
        for (int k = 0; k < 6; ++k) {
            snprintf(nm[k], sizeof(nm[k]), "pop_%s%d", what[k], b);
            IGM_TRY(workspace(c, nm[k], sz[k] * SL, &p[k]));
        }
        Q.buf[b] = PopBuf{(float4*)p[0], (pop_f3*)p[1], (pop_f3*)p[2], (int*)p[3], (int*)p[4], (uint8_t*)p[5]};
    }
    void *ppar, *pxb, *pnl, *pnnb, *pcell, *pgp, *pgn, *pbent, *pbdeg, *pfl, *pfli, *pnf, *pke, *pbb;
    IGM_TRY(workspace(c, "pop_par", sizeof(int) * S, &ppar));
    IGM_TRY(workspace(c, "pop_xb", sizeof(pop_f3) * SL, &pxb));
    // (Q.kq above: the list capacity, kPopListCap or a smaller neigh_capacity given in the
    // params -- the default 64 is the LDS engine's budget)
    IGM_TRY(workspace(c, "pop_nl", sizeof(uint2) * SL * Q.kq, &pnl));
    IGM_TRY(workspace(c, "pop_nnb", sizeof(uint16_t) * SL, &pnnb));
    IGM_TRY(workspace(c, "pop_cell", sizeof(int) * (size_t)S * kPopCells, &pcell));
    IGM_TRY(workspace(c, "pop_gp", sizeof(float) * 8 * (size_t)S, &pgp));
    IGM_TRY(workspace(c, "pop_gn", sizeof(int) * 8 * (size_t)S, &pgn));
    IGM_TRY(workspace(c, "pop_bent", sizeof(uint32_t) * SL * Q.bdmax * 2, &pbent));
    IGM_TRY(workspace(c, "pop_bdeg", sizeof(uint16_t) * SL * 2, &pbdeg));
    {
        void *pinv, *prm;
        IGM_TRY(workspace(c, "pop_inv", sizeof(int) * SL, &pinv));
        IGM_TRY(workspace(c, "pop_remap", sizeof(int) * SL, &prm));
        Q.inv = (int*)pinv;
        Q.remap = (int*)prm;
    }
    IGM_TRY(workspace(c, "pop_flag", sizeof(int) * 2 * (size_t)S, &pfl));
    IGM_TRY(workspace(c, "pop_flist", sizeof(int) * (size_t)S, &pfli));
    IGM_TRY(workspace(c, "pop_nflag", sizeof(int) * 2 * kPopMaxGroups, &pnf));
    IGM_TRY(workspace(c, "pop_ke", sizeof(double) * (size_t)S * Q.nbs, &pke));
    IGM_TRY(workspace(c, "pop_bb", sizeof(float) * 6 * (size_t)S * Q.nbs, &pbb));
    void* pnr = A.nrebuild;
    if (!pnr) IGM_TRY(workspace(c, "pop_nreb", sizeof(int) * (size_t)S, &pnr));
    // two-level lists: the outer margin in units of the largest radius (0: one level)
    const float rmax0 = 0.5f * (pr.P.cut_list - pr.P.skin);
    float margin = 0.0f;
    if (const char* e = getenv("IGM_POP_OUTER")) margin = (float)atof(e) * rmax0;
    if (kPopFused) margin = 0.0f;
    Q.two = margin > 0.0f ? 1 : 0;
    constexpr int kOuterRow = kPopOuterCap + 2;
    {
        void *pfl2, *pfli2;
        IGM_TRY(workspace(c, "pop_oflag", sizeof(int) * 2 * (size_t)S, &pfl2));
        IGM_TRY(workspace(c, "pop_flist2", sizeof(int) * (size_t)S, &pfli2));
        Q.oflag[0] = (int*)pfl2;
        Q.oflag[1] = (int*)pfl2 + S;
        Q.flist2 = (int*)pfli2;
        if (Q.two) {
            void *pxo, *pnlo, *pnnbo;
            Q.kqo = kPopOuterCap / 4;
            IGM_TRY(workspace(c, "pop_xo", sizeof(float4) * SL, &pxo));
            IGM_TRY(workspace(c, "pop_nlo", sizeof(uint2) * SL * Q.kqo, &pnlo));
            IGM_TRY(workspace(c, "pop_nnbo", sizeof(uint16_t) * SL, &pnnbo));
            Q.xo = (float4*)pxo;
            Q.nlo = (uint2*)pnlo;
            Q.nnbo = (uint16_t*)pnnbo;
        }
    }
    Q.par = (int*)ppar;
    Q.xb = (pop_f3*)pxb;
    Q.nl = (uint2*)pnl;
    Q.nnb = (uint16_t*)pnnb;
    Q.cell = (int*)pcell;
    Q.gp = (float*)pgp;
    Q.gn = (int*)pgn;
    Q.bentb[0] = (uint32_t*)pbent;
    Q.bentb[1] = (uint32_t*)pbent + SL * Q.bdmax;
    Q.bdegb[0] = (uint16_t*)pbdeg;
    Q.bdegb[1] = (uint16_t*)pbdeg + SL;
    // bond pruning at list builds (the permute; IGM_POP_BOND_PRUNE=0 turns it off: a test
    // switch -- the forces are bitwise the same either way).  Not with two-level lists (their
    // inner builds move the build positions without a permute) nor the fused engine.
    {
        const char* e = getenv("IGM_POP_BOND_PRUNE");
        if ((e ? atoi(e) != 0 : true) && !Q.two && !kPopFused) {
            void *pbc, *pbcn, *pbpr;
            IGM_TRY(workspace(c, "pop_bc", sizeof(uint32_t) * SL * Q.bdmax, &pbc));
            IGM_TRY(workspace(c, "pop_bcn", sizeof(uint16_t) * SL, &pbcn));
            IGM_TRY(workspace(c, "pop_bpr", sizeof(int) * 2 * (size_t)S, &pbpr));
            // ages start large: the first build prunes
            IGM_HIP_CHECK(c, hipMemsetAsync(pbpr, 0x3f, sizeof(int) * 2 * (size_t)S, c->stream));
            Q.bc = (uint32_t*)pbc;
            Q.bcn = (uint16_t*)pbcn;
            Q.bpr = (int*)pbpr;
            Q.bage = (int*)pbpr + S;
            // Prune only at builds whose replaced lists served >= 6 steps (IGM_POP_PRUNE_AGE, tuning):
            // a structure rebuilding every few steps pays the permute's partner gathers and saves
            // little (measured on the 125-structure shard, full protocol, same box: always -1.4 %,
            // age >= 6 -3.2 % against no pruning; frustrated -0.9 %, config E +0.4 %; profiles/r06_ab)
            const char* ea = getenv("IGM_POP_PRUNE_AGE");
            Q.prune_age = ea ? atoi(ea) : 6;
        }
    }
    Q.flag[0] = (int*)pfl;
    Q.flag[1] = (int*)pfl + S;
    Q.flist = (int*)pfli;
    Q.nflag = (int*)pnf;
    Q.nflag2 = (int*)pnf + kPopMaxGroups;
    const bool sprof = IGM_POP_SORT_PROF && getenv("IGM_POP_SORT_PROF") != nullptr;  // profiling builds only
    if (sprof) {
        void* psp;
        IGM_TRY(workspace(c, "pop_sprof", sizeof(unsigned long long) * 8, &psp));
        IGM_HIP_CHECK(c, hipMemsetAsync(psp, 0, sizeof(unsigned long long) * 8, c->stream));
        Q.sprof = (unsigned long long*)psp;
    }
    Q.kep = (double*)pke;
    Q.bbp = (float*)pbb;
    Q.nrebuild = (int*)pnr;
    (void)nsl;
    // dof of group nonfixed, per structure (atom flags may differ between structures)
    {
        const size_t nfl = pr.cm.afs ? (size_t)S * N : (size_t)N;
        std::vector<uint32_t> fl(nfl);
        IGM_HIP_CHECK(c, hipMemcpyAsync(fl.data(), pr.cm.aflags, sizeof(uint32_t) * nfl, hipMemcpyDeviceToHost,
                                        c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        std::vector<double> dofs(S);
        for (int st = 0; st < S; ++st) {
            const uint32_t* f = fl.data() + (size_t)st * pr.cm.afs;
            int nmob = 0;
            for (int i = 0; i < N; ++i) nmob += (f[i] & IGM_ATOM_FIXED) ? 0 : 1;
            dofs[st] = 3.0 * nmob - 3.0;
        }
        void* pdof;
        IGM_TRY(workspace(c, "pop_dof", sizeof(double) * S, &pdof));
        IGM_HIP_CHECK(c, hipMemcpyAsync(pdof, dofs.data(), sizeof(double) * S, hipMemcpyHostToDevice, c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        Q.dofs = (const double*)pdof;
    }
    // bond rows as CSR (per-structure offsets by a block scan, structure bases on the host):
    // the fused engine re-indexes bonds from atom space; the permute remaps slot space
    if (kPopFused) {
        void *pco, *pcb, *pcsr;
        IGM_TRY(workspace(c, "pop_coff", sizeof(int) * (size_t)S * (N + 1), &pco));
        hipLaunchKernelGGL(pop_csr_scan_kernel, dim3(S), dim3(1024), 0, c->stream, pr.cm.bonds.deg, N, (int*)pco);
        std::vector<int> tot(S);
        IGM_HIP_CHECK(c, hipMemcpy2DAsync(tot.data(), sizeof(int), (const int*)pco + N, sizeof(int) * (N + 1),
                                          sizeof(int), S, hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        std::vector<int64_t> cb(S);
        int64_t run = 0;
        for (int st = 0; st < S; ++st) {
            cb[st] = run;
            run += tot[st];
        }
        IGM_TRY(workspace(c, "pop_cbase", sizeof(int64_t) * (size_t)S, &pcb));
        IGM_TRY(workspace(c, "pop_csr", sizeof(uint32_t) * (size_t)(run > 0 ? run : 1), &pcsr));
        IGM_HIP_CHECK(c, hipMemcpyAsync(pcb, cb.data(), sizeof(int64_t) * S, hipMemcpyHostToDevice, c->stream));
        const int64_t nx = (int64_t)S * N;
        hipLaunchKernelGGL(pop_csr_fill_kernel, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, c->stream,
                           pr.cm.bonds, S, N, pr.cm.nslice, (const int*)pco, (const int64_t*)pcb, (uint32_t*)pcsr);
        IGM_HIP_CHECK(c, hipGetLastError());
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));  // cb (host) must outlive the copy
        Q.coff = (const int*)pco;
        Q.cbase = (const int64_t*)pcb;
        Q.csr = (const uint32_t*)pcsr;
    }
    // the sort keeps its ids in LDS when they fit beside the cell counts (200 kb: 29 839 atoms)
    auto knob = [](const char* name, int dflt) {
        const char* e = getenv(name);
        return e ? atoi(e) : dflt;
    };
    // The sort: the single-workgroup LDS sort (default) or the split sort (IGM_POP_SORT=1;
    // both give the same slot order at the same cell cap, tests/test_mstep_paths_gpu.py).
    // Measured on config C (profiles/r06_ab): the split sort is 6 % slower at 125 structures
    // per GPU (full protocol: anneal 16.2 s against 15.3 s) and 16 % at pop = 1000 (protocol
    // x0.05: 6.01 s against 5.18 s): it moves the counts, ids and cell offsets through HBM/L2
    // in four launches where the LDS sort keeps them on one CU, and at these populations the
    // other structure group hides the LDS sort's latency.  Two-level lists and the fused
    // engine keep the LDS sort.  The split sort's counts live in HBM, so its grids take
    // kPopCellCap cells whatever the structure's size; the LDS sort's cap is what its LDS holds.
    const bool split = knob("IGM_POP_SORT", 0) != 0 && !Q.two && !kPopFused;
    Q.ccap = split ? kPopCellCap : pop_sort_cells(N);
    {  // x cells per cell side (IGM_POP_QX: A/B only)
        const char* e = getenv("IGM_POP_QX");
        Q.qx = e ? std::max(1, std::min(4, atoi(e))) : kPopQx;
    }
    const bool ids_lds = pop_sort_lds(true, N, Q.ccap) <= kLdsBytes;
    const size_t sort_lds = pop_sort_lds(ids_lds, N, Q.ccap);
    auto sort_kern = !ids_lds ? pop_sort_kernel<false, 0>
                     : N <= 16 * kPopSortNT ? pop_sort_kernel<true, 16>
                     : N <= 32 * kPopSortNT ? pop_sort_kernel<true, 32> : pop_sort_kernel<true, 0>;
    IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)sort_kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)sort_lds));
    if (split) {
        void *pcc, *ptd, *pct;
        IGM_TRY(workspace(c, "pop_ccnt", sizeof(int) * (size_t)S * kPopCntStride, &pcc));
        IGM_TRY(workspace(c, "pop_tid", sizeof(int) * SL, &ptd));
        IGM_TRY(workspace(c, "pop_ctot", sizeof(int) * (size_t)S * 8, &pct));
        IGM_HIP_CHECK(c, hipMemsetAsync(pcc, 0, sizeof(int) * (size_t)S * kPopCntStride, c->stream));
        IGM_HIP_CHECK(c, hipMemsetAsync(pct, 0, sizeof(int) * (size_t)S * 8, c->stream));
        Q.ccnt = (int*)pcc;
        Q.tid = (int*)ptd;
        Q.ctot = (int*)pct;
    }
    // structure slots of the build kernels' grids (IGM_POP_BUILD_SLOTS): a block loops over
    // the flagged structures b / nbs, + slots, ..., so the grid need not cover every
    // structure of the group (~1/6 of them rebuild at a step)
    const int bslots = std::max(1, knob("IGM_POP_BUILD_SLOTS", 128));
    // Structure groups on auxiliary streams: while one group waits in its latency-bound
    // sort, the others' force and integrate launches fill the CUs (measured on config C:
    // 2 groups 11 % faster than 1, 4 and 8 slower).  Tuning knobs: IGM_POP_GROUPS groups,
    // IGM_POP_CONC of them in flight together, IGM_POP_CHUNK steps per group before the
    // next ones run (0: every group advances in lock step).
    int ng = knob("IGM_POP_GROUPS", 2), nc = knob("IGM_POP_CONC", 0), chunk = knob("IGM_POP_CHUNK", 0);
    ng = ng < 1 ? 1 : (ng > S ? S : (ng > kPopMaxGroups ? kPopMaxGroups : ng));
    nc = nc < 1 || nc > ng ? ng : nc;
    if (chunk <= 0) nc = ng;
    // Forces ahead of the list builds (IGM_POP_EARLY=1, A/B only): the structures not rebuilt
    // at a step need only the integrate before their force evaluation, so a second stream per
    // group runs their forces (part 1) beside the flagged structures' sort, permute and fill,
    // and the flagged ones' forces (part 2) follow the fill; the next integrate waits for both.
    // Each structure is in exactly one part, so the results are bitwise those of one launch.
    // Measured on config C (profiles/r06_ab): 125 structures 16.3-17.3 s anneal against 15.3 s,
    // pop = 1000 (x0.05) 5.46 s against 5.17 s -- the steps are bound by the GPU's gather
    // throughput, not by the groups' launch chains, so the shorter chain buys nothing and the
    // second launch and cross-stream events cost.
    const bool early = knob("IGM_POP_EARLY", 0) != 0 && !kPopFused;
    auto force_kern = pop_force_kernel<kPopFused>;
    IGM_TRY(aux_streams(c, nc + (early ? ng : 0)));
    std::vector<hipEvent_t> ev_int(early ? ng : 0), ev_frc(early ? ng : 0);
    for (int g = 0; g < (early ? ng : 0); ++g) {
        IGM_TRY(pop_event(c, 2 * g, &ev_int[g]));
        IGM_TRY(pop_event(c, 2 * g + 1, &ev_frc[g]));
    }
    auto side = [&](int g) { return c->aux[nc + g]; };
    std::vector<PopArgs> V(ng);
    std::vector<int> g0(ng + 1);
    for (int g = 0; g <= ng; ++g) g0[g] = (int)((int64_t)S * g / ng);
    for (int g = 0; g < ng; ++g) V[g] = pop_view(Q, g0[g], g0[g + 1] - g0[g], g);
    auto grid_of = [&](int g) { return dim3(((g0[g + 1] - g0[g]) * Q.nbs + 7) & ~7); };  // padded for pop_block
    auto strm = [&](int g) { return c->aux[g % nc]; };
    const dim3 blk(kPopBS);
    const size_t n3 = (size_t)N * 3;
    // tuning diagnostic: list shape per run, sampled every IGM_POP_STATS steps (16 counters per run)
    const int stats_every = knob("IGM_POP_STATS", 0);
    unsigned long long* pst = nullptr;
    if (stats_every > 0) {
        void* p;
        IGM_TRY(workspace(c, "pop_stats", sizeof(unsigned long long) * 16 * 2 * IGM_MAX_STAGES, &p));
        IGM_HIP_CHECK(c, hipMemsetAsync(p, 0, sizeof(unsigned long long) * 16 * 2 * IGM_MAX_STAGES, c->stream));
        pst = (unsigned long long*)p;
    }
    Timed tm(c, "anneal");
    IGM_TRY(aux_fork(c, nc + (early ? ng : 0)));
    for (int g = 0; g < ng; ++g) {
        hipLaunchKernelGGL(pop_load_kernel, grid_of(g), blk, 0, strm(g), V[g], (const float*)A.xyz + g0[g] * n3);
        if (A.nseg == 0) {  // no runs (CG only): velocities 0, positions unchanged
            PopStep st;
            memset(&st, 0, sizeof(st));
            hipLaunchKernelGGL(pop_finish_kernel, grid_of(g), blk, 0, strm(g), V[g], st, A.xyz + g0[g] * n3,
                               A.vel + g0[g] * n3, A.forces_out ? A.forces_out + g0[g] * n3 : nullptr);
        }
    }
    long gbase = 0;  // steps of the earlier segments: the flag parity runs on across segments
    // Verlet skin per run (tuning knob IGM_POP_SKIN_SEG = "f0,f1,..." in units of the
    // largest radius; absent: the engine's skin for every run).  Any skin gives the same
    // forces -- the list holds every pair within cut_list = 2 rmax + skin and is rebuilt
    // once an atom moved skin / 2 -- so hot runs (frequent rebuilds) can trade longer
    // lists for fewer rebuilds and cold ones the reverse.
    std::vector<float> seg_skin(A.seg_skin, A.seg_skin + A.nseg);
    if (const char* e = getenv("IGM_POP_SKIN_SEG")) {  // the population engine's own (tuning)
        const float rmax = 0.5f * (pr.P.cut_list - pr.P.skin);
        int k = 0;
        for (const char* q = e; *q && k < A.nseg; ++k) {
            seg_skin[k] = (float)atof(q) * rmax;
            while (*q && *q != ',') ++q;
            if (*q == ',') ++q;
        }
    }
    float last_skin = pr.P.skin;
    for (int seg = 0; seg < A.nseg; ++seg) {
        if (seg_skin[seg] != last_skin || seg == 0) {  // a new cut: every list is rebuilt at the run's setup step
            for (int g = 0; g < ng; ++g) {
                V[g].P.cut_list = 2.0f * rmax0 + seg_skin[seg] + margin;  // (two-level: the outer cut)
                V[g].cut_in = 2.0f * rmax0 + seg_skin[seg];
                V[g].P.skin = seg_skin[seg];
                hipLaunchKernelGGL(pop_flag_all_kernel, dim3((g0[g + 1] - g0[g] + 255) / 256), dim3(256), 0, strm(g),
                                   V[g], (int)(gbase & 1));
            }
            last_skin = seg_skin[seg];
        }
        const float* vsrc = A.mode == 1 ? A.vel : A.vinit + (size_t)seg * n3;
        const size_t sstride = A.mode == 1 ? n3 : (size_t)A.nseg * n3;
        for (int g = 0; g < ng; ++g)
            hipLaunchKernelGGL(pop_setvel_kernel, grid_of(g), blk, 0, strm(g), V[g], vsrc + g0[g] * sstride,
                               sstride);
        PopStep st;
        memset(&st, 0, sizeof(st));
        st.dtv = A.dt;
        st.dtf = 0.5f * A.dt;
        st.vlim = A.seg_xmax[seg] / A.dt;
        st.vlimsq = st.vlim * st.vlim;
        st.trig = 0.25f * seg_skin[seg] * seg_skin[seg];
        st.trig_out = 0.25f * margin * margin;
        st.nsteps = A.seg_steps[seg];
        st.t0 = A.seg_t0[seg];
        st.t1 = A.seg_t1[seg];
        st.window = A.t_window;
        st.fraction = A.t_fraction;
        const float evf = A.seg_evf[seg], envf = A.seg_envf[seg];
        const int span = chunk > 0 ? chunk : st.nsteps + 1;
        for (int c0 = 0; c0 <= st.nsteps; c0 += span) {
            const int c1 = c0 + span - 1 < st.nsteps ? c0 + span - 1 : st.nsteps;
            for (int w0 = 0; w0 < ng; w0 += nc) {  // groups w0 .. w0 + nc - 1 run steps c0..c1 together
                for (int step = c0; step <= c1; ++step) {
                    st.integrate = step > 0;
                    st.rescale = step > 1;
                    st.prev = step - 1;
                    st.fp = (int)((gbase + step) & 1);
                    for (int g = w0; g < w0 + nc && g < ng; ++g) {
                        const int ns = g0[g + 1] - g0[g];
                        hipStream_t sg = strm(g);
                        const dim3 bgrid(std::min(ns, bslots) * Q.nbs);  // the build kernels' grid
                        hipLaunchKernelGGL(pop_integrate_kernel, grid_of(g), blk, 0, sg, V[g], st);
                        if (early) {  // the structures not rebuilt: forces beside the builds
                            PopStep s1 = st;
                            s1.part = 1;
                            IGM_HIP_CHECK(c, hipEventRecord(ev_int[g], sg));
                            IGM_HIP_CHECK(c, hipStreamWaitEvent(side(g), ev_int[g], 0));
                            hipLaunchKernelGGL(force_kern, grid_of(g), blk, 0, side(g), V[g], evf,
                                               envf, s1);
                            IGM_HIP_CHECK(c, hipEventRecord(ev_frc[g], side(g)));
                        }
                        if (split) {
                            hipLaunchKernelGGL(pop_count_kernel, dim3(ns * Q.nbs), blk, 0, sg, V[g], st.fp);
                            hipLaunchKernelGGL(pop_scan_kernel<kScanChunk / 8>, dim3(std::min(ns, bslots) * kScanChunks),
                                               dim3(kScanChunk / 8), 0, sg, V[g]);
                            hipLaunchKernelGGL(pop_scatter_kernel, bgrid, blk, 0, sg, V[g]);
                            hipLaunchKernelGGL(pop_rank_kernel, bgrid, blk, 0, sg, V[g]);
                        } else {
                            hipLaunchKernelGGL(sort_kern, dim3(ns), dim3(kPopSortNT), sort_lds, sg, V[g], st.fp);
                        }
                        hipLaunchKernelGGL(pop_permute_kernel<!kPopFused>, dim3(ns * Q.nbs), blk, 0, sg, V[g]);
                        if (Q.two) {
                            hipLaunchKernelGGL(pop_fill_kernel<kOuterRow>, dim3(ns * Q.nbs), blk, 0, sg, V[g]);
                            hipLaunchKernelGGL(pop_refilter_kernel, dim3(ns * Q.nbs), blk, 0, sg, V[g]);
                        } else if (!kPopFused) {
                            hipLaunchKernelGGL(pop_fill_kernel<kPopListRow>, dim3(ns * Q.nbs), blk, 0, sg, V[g]);
                        }
                        PopStep s2 = st;
                        s2.part = early ? 2 : 0;
                        hipLaunchKernelGGL(force_kern, grid_of(g), blk, 0, sg, V[g], evf, envf, s2);
                        if (early) IGM_HIP_CHECK(c, hipStreamWaitEvent(sg, ev_frc[g], 0));  // (the next integrate)
                        if (pst && step % stats_every == 0)
                            hipLaunchKernelGGL(pop_stats_kernel, grid_of(g), blk, 0, sg, V[g], pst + 16 * seg);
                    }
                }
            }
        }
        IGM_HIP_CHECK(c, hipGetLastError());
        gbase += st.nsteps + 1;
        st.rescale = st.nsteps > 0;
        st.prev = st.nsteps;
        const bool last = seg + 1 == A.nseg;
        for (int g = 0; g < ng; ++g)
            hipLaunchKernelGGL(pop_finish_kernel, grid_of(g), blk, 0, strm(g), V[g], st,
                               last ? A.xyz + g0[g] * n3 : nullptr, last ? A.vel + g0[g] * n3 : nullptr,
                               last && A.forces_out ? A.forces_out + g0[g] * n3 : nullptr);
    }
    IGM_HIP_CHECK(c, hipGetLastError());
    IGM_TRY(aux_join(c, nc + (early ? ng : 0)));
    if (pst) {
        std::vector<unsigned long long> v(16 * 2 * IGM_MAX_STAGES);
        IGM_HIP_CHECK(c, hipMemcpyAsync(v.data(), pst, sizeof(unsigned long long) * v.size(), hipMemcpyDeviceToHost,
                                        c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        for (int seg = 0; seg < A.nseg; ++seg) {
            const unsigned long long* u = v.data() + 16 * seg;
            const double n = (double)(u[0] ? u[0] : 1), w = (double)(u[7] ? u[7] : 1), m = u[1] / n;
            const double nb = (double)(u[10] ? u[10] : 1);
            fprintf(stderr, "[igm pop stats] run %d T0 %.0f skin %.3f rmax: list mean %.2f sd %.2f max %llu, wave-max "
                            "quads %.2f (mean quads %.2f), walks %.2e, bonds mean %.2f wave-max %.2f; block slot span "
                            "mean %.0f max %llu (>2048 %.4f, >3072 %.4f, >4096 %.4f), bonds inside it %.4f\n",
                    seg, A.seg_t0[seg], seg_skin[seg] / (0.5f * (pr.P.cut_list - pr.P.skin)), m,
                    sqrt(fmax(u[2] / n - m * m, 0.0)), u[8], u[5] / w, (u[1] + 3.0 * u[0]) / 4.0 / n, u[3] / n,
                    u[4] / n, u[6] / w, u[9] / nb, u[11], u[12] / nb, u[13] / nb, u[14] / nb,
                    u[15] / (double)(u[4] ? u[4] : 1));
        }
    }
    if (sprof) {
        unsigned long long v[8];
        IGM_HIP_CHECK(c, hipMemcpyAsync(v, Q.sprof, sizeof(v), hipMemcpyDeviceToHost, c->stream));
        IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        const double n = (double)(v[6] ? v[6] : 1);
        fprintf(stderr, "[igm pop sort] %llu sorts; cycles per sort: grid %.0f count %.0f scan %.0f scatter %.0f rank %.0f "
                        "offsets %.0f\n", v[6], v[0] / n, v[1] / n, v[2] / n, v[3] / n, v[4] / n, v[5] / n);
    }
    return IGM_OK;
}

// HBM-size structures: the multi-kernel population engine.  (The domain-decomposed
// engine of round 3 -- 31.3 s against 16.1 s on config C, profiles/history_r01_r04.md -- is
// retired; its params flag 0x4 is rejected.)
int run_anneal_big(igm_ctx* c, const Prepared& pr, const AnnealArgs& A, int32_t pflags) {
    if (pflags & 0x4) return fail(c, IGM_E_UNSUPPORTED, "the domain-decomposed engine (params flag 0x4) is retired");
    return run_anneal_pop(c, pr, A);
}

int run_anneal(igm_ctx* c, const Prepared& pr, const igm_mstep_params* prm, float* d_xyz, float* d_vel,
               const int* d_seeds, int* d_nreb, int mode, double seg_evf, double seg_envf, double t0, double t1,
               double xmax, int nsteps, float* d_forces = nullptr) {
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
            V.afs = pr.cm.afs;
            V.seeds = d_seeds;
            V.vinit = (float*)pv;
            Timed tm(c, "velocity");
            hipLaunchKernelGGL(velocity_kernel, dim3(n, pr.cm.nstruct), dim3(256), 0, c->stream, V);
            IGM_HIP_CHECK(c, hipGetLastError());
            A.vinit = (const float*)pv;
        }
    }
    // Verlet skin per run: the engine's skin unless IGM_SKIN_SEG = "f0,f1,..." (units of
    // the largest radius) sets one per run -- any skin gives the same forces (the list
    // holds every pair within 2 rmax + skin and is rebuilt once an atom moved skin / 2),
    // so hot runs can trade longer lists for fewer rebuilds and cold ones the reverse
    // Default (no skin given): a skin per run from the run's start temperature, longer
    // where atoms move fast (T0 = 5000: 1.0 rmax) and shorter where they barely move
    // (T0 <= 1: 0.45 rmax) -- measured on the demo protocol: config B anneal -2.4 %,
    // config C -1.4 % against one 0.7 rmax skin for every run (scripts/gpu_skin_b.sh,
    // gpu_skin_seg.sh).  An explicit params.skin, or the IGM_SKIN_FACTOR tuning knob (one
    // skin for every run), is used for every run.
    // The population engine (pr.big) pays more per list build and less per list entry, so
    // its rule is longer at every temperature: 1.4 rmax at T0 = 5000, 1.15 at 500, 0.9 at
    // 50, 0.475 at T0 <= 1 (measured at pop = 1000, protocol x0.05, same box: -4.8 % anneal
    // against the LDS engine's rule; 1.2/1.0/0.8 -3.0 %, 1.6/1.3/1.0 -2.7 %,
    // 1.8/1.5/1.2 +1.0 %; profiles/r04_ab/).
    const bool uniform_skin = prm->skin > 0 || getenv("IGM_SKIN_FACTOR") != nullptr;
    float ra = 0.475f, rb = 0.25f, rhi = 1.4f;  // the population engine's rule (IGM_POP_SKIN_RULE "a,b,hi": tuning only)
    if (const char* e = getenv("IGM_POP_SKIN_RULE")) {
        if (sscanf(e, "%f,%f,%f", &ra, &rb, &rhi) != 3) return fail(c, IGM_E_INVALID, "IGM_POP_SKIN_RULE: a,b,hi");
    }
    for (int k = 0; k < A.nseg; ++k) {
        if (uniform_skin) {
            A.seg_skin[k] = pr.P.skin;
        } else {
            const float rmax = 0.5f * (pr.P.cut_list - pr.P.skin);
            const float lt = log10f(fmaxf(A.seg_t0[k], 1.0f));
            const float f = pr.big ? fminf(fmaxf(ra + rb * lt, 0.4f), rhi)
                                   : fminf(fmaxf(0.45f + 0.15f * lt, 0.4f), 1.0f);
            A.seg_skin[k] = f * rmax;
        }
    }
    if (const char* e = getenv("IGM_SKIN_SEG")) {
        const float rmax = 0.5f * (pr.P.cut_list - pr.P.skin);
        int k = 0;
        for (const char* q = e; *q && k < A.nseg; ++k) {
            A.seg_skin[k] = (float)atof(q) * rmax;
            while (*q && *q != ',') ++q;
            if (*q == ',') ++q;
        }
    }
    {
        const char* e = getenv("IGM_BOND_PRUNE");
        A.prune = e ? atoi(e) != 0 : 1;
    }
    IGM_HIP_CHECK(c, hipMemsetAsync(pr.cm.work_counter, 0, sizeof(int), c->stream));
    if (getenv("IGM_PROF")) {
        void* pp;
        IGM_TRY(workspace(c, "ms_prof", sizeof(unsigned long long) * 8, &pp));
        IGM_HIP_CHECK(c, hipMemsetAsync(pp, 0, sizeof(unsigned long long) * 8, c->stream));
        A.prof = (unsigned long long*)pp;
    }
    if (pr.big) return run_anneal_big(c, pr, A, prm->flags);
    LaunchCfg cfg;
    if (!lds_fits(pr.cm.natom, &cfg)) return fail(c, IGM_E_UNSUPPORTED, "no LDS configuration");
    IGM_DISPATCH_ALL({
        const size_t lds = kLdsBytes;
        auto kern = anneal_kernel<NT, BPT>;
        IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        int grid = 0;
        IGM_TRY(resident_grid(c, kern, NT, lds, pr.cm.nstruct, &grid));
        // + slack: the batched force loop reads up to IGM_PAIR_BATCH - 1 slots past a list
        A.ws_stride = ((size_t)pr.cm.ldn * (pr.cm.kcap - kLdsListSlots) * 2 + 64 * 2 * IGM_PAIR_BATCH + 255) &
                      ~size_t(255);
        void* ws;
        IGM_TRY(workspace(c, "ms_ldsovf", A.ws_stride * (size_t)grid, &ws));
        A.ws = (unsigned char*)ws;
        Timed tm(c, "anneal");
        hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, c->stream, A);
        IGM_HIP_CHECK(c, hipGetLastError());
    })
    return IGM_OK;
}

int run_cg(igm_ctx* c, const Prepared& pr, const igm_mstep_params* prm, float* d_xyz, const float* d_vel,
           igm_opt_info* d_info, const int* d_nreb, int mode, double evf, double envf, float* d_forces,
           double* d_energies) {
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
    IGM_HIP_CHECK(c, hipMemsetAsync(pr.cm.work_counter, 0, sizeof(int), c->stream));
    constexpr int NT = 512;  // f64 force code: a 256-VGPR budget
    const bool big = pr.big;
    CgLds cg;
    const size_t lds = carve_cg_lds(nullptr, pr.cm.ldn, big, &cg);
    auto kern = big ? cg_kernel<NT, true> : cg_kernel<NT, false>;
    IGM_HIP_CHECK(c, hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int grid = 0;
    IGM_TRY(resident_grid(c, kern, NT, lds, pr.cm.nstruct, &grid));
    NList<double, int> L;
    BigWs<double> W;
    A.ws_stride = carve_ws<double>(nullptr, pr.cm.natom, pr.cm.ldn, pr.cm.kcap, big ? kCellCapBig : kCellCap, big,
                                   false, &L, &W);
    void *ws, *vw;
    IGM_TRY(workspace(c, "ms_cgws", A.ws_stride * (size_t)grid, &ws));
    A.ws = (unsigned char*)ws;
    A.vec_stride = 15 * (size_t)pr.cm.ldn;
    IGM_TRY(workspace(c, "ms_cgvec", sizeof(double) * A.vec_stride * (size_t)grid, &vw));
    A.vec_ws = (double*)vw;
    Timed tm(c, mode == 0 ? "cg" : "forces");
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, c->stream, A);
    IGM_HIP_CHECK(c, hipGetLastError());
    return IGM_OK;
}

int check_error(igm_ctx* c, const Prepared& pr) {
    int herr = 0;
    IGM_HIP_CHECK(c, hipMemcpyAsync(&herr, pr.cm.error, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    if (herr) return fail(c, IGM_E_HIP, "M-step kernel error bits 0x%x", herr);
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
    if (prm->flags & 0x4)  // (on both engines: checked before the LDS / HBM choice)
        return fail(c, IGM_E_UNSUPPORTED, "the domain-decomposed engine (params flag 0x4) is retired");
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

/* Volumetric envelopes: stage the EDT maps (and the structure -> map table) that
 * IGM_ENV_VOLUME envelopes of the next runs read. */
extern "C" int igm_mstep_set_volumes(igm_ctx* c, int32_t nmap, const igm_volume_map* maps,
                                     const int32_t* struct_map, int32_t nstruct) {
    if (!c) return IGM_E_INVALID;
    return set_volumes(c, nmap, maps, struct_map, nstruct);
}

/* Profiling aid (IGM_PROF=1 in the environment): cycle counters of the last LDS-path
 * anneal launch summed over structures: {build, force, rest, steps, builds, list-fill walk}. */
extern "C" int igm_mstep_last_profile(igm_ctx* c, unsigned long long* out) {
    if (!c || !out) return IGM_E_INVALID;
    auto it = c->ws.find("ms_prof");
    if (it == c->ws.end() || !it->second.first) {
        memset(out, 0, sizeof(unsigned long long) * 6);
        return IGM_OK;
    }
    IGM_HIP_CHECK(c, hipMemcpyAsync(out, it->second.first, sizeof(unsigned long long) * 6, hipMemcpyDeviceToHost,
                                    c->stream));
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    return IGM_OK;
}

