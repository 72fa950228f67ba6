// Domain-decomposed LDS engine (the M-step of structures too large for one CU's LDS:
// the 200 kb model, 29 838 beads).  Included by mstep.hip inside igm::ms after the
// LDS anneal kernel, whose force and list-build code it reuses.
//
// One structure is cut into K spatial domains (a kd-tree of K leaves: recursive
// quantile splits along the longest side of each node's box), and each domain is one
// 1024-thread workgroup that owns the atoms inside its box for the WHOLE protocol
// (one launch, 47 000 MD steps).  The K workgroups of a structure form a slot; slots
// run side by side (K x nslot workgroups, one per CU, all resident: a cooperative
// launch checks it).  Per workgroup, as in anneal_kernel:
//   * LDS: float4 positions of the RESIDENT atoms -- owned ones first (atom-id order),
//     then the halo (beads within cut_list of the box, and the bond partners of the
//     owned atoms), the build-time cell grid and the first 8 Verlet-list slots of
//     every owned atom; velocities, forces and last-build positions in VGPRs.
//   * the owned atoms' bonds re-indexed to resident locals (HBM, private, L2-hot).
// Per MD step the domains of a slot meet twice through a counter in HBM:
//   A  after the position update: every owner has stored its atoms' positions (by atom
//      id, write-through sc1 stores) and its displacement vote; each domain then reads
//      the halo positions back (sc1 loads) -- or, when any atom of the structure moved
//      past skin/2 (LAMMPS 'check yes' over the whole structure), re-cuts if the
//      domains are out of balance, re-classifies every atom and rebuilds its lists;
//   B  after the forces and the final kick: the K kinetic-energy partials, summed in
//      domain order (fix temp/rescale of the whole structure), bitwise the same in
//      every domain.
// Hand-offs follow the guide's write-through form (MI355X_MICROARCH.md, visibility
// table row 1): every handed-off byte is stored sc1 and read sc1, every storing wave
// drains its stores (vmcnt 0) before the workgroup barrier, one lane adds to the
// slot's counter (agent scope) and polls it (relaxed, sc1, s_sleep); every spin is
// bounded in time and checks a launch-wide abort word, so a capacity overflow or a
// missing workgroup ends the launch (the host then reruns the batch on the
// multi-kernel population engine) instead of hanging it.
// Every reduction has a fixed order and the domain cut is a deterministic function
// of the published positions, so a run is bitwise reproducible.
#pragma once

constexpr int kDdNT = 1024;
constexpr int kDdMaxK = 32;                // domains per structure
constexpr int kDdHeap = 64;                // kd-tree nodes, heap order (root 1)
constexpr int kDdCellCap = 2048;           // cells of a domain's build grid
// per workgroup shape: BPT owned atoms per thread; the resident (owned + halo) cap takes
// the LDS the smaller owned arrays leave (measured halo shares on annealed 200 kb
// structures: 43 % of the owned atoms at 12 domains, 59 % at 16, 75 % at 24)
__host__ __device__ constexpr int dd_own_cap(int nt, int bpt) { return nt * bpt; }
__host__ __device__ constexpr int dd_res_cap(int nt, int bpt) { return nt * bpt <= 2304 ? 5120 : 4096; }
constexpr int kDdBins = 256;               // histogram bins of a quantile split
constexpr int kDdSyncWords = 32;           // one 128-byte line per slot counter

struct DdArgs {
    AnnealArgs A;
    int K;          // domains (workgroups) per structure
    int nslot;      // structures in flight
    int bdmax;      // bond slots per owned atom
    int kg;         // Verlet-list overflow slots per owned atom (HBM)
    size_t gstride;  // bytes of one workgroup's list-overflow region
    float4* X;      // (nslot, natom) published positions, w = radius code
    float4* V;      // (nslot, natom) velocities handed over at a rebuild
    unsigned long long* ke;  // (nslot, kDdMaxK) kinetic-energy partials (f64 bits)
    int* vote;      // (nslot, kDdMaxK) displacement votes
    unsigned* sync;  // (nslot, kDdSyncWords) barrier counters
    int* abort;     // 1: capacity, 2: spin time limit
    uint32_t* bell;  // (grid, own cap / 64, bdmax, 64) owned atoms' bonds, partners as locals
    unsigned char* gell;  // (grid, gstride)
    float tol;      // re-cut when the largest domain holds more than (1 + tol) natom / K
    long long tmo;  // spin limit of one barrier, wall-clock ticks
    unsigned long long* stats;  // (8) builds, re-cuts, largest resident set (demand), largest owned set,
                                //     largest geometric halo, sums of resident / owned / halo sets over builds
    unsigned long long* prof;   // optional (kDdProf): wall-clock ticks per phase, summed over workgroups
};

// phases of the optional profile (thread 0 of every workgroup, wall clock)
enum {
    kPfIntegrate = 0,  // kick, drift, publish, vote
    kPfBarA,           // barrier A
    kPfHandOver,       // velocity hand-over + its barrier (rebuild steps)
    kPfScan,           // classification scans
    kPfRecut,          // kd cuts
    kPfBonds,          // resident set, bond partners, positions, bond re-index
    kPfList,           // Verlet lists
    kPfHalo,           // halo refresh
    kPfForce,          // forces
    kPfBarB,           // kinetic-energy sum + barrier B (setup steps: their barrier)
    kPfSteps,          // MD steps (count)
    kPfBuilds,         // builds (count)
    kDdProf = 16
};

// LDS of one domain.  The list region doubles as the build's scratch: the
// classification bitmaps, their prefix counts and the quantile histograms live there
// between a rebuild's start and its list build.
struct DdLds {
    Red r;
    float4* pos;      // resident cap: owned atoms, then the halo
    uint16_t* lid;    // resident cap: atom id of a local
    NList<float, uint16_t> L;
    float* cut;       // kDdHeap split value of a node
    int* dim;         // kDdHeap split axis of a node
    float* nbox;      // kDdHeap * 6 node boxes (lo, hi) while cutting
    float* hb;        // 2 * 16: histogram origin and 1/width of the nodes of a level
    float* box;       // 8: this domain's box lo[3], hi[3]
    float* gbb;       // 8: bounding box of the structure lo[3], hi[3]
    int* cnt;         // kDdMaxK atoms per domain under the current cut
    int* iv;          // 16 misc ints
    double* dv;       // 4 misc doubles
    unsigned long long* pf;  // kDdProf profile accumulators (thread 0)
    int nw;           // 32-bit words of a bitmap over the atom ids (even)
    uint32_t* bmO;    // owned by this domain
    uint32_t* bmH;    // resident halo
    int* pO;          // nw + 1 exclusive prefix popcounts
    int* pH;
    int* hist;        // 16 * kDdBins
    size_t bytes;     // LDS bytes of the carve
    size_t alias_bytes;
};

enum { kIvOwn = 0, kIvRes = 1, kIvAny = 2, kIvOk = 3, kIvHaveCut = 4 };

__host__ __device__ inline DdLds carve_dd_lds(void* smem, int natom, int nt, int bpt) {
    const int own = dd_own_cap(nt, bpt), res = dd_res_cap(nt, bpt);
    Carver cv(smem);
    DdLds m;
    m.r = carve_red<float>(cv, &m.L.gp, &m.L.gn);
    m.pos = cv.take<float4>(res);
    m.lid = cv.take<uint16_t>(res);
    m.L.cell = cv.take<uint16_t>(kDdCellCap + 8);
    m.L.nnb = cv.take<uint16_t>(own);
    m.L.sorted = cv.take<uint16_t>(res);
    m.cut = cv.take<float>(kDdHeap);
    m.dim = cv.take<int>(kDdHeap);
    m.nbox = cv.take<float>(kDdHeap * 6);
    m.hb = cv.take<float>(32);
    m.box = cv.take<float>(8);
    m.gbb = cv.take<float>(8);
    m.cnt = cv.take<int>(kDdMaxK);
    m.iv = cv.take<int>(16);
    m.dv = cv.take<double>(4);
    m.pf = cv.take<unsigned long long>(kDdProf);
    m.L.lell = cv.take<uint16_t>((size_t)kLdsListSlots * own);
    m.L.lstride = own;
    m.L.kl = kLdsListSlots;
    m.L.scratch = reinterpret_cast<int*>(m.L.lell);
    m.L.gell = nullptr;
    m.L.kg = 0;
    m.L.cellcap = kDdCellCap;
    m.bytes = cv.o;
    m.nw = (natom + 63) / 64 * 2;
    Carver ca(m.L.lell);
    m.bmO = ca.take<uint32_t>(m.nw);
    m.bmH = ca.take<uint32_t>(m.nw);
    m.pO = ca.take<int>(m.nw + 1);
    m.pH = ca.take<int>(m.nw + 1);
    m.hist = ca.take<int>(16 * kDdBins);
    m.alias_bytes = ca.o;
    return m;
}

// the list region must hold the aliases and the build scratch
__host__ __device__ inline bool dd_lds_ok(int natom, int nt, int bpt) {
    const DdLds m = carve_dd_lds(nullptr, natom, nt, bpt);
    const size_t lell = sizeof(uint16_t) * (size_t)kLdsListSlots * dd_own_cap(nt, bpt);
    return m.bytes <= kLdsBytes && m.alias_bytes <= lell &&
           build_scratch_bytes(kDdCellCap, dd_res_cap(nt, bpt)) <= lell;
}

typedef unsigned int dd_u4 __attribute__((ext_vector_type(4)));

// a float4 array of the slot as a buffer resource (uniform base: readfirstlane)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dd_rsrc(const float4* p, int n) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* u = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(u, (short)0, __builtin_amdgcn_readfirstlane(n * 16), 0x00020000);
}
// write-through (sc1) 16-byte load / store of element j
__device__ __forceinline__ float4 dd_ld(__amdgpu_buffer_rsrc_t r, uint32_t j) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, j * 16u, 0, 16);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
__device__ __forceinline__ void dd_st(__amdgpu_buffer_rsrc_t r, uint32_t j, const float4& x) {
    const dd_u4 v = {__float_as_uint(x.x), __float_as_uint(x.y), __float_as_uint(x.z), __float_as_uint(x.w)};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, j * 16u, 0, 16);
}

// Barrier of the slot's K domains.  Every thread calls it; thread 0 arrives, polls and,
// once all K have arrived, runs `f0` (it reads the handed-off words); the other
// threads wait at the workgroup barrier.  False (every thread) when the launch aborted.
template <typename F>
__device__ __forceinline__ bool dd_barrier(const DdArgs& D, unsigned* ctr, unsigned& nbar, int* okl, F&& f0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's hand-off stores are done
    __syncthreads();
    ++nbar;
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = nbar * (unsigned)D.K;
        int ok = 1;
        const long long t0 = wall_clock64();
        for (unsigned spin = 1; __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin) {
            __builtin_amdgcn_s_sleep(1);
            if ((spin & 31) == 0) {
                if (__hip_atomic_load(D.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    ok = 0;
                    break;
                }
                if (wall_clock64() - t0 > D.tmo) {
                    __hip_atomic_store(D.abort, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
            }
        }
        if (ok) f0();
        *okl = ok;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler order only: the payload loads are sc1
    __syncthreads();
    return *okl != 0;
}

// leaf [lo, hi) range of heap node h (the bits of h below its leading one, from the root)
__device__ __forceinline__ void dd_node_range(int h, int K, int& lo, int& hi) {
    lo = 0;
    hi = K;
    const int depth = 31 - __builtin_clz(h);
    for (int b = depth - 1; b >= 0; --b) {
        const int mid = lo + ((hi - lo) >> 1);
        if ((h >> b) & 1)
            lo = mid;
        else
            hi = mid;
    }
}

__device__ __forceinline__ float dd_coord(const float4& p, int dm) { return dm == 0 ? p.x : (dm == 1 ? p.y : p.z); }

extern __shared__ __attribute__((aligned(16))) unsigned char dd_lds[];

// (Re)build the domain of structure s: classify every atom under the cut (re-cut first
// when there is none or the domains are out of balance), the resident set, its
// positions, the owned atoms' bonds as locals, the Verlet lists.  Leaves the owned and
// resident counts in LDS; false (the launch's abort word set) past a capacity.  LDS
// goes through the namespace-scope dynamic-shared symbol.  (Measured: out of line, the
// call kept the step loop's registers in stack slots -- config C x0.02 anneal 860 ms
// against 735 ms inlined -- so it is inlined.)
template <int NT, int BPT>
__device__ __forceinline__ bool dd_build(const DdArgs& D, int s, float cut_list) {
    constexpr int NW = NT / 64;
    constexpr int kOwnCap = dd_own_cap(NT, BPT), kResCap = dd_res_cap(NT, BPT);
    const AnnealArgs& A = D.A;
    const int N = A.cm.natom;
    DdLds sm = carve_dd_lds(dd_lds, N, NT, BPT);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int K = D.K, slot = blockIdx.x / K, d = blockIdx.x - slot * K;
    const __amdgpu_buffer_rsrc_t rX = dd_rsrc(D.X + (size_t)slot * N, N);
    sm.L.gell = reinterpret_cast<uint16_t*>(D.gell + (size_t)blockIdx.x * D.gstride);
    sm.L.kg = D.kg;
    const int bdmax = D.bdmax;
    uint32_t* bell = D.bell + (size_t)blockIdx.x * (kOwnCap / 64) * bdmax * 64;
    const int nit = (N + NT - 1) / NT;  // scan rounds: wave w takes ids [it*NT + 64w, +64)
    const bool prof = D.prof != nullptr;
    long long tmark = prof ? wall_clock64() : 0;
    auto mark = [&](int k) {
        if (prof && t == 0) {
            const long long now = wall_clock64();
            sm.pf[k] += (unsigned long long)(now - tmark);
            tmark = now;
        }
    };
    auto count = [&](int k) {
        if (prof && t == 0) sm.pf[k] += 1ull;
    };
    bool have_cut = sm.iv[kIvHaveCut] != 0;
    int n_own = 0, n_res = 0;

    // leaf (domain) of position p under the current cut
    auto leaf_of = [&](const float4& p) {
        int h = 1, lo = 0, hi = K;
        while (hi - lo > 1) {
            const int mid = lo + ((hi - lo) >> 1);
            if (dd_coord(p, sm.dim[h]) < sm.cut[h]) {
                hi = mid;
                h = 2 * h;
            } else {
                lo = mid;
                h = 2 * h + 1;
            }
        }
        return lo;
    };
    // exclusive prefix popcounts of a bitmap (pf[nw] = total); ends with a barrier
    auto popc_scan = [&](const uint32_t* bm, int* pf) {
        const int nw = sm.nw, cpt = (nw + NT - 1) / NT, beg = t * cpt;
        int s0 = 0;
        for (int i = 0; i < cpt; ++i)
            if (beg + i < nw) s0 += __builtin_popcount(bm[beg + i]);
        int incl = s0;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) sm.r.wsum[w] = incl;
        __syncthreads();
        int run = incl - s0, total = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int x = sm.r.wsum[i];
            run += i < w ? x : 0;
            total += x;
        }
        for (int i = 0; i < cpt; ++i)
            if (beg + i < nw) {
                pf[beg + i] = run;
                run += __builtin_popcount(bm[beg + i]);
            }
        if (t == 0) pf[nw] = total;
        __syncthreads();
    };
    // one pass over every atom of the structure (published positions): the bounding
    // box and, under a cut, the classification bitmaps and the atoms per domain
    auto scan = [&](bool have_cut, float cut_list) {
        if (t < kDdMaxK) sm.cnt[t] = 0;
        const float b0 = sm.box[0], b1 = sm.box[1], b2 = sm.box[2], b3 = sm.box[3], b4 = sm.box[4], b5 = sm.box[5];
        const float cm = cut_list * 1.0001f, cut2 = cm * cm;  // margin: rounding of the box distance
        float mm[6] = {-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f};
        __syncthreads();
        constexpr int U = 8;  // chunks whose loads are in flight together
        for (int it0 = 0; it0 < nit; it0 += U) {
          float4 pp[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
              const int a = (it0 + u) * NT + w * 64 + lane;
              pp[u] = dd_ld(rX, a < N ? a : 0);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int base = (it0 + u) * NT + w * 64, a = base + lane;
            if (base >= N) break;
            const bool valid = a < N;
            const float4 p = pp[u];
            if (valid) {
                mm[0] = fmaxf(mm[0], -p.x);
                mm[1] = fmaxf(mm[1], -p.y);
                mm[2] = fmaxf(mm[2], -p.z);
                mm[3] = fmaxf(mm[3], p.x);
                mm[4] = fmaxf(mm[4], p.y);
                mm[5] = fmaxf(mm[5], p.z);
            }
            if (!have_cut) continue;
            const int lf = valid ? leaf_of(p) : -1;
            const bool own = lf == d;
            const float dx = fmaxf(fmaxf(b0 - p.x, p.x - b3), 0.0f), dy = fmaxf(fmaxf(b1 - p.y, p.y - b4), 0.0f),
                        dz = fmaxf(fmaxf(b2 - p.z, p.z - b5), 0.0f);
            const bool halo = valid && !own && p.w >= 0.0f && dx * dx + dy * dy + dz * dz < cut2;
            const uint64_t mo = __ballot(own), mh = __ballot(halo);
            if (lane == 0) {
                sm.bmO[base >> 5] = (uint32_t)mo;
                sm.bmO[(base >> 5) + 1] = (uint32_t)(mo >> 32);
                sm.bmH[base >> 5] = (uint32_t)mh;
                sm.bmH[(base >> 5) + 1] = (uint32_t)(mh >> 32);
            }
            for (int k = 0; k < K; ++k) {
                const int c = __builtin_popcountll(__ballot(lf == k));
                if (lane == 0 && c) atomicAdd(&sm.cnt[k], c);
            }
          }
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) mm[q] = wave_max_f32(mm[q]);
        float* redf = reinterpret_cast<float*>(sm.r.redb);
        if (lane == 0)
#pragma unroll
            for (int q = 0; q < 6; ++q) redf[w * 6 + q] = mm[q];
        __syncthreads();
        if (t < 6) {
            float m = redf[t];
            for (int i = 1; i < NW; ++i) m = fmaxf(m, redf[i * 6 + t]);
            sm.gbb[t] = t < 3 ? -m : m;  // lo[3], hi[3]
        }
        __syncthreads();
    };
    // kd cut: level by level, a histogram of every internal node's atoms along the
    // longest side of its box, split at the quantile of its leaf counts
    auto recut = [&]() {
        if (t < 6) sm.nbox[6 + t] = sm.gbb[t];
        __syncthreads();
        for (int L = 0; (1 << L) < K; ++L) {
            const int h0 = 1 << L, nh = h0;  // <= 16 nodes
            if (t < nh) {
                const int h = h0 + t;
                int lo, hi;
                dd_node_range(h, K, lo, hi);
                if (hi - lo > 1) {
                    const float* bx = sm.nbox + 6 * h;
                    int dm = 0;
                    float ext = bx[3] - bx[0];
                    for (int q = 1; q < 3; ++q)
                        if (bx[3 + q] - bx[q] > ext) {
                            ext = bx[3 + q] - bx[q];
                            dm = q;
                        }
                    if (!(ext > 0.0f)) ext = 1.0f;
                    sm.dim[h] = dm;
                    sm.hb[t] = bx[dm];
                    sm.hb[16 + t] = (float)kDdBins / ext;
                }
            }
            for (int k = t; k < nh * kDdBins; k += NT) sm.hist[k] = 0;
            __syncthreads();
            constexpr int U = 8;
            for (int it0 = 0; it0 < nit; it0 += U) {
              float4 pp[U];
#pragma unroll
              for (int u = 0; u < U; ++u) {
                  const int a = (it0 + u) * NT + t;
                  pp[u] = dd_ld(rX, a < N ? a : 0);
              }
#pragma unroll
              for (int u = 0; u < U; ++u) {
                if ((it0 + u) * NT + t >= N) break;
                const float4 p = pp[u];
                int h = 1, lo = 0, hi = K;
                for (int q = 0; q < L && hi - lo > 1; ++q) {
                    const int mid = lo + ((hi - lo) >> 1);
                    if (dd_coord(p, sm.dim[h]) < sm.cut[h]) {
                        hi = mid;
                        h = 2 * h;
                    } else {
                        lo = mid;
                        h = 2 * h + 1;
                    }
                }
                if (hi - lo > 1 && h >= h0) {
                    const int j = h - h0;
                    const float x = (dd_coord(p, sm.dim[h]) - sm.hb[j]) * sm.hb[16 + j];
                    const int bin = x >= 0.0f ? (x < (float)(kDdBins - 1) ? (int)x : kDdBins - 1) : 0;  // NaN -> 0
                    atomicAdd(&sm.hist[j * kDdBins + bin], 1);
                }
              }
            }
            __syncthreads();
            if (w < nh) {  // one wave per node: the quantile bin and the cut inside it
                const int h = h0 + w;
                int lo, hi;
                dd_node_range(h, K, lo, hi);
                if (hi - lo > 1) {
                    constexpr int BPL = kDdBins / 64;
                    int c[BPL], sl = 0;
#pragma unroll
                    for (int q = 0; q < BPL; ++q) {
                        c[q] = sm.hist[w * kDdBins + lane * BPL + q];
                        sl += c[q];
                    }
                    int incl = sl;
#pragma unroll
                    for (int off = 1; off < 64; off <<= 1) {
                        const int y = __shfl_up(incl, off);
                        if (lane >= off) incl += y;
                    }
                    const int total = __shfl(incl, 63);
                    const int mid = lo + ((hi - lo) >> 1);
                    const int target = (int)(((long long)total * (mid - lo)) / (hi - lo));
                    const int dm = sm.dim[h];
                    const float org = sm.hb[w], inv = sm.hb[16 + w];
                    int run = incl - sl;
                    bool found = false;
                    float cutv = org;
#pragma unroll
                    for (int q = 0; q < BPL; ++q) {
                        if (!found && c[q] > 0 && run < target && target <= run + c[q]) {
                            const float fr = (float)(target - run) / (float)c[q];
                            cutv = org + ((float)(lane * BPL + q) + fr) / inv;
                            found = true;
                        }
                        run += c[q];
                    }
                    const uint64_t fm = __ballot(found);
                    const int src = fm ? __builtin_ctzll(fm) : 0;
                    cutv = __shfl(cutv, src);
                    if (lane == 0) {
                        sm.cut[h] = cutv;
                        const float* bx = sm.nbox + 6 * h;
                        float* bl = sm.nbox + 6 * (2 * h);
                        float* br = sm.nbox + 6 * (2 * h + 1);
                        for (int q = 0; q < 6; ++q) {
                            bl[q] = bx[q];
                            br[q] = bx[q];
                        }
                        bl[3 + dm] = cutv;
                        br[dm] = cutv;
                    }
                }
            }
            __syncthreads();
        }
    };
    // this domain's box under the current cut (open sides infinite)
    auto my_box = [&]() {
        if (t == 0) {
            float bx[6] = {-3.0e38f, -3.0e38f, -3.0e38f, 3.0e38f, 3.0e38f, 3.0e38f};
            int h = 1, lo = 0, hi = K;
            while (hi - lo > 1) {
                const int mid = lo + ((hi - lo) >> 1), dm = sm.dim[h];
                if (d < mid) {
                    bx[3 + dm] = fminf(bx[3 + dm], sm.cut[h]);
                    hi = mid;
                    h = 2 * h;
                } else {
                    bx[dm] = fmaxf(bx[dm], sm.cut[h]);
                    lo = mid;
                    h = 2 * h + 1;
                }
            }
            for (int q = 0; q < 6; ++q) sm.box[q] = bx[q];
        }
        __syncthreads();
    };
    auto fail_capacity = [&]() {
        if (t == 0) __hip_atomic_store(D.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
    };

    // (Re)build the domain of structure s: classify every atom under the cut (re-cut
    // first when there is none or the domains are out of balance), the resident set,
    // its positions, the owned atoms' bonds as locals, the Verlet lists.
    {
        bool recut_done = false;
        for (;;) {
            if (have_cut) my_box();
            scan(have_cut, cut_list);
            mark(kPfScan);
            if (have_cut) {
                int mx = 0;
                for (int k = 0; k < K; ++k) mx = max(mx, sm.cnt[k]);
                const bool fits = mx <= kOwnCap;
                const bool balanced = (float)mx <= (1.0f + D.tol) * (float)N / (float)K;
                if (fits && (balanced || recut_done)) break;
                if (recut_done) return fail_capacity();
            }
            recut();
            mark(kPfRecut);
            if (t == 0 && D.stats) atomicAdd(&D.stats[1], 1ull);
            have_cut = true;
            recut_done = true;
        }
        popc_scan(sm.bmO, sm.pO);
        n_own = sm.pO[sm.nw];
        if (n_own > kOwnCap) return fail_capacity();
        for (int k = t; k < sm.nw; k += NT) {
            uint32_t m = sm.bmO[k];
            int o = sm.pO[k];
            while (m) {
                sm.lid[o++] = (uint16_t)(k * 32 + __builtin_ctz(m));
                m &= m - 1u;
            }
        }
        __syncthreads();
        int n_geo = 0;  // the geometric halo (statistics)
        if (D.stats) {
            popc_scan(sm.bmH, sm.pH);
            n_geo = sm.pH[sm.nw];
        }
        // the owned atoms' bond partners join the resident set
        const uint32_t* ent = A.cm.bonds.ent + A.cm.bonds.base[s];
        const int* soff = A.cm.bonds.soff + (size_t)s * (A.cm.nslice + 1);
        const int* deg = A.cm.bonds.deg + (size_t)s * N;
        for (int l = t; l < n_own; l += NT) {
            const int id = sm.lid[l], nd = deg[id];
            const uint32_t* g = ent + soff[id >> 6] + (id & 63);
            for (int k = 0; k < nd; ++k) {
                const uint32_t pj = g[(size_t)k * 64] & 0xffffu;
                if (!((sm.bmO[pj >> 5] >> (pj & 31)) & 1u)) atomicOr(&sm.bmH[pj >> 5], 1u << (pj & 31));
            }
        }
        __syncthreads();
        popc_scan(sm.bmH, sm.pH);
        n_res = n_own + sm.pH[sm.nw];
        if (t == 0 && D.stats) {
            atomicMax(&D.stats[2], (unsigned long long)n_res);
            atomicMax(&D.stats[3], (unsigned long long)n_own);
            atomicMax(&D.stats[4], (unsigned long long)n_geo);
            atomicAdd(&D.stats[5], (unsigned long long)n_res);
            atomicAdd(&D.stats[6], (unsigned long long)n_own);
            atomicAdd(&D.stats[7], (unsigned long long)n_geo);
        }
        if (n_res > kResCap) return fail_capacity();
        for (int k = t; k < sm.nw; k += NT) {
            uint32_t m = sm.bmH[k];
            int o = n_own + sm.pH[k];
            while (m) {
                sm.lid[o++] = (uint16_t)(k * 32 + __builtin_ctz(m));
                m &= m - 1u;
            }
        }
        __syncthreads();
        for (int l = t; l < n_res; l += NT) sm.pos[l] = dd_ld(rX, sm.lid[l]);
        // bonds of the owned atoms with partners as locals (partner local: owned rank, or
        // n_own + halo rank, from the bitmaps' prefix counts)
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const int l = b * NT + t;
            if (l >= n_own) continue;
            const int id = sm.lid[l], nd = deg[id];
            const uint32_t* g = ent + soff[id >> 6] + (id & 63);
            uint32_t* o = bell + (size_t)(l >> 6) * bdmax * 64 + (l & 63);
            for (int k = 0; k < nd; ++k) {
                const uint32_t e = g[(size_t)k * 64], pj = e & 0xffffu, wd = pj >> 5, bit = 1u << (pj & 31);
                const uint32_t below = bit - 1u, mo = sm.bmO[wd];
                const int loc = (mo & bit) ? sm.pO[wd] + __builtin_popcount(mo & below)
                                           : n_own + sm.pH[wd] + __builtin_popcount(sm.bmH[wd] & below);
                o[(size_t)k * 64] = (e & 0xffff0000u) | (uint32_t)loc;
            }
        }
        __syncthreads();  // positions complete; the bitmaps die here (the list build reuses the region)
        mark(kPfBonds);
        build_nlist_lds<NT>(n_res, n_own, sm.pos, sm.L, cut_list, sm.r);
        mark(kPfList);
        count(kPfBuilds);
        if (t == 0) {
            if (D.stats) atomicAdd(&D.stats[0], 1ull);
            sm.iv[kIvOwn] = n_own;
            sm.iv[kIvRes] = n_res;
            sm.iv[kIvHaveCut] = have_cut ? 1 : 0;
        }
        __syncthreads();
        return true;
    }
}

template <int NT, int BPT>
__global__ void __launch_bounds__(NT) dd_anneal_kernel(DdArgs D) {
    constexpr int kOwnCap = dd_own_cap(NT, BPT);
    const AnnealArgs& A = D.A;
    const int N = A.cm.natom;
    DdLds sm = carve_dd_lds(dd_lds, N, NT, BPT);
    const int t = threadIdx.x;
    // optional phase profile: thread 0 charges the wall-clock time since the last mark
    const bool prof = D.prof != nullptr;
    long long tmark = prof ? wall_clock64() : 0;
    if (prof && t < kDdProf) sm.pf[t] = 0ull;
    auto mark = [&](int k) {
        if (prof && t == 0) {
            const long long now = wall_clock64();
            sm.pf[k] += (unsigned long long)(now - tmark);
            tmark = now;
        }
    };
    auto count = [&](int k) {
        if (prof && t == 0) sm.pf[k] += 1ull;
    };
    const int K = D.K, slot = blockIdx.x / K, d = blockIdx.x - slot * K;
    if (slot >= D.nslot) return;
    unsigned* ctr = D.sync + (size_t)slot * kDdSyncWords;
    unsigned nbar = 0;
    const __amdgpu_buffer_rsrc_t rX = dd_rsrc(D.X + (size_t)slot * N, N);
    const __amdgpu_buffer_rsrc_t rV = dd_rsrc(D.V + (size_t)slot * N, N);
    int* vote = D.vote + slot * kDdMaxK;
    unsigned long long* kep = D.ke + slot * kDdMaxK;
    sm.L.gell = reinterpret_cast<uint16_t*>(D.gell + (size_t)blockIdx.x * D.gstride);
    sm.L.kg = D.kg;
    const int bdmax = D.bdmax;
    uint32_t* bell = D.bell + (size_t)blockIdx.x * (kOwnCap / 64) * bdmax * 64;
    int* okl = sm.iv + kIvOk;
    auto nop = [] {};

    float v[BPT][3], f[BPT][3], xb[BPT][3];
    int bdeg[BPT];
    uint32_t mobile = 0u, flk = 0u;
    int n_own = 0, n_res = 0;

    // the per-thread state of the owned atoms after a build (velocities: from the
    // hand-over buffer, or at a run's setup step from the run's velocities)
    auto load_state = [&](int s, const float* vsrc) {
        mobile = 0u;
        flk = 0u;
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const int l = b * NT + t;
            const bool in = l < n_own;
            const int id = in ? sm.lid[l] : 0;
            const float4 p = sm.pos[in ? l : 0];
            bdeg[b] = in ? A.cm.bonds.deg[(size_t)s * N + id] : 0;
            xb[b][0] = p.x;
            xb[b][1] = p.y;
            xb[b][2] = p.z;
            const uint32_t fl = in ? A.cm.aflags[(size_t)s * A.cm.afs + id] : 0u;
            flk |= (((fl & IGM_ATOM_FIXED) ? 1u : 0u) | (((fl >> 4) & 0xfu) << 1)) << (5 * b);
            const bool mob = in && !(fl & IGM_ATOM_FIXED);
            if (mob) mobile |= 1u << b;
            if (vsrc) {  // a run's setup step: the run's 'velocity create'
#pragma unroll
                for (int q = 0; q < 3; ++q) v[b][q] = mob ? vsrc[(size_t)id * 3 + q] : 0.0f;
            } else {
                const float4 vv = mob ? dd_ld(rV, id) : make_float4(0.f, 0.f, 0.f, 0.f);
                v[b][0] = vv.x;
                v[b][1] = vv.y;
                v[b][2] = vv.z;
            }
        }
    };

    for (int s = slot; s < A.cm.nstruct; s += D.nslot) {
        // publish the structure's start positions (a share of the ids per domain)
        {
            const float* xs = A.xyz + (size_t)s * N * 3;
            const int a0 = (int)((long long)N * d / K), a1 = (int)((long long)N * (d + 1) / K);
            int nmob = 0;
            for (int a = a0 + t; a < a1; a += NT) {
                const uint32_t fl = A.cm.aflags[(size_t)s * A.cm.afs + a];
                const float r = A.cm.radii[a];
                dd_st(rX, a, make_float4(xs[(size_t)a * 3], xs[(size_t)a * 3 + 1], xs[(size_t)a * 3 + 2],
                                         (fl & IGM_ATOM_BEAD) ? r : -(r + 1.0f)));
            }
            for (int a = t; a < N; a += NT) nmob += (A.cm.aflags[(size_t)s * A.cm.afs + a] & IGM_ATOM_FIXED) ? 0 : 1;
            double cnt[1] = {(double)nmob};
            block_sum<NT, 1>(cnt, sm.r.red0);
            sm.dv[1] = 3.0 * cnt[0] - 3.0;  // dof of group nonfixed (read after the barrier below)
        }
        if (!dd_barrier(D, ctr, nbar, okl, nop)) return;
        const double dof = sm.dv[1];
        int nbuild = 0;
        if (t == 0) sm.iv[kIvHaveCut] = 0;  // (read by the first build, after barriers)
        n_own = n_res = 0;  // nothing owned yet: the first run's setup step builds
        mobile = 0u;
        float last_skin = -1.0f;
        for (int seg = 0; seg < A.nseg; ++seg) {
            const float* vsrc =
                A.mode == 1 ? A.vel + (size_t)s * N * 3 : A.vinit + ((size_t)s * A.nseg + seg) * N * 3;
#pragma unroll
            for (int b = 0; b < BPT; ++b) {
                const int id = sm.lid[b * NT + t < n_own ? b * NT + t : 0];
#pragma unroll
                for (int q = 0; q < 3; ++q) v[b][q] = (mobile >> b & 1u) ? vsrc[(size_t)id * 3 + q] : 0.0f;
            }
            const int nsteps = A.seg_steps[seg];
            const float evf = A.seg_evf[seg], envf = A.seg_envf[seg];
            const float t0 = A.seg_t0[seg], t1 = A.seg_t1[seg];
            const float dtv = A.dt, dtf = 0.5f * A.dt;
            const float vlim = A.seg_xmax[seg] / dtv, vlimsq = vlim * vlim;
            const float skin = A.seg_skin[seg];
            const float trig = 0.25f * skin * skin;
            const float cut_list = A.P.cut_list - A.P.skin + skin;
            bool force_build = skin != last_skin;  // a new cut: rebuild at the run's setup step
            last_skin = skin;
            for (int step = 0; step <= nsteps; ++step) {
                int moved = force_build ? 1 : 0;
                force_build = false;
#pragma unroll
                for (int b = 0; b < BPT; ++b) {
                    const int l = b * NT + t;
                    if (l >= n_own) continue;
                    float4 p = sm.pos[l];
                    if (step > 0 && (mobile >> b & 1u)) {  // fix nve/limit: initial_integrate
                        kick_limit(v[b][0], v[b][1], v[b][2], f[b][0], f[b][1], f[b][2], dtf, vlim, vlimsq);
                        p.x += dtv * v[b][0];
                        p.y += dtv * v[b][1];
                        p.z += dtv * v[b][2];
                        sm.pos[l] = p;
                    }
                    if (p.w >= 0.0f) {
                        const float ddx = p.x - xb[b][0], ddy = p.y - xb[b][1], ddz = p.z - xb[b][2];
                        moved |= !(ddx * ddx + ddy * ddy + ddz * ddz <= trig);
                    }
                    dd_st(rX, sm.lid[l], p);
                }
                moved = __syncthreads_or(moved);
                if (t == 0) __hip_atomic_store(vote + d, moved, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                mark(kPfIntegrate);
                count(kPfSteps);
                // barrier A: positions of step `step` published; the structure's vote
                if (!dd_barrier(D, ctr, nbar, okl, [&] {
                        int any = 0;
                        for (int k = 0; k < K; ++k) any |= __hip_atomic_load(vote + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        sm.iv[kIvAny] = any;
                    }))
                    return;
                mark(kPfBarA);
                if (sm.iv[kIvAny]) {  // neigh_modify every 1 check yes, over the whole structure
#pragma unroll
                    for (int b = 0; b < BPT; ++b) {
                        const int l = b * NT + t;
                        if (l < n_own) dd_st(rV, sm.lid[l], make_float4(v[b][0], v[b][1], v[b][2], 0.0f));
                    }
                    if (!dd_barrier(D, ctr, nbar, okl, nop)) return;
                    mark(kPfHandOver);
                    if (!dd_build<NT, BPT>(D, s, cut_list)) return;
                    if (prof) tmark = wall_clock64();
                    n_own = sm.iv[kIvOwn];
                    n_res = sm.iv[kIvRes];
                    load_state(s, step == 0 ? vsrc : nullptr);
                    ++nbuild;
                    mark(kPfBonds);
                } else {  // the halo's new positions
                    for (int l = n_own + t; l < n_res; l += NT) sm.pos[l] = dd_ld(rX, sm.lid[l]);
                    __syncthreads();
                    mark(kPfHalo);
                }
                const float2* bt = A.cm.bonds.types + A.cm.bonds.tbase[s];
#pragma unroll 1
                for (int b = 0; b < BPT; ++b) {
                    const int l = b * NT + t;
                    if (l >= n_own) continue;
                    float fx, fy, fz;
                    const BondView B{bell + (size_t)(l >> 6) * bdmax * 64 + (l & 63), bt, nullptr, nullptr,
                                     pick<BPT>(bdeg, b)};
                    const uint32_t f5 = (flk >> (5 * b)) & 31u;
                    const uint32_t fla = ((f5 & 1u) ? IGM_ATOM_FIXED : 0u) | ((f5 >> 1) << 4);
                    atom_force_md<kLdsPairBatch>(s, l, sm.pos[l], fla, sm.pos, sm.L, pick<BPT>(xb, b, 0),
                                                 pick<BPT>(xb, b, 1), pick<BPT>(xb, b, 2), B, A.P, evf, envf, fx, fy,
                                                 fz, n_res - 1);
#pragma unroll
                    for (int i = 0; i < BPT; ++i)
                        if (b == i) {
                            f[i][0] = fx;
                            f[i][1] = fy;
                            f[i][2] = fz;
                        }
                }
                __syncthreads();  // (profile boundary: every wave's forces)
                mark(kPfForce);
                if (step == 0) {  // Verlet::setup: forces only (the barrier keeps the positions until all have read them)
                    if (!dd_barrier(D, ctr, nbar, okl, nop)) return;
                    mark(kPfBarB);
                    continue;
                }
                double ts[1] = {0.0};
#pragma unroll
                for (int b = 0; b < BPT; ++b) {  // final_integrate
                    if (!(mobile >> b & 1u)) continue;
                    kick_limit(v[b][0], v[b][1], v[b][2], f[b][0], f[b][1], f[b][2], dtf, vlim, vlimsq);
#pragma unroll
                    for (int q = 0; q < 3; ++q) ts[0] += (double)(v[b][q] * v[b][q]);
                }
                block_sum<NT, 1>(ts, (step & 1) ? sm.r.red1 : sm.r.red0);
                if (t == 0)
                    __hip_atomic_store(kep + d, (unsigned long long)__double_as_longlong(ts[0]), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                // barrier B: the structure's temperature (partials in domain order)
                if (!dd_barrier(D, ctr, nbar, okl, [&] {
                        double ke = 0.0;
                        for (int k = 0; k < K; ++k)
                            ke += __longlong_as_double(
                                (long long)__hip_atomic_load(kep + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                        sm.dv[0] = ke;
                    }))
                    return;
                mark(kPfBarB);
                const float factor =
                    temp_rescale_factor(sm.dv[0], dof, step, nsteps, t0, t1, A.t_window, A.t_fraction);
                if (factor != 1.0f)
#pragma unroll
                    for (int b = 0; b < BPT; ++b)
#pragma unroll
                        for (int q = 0; q < 3; ++q) v[b][q] *= factor;
            }
        }
        // the owned atoms' results, in atom order
        float* xo = A.xyz + (size_t)s * N * 3;
        float* vo = A.vel + (size_t)s * N * 3;
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const int l = b * NT + t;
            if (l >= n_own) continue;
            const int id = sm.lid[l];
            const float4 p = sm.pos[l];
            xo[(size_t)id * 3] = p.x;
            xo[(size_t)id * 3 + 1] = p.y;
            xo[(size_t)id * 3 + 2] = p.z;
#pragma unroll
            for (int q = 0; q < 3; ++q) vo[(size_t)id * 3 + q] = v[b][q];
            if (A.forces_out) {
                float* fo3 = A.forces_out + ((size_t)s * N + id) * 3;
#pragma unroll
                for (int q = 0; q < 3; ++q) fo3[q] = f[b][q];
            }
        }
        if (d == 0 && t == 0 && A.nrebuild) A.nrebuild[s] = nbuild;
        __syncthreads();
    }
    if (prof && t < kDdProf) atomicAdd(&D.prof[t], sm.pf[t]);
}
