// M-step violation statistics on the GPU: the per-structure record that
// ModelingStep.task builds after the optimisation (ModelingStep.py:511-557) with
// the violation ratios of igm/model/forces.py and get_violation_histogram
// (ModelingStep.py:859-869).  Compiled with -ffp-contract=off: the ratios are
// f64 expressions on f32 coordinates, restated operation by operation, so the
// histogram bins and the (ratio > tol) counts match the reference exactly.
#include "exact_math.h"
#include "igm_ctx.h"
#include "mstep_common.h"

namespace {

constexpr int kRec = 104;  // counts[101], violated_restr, n_violations, n_imposed
constexpr int kMaxClass = 16;

// np.histogram(v, bins=100, range=(0, 1)) bin of a value in [0, 1]
__device__ __forceinline__ int hist_bin(double v) {
    int i = (int)(v * 100.0);  // (a - first_edge) * norm
    if (i >= 100) i = 99;
    if (i < 0) i = 0;
    const double lo = (double)i * 0.01;                     // linspace(0, 1, 101)[i]
    const double hi = (i + 1 == 100) ? 1.0 : (double)(i + 1) * 0.01;
    if (v < lo) --i;
    else if (v >= hi && i != 99) ++i;
    return i;
}

__device__ __forceinline__ void record(int* h, double v, double tol) {
    if (v > 1.0) atomicAdd(&h[100], 1);  // overflow (v > vmax)
    else atomicAdd(&h[hist_bin(v)], 1);
    if (v != 0.0) atomicAdd(&h[101], 1);
    if (v > tol) atomicAdd(&h[102], 1);
    atomicAdd(&h[103], 1);
}

__device__ __forceinline__ float norm_f32(const float* a, const float* b) {
    const float dx = __fsub_rn(a[0], b[0]), dy = __fsub_rn(a[1], b[1]), dz = __fsub_rn(a[2], b[2]);
    return igm::sqrtf_rn(__fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
}

struct VArgs {
    int nstruct, natom, nclass_bonds, nenv;
    const float* xyz;
    const float* radii;
    const uint32_t* aflags;
    size_t afs;  // aflags stride between structures (IGM_MSTEP_STRUCT_FLAGS) or 0
    const igm_bond* shared;
    const int32_t* shared_class;
    int64_t nshared;
    const int64_t* sptr;
    const igm_bond* sbonds;
    const int32_t* sclass;
    double class_cr[kMaxClass];
    double env_abc[IGM_MAX_ENVELOPES][3];
    double env_k[IGM_MAX_ENVELOPES];
    double env_scale[IGM_MAX_ENVELOPES];  // ellipsoid: violation scale; volume: contact_range
    int env_kind[IGM_MAX_ENVELOPES];
    const igm::ms::VolMapDev* vmaps;       // volume maps (igm_mstep_set_volumes)
    const int4* vvox;
    const int* vsmap;
    double tol;
    int64_t* stats;
};

// ExpEnvelope.getScores (igm/model/forces.py:306-417) of one particle, restated with its
// NumPy semantics: f32 position minus float64 origin over float64 grid, round half to
// even, -1 outside the grid; the reference's inside-grid test `id_int.all() >= 0` is
// always true, so a -1 index reads the last voxel (Python negative indexing) and the
// score uses the -1 itself.
__device__ double volume_score(const float* p, const igm::ms::VolMapDev& m, const int4* vox, double k, double cr) {
    double o[3], g[3];
    int id[3], w[3];
    for (int d = 0; d < 3; ++d) {
        o[d] = (double)m.origin[d];
        g[d] = (double)m.grid[d];
        if (m.body == 0 && k < 0.0) {
            o[d] = o[d] * cr;
            g[d] = g[d] * cr;
        }
        if (m.body == 1 && k < 0.0) {
            o[d] = o[d] / cr;
            g[d] = g[d] / cr;
        }
        const double ix = ((double)p[d] - o[d]) / g[d];
        id[d] = (ix < 0.0 || ix >= (double)m.n[d]) ? -1 : (int)rint(ix);
        if (id[d] >= m.n[d]) id[d] = m.n[d] - 1;  // the reference raises IndexError here
        w[d] = id[d] < 0 ? m.n[d] - 1 : id[d];
    }
    const int4 r = vox[m.off + ((long long)w[0] * m.n[1] + w[1]) * m.n[2] + w[2]];
    const bool cond = (m.body == 0) ? ((r.w == 0 && k > 0.0) || (r.w != 0 && k < 0.0))
                                    : ((r.w != 0 && k > 0.0) || (r.w == 0 && k < 0.0));
    if (!cond) return 0.0;
    const double v0 = g[0] * (double)(r.x - id[0]), v1 = g[1] * (double)(r.y - id[1]),
                 v2 = g[2] * (double)(r.z - id[2]);
    // np.linalg.norm = sqrt(ddot): the reference BLAS sums (x0^2 + x2^2) + x1^2
    return igm::sqrt_rn((v0 * v0 + v2 * v2) + v1 * v1) / igm::sqrt_rn((g[0] * g[0] + g[2] * g[2]) + g[1] * g[1]);
}

__global__ void __launch_bounds__(256) violations_kernel(VArgs A) {
    __shared__ int h[kMaxClass * kRec];
    const int s = blockIdx.x, t = threadIdx.x;
    const int ncls = A.nclass_bonds + A.nenv;
    for (int k = t; k < ncls * kRec; k += 256) h[k] = 0;
    __syncthreads();
    const float* x = A.xyz + (size_t)s * A.natom * 3;
    const int64_t b0 = A.sptr ? A.sptr[s] : 0, b1 = A.sptr ? A.sptr[s + 1] : 0;
    const int64_t nb = A.nshared + (b1 - b0);
    for (int64_t q = t; q < nb; q += 256) {
        const bool sh = q < A.nshared;
        const igm_bond bd = sh ? A.shared[q] : A.sbonds[b0 + q - A.nshared];
        const int c = sh ? (A.shared_class ? A.shared_class[q] : 0) : (A.sclass ? A.sclass[b0 + q - A.nshared] : 0);
        if (c < 0 || c >= A.nclass_bonds) continue;
        const uint32_t i = bd.i, j = bd.j & 0x7fffffffu;
        const bool lower = (bd.j >> 31) != 0u;
        const double dist = (double)norm_f32(x + 3 * i, x + 3 * j);  // Particle.__sub__ (f32)
        const double cr = A.class_cr[c];
        const double d = cr > 0.0 ? cr * (double)__fadd_rn(A.radii[i], A.radii[j]) : (double)bd.r0;
        const double k = (double)bd.k;
        double ratio = 0.0;
        if (d != 0.0) {
            double score = 0.0;
            if (!lower) score = (dist <= d) ? 0.0 : k * (dist - d);   // HarmonicUpperBound.getScore
            else score = (dist >= d) ? 0.0 : k * (d - dist);          // HarmonicLowerBound.getScore
            ratio = score / (k * d);
        }
        record(&h[c * kRec], ratio, A.tol);
    }
    // EllipticEnvelope.getScores (forces.py:222-247)
    for (int e = 0; e < A.nenv; ++e) {
        int* he = &h[(A.nclass_bonds + e) * kRec];
        for (int a = t; a < A.natom; a += 256) {
            if (!(A.aflags[(size_t)s * A.afs + a] & (IGM_ATOM_ENV0 << e))) continue;
            const float* p = x + 3 * a;
            if (A.env_kind[e] == IGM_ENV_VOLUME) {
                record(he, volume_score(p, A.vmaps[A.vsmap ? A.vsmap[s] : 0], A.vvox, A.env_k[e], A.env_scale[e]),
                       A.tol);
                continue;
            }
            const double r = (double)A.radii[a];
            double acc = 0.0;
            for (int d = 0; d < 3; ++d) {
                const double s2 = (A.env_abc[e][d] - r) * (A.env_abc[e][d] - r);
                const float x2 = __fmul_rn(p[d], p[d]);  // x**2 in f32
                acc = acc + (double)x2 / s2;
            }
            const double k2 = igm::sqrt_rn(acc);
            double tv = 0.0;
            if (k2 > 1.0 && A.env_k[e] > 0.0) {
                const float nrm = igm::sqrtf_rn(__fadd_rn(__fadd_rn(__fmul_rn(p[0], p[0]), __fmul_rn(p[1], p[1])),
                                                          __fmul_rn(p[2], p[2])));
                tv = (1.0 - 1.0 / igm::sqrt_rn(k2)) * (double)nrm / A.env_scale[e];
            } else if (k2 < 1.0 && A.env_k[e] < 0.0) {
                tv = 1.0 - igm::sqrt_rn(k2);
            }
            record(he, tv > 0.0 ? tv : 0.0, A.tol);
        }
    }
    __syncthreads();
    for (int k = t; k < ncls * kRec; k += 256) A.stats[(size_t)s * ncls * kRec + k] = h[k];
}

}  // namespace

extern "C" int igm_mstep_violations(igm_ctx* c, uint32_t flags, const igm_mstep_params* prm, int32_t nstruct,
                                    int32_t natom, const float* xyz, const float* radii, const uint32_t* atom_flags,
                                    const igm_bond* shared_bonds, const int32_t* shared_class, int64_t nshared,
                                    const int64_t* sbond_ptr, const igm_bond* sbonds, const int32_t* sclass,
                                    int32_t nclass_bonds, const double* class_cr, const double* env_scale, double tol,
                                    int64_t* stats) {
    using namespace igm;
    if (!c || !prm || nstruct <= 0 || natom <= 0 || !xyz || !radii || !atom_flags || !stats || nclass_bonds < 0 ||
        nclass_bonds + prm->nenvelopes > kMaxClass || !class_cr)
        return fail(c, IGM_E_INVALID, "igm_mstep_violations: invalid arguments");
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    VArgs A;
    memset(&A, 0, sizeof(A));
    A.nstruct = nstruct;
    A.natom = natom;
    A.nclass_bonds = nclass_bonds;
    A.nenv = prm->nenvelopes;
    A.nshared = nshared;
    A.tol = tol;
    for (int k = 0; k < nclass_bonds; ++k) A.class_cr[k] = class_cr[k];
    for (int e = 0; e < A.nenv; ++e) {
        for (int d = 0; d < 3; ++d) A.env_abc[e][d] = prm->env_semiaxes[e][d];
        A.env_k[e] = prm->env_k[e];
        A.env_scale[e] = env_scale ? env_scale[e] : 0.1 * (prm->env_semiaxes[e][0] + prm->env_semiaxes[e][1] +
                                                             prm->env_semiaxes[e][2]) / 3.0;
        A.env_kind[e] = prm->env_kind[e];
        if (A.env_kind[e] == IGM_ENV_VOLUME) {
            if (!env_scale) A.env_scale[e] = 0.95;  // GenEnvelope's contact_range (genenvelope.py:48-58)
            if (c->vol_nmap <= 0) return fail(c, IGM_E_INVALID, "igm_mstep_violations: no volume map staged");
            if (c->vol_nsmap > 0 && c->vol_nsmap < nstruct)
                return fail(c, IGM_E_INVALID, "igm_mstep_violations: volume map index staged for %d structures",
                            c->vol_nsmap);
            void *pm, *pv, *ps;
            IGM_TRY(workspace(c, "vol_maps", 1, &pm));
            IGM_TRY(workspace(c, "vol_vox", 1, &pv));
            A.vmaps = (const igm::ms::VolMapDev*)pm;
            A.vvox = (const int4*)pv;
            if (c->vol_nsmap > 0) {
                IGM_TRY(workspace(c, "vol_smap", 1, &ps));
                A.vsmap = (const int*)ps;
            }
        }
    }
    int64_t nsb = 0;
    if (sbond_ptr) {
        if (flags & IGM_DEVICE_PTRS) {
            IGM_HIP_CHECK(c, hipMemcpyAsync(&nsb, sbond_ptr + nstruct, sizeof(int64_t), hipMemcpyDeviceToHost,
                                            c->stream));
            IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
        } else {
            nsb = sbond_ptr[nstruct];
        }
    }
    IGM_TRY(to_device(c, flags, "vi_xyz", xyz, (size_t)nstruct * natom * 3, &A.xyz));
    IGM_TRY(to_device(c, flags, "vi_radii", radii, (size_t)natom, &A.radii));
    A.afs = (prm->flags & IGM_MSTEP_STRUCT_FLAGS) ? (size_t)natom : 0;
    IGM_TRY(to_device(c, flags, "vi_flags", atom_flags, A.afs ? (size_t)nstruct * natom : (size_t)natom, &A.aflags));
    IGM_TRY(to_device(c, flags, "vi_shared", shared_bonds, (size_t)nshared, &A.shared));
    IGM_TRY(to_device(c, flags, "vi_shcls", shared_class, shared_class ? (size_t)nshared : 0, &A.shared_class));
    IGM_TRY(to_device(c, flags, "vi_sptr", sbond_ptr, sbond_ptr ? (size_t)nstruct + 1 : 0, &A.sptr));
    IGM_TRY(to_device(c, flags, "vi_sbonds", sbonds, (size_t)nsb, &A.sbonds));
    IGM_TRY(to_device(c, flags, "vi_scls", sclass, sclass ? (size_t)nsb : 0, &A.sclass));
    if (!sbond_ptr) A.sptr = nullptr;
    const int ncls = nclass_bonds + A.nenv;
    int64_t* d_stats;
    IGM_TRY(out_device(c, flags, "vi_stats", stats, (size_t)nstruct * ncls * kRec, &d_stats));
    A.stats = d_stats;
    {
        Timed tm(c, "violations");
        hipLaunchKernelGGL(violations_kernel, dim3(nstruct), dim3(256), 0, c->stream, A);
        IGM_HIP_CHECK(c, hipGetLastError());
    }
    IGM_TRY(to_host(c, flags, stats, (const int64_t*)d_stats, (size_t)nstruct * ncls * kRec));
    return finish(c, flags);
}
