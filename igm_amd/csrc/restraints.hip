// Per-structure restraint selection for configuration D: the DamID lamina envelope
// membership of Damid._apply_envelope (igm/restraints/damid.py:112-143) for every
// (structure, DamID row) at once.  A bead joins the structure's lamina envelope when
//     snormsq_ellipsoid(x_i, abc * (1 - cr), r_i) >= d_i^2          (damid.py:119-126)
// with the NumPy 1.x scalar arithmetic of snormsq_ellipsoid (damid.py:43-61): the
// float32 squares divided by float64 (abc*cutoff - r)^2 and summed in float64, compared
// with float64(d)^2.  Built with -ffp-contract=off, so membership is bit-exact.
#include <hip/hip_runtime.h>

#include "igm_ctx.h"

namespace {
using namespace igm;

__global__ void base_flags_kernel(const uint32_t* __restrict__ base, int natom, int64_t total,
                                  uint32_t* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < total) out[k] = base[k % natom];
}

struct SelArgs {
    int nstruct, natom;
    const float* xyz;  // (S, natom, 3) struct-major (the M-step layout)
    const float* radii;
    const igm_damid_row* rows;
    int64_t nrows;
    double abc[3];  // semiaxes * (1 - contact_range), float64 (damid.py:122-123)
    uint32_t bit;
    uint32_t* out;       // (S, natom)
    int* nsel;           // (S) selected rows
};

// grid (ceil(nrows / 256), S): consecutive rows across the wave, one structure per y
__global__ void __launch_bounds__(256) damid_select_kernel(SelArgs A) {
    const int s = blockIdx.y;
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int hit = 0;
    if (q < A.nrows) {
        const igm_damid_row w = A.rows[q];
        const int i = w.loc;
        if (i >= 0 && i < A.natom) {
            const float* x = A.xyz + ((size_t)s * A.natom + i) * 3;
            const double r = (double)A.radii[i];
            const double a = A.abc[0] - r, b = A.abc[1] - r, c = A.abc[2] - r;
            const double v = ((double)__fmul_rn(x[0], x[0]) / (a * a) + (double)__fmul_rn(x[1], x[1]) / (b * b)) +
                             (double)__fmul_rn(x[2], x[2]) / (c * c);
            const double d = (double)w.dist;
            if (v >= d * d) {
                atomicOr(&A.out[(size_t)s * A.natom + i], A.bit);
                hit = 1;
            }
        }
    }
    if (A.nsel) {
        for (int o = 32; o > 0; o >>= 1) hit += __shfl_xor(hit, o, 64);
        if ((threadIdx.x & 63) == 0 && hit) atomicAdd(&A.nsel[s], hit);
    }
}

}  // namespace

extern "C" int igm_damid_select(igm_ctx* c, uint32_t flags, int32_t nstruct, int32_t natom, const float* xyz,
                                const float* radii, const igm_damid_row* rows, int64_t nrows,
                                const double* semiaxes, double contact_range, uint32_t env_bit,
                                const uint32_t* base_flags, uint32_t* out_flags, int32_t* n_selected) {
    if (!c) return IGM_E_INVALID;
    if (nstruct <= 0 || natom <= 0 || nrows < 0 || !xyz || !radii || (nrows > 0 && !rows) || !semiaxes ||
        !base_flags || !out_flags || env_bit == 0u)
        return fail(c, IGM_E_INVALID, "igm_damid_select: invalid arguments");
    if (nrows > (int64_t)0x7fffffff * 256 || nstruct > 65535)
        return fail(c, IGM_E_UNSUPPORTED, "igm_damid_select: grid too large");
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    const float *d_xyz, *d_radii;
    const igm_damid_row* d_rows;
    const uint32_t* d_base;
    const size_t nf = (size_t)nstruct * natom;
    IGM_TRY(to_device(c, flags, "ds_xyz", xyz, nf * 3, &d_xyz));
    IGM_TRY(to_device(c, flags, "ds_radii", radii, (size_t)natom, &d_radii));
    IGM_TRY(to_device(c, flags, "ds_rows", rows, (size_t)nrows, &d_rows));
    IGM_TRY(to_device(c, flags, "ds_base", base_flags, (size_t)natom, &d_base));
    uint32_t* d_out;
    int32_t* d_nsel = nullptr;
    IGM_TRY(out_device(c, flags, "ds_out", out_flags, nf, &d_out));
    if (n_selected) {
        IGM_TRY(out_device(c, flags, "ds_nsel", n_selected, (size_t)nstruct, &d_nsel));
        IGM_HIP_CHECK(c, hipMemsetAsync(d_nsel, 0, sizeof(int32_t) * nstruct, c->stream));
    }
    hipLaunchKernelGGL(base_flags_kernel, dim3((unsigned)ceil_div((int64_t)nf, 256)), dim3(256), 0, c->stream, d_base,
                       natom, (int64_t)nf, d_out);
    IGM_HIP_CHECK(c, hipGetLastError());
    SelArgs A;
    A.nstruct = nstruct;
    A.natom = natom;
    A.xyz = d_xyz;
    A.radii = d_radii;
    A.rows = d_rows;
    A.nrows = nrows;
    const double cutoff = 1.0 - contact_range;
    for (int k = 0; k < 3; ++k) A.abc[k] = semiaxes[k] * cutoff;
    A.bit = env_bit;
    A.out = d_out;
    A.nsel = d_nsel;
    if (nrows > 0) {
        Timed tm(c, "damid_select");
        hipLaunchKernelGGL(damid_select_kernel, dim3((unsigned)ceil_div(nrows, 256), (unsigned)nstruct), dim3(256), 0,
                           c->stream, A);
        IGM_HIP_CHECK(c, hipGetLastError());
    }
    IGM_TRY(to_host(c, flags, out_flags, d_out, nf));
    if (n_selected) IGM_TRY(to_host(c, flags, n_selected, d_nsel, (size_t)nstruct));
    return finish(c, flags);
}
