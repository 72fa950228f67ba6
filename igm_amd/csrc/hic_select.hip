// M-step restraint assembly on the GPU: the Hi-C contact selection of
// interHiC._apply / intraHiC._apply (igm/restraints/inter_hic.py:294-312,
// intra_hic.py:294-312) for every actdist row and every structure at once.
//
// Reference semantics restated exactly (compiled with -ffp-contract=off):
//   ||x_i - x_j|| = np.linalg.norm(f32 vector) = sqrtf(fl32(fl32(dx^2 + dy^2) + dz^2))
//   (particle.py:35-36), compared in f32 with the f32 activation distance;
//   inter rows are applied first (all rows with chrom_i != chrom_j, file order),
//   then intra rows (ModelingStep.py:392-398); r0 = cr * (r_i + r_j) with the
//   radii sum in f32 and the product in f64 (NumPy 1.x), k = contact_kspring.
//
// Layout: xyz is struct-major (nstruct, natom, 3), the M-step layout.  One
// workgroup per (structure, block of rows): threads test rows in order, and the
// per-structure output order is restored by a block-level ballot prefix, so the
// bond list of each structure is in the reference's row order.
#include <hipcub/hipcub.hpp>

#include "exact_math.h"
#include "igm_ctx.h"

namespace {

constexpr int kRowsPerBlock = 1024;  // rows handled by one workgroup of 256 threads (4 per thread)

__device__ __forceinline__ bool selected(const float* x, const int32_t* chrom, int i, int j, float dist, int pass) {
    const bool inter = chrom[i] != chrom[j];
    if ((pass == 0) != inter) return false;
    const float dx = __fsub_rn(x[3 * i], x[3 * j]);
    const float dy = __fsub_rn(x[3 * i + 1], x[3 * j + 1]);
    const float dz = __fsub_rn(x[3 * i + 2], x[3 * j + 2]);
    const float d2 = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
    return igm::sqrt_le(d2, dist);  // RN(sqrt(d2)) <= dist, exactly
}

// pass 0 (inter) / 1 (intra): count selected rows per (structure, row block)
__global__ void __launch_bounds__(256) count_kernel(int natom, const float* __restrict__ xyz,
                                                    const int32_t* __restrict__ chrom,
                                                    const igm_actdist_row* __restrict__ act, int64_t n_act, int nblk,
                                                    int64_t* __restrict__ counts) {
    const int s = blockIdx.y;
    const int pass = blockIdx.z;
    const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock;
    const float* x = xyz + (size_t)s * natom * 3;
    int c = 0;
    for (int u = 0; u < kRowsPerBlock / 256; ++u) {
        const int64_t q = r0 + u * 256 + threadIdx.x;
        if (q < n_act) {
            const igm_actdist_row r = act[q];
            c += selected(x, chrom, r.row, r.col, r.dist, pass);
        }
    }
    // block sum
    __shared__ int red[4];
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0)
        counts[((size_t)s * 2 + pass) * nblk + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// write the selected rows in order: offsets come from the scan of count_kernel
__global__ void __launch_bounds__(256) fill_kernel(int natom, const float* __restrict__ xyz,
                                                   const float* __restrict__ radii, const int32_t* __restrict__ chrom,
                                                   const igm_actdist_row* __restrict__ act, int64_t n_act, int nblk,
                                                   const int64_t* __restrict__ offs, double cr, double kspring,
                                                   int inter_class, int intra_class, igm_bond* __restrict__ out,
                                                   int32_t* __restrict__ out_class) {
    const int s = blockIdx.y;
    const int pass = blockIdx.z;
    const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock;
    const float* x = xyz + (size_t)s * natom * 3;
    __shared__ int wtot[4];
    int64_t base = offs[((size_t)s * 2 + pass) * nblk + blockIdx.x];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int u = 0; u < kRowsPerBlock / 256; ++u) {
        const int64_t q = r0 + u * 256 + threadIdx.x;
        bool sel = false;
        int i = 0, j = 0;
        if (q < n_act) {
            const igm_actdist_row r = act[q];
            i = r.row;
            j = r.col;
            sel = selected(x, chrom, i, j, r.dist, pass);
        }
        const unsigned long long m = __ballot(sel);
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wtot[w] = __popcll(m);
        __syncthreads();
        int woff = 0, tot = 0;
        for (int k = 0; k < 4; ++k) {
            if (k < w) woff += wtot[k];
            tot += wtot[k];
        }
        if (sel) {
            igm_bond b;
            b.i = (uint32_t)i;
            b.j = (uint32_t)j;
            const float rs = __fadd_rn(radii[i], radii[j]);
            b.r0 = (float)(cr * (double)rs);
            b.k = (float)kspring;
            out[base + woff + before] = b;
            if (out_class) out_class[base + woff + before] = pass == 0 ? inter_class : intra_class;
        }
        base += tot;
        __syncthreads();
    }
}

// per structure: total = inter + intra; the output CSR is [inter rows | intra rows]
__global__ void ptr_kernel(int nstruct, int nblk, const int64_t* __restrict__ offs, const int64_t* __restrict__ counts,
                           int64_t* __restrict__ ptr) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s > nstruct) return;
    if (s == nstruct) {
        const size_t last = (size_t)nstruct * 2 * nblk - 1;
        ptr[s] = offs[last] + counts[last];
    } else {
        ptr[s] = offs[(size_t)s * 2 * nblk];
    }
}

}  // namespace

extern "C" int igm_hic_select(igm_ctx* c, uint32_t flags, int32_t nstruct, int32_t natom, const float* xyz,
                              const float* radii, const int32_t* chrom, const igm_actdist_row* act,
                              int64_t n_act, double contact_range,
                              double kspring, int32_t inter_class, int32_t intra_class, int64_t* out_ptr,
                              igm_bond* out_bonds, int32_t* out_class, int64_t* ntotal) {
    using namespace igm;
    if (!c || nstruct <= 0 || natom <= 0 || !xyz || !radii || !chrom || !out_ptr || !ntotal || n_act < 0 ||
        (n_act > 0 && !act))
        return fail(c, IGM_E_INVALID, "igm_hic_select: invalid arguments");
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    const float *d_xyz, *d_radii;
    const int32_t* d_chrom;
    const igm_actdist_row* d_act;
    IGM_TRY(to_device(c, flags, "hs_xyz", xyz, (size_t)nstruct * natom * 3, &d_xyz));
    IGM_TRY(to_device(c, flags, "hs_radii", radii, (size_t)natom, &d_radii));
    IGM_TRY(to_device(c, flags, "hs_chrom", chrom, (size_t)natom, &d_chrom));
    IGM_TRY(to_device(c, flags, "hs_act", act, (size_t)n_act, &d_act));
    const int nblk = (int)std::max<int64_t>(1, ceil_div(n_act, kRowsPerBlock));
    const size_t ncnt = (size_t)nstruct * 2 * nblk;
    void *p_cnt, *p_off, *p_ptr;
    IGM_TRY(workspace(c, "hs_cnt", sizeof(int64_t) * ncnt, &p_cnt));
    IGM_TRY(workspace(c, "hs_off", sizeof(int64_t) * ncnt, &p_off));
    int64_t* d_ptr;
    if (flags & IGM_DEVICE_PTRS) {
        d_ptr = out_ptr;
    } else {
        IGM_TRY(workspace(c, "hs_ptr", sizeof(int64_t) * (nstruct + 1), &p_ptr));
        d_ptr = (int64_t*)p_ptr;
    }
    int64_t* d_cnt = (int64_t*)p_cnt;
    int64_t* d_off = (int64_t*)p_off;
    Timed tm(c, "hic_select");
    if (n_act > 0) {
        hipLaunchKernelGGL(count_kernel, dim3(nblk, nstruct, 2), dim3(256), 0, c->stream, natom, d_xyz, d_chrom, d_act,
                           n_act, nblk, d_cnt);
    } else {
        IGM_HIP_CHECK(c, hipMemsetAsync(d_cnt, 0, sizeof(int64_t) * ncnt, c->stream));
    }
    IGM_HIP_CHECK(c, hipGetLastError());
    size_t tmp_bytes = 0;
    IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, d_cnt, d_off, (int)ncnt, c->stream));
    void* d_tmp;
    IGM_TRY(workspace(c, "hs_scan_tmp", tmp_bytes, &d_tmp));
    IGM_HIP_CHECK(c, hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_bytes, d_cnt, d_off, (int)ncnt, c->stream));
    hipLaunchKernelGGL(ptr_kernel, dim3((unsigned)ceil_div(nstruct + 1, 256)), dim3(256), 0, c->stream, nstruct, nblk,
                       d_off, d_cnt, d_ptr);
    IGM_HIP_CHECK(c, hipGetLastError());
    int64_t total = 0;
    IGM_HIP_CHECK(c, hipMemcpyAsync(&total, d_ptr + nstruct, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    *ntotal = total;
    if (!(flags & IGM_DEVICE_PTRS)) IGM_TRY(to_host(c, flags, out_ptr, (const int64_t*)d_ptr, (size_t)nstruct + 1));
    if (out_bonds && total > 0) {
        igm_bond* d_out;
        int32_t* d_cls = nullptr;
        IGM_TRY(out_device(c, flags, "hs_out", out_bonds, (size_t)total, &d_out));
        if (out_class) IGM_TRY(out_device(c, flags, "hs_cls", out_class, (size_t)total, &d_cls));
        hipLaunchKernelGGL(fill_kernel, dim3(nblk, nstruct, 2), dim3(256), 0, c->stream, natom, d_xyz, d_radii,
                           d_chrom, d_act, n_act, nblk, d_off, contact_range, kspring, inter_class,
                           intra_class, d_out, d_cls);
        IGM_HIP_CHECK(c, hipGetLastError());
        IGM_TRY(to_host(c, flags, out_bonds, d_out, (size_t)total));
        if (out_class) IGM_TRY(to_host(c, flags, out_class, d_cls, (size_t)total));
    }
    return finish(c, flags);
}

namespace {
// 32x32-atom tiles through LDS: both sides of the transpose are coalesced
__global__ void __launch_bounds__(256) transpose_kernel(int nbead, int nstruct, int natom, const float* __restrict__ src,
                                                        float* __restrict__ dst, int direction) {
    __shared__ float tile[32][32 * 3 + 1];
    const int b0 = blockIdx.x * 32, s0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    if (direction == 0) {  // src bead-major (nbead, nstruct, 3) -> dst (nstruct, natom, 3)
        for (int r = ty; r < 32; r += 8) {
            const int b = b0 + r;
            for (int q = tx; q < 96; q += 32) {
                const int s = s0 + q / 3;
                if (b < nbead && s < nstruct) tile[r][q] = src[((size_t)b * nstruct + s) * 3 + q % 3];
            }
        }
        __syncthreads();
        for (int r = ty; r < 32; r += 8) {
            const int s = s0 + r;
            for (int q = tx; q < 96; q += 32) {
                const int b = b0 + q / 3;
                if (b < nbead && s < nstruct) dst[((size_t)s * natom + b) * 3 + q % 3] = tile[q / 3][r * 3 + q % 3];
            }
        }
    } else {  // src struct-major (nstruct, natom, 3) -> dst bead-major (nbead, nstruct, 3)
        for (int r = ty; r < 32; r += 8) {
            const int s = s0 + r;
            for (int q = tx; q < 96; q += 32) {
                const int b = b0 + q / 3;
                if (b < nbead && s < nstruct) tile[q / 3][r * 3 + q % 3] = src[((size_t)s * natom + b) * 3 + q % 3];
            }
        }
        __syncthreads();
        for (int r = ty; r < 32; r += 8) {
            const int b = b0 + r;
            for (int q = tx; q < 96; q += 32) {
                const int s = s0 + q / 3;
                if (b < nbead && s < nstruct) dst[((size_t)b * nstruct + s) * 3 + q % 3] = tile[r][q];
            }
        }
    }
}
}  // namespace

extern "C" int igm_population_transpose(igm_ctx* c, uint32_t flags, int32_t nbead, int32_t nstruct, int32_t natom,
                                        const float* src, float* dst, int32_t direction) {
    using namespace igm;
    if (!c || nbead <= 0 || nstruct <= 0 || natom < nbead || !src || !dst || (direction != 0 && direction != 1))
        return fail(c, IGM_E_INVALID, "igm_population_transpose: invalid arguments");
    IGM_HIP_CHECK(c, hipSetDevice(c->device));
    const size_t nsrc = direction == 0 ? (size_t)nbead * nstruct * 3 : (size_t)nstruct * natom * 3;
    const size_t ndst = direction == 0 ? (size_t)nstruct * natom * 3 : (size_t)nbead * nstruct * 3;
    const float* d_src;
    float* d_dst;
    IGM_TRY(to_device(c, flags, "tr_src", src, nsrc, &d_src));
    if (flags & IGM_DEVICE_PTRS) {
        d_dst = dst;
    } else {
        void* p;
        IGM_TRY(workspace(c, "tr_dst", sizeof(float) * ndst, &p));
        d_dst = (float*)p;
        if (direction == 0)  // extra atoms keep the caller's values
            IGM_HIP_CHECK(c, hipMemcpyAsync(d_dst, dst, sizeof(float) * ndst, hipMemcpyHostToDevice, c->stream));
    }
    dim3 grid((unsigned)ceil_div(nbead, 32), (unsigned)ceil_div(nstruct, 32));
    hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, c->stream, nbead, nstruct, natom, d_src, d_dst,
                       direction);
    IGM_HIP_CHECK(c, hipGetLastError());
    IGM_TRY(to_host(c, flags, dst, (const float*)d_dst, ndst));
    return finish(c, flags);
}
