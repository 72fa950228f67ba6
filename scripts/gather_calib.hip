// Calibration of the gfx950 memory-side read counters for the access patterns of the
// population engine: every kernel below reads a KNOWN number of unique
// bytes from a 1 GiB buffer (4x the 256 MiB Infinity Cache, so nothing stays resident
// between the kernels), and rocprofv3 --pmc counts what the L2 asked of memory:
//   stream   float4 per lane, consecutive (the integrate/permute streams)           1 GiB
//   line8    float4 per lane, the 64 lanes' addresses permuted inside the wave's     1 GiB
//            1 KiB (whole 128-B lines, gathered)
//   perm16   float4 per lane at a bijective hash of the index (each float4 once,     1 GiB
//            the 64 lanes on 64 different lines: the force kernel's gathers)
//   perm12   the same positions read as 12-byte b96 loads (the fill's candidates)    0.75 GiB
//   halves   two lanes per 128-B line (2^23 lines, permuted), its two 64-B halves     256 MiB
//   same64   two lanes per line, both in the same 64-B half                          256 MiB
// Each kernel runs REPS times (the counters are summed per kernel name; divide by REPS).
// Build: scripts/build_calib.sh -> igm_amd/lib/calib/gather_calib; run on the box:
//   rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum -- igm_amd/lib/calib/gather_calib
//   rocprofv3 --pmc FETCH_SIZE -- igm_amd/lib/calib/gather_calib
// It prints each kernel's unique bytes and HIP-event time.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int kLog = 26;                  // 2^26 float4 = 1 GiB
constexpr unsigned kN = 1u << kLog;
constexpr unsigned kMask = kN - 1;
constexpr int kBS = 256;
constexpr int REPS = 4;

__device__ __forceinline__ unsigned perm(unsigned g) { return (g * 0x9E3779B1u) & kMask; }  // odd: a bijection

__global__ void __launch_bounds__(kBS) stream_kernel(const float4* __restrict__ a, float* out) {
    const unsigned g = blockIdx.x * kBS + threadIdx.x;
    const float4 v = a[g];
    if (v.x == 12345.0f) out[g & 1023] = v.y + v.z + v.w;  // (never true: keeps the load)
}

__global__ void __launch_bounds__(kBS) line8_kernel(const float4* __restrict__ a, float* out) {
    const unsigned g = blockIdx.x * kBS + threadIdx.x;
    const unsigned w = g & ~63u, l = g & 63u;
    const float4 v = a[w + ((l * 37u) & 63u)];  // 37 odd: a permutation of the wave's 64 slots
    if (v.x == 12345.0f) out[g & 1023] = v.y + v.z + v.w;
}

__global__ void __launch_bounds__(kBS) perm16_kernel(const float4* __restrict__ a, float* out) {
    const unsigned g = blockIdx.x * kBS + threadIdx.x;
    const float4 v = a[perm(g)];
    if (v.x == 12345.0f) out[g & 1023] = v.y + v.z + v.w;
}

__global__ void __launch_bounds__(kBS) perm12_kernel(const float4* __restrict__ a, float* out) {
    const unsigned g = blockIdx.x * kBS + threadIdx.x;
    const float* p = reinterpret_cast<const float*>(a + perm(g));
    typedef float f3 __attribute__((ext_vector_type(3)));
    const f3 v = *reinterpret_cast<const f3*>(p);
    if (v.x == 12345.0f) out[g & 1023] = v.y + v.z;
}

// two lanes per 128-B line of a permuted line order: halves = the line's two 64-B halves
// (float4 0 and 4), same64 = two float4 of one 64-B half (0 and 1).  If a gather miss makes
// the L2 fetch its whole 128-B line, halves costs one request per line; if it fetches 64-B
// sectors, two.  same64 is one request per line either way.
__global__ void __launch_bounds__(kBS) halves_kernel(const float4* __restrict__ a, float* out) {
    const unsigned g = blockIdx.x * kBS + threadIdx.x;  // g < kN / 4
    const unsigned line = perm(g >> 1) & (kMask >> 3);
    const float4 v = a[(line << 3) + ((g & 1) << 2)];
    if (v.x == 12345.0f) out[g & 1023] = v.y + v.z + v.w;
}
__global__ void __launch_bounds__(kBS) same64_kernel(const float4* __restrict__ a, float* out) {
    const unsigned g = blockIdx.x * kBS + threadIdx.x;
    const unsigned line = perm(g >> 1) & (kMask >> 3);
    const float4 v = a[(line << 3) + (g & 1)];
    if (v.x == 12345.0f) out[g & 1023] = v.y + v.z + v.w;
}

int main() {
    float4* a;
    float* out;
    CK(hipMalloc(&a, sizeof(float4) * (size_t)kN));
    CK(hipMalloc(&out, sizeof(float) * 1024));
    CK(hipMemset(a, 0, sizeof(float4) * (size_t)kN));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct K {
        const char* name;
        void (*fn)(const float4*, float*);
        double bytes;
    } ks[] = {{"stream", stream_kernel, 16.0 * kN},
              {"line8", line8_kernel, 16.0 * kN},
              {"perm16", perm16_kernel, 16.0 * kN},
              {"perm12", perm12_kernel, 12.0 * kN},
              {"halves", halves_kernel, 32.0 * (kN / 8)},
              {"same64", same64_kernel, 32.0 * (kN / 8)}};
    hipLaunchKernelGGL(stream_kernel, dim3(kN / kBS), dim3(kBS), 0, 0, a, out);  // (untimed: first-touch costs)
    CK(hipDeviceSynchronize());
    printf("{\"reps\": %d, \"buffer_bytes\": %.0f, \"kernels\": {", REPS, 16.0 * kN);
    for (int k = 0; k < 6; ++k) {
        float ms = 0.0f;
        const dim3 grid(k < 4 ? kN / kBS : kN / 4 / kBS);  // (halves, same64: 2 lanes per line, every line once)
        for (int r = 0; r < REPS; ++r) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(ks[k].fn, grid, dim3(kBS), 0, 0, a, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms += t;
        }
        printf("%s\"%s\": {\"unique_bytes_per_launch\": %.0f, \"ms_per_launch\": %.4f, \"unique_GBps\": %.1f}",
               k ? ", " : "", ks[k].name, ks[k].bytes, ms / REPS, ks[k].bytes / (ms / REPS * 1e-3) / 1e9);
    }
    printf("}}\n");
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
