// What the texture path charges for a gather (the population engine's force and fill kernels
// are bound there, profiles/r05_C): L2-resident data (a 1 MiB table, every XCD's L2 holds it),
// every wave instruction of 64 lanes touching G distinct 128-B lines with W bytes per lane.
// Prints the cycles one CU spends per wave-level gather instruction (2.4 GHz clock assumed;
// the kernel's HIP-event time x CUs / wave instructions), for
//   G = 64, 32, 16, 8, 4, 1 lines per instruction at W = 16 (b128), and
//   G = 64 at W = 12 (b96), 8 (b64), 4 (b32).
// Build: scripts/build_calib.sh; run: igm_amd/lib/calib/gather_rate
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

constexpr int kLines = 8192;  // 1 MiB of 128-B lines
constexpr int kBS = 256, kIters = 256, kBlocks = 256 * 8;

__device__ __forceinline__ unsigned mix(unsigned x) {
    x ^= x >> 15;
    x *= 0x2c1b3c6du;
    x ^= x >> 12;
    x *= 0x297a2d39u;
    return x ^ (x >> 15);
}

template <int G, int W>
__global__ void __launch_bounds__(kBS) gather_kernel(const unsigned char* __restrict__ tab, float* out) {
    const unsigned lane = threadIdx.x & 63, wave = (blockIdx.x * kBS + threadIdx.x) >> 6;
    constexpr int PER = 64 / G;        // lanes per line
    constexpr int SLOTS = 128 / 16;    // 16-B slots per line (a lane's W bytes start on one)
    float acc = 0.0f;
#pragma unroll 8
    for (int it = 0; it < kIters; ++it) {
        const unsigned line = mix(wave * 131071u + it * 64u + lane / PER) % kLines;
        const unsigned sub = (lane % PER) % SLOTS;
        const unsigned char* p = tab + line * 128u + sub * 16u;
        if (W == 16) {
            const float4 v = *reinterpret_cast<const float4*>(p);
            acc += v.x + v.w;
        } else if (W == 12) {
            typedef float f3 __attribute__((ext_vector_type(3)));
            const f3 v = *reinterpret_cast<const f3*>(p);
            acc += v.x + v.z;
        } else if (W == 8) {
            const float2 v = *reinterpret_cast<const float2*>(p);
            acc += v.x + v.y;
        } else {
            acc += *reinterpret_cast<const float*>(p);
        }
    }
    if (acc == 12345.0f) out[threadIdx.x] = acc;
}

template <int G, int W>
void run(const unsigned char* tab, float* out, hipEvent_t e0, hipEvent_t e1, int ncu, bool first) {
    hipLaunchKernelGGL((gather_kernel<G, W>), dim3(kBlocks), dim3(kBS), 0, 0, tab, out);  // warm
    CK(hipEventRecord(e0));
    for (int r = 0; r < 4; ++r) hipLaunchKernelGGL((gather_kernel<G, W>), dim3(kBlocks), dim3(kBS), 0, 0, tab, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double winst = 4.0 * kBlocks * (kBS / 64) * kIters;  // wave-level gather instructions
    const double cyc = ms * 1e-3 * 2.4e9 * ncu / winst;
    printf("%s\"G%d_W%d\": {\"ms\": %.4f, \"cu_cycles_per_wave_gather\": %.2f, \"lane_gathers_per_ns\": %.1f}",
           first ? "" : ", ", G, W, ms / 4, cyc, winst * 64 / (ms * 1e6));
}

int main() {
    unsigned char* tab;
    float* out;
    CK(hipMalloc(&tab, 128 * (size_t)kLines));
    CK(hipMalloc(&out, sizeof(float) * kBS));
    CK(hipMemset(tab, 0, 128 * (size_t)kLines));
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int ncu = pr.multiProcessorCount;
    printf("{\"cus\": %d, \"table_bytes\": %d, ", ncu, 128 * kLines);
    run<64, 16>(tab, out, e0, e1, ncu, true);
    run<32, 16>(tab, out, e0, e1, ncu, false);
    run<16, 16>(tab, out, e0, e1, ncu, false);
    run<8, 16>(tab, out, e0, e1, ncu, false);
    run<4, 16>(tab, out, e0, e1, ncu, false);
    run<1, 16>(tab, out, e0, e1, ncu, false);
    run<64, 12>(tab, out, e0, e1, ncu, false);
    run<64, 8>(tab, out, e0, e1, ncu, false);
    run<64, 4>(tab, out, e0, e1, ncu, false);
    printf("}\n");
    return 0;
}
