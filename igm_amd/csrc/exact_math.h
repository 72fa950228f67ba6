// Correctly rounded helpers for the kernels that restate NumPy/CPython
// arithmetic bit-for-bit (A-step, Hi-C selection, violation scoring).  The
// hardware v_sqrt_f32 / v_sqrt_f64 are not IEEE correctly rounded.
#pragma once
#include <hip/hip_runtime.h>

namespace igm {

// correctly rounded double sqrt (Tuckerman test around the hardware result)
__device__ __forceinline__ double sqrt_rn(double x) {
    double y = sqrt(x);
    if (!(x > 0.0) || isinf(x)) return y;
    const double ym = nextafter(y, 0.0), yp = nextafter(y, (double)INFINITY);
    if (fma(ym, y, -x) >= 0.0) return ym;
    if (fma(y, yp, -x) < 0.0) return yp;
    return y;
}

// correctly rounded float sqrt: sqrt of a 24-bit value rounded to 53 bits can
// never sit on a 24-bit rounding midpoint, so the second rounding is exact
__device__ __forceinline__ float sqrtf_rn(float x) { return (float)sqrt_rn((double)x); }

// RN(sqrt(d2)) <= dist  for f32 d2 >= 0 and f32 dist, decided exactly:
// <=> d2 < (dist + ulp(dist)/2)^2  (no ties exist), evaluated exactly in f64
__device__ __forceinline__ bool sqrt_le(float d2, float dist) {
    if (!(dist >= 0.0f)) return false;
    if (isinf(dist)) return d2 == d2;
    const double m = (double)dist + 0.5 * ((double)nextafterf(dist, INFINITY) - (double)dist);
    return (double)d2 < m * m;  // m has <= 25 significant bits: m*m is exact
}

// float('%.Nf' % x) with scale = 10^N (N <= 15): CPython formats the exact binary
// value rounded half-to-even to N decimals, and float() returns the double nearest
// that decimal, i.e. RN(k / 10^N).  x*scale is split exactly into hi + lo.
__device__ __forceinline__ double round_dec(double x, double scale) {
    if (!isfinite(x)) return x;
    const double hi = x * scale;
    const double lo = fma(x, scale, -hi);
    double r = rint(hi);
    const double t = hi - r;  // exact
    const double u = (t - 0.5) + lo;
    const double w = (t + 0.5) + lo;
    if (u > 0.0) {
        r += 1.0;
    } else if (u == 0.0) {
        if (fmod(r, 2.0) != 0.0) r += 1.0;
    } else if (w < 0.0) {
        r -= 1.0;
    } else if (w == 0.0) {
        if (fmod(r, 2.0) != 0.0) r -= 1.0;
    }
    return r / scale;
}

}  // namespace igm
