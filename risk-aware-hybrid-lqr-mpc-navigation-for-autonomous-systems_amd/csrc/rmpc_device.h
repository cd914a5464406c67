// rmpc_device.h -- device-side helpers shared by the CDNA4 kernels of librmpc.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rmpc.h"
#include "rmpc_wlog.h"

#define RMPC_PI 3.141592653589793
#define RMPC_WAVE 64

namespace rmpc {

// mpc_controller.py:540-546 / lqr_controller.py:244-250 / differential_drive.py:215-230
template <typename T>
__device__ __forceinline__ T wrap_pi(T a) {
    const T pi = (T)RMPC_PI;
    while (a > pi) a -= (T)2 * pi;
    while (a < -pi) a += (T)2 * pi;
    return a;
}

// sin and cos of one fp64 argument of moderate size (the unwrapped reference headings are a
// few pi; |x| >= 2^50 gives NaN, so such a robot takes the fallback law): x = q pi/2 + r by a
// two-part FMA reduction (accurate to ~1e-16 over that range), the fdlibm minimax
// polynomials on |r| <= pi/4 (sin: x + x^3 S(x^2); cos: 1 - x^2/2 + x^4 C(x^2), the
// 1 - x^2/2 rounding carried as in fdlibm's __kernel_cos), then the quadrant.  Against
// long-double sin/cos over |x| <= 100: abs error <= 1.2e-16 (2 ulp relative near zeros of
// the other function).  A fraction of the cost of the general library routine, whose
// large-argument path the wave would otherwise carry.  NaN/inf in -> NaN out.
__device__ __forceinline__ void sincos_moderate(double x0, double *sp, double *cp) {
    const double x = __builtin_fabs(x0) < 0x1p50 ? x0 : __builtin_nan("");
    const double q = __builtin_rint(x * 6.36619772367581382433e-01);   // 2/pi
    double r = __builtin_fma(-q, 1.57079632679489655800e+00, x);       // pi/2, high part
    r = __builtin_fma(-q, 6.12323399573676603587e-17, r);              // pi/2, low part
    const double z = r * r;
    const double ps = -1.66666666666666324348e-01 +
                      z * (8.33333333332248946124e-03 +
                           z * (-1.98412698298579493134e-04 +
                                z * (2.75573137070700676789e-06 +
                                     z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10))));
    const double s = __builtin_fma(r * z, ps, r);
    const double pc = 4.16666666666666019037e-02 +
                      z * (-1.38888888888741095749e-03 +
                           z * (2.48015872894767294178e-05 +
                                z * (-2.75573143513906633035e-07 +
                                     z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double c = w + (((1.0 - w) - hz) + z * z * pc);
    const int n = (int)(long long)q & 3;
    const double sa = (n & 1) ? c : s, ca = (n & 1) ? s : c;
    *sp = (n & 2) ? -sa : sa;
    *cp = ((n + 1) & 2) ? -ca : ca;
}

// numpy float remainder (npy_divmod): fmod, then move into the divisor's sign
__device__ __forceinline__ double np_mod(double a, double b) {
    double m = fmod(a, b);
    if (m != 0.0) {
        if ((b < 0) != (m < 0)) m += b;
    } else {
        m = copysign(0.0, b);
    }
    return m;
}

template <typename T>
__device__ __forceinline__ T clampv(T v, T lo, T hi) {
    return v < lo ? lo : (v > hi ? hi : v);
}

// Per-robot workspace record, lane-interleaved: element `off` of the lane lives at
// base[off * stride + lane].  Global tiles use stride 64 (one coalesced 512-B row per wave
// access); LDS tiles use the workgroup width (lane-contiguous, conflict-free ds_read_b64).
template <typename T>
struct WaveTile {
    T *base;
    int lane;
    int stride;
    __device__ __forceinline__ T &operator()(int off) const { return base[(size_t)off * stride + lane]; }
};

}  // namespace rmpc
