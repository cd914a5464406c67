// rmpc_device.h -- device-side helpers shared by the CDNA4 kernels of librmpc.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rmpc.h"

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
