// rmpc_misc.hip -- risk metrics, hybrid LQR/MPC switch with branch compaction, unicycle
// plant step and Figure-8 reference generation on CDNA4 (gfx950).  One lane per robot.
#include "rmpc_device.h"
#include "rmpc_internal.h"

namespace rmpc {

// risk_metrics.py:84-129
__device__ __forceinline__ double distance_risk(const RiskDevParams &p, double px, double py,
                                                const double *obs, int no, double *min_d, int *nid) {
    double md = INFINITY, mr = 0.0;
    int id = -1;
    for (int i = 0; i < no; i++) {
        const double dx = px - obs[3 * i], dy = py - obs[3 * i + 1];
        const double d = sqrt(dx * dx + dy * dy) - obs[3 * i + 2];
        if (d < md) { md = d; id = i; }
        double r;
        if (d <= p.d_safe) r = 1.0;
        else if (d >= p.d_trigger) r = 0.0;
        else r = 1.0 - (d - p.d_safe) / (p.d_trigger - p.d_safe);
        mr = fmax(mr, r);
    }
    *min_d = md;
    *nid = id;
    return mr;
}

// risk_metrics.py:131-171
__device__ __forceinline__ double predictive_risk(const RiskDevParams &p, const double *pred, int n,
                                                  const double *obs, int no) {
    if (no == 0 || n == 0) return 0.0;
    double sev = 0.0;
    for (int k = 0; k < n; k++) {
        const double px = pred[3 * k], py = pred[3 * k + 1];
        for (int i = 0; i < no; i++) {
            const double dx = px - obs[3 * i], dy = py - obs[3 * i + 1];
            const double d = sqrt(dx * dx + dy * dy) - obs[3 * i + 2];
            if (d < p.d_safe) {
                const double tw = 1.0 - ((double)k / (double)n) * 0.5;
                sev += tw * ((p.d_safe - d) / p.d_safe);
            }
        }
    }
    return fmin(1.0, sev / (double)(n * no) * 5.0);
}

__device__ __forceinline__ void normalise_weights(const RiskDevParams &p, double *al, double *be) {
    const double tot = p.alpha + p.beta;          // risk_metrics.py:79-82
    *al = p.alpha / tot;
    *be = p.beta / tot;
}

__global__ __launch_bounds__(256) void risk_kernel(RiskDevParams p, int64_t B, const double *x,
                                                   const double *pred, int n_pred,
                                                   const double *obs, int no, double *out,
                                                   uint8_t *use_mpc, int32_t *level) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double md;
    int nid;
    const double dr = no ? distance_risk(p, x[3 * b], x[3 * b + 1], obs, no, &md, &nid) : 0.0;
    if (!no) { md = INFINITY; nid = -1; }
    const double pr = pred ? predictive_risk(p, pred + (size_t)3 * n_pred * b, n_pred, obs, no) : 0.0;
    double al, be;
    normalise_weights(p, &al, &be);
    const double c = al * dr + be * pr;           // :198
    int lv = c < p.th_low ? 0 : (c < p.th_med ? 1 : (c < p.th_high ? 2 : 3));
    out[5 * b] = dr;
    out[5 * b + 1] = pr;
    out[5 * b + 2] = c;
    out[5 * b + 3] = md;
    out[5 * b + 4] = (double)nid;
    if (use_mpc) use_mpc[b] = c >= p.th_low;     // :212
    if (level) level[b] = lv;
}

// run_simulation.py:528-548: risk (no predicted states), 10-step dwell hysteresis, switch
// bookkeeping; robots are compacted into per-branch index lists so that each branch runs
// as full waves of one kernel (no LQR/MPC divergence inside a wave).
constexpr int DECIDE_BLK = 1024;      // threads per block of the switch kernel (16 waves)
__global__ __launch_bounds__(DECIDE_BLK) void hybrid_decide_kernel(RiskDevParams p, int64_t B, const double *x,
                                                                   const double *obs, int no, int32_t *prev_ctrl,
                                                                   int32_t *steps_since, uint8_t *used_mpc,
                                                                   double *risk_out, int32_t *idx_lqr,
                                                                   int32_t *idx_mpc, int32_t *counts,
                                                                   const double *pred, int n_pred, int32_t *zero_next) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // the other counter pair, which the previous step used (complete in stream order) and the
    // next step takes: zeroed here instead of a fill launch per step
    if (zero_next && b < 2) zero_next[b] = 0;
    const bool valid = b < B;
    bool mpc = false;
    if (valid) {
        double md;
        int nid;
        const double dr = no ? distance_risk(p, x[3 * b], x[3 * b + 1], obs, no, &md, &nid) : 0.0;
        double al, be;
        normalise_weights(p, &al, &be);
        // the reference's loop passes no predicted states (pr = 0); with use_pred, a robot whose
        // previous step ran MPC (used_mpc still holds that step's flag here) passes its x_pred
        const double pr = (pred && p.use_pred && used_mpc[b]) ? predictive_risk(p, pred + (size_t)3 * n_pred * b,
                                                                                  n_pred, obs, no)
                                                              : 0.0;
        const double c = al * dr + be * pr;
        const bool rec = c >= p.th_low;
        const int prev = prev_ctrl[b];
        int since = steps_since[b];
        if (since >= p.min_dwell) mpc = rec;                    // :533-534
        else mpc = prev >= 0 ? (prev == 1) : rec;              // :536-537
        const int cur = mpc ? 1 : 0;
        if (prev >= 0 && cur != prev) since = 0;                // :542-546
        else since += 1;
        prev_ctrl[b] = cur;
        steps_since[b] = since;
        used_mpc[b] = (uint8_t)mpc;
        if (risk_out) risk_out[b] = c;
    }
    // Compaction into the two branch lists (order inside a list is irrelevant: robots are
    // independent), one atomic per BLOCK and list: with one per wave, 2 x 1024 atomics on the
    // two adjacent counters serialised to 26 us of a 0.40 ms config-5 step.
    __shared__ int wcnt[2][DECIDE_BLK / 64], base[2];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t m1 = __ballot(valid && mpc), m0 = __ballot(valid && !mpc);
    if (lane == 0) {
        wcnt[1][w] = __popcll(m1);
        wcnt[0][w] = __popcll(m0);
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        int tot = 0;
        for (int i = 0; i < DECIDE_BLK / 64; i++) tot += wcnt[threadIdx.x][i];
        base[threadIdx.x] = tot ? atomicAdd(&counts[threadIdx.x], tot) : 0;
    }
    __syncthreads();
    if (valid) {
        const uint64_t m = mpc ? m1 : m0;
        const int l = mpc ? 1 : 0;
        int off = base[l];
        for (int i = 0; i < w; i++) off += wcnt[l][i];
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        (mpc ? idx_mpc : idx_lqr)[off + rank] = (int32_t)b;
    }
}

// differential_drive.py:111-172 (clip, Euler or RK4, while-wrap of theta)
__device__ __forceinline__ void plant_step(double x0, double x1, double x2, double u0, double u1, double dt,
                                           double v_max, double omega_max, int method, double *xn) {
    const double v = clampv(u0, -v_max, v_max), w = clampv(u1, -omega_max, omega_max);
    double n0, n1, n2;
    if (method == 0) {
        n0 = x0 + dt * (v * cos(x2));
        n1 = x1 + dt * (v * sin(x2));
        n2 = x2 + dt * w;
    } else {
        const double k10 = v * cos(x2), k11 = v * sin(x2), k12 = w;
        const double t2 = x2 + 0.5 * dt * k12;
        const double k20 = v * cos(t2), k21 = v * sin(t2), k22 = w;
        const double t3 = x2 + 0.5 * dt * k22;
        const double k30 = v * cos(t3), k31 = v * sin(t3), k32 = w;
        const double t4 = x2 + dt * k32;
        const double k40 = v * cos(t4), k41 = v * sin(t4), k42 = w;
        const double h = dt / 6.0;
        n0 = x0 + h * (k10 + 2 * k20 + 2 * k30 + k40);
        n1 = x1 + h * (k11 + 2 * k21 + 2 * k31 + k41);
        n2 = x2 + h * (k12 + 2 * k22 + 2 * k32 + k42);
    }
    xn[0] = n0;
    xn[1] = n1;
    xn[2] = wrap_pi(n2);
}

__global__ __launch_bounds__(256) void plant_kernel(int64_t B, const double *x, const double *u, double dt,
                                                    double v_max, double omega_max, int method,
                                                    double *xn) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    plant_step(x[3 * b], x[3 * b + 1], x[3 * b + 2], u[2 * b], u[2 * b + 1], dt, v_max, omega_max, method,
               xn + 3 * b);
}

// reference_generator.py:86-172 evaluated at t0[b] + i*dt
__device__ __forceinline__ double heading8(double A, double a, double t) {
    const double dpx = a * A * cos(a * t);
    const double c = cos(a * t), s = sin(a * t);
    const double dpy = a * A * (c * c - s * s);
    return atan2(dpy, dpx);
}

// one reference point (px, py, theta, v, omega) at time t
__device__ __forceinline__ void fig8_point(double A, double a, double dt, double t, double *xr, double *ur) {
    const double s = sin(a * t), c = cos(a * t);
    const double dpx = a * A * c, dpy = a * A * (c * c - s * s);
    const double th = atan2(dpy, dpx);
    xr[0] = A * s;
    xr[1] = A * s * c;
    xr[2] = th;
    ur[0] = sqrt(dpx * dpx + dpy * dpy);
    ur[1] = wrap_pi(heading8(A, a, t + dt) - th) / dt;       // :150-172 forward difference
}

__global__ __launch_bounds__(256) void figure8_kernel(int64_t B, const double *t0, int rows, double A, double a,
                                                      double dt, double *xr, double *ur) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= B * rows) return;
    const int64_t b = g / rows;
    const int i = (int)(g % rows);
    fig8_point(A, a, dt, t0[b] + (double)i * dt, xr + 3 * g, ur + 2 * g);
}

// Rows of the generate() table (t_j = j*dt exactly as np.arange) for table rows
// start[b] + k + i, clamped to the last row (get_trajectory_segment :299-326)
__global__ __launch_bounds__(256) void figure8_table_kernel(int64_t B, const int32_t *start, int32_t k, int rows,
                                                            int32_t table_len, double A, double a, double dt,
                                                            double *xr, double *ur) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= B * rows) return;
    const int64_t b = g / rows;
    const int i = (int)(g % rows);
    int64_t j = (int64_t)(start ? start[b] : 0) + k + i;
    if (j > table_len - 1) j = table_len - 1;
    fig8_point(A, a, dt, (double)j * dt, xr + 3 * g, ur + 2 * g);
}

// identity robot list 0..B-1 and its device-side length (whole-batch launches of the
// list-driven kernels)
__global__ __launch_bounds__(256) void iota_kernel(int64_t B, int32_t *idx, int32_t *count) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *count = (int32_t)B;
    if (i < B) idx[i] = (int32_t)i;
}

// per-robot first reference row of rollout step k in the end-padded table
__global__ __launch_bounds__(256) void ref_offsets_kernel(int64_t B, const int32_t *start, int32_t k, int32_t last,
                                                          int32_t *off) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int64_t j = (int64_t)(start ? start[b] : 0) + k;
    off[b] = (int32_t)(j < last ? j : last);
}

// rollout start: x = x0[b] or the reference at the start row; clear per-robot state
__global__ __launch_bounds__(256) void rollout_init_kernel(int64_t B, const int32_t *start, const double *x0,
                                                           int32_t table_len, double A, double a, double dt,
                                                           double *x, int32_t *prev_ctrl, int32_t *since,
                                                           int32_t *step_count, RmpcLqrCache *cache,
                                                           double *states, int32_t steps) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double xs[3], us[2];
    if (x0) {
        xs[0] = x0[3 * b]; xs[1] = x0[3 * b + 1]; xs[2] = x0[3 * b + 2];
    } else {
        int64_t j = start ? start[b] : 0;
        if (j > table_len - 1) j = table_len - 1;
        fig8_point(A, a, dt, (double)j * dt, xs, us);
    }
    x[3 * b] = xs[0]; x[3 * b + 1] = xs[1]; x[3 * b + 2] = xs[2];
    prev_ctrl[b] = -1;
    since[b] = 0;
    step_count[b] = 0;
    cache[b].valid = 0;
    if (states) {
        double *o = states + (size_t)b * (steps + 1) * 3;
        o[0] = xs[0]; o[1] = xs[1]; o[2] = xs[2];
    }
}

// plant step of a rollout, recording x_{k+1}, u_k (and the controller used)
__global__ __launch_bounds__(256) void rollout_plant_kernel(int64_t B, double *x, const double *u, double dt,
                                                            double v_max, double omega_max, int method, int32_t k,
                                                            int32_t steps, double *states, double *controls,
                                                            const uint8_t *used_now, int used_fill, uint8_t *used) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double xn[3];
    plant_step(x[3 * b], x[3 * b + 1], x[3 * b + 2], u[2 * b], u[2 * b + 1], dt, v_max, omega_max, method, xn);
    x[3 * b] = xn[0]; x[3 * b + 1] = xn[1]; x[3 * b + 2] = xn[2];
    if (states) {
        double *o = states + ((size_t)b * (steps + 1) + k + 1) * 3;
        o[0] = xn[0]; o[1] = xn[1]; o[2] = xn[2];
    }
    if (controls) {
        double *o = controls + ((size_t)b * steps + k) * 2;
        o[0] = u[2 * b]; o[1] = u[2 * b + 1];
    }
    // which controller ran: the hybrid switch's flag, else the mode's own (MPC 1, LQR 0)
    if (used) used[(size_t)b * steps + k] = used_now ? used_now[b] : (uint8_t)used_fill;
}

__global__ __launch_bounds__(256) void status_count_kernel(int64_t B, const int32_t *status, const uint8_t *mask,
                                                           unsigned long long *counts) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = b < B && (!mask || mask[b]);
    const int s = in ? status[b] : -1;
#pragma unroll
    for (int v = 0; v < 4; v++) {           // one atomic per wave and status value
        const uint64_t m = __ballot(s == v);
        if (m && (threadIdx.x & 63) == (unsigned)(__ffsll((unsigned long long)m) - 1))
            atomicAdd(counts + v, (unsigned long long)__popcll(m));
    }
}


}  // namespace rmpc

using namespace rmpc;

static inline unsigned nblk(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

hipError_t rmpc_launch_risk(const RiskDevParams &p, int64_t B, const double *x, const double *pred,
                            int n_pred, const double *obstacles, int n_obs, double *out,
                            uint8_t *use_mpc, int32_t *level, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(risk_kernel, dim3(nblk(B, 256)), dim3(256), 0, stream, p, B, x, pred, n_pred,
                       obstacles, n_obs, out, use_mpc, level);
    return hipGetLastError();
}

hipError_t rmpc_launch_hybrid_decide(const RiskDevParams &p, int64_t B, const double *x,
                                     const double *obstacles, int n_obs, int32_t *prev_ctrl,
                                     int32_t *steps_since, uint8_t *used_mpc, double *risk_out,
                                     int32_t *idx_lqr, int32_t *idx_mpc, int32_t *counts,
                                     hipStream_t stream, const double *pred, int n_pred, int32_t *zero_next) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(hybrid_decide_kernel, dim3(nblk(B, DECIDE_BLK)), dim3(DECIDE_BLK), 0, stream, p, B, x, obstacles,
                       n_obs, prev_ctrl, steps_since, used_mpc, risk_out, idx_lqr, idx_mpc, counts, pred, n_pred,
                       zero_next);
    return hipGetLastError();
}

hipError_t rmpc_launch_plant(int64_t B, const double *x, const double *u, double dt, double v_max,
                             double omega_max, int method, double *x_next, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(plant_kernel, dim3(nblk(B, 256)), dim3(256), 0, stream, B, x, u, dt, v_max,
                       omega_max, method, x_next);
    return hipGetLastError();
}

hipError_t rmpc_launch_figure8_table(int64_t B, const int32_t *start, int32_t k, int rows, int32_t table_len,
                                     double A, double a, double dt, double *x_refs, double *u_refs,
                                     hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(figure8_table_kernel, dim3(nblk(B * rows, 256)), dim3(256), 0, stream, B, start, k, rows,
                       table_len, A, a, dt, x_refs, u_refs);
    return hipGetLastError();
}

hipError_t rmpc_launch_iota(int64_t B, int32_t *idx, int32_t *count, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(iota_kernel, dim3(nblk(B, 256)), dim3(256), 0, stream, B, idx, count);
    return hipGetLastError();
}

hipError_t rmpc_launch_ref_offsets(int64_t B, const int32_t *start, int32_t k, int32_t last, int32_t *off,
                                   hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(ref_offsets_kernel, dim3(nblk(B, 256)), dim3(256), 0, stream, B, start, k, last, off);
    return hipGetLastError();
}

hipError_t rmpc_launch_rollout_init(int64_t B, const int32_t *start, const double *x0, int32_t table_len,
                                    double A, double a, double dt, double *x, int32_t *prev_ctrl,
                                    int32_t *since, int32_t *step_count, RmpcLqrCache *cache, double *states,
                                    int32_t steps, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(rollout_init_kernel, dim3(nblk(B, 256)), dim3(256), 0, stream, B, start, x0, table_len, A,
                       a, dt, x, prev_ctrl, since, step_count, cache, states, steps);
    return hipGetLastError();
}

hipError_t rmpc_launch_rollout_plant(int64_t B, double *x, const double *u, double dt, double v_max,
                                     double omega_max, int method, int32_t k, int32_t steps, double *states,
                                     double *controls, const uint8_t *used_now, int used_fill, uint8_t *used,
                                     hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(rollout_plant_kernel, dim3(nblk(B, 256)), dim3(256), 0, stream, B, x, u, dt, v_max,
                       omega_max, method, k, steps, states, controls, used_now, used_fill, used);
    return hipGetLastError();
}

hipError_t rmpc_launch_status_count(int64_t B, const int32_t *status, const uint8_t *mask,
                                    unsigned long long *counts, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(status_count_kernel, dim3(nblk(B, 256)), dim3(256), 0, stream, B, status, mask, counts);
    return hipGetLastError();
}

hipError_t rmpc_launch_figure8(int64_t B, const double *t0, int rows, double A, double a,
                               double dt, double *x_refs, double *u_refs, hipStream_t stream) {
    if (B <= 0 || rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(figure8_kernel, dim3(nblk(B * rows, 256)), dim3(256), 0, stream, B, t0, rows, A, a,
                       dt, x_refs, u_refs);
    return hipGetLastError();
}
