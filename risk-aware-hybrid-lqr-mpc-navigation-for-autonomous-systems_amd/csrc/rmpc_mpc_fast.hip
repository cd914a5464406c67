// rmpc_mpc_fast.hip -- register-resident LTV MPC solve (the hot path of BASELINE config 3).
//
// Same QP, same algebra (rmpc_riccati.h) and same primal-dual active-set iterations as the
// generic kernel in rmpc_mpc.hip, specialised on the horizon N and block size BS so that
// every per-step quantity of a robot (sin/cos of the unwrapped reference heading, the
// reference input and position, the hinge flags) lives in VGPRs for the whole solve.
// Only the block gains (written by the backward sweep, read by the forward sweep) and the
// block inputs go through a per-wave tile in memory as coalesced 16-byte-per-lane rows,
// with the forward sweep prefetching PF blocks ahead.  Obstacle rows are recomputed from
// registers on every pass instead of being streamed.
//
// One wave per workgroup, one lane per robot.  A robot that is not certified within the
// PDAS phase (cycling, ~1e-4 of instances) or has non-finite data is appended to a retry
// list that the generic kernel (projected-Newton phase, fallback law) consumes next on
// the same stream -- restarting from scratch, so results equal the generic path's.
#include "rmpc_device.h"
#include "rmpc_internal.h"
#include "rmpc_riccati.h"

namespace rmpc {

// A per-wave tile of 16-byte rows (one row = 64 lanes x double2) addressed with buffer
// instructions: the wave's base lives in one SGPR resource, the lane's byte offset in one
// VGPR and the row offset is a constant SGPR offset -- so no per-row 64-bit address is
// ever materialised (those got spilled, and a spill reload's vmcnt(0) wait defeated the
// forward sweep's prefetch).
struct WaveRows {
    __amdgpu_buffer_rsrc_t r;
    unsigned int vo;
    __device__ __forceinline__ WaveRows(double2 *base, int rows, int lane)
        : r(__builtin_amdgcn_make_buffer_rsrc(base, 0, rows * RMPC_WAVE * 16, 0x00020000)),
          vo((unsigned int)lane * 16u) {}
    __device__ __forceinline__ double2 ld(int row) const {
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, vo, row * RMPC_WAVE * 16, 0);
        return __builtin_bit_cast(double2, v);
    }
    __device__ __forceinline__ void st(int row, double2 x) const {
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, x), r, vo, row * RMPC_WAVE * 16, 0);
    }
};

template <int N, int BS>
__global__ __launch_bounds__(64, 1) void mpc_ltv_fast_kernel(MpcFastArgs a) {
    constexpr int NB = (N + BS - 1) / BS;
    constexpr int PF = 4;     // gain blocks prefetched ahead in the forward sweep
    const int lane = threadIdx.x;
    // Obstacles (x, y, d_safe + r) staged in LDS once: read from global inside the sweeps
    // they compile to vector loads (the pointer may alias the kernel's stores) whose
    // vmcnt(0) waits would drain the gain prefetch at every step.
    __shared__ double obs_s[3 * RMPC_MAX_OBSTACLES];
    if (lane < a.no) {
        obs_s[3 * lane] = a.obs[3 * lane];
        obs_s[3 * lane + 1] = a.obs[3 * lane + 1];
        obs_s[3 * lane + 2] = a.prm.d_safe + a.obs[3 * lane + 2];
    }
    __syncthreads();
    const int64_t t = (int64_t)blockIdx.x * RMPC_WAVE + lane;
    const int64_t n = a.index ? (int64_t)*a.count : a.B;
    if (t >= n) return;
    const int64_t b = a.index ? (int64_t)a.index[t] : t;
    const MpcDevParams &p = a.prm;
    const int no = a.no;
    const double dt = p.dt, rho = p.rho;
    const double Q0 = p.Q[0], Q1 = p.Q[1], Q2 = p.Q[2], R0 = p.R[0], R1 = p.R[1];
    const double *xr = a.x_refs + (size_t)b * a.ref_rows * 3;
    const double *ur = a.u_refs + (size_t)b * a.uref_rows * 2;
    const WaveRows gt(a.gains + (size_t)blockIdx.x * NB * 4 * RMPC_WAVE, NB * 4, lane);
    const WaveRows ut(a.usol + (size_t)blockIdx.x * NB * RMPC_WAVE, NB, lane);

    // ---- setup: np.unwrap'd reference heading, linearisation data (mpc_controller.py:391-428)
    // sin/cos of the heading and the reference speed stay in VGPRs; the reference position
    // and turn rate per step live in LDS ([field][k][lane]: lane-contiguous, conflict-free).
    extern __shared__ double lds[];
    double S[N], Cs[N], V0[N];
#define PX(k) lds[(0 * N + (k)) * RMPC_WAVE + lane]
#define PY(k) lds[(1 * N + (k)) * RMPC_WAVE + lane]
#define V1(k) lds[(2 * N + (k)) * RMPC_WAVE + lane]
    double corr = 0.0, prev = xr[2], th0 = 0.0;
    bool fin = true;
#pragma unroll
    for (int k = 0; k < N; k++) {
        const double th = xr[3 * k + 2];
        if (k > 0) corr += unwrap_step(prev, th);
        prev = th;
        const double thu = th + corr;
        if (k == 0) th0 = thu;
        sincos(thu, &S[k], &Cs[k]);
        V0[k] = ur[2 * k];
        V1(k) = ur[2 * k + 1];
        PX(k) = xr[3 * k];
        PY(k) = xr[3 * k + 1];
        fin = fin && isfinite(S[k] + Cs[k] + V0[k] + V1(k) + PX(k) + PY(k));
        __builtin_amdgcn_sched_barrier(0);
    }
    const double *x0p = a.x0 + 3 * b;
    const double x0a = th0 + wrap_pi(x0p[2] - th0);                // :397-401
    const double d0 = x0p[0] - xr[0], d1 = x0p[1] - xr[1], d2 = x0a - th0;
    fin = fin && isfinite(d0 + d1 + d2);

    uint32_t Hf[N];                   // hinge-row active flags of step k (bit o)
    uint32_t Bf[NB];                  // box state per block: bits 0-1 comp 0, bits 2-3 comp 1
#pragma unroll
    for (int k = 0; k < N; k++) Hf[k] = 0;
#pragma unroll
    for (int j = 0; j < NB; j++) Bf[j] = 0;

    int it = 0, cert = 0, used = 0;
    double J = 0.0;
    const int maxit = min(p.max_iter, a.pdas_cap);
    unsigned long long tp_b = 0, tp_f = 0, tp0 = a.prof ? __builtin_amdgcn_s_memtime() : 0ull;
    const unsigned long long tp_setup = tp0;
    uint64_t hist0 = 0, hist1 = 0, hist2 = 0, hist3 = 0;   // active-set signatures (cycles)
    while (fin && it < maxit) {
        it++;
        // Keep the per-step inputs opaque to the optimiser at every iteration: otherwise it
        // hoists everything derived from them (hinge normals of every row, linearisation
        // terms, box bounds) out of this loop and the live set no longer fits in VGPRs.
#pragma unroll
        for (int k = 0; k < N; k++) {
            asm volatile("" : "+v"(S[k]), "+v"(Cs[k]), "+v"(V0[k]));
        }
        // ---------------- backward block Riccati sweep
        if (a.prof) tp0 = __builtin_amdgcn_s_memtime();
        RicV<double> V;
        V.P00 = p.P[0]; V.P01 = 0; V.P02 = 0; V.P11 = p.P[1]; V.P12 = 0; V.P22 = p.P[2];
        V.p0 = -p.P[0] * 0.0; V.p1 = -p.P[1] * 0.0; V.p2 = -p.P[2] * 0.0;
#pragma unroll
        for (int j = NB - 1; j >= 0; j--) {
            const int k0 = j * BS;
            const int k1 = (k0 + BS < N) ? k0 + BS : N;
            RicW<double> W = ric_open(V);
            double lo0 = -1e300, hi0 = 1e300, lo1 = -1e300, hi1 = 1e300;
#pragma unroll
            for (int k = k1 - 1; k >= k0; k--) {
                double q00 = Q0, q01 = 0, q11 = Q1;
                double qv0 = -Q0 * 0.0, qv1 = -Q1 * 0.0, qv2 = -Q2 * 0.0;
                if (k > 0 && Hf[k]) {
                    for (int o = 0; o < no; o++) {      // branch-free: inactive rows add 0
                        double n0, n1, hb;
                        hinge_row_fast(PX(k), PY(k), obs_s[3 * o], obs_s[3 * o + 1], obs_s[3 * o + 2], n0, n1, hb);
                        const double w = ((Hf[k] >> o) & 1u) ? rho : 0.0;
                        q00 += w * n0 * n0;
                        q01 += w * n0 * n1;
                        q11 += w * n1 * n1;
                        qv0 -= w * hb * n0;
                        qv1 -= w * hb * n1;
                    }
                }
                const double vr = fabs(V0[k]) > 0.01 ? V0[k] : 0.1;     // :425
                const double a0 = -vr * S[k] * dt, a1 = vr * Cs[k] * dt;
                const double b0 = Cs[k] * dt, b1 = S[k] * dt;
                ric_step(W, a0, a1, b0, b1, dt, q00, q01, q11, Q2, qv0, qv1, qv2, R0, R1,
                         R0 * V0[k], R1 * V1(k));
                __builtin_amdgcn_sched_barrier(0);   // keep live ranges per step (see header)
            }
#pragma unroll
            for (int k = k0; k < k1; k++) {                            // :431-436 per block
                lo0 = fmax(lo0, -p.v_max - V0[k]);
                hi0 = fmin(hi0, p.v_max - V0[k]);
                lo1 = fmax(lo1, -p.omega_max - V1(k));
                hi1 = fmin(hi1, p.omega_max - V1(k));
            }
            const int bf0 = Bf[j] & 3, bf1 = (Bf[j] >> 2) & 3;
            double G[8];
            V = ric_block_bf(W, bf0, bf1, bf0 == 1 ? lo0 : hi0, bf1 == 1 ? lo1 : hi1, G);
            gt.st(j * 4 + 0, make_double2(G[0], G[1]));
            gt.st(j * 4 + 1, make_double2(G[2], G[3]));
            gt.st(j * 4 + 2, make_double2(G[4], G[5]));
            gt.st(j * 4 + 3, make_double2(G[6], G[7]));
            __builtin_amdgcn_sched_barrier(0);
        }
        if (a.prof) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            tp_b += t1 - tp0;
            tp0 = t1;
        }
        // ---------------- forward sweep + PDAS set update + objective
        // (opaque again: stops CSE from carrying backward-sweep values across this sweep)
#pragma unroll
        for (int k = 0; k < N; k++) asm volatile("" : "+v"(S[k]), "+v"(Cs[k]), "+v"(V0[k]));
        const double eps_h = 1e-14, eps_b = 1e-13;
        int changed = 0;
        used = 0;
        J = 0.0;
        double x0 = d0, x1 = d1, x2 = d2;
        double2 g[NB][4];
#pragma unroll
        for (int j = 0; j < NB && j < PF; j++)
#pragma unroll
            for (int q = 0; q < 4; q++) g[j][q] = gt.ld(j * 4 + q);
#pragma unroll
        for (int j = 0; j < NB; j++) {
            if (j + PF < NB) {
#pragma unroll
                for (int q = 0; q < 4; q++) g[j + PF][q] = gt.ld((j + PF) * 4 + q);
            }
            const int k0 = j * BS;
            const int k1 = (k0 + BS < N) ? k0 + BS : N;
            double lo0 = -1e300, hi0 = 1e300, lo1 = -1e300, hi1 = 1e300;
#pragma unroll
            for (int k = k0; k < k1; k++) {
                lo0 = fmax(lo0, -p.v_max - V0[k]);
                hi0 = fmin(hi0, p.v_max - V0[k]);
                lo1 = fmax(lo1, -p.omega_max - V1(k));
                hi1 = fmin(hi1, p.omega_max - V1(k));
            }
            const double e0 = g[j][0].x * x0 + g[j][0].y * x1 + g[j][1].x * x2 + g[j][3].x;
            const double e1 = g[j][1].y * x0 + g[j][2].x * x1 + g[j][2].y * x2 + g[j][3].y;
            const int bf0 = Bf[j] & 3, bf1 = (Bf[j] >> 2) & 3;
            const double u0v = bf0 == 0 ? e0 : (bf0 == 1 ? lo0 : hi0);
            const double u1v = bf1 == 0 ? e1 : (bf1 == 1 ? lo1 : hi1);
            const int ns0 = box_rule(bf0, e0, lo0, hi0, eps_b), ns1 = box_rule(bf1, e1, lo1, hi1, eps_b);
            if (ns0 != bf0 || ns1 != bf1) {
                changed = 1;
                Bf[j] = (uint32_t)(ns0 | (ns1 << 2));
            }
            ut.st(j, make_double2(u0v, u1v));
#pragma unroll
            for (int k = k0; k < k1; k++) {
                J += Q0 * x0 * x0 + Q1 * x1 * x1 + Q2 * x2 * x2;
                const double uu0 = u0v + V0[k], uu1 = u1v + V1(k);
                J += R0 * uu0 * uu0 + R1 * uu1 * uu1;
                uint32_t hk = Hf[k];
                for (int o = 0; o < no; o++) {          // branch-free row update
                    double n0, n1, hb;
                    const bool kept = hinge_row_fast(PX(k), PY(k), obs_s[3 * o], obs_s[3 * o + 1], obs_s[3 * o + 2], n0, n1, hb);
                    const double r = kept ? hb - n0 * x0 - n1 * x1 : -1.0;   // unkept: never active
                    const double rp = fmax(r, 0.0);
                    J += rho * rp * rp;
                    used |= (r > 1e-6);                                        // :485
                    if (k > 0) {
                        const uint32_t act = (hk >> o) & 1u;
                        const uint32_t na = act ? (r > -eps_h) : (r > eps_h);
                        changed |= (int)(na != act);
                        hk ^= (na ^ act) << o;
                    }
                }
                Hf[k] = hk;
                const double vr = fabs(V0[k]) > 0.01 ? V0[k] : 0.1;
                const double n0 = x0 + (-vr * S[k] * dt) * x2 + (Cs[k] * dt) * u0v;
                const double n1 = x1 + (vr * Cs[k] * dt) * x2 + (S[k] * dt) * u0v;
                const double n2 = x2 + dt * u1v;
                x0 = n0; x1 = n1; x2 = n2;
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        J += p.P[0] * x0 * x0 + p.P[1] * x1 * x1 + p.P[2] * x2 * x2;
        if (a.prof) tp_f += __builtin_amdgcn_s_memtime() - tp0;
        if (!changed) { cert = 1; break; }
        // PDAS cycling: a repeated active-set signature hands the robot to the
        // projected-Newton phase of the generic kernel
        uint64_t sig = 1469598103934665603ull;
#pragma unroll
        for (int k = 0; k < N; k++) sig = (sig ^ (uint64_t)Hf[k]) * 1099511628211ull;
#pragma unroll
        for (int j = 0; j < NB; j++) sig = (sig ^ (uint64_t)Bf[j]) * 1099511628211ull;
        if (sig == hist0 || sig == hist1 || sig == hist2 || sig == hist3) break;
        hist3 = hist2; hist2 = hist1; hist1 = hist0; hist0 = sig;
    }
    if (a.prof) {      // wave totals = max over lanes (the last lane saw every iteration)
        unsigned long long mb = tp_b, mf = tp_f, mi = (unsigned long long)it;
        for (int off = 32; off > 0; off >>= 1) {
            mb = max(mb, (unsigned long long)__shfl_xor((long long)mb, off));
            mf = max(mf, (unsigned long long)__shfl_xor((long long)mf, off));
            mi = max(mi, (unsigned long long)__shfl_xor((long long)mi, off));
        }
        if (lane == 0) {
            atomicAdd(a.prof + 16, mb);
            atomicAdd(a.prof + 17, mf);
            atomicAdd(a.prof + 18, mi);
            atomicAdd(a.prof + 19, __builtin_amdgcn_s_memtime() - tp_setup);
            atomicAdd(a.prof + 20, 1ull);
        }
    }
    if (!cert || !isfinite(J)) {
        const int slot = atomicAdd(a.retry_count, 1);        // the next stage takes over
        a.retry[slot] = (int32_t)b;
        if (a.retry_sets) {                                   // ... from this active set
            uint32_t *ws = a.retry_sets + (size_t)slot * (N + NB + 1);
#pragma unroll
            for (int k = 0; k < N; k++) ws[k] = Hf[k];
#pragma unroll
            for (int j = 0; j < NB; j++) ws[N + j] = Bf[j];
            ws[N + NB] = (uint32_t)it;
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < N; k++) asm volatile("" : "+v"(S[k]), "+v"(Cs[k]), "+v"(V0[k]));
    // ---- outputs (mpc_controller.py:484-520): x_pred = x_refs + dx (not unwrapped),
    // u = u_refs + du, omega ramp, step counter
    const int sc = a.step_count ? a.step_count[b] : 0;
    double x0 = d0, x1 = d1, x2 = d2;
    double uc0 = 0, uc1 = 0;
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const double2 u = ut.ld(j);
        const int k0 = j * BS;
        const int k1 = (k0 + BS < N) ? k0 + BS : N;
#pragma unroll
        for (int k = k0; k < k1; k++) {
            double v0 = u.x + V0[k], v1 = u.y + V1(k);
            if (k == 0) {
                if (sc < p.ramp_up_steps) {                           // :502-505
                    const double lim = p.omega_max * ((double)(sc + 1) / (double)p.ramp_up_steps);
                    v1 = clampv(v1, -lim, lim);
                }
                uc0 = v0;
                uc1 = v1;
            }
            if (a.u_seq) {
                a.u_seq[((size_t)b * N + k) * 2] = v0;
                a.u_seq[((size_t)b * N + k) * 2 + 1] = v1;
            }
            if (a.x_pred) {
                double *xp = a.x_pred + ((size_t)b * (N + 1) + k) * 3;
                xp[0] = x0 + PX(k);
                xp[1] = x1 + PY(k);
                xp[2] = x2 + xr[3 * k + 2];
            }
            const double vr = fabs(V0[k]) > 0.01 ? V0[k] : 0.1;
            const double n0 = x0 + (-vr * S[k] * dt) * x2 + (Cs[k] * dt) * u.x;
            const double n1 = x1 + (vr * Cs[k] * dt) * x2 + (S[k] * dt) * u.x;
            const double n2 = x2 + dt * u.y;
            x0 = n0; x1 = n1; x2 = n2;
        }
    }
    if (a.x_pred) {
        double *xp = a.x_pred + ((size_t)b * (N + 1) + N) * 3;
        xp[0] = x0 + xr[3 * N];
        xp[1] = x1 + xr[3 * N + 1];
        xp[2] = x2 + xr[3 * N + 2];
    }
    if (a.step_count) a.step_count[b] = sc + 1;                        // :507
    a.u0[2 * b] = uc0;
    a.u0[2 * b + 1] = uc1;
    if (a.cost) a.cost[b] = J;
    if (a.slack_used) a.slack_used[b] = (uint8_t)used;
    a.status[b] = RMPC_OPTIMAL;
    if (a.iters) a.iters[b] = it;
}

}  // namespace rmpc

using namespace rmpc;

#undef PX
#undef PY
#undef V1

bool rmpc_mpc_fast_supported(int N, int bs) {
    return (bs == 1 && (N == 6 || N == 10 || N == 20)) || (bs == 2 && N == 6);
}

hipError_t rmpc_launch_mpc_fast_f64(const MpcFastArgs &a, int N, int bs, hipStream_t stream) {
    const int64_t n = a.B;
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + RMPC_WAVE - 1) / RMPC_WAVE)), block(RMPC_WAVE);
    const size_t lds = (size_t)3 * N * RMPC_WAVE * sizeof(double);
    if (bs == 1 && N == 20) hipLaunchKernelGGL((mpc_ltv_fast_kernel<20, 1>), grid, block, lds, stream, a);
    else if (bs == 1 && N == 10) hipLaunchKernelGGL((mpc_ltv_fast_kernel<10, 1>), grid, block, lds, stream, a);
    else if (bs == 1 && N == 6) hipLaunchKernelGGL((mpc_ltv_fast_kernel<6, 1>), grid, block, lds, stream, a);
    else if (bs == 2 && N == 6) hipLaunchKernelGGL((mpc_ltv_fast_kernel<6, 2>), grid, block, lds, stream, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}
