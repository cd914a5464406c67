// rmpc_fast_body.h -- the lane-per-robot PDAS stage (fast_body), included by the stage kernel
// (rmpc_mpc_fast.hip: mpc_ltv_fast_kernel).  `wid` is the wave's index in the stage.
#pragma once
#include "rmpc_device.h"
#include "rmpc_internal.h"
#include "rmpc_riccati.h"

namespace rmpc {

// A per-wave tile of 16-byte rows (one row = 64 lanes x double2) addressed with buffer
// instructions: the wave's base lives in one SGPR resource, the lane's byte offset in one
// VGPR and the row offset is a constant SGPR offset -- so no per-row 64-bit address is
// ever materialised (those got spilled, and a spill reload's vmcnt(0) wait defeated the
// forward sweep's prefetch).
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));

#ifndef RMPC_GAIN_LD_AUX
#define RMPC_GAIN_LD_AUX 0     // cache policy of the gain-tile loads / stores (A/B: 2 = nt)
#endif
#ifndef RMPC_GAIN_ST_AUX
#define RMPC_GAIN_ST_AUX 0
#endif
template <int RB>      // bytes per lane and row: 16 or 8
struct WaveRows {
    __amdgpu_buffer_rsrc_t r;
    unsigned int vo;
    __device__ __forceinline__ WaveRows(void *base, int rows, int lane)
        : r(__builtin_amdgcn_make_buffer_rsrc(base, 0, rows * RMPC_WAVE * RB, 0x00020000)),
          vo((unsigned int)lane * RB) {}
    __device__ __forceinline__ u4v ld16(int row) const {
        return __builtin_amdgcn_raw_buffer_load_b128(r, vo, row * RMPC_WAVE * RB, RMPC_GAIN_LD_AUX);
    }
    __device__ __forceinline__ void st16(int row, u4v x) const {
        __builtin_amdgcn_raw_buffer_store_b128(x, r, vo, row * RMPC_WAVE * RB, RMPC_GAIN_ST_AUX);
    }
    __device__ __forceinline__ u2v ld8(int row) const {
        return __builtin_amdgcn_raw_buffer_load_b64(r, vo, row * RMPC_WAVE * RB, 0);
    }
    __device__ __forceinline__ void st8(int row, u2v x) const {
        __builtin_amdgcn_raw_buffer_store_b64(x, r, vo, row * RMPC_WAVE * RB, 0);
    }
};

// The 8 gain values of a block (K rows, k) as 16-byte rows: 4 per block in fp64, 2 in fp32
template <typename T> struct GainTile;
template <> struct GainTile<double> {
    WaveRows<16> w;
    __device__ __forceinline__ GainTile(void *base, int nb, int lane, int pr = 1) : w(base, nb * 4 / pr, lane) {}
    // Paired lanes (the fp64 refinement of config 4): two rows per block; in row 2j+q lane 2r's
    // slot holds G[2q], G[2q+1] and lane 2r+1's slot G[4+2q], G[5+2q].  Each lane stores its
    // half and reads both halves back (the pair's gains are bitwise identical).
    __device__ __forceinline__ void st_half(int j, const double G[8], int pp) const {
#pragma unroll
        for (int q = 0; q < 2; q++)
            w.st16(2 * j + q, __builtin_bit_cast(u4v, make_double2(G[4 * pp + 2 * q], G[4 * pp + 2 * q + 1])));
    }
    __device__ __forceinline__ void ld_pair(int j, double G[8], int pp) const {
        const unsigned v0 = w.vo - (unsigned)pp * 16u;
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const double2 x = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
                w.r, v0, (2 * j + q) * RMPC_WAVE * 16, RMPC_GAIN_LD_AUX));
            const double2 y = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
                w.r, v0 + 16u, (2 * j + q) * RMPC_WAVE * 16, RMPC_GAIN_LD_AUX));
            G[2 * q] = x.x; G[2 * q + 1] = x.y;
            G[4 + 2 * q] = y.x; G[5 + 2 * q] = y.y;
        }
    }
    __device__ __forceinline__ void st(int j, const double G[8]) const {
#pragma unroll
        for (int q = 0; q < 4; q++) w.st16(j * 4 + q, __builtin_bit_cast(u4v, make_double2(G[2 * q], G[2 * q + 1])));
    }
    __device__ __forceinline__ void ld(int j, double G[8]) const {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const double2 v = __builtin_bit_cast(double2, w.ld16(j * 4 + q));
            G[2 * q] = v.x;
            G[2 * q + 1] = v.y;
        }
    }
};
template <> struct GainTile<float> {
    WaveRows<16> w;
    __device__ __forceinline__ GainTile(void *base, int nb, int lane, int = 1) : w(base, nb * 2, lane) {}
    // Paired lanes (two lanes per robot, identical gains): each lane stores one half of the
    // block's 8 values (lane 2r: G0..3 in row 2j, lane 2r+1: G4..7 in row 2j+1, both at the
    // pair's own lane offsets) and reads both halves back.
    __device__ __forceinline__ void st_half(int j, const float G[8], int pp) const {
        const float4 v = pp ? make_float4(G[4], G[5], G[6], G[7]) : make_float4(G[0], G[1], G[2], G[3]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), w.r, w.vo + (unsigned)pp * RMPC_WAVE * 16u,
                                               j * 2 * RMPC_WAVE * 16, 0);
    }
    __device__ __forceinline__ void ld_pair(int j, float G[8], int pp) const {
        const unsigned v0 = w.vo - (unsigned)pp * 16u, v1 = v0 + 16u + RMPC_WAVE * 16u;
        const float4 x = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(w.r, v0, j * 2 * RMPC_WAVE * 16, 0));
        const float4 y = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(w.r, v1, j * 2 * RMPC_WAVE * 16, 0));
        G[0] = x.x; G[1] = x.y; G[2] = x.z; G[3] = x.w;
        G[4] = y.x; G[5] = y.y; G[6] = y.z; G[7] = y.w;
    }
    __device__ __forceinline__ void st(int j, const float G[8]) const {
#pragma unroll
        for (int q = 0; q < 2; q++)
            w.st16(j * 2 + q, __builtin_bit_cast(u4v, make_float4(G[4 * q], G[4 * q + 1], G[4 * q + 2], G[4 * q + 3])));
    }
    __device__ __forceinline__ void ld(int j, float G[8]) const {
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const float4 v = __builtin_bit_cast(float4, w.ld16(j * 2 + q));
            G[4 * q] = v.x; G[4 * q + 1] = v.y; G[4 * q + 2] = v.z; G[4 * q + 3] = v.w;
        }
    }
};

// Active-set flags packed into few VGPRs (the kernel runs at the register limit; the
// sweeps are fully unrolled, so every index is a compile-time constant and a get/set is one
// or two shift/mask instructions).  Hinge rows: 16 bits per step (bit o); box states:
// 4 bits per block (bits 0-1 component 0, bits 2-3 component 1).
template <int N> struct HingeFlags {
    uint32_t w[(N + 1) / 2];
    __device__ __forceinline__ uint32_t get(int k) const { return (w[k >> 1] >> (16 * (k & 1))) & 0xffffu; }
    __device__ __forceinline__ void set(int k, uint32_t v) {
        const int sh = 16 * (k & 1);
        w[k >> 1] = (w[k >> 1] & ~(0xffffu << sh)) | (v << sh);
    }
};
template <int NB> struct BoxFlags {
    uint32_t w[(NB + 7) / 8];
    __device__ __forceinline__ uint32_t get(int j) const { return (w[j >> 3] >> (4 * (j & 7))) & 0xfu; }
    __device__ __forceinline__ void set(int j, uint32_t v) {
        const int sh = 4 * (j & 7);
        w[j >> 3] = (w[j >> 3] & ~(0xfu << sh)) | (v << sh);
    }
};

// Value of the other lane of a pair (DPP quad_perm [1,0,3,2]): paired-lane robots
__device__ __forceinline__ float pair_xchg(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ double pair_xchg(double v) {
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)bits, 0xB1, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(bits >> 32), 0xB1, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ uint32_t pair_xchg(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}

#ifndef RMPC_OPQ
#define RMPC_OPQ 0
#endif
// Row geometry inputs made opaque where the row loops unroll (NO > 0): the reference
// positions and obstacles are loop-invariant LDS loads, and without this the optimiser hoists
// every row's normal and offset (60 rows x 3 values at N = 20) out of the PDAS loop and
// spills them to scratch.
template <int NO, typename T> __device__ __forceinline__ T opq(T v) {
    if constexpr (NO > 0 && RMPC_OPQ) asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ double rsq_approx(double x) { return __builtin_amdgcn_rsq(x); }
__device__ __forceinline__ float rsq_approx(float x) { return __builtin_amdgcn_rsqf(x); }

template <typename T> struct Big;
template <> struct Big<double> { static constexpr double v = 1e300; };
template <> struct Big<float> { static constexpr float v = 1e30f; };

// LTI = true: MPCController.solve (mpc_controller.py:150-314) in error coordinates
// e_k = x_k - x_ref,k (references padded with their last row).  The LTI model applied to
// absolute states then reads e_{k+1} = A e_k + B u_k + c_k with c_k = A x_ref,k - x_ref,k+1,
// so the sweeps are the LTV ones plus the affine term: p += P c_k before each backward step
// and + c_k in each forward step.  One linearisation (constants), |u| box, u_ref terms 0;
// per-step registers S/Cs/V0 hold c_k and the V1 slot the reference heading.
//
// NO > 0: the obstacle count is a compile-time constant (must equal a.no) and the row loops
// unroll, so the rows of a step and the state recursion interleave instead of running as a
// loop of dependent row chains; NO = 0 keeps the runtime loop (any n_o <= 16).
//
// PR = 2 (paired lanes): two lanes per robot, 32 robots per wave.  Both lanes run the same
// recursions on the same data (bitwise-identical Riccati, gains and trajectory); the hinge
// rows are split -- lane 2r+p owns obstacles p*NO/2 .. p*NO/2 + NO/2 - 1 -- and the rows'
// Hessian and gradient terms, objective share, set changes and slack flags are combined
// across the pair with one DPP swap (a + b on one lane, b + a on the other: identical).
// Used where the rows dominate a step (8 obstacles) and the batch fills only half the SIMDs
// at one lane per robot (BASELINE config 4: 32768 robots = 512 waves).
//
// WS: the warm start across calls (MpcFastArgs::prev_sets) is compiled in.  Config 3's instance
// is built both ways and the cold one launched when prev_sets is null: the read and write-back
// cost its register allocation ~1% (profiles/r03/ab_warm_start.txt).
template <int N, int BS, typename T, bool LTI, int NO = 0, int PR = 1, bool WS = true>
__device__ __forceinline__ void fast_body(MpcFastArgs a, const unsigned wid, int &its_out) {
    static_assert(!LTI || BS == 1, "LTI ignores move blocking");
    static_assert(PR == 1 || (PR == 2 && NO > 0 && NO % 2 == 0 && BS == 1 && !LTI && NO / 2 <= 4),
                  "paired lanes: compile-time rows, split evenly, block size 1, LTV");
    constexpr int NOL = NO / PR;           // rows per lane and step (compile-time rows)
    constexpr int NB = (N + BS - 1) / BS;
#ifndef RMPC_PF3
#define RMPC_PF3 4
#endif
    constexpr int PF = NO > 0 ? RMPC_PF3 : 4;     // gain blocks prefetched ahead in the forward sweep
    constexpr bool F64 = sizeof(T) == 8;
    const T BIG = Big<T>::v;
    const int lane = threadIdx.x;
    const unsigned long long t_entry = a.prof ? __builtin_amdgcn_s_memtime() : 0ull;   // (diagnostics)
    // Obstacles (x, y, d_safe + r) staged in LDS once: read from global inside the sweeps
    // they compile to vector loads (the pointer may alias the kernel's stores) whose
    // vmcnt(0) waits would drain the gain prefetch at every step.
    __shared__ T obs_s[3 * (RMPC_MAX_OBSTACLES + 1)];
    if (lane < a.no) {
        obs_s[3 * lane] = (T)a.obs[3 * lane];
        obs_s[3 * lane + 1] = (T)a.obs[3 * lane + 1];
        obs_s[3 * lane + 2] = (T)(a.prm.d_safe + a.obs[3 * lane + 2]);
    } else if (lane <= RMPC_MAX_OBSTACLES) {   // the rows' one-ahead prefetch reads slot no
        obs_s[3 * lane] = (T)0;
        obs_s[3 * lane + 1] = (T)0;
        obs_s[3 * lane + 2] = (T)0;
    }
    __syncthreads();
    const int pp = PR == 2 ? (lane & 1) : 0;           // the lane's half of its robot's rows
    const int obase = pp * NOL;                        // its first obstacle
    const int64_t t = (int64_t)wid * (RMPC_WAVE / PR) + lane / PR;
    const int64_t n = a.index ? (int64_t)*a.count : a.B;
    if (t >= n) return;
    const int64_t b = a.index ? (int64_t)a.index[t] : t;
    const MpcDevParams &p = a.prm;
    const int no = NO > 0 ? NO : a.no;
#ifndef RMPC_UB
#define RMPC_UB 1
#endif
#ifndef RMPC_UF
#define RMPC_UF 1
#endif
    constexpr bool UB = NO > 0 && RMPC_UB, UF = NO > 0 && RMPC_UF;
    const int nob = UB ? NO : a.no, nof = UF ? NO : a.no;
    constexpr int UNRB = UB ? NO : 2, UNRF = UF ? NO : 2;   // row-loop unroll (runtime: the compiler's own x2)
    const T dt = (T)p.dt, rho = (T)p.rho;
    const T Q0 = (T)p.Q[0], Q1 = (T)p.Q[1], Q2 = (T)p.Q[2], R0 = (T)p.R[0], R1 = (T)p.R[1];
    const T P0 = (T)p.P[0], P1 = (T)p.P[1], P2 = (T)p.P[2];
    const T vmax = (T)p.v_max, omax = (T)p.omega_max;
    const double *xr = a.x_refs + ref_row0(a.prm.ref_off, b, a.ref_rows) * 3;
    const double *ur = a.u_refs + ref_row0(a.prm.ref_off, b, a.uref_rows) * 2;
    // per-wave gain tile (sized for fp64; fp32 uses half)
    // (paired lanes, fp32: twice the waves, each with an fp32-sized tile -- the same buffer)
    const GainTile<T> gt(a.gains + (size_t)wid * NB * (PR == 2 ? 2 : 4) * RMPC_WAVE, NB, lane, PR);

    // ---- setup: np.unwrap'd reference heading, linearisation data (mpc_controller.py:391-428)
    // sin/cos of the heading and the reference speed stay in VGPRs; the reference position
    // and turn rate per step live in LDS ([field][k][lane]: lane-contiguous, conflict-free).
    // The unwrap and sin/cos run in fp64 for both T.
    extern __shared__ double lds_raw[];
    T *const lds = reinterpret_cast<T *>(lds_raw);
    // [field][k][robot of the wave]: paired lanes share their robot's entries (both lanes write
    // the same value; both read it -- a broadcast), so a paired wave holds 32 columns
    constexpr int LW = RMPC_WAVE / PR;
    const int ll = lane / PR;
    T S[N], Cs[N], V0[N];
#define PX(k) lds[(0 * N + (k)) * LW + ll]
#define PY(k) lds[(1 * N + (k)) * LW + ll]
#define V1(k) lds[(2 * N + (k)) * LW + ll]
    bool fin = true;
    T d0, d1, d2;
    T la0 = 0, la1 = 0, lb0 = 0, lb1 = 0;        // LTI: the one linearisation
    double xsN0 = 0, xsN1 = 0, xsN2 = 0;          // LTI: terminal reference state
    const double *x0p = a.x0 + 3 * b;
    if constexpr (LTI) {
        const double v = ur[0];
        const double vr = fabs(v) > 0.01 ? v : 0.1;                 // :186
        double sn, cs;
        sincos(xr[2], &sn, &cs);
        const double A0 = -vr * sn * p.dt, A1 = vr * cs * p.dt;
        la0 = (T)A0; la1 = (T)A1; lb0 = (T)(cs * p.dt); lb1 = (T)(sn * p.dt);
        const int last = a.ref_rows - 1;
#pragma unroll
        for (int k = 0; k < N; k++) {                              // :172-183 padding
            const int kr = k < last ? k : last, kn = k + 1 < last ? k + 1 : last;
            const double px = xr[3 * kr], py = xr[3 * kr + 1], th = xr[3 * kr + 2];
            S[k] = (T)(px + A0 * th - xr[3 * kn]);
            Cs[k] = (T)(py + A1 * th - xr[3 * kn + 1]);
            V0[k] = (T)(th - xr[3 * kn + 2]);
            V1(k) = (T)th;
            PX(k) = (T)px;
            PY(k) = (T)py;
            fin = fin && isfinite(S[k] + Cs[k] + V0[k] + V1(k));
            __builtin_amdgcn_sched_barrier(0);
        }
        const int kN = N < last ? N : last;
        xsN0 = xr[3 * kN]; xsN1 = xr[3 * kN + 1]; xsN2 = xr[3 * kN + 2];
        d0 = (T)(x0p[0] - xr[0]); d1 = (T)(x0p[1] - xr[1]); d2 = (T)(x0p[2] - xr[2]);
        fin = fin && isfinite(sn + cs + vr + xsN0 + xsN1 + xsN2);
    } else {
        double corr = 0.0, prev = 0.0, th0 = 0.0;
        // Full fp64 waves stage their robots' reference rows through LDS: each load instruction
        // reads 16 consecutive doubles of four robots' rows (four 128-B segments) instead of one
        // double of each of 64 rows, which at a full chip made the setup 2.5x its uncontended
        // time (64 cache lines per instruction).  Robots may come from an index list (the hybrid
        // switch's MPC branch) and rows from a shared table (rollouts): each 16-lane group
        // addresses its own robot's row.  The staging fills PX/PY/V1 and V0 directly and parks
        // the heading in S[k] for the unwrap / sin-cos loop below.
        // (round 3: also the paired-lane and fp32 instances -- a paired wave stages its 32
        // robots, and fp32 keeps the fp64 heading for the unwrap / sin-cos in TH)
#ifndef RMPC_COAL_ALL
#define RMPC_COAL_ALL 1
#endif
        constexpr int RW = RMPC_WAVE / PR;                   // robots per wave
        const bool coal = (F64 ? (PR == 1 || RMPC_COAL_ALL) : RMPC_COAL_ALL) && (int64_t)(wid + 1) * RW <= n;
        double TH[F64 ? 1 : N];                              // fp32: the staged fp64 headings
        if (coal) {
            constexpr int SP = 17;                           // scratch row stride in doubles (bank spread)
            double *const stg = lds_raw + (size_t)3 * N * LW * sizeof(T) / sizeof(double);
            const int64_t t0 = (int64_t)wid * RW;
            const int rr = lane >> 4, ee = lane & 15;
            // all of an array's loads are issued before the first LDS round (one memory latency
            // per array, not per round)
            // robot 4q + rr's first reference row in a shared table, else its robot index
            int64_t row[RW / 4];
#pragma unroll
            for (int q = 0; q < RW / 4; q++) {
                const int64_t tq = t0 + 4 * q + rr;
                const int64_t bq = a.index ? (int64_t)a.index[tq] : tq;
                row[q] = a.prm.ref_off ? (int64_t)a.prm.ref_off[bq] : bq;
            }
            // both arrays' loads are issued before the first LDS round (RMPC_SETUP_PF; 0: each
            // array's loads right before its own rounds, two memory latencies per wave); not for
            // paired lanes, whose fp64 N = 30 instance then spills (38 VGPRs against 2)
#ifndef RMPC_SETUP_PF
#define RMPC_SETUP_PF 1
#endif
            auto ld = [&](const double *src, const int W, const int rows, const int ne, auto &v)
                __attribute__((always_inline)) {
                constexpr int NP = sizeof(v) / sizeof(v[0]);
#pragma unroll
                for (int ps = 0; ps < NP; ps++)
#pragma unroll
                    for (int q = 0; q < RW / 4; q++) {
                        const int e = 16 * ps + ee;
                        const int64_t r0 = a.prm.ref_off ? row[q] : row[q] * rows;   // (ref_row0)
                        v[ps][q] = e < ne ? src[r0 * W + e] : 0.0;
                    }
            };
            auto rounds = [&](const int ne, auto &v, auto put) __attribute__((always_inline)) {
                constexpr int NP = sizeof(v) / sizeof(v[0]);
#pragma unroll
                for (int ps = 0; ps < NP; ps++) {
                    __syncthreads();
#pragma unroll
                    for (int q = 0; q < RW / 4; q++) stg[(4 * q + rr) * SP + ee] = v[ps][q];
                    __syncthreads();
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        if (16 * ps + i < ne) put(16 * ps + i, stg[ll * SP + i]);
                }
            };
            auto putx = [&](const int e, const double v) __attribute__((always_inline)) {
                if (e % 3 == 0) PX(e / 3) = (T)v;
                else if (e % 3 == 1) PY(e / 3) = (T)v;
                else if constexpr (F64) S[e / 3] = v;        // the heading, for the loop below
                else TH[e / 3] = v;
            };
            auto putu = [&](const int e, const double v) __attribute__((always_inline)) {
                if (e % 2 == 0) V0[e / 2] = (T)v;
                else V1(e / 2) = (T)v;
            };
            double vx[(3 * N + 15) / 16][RW / 4], vu[(2 * N + 15) / 16][RW / 4];
            ld(a.x_refs, 3, a.ref_rows, 3 * N, vx);
            constexpr bool SPF = RMPC_SETUP_PF && PR == 1;
            if constexpr (SPF) ld(a.u_refs, 2, a.uref_rows, 2 * N, vu);
            rounds(3 * N, vx, putx);
            if constexpr (!SPF) ld(a.u_refs, 2, a.uref_rows, 2 * N, vu);
            rounds(2 * N, vu, putu);
        }
#pragma unroll
        for (int k = 0; k < N; k++) {
            double th;
            if constexpr (F64) th = coal ? (double)S[k] : xr[3 * k + 2];
            else th = coal ? TH[k] : xr[3 * k + 2];
            if (k > 0) corr += unwrap_step(prev, th);
            prev = th;
            const double thu = th + corr;
            if (k == 0) th0 = thu;
            double sn, cs;
            sincos_moderate(thu, &sn, &cs);
            S[k] = (T)sn;
            Cs[k] = (T)cs;
            if (!coal) {
                V0[k] = (T)ur[2 * k];
                V1(k) = (T)ur[2 * k + 1];
                PX(k) = (T)xr[3 * k];
                PY(k) = (T)xr[3 * k + 1];
            }
            fin = fin && isfinite(S[k] + Cs[k] + V0[k] + V1(k) + PX(k) + PY(k));
            __builtin_amdgcn_sched_barrier(0);
        }
        const double x0a = th0 + wrap_pi(x0p[2] - th0);            // :397-401
        d0 = (T)(x0p[0] - xr[0]); d1 = (T)(x0p[1] - xr[1]); d2 = (T)(x0a - th0);
    }
    fin = fin && isfinite(d0 + d1 + d2);

    HingeFlags<N> Hf;                 // hinge-row active flags of step k (bit o)
    BoxFlags<NB> Bf;                  // box state per block
#pragma unroll
    for (int i = 0; i < (N + 1) / 2; i++) Hf.w[i] = 0;
#pragma unroll
    for (int i = 0; i < (NB + 7) / 8; i++) Bf.w[i] = 0;

    int it = 0, cert = 0, used = 0, cycled = 0;
    T J = 0;
    const int maxit0 = min(p.max_iter, a.pdas_cap);
    unsigned long long tp_b = 0, tp_f = 0, tp0 = a.prof ? __builtin_amdgcn_s_memtime() : 0ull;
    const unsigned long long tp_setup = tp0;
    uint64_t hist0 = 0, hist1 = 0, hist2 = 0, hist3 = 0;   // active-set signatures (cycles)
    // active-set signature of the current sets (paired lanes: the pair's combined row flags,
    // independent of the lane order)
    auto set_sig = [&]() {
        uint64_t sig = 1469598103934665603ull;
#pragma unroll
        for (int i = 0; i < (N + 1) / 2; i++) {
            uint32_t w = Hf.w[i];
            if constexpr (PR == 2) {       // lane-order-independent: (lane 2r's bits) | (lane 2r+1's) << NOL
                const uint32_t o = pair_xchg(w);
                w = pp ? (o | (w << NOL)) : (w | (o << NOL));
            }
            sig = (sig ^ (uint64_t)w) * 1099511628211ull;
        }
#pragma unroll
        for (int i = 0; i < (NB + 7) / 8; i++) sig = (sig ^ (uint64_t)Bf.w[i]) * 1099511628211ull;
        return sig;
    };
    if (a.warm_sets) {
        // Continuing pass over a compacted list: the previous pass handed this robot on with its
        // sets after `it` PDAS iterations (retry record at list position t).  The robot resumes
        // exactly where it stopped: the same sets, the same iteration count, and the cycle
        // history's newest entry (the signature of these sets).
        const uint32_t *ws = a.warm_sets + t;           // slot-minor records: coalesced
#pragma unroll
        for (int k = 0; k < N; k++) {
            const uint32_t w = ws[k * a.B];
            Hf.set(k, PR == 2 ? (w >> obase) & ((1u << NOL) - 1u) : w);
        }
#pragma unroll
        for (int j = 0; j < NB; j++) Bf.set(j, ws[(N + j) * a.B]);
        it = (int)ws[(N + NB) * a.B];
        if (a.warm_hist) {                              // the previous pass's cycle history
            const uint32_t *h = ws + (size_t)(N + NB + 1) * a.B;
            hist0 = (uint64_t)h[0] | (uint64_t)h[(size_t)a.B] << 32;
            hist1 = (uint64_t)h[(size_t)2 * a.B] | (uint64_t)h[(size_t)3 * a.B] << 32;
            hist2 = (uint64_t)h[(size_t)4 * a.B] | (uint64_t)h[(size_t)5 * a.B] << 32;
            hist3 = (uint64_t)h[(size_t)6 * a.B] | (uint64_t)h[(size_t)7 * a.B] << 32;
        } else if (it > 0) hist0 = set_sig();
    } else if (WS && a.prev_sets && a.prev_sets[(size_t)(N + NB) * a.B + b] + 1u == a.prev_stamp) {
        // Warm start from this robot's previous solve (rmpc_ctx_set_warm_start): the PDAS
        // counterpart of the reference's warm_start=True with get_warm_start's one-step shift
        // (mpc_controller.py:272-277, 470-475, 524-538).  Its certified sets, shifted by
        // prev_shift steps with the last step repeated, are the first iterate's sets; the QP and
        // its optimum are unchanged (the outputs come from the certified sets only).
        const uint32_t *ws = a.prev_sets + b;
        const int sh = a.prev_shift, shb = a.prev_shift / BS;
        const uint32_t hm = PR == 2 ? ((1u << NOL) - 1u) : (no >= 16 ? 0xffffu : ((1u << no) - 1u));
#pragma unroll
        for (int k = 1; k < N; k++) {
            const int ks = k + sh < N ? k + sh : N - 1;
            const uint32_t w = ws[(size_t)ks * a.B];
            Hf.set(k, (PR == 2 ? (w >> obase) : w) & hm);
        }
#pragma unroll
        for (int j = 0; j < NB; j++) {
            const int js = j + shb < NB ? j + shb : NB - 1;
            uint32_t v = ws[(size_t)(N + js) * a.B] & 0xfu;
            if ((v & 3u) == 3u) v &= ~3u;           // (never both bounds of a component)
            if ((v & 12u) == 12u) v &= ~12u;
            Bf.set(j, v);
        }
    }
    else if (a.init_zc) {
        // Zero-correction start: the hinge rows the reference inputs alone would violate start
        // active (the free response x_{k+1} = A_k x_k (+ c_k), du = 0).  The QP and its optimum
        // are unchanged; only the first PDAS iterate is closer to it.
        T x0 = d0, x1 = d1, x2 = d2;
#pragma unroll
        for (int k = 0; k < N; k++) {
            if (k > 0) {
                const T px = PX(k), py = PY(k);
                uint32_t h = 0;
#pragma unroll
                for (int o = 0; o < (NO > 0 ? NOL : RMPC_MAX_OBSTACLES); o++) {
                    if (NO == 0 && o >= a.no) break;
                    const T ox = obs_s[3 * (obase + o)], oy = obs_s[3 * (obase + o) + 1], sf = obs_s[3 * (obase + o) + 2];
                    const T ddx = px - ox, ddy = py - oy;
                    const T dd = ddx * ddx + ddy * ddy;
                    T y = rsq_approx(dd);
                    if constexpr (F64) {
                        const T hh = (T)0.5 * dd * y;
                        y = fma(y, fma(-hh, y, (T)0.5), y);
                    }
                    const T r = fma(-fma(ddy, x1, fma(ddx, x0, dd)), y, sf);
                    h |= (dd * y > (T)0.01 && r > (T)0) ? (1u << o) : 0u;
                }
                Hf.set(k, h);
            }
            if constexpr (LTI) {
                const T n0 = x0 + la0 * x2 + S[k], n1 = x1 + la1 * x2 + Cs[k];
                x2 = x2 + V0[k];
                x0 = n0; x1 = n1;
            } else {
                const T vr = fabs(V0[k]) > (T)0.01 ? V0[k] : (T)0.1;
                x0 = x0 + (-vr * S[k] * dt) * x2;
                x1 = x1 + (vr * Cs[k] * dt) * x2;
            }
        }
    }
    const int it_start = it;
    // (fp64 refinement of fp32-certified sets: `extra_cap` more PDAS solves from them)
    const int maxit = a.extra_cap > 0 ? min(p.max_iter, it + a.extra_cap) : maxit0;
    // The last GREG blocks the backward sweep forms (j < GREG) stay in registers instead of the
    // tile: the forward sweep and the output pass read them first, and a tile load of them
    // waits (in-order vmcnt) for every store of the sweep to complete.  Config 3's fp64 LTV
    // instances only (4 blocks: in flight 336.6-338.1M -> 345.0-350.7M solves/s, one batch
    // alone 188.0M -> 191.2M); elsewhere the extra registers spill.
#ifndef RMPC_GREG
#define RMPC_GREG 4
#endif
    constexpr int GREG0 = (F64 && PR == 1 && !LTI && N == 20 && BS == 1) ? RMPC_GREG : 0;
    constexpr int GREG = GREG0 < NB ? GREG0 : NB;
    T greg[GREG > 0 ? GREG : 1][8];
    // The next GLDS blocks (GREG <= j < GREG + GLDS) go to the setup's staging scratch in LDS,
    // free once the setup is done: [block][pair q][lane] pairs, each lane its own slots (a wave
    // per workgroup, so no barrier).  LDS accesses count in lgkmcnt, not behind the tile stores.
#ifndef RMPC_GLDS
#define RMPC_GLDS 2
#endif
    constexpr int GLDS = (GREG > 0 && GREG + RMPC_GLDS <= NB) ? RMPC_GLDS : 0;
    // Diagnostics builds only (scripts/build_variant.sh), both wrong by construction:
    // RMPC_GAIN_NOMEM drops the tile traffic of the blocks beyond GREG + GLDS (the forward sweep
    // reads block 0's gains there), RMPC_NOCERT runs every robot to the stage's cap and drops
    // its outputs -- together the upper bound of what removing the tile traffic could save.
#ifndef RMPC_GAIN_NOMEM
#define RMPC_GAIN_NOMEM 0
#endif
#ifndef RMPC_NOCERT
#define RMPC_NOCERT 0
#endif
    static_assert(GLDS * 8 * RMPC_WAVE * sizeof(T) <= RMPC_WAVE * 17 * sizeof(double), "LDS gain blocks exceed the scratch");
    struct alignas(2 * sizeof(T)) GPair { T x, y; };
    GPair *const glds = reinterpret_cast<GPair *>(lds_raw + (size_t)3 * N * LW * sizeof(T) / sizeof(double)) + lane;
    auto gload = [&](const int j, T *dst) __attribute__((always_inline)) {
        if (j < GREG) {
#pragma unroll
            for (int q = 0; q < 8; q++) dst[q] = greg[j < GREG ? j : 0][q];
        } else if (j < GREG + GLDS) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const GPair v = glds[((j - GREG) * 4 + q) * RMPC_WAVE];
                dst[2 * q] = v.x; dst[2 * q + 1] = v.y;
            }
        } else if constexpr (RMPC_GAIN_NOMEM && GREG > 0) {   // (diagnostics: no tile traffic)
#pragma unroll
            for (int q = 0; q < 8; q++) dst[q] = greg[0][q];
        } else if constexpr (PR == 2) gt.ld_pair(j, dst, pp);
        else gt.ld(j, dst);
    };
    while (fin && it < maxit) {
        it++;
        // Keep the per-step inputs opaque to the optimiser at every iteration: otherwise it
        // hoists everything derived from them (hinge normals of every row, linearisation
        // terms, box bounds) out of this loop and the live set no longer fits in VGPRs.
#pragma unroll
        for (int k = 0; k < N; k++) {
            asm volatile("" : "+v"(S[k]), "+v"(Cs[k]), "+v"(V0[k]));
        }
        // (NO > 0) nor the LDS-resident row inputs: a memory clobber per iteration keeps their
        // loads, and so every row's geometry, inside the loop
        if constexpr (NO > 0) asm volatile("" ::: "memory");
        // ---------------- backward block Riccati sweep
        if (a.prof) tp0 = __builtin_amdgcn_s_memtime();
        RicV<T> V;
        V.P00 = P0; V.P01 = 0; V.P02 = 0; V.P11 = P1; V.P12 = 0; V.P22 = P2;
        V.p0 = -P0 * (T)0; V.p1 = -P1 * (T)0; V.p2 = -P2 * (T)0;
#ifndef RMPC_BPF
#define RMPC_BPF 1
#endif
        // UB, RMPC_BPF: obstacles in registers for the sweep, the step's reference position and
        // turn rate loaded one step ahead (no LDS wait inside a step)
        constexpr bool BPF = UB && BS == 1 && NOL <= 4 && RMPC_BPF;
        static_assert(PR == 1 || BPF, "paired lanes use the register-held obstacles");
        T bx[BPF ? NOL : 1], by[BPF ? NOL : 1], bsf[BPF ? NOL : 1];
        T pxb = 0, pyb = 0, v1b = 0;
        if constexpr (BPF) {
#pragma unroll
            for (int o = 0; o < NOL; o++) {
                bx[o] = obs_s[3 * (obase + o)]; by[o] = obs_s[3 * (obase + o) + 1]; bsf[o] = obs_s[3 * (obase + o) + 2];
            }
            pxb = PX(N - 1); pyb = PY(N - 1); v1b = V1(N - 1);
        }
#pragma unroll
        for (int j = NB - 1; j >= 0; j--) {
            const int k0 = j * BS;
            const int k1 = (k0 + BS < N) ? k0 + BS : N;
            T G[8];
            if constexpr (BS == 1) {
                // single-step block: the fused step (rmpc_riccati.h ric_step1_bf)
                const int k = j;
                T q00 = Q0, q01 = 0, q11 = Q1;
                T qv0 = -Q0 * (T)0, qv1 = -Q1 * (T)0, qv2 = -Q2 * (T)0;
                T pxk = 0, pyk = 0, v1k;
                if constexpr (BPF) {
                    int anc = 0;       // per-step anchor: this step's prefetch after the previous step
                    asm volatile("" : "+v"(anc), "+v"(V.P00), "+v"(V.p0));
                    pxk = pxb; pyk = pyb; v1k = v1b;
                    if (k > 0) {
                        if (RMPC_BPF == 1) {    // (2: positions loaded in the rows' branch)
                            pxb = lds[(0 * N + k - 1) * LW + ll + anc];
                            pyb = lds[(1 * N + k - 1) * LW + ll + anc];
                        }
                        v1b = lds[(2 * N + k - 1) * LW + ll + anc];
                    }
                } else {
                    v1k = V1(k);
                }
                // paired lanes: this lane's rows accumulate from zero, then the pair adds up
                T r00 = 0, r01 = 0, r11 = 0, rv0 = 0, rv1 = 0;
                T &a00 = PR == 2 ? r00 : q00, &a01 = PR == 2 ? r01 : q01, &a11 = PR == 2 ? r11 : q11;
                T &av0 = PR == 2 ? rv0 : qv0, &av1 = PR == 2 ? rv1 : qv1;
                if (BPF && k > 0 && Hf.get(k)) {
                    if (RMPC_BPF == 2) { pxk = PX(k); pyk = PY(k); }
#pragma unroll
                    for (int o = 0; o < NOL; o++) {
                        if (__builtin_amdgcn_ballot_w64(((Hf.get(k) >> o) & 1u) != 0u)) {
                            T n0, n1, hb;
                            hinge_row_fast(pxk, pyk, bx[BPF ? o : 0], by[BPF ? o : 0], bsf[BPF ? o : 0], n0, n1, hb);
                            const T w = ((Hf.get(k) >> o) & 1u) ? rho : (T)0;
                            a00 += w * n0 * n0;
                            a01 += w * n0 * n1;
                            a11 += w * n1 * n1;
                            av0 -= w * hb * n0;
                            av1 -= w * hb * n1;
                        }
                    }
                } else if (!BPF && k > 0 && Hf.get(k)) {
                    const T px = opq<NO>(PX(k)), py = opq<NO>(PY(k));
                    T cx = opq<NO>(obs_s[0]), cy = opq<NO>(obs_s[1]), cs = opq<NO>(obs_s[2]);
                    _Pragma("unroll UNRB") for (int o = 0; o < nob; o++) {      // branch-free: inactive rows add 0
                        // obstacle o+1 loads while row o computes (LDS latency off the row chain)
                        const T nx = opq<NO>(obs_s[3 * o + 3]), ny = opq<NO>(obs_s[3 * o + 4]), ns = opq<NO>(obs_s[3 * o + 5]);
                        // fp64: skip a row no lane of the wave has active (wave-uniform branch)
                        if (!F64 || __builtin_amdgcn_ballot_w64(((Hf.get(k) >> o) & 1u) != 0u)) {
                            T n0, n1, hb;
                            hinge_row_fast(px, py, cx, cy, cs, n0, n1, hb);
                            const T w = ((Hf.get(k) >> o) & 1u) ? rho : (T)0;
                            q00 += w * n0 * n0;
                            q01 += w * n0 * n1;
                            q11 += w * n1 * n1;
                            qv0 -= w * hb * n0;
                            qv1 -= w * hb * n1;
                        }
                        cx = nx; cy = ny; cs = ns;
                    }
                }
                if constexpr (PR == 2) {
                    q00 += r00 + pair_xchg(r00); q01 += r01 + pair_xchg(r01); q11 += r11 + pair_xchg(r11);
                    qv0 += rv0 + pair_xchg(rv0); qv1 += rv1 + pair_xchg(rv1);
                }
                T a0, a1, b0, b1, lo0, hi0, lo1, hi1, us0, us1;
                if constexpr (LTI) {
                    a0 = la0; a1 = la1; b0 = lb0; b1 = lb1;
                    lo0 = -vmax; hi0 = vmax; lo1 = -omax; hi1 = omax;           // :230-234
                    us0 = 0; us1 = 0;
                    // affine term of the error dynamics: V(Ae + Bu + c) = V'(Ae + Bu), p' = p + P c
                    const T c0 = S[k], c1 = Cs[k], c2 = V0[k];
                    const T p0n = V.p0 + V.P00 * c0 + V.P01 * c1 + V.P02 * c2;
                    const T p1n = V.p1 + V.P01 * c0 + V.P11 * c1 + V.P12 * c2;
                    const T p2n = V.p2 + V.P02 * c0 + V.P12 * c1 + V.P22 * c2;
                    V.p0 = p0n; V.p1 = p1n; V.p2 = p2n;
                } else {
                    const T vr = fabs(V0[k]) > (T)0.01 ? V0[k] : (T)0.1;     // :425
                    a0 = -vr * S[k] * dt; a1 = vr * Cs[k] * dt;
                    b0 = Cs[k] * dt; b1 = S[k] * dt;
                    lo0 = -vmax - V0[k]; hi0 = vmax - V0[k];                 // :431-436
                    lo1 = -omax - v1k; hi1 = omax - v1k;
                    us0 = V0[k]; us1 = v1k;
                }
                const uint32_t bfj = Bf.get(j);
                const int bf0 = bfj & 3, bf1 = (bfj >> 2) & 3;
                V = ric_step1_bf(V, a0, a1, b0, b1, dt, q00, q01, q11, Q2, qv0, qv1, qv2, R0, R1,
                                 R0 * us0, R1 * us1, bf0, bf1, bf0 == 1 ? lo0 : hi0, bf1 == 1 ? lo1 : hi1, G);
            } else {
                RicW<T> W = ric_open(V);
                T lo0 = -BIG, hi0 = BIG, lo1 = -BIG, hi1 = BIG;
#pragma unroll
                for (int k = k1 - 1; k >= k0; k--) {
                    T q00 = Q0, q01 = 0, q11 = Q1;
                    T qv0 = -Q0 * (T)0, qv1 = -Q1 * (T)0, qv2 = -Q2 * (T)0;
                    if (k > 0 && Hf.get(k)) {
                        const T px = opq<NO>(PX(k)), py = opq<NO>(PY(k));
                        T cx = opq<NO>(obs_s[0]), cy = opq<NO>(obs_s[1]), cs = opq<NO>(obs_s[2]);
                        _Pragma("unroll UNRB") for (int o = 0; o < nob; o++) {      // branch-free: inactive rows add 0
                            const T nx = opq<NO>(obs_s[3 * o + 3]), ny = opq<NO>(obs_s[3 * o + 4]), ns = opq<NO>(obs_s[3 * o + 5]);
                            T n0, n1, hb;
                            hinge_row_fast(px, py, cx, cy, cs, n0, n1, hb);
                            cx = nx; cy = ny; cs = ns;
                            const T w = ((Hf.get(k) >> o) & 1u) ? rho : (T)0;
                            q00 += w * n0 * n0;
                            q01 += w * n0 * n1;
                            q11 += w * n1 * n1;
                            qv0 -= w * hb * n0;
                            qv1 -= w * hb * n1;
                        }
                    }
                    const T vr = fabs(V0[k]) > (T)0.01 ? V0[k] : (T)0.1;     // :425
                    const T a0 = -vr * S[k] * dt, a1 = vr * Cs[k] * dt;
                    const T b0 = Cs[k] * dt, b1 = S[k] * dt;
                    ric_step(W, a0, a1, b0, b1, dt, q00, q01, q11, Q2, qv0, qv1, qv2, R0, R1,
                             R0 * V0[k], R1 * V1(k));
                    __builtin_amdgcn_sched_barrier(0);   // keep live ranges per step (see header)
                }
#pragma unroll
                for (int k = k0; k < k1; k++) {                            // :431-436 per block
                    lo0 = fmax(lo0, -vmax - V0[k]);
                    hi0 = fmin(hi0, vmax - V0[k]);
                    lo1 = fmax(lo1, -omax - V1(k));
                    hi1 = fmin(hi1, omax - V1(k));
                }
                const uint32_t bfj = Bf.get(j);
                const int bf0 = bfj & 3, bf1 = (bfj >> 2) & 3;
                V = ric_block_bf(W, bf0, bf1, bf0 == 1 ? lo0 : hi0, bf1 == 1 ? lo1 : hi1, G);
            }
            if (j < GREG) {
#pragma unroll
                for (int q = 0; q < 8; q++) greg[j < GREG ? j : 0][q] = G[q];
            } else if (j < GREG + GLDS) {
#pragma unroll
                for (int q = 0; q < 4; q++) glds[((j - GREG) * 4 + q) * RMPC_WAVE] = GPair{G[2 * q], G[2 * q + 1]};
            } else if constexpr (RMPC_GAIN_NOMEM && GREG > 0) {
#pragma unroll
                for (int q = 0; q < 8; q++) asm volatile("" ::"v"(G[q]));
            } else if constexpr (PR == 2) {
                gt.st_half(j, G, pp);
            } else gt.st(j, G);
#ifndef RMPC_BSB
#define RMPC_BSB 0
#endif
            if constexpr (!BPF || RMPC_BSB) __builtin_amdgcn_sched_barrier(0);   // (A/B: 0 lets BPF steps overlap)
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
        if constexpr (NO > 0) asm volatile("" ::: "memory");   // ... and the backward's row loads
        const T eps_h = SetTol<T>::hinge, eps_b = SetTol<T>::box;
        int changed = 0;
        used = 0;
        J = 0;
        T x0 = d0, x1 = d1, x2 = d2;
        T g[NB][8];
#pragma unroll
        for (int j = 0; j < NB && j < PF; j++) {
            gload(j, g[j]);
        }
#ifndef RMPC_FPF
#define RMPC_FPF 1
#endif
        // UF, RMPC_FPF: the obstacles held in registers for the sweep and each step's reference
        // position loaded one step ahead, so no LDS latency sits on a step's row chains
        constexpr bool FPF = UF && BS == 1 && NOL <= 4 && RMPC_FPF;
        static_assert(PR == 1 || FPF, "paired lanes use the register-held obstacles");
        T obx[FPF ? NOL : 1], oby[FPF ? NOL : 1], obsf[FPF ? NOL : 1];
        T pxn = 0, pyn = 0, v1n = 0;
        T Jr = 0;                          // paired lanes: this lane's rows' share of the objective
        if constexpr (FPF) {
#pragma unroll
            for (int o = 0; o < NOL; o++) {
                obx[o] = obs_s[3 * (obase + o)]; oby[o] = obs_s[3 * (obase + o) + 1]; obsf[o] = obs_s[3 * (obase + o) + 2];
            }
            pxn = PX(0); pyn = PY(0); v1n = V1(0);
        }
#pragma unroll
        for (int j = 0; j < NB; j++) {
            if (j + PF < NB) {
                gload(j + PF, g[j + PF]);
            }
            if constexpr (UF && BS == 1) {
                // Compile-time rows, block size 1: the step with wave-mask (SGPR) set logic.
                // The box state is two bits per component (at lower, at upper); the rows' set
                // rule and the change/slack tests are boolean, so they compile to scalar mask
                // operations; and the residual comes from the row's geometry directly,
                // r = safe - (d^2 + dp.(p - o)) / dist (= hb - n.dp of hinge_row_fast).
                const int k = j;
                int anc = 0;       // per-step anchor (see the runtime-row path below)
#ifndef RMPC_FANC
#define RMPC_FANC 0
#endif
                if constexpr (RMPC_FANC == 1)   // (A/B: the state chain only)
                    asm volatile("" : "+v"(anc), "+v"(x0), "+v"(x1), "+v"(x2));
                else
                    asm volatile("" : "+v"(anc), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(J), "+v"(changed),
                                 "+v"(used), "+v"(Hf.w[k >> 1]), "+v"(Bf.w[j >> 3]));
                const T v1k = FPF ? v1n : V1(k);     // reference turn rate (LTV; LTI: heading, unused here)
                if constexpr (FPF) {
                    if (k + 1 < N) v1n = lds[(2 * N + k + 1) * LW + ll + anc];
                }
                T lo0, hi0, lo1, hi1;
                if constexpr (LTI) {
                    lo0 = -vmax; hi0 = vmax; lo1 = -omax; hi1 = omax;
                } else {
                    lo0 = -vmax - V0[k]; hi0 = vmax - V0[k];
                    lo1 = -omax - v1k; hi1 = omax - v1k;
                }
                const T e0 = g[j][0] * x0 + g[j][1] * x1 + g[j][2] * x2 + g[j][6];
                const T e1 = g[j][3] * x0 + g[j][4] * x1 + g[j][5] * x2 + g[j][7];
                const uint32_t bfj = Bf.get(j);
                const bool L0 = bfj & 1u, H0 = bfj & 2u, L1 = bfj & 4u, H1 = bfj & 8u;
                const T u0v = L0 ? lo0 : (H0 ? hi0 : e0);
                const T u1v = L1 ? lo1 : (H1 ? hi1 : e1);
                // box_rule_bf: free -> lower/upper when e leaves [lo, hi] by eps_b; a fixed
                // component stays while its multiplier map keeps its sign
                // (non-short-circuit & and |: no branches, only mask operations)
                const bool F0 = !(L0 | H0), F1 = !(L1 | H1);
                const bool nL0 = (L0 & !(e0 < (T)0)) | (F0 & (e0 < lo0 - eps_b));
                const bool nH0 = (H0 & !(e0 > (T)0)) | (F0 & (e0 > hi0 + eps_b));
                const bool nL1 = (L1 & !(e1 < (T)0)) | (F1 & (e1 < lo1 - eps_b));
                const bool nH1 = (H1 & !(e1 > (T)0)) | (F1 & (e1 > hi1 + eps_b));
                bool chg = (nL0 != L0) | (nH0 != H0) | (nL1 != L1) | (nH1 != H1);
                Bf.set(j, (nL0 ? 1u : 0u) | (nH0 ? 2u : 0u) | (nL1 ? 4u : 0u) | (nH1 ? 8u : 0u));
                J += Q0 * x0 * x0 + Q1 * x1 * x1 + Q2 * x2 * x2;
                const T uu0 = LTI ? u0v : u0v + V0[k], uu1 = LTI ? u1v : u1v + v1k;
                J += R0 * uu0 * uu0 + R1 * uu1 * uu1;
                const uint32_t hk = Hf.get(k);
                T px, py;
                if constexpr (FPF) {
                    px = pxn; py = pyn;
                    if (k + 1 < N) {
                        pxn = lds[(0 * N + k + 1) * LW + ll + anc];
                        pyn = lds[(1 * N + k + 1) * LW + ll + anc];
                    }
                } else {
                    px = lds[(0 * N + k) * LW + ll + anc];
                    py = lds[(1 * N + k) * LW + ll + anc];
                }
                const T *const ob = obs_s + anc;
                bool usd = false;
                uint32_t flips = 0;
#pragma unroll
                for (int o = 0; o < NOL; o++) {
                    const T ox = FPF ? obx[FPF ? o : 0] : ob[3 * o], oy = FPF ? oby[FPF ? o : 0] : ob[3 * o + 1];
                    const T sf = FPF ? obsf[FPF ? o : 0] : ob[3 * o + 2];
                    const T ddx = px - ox, ddy = py - oy;
                    const T dd = ddx * ddx + ddy * ddy;
                    T y = rsq_approx(dd);
                    if constexpr (F64) {       // one Newton step, as hinge_row_fast (fp32: rsq as is)
                        const T hh = (T)0.5 * dd * y;
                        y = fma(y, fma(-hh, y, (T)0.5), y);
                    }
                    const bool kept = dd * y > (T)0.01;                   // dist > 0.01 (:446)
                    const T t = fma(ddy, x1, fma(ddx, x0, dd));
                    const T r = kept ? fma(-t, y, sf) : (T)-1;                // unkept: never active
                    const T rp = fmax(r, (T)0);
                    if constexpr (PR == 2) Jr += rho * rp * rp;
                    else J += rho * rp * rp;
                    usd = usd | (r > (T)1e-6);                               // :485
                    if (k > 0) {
                        const bool act = (hk >> o) & 1u;
                        const bool na = (r > eps_h) | (act & (r > -eps_h));
                        const bool flip = na != act;
                        chg = chg | flip;
                        flips |= flip ? (1u << o) : 0u;
                    }
                }
                Hf.set(k, hk ^ flips);
                changed |= (int)chg;
                used |= (int)usd;
                if constexpr (LTI) {
                    const T n0 = x0 + la0 * x2 + lb0 * u0v + S[k];
                    const T n1 = x1 + la1 * x2 + lb1 * u0v + Cs[k];
                    const T n2 = x2 + dt * u1v + V0[k];
                    x0 = n0; x1 = n1; x2 = n2;
                } else {
                    const T vr = fabs(V0[k]) > (T)0.01 ? V0[k] : (T)0.1;
                    const T n0 = x0 + (-vr * S[k] * dt) * x2 + (Cs[k] * dt) * u0v;
                    const T n1 = x1 + (vr * Cs[k] * dt) * x2 + (S[k] * dt) * u0v;
                    const T n2 = x2 + dt * u1v;
                    x0 = n0; x1 = n1; x2 = n2;
                }
#ifndef RMPC_FSB
#define RMPC_FSB 0
#endif
                if constexpr (RMPC_FSB) __builtin_amdgcn_sched_barrier(0);   // (0, default: steps may overlap; cfg4 -3%)
                continue;
            }
            const int k0 = j * BS;
            const int k1 = (k0 + BS < N) ? k0 + BS : N;
            T lo0 = -BIG, hi0 = BIG, lo1 = -BIG, hi1 = BIG;
            if constexpr (LTI) {
                lo0 = -vmax; hi0 = vmax; lo1 = -omax; hi1 = omax;
            } else if constexpr (BS == 1) {
                lo0 = -vmax - V0[k0]; hi0 = vmax - V0[k0];
                lo1 = -omax - V1(k0); hi1 = omax - V1(k0);
            } else {
#pragma unroll
                for (int k = k0; k < k1; k++) {
                    lo0 = fmax(lo0, -vmax - V0[k]);
                    hi0 = fmin(hi0, vmax - V0[k]);
                    lo1 = fmax(lo1, -omax - V1(k));
                    hi1 = fmin(hi1, omax - V1(k));
                }
            }
            const T e0 = g[j][0] * x0 + g[j][1] * x1 + g[j][2] * x2 + g[j][6];
            const T e1 = g[j][3] * x0 + g[j][4] * x1 + g[j][5] * x2 + g[j][7];
            const uint32_t bfj = Bf.get(j);
                const int bf0 = bfj & 3, bf1 = (bfj >> 2) & 3;
            const T u0v = bf0 == 0 ? e0 : (bf0 == 1 ? lo0 : hi0);
            const T u1v = bf1 == 0 ? e1 : (bf1 == 1 ? lo1 : hi1);
            const int ns0 = box_rule_bf(bf0, e0, lo0, hi0, eps_b), ns1 = box_rule_bf(bf1, e1, lo1, hi1, eps_b);
            changed |= (int)(ns0 != bf0 || ns1 != bf1);
            Bf.set(j, (uint32_t)(ns0 | (ns1 << 2)));
#pragma unroll
            for (int k = k0; k < k1; k++) {
                // Unrolled rows (UF): a per-step anchor orders this step after the previous one
                // (its state, objective and flags) and feeds an opaque zero into the row-input
                // addresses, so the step's LDS loads and row geometry cannot be hoisted into an
                // earlier step (the whole sweep would otherwise load first and spill).
                int anc = 0;
                if constexpr (UF)
                    asm volatile("" : "+v"(anc), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(J), "+v"(changed),
                                 "+v"(used), "+v"(Hf.w[k >> 1]));
                J += Q0 * x0 * x0 + Q1 * x1 * x1 + Q2 * x2 * x2;
                const T uu0 = LTI ? u0v : u0v + V0[k], uu1 = LTI ? u1v : u1v + V1(k);
                J += R0 * uu0 * uu0 + R1 * uu1 * uu1;
                uint32_t hk = Hf.get(k);
                const T px = lds[(0 * N + k) * LW + ll + anc], py = lds[(1 * N + k) * LW + ll + anc];
                const T *const ob = obs_s + anc;
                T cx = ob[0], cy = ob[1], cs = ob[2];
                _Pragma("unroll UNRF") for (int o = 0; o < nof; o++) {          // branch-free row update
                    const T nx = ob[3 * o + 3], ny = ob[3 * o + 4], ns = ob[3 * o + 5];
                    T n0, n1, hb;
                    const bool kept = hinge_row_fast(px, py, cx, cy, cs, n0, n1, hb);
                    cx = nx; cy = ny; cs = ns;
                    const T r = kept ? hb - n0 * x0 - n1 * x1 : (T)-1;   // unkept: never active
                    const T rp = fmax(r, (T)0);
                    J += rho * rp * rp;
                    used |= (r > (T)1e-6);                                     // :485
                    if (k > 0) {
                        const uint32_t act = (hk >> o) & 1u;
                        const uint32_t na = act ? (r > -eps_h) : (r > eps_h);
                        changed |= (int)(na != act);
                        hk ^= (na ^ act) << o;
                    }
                }
                Hf.set(k, hk);
                if constexpr (LTI) {
                    const T n0 = x0 + la0 * x2 + lb0 * u0v + S[k];
                    const T n1 = x1 + la1 * x2 + lb1 * u0v + Cs[k];
                    const T n2 = x2 + dt * u1v + V0[k];
                    x0 = n0; x1 = n1; x2 = n2;
                } else {
                    const T vr = fabs(V0[k]) > (T)0.01 ? V0[k] : (T)0.1;
                    const T n0 = x0 + (-vr * S[k] * dt) * x2 + (Cs[k] * dt) * u0v;
                    const T n1 = x1 + (vr * Cs[k] * dt) * x2 + (S[k] * dt) * u0v;
                    const T n2 = x2 + dt * u1v;
                    x0 = n0; x1 = n1; x2 = n2;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        J += P0 * x0 * x0 + P1 * x1 * x1 + P2 * x2 * x2;
        if constexpr (PR == 2) {           // the pair's rows: objective share, changes, slack
            J += Jr + pair_xchg(Jr);
            changed |= (int)pair_xchg((uint32_t)changed);
            used |= (int)pair_xchg((uint32_t)used);
        }
        if (a.prof) tp_f += __builtin_amdgcn_s_memtime() - tp0;
        if constexpr (RMPC_NOCERT) {
            asm volatile("" ::"v"(J), "v"(changed), "v"(used));
            continue;
        }
        if (!changed) { cert = 1; break; }
        // PDAS cycling: a repeated active-set signature hands the robot to the
        // projected-Newton phase of the next stage
        const uint64_t sig = set_sig();
        if (sig == hist0 || sig == hist1 || sig == hist2 || sig == hist3) { cycled = 1; break; }
        hist3 = hist2; hist2 = hist1; hist1 = hist0; hist0 = sig;
    }
    its_out = it - it_start;
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
            const unsigned long long tw = __builtin_amdgcn_s_memtime() - tp_setup;
            atomicAdd(a.prof + 19, tw);
            atomicAdd(a.prof + 20, 1ull);
            atomicAdd(a.prof + 22, tp_setup - t_entry);                 // setup cycles
            // slowest wave: total cycles (high bits) | its loop iterations | backward share (%)
            const unsigned long long pb = mb * 100ull / (tw ? tw : 1ull);
            atomicMax(a.prof + 21, (tw << 16) | (mi << 8) | (pb & 0xffull));
            atomicAdd(a.prof + 56 + (mi < 7ull ? mi : 7ull), 1ull);     // waves per loop count
        }
    }
    if constexpr (RMPC_NOCERT) return;
    // The output pass's loads are issued here, before the hand-off's record stores of this
    // wave's other lanes, for the same vmcnt reason (below); not in an fp32 pass that hands
    // every certified robot to the refinement pass (it writes no outputs)
    const bool may_write = !a.refine;
    const int sc = (!LTI && a.step_count && may_write) ? a.step_count[b] : 0;
    T x0 = d0, x1 = d1, x2 = d2;
    double uc0 = 0, uc1 = 0;
    // The gains are prefetched PFO blocks ahead (8: 98 AGPRs against 136 at 4 -- the allocation
    // of the whole kernel moves -- and one batch alone 185.4M -> 188.7M solves/s at config 3).  A block's loads are
    // issued before the previous steps' output stores, and vmcnt counts loads and stores in
    // issue order, so a load-use wait never waits for those stores: loading each block at its
    // own step made every step wait for all earlier stores to complete (round 3: ~106k cycles
    // per lane for this pass at config 3 under full-chip load).
#ifndef RMPC_PFO
#define RMPC_PFO 8
#endif
    constexpr int PFO = RMPC_PFO;
    // x_pred's reference rows (LTV: the heading as given, not unwrapped; fp32 also the
    // positions) loaded before the first output store, for the same reason
    double xth[(!LTI && F64) ? N + 1 : 1], xrt0 = 0, xrt1 = 0;
    if constexpr (!LTI && F64) {
        if (a.x_pred && may_write) {
#pragma unroll
            for (int k = 0; k <= N; k++) xth[k] = xr[3 * k + 2];
            xrt0 = xr[3 * N]; xrt1 = xr[3 * N + 1];
        }
    }
    T go[NB][8];
    if (may_write) {
#pragma unroll
        for (int j = 0; j < NB && j < PFO; j++) gload(j, go[j]);
    }
    const bool finJ = isfinite(J);
    // fp32 pass of a refined request: a certified robot goes on, with its sets, to the fp64
    // refinement pass (a.refine), which writes the outputs
    const bool to_refine = a.refine && cert && finJ;
    if (!cert || !finJ || to_refine) {
        if constexpr (PR == 2) {           // the pair's combined row flags (bit o = obstacle o)
#pragma unroll
            for (int i = 0; i < (N + 1) / 2; i++) {
                const uint32_t w = Hf.w[i], o = pair_xchg(w);
                Hf.w[i] = pp ? (o | (w << NOL)) : (w | (o << NOL));
            }
            if (pp) return;                // lane 2r hands the robot over
        }
        // the next stage takes over: one atomic per wave for the lanes here (exec mask), each
        // lane's slot from its rank among them (per-lane atomics on the one counter serialise:
        // a first pass hands on ~21k robots at once)
        auto hand_on = [&](int32_t *list, int32_t *count, uint32_t *sets, bool hist) __attribute__((always_inline)) {
            const uint64_t m = __builtin_amdgcn_read_exec();
            const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            int base = 0;
            if (rank == 0) base = atomicAdd(count, (int)__popcll(m));
            const int slot = __builtin_amdgcn_readfirstlane(base) + rank;
            list[slot] = (int32_t)b;
            if (sets) {                                       // ... from this active set
                // slot-minor record (word w at sets[w * B + slot]): a wave's consecutive
                // slots make each word one coalesced store
                uint32_t *ws = sets + slot;
#pragma unroll
                for (int k = 0; k < N; k++) ws[k * a.B] = Hf.get(k);
#pragma unroll
                for (int j = 0; j < NB; j++) ws[(N + j) * a.B] = Bf.get(j);
                ws[(N + NB) * a.B] = (uint32_t)it;
                if (hist) {                                   // (an earlier pass: + the cycle history)
                    uint32_t *h = ws + (size_t)(N + NB + 1) * a.B;
                    h[0] = (uint32_t)hist0; h[(size_t)a.B] = (uint32_t)(hist0 >> 32);
                    h[(size_t)2 * a.B] = (uint32_t)hist1; h[(size_t)3 * a.B] = (uint32_t)(hist1 >> 32);
                    h[(size_t)4 * a.B] = (uint32_t)hist2; h[(size_t)5 * a.B] = (uint32_t)(hist2 >> 32);
                    h[(size_t)6 * a.B] = (uint32_t)hist3; h[(size_t)7 * a.B] = (uint32_t)(hist3 >> 32);
                }
            }
        };
        if (to_refine) hand_on(a.refine, a.refine_count, a.refine_sets, false);
        else if (cycled && a.cyc) hand_on(a.cyc, a.cyc_count, a.cyc_sets, false);   // (earlier pass: to the tail)
        else hand_on(a.retry, a.retry_count, a.retry_sets, a.rec_hist != 0);
        if (a.prof) atomicMax(a.prof + 23, __builtin_amdgcn_s_memtime() - t_entry);   // longest lane, entry to exit
        return;
    }
#pragma unroll
    for (int k = 0; k < N; k++) asm volatile("" : "+v"(S[k]), "+v"(Cs[k]), "+v"(V0[k]));
    // ---- outputs (mpc_controller.py:484-520): x_pred = x_refs + dx (not unwrapped),
    // u = u_refs + du, omega ramp, step counter.  In fp32 the fp64 references are re-read so
    // that only the deviations carry fp32 rounding.
    // LTI: u = du (no u_ref), x_pred = e + x_ref (absolute), no ramp or step count.
    if constexpr (PR == 2) {               // warm start: the pair's combined row flags
        if (WS && a.prev_sets) {
#pragma unroll
            for (int i = 0; i < (N + 1) / 2; i++) {
                const uint32_t w = Hf.w[i], o = pair_xchg(w);
                Hf.w[i] = pp ? (o | (w << NOL)) : (w | (o << NOL));
            }
        }
    }
    if (PR == 2 && pp) return;             // paired lanes: lane 2r writes the outputs
    const unsigned long long t_out0 = a.prof ? __builtin_amdgcn_s_memtime() : 0ull;   // (diagnostics)
#pragma unroll
    for (int j = 0; j < NB; j++) {
        T du0, du1;
        const int k0 = j * BS;
        const int k1 = (k0 + BS < N) ? k0 + BS : N;
        if (j + PFO < NB) {
            gload(j + PFO, go[j + PFO]);
        }
        {   // the certified inputs, re-derived from the last backward sweep's gains along the
            // same trajectory (no per-iteration input tile)
            const T *const g = go[j];
            T lo0 = -BIG, hi0 = BIG, lo1 = -BIG, hi1 = BIG;
            if constexpr (LTI) {
                lo0 = -vmax; hi0 = vmax; lo1 = -omax; hi1 = omax;
            } else {
#pragma unroll
                for (int k = k0; k < k1; k++) {
                    lo0 = fmax(lo0, -vmax - V0[k]);
                    hi0 = fmin(hi0, vmax - V0[k]);
                    lo1 = fmax(lo1, -omax - V1(k));
                    hi1 = fmin(hi1, omax - V1(k));
                }
            }
            const T e0 = g[0] * x0 + g[1] * x1 + g[2] * x2 + g[6];
            const T e1 = g[3] * x0 + g[4] * x1 + g[5] * x2 + g[7];
            const uint32_t bfj = Bf.get(j);
                const int bf0 = bfj & 3, bf1 = (bfj >> 2) & 3;
            du0 = bf0 == 0 ? e0 : (bf0 == 1 ? lo0 : hi0);
            du1 = bf1 == 0 ? e1 : (bf1 == 1 ? lo1 : hi1);
        }
#pragma unroll
        for (int k = k0; k < k1; k++) {
            double v0 = LTI ? (double)du0 : F64 ? (double)(du0 + V0[k]) : (double)du0 + ur[2 * k];
            double v1 = LTI ? (double)du1 : F64 ? (double)(du1 + V1(k)) : (double)du1 + ur[2 * k + 1];
            if (k == 0) {
                if (!LTI && sc < p.ramp_up_steps) {                   // :502-505 (LTV only)
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
                if constexpr (LTI) {
                    xp[0] = (double)(x0 + PX(k)); xp[1] = (double)(x1 + PY(k)); xp[2] = (double)(x2 + V1(k));
                } else if constexpr (F64) {
                    xp[0] = (double)(x0 + PX(k));
                    xp[1] = (double)(x1 + PY(k));
                    xp[2] = (double)x2 + xth[k];
                } else {
                    xp[0] = (double)x0 + xr[3 * k];
                    xp[1] = (double)x1 + xr[3 * k + 1];
                    xp[2] = (double)x2 + xr[3 * k + 2];
                }
            }
            if constexpr (LTI) {
                const T n0 = x0 + la0 * x2 + lb0 * du0 + S[k];
                const T n1 = x1 + la1 * x2 + lb1 * du0 + Cs[k];
                const T n2 = x2 + dt * du1 + V0[k];
                x0 = n0; x1 = n1; x2 = n2;
            } else {
                const T vr = fabs(V0[k]) > (T)0.01 ? V0[k] : (T)0.1;
                const T n0 = x0 + (-vr * S[k] * dt) * x2 + (Cs[k] * dt) * du0;
                const T n1 = x1 + (vr * Cs[k] * dt) * x2 + (S[k] * dt) * du0;
                const T n2 = x2 + dt * du1;
                x0 = n0; x1 = n1; x2 = n2;
            }
        }
    }
    if (a.x_pred) {
        double *xp = a.x_pred + ((size_t)b * (N + 1) + N) * 3;
        if constexpr (LTI) {
            xp[0] = (double)x0 + xsN0; xp[1] = (double)x1 + xsN1; xp[2] = (double)x2 + xsN2;
        } else if constexpr (F64) {
            xp[0] = (double)x0 + xrt0;
            xp[1] = (double)x1 + xrt1;
            xp[2] = (double)x2 + xth[N];
        } else {
            xp[0] = (double)x0 + xr[3 * N];
            xp[1] = (double)x1 + xr[3 * N + 1];
            xp[2] = (double)x2 + xr[3 * N + 2];
        }
    }
    if (!LTI && a.step_count) a.step_count[b] = sc + 1;                // :507 (LTV only)
    a.u0[2 * b] = uc0;
    a.u0[2 * b + 1] = uc1;
    if (a.cost) a.cost[b] = (double)J;
    if (a.slack_used) a.slack_used[b] = (uint8_t)used;
    a.status[b] = RMPC_OPTIMAL;
    if (a.iters) a.iters[b] = it;
    if (WS && a.prev_sets) {               // warm start of this robot's next solve: its certified sets
        uint32_t *ws = a.prev_sets + b;
#pragma unroll
        for (int k = 0; k < N; k++) ws[(size_t)k * a.B] = Hf.get(k);
#pragma unroll
        for (int j = 0; j < NB; j++) ws[(size_t)(N + j) * a.B] = Bf.get(j);
        ws[(size_t)(N + NB) * a.B] = a.prev_stamp;
    }
    if (a.prof) {
        const unsigned long long t_end = __builtin_amdgcn_s_memtime();
        atomicMax(a.prof + 23, t_end - t_entry);
        atomicAdd(a.prof + 11, t_end - t_out0);         // output pass cycles (summed over lanes)
        atomicAdd(a.prof + 12, 1ull);
    }
}

}  // namespace rmpc

#undef PX
#undef PY
#undef V1
