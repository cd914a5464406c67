// rmpc_group_body.h -- the lane-group tail's solve (group_solve) and its helpers, included by
// the tail kernel (rmpc_mpc_group.hip: mpc_group_kernel).
#pragma once
#include "rmpc_device.h"
#include "rmpc_internal.h"
#include "rmpc_riccati.h"

// 1: the forward-sweep maps G of the BS = 1 backward sweep formed lane-parallel after it
// (ric_gmap1_bf) instead of on the sequential recursion; 0: inside the recursion
#ifndef RMPC_DIAG_NOSTORE
#define RMPC_DIAG_NOSTORE 0   // timing diagnostics only: the backward sweep stores nothing
#endif
#ifndef RMPC_TAIL_DEFER_G
#define RMPC_TAIL_DEFER_G 1
#endif

// 1: the BS = 1 backward Riccati sweep as a parallel-in-time associative scan over the group's
// lanes (default); 0: the sequential sweep, computed redundantly by every lane of the group
#ifndef RMPC_TAIL_PSCAN
#define RMPC_TAIL_PSCAN 1
#endif

// 1: rollouts and adjoints of given inputs by group scans (default); 0: sequential sweeps
#ifndef RMPC_GROUP_SCAN
#define RMPC_GROUP_SCAN 1
#endif

namespace rmpc {

struct GroupArgs {
    MpcDevParams prm;
    int no;
    const double *x0, *x_refs, *u_refs, *obs;
    int ref_rows, uref_rows;
    int32_t *step_count;
    double *u0, *u_seq, *x_pred, *cost;
    int32_t *status, *iters;
    uint8_t *slack_used;
    const int32_t *index, *count;     // robots to solve (device-side length)
    int32_t *retry, *retry_count;     // not certified / non-finite -> generic kernel
    const uint32_t *warm;             // per list entry: hinge flags [N], box states [NB], iters
    int pdas_cap;                     // PDAS solves before projected Newton
    unsigned long long *prof;         // optional per-phase cycle counters (diagnostics)
    unsigned long long *prof_waves;   // optional per-wave phase records (RMPC_DENSE_PROF=2)
    int64_t nB;                       // rows of the per-robot output arrays (bounds checks)
    int32_t *chk;                     // optional bounds-check record (RMPC_GROUP_CHECK, host-mapped)
    int32_t *site;                    // optional per-wave progress words (RMPC_GROUP_CHECK=2, host-mapped)
    uint32_t *prev_sets;              // warm start across calls (MpcFastArgs::prev_sets): per robot,
                                      // [N + NB + 1][nB]; a certified robot's sets are written back
    uint32_t prev_stamp;              // ... with this stamp
    int32_t *count_out;               // optional (host-mapped): the list's length, for the next
                                      // launch's grid (rmpc_launch_mpc_group)
};

// RMPC_GROUP_CHECK: an out-of-range index sets a flag bit and (first hit only) records the
// site, the offending value and the workgroup.  System-scope atomics on host-mapped memory:
// the record stays readable by the host after a faulting launch.
__device__ __forceinline__ void diag_hit(int32_t *chk, int bit, int site, long long v) {
    __hip_atomic_fetch_or(chk, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    int z = 0;
    if (__hip_atomic_compare_exchange_strong(chk + 1, &z, site, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM)) {
        __hip_atomic_store(chk + 2, (int)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(chk + 3, (int)blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// retry-list append with an optional bounds check
__device__ __forceinline__ void group_retry(const GroupArgs &a, int64_t b) {
    const int slot = atomicAdd(a.retry_count, 1);
    if (a.chk && (slot < 0 || slot >= a.nB)) { diag_hit(a.chk, 4, 3, slot); return; }
    a.retry[slot] = (int32_t)b;
}

// RMPC_GROUP_CHECK=2: the last site each wave reached (lane 0 of the wave; diagnostics)
#define GSITE(s)                                                                                   \
    do {                                                                                           \
        if (a.site && threadIdx.x == 0)                                                            \
            __hip_atomic_store(a.site + blockIdx.x, (s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
    } while (0)

// diagnostics: s_memtime deltas per phase (wave-uniform), flushed once per robot round
#define GPROF(slot)                                                                   \
    do {                                                                              \
        if (prof_on) {                                                                \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();               \
            pacc[slot] += t_ - tprof;                                                 \
            tprof = t_;                                                               \
        }                                                                             \
    } while (0)

// One robot's LDS record (elements of the arithmetic type T).  Every region but the hinge rows has a compile-time
// offset, so the optimiser can prove the recursions' stores (gains, trajectory) disjoint
// from their loads (step data) and issue the loads ahead; per-step and per-block data are
// packed 16-byte aligned records (ds_read_b128).
template <int N, int NB, typename T>
struct GRec {
    static constexpr int STEP = 0;                 // [N][12]: a0 a1 b0 b1 us0 us1 q00 q01 q11 qv0 qv1 -
    static constexpr int BLK = STEP + 12 * N;      // [NB][12]: lo0 hi0 lo1 hi1 G0..G7
    static constexpr int XS = BLK + 12 * NB;       // [N+1][4]: trajectory deviations (x, y, th, -)
    static constexpr int ZC = XS + 4 * (N + 1);    // candidate of the last solve [2NB]
    static constexpr int ZZ = ZC + 2 * NB;         // projected-Newton iterate
    static constexpr int ZT = ZZ + 2 * NB;         // line-search trial point
    static constexpr int GR = ZT + 2 * NB;         // gradient at ZZ
    static constexpr int FR = GR + 2 * NB;         // hinge forces per step [N][2]
    static constexpr int ZF = FR + 2 * N;          // certified inputs, kept for the final write [2NB]
    static constexpr int XF = ZF + 2 * NB;         // certified trajectory [N+1][3]
    static constexpr int XR = XF + 3 * (N + 1);    // LTI: reference states (absolute form) [N+1][3]
    static constexpr int INT = XR + 3 * (N + 1);   // uint32: HF [N], BF [NB], NHF [N], NBF [NB]
    static constexpr int INTN = ((2 * N + 2 * NB) * 4 + (int)sizeof(T) - 1) / (int)sizeof(T);
    static constexpr int HR = INT + (INTN + 1) / 2 * 2;     // hinge rows [3][no][N] (runtime no)
    __host__ __device__ static int size(int no) {
        const int o = HR + 3 * no * N;
        return o + (8 - o % 32 + 32) % 32;         // stride = 8 (mod 32) elements: the groups'
    }                                              // broadcast reads fall on different banks
};

template <int G>
__device__ __forceinline__ bool gany(bool v, int grp) {
    const uint64_t m = __ballot(v);
    if (G == 64) return m != 0;
    return ((m >> (grp * G)) & ((1ull << G) - 1)) != 0;
}

// DPP lane move within a row of 16 lanes (lanes whose source is outside the row read 0)
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)bits, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(bits >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
enum {
    DPP_QUAD_XOR1 = 0xB1, DPP_QUAD_XOR2 = 0x4E,          // quad_perm [1,0,3,2] / [2,3,0,1]
    DPP_ROW_SHL = 0x100, DPP_ROW_SHR = 0x110, DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141
};

// Group reductions.  For G = 16 (one DPP row): quad butterflies, then the half-row and row
// mirrors.  Every stage adds a lane's value to its partner's and the partner does the same
// addition the other way round, so all lanes end with bitwise-identical results (the
// recursions that follow rely on that).  Wider groups use shuffles.
template <int G, typename V>
__device__ __forceinline__ V gsum(V v) {
    if constexpr (G == 16) {
        v += dpp_mov<DPP_QUAD_XOR1>(v);
        v += dpp_mov<DPP_QUAD_XOR2>(v);
        v += dpp_mov<DPP_ROW_HALF_MIRROR>(v);
        v += dpp_mov<DPP_ROW_MIRROR>(v);
    } else {
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
    }
    return v;
}

template <int G, typename V>
__device__ __forceinline__ V gmaxv(V v) {
    if constexpr (G == 16) {
        v = fmax(v, dpp_mov<DPP_QUAD_XOR1>(v));
        v = fmax(v, dpp_mov<DPP_QUAD_XOR2>(v));
        v = fmax(v, dpp_mov<DPP_ROW_HALF_MIRROR>(v));
        v = fmax(v, dpp_mov<DPP_ROW_MIRROR>(v));
    } else {
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    }
    return v;
}

// The value of the lane OFF below in the group (0 for the group's first OFF lanes)
template <int G, int OFF, typename V>
__device__ __forceinline__ V gshr(V v, int gl) {
    if constexpr (G == 16) {
        return dpp_mov<DPP_ROW_SHR + OFF>(v);
    } else {
        const V t = __shfl_up(v, OFF, G);
        return gl >= OFF ? t : (V)0;
    }
}

// The value of the lane OFF above in the group (meaningless for the group's last OFF lanes)
template <int G, int OFF, typename V>
__device__ __forceinline__ V gshl(V v) {
    if constexpr (G == 16) return dpp_mov<DPP_ROW_SHL + OFF>(v);
    else return __shfl_down(v, OFF, G);
}

// One Hillis-Steele stage of an inclusive scan of affine maps x -> F x + f (3x3, lane
// order = step order): lanes at or above OFF compose their map after the one OFF below.
template <int G, int OFF, typename V>
__device__ __forceinline__ void affine_scan_stage(V F[9], V f[3], int gl) {
    V P[9], p[3];
#pragma unroll
    for (int i = 0; i < 9; i++) P[i] = gshr<G, OFF>(F[i], gl);
#pragma unroll
    for (int i = 0; i < 3; i++) p[i] = gshr<G, OFF>(f[i], gl);
    if (gl >= OFF) {
        V nF[9], nf[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
#pragma unroll
            for (int c = 0; c < 3; c++)
                nF[3 * r + c] = F[3 * r] * P[c] + F[3 * r + 1] * P[3 + c] + F[3 * r + 2] * P[6 + c];
            nf[r] = F[3 * r] * p[0] + F[3 * r + 1] * p[1] + F[3 * r + 2] * p[2] + f[r];
        }
#pragma unroll
        for (int i = 0; i < 9; i++) F[i] = nF[i];
#pragma unroll
        for (int i = 0; i < 3; i++) f[i] = nf[i];
    }
}

// Exclusive prefix sum over the group's lanes in lane order (FWD) or in reverse lane order
// (the sum over the lanes above).  G = 16 is one DPP row (Hillis-Steele with row shifts);
// wider groups go through shuffles.
template <int G, bool FWD, typename V>
__device__ __forceinline__ V gscan_excl(V v, int gl) {
    if constexpr (G == 16) {
        constexpr int S = FWD ? DPP_ROW_SHR : DPP_ROW_SHL;
        v += dpp_mov<S + 1>(v);
        v += dpp_mov<S + 2>(v);
        v += dpp_mov<S + 4>(v);
        v += dpp_mov<S + 8>(v);
        return dpp_mov<S + 1>(v);
    } else {
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            const V t = FWD ? __shfl_up(v, off, G) : __shfl_down(v, off, G);
            if (FWD ? gl >= off : gl + off < G) v += t;
        }
        const V t = FWD ? __shfl_up(v, 1, G) : __shfl_down(v, 1, G);
        return (FWD ? gl >= 1 : gl + 1 < G) ? t : (V)0;
    }
}

// ---- parallel-in-time Riccati (Sarkka & Garcia-Fernandez, "Temporal parallelization of
// dynamic programming and linear quadratic control", IEEE TAC 2023).  Element of steps i..j:
// the conditional value function of reaching x_j from x_i,
//   (A, b, C, e, J):  x_j = A x_i + b + C lambda,  cost x_i'J x_i - 2 e'x_i + ...
// For one step with stage x'Wx + 2w'x + u'Ru + 2r'u over the free inputs (fixed ones at v),
// dynamics x' = A x + B u:  A, b = B v - B_f R_f^-1 r_f, C = B_f R_f^-1 B_f', e = -w, J = W;
// the terminal element is (0, 0, 0, -p_N, P_N).  The suffix product e_k (x) ... (x) e_N has
// (J, e) = (P_k, -p_k), the value function V_k(x) = x'P_k x + 2 p_k'x of the sequential sweep
// (rmpc_riccati.h ric_step1_bf), equal up to rounding.  Symmetric 3x3 as 00 01 02 11 12 22.
// Flat element (27 values): A at 0, b at 9, C at 12, e at 18, J at 21 (plain arrays promote
// to registers where a struct of arrays filled from DPP moves did not)
enum { PE_A = 0, PE_B = 9, PE_C = 12, PE_E = 18, PE_J = 21, PE_N = 27 };
__device__ __forceinline__ constexpr int sx(int i, int j) {      // (not recursive: folds when unrolled)
    return i <= j ? (i == 0 ? j : (i == 1 ? 2 + j : 5)) : (j == 0 ? i : (j == 1 ? 2 + i : 5));
}
template <typename T>
__device__ __forceinline__ void inv3(const T M[9], T Mi[9]) {
    const T c00 = M[4] * M[8] - M[5] * M[7], c01 = M[5] * M[6] - M[3] * M[8], c02 = M[3] * M[7] - M[4] * M[6];
    const T det = M[0] * c00 + M[1] * c01 + M[2] * c02;
    T id = fast_rcp(det);
    id = id * ((T)2 - det * id);
    id = id * ((T)2 - det * id);
    Mi[0] = c00 * id; Mi[1] = (M[2] * M[7] - M[1] * M[8]) * id; Mi[2] = (M[1] * M[5] - M[2] * M[4]) * id;
    Mi[3] = c01 * id; Mi[4] = (M[0] * M[8] - M[2] * M[6]) * id; Mi[5] = (M[2] * M[3] - M[0] * M[5]) * id;
    Mi[6] = c02 * id; Mi[7] = (M[1] * M[6] - M[0] * M[7]) * id; Mi[8] = (M[0] * M[4] - M[1] * M[3]) * id;
}
// x (earlier steps) then y (later steps).  APPLY: y contains the terminal element (A = b = C = 0),
// so only (e, J) of the result are formed.
template <typename T, bool APPLY = false>
__device__ __forceinline__ void pcombine(const T *x, const T *y, T *z) {
    T M[9], Mi[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            M[3 * i + j] = (i == j ? (T)1 : (T)0) + x[PE_C + sx(i, 0)] * y[PE_J + sx(0, j)] + x[PE_C + sx(i, 1)] * y[PE_J + sx(1, j)] +
                           x[PE_C + sx(i, 2)] * y[PE_J + sx(2, j)];
    inv3(M, Mi);
    T T2[9];                                   // T2 = Ax' Mi'
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            T2[3 * i + j] = x[PE_A + i] * Mi[3 * j] + x[PE_A + 3 + i] * Mi[3 * j + 1] + x[PE_A + 6 + i] * Mi[3 * j + 2];
    T s[3];                                    // ey - Jy bx
#pragma unroll
    for (int i = 0; i < 3; i++)
        s[i] = y[PE_E + i] - (y[PE_J + sx(i, 0)] * x[PE_B + 0] + y[PE_J + sx(i, 1)] * x[PE_B + 1] + y[PE_J + sx(i, 2)] * x[PE_B + 2]);
#pragma unroll
    for (int i = 0; i < 3; i++) z[PE_E + i] = T2[3 * i] * s[0] + T2[3 * i + 1] * s[1] + T2[3 * i + 2] * s[2] + x[PE_E + i];
    T V[9];                                    // T2 Jy
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            V[3 * i + j] = T2[3 * i] * y[PE_J + sx(0, j)] + T2[3 * i + 1] * y[PE_J + sx(1, j)] + T2[3 * i + 2] * y[PE_J + sx(2, j)];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = i; j < 3; j++)
            z[PE_J + sx(i, j)] = V[3 * i] * x[PE_A + j] + V[3 * i + 1] * x[PE_A + 3 + j] + V[3 * i + 2] * x[PE_A + 6 + j] + x[PE_J + sx(i, j)];
    if constexpr (!APPLY) {
        T T1[9];                               // T1 = Ay Mi
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                T1[3 * i + j] = y[PE_A + 3 * i] * Mi[j] + y[PE_A + 3 * i + 1] * Mi[3 + j] + y[PE_A + 3 * i + 2] * Mi[6 + j];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                z[PE_A + 3 * i + j] = T1[3 * i] * x[PE_A + j] + T1[3 * i + 1] * x[PE_A + 3 + j] + T1[3 * i + 2] * x[PE_A + 6 + j];
        T t[3];                                // bx + Cx ey
#pragma unroll
        for (int i = 0; i < 3; i++)
            t[i] = x[PE_B + i] + x[PE_C + sx(i, 0)] * y[PE_E + 0] + x[PE_C + sx(i, 1)] * y[PE_E + 1] + x[PE_C + sx(i, 2)] * y[PE_E + 2];
#pragma unroll
        for (int i = 0; i < 3; i++) z[PE_B + i] = T1[3 * i] * t[0] + T1[3 * i + 1] * t[1] + T1[3 * i + 2] * t[2] + y[PE_B + i];
        T U[9];                                // T1 Cx
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                U[3 * i + j] = T1[3 * i] * x[PE_C + sx(0, j)] + T1[3 * i + 1] * x[PE_C + sx(1, j)] + T1[3 * i + 2] * x[PE_C + sx(2, j)];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = i; j < 3; j++)
                z[PE_C + sx(i, j)] = U[3 * i] * y[PE_A + 3 * j] + U[3 * i + 1] * y[PE_A + 3 * j + 1] + U[3 * i + 2] * y[PE_A + 3 * j + 2] +
                                y[PE_C + sx(i, j)];
    }
}


enum { PH_PDAS = 0, PH_PN = 1, PH_DONE = 2, PH_IDLE = 3 };

// Stores from inside the uniform recursions: all lanes of a group hold identical values, so
// all of them store (no branch, no address select: the sweep stays one basic block and
// the scheduler can issue the next steps' LDS loads ahead of these stores; the plain
// stores took 7% off the tail launch against the former lane-0-or-junk-slot select).
// Stores that only some groups may make (GSTM) select a private junk slot instead.
__shared__ double grp_junk[64];

// LTI: MPCController.solve (mpc_controller.py:150-314) -- absolute states tracking the
// (padded) references, ONE linearisation at the first reference, |u| box, rows on absolute
// positions; no unwrap, ramp or step count.  Otherwise solve_with_ltv (:345-522).
template <int N, int BS, int G, typename T, bool LTI>
__device__ __forceinline__ void group_solve(const GroupArgs &a, T *const base0,
                                            int t, bool have, int gl, int grp) {
    constexpr int NB = (N + BS - 1) / BS;
    constexpr int KPL = (N + G - 1) / G;          // steps per lane
    const MpcDevParams &p = a.prm;
    const int no = a.no;
    const T dt = p.dt, rho = p.rho;
    const T Q0 = p.Q[0], Q1 = p.Q[1], Q2 = p.Q[2], R0 = p.R[0], R1 = p.R[1];
    const T P0 = p.P[0], P1 = p.P[1], P2 = p.P[2];
    const T eps_h = SetTol<T>::hinge, eps_b = SetTol<T>::box;
    if (a.chk && have && (t < 0 || t >= a.nB)) { diag_hit(a.chk, 8, 2, t); have = false; }
    int64_t b = have ? (int64_t)a.index[t] : 0;
    if (a.chk && have && (b < 0 || b >= a.nB)) { diag_hit(a.chk, 1, 1, b); b = 0; have = false; }
    GSITE(1);
    const double *xr = a.x_refs + ref_row0(a.prm.ref_off, b, a.ref_rows) * 3;
    const double *ur = a.u_refs + ref_row0(a.prm.ref_off, b, a.uref_rows) * 2;
    const bool prof_on = a.prof != nullptr;
    unsigned long long tprof = prof_on ? __builtin_amdgcn_s_memtime() : 0ull;
    const unsigned long long tstart = tprof;
    unsigned long long pacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

    // LDS views, re-derived from an opaque offset before each use so that the optimiser
    // cannot hoist the (loop-invariant) per-step data out of the iteration loop
    T *base = base0;
    T *const junk = reinterpret_cast<T *>(grp_junk) + threadIdx.x;
// GST: every lane of the group stores its (bitwise identical) copy -- no address select;
// GSTM: masked per group through the junk slot (groups whose values are not meaningful)
#define GST(ref, v) ((ref) = (v))
#define GSTM(ref, v, m) (*((m) && gl == 0 ? &(ref) : junk) = (v))
    auto refresh = [&]() __attribute__((always_inline)) {
        int o = 0;
        asm volatile("" : "+v"(o));
        base = base0 + o;
    };
    using RC = GRec<N, NB, T>;
#define STG(f, k) base[RC::STEP + 12 * (k) + (f)]
#define WQ(k, f) base[RC::STEP + 12 * (k) + 6 + (f)]
#define BND(f, j) base[RC::BLK + 12 * (j) + (f)]
#define GN(j, f) base[RC::BLK + 12 * (j) + 4 + (f)]
#define HN0(o, k) base[RC::HR + (o) * N + (k)]
#define HN1(o, k) base[RC::HR + (no + (o)) * N + (k)]
#define HB(o, k) base[RC::HR + (2 * no + (o)) * N + (k)]
#define XS(k, d) base[RC::XS + 4 * (k) + (d)]
#define ZC(i) base[RC::ZC + (i)]
#define ZZ(i) base[RC::ZZ + (i)]
#define ZT(i) base[RC::ZT + (i)]
#define GR(i) base[RC::GR + (i)]
#define FR(c, k) base[RC::FR + 2 * (k) + (c)]
#define ZF(i) base[RC::ZF + (i)]
#define XF(k, d) base[RC::XF + 3 * (k) + (d)]
#define XR(k, d) base[RC::XR + 3 * (k) + (d)]
#define HF(k) reinterpret_cast<uint32_t *>(base + RC::INT)[(k)]
#define BF(j) reinterpret_cast<uint32_t *>(base + RC::INT)[N + (j)]
#define NHF(k) reinterpret_cast<uint32_t *>(base + RC::INT)[N + NB + (k)]
#define NBF(j) reinterpret_cast<uint32_t *>(base + RC::INT)[2 * N + NB + (j)]

    bool fin = true;
    T d0, d1, d2;
    if constexpr (LTI) {
        // ---- setup (mpc_controller.py:172-270): references padded with their last row,
        // linearisation at (u_ref[0,0] guarded, theta_ref[0]), |u| box
        const double v = ur[0];
        const double vr = fabs(v) > 0.01 ? v : 0.1;                        // :186
        double sn, cs;
        sincos(xr[2], &sn, &cs);
        for (int k = gl; k <= N; k += G) {
            const int kr = k < a.ref_rows ? k : a.ref_rows - 1;
            const double px = xr[3 * kr], py = xr[3 * kr + 1], th = xr[3 * kr + 2];
            XR(k, 0) = (T)px; XR(k, 1) = (T)py; XR(k, 2) = (T)th;
            fin = fin && isfinite(px + py + th);
            if (k < N) {
                STG(0, k) = -vr * sn * dt;
                STG(1, k) = vr * cs * dt;
                STG(2, k) = cs * dt;
                STG(3, k) = sn * dt;
                STG(4, k) = (T)0;
                STG(5, k) = (T)0;
                for (int o = 0; o < no; o++) {                              // :238-270
                    const double ox = a.obs[3 * o], oy = a.obs[3 * o + 1];
                    const double ddx = px - ox, ddy = py - oy;
                    const double dist = sqrt(ddx * ddx + ddy * ddy);
                    if (dist > 0.01) {
                        const double nx = ddx / dist, ny = ddy / dist;
                        HN0(o, k) = (T)nx;
                        HN1(o, k) = (T)ny;
                        HB(o, k) = (T)(p.d_safe + a.obs[3 * o + 2] + nx * ox + ny * oy);
                    } else {
                        HN0(o, k) = 0; HN1(o, k) = 0; HB(o, k) = (T)(sizeof(T) == 8 ? -1e300 : -1e30);
                    }
                }
            }
        }
        for (int j = gl; j < NB; j += G) {                                  // :230-234
            BND(0, j) = -p.v_max; BND(1, j) = p.v_max; BND(2, j) = -p.omega_max; BND(3, j) = p.omega_max;
        }
        fin = fin && isfinite(sn + cs + vr);
        const double *x0p = a.x0 + 3 * b;
        d0 = (T)x0p[0]; d1 = (T)x0p[1]; d2 = (T)x0p[2];
    } else {
        // ---- setup (mpc_controller.py:391-468): unwrap (sequential, every lane), then the
        // linearisation and the hinge rows of this lane's steps, the blocked box per block
        double thl[KPL];
        double corr = 0.0, prev = xr[2], th0 = 0.0;
#pragma unroll
        for (int k = 0; k < N; k++) {
            const double th = xr[3 * k + 2];
            if (k > 0) corr += unwrap_step(prev, th);
            prev = th;
            const double thu = th + corr;
            if (k == 0) th0 = thu;
            if (k % G == gl) thl[k / G] = thu;
        }
#pragma unroll
        for (int i = 0; i < KPL; i++) {
            const int k = gl + G * i;
            if (k < N) {
                double sn, cs;
                sincos(thl[i], &sn, &cs);
                const double v = ur[2 * k], w = ur[2 * k + 1];
                const double vr = fabs(v) > 0.01 ? v : 0.1;                    // :425
                STG(0, k) = -vr * sn * dt;
                STG(1, k) = vr * cs * dt;
                STG(2, k) = cs * dt;
                STG(3, k) = sn * dt;
                STG(4, k) = v;
                STG(5, k) = w;
                const T px = (T)xr[3 * k], py = (T)xr[3 * k + 1];
                fin = fin && isfinite(sn + cs + v + w + px + py);
                for (int o = 0; o < no; o++) {
                    T n0, n1, hb;
                    // (in T, from the same rounded inputs as the lane-per-robot kernel's rows)
                    if (!hinge_row_fast(px, py, (T)a.obs[3 * o], (T)a.obs[3 * o + 1], (T)(p.d_safe + a.obs[3 * o + 2]),
                                        n0, n1, hb)) {
                        n0 = 0; n1 = 0; hb = (T)(sizeof(T) == 8 ? -1e300 : -1e30);   // row not kept
                    }
                    HN0(o, k) = n0;
                    HN1(o, k) = n1;
                    HB(o, k) = hb;
                }
            }
        }
        for (int j = gl; j < NB; j += G) {                                      // :431-436
            double lo0 = -1e300, hi0 = 1e300, lo1 = -1e300, hi1 = 1e300;
            for (int k = j * BS; k < (j + 1) * BS && k < N; k++) {
                lo0 = fmax(lo0, -p.v_max - ur[2 * k]);
                hi0 = fmin(hi0, p.v_max - ur[2 * k]);
                lo1 = fmax(lo1, -p.omega_max - ur[2 * k + 1]);
                hi1 = fmin(hi1, p.omega_max - ur[2 * k + 1]);
            }
            BND(0, j) = lo0; BND(1, j) = hi0; BND(2, j) = lo1; BND(3, j) = hi1;
        }
        const double *x0p = a.x0 + 3 * b;
        const double x0a = th0 + wrap_pi(x0p[2] - th0);                        // :397-401
        d0 = (T)(x0p[0] - xr[0]); d1 = (T)(x0p[1] - xr[1]); d2 = (T)(x0a - th0);

    }
    fin = fin && isfinite(d0 + d1 + d2);
    int it0 = 0;                      // iterations of the previous stage (reported in iters)
    {
        // (retry records are slot-minor: word w of list entry t at warm[w * nB + t])
        const uint32_t *ws = (a.warm && have) ? a.warm + t : nullptr;
        const int64_t S = a.nB;
        for (int k = gl; k < N; k += G) HF(k) = (ws && k > 0) ? ws[k * S] : 0u;
        for (int j = gl; j < NB; j += G) BF(j) = ws ? ws[(N + j) * S] : 0u;
        if (ws) it0 = (int)ws[(N + NB) * S];
    }
    __syncthreads();

    GPROF(0);
    GSITE(2);
    int phase = have ? PH_PDAS : PH_IDLE;
    if (gany<G>(have && !fin, grp)) {                 // fallback law: the generic kernel owns it
        if (gl == 0) group_retry(a, b);
        phase = PH_IDLE;
    }

    // ---- building blocks (all groups run them; `m` masks the LDS writes of the groups
    // for which the result is meaningful)

    // trajectory under the inputs Z (ZC / ZZ / ZT) -> XS, full objective (constants included,
    // as the fast kernel's J), and whether any hinge residual exceeds 1e-6 (slack_used, :485)
    // full objective of the inputs at zoff along the trajectory in XS (lane-parallel)
    auto cost = [&](int zoff, int &used) __attribute__((always_inline)) -> T {
        refresh();
        T jl = 0.0;
        int u = 0;
        for (int k = gl; k <= N; k += G) {
            const T y0 = XS(k, 0), y1 = XS(k, 1), y2 = XS(k, 2);
            // tracking error: the state deviation (LTV) or state minus reference (LTI)
            const T e0 = LTI ? y0 - XR(k, 0) : y0, e1 = LTI ? y1 - XR(k, 1) : y1, e2 = LTI ? y2 - XR(k, 2) : y2;
            if (k == N) {
                jl += P0 * e0 * e0 + P1 * e1 * e1 + P2 * e2 * e2;
            } else {
                jl += Q0 * e0 * e0 + Q1 * e1 * e1 + Q2 * e2 * e2;
                const int j = k / BS;
                const T uu0 = base[zoff + 2 * j] + STG(4, k), uu1 = base[zoff + 2 * j + 1] + STG(5, k);
                jl += R0 * uu0 * uu0 + R1 * uu1 * uu1;
                for (int o = 0; o < no; o++) {
                    const T r = HB(o, k) - HN0(o, k) * y0 - HN1(o, k) * y1;
                    if (r > 0) jl += rho * r * r;
                    u |= (r > 1e-6);
                }
            }
        }
        used = gany<G>(u, grp);
        return gsum<G>(jl);
    };

#if RMPC_GROUP_SCAN
    // Trajectory under given inputs, in parallel over the horizon.  The model is triangular:
    // theta integrates dt*w, and x, y integrate a_k*theta_k + b_k*v_k.  So the rollout is two
    // group prefix sums over contiguous chunks of C steps per lane.  Each lane then walks its
    // chunk, stores its states (XS, lanes of groups with m set) and adds its steps' objective
    // terms, the same terms as cost().
    constexpr int CH = (N + G - 1) / G;      // steps per lane in the scan layouts
    auto rollout_cost = [&](const T (&w0)[CH], const T (&w1)[CH], bool m, int &used) __attribute__((always_inline)) -> T {
        constexpr int C = CH;
        const int k0 = gl * C;
        T s0[C], s1[C], s2[C], s3[C];
        T a2 = 0;
#pragma unroll
        for (int i = 0; i < C; i++) {
            const int k = k0 + i;
            const int kk = k < N ? k : 0;
            s0[i] = STG(0, kk); s1[i] = STG(1, kk); s2[i] = STG(2, kk); s3[i] = STG(3, kk);
            a2 += dt * w1[i];
        }
        T th = d2 + gscan_excl<G, true>(a2, gl);
        T thc[C], a0 = 0, a1 = 0;
#pragma unroll
        for (int i = 0; i < C; i++) {
            thc[i] = th;
            if (k0 + i < N) {
                a0 += s0[i] * th + s2[i] * w0[i];
                a1 += s1[i] * th + s3[i] * w0[i];
                th += dt * w1[i];
            }
        }
        T px = d0 + gscan_excl<G, true>(a0, gl), py = d1 + gscan_excl<G, true>(a1, gl);
        T *const jk = junk;
        T jl = 0;
        int u = 0;
#pragma unroll
        for (int i = 0; i < C; i++) {
            const int k = k0 + i;
            if (k < N) {
                *(m ? &XS(k, 0) : jk) = px;
                *(m ? &XS(k, 1) : jk) = py;
                *(m ? &XS(k, 2) : jk) = thc[i];
                const T e0 = LTI ? px - XR(k, 0) : px, e1 = LTI ? py - XR(k, 1) : py;
                const T e2 = LTI ? thc[i] - XR(k, 2) : thc[i];
                jl += Q0 * e0 * e0 + Q1 * e1 * e1 + Q2 * e2 * e2;
                const T uu0 = w0[i] + STG(4, k), uu1 = w1[i] + STG(5, k);
                jl += R0 * uu0 * uu0 + R1 * uu1 * uu1;
                for (int o = 0; o < no; o++) {
                    const T r = HB(o, k) - HN0(o, k) * px - HN1(o, k) * py;
                    if (r > 0) jl += rho * r * r;
                    u |= (r > 1e-6);
                }
                px += s0[i] * thc[i] + s2[i] * w0[i];
                py += s1[i] * thc[i] + s3[i] * w0[i];
            }
        }
        if (k0 < N && k0 + C >= N) {          // this lane's chunk ends at the horizon: x_N
            *(m ? &XS(N, 0) : jk) = px;
            *(m ? &XS(N, 1) : jk) = py;
            *(m ? &XS(N, 2) : jk) = th;
            const T e0 = LTI ? px - XR(N, 0) : px, e1 = LTI ? py - XR(N, 1) : py;
            const T e2 = LTI ? th - XR(N, 2) : th;
            jl += P0 * e0 * e0 + P1 * e1 * e1 + P2 * e2 * e2;
        }
        used = gany<G>(u, grp);
        return gsum<G>(jl);
    };
    auto objective = [&](int zoff, bool m, int &used) __attribute__((always_inline)) -> T {
        refresh();
        const int k0 = gl * CH;
        T w0[CH], w1[CH];
#pragma unroll
        for (int i = 0; i < CH; i++) {
            const int k = k0 + i;
            const bool in = k < N;
            const int kk = in ? k : 0;
            w0[i] = in ? base[zoff + 2 * (kk / BS)] : (T)0;
            w1[i] = in ? base[zoff + 2 * (kk / BS) + 1] : (T)0;
        }
        const T J = rollout_cost(w0, w1, m, used);
        __syncthreads();
        return J;
    };
    // One Armijo trial of the projected-Newton search (BS = 1), fused: each lane forms its
    // steps' trial inputs z_t = clamp(z + alpha (z_c - z)) and their gradient term, rolls
    // out and costs them, and -- when the group accepts -- writes them to ZZ itself.
    auto ls_trial = [&](T alpha, bool m, T Fc, bool &acc, T &gdo) __attribute__((always_inline)) -> T {
        refresh();
        const int k0 = gl * CH;
        T w0[CH], w1[CH], gd = 0;
#pragma unroll
        for (int i = 0; i < CH; i++) {
            const int k = k0 + i;
            w0[i] = 0; w1[i] = 0;
            if (k < N) {
                const T z0 = ZZ(2 * k), z1 = ZZ(2 * k + 1);
                w0[i] = clampv(z0 + alpha * (ZC(2 * k) - z0), BND(0, k), BND(1, k));
                w1[i] = clampv(z1 + alpha * (ZC(2 * k + 1) - z1), BND(2, k), BND(3, k));
                gd += GR(2 * k) * (w0[i] - z0) + GR(2 * k + 1) * (w1[i] - z1);
            }
        }
        int u;
        const T Ft = rollout_cost(w0, w1, m, u);
        gd = gsum<G>(gd);
        gdo = gd;
        acc = m && Ft <= Fc + (T)1e-4 * gd;
        if (acc) {
#pragma unroll
            for (int i = 0; i < CH; i++) {
                const int k = k0 + i;
                if (k < N) { ZZ(2 * k) = w0[i]; ZZ(2 * k + 1) = w1[i]; }
            }
        }
        __syncthreads();
        return Ft;
    };
#else
    auto objective = [&](int zoff, bool m, int &used) __attribute__((always_inline)) -> T {
        refresh();
        T x0 = d0, x1 = d1, x2 = d2;
        // per step: inputs of its block + linearisation, step k+1's loaded while k computes
        T nx[6];
        auto ldo = [&](int k) __attribute__((always_inline)) {
            nx[0] = base[zoff + 2 * (k / BS)];
            nx[1] = base[zoff + 2 * (k / BS) + 1];
#pragma unroll
            for (int f = 0; f < 4; f++) nx[2 + f] = STG(f, k);
        };
        ldo(0);
#pragma unroll
        for (int k = 0; k < N; k++) {
            T c[6];
#pragma unroll
            for (int f = 0; f < 6; f++) c[f] = nx[f];
            if (k + 1 < N) ldo(k + 1);
            __builtin_amdgcn_sched_barrier(0);
            GSTM(XS(k, 0), x0, m); GSTM(XS(k, 1), x1, m); GSTM(XS(k, 2), x2, m);
            const T n0 = x0 + c[2] * x2 + c[4] * c[0];
            const T n1 = x1 + c[3] * x2 + c[5] * c[0];
            const T n2 = x2 + dt * c[1];
            x0 = n0; x1 = n1; x2 = n2;
        }
        GSTM(XS(N, 0), x0, m); GSTM(XS(N, 1), x1, m); GSTM(XS(N, 2), x2, m);
        __syncthreads();
        return cost(zoff, used);
    };
#endif

    // PDAS hinge rule of step k's rows at position (y0, y1): the next flags from the current h
    auto hinge_rule = [&](int k, uint32_t h, T y0, T y1) __attribute__((always_inline)) -> uint32_t {
        uint32_t nh = h;
        if (k > 0) {
            for (int o = 0; o < no; o++) {
                const T r = HB(o, k) - HN0(o, k) * y0 - HN1(o, k) * y1;
                const uint32_t act = (h >> o) & 1u;
                const uint32_t na = act ? (r > -eps_h) : (r > eps_h);
                nh ^= (na ^ act) << o;
            }
        }
        return nh;
    };

#if RMPC_GROUP_SCAN
    // Forward sweep of solve_test in parallel over the horizon (BS = 1).  With the box states
    // fixed, step k is the affine map x -> M_k x + m_k: a free input follows its gain row, a
    // fixed one sits at its bound.  Each lane composes the maps of its chunk of C steps, a
    // group scan of the composites gives every chunk's start state, and each lane then walks
    // its chunk with the step formulas of the sequential sweep (inputs, box rule, trajectory)
    // and applies the hinge rule to its steps' rows.
    auto forward_scan = [&](bool &bchg, bool &hchg) __attribute__((always_inline)) {
        constexpr int C = (N + G - 1) / G;
        const int k0 = gl * C;
        T rc[C][16];
        uint32_t rb[C];
        T F[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, f[3] = {0, 0, 0};
#pragma unroll
        for (int i = 0; i < C; i++) {
            const int k = k0 + i;
            const int kk = k < N ? k : N - 1;
#pragma unroll
            for (int q = 0; q < 12; q++) rc[i][q] = base[RC::BLK + 12 * kk + q];
#pragma unroll
            for (int q = 0; q < 4; q++) rc[i][12 + q] = base[RC::STEP + 12 * kk + q];
            rb[i] = BF(kk);
            if (k < N) {
                T c[16];
#pragma unroll
                for (int q = 0; q < 16; q++) c[q] = rc[i][q];
                const int bf0 = rb[i] & 3, bf1 = (rb[i] >> 2) & 3;
                const bool fr0 = bf0 == 0, fr1 = bf1 == 0;
                const T g00 = fr0 ? c[4] : (T)0, g01 = fr0 ? c[5] : (T)0, g02 = fr0 ? c[6] : (T)0;
                const T g10 = fr1 ? c[7] : (T)0, g11 = fr1 ? c[8] : (T)0, g12 = fr1 ? c[9] : (T)0;
                const T kp0 = fr0 ? c[10] : (bf0 == 1 ? c[0] : c[1]);
                const T kp1 = fr1 ? c[11] : (bf1 == 1 ? c[2] : c[3]);
                const T sa0 = c[12], sa1 = c[13], sb0 = c[14], sb1 = c[15];
                const T M[9] = {(T)1 + sb0 * g00, sb0 * g01, sa0 + sb0 * g02,
                                sb1 * g00, (T)1 + sb1 * g01, sa1 + sb1 * g02,
                                dt * g10, dt * g11, (T)1 + dt * g12};
                const T m[3] = {sb0 * kp0, sb1 * kp0, dt * kp1};
                T nF[9], nf[3];
#pragma unroll
                for (int r = 0; r < 3; r++) {
#pragma unroll
                    for (int cc = 0; cc < 3; cc++)
                        nF[3 * r + cc] = M[3 * r] * F[cc] + M[3 * r + 1] * F[3 + cc] + M[3 * r + 2] * F[6 + cc];
                    nf[r] = M[3 * r] * f[0] + M[3 * r + 1] * f[1] + M[3 * r + 2] * f[2] + m[r];
                }
#pragma unroll
                for (int q = 0; q < 9; q++) F[q] = nF[q];
#pragma unroll
                for (int q = 0; q < 3; q++) f[q] = nf[q];
            }
        }
        affine_scan_stage<G, 1>(F, f, gl);
        affine_scan_stage<G, 2>(F, f, gl);
        affine_scan_stage<G, 4>(F, f, gl);
        affine_scan_stage<G, 8>(F, f, gl);
        if constexpr (G >= 32) affine_scan_stage<G, 16>(F, f, gl);
        if constexpr (G >= 64) affine_scan_stage<G, 32>(F, f, gl);
        // the state after this lane's chunk, one lane up: the chunk's start state
        const T y0 = F[0] * d0 + F[1] * d1 + F[2] * d2 + f[0];
        const T y1 = F[3] * d0 + F[4] * d1 + F[5] * d2 + f[1];
        const T y2 = F[6] * d0 + F[7] * d1 + F[8] * d2 + f[2];
        T x0 = gshr<G, 1>(y0, gl), x1 = gshr<G, 1>(y1, gl), x2 = gshr<G, 1>(y2, gl);
        if (gl == 0) { x0 = d0; x1 = d1; x2 = d2; }
#pragma unroll
        for (int i = 0; i < C; i++) {
            const int k = k0 + i;
            if (k < N) {
                T c[16];
#pragma unroll
                for (int q = 0; q < 16; q++) c[q] = rc[i][q];
                const T lo0 = c[0], hi0 = c[1], lo1 = c[2], hi1 = c[3];
                const T e0 = c[4] * x0 + c[5] * x1 + c[6] * x2 + c[10];
                const T e1 = c[7] * x0 + c[8] * x1 + c[9] * x2 + c[11];
                const int bf0 = rb[i] & 3, bf1 = (rb[i] >> 2) & 3;
                const T u0v = bf0 == 0 ? e0 : (bf0 == 1 ? lo0 : hi0);
                const T u1v = bf1 == 0 ? e1 : (bf1 == 1 ? lo1 : hi1);
                const int ns0 = box_rule_bf(bf0, e0, lo0, hi0, eps_b), ns1 = box_rule_bf(bf1, e1, lo1, hi1, eps_b);
                bchg = bchg || ns0 != bf0 || ns1 != bf1;
                NBF(k) = (uint32_t)(ns0 | (ns1 << 2));
                ZC(2 * k) = u0v;
                ZC(2 * k + 1) = u1v;
                XS(k, 0) = x0; XS(k, 1) = x1; XS(k, 2) = x2;
                const uint32_t h = HF(k), nh = hinge_rule(k, h, x0, x1);
                NHF(k) = nh;
                hchg = hchg || nh != h;
                const T n0 = x0 + c[12] * x2 + c[14] * u0v;
                const T n1 = x1 + c[13] * x2 + c[15] * u0v;
                const T n2 = x2 + dt * u1v;
                x0 = n0; x1 = n1; x2 = n2;
            }
        }
        if (k0 < N && k0 + C >= N) { XS(N, 0) = x0; XS(N, 1) = x1; XS(N, 2) = x2; }
    };
#endif

    // the quadratic piece of the current sets (HF, BF; fixed components at their bounds):
    // backward Riccati sweep -> GN; forward sweep -> candidate ZC, trajectory XS, next box
    // states NBF; row test -> next hinge flags NHF.  Returns "some set would change".
    auto solve_test = [&]() __attribute__((always_inline)) -> bool {
        refresh();
        // per-step stage weights from the active rows (lane-parallel over steps)
        for (int k = gl; k < N; k += G) {
            T q00 = Q0, q01 = 0.0, q11 = Q1;
            T qv0 = -Q0 * (LTI ? XR(k, 0) : (T)0), qv1 = -Q1 * (LTI ? XR(k, 1) : (T)0);
            const uint32_t h = HF(k);
            if (k > 0 && h) {
                for (int o = 0; o < no; o++) {
                    if (!((h >> o) & 1u)) continue;
                    const T n0 = HN0(o, k), n1 = HN1(o, k), hb = HB(o, k);
                    q00 += rho * n0 * n0;
                    q01 += rho * n0 * n1;
                    q11 += rho * n1 * n1;
                    qv0 -= rho * hb * n0;
                    qv1 -= rho * hb * n1;
                }
            }
            WQ(k, 0) = q00; WQ(k, 1) = q01; WQ(k, 2) = q11; WQ(k, 3) = qv0; WQ(k, 4) = qv1;
            if constexpr (LTI) WQ(k, 5) = -Q2 * XR(k, 2);
        }
        __syncthreads();
        GPROF(2);
        refresh();
        // backward block Riccati sweep (uniform within the group)
        RicV<T> V;
        V.P00 = P0; V.P01 = 0; V.P02 = 0; V.P11 = P1; V.P12 = 0; V.P22 = P2;
        if constexpr (LTI) {
            V.p0 = -P0 * XR(N, 0); V.p1 = -P1 * XR(N, 1); V.p2 = -P2 * XR(N, 2);
        } else {
            V.p0 = -P0 * 0.0; V.p1 = -P1 * 0.0; V.p2 = -P2 * 0.0;
        }
        if constexpr (BS == 1) {
          if constexpr (RMPC_TAIL_PSCAN && RMPC_TAIL_DEFER_G && !RMPC_DIAG_NOSTORE) {
            // parallel-in-time sweep: lane gl holds elements gl*CPL .. gl*CPL + CPL - 1 of the
            // N steps and the terminal (index N), folds them, and an inclusive suffix scan over
            // lanes 0..LT gives each lane the value function at its first step; the chunk's
            // other step combines its element with the next lane's result.  Each lane then forms
            // its steps' forward maps G from those value functions while they are in registers.
            constexpr int CPL = (N + 1 + G - 1) / G;
            static_assert(CPL <= 2, "scan layout: at most two elements per lane");
            constexpr int LT = N / CPL;                  // the lane holding the terminal element
            const T iR0 = (T)1 / R0, iR1 = (T)1 / R1;
            auto pelem = [&](int idx, T *E) __attribute__((always_inline)) {
                const int k = idx < N ? idx : N - 1;     // (loads stay in range; selected below)
                const bool st = idx < N, tm = idx == N;
                const T a0 = STG(0, k), a1 = STG(1, k), b0 = STG(2, k), b1 = STG(3, k);
                const T us0 = STG(4, k), us1 = STG(5, k);
                const T q00 = WQ(k, 0), q01 = WQ(k, 1), q11 = WQ(k, 2), qv0 = WQ(k, 3), qv1 = WQ(k, 4);
                const T qv2 = LTI ? WQ(k, 5) : (T)0;
                const uint32_t bfk = BF(k);
                const int bf0 = bfk & 3, bf1 = (bfk >> 2) & 3;
                const T uc0 = bf0 == 1 ? BND(0, k) : BND(1, k), uc1 = bf1 == 1 ? BND(2, k) : BND(3, k);
                const T s0 = bf0 == 0 ? -us0 : uc0, s1 = bf1 == 0 ? -us1 : uc1;   // b = B s
                const T g0 = bf0 == 0 ? iR0 : (T)0, g1 = bf1 == 0 ? iR1 : (T)0;  // C = B_f R_f^-1 B_f'
#pragma unroll
                for (int q = 0; q < 9; q++) E[PE_A + q] = (q % 4 == 0 && !tm) ? (T)1 : (T)0;
                E[PE_A + 2] = st ? a0 : (T)0;
                E[PE_A + 5] = st ? a1 : (T)0;
                E[PE_B + 0] = st ? b0 * s0 : (T)0; E[PE_B + 1] = st ? b1 * s0 : (T)0; E[PE_B + 2] = st ? dt * s1 : (T)0;
                E[PE_C + 0] = st ? g0 * b0 * b0 : (T)0; E[PE_C + 1] = st ? g0 * b0 * b1 : (T)0; E[PE_C + 2] = 0;
                E[PE_C + 3] = st ? g0 * b1 * b1 : (T)0; E[PE_C + 4] = 0; E[PE_C + 5] = st ? g1 * dt * dt : (T)0;
                T pe0 = 0, pe1 = 0, pe2 = 0;             // terminal: e = -p_N
                if constexpr (LTI) { pe0 = P0 * XR(N, 0); pe1 = P1 * XR(N, 1); pe2 = P2 * XR(N, 2); }
                E[PE_E + 0] = st ? -qv0 : (tm ? pe0 : (T)0);
                E[PE_E + 1] = st ? -qv1 : (tm ? pe1 : (T)0);
                E[PE_E + 2] = st ? -qv2 : (tm ? pe2 : (T)0);
                E[PE_J + 0] = st ? q00 : (tm ? P0 : (T)0); E[PE_J + 1] = st ? q01 : (T)0; E[PE_J + 2] = 0;
                E[PE_J + 3] = st ? q11 : (tm ? P1 : (T)0); E[PE_J + 4] = 0; E[PE_J + 5] = st ? Q2 : (tm ? P2 : (T)0);
            };
            T E[PE_N];
            pelem(gl * CPL + CPL - 1, E);
            if constexpr (CPL == 2) {
                T e0[PE_N], t[PE_N];
                pelem(gl * CPL, e0);
                pcombine<T>(e0, E, t);
                #pragma unroll
                for (int q = 0; q < PE_N; q++) E[q] = t[q];
            }
            auto stage = [&](auto off_c) __attribute__((always_inline)) {
                constexpr int OFF = decltype(off_c)::value;
                T y[PE_N], z[PE_N];
#pragma unroll
                for (int q = 0; q < PE_N; q++) y[q] = gshl<G, OFF>(E[q]);
                pcombine<T>(E, y, z);
                const bool on = gl + OFF <= LT;      // (select, not a branch: no aggregate phi)
#pragma unroll
                for (int q = 0; q < PE_N; q++) E[q] = on ? z[q] : E[q];
            };
            if constexpr (LT >= 1) stage(std::integral_constant<int, 1>{});
            if constexpr (LT >= 2) stage(std::integral_constant<int, 2>{});
            if constexpr (LT >= 4) stage(std::integral_constant<int, 4>{});
            if constexpr (LT >= 8) stage(std::integral_constant<int, 8>{});
            if constexpr (LT >= 16) stage(std::integral_constant<int, 16>{});
            if constexpr (LT >= 32) stage(std::integral_constant<int, 32>{});
            // step k's forward map G from V_{k+1} = (J, -e) of the suffix starting at k + 1, in
            // registers (no LDS round trip of V_k and no barrier; the same operations as the
            // G pass below, so the same bits)
            auto gmap = [&](int k, const T *v) __attribute__((always_inline)) {
                RicV<T> Vn;
                Vn.P00 = v[PE_J + 0]; Vn.P01 = v[PE_J + 1]; Vn.P02 = v[PE_J + 2];
                Vn.P11 = v[PE_J + 3]; Vn.P12 = v[PE_J + 4]; Vn.P22 = v[PE_J + 5];
                Vn.p0 = -v[PE_E + 0]; Vn.p1 = -v[PE_E + 1]; Vn.p2 = -v[PE_E + 2];
                const uint32_t bfk = BF(k);
                const int bf0 = bfk & 3, bf1 = (bfk >> 2) & 3;
                T Gk[8];
                ric_gmap1_bf(Vn, STG(0, k), STG(1, k), STG(2, k), STG(3, k), dt, R0, R1, R0 * STG(4, k),
                             R1 * STG(5, k), bf0, bf1, bf0 == 1 ? BND(0, k) : BND(1, k),
                             bf1 == 1 ? BND(2, k) : BND(3, k), Gk);
#pragma unroll
                for (int q = 0; q < 8; q++) GN(k, q) = Gk[q];
            };
            // the next lane's suffix: V at this lane's last step + 1 (terminal inside)
            T sn[PE_N];
#pragma unroll
            for (int q = 0; q < 3; q++) sn[PE_E + q] = gshl<G, 1>(E[PE_E + q]);
#pragma unroll
            for (int q = 0; q < 6; q++) sn[PE_J + q] = gshl<G, 1>(E[PE_J + q]);
            const int k0 = gl * CPL;
            if constexpr (CPL == 2) {
                // the chunk's second step: its element, then the next lane's suffix
                T e1[PE_N], v1[PE_N];
                const int k1 = k0 + 1;
                pelem(k1, e1);
                pcombine<T, true>(e1, sn, v1);
                if (k1 <= N - 1) gmap(k1, sn);
                if (k0 <= N - 1) gmap(k0, v1);
            } else {
                if (k0 <= N - 1) gmap(k0, sn);
            }
          } else {
            // single-step blocks, software-pipelined: step j-1's record is loaded while step j
            // computes (the scheduler does not hoist LDS loads across unrolled steps itself)
            T nx[16];
            uint32_t nbf = 0;
            auto ld = [&](int j) __attribute__((always_inline)) {
#pragma unroll
                for (int f = 0; f < 12; f++) nx[f] = base[RC::STEP + 12 * j + f];
#pragma unroll
                for (int f = 0; f < 4; f++) nx[12 + f] = base[RC::BLK + 12 * j + f];
                nbf = BF(j);
            };
            ld(NB - 1);
#pragma unroll
            for (int j = NB - 1; j >= 0; j--) {
                T c[16];
#pragma unroll
                for (int f = 0; f < 16; f++) c[f] = nx[f];
                const uint32_t bfj = nbf;
                if (j > 0) ld(j - 1);
                __builtin_amdgcn_sched_barrier(0);
                const int bf0 = bfj & 3, bf1 = (bfj >> 2) & 3;
                T Gv[8];
                V = ric_step1_bf<T, !RMPC_TAIL_DEFER_G>(V, c[0], c[1], c[2], c[3], dt, c[6], c[7], c[8], Q2, c[9],
                                                        c[10], LTI ? c[11] : -Q2 * (T)0, R0, R1, R0 * c[4], R1 * c[5],
                                                        bf0, bf1, bf0 == 1 ? c[12] : c[13], bf1 == 1 ? c[14] : c[15], Gv);
                if constexpr (RMPC_DIAG_NOSTORE) {                 // timing diagnostics only
                    asm volatile("" :: "v"(V.P00), "v"(V.P01), "v"(V.P02), "v"(V.P11), "v"(V.P12), "v"(V.P22),
                                 "v"(V.p0), "v"(V.p1), "v"(V.p2));
                } else if constexpr (RMPC_TAIL_DEFER_G) {
                    // V_j for the G pass: P over step j's (consumed) stage weights, p over G5..G7
                    GST(WQ(j, 0), V.P00); GST(WQ(j, 1), V.P01); GST(WQ(j, 2), V.P02);
                    GST(WQ(j, 3), V.P11); GST(WQ(j, 4), V.P12); GST(WQ(j, 5), V.P22);
                    GST(GN(j, 5), V.p0); GST(GN(j, 6), V.p1); GST(GN(j, 7), V.p2);
                } else {
#pragma unroll
                    for (int q = 0; q < 8; q++) GST(GN(j, q), Gv[q]);
                }
            }
          }
            if constexpr (RMPC_TAIL_DEFER_G && !(RMPC_TAIL_PSCAN && !RMPC_DIAG_NOSTORE)) {
                // G pass, lane-parallel over the steps: each step's forward map from the value
                // function of the step after it (the sweep above stored it), so the 32 flops of G
                // per step leave the sequential recursion
                __syncthreads();
                constexpr int KG = (NB + G - 1) / G;
                T Gl[KG][8];
#pragma unroll
                for (int i = 0; i < KG; i++) {
                    const int j = gl + G * i;
                    if (j < NB) {
                        RicV<T> Vn;
                        if (j == NB - 1) {                   // terminal value function
                            Vn.P00 = P0; Vn.P01 = 0; Vn.P02 = 0; Vn.P11 = P1; Vn.P12 = 0; Vn.P22 = P2;
                            if constexpr (LTI) {
                                Vn.p0 = -P0 * XR(N, 0); Vn.p1 = -P1 * XR(N, 1); Vn.p2 = -P2 * XR(N, 2);
                            } else {
                                Vn.p0 = -P0 * 0.0; Vn.p1 = -P1 * 0.0; Vn.p2 = -P2 * 0.0;
                            }
                        } else {
                            Vn.P00 = WQ(j + 1, 0); Vn.P01 = WQ(j + 1, 1); Vn.P02 = WQ(j + 1, 2);
                            Vn.P11 = WQ(j + 1, 3); Vn.P12 = WQ(j + 1, 4); Vn.P22 = WQ(j + 1, 5);
                            Vn.p0 = GN(j + 1, 5); Vn.p1 = GN(j + 1, 6); Vn.p2 = GN(j + 1, 7);
                        }
                        const uint32_t bfj = BF(j);
                        const int bf0 = bfj & 3, bf1 = (bfj >> 2) & 3;
                        ric_gmap1_bf(Vn, STG(0, j), STG(1, j), STG(2, j), STG(3, j), dt, R0, R1, R0 * STG(4, j),
                                     R1 * STG(5, j), bf0, bf1, bf0 == 1 ? BND(0, j) : BND(1, j),
                                     bf1 == 1 ? BND(2, j) : BND(3, j), Gl[i]);
                    }
                }
                __syncthreads();
#pragma unroll
                for (int i = 0; i < KG; i++) {
                    const int j = gl + G * i;
                    if (j < NB) {
#pragma unroll
                        for (int q = 0; q < 8; q++) GN(j, q) = Gl[i][q];
                    }
                }
            }
        } else {
#pragma unroll
            for (int j = NB - 1; j >= 0; j--) {
                const int k0 = j * BS, k1 = (k0 + BS < N) ? k0 + BS : N;
                const uint32_t bfj = BF(j);
                const int bf0 = bfj & 3, bf1 = (bfj >> 2) & 3;
                T Gv[8];
                RicW<T> W = ric_open(V);
#pragma unroll
                for (int k = k1 - 1; k >= k0; k--) {
                    ric_step(W, STG(0, k), STG(1, k), STG(2, k), STG(3, k), dt, WQ(k, 0), WQ(k, 1), WQ(k, 2), Q2,
                             WQ(k, 3), WQ(k, 4), LTI ? WQ(k, 5) : -Q2 * (T)0, R0, R1, R0 * STG(4, k), R1 * STG(5, k));
                }
                V = ric_block_bf(W, bf0, bf1, bf0 == 1 ? BND(0, j) : BND(1, j), bf1 == 1 ? BND(2, j) : BND(3, j), Gv);
#pragma unroll
                for (int q = 0; q < 8; q++) GST(GN(j, q), Gv[q]);
            }
        }
        __syncthreads();
        GPROF(3);
        refresh();
        // forward sweep: inputs (free: gains; fixed: bound), box rule on the value (free) or
        // the multiplier (fixed), trajectory
        bool bchg = false, hchg = false;
#if RMPC_GROUP_SCAN
        if constexpr (BS == 1) {
            forward_scan(bchg, hchg);
        } else
#endif
        {   // sequential sweep (block size > 1)
            T x0 = d0, x1 = d1, x2 = d2;
            // block record (bounds + gains) and step data of block j+1 loaded while j computes
            T nx[16];
            uint32_t nbf = 0;
            auto ldf = [&](int j) __attribute__((always_inline)) {
#pragma unroll
                for (int f = 0; f < 12; f++) nx[f] = base[RC::BLK + 12 * j + f];
#pragma unroll
                for (int f = 0; f < 4; f++) nx[12 + f] = BS == 1 ? base[RC::STEP + 12 * j + f] : (T)0;
                nbf = BF(j);
            };
            ldf(0);
#pragma unroll
            for (int j = 0; j < NB; j++) {
                T c[16];
#pragma unroll
                for (int f = 0; f < 16; f++) c[f] = nx[f];
                const uint32_t bfj = nbf;
                if (j + 1 < NB) ldf(j + 1);
                __builtin_amdgcn_sched_barrier(0);
                const T lo0 = c[0], hi0 = c[1], lo1 = c[2], hi1 = c[3];
                const T e0 = c[4] * x0 + c[5] * x1 + c[6] * x2 + c[10];
                const T e1 = c[7] * x0 + c[8] * x1 + c[9] * x2 + c[11];
                const int bf0 = bfj & 3, bf1 = (bfj >> 2) & 3;
                const T u0v = bf0 == 0 ? e0 : (bf0 == 1 ? lo0 : hi0);
                const T u1v = bf1 == 0 ? e1 : (bf1 == 1 ? lo1 : hi1);
                const int ns0 = box_rule_bf(bf0, e0, lo0, hi0, eps_b), ns1 = box_rule_bf(bf1, e1, lo1, hi1, eps_b);
                bchg = bchg || ns0 != bf0 || ns1 != bf1;
                NBF(j) = (uint32_t)(ns0 | (ns1 << 2));
                GST(ZC(2 * j), u0v);
                GST(ZC(2 * j + 1), u1v);
#pragma unroll
                for (int k = j * BS; k < (j + 1) * BS && k < N; k++) {
                    GST(XS(k, 0), x0); GST(XS(k, 1), x1); GST(XS(k, 2), x2);
                    const T sa0 = BS == 1 ? c[12] : STG(0, k), sa1 = BS == 1 ? c[13] : STG(1, k);
                    const T sb0 = BS == 1 ? c[14] : STG(2, k), sb1 = BS == 1 ? c[15] : STG(3, k);
                    const T n0 = x0 + sa0 * x2 + sb0 * u0v;
                    const T n1 = x1 + sa1 * x2 + sb1 * u0v;
                    const T n2 = x2 + dt * u1v;
                    x0 = n0; x1 = n1; x2 = n2;
                }
            }
            GST(XS(N, 0), x0); GST(XS(N, 1), x1); GST(XS(N, 2), x2);
            __syncthreads();
            GPROF(4);
            refresh();
            // hinge rule per row (lane-parallel over steps)
            for (int k = gl; k < N; k += G) {
                const uint32_t h = HF(k), nh = hinge_rule(k, h, XS(k, 0), XS(k, 1));
                NHF(k) = nh;
                hchg = hchg || nh != h;
            }
        }
        const bool chg = gany<G>(bchg || hchg, grp);
        __syncthreads();
        GPROF(5);
        return chg;
    };

    // gradient of the objective at ZZ (whose trajectory is in XS): hinge forces per step
    // (lane-parallel), then the adjoint recursion (uniform) -> GR
    auto gradient_seq = [&](bool m) __attribute__((always_inline)) {
        refresh();
        for (int k = gl; k < N; k += G) {
            T f0 = 0.0, f1 = 0.0;
            if (k > 0) {
                const T y0 = XS(k, 0), y1 = XS(k, 1);
                for (int o = 0; o < no; o++) {
                    const T r = HB(o, k) - HN0(o, k) * y0 - HN1(o, k) * y1;
                    if (r > 0) {
                        f0 -= 2 * rho * r * HN0(o, k);
                        f1 -= 2 * rho * r * HN1(o, k);
                    }
                }
            }
            if (m) { FR(0, k) = f0; FR(1, k) = f1; }
        }
        __syncthreads();
        refresh();
        T l0 = 2 * P0 * (LTI ? XS(N, 0) - XR(N, 0) : XS(N, 0));
        T l1 = 2 * P1 * (LTI ? XS(N, 1) - XR(N, 1) : XS(N, 1));
        T l2 = 2 * P2 * (LTI ? XS(N, 2) - XR(N, 2) : XS(N, 2));
#pragma unroll
        for (int j = NB - 1; j >= 0; j--) {
            T g0 = 0.0, g1 = 0.0;
            const T z0 = ZZ(2 * j), z1 = ZZ(2 * j + 1);
#pragma unroll
            for (int k = ((j + 1) * BS < N ? (j + 1) * BS : N) - 1; k >= j * BS; k--) {
                g0 += STG(2, k) * l0 + STG(3, k) * l1 + 2 * R0 * (z0 + STG(4, k));
                g1 += dt * l2 + 2 * R1 * (z1 + STG(5, k));
                const T m0 = 2 * Q0 * (LTI ? XS(k, 0) - XR(k, 0) : XS(k, 0)) + l0 + (k > 0 ? FR(0, k) : (T)0);
                const T m1 = 2 * Q1 * (LTI ? XS(k, 1) - XR(k, 1) : XS(k, 1)) + l1 + (k > 0 ? FR(1, k) : (T)0);
                const T m2 = 2 * Q2 * (LTI ? XS(k, 2) - XR(k, 2) : XS(k, 2)) + STG(0, k) * l0 + STG(1, k) * l1 + l2;
                l0 = m0; l1 = m1; l2 = m2;
            }
            GSTM(GR(2 * j), g0, m); GSTM(GR(2 * j + 1), g1, m);
        }
        __syncthreads();
    };

#if RMPC_GROUP_SCAN
    // The adjoint is a pair of suffix sums too: lambda_{x,y} accumulate 2Q e + hinge forces,
    // and lambda_theta accumulates 2Q e_theta + a_k . lambda_{x,y}(k+1).  Two reverse group
    // scans over the same chunks, then each lane forms its steps' gradient (BS = 1).
    // With `sets`, the same pass also builds the projected-Newton sets of the groups with m:
    // epsilon-active box components and the hinge rows with r > 0.
    auto gradient = [&](bool m, bool sets) __attribute__((always_inline)) {
        if constexpr (BS == 1) {
            refresh();
            constexpr int C = (N + G - 1) / G;
            const int k0 = gl * C;
            T c0[C], c1[C], c2[C];
            uint32_t nhb[C];
            T A0 = 0, A1 = 0;
#pragma unroll
            for (int i = 0; i < C; i++) {
                const int k = k0 + i;
                c0[i] = 0; c1[i] = 0; c2[i] = 0;
                nhb[i] = 0;
                if (k < N) {
                    const T y0 = XS(k, 0), y1 = XS(k, 1), y2 = XS(k, 2);
                    T f0 = 0, f1 = 0;
                    if (k > 0) {
                        for (int o = 0; o < no; o++) {
                            const T r = HB(o, k) - HN0(o, k) * y0 - HN1(o, k) * y1;
                            if (r > 0) {
                                f0 -= 2 * rho * r * HN0(o, k);
                                f1 -= 2 * rho * r * HN1(o, k);
                                nhb[i] |= 1u << o;
                            }
                        }
                    }
                    c0[i] = 2 * Q0 * (LTI ? y0 - XR(k, 0) : y0) + f0;
                    c1[i] = 2 * Q1 * (LTI ? y1 - XR(k, 1) : y1) + f1;
                    c2[i] = 2 * Q2 * (LTI ? y2 - XR(k, 2) : y2);
                    A0 += c0[i];
                    A1 += c1[i];
                }
            }
            const T t0 = 2 * P0 * (LTI ? XS(N, 0) - XR(N, 0) : XS(N, 0));
            const T t1 = 2 * P1 * (LTI ? XS(N, 1) - XR(N, 1) : XS(N, 1));
            const T t2 = 2 * P2 * (LTI ? XS(N, 2) - XR(N, 2) : XS(N, 2));
            T L0 = t0 + gscan_excl<G, false>(A0, gl), L1 = t1 + gscan_excl<G, false>(A1, gl);
            T l0n[C], l1n[C], A2 = 0;
#pragma unroll
            for (int i = C - 1; i >= 0; i--) {
                const int k = k0 + i;
                l0n[i] = L0; l1n[i] = L1;
                if (k < N) {
                    c2[i] += STG(0, k) * L0 + STG(1, k) * L1;
                    A2 += c2[i];
                    L0 += c0[i];
                    L1 += c1[i];
                }
            }
            T L2 = t2 + gscan_excl<G, false>(A2, gl);
            T *const jk = junk;
            T gz[C][2], zz[C][2], wl = 0;
#pragma unroll
            for (int i = C - 1; i >= 0; i--) {
                const int k = k0 + i;
                gz[i][0] = 0; gz[i][1] = 0; zz[i][0] = 0; zz[i][1] = 0;
                if (k < N) {
                    zz[i][0] = ZZ(2 * k); zz[i][1] = ZZ(2 * k + 1);
                    const T g0 = STG(2, k) * l0n[i] + STG(3, k) * l1n[i] + 2 * R0 * (zz[i][0] + STG(4, k));
                    const T g1 = dt * L2 + 2 * R1 * (zz[i][1] + STG(5, k));
                    *(m ? &GR(2 * k) : jk) = g0;
                    *(m ? &GR(2 * k + 1) : jk) = g1;
                    gz[i][0] = g0; gz[i][1] = g1;
                    L2 += c2[i];
                    if (sets) {
#pragma unroll
                        for (int c = 0; c < 2; c++) {
                            const T lo = BND(2 * c, k), hi = BND(2 * c + 1, k);
                            wl = fmax(wl, fabs(zz[i][c] - clampv(zz[i][c] - gz[i][c], lo, hi)));
                        }
                    }
                }
            }
            if (sets) {
                const T eps = fmin(SetTol<T>::pn, gmaxv<G>(wl));
#pragma unroll
                for (int i = 0; i < C; i++) {
                    const int k = k0 + i;
                    if (k < N && m) {
                        uint32_t w = 0;
#pragma unroll
                        for (int c = 0; c < 2; c++) {
                            const T lo = BND(2 * c, k), hi = BND(2 * c + 1, k), z = zz[i][c], g = gz[i][c];
                            const uint32_t st = (z <= lo + eps && g > 0) ? 1u : ((z >= hi - eps && g < 0) ? 2u : 0u);
                            w |= st << (2 * c);
                        }
                        BF(k) = w;
                        HF(k) = nhb[i];
                    }
                }
            }
            __syncthreads();
        } else {
            gradient_seq(m);
        }
    };
#else
    auto gradient = [&](bool m, bool) __attribute__((always_inline)) { gradient_seq(m); };
#endif

    // ---- the iteration loop (groups in lockstep)
    bool done_ok = false;             // certified with a finite objective: written after the loop
    double J_out = 0.0;
    int used_out = 0, it_out = 0;
    int it = 0, cyc = 0;
    T F = 0.0;
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    const int max_iter = p.max_iter;
    while (__any(phase <= PH_PN)) {
        GSITE(3);
        const bool act = phase <= PH_PN;
        const bool pn = phase == PH_PN;
        if (__any(pn)) {
            // projected Newton: gradient at z, epsilon-active box components, hinge rows with
            // r > 0 -- the sets of this solve (projected-Newton phase)
#if RMPC_GROUP_SCAN
            if constexpr (BS == 1) {
                gradient(pn, true);
            } else
#endif
            {
            gradient(pn, false);
            refresh();
            T wl = 0.0;
            for (int i = gl; i < 2 * NB; i += G) {
                const int j = i >> 1, c = i & 1;
                const T lo = BND(2 * c, j), hi = BND(2 * c + 1, j), z = ZZ(i);
                wl = fmax(wl, fabs(z - clampv(z - GR(i), lo, hi)));
            }
            const T eps = fmin(SetTol<T>::pn, gmaxv<G>(wl));
            if (pn) {
                for (int j = gl; j < NB; j += G) {
                    uint32_t w = 0;
#pragma unroll
                    for (int c = 0; c < 2; c++) {
                        const T lo = BND(2 * c, j), hi = BND(2 * c + 1, j), z = ZZ(2 * j + c), g = GR(2 * j + c);
                        const uint32_t s = (z <= lo + eps && g > 0) ? 1u : ((z >= hi - eps && g < 0) ? 2u : 0u);
                        w |= s << (2 * c);
                    }
                    BF(j) = w;
                }
                for (int k = gl; k < N; k += G) {
                    uint32_t nh = 0;
                    if (k > 0) {
                        const T y0 = XS(k, 0), y1 = XS(k, 1);
                        for (int o = 0; o < no; o++)
                            if (HB(o, k) - HN0(o, k) * y0 - HN1(o, k) * y1 > 0) nh |= 1u << o;
                    }
                    HF(k) = nh;
                }
            }
            __syncthreads();
            }
            GPROF(1);
        }
        if (act) it++;
        const bool chg = solve_test();
        GSITE(4);
        const bool cert = act && !chg;
        if (__any(cert)) {
            // ---- certified: objective of the candidate (its trajectory is in XS from the
            // certifying solve's forward sweep), and a copy of inputs + trajectory kept for
            // the single output write after the loop (later sweeps overwrite ZC / XS)
            int used = 0;
            const T J = cost(RC::ZC, used);
            refresh();
            if (cert && isfinite(J)) {
                for (int i = gl; i < 2 * NB; i += G) ZF(i) = ZC(i);
                for (int k = gl; k <= N; k += G) {
                    XF(k, 0) = XS(k, 0); XF(k, 1) = XS(k, 1); XF(k, 2) = XS(k, 2);
                }
                done_ok = true;
                J_out = J;
                used_out = used;
                it_out = it0 + it;
            } else if (cert && gl == 0) {
                group_retry(a, b);
            }
            __syncthreads();
            GPROF(6);
        }
        if (cert) phase = PH_DONE;
        // PDAS groups: take the new sets; cycle / cap -> projected Newton
        bool to_pn = false, fail = false;
        if (phase == PH_PDAS) {
            refresh();
            for (int k = gl; k < N; k += G) HF(k) = NHF(k);
            for (int j = gl; j < NB; j += G) BF(j) = NBF(j);
            if (a.pdas_cap > 4) {
                uint64_t sig = 1469598103934665603ull;
                for (int k = 0; k < N; k++) sig = (sig ^ (uint64_t)NHF(k)) * 1099511628211ull;
                for (int j = 0; j < NB; j++) sig = (sig ^ (uint64_t)NBF(j)) * 1099511628211ull;
                if (sig == s0 || sig == s1 || sig == s2 || sig == s3) cyc = 1;
                s3 = s2; s2 = s1; s1 = s0; s0 = sig;
            }
            if (it >= a.pdas_cap || cyc) {
                if (it < max_iter) to_pn = true;
                else fail = true;
            }
        }
        __syncthreads();
        if (__any(to_pn)) {          // z = projected last candidate, F = objective(z)
            refresh();
            if (to_pn) {
                for (int i = gl; i < 2 * NB; i += G) {
                    const int j = i >> 1, c = i & 1;
                    ZZ(i) = clampv(ZC(i), BND(2 * c, j), BND(2 * c + 1, j));
                }
            }
            __syncthreads();
            int u;
            const T f = objective(RC::ZZ, to_pn, u);
            if (to_pn) { F = f; phase = PH_PN; }
            __syncthreads();
        }
        GPROF(7);
        // projected-Newton groups that did not certify: Armijo along the projection arc
        bool searching = pn && !cert;
        if (__any(searching)) {
            refresh();
            T alpha = 1.0;
            for (int ls = 0; ls < 40 && __any(searching); ls++) {
#if RMPC_GROUP_SCAN
                if constexpr (BS == 1) {
                    bool acc;
                    T gd;
                    const T Ft = ls_trial(alpha, searching, F, acc, gd);
                    if (acc) {
                        F = Ft;
                        searching = false;
                    }
                    {              // safeguarded quadratic interpolation: q(s) = F + gd s + c s^2, q(1) = Ft
                        const T c = Ft - F - gd;
                        const T s = c > (T)0 ? -gd / ((T)2 * c) : (T)0.5;
                        alpha *= fmin(fmax(s, (T)0.1), (T)0.5);
                    }
                    continue;
                }
#endif
                T gd = 0.0;
                for (int i = gl; i < 2 * NB; i += G) {
                    const int j = i >> 1, c = i & 1;
                    const T z = ZZ(i);
                    const T zt = clampv(z + alpha * (ZC(i) - z), BND(2 * c, j), BND(2 * c + 1, j));
                    if (searching) ZT(i) = zt;
                    gd += GR(i) * (zt - z);
                }
                gd = gsum<G>(gd);
                __syncthreads();
                int u;
                const T Ft = objective(RC::ZT, searching, u);
                refresh();
                const bool acc = searching && Ft <= F + (T)1e-4 * gd;
                if (acc) {
                    for (int i = gl; i < 2 * NB; i += G) ZZ(i) = ZT(i);
                    F = Ft;
                    searching = false;
                }
                alpha *= (T)0.5;                 // (block size > 1: fixed factor)
                __syncthreads();
            }
            if (searching) fail = true;          // no acceptable step
            GPROF(8);
            GSITE(5);
        }
        if (prof_on) pacc[9]++;
        if (phase == PH_PN && !cert && it >= max_iter) fail = true;
        if (fail) {
            if (gl == 0) group_retry(a, b);
            phase = PH_IDLE;
        }
        if (prof_on && gl == 0 && (cert || fail))   // per robot: tail iterations (histogram)
            atomicAdd(a.prof + 24 + min(it, 31), 1ull);
    }
    // ---- outputs of every certified robot of the wave, once (mpc_controller.py:484-520)
    GSITE(6);
    if (__any(done_ok)) {
        refresh();
        if (done_ok) {
            const int sc = (!LTI && a.step_count) ? a.step_count[b] : 0;
            constexpr bool F64 = sizeof(T) == 8;
            // Every global load of the pass is issued before its first store: gfx950 counts
            // loads and stores in one in-order vmcnt, so a load behind the u_seq / x_pred
            // stores would wait for all of them to complete (the lane-per-robot kernel's
            // output pass, HISTORY.md section 3)
            constexpr int KU = (N + G - 1) / G, KX = (N + 1 + G - 1) / G;
            double urv[F64 ? 1 : KU][2], xrv[LTI ? 1 : KX][3];
            if constexpr (!F64) {
#pragma unroll
                for (int i = 0; i < KU; i++) {
                    const int k = gl + G * i;
                    urv[i][0] = k < N ? ur[2 * k] : 0.0;
                    urv[i][1] = k < N ? ur[2 * k + 1] : 0.0;
                }
            }
            if constexpr (!LTI) {
#pragma unroll
                for (int i = 0; i < KX; i++) {
                    const int k = gl + G * i;
                    const bool in = a.x_pred && k <= N;
                    xrv[i][0] = in ? xr[3 * k] : 0.0;
                    xrv[i][1] = in ? xr[3 * k + 1] : 0.0;
                    xrv[i][2] = in ? xr[3 * k + 2] : 0.0;
                }
            }
#pragma unroll
            for (int i = 0; i < KU; i++) {
                const int k = gl + G * i;
                if (k >= N) break;
                const int j = k / BS;
                // fp64: u = du + u_ref in the record; fp32: du + the fp64 u_ref (only the
                // deviation carries fp32 rounding, as in the lane-per-robot kernel)
                const double v0 = F64 ? (double)(ZF(2 * j) + STG(4, k)) : (double)ZF(2 * j) + urv[F64 ? 0 : i][0];
                double v1 = F64 ? (double)(ZF(2 * j + 1) + STG(5, k)) : (double)ZF(2 * j + 1) + urv[F64 ? 0 : i][1];
                if (!LTI && k == 0 && sc < p.ramp_up_steps) {              // :502-505 (LTV only)
                    const double lim = p.omega_max * ((double)(sc + 1) / (double)p.ramp_up_steps);
                    v1 = clampv(v1, -lim, lim);
                }
                if (a.u_seq) {
                    a.u_seq[((size_t)b * N + k) * 2] = v0;
                    a.u_seq[((size_t)b * N + k) * 2 + 1] = v1;
                }
                if (k == 0) {
                    a.u0[2 * b] = v0;
                    a.u0[2 * b + 1] = v1;
                }
            }
            if (a.x_pred) {                                                 // :497
#pragma unroll
                for (int i = 0; i < KX; i++) {
                    const int k = gl + G * i;
                    if (k > N) break;
                    double *xp = a.x_pred + ((size_t)b * (N + 1) + k) * 3;
                    if constexpr (LTI) {                                    // absolute states
                        xp[0] = (double)XF(k, 0); xp[1] = (double)XF(k, 1); xp[2] = (double)XF(k, 2);
                    } else {
                        xp[0] = (double)XF(k, 0) + xrv[i][0];
                        xp[1] = (double)XF(k, 1) + xrv[i][1];
                        xp[2] = (double)XF(k, 2) + xrv[i][2];
                    }
                }
            }
            if (gl == 0) {
                if (!LTI && a.step_count) a.step_count[b] = sc + 1;         // :507 (LTV only)
                if (a.cost) a.cost[b] = J_out;
                if (a.slack_used) a.slack_used[b] = (uint8_t)used_out;
                a.status[b] = RMPC_OPTIMAL;
                if (a.iters) a.iters[b] = it_out;
            }
            if (a.prev_sets) {             // warm start of this robot's next solve: its certified sets
                for (int k = gl; k < N; k += G) a.prev_sets[(size_t)k * a.nB + b] = HF(k);
                for (int j = gl; j < NB; j += G) a.prev_sets[(size_t)(N + j) * a.nB + b] = BF(j);
                if (gl == 0) a.prev_sets[(size_t)(N + NB) * a.nB + b] = a.prev_stamp;
            }
        }
    }
    GSITE(7);
    if (prof_on && gl == 0 && grp == 0) {
        for (int q = 0; q < 10; q++) atomicAdd(a.prof + q, pacc[q]);
        atomicAdd(a.prof + 10, 1ull);
        if (a.prof_waves) {          // per-wave record: phases, loop iterations, total cycles
            unsigned long long *r = a.prof_waves + (size_t)blockIdx.x * 16;
            for (int q = 0; q < 10; q++) r[q] = pacc[q];
            r[10] = __builtin_amdgcn_s_memtime() - tstart;
        }
    }
#undef STG
#undef BND
#undef HN0
#undef HN1
#undef HB
#undef WQ
#undef GN
#undef XS
#undef ZC
#undef ZZ
#undef ZT
#undef GR
#undef FR
#undef ZF
#undef XF
#undef XR
#undef HF
#undef BF
#undef NHF
#undef NBF
#undef GST
#undef GSTM
}

// lanes per robot: 16 (four robots per wave) while the record leaves room for four waves
// per CU, else 32
static inline int group_lanes(int N, int bs) { return N > 20 ? 32 : 16; }

// record bytes per robot in the arithmetic of `f32` (the kernel strides records by
// GRec<N, NB, T>::size(no) elements of T)
template <typename T>
static inline size_t group_rec_bytes_t(int N, int bs, int no) {
    if (bs == 2 && N == 6) return GRec<6, 3, T>::size(no) * sizeof(T);
    switch (N) {
        case 6: return GRec<6, 6, T>::size(no) * sizeof(T);
        case 10: return GRec<10, 10, T>::size(no) * sizeof(T);
        case 20: return GRec<20, 20, T>::size(no) * sizeof(T);
        default: return GRec<30, 30, T>::size(no) * sizeof(T);
    }
}
static inline size_t group_rec_bytes(int N, int bs, int no, bool f32) {
    return f32 ? group_rec_bytes_t<float>(N, bs, no) : group_rec_bytes_t<double>(N, bs, no);
}

}  // namespace rmpc
