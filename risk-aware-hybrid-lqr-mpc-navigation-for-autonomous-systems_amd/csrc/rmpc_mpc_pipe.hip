// rmpc_mpc_pipe.hip -- the MPC pipeline's first two stages in one launch (gfx950).
//
// The stage kernels run in sequence: the lane-per-robot PDAS stage (mpc_ltv_fast_kernel) hands
// the robots it does not certify to a retry list, and the lane-group tail (mpc_group_kernel)
// starts only when the whole stage has ended.  The stage ends when its slowest waves reach the
// PDAS cap, and most of the chip is idle long before that: most waves certify all 64 robots in
// one to three solves.  Here every wave runs its robots' PDAS stage (fast_body) and then turns
// consumer: it takes retry entries as they are published and solves them four at a time with the
// lane-group tail's code (group_solve), on the SIMD its own stage left free.  So the tail of the
// hard robots starts when they are handed on, not when the last wave of the stage ends, and the
// launch between the stages is gone.
//
// Hand-off protocol (agent scope; MI355X has one L2 per XCD):
//   producer (fast_body<..., PUB>'s hand-on): reserve a slot (atomicAdd on the list count),
//     store the robot and its sets write-through (agent-scope stores), wait for them (vmcnt(0)),
//     store the call's stamp into ready[slot]; after its stage every wave waits for its
//     stores and adds 1 to `done`.  No release fence: at agent scope it writes back the whole
//     L2, full of the stage's gain tiles (measured: 9 ms instead of 0.34 ms per launch).
//   consumer: takes a ticket of four slots (one atomic add on `head`), waits for each slot's
//     stamp, then reads the entry and its sets with agent-scope loads (group_solve<..., SC1>):
//     no acquire fence, which would invalidate the CU's cached inputs.
// Forward progress: a wave waits for future hand-ons only when every wave of the grid has
// started (`started` == grid), so a waiting wave never keeps a wave of its own grid from being
// placed; before that it claims only reserved slots (CAS, never past the count) and leaves when
// there are none.  Producers never wait.  A ticket past the final count (`done` == grid) ends
// the wave.  Every wait is bounded (~0.2 s) as a last-resort guard against a hang.
#include "rmpc_fast_body.h"
#include "rmpc_group_body.h"

#include <algorithm>
#include <vector>

namespace rmpc {

struct PipeCtl {
    int32_t *started, *head, *done;   // zeroed before the launch (the context's counter set)
    int32_t *count;                   // the retry list's count (MpcFastArgs::retry_count)
    const uint32_t *ready;            // per retry slot: the stamp of the call that published it
    uint32_t stamp;
    int sleep;                        // s_sleep(16) rounds between two polls of a slot's stamp
    int nowait;                       // 1: never wait for future hand-ons (claim reserved slots only)
    unsigned long long *diag;         // RMPC_PIPE_DIAG: per wave [start, stage end, rounds, first
                                      // round start, last round end, exit] (s_memrealtime ticks)
};

#define RMPC_PIPE_SPIN_TICKS 20000000ull   // s_memrealtime ticks (100 MHz): 0.2 s

__device__ __forceinline__ int rlx_load(const int32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Lane 0 of a wave: the next run of `want` retry slots for this wave, or -1 (leave).
//  - While not every wave of the grid has started, waiting is not allowed: claim only slots
//    already reserved (CAS on head, never past the count), else leave.
//  - Once every wave has started: take a ticket (one atomic add on head).  The slots may not be
//    reserved yet; the groups wait for them slot by slot (below).  No polling of shared words
//    here: with ~1000 waves polling one cache line, every claim and every hand-on atomic on that
//    line queued behind the polls (measured: the tail ran at one round per ~11 us, 9.8 ms per
//    launch instead of 0.34 ms).
__device__ __forceinline__ int pipe_claim(const PipeCtl pc, int want) {
    const unsigned waves = gridDim.x;
    if (!pc.nowait && (unsigned)rlx_load(pc.started) >= waves) {
        const int h = __hip_atomic_fetch_add(pc.head, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // every stage done and the ticket past the (final) count: leave without waiting
        if ((unsigned)rlx_load(pc.done) >= waves && h >= rlx_load(pc.count)) return -1;
        return h;
    }
    for (;;) {
        const int c = rlx_load(pc.count);
        int hh = rlx_load(pc.head);
        if (hh >= c) return -1;
        if (__hip_atomic_compare_exchange_strong(pc.head, &hh, hh + want < c ? hh + want : c, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return hh;
    }
}

// Wait for slot t's stamp.  False when the slot will never be filled: every wave's stage is done
// (`done` == grid: their hand-ons had completed before they counted, so the count is final) and
// t is past the count.  The slot's own stamp word is polled (one line per wave's four slots,
// spread over the chip); the shared `done` word every 4th poll.  Bounded: 0.2 s.
__device__ __forceinline__ bool pipe_wait_slot(const PipeCtl pc, int t) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned i = 0;; i++) {
        if (__hip_atomic_load(pc.ready + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == pc.stamp) return true;
        if ((i & 3u) == 3u && (unsigned)rlx_load(pc.done) >= gridDim.x) {
            if (t >= rlx_load(pc.count)) return false;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > RMPC_PIPE_SPIN_TICKS) return false;
        for (int q = 0; q < pc.sleep; q++) __builtin_amdgcn_s_sleep(16);
    }
}

template <int N, int BS, typename T, int NO, bool WS, int G>
__global__ __launch_bounds__(64, 1) void mpc_pipe_kernel(MpcFastArgs fa, GroupArgs ga, PipeCtl pc) {
    constexpr int NB = (N + BS - 1) / BS, RPW = 64 / G;
    const int lane = threadIdx.x;
    unsigned long long *const dg = pc.diag ? pc.diag + (size_t)blockIdx.x * 8 : nullptr;
    if (dg && lane == 0) dg[0] = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) __hip_atomic_fetch_add(pc.started, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---- stage 1: this wave's robots (hand-ons published slot by slot)
    fast_body<N, BS, T, false, NO, 1, WS, true>(fa, blockIdx.x);
    // every hand-on of this wave has completed (its stamp stores included) before `done` counts it
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(pc.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dg && lane == 0) dg[1] = __builtin_amdgcn_s_memrealtime();
    unsigned long long rounds = 0;
    // ---- stage 2: lane-group solves of published retry entries, RPW per round
    extern __shared__ double lds_raw[];
    T *const lds = reinterpret_cast<T *>(lds_raw);
    const int gl = lane % G, grp = lane / G;
    const int rec = GRec<N, NB, T>::size(ga.no);
    for (;;) {
        int h = -1;
        if (lane == 0) h = pipe_claim(pc, RPW);
        h = __shfl(h, 0);
        if (h < 0) break;
        const int t = h + grp;
        const bool have = pipe_wait_slot(pc, t);
        if (!__ballot(have)) break;             // a run past the final count: nothing left
        if (dg && lane == 0 && rounds++ == 0) dg[3] = __builtin_amdgcn_s_memrealtime();
        // (the entry and its sets are read with agent-scope loads inside group_solve: no acquire
        // fence, which would drop this CU's cached inputs; only the compiler's order is pinned)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __syncthreads();
        group_solve<N, BS, G, T, false, true>(ga, lds + grp * rec, t, have, gl, grp);
        __syncthreads();
        if (dg && lane == 0) dg[4] = __builtin_amdgcn_s_memrealtime();
    }
    if (dg && lane == 0) {
        dg[2] = rounds;
        dg[5] = __builtin_amdgcn_s_memrealtime();
    }
}

}  // namespace rmpc

using namespace rmpc;

bool rmpc_mpc_pipe_supported(int N, int bs, int prec, bool lti, int no) {
    return N == 20 && bs == 1 && prec == RMPC_F64 && !lti && no == 3 && rmpc_mpc_group_supported(20, 1, 3);
}

hipError_t rmpc_launch_mpc_pipe(const MpcFastArgs &a, int N, int bs, int32_t *retry2, int32_t *retry2_count,
                                int tail_cap, int32_t *ctr, hipStream_t stream) {
    const int64_t n = a.B;
    if (n <= 0) return hipSuccess;
    if (!rmpc_mpc_pipe_supported(N, bs, RMPC_F64, false, a.no) || !a.ready || !a.retry_sets) return hipErrorInvalidValue;
    GroupArgs ga;
    memset(&ga, 0, sizeof(ga));
    ga.prm = a.prm;
    ga.no = a.no;
    ga.x0 = a.x0; ga.x_refs = a.x_refs; ga.u_refs = a.u_refs; ga.obs = a.obs;
    ga.ref_rows = a.ref_rows; ga.uref_rows = a.uref_rows;
    ga.step_count = a.step_count;
    ga.u0 = a.u0; ga.u_seq = a.u_seq; ga.x_pred = a.x_pred; ga.cost = a.cost;
    ga.status = a.status; ga.iters = a.iters; ga.slack_used = a.slack_used;
    ga.index = a.retry; ga.count = a.retry_count;
    ga.retry = retry2; ga.retry_count = retry2_count;
    ga.warm = a.retry_sets;
    ga.pdas_cap = tail_cap < RMPC_PDAS_ITERS ? tail_cap : RMPC_PDAS_ITERS;
    ga.ls_beta = 0.0;
    ga.nB = a.B;
    ga.prev_sets = a.prev_sets;
    ga.prev_stamp = a.prev_stamp;
    PipeCtl pc;
    pc.started = ctr;
    pc.head = ctr + 1;
    pc.done = ctr + 2;
    pc.count = a.retry_count;
    pc.ready = a.ready;
    pc.stamp = a.ready_stamp;
    pc.sleep = rmpc_knob("RMPC_PIPE_SLEEP") ? atoi(rmpc_knob("RMPC_PIPE_SLEEP")) : 1;
    pc.nowait = rmpc_knob("RMPC_PIPE_NOWAIT") ? 1 : 0;
    pc.diag = nullptr;
    const int64_t waves = (n + RMPC_WAVE - 1) / RMPC_WAVE;
    if (rmpc_knob("RMPC_PIPE_DIAG")) {                  // diagnostics: synchronises the stream
        const hipError_t e = hipMalloc((void **)&pc.diag, (size_t)waves * 8 * sizeof(unsigned long long));
        if (e != hipSuccess) return e;
        (void)hipMemsetAsync(pc.diag, 0, (size_t)waves * 8 * sizeof(unsigned long long), stream);
    }
    constexpr int G = 16;
    const size_t lds_fast = (size_t)3 * N * RMPC_WAVE * sizeof(double) + (size_t)RMPC_WAVE * 17 * sizeof(double);
    const size_t lds_group = (size_t)(64 / G) * GRec<20, 20, double>::size(a.no) * sizeof(double);
    const size_t lds = lds_fast > lds_group ? lds_fast : lds_group;
    const void *fn = a.prev_sets ? (const void *)mpc_pipe_kernel<20, 1, double, 3, true, G>
                                 : (const void *)mpc_pipe_kernel<20, 1, double, 3, false, G>;
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    const dim3 grid((unsigned)((n + RMPC_WAVE - 1) / RMPC_WAVE)), block(RMPC_WAVE);
    MpcFastArgs fa = a;
    void *args[] = {&fa, &ga, &pc};
    const hipError_t e = hipLaunchKernel(fn, grid, block, args, lds, stream);
    if (e != hipSuccess) return e;
    if (pc.diag) {          // per-wave timeline summary, microseconds from the first wave's start
        std::vector<unsigned long long> h((size_t)waves * 8);
        hipError_t e2 = hipMemcpyAsync(h.data(), pc.diag, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream);
        if (e2 == hipSuccess) e2 = hipStreamSynchronize(stream);
        (void)hipFree(pc.diag);
        if (e2 != hipSuccess) return e2;
        unsigned long long t0 = ~0ull;
        for (int64_t w = 0; w < waves; w++) t0 = std::min(t0, h[w * 8]);
        auto us = [&](unsigned long long v) { return v ? (double)(v - t0) / 100.0 : -1.0; };
        std::vector<double> st, se, fr, lr, ex;
        long long rounds = 0, workers = 0;
        for (int64_t w = 0; w < waves; w++) {
            const unsigned long long *r = &h[w * 8];
            st.push_back(us(r[0])); se.push_back(us(r[1])); ex.push_back(us(r[5]));
            if (r[2]) { fr.push_back(us(r[3])); lr.push_back(us(r[4])); rounds += (long long)r[2]; workers++; }
        }
        auto q = [](std::vector<double> v, double p) {
            if (v.empty()) return -1.0;
            std::sort(v.begin(), v.end());
            return v[(size_t)(p * (double)(v.size() - 1))];
        };
        fprintf(stderr, "[pipe] waves %lld | start max %.1f | stage end p50 %.1f p90 %.1f max %.1f | %lld tail rounds on %lld waves "
                "| first round start min %.1f p50 %.1f max %.1f | last round end p50 %.1f max %.1f | exit max %.1f us\n",
                (long long)waves, q(st, 1.0), q(se, 0.5), q(se, 0.9), q(se, 1.0), rounds, workers, q(fr, 0.0), q(fr, 0.5),
                q(fr, 1.0), q(lr, 0.5), q(lr, 1.0), q(ex, 1.0));
    }
    return hipGetLastError();
}
