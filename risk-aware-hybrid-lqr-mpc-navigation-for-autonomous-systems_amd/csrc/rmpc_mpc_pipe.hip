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
//   producer (fast_body's hand-on): reserve a slot (atomicAdd on the list count), store the
//     robot and its sets, release fence + vmcnt(0), store the call's stamp into ready[slot];
//     after its stage every wave releases and adds 1 to `done`.
//   consumer: claims a run of reserved slots with a CAS on `head` (never past the count), waits
//     for each claimed slot's stamp (its producer is running and never waits, so the wait is
//     short), acquires, then reads the entry.
// Forward progress: a wave waits for work only when every wave of the grid has started
// (`started` == grid), so a waiting wave never keeps a wave of its own grid from being placed;
// before that it takes only what is already there and leaves.  Producers never wait.  A wave
// leaves when every wave's stage is done (`done` == grid; the count is then final) and the
// list is drained.  Every spin is bounded (~0.2 s) as a last-resort guard against a hang.
#include "rmpc_fast_body.h"
#include "rmpc_group_body.h"

namespace rmpc {

struct PipeCtl {
    int32_t *started, *head, *done;   // zeroed before the launch (the context's counter set)
    int32_t *count;                   // the retry list's count (MpcFastArgs::retry_count)
    const uint32_t *ready;            // per retry slot: the stamp of the call that published it
    uint32_t stamp;
};

#define RMPC_PIPE_SPIN_TICKS 20000000ull   // s_memrealtime ticks (100 MHz): 0.2 s

__device__ __forceinline__ int rlx_load(const int32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Lane 0 of a wave: claim up to `want` published-or-reserved retry slots.  Returns the first
// slot in *h and the number claimed (> 0), or -1: nothing left for this wave.
__device__ __forceinline__ int pipe_claim(const PipeCtl pc, int want, int *h) {
    const unsigned waves = gridDim.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const int c = rlx_load(pc.count);
        int hh = rlx_load(pc.head);
        if (hh < c) {
            const int n = c - hh < want ? c - hh : want;
            if (__hip_atomic_compare_exchange_strong(pc.head, &hh, hh + n, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
                *h = hh;
                return n;
            }
            continue;
        }
        // nothing reserved beyond the head
        if ((unsigned)__hip_atomic_load(pc.done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= waves) {
            // every stage has handed on what it will: the count is final
            if (rlx_load(pc.head) >= rlx_load(pc.count)) return -1;
            continue;
        }
        // waiting is safe only once every wave of the grid has been placed
        if ((unsigned)rlx_load(pc.started) < waves) return -1;
        if (__builtin_amdgcn_s_memrealtime() - t0 > RMPC_PIPE_SPIN_TICKS) return -1;
        __builtin_amdgcn_s_sleep(8);
    }
}

template <int N, int BS, typename T, int NO, bool WS, int G>
__global__ __launch_bounds__(64, 1) void mpc_pipe_kernel(MpcFastArgs fa, GroupArgs ga, PipeCtl pc) {
    constexpr int NB = (N + BS - 1) / BS, RPW = 64 / G;
    const int lane = threadIdx.x;
    if (lane == 0) __hip_atomic_fetch_add(pc.started, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---- stage 1: this wave's robots (hand-ons published slot by slot)
    fast_body<N, BS, T, false, NO, 1, WS>(fa, blockIdx.x);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(pc.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---- stage 2: lane-group solves of published retry entries, RPW per round
    extern __shared__ double lds_raw[];
    T *const lds = reinterpret_cast<T *>(lds_raw);
    const int gl = lane % G, grp = lane / G;
    const int rec = GRec<N, NB, T>::size(ga.no);
    for (;;) {
        int h = 0, n = -1;
        if (lane == 0) n = pipe_claim(pc, RPW, &h);
        n = __shfl(n, 0);
        h = __shfl(h, 0);
        if (n < 0) break;
        const int t = h + grp;
        bool have = grp < n;
        if (have) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(pc.ready + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != pc.stamp) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > RMPC_PIPE_SPIN_TICKS) { have = false; break; }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __syncthreads();
        group_solve<N, BS, G, T, false>(ga, lds + grp * rec, t, have, gl, grp);
        __syncthreads();
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
    return hipGetLastError();
}
