// rmpc_mpc_group.hip -- lane-group-per-robot MPC tail solver (Riccati form).
//
// The lane-per-robot kernel (rmpc_mpc_fast.hip) runs one robot per lane: every quantity of
// an active-set iteration -- the hinge rows of every step and obstacle, the box bounds, the
// set rules, the objective terms -- sits on that lane's sequential instruction stream next
// to the Riccati recursion, ~15k instructions per iteration.  For the few robots that need
// many iterations this stream is the launch's critical path.
//
// Here a group of G lanes (G = 16: four robots per wave) owns one robot.  Only the two
// recursions stay sequential -- the backward block Riccati sweep (rmpc_riccati.h, the same
// algebra as the other kernels) and the forward state/input sweep, both computed
// redundantly by the group's lanes from LDS broadcasts.  Everything else is spread over the
// group: the linearisation and hinge rows are built once per robot (step k on lane k mod G),
// each iteration's per-step hinge weights, set tests, cost terms, hinge forces and box
// rules run lane-parallel over steps or blocks, and group reductions go through shuffles.
//
// Algorithm (that of the round-1 condensed wave-per-robot tail, which it replaced; HISTORY.md):
// PDAS from the previous stage's active sets (cap + cycle detection), then projected Newton
// with an Armijo search along the projection arc, every candidate certified by the
// set-reproduction test, so the result is the QP's exact optimum.  Robots that do not
// certify (or carry non-finite data) go on to the generic kernel.
//
// The groups of a wave run in lockstep (one shared loop; a group that is done is masked),
// LTV formulation (mpc_controller.py:345-522).
#include "rmpc_group_body.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace rmpc {

// One wave per workgroup, 64/G list entries per wave per round.  The grid is capped
// (rmpc_launch_mpc_group: GROUP_GRID_MAX waves, fewer when the list's capacity is smaller) and
// the waves loop over rounds until the device-side count is covered; every wave reads the same
// count, so every wave reaches the exit.  The list's capacity is the whole batch, but a launch
// hands a few thousand robots to this stage: a grid over the capacity (16384 one-wave
// workgroups at config 3, ~950 with work) kept the SIMDs it passed through idle for 28% of the
// in-flight run, one dispatch gap per empty workgroup (profiles/r05/wave_timeline_*.json).
// (Round 1's persistent form faulted beyond its first round; that tree's tail is gone, and
// round 2 ran this loop with every config-3 robot through it, 16 rounds per wave, bounds-checked
// and bitwise equal: HISTORY.md section 3.)
template <int N, int BS, int G, typename T, bool LTI>
__global__ __launch_bounds__(64, 1) void mpc_group_kernel(GroupArgs a) {
    constexpr int NB = (N + BS - 1) / BS, RPW = 64 / G;
    RMPC_WLOG_BEGIN
    extern __shared__ double lds_raw[];
    T *const lds = reinterpret_cast<T *>(lds_raw);
    const int lane = threadIdx.x, gl = lane % G, grp = lane / G;
    const int rec = GRec<N, NB, T>::size(a.no);
    const int cnt = *a.count;
    if (a.chk && lane == 0 && blockIdx.x == 0 && (cnt < 0 || cnt > a.nB)) diag_hit(a.chk, 2, 4, cnt);
    if (a.count_out && lane == 0 && blockIdx.x == 0)
        __hip_atomic_store(a.count_out, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int t0 = blockIdx.x * RPW; t0 < cnt; t0 += gridDim.x * RPW) {
        const int t = t0 + grp;
        group_solve<N, BS, G, T, LTI>(a, lds + grp * rec, t, t < cnt, gl, grp);
        __syncthreads();           // (the next round rewrites the groups' LDS records)
    }
    GSITE(8);
    RMPC_WLOG_END(WL_GROUP)
}

}  // namespace rmpc

using namespace rmpc;
RMPC_WLOG_SETTER(rmpc_wlog_set_group)

// the tail's grid cap in waves (1024: one per SIMD of the chip)
#define GROUP_GRID_MAX 1024

void GroupDiag::release() {
    if (pw) (void)hipFree(pw);
    if (chk_host) (void)hipHostFree(chk_host);
    if (site_host) (void)hipHostFree(site_host);
    pw = nullptr; pw_cap = 0; chk_host = nullptr; site_host = nullptr; site_cap = 0;
}

// fp64 only: a refined fp32 request's tail is fp64 too (it returns fp64 optima).  (An fp32 tail
// ran config 4 faster, 42.9M against 38.7M solves/s, but with every robot routed through it its
// control error reached 1.9e-4 relative, above the north star's 1e-4: removed, HISTORY.md.)
bool rmpc_mpc_group_supported(int N, int bs, int no) {
    const bool inst = (bs == 1 && (N == 6 || N == 10 || N == 20 || N == 30)) || (bs == 2 && N == 6);
    if (!inst || no > 16) return false;
    const size_t lds = (size_t)(64 / group_lanes(N, bs)) * group_rec_bytes(N, bs, no, false);
    return lds <= 160 * 1024;
}

hipError_t rmpc_launch_mpc_group(const MpcDevParams &prm, int N, int bs, int no, int64_t capacity,
                                 const double *x0, const double *x_refs, int ref_rows,
                                 const double *u_refs, int uref_rows, const double *obstacles,
                                 int32_t *step_count, double *u0, double *u_seq, double *x_pred,
                                 double *cost, int32_t *status, uint8_t *slack_used, int32_t *iters,
                                 const int32_t *index, const int32_t *count, int32_t *retry,
                                 int32_t *retry_count, int pdas_cap, const uint32_t *warm,
                                 hipStream_t stream, unsigned long long *prof, bool lti,
                                 GroupDiag *diag, uint32_t *prev_sets, uint32_t prev_stamp,
                                 int32_t *count_out, int prev_count) {
    if (capacity <= 0) return hipSuccess;
    if (!rmpc_mpc_group_supported(N, bs, no) || (lti && bs != 1)) return hipErrorInvalidValue;
    GroupArgs a;
    a.prm = prm;
    a.no = no;
    a.x0 = x0; a.x_refs = x_refs; a.u_refs = u_refs; a.obs = obstacles;
    a.ref_rows = ref_rows; a.uref_rows = uref_rows;
    a.step_count = step_count;
    a.u0 = u0; a.u_seq = u_seq; a.x_pred = x_pred; a.cost = cost;
    a.status = status; a.iters = iters; a.slack_used = slack_used;
    a.index = index; a.count = count; a.retry = retry; a.retry_count = retry_count;
    a.warm = warm;
    a.prof = prof;
    a.prof_waves = nullptr;
    a.nB = capacity;
    a.chk = nullptr;
    a.site = nullptr;
    a.prev_sets = prev_sets;
    a.prev_stamp = prev_stamp;
    a.count_out = count_out;
    const int G = group_lanes(N, bs), rpw = 64 / G;
    const int64_t need = (capacity + rpw - 1) / rpw;
    // capped grid (the kernel loops over rounds): GROUP_GRID_MAX waves, one per SIMD of the chip
    // (RMPC_GROUP_GRID=<waves>: another cap, A/B)
    int64_t gmax = rmpc_knob("RMPC_GROUP_GRID") ? atoll(rmpc_knob("RMPC_GROUP_GRID")) : GROUP_GRID_MAX;
    // Sized from the list length this launch site saw last time (prev_count, a host-mapped word
    // the kernel writes; -1: unknown): every empty workgroup still takes an LDS slot and a SIMD
    // in flight, where a few hundred of the 1024 have work (config 3, eight batches in flight).
    // The round loop covers a longer list, so the hint only moves the cost, never the result.
    // A list longer than GROUP_GRID_MAX rounds (the LTI-group path's whole batches) keeps a
    // workgroup per round: looping 16 rounds per workgroup left the launch waiting on the
    // workgroups whose rounds held the hardest robots (LTI one batch alone 169M -> 157M).
    if (prev_count >= 0 && !rmpc_knob("RMPC_GROUP_GRID")) {
        const int64_t rounds = ((int64_t)prev_count + rpw - 1) / rpw;
        const int64_t want = rounds > GROUP_GRID_MAX ? rounds + 64 : rounds * 3 / 2 + 64;
        gmax = rounds > GROUP_GRID_MAX ? want : (want < GROUP_GRID_MAX ? want : GROUP_GRID_MAX);
    }
    const int64_t grid = need < gmax ? need : (gmax > 0 ? gmax : need);
    // diagnostics buffers (RMPC_DENSE_PROF=2, RMPC_GROUP_CHECK): owned by the caller's context
    const char *pe = rmpc_knob("RMPC_DENSE_PROF");
    if (diag && prof && pe && atoi(pe) >= 2) {
        if (diag->pw_cap < grid) {
            if (diag->pw) (void)hipFree(diag->pw);
            diag->pw = nullptr;
            diag->pw_cap = 0;
            const hipError_t e = hipMalloc((void **)&diag->pw, (size_t)grid * 16 * sizeof(unsigned long long));
            if (e != hipSuccess) return e;
            diag->pw_cap = grid;
        }
        const hipError_t e = hipMemsetAsync(diag->pw, 0, (size_t)grid * 16 * sizeof(unsigned long long), stream);
        if (e != hipSuccess) return e;
        a.prof_waves = diag->pw;
    }
    const char *ce = rmpc_knob("RMPC_GROUP_CHECK");
    const int check = diag && ce ? atoi(ce) : 0;
    if (check > 0) {                     // RMPC_GROUP_CHECK=1: bounds checks; =2: + per-wave sites
        hipError_t e = hipStreamSynchronize(stream);        // the record is rewritten from the host
        if (e != hipSuccess) return e;
        if (!diag->chk_host) {
            e = hipHostMalloc((void **)&diag->chk_host, 8 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent);
            if (e != hipSuccess) return e;
        }
        memset(diag->chk_host, 0, 8 * sizeof(int32_t));
        e = hipHostGetDevicePointer((void **)&a.chk, diag->chk_host, 0);
        if (e != hipSuccess) return e;
        if (check >= 2) {
            if (diag->site_cap < grid) {
                if (diag->site_host) (void)hipHostFree(diag->site_host);
                diag->site_host = nullptr;
                diag->site_cap = 0;
                e = hipHostMalloc((void **)&diag->site_host, (size_t)grid * sizeof(int32_t),
                                  hipHostMallocMapped | hipHostMallocCoherent);
                if (e != hipSuccess) return e;
                diag->site_cap = grid;
            }
            memset(diag->site_host, 0, (size_t)grid * sizeof(int32_t));
            e = hipHostGetDevicePointer((void **)&a.site, diag->site_host, 0);
            if (e != hipSuccess) return e;
        }
    }
    a.pdas_cap = pdas_cap < RMPC_PDAS_ITERS ? pdas_cap : RMPC_PDAS_ITERS;
    size_t lds = (size_t)rpw * group_rec_bytes(N, bs, no, false);
    const dim3 g((unsigned)grid), blk(64);
#define GK(n, b, g, t, l) (const void *)mpc_group_kernel<n, b, g, t, l>
    const void *fn = (bs == 1 && N == 30)   ? (lti ? GK(30, 1, 32, double, true) : GK(30, 1, 32, double, false))
                     : (bs == 1 && N == 20) ? (lti ? GK(20, 1, 16, double, true) : GK(20, 1, 16, double, false))
                     : (bs == 1 && N == 10) ? (lti ? GK(10, 1, 16, double, true) : GK(10, 1, 16, double, false))
                     : (bs == 1 && N == 6)  ? (lti ? GK(6, 1, 16, double, true) : GK(6, 1, 16, double, false))
                                            : GK(6, 2, 16, double, false);
#undef GK
    lds = rmpc_lds_slot_pad(fn, lds);          // one LDS slot (RMPC_LDS_SLOT)
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    void *args[] = {&a};
    {
        const hipError_t e = hipLaunchKernel(fn, g, blk, args, lds, stream);
        if (e != hipSuccess) return e;
    }
    if (a.prof_waves) {           // the slowest waves' phase breakdown (diagnostics)
        const int64_t n = grid;
        unsigned long long *h = (unsigned long long *)malloc((size_t)n * 16 * sizeof(unsigned long long));
        hipError_t e = hipMemcpyAsync(h, a.prof_waves, (size_t)n * 16 * sizeof(unsigned long long),
                                      hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        for (int rank = 0; rank < 3 && e == hipSuccess; rank++) {
            int64_t best = -1;
            for (int64_t w = 0; w < n; w++)
                if (h[w * 16 + 10] && (best < 0 || h[w * 16 + 10] > h[best * 16 + 10])) best = w;
            if (best < 0) break;
            const unsigned long long *r = h + best * 16;
            fprintf(stderr, "[group wave %lld] total %llu | setup %llu pn-pre %llu weights %llu back %llu fwd %llu rows %llu "
                    "out %llu upd %llu ls %llu | loop-its %llu\n", (long long)best, r[10], r[0], r[1], r[2], r[3], r[4],
                    r[5], r[6], r[7], r[8], r[9]);
            h[best * 16 + 10] = 0;
        }
        free(h);
        if (e != hipSuccess) return e;
    }
    if (a.chk) {                  // read from host-mapped memory: valid even if the launch faulted
        const hipError_t e = hipStreamSynchronize(stream);
        const int32_t *r = diag->chk_host;
        fprintf(stderr, "[group check] grid %lld: flags %d (1 robot index, 2 list count, 4 retry slot, "
                "8 list entry) first site %d value %d block %d; launch: %s\n", (long long)grid,
                r[0], r[1], r[2], r[3], hipGetErrorString(e));
        if (a.site) {             // waves by last site reached (8 = exited)
            long long hist[16] = {0};
            for (int64_t w = 0; w < grid; w++) hist[diag->site_host[w] & 15]++;
            fprintf(stderr, "[group check] waves by last site 0..9:");
            for (int q = 0; q < 10; q++) fprintf(stderr, " %lld", hist[q]);
            fprintf(stderr, "\n");
        }
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}
