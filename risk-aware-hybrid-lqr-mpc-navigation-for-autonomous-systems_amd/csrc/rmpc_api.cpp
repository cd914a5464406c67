// rmpc_api.cpp -- the C-ABI of librmpc.so (see include/rmpc.h).
//
// Host-pointer entry points stage through device buffers owned by the context (grow-only,
// allocated outside the launch path) on the context's stream and return after the
// results are back; the _dev entry points only validate and enqueue on the caller's
// stream.  There is no CPU compute path: every result is produced by a HIP kernel.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rmpc.h"
#include "rmpc_internal.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(RMPC_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));          \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
        }
        p = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

enum {
    SB_X0, SB_XREF, SB_UREF, SB_OBS, SB_STEP, SB_U0, SB_USEQ, SB_XPRED, SB_COST, SB_STATUS,
    SB_SLACK, SB_ITERS, SB_CACHE, SB_ERR, SB_K, SB_P, SB_EXTRA0, SB_EXTRA1, SB_EXTRA2, SB_EXTRA3,
    SB_COUNT
};

struct RmpcCtx {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf ws;                 // solver workspace
    DevBuf stage[SB_COUNT];    // staging buffers for host-pointer entry points
    // small host-array MPC calls (rmpc_mpc_solve_batch, <= RMPC_PACK_MAX bytes): every array
    // packed into one pinned host block and one device block, one copy each way
    void *pin = nullptr;
    size_t pin_cap = 0;
    DevBuf pack;
    DevBuf idx_lqr, idx_mpc, counts, hyb_status;
    DevBuf fast_gains, retry, retry2, retry_count, prof, retry_sets;
    DevBuf refine, refine_sets;     // fp32 requests: the fp32-certified robots and their sets
    // multi-pass lane-per-robot stage: the earlier passes' hand-on lists and their sets
    DevBuf pass_list[2], pass_sets[2];
    int passes[2] = {0, 0};           // rmpc_ctx_set_stage_passes: the earlier passes' caps (0: none)
    int lanes = 0;                    // rmpc_ctx_set_lanes_per_robot (0: the library default)
    GroupDiag gdiag;           // lane-group tail diagnostics (RMPC_GROUP_CHECK, RMPC_DENSE_PROF=2)
    // per tail launch site, the list length its last launch saw (host-mapped words the tail
    // kernel writes; -1 before the first): the next launch's grid (rmpc_launch_mpc_group)
    int32_t *tail_hint_h = nullptr, *tail_hint_d = nullptr;
    int32_t tail_est[8] = {-1, -1, -1, -1, -1, -1, -1, -1};   // per site: decaying max of the lengths seen
    // closed-loop rollout state (rmpc_rollout_batch)
    DevBuf ro_x, ro_xr, ro_ur, ro_u, ro_step, ro_cache, ro_prev, ro_since, ro_status, ro_used,
        ro_risk, ro_counts, ro_off, ro_pred;
    // stage timing of the last MPC launch (rmpc_ctx_set_timing): events before/after
    // the lane-per-robot, wave-per-robot and generic stages
    bool timing = false;
    bool timed = false;
    int fast_cap = 0, tail_cap = 0;   // rmpc_ctx_set_stage_caps (0: library default)
    bool use_side = true;             // rmpc_ctx_set_side_stream
    bool cold_rows = false;           // rmpc_ctx_set_cold_start: 1 = zero-correction rows active
    // rmpc_ctx_set_warm_start: per-robot active sets of each robot's previous solve
    // (MpcFastArgs::prev_sets), valid for the batch shape warm_B / warm_key they were made for
    bool warm_on = false;
    DevBuf warm_sets;
    int64_t warm_B = -1;
    int64_t warm_key = -1;
    uint32_t warm_calls = 0;          // stamp of the last warm call (MpcFastArgs::prev_stamp)
    // retry_count: two sets of list counters (RMPC_COUNT_WORDS words at word 0 and 32), used
    // by alternate pipelines; set k is zero in stream order when counts_zero[k] (the
    // previous pipeline's lane-per-robot kernel zeroed it), so the next needs no fill launch
    int count_set = 0;
    bool counts_zero[2] = {false, false};
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // hybrid step: two pairs of branch counters (words 0-1 and 16-17 of `counts`), alternated
    // per step; each step's switch kernel zeroes the pair the next step takes (hyb_ready: both
    // pairs are in that state).  The LQR branch runs on `side`, forked from and joined back to
    // the step's stream (hev), beside the MPC branch's half-empty lane-per-robot stage.
    int hyb_set = 0;
    bool hyb_ready = false;
    hipStream_t side = nullptr;
    hipEvent_t hev[2] = {nullptr, nullptr};
    // fp32 requests: the fp64 refinement pass runs on `side` beside the tail (rev: fork/join);
    // the robots it hands on go to a list of their own (retry_r, sets retry_sets_r)
    hipEvent_t rev[2] = {nullptr, nullptr};
    DevBuf retry_r, retry_sets_r;
    // Consecutive calls share state on the device (list counters zeroed by the previous
    // pipeline, the hybrid step's counter pairs, warm-start sets and stamps), which is correct
    // in stream order.  A call on another stream than the previous call's first waits for that
    // call (order_calls): an event recorded at the end of every stateful call (last_ev).
    hipEvent_t last_ev = nullptr;
    hipStream_t last_s = nullptr;
    bool last_valid = false;
    std::mutex mu;
    // multi-device context (rmpc_ctx_create_multi): one single-device context per entry;
    // empty for a single-device context
    std::vector<RmpcCtx *> sub;
};

// ------------------------------------------------------------------ multi-device split/gather
// A per-robot host array of a batch entry point: `row` bytes per robot, copied to the shards
// (in) and/or gathered back from them (out).  NULL arrays stay NULL in every shard.
struct RowArr {
    void *p;
    size_t row;
    bool in, out;
};

// Robots of shard d of n: blocks of RMPC_SPLIT_BLOCK consecutive robots dealt round-robin
// (block k to shard k mod n).  Robot difficulty follows the Figure-8 phase, which varies
// slowly with the robot index, so every shard gets the batch's mix (a contiguous split
// hands the obstacle-adjacent arcs to a few devices: HISTORY.md section 7).
#define RMPC_SPLIT_BLOCK 64

// Runs fn(sub_ctx, B_d, shard_pointers) for every device concurrently (one host thread
// each) on packed copies of its robots' rows, then scatters the outputs back in input order.
template <class F>
static int multi_run(RmpcCtx *c, int64_t B, std::vector<RowArr> arrs, F fn) {
    const int n = (int)c->sub.size();
    const int64_t nblk = (B + RMPC_SPLIT_BLOCK - 1) / RMPC_SPLIT_BLOCK;
    std::vector<int> rc(n, RMPC_OK);
    std::vector<std::string> err(n);
    auto work = [&](int d) {
        int64_t Bd = 0;
        for (int64_t k = d; k < nblk; k += n) Bd += std::min<int64_t>(RMPC_SPLIT_BLOCK, B - k * RMPC_SPLIT_BLOCK);
        if (Bd == 0) return;
        std::vector<std::vector<char>> st(arrs.size());
        std::vector<void *> q(arrs.size(), nullptr);
        for (size_t a = 0; a < arrs.size(); a++) {
            if (!arrs[a].p) continue;
            st[a].resize((size_t)Bd * arrs[a].row);
            q[a] = st[a].data();
            if (!arrs[a].in) continue;
            size_t off = 0;
            for (int64_t k = d; k < nblk; k += n) {
                const int64_t b0 = k * RMPC_SPLIT_BLOCK, m = std::min<int64_t>(RMPC_SPLIT_BLOCK, B - b0);
                memcpy(st[a].data() + off, (const char *)arrs[a].p + (size_t)b0 * arrs[a].row, (size_t)m * arrs[a].row);
                off += (size_t)m * arrs[a].row;
            }
        }
        rc[d] = fn(c->sub[d], Bd, q.data());
        if (rc[d] != RMPC_OK) { err[d] = g_last_error; return; }
        for (size_t a = 0; a < arrs.size(); a++) {
            if (!arrs[a].p || !arrs[a].out) continue;
            size_t off = 0;
            for (int64_t k = d; k < nblk; k += n) {
                const int64_t b0 = k * RMPC_SPLIT_BLOCK, m = std::min<int64_t>(RMPC_SPLIT_BLOCK, B - b0);
                memcpy((char *)arrs[a].p + (size_t)b0 * arrs[a].row, st[a].data() + off, (size_t)m * arrs[a].row);
                off += (size_t)m * arrs[a].row;
            }
        }
    };
    std::vector<std::thread> th;
    for (int d = 1; d < n; d++) th.emplace_back(work, d);
    work(0);
    for (auto &t : th) t.join();
    for (int d = 0; d < n; d++)
        if (rc[d] != RMPC_OK) return fail(rc[d], "device slot %d (device %d): %s", d, c->sub[d]->device, err[d].c_str());
    return RMPC_OK;
}


static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
#define RMPC_PACK_MAX ((size_t)256 << 10)   // bytes: the packed host-array path (rmpc_mpc_solve_batch)

extern "C" {

int rmpc_abi_version(void) { return RMPC_ABI_VERSION; }

const char *rmpc_last_error(void) { return g_last_error.c_str(); }

int rmpc_device_count(int *count) {
    if (!count) return fail(RMPC_EINVAL, "count is NULL");
    HIP_TRY(hipGetDeviceCount(count));
    return RMPC_OK;
}

static hipStream_t own(RmpcCtx *c);

int rmpc_ctx_create(int device_id, RmpcCtx **out) {
    if (!out) return fail(RMPC_EINVAL, "out is NULL");
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device_id < 0 || device_id >= n) return fail(RMPC_EINVAL, "device %d out of range (%d devices)", device_id, n);
    HIP_TRY(hipSetDevice(device_id));
    RmpcCtx *c = new RmpcCtx();
    c->device = device_id;
    // The context's own stream (host-pointer entry points) is made here, also for contexts
    // used only through the _dev entry points: creating it on first use measured slower with
    // batches in flight (config 4 68.0M against 70.1M, config 5 402M against 419M solves/s) --
    // the streams of a process share GPU_MAX_HW_QUEUES hardware queues, and which ones share
    // depends on the order they are made (HISTORY.md section 1)
    if (!own(c)) {
        delete c;
        return fail(RMPC_EHIP, "hipStreamCreate failed");
    }
    *out = c;
    return RMPC_OK;
}

int rmpc_ctx_create_multi(const int32_t *device_ids, int32_t n, RmpcCtx **out) {
    if (!out || !device_ids || n < 1) return fail(RMPC_EINVAL, "device_ids/out NULL or n < 1");
    if (n == 1) return rmpc_ctx_create(device_ids[0], out);
    RmpcCtx *c = new RmpcCtx();
    c->device = device_ids[0];
    for (int i = 0; i < n; i++) {
        RmpcCtx *s = nullptr;
        const int rc = rmpc_ctx_create(device_ids[i], &s);
        if (rc != RMPC_OK) {
            const std::string e = g_last_error;
            for (RmpcCtx *t : c->sub) rmpc_ctx_destroy(t);
            delete c;
            return fail(rc, "device slot %d: %s", i, e.c_str());
        }
        c->sub.push_back(s);
    }
    *out = c;
    return RMPC_OK;
}

int rmpc_ctx_device_count(const RmpcCtx *c, int32_t *n) {
    if (!c || !n) return fail(RMPC_EINVAL, "ctx or n is NULL");
    *n = c->sub.empty() ? 1 : (int32_t)c->sub.size();
    return RMPC_OK;
}

int rmpc_ctx_destroy(RmpcCtx *c) {
    if (!c) return RMPC_OK;
    if (!c->sub.empty()) {
        for (RmpcCtx *s : c->sub) rmpc_ctx_destroy(s);
        delete c;
        return RMPC_OK;
    }
    (void)hipSetDevice(c->device);
    // every queued use of the buffers first: the context's stream, the last stateful call
    // (which may have run on a caller stream, order_calls) and the side branch
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->last_valid && c->last_ev) (void)hipEventSynchronize(c->last_ev);
    if (c->side) (void)hipStreamSynchronize(c->side);
    c->ws.release();
    for (auto &b : c->stage) b.release();
    c->pack.release();
    if (c->pin) (void)hipHostFree(c->pin);
    c->pin = nullptr;
    c->idx_lqr.release();
    c->idx_mpc.release();
    c->counts.release();
    c->hyb_status.release();
    c->fast_gains.release();
    c->retry.release();
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->side) {
        (void)hipStreamSynchronize(c->side);
        (void)hipStreamDestroy(c->side);
    }
    for (auto &e : c->hev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : c->rev)
        if (e) (void)hipEventDestroy(e);
    if (c->last_ev) (void)hipEventDestroy(c->last_ev);
    c->retry_r.release();
    c->retry_sets_r.release();
    for (int i = 0; i < 2; i++) { c->pass_list[i].release(); c->pass_sets[i].release(); }
    c->retry2.release();
    c->retry_sets.release();
    c->refine.release();
    c->refine_sets.release();
    c->warm_sets.release();
    for (DevBuf *d : {&c->ro_x, &c->ro_xr, &c->ro_ur, &c->ro_u, &c->ro_step, &c->ro_cache, &c->ro_prev,
                      &c->ro_since, &c->ro_status, &c->ro_used, &c->ro_risk, &c->ro_counts, &c->ro_off, &c->ro_pred})
        d->release();
    c->prof.release();
    c->retry_count.release();
    c->gdiag.release();
    if (c->tail_hint_h) (void)hipHostFree(c->tail_hint_h);
    c->tail_hint_h = c->tail_hint_d = nullptr;
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return RMPC_OK;
}

int rmpc_ctx_synchronize(RmpcCtx *c) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    for (RmpcCtx *s : c->sub) {
        const int rc = rmpc_ctx_synchronize(s);
        if (rc != RMPC_OK) return rc;
    }
    if (!c->sub.empty()) return RMPC_OK;
    if (c->stream) HIP_TRY(hipStreamSynchronize(c->stream));
    return RMPC_OK;
}

int rmpc_ctx_set_timing(RmpcCtx *c, int32_t on) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    if (!c->sub.empty()) return fail(RMPC_ENOTSUP, "diagnostics take a single-device context");
    HIP_TRY(hipSetDevice(c->device));
    if (on)
        for (auto &e : c->ev)
            if (!e) HIP_TRY(hipEventCreate(&e));
    c->timing = on != 0;
    c->timed = false;
    return RMPC_OK;
}

int rmpc_ctx_set_stage_caps(RmpcCtx *c, int32_t fast_cap, int32_t tail_cap) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    if (fast_cap < 0 || fast_cap > 64 || tail_cap < 0 || tail_cap > 64)
        return fail(RMPC_EINVAL, "stage caps must be in [0, 64]");
    c->fast_cap = fast_cap;
    c->tail_cap = tail_cap;
    for (auto &sc : c->sub) {
        sc->fast_cap = fast_cap;
        sc->tail_cap = tail_cap;
    }
    return RMPC_OK;
}

int rmpc_ctx_set_stage_passes(RmpcCtx *c, int32_t first_cap, int32_t second_cap) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    if (first_cap < 0 || first_cap > 64 || second_cap < 0 || second_cap > 64 ||
        (second_cap > 0 && second_cap <= first_cap))
        return fail(RMPC_EINVAL, "pass caps must be in [0, 64], the second above the first (or 0)");
    c->passes[0] = first_cap;
    c->passes[1] = first_cap > 0 ? second_cap : 0;
    for (auto &sc : c->sub) {
        sc->passes[0] = c->passes[0];
        sc->passes[1] = c->passes[1];
    }
    return RMPC_OK;
}

int rmpc_ctx_set_lanes_per_robot(RmpcCtx *c, int32_t lanes) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    if (lanes < 0 || lanes > 2) return fail(RMPC_EINVAL, "lanes per robot %d: 0 (default), 1 or 2", lanes);
    c->lanes = lanes;
    for (auto &sc : c->sub) sc->lanes = lanes;
    return RMPC_OK;
}

int rmpc_ctx_set_side_stream(RmpcCtx *c, int32_t on) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    c->use_side = on != 0;
    for (auto &sc : c->sub) sc->use_side = on != 0;
    return RMPC_OK;
}

int rmpc_ctx_set_cold_start(RmpcCtx *c, int32_t mode) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    if (mode != 0 && mode != 1) return fail(RMPC_EINVAL, "cold-start mode %d: 0 or 1", mode);
    c->cold_rows = mode == 1;
    for (auto &sc : c->sub) sc->cold_rows = mode == 1;
    return RMPC_OK;
}

int rmpc_ctx_set_warm_start(RmpcCtx *c, int32_t on) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    c->warm_on = on != 0;
    c->warm_B = -1;                   // (re)start from the cold sets
    for (auto &sc : c->sub) {
        sc->warm_on = on != 0;
        sc->warm_B = -1;
    }
    return RMPC_OK;
}

int rmpc_mpc_stage_times(RmpcCtx *c, double *out3) {
    if (!c || !out3) return fail(RMPC_EINVAL, "ctx or out is NULL");
    if (!c->sub.empty()) return fail(RMPC_ENOTSUP, "diagnostics take a single-device context");
    if (!c->timed) return fail(RMPC_EINVAL, "no timed MPC launch on this context (rmpc_ctx_set_timing)");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipEventSynchronize(c->ev[3]));
    for (int i = 0; i < 3; i++) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]));
        out3[i] = ms;
    }
    return RMPC_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------ helpers
static int check_mpc_params(const RmpcMpcParams *p, int ref_rows, int uref_rows, int n_obs) {
    if (!p) return fail(RMPC_EINVAL, "params is NULL");
    const int N = p->horizon;
    if (N < 1 || N > RMPC_MAX_HORIZON) return fail(RMPC_EINVAL, "horizon %d not in [1, %d]", N, RMPC_MAX_HORIZON);
    if (n_obs < 0 || n_obs > RMPC_MAX_OBSTACLES) return fail(RMPC_EINVAL, "n_obs %d not in [0, %d]", n_obs, RMPC_MAX_OBSTACLES);
    if (p->formulation != RMPC_LTV && p->formulation != RMPC_LTI) return fail(RMPC_EINVAL, "bad formulation %d", p->formulation);
    if (p->formulation == RMPC_LTV) {
        if (p->block_size < 1) return fail(RMPC_EINVAL, "block_size %d < 1", p->block_size);
        if (ref_rows < N + 1) return fail(RMPC_EINVAL, "LTV needs ref_rows >= N+1 (%d < %d)", ref_rows, N + 1);
        if (uref_rows < N) return fail(RMPC_EINVAL, "LTV needs uref_rows >= N (%d < %d)", uref_rows, N);
    }
    if (ref_rows < 1 || uref_rows < 1) return fail(RMPC_EINVAL, "empty reference arrays");
    if (p->precision != RMPC_F64 && p->precision != RMPC_F32)
        return fail(RMPC_EINVAL, "precision %d is neither RMPC_F64 nor RMPC_F32", p->precision);
    if (!(p->dt > 0) || !(p->slack_penalty >= 0) || !(p->R[0] > 0) || !(p->R[1] > 0))
        return fail(RMPC_EINVAL, "dt, R must be > 0 and slack_penalty >= 0");
    return RMPC_OK;
}

static MpcDevParams to_dev(const RmpcMpcParams *p) {
    MpcDevParams d;
    for (int i = 0; i < 3; i++) { d.Q[i] = p->Q[i]; d.P[i] = p->P[i]; }
    d.R[0] = p->R[0];
    d.R[1] = p->R[1];
    d.d_safe = p->d_safe;
    d.rho = p->slack_penalty;
    d.v_max = p->v_max;
    d.omega_max = p->omega_max;
    d.dt = p->dt;
    d.ltv = p->formulation == RMPC_LTV;
    d.soft = p->soft;
    d.max_iter = p->max_iter > 0 ? p->max_iter : 64;
    d.ramp_up_steps = p->ramp_up_steps > 0 ? p->ramp_up_steps : 10;
    d.ref_off = nullptr;
    return d;
}

static LqrDevParams to_dev(const RmpcLqrParams *p) {
    LqrDevParams d;
    for (int i = 0; i < 3; i++) d.Q[i] = p->Q[i];
    d.R[0] = p->R[0];
    d.R[1] = p->R[1];
    d.dt = p->dt;
    d.v_max = p->v_max;
    d.omega_max = p->omega_max;
    d.max_iter = p->max_iter > 0 ? p->max_iter : 64;
    d.use_cache = p->use_cache;
    d.ref_off = nullptr;
    return d;
}

static RiskDevParams to_dev(const RmpcRiskParams *p) {
    RiskDevParams d;
    d.d_safe = p->d_safe;
    d.d_trigger = p->d_trigger;
    d.alpha = p->alpha;
    d.beta = p->beta;
    d.th_low = p->threshold_low;
    d.th_med = p->threshold_medium;
    d.th_high = p->threshold_high;
    d.min_dwell = p->min_dwell_steps;
    d.use_pred = p->use_predicted;
    return d;
}

static hipError_t ensure_ws(RmpcCtx *c, const MpcLayout &L, int64_t B) {
    const size_t waves = (size_t)((B + RMPC_WAVE_LANES - 1) / RMPC_WAVE_LANES);
    return c->ws.ensure(waves * (size_t)L.REC * RMPC_WAVE_LANES * sizeof(double));
}

// The side stream for a pipeline's independent branch (config 4's refinement, config 5's LQR
// branch): one per context, created on first use.  (One stream shared by all contexts of a
// device serialised the batches in flight through its FIFO order: config 5 fell from ~400M to
// 233M steps/s.)
static hipError_t side_stream(RmpcCtx *c) {
    if (c->side) return hipSuccess;
    const hipError_t e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
    if (e != hipSuccess) c->side = nullptr;
    return e;
}

// Stream order between consecutive stateful calls of one context (RmpcCtx::last_ev): a call
// on another stream than the previous one waits for the previous call's end on the device.
static hipError_t order_calls(RmpcCtx *c, hipStream_t s) {
    if (c->last_valid && c->last_s != s) return hipStreamWaitEvent(s, c->last_ev, 0);
    return hipSuccess;
}
static hipError_t mark_call(RmpcCtx *c, hipStream_t s) {
    if (!c->last_ev) {
        const hipError_t e = hipEventCreateWithFlags(&c->last_ev, hipEventDisableTiming);
        if (e != hipSuccess) { c->last_ev = nullptr; return e; }
    }
    const hipError_t e = hipEventRecord(c->last_ev, s);
    c->last_valid = e == hipSuccess;
    c->last_s = s;
    return e;
}

// The context's own stream (host-pointer entry points), created on first use; NULL (the null
// stream) if creation fails
static hipStream_t own(RmpcCtx *c) {
    if (!c->stream && hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) c->stream = nullptr;
    return c->stream;
}

// _dev entry points run on the caller's stream; NULL is the null (default) stream, as in
// HIP itself -- so torch's default stream (handle 0) works unchanged.
static hipStream_t pick(RmpcCtx *, void *s) { return (hipStream_t)s; }

// RMPC_DEBUG_SYNC=1: synchronise after each kernel of a solve and report (diagnostics)
static void dbg_sync(hipStream_t s, const char *what) {
    static const bool on = rmpc_knob("RMPC_DEBUG_SYNC") != nullptr;
    if (!on) return;
    const hipError_t e = hipStreamSynchronize(s);
    fprintf(stderr, "[rmpc] %s done: %s\n", what, hipGetErrorString(e));
}

// The context's current list-counter set, at zero before a pipeline appends to it: a fill
// launch only when the previous pipeline did not zero it (the generic kernel's MpcArgs::
// zero_next).  A pipeline that zeroes the other set calls flip_counts once that launch is
// enqueued.
static hipError_t take_counts(RmpcCtx *c, hipStream_t s, int32_t **cnt) {
    hipError_t e = c->retry_count.ensure(64 * sizeof(int32_t));
    if (e != hipSuccess) return e;
    const int k = c->count_set;
    *cnt = (int32_t *)c->retry_count.p + 32 * k;
    if (!c->counts_zero[k]) {
        e = hipMemsetAsync(*cnt, 0, RMPC_COUNT_WORDS * sizeof(int32_t), s);
        if (e != hipSuccess) return e;
    }
    c->counts_zero[k] = false;
    return hipSuccess;
}
static int32_t *other_counts(RmpcCtx *c) { return (int32_t *)c->retry_count.p + 32 * (1 - c->count_set); }
static void flip_counts(RmpcCtx *c) {
    c->counts_zero[1 - c->count_set] = true;
    c->count_set = 1 - c->count_set;
}

// Launch the MPC solve for B robots (or the robots of a device-side index list): the
// register-resident lane-per-robot kernel when (N, block size) is instantiated; the robots
// it does not certify within its PDAS cap go to the lane-group tail, and what
// that one hands on (non-finite data -> fallback law, uncertified) to the generic kernel.
// Otherwise the generic kernel alone.
size_t rmpc_kernel_static_lds(const void *fn) {
    static std::mutex mu;
    static std::vector<std::pair<const void *, size_t>> cache;
    std::lock_guard<std::mutex> lk(mu);
    for (const auto &e : cache)
        if (e.first == fn) return e.second;
    hipFuncAttributes at;
    const size_t v = hipFuncGetAttributes(&at, fn) == hipSuccess ? at.sharedSizeBytes : RMPC_LDS_SLOT;
    cache.emplace_back(fn, v);
    return v;
}

// the tail launch site `k`'s hint (RmpcCtx::tail_hint_h): its device word and last length
enum { TAIL_SITE_MAIN = 0, TAIL_SITE_REFINE = 1, TAIL_SITE_COLD = 2, TAIL_SITE_GENERIC = 3,
       TAIL_SITE_GENERIC_COLD = 4, TAIL_SITES = 8 };
static hipError_t tail_hint(RmpcCtx *c, int k, int32_t **dev, int *prev) {
    if (!c->tail_hint_h) {
        hipError_t e = hipHostMalloc((void **)&c->tail_hint_h, TAIL_SITES * sizeof(int32_t),
                                     hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) { c->tail_hint_h = nullptr; return e; }
        for (int i = 0; i < TAIL_SITES; i++) c->tail_hint_h[i] = -1;
        e = hipHostGetDevicePointer((void **)&c->tail_hint_d, c->tail_hint_h, 0);
        if (e != hipSuccess) { (void)hipHostFree(c->tail_hint_h); c->tail_hint_h = nullptr; return e; }
    }
    *dev = c->tail_hint_d + k;
    const int32_t v = __atomic_load_n(c->tail_hint_h + k, __ATOMIC_RELAXED);
#if RMPC_HINT_LAST
    *prev = v;
#else
    // a decaying maximum (1/8 per launch) of the lengths the launches at this site wrote: a
    // list that fluctuates from call to call (closed loops) keeps the grid of its longer calls,
    // where the last length alone left rounds of two on the critical path
    int32_t &e = c->tail_est[k];
    if (v >= 0) e = e < 0 ? v : (v > e - e / 8 ? v : e - e / 8);
    *prev = e;
#endif
    return hipSuccess;
}

static int launch_mpc_impl(RmpcCtx *c, const RmpcMpcParams *p, int64_t B, const double *x0,
                      const double *x_refs, int32_t ref_rows, const double *u_refs, int32_t uref_rows,
                      const double *obstacles, int32_t n_obs, int32_t *step_count, double *u0,
                      double *u_seq, double *x_pred, double *cost, int32_t *status, uint8_t *slack_used,
                      int32_t *iters, const int32_t *index, const int32_t *count, hipStream_t s,
                      const int32_t *ref_off = nullptr, int fast_cap = 0, int warm_shift = 0) {
    const int bs = p->formulation == RMPC_LTV ? p->block_size : 1;
    const MpcLayout L = rmpc_mpc_layout(p->horizon, bs, n_obs);
    HIP_TRY(ensure_ws(c, L, B));
    MpcDevParams d = to_dev(p);
    const bool lti = p->formulation == RMPC_LTI;
    d.ref_off = ref_off;
    // hard half-spaces (soft = 0 with obstacles): augmented-Lagrangian rounds in the generic kernel
    const bool hard = !p->soft && n_obs > 0;
    // An fp32 request (BASELINE config 4) computes in fp32 only where an fp64 pass re-solves and
    // re-certifies the fp32 pass's active sets: the soft LTV lane-per-robot instances with a
    // refinement pass (N = 20, and N = 30 with 8 obstacles).  Every other fp32 request runs the
    // fp64 pipeline, so every control an fp32 request returns is the fp64 optimum.
    const bool f32 = p->precision == RMPC_F32 && !lti && !hard && rmpc_mpc_refine_supported(p->horizon, bs, n_obs);
    const int prec = f32 ? RMPC_F32 : RMPC_F64;
    const bool fast = !hard && rmpc_mpc_fast_supported(p->horizon, bs, prec, lti, n_obs) &&
                      !rmpc_knob("RMPC_DISABLE_FAST");
    // fp64 without a lane-per-robot instance -- LTI (MPCController.solve, mpc_node's path),
    // or an LTV (N, block size) the fast kernel is not built for (N = 30) -- every robot
    // through the lane-group kernel from a cold start (RMPC_LTI_GENERIC=1: the generic kernel
    // alone), what it does not certify through the LDS generic kernel
    const bool lti_group = !fast && !f32 && !hard && !rmpc_knob("RMPC_LTI_GENERIC") &&
                           rmpc_mpc_group_supported(p->horizon, lti ? 1 : bs, n_obs);
    if (lti_group) {
        HIP_TRY(c->retry.ensure((size_t)B * sizeof(int32_t)));
        HIP_TRY(c->retry2.ensure((size_t)B * sizeof(int32_t)));
        int32_t *cnt = nullptr;
        HIP_TRY(take_counts(c, s, &cnt));
        const int32_t *list = index, *list_n = count;
        if (!index) {                                      // the whole batch: 0..B-1
            HIP_TRY(rmpc_launch_iota(B, (int32_t *)c->retry.p, cnt, s));
            list = (const int32_t *)c->retry.p;
            list_n = cnt;
        }
        int32_t *cnt2 = cnt + 8;
        const int cap = 11;
        int32_t *hint_d = nullptr;
        int hint_p = -1;
        HIP_TRY(tail_hint(c, TAIL_SITE_COLD, &hint_d, &hint_p));
        HIP_TRY(rmpc_launch_mpc_group(d, p->horizon, lti ? 1 : bs, n_obs, B, x0, x_refs, ref_rows, u_refs,
                                      uref_rows, obstacles, step_count, u0, u_seq, x_pred, cost, status, slack_used,
                                      iters, list, list_n, (int32_t *)c->retry2.p, cnt2, cap, nullptr, s, nullptr,
                                      lti, &c->gdiag, nullptr, 0, hint_d, hint_p));
        dbg_sync(s, "group (cold)");
        int32_t *ghint_d = nullptr;
        int ghint_p = -1;
        HIP_TRY(tail_hint(c, TAIL_SITE_GENERIC_COLD, &ghint_d, &ghint_p));
        HIP_TRY(rmpc_launch_mpc_f64(d, L, B, x0, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs,
                                    step_count, u0, u_seq, x_pred, cost, status, slack_used, iters,
                                    c->ws.p, (const int32_t *)c->retry2.p, cnt2, s, rmpc_mpc_lds_lanes(L),
                                    other_counts(c), ghint_d, ghint_p));
        if (B > 0) flip_counts(c);
        return RMPC_OK;
    }
    if (!fast && f32)                      // fp32 arithmetic: the generic kernel on a float record
        HIP_TRY(rmpc_launch_mpc_f32(d, L, B, x0, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs,
                                    step_count, u0, u_seq, x_pred, cost, status, slack_used, iters,
                                    c->ws.p, index, count, s));
    else if (!fast)
        HIP_TRY(rmpc_launch_mpc_f64(d, L, B, x0, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs,
                                    step_count, u0, u_seq, x_pred, cost, status, slack_used, iters,
                                    c->ws.p, index, count, s));
    else {
        const int nb = (p->horizon + bs - 1) / bs;
        const size_t waves = (size_t)((B + RMPC_WAVE_LANES - 1) / RMPC_WAVE_LANES);
        HIP_TRY(c->fast_gains.ensure(waves * nb * 4 * RMPC_WAVE_LANES * sizeof(double2)));
        HIP_TRY(c->retry.ensure((size_t)B * sizeof(int32_t)));
        int32_t *cnt = nullptr;
        HIP_TRY(take_counts(c, s, &cnt));
        MpcFastArgs a;
        memset(&a, 0, sizeof(a));
        a.prm = d;
        a.B = B;
        a.x0 = x0; a.x_refs = x_refs; a.u_refs = u_refs;
        a.ref_rows = ref_rows; a.uref_rows = uref_rows; a.no = n_obs;
        a.obs = obstacles;
        a.step_count = step_count;
        a.u0 = u0; a.u_seq = u_seq; a.x_pred = x_pred; a.cost = cost;
        a.status = status; a.iters = iters; a.slack_used = slack_used;
        a.gains = (double2 *)c->fast_gains.p;
        a.index = index;
        a.count = count;
        a.retry = (int32_t *)c->retry.p;
        a.retry_count = cnt;
        // default cap (sweeps with the lane-group tail): 7 at N <= 20 (BASELINE config 3; 9 for
        // LTI, whose harder instances would otherwise overfill the tail), 12 beyond (config 4)
        // (fast_cap: the caller's choice, e.g. the hybrid switch's MPC branch)
        a.pdas_cap = rmpc_knob("RMPC_FAST_CAP") ? atoi(rmpc_knob("RMPC_FAST_CAP"))
                     : fast_cap > 0           ? fast_cap
                     : c->fast_cap > 0        ? c->fast_cap
                                              : (p->horizon <= 20 ? (lti ? 9 : 7) : 12);
        a.init_zc = c->cold_rows ? 1 : 0;  // rmpc_ctx_set_cold_start
        a.lanes = c->lanes;                // rmpc_ctx_set_lanes_per_robot
        // the tail continues from each handed-on robot's sets (retry_sets)
        HIP_TRY(c->retry_sets.ensure((size_t)B * (p->horizon + nb + 1) * sizeof(uint32_t)));
        a.retry_sets = (uint32_t *)c->retry_sets.p;
        // warm start across calls (rmpc_ctx_set_warm_start; warm_shift steps since the previous
        // call): the robots' previous certified sets, used by a robot whose last solve was the
        // previous call (stamps; the hybrid step's MPC branch takes a different subset each
        // step), zero (= the cold start) whenever the batch shape differs from the previous call's
        if (c->warm_on && warm_shift > 0) {
            const size_t words = (size_t)B * (size_t)(p->horizon + nb + 1);
            const int64_t key = (int64_t)p->horizon | (int64_t)nb << 8 | (int64_t)n_obs << 16 |
                                (int64_t)lti << 24 | (int64_t)f32 << 25;
            HIP_TRY(c->warm_sets.ensure(words * sizeof(uint32_t)));
            if (c->warm_B != B || c->warm_key != key) {
                HIP_TRY(hipMemsetAsync(c->warm_sets.p, 0, words * sizeof(uint32_t), s));
                c->warm_B = B;
                c->warm_key = key;
                c->warm_calls = 0;
            }
            a.prev_sets = (uint32_t *)c->warm_sets.p;
            a.prev_shift = warm_shift;
            a.prev_stamp = ++c->warm_calls;
            // From warm sets most robots certify in their first or second solve, and a robot
            // still iterating after a few is one of the few hard ones: the tail's lane groups
            // take it sooner.  fp64 LTV at N <= 20: 2 after a one-step shift (config-3 closed
            // loop, 65536 robots: 191M -> 274M solves/s, three fleets in flight 410M -> 498M), 4
            // after a longer one (mpc_rate 5: 178M -> 210M, three fleets 299M -> 315M; cap 2 there
            // gave 169M / 248M); fp32 requests: 4 for the fp32 pass (config-4 closed loop, 32768
            // robots: 43.6M -> 64.2M, three fleets 61.6M -> 91.1M)
            // (profiles/r03/closed_loop_warm.txt).  The caller's caps win.
            // (Not on the first call after a reset, whose sets are all zero: a cold start, which
            // keeps the cold default.)
            if (!rmpc_knob("RMPC_FAST_CAP") && fast_cap <= 0 && c->fast_cap <= 0 && !lti && c->warm_calls > 1) {
                if (f32) a.pdas_cap = 4;
                else if (p->horizon <= 20) a.pdas_cap = warm_shift == 1 ? 2 : 4;
            }
        }
        // RMPC_DENSE_PROF=1: per-phase cycle counters of the fast and lane-group kernels to
        // stderr (synchronises the stream; diagnostics only)
        const bool prof = rmpc_knob("RMPC_DENSE_PROF") != nullptr;
        unsigned long long *pc = nullptr;
        if (prof) {
            HIP_TRY(c->prof.ensure(128 * sizeof(unsigned long long)));   // [64..127]: the refinement pass
            pc = (unsigned long long *)c->prof.p;
            HIP_TRY(hipMemsetAsync(pc, 0, 128 * sizeof(unsigned long long), s));
        }
        a.prof = pc;
        // Mixed precision for fp32 requests (BASELINE config 4): the fp32 lane-per-robot pass
        // only finds the active sets.  Every robot it certifies goes on, with its sets, to an
        // fp64 pass of the same kernel that re-solves the equality-constrained QP of those sets
        // in fp64, re-checks them (KKT) and continues PDAS from them if they change (up to
        // `extra_cap` solves); it writes the outputs, which are therefore fp64-exact.  What it
        // does not certify joins the fp64 tail's list.
        const bool refine = f32;
        if (refine) {
            HIP_TRY(c->refine.ensure((size_t)B * sizeof(int32_t)));
            HIP_TRY(c->refine_sets.ensure((size_t)B * (p->horizon + nb + 1) * sizeof(uint32_t)));
            a.refine = (int32_t *)c->refine.p;
            a.refine_count = cnt + 6;
            a.refine_sets = (uint32_t *)c->refine_sets.p;
        }
        if (c->timing) HIP_TRY(hipEventRecord(c->ev[0], s));
        // Multi-pass stage: pass i runs its robots for up to caps[i] PDAS solves in total and
        // hands the uncertified ones on, with their sets and iteration counts, to a compacted
        // list; the next pass continues exactly there (MpcFastArgs::warm_sets), so the iterate
        // path is the one-pass path and only the packing of robots into waves changes: a later
        // pass's waves hold no robot that has already certified.  The last pass runs to the
        // stage cap and hands on to the tail.
        int caps[2], ncap = 0;
        for (int i = 0; i < 2; i++)
            if (c->passes[i] > (ncap ? caps[ncap - 1] : 0) && c->passes[i] < a.pdas_cap) caps[ncap++] = c->passes[i];
        if (const char *sp = rmpc_knob("RMPC_FAST_SPLIT")) {   // (A/B: "c1[,c2]", "0" = one pass)
            ncap = 0;
            for (const char *q = sp; *q && ncap < 2;) {
                const int v = atoi(q);
                if (v > (ncap ? caps[ncap - 1] : 0) && v < a.pdas_cap) caps[ncap++] = v;
                while (*q && *q != ',') q++;
                if (*q == ',') q++;
            }
        }
        for (int i = 0; i < ncap; i++) {
            HIP_TRY(c->pass_list[i].ensure((size_t)B * sizeof(int32_t)));
            HIP_TRY(c->pass_sets[i].ensure((size_t)B * (p->horizon + nb + 1 + RMPC_REC_HIST) * sizeof(uint32_t)));
            MpcFastArgs ai = a;
            ai.pdas_cap = caps[i];
            ai.retry = (int32_t *)c->pass_list[i].p;
            ai.retry_count = cnt + 2 + i;
            ai.retry_sets = (uint32_t *)c->pass_sets[i].p;
            ai.rec_hist = 1;               // records with the cycle history; cycling robots to the tail
            ai.cyc = a.retry;
            ai.cyc_count = a.retry_count;
            ai.cyc_sets = a.retry_sets;
            HIP_TRY(rmpc_launch_mpc_fast(ai, p->horizon, bs, prec, s, lti));
            dbg_sync(s, "fast pass");
            a.index = ai.retry;            // the next pass: that list, from its sets and history
            a.count = ai.retry_count;
            a.warm_sets = ai.retry_sets;
            a.warm_hist = 1;
        }
        HIP_TRY(rmpc_launch_mpc_fast(a, p->horizon, bs, prec, s, lti));
        // tail: the lane-group Riccati kernel (RMPC_DISABLE_DENSE: no tail stage, A/B only)
        const bool group_tail = rmpc_mpc_group_supported(p->horizon, bs, n_obs) && !rmpc_knob("RMPC_DISABLE_DENSE");
        // The refinement and the tail work on disjoint robots (the fp32 pass's certified ones
        // and the rest): the refinement runs on the side stream while the tail runs here, and
        // the robots it hands on get a second, short tail launch after the join
        const bool refine_side = refine && group_tail && c->use_side;
        // Everything the side branch and the tails use is allocated before the fork, and every
        // error after the fork joins the side branch first (`join`): the call's stream must
        // never complete ahead of a refinement kernel that is still writing outputs.
        if (group_tail) HIP_TRY(c->retry2.ensure((size_t)B * sizeof(int32_t)));
        int32_t *hint_d[2] = {nullptr, nullptr};
        int hint_p[2] = {-1, -1};
        if (group_tail) {
            HIP_TRY(tail_hint(c, TAIL_SITE_MAIN, &hint_d[0], &hint_p[0]));
            HIP_TRY(tail_hint(c, TAIL_SITE_REFINE, &hint_d[1], &hint_p[1]));
        }
        if (refine_side) {
            HIP_TRY(side_stream(c));
            for (auto &e : c->rev)
                if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            HIP_TRY(c->retry_r.ensure((size_t)B * sizeof(int32_t)));
            HIP_TRY(c->retry_sets_r.ensure((size_t)B * (p->horizon + nb + 1) * sizeof(uint32_t)));
        }
        bool forked = false;
        auto join = [&]() -> hipError_t {    // side branch -> call's stream (host sync as a last resort)
            if (!forked) return hipSuccess;
            forked = false;
            hipError_t e = hipEventRecord(c->rev[1], c->side);
            if (e == hipSuccess) e = hipStreamWaitEvent(s, c->rev[1], 0);
            if (e != hipSuccess) (void)hipStreamSynchronize(c->side);
            return e;
        };
#define HIP_TRY_J(expr)                      \
    do {                                     \
        const hipError_t ej_ = (expr);       \
        if (ej_ != hipSuccess) {             \
            (void)join();                    \
            HIP_TRY(ej_);                    \
        }                                    \
    } while (0)
        if (refine) {
            dbg_sync(s, "fast (fp32 sets)");
            MpcFastArgs r = a;
            r.refine = nullptr; r.refine_count = nullptr; r.refine_sets = nullptr;
            r.index = a.refine;
            r.count = a.refine_count;
            r.warm_sets = a.refine_sets;
            r.warm_hist = 0;               // (refinement records carry no cycle history)
            // one fp64 solve from the fp32 sets: the robots whose sets it does not certify go
            // to the fp64 tail (config 4: 36.5M against 34.8M solves/s with 4 more solves here,
            // whose slowest waves set the pass's length)
            r.extra_cap = 1;
            r.prof = pc ? pc + 64 : nullptr;   // (diagnostics: the refinement pass's own counters)
            hipStream_t rs = s;
            if (refine_side) {
                r.retry = (int32_t *)c->retry_r.p;
                r.retry_count = cnt + 10;
                r.retry_sets = (uint32_t *)c->retry_sets_r.p;
                HIP_TRY(hipEventRecord(c->rev[0], s));
                HIP_TRY(hipStreamWaitEvent(c->side, c->rev[0], 0));
                forked = true;
                rs = c->side;
            }
            HIP_TRY_J(rmpc_launch_mpc_fast(r, p->horizon, bs, RMPC_F64, rs, lti));
        }
        if (c->timing) HIP_TRY_J(hipEventRecord(c->ev[1], s));
        dbg_sync(s, "fast");
        const int32_t *left = (const int32_t *)c->retry.p;
        const int32_t *left_n = cnt;
        // tail PDAS cap before projected Newton (sweeps: 4 at N <= 20, 6 beyond -- config 4)
        const int tail_cap = c->tail_cap > 0 ? c->tail_cap : (p->horizon <= 20 ? 4 : 6);
        // (a refined fp32 request takes the fp64 tail: it returns fp64 optima only)
        if (group_tail) {
            int32_t *cnt2 = cnt + 8;
            HIP_TRY_J(rmpc_launch_mpc_group(d, p->horizon, bs, n_obs, B, x0, x_refs, ref_rows, u_refs, uref_rows,
                                            obstacles, step_count, u0, u_seq, x_pred, cost, status, slack_used,
                                            iters, left, left_n, (int32_t *)c->retry2.p, cnt2, tail_cap,
                                            a.retry_sets, s, pc, lti, &c->gdiag, a.prev_sets, a.prev_stamp,
                                            hint_d[0], hint_p[0]));
            HIP_TRY(join());               // the refinement, before anything else on this stream
#undef HIP_TRY_J
            if (refine_side) {            // the refinement's hand-ons (same output list)
                HIP_TRY(rmpc_launch_mpc_group(d, p->horizon, bs, n_obs, B, x0, x_refs, ref_rows, u_refs, uref_rows,
                                              obstacles, step_count, u0, u_seq, x_pred, cost, status, slack_used,
                                              iters, (const int32_t *)c->retry_r.p, cnt + 10, (int32_t *)c->retry2.p,
                                              cnt2, tail_cap, (const uint32_t *)c->retry_sets_r.p, s, pc, lti,
                                              &c->gdiag, a.prev_sets, a.prev_stamp, hint_d[1], hint_p[1]));
            }
            if (prof) HIP_TRY(rmpc_diag_print_stage_prof(pc, cnt, refine, s));
            dbg_sync(s, "group");
            left = (const int32_t *)c->retry2.p;
            left_n = cnt2;
        }
        if (c->timing) HIP_TRY(hipEventRecord(c->ev[2], s));
        // what remains is rare (cycling beyond both, non-finite data): LDS generic kernel, in
        // the requested arithmetic (the lane-group tail between is fp64 for both)
        // (a refined fp32 request stays fp64 here too: every output it returns is the fp64 optimum)
        int32_t *ghint_d = nullptr;
        int ghint_p = -1;
        HIP_TRY(tail_hint(c, TAIL_SITE_GENERIC, &ghint_d, &ghint_p));
        HIP_TRY(rmpc_launch_mpc_f64(d, L, B, x0, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs,
                                        step_count, u0, u_seq, x_pred, cost, status, slack_used, iters,
                                        c->ws.p, left, left_n, s, rmpc_mpc_lds_lanes(L), other_counts(c),
                                        ghint_d, ghint_p));
        if (B > 0) flip_counts(c);         // (the next pipeline takes the set zeroed there)
        if (c->timing) {
            HIP_TRY(hipEventRecord(c->ev[3], s));
            c->timed = true;
        }
        dbg_sync(s, "generic");
    }
    return RMPC_OK;
}

static int launch_mpc(RmpcCtx *c, const RmpcMpcParams *p, int64_t B, const double *x0,
                      const double *x_refs, int32_t ref_rows, const double *u_refs, int32_t uref_rows,
                      const double *obstacles, int32_t n_obs, int32_t *step_count, double *u0,
                      double *u_seq, double *x_pred, double *cost, int32_t *status, uint8_t *slack_used,
                      int32_t *iters, const int32_t *index, const int32_t *count, hipStream_t s,
                      const int32_t *ref_off = nullptr, int fast_cap = 0, int warm_shift = 0) {
    HIP_TRY(order_calls(c, s));
    const int rc = launch_mpc_impl(c, p, B, x0, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs, step_count, u0,
                                   u_seq, x_pred, cost, status, slack_used, iters, index, count, s, ref_off, fast_cap,
                                   warm_shift);
    HIP_TRY(mark_call(c, s));
    return rc;
}

// stage a host array to the device (returns device pointer or nullptr when src is null)
template <typename T>
static int h2d(RmpcCtx *c, int slot, const T *src, size_t n, T **dst) {
    if (!src) { *dst = nullptr; return RMPC_OK; }
    HIP_TRY(c->stage[slot].ensure(align_up(n * sizeof(T), 256)));
    HIP_TRY(hipMemcpyAsync(c->stage[slot].p, src, n * sizeof(T), hipMemcpyHostToDevice, own(c)));
    *dst = (T *)c->stage[slot].p;
    return RMPC_OK;
}

template <typename T>
static int dalloc(RmpcCtx *c, int slot, const T *host, size_t n, T **dst) {
    if (!host) { *dst = nullptr; return RMPC_OK; }
    HIP_TRY(c->stage[slot].ensure(align_up(n * sizeof(T), 256)));
    *dst = (T *)c->stage[slot].p;
    return RMPC_OK;
}

template <typename T>
static int d2h(RmpcCtx *c, T *host, const T *dev, size_t n) {
    if (!host) return RMPC_OK;
    HIP_TRY(hipMemcpyAsync(host, dev, n * sizeof(T), hipMemcpyDeviceToHost, own(c)));
    return RMPC_OK;
}

#define RC(x)                           \
    do {                                \
        int rc_ = (x);                  \
        if (rc_ != RMPC_OK) return rc_; \
    } while (0)

// ------------------------------------------------------------------------------ MPC
extern "C" int rmpc_mpc_solve_batch_dev(RmpcCtx *c, const RmpcMpcParams *p, int64_t B, const double *x0,
                                        const double *x_refs, int32_t ref_rows, const double *u_refs,
                                        int32_t uref_rows, const double *obstacles, int32_t n_obs,
                                        int32_t *step_count, double *u0, double *u_seq, double *x_pred,
                                        double *cost, int32_t *status, uint8_t *slack_used, int32_t *iters,
                                        void *stream) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    if (!c->sub.empty()) return fail(RMPC_ENOTSUP, "device-pointer entry points take a single-device context");
    RC(check_mpc_params(p, ref_rows, uref_rows, n_obs));
    if (B < 0) return fail(RMPC_EINVAL, "B < 0");
    if (B == 0) return RMPC_OK;
    if (!x0 || !x_refs || !u_refs || !u0 || !status || (n_obs > 0 && !obstacles))
        return fail(RMPC_EINVAL, "required pointer is NULL");
    HIP_TRY(hipSetDevice(c->device));
    return launch_mpc(c, p, B, x0, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs, step_count, u0,
                      u_seq, x_pred, cost, status, slack_used, iters, nullptr, nullptr, pick(c, stream), nullptr, 0,
                      1);
}

extern "C" int rmpc_mpc_solve_batch(RmpcCtx *c, const RmpcMpcParams *p, int64_t B, const double *x0,
                                    const double *x_refs, int32_t ref_rows, const double *u_refs,
                                    int32_t uref_rows, const double *obstacles, int32_t n_obs,
                                    int32_t *step_count, double *u0, double *u_seq, double *x_pred,
                                    double *cost, int32_t *status, uint8_t *slack_used, int32_t *iters) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    RC(check_mpc_params(p, ref_rows, uref_rows, n_obs));
    if (B < 0) return fail(RMPC_EINVAL, "B < 0");
    if (B == 0) return RMPC_OK;
    if (!x0 || !x_refs || !u_refs || !u0 || !status || (n_obs > 0 && !obstacles))
        return fail(RMPC_EINVAL, "required pointer is NULL");
    const int N = p->horizon;
    if (!c->sub.empty())
        return multi_run(c, B,
                         {{(void *)x0, 24, true, false}, {(void *)x_refs, (size_t)ref_rows * 24, true, false},
                          {(void *)u_refs, (size_t)uref_rows * 16, true, false}, {step_count, 4, true, true},
                          {u0, 16, false, true}, {u_seq, (size_t)N * 16, false, true},
                          {x_pred, (size_t)(N + 1) * 24, false, true}, {cost, 8, false, true},
                          {status, 4, false, true}, {slack_used, 1, false, true}, {iters, 4, false, true}},
                         [&](RmpcCtx *sc, int64_t b, void **q) {
                             return rmpc_mpc_solve_batch(sc, p, b, (const double *)q[0], (const double *)q[1], ref_rows,
                                                         (const double *)q[2], uref_rows, obstacles, n_obs,
                                                         (int32_t *)q[3], (double *)q[4], (double *)q[5],
                                                         (double *)q[6], (double *)q[7], (int32_t *)q[8],
                                                         (uint8_t *)q[9], (int32_t *)q[10]);
                         });
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    {
        // Small batches (a drop-in MPCController: one robot per call): one pinned block and one
        // copy each way instead of a pageable copy per array (thirteen).  Layout: inputs, the
        // in/out step counts, outputs; absent optional arrays take no room and stay NULL.
        size_t off = 0;
        auto at = [&](size_t bytes) { const size_t o = off; off += align_up(bytes, 256); return o; };
        const size_t o_x0 = at((size_t)B * 24), o_xr = at((size_t)B * ref_rows * 24), o_ur = at((size_t)B * uref_rows * 16),
                     o_ob = at((size_t)n_obs * 24), o_sc = at(step_count ? (size_t)B * 4 : 0), o_u0 = at((size_t)B * 16),
                     o_us = at(u_seq ? (size_t)B * N * 16 : 0), o_xp = at(x_pred ? (size_t)B * (N + 1) * 24 : 0),
                     o_co = at(cost ? (size_t)B * 8 : 0), o_st = at((size_t)B * 4), o_sl = at(slack_used ? (size_t)B : 0),
                     o_it = at(iters ? (size_t)B * 4 : 0);
        if (off <= RMPC_PACK_MAX) {
            if (c->pin_cap < off) {
                if (c->pin) (void)hipHostFree(c->pin);
                c->pin = nullptr;
                c->pin_cap = 0;
                HIP_TRY(hipHostMalloc(&c->pin, align_up(off, 65536), hipHostMallocDefault));
                c->pin_cap = align_up(off, 65536);
            }
            HIP_TRY(c->pack.ensure(off));
            char *h = (char *)c->pin, *d = (char *)c->pack.p;
            memcpy(h + o_x0, x0, (size_t)B * 24);
            memcpy(h + o_xr, x_refs, (size_t)B * ref_rows * 24);
            memcpy(h + o_ur, u_refs, (size_t)B * uref_rows * 16);
            if (n_obs > 0) memcpy(h + o_ob, obstacles, (size_t)n_obs * 24);
            if (step_count) memcpy(h + o_sc, step_count, (size_t)B * 4);
            auto dp = [&](const void *user, size_t o) { return user ? (void *)(d + o) : nullptr; };
            // once the first copy is queued, every exit waits for the stream: a copy still
            // reading the pinned block must not meet the next call's writes (or its regrowth)
            const int rc = [&]() -> int {
                HIP_TRY(hipMemcpyAsync(d, h, o_u0, hipMemcpyHostToDevice, own(c)));
                RC(rmpc_mpc_solve_batch_dev(c, p, B, (const double *)(d + o_x0), (const double *)(d + o_xr), ref_rows,
                                            (const double *)(d + o_ur), uref_rows,
                                            n_obs > 0 ? (const double *)(d + o_ob) : nullptr, n_obs,
                                            (int32_t *)dp(step_count, o_sc), (double *)(d + o_u0),
                                            (double *)dp(u_seq, o_us), (double *)dp(x_pred, o_xp),
                                            (double *)dp(cost, o_co), (int32_t *)(d + o_st),
                                            (uint8_t *)dp(slack_used, o_sl), (int32_t *)dp(iters, o_it), own(c)));
                HIP_TRY(hipMemcpyAsync(h + o_sc, d + o_sc, off - o_sc, hipMemcpyDeviceToHost, own(c)));
                return RMPC_OK;
            }();
            const hipError_t es = hipStreamSynchronize(own(c));
            if (rc != RMPC_OK) return rc;
            HIP_TRY(es);
            if (step_count) memcpy(step_count, h + o_sc, (size_t)B * 4);
            memcpy(u0, h + o_u0, (size_t)B * 16);
            if (u_seq) memcpy(u_seq, h + o_us, (size_t)B * N * 16);
            if (x_pred) memcpy(x_pred, h + o_xp, (size_t)B * (N + 1) * 24);
            if (cost) memcpy(cost, h + o_co, (size_t)B * 8);
            memcpy(status, h + o_st, (size_t)B * 4);
            if (slack_used) memcpy(slack_used, h + o_sl, (size_t)B);
            if (iters) memcpy(iters, h + o_it, (size_t)B * 4);
            return RMPC_OK;
        }
    }
    double *dx0, *dxr, *dur, *dobs = nullptr, *du0, *duseq, *dxp, *dcost;
    int32_t *dstep, *dst, *dit;
    uint8_t *dsl;
    RC(h2d(c, SB_X0, x0, (size_t)B * 3, &dx0));
    RC(h2d(c, SB_XREF, x_refs, (size_t)B * ref_rows * 3, &dxr));
    RC(h2d(c, SB_UREF, u_refs, (size_t)B * uref_rows * 2, &dur));
    if (n_obs > 0) RC(h2d(c, SB_OBS, obstacles, (size_t)n_obs * 3, &dobs));
    RC(h2d(c, SB_STEP, step_count, (size_t)B, &dstep));
    RC(dalloc(c, SB_U0, u0, (size_t)B * 2, &du0));
    RC(dalloc(c, SB_USEQ, u_seq, (size_t)B * N * 2, &duseq));
    RC(dalloc(c, SB_XPRED, x_pred, (size_t)B * (N + 1) * 3, &dxp));
    RC(dalloc(c, SB_COST, cost, (size_t)B, &dcost));
    RC(dalloc(c, SB_STATUS, status, (size_t)B, &dst));
    RC(dalloc(c, SB_SLACK, slack_used, (size_t)B, &dsl));
    RC(dalloc(c, SB_ITERS, iters, (size_t)B, &dit));
    RC(rmpc_mpc_solve_batch_dev(c, p, B, dx0, dxr, ref_rows, dur, uref_rows, dobs, n_obs, dstep, du0,
                                duseq, dxp, dcost, dst, dsl, dit, own(c)));
    RC(d2h(c, u0, du0, (size_t)B * 2));
    RC(d2h(c, u_seq, duseq, (size_t)B * N * 2));
    RC(d2h(c, x_pred, dxp, (size_t)B * (N + 1) * 3));
    RC(d2h(c, cost, dcost, (size_t)B));
    RC(d2h(c, status, dst, (size_t)B));
    RC(d2h(c, slack_used, dsl, (size_t)B));
    RC(d2h(c, iters, dit, (size_t)B));
    RC(d2h(c, step_count, dstep, (size_t)B));
    HIP_TRY(hipStreamSynchronize(own(c)));
    return RMPC_OK;
}

// ------------------------------------------------------------------------------ LQR
static int check_lqr(const RmpcLqrParams *p) {
    if (!p) return fail(RMPC_EINVAL, "params is NULL");
    if (!(p->dt > 0) || !(p->R[0] > 0) || !(p->R[1] > 0)) return fail(RMPC_EINVAL, "dt, R must be > 0");
    return RMPC_OK;
}

extern "C" int rmpc_lqr_control_batch_dev(RmpcCtx *c, const RmpcLqrParams *p, int64_t B, const double *x,
                                          const double *x_ref, const double *u_ref, RmpcLqrCache *cache,
                                          double *u_out, double *err_out, double *K_out, double *P_out,
                                          int32_t *status, void *stream) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    if (!c->sub.empty()) return fail(RMPC_ENOTSUP, "device-pointer entry points take a single-device context");
    RC(check_lqr(p));
    if (B < 0) return fail(RMPC_EINVAL, "B < 0");
    if (B == 0) return RMPC_OK;
    if (!x || !x_ref || !u_ref || !u_out) return fail(RMPC_EINVAL, "required pointer is NULL");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(rmpc_launch_lqr_control(to_dev(p), B, x, x_ref, 3, u_ref, 2, cache, u_out, err_out, K_out,
                                    P_out, status, nullptr, nullptr, pick(c, stream)));
    return RMPC_OK;
}

extern "C" int rmpc_lqr_control_batch(RmpcCtx *c, const RmpcLqrParams *p, int64_t B, const double *x,
                                      const double *x_ref, const double *u_ref, RmpcLqrCache *cache,
                                      double *u_out, double *err_out, double *K_out, double *P_out,
                                      int32_t *status) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    RC(check_lqr(p));
    if (B < 0) return fail(RMPC_EINVAL, "B < 0");
    if (B == 0) return RMPC_OK;
    if (!x || !x_ref || !u_ref || !u_out) return fail(RMPC_EINVAL, "required pointer is NULL");
    if (!c->sub.empty())
        return multi_run(c, B,
                         {{(void *)x, 24, true, false}, {(void *)x_ref, 24, true, false}, {(void *)u_ref, 16, true, false},
                          {cache, sizeof(RmpcLqrCache), true, true}, {u_out, 16, false, true}, {err_out, 24, false, true},
                          {K_out, 48, false, true}, {P_out, 72, false, true}, {status, 4, false, true}},
                         [&](RmpcCtx *sc, int64_t b, void **q) {
                             return rmpc_lqr_control_batch(sc, p, b, (const double *)q[0], (const double *)q[1],
                                                           (const double *)q[2], (RmpcLqrCache *)q[3], (double *)q[4],
                                                           (double *)q[5], (double *)q[6], (double *)q[7],
                                                           (int32_t *)q[8]);
                         });
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    double *dx, *dxr, *dur, *du, *de, *dK, *dP;
    int32_t *dst;
    RmpcLqrCache *dc;
    RC(h2d(c, SB_X0, x, (size_t)B * 3, &dx));
    RC(h2d(c, SB_XREF, x_ref, (size_t)B * 3, &dxr));
    RC(h2d(c, SB_UREF, u_ref, (size_t)B * 2, &dur));
    RC(h2d(c, SB_CACHE, cache, (size_t)B, &dc));
    RC(dalloc(c, SB_U0, u_out, (size_t)B * 2, &du));
    RC(dalloc(c, SB_ERR, err_out, (size_t)B * 3, &de));
    RC(dalloc(c, SB_K, K_out, (size_t)B * 6, &dK));
    RC(dalloc(c, SB_P, P_out, (size_t)B * 9, &dP));
    RC(dalloc(c, SB_STATUS, status, (size_t)B, &dst));
    RC(rmpc_lqr_control_batch_dev(c, p, B, dx, dxr, dur, dc, du, de, dK, dP, dst, own(c)));
    RC(d2h(c, u_out, du, (size_t)B * 2));
    RC(d2h(c, err_out, de, (size_t)B * 3));
    RC(d2h(c, K_out, dK, (size_t)B * 6));
    RC(d2h(c, P_out, dP, (size_t)B * 9));
    RC(d2h(c, status, dst, (size_t)B));
    RC(d2h(c, cache, dc, (size_t)B));
    HIP_TRY(hipStreamSynchronize(own(c)));
    return RMPC_OK;
}

extern "C" int rmpc_lqr_gain_batch(RmpcCtx *c, const RmpcLqrParams *p, int64_t B, const double *v_r,
                                   const double *theta_r, int32_t guard_v, double *K_out, double *P_out,
                                   int32_t *status) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    RC(check_lqr(p));
    if (B < 0) return fail(RMPC_EINVAL, "B < 0");
    if (B == 0) return RMPC_OK;
    if (!v_r || !theta_r || !K_out) return fail(RMPC_EINVAL, "required pointer is NULL");
    if (!c->sub.empty())
        return multi_run(c, B,
                         {{(void *)v_r, 8, true, false}, {(void *)theta_r, 8, true, false}, {K_out, 48, false, true},
                          {P_out, 72, false, true}, {status, 4, false, true}},
                         [&](RmpcCtx *sc, int64_t b, void **q) {
                             return rmpc_lqr_gain_batch(sc, p, b, (const double *)q[0], (const double *)q[1], guard_v,
                                                        (double *)q[2], (double *)q[3], (int32_t *)q[4]);
                         });
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    double *dv, *dth, *dK, *dP;
    int32_t *dst;
    RC(h2d(c, SB_X0, v_r, (size_t)B, &dv));
    RC(h2d(c, SB_XREF, theta_r, (size_t)B, &dth));
    RC(dalloc(c, SB_K, K_out, (size_t)B * 6, &dK));
    RC(dalloc(c, SB_P, P_out, (size_t)B * 9, &dP));
    RC(dalloc(c, SB_STATUS, status, (size_t)B, &dst));
    HIP_TRY(rmpc_launch_lqr_gain(to_dev(p), B, dv, dth, guard_v, dK, dP, dst, own(c)));
    RC(d2h(c, K_out, dK, (size_t)B * 6));
    RC(d2h(c, P_out, dP, (size_t)B * 9));
    RC(d2h(c, status, dst, (size_t)B));
    HIP_TRY(hipStreamSynchronize(own(c)));
    return RMPC_OK;
}

// ------------------------------------------------------------------------------ risk / hybrid
extern "C" int rmpc_risk_batch(RmpcCtx *c, const RmpcRiskParams *rp, int64_t B, const double *x,
                               const double *pred, int32_t n_pred, const double *obstacles, int32_t n_obs,
                               double *out, uint8_t *use_mpc, int32_t *level) {
    if (!c || !rp) return fail(RMPC_EINVAL, "ctx/params is NULL");
    if (B < 0 || n_obs < 0 || n_obs > RMPC_MAX_OBSTACLES || (pred && n_pred < 0)) return fail(RMPC_EINVAL, "bad shape");
    if (B == 0) return RMPC_OK;
    if (!x || !out || (n_obs > 0 && !obstacles)) return fail(RMPC_EINVAL, "required pointer is NULL");
    if (!c->sub.empty())
        return multi_run(c, B,
                         {{(void *)x, 24, true, false}, {(void *)pred, (size_t)(pred ? n_pred : 0) * 24, true, false},
                          {out, 40, false, true}, {use_mpc, 1, false, true}, {level, 4, false, true}},
                         [&](RmpcCtx *sc, int64_t b, void **q) {
                             return rmpc_risk_batch(sc, rp, b, (const double *)q[0], (const double *)q[1], n_pred,
                                                    obstacles, n_obs, (double *)q[2], (uint8_t *)q[3], (int32_t *)q[4]);
                         });
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    double *dx, *dp, *dobs = nullptr, *dout;
    uint8_t *dm;
    int32_t *dl;
    RC(h2d(c, SB_X0, x, (size_t)B * 3, &dx));
    RC(h2d(c, SB_XREF, pred, (size_t)B * (pred ? n_pred : 0) * 3, &dp));
    if (n_obs > 0) RC(h2d(c, SB_OBS, obstacles, (size_t)n_obs * 3, &dobs));
    RC(dalloc(c, SB_U0, out, (size_t)B * 5, &dout));
    RC(dalloc(c, SB_SLACK, use_mpc, (size_t)B, &dm));
    RC(dalloc(c, SB_STATUS, level, (size_t)B, &dl));
    HIP_TRY(rmpc_launch_risk(to_dev(rp), B, dx, dp, n_pred, dobs, n_obs, dout, dm, dl, own(c)));
    RC(d2h(c, out, dout, (size_t)B * 5));
    RC(d2h(c, use_mpc, dm, (size_t)B));
    RC(d2h(c, level, dl, (size_t)B));
    HIP_TRY(hipStreamSynchronize(own(c)));
    return RMPC_OK;
}

static int hybrid_step_impl(RmpcCtx *c, const RmpcRiskParams *rp, const RmpcLqrParams *lp,
                       const RmpcMpcParams *mp, int64_t B, const double *x, const double *x_refs,
                       int32_t ref_rows, const double *u_refs, int32_t uref_rows, const double *obstacles,
                       int32_t n_obs, int32_t *prev_ctrl, int32_t *steps_since, int32_t *step_count,
                            RmpcLqrCache *cache, double *u_out, uint8_t *used_mpc, double *risk_out, void *stream,
                       const int32_t *ref_off, double *pred = nullptr) {
    if (!c || !rp || !lp) return fail(RMPC_EINVAL, "ctx/params is NULL");
    if (!c->sub.empty()) return fail(RMPC_ENOTSUP, "device-pointer entry points take a single-device context");

    RC(check_mpc_params(mp, ref_rows, uref_rows, n_obs));
    RC(check_lqr(lp));
    if (mp->formulation != RMPC_LTV) return fail(RMPC_EINVAL, "hybrid uses solve_with_ltv (formulation LTV)");
    if (B < 0) return fail(RMPC_EINVAL, "B < 0");
    if (B == 0) return RMPC_OK;
    if (!x || !x_refs || !u_refs || !prev_ctrl || !steps_since || !u_out || !used_mpc || (n_obs > 0 && !obstacles))
        return fail(RMPC_EINVAL, "required pointer is NULL");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    HIP_TRY(c->idx_lqr.ensure((size_t)B * sizeof(int32_t)));
    HIP_TRY(c->idx_mpc.ensure((size_t)B * sizeof(int32_t)));
    HIP_TRY(c->counts.ensure(256));
    HIP_TRY(c->hyb_status.ensure((size_t)B * sizeof(int32_t)));
    if (c->use_side) HIP_TRY(side_stream(c));
    for (auto &e : c->hev)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int32_t *const cbase = (int32_t *)c->counts.p;
    if (!c->hyb_ready) {          // first step (or after a failed launch): zero both pairs
        HIP_TRY(hipMemsetAsync(cbase, 0, 32 * sizeof(int32_t), s));
        c->hyb_set = 0;
    }
    c->hyb_ready = false;
    int32_t *const cnt = cbase + 16 * c->hyb_set;
    // pred [B][N+1][3] (rollouts with use_predicted): read here for the robots whose previous
    // step ran MPC, then overwritten by this step's MPC branch
    HIP_TRY(rmpc_launch_hybrid_decide(to_dev(rp), B, x, obstacles, n_obs, prev_ctrl, steps_since, used_mpc,
                                      risk_out, (int32_t *)c->idx_lqr.p, (int32_t *)c->idx_mpc.p, cnt, s, pred,
                                      mp->horizon + 1, cbase + 16 * (1 - c->hyb_set)));
    c->hyb_set ^= 1;
    c->hyb_ready = true;
    // LQR branch on the side stream (rmpc_ctx_set_side_stream; else in order on this one):
    // x_ref / u_ref = row 0 of the segment (get_reference_at_index(k)).  The branches touch
    // disjoint robots.
    const bool side = c->use_side;
    if (side) {
        HIP_TRY(hipEventRecord(c->hev[0], s));
        HIP_TRY(hipStreamWaitEvent(c->side, c->hev[0], 0));
    }
    LqrDevParams ld = to_dev(lp);
    ld.ref_off = ref_off;
    const hipError_t el = rmpc_launch_lqr_control(ld, B, x, x_refs, ref_rows * 3, u_refs, uref_rows * 2, cache,
                                                  u_out, nullptr, nullptr, nullptr, nullptr,
                                                  (const int32_t *)c->idx_lqr.p, cnt, side ? c->side : s);
    const hipError_t eh = side ? hipEventRecord(c->hev[1], c->side) : hipSuccess;
    if (el != hipSuccess || eh != hipSuccess) {   // no return ahead of the side branch
        if (side) (void)hipStreamSynchronize(c->side);
        HIP_TRY(el);
        HIP_TRY(eh);
    }
    // MPC branch: solve_with_ltv on the segment; writes u0 straight into u_out
    // the MPC branch holds only the robots near an obstacle: about half the batch, all of
    // them in the hard part of the distribution, so the tail has room for more of them and a
    // lower fast cap pays (BASELINE config 5 sweep: cap 6 77.9M against 76.4M at cap 7)
    const int rc = launch_mpc(c, mp, B, x, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs, step_count, u_out,
                              nullptr, pred, nullptr, (int32_t *)c->hyb_status.p, nullptr, nullptr,
                              (const int32_t *)c->idx_mpc.p, cnt + 1, s, ref_off,
                              c->fast_cap > 0 ? c->fast_cap : (mp->horizon <= 20 && !c->warm_on ? 6 : 0), 1);
    if (side) HIP_TRY(hipStreamWaitEvent(s, c->hev[1], 0));   // join: the step ends when both branches have
    return rc;
}

static int hybrid_step(RmpcCtx *c, const RmpcRiskParams *rp, const RmpcLqrParams *lp,
                       const RmpcMpcParams *mp, int64_t B, const double *x, const double *x_refs,
                       int32_t ref_rows, const double *u_refs, int32_t uref_rows, const double *obstacles,
                       int32_t n_obs, int32_t *prev_ctrl, int32_t *steps_since, int32_t *step_count,
                       RmpcLqrCache *cache, double *u_out, uint8_t *used_mpc, double *risk_out, void *stream,
                       const int32_t *ref_off, double *pred = nullptr) {
    if (!c) return fail(RMPC_EINVAL, "ctx/params is NULL");
    if (!c->sub.empty() || B <= 0)
        return hybrid_step_impl(c, rp, lp, mp, B, x, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs, prev_ctrl,
                                steps_since, step_count, cache, u_out, used_mpc, risk_out, stream, ref_off, pred);
    HIP_TRY(hipSetDevice(c->device));
    const hipStream_t s = pick(c, stream);
    HIP_TRY(order_calls(c, s));
    const int rc = hybrid_step_impl(c, rp, lp, mp, B, x, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs,
                                    prev_ctrl, steps_since, step_count, cache, u_out, used_mpc, risk_out, stream,
                                    ref_off, pred);
    HIP_TRY(mark_call(c, s));
    return rc;
}

extern "C" int rmpc_hybrid_step_batch_dev(RmpcCtx *c, const RmpcRiskParams *rp, const RmpcLqrParams *lp,
                                          const RmpcMpcParams *mp, int64_t B, const double *x,
                                          const double *x_refs, int32_t ref_rows, const double *u_refs,
                                          int32_t uref_rows, const double *obstacles, int32_t n_obs,
                                          int32_t *prev_ctrl, int32_t *steps_since, int32_t *step_count,
                                          RmpcLqrCache *cache, double *u_out, uint8_t *used_mpc,
                                          double *risk_out, void *stream) {
    return hybrid_step(c, rp, lp, mp, B, x, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs, prev_ctrl,
                       steps_since, step_count, cache, u_out, used_mpc, risk_out, stream, nullptr);
}

extern "C" int rmpc_hybrid_step_batch(RmpcCtx *c, const RmpcRiskParams *rp, const RmpcLqrParams *lp,
                                      const RmpcMpcParams *mp, int64_t B, const double *x,
                                      const double *x_refs, int32_t ref_rows, const double *u_refs,
                                      int32_t uref_rows, const double *obstacles, int32_t n_obs,
                                      int32_t *prev_ctrl, int32_t *steps_since, int32_t *step_count,
                                      RmpcLqrCache *cache, double *u_out, uint8_t *used_mpc, double *risk_out) {
    if (!c || !rp || !lp) return fail(RMPC_EINVAL, "ctx/params is NULL");
    RC(check_mpc_params(mp, ref_rows, uref_rows, n_obs));
    if (B < 0) return fail(RMPC_EINVAL, "B < 0");
    if (B == 0) return RMPC_OK;
    if (!x || !x_refs || !u_refs || !prev_ctrl || !steps_since || !u_out || !used_mpc || (n_obs > 0 && !obstacles))
        return fail(RMPC_EINVAL, "required pointer is NULL");
    if (!c->sub.empty())
        return multi_run(c, B,
                         {{(void *)x, 24, true, false}, {(void *)x_refs, (size_t)ref_rows * 24, true, false},
                          {(void *)u_refs, (size_t)uref_rows * 16, true, false}, {prev_ctrl, 4, true, true},
                          {steps_since, 4, true, true}, {step_count, 4, true, true},
                          {cache, sizeof(RmpcLqrCache), true, true}, {u_out, 16, false, true},
                          {used_mpc, 1, false, true}, {risk_out, 8, false, true}},
                         [&](RmpcCtx *sc, int64_t b, void **q) {
                             return rmpc_hybrid_step_batch(sc, rp, lp, mp, b, (const double *)q[0], (const double *)q[1],
                                                           ref_rows, (const double *)q[2], uref_rows, obstacles, n_obs,
                                                           (int32_t *)q[3], (int32_t *)q[4], (int32_t *)q[5],
                                                           (RmpcLqrCache *)q[6], (double *)q[7], (uint8_t *)q[8],
                                                           (double *)q[9]);
                         });
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    double *dx, *dxr, *dur, *dobs = nullptr, *du, *drisk;
    int32_t *dprev, *dsince, *dstep;
    RmpcLqrCache *dc;
    uint8_t *dused;
    RC(h2d(c, SB_X0, x, (size_t)B * 3, &dx));
    RC(h2d(c, SB_XREF, x_refs, (size_t)B * ref_rows * 3, &dxr));
    RC(h2d(c, SB_UREF, u_refs, (size_t)B * uref_rows * 2, &dur));
    if (n_obs > 0) RC(h2d(c, SB_OBS, obstacles, (size_t)n_obs * 3, &dobs));
    RC(h2d(c, SB_EXTRA1, prev_ctrl, (size_t)B, &dprev));
    RC(h2d(c, SB_EXTRA2, steps_since, (size_t)B, &dsince));
    RC(h2d(c, SB_STEP, step_count, (size_t)B, &dstep));
    RC(h2d(c, SB_CACHE, cache, (size_t)B, &dc));
    RC(dalloc(c, SB_U0, u_out, (size_t)B * 2, &du));
    RC(dalloc(c, SB_SLACK, used_mpc, (size_t)B, &dused));
    RC(dalloc(c, SB_COST, risk_out, (size_t)B, &drisk));
    RC(rmpc_hybrid_step_batch_dev(c, rp, lp, mp, B, dx, dxr, ref_rows, dur, uref_rows, dobs, n_obs, dprev,
                                  dsince, dstep, dc, du, dused, drisk, own(c)));
    RC(d2h(c, u_out, du, (size_t)B * 2));
    RC(d2h(c, used_mpc, dused, (size_t)B));
    RC(d2h(c, risk_out, drisk, (size_t)B));
    RC(d2h(c, prev_ctrl, dprev, (size_t)B));
    RC(d2h(c, steps_since, dsince, (size_t)B));
    RC(d2h(c, step_count, dstep, (size_t)B));
    RC(d2h(c, cache, dc, (size_t)B));
    HIP_TRY(hipStreamSynchronize(own(c)));
    return RMPC_OK;
}

// ------------------------------------------------------------------------------ plant / refs
extern "C" int rmpc_plant_step_batch(RmpcCtx *c, int64_t B, const double *x, const double *u, double dt,
                                     double v_max, double omega_max, int32_t method, double *x_next) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    if (B < 0 || (method != 0 && method != 1)) return fail(RMPC_EINVAL, "bad shape/method");
    if (B == 0) return RMPC_OK;
    if (!x || !u || !x_next) return fail(RMPC_EINVAL, "required pointer is NULL");
    if (!c->sub.empty())
        return multi_run(c, B, {{(void *)x, 24, true, false}, {(void *)u, 16, true, false}, {x_next, 24, false, true}},
                         [&](RmpcCtx *sc, int64_t b, void **q) {
                             return rmpc_plant_step_batch(sc, b, (const double *)q[0], (const double *)q[1], dt, v_max,
                                                          omega_max, method, (double *)q[2]);
                         });
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    double *dx, *du, *dn;
    RC(h2d(c, SB_X0, x, (size_t)B * 3, &dx));
    RC(h2d(c, SB_UREF, u, (size_t)B * 2, &du));
    RC(dalloc(c, SB_U0, x_next, (size_t)B * 3, &dn));
    HIP_TRY(rmpc_launch_plant(B, dx, du, dt, v_max, omega_max, method, dn, own(c)));
    RC(d2h(c, x_next, dn, (size_t)B * 3));
    HIP_TRY(hipStreamSynchronize(own(c)));
    return RMPC_OK;
}

extern "C" int rmpc_figure8_batch(RmpcCtx *c, int64_t B, const double *t0, int32_t rows, double A,
                                  double a, double dt, double *x_refs, double *u_refs) {
    if (!c) return fail(RMPC_EINVAL, "ctx is NULL");
    if (B < 0 || rows < 1) return fail(RMPC_EINVAL, "bad shape");
    if (B == 0) return RMPC_OK;
    if (!t0 || !x_refs || !u_refs) return fail(RMPC_EINVAL, "required pointer is NULL");
    if (!c->sub.empty())
        return multi_run(c, B,
                         {{(void *)t0, 8, true, false}, {x_refs, (size_t)rows * 24, false, true},
                          {u_refs, (size_t)rows * 16, false, true}},
                         [&](RmpcCtx *sc, int64_t b, void **q) {
                             return rmpc_figure8_batch(sc, b, (const double *)q[0], rows, A, a, dt, (double *)q[1],
                                                       (double *)q[2]);
                         });
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    double *dt0, *dxr, *dur;
    RC(h2d(c, SB_X0, t0, (size_t)B, &dt0));
    RC(dalloc(c, SB_XREF, x_refs, (size_t)B * rows * 3, &dxr));
    RC(dalloc(c, SB_UREF, u_refs, (size_t)B * rows * 2, &dur));
    HIP_TRY(rmpc_launch_figure8(B, dt0, rows, A, a, dt, dxr, dur, own(c)));
    RC(d2h(c, x_refs, dxr, (size_t)B * rows * 3));
    RC(d2h(c, u_refs, dur, (size_t)B * rows * 2));
    HIP_TRY(hipStreamSynchronize(own(c)));
    return RMPC_OK;
}

// ------------------------------------------------------------------------------ rollouts
extern "C" int rmpc_rollout_batch_dev(RmpcCtx *c, const RmpcRolloutParams *rp, const RmpcLqrParams *lp,
                                      const RmpcMpcParams *mp, const RmpcRiskParams *kp, int64_t B,
                                      const int32_t *start_index, const double *x0, const double *obstacles,
                                      int32_t n_obs, double *states, double *controls, uint8_t *used_mpc,
                                      int64_t *mpc_status, void *stream) {
    if (!c || !rp) return fail(RMPC_EINVAL, "ctx/params is NULL");
    if (!c->sub.empty()) return fail(RMPC_ENOTSUP, "device-pointer entry points take a single-device context");

    const int mode = rp->mode;
    if (mode < 0 || mode > 2) return fail(RMPC_EINVAL, "mode must be 0 (LQR), 1 (MPC) or 2 (hybrid)");
    if (rp->steps < 0 || rp->table_len < 1 || rp->mpc_rate < 1 || !(rp->dt > 0) ||
        (rp->plant_method != 0 && rp->plant_method != 1))
        return fail(RMPC_EINVAL, "bad rollout parameters");
    if (mode != 1 && !lp) return fail(RMPC_EINVAL, "LQR params required");
    if (mode != 0 && !mp) return fail(RMPC_EINVAL, "MPC params required");
    if (mode == 2 && !kp) return fail(RMPC_EINVAL, "risk params required");
    if (lp) RC(check_lqr(lp));
    const int rows = mode == 0 ? 1 : mp->horizon + 1;
    if (mode != 0) {
        RC(check_mpc_params(mp, rows, rows, n_obs));
        if (mp->formulation != RMPC_LTV) return fail(RMPC_EINVAL, "rollouts use solve_with_ltv (LTV)");
    }
    if (B < 0) return fail(RMPC_EINVAL, "B < 0");
    if (B == 0) return RMPC_OK;
    if (n_obs > 0 && !obstacles) return fail(RMPC_EINVAL, "obstacles is NULL");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    HIP_TRY(c->ro_x.ensure((size_t)B * 3 * sizeof(double)));
    // references: the generate() table, built once with `rows` copies of its last row appended,
    // so robot b's segment at step k is the `rows` rows from min(start_b + k, len - 1) on
    // (get_trajectory_segment's end clamp, reference_generator.py:299-326) -- the solves read
    // them from this shared table through per-robot row offsets (RMPC_ROLLOUT_REFS=copy: the
    // per-step per-robot segment copies instead)
    const bool copy_refs = rmpc_knob("RMPC_ROLLOUT_REFS") && !strcmp(rmpc_knob("RMPC_ROLLOUT_REFS"), "copy");
    const int64_t tab_rows = (int64_t)rp->table_len + rows;
    HIP_TRY(c->ro_xr.ensure((size_t)(copy_refs ? B * rows : tab_rows) * 3 * sizeof(double)));
    HIP_TRY(c->ro_ur.ensure((size_t)(copy_refs ? B * rows : tab_rows) * 2 * sizeof(double)));
    HIP_TRY(c->ro_off.ensure((size_t)B * sizeof(int32_t)));
    HIP_TRY(c->ro_u.ensure((size_t)B * 2 * sizeof(double)));
    HIP_TRY(c->ro_step.ensure((size_t)B * sizeof(int32_t)));
    HIP_TRY(c->ro_cache.ensure((size_t)B * sizeof(RmpcLqrCache)));
    HIP_TRY(c->ro_prev.ensure((size_t)B * sizeof(int32_t)));
    HIP_TRY(c->ro_since.ensure((size_t)B * sizeof(int32_t)));
    HIP_TRY(c->ro_status.ensure((size_t)B * sizeof(int32_t)));
    HIP_TRY(c->ro_used.ensure((size_t)B));
    HIP_TRY(c->ro_risk.ensure((size_t)B * sizeof(double)));
    HIP_TRY(c->ro_counts.ensure(4 * sizeof(unsigned long long)));
    double *x = (double *)c->ro_x.p, *xr = (double *)c->ro_xr.p, *ur = (double *)c->ro_ur.p;
    double *u = (double *)c->ro_u.p;
    int32_t *step = (int32_t *)c->ro_step.p, *prev = (int32_t *)c->ro_prev.p, *since = (int32_t *)c->ro_since.p;
    int32_t *status = (int32_t *)c->ro_status.p;
    RmpcLqrCache *cache = (RmpcLqrCache *)c->ro_cache.p;
    uint8_t *used_now = (uint8_t *)c->ro_used.p;
    // hybrid with use_predicted: the x_pred of each robot's last MPC solve, and no robot has
    // one before its first step
    double *pred = nullptr;
    if (mode == 2 && kp && kp->use_predicted) {
        HIP_TRY(c->ro_pred.ensure((size_t)B * (mp->horizon + 1) * 3 * sizeof(double)));
        pred = (double *)c->ro_pred.p;
        HIP_TRY(hipMemsetAsync(used_now, 0, (size_t)B, s));
    }
    unsigned long long *counts = (unsigned long long *)c->ro_counts.p;
    HIP_TRY(hipMemsetAsync(counts, 0, 4 * sizeof(unsigned long long), s));
    HIP_TRY(rmpc_launch_rollout_init(B, start_index, x0, rp->table_len, rp->A, rp->a, rp->dt, x, prev, since,
                                     step, cache, states, rp->steps, s));
    int32_t *off = copy_refs ? nullptr : (int32_t *)c->ro_off.p;
    if (!copy_refs)          // one "robot" whose segment is the whole padded table
        HIP_TRY(rmpc_launch_figure8_table(1, nullptr, 0, (int)tab_rows, rp->table_len, rp->A, rp->a, rp->dt, xr,
                                          ur, s));
    LqrDevParams ld = lp ? to_dev(lp) : LqrDevParams{};
    ld.ref_off = off;
    for (int k = 0; k < rp->steps; k++) {
        if (copy_refs)
            HIP_TRY(rmpc_launch_figure8_table(B, start_index, k, rows, rp->table_len, rp->A, rp->a, rp->dt, xr,
                                              ur, s));
        else
            HIP_TRY(rmpc_launch_ref_offsets(B, start_index, k, rp->table_len - 1, off, s));
        if (mode == 0) {                                   // run_simulation.py:77-80
            HIP_TRY(rmpc_launch_lqr_control(ld, B, x, xr, 3, ur, 2, cache, u, nullptr, nullptr, nullptr,
                                            nullptr, nullptr, nullptr, s));
        } else if (mode == 1) {                            // :250-259, zero-order hold in u
            if (k % rp->mpc_rate == 0) {
                // (warm start on the context: from each robot's solve mpc_rate steps earlier)
                RC(launch_mpc(c, mp, B, x, xr, rows, ur, rows, obstacles, n_obs, step, u, nullptr, nullptr,
                              nullptr, status, nullptr, nullptr, nullptr, nullptr, s, off, 0, rp->mpc_rate));
                HIP_TRY(rmpc_launch_status_count(B, status, nullptr, counts, s));
            }
        } else {                                           // :525-559
            RC(hybrid_step(c, kp, lp, mp, B, x, xr, rows, ur, rows, obstacles, n_obs, prev, since, step, cache, u,
                           used_now, (double *)c->ro_risk.p, s, off, pred));
            HIP_TRY(rmpc_launch_status_count(B, (const int32_t *)c->hyb_status.p, used_now, counts, s));
        }
        HIP_TRY(rmpc_launch_rollout_plant(B, x, u, rp->dt, rp->v_max, rp->omega_max, rp->plant_method, k,
                                          rp->steps, states, controls, mode == 2 ? used_now : nullptr,
                                          mode == 1 ? 1 : 0, used_mpc, s));
    }
    if (mpc_status)
        HIP_TRY(hipMemcpyAsync(mpc_status, counts, 4 * sizeof(unsigned long long), hipMemcpyDeviceToDevice, s));
    return RMPC_OK;
}

extern "C" int rmpc_rollout_batch(RmpcCtx *c, const RmpcRolloutParams *rp, const RmpcLqrParams *lp,
                                  const RmpcMpcParams *mp, const RmpcRiskParams *kp, int64_t B,
                                  const int32_t *start_index, const double *x0, const double *obstacles,
                                  int32_t n_obs, double *states, double *controls, uint8_t *used_mpc,
                                  int64_t *mpc_status) {
    if (!c || !rp) return fail(RMPC_EINVAL, "ctx/params is NULL");
    if (B < 0 || rp->steps < 0) return fail(RMPC_EINVAL, "bad shape");
    if (B == 0) return RMPC_OK;
    if (!c->sub.empty()) {        // per-device rollouts; the MPC status counts are summed
        const size_t K1 = (size_t)rp->steps;
        std::vector<int64_t> cnt(4 * c->sub.size(), 0);
        std::mutex cmu;
        const int rc = multi_run(
            c, B,
            {{(void *)start_index, 4, true, false}, {(void *)x0, 24, true, false}, {states, (K1 + 1) * 24, false, true},
             {controls, K1 * 16, false, true}, {used_mpc, K1, false, true}},
            [&](RmpcCtx *sc, int64_t b, void **q) {
                int64_t m[4] = {0, 0, 0, 0};
                const int r = rmpc_rollout_batch(sc, rp, lp, mp, kp, b, (const int32_t *)q[0], (const double *)q[1],
                                                 obstacles, n_obs, (double *)q[2], (double *)q[3], (uint8_t *)q[4],
                                                 mpc_status ? m : nullptr);
                std::lock_guard<std::mutex> g(cmu);
                for (int i = 0; i < 4; i++) cnt[i] += m[i];
                return r;
            });
        if (rc == RMPC_OK && mpc_status)
            for (int i = 0; i < 4; i++) mpc_status[i] = cnt[i];
        return rc;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    const size_t K = (size_t)rp->steps;
    int32_t *dstart;
    double *dx0, *dobs = nullptr, *dst, *dct;
    uint8_t *dused;
    RC(h2d(c, SB_EXTRA1, start_index, (size_t)B, &dstart));
    RC(h2d(c, SB_X0, x0, (size_t)B * 3, &dx0));
    if (n_obs > 0) RC(h2d(c, SB_OBS, obstacles, (size_t)n_obs * 3, &dobs));
    RC(dalloc(c, SB_XPRED, states, (size_t)B * (K + 1) * 3, &dst));
    RC(dalloc(c, SB_USEQ, controls, (size_t)B * K * 2, &dct));
    RC(dalloc(c, SB_SLACK, used_mpc, (size_t)B * K, &dused));
    int64_t *dcnt = nullptr;
    if (mpc_status) {
        HIP_TRY(c->stage[SB_ITERS].ensure(64));
        dcnt = (int64_t *)c->stage[SB_ITERS].p;
    }
    RC(rmpc_rollout_batch_dev(c, rp, lp, mp, kp, B, dstart, dx0, dobs, n_obs, dst, dct, dused, dcnt, own(c)));
    RC(d2h(c, states, dst, (size_t)B * (K + 1) * 3));
    RC(d2h(c, controls, dct, (size_t)B * K * 2));
    RC(d2h(c, used_mpc, dused, (size_t)B * K));
    if (mpc_status) RC(d2h(c, mpc_status, dcnt, (size_t)4));
    HIP_TRY(hipStreamSynchronize(own(c)));
    return RMPC_OK;
}

#if RMPC_WAVE_LOG
// ---- wave timeline log (diagnostics builds only, rmpc_wlog.h): begin allocates `cap` records
// on the current device and arms the MPC kernels' logs; end synchronises the device, copies the
// records shard by shard, packed, into `host` ([cap][4] uint64) and returns their number
// (-2 - n if a shard overflowed).
extern "C" hipError_t rmpc_wlog_set_fast(rmpc::WaveLog);
extern "C" hipError_t rmpc_wlog_set_group(rmpc::WaveLog);
extern "C" hipError_t rmpc_wlog_set_solve(rmpc::WaveLog);
static rmpc::WaveLog g_host_wlog = {nullptr, nullptr, 0};
extern "C" int rmpc_diag_wlog_begin(uint32_t cap) {
    if (!g_host_wlog.rec) {
        if (hipMalloc((void **)&g_host_wlog.rec, (size_t)cap * 32) != hipSuccess) return -1;
        if (hipMalloc((void **)&g_host_wlog.n, 64 * 128) != hipSuccess) return -1;
        g_host_wlog.cap = cap;
    }
    if (hipDeviceSynchronize() != hipSuccess || hipMemset(g_host_wlog.n, 0, 64 * 128) != hipSuccess) return -1;
    if (rmpc_wlog_set_fast(g_host_wlog) != hipSuccess || rmpc_wlog_set_group(g_host_wlog) != hipSuccess ||
        rmpc_wlog_set_solve(g_host_wlog) != hipSuccess)
        return -1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
extern "C" int64_t rmpc_diag_wlog_end(void *host, uint32_t cap) {
    if (!g_host_wlog.rec || hipDeviceSynchronize() != hipSuccess) return -1;
    const rmpc::WaveLog off = {nullptr, nullptr, 0};
    unsigned n[64 * 32];
    if (hipMemcpy(n, g_host_wlog.n, sizeof n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    const unsigned per = g_host_wlog.cap / 64u;
    int64_t m = 0;
    bool over = false;
    for (int s = 0; s < 64; s++) {
        unsigned k = n[32 * s];
        if (k > per) { over = true; k = per; }
        if (m + k > cap) { over = true; k = (unsigned)(cap - m); }
        if (k && hipMemcpy((char *)host + m * 32, g_host_wlog.rec + 4ull * per * s, (size_t)k * 32,
                           hipMemcpyDeviceToHost) != hipSuccess)
            return -1;
        m += k;
    }
    if (rmpc_wlog_set_fast(off) != hipSuccess || rmpc_wlog_set_group(off) != hipSuccess ||
        rmpc_wlog_set_solve(off) != hipSuccess)
        return -1;
    return over ? -2 - m : m;
}
#endif
