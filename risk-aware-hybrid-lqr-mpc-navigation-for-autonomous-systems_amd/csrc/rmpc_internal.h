// rmpc_internal.h -- host/device shared structs of librmpc.so (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rmpc.h"
#include "rmpc_wlog.h"

#define RMPC_PDAS_ITERS 32   // PDAS solves before the projected-Newton phase

// Diagnostics / A-B knobs (RMPC_FAST_CAP, RMPC_TAIL, RMPC_DENSE_PROF, ...): the library reads
// them only when RMPC_DIAG=1 is set too, so production behaviour never depends on the
// environment.  Returns getenv(name) in diagnostics mode, else NULL.
#include <stdlib.h>
#include <string.h>
static inline const char *rmpc_knob(const char *name) {
    const char *d = getenv("RMPC_DIAG");
    return (d && !strcmp(d, "1")) ? getenv(name) : nullptr;
}
#define RMPC_WAVE_LANES 64

// Flattened, kernel-argument form of RmpcMpcParams.
struct MpcDevParams {
    double Q[3], R[2], P[3];
    double d_safe, rho, v_max, omega_max, dt;
    int ltv, soft, max_iter, ramp_up_steps;
    // optional per-robot first reference row (rollouts: rows of one shared, end-padded Figure-8
    // table); NULL = robot b's segment starts at row b * ref_rows of its own arrays
    const int32_t *ref_off;
};

// first row of robot b's reference segment (x_refs / u_refs are [rows][3] / [rows][2])
__host__ __device__ __forceinline__ size_t ref_row0(const int32_t *ref_off, int64_t b, int rows) {
    return ref_off ? (size_t)ref_off[b] : (size_t)b * (size_t)rows;
}

// Offsets (in elements) of the fields of one robot's workspace record.
struct MpcLayout {
    int N, bs, nb, no;
    int A0, A1, B0, B1, US0, US1, XS0, XS1, XS2;
    int LO0, LO1, HI0, HI1, BF0, BF1;
    int HN0, HN1, HB, HACT;
    int HBO;   // original hinge right-hand sides (HB = HBO + shift in the hard-constraint mode)
    int K;     // 8 * nb: K rows (6) + k (2), per block
    int X0, X1, X2, U0, U1, Z0, Z1, G0, G1;
    int REC;
};

MpcLayout rmpc_mpc_layout(int N, int bs, int no);

// Arguments of the register-resident LTV kernel (rmpc_mpc_fast.hip).
struct MpcFastArgs {
    MpcDevParams prm;
    int64_t B;                       // robots (or capacity of `index`)
    const double *x0, *x_refs, *u_refs;
    int ref_rows, uref_rows, no;
    const double *obs;               // [no][3] (x, y, radius), device memory
    int32_t *step_count;
    double *u0, *u_seq, *x_pred, *cost;
    int32_t *status, *iters;
    uint8_t *slack_used;
    double2 *gains;                  // per-wave gain tiles
    const int32_t *index, *count;    // optional robot index list (device-side length)
    int32_t *retry, *retry_count;    // robots handed to the next stage
    int pdas_cap;                    // PDAS solves before a robot is handed on
    unsigned long long *prof;        // diagnostics: per-phase cycle counters (may be null)
    uint32_t *retry_sets;            // per retry slot: hinge flags [N], box states [NB], iters,
                                     // slot-minor (word w of slot s at [w * B + s]); the warm
                                     // start of the next stage (may be null)
    const uint32_t *warm_sets;       // continuing pass: the previous pass's retry_sets, read by
                                     // list position (null: cold start from empty sets)
    int extra_cap;                   // > 0 (with warm_sets): PDAS solves beyond the record's count
                                     // (the fp64 refinement pass) instead of pdas_cap in total
    // fp32 pass of a refined request (non-null): certified robots are appended here with their
    // sets (same record layout as retry_sets) for the fp64 refinement pass, which writes their
    // outputs; uncertified ones still go to `retry`
    int32_t *refine, *refine_count;
    uint32_t *refine_sets;
    // Warm start across calls (rmpc_ctx_set_warm_start): per ROBOT b, the active sets of its
    // previous certified solve, slot-minor [N + NB + 1][B] (hinge flags, box states, the stamp
    // of the call that wrote them); read shifted by prev_shift steps at the start (the last step
    // repeated) when the stamp is prev_stamp - 1 (the robot's last solve was the previous call),
    // written back with prev_stamp at certification (this kernel's output pass and the tail's).
    // All zero = the cold start.  Null: off.
    uint32_t *prev_sets;
    int prev_shift;
    uint32_t prev_stamp;
    int init_zc;                     // cold start: hinge rows violated by the free response start active
    // Multi-pass stage (rmpc_ctx_set_stage_passes).  An earlier pass's records (retry_sets) also
    // carry the cycle history after the iteration word -- RMPC_REC_HIST words, the four
    // newest active-set signatures as lo/hi pairs (rec_hist) -- and the next pass restores it
    // (warm_hist), so a continued robot detects a cycle exactly when the one-pass stage would;
    // a robot whose sets cycle in an earlier pass goes straight to the tail's list (cyc: list,
    // counter, records), as it would from the one-pass stage.  Null / 0: off.
    int rec_hist, warm_hist;
    int32_t *cyc, *cyc_count;
    uint32_t *cyc_sets;
    // lanes per robot (rmpc_ctx_set_lanes_per_robot): 1 = one lane per robot where an instance
    // has both forms (the fp32 N = 30 8-obstacle stage); 0 = the default (paired there)
    int lanes;
};
#define RMPC_REC_HIST 8
// LDS slot.  The LDS-using kernels of the MPC pipeline (the lane-per-robot stage, the lane-group
// tail, the generic kernel's leftover list) each run one wave per SIMD, four per CU, and with
// batches in flight they replace each other on the CUs.  A CU allocates each workgroup's LDS as
// one contiguous range, so a tail workgroup (37.6 KB) leaving a hole smaller than a stage
// workgroup (39.8 KB) kept the next stage wave off that SIMD, and a 121-KB generic workgroup
// could start only on an emptied CU.  Every such workgroup requests exactly one quarter of the
// CU's LDS instead (static + dynamic = RMPC_LDS_SLOT), so any hole fits any of them.
#define RMPC_LDS_SLOT (160 * 1024 / 4)
// static LDS bytes of a kernel (hipFuncGetAttributes, cached)
size_t rmpc_kernel_static_lds(const void *fn);
// the dynamic LDS to request: `need` padded up to the slot when the kernel takes most of one
// (at least 3/4: those instances are also the one-wave-per-SIMD ones; a smaller request, e.g.
// the fp32 N = 20 stage's 24 KB at 207 VGPRs, keeps its higher occupancy)
static inline size_t rmpc_lds_slot_pad(const void *fn, size_t need) {
    const size_t st = rmpc_kernel_static_lds(fn);
    return (need + st <= RMPC_LDS_SLOT && 4 * (need + st) >= 3 * RMPC_LDS_SLOT) ? RMPC_LDS_SLOT - st : need;
}


// list counters per set of a context (retry_count holds two sets, used by alternate calls)
#define RMPC_COUNT_WORDS 16

bool rmpc_mpc_fast_supported(int N, int bs, int prec, bool lti = false, int no = -1);
// an fp64 lane-per-robot instance that continues an fp32 request's certified sets
bool rmpc_mpc_refine_supported(int N, int bs, int no);
hipError_t rmpc_launch_mpc_fast(const MpcFastArgs &a, int N, int bs, int prec, hipStream_t stream,
                                bool lti = false);
// Diagnostics of the lane-group tail, owned by the context (released with it):
// RMPC_DENSE_PROF=2 per-wave phase records (device memory) and RMPC_GROUP_CHECK bounds-check
// records.  The check record and the per-wave progress words live in host-mapped (pinned,
// coherent) memory written with system-scope atomics, so the host can read them even after
// the launch has faulted and the stream is unusable.
struct GroupDiag {
    unsigned long long *pw = nullptr;   // [waves][16] phase records (device)
    int64_t pw_cap = 0;
    int32_t *chk_host = nullptr;        // [8]: flags, first site, value, block, ... (host-mapped)
    int32_t *site_host = nullptr;       // [waves]: last site each wave reached (host-mapped)
    int64_t site_cap = 0;
    void release();
};

bool rmpc_mpc_group_supported(int N, int bs, int no);
// diagnostics output (rmpc_diag.cpp; RMPC_DIAG=1 with RMPC_DENSE_PROF=1)
hipError_t rmpc_diag_print_stage_prof(const unsigned long long *pc, const int32_t *cnt, bool refine, hipStream_t s);
hipError_t rmpc_launch_mpc_group(const MpcDevParams &prm, int N, int bs, int no, int64_t capacity,
                                 const double *x0, const double *x_refs, int ref_rows,
                                 const double *u_refs, int uref_rows, const double *obstacles,
                                 int32_t *step_count, double *u0, double *u_seq, double *x_pred,
                                 double *cost, int32_t *status, uint8_t *slack_used, int32_t *iters,
                                 const int32_t *index, const int32_t *count, int32_t *retry,
                                 int32_t *retry_count, int pdas_cap, const uint32_t *warm,
                                 hipStream_t stream, unsigned long long *prof = nullptr,
                                 bool lti = false, GroupDiag *diag = nullptr, uint32_t *prev_sets = nullptr,
                                 uint32_t prev_stamp = 0, int32_t *count_out = nullptr, int prev_count = -1);

hipError_t rmpc_launch_mpc_f64(const MpcDevParams &prm, const MpcLayout &L, int64_t B,
                               const double *x0, const double *x_refs, int ref_rows,
                               const double *u_refs, int uref_rows, const double *obstacles,
                               int n_obs, int32_t *step_count, double *u0, double *u_seq,
                               double *x_pred, double *cost, int32_t *status, uint8_t *slack_used,
                               int32_t *iters, void *ws, const int32_t *index,
                               const int32_t *count, hipStream_t stream, int lds_lanes = 0,
                               int32_t *zero_next = nullptr, int32_t *count_out = nullptr, int prev_count = -1);
hipError_t rmpc_launch_mpc_f32(const MpcDevParams &prm, const MpcLayout &L, int64_t B,
                               const double *x0, const double *x_refs, int ref_rows,
                               const double *u_refs, int uref_rows, const double *obstacles,
                               int n_obs, int32_t *step_count, double *u0, double *u_seq,
                               double *x_pred, double *cost, int32_t *status, uint8_t *slack_used,
                               int32_t *iters, void *ws, const int32_t *index,
                               const int32_t *count, hipStream_t stream, int lds_lanes = 0,
                               int32_t *zero_next = nullptr, int32_t *count_out = nullptr, int prev_count = -1);
// lanes per workgroup for the LDS-resident generic kernel (0 = record too large for LDS)
int rmpc_mpc_lds_lanes(const MpcLayout &L);

struct LqrDevParams {
    double Q[3], R[2];
    double dt, v_max, omega_max;
    int max_iter, use_cache;
    const int32_t *ref_off;    // as MpcDevParams::ref_off (NULL: strided per-robot rows)
};

hipError_t rmpc_launch_lqr_control(const LqrDevParams &p, int64_t B, const double *x,
                                   const double *x_ref, int xref_stride, const double *u_ref,
                                   int uref_stride, RmpcLqrCache *cache, double *u_out,
                                   double *err_out, double *K_out, double *P_out, int32_t *status,
                                   const int32_t *index, const int32_t *count, hipStream_t stream);
hipError_t rmpc_launch_lqr_gain(const LqrDevParams &p, int64_t B, const double *v_r,
                                const double *theta_r, int guard, double *K_out, double *P_out,
                                int32_t *status, hipStream_t stream);

struct RiskDevParams {
    double d_safe, d_trigger, alpha, beta, th_low, th_med, th_high;
    int min_dwell;
    int use_pred;
};

hipError_t rmpc_launch_risk(const RiskDevParams &p, int64_t B, const double *x, const double *pred,
                            int n_pred, const double *obstacles, int n_obs, double *out,
                            uint8_t *use_mpc, int32_t *level, hipStream_t stream);
// pred [B][n_pred][3] (nullable): the predicted states of each robot's last MPC solve, used
// for robots whose used_mpc flag (read before it is overwritten) is set
hipError_t rmpc_launch_hybrid_decide(const RiskDevParams &p, int64_t B, const double *x,
                                     const double *obstacles, int n_obs, int32_t *prev_ctrl,
                                     int32_t *steps_since, uint8_t *used_mpc, double *risk_out,
                                     int32_t *idx_lqr, int32_t *idx_mpc, int32_t *counts,
                                     hipStream_t stream, const double *pred = nullptr, int n_pred = 0,
                                     int32_t *zero_next = nullptr);
hipError_t rmpc_launch_plant(int64_t B, const double *x, const double *u, double dt, double v_max,
                             double omega_max, int method, double *x_next, hipStream_t stream);
hipError_t rmpc_launch_figure8_table(int64_t B, const int32_t *start, int32_t k, int rows, int32_t table_len,
                                     double A, double a, double dt, double *x_refs, double *u_refs,
                                     hipStream_t stream);
hipError_t rmpc_launch_iota(int64_t B, int32_t *idx, int32_t *count, hipStream_t stream);
hipError_t rmpc_launch_ref_offsets(int64_t B, const int32_t *start, int32_t k, int32_t last, int32_t *off,
                                   hipStream_t stream);
hipError_t rmpc_launch_rollout_init(int64_t B, const int32_t *start, const double *x0, int32_t table_len,
                                    double A, double a, double dt, double *x, int32_t *prev_ctrl,
                                    int32_t *since, int32_t *step_count, RmpcLqrCache *cache, double *states,
                                    int32_t steps, hipStream_t stream);
hipError_t rmpc_launch_rollout_plant(int64_t B, double *x, const double *u, double dt, double v_max,
                                     double omega_max, int method, int32_t k, int32_t steps, double *states,
                                     double *controls, const uint8_t *used_now, int used_fill, uint8_t *used,
                                     hipStream_t stream);
hipError_t rmpc_launch_status_count(int64_t B, const int32_t *status, const uint8_t *mask,
                                    unsigned long long *counts, hipStream_t stream);
hipError_t rmpc_launch_figure8(int64_t B, const double *t0, int rows, double A, double a,
                               double dt, double *x_refs, double *u_refs, hipStream_t stream);
