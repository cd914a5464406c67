/*
 * rmpc.h -- C-ABI of the MI355X batched MPC / LQR solve path (librmpc.so).
 *
 * The reference (Erebuzzz/Risk-Aware-Hybrid-LQR-MPC-Navigation-for-Autonomous-Systems)
 * has no FFI: its hot path is a pure-Python class API.  Each entry point below
 * replaces one reference method for a whole batch of independent robots:
 *
 *   rmpc_mpc_solve_batch      MPCController.solve_with_ltv   mpc_controller.py:345-522
 *                             MPCController.solve (LTI)      mpc_controller.py:150-314
 *                             (+ _get_fallback_solution      mpc_controller.py:316-343)
 *   rmpc_lqr_control_batch    LQRController.compute_control_at_operating_point
 *                                                            lqr_controller.py:191-215
 *                             (compute_gain 92-147 incl. its 1e-6 K cache, compute_control 149-189)
 *   rmpc_lqr_gain_batch       LQRController.get_lqr_gain / compute_gain(force_recompute)
 *                                                            lqr_controller.py:92-147, 217-242
 *   rmpc_risk_batch           RiskMetrics.assess_risk        risk_metrics.py:173-222
 *   rmpc_hybrid_step_batch    one step of run_hybrid_simulation's switch
 *                                                            run_simulation.py:525-559
 *   rmpc_plant_step_batch     DifferentialDriveRobot.simulate_step  differential_drive.py:138-172
 *   rmpc_figure8_batch        ReferenceTrajectoryGenerator.get_reference_at_time / segment
 *                                                            reference_generator.py:86-172
 *   rmpc_rollout_batch        closed-loop rollouts of run_simulation.py --mode lqr|mpc|hybrid
 *                                                            run_simulation.py:34-96,139-280,413-576
 *
 * Conventions
 *   - Every array is row-major, C-contiguous and batch-major (robot index outermost).
 *   - Functions without the _dev suffix take HOST pointers; the library stages them
 *     through device buffers it owns inside the context and returns after the results
 *     are back on the host (synchronous).  The _dev variants take DEVICE pointers and
 *     a hipStream_t (passed as void*; NULL = the null stream, as in HIP) and are
 *     asynchronous.  A context's scratch and its carried state (list counters, warm-start
 *     sets, hybrid counters) are shared by its calls, which the library keeps in call order:
 *     a call issued on another stream than the context's previous stateful call first makes
 *     its stream wait for that call (an event recorded at the end of every stateful call), so
 *     consecutive calls may use different streams.  Calls of one context must not be issued
 *     concurrently from several host threads; batches meant to run at the same time use one
 *     context each.  rmpc_ctx_destroy waits for the context's last call and side branch.
 *   - Return value: 0 on success, a negative RMPC_E* code on an API error (bad shape,
 *     null pointer, HIP failure).  rmpc_last_error() gives a thread-local message.
 *   - Numerical failure is never an API error: per robot, `status` says what happened
 *     and the reference's fallback law has already been applied, so results are
 *     always defined (as in the reference, which swallows solver exceptions).
 */
#ifndef RMPC_H
#define RMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RMPC_ABI_VERSION 1

/* error codes */
#define RMPC_OK 0
#define RMPC_EINVAL (-1)   /* bad argument / shape */
#define RMPC_EHIP (-2)     /* HIP runtime error */
#define RMPC_ENOMEM (-3)   /* device allocation failed */
#define RMPC_ENOTSUP (-4)  /* configuration not supported by this build */

/* per-robot status (MPCSolution.status in the reference) */
#define RMPC_OPTIMAL 0            /* exact optimum of the QP (active set certified)  -> "optimal"  */
#define RMPC_OPTIMAL_INACCURATE 1 /* iteration cap hit, last iterate is box feasible -> "optimal"  */
#define RMPC_FALLBACK 2           /* non-finite data / no certified solution -> fallback law     */
#define RMPC_DARE_FALLBACK 3      /* LQR: DARE did not converge -> K = [[1,0,0],[0,0,1]]          */

/* formulation */
#define RMPC_LTV 0   /* MPCController.solve_with_ltv */
#define RMPC_LTI 1   /* MPCController.solve          */

/* arithmetic */
#define RMPC_F64 0
#define RMPC_F32 1

#define RMPC_MAX_HORIZON 64
#define RMPC_MAX_OBSTACLES 16

typedef struct RmpcMpcParams {
    int32_t horizon;       /* N (mpc_controller.py:111)                            */
    int32_t block_size;    /* move blocking, LTV only (:118-121)                    */
    int32_t formulation;   /* RMPC_LTV / RMPC_LTI                                   */
    int32_t soft;          /* use_soft_constraints (default 1; 0 = hard half-spaces,
                              :383-386, infeasible -> RMPC_FALLBACK)               */
    int32_t precision;     /* RMPC_F64 / RMPC_F32                                   */
    int32_t max_iter;      /* active-set iteration cap (<=0: default 64)            */
    int32_t ramp_up_steps; /* cold-start omega ramp length (:144, default 10)       */
    int32_t _pad0;
    double Q[3];           /* Q_diag (:124-125)                                     */
    double R[2];           /* R_diag                                                */
    double P[3];           /* P_diag                                                */
    double d_safe;
    double slack_penalty;  /* rho                                                   */
    double v_max;
    double omega_max;
    double dt;
} RmpcMpcParams;

typedef struct RmpcLqrParams {
    double Q[3];           /* Q_diag (lqr_controller.py:70-75)                      */
    double R[2];
    double dt;
    double v_max;
    double omega_max;
    int32_t max_iter;      /* SDA doubling-step cap (<=0: default 64)               */
    int32_t use_cache;     /* honour the 1e-6 operating-point cache (:112-114)      */
} RmpcLqrParams;

typedef struct RmpcRiskParams {
    double d_safe, d_trigger, alpha, beta;          /* risk_metrics.py:51-82 (alpha, beta raw) */
    double threshold_low, threshold_medium, threshold_high;
    int32_t min_dwell_steps;                         /* run_simulation.py:520 (10)  */
    int32_t use_predicted;  /* 0: the reference's switch (no predicted states, :525-531).
                               1 (rmpc_rollout_batch, hybrid mode): a robot whose previous step
                               ran MPC passes that solve's x_pred as predicted_states to
                               assess_risk (compute_predictive_risk, risk_metrics.py:131-171) */
} RmpcRiskParams;

/* Per-robot LQR gain cache (lqr_controller.py:84-90): K (6), last (v_r, theta_r), valid flag */
typedef struct RmpcLqrCache {
    double K[6];
    double last_v;
    double last_theta;
    int32_t valid;
    int32_t _pad0;
} RmpcLqrCache;

typedef struct RmpcCtx RmpcCtx;

/* ---- context / library ------------------------------------------------------------------ */
int rmpc_abi_version(void);
const char *rmpc_last_error(void);
int rmpc_ctx_create(int device_id, RmpcCtx **out);
/* A context over n devices (SURVEY 8(b) rmpc_ctx_create(device_ids, n); 8(e)): the host-pointer
 * batch entry points (rmpc_mpc_solve_batch, rmpc_lqr_control_batch, rmpc_hybrid_step_batch,
 * rmpc_rollout_batch) split the robots over the devices -- blocks of 64 robots dealt
 * round-robin, so every device gets the batch's difficulty mix -- run the shards concurrently
 * (one host thread and stream per device) and gather every output back in input order.
 * Results are bitwise those of a single-device context (robots are independent).  A device
 * id may repeat (several streams on one GPU).  The _dev entry points and the diagnostics
 * take single-device contexts only (RMPC_ENOTSUP otherwise).  n = 1 is rmpc_ctx_create. */
int rmpc_ctx_create_multi(const int32_t *device_ids, int32_t n, RmpcCtx **out);
int rmpc_ctx_device_count(const RmpcCtx *ctx, int32_t *n);
int rmpc_ctx_destroy(RmpcCtx *ctx);
int rmpc_ctx_synchronize(RmpcCtx *ctx);
int rmpc_device_count(int *count);
/* diagnostics: with timing on, each MPC launch on the lane-per-robot path records events
 * around its three stages; rmpc_mpc_stage_times waits for the last launch's events and
 * returns their device times in ms: out3[0] lane-per-robot kernel, out3[1] wave-per-robot
 * tail kernel, out3[2] generic kernel on what is left. */
int rmpc_ctx_set_timing(RmpcCtx *ctx, int32_t on);
/* Stage caps of the MPC pipeline on this context (a performance setting, no reference
 * counterpart; results are the same QP optimum either way): PDAS solves in the lane-per-robot
 * stage before a robot moves to the lane-group tail, and PDAS solves in the tail before
 * projected Newton.  0 = the library default (7 / 4 at N <= 20).  With several batches in
 * flight on several contexts, a longer first stage moves less work into the tail
 * (HISTORY.md section 1: (9, 4) at BASELINE configs 3 and 5).  They apply to the hybrid
 * step's MPC branch too (its default first-stage cap is 6).  fast_cap, tail_cap in [0, 64]. */
int rmpc_ctx_set_stage_caps(RmpcCtx *ctx, int32_t fast_cap, int32_t tail_cap);
/* Passes of the lane-per-robot stage on this context (a performance setting; results are the
 * same QP optimum, and the same iterate path robot by robot): with first_cap > 0 the stage runs
 * every robot for first_cap PDAS solves, then continues only the uncertified robots, compacted
 * into dense waves from their active sets and iteration counts, up to second_cap solves (0: no
 * third pass) and then up to the stage cap.  A pass whose cap is not below the stage cap is
 * skipped.  0, 0 (the default): one pass.  With batches in flight the compaction recovers the
 * lane slots that certified robots leave idle in a one-pass wave (HISTORY.md section 11).
 * Caps in [0, 64], second_cap above first_cap or 0. */
int rmpc_ctx_set_stage_passes(RmpcCtx *ctx, int32_t first_cap, int32_t second_cap);
/* Lanes per robot in the lane-per-robot stage on this context (a performance setting; results
 * are the same QP optimum): 0 (default) = the library's choice, which pairs two lanes per
 * robot in the fp32 N = 30, 8-obstacle stage (BASELINE config 4: the rows split over the pair,
 * and 32768 robots then fill every SIMD of one GPU); 1 = one lane per robot there too (half the
 * waves and no duplicated recursion: with batches in flight the other batches fill the SIMDs,
 * config 4 +13%; one batch alone -20%); 2 = paired.  Other instances have one form. */
int rmpc_ctx_set_lanes_per_robot(RmpcCtx *ctx, int32_t lanes);
/* Side stream on this context (a performance setting; results are identical): on (default),
 * a pipeline's independent branch -- the fp64 refinement of an fp32 request beside the tail,
 * the hybrid step's LQR branch beside the MPC branch -- runs on a second stream of the context,
 * forked from and joined back to the call's stream.  Off, the branches run in order on the
 * call's stream.  With several contexts in flight on their own streams, the side streams add
 * to the streams sharing the device's hardware queues (GPU_MAX_HW_QUEUES), and the other
 * batches already fill the chip: the bench turns them off there (HISTORY.md section 1). */
int rmpc_ctx_set_side_stream(RmpcCtx *ctx, int32_t on);
/* First active sets of a cold solve on this context (a performance setting; the QP and its
 * optimum are unchanged): 0 (default) starts every robot's PDAS from empty sets; 1 starts the
 * hinge rows that the start error's free response under the reference inputs violates active
 * (mpc_controller.py:439-468 rows).  Mode 1 lowers the PDAS work per robot (config 3: mean
 * iterations 2.18 -> 2.02, robots handed to the tail 3552 -> 2211) but lengthens the hardest
 * robots' chains: with batches in flight it pays (configs 4 / 5: +4%), one batch alone it
 * costs ~10% (HISTORY.md).  Warm-started solves (rmpc_ctx_set_warm_start) are unaffected. */
int rmpc_ctx_set_cold_start(RmpcCtx *ctx, int32_t mode);
/* Warm start across calls on this context (replaces the reference's warm_start=True solves
 * with get_warm_start's shifted previous solution, mpc_controller.py:272-277, 470-475,
 * 524-538).  On, every whole-batch MPC call (rmpc_mpc_solve_batch[_dev]; MPC-mode rollouts)
 * starts robot b's active-set iteration from the sets certified by robot b's previous solve on
 * this context, shifted by one step (MPC rollouts: by mpc_rate steps) with the last step repeated;
 * the context treats the robots of consecutive calls with the same (B, N, obstacle count,
 * formulation, precision) as the same controllers, and a call of another shape starts cold.
 * A performance setting like the reference's: the QP and its certified optimum do not change,
 * only the iteration count (`iters`).  Off (the default): every solve starts from empty sets.
 * The hybrid step's MPC branch (a different robot subset each step) warm-starts only the robots
 * whose previous solve was the previous call.  Turning it on resets the sets. */
int rmpc_ctx_set_warm_start(RmpcCtx *ctx, int32_t on);
int rmpc_mpc_stage_times(RmpcCtx *ctx, double *out3);

/* ---- MPC --------------------------------------------------------------------------------
 * x0        [B][3]
 * x_refs    [B][ref_rows][3]   LTV needs ref_rows >= N+1 (the whole array is np.unwrap'ed,
 *                              :392-393); LTI pads with the last row when ref_rows < N+1.
 * u_refs    [B][uref_rows][2]  LTV needs uref_rows >= N; LTI pads when uref_rows < N.
 * obstacles [n_obs][3]         (x, y, radius), shared by the batch, n_obs <= 16.
 * step_count[B]  in/out, LTV only: the controller's _step_count (:143, :502-507); NULL =
 *                all zero and not written back.
 * outputs: u0 [B][2]; u_seq [B][N][2]; x_pred [B][N+1][3]; cost [B]; status [B];
 *          slack_used [B]; iters [B] -- all but u0 and status may be NULL.
 */
int rmpc_mpc_solve_batch(RmpcCtx *ctx, const RmpcMpcParams *p, int64_t B, const double *x0,
                         const double *x_refs, int32_t ref_rows, const double *u_refs,
                         int32_t uref_rows, const double *obstacles, int32_t n_obs,
                         int32_t *step_count, double *u0, double *u_seq, double *x_pred,
                         double *cost, int32_t *status, uint8_t *slack_used, int32_t *iters);
int rmpc_mpc_solve_batch_dev(RmpcCtx *ctx, const RmpcMpcParams *p, int64_t B, const double *x0,
                             const double *x_refs, int32_t ref_rows, const double *u_refs,
                             int32_t uref_rows, const double *obstacles, int32_t n_obs,
                             int32_t *step_count, double *u0, double *u_seq, double *x_pred,
                             double *cost, int32_t *status, uint8_t *slack_used, int32_t *iters,
                             void *stream);

/* ---- LQR --------------------------------------------------------------------------------
 * x, x_ref [B][3]; u_ref [B][2]; cache [B] in/out (NULL = no cache, always recompute).
 * u_out [B][2]; err_out [B][3] (wrapped tracking error, :209-210) nullable;
 * K_out [B][2][3] nullable; P_out [B][3][3] nullable (P of the last DARE solved);
 * status [B] nullable (RMPC_OPTIMAL or RMPC_DARE_FALLBACK).
 */
int rmpc_lqr_control_batch(RmpcCtx *ctx, const RmpcLqrParams *p, int64_t B, const double *x,
                           const double *x_ref, const double *u_ref, RmpcLqrCache *cache,
                           double *u_out, double *err_out, double *K_out, double *P_out,
                           int32_t *status);
int rmpc_lqr_control_batch_dev(RmpcCtx *ctx, const RmpcLqrParams *p, int64_t B, const double *x,
                               const double *x_ref, const double *u_ref, RmpcLqrCache *cache,
                               double *u_out, double *err_out, double *K_out, double *P_out,
                               int32_t *status, void *stream);
/* gains only: v_r [B], theta_r [B] -> K [B][2][3], P [B][3][3] (nullable), status [B] nullable.
 * guard_v = 1 applies compute_gain's |v_r| < 1e-6 -> 0.01 guard (:120-122); 0 = get_lqr_gain. */
int rmpc_lqr_gain_batch(RmpcCtx *ctx, const RmpcLqrParams *p, int64_t B, const double *v_r,
                        const double *theta_r, int32_t guard_v, double *K_out, double *P_out,
                        int32_t *status);

/* ---- risk / hybrid ----------------------------------------------------------------------
 * rmpc_risk_batch: x [B][3]; pred [B][n_pred][3] nullable (predicted_states) ->
 *   out [B][5] = {distance_risk, predictive_risk, combined_risk, min_obstacle_distance,
 *                 nearest_obstacle_id}, use_mpc [B], level [B] (0 low .. 3 critical).
 * rmpc_hybrid_step_batch: one switching step for B robots (run_simulation.py:525-559):
 *   reads risk, dwell state (prev_ctrl [B]: -1 none, 0 LQR, 1 MPC; steps_since [B]),
 *   decides, runs LQR (x_ref/u_ref = row 0 of the segment) or MPC (the segment) for each
 *   robot on the device (robots compacted per branch), writes u_out [B][2], used_mpc [B],
 *   risk_out [B] (combined), and updates prev_ctrl / steps_since / step_count / cache.
 */
int rmpc_risk_batch(RmpcCtx *ctx, const RmpcRiskParams *rp, int64_t B, const double *x,
                    const double *pred, int32_t n_pred, const double *obstacles, int32_t n_obs,
                    double *out, uint8_t *use_mpc, int32_t *level);
int rmpc_hybrid_step_batch(RmpcCtx *ctx, const RmpcRiskParams *rp, const RmpcLqrParams *lp,
                           const RmpcMpcParams *mp, int64_t B, const double *x,
                           const double *x_refs, int32_t ref_rows, const double *u_refs,
                           int32_t uref_rows, const double *obstacles, int32_t n_obs,
                           int32_t *prev_ctrl, int32_t *steps_since, int32_t *step_count,
                           RmpcLqrCache *cache, double *u_out, uint8_t *used_mpc,
                           double *risk_out);
int rmpc_hybrid_step_batch_dev(RmpcCtx *ctx, const RmpcRiskParams *rp, const RmpcLqrParams *lp,
                               const RmpcMpcParams *mp, int64_t B, const double *x,
                               const double *x_refs, int32_t ref_rows, const double *u_refs,
                               int32_t uref_rows, const double *obstacles, int32_t n_obs,
                               int32_t *prev_ctrl, int32_t *steps_since, int32_t *step_count,
                               RmpcLqrCache *cache, double *u_out, uint8_t *used_mpc,
                               double *risk_out, void *stream);

/* ---- plant / references ------------------------------------------------------------------
 * rmpc_plant_step_batch: x [B][3], u [B][2] -> x_next [B][3]; method 0 euler, 1 rk4.
 * rmpc_figure8_batch: t0 [B] -> x_refs [B][rows][3], u_refs [B][rows][2] at t0 + i*dt.
 */
int rmpc_plant_step_batch(RmpcCtx *ctx, int64_t B, const double *x, const double *u, double dt,
                          double v_max, double omega_max, int32_t method, double *x_next);
int rmpc_figure8_batch(RmpcCtx *ctx, int64_t B, const double *t0, int32_t rows, double A,
                       double a, double dt, double *x_refs, double *u_refs);

/* ---- closed-loop rollouts (run_simulation.py --mode lqr | mpc | hybrid) -------------------
 * B independent robots tracking the Figure-8 reference TABLE of
 * ReferenceTrajectoryGenerator.generate (row j at t = j*dt, table_len rows; indices past the
 * end clamp to the last row as get_reference_at_index / get_trajectory_segment do,
 * reference_generator.py:196-230, 277-326).  Robot b starts at table row start_index[b]
 * (NULL = 0) from state x0[b] (NULL = the reference at that row, run_simulation.py:64-65).
 * Step k, all on the device: references at rows start+k.., control -- LQR:
 * compute_control_at_operating_point (:77-80); MPC: solve_with_ltv every mpc_rate steps with
 * the control held in between (:243-259); hybrid: risk + dwell switch + branch (:525-559) --
 * then DifferentialDriveRobot.simulate_step (differential_drive.py:138-172).
 * Outputs (each nullable): states [B][steps+1][3], controls [B][steps][2], used_mpc
 * [B][steps] (hybrid), mpc_status [4] = counts of MPC solve statuses over the rollout.
 */
typedef struct RmpcRolloutParams {
    int32_t mode;          /* 0 LQR, 1 MPC, 2 hybrid                                    */
    int32_t steps;         /* control steps                                             */
    int32_t table_len;     /* rows of generate(duration) = len(np.arange(0, duration, dt)) */
    int32_t mpc_rate;      /* MPC every mpc_rate steps (run_simulation.py:243, 5)       */
    int32_t plant_method;  /* 0 euler, 1 rk4                                            */
    int32_t _pad0;
    double dt;             /* simulation / reference step                               */
    double A, a;           /* Figure-8 amplitude and frequency (reference_generator.py) */
    double v_max;          /* DifferentialDriveRobot limits (run_simulation.py:52)      */
    double omega_max;
} RmpcRolloutParams;

int rmpc_rollout_batch(RmpcCtx *ctx, const RmpcRolloutParams *rp, const RmpcLqrParams *lp,
                       const RmpcMpcParams *mp, const RmpcRiskParams *kp, int64_t B,
                       const int32_t *start_index, const double *x0, const double *obstacles,
                       int32_t n_obs, double *states, double *controls, uint8_t *used_mpc,
                       int64_t *mpc_status);
int rmpc_rollout_batch_dev(RmpcCtx *ctx, const RmpcRolloutParams *rp, const RmpcLqrParams *lp,
                           const RmpcMpcParams *mp, const RmpcRiskParams *kp, int64_t B,
                           const int32_t *start_index, const double *x0, const double *obstacles,
                           int32_t n_obs, double *states, double *controls, uint8_t *used_mpc,
                           int64_t *mpc_status, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RMPC_H */
