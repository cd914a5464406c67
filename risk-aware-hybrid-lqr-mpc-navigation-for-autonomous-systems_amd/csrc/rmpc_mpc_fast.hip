// rmpc_mpc_fast.hip -- register-resident LTV MPC solve (the hot path of BASELINE config 3).
//
// Same QP, same algebra (rmpc_riccati.h) and same primal-dual active-set iterations as the
// generic kernel in rmpc_mpc.hip, specialised on the horizon N and block size BS so that
// every per-step quantity of a robot (sin/cos of the unwrapped reference heading, the
// reference input and position, the hinge flags) lives in VGPRs for the whole solve.
// Only the block gains (written by the backward sweep, read by the forward sweep) go
// through a per-wave tile in memory as coalesced 16-byte-per-lane rows, with the forward
// sweep prefetching PF blocks ahead; the certified inputs are re-derived from the last
// gains at output.  Obstacle rows are recomputed from registers on every pass instead of
// being streamed; the backward sweep skips a row no lane of the wave has active.
//
// Templated on the arithmetic type T: double for the fp64 configurations; float for fp32
// requests (BASELINE config 4: N=30, 8 obstacles), where the register-resident layout would
// not fit in fp64 at that horizon.  Inputs and outputs stay fp64 in both.
//
// One wave per workgroup, one lane per robot.  A robot that is not certified within the
// PDAS cap (or has non-finite data) is appended to a retry list, with its active sets, that
// the lane-group tail (rmpc_mpc_group.hip) continues from; the generic kernel takes what is
// left (fallback law).
#include "rmpc_fast_body.h"

namespace rmpc {
template <int N, int BS, typename T, bool LTI, int NO = 0, int PR = 1, bool WS = true>
__global__ __launch_bounds__(64, 1) void mpc_ltv_fast_kernel(MpcFastArgs a) {
    RMPC_WLOG_BEGIN
    int wl_its = 0;     // (wave-log builds: this lane's PDAS iterations in the launch)
    fast_body<N, BS, T, LTI, NO, PR, WS>(a, blockIdx.x, wl_its);
    RMPC_WLOG_END_ITS(WL_FAST, wl_its)
}
}  // namespace rmpc
RMPC_WLOG_SETTER(rmpc_wlog_set_fast)

using namespace rmpc;


bool rmpc_mpc_fast_supported(int N, int bs, int prec, bool lti, int no) {
    if (lti) return prec != RMPC_F32 && (N == 6 || N == 10 || N == 20);   // LTI: block size unused
    if (prec == RMPC_F32) return bs == 1 && (N == 20 || (N == 30 && no == 8));   // the refined shapes
    // fp64 N = 30: the paired-lane 8-obstacle instance (BASELINE config 4's shape) only
    if (bs == 1 && N == 30) return no == 8;
    return (bs == 1 && (N == 6 || N == 10 || N == 20)) || (bs == 2 && N == 6);
}

bool rmpc_mpc_refine_supported(int N, int bs, int no) {
    return bs == 1 && ((N == 30 && no == 8) || N == 20);
}

hipError_t rmpc_launch_mpc_fast(const MpcFastArgs &a, int N, int bs, int prec, hipStream_t stream, bool lti) {
    const int64_t n = a.B;
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + RMPC_WAVE - 1) / RMPC_WAVE)), block(RMPC_WAVE);
    // + the setup's staging scratch (64 robots x 17 doubles): 39.8 KB per wave at N = 20 in fp64,
    // so four waves still share a CU.  Paired lanes: 32 robot columns, no staging (fp64 N = 30:
    // 23 KB per wave)
    const size_t lds = (size_t)3 * N * RMPC_WAVE * (prec == RMPC_F32 ? sizeof(float) : sizeof(double)) +
                       (size_t)RMPC_WAVE * 17 * sizeof(double);
    const size_t lds2 = (size_t)3 * N * (RMPC_WAVE / 2) * (prec == RMPC_F32 ? sizeof(float) : sizeof(double)) +
                        (size_t)(RMPC_WAVE / 2) * 17 * sizeof(double);
    // every launch requests one LDS slot (rmpc_lds_slot_pad, RMPC_LDS_SLOT)
#define FK(kern, g, need) hipLaunchKernelGGL(kern, g, block, rmpc_lds_slot_pad((const void *)kern, need), stream, a)
    if (lti) {
        if (prec == RMPC_F32) return hipErrorInvalidValue;
        if (N == 20 && a.no == 3) FK((mpc_ltv_fast_kernel<20, 1, double, true, 3>), grid, lds);
        else if (N == 20) FK((mpc_ltv_fast_kernel<20, 1, double, true>), grid, lds);
        else if (N == 10) FK((mpc_ltv_fast_kernel<10, 1, double, true>), grid, lds);
        else if (N == 6) FK((mpc_ltv_fast_kernel<6, 1, double, true>), grid, lds);
        else return hipErrorInvalidValue;
    } else if (prec == RMPC_F32) {
        // paired lanes for the 8-obstacle N = 30 instance
        const dim3 grid2((unsigned)((n + RMPC_WAVE / 2 - 1) / (RMPC_WAVE / 2)));
        // one lane per robot on request (rmpc_ctx_set_lanes_per_robot): half the waves, no
        // duplicated recursion -- with batches in flight the other batches fill the SIMDs this
        // leaves idle (config 4 in flight +13%; one batch alone -20%)
        if (bs == 1 && N == 30 && a.no == 8 && a.lanes == 1)
            FK((mpc_ltv_fast_kernel<30, 1, float, false, 8, 1>), grid, lds);
        else if (bs == 1 && N == 30 && a.no == 8) FK((mpc_ltv_fast_kernel<30, 1, float, false, 8, 2>), grid2, lds2);
        else if (bs == 1 && N == 20) FK((mpc_ltv_fast_kernel<20, 1, float, false>), grid, lds);
        else return hipErrorInvalidValue;
    } else {
        const dim3 grid2((unsigned)((n + RMPC_WAVE / 2 - 1) / (RMPC_WAVE / 2)));
        // (N = 30, 8 obstacles in fp64: paired lanes -- fp64 requests and the fp32 requests'
        // refinement pass)
        if (bs == 1 && N == 30 && a.no == 8) FK((mpc_ltv_fast_kernel<30, 1, double, false, 8, 2>), grid2, lds2);
        else if (bs == 1 && N == 20 && a.no == 3 && a.prev_sets) FK((mpc_ltv_fast_kernel<20, 1, double, false, 3>), grid, lds);
        else if (bs == 1 && N == 20 && a.no == 3) FK((mpc_ltv_fast_kernel<20, 1, double, false, 3, 1, false>), grid, lds);
        else if (bs == 1 && N == 20) FK((mpc_ltv_fast_kernel<20, 1, double, false>), grid, lds);
        else if (bs == 1 && N == 10) FK((mpc_ltv_fast_kernel<10, 1, double, false>), grid, lds);
        else if (bs == 1 && N == 6) FK((mpc_ltv_fast_kernel<6, 1, double, false>), grid, lds);
        else if (bs == 2 && N == 6) FK((mpc_ltv_fast_kernel<6, 2, double, false>), grid, lds);
        else return hipErrorInvalidValue;
    }
#undef FK
    return hipGetLastError();
}
