// rmpc_diag.cpp -- diagnostics output of librmpc.so (RMPC_DIAG=1 builds of the A/B knobs only):
// the per-phase cycle counters of the lane-per-robot stage, the refinement pass and the
// lane-group tail (RMPC_DENSE_PROF=1), printed to stderr.  Nothing here runs in the product path.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "rmpc_internal.h"

// Reads the counters of the last MPC launch (pc: [0..63] stage and tail, [64..127] the
// refinement pass) and the context's list counts, synchronising the stream.
hipError_t rmpc_diag_print_stage_prof(const unsigned long long *pc, const int32_t *cnt, bool refine, hipStream_t s) {
    hipError_t e;
#define HIP_TRY(x)                         \
    do {                                   \
        if ((e = (x)) != hipSuccess) return e; \
    } while (0)
    unsigned long long h[64];
    int32_t cn[16];
    HIP_TRY(hipMemcpyAsync(h, pc, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(cn, cnt, sizeof(cn), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const double r = h[10] ? (double)h[10] : 1.0, li = h[9] ? (double)h[9] : 1.0;
    fprintf(stderr,
            "[group] in=%d (+%d from the refinement) out=%d rounds=%llu loop-its/round %.2f | cycles/round: setup %.0f pn-pre %.0f "
            "out %.0f upd %.0f ls %.0f | per loop-it: weights %.0f back %.0f fwd %.0f rows %.0f\n",
            cn[0], cn[10], cn[8], h[10], h[9] / r, h[0] / r, h[1] / r, h[6] / r, h[7] / r, h[8] / r,
            h[2] / li, h[3] / li, h[4] / li, h[5] / li);
    fprintf(stderr, "[group] tail iterations per robot:");
    for (int q = 0; q < 32; q++) fprintf(stderr, " %llu", h[24 + q]);
    fprintf(stderr, "\n");
    const double w = h[20] ? (double)h[20] : 1.0;
    fprintf(stderr, "[fast] waves=%llu per wave: total %.0f back %.0f fwd %.0f iters %.2f | per iter: back %.0f fwd %.0f"
            " | slowest wave: total %llu iters %llu back %llu%%\n",
            h[20], h[19] / w, h[16] / w, h[17] / w, h[18] / w, h[16] / (double)(h[18] ? h[18] : 1),
            h[17] / (double)(h[18] ? h[18] : 1), h[21] >> 16, (h[21] >> 8) & 0xff, h[21] & 0xff);
    fprintf(stderr, "[fast] waves by loop count 0..7+:");
    for (int q = 56; q < 64; q++) fprintf(stderr, " %llu", h[q]);
    fprintf(stderr, " | setup %.0f per wave, longest lane entry-to-exit %llu, output pass %.0f per lane\n",
            h[22] / w, h[23], h[11] / (double)(h[12] ? h[12] : 1));
    if (refine) {
        unsigned long long g[64];
        HIP_TRY(hipMemcpy(g, pc + 64, sizeof(g), hipMemcpyDeviceToHost));
        const double w2 = g[20] ? (double)g[20] : 1.0, i2 = g[18] ? (double)g[18] : 1.0;
        fprintf(stderr, "[refine] waves=%llu per wave: total %.0f back %.0f fwd %.0f iters %.2f setup %.0f | "
                "per iter: back %.0f fwd %.0f | slowest wave: total %llu iters %llu | loop counts 0..7+:",
                g[20], g[19] / w2, g[16] / w2, g[17] / w2, g[18] / w2, g[22] / w2, g[16] / i2, g[17] / i2,
                g[21] >> 16, (g[21] >> 8) & 0xff);
        for (int q = 56; q < 64; q++) fprintf(stderr, " %llu", g[q]);
        fprintf(stderr, "\n");
    }
    return hipSuccess;
#undef HIP_TRY
}
