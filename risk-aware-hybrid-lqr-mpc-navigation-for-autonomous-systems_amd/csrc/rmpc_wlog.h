// rmpc_wlog.h -- per-wave timeline log (diagnostics builds only: -DRMPC_WAVE_LOG=1 through
// scripts/build_variant.sh; the product library compiles none of this).
//
// Every wave of the MPC kernels writes one 32-byte record: kernel id and workgroup, start and
// end in s_memrealtime ticks (the 100 MHz device-wide clock, so waves of different XCDs and
// different kernels share one time base), the SIMD it ran on (HW_ID and XCC_ID) and the
// dispatch packet's address (which tells the launches of one kernel apart).
// scripts/wave_timeline.py turns the records of an in-flight run into per-SIMD occupancy.
//
// The record slot comes from one of 64 counters (one 128-B line each, by workgroup), taken with
// an atomic issued when the wave STARTS and consumed at its end: an atomic at the end held
// every SIMD for its round trip (~2-5 us under load) and on one counter serialised ~16k atomics
// per launch, both of which distorted the timeline they were measuring.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef RMPC_WAVE_LOG
#define RMPC_WAVE_LOG 0
#endif

namespace rmpc {
struct WaveLog {
    unsigned long long *rec;     // [64][cap / 64][4]
    unsigned int *n;             // [64][32]: slots taken per shard (beyond cap / 64 dropped)
    unsigned int cap;
};
enum { WL_FAST = 1, WL_GROUP = 2, WL_SOLVE = 3 };
}  // namespace rmpc

#if RMPC_WAVE_LOG
namespace rmpc {
// one instance per translation unit (no relocatable device code): each TU exports its setter
static __device__ WaveLog g_wlog;

// at the wave's start: the start time and the record slot (lane 0; ~0u when off or full)
__device__ __forceinline__ unsigned wl_take() {
    if (threadIdx.x != 0 || !g_wlog.rec) return ~0u;
    const unsigned sh = blockIdx.x & 63u;
    const unsigned i = atomicAdd(g_wlog.n + 32u * sh, 1u);
    return i < g_wlog.cap / 64u ? sh * (g_wlog.cap / 64u) + i : ~0u;
}

// at the wave's end (every lane calls; lane 0 writes).  `its`: this lane's PDAS iterations in
// the launch (stage 1; 0 elsewhere): the record keeps the wave's maximum and the lanes' sum
// (lane utilisation = sum / (64 x max))
__device__ __forceinline__ void wl_record(int kid, unsigned slot, unsigned long long t0, int its = 0) {
    int mx = its, sm = its;
    for (int off = 32; off > 0; off >>= 1) {
        mx = max(mx, __shfl_xor(mx, off));
        sm += __shfl_xor(sm, off);
    }
    if (threadIdx.x != 0 || slot == ~0u) return;
#if RMPC_WLOG_DRAIN
    // (variant: the end after the wave's outstanding memory operations -- its last stores --
    // have completed, which the SIMD's release waits for)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
    const unsigned long long dp = (unsigned long long)__builtin_amdgcn_dispatch_ptr();
    unsigned long long *r = g_wlog.rec + 4ull * slot;
    r[0] = ((unsigned long long)kid << 56) | ((unsigned long long)(mx & 0xff) << 48) |
           ((unsigned long long)(sm & 0xffff) << 32) | blockIdx.x;
    r[1] = t0;
    r[2] = t1;
    r[3] = (((dp >> 6) & 0xffffffull) << 40) | ((unsigned long long)(xcc & 0xff) << 32) | hw;
}
}  // namespace rmpc
#define RMPC_WLOG_BEGIN                                                  \
    const unsigned long long wl_t0_ = __builtin_amdgcn_s_memrealtime(); \
    const unsigned wl_slot_ = rmpc::wl_take();
#define RMPC_WLOG_END(kid) rmpc::wl_record(kid, wl_slot_, wl_t0_);
#define RMPC_WLOG_END_ITS(kid, its) rmpc::wl_record(kid, wl_slot_, wl_t0_, its);
#define RMPC_WLOG_SETTER(name) \
    extern "C" hipError_t name(rmpc::WaveLog w) { return hipMemcpyToSymbol(HIP_SYMBOL(rmpc::g_wlog), &w, sizeof w); }
#else
#define RMPC_WLOG_BEGIN
#define RMPC_WLOG_END(kid)
#define RMPC_WLOG_END_ITS(kid, its)
#define RMPC_WLOG_SETTER(name)
#endif
