// Probe (round 5): a device-wide admission gate for the lane-per-robot stage.  Each wave of a
// "producer" kernel adds 1 to a counter at its start; another stream waits (hipStreamWaitValue64,
// Gte) until the counter reaches the producer's wave count before launching its own kernel.
// Checks, for counter memory from hipExtMallocWithFlags(hipMallocSignalMemory) and from plain
// hipMalloc: the atomics work, the wait releases, and when the second kernel's first wave
// started relative to the producer's last wave start (s_memrealtime).
// Usage: probe_waitvalue [signal|device]
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probe_waitvalue.hip -o scripts/probe_waitvalue
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// producer: lane 0 of every wave adds 1 at its start, then the wave spins ~`spin` ticks
__global__ __launch_bounds__(64) void producer(unsigned long long *ctr, unsigned long long *t_start, long long spin) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        t_start[blockIdx.x] = t0;
    }
    while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < spin) __builtin_amdgcn_s_sleep(8);
}

__global__ void consumer(unsigned long long *t_first) {
    if (threadIdx.x == 0 && blockIdx.x == 0) t_first[0] = __builtin_amdgcn_s_memrealtime();
}

static int run(bool signal_mem) {
    unsigned long long *ctr = nullptr, *ts = nullptr, *tf = nullptr;
    if (signal_mem) CK(hipExtMallocWithFlags((void **)&ctr, 8, hipMallocSignalMemory));
    else CK(hipMalloc((void **)&ctr, 8));
    CK(hipMemset(ctr, 0, 8));
    const int waves = 4096;               // 4 rounds of a 1024-SIMD chip at one wave per SIMD
    CK(hipMalloc((void **)&ts, waves * 8));
    CK(hipMalloc((void **)&tf, 8));
    CK(hipDeviceSynchronize());
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    // a big LDS request keeps the producer at one wave per SIMD-ish (4 per CU)
    hipLaunchKernelGGL(producer, dim3(waves), dim3(64), 36 * 1024, a, ctr, ts, 2000LL);   // ~20 us each
    CK(hipGetLastError());
    CK(hipStreamWaitValue64(b, ctr, (unsigned long long)waves, hipStreamWaitValueGte));
    hipLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, b, tf);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(b));
    CK(hipStreamSynchronize(a));
    unsigned long long h[waves], f = 0, c = 0;
    CK(hipMemcpy(h, ts, sizeof h, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&f, tf, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&c, ctr, 8, hipMemcpyDeviceToHost));
    unsigned long long lo = ~0ull, hi = 0;
    for (int i = 0; i < waves; i++) { lo = h[i] < lo ? h[i] : lo; hi = h[i] > hi ? h[i] : hi; }
    printf("%s: counter %llu (expect %d); producer starts span %.1f us; consumer started %.1f us after the last producer "
           "wave start\n", signal_mem ? "signal memory" : "device memory", c, waves, (hi - lo) / 100.0,
           ((long long)f - (long long)hi) / 100.0);
    CK(hipStreamDestroy(a));
    CK(hipStreamDestroy(b));
    CK(hipFree(ts));
    CK(hipFree(tf));
    CK(hipFree(ctr));
    return c == (unsigned long long)waves ? 0 : 1;
}

int main(int argc, char **argv) {
    int ok = 0;
    CK(hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, 0));
    printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", ok);
    const bool sig = argc < 2 || argv[1][0] == 's';     // "signal" (default) or "device"
    return run(sig);
}
