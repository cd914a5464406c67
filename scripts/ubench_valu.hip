// Issue cost / dependent latency of the VALU ops the fast kernel is made of, one wave per
// SIMD (the fast kernel's occupancy at BASELINE config 3).  Prints cycles per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256

template <int OP, int CH>
__global__ __launch_bounds__(64, 1) void k(double *out, float *outf, unsigned long long *cyc, double s, float sf) {
    double a[CH];
    float f[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) { a[c] = s + threadIdx.x + c; f[c] = sf + threadIdx.x + c; }
    const double m = 1.0000001, q = 1e-9;
    const float mf = 1.0000001f, qf = 1e-9f;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < REP; r++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            if (OP == 0) a[c] = __builtin_fma(a[c], m, q);
            if (OP == 1) a[c] = a[c] * m;
            if (OP == 2) a[c] = a[c] + q;
            if (OP == 3) f[c] = __builtin_fmaf(f[c], mf, qf);
            if (OP == 4) a[c] = __builtin_amdgcn_rsq(a[c]);
            if (OP == 5) a[c] = __builtin_amdgcn_rcp(a[c]);
            if (OP == 6) f[c] = __builtin_amdgcn_rsqf(f[c]);
            if (OP == 7) { typedef float f2 __attribute__((ext_vector_type(2)));
                           f2 v = {f[c], a[c] > 0 ? 1.f : 2.f}; f2 w = {mf, mf}; f2 z = {qf, qf};
                           v = __builtin_elementwise_fma(v, w, z); f[c] = v.x; }
            if (OP == 8) a[c] = fmax(a[c], q);
        }
        asm volatile("" ::: "memory");
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double acc = 0; float accf = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) { acc += a[c]; accf += f[c]; }
    out[blockIdx.x * 64 + threadIdx.x] = acc;
    outf[blockIdx.x * 64 + threadIdx.x] = accf;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP, int CH>
void run(const char *name, double *o, float *of, unsigned long long *c, unsigned long long *h, int nb) {
    hipLaunchKernelGGL((k<OP, CH>), dim3(nb), dim3(64), 0, 0, o, of, c, 1.5, 1.5f);
    hipLaunchKernelGGL((k<OP, CH>), dim3(nb), dim3(64), 0, 0, o, of, c, 1.5, 1.5f);
    hipDeviceSynchronize();
    hipMemcpy(h, c, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < nb; i++) s += h[i];
    s /= nb;
    // s_memtime ticks at 100 MHz on gfx9 parts?  report raw ticks per op and let the ratio talk
    printf("%-10s chains=%2d  ticks/op=%.3f\n", name, CH, s / (REP * CH));
}

int main() {
    const int nb = 1024;
    double *o; float *of; unsigned long long *c;
    hipMalloc(&o, nb * 64 * 8); hipMalloc(&of, nb * 64 * 4); hipMalloc(&c, nb * 8);
    unsigned long long *h = new unsigned long long[nb];
#define R(op, nm) run<op, 1>(nm, o, of, c, h, nb); run<op, 8>(nm, o, of, c, h, nb);
    R(0, "fma_f64") R(1, "mul_f64") R(2, "add_f64") R(3, "fma_f32") R(4, "rsq_f64") R(5, "rcp_f64")
    R(6, "rsq_f32") R(7, "pk_fma_f32") R(8, "max_f64")
    return 0;
}
