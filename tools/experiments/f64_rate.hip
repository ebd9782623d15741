// f64 VALU issue rate on one MI355X: chains of independent v_fma_f64 / v_mul_f64+v_add_f64 at
// 1..4 waves per SIMD.  Prints wave-instructions per SIMD per core cycle (s_memtime) and the
// clock implied by s_memrealtime (100 MHz).  Build: hipcc -O3 --offload-arch=gfx950 f64_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k(double* out, int iters, unsigned long long* clk) {
    double a[16];
    const double x = out[threadIdx.x & 7] + 1.0, y = out[8 + (threadIdx.x & 7)];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = out[16 + i] + threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (MODE == 0) a[i] = __builtin_fma(a[i], x, y);
            else a[i] = a[i] * x + y;  // -ffp-contract=off: one mul, one add
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i];
    if (s == 12345.0) out[0] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

int main() {
    double* out; unsigned long long* clk;
    hipMalloc(&out, 64 * sizeof(double)); hipMemset(out, 0, 64 * sizeof(double));
    hipMalloc(&clk, 16);
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 20000;
    for (int mode = 0; mode < 2; ++mode)
        for (int wps = 1; wps <= 4; ++wps) {  // waves per SIMD: 4 SIMDs per CU, 256-thread blocks = 4 waves
            const int blocks = cus * wps;
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            auto launch = [&]() { if (mode == 0) k<0><<<blocks, 256>>>(out, iters, clk); else k<1><<<blocks, 256>>>(out, iters, clk); };
            launch(); hipDeviceSynchronize();
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            unsigned long long c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
            const double instr_per_wave = (double)iters * 16 * (mode == 0 ? 1 : 2);
            const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
            // per SIMD: wps waves each instr_per_wave instructions
            const double cyc = (double)c[0];
            printf("mode %s waves/SIMD %d: %.3f ms, wave0 %.0f cycles (clock %.2f GHz), cycles per wave-instr per SIMD %.2f, TFLOP/s %.1f\n",
                   mode == 0 ? "fma" : "mul+add", wps, ms, cyc, ghz, cyc / (instr_per_wave * wps),
                   (double)blocks * 256 * iters * 16 * 2 / (ms * 1e-3) / 1e12);
        }
    return 0;
}
