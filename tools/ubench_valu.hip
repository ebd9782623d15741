// VALU issue-rate microbenchmark for the candidate-sum inner loop (gfx950).
// Each wave runs ITER iterations of 16 independent accumulator chains of one instruction;
// the grid covers every SIMD several times.  Prints wave-instructions per CU-cycle.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITER 4096
#define OP16(INS)                                                                              \
    _Pragma("unroll") for (int j = 0; j < 16; ++j) asm volatile(INS : "+v"(acc[j]) : "v"(a), "v"(b));

template <int K>
__global__ __launch_bounds__(256) void kern(int* out, int a0, int b0) {
    int acc[16];
    for (int j = 0; j < 16; ++j) acc[j] = threadIdx.x + j;
    int a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
    for (int it = 0; it < ITER; ++it) {
        if constexpr (K == 0) { OP16("v_add_u32 %0, %1, %0") }
        if constexpr (K == 1) { OP16("v_dot2c_i32_i16 %0, %1, %2") }
        if constexpr (K == 2) { OP16("v_mad_i32_i24 %0, %1, %2, %0") }
        if constexpr (K == 3) { OP16("v_sad_u32 %0, %1, %2, %0") }
        if constexpr (K == 4) { OP16("v_dot4c_i32_i8 %0, %1, %2") }
        if constexpr (K == 5) { OP16("v_dot2_i32_i16 %0, %1, %2, %0") }
        if constexpr (K == 6) { OP16("v_mul_lo_u32 %0, %1, %0") }
        if constexpr (K == 7) { OP16("v_pk_mad_i16 %0, %1, %2, %0") }
        if constexpr (K == 8) { OP16("v_lshrrev_b32 %0, %1, %0") }
        if constexpr (K == 9) { OP16("v_floor_f32 %0, %0") }
        if constexpr (K == 10) { OP16("v_cvt_i32_f32 %0, %0") }
        if constexpr (K == 11) { OP16("v_cvt_u32_f32_e64 %0, |%0|") }
        if constexpr (K == 12) { OP16("v_add_u32_e64 %0, %1, %0") }
        if constexpr (K == 13) { OP16("v_cvt_flr_i32_f32 %0, %0") }
        if constexpr (K == 14) { OP16("v_max_i32 %0, %1, %0") }
        if constexpr (K == 15) { OP16("v_add_f32_e64 %0, |%1|, %0") }
        if constexpr (K == 16) { OP16("v_xor_b32 %0, %1, %0") }
        if constexpr (K == 17) { OP16("v_alignbit_b32 %0, %1, %0, 16") }
        if constexpr (K == 18) { OP16("v_cndmask_b32 %0, %1, %0, vcc") }
    }
    int s = 0;
    for (int j = 0; j < 16; ++j) s += acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static const char* names[] = {"v_add_u32", "v_dot2c_i32_i16", "v_mad_i32_i24", "v_sad_u32", "v_dot4c_i32_i8",
                              "v_dot2_i32_i16 (vop3p)", "v_mul_lo_u32", "v_pk_mad_i16", "v_lshrrev_b32", "v_floor_f32",
                              "v_cvt_i32_f32", "v_cvt_u32_f32_e64 |x|", "v_add_u32_e64", "v_cvt_flr_i32_f32",
                              "v_max_i32", "v_add_f32_e64 |x|", "v_xor_b32", "v_alignbit_b32", "v_cndmask_b32",
                              "v_mad_u64_u32"};

template <int K>
static void run(int* d, int cus, int wpc) {
    const int blocks = cus * wpc / 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, d, 1, 2);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, d, 1, 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double winst = (double)blocks * 4 * ITER * 16; /* wave-instructions */
    printf("%-24s waves/CU %2d  %.3f ms  %.2f Gwave-inst/s  %.3f wave-inst/CU/ns\n", names[K], wpc, ms,
           winst / ms / 1e6, winst / ms / 1e6 / cus);
}

int main() {
    int* d;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    hipMalloc(&d, sizeof(int) * cus * 32 * 64 * 4);
    printf("CUs %d clock %d kHz\n", cus, p.clockRate);
    for (int wpc : {16}) {
        run<0>(d, cus, wpc);
        run<1>(d, cus, wpc);
        run<3>(d, cus, wpc);
        run<8>(d, cus, wpc);
        run<9>(d, cus, wpc);
        run<10>(d, cus, wpc);
        run<11>(d, cus, wpc);
        run<12>(d, cus, wpc);
        run<13>(d, cus, wpc);
        run<14>(d, cus, wpc);
        run<15>(d, cus, wpc);
        run<16>(d, cus, wpc);
        run<17>(d, cus, wpc);
        run<18>(d, cus, wpc);
    }
    hipFree(d);
    return 0;
}
