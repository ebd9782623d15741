/* check_mfma_i8.hip — pins the operand layout of v_mfma_i32_16x16x64_i8 on gfx950 that
 * k_resid's int8 candidate sums (k_resid.h, mfma8_*) assume:
 *   A: lane l holds A[l & 15][16 * (l >> 4) + t], t = 0..15, byte t of the 16-byte operand
 *   B: lane l holds B[16 * (l >> 4) + t][l & 15]
 *   D: lane l holds D[4 * (l >> 4) + r][l & 15], r = 0..3
 * Build: hipcc --offload-arch=gfx950 -O2 tools/check_mfma_i8.hip -o tools/check_mfma_i8 */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k(const int8_t* A, const int8_t* B, const int* C, int* D) {
    const int l = threadIdx.x;
    int8_t a[16], b[16];
    for (int t = 0; t < 16; ++t) {
        a[t] = A[(l & 15) * 64 + 16 * (l >> 4) + t];
        b[t] = B[(16 * (l >> 4) + t) * 16 + (l & 15)];
    }
    v4i av, bv, cv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    for (int r = 0; r < 4; ++r) cv[r] = C[(4 * (l >> 4) + r) * 16 + (l & 15)];
    v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, cv, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = d[r];
}

int main() {
    int8_t hA[16 * 64], hB[64 * 16];
    int hC[256], hD[256];
    int8_t *dA, *dB;
    int *dC, *dD;
    hipMalloc(&dA, sizeof hA);
    hipMalloc(&dB, sizeof hB);
    hipMalloc(&dC, sizeof hC);
    hipMalloc(&dD, sizeof hD);
    int bad = 0;
    for (int trial = 0; trial < 4; ++trial) {
        srand(trial + 1);
        for (int i = 0; i < 16 * 64; ++i) hA[i] = (int8_t)(trial == 3 ? -128 : (rand() & 255));
        for (int i = 0; i < 64 * 16; ++i) hB[i] = (int8_t)(trial == 3 ? -128 : (rand() & 255));
        for (int i = 0; i < 256; ++i) hC[i] = trial == 2 ? (int)(0x7ff00000u + (unsigned)i) : (rand() % 100000) - 50000;
        hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
        hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
        hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
        hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
        for (int m = 0; m < 16; ++m)
            for (int nn = 0; nn < 16; ++nn) {
                int64_t s = hC[m * 16 + nn];
                for (int kk = 0; kk < 64; ++kk) s += (int64_t)hA[m * 64 + kk] * hB[kk * 16 + nn];
                const int32_t w = (int32_t)(uint32_t)(uint64_t)s; /* two's-complement wrap */
                if (w != hD[m * 16 + nn]) {
                    if (bad < 8) printf("trial %d D[%d][%d] = %d, expected %d (exact %lld)\n", trial, m, nn,
                                        hD[m * 16 + nn], w, (long long)s);
                    ++bad;
                }
            }
    }
    printf(bad ? "mfma_i32_16x16x64_i8 layout: MISMATCH (%d)\n" : "mfma_i32_16x16x64_i8 layout: OK%.0d\n", bad);
    return bad ? 1 : 0;
}
