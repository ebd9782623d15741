// Memory floor of k_resid_stream's traffic shape on config 2: one workgroup per unit reads
// the unit's 4608 int16 samples (9216 B) and writes 4608 u32 (18432 B), no compute.
// Variants: threads per workgroup, LDS bytes per workgroup (occupancy), a grid-stride copy.
// Build: hipcc --offload-arch=gfx950 -O3 stream_floor.hip -o stream_floor
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int N = 4608, NCH = N / 8;

template <int NT>
__global__ __launch_bounds__(NT) void k_unit(const uint4* __restrict__ src, uint4* __restrict__ dst, int lds_touch) {
    extern __shared__ uint32_t lds[];
    const int t = threadIdx.x;
    const uint4* s = src + (size_t)blockIdx.x * (NCH);
    uint4* d = dst + (size_t)blockIdx.x * (2 * NCH);
    constexpr int J = (NCH + NT - 1) / NT;
    uint4 q[J];
#pragma unroll
    for (int j = 0; j < J; ++j) q[j] = s[min(t + j * NT, NCH - 1)];
    if (lds_touch) lds[t] = q[0].x;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int c = t + j * NT;
        if (c < NCH) {
            const uint4 v = q[j];
            d[2 * c] = uint4{v.x & 0xffff, v.x >> 16, v.y & 0xffff, v.y >> 16};
            d[2 * c + 1] = uint4{v.z & 0xffff, v.z >> 16, v.w & 0xffff, v.w >> 16};
        }
    }
}

__global__ void k_grid(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t nch) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
    for (; i < nch; i += st) {
        const uint4 v = src[i];
        dst[2 * i] = uint4{v.x & 0xffff, v.x >> 16, v.y & 0xffff, v.y >> 16};
        dst[2 * i + 1] = uint4{v.z & 0xffff, v.z >> 16, v.w & 0xffff, v.w >> 16};
    }
}

int main() {
    const size_t units = 1000000;
    void *a, *b;
    CK(hipMalloc(&a, units * N * 2));
    CK(hipMalloc(&b, units * N * 4));
    CK(hipMemset(a, 1, units * N * 2));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = units * N * 6.0;
    auto run = [&](const char* name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%-40s %7.3f ms  %6.0f GB/s\n", name, best, bytes / best / 1e6);
        return 0;
    };
    for (int lds : {0, 10240, 20480, 32768}) {
        char nm[64];
        snprintf(nm, 64, "unit wg 128 thr, lds %d", lds);
        run(nm, [&] { hipLaunchKernelGGL(k_unit<128>, dim3(units), dim3(128), lds, 0, (const uint4*)a, (uint4*)b, lds > 0); });
        snprintf(nm, 64, "unit wg 256 thr, lds %d", lds);
        run(nm, [&] { hipLaunchKernelGGL(k_unit<256>, dim3(units), dim3(256), lds, 0, (const uint4*)a, (uint4*)b, lds > 0); });
    }
    for (int g : {1024, 4096, 16384})
        run("grid-stride", [&] { hipLaunchKernelGGL(k_grid, dim3(g), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, units * NCH); });
    return 0;
}
