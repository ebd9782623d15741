// PCIe copy concurrency probe: host->device and device->host at the same time, by SDMA
// (hipMemcpyAsync) or by a copy kernel on mapped page-locked host memory.
// Build: hipcc --offload-arch=gfx950 -O2 copy_probe.hip -o copy_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void kcopy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
    for (; i + 3 * st < n; i += 4 * st) {
        uint4 a = src[i], b = src[i + st], c = src[i + 2 * st], d = src[i + 3 * st];
        dst[i] = a; dst[i + st] = b; dst[i + 2 * st] = c; dst[i + 3 * st] = d;
    }
    for (; i < n; i += st) dst[i] = src[i];
}

int main() {
    const size_t B = 1ull << 30;
    void *h_in, *h_out, *d_in, *d_out;
    CK(hipHostMalloc(&h_in, B, hipHostMallocMapped));
    CK(hipHostMalloc(&h_out, B, hipHostMallocMapped));
    CK(hipMalloc(&d_in, B));
    CK(hipMalloc(&d_out, B));
    memset(h_in, 1, B);
    CK(hipMemset(d_out, 2, B));
    void *hm_in, *hm_out;
    CK(hipHostGetDevicePointer(&hm_in, h_in, 0));
    CK(hipHostGetDevicePointer(&hm_out, h_out, 0));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto h2d = [&](int mode, hipStream_t s) {
        if (mode == 0) return hipMemcpyAsync(d_in, h_in, B, hipMemcpyHostToDevice, s);
        hipLaunchKernelGGL(kcopy, dim3(mode), dim3(256), 0, s, (const uint4*)hm_in, (uint4*)d_in, B / 16);
        return hipGetLastError();
    };
    auto d2h = [&](int mode, hipStream_t s) {
        if (mode == 0) return hipMemcpyAsync(h_out, d_out, B, hipMemcpyDeviceToHost, s);
        hipLaunchKernelGGL(kcopy, dim3(mode), dim3(256), 0, s, (const uint4*)d_out, (uint4*)hm_out, B / 16);
        return hipGetLastError();
    };
    const int modes[] = {0, 32, 64, 128, 256};
    for (int rep = 0; rep < 2; ++rep)
        for (int mi : modes)
            for (int mo : modes) {
                if (mi && mo && mi != mo) continue;
                double t[3];
                for (int which = 0; which < 3; ++which) {
                    CK(hipDeviceSynchronize());
                    auto t0 = std::chrono::steady_clock::now();
                    if (which != 1) CK(h2d(mi, s1));
                    if (which != 0) CK(d2h(mo, s2));
                    CK(hipDeviceSynchronize());
                    t[which] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                }
                if (rep == 1)
                    printf("h2d %s%-4d d2h %s%-4d  h2d alone %6.1f ms (%5.1f GB/s)  d2h alone %6.1f ms (%5.1f GB/s)  both %6.1f ms (%5.1f GB/s total)\n",
                           mi ? "kern" : "sdma", mi, mo ? "kern" : "sdma", mo, t[0], B / t[0] / 1e6, t[1], B / t[1] / 1e6, t[2],
                           2 * B / t[2] / 1e6);
            }
    return 0;
}
