// Read-bandwidth vs working-set size (run on the GPU box): a 16-byte-per-lane read sweep over a buffer of S bytes,
// repeated; GB/s of the repeats (the first pass excluded). Shows where L2 (4 MB x 8 XCDs) and the memory-side cache
// (256 MB Infinity Cache) stop holding a re-read working set.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void rd(const double2* __restrict__ p, size_t n, double* out) {
    double acc = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = p[i];
        acc += v.x + v.y;
    }
    if (acc == 12345.678) out[0] = acc;
}

int main() {
    const size_t maxb = (size_t)2 << 30;
    double2* buf;
    double* out;
    if (hipMalloc(&buf, maxb) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 2;
    (void)hipMemset(buf, 0, maxb);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const size_t sizes_mb[] = {8, 16, 32, 64, 96, 128, 160, 192, 224, 256, 320, 512, 1024, 2048};
    printf("[");
    bool first = true;
    for (size_t mb : sizes_mb) {
        const size_t n = (mb << 20) / 16;
        const int reps = mb <= 256 ? 50 : 10;
        hipLaunchKernelGGL(rd, dim3(4096), dim3(256), 0, 0, buf, n, out);
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(rd, dim3(4096), dim3(256), 0, 0, buf, n, out);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%s{\"MB\": %zu, \"GBps\": %.1f, \"us_per_pass\": %.2f}", first ? "" : ", ", mb,
               (double)(mb << 20) * reps / (ms * 1e-3) / 1e9, ms * 1e3 / reps);
        first = false;
    }
    printf("]\n");
    return 0;
}
