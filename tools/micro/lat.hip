// microbenchmark (development): dependent-load latency for a footprint, and barrier cost, gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void chase(const unsigned* next, int steps, unsigned long long* out) {
    unsigned p = threadIdx.x;  // one wave, lanes walk independent chains
    long long t0 = clock64();
    for (int i = 0; i < steps; i++) p = next[p];
    long long t1 = clock64();
    if (threadIdx.x == 0) { out[0] = (unsigned long long)(t1 - t0); out[1] = p; }
}
__global__ void barriers(int n, unsigned long long* out) {
    long long t0 = clock64();
    for (int i = 0; i < n; i++) __syncthreads();
    long long t1 = clock64();
    if (threadIdx.x == 0) out[0] = (unsigned long long)(t1 - t0);
}
int main() {
    unsigned long long* d_out;
    hipMalloc(&d_out, 16);
    for (size_t mb : {1, 4, 64, 1024}) {
        size_t n = mb * (1 << 20) / 4;
        std::vector<unsigned> h(n);
        // random permutation cycle with stride to defeat locality, per lane offset
        size_t stride = 4099 * 16 + 17;
        for (size_t i = 0; i < n; i++) h[i] = (unsigned)((i + stride * 16) % n);
        unsigned* d;
        hipMalloc(&d, n * 4);
        hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
        const int steps = 2000;
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, steps, d_out);
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, steps, d_out);
        unsigned long long o[2];
        hipMemcpy(o, d_out, 16, hipMemcpyDeviceToHost);
        printf("footprint %5zu MB: %.0f cycles per dependent load\n", mb, (double)o[0] / steps);
        hipFree(d);
    }
    for (int t : {64, 256, 512, 1024}) {
        hipLaunchKernelGGL(barriers, dim3(1), dim3(t), 0, 0, 10000, d_out);
        unsigned long long o;
        hipMemcpy(&o, d_out, 8, hipMemcpyDeviceToHost);
        printf("barrier, %4d threads: %.1f cycles\n", t, (double)o / 10000);
    }
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("clock rate attr %d kHz\n", clk);
    return 0;
}
