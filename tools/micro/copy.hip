// Copy-kernel shapes for the achievable-HBM reference figure (development tool; bench.py reports
// the library's armour_copy_bandwidth). 2 x 2 GiB buffers, 20 reps each, HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v2d __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void copy_a(const v2d* __restrict__ s, v2d* __restrict__ d, long n) {
    const long stride = (long)gridDim.x * blockDim.x;
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const v2d a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
        d[i] = a; d[i + stride] = b; d[i + 2 * stride] = c; d[i + 3 * stride] = e;
    }
    for (; i < n; i += stride) d[i] = s[i];
}
template <int K, bool NT>
__global__ __launch_bounds__(256) void copy_b(const v2d* __restrict__ s, v2d* __restrict__ d, long n) {
    const long base = (long)blockIdx.x * 256 * K + threadIdx.x;
    v2d v[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const long i = base + k * 256;
        if (i < n) v[k] = NT ? __builtin_nontemporal_load(&s[i]) : s[i];
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
        const long i = base + k * 256;
        if (i < n) { if (NT) __builtin_nontemporal_store(v[k], &d[i]); else d[i] = v[k]; }
    }
}

int main() {
    const long bytes = 2L << 30, n = bytes / 16;
    v2d *a, *b;
    if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes)) return 1;
    (void)hipMemset(a, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        launch();
        (void)hipEventRecord(e0);
        for (int r = 0; r < 20; r++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s %.0f GB/s\n", name, 2.0 * bytes * 20 / (ms * 1e-3) / 1e9);
    };
    run("grid-stride x4 (library)", [&] { hipLaunchKernelGGL(copy_a, dim3(256 * 8), dim3(256), 0, 0, a, b, n); });
    run("grid-stride x4, 32/CU", [&] { hipLaunchKernelGGL(copy_a, dim3(256 * 32), dim3(256), 0, 0, a, b, n); });
    run("block x4", [&] { hipLaunchKernelGGL((copy_b<4, false>), dim3((n + 1023) / 1024), dim3(256), 0, 0, a, b, n); });
    run("block x4 nt", [&] { hipLaunchKernelGGL((copy_b<4, true>), dim3((n + 1023) / 1024), dim3(256), 0, 0, a, b, n); });
    run("block x8", [&] { hipLaunchKernelGGL((copy_b<8, false>), dim3((n + 2047) / 2048), dim3(256), 0, 0, a, b, n); });
    run("block x8 nt", [&] { hipLaunchKernelGGL((copy_b<8, true>), dim3((n + 2047) / 2048), dim3(256), 0, 0, a, b, n); });
    run("block x16 nt", [&] { hipLaunchKernelGGL((copy_b<16, true>), dim3((n + 4095) / 4096), dim3(256), 0, 0, a, b, n); });
    return 0;
}
