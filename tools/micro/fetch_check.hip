// microbenchmark (development): known-byte kernels for validating the rocprofv3 traffic counters
// (FETCH_SIZE / WRITE_SIZE, KiB) on gfx950 against the access shapes of the reach kernels:
//   rows8     each wave reads whole 512 B rows (64 lanes x 8 B), as the bundle engine's [row][64]
//             coefficient loads, streaming through a buffer once
//   rand8     the same 512 B rows, each wave drawing rows at random from a 16 GB buffer (L2 misses)
//   stream16  each lane reads 16 B (the guide's streaming case)
//   write8    each wave writes whole 512 B rows
// Each kernel runs once per launch over the sizes printed as "expect"; compare with the counters:
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_check ; rocprofv3 --pmc WRITE_SIZE -- ./fetch_check
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void rows8(const double* __restrict__ a, long rows, double* sink) {
    const int lane = threadIdx.x & 63;
    const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
    const long nw = ((long)gridDim.x * blockDim.x) >> 6;
    double s = 0;
    for (long r = wave; r < rows; r += nw) s += a[r * 64 + lane];
    if (s == 1234.5) sink[0] = s;
}
__global__ __launch_bounds__(256) void rand8(const double* __restrict__ a, long rows, int per_wave, double* sink) {
    const int lane = threadIdx.x & 63;
    const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
    unsigned long long st = 0x9e3779b97f4a7c15ull * (wave + 1);
    double s = 0;
    for (int k = 0; k < per_wave; k++) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        const long r = (long)((st >> 20) % (unsigned long long)rows);
        s += a[r * 64 + lane];
    }
    if (s == 1234.5) sink[0] = s;
}
__global__ __launch_bounds__(256) void stream16(const double2* __restrict__ a, long n2, double* sink) {
    double s = 0;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 1234.5) sink[0] = s;
}
__global__ __launch_bounds__(256) void write8(double* __restrict__ a, long rows) {
    const int lane = threadIdx.x & 63;
    const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
    const long nw = ((long)gridDim.x * blockDim.x) >> 6;
    for (long r = wave; r < rows; r += nw) a[r * 64 + lane] = (double)r;
}

int main() {
    const long bytes = 16L << 30;                  // 16 GB buffer: far beyond the 8 x 4 MB of L2
    const long rows = bytes / 512;
    double *a, *sink;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    hipMemset(a, 0, bytes);
    const int grid = 256 * 8;
    const long stream_bytes = 4L << 30;            // 4 GB read once
    const int per_wave = 4096;                      // random rows per wave
    const long rand_bytes = (long)grid * 4 * per_wave * 512;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms;
    hipLaunchKernelGGL(rows8, dim3(grid), dim3(256), 0, 0, a, stream_bytes / 512, sink);
    hipEventRecord(e0);
    hipLaunchKernelGGL(rows8, dim3(grid), dim3(256), 0, 0, a, stream_bytes / 512, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("rows8    expect read  %ld KiB per launch (%.0f GB/s)\n", stream_bytes / 1024, stream_bytes / ms / 1e6);
    hipEventRecord(e0);
    hipLaunchKernelGGL(rand8, dim3(grid), dim3(256), 0, 0, a, rows, per_wave, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("rand8    expect read  %ld KiB per launch (%.0f GB/s)\n", rand_bytes / 1024, rand_bytes / ms / 1e6);
    hipEventRecord(e0);
    hipLaunchKernelGGL(stream16, dim3(grid), dim3(256), 0, 0, (const double2*)a, stream_bytes / 16, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("stream16 expect read  %ld KiB per launch (%.0f GB/s)\n", stream_bytes / 1024, stream_bytes / ms / 1e6);
    hipEventRecord(e0);
    hipLaunchKernelGGL(write8, dim3(grid), dim3(256), 0, 0, a, stream_bytes / 512);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("write8   expect write %ld KiB per launch (%.0f GB/s)\n", stream_bytes / 1024, stream_bytes / ms / 1e6);
    hipDeviceSynchronize();
    return 0;
}
