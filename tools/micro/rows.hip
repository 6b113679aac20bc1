// microbenchmark (development): the bundle engine's member-step memory pattern on gfx950.
// Per wave and step: NT terms x 12 rows (each a 64-lane x 8 B = 512 B coalesced load) from random
// monomials of a per-workgroup arena, summed; optionally a 3-row store per step.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
template <int NT, bool STORE>
__global__ __launch_bounds__(256) void step(const double* arena, double* outbuf, long rows_per_wg, int steps, unsigned long long* cyc) {
    __shared__ double pad[12000];  // ~96 KB: one workgroup per CU
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double* a = arena + (long)blockIdx.x * rows_per_wg * 64 + lane;
    double* o = outbuf + (long)blockIdx.x * 4 * 64 * 3 * 4096 + wave * 64 * 3 * 4096 + lane;
    unsigned s = 12345u + blockIdx.x * 977u + wave * 131u;
    double acc[3] = {0, 0, 0};
    long long t0 = clock64();
    for (int it = 0; it < steps; it++) {
        double v[NT][12];
#pragma unroll
        for (int t = 0; t < NT; t++) {
            s = s * 1664525u + 1013904223u;
            const long row = (long)((s >> 8) % (unsigned)(rows_per_wg / 12)) * 12;
            const int rr = __builtin_amdgcn_readfirstlane((int)row);
#pragma unroll
            for (int e = 0; e < 12; e++) v[t][e] = a[((long)rr + e) * 64];
        }
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int e = 0; e < 12; e++) acc[e % 3] += v[t][e];
        if (STORE) {
#pragma unroll
            for (int e = 0; e < 3; e++) o[((long)(it & 4095) * 3 + e) * 64] = acc[e];
        }
    }
    long long t1 = clock64();
    if (lane == 0) cyc[blockIdx.x * 4 + wave] = (unsigned long long)(t1 - t0);
    if (acc[0] == 12345.678) pad[threadIdx.x] = acc[1];  // keep
}
template <int NT, bool STORE>
void run(const double* d, double* o, long rows, int ncu, unsigned long long* dc, const char* name) {
    const int steps = 2000;
    hipLaunchKernelGGL((step<NT, STORE>), dim3(ncu), dim3(256), 0, 0, d, o, rows, steps, dc);
    hipLaunchKernelGGL((step<NT, STORE>), dim3(ncu), dim3(256), 0, 0, d, o, rows, steps, dc);
    std::vector<unsigned long long> h(ncu * 4);
    hipMemcpy(h.data(), dc, 8 * h.size(), hipMemcpyDeviceToHost);
    double m = 0;
    for (auto c : h) m += c;
    m /= h.size();
    printf("%-28s %8.0f cycles per step (%d terms x 12 rows)\n", name, m / steps, NT);
}
int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const long rows = (64L << 20) / 512;  // 64 MB per workgroup
    double *d, *o;
    unsigned long long* dc;
    hipMalloc(&d, (size_t)ncu * rows * 512);
    hipMemset(d, 0, (size_t)ncu * rows * 512);
    hipMalloc(&o, (size_t)ncu * 4 * 64 * 3 * 4096 * 8);
    hipMalloc(&dc, ncu * 4 * 8);
    printf("CUs %d\n", ncu);
    run<1, false>(d, o, rows, ncu, dc, "1 term, no store");
    run<4, false>(d, o, rows, ncu, dc, "4 terms, no store");
    run<4, true>(d, o, rows, ncu, dc, "4 terms, store");
    run<8, false>(d, o, rows, ncu, dc, "8 terms, no store");
    run<1, true>(d, o, rows, 1, dc, "1 CU: 1 term, store");
    run<4, false>(d, o, rows, 1, dc, "1 CU: 4 terms, no store");
    return 0;
}
