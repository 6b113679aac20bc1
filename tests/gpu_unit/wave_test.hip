// TEST HARNESS — device checks of the wave primitives in armour-dev_amd/csrc/wave.h against the
// ds_bpermute-based __shfl family. Never part of the product library.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "wave.h"

using namespace armour;

__global__ void wave_kernel(const uint64_t* in, int* bad) {
    const int l = threadIdx.x;
    const uint64_t v = in[blockIdx.x * 64 + l];
    const double d = __builtin_bit_cast(double, v & 0x3FFFFFFFFFFFFFFFull) ;
    int nb = 0;
    for (int m = 1; m < 64; m <<= 1) {
        if (xor_u64(v, m) != __shfl_xor(v, m, 64)) nb |= 1;
        if (xor_u32((uint32_t)v, m) != (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64)) nb |= 2;
    }
    const double sh_nx = __shfl(d, (l + 1) & 63, 64);    // every lane active: no inactive-source reads
    const uint64_t sh_pv = __shfl(v, (l + 63) & 63, 64);
    const double nx = next_f64(d), ref_nx = l < 63 ? sh_nx : 0.0;
    if (__builtin_bit_cast(uint64_t, nx) != __builtin_bit_cast(uint64_t, ref_nx)) nb |= 4;
    const uint64_t pv = prev_u64(v), ref_pv = l > 0 ? sh_pv : 0ull;
    if (pv != ref_pv) nb |= 8;
    // butterfly sum equal on all lanes and within rounding of a sequential sum
    const double s = wave_sum(d);
    if (s != __shfl(s, 0, 64)) nb |= 16;
    const int iv = (int)(v & 0xFFFF);
    int ref = 0;
    for (int k = 0; k <= l; k++) ref += __shfl(iv, k, 64);
    if (wave_incl_scan(iv) != ref) nb |= 32;
    int mx = 0;
    for (int k = 0; k < 64; k++) mx = max(mx, __shfl(iv, k, 64));
    if (wave_max(iv) != mx) nb |= 64;
    bad[blockIdx.x * 64 + l] = nb;
}

extern "C" int wave_selftest(int blocks, const uint64_t* host_in, int* host_bad) {
    uint64_t* din = nullptr;
    int* dbad = nullptr;
    if (hipMalloc(&din, sizeof(uint64_t) * blocks * 64) != hipSuccess) return -1;
    if (hipMalloc(&dbad, sizeof(int) * blocks * 64) != hipSuccess) return -1;
    hipMemcpy(din, host_in, sizeof(uint64_t) * blocks * 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(wave_kernel, dim3(blocks), dim3(64), 0, 0, din, dbad);
    const hipError_t e = hipDeviceSynchronize();
    hipMemcpy(host_bad, dbad, sizeof(int) * blocks * 64, hipMemcpyDeviceToHost);
    hipFree(din);
    hipFree(dbad);
    return e == hipSuccess ? 0 : -2;
}
