// armour-mi355x — reach-set kernel: one 256-thread workgroup per (world, time interval) job.
// Persistent grid: each workgroup walks jobs job = blockIdx.x + k * gridDim.x and owns a private
// HBM arena (monomial storage) and a global fallback sort buffer for products larger than the
// LDS key buffer. LDS (~61 KB) holds the PZ handle table and the (hash, index) sort keys, so two
// workgroups fit per CU.
#include "reach.h"

namespace armour {

constexpr int REACH_THREADS = 256;
constexpr int KEY_CAP_LDS = 2048;

struct ReachArgs {
    int W, T;
    const double* q0;    // [W][NF]
    const double* qd0;
    const double* qdd0;
    uint64_t* arena_h;   // [grid][arena_cap]
    double* arena_c;     // [grid][arena_cap * 3]
    long arena_cap;
    uint64_t* gkh;       // [grid][gcap]
    uint32_t* gki;
    int* gkp;
    int gcap;
};

__global__ __launch_bounds__(REACH_THREADS, 2) void reach_kernel(const RobotParams* __restrict__ rpp, ReachArgs a, ReachOut out) {
    __shared__ PZH H[hs::COUNT];
    __shared__ uint64_t kh[KEY_CAP_LDS];
    __shared__ uint32_t ki[KEY_CAP_LDS];
    __shared__ int kp[KEY_CAP_LDS];
    __shared__ double red[(REACH_THREADS / 64) * 9];
    __shared__ int iscan[2 * REACH_THREADS];
    __shared__ Arena arena;
    __shared__ int err;
    __shared__ JrsJoint jrs[NF];
    __shared__ double scratch[2 * NF];
    __shared__ double q0s[NF], qd0s[NF], qdd0s[NF];

    const RobotParams& rp = *rpp;
    Ctx x;
    x.g = Grp{(int)threadIdx.x, (int)blockDim.x};
    x.H = H;
    x.opa = hs::OPA; x.opb = hs::OPB; x.opc = hs::OPC;
    x.A = &arena;
    x.kh = kh; x.ki = ki; x.kp = kp; x.cap_lds = KEY_CAP_LDS;
    x.gkh = a.gkh + (long)blockIdx.x * a.gcap;
    x.gki = a.gki + (long)blockIdx.x * a.gcap;
    x.gkp = a.gkp + (long)blockIdx.x * a.gcap;
    x.cap_glb = a.gcap;
    x.red = red;
    x.iscan = iscan;
    x.err = &err;
    x.thr = rp.simplify_threshold;

    const long njobs = (long)a.W * a.T;
    for (long job = blockIdx.x; job < njobs; job += gridDim.x) {
        const int w = (int)(job / a.T), t = (int)(job % a.T);
        if (threadIdx.x == 0) {
            arena.h = a.arena_h + (long)blockIdx.x * a.arena_cap;
            arena.c = a.arena_c + (long)blockIdx.x * a.arena_cap * 3;
            arena.hcap = a.arena_cap;
            arena.ccap = a.arena_cap * 3;
            arena.hused = 0;
            arena.cused = 0;
            err = 0;
        }
        if (threadIdx.x < NF) {
            q0s[threadIdx.x] = a.q0[w * NF + threadIdx.x];
            qd0s[threadIdx.x] = a.qd0[w * NF + threadIdx.x];
            qdd0s[threadIdx.x] = a.qdd0[w * NF + threadIdx.x];
        }
        __syncthreads();
        reach_job(x, rp, a.T, t, q0s, qd0s, qdd0s, out, job, jrs, scratch);
        if (threadIdx.x == 0 && err) atomicOr(&out.err[w], err);
        __syncthreads();
    }
}

}  // namespace armour
