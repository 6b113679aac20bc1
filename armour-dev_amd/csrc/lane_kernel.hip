// armour-mi355x — reach-set kernel, bundle form (lane_engine.h): one 256-thread workgroup (4 waves)
// per bundle of 64 consecutive (world, interval) jobs, lane = job. Persistent grid over bundles;
// each resident workgroup owns an HBM arena (union hashes, presence masks, [row][64] coefficients),
// a header pool ([row][64]) and global key buffers for operators beyond the LDS key capacity. LDS
// holds the handle table, keys, group heads, staged operand hashes and the cross-wave reduction
// rows; several resident workgroups per CU overlap one bundle's barriers and serial header work
// with the others' group rounds. Two shapes of the same kernel (identical arithmetic: the key and
// stage capacities only decide what lives in LDS):
//   LaneWide:  2048 LDS keys / staged hashes, 73 KB LDS, 256 VGPRs: two bundles per CU; the faster
//              one for a planner alone on the GPU whose batch fits one round of two per CU;
//   LaneDense: 1344 / 1024, 50.8 KB, 168 VGPRs (more spills): three per CU; faster per world once a
//              batch fills three per CU, and under concurrent planners, whose kernels then find
//              room on the CUs a reach launch holds.
#include "lane_engine.h"

namespace armour {
namespace lane {

struct LaneArgs {
    int W, T;
    const JrsJoint* jrs;   // [W][T][NF] from jrs_kernel
    const Op* prog;
    int nops;
    const int* slot_off;   // payload rows of every handle slot in the pool
    int nslots;
    long pool_rows;        // per workgroup (the last 2 NF rows: torque-radius scratch)
    double* pool;          // [grid][pool_rows][LG]
    uint64_t* arena_h;     // [grid][hcap]
    uint64_t* arena_m;     // [grid][hcap]
    double* arena_c;       // [grid][ccap][LG]
    long hcap, ccap;
    uint64_t* gkh;         // [grid][gcap]
    uint32_t* gki;
    int* gkp;              // [grid][gcap + 1]
    int* ggp;              // [grid][gcap + 1]
    int gcap;
    double* gout;          // [grid][ocap][9][LG]
    uint64_t* gm;          // [grid][ocap]
    int ocap;
    unsigned long long* bytes;
    double* dump;          // optional [nops][DUMP_W][LG] of bundle 0 (null: off)
    unsigned long long* prof;  // optional [2 * nops + 16] per-op cycles/terms + phase cycles
    unsigned long long* btime; // optional [bundles][2]: start / end wall clock of every bundle
    unsigned long long* occ;   // [8] largest use over the launch: arena hashes, arena rows, operator
                               // terms, link / torque k-only monomials (capacity headroom)
    ReachCounters rc;          // rc.occ == occ, rc.bytes == bytes; published by the last workgroup
    const int* wlist;      // null: every world of the batch; else only these worlds (a retry)
    int nlist;
};

struct LaneWide {
    static constexpr int KEYS = 2048, STAGE = 2048, WPE = 2, PER_CU = 2;
};
struct LaneDense {
    static constexpr int KEYS = 1344, STAGE = 1024, WPE = 3, PER_CU = 3;
};

// S::WPE waves per SIMD (2: 256 VGPRs, 3: 168)
template <class S>
__global__ __attribute__((amdgpu_flat_work_group_size(LT, LT), amdgpu_waves_per_eu(S::WPE, S::WPE))) void lane_reach_kernel(const RobotParams* __restrict__ rpp, LaneArgs a, ReachOut out) {
    __shared__ LH H[MAX_SLOTS];
    __shared__ uint64_t kh[S::KEYS];
    __shared__ uint32_t ki[S::KEYS];
    __shared__ int kp[S::KEYS + 1];
    __shared__ int gp[S::KEYS + 1];
    __shared__ uint64_t stage[S::STAGE];
    __shared__ uint64_t rmask[128];
    __shared__ double red[(LW - 1) * RCH * LG];
    __shared__ int iscan[LW];
    __shared__ LArena arena;
    __shared__ int err;
    __shared__ int occ[4];
    __shared__ int last;

    span_start(a.rc);
    const RobotParams& rp = *rpp;
    const long wg = blockIdx.x;
    LCtx x;
    x.tid = threadIdx.x;
    x.wave = x.tid >> 6;
    x.lane = x.tid & 63;
    x.H = H;
    x.pool = a.pool + wg * a.pool_rows * LG;
    x.A = &arena;
    x.kh = kh; x.ki = ki; x.kp = kp; x.gp = gp; x.cap_lds = S::KEYS;
    x.lkh = (LAS uint64_t*)(void*)kh;
    x.lki = (LAS uint32_t*)(void*)ki;
    x.lgp = (LAS int*)(void*)gp;
    x.gkh = a.gkh + wg * a.gcap;
    x.gki = a.gki + wg * a.gcap;
    x.gkp = a.gkp + wg * (a.gcap + 1);
    x.ggp = a.ggp + wg * (a.gcap + 1);
    x.cap_glb = a.gcap;
    x.gout = a.gout + wg * (long)a.ocap * 9 * LG;
    x.gm = a.gm + wg * (long)a.ocap;
    x.cap_out = a.ocap;
    x.rmask = rmask;
    x.stage = stage;
    x.stage_cap = S::STAGE;
    x.red = red;
    x.scr = x.pool + (a.pool_rows - 2 * NF) * LG;  // torque scratch: the pool's last 2 NF rows
    x.iscan = iscan;
    x.err = &err;
    x.occ = occ;
    x.thr = rp.simplify_threshold;
    x.prof = LANE_PROF ? a.prof : nullptr;
    x.nops = a.nops;

    // a retry (wlist) runs the listed worlds' jobs only, as consecutive bundles of their own
    const long njobs = (long)(a.wlist ? a.nlist : a.W) * a.T;
    const long nb = (njobs + LG - 1) / LG;
    for (long b = blockIdx.x; b < nb; b += gridDim.x) {
        if (x.tid == 0) {
            arena.h = a.arena_h + wg * a.hcap;
            arena.m = a.arena_m + wg * a.hcap;
            arena.c = a.arena_c + wg * a.ccap * LG;
            arena.hcap = a.hcap;
            arena.ccap = a.ccap;
            arena.hused = 0;
            arena.cused = 0;
            arena.bytes = 0;
            err = 0;
            occ[0] = occ[1] = occ[2] = occ[3] = 0;
        }
        for (int k = x.tid; k < a.nslots; k += LT) H[k].off = a.slot_off[k];
        long job = b * LG + x.lane;
        x.valid = job < njobs;
        job = x.valid ? job : njobs - 1;
        x.job = a.wlist ? (long)a.wlist[job / a.T] * a.T + job % a.T : job;
        x.jrs = a.jrs + x.job * NF;
        __syncthreads();
        unsigned long long* const btime = LANE_PROF ? a.btime : nullptr;
        const unsigned long long t0 = btime ? wall_clock64() : 0;
        run_program(x, rp, a.prog, a.nops, out, b == 0 ? a.dump : nullptr);
        __syncthreads();
        if (btime && x.tid == 0) {
            btime[2 * b] = t0;
            btime[2 * b + 1] = wall_clock64();
        }
        if (err && x.wave == 0 && x.valid) atomicOr(&out.err[x.job / a.T], err);
        if (x.tid == 0) {
            atomicAdd(a.bytes, arena.bytes);
            atomicMax(&a.occ[0], (unsigned long long)arena.hused);
            atomicMax(&a.occ[1], (unsigned long long)max((long)occ[3], arena.cused));
            for (int k = 0; k < 3; k++) atomicMax(&a.occ[2 + k], (unsigned long long)occ[k]);
        }
        __syncthreads();
    }
    publish_counters(a.rc, out.err, a.W, &last);
}

}  // namespace lane
}  // namespace armour
