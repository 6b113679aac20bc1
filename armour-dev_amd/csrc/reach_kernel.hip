// armour-mi355x — reach-set kernel: one workgroup per (world, time interval) job.
// Persistent grid: each workgroup walks jobs job = blockIdx.x + k * gridDim.x, interprets the
// reach program (reach.h) for each, and owns a private HBM arena (monomial storage) plus a global
// fallback sort buffer for products larger than the LDS key buffer. LDS (<= 40 KB) holds the PZ
// handle table and payload pool, the (hash, index) keys and the operand staging buffer.
// Two widths of the same kernel: 128 threads, four workgroups (eight waves) per CU, for batches
// up to JOB_ENGINE_JOBS; 256 threads, two per CU, for batches that fit the chip in one round
// (<= 2 x CUs jobs), where a job's latency is the reach time and the extra waves shorten the large
// operators' passes. Both at the VGPR budget of two waves per SIMD. (Rounds 4-5 also carried a
// third form whose arena lived in LDS, compacted to the live values between ops: bitwise the HBM
// arena, but slower, 3.43 against 3.28 ms per single plan; removed in round 6)
#include "reach.h"

namespace armour {

#ifndef REACH_CFG_THREADS
#define REACH_CFG_THREADS 128
#define REACH_CFG_KEYS 1024
#define REACH_CFG_STAGE 1152
#define REACH_CFG_WG_PER_CU 4
#endif
#ifndef REACH_CFG_WAVES_PER_SIMD
#define REACH_CFG_WAVES_PER_SIMD 2
#endif
constexpr int REACH_THREADS = REACH_CFG_THREADS;   // two waves per job, four jobs resident per CU
constexpr int REACH_WIDE_THREADS = 256;            // four waves per job, two jobs resident per CU
constexpr int REACH_WIDE_PER_CU = 2;
constexpr int KEY_CAP_LDS = REACH_CFG_KEYS;
constexpr int STAGE_DOUBLES = REACH_CFG_STAGE;
constexpr int REACH_WG_PER_CU = REACH_CFG_WG_PER_CU;
constexpr int POOL_DOUBLES = 1024;   // handle payloads (ProgramBuilder::slot_offsets)

// The reach phase's counters: the algorithmic byte count, the capacity maxima occ[8] (arena
// hashes, arena rows, operator terms, link / torque k-only monomials) and the per-world error
// flags. jrs_kernel zeroes them; the reach kernel's last workgroup publishes them in mapped host
// memory (hsum[0] bytes, hsum[1..8] occ, hsum[RSUM_ERR + w] world w's flags, and last
// hsum[RSUM_SEQ] = the launch's sequence number). So the host reads them after one event wait, and
// no fill or copy runs on the reach stream: under concurrent planners such a blit kernel would wait
// for CUs another planner's persistent reach kernel holds. The host checks the sequence number
// before it trusts the other words (a launch whose last workgroup did not publish fails loudly
// instead of leaving the previous batch's flags and capacities in place).
constexpr int RSUM_SEQ = 9;
constexpr int RSUM_ERR = 10;
struct ReachCounters {
    unsigned long long* bytes;  // [1]
    unsigned long long* occ;    // [8]
    unsigned* done;             // [1] workgroups finished (the last one resets it to 0)
    long long* hsum;            // mapped host [RSUM_ERR + W]
    long long seq;              // this launch's sequence number (planner.hip run_reach)
    unsigned* pc_next;          // the plane cache pool counter of the solver (NlpDev::pcnext; may be null)
};

__device__ inline void zero_counters(const ReachCounters& c, int* err, int W) {
    if (blockIdx.x != 0) return;
    for (int k = threadIdx.x; k < W; k += blockDim.x) err[k] = 0;
    if (threadIdx.x < 8) c.occ[threadIdx.x] = 0;
    if (threadIdx.x == 0) *c.bytes = 0;
    if (threadIdx.x == 0 && c.pc_next) *c.pc_next = 0;
}

// The launch's execution span on the device clock (wall_clock64, s_memrealtime): the first
// workgroup's start in occ[5] (as ~t, so that atomicMax keeps the earliest) and the last
// workgroup's end in occ[6], published with the other counters (hsum[6], hsum[7]). This is the
// quantity rocprofv3 --kernel-trace reports as the kernel's duration; HIP events around the launch
// also count the time the kernel waits for CUs that other planners' kernels hold (bench.py's
// roofline takes the span, armour_get_reach_span).
__device__ inline void span_start(const ReachCounters& c) {
    if (threadIdx.x == 0) atomicMax(&c.occ[5], ~(unsigned long long)wall_clock64());
}
// after a workgroup's last job: the last workgroup of the grid copies the counters out (reads
// through device-scope atomics, so every other workgroup's updates are seen)
__device__ inline void publish_counters(const ReachCounters& c, int* err, int W, int* last) {
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicMax(&c.occ[6], (unsigned long long)wall_clock64());
        __threadfence();
        *last = atomicAdd(c.done, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!*last) return;
    __threadfence();
    for (int k = threadIdx.x; k < W; k += blockDim.x) c.hsum[RSUM_ERR + k] = atomicOr(&err[k], 0);
    if (threadIdx.x < 8) c.hsum[1 + threadIdx.x] = (long long)atomicMax(&c.occ[threadIdx.x], 0ull);
    if (threadIdx.x == 0) {
        c.hsum[0] = (long long)atomicAdd(c.bytes, 0ull);
        atomicExch(c.done, 0u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        c.hsum[RSUM_SEQ] = c.seq;  // after every other word of this launch
    }
}

// JRS scalars of every (world, interval, joint) (KPR/Trajectory.cu:63-254), one thread each;
// block 0 also zeroes the reach phase's counters
__global__ void jrs_kernel(const RobotParams* __restrict__ rpp, int W, int T, const double* q0, const double* qd0,
                           const double* qdd0, JrsJoint* out, ReachCounters rc, int* err) {
    zero_counters(rc, err, W);
    const long n = (long)W * T * NF;
    for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
        const int i = (int)(idx % NF);
        const long j = idx / NF;
        const int t = (int)(j % T), w = (int)(j / T);
        out[idx] = jrs_joint(*rpp, T, t, i, q0[w * NF + i], qd0[w * NF + i], qdd0[w * NF + i]);
    }
}

// ARMTD comparison planner (ACMP/Trajectory.cu:29-72): the offline JRS tables of cos / sin of the
// relative joint angle rotated by q0, as the JRS scalars the reach program's MAKEROT reads (the
// k-generator and the radius of the cos / sin 1-D PZs; radius x 5 as :43, :56). tables:
// [W][NF][6][T] = c_cos, g_cos, r_cos, c_sin, g_sin, r_sin (armtd_main.cu:70-90)
__global__ void jrs_armtd_kernel(int W, int T, const double* q0, const double* tables, JrsJoint* out, ReachCounters rc,
                                 int* err) {
    zero_counters(rc, err, W);
    const long n = (long)W * T * NF;
    for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
        const int i = (int)(idx % NF);
        const long j = idx / NF;
        const int t = (int)(j % T), w = (int)(j / T);
        const double* tb = tables + ((long)w * NF + i) * 6 * T;
        const double c_cos = tb[0 * T + t], g_cos = tb[1 * T + t], r_cos = tb[2 * T + t];
        const double c_sin = tb[3 * T + t], g_sin = tb[4 * T + t], r_sin = tb[5 * T + t];
        const double cq = cos(q0[w * NF + i]), sq = sin(q0[w * NF + i]);
        JrsJoint J = {};
        J.cos_c = cq * c_cos - sq * c_sin;
        J.cos_k = cq * g_cos - sq * g_sin;
        J.cos_e = (fabs(cq) * r_cos + fabs(sq) * r_sin) * 5.0;
        J.sin_c = cq * c_sin + sq * c_cos;
        J.sin_k = cq * g_sin + sq * g_cos;
        J.sin_e = (fabs(cq) * r_sin + fabs(sq) * r_cos) * 5.0;
        out[idx] = J;
    }
}

struct ReachArgs {
    int W, T;
    const JrsJoint* jrs;  // [W][T][NF] from jrs_kernel
    const double* q0;    // [W][NF]
    const double* qd0;
    const double* qdd0;
    const Op* prog;      // reach program (device copy of ProgramBuilder::ops)
    int nops;
    const int* slot_off; // payload offset of every handle slot in the LDS pool
    int nslots;
    uint64_t* arena_h;   // [grid][arena_cap]
    double* arena_c;     // [grid][arena_cap * 3]
    long arena_cap;
    uint64_t* gkh;       // [grid][gcap]
    uint32_t* gki;
    int* gkp;
    int gcap;
    double* gout;        // [grid][gcap * 9]
    unsigned long long* bytes;  // algorithmic monomial bytes of all jobs (one atomic per job)
    ReachCounters rc;           // rc.occ[3] / [4]: largest link / torque k-only monomial counts
    int ntq;                    // torque PZs per job (NF; the ARMTD program has none)
    unsigned long long* prof;   // optional per-op [cycles, terms] (null: off)
    int mode;                   // engine diagnostics (Ctx::mode)
    unsigned long long* phase;  // optional phase cycle totals [16] (null: off; exclusive with prof)
    double* dump;               // optional op-by-op state of job 0 (null: off)
};

// 2 waves per SIMD: 256 registers per lane (VGPR + AGPR); NT threads per job
template <int NT>
__global__ __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(REACH_CFG_WAVES_PER_SIMD, REACH_CFG_WAVES_PER_SIMD))) void reach_kernel(const RobotParams* __restrict__ rpp, ReachArgs a, ReachOut out) {
    __shared__ PZH H[MAX_SLOTS];
    __shared__ double pool[POOL_DOUBLES + 9];  // + 9: header reads of a full 3x3 past a small slot
    __shared__ uint64_t kh[KEY_CAP_LDS];
    __shared__ uint32_t ki[KEY_CAP_LDS];
    __shared__ int kp[KEY_CAP_LDS];
    __shared__ double stage[STAGE_DOUBLES];
    __shared__ double red[(NT / 64) * 18];
    __shared__ int iscan[NT / 64];
    __shared__ Arena arena;
    __shared__ int err;
    __shared__ JrsJoint jrs[NF];
    __shared__ double scratch[2 * NF];
    __shared__ double q0s[NF], qd0s[NF], qdd0s[NF];
    __shared__ unsigned long long phase_acc[16];
    __shared__ int last;

    span_start(a.rc);
    const RobotParams& rp = *rpp;
    Ctx x;
    x.g = Grp{(int)threadIdx.x, (int)blockDim.x};
    x.H = H;
    x.pool = pool;
    x.A = &arena;
    x.ah = a.arena_h + (long)blockIdx.x * a.arena_cap;
    x.ac = a.arena_c + (long)blockIdx.x * a.arena_cap * 3;
    for (int k = threadIdx.x; k < a.nslots; k += blockDim.x) H[k].off = a.slot_off[k];
    x.kh = kh; x.ki = ki; x.kp = kp; x.cap_lds = KEY_CAP_LDS;
    x.gkh = a.gkh + (long)blockIdx.x * a.gcap;
    x.gki = a.gki + (long)blockIdx.x * a.gcap;
    x.gkp = a.gkp + (long)blockIdx.x * a.gcap;
    x.cap_glb = a.gcap;
    x.gout = a.gout + (long)blockIdx.x * a.gcap * 9;
    x.stage = stage;
    x.stage_cap = STAGE_DOUBLES;
    x.red = red;
    x.iscan = iscan;
    x.err = &err;
    x.thr = rp.simplify_threshold;
    x.phase = a.phase ? phase_acc : nullptr;
    if (threadIdx.x < 16) phase_acc[threadIdx.x] = 0;
    x.mode = a.mode;

    const long njobs = (long)a.W * a.T;
    for (long job = blockIdx.x; job < njobs; job += gridDim.x) {
        const int w = (int)(job / a.T), t = (int)(job % a.T);
        if (threadIdx.x == 0) {
            arena.hcap = a.arena_cap;
            arena.ccap = a.arena_cap * 3;
            arena.hused = 0;
            arena.cused = 0;
            arena.bytes = 0;
            err = 0;
        }
        if (threadIdx.x < NF) {
            q0s[threadIdx.x] = a.q0[w * NF + threadIdx.x];
            qd0s[threadIdx.x] = a.qd0[w * NF + threadIdx.x];
            qdd0s[threadIdx.x] = a.qdd0[w * NF + threadIdx.x];
        }
        __syncthreads();
        run_program(x, rp, a.prog, a.nops, a.T, t, q0s, qd0s, qdd0s, out, job, jrs, scratch, a.prof,
                    job == 0 ? a.dump : nullptr, a.jrs + job * NF);
        if (threadIdx.x == 0) {
            if (err) atomicOr(&out.err[w], err);
            atomicAdd(a.bytes, (unsigned long long)arena.bytes);
            // this job's largest kept monomial counts (written by this thread in t0_emit_*), which
            // size the evaluation kernels (planner.hip eval_small_fits)
            int lm = 0, um = 0;
            for (int l = 0; l < out.NJ; l++) lm = max(lm, out.link_cnt[job * out.NJ + l]);
            for (int i = 0; i < a.ntq; i++) um = max(um, out.tq_cnt[job * NF + i]);
            atomicMax(&a.rc.occ[3], (unsigned long long)lm);
            atomicMax(&a.rc.occ[4], (unsigned long long)um);
        }
        if (a.phase && threadIdx.x < 16) {
            atomicAdd(&a.phase[threadIdx.x], phase_acc[threadIdx.x]);
            phase_acc[threadIdx.x] = 0;
        }
        __syncthreads();
    }
    publish_counters(a.rc, out.err, a.W, &last);
}

}  // namespace armour
