// armour-mi355x — host runtime and C ABI (include/armour_hip.h).
//
// One planner handle owns a HIP stream and every device buffer for up to max_worlds worlds of
// T time steps and max_obstacles obstacles, allocated once (the reference allocates per process,
// KPR/CollisionChecking.cu:17-53). A batch runs entirely on the device:
//   reach_kernel (JRS + PZ FK/RNEA + torque radius) -> bounds_kernel ->
//   armour-IPM passes (eval_kernel_t + ipm_rows_* / ipm_world_*) -> feasible_kernel;
// the host only sequences launches and reads one flag word per line-search round.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <string>
#include <vector>

#include "../../include/armour_hip.h"
#include "nlp_kernels.hip"
#include "reach_kernel.hip"
#include "lane_kernel.hip"
#include "robots.h"

using namespace armour;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCK(expr)                                                                               \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail(ARMOUR_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
hipError_t dalloc(T** p, size_t n) {
    return hipMalloc((void**)p, sizeof(T) * (n > 0 ? n : 1));
}
}  // namespace

// planners alive per device (armour_create / armour_destroy): the bundle kernel's shape depends on
// whether the GPU is shared (lane_shape_for)
static std::atomic<int> g_planners[64];

struct armour_planner {
    armour_config cfg;
    int T = 0, NJ = 0, Omax = 0, Wmax = 0, ncu = 0, reach_grid = 0;
    RobotParams rp;
    RobotParams* d_rp = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t rstream = nullptr;   // reach phase (the planner's stream unless CUs are reserved)
    int reach_cus = 0;               // CUs the reach stream may use
    hipEvent_t ev[6];
    hipEvent_t tev[2];        // sync-free solver tail: end of iteration it (parity it & 1)
    int tail_worlds = 16;     // sync-free tail below this many running worlds (ARMOUR_TAIL_WORLDS, 0: off)
    // reach program (ProgramBuilder::ops) on the device
    Op* d_prog = nullptr;
    int* d_slot_off = nullptr;
    JrsJoint* d_jrs = nullptr;
    int nops = 0, nslots = 0;
    unsigned long long* d_bytes = nullptr;
    unsigned long long* d_prof = nullptr;  // per-op [cycles, terms] when ARMOUR_PROFILE_OPS is set
    double* d_dump = nullptr;              // op-by-op state of job 0 when ARMOUR_DUMP_OPS is set
    double last_kernel_ms = 0, last_bytes = 0;
    double last_span_ms = -1;  // device-clock execution span of the last reach launch (armour_get_reach_span)
    int wall_khz = 0;          // hipDeviceAttributeWallClockRate
    unsigned long long* d_occ = nullptr;   // [8] reach capacity use of the last launch (ReachCounters)
    unsigned* d_done = nullptr;            // workgroups finished in the current reach launch
    long long* h_sum = nullptr;            // mapped host: reach counters published by the last workgroup
    ReachCounters rc{};                    // (reach_kernel.hip)
    long long reach_seq = 0;               // sequence number of the last reach launch (ReachCounters::seq)
    int* d_wlist = nullptr;                // [max_worlds] worlds of a capacity retry
    int last_retried = 0, last_failed = 0;
    std::vector<int> world_err;            // per world of the last batch: 0 or ARMOUR_E_CAPACITY
    // inputs
    double *q0 = nullptr, *qd0 = nullptr, *qdd0 = nullptr, *qdes = nullptr, *obs = nullptr, *xin = nullptr;
    // reach
    ReachOut ro;
    ReachArgs ra;
    // bundle engine (lane_kernel.hip): default; ARMOUR_ENGINE=job selects the per-job reach_kernel
    bool lane_engine = true;  // the last batch ran on the bundle engine
    bool has_lane = false, has_job = false;  // engines with buffers
    bool armtd = false;       // the ARMTD comparison planner (armour_create_armtd)
    double* d_tables = nullptr;  // ARMTD: offline JRS tables [W][NF][6][T]
    long job_max = 0;         // batches of at most this many jobs (W x T) run on the per-job engine
    bool job_fits = true;     // the reach program's payload pool fits the per-job engine's LDS
    bool job_narrow = false;  // ARMOUR_REACH_WIDE=0 (diagnostics): small batches on the 128-thread kernel too
    bool eval_f32 = false;    // ARMOUR_EVAL_F32: fp32 constraint evaluation (tolerance study only)
    bool eval_full = false;   // ARMOUR_EVAL_FULL: always the full-capacity evaluation kernels
    // largest link / torque k-monomial counts of the last reach (both engines record them in
    // occ[3], occ[4], published with the error flags), and the first launch's occupancy
    unsigned long long h_occ[8] = {};
    int mono_max[2] = {CAP_LM, CAP_UM};
    int lane_grid = 0;        // workgroups with an arena: the larger (dense) shape's resident set
    int lane_slots[2] = {0, 0};  // resident bundle workgroups of the wide / dense kernel shape
    int lane_shape = -1;      // ARMOUR_LANE_SHAPE: 0 wide, 1 dense, -1 chosen per launch
    int last_shape = 0;       // shape of the last first launch (a capacity retry uses it too)
    int dev = 0;              // the planner's device
    bool counted = false;     // counted in g_planners[dev]
    bool device_shared = false;  // ARMOUR_DEVICE_SHARED=1: other processes plan on this GPU too
    lane::LaneArgs la;

    // nlp
    NlpDev d;
    int* feas = nullptr;
    int* h_flags = nullptr;   // pinned host, mapped (NlpDev::flags)
    int* d_lists = nullptr;   // [6][max_worlds] active-world lists of the solver
    bool spec = true;         // speculative line-search rounds (ARMOUR_NO_SPEC: sequential only)
    bool spec_all = true;     // the sync-free tail's one-round line search (eval_trials_all, ipm_world_Cs_all)
    bool resto_spec = false;  // the restoration phase's one-round search (eval_trials_all, resto_world_Vs)
    bool resto_inline = true; // restoration phases inside the interior-point loop (ARMOUR_RESTO_INLINE=0: after it)
    bool da_lds = true;       // wide grids take ipm_rows_DA_lds (ARMOUR_DA_REGS=1: the register form)
    // In the sync-free tail the inline restoration phase runs on a second stream, concurrently with
    // the next interior-point iteration (ARMOUR_RESTO_CONCURRENT=0: on the solver stream): its worlds
    // are others than the interior point's, and its speculative rows start after the tail's
    // (resto_soff rows into gs / fs / partial_s), so only the append list RL is shared; ipm_loop
    // orders its publication (ev_ip, ev_pub) and joins the streams at the loop's end (ev_rend)
    bool resto_conc = false;
    hipStream_t rstream2 = nullptr;
    hipEvent_t ev_ip = nullptr, ev_pub = nullptr, ev_rend = nullptr;
    size_t resto_soff = 0;
    int tail_search = 1;      // its use (ARMOUR_TAIL_SEARCH): 0 rounds only, 1 adaptive, 2 always
    WorldState* h_ws = nullptr;
    double* h_f = nullptr;
    int* h_feas = nullptr;
    unsigned* h_pcnext = nullptr;  // pinned: the plane cache pool records the last build needed
    // state of the last batch
    int W = 0, O = 0;
    bool reached = false, planned = false;
    std::vector<void*> allocs;

    template <class T>
    int alloc(T** p, size_t n) {
        hipError_t e = dalloc(p, n);
        if (e != hipSuccess) return fail(ARMOUR_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
        allocs.push_back((void*)*p);
        return 0;
    }
};

// rows per block of the IPM row passes (ARMOUR_ROW_CHUNK overrides for diagnostics, a multiple of
// 256). Measured at 327 worlds (tools/chunk_sweep.sh): 2048 rows 34.8 ms of NLP, 1024 34.2 ms, 512
// 36.5 ms, 256 43.1 ms: shorter per-thread row loops help the latency-bound tail iterations until
// the per-block reductions dominate.
static int row_chunk() {
    const char* e = std::getenv("ARMOUR_ROW_CHUNK");
    const int c = e ? std::atoi(e) : 1024;
    return (c >= 256 && c % 256 == 0) ? c : 1024;
}

// capacity retry: a quarter of the workgroups, each with four workgroups' buffers
constexpr int RETRY_SCALE = 4;

// largest batch (jobs = worlds x T) that runs on the per-job engine; measured crossover, DESIGN.md §4
constexpr long JOB_ENGINE_JOBS = 5120;

static int planner_init(armour_planner* p, const armour_config* cfg, const armour_robot* robot, bool armtd = false) {
    p->cfg = *cfg;
    p->armtd = armtd;
    if (!robot && cfg->robot != 0) return fail(ARMOUR_E_ARG, "unknown robot id");
    if (cfg->num_time_steps <= 0 || (cfg->num_time_steps % 2) != 0)
        return fail(ARMOUR_E_ARG, "num_time_steps must be a positive even number (KPR/Parameters.h:16)");
    if (cfg->max_obstacles < 0 || cfg->max_obstacles > MAX_OBS || cfg->max_worlds <= 0)
        return fail(ARMOUR_E_ARG, "bad max_obstacles (0..40, MAX_OBSTACLE_NUM) / max_worlds");
    if (cfg->device >= 0) HIPCK(hipSetDevice(cfg->device));
    int dev = 0;
    HIPCK(hipGetDevice(&dev));
    p->dev = dev;
    g_planners[dev & 63]++;
    p->counted = true;
    // g_planners sees this process's planners only; planners of other processes on the same GPU
    // (torchrun ranks folded onto one device, several armour_main servers) are declared with
    // ARMOUR_DEVICE_SHARED=1 (it only chooses the bundle kernel's shape)
    if (const char* e = std::getenv("ARMOUR_DEVICE_SHARED")) p->device_shared = std::atoi(e) != 0;
    HIPCK(hipDeviceGetAttribute(&p->ncu, hipDeviceAttributeMultiprocessorCount, dev));
    if (hipDeviceGetAttribute(&p->wall_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) p->wall_khz = 0;
    if (robot) {
        if (!robot_from_tables(*robot, p->rp))
            return fail(ARMOUR_E_ARG, "invalid robot tables (num_joints 7..9, actuated joints first, M_min > 0, K > 0)");
    } else {
        kinova_gen3(p->rp);
    }
    p->T = cfg->num_time_steps;
    p->NJ = p->rp.num_joints;
    p->Omax = cfg->max_obstacles;
    p->Wmax = cfg->max_worlds;
    {
        // Concurrent planners share the GPU. The bundle reach kernel holds every CU it runs on for
        // its whole launch (persistent, 2 workgroups x 78 KB LDS per CU), so another planner's solver
        // kernels wait for it. ARMOUR_REACH_CU_RESERVE=k keeps k CUs out of the reach stream's CU mask
        // for them; ARMOUR_SOLVER_PRIORITY=1 gives the solver stream the highest queue priority.
        const char* pr = std::getenv("ARMOUR_SOLVER_PRIORITY");
        int lo = 0, hi = 0;
        HIPCK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        const int prio = (pr && std::atoi(pr) != 0) ? hi : 0;
        HIPCK(hipStreamCreateWithPriority(&p->stream, hipStreamNonBlocking, prio));
        const char* rv = std::getenv("ARMOUR_REACH_CU_RESERVE");
        const int reserve = rv ? std::atoi(rv) : 0;
        p->reach_cus = p->ncu;
        if (reserve > 0 && reserve < p->ncu) {
            std::vector<uint32_t> mask((p->ncu + 31) / 32, 0u);
            for (int c = 0; c < p->ncu; c++) mask[c / 32] |= 1u << (c % 32);
            for (int i = 0; i < reserve; i++) {
                const int c = (int)((long)i * p->ncu / reserve);
                mask[c / 32] &= ~(1u << (c % 32));
            }
            HIPCK(hipExtStreamCreateWithCUMask(&p->rstream, (uint32_t)mask.size(), mask.data()));
            p->reach_cus = p->ncu - reserve;
        } else {
            p->rstream = p->stream;
        }
    }
    for (int i = 0; i < 6; i++) HIPCK(hipEventCreate(&p->ev[i]));
    for (int i = 0; i < 2; i++) HIPCK(hipEventCreateWithFlags(&p->tev[i], hipEventDisableTiming));
    if (const char* e = std::getenv("ARMOUR_TAIL_WORLDS")) p->tail_worlds = std::atoi(e);
    p->da_lds = !std::getenv("ARMOUR_DA_REGS");
    if (const char* e = std::getenv("ARMOUR_TAIL_SEARCH"))
        p->tail_search = !std::strcmp(e, "rounds") ? 0 : !std::strcmp(e, "one") ? 2 : 1;
    const int T = p->T, NJ = p->NJ, Om = p->Omax > 0 ? p->Omax : 1, Wm = p->Wmax;
    int rc = 0;
    if ((rc = p->alloc(&p->d_rp, 1))) return rc;
    HIPCK(hipMemcpy(p->d_rp, &p->rp, sizeof(RobotParams), hipMemcpyHostToDevice));
    if ((rc = p->alloc(&p->q0, (size_t)Wm * NF)) || (rc = p->alloc(&p->qd0, (size_t)Wm * NF)) ||
        (rc = p->alloc(&p->qdd0, (size_t)Wm * NF)) || (rc = p->alloc(&p->qdes, (size_t)Wm * NF)) ||
        (rc = p->alloc(&p->xin, (size_t)Wm * NF)) || (rc = p->alloc(&p->obs, (size_t)Wm * Om * 12)))
        return rc;
    // reach outputs
    const size_t jobs = (size_t)Wm * T;
    ReachOut& ro = p->ro;
    ro.T = T;
    ro.NJ = NJ;
    if ((rc = p->alloc(&ro.link_hash, jobs * NJ * CAP_LM)) || (rc = p->alloc(&ro.link_coef, jobs * NJ * CAP_LM * 3)) ||
        (rc = p->alloc(&ro.link_cnt, jobs * NJ)) || (rc = p->alloc(&ro.link_center, jobs * NJ * 3)) ||
        (rc = p->alloc(&ro.link_rad, jobs * NJ * 3)) || (rc = p->alloc(&ro.link_gens, jobs * NJ * 18)) ||
        (rc = p->alloc(&ro.tq_hash, jobs * NF * CAP_UM)) || (rc = p->alloc(&ro.tq_coef, jobs * NF * CAP_UM)) ||
        (rc = p->alloc(&ro.tq_cnt, jobs * NF)) || (rc = p->alloc(&ro.tq_center, jobs * NF)) ||
        (rc = p->alloc(&ro.tq_rad, jobs * NF)) || (rc = p->alloc(&ro.torque_radius, jobs * NF)) ||
        (rc = p->alloc(&ro.err, (size_t)Wm)))
        return rc;
    // reach program
    {
        ProgramBuilder pb;
        pb.build(p->rp, p->armtd);
        int pool = 0;
        const std::vector<int> off = pb.slot_offsets(&pool);
        {
            const char* eng = std::getenv("ARMOUR_ENGINE");
            const bool job_engine = eng && std::strcmp(eng, "job") == 0;
            // the bundle engine's payload pool lives in HBM, sized below; the per-job engine's in LDS
            // (POOL_DOUBLES): a robot whose program does not fit it (Fetch: 8 links) runs on the
            // bundle engine only
            p->job_fits = pool <= POOL_DOUBLES;
            if (pb.nslots > MAX_SLOTS || (job_engine && pool > POOL_DOUBLES)) {
                char buf[200];
                std::snprintf(buf, sizeof(buf), "reach program needs %d handle slots (kernel: %d) and %d payload doubles (per-job engine: %d)",
                              pb.nslots, MAX_SLOTS, pool, POOL_DOUBLES);
                return fail(ARMOUR_E_CAPACITY, buf);
            }
        }
        p->nops = (int)pb.ops.size();
        p->nslots = pb.nslots;
        if ((rc = p->alloc(&p->d_prog, pb.ops.size())) || (rc = p->alloc(&p->d_bytes, 1)) ||
            (rc = p->alloc(&p->d_slot_off, off.size())))
            return rc;
        HIPCK(hipMemcpy(p->d_prog, pb.ops.data(), sizeof(Op) * pb.ops.size(), hipMemcpyHostToDevice));
        HIPCK(hipMemcpy(p->d_slot_off, off.data(), sizeof(int) * off.size(), hipMemcpyHostToDevice));
        if (std::getenv("ARMOUR_PROFILE_OPS")) {
            // =3: no op profiling; [start, end] wall clock (100 MHz) of every bundle of the last launch
            // after the op tables (bundle-engine load balance)
            const size_t nbt = 2 * (((size_t)p->Wmax * p->T + lane::LG - 1) / lane::LG);
            const size_t n = 2 * pb.ops.size() + 16 + 8 * OP_NCODES + nbt;
            if ((rc = p->alloc(&p->d_prof, n))) return rc;
            HIPCK(hipMemset(p->d_prof, 0, sizeof(unsigned long long) * n));
        }
    }
    // reach workspace: four resident workgroups per CU, each with a private arena
    {
        // ARMOUR_REACH_WG_PER_CU (diagnostics): fewer resident workgroups per CU than the 4 that fit
        const char* wg = std::getenv("ARMOUR_REACH_WG_PER_CU");
        int fit = REACH_WG_PER_CU;  // as many as the CU's LDS holds (a persistent grid larger than
        {                           // the resident set would run its last workgroups one job late)
            hipFuncAttributes fa{};
            int lds_cu = 0;
            HIPCK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&reach_kernel<REACH_THREADS>)));
            HIPCK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
            if (fa.sharedSizeBytes > 0) fit = std::max(1, std::min<int>(fit, (int)(lds_cu / fa.sharedSizeBytes)));
        }
        const int per = wg ? std::atoi(wg) : fit;
        p->reach_grid = (per >= 1 && per <= fit ? per : fit) * p->ncu;
    }
    // Engine choice per batch. The bundle engine (lane_kernel.hip) runs 64 jobs per workgroup and
    // fills the chip from ~2 x CUs x 64 jobs on, but one bundle takes ~18 ms whatever its size. The
    // per-job engine (reach_kernel.hip) runs one job per workgroup, ~4 ms per round of up to
    // 4 x CUs jobs. So small batches (the drop-in's single plan) take the per-job engine:
    // batches of at most job_max jobs (ARMOUR_JOB_ENGINE_JOBS; ARMOUR_ENGINE=job|lane forces one).
    {
        const char* eng = std::getenv("ARMOUR_ENGINE");
        const char* jm = std::getenv("ARMOUR_JOB_ENGINE_JOBS");
        p->job_max = jm ? std::atol(jm) : JOB_ENGINE_JOBS;
        const char* wide = std::getenv("ARMOUR_REACH_WIDE");
        p->job_narrow = wide && std::atoi(wide) == 0;
        if (eng && std::strcmp(eng, "job") == 0) p->job_max = (long)Wm * T;
        if ((eng && std::strcmp(eng, "lane") == 0) || !p->job_fits) p->job_max = 0;
        p->has_job = p->job_max > 0;
        p->has_lane = (long)Wm * T > p->job_max;
        if (p->has_job) p->reach_grid = (int)std::min<long>(p->reach_grid, std::min<long>(p->job_max, (long)Wm * T));
    }
    ReachArgs& ra = p->ra;
    ra.prog = p->d_prog;
    ra.nops = p->nops;
    ra.slot_off = p->d_slot_off;
    ra.nslots = p->nslots;
    ra.bytes = p->d_bytes;
    // ARMOUR_PROFILE_OPS=1: per-op cycles/terms; =2: phase totals (each distorts the other)
    const char* pm = std::getenv("ARMOUR_PROFILE_OPS");
    ra.prof = (pm && std::atoi(pm) == 2) ? nullptr : p->d_prof;
    ra.phase = (pm && std::atoi(pm) == 2) ? p->d_prof + 2 * p->nops : nullptr;
    ra.mode = std::getenv("ARMOUR_ENGINE_MODE") ? std::atoi(std::getenv("ARMOUR_ENGINE_MODE")) : 0;
    ra.dump = nullptr;
    if (std::getenv("ARMOUR_DUMP_OPS")) {
        if ((rc = p->alloc(&p->d_dump, (size_t)p->nops * DUMP_W))) return rc;
        HIPCK(hipMemset(p->d_dump, 0, sizeof(double) * p->nops * DUMP_W));
        ra.dump = p->d_dump;
    }
    if ((rc = p->alloc(&p->d_jrs, jobs * NF)) || (rc = p->alloc(&p->d_occ, 8)) || (rc = p->alloc(&p->d_done, 1))) return rc;
    HIPCK(hipMemset(p->d_done, 0, sizeof(unsigned)));
    {
        long long* dsum = nullptr;
        HIPCK(hipHostMalloc((void**)&p->h_sum, sizeof(long long) * (RSUM_ERR + (size_t)Wm), hipHostMallocMapped));
        HIPCK(hipHostGetDevicePointer((void**)&dsum, p->h_sum, 0));
        p->rc = ReachCounters{p->d_bytes, p->d_occ, p->d_done, dsum, 0};
        p->h_sum[RSUM_SEQ] = 0;
        ra.rc = p->rc;
        ra.ntq = p->armtd ? 0 : NF;
    }
    {
        const char* f32 = std::getenv("ARMOUR_EVAL_F32");
        p->eval_f32 = f32 && std::atoi(f32) != 0;
        const char* ef = std::getenv("ARMOUR_EVAL_FULL");
        p->eval_full = ef && std::atoi(ef) != 0;
    }
    if (p->has_job) {
        ra.arena_cap = 1 << 17;
        ra.gcap = 1 << 15;
        if ((rc = p->alloc(&ra.arena_h, (size_t)p->reach_grid * ra.arena_cap)) ||
            (rc = p->alloc(&ra.arena_c, (size_t)p->reach_grid * ra.arena_cap * 3)) ||
            (rc = p->alloc(&ra.gkh, (size_t)p->reach_grid * ra.gcap)) || (rc = p->alloc(&ra.gki, (size_t)p->reach_grid * ra.gcap)) ||
            (rc = p->alloc(&ra.gkp, (size_t)p->reach_grid * ra.gcap)) ||
            (rc = p->alloc(&ra.gout, (size_t)p->reach_grid * ra.gcap * 9)))
            return rc;
    }
    if (p->has_lane) {
        // LANE_WG_PER_CU resident bundle workgroups per CU (as many as the CU's LDS holds), each
        // with its own arena; sizes from the measured per-job use (~16.5k monomials) times the union
        // inflation, with margin
        lane::LaneArgs& la = p->la;
        const long bundles = ((long)Wm * T + lane::LG - 1) / lane::LG;
        {
            int lds_cu = 0;
            HIPCK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
            const void* fn[2] = {reinterpret_cast<const void*>(&lane::lane_reach_kernel<lane::LaneWide>),
                                 reinterpret_cast<const void*>(&lane::lane_reach_kernel<lane::LaneDense>)};
            const int want[2] = {lane::LaneWide::PER_CU, lane::LaneDense::PER_CU};
            for (int k = 0; k < 2; k++) {
                hipFuncAttributes fa{};
                HIPCK(hipFuncGetAttributes(&fa, fn[k]));
                int per_cu = want[k];
                if (fa.sharedSizeBytes > 0) per_cu = std::max(1, std::min<int>(per_cu, (int)(lds_cu / fa.sharedSizeBytes)));
                p->lane_slots[k] = p->reach_cus * per_cu;
            }
            const char* sh = std::getenv("ARMOUR_LANE_SHAPE");
            if (sh && std::strcmp(sh, "wide") == 0) p->lane_shape = 0;
            if (sh && std::strcmp(sh, "dense") == 0) p->lane_shape = 1;
        }
        const long slots = std::max(p->lane_slots[0], p->lane_slots[1]);
        p->lane_grid = (int)(bundles < slots ? bundles : slots);
        const char* hc = std::getenv("ARMOUR_LANE_HCAP");
        const char* cc = std::getenv("ARMOUR_LANE_CCAP");
        la.hcap = hc ? std::atol(hc) : (1L << 16);
        la.ccap = cc ? std::atol(cc) : (1L << 17);
        la.gcap = 1 << 15;
        la.ocap = 4096;
        int pool = 0;
        {
            ProgramBuilder pb;
            pb.build(p->rp, p->armtd);
            (void)pb.slot_offsets(&pool);
        }
        la.pool_rows = pool + 9 + 2 * NF;  // + the torque-radius scratch rows (lane_kernel.hip)
        // buffers of at least RETRY_SCALE workgroups, so even a one-world batch has a capacity retry
        const size_t G = (size_t)std::max(p->lane_grid, RETRY_SCALE), LGs = lane::LG;
        if ((rc = p->alloc(&la.pool, G * la.pool_rows * LGs)) || (rc = p->alloc(&la.arena_h, G * la.hcap)) ||
            (rc = p->alloc(&la.arena_m, G * la.hcap)) || (rc = p->alloc(&la.arena_c, G * la.ccap * LGs)) ||
            (rc = p->alloc(&la.gkh, G * la.gcap)) || (rc = p->alloc(&la.gki, G * la.gcap)) ||
            (rc = p->alloc(&la.gkp, G * (la.gcap + 1))) || (rc = p->alloc(&la.ggp, G * (la.gcap + 1))) ||
            (rc = p->alloc(&la.gout, G * la.ocap * 9 * LGs)) || (rc = p->alloc(&la.gm, G * la.ocap)))
            return rc;
        if ((rc = p->alloc(&p->d_wlist, (size_t)Wm))) return rc;
        la.occ = p->d_occ;
        la.rc = p->rc;
        la.wlist = nullptr;
        la.nlist = 0;
        la.prog = p->d_prog;
        la.nops = p->nops;
        la.slot_off = p->d_slot_off;
        la.nslots = p->nslots;
        la.bytes = p->d_bytes;
        const bool btimes = pm && std::atoi(pm) == 3;
        la.prof = btimes ? nullptr : p->d_prof;
        la.btime = btimes ? p->d_prof + 2 * p->nops + 16 + 8 * OP_NCODES : nullptr;
        la.dump = nullptr;
        if (p->d_dump) {
            (void)hipFree(p->d_dump);
            p->allocs.erase(std::find(p->allocs.begin(), p->allocs.end(), (void*)p->d_dump));
            if ((rc = p->alloc(&p->d_dump, (size_t)p->nops * DUMP_W * lane::LG))) return rc;
            HIPCK(hipMemset(p->d_dump, 0, sizeof(double) * p->nops * DUMP_W * lane::LG));
            la.dump = p->d_dump;
            ra.dump = nullptr;  // the op dump follows the bundle engine when it exists
        }
    }
    // NLP
    NlpDev& d = p->d;
    d.rp = p->d_rp;
    d.diag = std::getenv("ARMOUR_EVAL_SKIP") ? std::atoi(std::getenv("ARMOUR_EVAL_SKIP")) : 0;
    d.T = T;
    d.NJ = NJ;
    d.ro = ro;
    if (cfg->max_iter > 0) d.opt.max_iter = cfg->max_iter;
    if (const char* ms = std::getenv("ARMOUR_MU_STRATEGY"))  // adaptive (default) or monotone
        d.opt.mu_strategy = std::strcmp(ms, "monotone") == 0 ? 0 : 1;
    if (const char* rs = std::getenv("ARMOUR_RESTORATION"))  // restoration phases per solve (0: none)
        d.opt.resto_max = std::atoi(rs) < 0 ? 0 : std::atoi(rs);
    d.resto = 0;
    d.armtd = p->armtd ? 1 : 0;
    d.nt = p->armtd ? 0 : NF * T;
    d.krange = nullptr;
    if (p->armtd) {
        d.opt.tol = 1e-7;  // IPOPT_OPTIMIZATION_TOLERANCE (ACMP/Parameters.h:42)
        double* kr = nullptr;
        if ((rc = p->alloc(&p->d_tables, (size_t)Wm * NF * 6 * T)) || (rc = p->alloc(&kr, (size_t)Wm * NF))) return rc;
        d.krange = kr;
    }
    d.lcs = (long)(jobs * NJ * 3);
    const size_t mmax = (size_t)d.nt + (size_t)T * NJ * Om + NF * 4;
    const size_t Rmax = mmax + NF;
    if ((rc = p->alloc(&d.L, Wm * Rmax)) || (rc = p->alloc(&d.U, Wm * Rmax)) || (rc = p->alloc(&d.g, 2 * Wm * mmax)) ||
        (rc = p->alloc(&d.J, 2 * Wm * mmax * NF)) || (rc = p->alloc(&d.f, 2 * (size_t)Wm)) ||
        (rc = p->alloc(&d.grad, 2 * (size_t)Wm * NF)) || (rc = p->alloc(&d.link_c, 3 * jobs * NJ * 3)))
        return rc;
    d.njn = (long)(jobs * NJ * Om * 3);
    d.njd = (long)(jobs * NJ * NF * 3);
    if ((rc = p->alloc(&d.jn, 2 * (size_t)d.njn)) || (rc = p->alloc(&d.jd, 2 * (size_t)d.njd))) return rc;
    double** rowbufs[] = {&d.slo, &d.shi, &d.zlo, &d.zhi, &d.dslo, &d.dshi};
    for (double** b : rowbufs)
        if ((rc = p->alloc(b, Wm * Rmax))) return rc;
    const int nblk_max = (int)((Rmax + row_chunk() - 1) / row_chunk());
    if ((rc = p->alloc(&d.partial, (size_t)Wm * nblk_max * KA)) || (rc = p->alloc(&d.partial2, (size_t)Wm * nblk_max * KA2)) ||
        (rc = p->alloc(&d.ws, (size_t)Wm)) ||
        (rc = p->alloc(&p->feas, (size_t)Wm)))
        return rc;
    // the solver's counts for the host live in mapped host memory (NlpDev::flags: [0, 1] a round's
    // running / searching worlds, [2, 8) the sync-free tail's lagged counts, [8, 10) the concurrent
    // restoration's published list lengths): kernels store them, the host reads them after an
    // event or a synchronised round (no fill or copy per round)
    HIPCK(hipHostMalloc((void**)&p->h_flags, 12 * sizeof(int), hipHostMallocMapped));
    HIPCK(hipHostGetDevicePointer((void**)&d.flags, p->h_flags, 0));
    // active-world lists: two per iteration (ping-pong), two per line-search round
    // (+ two for the restoration phases inside the interior-point loop)
    if ((rc = p->alloc(&p->d_lists, 6 * (size_t)Wm)) || (rc = p->alloc(&d.cnt, 16))) return rc;
    // certified plane cache: one record pool sized for PC_K records per (link, obstacle) pair of
    // every (world, t) (ARMOUR_PC_K, 1..36); each (world, t) block takes its records from the pool
    // with one atomic (pcbase). The survey workload keeps 5.3 planes per pair on average. A build
    // that needs more than the pool is repeated on a larger pool (ensure_plane_cache); if that pool
    // cannot be allocated, the cache is not marked ready and the solve runs on the full scan
    // (bitwise the same results, slower). Round 4 reserved all 36 per pair (42 MB per world at
    // T = 100, O = 20), which capped the batch a GPU can hold. The pool counter is 32-bit: a batch
    // whose 36 records per pair could exceed it does not use the cache.
    d.pcache = !(std::getenv("ARMOUR_PLANE_CACHE") && std::atoi(std::getenv("ARMOUR_PLANE_CACHE")) == 0) &&
               (double)COMB * NJ * std::max(Om, 1) * (double)jobs < 4294967295.0;
    d.pcready = 0;
    {
        const char* pk = std::getenv("ARMOUR_PC_K");
        const int k = pk ? std::atoi(pk) : PC_K;
        d.pc_pool = std::max(1L, (long)std::min(std::max(k, 1), COMB) * NJ * std::max(Om, 1) * (long)jobs);
    }
    if (d.pcache && ((rc = p->alloc(&d.pc, 5 * (size_t)d.pc_pool)) || (rc = p->alloc(&d.pcp, (size_t)d.pc_pool)) ||
                     (rc = p->alloc(&d.pcoff, jobs * NJ * (size_t)Om)) || (rc = p->alloc(&d.pcok, jobs)) ||
                     (rc = p->alloc(&d.pcbase, jobs)) || (rc = p->alloc(&d.pcnext, 1))))
        return rc;
    if (d.pcache) {
        HIPCK(hipMemset(d.pcnext, 0, sizeof(unsigned)));
        HIPCK(hipHostMalloc((void**)&p->h_pcnext, sizeof(unsigned)));
        p->rc.pc_next = d.pcnext;
        p->ra.rc.pc_next = d.pcnext;
        p->la.rc.pc_next = d.pcnext;
    }
    // speculative line-search slots (values only): every world x (max_ls - 1) trials. The speculative
    // round reads the plane cache (ARMOUR planner, fp64); otherwise the rounds run one by one.
    d.K = d.opt.max_ls - 1;
    p->spec = !std::getenv("ARMOUR_NO_SPEC") && d.K > 0 && d.K <= EV_MAXK && d.pcache && !p->armtd && !p->eval_f32;
    // The sync-free tail may search all max_ls trials of its (at most tail_worlds) running worlds in
    // one round (run_solver)
    p->spec_all = p->spec && p->tail_search > 0 && (d.K + 1) * NJ * Om <= UB_FULL;
    // the restoration phase searches all max_ls trials of up to every world at once
    p->resto_spec = p->spec && d.opt.resto_max > 0 && d.opt.max_ls <= EV_MAXK + 1 && d.opt.max_ls * NJ * Om <= UB_FULL &&
                    !std::getenv("ARMOUR_RESTO_ROUNDS");
    p->resto_inline = p->resto_spec && !(std::getenv("ARMOUR_RESTO_INLINE") && std::atoi(std::getenv("ARMOUR_RESTO_INLINE")) == 0);
    p->resto_conc = p->resto_inline && p->spec_all && p->tail_worlds > 0 &&
                    !(std::getenv("ARMOUR_RESTO_CONCURRENT") && std::atoi(std::getenv("ARMOUR_RESTO_CONCURRENT")) == 0);
    if (p->resto_conc) {
        HIPCK(hipStreamCreateWithFlags(&p->rstream2, hipStreamNonBlocking));
        HIPCK(hipEventCreateWithFlags(&p->ev_ip, hipEventDisableTiming));
        HIPCK(hipEventCreateWithFlags(&p->ev_pub, hipEventDisableTiming));
        HIPCK(hipEventCreateWithFlags(&p->ev_rend, hipEventDisableTiming));
    }
    if (p->spec) {
        // rows of the speculative slots: the interior point's rounds use the first Wm x K (the
        // sync-free tail's one-round search the first nall); a restoration phase Wm x max_ls, after
        // the tail's rows when it runs concurrently with the tail (resto_soff)
        const size_t nall = p->spec_all ? (size_t)std::min(Wm, std::max(p->tail_worlds, 0)) * (d.K + 1) : 0;
        p->resto_soff = p->resto_conc ? nall : 0;
        const size_t nres = p->resto_spec ? (size_t)Wm * d.opt.max_ls + p->resto_soff : 0;
        const size_t ns = std::max(std::max((size_t)Wm * d.K, nall), nres);
        if ((rc = p->alloc(&d.gs, ns * mmax)) || (rc = p->alloc(&d.fs, ns)) || (rc = p->alloc(&d.partial_s, ns * nblk_max * KA)))
            return rc;
    }
    HIPCK(hipMemset(d.cnt, 0, 16 * sizeof(unsigned)));
    d.rl_app = nullptr;
    d.pend_flag = nullptr;
    d.lcount = nullptr;
    d.b_in_cs = 0;
    d.bt_flag = nullptr;
    d.lrun_out = nullptr;
    d.nrun_flag = nullptr;
    d.lcount_out = nullptr;
    d.wl = nullptr;
    d.wl_run = p->d_lists;
    d.wl_search = p->d_lists + 2 * Wm;
    d.ls0 = 0;
    HIPCK(hipHostMalloc((void**)&p->h_ws, Wm * sizeof(WorldState)));
    HIPCK(hipHostMalloc((void**)&p->h_f, 2 * Wm * sizeof(double)));
    HIPCK(hipHostMalloc((void**)&p->h_feas, Wm * sizeof(int)));
    d.q0 = p->q0;
    d.qd0 = p->qd0;
    d.qdd0 = p->qdd0;
    d.qdes = p->qdes;
    d.obs = p->obs;
    return 0;
}

static int upload_worlds(armour_planner* p, int W, const armour_world* worlds) {
    if (W <= 0 || W > p->Wmax || !worlds) return fail(ARMOUR_E_ARG, "num_worlds out of range");
    const int O = worlds[0].num_obstacles;
    if (O < 0 || O > p->Omax) return fail(ARMOUR_E_ARG, "num_obstacles exceeds max_obstacles");
    std::vector<double> a(4 * (size_t)W * NF), ob((size_t)W * (O > 0 ? O : 1) * 12, 0.0);
    for (int w = 0; w < W; w++) {
        if (worlds[w].num_obstacles != O) return fail(ARMOUR_E_ARG, "all worlds of a batch must have the same num_obstacles");
        if (O > 0 && !worlds[w].obstacles) return fail(ARMOUR_E_ARG, "null obstacles");
        for (int i = 0; i < NF; i++) {
            a[0 * (size_t)W * NF + w * NF + i] = worlds[w].q0[i];
            a[1 * (size_t)W * NF + w * NF + i] = worlds[w].qd0[i];
            a[2 * (size_t)W * NF + w * NF + i] = worlds[w].qdd0[i];
            a[3 * (size_t)W * NF + w * NF + i] = worlds[w].q_des[i];
        }
        if (O > 0) std::memcpy(&ob[(size_t)w * O * 12], worlds[w].obstacles, sizeof(double) * O * 12);
    }
    const size_t bytes = sizeof(double) * W * NF;
    HIPCK(hipMemcpyAsync(p->q0, &a[0], bytes, hipMemcpyHostToDevice, p->stream));
    HIPCK(hipMemcpyAsync(p->qd0, &a[(size_t)W * NF], bytes, hipMemcpyHostToDevice, p->stream));
    HIPCK(hipMemcpyAsync(p->qdd0, &a[2 * (size_t)W * NF], bytes, hipMemcpyHostToDevice, p->stream));
    HIPCK(hipMemcpyAsync(p->qdes, &a[3 * (size_t)W * NF], bytes, hipMemcpyHostToDevice, p->stream));
    if (O > 0) HIPCK(hipMemcpyAsync(p->obs, ob.data(), sizeof(double) * ob.size(), hipMemcpyHostToDevice, p->stream));
    HIPCK(hipStreamSynchronize(p->stream));  // host staging vectors die at return
    p->W = W;
    p->O = O;
    NlpDev& d = p->d;
    d.W = W;
    d.O = O;
    d.pcready = 0;
    d.m = d.nt + p->T * p->NJ * O + NF * 4;
    d.R = d.m + NF;
    d.chunk = row_chunk();
    d.nblk = (d.R + d.chunk - 1) / d.chunk;
    return 0;
}

// the ARMTD batch: armour_world fields (qdd0 = 0) plus the JRS tables and k_range
static int upload_armtd(armour_planner* p, int W, const armour_armtd_world* worlds) {
    if (!p->armtd) return fail(ARMOUR_E_ARG, "not an ARMTD planner (armour_create_armtd)");
    if (W <= 0 || W > p->Wmax || !worlds) return fail(ARMOUR_E_ARG, "num_worlds out of range");
    std::vector<armour_world> base(W);
    const size_t ntab = (size_t)NF * 6 * p->T;
    std::vector<double> tab((size_t)W * ntab), kr((size_t)W * NF);
    for (int w = 0; w < W; w++) {
        if (!worlds[w].jrs_tables) return fail(ARMOUR_E_ARG, "null jrs_tables");
        armour_world& b = base[w];
        for (int i = 0; i < NF; i++) {
            b.q0[i] = worlds[w].q0[i];
            b.qd0[i] = worlds[w].qd0[i];
            b.qdd0[i] = 0.0;
            b.q_des[i] = worlds[w].q_des[i];
            kr[(size_t)w * NF + i] = worlds[w].k_range[i];
        }
        b.num_obstacles = worlds[w].num_obstacles;
        b.obstacles = worlds[w].obstacles;
        std::memcpy(&tab[(size_t)w * ntab], worlds[w].jrs_tables, sizeof(double) * ntab);
    }
    HIPCK(hipMemcpyAsync(p->d_tables, tab.data(), sizeof(double) * tab.size(), hipMemcpyHostToDevice, p->stream));
    HIPCK(hipMemcpyAsync((double*)p->d.krange, kr.data(), sizeof(double) * kr.size(), hipMemcpyHostToDevice, p->stream));
    return upload_worlds(p, W, base.data());  // ends in a synchronisation: tab / kr outlive the copies
}

// Bundle kernel shape of a launch of `bundles` bundles (lane_kernel.hip): the dense shape (three
// per CU) when the batch does not fit one round of the wide shape (two per CU), or when other
// planners share the device (this process's live planners, or ARMOUR_DEVICE_SHARED=1 for planners
// in other processes) and the batch holds more than one bundle per CU; else the wide shape.
// Measured: three planners x 327 worlds dense 5324-5363 against 5187 plans/s;
// three planners x 85 worlds (config 4's 256-world job) wide 63.5 against 72.1 ms.
static int lane_shape_for(armour_planner* p, long bundles) {
    int shape = p->lane_shape;
    if (shape < 0)
        shape = (bundles > p->lane_slots[0] ||
                 ((p->device_shared || g_planners[p->dev & 63].load() > 1) && bundles > p->reach_cus)) ? 1 : 0;
    p->last_shape = shape;
    return shape;
}
static void launch_lane(int shape, int grid, hipStream_t s, const RobotParams* rp, const lane::LaneArgs& la,
                        const ReachOut& ro) {
    if (shape == 1)
        hipLaunchKernelGGL(lane::lane_reach_kernel<lane::LaneDense>, dim3(grid), dim3(lane::LT), 0, s, rp, la, ro);
    else
        hipLaunchKernelGGL(lane::lane_reach_kernel<lane::LaneWide>, dim3(grid), dim3(lane::LT), 0, s, rp, la, ro);
}

// reach set for the uploaded batch. The whole phase is three kernel launches on the reach stream
// (JRS, reach, and a capacity retry when needed) and one event wait: jrs_kernel zeroes the
// counters, the reach kernel's last workgroup publishes them in mapped host memory
// (ReachCounters), and the constraint bounds are formed by the solver's ipm_rows_init. Nothing
// else is queued here, so under concurrent planners no small kernel waits for CUs another
// planner's persistent reach kernel holds.
static int run_reach(armour_planner* p) {
    hipStream_t rs = p->rstream;
    ReachArgs ra = p->ra;
    ra.W = p->W;
    ra.T = p->T;
    ra.q0 = p->q0;
    ra.qd0 = p->qd0;
    ra.qdd0 = p->qdd0;
    const long jobs = (long)p->W * p->T;
    const int grid = (int)(jobs < p->reach_grid ? jobs : p->reach_grid);
    p->lane_engine = !(p->has_job && jobs <= p->job_max);
    const long nj = jobs * NF;
    HIPCK(hipEventRecord(p->ev[3], rs));
    if (p->armtd)
        hipLaunchKernelGGL(jrs_armtd_kernel, dim3((int)((nj + 127) / 128)), dim3(128), 0, rs, p->W, p->T, p->q0, p->d_tables,
                           p->d_jrs, p->rc, p->ro.err);
    else
        hipLaunchKernelGGL(jrs_kernel, dim3((int)((nj + 127) / 128)), dim3(128), 0, rs, p->d_rp, p->W, p->T, p->q0, p->qd0,
                           p->qdd0, p->d_jrs, p->rc, p->ro.err);
    ra.jrs = p->d_jrs;
    ra.rc.seq = ++p->reach_seq;
    if (p->lane_engine) {
        lane::LaneArgs la = p->la;
        la.W = p->W;
        la.T = p->T;
        la.jrs = p->d_jrs;
        la.rc.seq = p->reach_seq;
        const long bundles = (jobs + lane::LG - 1) / lane::LG;
        const int shape = lane_shape_for(p, bundles);
        const long slots = std::min<long>(p->lane_slots[shape], p->lane_grid);
        const int lg = (int)(bundles < slots ? bundles : slots);
        launch_lane(shape, lg, rs, p->d_rp, la, p->ro);
    } else {
        // a batch that fits the chip in one round at two jobs per CU takes the wide kernel
        if (jobs <= (long)REACH_WIDE_PER_CU * p->ncu && !p->job_narrow)
            hipLaunchKernelGGL(reach_kernel<REACH_WIDE_THREADS>, dim3(grid), dim3(REACH_WIDE_THREADS), 0, rs, p->d_rp, ra, p->ro);
        else
            hipLaunchKernelGGL(reach_kernel<REACH_THREADS>, dim3(grid), dim3(REACH_THREADS), 0, rs, p->d_rp, ra, p->ro);
    }
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(p->ev[4], rs));
    HIPCK(hipEventSynchronize(p->ev[4]));
    const volatile long long* sum = p->h_sum;
    if (sum[RSUM_SEQ] != p->reach_seq)
        return fail(ARMOUR_E_HIP, "reach kernel finished without publishing its counters (sequence number mismatch)");
    std::vector<int> err(p->W);
    for (int w = 0; w < p->W; w++) err[w] = (int)sum[RSUM_ERR + w];
    for (int k = 0; k < 8; k++) p->h_occ[k] = (unsigned long long)sum[1 + k];
    {
        // the launch's execution span on the device clock (reach_kernel.hip span_start): occ[5]
        // holds ~(first workgroup start), occ[6] the last workgroup's end
        const unsigned long long t0 = ~p->h_occ[5], t1 = p->h_occ[6];
        p->last_span_ms = (p->h_occ[5] != 0 && t1 >= t0 && p->wall_khz > 0) ? (double)(t1 - t0) / p->wall_khz : -1.0;
    }
    {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, p->ev[3], p->ev[4]);
        p->last_kernel_ms = ms;
        p->last_bytes = (double)sum[0];
    }
    // Capacity isolation. A bundle that overflowed its arena / key buffers flags every world it
    // holds. Those worlds' jobs run again in a second launch of a quarter of the workgroups, each
    // with four workgroups' buffers (4x the arena, key and output capacity). A world that still
    // overflows gets ARMOUR_E_CAPACITY in its result and is not planned; the batch goes on.
    // (armour_get_reach_occupancy reports the first launch against its 1x capacities: h_occ.)
    std::vector<int> retry;
    for (int w = 0; w < p->W; w++)
        if (err[w]) retry.push_back(w);
    p->last_retried = (int)retry.size();
    unsigned long long mono[2] = {p->h_occ[3], p->h_occ[4]};
    if (!retry.empty() && p->lane_engine) {
        lane::LaneArgs la = p->la;
        la.W = p->W;
        la.T = p->T;
        la.jrs = p->d_jrs;
        la.hcap *= RETRY_SCALE;
        la.ccap *= RETRY_SCALE;
        la.gcap *= RETRY_SCALE;
        la.ocap *= RETRY_SCALE;
        la.pool_rows *= RETRY_SCALE;
        la.wlist = p->d_wlist;
        la.nlist = (int)retry.size();
        la.dump = nullptr;   // the op dump and bundle times stay those of the first launch
        la.btime = nullptr;
        la.rc.seq = ++p->reach_seq;
        HIPCK(hipMemcpyAsync(p->d_wlist, retry.data(), sizeof(int) * retry.size(), hipMemcpyHostToDevice, rs));
        HIPCK(hipMemsetAsync(p->ro.err, 0, sizeof(int) * p->W, rs));
        const long bundles = ((long)retry.size() * p->T + lane::LG - 1) / lane::LG;
        const long g = std::max(p->lane_grid, RETRY_SCALE) / RETRY_SCALE;
        launch_lane(p->last_shape, (int)(bundles < g ? bundles : g), rs, p->d_rp, la, p->ro);
        HIPCK(hipGetLastError());
        HIPCK(hipEventRecord(p->ev[5], rs));
        HIPCK(hipEventSynchronize(p->ev[5]));
        if (sum[RSUM_SEQ] != p->reach_seq)
            return fail(ARMOUR_E_HIP, "capacity retry finished without publishing its counters (sequence number mismatch)");
        for (int w = 0; w < p->W; w++) err[w] = (int)sum[RSUM_ERR + w];
        mono[0] = (unsigned long long)sum[1 + 3];   // maxima over both launches (occ accumulates)
        mono[1] = (unsigned long long)sum[1 + 4];
    }
    p->mono_max[0] = (int)std::min<unsigned long long>(mono[0], 1u << 30);
    p->mono_max[1] = p->armtd ? 0 : (int)std::min<unsigned long long>(mono[1], 1u << 30);
    p->world_err.assign(p->W, 0);
    p->last_failed = 0;
    for (int w = 0; w < p->W; w++)
        if (err[w]) {
            p->world_err[w] = ARMOUR_E_CAPACITY;
            p->last_failed++;
        }
    if (p->last_failed) {
        char buf[200];
        std::snprintf(buf, sizeof(buf), "%d world(s) exceeded a reach-set capacity (first: world %d); the rest are planned",
                      p->last_failed, (int)(std::find_if(err.begin(), err.end(), [](int e) { return e != 0; }) - err.begin()));
        g_err = buf;
    }
    p->reached = true;
    p->d.pcready = 0;
    return 0;
}

// the certified plane cache of the current reach sets and obstacles (plane_cache_kernel)
static void ensure_plane_cache(armour_planner* p) {
    NlpDev& d = p->d;
    if (!d.pcache || d.pcready || d.O == 0 || p->eval_f32) return;
    // The pool is sized at creation for ARMOUR_PC_K records per pair; a build whose blocks need
    // more (the count is known only on the device) is repeated on a pool of 1.25x what it needed,
    // so every block is cached. One host wait on the build, which the solver's first kernels wait
    // for anyway. The cache is marked ready only when the last build fitted its pool: the cached
    // kernels read every block's records from its pool offset, and a block that did not fit has
    // none there. Otherwise (the larger pool cannot be allocated) this solve runs on the full
    // 36-plane scan, whose values, planes and tie-breaks are bitwise the cache's, and without the
    // speculative searches that read only the cache (run_solver, ipm_loop, run_resto).
    bool fits = false;
    for (int attempt = 0; attempt < 3; attempt++) {
        hipLaunchKernelGGL(plane_cache_kernel, dim3(p->T, p->W), dim3(EVAL_THREADS), 0, p->stream, d);
        if (hipMemcpyAsync(p->h_pcnext, d.pcnext, sizeof(unsigned), hipMemcpyDeviceToHost, p->stream) != hipSuccess ||
            hipStreamSynchronize(p->stream) != hipSuccess)
            break;
        const long need = (long)*p->h_pcnext;
        (void)hipMemsetAsync(d.pcnext, 0, sizeof(unsigned), p->stream);
        if (need <= d.pc_pool) {
            fits = true;
            break;
        }
        if (attempt == 2) break;
        const long grow = need + need / 4;
        double* pc = nullptr;
        uint16_t* pcp = nullptr;
        if (std::getenv("ARMOUR_PC_GROW_FAIL") || dalloc(&pc, 5 * (size_t)grow) != hipSuccess) break;
        if (dalloc(&pcp, (size_t)grow) != hipSuccess) { (void)hipFree(pc); break; }
        for (void*& a : p->allocs) {
            if (a == (void*)d.pc) { (void)hipFree(a); a = pc; }
            else if (a == (void*)d.pcp) { (void)hipFree(a); a = pcp; }
        }
        d.pc = pc;
        d.pcp = pcp;
        d.pc_pool = grow;
    }
    d.pcready = fits ? 1 : 0;
}

static int nside_count(const armour_planner* p) {
    // finite constraint sides: torque 2/row, collision 1/row, extrema 2/row, box 2/variable
    return 2 * p->d.nt + p->T * p->NJ * p->O + 2 * 4 * NF + 2 * NF;
}

// g and J of every world of the batch (eval_kernel_t): fp64, or float for the tolerance study
// (the ARMTD planner's extrema and cost in their own instantiation)
// and the collision rows from the certified plane cache when it is built (points in its box: every
// solver point; `cached` = false for a caller's x outside it)
// the small-capacity evaluation kernels (eval_kernel_small, eval_trials_small: a third of the LDS,
// five blocks per CU) when the last reach's largest PZs and this batch's pair tables fit them
static bool eval_small_fits(const armour_planner* p) {
    return !p->eval_full && !p->armtd && !p->eval_f32 && p->mono_max[0] <= LM_S && p->mono_max[1] <= UM_S;
}
static void launch_eval(armour_planner* p, dim3 grid, const NlpDev& d, int mode, bool cached = true, hipStream_t s = nullptr) {
    if (!s) s = p->stream;
    const bool c = cached && d.pcready && d.O > 0;
    if (c && eval_small_fits(p) && eval_pair_doubles(p->NJ * d.O) <= UB_S) {
        hipLaunchKernelGGL(eval_kernel_small, grid, dim3(EVAL_THREADS), 0, s, d, mode);
        return;
    }
    auto k = p->eval_f32 ? (d.armtd ? eval_kernel_t<float, true, false> : eval_kernel_t<float, false, false>)
                         : c ? (d.armtd ? eval_kernel_t<double, true, true> : eval_kernel_t<double, false, true>)
                             : (d.armtd ? eval_kernel_t<double, true, false> : eval_kernel_t<double, false, false>);
    hipLaunchKernelGGL(k, grid, dim3(EVAL_THREADS), 0, s, d, mode);
}

// The interior-point loop over the nrun worlds listed in the first iteration list (d_lists[0..]):
// every world there starts an iteration with pass A at its current point (a fresh solve, or a
// restart after a restoration phase).
static int ipm_loop(armour_planner* p, int nrun) {
    NlpDev& d = p->d;
    int* Li[2] = {p->d_lists, p->d_lists + p->Wmax};                  // worlds of an iteration
    int* Ls[2] = {p->d_lists + 2 * p->Wmax, p->d_lists + 3 * p->Wmax};  // worlds of a line-search round
    const int ns = nside_count(p);
    // Restoration phases inside the loop (with the speculative machinery): after an iteration's
    // interior-point launches, one phase iteration (run_resto's one-round form) for the worlds whose
    // line search failed and are still in their phase. Failures (accept_trial) and the worlds a
    // phase iteration keeps are appended to one list RL (cnt[12]); resto_publish moves it into the
    // phase list PL of the next phase iteration, so an iteration may launch no phase work at all
    // and the appends wait for the next one that does. The host decides from the list length the
    // round's last world kernel stores (pend_flag): in a synchronised iteration exactly (the length
    // after round 0, plus the worlds still searching, which alone can fail now); in the sync-free
    // tail from the length two iterations back (the last one it has read), so a phase starts at
    // most two iterations late and at most two idle phase iterations follow the last one. Worlds
    // still in a phase when the loop ends finish it after the loop (run_solver: run_resto), and so
    // does a restarted world's interior point (the next ipm_loop). A loop over one world runs its
    // phases after the loop: there is no other world's iteration to overlap them with.
    const bool inl = p->resto_inline && d.pcready && nrun > 1;
    int* RL = p->d_lists + 4 * p->Wmax;
    int* PL = p->d_lists + 5 * p->Wmax;
    volatile int* flr = p->h_flags;
    const int W0 = nrun;
    int pend_known = 0;  // the latest list length the host has read
    int ub = 0;          // an upper bound of the list's length now: the last phase grid, plus every
                         // interior-point world launched since (each could have failed)
    if (inl) HIPCK(hipMemsetAsync(d.cnt + 12, 0, sizeof(unsigned), p->stream));
    // conc: this phase iteration runs on the second stream, concurrently with the next
    // interior-point iteration (sync-free tail, p->resto_conc). The phase's worlds are not the
    // interior point's (an iteration's list may still name a world that failed after the list was
    // formed: the world kernels write back only the worlds they work on, nlp_kernels.hip ws_copy),
    // and its speculative rows start resto_soff rows in (after the tail's); the
    // one shared structure is the append list RL (cnt[12]): interior-point failures and the phase's
    // kept worlds append to it with atomics, and resto_publish moves it to the phase list. So the
    // publish waits for the interior-point iteration that appended (ev_ip), and the next
    // interior-point iteration waits for the publish (ev_pub), not for the phase iteration. An
    // interior-point iteration's snapshot of the list (pend_flag) may then miss the worlds the
    // concurrent phase iteration keeps, so the host also reads the length each publish moved
    // (flags[8 + (it & 1)], pub_known): a phase iteration that had worlds is followed by another at
    // most two iterations later, as long as the loop runs.
    bool conc_used = false;
    bool pub_launched[2] = {false, false};
    int pub_known = 0;
    auto resto_iter = [&](int it, int bound, bool conc) -> int {
        pub_launched[it & 1] = false;
        if (!inl || bound <= 0) return 0;
        hipStream_t s = p->stream;
        if (conc) {
            s = p->rstream2;
            HIPCK(hipEventRecord(p->ev_ip, p->stream));
            HIPCK(hipStreamWaitEvent(s, p->ev_ip, 0));
            conc_used = true;
        }
        hipLaunchKernelGGL(resto_publish, dim3(1), dim3(256), 0, s, d, (const int*)RL, PL,
                           conc ? d.flags + 8 + (it & 1) : nullptr);
        pub_launched[it & 1] = conc;
        if (conc) {
            HIPCK(hipEventRecord(p->ev_pub, s));
            HIPCK(hipStreamWaitEvent(p->stream, p->ev_pub, 0));
        }
        const int nb = std::min(W0, bound);
        ub = nb;  // the phase keeps at most the worlds it took
        NlpDev dr = d;
        dr.resto = 1;
        dr.K = d.opt.max_ls;
        dr.b_in_cs = 0;
        dr.rflag = -1;
        dr.wl = PL;
        dr.lcount = d.cnt + 14;
        dr.rl_app = RL;
        dr.pend_flag = nullptr;
        if (conc) {
            dr.gs = d.gs + p->resto_soff * (size_t)d.m;
            dr.fs = d.fs + p->resto_soff;
            dr.partial_s = d.partial_s + p->resto_soff * (size_t)d.nblk * KA;
        }
        hipLaunchKernelGGL(resto_rows_G, dim3(d.nblk, nb), dim3(ROW_THREADS), 0, s, dr);
        hipLaunchKernelGGL(resto_world_G, dim3(nb), dim3(64), 0, s, dr);
        hipLaunchKernelGGL(eval_trials_all, dim3(p->T, nb), dim3(EVAL_THREADS), 0, s, dr);
        hipLaunchKernelGGL(resto_rows_Vs, dim3(d.nblk, nb * dr.K), dim3(ROW_THREADS), 0, s, dr);
        hipLaunchKernelGGL(resto_world_Vs, dim3(nb), dim3(64), 0, s, dr);
        launch_eval(p, dim3(p->T, nb), dr, 5, true, s);
        return 0;
    };
    // Launches cover the active worlds only (NlpDev::wl): every line-search round's ipm_world_C
    // compacts the worlds still running / still searching into the next lists and publishes the
    // counts in mapped host memory, read after the round's one host synchronisation. Inactive
    // worlds in a list (finished by ipm_world_A / _D since) exit at once. A world's arithmetic does
    // not depend on which block serves it, so the results are those of full launches.
    // Sync-free tail: once at most tail_worlds worlds run (and the speculative round is available),
    // an iteration is launched without waiting for the previous one. Grids are sized by the last
    // known running count (an upper bound: the count only falls), every launch reads the true list
    // lengths from device memory (the running count of iteration it in cnt[8 + (it & 1)], the
    // searching count in cnt[5]), and the host learns iteration it's running count one iteration
    // later (event tev[it & 1], flags[2 + (it & 1)]). Blocks past a list's length exit at once, so a
    // world's arithmetic is that of the synchronised loop.
    int cur = 0;
    bool tail = false;       // iteration it - 1 ran sync-free (its running count not yet read)
    // worlds that backtracked (searched past round 0) in the latest iteration the host knows of: the
    // tail takes the one-round search while they do (ARMOUR_TAIL_SEARCH=adaptive). A converging
    // world mostly accepts round 0's trial, which its own full evaluation serves faster than the
    // values of every trial plus the chosen one's full evaluation; a backtracking world saves a
    // round. The choice changes launches only, never a world's arithmetic.
    int backtracked = nrun;
    for (int it = 0; it <= d.opt.max_iter && nrun > 0; it++) {
        const bool tl = it > 0 && p->spec && d.pcready && nrun <= p->tail_worlds;
        // this iteration's failed line searches, and the list length its last world kernel reports
        d.rl_app = inl ? RL : nullptr;
        d.pend_flag = inl ? d.flags + 6 + (it & 1) : nullptr;
        NlpDev di = d;
        di.wl = Li[cur];
        if (tl) di.lcount = d.cnt + 8 + (it & 1);
        // pass D of the previous iteration (accept its trial point) shares one sweep over the rows
        // with this iteration's pass A
        if (it == 0) {
            hipLaunchKernelGGL(ipm_rows_A, dim3(d.nblk, nrun), dim3(ROW_THREADS), 0, p->stream, di);
            hipLaunchKernelGGL(ipm_world_A, dim3(nrun), dim3(64), 0, p->stream, di, ns);
        } else {
            // the LDS-accumulator form for grids of several blocks per CU (nlp_kernels.hip rows_DA_body)
            const bool wide = p->da_lds && (long)d.nblk * nrun >= 4L * p->ncu;
            hipLaunchKernelGGL(wide ? ipm_rows_DA_lds : ipm_rows_DA, dim3(d.nblk, nrun), dim3(ROW_THREADS), 0, p->stream, di);
            hipLaunchKernelGGL(ipm_world_DA, dim3(nrun), dim3(64), 0, p->stream, di, ns);
        }
        const bool one = tl && p->spec_all && (p->tail_search == 2 || backtracked > 0);
        hipLaunchKernelGGL(ipm_rows_B, dim3(d.nblk, nrun), dim3(ROW_THREADS), 0, p->stream, di);
        if (!one) hipLaunchKernelGGL(ipm_world_B, dim3(nrun), dim3(64), 0, p->stream, di);
        if (one) {
            // The tail's line search in one round: the values of all max_ls trials of every running
            // world at once (round 0's included, the step taken from pass B's partials), then pass
            // B's world step, the acceptance tests in trial order and round 0's running list and
            // counts (ipm_world_Cs_all), then the chosen trial in full. Four launches where pass B's
            // world step and round 0 took four and the speculative round four more; the tests, and
            // so the plans, are those of sequential rounds.
            NlpDev ds = d;
            ds.K = d.K + 1;
            ds.b_in_cs = 1;  // pass B's world step in ipm_world_Cs_all
            ds.wl = Li[cur];
            ds.wl_run = Li[1 - cur];
            ds.lcount = di.lcount;
            ds.lrun_out = d.cnt + 8 + ((it + 1) & 1);
            ds.nrun_flag = d.flags + 2 + (it & 1);
            ds.bt_flag = d.flags + 4 + (it & 1);
            hipLaunchKernelGGL(eval_trials_all, dim3(p->T, nrun), dim3(EVAL_THREADS), 0, p->stream, ds);
            hipLaunchKernelGGL(ipm_rows_Cs, dim3(d.nblk, nrun * ds.K), dim3(ROW_THREADS), 0, p->stream, ds);
            hipLaunchKernelGGL(ipm_world_Cs_all, dim3(nrun), dim3(64), 0, p->stream, ds);
            launch_eval(p, dim3(p->T, nrun), ds, 5);
            ub = std::min(W0, ub + nrun);
            if (int rc = resto_iter(it, pend_known > 0 || pub_known > 0 ? ub : 0, p->resto_conc)) return rc;
            HIPCK(hipEventRecord(p->tev[it & 1], p->stream));
            HIPCK(hipGetLastError());
            cur = 1 - cur;
            if (tail) {
                HIPCK(hipEventSynchronize(p->tev[(it - 1) & 1]));
                if (inl) pend_known = flr[6 + ((it - 1) & 1)];
                pub_known = pub_launched[(it - 1) & 1] ? flr[8 + ((it - 1) & 1)] : 0;
                const int prev = ((volatile int*)p->h_flags)[2 + ((it - 1) & 1)];
                backtracked = ((volatile int*)p->h_flags)[4 + ((it - 1) & 1)];
                if (prev == 0) break;
                nrun = prev < nrun ? prev : nrun;
            }
            tail = true;
            continue;
        }
        // Round 0 of the line search for every running world, then one host synchronisation. The
        // worlds still searching after it (the tail of the backtracking) run the remaining rounds
        // without one: a few of them all remaining trials at once (speculative round, ipm_world_Cs),
        // more of them round by round with grids sized by round 0's count and the list lengths in
        // device memory (cnt[4 + r & 1]). Either way the arithmetic is that of sequential rounds.
        int nnext = 0, nsearch = 0;
        {
            NlpDev dc = d;
            dc.wl = Li[cur];
            dc.wl_run = Li[1 - cur];
            dc.wl_search = Ls[1];
            dc.ls0 = 1;
            dc.lcount_out = d.cnt + 5;
            dc.lrun_out = d.cnt + 8 + ((it + 1) & 1);
            if (tl) {
                dc.lcount = di.lcount;
                dc.nrun_flag = d.flags + 2 + (it & 1);
                dc.bt_flag = d.flags + 4 + (it & 1);
            }
            launch_eval(p, dim3(p->T, nrun), dc, 1);
            hipLaunchKernelGGL(ipm_rows_C, dim3(d.nblk, nrun), dim3(ROW_THREADS), 0, p->stream, dc);
            hipLaunchKernelGGL(ipm_world_C, dim3(nrun), dim3(64), 0, p->stream, dc);
            if (!tl) {
                HIPCK(hipStreamSynchronize(p->stream));
                nnext = ((volatile int*)p->h_flags)[0];
                nsearch = ((volatile int*)p->h_flags)[1];
                backtracked = nsearch;
                if (inl) pend_known = flr[6 + (it & 1)];  // after round 0 (ipm_world_C's last block)
            }
        }
        if (tl) {
            // the speculative round over at most nrun list entries, then the iteration's end event
            NlpDev ds = d;
            ds.wl = Ls[1];
            ds.lcount = d.cnt + 5;
            if (eval_small_fits(p) && d.K * p->NJ * d.O <= UB_TS)
                hipLaunchKernelGGL(eval_trials_small, dim3(p->T, nrun), dim3(EVAL_THREADS), 0, p->stream, ds);
            else
                hipLaunchKernelGGL(eval_trials_kernel, dim3(p->T, nrun), dim3(EVAL_THREADS), 0, p->stream, ds);
            hipLaunchKernelGGL(ipm_rows_Cs, dim3(d.nblk, nrun * d.K), dim3(ROW_THREADS), 0, p->stream, ds);
            hipLaunchKernelGGL(ipm_world_Cs, dim3(nrun), dim3(64), 0, p->stream, ds);
            launch_eval(p, dim3(p->T, nrun), ds, 5);
            ub = std::min(W0, ub + nrun);
            if (int rc = resto_iter(it, pend_known > 0 || pub_known > 0 ? ub : 0, p->resto_conc)) return rc;
            HIPCK(hipEventRecord(p->tev[it & 1], p->stream));
            HIPCK(hipGetLastError());
            cur = 1 - cur;
            if (tail) {
                // iteration it - 1's running count: the worlds iteration it was launched for
                HIPCK(hipEventSynchronize(p->tev[(it - 1) & 1]));
                if (inl) pend_known = flr[6 + ((it - 1) & 1)];
                pub_known = pub_launched[(it - 1) & 1] ? flr[8 + ((it - 1) & 1)] : 0;
                const int prev = ((volatile int*)p->h_flags)[2 + ((it - 1) & 1)];
                backtracked = ((volatile int*)p->h_flags)[4 + ((it - 1) & 1)];
                if (prev == 0) break;  // iteration it had nothing to do
                nrun = prev < nrun ? prev : nrun;
            }
            tail = true;
            continue;
        }
        if (nsearch > 0 && p->spec && d.pcready) {
            // the worlds still searching: the values of all remaining trials at once, the acceptance
            // tests in trial order, then the chosen trial in full
            NlpDev ds = d;
            ds.wl = Ls[1];
            if (eval_small_fits(p) && d.K * p->NJ * d.O <= UB_TS)
                hipLaunchKernelGGL(eval_trials_small, dim3(p->T, nsearch), dim3(EVAL_THREADS), 0, p->stream, ds);
            else
                hipLaunchKernelGGL(eval_trials_kernel, dim3(p->T, nsearch), dim3(EVAL_THREADS), 0, p->stream, ds);
            hipLaunchKernelGGL(ipm_rows_Cs, dim3(d.nblk, nsearch * d.K), dim3(ROW_THREADS), 0, p->stream, ds);
            hipLaunchKernelGGL(ipm_world_Cs, dim3(nsearch), dim3(64), 0, p->stream, ds);
            launch_eval(p, dim3(p->T, nsearch), ds, 5);
        } else if (nsearch > 0) {
            for (int ls = 1; ls < d.opt.max_ls; ls++) {
                NlpDev dc = d;
                dc.wl = Ls[ls & 1];
                dc.lcount = d.cnt + 4 + (ls & 1);
                dc.wl_search = Ls[(ls + 1) & 1];
                dc.lcount_out = d.cnt + 4 + ((ls + 1) & 1);
                dc.ls0 = 0;
                launch_eval(p, dim3(p->T, nsearch), dc, 1);
                hipLaunchKernelGGL(ipm_rows_C, dim3(d.nblk, nsearch), dim3(ROW_THREADS), 0, p->stream, dc);
                hipLaunchKernelGGL(ipm_world_C, dim3(nsearch), dim3(64), 0, p->stream, dc);
            }
        }
        // (the phase list's bound: its length after round 0, plus the worlds that searched past
        // round 0 and so could have failed)
        if (inl) ub = std::min(W0, pend_known + nsearch);
        if (int rc = resto_iter(it, ub, false)) return rc;
        if (nnext == 0) break;  // every world converged, hit the cap, failed or is in a restoration phase
        HIPCK(hipGetLastError());
        cur = 1 - cur;
        nrun = nnext;
    }
    if (conc_used) {  // the last phase iteration, before anything reads its worlds or reuses PL
        HIPCK(hipEventRecord(p->ev_rend, p->rstream2));
        HIPCK(hipStreamWaitEvent(p->stream, p->ev_rend, 0));
    }
    d.rl_app = nullptr;
    d.pend_flag = nullptr;
    HIPCK(hipGetLastError());
    return 0;
}

// One restoration phase for the n worlds of `list` (status WS_RESTO), all together: per iteration
// the Gauss-Newton pass and world step, then the Armijo search. With the speculative machinery
// (p->resto_spec) the search is one round — the values of all max_ls trials, their sums, the tests
// in trial order and the chosen trial's full evaluation — and iterations are launched without a
// host synchronisation: the host reads iteration k - 1's count of worlds still in the phase (mapped
// flags[2 + (k - 1) & 1], written by resto_world_G) after launching iteration k, so at most one
// empty iteration is launched. Otherwise one trial per round (a full evaluation each; rounds after
// the first launched without a synchronisation, their blocks exit for worlds that stopped). The
// worlds leave with status 0 (every row within its bounds: restart), 2 (iteration cap) or 5 (local
// infeasibility). Either way the arithmetic and decisions are the oracle's sequential ones.
static int run_resto(armour_planner* p, const int* list, int n) {
    NlpDev dr = p->d;
    dr.wl = list;
    dr.resto = 1;
    dr.lcount = nullptr;
    dr.b_in_cs = 0;
    const volatile int* fl = p->h_flags;
    const int guard = 4 * (dr.opt.max_iter + 1);
    if (p->resto_spec && p->d.pcready) {
        // iteration k works on list L[k & 1] (the first: `list`, n entries); resto_world_Vs appends
        // the worlds still in the phase to L[(k + 1) & 1] and stores its length in cnt[8 + ((k + 1) & 1)]
        // (the next launches' lcount) and flags[2 + (k & 1)] (read by the host after iteration k + 1
        // is launched: the grid bound of iteration k + 2, or the end)
        int* L[2] = {const_cast<int*>(list), p->d_lists + 3 * p->Wmax};
        dr.K = dr.opt.max_ls;
        dr.rflag = -1;
        int nb = n;  // grid bound: the last count the host knows (counts only fall)
        for (int k = 0; k < guard; k++) {
            NlpDev di = dr;
            di.wl = L[k & 1];
            di.wl_run = L[(k + 1) & 1];
            di.lcount = k == 0 ? nullptr : p->d.cnt + 8 + (k & 1);
            di.lrun_out = p->d.cnt + 8 + ((k + 1) & 1);
            di.nrun_flag = p->d.flags + 2 + (k & 1);
            hipLaunchKernelGGL(resto_rows_G, dim3(dr.nblk, nb), dim3(ROW_THREADS), 0, p->stream, di);
            hipLaunchKernelGGL(resto_world_G, dim3(nb), dim3(64), 0, p->stream, di);
            hipLaunchKernelGGL(eval_trials_all, dim3(p->T, nb), dim3(EVAL_THREADS), 0, p->stream, di);
            hipLaunchKernelGGL(resto_rows_Vs, dim3(dr.nblk, nb * dr.K), dim3(ROW_THREADS), 0, p->stream, di);
            hipLaunchKernelGGL(resto_world_Vs, dim3(nb), dim3(64), 0, p->stream, di);
            launch_eval(p, dim3(p->T, nb), di, 5);
            HIPCK(hipEventRecord(p->tev[k & 1], p->stream));
            HIPCK(hipGetLastError());
            if (k > 0) {
                HIPCK(hipEventSynchronize(p->tev[(k - 1) & 1]));
                const int prev = fl[2 + ((k - 1) & 1)];  // worlds iteration k was launched for
                if (prev == 0) break;
                nb = prev < nb ? prev : nb;
            }
        }
        HIPCK(hipStreamSynchronize(p->stream));
        return 0;
    }
    dr.rflag = 0;
    dr.lrun_out = nullptr;
    for (int k = 0; k < guard; k++) {
        hipLaunchKernelGGL(resto_rows_G, dim3(dr.nblk, n), dim3(ROW_THREADS), 0, p->stream, dr);
        hipLaunchKernelGGL(resto_world_G, dim3(n), dim3(64), 0, p->stream, dr);
        HIPCK(hipStreamSynchronize(p->stream));
        if (fl[0] == 0) break;
        for (int ls = 0; ls < dr.opt.max_ls; ls++) {
            launch_eval(p, dim3(p->T, n), dr, 1);
            hipLaunchKernelGGL(resto_rows_V, dim3(dr.nblk, n), dim3(ROW_THREADS), 0, p->stream, dr);
            hipLaunchKernelGGL(resto_world_V, dim3(n), dim3(64), 0, p->stream, dr);
            if (ls == 0) {
                HIPCK(hipStreamSynchronize(p->stream));
                if (fl[1] == 0) break;
            }
        }
        HIPCK(hipGetLastError());
    }
    return 0;
}

static int run_solver(armour_planner* p) {
    NlpDev& d = p->d;
    const int W = p->W;
    int* Li0 = p->d_lists;                  // the interior-point loop's first list
    int* Lr = p->d_lists + 2 * p->Wmax;     // worlds of a restoration phase
    d.wl = nullptr;
    d.wl_run = Li0;
    d.ls0 = 0;
    d.resto = 0;
    ensure_plane_cache(p);
    hipLaunchKernelGGL(ipm_world_init, dim3((W + 63) / 64), dim3(64), 0, p->stream, d);
    launch_eval(p, dim3(p->T, W), d, 0);
    hipLaunchKernelGGL(ipm_rows_init, dim3(d.nblk, W), dim3(ROW_THREADS), 0, p->stream, d);
    HIPCK(hipGetLastError());
    int rc = ipm_loop(p, W);
    // Restoration phases: the worlds whose line search failed left the loop with
    // status WS_RESTO. They run their phase together; those that reached a point within every bound
    // restart the interior point (slacks and multipliers at that point), and may fail again (at
    // most resto_max phases per world, S.nresto).
    const volatile int* fl = p->h_flags;
    while (rc == 0 && d.opt.resto_max > 0) {
        hipLaunchKernelGGL(ipm_collect, dim3(1), dim3(1024), 0, p->stream, d, (const int*)nullptr, W, WS_RESTO, Lr, 0, -1);
        HIPCK(hipStreamSynchronize(p->stream));
        const int nr = fl[0];
        if (nr > 0 && (rc = run_resto(p, Lr, nr))) break;
        // the restarted worlds (WS_RESTART), running again from here. Collected whether or not a
        // phase ran just now: a phase that ran inside ipm_loop may have restarted a world while
        // other worlds were still iterating, and the loop never takes such a world back itself.
        hipLaunchKernelGGL(ipm_collect, dim3(1), dim3(1024), 0, p->stream, d, (const int*)nullptr, W, WS_RESTART, Li0, 0, 0);
        HIPCK(hipStreamSynchronize(p->stream));
        const int ni = fl[0];
        if (ni == 0) break;
        NlpDev di = d;
        di.wl = Li0;
        hipLaunchKernelGGL(ipm_rows_init, dim3(d.nblk, ni), dim3(ROW_THREADS), 0, p->stream, di);
        rc = ipm_loop(p, ni);
    }
    if (rc) return rc;
    // feasibility re-check and the sliced link centres at the final iterate (the current slot's,
    // armour_joint_position_center.out payload)
    hipLaunchKernelGGL(feasible_kernel, dim3(W), dim3(256), 0, p->stream, d, p->feas);
    HIPCK(hipGetLastError());
    return 0;
}

// Every entry point runs on its planner's device, whatever the calling thread's current device is
// (handles may be driven from other host threads); the caller's device is restored.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(const armour_planner* p) {
        int cur = -1;
        if (p && p->cfg.device >= 0 && hipGetDevice(&cur) == hipSuccess && cur != p->cfg.device &&
            hipSetDevice(p->cfg.device) == hipSuccess)
            prev = cur;
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

extern "C" {

const char* armour_last_error(void) { return g_err.c_str(); }

int armour_device_compute_units(int device) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        return fail(ARMOUR_E_HIP, "hipDeviceGetAttribute failed (no device?)");
    return n;
}

// streaming copy (the achievable-HBM reference kernel): each workgroup copies one contiguous 16 KiB
// block, four 16-B loads per lane in flight before its four stores, nontemporal both ways. Measured
// shapes (tools/micro/copy.hip, 2 x 2 GiB): this one 5.9 TB/s; without nt 5.6; grid-stride with
// four loads per lane (the round-4 kernel) 4.5; eight or sixteen per lane 4.3 / 5.2.
typedef double copy_v2d __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void copy_kernel(const copy_v2d* __restrict__ src, copy_v2d* __restrict__ dst, long n) {
    const long base = (long)blockIdx.x * 1024 + threadIdx.x;
    copy_v2d v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const long i = base + k * 256;
        if (i < n) v[k] = __builtin_nontemporal_load(&src[i]);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const long i = base + k * 256;
        if (i < n) __builtin_nontemporal_store(v[k], &dst[i]);
    }
}

double armour_copy_bandwidth(int device, size_t bytes, int reps) {
    int prev = -1;
    (void)hipGetDevice(&prev);
    struct Restore {
        int d;
        ~Restore() { if (d >= 0) (void)hipSetDevice(d); }
    } restore{prev};
    if (reps <= 0 || bytes < 16) return fail(ARMOUR_E_ARG, "bytes >= 16 and reps > 0");
    if (hipSetDevice(device) != hipSuccess) return fail(ARMOUR_E_HIP, "hipSetDevice failed (no device?)");
    const long n = (long)(bytes / 16);
    copy_v2d *a = nullptr, *b = nullptr;
    hipEvent_t e0, e1;
    if (hipMalloc((void**)&a, n * 16) != hipSuccess) return fail(ARMOUR_E_HIP, "hipMalloc failed");
    if (hipMalloc((void**)&b, n * 16) != hipSuccess) { (void)hipFree(a); return fail(ARMOUR_E_HIP, "hipMalloc failed"); }
    (void)hipMemset(a, 0, n * 16);
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const dim3 grid((unsigned)((n + 1023) / 1024)), blk(256);
    hipLaunchKernelGGL(copy_kernel, grid, blk, 0, nullptr, a, b, n);
    (void)hipEventRecord(e0, nullptr);
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(copy_kernel, grid, blk, 0, nullptr, a, b, n);
    (void)hipEventRecord(e1, nullptr);
    const hipError_t err = hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(a);
    (void)hipFree(b);
    if (err != hipSuccess || ms <= 0) return fail(ARMOUR_E_HIP, "copy kernel failed");
    return 2.0 * n * 16.0 * reps / (ms * 1e-3) / 1e9;
}

int armour_robot_builtin(int robot_id, armour_robot* out) {
    if (!out || robot_id != 0) return fail(ARMOUR_E_ARG, "unknown robot id / null output");
    RobotParams r;
    kinova_gen3(r);
    robot_to_tables(r, *out);
    return 0;
}

armour_planner* armour_create(const armour_config* cfg) { return armour_create_robot(cfg, nullptr); }

armour_planner* armour_create_robot(const armour_config* cfg, const armour_robot* robot) {
    if (!cfg) { fail(ARMOUR_E_ARG, "null config"); return nullptr; }
    // planner_init makes cfg->device current; the caller's current device is restored on return
    struct Restore {
        int dev = -1;
        Restore() { if (hipGetDevice(&dev) != hipSuccess) dev = -1; }
        ~Restore() { if (dev >= 0) (void)hipSetDevice(dev); }
    } restore;
    armour_planner* p = new armour_planner();
    if (planner_init(p, cfg, robot) != 0) {
        std::string keep = g_err;
        armour_destroy(p);
        g_err = keep;
        return nullptr;
    }
    return p;
}

armour_planner* armour_create_armtd(const armour_config* cfg) {
    if (!cfg) { fail(ARMOUR_E_ARG, "null config"); return nullptr; }
    struct Restore {
        int dev = -1;
        Restore() { if (hipGetDevice(&dev) != hipSuccess) dev = -1; }
        ~Restore() { if (dev >= 0) (void)hipSetDevice(dev); }
    } restore;
    armour_planner* p = new armour_planner();
    if (planner_init(p, cfg, nullptr, true) != 0) {
        std::string keep = g_err;
        armour_destroy(p);
        g_err = keep;
        return nullptr;
    }
    return p;
}

void armour_destroy(armour_planner* p) {
    DeviceScope device_scope(p);
    if (!p) return;
    if (p->stream) (void)hipStreamSynchronize(p->stream);
    for (void* a : p->allocs) (void)hipFree(a);
    if (p->h_flags) (void)hipHostFree(p->h_flags);
    if (p->h_sum) (void)hipHostFree(p->h_sum);
    if (p->h_ws) (void)hipHostFree(p->h_ws);
    if (p->h_f) (void)hipHostFree(p->h_f);
    if (p->h_feas) (void)hipHostFree(p->h_feas);
    if (p->h_pcnext) (void)hipHostFree(p->h_pcnext);
    if (p->stream) {
        for (int i = 0; i < 6; i++) (void)hipEventDestroy(p->ev[i]);
        for (int i = 0; i < 2; i++) (void)hipEventDestroy(p->tev[i]);
        if (p->rstream2) (void)hipStreamSynchronize(p->rstream2);
        for (hipEvent_t e : {p->ev_ip, p->ev_pub, p->ev_rend})
            if (e) (void)hipEventDestroy(e);
        if (p->rstream2) (void)hipStreamDestroy(p->rstream2);
        if (p->rstream && p->rstream != p->stream) (void)hipStreamDestroy(p->rstream);
        (void)hipStreamDestroy(p->stream);
    }
    if (p->counted) g_planners[p->dev & 63]--;
    delete p;
}

int armour_plan(armour_planner* p, const armour_world* world, armour_plan_output* out) {
    if (!p || !world || !out) return fail(ARMOUR_E_ARG, "null argument");
    int rc = armour_plan_batch(p, 1, world, &out->result, &out->timing);
    if (rc) return rc;
    if (out->constraints && (rc = armour_get_constraints(p, 0, out->constraints))) return rc;
    if (out->joint_bounds && (rc = armour_get_joint_bounds(p, out->joint_bounds))) return rc;
    if (out->link_centers && (rc = armour_get_link_centers(p, 0, out->link_centers))) return rc;
    if (out->link_generators && (rc = armour_get_link_generators(p, 0, out->link_generators))) return rc;
    if (out->torque_radius && (rc = armour_get_torque_radius(p, 0, out->torque_radius))) return rc;
    return 0;
}

int armour_num_constraints(const armour_planner* p, int O) { return p ? p->d.nt + p->T * p->NJ * O + NF * 4 : ARMOUR_E_ARG; }
int armour_num_joints(const armour_planner* p) { return p ? p->NJ : ARMOUR_E_ARG; }

int armour_get_joint_bounds(const armour_planner* p, double* b) {
    DeviceScope device_scope(p);
    if (!p || !b) return fail(ARMOUR_E_ARG, "null argument");
    const RobotParams& rp = p->rp;
    for (int i = 0; i < NF; i++) {
        b[2 * i] = rp.state_lb[i] + rp.qe;
        b[2 * i + 1] = rp.state_ub[i] - rp.qe;
        b[2 * NF + 2 * i] = -rp.speed_limits[i] + rp.qde;
        b[2 * NF + 2 * i + 1] = rp.speed_limits[i] - rp.qde;
    }
    return 0;
}

static int reach_uploaded(armour_planner* p, armour_timing* timing, std::chrono::steady_clock::time_point t0);
static int plan_uploaded(armour_planner* p, armour_result* results, armour_timing* timing,
                         std::chrono::steady_clock::time_point t0);

int armour_reach_batch(armour_planner* p, int W, const armour_world* worlds, armour_timing* timing) {
    DeviceScope device_scope(p);
    if (!p) return fail(ARMOUR_E_ARG, "null planner");
    if (p->armtd) return fail(ARMOUR_E_ARG, "an ARMTD planner takes armour_armtd_world (armour_reach_armtd_batch)");
    p->reached = p->planned = false;
    auto t0 = std::chrono::steady_clock::now();
    const int rc = upload_worlds(p, W, worlds);
    return rc ? rc : reach_uploaded(p, timing, t0);
}

int armour_reach_armtd_batch(armour_planner* p, int W, const armour_armtd_world* worlds, armour_timing* timing) {
    DeviceScope device_scope(p);
    if (!p) return fail(ARMOUR_E_ARG, "null planner");
    p->reached = p->planned = false;
    auto t0 = std::chrono::steady_clock::now();
    const int rc = upload_armtd(p, W, worlds);
    return rc ? rc : reach_uploaded(p, timing, t0);
}

int armour_plan_armtd_batch(armour_planner* p, int W, const armour_armtd_world* worlds, armour_result* results,
                            armour_timing* timing) {
    DeviceScope device_scope(p);
    if (!p || !results) return fail(ARMOUR_E_ARG, "null planner / results");
    p->reached = p->planned = false;
    auto t0 = std::chrono::steady_clock::now();
    const int rc = upload_armtd(p, W, worlds);
    return rc ? rc : plan_uploaded(p, results, timing, t0);
}

static int reach_uploaded(armour_planner* p, armour_timing* timing, std::chrono::steady_clock::time_point t0) {
    int rc = 0;
    HIPCK(hipEventRecord(p->ev[0], p->rstream));
    if ((rc = run_reach(p))) return rc;
    HIPCK(hipEventRecord(p->ev[1], p->rstream));
    HIPCK(hipEventSynchronize(p->ev[1]));
    if (timing) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, p->ev[0], p->ev[1]);
        timing->reach_ms = ms;
        timing->nlp_ms = 0;
        timing->reach_kernel_ms = p->last_kernel_ms;
        timing->reach_bytes = p->last_bytes;
        timing->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return 0;
}

int armour_plan_batch(armour_planner* p, int W, const armour_world* worlds, armour_result* results, armour_timing* timing) {
    DeviceScope device_scope(p);
    if (!p || !results) return fail(ARMOUR_E_ARG, "null planner / results");
    if (p->armtd) return fail(ARMOUR_E_ARG, "an ARMTD planner takes armour_armtd_world (armour_plan_armtd_batch)");
    p->reached = p->planned = false;
    auto t0 = std::chrono::steady_clock::now();
    const int rc = upload_worlds(p, W, worlds);
    return rc ? rc : plan_uploaded(p, results, timing, t0);
}

static int plan_uploaded(armour_planner* p, armour_result* results, armour_timing* timing,
                         std::chrono::steady_clock::time_point t0) {
    int rc = 0;
    const int W = p->W;
    // the reach phase on the reach stream (ev[0] .. ev[1]; run_reach ends in a host wait for it),
    // then the solver on the planner's stream (ev[1] .. ev[2])
    HIPCK(hipEventRecord(p->ev[0], p->rstream));
    if ((rc = run_reach(p))) return rc;
    HIPCK(hipEventRecord(p->ev[1], p->rstream));
    if ((rc = run_solver(p))) return rc;
    HIPCK(hipEventRecord(p->ev[2], p->stream));
    HIPCK(hipMemcpyAsync(p->h_ws, p->d.ws, sizeof(WorldState) * W, hipMemcpyDeviceToHost, p->stream));
    HIPCK(hipMemcpyAsync(p->h_f, p->d.f, sizeof(double) * 2 * p->Wmax, hipMemcpyDeviceToHost, p->stream));
    HIPCK(hipMemcpyAsync(p->h_feas, p->feas, sizeof(int) * W, hipMemcpyDeviceToHost, p->stream));
    HIPCK(hipStreamSynchronize(p->stream));
    for (int w = 0; w < W; w++) {
        const WorldState& S = p->h_ws[w];
        armour_result& r = results[w];
        for (int i = 0; i < NF; i++) r.k_opt[i] = S.x[i];
        r.feasible = p->h_feas[w];
        r.solver_status = S.status == 1 ? 0 : S.status == 2 ? 1 : S.status == 3 ? 2 : S.status == 5 ? 4 : 3;
        r.iterations = S.iter;
        r.evaluations = S.nevals;
        r.cost = p->h_f[S.cur * p->d.W + w] / p->rp.cost_scale;
        r.kkt_error = S.kkt;
        r.error = p->world_err[w];
        // a world the solver left in a non-terminal state (running, in a restoration phase, or
        // waiting to restart) is a solver fault, never a silent "not planned"
        if (!r.error && (S.status == 0 || S.status == WS_RESTO || S.status == WS_RESTART)) r.error = ARMOUR_E_INTERNAL;
        if (r.error) {
            r.solver_status = 3;
            r.feasible = 0;
        }
    }
    p->planned = true;
    if (timing) {
        float a = 0, b = 0;
        (void)hipEventElapsedTime(&a, p->ev[0], p->ev[1]);
        (void)hipEventElapsedTime(&b, p->ev[1], p->ev[2]);
        timing->reach_ms = a;
        timing->nlp_ms = b;
        timing->reach_kernel_ms = p->last_kernel_ms;
        timing->reach_bytes = p->last_bytes;
        timing->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return 0;
}

int armour_eval_constraints(armour_planner* p, int w, const double* x, double* g, double* jac) {
    DeviceScope device_scope(p);
    if (!p || !x || !g) return fail(ARMOUR_E_ARG, "null argument");
    if (!p->reached) return fail(ARMOUR_E_STATE, "no reach set: call armour_reach_batch or armour_plan_batch first");
    if (w < 0 || w >= p->W) return fail(ARMOUR_E_ARG, "world index out of range");
    NlpDev& d = p->d;
    // evaluate every world of the batch at x in slot 0 (ws.x is the solver's start/end point, so
    // a subsequent query of solver outputs must re-plan)
    // (on the planner's stream, so the copies are ordered with its kernels)
    std::vector<WorldState> ws(p->W);
    HIPCK(hipMemcpyAsync(ws.data(), d.ws, sizeof(WorldState) * p->W, hipMemcpyDeviceToHost, p->stream));
    HIPCK(hipStreamSynchronize(p->stream));
    for (int i = 0; i < p->W; i++) {
        for (int j = 0; j < NF; j++) ws[i].x[j] = x[j];
        ws[i].status = 0;
        ws[i].cur = 0;
    }
    HIPCK(hipMemcpyAsync(d.ws, ws.data(), sizeof(WorldState) * p->W, hipMemcpyHostToDevice, p->stream));
    ensure_plane_cache(p);
    bool inbox = true;
    for (int j = 0; j < NF; j++) inbox = inbox && std::fabs(x[j]) <= PC_XBOX;
    launch_eval(p, dim3(p->T, p->W), d, 0, inbox);
    HIPCK(hipGetLastError());
    HIPCK(hipMemcpyAsync(g, d.g + gidx(d, 0, w, 0), sizeof(double) * d.m, hipMemcpyDeviceToHost, p->stream));
    if (jac) HIPCK(hipMemcpyAsync(jac, d.J + gidx(d, 0, w, 0) * NF, sizeof(double) * d.m * NF, hipMemcpyDeviceToHost, p->stream));
    HIPCK(hipStreamSynchronize(p->stream));
    p->planned = false;
    return 0;
}

int armour_get_constraints(armour_planner* p, int w, double* g) {
    DeviceScope device_scope(p);
    if (!p || !g) return fail(ARMOUR_E_ARG, "null argument");
    if (!p->planned) return fail(ARMOUR_E_STATE, "no plan");
    if (w < 0 || w >= p->W) return fail(ARMOUR_E_ARG, "world index out of range");
    const int cur = p->h_ws[w].cur;
    HIPCK(hipMemcpy(g, p->d.g + gidx(p->d, cur, w, 0), sizeof(double) * p->d.m, hipMemcpyDeviceToHost));
    return 0;
}

int armour_get_link_centers(armour_planner* p, int w, double* c) {
    DeviceScope device_scope(p);
    if (!p || !c) return fail(ARMOUR_E_ARG, "null argument");
    if (!p->planned) return fail(ARMOUR_E_STATE, "no plan");
    if (w < 0 || w >= p->W) return fail(ARMOUR_E_ARG, "world index out of range");
    HIPCK(hipMemcpy(c, p->d.link_c + 2 * p->d.lcs + (size_t)w * p->T * p->NJ * 3, sizeof(double) * p->T * p->NJ * 3, hipMemcpyDeviceToHost));
    return 0;
}

int armour_get_link_generators(armour_planner* p, int w, double* gens) {
    DeviceScope device_scope(p);
    if (!p || !gens) return fail(ARMOUR_E_ARG, "null argument");
    if (!p->reached) return fail(ARMOUR_E_STATE, "no reach set");
    if (w < 0 || w >= p->W) return fail(ARMOUR_E_ARG, "world index out of range");
    const size_t n = (size_t)p->T * p->NJ;
    std::vector<double> cm(n * 18);
    HIPCK(hipMemcpy(cm.data(), p->ro.link_gens + (size_t)w * n * 18, sizeof(double) * n * 18, hipMemcpyDeviceToHost));
    for (size_t j = 0; j < n; j++)
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 6; c++) gens[j * 18 + r * 6 + c] = cm[j * 18 + r + 3 * c];
    return 0;
}

int armour_get_torque_radius(armour_planner* p, int w, double* radius) {
    DeviceScope device_scope(p);
    if (!p || !radius) return fail(ARMOUR_E_ARG, "null argument");
    if (!p->reached) return fail(ARMOUR_E_STATE, "no reach set");
    if (w < 0 || w >= p->W) return fail(ARMOUR_E_ARG, "world index out of range");
    HIPCK(hipMemcpy(radius, p->ro.torque_radius + (size_t)w * p->T * NF, sizeof(double) * p->T * NF, hipMemcpyDeviceToHost));
    return 0;
}

int armour_get_reach_profile(armour_planner* p, unsigned long long* cycles_terms, int capacity) {
    DeviceScope device_scope(p);
    if (!p) return fail(ARMOUR_E_ARG, "null planner");
    if (!p->d_prof) return fail(ARMOUR_E_STATE, "op profiling is off (set ARMOUR_PROFILE_OPS before armour_create)");
    // capacity in pairs: nops + 8 -> per-op [cycles, terms] + 16 phase totals; nops + 8 + 4 * OP_NCODES
    // adds the bundle engine's phase cycles per op code [OP_NCODES][8]
    // adds the bundle engine's phase cycles per op code [OP_NCODES][8]; + ceil(max_worlds * T / 64)
    // adds every bundle's [start, end] wall clock (ARMOUR_PROFILE_OPS=3)
    if (cycles_terms && capacity >= p->nops + 8) {
        const size_t nb = ((size_t)p->Wmax * p->T + lane::LG - 1) / lane::LG;
        const size_t n = capacity >= p->nops + 8 + 4 * OP_NCODES + (long)nb ? 2 * p->nops + 16 + 8 * OP_NCODES + 2 * nb
                         : capacity >= p->nops + 8 + 4 * OP_NCODES ? 2 * p->nops + 16 + 8 * OP_NCODES : 2 * p->nops + 16;
        HIPCK(hipMemcpy(cycles_terms, p->d_prof, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
    }
    return p->nops;
}

int armour_get_reach_dump(armour_planner* p, double* dump, int capacity) {
    DeviceScope device_scope(p);
    if (!p) return fail(ARMOUR_E_ARG, "null planner");
    if (!p->d_dump) return fail(ARMOUR_E_STATE, "op dump is off (set ARMOUR_DUMP_OPS before armour_create)");
    if (!p->lane_engine && p->has_lane)
        return fail(ARMOUR_E_STATE, "the op dump follows the bundle engine, and the last batch ran on the per-job engine");
    if (dump && capacity >= p->nops) {
        if (p->lane_engine) {
            // [nops][DUMP_W][64] of bundle 0: lane ARMOUR_DUMP_LANE (default 0) = job of that index
            const char* ls = std::getenv("ARMOUR_DUMP_LANE");
            const int l = ls ? std::atoi(ls) & 63 : 0;
            std::vector<double> all((size_t)p->nops * DUMP_W * lane::LG);
            HIPCK(hipMemcpy(all.data(), p->d_dump, sizeof(double) * all.size(), hipMemcpyDeviceToHost));
            for (int k = 0; k < p->nops * DUMP_W; k++) dump[k] = all[(size_t)k * lane::LG + l];
        } else {
            HIPCK(hipMemcpy(dump, p->d_dump, sizeof(double) * DUMP_W * p->nops, hipMemcpyDeviceToHost));
        }
    }
    return p->nops;
}

int armour_get_monomial_counts(armour_planner* p, int w, int* link_counts, int* torque_counts) {
    DeviceScope device_scope(p);
    if (!p) return fail(ARMOUR_E_ARG, "null planner");
    if (!p->reached) return fail(ARMOUR_E_STATE, "no reach set");
    if (w < 0 || w >= p->W) return fail(ARMOUR_E_ARG, "world index out of range");
    const size_t j0 = (size_t)w * p->T;
    if (link_counts)
        HIPCK(hipMemcpy(link_counts, p->ro.link_cnt + j0 * p->NJ, sizeof(int) * p->T * p->NJ, hipMemcpyDeviceToHost));
    if (torque_counts)
        HIPCK(hipMemcpy(torque_counts, p->ro.tq_cnt + j0 * NF, sizeof(int) * p->T * NF, hipMemcpyDeviceToHost));
    return 0;
}

int armour_get_reach_span(armour_planner* p, double* span_ms) {
    if (!p || !span_ms) return fail(ARMOUR_E_ARG, "null planner or output");
    if (!p->reached) return fail(ARMOUR_E_STATE, "no reach set");
    *span_ms = p->last_span_ms;
    return p->last_span_ms >= 0 ? 0 : fail(ARMOUR_E_STATE, "no device clock span for the last reach");
}

int armour_get_plane_cache_stats(armour_planner* p, long long* out, int n) {
    DeviceScope device_scope(p);
    if (!p) return fail(ARMOUR_E_ARG, "null planner");
    if (!p->reached) return fail(ARMOUR_E_STATE, "no reach set");
    NlpDev& d = p->d;
    if (!d.pcache || p->eval_f32 || d.O == 0) return fail(ARMOUR_E_STATE, "plane cache off (ARMOUR_PLANE_CACHE=0, float study or no obstacles)");
    ensure_plane_cache(p);
    const size_t blocks = (size_t)p->W * p->T, NP = (size_t)p->NJ * d.O;
    std::vector<unsigned> off(blocks * NP);
    std::vector<unsigned char> ok(blocks);
    HIPCK(hipMemcpyAsync(off.data(), d.pcoff, sizeof(unsigned) * off.size(), hipMemcpyDeviceToHost, p->stream));
    HIPCK(hipMemcpyAsync(ok.data(), d.pcok, blocks, hipMemcpyDeviceToHost, p->stream));
    HIPCK(hipStreamSynchronize(p->stream));
    long long kept = 0, nok = 0, mx = 0;
    for (unsigned v : off) {
        kept += v & 255;
        mx = std::max<long long>(mx, v & 255);
    }
    for (unsigned char v : ok) nok += v;
    unsigned miss = 0;
    HIPCK(hipMemcpy(&miss, d.cnt + 7, sizeof(unsigned), hipMemcpyDeviceToHost));
    const long long st[ARMOUR_PC_COUNT] = {kept, (long long)off.size(), nok, (long long)blocks, mx, d.pc_pool, miss};
    for (int k = 0; k < n && k < ARMOUR_PC_COUNT; k++) out[k] = st[k];
    return ARMOUR_PC_COUNT;
}

int armour_get_reach_occupancy(armour_planner* p, long long* used, long long* caps, int n) {
    DeviceScope device_scope(p);
    if (!p) return fail(ARMOUR_E_ARG, "null planner");
    if (!p->reached) return fail(ARMOUR_E_STATE, "no reach set");
    if (!p->lane_engine || !p->d_occ)
        return fail(ARMOUR_E_STATE, "occupancy is recorded by the bundle engine only (this batch ran on the per-job engine)");
    const unsigned long long* o = p->h_occ;  // the first launch's maxima (a retry's 4x buffers excluded)
    const long long u[ARMOUR_OCC_COUNT] = {(long long)o[0], (long long)o[1], (long long)o[2], (long long)o[3],
                                           (long long)o[4], p->last_retried, p->last_failed};
    const long long c[ARMOUR_OCC_COUNT] = {p->la.hcap, p->la.ccap, std::min<long long>(p->la.gcap, (1 << 16) - 1),
                                           CAP_LM, CAP_UM, p->W, p->W};
    for (int k = 0; k < n && k < ARMOUR_OCC_COUNT; k++) {
        if (used) used[k] = u[k];
        if (caps) caps[k] = c[k];
    }
    return ARMOUR_OCC_COUNT;
}

int armour_get_reach_program(const armour_planner* p, int* codes, int capacity) {
    DeviceScope device_scope(p);
    if (!p) return fail(ARMOUR_E_ARG, "null planner");
    if (codes && capacity >= p->nops) {
        std::vector<Op> ops(p->nops);
        HIPCK(hipMemcpy(ops.data(), p->d_prog, sizeof(Op) * p->nops, hipMemcpyDeviceToHost));
        for (int k = 0; k < p->nops; k++) codes[k] = ops[k].code;
    }
    return p->nops;
}

}  // extern "C"
