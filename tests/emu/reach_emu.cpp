// TEST HARNESS — sequential host emulation of the reach kernel's workgroup program
// (armour-dev_amd/csrc/reach.h) with a 1-thread group. Used only by tests/ to check the GPU
// algorithm against the CPU oracle without a GPU; never part of the product library.
#include <cstdlib>
#include <cstring>
#include <vector>
#include "reach.h"
#include "robots.h"

using namespace armour;

static double* g_dump = nullptr;
static int g_unfused = 0;
extern "C" void emu_set_dump(double* d) { g_dump = d; }
extern "C" void emu_set_unfused(int u) { g_unfused = u; }
extern "C" void emu_set_stats(int* st) { armour::g_op_stats = st; }
extern "C" void emu_set_hash_sink(void (*f)(int, const uint64_t*, int)) { armour::g_hash_sink = f; }
static RobotParams g_rp;
static bool g_init = false;
static ProgramBuilder g_pbf, g_pbu;  // fused / composed cross products
// robot tables (include/armour_hip.h armour_robot); null: the built-in Kinova Gen3
extern "C" int emu_set_robot(const armour_robot* r) {
    if (r) {
        if (!robot_from_tables(*r, g_rp)) return -1;
    } else {
        kinova_gen3(g_rp);
    }
    g_init = true;
    g_pbf = ProgramBuilder();
    g_pbu = ProgramBuilder();
    return 0;
}
extern "C" int emu_reach(int T, int t, const double* q0, const double* qd0, const double* qdd0,
                         double* link_gens, double* link_center, double* link_rad, int* link_cnt,
                         uint16_t* link_hash, double* link_coef, double* tq_center, double* tq_rad,
                         int* tq_cnt, uint16_t* tq_hash, double* tq_coef, double* torque_radius,
                         long* arena_used, double* arena_bytes, int* nops, int* nslots) {
    if (!g_init) emu_set_robot(nullptr);
    RobotParams& rp = g_rp;
    ProgramBuilder& pb = g_unfused ? g_pbu : g_pbf;
    if (pb.ops.empty()) {
        pb.fused = !g_unfused;
        pb.build(rp);
    }
    const long cap = 1 << 22;
    std::vector<uint64_t> ah(cap);
    std::vector<double> ac(cap * 3);
    // handles as LDS leaves them (garbage): run_program must not depend on their contents
    std::vector<PZH> H(MAX_SLOTS);
    for (int k = 0; k < MAX_SLOTS; k++) {
        H[k].cnt = 1000 + 37 * k;
        H[k].hoff = 7 * k;
        H[k].coff = 11 * k;
        H[k].stride = 9;
    }
    int pool_n = 0;
    const std::vector<int> off = pb.slot_offsets(&pool_n);
    std::vector<double> pool(pool_n + 9);
    for (int k = 0; k < pb.nslots; k++) H[k].off = off[k];
    const int kcap = 1 << 16;
    std::vector<uint64_t> kh(kcap);
    std::vector<uint32_t> ki(kcap);
    std::vector<int> kp(kcap);
    double red[18];
    int iscan[2];
    Arena A{cap, cap * 3, 0, 0, 0.0};
    int err = 0;
    Ctx x;
    x.g = Grp{0, 1};
    x.H = H.data();
    x.pool = pool.data();
    x.A = &A;
    x.ah = ah.data();
    x.ac = ac.data();
    x.kh = kh.data(); x.ki = ki.data(); x.kp = kp.data(); x.cap_lds = kcap;
    x.gkh = kh.data(); x.gki = ki.data(); x.gkp = kp.data(); x.cap_glb = kcap;
    std::vector<double> gout(9 * (size_t)kcap);
    x.gout = gout.data();
    std::vector<double> stage(4096);
    x.stage = stage.data();
    x.stage_cap = 4096;
    x.red = red;
    x.iscan = iscan;
    x.err = &err;
    x.thr = rp.simplify_threshold;
    x.phase = nullptr;
    x.mode = 0;
    int werr = 0;
    ReachOut out;
    out.T = 1;
    out.NJ = rp.num_joints;
    out.link_hash = link_hash; out.link_coef = link_coef; out.link_cnt = link_cnt;
    out.link_center = link_center; out.link_rad = link_rad; out.link_gens = link_gens;
    out.tq_hash = tq_hash; out.tq_coef = tq_coef; out.tq_cnt = tq_cnt; out.tq_center = tq_center;
    out.tq_rad = tq_rad; out.torque_radius = torque_radius; out.err = &werr;
    JrsJoint jrs[NF];
    double scratch[2 * NF];
    run_program(x, rp, pb.ops.data(), (int)pb.ops.size(), T, t, q0, qd0, qdd0, out, 0, jrs, scratch, nullptr, g_dump);
    *arena_used = A.hused;
    if (arena_bytes) *arena_bytes = A.bytes;
    if (nops) *nops = (int)pb.ops.size();
    if (nslots) *nslots = pb.nslots;
    return err;
}

// the op program (code, o, a, b, c, i) of the fused (or composed) build, for analysis tools
extern "C" int emu_program(int unfused, int* out, int cap) {
    static RobotParams rp;
    kinova_gen3(rp);
    ProgramBuilder pb;
    pb.fused = !unfused;
    pb.build(rp);
    const int n = (int)pb.ops.size();
    for (int k = 0; k < n && k < cap; k++) {
        const Op& op = pb.ops[k];
        out[6 * k] = op.code; out[6 * k + 1] = op.o; out[6 * k + 2] = op.a;
        out[6 * k + 3] = op.b; out[6 * k + 4] = op.c; out[6 * k + 5] = op.i;
    }
    return n;
}
