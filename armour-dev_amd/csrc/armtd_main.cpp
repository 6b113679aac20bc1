// armtd_main — drop-in replacement for the ARMTD comparison planner process
// (kinova_planner_realtime_armtd_comparison/armtd_main.cu, "ACMP/"), built on the C ABI of
// libarmour_hip.so (armour_create_armtd / armour_plan_armtd_batch).
//
// Same file protocol as the reference (ACMP/armtd_main.cu:4-8, 37-102, 217-267; written and read by
// KSI/uarmtd_planner.m:268-360):
//   in : <buffer>/armtd.in  7 q0, 7 qd0, 7 q_des, then per joint T values each of c_cos, g_cos,
//                           r_cos, c_sin, g_sin, r_sin and its k_range, then int O and O x 12
//                           obstacle doubles
//   out: <buffer>/armtd.out                         k_opt (7 lines, precision 10) or -1, then ms
//        <buffer>/armtd_joint_position_center.out   T*NJ rows of 3 (sliced link centres)
//        <buffer>/armtd_joint_position_radius.out   T*NJ*3 rows of 6 (link generators)
//        <buffer>/armtd_constraints.out             m constraint values (precision 6)
// Errors follow the reference: unreadable input or a bad obstacle count writes -1 to armtd.out
// and exits non-zero.
//
// Buffer directory: argv[1], else $ARMOUR_BUFFER_DIR, else the build-time ARMOUR_BUFFER_PATH,
// else <directory of this executable>/buffer/. Time steps: $ARMOUR_NUM_TIME_STEPS, default 100
// (NUM_TIME_STEPS, ACMP/Parameters.h:17).
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/armour_hip.h"

namespace {

constexpr int NF = ARMOUR_NUM_FACTORS;
constexpr int MAX_OBSTACLES = 40;  // MAX_OBSTACLE_NUM (ACMP/Parameters.h:24)

std::string buffer_dir(int argc, char** argv) {
    std::string d;
    if (argc > 1) d = argv[1];
    else if (const char* e = std::getenv("ARMOUR_BUFFER_DIR")) d = e;
#ifdef ARMOUR_BUFFER_PATH
    else d = ARMOUR_BUFFER_PATH;
#else
    else {
        char buf[4096];
        const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
        std::string exe = n > 0 ? std::string(buf, (size_t)n) : std::string("./armtd_main");
        d = exe.substr(0, exe.find_last_of('/') + 1) + "buffer";
    }
#endif
    if (!d.empty() && d.back() != '/') d += '/';
    return d;
}

int fail_out(const std::string& out1, const char* msg) {
    std::fprintf(stderr, "        armtd_main: %s\n", msg);
    std::ofstream o(out1);
    o << -1;
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string dir = buffer_dir(argc, argv);
    const std::string in = dir + "armtd.in", out1 = dir + "armtd.out";
    { std::ofstream o(out1); }  // a fresh armtd.out on every run (ACMP/armtd_main.cu:35)

    int T = 100;
    if (const char* e = std::getenv("ARMOUR_NUM_TIME_STEPS")) T = std::atoi(e);
    if (T <= 0) return fail_out(out1, "bad ARMOUR_NUM_TIME_STEPS");

    armour_armtd_world w;
    std::vector<double> tables((size_t)NF * 6 * T), obs;
    int O = 0;
    {
        std::ifstream is(in);
        if (!is.is_open()) return fail_out(out1, "error reading input file");
        for (double* v : {w.q0, w.qd0, w.q_des})
            for (int i = 0; i < NF; i++) is >> v[i];
        for (int i = 0; i < NF; i++) {  // ACMP/armtd_main.cu:70-90
            for (int k = 0; k < 6; k++)
                for (int j = 0; j < T; j++) is >> tables[((size_t)i * 6 + k) * T + j];
            is >> w.k_range[i];
        }
        is >> O;
        if (O > MAX_OBSTACLES || O < 0) return fail_out(out1, "number of obstacles larger than MAX_OBSTACLE_NUM");
        obs.assign((size_t)O * ARMOUR_OBSTACLE_DOUBLES, 0.0);
        for (double& v : obs) is >> v;
    }
    w.jrs_tables = tables.data();
    w.num_obstacles = O;
    w.obstacles = O > 0 ? obs.data() : nullptr;

    armour_config cfg{0, T, O, 1, 0, 0};
    armour_planner* p = armour_create_armtd(&cfg);
    if (!p) return fail_out(out1, armour_last_error());
    armour_result r;
    armour_timing tm;
    if (armour_plan_armtd_batch(p, 1, &w, &r, &tm) != 0) {
        const int rc = fail_out(out1, armour_last_error());
        armour_destroy(p);
        return rc;
    }
    std::cout << "        HIP: reachable sets " << tm.reach_ms << " ms, solver " << tm.nlp_ms << " ms, "
              << (r.feasible ? "found a feasible solution" : "no feasible solution") << std::endl;
    if (r.error) std::fprintf(stderr, "        armtd_main: %s\n", armour_last_error());

    const int NJ = armour_num_joints(p);
    const int m = armour_num_constraints(p, O);
    std::vector<double> centers((size_t)T * NJ * 3), gens((size_t)T * NJ * 18), g(m);
    int rc = armour_get_link_centers(p, 0, centers.data());
    rc = rc ? rc : armour_get_link_generators(p, 0, gens.data());
    rc = rc ? rc : armour_get_constraints(p, 0, g.data());
    if (rc) {
        const int e = fail_out(out1, armour_last_error());
        armour_destroy(p);
        return e;
    }
    armour_destroy(p);

    {
        std::ofstream o(out1);
        o << std::setprecision(10);
        if (r.feasible)
            for (int i = 0; i < NF; i++) o << r.k_opt[i] << '\n';
        else
            o << -1 << '\n';
        o << (long)(tm.reach_ms + tm.nlp_ms);
    }
    {
        std::ofstream o(dir + "armtd_joint_position_center.out");
        o << std::setprecision(10);
        for (int t = 0; t < T; t++)
            for (int j = 0; j < NJ; j++) {
                for (int l = 0; l < 3; l++) o << centers[((size_t)t * NJ + j) * 3 + l] << ' ';
                o << '\n';
            }
    }
    {
        std::ofstream o(dir + "armtd_joint_position_radius.out");
        o << std::setprecision(10);
        for (int t = 0; t < T; t++)
            for (int j = 0; j < NJ; j++)
                for (int k = 0; k < 3; k++) {
                    for (int l = 0; l < 6; l++) o << gens[(((size_t)t * NJ + j) * 3 + k) * 6 + l] << ' ';
                    o << '\n';
                }
    }
    {
        std::ofstream o(dir + "armtd_constraints.out");
        o << std::setprecision(6);
        for (int i = 0; i < m; i++) o << g[i] << '\n';
    }
    return 0;
}
