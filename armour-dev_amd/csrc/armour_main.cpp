// armour_main — drop-in replacement for the reference planner process
// (kinova_planner_realtime/armour_main.cu), built on the C ABI of libarmour_hip.so.
//
// Same file protocol as the reference (armour_main.cu:5-10, 37-77, 319-398; driven by
// KSI/uarmtd_planner.m:167-230):
//   in : <buffer>/armour.in   7 q0, 7 qd0, 7 qdd0, 7 q_des, int O, O x 12 obstacle doubles
//   out: <buffer>/armour.out                         k_opt (7 lines, precision 10) or -1, then ms
//        <buffer>/armour_joint_position_center.out   T*NJ rows of 3 (sliced link centres)
//        <buffer>/armour_joint_position_radius.out   T*NJ*3 rows of 6 (link generators)
//        <buffer>/armour_control_input_radius.out    T rows of 7 (torque radius)
//        <buffer>/armour_constraints.out             m constraint values (precision 6), then the
//                                                    14 position and 14 velocity bounds
// Errors follow the reference: unreadable input or a bad obstacle count writes -1 to armour.out
// and exits non-zero (the reference's bare `throw;` terminates the process).
//
// Buffer directory: argv[1], else $ARMOUR_BUFFER_DIR, else the build-time ARMOUR_BUFFER_PATH
// (the reference bakes it into BufferPath.h), else <directory of this executable>/buffer/.
// Time steps: $ARMOUR_NUM_TIME_STEPS, default 128 (NUM_TIME_STEPS, KPR/Parameters.h:17).
#include <unistd.h>

#include <chrono>
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
constexpr int MAX_OBSTACLES = 40;  // MAX_OBSTACLE_NUM (KPR/Parameters.h:26)

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
        std::string exe = n > 0 ? std::string(buf, (size_t)n) : std::string("./armour_main");
        d = exe.substr(0, exe.find_last_of('/') + 1) + "buffer";
    }
#endif
    if (!d.empty() && d.back() != '/') d += '/';
    return d;
}

int fail_out(const std::string& out1, const char* msg) {
    std::fprintf(stderr, "        armour_main: %s\n", msg);
    std::ofstream o(out1);
    o << -1;
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string dir = buffer_dir(argc, argv);
    const std::string in = dir + "armour.in", out1 = dir + "armour.out";
    // a fresh armour.out on every run, as the reference (armour_main.cu:36-37)
    { std::ofstream o(out1); }

    double q0[NF], qd0[NF], qdd0[NF], qdes[NF];
    int O = 0;
    std::vector<double> obs;
    {
        std::ifstream is(in);
        if (!is.is_open()) return fail_out(out1, "error reading input file");
        for (double* v : {q0, qd0, qdd0, qdes})
            for (int i = 0; i < NF; i++) is >> v[i];
        is >> O;
        if (O > MAX_OBSTACLES || O < 0) return fail_out(out1, "number of obstacles larger than MAX_OBSTACLE_NUM");
        obs.assign((size_t)O * ARMOUR_OBSTACLE_DOUBLES, 0.0);
        for (double& v : obs) is >> v;
    }

    int T = 128;
    if (const char* e = std::getenv("ARMOUR_NUM_TIME_STEPS")) T = std::atoi(e);
    armour_config cfg{0, T, O, 1, 0, 0};
    armour_planner* p = armour_create(&cfg);
    if (!p) return fail_out(out1, armour_last_error());

    armour_world w;
    for (int i = 0; i < NF; i++) { w.q0[i] = q0[i]; w.qd0[i] = qd0[i]; w.qdd0[i] = qdd0[i]; w.q_des[i] = qdes[i]; }
    w.num_obstacles = O;
    w.obstacles = O > 0 ? obs.data() : nullptr;

    armour_result r;
    armour_timing tm;
    if (armour_plan_batch(p, 1, &w, &r, &tm) != 0) {
        const int rc = fail_out(out1, armour_last_error());
        armour_destroy(p);
        return rc;
    }
    std::cout << "        HIP: reachable sets " << tm.reach_ms << " ms, solver " << tm.nlp_ms << " ms, "
              << (r.feasible ? "found a feasible solution" : "no feasible solution") << std::endl;
    // a reach set over the library's capacity is not planned: reported as no feasible solution
    // (-1, MATLAB keeps its braking trajectory), with the reason on stderr
    if (r.error) std::fprintf(stderr, "        armour_main: %s\n", armour_last_error());

    const int NJ = armour_num_joints(p);
    const int m = armour_num_constraints(p, O);
    std::vector<double> centers((size_t)T * NJ * 3), gens((size_t)T * NJ * 18), rad((size_t)T * NF), g(m), bounds(4 * NF);
    int rc = armour_get_link_centers(p, 0, centers.data());
    rc = rc ? rc : armour_get_link_generators(p, 0, gens.data());
    rc = rc ? rc : armour_get_torque_radius(p, 0, rad.data());
    rc = rc ? rc : armour_get_constraints(p, 0, g.data());
    rc = rc ? rc : armour_get_joint_bounds(p, bounds.data());
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
        std::ofstream o(dir + "armour_joint_position_center.out");
        o << std::setprecision(10);
        for (int t = 0; t < T; t++)
            for (int j = 0; j < NJ; j++) {
                for (int l = 0; l < 3; l++) o << centers[((size_t)t * NJ + j) * 3 + l] << ' ';
                o << '\n';
            }
    }
    {
        std::ofstream o(dir + "armour_joint_position_radius.out");
        o << std::setprecision(10);
        for (int t = 0; t < T; t++)
            for (int j = 0; j < NJ; j++)
                for (int k = 0; k < 3; k++) {
                    for (int l = 0; l < 6; l++) o << gens[(((size_t)t * NJ + j) * 3 + k) * 6 + l] << ' ';
                    o << '\n';
                }
    }
    {
        std::ofstream o(dir + "armour_control_input_radius.out");
        o << std::setprecision(10);
        for (int t = 0; t < T; t++) {
            for (int j = 0; j < NF; j++) o << rad[(size_t)t * NF + j] << ' ';
            o << '\n';
        }
    }
    {
        std::ofstream o(dir + "armour_constraints.out");
        o << std::setprecision(6);
        for (int i = 0; i < m; i++) o << g[i] << '\n';
        for (int i = 0; i < 4 * NF; i++) o << bounds[i] << '\n';
    }
    return 0;
}
