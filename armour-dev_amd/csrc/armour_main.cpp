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
//
// Served mode ("optional persistent daemon keeps GPU context warm"). MATLAB starts a
// new armour_main for every replan (uarmtd_planner.m:200); process start, HIP initialisation and
// the planner's allocations are ~97 % of such a run. `armour_main --serve [buffer]` creates the
// planner once (max_obstacles = MAX_OBSTACLE_NUM) and listens on <buffer>/armour.sock (or
// $ARMOUR_SERVE_SOCKET). A plain `armour_main` first tries that socket: when a server answers, it
// sends its buffer directory, the server plans that directory's armour.in and writes the same five
// files, and the client exits with the server's status. Otherwise it plans in-process. The HIP
// library is loaded with dlopen only on the in-process and server paths, so a served client never
// maps the HIP runtime.
// The request is one line: the client's buffer directory as an absolute path (realpath), the
// horizon T and every ARMOUR_* setting of the client's environment that changes a plan (plan_env),
// tab-separated. A server whose T or settings differ answers REFUSED and the client plans
// in-process, so a server never plans another horizon or solver configuration than the client
// would. The client truncates armour.out before it asks (MATLAB never reads a previous replan's
// k_opt) and waits at most $ARMOUR_SERVE_TIMEOUT_MS (default 10000, the reference's time budget
// scale) for the answer; a server that does not answer in time leaves -1 in armour.out and a
// non-zero exit, as any failed replan.
#include <dlfcn.h>
#include <fcntl.h>
#include <limits.h>
#include <poll.h>
#include <signal.h>
#include <sys/file.h>
#include <sys/time.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/armour_hip.h"

extern char** environ;

namespace {

constexpr int NF = ARMOUR_NUM_FACTORS;
constexpr int MAX_OBSTACLES = 40;  // MAX_OBSTACLE_NUM (KPR/Parameters.h:26)

std::string exe_dir() {
    char buf[4096];
    const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
    const std::string exe = n > 0 ? std::string(buf, (size_t)n) : std::string("./armour_main");
    return exe.substr(0, exe.find_last_of('/') + 1);
}

std::string buffer_dir(const char* arg) {
    std::string d;
    if (arg) d = arg;
    else if (const char* e = std::getenv("ARMOUR_BUFFER_DIR")) d = e;
#ifdef ARMOUR_BUFFER_PATH
    else d = ARMOUR_BUFFER_PATH;
#else
    else d = exe_dir() + "buffer";
#endif
    if (!d.empty() && d.back() != '/') d += '/';
    return d;
}

std::string socket_path(const std::string& dir) {
    if (const char* e = std::getenv("ARMOUR_SERVE_SOCKET")) return e;
    return dir + "armour.sock";
}

int fail_out(const std::string& out1, const char* msg) {
    std::fprintf(stderr, "        armour_main: %s\n", msg);
    std::ofstream o(out1);
    o << -1;
    return 1;
}

// the C ABI of libarmour_hip.so, resolved at run time
struct Lib {
    decltype(&armour_create) create;
    decltype(&armour_destroy) destroy;
    decltype(&armour_last_error) last_error;
    decltype(&armour_plan) plan;
    decltype(&armour_num_joints) num_joints;
    decltype(&armour_num_constraints) num_constraints;

    bool load(std::string& why) {
        const char* env = std::getenv("ARMOUR_LIB");
        const std::string path = env ? env : exe_dir() + "libarmour_hip.so";
        void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            why = dlerror();
            return false;
        }
        bool ok = true;
        auto sym = [&](auto& f, const char* name) {
            f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
            ok = ok && f;
        };
        sym(create, "armour_create");
        sym(destroy, "armour_destroy");
        sym(last_error, "armour_last_error");
        sym(plan, "armour_plan");
        sym(num_joints, "armour_num_joints");
        sym(num_constraints, "armour_num_constraints");
        if (!ok) why = "libarmour_hip.so lacks an armour_* symbol";
        return ok;
    }
};

int time_steps() {
    const char* e = std::getenv("ARMOUR_NUM_TIME_STEPS");
    return e ? std::atoi(e) : 128;
}

// output text of one .out file: numbers as printf's %.<prec>g (the ofstream setprecision format)
struct Text {
    std::string s;
    Text& num(double v, int prec) {
        char b[40];
        const auto r = std::to_chars(b, b + sizeof(b), v, std::chars_format::general, prec);
        s.append(b, r.ptr);
        return *this;
    }
    Text& ch(char c) { s += c; return *this; }
    Text& str(const std::string& t) { s += t; return *this; }
    bool save(const std::string& path) {  // writes and clears
        FILE* f = std::fopen(path.c_str(), "wb");
        const bool ok = f && std::fwrite(s.data(), 1, s.size(), f) == s.size();
        if (f) std::fclose(f);
        if (!ok) std::fprintf(stderr, "armour_main: cannot write %s\n", path.c_str());
        s.clear();
        return ok;
    }
};

// Served outputs are written as <file>.part and renamed into place only while the client still
// waits, under an flock on <dir>/armour.lock that a timed-out client also takes before it writes
// its -1: a plan that finishes after its client gave up (or after the next client truncated
// armour.out) is discarded, never mixed into a later replan's files.
bool peer_waiting(int fd) {
    pollfd pf{fd, POLLIN, 0};
    if (poll(&pf, 1, 0) < 0 || (pf.revents & (POLLHUP | POLLERR | POLLNVAL))) return false;
    if (pf.revents & POLLIN) {
        char b;
        return recv(fd, &b, 1, MSG_PEEK | MSG_DONTWAIT) > 0;  // 0: the client closed its end
    }
    return true;
}
struct DirLock {
    int fd;
    explicit DirLock(const std::string& dir) : fd(open((dir + "armour.lock").c_str(), O_CREAT | O_RDWR, 0644)) {
        if (fd >= 0) (void)!flock(fd, LOCK_EX);
    }
    ~DirLock() {
        if (fd >= 0) { (void)!flock(fd, LOCK_UN); close(fd); }
    }
};

// One replan of the buffer directory `dir`: read armour.in, plan, write the five outputs. With
// `served` a planner of the right horizon is given (capacity MAX_OBSTACLE_NUM) and `client` is the
// requesting socket (outputs committed only while it waits); otherwise a planner is created for
// this input and destroyed.
int plan_dir(const Lib& L, armour_planner* served, const std::string& dir, int client = -1) {
    const std::string in = dir + "armour.in", out1 = dir + "armour.out";
    // a fresh armour.out on every run, as the reference (armour_main.cu:36-37); a served request's
    // client truncated it already (a server must not touch the file of a client that gave up)
    if (client < 0) { std::ofstream o(out1); }
    // served: the .part files written so far are removed on every return that does not commit
    // them, and a failure writes its -1 under the directory lock only while the client waits (the
    // commit protocol below), so a late failure never touches a directory its client left
    std::vector<std::string> parts;
    struct PartSweep {
        std::vector<std::string>& parts;
        ~PartSweep() {
            for (const auto& f : parts) std::remove((f + ".part").c_str());
        }
    } sweep{parts};
    auto fail = [&](const char* msg) {
        if (client < 0) return fail_out(out1, msg);
        DirLock lk(dir);
        if (peer_waiting(client)) return fail_out(out1, msg);
        std::fprintf(stderr, "armour_main --serve: client of %s gave up; failure (%s) discarded\n", dir.c_str(), msg);
        return 1;
    };

    double q0[NF], qd0[NF], qdd0[NF], qdes[NF];
    int O = 0;
    std::vector<double> obs;
    {
        std::ifstream is(in);
        if (!is.is_open()) return fail("error reading input file");
        for (double* v : {q0, qd0, qdd0, qdes})
            for (int i = 0; i < NF; i++) is >> v[i];
        is >> O;
        if (O > MAX_OBSTACLES || O < 0) return fail("number of obstacles larger than MAX_OBSTACLE_NUM");
        obs.assign((size_t)O * ARMOUR_OBSTACLE_DOUBLES, 0.0);
        for (double& v : obs) is >> v;
    }

    const int T = time_steps();
    armour_planner* p = served;
    if (!p) {
        armour_config cfg{0, T, O, 1, 0, 0};
        p = L.create(&cfg);
        if (!p) return fail(L.last_error());
    }
    struct Owned {
        const Lib& L;
        armour_planner* p;
        ~Owned() { if (p) L.destroy(p); }
    } owned{L, served ? nullptr : p};

    armour_world w;
    for (int i = 0; i < NF; i++) { w.q0[i] = q0[i]; w.qd0[i] = qd0[i]; w.qdd0[i] = qdd0[i]; w.q_des[i] = qdes[i]; }
    w.num_obstacles = O;
    w.obstacles = O > 0 ? obs.data() : nullptr;

    // one plan through the single-world entry (armour_plan): the result and the payloads of the
    // five .out files
    const int NJ = L.num_joints(p);
    const int m = L.num_constraints(p, O);
    std::vector<double> centers((size_t)T * NJ * 3), gens((size_t)T * NJ * 18), rad((size_t)T * NF), g(m), bounds(4 * NF);
    armour_plan_output po{};
    po.constraints = g.data();
    po.joint_bounds = bounds.data();
    po.link_centers = centers.data();
    po.link_generators = gens.data();
    po.torque_radius = rad.data();
    if (L.plan(p, &w, &po) != 0) return fail(L.last_error());
    const armour_result& r = po.result;
    const armour_timing& tm = po.timing;
    std::cout << "        HIP: reachable sets " << tm.reach_ms << " ms, solver " << tm.nlp_ms << " ms, "
              << (r.feasible ? "found a feasible solution" : "no feasible solution") << std::endl;
    // a reach set over the library's capacity is not planned: reported as no feasible solution
    // (-1, MATLAB keeps its braking trajectory), with the reason on stderr
    if (r.error) std::fprintf(stderr, "        armour_main: %s\n", L.last_error());

    // the reference's writers are ofstreams at setprecision(10) / (6) (armour_main.cu:319-398),
    // i.e. printf's %.10g / %.6g; std::to_chars(general, precision) is specified as exactly that
    // conversion and is several times faster for the ~40k numbers a T = 128 plan writes
    auto dst = [&](const std::string& name) {  // served: the .part files to commit (`parts`)
        if (client < 0) return dir + name;
        parts.push_back(dir + name);
        return dir + name + ".part";
    };
    Text o;
    if (r.feasible)
        for (int i = 0; i < NF; i++) o.num(r.k_opt[i], 10).ch('\n');
    else
        o.str("-1\n");
    o.str(std::to_string((long)(tm.reach_ms + tm.nlp_ms)));
    if (!o.save(dst("armour.out"))) return 1;
    for (int t = 0; t < T; t++)
        for (int j = 0; j < NJ; j++) {
            for (int l = 0; l < 3; l++) o.num(centers[((size_t)t * NJ + j) * 3 + l], 10).ch(' ');
            o.ch('\n');
        }
    if (!o.save(dst("armour_joint_position_center.out"))) return 1;
    for (int t = 0; t < T; t++)
        for (int j = 0; j < NJ; j++)
            for (int k = 0; k < 3; k++) {
                for (int l = 0; l < 6; l++) o.num(gens[(((size_t)t * NJ + j) * 3 + k) * 6 + l], 10).ch(' ');
                o.ch('\n');
            }
    if (!o.save(dst("armour_joint_position_radius.out"))) return 1;
    for (int t = 0; t < T; t++) {
        for (int j = 0; j < NF; j++) o.num(rad[(size_t)t * NF + j], 10).ch(' ');
        o.ch('\n');
    }
    if (!o.save(dst("armour_control_input_radius.out"))) return 1;
    for (int i = 0; i < m; i++) o.num(g[i], 6).ch('\n');
    for (int i = 0; i < 4 * NF; i++) o.num(bounds[i], 6).ch('\n');
    if (!o.save(dst("armour_constraints.out"))) return 1;
    if (client >= 0) {
        if (const char* e = std::getenv("ARMOUR_SERVE_DELAY_MS")) usleep((useconds_t)std::atol(e) * 1000);  // tests
        DirLock lk(dir);
        const bool keep = peer_waiting(client);
        for (const auto& f : parts) {
            const std::string tmp = f + ".part";
            if (!keep || std::rename(tmp.c_str(), f.c_str()) != 0) std::remove(tmp.c_str());
        }
        parts.clear();
        if (!keep) {
            std::fprintf(stderr, "armour_main --serve: client of %s gave up; plan discarded\n", dir.c_str());
            return 1;
        }
    }
    return 0;
}

bool fill_addr(sockaddr_un& a, const std::string& path) {
    std::memset(&a, 0, sizeof(a));
    a.sun_family = AF_UNIX;
    if (path.size() >= sizeof(a.sun_path)) return false;
    std::memcpy(a.sun_path, path.c_str(), path.size());
    return true;
}

// ARMOUR_* settings of this process that change a plan (everything but the serving plumbing),
// sorted, as "K=V" joined by ';': client and server must agree on them
std::string plan_env() {
    static const char* plumbing[] = {"ARMOUR_BUFFER_DIR=", "ARMOUR_SERVE_SOCKET=", "ARMOUR_NO_SERVE=",
                                     "ARMOUR_SERVE_TIMEOUT_MS=", "ARMOUR_SERVE_DELAY_MS=", "ARMOUR_LIB="};
    std::vector<std::string> kv;
    for (char** e = environ; *e; e++) {
        const std::string v = *e;
        if (v.rfind("ARMOUR_", 0) != 0) continue;
        bool skip = false;
        for (const char* p : plumbing) skip = skip || v.rfind(p, 0) == 0;
        if (!skip) kv.push_back(v);
    }
    std::sort(kv.begin(), kv.end());
    std::string out;
    for (const auto& v : kv) out += (out.empty() ? "" : ";") + v;
    return out;
}

constexpr unsigned char SERVE_REFUSED = 254;  // server: T or settings differ (client plans in-process)

// client: -1 when no server answers or the server refuses the request (plan in-process), else the
// server's exit status
int try_served(const std::string& dir) {
    sockaddr_un a;
    if (!fill_addr(a, socket_path(dir))) return -1;
    char real[PATH_MAX];
    if (!realpath(dir.c_str(), real)) return -1;  // in-process: it reports the missing directory
    const int fd = socket(AF_UNIX, SOCK_STREAM, 0);
    if (fd < 0) return -1;
    if (connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
        close(fd);
        return -1;
    }
    const char* te = std::getenv("ARMOUR_SERVE_TIMEOUT_MS");
    const long ms = te ? std::atol(te) : 10000;
    timeval tv{ms / 1000, (ms % 1000) * 1000};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    const std::string out1 = std::string(real) + "/armour.out";
    { std::ofstream o(out1); }  // a fresh armour.out whatever the server does
    const std::string req = std::string(real) + "\t" + std::to_string(time_steps()) + "\t" + plan_env() + "\n";
    unsigned char rc = 1;
    const bool sent = write(fd, req.data(), req.size()) == (ssize_t)req.size();
    const bool got = sent && read(fd, &rc, 1) == 1;
    close(fd);
    if (got && rc == SERVE_REFUSED) return -1;
    if (!got) {
        // the socket is closed first, so a server that finishes later sees the client gone and
        // discards its plan; the lock orders this -1 against a commit already under way
        DirLock lk(std::string(real) + "/");
        return fail_out(out1, "the planning server did not answer (ARMOUR_SERVE_TIMEOUT_MS)");
    }
    return (int)rc;
}

std::string g_sock;
void on_signal(int) {
    if (!g_sock.empty()) unlink(g_sock.c_str());
    _exit(0);
}

int serve(const Lib& L, const std::string& dir) {
    const int T = time_steps();
    armour_config cfg{0, T, MAX_OBSTACLES, 1, 0, 0};
    armour_planner* p = L.create(&cfg);
    if (!p) {
        std::fprintf(stderr, "armour_main --serve: %s\n", L.last_error());
        return 1;
    }
    g_sock = socket_path(dir);
    sockaddr_un a;
    if (!fill_addr(a, g_sock)) {
        std::fprintf(stderr, "armour_main --serve: socket path too long: %s\n", g_sock.c_str());
        return 1;
    }
    const int fd = socket(AF_UNIX, SOCK_STREAM, 0);
    unlink(g_sock.c_str());
    if (fd < 0 || bind(fd, (sockaddr*)&a, sizeof(a)) != 0 || listen(fd, 16) != 0) {
        std::perror("armour_main --serve: socket");
        return 1;
    }
    signal(SIGTERM, on_signal);
    signal(SIGINT, on_signal);
    signal(SIGPIPE, SIG_IGN);
    const std::string env = plan_env();
    std::fprintf(stderr, "armour_main: serving %s (T = %d)\n", g_sock.c_str(), T);
    for (;;) {
        const int c = accept(fd, nullptr, nullptr);
        if (c < 0) continue;
        timeval tv{5, 0};  // a client that connects and sends nothing does not hold the server
        setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        std::string req;
        char buf[512];
        ssize_t n;
        while (req.find('\n') == std::string::npos && (n = read(c, buf, sizeof(buf))) > 0) req.append(buf, (size_t)n);
        const size_t e = req.find('\n');
        unsigned char rc = 1;
        if (e != std::string::npos) {
            // "<abs dir>\t<T>\t<settings>": plan only what this server's planner and environment
            // would plan for the client (else REFUSED: the client plans in-process)
            const std::string line = req.substr(0, e);
            const size_t t1 = line.find('\t'), t2 = t1 == std::string::npos ? t1 : line.find('\t', t1 + 1);
            if (t2 == std::string::npos || line.substr(t1 + 1, t2 - t1 - 1) != std::to_string(T) ||
                line.substr(t2 + 1) != env) {
                rc = SERVE_REFUSED;
            } else {
                std::string d = line.substr(0, t1);
                if (!d.empty() && d.back() != '/') d += '/';
                // a request whose client already gave up (it waited in the backlog behind a long
                // plan) is not planned
                rc = peer_waiting(c) ? (unsigned char)plan_dir(L, p, d, c) : 1;
                if (rc == SERVE_REFUSED) rc = 1;
            }
        }
        (void)!write(c, &rc, 1);
        close(c);
    }
}

}  // namespace

int main(int argc, char** argv) {
    const bool served = argc > 1 && std::strcmp(argv[1], "--serve") == 0;
    const char* arg = served ? (argc > 2 ? argv[2] : nullptr) : (argc > 1 ? argv[1] : nullptr);
    const std::string dir = buffer_dir(arg);
    if (!served && !std::getenv("ARMOUR_NO_SERVE")) {
        const int rc = try_served(dir);
        if (rc >= 0) return rc;
    }
    Lib L;
    std::string why;
    if (!L.load(why)) return fail_out(dir + "armour.out", why.c_str());
    return served ? serve(L, dir) : plan_dir(L, nullptr, dir);
}
