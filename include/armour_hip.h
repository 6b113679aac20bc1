/* armour_hip.h — C ABI of the MI355X-native ARMOUR planner (libarmour_hip.so).
 *
 * Drop-in boundary. The reference exposes its hot path to MATLAB as a process
 * (KPR/armour_main.cu:12-400) driven through text files by KSI/uarmtd_planner.m:167-230; there is
 * no mex entry. This library is what that process becomes: one call plans a batch of worlds on a
 * GPU, each world being exactly one armour.in (KPR/README.md:99-112, armour_main.cu:54-77), each
 * result exactly one armour*.out set (armour_main.cu:319-398). The drop-in executable
 * `armour_main` (armour-dev_amd/csrc/armour_main.cpp) speaks the file protocol on top of it.
 *
 * Plain C types only; caller-owned inputs and outputs; one planner handle per thread.
 * Every function returns 0 on success or a negative ARMOUR_E_* code; armour_last_error() gives
 * the message (thread-local).
 */
#ifndef ARMOUR_HIP_H
#define ARMOUR_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ARMOUR_NUM_FACTORS 7      /* NUM_FACTORS (KPR/KinovaWithoutGripperInfo.h:14) */
#define ARMOUR_OBSTACLE_DOUBLES 12 /* center + 3 generators (armour_main.cu:45, uarmtd_planner.m:189) */

enum {
    ARMOUR_OK = 0,
    ARMOUR_E_ARG = -1,       /* invalid argument (sizes, null pointers) */
    ARMOUR_E_HIP = -2,       /* HIP runtime error / no device */
    ARMOUR_E_CAPACITY = -3,  /* a reach-set job exceeded its arena / sort / output capacity */
    ARMOUR_E_STATE = -4,     /* query before a plan / reach call */
    ARMOUR_E_INTERNAL = -5   /* per-world result only: the solver left this world in a non-terminal
                                state (a solver fault; reported infeasible, not planned) */
};

typedef struct armour_planner armour_planner;

typedef struct armour_config {
    int robot;           /* 0: Kinova Gen3 without gripper (KPR/KinovaWithoutGripperInfo.h) */
    int num_time_steps;  /* NUM_TIME_STEPS (KPR/Parameters.h:17), runtime here, must be even */
    int max_obstacles;   /* per world; MAX_OBSTACLE_NUM (KPR/Parameters.h:26) is 40 */
    int max_worlds;      /* batch capacity */
    int device;          /* HIP device ordinal (-1: current device) */
    int max_iter;        /* solver iteration cap (0: default 100) */
} armour_config;

/* one planning problem: the content of armour.in */
typedef struct armour_world {
    double q0[ARMOUR_NUM_FACTORS];
    double qd0[ARMOUR_NUM_FACTORS];
    double qdd0[ARMOUR_NUM_FACTORS];
    double q_des[ARMOUR_NUM_FACTORS];
    int num_obstacles;
    const double* obstacles; /* [num_obstacles][12] */
} armour_world;

/* one planning result: armour.out (k_opt or infeasible) + solver statistics */
typedef struct armour_result {
    double k_opt[ARMOUR_NUM_FACTORS]; /* normalised, in [-1, 1] (MATLAB scales by pi/48) */
    int feasible;        /* finalize_solution re-check (KPR/NLPclass.cu:449-538) */
    int solver_status;   /* 0 converged, 1 iteration cap, 2 line-search failure (no restoration phase
                            left), 3 not planned (see error), 4 local infeasibility (the restoration
                            phase found no point within the bounds: Ipopt's Infeasible_Problem_Detected
                            role) */
    int iterations;
    int evaluations;
    double cost;         /* objective / COST_FUNCTION_OPTIMALITY_SCALE at k_opt */
    double kkt_error;
    int error;           /* 0, or ARMOUR_E_CAPACITY: this world's reach set exceeded a capacity even
                            after the retry with 4x buffers; it is reported infeasible and not planned,
                            the other worlds of the batch are (armour_plan_batch still returns 0);
                            or ARMOUR_E_INTERNAL (a solver fault, never expected) */
} armour_result;

/* timings of the last batch, device-side (hipEvents on the planner's stream), milliseconds */
typedef struct armour_timing {
    double reach_ms;     /* JRS + PZ FK/RNEA + torque radius + hyperplanes */
    double nlp_ms;       /* solver */
    double total_ms;     /* incl. host<->device copies of inputs and results */
    double reach_kernel_ms; /* reach_kernel alone (hipEvents around its launch) */
    double reach_bytes;  /* algorithmic monomial bytes the PZ operators read + wrote */
} armour_timing;

armour_planner* armour_create(const armour_config* cfg);
void armour_destroy(armour_planner* p);

/* Robot tables: the content of the reference's compile-time robot header (Kinova:
 * KPR/KinovaWithoutGripperInfo.h:10-112; Fetch: ACMP/FetchInfo.h:8-107) as run-time data, so a
 * robot is data rather than a rebuild. Joint i rotates about axis |axes[i]| (1 x, 2 y, 3 z; negative:
 * reversed; 0: fixed) after the frame offset trans[i] / rots[i] (URDF joint origin xyz / rpy);
 * link i (the child of joint i) has mass, centre of mass, inertia (row-major 3x3) and a box
 * zonotope (centre, half extents: the STL bounding box of create_pz_bounding_boxes.m). The first
 * ARMOUR_NUM_FACTORS joints are the actuated ones. armour_amd/robot_tables.py builds these from a
 * URDF and its meshes. */
#define ARMOUR_MAX_JOINTS 9
typedef struct armour_robot {
    int num_joints;                               /* NUM_JOINTS, 7..9 */
    int axes[ARMOUR_MAX_JOINTS];
    int wrap[ARMOUR_NUM_FACTORS];                 /* continuous joints: cost term wrapped to [-pi, pi] */
    double trans[(ARMOUR_MAX_JOINTS + 1) * 3];
    double rots[ARMOUR_MAX_JOINTS * 3];
    double mass[ARMOUR_MAX_JOINTS];
    double com[ARMOUR_MAX_JOINTS * 3];
    double inertia[ARMOUR_MAX_JOINTS * 9];
    double mass_uncertainty, inertia_uncertainty;
    double friction[ARMOUR_MAX_JOINTS], damping[ARMOUR_MAX_JOINTS], armature[ARMOUR_MAX_JOINTS];
    double state_lb[ARMOUR_NUM_FACTORS], state_ub[ARMOUR_NUM_FACTORS];  /* +-1000: continuous */
    double speed_limits[ARMOUR_NUM_FACTORS], torque_limits[ARMOUR_NUM_FACTORS];
    double gravity;
    double link_center[ARMOUR_MAX_JOINTS * 3], link_generators[ARMOUR_MAX_JOINTS * 3];
    double alpha, V_m, M_max, M_min, K;           /* ultimate bound of the robust controller */
} armour_robot;

/* compute units of a HIP device (< 0: error). The reach kernel runs one 64-job bundle per CU at a
 * time, so batches of whole bundle waves, W = k * CUs * 64 / num_time_steps worlds, fill the chip. */
int armour_device_compute_units(int device);

/* Diagnostics: device-to-device copy bandwidth of `bytes` (two buffers of that size) with a
 * 16-B-per-lane streaming kernel, `reps` timed copies; GB/s of read + write bytes, or a negative
 * ARMOUR_E_* code. The achievable HBM figure the roofline fractions are read against. */
double armour_copy_bandwidth(int device, size_t bytes, int reps);

/* built-in tables (robot id 0: Kinova Gen3 without gripper); 0 / ARMOUR_E_ARG */
int armour_robot_builtin(int robot_id, armour_robot* out);
/* armour_create with the given robot tables (cfg->robot is ignored) */
armour_planner* armour_create_robot(const armour_config* cfg, const armour_robot* robot);
const char* armour_last_error(void);

/* constraints of a world with O obstacles: 7T + NJ*T*O + 28 (KPR/NLPclass.cu:47-49); ARMTD
 * planners NJ*T*O + 28 (ACMP/NLPclass.cu:45-46) */
int armour_num_constraints(const armour_planner* p, int num_obstacles);

/* Plan a batch (all worlds must carry the same number of obstacles). Replaces
 * armour_main.cu:87-316 for each world. */
int armour_plan_batch(armour_planner* p, int num_worlds, const armour_world* worlds, armour_result* results,
                      armour_timing* timing);

/* One plan, the whole of one armour_main.cu process (:37-398) on a planner handle: the single-world
 * entry of SURVEY.md §8(b). Inputs are the content of armour.in (caller-owned); the result and timing
 * are written into *out, and so is every output array the caller supplies (null: skipped) — the
 * payloads of the five .out files. Equivalent to armour_plan_batch with one world followed by the
 * getters (world 0). 0 or a negative ARMOUR_E_* code; thread-safe per handle like every entry. */
typedef struct armour_plan_output {
    armour_result result;       /* k_opt (armour.out unless infeasible), feasible, solver status ... */
    armour_timing timing;
    double* constraints;        /* [m] at the final iterate (armour_constraints.out, first m lines) */
    double* joint_bounds;       /* [28] (armour_constraints.out, last 28 lines) */
    double* link_centers;       /* [T][NJ][3] (armour_joint_position_center.out) */
    double* link_generators;    /* [T][NJ][3][6] (armour_joint_position_radius.out) */
    double* torque_radius;      /* [T][7] (armour_control_input_radius.out) */
} armour_plan_output;
int armour_plan(armour_planner* p, const armour_world* world, armour_plan_output* out);

/* The ARMTD comparison planner (kinova_planner_realtime_armtd_comparison/, "ACMP/"): the content
 * of one armtd.in (ACMP/armtd_main.cu:37-102). Joint rotations come from offline JRS tables that the
 * caller slices (KSI/uarmtd_planner.m:260-318) instead of the Bernstein trajectory; the plan keeps
 * forward kinematics and collision avoidance (no RNEA, no torque rows), with the constant-
 * acceleration joint extrema and cost of ACMP/Trajectory.cu:83-383, ACMP/NLPclass.cu:186-246. */
typedef struct armour_armtd_world {
    double q0[ARMOUR_NUM_FACTORS];
    double qd0[ARMOUR_NUM_FACTORS];
    double q_des[ARMOUR_NUM_FACTORS];
    const double* jrs_tables;  /* [7][6][num_time_steps]: per joint c_cos, g_cos, r_cos, c_sin, g_sin, r_sin */
    double k_range[ARMOUR_NUM_FACTORS];
    int num_obstacles;
    const double* obstacles;   /* [num_obstacles][12] */
} armour_armtd_world;

/* an ARMTD planner (the reference's NUM_TIME_STEPS is 100, ACMP/Parameters.h:17; solver tolerance
 * 1e-7, :42); armour_num_constraints gives 7*T*O + 28, the getters work as for armour_create */
armour_planner* armour_create_armtd(const armour_config* cfg);
int armour_plan_armtd_batch(armour_planner* p, int num_worlds, const armour_armtd_world* worlds,
                            armour_result* results, armour_timing* timing);
int armour_reach_armtd_batch(armour_planner* p, int num_worlds, const armour_armtd_world* worlds, armour_timing* timing);

/* Reach-set half only (armour_main.cu:87-222) for a batch; enables armour_eval_constraints. */
int armour_reach_batch(armour_planner* p, int num_worlds, const armour_world* worlds, armour_timing* timing);

/* eval_g / eval_jac_g (KPR/NLPclass.cu:272-396) of world w of the last batch at x; jac (m x 7,
 * row-major) may be null. The parity-pinning entry. */
int armour_eval_constraints(armour_planner* p, int w, const double* x, double* g, double* jac);

/* Outputs of world w of the last batch (the armour_*.out payloads, armour_main.cu:340-398) */
int armour_get_constraints(armour_planner* p, int w, double* g);              /* m values at k_opt */
int armour_get_link_centers(armour_planner* p, int w, double* centers);       /* [T][NJ][3] sliced at the
                                                                               last evaluated point: k_opt after a plan */
int armour_get_link_generators(armour_planner* p, int w, double* gens);       /* [T][NJ][3][6] */
int armour_get_torque_radius(armour_planner* p, int w, double* radius);       /* [T][7] */
int armour_num_joints(const armour_planner* p);
/* k-only monomials of world w's link PZs [T][NJ] and torque PZs [T][7] after reduce_link_PZ /
 * reduce (the M_links, M_tau of SURVEY.md §8(d)'s per-plan byte count); either may be null */
int armour_get_monomial_counts(armour_planner* p, int w, int* link_counts, int* torque_counts);
/* the 28 trailing values of armour_constraints.out (armour_main.cu:385-396): per joint
 * [lb + qe, ub - qe] then per joint [-v + qde, v - qde] */
int armour_get_joint_bounds(const armour_planner* p, double* bounds28);

/* Diagnostics (no reference counterpart). The reach kernel interprets a fixed op program built
 * from the robot tables; these expose it for profiling. armour_get_reach_program writes the op
 * codes (if capacity >= count) and returns the op count. armour_get_reach_profile writes
 * [cycles, terms] per op accumulated over all jobs when the environment variable
 * ARMOUR_PROFILE_OPS was set at armour_create, followed by 16 phase counters of the operator
 * paths (capacity counts pairs: >= op count + 8), and returns the op count. */
int armour_get_reach_program(const armour_planner* p, int* codes, int capacity);
/* Capacity headroom of the last reach (bundle engine): for k < n writes the largest use over the
 * batch and its capacity: [0] arena union hashes, [1] arena coefficient rows, [2] terms of one
 * operator (sort keys), [3] k-only monomials of a link PZ (reduce_link_PZ output), [4] k-only
 * monomials of a torque PZ, [5] worlds retried with 4x buffers (cap: W), [6] worlds that still
 * failed (cap: W). Returns ARMOUR_OCC_COUNT. */
#define ARMOUR_OCC_COUNT 7
int armour_get_reach_occupancy(armour_planner* p, long long* used, long long* caps, int n);
int armour_get_reach_profile(armour_planner* p, unsigned long long* cycles_terms, int capacity);
/* Certified plane cache of the current reach sets, built on demand: for k < n
 * writes [0] planes kept over all (world, t, link, obstacle) pairs, [1] pairs, [2] (world, t) blocks
 * whose cache region held every kept plane, [3] blocks, [4] most planes kept for one pair,
 * [5] records in the cache pool, [6] evaluations that found a point outside the cache's box (rows
 * NaN; the solver never produces one). Returns ARMOUR_PC_COUNT; ARMOUR_E_STATE when the cache is off. */
#define ARMOUR_PC_COUNT 7
int armour_get_plane_cache_stats(armour_planner* p, long long* out, int n);
/* Execution span of the last reach launch on the device clock (wall_clock64): from the first
 * workgroup's start to the last workgroup's end, the duration rocprofv3 --kernel-trace reports
 * for the kernel (the reach_kernel_ms of armour_timing, HIP events around the launch, also counts
 * the time the launch waits for CUs held by other planners' kernels). Milliseconds. */
int armour_get_reach_span(armour_planner* p, double* span_ms);
/* op-by-op state of job 0 (world 0, t = 0) of the last reach: per op 8 doubles [monomial count,
 * block size, centre[0..2], nominal ind[0], interval ind[0], sum|m|[0]] of the op's output, when
 * ARMOUR_DUMP_OPS was set at armour_create; returns the op count. */
int armour_get_reach_dump(armour_planner* p, double* dump, int capacity);

#ifdef __cplusplus
}
#endif
#endif
