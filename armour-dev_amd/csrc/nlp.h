// armour-mi355x — device data layout of the batched NLP (W worlds planned together).
#pragma once
#include "reach.h"

namespace armour {

constexpr int EVAL_THREADS = 256;
constexpr int ROW_THREADS = 256;
constexpr int MAX_FILTER = 64;
constexpr int KA = 56;   // partial-sum slots per row block (pass A is the largest user)
constexpr int KA2 = 8;   // pass D's partial sums (partial2), kept apart so the fused D + A pass writes both

// solver options (oracle/src/ipm.h IpmOptions)
struct IpmOpts {
    double tol = 1e-4;
    int max_iter = 100;
    double mu0 = 0.1;
    double kappa_eps = 10.0;
    double kappa_mu = 0.2;
    double theta_mu = 1.5;
    double tau_min = 0.99;
    double bound_push = 1e-2;
    double eta = 1e-4;
    int max_ls = 10;
    double kappa_sigma = 1e10;
    double s_max = 100.0;
    double inf_bound = 1e19;
    // barrier strategy: 1 adaptive (default: the reference's IPOPT_MU_STRATEGY "adaptive",
    // KPR/Parameters.h:57, restated with Ipopt's LOQO mu oracle and kkt-error globalisation, mu on a
    // 2^(1/8) grid with floor tol / 10, as oracle/src/ipm.cpp); 0 monotone
    // (ARMOUR_MU_STRATEGY=monotone)
    int mu_strategy = 1;
    // restoration phase (nlp_kernels.hip resto_*, oracle/src/ipm.cpp restoration): phases per
    // solve (ARMOUR_RESTORATION=0: none), violation target inside the bounds, box barrier weight,
    // stall ratio
    int resto_max = 3;
    double resto_delta = 1e-6;
    double resto_mu = 1e-8;
    double resto_stall = 1e-4;
};

struct WorldState {
    double x[NF], xt[NF], dx[NF];
    double H[NF * NF];
    double mu, alpha, ap, ad, theta0, phi0, Dphi, theta_max, theta_min, kkt;
    double sw_dphi, sw_theta;          // pow(-Dphi, 2.3) (Dphi < 0) and pow(theta0, 1.1) of this
                                       // iteration: the switching condition's powers, once per iteration
    double wa_old_a[NF], wa_old_b[NF];   // sum (z_lo - z_hi) a  and  sum (dz_lo - dz_hi) a at x
    double filt_theta[MAX_FILTER], filt_phi[MAX_FILTER];
    int nfilt;
    int cur;           // eval slot holding the current point
    int status;        // 0 running, 1 converged, 2 max_iter, 3 line-search failure, 4 reach over capacity,
                       // 5 local infeasibility (the restoration phase stalled or failed), 6 in the
                       // restoration phase (WS_RESTO), 7 restarting after it (WS_RESTART)
    int searching;     // 1 while the line search of this iteration has not accepted
    int accepted_ok;   // last acceptance passed the filter (0: forced after max_ls trials)
    int ftype;
    int first_update, nfail, iter, nevals, ls;
    int spec_k;        // trial of the speculative round that ended the line search (-1: none)
    // adaptive barrier: free (oracle) mode, and the KKT errors the globalisation compares against
    // (free mode: the last <= 4; fixed mode: the one at the switch)
    int free_mode, nref;
    double kkt_ref[4];
    // restoration phase: phases entered, consecutive stalled iterations, a chosen step waiting
    // for its full evaluation (applied by the next resto_world_G), Phi of the previous iteration
    int nresto, rstall, rpend;
    double rphi;
};
constexpr int WS_RESTO = 6;
// A world whose restoration phase reached a point within every bound waits for its slacks and
// multipliers (ipm_rows_init) before it runs again: status 0 would let a phase run inside the
// interior-point loop hand it back to lists that still name it (planner.hip ipm_loop)
constexpr int WS_RESTART = 7;

struct NlpDev {
    int W, T, NJ, O, m, R, nblk, chunk;
    // the ARMTD comparison planner (ACMP/NLPclass.cu): no torque rows (nt = 0, else NF * T),
    // constant-acceleration extrema and cost with a per-world k_range [W][NF]
    int armtd, nt;
    const double* krange;
    int diag;               // diagnostics (ARMOUR_EVAL_SKIP): bit 0 skip slicing, bit 1 skip collision rows
    const RobotParams* rp;
    IpmOpts opt;
    // per-world inputs
    const double* q0;
    const double* qd0;
    const double* qdd0;
    const double* qdes;
    const double* obs;      // [W][O][12]
    // reach outputs
    ReachOut ro;
    // row bounds [W][R]
    double *L, *U;
    // evaluation slots: g [2][W][m], J [2][W][m][NF], f [2][W], grad [2][W][NF]. The collision
    // rows' Jacobian is held compactly: row (l, t, o) is J = n . dc/dx with n the winning plane's
    // signed normal, jn [2][W][T * NJ * O][3], and dc/dx the sliced link centre's derivatives,
    // jd [2][W][T][NJ][NF][3] (shared by the row's O obstacles); J keeps the other rows (and, after a
    // start-point / caller evaluation, mode 0, the collision rows dense too). row_va expands them.
    double* g;
    double* J;
    double* jn;
    double* jd;
    long njn, njd;          // per-slot sizes of jn, jd (W * T * NJ * Omax * 3, W * T * NJ * NF * 3)
    double* f;
    double* grad;
    double* link_c;         // [3][lcs]: [slot][W][T][NJ][3] sliced link centres of each eval slot's
                            // latest evaluation; region 2 the final iterate's (feasible_kernel)
    long lcs;
    // solver row state [W][R]
    double *slo, *shi, *zlo, *zhi, *dslo, *dshi;
    double* partial;        // [W][nblk][KA]
    double* partial2;       // [W][nblk][KA2]: pass D
    WorldState* ws;         // [W]
    int* flags;             // mapped host memory: [0] worlds running (round 0 of an iteration),
                            // [1] worlds still searching after the last line-search round
    // Active-world compaction: a solver launch covers only the worlds of list `wl` (blockIdx -> wl[b];
    // null: every world, blockIdx = world). ipm_world_C appends the worlds still running (round 0)
    // and still searching into wl_run / wl_search; the last block publishes the counts to flags.
    const int* wl;
    int* wl_run;
    int* wl_search;
    unsigned* cnt;          // device: [0] running, [1] searching, [2] block ticket
    int ls0;                // this ipm_world_C launch is round 0 of an iteration
    // rounds launched without a host synchronisation: grids sized by an upper bound, the list's
    // true length in device memory (lcount; null: the grid is exact); ipm_world_C stores the length
    // of the list it appends to into lcount_out
    const unsigned* lcount;
    unsigned* lcount_out;
    // sync-free tail iterations (few worlds running): ipm_world_C of round 0 also stores the running
    // count into lrun_out (device, read as the next iteration's lcount) and nrun_flag (mapped host
    // memory, read by the host one iteration later)
    unsigned* lrun_out;
    int* nrun_flag;
    int* bt_flag;           // mapped host: worlds of this iteration that searched past round 0
    // Speculative line-search round: the values (g, f) of the remaining K = max_ls - 1 trial points
    // of every world still searching after round 0, [list entry i][trial k] (eval_trials_kernel,
    // ipm_world_Cs); the trial that ends the search is then evaluated in full into the world's trial
    // slot (eval_kernel_t mode 5).
    int K;
    double *gs, *fs, *partial_s;
    // sync-free tail, one-round line search (planner.hip run_solver): pass B's world step runs in
    // ipm_world_Cs_all; the trial passes before it take the first step from pass B's partials
    // (pass_b_alpha) and every running world searches
    int b_in_cs;
    // restoration launches: the trial and full evaluations take the worlds in the restoration
    // phase (status WS_RESTO) instead of the searching ones
    int resto;
    int rflag;              // mapped host flag that resto_world_G's count goes to
    // restoration phases inside the interior-point loop (planner.hip ipm_loop): a world whose line
    // search fails is appended here (cnt[12]), and so is every world resto_world_Vs keeps in its
    // phase; resto_publish moves the list into the next phase iteration's (null: phases run after
    // the loop, run_resto). pend_flag: mapped host flag the round's last world kernel stores the
    // list's length into (the host's view of pending phase work)
    int* rl_app;
    int* pend_flag;
    // Certified plane cache (plane_cache_kernel). The 36 planes of a buffered
    // obstacle and their offsets d, delta do not depend on x; only A . c(x) does. For every
    // (world, t, link, obstacle) the cache holds the planes that can attain the maximum for some x in
    // the box |x_i| <= PC_XBOX, in the reference's scan order. The records of a (world, t) block are
    // n = its kept-plane count contiguous records at pcbase[w][t] of one pool: [5][n] (A0 A1 A2,
    // P = d + delta, N = -d + delta) from pc + 5 pcbase, the pair (l * O + o) of each from
    // pcp + pcbase; pcoff [W][T][NJ * O] = (first record << 8) | count; pcok [W][T] = 1 when the pool
    // held the block (the host sizes the pool from the count every build needed, ensure_plane_cache,
    // so a build that ran out is repeated on a larger pool and every block is cached).
    int pcache;             // cache enabled (ARMOUR_PLANE_CACHE=0 disables it)
    int pcready;            // built for the current reach sets and obstacles
    long pc_pool;           // records in the pool
    double* pc;             // [5 pc_pool]
    uint16_t* pcp;          // [pc_pool]
    unsigned* pcoff;
    unsigned char* pcok;
    unsigned long long* pcbase;  // [W][T] first pool record of each block
    unsigned* pcnext;            // pool records handed out by the current build (zeroed by jrs_kernel)
};
constexpr int EV_MAXK = 9;   // speculative trials per world (max_ls - 1)
constexpr int PC_K = 12;               // initial pool: records per pair per block (ARMOUR_PC_K; the survey workload keeps 5.3)
constexpr double PC_XBOX = 1.0 + 1e-6; // certified box of x (the solver keeps |x_i| <= 1)
constexpr double PC_RADF = 1.0001;     // >= PC_XBOX^21, the largest monomial degree sum (7 x 3)
constexpr double PC_MARGIN = 1e-9;     // >> the rounding of the bound and of A . c (~1e-15)

AD int world_of(const NlpDev& d, int b) { return d.wl ? d.wl[b] : b; }

AD long gidx(const NlpDev& d, int slot, int w, long r) { return ((long)slot * d.W + w) * d.m + r; }

}  // namespace armour
