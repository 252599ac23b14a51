/*
 * cmpc.h -- C ABI of the MI355X batched SCP centroidal-MPC solver (libcmpc.so).
 *
 * Drop-in boundary for the reference's per-SCP-iteration hot path
 * (ahmadgazar/centroidal-MPC, paths relative to the reference root):
 *
 *   reference interface                                    replaced by
 *   -----------------------------------------------------  --------------------------------
 *   Centroidal_model.__init__ contact / warm-start arrays   cmpc_upload
 *     src/centroidal_model.py:127-187
 *   Centroidal_model.compute_trajectory_data (JAX, fp32)    cmpc_linearize / cmpc_get_linearization
 *     src/centroidal_model.py:189-291
 *   sum_up_all_costs / stack_up_all_constraints (numpy)     cmpc_assemble / cmpc_export_qp
 *     src/scp_solver.py:10-48, src/cost.py, src/constraints.py
 *   solve_subproblem: osqp.OSQP().setup(P,q,A,l,u,...)      cmpc_qp_solve / cmpc_get_qp_solution
 *     .solve()   src/scp_solver.py:59-68
 *   compute_model_accuracy / trust-region test / accept     cmpc_scp_iterate (one full iteration)
 *     src/scp_solver.py:71-87,151-177
 *   solve_scp (while loop)                                  cmpc_solve_scp / cmpc_get_solution
 *     src/scp_solver.py:118-179
 *
 * Conventions: every function returns 0 on success and a negative code on error
 * (cmpc_last_error(h) gives the message; no C++ exception crosses the ABI).  Host
 * buffers are C-contiguous float64 (int8/int32 where stated) and owned by the caller;
 * the library copies in/out.  Device state is owned by the handle.  A handle is bound to
 * one device and is not thread-safe.  Calls that launch GPU work are asynchronous on the
 * handle's stream unless documented as synchronous; getters synchronize.  (Inside
 * cmpc_scp_iterate the covariance scan of a deterministic batch may run on a second,
 * low-priority stream of the handle; the handle's stream waits for it behind the QP, so
 * work ordered after the call on the handle's stream sees its results.)
 *
 * Layouts (B problems, horizon N, nc contacts, nu = 12 controls):
 *   logic (B,N,nc) int8 | pos (B,N,nc,3) | rot (B,N,nc,3,3) | Xbar (B,N+1,9) | Ubar (B,N,nu)
 *   f (B,N,9) | A (B,N,9,9) | Bu (B,N,9,nu) | C (B,N,9,3nc) | K (B,N,nu,9) | Sigma (B,N+1,9,9)
 */
#ifndef CMPC_H
#define CMPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CMPC_ROBOT_SOLO12 0
#define CMPC_ROBOT_TALOS 1
#define CMPC_PREC_F64 0
#define CMPC_PREC_F32 1

/* per-problem QP status codes (OSQP's values, src/scp_solver.py:65: only 'solved' counts):
 *   1  solved: merit = max(prim / eps_p, dual / eps_d, compl / eps_d) <= 1
 *   2  solved inaccurate: mu stalled for 3 iterations within 1e3 of the tolerance (the final
 *      merit is reported by cmpc_get_qp_info); a failure for the SCP loop, as in the reference
 *  -2  iteration cap
 *  -3  primal infeasible: Farkas certificate |E'nu + G'lambda| <= 1e-4 |(nu, lambda)|,
 *      b'nu + h'lambda <= -1e-4 |(nu, lambda)| on the diverging multipliers (OSQP's default
 *      eps_prim_inf); an infeasible QP whose multipliers have not diverged that far by the
 *      iteration cap ends with -2
 *  -4  dual infeasible: never returned; P > 0 on (x, u) and the only other variable t has cost
 *      +1 with t >= 0, so the subproblem is bounded below
 * -10  non-finite values */
#define CMPC_QP_SOLVED 1
#define CMPC_QP_SOLVED_INACCURATE 2
#define CMPC_QP_MAX_ITER (-2)
#define CMPC_QP_PRIMAL_INFEASIBLE (-3)
#define CMPC_QP_DUAL_INFEASIBLE (-4)
#define CMPC_QP_NONFINITE (-10)

#define CMPC_SCP_RUNNING 0
#define CMPC_SCP_CONVERGED 1      /* loop ended after an accepted iteration */
#define CMPC_SCP_MAX_ITER 2       /* loop ended on max_iterations / omega_max */
#define CMPC_SCP_QP_FAILED (-1)   /* reference returns False (src/scp_solver.py:146-148) */

/* SCP modes.  REFERENCE reproduces src/scp_solver.py:118-179 exactly, including quirk Q1: the
 * linearization point stays at the warm start (traj_tuple is never reassigned, :129-130), so the
 * loop ends after the first accepted iteration.  GUSTO implements the GuSTO scheme the
 * reference cites (:113-117): an accepted solution becomes the next linearization point and the
 * loop runs until convergence(traj, prev) (:51-56, spectral norms) < convergence_threshold.
 * The tracking cost and the initial / final state constraints stay on the warm start in both. */
#define CMPC_SCP_MODE_REFERENCE 0
#define CMPC_SCP_MODE_GUSTO 1

typedef struct cmpc_handle_s *cmpc_handle;

/* Parameters of one problem class: the conf_* attributes the hot path reads
 * (config/conf_solo12_trot.py:7-94).  Matrices are row-major; R and cov_w use the
 * top-left nu x nu / 3nc x 3nc corner. */
typedef struct {
    double mass, gravity, dt, mu, beta_u;
    double foot_range[4];   /* lxp, lxn, lyp, lyn (TALOS CoP box) */
    double Wx[9];           /* diag(state_cost_weights) */
    double Wu[12];          /* diag(control_cost_weights) */
    double Q[81];           /* LQR state weight */
    double R[144];          /* LQR control weight */
    double cov_w[144];      /* contact-position noise (3nc x 3nc) */
    double cov_eta[81];     /* additive noise (already scaled by dt) */
    int32_t stochastic;     /* STOCHASTIC_OCP: chance-constraint back-off in friction rows */
    int32_t tracking;       /* solo12 && !DYNAMICS_FIRST: state tracking cost */
    /* scp_params */
    double tr_radius0, omega0, omega_max, rho0, rho1, beta_succ, beta_fail, gamma_fail;
    double convergence_threshold;
    int32_t max_iterations;
} cmpc_params;

/* QP solver settings (defaults by cmpc_default_qp_settings) */
typedef struct {
    int32_t max_iter;       /* interior-point iterations (default 60) */
    double eps_abs;         /* absolute tolerance; 0 (default): fp64 1e-10, fp32 1e-6 (Solo12 fp64: after a
                             * rejected polish, complementarity against 10x the primal tolerance) */
    double eps_rel;         /* relative tolerance; 0 (default): as eps_abs */
    double step_fraction;   /* fraction-to-boundary in (0, 1); 0 (default) picks the robot's:
                             * Solo12 0.999, TALOS 0.995 (same-box measured) */
    /* Solo12 starting point: after the least-squares initialization step, s and lambda are
     * floored row by row at these values (default 0.1, 0.1); 0 selects CVXOPT's shift of every
     * row by 1 + the largest violation, which TALOS handles always use */
    double init_floor_s, init_floor_l;
    /* waves per problem of the QP workgroup: 1 (knots k, k + 64, ... on one wave), 2 (the
     * per-knot phases on two waves, one end of the Schur recurrence on each) or 4 (four chains of
     * the recurrence, N >= 16; shorter horizons get 2); 0 (default) picks 4 when every problem
     * gets a CU of its own and N >= 40, else 2 when two waves per problem still fit the device in
     * one round (2 B <= 4 x CUs) and N + 1 > 64, else 1 */
    int32_t waves_per_problem;
    /* solution polishing, as the reference's OSQP setup (polish=True, src/scp_solver.py:62): once
     * the iterate meets this tolerance (relative and absolute, like eps), the equality-constrained
     * QP on the guessed active set is solved with one more factorization; accepted when the
     * polished point meets eps with s, lambda >= 0 (then it is the exact minimizer), else the
     * interior-point iterations go on.  < 0 (default): the robot's (fp64 Solo12 1e-7 with split launches, 3e-8 without; TALOS off;
     * fp32 off); 0: off */
    double polish_eps;
} cmpc_qp_settings;

/* Per-phase device timings of the last cmpc_scp_iterate (milliseconds, HIP events). */
typedef struct {
    float linearize_ms, assemble_ms, qp_ms, accept_ms, total_ms;
} cmpc_timing;

/* Returns -2 for invalid sizes, -5 for TALOS in fp32 (unsupported: its QPs need fp64). */
int cmpc_create(cmpc_handle *out, int device, int robot, int N, int max_batch, int precision);
int cmpc_destroy(cmpc_handle h);
const char *cmpc_last_error(cmpc_handle h);
int cmpc_version(void);

int cmpc_default_qp_settings(int precision, cmpc_qp_settings *s);
int cmpc_set_qp_settings(cmpc_handle h, const cmpc_qp_settings *s);
int cmpc_set_params(cmpc_handle h, int n_classes, const cmpc_params *classes);

/* Copy B problems to the device and reset their SCP state
 * (weight = omega0, radius = trust_region_radius0, iteration 0). */
int cmpc_upload(cmpc_handle h, int B, const int32_t *class_id, const int8_t *logic, const double *pos,
                const double *rot, const double *Xbar, const double *Ubar);

/* Override the per-problem trust-region weight / radius (B entries each; NULL keeps the current
 * values).  Replaces the trust_region_updates={'weight','radius'} argument of
 * stack_up_all_constraints (reference src/scp_solver.py:28, src/constraints.py:260). */
int cmpc_set_trust_region(cmpc_handle h, const double *weight, const double *radius);

/* ---- on-device contact plans (replaces the host construction of src/contact_plan.py:40-48,
 * 112-264 and src/centroidal_model.py:127-187 for large batches) ---- */
#define CMPC_GAIT_TROT 0
#define CMPC_GAIT_PACE 1
#define CMPC_GAIT_BOUND 2
typedef struct {
    int32_t type;            /* CMPC_GAIT_* (conf gait['type']) */
    int32_t nb_steps;        /* gait['nbSteps'] */
    int32_t step_knots;      /* gait['stepKnots'] */
    int32_t support_knots;   /* gait['supportKnots'] */
    double step_length;      /* gait['stepLength'] */
} cmpc_gait;
/* Build the contact plans of B problems on the device: phases [support, step A, support, step B]
 * x nb_steps + support, swing feet inactive, stance feet at foot0 advanced by step_length per
 * completed step (bit-identical to the host construction), identity rotations.
 * foot0 (B, nc, 3) in the contact order FR, FL, HR, HL (solo12) / FR, FL (TALOS).  The plan must
 * cover N knots; every knot needs an active contact (TALOS supports only PACE). */
int cmpc_generate_contact_plans(cmpc_handle h, int B, const cmpc_gait *gaits, const double *foot0);
/* Upload warm starts for the B problems whose plans are on the device and reset their SCP state
 * (as cmpc_upload).  Ubar == NULL fills the reference's warm-start controls on the device
 * (src/centroidal_model.py:176-183). */
int cmpc_upload_states(cmpc_handle h, int B, const int32_t *class_id, const double *Xbar, const double *Ubar);
/* Read the device contact plans back: logic (B,N,nc) int8, pos (B,N,nc,3), rot (B,N,nc,9). */
int cmpc_get_contact_plans(cmpc_handle h, int8_t *logic, double *pos, double *rot);
/* Read the warm-start controls (B,N,nu) (e.g. after cmpc_upload_states with Ubar == NULL). */
int cmpc_get_warm_start(cmpc_handle h, double *Xbar, double *Ubar);

/* Select the SCP mode for subsequent iterations (default CMPC_SCP_MODE_REFERENCE). */
int cmpc_set_scp_mode(cmpc_handle h, int mode);

/* Nonlinear rollout of the uploaded problems' dynamics along (X (B,N+1,9), U (B,N,nu)) into
 * out (B,N+1,9); the contact data of the last knot is reused at k = N.  Replaces
 * Centroidal_model.integrate_dynamics_trajectory (reference src/centroidal_model.py:243-255). */
int cmpc_rollout(cmpc_handle h, const double *X, const double *U, double *out);

/* ---- hot-path phases (asynchronous) ---- */
int cmpc_linearize(cmpc_handle h);                 /* f, A, Bu, C, K, Sigma for all problems */
int cmpc_assemble(cmpc_handle h);                  /* structured QP from linearization + SCP state */
int cmpc_qp_solve(cmpc_handle h);                  /* batched interior-point QP */
int cmpc_accept(cmpc_handle h, int fixed_iters);   /* trust-region test, rho, accept/reject */
/* One full SCP iteration for every active problem: linearize -> assemble -> QP -> accept.
 * fixed_iters != 0: every problem iterates (benchmark fixed-K mode); 0: finished problems
 * are skipped (reference semantics). */
int cmpc_scp_iterate(cmpc_handle h, int fixed_iters);
/* Run the reference's while loop to completion (synchronous). */
int cmpc_solve_scp(cmpc_handle h, int fixed_iters, int *n_iterations_out);
int cmpc_synchronize(cmpc_handle h);

/* ---- getters (synchronous; NULL pointers are skipped) ---- */
/* The last linearization (knot-major).  In reference mode the SCP loop does not store the dense
 * A, Bu, C (the QP reads the stage record, the accept step the closed form); this getter and
 * cmpc_export_qp first recompute them with one more k_lin_knots pass, which rewrites identical
 * values because the linearization point never moves there (quirk Q1). */
int cmpc_get_linearization(cmpc_handle h, double *f, double *A, double *Bu, double *C, double *K,
                           double *Sigma);
int cmpc_qp_sizes(cmpc_handle h, int32_t *n, int32_t *m, int32_t *nnzP, int32_t *nnzA);
/* CSC export of problem b's QP in the reference's exact row order (parity/debug only). */
int cmpc_export_qp(cmpc_handle h, int b, double *P_x, int32_t *P_i, int32_t *P_p, double *q, double *A_x,
                   int32_t *A_i, int32_t *A_p, double *l, double *u);
/* z in the reference's variable layout (B, n) and y in its row layout (B, m). */
/* Problem b's QP given in the reference's CSC layout (P, q, A, l, u as src/scp_solver.py:59-68
 * hands them to OSQP; n variables, m rows, int32 indices) decoded into the device's structured
 * form, for a following cmpc_qp_solve.  The QP must have the stage structure: the handle's sizes,
 * a diagonal cost with one Wx / Wu for all knots, centroidal dynamics blocks, the reference's
 * friction, CoP, trust-region and slack rows (csrc/load_qp.cpp lists every check).  Otherwise -2
 * and a message naming the offending row.  Installs a parameter class with the decoded weights
 * and dt / mass for problem b.  Replaces the OSQP call of solve_subproblem for QPs not built by
 * cmpc_assemble. */
int cmpc_load_qp(cmpc_handle h, int b, int n, int m, const double *P_x, const int32_t *P_i, const int32_t *P_p,
                 const double *q, const double *A_x, const int32_t *A_i, const int32_t *A_p, const double *l,
                 const double *u);
int cmpc_get_qp_solution(cmpc_handle h, double *z, double *y, int32_t *status, int32_t *iters);
/* Per-problem exit data of the last QP solve: final merit (<= 1 when solved) and the number of
 * iterative-refinement steps taken (B entries each; NULL skips). */
int cmpc_get_qp_info(cmpc_handle h, double *merit, int32_t *n_refine);
/* Per problem (B entries each; NULL skips): tail_steps, the Newton steps of the last QP solve that
 * ran on the whole workgroup after the problem was handed over (grouped kernel k_qp_group: the last
 * problem of a group, once the others have stopped; 0 for problems solved on their own waves only);
 * polish, the solution polishing of that solve (1 accepted: the returned solution is the polished
 * one; -1 tried and rejected; 0 not tried). */
int cmpc_get_qp_exit(cmpc_handle h, int32_t *tail_steps, int32_t *polish);
/* The accepted iterate of each problem (X, U) with that iteration's LQR gains and covariances.
 * Reference mode serves K and Sigma from the live linearization arrays, which every iteration
 * recomputes bit-identically (quirk Q1; the reference keeps references to that iteration's
 * arrays).  GuSTO mode and new contact plans copy them per accept. */
int cmpc_get_solution(cmpc_handle h, double *X, double *U, double *K, double *Sigma, int32_t *n_accepted,
                      int32_t *iterations, int32_t *scp_status, double *weight, double *radius);
/* Page-lock a caller's host range (hipHostRegister) so getters write it by DMA at full link rate
 * (cmpc_get_solution: X, U, K, Sigma of a 1024-problem N=100 batch are 172 MB); unregister
 * before freeing it.  Optional: pageable buffers work, through the runtime's staging copies. */
int cmpc_host_register(cmpc_handle h, void *ptr, size_t bytes);
/* Reference mode: stream the accepted K (B,N,nu,9) and Sigma (B,N+1,9,9) of the next solve into
 * these page-locked host buffers (NULL skips) while it runs.  The linearization point never moves
 * (quirk Q1), so K is final after the first iteration's linearization and Sigma after its
 * covariance scan: the copies run on a copy stream's DMA behind the QP.  A following
 * cmpc_get_solution given the same pointers only waits for them.  Armed until the next upload
 * (or a mode / parameter / plan change); only problems with n_accepted > 0 have accepted K / Sigma
 * (the others get the linearization's, as cmpc_get_solution returns them). */
int cmpc_prefetch_ks(cmpc_handle h, double *K, double *Sigma);
int cmpc_host_unregister(cmpc_handle h, void *ptr);
/* The last iteration of each problem (B entries each; NULL skips). */
int cmpc_get_iteration_log(cmpc_handle h, double *tr_norm, double *rho, int32_t *qp_status,
                           int32_t *qp_iters, int32_t *decision);

/* One SCP iteration of one problem: what the reference prints per iteration
 * (src/scp_solver.py:135-178, banners and decisions) and the trust region it ran with. */
#define CMPC_DECISION_ACCEPT 1
#define CMPC_DECISION_REJECT_RHO 2   /* inside the trust region, rho > rho1: radius *= beta_fail */
#define CMPC_DECISION_REJECT_TR 3    /* outside the trust region: weight *= gamma_fail */
#define CMPC_DECISION_QP_FAILED (-1) /* the reference returns False */
typedef struct {
    double weight, radius;   /* trust-region weight / radius of this iteration's QP */
    double tr_norm;          /* ||X_sol - X_lin||_2 (spectral norm, quirk Q6) */
    double rho;              /* model-accuracy ratio; NaN where the reference does not evaluate it */
    int32_t iteration, qp_status, qp_iters, decision;
} cmpc_iter_record;
/* Every SCP iteration of every problem since its upload, in order: records (B, cap), iteration i
 * of problem b at records[b * cap + i]; n_records (B) = iterations recorded.  The device keeps
 * max(max_iterations) records per problem (the larger of the parameter classes'); iterations
 * beyond it (fixed-K runs past max_iterations) are not recorded.  cap may be any size >= 1. */
int cmpc_get_iteration_history(cmpc_handle h, int cap, cmpc_iter_record *records, int32_t *n_records);
/* Accepted iterate j (0-based, in acceptance order) of every problem: X (B,N+1,9), U (B,N,nu),
 * K (B,N,nu,9), Sigma (B,N+1,9,9) (NULL skips); zeros for problems with fewer than j + 1 accepted
 * iterates.  The reference appends every accepted iterate to its lists (src/scp_solver.py:162-167);
 * the device keeps up to max(max_iterations) per problem.  Reference mode: K and Sigma are those of
 * the (fixed) linearization point, bit-identical for every iterate (quirk Q1). */
int cmpc_get_accepted(cmpc_handle h, int j, double *X, double *U, double *K, double *Sigma);
/* Current linearization point (B,N+1,9) / (B,N,nu) and the last convergence measure
 * ||dU||/||U|| + ||dX||/||X|| of each problem (0 in reference mode, quirk Q1). */
int cmpc_get_linearization_point(cmpc_handle h, double *X, double *U, double *convergence);
/* Linear interpolation of the accepted solution with n_inner sub-steps per interval, on the
 * device: X_out (B,9,N*n_inner), U_out (B,nu,(N-1)*n_inner) in the reference's layout (column
 * i*n_inner + j = v_i + j (v_{i+1} - v_i) / n_inner).  Replaces interpolate_SCP_solution
 * (reference src/scp_solver.py:95-111, N_inner = 10). */
int cmpc_interpolate(cmpc_handle h, int n_inner, double *X_out, double *U_out);
int cmpc_get_timing(cmpc_handle h, cmpc_timing *t);
/* Accumulate per-phase HIP-event timings of every cmpc_scp_iterate between begin and end
 * (no host synchronization inside the region; end synchronizes and sums). */
int cmpc_timing_begin(cmpc_handle h);
int cmpc_timing_end(cmpc_handle h, cmpc_timing *t, int *n_iterations);
/* Sum over problems of the interior-point iterations of the last QP solve. */
int cmpc_get_qp_iterations_total(cmpc_handle h, int64_t *total);
/* Diagnostic builds (libcmpc_diag.so, -DCMPC_STAMPS): per-problem shader-cycle counters of the
 * QP kernel's phases, (B, 16); zeros in the production library. */
int cmpc_debug_stamps(cmpc_handle h, uint64_t *out);
/* The QP kernel the next cmpc_qp_solve / cmpc_scp_iterate launches for the uploaded batch, e.g.
 * "k_qp_group<4>" (four problems per four-wave workgroup) or "k_qp_ipm<2>" (one problem per
 * two-wave workgroup); written NUL-terminated into buf (at most n bytes).  For measurement labels. */
int cmpc_get_qp_kernel(cmpc_handle h, char *buf, int n);

/* ---- multi-GPU batch split over RCCL (one process per GPU, one handle per process) ----
 * The problems are independent: nothing crosses GPUs inside the SCP loop.  Rank r owns a
 * contiguous slice of the global batch; RCCL carries the shared parameters, the max-reduction of
 * the timed region and the gather of the results.  The reference is single-process
 * (src/scp_solver.py:118-179); this is the north star's batch split. */
#define CMPC_COMM_ID_BYTES 128
/* ncclGetUniqueId: called by rank 0, handed to the other ranks out of band (cmpc/shard.py). */
int cmpc_comm_get_unique_id(uint8_t *id_out);
/* ncclCommInitRank on the handle's device (collective over the nranks processes). */
int cmpc_comm_init(cmpc_handle h, int nranks, int rank, const uint8_t *id);
int cmpc_comm_destroy(cmpc_handle h);
/* Broadcast the root's parameter classes (classes holds n_classes entries of capacity; root's
 * count wins) and install them with cmpc_set_params on every rank. */
int cmpc_comm_bcast_params(cmpc_handle h, int root, int n_classes, cmpc_params *classes);
/* In-place elementwise max over ranks of n doubles (also the barrier of the timed region). */
int cmpc_comm_allreduce_max(cmpc_handle h, double *v, int n);
/* Gather every rank's accepted solutions and per-problem statuses to root, rank-major (= the
 * global problem order of contiguous slices).  Ranks may hold different batch sizes B_r (the
 * last slices of ceil(B / G) are short); root's buffers hold the global batch sum_r B_r:
 * X (.., N+1, 9), U (.., N, nu), scp_status, iterations, qp_status (NULL skips).  Non-root ranks
 * may pass NULL. */
int cmpc_comm_gather_solution(cmpc_handle h, int root, double *X, double *U, int32_t *scp_status,
                              int32_t *iterations, int32_t *qp_status);

#ifdef __cplusplus
}
#endif
#endif /* CMPC_H */
