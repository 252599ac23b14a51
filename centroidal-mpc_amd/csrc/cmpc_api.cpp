// C ABI of libcmpc.so (declared in include/cmpc.h): handle lifecycle, device memory, kernel
// launches and the host-side CSC export used for parity tests.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <tuple>
#include <vector>

#include "cmpc.h"
#include "common.hpp"
#include "handle.hpp"

namespace cmpc {
template <typename T, int R> __global__ void k_linearize(DevBuf<T>, int);
template <typename T, int R> __global__ void k_lin_knots(DevBuf<T>, int, int);
template <typename T, int R> __global__ void k_cov_scan(DevBuf<T>, int);
template <typename T, int R, bool FULL> __global__ void k_assemble(DevBuf<T>, int);
template <typename T, int R, int NTT, int MODE> __global__ void k_qp_ipm(DevBuf<T>, int, int, T, T, T, T, T, T, int *);
template <typename T> __global__ void k_qp_split(DevBuf<T>, int, int, int, int *);
size_t ipm_state_bytes(int prec_bytes);
template <typename T, int R, int P> __global__ void k_qp_group(DevBuf<T>, const int *, int, int, int, T, T, T, T, T, T);
template <typename T> __global__ void k_qp_order(DevBuf<T>, int, int, int *);
size_t ipm_group_lds_bytes(int N, int prec_bytes, int P);
int ipm_pair_max_batch();
template <typename T> __global__ void k_interpolate(DevBuf<T>, int, int, T *, T *);
template <typename T, int R> __global__ void k_contact_plan(DevBuf<T>, const cmpc_gait *, const T *, uint8_t *, T *, T *);
template <typename T, int R> __global__ void k_default_controls(DevBuf<T>, T *);
size_t ipm_lds_bytes(int N, int prec_bytes, int nt);
template <typename T, int R> __global__ void k_accept(DevBuf<T>, int);
template <typename T> __global__ void k_keep_accepted(DevBuf<T>);
template <typename T> __global__ void k_knot_major(const T *, size_t, size_t, size_t, int, double *);
template <typename T, int R> __global__ void k_rollout(DevBuf<T>, const T *, const T *, T *);
__global__ void k_widen(const float *, size_t, double *);
size_t ipm_workspace_elems(int N, int robot);
}  // namespace cmpc

using namespace cmpc;
using namespace cmpc_host;

namespace {

// Inverse standard normal CDF (Acklam's rational approximation refined by Halley steps on
// erfc), to reproduce scipy.stats.norm.ppf for xi (reference src/constraints.py:157).
double norm_ppf(double p) {
    static const double a[] = {-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
                               1.383577518672690e+02, -3.066479806614716e+01, 2.506628277459239e+00};
    static const double b[] = {-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
                               6.680131188771972e+01, -1.328068155288572e+01};
    static const double c[] = {-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
                               -2.549732539343734e+00, 4.374664141464968e+00, 2.938163982698783e+00};
    static const double d[] = {7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
                               3.754408661907416e+00};
    double x;
    const double pl = 0.02425;
    if (p < pl) {
        double q = std::sqrt(-2 * std::log(p));
        x = (((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
            ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
    } else if (p <= 1 - pl) {
        double q = p - 0.5, r = q * q;
        x = (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q /
            (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1);
    } else {
        double q = std::sqrt(-2 * std::log(1 - p));
        x = -(((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
            ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
    }
    for (int i = 0; i < 3; ++i) {
        double e = 0.5 * std::erfc(-x / std::sqrt(2.0)) - p;
        double u = e * std::sqrt(2 * M_PI) * std::exp(x * x / 2);
        x = x - u / (1 + x * u / 2);
    }
    return x;
}

}  // namespace

namespace {

template <typename T> DevParams<T> conv_params(const cmpc_params &p, int nw) {
    DevParams<T> d{};
    d.mass = T(p.mass); d.gravity = T(p.gravity); d.dt = T(p.dt); d.mu = T(p.mu);
    d.xi = T(norm_ppf(1.0 - (p.beta_u / 5.0 * 3.0)));
    for (int i = 0; i < 4; ++i) d.foot_range[i] = T(p.foot_range[i]);
    for (int i = 0; i < 9; ++i) d.Wx[i] = T(p.Wx[i]);
    for (int i = 0; i < 12; ++i) d.Wu[i] = T(p.Wu[i]);
    for (int i = 0; i < 81; ++i) { d.Q[i] = T(p.Q[i]); d.cov_eta[i] = T(p.cov_eta[i]); }
    for (int i = 0; i < 144; ++i) d.R[i] = T(p.R[i]);
    // cov_w arrives as a 12x12 row-major buffer whose top-left nw x nw corner is used
    for (int i = 0; i < nw; ++i)
        for (int j = 0; j < nw; ++j) d.cov_w[i * nw + j] = T(p.cov_w[i * 12 + j]);
    d.stochastic = p.stochastic; d.tracking = p.tracking;
    d.tr_radius0 = p.tr_radius0; d.omega0 = p.omega0; d.omega_max = p.omega_max; d.rho0 = p.rho0;
    d.rho1 = p.rho1; d.beta_succ = p.beta_succ; d.beta_fail = p.beta_fail; d.gamma_fail = p.gamma_fail;
    d.conv_thr = p.convergence_threshold; d.max_iterations = p.max_iterations;
    return d;
}

// QP waves per problem: the setting, or (0) two when the batch at two waves per problem still runs
// in one round on the device (one wave per SIMD at ~500 registers per lane) and the horizon needs
// more than one pass of 64 knots
// Four waves (schur_pt.hpp: the Schur recurrence as four chains) when every problem still gets a
// CU of its own and the horizon gives each chain a few blocks.
// The four chains need N >= 16 (pt_seps gives every chain a few blocks), so a request for four waves
// on a shorter horizon gets two, from the setting and from the diagnostic override alike.
int qp_waves(cmpc_handle h) {
    auto fit = [&](int w) { return w == 4 && h->N < 16 ? 2 : w; };
    if (const char *e = std::getenv("CMPC_QP_WAVES")) {   // diagnostic override (timing experiments)
        const int w = std::atoi(e);
        if (w == 1 || w == 2 || w == 4) return fit(w);
    }
    if (h->qs.waves_per_problem > 0) return fit(h->qs.waves_per_problem);
    if (h->N >= 40 && (long)h->B <= (long)h->n_cu) return 4;
    return (h->N + 1 > 64 && 2L * h->B <= 4L * h->n_cu) ? 2 : 1;
}

// Grouped QP workgroups (k_qp_group: P problems per P-wave workgroup, one per wave, all P waves on
// the last one once the others have stopped) in place of one wave per problem, for fp64 batches
// that fit k_qp_order: four problems per workgroup where the four-chain recurrence applies (N >= 40)
// and four regions fit a CU's LDS, else two.  Same-box A/B (profiles/r03c_pair_ab.log): pairs took
// the metric config's QP from 2.93 to 2.75 ms; BASELINE C3 (fp32, two Newton steps, no tail to
// balance) 0.744 -> 0.752 ms, so fp32 keeps one wave per problem.  Two two-wave problems per
// four-wave workgroup (round 3, k_qp_group<.., 2, 2>) were a measured wash on the 512-problem
// shard and -4% on C4 (profiles/r03g_group2w_ab.log): gfx950 has no half-workgroup barrier, and the
// LDS spin barrier that stood in for it cost what the tail gained; removed in round 4.
// Diagnostics: CMPC_QP_PAIR=0 turns grouping off, =2 keeps the groups but never shares a problem;
// CMPC_QP_GROUP=2|4 forces the group size.  Returns P, or 0 for one wave per problem.
int qp_group(cmpc_handle h) {
    const int w = qp_waves(h);
    if (w != 1 || h->B < 2 || h->B > ipm_pair_max_batch() || h->prec != CMPC_PREC_F64) return 0;
    // Off by default since round 4: with this round's kernel changes the fused grouped kernel
    // (one-wave loop and the all-wave tail in one code object, ~600 SGPR and 200-480 VGPR spills)
    // stopped on memory-aperture faults on the GPU -- k_qp_group<double, 1, 2> shared and
    // k_qp_group<double, 0, 4> even unshared, i.e. running only the one-wave loop that k_qp_ipm<.., 64>
    // runs without fault on the same batch ("Grouped workgroups").  CMPC_QP_PAIR=1 (shared)
    // or 2 (unshared) selects it for diagnostics.
    {
        const char *e = std::getenv("CMPC_QP_PAIR");
        if (!e || (e[0] != '1' && e[0] != '2')) return 0;
    }
    const size_t cap = 160 * 1024 - 1024;
    const int esz = (int)h->esz();
    int P = h->N >= 40 && ipm_group_lds_bytes(h->N, esz, 4) <= cap ? 4 : 2;
    if (const char *e = std::getenv("CMPC_QP_GROUP")) {
        if (e[0] == '2') P = 2;
        if (e[0] == '4' && h->N >= 40) P = 4;
    }
    if (ipm_group_lds_bytes(h->N, esz, P) > cap) P = 2;
    // TALOS pairs (k_qp_group<double, 1, 2> with hand-over: TALOS batches of N < 40, no BASELINE
    // configuration) stopped on a memory-aperture fault in round 4 (N = 40, 9 problems) that the
    // instrumented build (per-phase progress trace) did not reproduce; they run one wave per problem
    // until it is found ("Grouped workgroups").  Solo12 pairs and all quads are unaffected.
    if (P == 2 && h->robot == CMPC_ROBOT_TALOS) return 0;
    return ipm_group_lds_bytes(h->N, esz, P) <= cap ? P : 0;
}

// CMPC_QP_PAIR=2: grouped workgroups whose waves never share a problem (diagnostic: the cost of the
// grouping itself)
int qp_pair_share() {
    const char *e = std::getenv("CMPC_QP_PAIR");
    return e && e[0] == '2' ? 0 : 1;
}

// Split QP launches (k_qp_ipm MODE 1 head + MODE 2 tail): for fp64 batches of one wave per problem
// that fill the device (B > CUs, so two waves per problem do not fit one round), the slowest
// problems' last Newton steps run on four waves (two below N = 40) in a second launch, one problem
// per CU, once every other problem has finished (k_qp_split picks the yield iteration from the
// previous launch's Newton counts).  Round 4's replacement for the grouped kernel (qp_group).
// CMPC_QP_SPLIT=0 turns it off.  Returns the tail launch's waves per problem, or 0.
int qp_split(cmpc_handle h) {
    const int w = qp_waves(h);
    if (h->prec != CMPC_PREC_F64 || w > 2 || h->B <= h->n_cu || qp_group(h)) return 0;
    if (const char *e = std::getenv("CMPC_QP_SPLIT"))
        if (e[0] == '0') return 0;
    if (w == 2 && h->N < 40) return 0;   // (a two-wave head needs the four-wave tail)
    if (const char *e = std::getenv("CMPC_QP_TAIL_WAVES"))   // diagnostic override (A/B runs)
        if (e[0] == '2' && w == 1) return 2;
    return h->N >= 40 ? 4 : 2;
}

// Tail capacity of a split launch: at most one problem per CU in the tail (k_qp_split).
// CMPC_QP_SPLIT_CAP overrides (A/B runs: profiles/r04e_tail_shape_ab.log).
int qp_split_cap(cmpc_handle h, int tw) {
    (void)tw;
    if (const char *e = std::getenv("CMPC_QP_SPLIT_CAP")) {
        const int c = std::atoi(e);
        if (c > 0) return c;
    }
    return h->n_cu;
}

// Yield iteration of a split launch on a never-solved batch (the reference's use: every solve_scp
// call is a new problem, src/scp_solver.py:118-179), where there are no Newton counts to pick it
// from: the robot's prior, above its typical counts so that few problems exceed it (Solo12 trot
// N=100: 4-8 steps, 6 leaves ~10% for the tail; TALOS N=200: 12-17, 15).  CMPC_QP_SPLIT_FRESH=0
// turns it off (the first launch is then unsplit).
int qp_split_prior(cmpc_handle h) {
    if (const char *e = std::getenv("CMPC_QP_SPLIT_FRESH"))
        if (e[0] == '0') return 0;
    return h->robot == 1 ? 15 : 6;
}

// QP step fraction: the setting, or (0) the robot's. Same-box A/B, bench lines A B A B:
// Solo12 trot N=100 x 1024 0.995 -> 0.999 316.8k -> 319.5k SCP it/s, 4.81 -> 4.67 Newton steps
// (profiles/r02_eta999_ab.jsonl); TALOS N=200 x 512 0.999 -> 0.995 56.2k -> 59.4k
// (profiles/r02_talos_eta_ab.jsonl).
double qp_step_fraction(cmpc_handle h) {
    if (h->qs.step_fraction > 0) return h->qs.step_fraction;
    return h->robot == 1 ? 0.995 : 0.999;
}

// Stopping tolerances: the settings, or (0) the default: fp64 1e-10, fp32 1e-6 (qp_ipm.hip
// COMP_PRIMAL_SCALE for Solo12's complementarity after a rejected polish).
double qp_eps_default(cmpc_handle h) {
    return h->prec != CMPC_PREC_F64 ? 1e-6 : 1e-10;
}
double qp_eps_env() {   // CMPC_QP_EPS: diagnostic override of both tolerances (A/B runs)
    const char *e = std::getenv("CMPC_QP_EPS");
    return e ? std::atof(e) : 0.0;
}
double qp_eps_abs(cmpc_handle h) {
    if (qp_eps_env() > 0) return qp_eps_env();
    return h->qs.eps_abs > 0 ? h->qs.eps_abs : qp_eps_default(h);
}
double qp_eps_rel(cmpc_handle h) {
    if (qp_eps_env() > 0) return qp_eps_env();
    return h->qs.eps_rel > 0 ? h->qs.eps_rel : qp_eps_default(h);
}

// Polishing tolerance: the setting, or (< 0) the robot's.  Same-box sweeps (profiles/r04a_polish_sweep.log):
// Solo12 trot N=100 x 1024 polishes at 1e-7 on 820 of 1024 problems (1 wrong guess), 4.67 Newton
// steps against 5.48 without, 281.8k SCP it/s against 276.8k (1e-8: 273.0k).  TALOS (BASELINE C4
// from its fourth SCP iteration) guesses wrong on 384 of 512 at 1e-7 and 99-166 at 1e-8 / 1e-9, where
// every rejected polish costs a factorization: 51.7k against 54.3k without, so TALOS does not polish.
// fp32 (C3) is not polished.  Round-4 sweep with the final stopping rule (profiles/r04d_polish_sweep2.log):
// split launches (the metric config) 1e-7 324k, 3e-8 312k, 1e-8 300k; four waves per problem without a
// split (C2, the 4- and 8-GPU shards), where the launch lasts as long as its slowest problem and a
// rejected first guess lands on it, 1e-7 166k (3 rejected), 3e-8 262k (none), 1e-8 229k.
double qp_polish_eps(cmpc_handle h) {
    if (h->prec != CMPC_PREC_F64) return 0.0;
    if (const char *e = std::getenv("CMPC_QP_POLISH_EPS"))   // diagnostic override (A/B runs)
        return std::atof(e);
    if (h->qs.polish_eps >= 0) return h->qs.polish_eps;
    if (h->robot == 1) return 0.0;
    return qp_split(h) ? 1e-7 : 3e-8;
}

// Covariance scan placement.  Sigma feeds only the chance-constraint back-off of stochastic
// problems (k_assemble) and the outputs, so inside cmpc_scp_iterate the scan of a deterministic
// batch leaves the critical path:
// - when the QP leaves SIMDs free (scan_beside_qp), k_cov_scan runs on the low-priority side
//   stream, started when the assembly ends, and the main stream waits for it right behind the QP;
// - when the QP fills the device with one wave per SIMD, a separate scan kernel's waves delay the
//   QP's dispatch, so the QP kernel runs the scans itself: each workgroup whose problem has
//   converged takes scan jobs from a counter (k_qp_ipm, d.scan_ctr).
// Either way k_accept, k_keep_accepted, the getters and the next linearization (which rewrites
// Acl / Qw) are ordered after the scans.
template <typename T, int R> void launch_scan(cmpc_handle h, hipStream_t s, int only_active) {
    hipLaunchKernelGGL((k_cov_scan<T, R>), dim3(h->B), dim3(64), 0, s, h->buf<T>(), only_active);
}

// Only where the QP leaves room: two-wave QP workgroups, or fewer QP waves than SIMDs.  With one
// wave per SIMD over the whole device (the metric config, 1024 problems) the scan's waves delayed
// the QP's dispatch: 318.7k -> 258.8k SCP it/s, while two-wave batches gained (C2 161.2k -> 165.5k,
// C4 59.5k -> 60.5k; same-box A/B, profiles/r02_scan_overlap_ab.txt).
bool scan_beside_qp(cmpc_handle h) {
    const int w = qp_waves(h);
    return w >= 2 || (long)h->B * w < 4L * h->n_cu;
}

bool any_stochastic(cmpc_handle h) {
    for (auto &p : h->hparams)
        if (p.stochastic) return true;
    return false;
}

// settle a deferred or running side-stream scan (before anything that is not assembly or QP)
template <typename T, int R> void settle_scan(cmpc_handle h, int only_active) {
    if (h->scan_deferred) {
        launch_scan<T, R>(h, h->stream, only_active);
        h->scan_deferred = false;
    }
    if (h->scan_pending) {
        HIPCHK(hipStreamWaitEvent(h->stream, h->ev_scan, 0));
        h->scan_pending = false;
    }
}

template <typename T, int R> void launch_phase(cmpc_handle h, int phase, int only_active, bool overlap = false) {
    DevBuf<T> d = h->buf<T>();
    const int B = h->B;
    if (B == 0) return;
    if (phase == 0 || phase == 3) settle_scan<T, R>(h, only_active);
    switch (phase) {
    case 0:
        // one knot per lane (diagonal R; also writes the linearization part of the stage records),
        // or one workgroup per problem (general R); then the per-problem covariance scan
        // Reference mode skips the dense A, Bu, C (nothing in the SCP loop reads them: the QP uses
        // the stage record, k_accept the closed form); GuSTO mode keeps them, since its
        // linearization point moves and the getters could not recompute them later.
        if (h->lin_lane) {
            const long n = (long)B * h->N;
            const int dense = h->scp_mode == CMPC_SCP_MODE_GUSTO ? 1 : 0;
            hipLaunchKernelGGL((k_lin_knots<T, R>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, d,
                               only_active, dense);
            h->lin_dense = dense != 0;
        } else {
            hipLaunchKernelGGL((k_linearize<T, R>), dim3(B), dim3(256), 0, h->stream, d, only_active);
            h->lin_dense = true;
        }
        h->lin_lane_done = h->lin_lane;
        if (overlap && !any_stochastic(h)) {
            h->scan_deferred = true;   // beside the QP (case 1) or inside it (case 2)
            h->scan_oa = only_active;
        }
        else
            launch_scan<T, R>(h, h->stream, only_active);
        break;
    case 1: {
        const long n = (long)B * (h->N + 1);
        if (h->lin_lane_done)
            hipLaunchKernelGGL((k_assemble<T, R, false>), dim3((unsigned)((n + 127) / 128)), dim3(128), 0, h->stream, d,
                               only_active);
        else
            hipLaunchKernelGGL((k_assemble<T, R, true>), dim3((unsigned)((n + 127) / 128)), dim3(128), 0, h->stream, d,
                               only_active);
        if (h->scan_deferred && scan_beside_qp(h)) {
            HIPCHK(hipEventRecord(h->ev_asm, h->stream));
            HIPCHK(hipStreamWaitEvent(h->side, h->ev_asm, 0));
            launch_scan<T, R>(h, h->side, only_active);
            HIPCHK(hipEventRecord(h->ev_scan, h->side));
            h->scan_deferred = false;
            h->scan_pending = true;
        }
        break;
    }
    case 2: {
        // one workgroup per problem (one or two waves, cmpc_qp_settings::waves_per_problem); the
        // (N+2) x 9 Schur vector and the sweep rings in LDS, the Schur blocks in the workspace
        const int nt = 64 * qp_waves(h);
        const T eta = T(qp_step_fraction(h));
        if (const int P = qp_group(h)) {
            const size_t lds = ipm_group_lds_bytes(h->N, (int)sizeof(T), P);
            const void *fn = P == 4 ? reinterpret_cast<const void *>(&k_qp_group<T, R, 4>)
                                    : reinterpret_cast<const void *>(&k_qp_group<T, R, 2>);
            HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            if (h->scan_deferred) {   // the scans run in the QP's waves
                HIPCHK(hipMemsetAsync(h->scan_ctr, 0, sizeof(unsigned), h->stream));
                d.scan_ctr = (unsigned *)h->scan_ctr;
                h->scan_deferred = false;
            }
            hipLaunchKernelGGL((k_qp_order<T>), dim3(1), dim3(1024), 0, h->stream, d, only_active, P, (int *)h->qp_order);
            const unsigned ng = (unsigned)((B + P - 1) / P);
            if (P == 4)
                hipLaunchKernelGGL((k_qp_group<T, R, 4>), dim3(ng), dim3(256), lds, h->stream, d, (const int *)h->qp_order,
                                   only_active, qp_pair_share(), h->qs.max_iter, T(qp_eps_abs(h)), T(qp_eps_rel(h)), eta,
                                   T(h->qs.init_floor_s), T(h->qs.init_floor_l), T(qp_polish_eps(h)));
            else
                hipLaunchKernelGGL((k_qp_group<T, R, 2>), dim3(ng), dim3(128), lds, h->stream, d, (const int *)h->qp_order,
                                   only_active, qp_pair_share(), h->qs.max_iter, T(qp_eps_abs(h)), T(qp_eps_rel(h)), eta,
                                   T(h->qs.init_floor_s), T(h->qs.init_floor_l), T(qp_polish_eps(h)));
            if (h->scan_pending) {
                HIPCHK(hipStreamWaitEvent(h->stream, h->ev_scan, 0));
                h->scan_pending = false;
            }
            break;
        }
        const size_t lds = ipm_lds_bytes(h->N, (int)sizeof(T), nt);
        const int tw = qp_split(h);
        const void *fn = nt == 256   ? reinterpret_cast<const void *>(&k_qp_ipm<T, R, 256, 0>)
                         : nt == 128 ? reinterpret_cast<const void *>(&k_qp_ipm<T, R, 128, 0>)
                                     : reinterpret_cast<const void *>(&k_qp_ipm<T, R, 64, 0>);
        HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        if (h->scan_deferred) {   // the scans run in the QP's workgroups (one-wave kernel only)
            need(nt == 64, "internal: QP scan jobs need the one-wave kernel");
            HIPCHK(hipMemsetAsync(h->scan_ctr, 0, sizeof(unsigned), h->stream));
            d.scan_ctr = (unsigned *)h->scan_ctr;
            h->scan_deferred = false;
        }
        const T ea = T(qp_eps_abs(h)), er = T(qp_eps_rel(h)), fs = T(h->qs.init_floor_s), fl = T(h->qs.init_floor_l),
                pe = T(qp_polish_eps(h));
        if constexpr (sizeof(T) == 8) {
            if (tw) {   // split launches: head (one wave per problem, the slowest leave), tail
                int *sp = (int *)h->qp_split;
                hipLaunchKernelGGL((k_qp_split<T>), dim3(1), dim3(1024), 0, h->stream, d, only_active,
                                   qp_split_cap(h, tw), qp_split_prior(h), sp);
                if (nt == 128) {   // two-wave head (BASELINE C4: TALOS N=200 x 512)
                    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_qp_ipm<T, R, 128, 1>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                    hipLaunchKernelGGL((k_qp_ipm<T, R, 128, 1>), dim3(B), dim3(128), lds, h->stream, d, only_active,
                                       h->qs.max_iter, ea, er, eta, fs, fl, pe, sp);
                } else {
                    hipLaunchKernelGGL((k_qp_ipm<T, R, 64, 1>), dim3(B), dim3(64), lds, h->stream, d, only_active,
                                       h->qs.max_iter, ea, er, eta, fs, fl, pe, sp);
                }
                DevBuf<T> dt = d;
                dt.scan_ctr = nullptr;
                const size_t lt = ipm_lds_bytes(h->N, (int)sizeof(T), 64 * tw);
                const void *ft = tw == 4 ? reinterpret_cast<const void *>(&k_qp_ipm<T, R, 256, 2>)
                                         : reinterpret_cast<const void *>(&k_qp_ipm<T, R, 128, 2>);
                HIPCHK(hipFuncSetAttribute(ft, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lt));
                if (tw == 4)
                    hipLaunchKernelGGL((k_qp_ipm<T, R, 256, 2>), dim3(B), dim3(256), lt, h->stream, dt, only_active,
                                       h->qs.max_iter, ea, er, eta, fs, fl, pe, sp);
                else
                    hipLaunchKernelGGL((k_qp_ipm<T, R, 128, 2>), dim3(B), dim3(128), lt, h->stream, dt, only_active,
                                       h->qs.max_iter, ea, er, eta, fs, fl, pe, sp);
                if (h->scan_pending) {
                    HIPCHK(hipStreamWaitEvent(h->stream, h->ev_scan, 0));
                    h->scan_pending = false;
                }
                break;
            }
        }
        if (nt == 256)
            hipLaunchKernelGGL((k_qp_ipm<T, R, 256, 0>), dim3(B), dim3(256), lds, h->stream, d, only_active,
                               h->qs.max_iter, ea, er, eta, fs, fl, pe, nullptr);
        else if (nt == 128)
            hipLaunchKernelGGL((k_qp_ipm<T, R, 128, 0>), dim3(B), dim3(128), lds, h->stream, d, only_active,
                               h->qs.max_iter, ea, er, eta, fs, fl, pe, nullptr);
        else
            hipLaunchKernelGGL((k_qp_ipm<T, R, 64, 0>), dim3(B), dim3(64), lds, h->stream, d, only_active,
                               h->qs.max_iter, ea, er, eta, fs, fl, pe, nullptr);
        if (h->scan_pending) {   // join behind the QP
            HIPCHK(hipStreamWaitEvent(h->stream, h->ev_scan, 0));
            h->scan_pending = false;
        }
        break;
    }
    case 3:
        hipLaunchKernelGGL((k_accept<T, R>), dim3(B), dim3(64), 0, h->stream, d, only_active ? 0 : 1);   // ACC_NT
        {
            const int per = h->ks_live ? (h->N + 1) * 9 + h->N * NU                // X | U
                                       : (h->N + 1) * 90 + h->N * NU * 10;   // X, Sigma | U, K elements per problem
            hipLaunchKernelGGL((k_keep_accepted<T>), dim3((unsigned)std::min(16, (per + 255) / 256), B), dim3(256), 0,
                               h->stream, d);
        }
        break;
    }
    HIPCHK(hipGetLastError());
}

template <typename T> void interpolate_impl(cmpc_handle h, int ni, double *Xo, double *Uo) {
    const size_t B = h->B, N = h->N, nx = B * 9 * N * ni, nuo = B * NU * (N - 1) * ni;
    void *dX = nullptr, *dU = nullptr;
    HIPCHK(hipMalloc(&dX, nx * sizeof(T)));
    HIPCHK(hipMalloc(&dU, std::max<size_t>(nuo, 1) * sizeof(T)));
    struct Free {
        void *p[2];
        ~Free() { for (void *q : p) if (q) (void)hipFree(q); }
    } fr{{dX, dU}};
    const long n = (long)(nx + nuo);
    hipLaunchKernelGGL((k_interpolate<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, h->buf<T>(),
                       ni, (int)NU, (T *)dX, (T *)dU);
    HIPCHK(hipGetLastError());
    from_dev<T>(h, Xo, dX, nx);
    from_dev<T>(h, Uo, dU, nuo);
}

template <typename T, int R> void plan_impl(cmpc_handle h, const cmpc_gait *gaits, const double *foot0) {
    const size_t B = h->B, NC = h->NC;
    void *dg = nullptr, *df = nullptr;
    HIPCHK(hipMalloc(&dg, B * sizeof(cmpc_gait)));
    HIPCHK(hipMalloc(&df, B * NC * 3 * sizeof(T)));
    struct Free {
        void *p[2];
        ~Free() { for (void *q : p) if (q) (void)hipFree(q); }
    } fr{{dg, df}};
    HIPCHK(hipMemcpyAsync(dg, gaits, B * sizeof(cmpc_gait), hipMemcpyHostToDevice, h->stream));
    to_dev<T>(h, df, foot0, B * NC * 3);
    const long n = (long)B * h->N;
    hipLaunchKernelGGL((k_contact_plan<T, R>), dim3((unsigned)((n + 127) / 128)), dim3(128), 0, h->stream,
                       h->buf<T>(), (const cmpc_gait *)dg, (const T *)df, (uint8_t *)h->logic, (T *)h->pos,
                       (T *)h->rot);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(h->stream));
}

template <typename T, int R> void default_controls_impl(cmpc_handle h) {
    const long n = (long)h->B * h->N;
    hipLaunchKernelGGL((k_default_controls<T, R>), dim3((unsigned)((n + 127) / 128)), dim3(128), 0, h->stream,
                       h->buf<T>(), (T *)h->Ubar);
    HIPCHK(hipGetLastError());
}

template <typename T, int R> void rollout_impl(cmpc_handle h, const double *X, const double *U, double *out) {
    const size_t nx = (size_t)h->B * (h->N + 1) * 9, nu = (size_t)h->B * h->N * NU;
    void *dX = nullptr, *dU = nullptr, *dO = nullptr;
    HIPCHK(hipMalloc(&dX, nx * sizeof(T)));
    HIPCHK(hipMalloc(&dU, nu * sizeof(T)));
    HIPCHK(hipMalloc(&dO, nx * sizeof(T)));
    struct Free {
        void *p[3];
        ~Free() { for (void *q : p) if (q) (void)hipFree(q); }
    } fr{{dX, dU, dO}};
    to_dev<T>(h, dX, X, nx);
    // U arrives with the handle's per-knot width NU (zero-padded contacts beyond nu)
    to_dev<T>(h, dU, U, nu);
    const long n = (long)h->B * (h->N + 1);
    hipLaunchKernelGGL((k_rollout<T, R>), dim3((unsigned)((n + 127) / 128)), dim3(128), 0, h->stream, h->buf<T>(),
                       (const T *)dX, (const T *)dU, (T *)dO);
    HIPCHK(hipGetLastError());
    from_dev<T>(h, out, dO, nx);
}

// The dense A, Bu, C for the getters and the CSC export: reference mode's SCP loop does not store
// them (launch_phase, case 0); its linearization point never moves (quirk Q1), so one more
// k_lin_knots pass over every problem rewrites the same values and adds the dense arrays.
template <typename T, int R> void ensure_dense_impl(cmpc_handle h) {
    DevBuf<T> d = h->buf<T>();
    const long n = (long)h->B * h->N;
    hipLaunchKernelGGL((k_lin_knots<T, R>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, d, 0, 1);
    HIPCHK(hipGetLastError());
}
}  // namespace

namespace cmpc_host {

void ensure_dense(cmpc_handle h) {
    settle_all(h);
    if (h->lin_dense || !h->lin_lane_done || h->B == 0) return;
    if (h->prec == CMPC_PREC_F64) {
        if (h->robot == 0) ensure_dense_impl<double, 0>(h); else ensure_dense_impl<double, 1>(h);
    } else {
        if (h->robot == 0) ensure_dense_impl<float, 0>(h); else ensure_dense_impl<float, 1>(h);
    }
    h->lin_dense = true;
}


// Reference mode serves accepted K / Sigma from the live arrays (cmpc_handle_::ks_live); before
// anything can make them differ from the accepted iteration's (GuSTO mode moves the linearization
// point, new contact plans change it), they are copied to Kacc / Sacc once and copied per accept
// from then on.
void materialize_accepted_ks(cmpc_handle h) {
    if (h->pf_armed || h->pfK_issued || h->pfS_issued) {   // a prefetch serves live arrays only
        if (h->pfK_issued || h->pfS_issued) HIPCHK(hipStreamSynchronize(h->copy));
        h->pf_armed = h->pfK_issued = h->pfS_issued = false;
        h->pf_K = h->pf_S = nullptr;
    }
    if (!h->ks_live) return;
    settle_all(h);   // Sigma of a deferred scan first
    if (h->B > 0) {
        const size_t e = h->esz();
        HIPCHK(hipMemcpyAsync(h->Kacc, h->K, (size_t)h->max_batch * h->N * NU * 9 * e, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(hipMemcpyAsync(h->Sacc, h->Sig, (size_t)h->max_batch * (h->N + 1) * 81 * e, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
    }
    h->ks_live = false;
}


// A scan left deferred or running on the side stream (cmpc_scp_iterate stopped between its phases,
// e.g. by an error) is settled before anything reads Sigma or relaunches the linearization.
void settle_all(cmpc_handle h) {
    if (!h->scan_deferred && !h->scan_pending) return;
    if (h->prec == CMPC_PREC_F64) {
        if (h->robot == 0) settle_scan<double, 0>(h, h->scan_oa); else settle_scan<double, 1>(h, h->scan_oa);
    } else {
        if (h->robot == 0) settle_scan<float, 0>(h, h->scan_oa); else settle_scan<float, 1>(h, h->scan_oa);
    }
}

}  // namespace cmpc_host

namespace {

void phase(cmpc_handle h, int ph, int only_active, bool overlap = false) {
    need(h->B > 0, "no problems uploaded");
    need(h->n_classes > 0, "parameters not set");
    if (h->prec == CMPC_PREC_F64) {
        if (h->robot == 0) launch_phase<double, 0>(h, ph, only_active, overlap);
        else launch_phase<double, 1>(h, ph, only_active, overlap);
    } else {
        if (h->robot == 0) launch_phase<float, 0>(h, ph, only_active, overlap);
        else launch_phase<float, 1>(h, ph, only_active, overlap);
    }
}

// Iteration records and accepted-iterate slots for max(max_iterations) iterations per problem (the
// reference appends every accepted iterate, src/scp_solver.py:162-167); the K / Sigma slots only
// in GuSTO mode, where they differ between accepts.  Grown before an iteration needs them; a
// regrow drops earlier records (capacity changes only with new parameter classes).
void ensure_history(cmpc_handle h) {
    int cap = 1;
    for (auto &p : h->hparams) cap = std::max(cap, (int)p.max_iterations);
    cap = std::min(cap, 4096);
    const size_t Bm = h->max_batch, K1 = h->N + 1, e = h->esz(), LS = (size_t)h->max_batch * h->N;
    if (h->log_cap < cap) {
        h->regrow(h->hlog, Bm * cap * sizeof(cmpc_iter_record));
        h->log_cap = cap;
    }
    if (h->hist_cap < cap) {
        h->regrow(h->hX, (size_t)cap * Bm * K1 * 9 * e);
        h->regrow(h->hU, (size_t)cap * Bm * h->N * NU * e);
        h->hist_cap = cap;
    }
    if (h->scp_mode == CMPC_SCP_MODE_GUSTO && h->hks_cap < h->hist_cap) {
        h->regrow(h->hK, (size_t)h->hist_cap * NU * 9 * LS * e);
        h->regrow(h->hS, (size_t)h->hist_cap * Bm * K1 * 81 * e);
        h->hks_cap = h->hist_cap;
    }
}

// ---- K / Sigma prefetch (cmpc_prefetch_ks).  In reference mode the linearization point never
// moves (Q1): K is final once the first iteration's linearization ran and Sigma once its scan ran,
// and the accepted K / Sigma are those arrays.  The copies to the caller's page-locked buffers
// then run on the copy stream's DMA while the QP runs (K) or while the accept step and the
// caller's own getters run (Sigma).
void pf_disarm(cmpc_handle h) {
    if (h->pfK_issued || h->pfS_issued) HIPCHK(hipStreamSynchronize(h->copy));
    h->pf_armed = h->pfK_issued = h->pfS_issued = false;
    h->pf_K = h->pf_S = nullptr;
}

double *pf_staging(cmpc_handle h, size_t bytes) {
    if (bytes > h->pf_stage_bytes) {
        HIPCHK(hipStreamSynchronize(h->copy));
        h->regrow(h->pf_stage, bytes);
        h->pf_stage_bytes = bytes;
    }
    return (double *)h->pf_stage;
}

// after phase 0 on the main stream: K (transposed / widened on the main stream, ~40 us) to the host
void pf_issue_K(cmpc_handle h) {
    if (!h->pf_armed || h->pfK_issued || !h->pf_K || h->scp_mode != CMPC_SCP_MODE_REFERENCE || !h->ks_live) return;
    const size_t B = h->B, N = h->N, LS = (size_t)h->max_batch * N, nK = B * N * NU * 9;
    double *stg = pf_staging(h, (nK + (h->prec == CMPC_PREC_F32 ? B * (N + 1) * 81 : 0)) * sizeof(double));
    const dim3 grid((unsigned)((B * N + 31) / 32), (unsigned)((NU * 9 + 31) / 32));
    if (h->prec == CMPC_PREC_F32)
        hipLaunchKernelGGL((k_knot_major<float>), grid, dim3(256), 0, h->stream, (const float *)h->K, LS, (size_t)0, B * N,
                           (int)(NU * 9), stg);
    else
        hipLaunchKernelGGL((k_knot_major<double>), grid, dim3(256), 0, h->stream, (const double *)h->K, LS, (size_t)0,
                           B * N, (int)(NU * 9), stg);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(h->ev_pf_src, h->stream));
    HIPCHK(hipStreamWaitEvent(h->copy, h->ev_pf_src, 0));
    HIPCHK(hipMemcpyAsync(h->pf_K, stg, nK * sizeof(double), hipMemcpyDeviceToHost, h->copy));
    HIPCHK(hipEventRecord(h->ev_pfK, h->copy));
    h->pfK_issued = true;
}

// after the QP on the main stream (the covariance scans have joined it there): Sigma to the host
void pf_issue_S(cmpc_handle h) {
    if (!h->pf_armed || h->pfS_issued || !h->pf_S || h->scp_mode != CMPC_SCP_MODE_REFERENCE || !h->ks_live) return;
    if (h->scan_deferred || h->scan_pending) return;   // not yet joined (phase-by-phase callers)
    const size_t B = h->B, N = h->N, nS = B * (N + 1) * 81, nK = B * N * NU * 9;
    const void *src = h->Sig;
    if (h->prec == CMPC_PREC_F32) {
        double *stg = pf_staging(h, (nK + nS) * sizeof(double)) + nK;
        hipLaunchKernelGGL(k_widen, dim3((unsigned)std::min<size_t>((nS + 255) / 256, 4096)), dim3(256), 0, h->stream,
                           (const float *)h->Sig, nS, stg);
        HIPCHK(hipGetLastError());
        src = stg;
    }
    HIPCHK(hipEventRecord(h->ev_pf_src, h->stream));
    HIPCHK(hipStreamWaitEvent(h->copy, h->ev_pf_src, 0));
    HIPCHK(hipMemcpyAsync(h->pf_S, src, nS * sizeof(double), hipMemcpyDeviceToHost, h->copy));
    HIPCHK(hipEventRecord(h->ev_pfS, h->copy));
    h->pfS_issued = true;
}

void reset_scp(cmpc_handle h, const int32_t *class_id) {
    settle_all(h);
    pf_disarm(h);   // a prefetch belongs to one solve of one upload   // a scan still pending reads the previous batch's arrays
    h->ks_live = h->scp_mode == CMPC_SCP_MODE_REFERENCE;
    h->lin_lane_done = false;   // new inputs: nothing to recompute densely until the next linearization
    std::vector<ScpState> st(h->B);
    for (int b = 0; b < h->B; ++b) {
        const cmpc_params &p = h->hparams[class_id[b]];
        ScpState s{};
        s.weight = p.omega0; s.radius = p.tr_radius0; s.active = 1; s.status = CMPC_SCP_RUNNING;
        st[b] = s;
    }
    HIPCHK(hipMemcpyAsync(h->scp, st.data(), st.size() * sizeof(ScpState), hipMemcpyHostToDevice, h->stream));
    // a new batch has no Newton-step counts: the first grouped QP launch orders its problems by
    // index (k_qp_order), not by counts learned on whatever the handle solved before
    HIPCHK(hipMemsetAsync(h->qp_iters, 0, (size_t)h->B * 4, h->stream));
    HIPCHK(hipMemsetAsync(h->qp_tail, 0, (size_t)h->B * 4, h->stream));
    HIPCHK(hipMemsetAsync(h->qp_polish, 0, (size_t)h->B * 4, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
}

// Knots [kn0, kn0 + n) of an element-major array (DevBuf::LS) into the knot-major host layout
// dst[kn][e] (e < ne): transposed (and widened to fp64) on the device into the handle's scratch
// buffer, then one contiguous copy.
void dl_knots(cmpc_handle h, double *dst, const void *src, size_t kn0, size_t n, size_t ne) {
    if (!dst || n == 0) return;
    const size_t LS = (size_t)h->max_batch * h->N;
    double *tmp = (double *)h->scratch_bytes_at_least(n * ne * sizeof(double));
    const dim3 grid((unsigned)((n + 31) / 32), (unsigned)((ne + 31) / 32));
    if (h->prec == CMPC_PREC_F64)
        hipLaunchKernelGGL((k_knot_major<double>), grid, dim3(256), 0, h->stream, (const double *)src, LS, kn0, n,
                           (int)ne, tmp);
    else
        hipLaunchKernelGGL((k_knot_major<float>), grid, dim3(256), 0, h->stream, (const float *)src, LS, kn0, n,
                           (int)ne, tmp);
    HIPCHK(hipGetLastError());
    from_dev_raw(h, dst, tmp, n * ne * sizeof(double));
}

std::vector<ScpState> get_scp(cmpc_handle h) {
    std::vector<ScpState> st(h->B);
    from_dev_raw(h, st.data(), h->scp, st.size() * sizeof(ScpState));
    return st;
}

}  // namespace

extern "C" {

int cmpc_version(void) { return 1; }

const char *cmpc_last_error(cmpc_handle h) { return h ? h->err.c_str() : "null handle"; }

int cmpc_default_qp_settings(int precision, cmpc_qp_settings *s) {
    if (!s) return -1;
    s->max_iter = precision == CMPC_PREC_F64 ? 60 : 40;
    s->eps_abs = 0.0;   // the robot's (qp_eps_default)
    s->eps_rel = 0.0;
    s->step_fraction = 0.0;     // the robot's default, qp_step_fraction
    s->init_floor_s = 0.1;
    s->init_floor_l = 0.1;
    s->waves_per_problem = 0;
    s->polish_eps = -1.0;   // the robot's (qp_polish_eps)
    return 0;
}

int cmpc_create(cmpc_handle *out, int device, int robot, int N, int max_batch, int precision) {
    if (!out) return -1;
    *out = nullptr;
    if (robot != 0 && robot != 1) return -2;
    if (N < 2 || N > 255 || max_batch < 1) return -2;
    if (precision != CMPC_PREC_F64 && precision != CMPC_PREC_F32) return -2;
    // TALOS QPs need fp64: the CoP rows at centimetre scale next to the friction rows, and
    // D = lambda / s spanning 1e15 (fp64 needs iterative refinement there), took every
    // fp32 solve to non-finite values by its third Newton step (N = 40).  Every BASELINE TALOS
    // configuration is fp64.
    if (robot == CMPC_ROBOT_TALOS && precision == CMPC_PREC_F32) return -5;
    cmpc_handle h = new cmpc_handle_s();
    h->device = device; h->robot = robot; h->N = N; h->max_batch = max_batch; h->prec = precision;
    h->NC = robot == 0 ? 4 : 2;
    h->NI = 25;
    h->SS = robot == 0 ? Stage<0>::SIZE : Stage<1>::SIZE;
    cmpc_default_qp_settings(precision, &h->qs);
    int rc = guard(h, [&] {
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        need(device >= 0 && device < ndev, "invalid device id");
        HIPCHK(hipSetDevice(device));
        HIPCHK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        int prio_low = 0, prio_high = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&prio_low, &prio_high));
        HIPCHK(hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, prio_low));
        HIPCHK(hipEventCreateWithFlags(&h->ev_asm, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&h->ev_scan, hipEventDisableTiming));
        HIPCHK(hipStreamCreateWithFlags(&h->copy, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&h->ev_pf_src, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&h->ev_pfK, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&h->ev_pfS, hipEventDisableTiming));
        h->scan_ctr = h->dalloc(16);
        h->qp_order = h->dalloc(((size_t)max_batch + 8) * 4);   // ceil(B / P) P slots
        HIPCHK(hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, device));
        for (auto &e : h->ev) HIPCHK(hipEventCreate(&e));
        const size_t Bm = max_batch, K1 = N + 1, NB = N + 2, e = h->esz(), NC = h->NC;
        h->class_id = h->dalloc(Bm * 4);
        h->logic = h->dalloc(Bm * N * NC);
        h->pos = h->dalloc(Bm * N * NC * 3 * e);
        h->rot = h->dalloc(Bm * N * NC * 9 * e);
        h->Xbar = h->dalloc(Bm * K1 * 9 * e);
        h->Ubar = h->dalloc(Bm * N * NU * e);
        h->Xlin = h->dalloc(Bm * K1 * 9 * e);
        h->Ulin = h->dalloc(Bm * N * NU * e);
        h->f = h->dalloc(Bm * N * 9 * e);
        h->A = h->dalloc(Bm * N * 81 * e);
        h->Bu = h->dalloc(Bm * N * 9 * NU * e);
        h->C = h->dalloc(Bm * N * 9 * 3 * NC * e);
        h->K = h->dalloc(Bm * N * NU * 9 * e);
        h->Sig = h->dalloc(Bm * K1 * 81 * e);
        h->Acl = h->dalloc(Bm * N * 81 * e);
        h->Qw = h->dalloc(Bm * N * 81 * e);
        h->stage = h->dalloc(Bm * KPC * h->SS * e);
        h->cw = h->dalloc(Bm * e);
        h->xs = h->dalloc(Bm * K1 * 9 * e);
        h->us = h->dalloc(Bm * N * NU * e);
        h->ts = h->dalloc(Bm * K1 * e);
        h->nus = h->dalloc(Bm * NB * 9 * e);
        h->lams = h->dalloc(Bm * K1 * h->NI * e);
        h->qp_status = h->dalloc(Bm * 4);
        h->qp_iters = h->dalloc(Bm * 4);
        h->qp_merit = h->dalloc(Bm * e);
        h->qp_nref = h->dalloc(Bm * 4);
        h->qp_tail = h->dalloc(Bm * 4);
        h->qp_polish = h->dalloc(Bm * 4);
        h->qp_state = h->dalloc(Bm * ipm_state_bytes((int)e));
        h->qp_split = h->dalloc((Bm + 2) * 4);
        h->ws_stride = ipm_workspace_elems(N, robot);
        h->ws = h->dalloc(Bm * h->ws_stride * e);
        h->scp = h->dalloc(Bm * sizeof(ScpState));
        h->Xacc = h->dalloc(Bm * K1 * 9 * e);
        h->Uacc = h->dalloc(Bm * N * NU * e);
        h->Kacc = h->dalloc(Bm * N * NU * 9 * e);
        h->Sacc = h->dalloc(Bm * K1 * 81 * e);
        h->stamps = h->dalloc(Bm * 16 * 8);
        HIPCHK(hipStreamSynchronize(h->stream));
    });
    if (rc != 0) {
        std::fprintf(stderr, "cmpc_create: %s\n", h->err.c_str());
        cmpc_destroy(h);
        return rc;
    }
    *out = h;
    return 0;
}

int cmpc_destroy(cmpc_handle h) {
    if (!h) return 0;
    (void)hipSetDevice(h->device);
    if (h->side) (void)hipStreamSynchronize(h->side);
    if (h->copy) (void)hipStreamSynchronize(h->copy);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->comm && h->comm_free) h->comm_free(h->comm);
    for (void *p : h->allocs) (void)hipFree(p);
    if (h->scratch) (void)hipFree(h->scratch);
    for (auto &e : h->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto &a : h->ev_pool)
        for (auto &e : a) (void)hipEventDestroy(e);
    for (hipEvent_t e : {h->ev_pf_src, h->ev_pfK, h->ev_pfS})
        if (e) (void)hipEventDestroy(e);
    if (h->copy) (void)hipStreamDestroy(h->copy);
    if (h->ev_asm) (void)hipEventDestroy(h->ev_asm);
    if (h->ev_scan) (void)hipEventDestroy(h->ev_scan);
    if (h->side) (void)hipStreamDestroy(h->side);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return 0;
}

int cmpc_set_qp_settings(cmpc_handle h, const cmpc_qp_settings *s) {
    return guard(h, [&] {
        need(s && s->max_iter > 0 && s->step_fraction >= 0 && s->step_fraction < 1 && s->init_floor_s >= 0 &&
                 s->init_floor_l >= 0 && (s->init_floor_s > 0) == (s->init_floor_l > 0) &&
                 (s->waves_per_problem == 0 || s->waves_per_problem == 1 || s->waves_per_problem == 2 ||
                  s->waves_per_problem == 4), "invalid QP settings");
        h->qs = *s;
    });
}

int cmpc_set_params(cmpc_handle h, int n_classes, const cmpc_params *classes) {
    return guard(h, [&] {
        need(n_classes > 0 && classes, "no parameter classes");
        // new R or noise change the next linearization's K / Sigma: the accepted ones are copied out
        // of the live arrays first
        materialize_accepted_ks(h);
        for (int i = 0; i < n_classes; ++i) {
            const cmpc_params &p = classes[i];
            need(p.mass > 0 && p.dt > 0 && p.mu > 0, "invalid mass/dt/mu");
            for (int j = 0; j < 9; ++j) need(p.Wx[j] > 0, "state_cost_weights must be positive");
            for (int j = 0; j < 12; ++j) need(p.Wu[j] > 0, "control_cost_weights must be positive");
            need(p.omega0 > 0 && p.tr_radius0 > 0 && p.max_iterations > 0, "invalid scp_params");
        }
        h->hparams.assign(classes, classes + n_classes);
        h->n_classes = n_classes;
        // the knot-per-lane linearization needs a diagonal LQR weight R (every reference config);
        // CMPC_LIN_LEGACY=1 forces the workgroup-per-problem kernel
        bool diag = true;
        for (int i = 0; i < n_classes; ++i)
            for (int r = 0; r < 12; ++r)
                for (int c = 0; c < 12; ++c)
                    if (r != c && classes[i].R[r * 12 + c] != 0.0) diag = false;
        const char *leg = std::getenv("CMPC_LIN_LEGACY");
        h->lin_lane = diag && !(leg && leg[0] == '1');
        const int nw = 3 * h->NC;
        if (h->params) { HIPCHK(hipFree(h->params)); h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), h->params)); }
        if (h->prec == CMPC_PREC_F64) {
            std::vector<DevParams<double>> v;
            for (int i = 0; i < n_classes; ++i) v.push_back(conv_params<double>(classes[i], nw));
            h->params = h->dalloc(v.size() * sizeof(v[0]));
            HIPCHK(hipMemcpyAsync(h->params, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice, h->stream));
        } else {
            std::vector<DevParams<float>> v;
            for (int i = 0; i < n_classes; ++i) v.push_back(conv_params<float>(classes[i], nw));
            h->params = h->dalloc(v.size() * sizeof(v[0]));
            HIPCHK(hipMemcpyAsync(h->params, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice, h->stream));
        }
        HIPCHK(hipStreamSynchronize(h->stream));
    });
}

int cmpc_upload(cmpc_handle h, int B, const int32_t *class_id, const int8_t *logic, const double *pos,
                const double *rot, const double *Xbar, const double *Ubar) {
    return guard(h, [&] {
        need(h->n_classes > 0, "call cmpc_set_params first");
        need(B >= 1 && B <= h->max_batch, "batch size out of range");
        need(class_id && logic && pos && rot && Xbar && Ubar, "null input buffer");
        const int N = h->N, NC = h->NC;
        for (int b = 0; b < B; ++b) need(class_id[b] >= 0 && class_id[b] < h->n_classes, "class_id out of range");
        for (size_t k = 0; k < (size_t)B * N; ++k) {
            int act = 0;
            for (int c = 0; c < NC; ++c) {
                need(logic[k * NC + c] == 0 || logic[k * NC + c] == 1, "contact logic must be 0/1");
                act += logic[k * NC + c];
            }
            need(act > 0, "a knot without active contact (the reference divides by zero there)");
        }
        h->B = B;
        h->plans_B = 0;
        HIPCHK(hipMemcpyAsync(h->class_id, class_id, (size_t)B * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(hipMemcpyAsync(h->logic, logic, (size_t)B * N * NC, hipMemcpyHostToDevice, h->stream));
        auto up = [&](void *dst, const double *src, size_t n) {
            if (h->prec == CMPC_PREC_F64) to_dev<double>(h, dst, src, n); else to_dev<float>(h, dst, src, n);
        };
        up(h->pos, pos, (size_t)B * N * NC * 3);
        up(h->rot, rot, (size_t)B * N * NC * 9);
        up(h->Xbar, Xbar, (size_t)B * (N + 1) * 9);
        up(h->Ubar, Ubar, (size_t)B * N * NU);
        // the linearization point starts at the warm start
        HIPCHK(hipMemcpyAsync(h->Xlin, h->Xbar, (size_t)B * (N + 1) * 9 * h->esz(), hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(hipMemcpyAsync(h->Ulin, h->Ubar, (size_t)B * N * NU * h->esz(), hipMemcpyDeviceToDevice, h->stream));
        reset_scp(h, class_id);
    });
}

int cmpc_set_trust_region(cmpc_handle h, const double *weight, const double *radius) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        auto st = get_scp(h);
        for (int b = 0; b < h->B; ++b) {
            if (weight) { need(weight[b] > 0, "trust-region weight must be > 0"); st[b].weight = weight[b]; }
            if (radius) { need(radius[b] > 0, "trust-region radius must be > 0"); st[b].radius = radius[b]; }
        }
        HIPCHK(hipMemcpyAsync(h->scp, st.data(), st.size() * sizeof(ScpState), hipMemcpyHostToDevice, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
    });
}

int cmpc_generate_contact_plans(cmpc_handle h, int B, const cmpc_gait *gaits, const double *foot0) {
    return guard(h, [&] {
        materialize_accepted_ks(h);   // the accepted K / Sigma belong to the old plans
        need(B >= 1 && B <= h->max_batch, "batch size out of range");
        need(gaits && foot0, "null input buffer");
        for (int b = 0; b < B; ++b) {
            const cmpc_gait &g = gaits[b];
            need(g.type == CMPC_GAIT_TROT || g.type == CMPC_GAIT_PACE || g.type == CMPC_GAIT_BOUND, "unknown gait type");
            need(g.nb_steps >= 1 && g.step_knots >= 1 && g.support_knots >= 1, "invalid gait knots");
            need((long)g.nb_steps * 2 * (g.step_knots + g.support_knots) + g.support_knots >= h->N,
                 "contact plan shorter than the horizon N (raise nb_steps)");
            need(h->robot == 0 || g.type == CMPC_GAIT_PACE,
                 "TALOS plans support PACE only (other gaits swing both feet: a knot without active contact)");
        }
        h->B = B;
        if (h->prec == CMPC_PREC_F64) {
            if (h->robot == 0) plan_impl<double, 0>(h, gaits, foot0); else plan_impl<double, 1>(h, gaits, foot0);
        } else {
            if (h->robot == 0) plan_impl<float, 0>(h, gaits, foot0); else plan_impl<float, 1>(h, gaits, foot0);
        }
        h->plans_B = B;
    });
}

int cmpc_upload_states(cmpc_handle h, int B, const int32_t *class_id, const double *Xbar, const double *Ubar) {
    return guard(h, [&] {
        need(h->n_classes > 0, "call cmpc_set_params first");
        need(h->plans_B == B && B >= 1, "no device contact plans for this batch (cmpc_generate_contact_plans)");
        need(class_id && Xbar, "null input buffer");
        for (int b = 0; b < B; ++b) need(class_id[b] >= 0 && class_id[b] < h->n_classes, "class_id out of range");
        const int N = h->N;
        h->B = B;
        HIPCHK(hipMemcpyAsync(h->class_id, class_id, (size_t)B * 4, hipMemcpyHostToDevice, h->stream));
        auto up = [&](void *dst, const double *src, size_t n) {
            if (h->prec == CMPC_PREC_F64) to_dev<double>(h, dst, src, n); else to_dev<float>(h, dst, src, n);
        };
        up(h->Xbar, Xbar, (size_t)B * (N + 1) * 9);
        if (Ubar) {
            up(h->Ubar, Ubar, (size_t)B * N * NU);
        } else if (h->prec == CMPC_PREC_F64) {
            if (h->robot == 0) default_controls_impl<double, 0>(h); else default_controls_impl<double, 1>(h);
        } else {
            if (h->robot == 0) default_controls_impl<float, 0>(h); else default_controls_impl<float, 1>(h);
        }
        HIPCHK(hipMemcpyAsync(h->Xlin, h->Xbar, (size_t)B * (N + 1) * 9 * h->esz(), hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(hipMemcpyAsync(h->Ulin, h->Ubar, (size_t)B * N * NU * h->esz(), hipMemcpyDeviceToDevice, h->stream));
        reset_scp(h, class_id);
    });
}

int cmpc_get_contact_plans(cmpc_handle h, int8_t *logic, double *pos, double *rot) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        const size_t B = h->B, N = h->N, NC = h->NC;
        auto dl = [&](double *dst, void *src, size_t n) {
            if (h->prec == CMPC_PREC_F64) from_dev<double>(h, dst, src, n); else from_dev<float>(h, dst, src, n);
        };
        if (logic) from_dev_raw(h, logic, h->logic, B * N * NC);
        dl(pos, h->pos, B * N * NC * 3);
        dl(rot, h->rot, B * N * NC * 9);
    });
}

int cmpc_get_warm_start(cmpc_handle h, double *Xbar, double *Ubar) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        const size_t B = h->B, N = h->N;
        auto dl = [&](double *dst, void *src, size_t n) {
            if (h->prec == CMPC_PREC_F64) from_dev<double>(h, dst, src, n); else from_dev<float>(h, dst, src, n);
        };
        dl(Xbar, h->Xbar, B * (N + 1) * 9);
        dl(Ubar, h->Ubar, B * N * NU);
    });
}

int cmpc_set_scp_mode(cmpc_handle h, int mode) {
    return guard(h, [&] {
        need(mode == CMPC_SCP_MODE_REFERENCE || mode == CMPC_SCP_MODE_GUSTO, "unknown SCP mode");
        if (mode != CMPC_SCP_MODE_REFERENCE) materialize_accepted_ks(h);
        h->scp_mode = mode;
    });
}

int cmpc_get_linearization_point(cmpc_handle h, double *X, double *U, double *convergence) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        const size_t B = h->B, N = h->N;
        auto dl = [&](double *dst, void *src, size_t n) {
            if (h->prec == CMPC_PREC_F64) from_dev<double>(h, dst, src, n); else from_dev<float>(h, dst, src, n);
        };
        dl(X, h->Xlin, B * (N + 1) * 9);
        dl(U, h->Ulin, B * N * NU);
        if (convergence) {
            auto st = get_scp(h);
            for (size_t b = 0; b < B; ++b) convergence[b] = st[b].conv;
        }
    });
}

int cmpc_interpolate(cmpc_handle h, int n_inner, double *X_out, double *U_out) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        need(n_inner >= 1 && X_out && U_out, "invalid interpolation arguments");
        if (h->prec == CMPC_PREC_F64) interpolate_impl<double>(h, n_inner, X_out, U_out);
        else interpolate_impl<float>(h, n_inner, X_out, U_out);
    });
}

int cmpc_rollout(cmpc_handle h, const double *X, const double *U, double *out) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        need(h->n_classes > 0, "parameters not set");
        need(X && U && out, "null buffer");
        if (h->prec == CMPC_PREC_F64) {
            if (h->robot == 0) rollout_impl<double, 0>(h, X, U, out); else rollout_impl<double, 1>(h, X, U, out);
        } else {
            if (h->robot == 0) rollout_impl<float, 0>(h, X, U, out); else rollout_impl<float, 1>(h, X, U, out);
        }
    });
}

int cmpc_linearize(cmpc_handle h) { return guard(h, [&] { phase(h, 0, 0); }); }
int cmpc_assemble(cmpc_handle h) { return guard(h, [&] { phase(h, 1, 0); }); }
int cmpc_qp_solve(cmpc_handle h) { return guard(h, [&] { phase(h, 2, 0); }); }
int cmpc_accept(cmpc_handle h, int fixed_iters) {
    return guard(h, [&] {
        ensure_history(h);
        phase(h, 3, fixed_iters ? 0 : 1);
    });
}

int cmpc_scp_iterate(cmpc_handle h, int fixed_iters) {
    return guard(h, [&] {
        const int oa = fixed_iters ? 0 : 1;
        ensure_history(h);
        hipEvent_t *ev = h->ev;
        if (h->accumulate) {
            if (h->ev_used == h->ev_pool.size()) {
                std::array<hipEvent_t, 5> a;
                for (auto &e : a) HIPCHK(hipEventCreate(&e));
                h->ev_pool.push_back(a);
            }
            ev = h->ev_pool[h->ev_used++].data();
        }
        HIPCHK(hipEventRecord(ev[0], h->stream));
        phase(h, 0, oa, true);   // the covariance scan may run beside the QP (launch_phase)
        pf_issue_K(h);
        HIPCHK(hipEventRecord(ev[1], h->stream));
        phase(h, 1, oa);
        HIPCHK(hipEventRecord(ev[2], h->stream));
        phase(h, 2, oa);
        pf_issue_S(h);
        HIPCHK(hipEventRecord(ev[3], h->stream));
        phase(h, 3, oa);
        HIPCHK(hipEventRecord(ev[4], h->stream));
        if (!h->accumulate) h->timed = true;
    });
}

int cmpc_solve_scp(cmpc_handle h, int fixed_iters, int *n_iterations_out) {
    return guard(h, [&] {
        int maxit = 0;
        for (auto &p : h->hparams) maxit = std::max(maxit, p.max_iterations);
        int it = 0;
        for (; it < maxit; ++it) {
            if (cmpc_scp_iterate(h, fixed_iters) != 0) throw Fail{-3, h->err};
            if (!fixed_iters) {
                auto st = get_scp(h);
                bool any = false;
                for (auto &s : st) any |= s.active != 0;
                if (!any) { ++it; break; }
            }
        }
        HIPCHK(hipStreamSynchronize(h->stream));
        if (n_iterations_out) *n_iterations_out = it;
    });
}

int cmpc_synchronize(cmpc_handle h) { return guard(h, [&] { HIPCHK(hipStreamSynchronize(h->stream)); }); }

int cmpc_get_linearization(cmpc_handle h, double *f, double *A, double *Bu, double *C, double *K, double *Sigma) {
    return guard(h, [&] {
        const size_t B = h->B, N = h->N, NC = h->NC;
        ensure_dense(h);
        auto dl = [&](double *dst, void *src, size_t n) {
            if (h->prec == CMPC_PREC_F64) from_dev<double>(h, dst, src, n); else from_dev<float>(h, dst, src, n);
        };
        dl_knots(h, f, h->f, 0, B * N, 9);
        dl_knots(h, A, h->A, 0, B * N, 81);
        dl_knots(h, Bu, h->Bu, 0, B * N, 9 * NU);
        dl_knots(h, C, h->C, 0, B * N, 9 * 3 * NC);
        dl_knots(h, K, h->K, 0, B * N, NU * 9);
        dl(Sigma, h->Sig, B * (N + 1) * 81);
    });
}

int cmpc_qp_sizes(cmpc_handle h, int32_t *n, int32_t *m, int32_t *nnzP, int32_t *nnzA) {
    return guard(h, [&] {
        const int N = h->N, NC = h->NC;
        if (n) *n = 9 * (N + 1) + NU * N + (N + 1) + N;
        const int mcop = h->robot == 1 ? 2 * NC * N : 0;
        if (m) *m = 9 + 9 * N + 9 + mcop + 5 * NC * N + 8 * (N + 1) + (N + 1);
        if (nnzP) *nnzP = 9 * (N + 1) + NU * N;
        // upper bound on stored entries (explicit zeros are dropped at export)
        if (nnzA) *nnzA = 9 + 9 * N * (9 + NU + 1) + 9 + mcop + 4 * 3 * NC * N + 4 * 8 * (N + 1) + (N + 1);
    });
}

int cmpc_export_qp(cmpc_handle h, int b, double *P_x, int32_t *P_i, int32_t *P_p, double *q, double *A_x,
                   int32_t *A_i, int32_t *A_p, double *l, double *u) {
    return guard(h, [&] {
        need(b >= 0 && b < h->B, "problem index out of range");
        const int N = h->N, NC = h->NC, K1 = N + 1, NUPC = NU / NC, FO = h->robot == 0 ? 0 : 2, SS = h->SS;
        ensure_dense(h);
        const int n = 9 * K1 + NU * N + K1 + N;
        auto dl = [&](std::vector<double> &dst, void *src, size_t off, size_t cnt) {
            dst.resize(cnt);
            const size_t e = h->esz();
            if (h->prec == CMPC_PREC_F64) from_dev<double>(h, dst.data(), (char *)src + off * e, cnt);
            else from_dev<float>(h, dst.data(), (char *)src + off * e, cnt);
        };
        std::vector<double> st, A, Bm, xb;
        const int KP = KPC;
        dl(st, h->stage, (size_t)b * KP * SS, (size_t)KP * SS);
        auto sf = [&](int k, int f) { return st[(size_t)f * KP + k]; };   // field-major records
        A.resize((size_t)N * 81);
        Bm.resize((size_t)N * 9 * NU);
        dl_knots(h, A.data(), h->A, (size_t)b * N, N, 81);
        dl_knots(h, Bm.data(), h->Bu, (size_t)b * N, N, 9 * NU);
        dl(xb, h->Xbar, (size_t)b * K1 * 9, (size_t)K1 * 9);
        std::vector<int8_t> lg((size_t)N * NC);
        from_dev_raw(h, lg.data(), (char *)h->logic + (size_t)b * N * NC, lg.size());
        int32_t cid = 0;
        from_dev_raw(h, &cid, (char *)h->class_id + (size_t)b * 4, 4);
        const cmpc_params &p = h->hparams[cid];
        ScpState sc;
        from_dev_raw(h, &sc, (char *)h->scp + (size_t)b * sizeof(ScpState), sizeof(ScpState));
        const double cw = -1.0 / sc.weight;
        auto xi = [&](int k) { return 9 * k; };
        auto ui = [&](int k) { return 9 * K1 + NU * k; };
        auto ti = [&](int k) { return 9 * K1 + NU * N + k; };
        // ---- P (diagonal) and q
        int pp = 0;
        for (int c = 0; c < n; ++c) {
            P_p[c] = pp;
            double v = 0;
            if (c < 9 * K1) v = p.Wx[c % 9];
            else if (c < 9 * K1 + NU * N) v = p.Wu[(c - 9 * K1) % NU];
            if (v != 0) { P_x[pp] = v; P_i[pp] = c; ++pp; }
        }
        P_p[n] = pp;
        for (int c = 0; c < n; ++c) q[c] = 0;
        for (int k = 0; k < K1; ++k)
            for (int i = 0; i < 9; ++i) q[xi(k) + i] = sf(k, 9 + i);
        for (int k = 0; k < K1; ++k) q[ti(k)] = 1.0;
        // ---- A rows in the reference order
        std::vector<std::tuple<int, int, double>> tr;   // (col, row, val)
        int row = 0;
        const double inf = INFINITY;
        auto add = [&](int c, double v) { if (v != 0.0) tr.emplace_back(c, row, v); };
        for (int i = 0; i < 9; ++i, ++row) { add(xi(0) + i, 1.0); l[row] = u[row] = xb[i]; }
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < 9; ++i, ++row) {
                for (int j = 0; j < 9; ++j) add(xi(k) + j, A[(size_t)k * 81 + i * 9 + j]);
                for (int j = 0; j < NU; ++j) add(ui(k) + j, Bm[(size_t)k * 9 * NU + i * NU + j]);
                add(xi(k + 1) + i, -1.0);
                const double r = sf(k, i);
                l[row] = r - 1e-12; u[row] = r + 1e-12;
            }
        for (int i = 0; i < 9; ++i, ++row) { add(xi(N) + i, 1.0); l[row] = u[row] = xb[(size_t)N * 9 + i]; }
        if (h->robot == 1) {
            for (int c = 0; c < NC; ++c)
                for (int dd = 0; dd < 2; ++dd)
                    for (int k = 0; k < N; ++k, ++row) {
                        if (lg[(size_t)k * NC + c]) {
                            add(ui(k) + NUPC * c + dd, 1.0);
                            l[row] = -p.foot_range[dd == 0 ? 1 : 3];
                            u[row] = p.foot_range[dd == 0 ? 0 : 2];
                        } else { l[row] = 0; u[row] = 0; }
                    }
        }
        for (int c = 0; c < NC; ++c)
            for (int k = 0; k < N; ++k)
                for (int r = 0; r < 5; ++r, ++row) {
                    l[row] = -inf; u[row] = 0;
                    if (lg[(size_t)k * NC + c] && r < 4) {
                        const int cs = 32 + 32 * c;
                        for (int qq = 0; qq < 3; ++qq) add(ui(k) + NUPC * c + FO + qq, sf(k, cs + 4 + 3 * r + qq));
                        u[row] = sf(k, cs + 16 + r);
                    }
                }
        for (int k = 0; k < K1; ++k)
            for (int j = 0; j < 8; ++j, ++row) {
                for (int i = 0; i < 3; ++i) add(xi(k) + 6 + i, ((j >> i) & 1) ? -1.0 : 1.0);
                add(ti(k), cw);
                l[row] = -inf; u[row] = sf(k, 18 + j);
            }
        for (int k = 0; k < K1; ++k, ++row) { add(ti(k), -1.0); l[row] = -inf; u[row] = 0; }
        std::stable_sort(tr.begin(), tr.end(), [](auto &a, auto &c) {
            return std::get<0>(a) != std::get<0>(c) ? std::get<0>(a) < std::get<0>(c) : std::get<1>(a) < std::get<1>(c);
        });
        int ci = 0;
        for (size_t e = 0; e < tr.size(); ++e) {
            while (ci <= std::get<0>(tr[e])) A_p[ci++] = (int)e;
            A_x[e] = std::get<2>(tr[e]);
            A_i[e] = std::get<1>(tr[e]);
        }
        while (ci <= n) A_p[ci++] = (int)tr.size();
    });
}

int cmpc_get_qp_solution(cmpc_handle h, double *z, double *y, int32_t *status, int32_t *iters) {
    return guard(h, [&] {
        const int B = h->B, N = h->N, NC = h->NC, K1 = N + 1, NB = N + 2, NI = h->NI;
        const int n = 9 * K1 + NU * N + K1 + N;
        std::vector<double> xs, us, ts, nus, lams;
        auto dl = [&](std::vector<double> &dst, void *src, size_t cnt) {
            dst.resize(cnt);
            if (h->prec == CMPC_PREC_F64) from_dev<double>(h, dst.data(), src, cnt); else from_dev<float>(h, dst.data(), src, cnt);
        };
        if (z) {
            dl(xs, h->xs, (size_t)B * K1 * 9);
            dl(us, h->us, (size_t)B * N * NU);
            dl(ts, h->ts, (size_t)B * K1);
            for (int b = 0; b < B; ++b) {
                double *zb = z + (size_t)b * n;
                std::memcpy(zb, &xs[(size_t)b * K1 * 9], sizeof(double) * K1 * 9);
                std::memcpy(zb + 9 * K1, &us[(size_t)b * N * NU], sizeof(double) * N * NU);
                std::memcpy(zb + 9 * K1 + NU * N, &ts[(size_t)b * K1], sizeof(double) * K1);
                for (int k = 0; k < N; ++k) zb[9 * K1 + NU * N + K1 + k] = 0.0;
            }
        }
        if (y) {
            int32_t m = 0;
            cmpc_qp_sizes(h, nullptr, &m, nullptr, nullptr);
            dl(nus, h->nus, (size_t)B * NB * 9);
            dl(lams, h->lams, (size_t)B * K1 * NI);
            const int CP = 9 + 4 * NC;
            for (int b = 0; b < B; ++b) {
                double *yb = y + (size_t)b * m;
                const double *nb = &nus[(size_t)b * NB * 9];
                const double *lb = &lams[(size_t)b * K1 * NI];
                int row = 0;
                for (int i = 0; i < 9 * NB; ++i) {
                    // nus blocks: init | dyn 0..N-1 | final  == rows init, dyn, final
                    yb[row++] = nb[i];
                }
                if (h->robot == 1)
                    for (int c = 0; c < NC; ++c)
                        for (int dd = 0; dd < 2; ++dd)
                            for (int k = 0; k < N; ++k)
                                yb[row++] = lb[(size_t)k * NI + CP + 4 * c + 2 * dd] - lb[(size_t)k * NI + CP + 4 * c + 2 * dd + 1];
                for (int c = 0; c < NC; ++c)
                    for (int k = 0; k < N; ++k)
                        for (int r = 0; r < 5; ++r) yb[row++] = r < 4 ? lb[(size_t)k * NI + 9 + 4 * c + r] : 0.0;
                for (int k = 0; k < K1; ++k)
                    for (int j = 0; j < 8; ++j) yb[row++] = lb[(size_t)k * NI + j];
                for (int k = 0; k < K1; ++k) yb[row++] = lb[(size_t)k * NI + 8];
            }
        }
        if (status) from_dev_raw(h, status, h->qp_status, (size_t)B * 4);
        if (iters) from_dev_raw(h, iters, h->qp_iters, (size_t)B * 4);
    });
}

int cmpc_get_qp_info(cmpc_handle h, double *merit, int32_t *n_refine) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        if (h->prec == CMPC_PREC_F64) from_dev<double>(h, merit, h->qp_merit, h->B);
        else from_dev<float>(h, merit, h->qp_merit, h->B);
        if (n_refine) from_dev_raw(h, n_refine, h->qp_nref, (size_t)h->B * 4);
    });
}

int cmpc_get_qp_exit(cmpc_handle h, int32_t *tail_steps, int32_t *polish) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        if (tail_steps) from_dev_raw(h, tail_steps, h->qp_tail, (size_t)h->B * 4);
        if (polish) from_dev_raw(h, polish, h->qp_polish, (size_t)h->B * 4);
    });
}

int cmpc_get_solution(cmpc_handle h, double *X, double *U, double *K, double *Sigma, int32_t *n_accepted,
                      int32_t *iterations, int32_t *scp_status, double *weight, double *radius) {
    return guard(h, [&] {
        settle_all(h);
        const size_t B = h->B, N = h->N, K1 = N + 1, LS = (size_t)h->max_batch * N;
        // Everything is brought into the host layouts on the device first (fp64; K transposed to
        // knot-major; fp32 handles widened), then one batch of asynchronous copies and one
        // synchronization.  Destinations the caller pinned (cmpc_host_register) are written by DMA
        // at full link rate; pageable ones through the runtime's staging.  NULL skips an array.
        const size_t nX = B * K1 * 9, nU = B * N * NU, nK = B * N * NU * 9, nS = B * K1 * 81;
        const void *Ssrc = h->ks_live ? h->Sig : h->Sacc, *Ksrc = h->ks_live ? h->K : h->Kacc;
        // arrays the solve already streamed into these same buffers (cmpc_prefetch_ks): only wait
        bool waitK = false, waitS = false;
        if (K && h->pfK_issued && K == h->pf_K) { waitK = true; K = nullptr; }
        if (Sigma && h->pfS_issued && Sigma == h->pf_S) { waitS = true; Sigma = nullptr; }
        const bool f32 = h->prec == CMPC_PREC_F32;
        size_t need_el = K ? nK : 0;
        if (f32) need_el += (X ? nX : 0) + (U ? nU : 0) + (Sigma ? nS : 0);
        double *stg = need_el ? (double *)h->scratch_bytes_at_least(need_el * sizeof(double)) : nullptr;
        const double *srcX = (const double *)h->Xacc, *srcU = (const double *)h->Uacc, *srcS = (const double *)Ssrc,
                     *srcK = nullptr;
        size_t off = 0;
        auto widen = [&](const void *src, size_t n) {
            double *dst = stg + off;
            off += n;
            hipLaunchKernelGGL(k_widen, dim3((unsigned)std::min<size_t>((n + 255) / 256, 4096)), dim3(256), 0, h->stream,
                               (const float *)src, n, dst);
            return (const double *)dst;
        };
        if (K) {
            const dim3 grid((unsigned)((B * N + 31) / 32), (unsigned)((NU * 9 + 31) / 32));
            if (f32)
                hipLaunchKernelGGL((k_knot_major<float>), grid, dim3(256), 0, h->stream, (const float *)Ksrc, LS, (size_t)0,
                                   B * N, (int)(NU * 9), stg);
            else
                hipLaunchKernelGGL((k_knot_major<double>), grid, dim3(256), 0, h->stream, (const double *)Ksrc, LS, (size_t)0,
                                   B * N, (int)(NU * 9), stg);
            srcK = stg;
            off = nK;
        }
        if (f32) {
            if (X) srcX = widen(h->Xacc, nX);
            if (U) srcU = widen(h->Uacc, nU);
            if (Sigma) srcS = widen(Ssrc, nS);
        }
        HIPCHK(hipGetLastError());
        auto out = [&](double *dst, const double *src, size_t n) {
            if (dst && n) HIPCHK(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        };
        out(K, srcK, nK);
        out(X, srcX, nX);
        out(U, srcU, nU);
        out(Sigma, srcS, nS);
        std::vector<ScpState> st(B);
        HIPCHK(hipMemcpyAsync(st.data(), h->scp, B * sizeof(ScpState), hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        if (waitK) HIPCHK(hipEventSynchronize(h->ev_pfK));
        if (waitS) HIPCHK(hipEventSynchronize(h->ev_pfS));
        for (size_t b = 0; b < B; ++b) {
            if (n_accepted) n_accepted[b] = st[b].n_accepted;
            if (iterations) iterations[b] = st[b].iter;
            if (scp_status) scp_status[b] = st[b].status;
            if (weight) weight[b] = st[b].weight;
            if (radius) radius[b] = st[b].radius;
        }
    });
}

int cmpc_prefetch_ks(cmpc_handle h, double *K, double *Sigma) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        need(h->scp_mode == CMPC_SCP_MODE_REFERENCE && h->ks_live,
             "prefetch serves reference mode's live K / Sigma (upload first; not in GuSTO mode)");
        pf_disarm(h);
        h->pf_K = K;
        h->pf_S = Sigma;
        h->pf_armed = K || Sigma;
        // staging sized now, not inside the solve
        const size_t B = h->B, N = h->N;
        pf_staging(h, (B * N * NU * 9 + (h->prec == CMPC_PREC_F32 ? B * (N + 1) * 81 : 0)) * sizeof(double));
    });
}

int cmpc_host_register(cmpc_handle h, void *ptr, size_t bytes) {
    return guard(h, [&] {
        need(ptr != nullptr && bytes > 0, "invalid host range");
        HIPCHK(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    });
}

int cmpc_host_unregister(cmpc_handle h, void *ptr) {
    return guard(h, [&] {
        need(ptr != nullptr, "invalid host pointer");
        HIPCHK(hipHostUnregister(ptr));
    });
}

int cmpc_get_iteration_log(cmpc_handle h, double *tr_norm, double *rho, int32_t *qp_status, int32_t *qp_iters,
                           int32_t *decision) {
    return guard(h, [&] {
        auto st = get_scp(h);
        for (int b = 0; b < h->B; ++b) {
            if (tr_norm) tr_norm[b] = st[b].tr_norm;
            if (rho) rho[b] = st[b].rho;
            if (qp_status) qp_status[b] = st[b].qp_status;
            if (qp_iters) qp_iters[b] = st[b].qp_iters;
            if (decision) decision[b] = st[b].decision;
        }
    });
}

int cmpc_get_iteration_history(cmpc_handle h, int cap, cmpc_iter_record *records, int32_t *n_records) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        need(cap >= 1, "cap must be >= 1");
        auto st = get_scp(h);
        std::vector<cmpc_iter_record> all;
        if (h->log_cap > 0) {
            all.resize((size_t)h->B * h->log_cap);
            from_dev_raw(h, all.data(), h->hlog, all.size() * sizeof(cmpc_iter_record));
        }
        for (int b = 0; b < h->B; ++b) {
            const int n = std::min(std::min(st[b].iter, h->log_cap), cap);
            if (n_records) n_records[b] = n;
            if (!records) continue;
            for (int i = 0; i < cap; ++i) {
                cmpc_iter_record r{};
                if (i < n) r = all[(size_t)b * h->log_cap + i];
                records[(size_t)b * cap + i] = r;
            }
        }
    });
}

int cmpc_get_accepted(cmpc_handle h, int j, double *X, double *U, double *K, double *Sigma) {
    return guard(h, [&] {
        need(h->B > 0, "no problems uploaded");
        need(j >= 0, "accepted index must be >= 0");
        settle_all(h);
        const size_t B = h->B, N = h->N, K1 = N + 1, Bm = h->max_batch, e = h->esz();
        const size_t LS = Bm * N;
        auto st = get_scp(h);
        bool any = false;
        for (size_t b = 0; b < B; ++b) any |= j < st[b].n_accepted;
        need(!any || j < h->hist_cap, "accepted iterate beyond the kept history (max_iterations)");
        auto dl = [&](double *dst, void *src, size_t n) {
            if (h->prec == CMPC_PREC_F64) from_dev<double>(h, dst, src, n); else from_dev<float>(h, dst, src, n);
        };
        if (any) {
            dl(X, (char *)h->hX + (size_t)j * Bm * K1 * 9 * e, B * K1 * 9);
            dl(U, (char *)h->hU + (size_t)j * Bm * N * NU * e, B * N * NU);
            const bool gusto_ks = h->hks_cap > j && !h->ks_live && h->scp_mode == CMPC_SCP_MODE_GUSTO;
            // reference mode: the accepted K / Sigma are the fixed linearization point's (Q1)
            dl_knots(h, K, gusto_ks ? (char *)h->hK + (size_t)j * NU * 9 * LS * e : (h->ks_live ? h->K : h->Kacc), 0,
                     B * N, NU * 9);
            dl(Sigma, gusto_ks ? (char *)h->hS + (size_t)j * Bm * K1 * 81 * e : (h->ks_live ? h->Sig : h->Sacc),
               B * K1 * 81);
        }
        for (size_t b = 0; b < B; ++b) {
            if (any && j < st[b].n_accepted) continue;
            if (X) std::fill(X + b * K1 * 9, X + (b + 1) * K1 * 9, 0.0);
            if (U) std::fill(U + b * N * NU, U + (b + 1) * N * NU, 0.0);
            if (K) std::fill(K + b * N * NU * 9, K + (b + 1) * N * NU * 9, 0.0);
            if (Sigma) std::fill(Sigma + b * K1 * 81, Sigma + (b + 1) * K1 * 81, 0.0);
        }
    });
}

int cmpc_get_timing(cmpc_handle h, cmpc_timing *t) {
    return guard(h, [&] {
        need(t != nullptr, "null timing");
        need(h->timed, "no timed iteration yet");
        HIPCHK(hipEventSynchronize(h->ev[4]));
        float ms[4];
        for (int i = 0; i < 4; ++i) HIPCHK(hipEventElapsedTime(&ms[i], h->ev[i], h->ev[i + 1]));
        t->linearize_ms = ms[0]; t->assemble_ms = ms[1]; t->qp_ms = ms[2]; t->accept_ms = ms[3];
        HIPCHK(hipEventElapsedTime(&t->total_ms, h->ev[0], h->ev[4]));
    });
}

int cmpc_timing_begin(cmpc_handle h) {
    return guard(h, [&] {
        h->accumulate = true;
        h->ev_used = 0;
    });
}

int cmpc_timing_end(cmpc_handle h, cmpc_timing *t, int *n_iterations) {
    return guard(h, [&] {
        need(t != nullptr, "null timing");
        need(h->accumulate, "cmpc_timing_begin was not called");
        h->accumulate = false;
        cmpc_timing acc{0, 0, 0, 0, 0};
        for (size_t i = 0; i < h->ev_used; ++i) {
            auto &ev = h->ev_pool[i];
            HIPCHK(hipEventSynchronize(ev[4]));
            float ms[4], tot;
            for (int p = 0; p < 4; ++p) HIPCHK(hipEventElapsedTime(&ms[p], ev[p], ev[p + 1]));
            HIPCHK(hipEventElapsedTime(&tot, ev[0], ev[4]));
            acc.linearize_ms += ms[0]; acc.assemble_ms += ms[1]; acc.qp_ms += ms[2]; acc.accept_ms += ms[3];
            acc.total_ms += tot;
        }
        *t = acc;
        if (n_iterations) *n_iterations = (int)h->ev_used;
    });
}

int cmpc_get_qp_iterations_total(cmpc_handle h, int64_t *total) {
    return guard(h, [&] {
        need(total != nullptr, "null output");
        std::vector<int32_t> it(h->B);
        from_dev_raw(h, it.data(), h->qp_iters, (size_t)h->B * 4);
        int64_t s = 0;
        for (int v : it) s += v;
        *total = s;
    });
}

int cmpc_get_qp_kernel(cmpc_handle h, char *buf, int n) {
    return guard(h, [&] {
        need(buf != nullptr && n > 0, "null output");
        const int P = qp_group(h);
        const int tw = qp_split(h);
        const std::string s = P    ? "k_qp_group<" + std::to_string(P) + ">"
                              : tw ? "k_qp_ipm<" + std::to_string(qp_waves(h)) + ">+tail<" + std::to_string(tw) + ">"
                                   : "k_qp_ipm<" + std::to_string(qp_waves(h)) + ">";
        std::snprintf(buf, (size_t)n, "%s", s.c_str());
    });
}

int cmpc_debug_stamps(cmpc_handle h, uint64_t *out) {
    return guard(h, [&] {
        need(out != nullptr, "null output");
        from_dev_raw(h, out, h->stamps, (size_t)h->B * 16 * 8);
    });
}

}  // extern "C"
