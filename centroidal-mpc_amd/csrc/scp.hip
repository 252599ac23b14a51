// SCP accept/reject step for every problem (one workgroup per problem).
//
// Replaces the body of solve_scp after the QP (reference src/scp_solver.py:149-177):
//   * trust-region test ||X_sol - X_prev||_2 < radius with the SPECTRAL norm of the
//     9 x (N+1) difference (quirk Q6): sigma_max^2 = lambda_max(D D'), D D' 9x9 Gram matrix,
//     cyclic Jacobi eigenvalues (double);
//   * model accuracy rho = sum_k ||nl_k[6:] - lin_k[6:]||^2 / sum_k ||lin_k||^2 over k < N
//     (compute_model_accuracy :71-87, nonlinear rollout :243-255);
//   * GuSTO updates: radius *= beta_fail | accept (+ radius = min(beta_succ r, r0)) |
//     weight *= gamma_fail; QP failure ends the problem with status QP_FAILED (:146-148).
// The linearization point is never updated, exactly as in the reference (quirk Q1).
#include "common.hpp"

namespace cmpc {

enum { DEC_NONE = 0, DEC_ACCEPT = 1, DEC_REJECT_RHO = 2, DEC_REJECT_TR = 3, DEC_QP_FAILED = -1 };

// Largest eigenvalue of the symmetric positive semidefinite n x n matrix g (row-major, in LDS) by
// multisection on the wave: lane l tests the shift s_l = lo + (l + 1) (hi - lo) / 65 for
// s_l I - g positive definite (LDL' pivots all positive, i.e. s_l > lambda_max, Sylvester's
// inertia), and the lowest passing lane brackets lambda_max 65x tighter per round.  Start
// bracket: max diagonal <= lambda_max <= Gershgorin bound.  Every lane runs the same rounds on
// the same values, so the result is wave-uniform and deterministic; error ~ n eps ||g|| (the
// backward error of the LDL' inertia), like a converged Jacobi sweep.  Must be called by a
// whole 64-lane wave.
template <int n> __device__ double lambda_max_psd(const double *g) {
    const int lane = threadIdx.x & (WAVE - 1);
    double lo = 0.0, hi = 0.0;
    for (int i = 0; i < n; ++i) {
        double r = 0.0;
        for (int j = 0; j < n; ++j) r += fabs(g[i * n + j]);
        lo = fmax(lo, g[i * n + i]);
        hi = fmax(hi, r);
    }
    hi *= 1.0 + 4.0 * n * 2.3e-16;   // Gershgorin, rounded up
    for (int round = 0; round < 16 && hi - lo > 2.3e-16 * hi; ++round) {
        const double w = hi - lo;
        const double s = lo + w * (double(lane + 1) / 65.0);
        double c[n * (n + 1) / 2];   // upper triangle of s I - g, row-packed, eliminated in place
        auto at = [](int i, int j) { return i * n - i * (i - 1) / 2 + (j - i); };
#pragma unroll
        for (int i = 0; i < n; ++i)
#pragma unroll
            for (int j = i; j < n; ++j) c[at(i, j)] = (i == j ? s : 0.0) - g[i * n + j];
        bool pd = true;
#pragma unroll
        for (int k = 0; k < n; ++k) {
            const double piv = c[at(k, k)];
            pd = pd && piv > 0.0;
            const double inv = 1.0 / piv;
#pragma unroll
            for (int i = k + 1; i < n; ++i) {
                const double f = c[at(k, i)] * inv;
#pragma unroll
                for (int j = i; j < n; ++j) c[at(i, j)] = fma(-f, c[at(k, j)], c[at(i, j)]);
            }
        }
        const unsigned long long m = __ballot(pd);
        if (m == 0) {
            lo = lo + w * (64.0 / 65.0);
        } else {
            const int l = __ffsll((long long)m) - 1;
            hi = lo + w * (double(l + 1) / 65.0);
            if (l > 0) lo = lo + w * (double(l) / 65.0);
        }
    }
    return 0.5 * (lo + hi);
}

// Spectral norm of the (rows x cols) matrix V[c][r] - W[c][r] (W may be null): sqrt of the largest
// eigenvalue of the rows x rows Gram matrix.  Columns go through LDS in chunks of SN_CC (one
// coalesced pass over the contiguous V, W), each thread accumulates its Gram entries in column
// order; eigenvalue by multisection on the (single-wave) workgroup.
constexpr int SN_CC = 256;
template <int rows, typename T>
__device__ double spec_norm(const T *V, const T *W, int cols, double *gram, double *buf /* rows * SN_CC */) {
    constexpr int PER = (rows * rows + WAVE - 1) / WAVE;
    const int tid = threadIdx.x;
    double g[PER];
#pragma unroll
    for (int p = 0; p < PER; ++p) g[p] = 0.0;
    for (int c0 = 0; c0 < cols; c0 += SN_CC) {
        const int nc = min(SN_CC, cols - c0);
        const T *v = V + (size_t)c0 * rows, *w = W ? W + (size_t)c0 * rows : nullptr;
        for (int e = tid; e < nc * rows; e += WAVE) buf[e] = double(v[e]) - (w ? double(w[e]) : 0.0);
        __syncthreads();
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const int e = tid + p * WAVE;
            if (e < rows * rows) {
                const int i = e / rows, j = e % rows;
                for (int c = 0; c < nc; ++c) g[p] = fma(buf[c * rows + i], buf[c * rows + j], g[p]);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int p = 0; p < PER; ++p)
        if (tid + p * WAVE < rows * rows) gram[tid + p * WAVE] = g[p];
    __syncthreads();
    const double v = sqrt(fmax(lambda_max_psd<rows>(gram), 0.0));
    __syncthreads();   // gram is reused by the next call
    return v;
}

// x+ = x + dt F(x, u) for the knot-k contact data (integrate_model_one_step)
template <typename T, int ROBOT>
__device__ void step_dyn(const DevParams<T> &prm, const T *x, const T *u, const T *p, const T *R, const uint8_t *lg,
                         T *o) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    const T m = prm.mass;
    T F[9] = {(T(1) / m) * x[3], (T(1) / m) * x[4], (T(1) / m) * x[5], 0, 0, m * prm.gravity, 0, 0, 0};
    for (int c = 0; c < NC; ++c) {
        const T a = T(lg[c]);
        const T *f = u + NUPC * c + FO;
        T pc[3] = {p[3 * c] - x[0], p[3 * c + 1] - x[1], p[3 * c + 2] - x[2]};
        T v[3];
        cross3(pc, f, v);
        if (ROBOT == 1) {
            const T *Rc = R + 9 * c;
            const T *cp = u + NUPC * c;
            T q[3], w[3];
            for (int z = 0; z < 3; ++z) q[z] = Rc[z * 3] * cp[0] + Rc[z * 3 + 1] * cp[1];
            cross3(q, f, w);
            for (int z = 0; z < 3; ++z) v[z] += w[z] + Rc[z * 3 + 2] * cp[5];
        }
        for (int z = 0; z < 3; ++z) { F[3 + z] += a * f[z]; F[6 + z] += a * v[z]; }
    }
    for (int i = 0; i < 9; ++i) o[i] = x[i] + F[i] * prm.dt;
}

// one wave per problem: the kernel needs ~250 registers (the 9 x 9 Jacobi lives in them), and
// with 64-thread workgroups four problems still share a CU (a 256-thread workgroup ran one per CU)
constexpr int ACC_NT = 64;
constexpr int ACC_KC = 128, ACC_REC = 9 + 9 + NU;   // knots per rho chunk, LDS record per knot

// Linear prediction f + A dx + B du of knot kn (compute_model_accuracy, src/scp_solver.py:71-87),
// with A and B at the linearization point (xb, ub) in the closed form k_lin_knots uses
// (src/centroidal_model.py:230-232): A = [[I, beta I, 0], [0, I, 0], [[dt w]x, 0, I]], B from
// contact_B.  The sum runs in the dense product's order over its nonzero entries (a zero entry's
// fma is an exact no-op), so the prediction is bit-identical to f + A dx + B du with the dense
// arrays, which reference mode no longer stores.
template <typename T, int ROBOT>
__device__ __forceinline__ void lin_predict(const DevBuf<T> &d, const DevParams<T> &prm, size_t kn, const T *xb, const T *ub,
                                            const T *xs, const T *us, T *lin) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    T x[9], u[NU], dx[9], du[NU];
    for (int i = 0; i < 9; ++i) { x[i] = xb[i]; dx[i] = xs[i] - x[i]; }
    for (int i = 0; i < NU; ++i) { u[i] = ub[i]; du[i] = us[i] - u[i]; }
    const T *p = d.pos + kn * 3 * NC, *rot = d.rot + kn * 9 * NC;
    T a[NC], lev[NC][3], w[3] = {T(0), T(0), T(0)};
    for (int c = 0; c < NC; ++c) a[c] = T(d.logic[kn * NC + c]);
    for (int c = 0; c < NC; ++c)
        for (int z = 0; z < 3; ++z) {
            lev[c][z] = p[3 * c + z] - x[z];
            if (ROBOT == 1) lev[c][z] += rot[9 * c + z * 3] * u[NUPC * c] + rot[9 * c + z * 3 + 1] * u[NUPC * c + 1];
            w[z] = fma(a[c], u[NUPC * c + FO + z], w[z]);
        }
    const T dt = prm.dt, beta = dt / prm.mass;
    const T Wm[3][3] = {{T(0), -dt * w[2], dt * w[1]}, {dt * w[2], T(0), -dt * w[0]}, {-dt * w[1], dt * w[0], T(0)}};
    for (int i = 0; i < 9; ++i) lin[i] = d.f[(size_t)i * d.LS + kn];
    for (int i = 0; i < 3; ++i) lin[i] = fma(beta, dx[3 + i], lin[i] + dx[i]);     // j = i, then j = i + 3
    for (int i = 3; i < 6; ++i) lin[i] = lin[i] + dx[i];
    for (int i = 6; i < 9; ++i) {
        T v = lin[i];
        for (int j = 0; j < 3; ++j) v = fma(Wm[i - 6][j], dx[j], v);              // j < 3, then j = i
        lin[i] = v + dx[i];
    }
    for (int c = 0; c < NC; ++c) {
        ContactB<T, ROBOT> Bc;
        contact_B<T, ROBOT>(dt * a[c], lev[c], u + NUPC * c + FO, rot + 9 * c, Bc);
        for (int i = 3; i < 9; ++i)
            for (int q = 0; q < NUPC; ++q) lin[i] = fma(Bc.b[i - 3][q], du[NUPC * c + q], lin[i]);
    }
}

template <typename T, int ROBOT>
__global__ void __launch_bounds__(ACC_NT) k_accept(DevBuf<T> d, int fixed_iters) {
    constexpr int NC = Robot<ROBOT>::NC;
    const int b = blockIdx.x;
    if (b >= d.B) return;
    ScpState &sc = d.scp[b];
    if (!sc.active) {
        if (threadIdx.x == 0) sc.keep = 0;
        return;
    }
    __shared__ T red[2 * 4];
    __shared__ double gram[NU * NU];
    __shared__ double smem[ACC_KC * ACC_REC];   // rho records, then spectral-norm column chunks
    static_assert(NU * SN_CC <= ACC_KC * ACC_REC, "LDS");
    T *acc_sm = reinterpret_cast<T *>(smem);
    const int tid = threadIdx.x, N = d.N, K1 = N + 1;
    const DevParams<T> &prm = d.params[d.class_id[b]];
    const T *Xs = d.xs + (size_t)b * K1 * 9, *Us = d.us + (size_t)b * N * NU;
    // previous solution = the linearization point (the warm start in reference mode, quirk Q1)
    T *Xb = d.Xlin + (size_t)b * K1 * 9, *Ub = d.Ulin + (size_t)b * N * NU;
    const int qst = d.qp_status[b];
    // ---- rho (fp of the compute type), in two passes: per knot the nonlinear step and (dx, du)
    // into LDS, then per (knot, row) the linearized row from that row of A and B (neighbouring
    // threads read neighbouring rows: coalesced, where a thread per knot strides 648 B)
    T acc[2] = {T(0), T(0)};
    for (int k0 = 0; k0 < N; k0 += ACC_KC) {
        const int nk = min(ACC_KC, N - k0);
        for (int kk = tid; kk < nk; kk += ACC_NT) {
            const int k = k0 + kk;
            const size_t kn = (size_t)b * N + k;
            T *rec = acc_sm + kk * ACC_REC;   // nl (9) | lin (9)
            step_dyn<T, ROBOT>(prm, Xs + (size_t)k * 9, Us + (size_t)k * NU, d.pos + kn * 3 * NC, d.rot + kn * 9 * NC,
                               d.logic + kn * NC, rec);
            lin_predict<T, ROBOT>(d, prm, kn, Xb + (size_t)k * 9, Ub + (size_t)k * NU, Xs + (size_t)k * 9,
                                  Us + (size_t)k * NU, rec + 9);
        }
        __syncthreads();
        for (int p = tid; p < nk * 9; p += ACC_NT) {
            const int kk = p % nk, i = p / nk;
            const T *rec = acc_sm + kk * ACC_REC;
            const T lin = rec[9 + i];
            if (i >= 6) acc[0] += sq(rec[i] - lin);
            acc[1] += lin * lin;
        }
        __syncthreads();
    }
    block_reduce<T, ACC_NT, 2, 0>(acc, red);
    const double rho = double(acc[0]) / double(acc[1]);
    // ---- spectral norm of X_sol - X_prev (quirk Q6)
    const double tr = spec_norm<9>(Xs, Xb, K1, gram, smem);
    // ---- GuSTO mode: convergence(sol, lin) = |dU|_2 / |U|_2 + |dX|_2 / |X|_2 (src/scp_solver.py:51-56),
    // needed only when this iteration is accepted (evaluated for every problem, cheap)
    double conv = 0.0;
    if (d.scp_mode == CMPC_SCP_MODE_GUSTO) {
        const double nx = spec_norm<9>(Xs, (const T *)nullptr, K1, gram, smem);
        const double nu_d = spec_norm<NU>(Us, Ub, N, gram, smem);
        const double nu_n = spec_norm<NU>(Us, (const T *)nullptr, N, gram, smem);
        conv = nu_d / nu_n + tr / nx;
    }
    if (tid == 0) {
        int dec;
        const double w_it = sc.weight, r_it = sc.radius;   // the trust region this iteration's QP ran with
        sc.qp_status = qst;
        sc.qp_iters = d.qp_iters[b];
        sc.tr_norm = tr;
        sc.rho = rho;
        if (qst != 1) {
            dec = DEC_QP_FAILED;
            sc.success = 0;
        } else if (tr < sc.radius) {
            if (rho > prm.rho1) {
                sc.radius *= prm.beta_fail;
                sc.success = 0;
                dec = DEC_REJECT_RHO;
            } else {
                sc.success = 1;
                sc.n_accepted += 1;
                dec = DEC_ACCEPT;
                if (rho < prm.rho0) sc.radius = fmin(prm.beta_succ * sc.radius, prm.tr_radius0);
            }
        } else {
            sc.weight *= prm.gamma_fail;
            sc.success = 0;
            dec = DEC_REJECT_TR;
        }
        sc.decision = dec;
        if (d.hlog && sc.iter < d.log_cap) {
            cmpc_iter_record rec;
            rec.weight = w_it; rec.radius = r_it; rec.tr_norm = tr;
            rec.rho = (dec == DEC_ACCEPT || dec == DEC_REJECT_RHO) ? rho : __builtin_nan("");
            rec.iteration = sc.iter; rec.qp_status = qst; rec.qp_iters = sc.qp_iters; rec.decision = dec;
            d.hlog[(size_t)b * d.log_cap + sc.iter] = rec;
        }
        sc.iter += 1;
        if (dec == DEC_QP_FAILED) {
            sc.status = CMPC_SCP_QP_FAILED;
            if (!fixed_iters) sc.active = 0;
        } else if (!fixed_iters) {
            // loop condition of src/scp_solver.py:132-133; reference mode: convergence == 0 (Q1)
            if (dec == DEC_ACCEPT) sc.conv = conv;
            const bool conv_ok = d.scp_mode == CMPC_SCP_MODE_GUSTO ? sc.conv < prm.conv_thr : 0.0 < prm.conv_thr;
            const bool cont = sc.iter < prm.max_iterations && sc.weight < prm.omega_max &&
                              !(sc.iter != 0 && sc.success && conv_ok);
            if (!cont) {
                sc.active = 0;
                sc.status = sc.success ? CMPC_SCP_CONVERGED : CMPC_SCP_MAX_ITER;
            }
        } else {
            if (dec == DEC_ACCEPT) sc.conv = conv;
            if (sc.status == CMPC_SCP_RUNNING && sc.success) sc.status = CMPC_SCP_CONVERGED;
        }
        sc.keep = dec == DEC_ACCEPT;
    }
}

// Accepted iterations keep X, U and (d.copy_ks) this iteration's LQR gains / covariances (and, GuSTO
// mode, become the linearization point): a grid over (element chunk, problem), so the ~170 KB per
// accepted problem stream at HBM rate (one wave per problem copying them latency-bound took
// ~200 us per SCP iteration at batch 1024, N = 100).  In reference mode the gains and covariances
// are served from the live arrays (cmpc_handle_::ks_live) and only X, U are copied.
template <typename T>
__global__ void __launch_bounds__(256) k_keep_accepted(DevBuf<T> d) {
    const int b = blockIdx.y;
    if (b >= d.B || !d.scp[b].keep) return;
    const int N = d.N, K1 = N + 1;
    const int nx = K1 * 9, nu = N * NU, nk = N * NU * 9, ns = K1 * 81;
    const bool gusto = d.scp_mode == CMPC_SCP_MODE_GUSTO;
    const T *Xs = d.xs + (size_t)b * nx, *Us = d.us + (size_t)b * nu;
    const int ne = nx + nu + (d.copy_ks ? nk + ns : 0);
    // history slot of this accept (the reference appends every accepted iterate)
    const int slot = d.scp[b].n_accepted - 1;
    const bool hist = d.hX && slot >= 0 && slot < d.hist_cap;
    const size_t Bm = d.LS / N;   // max_batch
    for (int e = blockIdx.x * 256 + threadIdx.x; e < ne; e += gridDim.x * 256) {
        if (e < nx) {
            const T v = Xs[e];
            d.Xacc[(size_t)b * nx + e] = v;
            if (gusto) d.Xlin[(size_t)b * nx + e] = v;
            if (hist) d.hX[((size_t)slot * Bm + b) * nx + e] = v;
        } else if (e < nx + nu) {
            const int i = e - nx;
            const T v = Us[i];
            d.Uacc[(size_t)b * nu + i] = v;
            if (gusto) d.Ulin[(size_t)b * nu + i] = v;
            if (hist) d.hU[((size_t)slot * Bm + b) * nu + i] = v;
        } else if (e < nx + nu + nk) {   // element-major, like K
            const int i = e - nx - nu;
            const size_t j = (size_t)(i / N) * d.LS + (size_t)b * N + i % N;
            const T v = d.K[j];
            d.Kacc[j] = v;
            if (hist && d.hK) d.hK[(size_t)slot * (NU * 9) * d.LS + j] = v;
        } else {
            const size_t j = (size_t)b * ns + (e - nx - nu - nk);
            const T v = d.Sig[j];
            d.Sacc[j] = v;
            if (hist && d.hS) d.hS[(size_t)slot * Bm * ns + j] = v;
        }
    }
}

// Knots [kn0, kn0 + n) of an element-major array (element e of knot k at e * LS + k) into a
// knot-major fp64 copy dst[k][e] for the host getters: 32 x 32 tiles through LDS, so both the
// knot-contiguous reads and the element-contiguous writes are coalesced.
template <typename T>
__global__ void __launch_bounds__(256) k_knot_major(const T *src, size_t LS, size_t kn0, size_t n, int ne,
                                                    double *dst) {
    __shared__ double tile[32][33];
    const size_t k0 = (size_t)blockIdx.x * 32;
    const int e0 = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int r = ty; r < 32; r += 8) {
        const int e = e0 + r;
        const size_t k = k0 + tx;
        if (e < ne && k < n) tile[r][tx] = double(src[(size_t)e * LS + kn0 + k]);
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const size_t k = k0 + r;
        const int e = e0 + tx;
        if (e < ne && k < n) dst[k * ne + e] = tile[tx][r];
    }
}

// interpolate_SCP_solution (src/scp_solver.py:95-111) of the accepted solution, one thread per
// (problem, output column, row): column i * ni + j = v_i + j * ((v_{i+1} - v_i) / ni).
// X_out (B, 9, N * ni), U_out (B, nu, (N - 1) * ni), nu = nu_out (reference control width).
template <typename T>
__global__ void __launch_bounds__(256) k_interpolate(DevBuf<T> d, int ni, int nu_out, T *Xo, T *Uo) {
    const int N = d.N, cx = N * ni, cu = (N - 1) * ni;
    const long per = 9L * cx + (long)nu_out * cu;
    const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (long)d.B * per) return;
    const int b = (int)(g / per);
    long e = g % per;
    if (e < 9L * cx) {
        const int r = (int)(e / cx), col = (int)(e % cx), i = col / ni, j = col % ni;
        const T *X = d.Xacc + (size_t)b * (N + 1) * 9;
        const T v0 = X[(size_t)i * 9 + r], v1 = X[(size_t)(i + 1) * 9 + r];
        Xo[(size_t)b * 9 * cx + e] = v0 + T(j) * ((v1 - v0) / T(ni));
    } else {
        e -= 9L * cx;
        const int r = (int)(e / cu), col = (int)(e % cu), i = col / ni, j = col % ni;
        const T *U = d.Uacc + (size_t)b * N * NU;
        const T v0 = U[(size_t)i * NU + r], v1 = U[(size_t)(i + 1) * NU + r];
        Uo[(size_t)b * nu_out * cu + e] = v0 + T(j) * ((v1 - v0) / T(ni));
    }
}
template __global__ void k_interpolate<double>(DevBuf<double>, int, int, double *, double *);
template __global__ void k_interpolate<float>(DevBuf<float>, int, int, float *, float *);

// nonlinear rollout x+_k = x_k + dt F(x_k, u_k) along (X, U) for k = 0..N (reference
// integrate_dynamics_trajectory, src/centroidal_model.py:243-255; at k = N the reference's JAX
// gathers clamp to the last control / contact row, quirk Q9).  One thread per (problem, knot).
template <typename T, int ROBOT>
__global__ void __launch_bounds__(128) k_rollout(DevBuf<T> d, const T *X, const T *U, T *out) {
    constexpr int NC = Robot<ROBOT>::NC;
    const int N = d.N, K1 = N + 1;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)d.B * K1) return;
    const int b = (int)(i / K1), k = (int)(i % K1), kc = k < N ? k : N - 1;
    const size_t kn = (size_t)b * N + kc;
    step_dyn<T, ROBOT>(d.params[d.class_id[b]], X + (size_t)i * 9, U + kn * NU, d.pos + kn * 3 * NC, d.rot + kn * 9 * NC,
                       d.logic + kn * NC, out + (size_t)i * 9);
}

template __global__ void k_rollout<double, 0>(DevBuf<double>, const double *, const double *, double *);
template __global__ void k_rollout<double, 1>(DevBuf<double>, const double *, const double *, double *);
template __global__ void k_rollout<float, 0>(DevBuf<float>, const float *, const float *, float *);
template __global__ void k_rollout<float, 1>(DevBuf<float>, const float *, const float *, float *);

// fp32 handles: widen n values into the fp64 staging buffer of a getter (coalesced, grid-stride)
__global__ void __launch_bounds__(256) k_widen(const float *src, size_t n, double *dst) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = double(src[i]);
}

template __global__ void k_knot_major<double>(const double *, size_t, size_t, size_t, int, double *);
template __global__ void k_knot_major<float>(const float *, size_t, size_t, size_t, int, double *);
template __global__ void k_keep_accepted<double>(DevBuf<double>);
template __global__ void k_keep_accepted<float>(DevBuf<float>);
template __global__ void k_accept<double, 0>(DevBuf<double>, int);
template __global__ void k_accept<double, 1>(DevBuf<double>, int);
template __global__ void k_accept<float, 0>(DevBuf<float>, int);
template __global__ void k_accept<float, 1>(DevBuf<float>, int);

}  // namespace cmpc
