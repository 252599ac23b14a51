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

// Largest eigenvalue of the symmetric n x n matrix a (row-major, in LDS: rotations index it at run
// time, which would put a private array in scratch memory), cyclic Jacobi on one thread.
template <int n> __device__ double jacobi_lambda_max(double *a_) {
    auto a = [&](int i, int j) -> double & { return a_[i * n + j]; };
    for (int sweep = 0; sweep < 40; ++sweep) {
        double off = 0.0, tot = 0.0;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                tot += a(i, j) * a(i, j);
                if (i != j) off += a(i, j) * a(i, j);
            }
        if (off <= 1e-30 * tot || off == 0.0) break;
        for (int p = 0; p < n - 1; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = a(p, q);
                if (apq == 0.0) continue;
                const double theta = (a(q, q) - a(p, p)) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; ++k) {
                    const double akp = a(k, p), akq = a(k, q);
                    a(k, p) = c * akp - s * akq;
                    a(k, q) = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = a(p, k), aqk = a(q, k);
                    a(p, k) = c * apk - s * aqk;
                    a(q, k) = s * apk + c * aqk;
                }
            }
    }
    double m = a(0, 0);
    for (int i = 1; i < n; ++i) m = fmax(m, a(i, i));
    return m;
}

// The same in registers for small n: every rotation loop unrolled so all indices are constants
// (the matrix lives in VGPRs; LDS or scratch put a ~100-cycle access in every dependent step)
template <int n> __device__ double jacobi_lambda_max_reg(const double *g) {
    double a[n][n];
#pragma unroll
    for (int i = 0; i < n; ++i)
#pragma unroll
        for (int j = 0; j < n; ++j) a[i][j] = g[i * n + j];
    for (int sweep = 0; sweep < 40; ++sweep) {
        double off = 0.0, tot = 0.0;
#pragma unroll
        for (int i = 0; i < n; ++i)
#pragma unroll
            for (int j = 0; j < n; ++j) {
                tot += a[i][j] * a[i][j];
                if (i != j) off += a[i][j] * a[i][j];
            }
        if (off <= 1e-30 * tot || off == 0.0) break;
#pragma unroll
        for (int p = 0; p < n - 1; ++p)
#pragma unroll
            for (int q = p + 1; q < n; ++q) {
                const double apq = a[p][q];
                // apq == 0: identity rotation (c = 1, s = 0), kept branch-free
                const double theta = (a[q][q] - a[p][p]) / (2.0 * (apq != 0.0 ? apq : 1.0));
                const double t0 = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double t = apq != 0.0 ? t0 : 0.0;
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
                for (int k = 0; k < n; ++k) {
                    const double akp = a[k][p], akq = a[k][q];
                    a[k][p] = c * akp - s * akq;
                    a[k][q] = s * akp + c * akq;
                }
#pragma unroll
                for (int k = 0; k < n; ++k) {
                    const double apk = a[p][k], aqk = a[q][k];
                    a[p][k] = c * apk - s * aqk;
                    a[q][k] = s * apk + c * aqk;
                }
            }
    }
    double m = a[0][0];
#pragma unroll
    for (int i = 1; i < n; ++i) m = fmax(m, a[i][i]);
    return m;
}

// Spectral norm of the (rows x cols) matrix V[c][r] - W[c][r] (W may be null): sqrt of the largest
// eigenvalue of the rows x rows Gram matrix, accumulated over the workgroup (Gram entry per
// thread), Jacobi on thread 0.  All threads receive the value.
template <int rows, typename T>
__device__ double spec_norm(const T *V, const T *W, int cols, double *gram, double *res) {
    const int tid = threadIdx.x;
    for (int e = tid; e < rows * rows; e += blockDim.x) {
        const int i = e / rows, j = e % rows;
        double g = 0.0;
        for (int c = 0; c < cols; ++c) {
            const double vi = double(V[(size_t)c * rows + i]) - (W ? double(W[(size_t)c * rows + i]) : 0.0);
            const double vj = double(V[(size_t)c * rows + j]) - (W ? double(W[(size_t)c * rows + j]) : 0.0);
            g += vi * vj;
        }
        gram[e] = g;
    }
    __syncthreads();
    if (tid == 0) {
        if constexpr (rows <= 9) *res = sqrt(fmax(jacobi_lambda_max_reg<rows>(gram), 0.0));
        else *res = sqrt(fmax(jacobi_lambda_max<rows>(gram), 0.0));   // in place (LDS)
    }
    __syncthreads();
    return *res;
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

template <typename T, int ROBOT>
__global__ void __launch_bounds__(ACC_NT) k_accept(DevBuf<T> d, int fixed_iters) {
    constexpr int NC = Robot<ROBOT>::NC;
    const int b = blockIdx.x;
    if (b >= d.B) return;
    ScpState &sc = d.scp[b];
    if (!sc.active) return;
    __shared__ T red[2 * 4];
    __shared__ double gram[NU * NU], nres[4];
    __shared__ T acc_sm[ACC_KC * ACC_REC];
    __shared__ int dec_sh;
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
            T *rec = acc_sm + kk * ACC_REC;   // nl (9) | dx (9) | du (NU)
            step_dyn<T, ROBOT>(prm, Xs + (size_t)k * 9, Us + (size_t)k * NU, d.pos + kn * 3 * NC, d.rot + kn * 9 * NC,
                               d.logic + kn * NC, rec);
            for (int i = 0; i < 9; ++i) rec[9 + i] = Xs[(size_t)k * 9 + i] - Xb[(size_t)k * 9 + i];
            for (int i = 0; i < NU; ++i) rec[18 + i] = Us[(size_t)k * NU + i] - Ub[(size_t)k * NU + i];
        }
        __syncthreads();
        for (int p = tid; p < nk * 9; p += ACC_NT) {
            const int kk = p % nk, i = p / nk;   // neighbouring threads: neighbouring knots (element-major arrays)
            const size_t kn = (size_t)b * N + k0 + kk;
            const T *rec = acc_sm + kk * ACC_REC;
            const T *Ar = d.A + (size_t)(i * 9) * d.LS + kn, *Br = d.Bu + (size_t)(i * NU) * d.LS + kn;
            T lin = d.f[(size_t)i * d.LS + kn];
            for (int j = 0; j < 9; ++j) lin = fma(Ar[(size_t)j * d.LS], rec[9 + j], lin);
            for (int j = 0; j < NU; ++j) lin = fma(Br[(size_t)j * d.LS], rec[18 + j], lin);
            if (i >= 6) acc[0] += sq(rec[i] - lin);
            acc[1] += lin * lin;
        }
        __syncthreads();
    }
    block_reduce<T, ACC_NT, 2, 0>(acc, red);
    const double rho = double(acc[0]) / double(acc[1]);
    // ---- spectral norm of X_sol - X_prev (quirk Q6)
    const double tr = spec_norm<9>(Xs, Xb, K1, gram, &nres[0]);
    // ---- GuSTO mode: convergence(sol, lin) = |dU|_2 / |U|_2 + |dX|_2 / |X|_2 (src/scp_solver.py:51-56),
    // needed only when this iteration is accepted (evaluated for every problem, cheap)
    double conv = 0.0;
    if (d.scp_mode == CMPC_SCP_MODE_GUSTO) {
        const double nx = spec_norm<9>(Xs, (const T *)nullptr, K1, gram, &nres[1]);
        const double nu_d = spec_norm<NU>(Us, Ub, N, gram, &nres[2]);
        const double nu_n = spec_norm<NU>(Us, (const T *)nullptr, N, gram, &nres[3]);
        conv = nu_d / nu_n + tr / nx;
    }
    if (tid == 0) {
        int dec;
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
        dec_sh = dec;
    }
    __syncthreads();
    if (dec_sh != DEC_ACCEPT) return;
    // accepted: keep X, U and this iteration's LQR gains / covariances
    for (int e = tid; e < K1 * 9; e += ACC_NT) d.Xacc[(size_t)b * K1 * 9 + e] = Xs[e];
    for (int e = tid; e < N * NU; e += ACC_NT) d.Uacc[(size_t)b * N * NU + e] = Us[e];
    for (int e = tid; e < N * NU * 9; e += ACC_NT) {   // element-major K -> the knot-major accepted copy
        const int q = e / N, k = e % N;
        d.Kacc[((size_t)b * N + k) * NU * 9 + q] = d.K[(size_t)q * d.LS + (size_t)b * N + k];
    }
    for (int e = tid; e < K1 * 81; e += ACC_NT) d.Sacc[(size_t)b * K1 * 81 + e] = d.Sig[(size_t)b * K1 * 81 + e];
    if (d.scp_mode == CMPC_SCP_MODE_GUSTO) {   // the accepted solution becomes the linearization point
        for (int e = tid; e < K1 * 9; e += ACC_NT) Xb[e] = Xs[e];
        for (int e = tid; e < N * NU; e += ACC_NT) Ub[e] = Us[e];
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

template __global__ void k_accept<double, 0>(DevBuf<double>, int);
template __global__ void k_accept<double, 1>(DevBuf<double>, int);
template __global__ void k_accept<float, 0>(DevBuf<float>, int);
template __global__ void k_accept<float, 1>(DevBuf<float>, int);

}  // namespace cmpc
