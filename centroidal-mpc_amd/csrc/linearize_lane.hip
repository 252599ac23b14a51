// Linearization with one knot per lane (the default path; diagonal LQR weight R, as in every
// reference config): f, A, B, C (closed form), the LQR gain K of two Riccati steps from P = Q, and
// the covariance-scan helpers Acl = A + B K, Qw = C W C' + eta, all in one lane's registers.
//
// Replaces Centroidal_model.compute_everything / integrate_model_one_step (reference
// src/centroidal_model.py:189-241, compute_lqr_feedback_gains :217-228): every knot of every
// problem is independent, so the wave holds 64 knots and every lane runs the same straight-line
// program on its own knot (no LDS, no barriers).  The Riccati step is taken in information form,
// which only inverts 9x9 SPD matrices instead of the reference's 12x12 R + B'PB:
//   P+ = Q + A' P A - A'PB (R + B'PB)^-1 B'PA = Q + A' N^-1 A,   N = P^-1 + B R^-1 B'
//   K  = -(R + B'P2 B)^-1 B'P2 A = -R^-1 B' N2^-1 A
// (Woodbury / push-through identities; B has rows 3..8 only, so B R^-1 B' is a 6x6 block G).
// A = [[I, beta I, 0], [0, I, 0], [W, 0, I]] (beta = dt/m, W = dt [sum a_i f_i]x) is used through
// its block structure, never as a dense matrix.  The covariance scan itself (sequential over the
// knots) runs in k_cov_scan, one wave per problem on the matrix cores.
//
// The kernel also writes the parts of the QP stage record that depend only on the linearization
// (dynamics rhs r_k = A xbar + B ubar - f, the compact A and B data, the friction rows G), which
// k_assemble computed from these arrays before; k_assemble<.., false> then adds the fields that
// depend on the SCP state (trust-region bounds and weight, tracking gradient, chance back-off).
// Outputs are element-major (DevBuf::LS): lane kn writes element e at e * LS + kn, so every store
// of the wave is one contiguous 512-B (fp64) transaction.
//
// Non-diagonal R falls back to k_linearize (linearize.hip), which works with R + B'PB directly.
#include "common.hpp"
#include "cov_scan.hpp"

namespace cmpc {

__device__ __forceinline__ constexpr int sp9(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

template <typename T> __device__ __forceinline__ T rcp_l(T p) {
    T r;
    if constexpr (sizeof(T) == 8) r = __builtin_amdgcn_rcp(p); else r = __builtin_amdgcn_rcpf(p);
    r = fma(r, fma(-p, r, T(1)), r);
    return fma(r, fma(-p, r, T(1)), r);
}

// Inverse of a 9x9 SPD matrix (packed lower, sp9) by Cholesky: M^-1 = L^-T L^-1.  In registers,
// fully unrolled (compile-time indices).
template <typename T> __device__ __forceinline__ void inv_spd9(const T (&m)[45], T (&out)[45]) {
    T L[45], id[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        T d = m[sp9(j, j)];
#pragma unroll
        for (int q = 0; q < j; ++q) d = fma(-L[sp9(j, q)], L[sp9(j, q)], d);
        const T ljj = sqrt(d);
        id[j] = rcp_l(ljj);
        L[sp9(j, j)] = ljj;
#pragma unroll
        for (int i = j + 1; i < 9; ++i) {
            T v = m[sp9(i, j)];
#pragma unroll
            for (int q = 0; q < j; ++q) v = fma(-L[sp9(i, q)], L[sp9(j, q)], v);
            L[sp9(i, j)] = v * id[j];
        }
    }
    T Li[45];   // L^-1, lower
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        Li[sp9(j, j)] = id[j];
#pragma unroll
        for (int i = j + 1; i < 9; ++i) {
            T v = T(0);
#pragma unroll
            for (int k = j; k < i; ++k) v = fma(L[sp9(i, k)], Li[sp9(k, j)], v);
            Li[sp9(i, j)] = -v * id[i];
        }
    }
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
            T v = T(0);
#pragma unroll
            for (int k = i; k < 9; ++k) v = fma(Li[sp9(k, i)], Li[sp9(k, j)], v);
            out[sp9(i, j)] = v;
        }
}

// Column j of M A (row k), for the centroidal A: column block c: M[:,c] + M[:,L] W; block l:
// beta M[:,c] + M[:,l]; block L: M[:,L].  Wm = W (3x3, dt [w]x).
template <typename T>
__device__ __forceinline__ T MA_at(const T (&M)[45], T beta, const T (&Wm)[3][3], int k, int j) {
    if (j < 3) return M[sp9(k, j)] + M[sp9(k, 6)] * Wm[0][j] + M[sp9(k, 7)] * Wm[1][j] + M[sp9(k, 8)] * Wm[2][j];
    if (j < 6) return fma(beta, M[sp9(k, j - 3)], M[sp9(k, j)]);
    return M[sp9(k, j)];
}

// out = Q + A' M A (packed lower; Q diagonal-or-dense from the parameters)
template <typename T>
__device__ __forceinline__ void atma(const T (&M)[45], T beta, const T (&Wm)[3][3], const T *Q, T (&out)[45]) {
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
            const int rb = i / 3, ii = i % 3;
            T v;
            if (rb == 0)
                v = MA_at(M, beta, Wm, ii, j) + Wm[0][ii] * MA_at(M, beta, Wm, 6, j) + Wm[1][ii] * MA_at(M, beta, Wm, 7, j) +
                    Wm[2][ii] * MA_at(M, beta, Wm, 8, j);
            else if (rb == 1)
                v = fma(beta, MA_at(M, beta, Wm, ii, j), MA_at(M, beta, Wm, 3 + ii, j));
            else
                v = MA_at(M, beta, Wm, 6 + ii, j);
            out[sp9(i, j)] = v + Q[i * 9 + j];
        }
}

template <typename T, int ROBOT>
__global__ void __launch_bounds__(256, 1) k_lin_knots(DevBuf<T> d, int only_active, int dense) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO, NW = 3 * NC;
    const int N = d.N;
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)d.B * N) return;
    const int b = (int)(t / N), k = (int)(t % N);
    if (only_active && !d.scp[b].active) return;
    const DevParams<T> &prm = d.params[d.class_id[b]];
    const size_t kn = (size_t)b * N + k;
    // ---- inputs of the knot (the linearization point and the contact data)
    T x[9], u[NU], p[3 * NC], rot[9 * NC], a[NC];
    const T *xs = d.Xlin + ((size_t)b * (N + 1) + k) * 9, *us = d.Ulin + kn * NU;
#pragma unroll
    for (int i = 0; i < 9; ++i) x[i] = xs[i];
#pragma unroll
    for (int i = 0; i < NU; ++i) u[i] = us[i];
#pragma unroll
    for (int i = 0; i < 3 * NC; ++i) p[i] = d.pos[kn * 3 * NC + i];
#pragma unroll
    for (int i = 0; i < 9 * NC; ++i) rot[i] = d.rot[kn * 9 * NC + i];
#pragma unroll
    for (int c = 0; c < NC; ++c) a[c] = T(d.logic[kn * NC + c]);
    const T dt = prm.dt, m = prm.mass, beta = dt / m;
    // levers: p_c - com (+ R_c[:, 0:2] cop_c for TALOS)
    T lev[NC][3], w[3] = {T(0), T(0), T(0)};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
#pragma unroll
        for (int z = 0; z < 3; ++z) {
            lev[c][z] = p[3 * c + z] - x[z];
            if (ROBOT == 1) lev[c][z] += rot[9 * c + z * 3] * u[NUPC * c] + rot[9 * c + z * 3 + 1] * u[NUPC * c + 1];
            w[z] = fma(a[c], u[NUPC * c + FO + z], w[z]);
        }
    }
    auto em = [&](T *base, int e) -> T & { return base[(size_t)e * d.LS + kn]; };
    using St = Stage<ROBOT>;
    const SV<T> st{d.stage + (size_t)b * St::SIZE * KPC + k};   // field-major stage record (common.hpp)
    T fx[9];
    // ---- f = x + dt F(x, u)   (src/centroidal_model.py:189-212)
    {
        T F[9];
#pragma unroll
        for (int i = 0; i < 3; ++i) F[i] = (T(1) / m) * x[3 + i];
#pragma unroll
        for (int i = 0; i < 3; ++i) F[3 + i] = w[i];
        F[5] += m * prm.gravity;
#pragma unroll
        for (int r = 0; r < 3; ++r) F[6 + r] = T(0);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const T *f = u + NUPC * c + FO;
            T lf[3];
            cross3(lev[c], f, lf);
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                T v = lf[r];
                if (ROBOT == 1) v += rot[9 * c + r * 3 + 2] * u[NUPC * c + 5];
                F[6 + r] = fma(a[c], v, F[6 + r]);
            }
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) fx[i] = x[i] + F[i] * dt;
#pragma unroll
        for (int i = 0; i < 9; ++i) em(d.f, i) = fx[i];
    }
    const T Wm[3][3] = {{T(0), -dt * w[2], dt * w[1]}, {dt * w[2], T(0), -dt * w[0]}, {-dt * w[1], dt * w[0], T(0)}};
    // ---- A, B, C (jacfwd at :230-232), closed form, and the linearization part of the stage record.
    // The dense A, B, C are stored only with `dense` (GuSTO mode, or on demand for the getters): the
    // QP takes its dynamics from the stage record and k_accept's linear prediction recomputes the
    // same closed form, so in reference mode the SCP loop never reads them.
    {
#pragma unroll
        for (int i = 0; i < 9; ++i)
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                T v = (i == j) ? T(1) : T(0);
                if (i < 3 && j == i + 3) v = beta;
                if (i >= 6 && j < 3) v = Wm[i - 6][j];
                if (dense) em(d.A, i * 9 + j) = v;
            }
        // r_k = A xbar + B ubar - f (src/constraints.py:36-45)
        T r[9];
#pragma unroll
        for (int i = 0; i < 3; ++i) r[i] = fma(beta, x[3 + i], x[i]);
#pragma unroll
        for (int i = 3; i < 6; ++i) r[i] = x[i];
#pragma unroll
        for (int i = 6; i < 9; ++i) r[i] = x[i] + Wm[i - 6][0] * x[0] + Wm[i - 6][1] * x[1] + Wm[i - 6][2] * x[2];
        const T ml = prm.mu / sqrt(T(2));
        const T Fmu[4][3] = {{1, 0, -ml}, {-1, 0, -ml}, {0, 1, -ml}, {0, -1, -ml}};
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            ContactB<T, ROBOT> Bc;
            contact_B<T, ROBOT>(dt * a[c], lev[c], u + NUPC * c + FO, rot + 9 * c, Bc);
#pragma unroll
            for (int i = 0; i < 9; ++i)
#pragma unroll
                for (int q = 0; q < NUPC; ++q)
                    if (dense) em(d.Bu, i * NU + NUPC * c + q) = i < 3 ? T(0) : Bc.b[i - 3][q];
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
                for (int q = 0; q < NUPC; ++q) r[3 + i] = fma(Bc.b[i][q], u[NUPC * c + q], r[3 + i]);
            const T *f = u + NUPC * c + FO;
            const T fs[3][3] = {{T(0), -f[2], f[1]}, {f[2], T(0), -f[0]}, {-f[1], f[0], T(0)}};
#pragma unroll
            for (int i = 0; i < 9; ++i)
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    if (dense) em(d.C, i * NW + 3 * c + q) = i < 6 ? T(0) : -dt * a[c] * fs[i - 6][q];
            // per-contact stage fields: alpha, lever, friction rows (F_mu R')[0:4], TALOS cop / tau columns
            const SV<T> cs = st + (St::CON + St::CS * c);
            cs[St::ALPHA] = dt * a[c];
#pragma unroll
            for (int z = 0; z < 3; ++z) cs[St::LEVER + z] = lev[c][z];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    cs[St::G + rr * 3 + q] = Fmu[rr][0] * rot[9 * c + q * 3] + Fmu[rr][1] * rot[9 * c + q * 3 + 1] +
                                             Fmu[rr][2] * rot[9 * c + q * 3 + 2];
            if (ROBOT == 1) {
#pragma unroll
                for (int rr = 0; rr < 3; ++rr) {
                    cs[St::BCOP + rr * 2] = Bc.b[3 + rr][0];
                    cs[St::BCOP + rr * 2 + 1] = Bc.b[3 + rr][1];
                    cs[St::BTAU + rr] = Bc.b[3 + rr][5];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) st[St::R + i] = r[i] - fx[i];
#pragma unroll
        for (int q = 0; q < 3; ++q) st[St::W + q] = dt * w[q];
    }
    // ---- G = B R^-1 B' (rows 3..8), R diagonal
    T G[21];   // packed lower 6x6
#pragma unroll
    for (int e = 0; e < 21; ++e) G[e] = T(0);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        ContactB<T, ROBOT> Bc;
        contact_B<T, ROBOT>(dt * a[c], lev[c], u + NUPC * c + FO, rot + 9 * c, Bc);
#pragma unroll
        for (int q = 0; q < NUPC; ++q) {
            const T ri = T(1) / prm.R[(NUPC * c + q) * (NU + 1)];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const T bi = Bc.b[i][q] * ri;
#pragma unroll
                for (int j = 0; j <= i; ++j) G[i * (i + 1) / 2 + j] = fma(bi, Bc.b[j][q], G[i * (i + 1) / 2 + j]);
            }
        }
    }
    // ---- two Riccati steps from P = Q in information form, then N2^-1
    T P[45], Ni[45];
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) P[sp9(i, j)] = prm.Q[i * 9 + j];
#pragma unroll 1
    for (int it = 0; it < 3; ++it) {
        T Nm[45];
        inv_spd9(P, Nm);   // P^-1
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) Nm[sp9(3 + i, 3 + j)] += G[i * (i + 1) / 2 + j];
        inv_spd9(Nm, Ni);  // N^-1
        if (it < 2) atma(Ni, beta, Wm, prm.Q, P);
    }
    // ---- Y6 = rows 3..8 of N2^-1 A;  K = -R^-1 B' Y6;  Acl = A - E6 G Y6
    T Y6[6][9];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int j = 0; j < 9; ++j) Y6[r][j] = MA_at(Ni, beta, Wm, 3 + r, j);
    {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            ContactB<T, ROBOT> Bc;
            contact_B<T, ROBOT>(dt * a[c], lev[c], u + NUPC * c + FO, rot + 9 * c, Bc);
#pragma unroll
            for (int q = 0; q < NUPC; ++q) {
                const T ri = T(1) / prm.R[(NUPC * c + q) * (NU + 1)];
#pragma unroll
                for (int j = 0; j < 9; ++j) {
                    T v = T(0);
#pragma unroll
                    for (int r = 0; r < 6; ++r) v = fma(Bc.b[r][q], Y6[r][j], v);
                    em(d.K, (NUPC * c + q) * 9 + j) = -ri * v;
                }
            }
        }
    }
    {
#pragma unroll
        for (int i = 0; i < 9; ++i)
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                T v = (i == j) ? T(1) : T(0);
                if (i < 3 && j == i + 3) v = beta;
                if (i >= 6 && j < 3) v = Wm[i - 6][j];
                if (i >= 3) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) {
                        const int ia = i - 3;
                        const T g = G[ia >= r ? ia * (ia + 1) / 2 + r : r * (r + 1) / 2 + ia];
                        v = fma(-g, Y6[r][j], v);
                    }
                }
                em(d.Acl, i * 9 + j) = v;
            }
    }
    // ---- Qw = C W C' + eta (C: rows 6..8, -dt a_c [f_c]x)
    {
        T Cl[3][NW];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const T *f = u + NUPC * c + FO;
            const T fs[3][3] = {{T(0), -f[2], f[1]}, {f[2], T(0), -f[0]}, {-f[1], f[0], T(0)}};
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int q = 0; q < 3; ++q) Cl[r][3 * c + q] = -dt * a[c] * fs[r][q];
        }
        T CW[3][NW];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                T v = T(0);
#pragma unroll
                for (int q = 0; q < NW; ++q) v = fma(Cl[r][q], prm.cov_w[q * NW + j], v);
                CW[r][j] = v;
            }
#pragma unroll
        for (int i = 0; i < 9; ++i)
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                T v = prm.cov_eta[i * 9 + j];
                if (i >= 6 && j >= 6) {
#pragma unroll
                    for (int q = 0; q < NW; ++q) v = fma(CW[i - 6][q], Cl[j - 6][q], v);
                }
                em(d.Qw, i * 9 + j) = v;
            }
    }
}

// Covariance scan kernel: one wave per problem (cov_scan.hpp).
template <typename T, int ROBOT> __global__ void __launch_bounds__(64, 4) k_cov_scan(DevBuf<T> d, int only_active) {
    const int b = blockIdx.x;
    if (b >= d.B) return;
    if (only_active && !d.scp[b].active) return;
    __shared__ T lds[SCAN_LDS];
    cov_scan_problem<T, ROBOT>(d, b, (T *)lds);
}

#define INST(T, R)                                                     \
    template __global__ void k_lin_knots<T, R>(DevBuf<T>, int, int); \
    template __global__ void k_cov_scan<T, R>(DevBuf<T>, int);
INST(double, 0)
INST(double, 1)
INST(float, 0)
INST(float, 1)
#undef INST

}  // namespace cmpc
