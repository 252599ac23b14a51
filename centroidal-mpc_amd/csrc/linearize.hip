// Linearization kernel: per knot f, A, B, C (closed form), LQR gain K (2 Riccati steps from
// P = Q) and the covariance scan Sigma_{k+1} = (A + B K) Sigma_k (A + B K)' + C W C' + eta.
//
// Replaces Centroidal_model.compute_trajectory_data / compute_everything /
// integrate_model_one_step (reference src/centroidal_model.py:189-291), which JAX runs as a
// sequential fori_loop with three jacfwd traces per knot and propagates two all-zero
// covariance-gradient tensors of O(N^2) size (they are identically zero, quirk Q3, and are
// elided here).
//
// Mapping: one workgroup (4 waves) per problem; each wave linearizes knots k = wave, wave+4, ...
// with its small matrices staged in LDS (lanes over matrix entries); then wave 0 runs the
// O(N) covariance scan for the problem.  Per knot: ~14 kflop (LQR) in LDS, ~3 KB of HBM
// traffic (inputs 0.6 KB, outputs f/A/B/C/K/Acl/Qw 2.6 KB at fp64).
#include "common.hpp"

namespace cmpc {

// C[m x n] = op(A) * op(B) with lanes over output entries; row-major LDS operands.
// ta: A stored as (k x m) and used transposed; tb: B stored as (n x k) and used transposed.
template <typename T>
__device__ __forceinline__ void wmm(T *Cm, const T *Am, const T *Bm, int m, int n, int k, bool ta, bool tb,
                                    int lane, T beta_c = T(0), const T *Cadd = nullptr, T alpha = T(1)) {
    for (int e = lane; e < m * n; e += WAVE) {
        const int i = e / n, j = e % n;
        T acc = T(0);
        for (int q = 0; q < k; ++q) {
            const T a = ta ? Am[q * m + i] : Am[i * k + q];
            const T b = tb ? Bm[j * k + q] : Bm[q * n + j];
            acc = fma(a, b, acc);
        }
        T v = alpha * acc;
        if (Cadd) v += Cadd[e];
        else if (beta_c != T(0)) v += beta_c * Cm[e];   // never read an uninitialized C when beta = 0
        Cm[e] = v;
    }
    wave_sync();
}

// In-place Cholesky (lower) of an SPD n x n LDS matrix; the strict upper part is left stale.
template <typename T> __device__ void wchol(T *M, int n, int lane) {
    for (int c = 0; c < n; ++c) {
        const T d = sqrt(M[c * n + c]);
        const T id = T(1) / d;
        wave_sync();
        for (int i = c + 1 + lane; i < n; i += WAVE) M[i * n + c] *= id;
        if (lane == 0) M[c * n + c] = d;
        wave_sync();
        const int rem = n - c - 1;
        for (int e = lane; e < rem * rem; e += WAVE) {
            const int i = c + 1 + e / rem, j = c + 1 + e % rem;
            if (j <= i) M[i * n + j] -= M[i * n + c] * M[j * n + c];
        }
        wave_sync();
    }
}

// X (n x r, row-major) <- M^-1 X for the Cholesky factor L (lower) in M; lanes over columns.
template <typename T> __device__ void wchol_solve(const T *L, T *X, int n, int r, int lane) {
    for (int j = lane; j < r; j += WAVE) {
        for (int i = 0; i < n; ++i) {          // forward  L y = x
            T s = X[i * r + j];
            for (int q = 0; q < i; ++q) s -= L[i * n + q] * X[q * r + j];
            X[i * r + j] = s / L[i * n + i];
        }
        for (int i = n - 1; i >= 0; --i) {     // backward L' z = y
            T s = X[i * r + j];
            for (int q = i + 1; q < n; ++q) s -= L[q * n + i] * X[q * r + j];
            X[i * r + j] = s / L[i * n + i];
        }
    }
    wave_sync();
}

template <typename T, int ROBOT> struct LinSmem {
    static constexpr int NC = Robot<ROBOT>::NC;
    T x[9], u[NU], p[3 * NC], R[9 * NC], a[NC];
    T A[81], Bm[9 * NU], Cm[9 * 3 * NC];
    T P[81], AtP[81], AtPA[81], PB[9 * NU], AtPB[9 * NU], M[NU * NU], X[NU * 9], tmp[9 * 3 * NC];
};

template <typename T, int ROBOT>
__device__ void linearize_knot(const DevBuf<T> &d, const DevParams<T> &prm, int b, int k, LinSmem<T, ROBOT> &s,
                               int lane) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    constexpr int NW = 3 * NC;
    const int N = d.N;
    const size_t kn = (size_t)b * N + k;
    // ---- stage inputs
    if (lane < 9) s.x[lane] = d.Xbar[((size_t)b * (N + 1) + k) * 9 + lane];
    if (lane < NU) s.u[lane] = d.Ubar[kn * NU + lane];
    if (lane < 3 * NC) s.p[lane] = d.pos[kn * 3 * NC + lane];
    if (lane < 9 * NC) s.R[lane] = d.rot[kn * 9 * NC + lane];
    if (lane < NC) s.a[lane] = T(d.logic[kn * NC + lane]);
    wave_sync();
    const T dt = prm.dt, m = prm.mass;
    // ---- f = x + dt * F(x, u)   (src/centroidal_model.py:189-212)
    if (lane < 9) {
        const int i = lane;
        T F;
        if (i < 3) {
            F = (T(1) / m) * s.x[3 + i];
        } else if (i < 6) {
            F = (i == 5) ? m * prm.gravity : T(0);
            for (int c = 0; c < NC; ++c) F += s.a[c] * s.u[NUPC * c + FO + (i - 3)];
        } else {
            F = T(0);
            const int r = i - 6, r1 = (r + 1) % 3, r2 = (r + 2) % 3;
            for (int c = 0; c < NC; ++c) {
                const T *f = &s.u[NUPC * c + FO];
                T l1 = s.p[3 * c + r1] - s.x[r1], l2 = s.p[3 * c + r2] - s.x[r2];
                T v = l1 * f[r2] - l2 * f[r1];
                if (ROBOT == 1) {
                    const T *Rc = &s.R[9 * c];
                    // (R[:,0:2] cop) x f  +  R[:,2] tau
                    T q1 = Rc[r1 * 3 + 0] * s.u[NUPC * c] + Rc[r1 * 3 + 1] * s.u[NUPC * c + 1];
                    T q2 = Rc[r2 * 3 + 0] * s.u[NUPC * c] + Rc[r2 * 3 + 1] * s.u[NUPC * c + 1];
                    v += q1 * f[r2] - q2 * f[r1] + Rc[r * 3 + 2] * s.u[NUPC * c + 5];
                }
                F += s.a[c] * v;
            }
        }
        d.f[kn * 9 + i] = s.x[i] + F * dt;
    }
    // ---- A, B, C closed form (jacfwd at :230-232)
    for (int e = lane; e < 81; e += WAVE) {
        const int i = e / 9, j = e % 9;
        T v = (i == j) ? T(1) : T(0);
        if (i < 3 && j == i + 3) v = dt * (T(1) / m);
        if (i >= 6 && j < 3) {   // d/dc [(p - c) x f] = [f]x ; entry (r, j) of [sum a f]x
            const int r = i - 6;
            T w[3] = {0, 0, 0};
            for (int c = 0; c < NC; ++c)
                for (int q = 0; q < 3; ++q) w[q] += s.a[c] * s.u[NUPC * c + FO + q];
            const T sk[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
            v = dt * sk[r * 3 + j];
        }
        s.A[e] = v;
        d.A[kn * 81 + e] = v;
    }
    for (int e = lane; e < 9 * NU; e += WAVE) {
        const int i = e / NU, j = e % NU, c = j / NUPC, q = j % NUPC;
        const T ac = dt * s.a[c];
        T v = T(0);
        const T *f = &s.u[NUPC * c + FO];
        T lev[3];
        for (int z = 0; z < 3; ++z) lev[z] = s.p[3 * c + z] - s.x[z];
        if (ROBOT == 1) {
            const T *Rc = &s.R[9 * c];
            for (int z = 0; z < 3; ++z) lev[z] += Rc[z * 3 + 0] * s.u[NUPC * c] + Rc[z * 3 + 1] * s.u[NUPC * c + 1];
        }
        if (q >= FO && q < FO + 3) {
            const int fq = q - FO;
            if (i >= 3 && i < 6) v = (i - 3 == fq) ? ac : T(0);
            if (i >= 6) {
                const T sk[9] = {0, -lev[2], lev[1], lev[2], 0, -lev[0], -lev[1], lev[0], 0};
                v = ac * sk[(i - 6) * 3 + fq];
            }
        } else if (ROBOT == 1 && i >= 6) {
            const T *Rc = &s.R[9 * c];
            const int r = i - 6;
            if (q < 2) {   // -[f]x R[:, q]
                const T sk[9] = {0, -f[2], f[1], f[2], 0, -f[0], -f[1], f[0], 0};
                T acc = 0;
                for (int z = 0; z < 3; ++z) acc += sk[r * 3 + z] * Rc[z * 3 + q];
                v = -ac * acc;
            } else {       // tau: R[:, 2]
                v = ac * Rc[r * 3 + 2];
            }
        }
        s.Bm[e] = v;
        d.Bu[kn * 9 * NU + e] = v;
    }
    for (int e = lane; e < 9 * NW; e += WAVE) {
        const int i = e / NW, j = e % NW, c = j / 3, q = j % 3;
        T v = T(0);
        if (i >= 6) {   // -dt a [f]x
            const T *f = &s.u[NUPC * c + FO];
            const T sk[9] = {0, -f[2], f[1], f[2], 0, -f[0], -f[1], f[0], 0};
            v = -dt * s.a[c] * sk[(i - 6) * 3 + q];
        }
        s.Cm[e] = v;
        d.C[kn * 9 * NW + e] = v;
    }
    for (int e = lane; e < 81; e += WAVE) s.P[e] = prm.Q[e];
    wave_sync();
    // ---- LQR: two Riccati steps from P = Q, then K   (src/centroidal_model.py:217-228)
    for (int it = 0; it < 3; ++it) {
        wmm(s.AtP, s.A, s.P, 9, 9, 9, true, false, lane);            // A' P
        wmm(s.PB, s.P, s.Bm, 9, NU, 9, false, false, lane);          // P B
        wmm(s.M, s.Bm, s.PB, NU, NU, 9, true, false, lane, T(0), prm.R);   // R + B' P B
        wmm(s.AtPB, s.AtP, s.Bm, 9, NU, 9, false, false, lane);      // A' P B
        if (it < 2) wmm(s.AtPA, s.AtP, s.A, 9, 9, 9, false, false, lane);
        wchol(s.M, NU, lane);
        for (int e = lane; e < NU * 9; e += WAVE) s.X[e] = s.AtPB[(e % 9) * NU + e / 9];   // (A'PB)' = B'PA
        wave_sync();
        wchol_solve(s.M, s.X, NU, 9, lane);                           // (R + B'PB)^-1 B'PA
        if (it < 2) {
            // P = Q + A'PA - A'PB X
            for (int e = lane; e < 81; e += WAVE) {
                const int i = e / 9, j = e % 9;
                T acc = T(0);
                for (int q = 0; q < NU; ++q) acc = fma(s.AtPB[i * NU + q], s.X[q * 9 + j], acc);
                s.P[e] = prm.Q[e] + s.AtPA[e] - acc;
            }
            wave_sync();
        }
    }
    for (int e = lane; e < NU * 9; e += WAVE) d.K[kn * NU * 9 + e] = -s.X[e];
    // ---- scan helpers: Acl = A + B K, Qw = C W C' + eta
    for (int e = lane; e < 81; e += WAVE) {
        const int i = e / 9, j = e % 9;
        T acc = s.A[e];
        for (int q = 0; q < NU; ++q) acc -= s.Bm[i * NU + q] * s.X[q * 9 + j];
        d.Acl[kn * 81 + e] = acc;
    }
    for (int e = lane; e < 9 * NW; e += WAVE) {
        const int i = e / NW, j = e % NW;
        T acc = T(0);
        for (int q = 0; q < NW; ++q) acc = fma(s.Cm[i * NW + q], prm.cov_w[q * NW + j], acc);
        s.tmp[e] = acc;
    }
    wave_sync();
    for (int e = lane; e < 81; e += WAVE) {
        const int i = e / 9, j = e % 9;
        T acc = prm.cov_eta[e];
        for (int q = 0; q < NW; ++q) acc = fma(s.tmp[i * NW + q], s.Cm[j * NW + q], acc);
        d.Qw[kn * 81 + e] = acc;
    }
    wave_sync();
}

template <typename T, int ROBOT>
__global__ void __launch_bounds__(256) k_linearize(DevBuf<T> d, int only_active) {
    const int b = blockIdx.x;
    if (b >= d.B) return;
    if (only_active && !d.scp[b].active) return;
    __shared__ LinSmem<T, ROBOT> sm[4];
    __shared__ T S[81], Tm[81];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const DevParams<T> &prm = d.params[d.class_id[b]];
    const int N = d.N;
    for (int k = wid; k < N; k += 4) linearize_knot<T, ROBOT>(d, prm, b, k, sm[wid], lane);
    __syncthreads();
    __threadfence_block();
    if (wid != 0) return;
    // ---- covariance scan (src/centroidal_model.py:234-238, 266, 284)
    for (int e = lane; e < 81; e += WAVE) {
        S[e] = T(0);
        d.Sig[((size_t)b * (N + 1)) * 81 + e] = T(0);
    }
    wave_sync();
    for (int k = 0; k < N; ++k) {
        const T *Ac = d.Acl + ((size_t)b * N + k) * 81;
        const T *Qw = d.Qw + ((size_t)b * N + k) * 81;
        for (int e = lane; e < 81; e += WAVE) {     // Tm = Acl S
            const int i = e / 9, j = e % 9;
            T acc = T(0);
            for (int q = 0; q < 9; ++q) acc = fma(Ac[i * 9 + q], S[q * 9 + j], acc);
            Tm[e] = acc;
        }
        wave_sync();
        T out[2];
        for (int r = 0, e = lane; e < 81; e += WAVE, ++r) {   // Tm Acl' + Qw
            const int i = e / 9, j = e % 9;
            T acc = Qw[e];
            for (int q = 0; q < 9; ++q) acc = fma(Tm[i * 9 + q], Ac[j * 9 + q], acc);
            out[r] = acc;
        }
        wave_sync();
        for (int r = 0, e = lane; e < 81; e += WAVE, ++r) {
            S[e] = out[r];
            d.Sig[((size_t)b * (N + 1) + k + 1) * 81 + e] = out[r];
        }
        wave_sync();
    }
}

template __global__ void k_linearize<double, 0>(DevBuf<double>, int);
template __global__ void k_linearize<double, 1>(DevBuf<double>, int);
template __global__ void k_linearize<float, 0>(DevBuf<float>, int);
template __global__ void k_linearize<float, 1>(DevBuf<float>, int);

}  // namespace cmpc
