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
// with its small matrices staged in LDS (lanes over matrix entries); k_cov_scan then runs the
// O(N) covariance scan for the problem.  Used when R is not diagonal (k_lin_knots otherwise).  Per knot: ~14 kflop (LQR) in LDS, ~3 KB of HBM
// traffic (inputs 0.6 KB, outputs f/A/B/C/K/Acl/Qw 2.6 KB at fp64).
#include "common.hpp"

namespace cmpc {

// C[M x N] = alpha op(A) op(B) (+ Cadd) with lanes over output entries; row-major LDS operands.
// TA: A stored as (K x M) and used transposed; TB: B stored as (N x K) and used transposed.  The
// dimensions are compile-time so every lane's K operands are read before its multiply chain.
template <int M, int N, int K, bool TA, bool TB, typename T>
__device__ __forceinline__ void wmm(T *Cm, const T *Am, const T *Bm, int lane, const T *Cadd = nullptr,
                                    T alpha = T(1)) {
#pragma unroll
    for (int e0 = 0; e0 < M * N; e0 += WAVE) {
        const int e = e0 + lane;
        if (e < M * N) {
            const int i = e / N, j = e % N;
            T a[K], bb[K];
#pragma unroll
            for (int q = 0; q < K; ++q) {
                a[q] = TA ? Am[q * M + i] : Am[i * K + q];
                bb[q] = TB ? Bm[j * K + q] : Bm[q * N + j];
            }
            T s0 = T(0), s1 = T(0);
#pragma unroll
            for (int q = 0; q < K; q += 2) {
                s0 = fma(a[q], bb[q], s0);
                if (q + 1 < K) s1 = fma(a[q + 1], bb[q + 1], s1);
            }
            T v = alpha * (s0 + s1);
            if (Cadd) v += Cadd[e];
            Cm[e] = v;
        }
    }
    wave_sync();
}

// fp64: the same product on the matrix cores (v_mfma_f64_16x16x4_f64, M, N <= 16): one LDS read
// per operand per lane and 4-wide k block instead of 2K reads per output.  Lane maps
// (cdna_hip_programming.md, f64): A lane l = A[l & 15][4 kb + (l >> 4)], B lane l =
// B[4 kb + (l >> 4)][l & 15], C/D lane l register r = C[(l >> 4) + 4 r][l & 15].
typedef double lin_v4d __attribute__((ext_vector_type(4)));
template <int M, int N, int K, bool TA, bool TB>
__device__ __forceinline__ void wmm(double *Cm, const double *Am, const double *Bm, int lane,
                                    const double *Cadd = nullptr, double alpha = 1.0) {
    static_assert(M <= 16 && N <= 16, "one 16x16 tile");
    const int r16 = lane & 15, q4 = lane >> 4;
    lin_v4d acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kb = 0; kb < (K + 3) / 4; ++kb) {
        const int kk = 4 * kb + q4;
        const bool ka = kk < K;
        const int kc = ka ? kk : K - 1;
        const int ia = r16 < M ? r16 : M - 1, jb = r16 < N ? r16 : N - 1;
        const double a = TA ? Am[kc * M + ia] : Am[ia * K + kc];
        const double bb = TB ? Bm[jb * K + kc] : Bm[kc * N + jb];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64((ka && r16 < M) ? a : 0.0, (ka && r16 < N) ? bb : 0.0, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = q4 + 4 * r, j = r16;
        if (i < M && j < N) {
            double v = alpha * acc[r];
            if (Cadd) v += Cadd[i * N + j];
            Cm[i * N + j] = v;
        }
    }
    wave_sync();
}

// entry (r, j) of the cross-product matrix [v]x by selects (a runtime-indexed local array would
// live in scratch memory)
template <typename T, typename V> __device__ __forceinline__ T skew_at(const V &v, int r, int j) {
    const int idx = 3 - r - j;
    const T e = idx == 0 ? T(v[0]) : (idx == 1 ? T(v[1]) : T(v[2]));
    return r == j ? T(0) : ((j - r + 3) % 3 == 1 ? -e : e);
}

template <typename T> __device__ __forceinline__ T lin_rcp(T p) {
    T r;
    if constexpr (sizeof(T) == 8) r = __builtin_amdgcn_rcp(p); else r = __builtin_amdgcn_rcpf(p);
    r = fma(r, fma(-p, r, T(1)), r);
    return fma(r, fma(-p, r, T(1)), r);
}

// In-place inverse of an SPD n x n LDS matrix by Gauss-Jordan over the lanes (no pivoting; the
// LQR matrix R + B'PB is SPD with R > 0), branch-free, the next pivot's reciprocal formed one
// pivot ahead from broadcast reads so its chain overlaps the update.
template <int n, typename T> __device__ __forceinline__ void wgj_inv(T *M, int lane) {
    constexpr int E = (n * n + WAVE - 1) / WAVE;
    T a[E];
    int ii[E], jj[E];
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int e = lane + r * WAVE;
        ii[r] = e < n * n ? e / n : n;
        jj[r] = e < n * n ? e % n : n;
        a[r] = e < n * n ? M[e] : T(0);
    }
    T ip = lin_rcp(M[0]);
#pragma unroll
    for (int c = 0; c < n; ++c) {
        T aic[E], acj[E];
#pragma unroll
        for (int r = 0; r < E; ++r) {
            aic[r] = M[(ii[r] < n ? ii[r] : 0) * n + c];
            acj[r] = M[c * n + (jj[r] < n ? jj[r] : 0)];
        }
        T ipn = T(0);
        if (c + 1 < n) ipn = lin_rcp(fma(-(M[(c + 1) * n + c] * ip), M[c * n + c + 1], M[(c + 1) * n + c + 1]));
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const T mi = aic[r] * ip;
            const T gen = fma(-mi, acj[r], a[r]), row = acj[r] * ip, col = -mi;
            a[r] = ii[r] == c ? (jj[r] == c ? ip : row) : (jj[r] == c ? col : gen);
        }
        wave_sync();
#pragma unroll
        for (int r = 0; r < E; ++r)
            if (lane + r * WAVE < n * n) M[lane + r * WAVE] = a[r];
        wave_sync();
        ip = ipn;
    }
}

template <typename T, int ROBOT> struct LinSmem {
    static constexpr int NC = Robot<ROBOT>::NC;
    T x[9], u[NU], p[3 * NC], R[9 * NC], a[NC];
    T A[81], Bm[9 * NU], Cm[9 * 3 * NC];
    T P[81], AtP[81], AtPA[81], PB[9 * NU], AtPB[9 * NU], M[NU * NU], X[NU * 9];   // PB doubles as C W scratch
};

template <typename T, int ROBOT>
__device__ void linearize_knot(const DevBuf<T> &d, const DevParams<T> &prm, int b, int k, LinSmem<T, ROBOT> &s,
                               int lane) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    constexpr int NW = 3 * NC;
    const int N = d.N;
    const size_t kn = (size_t)b * N + k;
    // ---- stage inputs
    if (lane < 9) s.x[lane] = d.Xlin[((size_t)b * (N + 1) + k) * 9 + lane];   // linearization point
    if (lane < NU) s.u[lane] = d.Ulin[kn * NU + lane];
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
        d.f[(size_t)i * d.LS + kn] = s.x[i] + F * dt;
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
            v = dt * skew_at<T>(w, r, j);
        }
        s.A[e] = v;
        d.A[(size_t)e * d.LS + kn] = v;
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
                v = ac * skew_at<T>(lev, i - 6, fq);
            }
        } else if (ROBOT == 1 && i >= 6) {
            const T *Rc = &s.R[9 * c];
            const int r = i - 6;
            if (q < 2) {   // -[f]x R[:, q]
                T acc = 0;
                for (int z = 0; z < 3; ++z) acc += skew_at<T>(f, r, z) * Rc[z * 3 + q];
                v = -ac * acc;
            } else {       // tau: R[:, 2]
                v = ac * Rc[r * 3 + 2];
            }
        }
        s.Bm[e] = v;
        d.Bu[(size_t)e * d.LS + kn] = v;
    }
    for (int e = lane; e < 9 * NW; e += WAVE) {
        const int i = e / NW, j = e % NW, c = j / 3, q = j % 3;
        T v = T(0);
        if (i >= 6) {   // -dt a [f]x
            const T *f = &s.u[NUPC * c + FO];
            v = -dt * s.a[c] * skew_at<T>(f, i - 6, q);
        }
        s.Cm[e] = v;
        d.C[(size_t)e * d.LS + kn] = v;
    }
    for (int e = lane; e < 81; e += WAVE) s.P[e] = prm.Q[e];
    wave_sync();
    // ---- LQR: two Riccati steps from P = Q, then K   (src/centroidal_model.py:217-228)
    //   X = (R + B'PB)^-1 B'PA (Gauss-Jordan inverse over the lanes), P = Q + A'PA - A'PB X
    for (int it = 0; it < 3; ++it) {
        wmm<9, 9, 9, true, false>(s.AtP, s.A, s.P, lane);            // A' P
        wmm<9, NU, 9, false, false>(s.PB, s.P, s.Bm, lane);          // P B
        wmm<NU, NU, 9, true, false>(s.M, s.Bm, s.PB, lane, prm.R);   // R + B' P B
        wmm<9, NU, 9, false, false>(s.AtPB, s.AtP, s.Bm, lane);      // A' P B
        if (it < 2) wmm<9, 9, 9, false, false>(s.AtPA, s.AtP, s.A, lane);
        wgj_inv<NU>(s.M, lane);
        wmm<NU, 9, NU, false, true>(s.X, s.M, s.AtPB, lane);         // (R + B'PB)^-1 (A'PB)'
        if (it < 2) {
            // P = Q + A'PA - A'PB X
            wmm<9, 9, NU, false, false>(s.P, s.AtPB, s.X, lane, s.AtPA, T(-1));
            for (int e = lane; e < 81; e += WAVE) s.P[e] += prm.Q[e];
            wave_sync();
        }
    }
    for (int e = lane; e < NU * 9; e += WAVE) d.K[(size_t)e * d.LS + kn] = -s.X[e];
    // ---- scan helpers: Acl = A + B K, Qw = C W C' + eta
    for (int e = lane; e < 81; e += WAVE) {
        const int i = e / 9, j = e % 9;
        T acc = s.A[e];
        for (int q = 0; q < NU; ++q) acc -= s.Bm[i * NU + q] * s.X[q * 9 + j];
        d.Acl[(size_t)e * d.LS + kn] = acc;
    }
    static_assert(9 * NW <= 9 * NU, "C W scratch");
    T *cw = s.PB;
    for (int e = lane; e < 9 * NW; e += WAVE) {
        const int i = e / NW, j = e % NW;
        T acc = T(0);
        for (int q = 0; q < NW; ++q) acc = fma(s.Cm[i * NW + q], prm.cov_w[q * NW + j], acc);
        cw[e] = acc;
    }
    wave_sync();
    for (int e = lane; e < 81; e += WAVE) {
        const int i = e / 9, j = e % 9;
        T acc = prm.cov_eta[e];
        for (int q = 0; q < NW; ++q) acc = fma(cw[i * NW + q], s.Cm[j * NW + q], acc);
        d.Qw[(size_t)e * d.LS + kn] = acc;
    }
    wave_sync();
}

// The general-R path (non-diagonal LQR weight): one workgroup (4 waves) per problem, one wave per
// knot; the covariance scan then runs in k_cov_scan (linearize_lane.hip).
template <typename T, int ROBOT>
__global__ void __launch_bounds__(256, 4) k_linearize(DevBuf<T> d, int only_active) {
    const int b = blockIdx.x;
    if (b >= d.B) return;
    if (only_active && !d.scp[b].active) return;
    // four per-wave scratch records (under 40 KB at fp64: four workgroups per CU)
    __shared__ LinSmem<T, ROBOT> sm[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const DevParams<T> &prm = d.params[d.class_id[b]];
    const int N = d.N;
#ifdef CMPC_STAMPS
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
    for (int k = wid; k < N; k += 4) linearize_knot<T, ROBOT>(d, prm, b, k, sm[wid], lane);
#ifdef CMPC_STAMPS
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#endif
#ifdef CMPC_STAMPS
    if (lane == 0) {
        d.stamps[(size_t)b * 16 + 9] = t1 - t0;
        d.stamps[(size_t)b * 16 + 10] = 0;
    }
#endif
}

template __global__ void k_linearize<double, 0>(DevBuf<double>, int);
template __global__ void k_linearize<double, 1>(DevBuf<double>, int);
template __global__ void k_linearize<float, 0>(DevBuf<float>, int);
template __global__ void k_linearize<float, 1>(DevBuf<float>, int);

}  // namespace cmpc
