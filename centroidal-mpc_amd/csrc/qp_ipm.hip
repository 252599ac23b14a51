// Batched structured interior-point QP (Mehrotra predictor-corrector) for the SCP subproblem.
//
// Replaces solve_subproblem (reference src/scp_solver.py:59-68: osqp.OSQP().setup(P, q, A, l,
// u, eps_abs=1e-7, eps_rel=1e-7, polish=True).solve()).  Same QP, same unique minimizer; the
// algorithm is chosen for the GPU: ~10-25 Newton steps instead of hundreds to thousands of
// ADMM iterations, each step exploiting the stage structure ("QP").
//
// Newton system.  With Phi = H + G'DG (block diagonal per knot; the TR slack t_k is eliminated
// inside its knot) the equality multipliers solve the dual Schur system S dnu = rhs with
// S = E Phi^-1 E' block tridiagonal: N+2 blocks of 9x9 (init row, N dynamics rows, final
// row).  Friction rows use the push-through form Phi^-1 G'D = W^-1 G'(D^-1 + G W^-1 G')^-1 so
// no D * r product ever forms (D = lambda/s reaches 1e15+ near convergence).
//
// Mapping (one 128-thread workgroup per problem, all IPM iterations in one launch):
//   thread k <-> knot k for every per-knot phase (residuals, Phi factors, S blocks, Newton
//   back-substitution, step length); waves 0 and 1 run the two ends of the block factorization
//   of S and of the two block sweeps per Newton solve.  Problems are independent, so the grid
//   needs no inter-workgroup communication.
// Layout: every per-knot workspace array and the stage records are field-major, knot-minor
// (field f of knot k at base + f * KPC + k, common.hpp), so each field access of a wave is one
// contiguous 512-B transaction; per-block vectors (nu, r_e) use the same scheme over the N + 2
// Schur blocks.  The Schur right-hand side / direction dnu never leave LDS.
#include <limits>

#include "common.hpp"
#include "cov_scan.hpp"

// Phases are always inlined: an outlined phase gets its Ctx by reference, i.e. a generic pointer to
// the caller's scratch, and then does every access through flat instructions (round 4: the
// refinement phases phase_lres / phase_dz_refine were outlined in k_qp_group<.., 2> once the kernel
// grew, 431 flat loads and stores, and the kernel faulted with a memory aperture violation on its
// first refinement; inlined, no flat instruction is left).  CMPC_NOINLINE (diagnostic builds) outlines them.
#ifdef CMPC_NOINLINE
#define PHASE_ATTR __attribute__((noinline))
#elif defined(CMPC_PHASE_FREE)   // diagnostic builds: the compiler's own inlining decisions
#define PHASE_ATTR
#else
#define PHASE_ATTR __attribute__((always_inline))
#endif
#define WF(f) (Ws<ROBOT>::f)   // workspace field row
#ifndef QP_MIN_WAVES
#define QP_MIN_WAVES 1   // __launch_bounds__ waves per SIMD (2: 256 registers, four workgroups per CU)
#endif
#ifndef QP_MIN_WAVES_2W
#define QP_MIN_WAVES_2W QP_MIN_WAVES   // the same for the two-wave kernel
#endif
#ifndef QP_KE
#define QP_KE 8
#endif

namespace cmpc {

// workgroup: NTT threads (template; 64 = one wave, 128 = two), knots k, k + NTT, ... per thread
// Stored parts of the Phi factors (phase_factor -> phase_sblock); the w and direction phases
// recompute everything they need (the trust-region Cholesky factor, each contact's G W^-1, Kinv,
// F and W'^-1: tr_factor, fric_factor, fric_F, contact_wd), which costs less than its HBM round trip.
constexpr int FU = 12, FU_F = 0, FU_WI = 6;   // per contact: F = [Phi_u^-1] force block, packed 6 | 1 / W' diagonal 6
constexpr int FX = 6, FX_ML = 0;               // per knot: M_LL = [Phi^-1]_LL packed 6

// Workspace of one problem.  Per-knot arrays and the per-block vectors (nu, r_e; block j in
// column j) are field rows of pitch KPC (field-major, see the layout note above); their offsets
// are compile-time constants.  The Schur blocks follow the field rows (see tw_factor_ends).
constexpr int NBMAX = 257;   // Schur blocks at the largest supported horizon (N = 255)
template <int ROBOT> struct Ws {
    static constexpr int NI = Rows<ROBOT>::NI, NC = Robot<ROBOT>::NC;
    enum : int {   // field rows
        s = 0, l = s + NI, x = l + NI, u = x + 9, t = u + NU, nu = t + 1, rdx = nu + 9, rdt = rdx + 9,
        rdu = rdt + 1, rde = rdu + NU, rdi = rde + 9, facx = rdi + NI, facu = facx + FX, wx = facu + NC * FU,
        wt = wx + 9, wu = wt + 1, dx = wu + NU, dt = dx + 9, du = dt + 1, ds = du + NU, dl = ds + NI,
        dsa = dl + NI, dla = dsa + NI, dn0 = dla + NI, ub = dn0 + 9, NF = ub + NU
    };
    // Schur blocks (block-major 9x9): S_jj -> I_j, and S_{j,j+1} -> X_{j+1} / Y_j (tw_factor_ends);
    // four-wave workgroups also the fill factors H_j and the separator scratch (schur_pt.hpp)
    static constexpr size_t Sd = (size_t)NF * KPC, So = Sd + (size_t)NBMAX * 81, Sh = So + (size_t)NBMAX * 81,
                            Sx = Sh + (size_t)NBMAX * 81;
    static constexpr size_t total = (Sx + (size_t)16 * 81 + 7) & ~size_t(7);
};

template <typename T> __device__ __forceinline__ T rcp_nr(T p) {
    // reciprocal: hardware estimate + two Newton steps (full precision)
    T r;
    if constexpr (sizeof(T) == 8) r = __builtin_amdgcn_rcp(p); else r = __builtin_amdgcn_rcpf(p);
    r = fma(r, fma(-p, r, T(1)), r);
    r = fma(r, fma(-p, r, T(1)), r);
    return r;
}
// LDS-qualified element type (keeps ds_* instructions in outlined helpers)
template <typename T> using LdsT = __attribute__((address_space(3))) T;
// global-qualified element type: in an outlined helper a plain T * is a flat pointer, and flat
// loads count in both vmcnt and lgkmcnt, so every LDS wait would also wait for the HBM loads in
// flight (the meeting block's operands, the sweep's next chunk of blocks)
template <typename T> using GlbT = __attribute__((address_space(1))) T;

// a / b as a * (1 / b): the IEEE fp64 division is a ~10-instruction sequence; the reciprocal with
// two Newton steps is within an ulp or two, which the interior-point iteration does not notice
template <typename T> __device__ __forceinline__ T fdiv(T a, T b) { return a * rcp_nr(b); }

template <typename T> __device__ __forceinline__ T tr_sign(int j, int i) { return ((j >> i) & 1) ? T(-1) : T(1); }

// ------------------------------------------------------------------ compact A, B operators
// A = [[I, beta I, 0], [0, I, 0], [[w]x, 0, I]] in (c, l, L) blocks.
template <typename T, typename W> __device__ __forceinline__ void opA(const W &w, T beta, const T *x, T *o) {
    for (int i = 0; i < 3; ++i) o[i] = x[i] + beta * x[3 + i];
    for (int i = 0; i < 3; ++i) o[3 + i] = x[3 + i];
    T wc[3];
    cross3(w, x, wc);
    for (int i = 0; i < 3; ++i) o[6 + i] = x[6 + i] + wc[i];
}
template <typename T, typename W> __device__ __forceinline__ void opAT(const W &w, T beta, const T *v, T *o) {
    T vw[3];
    cross3(v + 6, w, vw);   // [w]x' v_L = v_L x w
    for (int i = 0; i < 3; ++i) o[i] = v[i] + vw[i];
    for (int i = 0; i < 3; ++i) o[3 + i] = beta * v[i] + v[3 + i];
    for (int i = 0; i < 3; ++i) o[6 + i] = v[6 + i];
}
template <typename T, int ROBOT, typename SR> __device__ __forceinline__ void opB(const SR &st, const T *u, T *o) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    using S = Stage<ROBOT>;
    for (int i = 0; i < 9; ++i) o[i] = T(0);
    for (int c = 0; c < NC; ++c) {
        const auto cs = st + (S::CON + S::CS * c);
        const T a = cs[S::ALPHA];
        const T *f = u + NUPC * c + FO;
        T lf[3];
        cross3(cs + S::LEVER, f, lf);
        for (int i = 0; i < 3; ++i) { o[3 + i] += a * f[i]; o[6 + i] += a * lf[i]; }
        if (ROBOT == 1) {
            const T *cp = u + NUPC * c;
            for (int r = 0; r < 3; ++r)
                o[6 + r] += cs[S::BCOP + 2 * r] * cp[0] + cs[S::BCOP + 2 * r + 1] * cp[1] + cs[S::BTAU + r] * cp[5];
        }
    }
}
template <typename T, int ROBOT, typename SR> __device__ __forceinline__ void opBT(const SR &st, const T *v, T *o) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    using S = Stage<ROBOT>;
    for (int c = 0; c < NC; ++c) {
        const auto cs = st + (S::CON + S::CS * c);
        const T a = cs[S::ALPHA];
        T vl[3];
        cross3(v + 6, cs + S::LEVER, vl);   // [lev]x' v_L = v_L x lev
        T *oc = o + NUPC * c;
        for (int i = 0; i < 3; ++i) oc[FO + i] = a * (v[3 + i] + vl[i]);
        if (ROBOT == 1) {
            for (int q = 0; q < 2; ++q) {
                T acc = T(0);
                for (int r = 0; r < 3; ++r) acc += cs[S::BCOP + 2 * r + q] * v[6 + r];
                oc[q] = acc;
            }
            oc[5] = cs[S::BTAU] * v[6] + cs[S::BTAU + 1] * v[7] + cs[S::BTAU + 2] * v[8];
        }
    }
}

// The three separator blocks of the four-chain recurrence (schur_pt.hpp).  Passed by value to the
// outlined chain functions: as a reference to an array in the caller's scratch every access was a
// flat load.
struct Seps {
    int v[3];
    __device__ __forceinline__ int operator[](int i) const { return v[i]; }
    __device__ __forceinline__ int &operator[](int i) { return v[i]; }
};

// ------------------------------------------------------------------ per-problem context
template <typename T, int ROBOT> struct Ctx {
    static constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    static constexpr int NI = Rows<ROBOT>::NI;
    using R_ = Rows<ROBOT>;
    using S = Stage<ROBOT>;
    int N;
    const DevParams<T> *prm;
    const T *stage;       // (SIZE, KPC) field-major
    const uint8_t *logic; // (N, NC)
    const T *xbar;        // (N+1, 9)
    T cw, beta;
    T *ws;
    T *Sd, *So;           // Schur diagonal blocks / inverses and couplings (workspace, see tw_factor_ends)
    LdsT<T> *vb;          // Schur rhs -> direction dnu, (N+2) x 9 block vector in LDS
    T dcap;               // cap on D = lambda/s for the CoP rows (D-form, folded into W_cop)
    T fls, fll;           // Solo12 starting-point floors of s, lambda (0: CVXOPT shift)
    const LdsT<T> *wt;    // LDS copy of the cost weights: Wx | 1/Wx | Wu | 1/Wu (parameter loads
                          // next to workspace stores were each waited on alone)
    __device__ T Wx(int i) const { return wt[i]; }
    __device__ T iWx(int i) const { return wt[9 + i]; }
    __device__ T Wu(int i) const { return wt[18 + i]; }
    __device__ T iWu(int i) const { return wt[18 + NU + i]; }
    __device__ T Dform(T l, T s_) const { return fmin(fdiv(l, s_), dcap); }

    __device__ SV<const T> st(int k) const { return SV<const T>{stage + k}; }
    // per-knot record k / per-block vector j of workspace field row f (Ws<ROBOT>::...)
    __device__ SV<T> kv(int f, int k) const { return SV<T>{ws + f * KPC + k}; }
    __device__ SV<T> bv(int f, int j) const { return SV<T>{ws + f * KPC + j}; }
    // contact-active bits of knot k, loaded once per phase (0 at k = N: only the TR rows exist)
    const LdsT<uint8_t> *cm = nullptr;   // per-knot contact masks in LDS (set once per solve)
    // multi-wave workgroups: w_x of knot k (k >= 1) parked here by phase_w and added to Schur block
    // k after the phase's barrier (add_wx), since block k's other terms come from another wave
    LdsT<T> *wxs = nullptr;
    LdsT<T> *bus = nullptr;   // four-wave split w phases: B w_u of knot k at block 1 + k (add_wx)
    T *Sh = nullptr, *Sx = nullptr;   // four-wave workgroups: fill factors, separator scratch (schur_pt.hpp)
    Seps sp{{0, 0, 0}};               // four-wave workgroups: separator blocks
    LdsT<T> *sbv = nullptr, *hy = nullptr;   // separator right-hand-side terms, fill products
    __device__ unsigned cmask(int k) const { return cm ? unsigned(cm[k]) : cmask_mem(k); }
    __device__ unsigned cmask_mem(int k) const {
        if (k >= N) return 0u;
        const uint8_t *lg = logic + (size_t)k * NC;
        unsigned m = 0;
        if (NC == 4) {
            const uint32_t v = *reinterpret_cast<const uint32_t *>(lg);
            for (int c = 0; c < 4; ++c) m |= ((v >> (8 * c)) & 0xffu) ? (1u << c) : 0u;
        } else {
            const uint32_t v = *reinterpret_cast<const uint16_t *>(lg);
            for (int c = 0; c < 2; ++c) m |= ((v >> (8 * c)) & 0xffu) ? (1u << c) : 0u;
        }
        return m;
    }
    __device__ static bool present_m(unsigned m, int row) {
        if (row < R_::FR) return true;
        if (row < R_::CP) return (m >> ((row - R_::FR) / 4)) & 1u;
        return (m >> ((row - R_::CP) / 4)) & 1u;
    }
    __device__ bool present(int k, int row) const { return present_m(cmask(k), row); }
    __device__ SV<T> var_x(int k) const { return kv(Ws<ROBOT>::x, k); }
    __device__ SV<T> var_u(int k) const { return kv(Ws<ROBOT>::u, k); }
};

// The Schur diagonal blocks S_jj and their inverses I_j are symmetric and stored packed (lower
// triangle, row-major: (i, j), j <= i at i (i + 1) / 2 + j; 45 of a block's 81 slots)
__device__ __forceinline__ int pk9(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// The coupling blocks S_{j,j+1} = -M A' (and the first / last, +M A' and -M) share the structure of
// M A' = [[Mc, 0, Mc W'], [beta Ml, Ml, 0], [0, 0, M_LL]]: 27 structural nonzeros of 81, stored
// compactly (row-major over the pattern) until the factorization overwrites the block with the
// dense X_j / Y_j.  cp9(i, j): compact slot of (i, j), or -1 off the pattern.
__device__ __forceinline__ int cp9(int i, int j) {
    if (i < 3) return j == i ? 4 * i : (j >= 6 ? 4 * i + 1 + (j - 6) : -1);
    if (i < 6) return j == i - 3 ? 12 + 2 * (i - 3) : (j == i ? 13 + 2 * (i - 3) : -1);
    return j >= 6 ? 18 + 3 * (i - 6) + (j - 6) : -1;
}

// 3x3 symmetric packed (00,10,11,20,21,22) helpers
template <typename T> __device__ __forceinline__ T sym3(const T *p, int i, int j) {
    if (i < j) { int t = i; i = j; j = t; }
    return p[i * (i + 1) / 2 + j];
}
// inverse of a 4x4 SPD matrix (Cholesky), packed symmetric (10 entries, row i col j<=i)
template <typename T> __device__ void inv4spd(T (&a)[4][4], T *out) {
    T Lm[4][4] = {};
    for (int j = 0; j < 4; ++j) {
        T d = a[j][j];
        for (int q = 0; q < j; ++q) d -= Lm[j][q] * Lm[j][q];
        d = sqrt(d);
        Lm[j][j] = d;
        for (int i = j + 1; i < 4; ++i) {
            T v = a[i][j];
            for (int q = 0; q < j; ++q) v -= Lm[i][q] * Lm[j][q];
            Lm[i][j] = fdiv(v, d);
        }
    }
    T Li[4][4] = {};
    for (int c = 0; c < 4; ++c) Li[c][c] = rcp_nr(Lm[c][c]);
    for (int c = 0; c < 4; ++c) {
        for (int i = c + 1; i < 4; ++i) {
            T v = T(0);
            for (int q = c; q < i; ++q) v += Lm[i][q] * Li[q][c];
            Li[i][c] = -v * Li[i][i];
        }
    }
    int p = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j <= i; ++j) {
            T v = T(0);
            for (int q = i; q < 4; ++q) v += Li[q][i] * Li[q][j];
            out[p++] = v;
        }
}
__device__ __forceinline__ int p4(int i, int j) { if (i < j) { int t = i; i = j; j = t; } return i * (i + 1) / 2 + j; }

// iterative refinement of the corrector direction when its step length falls below
// QP_REFINE_ALPHA, or mu failed to halve in the previous iteration, while the merit is already
// below QP_REFINE_MERIT (late in the solve)
#define QP_REFINE_ALPHA 0.5
#define QP_REFINE_MERIT 1e6
// relative threshold of the primal-infeasibility certificate: OSQP's default eps_prim_inf, the
// value the reference's osqp.setup call runs with
#define QP_EPS_PINF 1e-4

// relative floor on D^-1 in the push-through blocks (K = D^-1 + G W^-1 G')
template <typename T> constexpr double KFLOOR = sizeof(T) == 8 ? 1e-12 : 1e-6;
// The friction block's floor is higher: at a zero contact force all four pyramid rows are active
// and K tends to the rank-3 G W^-1 G' (four rows in 3-D), so a 1e-12 floor let cond(K) reach
// 1e12, the direction's complementarity residual grew to 0.1-0.5 and refinement with the same
// factor could not recover (TALOS QPs with other cost weights stalled at the iteration cap;
// tests/test_gpu_load_qp.py, oracle/ipm_mirror.py).  At 1e-9 every such case solves, with fewer
// refinements; only the direction is perturbed, the stopping test stays on the true residuals.
template <typename T> constexpr double KFLOOR_FR = sizeof(T) == 8 ? 1e-9 : 1e-6;

// in-place Cholesky of an 8x8 SPD matrix, packed lower (row j, col q <= j at j(j+1)/2 + q), with
// a pivot floor relative to the original diagonal
template <typename T> __device__ void chol8(T (&a)[36]) {
    for (int j = 0; j < 8; ++j) {
        const T d0 = a[j * (j + 1) / 2 + j];
        T d = d0;
        for (int q = 0; q < j; ++q) d -= a[j * (j + 1) / 2 + q] * a[j * (j + 1) / 2 + q];
        d = sqrt(fmax(d, T(KFLOOR<T>) * d0));
        const T id = rcp_nr(d);
        a[j * (j + 1) / 2 + j] = id;   // the factor record keeps 1 / L_jj
        for (int i = j + 1; i < 8; ++i) {
            T v = a[i * (i + 1) / 2 + j];
            for (int q = 0; q < j; ++q) v -= a[i * (i + 1) / 2 + q] * a[j * (j + 1) / 2 + q];
            a[i * (i + 1) / 2 + j] = v * id;
        }
    }
}

// (L, t) block factor of knot k from its trust-region and slack rows (s, lambda of rows 0..8):
//   K = D_TR^-1 + Y G_L' (8x8 SPD; Y = G_L W_L^-1; D^-1 floored: at a vertex of the trust
//   region more than 3 rows are active and K -> rank 3),  L L' = K (packed, 1 / L_jj on the
//   diagonal),  z1 = L^-1 1,  D_sl = lambda_8 / s_8,  1 / den = 1 / (D_sl + cw^2 |z1|^2).
// Recomputed in registers by every phase that needs it: cheaper than an HBM round trip.
template <typename T, int ROBOT>
__device__ __forceinline__ void tr_factor(const Ctx<T, ROBOT> &C, const T *s, const T *lm, T (&Lk)[36], T (&z1)[8],
                                          T &iden, T &dsl) {
    const T wl[3] = {C.iWx(6), C.iWx(7), C.iWx(8)};
    const T kfl = T(KFLOOR<T>) * T(8) * (wl[0] + wl[1] + wl[2]);
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int q = 0; q <= j; ++q) {
            T v = T(0);
            for (int i = 0; i < 3; ++i) v += tr_sign<T>(j, i) * tr_sign<T>(q, i) * wl[i];
            if (q == j) v += fmax(fdiv(s[j], lm[j]), kfl);
            Lk[j * (j + 1) / 2 + q] = v;
        }
    chol8(Lk);
    T kap = T(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        T a1 = T(1);
        for (int q = 0; q < j; ++q) a1 -= Lk[j * (j + 1) / 2 + q] * z1[q];
        z1[j] = a1 * Lk[j * (j + 1) / 2 + j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) kap += z1[j] * z1[j];
    dsl = fdiv(lm[8], s[8]);
    iden = rcp_nr(dsl + C.cw * C.cw * kap);
}

// friction block of one contact (4 pyramid rows, s4 / l4 their slacks and multipliers):
// Gw = G W^-1 (4x3) and Kinv = (D^-1 + G W^-1 G')^-1 (packed), with a floor on D^-1 relative to
// tr(G W^-1 G') (at a zero force all four rows are active and K -> rank 3).  Inactive contacts:
// Gw = 0, Kinv = I, so (with rhat = 0 on their rows) they contribute nothing.
template <typename T>
__device__ __forceinline__ void fric_factor(const T (&G)[12], const T (&wi)[3], const T *s4, const T *l4, bool act,
                                            T (&Gw)[4][3], T (&Ki)[10]) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q) Gw[r][q] = G[3 * r + q] * wi[q];
    T Km[4][4], tr = T(0);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            T acc = T(0);
            for (int z = 0; z < 3; ++z) acc += Gw[r][z] * G[3 * q + z];
            Km[r][q] = acc;
        }
    for (int r = 0; r < 4; ++r) tr += Km[r][r];
    const T kfloor = T(KFLOOR_FR<T>) * tr + T(sizeof(T) == 8 ? 1e-300 : 1e-37);
    for (int r = 0; r < 4; ++r) Km[r][r] += fmax(fdiv(s4[r], act ? l4[r] : T(1)), kfloor);
    inv4spd(Km, Ki);
    // masking by arithmetic (every value is finite: lambda -> 1 on inactive rows); per-lane
    // selects here make the compiler split the contact code into divergent regions
    const T on = act ? T(1) : T(0), off = T(1) - on;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q) Gw[r][q] *= on;
#pragma unroll
    for (int q = 0; q < 10; ++q) Ki[q] = (q == 0 || q == 2 || q == 5 || q == 9) ? fma(Ki[q], on, off) : Ki[q] * on;
}

// force block of Phi_u^-1 for one contact: F = W^-1 - Gw' Kinv Gw (packed 00,10,11,20,21,22);
// inactive contacts (Gw = 0): F = W^-1
template <typename T>
__device__ __forceinline__ void fric_F(const T (&Gw)[4][3], const T (&Ki)[10], const T (&wi)[3], T (&F)[6]) {
    int p = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
            T acc = (i == j) ? wi[i] : T(0);
            for (int r = 0; r < 4; ++r)
                for (int q = 0; q < 4; ++q) acc -= Gw[r][i] * Ki[p4(r, q)] * Gw[q][j];
            F[p++] = acc;
        }
}

// inverse diagonal of W' for one contact's controls: 1 / W, except TALOS's CoP coordinates of an
// active contact, whose two bound rows fold in as D-form (1 / (W + D_lo + D_hi)); s, lm indexed by row
template <typename T, int ROBOT, typename SA>
__device__ __forceinline__ void contact_wd(const Ctx<T, ROBOT> &C, int c, bool act, const SA &s, const SA &lm,
                                           T (&wd)[Robot<ROBOT>::NUPC]) {
    constexpr int NUPC = Robot<ROBOT>::NUPC;
#pragma unroll
    for (int q = 0; q < NUPC; ++q) wd[q] = C.iWu(NUPC * c + q);
    if (ROBOT == 1) {
#pragma unroll
        for (int dd = 0; dd < 2; ++dd) {
            const int r0 = Rows<ROBOT>::CP + 4 * c + 2 * dd;
            const T v = T(1) / (C.Wu(NUPC * c + dd) + C.Dform(lm[r0], s[r0]) + C.Dform(lm[r0 + 1], s[r0 + 1]));
            wd[dd] = act ? v : wd[dd];
        }
    }
}

// ------------------------------------------------------------------ phases
// (1) residuals of knot k; returns norm contributions
// prim / dual / comp: residual maxima; mu: complementarity sum over cnt rows; sp / sd: scales of
// the relative tolerances
template <typename T, int ROBOT> struct Norms { T prim, dual, comp, mu, sp, sd, lmax, cnt, smin, lmin; };
template <typename T> __device__ __forceinline__ T big_value() { return std::numeric_limits<T>::max(); }

// Per-knot phases follow load -> compute -> store: every store into the workspace comes after
// the last load (the compiler cannot move a load above a store that may alias it, so interleaving
// them serializes one memory round trip per row).
template <int n, typename T, typename P> __device__ __forceinline__ void ldv(const P &p, T (&o)[n]) {
#pragma unroll
    for (int i = 0; i < n; ++i) o[i] = p[i];
}
template <int n, typename T, typename P> __device__ __forceinline__ void stv(P p, const T (&v)[n]) {
#pragma unroll
    for (int i = 0; i < n; ++i) p[i] = v[i];
}

// The field records are passed as restrict-qualified pointers (field f at p[f * KPC]): loads may
// then move above the stores, so every result row is stored as soon as it is formed and the
// phase never holds the whole knot in registers (holding it serialized the loads of late rows
// behind one memory round trip each).
// Accumulation type of the residuals (kept as a hook: fp64 residuals for the fp32 kernels were
// tried, Acc<float> = double, and cost C3's QP 15% (0.73 -> 0.84 ms) without changing its exits;
// the fp32 floor on Solo12 trot came from the dual scale, see the multiplier term below).
template <typename T> struct Acc { using type = T; };

// PART (four-wave workgroups with one pass of knots, split_knots): -1 the whole knot; 0 the state
// part (dynamics and boundary rows, trust-region and slack rows, r_dx, r_dt); 1 the contact part
// (friction / CoP rows, r_du).  The norms of both parts meet in the block reduction.
template <typename T, int ROBOT, int PART = -1>
__device__ __forceinline__ void resid_knot(const Ctx<T, ROBOT> &C, int k, Norms<T, ROBOT> &nm, const T *__restrict__ stp,
                                           const T *__restrict__ xs, const T *__restrict__ us, const T *__restrict__ ts,
                                           const T *__restrict__ ss, const T *__restrict__ ls, const T *__restrict__ nus,
                                           T *__restrict__ rdx_o, T *__restrict__ rdt_o, T *__restrict__ rdu_o,
                                           T *__restrict__ rde_o, T *__restrict__ rdi_o) {
    using S = Stage<ROBOT>;
    using R_ = Rows<ROBOT>;
    using A = typename Acc<T>::type;
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    constexpr int ld = KPC;
    const int N = C.N;
    const bool hu = k < N;
    const DevParams<T> &P = *C.prm;
    const SV<const T> st{stp};
    const unsigned msk = C.cmask(k);
    // non-finite detector: the norms are fmax / fmin reductions, which drop NaNs, so every residual
    // also enters a sum that reaches nm.mu multiplied by zero (NaN or inf there makes mu NaN; the
    // stopping test and the polished iterate's verification check mu)
    A nanchk = A(0);
    A x[9], u[NU], x1[9], nk[9], n1[9], w[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        x[i] = xs[i * ld];
        x1[i] = xs[i * ld + 1];   // x_{k+1} (k = N: unused)
        nk[i] = nus[i * ld];      // nu blocks k, k + 1
        n1[i] = nus[i * ld + 1];
    }
    if (sizeof(T) == 4 && PART != 1) {
        // fp32: the dual scale also counts the multipliers the rows sum.  E' nu = -nu_k + A_k' nu_{k+1}
        // cancels (Solo12 trot: |nu| ~ 1e5 against |E' nu| ~ 2e3), and |nu| in fp32 alone carries
        // ~6e-8 |nu| of rounding into every dual row: without this term the 1e-6 relative test sat
        // below the representable floor (merit 2.4-3 for ever, tests/golden trot_f32).
        A nmag = A(0);
#pragma unroll
        for (int i = 0; i < 9; ++i) nmag = fmax(nmag, fmax(fabs(nk[i]), fabs(n1[i])));
        nm.sd = fmax(nm.sd, T(nmag));
    }
#pragma unroll
    for (int i = 0; i < NU; ++i) u[i] = us[i * ld];   // k = N: padding column (values unused)
    for (int i = 0; i < 3; ++i) w[i] = st[S::W + i];
    const A t = ts[0], beta = C.beta, cw = C.cw;
    // E' nu at knot k (kept for the dual rows at the end)
    A ex[9], eu[NU];
    for (int i = 0; i < 9; ++i) ex[i] = (k == 0) ? nk[i] : -nk[i];
    if (k == N) for (int i = 0; i < 9; ++i) ex[i] += n1[i];
    if (hu && PART == 1) opBT<A, ROBOT>(st, n1, eu);
    if (hu && PART != 1) {
        A a[9];
        opAT(w, beta, n1, a);
        for (int i = 0; i < 9; ++i) ex[i] += a[i];
        if (PART != 0) opBT<A, ROBOT>(st, n1, eu);
        // dynamics row block 1 + k first: its loads (x_{k+1}, r_k) are then dead before the rows
        A ax[9], bu[9];
        opA(w, beta, x, ax);
        opB<A, ROBOT>(st, u, bu);
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const A ez = ax[i] + bu[i] - x1[i], r = st[S::R + i];
            const A re = ez - r;
            rde_o[i * ld + 1 + k] = T(re);
            nanchk += re;
            nm.prim = fmax(nm.prim, T(fabs(re)));
            nm.sp = fmax(nm.sp, T(fmax(fabs(ez), fabs(r))));
        }
    }
    if (PART != 1 && (k == 0 || k == N)) {   // boundary rows: block 0 (initial state) / N + 1 (final state)
        const T *xb = C.xbar + (size_t)k * 9;
        for (int i = 0; i < 9; ++i) {
            const A rb = x[i] - A(xb[i]);
            rde_o[i * ld + (k == 0 ? 0 : N + 1)] = T(rb);
            nm.prim = fmax(nm.prim, T(fabs(rb)));
            nm.sp = fmax(nm.sp, T(fmax(fabs(x[i]), A(fabs(xb[i])))));
        }
    }
    // inequality rows: r_i = g'z - h + s, complementarity and norms; G' lambda accumulated on the fly
    A gL[3] = {A(0), A(0), A(0)}, gt = A(0), gu[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) gu[i] = A(0);
    // complementarity sums in short per-group chains (one long serial chain made the scheduler
    // keep every row's product live until the end); the row count is exact in integers
    T mug = T(0);
    auto row = [&](int r, bool pr, A g, A h) {
        const A v = g - h, sr = ss[r * ld], lr = ls[r * ld];
        rdi_o[r * ld] = pr ? T(v + sr) : T(0);
        nanchk += pr ? v + sr + lr : A(0);
        const T c = pr ? T(sr * lr) : T(0);
        nm.prim = fmax(nm.prim, pr ? T(v) : T(0));
        nm.sp = fmax(nm.sp, pr ? T(fmax(fabs(g), fabs(g - v))) : T(0));
        nm.comp = fmax(nm.comp, c);
        mug += c;
        nm.lmax = fmax(nm.lmax, pr ? T(lr) : T(0));
        nm.smin = fmin(nm.smin, pr ? T(sr) : big_value<T>());   // (the polished iterate's sign check)
        nm.lmin = fmin(nm.lmin, pr ? T(lr) : big_value<T>());
        return pr ? lr : A(0);
    };
    nm.cnt += T((PART != 1 ? 9 : 0) + (hu && PART != 0 ? 4 * (1 + Robot<ROBOT>::COP) * __builtin_popcount(msk) : 0));
    if (PART != 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const A g = tr_sign<A>(j, 0) * x[6] + tr_sign<A>(j, 1) * x[7] + tr_sign<A>(j, 2) * x[8] + cw * t;
            const A lr = row(j, true, g, st[S::BTR + j]);
            for (int i = 0; i < 3; ++i) gL[i] += tr_sign<A>(j, i) * lr;
            gt += cw * lr;
        }
        gt -= row(8, true, -t, A(0));
        nm.mu += mug;
    }
#pragma unroll
    for (int c = 0; c < (PART != 0 ? NC : 0); ++c) {
        mug = T(0);
        const bool pr = hu && ((msk >> c) & 1u);
        const auto cs = st + (S::CON + S::CS * c);
        const A *f = u + NUPC * c + FO;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const A g0 = cs[S::G + 3 * r], g1 = cs[S::G + 3 * r + 1], g2 = cs[S::G + 3 * r + 2];
            const A lr = row(R_::FR + 4 * c + r, pr, g0 * f[0] + g1 * f[1] + g2 * f[2], cs[S::H + r]);
            gu[NUPC * c + FO] += g0 * lr;
            gu[NUPC * c + FO + 1] += g1 * lr;
            gu[NUPC * c + FO + 2] += g2 * lr;
        }
        if (ROBOT == 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {   // cop <= hi | -cop <= -lo (lo = -(lxn | lyn))
                const int dd = q / 2;
                const A cop = u[NUPC * c + dd];
                const A lr = (q % 2 == 0) ? row(R_::CP + 4 * c + q, pr, cop, P.foot_range[dd == 0 ? 0 : 2])
                                          : row(R_::CP + 4 * c + q, pr, -cop, P.foot_range[dd == 0 ? 1 : 3]);
                gu[NUPC * c + dd] += (q % 2 == 0) ? lr : -lr;
            }
        }
        nm.mu += mug;
    }
    if (PART != 1) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const A hx = A(C.Wx(i)) * x[i], q = st[S::QX + i];
        const A g = (i >= 6) ? gL[i - 6] : A(0);
        const A rd = hx + q + ex[i] + g;
        rdx_o[i * ld] = T(rd);
        nanchk += rd;
        nm.dual = fmax(nm.dual, T(fabs(rd)));
        nm.sd = fmax(nm.sd, T(fmax(fabs(hx), fmax(fabs(q), fmax(fabs(ex[i]), fabs(g))))));
    }
    const A rdt = A(1) + gt;
    rdt_o[0] = T(rdt);
    nm.dual = fmax(nm.dual, T(fabs(rdt)));
    nm.sd = fmax(nm.sd, T(1));
    }
    if (hu && PART != 0) {
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            const A h = A(C.Wu(i)) * u[i];
            const A rd = h + eu[i] + gu[i];
            rdu_o[i * ld] = T(rd);
            nanchk += rd;
            nm.dual = fmax(nm.dual, T(fabs(rd)));
            nm.sd = fmax(nm.sd, T(fmax(fabs(h), fmax(fabs(eu[i]), fabs(gu[i])))));
        }
    }
    nm.mu += T(A(0) * nanchk);
}

template <typename T, int ROBOT, int PART = -1> __device__ PHASE_ATTR void phase_residual(const Ctx<T, ROBOT> &C, int k, Norms<T, ROBOT> &nm) {
    T *ws = C.ws;
    resid_knot<T, ROBOT, PART>(C, k, nm, C.stage + k, ws + WF(x) * KPC + k, ws + WF(u) * KPC + k, ws + WF(t) * KPC + k,
                         ws + WF(s) * KPC + k, ws + WF(l) * KPC + k, ws + WF(nu) * KPC + k, ws + WF(rdx) * KPC + k,
                         ws + WF(rdt) * KPC + k, ws + WF(rdu) * KPC + k, ws + WF(rde) * KPC, ws + WF(rdi) * KPC + k);
}

// (1b) primal-infeasibility certificate terms of knot k (rare; after the residual phase):
// cm[0] = max |E'nu + G'lambda| = |r_d - H z - q| over the knot's x, t, u entries, cm[1] = max |nu|
// (lambda's max comes from the residual phase), cs += b'nu + h'lambda over the rows the knot owns
template <typename T, int ROBOT>
__device__ PHASE_ATTR void phase_cert(const Ctx<T, ROBOT> &C, int k, T (&cm)[2], T &cs) {
    using S = Stage<ROBOT>;
    using R_ = Rows<ROBOT>;
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC;
    const int N = C.N;
    const bool hu = k < N;
    const SV<const T> st = C.st(hu ? k : 0);
    const unsigned msk = C.cmask(k);
    const SV<T> x = C.var_x(k), rdx = C.kv(WF(rdx), k), lm = C.kv(WF(l), k), nk = C.bv(WF(nu), k),
                n1 = C.bv(WF(nu), k + 1);
    for (int i = 0; i < 9; ++i) {
        cm[0] = fmax(cm[0], fabs(rdx[i] - C.Wx(i) * x[i] - C.st(k)[S::QX + i]));
        cm[1] = fmax(cm[1], fabs(nk[i]));
        if (k == N) cm[1] = fmax(cm[1], fabs(n1[i]));
    }
    cm[0] = fmax(cm[0], fabs(C.kv(WF(rdt), k)[0] - T(1)));
    if (hu) {
        const SV<T> u = C.var_u(k), rdu = C.kv(WF(rdu), k);
        for (int i = 0; i < NU; ++i) cm[0] = fmax(cm[0], fabs(rdu[i] - C.Wu(i) * u[i]));
        for (int i = 0; i < 9; ++i) cs = fma(st[S::R + i], n1[i], cs);
    }
    if (k == 0 || k == N) {
        const T *xb = C.xbar + (size_t)k * 9;
        for (int i = 0; i < 9; ++i) cs = fma(xb[i], k == 0 ? nk[i] : n1[i], cs);
    }
    const SV<const T> sk = C.st(k);
    for (int j = 0; j < 8; ++j) cs = fma(sk[S::BTR + j], lm[j], cs);   // slack rows: h = 0
    if (!hu) return;
    for (int c = 0; c < NC; ++c) {
        if (!((msk >> c) & 1u)) continue;
        const auto cs_ = st + (S::CON + S::CS * c);
        for (int r = 0; r < 4; ++r) cs = fma(cs_[S::H + r], lm[R_::FR + 4 * c + r], cs);
        if (ROBOT == 1)
            for (int q = 0; q < 4; ++q) {   // cop <= hi | -cop <= -lo: h = hi | lxn, lyn
                const int dd = q / 2;
                cs = fma(C.prm->foot_range[dd == 0 ? (q % 2) : 2 + (q % 2)], lm[R_::CP + 4 * c + q], cs);
            }
    }
    (void)NUPC;
}

// (2) Phi factors of knot k
// s, lambda and the friction rows G of knot k: loaded once for the Phi factors and the
// predictor's w, which run back to back on the same knot (the factor stores in between would
// otherwise force w to reload them)
template <typename T, int ROBOT> struct KnotSL {
    T s[Rows<ROBOT>::NI], l[Rows<ROBOT>::NI], G[Robot<ROBOT>::NC][12];
};
template <typename T, int ROBOT> __device__ __forceinline__ void load_knot_sl(const Ctx<T, ROBOT> &C, int k, KnotSL<T, ROBOT> &kl) {
    using S = Stage<ROBOT>;
    constexpr int NC = Robot<ROBOT>::NC;
    ldv(C.kv(WF(s), k), kl.s);
    ldv(C.kv(WF(l), k), kl.l);
    const auto st = C.st(k < C.N ? k : 0);
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int e = 0; e < 12; ++e) kl.G[c][e] = st[S::CON + S::CS * c + S::G + e];
}

// PART as in resid_knot: 0 the (L, t) block (facx), 1 the contacts (facu), -1 both
template <typename T, int ROBOT, int PART = -1>
__device__ __forceinline__ void phase_factor(const Ctx<T, ROBOT> &C, int k, const KnotSL<T, ROBOT> &kl) {
    using R_ = Rows<ROBOT>;
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    const int N = C.N;
    const T *s = kl.s, *lm = kl.l;
    const unsigned msk = C.cmask(k);
    const auto &Gr = kl.G;
    const SV<T> fx = C.kv(WF(facx), k);
    // (L, t) block in push-through form (no D * r product, no cancellation as rows pin L or t),
    // see tr_factor; stored: M_LL = [Phi^-1]_LL = W_L^-1 - Z'Z + cw^2 g g' / den with
    // Z = L^-1 Y, g = Z' z1 (phase_sblock).  L, z1, den are recomputed where they are used.
    if (PART != 1) {
    const T wl[3] = {C.iWx(6), C.iWx(7), C.iWx(8)};
    T Lk[36], z1[8], iden, dsl;
    tr_factor(C, s, lm, Lk, z1, iden, dsl);
    T Z[8][3];
    for (int j = 0; j < 8; ++j) {
        T az[3];
        for (int i = 0; i < 3; ++i) az[i] = tr_sign<T>(j, i) * wl[i];
        for (int q = 0; q < j; ++q) {
            const T l = Lk[j * (j + 1) / 2 + q];
            for (int i = 0; i < 3; ++i) az[i] -= l * Z[q][i];
        }
        const T il = Lk[j * (j + 1) / 2 + j];
        for (int i = 0; i < 3; ++i) Z[j][i] = az[i] * il;
    }
    T g[3] = {0, 0, 0};
    for (int j = 0; j < 8; ++j)
        for (int i = 0; i < 3; ++i) g[i] += Z[j][i] * z1[j];
    for (int i = 0, p = 0; i < 3; ++i)
        for (int q = 0; q <= i; ++q, ++p) {
            T zz = T(0);
            for (int j = 0; j < 8; ++j) zz += Z[j][i] * Z[j][q];
            fx[FX_ML + p] = (i == q ? wl[i] : T(0)) - zz + C.cw * C.cw * g[i] * g[q] * iden;
        }
    }
    if (k >= N) return;
#pragma unroll
    for (int c = 0; c < (PART != 0 ? NC : 0); ++c) {
        const SV<T> fu = C.kv(WF(facu), k) + c * FU;
        const bool act = (msk >> c) & 1u;
        // Winvd: inverse diagonal of W' (CoP rows fold into their coordinate's diagonal); TALOS only:
        // Solo12's is 1 / Wu, which phase_sblock does not need (no CoP columns)
        if (ROBOT == 1)
            for (int q = 0; q < NUPC; ++q) fu[FU_WI + q] = C.iWu(NUPC * c + q);
        if (ROBOT == 1 && act) {
            for (int dd = 0; dd < 2; ++dd) {
                const int r0 = R_::CP + 4 * c + 2 * dd;
                fu[FU_WI + dd] = T(1) / (C.Wu(NUPC * c + dd) + C.Dform(lm[r0], s[r0]) + C.Dform(lm[r0 + 1], s[r0 + 1]));
            }
        }
        const T wi[3] = {C.iWu(NUPC * c + FO), C.iWu(NUPC * c + FO + 1), C.iWu(NUPC * c + FO + 2)};
        if (!act) {
            fu[FU_F] = wi[0]; fu[FU_F + 1] = T(0); fu[FU_F + 2] = wi[1]; fu[FU_F + 3] = T(0); fu[FU_F + 4] = T(0); fu[FU_F + 5] = wi[2];
            continue;
        }
        T Gw[4][3], Ki[10];
        fric_factor(Gr[c], wi, s + R_::FR + 4 * c, lm + R_::FR + 4 * c, true, Gw, Ki);
        // F = W^-1 - Gw' Kinv Gw  (stored for phase_sblock)
        T F[6];
        fric_F(Gw, Ki, wi, F);
        for (int q = 0; q < 6; ++q) fu[FU_F + q] = F[q];
    }
}

// local solve of the (L, t) block of knot k (unknowns dL, dt, dlam_TR[8], dlam_slack):
//   W_L dL + G_L' dlam = vL;  cw 1'dlam - dlam_sl = vt;  G_L dL + cw 1 dt - D^-1 dlam = -rh[0:8];
//   -dt - D_sl^-1 dlam_sl = -rh[8]
// dt = (vt + D_sl rh_8 - cw z1'y) / den with y = L^-1 (Y vL + rh);  dlam = L^-T (y + cw dt z1);
// dL = W_L^-1 (vL - G_L' dlam);  dlam_sl = cw 1'dlam - vt  (the t row of the dual residual)
template <typename T, int ROBOT>
__device__ __forceinline__ void tr_local(const Ctx<T, ROBOT> &C, const T (&Lk)[36], const T (&z1)[8], T fdsl, T fden,
                                         const T *vL, T vt, const T *rh, T *dL, T &dt, T *dlt, T &dls) {
    const T wl[3] = {rcp_nr(C.Wx(6)), rcp_nr(C.Wx(7)), rcp_nr(C.Wx(8))};
    T y[8];
    for (int j = 0; j < 8; ++j) {
        T v = rh[j];
        for (int i = 0; i < 3; ++i) v += tr_sign<T>(j, i) * wl[i] * vL[i];
        for (int q = 0; q < j; ++q) v -= Lk[j * (j + 1) / 2 + q] * y[q];
        y[j] = v * Lk[j * (j + 1) / 2 + j];
    }
    T zy = T(0);
    for (int j = 0; j < 8; ++j) zy += z1[j] * y[j];
    dt = (vt + fdsl * rh[8] - C.cw * zy) * fden;
    for (int j = 0; j < 8; ++j) y[j] += C.cw * dt * z1[j];
    for (int j = 7; j >= 0; --j) {
        T v = y[j];
        for (int q = j + 1; q < 8; ++q) v -= Lk[q * (q + 1) / 2 + j] * dlt[q];
        dlt[j] = v * Lk[j * (j + 1) / 2 + j];
    }
    T sl = T(0);
    for (int j = 0; j < 8; ++j) sl += dlt[j];
    dls = C.cw * sl - vt;
    for (int i = 0; i < 3; ++i) {
        T gl = T(0);
        for (int j = 0; j < 8; ++j) gl += tr_sign<T>(j, i) * dlt[j];
        dL[i] = wl[i] * (vL[i] - gl);
    }
}

// (3) S blocks owned by knot k
template <typename T, int ROBOT> __device__ PHASE_ATTR void phase_sblock(const Ctx<T, ROBOT> &C, int k) {
    using S = Stage<ROBOT>;
    constexpr int NC = Robot<ROBOT>::NC;
    const int N = C.N;
    const T beta = C.beta;
    const bool hu = k < N;
    // loads: M_k, M_{k+1} (1/Wx[0:6] | M_LL packed), the stage's A/B data, the contacts' F, W'^-1
    T f0[12], f1[12];
    for (int i = 0; i < 6; ++i) f0[i] = f1[i] = C.iWx(i);
    {
        T m0[6], m1[6];
        ldv(C.kv(WF(facx), k) + FX_ML, m0);
        ldv(C.kv(WF(facx), hu ? k + 1 : k) + FX_ML, m1);
        for (int i = 0; i < 6; ++i) { f0[6 + i] = m0[i]; f1[6 + i] = m1[i]; }
    }
    const auto st = C.st(k);
    T w[3], w1[3];
    ldv(st + S::W, w);
    ldv(C.st(k + 1 < N ? k + 1 : k) + S::W, w1);
    T al[NC], lev[NC][3], F[NC][6], wd[NC][6];
    for (int c = 0; c < NC; ++c) {
        const auto cs = st + (S::CON + S::CS * c);
        al[c] = hu ? cs[S::ALPHA] : T(0);
        ldv(cs + S::LEVER, lev[c]);
        const SV<T> fu = C.kv(WF(facu), k) + c * FU;
        ldv(fu + FU_F, F[c]);
        if (ROBOT == 1) ldv(fu + FU_WI, wd[c]);
    }
    T bc[NC][6], bt[NC][3];
    if (ROBOT == 1)
        for (int c = 0; c < NC; ++c) {
            const auto cs = st + (S::CON + S::CS * c);
            ldv(cs + S::BCOP, bc[c]);
            ldv(cs + S::BTAU, bt[c]);
        }
    auto Mfull = [&](const T *f, int i, int j) -> T {   // M_k entry
        if (i < 6 || j < 6) return (i == j && i < 6) ? f[i] : T(0);
        return sym3(f + 6, i - 6, j - 6);
    };
    // M A' blocks:  [[Mc, 0, Mc W'], [beta Ml, Ml, 0], [0, 0, ML]]
    auto MAt = [&](const T *f, const T *wv, int i, int j) -> T {
        const T Wm[3][3] = {{0, -wv[2], wv[1]}, {wv[2], 0, -wv[0]}, {-wv[1], wv[0], 0}};
        if (i < 3) {
            if (j < 3) return (i == j) ? f[i] : T(0);
            if (j < 6) return T(0);
            return f[i] * Wm[j - 6][i];
        }
        if (i < 6) {
            if (j < 3) return (i - 3 == j) ? beta * f[i] : T(0);
            if (j < 6) return (i == j) ? f[i] : T(0);
            return T(0);
        }
        if (j < 6) return T(0);
        return sym3(f + 6, i - 6, j - 6);
    };
    if (k == 0) {
        T *Sd = C.Sd, *So = C.So;
        for (int i = 0; i < 9; ++i)
            for (int j = 0; j < 9; ++j) {
                if (j <= i) Sd[pk9(i, j)] = Mfull(f0, i, j);
                if (cp9(i, j) >= 0) So[cp9(i, j)] = MAt(f0, w, i, j);   // compact coupling block
            }
    }
    if (k == N) {
        T *Sd = C.Sd + (size_t)(N + 1) * 81;
        for (int i = 0; i < 9; ++i)
            for (int j = 0; j <= i; ++j) Sd[pk9(i, j)] = Mfull(f0, i, j);
        return;
    }
    const T Wm[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    T Sm[9][9];
    // A M A'
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j) Sm[i][j] = T(0);
    const T *mc = f0, *ml = f0 + 3;
    for (int a = 0; a < 3; ++a) {
        Sm[a][a] = mc[a] + beta * beta * ml[a];
        Sm[a][3 + a] = Sm[3 + a][a] = beta * ml[a];
        Sm[3 + a][3 + a] = ml[a];
    }
    for (int a = 0; a < 3; ++a)
        for (int bb = 0; bb < 3; ++bb) {
            Sm[a][6 + bb] = mc[a] * Wm[bb][a];   // Mc W'
            Sm[6 + bb][a] = Sm[a][6 + bb];
            T acc = sym3(f0 + 6, a, bb);
            for (int q = 0; q < 3; ++q) acc += Wm[a][q] * mc[q] * Wm[bb][q];
            Sm[6 + a][6 + bb] = acc;
        }
    // B Phi_u^-1 B'  (inactive contacts: alpha = 0)
    for (int c = 0; c < NC; ++c) {
        const T *lv = lev[c];
        const T Lm[3][3] = {{0, -lv[2], lv[1]}, {lv[2], 0, -lv[0]}, {-lv[1], lv[0], 0}};
        T Fm[3][3], FL[3][3];   // F, F Lambda'
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Fm[i][j] = sym3(F[c], i, j);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) FL[i][j] = Fm[i][0] * Lm[j][0] + Fm[i][1] * Lm[j][1] + Fm[i][2] * Lm[j][2];
        const T a2 = al[c] * al[c];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                Sm[3 + i][3 + j] += a2 * Fm[i][j];
                Sm[3 + i][6 + j] += a2 * FL[i][j];
                Sm[6 + j][3 + i] += a2 * FL[i][j];
                T acc = T(0);
                for (int q = 0; q < 3; ++q) acc += Lm[i][q] * FL[q][j];
                Sm[6 + i][6 + j] += a2 * acc;
            }
        if (ROBOT == 1) {
            const T on = al[c] != T(0) ? T(1) : T(0);
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j)
                    Sm[6 + i][6 + j] += on * (bc[c][2 * i] * wd[c][0] * bc[c][2 * j] +
                                              bc[c][2 * i + 1] * wd[c][1] * bc[c][2 * j + 1] +
                                              bt[c][i] * wd[c][5] * bt[c][j]);
        }
    }
    // + M_{k+1}
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j) Sm[i][j] += Mfull(f1, i, j);
    T *Sd = C.Sd + (size_t)(1 + k) * 81;   // packed lower triangle
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) Sd[i * (i + 1) / 2 + j] = Sm[i][j];
    T *So = C.So + (size_t)(1 + k) * 81;   // compact coupling block (cp9)
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int j = 0; j < 9; ++j)
            if (cp9(i, j) >= 0) So[cp9(i, j)] = k + 1 < N ? -MAt(f1, w1, i, j) : -Mfull(f1, i, j);
}

// (4) two-ended ("twisted") block-Thomas factorization of the SPD block-tridiagonal S with
// explicit symmetric inverses.  Lanes 0..31 eliminate from the top, lanes 32..63 from the bottom
// (one wave per problem, so four problems share a CU), and the two ends meet at block m:
//   top    (j < m):  X_j = S_{j,j-1} I_{j-1},  I_j = (S_jj - X_j S_{j-1,j})^-1      So[j-1] <- X_j
//   bottom (j > m):  Y_j = S_{j,j+1} I_{j+1},  I_j = (S_jj - Y_j S_{j+1,j})^-1      So[j]   <- Y_j
//   meet   (j = m):  I_m = (S_mm - X_m S_{m-1,m} - Y_m S_{m+1,m})^-1
// Sd[j] holds S_jj on input and I_j on output (packed, pk9), So[j] holds S_{j,j+1} on input (both in the
// workspace, so the kernel's LDS stays small and several problems share a CU).  Each half-wave
// keeps its previous inverse and the step's blocks in a small LDS scratch; the next step's raw
// blocks are fetched one step ahead (a step is thousands of cycles).  Inverses by Gauss-Jordan
// sweeps over the 32 lanes of a half (SPD: no pivoting) with a pivot floor relative to the
// original diagonal (near the solution of a degenerate QP the Schur blocks are differences of
// O(M) numbers).  Per-half LDS scratch: A (current) | P (previous inverse) | Xb | Ob | Dd (original diagonal) | Dn (S_jj).
template <typename T> __device__ __forceinline__ T dot9(const LdsT<T> *a, const LdsT<T> *b) {
    T av[9], bv[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) { av[q] = a[q]; bv[q] = b[q]; }
    T s0 = av[0] * bv[0], s1 = av[1] * bv[1], s2 = av[2] * bv[2];
#pragma unroll
    for (int q = 3; q < 9; q += 3) { s0 = fma(av[q], bv[q], s0); s1 = fma(av[q + 1], bv[q + 1], s1); s2 = fma(av[q + 2], bv[q + 2], s2); }
    return s0 + s1 + s2;
}
constexpr int TW_SCRATCH = 5 * 88 + 16;

// One step over L lanes: L = 32 is a half-wave (one end of the twisted recurrence), L = 64 the
// whole wave (the meeting block).  Lane l of the group holds the NE = ceil(81 / L) elements
// e = l + L q of the 9x9 blocks (the last one clamped and masked past 80).
// With vb != nullptr the step also runs the forward elimination of the right-hand side held in
// vb (the predictor's, known before the factorization): y_j = b_j - X_j y_jx (an end), or at the
// meeting block x_m = I_m (b_m - X_m y_{m-1} - Y_m y_{m+1}), with X_j / Y_j read from the LDS
// scratch while they are there.
//   Op, Ip: X = Op' Ip, A -= X Op   (Op = S_{j-1,j}; the bottom end lands S_{j,j+1}' here, so
//           the same code forms Y_j = S_{j,j+1} I_{j+1} and A -= Y_j S_{j,j+1}')
//   Oq, Iq: Y = Oq Iq, A -= Y Oq'   (meeting block only)
template <typename T, int L>
__device__ __forceinline__ void tw_step(const LdsT<T> *Dn, const LdsT<T> *Op, const LdsT<T> *Ip, const LdsT<T> *Oq,
                                        const LdsT<T> *Iq, GlbT<T> *Xout, GlbT<T> *Yout, GlbT<T> *Iout, LdsT<T> *A, LdsT<T> *P,
                                        LdsT<T> *Xb, LdsT<T> *Dd, LdsT<T> *vb = nullptr, int j = 0, int jx = 0,
                                        int jy = 0, unsigned long long *sub = nullptr) {
    constexpr int NE = (81 + L - 1) / L;
#ifdef CMPC_STAMPS
    unsigned long long tq = __builtin_amdgcn_s_memtime();
#define SUBSTAMP(i) do { if (sub) { const unsigned long long tn = __builtin_amdgcn_s_memtime(); sub[i] += tn - tq; tq = tn; } } while (0)
#else
#define SUBSTAMP(i) do { } while (0)
#endif
    // lanes past element 80 hold a clamped copy of element 80 and compute bit-identical values,
    // so their LDS stores (the same value to the same slot) need no mask; global stores keep it
    const int l = threadIdx.x & (L - 1);
    int e[NE], ii[NE], cc[NE];
    bool ok[NE];
#pragma unroll
    for (int q = 0; q < NE; ++q) {
        ok[q] = l + L * q < 81;
        e[q] = ok[q] ? l + L * q : 80;
        ii[q] = e[q] / 9;
        cc[q] = e[q] % 9;
    }
    T a[NE], x[NE], y[NE];
#pragma unroll
    for (int q = 0; q < NE; ++q) { a[q] = Dn[e[q]]; x[q] = T(0); y[q] = T(0); }
    T rv = (vb && l < 9) ? vb[j * 9 + l] : T(0);   // b_j (fused elimination)
    // original diagonal of S_jj (pivot floor): entries 0, 10, ..., 80
#pragma unroll
    for (int q = 0; q < NE; ++q)
        if (e[q] % 10 == 0) Dd[e[q] / 10] = a[q];
    // 9-term dot products with every LDS operand read before the first multiply
    auto dot = [&](auto fa, auto fb) -> T {
        T u[9], v[9];
#pragma unroll
        for (int m = 0; m < 9; ++m) { u[m] = fa(m); v[m] = fb(m); }
        T s0 = u[0] * v[0], s1 = u[1] * v[1], s2 = u[2] * v[2];
#pragma unroll
        for (int m = 3; m < 9; m += 3) { s0 = fma(u[m], v[m], s0); s1 = fma(u[m + 1], v[m + 1], s1); s2 = fma(u[m + 2], v[m + 2], s2); }
        return s0 + s1 + s2;
    };
    if (Op) {   // X = Op' I_{j-1};  A -= X Op
#pragma unroll
        for (int q = 0; q < NE; ++q)
            x[q] = dot([&](int m) { return Op[m * 9 + ii[q]]; }, [&](int m) { return Ip[m * 9 + cc[q]]; });
#pragma unroll
        for (int q = 0; q < NE; ++q) Xb[e[q]] = x[q];
        wave_sync();
        if (vb && l < 9) rv -= dot9(Xb + l * 9, vb + jx * 9);
#pragma unroll
        for (int q = 0; q < NE; ++q)
            a[q] -= dot([&](int m) { return Xb[ii[q] * 9 + m]; }, [&](int m) { return Op[m * 9 + cc[q]]; });
        wave_sync();
    }
    if (Oq) {   // Y = Oq I_{j+1};  A -= Y Oq'   (Oq = S_{j,j+1})
#pragma unroll
        for (int q = 0; q < NE; ++q)
            y[q] = dot([&](int m) { return Oq[ii[q] * 9 + m]; }, [&](int m) { return Iq[m * 9 + cc[q]]; });
#pragma unroll
        for (int q = 0; q < NE; ++q) Xb[e[q]] = y[q];
        wave_sync();
        if (vb && l < 9) rv -= dot9(Xb + l * 9, vb + jy * 9);
#pragma unroll
        for (int q = 0; q < NE; ++q)
            a[q] -= dot([&](int m) { return Xb[ii[q] * 9 + m]; }, [&](int m) { return Oq[cc[q] * 9 + m]; });
        wave_sync();
    }
#pragma unroll
    for (int q = 0; q < NE; ++q) {
        A[e[q]] = a[q];
        if (!ok[q]) continue;
        if (Op) Xout[e[q]] = x[q];
        if (Oq) Yout[e[q]] = y[q];
    }
    wave_sync();
    SUBSTAMP(0);
    // Gauss-Jordan, branch-free, with the next pivot's reciprocal computed one pivot ahead: every
    // lane forms A'_{c+1,c+1} = A_{c+1,c+1} - (A_{c+1,c} / p_c) A_{c,c+1} (the same expression the
    // owning lane stores) from broadcast reads, so its reciprocal chain overlaps the update
    T ip = rcp_nr(fmax(A[0], T(1e-13) * Dd[0]));
#pragma unroll
    for (int c = 0; c < 9; ++c) {
        T aic[NE], acj[NE];
#pragma unroll
        for (int q = 0; q < NE; ++q) { aic[q] = A[ii[q] * 9 + c]; acj[q] = A[c * 9 + cc[q]]; }
        T ipn = T(0);
        if (c < 8) {
            const T ncc = A[(c + 1) * 9 + c + 1], nic = A[(c + 1) * 9 + c], nci = A[c * 9 + c + 1];
            ipn = rcp_nr(fmax(fma(-(nic * ip), nci, ncc), T(1e-13) * Dd[c + 1]));
        }
#pragma unroll
        for (int q = 0; q < NE; ++q) {
            const T mi = aic[q] * ip;
            const T gen = fma(-mi, acj[q], a[q]), row = acj[q] * ip, col = -mi;
            // selects, not branches (the compiler otherwise splits the lanes into divergent paths)
            const bool ic = __builtin_unpredictable(ii[q] == c), jc = __builtin_unpredictable(cc[q] == c);
            a[q] = ic ? (jc ? ip : row) : (jc ? col : gen);
        }
        wave_sync();
#pragma unroll
        for (int q = 0; q < NE; ++q) A[e[q]] = a[q];
        wave_sync();
        ip = ipn;
    }
    SUBSTAMP(1);
#pragma unroll
    for (int q = 0; q < NE; ++q) {
        P[e[q]] = a[q];
        if (ok[q] && ii[q] >= cc[q]) Iout[ii[q] * (ii[q] + 1) / 2 + cc[q]] = a[q];   // packed
    }
    if (vb) {
        if (Op && Oq) {   // meeting block: x_m = I_m (b_m - X_m y_{m-1} - Y_m y_{m+1})
            if (l < 9) Xb[l] = rv;
            wave_sync();
            if (l < 9) vb[j * 9 + l] = dot9(A + l * 9, Xb);
        } else if (l < 9) {
            vb[j * 9 + l] = rv;
        }
    }
    wave_sync();
    SUBSTAMP(2);
#undef SUBSTAMP
}

// One end's step on a half-wave with the symmetric structure used (the ends' counterpart of
// tw_step<T, 32>): X = Op' I_{j-1} is formed whole (81 elements, three per lane: it is not
// symmetric), A = S_jj - X Op and its Gauss-Jordan inverse only on the upper triangle (45
// elements, two per lane).  Gauss-Jordan on a symmetric matrix keeps A[j][i] = A[i][j] while i
// and j are both pivoted or both not, and A[j][i] = -A[i][j] while exactly one is: at pivot c an
// element reads A[i][c] = U[min(i,c)][max(i,c)] and A[c][j] = (c > j ? -1 : 1) U[min][max] from
// the stored upper triangle U.  The inverse is mirrored into P (full, for the next step) and
// stored packed into Iout.
template <typename T, int L>
__device__ __forceinline__ void tw_step_sym(const LdsT<T> *Dn, const LdsT<T> *Op, const LdsT<T> *Ip, GlbT<T> *Xout, GlbT<T> *Iout,
                                            LdsT<T> *A, LdsT<T> *P, LdsT<T> *Xb, LdsT<T> *Dd, LdsT<T> *vb, int j,
                                            int jx, unsigned long long *sub = nullptr) {
#ifdef CMPC_STAMPS
    unsigned long long tq = __builtin_amdgcn_s_memtime();
#define SUBSTAMP(i) do { if (sub) { const unsigned long long tn = __builtin_amdgcn_s_memtime(); sub[i] += tn - tq; tq = tn; } } while (0)
#else
#define SUBSTAMP(i) do { } while (0)
#endif
    constexpr int NX = (81 + L - 1) / L, NU2 = (45 + L - 1) / L;   // X / upper-triangle elements per lane
    const int l = threadIdx.x & (L - 1);
    // X elements (all 81): e = l + L q, clamped to 80 past the end (bit-identical duplicates)
    int e[NX], ii[NX], cc[NX];
    bool ok[NX];
#pragma unroll
    for (int q = 0; q < NX; ++q) {
        ok[q] = l + L * q < 81;
        e[q] = ok[q] ? l + L * q : 80;
        ii[q] = e[q] / 9;
        cc[q] = e[q] % 9;
    }
    // upper-triangle elements u = l + L q (row-major over i <= j), clamped to 44 = (8, 8)
    int iu[NU2], ju[NU2];
    bool oku[NU2];
#pragma unroll
    for (int q = 0; q < NU2; ++q) {
        oku[q] = l + L * q < 45;
        int r = oku[q] ? l + L * q : 44, row = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {   // walk the rows (lengths 9, 8, ..., 1)
            const bool past = r >= 9 - i && row == i;
            r = past ? r - (9 - i) : r;
            row = past ? i + 1 : row;
        }
        iu[q] = row;
        ju[q] = row + r;
    }
    T au[NU2];
#pragma unroll
    for (int q = 0; q < NU2; ++q) {
        au[q] = Dn[iu[q] * 9 + ju[q]];
        if (iu[q] == ju[q]) Dd[iu[q]] = au[q];   // original diagonal (pivot floor)
    }
    T rv = (vb && l < 9) ? vb[j * 9 + l] : T(0);   // b_j (fused elimination)
    auto dot = [&](auto fa, auto fb) -> T {
        T u[9], v[9];
#pragma unroll
        for (int m = 0; m < 9; ++m) { u[m] = fa(m); v[m] = fb(m); }
        T s0 = u[0] * v[0], s1 = u[1] * v[1], s2 = u[2] * v[2];
#pragma unroll
        for (int m = 3; m < 9; m += 3) { s0 = fma(u[m], v[m], s0); s1 = fma(u[m + 1], v[m + 1], s1); s2 = fma(u[m + 2], v[m + 2], s2); }
        return s0 + s1 + s2;
    };
    if (Op) {   // X = Op' I_{j-1} (whole);  A -= X Op (upper triangle)
        T x[NX];
#pragma unroll
        for (int q = 0; q < NX; ++q)
            x[q] = dot([&](int m) { return Op[m * 9 + ii[q]]; }, [&](int m) { return Ip[m * 9 + cc[q]]; });
#pragma unroll
        for (int q = 0; q < NX; ++q) Xb[e[q]] = x[q];
        wave_sync();
        if (vb && l < 9) rv -= dot9(Xb + l * 9, vb + jx * 9);
#pragma unroll
        for (int q = 0; q < NU2; ++q)
            au[q] -= dot([&](int m) { return Xb[iu[q] * 9 + m]; }, [&](int m) { return Op[m * 9 + ju[q]]; });
#pragma unroll
        for (int q = 0; q < NX; ++q)
            if (ok[q]) Xout[e[q]] = x[q];
    }
#pragma unroll
    for (int q = 0; q < NU2; ++q) A[iu[q] * 9 + ju[q]] = au[q];
    wave_sync();
    SUBSTAMP(0);
    T ip = rcp_nr(fmax(A[0], T(1e-13) * Dd[0]));
#pragma unroll
    for (int c = 0; c < 9; ++c) {
        T aic[NU2], acj[NU2];
#pragma unroll
        for (int q = 0; q < NU2; ++q) {
            const int i = iu[q], jj = ju[q];
            const T v1 = A[min(i, c) * 9 + max(i, c)], v2 = A[min(c, jj) * 9 + max(c, jj)];
            aic[q] = v1;
            acj[q] = c > jj ? -v2 : v2;
        }
        T ipn = T(0);
        if (c < 8) {   // A'[c+1][c+1] = U[c+1][c+1] - U[c][c+1]^2 / p_c (both indices unpivoted)
            const T ncc = A[(c + 1) * 9 + c + 1], nci = A[c * 9 + c + 1];
            ipn = rcp_nr(fmax(fma(-(nci * ip), nci, ncc), T(1e-13) * Dd[c + 1]));
        }
#pragma unroll
        for (int q = 0; q < NU2; ++q) {
            const T mi = aic[q] * ip;
            const T gen = fma(-mi, acj[q], au[q]), row = acj[q] * ip, col = -mi;
            const bool ic = __builtin_unpredictable(iu[q] == c), jc = __builtin_unpredictable(ju[q] == c);
            au[q] = ic ? (jc ? ip : row) : (jc ? col : gen);
        }
        wave_sync();
#pragma unroll
        for (int q = 0; q < NU2; ++q) A[iu[q] * 9 + ju[q]] = au[q];
        wave_sync();
        ip = ipn;
    }
    SUBSTAMP(1);
#pragma unroll
    for (int q = 0; q < NU2; ++q) {
        P[iu[q] * 9 + ju[q]] = au[q];
        P[ju[q] * 9 + iu[q]] = au[q];
        if (oku[q]) Iout[ju[q] * (ju[q] + 1) / 2 + iu[q]] = au[q];   // packed (row ju >= column iu)
    }
    if (vb && l < 9) vb[j * 9 + l] = rv;
    wave_sync();
    SUBSTAMP(2);
#undef SUBSTAMP
}

// the two ends, one per group of L lanes: with one wave per problem (L = 32) lanes 0..31 the top
// blocks 0..m-1 and lanes 32..63 the bottom blocks NB-1..m+1; with two waves per problem (L = 64)
// wave 0 the top and wave 1 the bottom, so every step has half the elements per lane (for even
// NB the top end has one step more; the bottom group idles in it).
// The raw blocks of step s + 1 are loaded during step s and landed in LDS at its end, inside
// the same loop iteration: registers carried over the back-edge with loads in flight would make
// the compiler drain the whole memory queue (this step's stores included) at the loop header.
// The bottom end lands its coupling block S_{j,j+1} transposed, so both ends run the same step.
template <typename T, int L>
__device__ void tw_factor_ends(T *Sd_, T *So_, int NB, int m, LdsT<T> *sh, LdsT<T> *vb, unsigned long long *stamp_out) {
    GlbT<T> *Sd = (GlbT<T> *)Sd_, *So = (GlbT<T> *)So_;
    constexpr int NE = (81 + L - 1) / L;
    const int l = threadIdx.x & (L - 1);
    const bool top = (threadIdx.x & L) == 0;
    LdsT<T> *A = sh + (top ? 0 : TW_SCRATCH), *P = A + 88, *Xb = A + 176, *Ob = A + 264, *Dd = A + 352,
            *Dn = A + 368;
    const int j0 = top ? 0 : NB - 1, dj = top ? 1 : -1, nstep = top ? m : NB - 1 - m;
    int e[NE], et[NE], ep[NE], ec[NE];
    bool ok[NE];
    T em[NE];
#pragma unroll
    for (int q = 0; q < NE; ++q) {
        ok[q] = l + L * q < 81;
        e[q] = ok[q] ? l + L * q : 80;
        et[q] = top ? e[q] : (e[q] % 9) * 9 + e[q] / 9;   // landing slot of a coupling element
        ep[q] = pk9(e[q] / 9, e[q] % 9);                   // packed slot of a diagonal-block element
        const int c = cp9(e[q] / 9, e[q] % 9);            // compact slot of a coupling element
        ec[q] = c >= 0 ? c : 0;
        em[q] = c >= 0 ? T(1) : T(0);                     // off-pattern elements land as zeros
    }
    unsigned long long sub[4] = {0, 0, 0, 0};
    unsigned long long *subp = (stamp_out && top) ? sub : nullptr;
    {
        const GlbT<T> *D0 = Sd + (size_t)j0 * 81;
        T v[NE];
#pragma unroll
        for (int q = 0; q < NE; ++q) v[q] = D0[ep[q]];
#pragma unroll
        for (int q = 0; q < NE; ++q) Dn[e[q]] = v[q];
    }
    wave_sync();
    for (int s = 0, j = j0; s < m; ++s, j += dj) {
        const bool act = s < nstep;
        // raw blocks of the next step (clamped past the end: branch-free loads)
        const int jn = s + 1 < nstep ? j + dj : j;
        const GlbT<T> *On = So + (size_t)(top ? (jn > 0 ? jn - 1 : 0) : jn) * 81, *Dnx = Sd + (size_t)jn * 81;
        T pv[NE], nv[NE];
#pragma unroll
        for (int q = 0; q < NE; ++q) { pv[q] = On[ec[q]] * em[q]; nv[q] = Dnx[ep[q]]; }
        if (act) {
            if (s == 0)
                tw_step_sym<T, L>(Dn, nullptr, nullptr, nullptr, Sd + (size_t)j * 81, A, P, Xb, Dd, vb, j, 0, subp);
            else
                tw_step_sym<T, L>(Dn, Ob, P, So + (size_t)(top ? j - 1 : j) * 81, Sd + (size_t)j * 81, A, P, Xb, Dd, vb,
                               j, j - dj, subp);
        }
#ifdef CMPC_STAMPS
        const unsigned long long tl = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
        for (int q = 0; q < NE; ++q) { Ob[et[q]] = pv[q]; Dn[e[q]] = nv[q]; }   // clamped lanes: same values
        wave_sync();
#ifdef CMPC_STAMPS
        if (subp) sub[3] += __builtin_amdgcn_s_memtime() - tl;
#endif
    }
    if (stamp_out && top && l == 0)
        for (int i = 0; i < 4; ++i) stamp_out[12 + i] += sub[i];
}

// the meeting block (whole wave): I_{m-1} and I_{m+1} are the two halves' previous inverses in LDS
template <typename T> __device__ void tw_factor_meet(T *Sd_, T *So_, int m, LdsT<T> *sh, LdsT<T> *vb) {
    GlbT<T> *Sd = (GlbT<T> *)Sd_, *So = (GlbT<T> *)So_;
    const int lane = threadIdx.x & 63;
    const int e0 = lane, e1 = lane + 64;
    const bool has1 = e1 < 81;
    LdsT<T> *A = sh, *P = A + 88, *Xb = A + 176, *Op = A + 264, *Dd = A + 352;
    LdsT<T> *Pq = sh + TW_SCRATCH + 88, *Oq = sh + TW_SCRATCH + 264;
    auto cpl = [&](const GlbT<T> *blk, int e) -> T {   // compact coupling block -> element e (zero off-pattern)
        const int c = cp9(e / 9, e % 9);
        return blk[c >= 0 ? c : 0] * (c >= 0 ? T(1) : T(0));
    };
    Op[e0] = cpl(So + (size_t)(m - 1) * 81, e0);
    Oq[e0] = cpl(So + (size_t)m * 81, e0);
    if (has1) { Op[e1] = cpl(So + (size_t)(m - 1) * 81, e1); Oq[e1] = cpl(So + (size_t)m * 81, e1); }
    LdsT<T> *Dn = A + 368;
    Dn[e0] = Sd[(size_t)m * 81 + pk9(e0 / 9, e0 % 9)];
    if (has1) Dn[e1] = Sd[(size_t)m * 81 + pk9(e1 / 9, e1 % 9)];
    wave_sync();
    tw_step<T, 64>(Dn, Op, P, Oq, Pq, So + (size_t)(m - 1) * 81, So + (size_t)m * 81, Sd + (size_t)m * 81, A, P,
                   Xb, Dd, vb, m, m - 1, m + 1);
}

// Chunked, double-buffered stream of 9x9 blocks from the workspace into a half-wave's LDS ring:
// each sweep iteration issues the next K blocks (three elements per lane, coalesced), runs K
// sweep steps out of the current LDS chunk, then lands the next chunk, so one chunk's L2 /
// Infinity-Cache latency hides behind K dependent steps.  Loads, their landing and their use
// stay inside one loop iteration (no in-flight registers carried over the back-edge, where the
// compiler's wait counting would drain the queue), and the loads are branch-free (a clamped
// index past the end re-reads the last block).
constexpr int RSLOT = 88;
template <typename T, int K, bool PK = false> struct ChunkStream {   // PK: packed symmetric blocks
    const GlbT<T> *base;   // block i at base + i * step
    long step;
    int n;
    LdsT<T> *buf;    // 2 x K slots of RSLOT
    T r[K][3];
    __device__ __forceinline__ void issue(int c) {
        const int l = threadIdx.x & 31;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const int i = c * K + q;
            const GlbT<T> *p = base + (i < n ? i : n - 1) * step;
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                const int el = l + 32 * g < 81 ? l + 32 * g : 80;
                r[q][g] = p[PK ? pk9(el / 9, el % 9) : el];
            }
        }
    }
    __device__ __forceinline__ void land(int c) {
        const int l = threadIdx.x & 31;
        LdsT<T> *b = buf + (c & 1) * K * RSLOT;
#pragma unroll
        for (int q = 0; q < K; ++q)
#pragma unroll
            for (int g = 0; g < 3; ++g) b[q * RSLOT + (l + 32 * g < 81 ? l + 32 * g : 80)] = r[q][g];   // clamped: same value
    }
    __device__ __forceinline__ const LdsT<T> *blk(int i) const {
        return buf + ((i / K) & 1) * K * RSLOT + (i % K) * RSLOT;
    }
};
constexpr int KE = QP_KE;   // blocks per chunk of the sweep streams
constexpr int SWEEP_LDS = 2 * KE * RSLOT;   // per half-wave: 2 x 8 slots = 2 x (2 x 4) slots

// (5c) two-ended block sweeps with the twisted factors (one end per half-wave): rhs -> dnu in
// place in the LDS vector vb
//   top:    y_0 = b_0, y_j = b_j - X_j y_{j-1}           bottom: y_j = b_j - Y_j y_{j+1}
//   meet:   x_m = I_m (b_m - X_m y_{m-1} - Y_m y_{m+1})
//   up:     x_j = I_j y_j - X_{j+1}' x_{j+1}  (j < m)   down: x_j = I_j y_j - Y_{j-1}' x_{j-1}  (j > m)
// X_j sits at So[j-1], Y_j at So[j].  Three stages separated by workgroup barriers; each half
// uses 9 of its lanes per step and its own block ring.
template <typename T> __device__ void tw_solve_elim(const T *Xs, int NB, int m, LdsT<T> *vb, LdsT<T> *ring) {
    const int lane = threadIdx.x & 63, l = lane & 31;
    const bool top = lane < 32;
    const int lr = l < 9 ? l : 0;
    // step i: top j = i + 1 (X_j at So[i]); bottom j = NB - 2 - i (Y_j at So[NB - 2 - i])
    const int n = top ? m - 1 : NB - 2 - m, nmax = m - 1;
    const GlbT<T> *Xg = (const GlbT<T> *)Xs;
    ChunkStream<T, KE> X{top ? Xg : Xg + (size_t)(NB - 2) * 81, top ? 81L : -81L, n > 0 ? n : 1, ring, {}};
    X.issue(0);
    X.land(0);
    for (int c = 0; c * KE < nmax; ++c) {
        X.issue(c + 1);
        wave_sync();
        for (int q = 0; q < KE; ++q) {
            const int i = c * KE + q;
            if (i >= nmax) break;
            const int j = top ? i + 1 : NB - 2 - i, jp = top ? j - 1 : j + 1;
            if (l < 9 && i < n) {
                const LdsT<T> *xr = X.blk(i) + lr * 9;
                const LdsT<T> *yp = vb + jp * 9;
                T xv[9], yv[9];
#pragma unroll
                for (int e = 0; e < 9; ++e) { xv[e] = xr[e]; yv[e] = yp[e]; }
                const T bj = vb[j * 9 + l];
                T s0 = xv[0] * yv[0], s1 = xv[1] * yv[1], s2 = xv[2] * yv[2];
#pragma unroll
                for (int e = 3; e < 9; e += 3) {
                    s0 = fma(xv[e], yv[e], s0); s1 = fma(xv[e + 1], yv[e + 1], s1); s2 = fma(xv[e + 2], yv[e + 2], s2);
                }
                vb[j * 9 + l] = bj - (s0 + s1 + s2);
            }
            wave_sync();
        }
        X.land(c + 1);
    }
    wave_sync();
}
template <typename T>
__device__ void tw_solve_meet(const T *Ii, const T *Xs, int NB, int m, LdsT<T> *vb, LdsT<T> *sh) {
    const int lane = threadIdx.x & 63;
    if (lane < 9) {
        T v = vb[m * 9 + lane];
        const GlbT<T> *X = (const GlbT<T> *)Xs + (size_t)(m - 1) * 81 + lane * 9, *Y = (const GlbT<T> *)Xs + (size_t)m * 81 + lane * 9;
        const LdsT<T> *yp = vb + (m - 1) * 9, *yn = vb + (m + 1) * 9;
        for (int q = 0; q < 9; ++q) v = fma(-X[q], yp[q], fma(-Y[q], yn[q], v));
        sh[lane] = v;
    }
    wave_sync();
    if (lane < 9) {
        const GlbT<T> *I = (const GlbT<T> *)Ii + (size_t)m * 81;   // packed
        T v = T(0);
        for (int q = 0; q < 9; ++q) v = fma(I[pk9(lane, q)], sh[q], v);
        vb[m * 9 + lane] = v;
    }
    wave_sync();
}
// The back sweep's local terms z_j = I_j y_j for every block but the meeting one, all blocks in
// parallel (thread per block, in place in vb) once the elimination and the meeting block are
// done: the sequential step is then a single 9-term product.
template <typename T, int NTT> __device__ void tw_solve_local(const T *Ii, int NB, int m, LdsT<T> *vb) {
    for (int j = threadIdx.x & (NTT - 1); j < NB; j += NTT) {
        if (j == m) continue;
        const GlbT<T> *I = (const GlbT<T> *)Ii + (size_t)j * 81;   // packed
        T iv[45], y[9];
#pragma unroll
        for (int p = 0; p < 45; ++p) iv[p] = I[p];
#pragma unroll
        for (int i = 0; i < 9; ++i) y[i] = vb[j * 9 + i];
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            T a = iv[pk9(i, 0)] * y[0];
#pragma unroll
            for (int q = 1; q < 9; ++q) a = fma(iv[pk9(i, q)], y[q], a);
            vb[j * 9 + i] = a;
        }
    }
}
template <typename T>
__device__ void tw_solve_back(const T *Xs, int NB, int m, LdsT<T> *vb, LdsT<T> *ring) {
    const int lane = threadIdx.x & 63, l = lane & 31;
    const bool top = lane < 32;
    const int lr = l < 9 ? l : 0;
    // step i: top j = m - 1 - i (X_{j+1} at So[j]); bottom j = m + 1 + i (Y_{j-1} at So[j-1]);
    // vb[j] holds z_j = I_j y_j (tw_solve_local)
    const int n = top ? m : NB - 1 - m, nmax = m;
    ChunkStream<T, KE> X{(const GlbT<T> *)Xs + (size_t)(top ? m - 1 : m) * 81, top ? -81L : 81L, n > 0 ? n : 1, ring, {}};
    X.issue(0);
    X.land(0);
    for (int c = 0; c * KE < nmax; ++c) {
        X.issue(c + 1);
        wave_sync();
        for (int q = 0; q < KE; ++q) {
            const int i = c * KE + q;
            if (i >= nmax) break;
            const int j = top ? m - 1 - i : m + 1 + i, jn = top ? j + 1 : j - 1;
            T v = T(0);
            const bool act = l < 9 && i < n;
            if (act) {
                const LdsT<T> *xb = X.blk(i);
                const LdsT<T> *xn = vb + jn * 9;
                T xc[9], nv[9];
#pragma unroll
                for (int e = 0; e < 9; ++e) { xc[e] = xb[e * 9 + lr]; nv[e] = xn[e]; }
                T s0 = vb[j * 9 + lr] - xc[0] * nv[0], s1 = -(xc[1] * nv[1]), s2 = -(xc[2] * nv[2]);
#pragma unroll
                for (int e = 3; e < 9; e += 3) { s0 = fma(-xc[e], nv[e], s0); s1 = fma(-xc[e + 1], nv[e + 1], s1); s2 = fma(-xc[e + 2], nv[e + 2], s2); }
                v = s0 + s1 + s2;
            }
            wave_sync();
            if (act) vb[j * 9 + l] = v;
            wave_sync();
        }
        X.land(c + 1);
    }
    wave_sync();
}

#include "schur_pt.hpp"

// r_hat = r_i - r_c / lambda of one row.  corr 0 (predictor): r_c = s lambda; 1 (corrector):
// r_c = s lambda + ds_aff dlambda_aff - sigma mu (a = the dsa field: the predictor's product);
// 2 (refinement): r_c = a, the dsa field then holding the complementarity residual of the corrector
// direction (phase_lres).  Absent rows: 0.  The w phase and the direction phase both form it (the
// direction phase recomputes it from s, lambda, r_i and dsa, which it loads anyway, instead of a
// stored r_hat: one field row less written and read per Newton solve).
template <typename T>
__device__ __forceinline__ T rhat_row(int corr, bool pr, T rd, T sr, T lr, T a, T sigma_mu) {
    const T cc = corr ? (corr == 2 ? a : a - sigma_mu) : T(0);
    const T rc = (corr == 2 ? T(0) : sr * lr) + cc;
    const T v = rd - fdiv(rc, pr ? lr : T(1));
    return pr ? v : T(0);
}
// r_hat for the rows of knot k, rows [R0, R1): all of them, or one part's (PART as in resid_knot)
template <typename T, int ROBOT, int R0 = 0, int R1 = Rows<ROBOT>::NI>
__device__ __forceinline__ void rhat_rows(const Ctx<T, ROBOT> &C, int k, int corr, T sigma_mu, const T *s, const T *lm,
                                          T *rh) {
    constexpr int NI = Rows<ROBOT>::NI;
    const unsigned msk = C.cmask(k);
    // every row's loads in one batch (a branch per row serialized them)
    T rd[NI], a[NI];
    const SV<T> rdi = C.kv(WF(rdi), k);
#pragma unroll
    for (int r = R0; r < R1; ++r) { rd[r] = rdi[r]; a[r] = T(0); }
    if (corr) {   // corrector: + ds_aff dlambda_aff - sigma mu (the product, stored by the predictor)
        const SV<T> dsa = C.kv(WF(dsa), k);
#pragma unroll
        for (int r = R0; r < R1; ++r) a[r] = dsa[r];
    }
#pragma unroll
    for (int r = R0; r < R1; ++r) rh[r] = rhat_row(corr, Ctx<T, ROBOT>::present_m(msk, r), rd[r], s[r], lm[r], a[r], sigma_mu);
}

// (5a) particular solution w = Phi^-1 (r_d + G' D rhat) (friction rows in push-through form)
// getG(c, G): the friction rows of contact c (from registers in the predictor, which shares the
// factor phase's loads, or from the stage record)
// PART as in resid_knot: 0 the (x, t) part (w_x, the trust-region / slack rows of r_hat, the
// right-hand side but B w_u), 1 the controls (w_u, the contact rows of r_hat, B w_u into the side
// array C.bus, subtracted with add_wx), -1 both
template <typename T, int ROBOT, typename GF, int PART = -1>
__device__ __forceinline__ void phase_w_core(const Ctx<T, ROBOT> &C, int k, int corr, T sigma_mu,
                                             const T (&sv)[Rows<ROBOT>::NI], const T (&lv)[Rows<ROBOT>::NI], GF &&getG) {
    using R_ = Rows<ROBOT>;
    constexpr int NI = R_::NI, NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    const int N = C.N;
    const bool hu = k < N;
    constexpr int RA = PART == 1 ? R_::FR : 0, RB = PART == 0 ? R_::FR : NI;   // this part's rows
    T rh[NI];
    rhat_rows<T, ROBOT, RA, RB>(C, k, corr, sigma_mu, sv, lv, rh);   // (phase_dz forms it again)
    T rdx[9], rdu[NU];
    ldv(C.kv(WF(rdx), k), rdx);
    ldv(C.kv(WF(rdu), k), rdu);   // k = N: unused
    const T rdt = C.kv(WF(rdt), k)[0];
    T wx[9], wt;
    for (int i = 0; i < 6; ++i) wx[i] = C.iWx(i) * rdx[i];
    if (PART != 1) {   // (L, t): w = -(local solve with v = -r_d)
        T Lk[36], z1[8], iden, dsl;
        tr_factor(C, sv, lv, Lk, z1, iden, dsl);
        const T vL[3] = {-rdx[6], -rdx[7], -rdx[8]};
        T dL[3], dt, dlt[8], dls;
        tr_local(C, Lk, z1, dsl, iden, vL, -rdt, rh, dL, dt, dlt, dls);
        for (int i = 0; i < 3; ++i) wx[6 + i] = -dL[i];
        wt = -dt;
    }
    T ou[NU];
    if (hu && PART != 0) {
        T vu[NU];
        for (int i = 0; i < NU; ++i) vu[i] = rdu[i];
        if (ROBOT == 1) {   // CoP rows (D-form, folded into W_cop); absent rows: lambda = 0 -> D = 0, rhat = 0
            for (int c = 0; c < NC; ++c)
                for (int dd = 0; dd < 2; ++dd) {
                    const int r0 = R_::CP + 4 * c + 2 * dd;
                    vu[NUPC * c + dd] += C.Dform(lv[r0], sv[r0]) * rh[r0] - C.Dform(lv[r0 + 1], sv[r0 + 1]) * rh[r0 + 1];
                }
        }
        const unsigned msk = C.cmask(k);
#pragma unroll
        for (int c = 0; c < NC; ++c) {   // Phi_u^-1 (vu + G' D rhat) contact by contact
            const bool act = (msk >> c) & 1u;
            T G[12];
            getG(c, G);
            const T wi[3] = {C.iWu(NUPC * c + FO), C.iWu(NUPC * c + FO + 1), C.iWu(NUPC * c + FO + 2)};
            T Gw[4][3], Ki[10], F[6], wd[NUPC];
            fric_factor(G, wi, sv + R_::FR + 4 * c, lv + R_::FR + 4 * c, act, Gw, Ki);
            fric_F(Gw, Ki, wi, F);
            contact_wd(C, c, act, sv, lv, wd);
            const T *vc = vu + NUPC * c;
            for (int q = 0; q < NUPC; ++q) ou[NUPC * c + q] = wd[q] * vc[q];
            for (int i = 0; i < 3; ++i)
                ou[NUPC * c + FO + i] = sym3(F, i, 0) * vc[FO] + sym3(F, i, 1) * vc[FO + 1] + sym3(F, i, 2) * vc[FO + 2];
            T kr[4];
            for (int r = 0; r < 4; ++r) {
                T acc = T(0);
                for (int q = 0; q < 4; ++q) acc += Ki[p4(r, q)] * rh[R_::FR + 4 * c + q];
                kr[r] = acc;
            }
            for (int i = 0; i < 3; ++i) {
                T acc = T(0);
                for (int r = 0; r < 4; ++r) acc += Gw[r][i] * kr[r];
                ou[NUPC * c + FO + i] += acc;
            }
        }
    }
    // stores
    (void)wt;   // w_x, w_t enter only the right-hand side below; w_u is read by phase_dz
    if (hu && PART != 0) stv(C.kv(WF(wu), k), ou);
    // the Schur right-hand side, fused: block 1 + k = r_k - A_k wx_k - B_k wu_k + wx_{k+1}.  Thread
    // k writes all but the last term; after a wave-level fence (block k was written by lane k - 1
    // in this pass or an earlier one: the lanes of the one wave run in lockstep) it adds its own
    // wx_k to block k.  Block 0 = r_init - wx_0, block N + 1 = r_final - wx_N.
    {
        using S = Stage<ROBOT>;
        LdsT<T> *vb = C.vb;
        if (PART == 1) {   // B w_u of knot k into the side array (block 1 + k)
            if (hu) {
                T bu[9];
                opB<T, ROBOT>(C.st(k), ou, bu);
                for (int i = 0; i < 9; ++i) C.bus[(1 + k) * 9 + i] = bu[i];
            }
            return;
        }
        T r0[9], r1[9];
        ldv(C.bv(WF(rde), k == N ? N + 1 : 0), r0);   // boundary rows (k = 0: init, k = N: final)
        ldv(C.bv(WF(rde), hu ? 1 + k : 0), r1);       // dynamics rows of knot k
        if (k == 0) for (int i = 0; i < 9; ++i) vb[i] = r0[i] - wx[i];
        if (k == N) for (int i = 0; i < 9; ++i) vb[(N + 1) * 9 + i] = r0[i] - wx[i];
        if (hu) {
            T ax[9], bu[9];
            const auto st = C.st(k);
            opA(st + S::W, C.beta, wx, ax);
            if (PART != 0) opB<T, ROBOT>(st, ou, bu);
            for (int i = 0; i < 9; ++i) vb[(1 + k) * 9 + i] = r1[i] - (ax[i] + (PART != 0 ? bu[i] : T(0)));
        }
        if (C.wxs) {
            if (k >= 1)
                for (int i = 0; i < 9; ++i) C.wxs[k * 9 + i] = wx[i];
        } else {
            wave_sync();
            if (k >= 1)
                for (int i = 0; i < 9; ++i) vb[k * 9 + i] += wx[i];
        }
    }
}
// the deferred last term of the fused right-hand side (multi-wave workgroups): block k += w_x,k
// (and, after split w phases, minus the control part's B w_u, block 1 + k of bus)
template <typename T, int NTT>
__device__ __forceinline__ void add_wx(LdsT<T> *vb, const LdsT<T> *wxs, int N, const LdsT<T> *bus = nullptr) {
    if (bus)
        for (int e = 9 + (int)(threadIdx.x & (NTT - 1)); e < (N + 1) * 9; e += NTT) vb[e] += wxs[e] - bus[e];
    else
        for (int e = 9 + (int)(threadIdx.x & (NTT - 1)); e < (N + 1) * 9; e += NTT) vb[e] += wxs[e];
}
template <typename T, int ROBOT, int PART = -1> __device__ __forceinline__ void phase_w(const Ctx<T, ROBOT> &C, int k, int corr, T sigma_mu) {
    using S = Stage<ROBOT>;
    constexpr int NI = Rows<ROBOT>::NI;
    T sv[NI], lv[NI];
    ldv(C.kv(WF(s), k), sv);
    ldv(C.kv(WF(l), k), lv);
    const auto st = C.st(k);
    auto getG = [&](int c, T (&G)[12]) { ldv(st + (S::CON + S::CS * c + S::G), G); };
    phase_w_core<T, ROBOT, decltype(getG) &, PART>(C, k, corr, sigma_mu, sv, lv, getG);
}
template <typename T, int ROBOT, int PART = -1>
__device__ __forceinline__ void phase_w_pred(const Ctx<T, ROBOT> &C, int k, const KnotSL<T, ROBOT> &kl) {
    auto getG = [&](int c, T (&G)[12]) {
#pragma unroll
        for (int e = 0; e < 12; ++e) G[e] = kl.G[c][e];
    };
    phase_w_core<T, ROBOT, decltype(getG) &, PART>(C, k, 0, T(0), kl.s, kl.l, getG);
}



// (5d) direction at knot k from dnu; returns the max step allowed by this knot's rows
// rows of knot k: ds = -r_i - G dz; dlambda from the push-through solves (TR, slack: dlt, dls;
// friction: Kinv (Gw v + rhat) with v = -(rdu + E'dnu_u) on the forces) or the D-form (CoP);
// returns the largest step keeping s, lambda >= 0, and accumulates the three coefficients of
// sum_r (s + a ds)(lambda + a dl).  Restrict-qualified field pointers (field f at p[f * KPC]) and
// contact-by-contact streaming: each row's step is stored as soon as it is formed, so the knot
// is never held in registers whole.  Inactive contacts: G = Gw = 0, Kinv = I, rhat = 0 -> zero
// steps.
// ACC (refinement): the solve gives the correction of the corrector direction; the stored
// direction becomes direction + correction and the ratio test runs on the sum.
// PART as in resid_knot: 0 the (x, t) part and the trust-region / slack rows, 1 the controls and
// the contact rows (-1 both)
// r_hat is formed here again (rhat_row with corr / sigma_mu, from s, lambda, r_i and, corr >= 1,
// the dsa field), as the w phase formed it.  prod (the predictor after the initialization step):
// only ds_aff dlambda_aff is stored; its dx, dt, du and dlambda are dead (the corrector replaces
// them), so they are not written.
template <typename T, int ROBOT, bool ACC = false, int PART = -1>
__device__ __forceinline__ T dz_knot(const Ctx<T, ROBOT> &C, int k, T (&mus)[3], bool prod, int corr, T sigma_mu,
                                     const T *__restrict__ stp,
                                     const T *__restrict__ dsap, const T *__restrict__ rdxp, const T *__restrict__ rdtp,
                                     const T *__restrict__ wup, const T *__restrict__ ss, const T *__restrict__ ls,
                                     const T *__restrict__ rdip, const T *__restrict__ rdup,
                                     T *__restrict__ dxo, T *__restrict__ dto, T *__restrict__ duo, T *__restrict__ ds,
                                     T *__restrict__ dl) {
    using S = Stage<ROBOT>;
    using R_ = Rows<ROBOT>;
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    constexpr int ld = KPC;
    const int N = C.N;
    const bool hu = k < N;
    const SV<const T> st{stp};   // knot kc (= k, or 0 at k = N where no contact row exists)
    const unsigned msk = C.cmask(k);
    // E' dnu at knot k from the LDS blocks k, k+1 (k = 0: block 0 is the init rows; k = N: block
    // N+1 the final rows); the knot-type cases are selects (one basic block)
    const LdsT<T> *vb = C.vb;
    T dk[9], d1[9], ex[9], eu[NU], a[9], w[3];
    for (int i = 0; i < 9; ++i) { dk[i] = vb[k * 9 + i]; d1[i] = vb[(k + 1) * 9 + i]; }
    for (int i = 0; i < 3; ++i) w[i] = st[S::W + i];
    if (PART != 1) {
        opAT(w, C.beta, d1, a);
        for (int i = 0; i < 9; ++i)
            ex[i] = (k == 0 ? dk[i] : -dk[i]) + (hu ? a[i] : T(0)) + (k == N ? d1[i] : T(0));
    }
    if (PART != 0) opBT<T, ROBOT>(st, d1, eu);
    T amax = T(1);
    // stores: corrector ds, dl; predictor ds_aff dl_aff in the ds field (the corrector's r_hat
    // term) or, in the initialization step (whose full step is the affine one), ds_aff itself
    auto emit = [&](int r, bool pr, T g, T dlr, T sr, T lr, T rdir) {
        T dsr = pr ? -rdir - g : T(0);
        if (ACC) { dsr += ds[r * ld]; dlr += dl[r * ld]; }
        ds[r * ld] = prod ? dsr * dlr : dsr;
        if (!prod) dl[r * ld] = dlr;
        // sum_r (s + a ds)(lambda + a dl) = mus0 + a mus1 + a^2 mus2 (absent rows: lambda = ds = dl = 0)
        mus[0] = fma(sr, lr, mus[0]);
        mus[1] = fma(sr, dlr, fma(lr, dsr, mus[1]));
        mus[2] = fma(dsr, dlr, mus[2]);
        // branch-free ratio tests (selects keep the row loop one basic block)
        const T qs = fdiv(-sr, dsr < T(0) ? dsr : T(-1)), ql = fdiv(-lr, dlr < T(0) ? dlr : T(-1));
        amax = fmin(amax, fmin(dsr < T(0) ? qs : T(1), dlr < T(0) ? ql : T(1)));
    };
    // the knot's control-sized records, loaded with the (x, t) rows (per-contact loads next to
    // their use were each waited on alone)
    T wuv[NU], rduv[NU];
#pragma unroll
    for (int q = 0; q < (PART != 0 ? NU : 0); ++q) { wuv[q] = wup[q * ld]; rduv[q] = rdup[q * ld]; }
    // (x, t) part and the trust-region / slack rows
    if (PART != 1) {
        T rdx[9], s9[9], l9[9], rh9[9], ri9[9], a9[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            rdx[i] = rdxp[i * ld];
            s9[i] = ss[i * ld];
            l9[i] = ls[i * ld];
            ri9[i] = rdip[i * ld];
            a9[i] = T(0);
        }
        if (corr)
#pragma unroll
            for (int i = 0; i < 9; ++i) a9[i] = dsap[i * ld];
#pragma unroll
        for (int i = 0; i < 9; ++i) rh9[i] = rhat_row(corr, true, ri9[i], s9[i], l9[i], a9[i], sigma_mu);
        const T rdt = rdtp[0];
        T dx[9], dtt, dlt[8], dls;
        for (int i = 0; i < 6; ++i) dx[i] = -C.iWx(i) * (rdx[i] + ex[i]);
        {
            T Lk[36], z1[8], iden, dsl;
            tr_factor(C, s9, l9, Lk, z1, iden, dsl);
            const T vL[3] = {-(rdx[6] + ex[6]), -(rdx[7] + ex[7]), -(rdx[8] + ex[8])};
            tr_local(C, Lk, z1, dsl, iden, vL, -rdt, rh9, dx + 6, dtt, dlt, dls);
        }
        // the rows' g'dz use the correction itself (ds = -r_i - g'dz is linear in the solve)
        if (!prod) {
#pragma unroll
            for (int i = 0; i < 9; ++i) dxo[i * ld] = ACC ? dxo[i * ld] + dx[i] : dx[i];
            dto[0] = ACC ? dto[0] + dtt : dtt;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
            emit(j, true, tr_sign<T>(j, 0) * dx[6] + tr_sign<T>(j, 1) * dx[7] + tr_sign<T>(j, 2) * dx[8] + C.cw * dtt,
                 dlt[j], s9[j], l9[j], ri9[j]);
        emit(8, true, -dtt, dls, s9[8], l9[8], ri9[8]);
    }
    // contacts, one at a time: du = -w_u - Phi_u^-1 E'dnu_u, then the contact's rows
#pragma unroll
    for (int c = 0; c < (PART != 0 ? NC : 0); ++c) {
        const bool pr = hu && ((msk >> c) & 1u);
        const auto cs = st + (S::CON + S::CS * c);
        T G[12], s4[4], l4[4], rh4[4], ri4[4], a4[4] = {T(0), T(0), T(0), T(0)}, vf[3];
        for (int e = 0; e < 12; ++e) G[e] = cs[S::G + e];
        for (int r = 0; r < 4; ++r) {
            const int row = R_::FR + 4 * c + r;
            s4[r] = ss[row * ld]; l4[r] = ls[row * ld]; ri4[r] = rdip[row * ld];
        }
        if (corr)
            for (int r = 0; r < 4; ++r) a4[r] = dsap[(R_::FR + 4 * c + r) * ld];
        for (int r = 0; r < 4; ++r) rh4[r] = rhat_row(corr, pr, ri4[r], s4[r], l4[r], a4[r], sigma_mu);
        const T wi[3] = {C.iWu(NUPC * c + FO), C.iWu(NUPC * c + FO + 1), C.iWu(NUPC * c + FO + 2)};
        T Gw[4][3], Ki[10], F[6], wd[NUPC], au[NUPC], du[NUPC];
        fric_factor(G, wi, s4, l4, pr, Gw, Ki);
        fric_F(Gw, Ki, wi, F);
        {
            const SV<const T> sS{ss}, lS{ls};
            contact_wd(C, c, pr, sS, lS, wd);
        }
        const T *ec = eu + NUPC * c;
        for (int q = 0; q < NUPC; ++q) au[q] = wd[q] * ec[q];
        for (int i = 0; i < 3; ++i)
            au[FO + i] = sym3(F, i, 0) * ec[FO] + sym3(F, i, 1) * ec[FO + 1] + sym3(F, i, 2) * ec[FO + 2];
        // unconditional loads (kc keeps the addresses valid at k = N) masked by arithmetic: a
        // select on a loaded value becomes a branch around the load and a wait per row
        const T hf = hu ? T(1) : T(0);
        for (int q = 0; q < NUPC; ++q) du[q] = (-wuv[NUPC * c + q] - au[q]) * hf;
        if (hu && !prod)
            for (int q = 0; q < NUPC; ++q) duo[(NUPC * c + q) * ld] = ACC ? duo[(NUPC * c + q) * ld] + du[q] : du[q];
        for (int i = 0; i < 3; ++i) vf[i] = -(rduv[NUPC * c + FO + i] + ec[FO + i]) * hf;
        T z[4];
        for (int r = 0; r < 4; ++r) z[r] = Gw[r][0] * vf[0] + Gw[r][1] * vf[1] + Gw[r][2] * vf[2] + rh4[r];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            T acc = T(0);
            for (int q = 0; q < 4; ++q) acc += Ki[p4(r, q)] * z[q];
            const T gr = G[3 * r] * du[FO] + G[3 * r + 1] * du[FO + 1] + G[3 * r + 2] * du[FO + 2];
            emit(R_::FR + 4 * c + r, pr, gr, hu ? acc : T(0), s4[r], l4[r], ri4[r]);
        }
        if (ROBOT == 1) {   // CoP rows (D-form)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = R_::CP + 4 * c + q, dd = q / 2;
                const T sr = ss[r * ld], lr = ls[r * ld], rir = rdip[r * ld], ar = corr ? dsap[r * ld] : T(0);
                const T gr = (q % 2 == 0) ? du[dd] : -du[dd];
                const T rhr = rhat_row(corr, pr, rir, sr, lr, ar, sigma_mu);
                emit(r, pr, gr, pr ? C.Dform(lr, sr) * (gr + rhr) : T(0), sr, lr, rir);
            }
        }
    }
    return amax;
}

template <typename T, int ROBOT, int PART = -1>
__device__ PHASE_ATTR T phase_dz(const Ctx<T, ROBOT> &C, int k, int corr, bool init, T sigma_mu, T (&mus)[3]) {
    const int kc = k < C.N ? k : 0;   // k = N: no controls or contacts
    T *ws = C.ws;
    return dz_knot<T, ROBOT, false, PART>(C, k, mus, !corr && !init, corr, sigma_mu, C.stage + kc,
                             ws + WF(dsa) * KPC + k, ws + WF(rdx) * KPC + k,
                             ws + WF(rdt) * KPC + k, ws + WF(wu) * KPC + kc, ws + WF(s) * KPC + k,
                             ws + WF(l) * KPC + k, ws + WF(rdi) * KPC + k, ws + WF(rdu) * KPC + kc,
                             ws + WF(dx) * KPC + k, ws + WF(dt) * KPC + k,
                             ws + WF(du) * KPC + k, ws + (corr ? WF(ds) : WF(dsa)) * KPC + k,
                             ws + (corr ? WF(dl) : WF(dla)) * KPC + k);
}

// the refinement's correction added to the corrector direction (dz_knot<ACC>): same inputs as the
// corrector's, whose fields phase_lres has overwritten with the Newton system's residuals
template <typename T, int ROBOT> __device__ PHASE_ATTR T phase_dz_refine(const Ctx<T, ROBOT> &C, int k) {
    const int kc = k < C.N ? k : 0;
    T *ws = C.ws;
    T mus[3] = {T(0), T(0), T(0)};
    return dz_knot<T, ROBOT, true>(C, k, mus, false, 2, T(0), C.stage + kc, ws + WF(dsa) * KPC + k, ws + WF(rdx) * KPC + k,
                                   ws + WF(rdt) * KPC + k, ws + WF(wu) * KPC + kc, ws + WF(s) * KPC + k,
                                   ws + WF(l) * KPC + k, ws + WF(rdi) * KPC + k, ws + WF(rdu) * KPC + kc,
                                   ws + WF(dx) * KPC + k, ws + WF(dt) * KPC + k, ws + WF(du) * KPC + k,
                                   ws + WF(ds) * KPC + k, ws + WF(dl) * KPC + k);
}

// (5e) residual of the Newton system at the corrector direction, knot k (iterative refinement):
//   e_x = W dx + E'_x dnu + G'_x dl + r_dx     e_t = cw 1'dl_TR - dl_sl + r_dt
//   e_u = W du + E'_u dnu + G'_u dl + r_du     e_e = E dz + r_e
//   e_i = G dz + ds + r_i                      e_c = s dl + lambda ds + r_c
// with r_c = s lambda + ds_aff dl_aff - sigma mu.  The residuals overwrite r_dx, r_dt, r_du, r_e,
// r_i and (e_c) the dsa field, which the corrector no longer needs; dnu (in LDS) is saved to the
// dn0 field.  The same w / Schur / direction phases then solve for the correction.
template <typename T, int ROBOT> __device__ PHASE_ATTR void phase_lres(const Ctx<T, ROBOT> &C, int k, T sigma_mu) {
    using S = Stage<ROBOT>;
    using R_ = Rows<ROBOT>;
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    const int N = C.N;
    const bool hu = k < N;
    const int kc = hu ? k : 0;
    const SV<const T> st = C.st(kc);
    const unsigned msk = C.cmask(k);
    const LdsT<T> *vb = C.vb;
    T dk[9], d1[9], dx[9], dx1[9], du[NU], rdx[9], rdu[NU], w[3];
    for (int i = 0; i < 9; ++i) { dk[i] = vb[k * 9 + i]; d1[i] = vb[(k + 1) * 9 + i]; }
    ldv(C.kv(WF(dx), k), dx);
    ldv(C.kv(WF(dx), hu ? k + 1 : k), dx1);
    ldv(C.kv(WF(du), kc), du);
    ldv(C.kv(WF(rdx), k), rdx);
    ldv(C.kv(WF(rdu), kc), rdu);
    ldv(st + S::W, w);
    const T dt = C.kv(WF(dt), k)[0], rdt = C.kv(WF(rdt), k)[0];
    T re0[9], re1[9];
    ldv(C.bv(WF(rde), k == N ? N + 1 : 0), re0);
    ldv(C.bv(WF(rde), hu ? 1 + k : 0), re1);
    // E' dnu at knot k (as in resid_knot)
    T ex[9], eu[NU], a[9];
    opAT(w, C.beta, d1, a);
    opBT<T, ROBOT>(st, d1, eu);
    for (int i = 0; i < 9; ++i) ex[i] = (k == 0 ? dk[i] : -dk[i]) + (hu ? a[i] : T(0)) + (k == N ? d1[i] : T(0));
    // rows: e_i, e_c and G' dl
    T gL[3] = {T(0), T(0), T(0)}, gt = T(0), gu[NU];
    for (int i = 0; i < NU; ++i) gu[i] = T(0);
    const SV<T> sS = C.kv(WF(s), k), lS = C.kv(WF(l), k), dsS = C.kv(WF(ds), k), dlS = C.kv(WF(dl), k),
                riS = C.kv(WF(rdi), k), caS = C.kv(WF(dsa), k);
    auto row = [&](int r, bool pr, T g) {   // g = g'dz of the row; returns dl (0 on absent rows)
        const T sr = sS[r], lr = lS[r], dsr = dsS[r], dlr = dlS[r], ri = riS[r], pa = caS[r];
        const T ei = g + dsr + ri;
        const T ec = fma(sr, dlr, fma(lr, dsr, fma(sr, lr, pa - sigma_mu)));
        riS[r] = pr ? ei : T(0);
        caS[r] = pr ? ec : T(0);
        return pr ? dlr : T(0);
    };
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const T dlr = row(j, true, tr_sign<T>(j, 0) * dx[6] + tr_sign<T>(j, 1) * dx[7] + tr_sign<T>(j, 2) * dx[8] + C.cw * dt);
        for (int i = 0; i < 3; ++i) gL[i] += tr_sign<T>(j, i) * dlr;
        gt += C.cw * dlr;
    }
    gt -= row(8, true, -dt);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const bool pr = hu && ((msk >> c) & 1u);
        const auto cs = st + (S::CON + S::CS * c);
        const T *f = du + NUPC * c + FO;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const T g0 = cs[S::G + 3 * r], g1 = cs[S::G + 3 * r + 1], g2 = cs[S::G + 3 * r + 2];
            const T dlr = row(R_::FR + 4 * c + r, pr, g0 * f[0] + g1 * f[1] + g2 * f[2]);
            gu[NUPC * c + FO] += g0 * dlr;
            gu[NUPC * c + FO + 1] += g1 * dlr;
            gu[NUPC * c + FO + 2] += g2 * dlr;
        }
        if (ROBOT == 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int dd = q / 2;
                const T dcop = du[NUPC * c + dd];
                const T dlr = row(R_::CP + 4 * c + q, pr, (q % 2 == 0) ? dcop : -dcop);
                gu[NUPC * c + dd] += (q % 2 == 0) ? dlr : -dlr;
            }
        }
    }
    // dual rows
    T ox[9];
    for (int i = 0; i < 9; ++i) ox[i] = C.Wx(i) * dx[i] + ex[i] + (i >= 6 ? gL[i - 6] : T(0)) + rdx[i];
    stv(C.kv(WF(rdx), k), ox);
    C.kv(WF(rdt), k)[0] = gt + rdt;
    if (hu) {
        T ou[NU];
        for (int i = 0; i < NU; ++i) ou[i] = C.Wu(i) * du[i] + eu[i] + gu[i] + rdu[i];
        stv(C.kv(WF(rdu), k), ou);
    }
    // equality rows
    if (hu) {
        T ax[9], bu[9], oe[9];
        opA(w, C.beta, dx, ax);
        opB<T, ROBOT>(st, du, bu);
        for (int i = 0; i < 9; ++i) oe[i] = ax[i] + bu[i] - dx1[i] + re1[i];
        stv(C.bv(WF(rde), 1 + k), oe);
    }
    if (k == 0 || k == N) {
        T ob[9];
        for (int i = 0; i < 9; ++i) ob[i] = dx[i] + re0[i];
        stv(C.bv(WF(rde), k == 0 ? 0 : N + 1), ob);
    }
    // dnu saved for the sum after the correction solve
    stv(C.bv(WF(dn0), k), dk);
    if (k == N) stv(C.bv(WF(dn0), N + 1), d1);
}

// z, nu, s, lambda += a * direction (dnu from the LDS vector)
template <typename T, int ROBOT> __device__ PHASE_ATTR void phase_update(const Ctx<T, ROBOT> &C, int k, T a, bool affine = false) {
    constexpr int NI = Rows<ROBOT>::NI;
    const int N = C.N;
    const LdsT<T> *vb = C.vb;
    {
        T x[9], dx[9], n1[9], n0[9], u[NU], du[NU];
        ldv(C.var_x(k), x);
        ldv(C.kv(WF(dx), k), dx);
        const T t = C.kv(WF(t), k)[0], dt = C.kv(WF(dt), k)[0];
        ldv(C.bv(WF(nu), 1 + k), n1);        // k < N: dynamics block k; k = N: final
        ldv(C.bv(WF(nu), 0), n0);
        ldv(C.var_u(k), u);
        ldv(C.kv(WF(du), k), du);
        for (int i = 0; i < 9; ++i) {
            x[i] += a * dx[i];
            n1[i] += a * vb[(1 + k) * 9 + i];
            n0[i] += a * vb[i];
        }
        for (int i = 0; i < NU; ++i) u[i] += a * du[i];
        stv(C.var_x(k), x);
        C.kv(WF(t), k)[0] = t + a * dt;
        stv(C.bv(WF(nu), 1 + k), n1);
        if (k == 0) stv(C.bv(WF(nu), 0), n0);
        if (k < N) stv(C.var_u(k), u);
    }
    const SV<T> s = C.kv(WF(s), k), lm = C.kv(WF(l), k);
    const SV<T> ds = C.kv(affine ? WF(dsa) : WF(ds), k), dl = C.kv(affine ? WF(dla) : WF(dl), k);
    T sv[NI], dsv[NI], lv[NI], dlv[NI];   // absent rows: ds = dl = 0 (s stays 1, lambda 0)
    ldv(s, sv); ldv(ds, dsv);
    ldv(lm, lv); ldv(dl, dlv);
    for (int r = 0; r < NI; ++r) { sv[r] += a * dsv[r]; lv[r] += a * dlv[r]; }
    stv(s, sv);
    stv(lm, lv);
}


// ---- solution polishing (the reference's osqp.setup(..., polish=True), src/scp_solver.py:62)
// Once the iterate meets the polishing tolerance, the equality-constrained QP on the guessed active
// set is solved with one more Newton step of the same structured system (oracle/ipm_mirror.py
// _polish is the CPU counterpart, step for step):
//   * active set from the Tapia indicators of the last step: row r is active when s_r / s_r,prev <
//     lambda_r / lambda_r,prev (s vanishing while lambda settles; lambda > s alone misreads rows
//     where both are small, e.g. the weakly active friction rows that hold the Newton tail), with
//     s_prev = s - alpha ds, lambda_prev = lambda - alpha dlambda from the last step's direction
//     (still in the ds / dl fields) and step length;
//   * active rows get s = rel lambda (D = 1 / rel, so D^-1 meets the push-through floors), inactive
//     rows lambda = rel s (D = rel: the row drops out); the residual pass, the Newton step with
//     sigma = 0 (predictor semantics) and a full step (alpha = 1) then give the reduced KKT solution;
//   * a residual pass verifies it: merit <= 1 at eps and s, lambda >= -tolerance on every row, i.e.
//     an exact KKT point (the minimizer); otherwise the iterate before the polish is restored and
//     the interior-point iterations go on.
// Backups while the polish runs: s, lambda in the ds, dl fields (whose last direction the
// classification has consumed), x, t, u in wx, wt, ub, nu in dn0 (fields no other phase uses then).
constexpr double POLISH_REL = 1e-14;
template <typename T, int ROBOT> __device__ PHASE_ATTR void phase_polish_prep(const Ctx<T, ROBOT> &C, int k, T alpha) {
    constexpr int NI = Rows<ROBOT>::NI;
    const int N = C.N;
    const unsigned msk = C.cmask(k);
    T s[NI], l[NI], ds[NI], dl[NI], x[9], u[NU], n1[9], n0[9];
    ldv(C.kv(WF(s), k), s);
    ldv(C.kv(WF(l), k), l);
    ldv(C.kv(WF(ds), k), ds);
    ldv(C.kv(WF(dl), k), dl);
    ldv(C.var_x(k), x);
    ldv(C.var_u(k), u);   // k = N: padding column
    ldv(C.bv(WF(nu), 1 + k), n1);
    ldv(C.bv(WF(nu), 0), n0);
    const T t = C.kv(WF(t), k)[0];
    const T rel = T(POLISH_REL);
    T s1[NI], l1[NI];
#pragma unroll
    for (int r = 0; r < NI; ++r) {
        const bool pr = Ctx<T, ROBOT>::present_m(k < N ? msk : 0u, r);
        const T sp = s[r] - alpha * ds[r], lp = l[r] - alpha * dl[r];
        const bool act = pr && s[r] * lp < l[r] * sp;
        s1[r] = act ? rel * l[r] : s[r];
        l1[r] = pr ? (act ? l[r] : rel * s[r]) : l[r];
    }
    stv(C.kv(WF(ds), k), s);
    stv(C.kv(WF(dl), k), l);
    stv(C.kv(WF(wx), k), x);
    C.kv(WF(wt), k)[0] = t;
    stv(C.kv(WF(ub), k), u);
    stv(C.bv(WF(dn0), 1 + k), n1);
    if (k == 0) stv(C.bv(WF(dn0), 0), n0);
    stv(C.kv(WF(s), k), s1);
    stv(C.kv(WF(l), k), l1);
}
// the iterate before the polish, back from its backups (a rejected polish)
template <typename T, int ROBOT> __device__ PHASE_ATTR void phase_polish_rollback(const Ctx<T, ROBOT> &C, int k) {
    constexpr int NI = Rows<ROBOT>::NI;
    T s[NI], l[NI], x[9], u[NU], n1[9], n0[9];
    ldv(C.kv(WF(ds), k), s);
    ldv(C.kv(WF(dl), k), l);
    ldv(C.kv(WF(wx), k), x);
    ldv(C.kv(WF(ub), k), u);
    ldv(C.bv(WF(dn0), 1 + k), n1);
    ldv(C.bv(WF(dn0), 0), n0);
    const T t = C.kv(WF(wt), k)[0];
    stv(C.kv(WF(s), k), s);
    stv(C.kv(WF(l), k), l);
    stv(C.var_x(k), x);
    if (k < C.N) stv(C.var_u(k), u);
    C.kv(WF(t), k)[0] = t;
    stv(C.bv(WF(nu), 1 + k), n1);
    if (k == 0) stv(C.bv(WF(nu), 0), n0);
}

// initialization step: full Newton step for z and nu; s = h - gz at the new z; lambda += dlambda.
// vmax receives (max -s, max -lambda) over this knot's rows.
// Starting point after the initialization step: s = h - g'z at the new z for the present rows
// (absent rows keep s = 1, lambda = 0: their affine step is zero).  Solo12: s and lambda floored
// row by row (cmpc_qp_settings init_floor_s / _l, default 0.1).  TALOS, or floors 0: vmax
// collects the largest violations for CVXOPT's shift of every row (phase_init_shift).  On Solo12
// the shift starts at mu ~ 700, far from the central path (trot N=100 x 1024: 9.1 Newton steps
// on average, max 12; 5.2, max 7 with the floors); on TALOS the floors were not robust
// (oracle/ipm_mirror.py).  Branch-free with each row group's loads batched.
template <typename T, int ROBOT>
__device__ __forceinline__ void init_s_knot(const Ctx<T, ROBOT> &C, int k, T (&vmax)[2], const T *__restrict__ stp,
                                            const T *__restrict__ xs, const T *__restrict__ us,
                                            const T *__restrict__ ts, T *__restrict__ ss, T *__restrict__ ls) {
    using S = Stage<ROBOT>;
    using R_ = Rows<ROBOT>;
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    constexpr int ld = KPC;
    const bool hu = k < C.N;
    const SV<const T> st{stp};
    const unsigned msk = C.cmask(k);
    T x[3], u[NU];
    for (int i = 0; i < 3; ++i) x[i] = xs[(6 + i) * ld];
    for (int i = 0; i < NU; ++i) u[i] = us[i * ld];   // k = N: padding column (unused)
    const T t = ts[0];
    const bool floors = ROBOT == 0 && C.fls > T(0);
    auto put = [&](int r, bool pr, T v) {   // v = g'z - h
        const T l = ls[r * ld];
        if (floors) {
            ss[r * ld] = pr ? fmax(-v, C.fls) : T(1);
            ls[r * ld] = pr ? fmax(l, C.fll) : l;
        } else {
            ss[r * ld] = pr ? -v : T(1);
            vmax[0] = fmax(vmax[0], pr ? v : T(-1e300));
            vmax[1] = fmax(vmax[1], pr ? -l : T(-1e300));
        }
    };
#pragma unroll
    for (int j = 0; j < 8; ++j)
        put(j, true, tr_sign<T>(j, 0) * x[0] + tr_sign<T>(j, 1) * x[1] + tr_sign<T>(j, 2) * x[2] + C.cw * t - st[S::BTR + j]);
    put(8, true, -t);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const bool pr = hu && ((msk >> c) & 1u);
        const auto cs = st + (S::CON + S::CS * c);
        T G[12], H[4];
        for (int e = 0; e < 12; ++e) G[e] = cs[S::G + e];
        for (int r = 0; r < 4; ++r) H[r] = cs[S::H + r];
        const T *f = u + NUPC * c + FO;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            put(R_::FR + 4 * c + r, pr, G[3 * r] * f[0] + G[3 * r + 1] * f[1] + G[3 * r + 2] * f[2] - H[r]);
        if (ROBOT == 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {   // cop <= hi | -cop <= -lo
                const int dd = q / 2;
                const T cop = u[NUPC * c + dd];
                put(R_::CP + 4 * c + q, pr,
                    (q % 2 == 0) ? cop - C.prm->foot_range[dd == 0 ? 0 : 2] : -cop - C.prm->foot_range[dd == 0 ? 1 : 3]);
            }
        }
    }
}

template <typename T, int ROBOT> __device__ PHASE_ATTR void phase_init_step(const Ctx<T, ROBOT> &C, int k, T (&vmax)[2]) {
    phase_update<T, ROBOT>(C, k, T(1), true);   // z, nu, lambda: full affine step; s recomputed below
    T *ws = C.ws;
    init_s_knot<T, ROBOT>(C, k, vmax, C.stage + k, ws + WF(x) * KPC + k, ws + WF(u) * KPC + k, ws + WF(t) * KPC + k,
                          ws + WF(s) * KPC + k, ws + WF(l) * KPC + k);
}
template <typename T, int ROBOT> __device__ PHASE_ATTR void phase_init_shift(const Ctx<T, ROBOT> &C, int k, T sh_s, T sh_l) {
    constexpr int NI = Rows<ROBOT>::NI;
    const SV<T> s = C.kv(WF(s), k), lm = C.kv(WF(l), k);
    for (int r = 0; r < NI; ++r) {
        if (!C.present(k, r)) continue;
        s[r] += sh_s;
        lm[r] += sh_l;
    }
}

// Forward elimination + separator / meeting-block solve of the right-hand side in vb, and the back
// substitution, with the factors of this Newton step: the two-ended recurrence (one or two waves)
// or the four chains of schur_pt.hpp (four waves).  Barriers included.
template <typename T, int NTT, int WG, typename CT>
__device__ __forceinline__ void schur_forward(const CT &C, int NB, int NBm, LdsT<T> *ring, LdsT<T> *shl) {
    const int tid = threadIdx.x & (NTT - 1);
    if constexpr (NTT >= 256) {
        pt_solve_elim<T>(C.So, NB, C.sp, C.vb, ring, C.sbv);
        gsync<NTT, WG>();
        pt_fill_rhs<T, NTT>(C.Sh, C.sp, C.vb, C.hy);
        gsync<NTT, WG>();
        if (tid < 64) {
            pt_fill_sum<T>(C.sp, C.hy, C.sbv);
            pt_reduced<T>(C.Sd, C.Sx, C.sp, shl, C.vb, C.sbv, false);
        }
        gsync<NTT, WG>();
    } else {
        if (tid < 64) tw_solve_elim<T>(C.So, NB, NBm, C.vb, ring);
        gsync<NTT, WG>();
        if (tid < 64) tw_solve_meet<T>(C.Sd, C.So, NB, NBm, C.vb, shl);
        gsync<NTT, WG>();
    }
}
template <typename T, int NTT, int WG, typename CT>
__device__ __forceinline__ void schur_backward(const CT &C, int NB, int NBm, LdsT<T> *ring) {
    const int tid = threadIdx.x & (NTT - 1);
    if constexpr (NTT >= 256) {
        pt_solve_local<T, NTT>(C.Sd, C.Sh, NB, C.sp, C.vb);
        gsync<NTT, WG>();
        pt_solve_back<T>(C.So, NB, C.sp, C.vb, ring);
        gsync<NTT, WG>();
    } else {
        tw_solve_local<T, NTT>(C.Sd, NB, NBm, C.vb);
        gsync<NTT, WG>();
        if (tid < 64) tw_solve_back<T>(C.So, NB, NBm, C.vb, ring);
        gsync<NTT, WG>();
    }
}

// One step of iterative refinement of the corrector direction; returns the new step bound.
// (Inlined: as an outlined call, the registers live across it were reloaded from scratch all over
// the Newton step.)
template <typename T, int ROBOT, int NTT, int WG>
__device__ __forceinline__ T refine_direction(const Ctx<T, ROBOT> &C, T sigma_mu, LdsT<T> *ring, LdsT<T> *shl,
                                                        T *red) {
    const int tid = threadIdx.x & (NTT - 1), K1 = C.N + 1, NB = C.N + 2, NBm = NB / 2;
    for (int k = tid; k < K1; k += NTT) phase_lres<T, ROBOT>(C, k, sigma_mu);
    gsync<NTT, WG>();
    for (int k = tid; k < K1; k += NTT) phase_w<T, ROBOT>(C, k, 2, T(0));
    gsync<NTT, WG>();
    if (NTT > 64) {
        add_wx<T, NTT>(C.vb, C.wxs, C.N);
        gsync<NTT, WG>();
    }
    schur_forward<T, NTT, WG>(C, NB, NBm, ring, shl);
    schur_backward<T, NTT, WG>(C, NB, NBm, ring);
    T ar[1] = {T(1)};
    for (int k = tid; k < K1; k += NTT) ar[0] = fmin(ar[0], phase_dz_refine<T, ROBOT>(C, k));
    block_reduce<T, NTT, 1, 2, WG>(ar, red);   // (its barriers order the dnu reads before the sum)
    for (int e = tid; e < NB * 9; e += NTT) C.vb[e] += C.ws[(WF(dn0) + e % 9) * KPC + e / 9];
    gsync<NTT, WG>();
    return ar[0];
}

// ------------------------------------------------------------------ kernels
// Four-wave groups: the per-knot phases use only the first two waves at one knot per thread (up to
// 128 knots), and their time is one knot's instruction stream, so the heaviest ones (residual,
// direction) split each knot into a state part (waves 0, 1) and a contact part (waves 2, 3).
template <int G> constexpr bool split_knots() { return G >= 256; }

// Stopping test: primal residual <= eps_abs + eps_rel * (primal scale), dual residual and the
// largest complementarity product s_i lambda_i <= eps_abs + eps_rel * (dual scale).  On degenerate
// Solo12 trot problems the dual scale (~1e5, dominated by the dynamics multipliers' E' nu) lets a
// solve stop with one friction row at s lambda ~ 5e-6 and a solution up to 7e-5 away from the exact
// minimizer (the round-4 headline check).  Such problems are exactly the ones whose polishing guess
// fails (their active set is undecided), so on Solo12 fp64 a problem whose polish was rejected (or
// with polishing off) measures complementarity against 10x the primal tolerance instead, which lands
// it within 4e-7 (64 trot N=100 problems of the CPU mirror); every other problem ends polished, i.e.
// at the exact minimizer.  Same-box (profiles/r04a_stop_ab.log): the primal test for every problem
// took 4.67 Newton steps and 282k SCP it/s, this one 3.2 and ~340k.  TALOS keeps the dual scale
// (within 9e-7 of the minimizer already), and so does fp32.
#ifdef CMPC_COMP_DUAL   // diagnostic builds: round 3's test (the dual scale) for every robot
template <int ROBOT> __device__ __forceinline__ constexpr bool COMP_PRIMAL_SCALE() { return false; }
#else
template <int ROBOT> __device__ __forceinline__ constexpr bool COMP_PRIMAL_SCALE() { return ROBOT == 0; }
#endif

// Newton-loop state of one problem's solve (carried across k_qp_group's change of mode).  A solve
// handed over after the stopping test of iteration `it` (yielded) resumes there on all waves: the
// residual pass of that iteration is done (its outputs are in the workspace), and mu / cnt are its
// complementarity mean and row count.
template <typename T> struct IpmState {
    int status, it, stall, n_refine, yielded, resume, tail;
    int ptried, polish;   // polishing attempts / the outcome (1 accepted, -1 rejected)
    int pit;              // iteration of the last attempt (a second one needs a Newton step since)
    T mu_prev, merit, prim_prev, mu, cnt;
    T alpha_last;         // step length of the last Newton step (the polish's active-set guess)
#ifdef CMPC_STAMPS
    unsigned long long t_acc[12];
#endif
};
template <typename T> __device__ __forceinline__ IpmState<T> ipm_state0() {
    IpmState<T> S;
    S.status = CMPC_QP_MAX_ITER;
    S.it = S.stall = S.n_refine = S.yielded = S.resume = S.tail = S.ptried = S.polish = S.pit = 0;
    S.mu_prev = T(-1);
    S.merit = S.prim_prev = S.mu = S.cnt = T(0);
    S.alpha_last = T(1);
#ifdef CMPC_STAMPS
    for (int i = 0; i < 12; ++i) S.t_acc[i] = 0;
#endif
    return S;
}

// LDS of one solve besides what Ctx points to: this thread's sweep ring, the recurrence scratch
// of the two ends, the reduction scratch (private to the group)
template <typename T> struct IpmLds {
    LdsT<T> *ring, *shl;
    T *red;
};

// Problem b's context; its cost weights and contact masks copied by the group's G threads into
// the given LDS slots (the caller syncs the group before they are read)
template <typename T, int ROBOT, int G>
__device__ __forceinline__ void ctx_setup(const DevBuf<T> &d, int b, Ctx<T, ROBOT> &C, LdsT<T> *wts, LdsT<uint8_t> *cms,
                                          T floor_s, T floor_l) {
    const int tid = threadIdx.x & (G - 1), N = d.N, K1 = N + 1;
    C.N = N;
    C.prm = d.params + d.class_id[b];
    C.stage = d.stage + (size_t)b * Stage<ROBOT>::SIZE * KPC;
    C.logic = d.logic + (size_t)b * N * Robot<ROBOT>::NC;
    C.xbar = d.Xbar + (size_t)b * K1 * 9;
    C.cw = d.cw[b];
    C.beta = C.prm->dt / C.prm->mass;
    C.fls = floor_s;
    C.fll = floor_l;
    {
        T wmax = T(1);
        for (int i = 0; i < 9; ++i) wmax = fmax(wmax, C.prm->Wx[i]);
        C.dcap = T(1e12) * wmax;
    }
    C.ws = d.ws + (size_t)b * d.ws_stride;
    if (tid < 9) { wts[tid] = C.prm->Wx[tid]; wts[9 + tid] = T(1) / C.prm->Wx[tid]; }
    if (tid < NU) { wts[18 + tid] = C.prm->Wu[tid]; wts[18 + NU + tid] = T(1) / C.prm->Wu[tid]; }
    C.wt = wts;
    // contact masks of every knot, once per solve (each phase read them from global memory
    // first thing, and everything after waited on that load)
    C.cm = nullptr;
    for (int k = tid; k < K1; k += G) cms[k] = (uint8_t)C.cmask_mem(k);
    C.cm = cms;
    C.Sd = C.ws + Ws<ROBOT>::Sd;
    C.So = C.ws + Ws<ROBOT>::So;
}

// Starting point of the initialization step: z = (xlin, ulin, 0), nu = 0, s = lambda = 1
template <typename T, int ROBOT, int G, int WG>
__device__ __forceinline__ void ipm_start(const DevBuf<T> &d, const Ctx<T, ROBOT> &C, int b) {
    constexpr int NI = Rows<ROBOT>::NI;
    const int tid = threadIdx.x & (G - 1), N = C.N, K1 = N + 1, NB = N + 2;
    for (int k = tid; k < K1; k += G) {
        const SV<T> x = C.var_x(k);
        const T *xl = d.Xlin + ((size_t)b * K1 + k) * 9;   // start at the linearization point
        const T *ubar = d.Ulin + ((size_t)b * N + (k < N ? k : 0)) * NU;
        T xv[9], uv[NU];   // loads first (interleaved with the stores they would be serialized)
        for (int i = 0; i < 9; ++i) xv[i] = xl[i];
        for (int i = 0; i < NU; ++i) uv[i] = ubar[i];
        for (int i = 0; i < 9; ++i) x[i] = xv[i];
        C.kv(WF(t), k)[0] = T(0);
        if (k < N) { const SV<T> u = C.var_u(k); for (int i = 0; i < NU; ++i) u[i] = uv[i]; }
        const SV<T> s = C.kv(WF(s), k), lm = C.kv(WF(l), k), dsa = C.kv(WF(dsa), k), dla = C.kv(WF(dla), k);
        const unsigned msk = C.cmask(k);
        for (int r = 0; r < NI; ++r) {
            s[r] = T(1);
            lm[r] = Ctx<T, ROBOT>::present_m(msk, r) ? T(1) : T(0);
            dsa[r] = T(0);
            dla[r] = T(0);
        }
    }
    for (int j = tid; j < NB; j += G) {
        const SV<T> nu = C.bv(WF(nu), j);
        for (int i = 0; i < 9; ++i) nu[i] = T(0);
    }
    gsync<G, WG>();
}

// Hand-over of a grouped problem (k_qp_group), decided by the problems' Newton-step counts only,
// never by timing.  gf: per wave of the workgroup, cont[w] (gf[w]) = the last iteration whose
// stopping test let wave w's problem continue, done[w] (gf[4 + w]) = 1 once it has left its loop
// (cont frozen).  After its own stopping test of iteration `it` let it continue, a wave publishes
// cont[w] = it and asks whether every other problem of the group finished by iteration `it` (done
// with cont < it).  It waits only for problems whose status at `it` is not yet published, and only
// while none is known to continue (cont >= it); every wave publishes before it waits, so no two
// waves wait on each other.  So the last problem is handed over right after the stopping test of
// the iteration in which the slowest other problem stopped, whatever the waves' relative speed:
// results are bit-reproducible (tests/test_gpu_qp_pair.py).  The spin is bounded (~60 ms); past it
// the problem just finishes on its own wave (correct, only slower).
__device__ __forceinline__ bool group_handover(LdsT<int> *gf, int P, int w, int it) {
    volatile LdsT<int> *cont = gf, *done = gf + 4;
    if ((threadIdx.x & 63) == 0) cont[w] = it;
    for (int spin = 0; spin < (1 << 20); ++spin) {
        bool any_cont = false, unknown = false;
        for (int q = 0; q < P; ++q) {
            if (q == w) continue;
            const int dq = __builtin_amdgcn_readfirstlane(done[q]);   // done before cont: cont is
            const int cq = __builtin_amdgcn_readfirstlane(cont[q]);   // final once done reads 1
            if (cq >= it) any_cont = true;
            else if (!dq) unknown = true;
        }
        if (any_cont) return false;
        if (!unknown) return true;
        __builtin_amdgcn_s_sleep(2);
    }
    return false;
}
__device__ __forceinline__ void group_done(LdsT<int> *gf, int w) {
    if ((threadIdx.x & 63) == 0) ((volatile LdsT<int> *)gf)[4 + w] = 1;
}

// Newton iterations of problem b on a group of G threads (the workgroup, or one wave of a WG-thread
// workgroup), from S.it until the stopping test, a failure exit or the cap (S.resume: from after the
// stopping test of S.it).  With gf set (k_qp_group, one wave per problem), the loop also leaves
// (S.yielded) when group_handover hands the problem to the whole workgroup.
template <typename T, int ROBOT, int G, int WG>
__device__ __forceinline__ void ipm_loop(const DevBuf<T> &d, const Ctx<T, ROBOT> &C, int b, IpmState<T> &S,
                                         const IpmLds<T> &L, int max_iter, T eps_abs, T eps_rel, T eta,
                                         T polish_eps, LdsT<int> *gf = nullptr, int gP = 0, int yield_at = 0) {
    const int tid = threadIdx.x & (G - 1), N = C.N, K1 = N + 1, NB = N + 2, NBm = NB / 2;
    (void)b;
#ifdef CMPC_STAMPS
    unsigned long long t_prev = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                                               \
    do {                                                                       \
        const unsigned long long t_now = __builtin_amdgcn_s_memtime();         \
        S.t_acc[i] += t_now - t_prev;                                          \
        t_prev = t_now;                                                        \
    } while (0)
#else
#define STAMP(i) do { } while (0)
#endif
    int status = S.status, it = S.it, stall = S.stall, n_refine = S.n_refine;
    T mu_prev = S.mu_prev, merit = S.merit, prim_prev = S.prim_prev, alpha_last = S.alpha_last;
    bool resume = S.resume != 0;
    S.resume = 0;
    // pm: 0 a Newton step; 1 the polishing step (its own residual pass and Newton system, full step);
    // 2 the residual pass that verifies the polished iterate (accepted: solved; rejected: rolled back
    // and iteration `it` redone as a Newton step, the stopping-test state restored)
    int pm = 0, stall_s = 0;
    T mu_prev_s = T(0), prim_prev_s = T(0);
    // it == 0 is the initialization step: one full Newton step from s = lambda = 1 gives an
    // equality-feasible least-squares start; s and lambda are then floored row by row (Solo12)
    // or shifted by 1 + the largest violation (TALOS), see init_s_knot.
    for (it = S.it; it <= max_iter;) {
        const bool init = (it == 0) && pm == 0;
        T mu, cnt;   // complementarity mean and row count of this iteration's residual pass
        if (resume) {   // handed over after this iteration's stopping test (k_qp_group)
            resume = false;
            mu = S.mu;
            cnt = S.cnt;
        } else {
        if (pm == 1) {   // polishing: active-set guess, backups, the reduced system's s and lambda
            for (int k = tid; k < K1; k += G) phase_polish_prep<T, ROBOT>(C, k, alpha_last);
            gsync<G, WG>();
        }
        Norms<T, ROBOT> nm{0, 0, 0, 0, 0, 0, 0, 0, big_value<T>(), big_value<T>()};
        if constexpr (split_knots<G>()) {   // a thread pair per knot: state part | contact part
            // (the part is the wave's: a uniform branch)
            if (__builtin_amdgcn_readfirstlane(tid) < 128) {
                for (int k = tid & 127; k < K1; k += 128) phase_residual<T, ROBOT, 0>(C, k, nm);
            } else {
                for (int k = tid & 127; k < K1; k += 128) phase_residual<T, ROBOT, 1>(C, k, nm);
            }
        } else {
            for (int k = tid; k < K1; k += G) phase_residual<T, ROBOT>(C, k, nm);
        }
        T mx[6] = {nm.prim, nm.dual, nm.comp, nm.sp, nm.sd, nm.lmax};
        block_reduce<T, G, 6, 1, WG>(mx, L.red);
        T sm2[2] = {nm.mu, nm.cnt};
        block_reduce<T, G, 2, 0, WG>(sm2, L.red);
        STAMP(0);
        const T prim = mx[0], dual = mx[1], comp = mx[2], sp = mx[3], sdd = mx[4];
        mu = sm2[0] / fmax(sm2[1], T(1));
        cnt = sm2[1];
        // complementarity against the dual scale; on Solo12 fp64, once a polish was rejected (or
        // with polishing off), against 10x the primal tolerance instead (COMP_PRIMAL_SCALE)
        const bool strict = COMP_PRIMAL_SCALE<ROBOT>() && sizeof(T) == 8 && (!(polish_eps > T(0)) || S.polish < 0);
        const T ep = eps_abs + eps_rel * sp, ed = eps_abs + eps_rel * sdd, ec = strict ? T(10) * ep : ed;
        if (pm == 2) {   // the polished iterate: an exact KKT point within eps, or back to the old one
            T mn[2] = {nm.smin, nm.lmin};
            block_reduce<T, G, 2, 2, WG>(mn, L.red);
            // primal side 100x tighter than the stopping test: the interior-point iterates satisfy
            // their rows to rounding, and a polished point must not trade that for its active set
            // (a TALOS N=50 polish verified at eps left a 1.7e-8 row violation)
            const T mp = fmax(prim / (T(0.01) * ep), fmax(dual / ed, comp / ec));
            if (mp <= T(1) && mn[0] >= -T(0.01) * ep && mn[1] >= -ed && mu == mu) {   // (mu: the non-finite detector)
                merit = mp;
                status = CMPC_QP_SOLVED;
                S.polish = 1;
                break;
            }
            S.polish = -1;
            for (int k = tid; k < K1; k += G) phase_polish_rollback<T, ROBOT>(C, k);
            gsync<G, WG>();
            stall = stall_s;
            mu_prev = mu_prev_s;
            prim_prev = prim_prev_s;
            pm = 0;
            continue;   // iteration `it` again, as a Newton step
        }
        if (pm == 1) goto newton_system;
        merit = fmax(prim / ep, fmax(dual / ed, comp / ec));
        if (!(merit == merit) || !(mu == mu)) { status = CMPC_QP_NONFINITE; break; }
        stall_s = stall;
        mu_prev_s = mu_prev;
        prim_prev_s = prim_prev;
        if (!init) {
            if (merit <= T(1)) { status = CMPC_QP_SOLVED; break; }
            // primal infeasibility (Farkas, OSQP's test on the diverging multipliers), checked once
            // the primal residual stagnates away from the solution:
            // |E'nu + G'lambda| <= eps |(nu, lambda)| and b'nu + h'lambda <= -eps |(nu, lambda)|
            if (it >= 3 && prim > T(0.9) * prim_prev && merit > T(1e3)) {
                T cm[2] = {T(0), mx[5]}, cs[1] = {T(0)};
                for (int k = tid; k < K1; k += G) phase_cert<T, ROBOT>(C, k, cm, cs[0]);
                block_reduce<T, G, 2, 1, WG>(cm, L.red);
                block_reduce<T, G, 1, 0, WG>(cs, L.red);
                if (cm[0] <= T(QP_EPS_PINF) * cm[1] && cs[0] <= -T(QP_EPS_PINF) * cm[1]) {
                    status = CMPC_QP_PRIMAL_INFEASIBLE;
                    break;
                }
            }
            prim_prev = prim;
            // stall guard: mu not decreasing for 3 iterations while within 1e3x of the tolerance;
            // reported as 'solved inaccurate', a failure for the SCP loop as in the reference (Q13)
            stall = (mu_prev >= T(0) && mu >= T(0.5) * mu_prev) ? stall + 1 : 0;
            mu_prev = mu;
            if (stall >= 3 && merit <= T(1e3)) { status = CMPC_QP_SOLVED_INACCURATE; break; }
        }
        if (it == max_iter) break;
        // polishing once the iterate meets polish_eps (after at least one Newton step past the
        // initialization, whose direction the active-set guess reads)
        if (polish_eps > T(0) && !S.ptried && it > 1 &&
            fmax(prim / (polish_eps * (T(1) + sp)), fmax(dual, comp) / (polish_eps * (T(1) + sdd))) <= T(1)) {
            S.ptried = 1;
            S.pit = it;
            pm = 1;
            continue;
        }
        // a second attempt for a problem whose first guess failed, once it meets the dual-scale test
        // at eps (the strict test then still runs): the active set is usually settled by then (CPU
        // mirror: 3 of the 4 rejected problems of 64, one Newton step less each, exact solutions)
        if (strict && S.ptried == 1 && S.polish < 0 && it > S.pit && fmax(prim / ep, fmax(dual, comp) / ed) <= T(1)) {
            S.ptried = 2;
            S.pit = it;
            pm = 1;
            continue;
        }
        // k_qp_group: every other problem of the workgroup has stopped, so this one continues on
        // all waves from here (the residual pass of this iteration is in the workspace)
        // split launch (k_qp_ipm MODE 1, head): a problem still running after the stopping test of
        // iteration yield_at leaves for the tail launch, which resumes it here on all its waves
        if ((gf && group_handover(gf, gP, (int)(threadIdx.x >> 6), it)) || (yield_at > 0 && it >= yield_at)) {
            S.yielded = 1;
            S.resume = 1;
            S.mu = mu;
            S.cnt = cnt;
            break;
        }
        }   // (residual pass and stopping test)
    newton_system:
        // ---- Phi factors and the predictor's particular solution (knot-local), then the S blocks
        // and the predictor's Schur right-hand side
        if constexpr (split_knots<G>()) {
            if (__builtin_amdgcn_readfirstlane(tid) < 128) {
                for (int k = tid & 127; k < K1; k += 128) {
                    KnotSL<T, ROBOT> kl;
                    load_knot_sl(C, k, kl);
                    phase_factor<T, ROBOT, 0>(C, k, kl);
                    phase_w_pred<T, ROBOT, 0>(C, k, kl);
                }
            } else {
                for (int k = tid & 127; k < K1; k += 128) {
                    KnotSL<T, ROBOT> kl;
                    load_knot_sl(C, k, kl);
                    phase_factor<T, ROBOT, 1>(C, k, kl);
                    phase_w_pred<T, ROBOT, 1>(C, k, kl);
                }
            }
        } else {
            for (int k = tid; k < K1; k += G) {
                KnotSL<T, ROBOT> kl;
                load_knot_sl(C, k, kl);
                phase_factor<T, ROBOT>(C, k, kl);
                phase_w_pred<T, ROBOT>(C, k, kl);
            }
        }
        gsync<G, WG>();
        STAMP(1);
        if (G > 64) add_wx<T, G>(C.vb, C.wxs, N, C.bus);
        for (int k = tid; k < K1; k += G) phase_sblock<T, ROBOT>(C, k);
        gsync<G, WG>();
        STAMP(2);
        // ---- factorization of S with the predictor's forward elimination fused in
#ifdef CMPC_STAMPS
        unsigned long long *fst = d.stamps + (size_t)b * 16;
#else
        unsigned long long *fst = nullptr;
#endif
        if (G >= 256) {   // four chains and the separator system (schur_pt.hpp)
#ifdef CMPC_STAMPS
            const unsigned long long tc0 = __builtin_amdgcn_s_memtime();
#endif
            pt_factor_chains<T>(C.Sd, C.So, C.Sh, C.Sx, NB, C.sp, L.shl, C.vb, C.sbv);   // (this wave's scratch)
#ifdef CMPC_STAMPS
            const unsigned long long tc1 = __builtin_amdgcn_s_memtime();
#endif
            gsync<G, WG>();
#ifdef CMPC_STAMPS
            const unsigned long long tc2 = __builtin_amdgcn_s_memtime();
#endif
            if (tid < 64) pt_reduced<T>(C.Sd, C.Sx, C.sp, L.shl, C.vb, C.sbv, true);
            gsync<G, WG>();
#ifdef CMPC_STAMPS
            if (tid == 0) { fst[12] += tc1 - tc0; fst[13] += tc2 - tc1; fst[14] += __builtin_amdgcn_s_memtime() - tc2; }
            if (tid == 64) fst[15] += tc1 - tc0;   // an interior chain
#endif
        } else {
            if (G >= 128) {   // one end per wave (waves 0 and 1)
                if (tid < 128) tw_factor_ends<T, 64>(C.Sd, C.So, NB, NBm, L.shl, C.vb, fst);
            } else {            // one end per half of wave 0
                tw_factor_ends<T, 32>(C.Sd, C.So, NB, NBm, L.shl, C.vb, fst);
            }
            gsync<G, WG>();
            if (tid < 64) tw_factor_meet<T>(C.Sd, C.So, NBm, L.shl, C.vb);
            gsync<G, WG>();
        }
        STAMP(3);
        // ---- predictor (affine) and corrector; the initialization step and the polishing step take the
        // predictor's direction alone (full stores into the affine fields)
        const bool one_step = init || pm == 1;
        T sigma_mu = T(0);
        T alpha = T(1);
        for (int corr = 0; corr < 2; ++corr) {
            if (corr) {
                if constexpr (split_knots<G>()) {
                    if (__builtin_amdgcn_readfirstlane(tid) < 128) {
                        for (int k = tid & 127; k < K1; k += 128) phase_w<T, ROBOT, 0>(C, k, corr, sigma_mu);
                    } else {
                        for (int k = tid & 127; k < K1; k += 128) phase_w<T, ROBOT, 1>(C, k, corr, sigma_mu);
                    }
                } else {
                    for (int k = tid; k < K1; k += G) phase_w<T, ROBOT>(C, k, corr, sigma_mu);
                }
                gsync<G, WG>();
                if (G > 64) {
                    add_wx<T, G>(C.vb, C.wxs, N, C.bus);
                    gsync<G, WG>();
                }
                STAMP(4);
                STAMP(5);   // (the right-hand side is formed inside phase_w)
                schur_forward<T, G, WG>(C, NB, NBm, L.ring, L.shl);
            }
            schur_backward<T, G, WG>(C, NB, NBm, L.ring);
            STAMP(6);
            T am[1] = {T(1)}, mus[3] = {T(0), T(0), T(0)};
            if constexpr (split_knots<G>()) {
                if (__builtin_amdgcn_readfirstlane(tid) < 128) {
                    for (int k = tid & 127; k < K1; k += 128) am[0] = fmin(am[0], phase_dz<T, ROBOT, 0>(C, k, corr, one_step, sigma_mu, mus));
                } else {
                    for (int k = tid & 127; k < K1; k += 128) am[0] = fmin(am[0], phase_dz<T, ROBOT, 1>(C, k, corr, one_step, sigma_mu, mus));
                }
            } else {
                for (int k = tid; k < K1; k += G) am[0] = fmin(am[0], phase_dz<T, ROBOT>(C, k, corr, one_step, sigma_mu, mus));
            }
            block_reduce<T, G, 1, 2, WG>(am, L.red);
            STAMP(7);
            alpha = am[0];
            if (one_step) break;
            if (corr == 0) {   // Mehrotra centering from the affine step's complementarity
                block_reduce<T, G, 3, 0, WG>(mus, L.red);
                const T mu_aff = (mus[0] + alpha * (mus[1] + alpha * mus[2])) / fmax(cnt, T(1));
                const T sg = mu_aff / fmax(mu, std::numeric_limits<T>::min());
                sigma_mu = sg * sg * sg * mu;
            } else if ((alpha < T(QP_REFINE_ALPHA) || stall > 0) && merit < T(QP_REFINE_MERIT)) {
                // the step collapsed, or mu did not halve in the last iteration, late in the solve:
                // one step of iterative refinement of the corrector direction (residual of the
                // Newton system with the exact operators, correction solved with the same
                // factorization; see oracle/ipm_mirror.py)
                alpha = refine_direction<T, ROBOT, G, WG>(C, sigma_mu, L.ring, L.shl, L.red);
                ++n_refine;
            }
        }
        if (init) {
            T vmax[2] = {T(-1e300), T(-1e300)};
            for (int k = tid; k < K1; k += G) phase_init_step<T, ROBOT>(C, k, vmax);
            if (ROBOT == 1 || !(C.fls > T(0))) {   // CVXOPT shift (Solo12 floors inside init_s_knot)
                block_reduce<T, G, 2, 1, WG>(vmax, L.red);
                const T sh_s = vmax[0] >= T(0) ? T(1) + vmax[0] : T(0);
                const T sh_l = vmax[1] >= T(0) ? T(1) + vmax[1] : T(0);
                for (int k = tid; k < K1; k += G) phase_init_shift<T, ROBOT>(C, k, sh_s, sh_l);
            }
            gsync<G, WG>();
            ++it;
            continue;
        }
        if (pm == 1) {   // the reduced system's solution: a full step, verified by the next residual pass
            for (int k = tid; k < K1; k += G) phase_update<T, ROBOT>(C, k, T(1), true);
            gsync<G, WG>();
            pm = 2;
            continue;
        }
        alpha = fmin(T(1), eta * alpha);
        for (int k = tid; k < K1; k += G) phase_update<T, ROBOT>(C, k, alpha);
        gsync<G, WG>();
        STAMP(8);
        alpha_last = alpha;
        ++it;
    }
    S.status = status;
    S.it = it;
    S.stall = stall;
    S.n_refine = n_refine;
    S.mu_prev = mu_prev;
    S.merit = merit;
    S.prim_prev = prim_prev;
    S.alpha_last = alpha_last;
#undef STAMP
}

// Solution, multipliers and exit record of problem b
template <typename T, int ROBOT, int G>
__device__ __forceinline__ void ipm_finish(const DevBuf<T> &d, const Ctx<T, ROBOT> &C, int b, const IpmState<T> &S) {
    constexpr int NI = Rows<ROBOT>::NI;
    const int tid = threadIdx.x & (G - 1), N = C.N, K1 = N + 1, NB = N + 2;
    for (int k = tid; k < K1; k += G) {
        T x[9], u[NU], lm[NI];
        ldv(C.var_x(k), x);
        ldv(C.var_u(k), u);
        ldv(C.kv(WF(l), k), lm);
        const unsigned msk = C.cmask(k);
        for (int i = 0; i < 9; ++i) d.xs[((size_t)b * K1 + k) * 9 + i] = x[i];
        d.ts[(size_t)b * K1 + k] = C.kv(WF(t), k)[0];
        if (k < N) for (int i = 0; i < NU; ++i) d.us[((size_t)b * N + k) * NU + i] = u[i];
        // (fmax: a polished solution's inactive rows carry multipliers of rounding size, either sign)
        for (int r = 0; r < NI; ++r)
            d.lams[((size_t)b * K1 + k) * NI + r] = Ctx<T, ROBOT>::present_m(msk, r) ? fmax(lm[r], T(0)) : T(0);
    }
    for (int e = tid; e < NB * 9; e += G) d.nus[(size_t)b * NB * 9 + e] = C.ws[(WF(nu) + e % 9) * KPC + e / 9];
    if (tid == 0) {
        d.qp_status[b] = S.status;
        d.qp_iters[b] = S.it;
        d.qp_merit[b] = S.merit;
        d.qp_nref[b] = S.n_refine;
        d.qp_tail[b] = S.tail;
        d.qp_polish[b] = S.polish;
#ifdef CMPC_STAMPS
        for (int i = 0; i < 9; ++i) d.stamps[(size_t)b * 16 + i] = S.t_acc[i];   // 9..11: k_linearize, 12..15: tw_factor_ends
#endif
    }
}

// One workgroup per problem: one, two or four waves (cmpc_api.cpp qp_waves).
// Split launches (MODE; cmpc_api.cpp qp_split): a launch of one (two) waves per problem that fills
// the device lasts as long as its slowest problems.  MODE 1 (head, one or two waves per problem)
// lets a problem still running after the stopping test of iteration split[0] leave: its
// Newton-loop state goes to d.qp_state and its index to the tail list split[2 + i] (count split[1]);
// MODE 2 (tail, two or four waves per problem) resumes the listed problems there, one per workgroup
// (workgroups past the count leave at once).  Which problems leave depends on Newton-step counts
// only, and a resumed problem runs the all-wave algorithm from that iteration, so results are
// reproducible run to run.  MODE 0: the whole solve.
template <typename T, int ROBOT, int NTT, int MODE>
__global__ void __launch_bounds__(NTT, NTT == 128 ? QP_MIN_WAVES_2W : QP_MIN_WAVES) k_qp_ipm(DevBuf<T> d, int only_active, int max_iter, T eps_abs, T eps_rel,
                                               T eta, T floor_s, T floor_l, T polish_eps, int *split) {
    static_assert(MODE != 1 || NTT <= 128, "the head launch runs one or two waves per problem");
    static_assert(MODE != 2 || NTT > 64, "the tail launch runs two or four waves per problem");
    extern __shared__ __attribute__((aligned(16))) unsigned char dsmem[];
    int b = blockIdx.x;
    if constexpr (MODE == 2) {
        if (b >= __builtin_amdgcn_readfirstlane(split[1])) return;
        b = __builtin_amdgcn_readfirstlane(split[2 + b]);
    } else {
        if (b >= d.B) return;
        if (only_active && !d.scp[b].active) return;
    }
    __shared__ T red[8 * (NTT / 64)];
    __shared__ T sh[NTT >= 256 ? 4 * PT_SCRATCH : 2 * TW_SCRATCH];
    __shared__ T sbv_s[NTT >= 256 ? 6 * 9 : 1];
    __shared__ T wts[18 + 2 * NU];
    __shared__ uint8_t cms[KPC];
    const int tid = threadIdx.x, N = d.N, NB = N + 2;
    Ctx<T, ROBOT> C{};
    ctx_setup<T, ROBOT, NTT>(d, b, C, (LdsT<T> *)wts, (LdsT<uint8_t> *)cms, floor_s, floor_l);
    __syncthreads();
    // dynamic LDS: the (N+2) x 9 Schur vector, then two block rings per wave for the sweeps
    C.vb = (LdsT<T> *)reinterpret_cast<T *>(dsmem);
    // rings: one per half-wave of wave 0 (two-ended sweeps), one per wave (four-wave chains)
    constexpr int NRING = NTT >= 256 ? 4 : 2;
    const int vec = (NB * 9 + 7) & ~7;
    IpmLds<T> L;
    L.ring = C.vb + vec + (NTT >= 256 ? (tid >> 6) : ((tid & 63) >> 5)) * SWEEP_LDS;
    // recurrence scratch: the two ends' (two-ended kernels), this wave's (four chains; pt_reduced
    // runs on wave 0, whose block is the first)
    L.shl = (LdsT<T> *)sh + (NTT >= 256 ? (tid >> 6) * PT_SCRATCH : 0);
    L.red = red;
    if (NTT > 64) C.wxs = C.vb + vec + NRING * SWEEP_LDS;
    if (NTT >= 256) {
        C.Sh = C.ws + Ws<ROBOT>::Sh;
        C.Sx = C.ws + Ws<ROBOT>::Sx;
        pt_seps<T>(NB, C.sp);
        C.sbv = (LdsT<T> *)sbv_s;
        C.hy = C.wxs + vec;
        C.bus = C.hy + vec;
    }
    IpmState<T> S = ipm_state0<T>();
    if constexpr (MODE == 2) {   // resumed after the head launch's stopping test of iteration S.it
        S = reinterpret_cast<const IpmState<T> *>(d.qp_state)[b];
        S.yielded = 0;
        const int it0 = S.it;
        ipm_loop<T, ROBOT, NTT, NTT>(d, C, b, S, L, max_iter, eps_abs, eps_rel, eta, polish_eps);
        S.tail = S.it - it0;
        ipm_finish<T, ROBOT, NTT>(d, C, b, S);
        return;
    }
    ipm_start<T, ROBOT, NTT, NTT>(d, C, b);
    const int yield_at = MODE == 1 ? __builtin_amdgcn_readfirstlane(split[0]) : 0;
    ipm_loop<T, ROBOT, NTT, NTT>(d, C, b, S, L, max_iter, eps_abs, eps_rel, eta, polish_eps, nullptr, 0, yield_at);
    if (MODE == 1 && S.yielded) {
        if (tid == 0) {
            reinterpret_cast<IpmState<T> *>(d.qp_state)[b] = S;
            split[2 + atomicAdd(split + 1, 1)] = b;
        }
    } else {
        ipm_finish<T, ROBOT, NTT>(d, C, b, S);
    }
    // Covariance scans of a deterministic batch (cmpc_api.cpp launch_phase): a workgroup whose QP
    // has finished takes scan jobs from the counter until none is left, so the scans fill the
    // SIMDs of problems that converged early.  Every workgroup leaves after one failed take.  Only
    // the one-wave kernel has the loop (two-wave batches run the scan on a side stream, and the
    // loop's code costs the two-wave kernel registers).
    if constexpr (NTT == 64) if (d.scan_ctr) {
        __shared__ int job;
        __syncthreads();   // the dynamic LDS is free from here on
        LdsT<T> *scan_lds = (LdsT<T> *)reinterpret_cast<T *>(dsmem);
        for (;;) {
            if (tid == 0) job = (int)atomicAdd(d.scan_ctr, 1u);
            __syncthreads();
            const int j = job;
            __syncthreads();
            if (j >= d.B) break;
            if (only_active && !d.scp[j].active) continue;
            if (tid < 64) cov_scan_problem<T, ROBOT>(d, j, scan_lds);
        }
    }
}

// Yield iteration of a split launch (MODE 1): the smallest K >= 2 such that at most `cap`
// problems took more than K Newton-loop iterations in the previous QP launch (so the tail launch
// runs in one round, a problem per CU); for a batch never solved (its counts are cleared by the
// upload) the prior k_fresh; 0 (no split) when no such K exists.  split[1] (the tail count) reset.
// One workgroup of 1024 threads.
template <typename T> __global__ void __launch_bounds__(1024) k_qp_split(DevBuf<T> d, int only_active, int cap, int k_fresh, int *split) {
    __shared__ int hist[64];
    if (threadIdx.x < 64) hist[threadIdx.x] = 0;
    __syncthreads();
    for (int b = threadIdx.x; b < d.B; b += 1024) {
        const int it = (only_active && !d.scp[b].active) ? 0 : d.qp_iters[b];
        atomicAdd(&hist[it < 0 ? 0 : (it > 63 ? 63 : it)], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int K = 0, above = 0, any = 0;
        for (int k = 63; k >= 1; --k) any += hist[k];
        if (any == 0) K = k_fresh;   // a batch never solved: the robot's prior (cmpc_api.cpp qp_split_prior)
        else
            for (int k = 63; k >= 2; --k) {   // above = #(iterations > k - 1) as k decreases
                if (above + hist[k] > cap) { K = k; break; }
                above += hist[k];
            }
        // K: the largest count whose inclusion would exceed the cap, so #(iterations > K) <= cap
        split[0] = K;
        split[1] = 0;
    }
}

// ------------------------------------------------------------------ grouped problems
// Batches of one wave per problem (the metric config: 1024 problems, one per SIMD) last as long as
// their slowest problem: trot N=100 x 1024 takes 4 to 7 Newton steps per problem, so the SIMD of a
// 4-step problem idles for three steps.  k_qp_group holds P problems per P-wave workgroup, one per
// wave (the one-wave algorithm, ipm_loop<.., 64, 64 P>); once all but one have stopped, the last
// one is handed over (group_handover: right after the stopping test of the iteration in which the
// slowest other problem stopped, so the hand-over point depends on Newton-step counts, never on
// timing) and all P waves finish it from there: with the two-wave algorithm (P = 2: one knot per
// thread, one end of the Schur recurrence per wave) or the four-wave one (P = 4: four chains
// around three separators, schur_pt.hpp).  k_qp_order puts the problems that took the most Newton
// steps in the previous launch with those that took the fewest (inactive problems count zero).
//
// LDS of one wave's problem (elements of T): Schur vector | two sweep rings (the two halves of
// the wave) | recurrence scratch of the two ends | reductions | cost weights | contact masks.  When
// all waves finish the last problem, it keeps its region; the other regions hold the w_x side
// array and (P = 4) the fill products in their Schur-vector slots, and each wave uses its own
// region's first ring and recurrence scratch.
template <typename T> struct GroupLds {
    static constexpr int RING = 2 * SWEEP_LDS, SH = 2 * TW_SCRATCH, RED = 32, WTS = 48;
    static constexpr int CMS = (KPC + 8 * (int)sizeof(T) - 1) / (8 * (int)sizeof(T)) * 8;
    static_assert(SH >= PT_SCRATCH, "a region holds a four-chain wave's recurrence scratch");
    __host__ __device__ static constexpr int vec(int N) { return ((N + 2) * 9 + 7) & ~7; }
    __host__ __device__ static constexpr int region(int N) { return vec(N) + RING + SH + RED + WTS + CMS; }
};

// P problems per P-wave workgroup (P = 2 or 4), one per wave until the hand-over.
template <typename T, int ROBOT, int P>
__global__ void __launch_bounds__(64 * P, 1) k_qp_group(DevBuf<T> d, const int *order, int only_active, int share,
                                                        int max_iter, T eps_abs, T eps_rel, T eta, T floor_s,
                                                        T floor_l, T polish_eps) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dsmem[];
    using GL = GroupLds<T>;
    constexpr int WG = 64 * P;
    static_assert(P == 2 || P == 4, "two or four waves per workgroup");
    __shared__ int rem, gflags[8];   // gflags: cont[4] | done[4] (group_handover)
    __shared__ IpmState<T> Ss;
    __shared__ T sbv_s[P == 4 ? 6 * 9 : 1];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, N = d.N, NB = N + 2;
    const int RG = GL::region(N);
    LdsT<T> *base = (LdsT<T> *)reinterpret_cast<T *>(dsmem);
    auto region = [&](int v) { return base + (size_t)v * RG; };
    auto after_vec = [&](LdsT<T> *R) { return R + GL::vec(N); };
    auto wts_of = [&](LdsT<T> *R) { return after_vec(R) + GL::RING + GL::SH + GL::RED; };
    auto cms_of = [&](LdsT<T> *R) { return (LdsT<uint8_t> *)(after_vec(R) + GL::RING + GL::SH + GL::RED + GL::WTS); };
    LdsT<int> *gf = (LdsT<int> *)gflags;
    if (threadIdx.x == 0) rem = -1;
    if (threadIdx.x < 8) gflags[threadIdx.x] = threadIdx.x < 4 ? -1 : 0;
    __syncthreads();
    // one problem per wave.  The problem index is the same on every lane of the wave: as a uniform
    // (scalar) value, every pointer derived from it stays in SGPRs (as a per-lane value the one-wave
    // mode spilled 888 B per lane and ran 11% slower than k_qp_ipm<.., 64>)
    const int slot = P * blockIdx.x + w;
    const int b = __builtin_amdgcn_readfirstlane(slot < d.B ? order[slot] : -1);
    if (b >= 0 && (!only_active || d.scp[b].active)) {
        LdsT<T> *R = region(w);
        Ctx<T, ROBOT> C{};
        ctx_setup<T, ROBOT, 64>(d, b, C, wts_of(R), cms_of(R), floor_s, floor_l);
        gsync<64, WG>();
        C.vb = R;
        IpmLds<T> L;
        L.ring = after_vec(R) + (lane >> 5) * SWEEP_LDS;   // the two ends' sweeps: halves of the wave
        L.shl = after_vec(R) + GL::RING;
        L.red = (T *)(after_vec(R) + GL::RING + GL::SH);
        IpmState<T> S = ipm_state0<T>();
        ipm_start<T, ROBOT, 64, WG>(d, C, b);
        ipm_loop<T, ROBOT, 64, WG>(d, C, b, S, L, max_iter, eps_abs, eps_rel, eta, polish_eps, share ? gf : nullptr, P);
        if (S.yielded) {
            if (lane == 0) {
                Ss = S;
                rem = w;
            }
        } else {
            group_done(gf, w);                   // stopped: the last problem may be handed over
            ipm_finish<T, ROBOT, 64>(d, C, b, S);   // while this wave writes the outputs (global memory only)
        }
    } else {
        group_done(gf, w);
    }
    __syncthreads();   // the first s_barrier of any wave since the start
    // the last problem, if it was handed over, on all waves
    const int r = rem;
    if (r >= 0) {
        const int b2 = __builtin_amdgcn_readfirstlane(order[P * blockIdx.x + r]);
        LdsT<T> *R = region(r);
        Ctx<T, ROBOT> C{};
        ctx_setup<T, ROBOT, WG>(d, b2, C, wts_of(R), cms_of(R), floor_s, floor_l);   // (the same values)
        __syncthreads();
        C.vb = R;
        IpmLds<T> L;
        const int wv = threadIdx.x >> 6;
        if constexpr (P == 4) {   // four waves: four chains, split knots; the other regions' Schur-vector
                                  // slots, each wave its own region's ring and scratch
            C.Sh = C.ws + Ws<ROBOT>::Sh;
            C.Sx = C.ws + Ws<ROBOT>::Sx;
            pt_seps<T>(NB, C.sp);
            C.sbv = (LdsT<T> *)sbv_s;
            C.wxs = region((r + 1) % P);
            C.hy = region((r + 2) % P);
            C.bus = region((r + 3) % P);
            L.ring = after_vec(region(wv));
            L.shl = after_vec(region(wv)) + GL::RING;
        } else {   // two waves: the ends' sweeps on the halves of wave 0
            C.wxs = region(1 - r);
            L.ring = after_vec(R) + (lane >> 5) * SWEEP_LDS;
            L.shl = after_vec(R) + GL::RING;
        }
        L.red = (T *)(after_vec(R) + GL::RING + GL::SH);
        IpmState<T> S = Ss;
        S.yielded = 0;
        const int it0 = S.it;
#ifdef CMPC_STAMPS
        const unsigned long long tb0 = __builtin_amdgcn_s_memtime();
#endif
        ipm_loop<T, ROBOT, WG, WG>(d, C, b2, S, L, max_iter, eps_abs, eps_rel, eta, polish_eps);
        S.tail = S.it - it0;
        ipm_finish<T, ROBOT, WG>(d, C, b2, S);
#ifdef CMPC_STAMPS
        if (threadIdx.x == 0) {   // slots 9, 10: cycles and Newton steps on all waves
            d.stamps[(size_t)b2 * 16 + 9] = __builtin_amdgcn_s_memtime() - tb0;
            d.stamps[(size_t)b2 * 16 + 10] = (unsigned long long)(S.it - it0);
        }
#endif
    }
    // covariance scan jobs of a deterministic batch, each wave on its own (as in k_qp_ipm<.., 64>)
    if (d.scan_ctr) {
        __syncthreads();   // the dynamic LDS is free from here on
        LdsT<T> *R = base + (size_t)(threadIdx.x >> 6) * (RG / 8 * 8);   // a slice per wave
        for (;;) {
            int j = 0;
            if (lane == 0) j = (int)atomicAdd(d.scan_ctr, 1u);
            j = __shfl(j, 0, 64);
            if (j >= d.B) break;
            if (only_active && !d.scp[j].active) continue;
            cov_scan_problem<T, ROBOT>(d, j, R);
        }
    }
}

// Group order of k_qp_group: problems sorted by the Newton steps of their previous QP (stable
// counting sort over ORD_KEYS buckets; inactive problems count zero).  With ng = ceil(B / P)
// groups, slot P g holds the g-th slowest problem and slots P g + 1 .. P g + P - 1 the fastest
// remaining ones in order (-1 once they run out).  One workgroup of 1024 threads, B <= ORD_MAXB;
// deterministic (ranks inside a bucket by index).
constexpr int ORD_KEYS = 16, ORD_MAXB = 8192;
template <typename T> __global__ void __launch_bounds__(1024) k_qp_order(DevBuf<T> d, int only_active, int P, int *order) {
    __shared__ int cnt[ORD_KEYS][ORD_MAXB / 64], start[ORD_KEYS], sorted[ORD_MAXB];
    const int B = d.B, nch = (B + 63) / 64, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    auto key = [&](int bb) -> int {
        if (bb >= B) return -1;
        if (only_active && !d.scp[bb].active) return 0;
        const int it = d.qp_iters[bb];
        return it < 0 ? 0 : (it >= ORD_KEYS ? ORD_KEYS - 1 : it);
    };
    for (int c = wv; c < nch; c += 16) {
        const int k0 = key(64 * c + lane);
        for (int k = 0; k < ORD_KEYS; ++k) {
            const unsigned long long m = __ballot(k0 == k);
            if (lane == 0) cnt[k][c] = __popcll(m);
        }
    }
    __syncthreads();
    if (threadIdx.x < ORD_KEYS) {   // offsets of each chunk inside its bucket
        int run = 0;
        for (int c = 0; c < nch; ++c) {
            const int t = cnt[threadIdx.x][c];
            cnt[threadIdx.x][c] = run;
            run += t;
        }
        start[threadIdx.x] = run;
    }
    __syncthreads();
    if (threadIdx.x == 0) {   // bucket starts
        int run = 0;
        for (int k = 0; k < ORD_KEYS; ++k) {
            const int t = start[k];
            start[k] = run;
            run += t;
        }
    }
    __syncthreads();
    for (int c = wv; c < nch; c += 16) {
        const int bb = 64 * c + lane, k0 = key(bb);
        int rank = 0;
        for (int k = 0; k < ORD_KEYS; ++k) {
            const unsigned long long m = __ballot(k0 == k);
            if (k0 == k) rank = __popcll(m & ((1ull << lane) - 1ull));
        }
        if (k0 >= 0) sorted[start[k0] + cnt[k0][c] + rank] = bb;
    }
    __syncthreads();
    const int ng = (B + P - 1) / P, nfast = B - ng;
    for (int t = threadIdx.x; t < ng * P; t += 1024) {
        const int g = t / P, q = t % P;
        if (q == 0) {
            order[t] = sorted[B - 1 - g];
        } else {
            const int f = g * (P - 1) + q - 1;
            order[t] = f < nfast ? sorted[f] : -1;
        }
    }
}

#define INST(T, R)                                                                       \
    template __global__ void k_qp_ipm<T, R, 64, 0>(DevBuf<T>, int, int, T, T, T, T, T, T, int *);     \
    template __global__ void k_qp_ipm<T, R, 128, 0>(DevBuf<T>, int, int, T, T, T, T, T, T, int *);    \
    template __global__ void k_qp_ipm<T, R, 256, 0>(DevBuf<T>, int, int, T, T, T, T, T, T, int *);    \
    template __global__ void k_qp_group<T, R, 2>(DevBuf<T>, const int *, int, int, int, T, T, T, T, T, T); \
    template __global__ void k_qp_group<T, R, 4>(DevBuf<T>, const int *, int, int, int, T, T, T, T, T, T);
INST(double, 0)
INST(double, 1)
INST(float, 0)
INST(float, 1)
#undef INST
// split launches: fp64 only (fp32 batches take two Newton steps, no tail to split off)
template __global__ void k_qp_ipm<double, 0, 64, 1>(DevBuf<double>, int, int, double, double, double, double, double, double, int *);
template __global__ void k_qp_ipm<double, 1, 64, 1>(DevBuf<double>, int, int, double, double, double, double, double, double, int *);
template __global__ void k_qp_ipm<double, 0, 128, 1>(DevBuf<double>, int, int, double, double, double, double, double, double, int *);
template __global__ void k_qp_ipm<double, 1, 128, 1>(DevBuf<double>, int, int, double, double, double, double, double, double, int *);
template __global__ void k_qp_ipm<double, 0, 128, 2>(DevBuf<double>, int, int, double, double, double, double, double, double, int *);
template __global__ void k_qp_ipm<double, 1, 128, 2>(DevBuf<double>, int, int, double, double, double, double, double, double, int *);
template __global__ void k_qp_ipm<double, 0, 256, 2>(DevBuf<double>, int, int, double, double, double, double, double, double, int *);
template __global__ void k_qp_ipm<double, 1, 256, 2>(DevBuf<double>, int, int, double, double, double, double, double, double, int *);
template __global__ void k_qp_split<double>(DevBuf<double>, int, int, int, int *);
template __global__ void k_qp_order<double>(DevBuf<double>, int, int, int *);
template __global__ void k_qp_order<float>(DevBuf<float>, int, int, int *);

// dynamic LDS of k_qp_group with P problems per workgroup
size_t ipm_group_lds_bytes(int N, int prec_bytes, int P) {
    const size_t e = prec_bytes == 8 ? GroupLds<double>::region(N) : GroupLds<float>::region(N);
    return (size_t)P * e * prec_bytes;
}
int ipm_pair_max_batch() { return ORD_MAXB; }

size_t ipm_lds_bytes(int N, int prec_bytes, int nt) {
    const size_t vec = (((size_t)(N + 2) * 9 + 7) & ~size_t(7));
    // vb, the sweep rings (two; one per wave with four waves), the w_x side array, the fill
    // products of the four-wave solves and their split w phases' B w_u side array; at least one
    // covariance scan's buffers (the scan jobs)
    const size_t nring = nt >= 256 ? 4 : 2;
    return std::max<size_t>(vec + nring * SWEEP_LDS + (nt > 64 ? vec : 0) + (nt >= 256 ? 2 * vec : 0), SCAN_LDS) * prec_bytes;
}

size_t ipm_state_bytes(int prec_bytes) { return prec_bytes == 8 ? sizeof(IpmState<double>) : sizeof(IpmState<float>); }

size_t ipm_workspace_elems(int N, int robot) {
    (void)N;
    return robot == 0 ? Ws<0>::total : Ws<1>::total;
}

}  // namespace cmpc
