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
// Mapping (one 256-thread workgroup per problem, all IPM iterations in one launch):
//   thread k <-> knot k for every per-knot phase (residuals, Phi factors, S blocks, Newton
//   back-substitution, step length); wave 0 runs the O(N) block-Cholesky of S and the two
//   block sweeps per Newton solve with the 9x9 blocks staged in LDS.  Problems are
//   independent, so the grid needs no inter-workgroup communication.
#include "common.hpp"

namespace cmpc {

constexpr int NT = IPM_NT;   // two waves: the two ends of the Schur sweeps; knots k, k + 128, ...
constexpr int FU = 34;   // per-contact factor record: Gw 12 | Kinv 10 | F 6 | Winvd 6
// per-knot (x, t) factor record: 1/Wx[0:6] | M_LL packed 6 | chol(K_TR) packed 36 (diagonal as 1/L_jj) | z1 = L^-1 1 (8) |
// 1/den | D_slack  (K_TR = D_TR^-1 + G_L W_L^-1 G_L', see phase_factor)
constexpr int FX = 64, FX_ML = 6, FX_L = 12, FX_Z1 = 48, FX_DEN = 56, FX_DSL = 57;

// Workspace offsets (elements) for one problem.
struct WsLayout {
    size_t s, l, x, u, t, nu, rdx, rdt, rdu, rde, rdi, facx, facu, Sd, So, wx, wt, wu, rhs, dnu, dx, dt, du,
        ds, dl, dsa, dla, rh, total;
    __host__ __device__ WsLayout(int N, int NI, int NC) {
        const size_t K1 = N + 1, NB = N + 2;
        size_t o = 0;
        auto take = [&](size_t n) { size_t r = o; o += (n + 7) & ~size_t(7); return r; };
        s = take(K1 * NI); l = take(K1 * NI); x = take(K1 * 9); u = take(N * NU); t = take(K1);
        nu = take(NB * 9); rdx = take(K1 * 9); rdt = take(K1); rdu = take(N * NU); rde = take(NB * 9);
        rdi = take(K1 * NI); facx = take(K1 * FX); facu = take((size_t)N * NC * FU); Sd = take(NB * 81);
        So = take((N + 1) * 81); wx = take(K1 * 9); wt = take(K1); wu = take(N * NU); rhs = take(NB * 9);
        dnu = take(NB * 9); dx = take(K1 * 9); dt = take(K1); du = take(N * NU); ds = take(K1 * NI);
        dl = take(K1 * NI); dsa = take(K1 * NI); dla = take(K1 * NI);
        rh = take(K1 * NI);
        total = o;
    }
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

// a / b as a * (1 / b): the IEEE fp64 division is a ~10-instruction sequence; the reciprocal with
// two Newton steps is within an ulp or two, which the interior-point iteration does not notice
template <typename T> __device__ __forceinline__ T fdiv(T a, T b) { return a * rcp_nr(b); }

template <typename T> __device__ __forceinline__ T tr_sign(int j, int i) { return ((j >> i) & 1) ? T(-1) : T(1); }

// ------------------------------------------------------------------ compact A, B operators
// A = [[I, beta I, 0], [0, I, 0], [[w]x, 0, I]] in (c, l, L) blocks.
template <typename T> __device__ __forceinline__ void opA(const T *w, T beta, const T *x, T *o) {
    for (int i = 0; i < 3; ++i) o[i] = x[i] + beta * x[3 + i];
    for (int i = 0; i < 3; ++i) o[3 + i] = x[3 + i];
    T wc[3];
    cross3(w, x, wc);
    for (int i = 0; i < 3; ++i) o[6 + i] = x[6 + i] + wc[i];
}
template <typename T> __device__ __forceinline__ void opAT(const T *w, T beta, const T *v, T *o) {
    T vw[3];
    cross3(v + 6, w, vw);   // [w]x' v_L = v_L x w
    for (int i = 0; i < 3; ++i) o[i] = v[i] + vw[i];
    for (int i = 0; i < 3; ++i) o[3 + i] = beta * v[i] + v[3 + i];
    for (int i = 0; i < 3; ++i) o[6 + i] = v[6 + i];
}
template <typename T, int ROBOT> __device__ __forceinline__ void opB(const T *st, const T *u, T *o) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    using S = Stage<ROBOT>;
    for (int i = 0; i < 9; ++i) o[i] = T(0);
    for (int c = 0; c < NC; ++c) {
        const T *cs = st + S::CON + S::CS * c;
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
template <typename T, int ROBOT> __device__ __forceinline__ void opBT(const T *st, const T *v, T *o) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    using S = Stage<ROBOT>;
    for (int c = 0; c < NC; ++c) {
        const T *cs = st + S::CON + S::CS * c;
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

// ------------------------------------------------------------------ per-problem context
template <typename T, int ROBOT> struct Ctx {
    static constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    static constexpr int NI = Rows<ROBOT>::NI;
    using R_ = Rows<ROBOT>;
    using S = Stage<ROBOT>;
    int N;
    const DevParams<T> *prm;
    const T *stage;       // (N+1, SIZE)
    const uint8_t *logic; // (N, NC)
    const T *xbar;        // (N+1, 9)
    T cw, beta;
    T *ws;
    WsLayout L;
    T *Sd, *So;           // Schur blocks: LDS-resident when they fit (SL), else workspace
    T dcap;               // cap on D = lambda/s for the CoP rows (D-form, folded into W_cop)
    __device__ T Dform(T l, T s_) const { return fmin(fdiv(l, s_), dcap); }

    __device__ const T *st(int k) const { return stage + (size_t)k * S::SIZE; }
    // contact-active bits of knot k, loaded once per phase (0 at k = N: only the TR rows exist)
    __device__ unsigned cmask(int k) const {
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
    // g'z - h of row `row` at knot k for the knot-local (x, t, u)
    __device__ T gz(int k, int row, const T *x, T t, const T *u, bool with_h) const {
        if (row < 8) {
            T v = tr_sign<T>(row, 0) * x[6] + tr_sign<T>(row, 1) * x[7] + tr_sign<T>(row, 2) * x[8] + cw * t;
            return with_h ? v - st(k)[S::BTR + row] : v;
        }
        if (row == 8) return -t;
        if (row < R_::CP) {
            const int c = (row - R_::FR) / 4, r = (row - R_::FR) % 4;
            const T *cs = st(k) + S::CON + S::CS * c;
            const T *f = u + NUPC * c + FO;
            T v = cs[S::G + 3 * r] * f[0] + cs[S::G + 3 * r + 1] * f[1] + cs[S::G + 3 * r + 2] * f[2];
            return with_h ? v - cs[S::H + r] : v;
        }
        const int c = (row - R_::CP) / 4, dd = ((row - R_::CP) % 4) / 2, side = (row - R_::CP) % 2;
        const T cop = u[NUPC * c + dd];
        if (side == 0) {   // cop <= hi
            return with_h ? cop - prm->foot_range[dd == 0 ? 0 : 2] : cop;
        } else {           // -cop <= -lo, lo = -(lxn | lyn)
            return with_h ? -cop - prm->foot_range[dd == 0 ? 1 : 3] : -cop;
        }
    }
    // accumulate G' v of knot k into (gx (L part), gt, gu)
    __device__ void gtv(int k, const T *v, T *gL, T &gt, T *gu) const {
        gL[0] = gL[1] = gL[2] = T(0);
        gt = T(0);
        for (int j = 0; j < 8; ++j) {
            for (int i = 0; i < 3; ++i) gL[i] += tr_sign<T>(j, i) * v[j];
            gt += cw * v[j];
        }
        gt -= v[8];
        if (k >= N) return;
        for (int i = 0; i < NU; ++i) gu[i] = T(0);
        for (int c = 0; c < NC; ++c) {   // rows of inactive contacts carry v = 0 and G = 0
            const T *cs = st(k) + S::CON + S::CS * c;
            for (int r = 0; r < 4; ++r) {
                const T vr = v[R_::FR + 4 * c + r];
                for (int q = 0; q < 3; ++q) gu[NUPC * c + FO + q] += cs[S::G + 3 * r + q] * vr;
            }
            if (ROBOT == 1) {
                for (int dd = 0; dd < 2; ++dd)
                    gu[NUPC * c + dd] += v[R_::CP + 4 * c + 2 * dd] - v[R_::CP + 4 * c + 2 * dd + 1];
            }
        }
    }
    __device__ T *var_x(int k) const { return ws + L.x + (size_t)k * 9; }
    __device__ T *var_u(int k) const { return ws + L.u + (size_t)k * NU; }
};

// 3x3 symmetric packed (00,10,11,20,21,22) helpers
template <typename T> __device__ __forceinline__ T sym3(const T *p, int i, int j) {
    if (i < j) { int t = i; i = j; j = t; }
    return p[i * (i + 1) / 2 + j];
}
template <typename T> __device__ void inv3sym(const T (&a)[3][3], T *out) {
    const T c00 = a[1][1] * a[2][2] - a[1][2] * a[2][1];
    const T c01 = a[1][2] * a[2][0] - a[1][0] * a[2][2];
    const T c02 = a[1][0] * a[2][1] - a[1][1] * a[2][0];
    const T det = a[0][0] * c00 + a[0][1] * c01 + a[0][2] * c02;
    const T id = T(1) / det;
    const T c11 = a[0][0] * a[2][2] - a[0][2] * a[2][0];
    const T c12 = a[0][2] * a[1][0] - a[0][0] * a[1][2];
    const T c22 = a[0][0] * a[1][1] - a[0][1] * a[1][0];
    out[0] = c00 * id; out[1] = c01 * id; out[2] = c11 * id;
    out[3] = c02 * id; out[4] = c12 * id; out[5] = c22 * id;
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

// relative floor on D^-1 in the push-through blocks (K = D^-1 + G W^-1 G')
template <typename T> constexpr double KFLOOR = sizeof(T) == 8 ? 1e-12 : 1e-6;

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

// ------------------------------------------------------------------ phases
// (1) residuals of knot k; returns norm contributions
template <typename T, int ROBOT> struct Norms { T prim, dual, comp, mu, sp, sd, lmax, cnt; };

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

template <typename T, int ROBOT> __device__ void phase_residual(const Ctx<T, ROBOT> &C, int k, Norms<T, ROBOT> &nm) {
    using S = Stage<ROBOT>;
    constexpr int NI = Rows<ROBOT>::NI;
    const int N = C.N;
    const bool hu = k < N;
    const DevParams<T> &P = *C.prm;
    const T *nu = C.ws + C.L.nu;
    const T *st = C.st(k);
    T x[9], u[NU], sv[NI], lm[NI];
    ldv(C.var_x(k), x);
    ldv(C.var_u(hu ? k : 0), u);   // k = N: no controls (values unused)
    ldv(C.ws + C.L.s + (size_t)k * NI, sv);
    ldv(C.ws + C.L.l + (size_t)k * NI, lm);
    const T t = C.ws[C.L.t + k];
    const unsigned msk = C.cmask(k);
    T lv[NI];
#pragma unroll
    for (int r = 0; r < NI; ++r) lv[r] = Ctx<T, ROBOT>::present_m(msk, r) ? lm[r] : T(0);
    T gL[3], gt, gu[NU];
    C.gtv(k, lv, gL, gt, gu);
    // E' nu at knot k
    T ex[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, eu[NU];
    if (k == 0) for (int i = 0; i < 9; ++i) ex[i] += nu[i];
    if (hu) {
        T a[9];
        opAT(st + S::W, C.beta, nu + (size_t)(1 + k) * 9, a);
        for (int i = 0; i < 9; ++i) ex[i] += a[i];
        opBT<T, ROBOT>(st, nu + (size_t)(1 + k) * 9, eu);
    }
    if (k >= 1) for (int i = 0; i < 9; ++i) ex[i] -= nu[(size_t)k * 9 + i];
    if (k == N) for (int i = 0; i < 9; ++i) ex[i] += nu[(size_t)(N + 1) * 9 + i];
    T rdx[9];
    for (int i = 0; i < 9; ++i) {
        const T hx = P.Wx[i] * x[i], q = st[S::QX + i];
        const T g = (i >= 6) ? gL[i - 6] : T(0);
        rdx[i] = hx + q + ex[i] + g;
        nm.dual = fmax(nm.dual, fabs(rdx[i]));
        nm.sd = fmax(nm.sd, fmax(fabs(hx), fmax(fabs(q), fmax(fabs(ex[i]), fabs(g)))));
    }
    const T rdt = T(1) + gt;
    nm.dual = fmax(nm.dual, fabs(rdt));
    nm.sd = fmax(nm.sd, T(1));
    T rdu[NU], rde[9], rdb[9];
    if (hu) {
        for (int i = 0; i < NU; ++i) {
            const T h = P.Wu[i] * u[i];
            rdu[i] = h + eu[i] + gu[i];
            nm.dual = fmax(nm.dual, fabs(rdu[i]));
            nm.sd = fmax(nm.sd, fmax(fabs(h), fmax(fabs(eu[i]), fabs(gu[i]))));
        }
        // dynamics row block 1+k
        T ax[9], bu[9], x1[9];
        ldv(C.var_x(k + 1), x1);
        opA(st + S::W, C.beta, x, ax);
        opB<T, ROBOT>(st, u, bu);
        for (int i = 0; i < 9; ++i) {
            const T ez = ax[i] + bu[i] - x1[i], r = st[S::R + i];
            rde[i] = ez - r;
            nm.prim = fmax(nm.prim, fabs(rde[i]));
            nm.sp = fmax(nm.sp, fmax(fabs(ez), fabs(r)));
        }
    }
    const bool bnd = (k == 0 || k == N);
    if (bnd) {
        const T *xb = C.xbar + (size_t)k * 9;
        for (int i = 0; i < 9; ++i) {
            rdb[i] = x[i] - xb[i];
            nm.prim = fmax(nm.prim, fabs(rdb[i]));
            nm.sp = fmax(nm.sp, fmax(fabs(x[i]), fabs(xb[i])));
        }
    }
    T rdi[NI];
#pragma unroll
    for (int r = 0; r < NI; ++r) {
        const bool pr = Ctx<T, ROBOT>::present_m(msk, r);
        const T g = C.gz(k, r, x, t, u, false);
        const T v = C.gz(k, r, x, t, u, true);
        rdi[r] = pr ? v + sv[r] : T(0);
        const T c = pr ? sv[r] * lm[r] : T(0);
        nm.prim = fmax(nm.prim, pr ? v : T(0));
        nm.sp = fmax(nm.sp, pr ? fmax(fabs(g), fabs(g - v)) : T(0));
        nm.comp = fmax(nm.comp, c);
        nm.mu += c;
        nm.cnt += pr ? T(1) : T(0);
        nm.lmax = fmax(nm.lmax, pr ? lm[r] : T(0));
    }
    // stores
    stv(C.ws + C.L.rdx + (size_t)k * 9, rdx);
    C.ws[C.L.rdt + k] = rdt;
    if (hu) {
        stv(C.ws + C.L.rdu + (size_t)k * NU, rdu);
        stv(C.ws + C.L.rde + (size_t)(1 + k) * 9, rde);
    }
    if (bnd) stv(C.ws + C.L.rde + (size_t)(k == 0 ? 0 : N + 1) * 9, rdb);
    stv(C.ws + C.L.rdi + (size_t)k * NI, rdi);
}

// (2) Phi factors of knot k
template <typename T, int ROBOT> __device__ void phase_factor(const Ctx<T, ROBOT> &C, int k) {
    using S = Stage<ROBOT>;
    using R_ = Rows<ROBOT>;
    constexpr int NI = R_::NI, NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    const int N = C.N;
    const DevParams<T> &P = *C.prm;
    const T *s = C.ws + C.L.s + (size_t)k * NI, *lm = C.ws + C.L.l + (size_t)k * NI;
    T *fx = C.ws + C.L.facx + (size_t)k * FX;
    // (L, t) block in push-through form (no D * r product, no cancellation as rows pin L or t):
    //   K = D_TR^-1 + Y G_L' (8x8 SPD; Y = G_L W_L^-1; D^-1 floored: at a vertex of the trust
    //   region more than 3 rows are active and K -> rank 3),  L L' = K,  z1 = L^-1 1,
    //   den = D_slack + cw^2 |z1|^2,  Z = L^-1 Y,  g = Z' z1,
    //   M_LL = [Phi^-1]_LL = W_L^-1 - Z'Z + cw^2 g g' / den
    const T wl[3] = {T(1) / P.Wx[6], T(1) / P.Wx[7], T(1) / P.Wx[8]};
    const T kfl = T(KFLOOR<T>) * T(8) * (wl[0] + wl[1] + wl[2]);
    T Lk[36];
    for (int j = 0; j < 8; ++j)
        for (int q = 0; q <= j; ++q) {
            T v = T(0);
            for (int i = 0; i < 3; ++i) v += tr_sign<T>(j, i) * tr_sign<T>(q, i) * wl[i];
            if (q == j) v += fmax(fdiv(s[j], lm[j]), kfl);
            Lk[j * (j + 1) / 2 + q] = v;
        }
    chol8(Lk);
    T z1[8], Z[8][3];
    for (int j = 0; j < 8; ++j) {
        T a1 = T(1), az[3];
        for (int i = 0; i < 3; ++i) az[i] = tr_sign<T>(j, i) * wl[i];
        for (int q = 0; q < j; ++q) {
            const T l = Lk[j * (j + 1) / 2 + q];
            a1 -= l * z1[q];
            for (int i = 0; i < 3; ++i) az[i] -= l * Z[q][i];
        }
        const T il = Lk[j * (j + 1) / 2 + j];
        z1[j] = a1 * il;
        for (int i = 0; i < 3; ++i) Z[j][i] = az[i] * il;
    }
    T kap = T(0), g[3] = {0, 0, 0};
    for (int j = 0; j < 8; ++j) {
        kap += z1[j] * z1[j];
        for (int i = 0; i < 3; ++i) g[i] += Z[j][i] * z1[j];
    }
    const T dsl = fdiv(lm[8], s[8]);
    const T iden = rcp_nr(dsl + C.cw * C.cw * kap);
    for (int i = 0; i < 6; ++i) fx[i] = T(1) / P.Wx[i];
    for (int i = 0, p = 0; i < 3; ++i)
        for (int q = 0; q <= i; ++q, ++p) {
            T zz = T(0);
            for (int j = 0; j < 8; ++j) zz += Z[j][i] * Z[j][q];
            fx[FX_ML + p] = (i == q ? wl[i] : T(0)) - zz + C.cw * C.cw * g[i] * g[q] * iden;
        }
    for (int e = 0; e < 36; ++e) fx[FX_L + e] = Lk[e];
    for (int j = 0; j < 8; ++j) fx[FX_Z1 + j] = z1[j];
    fx[FX_DEN] = iden;
    fx[FX_DSL] = dsl;
    if (k >= N) return;
    for (int c = 0; c < NC; ++c) {
        T *fu = C.ws + C.L.facu + ((size_t)k * NC + c) * FU;
        const T *Wc = P.Wu + NUPC * c;
        // Winvd: inverse diagonal of W' (CoP rows fold into their coordinate's diagonal)
        for (int q = 0; q < NUPC; ++q) fu[28 + q] = T(1) / Wc[q];
        if (ROBOT == 1 && C.logic[k * NC + c]) {
            for (int dd = 0; dd < 2; ++dd) {
                const int r0 = R_::CP + 4 * c + 2 * dd;
                fu[28 + dd] = T(1) / (Wc[dd] + C.Dform(lm[r0], s[r0]) + C.Dform(lm[r0 + 1], s[r0 + 1]));
            }
        }
        const T wi[3] = {T(1) / Wc[FO], T(1) / Wc[FO + 1], T(1) / Wc[FO + 2]};
        if (!C.logic[k * NC + c]) {
            for (int q = 0; q < 12; ++q) fu[q] = T(0);
            for (int q = 0; q < 10; ++q) fu[12 + q] = T(0);
            fu[12 + 0] = fu[12 + 2] = fu[12 + 5] = fu[12 + 9] = T(1);
            fu[22] = wi[0]; fu[23] = T(0); fu[24] = wi[1]; fu[25] = T(0); fu[26] = T(0); fu[27] = wi[2];
            continue;
        }
        const T *cs = C.st(k) + S::CON + S::CS * c;
        T Gw[4][3];
        for (int r = 0; r < 4; ++r)
            for (int q = 0; q < 3; ++q) { Gw[r][q] = cs[S::G + 3 * r + q] * wi[q]; fu[3 * r + q] = Gw[r][q]; }
        T Km[4][4], tr = T(0);
        for (int r = 0; r < 4; ++r)
            for (int q = 0; q < 4; ++q) {
                T acc = T(0);
                for (int z = 0; z < 3; ++z) acc += Gw[r][z] * cs[S::G + 3 * q + z];
                Km[r][q] = acc;
            }
        for (int r = 0; r < 4; ++r) tr += Km[r][r];
        // floor on D^-1: at a zero force all four pyramid rows are active (K -> rank 3)
        const T kfloor = T(KFLOOR<T>) * tr + T(sizeof(T) == 8 ? 1e-300 : 1e-37);
        for (int r = 0; r < 4; ++r) Km[r][r] += fmax(fdiv(s[R_::FR + 4 * c + r], lm[R_::FR + 4 * c + r]), kfloor);
        T Ki[10];
        inv4spd(Km, Ki);
        for (int q = 0; q < 10; ++q) fu[12 + q] = Ki[q];
        // F = W^-1 - Gw' Kinv Gw
        int p = 0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j <= i; ++j) {
                T acc = (i == j) ? wi[i] : T(0);
                for (int r = 0; r < 4; ++r)
                    for (int q = 0; q < 4; ++q) acc -= Gw[r][i] * Ki[p4(r, q)] * Gw[q][j];
                fu[22 + p++] = acc;
            }
    }
}

// Phi_u^-1 vu for the control blocks of knot k < N (friction rows in push-through form)
template <typename T, int ROBOT> __device__ void phi_solve_u(const Ctx<T, ROBOT> &C, int k, const T *vu, T *ou) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    for (int c = 0; c < NC; ++c) {
        const T *fu = C.ws + C.L.facu + ((size_t)k * NC + c) * FU;
        const T *vc = vu + NUPC * c;
        T *oc = ou + NUPC * c;
        for (int q = 0; q < NUPC; ++q) oc[q] = fu[28 + q] * vc[q];
        for (int i = 0; i < 3; ++i)
            oc[FO + i] = sym3(fu + 22, i, 0) * vc[FO] + sym3(fu + 22, i, 1) * vc[FO + 1] + sym3(fu + 22, i, 2) * vc[FO + 2];
    }
}

// local solve of the (L, t) block of knot k (unknowns dL, dt, dlam_TR[8], dlam_slack):
//   W_L dL + G_L' dlam = vL;  cw 1'dlam - dlam_sl = vt;  G_L dL + cw 1 dt - D^-1 dlam = -rh[0:8];
//   -dt - D_sl^-1 dlam_sl = -rh[8]
// dt = (vt + D_sl rh_8 - cw z1'y) / den with y = L^-1 (Y vL + rh);  dlam = L^-T (y + cw dt z1);
// dL = W_L^-1 (vL - G_L' dlam);  dlam_sl = cw 1'dlam - vt  (the t row of the dual residual)
template <typename T, int ROBOT>
__device__ void tr_local(const Ctx<T, ROBOT> &C, int k, const T *vL, T vt, const T *rh, T *dL, T &dt, T *dlt, T &dls) {
    const T *fx = C.ws + C.L.facx + (size_t)k * FX;
    const T *Lk = fx + FX_L, *z1 = fx + FX_Z1;
    const T wl[3] = {rcp_nr(C.prm->Wx[6]), rcp_nr(C.prm->Wx[7]), rcp_nr(C.prm->Wx[8])};
    T y[8];
    for (int j = 0; j < 8; ++j) {
        T v = rh[j];
        for (int i = 0; i < 3; ++i) v += tr_sign<T>(j, i) * wl[i] * vL[i];
        for (int q = 0; q < j; ++q) v -= Lk[j * (j + 1) / 2 + q] * y[q];
        y[j] = v * Lk[j * (j + 1) / 2 + j];
    }
    T zy = T(0);
    for (int j = 0; j < 8; ++j) zy += z1[j] * y[j];
    dt = (vt + fx[FX_DSL] * rh[8] - C.cw * zy) * fx[FX_DEN];
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
template <typename T, int ROBOT> __device__ void phase_sblock(const Ctx<T, ROBOT> &C, int k) {
    using S = Stage<ROBOT>;
    constexpr int NC = Robot<ROBOT>::NC;
    const int N = C.N;
    const T beta = C.beta;
    const T *fx = C.ws + C.L.facx + (size_t)k * FX;
    auto Mfull = [&](const T *f, int i, int j) -> T {   // M_k entry
        if (i < 6 || j < 6) return (i == j && i < 6) ? f[i] : T(0);
        return sym3(f + 6, i - 6, j - 6);
    };
    // M A' blocks:  [[Mc, 0, Mc W'], [beta Ml, Ml, 0], [0, 0, ML]]
    auto MAt = [&](const T *f, const T *w, int i, int j) -> T {
        const T Wm[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
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
                Sd[i * 9 + j] = Mfull(fx, i, j);
                So[i * 9 + j] = MAt(fx, C.st(0) + S::W, i, j);
            }
    }
    if (k == N) {
        T *Sd = C.Sd + (size_t)(N + 1) * 81;
        for (int i = 0; i < 9; ++i)
            for (int j = 0; j < 9; ++j) Sd[i * 9 + j] = Mfull(fx, i, j);
        return;
    }
    const T *fx1 = fx + FX;
    const T *w = C.st(k) + S::W;
    const T Wm[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    T Sm[9][9];
    // A M A'
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j) Sm[i][j] = T(0);
    const T *mc = fx, *ml = fx + 3;
    for (int a = 0; a < 3; ++a) {
        Sm[a][a] = mc[a] + beta * beta * ml[a];
        Sm[a][3 + a] = Sm[3 + a][a] = beta * ml[a];
        Sm[3 + a][3 + a] = ml[a];
    }
    for (int a = 0; a < 3; ++a)
        for (int bb = 0; bb < 3; ++bb) {
            Sm[a][6 + bb] = mc[a] * Wm[bb][a];   // Mc W'
            Sm[6 + bb][a] = Sm[a][6 + bb];
            T acc = sym3(fx + 6, a, bb);
            for (int q = 0; q < 3; ++q) acc += Wm[a][q] * mc[q] * Wm[bb][q];
            Sm[6 + a][6 + bb] = acc;
        }
    // B Phi_u^-1 B'
    for (int c = 0; c < NC; ++c) {
        const T *cs = C.st(k) + S::CON + S::CS * c;
        const T al = cs[S::ALPHA];
        if (al == T(0)) continue;
        const T *fu = C.ws + C.L.facu + ((size_t)k * NC + c) * FU;
        const T *lv = cs + S::LEVER;
        const T Lm[3][3] = {{0, -lv[2], lv[1]}, {lv[2], 0, -lv[0]}, {-lv[1], lv[0], 0}};
        T F[3][3], FL[3][3];   // F, F Lambda'
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) F[i][j] = sym3(fu + 22, i, j);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) FL[i][j] = F[i][0] * Lm[j][0] + F[i][1] * Lm[j][1] + F[i][2] * Lm[j][2];
        const T a2 = al * al;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                Sm[3 + i][3 + j] += a2 * F[i][j];
                Sm[3 + i][6 + j] += a2 * FL[i][j];
                Sm[6 + j][3 + i] += a2 * FL[i][j];
                T acc = T(0);
                for (int q = 0; q < 3; ++q) acc += Lm[i][q] * FL[q][j];
                Sm[6 + i][6 + j] += a2 * acc;
            }
        if (ROBOT == 1) {
            const T *bc = cs + S::BCOP, *bt = cs + S::BTAU;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j)
                    Sm[6 + i][6 + j] += bc[2 * i] * fu[28] * bc[2 * j] + bc[2 * i + 1] * fu[29] * bc[2 * j + 1] +
                                        bt[i] * fu[33] * bt[j];
        }
    }
    // + M_{k+1}
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j) Sm[i][j] += Mfull(fx1, i, j);
    T *Sd = C.Sd + (size_t)(1 + k) * 81;
    for (int e = 0; e < 81; ++e) Sd[e] = Sm[e / 9][e % 9];
    T *So = C.So + (size_t)(1 + k) * 81;
    if (k + 1 < N) {
        const T *w1 = C.st(k + 1) + S::W;
        for (int i = 0; i < 9; ++i)
            for (int j = 0; j < 9; ++j) So[i * 9 + j] = -MAt(fx1, w1, i, j);
    } else {
        for (int i = 0; i < 9; ++i)
            for (int j = 0; j < 9; ++j) So[i * 9 + j] = -Mfull(fx1, i, j);
    }
}


// (4) two-ended ("twisted") block-Thomas factorization of the SPD block-tridiagonal S with
// explicit symmetric inverses.  Wave 0 eliminates from the top, wave 1 from the bottom, and the
// two meet at block m:
//   top    (j < m):  X_j = S_{j,j-1} I_{j-1},  I_j = (S_jj - X_j S_{j-1,j})^-1      So[j-1] <- X_j
//   bottom (j > m):  Y_j = S_{j,j+1} I_{j+1},  I_j = (S_jj - Y_j S_{j+1,j})^-1      So[j]   <- Y_j
//   meet   (j = m):  I_m = (S_mm - X_m S_{m-1,m} - Y_m S_{m+1,m})^-1
// Sd[j] <- I_j (LDS when it fits: the inverses are re-read by every sweep); So[j] holds
// S_{j,j+1} on input and lives in global memory: each step stages the raw block it needs into
// LDS scratch from registers loaded one step ahead.  Inverses by Gauss-Jordan sweeps over the
// 64 lanes (SPD: no pivoting) with a pivot floor relative to the original diagonal (near the
// solution of a degenerate QP the Schur blocks are differences of O(M) numbers).
template <typename T, typename PS>
__device__ __forceinline__ void tw_step(PS *Sd, const LdsT<T> *Op, const LdsT<T> *Oq, T *OwTop, T *OwBot, int j,
                                        LdsT<T> *A, LdsT<T> *Xb) {
    const int lane = threadIdx.x & 63;
    const int e0 = lane, e1 = lane + 64;
    const bool has1 = e1 < 81;
    const int i0 = e0 / 9, c0 = e0 % 9, i1 = e1 / 9, c1 = e1 % 9;
    PS *Dj = Sd + (size_t)j * 81;
    T a0 = Dj[e0], a1 = has1 ? Dj[e1] : T(0);
    T x0 = T(0), x1 = T(0), y0 = T(0), y1 = T(0);
    if (Op) {   // X = Op' I_{j-1};  A -= X Op   (Op = S_{j-1,j})
        const PS *Ip = Sd + (size_t)(j - 1) * 81;
        for (int m = 0; m < 9; ++m) {
            x0 = fma(Op[m * 9 + i0], Ip[m * 9 + c0], x0);
            if (has1) x1 = fma(Op[m * 9 + i1], Ip[m * 9 + c1], x1);
        }
        Xb[e0] = x0;
        if (has1) Xb[e1] = x1;
        wave_sync();
        for (int m = 0; m < 9; ++m) {
            a0 = fma(-Xb[i0 * 9 + m], Op[m * 9 + c0], a0);
            if (has1) a1 = fma(-Xb[i1 * 9 + m], Op[m * 9 + c1], a1);
        }
        wave_sync();
    }
    if (Oq) {   // Y = Oq I_{j+1};  A -= Y Oq'   (Oq = S_{j,j+1})
        const PS *Iq = Sd + (size_t)(j + 1) * 81;
        for (int m = 0; m < 9; ++m) {
            y0 = fma(Oq[i0 * 9 + m], Iq[m * 9 + c0], y0);
            if (has1) y1 = fma(Oq[i1 * 9 + m], Iq[m * 9 + c1], y1);
        }
        Xb[e0] = y0;
        if (has1) Xb[e1] = y1;
        wave_sync();
        for (int m = 0; m < 9; ++m) {
            a0 = fma(-Xb[i0 * 9 + m], Oq[c0 * 9 + m], a0);
            if (has1) a1 = fma(-Xb[i1 * 9 + m], Oq[c1 * 9 + m], a1);
        }
        wave_sync();
    }
    A[e0] = a0;
    if (has1) A[e1] = a1;
    if (Op) { OwTop[e0] = x0; if (has1) OwTop[e1] = x1; }
    if (Oq) { OwBot[e0] = y0; if (has1) OwBot[e1] = y1; }
    wave_sync();
    for (int c = 0; c < 9; ++c) {
        const T p = fmax(A[c * 9 + c], T(1e-13) * Dj[c * 9 + c]);
        const T ip = rcp_nr(p);
        const T aic0 = A[i0 * 9 + c], acj0 = A[c * 9 + c0], aij0 = A[e0];
        T aic1 = T(0), acj1 = T(0), aij1 = T(0);
        if (has1) { aic1 = A[i1 * 9 + c]; acj1 = A[c * 9 + c1]; aij1 = A[e1]; }
        wave_sync();
        auto upd = [&](int i, int cc, T aic, T acj, T aij) -> T {
            if (i != c && cc != c) return fma(-aic * ip, acj, aij);
            if (i == c && cc != c) return acj * ip;
            if (i != c && cc == c) return -aic * ip;
            return ip;
        };
        A[e0] = upd(i0, c0, aic0, acj0, aij0);
        if (has1) A[e1] = upd(i1, c1, aic1, acj1, aij1);
        wave_sync();
    }
    Dj[e0] = A[e0];
    if (has1) Dj[e1] = A[e1];
    wave_sync();
}

// per-wave LDS scratch of the factorization: A | Xb | Ob (96 each)
constexpr int TW_SCRATCH = 288;

// the two ends (threads 0..127: wave 0 top blocks 0..m-1, wave 1 bottom blocks NB-1..m+1)
template <typename T, typename PS> __device__ void tw_factor_ends(PS *Sd, T *So, int NB, int m, LdsT<T> *sh) {
    const int lane = threadIdx.x & 63;
    const int e0 = lane, e1 = lane + 64;
    const bool has1 = e1 < 81;
    const bool top = (threadIdx.x >> 6) == 0;
    LdsT<T> *A = sh + (top ? 0 : TW_SCRATCH), *Xb = A + 96, *Ob = A + 192;
    T p0 = T(0), p1 = T(0);
    auto fetch = [&](int blk) { p0 = So[(size_t)blk * 81 + e0]; p1 = has1 ? So[(size_t)blk * 81 + e1] : T(0); };
    if (top) {
        if (m > 1) fetch(0);
        tw_step<T, PS>(Sd, nullptr, nullptr, nullptr, nullptr, 0, A, Xb);
        for (int j = 1; j < m; ++j) {
            Ob[e0] = p0;
            if (has1) Ob[e1] = p1;
            wave_sync();
            if (j + 1 < m) fetch(j);
            tw_step<T, PS>(Sd, Ob, nullptr, So + (size_t)(j - 1) * 81, nullptr, j, A, Xb);
        }
    } else {
        if (NB - 2 > m) fetch(NB - 2);
        tw_step<T, PS>(Sd, nullptr, nullptr, nullptr, nullptr, NB - 1, A, Xb);
        for (int j = NB - 2; j > m; --j) {
            Ob[e0] = p0;
            if (has1) Ob[e1] = p1;
            wave_sync();
            if (j - 1 > m) fetch(j - 1);
            tw_step<T, PS>(Sd, nullptr, Ob, nullptr, So + (size_t)j * 81, j, A, Xb);
        }
    }
}

// the meeting block (wave 0, after a workgroup barrier)
template <typename T, typename PS> __device__ void tw_factor_meet(PS *Sd, T *So, int m, LdsT<T> *sh) {
    const int lane = threadIdx.x & 63;
    const int e0 = lane, e1 = lane + 64;
    const bool has1 = e1 < 81;
    LdsT<T> *A = sh, *Xb = A + 96, *Op = A + 192, *Oq = sh + TW_SCRATCH + 192;
    Op[e0] = So[(size_t)(m - 1) * 81 + e0];
    Oq[e0] = So[(size_t)m * 81 + e0];
    if (has1) { Op[e1] = So[(size_t)(m - 1) * 81 + e1]; Oq[e1] = So[(size_t)m * 81 + e1]; }
    wave_sync();
    tw_step<T, PS>(Sd, Op, Oq, So + (size_t)(m - 1) * 81, So + (size_t)m * 81, m, A, Xb);
}

// (5c) two-ended block sweeps with the twisted factors: rhs -> dnu (vector staged in LDS vb)
//   top:    y_0 = b_0, y_j = b_j - X_j y_{j-1}           bottom: y_j = b_j - Y_j y_{j+1}
//   meet:   x_m = I_m (b_m - X_m y_{m-1} - Y_m y_{m+1})
//   up:     x_j = I_j y_j - X_{j+1}' x_{j+1}  (j < m)   down: x_j = I_j y_j - Y_{j-1}' x_{j-1}  (j > m)
// X_j sits at So[j-1], Y_j at So[j] (global; lane r < 9 reads its row / column one step ahead).
// Three stages separated by workgroup barriers.
template <typename T> __device__ __forceinline__ void ld_row(const T *p, T (&r)[9]) {
    for (int q = 0; q < 9; ++q) r[q] = p[q];
}
template <typename T> __device__ __forceinline__ void ld_col(const T *p, T (&r)[9]) {
    for (int q = 0; q < 9; ++q) r[q] = p[q * 9];
}

template <typename T> __device__ void tw_solve_elim(const T *Xs, const T *rhs, int NB, int m, LdsT<T> *vb) {
    const int lane = threadIdx.x & 63;
    const bool top = (threadIdx.x >> 6) == 0;
    const int lr = lane < 9 ? lane : 0;
    const int lo = top ? 0 : m + 1, hi = top ? m + 1 : NB;   // rhs blocks staged by this wave
    for (int e = lo * 9 + lane; e < hi * 9; e += WAVE) vb[e] = rhs[e];
    wave_sync();
    T nx[9], cur[9];
    if (top) {
        if (m > 1) ld_row(Xs + lr * 9, nx);                             // X_1 at So[0]
        for (int j = 1; j < m; ++j) {
            for (int q = 0; q < 9; ++q) cur[q] = nx[q];
            if (j + 1 < m) ld_row(Xs + (size_t)j * 81 + lr * 9, nx);     // X_{j+1} at So[j]
            if (lane < 9) {
                const LdsT<T> *yp = vb + (size_t)(j - 1) * 9;
                T v = vb[(size_t)j * 9 + lane];
                for (int q = 0; q < 9; ++q) v = fma(-cur[q], yp[q], v);
                vb[(size_t)j * 9 + lane] = v;
            }
            wave_sync();
        }
    } else {
        if (NB - 2 > m) ld_row(Xs + (size_t)(NB - 2) * 81 + lr * 9, nx);     // Y_{NB-2} at So[NB-2]
        for (int j = NB - 2; j > m; --j) {
            for (int q = 0; q < 9; ++q) cur[q] = nx[q];
            if (j - 1 > m) ld_row(Xs + (size_t)(j - 1) * 81 + lr * 9, nx);
            if (lane < 9) {
                const LdsT<T> *yn = vb + (size_t)(j + 1) * 9;
                T v = vb[(size_t)j * 9 + lane];
                for (int q = 0; q < 9; ++q) v = fma(-cur[q], yn[q], v);
                vb[(size_t)j * 9 + lane] = v;
            }
            wave_sync();
        }
    }
}
template <typename T, typename PS>
__device__ void tw_solve_meet(const PS *Ii, const T *Xs, int NB, int m, LdsT<T> *vb, LdsT<T> *sh) {
    const int lane = threadIdx.x & 63;
    if (lane < 9) {
        T v = vb[(size_t)m * 9 + lane];
        const T *X = Xs + (size_t)(m - 1) * 81 + lane * 9, *Y = Xs + (size_t)m * 81 + lane * 9;
        const LdsT<T> *yp = vb + (size_t)(m - 1) * 9, *yn = vb + (size_t)(m + 1) * 9;
        for (int q = 0; q < 9; ++q) v = fma(-X[q], yp[q], fma(-Y[q], yn[q], v));
        sh[lane] = v;
    }
    wave_sync();
    if (lane < 9) {
        const PS *I = Ii + (size_t)m * 81 + lane * 9;
        T v = T(0);
        for (int q = 0; q < 9; ++q) v = fma(I[q], sh[q], v);
        vb[(size_t)m * 9 + lane] = v;
    }
    wave_sync();
}
template <typename T, typename PS>
__device__ void tw_solve_back(const PS *Ii, const T *Xs, T *dnu, int NB, int m, LdsT<T> *vb) {
    const int lane = threadIdx.x & 63;
    const bool top = (threadIdx.x >> 6) == 0;
    const int lr = lane < 9 ? lane : 0;
    T nx[9], cur[9];
    if (top) {
        if (m >= 1) ld_col(Xs + (size_t)(m - 1) * 81 + lr, nx);         // X_m at So[m-1]
        for (int j = m - 1; j >= 0; --j) {
            for (int q = 0; q < 9; ++q) cur[q] = nx[q];
            if (j >= 1) ld_col(Xs + (size_t)(j - 1) * 81 + lr, nx);     // X_j at So[j-1]
            T v = T(0);
            if (lane < 9) {
                const PS *I = Ii + (size_t)j * 81 + lane * 9;   // symmetric: row == column
                const LdsT<T> *y = vb + (size_t)j * 9;
                for (int q = 0; q < 9; ++q) v = fma(I[q], y[q], v);
                const LdsT<T> *xn = vb + (size_t)(j + 1) * 9;
                for (int q = 0; q < 9; ++q) v = fma(-cur[q], xn[q], v);
            }
            wave_sync();
            if (lane < 9) vb[(size_t)j * 9 + lane] = v;
            wave_sync();
        }
    } else {
        if (m + 1 < NB) ld_col(Xs + (size_t)m * 81 + lr, nx);            // Y_m at So[m]
        for (int j = m + 1; j < NB; ++j) {
            for (int q = 0; q < 9; ++q) cur[q] = nx[q];
            if (j + 1 < NB) ld_col(Xs + (size_t)j * 81 + lr, nx);       // Y_j at So[j]
            T v = T(0);
            if (lane < 9) {
                const PS *I = Ii + (size_t)j * 81 + lane * 9;
                const LdsT<T> *y = vb + (size_t)j * 9;
                for (int q = 0; q < 9; ++q) v = fma(I[q], y[q], v);
                const LdsT<T> *xp = vb + (size_t)(j - 1) * 9;
                for (int q = 0; q < 9; ++q) v = fma(-cur[q], xp[q], v);
            }
            wave_sync();
            if (lane < 9) vb[(size_t)j * 9 + lane] = v;
            wave_sync();
        }
    }
    const int lo = top ? 0 : m, hi = top ? m : NB;
    for (int e = lo * 9 + lane; e < hi * 9; e += WAVE) dnu[e] = vb[e];
}

// r_hat = r_i - r_c / lambda for the rows of knot k  (rc supplied per mode)
template <typename T, int ROBOT>
__device__ void rhat_rows(const Ctx<T, ROBOT> &C, int k, int corr, T sigma_mu, T *rh) {
    constexpr int NI = Rows<ROBOT>::NI;
    const T *s = C.ws + C.L.s + (size_t)k * NI, *lm = C.ws + C.L.l + (size_t)k * NI;
    const T *rdi = C.ws + C.L.rdi + (size_t)k * NI;
    const T *dsa = C.ws + C.L.dsa + (size_t)k * NI, *dla = C.ws + C.L.dla + (size_t)k * NI;
    const unsigned msk = C.cmask(k);
    for (int r = 0; r < NI; ++r) {
        const bool pr = Ctx<T, ROBOT>::present_m(msk, r);
        T rc = s[r] * lm[r];
        if (corr) rc += dsa[r] * dla[r] - sigma_mu;
        const T v = rdi[r] - fdiv(rc, pr ? lm[r] : T(1));
        rh[r] = pr ? v : T(0);
    }
}

// (5a) particular solution w = Phi^-1 (r_d + G' D rhat) (friction rows in push-through form)
template <typename T, int ROBOT> __device__ void phase_w(const Ctx<T, ROBOT> &C, int k, int corr, T sigma_mu) {
    using R_ = Rows<ROBOT>;
    constexpr int NI = R_::NI, NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    const int N = C.N;
    const bool hu = k < N;
    T rh[NI];
    rhat_rows(C, k, corr, sigma_mu, rh);   // kept for phase_dz (stored below)
    T rdx[9], fxd[6], rdu[NU];
    ldv(C.ws + C.L.rdx + (size_t)k * 9, rdx);
    ldv(C.ws + C.L.facx + (size_t)k * FX, fxd);
    if (hu) ldv(C.ws + C.L.rdu + (size_t)k * NU, rdu);
    const T rdt = C.ws[C.L.rdt + k];
    T wx[9], wt;
    for (int i = 0; i < 6; ++i) wx[i] = fxd[i] * rdx[i];
    {   // (L, t): w = -(local solve with v = -r_d)
        const T vL[3] = {-rdx[6], -rdx[7], -rdx[8]};
        T dL[3], dt, dlt[8], dls;
        tr_local(C, k, vL, -rdt, rh, dL, dt, dlt, dls);
        for (int i = 0; i < 3; ++i) wx[6 + i] = -dL[i];
        wt = -dt;
    }
    T ou[NU];
    if (hu) {
        T vu[NU];
        for (int i = 0; i < NU; ++i) vu[i] = rdu[i];
        if (ROBOT == 1) {   // CoP rows (D-form, folded into W_cop); absent rows: lambda = 0 -> D = 0, rhat = 0
            const T *s = C.ws + C.L.s + (size_t)k * NI, *lm = C.ws + C.L.l + (size_t)k * NI;
            for (int c = 0; c < NC; ++c)
                for (int dd = 0; dd < 2; ++dd) {
                    const int r0 = R_::CP + 4 * c + 2 * dd;
                    vu[NUPC * c + dd] += C.Dform(lm[r0], s[r0]) * rh[r0] - C.Dform(lm[r0 + 1], s[r0 + 1]) * rh[r0 + 1];
                }
        }
        phi_solve_u(C, k, vu, ou);
        for (int c = 0; c < NC; ++c) {
            // inactive contacts: Gw = 0, Kinv = I and rhat = 0, so they contribute nothing
            const T *fu = C.ws + C.L.facu + ((size_t)k * NC + c) * FU;
            T g[22];
            ldv(fu, g);
            T kr[4];
            for (int r = 0; r < 4; ++r) {
                T acc = T(0);
                for (int q = 0; q < 4; ++q) acc += g[12 + p4(r, q)] * rh[R_::FR + 4 * c + q];
                kr[r] = acc;
            }
            for (int i = 0; i < 3; ++i) {
                T acc = T(0);
                for (int r = 0; r < 4; ++r) acc += g[3 * r + i] * kr[r];
                ou[NUPC * c + FO + i] += acc;
            }
        }
    }
    // stores
    stv(C.ws + C.L.wx + (size_t)k * 9, wx);
    C.ws[C.L.wt + k] = wt;
    if (hu) stv(C.ws + C.L.wu + (size_t)k * NU, ou);
    stv(C.ws + C.L.rh + (size_t)k * NI, rh);
}


// (5b) Schur right-hand side blocks owned by knot k: rhs = r_e - E w
template <typename T, int ROBOT> __device__ void phase_rhs(const Ctx<T, ROBOT> &C, int k) {
    using S = Stage<ROBOT>;
    const int N = C.N;
    const T *wx = C.ws + C.L.wx + (size_t)k * 9;
    const T *rde = C.ws + C.L.rde;
    T *rhs = C.ws + C.L.rhs;
    if (k == 0) for (int i = 0; i < 9; ++i) rhs[i] = rde[i] - wx[i];
    if (k == N) for (int i = 0; i < 9; ++i) rhs[(size_t)(N + 1) * 9 + i] = rde[(size_t)(N + 1) * 9 + i] - wx[i];
    if (k < N) {
        T ax[9], bu[9];
        opA(C.st(k) + S::W, C.beta, wx, ax);
        opB<T, ROBOT>(C.st(k), C.ws + C.L.wu + (size_t)k * NU, bu);
        const T *wx1 = wx + 9;
        for (int i = 0; i < 9; ++i)
            rhs[(size_t)(1 + k) * 9 + i] = rde[(size_t)(1 + k) * 9 + i] - (ax[i] + bu[i] - wx1[i]);
    }
}

// (5d) direction at knot k from dnu; returns the max step allowed by this knot's rows
// rows of knot k: ds = -r_i - G dz; dlambda from the push-through solves (TR, slack: dlt, dls;
// friction: Kinv (Gw v + rhat) with v = -(rdu + E'dnu_u) on the forces) or the D-form (CoP);
// returns the largest step keeping s, lambda >= 0.  The memory operands are restrict-qualified
// so the loads of s, lambda, r_i, the stage and the friction factors are not held behind the
// stores of ds, dlambda.  Inactive contacts: G = Gw = 0, Kinv = I, rhat = 0 -> zero steps.
template <typename T, int ROBOT>
__device__ __forceinline__ T dz_rows(const Ctx<T, ROBOT> &C, int k, const T (&dx)[9], T dtt, const T (&du)[NU],
                                     const T (&eu)[NU], const T (&dlt)[8], T dls, const T (&rh)[Rows<ROBOT>::NI],
                                     const T *__restrict__ st, const T *__restrict__ fu, const T *__restrict__ rdu,
                                     const T *__restrict__ rdi, const T *__restrict__ sv, const T *__restrict__ lm,
                                     T *__restrict__ ds, T *__restrict__ dl) {
    using S = Stage<ROBOT>;
    using R_ = Rows<ROBOT>;
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    const bool hu = k < C.N;
    const unsigned msk = C.cmask(k);
    T amax = T(1);
    auto emit = [&](int r, bool pr, T g, T dlr) {
        const T dsr = pr ? -rdi[r] - g : T(0);
        ds[r] = dsr;
        dl[r] = dlr;
        // branch-free ratio tests (selects keep the row loop one basic block)
        const T qs = fdiv(-sv[r], dsr < T(0) ? dsr : T(-1)), ql = fdiv(-lm[r], dlr < T(0) ? dlr : T(-1));
        amax = fmin(amax, fmin(dsr < T(0) ? qs : T(1), dlr < T(0) ? ql : T(1)));
    };
#pragma unroll
    for (int j = 0; j < 8; ++j)
        emit(j, true, tr_sign<T>(j, 0) * dx[6] + tr_sign<T>(j, 1) * dx[7] + tr_sign<T>(j, 2) * dx[8] + C.cw * dtt,
             dlt[j]);
    emit(8, true, -dtt, dls);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const bool pr = hu && ((msk >> c) & 1u);
        const T *cs = st + S::CON + S::CS * c;
        const T *g = fu + c * FU;
        T vf[3];
        for (int i = 0; i < 3; ++i) vf[i] = hu ? -(rdu[NUPC * c + FO + i] + eu[NUPC * c + FO + i]) : T(0);
        T z[4];
        for (int r = 0; r < 4; ++r)
            z[r] = g[3 * r] * vf[0] + g[3 * r + 1] * vf[1] + g[3 * r + 2] * vf[2] + rh[R_::FR + 4 * c + r];
        for (int r = 0; r < 4; ++r) {
            T acc = T(0);
            for (int q = 0; q < 4; ++q) acc += g[12 + p4(r, q)] * z[q];
            const T gr = cs[S::G + 3 * r] * du[NUPC * c + FO] + cs[S::G + 3 * r + 1] * du[NUPC * c + FO + 1] +
                         cs[S::G + 3 * r + 2] * du[NUPC * c + FO + 2];
            emit(R_::FR + 4 * c + r, pr, gr, hu ? acc : T(0));
        }
    }
    if (ROBOT == 1) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const bool pr = hu && ((msk >> c) & 1u);
            for (int q = 0; q < 4; ++q) {
                const int r = R_::CP + 4 * c + q, dd = q / 2;
                const T gr = (q % 2 == 0) ? du[NUPC * c + dd] : -du[NUPC * c + dd];
                emit(r, pr, gr, pr ? C.Dform(lm[r], sv[r]) * (gr + rh[r]) : T(0));
            }
        }
    }
    return amax;
}

template <typename T, int ROBOT>
__device__ T phase_dz(const Ctx<T, ROBOT> &C, int k, int corr, T sigma_mu) {
    using S = Stage<ROBOT>;
    using R_ = Rows<ROBOT>;
    constexpr int NI = R_::NI, NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    const int N = C.N;
    const bool hu = k < N;
    // E' dnu at knot k; the knot-type cases are selects over in-range blocks (one basic block)
    const T *dnu = C.ws + C.L.dnu;
    const int kc = hu ? k : 0;   // k = N: no controls or contacts (stage / factor records unused)
    T ex[9], eu[NU], a[9], d0[9], dk[9], dN[9];
    opAT(C.st(k) + S::W, C.beta, dnu + (size_t)(1 + k) * 9, a);   // k = N: block N+1 (unused)
    opBT<T, ROBOT>(C.st(kc), dnu + (size_t)(1 + kc) * 9, eu);
    ldv(dnu, d0);
    ldv(dnu + (size_t)k * 9, dk);
    ldv(dnu + (size_t)(N + 1) * 9, dN);
    for (int i = 0; i < 9; ++i)
        ex[i] = (k == 0 ? d0[i] : T(0)) + (hu ? a[i] : T(0)) - (k >= 1 ? dk[i] : T(0)) + (k == N ? dN[i] : T(0));
    T rh[NI], rdx[9], fxd[6], wu[NU];
    ldv(C.ws + C.L.rh + (size_t)k * NI, rh);   // this step's rhat, from phase_w
    ldv(C.ws + C.L.rdx + (size_t)k * 9, rdx);
    ldv(C.ws + C.L.facx + (size_t)k * FX, fxd);
    ldv(C.ws + C.L.wu + (size_t)kc * NU, wu);
    const T rdt = C.ws[C.L.rdt + k];
    T dx[9], dtt, du[NU], dlt[8], dls;
    for (int i = 0; i < 6; ++i) dx[i] = -fxd[i] * (rdx[i] + ex[i]);
    {
        const T vL[3] = {-(rdx[6] + ex[6]), -(rdx[7] + ex[7]), -(rdx[8] + ex[8])};
        tr_local(C, k, vL, -rdt, rh, dx + 6, dtt, dlt, dls);
    }
    {
        T au[NU];
        phi_solve_u(C, kc, eu, au);
        for (int i = 0; i < NU; ++i) du[i] = hu ? -wu[i] - au[i] : T(0);
    }
    stv(C.ws + C.L.dx + (size_t)k * 9, dx);
    C.ws[C.L.dt + k] = dtt;
    if (hu) stv(C.ws + C.L.du + (size_t)k * NU, du);
    return dz_rows<T, ROBOT>(C, k, dx, dtt, du, eu, dlt, dls, rh, C.st(k), C.ws + C.L.facu + (size_t)kc * NC * FU,
                             C.ws + C.L.rdu + (size_t)kc * NU, C.ws + C.L.rdi + (size_t)k * NI,
                             C.ws + C.L.s + (size_t)k * NI, C.ws + C.L.l + (size_t)k * NI,
                             C.ws + (corr ? C.L.ds : C.L.dsa) + (size_t)k * NI,
                             C.ws + (corr ? C.L.dl : C.L.dla) + (size_t)k * NI);
}

template <typename T, int ROBOT> __device__ T mu_after(const Ctx<T, ROBOT> &C, int k, T a) {
    constexpr int NI = Rows<ROBOT>::NI;
    const T *s = C.ws + C.L.s + (size_t)k * NI, *lm = C.ws + C.L.l + (size_t)k * NI;
    const T *ds = C.ws + C.L.dsa + (size_t)k * NI, *dl = C.ws + C.L.dla + (size_t)k * NI;
    T acc = T(0);
    for (int r = 0; r < NI; ++r)
        acc += (s[r] + a * ds[r]) * (lm[r] + a * dl[r]);   // absent rows: lambda = dl = 0
    return acc;
}

template <typename T, int ROBOT> __device__ void phase_update(const Ctx<T, ROBOT> &C, int k, T a, bool affine = false) {
    constexpr int NI = Rows<ROBOT>::NI;
    const int N = C.N;
    {
        T x[9], dx[9];
        ldv(C.var_x(k), x);
        ldv(C.ws + C.L.dx + (size_t)k * 9, dx);
        const T t = C.ws[C.L.t + k], dt = C.ws[C.L.dt + k];
        T n1[9], dn1[9], n0[9], dn0[9];
        ldv(C.ws + C.L.nu + (size_t)(1 + k) * 9, n1);        // k < N: dynamics block k; k = N: final
        ldv(C.ws + C.L.dnu + (size_t)(1 + k) * 9, dn1);
        if (k == 0) { ldv(C.ws + C.L.nu, n0); ldv(C.ws + C.L.dnu, dn0); }
        T u[NU], du[NU];
        if (k < N) { ldv(C.var_u(k), u); ldv(C.ws + C.L.du + (size_t)k * NU, du); }
        for (int i = 0; i < 9; ++i) { x[i] += a * dx[i]; n1[i] += a * dn1[i]; n0[i] += a * dn0[i]; }
        for (int i = 0; i < NU; ++i) u[i] += a * du[i];
        stv(C.var_x(k), x);
        C.ws[C.L.t + k] = t + a * dt;
        stv(C.ws + C.L.nu + (size_t)(1 + k) * 9, n1);
        if (k == 0) stv(C.ws + C.L.nu, n0);
        if (k < N) stv(C.var_u(k), u);
    }
    T *s = C.ws + C.L.s + (size_t)k * NI, *lm = C.ws + C.L.l + (size_t)k * NI;
    const T *ds = C.ws + (affine ? C.L.dsa : C.L.ds) + (size_t)k * NI;
    const T *dl = C.ws + (affine ? C.L.dla : C.L.dl) + (size_t)k * NI;
    T sv[NI], dsv[NI];   // absent rows: ds = dl = 0 (s stays 1, lambda 0)
    ldv(s, sv); ldv(ds, dsv);
    for (int r = 0; r < NI; ++r) sv[r] += a * dsv[r];
    T lv[NI], dlv[NI];
    ldv(lm, lv); ldv(dl, dlv);
    stv(s, sv);
    for (int r = 0; r < NI; ++r) lv[r] += a * dlv[r];
    stv(lm, lv);
}


// initialization step: full Newton step for z and nu; s = h - gz at the new z; lambda += dlambda.
// vmax receives (max -s, max -lambda) over this knot's rows.
template <typename T, int ROBOT> __device__ void phase_init_step(const Ctx<T, ROBOT> &C, int k, T (&vmax)[2]) {
    constexpr int NI = Rows<ROBOT>::NI;
    phase_update<T, ROBOT>(C, k, T(1), true);   // z, nu, lambda: full affine step; s recomputed below
    const int N = C.N;
    const T *x = C.var_x(k);
    const T t = C.ws[C.L.t + k];
    const T *u = C.var_u(k < N ? k : 0);   // k = N: rows of u are absent (values unused)
    T *s = C.ws + C.L.s + (size_t)k * NI, *lm = C.ws + C.L.l + (size_t)k * NI;
    for (int r = 0; r < NI; ++r) {
        if (!C.present(k, r)) continue;
        s[r] = -C.gz(k, r, x, t, u, true);
        vmax[0] = fmax(vmax[0], -s[r]);
        vmax[1] = fmax(vmax[1], -lm[r]);
    }
}
template <typename T, int ROBOT> __device__ void phase_init_shift(const Ctx<T, ROBOT> &C, int k, T sh_s, T sh_l) {
    constexpr int NI = Rows<ROBOT>::NI;
    T *s = C.ws + C.L.s + (size_t)k * NI, *lm = C.ws + C.L.l + (size_t)k * NI;
    for (int r = 0; r < NI; ++r) {
        if (!C.present(k, r)) continue;
        s[r] += sh_s;
        lm[r] += sh_l;
    }
}

// ------------------------------------------------------------------ kernel
template <typename T, int ROBOT, bool SL>
__global__ void __launch_bounds__(NT) k_qp_ipm(DevBuf<T> d, int only_active, int max_iter, T eps_abs, T eps_rel,
                                               T eta) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dsmem[];
    constexpr int NI = Rows<ROBOT>::NI;
    const int b = blockIdx.x;
    if (b >= d.B) return;
    if (only_active && !d.scp[b].active) return;
    __shared__ T red[8 * (NT / 64)];
    __shared__ T sh[2 * TW_SCRATCH];
    const int tid = threadIdx.x, N = d.N, K1 = N + 1, NB = N + 2, NBm = NB / 2;
    Ctx<T, ROBOT> C{N, nullptr, nullptr, nullptr, nullptr, T(0), T(0), nullptr, WsLayout(N, NI, Robot<ROBOT>::NC),
                    nullptr, nullptr, T(0)};
    C.prm = d.params + d.class_id[b];
    C.stage = d.stage + (size_t)b * K1 * Stage<ROBOT>::SIZE;
    C.logic = d.logic + (size_t)b * N * Robot<ROBOT>::NC;
    C.xbar = d.Xbar + (size_t)b * K1 * 9;
    C.cw = d.cw[b];
    C.beta = C.prm->dt / C.prm->mass;
    {
        T wmax = T(1);
        for (int i = 0; i < 9; ++i) wmax = fmax(wmax, C.prm->Wx[i]);
        C.dcap = T(1e12) * wmax;
    }
    C.ws = d.ws + (size_t)b * d.ws_stride;
    T *vbuf = reinterpret_cast<T *>(dsmem);
    LdsT<T> *vbl = (LdsT<T> *)vbuf, *shl = (LdsT<T> *)sh;
    // the Schur inverses sit in LDS when they fit (SL); the off-diagonal factors always in HBM
    C.Sd = SL ? vbuf + (((size_t)NB * 9 + 7) & ~size_t(7)) : C.ws + C.L.Sd;
    C.So = C.ws + C.L.So;
#ifdef CMPC_STAMPS
    unsigned long long t_prev = __builtin_amdgcn_s_memtime(), t_acc[12] = {};
#define STAMP(i)                                                               \
    do {                                                                       \
        const unsigned long long t_now = __builtin_amdgcn_s_memtime();         \
        t_acc[i] += t_now - t_prev;                                            \
        t_prev = t_now;                                                        \
    } while (0)
#else
#define STAMP(i) do { } while (0)
#endif
    // ---- starting point of the initialization step: z = (xbar, ubar, 0), nu = 0, s = lambda = 1
    for (int k = tid; k < K1; k += NT) {
        T *x = C.var_x(k);
        for (int i = 0; i < 9; ++i) x[i] = C.xbar[(size_t)k * 9 + i];
        C.ws[C.L.t + k] = T(0);
        const T *ubar = d.Ubar + ((size_t)b * N + (k < N ? k : 0)) * NU;
        if (k < N) { T *u = C.var_u(k); for (int i = 0; i < NU; ++i) u[i] = ubar[i]; }
        T *s = C.ws + C.L.s + (size_t)k * NI, *lm = C.ws + C.L.l + (size_t)k * NI;
        for (int r = 0; r < NI; ++r) {
            s[r] = T(1);
            lm[r] = C.present(k, r) ? T(1) : T(0);
        }
        T *dsa = C.ws + C.L.dsa + (size_t)k * NI, *dla = C.ws + C.L.dla + (size_t)k * NI;
        for (int r = 0; r < NI; ++r) { dsa[r] = T(0); dla[r] = T(0); }
    }
    for (int e = tid; e < NB * 9; e += NT) C.ws[C.L.nu + e] = T(0);
    __syncthreads();
    int status = CMPC_QP_MAX_ITER, it = 0, stall = 0;
    T mu_prev = T(-1);
    // it == 0 is the initialization step (CVXOPT-style): one full Newton step from
    // s = lambda = 1 gives an equality-feasible least-squares start; s and lambda are then
    // shifted by (1 + max violation) where negative.
    for (it = 0; it <= max_iter; ++it) {
        const bool init = (it == 0);
        Norms<T, ROBOT> nm{0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = tid; k < K1; k += NT) phase_residual<T, ROBOT>(C, k, nm);
        T mx[6] = {nm.prim, nm.dual, nm.comp, nm.sp, nm.sd, nm.lmax};
        block_reduce<T, NT, 6, 1>(mx, red);
        T sm2[2] = {nm.mu, nm.cnt};
        block_reduce<T, NT, 2, 0>(sm2, red);
        STAMP(0);
        const T prim = mx[0], dual = mx[1], comp = mx[2], sp = mx[3], sdd = mx[4];
        const T mu = sm2[0] / fmax(sm2[1], T(1));
        const T ep = eps_abs + eps_rel * sp, ed = eps_abs + eps_rel * sdd;
        const T merit = fmax(prim / ep, fmax(dual / ed, comp / ed));
        if (!(merit == merit) || !(mu == mu)) { status = CMPC_QP_NONFINITE; break; }
        if (!init) {
            if (merit <= T(1)) { status = 1; break; }
            // stall guard: mu not decreasing for 3 iterations while within 1e3x of tolerance
            stall = (mu_prev >= T(0) && mu >= T(0.5) * mu_prev) ? stall + 1 : 0;
            mu_prev = mu;
            if (stall >= 3 && merit <= T(1e3)) { status = 1; break; }
        }
        if (it == max_iter) break;
        // ---- factorization
        for (int k = tid; k < K1; k += NT) phase_factor<T, ROBOT>(C, k);
        __syncthreads();
        STAMP(1);
        for (int k = tid; k < K1; k += NT) phase_sblock<T, ROBOT>(C, k);
        __syncthreads();
        STAMP(2);
        if (SL) {
            if (tid < 128) tw_factor_ends<T, LdsT<T>>((LdsT<T> *)C.Sd, C.So, NB, NBm, shl);
            __syncthreads();
            if (tid < 64) tw_factor_meet<T, LdsT<T>>((LdsT<T> *)C.Sd, C.So, NBm, shl);
        } else {
            if (tid < 128) tw_factor_ends<T, T>(C.Sd, C.So, NB, NBm, shl);
            __syncthreads();
            if (tid < 64) tw_factor_meet<T, T>(C.Sd, C.So, NBm, shl);
        }
        STAMP(3);
        __syncthreads();
        // ---- predictor (affine) and corrector
        T sigma_mu = T(0);
        T alpha = T(1);
        for (int corr = 0; corr < 2; ++corr) {
            for (int k = tid; k < K1; k += NT) phase_w<T, ROBOT>(C, k, corr, sigma_mu);
            __syncthreads();
            STAMP(4);
            for (int k = tid; k < K1; k += NT) phase_rhs<T, ROBOT>(C, k);
            __syncthreads();
            STAMP(5);
            if (tid < 128) tw_solve_elim<T>(C.So, C.ws + C.L.rhs, NB, NBm, vbl);
            __syncthreads();
            if (SL) {
                if (tid < 64) tw_solve_meet<T, LdsT<T>>((LdsT<T> *)C.Sd, C.So, NB, NBm, vbl, shl);
                __syncthreads();
                if (tid < 128) tw_solve_back<T, LdsT<T>>((LdsT<T> *)C.Sd, C.So, C.ws + C.L.dnu, NB, NBm, vbl);
            } else {
                if (tid < 64) tw_solve_meet<T, T>(C.Sd, C.So, NB, NBm, vbl, shl);
                __syncthreads();
                if (tid < 128) tw_solve_back<T, T>(C.Sd, C.So, C.ws + C.L.dnu, NB, NBm, vbl);
            }
            __syncthreads();
            STAMP(6);
            T am[1] = {T(1)};
            for (int k = tid; k < K1; k += NT) am[0] = fmin(am[0], phase_dz<T, ROBOT>(C, k, corr, sigma_mu));
            block_reduce<T, NT, 1, 2>(am, red);
            STAMP(7);
            alpha = am[0];
            if (init) break;
            if (corr == 0) {
                T ma[1] = {T(0)};
                for (int k = tid; k < K1; k += NT) ma[0] += mu_after<T, ROBOT>(C, k, alpha);
                block_reduce<T, NT, 1, 0>(ma, red);
                const T mu_aff = ma[0] / fmax(sm2[1], T(1));
                const T sg = mu_aff / fmax(mu, T(1e-300));
                sigma_mu = sg * sg * sg * mu;
            }
        }
        if (init) {
            T vmax[2] = {T(-1e300), T(-1e300)};
            for (int k = tid; k < K1; k += NT) phase_init_step<T, ROBOT>(C, k, vmax);
            block_reduce<T, NT, 2, 1>(vmax, red);
            const T sh_s = vmax[0] >= T(0) ? T(1) + vmax[0] : T(0);
            const T sh_l = vmax[1] >= T(0) ? T(1) + vmax[1] : T(0);
            for (int k = tid; k < K1; k += NT) phase_init_shift<T, ROBOT>(C, k, sh_s, sh_l);
            __syncthreads();
            continue;
        }
        alpha = fmin(T(1), eta * alpha);
        for (int k = tid; k < K1; k += NT) phase_update<T, ROBOT>(C, k, alpha);
        __syncthreads();
        STAMP(8);
    }
    // ---- outputs: solution and multipliers
    for (int k = tid; k < K1; k += NT) {
        const T *x = C.var_x(k);
        for (int i = 0; i < 9; ++i) d.xs[((size_t)b * K1 + k) * 9 + i] = x[i];
        d.ts[(size_t)b * K1 + k] = C.ws[C.L.t + k];
        if (k < N) { const T *u = C.var_u(k); for (int i = 0; i < NU; ++i) d.us[((size_t)b * N + k) * NU + i] = u[i]; }
        const T *lm = C.ws + C.L.l + (size_t)k * NI;
        for (int r = 0; r < NI; ++r) d.lams[((size_t)b * K1 + k) * NI + r] = C.present(k, r) ? lm[r] : T(0);
    }
    for (int e = tid; e < NB * 9; e += NT) d.nus[(size_t)b * NB * 9 + e] = C.ws[C.L.nu + e];
    if (tid == 0) {
        d.qp_status[b] = status;
        d.qp_iters[b] = it;
#ifdef CMPC_STAMPS
        for (int i = 0; i < 12; ++i) d.stamps[(size_t)b * 16 + i] = t_acc[i];
#endif
    }
#undef STAMP
}

#define INST(T, R)                                                                   \
    template __global__ void k_qp_ipm<T, R, false>(DevBuf<T>, int, int, T, T, T);     \
    template __global__ void k_qp_ipm<T, R, true>(DevBuf<T>, int, int, T, T, T);
INST(double, 0)
INST(double, 1)
INST(float, 0)
INST(float, 1)
#undef INST

size_t ipm_vec_lds_bytes(int N, int prec_bytes) { return (((size_t)(N + 2) * 9 + 7) & ~size_t(7)) * prec_bytes; }
size_t ipm_schur_lds_bytes(int N, int prec_bytes) { return (size_t)(N + 2) * 81 * prec_bytes; }

size_t ipm_workspace_elems(int N, int robot) {
    return robot == 0 ? WsLayout(N, Rows<0>::NI, Robot<0>::NC).total : WsLayout(N, Rows<1>::NI, Robot<1>::NC).total;
}

}  // namespace cmpc
