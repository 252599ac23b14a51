// Structured QP assembly: one stage record per (problem, knot).
//
// Replaces sum_up_all_costs / stack_up_all_constraints (reference src/scp_solver.py:10-48)
// and the constraint builders of src/constraints.py, which materialize a dense n x n cost and
// dense constraint blocks and vstack them into CSC every SCP iteration.  Here the QP stays in
// its per-knot structure; cmpc_export_qp rebuilds the reference's CSC (exact row order) on the
// host for parity tests only.
//
// Record (see Stage<ROBOT> in common.hpp): dynamics rhs r_k = A_k xbar_k + B_k ubar_k - f_k
// (src/constraints.py:36-45), tracking gradient qx_k = -Wx xbar_k (src/cost.py:21-29), trust-
// region bounds btr_kj = radius + s_j' Lbar_k (src/constraints.py:278-286), the compact A_k
// (skew vector w_k = dt sum a_i f_i) and B_k (alpha_i = dt a_i, lever_i, TALOS cop/tau
// columns), friction rows G = (F_mu R')[0:4] (src/constraints.py:171-185) and their upper
// bounds h (0, or minus the chance-constraint back-off 2 xi G_u sqrt(K Sigma K')_uu,
// src/constraints.py:186-214).  Thread per knot; HBM-bound.  Records are stored field-major per
// problem (field f of knot k at stage[(b * SIZE + f) * KPC + k]) so the QP kernel's per-knot
// loads coalesce.
//
// FULL = false (the default path): k_lin_knots has already written the fields that depend only on
// the linearization (r, w, the per-contact alpha / lever / G / cop / tau), so this kernel writes
// the ones that depend on the warm start and the SCP state: qx, the trust-region bounds, cw and h.
// FULL = true follows the legacy k_linearize (non-diagonal R) and writes the whole record.
#include "common.hpp"

namespace cmpc {

template <typename T, int ROBOT, bool FULL>
__global__ void __launch_bounds__(128) k_assemble(DevBuf<T> d, int only_active) {
    constexpr int NC = Robot<ROBOT>::NC, NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    using St = Stage<ROBOT>;
    const int N = d.N, K1 = N + 1;
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)d.B * K1) return;
    const int b = (int)(gid / K1), k = (int)(gid % K1);
    const ScpState &sc = d.scp[b];
    if (only_active && !sc.active) return;
    const DevParams<T> &prm = d.params[d.class_id[b]];
    const SV<T> st{d.stage + (size_t)b * St::SIZE * KPC + k};   // field-major record (common.hpp)
    const T *xr = d.Xbar + gid * 9;   // warm start: tracking reference (src/cost.py:21-29)
    const T *xb = d.Xlin + gid * 9;   // linearization point (= warm start in reference mode, quirk Q1)
    const T radius = T(sc.radius);
    if (k == 0) d.cw[b] = T(-1.0 / sc.weight);
    for (int i = 0; i < 9; ++i) st[St::QX + i] = prm.tracking ? -prm.Wx[i] * xr[i] : T(0);
    for (int j = 0; j < 8; ++j) {
        const T s0 = (j & 1) ? T(-1) : T(1), s1 = (j & 2) ? T(-1) : T(1), s2 = (j & 4) ? T(-1) : T(1);
        st[St::BTR + j] = radius + (s0 * xb[6] + s1 * xb[7] + s2 * xb[8]);
    }
    if (k == N) return;
    const size_t kn = (size_t)b * N + k;
    auto em = [&](const T *base, int e) -> T { return base[(size_t)e * d.LS + kn]; };   // element-major
    const T *ub = d.Ulin + kn * NU;
    if (FULL)
        for (int i = 0; i < 9; ++i) {
            T acc = -em(d.f, i);
            for (int j = 0; j < 9; ++j) acc = fma(em(d.A, i * 9 + j), xb[j], acc);
            for (int j = 0; j < NU; ++j) acc = fma(em(d.Bu, i * NU + j), ub[j], acc);
            st[St::R + i] = acc;
        }
    const T dt = prm.dt;
    const T *pos = d.pos + kn * 3 * NC, *rot = d.rot + kn * 9 * NC;
    const uint8_t *lg = d.logic + kn * NC;
    if (FULL) {
        T w[3] = {0, 0, 0};
        for (int c = 0; c < NC; ++c)
            for (int q = 0; q < 3; ++q) w[q] += T(lg[c]) * ub[NUPC * c + FO + q];
        for (int q = 0; q < 3; ++q) st[St::W + q] = dt * w[q];
    }
    const T ml = prm.mu / sqrt(T(2));
    const T Fmu[4][3] = {{1, 0, -ml}, {-1, 0, -ml}, {0, 1, -ml}, {0, -1, -ml}};
    for (int c = 0; c < NC; ++c) {
        const SV<T> cs = st + (St::CON + St::CS * c);
        const T a = T(lg[c]);
        const T *Rc = rot + 9 * c;
        const T *uc = ub + NUPC * c;
        if (FULL) {
            cs[St::ALPHA] = dt * a;
            T lev[3];
            for (int z = 0; z < 3; ++z) lev[z] = pos[3 * c + z] - xb[z];
            if (ROBOT == 1)
                for (int z = 0; z < 3; ++z) lev[z] += Rc[z * 3 + 0] * uc[0] + Rc[z * 3 + 1] * uc[1];
            for (int z = 0; z < 3; ++z) cs[St::LEVER + z] = lev[z];
            // friction rows 0..3: (F_mu R')[r, :]
            for (int r = 0; r < 4; ++r)
                for (int q = 0; q < 3; ++q) {
                    T g = T(0);
                    for (int z = 0; z < 3; ++z) g = fma(Fmu[r][z], Rc[q * 3 + z], g);
                    cs[St::G + r * 3 + q] = g;
                }
        }
        T h[4] = {0, 0, 0, 0};
        if (prm.stochastic && k > 0 && lg[c]) {
            // K rows 3c..3c+2 (reference uses Debris.idx*3, also for TALOS), Sigma_k = Covs[k]
            const T *Sg = d.Sig + ((size_t)b * K1 + k) * 81;
            T KS[3][9];
            for (int r = 0; r < 3; ++r)
                for (int j = 0; j < 9; ++j) {
                    T acc = T(0);
                    for (int q = 0; q < 9; ++q) acc = fma(em(d.K, (3 * c + r) * 9 + q), Sg[q * 9 + j], acc);
                    KS[r][j] = acc;
                }
            for (int uu = 0; uu < 3; ++uu) {
                T v = T(0);
                for (int j = 0; j < 9; ++j) v = fma(KS[uu][j], em(d.K, (3 * c + uu) * 9 + j), v);
                const T sv = sqrt(v);
                for (int r = 0; r < 4; ++r) {
                    const T g = cs[St::G + r * 3 + uu];
                    if (g > T(1e-6) && sv > T(1e-6)) h[r] -= prm.xi * (T(2) * g * sv);
                }
            }
        }
        for (int r = 0; r < 4; ++r) cs[St::H + r] = h[r];
        if (FULL && ROBOT == 1) {
            // cop columns of B rows 6..8: -a dt [f]x R[:, 0:2];  tau column: a dt R[:, 2]
            const T *fc = uc + FO;
            const T sk[9] = {0, -fc[2], fc[1], fc[2], 0, -fc[0], -fc[1], fc[0], 0};
            for (int r = 0; r < 3; ++r) {
                for (int q = 0; q < 2; ++q) {
                    T acc = T(0);
                    for (int z = 0; z < 3; ++z) acc += sk[r * 3 + z] * Rc[z * 3 + q];
                    cs[St::BCOP + r * 2 + q] = -dt * a * acc;
                }
                cs[St::BTAU + r] = dt * a * Rc[r * 3 + 2];
            }
        }
    }
}

#define INST(T, R)                                                      \
    template __global__ void k_assemble<T, R, true>(DevBuf<T>, int);  \
    template __global__ void k_assemble<T, R, false>(DevBuf<T>, int);
INST(double, 0)
INST(double, 1)
INST(float, 0)
INST(float, 1)
#undef INST

}  // namespace cmpc
