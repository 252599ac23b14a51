// cmpc_load_qp: a subproblem given in the reference's CSC layout (P, q, A, l, u as
// solve_subproblem receives them, src/scp_solver.py:59-68) decoded into the structured form the
// QP kernel solves, so the device solver takes QPs that were not assembled on the device.
//
// The kernel exploits the stage structure, so the QP must have it; every assumption is checked
// and a QP that breaks one is refused with -2 and a message naming the row or column:
//   * variables z = [x_0..x_N | u_0..u_{N-1} | t_0..t_N | s_0..s_{N-1}] (src/optimizer.py), rows
//     init | dynamics | final | [TALOS CoP] | friction | trust region | slack
//     (src/scp_solver.py:28-48), sizes from the handle's robot and N;
//   * P diagonal: one state weight vector Wx for every knot, one control weight vector Wu, zero on
//     t and s; q: any tracking gradient on the states, 0 on u and s, 1 on t;
//   * dynamics blocks of the centroidal form (src/centroidal_model.py:189-241):
//     A_k = [[I, beta I, 0], [0, I, 0], [[w]x, 0, I]],  B_k = sum over contacts of
//     alpha [0; I; [lever]x] on the forces (+ the TALOS CoP / torque columns of rows 6..8),
//     the -I on x_{k+1}, equal bounds (the reference's r +- 1e-12);
//   * friction rows G (4 filled + the empty 5th, quirk Q4) with lower bound -inf, present exactly
//     where the dynamics use the contact; TALOS CoP box rows with one foot_range;
//   * trust-region rows with the (+-1, +-1, +-1) pattern on the angular momentum and one slack
//     coefficient -1/omega; slack rows -t <= 0.
// What the kernel reads outside the stage record is installed too: a parameter class (a copy of
// the problem's class with the decoded Wx, Wu, mass = dt / beta and, TALOS, foot_range), the
// slack coefficient, the boundary states (X̄ at knots 0 and N), the contact masks, and a starting
// point (x_0 on every knot, zero controls).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "cmpc.h"
#include "common.hpp"
#include "handle.hpp"

using namespace cmpc;
using namespace cmpc_host;

namespace {

struct Csr {   // row access to a CSC matrix
    std::vector<int> p, c;
    std::vector<double> v;
};

Csr to_csr(int m, int n, const double *x, const int32_t *ii, const int32_t *pp) {
    Csr r;
    r.p.assign(m + 1, 0);
    need(pp[0] == 0 && pp[n] >= 0, "A: invalid column pointers");
    for (int j = 0; j < n; ++j) {
        need(pp[j + 1] >= pp[j], "A: column pointers not monotone");
        for (int e = pp[j]; e < pp[j + 1]; ++e) {
            need(ii[e] >= 0 && ii[e] < m, "A: row index out of range");
            ++r.p[ii[e] + 1];
        }
    }
    for (int i = 0; i < m; ++i) r.p[i + 1] += r.p[i];
    r.c.resize(pp[n]);
    r.v.resize(pp[n]);
    std::vector<int> fill(r.p.begin(), r.p.end() - 1);
    for (int j = 0; j < n; ++j)
        for (int e = pp[j]; e < pp[j + 1]; ++e) {
            const int d = fill[ii[e]]++;
            r.c[d] = j;
            r.v[d] = x[e];
        }
    return r;
}

bool close(double a, double b, double scale, double tol = 1e-10) { return std::fabs(a - b) <= tol * scale; }

std::string at(const char *what, int k, int i = -1) {
    return std::string(what) + " (knot " + std::to_string(k) + (i >= 0 ? ", row " + std::to_string(i) : "") + ")";
}

}  // namespace

extern "C" int cmpc_load_qp(cmpc_handle h, int b, int n, int m, const double *P_x, const int32_t *P_i,
                            const int32_t *P_p, const double *q, const double *A_x, const int32_t *A_i,
                            const int32_t *A_p, const double *l, const double *u) {
    return guard(h, [&] {
        need(P_x && P_i && P_p && q && A_x && A_i && A_p && l && u, "null QP buffer");
        need(b >= 0 && b < h->B, "problem index out of range (upload a batch first)");
        need(h->n_classes > 0, "call cmpc_set_params first");
        const int N = h->N, K1 = N + 1, NC = h->NC, robot = h->robot;
        const int NUPC = NU / NC, FO = robot == 0 ? 0 : 2;
        const int nx = 9 * K1, iu = nx, it = nx + NU * N, is = it + K1;
        const int n_exp = is + N;
        const int mcop = robot == 1 ? 2 * NC * N : 0;
        const int r_dyn = 9, r_fin = 9 + 9 * N, r_cop = r_fin + 9, r_fr = r_cop + mcop, r_tr = r_fr + 5 * NC * N,
                  r_sl = r_tr + 8 * K1, m_exp = r_sl + K1;
        need(n == n_exp, "n = " + std::to_string(n) + ", the handle's layout has " + std::to_string(n_exp) + " variables");
        need(m == m_exp, "m = " + std::to_string(m) + ", the handle's layout has " + std::to_string(m_exp) + " rows");
        const double INF = 1e20;

        // ---- cost: diagonal P, one Wx / Wu for all knots
        std::vector<double> pd(n, 0.0);
        need(P_p[0] == 0, "P: invalid column pointers");
        for (int j = 0; j < n; ++j) need(P_p[j + 1] >= P_p[j], "P: column pointers not monotone");
        for (int j = 0; j < n; ++j)
            for (int e = P_p[j]; e < P_p[j + 1]; ++e) {
                need(P_i[e] >= 0 && P_i[e] < n, "P: row index out of range");
                if (P_x[e] == 0.0) continue;
                need(P_i[e] == j, "P has an off-diagonal entry at (" + std::to_string(P_i[e]) + ", " + std::to_string(j) + ")");
                pd[j] += P_x[e];
            }
        cmpc_params prm = h->hparams[0];
        {
            int32_t cid = 0;
            from_dev_raw(h, &cid, (char *)h->class_id + (size_t)b * 4, 4);
            prm = h->hparams[cid];
        }
        for (int i = 0; i < 9; ++i) {
            prm.Wx[i] = pd[i];
            need(pd[i] > 0, "P: state weight " + std::to_string(i) + " must be positive");
            for (int k = 1; k < K1; ++k) need(close(pd[9 * k + i], pd[i], pd[i], 1e-12), at("P: state weights differ", k, i));
        }
        for (int i = 0; i < NU; ++i) {
            prm.Wu[i] = pd[iu + i];
            need(pd[iu + i] > 0, "P: control weight " + std::to_string(i) + " must be positive");
            for (int k = 1; k < N; ++k)
                need(close(pd[iu + NU * k + i], pd[iu + i], pd[iu + i], 1e-12), at("P: control weights differ", k, i));
        }
        for (int j = it; j < n; ++j) need(pd[j] == 0.0, "P must be zero on the slacks t, s");
        for (int j = iu; j < it; ++j) need(q[j] == 0.0, "q must be zero on the controls");
        for (int j = it; j < is; ++j) need(q[j] == 1.0, "q must be 1 on the trust-region slacks t");
        for (int j = is; j < n; ++j) need(q[j] == 0.0, "q must be zero on the unused slacks s");

        const Csr A = to_csr(m, n, A_x, A_i, A_p);
        auto row = [&](int r, auto &&fn) {
            for (int e = A.p[r]; e < A.p[r + 1]; ++e)
                if (A.v[e] != 0.0) fn(A.c[e], A.v[e]);
        };
        auto empty = [&](int r) {
            bool ok = true;
            row(r, [&](int, double) { ok = false; });
            return ok;
        };
        auto equality = [&](int r) {
            const double mid = 0.5 * (l[r] + u[r]);
            need(u[r] - l[r] <= 1e-9 * (1 + std::fabs(mid)), "row " + std::to_string(r) + " must be an equality");
            return mid;
        };
        for (int j = is; j < n; ++j)
            for (int e = A_p[j]; e < A_p[j + 1]; ++e) need(A_x[e] == 0.0, "the unused slacks s must not appear in A");

        using S = Stage<0>;   // offsets are robot-independent below CON + CS * NC
        const int SIZE = robot == 0 ? Stage<0>::SIZE : Stage<1>::SIZE;
        std::vector<double> st((size_t)SIZE * KPC, 0.0);
        auto put = [&](int f, int k, double v) { st[(size_t)f * KPC + k] = v; };
        std::vector<double> xb((size_t)K1 * 9, 0.0);
        std::vector<int8_t> logic((size_t)N * NC, 0);

        // ---- boundary rows
        for (int i = 0; i < 9; ++i) {
            int nz = 0;
            row(i, [&](int c, double v) { need(c == i && v == 1.0, at("initial-state row must be x_0", 0, i)); ++nz; });
            need(nz == 1, at("initial-state row must be x_0", 0, i));
            xb[i] = equality(i);
            nz = 0;
            row(r_fin + i, [&](int c, double v) {
                need(c == 9 * N + i && v == 1.0, at("final-state row must be x_N", N, i));
                ++nz;
            });
            need(nz == 1, at("final-state row must be x_N", N, i));
            xb[(size_t)N * 9 + i] = equality(r_fin + i);
        }

        // ---- friction rows first: which contacts are present at each knot
        for (int c = 0; c < NC; ++c)
            for (int k = 0; k < N; ++k) {
                const int r0 = r_fr + (c * N + k) * 5, fcol = iu + NU * k + NUPC * c + FO;
                bool any = false;
                for (int j = 0; j < 4; ++j) any = any || !empty(r0 + j);
                need(empty(r0 + 4), at("the fifth friction row must be empty (quirk Q4)", k, c));
                logic[(size_t)k * NC + c] = any ? 1 : 0;
                for (int j = 0; j < 4; ++j) {
                    need(l[r0 + j] <= -INF, at("friction rows have no lower bound", k, c));
                    if (!any) {
                        need(u[r0 + j] >= 0, at("an absent contact's friction row is infeasible", k, c));
                        continue;
                    }
                    double g[3] = {0, 0, 0};
                    row(r0 + j, [&](int col, double v) {
                        need(col >= fcol && col < fcol + 3, at("friction row outside the contact's force", k, c));
                        g[col - fcol] = v;
                    });
                    for (int z = 0; z < 3; ++z) put(S::CON + S::CS * c + S::G + 3 * j + z, k, g[z]);
                    put(S::CON + S::CS * c + S::H + j, k, u[r0 + j]);
                }
            }

        // ---- TALOS CoP box rows: one foot_range
        if (robot == 1) {
            bool have[2] = {false, false};
            double fr[4] = {0, 0, 0, 0};   // lxp, lxn, lyp, lyn
            for (int c = 0; c < NC; ++c)
                for (int d = 0; d < 2; ++d)
                    for (int k = 0; k < N; ++k) {
                        const int r = r_cop + (c * 2 + d) * N + k, col = iu + NU * k + NUPC * c + d;
                        if (!logic[(size_t)k * NC + c]) {
                            need(empty(r) && l[r] <= 0 && u[r] >= 0, at("an absent contact's CoP row must be empty", k, c));
                            continue;
                        }
                        int nz = 0;
                        row(r, [&](int cc, double v) { need(cc == col && v == 1.0, at("CoP row must bound the contact's CoP", k, c)); ++nz; });
                        need(nz == 1, at("CoP row must bound the contact's CoP", k, c));
                        const double hi = u[r], lo = -l[r];
                        if (!have[d]) {
                            fr[2 * d] = hi;
                            fr[2 * d + 1] = lo;
                            have[d] = true;
                        }
                        need(close(hi, fr[2 * d], 1 + std::fabs(hi), 1e-12) && close(lo, fr[2 * d + 1], 1 + std::fabs(lo), 1e-12),
                             at("CoP bounds differ from the first contact's (one foot_range per QP)", k, c));
                    }
            for (int i = 0; i < 4; ++i) prm.foot_range[i] = fr[i];
        }

        // ---- dynamics rows: decode beta, w, alpha, lever (+ TALOS CoP / torque columns), rebuild, compare
        double beta = 0;
        std::vector<double> Aem((size_t)81 * N), Bem((size_t)9 * NU * N);   // element-major [e][k], for the getters
        for (int k = 0; k < N; ++k) {
            double Ad[9][9] = {}, Bd[9][NU] = {};
            for (int i = 0; i < 9; ++i) {
                const int r = r_dyn + 9 * k + i;
                bool next = false;
                row(r, [&](int c, double v) {
                    if (c >= 9 * k && c < 9 * k + 9) Ad[i][c - 9 * k] = v;
                    else if (c >= iu + NU * k && c < iu + NU * (k + 1)) Bd[i][c - iu - NU * k] = v;
                    else if (c == 9 * (k + 1) + i && v == -1.0) next = true;
                    else need(false, at("dynamics row has an entry outside x_k, u_k, x_{k+1}", k, i));
                });
                need(next, at("dynamics row must carry -1 on x_{k+1}", k, i));
                put(S::R + i, k, equality(r));
            }
            if (k == 0) beta = Ad[0][3];
            const double w[3] = {Ad[8][1], Ad[6][2], Ad[7][0]};
            for (int i = 0; i < 3; ++i) put(S::W + i, k, w[i]);
            double Ar[9][9] = {};
            for (int i = 0; i < 9; ++i) Ar[i][i] = 1;
            for (int i = 0; i < 3; ++i) Ar[i][3 + i] = beta;
            const double sk[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) Ar[6 + i][j] = sk[i][j];
            double sa = 1;
            for (int i = 0; i < 9; ++i)
                for (int j = 0; j < 9; ++j) sa = std::fmax(sa, std::fabs(Ad[i][j]));
            for (int i = 0; i < 9; ++i)
                for (int j = 0; j < 9; ++j)
                    need(close(Ad[i][j], Ar[i][j], sa), at("A_k is not of the centroidal form", k, i));
            double Br[9][NU] = {}, sb = 1;
            for (int i = 0; i < 9; ++i)
                for (int j = 0; j < NU; ++j) sb = std::fmax(sb, std::fabs(Bd[i][j]));
            for (int c = 0; c < NC; ++c) {
                const int f0 = NUPC * c + FO;
                const double a = Bd[3][f0];
                need((a != 0.0) == (logic[(size_t)k * NC + c] != 0),
                     at("a contact's force enters the dynamics exactly where its friction rows exist", k, c));
                double lev[3] = {0, 0, 0};
                if (a != 0.0) { lev[0] = Bd[8][f0 + 1] / a; lev[1] = Bd[6][f0 + 2] / a; lev[2] = Bd[7][f0] / a; }
                const int cb = S::CON + S::CS * c;
                put(cb + S::ALPHA, k, a);
                for (int z = 0; z < 3; ++z) put(cb + S::LEVER + z, k, lev[z]);
                const double sl[3][3] = {{0, -lev[2], lev[1]}, {lev[2], 0, -lev[0]}, {-lev[1], lev[0], 0}};
                for (int i = 0; i < 3; ++i) {
                    Br[3 + i][f0 + i] = a;
                    for (int j = 0; j < 3; ++j) Br[6 + i][f0 + j] = a * sl[i][j];
                }
                if (robot == 1) {
                    for (int r = 0; r < 3; ++r) {
                        for (int qd = 0; qd < 2; ++qd) {
                            Br[6 + r][NUPC * c + qd] = Bd[6 + r][NUPC * c + qd];
                            put(cb + S::BCOP + 2 * r + qd, k, Bd[6 + r][NUPC * c + qd]);
                        }
                        Br[6 + r][NUPC * c + 5] = Bd[6 + r][NUPC * c + 5];
                        put(cb + S::BTAU + r, k, Bd[6 + r][NUPC * c + 5]);
                    }
                }
            }
            for (int i = 0; i < 9; ++i)
                for (int j = 0; j < NU; ++j)
                    need(close(Bd[i][j], Br[i][j], sb), at("B_k is not of the centroidal form", k, i));
            for (int i = 0; i < 9; ++i) {
                for (int j = 0; j < 9; ++j) Aem[(size_t)(i * 9 + j) * N + k] = Ad[i][j];
                for (int j = 0; j < NU; ++j) Bem[(size_t)(i * NU + j) * N + k] = Bd[i][j];
            }
        }
        need(beta > 0, "A_0 must carry dt / mass > 0 on the momentum columns");
        prm.mass = prm.dt / beta;

        // ---- trust region (8 rows per knot: s_j' L_k + cw t_k <= btr) and the slack rows
        double cw = 0;
        for (int k = 0; k < K1; ++k) {
            for (int j = 0; j < 8; ++j) {
                const int r = r_tr + 8 * k + j;
                double coef[3] = {0, 0, 0}, ct = 0;
                row(r, [&](int c, double v) {
                    if (c >= 9 * k + 6 && c < 9 * k + 9) coef[c - 9 * k - 6] = v;
                    else if (c == it + k) ct = v;
                    else need(false, at("trust-region row outside L_k, t_k", k, j));
                });
                for (int z = 0; z < 3; ++z)
                    need(coef[z] == (((j >> z) & 1) ? -1.0 : 1.0), at("trust-region row must have the +-1 pattern", k, j));
                if (k == 0 && j == 0) cw = ct;
                need(ct < 0 && close(ct, cw, std::fabs(cw), 1e-12), at("one trust-region slack coefficient -1/omega", k, j));
                need(l[r] <= -INF, at("trust-region rows have no lower bound", k, j));
                put(S::BTR + j, k, u[r]);
            }
            const int r = r_sl + k;
            int nz = 0;
            row(r, [&](int c, double v) { need(c == it + k && v == -1.0, at("slack row must be -t_k <= 0", k)); ++nz; });
            need(nz == 1 && u[r] == 0.0 && l[r] <= -INF, at("slack row must be -t_k <= 0", k));
        }
        for (int k = 0; k < K1; ++k)
            for (int i = 0; i < 9; ++i) put(S::QX + i, k, q[9 * k + i]);

        // ---- install: a parameter class for this problem, then the device arrays.
        // The other problems' accepted K / Sigma leave the live arrays (the class list changes), and
        // their dense A, Bu are written now from their own linearization points: a later getter or
        // export must not rerun k_lin_knots, which would rebuild problem b's stage record from the
        // synthetic starting point below.  Problem b's dense A, Bu are the loaded ones.  A later
        // cmpc_linearize re-linearizes every problem at its stored point, b included.
        materialize_accepted_ks(h);
        ensure_dense(h);
        {
            // an identical class is reused, so repeated loads do not grow the class list
            int32_t cid = -1;
            for (size_t i = 0; i < h->hparams.size() && cid < 0; ++i)
                if (std::memcmp(&h->hparams[i], &prm, sizeof(prm)) == 0) cid = (int32_t)i;
            if (cid < 0) {
                std::vector<cmpc_params> cls = h->hparams;
                cls.push_back(prm);
                const int rc = cmpc_set_params(h, (int)cls.size(), cls.data());
                need(rc == 0, "cmpc_set_params: " + h->err);
                cid = (int32_t)cls.size() - 1;
            }
            HIPCHK(hipMemcpyAsync((char *)h->class_id + (size_t)b * 4, &cid, 4, hipMemcpyHostToDevice, h->stream));
        }
        // X̄: the boundary states at knots 0 and N (the QP reads no other knot of it); starting point
        // x_0 on every knot, zero controls
        std::vector<double> xl((size_t)K1 * 9), ul((size_t)N * NU, 0.0);
        for (int k = 0; k < K1; ++k)
            for (int i = 0; i < 9; ++i) xl[(size_t)k * 9 + i] = xb[i];
        std::vector<double> xbv = xl;
        for (int i = 0; i < 9; ++i) xbv[(size_t)N * 9 + i] = xb[(size_t)N * 9 + i];
        const size_t e = h->esz();
        auto up = [&](void *base, size_t off_elems, const std::vector<double> &v) {
            if (e == 8) to_dev<double>(h, (char *)base + off_elems * 8, v.data(), v.size());
            else to_dev<float>(h, (char *)base + off_elems * 4, v.data(), v.size());
        };
        up(h->stage, (size_t)b * SIZE * KPC, st);
        up(h->Xbar, (size_t)b * K1 * 9, xbv);
        up(h->Xlin, (size_t)b * K1 * 9, xl);
        up(h->Ulin, (size_t)b * N * NU, ul);
        up(h->cw, (size_t)b, std::vector<double>{cw});
        {   // element e of (b, k) at e * LS + b * N + k
            const size_t LS = (size_t)h->max_batch * N;
            std::vector<double> tmp(N);
            for (int el = 0; el < 81; ++el) {
                std::copy(&Aem[(size_t)el * N], &Aem[(size_t)el * N] + N, tmp.begin());
                up(h->A, el * LS + (size_t)b * N, tmp);
            }
            for (int el = 0; el < 9 * NU; ++el) {
                std::copy(&Bem[(size_t)el * N], &Bem[(size_t)el * N] + N, tmp.begin());
                up(h->Bu, el * LS + (size_t)b * N, tmp);
            }
            h->lin_dense = true;
        }
        HIPCHK(hipMemcpyAsync((char *)h->logic + (size_t)b * N * NC, logic.data(), logic.size(), hipMemcpyHostToDevice,
                              h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
    });
}
