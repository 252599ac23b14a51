// Partitioned block-tridiagonal factorization and solves of the dual Schur system for
// four-wave QP workgroups (NTT = 256: small per-GPU batches, one problem per CU).
//
// The two-ended recurrence (tw_factor_ends) runs two chains of NB / 2 dependent 9x9 steps; with
// one problem per CU, four waves are available.  Three separator blocks s0 < s1 < s2 split the
// N + 2 blocks into four chunks, one chain per wave, all running at once:
//   wave 0  top end      blocks 0 .. s0-1, top-down      (as tw_factor_ends' top)
//   wave 1  interior     blocks s0+1 .. s1-1, top-down, carrying the fill coupling to s0
//   wave 2  interior     blocks s1+1 .. s2-1, top-down, carrying the fill coupling to s1
//   wave 3  bottom end   blocks NB-1 .. s2+1, bottom-up  (as tw_factor_ends' bottom)
// An interior chain over [a, b] with left separator L = a - 1 and right separator R = b + 1
// eliminates block j with the standard step (I_j = (S_jj - X_j S_{j-1,j})^-1, X_{j+1} =
// S_{j+1,j} I_j) and also carries G_j = S~_{L,j}, the coupling to L created by the elimination:
//   G_a = S_{L,a};  H_j = G_j I_j;  G_{j+1} = -H_j S_{j,j+1};  S~_LL -= H_j G_j';  b~_L -= H_j y_j
// which never feeds back into the chain (the fill runs beside it on the same wave).  At its end
// each chain hands its separators their Schur-complement terms: the X (top-down) or Y
// (bottom-up) term of the block it stops next to, and (interior) the accumulated fill term and
// the coupling S~_{L,R} = G_{b+1}.  The three separators then form a 3-block tridiagonal system,
// factored and solved by wave 0 (pt_reduced), and the back substitution runs per chunk again:
//   x_j = I_j y_j - H_j' x_L - X_{j+1}' x_{j+1}   (interior; the first two terms for all blocks
//   at once, pt_solve_local, then one 9-term product per sequential step, pt_solve_back).
// For NB = 102 the longest chain has 27 steps against the two-ended recurrence's 51.
//
// Storage (workspace): Sd[j] I_j packed (separators: the reduced factors' inverses); So[j] the
// X / Y factors as in tw_factor_ends (X_j at So[j-1] top-down, Y_j at So[j] bottom-up, the
// separators' X / Y terms included); Sh[j] H_j (interior blocks); Sx separator scratch (below).
#pragma once
// (included by qp_ipm.hip inside namespace cmpc, after the two-ended recurrence's helpers)

// Separator scratch slots of 81 (Ws::Sx): the Schur-complement terms of separator c from the chain
// above (dSa, packed 45) and below (dSb, packed 45), the couplings S~_{s0,s1}, S~_{s1,s2} (rows:
// the upper separator), and the reduced factors X^_1, X^_2.
constexpr int PT_DSA = 0, PT_DSB = 3, PT_CPL = 6, PT_XH = 8, PT_SX_SLOTS = 10;
// LDS scratch of one wave: tw_step_sym's A | P | Xb | Ob | Dd | Dn (TW_SCRATCH), then G | H
constexpr int PT_SCRATCH = TW_SCRATCH + 2 * 88;
// Chunk lengths: an interior step costs more than an end step (its fill products: measured on
// trot N=100 x 128 with the fp64 matrix-core fill, 5.4k against 4.0k cycles; fp32, VALU fill,
// ~1.6x), so the ends get the larger share of the non-separator blocks: le = r li with
// 2 le + 2 li = NB - 3, r = 1.35 (fp64) / 1.6 (fp32).
template <typename T> __device__ __forceinline__ void pt_seps(int NB, Seps &s) {
    const int le = sizeof(T) == 8 ? (NB - 3) * 135 / 470 : (NB - 3) * 8 / 26, rem = NB - 3 - 2 * le, li = rem / 2;
    s[0] = le;
    s[1] = s[0] + 1 + li;
    s[2] = s[1] + 1 + (rem - li);
}

// X = Op' P (81, two per lane), stored to Xout; dS = X Op (upper triangle, packed into dSout);
// with vb, db = X y_jy (lanes 0..8).  The separator terms of a chain's end (Op = S_{b,R}, or the
// bottom end's transposed landing, P = the last inverse).
template <typename T>
__device__ __forceinline__ void pt_contrib(const LdsT<T> *Op, const LdsT<T> *P, LdsT<T> *Xb, GlbT<T> *Xout, GlbT<T> *dSout,
                                           const LdsT<T> *vb, int jy, LdsT<T> *db) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int e = l + 64 * q < 81 ? l + 64 * q : 80, i = e / 9, c = e % 9;
        T s = T(0);
#pragma unroll
        for (int m = 0; m < 9; ++m) s = fma(Op[m * 9 + i], P[m * 9 + c], s);
        Xb[e] = s;
        if (l + 64 * q < 81) Xout[e] = s;
    }
    wave_sync();
    if (l < 45) {
        int r = l, i = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {   // upper-triangle element l -> (i, j)
            const bool past = r >= 9 - k && i == k;
            r = past ? r - (9 - k) : r;
            i = past ? k + 1 : i;
        }
        const int j = i + r;
        T s = T(0);
#pragma unroll
        for (int m = 0; m < 9; ++m) s = fma(Xb[i * 9 + m], Op[m * 9 + j], s);
        dSout[j * (j + 1) / 2 + i] = s;   // packed lower (row j >= column i)
    }
    if (vb && l < 9) db[l] = dot9(Xb + l * 9, vb + jy * 9);
    wave_sync();
}

// One chain per wave (see the file comment), the predictor's forward elimination fused in (vb).
// sbv: separator right-hand-side terms, [c][0] from above, [c][1] from below (9 each).
template <typename T>
__device__ __attribute__((noinline)) void pt_factor_chains(T *Sd_, T *So_, T *Sh_, T *Sx_, int NB, Seps sp, LdsT<T> *shw, LdsT<T> *vb,
                                 LdsT<T> *sbv) {
    GlbT<T> *Sd = (GlbT<T> *)Sd_, *So = (GlbT<T> *)So_, *Sh = (GlbT<T> *)Sh_, *Sx = (GlbT<T> *)Sx_;
    constexpr int L = 64, NE = 2;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const bool bottom = w == 3, interior = w == 1 || w == 2;
    LdsT<T> *A = shw, *P = A + 88, *Xb = A + 176, *Ob = A + 264, *Dd = A + 352, *Dn = A + 368, *G = A + TW_SCRATCH,
            *H = G + 88;
    const int j0 = w == 0 ? 0 : bottom ? NB - 1 : sp[w - 1] + 1;
    const int dj = bottom ? -1 : 1;
    const int nstep = w == 0 ? sp[0] : bottom ? NB - 1 - sp[2] : sp[w] - sp[w - 1] - 1;
    int e[NE], et[NE], ep[NE], ec[NE];
    T em[NE];
#pragma unroll
    for (int q = 0; q < NE; ++q) {
        e[q] = l + L * q < 81 ? l + L * q : 80;
        et[q] = bottom ? (e[q] % 9) * 9 + e[q] / 9 : e[q];
        ep[q] = pk9(e[q] / 9, e[q] % 9);
        const int c = cp9(e[q] / 9, e[q] % 9);
        ec[q] = c >= 0 ? c : 0;
        em[q] = c >= 0 ? T(1) : T(0);
    }
    // first diagonal block, and (interior) G_a = S_{L,a} = So[a - 1] (rows L, columns a)
    {
        const GlbT<T> *D0 = Sd + (size_t)j0 * 81;
        T v[NE], g[NE];
#pragma unroll
        for (int q = 0; q < NE; ++q) { v[q] = D0[ep[q]]; g[q] = interior ? So[(size_t)(j0 - 1) * 81 + ec[q]] * em[q] : T(0); }
#pragma unroll
        for (int q = 0; q < NE; ++q) { Dn[e[q]] = v[q]; if (interior) G[e[q]] = g[q]; }
    }
    // upper-triangle element of this lane for the fill accumulation S~_LL -= H G' (lanes 0..44)
    int ai = 0, aj = 0;
    {
        int r = l < 45 ? l : 44;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const bool past = r >= 9 - k && ai == k;
            r = past ? r - (9 - k) : r;
            ai = past ? k + 1 : ai;
        }
        aj = ai + r;
    }
    T accS = T(0), accb = T(0);
    typedef double v4d __attribute__((ext_vector_type(4)));
    const int r16 = l & 15, q4 = l >> 4;
    [[maybe_unused]] v4d Gt = {0.0, 0.0, 0.0, 0.0}, accS4 = {0.0, 0.0, 0.0, 0.0}, accB4 = {0.0, 0.0, 0.0, 0.0},
                         Ht = {0.0, 0.0, 0.0, 0.0}, Gn = {0.0, 0.0, 0.0, 0.0};
    [[maybe_unused]] const v4d zero4 = {0.0, 0.0, 0.0, 0.0};
    [[maybe_unused]] double oa[3] = {0.0, 0.0, 0.0}, yb[3] = {0.0, 0.0, 0.0};   // pipelined fill operands
    if constexpr (sizeof(T) == 8) {
        if (interior) {   // -G_a' in the accumulator layout: lane l holds -G_a[l & 15][(l >> 4) + 4 r]
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int c = q4 + 4 * r, cp = (r16 < 9 && c < 9) ? cp9(r16, c) : -1;
                Gt[r] = cp >= 0 ? -double(So[(size_t)(j0 - 1) * 81 + cp]) : 0.0;
            }
        }
    }
    wave_sync();
    for (int s = 0, j = j0; s < nstep; ++s, j += dj) {
        // raw blocks of the next step, or (last step) the coupling to the separator that follows
        const bool last = s + 1 == nstep;
        const int jn = last ? j : j + dj;
        const GlbT<T> *On = So + (size_t)(bottom ? (last ? j - 1 : jn) : (last ? j : jn - 1)) * 81, *Dnx = Sd + (size_t)jn * 81;
        T pv[NE], nv[NE];
#pragma unroll
        for (int q = 0; q < NE; ++q) { pv[q] = On[ec[q]] * em[q]; nv[q] = Dnx[ep[q]]; }
        if (s == 0)
            tw_step_sym<T, L>(Dn, nullptr, nullptr, nullptr, Sd + (size_t)j * 81, A, P, Xb, Dd, vb, j, 0);
        else
            tw_step_sym<T, L>(Dn, Ob, P, So + (size_t)(bottom ? j : j - 1) * 81, Sd + (size_t)j * 81, A, P, Xb, Dd, vb, j,
                              j - dj);
#pragma unroll
        for (int q = 0; q < NE; ++q) { Ob[et[q]] = pv[q]; Dn[e[q]] = nv[q]; }
        wave_sync();
#ifndef PT_EXP
#define PT_EXP 0   // diagnostic builds: 1 = no fill at all (timing only), 2 = no H stores, 3 = no fill MFMAs
#endif
        if (interior && PT_EXP != 1) {
            // H_j = G_j I_j -> Sh[j]; S~_LL += H_j G_j' (subtracted at the reduced system); b~_L += H_j y_j;
            // G_{j+1} = -H_j S_{j,j+1} (Ob now holds S_{j,j+1}: the next step's coupling, or S_{b,R})
            if constexpr (sizeof(T) == 8) {
                // on the matrix cores, transposed so every product's result feeds the next one from
                // the accumulator layout (lane l: D[(l >> 4) + 4 r][l & 15] = B operand of k-slice r;
                // the D registers of M' are the A operand of M).  Gt holds -G' (the sign goes into
                // P's operand).  Software-pipelined over the blocks so the MFMAs run under the next
                // step's VALU recurrence: here, for block j - 1, S -= H G', b += H y and
                // -G_j' = Ob_{j-1}' H_{j-1}' (operands loaded last iteration), H_{j-1} stored; then
                // for block j, H_j' = -P (-G_j') is issued and left running.
                if (s > 0 && PT_EXP != 3) {
#pragma unroll
                    for (int kb = 0; kb < 3; ++kb) Gn = __builtin_amdgcn_mfma_f64_16x16x4f64(oa[kb], Ht[kb], kb ? Gn : zero4, 0, 0, 0);
#pragma unroll
                    for (int kb = 0; kb < 3; ++kb) {
                        accS4 = __builtin_amdgcn_mfma_f64_16x16x4f64(Ht[kb], Gt[kb], accS4, 0, 0, 0);   // -= H G'
                        accB4 = __builtin_amdgcn_mfma_f64_16x16x4f64(Ht[kb], yb[kb], accB4, 0, 0, 0);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int c = q4 + 4 * r;
                        if (r16 < 9 && c < 9 && PT_EXP != 2) Sh[(size_t)(j - dj) * 81 + r16 * 9 + c] = Ht[r];   // H_{j-1}[r16][c]
                    }
                    Gt = Gn;
                }
                double pa[3];
#pragma unroll
                for (int kb = 0; kb < 3; ++kb) {
                    const int k = 4 * kb + q4, kk = k < 9 ? k : 0, rr = r16 < 9 ? r16 : 0;
                    const bool ok = r16 < 9 && k < 9;
                    pa[kb] = ok ? -P[rr * 9 + kk] : 0.0;
                    oa[kb] = ok ? Ob[kk * 9 + rr] : 0.0;           // S_{j,j+1}' for the next -G'
                    yb[kb] = (vb && k < 9) ? vb[j * 9 + kk] : 0.0;  // y_j
                }
                if (PT_EXP != 3) {
                    Ht = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[0], Gt[0], zero4, 0, 0, 0);
                    Ht = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[1], Gt[1], Ht, 0, 0, 0);
                    Ht = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[2], Gt[2], Ht, 0, 0, 0);
                } else {
                    Ht[0] += pa[0]; Ht[1] += pa[1]; Ht[2] += pa[2]; Ht[3] += oa[0] + yb[0];
                }
            } else {
                T hv[NE];
#pragma unroll
                for (int q = 0; q < NE; ++q) {
                    const int i = e[q] / 9, c = e[q] % 9;
                    T s2 = T(0);
#pragma unroll
                    for (int m = 0; m < 9; ++m) s2 = fma(G[i * 9 + m], P[m * 9 + c], s2);
                    hv[q] = s2;
                }
#pragma unroll
                for (int q = 0; q < NE; ++q) {
                    H[e[q]] = hv[q];
                    if (l + L * q < 81) Sh[(size_t)j * 81 + e[q]] = hv[q];
                }
                wave_sync();
                {
                    T s2 = T(0);
#pragma unroll
                    for (int m = 0; m < 9; ++m) s2 = fma(H[ai * 9 + m], G[aj * 9 + m], s2);
                    accS += s2;
                }
                if (vb && l < 9) accb += dot9(H + l * 9, vb + j * 9);
                T gv[NE];
#pragma unroll
                for (int q = 0; q < NE; ++q) {
                    const int i = e[q] / 9, c = e[q] % 9;
                    T s2 = T(0);
#pragma unroll
                    for (int m = 0; m < 9; ++m) s2 = fma(H[i * 9 + m], Ob[m * 9 + c], s2);
                    gv[q] = -s2;
                }
                wave_sync();
#pragma unroll
                for (int q = 0; q < NE; ++q) G[e[q]] = gv[q];
                wave_sync();
            }
        }
    }
    // separator terms: the X (Y) term of the separator next to the chain's last block
    const int jl = j0 + dj * (nstep - 1);                  // last eliminated block
    const int c_ab = bottom ? 2 : w;                        // separator that follows the chain
    pt_contrib<T>(Ob, P, Xb, So + (size_t)(bottom ? jl - 1 : jl) * 81, Sx + (size_t)(bottom ? PT_DSB + 2 : PT_DSA + c_ab) * 81,
                  vb, jl, sbv + (c_ab * 2 + (bottom ? 1 : 0)) * 9);
    if (interior) {
        // the fill terms of the left separator L = s_{w-1} and the coupling S~_{L,R} = G_{b+1}
        if constexpr (sizeof(T) == 8) {
            // the pipeline's last stage for block b: its fill terms and -G_{b+1}' = Ob' H_b' (oa
            // holds S_{b,R}', loaded with the last block)
#pragma unroll
            for (int kb = 0; kb < 3; ++kb) {
                Gn = __builtin_amdgcn_mfma_f64_16x16x4f64(oa[kb], Ht[kb], kb ? Gn : zero4, 0, 0, 0);
                accS4 = __builtin_amdgcn_mfma_f64_16x16x4f64(Ht[kb], Gt[kb], accS4, 0, 0, 0);
                accB4 = __builtin_amdgcn_mfma_f64_16x16x4f64(Ht[kb], yb[kb], accB4, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = q4 + 4 * r;   // accumulator row
                if (i < 9 && r16 < 9) {
                    if (i >= r16) Sx[(size_t)(PT_DSB + w - 1) * 81 + i * (i + 1) / 2 + r16] = -accS4[r];
                    Sx[(size_t)(PT_CPL + w - 1) * 81 + r16 * 9 + i] = -Gn[r];   // G_{b+1}[r16][i]
                    if (vb && r16 == 0) sbv[((w - 1) * 2 + 1) * 9 + i] = accB4[r];
                    Sh[(size_t)jl * 81 + r16 * 9 + i] = Ht[r];   // H_b
                }
            }
        } else {
            if (l < 45) Sx[(size_t)(PT_DSB + w - 1) * 81 + aj * (aj + 1) / 2 + ai] = accS;
            if (vb && l < 9) sbv[((w - 1) * 2 + 1) * 9 + l] = accb;
#pragma unroll
            for (int q = 0; q < NE; ++q)
                if (l + L * q < 81) Sx[(size_t)(PT_CPL + w - 1) * 81 + e[q]] = G[e[q]];
        }
    }
}

// The 3-block separator system (wave 0): S^_cc = S_{s_c s_c} - dSa_c - dSb_c, S^_{c,c+1} = the
// interior chains' couplings; factored top-down (I^_c -> Sd[s_c], X^_c -> Sx) and, with the
// predictor's right-hand side (factor == true), solved; without factoring, solved with the stored
// factors (corrector / refinement).  The right-hand side of separator c is b_{s_c} minus its terms
// from above and below (sbv; the interior chains' fill terms for the solves come from hy).
template <typename T>
__device__ __attribute__((noinline)) void pt_reduced(T *Sd_, T *Sx_, Seps sp, LdsT<T> *shw, LdsT<T> *vb, const LdsT<T> *sbv, bool factor) {
    GlbT<T> *Sd = (GlbT<T> *)Sd_, *Sx = (GlbT<T> *)Sx_;
    const int l = threadIdx.x & 63;
    LdsT<T> *A = shw, *P = A + 88, *Xb = A + 176, *Ob = A + 264, *Dd = A + 352, *Dn = A + 368;
    // right-hand sides of the separators
    if (l < 27) {
        const int c = l / 9, i = l % 9;
        vb[sp[c] * 9 + i] -= sbv[(c * 2) * 9 + i] + sbv[(c * 2 + 1) * 9 + i];
    }
    wave_sync();
    if (factor) {
        for (int c = 0; c < 3; ++c) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int e = l + 64 * q < 81 ? l + 64 * q : 80, i = e / 9, jj = e % 9, pk = pk9(i, jj);
                Dn[e] = Sd[(size_t)sp[c] * 81 + pk] - Sx[(size_t)(PT_DSA + c) * 81 + pk] - Sx[(size_t)(PT_DSB + c) * 81 + pk];
                if (c > 0) Ob[e] = Sx[(size_t)(PT_CPL + c - 1) * 81 + e];   // S^_{c-1,c}
            }
            wave_sync();
            if (c == 0)
                tw_step_sym<T, 64>(Dn, nullptr, nullptr, nullptr, Sd + (size_t)sp[0] * 81, A, P, Xb, Dd, vb, sp[0], 0);
            else
                tw_step_sym<T, 64>(Dn, Ob, P, Sx + (size_t)(PT_XH + c - 1) * 81, Sd + (size_t)sp[c] * 81, A, P, Xb, Dd, vb,
                                   sp[c], sp[c - 1]);
        }
    } else {
        // forward: y^_c = b^_c - X^_c y^_{c-1}
        for (int c = 1; c < 3; ++c) {
            if (l < 9) {
                const GlbT<T> *X = Sx + (size_t)(PT_XH + c - 1) * 81 + l * 9;
                const LdsT<T> *yp = vb + sp[c - 1] * 9;
                T v = vb[sp[c] * 9 + l];
#pragma unroll
                for (int m = 0; m < 9; ++m) v = fma(-X[m], yp[m], v);
                vb[sp[c] * 9 + l] = v;
            }
            wave_sync();
        }
    }
    // back: x_2 = I^_2 y^_2;  x_c = I^_c y^_c - X^_{c+1}' x_{c+1}
    for (int c = 2; c >= 0; --c) {
        T v = T(0);
        if (l < 9) {
            const GlbT<T> *I = Sd + (size_t)sp[c] * 81;
            const LdsT<T> *y = vb + sp[c] * 9;
#pragma unroll
            for (int m = 0; m < 9; ++m) v = fma(I[pk9(l, m)], y[m], v);
            if (c < 2) {
                const GlbT<T> *X = Sx + (size_t)(PT_XH + c) * 81;
                const LdsT<T> *xn = vb + sp[c + 1] * 9;
#pragma unroll
                for (int m = 0; m < 9; ++m) v = fma(-X[m * 9 + l], xn[m], v);
            }
        }
        wave_sync();
        if (l < 9) vb[sp[c] * 9 + l] = v;
        wave_sync();
    }
    (void)Xb;
}

// Forward elimination of a right-hand side (vb) along the four chains (lanes 0..31 of each wave,
// one block ring per wave); the separators' X / Y terms into sbv[c][0] / sbv[2][1].
template <typename T> __device__ __attribute__((noinline)) void pt_solve_elim(const T *Xs, int NB, Seps sp, LdsT<T> *vb, LdsT<T> *ring, LdsT<T> *sbv) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l >= 32) return;
    const bool bottom = w == 3;
    const int lr = l < 9 ? l : 0;
    // block of step i: top-down j = j1 + i with X_j at So[j - 1]; bottom-up j = NB - 2 - i with Y_j at So[j].
    // The last step (i = n - 1) is the separator's term, written to sbv instead of vb.
    const int j1 = w == 0 ? 1 : bottom ? NB - 2 : sp[w - 1] + 2;
    const int n = w == 0 ? sp[0] : bottom ? NB - 1 - sp[2] : sp[w] - sp[w - 1] - 1;
    const int dj = bottom ? -1 : 1;
    LdsT<T> *sep = sbv + ((bottom ? 2 : w) * 2 + (bottom ? 1 : 0)) * 9;
    const GlbT<T> *Xg = (const GlbT<T> *)Xs;
    ChunkStream<T, KE> X{Xg + (size_t)(bottom ? j1 : j1 - 1) * 81, bottom ? -81L : 81L, n, ring, {}};
    X.issue(0);
    X.land(0);
    for (int c = 0; c * KE < n; ++c) {
        X.issue(c + 1);
        wave_sync();
        for (int q = 0; q < KE; ++q) {
            const int i = c * KE + q;
            if (i >= n) break;
            const int j = j1 + dj * i, jp = j - dj;
            if (l < 9) {
                const LdsT<T> *xr = X.blk(i) + lr * 9;
                const T s = dot9(xr, vb + jp * 9);
                if (i + 1 < n) vb[j * 9 + l] -= s;
                else sep[l] = s;
            }
            wave_sync();
        }
        X.land(c + 1);
    }
    wave_sync();
}

// fill terms of the interior chunks' left separators: hy[t] = (H_j y_j)_i for block j of chunk
// 1 or 2, row i (all threads), summed per separator into sbv[c][1] by wave 0 after a barrier
template <typename T, int NTT> __device__ __attribute__((noinline)) void pt_fill_rhs(const T *Sh_, Seps sp, const LdsT<T> *vb, LdsT<T> *hy) {
    const GlbT<T> *Sh = (const GlbT<T> *)Sh_;
    const int a = sp[0] + 1, n = sp[2] - a;   // blocks s0+1 .. s2-1 (the separator s1 between them gives 0)
    for (int t = threadIdx.x; t < 9 * n; t += NTT) {
        const int j = a + t / 9, i = t % 9;
        T s = T(0);
        if (j != sp[1]) {
            const GlbT<T> *Hr = Sh + (size_t)j * 81 + i * 9;
#pragma unroll
            for (int m = 0; m < 9; ++m) s = fma(Hr[m], vb[j * 9 + m], s);
        }
        hy[t] = s;
    }
}
template <typename T> __device__ void pt_fill_sum(Seps sp, const LdsT<T> *hy, LdsT<T> *sbv) {
    const int l = threadIdx.x & 63;
    if (l < 18) {
        const int c = l / 9, i = l % 9, a = sp[0] + 1;
        const int j0 = c == 0 ? a : sp[1] + 1, j1 = c == 0 ? sp[1] : sp[2];
        T s = T(0);
        for (int j = j0; j < j1; ++j) s += hy[(j - a) * 9 + i];
        sbv[(c * 2 + 1) * 9 + i] = s;
    }
    wave_sync();
}

// local back-substitution terms of every non-separator block (all threads):
// z_j = I_j y_j (- H_j' x_L for the interior chunks' blocks)
template <typename T, int NTT> __device__ __attribute__((noinline)) void pt_solve_local(const T *Ii, const T *Sh_, int NB, Seps sp, LdsT<T> *vb) {
    const GlbT<T> *Sh = (const GlbT<T> *)Sh_;
    for (int j = threadIdx.x; j < NB; j += NTT) {
        if (j == sp[0] || j == sp[1] || j == sp[2]) continue;
        const GlbT<T> *I = (const GlbT<T> *)Ii + (size_t)j * 81;   // packed
        T iv[45], y[9], z[9];
#pragma unroll
        for (int p = 0; p < 45; ++p) iv[p] = I[p];
#pragma unroll
        for (int i = 0; i < 9; ++i) y[i] = vb[j * 9 + i];
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            T a = iv[pk9(i, 0)] * y[0];
#pragma unroll
            for (int q = 1; q < 9; ++q) a = fma(iv[pk9(i, q)], y[q], a);
            z[i] = a;
        }
        const int L = (j > sp[0] && j < sp[1]) ? sp[0] : (j > sp[1] && j < sp[2]) ? sp[1] : -1;
        if (L >= 0) {
            T xl[9];
#pragma unroll
            for (int m = 0; m < 9; ++m) xl[m] = vb[L * 9 + m];
            const GlbT<T> *Hj = Sh + (size_t)j * 81;
#pragma unroll
            for (int m = 0; m < 9; ++m) {
                T hm[9];
#pragma unroll
                for (int i = 0; i < 9; ++i) hm[i] = Hj[m * 9 + i];
#pragma unroll
                for (int i = 0; i < 9; ++i) z[i] = fma(-hm[i], xl[m], z[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) vb[j * 9 + i] = z[i];
    }
}

// back substitution along the chains (lanes 0..31 of each wave): top-down chunks from their last
// block up, x_j = z_j - X_{j+1}' x_{j+1} (X_{j+1} at So[j]); the bottom chunk down from s2 + 1,
// x_j = z_j - Y_{j-1}' x_{j-1} (Y_{j-1} at So[j-1])
template <typename T> __device__ __attribute__((noinline)) void pt_solve_back(const T *Xs, int NB, Seps sp, LdsT<T> *vb, LdsT<T> *ring) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l >= 32) return;
    const bool bottom = w == 3;
    const int lr = l < 9 ? l : 0;
    const int jb = bottom ? sp[2] + 1 : sp[w] - 1;   // first block of the sweep
    const int n = w == 0 ? sp[0] : bottom ? NB - 1 - sp[2] : sp[w] - sp[w - 1] - 1;
    ChunkStream<T, KE> X{(const GlbT<T> *)Xs + (size_t)(bottom ? jb - 1 : jb) * 81, bottom ? 81L : -81L, n, ring, {}};
    X.issue(0);
    X.land(0);
    for (int c = 0; c * KE < n; ++c) {
        X.issue(c + 1);
        wave_sync();
        for (int q = 0; q < KE; ++q) {
            const int i = c * KE + q;
            if (i >= n) break;
            const int j = bottom ? jb + i : jb - i, jn = bottom ? j - 1 : j + 1;
            T v = T(0);
            if (l < 9) {
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
            if (l < 9) vb[j * 9 + l] = v;
            wave_sync();
        }
        X.land(c + 1);
    }
    wave_sync();
}

