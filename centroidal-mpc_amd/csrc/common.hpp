// Shared definitions for the cmpc HIP kernels (gfx950 / CDNA4).
//
// Robot configurations are compile-time (template ROBOT): solo12 has 4 point contacts with
// 3-D forces; TALOS has 2 contacts with u_i = [cop_x, cop_y, fx, fy, fz, tau_z]
// (reference src/centroidal_model.py:189-212, src/optimizer.py:37-74).  nu = 12 for both.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc.h"

namespace cmpc {

constexpr int NX = 9;
constexpr int NU = 12;
constexpr int IPM_NT = 64;    // threads per QP workgroup (one problem, one wave)
constexpr int WAVE = 64;

template <int ROBOT> struct Robot;
template <> struct Robot<0> {             // solo12
    static constexpr int NC = 4, NUPC = 3, FO = 0, COP = 0;
};
template <> struct Robot<1> {             // TALOS
    static constexpr int NC = 2, NUPC = 6, FO = 2, COP = 1;
};

// Inequality rows per knot: TR L1 (8) | TR slack (1) | friction 4 per contact | CoP 4 per contact
template <int ROBOT> struct Rows {
    static constexpr int NC = Robot<ROBOT>::NC;
    static constexpr int TR = 0, SL = 8, FR = 9, CP = 9 + 4 * NC;
    static constexpr int NI = 9 + 4 * NC * (1 + Robot<ROBOT>::COP);   // 25 for both robots
};

// Stage record (assembled structured QP, one per knot), see assemble.hip.
template <int ROBOT> struct Stage {
    static constexpr int NC = Robot<ROBOT>::NC;
    static constexpr int R = 0, QX = 9, BTR = 18, W = 26, CON = 32, CS = 32;
    // per-contact slot offsets
    static constexpr int ALPHA = 0, LEVER = 1, G = 4, H = 16, BCOP = 20, BTAU = 26;
    static constexpr int SIZE = CON + CS * NC;
};

// Parameters of one problem class, in the compute type.
template <typename T> struct DevParams {
    T mass, gravity, dt, mu, xi;
    T foot_range[4];
    T Wx[9], Wu[12], Q[81], R[144], cov_w[144], cov_eta[81];
    int stochastic, tracking;
    double tr_radius0, omega0, omega_max, rho0, rho1, beta_succ, beta_fail, gamma_fail, conv_thr;
    int max_iterations;
};

// Per-problem SCP state (always double: it mirrors the reference's Python floats).
struct ScpState {
    double weight, radius;
    double tr_norm, rho;
    int iter, status, success, n_accepted;
    int qp_status, qp_iters, decision, active;
    double conv;   // convergence measure of the last accepted iteration (GuSTO mode)
    int keep, pad;   // this iteration was accepted: k_keep_accepted copies its solution/gains
};

// Device buffers of one handle.
template <typename T> struct DevBuf {
    int B, N;
    const int32_t *class_id;
    const DevParams<T> *params;
    const uint8_t *logic;    // (B,N,NC)
    const T *pos, *rot;      // (B,N,NC,3) (B,N,NC,9)
    const T *Xbar, *Ubar;    // (B,N+1,9) (B,N,NU) warm start: tracking reference, boundary states
    T *Xlin, *Ulin;          // (B,N+1,9) (B,N,NU) linearization point (= warm start in reference mode)
    int scp_mode;            // CMPC_SCP_MODE_*
    int copy_ks;             // k_keep_accepted also copies K, Sigma (see cmpc_handle_::ks_live)
    // linearization.  The per-knot arrays are element-major: element e of knot kn = b * N + k at
    // X[e * LS + kn] (LS = max_batch * N), so the knot-per-lane kernels read and write them
    // coalesced; the C ABI getters transpose to the knot-major layouts of include/cmpc.h.
    T *f, *A, *Bu, *C, *K;          // elements 9 | 81 | 9 * NU | 9 * 3NC | NU * 9 (row-major per knot)
    T *Sig;                         // (B, N+1, 81) knot-major (written by the scan, one wave per problem)
    T *Acl, *Qw;                    // scan helpers, 81 elements each, element-major
    size_t LS;
    // assembled stage records (B,N+1,SIZE) and per-problem cw = -1/omega
    T *stage;
    T *cw;
    // QP solution / multipliers
    T *xs, *us, *ts;                // (B,N+1,9) (B,N,NU) (B,N+1)
    T *nus;                         // (B,N+2,9)
    T *lams;                        // (B,N+1,NI)
    int32_t *qp_status, *qp_iters;
    T *qp_merit;                    // (B) final merit (residual / tolerance; <= 1 when solved)
    int32_t *qp_nref;               // (B) refinement steps taken
    int32_t *qp_tail;               // (B) Newton steps run on the whole workgroup after a hand-over (k_qp_group)
    int32_t *qp_polish;             // (B) solution polishing: 1 accepted, -1 rejected, 0 not tried
    void *qp_state;                 // (B) Newton-loop state of a problem left for the tail launch (split QP)
    // IPM workspace
    T *ws;
    size_t ws_stride;               // elements per problem
    // SCP
    ScpState *scp;
    unsigned long long *stamps;     // (B,16) per-phase cycle counters (diagnostic builds only)
    unsigned *scan_ctr;             // k_qp_ipm: covariance-scan job counter (nullptr: no scans)
    T *Xacc, *Uacc, *Kacc, *Sacc;   // accepted solution (B,N+1,9) (B,N,NU) (108,LS) (B,N+1,81)
    // per-iteration records (B, log_cap) and accepted-iterate history: slot j of X (B,N+1,9),
    // U (B,N,NU), K (108,LS) element-major, Sigma (B,N+1,81), hist_cap slots (K, Sigma: GuSTO
    // mode only; nullptr when not allocated)
    cmpc_iter_record *hlog;
    int log_cap, hist_cap;
    T *hX, *hU, *hK, *hS;
};

// ---------------------------------------------------------------- knot-minor layouts
// Per-knot records (stage records, IPM workspace) are stored field-major, knot-minor: field f
// of knot k at p[f * KPC + k].  Thread k <-> knot k, so every field load or store of a wave is
// one contiguous 512-B (fp64) access instead of 64 separate lines.  The pitch is a compile-time
// constant covering every supported horizon (N + 2 <= 257 Schur blocks), so all field offsets
// fold into immediates; the unused tail of each field row is never touched (no HBM traffic).
constexpr int KPC = 264;

// strided view of one knot's record: element i at p[i * KPC]
template <typename T> struct SV {
    T *p;
    __device__ __forceinline__ T &operator[](int i) const { return p[i * KPC]; }
    __device__ __forceinline__ SV operator+(int n) const { return SV{p + n * KPC}; }
};

// ---------------------------------------------------------------- small helpers
template <typename T> __device__ __forceinline__ T sq(T a) { return a * a; }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T> __device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
template <typename T> __device__ __forceinline__ T wave_min(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
template <typename T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Barrier of a thread group of G threads inside a workgroup of WG threads (G, WG multiples of 64,
// G | WG, groups aligned to G): the workgroup barrier when the group is the workgroup; a wave-level
// barrier with workgroup-scope fences (the same waits on LDS and global memory as __syncthreads,
// without the s_barrier the other waves of the workgroup are not part of) when it is one wave of
// a larger workgroup (k_qp_group: one problem per wave until the last one is handed over).
template <int G, int WG> __device__ __forceinline__ void gsync() {
    static_assert(G == WG || G == 64, "a group is the workgroup or one of its waves");
    if constexpr (G == WG) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
}

// Reductions over a group of NT threads (multiple of 64; the workgroup, or one wave of a larger one,
// see gsync).  `red` is LDS scratch of at least NT/64 * NV elements, private to the group.  All
// threads of the group receive the result.
template <typename T, int NT, int NV, int OP, int WG = NT>   // OP: 0 sum, 1 max, 2 min
__device__ __forceinline__ void block_reduce(T (&v)[NV], T *red) {
    const int lane = threadIdx.x & 63, wid = (threadIdx.x & (NT - 1)) >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        T a = v[i];
        a = OP == 0 ? wave_sum(a) : OP == 1 ? wave_max(a) : wave_min(a);
        if (lane == 0) red[wid * NV + i] = a;
    }
    gsync<NT, WG>();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        T a = red[i];
#pragma unroll
        for (int w = 1; w < NT / 64; ++w) {
            T b = red[w * NV + i];
            a = OP == 0 ? a + b : OP == 1 ? fmax(a, b) : fmin(a, b);
        }
        v[i] = a;
    }
    gsync<NT, WG>();
}

// skew(v) * x  == v cross x
template <typename A, typename B, typename T> __device__ __forceinline__ void cross3(const A &a, const B &b, T *o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// (shared by k_lin_knots, which writes the dense B, and k_accept's linear prediction)
// rows 3..8 of the per-contact input matrix B_c (6 x NUPC) of contact c
template <typename T, int ROBOT> struct ContactB {
    static constexpr int NUPC = Robot<ROBOT>::NUPC;
    T b[6][NUPC];
};

template <typename T, int ROBOT>
__device__ __forceinline__ void contact_B(T dta, const T (&lev)[3], const T *f, const T *Rc, ContactB<T, ROBOT> &B) {
    constexpr int NUPC = Robot<ROBOT>::NUPC, FO = Robot<ROBOT>::FO;
    const T sk[3][3] = {{T(0), -lev[2], lev[1]}, {lev[2], T(0), -lev[0]}, {-lev[1], lev[0], T(0)}};
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int q = 0; q < NUPC; ++q) B.b[a][q] = T(0);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        B.b[q][FO + q] = dta;
#pragma unroll
        for (int r = 0; r < 3; ++r) B.b[3 + r][FO + q] = dta * sk[r][q];
    }
    if (ROBOT == 1) {
        const T fs[3][3] = {{T(0), -f[2], f[1]}, {f[2], T(0), -f[0]}, {-f[1], f[0], T(0)}};
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int q = 0; q < 2; ++q)   // d/dcop [(R2 cop) x f] = -[f]x R[:, q]
                B.b[3 + r][q] = -dta * (fs[r][0] * Rc[0 * 3 + q] + fs[r][1] * Rc[1 * 3 + q] + fs[r][2] * Rc[2 * 3 + q]);
            B.b[3 + r][5] = dta * Rc[r * 3 + 2];   // tau
        }
    }
}

}  // namespace cmpc
