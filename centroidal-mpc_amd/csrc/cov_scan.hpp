// Covariance scan of one problem (shared by k_cov_scan, linearize_lane.hip, and the QP kernel,
// whose workgroups run the scans of a deterministic batch once their own QP has finished; see
// cmpc_api.cpp launch_phase).
#pragma once
#include "common.hpp"

namespace cmpc {

// Covariance scan (src/centroidal_model.py:234-238, 266, 284), one wave per problem:
// Sigma_{k+1} = Acl_k Sigma_k Acl_k' + Qw_k from the per-knot helpers of k_lin_knots.  The
// per-step blocks stream through LDS in double-buffered chunks of KS steps (each chunk's loads
// issued a chunk ahead inside one loop iteration); fp64 keeps Sigma in the matrix-core
// accumulator layout for the whole scan (see linearize.hip).
constexpr int SKS = 4;
constexpr int SCAN_CH = 2 * SKS * 81;
constexpr int SCAN_LDS = 2 * SCAN_CH + 2 * 81;   // LDS elements of one scan: chunk buffers, S, Tm

// Problem b's scan on the calling wave (lanes 0..63); lds: SCAN_LDS elements of shared memory.
template <typename T, int ROBOT, typename LP> __device__ __forceinline__ void cov_scan_problem(const DevBuf<T> &d, int b, LP lds) {
    constexpr int CH = SCAN_CH;
    constexpr int PL = (CH + WAVE - 1) / WAVE;
    const LP buf = lds, S = lds + 2 * CH, Tm = lds + 2 * CH + 81;
    const int lane = threadIdx.x & (WAVE - 1), N = d.N;
    const T *Acl = d.Acl + (size_t)b * N, *Qw = d.Qw + (size_t)b * N;   // element-major (DevBuf::LS)
    T reg[PL];
    auto issue = [&](int c) {
#pragma unroll
        for (int r = 0; r < PL; ++r) {
            const int e = min(lane + r * WAVE, CH - 1), blk = e / 81, w = e % 81;
            const int k = min(c * SKS + blk % SKS, N - 1);
            reg[r] = (blk < SKS ? Acl : Qw)[(size_t)w * d.LS + k];
        }
    };
    auto land = [&](int c) {
        const LP dst = buf + (c & 1) * CH;
#pragma unroll
        for (int r = 0; r < PL; ++r)
            if (lane + r * WAVE < CH) dst[lane + r * WAVE] = reg[r];
    };
    for (int e = lane; e < 81; e += WAVE) {
        S[e] = T(0);
        d.Sig[((size_t)b * (N + 1)) * 81 + e] = T(0);
    }
    issue(0);
    land(0);
    wave_sync();
    typedef double v4d __attribute__((ext_vector_type(4)));
    [[maybe_unused]] v4d Sreg = {0.0, 0.0, 0.0, 0.0};
    const int r16 = lane & 15, q4 = lane >> 4;
    for (int c = 0; c * SKS < N; ++c) {
        issue(c + 1);
        const LP cb = buf + (c & 1) * CH;
        for (int q = 0; q < SKS; ++q) {
            const int k = c * SKS + q;
            if (k >= N) break;
            const LP Ac = cb + q * 81, Q = cb + (SKS + q) * 81;
            if constexpr (sizeof(T) == 8) {
                double av[3];   // Acl[l & 15][4 kb + (l >> 4)] (zero outside 9 x 9)
#pragma unroll
                for (int kb = 0; kb < 3; ++kb) {
                    const int mm = 4 * kb + q4;
                    av[kb] = (r16 < 9 && mm < 9) ? Ac[(r16 < 9 ? r16 : 0) * 9 + (mm < 9 ? mm : 0)] : 0.0;
                }
                v4d qw;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = q4 + 4 * r;
                    qw[r] = (i < 9 && r16 < 9) ? Q[(i < 9 ? i : 0) * 9 + (r16 < 9 ? r16 : 0)] : 0.0;
                }
                v4d Y = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int kb = 0; kb < 3; ++kb) Y = __builtin_amdgcn_mfma_f64_16x16x4f64(Sreg[kb], av[kb], Y, 0, 0, 0);
                Sreg = qw;
#pragma unroll
                for (int kb = 0; kb < 3; ++kb) Sreg = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kb], Y[kb], Sreg, 0, 0, 0);
                T *so = d.Sig + ((size_t)b * (N + 1) + k + 1) * 81;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = q4 + 4 * r;
                    if (i < 9 && r16 < 9) so[i * 9 + r16] = Sreg[r];
                }
                continue;
            }
            for (int e = lane; e < 81; e += WAVE) {     // Tm = Acl S
                const int i = e / 9, j = e % 9;
                T acc = T(0);
#pragma unroll
                for (int mm = 0; mm < 9; ++mm) acc = fma(Ac[i * 9 + mm], S[mm * 9 + j], acc);
                Tm[e] = acc;
            }
            wave_sync();
            T out[2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {   // Tm Acl' + Qw
                const int e = min(lane + r * WAVE, 80), i = e / 9, j = e % 9;
                T acc = Q[e];
#pragma unroll
                for (int mm = 0; mm < 9; ++mm) acc = fma(Tm[i * 9 + mm], Ac[j * 9 + mm], acc);
                out[r] = acc;
            }
            wave_sync();
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int e = lane + r * WAVE;
                if (e < 81) {
                    S[e] = out[r];
                    d.Sig[((size_t)b * (N + 1) + k + 1) * 81 + e] = out[r];
                }
            }
            wave_sync();
        }
        land(c + 1);
        wave_sync();
    }
}

}  // namespace cmpc
