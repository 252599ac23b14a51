// Host-side state of a libcmpc handle and the helpers shared by the C ABI translation units
// (cmpc_api.cpp: lifecycle, kernels, export; comm.cpp: RCCL batch split).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <string>
#include <vector>

#include "cmpc.h"
#include "common.hpp"

namespace cmpc_host {

struct Fail {
    int code;
    std::string msg;
};

}  // namespace cmpc_host

#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) throw cmpc_host::Fail{-3, std::string(#x) + ": " + hipGetErrorString(e_)}; \
    } while (0)

struct cmpc_handle_s {
    int device = 0, robot = 0, N = 0, max_batch = 0, prec = 0, B = 0, n_classes = 0;
    int NC = 4, NI = 25, SS = 160;
    int n_cu = 256;   // compute units of the device (QP waves-per-problem choice)
    hipStream_t stream = nullptr;
    // Covariance scan beside the QP (deterministic batches inside cmpc_scp_iterate; see
    // cmpc_api.cpp launch_phase): a low-priority side stream, the event after the assembly that
    // starts it, and the event after the scan that the main stream waits for behind the QP.
    hipStream_t side = nullptr;
    hipEvent_t ev_asm = nullptr, ev_scan = nullptr;
    bool scan_deferred = false, scan_pending = false;
    int scan_oa = 0;            // only_active of the deferred scan (settle_all)
    void *scan_ctr = nullptr;   // job counter of the scans run by the QP kernel's workgroups
    void *qp_order = nullptr;   // (max_batch + 8) problem slots of the grouped QP kernel (k_qp_order)
    hipEvent_t ev[5] = {};
    bool timed = false;
    // accumulated timing: one 5-event record per cmpc_scp_iterate since cmpc_timing_reset
    std::vector<std::array<hipEvent_t, 5>> ev_pool;
    size_t ev_used = 0;
    bool accumulate = false;
    std::string err;
    cmpc_qp_settings qs{};
    std::vector<cmpc_params> hparams;
    std::vector<void *> allocs;
    size_t ws_stride = 0;
    // device pointers (typed by precision at use)
    void *class_id = nullptr, *params = nullptr, *logic = nullptr, *pos = nullptr, *rot = nullptr, *Xbar = nullptr,
         *Ubar = nullptr, *f = nullptr, *A = nullptr, *Bu = nullptr, *C = nullptr, *K = nullptr, *Sig = nullptr,
         *Acl = nullptr, *Qw = nullptr, *stage = nullptr, *cw = nullptr, *xs = nullptr, *us = nullptr, *ts = nullptr,
         *nus = nullptr, *lams = nullptr, *qp_status = nullptr, *qp_iters = nullptr, *qp_merit = nullptr,
         *qp_nref = nullptr, *qp_tail = nullptr, *qp_polish = nullptr, *qp_state = nullptr, *qp_split = nullptr, *ws = nullptr, *scp = nullptr,
         *Xacc = nullptr, *Uacc = nullptr, *Kacc = nullptr, *Sacc = nullptr, *stamps = nullptr, *Xlin = nullptr,
         *Ulin = nullptr;
    int scp_mode = CMPC_SCP_MODE_REFERENCE;
    // Reference mode never moves the linearization point (quirk Q1), so every SCP iteration
    // recomputes bit-identical K and Sigma from the same inputs: an accepted iteration's gains and
    // covariances are the live arrays, and k_keep_accepted copies only X and U (the reference
    // keeps references to that iteration's arrays, no copy).  Cleared (after copying the live
    // arrays into Kacc / Sacc) when the mode turns to GuSTO or the contact plans change; set
    // again by the next upload.
    bool ks_live = true;
    bool lin_lane = true;   // knot-per-lane linearization (diagonal R); else k_linearize
    bool lin_lane_done = false;   // the last linearization came from k_lin_knots (stage partly written)
    bool lin_dense = false;       // the dense A, Bu, C arrays hold the last linearization (see ensure_dense)
    // RCCL communicator of the batch split (comm.cpp); nullptr until cmpc_comm_init
    void *comm = nullptr;
    int comm_rank = 0, comm_size = 1;
    void (*comm_free)(void *) = nullptr;   // set by cmpc_comm_init, called by cmpc_destroy
    int plans_B = 0;   // problems whose contact plans were built on the device
    // per-iteration records and the accepted-iterate history (ensure_history): capacities in
    // iterations per problem; the K / Sigma slots exist only once GuSTO mode ran
    void *hlog = nullptr, *hX = nullptr, *hU = nullptr, *hK = nullptr, *hS = nullptr;
    int log_cap = 0, hist_cap = 0, hks_cap = 0;
    // K / Sigma prefetch of the reference-mode loop (cmpc_prefetch_ks): pinned host targets, a copy
    // stream, the staging of the transposed (or widened) arrays, and what has been issued
    double *pf_K = nullptr, *pf_S = nullptr;
    hipStream_t copy = nullptr;
    hipEvent_t ev_pf_src = nullptr, ev_pfK = nullptr, ev_pfS = nullptr;
    void *pf_stage = nullptr;
    size_t pf_stage_bytes = 0;
    bool pf_armed = false, pfK_issued = false, pfS_issued = false;
    // grow-only device scratch of the host getters (knot-major staging copies)
    void *scratch = nullptr;
    size_t scratch_bytes = 0;

    size_t esz() const { return prec == CMPC_PREC_F64 ? 8 : 4; }
    void *dalloc(size_t bytes) {
        void *p = nullptr;
        HIPCHK(hipMalloc(&p, std::max<size_t>(bytes, 16)));
        HIPCHK(hipMemsetAsync(p, 0, std::max<size_t>(bytes, 16), stream));
        allocs.push_back(p);
        return p;
    }
    // replace a handle allocation by a zeroed one of `bytes` (old contents dropped)
    void regrow(void *&p, size_t bytes) {
        if (p) {
            HIPCHK(hipStreamSynchronize(stream));
            HIPCHK(hipFree(p));
            allocs.erase(std::find(allocs.begin(), allocs.end(), p));
            p = nullptr;
        }
        p = dalloc(bytes);
    }
    void *scratch_bytes_at_least(size_t bytes) {
        if (bytes > scratch_bytes) {
            if (scratch) {
                HIPCHK(hipStreamSynchronize(stream));
                HIPCHK(hipFree(scratch));
                scratch = nullptr;
                scratch_bytes = 0;
            }
            HIPCHK(hipMalloc(&scratch, bytes));
            scratch_bytes = bytes;
        }
        return scratch;
    }
    template <typename T> cmpc::DevBuf<T> buf() const {
        cmpc::DevBuf<T> d;
        d.B = B; d.N = N;
        d.class_id = (const int32_t *)class_id; d.params = (const cmpc::DevParams<T> *)params;
        d.logic = (const uint8_t *)logic; d.pos = (const T *)pos; d.rot = (const T *)rot;
        d.Xbar = (const T *)Xbar; d.Ubar = (const T *)Ubar;
        d.Xlin = (T *)Xlin; d.Ulin = (T *)Ulin; d.scp_mode = scp_mode; d.copy_ks = ks_live ? 0 : 1;
        d.f = (T *)f; d.A = (T *)A; d.Bu = (T *)Bu; d.C = (T *)C; d.K = (T *)K; d.Sig = (T *)Sig;
        d.Acl = (T *)Acl; d.Qw = (T *)Qw; d.stage = (T *)stage; d.cw = (T *)cw;
        d.LS = (size_t)max_batch * N;
        d.xs = (T *)xs; d.us = (T *)us; d.ts = (T *)ts; d.nus = (T *)nus; d.lams = (T *)lams;
        d.qp_status = (int32_t *)qp_status; d.qp_iters = (int32_t *)qp_iters;
        d.qp_merit = (T *)qp_merit; d.qp_nref = (int32_t *)qp_nref; d.qp_tail = (int32_t *)qp_tail; d.qp_polish = (int32_t *)qp_polish; d.qp_state = qp_state;
        d.ws = (T *)ws; d.ws_stride = ws_stride; d.scp = (cmpc::ScpState *)scp;
        d.Xacc = (T *)Xacc; d.Uacc = (T *)Uacc; d.Kacc = (T *)Kacc; d.Sacc = (T *)Sacc;
        d.stamps = (unsigned long long *)stamps;
        d.scan_ctr = nullptr;
        d.hlog = (cmpc_iter_record *)hlog; d.log_cap = log_cap; d.hist_cap = hist_cap;
        d.hX = (T *)hX; d.hU = (T *)hU;
        d.hK = hks_cap >= hist_cap ? (T *)hK : nullptr; d.hS = hks_cap >= hist_cap ? (T *)hS : nullptr;
        return d;
    }
};

namespace cmpc_host {

template <typename F> inline int guard(cmpc_handle h, F &&fn) {
    try {
        if (!h) return -1;
        HIPCHK(hipSetDevice(h->device));
        fn();
        h->err.clear();
        return 0;
    } catch (const Fail &f) {
        if (h) h->err = f.msg;
        return f.code;
    } catch (const std::exception &e) {
        if (h) h->err = e.what();
        return -9;
    }
}

inline void need(bool ok, const std::string &msg) {
    if (!ok) throw Fail{-2, msg};
}

template <typename T> inline void to_dev(cmpc_handle h, void *dst, const double *src, size_t n) {
    if (sizeof(T) == 8) {
        HIPCHK(hipMemcpyAsync(dst, src, n * 8, hipMemcpyHostToDevice, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
    } else {
        std::vector<T> tmp(n);
        for (size_t i = 0; i < n; ++i) tmp[i] = T(src[i]);
        HIPCHK(hipMemcpyAsync(dst, tmp.data(), n * sizeof(T), hipMemcpyHostToDevice, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
    }
}

template <typename T> inline void from_dev(cmpc_handle h, double *dst, const void *src, size_t n) {
    if (!dst) return;
    if (sizeof(T) == 8) {
        HIPCHK(hipMemcpyAsync(dst, src, n * 8, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
    } else {
        std::vector<T> tmp(n);
        HIPCHK(hipMemcpyAsync(tmp.data(), src, n * sizeof(T), hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        for (size_t i = 0; i < n; ++i) dst[i] = double(tmp[i]);
    }
}

inline void from_dev_raw(cmpc_handle h, void *dst, const void *src, size_t bytes) {
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
}

// cmpc_api.cpp: shared by the entry points of every translation unit
void settle_all(cmpc_handle h);              // run / join a deferred or side-stream covariance scan
void ensure_dense(cmpc_handle h);            // the dense A, Bu, C of the last linearization
void materialize_accepted_ks(cmpc_handle h); // accepted K / Sigma out of the live arrays

}  // namespace cmpc_host
