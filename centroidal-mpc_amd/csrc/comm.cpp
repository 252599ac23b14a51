// Multi-GPU batch split over RCCL (xGMI): one process per GPU, one handle per process.
//
// The SCP problems are independent, so nothing crosses GPUs inside the hot loop.
// RCCL carries only what surrounds it:
//   * the shared parameter classes, broadcast from rank 0 (cmpc_comm_bcast_params);
//   * a max-reduction across ranks (the timed region's barrier and its max-over-ranks clock);
//   * the gather of every rank's per-problem results to rank 0 (cmpc_comm_gather_solution), with
//     the rank-major order of the contiguous batch slices, i.e. the global problem order.
// The reference has no distributed code (single process, src/scp_solver.py:118-179); this is the
// batch split of the north star.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "handle.hpp"

using namespace cmpc;
using namespace cmpc_host;

namespace {

#define NCCLCHK(x)                                                                              \
    do {                                                                                        \
        ncclResult_t r_ = (x);                                                                  \
        if (r_ != ncclSuccess) throw Fail{-4, std::string(#x) + ": " + ncclGetErrorString(r_)}; \
    } while (0)

ncclComm_t comm_of(cmpc_handle h) {
    need(h->comm != nullptr, "no communicator (cmpc_comm_init)");
    return (ncclComm_t)h->comm;
}

void free_comm(void *c) { (void)ncclCommDestroy((ncclComm_t)c); }

// device scratch freed at scope exit
struct DevTmp {
    void *p = nullptr;
    explicit DevTmp(size_t bytes) { HIPCHK(hipMalloc(&p, bytes < 16 ? 16 : bytes)); }
    ~DevTmp() { if (p) (void)hipFree(p); }
};

}  // namespace

extern "C" {

int cmpc_comm_get_unique_id(uint8_t *id_out) {
    if (!id_out) return -1;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return -4;
    std::memcpy(id_out, id.internal, CMPC_COMM_ID_BYTES);
    return 0;
}

int cmpc_comm_init(cmpc_handle h, int nranks, int rank, const uint8_t *id) {
    return guard(h, [&] {
        need(id != nullptr && nranks >= 1 && rank >= 0 && rank < nranks, "invalid communicator arguments");
        need(h->comm == nullptr, "communicator already initialized");
        ncclUniqueId uid;
        std::memcpy(uid.internal, id, CMPC_COMM_ID_BYTES);
        ncclComm_t c = nullptr;
        NCCLCHK(ncclCommInitRank(&c, nranks, uid, rank));
        h->comm = c;
        h->comm_rank = rank;
        h->comm_size = nranks;
        h->comm_free = free_comm;
    });
}

int cmpc_comm_destroy(cmpc_handle h) {
    return guard(h, [&] {
        if (!h->comm) return;
        HIPCHK(hipStreamSynchronize(h->stream));
        NCCLCHK(ncclCommDestroy((ncclComm_t)h->comm));
        h->comm = nullptr;
    });
}

int cmpc_comm_bcast_params(cmpc_handle h, int root, int n_classes, cmpc_params *classes) {
    int rc = guard(h, [&] {
        ncclComm_t c = comm_of(h);
        need(root >= 0 && root < h->comm_size, "invalid root");
        need(classes != nullptr, "null parameter buffer");
        // the count first (the receivers' n_classes is the capacity of their buffer)
        DevTmp dn(sizeof(int32_t));
        int32_t n = n_classes;
        HIPCHK(hipMemcpyAsync(dn.p, &n, sizeof(n), hipMemcpyHostToDevice, h->stream));
        NCCLCHK(ncclBroadcast(dn.p, dn.p, 1, ncclInt32, root, c, h->stream));
        HIPCHK(hipMemcpyAsync(&n, dn.p, sizeof(n), hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        need(n >= 1 && n <= n_classes, "parameter buffer smaller than the root's class count");
        const size_t bytes = (size_t)n * sizeof(cmpc_params);
        DevTmp dp(bytes);
        HIPCHK(hipMemcpyAsync(dp.p, classes, bytes, hipMemcpyHostToDevice, h->stream));
        NCCLCHK(ncclBroadcast(dp.p, dp.p, bytes, ncclUint8, root, c, h->stream));
        HIPCHK(hipMemcpyAsync(classes, dp.p, bytes, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        n_classes = n;
    });
    if (rc != 0) return rc;
    return cmpc_set_params(h, n_classes, classes);
}

int cmpc_comm_allreduce_max(cmpc_handle h, double *v, int n) {
    return guard(h, [&] {
        ncclComm_t c = comm_of(h);
        need(v != nullptr && n >= 1, "invalid buffer");
        DevTmp d((size_t)n * sizeof(double));
        HIPCHK(hipMemcpyAsync(d.p, v, (size_t)n * sizeof(double), hipMemcpyHostToDevice, h->stream));
        NCCLCHK(ncclAllReduce(d.p, d.p, (size_t)n, ncclFloat64, ncclMax, c, h->stream));
        HIPCHK(hipMemcpyAsync(v, d.p, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
    });
}

int cmpc_comm_gather_solution(cmpc_handle h, int root, double *X, double *U, int32_t *scp_status,
                              int32_t *iterations, int32_t *qp_status) {
    return guard(h, [&] {
        ncclComm_t c = comm_of(h);
        need(root >= 0 && root < h->comm_size, "invalid root");
        need(h->B > 0, "no problems uploaded");
        const int G = h->comm_size;
        const bool is_root = h->comm_rank == root;
        // every rank must hold the same batch size (ncclGather sends equal counts)
        {
            double bb[2] = {double(h->B), -double(h->B)};
            DevTmp d(sizeof(bb));
            HIPCHK(hipMemcpyAsync(d.p, bb, sizeof(bb), hipMemcpyHostToDevice, h->stream));
            NCCLCHK(ncclAllReduce(d.p, d.p, 2, ncclFloat64, ncclMax, c, h->stream));
            HIPCHK(hipMemcpyAsync(bb, d.p, sizeof(bb), hipMemcpyDeviceToHost, h->stream));
            HIPCHK(hipStreamSynchronize(h->stream));
            need(bb[0] == -bb[1], "ranks hold different batch sizes (pad the slices)");
        }
        const size_t B = h->B, N = h->N, e = h->esz();
        const size_t nx = B * (N + 1) * 9, nu = B * N * NU;
        const ncclDataType_t dt = h->prec == CMPC_PREC_F64 ? ncclFloat64 : ncclFloat32;
        // per-problem integers packed on the device: scp status | SCP iterations | QP status
        std::vector<ScpState> st(B);
        from_dev_raw(h, st.data(), h->scp, B * sizeof(ScpState));
        std::vector<int32_t> iv(3 * B);
        for (size_t b = 0; b < B; ++b) {
            iv[b] = st[b].status;
            iv[B + b] = st[b].iter;
            iv[2 * B + b] = st[b].qp_status;
        }
        DevTmp di(iv.size() * 4);
        HIPCHK(hipMemcpyAsync(di.p, iv.data(), iv.size() * 4, hipMemcpyHostToDevice, h->stream));
        DevTmp rx(is_root ? G * nx * e : 16), ru(is_root ? G * nu * e : 16), ri(is_root ? G * iv.size() * 4 : 16);
        NCCLCHK(ncclGroupStart());
        NCCLCHK(ncclGather(h->Xacc, rx.p, nx, dt, root, c, h->stream));
        NCCLCHK(ncclGather(h->Uacc, ru.p, nu, dt, root, c, h->stream));
        NCCLCHK(ncclGather(di.p, ri.p, iv.size(), ncclInt32, root, c, h->stream));
        NCCLCHK(ncclGroupEnd());
        HIPCHK(hipStreamSynchronize(h->stream));
        if (!is_root) return;
        if (h->prec == CMPC_PREC_F64) {
            from_dev<double>(h, X, rx.p, G * nx);
            from_dev<double>(h, U, ru.p, G * nu);
        } else {
            from_dev<float>(h, X, rx.p, G * nx);
            from_dev<float>(h, U, ru.p, G * nu);
        }
        std::vector<int32_t> all(G * iv.size());
        from_dev_raw(h, all.data(), ri.p, all.size() * 4);
        for (int g = 0; g < G; ++g)
            for (size_t b = 0; b < B; ++b) {
                const int32_t *blk = &all[(size_t)g * 3 * B];
                if (scp_status) scp_status[g * B + b] = blk[b];
                if (iterations) iterations[g * B + b] = blk[B + b];
                if (qp_status) qp_status[g * B + b] = blk[2 * B + b];
            }
    });
}

}  // extern "C"
