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
        const int G = h->comm_size, rank = h->comm_rank;
        const bool is_root = rank == root;
        // every rank's batch size (slices of ceil(B / G) leave the last ranks short): ncclGather
        // sends equal counts, so each rank sends its slice padded to the largest and the root
        // packs the blocks back to back (rank-major = the global order of contiguous slices)
        std::vector<double> bs(G, 0.0);
        bs[rank] = double(h->B);
        {
            DevTmp d(G * sizeof(double));
            HIPCHK(hipMemcpyAsync(d.p, bs.data(), G * sizeof(double), hipMemcpyHostToDevice, h->stream));
            NCCLCHK(ncclAllReduce(d.p, d.p, (size_t)G, ncclFloat64, ncclMax, c, h->stream));
            HIPCHK(hipMemcpyAsync(bs.data(), d.p, G * sizeof(double), hipMemcpyDeviceToHost, h->stream));
            HIPCHK(hipStreamSynchronize(h->stream));
        }
        size_t Bmax = 0;
        for (double v : bs) Bmax = std::max(Bmax, (size_t)v);
        const size_t B = h->B, N = h->N, e = h->esz();
        const size_t px = (N + 1) * 9, pu = N * NU;   // per problem
        const ncclDataType_t dt = h->prec == CMPC_PREC_F64 ? ncclFloat64 : ncclFloat32;
        // per-problem integers: scp status | SCP iterations | QP status, padded to Bmax
        std::vector<ScpState> st(B);
        from_dev_raw(h, st.data(), h->scp, B * sizeof(ScpState));
        std::vector<int32_t> iv(3 * Bmax, 0);
        for (size_t b = 0; b < B; ++b) {
            iv[b] = st[b].status;
            iv[Bmax + b] = st[b].iter;
            iv[2 * Bmax + b] = st[b].qp_status;
        }
        DevTmp di(iv.size() * 4), sx(Bmax * px * e), su(Bmax * pu * e);
        HIPCHK(hipMemcpyAsync(di.p, iv.data(), iv.size() * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(hipMemsetAsync(sx.p, 0, Bmax * px * e, h->stream));
        HIPCHK(hipMemsetAsync(su.p, 0, Bmax * pu * e, h->stream));
        HIPCHK(hipMemcpyAsync(sx.p, h->Xacc, B * px * e, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(hipMemcpyAsync(su.p, h->Uacc, B * pu * e, hipMemcpyDeviceToDevice, h->stream));
        DevTmp rx(is_root ? G * Bmax * px * e : 16), ru(is_root ? G * Bmax * pu * e : 16),
            ri(is_root ? G * iv.size() * 4 : 16);
        NCCLCHK(ncclGroupStart());
        NCCLCHK(ncclGather(sx.p, rx.p, Bmax * px, dt, root, c, h->stream));
        NCCLCHK(ncclGather(su.p, ru.p, Bmax * pu, dt, root, c, h->stream));
        NCCLCHK(ncclGather(di.p, ri.p, iv.size(), ncclInt32, root, c, h->stream));
        NCCLCHK(ncclGroupEnd());
        HIPCHK(hipStreamSynchronize(h->stream));
        if (!is_root) return;
        std::vector<int32_t> all(G * iv.size());
        from_dev_raw(h, all.data(), ri.p, all.size() * 4);
        size_t off = 0;
        for (int g = 0; g < G; ++g) {
            const size_t Bg = (size_t)bs[g];
            auto dl = [&](double *dst, const DevTmp &src, size_t per) {
                if (!dst || Bg == 0) return;
                const char *blk = (const char *)src.p + (size_t)g * Bmax * per * e;
                if (h->prec == CMPC_PREC_F64) from_dev<double>(h, dst + off * per, blk, Bg * per);
                else from_dev<float>(h, dst + off * per, blk, Bg * per);
            };
            dl(X, rx, px);
            dl(U, ru, pu);
            const int32_t *blk = &all[(size_t)g * 3 * Bmax];
            for (size_t b = 0; b < Bg; ++b) {
                if (scp_status) scp_status[off + b] = blk[b];
                if (iterations) iterations[off + b] = blk[Bmax + b];
                if (qp_status) qp_status[off + b] = blk[2 * Bmax + b];
            }
            off += Bg;
        }
    });
}

}  // extern "C"
