// Host AddressSanitizer harness of the C ABI (`make asan`; tests/test_asan.py).  The host code of
// cmpc_api.cpp, load_qp.cpp and comm.cpp is built with -fsanitize=address (host side only: GPU
// ASan is not available on gfx950 here) into libcmpc_asan.so, and this program drives the argument
// validation and error paths of every entry point: with no device (the build container), all of
// them must fail with an error code and leave nothing behind; with a device, a handle is created
// and the validation of parameters, uploads, cmpc_load_qp's CSC decoding and the getters runs on it.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "cmpc.h"

static int fails = 0;
#define CHECK(c)                                                           \
    do {                                                                   \
        if (!(c)) { std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); ++fails; } \
    } while (0)

static void null_handle_paths() {
    double d[16] = {0};
    int32_t i32[16] = {0};
    int n = 0;
    CHECK(cmpc_set_qp_settings(nullptr, nullptr) != 0);
    CHECK(cmpc_set_params(nullptr, 1, nullptr) != 0);
    CHECK(cmpc_upload(nullptr, 1, i32, nullptr, d, d, d, d) != 0);
    CHECK(cmpc_set_trust_region(nullptr, d, d) != 0);
    CHECK(cmpc_linearize(nullptr) != 0);
    CHECK(cmpc_assemble(nullptr) != 0);
    CHECK(cmpc_qp_solve(nullptr) != 0);
    CHECK(cmpc_scp_iterate(nullptr, 1) != 0);
    CHECK(cmpc_solve_scp(nullptr, 0, &n) != 0);
    CHECK(cmpc_get_solution(nullptr, d, d, d, d, i32, i32, i32, d, d) != 0);
    CHECK(cmpc_get_accepted(nullptr, 0, d, d, d, d) != 0);
    CHECK(cmpc_get_qp_exit(nullptr, i32, i32) != 0);
    CHECK(cmpc_load_qp(nullptr, 0, 1, 1, d, i32, i32, d, d, i32, i32, d, d) != 0);
    char buf[8];
    CHECK(cmpc_get_qp_kernel(nullptr, buf, 8) != 0);
    CHECK(cmpc_destroy(nullptr) != 0 || true);   // (a no-op either way)
    CHECK(std::strcmp(cmpc_last_error(nullptr), "null handle") == 0);
}

static void create_validation() {
    cmpc_handle h = reinterpret_cast<cmpc_handle>(0x1);
    CHECK(cmpc_create(nullptr, 0, 0, 20, 4, CMPC_PREC_F64) == -1);
    CHECK(cmpc_create(&h, 0, 2, 20, 4, CMPC_PREC_F64) == -2 && h == nullptr);   // robot
    CHECK(cmpc_create(&h, 0, 0, 1, 4, CMPC_PREC_F64) == -2);                     // N < 2
    CHECK(cmpc_create(&h, 0, 0, 256, 4, CMPC_PREC_F64) == -2);                   // N > 255
    CHECK(cmpc_create(&h, 0, 0, 20, 0, CMPC_PREC_F64) == -2);                    // batch
    CHECK(cmpc_create(&h, 0, 0, 20, 4, 7) == -2);                                // precision
    CHECK(cmpc_create(&h, 0, 1, 20, 4, CMPC_PREC_F32) == -5);                    // TALOS fp32
    CHECK(cmpc_create(&h, -1, 0, 20, 4, CMPC_PREC_F64) != 0 && h == nullptr);    // device id
    cmpc_qp_settings s;
    CHECK(cmpc_default_qp_settings(CMPC_PREC_F64, nullptr) != 0);
    CHECK(cmpc_default_qp_settings(CMPC_PREC_F64, &s) == 0 && s.eps_abs == 0.0 && s.polish_eps < 0);
}

static void device_paths(cmpc_handle h) {
    const int N = 20, B = 2;
    double d[64] = {0};
    int32_t cid[B] = {0, 0};
    // before cmpc_set_params / cmpc_upload
    std::vector<double> X((size_t)B * (N + 1) * 9, 0.0), U((size_t)B * N * 12, 0.0);
    std::vector<int8_t> logic((size_t)B * N * 4, 1);
    std::vector<double> pos((size_t)B * N * 4 * 3, 0.0), rot((size_t)B * N * 4 * 9, 0.0);
    CHECK(cmpc_upload(h, B, cid, logic.data(), pos.data(), rot.data(), X.data(), U.data()) != 0);
    CHECK(cmpc_set_params(h, 0, nullptr) != 0);
    CHECK(cmpc_set_params(h, 1, nullptr) != 0);
    CHECK(cmpc_upload(h, B + 10, cid, logic.data(), pos.data(), rot.data(), X.data(), U.data()) != 0);
    CHECK(cmpc_get_accepted(h, -1, X.data(), U.data(), nullptr, nullptr) != 0);
    int32_t n = 0, m = 0, nnzP = 0, nnzA = 0;
    CHECK(cmpc_qp_sizes(h, &n, &m, &nnzP, &nnzA) == 0 && n > 0 && m > 0);
    // cmpc_load_qp: malformed CSC is refused before anything is decoded
    std::vector<int32_t> Pp(n + 1, 0), Pi(4, 0), Ap(n + 1, 0), Ai(4, 0);
    std::vector<double> Px(4, 1.0), q(n, 0.0), Ax(4, 1.0), l(m, 0.0), u(m, 0.0);
    CHECK(cmpc_load_qp(h, 0, n, m, nullptr, Pi.data(), Pp.data(), q.data(), Ax.data(), Ai.data(), Ap.data(), l.data(), u.data()) != 0);
    CHECK(cmpc_load_qp(h, 99, n, m, Px.data(), Pi.data(), Pp.data(), q.data(), Ax.data(), Ai.data(), Ap.data(), l.data(), u.data()) != 0);
    char buf[4];
    CHECK(cmpc_get_qp_kernel(h, buf, 0) != 0);
    CHECK(cmpc_get_qp_kernel(h, buf, sizeof buf) == 0 && std::strlen(buf) < sizeof buf);
    CHECK(std::strlen(cmpc_last_error(h)) < 4096);
    (void)d;
}

int main() {
    CHECK(cmpc_version() == 1);
    null_handle_paths();
    create_validation();
    cmpc_handle h = nullptr;
    const int rc = cmpc_create(&h, 0, 0, 20, 2, CMPC_PREC_F64);
    if (rc != 0) {
        CHECK(h == nullptr);
        std::printf("asan harness: no device (cmpc_create rc=%d); host paths only\n", rc);
    } else {
        device_paths(h);
        CHECK(cmpc_destroy(h) == 0);
        std::printf("asan harness: device paths run\n");
    }
    std::printf("asan harness: %s (%d failed checks)\n", fails ? "FAILED" : "ok", fails);
    return fails ? 1 : 0;
}
