// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the QP kernel
// uses: known-byte streaming reads and writes of 8 B per lane (one fp64 per
// lane, a wave reading 512 contiguous bytes: the knot-minor field rows of k_qp_ipm) and of 16 B per
// lane (the width MI355X_MICROARCH.md calibrates), over 1 GiB buffers (4x the Infinity Cache).
// Each kernel runs once per launch of this binary; profile with one counter pass at a time:
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib      rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
// and compare the per-dispatch counter with the bytes printed here.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__global__ void k_read8(const double *__restrict__ a, size_t n, double *out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 1234.5) out[0] = s;   // keeps the loads; never true for the zero-filled input
}
__global__ void k_read16(const double2 *__restrict__ a, size_t n, double *out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 1234.5) out[0] = s;
}
__global__ void k_write8(double *__restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = 1.0;
}
__global__ void k_write16(double2 *__restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = make_double2(1.0, 2.0);
}

int main() {
    const size_t bytes = size_t(1) << 30;
    double *a = nullptr, *out = nullptr;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&out, 64));
    CHK(hipMemset(a, 0, bytes));
    CHK(hipDeviceSynchronize());
    const int grid = 256 * 8, block = 256;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    float ms;
    // flush: write the whole buffer once more so nothing of it is read from a warm cache first
    k_write16<<<grid, block>>>((double2 *)a, bytes / 16);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0)); k_read8<<<grid, block>>>(a, bytes / 8, out); CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1)); std::printf("k_read8   read  %zu B  %.3f ms  %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    CHK(hipEventRecord(e0)); k_read16<<<grid, block>>>((const double2 *)a, bytes / 16, out); CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1)); std::printf("k_read16  read  %zu B  %.3f ms  %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    CHK(hipEventRecord(e0)); k_write8<<<grid, block>>>(a, bytes / 8); CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1)); std::printf("k_write8  write %zu B  %.3f ms  %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    CHK(hipEventRecord(e0)); k_write16<<<grid, block>>>((double2 *)a, bytes / 16); CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1)); std::printf("k_write16 write %zu B  %.3f ms  %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    CHK(hipFree(a)); CHK(hipFree(out));
    return 0;
}
