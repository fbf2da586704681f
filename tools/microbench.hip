// Calibration microbenchmarks for the roofline numbers used in bench.py / DESIGN.md:
//   fp64_addmul : independent v_add_f64 / v_mul_f64 chains -> fp64 VALU issue rate
//   copy8 / copy16 : streaming copy with 8-B and 16-B lanes over 1 GiB -> HBM GB/s,
//                    and (under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE) the counter
//                    calibration factor for those access widths
//   lds_read8   : ds_read_b64 throughput
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

constexpr int kChains = 8;
constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void fp64_addmul(double* out, double a, double b) {
    double v[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            v[c] = v[c] * a;
            v[c] = v[c] + b;
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += v[c];
    if (s == 12345.678) out[threadIdx.x] = s;  // keep live
}

__global__ __launch_bounds__(256) void copy8(const double* __restrict__ a, double* __restrict__ b, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t st = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += st) b[i] = a[i];
}

__global__ __launch_bounds__(256) void copy16(const double2* __restrict__ a, double2* __restrict__ b, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t st = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += st) b[i] = a[i];
}

__global__ __launch_bounds__(256) void read8(const double* __restrict__ a, double* __restrict__ out, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t st = (size_t)gridDim.x * blockDim.x;
    double s = 0;
    for (; i < n; i += st) s += a[i];
    if (s == 12345.678) out[0] = s;
}

__global__ __launch_bounds__(256) void lds_read8(double* out, int iters) {
    __shared__ double sm[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i;
    __syncthreads();
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    int base = threadIdx.x;
    for (int it = 0; it < iters; ++it) {
        s0 += sm[(base + it * 64) & 4095];
        s1 += sm[(base + it * 64 + 1024) & 4095];
        s2 += sm[(base + it * 64 + 2048) & 4095];
        s3 += sm[(base + it * 64 + 3072) & 4095];
    }
    if (s0 + s1 + s2 + s3 == 12345.678) out[0] = s0;
}

int main() {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    double* out;
    CK(hipMalloc(&out, 4096 * sizeof(double)));
    float ms;
    // fp64 VALU
    {
        const int blocks = 256 * 16;
        hipLaunchKernelGGL(fp64_addmul, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 1e-9);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(fp64_addmul, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 1e-9);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double ops = (double)blocks * 256 * kIters * kChains * 2;
        printf("fp64_addmul: %.3f ms  %.2f T lane-ops/s (add+mul, no FMA)\n", ms, ops / (ms * 1e-3) / 1e12);
    }
    const size_t bytes = (size_t)1 << 30;
    double *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    const int grid = 256 * 8;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(copy8, dim3(grid), dim3(256), 0, 0, a, b, bytes / 8);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(copy8, dim3(grid), dim3(256), 0, 0, a, b, bytes / 8);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("copy8 (1 GiB read + 1 GiB write): %.3f ms  %.1f GB/s\n", ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
        hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, 0, (const double2*)a, (double2*)b, bytes / 16);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, 0, (const double2*)a, (double2*)b, bytes / 16);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("copy16 (1 GiB read + 1 GiB write): %.3f ms  %.1f GB/s\n", ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
        hipLaunchKernelGGL(read8, dim3(grid), dim3(256), 0, 0, a, out, bytes / 8);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(read8, dim3(grid), dim3(256), 0, 0, a, out, bytes / 8);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("read8 (1 GiB read): %.3f ms  %.1f GB/s\n", ms, 1.0 * bytes / (ms * 1e-3) / 1e9);
    }
    {
        const int iters = 4096, blocks = 256 * 8;
        hipLaunchKernelGGL(lds_read8, dim3(blocks), dim3(256), 0, 0, out, iters);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(lds_read8, dim3(blocks), dim3(256), 0, 0, out, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double rd = (double)blocks * 256 * iters * 4 * 8;
        printf("lds_read8: %.3f ms  %.1f TB/s aggregate ds_read_b64\n", ms, rd / (ms * 1e-3) / 1e12);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
