// Microbenchmark: the data movement of K5c (csrc/of3d_dev.hpp k_wz_solve_c) alone, for two
// layouts of the W-xy workspace, at configs[2] (c3) size: 9 fields of 128 x 512 x 512 fp64.
//   plain : [field][z][y][x]            — a block's window row (32 columns) is 256 B, rows a plane apart
//   tiled : [field][y][x / 32][z][32]   — a block's 106-plane window is one contiguous 26.5 KiB run
// Same grid (32 columns x 1 row x 64 planes per 4-wave block, XCD-aware z-chunk order), LDS-DMA
// 1-KiB wave-instructions, NB window buffers (one or two fields ahead), one barrier per field, no
// arithmetic (each thread adds one LDS value per field so the loads stay live).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_window tools/mb_window.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

__device__ __forceinline__ void glds16(const void* src, unsigned lds_byte) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_byte)
                 : "memory");
}

constexpr int RW = 21, ZC = 64, H = ZC + 2 * RW, RPWI = 4, HG = (H + RPWI - 1) / RPWI, NW = 4;
constexpr int NJ2 = (HG + NW - 1) / NW;

template <bool TILED, int NB>
__global__ __launch_bounds__(256, 2) void k_window(const double* __restrict__ Q, int nz, int ny, int nx, size_t fs,
                                                   double* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const double* sm = reinterpret_cast<const double*>(smem);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // XCD-aware block order as k5c_block: the z chunks of one (column block, row) 8 ids apart
    const unsigned gx = gridDim.x, gxy = gx * gridDim.y, nzc = gridDim.z;
    const unsigned b = blockIdx.x + gx * (blockIdx.y + gridDim.y * blockIdx.z);
    const unsigned full = (gxy * nzc) / (8 * nzc) * (8 * nzc);
    unsigned rest, zc;
    if (b < full) {
        const unsigned j = b >> 3;
        zc = j % nzc;
        rest = (j / nzc) * 8 + (b & 7);
    } else {
        const unsigned l = b - full;
        zc = l % nzc;
        rest = full / nzc + l / nzc;
    }
    const int bx = rest % gx, by = rest / gx, zc0 = zc * ZC;
    const int nxt = nx / 32;
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    auto issue = [&](int f, int buf) {
        const unsigned lb = lds0 + (unsigned)(buf * HG * 1024);
#pragma unroll
        for (int j = 0; j < NJ2; ++j) {
            const int pg = min(w + NW * j, HG - 1);
            const int row = min(RPWI * pg + lane / 16, H - 1);
            const int z = min(max(zc0 - RW + row, 0), nz - 1);
            const double* src = TILED ? Q + f * fs + (((size_t)by * nxt + bx) * nz + z) * 32 + 2 * (lane % 16)
                                      : Q + f * fs + (size_t)z * ny * nx + (size_t)by * nx + bx * 32 + 2 * (lane % 16);
            glds16(src, __builtin_amdgcn_readfirstlane(lb + (unsigned)(pg * 1024)));
        }
    };
    double acc = 0.0;
#pragma unroll
    for (int f = 0; f < NB - 1; ++f) issue(f, f);
#pragma unroll
    for (int f = 0; f < 9; ++f) {
        const int ahead = min(NB - 2, 8 - f);
        if (ahead >= 1)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NJ2) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (f + NB - 1 < 9) issue(f + NB - 1, (f + NB - 1) % NB);
        acc += sm[(f % NB) * HG * 128 + threadIdx.x];
    }
    out[blockIdx.x + gx * (blockIdx.y + (size_t)gridDim.y * blockIdx.z)] = acc;
}

template <bool TILED, int NB>
double run(const double* Q, int nz, int ny, int nx, size_t fs, double* out, int reps) {
    dim3 g(nx / 32, ny, nz / ZC);
    const size_t lds = (size_t)NB * HG * 1024;
    CK(hipFuncSetAttribute((const void*)k_window<TILED, NB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t ev0, ev1;
    CK(hipEventCreate(&ev0));
    CK(hipEventCreate(&ev1));
    for (int i = 0; i < 3; ++i) k_window<TILED, NB><<<g, 256, lds>>>(Q, nz, ny, nx, fs, out);
    CK(hipEventRecord(ev0));
    for (int i = 0; i < reps; ++i) k_window<TILED, NB><<<g, 256, lds>>>(Q, nz, ny, nx, fs, out);
    CK(hipEventRecord(ev1));
    CK(hipEventSynchronize(ev1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, ev0, ev1));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int nz = argc > 1 ? atoi(argv[1]) : 128, ny = argc > 2 ? atoi(argv[2]) : 512, nx = argc > 3 ? atoi(argv[3]) : 512;
    const int reps = 20;
    const size_t fs = (size_t)nz * ny * nx;
    double *Q, *out;
    CK(hipMalloc(&Q, 9 * fs * sizeof(double)));
    CK(hipMemset(Q, 0, 9 * fs * sizeof(double)));
    CK(hipMalloc(&out, (size_t)(nx / 32) * ny * (nz / ZC) * sizeof(double)));
    const double gb = 9.0 * fs * sizeof(double) / 1e9;  // compulsory bytes (the window halo comes from L2)
    for (int round = 0; round < 2; ++round) {
        const double p2 = run<false, 2>(Q, nz, ny, nx, fs, out, reps), t2 = run<true, 2>(Q, nz, ny, nx, fs, out, reps);
        const double p3 = run<false, 3>(Q, nz, ny, nx, fs, out, reps), t3 = run<true, 3>(Q, nz, ny, nx, fs, out, reps);
        printf("%dx%dx%d  plain NB2 %.3f ms (%.0f GB/s)  tiled NB2 %.3f ms (%.0f GB/s)  plain NB3 %.3f ms (%.0f GB/s)  "
               "tiled NB3 %.3f ms (%.0f GB/s)\n",
               nz, ny, nx, p2, gb / p2 * 1e3, t2, gb / t2 * 1e3, p3, gb / p3 * 1e3, t3, gb / t3 * 1e3);
    }
    CK(hipFree(Q));
    CK(hipFree(out));
    return 0;
}
