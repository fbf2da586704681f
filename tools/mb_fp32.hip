// fp32 VALU issue rate on gfx950: scalar v_add/v_mul_f32 vs packed v_pk_add/mul_f32 vs fp64
// (independent chains, 8 waves per SIMD).  Decides whether a VALU-bound fp32 pass gains from
// packing.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/mb_fp32 tools/mb_fp32.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

constexpr int kChains = 8, kIters = 4096;
typedef float f2 __attribute__((ext_vector_type(2)));

template <typename T>
__global__ __launch_bounds__(256) void addmul(float* out, T a, T b) {
    T v[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) v[c] = (T)(threadIdx.x * 1e-3f + c);
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            v[c] = v[c] * a;
            v[c] = v[c] + b;
        }
    }
    T s = v[0];
#pragma unroll
    for (int c = 1; c < kChains; ++c) s = s + v[c];
    float t;
    if constexpr (sizeof(T) == 8 && __is_same(T, f2)) t = s.x + s.y; else t = (float)s;
    if (t == 12345.678f) out[threadIdx.x] = t;
}

template <typename K, typename... A>
float timeit(K k, int blocks, A... a) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, a...);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, a...);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 5;
}

int main() {
    float* out;
    CK(hipMalloc(&out, 4096));
    const int blocks = 256 * 8 * 4;  // 8 waves per SIMD over 256 CUs (256-thread blocks)
    const double ops = (double)blocks * 256 * kIters * kChains * 2;  // lane-ops (add + mul)
    float ms = timeit(addmul<float>, blocks, out, 0.999f, 0.001f);
    printf("{\"kernel\": \"fp32 scalar\", \"ms\": %.4f, \"Tlaneops\": %.2f}\n", ms, ops / ms / 1e9);
    ms = timeit(addmul<f2>, blocks, out, (f2){0.999f, 0.998f}, (f2){0.001f, 0.002f});
    printf("{\"kernel\": \"fp32 packed\", \"ms\": %.4f, \"Tlaneops\": %.2f}\n", ms, 2 * ops / ms / 1e9);
    ms = timeit(addmul<double>, blocks, out, 0.999, 0.001);
    printf("{\"kernel\": \"fp64\", \"ms\": %.4f, \"Tlaneops\": %.2f}\n", ms, ops / ms / 1e9);
    return 0;
}
