#pragma once
// of3d_dev.hpp — device code of libof3d (kernels, pass helpers, geometry constants).
// Included by every translation unit; the kernel templates are instantiated only in the
// unit that takes their address (kt_*.hip getters, of3d_host.hip for the small kernels).
//
//
// Re-design (not a port) of the hot path of ScientistRachel/OpticalFlow3D_dev
// src/Python/calc_flow.py:175-360 (calc_flow3D) and :18-173 (calc_flow2D).
// The reference runs 40 scipy.ndimage.correlate1d passes over full fp64
// volumes plus a per-voxel LAPACK cgeev; here the same arithmetic is a
// five-kernel device pipeline over HBM-resident fields:
//
//   K0c tderiv   : temporal derivative of the centre frame (T2)
//   K1c grad_xy  : y and x passes of the four gradient filters (T4), column march:
//                  register rings down each column, LDS tiles for the x pass
//   K2c grad_z   : z pass of the four gradients (T4), z march with register rings
//   K34 prod_wyx : the 9 (2D: 5) structure-tensor products + W y (register ring)
//                  + W x (LDS tiles) in one pass (T5); the plan autotunes its shape
//   K5c wz_solve : W z pass (T5, LDS-DMA windows) + closed-form 3x3 solve (T6) +
//                  fp64 smallest eigenvalue (T7);  2D: 2x2 solve + rel (T8)
//
// The earlier kernels (k_tderiv_vec, k_grad_xy, k_grad_z, k_prod_wy + k_wx,
// k_wz_solve_dma / k_wz_solve) remain for radii and input types without a
// compiled column-march instance, and as the A/B reference (bit-identical).
//
// Bit-exactness: every 1-D pass evaluates scipy's NI_Correlate1D order for
// (anti)symmetric taps  o = c0*w0; for k=r..1: o += (c[-k] +- c[+k]) * w[-k]
// with indices clamped to the GLOBAL volume edge at every pass
// (mode='nearest'); products and the solve copy calc_flow.py's expression
// trees.  Built with -ffp-contract=off (no FMA) and IEEE div/sqrt.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/of3d.h"

namespace {

thread_local std::string g_err;

int fail(const std::string& msg) {
    g_err = msg;
    return -1;
}

#define OF3D_HIP(call)                                                                    \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess) return fail(std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int kMaxR = 48;          // largest supported tap radius (LDS tiles)
constexpr int kMaxT = 2 * 32 + 1;  // largest temporal window (rt <= 32)
constexpr double kEps = 2.220446049250313e-16;  // np.finfo(float).eps, calc_flow.py:155,338

// Half taps on the device: h[0] = centre tap w[r], h[k] = w[r-k] (left side),
// exactly the coefficients scipy multiplies by in the symmetric branch.
// F = the arithmetic type of the filter passes: double (exact mode) or float
// (OF3D_FP32 plans); taps are stored in F.
template <typename F>
struct DevTaps {
    const F* g;  // gauss   (rd)
    const F* d;  // deriv   (rd, antisymmetric)
    const F* s;  // smooth  (rs)
    const F* t;  // tderiv  (rt, antisymmetric)
    const F* w;  // window  (rw)
    // step-order copies (hr[q] = w[q], q < r, then kTapPad zeros), see lds_pass
    const F *gr, *dr, *sr, *tr, *wr;
    int rd, rs, rt, rw;
};

struct Frames {
    const void* p[kMaxT];  // frames c-rt .. c+rt
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

template <typename T, typename F>
__device__ __forceinline__ F ldf(const void* p, size_t i) {
    return (F)(reinterpret_cast<const T*>(p)[i]);
}

// 1-D pass over a staged LDS line, R consecutive outputs per thread at line
// positions base..base+R-1 (elements `st` doubles apart); the staged line
// already holds the clamped halo (positions base-r .. base+R-1+r valid).
// Summation order per output is scipy's: o = c*w0; k = r..1: o += (lo +- hi)*w.
//
// Register reuse without register moves: at step q (k = r-q) output i needs
// lo = s[base-r+q+i] and hi = s[base+r-q+i].  Both are streams indexed by
// (q+i) and (q-i); each lives in a ring of M slots (L[m % M], U[m % M]), and
// the q loop is unrolled by M so every slot index is a compile-time constant.
// Per step: 2 LDS reads, 3R fp64 ops, ~3R live doubles, any radius.
// Weights: h[0] is the centre tap; hr[q] = h[r - q] = w[q] is the weight of step
// q (outermost tap first), padded with kTapPad zeros past hr[r - 1].  PRE: each
// M-step block takes its M weights with one uniform load issued a block ahead
// (no scalar load + wait inside the steps; costs 2M registers, so kernels at
// their register cap keep PRE off).
constexpr int kTapPad = 8;  // >= the largest M

template <int R, bool ANTI, bool PRE = true, int D = 1, bool WRAP = false, typename F>
__device__ __forceinline__ void lds_pass(const F* __restrict__ s, int st, int base, const F* __restrict__ h,
                                         const F* __restrict__ hr, int r, F (&out)[R], int wmask = 0) {
    // WRAP: the staged line is a ring of (wmask + 1) positions (power of two)
    auto at = [&](int i) { return WRAP ? s[(i & wmask) * st] : s[i * st]; };
    // Ring of M = R + D - 1 slots per stream: the two reads issued after step q
    // are first consumed at step q + D (prefetch distance D hides LDS latency).
    constexpr int M = R + D - 1;
    static_assert(M <= kTapPad, "tap padding too short for this ring");
    F L[M], U[M];
#pragma unroll
    for (int i = 0; i < R; ++i) out[i] = at(base + i) * h[0];
#pragma unroll
    for (int m = 0; m < M; ++m) L[m] = at(base - r + m);           // S_lo[0 .. M-1]
#pragma unroll
    for (int m = -(R - 1); m < D; ++m) U[((m % M) + M) % M] = at(base + r - m);  // S_hi[-(R-1) .. D-1]
    F wb[M];  // weights of the current block
    if constexpr (PRE) {
#pragma unroll
        for (int m = 0; m < M; ++m) wb[m] = hr[m];
    }
    auto step = [&](int q, auto jc) {  // phase j = q mod M (compile-time)
        constexpr int j = decltype(jc)::value;
        const F wk = PRE ? wb[j] : hr[q];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const F lo = L[(j + i) % M];
            const F hi = U[((j - i) % M + M) % M];
            out[i] = out[i] + (ANTI ? (lo - hi) : (lo + hi)) * wk;
        }
        L[j] = at(base - r + q + M);           // S_lo[q+M]   (slot of S_lo[q], done)
        U[(j + D) % M] = at(base + r - q - D);  // S_hi[q+D]   (slot of S_hi[q-R+1], done)
    };
    int q = 0;
    for (; q + M <= r; q += M) {
        F wn[M];  // next block's weights, in flight during this block
        if constexpr (PRE) {
#pragma unroll
            for (int m = 0; m < M; ++m) wn[m] = hr[q + M + m];
        }
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (step(q + J, std::integral_constant<int, J>{}), ...);
        }(std::make_integer_sequence<int, M>{});
        if constexpr (PRE) {
#pragma unroll
            for (int m = 0; m < M; ++m) wb[m] = wn[m];
        }
    }
    const int t = r - q;  // 0 .. M-1 remaining steps
    [&]<int... J>(std::integer_sequence<int, J...>) {
        ((J < t ? step(q + J, std::integral_constant<int, J>{}) : void()), ...);
    }(std::make_integer_sequence<int, M - 1>{});
}

// lds_pass with a compile-time radius RW and the half taps in registers
// (h[k] = w[RW - k]: uniform, so SGPRs): fully unrolled, no weight loads or
// waits inside the pass, same scipy order.  Stream rings as in lds_pass
// (prefetch distance D); reads past the last needed element are skipped.
// SOLO: every element read stays a single ds_read_b64 / _b32 (an empty fence after each): the
// compiler otherwise pairs reads one window row apart into ds_read2_b64, which moves 1 KiB per
// wave-instruction in 8 LDS cycles where two ds_read_b64 take 4 (MI355X_MICROARCH.md, LDS table)
template <int R, int RW, int D, bool ANTI = false, bool SOLO = false, typename F>
__device__ __forceinline__ void lds_pass_c(const F* __restrict__ s, int st, int base, const F (&h)[RW + 1],
                                           F (&out)[R]) {
    constexpr int M = R + D - 1;
    auto rd = [&](int i) {
        const F v = s[i * st];
        if constexpr (SOLO) asm volatile("" ::: "memory");
        return v;
    };
    F L[M], U[M];
#pragma unroll
    for (int i = 0; i < R; ++i) out[i] = rd(base + i) * h[0];
#pragma unroll
    for (int m = 0; m < M; ++m) L[m] = rd(base - RW + m);  // S_lo[0 .. M-1]
#pragma unroll
    for (int m = -(R - 1); m < D; ++m) U[((m % M) + M) % M] = rd(base + RW - m);  // S_hi[-(R-1) .. D-1]
#pragma unroll
    for (int q = 0; q < RW; ++q) {  // k = RW - q, outermost tap first
        const int j = q % M;
        const F wk = h[RW - q];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const F lo = L[(j + i) % M];
            const F hi = U[((j - i) % M + M) % M];
            out[i] = out[i] + (ANTI ? (lo - hi) : (lo + hi)) * wk;
        }
        if (q + M <= RW + R - 2) L[j] = rd(base - RW + q + M);  // S_lo[q+M]
        if (q + D <= RW - 1) U[(j + D) % M] = rd(base + RW - q - D);  // S_hi[q+D]
    }
}
// The wave-specialised K34's consumers read single elements (fp64: c3 K34 1.65 -> 1.60 ms, c4
// 10.93 -> 10.87, same box, profiles/r06/abk5/).  K5c keeps the compiler's ds_read2_b64 pairs: single
// reads there cost its CSE of the window's centre values (576 instead of 450 reads per field set)
// and measured slower (c3 K5c 0.978 -> 1.015 ms, c4 6.82 -> 6.97); so did the lockstep K34 forms
// (c2 K34 0.17 -> 0.19 ms)
constexpr bool k5c_solo64 = false;
template <typename F>
constexpr bool k5c_solo = sizeof(F) == 8 && k5c_solo64;
constexpr bool k34_solo = true;

// ---------------------------------------------------------------------------
// K0: temporal derivative of the centre frame (T2, calc_flow.py:276-277):
//   dt0 = I[c]*T[0] + sum_{k=rt..1} (I[c-k] - I[c+k]) * T[k]
// (scipy's antisymmetric order, outer tap first; the reference filters all Nt
// frames and keeps the centre — only the centre line is formed here).
// Streaming, one voxel per lane; frames by stride (one stack) or pointer table.
// ---------------------------------------------------------------------------
template <typename T, typename F>
__global__ __launch_bounds__(256) void k_tderiv(Frames fr, long long fstride, size_t off0, size_t n, int rt,
                                                const F* __restrict__ ht, F* __restrict__ D0) {
    const size_t st = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += st) {
        const size_t idx = off0 + i;
        F c, dt;
        if (fstride) {
            const T* p = reinterpret_cast<const T*>(fr.p[0]) + idx;
            c = (F)p[(long long)rt * fstride];
            dt = c * ht[0];
            for (int k = rt; k >= 1; --k)
                dt = dt + ((F)p[(long long)(rt - k) * fstride] - (F)p[(long long)(rt + k) * fstride]) * ht[k];
        } else {
            c = ldf<T, F>(fr.p[rt], idx);
            dt = c * ht[0];
            for (int k = rt; k >= 1; --k)
                dt = dt + (ldf<T, F>(fr.p[rt - k], idx) - ldf<T, F>(fr.p[rt + k], idx)) * ht[k];
        }
        D0[i] = dt;
    }
}

// Vectorised K0 (any frame order, e.g. a device ring buffer; every frame
// aligned to the vector width): each lane handles V consecutive voxels with
// one 8- or 16-byte load per frame.
template <typename T>
struct K0Vec {
    static constexpr int V = sizeof(T) == 1 ? 8 : (sizeof(T) == 8 ? 2 : 4);
    static constexpr int B = V * (int)sizeof(T);  // 8 or 16 bytes
};

template <typename T, typename F>
__device__ __forceinline__ void load_vec(const T* p, F (&v)[K0Vec<T>::V]) {
    constexpr int V = K0Vec<T>::V;
    T t[V];
    if constexpr (K0Vec<T>::B == 8) {
        const unsigned long long raw = *reinterpret_cast<const unsigned long long*>(p);
        __builtin_memcpy(t, &raw, 8);
    } else {
        const uint4 raw = *reinterpret_cast<const uint4*>(p);
        __builtin_memcpy(t, &raw, 16);
    }
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = (F)t[i];
}

template <typename T, typename F>
__global__ __launch_bounds__(256) void k_tderiv_vec(Frames fr, size_t off0, size_t ngroups, int rt,
                                                    const F* __restrict__ ht, F* __restrict__ D0) {
    constexpr int V = K0Vec<T>::V;
    const size_t st = (size_t)gridDim.x * 256;
    for (size_t gi = (size_t)blockIdx.x * 256 + threadIdx.x; gi < ngroups; gi += st) {
        const size_t o = off0 + gi * V;
        F c[V], a[V], b[V], dt[V];
        load_vec<T, F>(reinterpret_cast<const T*>(fr.p[rt]) + o, c);
#pragma unroll
        for (int i = 0; i < V; ++i) dt[i] = c[i] * ht[0];
        for (int k = rt; k >= 1; --k) {
            load_vec<T, F>(reinterpret_cast<const T*>(fr.p[rt - k]) + o, a);
            load_vec<T, F>(reinterpret_cast<const T*>(fr.p[rt + k]) + o, b);
            const F w = ht[k];
#pragma unroll
            for (int i = 0; i < V; ++i) dt[i] = dt[i] + (a[i] - b[i]) * w;
        }
        if constexpr (sizeof(F) == 8) {
            double2* d = reinterpret_cast<double2*>(D0 + gi * V);
#pragma unroll
            for (int i = 0; i < V / 2; ++i) d[i] = make_double2(dt[2 * i], dt[2 * i + 1]);
        } else {
#pragma unroll
            for (int i = 0; i < V; ++i) D0[gi * V + i] = dt[i];
        }
    }
}

// K0 with a compile-time temporal radius: all 2RT+1 frame loads of a lane issued
// before the first use (the runtime-rt loop above keeps only two in flight per lane:
// latency-bound at 4.3 TB/s on c2).  Same arithmetic order.
// One vector group of K0c: voxels o .. o + V - 1 of every frame -> D0g[0 .. V - 1] (shared by
// the K0c kernel and the next-frame K0 inside the fused K5c, so both compute the same bits).
template <typename T, typename F, int RT>
__device__ __forceinline__ void k0_group_dt(const Frames& fr, size_t o, const F (&h)[RT + 1], F (&dt)[K0Vec<T>::V]) {
    constexpr int V = K0Vec<T>::V, NW = 2 * RT + 1;
    using Raw = typename std::conditional<K0Vec<T>::B == 8, unsigned long long, uint4>::type;
    Raw raw[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) raw[i] = *reinterpret_cast<const Raw*>(reinterpret_cast<const T*>(fr.p[i]) + o);
    auto val = [&](int i, int e) {
        T t[V];
        __builtin_memcpy(t, &raw[i], sizeof(Raw));
        return (F)t[e];
    };
#pragma unroll
    for (int e = 0; e < V; ++e) dt[e] = val(RT, e) * h[0];
#pragma unroll
    for (int k = RT; k >= 1; --k)
#pragma unroll
        for (int e = 0; e < V; ++e) dt[e] = dt[e] + (val(RT - k, e) - val(RT + k, e)) * h[k];
}
template <typename F, int V>
__device__ __forceinline__ void k0_store(const F (&dt)[V], F* __restrict__ D0g) {
    if constexpr (sizeof(F) == 8) {
        double2* d = reinterpret_cast<double2*>(D0g);
#pragma unroll
        for (int i = 0; i < V / 2; ++i) d[i] = make_double2(dt[2 * i], dt[2 * i + 1]);
    } else {
#pragma unroll
        for (int i = 0; i < V; ++i) D0g[i] = dt[i];
    }
}
template <typename T, typename F, int RT>
__device__ __forceinline__ void k0_group(const Frames& fr, size_t o, const F (&h)[RT + 1], F* __restrict__ D0g) {
    F dt[K0Vec<T>::V];
    k0_group_dt<T, F, RT>(fr, o, h, dt);
    k0_store<F, K0Vec<T>::V>(dt, D0g);
}

template <typename T, typename F, int RT>
__global__ __launch_bounds__(256) void k_tderiv_vec_c(Frames fr, size_t off0, size_t ngroups, const F* __restrict__ ht,
                                                      F* __restrict__ D0) {
    constexpr int V = K0Vec<T>::V;
    F h[RT + 1];
#pragma unroll
    for (int k = 0; k <= RT; ++k) h[k] = ht[k];
    const size_t st = (size_t)gridDim.x * 256;
    for (size_t gi = (size_t)blockIdx.x * 256 + threadIdx.x; gi < ngroups; gi += st)
        k0_group<T, F, RT>(fr, off0 + gi * V, h, D0 + gi * V);
}

// K0 batching (of3d_plan_execute_ahead): the temporal derivatives of M consecutive output
// frames of a time series in one pass — frames c-rt .. c+M-1+rt, each loaded once (2rt + M
// loads for M derivatives instead of M (2rt + 1)); output m (centre c + m) in the order of
// k0_group_dt (bit-identical), to D0 + m * dstride.
template <typename T, typename F, int RT, int M>
__global__ __launch_bounds__(256) void k_tderiv_multi(Frames fr, size_t off0, size_t ngroups,
                                                      const F* __restrict__ ht, F* __restrict__ D0,
                                                      size_t dstride) {
    constexpr int V = K0Vec<T>::V, NW = 2 * RT + M;
    static_assert(NW <= kMaxT, "frame table");
    using Raw = typename std::conditional<K0Vec<T>::B == 8, unsigned long long, uint4>::type;
    F h[RT + 1];
#pragma unroll
    for (int k = 0; k <= RT; ++k) h[k] = ht[k];
    const size_t st = (size_t)gridDim.x * 256;
    for (size_t gi = (size_t)blockIdx.x * 256 + threadIdx.x; gi < ngroups; gi += st) {
        const size_t o = off0 + gi * V;
        Raw raw[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) raw[i] = *reinterpret_cast<const Raw*>(reinterpret_cast<const T*>(fr.p[i]) + o);
        auto val = [&](int i, int e) {
            T t[V];
            __builtin_memcpy(t, &raw[i], sizeof(Raw));
            return (F)t[e];
        };
        F dt[M][V];
#pragma unroll
        for (int e = 0; e < V; ++e) {  // one voxel at a time: its NW frame values converted once
            F x[NW];
#pragma unroll
            for (int i = 0; i < NW; ++i) x[i] = val(i, e);
#pragma unroll
            for (int m = 0; m < M; ++m) {
                dt[m][e] = x[RT + m] * h[0];
#pragma unroll
                for (int k = RT; k >= 1; --k) dt[m][e] = dt[m][e] + (x[RT + m - k] - x[RT + m + k]) * h[k];
            }
        }
#pragma unroll
        for (int m = 0; m < M; ++m) k0_store<F, V>(dt[m], D0 + m * dstride + gi * V);
    }
}

// The NEXT frame's temporal derivative, computed inside the current frame's K5c (frame
// pipelining, of3d_plan_execute_next): the K0 stage is pure HBM streaming and K5c is VALU-bound,
// so its loads ride in K5c's memory slack instead of taking a launch of their own.
template <typename F>
struct K0Next {
    Frames fr;        // frames c-rt .. c+rt of the next output frame
    size_t off0;      // element offset of the first voxel (plane zb0) in each frame
    size_t ngroups;   // vector groups of K0Vec<T>::V voxels
    const F* ht;      // temporal taps h[0 .. rt]
    F* D0;            // its dt0 (the plan's dt0 field, origin zb0)
};

// ---------------------------------------------------------------------------
// K1: y and x passes of the gradient filters (calc_flow.py:279-288, y first):
//   A1 = y(G)[dt0], A2 = y(D)[I], A3 = y(S)[I]
//   B1 = x(G)[A1] (dt), B2 = x(S)[A2] (dy), B3 = x(D)[A3] (dx), B4 = x(S)[A3] (dz)
// Block = one 64-wide staged column strip (64 - 2rd output columns) x K1_TY
// output rows, walking K1_NZB planes; lane = staged column.  The next plane's
// I / dt0 rows are fetched into registers during this plane's passes.  The y
// pass is a ring pass down each lane's column; the x pass reads neighbour
// columns from LDS.
// ---------------------------------------------------------------------------
constexpr int K1_R = 4, K1_TY = 4 * K1_R, K1_NZB = 4;

template <typename T, typename F, int NJ>
__global__ __launch_bounds__(256, 3) void k_grad_xy(const T* __restrict__ Ic, const F* __restrict__ D0, int ny,
                                                 int nx, int nzp, DevTaps<F> tp, F* __restrict__ B, size_t fs,
                                                 int need_b4) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* smem = reinterpret_cast<F*>(smem_raw);
    const int rd = tp.rd, rs = tp.rs;
    const int RH = K1_TY + 2 * rd;
    F* sI = smem;
    F* sT = sI + RH * 64;
    F* sA1 = sT + RH * 64;
    F* sA2 = sA1 + K1_TY * 64;
    F* sA3 = sA2 + K1_TY * 64;
    const int lane = threadIdx.x, w = threadIdx.y;
    const int x0 = blockIdx.x * (64 - 2 * rd), y0 = blockIdx.y * K1_TY;
    const int zb = blockIdx.z * K1_NZB;
    const int nzb = min(K1_NZB, nzp - zb);
    const size_t ps = (size_t)ny * nx;
    const int gx = clampi(x0 - rd + lane, 0, nx - 1);
    int roff[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) roff[j] = clampi(y0 - rd + w + 4 * j, 0, ny - 1) * nx + gx;
    F rI[NJ], rT[NJ];
    auto fetch = [&](int t) {
        const T* ip = Ic + (size_t)(zb + t) * ps;
        const F* dp = D0 + (size_t)(zb + t) * ps;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            if (w + 4 * j < RH) {
                rI[j] = (F)ip[roff[j]];
                rT[j] = dp[roff[j]];
            }
    };
    fetch(0);
    const int gxo = x0 + lane - rd;
    const bool xout = lane >= rd && lane < 64 - rd && gxo < nx;
    for (int t = 0; t < nzb; ++t) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int row = w + 4 * j;
            if (row < RH) {
                sI[row * 64 + lane] = rI[j];
                sT[row * 64 + lane] = rT[j];
            }
        }
        __syncthreads();
        if (t + 1 < nzb) fetch(t + 1);
        {
            F a[K1_R];
            const int base = rd + w * K1_R;
            lds_pass<K1_R, false, false>(sT + lane, 64, base, tp.g, tp.gr, rd, a);
#pragma unroll
            for (int i = 0; i < K1_R; ++i) sA1[(w * K1_R + i) * 64 + lane] = a[i];
            lds_pass<K1_R, true, false>(sI + lane, 64, base, tp.d, tp.dr, rd, a);
#pragma unroll
            for (int i = 0; i < K1_R; ++i) sA2[(w * K1_R + i) * 64 + lane] = a[i];
            lds_pass<K1_R, false, false>(sI + lane, 64, base, tp.s, tp.sr, rs, a);
#pragma unroll
            for (int i = 0; i < K1_R; ++i) sA3[(w * K1_R + i) * 64 + lane] = a[i];
        }
        __syncthreads();
        if (xout) {
            F* bp = B + (size_t)(zb + t) * ps + gxo;
#pragma unroll
            for (int i = 0; i < K1_R; ++i) {
                const int row = w * K1_R + i;
                const int gy = y0 + row;
                if (gy >= ny) break;
                const int c = row * 64 + lane;
                F b1 = sA1[c] * tp.g[0], b2 = sA2[c] * tp.s[0], b3 = sA3[c] * tp.d[0], b4 = sA3[c] * tp.s[0];
                for (int k = rd; k >= 1; --k) {
                    b1 = b1 + (sA1[c - k] + sA1[c + k]) * tp.g[k];
                    b3 = b3 + (sA3[c - k] - sA3[c + k]) * tp.d[k];
                }
                for (int k = rs; k >= 1; --k) {
                    b2 = b2 + (sA2[c - k] + sA2[c + k]) * tp.s[k];
                    b4 = b4 + (sA3[c - k] + sA3[c + k]) * tp.s[k];
                }
                const size_t o = (size_t)gy * nx;
                bp[o] = b1;
                bp[fs + o] = b2;
                bp[2 * fs + o] = b3;
                if (need_b4) bp[3 * fs + o] = b4;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// K2: z pass of the gradients (calc_flow.py:279-288, last pass, axis 0):
//   dt = z(G)[B1], dy = z(S)[B2], dx = z(S)[B3], dz = z(D)[B4]
// One field per block: 64 x-columns of one row, K2_ZC output planes; the
// (K2_ZC + 2r)-plane clamped window is staged in LDS, ring pass per lane.
// ---------------------------------------------------------------------------
constexpr int K2_R = 4, K2_ZC = 4 * K2_R;

template <typename F>
__global__ __launch_bounds__(256) void k_grad_z(const F* __restrict__ B, int zb0, F* __restrict__ G, int zg0, int nzg,
                                                int nz, int ny, int nx, size_t fs, DevTaps<F> tp) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* sm = reinterpret_cast<F*>(smem_raw);
    const int f = blockIdx.z & 3;
    const int zc = blockIdx.z >> 2;
    const F* h = f == 0 ? tp.g : (f == 3 ? tp.d : tp.s);
    const F* hr = f == 0 ? tp.gr : (f == 3 ? tp.dr : tp.sr);
    const int r = (f == 0 || f == 3) ? tp.rd : tp.rs;
    const int H = K2_ZC + 2 * r;
    const int lane = threadIdx.x, g = threadIdx.y;
    const int x = blockIdx.x * 64 + lane;
    const int xs = x < nx ? x : nx - 1;
    const int y = blockIdx.y;
    const int zc0 = zg0 + zc * K2_ZC;
    const size_t ps = (size_t)ny * nx, col = (size_t)y * nx + xs;
    const F* src = B + f * fs + col;
    for (int row = g; row < H; row += 4)
        sm[row * 64 + lane] = src[(size_t)(clampi(zc0 - r + row, 0, nz - 1) - zb0) * ps];
    __syncthreads();
    F out[K2_R];
    if (f == 3)
        lds_pass<K2_R, true>(sm + lane, 64, r + g * K2_R, h, hr, r, out);
    else
        lds_pass<K2_R, false>(sm + lane, 64, r + g * K2_R, h, hr, r, out);
    if (x >= nx) return;
    F* dst = G + f * fs + (size_t)y * nx + x;
#pragma unroll
    for (int i = 0; i < K2_R; ++i) {
        const int zl = zc0 + g * K2_R + i - zg0;
        if (zl < nzg) dst[(size_t)zl * ps] = out[i];
    }
}

// ---------------------------------------------------------------------------
// K3: structure-tensor products + W y pass (calc_flow.py:300-313; 2D :133-141).
// Gradient field index: 0 dt, 1 dy, 2 dx, 3 dz.
// 3D product order: tx ty tz xy xz x2 yz y2 z2 ;  2D: tx ty xy x2 y2.
// Block = 64 x-columns x K3_YC rows of one plane.  Per product: the product
// over the (K3_YC + 2rw)-row clamped halo is staged in LDS (double-buffered;
// the next product's gradient loads are in flight during this product's
// pass), then each thread produces K3_R rows by a register-rotated window.
// ---------------------------------------------------------------------------
constexpr int K3_R = 8, K3_YC = 4 * K3_R;

// Streaming form: a block owns one 64-column strip of one plane and one
// product, and marches down the whole column height K3_STEP rows at a time.
// The LDS window holds rows y' = y0 .. y0 + K3_STEP + 2rw - 1 (y' = y + rw);
// after each step its last 2rw rows move to the front (so every row is
// loaded from memory once, and every tap read is a constant LDS offset); the
// next step's rows are fetched into registers during the current pass.
constexpr int K3_STEP = K3_YC;

template <typename F, int NP, int TJ>  // TJ >= ceil(2rw / 4): window rows each thread carries over
__global__ __launch_bounds__(256) void k_prod_wy(const F* __restrict__ G, F* __restrict__ P, int ny, int nx,
                                                 size_t fs, const F* __restrict__ hw, const F* __restrict__ hwr,
                                                 int rw) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* sm = reinterpret_cast<F*>(smem_raw);
    constexpr int NJ = K3_STEP / 4;  // new rows per thread per step
    const int lane = threadIdx.x, g = threadIdx.y;
    const int x = blockIdx.x * 64 + lane;
    const int xs = x < nx ? x : nx - 1;
    const int p = blockIdx.z % NP;
    const size_t pl = (size_t)(blockIdx.z / NP) * ny * nx;
    // packed product table (4 bits per entry)
    constexpr unsigned long long pa = NP == 9 ? 0x311222312ull : 0x12212ull;  // a[] = {2,1,3,2,2,2,1,1,3} / {2,1,2,2,1}
    constexpr unsigned long long pb = NP == 9 ? 0x313231000ull : 0x12100ull;  // b[] = {0,0,0,1,3,2,3,1,3} / {0,0,1,2,1}
    const F* ga = G + (size_t)((pa >> (4 * p)) & 15u) * fs + pl + xs;
    const F* gb = G + (size_t)((pb >> (4 * p)) & 15u) * fs + pl + xs;
    const int h2 = 2 * rw;
    F* col = sm + lane;
    for (int b = g; b < h2; b += 4) {  // prologue: y' in [0, 2rw)
        const size_t o = (size_t)clampi(b - rw, 0, ny - 1) * nx;
        col[b * 64] = ga[o] * gb[o];
    }
    F ra[NJ], rb[NJ];
    auto fetch = [&](int yp0) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const size_t o = (size_t)clampi(yp0 + g + 4 * j - rw, 0, ny - 1) * nx;
            ra[j] = ga[o];
            rb[j] = gb[o];
        }
    };
    fetch(h2);
    F* o = P + p * fs + pl + x;
    F tl[TJ];
    for (int y0 = 0; y0 < ny; y0 += K3_STEP) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) col[(h2 + g + 4 * j) * 64] = ra[j] * rb[j];
        __syncthreads();
        const bool more = y0 + K3_STEP < ny;
        if (more) fetch(y0 + K3_STEP + h2);
        F out[K3_R];
        lds_pass<K3_R, false, (TJ <= 8)>(col, 64, rw + g * K3_R, hw, hwr, rw, out);
        if (x < nx) {
#pragma unroll
            for (int i = 0; i < K3_R; ++i) {
                const int y = y0 + g * K3_R + i;
                if (y < ny) o[(size_t)y * nx] = out[i];
            }
        }
        if (more) {
#pragma unroll
            for (int j = 0; j < TJ; ++j)
                if (g + 4 * j < h2) tl[j] = col[(K3_STEP + g + 4 * j) * 64];
            __syncthreads();
#pragma unroll
            for (int j = 0; j < TJ; ++j)
                if (g + 4 * j < h2) col[(g + 4 * j) * 64] = tl[j];
        }
    }
}

// ---------------------------------------------------------------------------
// K4: W x pass over NF fields.  Block = 64 rows x K4_TX x-outputs of one
// plane; lane = row, so each thread walks its row with a register-rotated
// window (K4_R outputs) over an LDS tile of odd pitch (conflict-free column
// access); results go back through LDS for coalesced row stores.
// ---------------------------------------------------------------------------
constexpr int K4_R = 8, K4_TX = 4 * K4_R, K4_ROWS = 64;

// Streaming form: a block owns 64 rows of one plane and one field, and marches
// along x K4_TX columns at a time.  The LDS window holds columns
// x' = x0 .. x0 + K4_TX + 2ha - 1 (x' = x + ha) of every row, ha = rw rounded
// up to 16 columns, so every 32-column fetch starts on a 128-byte line (odd
// pitch so lane = row reads are conflict-free); after each step the last 2ha
// columns move to the front.  Results leave through a transposing LDS tile for
// coalesced row stores; the next step's columns are fetched into registers
// during the current pass.
constexpr int k4_halo(int rw) { return (rw + 15) & ~15; }

template <typename F, int NF, int TJ>  // TJ >= ceil(2ha / 32): tail column groups per loader lane
__global__ __launch_bounds__(256, TJ == 1 ? 3 : 2) void k_wx(const F* __restrict__ P, F* __restrict__ Q, int ny,
                                                             int nx, size_t fs, const F* __restrict__ hw,
                                                             const F* __restrict__ hwr, int rw) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* sm = reinterpret_cast<F*>(smem_raw);
    const int ha = k4_halo(rw);
    const int h2 = 2 * ha;
    const int PP = (K4_TX + h2) | 1;
    constexpr int OP = K4_TX + 1;
    F* so = sm + K4_ROWS * PP;  // output tile [row][K4_TX]
    const int lane = threadIdx.x, g = threadIdx.y;
    const int y0 = blockIdx.y * K4_ROWS;
    const int f = blockIdx.z % NF;
    const size_t pl = (size_t)(blockIdx.z / NF) * ny * nx;
    const F* src = P + f * fs + pl;
    F* dst = Q + f * fs + pl;
    // loader mapping: lanes 0..31 / 32..63 -> two rows, 32 consecutive columns
    const int lc = lane & 31, lr = (lane >> 5) + 2 * g;  // rows lr, lr + 8, ..., lr + 56
    int roff[8];  // row offsets (ny * nx < 2^31 per plan)
#pragma unroll
    for (int j = 0; j < 8; ++j) roff[j] = min(y0 + lr + 8 * j, ny - 1) * nx;
    auto colv = [&](int j, int xp) { return src[roff[j] + clampi(xp - ha, 0, nx - 1)]; };
    for (int xp = lc; xp < h2; xp += 32)
#pragma unroll
        for (int j = 0; j < 8; ++j) sm[(lr + 8 * j) * PP + xp] = colv(j, xp);
    F rv[8];
    auto fetch = [&](int xp0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) rv[j] = colv(j, xp0 + lc);
    };
    fetch(h2);
    F tl[TJ][8];
    for (int x0 = 0; x0 < nx; x0 += K4_TX) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sm[(lr + 8 * j) * PP + h2 + lc] = rv[j];
        __syncthreads();
        const bool more = x0 + K4_TX < nx;
        if (more) fetch(x0 + K4_TX + h2);
        F out[K4_R];
        lds_pass<K4_R, false, (TJ > 1)>(sm + lane * PP, 1, ha + g * K4_R, hw, hwr, rw, out);
#pragma unroll
        for (int i = 0; i < K4_R; ++i) so[lane * OP + g * K4_R + i] = out[i];
        if (more) {
#pragma unroll
            for (int t = 0; t < TJ; ++t)
                if (lc + 32 * t < h2)
#pragma unroll
                    for (int j = 0; j < 8; ++j) tl[t][j] = sm[(lr + 8 * j) * PP + K4_TX + lc + 32 * t];
        }
        __syncthreads();
        const int x = x0 + lc;
        if (x < nx)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int y = y0 + lr + 8 * j;
                if (y < ny) dst[(size_t)y * nx + x] = so[(lr + 8 * j) * OP + lc];
            }
        if (more) {
#pragma unroll
            for (int t = 0; t < TJ; ++t)
                if (lc + 32 * t < h2)
#pragma unroll
                    for (int j = 0; j < 8; ++j) sm[(lr + 8 * j) * PP + lc + 32 * t] = tl[t][j];
        }
    }
}

// ---------------------------------------------------------------------------
// K34: products + W y + W x in one pass (calc_flow.py:300-313 y and x passes;
// 2D :133-141), so the W-y result never goes to HBM.
//
// Block = one product of one plane, a column block of CW = blockDim.x staged
// columns (TX outputs + RW halo columns each side, clamped at the volume
// edge), one chunk of rows.  Thread = staged column, marching down its rows:
//   phase A (W y, registers only): the column's products live in a register
//     ring of NR slots (row j in slot (j - y0 + RW) mod NR); the loop is
//     unrolled by NR so every slot index is a compile-time constant, no moves,
//     no LDS reads.  Gradient loads run PD rows ahead (raw ring of PD).  Each
//     step writes its W-y row value into an LDS tile row (S rows per tile).
//   phase B (W x, every S rows): the tile's S rows x TX columns through
//     lds_pass (RB = 4 consecutive columns per item, lane = tile row, odd pitch),
//     results through an LDS out tile to coalesced row stores.
// Blocks are numbered XCD-aware: the blocks of one (plane, row chunk) group
// share blockIdx.x % 8 (one XCD's L2 under round-robin placement), so the four
// gradient rows that 9 products x column blocks read come from one L2.
// ---------------------------------------------------------------------------
constexpr int k34_nr(int rw, int s) { return ((2 * rw + 2 + s - 1) / s) * s; }
// K34 block -> (plane zl, row chunk yc, column block bx, product p).  The linear workgroup id
// b runs on XCD b % 8 (round-robin dispatch), so blocks that should share an L2 share b % 8:
// group g = (plane, run of cpg row chunks) = (b / 8 / mb) * 8 + b % 8, members (chunk in the
// run, product, column block).  (A chunk-major order — each XCD running its planes' row chunks
// one after another — measured slower everywhere, round 4: profiles/r04/ab_k34_cm.txt.)
struct K34Blk {
    int zl, yc, bx, p;
    bool ok;
};
template <int NP>
__device__ __forceinline__ K34Blk k34_block(int nbx, int nyb, int cpg, int ngroups) {
    const int kb = blockIdx.x >> 3, xcd = blockIdx.x & 7;
    K34Blk r;
    const int mb = cpg * NP * nbx;
    const int g = (kb / mb) * 8 + xcd;
    int m = kb % mb;
    r.bx = m % nbx;
    m /= nbx;
    r.p = m % NP;
    const int ycl = m / NP, nyg = (nyb + cpg - 1) / cpg;
    r.zl = g / nyg;
    r.yc = (g % nyg) * cpg + ycl;
    r.ok = g < ngroups && r.yc < nyb;
    return r;
}

// W-y tile row r starts at r cwp + 28 (r / 4): with cwp = 1 (mod 32) every row start is
// r mod 4 (mod 32) elements (bank-conflict-free phase B, see k_prod_wyx)
__host__ __device__ constexpr int k34_row(int r, int cwp) { return r * cwp + 28 * (r / 4); }
__host__ __device__ constexpr int k34_tile(int s, int cwp) { return s * cwp + 28 * (s / 4); }  // per tile buffer
// tile row pitch for a block of tx outputs: its 2 rw halo positions, = 1 (mod 32)
__host__ __device__ constexpr int k34_pitch(int tx, int rw) { return ((tx + 2 * rw + 31) & ~31) + 1; }

// value of lane `lane` (wave-uniform index) of a per-lane F, to every lane of the wave
template <typename F>
__device__ __forceinline__ F bcast_lane(F v, int lane) {
    if constexpr (sizeof(F) == 8) {
        const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, lane);
        const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), lane);
        return __builtin_bit_cast(F, ((unsigned long long)hi << 32) | lo);
    } else {
        return __builtin_bit_cast(F, __builtin_amdgcn_readlane(__builtin_bit_cast(unsigned, v), lane));
    }
}

__device__ __forceinline__ void lds_barrier() {
    // LDS-only barrier: global loads in flight stay in flight (__syncthreads
    // would also drain vmcnt, i.e. the phase-A prefetch)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}


// Raw buffer access (one SGPR descriptor per plane-field, 32-bit SGPR row offset +
// one VGPR lane offset): no per-load 64-bit address VALU, no address VGPRs.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
template <typename F>
__device__ __forceinline__ F buf_ld(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
    if constexpr (sizeof(F) == 8)
        return __builtin_bit_cast(F, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
    else
        return __builtin_bit_cast(F, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
// Buffer stores with the default cache policy (non-temporal stores measured neutral: c3 fp64
// 3.707 vs 3.718 ms, c5 fp32 120.65 vs 120.76; every stored field is re-read by a later kernel).
constexpr int kStAux = 0;
template <typename F>
__device__ __forceinline__ void buf_st(F v, __amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
    if constexpr (sizeof(F) == 8)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), v),
                                              r, voff, soff, kStAux);
    else
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, kStAux);
}
// N consecutive values from registers, as 16-byte stores (N * sizeof(F) a multiple of 16)
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
template <typename F, int N>
__device__ __forceinline__ void buf_st_n(const F (&v)[N], __amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
    constexpr int PER = 16 / (int)sizeof(F);
    if constexpr (N % PER != 0) {  // not whole 16-byte pieces: element stores
#pragma unroll
        for (int i = 0; i < N; ++i) buf_st<F>(v[i], r, voff + i * (unsigned)sizeof(F), soff);
        return;
    }
#pragma unroll
    for (int i = 0; i < N; i += PER) {
        F w[PER];
#pragma unroll
        for (int e = 0; e < PER; ++e) w[e] = v[i + e];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, w), r, voff + i * (unsigned)sizeof(F), soff,
                                               kStAux);
    }
}

// W-xy hand-off layout (K34 writes, K5c reads; csrc/of3d_host.hip picks it per plan).
// zt == 0: field-major planes [z][y][x].  zt > 0 (zt = the workspace's planes): z-tiled
// [y][x / 32][z][32] — K5c's block (32 columns of one row, ZC + 2 RW planes) then reads each field
// window as ONE contiguous run instead of ZC + 2 RW pieces of 256 B a plane apart: the window
// reads alone take 0.385 instead of 0.488 ms at c3, 3.13 instead of 4.0-4.2 ms at c4
// (tools/mb_window.hip).  K34 stores per tile of rows from yb: a buffer descriptor at the tile's
// first row and 32-bit per-lane byte offsets (a tile of S rows spans S nx zt elements), through one
// branch-free formula whose uniform parameters select the layout (a per-store select of the two
// formulas cost the lockstep K34 36 VGPRs: 3 -> 2 waves per SIMD at c2).
struct WxyMap {
    unsigned rs, cm, msk, sh;  // row stride (bytes); column-tile multiplier, mask, shift
};
template <typename F>
__device__ __forceinline__ WxyMap wxy_map(int nx, int zt) {
    constexpr unsigned ES = sizeof(F);
    return zt ? WxyMap{(unsigned)nx * (unsigned)zt * ES, (unsigned)zt * 32u, 31u, 5u}
              : WxyMap{(unsigned)nx * ES, 0u, ~0u, 31u};
}
template <typename F>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wxy_rsrc(F* Qp, int zl, int yb, int ny, int nx, int zt) {
    return zt ? buf_rsrc(Qp + ((size_t)yb * nx * zt + (size_t)zl * 32)) : buf_rsrc(Qp + ((size_t)zl * ny + yb) * nx);
}
// byte offset of row r (of the tile) at column x (x .. x + RB - 1 in one 32-column tile: RB | 32 and
// x a multiple of RB); plain planes: r nx + x (x >> 31 = 0, mask all ones)
template <typename F>
__device__ __forceinline__ unsigned wxy_off(const WxyMap& m, int r, int x) {
    const unsigned ux = (unsigned)x;
    return (unsigned)r * m.rs + ((ux >> m.sh) * m.cm + (ux & m.msk)) * (unsigned)sizeof(F);
}

// OCC: waves per SIMD the register budget is cut for (3: 168 VGPRs; 2: 256, for 8-wave blocks,
// which run one per CU anyway); PDX: gradient prefetch rows (0: as far as OCC 3 allows);
// DB: LDS prefetch distance of the phase-B pass; UQ: staging (below).
template <typename F, int NP, int RW, int S, int RB = 4, int OCC = 3, int PDX = 0, int DB = 2,
          bool UQ = false>
__global__ __launch_bounds__(512, OCC) void k_prod_wyx(const F* __restrict__ G, F* __restrict__ Q, int ny,
                                                       int nx, size_t fs, const F* __restrict__ hw, int tx,
                                                       int nyc, int nbx, int nyb, int cpg, int ngroups, int yb0,
                                                       int yb1, int zt) {
    constexpr int NR = k34_nr(RW, S);
    // gradient prefetch distance (rows): as far as 168 VGPRs (3 waves/SIMD) allow
    constexpr int PD0 = PDX ? PDX : (sizeof(F) == 8 ? (RW >= 18 ? 2 : 4) : (RW >= 18 ? 4 : 8));
    constexpr int PD = PD0;
    // RB: W-x outputs per phase-B item (RB 2 measured slower: c2 +16 %, c3 +15 %; not instantiated)
    constexpr unsigned ES = sizeof(F);
    static_assert(NR % PD == 0 && NR % S == 0, "ring sizes");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* sw = reinterpret_cast<F*>(smem_raw);  // two W-y tiles [2][S][cwp] (tile n in buffer n & 1)
    const int cwp = UQ ? k34_pitch(min(tx, nx), RW) : (int)blockDim.x + 1;
    const int t = threadIdx.x;
    // XCD-aware block decode: group g = (plane, run of cpg row chunks), member m = (chunk in the
    // run, product, column block): one group's blocks share an XCD and are dispatched together
    const K34Blk kbk = k34_block<NP>(nbx, nyb, cpg, ngroups);
    if (!kbk.ok) return;
    const int bx = kbk.bx, p = kbk.p, zl = kbk.zl, yc = kbk.yc;
    // output rows [yb0, yb1) (row-slab plans: the rank's own rows; loads still clamp at [0, ny))
    const int y0 = yb0 + yc * nyc, nrows = min(nyc, yb1 - y0);
    const int xo0 = bx * tx;
    const int txu = min(tx, nx - xo0);  // useful outputs of this block
    // Staged columns, tile position i <-> column xo0 - RW + i.
    // UQ = false: thread t stages column clamp(xo0 - RW + t) at position t, halo positions
    //   outside the volume (mode='nearest') recomputed as duplicates of the edge column
    //   (txu + 2 RW <= blockDim.x by the host's geometry).
    // UQ = true: the block's outputs and their W-x halo inside the volume, each once
    //   ([sxs, sxs + ns), ns <= blockDim.x): thread t holds column sxs + t at position padL + t;
    //   the positions outside the volume are edge replicas copied once per tile (no halo work
    //   at all for a block covering the whole row).
    const int sxs = UQ ? max(xo0 - RW, 0) : xo0 - RW;
    const int ns = UQ ? min(xo0 + txu + RW, nx) - sxs : txu + 2 * RW;
    const int padL = UQ ? sxs - (xo0 - RW) : 0, padR = UQ ? (xo0 + txu + RW) - (sxs + ns) : 0;
    // waves with no staged column leave at once; barriers count only the waves still running
    const int wa = (ns + 63) >> 6, ca = 64 * wa;
    if (t >= ca) return;
    const unsigned vof = (unsigned)clampi(sxs + t, 0, nx - 1) * ES;  // staged column of this thread
    // wave index in an SGPR: the edge-replica branches below are scalar, not exec-masked
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6), ln = t & 63;
    const bool lpad = UQ && padL > 0 && wv == 0;                  // wave 0 holds column 0 in lane 0
    const bool rpad = UQ && padR > 0 && wv == ((ns - 1) >> 6);    // this wave holds column nx - 1
    // UQ: lanes past ns (last wave) compute a duplicate and store it past the row's positions
    // (pitch cwp >= txu + 2 RW + 1; that slot only feeds outputs >= txu, never stored)
    const int wpos = !UQ ? t : (t < ns ? padL + t : padL + ns + padR);
    // W-y result of one row into the tile; the edge replicas are copied once per tile by the
    // wave that wrote the edge column (its own LDS writes are ordered before its reads)
    auto put = [&](F* row, F a) { row[wpos] = a; };
    auto replicas = [&](F* tile) {
        if (lpad) {
#pragma unroll
            for (int r = 0; r < S; ++r) {
                F* row = tile + k34_row(r, cwp);
                const F e = row[padL];
                if (ln < padL) row[ln] = e;
            }
        }
        if (rpad) {
#pragma unroll
            for (int r = 0; r < S; ++r) {
                F* row = tile + k34_row(r, cwp);
                const F e = row[padL + ns - 1];
                if (ln < padR) row[padL + ns + ln] = e;
            }
        }
    };
    constexpr unsigned long long pa = NP == 9 ? 0x311222312ull : 0x12212ull;  // as k_prod_wy
    constexpr unsigned long long pb = NP == 9 ? 0x313231000ull : 0x12100ull;
    const size_t pl = (size_t)zl * ny * nx;
    const auto ra_ = buf_rsrc(G + (size_t)((pa >> (4 * p)) & 15u) * fs + pl);
    const auto rb_ = buf_rsrc(G + (size_t)((pb >> (4 * p)) & 15u) * fs + pl);
    F* const Qp = Q + (size_t)p * fs;
    const WxyMap wm = wxy_map<F>(nx, zt);
    const unsigned rowb = (unsigned)nx * ES;
    F h[RW + 1];
#pragma unroll
    for (int k = 0; k <= RW; ++k) h[k] = hw[k];
    auto rowoff = [&](int idx) { return (unsigned)clampi(y0 - RW + idx, 0, ny - 1) * rowb; };
    F ring[NR], ra[PD], rb[PD];
#pragma unroll
    for (int i = 0; i <= 2 * RW; ++i) {
        const unsigned o = rowoff(i);
        ring[i] = buf_ld<F>(ra_, vof, o) * buf_ld<F>(rb_, vof, o);
    }
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        const unsigned o = rowoff(2 * RW + 1 + i);
        ra[(2 * RW + 1 + i) % PD] = buf_ld<F>(ra_, vof, o);
        rb[(2 * RW + 1 + i) % PD] = buf_ld<F>(rb_, vof, o);
    }
    const int nseg = (txu + RB - 1) / RB;
    // phase B: W x over tile buffer `tile` (rows r < S), RB consecutive outputs per item
    // stored straight from registers (rows [yb, yb + nr) only).  One barrier per tile:
    // the other buffer is being filled by phase A meanwhile.
    // Item -> lane, conflict-free for both LDS read forms (ds_read_b64: 32-lane groups,
    // 64 banks; ds_read2_b64: 16-lane groups, 32 banks): lane bits b5..b0 give row
    // (b3b2) + 4 b5 and segment (b1b0) + 4 b4, and row r starts at rowoff(r) =
    // r cwp + off(r) with rowoff(r) = r mod 4 (mod 32 doubles), so a lane reads at
    // (b3b2) + 4 (b1b0) + 16 b4 (mod 32): 16 distinct mod 16, 32 distinct mod 32.
    // S = 4: rows (b3b2), segment (b1b0) + 4 b4 + 8 b5.
    constexpr int RPW = S < 8 ? S : 8, SPW = 64 / RPW;  // rows / segments per wave-item group
    constexpr int RG = S / RPW;                          // row groups
    const int nsgw = (nseg + SPW - 1) / SPW;
    auto phase_b = [&](const F* tile, int yb, int nr) {
        lds_barrier();
        const auto rq_ = wxy_rsrc(Qp, zl, yb, ny, nx, zt);
        for (int i = t; i < 64 * RG * nsgw; i += ca) {
            const int l = i & 63, wg = i >> 6;
            const int r = (wg % RG) * RPW + ((l >> 2) & 3) + (S >= 8 ? 4 * (l >> 5) : 0);
            const int sg = (wg / RG) * SPW + (l & 3) + 4 * ((l >> 4) & 1) + (S >= 8 ? 0 : 8 * (l >> 5));
            if (sg >= nseg) continue;
            F out[RB];
            lds_pass_c<RB, RW, DB>(tile + k34_row(r, cwp), 1, RW + RB * sg, h, out);
            if (r < nr) {
                // row offset per lane in voffset (a divergent soffset would be a waterfall loop)
                const int c0 = RB * sg;
                const unsigned vo = wxy_off<F>(wm, r, xo0 + c0);
                if (c0 + RB <= txu) {
                    buf_st_n<F, RB>(out, rq_, vo, 0);
                } else {
                    for (int e = 0; e < RB; ++e)
                        if (c0 + e < txu) buf_st<F>(out[e], rq_, vo + e * ES, 0);
                }
            }
        }
    };
    for (int u0 = 0; u0 < nrows; u0 += NR) {
        bool done = false;
        [&]<int... H>(std::integer_sequence<int, H...>) {
            (
                [&] {
                    if (done) return;
                    constexpr int h0 = H * S;
                    F* tile = sw + (((u0 + h0) / S) & 1) * k34_tile(S, cwp);
                    // two rows per step, their tap chains interleaved (ILP: a single chain issues
                    // one fp64 op per dependent latency).  Row j+1's new product lands in row j's
                    // outermost slot, so it is written after row j's first tap.
                    [&]<int... J>(std::integer_sequence<int, J...>) {
                        (
                            [&] {
                                constexpr int j = h0 + 2 * J;  // step within the ring period
                                constexpr int ic = j + 2 * RW + 1, ic1 = ic + 1;
                                ring[ic % NR] = ra[ic % PD] * rb[ic % PD];
                                const unsigned o = rowoff(u0 + ic + PD);
                                ra[ic % PD] = buf_ld<F>(ra_, vof, o);
                                rb[ic % PD] = buf_ld<F>(rb_, vof, o);
                                F p1 = ra[ic1 % PD] * rb[ic1 % PD];
                                const unsigned o1 = rowoff(u0 + ic1 + PD);
                                ra[ic1 % PD] = buf_ld<F>(ra_, vof, o1);
                                rb[ic1 % PD] = buf_ld<F>(rb_, vof, o1);
                                F a0 = ring[(j + RW) % NR] * h[0];
                                F a1 = ring[(j + 1 + RW) % NR] * h[0];
                                a0 = a0 + (ring[j % NR] + ring[(j + 2 * RW) % NR]) * h[RW];
                                a1 = a1 + (ring[(j + 1) % NR] + ring[(j + 1 + 2 * RW) % NR]) * h[RW];
                                ring[ic1 % NR] = p1;  // slot of row j - RW (NR = 2 RW + 2): free now
#pragma unroll
                                for (int k = RW - 1; k >= 1; --k) {
                                    a0 = a0 + (ring[(j + RW - k) % NR] + ring[(j + RW + k) % NR]) * h[k];
                                    a1 = a1 + (ring[(j + 1 + RW - k) % NR] + ring[(j + 1 + RW + k) % NR]) * h[k];
                                }
                                put(tile + k34_row(j % S, cwp), a0);
                                put(tile + k34_row((j + 1) % S, cwp), a1);
                            }(),
                            ...);
                    }(std::make_integer_sequence<int, S / 2>{});
                    const int yb = u0 + h0;
                    if constexpr (UQ) replicas(tile);
                    phase_b(tile, y0 + yb, min(S, nrows - yb));
                    if (yb + S >= nrows) done = true;
                }(),
                ...);
        }(std::make_integer_sequence<int, NR / S>{});
        if (done) break;
    }
}

// K34 with specialised waves (unique staging, 1024 threads): waves 0..7 are producers —
// phase A (products + W y, one staged column per thread, register ring) writing the W-y
// tile — and waves 8..15 consumers — phase B (W x + stores) of the PREVIOUS tile, so the
// producers' gradient loads and the consumers' LDS reads / stores overlap each other's
// arithmetic instead of alternating in lockstep.  One barrier per tile, two tile buffers:
// producers write tile t + 1 while consumers read tile t.  Same arithmetic and order as
// k_prod_wyx (bit-identical).  128-VGPR budget (16 waves per CU): prefetch depth PD.
// Ablation at c3 (round 2, timing-only experiment builds since removed): without the W-xy
// stores 1.13 ms vs 1.72 — but that build had no phase-B arithmetic either (dead code without
// its stores; checked in the device assembly in round 3), i.e. the producers alone; gradient
// loads from one cache-resident row 1.48.  Staging the stores through a wave-private LDS transpose (whole
// rows per store instruction) measured slower (1.88 ms): the 72 B/voxel W-xy hand-off to
// K5c itself, not its access pattern, is the cost.
// (12-wave blocks — 4 consumer waves, 168 VGPRs, deeper prefetch, 8-row tiles — measured
// slower: c3 1.95 vs 1.72 ms, c2 0.27 vs 0.19: the 16-wave occupancy hides more.)
// The producers' two row chains side by side: without the two empty asm fences in phase A the
// scheduler issued half of its ops right behind the op they depend on; with them 2 %.  Same ops,
// same order per chain (bit-identical).  c3 K34 1.665 -> 1.631 ms, c4 equal
// (profiles/r04/ab_k34ilp/).  The packed fp32 kernel spills with it and keeps its form.
// NPW: producer waves (staged columns 64 NPW), the other 16 - NPW consume.  8 + 8 suits a row
// whose blocks stage 512 columns (c3: the whole 512-wide row, no halo); 9 + 7 lets a 1024-wide
// row (c4) take two blocks of 512 outputs + 15 halo columns (527 staged) instead of three of 344
// (374 staged: two of the eight producer waves idle, a third of the consumers' capacity unused).
template <typename F, int NP, int RW, int S, int PD = 2, int DB = 2, int NPW = 8>
__global__ __launch_bounds__(1024) void k_prod_wyx_ws(const F* __restrict__ G, F* __restrict__ Q, int ny, int nx,
                                                      size_t fs, const F* __restrict__ hw, int tx, int nyc, int nbx,
                                                      int nyb, int cpg, int ngroups, int yb0, int yb1, int zt) {
    constexpr int RB = 4, CWA = 64 * NPW, NCT = 1024 - CWA;  // producer threads; consumer threads
    constexpr int NR = k34_nr(RW, S);
    constexpr unsigned ES = sizeof(F);
    static_assert(NR % PD == 0 && NR % S == 0, "ring sizes");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* sw = reinterpret_cast<F*>(smem_raw);  // two W-y tiles [2][S][cwp]
    const int cwp = k34_pitch(min(tx, nx), RW);
    const int t = threadIdx.x;
    const K34Blk kbk = k34_block<NP>(nbx, nyb, cpg, ngroups);
    if (!kbk.ok) return;
    const int bx = kbk.bx, p = kbk.p, zl = kbk.zl, yc = kbk.yc;
    // output rows [yb0, yb1) (row-slab plans: the rank's own rows; loads still clamp at [0, ny))
    const int y0 = yb0 + yc * nyc, nrows = min(nyc, yb1 - y0);
    const int xo0 = bx * tx;
    const int txu = min(tx, nx - xo0);
    const int sxs = max(xo0 - RW, 0);
    const int ns = min(xo0 + txu + RW, nx) - sxs;
    const int padL = sxs - (xo0 - RW), padR = (xo0 + txu + RW) - (sxs + ns);
    const int wa = (ns + 63) >> 6;
    const bool prod = t < CWA;
    // producer waves with no staged column: every wave still takes one barrier per tile
    // (a wave-uniform test, so the whole wave takes this branch)
    if (prod && __builtin_amdgcn_readfirstlane(t >> 6) >= wa) {
        for (int tt = 0; tt < (nrows + S - 1) / S; ++tt) lds_barrier();
        return;
    }
    F h[RW + 1];
#pragma unroll
    for (int k = 0; k <= RW; ++k) h[k] = hw[k];
    const size_t pl = (size_t)zl * ny * nx;
    const unsigned rowb = (unsigned)nx * ES;
    const int ntiles = (nrows + S - 1) / S;
    if (prod) {
        const unsigned vof = (unsigned)clampi(sxs + t, 0, nx - 1) * ES;
        const int wv = __builtin_amdgcn_readfirstlane(t >> 6), ln = t & 63;
        const bool lpad = padL > 0 && wv == 0;
        const bool rpad = padR > 0 && wv == ((ns - 1) >> 6);
        const int wpos = t < ns ? padL + t : padL + ns + padR;
        auto replicas = [&](F* tile) {
            if (lpad) {
#pragma unroll
                for (int r = 0; r < S; ++r) {
                    F* row = tile + k34_row(r, cwp);
                    const F e = row[padL];
                    if (ln < padL) row[ln] = e;
                }
            }
            if (rpad) {
#pragma unroll
                for (int r = 0; r < S; ++r) {
                    F* row = tile + k34_row(r, cwp);
                    const F e = row[padL + ns - 1];
                    if (ln < padR) row[padL + ns + ln] = e;
                }
            }
        };
        constexpr unsigned long long pa = NP == 9 ? 0x311222312ull : 0x12212ull;
        constexpr unsigned long long pb = NP == 9 ? 0x313231000ull : 0x12100ull;
        const auto ra_ = buf_rsrc(G + (size_t)((pa >> (4 * p)) & 15u) * fs + pl);
        const auto rb_ = buf_rsrc(G + (size_t)((pb >> (4 * p)) & 15u) * fs + pl);
        auto rowoff = [&](int idx) { return (unsigned)clampi(y0 - RW + idx, 0, ny - 1) * rowb; };
        F ring[NR], ra[PD], rb[PD];
#pragma unroll
        for (int i = 0; i <= 2 * RW; ++i) {
            const unsigned o = rowoff(i);
            ring[i] = buf_ld<F>(ra_, vof, o) * buf_ld<F>(rb_, vof, o);
        }
#pragma unroll
        for (int i = 0; i < PD; ++i) {
            const unsigned o = rowoff(2 * RW + 1 + i);
            ra[(2 * RW + 1 + i) % PD] = buf_ld<F>(ra_, vof, o);
            rb[(2 * RW + 1 + i) % PD] = buf_ld<F>(rb_, vof, o);
        }
        for (int u0 = 0; u0 < nrows; u0 += NR) {
            bool done = false;
            [&]<int... H>(std::integer_sequence<int, H...>) {
                (
                    [&] {
                        if (done) return;
                        constexpr int h0 = H * S;
                        F* tile = sw + (((u0 + h0) / S) & 1) * k34_tile(S, cwp);
                        [&]<int... J>(std::integer_sequence<int, J...>) {
                            (
                                [&] {
                                    constexpr int j = h0 + 2 * J;
                                    constexpr int ic = j + 2 * RW + 1, ic1 = ic + 1;
                                    ring[ic % NR] = ra[ic % PD] * rb[ic % PD];
                                    const unsigned o = rowoff(u0 + ic + PD);
                                    ra[ic % PD] = buf_ld<F>(ra_, vof, o);
                                    rb[ic % PD] = buf_ld<F>(rb_, vof, o);
                                    F p1 = ra[ic1 % PD] * rb[ic1 % PD];
                                    const unsigned o1 = rowoff(u0 + ic1 + PD);
                                    ra[ic1 % PD] = buf_ld<F>(ra_, vof, o1);
                                    rb[ic1 % PD] = buf_ld<F>(rb_, vof, o1);
                                    F a0 = ring[(j + RW) % NR] * h[0];
                                    F a1 = ring[(j + 1 + RW) % NR] * h[0];
                                    a0 = a0 + (ring[j % NR] + ring[(j + 2 * RW) % NR]) * h[RW];
                                    a1 = a1 + (ring[(j + 1) % NR] + ring[(j + 1 + 2 * RW) % NR]) * h[RW];
                                    ring[ic1 % NR] = p1;
#pragma unroll
                                    for (int k = RW - 1; k >= 1; --k) {
                                        // the two rows' chains side by side (the scheduler otherwise
                                        // runs half the ops back to back on their predecessor)
                                        F s0 = ring[(j + RW - k) % NR] + ring[(j + RW + k) % NR];
                                        F s1 = ring[(j + 1 + RW - k) % NR] + ring[(j + 1 + RW + k) % NR];
                                        asm volatile("" : "+v"(s0), "+v"(s1));
                                        s0 = s0 * h[k];
                                        s1 = s1 * h[k];
                                        asm volatile("" : "+v"(s0), "+v"(s1));
                                        a0 = a0 + s0;
                                        a1 = a1 + s1;
                                    }
                                    tile[k34_row(j % S, cwp) + wpos] = a0;
                                    tile[k34_row((j + 1) % S, cwp) + wpos] = a1;
                                }(),
                                ...);
                        }(std::make_integer_sequence<int, S / 2>{});
                        replicas(tile);
                        lds_barrier();  // tile published; the consumers are done with the other buffer
                        if (u0 + h0 + S >= nrows) done = true;
                    }(),
                    ...);
            }(std::make_integer_sequence<int, NR / S>{});
            if (done) break;
        }
    } else {
        const int tb = t - CWA;
        F* const Qp = Q + (size_t)p * fs;
        const WxyMap wm = wxy_map<F>(nx, zt);
        const int nseg = (txu + RB - 1) / RB;
        constexpr int RPW = S < 8 ? S : 8, SPW = 64 / RPW;
        constexpr int RG = S / RPW;
        const int nsgw = (nseg + SPW - 1) / SPW;
        // 7 consumer waves (9 producers): a tile whose item groups are one more than whole rounds
        // of 7 (a 512-wide row at 4 or 8 rows: 8 groups) would make ONE wave run that group as a
        // second round (its SIMD then carries ~17 % more VALU work per tile than the others); that
        // group's 256 outputs go instead as single outputs to the first 4 consumer waves, one per
        // lane, which spreads them over 4 SIMDs (same arithmetic per output: bit-identical)
        constexpr int NCW = NCT / 64, COLS = SPW * RB;
        const int ngrp = RG * nsgw;
        const bool spread = NPW != 8 && RG == 1 && ngrp % NCW == 1;
        const int nmain = spread ? ngrp - 1 : ngrp;
        for (int tt = 0; tt < ntiles; ++tt) {
            lds_barrier();  // tile tt written
            const F* tile = sw + (tt & 1) * k34_tile(S, cwp);
            const int yb = y0 + tt * S, nr = min(S, nrows - tt * S);
            const auto rq_ = wxy_rsrc(Qp, zl, yb, ny, nx, zt);
            if (spread && tb < RPW * COLS) {  // the leftover group: row tb / COLS, one column per lane
                const int r = tb / COLS, c0 = (ngrp - 1) * COLS + tb % COLS;
                if (c0 < txu) {
                    F o1[1];
                    lds_pass_c<1, RW, DB, false, k34_solo && sizeof(F) == 8>(tile + k34_row(r, cwp), 1, RW + c0, h, o1);
                    if (r < nr) buf_st<F>(o1[0], rq_, wxy_off<F>(wm, r, xo0 + c0), 0);
                }
            }
            for (int i = tb; i < 64 * nmain; i += NCT) {
                const int l = i & 63, wg = i >> 6;
                const int r = (wg % RG) * RPW + ((l >> 2) & 3) + (S >= 8 ? 4 * (l >> 5) : 0);
                const int sg = (wg / RG) * SPW + (l & 3) + 4 * ((l >> 4) & 1) + (S >= 8 ? 0 : 8 * (l >> 5));
                if (sg >= nseg) continue;
                F out[RB];
                lds_pass_c<RB, RW, DB, false, k34_solo && sizeof(F) == 8>(tile + k34_row(r, cwp), 1, RW + RB * sg, h, out);
                if (r < nr) {
                    const int c0 = RB * sg;
                    const unsigned vo = wxy_off<F>(wm, r, xo0 + c0);
                    if (c0 + RB <= txu) {
                        buf_st_n<F, RB>(out, rq_, vo, 0);
                    } else {
                        for (int e = 0; e < RB; ++e)
                            if (c0 + e < txu) buf_st<F>(out[e], rq_, vo + e * ES, 0);
                    }
                }
            }
        }
    }
}

// Packed-fp32 K34 (OF3D_FP32 plans): k_prod_wyx_ws's producer / consumer split on CDNA's
// packed fp32 math (v_pk_mul_f32 / v_pk_add_f32: two lanes of work per instruction, each
// element rounded as the scalar op — bit-identical to the fp32 kernels).  8-wave blocks
// (two per CU): waves 0..3 producers, one PAIR of staged columns per thread (512 staged
// columns), phase A on float2 {column c, c + 1}; waves 4..7 consumers, phase B on float2
// {row 2p, row 2p + 1}.  The W-y tile is stored row-pair interleaved — tile2[p][x] =
// {W-y(2p, x), W-y(2p + 1, x)} — so both phases read and write aligned float2: the
// producer's two rows j, j + 1 of columns c, c + 1 are the pair row j / 2 at x = c, c + 1.
// Pair pitch P2 = 1 (mod 32) float2: the consumers' 4 pairs x 4 segments of a 16-lane
// group hit 32 distinct banks.  Ring, prefetch and tile double-buffering as k_prod_wyx_ws.
template <int NP, int RW, int S, int PD = 2, int DB = 2>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_prod_wyx_pk(const float* __restrict__ G, float* __restrict__ Q, int ny,
                                                     int nx, size_t fs, const float* __restrict__ hw, int tx,
                                                     int nyc, int nbx, int nyb, int cpg, int ngroups, int yb0,
                                                     int yb1, int zt) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    constexpr int RB = 4, NPT = 256;  // outputs per consumer item; producer (= consumer) threads
    constexpr int NR = k34_nr(RW, S);
    static_assert(NR % PD == 0 && NR % S == 0 && S % 2 == 0 && (S == 8 || S == 4), "ring sizes");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    f2* sw = reinterpret_cast<f2*>(smem_raw);  // two tiles [2][S / 2][P2]
    const int P2 = k34_pitch(min(tx, nx), RW);
    const int TB = (S / 2) * P2;  // float2 per tile buffer
    const int t = threadIdx.x;
    const K34Blk kbk = k34_block<NP>(nbx, nyb, cpg, ngroups);
    if (!kbk.ok) return;
    const int bx = kbk.bx, p = kbk.p, zl = kbk.zl, yc = kbk.yc;
    const int y0 = yb0 + yc * nyc, nrows = min(nyc, yb1 - y0);
    const int xo0 = bx * tx;
    const int txu = min(tx, nx - xo0);
    const int sxs = max(xo0 - RW, 0);
    const int ns = min(xo0 + txu + RW, nx) - sxs;
    const int padL = sxs - (xo0 - RW), padR = (xo0 + txu + RW) - (sxs + ns);
    const int npair = (ns + 1) >> 1;  // column pairs staged
    const int wa = (npair + 63) >> 6;
    const bool prod = t < NPT;
    // producer waves with no staged column pair: every wave still takes one barrier per tile
    // (a wave-uniform test, so the whole wave takes this branch)
    if (prod && __builtin_amdgcn_readfirstlane(t >> 6) >= wa) {
        for (int tt = 0; tt < (nrows + S - 1) / S; ++tt) lds_barrier();
        return;
    }
    f2 h[RW + 1];
#pragma unroll
    for (int k = 0; k <= RW; ++k) h[k] = (f2){hw[k], hw[k]};
    const size_t pl = (size_t)zl * ny * nx;
    const unsigned rowb = (unsigned)nx * 4u;
    const int ntiles = (nrows + S - 1) / S;
    if (prod) {
        const int wv = __builtin_amdgcn_readfirstlane(t >> 6), ln = t & 63;
        const bool lpad = padL > 0 && wv == 0;
        const bool rpad = padR > 0 && wv == ((npair - 1) >> 6);
        const int wpos = padL + 2 * t;  // tile column of this thread's first staged column
        auto replicas = [&](f2* tile) {
            if (lpad) {
#pragma unroll
                for (int q = 0; q < S / 2; ++q) {
                    f2* row = tile + q * P2;
                    const f2 e = row[padL];
                    if (ln < padL) row[ln] = e;
                }
            }
            if (rpad) {
#pragma unroll
                for (int q = 0; q < S / 2; ++q) {
                    f2* row = tile + q * P2;
                    const f2 e = row[padL + ns - 1];
                    if (ln < padR) row[padL + ns + ln] = e;
                }
            }
        };
        constexpr unsigned long long pa = NP == 9 ? 0x311222312ull : 0x12212ull;
        constexpr unsigned long long pb = NP == 9 ? 0x313231000ull : 0x12100ull;
        const auto ra_ = buf_rsrc(G + (size_t)((pa >> (4 * p)) & 15u) * fs + pl);
        const auto rb_ = buf_rsrc(G + (size_t)((pb >> (4 * p)) & 15u) * fs + pl);
        auto rowoff = [&](int idx) { return (unsigned)clampi(y0 - RW + idx, 0, ny - 1) * rowb; };
        // the column pair as ONE 8-byte load (dword-aligned buffer load): columns c, c + 1 when
        // both are inside the row, else the row's last two with the last one duplicated (the
        // clamped pair of the scalar form)
        const int cp = sxs + 2 * t;
        const bool dup = cp > nx - 2;
        const unsigned vp = (unsigned)(dup ? nx - 2 : cp) * 4u;
        auto ld2 = [&](const __amdgpu_buffer_rsrc_t& r, unsigned o) {
            f2 v = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, vp, o, 0));
            if (dup) v.x = v.y;
            return v;
        };
        f2 ring[NR], ra[PD], rb[PD];
#pragma unroll
        for (int i = 0; i <= 2 * RW; ++i) {
            const unsigned o = rowoff(i);
            ring[i] = ld2(ra_, o) * ld2(rb_, o);
        }
#pragma unroll
        for (int i = 0; i < PD; ++i) {
            const unsigned o = rowoff(2 * RW + 1 + i);
            ra[(2 * RW + 1 + i) % PD] = ld2(ra_, o);
            rb[(2 * RW + 1 + i) % PD] = ld2(rb_, o);
        }
        for (int u0 = 0; u0 < nrows; u0 += NR) {
            bool done = false;
            [&]<int... H>(std::integer_sequence<int, H...>) {
                (
                    [&] {
                        if (done) return;
                        constexpr int h0 = H * S;
                        f2* tile = sw + (((u0 + h0) / S) & 1) * TB;
                        [&]<int... J>(std::integer_sequence<int, J...>) {
                            (
                                [&] {
                                    constexpr int j = h0 + 2 * J;
                                    constexpr int ic = j + 2 * RW + 1, ic1 = ic + 1;
                                    ring[ic % NR] = ra[ic % PD] * rb[ic % PD];
                                    const unsigned o = rowoff(u0 + ic + PD);
                                    ra[ic % PD] = ld2(ra_, o);
                                    rb[ic % PD] = ld2(rb_, o);
                                    f2 p1 = ra[ic1 % PD] * rb[ic1 % PD];
                                    const unsigned o1 = rowoff(u0 + ic1 + PD);
                                    ra[ic1 % PD] = ld2(ra_, o1);
                                    rb[ic1 % PD] = ld2(rb_, o1);
                                    f2 a0 = ring[(j + RW) % NR] * h[0];
                                    f2 a1 = ring[(j + 1 + RW) % NR] * h[0];
                                    a0 = a0 + (ring[j % NR] + ring[(j + 2 * RW) % NR]) * h[RW];
                                    a1 = a1 + (ring[(j + 1) % NR] + ring[(j + 1 + 2 * RW) % NR]) * h[RW];
                                    ring[ic1 % NR] = p1;
#pragma unroll
                                    for (int k = RW - 1; k >= 1; --k) {
                                        a0 = a0 + (ring[(j + RW - k) % NR] + ring[(j + RW + k) % NR]) * h[k];
                                        a1 = a1 + (ring[(j + 1 + RW - k) % NR] + ring[(j + 1 + RW + k) % NR]) * h[k];
                                    }
                                    // rows j, j + 1 (pair (j % S) / 2) at columns wpos, wpos + 1
                                    // (threads past the staged pairs write nothing: wpos would
                                    // run into the next pair row)
                                    if (t < npair) {
                                        f2* q = tile + ((j % S) / 2) * P2 + wpos;
                                        q[0] = (f2){a0.x, a1.x};
                                        q[1] = (f2){a0.y, a1.y};
                                    }
                                }(),
                                ...);
                        }(std::make_integer_sequence<int, S / 2>{});
                        replicas(tile);
                        lds_barrier();  // tile published; the consumers are done with the other buffer
                        if (u0 + h0 + S >= nrows) done = true;
                    }(),
                    ...);
            }(std::make_integer_sequence<int, NR / S>{});
            if (done) break;
        }
    } else {
        const int tb = t - NPT;
        float* const Qp = Q + (size_t)p * fs;
        const WxyMap wm = wxy_map<float>(nx, zt);
        const int nseg = (txu + RB - 1) / RB;
        constexpr int PP = S / 2, SPW = 64 / PP;  // pairs per tile; segments per wave item
        const int nsgw = (nseg + SPW - 1) / SPW;
        for (int tt = 0; tt < ntiles; ++tt) {
            lds_barrier();  // tile tt written
            const f2* tile = sw + (tt & 1) * TB;
            const int yb = y0 + tt * S, nr = min(S, nrows - tt * S);
            const auto rq_ = wxy_rsrc(Qp, zl, yb, ny, nx, zt);
            for (int i = tb; i < 64 * nsgw; i += NPT) {
                const int l = i & 63, wg = i >> 6;
                const int pr = l % PP, sg = wg * SPW + l / PP;
                if (sg >= nseg) continue;
                f2 out[RB];
                lds_pass_c<RB, RW, DB>(tile + pr * P2, 1, RW + RB * sg, h, out);
                const int c0 = RB * sg;
#pragma unroll
                for (int e2 = 0; e2 < 2; ++e2) {
                    const int r = 2 * pr + e2;
                    if (r < nr) {
                        float o[RB];
#pragma unroll
                        for (int e = 0; e < RB; ++e) o[e] = e2 ? out[e].y : out[e].x;
                        const unsigned vo = wxy_off<float>(wm, r, xo0 + c0);
                        if (c0 + RB <= txu) {
                            buf_st_n<float, RB>(o, rq_, vo, 0);
                        } else {
                            for (int e = 0; e < RB; ++e)
                                if (c0 + e < txu) buf_st<float>(o[e], rq_, vo + e * 4u, 0);
                        }
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// K2c: the gradient z pass (calc_flow.py:279-288, axis 0) as a z march: thread = one
// (y, x) column, lanes along x (coalesced), marching a chunk of zc output planes with a
// register ring of NR planes per field (compile-time slots, as K34); no LDS, no
// barriers, every input plane read once per chunk.  dt = z(G)[B1], dy = z(S)[B2],
// dx = z(S)[B3], dz = z(D)[B4], same order as k_grad_z: bit-identical.
// ---------------------------------------------------------------------------
template <typename F, int RD, int RS>
__global__ __launch_bounds__(256, 3) void k_grad_z_c(const F* __restrict__ B, int zb0, F* __restrict__ G, int zg0,
                                                     int nzg, int nz, int plane, size_t fs, DevTaps<F> tp, int zc) {
    constexpr int NR = ((2 * RD + 2 + 7) / 8) * 8, PD = 4;
    static_assert(NR % PD == 0 && RS <= RD, "ring sizes");
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= plane) return;
    const int zc0 = zg0 + blockIdx.y * zc;
    const int nrows = min(zc, zg0 + nzg - zc0);
    F hg[RD + 1], hd[RD + 1], hs[RS + 1];
#pragma unroll
    for (int k = 0; k <= RD; ++k) hg[k] = tp.g[k], hd[k] = tp.d[k];
#pragma unroll
    for (int k = 0; k <= RS; ++k) hs[k] = tp.s[k];
    const F* b = B + col;
    F* g = G + col;
    auto src = [&](int idx) { return (size_t)(clampi(zc0 - RD + idx, 0, nz - 1) - zb0) * plane; };
    F ring[4][NR], raw[4][PD];
#pragma unroll
    for (int i = 0; i <= 2 * RD; ++i) {
        const size_t o = src(i);
#pragma unroll
        for (int f = 0; f < 4; ++f) ring[f][i] = b[f * fs + o];
    }
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        const size_t o = src(2 * RD + 1 + i);
#pragma unroll
        for (int f = 0; f < 4; ++f) raw[f][(2 * RD + 1 + i) % PD] = b[f * fs + o];
    }
    for (int u0 = 0; u0 < nrows; u0 += NR) {
        bool done = false;
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (
                [&] {
                    if (done) return;
                    constexpr int j = J;
                    constexpr int ic = j + 2 * RD + 1, c = (j + RD) % NR;
                    const size_t o = src(u0 + ic + PD);
#pragma unroll
                    for (int f = 0; f < 4; ++f) {
                        ring[f][ic % NR] = raw[f][ic % PD];
                        raw[f][ic % PD] = b[f * fs + o];
                    }
                    F o0 = ring[0][c] * hg[0], o3 = ring[3][c] * hd[0];
                    F o1 = ring[1][c] * hs[0], o2 = ring[2][c] * hs[0];
#pragma unroll
                    for (int k = RD; k >= 1; --k) {
                        o0 = o0 + (ring[0][(j + RD - k) % NR] + ring[0][(j + RD + k) % NR]) * hg[k];
                        o3 = o3 + (ring[3][(j + RD - k) % NR] - ring[3][(j + RD + k) % NR]) * hd[k];
                    }
#pragma unroll
                    for (int k = RS; k >= 1; --k) {
                        o1 = o1 + (ring[1][(j + RD - k) % NR] + ring[1][(j + RD + k) % NR]) * hs[k];
                        o2 = o2 + (ring[2][(j + RD - k) % NR] + ring[2][(j + RD + k) % NR]) * hs[k];
                    }
                    const size_t d = (size_t)(zc0 + u0 + j - zg0) * plane;
                    g[d] = o0;
                    g[fs + d] = o1;
                    g[2 * fs + d] = o2;
                    g[3 * fs + d] = o3;
                    if (u0 + j + 1 >= nrows) done = true;
                }(),
                ...);
        }(std::make_integer_sequence<int, NR>{});
        if (done) break;
    }
}

// ---------------------------------------------------------------------------
// K1c: K1 as a column march (the K34 scheme, calc_flow.py:279-288 y and x passes):
// thread = staged column of one plane (RD halo columns each side), marching its rows.
// Register rings of the centre frame I and of dt0 (NR rows, compile-time slots) give
// the y passes A1 = y(G)[dt0], A2 = y(D)[I], A3 = y(S)[I] with no LDS reads; each row
// lands in three LDS tiles (double-buffered, S rows).  Every S rows the x passes
// B1 = x(G)[A1] (dt), B2 = x(S)[A2] (dy), B3 = x(D)[A3] (dx), B4 = x(S)[A3] (dz)
// run over the tile with lds_pass_c (same item -> lane map as k_prod_wyx) and store
// from registers.  Same expression order as k_grad_xy: bit-identical.
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T buf_ld_raw(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
    if constexpr (sizeof(T) == 1)
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b8(r, voff, soff, 0));
    else if constexpr (sizeof(T) == 2)
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0));
    else
        return buf_ld<T>(r, voff, soff);
}

template <typename T, typename F, int RD, int RS, int S>
__global__ __launch_bounds__(256, 3) void k_grad_xy_c(const T* __restrict__ Ic, const F* __restrict__ D0, int ny,
                                                      int nx, DevTaps<F> tp, F* __restrict__ B, size_t fs,
                                                      int need_b4, int tx, int nyc, int nbx, int nyb) {
    constexpr int NR = ((2 * RD + 2 + S - 1) / S) * S;
    constexpr int PD = NR % 8 == 0 ? 8 : 4;
    constexpr int RB = 4;
    constexpr unsigned ES = sizeof(F);
    static_assert(NR % PD == 0 && NR % S == 0 && RS <= RD, "ring sizes");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* sm = reinterpret_cast<F*>(smem_raw);  // [2 buffers][3 tiles][k34_tile(S, cwp)]
    const int cw = blockDim.x, cwp = cw + 1, tl = k34_tile(S, cwp);
    const int t = threadIdx.x;
    int b = blockIdx.x;
    const int bx = b % nbx;
    b /= nbx;
    const int yc = b % nyb, z = b / nyb;
    const int y0 = yc * nyc, nrows = min(nyc, ny - y0);
    const int xo0 = bx * tx;
    const int txu = min(tx, nx - xo0);
    const int wa = (min(cw, txu + 2 * RD) + 63) >> 6, ca = 64 * wa;
    if (t >= ca) return;
    const size_t ps = (size_t)ny * nx;
    const unsigned gx = (unsigned)clampi(xo0 - RD + t, 0, nx - 1);
    const auto ri_ = buf_rsrc(Ic + (size_t)z * ps);
    const auto rt_ = buf_rsrc(D0 + (size_t)z * ps);
    F* bz = B + (size_t)z * ps + xo0;
    const auto rb0 = buf_rsrc(bz), rb1 = buf_rsrc(bz + fs), rb2 = buf_rsrc(bz + 2 * fs), rb3 = buf_rsrc(bz + 3 * fs);
    F hg[RD + 1], hd[RD + 1], hs[RS + 1];
#pragma unroll
    for (int k = 0; k <= RD; ++k) hg[k] = tp.g[k], hd[k] = tp.d[k];
#pragma unroll
    for (int k = 0; k <= RS; ++k) hs[k] = tp.s[k];
    auto row = [&](int idx) { return (unsigned)clampi(y0 - RD + idx, 0, ny - 1) * (unsigned)nx; };
    F ri[NR], rt[NR], pt[PD];
    T pi[PD];
#pragma unroll
    for (int i = 0; i <= 2 * RD; ++i) {
        const unsigned o = row(i);
        ri[i] = (F)buf_ld_raw<T>(ri_, gx * (unsigned)sizeof(T), o * (unsigned)sizeof(T));
        rt[i] = buf_ld<F>(rt_, gx * ES, o * ES);
    }
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        const unsigned o = row(2 * RD + 1 + i);
        pi[(2 * RD + 1 + i) % PD] = buf_ld_raw<T>(ri_, gx * (unsigned)sizeof(T), o * (unsigned)sizeof(T));
        pt[(2 * RD + 1 + i) % PD] = buf_ld<F>(rt_, gx * ES, o * ES);
    }
    const int nseg = (txu + RB - 1) / RB;
    constexpr int RPW = S < 8 ? S : 8, SPW = 64 / RPW, RG = S / RPW;
    const int nsgw = (nseg + SPW - 1) / SPW;
    const unsigned rowb = (unsigned)nx * ES;
    auto store = [&](const F (&v)[RB], __amdgpu_buffer_rsrc_t rs, unsigned vo, int c0) {
        if (c0 + RB <= txu) {
            buf_st_n<F, RB>(v, rs, vo, 0);
        } else {
            for (int e = 0; e < RB; ++e)
                if (c0 + e < txu) buf_st<F>(v[e], rs, vo + e * ES, 0);
        }
    };
    auto phase_b = [&](const F* tiles, int yb, int nr) {
        lds_barrier();
        for (int i = t; i < 64 * RG * nsgw; i += ca) {
            const int l = i & 63, wg = i >> 6;
            const int r = (wg % RG) * RPW + ((l >> 2) & 3) + (S >= 8 ? 4 * (l >> 5) : 0);
            const int sg = (wg / RG) * SPW + (l & 3) + 4 * ((l >> 4) & 1) + (S >= 8 ? 0 : 8 * (l >> 5));
            if (sg >= nseg || r >= nr) continue;
            const int c0 = RB * sg, base = RD + RB * sg;
            const unsigned vo = (unsigned)(yb + r) * rowb + (unsigned)c0 * ES;
            const int ro = k34_row(r, cwp);
            F o[RB];
            lds_pass_c<RB, RD, 2>(tiles + ro, 1, base, hg, o);  // dt
            store(o, rb0, vo, c0);
            lds_pass_c<RB, RS, 2>(tiles + tl + ro, 1, base, hs, o);  // dy
            store(o, rb1, vo, c0);
            lds_pass_c<RB, RD, 2, true>(tiles + 2 * tl + ro, 1, base, hd, o);  // dx
            store(o, rb2, vo, c0);
            if (need_b4) {
                lds_pass_c<RB, RS, 2>(tiles + 2 * tl + ro, 1, base, hs, o);  // dz (pre-z)
                store(o, rb3, vo, c0);
            }
        }
    };
    for (int u0 = 0; u0 < nrows; u0 += NR) {
        bool done = false;
        [&]<int... H>(std::integer_sequence<int, H...>) {
            (
                [&] {
                    if (done) return;
                    constexpr int h0 = H * S;
                    F* tiles = sm + (((u0 + h0) / S) & 1) * (3 * tl);
                    [&]<int... J>(std::integer_sequence<int, J...>) {
                        (
                            [&] {
                                constexpr int j = h0 + J;
                                constexpr int ic = j + 2 * RD + 1;
                                ri[ic % NR] = (F)pi[ic % PD];
                                rt[ic % NR] = pt[ic % PD];
                                const unsigned o = row(u0 + ic + PD);
                                pi[ic % PD] = buf_ld_raw<T>(ri_, gx * (unsigned)sizeof(T), o * (unsigned)sizeof(T));
                                pt[ic % PD] = buf_ld<F>(rt_, gx * ES, o * ES);
                                constexpr int c = (j + RD) % NR;
                                F a1 = rt[c] * hg[0], a2 = ri[c] * hd[0], a3 = ri[c] * hs[0];
#pragma unroll
                                for (int k = RD; k >= 1; --k) {
                                    a1 = a1 + (rt[(j + RD - k) % NR] + rt[(j + RD + k) % NR]) * hg[k];
                                    a2 = a2 + (ri[(j + RD - k) % NR] - ri[(j + RD + k) % NR]) * hd[k];
                                }
#pragma unroll
                                for (int k = RS; k >= 1; --k)
                                    a3 = a3 + (ri[(j + RD - k) % NR] + ri[(j + RD + k) % NR]) * hs[k];
                                const int ro = k34_row(j % S, cwp) + t;
                                tiles[ro] = a1;
                                tiles[tl + ro] = a2;
                                tiles[2 * tl + ro] = a3;
                            }(),
                            ...);
                    }(std::make_integer_sequence<int, S>{});
                    const int yb = u0 + h0;
                    phase_b(tiles, y0 + yb, min(S, nrows - yb));
                    if (yb + S >= nrows) done = true;
                }(),
                ...);
        }(std::make_integer_sequence<int, NR / S>{});
        if (done) break;
    }
}

// 16-byte global -> LDS copy (LDS-DMA): lane i's 16 bytes land at lds_byte + 16 i.
// Inline asm keeps it out of the compiler's wait bookkeeping (the compiler
// would drain it with vmcnt(0) before every LDS read); waits are explicit.
__device__ __forceinline__ void glds16(const void* src, unsigned lds_byte) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_byte)
                 : "memory");
}

// ---------------------------------------------------------------------------
// K12: the gradient y, x and z passes in one kernel (calc_flow.py:279-288) — the four
// pre-z fields never leave the CU (K1c + K2c write and re-read them through HBM).
// Block = TY = 4 rows x TX = CW - 2 RD output columns (CW = 64 NWX staged columns: NWX waves
// per row, 3 in fp64, 2 in fp32), marching a chunk of output planes.  Wave w: part h = w % NWX
// (staged column c = 64 h + lane), role / row r = w / NWX.  Per input plane (one step):
//   staging (LDS-DMA): the plane's TY + 2 RD rows of dt0 and of the centre frame I (the
//     block's staged columns, 16-byte granules) go straight into LDS, a chunk of K (3, 2 or 1
//     where LDS is short) planes at a time, two chunks ahead (2 K plane slots): one chunk's loads
//     stay in flight while the previous chunk computes; one vmcnt(0) per chunk;
//   y passes (LDS -> registers): role 0 A1 = y(G)[dt0], role 1 A2 = y(D)[I], role 2
//     A3 = y(S)[I] of the thread's staged column (clamped at the global edge), results
//     into LDS tiles (two buffers);
//   x passes (LDS): thread (row r, staged column c) forms B1 = x(G)[A1], B2 = x(S)[A2],
//     B3 = x(D)[A3], B4 = x(S)[A3] for output column c - RD (lanes past the block's
//     outputs compute clamped duplicates and store nothing);
//   z passes (registers): B1..B4 enter per-thread register rings (NR = 2 RD + 2 slots for
//     the radius-RD fields, NRS = RD + 1 for the smooth ones; compile-time slots: the plane
//     loop is unrolled by NR); dt = z(G)[B1] and dz = z(D)[B4] leave once plane q + RD is
//     in, dy = z(S)[B2] and dx = z(S)[B3] once plane q + RS is.
// One barrier per step; the y passes of step s + 1 run beside the x / z passes of step s
// (the A tiles alternate), so each wave has two independent streams of work per step.
// Same expression order as K1c + K2c (scipy's), staged rows/columns clamped at the global
// edge, planes clamped to [0, nzc): bit-identical.  Blocks are numbered XCD-aware (the
// tiles of one XCD form a band of rows, so the halo rows of neighbouring tiles share an L2).
// Needs nx * sizeof(F) and nx * sizeof(T) multiples of 16 bytes and 16-byte aligned planes.
// ---------------------------------------------------------------------------
constexpr int K12_TY = 4;  // rows per block
// staged columns per block row: 64 per wave, k12_nwx waves per row.  fp64: 3 waves (192
// staged columns, 180 outputs at rd 6): 12-wave blocks = 3 waves per SIMD instead of 2 (the
// kernel is bound by each wave's dependent chain, so a third wave per SIMD is what pays), at
// 168 VGPRs (one x window live at a time) and one plane per DMA chunk (LDS); and 5 % of the
// staged columns of a 512-wide plane wasted instead of 13 %.  Same box: c3 K12 0.617 -> 0.462
// ms, c4 4.09 -> 3.37 ms (profiles/r04/ab_k12n3/).  fp32 keeps 2 (two 8-wave blocks per CU).
template <typename F>
__host__ __device__ constexpr int k12_nwx() { return sizeof(F) == 8 ? 3 : 2; }
template <typename F>
__host__ __device__ constexpr int k12_cw() { return 64 * k12_nwx<F>(); }
template <typename F>
__host__ __device__ constexpr int k12_threads() { return k12_cw<F>() * K12_TY; }
// z passes one step late (k_grad_xyz_c) in the fp32 kernels: c5 K12 18.2-18.5 -> 17.4 ms; the
// fp64 kernel measured slower so (c3 0.602 -> 0.645 ms, same box, profiles/r03_ab/k12_defer/)
template <typename F>
constexpr bool k12_defer() { return sizeof(F) == 4; }
template <typename F, int RD>
__host__ __device__ constexpr int k12_tx() { return k12_cw<F>() - 2 * RD; }
// LDS bytes of one staged plane: NRW rows of dt0 (CW + EPL columns) and of I (CW + EPL_T)
template <typename T, typename F, int RD>
__host__ __device__ constexpr int k12_slot_granules() {
    return (K12_TY + 2 * RD) * ((k12_cw<F>() * (int)sizeof(F)) / 16 + 1 + (k12_cw<F>() * (int)sizeof(T)) / 16 + 1);
}
template <typename T, typename F, int RD>
__host__ __device__ constexpr int k12_slot_bytes() { return ((k12_slot_granules<T, F, RD>() + 63) / 64) * 1024; }
// A tiles: [2 buffers][3 fields][even / odd copy][TY][AP]; the odd copy is the row
// shifted by one element, so every x-pass window starts 16-byte aligned in one of the two
// (pairs read as ds_read_b128: 4 LDS cycles per 16 B; ds_read2_b64 costs 16).  Pitch
// CW + 4 (132 / 196): the odd copy sits 128 B (mod 256) from the even one (conflict-free
// b128 groups).
template <typename F>
__host__ __device__ constexpr int k12_ap() { return k12_cw<F>() + 4; }
// fp64 (round 6): ONE copy per A row; the x windows read single 8-byte elements (ds_read_b64:
// 2 LDS cycles per 512 B, the b128 rate; kept from pairing into ds_read2_b64 by empty fences) —
// half the y-pass LDS writes and half the A-tile bytes, which buys the third DMA slot below.
// fp32 keeps the odd-shifted copies (its 4-byte reads would run at half rate).
constexpr bool k12_odd_fp64 = false;
constexpr bool k12_ysolo = true;  // fp64 y-pass reads of dt0 as single ds_read_b64s
template <typename F>
__host__ __device__ constexpr bool k12_odd() { return sizeof(F) == 4 || k12_odd_fp64; }
template <typename F>
__host__ __device__ constexpr int k12_a_bytes() {
    return 2 * 3 * (k12_odd<F>() ? 2 : 1) * K12_TY * k12_ap<F>() * (int)sizeof(F);
}
// planes per DMA chunk: 2 where two chunks of slots + the A tiles fit 80 KiB and the
// kernel's registers allow 4 waves per SIMD (fp32 rd 3 / 6: two 8-wave blocks per CU),
// else 3 where they fit 160 KiB, else 2
template <typename T, typename F, int RD>
__host__ __device__ constexpr int k12_k() {
    if (sizeof(F) == 4 && RD <= 6 && 4 * k12_slot_bytes<T, F, RD>() + k12_a_bytes<F>() <= 80 * 1024)
        return 2;
    if (6 * k12_slot_bytes<T, F, RD>() + k12_a_bytes<F>() <= 160 * 1024) return 3;
    return 4 * k12_slot_bytes<T, F, RD>() + k12_a_bytes<F>() <= 160 * 1024 ? 2 : 1;
}
// chunks of DMA slots: DEEP instances 3 (each plane's loads get two steps to land) for one-plane
// chunks of the non-deferred (fp64) kernel where three slots fit beside the A tiles, else 2 (one
// step).  The host takes DEEP for marches of >= 128 planes: same box, c4 (256-plane marches) K12
// 3.19 -> 3.10 ms; c3 (64) equal; c2 (32) 0.088 -> 0.091 (profiles/r06/abk12/)
template <typename T, typename F, int RD, bool DEEP>
__host__ __device__ constexpr int k12_nch() {
    return DEEP && !k12_defer<F>() && k12_k<T, F, RD>() == 1 &&
                   3 * k12_slot_bytes<T, F, RD>() + k12_a_bytes<F>() <= 160 * 1024
               ? 3
               : 2;
}
template <typename T, typename F, int RD, bool DEEP = false>
__host__ __device__ constexpr int k12_lds_bytes() {
    return k12_nch<T, F, RD, DEEP>() * k12_k<T, F, RD>() * k12_slot_bytes<T, F, RD>() + k12_a_bytes<F>();
}

template <typename T, typename F, int RD, int RS, bool DEEP = false>
__global__ __launch_bounds__(k12_threads<F>()) void k_grad_xyz_c(const T* __restrict__ Ic, const F* __restrict__ D0,
                                                             int zin0, int nzc, int ny, int nx, DevTaps<F> tp,
                                                             F* __restrict__ G, size_t fs, int zg0, int q0, int nq,
                                                             int zc, int ntile, int nbx) {
    constexpr int TY = K12_TY, TX = k12_tx<F, RD>(), NRW = TY + 2 * RD, CW = k12_cw<F>();
    constexpr int NWX = k12_nwx<F>(), NWV = NWX * TY;  // waves per row; per block
    constexpr int NR = 2 * RD + 2, NRS = RD + 1, AP = k12_ap<F>();  // ring slots; A tile pitch
    constexpr bool ODD = k12_odd<F>();
    constexpr int AF = (ODD ? 2 : 1) * TY * AP, AB = 3 * AF;  // A field stride (even [+ odd] copy), buffer stride
    static_assert(NRS >= 2 * RS + 1 && NR % NRS == 0 && NR % 2 == 0 && TX >= 8, "K12 geometry");
    constexpr int EF = 16 / (int)sizeof(F), ET = 16 / (int)sizeof(T);  // elements per granule
    constexpr int GD = CW / EF + 1, GI = CW / ET + 1;                   // granules per staged row
    constexpr int NG = NRW * (GD + GI), NJ = (NG + 63) / 64;            // granules / DMA instrs per plane
    constexpr int K = k12_k<T, F, RD>();  // planes per DMA chunk
    constexpr int NCH = k12_nch<T, F, RD, DEEP>();  // chunks of slots (DMA issued NCH - 1 chunks ahead)
    constexpr int SLOT = k12_slot_bytes<T, F, RD>(), NSLOT = NCH * K;
    static_assert(k12_lds_bytes<T, F, RD, DEEP>() <= 160 * 1024, "K12 LDS");
    constexpr int NJW = (NJ + NWV - 1) / NWV;                           // DMA instrs per wave per plane
    constexpr int NJMIN = NJ / NWV;  // ... on the waves with the fewest (NJW - 1 or NJW)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* At = reinterpret_cast<F*>(smem_raw + NSLOT * SLOT);  // [2 buffers][3 fields][even, odd][TY][AP]
    const int t = threadIdx.x, lane = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    // (row role, column part) of wave w, as rp = role * NWX + part: fp64 spreads the roles' work
    // evenly over the SIMDs (wave w runs on SIMD w % 4; roles 0 / 1 / 2 / 3 do 180 / 180 / 132 /
    // 104 fp64 ops per step): SIMDs get roles {0,0,3} {1,1,3} {0,2,3} {1,2,2} instead of {0,1,2}
    // {0,1,3} {0,2,3} {1,2,3} (busiest SIMD 464 instead of 492 ops per step).  Same box: c3 K12
    // 0.445 / 0.447 -> 0.435 / 0.438 ms, c4 3.26 -> 3.22, c2 0.089 -> 0.087 (profiles/r05/ab_k12_perm/)
    const int rp = NWX == 3 ? (int)((0x8ba976415230ull >> (4 * w)) & 15u) : w;
    const int role = rp / NWX, c = 64 * (rp % NWX) + lane;
    const int per = (ntile + 7) >> 3;
    const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (tile >= ntile) return;  // block-uniform
    const int by = tile / nbx, bx = tile - by * nbx;
    const int y0 = by * TY, x0 = bx * TX;
    const int qa = q0 + (int)blockIdx.y * zc, nout = min(zc, q0 + nq - qa);
    const size_t plane = (size_t)ny * nx;
    // staged columns: dt0 from gd0, I from gi0 (granule-aligned starts of the block's window)
    const int xs = max(x0 - RD, 0);
    const int gd0 = xs / EF * EF, gi0 = xs / ET * ET;
    const int gc = clampi(x0 - RD + c, 0, nx - 1);  // this thread's staged column (y passes)
    const int pd = gc - gd0, pi = gc - gi0;         // its LDS positions in the dt0 / I rows
    // DMA sources of this wave's instructions (plane-relative element offsets): instruction
    // j = w + NWV i covers granules 64 j .. 64 j + 63 of the slot (dt0 rows, then I rows)
    unsigned doff[NJW];
    bool isd[NJW];
#pragma unroll
    for (int i = 0; i < NJW; ++i) {
        const int g = min(64 * (w + NWV * i) + lane, NG - 1);
        if (g < NRW * GD) {
            const int r = g / GD, q = g - r * GD;
            isd[i] = true;
            doff[i] = (unsigned)clampi(y0 - RD + r, 0, ny - 1) * (unsigned)nx + (unsigned)min(gd0 + q * EF, nx - EF);
        } else {
            const int gg = g - NRW * GD, r = gg / GI, q = gg - r * GI;
            isd[i] = false;
            doff[i] = (unsigned)clampi(y0 - RD + r, 0, ny - 1) * (unsigned)nx + (unsigned)min(gi0 + q * ET, nx - ET);
        }
    }
    const unsigned lds0 = (unsigned)(uintptr_t)smem_raw;
    const int nsteps = nout + 2 * RD;
    auto issue_plane = [&](int s) {  // DMA of step s's plane into slot s % NSLOT
        const size_t pz = (size_t)(clampi(qa - RD + s, 0, nzc - 1) - zin0) * plane;
        const unsigned sb = lds0 + (unsigned)((s % NSLOT) * SLOT);
#pragma unroll
        for (int i = 0; i < NJW; ++i) {
            if (w + NWV * i < NJ) {
                const void* src = isd[i] ? (const void*)(D0 + pz + doff[i]) : (const void*)(Ic + pz + doff[i]);
                glds16(src, __builtin_amdgcn_readfirstlane(sb + (unsigned)((w + NWV * i) * 1024)));
            }
        }
    };
    auto issue_chunk = [&](int m) {
        for (int s = m * K; s < min((m + 1) * K, nsteps); ++s) issue_plane(s);
    };
    F hg[RD + 1], hd[RD + 1], hs[RS + 1];
#pragma unroll
    for (int k = 0; k <= RD; ++k) hg[k] = tp.g[k], hd[k] = tp.d[k];
#pragma unroll
    for (int k = 0; k <= RS; ++k) hs[k] = tp.s[k];
    // x / z passes: output column x0 + c - RD (reads clamped into the block's outputs);
    // stores of lanes outside the volume are skipped
    const int cx = clampi(c, RD, RD + TX - 1);
    const int xo = x0 + c - RD, yo = y0 + role;
    const bool st_ok = c >= RD && c < RD + TX && xo < nx && yo < ny;
    constexpr unsigned ES = sizeof(F);
    const unsigned vout = (unsigned)(xo < 0 ? 0 : xo) * ES, sout = (unsigned)(yo < ny ? yo : 0) * (unsigned)nx * ES;
    F r1[NR], r2[NRS], r3[NRS], r4[NR];  // z rings of B1 .. B4
    // ---- y passes of step s (roles 0..2): staged rows of slot s % NSLOT -> A tile s & 1 ----
    auto ypass_step = [&](int s, int par) {
        F* A = At + par * AB;
        const unsigned char* slot = smem_raw + (s % NSLOT) * SLOT;
        auto ypass = [&]<int R, bool ANTI, bool DT>(const F(&h)[R + 1]) {
            F v[NRW];
            if constexpr (DT) {
                const F* rd_ = reinterpret_cast<const F*>(slot) + pd;
#pragma unroll
                for (int i = 0; i < NRW; ++i) {
                    v[i] = rd_[i * GD * EF];
                    // fp64: single ds_read_b64s, not pairs of rows in ds_read2_b64 (half rate)
                    if constexpr (k12_ysolo && sizeof(F) == 8) asm volatile("" ::: "memory");
                }
            } else {
                const T* ri_ = reinterpret_cast<const T*>(slot + NRW * GD * 16) + pi;
#pragma unroll
                for (int i = 0; i < NRW; ++i) v[i] = (F)ri_[i * GI * ET];
            }
            F* a = A + role * AF + c;  // even copy at c, odd copy at c - 1
#pragma unroll
            for (int r = 0; r < TY; ++r) {
                F o = v[r + RD] * h[0];
#pragma unroll
                for (int k = R; k >= 1; --k)
                    o = o + (ANTI ? (v[r + RD - k] - v[r + RD + k]) : (v[r + RD - k] + v[r + RD + k])) * h[k];
                a[r * AP] = o;
                // odd copy at c - 1; lane c = 0 writes the pad column AP - 1 of the row before
                // (even copy's last row for r = 0), which no window reads: no exec mask
                if constexpr (ODD) a[TY * AP + r * AP - 1] = o;
            }
        };
        if (role == 0)
            ypass.template operator()<RD, false, true>(hg);
        else if (role == 1)
            ypass.template operator()<RD, true, false>(hd);
        else if (role == 2)
            ypass.template operator()<RS, false, false>(hs);
    };
    // Schedule (one barrier per step; the y passes of step s + 1 run beside the x / z passes
    // of step s, in the other A buffer):
    //   prologue: chunk 0 loaded; chunk 1 issued; y(0)
    //   step s:   [last step of a chunk: vmcnt(0) — retires the next chunk's DMA, issued a
    //             chunk ago] barrier [then: issue the chunk after it into the slots of the
    //             chunk just finished] x / z (s), y (s + 1)
    // ---- z passes of step s (ring slot j = s mod NR): registers only ----
    auto zpass = [&](int s, auto jc) {
        constexpr int j = decltype(jc)::value;
        auto slotz = [](int i, int n) { return ((i % n) + n) % n; };
        if (s >= 2 * RD) {  // plane q = qa + s - 2 RD: dt and dz
            const int q = qa + s - 2 * RD;
            constexpr int cz = j - RD;
            F o1 = r1[slotz(cz, NR)] * hg[0], o4 = r4[slotz(cz, NR)] * hd[0];
#pragma unroll
            for (int k = RD; k >= 1; --k) {
                o1 = o1 + (r1[slotz(cz - k, NR)] + r1[slotz(cz + k, NR)]) * hg[k];
                o4 = o4 + (r4[slotz(cz - k, NR)] - r4[slotz(cz + k, NR)]) * hd[k];
            }
            if (NCH == 3 || st_ok) {  // NCH 3: every lane stores (vmcnt counts), others out of range
                const size_t pq = (size_t)(q - zg0) * plane;
                const unsigned vo = NCH == 3 && !st_ok ? 0x80000000u : vout;
                buf_st<F>(o1, buf_rsrc(G + pq), vo, sout);
                buf_st<F>(o4, buf_rsrc(G + 3 * fs + pq), vo, sout);
            }
        }
        if (s >= RD + RS && s < nout + RD + RS) {  // plane q = qa + s - RD - RS: dy and dx
            const int q = qa + s - RD - RS;
            constexpr int cz = j - RS;
            F o2 = r2[slotz(cz, NRS)] * hs[0], o3 = r3[slotz(cz, NRS)] * hs[0];
#pragma unroll
            for (int k = RS; k >= 1; --k) {
                o2 = o2 + (r2[slotz(cz - k, NRS)] + r2[slotz(cz + k, NRS)]) * hs[k];
                o3 = o3 + (r3[slotz(cz - k, NRS)] + r3[slotz(cz + k, NRS)]) * hs[k];
            }
            if (NCH == 3 || st_ok) {
                const size_t pq = (size_t)(q - zg0) * plane;
                const unsigned vo = NCH == 3 && !st_ok ? 0x80000000u : vout;
                buf_st<F>(o2, buf_rsrc(G + fs + pq), vo, sout);
                buf_st<F>(o3, buf_rsrc(G + 2 * fs + pq), vo, sout);
            }
        }
    };
    // NCH 3 (one-plane chunks): at step s plane s + 1 must have landed.  Issued at step s - 2
    // (right after that step's barrier); behind it this wave issued the stores of steps s - 2 and
    // s - 1 (unconditional: zst of them) and plane s + 2's loads (>= NJMIN): wait until at most
    // that many are left, rounded down to a few immediates (a smaller count only waits longer)
    auto zst = [&](int q) { return (q >= 2 * RD ? 2 : 0) + (q >= RD + RS && q < nout + RD + RS ? 2 : 0); };
    auto wait_plane = [&](int s) {
        const int cnt = zst(s - 2) + zst(s - 1) + (s + 2 < nsteps ? NJMIN : 0);
        if (cnt >= 8 + NJMIN)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + NJMIN) : "memory");
        else if (cnt >= 4 + NJMIN)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 + NJMIN) : "memory");
        else if (cnt >= NJMIN)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NJMIN) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    issue_chunk(0);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int m = 1; m < NCH; ++m) issue_chunk(m);  // (clamped to nsteps)
    ypass_step(0, 0);
    for (int u0 = 0; u0 < nsteps; u0 += NR) {
        bool done = false;
        [&]<int... J>(std::integer_sequence<int, J...>) {
            (
                [&] {
                    if (done) return;
                    constexpr int j = J;
                    const int s = u0 + j;
                    const bool chunk_end = s % K == K - 1;
                    if (chunk_end) {
                        if constexpr (NCH == 3)
                            wait_plane(s);
                        else
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    lds_barrier();
                    if (chunk_end) {
                        const int m2 = s / K + NCH;
                        if (m2 * K < nsteps) issue_chunk(m2);
                    }
                    // k12_defer: the z passes of step s - 1 here, ahead of this step's x-window
                    // reads in program order: register-only work the scheduler can run while those
                    // LDS reads are in flight (their ring slots exclude slot j, written below)
                    if constexpr (k12_defer<F>())
                        if (s >= 1) zpass(s - 1, std::integral_constant<int, (j + NR - 1) % NR>{});
                    // ---- x passes: thread (row `role`, staged column cx) of A tile s & 1 ----
                    // window [cx - R, cx + R] of a field row, as 16-byte pairs from the copy
                    // where it starts aligned
                    const F* arow = At + (j & 1) * AB + role * AP;  // NR even: parity of s
                    auto window = [&]<int R>(int f, F (&x)[2 * R + 2]) {
                        const int st = cx - R;
                        if constexpr (!ODD) {  // single elements, one ds_read_b64 each
                            const F* q = arow + f * AF + st;
#pragma unroll
                            for (int i = 0; i <= 2 * R; ++i) {
                                x[i] = q[i];
                                asm volatile("" ::: "memory");  // no pairing into ds_read2_b64
                            }
                            return;
                        }
                        const F* q = arow + f * AF + ((st & 1) ? TY * AP + st - 1 : st);
                        typedef F F2 __attribute__((ext_vector_type(2)));
                        const F2* q2 = reinterpret_cast<const F2*>(__builtin_assume_aligned(q, 2 * sizeof(F)));
#pragma unroll
                        for (int i = 0; i <= R; ++i) {
                            const F2 v2 = q2[i];
                            x[2 * i] = v2.x;
                            x[2 * i + 1] = v2.y;
                        }
                    };
                    F b1, b2, b3, b4;
                    if constexpr (NWX == 3) {
                        // 12-wave blocks (168 VGPRs): one x window live at a time, each window's
                        // reads pinned behind the previous field's pass (3 waves per SIMD hide
                        // the three LDS round trips)
                        {
                            F x1[2 * RD + 2];
                            window.template operator()<RD>(0, x1);
                            b1 = x1[RD] * hg[0];
#pragma unroll
                            for (int k = RD; k >= 1; --k) b1 = b1 + (x1[RD - k] + x1[RD + k]) * hg[k];
                        }
                        asm volatile("" : "+v"(b1)::"memory");
                        {
                            F x3[2 * RD + 2];
                            window.template operator()<RD>(2, x3);
                            b3 = x3[RD] * hd[0], b4 = x3[RD] * hs[0];
#pragma unroll
                            for (int k = RD; k >= 1; --k) b3 = b3 + (x3[RD - k] - x3[RD + k]) * hd[k];
#pragma unroll
                            for (int k = RS; k >= 1; --k) b4 = b4 + (x3[RD - k] + x3[RD + k]) * hs[k];
                        }
                        asm volatile("" : "+v"(b3), "+v"(b4)::"memory");
                        {
                            F x2[2 * RS + 2];
                            window.template operator()<RS>(1, x2);
                            b2 = x2[RS] * hs[0];
#pragma unroll
                            for (int k = RS; k >= 1; --k) b2 = b2 + (x2[RS - k] + x2[RS + k]) * hs[k];
                        }
                    } else {
                        F x1[2 * RD + 2], x2[2 * RS + 2], x3[2 * RD + 2];
                        window.template operator()<RD>(0, x1);
                        window.template operator()<RS>(1, x2);
                        window.template operator()<RD>(2, x3);
                        b1 = x1[RD] * hg[0], b2 = x2[RS] * hs[0], b3 = x3[RD] * hd[0], b4 = x3[RD] * hs[0];
#pragma unroll
                        for (int k = RD; k >= 1; --k) {
                            b1 = b1 + (x1[RD - k] + x1[RD + k]) * hg[k];
                            b3 = b3 + (x3[RD - k] - x3[RD + k]) * hd[k];
                        }
#pragma unroll
                        for (int k = RS; k >= 1; --k) {
                            b2 = b2 + (x2[RS - k] + x2[RS + k]) * hs[k];
                            b4 = b4 + (x3[RD - k] + x3[RD + k]) * hs[k];
                        }
                    }
                    r1[j % NR] = b1;
                    r4[j % NR] = b4;
                    r2[j % NRS] = b2;
                    r3[j % NRS] = b3;
                    // ---- y passes of the next step (independent work for the scheduler) ----
                    if (s + 1 < nsteps) ypass_step(s + 1, (j + 1) & 1);
                    // ---- z passes (k12_defer: at the next step; the last step's here) ----
                    if (!k12_defer<F>() || s + 1 >= nsteps) zpass(s, std::integral_constant<int, j>{});
                    if (s + 1 >= nsteps) done = true;
                }(),
                ...);
        }(std::make_integer_sequence<int, NR>{});
        if (done) break;
    }
}

// ---------------------------------------------------------------------------
// Solves.  Expression trees copied from calc_flow.py:337-340 (3D) and
// :154-168 (2D); numpy's x**-1 is a correctly rounded reciprocal, x**2 = x*x.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void solve3(double x2, double y2, double z2, double xy, double xz, double yz, double tx,
                                       double ty, double tz, double& vx, double& vy, double& vz) {
    double det = x2 * y2 * z2;
    det = det + 2.0 * xy * xz * yz;
    det = det - y2 * (xz * xz);
    det = det - z2 * (xy * xy);
    det = det - x2 * (yz * yz);
    const double nR = -(1.0 / (det + kEps));
    vx = nR * ((y2 * z2 - yz * yz) * tx + (xz * yz - xy * z2) * ty + (xy * yz - xz * y2) * tz);
    vy = nR * ((yz * xz - xy * z2) * tx + (x2 * z2 - xz * xz) * ty + (xz * xy - x2 * yz) * tz);
    vz = nR * ((xy * yz - y2 * xz) * tx + (xy * xz - x2 * yz) * ty + (x2 * y2 - xy * xy) * tz);
}

// cos((2/3) acos(u)) for u in [0, 1]: a degree-16 polynomial in t = 2u - 1 (Chebyshev fit,
// monomial coefficients in t, |coef| <= 0.77: Horner is stable), max error 1.4e-15 — analytic on
// [0, 1] (the acos branch points at u = +-1 cancel in the even cosine at u = 1; u = -1 is outside).
// Coefficients from tools/eig_poly.py.  Replaces the library acos and a cos series (~110 VALU
// instructions per voxel, a third of K5c's solve tail) by 16 FMAs.
// one Horner step c * t + k with k in an SGPR pair (written out: the compiler's own choice, a
// v_fmac_f64 with k moved into VGPRs first, costs two v_mov per coefficient and voxel)
__device__ __forceinline__ double fma_sk(double c, double t, double k) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(c), "v"(t), "s"(k));
    return d;
}
__device__ __forceinline__ double cos_two_thirds_acos(double u) {
    const double t = 2.0 * u - 1.0;
    double c = fma_sk(-1.627207239089953e-10, t, 5.267127096337474e-10);
    c = fma_sk(c, t, -1.0560891259645176e-09);
    c = fma_sk(c, t, 3.6015719568912613e-09);
    c = fma_sk(c, t, -1.3476196916010413e-08);
    c = fma_sk(c, t, 4.617990510403794e-08);
    c = fma_sk(c, t, -1.594699400417876e-07);
    c = fma_sk(c, t, 5.639770165191962e-07);
    c = fma_sk(c, t, -2.035894233312921e-06);
    c = fma_sk(c, t, 7.541131934033293e-06);
    c = fma_sk(c, t, -2.8919931795498364e-05);
    c = fma_sk(c, t, 0.00011642544430647587);
    c = fma_sk(c, t, -0.0005041246915259092);
    c = fma_sk(c, t, 0.0024663528157121257);
    c = fma_sk(c, t, -0.015509188436476284);
    c = fma_sk(c, t, 0.2474090663228402);
    return fma_sk(c, t, 0.7660444431189779);
}

// Smallest eigenvalue of the symmetric 3x3 [[a d e][d b f][e f c]] in fp64
// (trigonometric closed form).  The reference gets it from LAPACK cgeev in
// complex64 (calc_flow.py:355-357); fp64 here, stored as float32 like the
// reference's output (or kept fp64 with OF3D_REL_F64).
// lambda_min = q + 2p cos(phi + 2pi/3) = q - 2p cos(pi/3 - phi), phi = acos(r)/3 in [0, pi/3];
// pi/3 - acos(r)/3 = (2/3) acos(u) with u = sqrt((1 - r) / 2) (acos(-r) = 2 acos(u)), so
// lambda_min = q - 2p cos((2/3) acos(u)): one polynomial, no acos / cos.  Same conditioning as
// the acos form: near r = 1 (the two SMALLEST eigenvalues nearly equal: flat / isotropic or
// rank-1 regions) r's rounding reaches u through a square root, an error of ~sqrt(eps) p —
// tools/eig_poly.py measures 1.7e-8 lambda_max there.  That is far inside the float32 rel's
// 1e-6 lambda_max, but not the fp64 rel's 1e-10 (OF3D_REL_F64, MATLAB's pageeig,
// M/calc_flow3D.m:235-236), so the fp64-rel instances (REFINE) take eigmin3_deflate below for
// w = (1 - r) / 2 < 1e-6: there lambda_max is simple and far from the pair, so its eigenvector
// is well conditioned, and the pair's smaller eigenvalue comes from the 2x2 block on the plane
// orthogonal to it with the cancellation-free 2x2 formula (max 1e-13 lambda_max over
// tools/eig_poly.py's near-degenerate, isotropic and rank-1 sets; tests/test_eig_formula.py).
// The branch is taken by whole waves only where such tensors occur; float32-rel instances
// never compile it.
// It works on the scaled matrix B = (T - qI) / p (entries O(1), the caller's B11 .. B23), so the
// cross products' squared norms neither underflow nor overflow whatever the tensor's magnitude
// (unscaled, entries below ~1e-77 or above ~1e77 gave NaN); the caller multiplies by p.
__device__ __forceinline__ double eigmin3_deflate(double aq, double bq, double cq, double d, double e, double f,
                                               double w) {
    // B's largest eigenvalue 2 cos(phi) with phi = (2/3) asin(u): cos(phi) = 1 - (2/9) w + O(w^2)
    // (an error in mu only tilts the eigenvector, which moves the 2x2 block's eigenvalues at
    // second order)
    const double mu = 2.0 * (1.0 - (2.0 / 9.0) * w);
    const double m00 = aq - mu, m11 = bq - mu, m22 = cq - mu;
    // the eigenvector of mu: the longest cross product of two rows of E - mu I (rank 2)
    const double c0x = d * f - e * m11, c0y = e * d - m00 * f, c0z = m00 * m11 - d * d;
    const double c1x = d * m22 - e * f, c1y = e * e - m00 * m22, c1z = m00 * f - d * e;
    const double c2x = m11 * m22 - f * f, c2y = f * e - d * m22, c2z = d * f - m11 * e;
    const double n0 = c0x * c0x + c0y * c0y + c0z * c0z, n1 = c1x * c1x + c1y * c1y + c1z * c1z,
                 n2 = c2x * c2x + c2y * c2y + c2z * c2z;
    double vx = c0x, vy = c0y, vz = c0z, nn = n0;
    if (n1 > nn) vx = c1x, vy = c1y, vz = c1z, nn = n1;
    if (n2 > nn) vx = c2x, vy = c2y, vz = c2z, nn = n2;
    const double iv = 1.0 / sqrt(nn);
    vx *= iv, vy *= iv, vz *= iv;
    // an orthonormal basis (u1, u2) of the plane orthogonal to v
    double ux, uy, uz;
    if (fabs(vx) > fabs(vy)) {
        const double s = 1.0 / sqrt(vx * vx + vz * vz);
        ux = -vz * s, uy = 0.0, uz = vx * s;
    } else {
        const double s = 1.0 / sqrt(vy * vy + vz * vz);
        ux = 0.0, uy = vz * s, uz = -vy * s;
    }
    const double wx = vy * uz - vz * uy, wy = vz * ux - vx * uz, wz = vx * uy - vy * ux;
    // the 2x2 block [[al ga][ga be]] of E on that plane
    const double e1x = aq * ux + d * uy + e * uz, e1y = d * ux + bq * uy + f * uz, e1z = e * ux + f * uy + cq * uz;
    const double e2x = aq * wx + d * wy + e * wz, e2y = d * wx + bq * wy + f * wz, e2z = e * wx + f * wy + cq * wz;
    const double al = ux * e1x + uy * e1y + uz * e1z;
    const double be = wx * e2x + wy * e2y + wz * e2z;
    const double ga = ux * e2x + uy * e2y + uz * e2z;
    const double h = (al - be) * 0.5;
    return (al + be) * 0.5 - sqrt(h * h + ga * ga);
}

template <bool REFINE = false>
__device__ __forceinline__ double eigmin3(double a, double b, double c, double d, double e, double f) {
    const double p1 = d * d + e * e + f * f;
    if (p1 == 0.0) return fmin(a, fmin(b, c));
    // constant divisions as multiplications by the rounded reciprocal (not bit-matched
    // anyway; an IEEE division is a ~10-instruction sequence)
    constexpr double third = 1.0 / 3.0, sixth = 1.0 / 6.0;
    const double q = (a + b + c) * third;
    const double aq = a - q, bq = b - q, cq = c - q;
    const double p2 = aq * aq + bq * bq + cq * cq + 2.0 * p1;
    // p = sqrt(x) and 1 / p from one reciprocal square root (v_rsq_f64 + 2 Newton steps: ~1e-16
    // relative; the IEEE sqrt and division sequences cost twice the instructions); tensors
    // too small for the hardware estimate take the IEEE path (p1 > 0, so x > 0)
    const double x = p2 * sixth;
    double p, ip;
    if (x > 1e-290 && x < 1e290) {
        ip = __builtin_amdgcn_rsq(x);
        ip = ip * (1.5 - 0.5 * x * ip * ip);
        ip = ip * (1.5 - 0.5 * x * ip * ip);
        p = x * ip;
    } else {
        p = sqrt(x);
        ip = 1.0 / p;
    }
    const double B11 = aq * ip, B22 = bq * ip, B33 = cq * ip, B12 = d * ip, B13 = e * ip, B23 = f * ip;
    const double detB =
        B11 * (B22 * B33 - B23 * B23) - B12 * (B12 * B33 - B23 * B13) + B13 * (B12 * B23 - B22 * B13);
    double r = 0.5 * detB;
    r = fmin(1.0, fmax(-1.0, r));
    // u = sqrt(w), w in [0, 1], the same way (w floored at 1e-290: u < 1e-145 reads as 0)
    const double w = fmax((1.0 - r) * 0.5, 1e-290);
    if constexpr (REFINE) {
        if (w < 1e-6) return q + p * eigmin3_deflate(B11, B22, B33, B12, B13, B23, w);
    }
    double iu = __builtin_amdgcn_rsq(w);
    iu = iu * (1.5 - 0.5 * w * iu * iu);
    iu = iu * (1.5 - 0.5 * w * iu * iu);
    return q - 2.0 * p * cos_two_thirds_acos(w * iu);
}

// eigmin3 for G tensors at once, straight-line: the per-tensor branches of eigmin3 become
// per-lane selects, and its rare paths (tensors too small / large for the rsq estimate; the
// fp64-rel deflation) wave-uniform branches taken only when some lane of the wave needs them.
// Every tensor goes through exactly eigmin3<REFINE>'s operations (bit-identical), but as G
// independent chains the scheduler can interleave: K5c's epilogue ran one dependent chain per
// voxel (IEEE divisions, rsq Newton steps, the polynomial) with two waves per SIMD to hide it.
template <bool REFINE, int G>
__device__ __forceinline__ void eigmin3_group(const double (&a)[G], const double (&b)[G], const double (&c)[G],
                                              const double (&d)[G], const double (&e)[G], const double (&f)[G],
                                              double (&out)[G]) {
    constexpr double third = 1.0 / 3.0, sixth = 1.0 / 6.0;
    double q[G], aq[G], bq[G], cq[G], x[G], p[G], ip[G];
    bool diag[G], slow[G], any_slow = false;
#pragma unroll
    for (int i = 0; i < G; ++i) {
        const double p1 = d[i] * d[i] + e[i] * e[i] + f[i] * f[i];
        diag[i] = p1 == 0.0;
        q[i] = (a[i] + b[i] + c[i]) * third;
        aq[i] = a[i] - q[i], bq[i] = b[i] - q[i], cq[i] = c[i] - q[i];
        const double p2 = aq[i] * aq[i] + bq[i] * bq[i] + cq[i] * cq[i] + 2.0 * p1;
        x[i] = p2 * sixth;
        double r = __builtin_amdgcn_rsq(x[i]);
        r = r * (1.5 - 0.5 * x[i] * r * r);
        r = r * (1.5 - 0.5 * x[i] * r * r);
        ip[i] = r;
        p[i] = x[i] * r;
        slow[i] = !diag[i] && !(x[i] > 1e-290 && x[i] < 1e290);
        any_slow |= slow[i];
    }
    if (__builtin_expect(__any(any_slow), 0)) {  // IEEE sqrt / division where rsq cannot serve
#pragma unroll
        for (int i = 0; i < G; ++i)
            if (slow[i]) {
                p[i] = sqrt(x[i]);
                ip[i] = 1.0 / p[i];
            }
    }
    double B11[G], B22[G], B33[G], B12[G], B13[G], B23[G], w[G];
    bool defl[G], any_defl = false;
#pragma unroll
    for (int i = 0; i < G; ++i) {
        B11[i] = aq[i] * ip[i], B22[i] = bq[i] * ip[i], B33[i] = cq[i] * ip[i];
        B12[i] = d[i] * ip[i], B13[i] = e[i] * ip[i], B23[i] = f[i] * ip[i];
        const double detB = B11[i] * (B22[i] * B33[i] - B23[i] * B23[i]) - B12[i] * (B12[i] * B33[i] - B23[i] * B13[i]) +
                            B13[i] * (B12[i] * B23[i] - B22[i] * B13[i]);
        double r = 0.5 * detB;
        r = fmin(1.0, fmax(-1.0, r));
        w[i] = fmax((1.0 - r) * 0.5, 1e-290);
        defl[i] = REFINE && !diag[i] && w[i] < 1e-6;
        any_defl |= defl[i];
        double iu = __builtin_amdgcn_rsq(w[i]);
        iu = iu * (1.5 - 0.5 * w[i] * iu * iu);
        iu = iu * (1.5 - 0.5 * w[i] * iu * iu);
        out[i] = q[i] - 2.0 * p[i] * cos_two_thirds_acos(w[i] * iu);
    }
    if constexpr (REFINE) {
        if (__builtin_expect(__any(any_defl), 0)) {
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (defl[i]) out[i] = q[i] + p[i] * eigmin3_deflate(B11[i], B22[i], B33[i], B12[i], B13[i], B23[i], w[i]);
        }
    }
#pragma unroll
    for (int i = 0; i < G; ++i)
        if (diag[i]) out[i] = fmin(a[i], fmin(b[i], c[i]));
}

// K5: W z pass + solve + reliability.  Block = 64 x-columns of one row and
// K5_ZC output planes; per field the (K5_ZC + 2rw)-plane clamped window is
// staged in LDS (double-buffered, next field's loads in flight during this
// field's pass); each thread keeps its K5_R outputs of all 9 fields in
// registers for the pointwise solve.
// Geometry: 64 lanes x G z-groups x R planes per thread (z-block of G*R planes).
// R = 8, G = 8 up to rw 24 (64-plane blocks), else R = 4, G = 8.
struct K5Geom {
    int r, g;
};
constexpr K5Geom k5_geom(int rw) { return {rw <= 24 ? 8 : 4, 8}; }

// Pointwise tail of K5: solve + reliability for the thread's R planes, in
// fp64 whatever the pass type F (fp32 plans solve their float tensor in fp64).
// (K5c: G voxels at a time through solve3 and eigmin3_group — straight-line code, G independent
// chains; the legacy kernels keep G = 1, the same operations per voxel: bit-identical)
template <typename F, typename RelT, int K5_R, int G = 1>
__device__ __forceinline__ void k5_solve_store(const F (&acc)[9][K5_R], int z0l, int nzo, size_t o0, size_t ps,
                                               F* __restrict__ vx, F* __restrict__ vy, F* __restrict__ vz,
                                               RelT* __restrict__ rel) {
    static_assert(K5_R % G == 0, "voxel groups");
    if constexpr (G == 1) {
#pragma unroll
        for (int i = 0; i < K5_R; ++i) {
            if (z0l + i >= nzo) break;
            // field order: tx ty tz xy xz x2 yz y2 z2
            const double tx = acc[0][i], ty = acc[1][i], tz = acc[2][i], xy = acc[3][i], xz = acc[4][i],
                         x2 = acc[5][i], yz = acc[6][i], y2 = acc[7][i], z2 = acc[8][i];
            double ox, oy, oz;
            solve3(x2, y2, z2, xy, xz, yz, tx, ty, tz, ox, oy, oz);
            const size_t o = (size_t)(z0l + i) * ps + o0;
            vx[o] = (F)ox;
            vy[o] = (F)oy;
            vz[o] = (F)oz;
            rel[o] = (RelT)eigmin3<std::is_same_v<RelT, double>>(x2, y2, z2, xy, xz, yz);
        }
    } else {
#pragma unroll
        for (int g0 = 0; g0 < K5_R; g0 += G) {
            if (z0l + g0 >= nzo) break;
            double x2[G], y2[G], z2[G], xy[G], xz[G], yz[G], lam[G];
#pragma unroll
            for (int i = 0; i < G; ++i) {
                const int k = g0 + i;
                const double tx = acc[0][k], ty = acc[1][k], tz = acc[2][k];
                xy[i] = acc[3][k], xz[i] = acc[4][k], x2[i] = acc[5][k], yz[i] = acc[6][k], y2[i] = acc[7][k],
                z2[i] = acc[8][k];
                double ox, oy, oz;
                solve3(x2[i], y2[i], z2[i], xy[i], xz[i], yz[i], tx, ty, tz, ox, oy, oz);
                if (z0l + k < nzo) {
                    const size_t o = (size_t)(z0l + k) * ps + o0;
                    vx[o] = (F)ox;
                    vy[o] = (F)oy;
                    vz[o] = (F)oz;
                }
            }
            eigmin3_group<std::is_same_v<RelT, double>, G>(x2, y2, z2, xy, xz, yz, lam);
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (z0l + g0 + i < nzo) rel[(size_t)(z0l + g0 + i) * ps + o0] = (RelT)lam[i];
        }
    }
}

template <typename F, typename RelT, int NJ, int K5_R, int K5_G>
__global__ __launch_bounds__(64 * K5_G) void k_wz_solve(const F* __restrict__ Q, int zq0, int nz, int ny, int nx,
                                                  size_t fs, const F* __restrict__ hw, const F* __restrict__ hwr,
                                                  int rw, int zo0, int nzo, F* __restrict__ vx, F* __restrict__ vy,
                                                  F* __restrict__ vz, RelT* __restrict__ rel) {
    constexpr int K5_ZC = K5_G * K5_R;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* sm = reinterpret_cast<F*>(smem_raw);
    const int H = K5_ZC + 2 * rw;
    const int lane = threadIdx.x, g = threadIdx.y;
    const int x = blockIdx.x * 64 + lane;
    const int xs = x < nx ? x : nx - 1;
    const int y = blockIdx.y;
    const int zc0 = zo0 + blockIdx.z * K5_ZC;
    const size_t ps = (size_t)ny * nx, col = (size_t)y * nx + xs;
    F rq[NJ];
    auto fetch = [&](int f) {
        const F* q = Q + f * fs + col;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int row = g + K5_G * j;
            if (row < H) rq[j] = q[(size_t)(clampi(zc0 - rw + row, 0, nz - 1) - zq0) * ps];
        }
    };
    F acc[9][K5_R];
    fetch(0);
#pragma unroll
    for (int f = 0; f < 9; ++f) {
        F* buf = sm + (f & 1) * H * 64;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int row = g + K5_G * j;
            if (row < H) buf[row * 64 + lane] = rq[j];
        }
        __syncthreads();
        if (f + 1 < 9) fetch(f + 1);
        lds_pass<K5_R, false, false>(buf + lane, 64, rw + g * K5_R, hw, hwr, rw, acc[f]);
    }
    if (x >= nx) return;
    k5_solve_store<F, RelT, K5_R>(acc, zc0 + g * K5_R - zo0, nzo, (size_t)y * nx + x, ps, vx, vy, vz, rel);
}


// K5 with LDS-DMA staging: the field windows are loaded straight into NB LDS
// buffers, NB - 1 fields ahead of the pass (no staging registers, no VGPR cost
// for the prefetch), so a CU keeps up to (NB - 1) windows of loads in flight
// instead of one field.  One wave-instruction moves 64 lanes x 16 B = RPW rows
// of the 64-column window (RPW = 2 for fp64, 4 for fp32).  Needs nx a
// multiple of 16 B / sizeof(F) (16-byte aligned rows).
// (A persistent form that also prefetches the next tile during the epilogue
// spilled registers and measured slower.)
template <typename F, typename RelT, int NJ2, int K5_R, int K5_G, int NB>
__global__ __launch_bounds__(64 * K5_G) void k_wz_solve_dma(const F* __restrict__ Q, int zq0, int nz, int ny, int nx,
                                                      size_t fs, const F* __restrict__ hw,
                                                      const F* __restrict__ hwr, int rw, int zo0, int nzo,
                                                      F* __restrict__ vx, F* __restrict__ vy, F* __restrict__ vz,
                                                      RelT* __restrict__ rel) {
    constexpr int K5_ZC = K5_G * K5_R;
    constexpr int EPL = 16 / (int)sizeof(F);  // elements per lane per load
    constexpr int RPW = EPL;                  // window rows per wave-instruction
    constexpr int LPR = 64 / RPW;             // lanes per row
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* sm = reinterpret_cast<F*>(smem_raw);
    const int H = K5_ZC + 2 * rw;
    const int HG = (H + RPW - 1) / RPW;  // row groups per window
    const int lane = threadIdx.x, g = threadIdx.y;
    const int x = blockIdx.x * 64 + lane;
    const int y = blockIdx.y;
    const int zc0 = zo0 + blockIdx.z * K5_ZC;
    const size_t ps = (size_t)ny * nx;
    const int xc = min((int)blockIdx.x * 64 + EPL * (lane % LPR), nx - EPL);  // this lane's columns
    const F* qrow = Q + (size_t)y * nx + xc;
    const unsigned lds0 = (unsigned)(uintptr_t)smem_raw;
    auto issue = [&](int f, int b) {
        const F* q = qrow + f * fs;
        const unsigned lb = lds0 + (unsigned)(b * HG * 1024);
#pragma unroll
        for (int j = 0; j < NJ2; ++j) {
            const int p = min(g + K5_G * j, HG - 1);  // surplus slots repeat the last group: equal counts per wave
            const int row = min(RPW * p + lane / LPR, H - 1);
            const F* src = q + (size_t)(clampi(zc0 - rw + row, 0, nz - 1) - zq0) * ps;
            glds16(src, __builtin_amdgcn_readfirstlane(lb + (unsigned)(p * 1024)));
        }
    };
    F acc[9][K5_R];
#pragma unroll
    for (int f = 0; f < NB - 1; ++f) issue(f, f);
#pragma unroll
    for (int f = 0; f < 9; ++f) {
        // field f landed (loads of the fields issued after it may stay in flight: loads
        // retire in issue order), and every wave is done reading the buffer the next
        // issue overwrites
        const int ahead = min(NB - 2, 8 - f);
        if (ahead >= 2)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * NJ2) : "memory");
        else if (ahead == 1)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NJ2) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (f + NB - 1 < 9) issue(f + NB - 1, (f + NB - 1) % NB);
        lds_pass<K5_R, false>(sm + (f % NB) * HG * RPW * 64 + lane, 64, rw + g * K5_R, hw, hwr, rw, acc[f]);
    }
    if (x >= nx) return;
    k5_solve_store<F, RelT, K5_R>(acc, zc0 + g * K5_R - zo0, nzo, (size_t)y * nx + x, ps, vx, vy, vz, rel);
}

// voxels per straight-line group in K5c's epilogue (k5_solve_store): 4 in fp64 (206 VGPRs either
// way, set by the nine fields' accumulators); 1 in fp32, where the four voxels' fp64 epilogue state
// took the kernel from 112 to 158 VGPRs, 4 -> 3 waves per SIMD — the round-4/5 c5 regression (same
// box, round-3 tree vs round-6: K5c 35.1 vs 36.6 ms, profiles/r06/ab_c5_r03/; G 1 vs 4 on one box:
// K5c 35.3 / 35.2 vs 36.6 / 36.7 ms, frame 102.8 / 102.9 vs 104.0 / 104.4, profiles/r06/ab6/c5_*)
template <typename F>
constexpr int K5C_G = sizeof(F) == 8 ? 4 : 1;
// LDS-read distance of K5c's W z passes (lds_pass_c's D: window values read D taps ahead).  fp64:
// 3 (c3 K5c 0.993 / 0.994 -> 0.979 / 0.974 ms over four same-box pairs, c4 6.80 -> 6.75; 4: c3
// 0.98, c4 slower; the VGPR count stays 206, set by the epilogue); fp32 keeps 2 (c5: 36.0 vs
// 36.1 ms).  profiles/r05/ab_k5c_d/
template <typename F>
constexpr int K5C_D = sizeof(F) == 8 ? 3 : 2;

// K5c block coordinates from the launch's (columns, rows, z chunks) grid, XCD-aware: the
// linear workgroup id b runs on XCD b % 8, so the z chunks of one (column block, row) — whose
// windows share 2 rw W-xy planes — get ids 8 apart (same XCD, dispatched back to back) and
// the shared planes come from that XCD's L2 instead of HBM twice.  A bijection on the grid
// (the tail past the last whole group of 8 z-chunk sets keeps the plain order).
struct K5Block {
    int bx, by, bz;
};
__device__ __forceinline__ K5Block k5c_block() {
    if (gridDim.z == 1) return {(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
    const unsigned gx = gridDim.x, gxy = gx * gridDim.y, nz = gridDim.z;
    const unsigned b = blockIdx.x + gx * (blockIdx.y + gridDim.y * blockIdx.z);
    const unsigned full = (gxy * nz) / (8 * nz) * (8 * nz);
    unsigned rest, zc;
    if (b < full) {
        const unsigned j = b >> 3;
        zc = j % nz;
        rest = (j / nz) * 8 + (b & 7);
    } else {
        const unsigned l = b - full;
        zc = l % nz;
        rest = full / nz + l / nz;
    }
    return {(int)(rest % gx), (int)(rest / gx), (int)zc};
}

// K5c: the LDS-DMA W z + solve with a compile-time window radius (taps in SGPRs,
// lds_pass_c: no weight loads or waits inside the passes) and narrow blocks: CB = 32
// columns x 2 z-groups per wave, 4 waves (256 threads), R planes per z-group, so a
// block holds ZC = 8 R output planes of 32 columns and its window of ZC + 2RW planes
// per field takes NB buffers of HG 1-KiB row groups (fp64, RW 15: 24 KiB each).  Two
// blocks fit a CU: one block's prologue / epilogue overlaps another's passes.
// RT0 > 0: after its solve, every block also forms its share of the next frame's dt0 (K0Next,
// input type T0): a contiguous range of voxel groups per block, the K0c arithmetic (k0_group).
template <typename F, typename RelT, int RW, int NB, int R, int NW = 4, int RT0 = 0, typename T0 = uint16_t>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 1 : (R == 8 ? 2 : 3)) void k_wz_solve_c(
    const F* __restrict__ Q, int zq0, int nz, int ny, int nx, size_t fs, const F* __restrict__ hw, int zo0, int nzo,
    F* __restrict__ vx, F* __restrict__ vy, F* __restrict__ vz, RelT* __restrict__ rel, int yo0, K0Next<F> k0, int zt) {
    // NW 8: 128-plane blocks (one per CU), window 1.33x the output planes instead of 1.66x
    constexpr int CB = 32, LPC = 64 / CB;  // columns per block, z-groups per wave
    constexpr int ZC = NW * LPC * R;                // output planes per block (R planes per z-group)
    constexpr int H = ZC + 2 * RW;                  // window rows (planes)
    constexpr int EPL = 16 / (int)sizeof(F);        // elements per lane per DMA
    constexpr int LPR = CB / EPL;                   // lanes per window row
    constexpr int RPWI = 64 / LPR;                  // window rows per wave-instruction (1 KiB)
    constexpr int HG = (H + RPWI - 1) / RPWI;       // row groups per window
    constexpr int NJ2 = (HG + NW - 1) / NW;         // row groups per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    F* sm = reinterpret_cast<F*>(smem_raw);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int col = lane % CB, gz = w * LPC + lane / CB;
    const K5Block kb = k5c_block();
    const int x = kb.bx * CB + col;
    const int y = yo0 + kb.by;  // outputs: rows [yo0, yo0 + gridDim.y) in a compact layout
    const int zc0 = zo0 + kb.bz * ZC;
    const size_t ps = (size_t)ny * nx;
    const int xc = min(kb.bx * CB + EPL * (lane % LPR), nx - EPL);  // this lane's DMA columns
    // the window column of this lane: plane-major rows (zt == 0) or one z-tiled run (zt > 0, nx a
    // multiple of 32: xc & 31 is the lane's column in the tile)
    const F* qrow = zt ? Q + ((size_t)y * (nx >> 5) + (xc >> 5)) * zt * 32 + (xc & 31) : Q + (size_t)y * nx + xc;
    const size_t zs = zt ? 32 : ps;  // element stride of one window plane
    const unsigned lds0 = (unsigned)(uintptr_t)smem_raw;
    F h[RW + 1];
#pragma unroll
    for (int k = 0; k <= RW; ++k) h[k] = hw[k];
    auto issue = [&](int f, int b) {
        const F* q = qrow + f * fs;
        const unsigned lb = lds0 + (unsigned)(b * HG * 1024);
#pragma unroll
        for (int j = 0; j < NJ2; ++j) {
            const int pg = min(w + NW * j, HG - 1);  // surplus slots repeat the last group: equal counts per wave
            const int row = min(RPWI * pg + lane / LPR, H - 1);
            const F* src = q + (size_t)(clampi(zc0 - RW + row, 0, nz - 1) - zq0) * zs;
            glds16(src, __builtin_amdgcn_readfirstlane(lb + (unsigned)(pg * 1024)));
        }
    };
    F acc[9][R];
#pragma unroll
    for (int f = 0; f < NB - 1; ++f) issue(f, f);
    // RT0 > 0: the next frame's dt0 for this block's first groups, loaded right behind the
    // first field's DMA (the two latencies overlap) and held to the end (stores after the solve)
    constexpr int V0 = K0Vec<T0>::V, NG0 = RT0 > 0 ? 2 : 0;
    F dtn[NG0 > 0 ? NG0 : 1][V0];
    size_t k0g0 = 0, k0g1 = 0;
    if constexpr (RT0 > 0) {
        const size_t nblk = (size_t)gridDim.x * gridDim.y * gridDim.z;
        const size_t lin = blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z);
        const size_t per = (k0.ngroups + nblk - 1) / nblk;
        k0g0 = lin * per;
        k0g1 = min(k0g0 + per, k0.ngroups);
        F h0[RT0 + 1];
#pragma unroll
        for (int k = 0; k <= RT0; ++k) h0[k] = k0.ht[k];
#pragma unroll
        for (int j = 0; j < NG0; ++j) {
            const size_t gi = k0g0 + threadIdx.x + (size_t)j * 64 * NW;
            if (gi < k0g1) k0_group_dt<T0, F, RT0>(k0.fr, k0.off0 + gi * V0, h0, dtn[j]);
        }
    }
#pragma unroll
    for (int f = 0; f < 9; ++f) {
        // as k_wz_solve_dma: field f landed, the buffer the next issue overwrites is free
        const int ahead = min(NB - 2, 8 - f);
        if (ahead >= 2)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * NJ2) : "memory");
        else if (ahead == 1)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NJ2) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (f + NB - 1 < 9) issue(f + NB - 1, (f + NB - 1) % NB);
        lds_pass_c<R, RW, K5C_D<F>, false, k5c_solo<F>>(sm + (f % NB) * HG * RPWI * CB + col, CB, RW + gz * R, h,
                                                    acc[f]);
        // pin the pass here: without it the compiler sinks every field's arithmetic below the
        // last barrier and keeps all 9 windows' LDS reads live in registers (spills)
#pragma unroll
        for (int i = 0; i < R; ++i) asm volatile("" : "+v"(acc[f][i]));
    }
    if (x < nx)
        k5_solve_store<F, RelT, R, K5C_G<F>>(acc, zc0 + gz * R - zo0, nzo, (size_t)kb.by * nx + x, (size_t)gridDim.y * nx, vx,
                                   vy, vz, rel);
    if constexpr (RT0 > 0) {  // the next frame's dt0: the held groups, then any rest of [k0g0, k0g1)
#pragma unroll
        for (int j = 0; j < NG0; ++j) {
            const size_t gi = k0g0 + threadIdx.x + (size_t)j * 64 * NW;
            if (gi < k0g1) k0_store<F, V0>(dtn[j], k0.D0 + gi * V0);
        }
        F h0[RT0 + 1];
#pragma unroll
        for (int k = 0; k <= RT0; ++k) h0[k] = k0.ht[k];
        for (size_t gi = k0g0 + threadIdx.x + (size_t)NG0 * 64 * NW; gi < k0g1; gi += 64 * NW)
            k0_group<T0, F, RT0>(k0.fr, k0.off0 + gi * V0, h0, k0.D0 + gi * V0);
    }
}
constexpr int k5c_zc(int r, int nw = 4) { return 2 * nw * r; }  // output planes per K5c block (R per z-group)
template <typename F>
constexpr int k5c_groups(int rw, int r, int nw = 4) {
    constexpr int rpwi = 64 / (32 / (16 / (int)sizeof(F)));
    return (k5c_zc(r, nw) + 2 * rw + rpwi - 1) / rpwi;
}

// ---------------------------------------------------------------------------
// General-radius path (any xyzSig / wSig the reference accepts, calc_flow.py:230-267,
// beyond the tiled kernels' LDS limits): every 1-D pass as its own streaming kernel
// straight from global memory (L2), one output per thread, the same scipy order and
// global-edge clamping; products and solves pointwise.  Not tuned: it exists so that no
// parameter the reference takes is refused.
// ---------------------------------------------------------------------------
template <typename T, typename F>
__global__ __launch_bounds__(256) void k_cast_gen(const T* __restrict__ in, F* __restrict__ out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) out[i] = (F)in[i];
}

// out[q] (planes [q0, q1), origin out_z0) = pass along `axis` (0 x, 1 y, 2 z) of in (origin
// in_z0); z indices clamp to [0, zhi); half taps h[0..r] (h[k] = w[r - k]); anti: lo - hi
template <typename F>
__global__ __launch_bounds__(256) void k_corr_gen(const F* __restrict__ in, int in_z0, F* __restrict__ out, int out_z0,
                                                  int q0, int q1, int ny, int nx, int axis, const F* __restrict__ h,
                                                  int r, int anti, int zhi) {
    const size_t plane = (size_t)ny * nx, n = (size_t)(q1 - q0) * plane;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const int q = q0 + (int)(i / plane);
        const size_t rem = i % plane;
        const int y = (int)(rem / nx), x = (int)(rem % nx);
        auto at = [&](int d) -> F {
            int zz = q, yy = y, xx = x;
            if (axis == 0)
                xx = clampi(x + d, 0, nx - 1);
            else if (axis == 1)
                yy = clampi(y + d, 0, ny - 1);
            else
                zz = clampi(q + d, 0, zhi - 1);
            return in[(size_t)(zz - in_z0) * plane + (size_t)yy * nx + xx];
        };
        F o = at(0) * h[0];
        for (int k = r; k >= 1; --k) o = o + (anti ? (at(-k) - at(k)) : (at(-k) + at(k))) * h[k];
        out[(size_t)(q - out_z0) * plane + rem] = o;
    }
}

// the structure-tensor products (tables as k_prod_wyx): P[p] = G[a(p)] * G[b(p)], n points
template <typename F>
__global__ __launch_bounds__(256) void k_prod_gen(const F* __restrict__ G, F* __restrict__ P, size_t fs, size_t n,
                                                  int np) {
    const unsigned long long pa = np == 9 ? 0x311222312ull : 0x12212ull, pb = np == 9 ? 0x313231000ull : 0x12100ull;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        for (int p = 0; p < np; ++p)
            P[p * fs + i] = G[((pa >> (4 * p)) & 15u) * fs + i] * G[((pb >> (4 * p)) & 15u) * fs + i];
}

// Reliability of given structure tensors (of3d_rel3d): field-major [6][n] in the order
// x2 y2 z2 xy xz yz, the same eigmin3 instance the solve kernels use for RelT
template <typename RelT>
__global__ __launch_bounds__(256) void k_rel3d(const double* __restrict__ T, size_t n, RelT* __restrict__ rel) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        rel[i] = (RelT)eigmin3<std::is_same_v<RelT, double>>(T[i], T[n + i], T[2 * n + i], T[3 * n + i],
                                                             T[4 * n + i], T[5 * n + i]);
}

// 3D solve + reliability from the nine windowed fields (order tx ty tz xy xz x2 yz y2 z2)
template <typename F, typename RelT>
__global__ __launch_bounds__(256) void k_solve3_gen(const F* __restrict__ W, size_t fs, size_t n, F* __restrict__ vx,
                                                    F* __restrict__ vy, F* __restrict__ vz, RelT* __restrict__ rel) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const double tx = W[i], ty = W[fs + i], tz = W[2 * fs + i], xy = W[3 * fs + i], xz = W[4 * fs + i],
                     x2 = W[5 * fs + i], yz = W[6 * fs + i], y2 = W[7 * fs + i], z2 = W[8 * fs + i];
        double ox, oy, oz;
        solve3(x2, y2, z2, xy, xz, yz, tx, ty, tz, ox, oy, oz);
        vx[i] = (F)ox;
        vy[i] = (F)oy;
        vz[i] = (F)oz;
        rel[i] = (RelT)eigmin3<std::is_same_v<RelT, double>>(x2, y2, z2, xy, xz, yz);
    }
}

// 2D (calc_flow.py:154-168). field order: tx ty xy x2 y2
// (grid-stride over a 64-bit count: a 2D batch plan may hold more than 2^31 pixels)
template <typename F>
__global__ __launch_bounds__(256) void k_solve2d(const F* __restrict__ Q, size_t fs, size_t n, F* __restrict__ vx,
                                                 F* __restrict__ vy, F* __restrict__ rel) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const double tx = Q[i], ty = Q[fs + i], xy = Q[2 * fs + i], x2 = Q[3 * fs + i], y2 = Q[4 * fs + i];
    const double det = (x2 * y2) - (xy * xy);
    const double R = 1.0 / (det + kEps);
    vx[i] = (F)(R * ((y2 * -tx) + (-xy * -ty)));
    vy[i] = (F)(R * ((-xy * -tx) + (x2 * -ty)));
    const double tr = x2 + y2;
    const double disc = tr * tr - 4.0 * det;
    const double L1 = (tr + sqrt(disc)) / 2.0;
    const double L2 = (tr - sqrt(disc)) / 2.0;
    // np.minimum propagates NaN
    rel[i] = (F)((L1 != L1) ? L1 : ((L2 != L2) ? L2 : (L1 < L2 ? L1 : L2)));
    }
}

// ---------------------------------------------------------------------------
// Downstream statistics (the reference's
// example_analysis_script.ipynb cells 4-6) in one pass over resident outputs:
//   mask = rel > thresh; v = v*mask, v == 0 -> NaN; vx, vy *= xyscale/tscale
//   (as (v*xyscale)/tscale), vz likewise with zscale;
//   magnitude = sqrt((vx*vx + vy*vy) + vz*vz); theta = atan2(vy, vx);
//   phi = atan(vz / sqrt(vx*vx + vy*vy)).  2D: vz == nullptr, no phi.
// ---------------------------------------------------------------------------
template <typename VT, typename RelT>
__global__ __launch_bounds__(256) void k_flow_stats(const VT* __restrict__ vx, const VT* __restrict__ vy,
                                                    const VT* __restrict__ vz, const RelT* __restrict__ rel, size_t n,
                                                    double thresh, double sxy, double sz, double st,
                                                    double* __restrict__ ox, double* __restrict__ oy,
                                                    double* __restrict__ oz, double* __restrict__ mag,
                                                    double* __restrict__ theta, double* __restrict__ phi) {
    const size_t stride = (size_t)gridDim.x * 256;
    const double qnan = __builtin_nan("");
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const double m = ((double)rel[i] > thresh) ? 1.0 : 0.0;  // numpy: v * bool mask
        auto fix = [&](double v, double scale) {
            v = v * m;
            if (v == 0.0) v = qnan;
            return (v * scale) / st;
        };
        const double x = fix((double)vx[i], sxy), y = fix((double)vy[i], sxy);
        const double xy2 = x * x + y * y;
        ox[i] = x;
        oy[i] = y;
        theta[i] = atan2(y, x);
        if (vz) {
            const double z = fix((double)vz[i], sz);
            oz[i] = z;
            mag[i] = sqrt(xy2 + z * z);
            phi[i] = atan(z / sqrt(xy2));
        } else {
            mag[i] = sqrt(xy2);
        }
    }
}

constexpr int K1C_S = 4;

// LDS-DMA K5: NB window buffers of ceil(H / RPW) 1-KB row groups (RPW = 16 B /
// sizeof(F) rows); NJ2 = groups per wave.
template <typename F>
constexpr int k5_groups(int rw) {
    constexpr int rpw = 16 / (int)sizeof(F);
    return (k5_geom(rw).g * k5_geom(rw).r + 2 * rw + rpw - 1) / rpw;
}
template <typename F>
int k5_dma_nb(int rw) {
    const size_t buf = (size_t)k5_groups<F>(rw) * 1024, lim = 160 * 1024;
    return 3 * buf <= lim ? 3 : (2 * buf <= lim ? 2 : 0);
}

}  // namespace
