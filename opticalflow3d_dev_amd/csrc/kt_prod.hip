// kt_prod.hip — kernel instances and their getters (see kernels.hpp).
#include "of3d_dev.hpp"
#include "kernels.hpp"

namespace of3dk {

// K34 instances: W radii with a compiled register ring, wSig 3..7 (others use K3 + K4)
template <typename F, int NP>
const void* k34_fn(int rw, int s, int rb) {
#define OF3D_K34(RW, SA, SB)                                    \
    case RW:                                                    \
        if (s == SA) return rb == 2 ? nullptr : (const void*)k_prod_wyx<F, NP, RW, SA>;                                     \
        if (s == SB) return rb == 2 ? nullptr : (const void*)k_prod_wyx<F, NP, RW, SB>;                                     \
        return nullptr;
    switch (rw) {
        OF3D_K34(9, 16, 8)
        OF3D_K34(12, 16, 8)
        OF3D_K34(15, 16, 8)
        OF3D_K34(18, 8, 4)  // register ring of 38-48 rows: shorter tiles
        OF3D_K34(21, 8, 4)
        default: return nullptr;
    }
#undef OF3D_K34
}

// Unique-staging instances (k_prod_wyx UQ: no duplicated halo columns, edge replicas copied)
// for 8-wave blocks, cut for 2 waves per SIMD (256 VGPRs: an 8-wave block runs one per CU
// anyway): gradient prefetch 4 rows, phase-B LDS distance 2.  c3 (rw 21): 8-row tiles
// 1.85 ms vs 1.92 (4-row) and 2.02 (duplicate staging, 4-wave blocks); 16-row tiles and
// deeper prefetch (8, 11 rows) or LDS distance 4 within noise.
template <typename F, int NP>
const void* k34_fn_uq(int rw, int s) {
#define OF3D_K34U(RW)                                                                      \
    if (rw == RW) {                                                                        \
        if (s == 8) return (const void*)k_prod_wyx<F, NP, RW, 8, 4, 2, 4, 2, true>;        \
        if (s == 4) return (const void*)k_prod_wyx<F, NP, RW, 4, 4, 2, 4, 2, true>;        \
    }
    OF3D_K34U(21)
    OF3D_K34U(18)
    OF3D_K34U(15)
    OF3D_K34U(12)
    OF3D_K34U(9)
#undef OF3D_K34U
    return nullptr;
}

// Wave-specialised instances (k_prod_wyx_ws: npw producer + 16 - npw consumer waves, 64 npw
// staged columns, 128 VGPRs): npw 8 (512 staged columns), and in fp64 npw 9 (576: two blocks
// per 1024-wide row)
// pd: gradient prefetch rows of the producers (2; 4 for fp64 radii up to 15 at 4-row tiles,
// where the 2 rw + 2 row register ring leaves the room)
template <typename F, int NP>
const void* k34_fn_ws(int rw, int s, int npw, int pd) {
    if (npw != 8 && (npw != 9 || sizeof(F) != 8)) return nullptr;
    if (pd == 4) {
        if (sizeof(F) != 8 || s != 4) return nullptr;
#define OF3D_K34W4(RW) \
        if (rw == RW) return npw == 8 ? (const void*)k_prod_wyx_ws<F, NP, RW, 4, 4, 2, 8> : (const void*)k_prod_wyx_ws<F, NP, RW, 4, 4, 2, 9>;
        OF3D_K34W4(15)
        OF3D_K34W4(12)
        OF3D_K34W4(9)
#undef OF3D_K34W4
        return nullptr;
    }
    if (pd != 2) return nullptr;
#define OF3D_K34W(RW)                                                                                              \
    if (rw == RW) {                                                                                                \
        if (s == 8) return npw == 8 ? (const void*)k_prod_wyx_ws<F, NP, RW, 8> : (const void*)k_prod_wyx_ws<F, NP, RW, 8, 2, 2, 9>; \
        if (s == 4) return npw == 8 ? (const void*)k_prod_wyx_ws<F, NP, RW, 4> : (const void*)k_prod_wyx_ws<F, NP, RW, 4, 2, 2, 9>; \
    }
    OF3D_K34W(21)
    OF3D_K34W(18)
    OF3D_K34W(15)
    OF3D_K34W(12)
    OF3D_K34W(9)
#undef OF3D_K34W
    return nullptr;
}

// Packed-fp32 instances (k_prod_wyx_pk: 4 producer + 4 consumer waves on float2 lanes)
template <int NP>
const void* k34_fn_pk(int rw, int s) {
#define OF3D_K34P(RW)                                                      \
    if (rw == RW) {                                                        \
        if (s == 8) return (const void*)k_prod_wyx_pk<NP, RW, 8>;          \
        if (s == 4) return (const void*)k_prod_wyx_pk<NP, RW, 4>;          \
    }
    OF3D_K34P(21)
    OF3D_K34P(18)
    OF3D_K34P(15)
    OF3D_K34P(12)
    OF3D_K34P(9)
#undef OF3D_K34P
    return nullptr;
}
template const void* k34_fn_pk<9>(int, int);
template const void* k34_fn_pk<5>(int, int);

template const void* k34_fn_ws<double, 9>(int, int, int, int);
template const void* k34_fn_ws<double, 5>(int, int, int, int);
template const void* k34_fn_ws<float, 9>(int, int, int, int);
template const void* k34_fn_ws<float, 5>(int, int, int, int);
template const void* k34_fn_uq<double, 9>(int, int);
template const void* k34_fn_uq<double, 5>(int, int);
template const void* k34_fn_uq<float, 9>(int, int);
template const void* k34_fn_uq<float, 5>(int, int);

template const void* k34_fn<double, 9>(int, int, int);
template const void* k34_fn<double, 5>(int, int, int);
template const void* k34_fn<float, 9>(int, int, int);
template const void* k34_fn<float, 5>(int, int, int);

}  // namespace of3dk
