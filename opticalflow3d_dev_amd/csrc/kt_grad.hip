// kt_grad.hip — kernel instances and their getters (see kernels.hpp).
#include "of3d_dev.hpp"
#include "kernels.hpp"

namespace of3dk {

// compile-time-rt K0 instances: u8 / u16 / f32 input, rt 3, 6, 9 (tSig 1, 2, 3)
template <typename F>
const void* k0c_fn(int dtype, int rt) {
#define OF3D_K0C(T)                                                   \
    if (rt == 3) return (const void*)k_tderiv_vec_c<T, F, 3>;        \
    if (rt == 6) return (const void*)k_tderiv_vec_c<T, F, 6>;        \
    if (rt == 9) return (const void*)k_tderiv_vec_c<T, F, 9>;        \
    return nullptr;
    switch (dtype) {
        case OF3D_U8: { OF3D_K0C(uint8_t) }
        case OF3D_U16: { OF3D_K0C(uint16_t) }
        case OF3D_F32: { OF3D_K0C(float) }
        default: return nullptr;
    }
#undef OF3D_K0C
}

// K0 batching instances (k_tderiv_multi): M = 2..5 consecutive outputs, the K0c dtypes and radii
template <typename F>
const void* k0m_fn(int dtype, int rt, int m) {
#define OF3D_K0M_M(T, RT)                                                    \
    if (m == 2) return (const void*)k_tderiv_multi<T, F, RT, 2>;            \
    if (m == 3) return (const void*)k_tderiv_multi<T, F, RT, 3>;            \
    if (m == 4) return (const void*)k_tderiv_multi<T, F, RT, 4>;            \
    if (m == 5) return (const void*)k_tderiv_multi<T, F, RT, 5>;            \
    return nullptr;
#define OF3D_K0M(T)                         \
    if (rt == 3) { OF3D_K0M_M(T, 3) }       \
    if (rt == 6) { OF3D_K0M_M(T, 6) }       \
    if (rt == 9) { OF3D_K0M_M(T, 9) }       \
    return nullptr;
    switch (dtype) {
        case OF3D_U8: { OF3D_K0M(uint8_t) }
        case OF3D_U16: { OF3D_K0M(uint16_t) }
        case OF3D_F32: { OF3D_K0M(float) }
        default: return nullptr;
    }
#undef OF3D_K0M
#undef OF3D_K0M_M
}

// K1c instances: input dtypes u8 / u16 / f32, (rd, rs) = (3, 1), (6, 2), (9, 3) (xyzSig 1, 2, 3);
// others use k_grad_xy.

template <typename F>
const void* k1c_fn(int dtype, int rd, int rs) {
#define OF3D_K1C(T)                                                                           \
    if (rd == 3 && rs == 1) return (const void*)k_grad_xy_c<T, F, 3, 1, K1C_S>;               \
    if (rd == 6 && rs == 2) return (const void*)k_grad_xy_c<T, F, 6, 2, K1C_S>;               \
    if (rd == 9 && rs == 3) return (const void*)k_grad_xy_c<T, F, 9, 3, K1C_S>;               \
    return nullptr;
    switch (dtype) {
        case OF3D_U8: { OF3D_K1C(uint8_t) }
        case OF3D_U16: { OF3D_K1C(uint16_t) }
        case OF3D_F32: { OF3D_K1C(float) }
        default: return nullptr;
    }
#undef OF3D_K1C
}

template const void* k0c_fn<double>(int, int);
template const void* k0m_fn<double>(int, int, int);
template const void* k0m_fn<float>(int, int, int);
template const void* k1c_fn<double>(int, int, int);
template const void* k0c_fn<float>(int, int);
template const void* k1c_fn<float>(int, int, int);

}  // namespace of3dk
