// kt_grad_legacy.hip — kernel instances and their getters (see kernels.hpp).
#include "of3d_dev.hpp"
#include "kernels.hpp"

namespace of3dk {

template <typename T, typename F>
const void* k1_kernel(int rd) {
    const int nj = (K1_TY + 2 * rd + 3) / 4;
    if (nj <= 8) return (const void*)k_grad_xy<T, F, 8>;
    if (nj <= 12) return (const void*)k_grad_xy<T, F, 12>;
    return (const void*)k_grad_xy<T, F, 16>;
}

template <typename F>
const void* k1_kernel_dt(int dtype, int rd) {
    switch (dtype) {
        case OF3D_U8: return k1_kernel<uint8_t, F>(rd);
        case OF3D_U16: return k1_kernel<uint16_t, F>(rd);
        case OF3D_I16: return k1_kernel<int16_t, F>(rd);
        case OF3D_U32: return k1_kernel<uint32_t, F>(rd);
        case OF3D_I32: return k1_kernel<int32_t, F>(rd);
        case OF3D_F32: return k1_kernel<float, F>(rd);
        default: return k1_kernel<double, F>(rd);
    }
}

template <typename F>
const void* k0v_kernel_dt(int dtype) {
    switch (dtype) {
        case OF3D_U8: return (const void*)k_tderiv_vec<uint8_t, F>;
        case OF3D_U16: return (const void*)k_tderiv_vec<uint16_t, F>;
        case OF3D_I16: return (const void*)k_tderiv_vec<int16_t, F>;
        case OF3D_U32: return (const void*)k_tderiv_vec<uint32_t, F>;
        case OF3D_I32: return (const void*)k_tderiv_vec<int32_t, F>;
        case OF3D_F32: return (const void*)k_tderiv_vec<float, F>;
        default: return (const void*)k_tderiv_vec<double, F>;
    }
}

template <typename F>
const void* k0_kernel_dt(int dtype) {
    switch (dtype) {
        case OF3D_U8: return (const void*)k_tderiv<uint8_t, F>;
        case OF3D_U16: return (const void*)k_tderiv<uint16_t, F>;
        case OF3D_I16: return (const void*)k_tderiv<int16_t, F>;
        case OF3D_U32: return (const void*)k_tderiv<uint32_t, F>;
        case OF3D_I32: return (const void*)k_tderiv<int32_t, F>;
        case OF3D_F32: return (const void*)k_tderiv<float, F>;
        default: return (const void*)k_tderiv<double, F>;
    }
}

template const void* k1_kernel_dt<double>(int, int);
template const void* k0v_kernel_dt<double>(int);
template const void* k0_kernel_dt<double>(int);
template const void* k1_kernel_dt<float>(int, int);
template const void* k0v_kernel_dt<float>(int);
template const void* k0_kernel_dt<float>(int);

}  // namespace of3dk
