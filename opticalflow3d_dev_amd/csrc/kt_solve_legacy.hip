// kt_solve_legacy.hip — kernel instances and their getters (see kernels.hpp).
#include "of3d_dev.hpp"
#include "kernels.hpp"

namespace of3dk {

template <typename F, typename RelT>
const void* k5_kernel(int rw) {
    // NJ = rows per thread of the staged window: ceil((G * R + 2rw) / G)
    const K5Geom k = k5_geom(rw);
    if (k.r == 8)
        return rw <= 16 ? (const void*)k_wz_solve<F, RelT, 12, 8, 8> : (const void*)k_wz_solve<F, RelT, 14, 8, 8>;
    const int nj = (8 * 4 + 2 * rw + 7) / 8;
    switch (nj <= 10 ? 10 : (nj <= 12 ? 12 : 16)) {
        case 10: return (const void*)k_wz_solve<F, RelT, 10, 4, 8>;
        case 12: return (const void*)k_wz_solve<F, RelT, 12, 4, 8>;
        default: return (const void*)k_wz_solve<F, RelT, 16, 4, 8>;
    }
}

template <typename F, typename RelT>
const void* k5_dma_kernel(int rw, int nb) {
    const K5Geom k = k5_geom(rw);
    const int nj2 = (k5_groups<F>(rw) + k.g - 1) / k.g;
#define OF3D_K5D(NJ2, R)                                                     \
    (nb == 3 ? (const void*)k_wz_solve_dma<F, RelT, NJ2, R, 8, 3>            \
             : (const void*)k_wz_solve_dma<F, RelT, NJ2, R, 8, 2>)
    if constexpr (sizeof(F) == 8) {
        if (k.r == 8) return nj2 <= 6 ? OF3D_K5D(6, 8) : OF3D_K5D(7, 8);  // rw <= 24: nj2 <= 7
        return nj2 <= 6 ? OF3D_K5D(6, 4) : (nj2 <= 7 ? OF3D_K5D(7, 4) : OF3D_K5D(8, 4));  // rw <= 48: nj2 <= 8
    } else {
        if (k.r == 8) return nj2 <= 3 ? OF3D_K5D(3, 8) : OF3D_K5D(4, 8);  // rw <= 24: nj2 <= 4
        return nj2 <= 3 ? OF3D_K5D(3, 4) : OF3D_K5D(4, 4);                // rw <= 48: nj2 <= 4
    }
#undef OF3D_K5D
}

template const void* k5_kernel<double, float>(int);
template const void* k5_kernel<double, double>(int);
template const void* k5_dma_kernel<double, float>(int, int);
template const void* k5_dma_kernel<double, double>(int, int);
template const void* k5_kernel<float, float>(int);
template const void* k5_kernel<float, double>(int);
template const void* k5_dma_kernel<float, float>(int, int);
template const void* k5_dma_kernel<float, double>(int, int);

}  // namespace of3dk
