// kt_prod_legacy.hip — kernel instances and their getters (see kernels.hpp).
#include "of3d_dev.hpp"
#include "kernels.hpp"

namespace of3dk {

template <typename F>
const void* k3_kernel(int np, int rw) {
    const int tj = (2 * rw + 3) / 4;  // <= 24 for rw <= 48
    if (np == 9) {
        if (tj <= 8) return (const void*)k_prod_wy<F, 9, 8>;
        if (tj <= 12) return (const void*)k_prod_wy<F, 9, 12>;
        return (const void*)k_prod_wy<F, 9, 24>;
    }
    if (tj <= 8) return (const void*)k_prod_wy<F, 5, 8>;
    if (tj <= 12) return (const void*)k_prod_wy<F, 5, 12>;
    return (const void*)k_prod_wy<F, 5, 24>;
}

template <typename F>
const void* k4_kernel(int nf, int rw) {
    const int tj = (2 * k4_halo(rw) + 31) / 32;  // <= 3 for rw <= 48
    if (nf == 9)
        return tj <= 1 ? (const void*)k_wx<F, 9, 1>
                       : (tj == 2 ? (const void*)k_wx<F, 9, 2> : (const void*)k_wx<F, 9, 3>);
    return tj <= 1 ? (const void*)k_wx<F, 5, 1> : (tj == 2 ? (const void*)k_wx<F, 5, 2> : (const void*)k_wx<F, 5, 3>);
}

template const void* k3_kernel<double>(int, int);
template const void* k4_kernel<double>(int, int);
template const void* k3_kernel<float>(int, int);
template const void* k4_kernel<float>(int, int);

}  // namespace of3dk
