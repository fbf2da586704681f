// kt_solve.hip — kernel instances and their getters (see kernels.hpp).
#include "of3d_dev.hpp"
#include "kernels.hpp"

namespace of3dk {

// K5c instances (window radii with a compiled pass; others use k_wz_solve_dma)
template <typename F, typename RelT>
const void* k5c_fn(int rw, int nb, int r) {
#define OF3D_K5C(RW) \
    case RW:                                                                                            \
        if (r == 4) return nb == 3 ? (const void*)k_wz_solve_c<F, RelT, RW, 3, 4> : nullptr;            \
        return nb == 3 ? (const void*)k_wz_solve_c<F, RelT, RW, 3, 8> : (const void*)k_wz_solve_c<F, RelT, RW, 2, 8>;
    switch (rw) {
        OF3D_K5C(12)
        OF3D_K5C(15)
        OF3D_K5C(21)
        default: return nullptr;
    }
#undef OF3D_K5C
}

template const void* k5c_fn<double, float>(int, int, int);
template const void* k5c_fn<double, double>(int, int, int);
template const void* k5c_fn<float, float>(int, int, int);
template const void* k5c_fn<float, double>(int, int, int);

}  // namespace of3dk
