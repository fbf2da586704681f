// kt_solve.hip — kernel instances and their getters (see kernels.hpp).
#include "of3d_dev.hpp"
#include "kernels.hpp"

namespace of3dk {

// K5c instances (window radii with a compiled pass, wSig 3..7; others use k_wz_solve_dma)
// rt0 > 0: the instance that also forms the next frame's dt0 (uint16 frames; (rw, rt) of
// configs[1..4]: (15, 6) and (21, 9))
template <typename F, typename RelT>
const void* k5c_fn(int rw, int nb, int r, int nw, int rt0) {
    if (rt0 > 0) {
        if (nw != 4 || (r != 8 && r != 4)) return nullptr;
        if (r == 4) {  // 32-plane blocks (three per CU, three window buffers): cache-resident workspaces
            if (nb != 3) return nullptr;
            if (rw == 21 && rt0 == 9) return (const void*)k_wz_solve_c<F, RelT, 21, 3, 4, 4, 9>;
            if (rw == 15 && rt0 == 6) return (const void*)k_wz_solve_c<F, RelT, 15, 3, 4, 4, 6>;
            return nullptr;
        }
        if (rw == 21 && rt0 == 9)
            return nb == 3 ? (const void*)k_wz_solve_c<F, RelT, 21, 3, 8, 4, 9> : (const void*)k_wz_solve_c<F, RelT, 21, 2, 8, 4, 9>;
        if (rw == 15 && rt0 == 6)
            return nb == 3 ? (const void*)k_wz_solve_c<F, RelT, 15, 3, 8, 4, 6> : (const void*)k_wz_solve_c<F, RelT, 15, 2, 8, 4, 6>;
        return nullptr;
    }
#define OF3D_K5C(RW) \
    case RW:                                                                                            \
        if (nw == 8) return nb == 3 ? (const void*)k_wz_solve_c<F, RelT, RW, 3, 8, 8> : nullptr;        \
        if (r == 4) return nb == 3 ? (const void*)k_wz_solve_c<F, RelT, RW, 3, 4> : nullptr;            \
        return nb == 3 ? (const void*)k_wz_solve_c<F, RelT, RW, 3, 8> : (const void*)k_wz_solve_c<F, RelT, RW, 2, 8>;
    switch (rw) {
        OF3D_K5C(9)
        OF3D_K5C(12)
        OF3D_K5C(15)
        OF3D_K5C(18)
        OF3D_K5C(21)
        default: return nullptr;
    }
#undef OF3D_K5C
}

template const void* k5c_fn<double, float>(int, int, int, int, int);
template const void* k5c_fn<double, double>(int, int, int, int, int);
template const void* k5c_fn<float, float>(int, int, int, int, int);
template const void* k5c_fn<float, double>(int, int, int, int, int);

}  // namespace of3dk
