// kt_prod.hip — kernel instances and their getters (see kernels.hpp).
#include "of3d_dev.hpp"
#include "kernels.hpp"

namespace of3dk {

// K34 instances: W radii with a compiled register ring (others use K3 + K4)
template <typename F, int NP>
const void* k34_fn(int rw, int s, int rb) {
#define OF3D_K34(RW, SA, SB)                                    \
    case RW:                                                    \
        if (s == SA) return rb == 2 ? nullptr : (const void*)k_prod_wyx<F, NP, RW, SA>;                                     \
        if (s == SB) return rb == 2 ? nullptr : (const void*)k_prod_wyx<F, NP, RW, SB>;                                     \
        return nullptr;
    switch (rw) {
        OF3D_K34(12, 16, 8)
        OF3D_K34(15, 16, 8)
        OF3D_K34(21, 8, 4)  // register ring of 44-48 rows: shorter tiles
        default: return nullptr;
    }
#undef OF3D_K34
}

template const void* k34_fn<double, 9>(int, int, int);
template const void* k34_fn<double, 5>(int, int, int);
template const void* k34_fn<float, 9>(int, int, int);
template const void* k34_fn<float, 5>(int, int, int);

}  // namespace of3dk
