// kt_grad3.hip — K12 (fused gradient y/x/z passes) instances and their getter (kernels.hpp).
#include "of3d_dev.hpp"
#include "kernels.hpp"

namespace of3dk {

// K12 instances: input dtypes u8 / u16 / f32, (rd, rs) = (3, 1), (6, 2), (9, 3) (xyzSig 1, 2, 3);
// fp32 only at rd 9; other radii / dtypes run K1c + K2c (or the older kernels).
// deep: the three-DMA-slot instance (fp64 rd 6; for marches of >= 128 planes), where one exists
template <typename F>
const void* k12_fn(int dtype, int rd, int rs, bool deep) {
#define OF3D_K12(T)                                                                \
    if (rd == 3 && rs == 1) return (const void*)k_grad_xyz_c<T, F, 3, 1>;          \
    if constexpr (sizeof(F) == 8)                                                  \
        if (deep && rd == 6 && rs == 2) return (const void*)k_grad_xyz_c<T, F, 6, 2, true>; \
    if (rd == 6 && rs == 2) return (const void*)k_grad_xyz_c<T, F, 6, 2>;          \
    if constexpr (sizeof(F) == 4) /* fp64 at rd 9 spills registers */              \
        if (rd == 9 && rs == 3) return (const void*)k_grad_xyz_c<T, F, 9, 3>;      \
    return nullptr;
    switch (dtype) {
        case OF3D_U8: { OF3D_K12(uint8_t) }
        case OF3D_U16: { OF3D_K12(uint16_t) }
        case OF3D_F32: { OF3D_K12(float) }
        default: return nullptr;
    }
#undef OF3D_K12
}

// dynamic LDS bytes of the K12 instance for (dtype, rd) (0: none)
template <typename F>
size_t k12_lds(int dtype, int rd, bool deep) {
#define OF3D_K12L(T)                                                  \
    if (rd == 3) return (size_t)k12_lds_bytes<T, F, 3>();             \
    if (rd == 6 && deep) return (size_t)k12_lds_bytes<T, F, 6, true>(); \
    if (rd == 6) return (size_t)k12_lds_bytes<T, F, 6>();             \
    if (rd == 9) return (size_t)k12_lds_bytes<T, F, 9>();             \
    return 0;
    switch (dtype) {
        case OF3D_U8: { OF3D_K12L(uint8_t) }
        case OF3D_U16: { OF3D_K12L(uint16_t) }
        case OF3D_F32: { OF3D_K12L(float) }
        default: return 0;
    }
#undef OF3D_K12L
}

template const void* k12_fn<double>(int, int, int, bool);
template const void* k12_fn<float>(int, int, int, bool);
template size_t k12_lds<double>(int, int, bool);
template size_t k12_lds<float>(int, int, bool);

}  // namespace of3dk
