#pragma once
// kernels.hpp — getters of the kernel instances (host stub addresses for hipLaunchKernel /
// hipFuncSetAttribute).  Each family lives in its own translation unit (kt_*.hip) so the
// library builds in parallel; the templates below are explicitly instantiated there for
// F = double (exact mode) and float (OF3D_FP32).
namespace of3dk {
template <typename F> const void* k1_kernel_dt(int dtype, int rd);          // kt_grad_legacy.hip
template <typename F> const void* k0v_kernel_dt(int dtype);                  // kt_grad_legacy.hip
template <typename F> const void* k0_kernel_dt(int dtype);                   // kt_grad_legacy.hip
template <typename F> const void* k0c_fn(int dtype, int rt);                 // kt_grad.hip
template <typename F> const void* k0m_fn(int dtype, int rt, int m);          // kt_grad.hip (K0 batching)
template <typename F> const void* k1c_fn(int dtype, int rd, int rs);         // kt_grad.hip
template <typename F> const void* k12_fn(int dtype, int rd, int rs, bool deep = false);         // kt_grad3.hip (fused y/x/z gradients)
template <typename F> size_t k12_lds(int dtype, int rd, bool deep = false);                     // kt_grad3.hip
template <typename F> const void* k3_kernel(int np, int rw);                 // kt_prod_legacy.hip
template <typename F> const void* k4_kernel(int nf, int rw);                 // kt_prod_legacy.hip
template <typename F, int NP> const void* k34_fn(int rw, int s, int rb);     // kt_prod.hip
template <typename F, int NP> const void* k34_fn_uq(int rw, int s);         // kt_prod.hip (8-wave, unique staging)
template <typename F, int NP> const void* k34_fn_ws(int rw, int s, int npw, int pd);  // kt_prod.hip (16-wave, specialised)
template <int NP> const void* k34_fn_pk(int rw, int s);                        // kt_prod.hip (packed fp32)
template <typename F, typename RelT> const void* k5_kernel(int rw);          // kt_solve_legacy.hip
template <typename F, typename RelT> const void* k5_dma_kernel(int rw, int nb);  // kt_solve_legacy.hip
template <typename F, typename RelT> const void* k5c_fn(int rw, int nb, int r, int nw, int rt0 = 0);  // kt_solve.hip
}  // namespace of3dk
