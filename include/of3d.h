/*
 * of3d.h — C-ABI of the MI355X (gfx950) Lucas–Kanade optical-flow engine.
 *
 * Drop-in boundary for the hot path of ScientistRachel/OpticalFlow3D_dev:
 *   calc_flow3D(images, xyzSig, tSig, wSig) -> (vx, vy, vz, rel)   src/Python/calc_flow.py:175-360
 *   calc_flow2D(images, xySig,  tSig, wSig) -> (vx, vy, rel)       src/Python/calc_flow.py:18-173
 * The reference has no FFI of its own (pure NumPy/SciPy); the Python host in
 * opticalflow3d_dev_amd/calc_flow.py keeps those signatures and binds these
 * entry points with ctypes (binding shown in INTEGRATION.md).
 *
 * Conventions
 *  - Plain pointers and sizes only.  Arrays are C-ordered, x fastest:
 *    images (Nt, Nz, Ny, Nx) / (Nt, Ny, Nx); outputs (Nz, Ny, Nx) / (Ny, Nx).
 *  - Host entry points (of3d_flow3d / of3d_flow2d): the caller owns every host
 *    buffer; the library owns device memory (cached per shape+taps).
 *  - Device entry point (of3d_plan_execute): every pointer is device memory,
 *    work is enqueued on the given HIP stream (NULL = the device's null stream,
 *    HIP's own convention: ordered with the caller's default-stream work) and
 *    the call returns without synchronising.
 *  - Return 0 on success; non-zero = error, text in of3d_last_error()
 *    (thread-local).  The Python host maps the reference's argument checks
 *    (calc_flow.py:212-222) to SystemExit itself before calling in.
 *  - Taps are passed explicitly (full odd-length vectors, centre at index r),
 *    computed by the caller exactly as calc_flow.py:230-267 does; the library
 *    checks (anti)symmetry like scipy's NI_Correlate1D and uses the symmetric
 *    summation order (bit-exact with scipy.ndimage.correlate1d).
 */
#ifndef OF3D_H
#define OF3D_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OF3D_VERSION 10000 /* 1.0.0 */

/* element type of the input image stack (reference accepts any real dtype and
 * casts with images.astype(np.float64), calc_flow.py:225 / :67) */
enum of3d_dtype {
    OF3D_U8 = 1,
    OF3D_U16 = 2,
    OF3D_I16 = 3,
    OF3D_U32 = 4,
    OF3D_I32 = 5,
    OF3D_F32 = 6,
    OF3D_F64 = 7
};

/* arithmetic mode.  FP64_EXACT: fp64, no FMA contraction, scipy summation
 * order — vx/vy/vz bit-identical to the reference.  OR in OF3D_REL_F64 to get
 * the 3D reliability as float64 (the fp64 eigen-solve before the float32
 * cast; MATLAB's calc_flow3D.m:235-236 keeps rel in double).
 * OF3D_FP32 (plans only; configs[4]'s "fp32 path"): the filter passes and the
 * structure tensor in float32 (same scipy order), the 3x3 solve and the
 * eigenvalue in fp64, every output float32: half the workspace and HBM
 * traffic; accuracy max|dv| <= 1e-4 max|v| against the fp64 result. */
enum of3d_mode { OF3D_FP64_EXACT = 0, OF3D_REL_F64 = 0x100, OF3D_FP32 = 0x200 };

/* Filter taps (calc_flow.py:230-267).  Each vector has 2r+1 entries. */
typedef struct of3d_taps {
    const double* gauss;  /* fderiv == fx, radius rd = ceil(3*sig)       (:233,:253) */
    const double* deriv;  /* fderiv*gderiv, radius rd, antisymmetric     (:239)      */
    int rd;
    const double* smooth; /* fsmooth, radius rs = ceil(3*sig/4)          (:234)      */
    int rs;
    const double* tderiv; /* ft*gt, radius rt = ceil(3*tSig), antisym.    (:260)      */
    int rt;
    const double* window; /* gw, radius rw = ceil(3*wSig)                (:264)      */
    int rw;
} of3d_taps;

/* Optional timing record filled by the host entry points (milliseconds). */
typedef struct of3d_perf {
    double ms_h2d;     /* input upload                       */
    double ms_kernels; /* device time of the kernel pipeline  */
    double ms_d2h;     /* output download                     */
    double ms_total;   /* wall time of the call               */
} of3d_perf;

typedef struct of3d_plan of3d_plan;

/* Library version (OF3D_VERSION). */
int of3d_version(void);

/* Build provenance, a JSON object: {"src_hash": sha256 (first 16 hex digits) of the sources
 * the library was compiled from (csrc/Makefile HASH_FILES), "arch", "extra": the EXTRA
 * compile flags (empty for a product build), "flags"}.  The Python loader compares src_hash
 * with the sources beside the library and refuses a stale or EXTRA-flagged build.  No
 * reference counterpart (the reference has no compiled code). */
const char* of3d_build_info(void);

/* Last error message of the calling thread ("" if none). */
const char* of3d_last_error(void);

/* Number of visible HIP devices (0 when no GPU / no driver). */
int of3d_device_count(void);

/* Free the plans the host entry points cache (of3d_flow3d / of3d_flow2d keep the device
 * workspace of their last two shapes resident; tens of GB at configs[3]).  No reference
 * counterpart (calc_flow3D allocates per call). */
int of3d_cache_clear(void);

/* ---- host entry points (replace calc_flow3D / calc_flow2D) -------------- */

/* calc_flow3D (calc_flow.py:175-360).  images: (nt, nz, ny, nx) of `dtype`;
 * nt odd, only the centre frame c = (nt-1)/2 and frames c-rt..c+rt are read.
 * vx, vy, vz: float64 (nz, ny, nx); rel: float32 (nz, ny, nx) — the reference
 * returns rel from complex64 LAPACK, hence float32 (calc_flow.py:355-357) —
 * or float64 when mode has OF3D_REL_F64. */
int of3d_flow3d(const void* images, int dtype, int64_t nt, int64_t nz, int64_t ny, int64_t nx,
                const of3d_taps* taps, int mode, int device, double* vx, double* vy, double* vz,
                void* rel, of3d_perf* perf);

/* calc_flow2D (calc_flow.py:18-173).  images (nt, ny, nx); outputs float64
 * (ny, nx); rel = min root of the 2x2 characteristic quadratic (NaN where the
 * discriminant rounds negative, as NumPy gives). */
int of3d_flow2d(const void* images, int dtype, int64_t nt, int64_t ny, int64_t nx,
                const of3d_taps* taps, int mode, int device, double* vx, double* vy, double* rel,
                of3d_perf* perf);

/* ---- device-resident plan (streaming driver, benchmarks, z-slab shards) -- */

/* ndim 3: volume (nz, ny, nx); ndim 2: nz independent 2D frames processed
 * together (a batch of output frames: plane b of every frame pointer is the
 * image of window b, e.g. a series shifted by 0 .. 2rt frames; nz = 1 is
 * calc_flow2D's single frame).  Allocates the device workspace on `device`
 * for outputs over up to `max_out_planes` planes (<= 0: all nz). */
int of3d_plan_create(of3d_plan** plan, int ndim, int64_t nz, int64_t ny, int64_t nx,
                     const of3d_taps* taps, int mode, int device, int64_t max_out_planes);
int of3d_plan_destroy(of3d_plan* plan);

/* Device bytes held by the plan's workspace. */
size_t of3d_plan_workspace_bytes(const of3d_plan* plan);

/* Input planes a shard computing output planes [z_out0, z_out1) must hold
 * resident (global plane indices [*z_in0, *z_in1)): the stencil halo. */
int of3d_plan_input_range(const of3d_plan* plan, int64_t z_out0, int64_t z_out1, int64_t* z_in0,
                          int64_t* z_in1);

/* Run the pipeline for output planes [z_out0, z_out1) of the centre frame.
 * d_frames: host array of 2*rt+1 DEVICE pointers, frame c-rt .. c+rt of the
 *   stack, each pointing at global plane `frame_z0` of its frame (planes
 *   contiguous, row stride nx, plane stride ny*nx, elements of `dtype`).
 *   The frames must hold the planes of of3d_plan_input_range().
 * d_vx/d_vy/d_vz: float64 (z_out1-z_out0, ny, nx) (d_vz ignored for 2D);
 * d_rel: float32 for 3D (float64 if the plan's mode has OF3D_REL_F64),
 * float64 for 2D.  OF3D_FP32 plans: every output float32.
 * stream: hipStream_t, or NULL for the null stream (round 5; it used to mean the plan's own
 * non-blocking stream, which a torch caller passing its default stream's handle 0 got
 * unordered with its own kernels). */
int of3d_plan_execute(of3d_plan* plan, const void* const* d_frames, int dtype, int64_t frame_z0,
                      int64_t z_out0, int64_t z_out1, void* d_vx, void* d_vy, void* d_vz,
                      void* d_rel, void* stream);

/* Frame pipelining for a time series (the reference's per-frame loop, calc_flow.py:512-534):
 * of3d_plan_execute for d_frames, and — where the plan has the fused instance (uint16 frames,
 * serial schedule) — the W-z/solve kernel of this call also forms the temporal derivative of
 * the NEXT output frame from d_frames_next (2*rt+1 device pointers, same frame_z0 / planes;
 * their contents must be final when this call is enqueued).  The next of3d_plan_execute_next
 * call for exactly those frames and planes then skips its own K0 launch (a pure HBM stream
 * riding in the VALU-bound kernel's memory slack).  d_frames_next NULL: no lookahead.  Any
 * other call (of3d_plan_execute included) recomputes.  Results are bit-identical to
 * of3d_plan_execute (the same K0 arithmetic, k0_group). */
int of3d_plan_execute_next(of3d_plan* plan, const void* const* d_frames, const void* const* d_frames_next, int dtype,
                           int64_t frame_z0, int64_t z_out0, int64_t z_out1, void* d_vx, void* d_vy, void* d_vz,
                           void* d_rel, void* stream);

/* K0 batching for a time series (calc_flow.py:512-534 again): d_frames holds the frames
 * c-rt .. c+rt+n_ahead (2*rt+1+n_ahead device pointers: the current window, then the next
 * n_ahead frames, all resident and final when this call is enqueued).  of3d_plan_execute for
 * the window d_frames[0 .. 2rt]; where the plan runs the fused gradient kernel (serial
 * schedule, the vectorised frame layout) and no earlier call formed this window's temporal
 * derivative, one pass over the 2rt+1+m frames forms it AND the next m-1 windows' (m =
 * min(n_ahead, 4) + 1: 2rt+m frame reads for m derivatives instead of m(2rt+1)); the later
 * of3d_plan_execute_ahead calls for exactly those windows (frame pointers, dtype, frame_z0,
 * planes) skip their K0.  Calls on one stream (or otherwise ordered); any other execute call
 * drops the formed derivatives.  n_ahead past 65 - (2rt+1) frames is clamped (no batching
 * beyond the 65-frame pointer table); radii without a batched K0 instance (rt other than
 * 3, 6, 9) run the plain K0.  Bit-identical to of3d_plan_execute. */
int of3d_plan_execute_ahead(of3d_plan* plan, const void* const* d_frames, int n_ahead, int dtype, int64_t frame_z0,
                            int64_t z_out0, int64_t z_out1, void* d_vx, void* d_vy, void* d_vz, void* d_rel,
                            void* stream);

/* Per-stage timing with HIP events recorded on the launch stream.
 * of3d_plan_set_timing(plan, slots): keep a ring of `slots` executions
 * (0 = off; no host synchronisation is added to of3d_plan_execute).
 * of3d_plan_stage_times: average device time (ms) per stage over the
 * executions recorded since the previous read (at most `slots`), then reset;
 * returns the number of stages written (<= cap).  Stage names:
 * of3d_stage_name(i) = grad_xy, grad_z, prod_wy, wx, wz_solve.
 * of3d_plan_set_timing_mask(plan, mask): time only the stages in the bit
 * mask (bit i = stage i; default all).  Each event is a barrier packet
 * between two kernels, so fewer events perturb the pipeline less; stages
 * outside the mask read back as -1. */
int of3d_plan_set_timing(of3d_plan* plan, int slots);
int of3d_plan_set_timing_mask(of3d_plan* plan, unsigned mask);
int of3d_plan_stage_times(of3d_plan* plan, double* ms, int cap);

/* Overlap mode (3D plans with the fused products/W-xy kernel): of3d_plan_execute
 * splits the output planes into chunks of `chunk_planes` (<= 0: off, the default
 * unless OF3D_ZCHUNK is set; at most 16 chunks) and runs the HBM-bound gradient
 * stages of chunk c+1 on the caller's stream beside the VALU-bound W-xy / W-z /
 * solve stages of chunk c on the plan's second stream (joined back into the
 * caller's stream before the call's work completes).  Results are bit-identical
 * to the serial order.  A per-stage profile (timing mask with several stages)
 * runs serially; with one timed stage its time is summed over the chunks.  Fails while the
 * plan has an output row range (of3d_plan_set_rows), as set_rows fails on a chunked plan. */
int of3d_plan_set_overlap(of3d_plan* plan, int64_t chunk_planes);

/* Output rows (3D plans with the fused products/W-xy and W-z kernels): of3d_plan_execute
 * then writes only rows [y0, y1) of each output plane, as a compact (z_out1-z_out0,
 * y1-y0, nx) array; the earlier stages still run on every row (the W-y halo).  A row-slab
 * shard runs its rows + rd + rw halo rows as the plan's volume and keeps its own rows
 * this way (no reference counterpart: calc_flow.py:512's parallel loop, split by rows).
 * Fails (non-zero) where those kernels are not in use; (0, ny) restores the default. */
int of3d_plan_set_rows(of3d_plan* plan, int64_t y0, int64_t y1);

/* Kernel families this plan has launched so far, comma-separated (e.g.
 * "k_tderiv_c,k_grad_xyz_c,k_prod_wyx_ws,k_wz_solve_c"), written NUL-terminated into
 * buf (at most n bytes); returns the full length.  Diagnostics: which kernels a
 * parameter set / volume shape runs on (no reference counterpart). */
int of3d_plan_kernels(const of3d_plan* plan, char* buf, size_t n);
const char* of3d_stage_name(int i);

/* The plan's kernel geometry as a JSON object, written like of3d_plan_kernels (returns the
 * full length): the W-xy hand-off layout (wxy_zt: 0 plain planes, else z-tiled), the K34 shape
 * the autotune kept (staged columns, tile rows s, outputs per block, threads, candidates), the K5c
 * block (planes per z-group, waves), and of the LAST execution the K12 march length and grid and
 * the batched-K0 windows.  Diagnostics for tests and benchmarks (no reference counterpart). */
int of3d_plan_geometry(const of3d_plan* plan, char* buf, size_t n);

/* Copy `bytes` from src to dst on `stream` with a kernel of at most
 * `max_blocks` workgroups (0 = 64).  Either side may be pinned host memory
 * (hipHostMalloc / torch pin_memory): used to download a frame's outputs
 * over PCIe while the next frame's kernels keep the rest of the GPU (the
 * runtime's own device->host copy runs as a full-GPU blit kernel).
 * No reference counterpart: process_flow's per-frame output transfer
 * (calc_flow.py:526-529 writes host arrays). */
int of3d_copy_async(void* dst, const void* src, size_t bytes, int max_blocks, void* stream);

/* Downstream statistics on resident outputs (device pointers), one pass —
 * the reference's example_analysis_script.ipynb cells 4-6:
 * mask = rel > thresh (thresh: e.g. the 90th percentile of rel); each of
 * vx, vy, vz multiplied by the mask, exact zeros -> NaN, then scaled to
 * physical units ((v*xyscale)/tscale; vz with zscale); magnitude, theta =
 * atan2(vy, vx), phi = atan(vz / sqrt(vx^2 + vy^2)).  Inputs float64 (or
 * float32 with v_f32), rel float32 (or float64 with rel_f64); outputs
 * float64.  2D: vz = out_vz = phi = NULL.  Enqueued on `stream`. */
int of3d_flow_stats(const void* vx, const void* vy, const void* vz, const void* rel, int v_f32, int rel_f64,
                    int64_t n, double thresh, double xyscale, double zscale, double tscale, double* out_vx,
                    double* out_vy, double* out_vz, double* magnitude, double* theta, double* phi, void* stream);

/* Reliability (smallest eigenvalue) of n given symmetric 3x3 structure tensors
 * resident on the device: `tensor` is field-major [6][n] float64 in the order
 * x2 y2 z2 xy xz yz (calc_flow.py:352-354's matrix (x2 xy xz / xy y2 yz /
 * xz yz z2)); `rel` receives float32 (the reference's complex64 cgeev
 * precision, calc_flow.py:355-357) or, with rel_f64, float64 (MATLAB's double
 * pageeig, M/calc_flow3D.m:235-236) — exactly the values the flow kernels
 * store for those tensors.  Enqueued on `stream`. */
int of3d_rel3d(const double* tensor, int64_t n, void* rel, int rel_f64, void* stream);

/* Blocking copy of n buffers on the GPU's DMA (SDMA) engines through the HSA
 * runtime: no compute units and no HIP stream involved, so a download does
 * not contend with kernels for the memory pipeline.  Host buffers must be
 * pinned.  The caller orders it after the producing work (e.g. a download
 * thread after hipEventSynchronize).  Releases no locks of its own; safe to
 * call from several threads. */
int of3d_dma_copy(void* const* dst, const void* const* src, const size_t* bytes, int n);

#ifdef __cplusplus
}
#endif
#endif /* OF3D_H */
