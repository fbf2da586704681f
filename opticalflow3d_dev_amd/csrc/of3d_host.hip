// of3d_host.hip — host side of libof3d: plans, the stage pipeline, the C-ABI (include/of3d.h).
// Device code: of3d_dev.hpp; kernel instances behind getters in kt_*.hip (kernels.hpp).
#include "of3d_dev.hpp"
#include "kernels.hpp"

namespace {

using namespace of3dk;


// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
size_t dtype_size(int dt) {
    switch (dt) {
        case OF3D_U8: return 1;
        case OF3D_U16:
        case OF3D_I16: return 2;
        case OF3D_U32:
        case OF3D_I32:
        case OF3D_F32: return 4;
        case OF3D_F64: return 8;
        default: return 0;
    }
}

// scipy NI_Correlate1D symmetry classification: +1, -1, 0
int symmetry(const double* w, int r) {
    bool sym = true, anti = true;
    for (int k = 1; k <= r; ++k) {
        if (std::fabs(w[r + k] - w[r - k]) > kEps) sym = false;
        if (std::fabs(w[r + k] + w[r - k]) > kEps) anti = false;
    }
    return sym ? 1 : (anti ? -1 : 0);
}

const char* kStageNames[] = {"grad_xy", "grad_z", "prod_wy", "wx", "wz_solve"};
constexpr int kStages = 5;
constexpr int kMaxChunks = 16;  // overlap mode: most z chunks per execution

}  // namespace

// kernel families (of3d_plan_kernels)
enum : unsigned {
    KU_K0C = 1u << 0, KU_K0 = 1u << 1, KU_K1C = 1u << 2, KU_K1 = 1u << 3, KU_K12 = 1u << 4, KU_K2C = 1u << 5,
    KU_K2 = 1u << 6, KU_K34 = 1u << 7, KU_K34WS = 1u << 8, KU_K3 = 1u << 9, KU_K4 = 1u << 10, KU_K5C = 1u << 11,
    KU_K5C_2 = 1u << 12 /* (the packed-fp32 K5c, removed) */, KU_K5DMA = 1u << 13, KU_K5 = 1u << 14, KU_SOLVE2D = 1u << 15, KU_GENERAL = 1u << 16,
    KU_K34PK = 1u << 17, KU_K5C_NEXT = 1u << 18, KU_K0M = 1u << 19,
};
constexpr const char* kKernelNames[] = {"k_tderiv_c", "k_tderiv",     "k_grad_xy_c",    "k_grad_xy",  "k_grad_xyz_c",
                                        "k_grad_z_c", "k_grad_z",     "k_prod_wyx",     "k_prod_wyx_ws", "k_prod_wy",
                                        "k_wx",       "k_wz_solve_c", "k_wz_solve_c2",  "k_wz_solve_dma", "k_wz_solve",
                                        "k_solve2d",  "general",      "k_prod_wyx_pk",  "k_wz_solve_c_next",
                                        "k_tderiv_multi"};

// Kernel-family switches, read from the environment once per plan (at of3d_plan_create; the
// host entry's plan cache keys on them too).  The defaults are the product; the tests force each
// family in turn to check that every one gives the same bits (INTEGRATION.md §5 lists them).
struct Knobs {
    bool k0c = true;      // OF3D_K0C=0: runtime-radius K0 instead of the compile-time one
    bool k1c = true;      // OF3D_K1C=0: k_grad_xy instead of the column-march K1c
    bool k2c = true;      // OF3D_K2C=0: k_grad_z instead of the z-march K2c
    int k12 = -1;         // OF3D_K12: 0 off, 1 forced, -1 by volume size
    int k12_zc = 0;       // OF3D_K12_ZC: forced K12 march length (planes; 0: by volume size)
    bool k34 = true;      // OF3D_K34=0: K3 + K4 instead of the fused K34
    int k34_uq = -1;      // OF3D_K34_UQ: 0 duplicate staging, 1 unique, 2 wave-specialised, 3 packed fp32 only
    bool k34_ws = true;   // OF3D_K34_WS=0: no wave-specialised candidates
    bool k34_pk = true;   // OF3D_K34_PK=0: no packed-fp32 candidates
    int k34_cand = -1;    // OF3D_K34_CAND=i: pin candidate i (no autotune)
    bool k34_strict = false;  // OF3D_K34_CAND_STRICT=1: a pin past the candidates fails
    bool k34_tune = true;     // OF3D_K34_TUNE=0: the heuristic pick, untimed
    bool k5c = true;      // OF3D_K5C=0: k_wz_solve_dma / k_wz_solve instead of K5c
    int k5c_r = 0;        // OF3D_K5C_R=4 / 8: 32- / 64-plane K5c blocks (0: by workspace size)
    int k5c_nw = 4;       // OF3D_K5C_NW=8: 8-wave, 128-plane K5c blocks
    int wxy_tile = -1;    // OF3D_WXY_TILE=0 / 1: the W-xy hand-off in plain planes / z-tiled (-1: by size)
    bool pipe = true;     // OF3D_PIPE=0: no next-frame K0 inside K5c
    bool general = false;  // OF3D_GENERAL=1: the general-radius path
    int64_t zchunk = 0;   // OF3D_ZCHUNK: overlap mode's z chunk (planes; 0 serial)
    int verbose = 0;      // OF3D_VERBOSE: plan choices on stderr
    static Knobs read() {
        Knobs k;
        auto iv = [](const char* name, long dflt) {
            const char* e = getenv(name);
            return (e && e[0]) ? atol(e) : dflt;
        };
        k.k0c = iv("OF3D_K0C", 1) != 0;
        k.k1c = iv("OF3D_K1C", 1) != 0;
        k.k2c = iv("OF3D_K2C", 1) != 0;
        k.k12 = (int)iv("OF3D_K12", -1);
        k.k12_zc = (int)iv("OF3D_K12_ZC", 0);
        k.k34 = iv("OF3D_K34", 1) != 0;
        k.k34_uq = (int)iv("OF3D_K34_UQ", -1);
        k.k34_ws = iv("OF3D_K34_WS", 1) != 0;
        k.k34_pk = iv("OF3D_K34_PK", 1) != 0;
        k.k34_cand = (int)iv("OF3D_K34_CAND", -1);
        k.k34_strict = iv("OF3D_K34_CAND_STRICT", 0) == 1;
        k.k34_tune = iv("OF3D_K34_TUNE", 1) != 0;
        k.k5c = iv("OF3D_K5C", 1) != 0;
        k.k5c_r = (int)iv("OF3D_K5C_R", 0);
        k.k5c_r = k.k5c_r == 4 ? 4 : (k.k5c_r == 8 ? 8 : 0);
        k.k5c_nw = iv("OF3D_K5C_NW", 4) == 8 ? 8 : 4;
        k.wxy_tile = (int)iv("OF3D_WXY_TILE", -1);
        k.pipe = iv("OF3D_PIPE", 1) != 0;
        k.general = iv("OF3D_GENERAL", 0) == 1;
        k.zchunk = std::max(0L, iv("OF3D_ZCHUNK", 0));
        k.verbose = (int)iv("OF3D_VERBOSE", 0);
        return k;
    }
    auto tie() const {
        return std::tie(k0c, k1c, k2c, k12, k12_zc, k34, k34_uq, k34_ws, k34_pk, k34_cand, k34_strict, k34_tune, k5c,
                        k5c_r, k5c_nw, wxy_tile, pipe, general, zchunk, verbose);
    }
    bool operator==(const Knobs& o) const { return tie() == o.tie(); }
};

struct of3d_plan {
    Knobs kn;  // read at creation
    int ndim = 3;
    bool rel64 = false;  // OF3D_REL_F64
    bool fp32 = false;   // OF3D_FP32: passes in float
    int64_t nz = 1, ny = 1, nx = 1;
    int rd = 0, rs = 0, rt = 0, rw = 0;
    int device = 0;
    int ncu = 256;           // compute units of the device (K12 march-length model)
    int64_t cap_planes = 0;  // planes per workspace field
    std::vector<double> htaps;  // host copy of half taps (g | d | s | t | w)
    double* d_taps = nullptr;   // fp64 taps
    float* d_taps32 = nullptr;  // the same rounded to float (OF3D_FP32)
    void* X = nullptr;          // 9 fields of the pass type
    void* Y = nullptr;          // 9 fields
    size_t fs = 0;        // field stride (elements)
    hipStream_t stream = nullptr;
    size_t k1_lds = 0, k2_lds = 0, k3_lds = 0, k4_lds = 0, k5_lds = 0;
    int k5_nb = 0;       // LDS-DMA K5 buffers (0: register-staged K5)
    size_t k5d_lds = 0;
    bool general = false;  // radii beyond the tiled kernels' limits: the general-radius path
    // K5c (compile-time-radius W z + solve); nullptr: k_wz_solve_dma / k_wz_solve
    const void* k5c = nullptr;
    size_t k5c_lds = 0;
    int k5c_r = 8;  // planes per z-group (8: 64-plane blocks, 2 per CU; 4: 32-plane blocks, 3 per CU)
    const void* k5c_next = nullptr;  // K5c that also forms the next frame's dt0 (frame pipelining)
    // W-xy hand-off layout (K34 -> K5c, csrc/of3d_dev.hpp wxy_rsrc): 0 plain planes, else z-tiled
    // [y][x / 32][z][32] with this many planes (cap_planes)
    int wxy_zt = 0;
    // frame pipelining (of3d_plan_execute_next): the dt0 a previous call formed for these frames
    bool pipe_valid = false;
    const void* pipe_frames[kMaxT] = {};
    int64_t pipe_fz0 = 0, pipe_zo0 = 0, pipe_zo1 = 0;
    int pipe_dtype = 0;
    bool pipe_k12 = false;  // the producing call's flow (dt0 in Y4 with K12, else Y0)
    // K0 batching (of3d_plan_execute_ahead): dt0 slots Y4 .. Y4 + kDtSlots - 1 (K12 flow, whose
    // workspace leaves Y4..Y8 free), each tagged with the window it was formed for; the call
    // that uses a slot consumes it, and any other call drops them all
    static constexpr int kDtSlots = 5;  // Y4 .. Y8
    struct DtSlot {
        bool valid = false;
        const void* frames[kMaxT] = {};
        int dtype = 0;
        int64_t fz0 = 0, zo0 = 0, zo1 = 0;
    } dts[kDtSlots];
    int k5c_nw = 4;       // K5c waves per block (8: 128-plane blocks)
    int64_t ya = 0, yb = 0;  // output rows [ya, yb) (of3d_plan_set_rows; default all)
    unsigned used = 0;       // kernel families launched so far (KU_* bits, of3d_plan_kernels)
    // geometry of the last execution (of3d_plan_geometry): K12 march length and grid, K0 windows
    int last_k12_zc = 0, last_k12_gx = 0, last_k12_gy = 0, last_k12_deep = 0, last_k0m = 0;
    hipEvent_t ev_done = nullptr;  // recorded on the caller's stream at the end of every execution
    // fused K34 (products + W y + W x); fn == nullptr: separate K3 and K4
    struct K34Geom {
        const void* fn = nullptr;
        int cw = 0, s = 0, tx = 0, nbx = 0;
        size_t lds = 0;
        int nthr = 0;  // threads per block when not cw (wave-specialised: 2 cw; packed fp32: cw)
    } k34;
    std::vector<K34Geom> k34_cand;  // geometries that keep >= 8 waves per CU (k34_tune picks)
    bool host_ev = false;            // host entry: record into ev[]
    hipEvent_t ev[kStages + 1] = {};
    // overlap mode (run_t): output planes per chunk (0 = serial), second stream, chunk events
    int64_t zchunk = 0;
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipEvent_t ev_chunk[kMaxChunks] = {};
    int timing_slots = 0;            // of3d_plan_set_timing: ring of per-execution event sets
    int tev_per_slot = kStages + 1;  // events per slot: serial boundaries or 2 per chunk of one stage
    std::vector<int> tchunks;        // per slot: chunks timed (overlap mode, one stage) or 0 (serial)
    unsigned timing_mask = (1u << kStages) - 1;  // stages timed (events at their two boundaries)
    std::vector<hipEvent_t> tev;     // timing_slots * (kStages + 1)
    int64_t tcount = 0;              // executions recorded since the last of3d_plan_stage_times
    double stage_ms[kStages] = {};
    int stages_run = 0;
    // host-entry staging
    void* d_in = nullptr;
    size_t d_in_bytes = 0;
    void* d_out = nullptr;
    size_t d_out_bytes = 0;
};

namespace {

int build_taps(const of3d_taps* t, of3d_plan* p) {
    if (!t || !t->gauss || !t->deriv || !t->smooth || !t->tderiv || !t->window) return fail("of3d: null taps");
    if (t->rd < 0 || t->rs < 0 || t->rt < 0 || t->rw < 0) return fail("of3d: negative tap radius");
    if (t->rd > 4096 || t->rs > 4096 || t->rw > 4096) return fail("of3d: spatial tap radius exceeds 4096");
    if (2 * t->rt + 1 > kMaxT) return fail("of3d: temporal tap radius exceeds 32");
    struct {
        const double* w;
        int r;
        int want;
        const char* name;
    } f[5] = {{t->gauss, t->rd, 1, "gauss"},
              {t->deriv, t->rd, -1, "deriv"},
              {t->smooth, t->rs, 1, "smooth"},
              {t->tderiv, t->rt, -1, "tderiv"},
              {t->window, t->rw, 1, "window"}};
    p->htaps.clear();
    for (auto& e : f) {
        if (e.r > 0 && symmetry(e.w, e.r) != e.want)
            return fail(std::string("of3d: taps '") + e.name + "' do not have the expected (anti)symmetry");
        for (int k = 0; k <= e.r; ++k) p->htaps.push_back(e.w[e.r - k]);
    }
    for (auto& e : f) {  // step-order copies for lds_pass: w[0 .. r-1], then kTapPad zeros
        for (int q = 0; q < e.r; ++q) p->htaps.push_back(e.w[q]);
        for (int z = 0; z < kTapPad; ++z) p->htaps.push_back(0.0);
    }
    p->rd = t->rd;
    p->rs = t->rs;
    p->rt = t->rt;
    p->rw = t->rw;
    return 0;
}

template <typename F>
DevTaps<F> dev_taps(const of3d_plan* p) {
    DevTaps<F> d;
    const F* b;
    if constexpr (sizeof(F) == 8)
        b = p->d_taps;
    else
        b = p->d_taps32;
    d.g = b;
    d.d = d.g + p->rd + 1;
    d.s = d.d + p->rd + 1;
    d.t = d.s + p->rs + 1;
    d.w = d.t + p->rt + 1;
    d.gr = d.w + p->rw + 1;
    d.dr = d.gr + p->rd + kTapPad;
    d.sr = d.dr + p->rd + kTapPad;
    d.tr = d.sr + p->rs + kTapPad;
    d.wr = d.tr + p->rt + kTapPad;
    d.rd = p->rd;
    d.rs = p->rs;
    d.rt = p->rt;
    d.rw = p->rw;
    return d;
}

unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }





int k0_vec_width(int dtype) {
    const size_t es = dtype_size(dtype);
    return es == 1 ? 8 : (es == 8 ? 2 : 4);
}









// K34 geometry.  Two kernel families:
//  - duplicate staging (k_prod_wyx UQ = false, 168 VGPRs): blocks of nw in {1, 2, 3, 4} waves,
//    cw = 64 nw staged columns, tx = (cw - 2 rw) & ~3 outputs (halo columns recomputed,
//    clamped ones as duplicates of the edge column);
//  - unique staging (UQ = true, 256 VGPRs, nw in {4, 8}): each column once, edge replicas
//    copied, so a block covering the whole row (nx <= 64 nw) stages no halo at all; the column
//    stride is the one with the fewest staged lanes.
// The heuristic pick: fewest staged lanes among the duplicate-staging shapes keeping >= 8 waves
// per CU resident (LDS and registers from the occupancy API), ties to the higher occupancy;
// k34_tune then times every candidate of both families on the plan's workspace.
// Staged lanes of the stride-tx unique-staging partition of a row, and the widest block.
long k34_lanes(int nx, int rw, int tx, int& widest) {
    long lanes = 0;
    widest = 0;
    for (int x0 = 0; x0 < nx; x0 += tx) {
        const int txu = std::min(tx, nx - x0);
        const int ns = std::min(x0 + txu + rw, nx) - std::max(x0 - rw, 0);
        widest = std::max(widest, ns);
        lanes += 64L * ((ns + 63) / 64);
    }
    return lanes;
}

template <typename F>
int k34_setup(of3d_plan* p, int np) {
    p->k34 = {};
    p->k34_cand.clear();
    const Knobs& kn = p->kn;
    if (!kn.k34) return 0;
    const int rw = p->rw, nx = (int)p->nx;
    const size_t es = sizeof(F);
    if ((size_t)p->ny * p->nx * es > 0x7fffffffu) return 0;  // 32-bit buffer offsets within a plane
    long best_lanes = 0;
    int best_waves = 0;
    const int uq = kn.k34_uq;  // 0: duplicate staging only, 1: unique only (2: specialised, 3: packed fp32 only)
    auto occupancy = [&](const void* fn, int cw, size_t lds, int& waves) -> int {
        OF3D_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        int nb = 0;
        OF3D_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, cw, lds));
        waves = nb * (cw / 64);
        return 0;
    };
    // the unique-staging column stride for blocks of cw staged columns: fewest staged lanes (64 per
    // started wave of each block), ties to the wider stride (fewer blocks); 0: none fits
    auto uq_stride = [&](int cw) {
        int tx = 0;
        long lanes = 0;
        for (int nbx = 1; nbx <= 64; ++nbx) {
            const int t = nbx == 1 ? nx : ((nx + nbx - 1) / nbx + 3) & ~3;
            if (t < 8) break;
            int widest = 0;
            const long l = k34_lanes(nx, rw, t, widest);
            if (widest > cw) continue;
            if (!tx || l < lanes) tx = t, lanes = l;
        }
        return tx;
    };
    for (int s : {16, 8, 4}) {
        // wave-specialised with 9 producer waves (576 staged columns, fp64): rows whose 512-column
        // blocks would need more than 512 staged columns (nx 1024: 2 x (512 + 15) instead of 3 x 344)
        for (int pd : {2, 4}) {
            const void* f9 = (uq != 0 && uq != 1 && uq != 3 && kn.k34_ws)
                                 ? (np == 9 ? k34_fn_ws<F, 9>(rw, s, 9, pd) : k34_fn_ws<F, 5>(rw, s, 9, pd)) : nullptr;
            const int tx = f9 ? uq_stride(576) : 0, tx8 = uq_stride(512);
            if (tx && (!tx8 || (nx + tx - 1) / tx < (nx + tx8 - 1) / tx8)) {  // only where it saves blocks
                const size_t lds = (size_t)2 * k34_tile(s, k34_pitch(std::min(tx, nx), rw)) * es;
                int w9 = 0;
                if (lds <= 160 * 1024 && !occupancy(f9, 1024, lds, w9) && w9 >= 16)
                    p->k34_cand.push_back({f9, 576, s, tx, (nx + tx - 1) / tx, lds, 1024});
            }
        }
        const void* fd = uq == 1 ? nullptr : (np == 9 ? k34_fn<F, 9>(rw, s, 4) : k34_fn<F, 5>(rw, s, 4));
        const void* fu = uq == 0 ? nullptr : (np == 9 ? k34_fn_uq<F, 9>(rw, s) : k34_fn_uq<F, 5>(rw, s));
        for (int nw : {1, 2, 3, 4, 8}) {  // launch bound 512
            const int cw = 64 * nw;
            if (fd && nw <= 4) {  // duplicate staging
                const int tx = (cw - 2 * rw) & ~3;  // whole phase-B items
                if (tx >= 8) {
                    const int nbx = (nx + tx - 1) / tx;
                    const size_t lds = (size_t)2 * k34_tile(s, cw + 1) * es;  // two W-y tiles
                    int waves = 0;
                    if (lds <= 160 * 1024 && !occupancy(fd, cw, lds, waves) && waves > 0) {
                        const long lanes = (long)(nbx - 1) * cw + 64 * ((nx - (nbx - 1) * tx + 2 * rw + 63) / 64);
                        const bool ok = waves >= 8, best_ok = best_waves >= 8;
                        if (ok) p->k34_cand.push_back({fd, cw, s, tx, nbx, lds});
                        const bool better =
                            !p->k34.fn || (ok && !best_ok) ||
                            (ok == best_ok &&
                             (ok ? (lanes < best_lanes || (lanes == best_lanes && waves > best_waves)) : waves > best_waves));
                        if (better) {
                            p->k34 = {fd, cw, s, tx, nbx, lds};
                            best_lanes = lanes;
                            best_waves = waves;
                        }
                    }
                }
            }
            if (fu && nw >= 4) {  // unique staging: the column stride with the fewest staged lanes
                const int tx = uq_stride(cw);
                if (tx) {
                    const int nbx = (nx + tx - 1) / tx;
                    const size_t lds = (size_t)2 * k34_tile(s, k34_pitch(std::min(tx, nx), rw)) * es;
                    int waves = 0;
                    if (lds <= 160 * 1024 && !occupancy(fu, cw, lds, waves) && waves >= nw)
                        p->k34_cand.push_back({fu, cw, s, tx, nbx, lds});
                    // the wave-specialised form of the same geometry (8 producer + 8 consumer waves)
                    const void* fw =
                (nw == 8 && kn.k34_ws) ? (np == 9 ? k34_fn_ws<F, 9>(rw, s, 8, 2) : k34_fn_ws<F, 5>(rw, s, 8, 2)) : nullptr;
                    int wsw = 0;
                    if (fw && lds <= 160 * 1024 && !occupancy(fw, 2 * cw, lds, wsw) && wsw >= 2 * nw)
                        p->k34_cand.push_back({fw, cw, s, tx, nbx, lds, 2 * cw});
                    // ... with 4 rows of gradient prefetch (fp64 radii <= 15, 4-row tiles)
                    const void* fw4 = (nw == 8 && kn.k34_ws)
                                          ? (np == 9 ? k34_fn_ws<F, 9>(rw, s, 8, 4) : k34_fn_ws<F, 5>(rw, s, 8, 4))
                                          : nullptr;
                    if (fw4 && lds <= 160 * 1024 && !occupancy(fw4, 2 * cw, lds, wsw) && wsw >= 2 * nw)
                        p->k34_cand.push_back({fw4, cw, s, tx, nbx, lds, 2 * cw});
                    // fp32: the packed form (column pairs / row pairs on float2, 8-wave blocks)
                    if constexpr (sizeof(F) == 4) {
                        const void* fp =
                            (nw == 8 && kn.k34_pk) ? (np == 9 ? k34_fn_pk<9>(rw, s) : k34_fn_pk<5>(rw, s)) : nullptr;
                        const size_t lpk = (size_t)s * k34_pitch(std::min(tx, nx), rw) * 8;
                        int pkw = 0;
                        if (fp && lpk <= 160 * 1024 && !occupancy(fp, cw, lpk, pkw) && pkw >= nw)
                            p->k34_cand.push_back({fp, cw, s, tx, nbx, lpk, cw});
                    }
                }
            }
        }
    }
    if (uq == 2 || uq == 3) {  // tests: wave-specialised (3: packed fp32) only
        std::vector<of3d_plan::K34Geom> ws;
        for (const auto& k : p->k34_cand)
            if (k.nthr && (uq == 2 || k.nthr == k.cw)) ws.push_back(k);
        p->k34_cand = ws;
        p->k34 = ws.empty() ? of3d_plan::K34Geom{} : ws.front();
    }
    if (!p->k34.fn && !p->k34_cand.empty()) p->k34 = p->k34_cand.front();
    for (const auto& k : p->k34_cand)
        OF3D_HIP(hipFuncSetAttribute(k.fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    if (p->k34.fn)
        OF3D_HIP(hipFuncSetAttribute(p->k34.fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    if (kn.verbose && p->k34.fn)
        fprintf(stderr, "of3d: K34 cw=%d s=%d tx=%d nbx=%d lds=%zu lanes=%ld waves/CU=%d\n", p->k34.cw, p->k34.s,
                p->k34.tx, p->k34.nbx, p->k34.lds, best_lanes, best_waves);
    return 0;
}


template <typename F>
int k5c_setup(of3d_plan* p) {
    p->k5c = nullptr;
    p->k5c_next = nullptr;
    p->k5c_nw = 4;
    if (!p->kn.k5c) return 0;
    if (p->ndim != 3 || p->nx % (16 / (int)sizeof(F))) return 0;  // 16-byte DMA rows
    // planes per z-group: 8 (64-plane blocks) or 4 (32; OF3D_K5C_R=4), the compiled instances
    // (k5c_fn).  A 128-plane fp32 instance (R 16, 191 VGPRs) measured slower (c5 fp32 41.8 vs
    // 39.7 ms), so did 6 planes (48-plane blocks, three per CU: c3 K5c 1.00 -> 1.05 ms,
    // profiles/r04/ab_k5r6/) and the packed-fp32 K5c (float2 lanes: c5 36.5 vs 34.5 ms, round 4,
    // profiles/r04/ab_k5c_fp32/; removed in round 5)
    // by size (OF3D_K5C_R unset): 32-plane blocks (three per CU) where the nine W-xy fields mostly sit
    // in the 256 MB Infinity Cache, so the window's 1.94x re-read costs little and the third block
    // per CU pays: c2 (302 MB) K5c 0.109 / 0.109 vs 0.118 / 0.115 ms, frame 0.379 / 0.378 vs
    // 0.388 / 0.381 (profiles/r05/ab_c2_k5c_r4/); 64-plane blocks for every larger workspace
    int r = p->kn.k5c_r;
    if (r == 0) r = (size_t)9 * p->cap_planes * p->ny * p->nx * sizeof(F) <= ((size_t)320 << 20) ? 4 : 8;
    // OF3D_K5C_NW=8: 8-wave blocks of 128 output planes (window 1.33x the outputs instead of
    // 1.66x; one block per CU) — bit-identical but measured no faster (c3 1.118 vs 1.121 ms,
    // c4 8.54 vs 7.90, c5 fp32 43.6 vs 40.4): K5c is not bound by its window re-reads
    int nw = p->kn.k5c_nw;
    if (nw == 8) r = 8;  // the 8-wave instances are R 8 only (k5c_fn): grid and LDS follow r
    size_t buf = (size_t)k5c_groups<F>(p->rw, r, nw) * 1024;
    int nb = nw == 8 ? (3 * buf <= 160 * 1024 ? 3 : 0) : (2 * 3 * buf <= 160 * 1024 ? 3 : 2);  // 4 waves: two blocks per CU
    const void* fn = nb ? (p->rel64 ? k5c_fn<F, double>(p->rw, nb, r, nw) : k5c_fn<F, float>(p->rw, nb, r, nw)) : nullptr;
    if (!fn && nw == 8) {  // no 8-wave instance: the 4-wave one
        nw = 4;
        buf = (size_t)k5c_groups<F>(p->rw, r, nw) * 1024;
        nb = 2 * 3 * buf <= 160 * 1024 ? 3 : 2;
        fn = p->rel64 ? k5c_fn<F, double>(p->rw, nb, r, nw) : k5c_fn<F, float>(p->rw, nb, r, nw);
    }
    if (!fn) return 0;
    p->k5c_nw = nw;
    p->k5c_r = r;
    p->k5c_lds = nb * buf;
    OF3D_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p->k5c_lds));
    p->k5c = fn;
    // the same geometry with the next frame's K0 after the solve (uint16 frames; OF3D_PIPE=0: off)
    p->k5c_next = nullptr;
    if (p->kn.pipe) {
        const void* fx = p->rel64 ? k5c_fn<F, double>(p->rw, nb, r, nw, p->rt) : k5c_fn<F, float>(p->rw, nb, r, nw, p->rt);
        if (fx) {
            OF3D_HIP(hipFuncSetAttribute(fx, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p->k5c_lds));
            p->k5c_next = fx;
        }
    }
    return 0;
}

// One K34 launch over ng planes of nf products.  Rows are cut into chunks of >= 32
// rows (each chunk re-reads 2 rw halo rows) until there are >= 2048 blocks; blocks of one group share an XCD: all row chunks of a plane when there are
// planes enough to spread over the 8 XCDs (their halo rows then come from one L2).
template <typename K, typename F>
hipError_t launch_k34(const K& k, const F* G, F* P, int ng, int nf, int ny, int nx, size_t fs, const F* hw,
                      hipStream_t s, int zt, int yb0 = 0, int yb1 = -1) {
    if (yb1 < 0) yb1 = ny;
    const int nyo = yb1 - yb0;  // output rows (row-slab plans: the rank's own rows)
    int tx = k.tx, nbx = k.nbx;
    const int nyb_max = std::max(1, nyo / 32);
    // block target 2048: longer row chunks re-read fewer halo rows (c3 wave-specialised K34 1.67
    // vs 1.76 ms at 4096, 1.73 at 1024; c2 lockstep K34 0.175 vs 0.191 ms, frame 0.420 vs 0.435;
    // c4 neutral).  (A chunk-major block order for L2 reuse measured slower: round 4.)
    const long target = 2048;
    int nyb = 1;
    while (nyb < nyb_max && (long)ng * nyb * nf * k.nbx < target) ++nyb;
    int nyc = (nyo + nyb - 1) / nyb;
    nyc = (nyc + k.s - 1) / k.s * k.s;
    nyb = (nyo + nyc - 1) / nyc;
    int cpg = ng >= 32 ? nyb : 1;
    int groups = ng * ((nyb + cpg - 1) / cpg);
    const int mb = cpg * nf * k.nbx;
    const unsigned blocks = (unsigned)(8 * ((groups + 7) / 8) * mb);
    void* args[] = {(void*)&G,   (void*)&P,   (void*)&ny,  (void*)&nx,  (void*)&fs,     (void*)&hw,  (void*)&tx,
                    (void*)&nyc, (void*)&nbx, (void*)&nyb, (void*)&cpg, (void*)&groups, (void*)&yb0, (void*)&yb1,
                    (void*)&zt};
    return hipLaunchKernel(k.fn, dim3(blocks), dim3(k.nthr ? k.nthr : k.cw), args, k.lds, s);
}

// K34 autotune at plan creation: every candidate geometry of k34_setup timed on the
// plan's own workspace (whole volume, contents irrelevant to the time), the fastest kept.
// Measured picks differ by config (c2: 2-wave blocks; c3: 4-wave blocks, 4-row tiles).
// Tuning input: a deterministic pseudo-random field of gradient-like magnitudes.  Timings on
// zeros run at a higher clock than on data (the fp64 VALU's DVFS give-back: c3 K34 1.41 ms
// on zeros vs 1.64 on data) and need not rank the candidates as data does.
template <typename F>
__global__ __launch_bounds__(256) void k_fill_tune(F* __restrict__ p, size_t n) {
    const size_t st = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += st) {
        unsigned h = (unsigned)i * 2654435761u;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        p[i] = (F)((int)(h & 0xffffu) - 32768) * (F)(1.0 / 256);
    }
}

template <typename F>
int k34_tune(of3d_plan* p) {
    if (p->k34_cand.size() <= 1) return 0;
    const int nf = p->ndim == 3 ? 9 : 5, ng = (int)std::min<int64_t>(p->nz, p->cap_planes);
    F* G = (F*)(p->ndim == 3 ? p->Y : p->X);
    F* P = (F*)(p->ndim == 3 ? p->X : p->Y);
    const F* hw = dev_taps<F>(p).w;
    struct Events {  // destroyed on every path out
        hipEvent_t e0 = nullptr, e1 = nullptr;
        ~Events() {
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
        }
    } ev;
    OF3D_HIP(hipEventCreate(&ev.e0));
    OF3D_HIP(hipEventCreate(&ev.e1));
    hipEvent_t e0 = ev.e0, e1 = ev.e1;
    // the heuristic pick (k34_setup) stays unless another shape is >= 2 % faster: stable
    // choices from run to run (candidates within noise of each other otherwise flip)
    size_t h0 = 0;
    for (size_t i = 0; i < p->k34_cand.size(); ++i)
        if (p->k34_cand[i].fn == p->k34.fn && p->k34_cand[i].cw == p->k34.cw && p->k34_cand[i].nthr == p->k34.nthr) h0 = i;
    std::swap(p->k34_cand[0], p->k34_cand[h0]);
    const size_t nc = p->k34_cand.size();
    // the gradient fields K34 reads (3D: 4, 2D: 3) as data-like values
    const size_t nfill = (size_t)(p->ndim == 3 ? 4 : 3) * p->fs;
    hipLaunchKernelGGL(k_fill_tune<F>, dim3(2048), dim3(256), 0, p->stream, G, nfill);
    OF3D_HIP(hipGetLastError());
    for (size_t i = 0; i < nc; ++i)  // warm every candidate (code load, caches)
        OF3D_HIP(launch_k34(p->k34_cand[i], (const F*)G, P, ng, nf, (int)p->ny, (int)p->nx, p->fs, hw, p->stream, p->wxy_zt));
    // best of three, the candidates interleaved round-robin (clock drift over the tune hits
    // every candidate alike); each sample two launches back to back, timed together (a single
    // launch after a synchronisation ran up to 5 % off the sustained time of a series: round 5,
    // c4: the duplicate-staging form 10.65 ms in the tune, 11.23 sustained)
    std::vector<float> ms(nc, 1e30f);
    for (int rep = 0; rep < 3; ++rep) {
        for (size_t i = 0; i < nc; ++i) {
            OF3D_HIP(launch_k34(p->k34_cand[i], (const F*)G, P, ng, nf, (int)p->ny, (int)p->nx, p->fs, hw, p->stream, p->wxy_zt));
            OF3D_HIP(hipEventRecord(e0, p->stream));
            for (int k = 0; k < 2; ++k)
                OF3D_HIP(launch_k34(p->k34_cand[i], (const F*)G, P, ng, nf, (int)p->ny, (int)p->nx, p->fs, hw, p->stream, p->wxy_zt));
            OF3D_HIP(hipEventRecord(e1, p->stream));
            OF3D_HIP(hipEventSynchronize(e1));
            float m = 0.f;
            OF3D_HIP(hipEventElapsedTime(&m, e0, e1));
            ms[i] = std::min(ms[i], 0.5f * m);
        }
    }
    // the fastest candidate, unless it is within 2 % of the heuristic pick (index 0)
    size_t bi = 0;
    for (size_t i = 1; i < nc; ++i)
        if (ms[i] < ms[bi]) bi = i;
    if (!(ms[bi] < 0.98f * ms[0])) bi = 0;
    const float best = ms[bi];
    p->k34 = p->k34_cand[bi];
    if (p->kn.verbose)
        fprintf(stderr, "of3d: K34 tuned over %zu shapes: cand=%zu cw=%d s=%d tx=%d nbx=%d thr=%d lds=%zu (%.3f ms)\n",
                p->k34_cand.size(), bi, p->k34.cw, p->k34.s, p->k34.tx, p->k34.nbx, p->k34.nthr, p->k34.lds, best);
    if (p->kn.verbose > 1)
        for (size_t i = 0; i < nc; ++i)
            fprintf(stderr, "of3d:   K34 cand %zu: cw=%d s=%d tx=%d thr=%d lds=%zu %.3f ms\n", i, p->k34_cand[i].cw,
                    p->k34_cand[i].s, p->k34_cand[i].tx, p->k34_cand[i].nthr, p->k34_cand[i].lds, ms[i]);
    return 0;
}

template <typename F>
int set_attrs_t(of3d_plan* p) {
    const size_t e = sizeof(F);
    p->k1_lds = (size_t)(2 * (K1_TY + 2 * p->rd) + 3 * K1_TY) * 64 * e;
    p->k2_lds = (size_t)(K2_ZC + 2 * std::max(p->rd, p->rs)) * 64 * e;
    p->k3_lds = (size_t)(K3_STEP + 2 * p->rw) * 64 * e;
    p->k4_lds = (size_t)K4_ROWS * (((K4_TX + 2 * k4_halo(p->rw)) | 1) + (K4_TX + 1)) * e;
    p->k5_lds = (size_t)2 * (k5_geom(p->rw).g * k5_geom(p->rw).r + 2 * p->rw) * 64 * e;
    const size_t lim = 160 * 1024;
    if (p->k3_lds > lim || p->k4_lds > lim || p->k5_lds > lim) return fail("of3d: wSig too large for the LDS tiles");
    auto attr = [&](const void* k, size_t b) -> int {
        OF3D_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b));
        return 0;
    };
    int rc = 0;
    for (int dt = OF3D_U8; dt <= OF3D_F64; ++dt) rc |= attr(k1_kernel_dt<F>(dt, p->rd), p->k1_lds);
    rc |= attr((const void*)k_grad_z<F>, p->k2_lds);
    rc |= attr(k3_kernel<F>(9, p->rw), p->k3_lds) | attr(k3_kernel<F>(5, p->rw), p->k3_lds);
    rc |= attr(k4_kernel<F>(9, p->rw), p->k4_lds) | attr(k4_kernel<F>(5, p->rw), p->k4_lds);
    rc |= attr(k5_kernel<F, float>(p->rw), p->k5_lds) | attr(k5_kernel<F, double>(p->rw), p->k5_lds);
    constexpr int epl = 16 / (int)sizeof(F);
    p->k5_nb = (p->nx % epl == 0) ? k5_dma_nb<F>(p->rw) : 0;
    if (p->k5_nb) {
        p->k5d_lds = (size_t)p->k5_nb * k5_groups<F>(p->rw) * 1024;
        rc |= attr(k5_dma_kernel<F, float>(p->rw, p->k5_nb), p->k5d_lds) |
              attr(k5_dma_kernel<F, double>(p->rw, p->k5_nb), p->k5d_lds);
    }
    if (rc) return -1;
    for (int dt : {OF3D_U8, OF3D_U16, OF3D_F32}) {
        if (const void* f = k1c_fn<F>(dt, p->rd, p->rs))
            OF3D_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        for (bool deep : {false, true})
            if (const void* f = k12_fn<F>(dt, p->rd, p->rs, deep))
                OF3D_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)k12_lds<F>(dt, p->rd, deep)));
    }
    if (k5c_setup<F>(p)) return -1;
    return k34_setup<F>(p, p->ndim == 3 ? 9 : 5);
}

// Radii the tiled kernels cannot stage (the legacy K1's 64-wide strips need rd <= 24, every
// tile at most 160 KiB of LDS, kMaxR for the tap padding) run the general-radius path
// (k_corr_gen passes: the same arithmetic, any radius).  OF3D_GENERAL=1 forces it (tests).
bool needs_general(const of3d_plan* p) {
    if (p->kn.general) return true;
    if (p->rd > 24 || p->rs > kMaxR || p->rw > kMaxR) return true;
    const size_t e = p->fp32 ? 4 : 8, lim = 160 * 1024;
    const size_t k3 = (size_t)(K3_STEP + 2 * p->rw) * 64 * e;
    const size_t k4 = (size_t)K4_ROWS * (((K4_TX + 2 * k4_halo(p->rw)) | 1) + (K4_TX + 1)) * e;
    const size_t k5 = (size_t)2 * (k5_geom(p->rw).g * k5_geom(p->rw).r + 2 * p->rw) * 64 * e;
    const size_t k2 = (size_t)(K2_ZC + 2 * std::max(p->rd, p->rs)) * 64 * e;
    return k3 > lim || k4 > lim || k5 > lim || k2 > lim;
}

int set_attrs(of3d_plan* p) {
    p->general = needs_general(p);
    if (p->general) return 0;
    return p->fp32 ? set_attrs_t<float>(p) : set_attrs_t<double>(p);
}

struct Ranges {
    int64_t zo0, zo1, zg0, zg1, zb0, zb1;
};

Ranges ranges(const of3d_plan* p, int64_t zo0, int64_t zo1) {
    Ranges r;
    r.zo0 = zo0;
    r.zo1 = zo1;
    if (p->ndim == 2) {  // planes = independent frames of a batch: no halo
        r.zg0 = r.zb0 = zo0;
        r.zg1 = r.zb1 = zo1;
        return r;
    }
    r.zg0 = std::max<int64_t>(zo0 - p->rw, 0);
    r.zg1 = std::min<int64_t>(zo1 + p->rw, p->nz);
    r.zb0 = std::max<int64_t>(r.zg0 - p->rd, 0);
    r.zb1 = std::min<int64_t>(r.zg1 + p->rd, p->nz);
    return r;
}

// General-radius pipeline (any radius; see needs_general).  3D workspace use: Y0 dt0, Y1 the
// centre frame in F, X0..2 the y passes, Y2..5 the x passes (pre-z), X0..3 the gradients,
// Y0..8 the products, X0..8 W-y, Y0..8 W-x, X0..8 W-z; 2D the same without z.  Plane ranges
// and clamping as the tiled pipeline: inputs [zb0, zb1), gradients / products [zg0, zg1)
// (z pass clamped at zb1), outputs [zo0, zo1) (W z clamped at zg1).  Stage events: grad_xy
// = dt0 + y / x passes, grad_z = gradient z pass, prod_wy = products + W y + W x, wz_solve.
template <typename F, typename Mark>
int run_general(of3d_plan* p, const Frames& fr, int dtype, int64_t frame_z0, const Ranges& R, F* vx, F* vy, F* vz,
                void* rel, hipStream_t st, Mark& mark) {
    const bool d3 = p->ndim == 3;
    const int ny = (int)p->ny, nx = (int)p->nx;
    const size_t plane = (size_t)ny * nx, fs = p->fs, es = dtype_size(dtype);
    F* X = (F*)p->X;
    F* Y = (F*)p->Y;
    const DevTaps<F> tp = dev_taps<F>(p);
    auto grid = [&](size_t n) { return dim3((unsigned)std::min<size_t>((n + 255) / 256, 256 * 64)); };
    const int zb0 = (int)R.zb0, zb1 = (int)R.zb1, zg0 = (int)R.zg0, zg1 = (int)R.zg1, zo0 = (int)R.zo0,
              zo1 = (int)R.zo1;
    auto pass = [&](const F* in, int in_z0, F* out, int out_z0, int q0, int q1, int axis, const F* h, int r, int anti,
                    int zhi) -> int {
        if (q1 <= q0) return 0;
        hipLaunchKernelGGL(k_corr_gen<F>, grid((size_t)(q1 - q0) * plane), dim3(256), 0, st, in, in_z0, out, out_z0, q0,
                           q1, ny, nx, axis, h, r, anti, zhi);
        OF3D_HIP(hipGetLastError());
        return 0;
    };
    if (mark(0)) return -1;
    // dt0 (the streaming K0 for any rt) and the centre frame as F, planes [zb0, zb1)
    {
        size_t off0 = (size_t)(zb0 - frame_z0) * plane, n = (size_t)(zb1 - zb0) * plane;
        long long fstride = 0;
        int rt_arg = p->rt;
        F* D0 = Y;
        const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 256 * 16);
        void* args[] = {(void*)&fr, (void*)&fstride, (void*)&off0, (void*)&n, (void*)&rt_arg, (void*)&tp.t, (void*)&D0};
        OF3D_HIP(hipLaunchKernel(k0_kernel_dt<F>(dtype), dim3(blocks), dim3(256), args, 0, st));
        const void* Ic = (const char*)fr.p[p->rt] + off0 * es;
        F* If = Y + fs;
        switch (dtype) {
#define OF3D_CAST(C, T)                                                                                         \
    case C:                                                                                                     \
        hipLaunchKernelGGL((k_cast_gen<T, F>), grid(n), dim3(256), 0, st, (const T*)Ic, If, n);                   \
        break;
            OF3D_CAST(OF3D_U8, uint8_t)
            OF3D_CAST(OF3D_U16, uint16_t)
            OF3D_CAST(OF3D_I16, int16_t)
            OF3D_CAST(OF3D_U32, uint32_t)
            OF3D_CAST(OF3D_I32, int32_t)
            OF3D_CAST(OF3D_F32, float)
            OF3D_CAST(OF3D_F64, double)
#undef OF3D_CAST
            default: return fail("of3d: unsupported dtype");
        }
        OF3D_HIP(hipGetLastError());
    }
    const int pz0 = zb0, pz1 = zb1;  // planes of the y / x passes (3D: the input range; 2D: plane 0)
    // y passes: A1 = y(G)[dt0], A2 = y(D)[I], A3 = y(S)[I]
    if (pass(Y, pz0, X, pz0, pz0, pz1, 1, tp.g, p->rd, 0, 1) || pass(Y + fs, pz0, X + fs, pz0, pz0, pz1, 1, tp.d, p->rd, 1, 1) ||
        pass(Y + fs, pz0, X + 2 * fs, pz0, pz0, pz1, 1, tp.s, p->rs, 0, 1))
        return -1;
    // x passes: B1 = x(G)[A1] (dt), B2 = x(S)[A2] (dy), B3 = x(D)[A3] (dx), B4 = x(S)[A3] (pre-z dz)
    if (pass(X, pz0, Y + 2 * fs, pz0, pz0, pz1, 0, tp.g, p->rd, 0, 1) ||
        pass(X + fs, pz0, Y + 3 * fs, pz0, pz0, pz1, 0, tp.s, p->rs, 0, 1) ||
        pass(X + 2 * fs, pz0, Y + 4 * fs, pz0, pz0, pz1, 0, tp.d, p->rd, 1, 1) ||
        (d3 && pass(X + 2 * fs, pz0, Y + 5 * fs, pz0, pz0, pz1, 0, tp.s, p->rs, 0, 1)))
        return -1;
    if (mark(1)) return -1;
    const F* Gr;
    int gz0, gz1;
    if (d3) {  // z passes into X0..3 over [zg0, zg1): dt G, dy S, dx S, dz D
        if (pass(Y + 2 * fs, zb0, X, zg0, zg0, zg1, 2, tp.g, p->rd, 0, zb1) ||
            pass(Y + 3 * fs, zb0, X + fs, zg0, zg0, zg1, 2, tp.s, p->rs, 0, zb1) ||
            pass(Y + 4 * fs, zb0, X + 2 * fs, zg0, zg0, zg1, 2, tp.s, p->rs, 0, zb1) ||
            pass(Y + 5 * fs, zb0, X + 3 * fs, zg0, zg0, zg1, 2, tp.d, p->rd, 1, zb1))
            return -1;
        Gr = X;
        gz0 = zg0, gz1 = zg1;
    } else {
        Gr = Y + 2 * fs;  // dt, dy, dx (2D: the batch's planes, origin zb0 = zg0)
        gz0 = zg0, gz1 = zg1;
    }
    if (mark(2)) return -1;
    const int np = d3 ? 9 : 5;
    F* Pp = d3 ? Y : X;  // products
    F* Wy = d3 ? X : Y;
    {
        const size_t n = (size_t)(gz1 - gz0) * plane;
        hipLaunchKernelGGL(k_prod_gen<F>, grid(n), dim3(256), 0, st, Gr, Pp, fs, n, np);
        OF3D_HIP(hipGetLastError());
    }
    for (int f = 0; f < np; ++f)
        if (pass(Pp + f * fs, gz0, Wy + f * fs, gz0, gz0, gz1, 1, tp.w, p->rw, 0, 1) ||
            pass(Wy + f * fs, gz0, Pp + f * fs, gz0, gz0, gz1, 0, tp.w, p->rw, 0, 1))
            return -1;
    if (mark(3) || mark(4)) return -1;  // W-xy in Pp ("wx" stays folded into "prod_wy")
    if (d3) {
        for (int f = 0; f < 9; ++f)
            if (pass(Pp + f * fs, zg0, X + f * fs, zo0, zo0, zo1, 2, tp.w, p->rw, 0, zg1)) return -1;
        const size_t n = (size_t)(zo1 - zo0) * plane;
        if (p->rel64)
            hipLaunchKernelGGL((k_solve3_gen<F, double>), grid(n), dim3(256), 0, st, (const F*)X, fs, n, vx, vy, vz,
                               (double*)rel);
        else
            hipLaunchKernelGGL((k_solve3_gen<F, float>), grid(n), dim3(256), 0, st, (const F*)X, fs, n, vx, vy, vz,
                               (float*)rel);
    } else {
        const size_t n = (size_t)(zo1 - zo0) * plane;
        hipLaunchKernelGGL(k_solve2d<F>, dim3((unsigned)std::min<size_t>((n + 255) / 256, 256 * 64)), dim3(256), 0, st,
                           (const F*)Pp, fs, n, vx, vy, (F*)rel);
    }
    OF3D_HIP(hipGetLastError());
    return mark(5);
}

// The stage pipeline over output planes [zo0, zo1).  Stage launches take plane sub-ranges:
//   K0 + K1 : pre-z fields B on planes [b0, b1)      (input frames, D0 temporary)
//   K2      : gradients G on planes [q0, q1)         (reads B on [q0 - rd, q1 + rd))
//   K34     : W-xy of the products, Q on [q0, q1)     (per plane)
//   K5      : outputs on [o0, o1)                     (reads Q on [o0 - rw, o1 + rw))
// Workspace (3D): Y0 = D0, Y4..7 = B, Y0..3 = G, X0..8 = Q; plane origins zb0 (D0, B) and
// zg0 (G, Q).  Serial mode: one chunk on the caller's stream.  Overlap mode (fused K34,
// p->zchunk > 0): the output range in chunks of zchunk planes, K0-K2 of every chunk on the
// caller's stream and K34 + K5 on the plan's second stream, each chunk's K34 behind an
// event after its K2 — the HBM-bound K0-K2 of chunk c+1 run beside the VALU-bound K34/K5
// of chunk c.  Every plane range is disjoint from the ones the other stream touches at the
// same time (B/G/D0 planes of later chunks lie above the G/Q planes of earlier ones), and
// the results are those of the serial order (same kernels, same planes, global clamping).
template <typename F>
int run_t(of3d_plan* p, const void* const* d_frames, int dtype, int64_t frame_z0, int64_t zo0, int64_t zo1, void* vx_,
          void* vy_, void* vz_, void* rel, hipStream_t s, const void* const* d_next, bool pipe, int ahead) {
    if (!p) return fail("of3d: null plan");
    F* vx = (F*)vx_;
    F* vy = (F*)vy_;
    F* vz = (F*)vz_;
    F* X = (F*)p->X;
    F* Y = (F*)p->Y;
    if (zo0 < 0 || zo1 > p->nz || zo0 >= zo1) return fail("of3d: bad output plane range");
    const Ranges R = ranges(p, zo0, zo1);
    if (R.zb1 - R.zb0 > p->cap_planes) return fail("of3d: output range exceeds the plan's workspace");
    if (frame_z0 > R.zb0) return fail("of3d: frames do not hold the stencil halo planes");
    if (dtype_size(dtype) == 0) return fail("of3d: unsupported dtype");
    const int ny = (int)p->ny, nx = (int)p->nx;
    const bool d3 = p->ndim == 3;
    Frames fr{};
    for (int i = 0; i < 2 * p->rt + 1; ++i) {
        if (!d_frames[i]) return fail("of3d: null frame pointer");
        fr.p[i] = d_frames[i];
    }
    const DevTaps<F> tp = dev_taps<F>(p);
    const size_t fs = p->fs;
    const size_t plane = (size_t)ny * nx;
    const size_t es = dtype_size(dtype);
    const int nwin = 2 * p->rt + 1;
    const int nf = d3 ? 9 : 5;
    // frame pipelining: this call's dt0 was formed by the previous of3d_plan_execute_next call
    // (inside its K5c) for exactly these frames and planes -> no K0 launch here
    bool skip_k0 = pipe && p->pipe_valid && p->pipe_dtype == dtype && p->pipe_fz0 == frame_z0 &&
                   p->pipe_zo0 == zo0 && p->pipe_zo1 == zo1;
    for (int i = 0; skip_k0 && i < nwin; ++i) skip_k0 = p->pipe_frames[i] == d_frames[i];
    p->pipe_valid = false;
    // ... and this call's K5c forms the next frame's dt0 (serial schedule, uint16 frames, the
    // vectorised K0 layout: every frame 8-byte aligned at plane zb0, whole groups of 4 voxels)
    K0Next<F> k0n{};
    bool fuse_next = false;
    // (the fused W kernel keeps W-xy in X; with the K3 + K4 fallback K5c reads Y, where dt0 goes)
    if (d_next && pipe && p->k5c_next && p->k34.fn && dtype == OF3D_U16 && !p->general && p->zchunk <= 0) {
        const size_t off0 = (size_t)(R.zb0 - frame_z0) * plane, n = (size_t)(R.zb1 - R.zb0) * plane;
        constexpr int V = K0Vec<uint16_t>::V;
        fuse_next = off0 % V == 0 && n % V == 0;
        for (int i = 0; fuse_next && i < nwin; ++i)
            fuse_next = d_next[i] && ((uintptr_t)d_next[i] % (V * sizeof(uint16_t))) == 0;
        if (fuse_next) {
            for (int i = 0; i < nwin; ++i) k0n.fr.p[i] = d_next[i];
            k0n.off0 = off0;
            k0n.ngroups = n / V;
            k0n.ht = tp.t;
        }
    }
    // K12 (fused gradient y/x/z passes, 3D): dt0 then lives in Y4 (K12 writes G = Y0..3
    // while other blocks still read dt0 planes), the pre-z fields B are never formed
    // (LDS-DMA staging: 16-byte rows and planes of dt0 and of the centre frame)
    const bool k12_al = (nx * sizeof(F)) % 16 == 0 && (nx * es) % 16 == 0 &&
                        ((uintptr_t)d_frames[p->rt] + (size_t)(R.zb0 - frame_z0) * plane * es) % 16 == 0;
    // K12 pays where its blocks can march >= 32 planes and still fill the GPU: fp64 (one 12-wave
    // block per CU), one round of 32-plane marches on every CU — c2 (256^2 x 64: 256 blocks) K0
    // + K12 0.110 ms vs K0 + K1c + K2c 0.142, frame 0.377 vs 0.420 (round 5; with 16-plane
    // marches 0.126: K1c + K2c had measured faster); fp32, 1024 blocks; c3: K12 0.62 vs 0.83 ms.
    // OF3D_K12=1 forces it, OF3D_K12=0 disables it
    const int k12_tiles = (int)cdiv(nx, k12_cw<F>() - 2 * p->rd) * (int)cdiv(ny, K12_TY);
    const bool k12_big = (long)k12_tiles * cdiv(R.zg1 - R.zg0, 32) >= (sizeof(F) == 8 ? p->ncu : 1024);
    // (fp32 plans, rd <= 6: two blocks per CU — c3 0.27 + 0.36 ms vs K1c + K2c 0.43 + 0.25, c5
    // 12.7 + 21.3 vs 23.5 + 13.2; rd 9 in fp32 runs one block per CU: K1c + K2c)
    const void* k12 = (d3 && p->kn.k12 != 0 && k12_al && plane * sizeof(F) <= 0x7fffffffu &&
                       ((k12_big && (sizeof(F) == 8 || p->rd <= 6)) || p->kn.k12 == 1))
                          ? k12_fn<F>(dtype, p->rd, p->rs) : nullptr;
    // K0 batching (of3d_plan_execute_ahead, `ahead` >= 0 frames past the window in d_frames):
    // this call's dt0 from a slot an earlier call formed for exactly this window, else one
    // k_tderiv_multi pass forms it and the next min(ahead, kDtSlots - 1) windows' (K12 flow,
    // serial schedule, the vectorised K0 layout).  Same bits as K0 (k0_group_dt's order).
    int dslot = 0, k0m = 0;  // slot holding this call's dt0; windows of a batched K0 launch
    const void* k0m_k = nullptr;
    Frames frm{};
    // (the fused W kernel writes W-xy to X; the K3 + K4 fallback writes it to Y over the slots)
    if (ahead >= 0 && d3 && k12 && p->k34.fn && p->zchunk <= 0 && !p->general) {
        for (int sl = 0; sl < of3d_plan::kDtSlots && !skip_k0; ++sl) {
            auto& d = p->dts[sl];
            bool hit = d.valid && d.dtype == dtype && d.fz0 == frame_z0 && d.zo0 == zo0 && d.zo1 == zo1;
            for (int i = 0; hit && i < nwin; ++i) hit = d.frames[i] == d_frames[i];
            if (hit) skip_k0 = true, dslot = sl, d.valid = false;  // consumed
        }
        const int m = std::min(ahead, of3d_plan::kDtSlots - 1) + 1;
        if (!skip_k0)
            for (auto& d : p->dts) d.valid = false;
        if (!skip_k0 && m >= 2) {
            const int V = k0_vec_width(dtype);
            const size_t off0 = (size_t)(R.zb0 - frame_z0) * plane, n = (size_t)(R.zb1 - R.zb0) * plane;
            bool vec = off0 % V == 0 && n % V == 0;
            for (int i = 0; vec && i < nwin + m - 1; ++i) {
                vec = d_frames[i] && ((uintptr_t)d_frames[i] % ((size_t)V * es)) == 0;
                frm.p[i] = d_frames[i];
            }
            k0m_k = vec ? k0m_fn<F>(dtype, p->rt, m) : nullptr;
            if (k0m_k) k0m = m;
        }
    } else {
        for (auto& d : p->dts) d.valid = false;
    }
    // field buffers
    // a pipelined dt0 lives where the producing call's flow put it (Y4 with K12, else Y0): whether
    // a call runs K12 is decided per call (alignment, OF3D_K12), so the flows must agree
    if (skip_k0 && pipe && p->pipe_k12 != (k12 != nullptr)) skip_k0 = false;
    F* D0b = k12 ? Y + (4 + dslot) * fs : Y;  // temporal derivative (K0 -> K1 / K12), origin zb0
    k0n.D0 = D0b;
    F* Bb = d3 ? Y + 4 * fs : X;       // pre-z fields (3D) / final gradients (2D), origin zb0
    const F* Gb = d3 ? Y : X;          // gradients, origin zg0
    F* Pb = d3 ? X : Y;                // K3 W-y (fallback) / K34 W-xy
    F* Qb = p->k34.fn ? Pb : (d3 ? Y : X);  // W-xy (K4 fallback writes the other buffer)

    // ---- stage launches over plane sub-ranges ----
    auto k01 = [&](int64_t b0, int64_t b1, hipStream_t st) -> int {
        if (b1 <= b0) return 0;
        const int nb = (int)(b1 - b0);
        if (k0m) {  // batched K0: this window's dt0 (slot 0) and the next k0m - 1 windows'
            size_t off0 = (size_t)(b0 - frame_z0) * plane, ng = (size_t)nb * plane / k0_vec_width(dtype);
            F* D0 = Y + 4 * fs + (size_t)(b0 - R.zb0) * plane;
            size_t dstride = fs;
            const unsigned blocks = (unsigned)std::min<size_t>((ng + 255) / 256, 256 * 32);
            void* margs[] = {(void*)&frm, (void*)&off0, (void*)&ng, (void*)&tp.t, (void*)&D0, (void*)&dstride};
            OF3D_HIP(hipLaunchKernel(k0m_k, dim3(blocks), dim3(256), margs, 0, st));
            p->used |= KU_K0M;
            p->last_k0m = k0m;
        } else if (!skip_k0) {  // (else: dt0 formed by an earlier call: K5c's next / a batched K0)
            long long fstride = 0;
            if (nwin > 1) {
                const long long d = (const char*)d_frames[1] - (const char*)d_frames[0];
                bool eq = d > 0 && d % (long long)es == 0;
                for (int i = 2; eq && i < nwin; ++i) eq = ((const char*)d_frames[i] - (const char*)d_frames[i - 1]) == d;
                if (eq) fstride = d / (long long)es;
            }
            size_t off0 = (size_t)(b0 - frame_z0) * plane, n = (size_t)nb * plane;
            int rt_arg = p->rt;
            F* D0 = D0b + (size_t)(b0 - R.zb0) * plane;
            const int V = k0_vec_width(dtype);
            const size_t vb = (size_t)V * es;
            bool vec = off0 % V == 0 && n % V == 0;
            for (int i = 0; vec && i < nwin; ++i) vec = ((uintptr_t)d_frames[i] % vb) == 0;
            if (vec) {
                size_t ng = n / V;
                const unsigned blocks = (unsigned)std::min<size_t>((ng + 255) / 256, 256 * 32);
                void* args[] = {(void*)&fr, (void*)&off0, (void*)&ng, (void*)&rt_arg, (void*)&tp.t, (void*)&D0};
                const void* k0 = p->kn.k0c ? k0c_fn<F>(dtype, p->rt) : nullptr;
                if (k0) {
                    void* cargs[] = {(void*)&fr, (void*)&off0, (void*)&ng, (void*)&tp.t, (void*)&D0};
                    OF3D_HIP(hipLaunchKernel(k0, dim3(blocks), dim3(256), cargs, 0, st));
                    p->used |= KU_K0C;
                } else {
                    OF3D_HIP(hipLaunchKernel(k0v_kernel_dt<F>(dtype), dim3(blocks), dim3(256), args, 0, st));
                    p->used |= KU_K0;
                }
            } else {
                const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 256 * 16);
                void* args[] = {(void*)&fr, (void*)&fstride, (void*)&off0, (void*)&n, (void*)&rt_arg, (void*)&tp.t,
                                (void*)&D0};
                OF3D_HIP(hipLaunchKernel(k0_kernel_dt<F>(dtype), dim3(blocks), dim3(256), args, 0, st));
                p->used |= KU_K0;
            }
        }
        if (k12) return 0;  // the y / x passes run inside K12 (stage grad_z)
        const size_t off1 = (size_t)(b0 - frame_z0) * plane;
        const void* Ic = (const char*)d_frames[p->rt] + off1 * es;
        const F* D0c = D0b + (size_t)(b0 - R.zb0) * plane;
        F* Bo = Bb + (size_t)(b0 - R.zb0) * plane;
        int need_b4 = d3, nb_arg = nb;
        dim3 g(cdiv(nx, 64 - 2 * p->rd), cdiv(ny, K1_TY), cdiv(nb, K1_NZB));
        void* args[] = {(void*)&Ic, (void*)&D0c, (void*)&ny, (void*)&nx, (void*)&nb_arg, (void*)&tp,
                        (void*)&Bo, (void*)&fs, (void*)&need_b4};
        // (32-bit buffer offsets within a plane: planes up to 2 GiB)
        const bool k1c_ok = p->kn.k1c && plane * sizeof(F) <= 0x7fffffffu;
        const void* k1c = k1c_ok ? k1c_fn<F>(dtype, p->rd, p->rs) : nullptr;
        if (k1c) {
            // column march: 128-column blocks up to nx 256, else 256; rows in chunks of >= 32
            const int cw = nx <= 256 ? 128 : 256;  // c2: 128 (86 vs 98 us), c3: 256 (0.65 vs 0.69 ms)
            int tx = (cw - 2 * p->rd) & ~3, nbx = (nx + tx - 1) / tx;
            int nyc = std::min(ny, 32), nyb;
            while (true) {
                nyc = (nyc + K1C_S - 1) / K1C_S * K1C_S;
                nyb = (ny + nyc - 1) / nyc;
                if ((long)nb * nyb * nbx <= 8192 || nyc >= ny) break;
                nyc *= 2;
            }
            const size_t lds = (size_t)6 * k34_tile(K1C_S, cw + 1) * sizeof(F);
            const unsigned blocks = (unsigned)((long)nb * nyb * nbx);
            void* cargs[] = {(void*)&Ic, (void*)&D0c, (void*)&ny, (void*)&nx, (void*)&tp, (void*)&Bo,
                             (void*)&fs, (void*)&need_b4, (void*)&tx, (void*)&nyc, (void*)&nbx, (void*)&nyb};
            OF3D_HIP(hipLaunchKernel(k1c, dim3(blocks), dim3(cw), cargs, lds, st));
            p->used |= KU_K1C;
        } else {
            OF3D_HIP(hipLaunchKernel(k1_kernel_dt<F>(dtype, p->rd), g, dim3(64, 4), args, p->k1_lds, st));
            p->used |= KU_K1;
        }
        return 0;
    };
    auto k2 = [&](int64_t q0, int64_t q1, hipStream_t st) -> int {
        if (q1 <= q0 || !d3) return 0;
        const int ng = (int)(q1 - q0);
        if (k12) {
            // K12 over output planes [q0, q1): the centre frame and dt0 from plane zb0 on
            const void* Ic = (const char*)d_frames[p->rt] + (size_t)(R.zb0 - frame_z0) * plane * es;
            const F* D0c = D0b;
            F* Go = Y;
            const int tx = k12_cw<F>() - 2 * p->rd;
            int nbx = (int)cdiv(nx, tx), ntile = nbx * (int)cdiv(ny, K12_TY);
            int zin0 = (int)R.zb0, nzc = (int)R.zb1, zg0 = (int)R.zg0, qa = (int)q0, nq = ng;
            // planes per block: the longest march (up to 256) that still gives >= 1024 blocks
            // (each march re-forms 2 rd halo planes), at least 16.  Measured: c5 fp32 K12 20.7 /
            // 20.0 / 19.7 ms at 64 / 128 / 256, c4 fp64 4.40 / 4.12 at 64 / 128; c3 keeps 64
            int zc = p->kn.k12_zc;  // OF3D_K12_ZC: forced march length (tests)
            if (zc <= 0 && k12_nwx<F>() == 3) {
                // fp64 (one 12-wave block per CU): the march with the fewest block-steps on the
                // busiest CU, rounds of blocks x (march + 2 rd halo steps); ties to the longer
                // march.  c2: 32 planes (one round of 256 blocks: K12 0.090 ms vs 0.107 at 16 and
                // 0.107 at 64), c3: 64 (three rounds), c4: 256
                long best = 0;
                for (int z = 256; z >= 16; z /= 2) {
                    const long rounds = cdiv((long)ntile * cdiv(nq, z), std::max(p->ncu, 1));
                    const long cost = rounds * (std::min(z, nq) + 2 * p->rd);
                    if (!best || cost < best) best = cost, zc = z;
                }
            } else if (zc <= 0) {
                zc = 256;  // fp32 (two blocks per CU): the longest march with >= 1024 blocks
                while (zc > 16 && (long)ntile * cdiv(nq, zc) < 1024) zc /= 2;
            }
            const unsigned gx = 8 * cdiv(ntile, 8);
            // marches of >= 128 planes: the three-DMA-slot instance (fp64 rd 6; the others have one)
            const bool deep = zc >= 128;
            const void* k12x = deep ? k12_fn<F>(dtype, p->rd, p->rs, true) : k12;
            const size_t lds = k12_lds<F>(dtype, p->rd, deep);
            void* args[] = {(void*)&Ic, (void*)&D0c, (void*)&zin0, (void*)&nzc, (void*)&ny, (void*)&nx, (void*)&tp,
                            (void*)&Go, (void*)&fs, (void*)&zg0, (void*)&qa, (void*)&nq, (void*)&zc, (void*)&ntile,
                            (void*)&nbx};
            OF3D_HIP(hipLaunchKernel(k12x, dim3(gx, cdiv(nq, zc)), dim3(k12_threads<F>()), args, lds, st));
            p->used |= KU_K12;
            p->last_k12_zc = zc, p->last_k12_gx = (int)gx, p->last_k12_gy = (int)cdiv(nq, zc);
            p->last_k12_deep = k12x != k12;
            return 0;
        }
        const void* k2c = nullptr;
        if (p->kn.k2c) {
            if (p->rd == 6 && p->rs == 2) k2c = (const void*)k_grad_z_c<F, 6, 2>;
            if (p->rd == 3 && p->rs == 1) k2c = (const void*)k_grad_z_c<F, 3, 1>;
        }
        const F* Bc = Bb;
        F* Go = Y + (size_t)(q0 - R.zg0) * plane;
        // input planes clamp at zb1 (= nz at the top edge): see the K5 launch
        int zb0 = (int)R.zb0, zg0 = (int)q0, ngz = ng, nzz = (int)R.zb1;
        if (k2c) {
            // z march: 256 columns per block, chunks of >= 32 planes (2 rd halo planes re-read per chunk)
            const int pl = (int)plane;
            int zc = std::min(ng, 32);
            while ((long)cdiv(pl, 256) * cdiv(ng, zc) > 8192 && zc < ng) zc *= 2;
            void* args[] = {(void*)&Bc, (void*)&zb0, (void*)&Go, (void*)&zg0, (void*)&ngz, (void*)&nzz, (void*)&pl,
                            (void*)&fs, (void*)&tp, (void*)&zc};
            OF3D_HIP(hipLaunchKernel(k2c, dim3(cdiv(pl, 256), cdiv(ng, zc)), dim3(256), args, 0, st));
            p->used |= KU_K2C;
        } else {
            dim3 g(cdiv(nx, 64), ny, cdiv(ng, K2_ZC) * 4);
            hipLaunchKernelGGL(k_grad_z<F>, g, dim3(64, 4), p->k2_lds, st, Bc, zb0, Go, zg0, ngz, nzz, ny, nx, fs, tp);
            OF3D_HIP(hipGetLastError());
            p->used |= KU_K2;
        }
        return 0;
    };
    auto k34 = [&](int64_t q0, int64_t q1, hipStream_t st) -> int {
        if (q1 <= q0) return 0;
        const int ng = (int)(q1 - q0);
        const size_t o = (size_t)(q0 - R.zg0) * plane;
        // (z-tiled W-xy: plane q0 starts 32 elements per plane in, csrc/of3d_dev.hpp wxy_rsrc)
        const size_t op = p->wxy_zt ? (size_t)(q0 - R.zg0) * 32 : o;
        OF3D_HIP(launch_k34(p->k34, Gb + o, Pb + op, ng, nf, ny, nx, fs, tp.w, st, p->wxy_zt, (int)p->ya, (int)p->yb));
        p->used |= p->k34.nthr ? (p->k34.nthr == p->k34.cw ? KU_K34PK : KU_K34WS) : KU_K34;
        return 0;
    };
    auto k3k4 = [&](hipStream_t st) -> int {  // fallback: W y and W x as two kernels (whole range)
        const int ng = (int)(R.zg1 - R.zg0);
        F* P = Pb;
        const F* G = Gb;
        {
            dim3 g(cdiv(nx, 64), 1, ng * nf);
            int rw_arg = p->rw;
            void* args[] = {(void*)&G, (void*)&P, (void*)&ny, (void*)&nx, (void*)&fs, (void*)&tp.w, (void*)&tp.wr,
                            (void*)&rw_arg};
            OF3D_HIP(hipLaunchKernel(k3_kernel<F>(nf, p->rw), g, dim3(64, 4), args, p->k3_lds, st));
            p->used |= KU_K3;
        }
        return 0;
    };
    auto k4 = [&](hipStream_t st) -> int {
        const int ng = (int)(R.zg1 - R.zg0);
        dim3 g(1, cdiv(ny, K4_ROWS), ng * nf);
        int rw_arg = p->rw;
        const F* Pc = Pb;
        F* Q = Qb;
        void* args[] = {(void*)&Pc, (void*)&Q, (void*)&ny, (void*)&nx, (void*)&fs, (void*)&tp.w, (void*)&tp.wr,
                        (void*)&rw_arg};
        OF3D_HIP(hipLaunchKernel(k4_kernel<F>(nf, p->rw), g, dim3(64, 4), args, p->k4_lds, st));
        p->used |= KU_K4;
        return 0;
    };
    auto k5 = [&](int64_t o0, int64_t o1, int64_t q1, hipStream_t st) -> int {
        if (o1 <= o0) return 0;
        const size_t oo = (size_t)(o0 - R.zo0) * (size_t)(p->yb - p->ya) * nx;  // output planes: own rows
        F* ovx = vx + oo;
        F* ovy = vy + oo;
        F* ovz = d3 ? vz + oo : nullptr;
        void* orel = (char*)rel + oo * (p->rel64 ? sizeof(double) : sizeof(float));  // 3D rel (2D: oo = 0)
        if (d3) {
            const K5Geom kg = k5_geom(p->rw);
            const int no = (int)(o1 - o0);
            dim3 g(cdiv(nx, 64), ny, cdiv(no, kg.g * kg.r));
            int zg0 = (int)R.zg0, zoa = (int)o0, rw_arg = p->rw, noa = no;
            // window planes clamp at q1 (= nz at the volume's top edge): the rows a block loads
            // past its last output plane stay inside the W-xy planes computed so far
            int zq1 = (int)q1;
            const F* Qc = Qb;
            void* args[] = {(void*)&Qc, (void*)&zg0, (void*)&zq1, (void*)&ny, (void*)&nx, (void*)&fs, (void*)&tp.w,
                            (void*)&tp.wr, (void*)&rw_arg, (void*)&zoa, (void*)&noa, (void*)&ovx, (void*)&ovy,
                            (void*)&ovz, (void*)&orel};
            if (p->k5c) {
                dim3 gc(cdiv(nx, 32), (unsigned)(p->yb - p->ya), cdiv(no, k5c_zc(p->k5c_r, p->k5c_nw)));
                int yo0 = (int)p->ya;
                void* cargs[] = {(void*)&Qc, (void*)&zg0, (void*)&zq1, (void*)&ny,  (void*)&nx,  (void*)&fs,
                                 (void*)&tp.w, (void*)&zoa, (void*)&noa, (void*)&ovx, (void*)&ovy, (void*)&ovz,
                                 (void*)&orel, (void*)&yo0, (void*)&k0n, (void*)&p->wxy_zt};
                OF3D_HIP(hipLaunchKernel(fuse_next ? p->k5c_next : p->k5c, gc, dim3(64 * p->k5c_nw), cargs, p->k5c_lds, st));
                p->used |= fuse_next ? KU_K5C_NEXT : KU_K5C;
            } else if (p->k5_nb) {
                const void* k = p->rel64 ? k5_dma_kernel<F, double>(p->rw, p->k5_nb) : k5_dma_kernel<F, float>(p->rw, p->k5_nb);
                OF3D_HIP(hipLaunchKernel(k, g, dim3(64, kg.g), args, p->k5d_lds, st));
                p->used |= KU_K5DMA;
            } else {
                const void* k = p->rel64 ? k5_kernel<F, double>(p->rw) : k5_kernel<F, float>(p->rw);
                OF3D_HIP(hipLaunchKernel(k, g, dim3(64, kg.g), args, p->k5_lds, st));
                p->used |= KU_K5;
            }
        } else {
            // (2D: planes [o0, o1) of a batch of independent frames)
            const size_t n = (size_t)(o1 - o0) * plane;  // (64-bit: a batch may exceed 2^31 pixels)
            hipLaunchKernelGGL(k_solve2d<F>, dim3((unsigned)std::min<size_t>((n + 255) / 256, 256 * 64)), dim3(256), 0,
                               st, (const F*)Qb + (size_t)(o0 - R.zg0) * plane, fs, n, ovx, ovy, (F*)orel);
            p->used |= KU_SOLVE2D;
        }
        OF3D_HIP(hipGetLastError());
        return 0;
    };

    // ---- schedule ----
    const int slot = p->timing_slots ? (int)(p->tcount % p->timing_slots) : 0;
    hipEvent_t* evs = p->host_ev ? p->ev : (p->timing_slots ? &p->tev[(size_t)slot * p->tev_per_slot] : nullptr);
    const unsigned tmask = p->host_ev ? (1u << kStages) - 1 : p->timing_mask;
    if (p->general) {
        p->used |= KU_GENERAL;
        const unsigned bmask = tmask | (tmask << 1);
        auto mark = [&](int i) -> int {
            if (evs && ((bmask >> i) & 1u)) OF3D_HIP(hipEventRecord(evs[i], s));
            return 0;
        };
        if (run_general<F>(p, fr, dtype, frame_z0, R, vx, vy, vz, rel, s, mark)) return -1;
        if (!p->host_ev && p->timing_slots) {
            p->tchunks[slot] = 0;
            ++p->tcount;
        }
        p->stages_run = kStages;
        return 0;
    }
    const bool one_stage = evs && !p->host_ev && (tmask & (tmask - 1)) == 0;
    // overlap only with the fused K34, and with no per-stage profile requested
    const int64_t nout = R.zo1 - R.zo0;
    int nch = 1;
    if (d3 && p->k34.fn && p->zchunk > 0 && (!evs || one_stage)) {
        nch = (int)std::min<int64_t>((nout + p->zchunk - 1) / p->zchunk, kMaxChunks);
        if (nch < 2) nch = 1;
    }
    if (nch > 1) fuse_next = false, k0m = 0;  // (zchunk > 0 already excluded both; the invariant)
    if (nch == 1) {
        // serial: boundary i opens stage i and closes stage i-1; untimed stages get no events
        // (every event is a barrier packet between kernels: a few microseconds each)
        const unsigned bmask = tmask | (tmask << 1);
        auto mark = [&](int i) -> int {
            if (evs && ((bmask >> i) & 1u)) OF3D_HIP(hipEventRecord(evs[i], s));
            return 0;
        };
        if (mark(0) || k01(R.zb0, R.zb1, s) || mark(1) || k2(R.zg0, R.zg1, s) || mark(2)) return -1;
        if (p->k34.fn) {
            if (k34(R.zg0, R.zg1, s) || mark(3)) return -1;  // "prod_wy" holds W x too; "wx" stays empty
        } else {
            if (k3k4(s) || mark(3) || k4(s)) return -1;
        }
        if (mark(4) || k5(R.zo0, R.zo1, R.zg1, s) || mark(5)) return -1;
        if (!p->host_ev && p->timing_slots) {
            p->tchunks[slot] = 0;
            ++p->tcount;
        }
        for (int j = 1; j < k0m; ++j) {  // the batched windows the next calls may skip K0 for
            auto& d = p->dts[j];
            d.valid = true;
            for (int i = 0; i < nwin; ++i) d.frames[i] = d_frames[j + i];
            d.dtype = dtype;
            d.fz0 = frame_z0;
            d.zo0 = zo0;
            d.zo1 = zo1;
        }
        if (fuse_next && p->k5c && d3) {  // the next call may skip its K0
            p->pipe_valid = true;
            for (int i = 0; i < nwin; ++i) p->pipe_frames[i] = d_next[i];
            p->pipe_fz0 = frame_z0;
            p->pipe_zo0 = zo0;
            p->pipe_zo1 = zo1;
            p->pipe_dtype = dtype;
            p->pipe_k12 = k12 != nullptr;
        }
    } else {
        // overlap: chunk c = outputs [o_c, o_c+1); its G/Q planes end rw above, its B planes rd above that
        hipStream_t s2 = p->stream2;
        OF3D_HIP(hipEventRecord(p->ev_fork, s));
        OF3D_HIP(hipStreamWaitEvent(s2, p->ev_fork, 0));
        const int tst = one_stage ? __builtin_ctz(tmask) : -1;  // the one timed stage (events per chunk)
        int64_t b_prev = R.zb0, q_prev = R.zg0;
        const int64_t cz = (nout + nch - 1) / nch;
        for (int c = 0; c < nch; ++c) {
            const int64_t o0 = R.zo0 + c * cz, o1 = std::min(o0 + cz, R.zo1);
            const bool last = c == nch - 1;
            const int64_t q1 = last ? R.zg1 : std::min(o1 + p->rw, R.zg1);
            const int64_t b1 = last ? R.zb1 : std::min(q1 + p->rd, R.zb1);
            auto tm = [&](int stage, int edge, hipStream_t st) -> int {
                if (stage == tst) OF3D_HIP(hipEventRecord(evs[2 * c + edge], st));
                return 0;
            };
            if (tm(0, 0, s) || k01(b_prev, b1, s) || tm(0, 1, s) || tm(1, 0, s) || k2(q_prev, q1, s) || tm(1, 1, s))
                return -1;
            OF3D_HIP(hipEventRecord(p->ev_chunk[c], s));
            OF3D_HIP(hipStreamWaitEvent(s2, p->ev_chunk[c], 0));
            if (tm(2, 0, s2) || k34(q_prev, q1, s2) || tm(2, 1, s2) || tm(4, 0, s2) || k5(o0, o1, q1, s2) ||
                tm(4, 1, s2))
                return -1;
            b_prev = b1;
            q_prev = q1;
        }
        OF3D_HIP(hipEventRecord(p->ev_join, s2));
        OF3D_HIP(hipStreamWaitEvent(s, p->ev_join, 0));
        if (!p->host_ev && p->timing_slots) {
            p->tchunks[slot] = one_stage ? nch : 0;
            ++p->tcount;
        }
    }
    p->stages_run = kStages;
    return 0;
}

// pipe: an of3d_plan_execute_next call (may use the dt0 the previous such call formed for
// these frames); d_next: the next output frame's frames (NULL: none)
// ahead >= 0: an of3d_plan_execute_ahead call (d_frames holds 2 rt + 1 + ahead frames)
int run(of3d_plan* p, const void* const* d_frames, int dtype, int64_t frame_z0, int64_t zo0, int64_t zo1, void* vx,
        void* vy, void* vz, void* rel, hipStream_t s, const void* const* d_next = nullptr, bool pipe = false,
        int ahead = -1) {
    const int rc = p->fp32 ? run_t<float>(p, d_frames, dtype, frame_z0, zo0, zo1, vx, vy, vz, rel, s, d_next, pipe, ahead)
                           : run_t<double>(p, d_frames, dtype, frame_z0, zo0, zo1, vx, vy, vz, rel, s, d_next, pipe, ahead);
    // completion marker: plan_free waits for the plan's own work only (not the whole device)
    if (rc == 0 && p->ev_done) OF3D_HIP(hipEventRecord(p->ev_done, s));
    return rc;
}

void plan_free(of3d_plan* p);

// The z-tiled W-xy layout addresses a K34 tile of S rows through ONE buffer descriptor with 32-bit
// byte offsets (csrc/of3d_dev.hpp wxy_rsrc / wxy_off): S * nx * cap_planes elements must stay below
// 2^31 bytes for the largest S of any K34 candidate the autotune may pick (an fp64 plan
// of nz = nx = 4096, ny = 64 would span 2 GiB per 16-row tile, and stores past it are dropped by the
// descriptor's range check without an error).  Plans past it keep the plain planes.
bool wxy_tile_fits(const of3d_plan* p) {
    int smax = p->k34.s;
    for (const auto& k : p->k34_cand) smax = std::max(smax, k.s);
    const size_t es = p->fp32 ? sizeof(float) : sizeof(double);
    return (size_t)smax * (size_t)p->nx * (size_t)p->cap_planes * es <= 0x7fffffffu;
}

int plan_create(of3d_plan** out, int ndim, int64_t nz, int64_t ny, int64_t nx, const of3d_taps* taps, int mode,
                int device, int64_t max_out_planes) {
    if (!out) return fail("of3d: null plan pointer");
    *out = nullptr;
    if ((mode & ~(OF3D_REL_F64 | OF3D_FP32)) != OF3D_FP64_EXACT) return fail("of3d: unsupported mode");
    if (ndim != 2 && ndim != 3) return fail("of3d: ndim must be 2 or 3");
    // (2D: nz independent frames processed together — a batch of output frames; no coupling)
    if (nz < 1 || ny < 1 || nx < 1) return fail("of3d: empty volume");
    if (ny * nx > (int64_t)INT32_MAX || nz > 65535) return fail("of3d: volume too large for one plan");
    // every error path below frees whatever the plan holds so far (plan_free takes partial plans)
    struct Owner {
        of3d_plan* p = new of3d_plan;
        ~Owner() { plan_free(p); }
        of3d_plan* get() const { return p; }
        of3d_plan* operator->() const { return p; }
        of3d_plan* release() { of3d_plan* q = p; p = nullptr; return q; }
    } p;
    p->kn = Knobs::read();
    p->ndim = ndim;
    p->rel64 = (mode & OF3D_REL_F64) != 0;
    p->fp32 = (mode & OF3D_FP32) != 0;
    p->nz = nz;
    p->ny = ny;
    p->nx = nx;
    p->ya = 0;
    p->yb = ny;
    p->device = device;
    if (build_taps(taps, p.get())) return -1;
    OF3D_HIP(hipSetDevice(device));
    OF3D_HIP(hipDeviceGetAttribute(&p->ncu, hipDeviceAttributeMultiprocessorCount, device));
    int64_t mo = (max_out_planes <= 0 || max_out_planes > nz) ? nz : max_out_planes;
    p->cap_planes = ndim == 2 ? mo : std::min<int64_t>(nz, mo + 2 * (p->rw + p->rd));
    p->fs = (size_t)p->cap_planes * ny * nx;
    if (set_attrs(p.get())) return -1;
    // the z-tiled W-xy hand-off wherever the fused K34 writes it and K5c reads it (nx a multiple
    // of the 32-column K5c tile), for fp64 workspaces of >= 128 planes: K5c's contiguous windows
    // gain more there than K34's 256-byte store pieces cost (same box, tiled vs planes: c3 frame
    // 3.164 / 3.151 vs 3.175 / 3.183 ms, c4 21.58 vs 21.98; c2 (64 planes) 0.389 / 0.387 vs 0.381 /
    // 0.385, c5 fp32 (128-byte pieces) 102.5 vs 102.1: planes there; profiles/r05/ab_wxy_tile2/)
    p->wxy_zt = (ndim == 3 && p->kn.wxy_tile != 0 && !p->general && p->k34.fn && p->k5c && nx % 32 == 0 &&
                 (p->kn.wxy_tile == 1 || (!p->fp32 && p->cap_planes >= 128)) && wxy_tile_fits(p.get()))
                    ? (int)p->cap_planes : 0;
    OF3D_HIP(hipMalloc(&p->d_taps, p->htaps.size() * sizeof(double)));
    OF3D_HIP(hipMemcpy(p->d_taps, p->htaps.data(), p->htaps.size() * sizeof(double), hipMemcpyHostToDevice));
    {
        std::vector<float> h32(p->htaps.begin(), p->htaps.end());  // round-to-nearest, as numpy's astype
        OF3D_HIP(hipMalloc(&p->d_taps32, h32.size() * sizeof(float)));
        OF3D_HIP(hipMemcpy(p->d_taps32, h32.data(), h32.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    const size_t es = p->fp32 ? sizeof(float) : sizeof(double);
    OF3D_HIP(hipMalloc(&p->X, 9 * p->fs * es));
    OF3D_HIP(hipMalloc(&p->Y, 9 * p->fs * es));
    OF3D_HIP(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    OF3D_HIP(hipStreamCreateWithFlags(&p->stream2, hipStreamNonBlocking));
    OF3D_HIP(hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming));
    OF3D_HIP(hipEventCreateWithFlags(&p->ev_join, hipEventDisableTiming));
    for (auto& e : p->ev_chunk) OF3D_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    p->zchunk = p->kn.zchunk;
    // OF3D_K34_CAND=i pins the i-th candidate geometry of the K34 autotune (tests run every
    // candidate and compare bits; multi-rank runs can pin one choice for every rank)
    if (p->kn.k34_cand >= 0) {
        const size_t i = (size_t)p->kn.k34_cand;
        if (i < p->k34_cand.size()) {
            p->k34 = p->k34_cand[i];
        } else {  // a pin meant for another plan shape (fewer candidates): keep the heuristic pick
            if (p->kn.k34_strict) return fail("of3d: OF3D_K34_CAND out of range");
            fprintf(stderr, "of3d: OF3D_K34_CAND=%zu ignored for this plan (%zu candidates)\n", i,
                    p->k34_cand.size());
        }
    } else if (p->kn.k34_tune) {
        OF3D_HIP(hipMemsetAsync(p->X, 0, 9 * p->fs * es, p->stream));  // defined (zero) tuning inputs
        OF3D_HIP(hipMemsetAsync(p->Y, 0, 9 * p->fs * es, p->stream));
        if ((p->fp32 ? k34_tune<float>(p.get()) : k34_tune<double>(p.get()))) return -1;
    }
    for (auto& e : p->ev) OF3D_HIP(hipEventCreate(&e));
    OF3D_HIP(hipEventCreateWithFlags(&p->ev_done, hipEventDisableTiming));
    *out = p.release();
    return 0;
}

void plan_free(of3d_plan* p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    if (p->stream) (void)hipStreamSynchronize(p->stream);
    // executions on callers' streams may still read the workspace: wait for the last one (every
    // execution records ev_done on its stream; a plan's executions are ordered by its caller, as
    // they share the workspace) — not for the whole device, which would also wait for unrelated
    // streams while the host-entry cache holds its lock
    if (p->ev_done) (void)hipEventSynchronize(p->ev_done);
    else (void)hipDeviceSynchronize();  // (a partial plan: no event yet)
    (void)hipFree(p->d_taps);
    (void)hipFree(p->d_taps32);
    (void)hipFree(p->X);
    (void)hipFree(p->Y);
    (void)hipFree(p->d_in);
    (void)hipFree(p->d_out);
    for (auto& e : p->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto e : p->tev) (void)hipEventDestroy(e);
    for (hipEvent_t e : {p->ev_fork, p->ev_join})
        if (e) (void)hipEventDestroy(e);
    for (auto e : p->ev_chunk)
        if (e) (void)hipEventDestroy(e);
    if (p->stream2) {
        (void)hipStreamSynchronize(p->stream2);
        (void)hipStreamDestroy(p->stream2);
    }
    if (p->stream) (void)hipStreamDestroy(p->stream);
    if (p->ev_done) (void)hipEventDestroy(p->ev_done);
    delete p;
}

// ---- host-entry plan cache (one plan per thread's last shape) ------------
struct CacheKey {
    int ndim, device, mode;
    int64_t nz, ny, nx;
    std::vector<double> taps;
    std::vector<int> radii;
    Knobs kn;  // a plan made under other kernel-family switches is another plan
    bool operator==(const CacheKey& o) const {
        return ndim == o.ndim && device == o.device && mode == o.mode && nz == o.nz && ny == o.ny && nx == o.nx && taps == o.taps &&
               radii == o.radii && kn == o.kn;
    }
};

std::mutex g_cache_mu;
struct CacheEntry {
    CacheKey key;
    of3d_plan* plan = nullptr;
};
std::vector<CacheEntry> g_cache;  // small LRU

CacheKey make_key(int ndim, int device, int mode, int64_t nz, int64_t ny, int64_t nx, const of3d_taps* t) {
    CacheKey k{ndim, device, mode, nz, ny, nx, {}, {t->rd, t->rs, t->rt, t->rw}, Knobs::read()};
    auto add = [&](const double* w, int r) { k.taps.insert(k.taps.end(), w, w + 2 * r + 1); };
    add(t->gauss, t->rd);
    add(t->deriv, t->rd);
    add(t->smooth, t->rs);
    add(t->tderiv, t->rt);
    add(t->window, t->rw);
    return k;
}

int host_flow(int ndim, const void* images, int dtype, int64_t nt, int64_t nz, int64_t ny, int64_t nx,
              const of3d_taps* taps, int mode, int device, double* vx, double* vy, double* vz, void* rel,
              of3d_perf* perf) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!images || !vx || !vy || !rel || (ndim == 3 && !vz)) return fail("of3d: null buffer");
    if (!taps) return fail("of3d: null taps");
    if (mode & OF3D_FP32) return fail("of3d: OF3D_FP32 is a plan mode (float outputs); use of3d_plan_*");
    const size_t es = dtype_size(dtype);
    if (!es) return fail("of3d: unsupported dtype");
    if (nt < 1 || !(nt & 1)) return fail("of3d: nt must be odd");
    const int64_t c = nt / 2;  // ceil(Nt/2)-1 for odd Nt (calc_flow.py:223)
    const int rt = taps->rt;
    if (taps->rt < 0 || 2 * rt + 1 > kMaxT) return fail("of3d: temporal tap radius exceeds 32");
    // plans evicted from the cache are freed after the lock is released (declared before it)
    struct Evicted {
        std::vector<of3d_plan*> v;
        ~Evicted() {
            for (of3d_plan* q : v) plan_free(q);
        }
    } evicted;
    std::lock_guard<std::mutex> lk(g_cache_mu);
    CacheKey key = make_key(ndim, device, mode, nz, ny, nx, taps);
    of3d_plan* p = nullptr;
    for (size_t i = 0; i < g_cache.size(); ++i)
        if (g_cache[i].key == key) {
            p = g_cache[i].plan;
            std::rotate(g_cache.begin(), g_cache.begin() + i, g_cache.begin() + i + 1);
            break;
        }
    if (!p) {
        if (plan_create(&p, ndim, nz, ny, nx, taps, mode, device, 0)) return -1;
        g_cache.insert(g_cache.begin(), CacheEntry{key, p});
        while (g_cache.size() > 2) {
            evicted.v.push_back(g_cache.back().plan);
            g_cache.pop_back();
        }
    }
    OF3D_HIP(hipSetDevice(device));
    const size_t vox = (size_t)nz * ny * nx;
    // Only frames c-rt..c+rt enter the result (time indices clamped to [0,nt)).
    const int nwin = 2 * rt + 1;
    const size_t in_bytes = (size_t)nwin * vox * es;
    if (p->d_in_bytes < in_bytes) {
        (void)hipFree(p->d_in);
        p->d_in = nullptr;
        OF3D_HIP(hipMalloc(&p->d_in, in_bytes));
        p->d_in_bytes = in_bytes;
    }
    const size_t rel_es = (ndim == 3 && !(mode & OF3D_REL_F64)) ? sizeof(float) : sizeof(double);
    const size_t out_bytes = vox * (3 * sizeof(double) + rel_es);
    if (p->d_out_bytes < out_bytes) {
        (void)hipFree(p->d_out);
        p->d_out = nullptr;
        OF3D_HIP(hipMalloc(&p->d_out, out_bytes));
        p->d_out_bytes = out_bytes;
    }
    hipStream_t s = p->stream;
    hipEvent_t e0 = p->ev[0], e1 = p->ev[1];
    const void* dptr[kMaxT];
    // distinct frames needed, uploaded once each
    std::vector<int64_t> src(nwin);
    for (int i = 0; i < nwin; ++i) src[i] = std::min<int64_t>(std::max<int64_t>(c - rt + i, 0), nt - 1);
    for (int i = 0; i < nwin; ++i) {
        char* dst = (char*)p->d_in + (size_t)i * vox * es;
        dptr[i] = dst;
        OF3D_HIP(hipMemcpyAsync(dst, (const char*)images + (size_t)src[i] * vox * es, vox * es, hipMemcpyHostToDevice, s));
    }
    OF3D_HIP(hipStreamSynchronize(s));
    const auto t1 = std::chrono::steady_clock::now();
    double* dvx = (double*)p->d_out;
    double* dvy = dvx + vox;
    double* dvz = dvy + vox;
    void* drel = (void*)(dvz + vox);
    p->host_ev = true;
    int rc = run(p, dptr, dtype, 0, 0, nz, dvx, dvy, ndim == 3 ? dvz : nullptr, drel, s);
    p->host_ev = false;
    if (rc) return rc;
    OF3D_HIP(hipStreamSynchronize(s));
    float kms = 0.f;
    OF3D_HIP(hipEventElapsedTime(&kms, p->ev[0], p->ev[kStages]));
    for (int i = 0; i < kStages; ++i) {
        float m = 0.f;
        (void)hipEventElapsedTime(&m, p->ev[i], p->ev[i + 1]);
        p->stage_ms[i] = m;
    }
    (void)e0;
    (void)e1;
    const auto t2 = std::chrono::steady_clock::now();
    OF3D_HIP(hipMemcpyAsync(vx, dvx, vox * sizeof(double), hipMemcpyDeviceToHost, s));
    OF3D_HIP(hipMemcpyAsync(vy, dvy, vox * sizeof(double), hipMemcpyDeviceToHost, s));
    if (ndim == 3) OF3D_HIP(hipMemcpyAsync(vz, dvz, vox * sizeof(double), hipMemcpyDeviceToHost, s));
    OF3D_HIP(hipMemcpyAsync(rel, drel, vox * rel_es, hipMemcpyDeviceToHost, s));
    OF3D_HIP(hipStreamSynchronize(s));
    const auto t3 = std::chrono::steady_clock::now();
    if (perf) {
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        perf->ms_h2d = ms(t0, t1);
        perf->ms_kernels = kms;
        perf->ms_d2h = ms(t2, t3);
        perf->ms_total = ms(t0, t3);
    }
    return 0;
}

}  // namespace

// ---------------------------------------------------------------------------
// Bounded-footprint copy (of3d_copy_async): 16-byte lanes, non-temporal
// stores, grid-stride over at most max_blocks workgroups; byte tail by block 0.
// ---------------------------------------------------------------------------
namespace {
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n16,
                                              const unsigned char* __restrict__ tsrc, unsigned char* __restrict__ tdst,
                                              int tail) {
    const size_t st = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += st)
        __builtin_nontemporal_store(src[i], &dst[i]);
    if (blockIdx.x == 0 && (int)threadIdx.x < tail) tdst[threadIdx.x] = tsrc[threadIdx.x];
}

__global__ __launch_bounds__(256) void k_copy_bytes(const unsigned char* __restrict__ src,
                                                    unsigned char* __restrict__ dst, size_t n) {
    const size_t st = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += st) dst[i] = src[i];
}

}  // namespace

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" {

int of3d_version(void) { return OF3D_VERSION; }

int of3d_cache_clear(void) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    for (auto& e : g_cache) plan_free(e.plan);
    g_cache.clear();
    return 0;
}

const char* of3d_last_error(void) { return g_err.c_str(); }

int of3d_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int of3d_flow3d(const void* images, int dtype, int64_t nt, int64_t nz, int64_t ny, int64_t nx, const of3d_taps* taps,
                int mode, int device, double* vx, double* vy, double* vz, void* rel, of3d_perf* perf) {
    return host_flow(3, images, dtype, nt, nz, ny, nx, taps, mode, device, vx, vy, vz, rel, perf);
}

int of3d_flow2d(const void* images, int dtype, int64_t nt, int64_t ny, int64_t nx, const of3d_taps* taps, int mode,
                int device, double* vx, double* vy, double* rel, of3d_perf* perf) {
    return host_flow(2, images, dtype, nt, 1, ny, nx, taps, mode, device, vx, vy, nullptr, rel, perf);
}

int of3d_plan_create(of3d_plan** plan, int ndim, int64_t nz, int64_t ny, int64_t nx, const of3d_taps* taps, int mode,
                     int device, int64_t max_out_planes) {
    return plan_create(plan, ndim, nz, ny, nx, taps, mode, device, max_out_planes);
}

int of3d_plan_destroy(of3d_plan* plan) {
    plan_free(plan);
    return 0;
}

size_t of3d_plan_workspace_bytes(const of3d_plan* p) {
    return p ? 18 * p->fs * (p->fp32 ? sizeof(float) : sizeof(double)) : 0;
}

int of3d_plan_input_range(const of3d_plan* p, int64_t zo0, int64_t zo1, int64_t* zi0, int64_t* zi1) {
    if (!p || !zi0 || !zi1) return fail("of3d: null argument");
    if (zo0 < 0 || zo1 > p->nz || zo0 >= zo1) return fail("of3d: bad output plane range");
    const Ranges r = ranges(p, zo0, zo1);
    *zi0 = r.zb0;
    *zi1 = r.zb1;
    return 0;
}

int of3d_plan_execute(of3d_plan* p, const void* const* d_frames, int dtype, int64_t frame_z0, int64_t zo0, int64_t zo1,
                      void* vx, void* vy, void* vz, void* rel, void* stream) {
    if (!p || !d_frames || !vx || !vy || !rel || (p->ndim == 3 && !vz)) return fail("of3d: null argument");
    OF3D_HIP(hipSetDevice(p->device));
    hipStream_t s = (hipStream_t)stream;  // NULL: the device's null stream (HIP's convention)
    return run(p, d_frames, dtype, frame_z0, zo0, zo1, vx, vy, vz, rel, s);
}

int of3d_plan_execute_next(of3d_plan* p, const void* const* d_frames, const void* const* d_frames_next, int dtype,
                           int64_t frame_z0, int64_t zo0, int64_t zo1, void* vx, void* vy, void* vz, void* rel,
                           void* stream) {
    if (!p || !d_frames || !vx || !vy || !rel || (p->ndim == 3 && !vz)) return fail("of3d: null argument");
    OF3D_HIP(hipSetDevice(p->device));
    hipStream_t s = (hipStream_t)stream;  // NULL: the device's null stream (HIP's convention)
    return run(p, d_frames, dtype, frame_z0, zo0, zo1, vx, vy, vz, rel, s, d_frames_next, true);
}

int of3d_plan_execute_ahead(of3d_plan* p, const void* const* d_frames, int n_ahead, int dtype, int64_t frame_z0,
                            int64_t zo0, int64_t zo1, void* vx, void* vy, void* vz, void* rel, void* stream) {
    if (!p || !d_frames || !vx || !vy || !rel || (p->ndim == 3 && !vz)) return fail("of3d: null argument");
    if (n_ahead < 0) return fail("of3d: n_ahead out of range");
    n_ahead = std::min(n_ahead, kMaxT - (2 * p->rt + 1));  // frames past kMaxT are not batched
    OF3D_HIP(hipSetDevice(p->device));
    hipStream_t s = (hipStream_t)stream;  // NULL: the device's null stream (HIP's convention)
    return run(p, d_frames, dtype, frame_z0, zo0, zo1, vx, vy, vz, rel, s, nullptr, false, n_ahead);
}

int of3d_plan_set_timing(of3d_plan* p, int slots) {
    if (!p) return fail("of3d: null plan");
    if (slots < 0 || slots > 4096) return fail("of3d: timing slots must be in [0, 4096]");
    OF3D_HIP(hipSetDevice(p->device));
    OF3D_HIP(hipDeviceSynchronize());  // executions may sit on any caller stream: events idle first
    for (auto e : p->tev) (void)hipEventDestroy(e);
    p->tev_per_slot = std::max(kStages + 1, 2 * kMaxChunks);
    p->tev.assign((size_t)slots * p->tev_per_slot, nullptr);
    for (auto& e : p->tev) OF3D_HIP(hipEventCreate(&e));
    p->tchunks.assign(slots, 0);
    p->timing_slots = slots;
    p->tcount = 0;
    return 0;
}

int of3d_plan_set_timing_mask(of3d_plan* p, unsigned mask) {
    if (!p) return fail("of3d: null plan");
    mask &= (1u << kStages) - 1;
    if (!mask) return fail("of3d: timing mask selects no stage");
    OF3D_HIP(hipSetDevice(p->device));
    OF3D_HIP(hipDeviceSynchronize());
    p->timing_mask = mask;
    p->tcount = 0;
    return 0;
}

int of3d_plan_stage_times(of3d_plan* p, double* ms, int cap) {
    if (!p || !ms) return fail("of3d: null argument");
    if (!p->timing_slots) return fail("of3d: timing not enabled on this plan");
    const int64_t n = std::min<int64_t>(p->tcount, p->timing_slots);
    if (n == 0) return fail("of3d: no timed executions since the last read");
    const int m = std::min(cap, kStages);
    std::vector<double> acc(kStages, 0.0);
    for (int64_t j = 0; j < n; ++j) {
        hipEvent_t* e = &p->tev[(size_t)j * p->tev_per_slot];
        if (const int nch = p->tchunks[j]) {  // overlap mode: the one timed stage, summed over its chunks
            const int st = __builtin_ctz(p->timing_mask);
            OF3D_HIP(hipEventSynchronize(e[2 * nch - 1]));
            for (int c = 0; c < nch; ++c) {
                float t = 0.f;
                OF3D_HIP(hipEventElapsedTime(&t, e[2 * c], e[2 * c + 1]));
                acc[st] += t;
            }
            continue;
        }
        int last = kStages;
        while (!((p->timing_mask >> (last - 1)) & 1u)) --last;  // closing boundary of the last timed stage
        OF3D_HIP(hipEventSynchronize(e[last]));
        for (int i = 0; i < kStages; ++i) {
            if (!((p->timing_mask >> i) & 1u)) continue;
            float t = 0.f;
            OF3D_HIP(hipEventElapsedTime(&t, e[i], e[i + 1]));
            acc[i] += t;
        }
    }
    for (int i = 0; i < m; ++i) ms[i] = ((p->timing_mask >> i) & 1u) ? acc[i] / (double)n : -1.0;
    if (p->k34.fn && m > 3) ms[3] = -1.0;  // fused K34: "prod_wy" holds W x too, "wx" is empty
    p->tcount = 0;
    return m;
}

int of3d_plan_set_rows(of3d_plan* p, int64_t y0, int64_t y1) {
    if (!p) return fail("of3d: null plan");
    if (y0 < 0 || y1 > p->ny || y0 >= y1) return fail("of3d: bad output row range");
    if (y0 != 0 || y1 != p->ny) {
        if (p->ndim != 3 || p->general || !p->k34.fn || !p->k5c || p->zchunk > 0)
            return fail("of3d: output row ranges need the fused K34 and K5c kernels (3D, serial)");
    }
    p->ya = y0;
    p->yb = y1;
    return 0;
}

int of3d_plan_kernels(const of3d_plan* p, char* buf, size_t n) {
    if (!p) return fail("of3d: null plan");
    std::string out;
    for (size_t i = 0; i < sizeof(kKernelNames) / sizeof(kKernelNames[0]); ++i)
        if ((p->used >> i) & 1u) out += (out.empty() ? "" : ",") + std::string(kKernelNames[i]);
    if (buf && n) {
        const size_t k = std::min(n - 1, out.size());
        memcpy(buf, out.data(), k);
        buf[k] = 0;
    }
    return (int)out.size();
}

int of3d_plan_geometry(const of3d_plan* p, char* buf, size_t n) {
    if (!p) return fail("of3d: null plan");
    int smax = p->k34.s;
    for (const auto& k : p->k34_cand) smax = std::max(smax, k.s);
    char tmp[768];
    snprintf(tmp, sizeof(tmp),
             "{\"ndim\": %d, \"nz\": %lld, \"ny\": %lld, \"nx\": %lld, \"fp32\": %d, \"general\": %d, "
             "\"cap_planes\": %lld, \"wxy_zt\": %d, \"k34\": {\"cw\": %d, \"s\": %d, \"tx\": %d, \"nbx\": %d, "
             "\"threads\": %d, \"lds\": %zu, \"candidates\": %zu, \"s_max\": %d}, \"k5c\": {\"r\": %d, \"nw\": %d, "
             "\"lds\": %zu}, \"k12\": {\"march\": %d, \"grid\": [%d, %d], \"deep\": %d}, \"k0_batch\": %d, \"ncu\": %d}",
             p->ndim, (long long)p->nz, (long long)p->ny, (long long)p->nx, (int)p->fp32, (int)p->general,
             (long long)p->cap_planes, p->wxy_zt, p->k34.cw, p->k34.s, p->k34.tx, p->k34.nbx,
             p->k34.nthr ? p->k34.nthr : p->k34.cw, p->k34.lds, p->k34_cand.size(), smax, p->k5c ? p->k5c_r : 0,
             p->k5c ? p->k5c_nw : 0, p->k5c_lds, p->last_k12_zc, p->last_k12_gx, p->last_k12_gy, p->last_k12_deep, p->last_k0m,
             p->ncu);
    const std::string out(tmp);
    if (buf && n) {
        const size_t k = std::min(n - 1, out.size());
        memcpy(buf, out.data(), k);
        buf[k] = 0;
    }
    return (int)out.size();
}

int of3d_plan_set_overlap(of3d_plan* p, int64_t chunk_planes) {
    if (!p) return fail("of3d: null plan");
    // the two modes exclude each other both ways (of3d_plan_set_rows refuses a chunked plan)
    if (chunk_planes > 0 && (p->ya != 0 || p->yb != p->ny))
        return fail("of3d: overlap mode needs the full row range (of3d_plan_set_rows(0, ny) first)");
    p->zchunk = chunk_planes > 0 ? chunk_planes : 0;
    return 0;
}

const char* of3d_stage_name(int i) { return (i >= 0 && i < kStages) ? kStageNames[i] : ""; }

int of3d_dma_copy(void* const* dst, const void* const* src, const size_t* bytes, int n) {
    if (n <= 0) return 0;
    if (!dst || !src || !bytes) return fail("of3d: null argument");
    static std::once_flag once;
    static hsa_status_t init = HSA_STATUS_ERROR;
    std::call_once(once, [] { init = hsa_init(); });  // reference-counted; the HIP runtime holds one too
    if (init != HSA_STATUS_SUCCESS) return fail("of3d: hsa_init failed");
    hsa_signal_t sig;
    if (hsa_signal_create(n, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return fail("of3d: hsa_signal_create failed");
    int issued = 0;
    std::string err;
    for (; issued < n; ++issued) {
        const int i = issued;
        if (bytes[i] == 0) {
            hsa_signal_subtract_relaxed(sig, 1);
            continue;
        }
        hsa_amd_pointer_info_t si{}, di{};
        si.size = sizeof(si);
        di.size = sizeof(di);
        if (hsa_amd_pointer_info(src[i], &si, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
            hsa_amd_pointer_info(dst[i], &di, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
            si.type == HSA_EXT_POINTER_TYPE_UNKNOWN || di.type == HSA_EXT_POINTER_TYPE_UNKNOWN) {
            err = "of3d: dma copy needs device or pinned host buffers";
            break;
        }
        if (hsa_amd_memory_async_copy(dst[i], di.agentOwner, src[i], si.agentOwner, bytes[i], 0, nullptr, sig) !=
            HSA_STATUS_SUCCESS) {
            err = "of3d: hsa_amd_memory_async_copy failed";
            break;
        }
    }
    if (issued < n) hsa_signal_subtract_relaxed(sig, n - issued);  // drop the copies never issued
    hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    hsa_signal_destroy(sig);
    if (!err.empty()) return fail(err.c_str());
    return 0;
}

int of3d_flow_stats(const void* vx, const void* vy, const void* vz, const void* rel, int v_f32, int rel_f64,
                    int64_t n, double thresh, double xyscale, double zscale, double tscale, double* out_vx,
                    double* out_vy, double* out_vz, double* magnitude, double* theta, double* phi, void* stream) {
    if (n < 0) return fail("of3d: negative element count");
    if (n == 0) return 0;
    if (!vx || !vy || !rel || !out_vx || !out_vy || !magnitude || !theta) return fail("of3d: null argument");
    if (vz && (!out_vz || !phi)) return fail("of3d: null argument");
    hipStream_t s = (hipStream_t)stream;
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 256 * 32);
    auto launch = [&](auto vt, auto rt) {
        using VT = decltype(vt);
        using RT = decltype(rt);
        hipLaunchKernelGGL((k_flow_stats<VT, RT>), dim3(blocks), dim3(256), 0, s, (const VT*)vx, (const VT*)vy,
                           (const VT*)vz, (const RT*)rel, (size_t)n, thresh, xyscale, zscale, tscale, out_vx, out_vy,
                           out_vz, magnitude, theta, phi);
    };
    if (v_f32)
        rel_f64 ? launch(float{}, double{}) : launch(float{}, float{});
    else
        rel_f64 ? launch(double{}, double{}) : launch(double{}, float{});
    OF3D_HIP(hipGetLastError());
    return 0;
}

int of3d_rel3d(const double* tensor, int64_t n, void* rel, int rel_f64, void* stream) {
    if (n < 0) return fail("of3d: negative element count");
    if (n == 0) return 0;
    if (!tensor || !rel) return fail("of3d: null argument");
    hipStream_t s = (hipStream_t)stream;
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 256 * 32);
    if (rel_f64)
        hipLaunchKernelGGL(k_rel3d<double>, dim3(blocks), dim3(256), 0, s, tensor, (size_t)n, (double*)rel);
    else
        hipLaunchKernelGGL(k_rel3d<float>, dim3(blocks), dim3(256), 0, s, tensor, (size_t)n, (float*)rel);
    OF3D_HIP(hipGetLastError());
    return 0;
}

int of3d_copy_async(void* dst, const void* src, size_t bytes, int max_blocks, void* stream) {
    if (bytes == 0) return 0;
    if (!dst || !src) return fail("of3d: null argument");
    if (max_blocks < 0) return fail("of3d: max_blocks must be >= 0");
    const unsigned mb = max_blocks ? (unsigned)max_blocks : 64u;
    hipStream_t s = (hipStream_t)stream;
    if ((uintptr_t)dst % 16 == 0 && (uintptr_t)src % 16 == 0) {
        const size_t n16 = bytes / 16;
        const int tail = (int)(bytes % 16);
        const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(mb, (n16 + 255) / 256));
        hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, s, (const u32x4*)src, (u32x4*)dst, n16,
                           (const unsigned char*)src + n16 * 16, (unsigned char*)dst + n16 * 16, tail);
    } else {
        const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(mb, (bytes + 255) / 256));
        hipLaunchKernelGGL(k_copy_bytes, dim3(blocks), dim3(256), 0, s, (const unsigned char*)src,
                           (unsigned char*)dst, bytes);
    }
    OF3D_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
