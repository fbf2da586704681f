/* of3d_cli — calc_flow3D (calc_flow.py:175-360) from C, through the C-ABI only (include/of3d.h,
 * libof3d.so): no Python, no torch.  What a non-Python caller of the boundary looks like.
 *
 *   of3d_cli --version
 *   of3d_cli IMAGES.u16 NT NZ NY NX TAPS.f64 OUT_PREFIX [rel64]
 *
 * IMAGES.u16: raw uint16 (nt, nz, ny, nx), C order.  TAPS.f64: raw float64 — the header
 * [rd, rs, rt, rw] then gauss (2rd+1), deriv (2rd+1), smooth (2rs+1), tderiv (2rt+1),
 * window (2rw+1), the reference's taps (taps.make_taps / calc_flow.py:230-267).  Writes
 * OUT_PREFIX{vx,vy,vz}.f64 and OUT_PREFIXrel.f32 (.f64 with rel64: OF3D_REL_F64).
 * Exit status 0 on success; errors print of3d_last_error(). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "of3d.h"

/* a regular file whole (NULL for anything ftell cannot size: pipes, FIFOs, errors) */
static void* read_file(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    long len = -1;
    if (fseek(f, 0, SEEK_END) == 0) len = ftell(f);
    if (len < 0 || fseek(f, 0, SEEK_SET) != 0) {
        fclose(f);
        return NULL;
    }
    void* buf = malloc(len > 0 ? (size_t)len : 1);
    if (buf && fread(buf, 1, (size_t)len, f) != (size_t)len) {
        free(buf);
        buf = NULL;
    }
    fclose(f);
    *n = (size_t)len;
    return buf;
}

static int write_file(const char* prefix, const char* name, const void* p, size_t n) {
    char path[4096];
    snprintf(path, sizeof path, "%s%s", prefix, name);
    FILE* f = fopen(path, "wb");
    if (!f) return -1;
    size_t w = fwrite(p, 1, n, f);
    fclose(f);
    return w == n ? 0 : -1;
}

int main(int argc, char** argv) {
    if (argc == 2 && strcmp(argv[1], "--version") == 0) {
        printf("of3d %d, %d device(s), %s\n", of3d_version(), of3d_device_count(), of3d_build_info());
        return 0;
    }
    if (argc < 8) {
        fprintf(stderr, "usage: %s IMAGES.u16 NT NZ NY NX TAPS.f64 OUT_PREFIX [rel64]\n", argv[0]);
        return 2;
    }
    const int64_t nt = atoll(argv[2]), nz = atoll(argv[3]), ny = atoll(argv[4]), nx = atoll(argv[5]);
    if (nt < 1 || nz < 1 || ny < 1 || nx < 1 || nz > 65535 || ny * nx > INT32_MAX) {
        fprintf(stderr, "of3d_cli: bad dimensions\n");
        return 2;
    }
    const int rel64 = argc > 8 && strcmp(argv[8], "rel64") == 0;
    size_t ni = 0, nt_ = 0;
    uint16_t* img = (uint16_t*)read_file(argv[1], &ni);
    double* tp = (double*)read_file(argv[6], &nt_);
    /* the stack's size as a quotient (no product of nt that could overflow): whole volumes of
       nz * ny * nx uint16 (ny * nx <= INT32_MAX and nz <= 65535, so that product fits), and exactly nt */
    const uint64_t vol_bytes = (uint64_t)nz * (uint64_t)(ny * nx) * sizeof(uint16_t);
    if (!img || !tp || ni % vol_bytes != 0 || ni / vol_bytes != (uint64_t)nt || nt_ < 4 * sizeof(double)) {
        fprintf(stderr, "of3d_cli: bad input files\n");
        return 2;
    }
    /* radii: whole numbers in [0, 4096] (rt <= 32, the library's limits) before any pointer
       arithmetic on them, and the file must hold exactly the taps they announce */
    for (int i = 0; i < 4; ++i)
        if (!(tp[i] >= 0.0 && tp[i] <= (i == 2 ? 32.0 : 4096.0)) || tp[i] != (double)(int)tp[i]) {
            fprintf(stderr, "of3d_cli: bad tap radius in the taps header\n");
            return 2;
        }
    of3d_taps taps;
    taps.rd = (int)tp[0];
    taps.rs = (int)tp[1];
    taps.rt = (int)tp[2];
    taps.rw = (int)tp[3];
    const size_t ntaps = 4 + (size_t)(2 * taps.rd + 1) * 2 + (2 * taps.rs + 1) + (2 * taps.rt + 1) + (2 * taps.rw + 1);
    if (ntaps * sizeof(double) != nt_) {
        fprintf(stderr, "of3d_cli: taps file size does not match its radii\n");
        return 2;
    }
    const double* q = tp + 4;
    taps.gauss = q, q += 2 * taps.rd + 1;
    taps.deriv = q, q += 2 * taps.rd + 1;
    taps.smooth = q, q += 2 * taps.rs + 1;
    taps.tderiv = q, q += 2 * taps.rt + 1;
    taps.window = q;
    const size_t nv = (size_t)(nz * ny * nx);
    double* vx = (double*)malloc(nv * sizeof(double));
    double* vy = (double*)malloc(nv * sizeof(double));
    double* vz = (double*)malloc(nv * sizeof(double));
    void* rel = malloc(nv * (rel64 ? sizeof(double) : sizeof(float)));
    if (!vx || !vy || !vz || !rel) {
        fprintf(stderr, "of3d_cli: out of host memory\n");
        return 1;
    }
    of3d_perf perf;
    if (of3d_flow3d(img, OF3D_U16, nt, nz, ny, nx, &taps, rel64 ? OF3D_REL_F64 : OF3D_FP64_EXACT, 0, vx, vy, vz, rel,
                    &perf) != 0) {
        fprintf(stderr, "of3d_cli: %s\n", of3d_last_error());
        return 1;
    }
    if (write_file(argv[7], "vx.f64", vx, nv * 8) || write_file(argv[7], "vy.f64", vy, nv * 8) ||
        write_file(argv[7], "vz.f64", vz, nv * 8) ||
        write_file(argv[7], rel64 ? "rel.f64" : "rel.f32", rel, nv * (rel64 ? 8 : 4))) {
        fprintf(stderr, "of3d_cli: cannot write outputs\n");
        return 1;
    }
    printf("of3d_cli: %lld x %lld x %lld, kernels %.3f ms, total %.3f ms\n", (long long)nz, (long long)ny,
           (long long)nx, perf.ms_kernels, perf.ms_total);
    free(img), free(tp), free(vx), free(vy), free(vz), free(rel);
    return 0;
}
