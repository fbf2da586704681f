"""Generate the golden fixtures in tests/golden/*.npz (run in the build container only).

The reference module ``/root/reference/src/Python/calc_flow.py`` imports
``tifffile`` and ``natsort`` at module level (calc_flow.py:12,16); neither is
installed here and neither is used by ``calc_flow2D``/``calc_flow3D``, so they
are replaced by empty stub modules.  The reference source is compiled from its
text (never from the shipped ``__pycache__``) into a private module object, and
only its OUTPUTS are written here: inputs (explicit), parameters, the
reference's vx/vy/[vz]/rel, plus the fp64 eigenvalue range of the restated
tensor (for the tighter 3D rel check).  No reference source is copied.

Usage:  python tests/golden/make_golden.py      (writes tests/golden/*.npz)
        python tests/golden/make_golden.py --only c3d_big_xyzsig9,c2d_big_sigmas   (just those)
"""

import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/src/Python/calc_flow.py"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

from oracle import cpu_ref  # noqa: E402


def load_reference():
    for name in ("tifffile", "natsort"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["natsort"].natsorted = sorted
    mod = types.ModuleType("calc_flow_reference")
    mod.__file__ = REF
    with open(REF, "r") as f:
        src = f.read()
    exec(compile(src, REF, "exec"), mod.__dict__)
    return mod


def rand_u16(shape, seed, hi=4096):
    return np.random.default_rng(seed).integers(0, hi, size=shape).astype(np.uint16)


def ramp_u16(shape, axes, slope, speed):
    """I(t, z, y, x) = 1000 + slope * (a_x x + a_y y + a_z z) + speed * t (uint16)."""
    nt, nz, ny, nx = shape
    t, z, y, x = np.meshgrid(*(np.arange(n, dtype=np.float64) for n in shape), indexing="ij")
    ax, ay, az = axes
    return np.round(1000 + slope * (ax * x + ay * y + az * z) + speed * t).astype(np.uint16)


def wave_u16(shape, k, freq, speed):
    """A plane wave 2000 + 900 sin(freq (k . (x, y, z)) + speed t) (uint16)."""
    t, z, y, x = np.meshgrid(*(np.arange(n, dtype=np.float64) for n in shape), indexing="ij")
    return np.round(2000 + 900 * np.sin(freq * (k[0] * x + k[1] * y + k[2] * z) + speed * t)).astype(np.uint16)


def smooth_noise_u16(shape, seed):
    """White noise smoothed by an isotropic Gaussian in z, y, x (sigma 2), per frame."""
    from scipy.ndimage import gaussian_filter

    rng = np.random.default_rng(seed)
    noise = rng.standard_normal(shape)
    sm = np.stack([gaussian_filter(f, 2.0, mode="wrap") for f in noise])
    return np.round(2000 + 800 * sm / sm.std()).astype(np.uint16)


CASES_3D = [
    # name, input builder, (sig, tsig, wsig)
    ("c3d_rand_s1", lambda: rand_u16((7, 6, 20, 24), 1), (1, 1, 2)),
    ("c3d_rand_c2params", lambda: rand_u16((13, 10, 24, 28), 2), (2, 2, 5)),
    ("c3d_rand_c3params", lambda: rand_u16((19, 6, 20, 22), 3), (2, 3, 7)),
    ("c3d_smooth_translate", lambda: cpu_ref.synthetic_stack_np((7, 12, 32, 32), seed=11), (1, 1, 2)),
    ("c3d_flat", lambda: np.full((7, 4, 8, 8), 1000, np.uint16), (1, 1, 2)),
    ("c3d_nz1", lambda: rand_u16((7, 1, 16, 12), 4), (1, 1, 5)),
    ("c3d_nz2", lambda: rand_u16((7, 2, 16, 12), 5), (1, 1, 5)),
    ("c3d_nz3", lambda: rand_u16((7, 3, 16, 12), 6), (1, 1, 5)),
    ("c3d_nz4", lambda: rand_u16((7, 4, 16, 12), 7), (1, 1, 5)),
    ("c3d_float32_nt11", lambda: np.random.default_rng(8).uniform(0, 1000, (11, 5, 12, 16)).astype(np.float32), (1, 1, 2)),
    ("c3d_frac_sigmas", lambda: rand_u16((7, 6, 16, 18), 9), (1.5, 1, 2.5)),
    ("c3d_nonsquare_odd", lambda: rand_u16((7, 5, 9, 33), 10), (1, 1, 3)),
    ("c3d_default_params", lambda: rand_u16((7, 8, 14, 18), 12), (3, 1, 4)),
    # round 2: the reference accepts any sigma (calc_flow.py:230-267): radii past the
    # tiled kernels' limits (rd 27 > 24, rw 51 > 48) run the general-radius path
    ("c3d_big_xyzsig9", lambda: rand_u16((7, 6, 30, 34), 13), (9, 1, 2)),
    ("c3d_big_wsig17", lambda: rand_u16((7, 5, 24, 26), 14), (1, 1, 17)),
    # the published benchmark's parameters (PFS/plot_figureS4_computation.ipynb) at Nz = 4
    ("c3d_pub_s3t1w4_nz4", lambda: rand_u16((7, 4, 40, 48), 15), (3, 1, 4)),
    # W radii 9 and 18 (wSig 3, 6): the fused K34 / K5c instances added for them
    ("c3d_wsig3", lambda: rand_u16((7, 6, 36, 40), 16), (2, 1, 3)),
    ("c3d_wsig6", lambda: rand_u16((7, 9, 44, 48), 17), (1, 1, 6)),
    # round 4: near-degenerate structure tensors (the fp64 rel's hard case: the two smallest
    # eigenvalues (nearly) equal) — a moving linear ramp along x+y+z (rank-1 tensor: lambda_min
    # = lambda_mid ~ 0 in the interior), a ramp and a plane wave in the xy plane (z2 = 0), and
    # isotropically smoothed noise (near-isotropic tensors); the plain trigonometric form misses
    # 1e-10 lambda_max on the planar ramp (5.7e-9 at 11 % of its voxels) and wave (3.3e-10)
    ("c3d_ramp_xyz_rank1", lambda: ramp_u16((7, 10, 24, 28), (1, 1, 1), 30, -25), (1, 1, 3)),
    ("c3d_ramp_xy_planar", lambda: ramp_u16((7, 10, 24, 28), (1, 3, 0), 14, 5), (1, 1, 2)),
    ("c3d_wave_planar", lambda: wave_u16((7, 10, 24, 28), (1, 2, 0), 0.35, -0.3), (1, 1, 3)),
    ("c3d_iso_smoothed_noise", lambda: smooth_noise_u16((7, 12, 30, 32), 18), (1, 1, 4)),
]

CASES_2D = [
    ("c2d_c1params", lambda: rand_u16((7, 48, 64), 21), (1, 1, 5)),
    ("c2d_tiny_s3", lambda: rand_u16((7, 5, 3), 22), (3, 1, 4)),
    ("c2d_flat", lambda: np.full((7, 8, 8), 1000, np.uint16), (1, 1, 2)),
    ("c2d_float32", lambda: np.random.default_rng(23).uniform(0, 1000, (11, 20, 24)).astype(np.float32), (1.5, 1, 2.5)),
    ("c2d_c2params", lambda: rand_u16((13, 30, 40), 24), (2, 2, 5)),
    ("c2d_smooth_translate", lambda: cpu_ref.synthetic_stack_np((7, 40, 36), seed=25), (1, 1, 3)),
    ("c2d_nonsquare", lambda: rand_u16((7, 3, 50), 26), (1, 1, 2)),
    ("c2d_big_sigmas", lambda: rand_u16((7, 40, 44), 27), (9, 1, 17)),
]

ERROR_CASES = [
    # name, dims, shape, tSig
    ("e3d_ndim", 3, (7, 8, 8), 1),
    ("e3d_short", 3, (5, 2, 8, 8), 1),
    ("e3d_even", 3, (8, 2, 8, 8), 1),
    ("e2d_ndim", 2, (7, 2, 8, 8), 1),
    ("e2d_short", 2, (5, 8, 8), 1),
    ("e2d_even", 2, (8, 8, 8), 1),
]


def main():
    only = None
    if "--only" in sys.argv:  # regenerate just these cases (the others' files stay as they are)
        only = set(sys.argv[sys.argv.index("--only") + 1].split(","))
    ref = load_reference()
    manifest = {}
    mpath = os.path.join(HERE, "manifest.json")
    if only and os.path.exists(mpath):
        with open(mpath) as f:
            manifest = json.load(f)
    for name, build, (s, t, w) in CASES_3D:
        if only and name not in only:
            continue
        img = build()
        vx, vy, vz, rel = ref.calc_flow3D(img, s, t, w)
        st = cpu_ref.structure_tensor3d(img, s, t, w, backend="restated")
        ovx, ovy, ovz = cpu_ref.solve3d(st)
        assert all(np.array_equal(a, b, equal_nan=True) for a, b in ((vx, ovx), (vy, ovy), (vz, ovz))), name
        lmin, lmax = cpu_ref.eig_fp64_3d(st)
        taps = cpu_ref.make_taps(s, t, w)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), images=img, params=np.array([s, t, w], float),
                            vx=vx, vy=vy, vz=vz, rel=rel, lmin64=lmin, lmax64=lmax,
                            **{"taps_" + k: v for k, v in taps.items()})
        manifest[name] = {"dims": 3, "shape": list(img.shape), "dtype": str(img.dtype), "params": [s, t, w],
                          "rel_dtype": str(rel.dtype)}
        print(name, img.shape, rel.dtype)
    for name, build, (s, t, w) in CASES_2D:
        if only and name not in only:
            continue
        img = build()
        with np.errstate(invalid="ignore"):
            vx, vy, rel = ref.calc_flow2D(img, s, t, w)
        taps = cpu_ref.make_taps(s, t, w)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), images=img, params=np.array([s, t, w], float),
                            vx=vx, vy=vy, rel=rel, **{"taps_" + k: v for k, v in taps.items()})
        manifest[name] = {"dims": 2, "shape": list(img.shape), "dtype": str(img.dtype), "params": [s, t, w],
                          "rel_dtype": str(rel.dtype)}
        print(name, img.shape, rel.dtype)
    if only:
        with open(mpath, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        return
    errors = {}
    for name, dims, shape, tsig in ERROR_CASES:
        fn = ref.calc_flow3D if dims == 3 else ref.calc_flow2D
        try:
            fn(np.zeros(shape, np.uint16), 1, tsig, 2)
            errors[name] = None
        except SystemExit as e:
            errors[name] = {"dims": dims, "shape": list(shape), "tSig": tsig, "message": str(e.code)}
    manifest["_errors"] = errors
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
