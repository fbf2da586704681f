"""Calibrate the oracle's CPU speed against the reference's own calc_flow3D
(build container only — /root/reference does not exist on the GPU box).

bench.py's ``cpu_baseline`` times ``oracle/cpu_ref.calc_flow3D`` (scipy
correlate1d + numpy eigvals(complex64), the reference's primitives) on the GPU
box's host.  The oracle skips work the reference does: the reference applies
the temporal derivative to all Nt frames and slices the centre afterwards
(calc_flow.py:276-277).  This script times both, on one thread, on the same
inputs, and writes the ratio t_reference / t_oracle to
``profiles/cpu_calibration.json``; bench.py reports the oracle's rate divided
by that ratio as ``reference_equiv``.

The reference module is loaded as tests/golden/make_golden.py does (empty
stubs for the unused tifffile/natsort imports, source compiled from text).

Usage:  python tools/calibrate_cpu.py [--repeats 1]
"""

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

# workloads: (name, Nt, Nz, Ny, Nx, sig, tsig, wsig) — c3 is a z-subvolume of 16 of 128 planes;
# c1 (Nz 0: 2D) is the series of 16 frames, every output frame's 7-frame window (calc_flow2D)
CASES = [
    ("c1_series", 16, 0, 256, 256, 1, 1, 5),
    ("c2_full", 13, 64, 256, 256, 2, 2, 5),
    ("c3_z16", 19, 16, 512, 512, 2, 3, 7),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=1)
    ap.add_argument("--cases", default="", help="comma-separated case names (default: all); others kept")
    args = ap.parse_args()
    want = set(c for c in args.cases.split(",") if c)
    from threadpoolctl import threadpool_limits

    import bench
    from make_golden import load_reference
    from oracle import cpu_ref

    ref = load_reference()
    path = os.path.join(REPO, "profiles", "cpu_calibration.json")
    out = {"host": os.uname().nodename, "cpus": os.cpu_count(), "threads": 1, "cases": {}}
    if want and os.path.exists(path):
        with open(path) as f:
            out["cases"] = json.load(f)["cases"]
    with threadpool_limits(limits=1):
        for name, nt, nz, ny, nx, s, t, w in CASES:
            if want and name not in want:
                continue
            if nz == 0:  # 2D series: every output frame
                from opticalflow3d_dev_amd import radii

                nwin = 2 * radii(s, t, w)[2] + 1
                frames = bench.synthetic_frames(nt, 1, ny, nx, seed=20260206 + 1)[:, 0]
                tr, to = [], []
                for _ in range(args.repeats):
                    t0 = time.perf_counter()
                    rr = [ref.calc_flow2D(frames[k:k + nwin], s, t, w) for k in range(nt - nwin + 1)]
                    tr.append(time.perf_counter() - t0)
                    t0 = time.perf_counter()
                    oo = [cpu_ref.calc_flow2D(frames[k:k + nwin], s, t, w, backend="scipy") for k in range(nt - nwin + 1)]
                    to.append(time.perf_counter() - t0)
                for r, o in zip(rr, oo):
                    for a, b in zip(r, o):
                        assert np.array_equal(a, b, equal_nan=True), name
                vox = (nt - nwin + 1) * ny * nx
                out["cases"][name] = {"shape": [nt, ny, nx], "params": [s, t, w], "outputs": nt - nwin + 1,
                                      "reference_s": round(min(tr), 4), "oracle_s": round(min(to), 4),
                                      "ratio": round(min(tr) / min(to), 4),
                                      "reference_mvox_s": round(vox / min(tr) / 1e6, 4),
                                      "oracle_mvox_s": round(vox / min(to) / 1e6, 4)}
                print(name, out["cases"][name], flush=True)
                continue
            frames = bench.synthetic_frames(nt, nz, ny, nx, seed=20260206 + 2)
            tr, to = [], []
            for _ in range(args.repeats):
                t0 = time.perf_counter()
                r = ref.calc_flow3D(frames, s, t, w)
                tr.append(time.perf_counter() - t0)
                t0 = time.perf_counter()
                o = cpu_ref.calc_flow3D(frames, s, t, w, backend="scipy")
                to.append(time.perf_counter() - t0)
            for a, b in zip(r[:3], o[:3]):
                assert np.array_equal(a, b), name
            vox = nz * ny * nx
            out["cases"][name] = {"shape": [nt, nz, ny, nx], "params": [s, t, w],
                                  "reference_s": round(min(tr), 3), "oracle_s": round(min(to), 3),
                                  "ratio": round(min(tr) / min(to), 4),
                                  "reference_mvox_s": round(vox / min(tr) / 1e6, 4),
                                  "oracle_mvox_s": round(vox / min(to) / 1e6, 4)}
            print(name, out["cases"][name], flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
