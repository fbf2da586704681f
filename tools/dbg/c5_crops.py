"""Diagnostic: c5 full volume (fp32) oracle crops in several series modes (prints a summary per crop)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import test_gpu_full_configs as T
import bench

mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
kb, pipe = {"plain": (0, False), "batch": (5, True), "pipe": (0, True)}[mode]
t0 = time.time()
sb = T._slab(T.C5, fp32=True, seed=20260206 + 5, k0_batch=kb, pipeline=pipe)
print("setup", round(time.time() - t0, 1), "s", bench.device_used_gb(sb.dev), flush=True)
T._run_steps(sb, int(os.environ.get("NSTEP", "2")))
print("kernels", sb.plan.kernels(), "window", sb.last_window, flush=True)
for box in [(248, 264, 1016, 1032, 1016, 1032), (248, 264, 1016, 1032, 1068, 1084), (100, 116, 1016, 1032, 1016, 1032),
            (248, 264, 100, 116, 100, 116), (0, 16, 0, 16, 0, 16), (300, 316, 1500, 1516, 1016, 1032)]:
    try:
        r = T._check(sb, box, True)
        print(box, "ok", r["rel_max_err_over_lmax"], flush=True)
    except AssertionError as e:
        r = e.args[0][1] if e.args and isinstance(e.args[0], tuple) else {}
        print(box, "FAIL", {k: r.get(k) for k in ("n_mismatch", "max_abs_diff_over_max", "rel_max_err_over_lmax")},
              "planes", r.get("mismatch_planes", [])[:20], flush=True)
sb.close()
