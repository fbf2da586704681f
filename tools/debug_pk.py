"""Debug: packed-fp32 K34 forced vs the older fp32 kernels; where do outputs differ?"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from test_gpu_kernel_families import CASES, _run  # noqa: E402

from opticalflow3d_dev_amd import _lib  # noqa: E402

for case in [int(a) for a in sys.argv[1:]] or [2]:
    shape, (s, t, w), ndim = CASES[case]
    img = np.random.default_rng(500 + case).integers(0, 4096, size=shape).astype(np.uint16)
    os.environ["OF3D_VERBOSE"] = "1"
    used = []
    new = _run(img, s, t, w, ndim, _lib.OF3D_FP32, old=False, force={"OF3D_K34_UQ": "3"}, kernels=used)
    ref = _run(img, s, t, w, ndim, _lib.OF3D_FP32, old=True)
    print("case", case, shape, (s, t, w), used, flush=True)
    vol = shape[1:]
    for name, a, b in zip("vx vy vz rel".split(), new, ref):
        a = a.reshape(vol)
        b = b.reshape(vol)
        bad = np.argwhere(a.view(np.uint32) != b.view(np.uint32))
        if len(bad) == 0:
            print(name, "ok")
            continue
        print(name, len(bad), "bad; z", np.unique(bad[:, 0])[:20], "y", np.unique(bad[:, 1])[:40],
              "x", np.unique(bad[:, 2])[:60], "xmax", bad[:, 2].max(), flush=True)
