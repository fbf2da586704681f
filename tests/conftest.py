import glob
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libof3d.so on the device)")


def _gpu_count():
    try:
        from opticalflow3d_dev_amd import _lib
        return _lib.load().of3d_device_count()
    except Exception:
        return 0


def pytest_collection_modifyitems(config, items):
    if any("gpu" in item.keywords for item in items):
        if _gpu_count() == 0:
            skip = pytest.mark.skip(reason="no HIP device visible")
            for item in items:
                if "gpu" in item.keywords:
                    item.add_marker(skip)


def golden_cases(prefix=""):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    out = {k: d[k] for k in d.files}
    s, t, w = (float(v) for v in out["params"])
    norm = lambda v: int(v) if v == int(v) else v
    out["sig"], out["tsig"], out["wsig"] = norm(s), norm(t), norm(w)
    out["taps"] = {k[5:]: out[k] for k in out if k.startswith("taps_")}
    return out


def golden_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))
