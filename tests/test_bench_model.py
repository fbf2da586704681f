"""bench.py's roofline bookkeeping on the CPU: stage model, kernel-family attribution of the
committed PMC summaries, and the fused (frame-pipelined) solve stage."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_kernel_family_pipelined_solve():
    assert bench.kernel_family("k_wz_solve_c<double, double, 21, 2, 8, 4, 9, unsigned short>") == "k_wz_solve_c_next"
    assert bench.kernel_family("k_wz_solve_c<double, double, 21, 2, 8, 4, 0, unsigned short>") == "k_wz_solve_c"
    assert bench.kernel_family("k_wz_solve_c<float, float, 15, 3, 8, 4>") == "k_wz_solve_c"
    assert bench.kernel_family("k_prod_wyx_ws<double, 9, 21, 4, 2, 2>") == "k_prod_wyx_ws"
    assert bench.kernel_family("k_tderiv_vec_c") == "k_tderiv_vec_c"
    assert "k_wz_solve_c_next" in bench.PLAN_FAMILIES


def test_pmc_traffic_attribution(tmp_path, monkeypatch):
    """A plain-solve PMC record is not reported as the fused kernel's traffic, and the series'
    first (plain) solve does not add to the fused one."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    ks = {"k_wz_solve_c<double, double, 21, 2, 8, 4>": {"dispatches": 5, "hbm_bytes_per_launch": 100.0},
          "k_tderiv_vec_c<unsigned short, double, 9>": {"dispatches": 5, "hbm_bytes_per_launch": 7.0}}
    (prof / "pmc_cx.json").write_text(json.dumps({"kernels": ks}))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.load_pmc_traffic("wz_solve", "cx", {"k_wz_solve_c"}) == 100
    assert bench.load_pmc_traffic("wz_solve", "cx", {"k_wz_solve_c", "k_wz_solve_c_next"}) is None
    ks["k_wz_solve_c<double, double, 21, 2, 8, 4, 9, unsigned short>"] = {"dispatches": 4,
                                                                          "hbm_bytes_per_launch": 140.0}
    (prof / "pmc_cx.json").write_text(json.dumps({"kernels": ks}))
    assert bench.load_pmc_traffic("wz_solve", "cx", {"k_wz_solve_c", "k_wz_solve_c_next"}) == 140
    assert bench.load_pmc_traffic("grad_xy", "cx", {"k_tderiv_vec_c"}) == 7


@pytest.mark.parametrize("sv", [8, 4])
def test_fused_solve_roofline_adds_k0(sv):
    rd, rs, rt, rw = 6, 2, 9, 21
    nwin, plane, n = 2 * rt + 1, 512 * 512, 128
    model = bench.stage_model(nwin, rd, rs, rt, rw, n, n, n, plane, sv)
    prof = {"grad_xy": 0.005, "grad_z": 0.6, "wz_solve": 1.3, "prod_wy_wx": 1.2}
    plain = bench.roofline(prof, "wz_solve", 1.3, model, "cx", 1, 1, nwin, sv, used={"k_wz_solve_c"})
    fused = bench.roofline(prof, "wz_solve", 1.3, model, "cx", 1, 1, nwin, sv,
                           used={"k_wz_solve_c", "k_wz_solve_c_next"})
    k0 = model["tderiv_next"]
    assert k0["bytes"] == (nwin * 2 + sv) * n * plane and k0["ops"] == (1 + 3 * rt) * n * plane
    assert fused["algorithmic_ops_per_launch"] == plain["algorithmic_ops_per_launch"] + k0["ops"]
    assert (fused["kernel_hbm"]["workspace_bytes_per_launch"]
            == plain["kernel_hbm"]["workspace_bytes_per_launch"] + k0["bytes"])
    # the model dict the caller holds is not modified
    assert model["wz_solve"]["ops"] == plain["algorithmic_ops_per_launch"]


def test_default_config_per_gpu_count():
    """--gpus N without --config runs the volume BASELINE.json names for N GPUs."""
    assert bench.default_config(1) == "c3"
    assert bench.default_config(2) == "c4" and bench.default_config(4) == "c4"
    assert bench.default_config(8) == "c5"
    assert bench.CONFIGS["c4"][:4] == (13, 256, 1024, 1024) and bench.CONFIGS["c5"][:4] == (13, 512, 2048, 2048)


@pytest.mark.parametrize("cfg,world,axis", [("c4", 2, 0), ("c4", 4, 0), ("c5", 8, 0), ("c4", 2, 1), ("c5", 8, 1),
                                            ("c3", 1, 0)])
def test_parity_box_straddles_the_first_cut(cfg, world, axis):
    """The slab parity crop holds planes (rows) of rank 0 AND rank 1 — both sides of the first
    cut — and lies inside the volume."""
    from opticalflow3d_dev_amd.shard import zslab_bounds

    nt, nz, ny, nx = bench.CONFIGS[cfg][:4]
    dims = (nz, ny, nx)
    cut = zslab_bounds(dims[axis], 0, world)[1] if world > 1 else dims[axis] // 2
    box = bench.parity_box(dims, axis, cut)
    for d in range(3):
        assert 0 <= box[2 * d] < box[2 * d + 1] <= dims[d] and box[2 * d + 1] - box[2 * d] == 16
    lo, hi = box[2 * axis], box[2 * axis + 1]
    assert lo < cut < hi
