#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per kernel.

Reads gpurun_out/pmc_<cfg>_<tag>/p*/run_counter_collection.csv, averages every
counter per dispatch of each kernel, and derives HBM traffic per launch:

  read bytes  = FETCH_SIZE[KB] * 1024 * fetch_factor
  write bytes = WRITE_SIZE[KB] * 1024 * write_factor

fetch/write factors come from the calibration run (tools/calib_hbm.hip under
rocprofv3, profiles/pmc_calibration.json): on gfx950 FETCH_SIZE under-counts
wide coalesced reads by 2x (MI355X_MICROARCH.md, HBM); other widths are
calibrated on a known byte count with the same access width as our kernels.

Usage: python tools/pmc_summary.py <pmc_dir> <out_json> [--calib profiles/pmc_calibration.json]
"""

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[a-z0-9_]+)(<[^(]*>)?\(", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name[:60]


def main():
    pmc_dir, out = sys.argv[1], sys.argv[2]
    calib_path = None
    if "--calib" in sys.argv:
        calib_path = sys.argv[sys.argv.index("--calib") + 1]
    calib = {}
    if calib_path and os.path.exists(calib_path):
        calib = json.load(open(calib_path))
    fetch_factor = calib.get("fetch_factor_8B", 2.0)
    write_factor = calib.get("write_factor_8B", 1.0)
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if not k.startswith("k_"):
                    continue
                # one row per (dispatch, counter); the value is already summed over XCDs/instances
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    res = {}
    for k, counters in acc.items():
        d = {c: sum(v) / len(v) for c, v in counters.items()}
        e = {"counters": d, "profiled_ms": sum(dur[k]) / len(dur[k]),
             # dispatches of this kernel per profiled run (autotune candidates: 2; the kernel in use: steps)
             "dispatches": max(len(v) for v in counters.values())}
        if "FETCH_SIZE" in d:
            e["hbm_read_bytes"] = d["FETCH_SIZE"] * 1024 * fetch_factor
        if "WRITE_SIZE" in d:
            e["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024 * write_factor
        if "hbm_read_bytes" in e and "hbm_write_bytes" in e:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
            e["l2_hit_rate"] = d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        if "SQ_LDS_BANK_CONFLICT" in d and "SQ_LDS_IDX_ACTIVE" in d:
            e["lds_conflict_frac"] = d["SQ_LDS_BANK_CONFLICT"] / max(1.0, d["SQ_LDS_IDX_ACTIVE"])
        if "GRBM_GUI_ACTIVE" in d:
            e["clock_ghz_est"] = d["GRBM_GUI_ACTIVE"] / 8 / (e["profiled_ms"] * 1e6)
        res[k] = e
    summary = {"source": pmc_dir, "fetch_factor": fetch_factor, "write_factor": write_factor,
               "calibration": calib_path, "kernels": res}
    with open(out, "w") as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)
    for k, e in sorted(res.items()):
        c = e["counters"]
        print(f"{k:40s} ms={e['profiled_ms']:.4f} "
              + " ".join(f"{n}={c[n]:.4g}" for n in sorted(c)))
        for n in ("hbm_read_bytes", "hbm_write_bytes", "l2_hit_rate", "lds_conflict_frac", "clock_ghz_est"):
            if n in e:
                print(f"    {n} = {e[n]:.4g}")


if __name__ == "__main__":
    main()
