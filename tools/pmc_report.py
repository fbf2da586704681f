#!/usr/bin/env python3
"""One line per kernel from a tools/pmc_summary.py JSON: per-voxel instruction
mix, fp64 VALU utilisation against the measured add/mul peak, HBM bytes."""
import json
import sys

FP64_PEAK = 33.2e12  # profiles/pmc_calibration.json (measured)
d = json.load(open(sys.argv[1]))["kernels"]
vox = float(sys.argv[2]) if len(sys.argv) > 2 else 64 * 256 * 256
for k, e in sorted(d.items()):
    c = e["counters"]
    g = lambda n: c.get(n, float("nan"))
    t = e["profiled_ms"] * 1e-3
    f64 = (g("SQ_INSTS_VALU_ADD_F64") + g("SQ_INSTS_VALU_MUL_F64") + g("SQ_INSTS_VALU_FMA_F64")) * 64
    print(f"{k:26s} ms={e['profiled_ms']:.3f} f64/vox={f64/vox:6.0f} VALU/vox={g('SQ_INSTS_VALU')*64/vox:6.0f} "
          f"int/vox={(g('SQ_INSTS_VALU_INT32')+g('SQ_INSTS_VALU_INT64'))*64/vox:5.0f} LDS/vox={g('SQ_INSTS_LDS')*64/vox:5.0f} "
          f"SALU/vox={g('SQ_INSTS_SALU')*64/vox:5.0f} f64util={f64/t/FP64_PEAK:.2f} "
          f"wait={g('SQ_WAIT_ANY')/g('SQ_WAVE_CYCLES'):.2f} waitinst={g('SQ_WAIT_INST_ANY')/g('SQ_WAVE_CYCLES'):.2f} "
          f"valuact={g('SQ_ACTIVE_INST_VALU')*4/g('SQ_WAVE_CYCLES'):.2f} waves={g('SQ_WAVES'):.0f} "
          f"rdB/vox={e.get('hbm_read_bytes',0)/vox:.0f} wrB/vox={e.get('hbm_write_bytes',0)/vox:.0f} l2hit={e.get('l2_hit_rate',0):.2f}")
