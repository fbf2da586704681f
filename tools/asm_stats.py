"""Static instruction mix of one kernel in a device-assembly file (make asm UNIT=...).

    python tools/asm_stats.py opticalflow3d_dev_amd/csrc/kt_grad3-gfx950.s k_grad_xyz_cItdLi6ELi2E [--dump]

Counts per class (VALU fp64 / other VALU, SALU, LDS, VMEM, branches, waits) over the function body,
and the resource lines (VGPRs, SGPRs, LDS, scratch).  --dump prints the body."""
import re
import sys
from collections import Counter


def body(path, key):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l):
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i], lines[i:i + 120]
    raise SystemExit(f"{key}: not found in {path}")


def classify(op):
    if op.startswith("v_") and "f64" in op:
        return "valu_f64"
    if op.startswith(("v_mfma", "v_smfmac")):
        return "mfma"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier"):
        return "wait/barrier"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    return "other"


def main():
    path, key = sys.argv[1], sys.argv[2]
    b, tail = body(path, key)
    ops = Counter()
    names = Counter()
    for l in b:
        s = l.strip()
        if not s or s.startswith((";", ".", "_")) or s.endswith(":"):
            continue
        op = s.split()[0]
        ops[classify(op)] += 1
        names[op] += 1
    print(" ".join(f"{k}={v}" for k, v in sorted(ops.items())))
    print("top:", ", ".join(f"{k} {v}" for k, v in names.most_common(30)))
    for l in tail:
        if re.search(r"num_vgpr|numbered_sgpr|private_seg_size|group_segment|; (NumVgprs|Occupancy|ScratchSize|LDSByteSize)", l):
            print(l.strip())
    if "--dump" in sys.argv:
        print("\n".join(b))


if __name__ == "__main__":
    main()
