"""End-to-end time-series throughput: TIFF in -> TIFF out.

Writes a synthetic ImageJ OneTif hyperstack of a bench.py config with
Nt = 2*rt+1 + frames - 1 time points into --dir, then times:

  pcie    raw pinned<->device copy rate of one frame's output bytes
  host    FlowStream only: one H2D frame per output, compute, D2H to pinned host
          memory (the PCIe-inclusive rate of the device path, no file I/O)
  stream  process_flow (device ring + overlapped TIFF writer)
  legacy  the reference's loop structure: per output frame, load the whole
          window, calc_flow3D (upload all 2*rt+1 frames), write 4 TIFFs in line

Prints one JSON line per mode: output frames/s and Mvox/s (output voxels).
"""

import argparse
import contextlib
import io
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import CONFIGS, synthetic_frames  # noqa: E402
from opticalflow3d_dev_amd import calc_flow3D, process_flow, radii  # noqa: E402
from opticalflow3d_dev_amd import tiff as tf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=12, help="output frames")
    ap.add_argument("--modes", default="pcie,host,stream,legacy")
    ap.add_argument("--dir", default=None)
    ap.add_argument("--d2h", default="dma", help="comma list of FlowStream download modes (dma,kernel,runtime)")
    ap.add_argument("--d2h-blocks", type=int, default=64)
    ap.add_argument("--depth", type=int, default=None,
                    help="FlowStream output sets in flight (default 3; 1 for c5, whose workspace and ring take 215 GB)")
    ap.add_argument("--precision", default=None, choices=("fp64", "fp32"),
                    help="default: fp32 for c5 (configs[4]'s path), else fp64")
    args = ap.parse_args()
    nt0, nz, ny, nx, s, t, w, _ = CONFIGS[args.config]
    precision = args.precision or ("fp32" if args.config == "c5" else "fp64")
    rd, rs, rt, rw = radii(s, t, w)
    nwin = 2 * rt + 1
    nt = nwin + args.frames - 1
    root = tempfile.mkdtemp(dir=args.dir)
    try:
        nvox = nz * ny * nx
        t_gen = time.perf_counter()
        if nvox * nt * 2 <= (8 << 30):
            stack = synthetic_frames(nt, nz, ny, nx, seed=0)
            tf.imwrite(os.path.join(root, "series.tif"), stack, imagej=True)
            del stack
        else:  # large configs: frames generated on the device, written page range by page range
            import torch

            from bench import synthetic_slab
            for f in range(nt):
                fr = synthetic_slab(1, nz, ny, nx, 0, nz, 20260206 + 7 + f, torch.device("cuda", 0))
                tf.write_planes(os.path.join(root, "series.tif"), (nt, nz, ny, nx), np.uint16, f * nz,
                                fr[0].cpu().numpy().view(np.uint16), imagej=True)
                del fr
                print(f"# wrote frame {f + 1}/{nt} ({time.perf_counter() - t_gen:.1f} s)", flush=True)
            torch.cuda.empty_cache()
        print(json.dumps({"input": "series.tif", "frames_in": nt, "bytes": nvox * nt * 2,
                          "write_s": round(time.perf_counter() - t_gen, 2), "precision": precision}), flush=True)
        out_es = 4 if precision == "fp32" else 8
        modes = []
        for m in args.modes.split(","):
            modes += [f"host:{d}" for d in args.d2h.split(",")] if m == "host" else [m]
        for mode in modes:
            out_dir = os.path.join(root, "OpticalFlow3D")
            shutil.rmtree(out_dir, ignore_errors=True)
            t0 = time.perf_counter()
            extra = {}
            if mode == "pcie":
                import torch
                d = torch.empty(nvox * (3 * out_es + 4) // 8, dtype=torch.float64, device="cuda")
                h = torch.empty_like(d, device="cpu").pin_memory()
                for direction in ("d2h", "h2d"):
                    src, dst = (d, h) if direction == "d2h" else (h, d)
                    dst.copy_(src, non_blocking=True)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(10):
                        dst.copy_(src, non_blocking=True)
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                    print(json.dumps({"mode": "pcie_" + direction, "bytes": d.numel() * 8,
                                      "GB_per_s": round(10 * d.numel() * 8 / dt / 1e9, 2)}), flush=True)
                from opticalflow3d_dev_amd import _lib
                q = nvox * 8
                for nsplit in (1, 4):
                    parts = [q * (3 * out_es + 4) // 8 // nsplit] * nsplit
                    offs = [sum(parts[:i]) for i in range(nsplit)]
                    t0 = time.perf_counter()
                    for _ in range(10):
                        _lib.dma_copy([h.data_ptr() + o for o in offs], [d.data_ptr() + o for o in offs], parts)
                    dt = time.perf_counter() - t0
                    print(json.dumps({"mode": f"dma_d2h_x{nsplit}", "GB_per_s": round(10 * sum(parts) / dt / 1e9, 2)}),
                          flush=True)
                del d, h
                torch.cuda.empty_cache()
                continue
            if mode.startswith("host"):
                from opticalflow3d_dev_amd.stream import FlowStream
                mm = tf.memmap(os.path.join(root, "series.tif"))
                fs = FlowStream(3, (nz, ny, nx), np.uint16, s, t, w, d2h=mode.split(":")[1],
                                d2h_blocks=args.d2h_blocks, precision=precision,
                                depth=args.depth or (1 if args.config == "c5" else 3))
                split = {"push": 0.0, "submit": 0.0, "wait": 0.0}
                for rep in range(2):  # rep 0 warms the plan (module load, workspace)
                    t0 = time.perf_counter()
                    pend = []
                    done_t = []
                    for k in split:
                        split[k] = 0.0
                    for k in fs.stats:
                        fs.stats[k] = 0
                    tr = fs.trace = [] if rep == 1 and os.environ.get("E2E_TRACE") else None
                    fs.free += fs.order  # a fresh series (the previous rep's last frames retire)
                    fs.order = []
                    for i in range(nt):
                        ta = time.perf_counter()
                        fs.push(mm[i])
                        tb = time.perf_counter()
                        if tr is not None:
                            tr += [(ta, f"push{i}"), (tb, "pushed")]
                        split["push"] += tb - ta
                        # lookahead: submit once the next window's newest frame is resident too
                        # (frame pipelining); the last window goes without
                        while len(fs.order) >= fs.nwin + fs.L or (i == nt - 1 and fs.ready):
                            pend.append(fs.submit())
                            tc = time.perf_counter()
                            split["submit"] += tc - tb
                            if len(pend) == fs.depth:
                                p = pend.pop(0)
                                p.result()
                                p.release()
                                done_t.append(time.perf_counter())
                                split["wait"] += done_t[-1] - tc
                                if tr is not None:
                                    tr += [(tc, "submitted"), (time.perf_counter(), "waited")]
                    for p in pend:
                        p.result()
                        p.release()
                    dt = time.perf_counter() - t0
                fs.close()
                if tr:
                    tr.sort()
                    for tt, what in tr[-60:]:
                        print(f"{1e3 * (tt - tr[-60][0]):9.3f} {what}")
                extra = {k: round(1e3 * v / args.frames, 3) for k, v in split.items()}
                # steady state: median spacing of consecutive frame completions (no pipeline fill/drain)
                extra["steady_ms_per_frame"] = round(1e3 * float(np.median(np.diff(done_t))), 3)
                extra["steady_mvox_per_s"] = round(nvox / 1e3 / extra["steady_ms_per_frame"], 2)
                if fs.stats["dl_n"]:
                    extra.update({k: round(1e3 * v / fs.stats["dl_n"], 3) for k, v in fs.stats.items() if k != "dl_n"})
            elif mode == "stream":
                with contextlib.redirect_stdout(io.StringIO()):
                    process_flow(root, "series", "OneTif", 3, s, t, w, precision=precision)
                dt = time.perf_counter() - t0
            elif mode == "legacy":
                if precision != "fp64":
                    continue  # the reference's loop is the fp64 calc_flow3D
                mm = tf.memmap(os.path.join(root, "series.tif"))
                os.makedirs(out_dir, exist_ok=True)
                for hh in range(args.frames):
                    out = calc_flow3D(np.asarray(mm[hh:hh + nwin]), s, t, w)
                    for n, a in zip(("vx", "vy", "vz", "rel"), out):
                        tf.imwrite(os.path.join(out_dir, f"series_{n}_t{hh + rt:04d}.tiff"), a,
                                   photometric="minisblack")
                dt = time.perf_counter() - t0
            else:
                raise SystemExit("unknown mode " + mode)
            print(json.dumps({"mode": mode, "config": args.config, "frames": args.frames,
                              "ms_per_frame": round(1e3 * dt / args.frames, 3),
                              "frames_per_s": round(args.frames / dt, 3),
                              "mvox_per_s": round(args.frames * nvox / dt / 1e6, 2),
                              "out_bytes_per_frame": nvox * (3 * out_es + 4), "precision": precision, **extra}),
                  flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
