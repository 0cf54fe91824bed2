"""Per-kernel-class time of one configuration on ONE stream (option streams = 1), so each
class's launch time is its own and the classes add up to the step:

    python scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 [--batch 256] [--opt key=value ...]

Prints one JSON line {class: {launches_per_step, avg_ms, ms_per_step}} (bench.py's workload
builder and event-timed profile classes; development tool, not part of the bench contract)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default=bench.HUBERT_ARCH)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--x3-variant", type=int, default=None)
    a = ap.parse_args()
    sys.argv = [sys.argv[0]] + (["--x3-variant", str(a.x3_variant)] if a.x3_variant is not None else []) + \
        sum((["--opt", o] for o in a.opt), [])
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    resnet_like = a.arch.startswith("ResNet") or a.arch.startswith("SimAM")
    B = a.batch or (128 if resnet_like else 256)
    w = bench.build_workload(args, a.arch, B, 0, dev)
    handles = [h for h in (w.get("fe"), w["model"]) if h is not None]
    tags = bench.HEAD_TAGS + bench.HUBERT_TAGS + tuple(f"h_cnn.c{i}" for i in range(1, 7)) + \
        tuple(f"res_tail.L{i}" for i in range(1, 5))
    out = {}
    for h in handles:
        r = bench.standalone_pass(w, h, tags, steps=a.steps)
        for k, v in r.items():
            out[k] = {"launches_per_step": v["launches_per_step"], "avg_ms": round(v["avg_ms"], 4),
                      "ms_per_step": round(v["avg_ms"] * v["launches_per_step"], 4)}
    print(json.dumps({"arch": a.arch, "batch": B, "streams": 1, "classes": out}), flush=True)


if __name__ == "__main__":
    main()
