"""Measure every conv kernel variant on every conv layer of the detectors and record the fastest.

    python tools/tune_conv.py [--models ssd,frcnn,retinanet] [--out <package>/data/conv_tiles_gfx950.json]

Each CONV record of a lowered plan is launched alone on its own buffers (arena filled with N(0, 0.5)
values: timing on all-zero data would read high, MI355X_MICROARCH.md "DVFS") with every tile id the
library accepts for it (csrc/conv.hip conv_launch; variants that refuse the shape are skipped), HIP
events around the reps.  The table maps plan.conv_key(record) -> tile; plan.conv_op applies it, so
the choice is deterministic across runs (csrc/conv.hip choose_tile remains the fallback for shapes
not in the table).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CANDIDATES = (1, 2, 3, 4, 5, 6, 10, 11, 12, 13, 14, 15, 16, 17, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 38, 39)


def time_record(L, O, rec, stream, reps):
    ptr = rec.ctypes.data_as(ctypes.c_void_p)
    sh = O.stream_handle(stream)
    if L.edgedet_plan_run(ptr, 1, sh) != 0:
        return None
    with torch.cuda.stream(stream):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            L.edgedet_plan_run(ptr, 1, sh)
        e1.record(stream)
        e1.synchronize()
    return e0.elapsed_time(e1) / reps


def tune_plan(plan, table, stream, log, done):
    from edgeml_amd import ops as O
    from edgeml_amd.plan import conv_key
    L = O.lib()
    a = plan.arena
    a.view(torch.float32)[: a.numel() // 4].normal_(0.0, 0.5)
    recs = plan.records.copy()
    recs["i"][:, O.LANE_FIELD] = 0
    for k, op in enumerate(plan.ops):
        if op.kind != O.CONV:
            continue
        key = conv_key(op)
        if key in done:
            continue
        done.add(key)
        base = recs[k:k + 1].copy()
        base["i"][0, 23] = 0
        t0 = time_record(L, O, base, stream, 3)
        reps = int(min(50, max(3, 2.0 / max(t0, 1e-3))))
        best, res = None, {}
        for t in CANDIDATES:
            r = base.copy()
            r["i"][0, 23] = t
            ms = time_record(L, O, r, stream, 2)
            if ms is None:
                continue
            ms = time_record(L, O, r, stream, reps)
            res[t] = round(ms * 1000, 2)
            if best is None or ms < res[best] / 1000 - 1e-9:
                best = t
        torch.cuda.synchronize()
        auto = time_record(L, O, base, stream, reps)
        table[key] = best
        log.append({"op": op.name, "key": key, "best": best, "auto_us": round(auto * 1000, 2), "us": res})
        print(f"{op.name:48s} auto {auto * 1000:8.1f} us  best t{best} {res[best]:8.1f} us", flush=True)
    a.zero_()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="ssd,frcnn,retinanet")
    ap.add_argument("--out", default=os.path.join(ROOT, "edgeml-object-detection_amd", "data", "conv_tiles_gfx950.json"))
    a = ap.parse_args()
    from edgeml_amd import models, plan as plan_mod
    plan_mod.CONV_TILES.clear()  # measure the library's own choice as "auto"
    # re-tune the shapes of the given models, keep the other entries of the existing table
    table, log, done = {}, [], set()
    if os.path.exists(a.out):
        with open(a.out) as f:
            table.update(json.load(f).get("tiles", {}))
    stream = torch.cuda.Stream()
    for name in a.models.split(","):
        if name == "ssd":
            m = models.ssdlite320_mobilenet_v3_large().to("cuda")
            shapes = [(32, 640, 640), (16, 640, 640), (8, 640, 640), (1, 640, 640), (2, 640, 640)]
        elif name == "frcnn":
            m = models.fasterrcnn_resnet50_fpn_v2().to("cuda")
            shapes = [(8, 640, 640), (1, 640, 640)]
        else:
            m = models.retinanet_resnet50_fpn_v2().to("cuda")
            shapes = [(8, 640, 640), (1, 640, 640)]
        for B, H, W in shapes:
            print(f"== {name} B={B} {H}x{W}", flush=True)
            p = m.plan(B, H, W)
            tune_plan(p, table, stream, log, done)
            m.plans.clear()
            del p
            torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump({"arch": "gfx950", "tiles": table}, f, indent=0, sort_keys=True)
    with open(os.path.join(ROOT, "gpurun_out", "tune_log.json") if os.path.isdir(os.path.join(ROOT, "gpurun_out"))
              else os.devnull, "w") as f:
        json.dump(log, f)
    gain = sum(l["auto_us"] - l["us"][l["best"]] for l in log)
    print(f"{len(table)} shapes; summed per-launch gain {gain:.0f} us")


if __name__ == "__main__":
    main()
