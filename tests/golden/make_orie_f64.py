"""Generate G5: the float64 ground truth of bench.py's ORIE leg (test/measurement fixture).

The ORIE leg (bench.py orie_vs_ref) runs 48 seeded synthetic 640x640 images (synthetic.make_batch,
seeds 7000..7047) through SSDLite (weak) and Faster R-CNN (strong) with seeded synthetic weights
(synthetic.synthetic_state_dict, seed 0).  This script runs the CPU oracle on the same inputs twice:
  * float64: every convolution / linear, BatchNorm, activation and SE of both detectors in float64
    (oracle dtype=torch.float64), the head outputs rounded to float32, then the reference's float32
    post-processing -- the "exact arithmetic" detector a float32 implementation
    approximates;
  * float32: the oracle as bench.py's CPU baseline runs it (this host's oneDNN blocking).
and stores both sets of detect.py files (detect.py:79-105 formatting, edgeml_amd.fmt) plus a checksum
of every input image, so a consumer can verify that it regenerated the same inputs.  The pseudo
ground-truth labels of the leg (the confident strong detections, conf >= 0.3) are taken from the
float64 strong files.

    python tests/golden/make_orie_f64.py [--n 48]        (about 6 minutes on 8 cores)

Writes tests/golden/g5_orie_f64.npz: for tag in (weak_f64, strong_f64, weak_f32, strong_f32):
<tag>_rows (sum N_i, 6) float64 and <tag>_count (n,) int64; image_sums (n,) float64 (the float64 sum
of each float32 input image); seeds (n,).
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

SEED0 = 7000  # bench.py orie_vs_ref: image i = synthetic.make_batch(1, 640, 640, seed=7000 + i)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=48)
    ap.add_argument("-o", default=os.path.join(ROOT, "tests", "golden", "g5_orie_f64.npz"))
    a = ap.parse_args()
    from edgeml_amd import fmt, synthetic
    from oracle.frcnn import FasterRCNNOracle
    from oracle.ssdlite import SSDLiteOracle
    torch.set_num_threads(os.cpu_count() or 1)
    sd_w, sd_s = synthetic.synthetic_state_dict("ssd", 91, True), synthetic.synthetic_state_dict("faster_rcnn", 91)
    models = {"weak_f64": SSDLiteOracle(sd_w, 91, True, dtype=torch.float64),
              "strong_f64": FasterRCNNOracle(sd_s, 91, dtype=torch.float64),
              "weak_f32": SSDLiteOracle(sd_w, 91, True), "strong_f32": FasterRCNNOracle(sd_s, 91)}
    rows = {k: [] for k in models}
    sums = []
    t0 = time.perf_counter()
    for i in range(a.n):
        img = synthetic.make_batch(1, 640, 640, seed=SEED0 + i)
        sums.append(float(img.double().sum()))
        for tag, m in models.items():
            p = m([img[0]])[0]
            rows[tag].append(fmt.format_detections(p["boxes"].numpy(), p["scores"].numpy(), p["labels"].numpy(),
                                                   640, 640))
        print(f"  image {i + 1}/{a.n} ({time.perf_counter() - t0:.0f} s)", flush=True)
    out = {"image_sums": np.asarray(sums), "seeds": SEED0 + np.arange(a.n)}
    for tag, rs in rows.items():
        out[tag + "_rows"] = np.concatenate([r.reshape(-1, 6) for r in rs], 0)
        out[tag + "_count"] = np.asarray([len(r) for r in rs], np.int64)
    np.savez_compressed(a.o, **out)
    print("wrote", a.o, {k: int(v.sum()) for k, v in out.items() if k.endswith("_count")})


if __name__ == "__main__":
    main()
