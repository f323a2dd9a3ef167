"""Generate the BatchNorm calibration tables used by edgeml_amd.synthetic (test/dev tool).

For each synthetic model variant: draw the seeded weights uncalibrated, run the CPU oracle forward
on a few seeded synthetic scenes, and at every BatchNorm set running_mean/running_var to the
per-channel statistics of that BN's actual input (layer by layer, so every BN sees the output of
already-calibrated layers).  Writes edgeml-object-detection_amd/data/calib_<variant>.npz.

    python tests/golden/make_calibration.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import edgeml_amd.synthetic as syn  # noqa: E402
from oracle.frcnn import FasterRCNNOracle  # noqa: E402
from oracle.ssdlite import SSDLiteOracle  # noqa: E402


def calibrate(kind, num_classes=91, reduced_tail=True, n_img=8, size=640):
    sd = syn.synthetic_state_dict(kind, num_classes, reduced_tail, calibrated=False)
    if kind == "ssd":
        model = SSDLiteOracle(sd, num_classes, reduced_tail)
    else:
        model = FasterRCNNOracle(sd, num_classes)
    stats = {}

    def hook(prefix, x):
        if prefix.startswith("__"):
            return
        m = x.mean(dim=(0, 2, 3))
        v = x.var(dim=(0, 2, 3), unbiased=False).clamp_min(1e-4)
        model.sd[prefix + ".running_mean"] = m
        model.sd[prefix + ".running_var"] = v
        stats[prefix + ".running_mean"] = m.numpy().astype(np.float32)
        stats[prefix + ".running_var"] = v.numpy().astype(np.float32)

    imgs = syn.make_batch(n_img, size, size, seed=7000)
    torch.manual_seed(0)
    model.forward_raw(list(imgs), hook=hook)
    path = syn.calib_path(kind, num_classes, reduced_tail)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    np.savez_compressed(path, **stats)
    print(f"wrote {path}: {len(stats) // 2} BatchNorm layers")


if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count())
    calibrate("ssd", 91, True)
    calibrate("ssd", 91, False)
    calibrate("faster_rcnn", 91, n_img=6)
