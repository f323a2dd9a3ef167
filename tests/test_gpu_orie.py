"""End-to-end parity in the consumer's space: detection files -> reward.py ORIE (north_star).

A small synthetic COCO-like set (mixed sizes) runs through the HIP engine (SSDLite weak, FRCNN
strong) and through the CPU oracle; both write detect.py-format .npy files; ORIE is computed from
each set with the reference's consumer restated in oracle/orie.py (serial, seeded harness).
Labels are pseudo ground truth (the oracle strong detector's confident boxes) so that the ensemble
mAPs are non-trivial.  Target: identical ORIE (max |dORIE| == 0).
"""
import os
import tempfile
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [(640, 640), (640, 640), (640, 640), (480, 640), (480, 640), (427, 640), (612, 612), (640, 480)]


def _write(dirpath, name, rows):
    from edgeml_amd import fmt
    os.makedirs(dirpath, exist_ok=True)
    fmt.save_npy(dirpath, name, rows)


def test_orie_identical_from_engine_and_oracle():
    from edgeml_amd import fmt, models, synthetic
    from oracle import orie
    from oracle.frcnn import FasterRCNNOracle
    from oracle.ssdlite import SSDLiteOracle
    warnings.filterwarnings("ignore")
    sd_w = synthetic.synthetic_state_dict("ssd", 91, True, seed=0)
    sd_s = synthetic.synthetic_state_dict("faster_rcnn", 91, seed=0)
    weak_g, strong_g = models.SSDLite320(sd_w, 91, True).to("cuda"), models.FasterRCNNFPNv2(sd_s, 91).to("cuda")
    weak_o, strong_o = SSDLiteOracle(sd_w, 91, True), FasterRCNNOracle(sd_s, 91)
    worst = 0.0
    with tempfile.TemporaryDirectory() as td:
        for i, (h, w) in enumerate(SIZES):
            name = f"{i:012d}.png"
            img = torch.from_numpy(synthetic.make_scene(500 + i, h, w)).float() / 255
            for tag, model in (("weak_g", weak_g), ("strong_g", strong_g)):
                p = model(img[None].cuda())[0]
                rows = fmt.format_detections(p["boxes"].cpu().numpy(), p["scores"].cpu().numpy(),
                                             p["labels"].cpu().numpy(), h, w)
                _write(os.path.join(td, tag), name, rows)
            for tag, model in (("weak_o", weak_o), ("strong_o", strong_o)):
                p = model([img])[0]
                rows = fmt.format_detections(p["boxes"].numpy(), p["scores"].numpy(), p["labels"].numpy(), h, w)
                _write(os.path.join(td, tag), name, rows)
                if tag == "strong_o":
                    gt = rows[rows[:, 5] >= 0.3][:, :5]
                    os.makedirs(os.path.join(td, "labels"), exist_ok=True)
                    with open(os.path.join(td, "labels", name[:-4] + ".txt"), "w") as f:
                        for r in gt:
                            f.write(" ".join([str(int(r[0]))] + [repr(float(v)) for v in r[1:]]) + "\n")
            for a, b in (("weak_g", "weak_o"), ("strong_g", "strong_o")):
                x = np.load(os.path.join(td, a, name[:-4] + ".npy"))
                y = np.load(os.path.join(td, b, name[:-4] + ".npy"))
                print(name, a, x.shape, y.shape)
        L = os.path.join(td, "labels")
        for E in (0, 3, len(SIZES) - 1):
            og = orie.orie_all(os.path.join(td, "weak_g"), os.path.join(td, "strong_g"), L, E)
            oo = orie.orie_all(os.path.join(td, "weak_o"), os.path.join(td, "strong_o"), L, E)
            d = float(np.abs(og - oo).max())
            worst = max(worst, d)
            print(f"E={E} ORIE engine {np.round(og, 4)} oracle {np.round(oo, 4)} max|d|={d}")
            assert np.any(oo != 0)
    assert worst <= 1e-9, worst
