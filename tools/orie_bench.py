"""Throughput of the GPU ORIE consumer at COCO-val scale (BASELINE config 4's reward.py step).

    python tools/orie_bench.py [--images 5000] [--ensemble 1000] [--weak-dets 300] [--strong-dets 100]
                               [--cpu-images 2]

Synthetic in-memory data of the detection-file shape (80 label classes, ~7 labels per image, weak
detector 300 rows per image as SSDLite's detections_per_img, strong 100 as Faster R-CNN's), TP flags
from the device box_correct.  Times the device AP evaluations of every image (2 x N ap_per_class
calls over E+1 images) and, for comparison, the CPU oracle's compute_orie (the reference's numpy
arithmetic) on --cpu-images images.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def synth(n, wd, sd, n_cls=80, seed=0):
    rng = np.random.default_rng(seed)
    labels, weak, strong = [], [], []
    for i in range(n):
        nl = int(rng.integers(0, 15))
        lab = (rng.integers(0, n_cls, nl), np.sort(rng.uniform(0, 1, (nl, 4)).reshape(nl, 2, 2), 1).reshape(nl, 4))
        labels.append(lab if nl else ())
        for out, nd in ((weak, wd), (strong, sd)):
            cls = rng.integers(0, n_cls, nd)
            box = np.sort(rng.uniform(0, 1, (nd, 4)).reshape(nd, 2, 2), 1).reshape(nd, 4)
            if nl:  # a share of detections near the labels
                k = rng.random(nd) < 0.3
                src = rng.integers(0, nl, nd)
                cls[k] = lab[0][src[k]]
                box[k] = lab[1][src[k]] + rng.normal(0, 0.01, (int(k.sum()), 4))
            conf = np.sort(rng.random(nd))[::-1]  # float64: distinct confidences (no tie-order ambiguity)
            out.append((cls, box, conf))
    return weak, strong, labels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=5000)
    ap.add_argument("--ensemble", type=int, default=1000)
    ap.add_argument("--weak-dets", type=int, default=300)
    ap.add_argument("--strong-dets", type=int, default=100)
    ap.add_argument("--cpu-images", type=int, default=2)
    a = ap.parse_args()
    from edgeml_amd import reward
    weak, strong, lab = synth(a.images, a.weak_dets, a.strong_dets)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    w_tp = reward.box_correct_batch(weak, lab)
    s_tp = reward.box_correct_batch(strong, lab)
    t_bc = time.perf_counter() - t0
    wd = [(t, w[2], w[0]) for t, w in zip(w_tp, weak)]
    sd = [(t, s[2], s[0]) for t, s in zip(s_tp, strong)]
    labels = [l[0] if len(l) else np.array([]) for l in lab]
    t0 = time.perf_counter()
    C, lab_cnt, ent_img, ent_flag, seg = reward._entries(wd, sd, labels)
    t_sort = time.perf_counter() - t0
    t0 = time.perf_counter()
    E, ens = reward.ensembles(len(labels), a.ensemble, 0)
    t_rng = time.perf_counter() - t0
    reward.orie_maps(wd, sd, labels, a.ensemble, 0, targets=np.arange(min(8, a.images)))  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    E, apv, nl = reward.orie_maps(wd, sd, labels, a.ensemble, 0)
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    res = {"images": a.images, "ensemble": E, "entries": int(len(ent_img)), "classes": int(C),
           "box_correct_s": round(t_bc, 3), "entry_sort_s": round(t_sort, 3), "ensemble_rng_s": round(t_rng, 3),
           "orie_maps_s": round(t_all, 3), "images_per_s": round(a.images / t_all, 1)}
    if a.cpu_images:
        from oracle import orie
        import warnings
        warnings.filterwarnings("ignore")
        t0 = time.perf_counter()
        for i in range(a.cpu_images):
            np.random.seed(i)
            orie.compute_orie(i, wd, sd, labels, a.ensemble)
        t_cpu = (time.perf_counter() - t0) / a.cpu_images
        res["cpu_oracle_s_per_image"] = round(t_cpu, 3)
        res["cpu_images_per_s"] = round(1 / t_cpu, 3)
        got = reward.orie_from_maps(E, apv[:a.cpu_images], nl[:a.cpu_images])
        ref = []
        for i in range(a.cpu_images):
            np.random.seed(0 + i)
            ref.append(orie.compute_orie(i, wd, sd, labels, a.ensemble))
        res["max_abs_diff_vs_oracle"] = float(np.max(np.abs(np.nan_to_num(np.array(ref)) - got)))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
