"""BASELINE configs[3] at full size on one GPU: 5,000 synthetic COCO-sized JPEG images through
edgeml_amd.pipeline (SSDLite weak + FRCNN strong detection files, then ORIE with E = 1,000, as
README.md:57 runs reward.py), timed per stage; then ORIE parity on a subset against the CPU oracle
pipeline (oracle forwards -> detect.py formatting -> oracle consumer).

    python tools/config4_full.py [--n 5000] [--num-ensemble 1000] [--subset 200] [--work DIR]

The subset check uses pseudo ground truth (the oracle strong detector's confident boxes, so the
ensemble mAPs are non-trivial) for both sides, E = subset - 1, seeded serial ensembles.
"""
import argparse
import concurrent.futures as cf
import os
import sys
import tempfile
import time
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
warnings.filterwarnings("ignore")

import numpy as np  # noqa: E402


def _make(args):
    """Write images [lo, hi) of the seeded synthetic set (same content as synthetic.make_dataset)."""
    from PIL import Image
    from edgeml_amd import synthetic
    img_dir, lab_dir, lo, hi, seed = args
    rs = np.random.RandomState(seed)
    sizes = [synthetic.COCO_SIZES[rs.randint(len(synthetic.COCO_SIZES))] for _ in range(hi)]
    for i in range(lo, hi):
        h, w = sizes[i]
        img, boxes = synthetic.make_scene(seed * 100003 + i, h, w, return_boxes=True)
        name = f"{i:012d}"
        Image.fromarray(img.transpose(1, 2, 0)).save(os.path.join(img_dir, name + ".jpg"), quality=90)
        with open(os.path.join(lab_dir, name + ".txt"), "w") as f:
            for b in boxes:
                f.write(" ".join(str(v) for v in b) + "\n")
    return hi - lo


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=5000)
    ap.add_argument("--num-ensemble", type=int, default=1000)
    ap.add_argument("--subset", type=int, default=200)
    ap.add_argument("--work", default="")
    a = ap.parse_args()
    td = a.work or tempfile.mkdtemp()
    img, lab, work = (os.path.join(td, d) for d in ("imgs", "labels", "work"))
    os.makedirs(img, exist_ok=True)
    os.makedirs(lab, exist_ok=True)
    from edgeml_amd.distributed import usable_cpus
    t0 = time.perf_counter()
    step = 250
    with cf.ProcessPoolExecutor(min(16, usable_cpus())) as ex:
        done = 0
        for k in ex.map(_make, [(img, lab, lo, min(lo + step, a.n), 1) for lo in range(0, a.n, step)]):
            done += k
            print(f"  wrote {done}/{a.n} images", flush=True)
    print(f"wrote {a.n} synthetic COCO-sized JPEG images in {time.perf_counter() - t0:.1f} s", flush=True)

    import torch
    from edgeml_amd import pipeline
    t0 = time.perf_counter()
    pipeline.main(pipeline.getargs([img, lab, work, "--num-ensemble", str(a.num_ensemble)]))
    el = time.perf_counter() - t0
    print(f"config 4 pipeline, {a.n} images, E={a.num_ensemble}: {el:.1f} s end to end "
          f"({a.n / el:.1f} images/s incl. JPEG decode, files and ORIE)", flush=True)
    with np.load(os.path.join(work, "reward", f"orie{a.num_ensemble}.npz")) as z:
        r = z["reward"]
    print(f"ORIE over {len(r)} images: {np.count_nonzero(r)} nonzero, finite {bool(np.all(np.isfinite(r)))}",
          flush=True)

    # ---- ORIE parity on a subset: engine files (from the run above) vs the oracle pipeline
    if a.subset <= 0:
        return
    from edgeml_amd import detect, fmt, reward, synthetic
    from oracle import orie
    from oracle.frcnn import FasterRCNNOracle
    from oracle.ssdlite import SSDLiteOracle
    torch.set_num_threads(usable_cpus())
    names = sorted(os.listdir(img))[:a.subset]
    sub = {k: os.path.join(td, "subset", k) for k in ("weak_g", "strong_g", "weak_o", "strong_o", "labels", "out")}
    for d in sub.values():
        os.makedirs(d, exist_ok=True)
    oracles = {"weak_o": SSDLiteOracle(synthetic.synthetic_state_dict("ssd", 91, True), 91, True),
               "strong_o": FasterRCNNOracle(synthetic.synthetic_state_dict("faster_rcnn", 91), 91)}
    t0 = time.perf_counter()
    for j, name in enumerate(names):
        stem = name[:-4]
        for tag, src in (("weak_g", "weak"), ("strong_g", "strong")):
            os.link(os.path.join(work, src, stem + ".npy"), os.path.join(sub[tag], stem + ".npy"))
        im = detect.read_image(os.path.join(img, name)) / 255
        for tag, model in oracles.items():
            p = model([im])[0]
            rows = fmt.format_detections(p["boxes"].numpy(), p["scores"].numpy(), p["labels"].numpy(),
                                         int(im.shape[-2]), int(im.shape[-1]))
            fmt.save_npy(sub[tag], name, rows)
            if tag == "strong_o":
                with open(os.path.join(sub["labels"], stem + ".txt"), "w") as f:
                    for r_ in rows[rows[:, 5] >= 0.3]:
                        f.write(" ".join([str(int(r_[0]))] + [repr(float(v)) for v in r_[1:5]]) + "\n")
        if (j + 1) % 20 == 0:
            print(f"  oracle pipeline {j + 1}/{len(names)} images ({time.perf_counter() - t0:.0f} s)", flush=True)
    E = len(names) - 1
    reward.main(reward.getargs([sub["weak_g"], sub["strong_g"], sub["labels"], sub["out"], "--num-ensemble", str(E),
                                "--seed", "1000"]))
    with np.load(os.path.join(sub["out"], f"orie{E}.npz")) as z:
        got = z["reward"]
    ref = orie.orie_all(sub["weak_o"], sub["strong_o"], sub["labels"], E, seed=1000)
    d = np.abs(got - ref)
    print(f"ORIE subset parity: {len(names)} images, E={E}: max |dORIE| = {d.max():.3e}, "
          f"{int(np.count_nonzero(d))} images differ, {int(np.count_nonzero(ref))} nonzero oracle ORIE", flush=True)
    # identity-paired file differences (rows paired by class and IoU >= 0.99, tools/rowpair.py)
    from tools import rowpair
    stems = [n[:-4] for n in names]
    for det in ("weak", "strong"):
        r = rowpair.compare_dirs(stems, lambda s_: np.load(os.path.join(sub[det + "_g"], s_ + ".npy")),
                                 lambda s_: np.load(os.path.join(sub[det + "_o"], s_ + ".npy")))
        print(f"{det} files engine vs oracle: {r}", flush=True)


if __name__ == "__main__":
    main()
