"""Generate golden fixtures by running the REFERENCE's own code (read-only, from /root/reference).

Run here (not on the GPU box — /root/reference does not travel):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

G1 (formatting, torch_models/detect.py:62-105): detect.main() is driven with a stub torchvision
   (read_image returns a tensor of the requested size, the detector ctor returns a fake model that
   replays seeded predictions).  The exact .npy bytes it writes are stored.
G2 (consumer, reward.py + lib/data.py + lib/metrics.py): synthetic weak/strong/label directories are
   fed to set_data(); box_iou / box_correct / ap_per_class / compute_ap / compute_orie (serial,
   np.random.seed(k) before each call) / compute_dcsb outputs are stored.
G3 (other consumers, on the G2 inputs): test.py test_map with a seeded 3-fold split and two
   synthetic estimate directories; lib/data.py extract_output_feature(k=25, 80 classes).

Only data (inputs and the reference's outputs) is written: tests/golden/g1_format.npz and
tests/golden/g2_orie.npz (+ the synthetic input directories packed into g2_inputs.npz).
"""
import io
import os
import sys
import tempfile
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True


# ------------------------------------------------------------------ stub torchvision
def install_stub(fake_preds, img_sizes):
    tv = types.ModuleType("torchvision")
    tv_io = types.ModuleType("torchvision.io")
    tv_ops = types.ModuleType("torchvision.ops")
    tv_models = types.ModuleType("torchvision.models")
    tv_det = types.ModuleType("torchvision.models.detection")
    tv_fr = types.ModuleType("torchvision.models.detection.faster_rcnn")
    tv_rn = types.ModuleType("torchvision.models.detection.retinanet")

    class ImageReadMode:
        RGB = "RGB"

    def read_image(path, mode=None):
        h, w = img_sizes[os.path.basename(path)]
        return torch.zeros((3, h, w), dtype=torch.uint8)

    class FakeModel(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.i = 0

        def forward(self, img):
            p = fake_preds[self.i]
            self.i += 1
            return [{"boxes": torch.from_numpy(p["boxes"]), "scores": torch.from_numpy(p["scores"]),
                     "labels": torch.from_numpy(p["labels"])}]

    def ctor(**kw):
        return FakeModel()

    tv_io.read_image = read_image
    tv_io.ImageReadMode = ImageReadMode
    tv_ops.roi_align = tv_ops.roi_pool = None
    tv_det.ssdlite320_mobilenet_v3_large = ctor
    tv_fr.fasterrcnn_resnet50_fpn_v2 = ctor
    tv_rn.retinanet_resnet50_fpn_v2 = ctor
    tv_det.faster_rcnn = tv_fr
    tv_det.retinanet = tv_rn
    tv_models.detection = tv_det
    tv.io, tv.ops, tv.models = tv_io, tv_ops, tv_models
    for name, mod in [("torchvision", tv), ("torchvision.io", tv_io), ("torchvision.ops", tv_ops),
                      ("torchvision.models", tv_models), ("torchvision.models.detection", tv_det),
                      ("torchvision.models.detection.faster_rcnn", tv_fr),
                      ("torchvision.models.detection.retinanet", tv_rn)]:
        sys.modules[name] = mod


def random_preds(rs, n, h, w, num_classes):
    x1 = rs.uniform(0, w * 0.9, n).astype(np.float32)
    y1 = rs.uniform(0, h * 0.9, n).astype(np.float32)
    x2 = np.minimum(x1 + rs.uniform(1, w * 0.5, n).astype(np.float32), np.float32(w))
    y2 = np.minimum(y1 + rs.uniform(1, h * 0.5, n).astype(np.float32), np.float32(h))
    scores = np.sort(rs.uniform(0.001, 1, n).astype(np.float32))[::-1].copy()
    labels = rs.randint(1, num_classes, n).astype(np.int64)
    return {"boxes": np.stack([x1, y1, x2, y2], 1).astype(np.float32), "scores": scores, "labels": labels}


def make_g1():
    rs = np.random.RandomState(0)
    cases = []
    # (dataset, name, H, W, n_dets)
    spec = [("coco", "000000000001.jpg", 480, 640, 300), ("coco", "000000000002.jpg", 640, 427, 57),
            ("coco", "000000000003.jpg", 612, 612, 0), ("coco", "000000000004.jpg", 333, 500, 91),
            ("voc", "000005.jpg", 375, 500, 40), ("voc", "000006.jpg", 500, 353, 0)]
    out = {}
    for ds in ("coco", "voc"):
        items = [s for s in spec if s[0] == ds]
        preds, sizes = [], {}
        for _, name, h, w, n in items:
            p = random_preds(rs, n, h, w, 91 if ds == "coco" else 21)
            if ds == "coco" and n == 91:          # cover every COCO id incl. the 11 dropped ones
                p["labels"] = np.arange(91, dtype=np.int64)
            preds.append(p)
            sizes[name] = (h, w)
        # detect.py:92 decrements the label array in place (`labels -= 1` on a numpy view of the
        # model's tensor), so keep pristine copies of the inputs for the fixture
        orig = {name[:-4]: {k: v.copy() for k, v in p.items()} for (_, name, h, w, n), p in zip(items, preds)}
        install_stub(preds, sizes)
        for m in list(sys.modules):
            if m in ("detect", "coco_labelmap"):
                del sys.modules[m]
        sys.path.insert(0, os.path.join(REF, "torch_models"))
        import detect  # reference torch_models/detect.py
        sys.path.pop(0)
        with tempfile.TemporaryDirectory() as td:
            img_dir, save_dir = os.path.join(td, "img"), os.path.join(td, "out")
            os.makedirs(img_dir)
            for _, name, h, w, n in items:
                open(os.path.join(img_dir, name), "wb").close()
            opts = types.SimpleNamespace(img_dir=img_dir, save_dir=save_dir, dataset=ds, model="ssd",
                                         model_path="")
            detect.main(opts)
            for (_, name, h, w, n), p in zip(items, preds):
                key = name[:-4]
                with open(os.path.join(save_dir, key + ".npy"), "rb") as f:
                    raw = f.read()
                out[f"{ds}/{key}/boxes"] = orig[key]["boxes"]
                out[f"{ds}/{key}/scores"] = orig[key]["scores"]
                out[f"{ds}/{key}/labels"] = orig[key]["labels"]
                out[f"{ds}/{key}/hw"] = np.array([h, w], dtype=np.int64)
                out[f"{ds}/{key}/npy_bytes"] = np.frombuffer(raw, dtype=np.uint8)
    import coco_labelmap
    out["coco_to_yolov5"] = np.array([coco_labelmap.coco_to_yolov5[i] for i in range(91)], dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "g1_format.npz"), **out)
    print("G1:", len(out), "arrays")


# ------------------------------------------------------------------ G2 consumer
def write_det_dir(path, rs, names, n_max, empty_every, score_scale, gt, hit, jitter):
    """Detections: with prob `hit` a jittered copy of a ground-truth box (same class), else noise."""
    os.makedirs(path)
    for i, name in enumerate(names):
        n = 0 if i % empty_every == 3 else rs.randint(1, n_max)
        cls = rs.randint(0, 8, n).astype(np.float64)
        xywh = np.column_stack([rs.uniform(0.1, 0.9, n), rs.uniform(0.1, 0.9, n),
                                rs.uniform(0.05, 0.4, n), rs.uniform(0.05, 0.4, n)])
        for j in range(n):
            if gt[i] and rs.rand() < hit:
                g = gt[i][rs.randint(len(gt[i]))]
                cls[j] = g[0]
                xywh[j] = np.asarray(g[1:]) * (1 + rs.normal(0, jitter, 4))
        conf = rs.uniform(0, 1, n) * score_scale
        np.save(os.path.join(path, name + ".npy"), np.column_stack([cls, xywh, conf]).reshape(n, 6))


def make_g2():
    install_stub([], {})
    for m in ("lib", "lib.data", "lib.metrics", "reward"):
        sys.modules.pop(m, None)
    sys.path.insert(0, REF)
    import reward
    from lib import metrics
    from lib.data import set_data
    sys.path.pop(0)
    rs = np.random.RandomState(1)
    N = 24
    names = [f"{i:012d}" for i in range(N)]
    out = {}
    with tempfile.TemporaryDirectory() as td:
        lab, weak, strong = (os.path.join(td, d) for d in ("labels", "weak", "strong"))
        os.makedirs(lab)
        gt = []
        for i, name in enumerate(names):
            gt.append([])
            with open(os.path.join(lab, name + ".txt"), "w") as f:
                if i % 7 == 5:
                    continue                      # image with no labels
                for _ in range(rs.randint(1, 6)):
                    row = (rs.randint(0, 8), *rs.uniform(0.1, 0.9, 2), *rs.uniform(0.05, 0.4, 2))
                    gt[-1].append(row)
                    f.write(" ".join(str(v) for v in row) + "\n")
        write_det_dir(weak, rs, names, 30, 9, 0.8, gt, 0.3, 0.3)
        write_det_dir(strong, rs, names, 30, 11, 1.0, gt, 0.6, 0.1)
        # pack the inputs so tests can rebuild the directories without the reference
        for d, tag in ((lab, "labels"), (weak, "weak"), (strong, "strong")):
            for f in sorted(os.listdir(d)):
                with open(os.path.join(d, f), "rb") as fh:
                    out[f"in/{tag}/{f}"] = np.frombuffer(fh.read(), dtype=np.uint8)
        weak_d, strong_d, labels = set_data(weak, strong, lab)
    for i in range(N):
        for tag, data in (("weak", weak_d), ("strong", strong_d)):
            tp, conf, cls = data[i]
            out[f"set/{tag}/{i}/tp"] = tp
            out[f"set/{tag}/{i}/conf"] = np.asarray(conf, dtype=np.float64)
            out[f"set/{tag}/{i}/cls"] = np.asarray(cls, dtype=np.float64)
        out[f"set/labels/{i}"] = np.asarray(labels[i], dtype=np.float64)
    for E in (0, 5, N - 1):
        vals = []
        for i in range(N):
            np.random.seed(1000 + i)
            vals.append(reward.compute_orie(i, weak_d, strong_d, labels, E))
        v = np.array(vals)
        out[f"orie/{E}"] = np.where(np.isnan(v), 0, v)
    out["dcsb"] = np.array([reward.compute_dcsb(i, weak_d, strong_d) for i in range(N)], dtype=np.int64)
    # unit vectors
    b1 = rs.uniform(0, 1, (7, 4))
    b1[:, 2:] += b1[:, :2]
    b2 = rs.uniform(0, 1, (9, 4))
    b2[:, 2:] += b2[:, :2]
    out["unit/box_iou/a"], out["unit/box_iou/b"] = b1, b2
    out["unit/box_iou/out"] = metrics.box_iou(b1, b2)
    dets = np.column_stack([b2, rs.uniform(0, 1, 9), rs.randint(0, 3, 9)])
    labs = np.column_stack([rs.randint(0, 3, 7), b1])
    out["unit/box_correct/dets"], out["unit/box_correct/labels"] = dets, labs
    out["unit/box_correct/out"] = metrics.box_correct(dets, labs, np.array([0.5]))
    tp = rs.rand(50, 1) > 0.5
    conf = rs.uniform(0, 1, 50)
    pc = rs.randint(0, 5, 50).astype(float)
    tc = rs.randint(0, 6, 30)
    out["unit/ap/tp"], out["unit/ap/conf"], out["unit/ap/pred_cls"], out["unit/ap/target_cls"] = tp, conf, pc, tc
    out["unit/ap/out"] = metrics.ap_per_class(tp, conf, pc, tc)
    rec = np.sort(rs.uniform(0, 1, 20))
    prec = rs.uniform(0, 1, 20)
    out["unit/compute_ap/rec"], out["unit/compute_ap/prec"] = rec, prec
    out["unit/compute_ap/out"] = np.array(metrics.compute_ap(rec, prec))
    xywh = rs.uniform(0, 1, (6, 4))
    out["unit/xywh2xyxy/in"], out["unit/xywh2xyxy/out"] = xywh, metrics.xywh2xyxy(xywh)
    np.savez_compressed(os.path.join(HERE, "g2_orie.npz"), **out)
    print("G2:", len(out), "arrays")


def make_g3():
    """G3 (other consumers of the detection files): test.py test_map (realized mAP vs offloading
    ratio) and lib/data.py extract_output_feature (stage-24 output features), on the G2 inputs."""
    install_stub([], {})
    for m in ("lib", "lib.data", "lib.metrics", "reward", "test"):
        sys.modules.pop(m, None)
    sys.path.insert(0, REF)
    import test as ref_test
    from lib.data import extract_output_feature, set_data
    sys.path.pop(0)
    with np.load(os.path.join(HERE, "g2_orie.npz"), allow_pickle=False) as z:
        g2 = {k: z[k] for k in z.files if k.startswith("in/")}
    rs = np.random.RandomState(3)
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for k, v in g2.items():
            _, tag, fname = k.split("/", 2)
            os.makedirs(os.path.join(td, tag), exist_ok=True)
            with open(os.path.join(td, tag, fname), "wb") as f:
                f.write(v.tobytes())
        weak_d, strong_d, labels = set_data(*(os.path.join(td, t) for t in ("weak", "strong", "labels")))
        N = len(labels)
        folds = 3
        split = np.zeros((folds, N), dtype=bool)
        perm = rs.permutation(N)
        for f in range(folds):
            split[f, perm[f::folds]] = True
        est_dirs = []
        for e in range(2):
            d = os.path.join(td, f"est{e}")
            os.makedirs(d)
            for f in range(folds):
                tr, va = rs.normal(0, 1, int((~split[f]).sum())), rs.normal(0, 1, int(split[f].sum()))
                np.savez(os.path.join(d, f"estimate{f + 1}.npz"), train_est=tr, val_est=va)
                out[f"in/est{e}/estimate{f + 1}/train_est"], out[f"in/est{e}/estimate{f + 1}/val_est"] = tr, va
            est_dirs.append(d)
        out["in/split"] = split
        out["test_map"] = ref_test.test_map(weak_d, strong_d, np.concatenate(labels).astype(int), est_dirs, split)
        feat = os.path.join(td, "features")
        names = sorted(f[:-4] for f in os.listdir(os.path.join(td, "weak")))
        for n in names + ["zz_no_output"]:
            os.makedirs(os.path.join(feat, n))
        extract_output_feature(os.path.join(td, "weak"), feat, 80, k=25)
        for n in names + ["zz_no_output"]:
            out[f"feature/{n}"] = np.load(os.path.join(feat, n, "stage24_output_features.npy"))
    np.savez_compressed(os.path.join(HERE, "g3_consumers.npz"), **out)
    print("G3:", len(out), "arrays")


if __name__ == "__main__":
    import warnings
    warnings.filterwarnings("ignore")
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        if "--g3-only" not in sys.argv:
            make_g1()
            make_g2()
        make_g3()
    print("done")
