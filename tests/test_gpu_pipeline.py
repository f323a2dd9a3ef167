"""End-to-end drop-in pipeline on the GPU (BASELINE config 4 in miniature):

  edgeml_amd.detect (CLI, detect.py:109-121 arguments) -> .npy files -> edgeml_amd.reward (CLI)

* every detector of the CLI (ssd, faster_rcnn, and the third choice, RetinaNet) in VOC mode
  (``--dataset voc``: 21-class checkpoints through ``--model-path``, labels shifted by one,
  detect.py:91) writes the files the CPU oracle's forward + the reference formatting writes;
* the GPU reward CLI on the engine's files gives the ORIE that the oracle consumer gives on the
  oracle's files (bit-identical).
"""
import os
import tempfile
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [(640, 640), (480, 640), (612, 612)]


def _images(root):
    from PIL import Image
    from edgeml_amd import synthetic
    os.makedirs(root)
    for i, (h, w) in enumerate(SIZES):
        img = synthetic.make_scene(900 + i, h, w)
        Image.fromarray(img.transpose(1, 2, 0)).save(os.path.join(root, f"{i:012d}.png"))


def _oracle_files(model, img_dir, out_dir, dataset):
    from edgeml_amd import detect, fmt
    os.makedirs(out_dir, exist_ok=True)
    for name in sorted(os.listdir(img_dir)):
        img = detect.read_image(os.path.join(img_dir, name)) / 255
        p = model([img])[0]
        rows = fmt.format_detections(p["boxes"].numpy(), p["scores"].numpy(), p["labels"].numpy(),
                                     int(img.shape[-2]), int(img.shape[-1]), dataset)
        fmt.save_npy(out_dir, name, rows)


@pytest.mark.parametrize("model,kind", [("ssd", "ssd"), ("faster_rcnn", "faster_rcnn"), ("retinanet", "retinanet")])
def test_detect_cli_voc_model_path_matches_oracle(model, kind):
    """The CLI's files are exactly the formatted engine outputs (byte-identical .npy), and those
    engine outputs match the oracle under the decision-replay protocol (tests/parity_models.py)."""
    from edgeml_amd import detect, fmt, synthetic
    from tests import parity_models as PM
    sd = synthetic.synthetic_state_dict(kind, 21, seed=0)  # the seed the BN calibration table was made for
    with tempfile.TemporaryDirectory() as td:
        img_dir, pth = os.path.join(td, "imgs"), os.path.join(td, "w.pth")
        _images(img_dir)
        torch.save(sd, pth)
        out = os.path.join(td, "engine")
        detect.main(detect.getargs([img_dir, out, "--dataset", "voc", "--model", model, "--model-path", pth]))
        assert sorted(os.listdir(out)) == [f"{i:012d}.npy" for i in range(len(SIZES))]
        m = detect.load_weak_models(model, pth, 21).to("cuda")
        for name in sorted(os.listdir(img_dir)):
            img = (detect.read_image(os.path.join(img_dir, name)) / 255)[None]
            _, _, h, w = img.shape
            plan = m.plan(1, h, w)
            plan.input.tensor().copy_(img.cuda())
            plan.run()
            torch.cuda.synchronize()
            n = int(plan.out_count.tensor()[0])
            rows = fmt.format_detections(plan.out_box.tensor()[0, :n].cpu().numpy(),
                                         plan.out_score.tensor()[0, :n].cpu().numpy(),
                                         plan.out_label.tensor()[0, :n].cpu().numpy(), h, w, "voc")
            got = np.load(os.path.join(out, name[:-4] + ".npy"))
            assert got.dtype == np.float64 and got.shape[1:] == (6,)
            assert got.tobytes() == rows.tobytes(), name
            assert got.shape[0] == 0 or (got[:, 0].min() >= 0 and got[:, 0].max() <= 19)
            if kind == "ssd":
                rep = PM.ssd_check(plan, sd, 21, True, img, f"cli voc ssd {name}")
            elif kind == "faster_rcnn":
                rep = PM.frcnn_check(plan, sd, 21, img, f"cli voc frcnn {name}")
            else:
                rep = PM.retina_check(plan, sd, 21, img, f"cli voc retinanet {name}")
            print(rep)


def test_pipeline_module_runs_config4_in_miniature():
    """edgeml_amd.pipeline: weak + strong detection files, then ORIE, in one process."""
    from edgeml_amd import pipeline, synthetic
    warnings.filterwarnings("ignore")
    with tempfile.TemporaryDirectory() as td:
        img, lab, work = (os.path.join(td, d) for d in ("imgs", "labels", "work"))
        synthetic.make_dataset(img, 5, seed=2, label_dir=lab)
        pipeline.main(pipeline.getargs([img, lab, work, "--num-ensemble", "3"]))
        for d in ("weak", "strong"):
            assert sorted(os.listdir(os.path.join(work, d))) == [f"{i:012d}.npy" for i in range(5)]
        with np.load(os.path.join(work, "reward", "orie3.npz")) as z:
            r = z["reward"]
        assert r.shape == (5,) and np.all(np.isfinite(r))


def test_detect_then_reward_cli_equals_oracle_pipeline():
    from edgeml_amd import detect, reward, synthetic
    from oracle import orie
    from oracle.frcnn import FasterRCNNOracle
    from oracle.ssdlite import SSDLiteOracle
    warnings.filterwarnings("ignore")
    with tempfile.TemporaryDirectory() as td:
        img_dir = os.path.join(td, "imgs")
        _images(img_dir)
        dirs = {k: os.path.join(td, k) for k in ("weak_g", "strong_g", "weak_o", "strong_o", "labels", "out")}
        detect.main(detect.getargs([img_dir, dirs["weak_g"], "--model", "ssd"]))
        detect.main(detect.getargs([img_dir, dirs["strong_g"], "--model", "faster_rcnn"]))
        _oracle_files(SSDLiteOracle(synthetic.synthetic_state_dict("ssd", 91, True), 91, True), img_dir,
                      dirs["weak_o"], "coco")
        _oracle_files(FasterRCNNOracle(synthetic.synthetic_state_dict("faster_rcnn", 91), 91), img_dir,
                      dirs["strong_o"], "coco")
        os.makedirs(dirs["labels"])
        for f in sorted(os.listdir(dirs["strong_o"])):  # pseudo ground truth: confident oracle boxes
            rows = np.load(os.path.join(dirs["strong_o"], f))
            with open(os.path.join(dirs["labels"], f[:-4] + ".txt"), "w") as fh:
                for r in rows[rows[:, 5] >= 0.3]:
                    fh.write(" ".join([str(int(r[0]))] + [repr(float(v)) for v in r[1:5]]) + "\n")
        E = len(SIZES) - 1
        reward.main(reward.getargs([dirs["weak_g"], dirs["strong_g"], dirs["labels"], dirs["out"],
                                    "--num-ensemble", str(E), "--seed", "1000"]))
        with np.load(os.path.join(dirs["out"], f"orie{E}.npz")) as z:
            got = z["reward"]
        ref = orie.orie_all(dirs["weak_o"], dirs["strong_o"], dirs["labels"], E, seed=1000)
        print("ORIE engine+GPU reward", got, "oracle", ref)
        assert np.any(ref != 0)
        np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("kind", ["ssd", "frcnn"])
def test_run_batches_matches_call(kind):
    """model.run_batches (the CLI's path: two batches in flight, each on its own plan instance,
    stream and side lanes) gives bit-identical detections to model(images) batch by batch, across a
    shape change, a ragged last batch and slot reuse; the decoded uint8 images (divided by 255 on
    the device) give the same detections as the host's float images.  The SSD case includes 16-image
    batches (two chains on side lanes) with both in-flight instances busy at once."""
    from edgeml_amd import models, synthetic
    if kind == "ssd":
        sd = synthetic.synthetic_state_dict("ssd", 91, True, seed=0)
        model = models.SSDLite320(sd, 91, True).to("cuda:0")
        shapes = [(480, 640, 2)] * 2 + [(480, 640, 1)] + [(640, 640, 16)] * 3
    else:
        model = models.fasterrcnn_resnet50_fpn_v2().to("cuda:0")
        shapes = [(480, 640, 2)] * 2 + [(480, 640, 1)] + [(640, 640, 2)] * 2
    batches, batches_u8 = [], []
    for i, (h, w, n) in enumerate(shapes):
        u8 = synthetic.make_batch_u8(n, h, w, seed=40 + i)
        batches.append((i, list(u8.float() / 255)))
        batches_u8.append((i, list(u8)))
    got = list(model.run_batches(batches, inflight=2))
    got_u8 = list(model.run_batches(batches_u8, inflight=2))
    assert [t for t, _ in got] == list(range(len(batches))) == [t for t, _ in got_u8]
    for (tag, dets), (_, dets_u8), (_, imgs) in zip(got, got_u8, batches):
        ref = model(imgs)
        assert len(dets) == len(imgs) == len(dets_u8)
        for (b, s, l), (bu, su, lu), r in zip(dets, dets_u8, ref):
            np.testing.assert_array_equal(b, r["boxes"].cpu().numpy())
            np.testing.assert_array_equal(s, r["scores"].cpu().numpy())
            np.testing.assert_array_equal(l, r["labels"].cpu().numpy())
            np.testing.assert_array_equal(bu, b)
            np.testing.assert_array_equal(su, s)
            np.testing.assert_array_equal(lu, l)
            assert len(s) > 0


@pytest.mark.parametrize("kind,B,H,W,inflight,n", [("ssd", 32, 640, 640, 4, 8), ("ssd", 8, 480, 640, 2, 8),
                                                   ("frcnn", 6, 427, 640, 3, 6)])
def test_run_batches_in_flight_reproducible(kind, B, H, W, inflight, n):
    """With the models' own in-flight counts (SSD: 32-image batches on two 16-image chains, four in
    flight; FRCNN: three in flight) every image's detections equal the one-batch-at-a-time result.
    Round 4's uint8 table kernels failed exactly this (profiles/r4k_lut_race.txt: whole batches or
    single images differing under concurrency, while every single-kernel parity test passed)."""
    from edgeml_amd import models, synthetic
    if kind == "ssd":
        model = models.SSDLite320(synthetic.synthetic_state_dict("ssd", 91, True, seed=0), 91, True).to("cuda:0")
    else:
        model = models.fasterrcnn_resnet50_fpn_v2().to("cuda:0")
    u8s = [synthetic.make_batch_u8(B, H, W, seed=300 + i) for i in range(n)]
    ref = [model(list(u.float() / 255)) for u in u8s]
    for rep in range(2):
        got = list(model.run_batches([(i, u.pin_memory() if rep else list(u)) for i, u in enumerate(u8s)],
                                     inflight=inflight))
        assert [t for t, _ in got] == list(range(n))
        for (t, dets) in got:
            for j, (b, s, l) in enumerate(dets):
                r = ref[t][j]
                np.testing.assert_array_equal(b, r["boxes"].cpu().numpy(), err_msg=f"rep {rep} batch {t} image {j}")
                np.testing.assert_array_equal(s, r["scores"].cpu().numpy())
                np.testing.assert_array_equal(l, r["labels"].cpu().numpy())
