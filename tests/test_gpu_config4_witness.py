"""configs[3] at COCO sizes, image by image, against the CPU oracle pipeline.

tests/test_gpu_config4.py runs config 4's topology (100 JPEGs, world 2 against world 1, byte for
byte); this checks its arithmetic.  Twenty images of tools/config4_full.py's 5,000-image set (seeded
synthetic scenes at the four COCO sizes, JPEG quality 90, decoded like detect.read_image), each run
on the engine in the batch the detect CLI puts it in over all 5,000 (distributed.size_batches at the
model's batch: an image's output bits depend on its batch), then:

* Faster R-CNN (the strong detector, plans at 800 x 1,199 / 1,066 / 1,201 after resize) end to end
  against the float32 oracle with tests/e2e_witness.check_image: every RPN and box-stage flip carries
  a boundary witness, identity-paired rows agree within north_star's 1e-3 or carry a witness, and
  the proposal-shift witness bounds the reference's own response (tests/e2e_witness.py);
* SSDLite (the weak detector, 320 x 320 after resize) through the decision replay of
  tests/parity_models.ssd_check on the target images of each batch (raw heads within RAW_TOL of the
  float32 oracle, or -- these JPEG scenes part the two float32 evaluations further on some images --
  no further from the float64 oracle than twice the float32 oracle is; every flip a boundary case);
* ORIE (reward.py --method orie, E = 19, pseudo ground truth = the oracle strong detector's rows with
  conf >= 0.3, seeded serial ensembles, the oracle consumer pinned to G2) of the engine's files
  against the oracle pipeline's files (oracle forwards -> detect.py formatting).
"""
import os
import tempfile
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_SET, TARGETS = 5000, list(range(20))
_C = {}


def _setup():
    if not _C:
        from edgeml_amd import distributed, models, synthetic
        from edgeml_amd.distributed import usable_cpus
        from tools.config4_witness import config4_image
        torch.set_num_threads(usable_cpus())
        rs = np.random.RandomState(1)
        sizes = [synthetic.COCO_SIZES[rs.randint(len(synthetic.COCO_SIZES))] for _ in range(N_SET)]
        sd_s, sd_w = synthetic.synthetic_state_dict("faster_rcnn", 91), synthetic.synthetic_state_dict("ssd", 91, True)
        eng_s, eng_w = models.FasterRCNNFPNv2(sd_s, 91).to("cuda"), models.SSDLite320(sd_w, 91, True).to("cuda")
        imgs = {}

        def img(i):
            if i not in imgs:
                imgs[i] = config4_image(i, sizes)
            return imgs[i]
        out = {}
        for tag, eng in (("strong", eng_s), ("weak", eng_w)):
            batches = [c for c in distributed.size_batches(sizes, eng.max_batch) if set(c) & set(TARGETS)]
            rows, checks = {}, []
            for c in batches:
                batch = [img(i).float() / 255 for i in c]  # = the CLI's uint8 path (/255 on the device)
                res = eng(batch)
                for b, i in enumerate(c):
                    if i in TARGETS:
                        rows[i] = tuple(res[b][k].cpu().numpy() for k in ("boxes", "scores", "labels"))
                # the checks read the plan's buffers: before the next batch of this size runs
                plan = eng.plan(len(c), *sizes[c[0]])
                checks.append(_witness(plan, c, batch, sd_s, sizes) if tag == "strong" else _ssd(plan, batch, sd_w, c))
            out[tag] = {"rows": rows, "checks": checks}
        _C.update(sizes=sizes, sd_s=sd_s, sd_w=sd_w, out=out, img=img)
    return _C


def _witness(plan, c, batch, sd, sizes):
    from oracle.frcnn import FasterRCNNOracle
    from tests import e2e_witness as W
    ref = FasterRCNNOracle(sd, 91)
    H, W_ = sizes[c[0]]
    reps, fails = {}, []
    for b, i in enumerate(c):
        if i not in TARGETS:
            continue
        A = W.oracle_side(ref, batch[b])
        B = W.engine_side(plan, b, A["anchors"])
        h, w = A["size"]
        scale = np.asarray([np.float32(W_) / np.float32(w), np.float32(H) / np.float32(h)] * 2, np.float32)
        rep, f = W.check_image(A, B, 91, scale, (H, W_))
        reps[i] = rep
        fails += [(i,) + tuple(x) for x in f]
    return reps, fails


def _ssd(plan, batch, sd, c):
    from tests import parity_models
    imgs = torch.stack(batch)
    return parity_models.ssd_check(plan, sd, 91, True, imgs, f"config4 ssd batch {c[0]}..", own_check=1,
                                   only=[b for b, i in enumerate(c) if i in TARGETS], f64_arbiter=True)


def test_config4_frcnn_end_to_end_witnessed():
    from tests import e2e_witness as W
    c = _setup()
    reps, fails = {}, []
    for r, f in c["out"]["strong"]["checks"]:
        reps.update(r)
        fails += f
    assert sorted(reps) == TARGETS, sorted(reps)
    sizes = sorted({tuple(c["sizes"][i]) for i in TARGETS})
    merged = W.merge(list(reps.values()))
    print("config4 frcnn:", len(reps), "images, sizes", sizes, merged)
    assert len(sizes) >= 3, sizes  # mixed COCO sizes, several FRCNN plans
    assert not fails, fails[:5]
    assert merged["identity_paired"] > 20 * len(reps)


def test_config4_ssd_decision_replay():
    c = _setup()
    reports = c["out"]["weak"]["checks"]
    assert reports and all(r["rows"] > 0 for r in reports), reports
    print("config4 ssd:", reports)


def test_config4_orie_against_oracle_pipeline():
    from edgeml_amd import fmt
    from oracle import orie
    from oracle.frcnn import FasterRCNNOracle
    from oracle.ssdlite import SSDLiteOracle
    from tools import rowpair
    warnings.filterwarnings("ignore")
    c = _setup()
    oracles = {"weak": SSDLiteOracle(c["sd_w"], 91, True), "strong": FasterRCNNOracle(c["sd_s"], 91)}
    names = [f"{i:012d}" for i in TARGETS]
    with tempfile.TemporaryDirectory() as td:
        d = lambda *p: os.path.join(td, *p)  # noqa: E731
        for sub in ("eng_weak", "eng_strong", "orc_weak", "orc_strong", "labels"):
            os.makedirs(d(sub))
        for i, name in zip(TARGETS, names):
            im = c["img"](i).float() / 255
            h, w = int(im.shape[-2]), int(im.shape[-1])
            for tag in ("weak", "strong"):
                bx, sc, lb = c["out"][tag]["rows"][i]
                fmt.save_npy(d("eng_" + tag), name + ".jpg", fmt.format_detections(bx, sc, lb, h, w))
                p = oracles[tag]([im])[0]
                rows = fmt.format_detections(p["boxes"].numpy(), p["scores"].numpy(), p["labels"].numpy(), h, w)
                fmt.save_npy(d("orc_" + tag), name + ".jpg", rows)
                if tag == "strong":
                    with open(d("labels", name + ".txt"), "w") as f:
                        for r in rows[rows[:, 5] >= 0.3]:
                            f.write(" ".join([str(int(r[0]))] + [repr(float(v)) for v in r[1:5]]) + "\n")
        E = len(TARGETS) - 1
        o = {s: orie.orie_all(d(s + "_weak"), d(s + "_strong"), d("labels"), E, seed=1000) for s in ("eng", "orc")}
        for tag in ("weak", "strong"):
            r = rowpair.compare_dirs(names, lambda nm: np.load(d("eng_" + tag, nm + ".npy")),
                                     lambda nm: np.load(d("orc_" + tag, nm + ".npy")))
            print(f"config4 {tag} engine vs oracle rows: {r}")
    assert np.all(np.isfinite(o["eng"])) and np.count_nonzero(o["orc"]) > len(TARGETS) // 2, o
    dv = np.abs(o["eng"] - o["orc"])
    print(f"config4 ORIE |engine - oracle|: max {dv.max():.3e} mean {dv.mean():.3e}, {np.count_nonzero(dv)} of "
          f"{len(dv)} images differ; oracle ORIE range {o['orc'].min():.3f}..{o['orc'].max():.3f}")
    # every row difference is witnessed above; what ORIE may move by is bounded by those rows' scores
    # (1e-3) and their flips at the 0.3 / IoU boundaries: a regression guard, measured in DESIGN.md
    assert dv.max() <= 0.05, dv
