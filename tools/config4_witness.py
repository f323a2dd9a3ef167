"""End-to-end FRCNN witness attribution on the config-4 subset (tools/config4_full.py's images 0..59).

    python tools/config4_witness.py [--images 0-59] [-o out.json]

tools/config4_full.py (profiles/r4h_config4_full.log) found one detection on each side unpaired in one
image of its 60-image ORIE subset (mixed COCO sizes, JPEG q = 90, seed 1).  This rebuilds those
images exactly (same seeded scenes and sizes, same JPEG encoder, decoded like read_image), runs the
engine on each image's own batch -- the batches the detect CLI forms over all 5,000 images
(distributed.size_batches at FRCNN's batch of 8; an image's output bits depend on its batch) -- and
attributes every end-to-end difference against the float32 CPU oracle with tests/e2e_witness.py.
"""
import argparse
import io
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_images(s):
    out = []
    for part in s.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def config4_image(i, sizes, seed=1):
    """Image i of tools/config4_full.py's set as read_image returns it (uint8 [3, H, W])."""
    from PIL import Image
    from edgeml_amd import synthetic
    h, w = sizes[i]
    img = synthetic.make_scene(seed * 100003 + i, h, w)
    buf = io.BytesIO()
    Image.fromarray(img.transpose(1, 2, 0)).save(buf, format="JPEG", quality=90)
    buf.seek(0)
    with Image.open(buf) as im:
        arr = np.asarray(im.convert("RGB"), dtype=np.uint8)
    return torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", default="0-59")
    ap.add_argument("--n", type=int, default=5000)
    ap.add_argument("-o", default="")
    args = ap.parse_args()
    from edgeml_amd import distributed, models, synthetic
    from edgeml_amd.distributed import usable_cpus
    from oracle.frcnn import FasterRCNNOracle
    from tests import e2e_witness as W
    torch.set_num_threads(usable_cpus())
    rs = np.random.RandomState(1)
    sizes = [synthetic.COCO_SIZES[rs.randint(len(synthetic.COCO_SIZES))] for _ in range(args.n)]
    targets = parse_images(args.images)
    sd = synthetic.synthetic_state_dict("faster_rcnn", 91)
    eng = models.FasterRCNNFPNv2(sd, 91).to("cuda")
    ref = FasterRCNNOracle(sd, 91)
    batches = [c for c in distributed.size_batches(sizes, eng.max_batch) if set(c) & set(targets)]
    reps, fails = {}, []
    for c in batches:
        imgs = {i: config4_image(i, sizes) for i in c}
        batch = [imgs[i].float() / 255 for i in c]  # = the CLI's uint8 path (/255 on the device, bit-identical)
        eng(batch)
        H, W_ = sizes[c[0]]
        plan = eng.plan(len(c), H, W_)
        for b, i in enumerate(c):
            if i not in targets:
                continue
            t0 = time.perf_counter()
            A = W.oracle_side(ref, batch[b])
            B = W.engine_side(plan, b, A["anchors"])
            h, w = A["size"]
            scale = np.asarray([np.float32(W_) / np.float32(w), np.float32(H) / np.float32(h)] * 2, np.float32)
            rep, f = W.check_image(A, B, 91, scale, (H, W_))
            reps[i] = rep
            fails += [(i,) + tuple(x) for x in f]
            print(f"image {i} ({H}x{W_}, batch {len(c)} slot {b}): {time.perf_counter() - t0:.1f}s "
                  f"{json.dumps(rep)}" + (f"  FAIL {f}" if f else ""), flush=True)
    out = {"images": len(reps), "merged": W.merge(list(reps.values())), "failures": [str(x) for x in fails],
           "with_unpaired": {i: r["rowpair"] for i, r in reps.items() if r["rowpair"]["unpaired"]}}
    print(json.dumps(out, indent=1))
    if args.o:
        with open(args.o, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
