"""SSD image-NMS phase profile (diagnostic): runs the SSD b=32 plan a few times on a -DNMS_PROFILE build
(libedgedet_nmsprof.so via EDGEDET_LIB; build.build(variant="nmsprof", defines=("NMS_PROFILE",))),
whose ssd_image_nms_kernel prints, for image 0 of each chain, its rounds and the s_memtime ticks
spent selecting, sorting, in NMS and writing out."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    assert "nmsprof" in os.environ.get("EDGEDET_LIB", ""), "run with EDGEDET_LIB=.../libedgedet_nmsprof.so"
    from edgeml_amd import models, synthetic
    m = models.ssdlite320_mobilenet_v3_large().to("cuda")
    plan = m.plan(32, 640, 640, True)
    plan.input.tensor().copy_(synthetic.make_batch_u8(32, 640, 640, seed=0).cuda())
    for _ in range(3):
        plan.run()
        torch.cuda.synchronize()
    print("dets per image:", plan.out_count.tensor().float().mean().item(), flush=True)


if __name__ == "__main__":
    main()
