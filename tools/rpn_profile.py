"""FRCNN RPN level-kernel phase profile (diagnostic): runs the FRCNN b=8 plan a few times on a
-DRPN_PROFILE build (libedgedet_rpnprof.so via EDGEDET_LIB; build.build(variant="rpnprof",
defines=("RPN_PROFILE",))), whose rpn_level_nms_kernel prints, for image 0 of each level, the
s_memtime ticks spent in radix select, compaction, sort, decode and NMS."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    assert "rpnprof" in os.environ.get("EDGEDET_LIB", ""), "run with EDGEDET_LIB=.../libedgedet_rpnprof.so"
    from edgeml_amd import models, synthetic
    m = models.fasterrcnn_resnet50_fpn_v2().to("cuda")
    plan = m.plan(8, 640, 640, True)
    plan.input.tensor().copy_(synthetic.make_batch_u8(8, 640, 640, seed=0).cuda())
    for _ in range(3):
        plan.run()
        torch.cuda.synchronize()
    print("dets per image:", plan.out_count.tensor().float().mean().item(), flush=True)


if __name__ == "__main__":
    main()
