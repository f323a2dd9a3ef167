"""BASELINE config 4 end to end: weak + strong detection outputs, then the ORIE rewards.

    python -m edgeml_amd.pipeline IMG_DIR LABEL_DIR WORK_DIR [--num-ensemble 1000] [--seed 0]
                                  [--weak ssd] [--strong faster_rcnn] [--dataset coco]
    python -m torch.distributed.run --standalone --nproc-per-node 8 -m edgeml_amd.pipeline ...

The reference runs the same steps as separate scripts (torch_models/detect.py once per detector,
then README.md:57 `python reward.py WEAK STRONG LABEL SAVE --method orie --num-ensemble 1000`);
here they share one process per GPU:
  WORK_DIR/weak/*.npy           edgeml_amd.detect --model <weak>  (rows gathered to rank 0, which writes)
  WORK_DIR/strong/*.npy         edgeml_amd.detect --model <strong>
  WORK_DIR/reward/orie<E>.npz   edgeml_amd.reward (each rank evaluates a block of target images)
Under torchrun the ranks meet at a barrier after each stage, so every rank reads complete files.
"""
import argparse
import os
import time

import torch


def _barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def main(opts):
    from . import detect, reward
    from . import distributed as dist_mod
    if not torch.cuda.is_available():
        raise RuntimeError("edgeml_amd.pipeline needs an MI355X (HIP) device; there is no CPU path")
    rank, _ = dist_mod.ensure_initialized()
    times = {}
    dirs = {k: os.path.join(opts.work_dir, k) for k in ("weak", "strong", "reward")}
    for stage, model in (("weak", opts.weak), ("strong", opts.strong)):
        t0 = time.perf_counter()
        detect.main(detect.getargs([opts.img_dir, dirs[stage], "--dataset", opts.dataset, "--model", model,
                                    "--decode", getattr(opts, "decode", "gpu")]))
        _barrier()
        times[stage] = time.perf_counter() - t0
    t0 = time.perf_counter()
    out = reward.main(reward.getargs([dirs["weak"], dirs["strong"], opts.label_dir, dirs["reward"],
                                      "--num-ensemble", str(opts.num_ensemble), "--seed", str(opts.seed)]))
    _barrier()
    times["reward"] = time.perf_counter() - t0
    if rank == 0:
        print("pipeline stage seconds:", {k: round(v, 2) for k, v in times.items()})
    return out


def getargs(argv=None):
    a = argparse.ArgumentParser()
    a.add_argument("img_dir")
    a.add_argument("label_dir")
    a.add_argument("work_dir")
    a.add_argument("--dataset", default="coco")
    a.add_argument("--weak", default="ssd")
    a.add_argument("--strong", default="faster_rcnn")
    a.add_argument("--num-ensemble", type=int, default=1000)
    a.add_argument("--seed", type=int, default=0)
    a.add_argument("--decode", choices=("gpu", "host"), default="gpu", help="JPEG decode path of the detect stages")
    return a.parse_args(argv)


if __name__ == "__main__":
    main(getargs())
