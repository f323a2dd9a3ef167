"""Measurement: host-to-device rate of ops.upload (the input upload kernel) against torch's DMA copy.

    python tools/upload_bw.py [--mb 39.3] [--reps 20]

Pinned uint8 source (one SSD batch of 32 640 x 640 images = 39.3 MB by default), device destination;
rates from HIP events around `reps` back-to-back copies on one stream."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=32 * 3 * 640 * 640 / 1e6)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from edgeml_amd import ops
    n = int(a.mb * 1e6)
    host = torch.randint(0, 256, (n,), dtype=torch.uint8).pin_memory()
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    for name, fn in (("ops.upload (kernel)", lambda: ops.upload([(dev, host)], s)),
                     ("torch copy_ (DMA)", lambda: dev.copy_(host, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        print(f"{name}: {n / 1e6:.1f} MB in {ms:.3f} ms = {n / ms / 1e6:.1f} GB/s", flush=True)
        assert torch.equal(dev[:1 << 20].cpu(), host[:1 << 20])


if __name__ == "__main__":
    main()
