"""BASELINE config 4 in small: N synthetic COCO-sized JPEG images through edgeml_amd.pipeline (SSDLite
weak + FRCNN strong detection files, then ORIE with E ensembles) on this GPU, with each stage's
wall time.  python tools/pipeline_bench.py [--n 512] [--num-ensemble 1000]"""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from edgeml_amd import pipeline, synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=512)
ap.add_argument("--num-ensemble", type=int, default=1000)
a = ap.parse_args()
with tempfile.TemporaryDirectory() as td:
    img, lab, work = (os.path.join(td, d) for d in ("imgs", "labels", "work"))
    t0 = time.perf_counter()
    synthetic.make_dataset(img, a.n, seed=1, label_dir=lab, ext=".jpg")
    print(f"wrote {a.n} synthetic JPEG images in {time.perf_counter() - t0:.1f} s", flush=True)
    t0 = time.perf_counter()
    pipeline.main(pipeline.getargs([img, lab, work, "--num-ensemble", str(a.num_ensemble)]))
    el = time.perf_counter() - t0
    print(f"config 4 pipeline, {a.n} images, E={a.num_ensemble}: {el:.1f} s end to end "
          f"({a.n / el:.1f} images/s incl. JPEG decode on the host)")
