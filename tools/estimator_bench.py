"""Time the device estimator fit (edgeml_amd.estimator.fit_folds: every fold, 100 epochs, one
launch) at COCO-val scale against the CPU oracle (oracle/estimator.py, torch CPU, the reference's
fit_CNN loop) on a bounded number of epochs.  python tools/estimator_bench.py [--n 5000] [--folds 5]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from edgeml_amd import estimator  # noqa: E402
from oracle import estimator as oest  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=5000)
ap.add_argument("--d0", type=int, default=205)
ap.add_argument("--folds", type=int, default=5)
ap.add_argument("--cpu-epochs", type=int, default=5)
a = ap.parse_args()
rng = np.random.default_rng(0)
x = rng.normal(0, 1, (a.n, a.d0)).astype(np.float32)
y = (np.tanh(0.5 * x[:, 20:25].sum(1)) + 0.05 * rng.normal(0, 1, a.n)).astype(np.float32)
fold = rng.permutation(np.arange(a.n) % a.folds)
split = np.stack([fold == f for f in range(a.folds)])
opts = estimator.CNNOpt()
estimator.fit_folds(x[:256], y[:256], split[:, :256], estimator.CNNOpt(max_epoch=1))  # warm
torch.cuda.synchronize()
t0 = time.perf_counter()
best, last, info = estimator.fit_folds(x, y, split, opts)
gpu = time.perf_counter() - t0
print(f"device: {a.folds} folds x {opts.max_epoch} epochs, N={a.n}, d0={a.d0}: {gpu:.3f} s "
      f"(best test loss per fold {np.round(info['test_loss'].min(1), 4).tolist()})")
torch.set_num_threads(16)
spec = info["spec"]
t0 = time.perf_counter()
oest.fit(x, y, split[0], spec, spec.init_state(np.random.default_rng(1)), estimator.CNNOpt(max_epoch=a.cpu_epochs))
cpu = time.perf_counter() - t0
per_fold = cpu / a.cpu_epochs * opts.max_epoch
print(f"cpu oracle (torch, 16 threads): {a.cpu_epochs} epochs of one fold {cpu:.2f} s -> "
      f"{per_fold:.1f} s per fold, {per_fold * a.folds:.1f} s for {a.folds} folds; "
      f"device speedup {per_fold * a.folds / gpu:.0f}x")
