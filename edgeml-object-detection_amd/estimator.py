"""Drop-in for regression.py's CNN estimator on the stage-24 features (BASELINE config 5, SURVEY.md
§8f row 2): trains lib/nn_model.py's EdgeDetectionNet (no conv layers: an MLP with
Linear-BatchNorm1d-ReLU-Dropout hidden layers) to predict the ORIE reward from the weak detector's
output features, one cross-validation fold per GPU workgroup, with the whole training loop in one
kernel (csrc/estimator.hip).

    python -m edgeml_amd.estimator data_dir reward_path split_path save_dir [--normalize] [--weight]
                                   [--stage 24] [--model CNN] [--seed 0]

Reads <data_dir>/<image>/stage24_output_features.npy (edgeml_amd.features writes them), the reward
npz (edgeml_amd.reward) and the k-fold split (k, N) bool; writes estimate<k>.npz {train_est,
val_est, train_time, val_time} into <save_dir>_best and <save_dir>_last, as regression.py:438-446
does through lib/utils.py parse_path / save_result (test.py / edgeml_amd.evaluate consume them).

Semantics follow regression.py:220-355 (CNNOpt defaults: lr 5e-3, gamma 0.5 at epochs 60/75/90,
weight decay 5e-5, 100 epochs, batch 64 in dataset order, linear [d0, 16, 16, 16, 16, 1]) with
two deliberate differences: the first linear width is the feature width (the reference hard-codes
145, which only fits VOC), and the weights are initialised from --seed with the reference's
distributions (Kaiming-uniform weights, PyTorch's default bias and BatchNorm init) instead of
torch's global RNG, whose stream cannot be reproduced here; dropout masks come from a
counter-based hash.  Parity: with dropout off, a fit equals the oracle (oracle/estimator.py,
torch CPU) within fp32 rounding; with dropout on it is the same algorithm with another random
stream (tests/test_gpu_estimator.py).  regression.py's sklearn models and hidden-layer feature
maps of the external YOLOv5 (stages 0-23) are out of scope.
"""
import argparse
import ctypes
import os
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import List

import numpy as np
import torch

from . import ops


@dataclass
class CNNOpt:
    """regression.py:220-236 (stage-24 case: no conv layers, resize=True)."""
    learning_rate: float = 5e-3
    gamma: float = 0.5
    weight_decay: float = 5e-5
    milestones: List = field(default_factory=lambda: [60, 75, 90])
    max_epoch: int = 100
    batch_size: int = 64
    weight: bool = False
    hidden: List = field(default_factory=lambda: [16, 16, 16, 16])
    dropout: float = 0.1


class MlpSpec:
    """State layout shared with csrc/estimator.hip mlp_layout: per layer W [d_out][d_in], b, and for
    hidden layers gamma, beta; then every hidden layer's running mean and var."""

    def __init__(self, dims):
        self.dims = [int(d) for d in dims]
        self.L = len(self.dims) - 1
        off, o = [], 0
        for l in range(self.L):
            din, dout = self.dims[l], self.dims[l + 1]
            ent = {"w": o, "b": o + dout * din}
            o += dout * din + dout
            if l < self.L - 1:
                ent["g"], ent["be"] = o, o + dout
                o += 2 * dout
            off.append(ent)
        self.np = o
        for l in range(self.L - 1):
            dout = self.dims[l + 1]
            off[l]["rm"], off[l]["rv"] = o, o + dout
            o += 2 * dout
        self.ns = o
        self.off = off

    def init_state(self, rng):
        """kaiming_uniform_ weights (bound sqrt(6 / fan_in), lib/nn_model.py:66,98), nn.Linear's default
        bias init (bound 1 / sqrt(fan_in)), BatchNorm1d weight 1 / bias 0 / running 0 and 1."""
        s = np.zeros(self.ns, np.float32)
        for l in range(self.L):
            din, dout = self.dims[l], self.dims[l + 1]
            e = self.off[l]
            s[e["w"]:e["w"] + dout * din] = rng.uniform(-1, 1, dout * din) * np.sqrt(6.0 / din)
            s[e["b"]:e["b"] + dout] = rng.uniform(-1, 1, dout) / np.sqrt(din)
            if l < self.L - 1:
                s[e["g"]:e["g"] + dout] = 1.0
                s[e["rv"]:e["rv"] + dout] = 1.0
        return s

    def pack(self, named):
        """The inverse of unpack: a state vector from EdgeDetectionNet-named arrays (a reference
        state_dict, num_batches_tracked ignored)."""
        s = np.zeros(self.ns, np.float32)
        ref = self.unpack(s)
        for k, v in ref.items():
            v[...] = np.asarray(named[k], np.float32).reshape(v.shape)  # views into s
        return s

    def unpack(self, state):
        """{name: array} in torch's EdgeDetectionNet naming (linear_stacks.<l>.<0|1>.*)."""
        out = {}
        for l in range(self.L):
            din, dout = self.dims[l], self.dims[l + 1]
            e = self.off[l]
            p = f"linear_stacks.{l}"
            out[p + ".0.weight"] = state[e["w"]:e["w"] + dout * din].reshape(dout, din)
            out[p + ".0.bias"] = state[e["b"]:e["b"] + dout]
            if l < self.L - 1:
                out[p + ".1.weight"] = state[e["g"]:e["g"] + dout]
                out[p + ".1.bias"] = state[e["be"]:e["be"] + dout]
                out[p + ".1.running_mean"] = state[e["rm"]:e["rm"] + dout]
                out[p + ".1.running_var"] = state[e["rv"]:e["rv"] + dout]
        return out


def _dims(d0, opts):
    return [int(d0)] + [int(h) for h in opts.hidden] + [1]


def fit_folds(features, rewards, split, opts=CNNOpt(), seed=0, device="cuda", init=None):
    """Train one estimator per fold of `split` ((k, N) bool, True = validation) on the device.

    features [N, d0], rewards [N] or [k, N] (per-fold targets, e.g. normalised against each fold's
    training set).  Returns (best, last, info):
    per fold dicts {train_est, val_est, train_time, val_time} as regression.py fit_CNN returns, and
    info = {train_loss, test_loss [k, epochs], best_state, last_state [k, ns]}."""
    if not torch.cuda.is_available():
        raise RuntimeError("edgeml_amd.estimator needs an MI355X (HIP) device; there is no CPU path")
    x = np.ascontiguousarray(np.asarray(features, dtype=np.float32))
    split = np.asarray(split, dtype=bool)
    N, d0 = x.shape
    k = split.shape[0]
    y = np.asarray(rewards, dtype=np.float32)
    y = np.ascontiguousarray(np.broadcast_to(y, (k, N)) if y.ndim == 1 else y.reshape(k, N))
    spec = MlpSpec(_dims(d0, opts))
    tr = [np.nonzero(~m)[0].astype(np.int32) for m in split]
    va = [np.nonzero(m)[0].astype(np.int32) for m in split]
    tr_off = np.concatenate([[0], np.cumsum([len(a) for a in tr])]).astype(np.int64)
    va_off = np.concatenate([[0], np.cumsum([len(a) for a in va])]).astype(np.int64)
    if init is None:
        rng = np.random.default_rng(seed)
        init = np.stack([spec.init_state(rng) for _ in range(k)])
    init = np.ascontiguousarray(np.asarray(init, np.float32).reshape(k, spec.ns))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    # named device buffers: they must outlive the asynchronous launches
    g_x, g_y = t(x), t(y)
    g_tr, g_tro = t(np.concatenate(tr + [np.zeros(1, np.int32)])), t(tr_off)
    g_va, g_vao = t(np.concatenate(va + [np.zeros(1, np.int32)])), t(va_off)
    g_init = t(init)
    g_best = torch.empty((k, spec.ns), dtype=torch.float32, device=device)
    g_last = torch.empty_like(g_best)
    g_adam = torch.empty((k, 2 * spec.np), dtype=torch.float32, device=device)
    g_trl = torch.empty((k, opts.max_epoch), dtype=torch.float32, device=device)
    g_tel = torch.empty_like(g_trl)
    L = ops.lib()
    dims_host = (ctypes.c_int32 * len(spec.dims))(*spec.dims)
    ms_host = (ctypes.c_int32 * max(1, len(opts.milestones)))(*(list(opts.milestones) or [0]))
    ops.check(L.edgedet_mlp_fit(ops._ptr(g_x), N, d0, ops._ptr(g_y), ops._ptr(g_tr), ops._ptr(g_tro), ops._ptr(g_va),
                                ops._ptr(g_vao), k, spec.L, dims_host, ops._ptr(g_init), ops._ptr(g_best),
                                ops._ptr(g_last), ops._ptr(g_adam), ops._ptr(g_trl), ops._ptr(g_tel), opts.max_epoch,
                                opts.batch_size, opts.learning_rate, opts.gamma, ms_host, len(opts.milestones),
                                opts.weight_decay, int(bool(opts.weight)), opts.dropout, int(seed) & (2 ** 64 - 1),
                                ops.stream_handle()))
    torch.cuda.synchronize()
    best, last = [], []
    for f in range(k):
        res = []
        for g_state in (g_best, g_last):
            st = g_state[f]
            ests, times = [], []
            for idx in (tr[f], va[f]):
                g_idx = t(idx if len(idx) else np.zeros(1, np.int32))
                out = torch.empty(max(len(idx), 1), dtype=torch.float32, device=device)
                t0 = time.perf_counter()
                ops.check(L.edgedet_mlp_predict(ops._ptr(g_x), d0, ops._ptr(g_idx), len(idx), spec.L, dims_host,
                                                ops._ptr(st), ops._ptr(out), ops.stream_handle()))
                torch.cuda.synchronize()
                times.append((time.perf_counter() - t0) / max(len(idx), 1))
                ests.append(out[:len(idx)].cpu().numpy())
            res.append({"train_est": ests[0], "val_est": ests[1], "train_time": times[0], "val_time": times[1]})
        best.append(res[0])
        last.append(res[1])
    info = {"train_loss": g_trl.cpu().numpy(), "test_loss": g_tel.cpu().numpy(),
            "best_state": g_best.cpu().numpy(), "last_state": g_last.cpu().numpy(), "spec": spec}
    return best, last, info


def normalize_rewards(train_reward, val_reward):
    """regression.py:431-434: rank transform to a uniform distribution."""
    val = np.array([np.sum(train_reward <= x) / len(train_reward) for x in val_reward])
    train = (np.argsort(np.argsort(train_reward)) + 1) / len(train_reward)
    return train, val


def parse_path(path):
    """lib/utils.py:8-22, including its treatment of absolute paths (the leading separator is
    dropped by os.path.join(*parts)), so outputs land where the reference puts them."""
    best, last = "", ""
    if path != "":
        parts = os.path.normpath(path).split(os.sep)
        name = parts[-1]
        parts[-1] = name + "_best"
        best = os.path.join(*parts)
        parts[-1] = name + "_last"
        last = os.path.join(*parts)
    return best, last


def save_result(path, result, index):
    """lib/utils.py:25-29."""
    Path(path).mkdir(parents=True, exist_ok=True)
    np.savez(os.path.join(path, f"estimate{index + 1}.npz"), **result)


def load_stage24(data_dir):
    """lib/data.py:87-124 with stage 24: every image directory's stage24_output_features.npy, in
    sorted order."""
    images = sorted(f for f in os.listdir(data_dir) if not os.path.isfile(os.path.join(data_dir, f)))
    return np.stack([np.load(os.path.join(data_dir, im, "stage24_output_features.npy"), allow_pickle=False)
                     for im in images]) if images else np.zeros((0, 0))


def main(opts):
    if opts.model != "CNN" or opts.stage != 24:
        raise SystemExit("edgeml_amd.estimator runs regression.py's CNN estimator on the stage-24 output features "
                         "(--model CNN --stage 24); the sklearn models and YOLOv5 hidden-layer maps are not built")
    features = load_stage24(opts.data_dir)
    with np.load(opts.reward_path, allow_pickle=False) as z:
        reward = z["reward"]
    assert len(features) == len(reward), "Inconsistent number of feature maps and offloading rewards."
    split = np.load(opts.split_path, allow_pickle=False)
    assert len(reward) == split.shape[1], "Inconsistent number of data points from the dataset and the split."
    cnn = CNNOpt(weight=opts.weight and opts.normalize)
    save_best, save_last = parse_path(opts.save_dir)
    y = np.zeros(split.shape, np.float32)  # per-fold targets (normalised against the fold's training set)
    for cv_idx, val_mask in enumerate(split):
        tr_r, va_r = reward[~val_mask], reward[val_mask]
        if opts.normalize:
            tr_r, va_r = normalize_rewards(tr_r, va_r)
        y[cv_idx, ~val_mask], y[cv_idx, val_mask] = tr_r, va_r
    t0 = time.perf_counter()
    best, last, info = fit_folds(features, y, split, cnn, seed=opts.seed)  # every fold in one launch
    print(f"trained {len(split)} folds x {cnn.max_epoch} epochs in {time.perf_counter() - t0:.2f} s")
    for cv_idx in range(len(split)):
        print(f"fold {cv_idx + 1}: best test loss {info['test_loss'][cv_idx].min():.6f}")
        save_result(save_best, best[cv_idx], cv_idx)
        save_result(save_last, last[cv_idx], cv_idx)
    return best, last


def getargs(argv=None):
    a = argparse.ArgumentParser()
    a.add_argument("data_dir")
    a.add_argument("reward_path")
    a.add_argument("split_path")
    a.add_argument("save_dir")
    a.add_argument("--normalize", action="store_true")
    a.add_argument("--weight", action="store_true")
    a.add_argument("--stage", type=int, default=24)
    a.add_argument("--resize", type=int, default=0)
    a.add_argument("--model", type=str, default="CNN")
    a.add_argument("--model-dir", type=str, default="")
    a.add_argument("--seed", type=int, default=0)
    return a.parse_args(argv)


if __name__ == "__main__":
    main(getargs())
