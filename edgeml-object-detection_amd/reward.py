"""Drop-in for reward.py (the ORIE / DCSB consumer of the detection files), TP matching and AP on the GPU.

    python -m edgeml_amd.reward weak_dir strong_dir label_dir save_dir [--method orie|dcsb]
                                [--num-ensemble 1000] [--seed 0]

Same arguments, same ``orie{E}.npz`` / ``dcsb.npz`` output (``reward``, ``time``) as reward.py:72-115.
Host side (this file): the file parsing of lib/data.py:11-43 and the ensemble draws of
reward.py:34-38 (numpy's Mersenne Twister, so the ensembles are the reference's).  Device side
(csrc/orie.hip, libedgedet.so): lib/metrics.py box_correct for every image (set_data's TP flags) and
the two ap_per_class evaluations of every compute_orie call.  Differences from the reference:
  * deterministic by design: the reference draws every image's ensemble from numpy's global RNG inside
    a thread pool (reward.py:78), so its ensembles depend on thread timing; here image i's ensemble is
    np.random.permutation after np.random.seed(seed + i), drawn serially;
  * equal confidences are ordered by (image, row) instead of by the reference's unstable quicksort
    (lib/metrics.py:101); with distinct confidences the AP values are bit-identical.
"""
import argparse
import os
import time
from pathlib import Path

import numpy as np
import torch

from . import ops


# ------------------------------------------------------------------------------ lib/data.py parsing
def xywh2xyxy(x):
    """lib/metrics.py:6-18 (float64, same op order)."""
    y = np.copy(x)
    y[:, 0] = x[:, 0] - x[:, 2] / 2
    y[:, 1] = x[:, 1] - x[:, 3] / 2
    y[:, 2] = x[:, 0] + x[:, 2] / 2
    y[:, 3] = x[:, 1] + x[:, 3] / 2
    return y


def load_data(path, files, with_conf=False):
    """lib/data.py:11-43: per file (cls int, xyxy float64[, conf]) or () when absent/empty."""
    data = []
    for file in files:
        file_path, file_data = os.path.join(path, file), tuple()
        if os.path.isfile(file_path + ".txt"):
            with open(file_path + ".txt", "r") as f:
                file_data = [line.strip().split(" ") for line in f.readlines()]
        elif os.path.isfile(file_path + ".npy"):
            file_data = np.load(file_path + ".npy", allow_pickle=False)
        if len(file_data) > 0:
            cols = [np.array(x).astype(float) for x in zip(*file_data)]
            if with_conf:
                file_data = (cols[0].astype(int), xywh2xyxy(np.stack(cols[1:-1], axis=1)), cols[-1])
            else:
                file_data = (cols[0].astype(int), xywh2xyxy(np.stack(cols[1:], axis=1)))
        else:
            file_data = tuple()
        data.append(file_data)
    return data


def _image_names(label_dir):
    return [".".join(name.split(".")[:-1]) for name in sorted(os.listdir(label_dir))]


# ------------------------------------------------------------------------------ device TP matching
def box_correct_batch(dets, labels, iou_thr=0.5, device="cuda"):
    """TP flag of every detection of every image (lib/metrics.py:38-64 per image, all images in one
    launch).  dets[i] = (cls, xyxy, conf) or (); labels[i] = (cls, xyxy) or ().  Returns a list of
    (n_i, 1) bool arrays."""
    n = len(dets)
    dn = np.array([len(d[0]) if len(d) else 0 for d in dets], np.int64)
    ln = np.array([len(l[0]) if len(l) else 0 for l in labels], np.int64)
    doff = np.concatenate([[0], np.cumsum(dn)]).astype(np.int64)
    loff = np.concatenate([[0], np.cumsum(ln)]).astype(np.int64)
    dbox = np.concatenate([d[1] for d in dets if len(d)] or [np.zeros((0, 4))]).astype(np.float64)
    dcls = np.concatenate([d[0] for d in dets if len(d)] or [np.zeros(0)]).astype(np.int32)
    lbox = np.concatenate([l[1] for l in labels if len(l)] or [np.zeros((0, 4))]).astype(np.float64)
    lcls = np.concatenate([l[0] for l in labels if len(l)] or [np.zeros(0)]).astype(np.int32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    g_dbox, g_dcls, g_doff, g_lbox, g_lcls, g_loff = (t(a) for a in (dbox if len(dbox) else np.zeros((1, 4)),
                                                                      dcls if len(dcls) else np.zeros(1, np.int32),
                                                                      doff,
                                                                      lbox if len(lbox) else np.zeros((1, 4)),
                                                                      lcls if len(lcls) else np.zeros(1, np.int32),
                                                                      loff))
    tp = torch.zeros(max(int(doff[-1]), 1), dtype=torch.uint8, device=device)
    ops.check(ops.lib().edgedet_box_correct(ops._ptr(g_dbox), ops._ptr(g_dcls), ops._ptr(g_doff), ops._ptr(g_lbox),
                                            ops._ptr(g_lcls), ops._ptr(g_loff), n, float(iou_thr), ops._ptr(tp),
                                            int(ln.max(initial=0)), ops.stream_handle()))
    tp = tp.cpu().numpy().astype(bool)
    return [tp[doff[i]:doff[i + 1]].reshape(-1, 1) for i in range(n)]


def set_data(weak, strong, label, device="cuda"):
    """lib/data.py:46-84: (weak_data, strong_data, labels) with weak/strong entries (tp (n,1) bool,
    conf, cls) and labels[i] the label classes; TP matching on the device."""
    img_names = _image_names(label)
    weak_raw = load_data(weak, img_names, True)
    strong_raw = load_data(strong, img_names, True)
    lab_raw = load_data(label, img_names)
    w_tp = box_correct_batch(weak_raw, lab_raw, device=device)
    s_tp = box_correct_batch(strong_raw, lab_raw, device=device)
    weak_data, strong_data, labels = [], [], []
    for w, s, l, wt, st in zip(weak_raw, strong_raw, lab_raw, w_tp, s_tp):
        weak_data.append((wt, w[2], w[0]) if len(w) else (np.zeros((0, 1), bool), np.array([]), np.array([])))
        strong_data.append((st, s[2], s[0]) if len(s) else (np.zeros((0, 1), bool), np.array([]), np.array([])))
        labels.append(l[0] if len(l) else np.array([]))
    return weak_data, strong_data, labels


# ------------------------------------------------------------------------------ ORIE
def ensembles(num_img, num_ensemble, seed, targets=None):
    """reward.py:27-38 ensemble draws, serial and seeded: np.random.seed(seed + i) before image i."""
    E = min(max(num_ensemble, 0), max(num_img - 1, 0))
    targets = range(num_img) if targets is None else targets
    out = np.zeros((len(targets), E), np.int32)
    for r, i in enumerate(targets):
        np.random.seed(seed + i)
        idx = np.arange(num_img - 1)
        if i < num_img - 1:
            idx[i:] += 1
        out[r] = np.random.permutation(idx)[:E]
    return E, out


def _entries(weak_data, strong_data, labels):
    """Sorted detection entries (the reference's per-evaluation argsort, done once for the dataset)."""
    lab_cls = np.unique(np.concatenate([np.asarray(l, np.int64) for l in labels if len(l)] or [np.zeros(0, np.int64)]))
    C = len(lab_cls)
    N = len(labels)
    lab_cnt = np.zeros((N, max(C, 1)), np.int32)
    for i, l in enumerate(labels):
        if len(l):
            ci = np.searchsorted(lab_cls, np.asarray(l, np.int64))
            np.add.at(lab_cnt[i], ci, 1)
    parts = []
    for strong, data in ((0, weak_data), (1, strong_data)):
        for i, (tp, conf, cls) in enumerate(data):
            if len(conf) == 0:
                continue
            cls = np.asarray(cls, np.int64)
            pos = np.searchsorted(lab_cls, cls)
            keep = (pos < C) & (lab_cls[np.minimum(pos, max(C - 1, 0))] == cls) if C else np.zeros(len(cls), bool)
            if not keep.any():
                continue
            rows = np.nonzero(keep)[0]
            parts.append((pos[keep], np.asarray(conf, np.float64)[keep], np.full(len(rows), i), rows,
                          np.full(len(rows), strong), np.asarray(tp)[keep, 0]))
    if parts:
        ci, conf, img, row, st, tp = (np.concatenate(x) for x in zip(*parts))
    else:
        ci = conf = img = row = st = tp = np.zeros(0)
    order = np.lexsort((st, row, img, -conf, ci))
    ci = ci[order].astype(np.int64)
    seg = np.searchsorted(ci, np.arange(C + 1)).astype(np.int64)
    flag = (tp[order].astype(np.uint8) | (st[order].astype(np.uint8) << 1)).astype(np.uint8)
    return C, lab_cnt, img[order].astype(np.int32), flag, seg


def orie_maps(weak_data, strong_data, labels, num_ensemble=1000, seed=0, targets=None, device="cuda"):
    """Per target image: (ap_weak[C], ap_strong[C], n_l[C]) over the image's ensemble (device)."""
    N = len(labels)
    targets = np.arange(N, dtype=np.int32) if targets is None else np.asarray(targets, np.int32)
    E, ens = ensembles(N, num_ensemble, seed, targets)
    C, lab_cnt, ent_img, ent_flag, seg = _entries(weak_data, strong_data, labels)
    n_eval = len(targets)
    if C == 0 or n_eval == 0:
        return E, np.zeros((n_eval, 2, 0)), np.zeros((n_eval, 0), np.int32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    g = [t(a if len(a) else np.zeros(1, a.dtype)) for a in (ent_img, ent_flag)]
    g_seg, g_lab, g_tgt = t(seg), t(lab_cnt), t(targets)
    g_ens = t(ens if ens.size else np.zeros((n_eval, 1), np.int32))
    ap = torch.zeros((n_eval, 2, C), dtype=torch.float64, device=device)
    nl = torch.zeros((n_eval, C), dtype=torch.int32, device=device)
    ops.check(ops.lib().edgedet_orie_ap(ops._ptr(g[0]), ops._ptr(g[1]), ops._ptr(g_seg), C, ops._ptr(g_lab), N,
                                        ops._ptr(g_tgt), ops._ptr(g_ens), E, n_eval, ops._ptr(ap), ops._ptr(nl),
                                        ops.stream_handle()))
    return E, ap.cpu().numpy(), nl.cpu().numpy()


def orie_from_maps(E, ap, nl):
    """reward.py:47-51 + main's NaN handling: (mean(strong AP) - mean(weak AP)) * (E + 1) over the
    ensemble's label classes (np.unique order), NaN -> 0."""
    out = np.zeros(len(ap))
    with np.errstate(invalid="ignore", divide="ignore"):
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            for r in range(len(ap)):
                u = nl[r] > 0
                weak_map = ap[r, 0, u][:, np.newaxis]
                strong_map = ap[r, 1, u][:, np.newaxis]
                out[r] = (np.mean(strong_map) - np.mean(weak_map)) * (E + 1)
    return np.where(np.isnan(out), 0, out)


def compute_orie_all(weak_data, strong_data, labels, num_ensemble=1000, seed=0, targets=None, device="cuda"):
    E, ap, nl = orie_maps(weak_data, strong_data, labels, num_ensemble, seed, targets, device)
    return orie_from_maps(E, ap, nl)


def compute_dcsb(img_idx, weak_data, strong_data):
    """reward.py:55-69."""
    return np.sum(strong_data[img_idx][1] > 0.5) - np.sum(weak_data[img_idx][1] > 0.5)


def main(opts):
    if not torch.cuda.is_available():
        raise RuntimeError("edgeml_amd.reward needs an MI355X (HIP) device; there is no CPU path")
    from . import distributed as dist_mod
    rank, world = dist_mod.ensure_initialized()
    device = f"cuda:{dist_mod.device_index()}"
    torch.cuda.set_device(device)
    weak_data, strong_data, labels = set_data(opts.weak_dir, opts.strong_dir, opts.label_dir, device)
    num_img = len(labels)
    start = time.perf_counter()
    if opts.method == "orie":
        mine = dist_mod.shard(list(range(num_img)), rank, world)
        vals = compute_orie_all(weak_data, strong_data, labels, opts.num_ensemble, opts.seed, mine, device)
        reward = dist_mod.gather_values(vals, mine, num_img, rank, world) if world > 1 else vals
    else:
        reward = np.array([compute_dcsb(i, weak_data, strong_data) for i in range(num_img)], dtype=int)
    execution_time = time.perf_counter() - start
    if rank == 0:
        print(f"Program takes {execution_time:.1f} seconds ({execution_time / 60:.1f}m/{execution_time / 3600:.2f}h).")
        Path(opts.save_dir).mkdir(parents=True, exist_ok=True)
        name = f"orie{opts.num_ensemble}.npz" if opts.method == "orie" else "dcsb.npz"
        np.savez(os.path.join(opts.save_dir, name), reward=reward, time=execution_time)
    return reward if rank == 0 else None


def getargs(argv=None):
    """reward.py:96-111 (same arguments and defaults) + --seed."""
    args = argparse.ArgumentParser()
    args.add_argument('weak_dir', help="Directory to the weak detector output files.")
    args.add_argument('strong_dir', help="Directory to the strong detector output files.")
    args.add_argument('label_dir', help="Directory to the ground truth annotations.")
    args.add_argument('save_dir', help="Directory to save the computed computed offloading rewards.")
    args.add_argument('--method', type=str, default="orie", choices=['orie', 'dcsb'],
                      help="Method used to compute the offloading reward.")
    args.add_argument('--num-ensemble', type=int, default=1000,
                      help="Number of ensemble images when computing the offloading reward.")
    args.add_argument('--seed', type=int, default=0, help="Ensemble draws: np.random.seed(seed + image index).")
    return args.parse_args(argv)


if __name__ == '__main__':
    main(getargs())
