"""Drop-in for test.py: realized mAP against the offloading ratio, ap_per_class on the GPU.

    python -m edgeml_amd.evaluate weak_dir strong_dir label_dir split_path save_dir --estimates DIR [DIR ...]

Same arguments and the same ``test_map.npy`` ([len(estimates), 11] float64) as test.py:47-76.  The
offload masks (test.py:30-38: per fold, the training estimates' threshold at each ratio applied to the
validation estimates) are host logic as in the reference; every mixture's ap_per_class
(test.py:39-42, lib/metrics.py:89-148) runs in csrc/orie.hip (edgedet_map_eval), bit-identical to
numpy's when confidences are distinct (equal confidences: (image, row) order, see reward.py).
"""
import argparse
import os
from pathlib import Path

import numpy as np
import torch

from . import ops
from .reward import _entries, set_data

offloading_ratios = np.arange(0, 1.01, 0.1)


def offload_masks(reward_estimates, dataset_split, n_img):
    """test.py:27-38 for every estimate: bool [len(estimates), len(ratios), n_img]."""
    out = np.zeros((len(reward_estimates), len(offloading_ratios), n_img), dtype=bool)
    for e, estimate_path in enumerate(reward_estimates):
        for cv_idx, val_mask in enumerate(dataset_split):
            reward_data = np.load(os.path.join(estimate_path, f"estimate{cv_idx + 1}.npz"))
            train_reward, val_reward = reward_data['train_est'], reward_data['val_est']
            for ratio_idx, offload_ratio in enumerate(offloading_ratios):
                reward_thresh = train_reward[np.argsort(-train_reward)[int((len(train_reward) - 1) * offload_ratio)]]
                out[e, ratio_idx, val_mask] = val_reward > reward_thresh
    return out


def _bits(mask):
    """bool [..., n] -> uint32 bitmaps [..., (n + 31) // 32] (bit i of word i // 32)."""
    n = mask.shape[-1]
    w = (n + 31) // 32
    pad = np.zeros(mask.shape[:-1] + (w * 32,), dtype=bool)
    pad[..., :n] = mask
    return np.packbits(pad.reshape(mask.shape[:-1] + (w, 32)), axis=-1, bitorder="little").view(np.uint32)[..., 0]


def map_of_mixtures(weak_data, strong_data, labels, strong_masks, device="cuda"):
    """mAP (np.mean of ap_per_class) of each weak/strong mixture; strong_masks bool [M, n_img]."""
    C, lab_cnt, ent_img, ent_flag, seg = _entries(weak_data, strong_data, labels)
    strong_masks = np.asarray(strong_masks, dtype=bool).reshape(-1, len(labels))
    M = len(strong_masks)
    if C == 0:
        return np.full(M, np.nan)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    g = [t(a if len(a) else np.zeros(1, a.dtype)) for a in (ent_img, ent_flag)]
    wm, sm = t(_bits(~strong_masks).view(np.int32)), t(_bits(strong_masks).view(np.int32))
    g_seg, g_lab = t(seg), t(lab_cnt)  # named: the device buffers must outlive the asynchronous launch
    ap = torch.zeros((M, 2, C), dtype=torch.float64, device=device)
    nl = torch.zeros((M, C), dtype=torch.int32, device=device)
    ops.check(ops.lib().edgedet_map_eval(ops._ptr(g[0]), ops._ptr(g[1]), ops._ptr(g_seg), C, ops._ptr(g_lab),
                                         len(labels), ops._ptr(wm), ops._ptr(sm), M, ops._ptr(ap), ops._ptr(nl),
                                         ops.stream_handle()))
    ap, nl = ap.cpu().numpy(), nl.cpu().numpy()
    out = np.zeros(M)
    for r in range(M):
        out[r] = np.mean(ap[r, 0, nl[r] > 0][:, np.newaxis])
    return out


def test_map(weak_data, strong_data, labels, reward_estimates, dataset_split, device="cuda"):
    """test.py:14-44: [len(estimates), len(ratios)] realized mAP."""
    masks = offload_masks(reward_estimates, dataset_split, len(weak_data))
    res = map_of_mixtures(weak_data, strong_data, labels, masks.reshape(-1, len(weak_data)), device)
    return res.reshape(len(reward_estimates), len(offloading_ratios))


test_map.__test__ = False  # not a pytest test


def main(opts):
    if not torch.cuda.is_available():
        raise RuntimeError("edgeml_amd.evaluate needs an MI355X (HIP) device; there is no CPU path")
    weak_data, strong_data, labels = set_data(opts.weak_dir, opts.strong_dir, opts.label_dir)
    dataset_split = np.load(opts.split_path)
    estimates = []
    if isinstance(opts.estimates, list):
        estimates = opts.estimates
    elif opts.estimates is not None:
        estimates = [opts.estimates]
    map_result = test_map(weak_data, strong_data, labels, estimates, dataset_split)
    Path(opts.save_dir).mkdir(parents=True, exist_ok=True)
    np.save(os.path.join(opts.save_dir, 'test_map.npy'), map_result)
    return map_result


def getargs(argv=None):
    """test.py:64-73."""
    args = argparse.ArgumentParser()
    args.add_argument('weak_dir', help="Directory to the weak detector output files.")
    args.add_argument('strong_dir', help="Directory to the strong detector output files.")
    args.add_argument('label_dir', help="Directory to the ground truth annotations.")
    args.add_argument('split_path', help="Path to the dataset split (for cross validation).")
    args.add_argument('save_dir', help="Directory to save the achieved mAP.")
    args.add_argument('--estimates', nargs='+', type=str, help='Directories to the reward estimation file(s).')
    return args.parse_args(argv)


if __name__ == '__main__':
    main(getargs())
