"""Drop-in for data_processing/extract_feature.py (lib/data.py:127-160 extract_output_feature): the
stage-24 "output features" of the regression estimators, computed for every image in one device
launch (csrc/orie.hip output_feature_kernel).

    python -m edgeml_amd.features output_dir save_dir label_dir [--k 25] [--dataset coco|voc]

Writes <save_dir>/<image>/stage24_output_features.npy, float64 [num_class + 5 k], like the reference.
"""
import argparse
import os
from pathlib import Path

import numpy as np
import torch

from . import ops


def _read_rows(output_path, img):
    fn = os.path.join(output_path, img)
    if os.path.isfile(fn + ".txt"):
        with open(fn + ".txt", "r") as f:
            data = [line.strip().split(" ") for line in f.readlines()]
        return np.array(data, dtype=float) if len(data) else np.zeros((0, 6))
    if os.path.isfile(fn + ".npy"):
        return np.asarray(np.load(fn + ".npy", allow_pickle=False), dtype=float)
    return np.zeros((0, 6))


def output_features(rows_per_image, num_class, k=25, device="cuda"):
    """[n_img, num_class + (ncol - 1) * k] float64 features from each image's detection rows."""
    ncol = max([r.shape[1] for r in rows_per_image if r.ndim == 2 and len(r)] or [6])
    rows = [np.asarray(r, dtype=np.float64).reshape(-1, ncol) if len(r) else np.zeros((0, ncol)) for r in rows_per_image]
    off = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    flat = np.concatenate(rows + [np.zeros((1, ncol))], 0)
    n = len(rows)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    out = torch.zeros((max(n, 1), num_class + (ncol - 1) * k), dtype=torch.float64, device=device)
    g_rows, g_off = t(flat), t(off)  # named: the device buffers must outlive the asynchronous launch
    ops.check(ops.lib().edgedet_output_features(ops._ptr(g_rows), ops._ptr(g_off), n, ncol, num_class, k,
                                                ops._ptr(out), ops.stream_handle()))
    return out[:n].cpu().numpy()


def extract_output_feature(output_path, feature_path, num_class, k=25, device="cuda"):
    """lib/data.py:127-160 (same file layout)."""
    img_names = sorted([f for f in os.listdir(feature_path) if not os.path.isfile(os.path.join(feature_path, f))])
    feats = output_features([_read_rows(output_path, n) for n in img_names], num_class, k, device)
    for n, f in zip(img_names, feats):
        np.save(os.path.join(feature_path, n, "stage24_output_features.npy"), f)


def main(opts):
    """data_processing/extract_feature.py:15-24."""
    num_class = 20 if opts.dataset == "voc" else 80
    img_names = ['.'.join(f.split('.')[:-1]) for f in sorted(os.listdir(opts.label_dir))]
    for img_name in img_names:
        Path(os.path.join(opts.save_dir, img_name)).mkdir(parents=True, exist_ok=True)
    new_img_names = sorted([f for f in os.listdir(opts.save_dir) if not os.path.isfile(os.path.join(opts.save_dir, f))])
    assert len(img_names) == len(new_img_names) and all(i == n for i, n in zip(img_names, new_img_names))
    extract_output_feature(opts.output_dir, opts.save_dir, num_class, opts.k)


def getargs(argv=None):
    args = argparse.ArgumentParser()
    args.add_argument('output_dir', help="Directory to the (weak detector's) detection output files.")
    args.add_argument('save_dir', help="Directory to save the extracted features.")
    args.add_argument('label_dir', help="Directory to the ground truth annotations.")
    args.add_argument('--k', type=int, default=25, help="Top-K bounding boxes to collect.")
    args.add_argument('--dataset', type=str, default="coco", help="The dataset to process ('coco' or 'voc').")
    return args.parse_args(argv)


if __name__ == '__main__':
    main(getargs())
