"""Detection -> YOLO-row formatting of torch_models/detect.py:79-105 (the file boundary to reward.py).

``format_detections`` reproduces the reference's numpy arithmetic exactly (float32 centre/size math,
label map, mask, division by the ORIGINAL width/height as Python ints, concatenation that promotes
to float64), so the .npy bytes written by ``save_npy`` are identical to the reference's for the same
boxes/scores/labels (pinned by tests/golden/g1_format.npz).
"""
import os

import numpy as np

from .labelmap import coco_to_yolov5

# coco_to_yolov5 as a lookup table (ids 0..90), for the vectorised batch formatter
_COCO_LUT = np.array([coco_to_yolov5[i] for i in range(max(coco_to_yolov5) + 1)], dtype=np.int64)


def format_detections(boxes, scores, labels, img_height, img_width, dataset="coco"):
    """boxes [K,4] float32 xyxy (original pixels), scores [K] float32, labels [K] int64 -> (N,6) float64."""
    boxes = np.asarray(boxes, dtype=np.float32).reshape(-1, 4)
    scores = np.asarray(scores, dtype=np.float32).reshape(-1)
    labels = np.asarray(labels, dtype=np.int64).reshape(-1)
    x_center = boxes[:, 0] + (boxes[:, 2] - boxes[:, 0]) / 2
    y_center = boxes[:, 1] + (boxes[:, 3] - boxes[:, 1]) / 2
    width = boxes[:, 2] - boxes[:, 0]
    height = boxes[:, 3] - boxes[:, 1]
    if dataset == "coco":
        labels = np.array([coco_to_yolov5[l] for l in labels])
    else:
        labels = labels - 1
    label_mask = labels != -1
    labels = labels[label_mask]
    x_center = x_center[label_mask] / img_width
    y_center = y_center[label_mask] / img_height
    width = width[label_mask] / img_width
    height = height[label_mask] / img_height
    scores = scores[label_mask]
    return np.concatenate((labels[:, np.newaxis], x_center[:, np.newaxis], y_center[:, np.newaxis],
                           width[:, np.newaxis], height[:, np.newaxis], scores[:, np.newaxis]), axis=1)


def format_batch(boxes, scores, labels, counts, img_height, img_width, dataset="coco"):
    """format_detections for a batch of equal-size images at once: boxes [B,K,4], scores [B,K],
    labels [B,K] padded per image, counts [B] -> list of (N_b,6) float64, each byte-identical to
    format_detections(boxes[b,:n_b], scores[b,:n_b], labels[b,:n_b], ...) (the same float32
    element-wise ops, the label map as a table lookup, the same promotion to float64)."""
    boxes = np.asarray(boxes, dtype=np.float32)
    scores = np.asarray(scores, dtype=np.float32)
    labels = np.asarray(labels, dtype=np.int64)
    x_center = boxes[..., 0] + (boxes[..., 2] - boxes[..., 0]) / 2
    y_center = boxes[..., 1] + (boxes[..., 3] - boxes[..., 1]) / 2
    width = boxes[..., 2] - boxes[..., 0]
    height = boxes[..., 3] - boxes[..., 1]
    valid = np.arange(labels.shape[1])[None, :] < np.asarray(counts).reshape(-1, 1)
    lab = np.where(valid, labels, 1)
    lab = _COCO_LUT[lab] if dataset == "coco" else lab - 1
    keep = valid & (lab != -1)
    cols = np.stack([lab.astype(np.float64), (x_center / img_width).astype(np.float64),
                     (y_center / img_height).astype(np.float64), (width / img_width).astype(np.float64),
                     (height / img_height).astype(np.float64), scores.astype(np.float64)], axis=-1)
    return [cols[b][keep[b]] for b in range(len(cols))]


def output_name(img_name):
    """detect.py:104 strips the last four characters (a 3-letter extension)."""
    return img_name[:-4]


def save_npy(save_dir, img_name, rows):
    path = os.path.join(save_dir, output_name(img_name) + ".npy")
    tmp = path + ".tmp.npy"
    np.save(tmp, rows)
    os.replace(tmp, path)  # never leave a partial file behind
    return path
