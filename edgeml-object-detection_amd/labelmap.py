"""COCO-91 category id -> YOLOv5-80 class index (torch_models/coco_labelmap.py:2-94).

The 11 ids that are not COCO-2017 detection categories (0 = background, 12, 26, 29, 30, 45, 66,
68, 69, 71, 83) map to -1 and are dropped by detect.py:94-95; the remaining 80 ids map to 0..79 in
increasing order.  Pinned byte-for-byte against the reference's dict by tests/golden/g1_format.npz.
"""
import numpy as np

DROPPED = (0, 12, 26, 29, 30, 45, 66, 68, 69, 71, 83)


def _build():
    table, nxt = {}, 0
    for cid in range(91):
        if cid in DROPPED:
            table[cid] = -1
        else:
            table[cid] = nxt
            nxt += 1
    return table


coco_to_yolov5 = _build()
COCO_TO_YOLOV5 = np.asarray([coco_to_yolov5[i] for i in range(91)], dtype=np.int64)
