"""MI355X-native detection-output collection (the hot path of torch_models/detect.py).

Public surface (mirrors the reference):
  * ``detect.load_weak_models(model_name, model_path, num_class)``   — detect.py:15-42
  * detector objects with the torchvision detection contract       — detect.py:72-81
    (``models.SSDLite320``, ``models.FasterRCNNFPNv2``)
  * ``detect.main`` / ``detect.getargs``                            — detect.py:62-121
  * ``fmt.format_detections`` / ``labelmap.coco_to_yolov5``         — detect.py:79-105, coco_labelmap.py
  * ``distributed`` — one process per GPU, contiguous shards, RCCL gather of the output rows
Compute runs in hand-written HIP kernels (csrc/, built into libedgedet.so by build.py); ``ops.lib()``
raises when the library is missing — there is no CPU fallback.
"""
__all__ = ["arch", "synthetic", "anchors", "ops", "plan", "models", "detect", "fmt", "labelmap", "distributed",
           "build"]
