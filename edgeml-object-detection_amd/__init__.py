"""MI355X-native detection-output collection (the hot path of torch_models/detect.py).

Public surface (mirrors the reference):
  * ``load_weak_models(model_name, model_path, num_class)``  — detect.py:15-42
  * detector objects with the torchvision detection contract — detect.py:72-81
  * ``detect.main`` / ``detect.getargs``                      — detect.py:62-121
Compute runs in hand-written HIP kernels (csrc/, built into libedgedet.so); importing
``edgeml_amd.ops`` on a machine without the built library raises.
"""
__all__ = ["arch", "synthetic", "ops", "models", "detect", "fmt", "labelmap", "distributed"]
