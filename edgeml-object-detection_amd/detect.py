"""Drop-in for torch_models/detect.py: same CLI, same output files, MI355X engine underneath.

    python -m edgeml_amd.detect img_dir save_dir [--dataset coco|voc] [--model ssd|faster_rcnn]
                                [--model-path PATH]

Behaviour kept from the reference (detect.py:62-106): images are taken in sorted(os.listdir) order,
read as RGB and scaled by 1/255, every image gets one ``<name[:-4]>.npy`` (N,6) float64 file
``[cls, xc, yc, w, h, conf]`` normalised by the original size, rows in score order, an empty result
still writes a (0,6) file.  Differences: images of equal size are batched across the whole list
(results are per image, but their last bits depend on the batch an image runs in: conv tiles are
chosen per batch size, so a different summation order can move a score by float32 rounding; the
grouping is a fixed function of the sorted list, so a given list always gives the same files) and
decoded ahead of the engine (baseline JPEGs:
Huffman decoding on a host thread pool, IDCT / upsampling / colour conversion on the GPU, csrc/jpeg.hip,
byte-identical to the host decoder; other files on the host),
and under ``torchrun`` the single-process run's batch list is split into contiguous blocks of
batches, one per GPU (so every file is byte-identical whatever the GPU count), with the output rows
gathered to rank 0 over RCCL (distributed.py).
"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np
import torch

from . import fmt, models


def load_weak_models(model_name: str, model_path: str, num_class: int):
    """detect.py:15-42.  ``model_path == ""`` asks the reference for downloaded COCO weights (a
    91-class model whatever --dataset says); offline this build substitutes seeded synthetic weights
    of the same architecture (edgeml_amd.synthetic).  Any other model name is RetinaNet
    (detect.py:34-38)."""
    sd = None
    if model_path != "":
        ckpt = torch.load(model_path, map_location="cpu", weights_only=True)
        sd = ckpt["model"] if isinstance(ckpt, dict) and "model" in ckpt and not torch.is_tensor(ckpt["model"]) \
            else ckpt
    if model_name == "ssd":
        if sd is None:
            return models.ssdlite320_mobilenet_v3_large(weights="DEFAULT")
        reduced = tuple(sd["backbone.features.1.3.0.weight"].shape)[1] == 80
        return models.SSDLite320(sd, num_class, reduced)
    if model_name == "faster_rcnn":
        if sd is None:
            return models.fasterrcnn_resnet50_fpn_v2(weights="DEFAULT")
        return models.FasterRCNNFPNv2(sd, num_class)
    if sd is None:
        return models.retinanet_resnet50_fpn_v2(weights="DEFAULT")
    return models.RetinaNetFPNv2(sd, num_class)


def read_image(path, out=None):
    """torchvision.io.read_image(path, ImageReadMode.RGB) -> uint8 [3,H,W] (PIL decoder); with `out`
    the image is written into that [3,H,W] uint8 tensor (a slot of a pinned batch buffer)."""
    from PIL import Image
    with Image.open(path) as im:
        arr = np.asarray(im.convert("RGB"), dtype=np.uint8)
    # the HWC -> CHW copy in numpy (single-threaded): this runs on the decode pool's threads, where a
    # torch copy would start its own intra-op thread team per call (measured 10x slower on a
    # 16-core share of a 256-core host)
    if out is not None:
        np.copyto(out.numpy(), arr.transpose(2, 0, 1))
        return out
    return torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1)))


class ObjectDetectionDataset:
    """detect.py:45-59."""

    def __init__(self, img_dir, names=None):
        self.img_dir = img_dir
        self.img_names = sorted(os.listdir(img_dir)) if names is None else list(names)

    def __len__(self):
        return len(self.img_names)

    def __getitem__(self, idx):
        return self.read_u8(idx) / 255

    def read_u8(self, idx, out=None):
        """The decoded uint8 [3,H,W] image (detect.py:57) before its `/ 255` (detect.py:58): the CLI
        uploads these bytes and the engine divides on the device, bit-identically."""
        return read_image(os.path.join(self.img_dir, self.img_names[idx]), out)


def _image_size(path):
    from PIL import Image
    with Image.open(path) as im:  # header only
        return im.size[1], im.size[0]


def image_sizes(dataset, workers=None):
    """(H, W) of every image of the dataset, from the file headers (no decode): JPEG / PNG headers parsed
    natively on host threads (edgedet_image_dims), any other file through PIL's header reader."""
    import ctypes
    import concurrent.futures as cf
    from . import ops
    from .distributed import usable_cpus
    paths = [os.path.join(dataset.img_dir, n) for n in dataset.img_names]
    n = len(paths)
    hw = np.zeros((n, 2), np.int32)
    if n:
        arr = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
        ops.lib().edgedet_image_dims(ctypes.cast(arr, ctypes.c_void_p), n, hw.ctypes.data, workers or usable_cpus())
    sizes = [(int(h), int(w)) for h, w in hw]
    rest = [i for i, (h, w) in enumerate(sizes) if h <= 0 or w <= 0]
    if rest:
        with cf.ThreadPoolExecutor(workers or usable_cpus()) as ex:
            for i, s in zip(rest, ex.map(_image_size, [paths[i] for i in rest])):
                sizes[i] = s
    return sizes


def _decoded_batches(dataset, chunks, sizes, workers=None, device_decode=True):
    """Yield (names, (H, W), batch) for the given batches of equal-size images (lists of dataset
    indices, distributed.size_batches).  With device_decode, a batch of JPEG files the device decoder
    handles is entropy-decoded by one library call on all usable host cores into one pinned buffer
    (jpeg.PackedBatch; reconstructed on the GPU by run_batches straight into the plan's input,
    byte-identical to the host decode); otherwise (another format, or a JPEG the device path does not
    take) the images are decoded on the host (PIL, one thread per usable core) straight into their
    slots of a pinned uint8 batch buffer.  The next two batches are in flight while the caller uses the
    current one."""
    import concurrent.futures as cf
    from . import jpeg
    from .distributed import usable_cpus
    workers = workers or usable_cpus()
    paths = [os.path.join(dataset.img_dir, n) for n in dataset.img_names]
    pin = torch.cuda.is_available()
    # packed batches one after another on one thread (each call uses every core); host decodes per image
    with cf.ThreadPoolExecutor(1) as packer, cf.ThreadPoolExecutor(workers) as ex:

        def host(c):
            h, w = sizes[c[0]]
            buf = torch.empty((len(c), 3, h, w), dtype=torch.uint8, pin_memory=pin)
            return "host", buf, [ex.submit(dataset.read_u8, i, buf[k]) for k, i in enumerate(c)]

        def sub(c):
            if device_decode and all(paths[i][-4:].lower() in (".jpg", "jpeg", ".jpe") for i in c):
                return "pk", None, [packer.submit(jpeg.batch_packets, [paths[i] for i in c], workers, pin)]
            return host(c)

        fut = [sub(c) for c in chunks[:2]]
        for j, c in enumerate(chunks):
            kind, buf, fs = fut[j]
            res = [f.result() for f in fs]
            if kind == "pk" and res[0] is None:  # a file the device path does not take
                kind, buf, fs = host(c)
                res = [f.result() for f in fs]
            if j + 2 < len(chunks):
                fut.append(sub(chunks[j + 2]))
            fut[j] = None
            yield [dataset.img_names[i] for i in c], sizes[c[0]], (res[0] if kind == "pk" else buf)


def detect_rows(model, images, dataset="coco"):
    """Run the engine on a list of [3,H,W] float images; return the .npy rows per image."""
    preds = model(images)
    rows = []
    for img, p in zip(images, preds):
        rows.append(fmt.format_detections(p["boxes"].cpu().numpy(), p["scores"].cpu().numpy(),
                                          p["labels"].cpu().numpy(), int(img.shape[-2]), int(img.shape[-1]),
                                          dataset))
    return rows


def main(opts):
    from . import distributed as dist_mod
    import time
    clock = [("start", time.perf_counter())]  # EDGEDET_DETECT_TIMING=1: phase times to stderr
    img_names = sorted(os.listdir(opts.img_dir))
    if not torch.cuda.is_available():
        raise RuntimeError("edgeml_amd.detect needs an MI355X (HIP) device; there is no CPU path")
    rank, world = dist_mod.ensure_initialized()
    dataset = ObjectDetectionDataset(opts.img_dir, img_names)
    num_class = 91 if opts.dataset == "coco" else 21
    device = f"cuda:{dist_mod.device_index()}"
    torch.cuda.set_device(device)
    if rank == 0:
        print(f"Using {device} device (world {world})")
    model = load_weak_models(opts.model, opts.model_path, num_class).to(device)
    model.eval()
    clock.append(("model", time.perf_counter()))
    Path(opts.save_dir).mkdir(parents=True, exist_ok=True)
    batch = min(getattr(opts, "batch", None) or model.max_batch, model.max_batch)
    results = {}
    # Batches of equal-size images across the whole list (sizes from the file headers, no decode),
    # formed exactly as a single-process run forms them; under torchrun each rank takes a contiguous
    # block of those batches balanced by the model's per-batch work, so outputs are independent of the
    # GPU count.  Decoded by a thread pool
    # one batch ahead of the engine (PIL releases the GIL while decoding).  Up to model.INFLIGHT
    # batches on the device at once (run_batches), so one batch's NMS tail overlaps the next
    # batch's backbone.
    sizes = image_sizes(dataset)
    clock.append(("sizes", time.perf_counter()))
    chunks = dist_mod.size_batches(sizes, batch)
    work = lambda c: model.batch_work(len(c), *sizes[c[0]])  # noqa: E731
    shards = [dist_mod.batch_shard(chunks, r, world, work) for r in range(world)]
    shard_names = [[img_names[i] for c in sh for i in c] for sh in shards]
    my_names = shard_names[rank]
    tagged = (((names, hw), buf) for names, hw, buf in
              _decoded_batches(dataset, shards[rank], sizes, device_decode=getattr(opts, "decode", "gpu") == "gpu"))
    # the .npy files are written by a thread pool: under one process as each batch's rows are ready
    # (overlapping the engine), under torchrun by rank 0 after the gather
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(dist_mod.usable_cpus()) as writers:
        pending = []
        for (names, (h, w)), counts, boxes, scores, labels in model.run_batches(tagged, raw=True):
            for name, rows in zip(names, fmt.format_batch(boxes, scores, labels, counts, h, w, opts.dataset)):
                results[name] = rows
                if world == 1:
                    pending.append(writers.submit(fmt.save_npy, opts.save_dir, name, rows))
        clock.append(("engine", time.perf_counter()))
        if world > 1:
            results = dist_mod.gather_rows(results, my_names, img_names, rank, world, shards=shard_names)
            if rank == 0:
                pending = [writers.submit(fmt.save_npy, opts.save_dir, name, results[name]) for name in img_names]
        for f in pending:
            f.result()  # re-raise a failed write
    clock.append(("files", time.perf_counter()))
    if os.environ.get("EDGEDET_DETECT_TIMING") == "1":
        print("detect timing (s): " + ", ".join(f"{k} {b - a:.3f}" for (_, a), (k, b) in zip(clock, clock[1:])) +
              f", images {len(my_names)}; engine phases (s): " +
              ", ".join(f"{k} {v:.3f}" for k, v in getattr(model, "phase_s", {}).items()), file=sys.stderr, flush=True)
    return results if rank == 0 else None


def getargs(argv=None):
    """detect.py:109-121 (same positional/optional arguments and defaults) + --batch, --decode."""
    args = argparse.ArgumentParser()
    args.add_argument('img_dir', help="Directory that saves the image dataset for detection.")
    args.add_argument('save_dir', help="Directory to save the detection outputs.")
    args.add_argument('--dataset', type=str, default="coco", help="The dataset to process ('coco' or 'voc').")
    args.add_argument('--model', type=str, default="ssd",
                      help="The object detector: 'ssd', 'faster_rcnn', anything else = RetinaNet.")
    args.add_argument("--model-path", type=str, default="",
                      help="Location of the saved object detection model weights (torchvision state_dict keys).")
    args.add_argument("--batch", type=int, default=0, help="Images per engine call (0 = model default).")
    args.add_argument("--decode", choices=("gpu", "host"), default="gpu",
                      help="JPEG decode: entropy decode on the host + reconstruction on the GPU (byte-identical), "
                           "or the whole decode on the host (PIL).")
    return args.parse_args(argv)


if __name__ == '__main__':
    main(getargs())
    sys.exit(0)
