"""The detectors of torch_models/detect.py on libedgedet.so.

``SSDLite320`` is torchvision's ``ssdlite320_mobilenet_v3_large`` (detect.py:24/26),
``FasterRCNNFPNv2`` is ``fasterrcnn_resnet50_fpn_v2`` (detect.py:30/32) and ``RetinaNetFPNv2`` is
``retinanet_resnet50_fpn_v2`` (detect.py:36/38).  They keep torchvision's detection-model contract
(detect.py:72-81): ``.to(device)``, ``.eval()``, ``.load_state_dict(sd)`` with torchvision's
state_dict keys, and ``model(Tensor[N,3,H,W] float32 in [0,1]) -> [{"boxes", "scores", "labels"}]``
with boxes in original pixels, scores descending, labels int64.

There is one lowering, the library's (csrc/lower.hip, also the C-ABI's ``edgedet_model_*``): the
state_dict is packed by ``edgedet_model_pack`` (BatchNorm folded, conv weights repacked and split into
bf16 planes) and each (batch, height, width, input dtype) becomes a plan.NativePlan: the library's op
records over a workspace this module allocates, with the named buffers the parity tests read.  This
module adds no arithmetic; every step runs in HIP kernels (ops.py fails loudly if the library is
missing).  Architecture and post-processing constants: SURVEY.md Appendix A.
"""
import math

import numpy as np
import time

import torch

from . import arch
from . import native
from . import ops
from .plan import NativePlan


def _check_keys(sd, table, what):
    missing = [k for k in table if k not in sd]
    unexpected = [k for k in sd if k not in table]
    bad = [k for k in table if k in sd and tuple(sd[k].shape) != tuple(table[k])]
    if missing or unexpected or bad:
        raise RuntimeError(f"Error(s) in loading state_dict for {what}: missing keys {missing[:5]}, "
                           f"unexpected keys {unexpected[:5]}, size mismatch {bad[:5]}")


class _Detector:
    kind = None
    max_batch = 32
    reduced_tail = True

    def __init__(self, state_dict, num_classes=91, device=None):
        self.num_classes = num_classes
        self.device = torch.device(device) if device is not None else None
        self.training = False
        self.plans = {}
        self.load_state_dict(state_dict)

    # torchvision-style surface ----------------------------------------------------------------
    def eval(self):
        self.training = False
        return self

    def train(self, mode=True):
        if mode:
            raise NotImplementedError("training is out of scope (SURVEY.md §2 row 7)")
        return self

    def to(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError(f"{type(self).__name__} runs on the MI355X HIP engine only (got {device}); "
                               f"there is no CPU fallback")
        self.device = device
        return self

    def cuda(self):
        return self.to("cuda")

    def load_state_dict(self, sd, strict=True):
        sd = {k: v for k, v in sd.items()}
        _check_keys(sd, self.table(), type(self).__name__)
        self.sd = sd
        self.blob = native.pack_state_dict(self.kind, sd, self.num_classes, self.reduced_tail)  # host uint8
        self._weights = {}
        self.plans = {}
        return self

    def state_dict(self):
        return dict(self.sd)

    def weights(self, device):
        """The packed weight blob on `device` (uploaded once per device, shared by every plan)."""
        key = str(torch.device(device))
        if key not in self._weights:
            self._weights[key] = torch.from_numpy(self.blob).to(device)
        return self._weights[key]

    def batch_work(self, B, H, W):
        """Relative device work of one batch of B images of H x W (the detect CLI's shard balance,
        distributed.batch_shard): proportional to the pixels the network runs on."""
        return float(B)

    def build_plan(self, B, H, W, u8=False):
        """A new plan of (B, H, W, u8) on this model's device (CPU when none is set: records and
        constants only, for host-side checks)."""
        return NativePlan(self, int(B), int(H), int(W), bool(u8), self.device or "cpu")

    # inference --------------------------------------------------------------------------------
    def plan(self, B, H, W, u8=False):
        """The plan of (B, H, W).  u8: the input buffer holds the decoded uint8 images
        (detect.py:57) and the transform divides by 255 on the device (bit-identical to the host's
        `image / 255`, detect.py:58); otherwise it holds the model contract's float images."""
        key = (int(B), int(H), int(W), bool(u8))
        if key not in self.plans:
            if self.device is None:
                self.to("cuda")
            self.plans[key] = self.build_plan(*key).finalize()
        return self.plans[key]

    @torch.no_grad()
    def __call__(self, images):
        if self.device is None:
            self.to("cuda")
        imgs = list(images) if not torch.is_tensor(images) or images.dim() == 3 else list(images.unbind(0))
        if torch.is_tensor(images) and images.dim() == 3:
            imgs = [images]
        results = [None] * len(imgs)
        groups = {}
        for idx, im in enumerate(imgs):
            groups.setdefault(tuple(im.shape[-2:]), []).append(idx)
        for (H, W), idxs in groups.items():
            for s in range(0, len(idxs), self.max_batch):
                chunk = idxs[s:s + self.max_batch]
                plan = self.plan(len(chunk), H, W)
                inp = plan.input.tensor()
                for j, idx in enumerate(chunk):
                    inp[j].copy_(imgs[idx].to(self.device, torch.float32), non_blocking=True)
                plan.run()
                counts = plan.out_count.tensor().cpu().tolist()
                boxes = plan.out_box.tensor()
                scores = plan.out_score.tensor()
                labels = plan.out_label.tensor()
                for j, idx in enumerate(chunk):
                    n = counts[j]
                    results[idx] = {"boxes": boxes[j, :n].clone(), "scores": scores[j, :n].clone(),
                                    "labels": labels[j, :n].clone()}
        return results

    forward = __call__

    INFLIGHT = 2  # batches on the device at once in run_batches (measured best on MI355X: bench --inflight)

    @torch.no_grad()
    def run_batches(self, batches, inflight=None, raw=False):
        """Yield (tag, [(boxes, scores, labels) host numpy arrays per image]) for each (tag, images) of
        `batches`, in order, with up to `inflight` batches on the device at once (raw=True: yield
        (tag, counts [B], boxes [B,K,4], scores [B,K], labels [B,K]) padded host arrays instead, the
        input of fmt.format_batch).  `images` is a list of [3,H,W] tensors or one [B,3,H,W] tensor; a
        pinned [B,3,H,W] tensor is uploaded as it is (no staging copy).  Each in-flight
        slot owns an independent plan (arena + outputs), a stream and pinned host staging, so batch
        k+1's upload and first layers run under batch k's low-occupancy NMS tail; a slot is reused
        only after its results have been copied to the host.  Images are either the model
        contract's float [3,H,W] tensors or the decoded uint8 [3,H,W] images (detect.py:57), which
        cross PCIe as bytes (4x fewer than float) and are divided by 255 on the device, bit-identical
        to the host's `image / 255` (detect.py:58).  Same arithmetic as __call__ (same plan
        lowering, same kernels, replayed from a hipGraph per slot)."""
        if self.device is None:
            self.to("cuda")
        n = max(1, int(inflight or self.INFLIGHT))
        # (B, H, W, u8) -> [slot dict] * n, kept on the model across calls (the plans, streams and
        # pinned buffers of a shape are built once)
        slots = self.__dict__.setdefault("_slots", {})
        for key in [k for k, v in slots.items() if len(v) != n]:
            del slots[key]
        pending = []  # (tag, slot, B)
        turn = [0]
        # host seconds per phase (EDGEDET_DETECT_TIMING: the detect CLI prints them): waiting for the
        # caller's next batch (its decode), building + capturing slot plans, issuing a batch (upload /
        # device decode, replay, D2H), waiting for a batch's results
        tm = self.__dict__.setdefault("phase_s", {})
        for k in ("input", "plans", "issue", "results", "caller"):
            tm.setdefault(k, 0.0)
        clk = [time.perf_counter()]

        def lap(k):
            t = time.perf_counter()
            tm[k] += t - clk[0]
            clk[0] = t

        def new_slot(key, first):
            B, H, W, u8 = key
            plan = self.plan(*key) if first else self.build_plan(*key).finalize()
            dt = torch.uint8 if u8 else torch.float32
            return {"plan": plan, "stream": torch.cuda.Stream(self.device), "jpeg": None,
                    "stage": torch.empty((B, 3, H, W), dtype=dt, pin_memory=True),
                    "count": torch.empty((B,), dtype=torch.int32, pin_memory=True),
                    "box": torch.empty(tuple(plan.out_box.shape), dtype=torch.float32, pin_memory=True),
                    "score": torch.empty(tuple(plan.out_score.shape), dtype=torch.float32, pin_memory=True),
                    "label": torch.empty(tuple(plan.out_label.shape), dtype=torch.int64, pin_memory=True),
                    "done": torch.cuda.Event()}

        def slot(key):
            if key not in slots:
                slots[key] = [new_slot(key, k == 0) for k in range(n)]
            turn[0] += 1
            return slots[key][turn[0] % n]

        def collect(tag, sl, B):
            lap("issue")
            sl["done"].synchronize()
            lap("results")
            sl["src"] = None
            if raw:
                return tag, sl["count"].numpy().copy(), sl["box"].numpy().copy(), sl["score"].numpy().copy(), \
                    sl["label"].numpy().copy()
            counts = sl["count"].tolist()
            box, score, label = sl["box"].numpy(), sl["score"].numpy(), sl["label"].numpy()
            return tag, [(box[j, :counts[j]].copy(), score[j, :counts[j]].copy(), label[j, :counts[j]].copy())
                         for j in range(B)]

        def emit(item):
            r = collect(*item)
            lap("results")
            yield r
            lap("caller")  # the caller's work on the rows (formatting, file writes)

        from .jpeg import BatchDecoder, PackedBatch, Packets
        for tag, imgs in batches:
            lap("input")
            whole = imgs if torch.is_tensor(imgs) and imgs.dim() == 4 else None
            if isinstance(imgs, (Packets, PackedBatch)):  # JPEG packets: decoded on the device into the plan's input
                shapes, dtypes, B = {imgs.hw}, {torch.uint8}, len(imgs)
            elif whole is not None:
                shapes, dtypes, B = {tuple(whole.shape[-2:])}, {whole.dtype}, whole.shape[0]
            else:
                imgs = list(imgs)
                shapes, dtypes, B = {tuple(im.shape[-2:]) for im in imgs}, {im.dtype for im in imgs}, len(imgs)
            if len(shapes) != 1 or len(dtypes) != 1 or B > self.max_batch or B == 0:
                raise ValueError("run_batches takes batches of 1..max_batch equal-size images of one dtype")
            H, W = shapes.pop()
            key = (B, H, W, dtypes.pop() == torch.uint8)
            if slots and key not in slots:
                # a new shape: finish the old shape's batches and free its plans (the CLI groups
                # images by size, so a real image set touches each shape in one run of batches)
                while pending:
                    yield from emit(pending.pop(0))
                for k in slots:
                    self.plans.pop(k, None)
                slots.clear()
            lap("issue")
            sl = slot(key)
            lap("plans")
            # the slot's previous batch (if any) must be on the host before its buffers are reused
            while any(p is sl for _, p, _ in pending):
                yield from emit(pending.pop(0))
            plan, stream = sl["plan"], sl["stream"]
            stage = sl["stage"]
            sl["done"].synchronize()  # a slot left in flight by an abandoned earlier call
            if isinstance(imgs, (Packets, PackedBatch)):
                src = None
            elif whole is not None and whole.dtype in (torch.uint8, torch.float32) and whole.is_contiguous() and \
                    (whole.is_pinned() or whole.device == self.device):
                # pinned host or already on the device: copied straight into the plan's input on the
                # slot stream (no staging); held until the slot is collected (the copy is asynchronous)
                if whole.is_cuda:
                    stream.wait_stream(torch.cuda.current_stream(self.device))
                src = sl["src"] = whole
            else:
                for j, im in enumerate(whole if whole is not None else imgs):
                    stage[j].copy_(im if key[3] else im.to(torch.float32))
                src = stage
            lap("issue")
            if plan.graph is None:
                # one hipGraph per slot plan (captured on first use): a batch is then one launch
                # instead of a host call per op, which kept the host, not the device, the bottleneck
                plan.capture(stream)
            lap("plans")
            with torch.cuda.stream(stream):
                if src is None:
                    if sl["jpeg"] is None:
                        sl["jpeg"] = BatchDecoder(self.device)
                    sl["jpeg"].decode(imgs, plan.input.tensor(), stream)
                else:
                    plan.input.tensor().copy_(src, non_blocking=True)
                plan.replay(stream)
                sl["count"].copy_(plan.out_count.tensor(), non_blocking=True)
                sl["box"].copy_(plan.out_box.tensor(), non_blocking=True)
                sl["score"].copy_(plan.out_score.tensor(), non_blocking=True)
                sl["label"].copy_(plan.out_label.tensor(), non_blocking=True)
                sl["done"].record(stream)
            pending.append((tag, sl, B))
            while len(pending) >= n:
                yield from emit(pending.pop(0))
        while pending:
            yield from emit(pending.pop(0))
        lap("issue")



# ====================================================================================== SSDLite
class SSDLite320(_Detector):
    """ssdlite320_mobilenet_v3_large."""

    kind = "ssd"
    # run_batches slots: four batches in flight hide the per-batch host work (upload issue, D2H wait,
    # row formatting) behind the device (end to end 18.3k -> 25.2k img/s, tools/e2e_sweep.py)
    INFLIGHT = 4
    SIZE = 320
    SCORE_THRESH, NMS_THRESH, DETS, TOPK = 0.001, 0.55, 300, 300
    max_batch = 64
    grids = [(20, 20), (10, 10), (5, 5), (3, 3), (2, 2), (1, 1)]  # head feature maps of the 320x320 input

    def __init__(self, state_dict, num_classes=91, reduced_tail=None, device=None):
        if reduced_tail is None:
            reduced_tail = tuple(state_dict["backbone.features.1.3.0.weight"].shape)[1] == 80
        self.reduced_tail = bool(reduced_tail)
        super().__init__(state_dict, num_classes, device)

    def table(self):
        return arch.ssdlite_table(self.num_classes, self.reduced_tail)

    def attach(self, P):
        """Named buffers of the SSDLite plan the parity tests read (csrc/lower.hip SSDLite)."""
        P.cls_logits, P.bbox_regression = P.buffer("cls_logits"), P.buffer("bbox_regression")
        P.scores_t, P.boxes = P.buffer("scores_t"), P.buffer("boxes")
        P.chains = 1 + next((int(r["i"][0]) for r in P.records if int(r["kind"]) == ops.FORK), 0)  # side lanes + 1


# ====================================================================================== FRCNN
class FasterRCNNFPNv2(_Detector):
    """fasterrcnn_resnet50_fpn_v2."""

    kind = "faster_rcnn"
    MEAN = (0.485, 0.456, 0.406)
    STD = (0.229, 0.224, 0.225)
    MIN_SIZE, MAX_SIZE, DIVISIBLE = 800, 1333, 32
    RPN_PRE, RPN_POST, RPN_NMS, RPN_MIN, RPN_SCORE = 1000, 1000, 0.7, 1e-3, 0.0
    BOX_SCORE, BOX_NMS, BOX_DETS, BOX_MIN = 0.05, 0.5, 100, 1e-2
    max_batch = 8
    # run_batches slots: a third batch fills the idle time around the small latency-bound launches
    # (RPN filtering, RoIAlign, merges): 347.7 -> 352.5 img/s at 3 against 2 (4: 347.8), alternated
    # runs on one box (tools/gpu_r3af.sh); 8.6 GB of workspace per slot
    INFLIGHT = 3

    def table(self):
        return arch.frcnn_table(self.num_classes)

    def resized_size(self, H, W):
        """[TV] GeneralizedRCNNTransform resize (detect.py:78): the scale is a float32
        tensor op, `min(800. / min_f32, 1333. / max_f32)` with `float / Tensor` = `reciprocal(t) * x`;
        the sizes are `floor(side * float(scale))` in double (`recompute_scale_factor=True`).  The
        library's lowering computes the same (csrc/lower.hip ResNetFPN::resized_size; the plan's
        PREPROCESS record carries it, tests/test_resize_rule.py)."""
        f32 = np.float32
        a = f32(f32(1.0) / f32(min(H, W))) * f32(self.MIN_SIZE)
        b = f32(f32(1.0) / f32(max(H, W))) * f32(self.MAX_SIZE)
        scale = float(min(a, b))
        return int(math.floor(H * scale)), int(math.floor(W * scale))

    def batch_work(self, B, H, W):
        """B x the resized image padded to /32 (GeneralizedRCNNTransform): FRCNN / RetinaNet cost
        scales with those pixels (799 x 1199 is 1.5x 800 x 800)."""
        h, w = self.resized_size(H, W)
        d = self.DIVISIBLE
        return float(B * (-(-h // d) * d) * (-(-w // d) * d))

    def attach(self, P):
        P.feats = [P.buffer(n) for n in ("backbone.fpn.layer_blocks.0.0.weight", "backbone.fpn.layer_blocks.1.0.weight",
                                         "backbone.fpn.layer_blocks.2.0.weight", "backbone.fpn.layer_blocks.3.0.weight",
                                         "backbone.fpn.extra_blocks.pool")]
        # per level (objectness [B,H,W,3], deltas [B,H,W,12]): the parity tests' RPN inputs
        P.rpn_heads = [(P.buffer(f"rpn.head.cls_logits@{l}"), P.buffer(f"rpn.head.bbox_pred@{l}")) for l in range(5)]
        P.proposals, P.proposal_count = P.buffer("proposals"), P.buffer("proposal_count")
        P.box_features = P.buffer("box_roi_pool")
        P.pred = P.buffer("box_predictor")
        P.box_scores, P.box_decoded = P.buffer("box_scores"), P.buffer("box_decoded")


class RetinaNetFPNv2(FasterRCNNFPNv2):
    """retinanet_resnet50_fpn_v2 (detect.py:34-38, the CLI's third model; oracle/retinanet.py).

    Shares the transform and the ResNet-50 body with Faster R-CNN.  FPN over C3..C5 with plain convs
    (bias, no norm) + LastLevelP6P7(2048, 256) (P6 on C5, P7 on relu(P6): the ReLU is applied as P7's
    conv loads its input).  The GroupNorm towers of the head never materialise a normalised tensor:
    GN_STATS turns each conv's output into per-(image, channel) scale / shift, which the next conv
    applies (with the ReLU) as it loads its A operand.  The cls / box convs of every level store
    straight into the concatenated [B, sum(HWA), K] / [B, sum(HWA), 4] tensors.
    """

    kind = "retinanet"
    SCORE, NMS, DETS, TOPK = 0.05, 0.5, 300, 1000
    A = arch.RETINA_ANCHORS

    def table(self):
        return arch.retinanet_table(self.num_classes)

    def attach(self, P):
        from . import ops
        P.cls_logits, P.bbox_regression = P.buffer("head.cls_logits"), P.buffer("head.bbox_regression")
        P.cand_count = P.buffer("retina.cand.count")
        sel = next(op for op in P.ops if op.kind == ops.RETINA_SELECT)
        P.level_anchors = [int(sel.i[11 + l]) for l in range(int(sel.i[1]))]  # anchors per level (parity tests)


# ====================================================================================== factories
def ssdlite320_mobilenet_v3_large(weights=None, num_classes=91, reduced_tail=True, state_dict=None, seed=0):
    """Builder mirroring torchvision's (detect.py:24,26).  ``weights="DEFAULT"`` would download COCO
    weights, impossible offline: pass ``state_dict=`` (e.g. torch.load(--model-path)) or get seeded
    synthetic weights (edgeml_amd.synthetic) in their place: seed 0 is the calibrated set (realistic
    detection counts), any other seed an uncalibrated draw."""
    from . import synthetic
    if state_dict is None:
        state_dict = synthetic.synthetic_state_dict("ssd", num_classes, reduced_tail, seed=seed, calibrated=seed == 0)
    return SSDLite320(state_dict, num_classes, reduced_tail)


def fasterrcnn_resnet50_fpn_v2(weights=None, num_classes=91, state_dict=None, seed=0):
    """Builder mirroring torchvision's (detect.py:30,32); see ssdlite320_mobilenet_v3_large."""
    from . import synthetic
    if state_dict is None:
        state_dict = synthetic.synthetic_state_dict("faster_rcnn", num_classes, seed=seed, calibrated=seed == 0)
    return FasterRCNNFPNv2(state_dict, num_classes)


def retinanet_resnet50_fpn_v2(weights=None, num_classes=91, state_dict=None, seed=0):
    """Builder mirroring torchvision's (detect.py:36,38); see ssdlite320_mobilenet_v3_large."""
    from . import synthetic
    if state_dict is None:
        state_dict = synthetic.synthetic_state_dict("retinanet", num_classes, seed=seed, calibrated=seed == 0)
    return RetinaNetFPNv2(state_dict, num_classes)
