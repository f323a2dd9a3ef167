"""The two detectors of torch_models/detect.py, lowered onto libedgedet.so.

``SSDLite320`` restates torchvision's ``ssdlite320_mobilenet_v3_large`` (detect.py:24/26) and
``FasterRCNNFPNv2`` restates ``fasterrcnn_resnet50_fpn_v2`` (detect.py:30/32).  Both keep
torchvision's detection-model contract (detect.py:72-81): ``.to(device)``, ``.eval()``,
``.load_state_dict(sd)`` with torchvision's state_dict keys, and
``model(Tensor[N,3,H,W] float32 in [0,1]) -> [{"boxes", "scores", "labels"}]`` with boxes in original
pixels, scores descending, labels int64.  Every arithmetic step runs in HIP kernels (plan.py lowers
the forward into one op list per input shape; ops.py loads the library and fails loudly if it is
missing).  Architecture and post-processing constants: SURVEY.md Appendix A.
"""
import math
import os

import numpy as np
import torch

from . import anchors as anc
from . import arch
from . import ops
from .plan import BufView, Op, Plan, WeightPack, conv_op, fold_bn, pack_conv_weight, pack_dw_weight, split_bf16x3

# InvertedResidual expand + depthwise as one fused kernel (no SE in between), with the expanded
# tensor kept in LDS.  Off by default: measured slower than the two ops (csrc/layers.hip
# mbconv_front_kernel header); EDGEDET_MBCONV_FUSE=1 selects it.
MBCONV_FUSE = os.environ.get("EDGEDET_MBCONV_FUSE", "0") == "1"
# A whole InvertedResidual without SE (expand, depthwise, project, residual) as one kernel where its
# input and output are at most 32 channels wide (SSDLite blocks 0.2 and 0.3, csrc/layers.hip
# mbconv_kernel).  Opt-in (EDGEDET_MB_BLOCK=1): correct, but measured 3.5-4.5x slower than the three
# separate ops (0.2: 255 vs 74 us per 16-image chain, 0.3: 260 vs 58 us; SSD 17.0k vs 25.2k img/s).
MB_BLOCK_FUSE = os.environ.get("EDGEDET_MB_BLOCK", "0") == "1"
# SSDLite features.0.0 + features.0.1 as one kernel (csrc/layers.hip ssd_stem_kernel); =0 lowers the
# three separate ops.
SSD_STEM_FUSE = os.environ.get("EDGEDET_SSD_STEM_FUSE", "1") == "1"
# ResNet bottleneck conv2 without its ReLU (applied by conv3's input load) where split-K pays;
# EDGEDET_SPLITK_DEFER=0 keeps the ReLU in conv2.
SPLITK_DEFER = os.environ.get("EDGEDET_SPLITK_DEFER", "1") == "1"


def _np(t):
    return t.detach().cpu().to(torch.float64).numpy()


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
        self.pack = WeightPack()
        self._w = {}
        self._pack_all()
        self.plans = {}
        return self

    def state_dict(self):
        return dict(self.sd)

    # weights ----------------------------------------------------------------------------------
    def _conv_bn(self, wkey, bnp, eps, cin_pad=None):
        """(w, b, K, Kpad, Cin) of a bias-free conv followed by BatchNorm prefix `bnp`."""
        key = ("cbn", wkey)
        if key not in self._w:
            s = self.sd
            wf, bf = fold_bn(_np(s[wkey]), _np(s[bnp + ".weight"]), _np(s[bnp + ".bias"]),
                             _np(s[bnp + ".running_mean"]), _np(s[bnp + ".running_var"]), eps)
            if wf.shape[1] == 1 and wf.shape[0] > 1 and cin_pad is None and self._is_dw(wkey):
                self._w[key] = (self.pack.add(pack_dw_weight(wf)), self.pack.add(bf), wf.shape[-1], None, wf.shape[0])
            else:
                wp, K, Kpad, cin = pack_conv_weight(wf, cin_pad)
                self._w[key] = (self._conv_w(wp), self.pack.add(bf), K, Kpad, cin)
        return self._w[key]

    def _conv_bias(self, wkey, bkey, perm=None):
        key = ("cb", wkey)
        if key not in self._w:
            w = _np(self.sd[wkey]).astype(np.float32)
            b = _np(self.sd[bkey]).astype(np.float32)
            if w.ndim == 2:
                w = w[:, :, None, None]
            wp, K, Kpad, cin = pack_conv_weight(w)
            self._w[key] = (self._conv_w(wp), self.pack.add(b), K, Kpad, cin)
        return self._w[key]

    def _is_dw(self, wkey):
        return False

    def _conv_nobias(self, wkey):
        """A conv without bias and without BatchNorm (RetinaNet GroupNorm towers): zero bias."""
        key = ("cn", wkey)
        if key not in self._w:
            w = _np(self.sd[wkey]).astype(np.float32)
            wp, K, Kpad, cin = pack_conv_weight(w)
            self._w[key] = (self._conv_w(wp), self.pack.add(np.zeros(w.shape[0], np.float32)), K, Kpad, cin)
        return self._w[key]

    def _conv_w(self, wp):
        """Pack a [Cout][Kpad] conv weight plus its three bf16 planes (the bf16x6 tiles' operand)."""
        ref = self.pack.add(wp)
        ref.split = self.pack.add_u16(split_bf16x3(wp))
        return ref

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

        def new_slot(key, first):
            B, H, W, u8 = key
            plan = self.plan(*key) if first else self.build_plan(*key).finalize()
            dt = torch.uint8 if u8 else torch.float32
            return {"plan": plan, "stream": torch.cuda.Stream(self.device),
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
            sl["done"].synchronize()
            sl["src"] = None
            if raw:
                return tag, sl["count"].numpy().copy(), sl["box"].numpy().copy(), sl["score"].numpy().copy(), \
                    sl["label"].numpy().copy()
            counts = sl["count"].tolist()
            box, score, label = sl["box"].numpy(), sl["score"].numpy(), sl["label"].numpy()
            return tag, [(box[j, :counts[j]].copy(), score[j, :counts[j]].copy(), label[j, :counts[j]].copy())
                         for j in range(B)]

        for tag, imgs in batches:
            whole = imgs if torch.is_tensor(imgs) and imgs.dim() == 4 else None
            if whole is not None:
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
                    yield collect(*pending.pop(0))
                for k in slots:
                    self.plans.pop(k, None)
                slots.clear()
            sl = slot(key)
            # the slot's previous batch (if any) must be on the host before its buffers are reused
            while any(p is sl for _, p, _ in pending):
                yield collect(*pending.pop(0))
            plan, stream = sl["plan"], sl["stream"]
            stage = sl["stage"]
            sl["done"].synchronize()  # a slot left in flight by an abandoned earlier call
            if whole is not None and whole.is_pinned() and whole.dtype in (torch.uint8, torch.float32) \
                    and whole.is_contiguous():
                src = sl["src"] = whole  # held until the slot is collected (the copy is asynchronous)
            else:
                for j, im in enumerate(whole if whole is not None else imgs):
                    stage[j].copy_(im if key[3] else im.to(torch.float32))
                src = stage
            if plan.graph is None:
                # one hipGraph per slot plan (captured on first use): a batch is then one launch
                # instead of a host call per op, which kept the host, not the device, the bottleneck
                plan.capture(stream)
            with torch.cuda.stream(stream):
                plan.input.tensor().copy_(src, non_blocking=True)
                plan.replay(stream)
                sl["count"].copy_(plan.out_count.tensor(), non_blocking=True)
                sl["box"].copy_(plan.out_box.tensor(), non_blocking=True)
                sl["score"].copy_(plan.out_score.tensor(), non_blocking=True)
                sl["label"].copy_(plan.out_label.tensor(), non_blocking=True)
                sl["done"].record(stream)
            pending.append((tag, sl, B))
            while len(pending) >= n:
                yield collect(*pending.pop(0))
        while pending:
            yield collect(*pending.pop(0))


# ====================================================================================== SSDLite
class SSDLite320(_Detector):
    """ssdlite320_mobilenet_v3_large."""

    kind = "ssd"
    BN_EPS = 1e-3
    # run_batches slots: four batches in flight hide the per-batch host work (upload issue, D2H wait,
    # row formatting) behind the device (end to end 18.3k -> 25.2k img/s, tools/e2e_sweep.py)
    INFLIGHT = 4
    SIZE = 320
    SCORE_THRESH, NMS_THRESH, DETS, TOPK = 0.001, 0.55, 300, 300
    max_batch = 64
    # "image": SSD_POSTPROCESS (class top-k pool + one global-order greedy pass per image);
    # "class": SSD_CLASS_NMS + MERGE_TOPK (every class's top-k fully NMS'd, then merged).
    postprocess = "image"
    CHAINS = 2
    IMAGE_POOL_MAX = 512 * 54  # (classes - 1) * TOPK that fits the image kernel's registers

    def __init__(self, state_dict, num_classes=91, reduced_tail=None, device=None):
        if reduced_tail is None:
            reduced_tail = tuple(state_dict["backbone.features.1.3.0.weight"].shape)[1] == 80
        self.reduced_tail = reduced_tail
        super().__init__(state_dict, num_classes, device)

    def table(self):
        return arch.ssdlite_table(self.num_classes, self.reduced_tail)

    def _is_dw(self, wkey):
        return tuple(self.sd[wkey].shape)[1] == 1 and tuple(self.sd[wkey].shape)[0] > 1

    def _pack_all(self):
        # pack eagerly in network order so the blob is laid out like the forward walks it
        self.build_plan(1, self.SIZE, self.SIZE, pack_only=True)

    def _se(self, p):
        key = ("se", p)
        if key not in self._w:
            w1 = _np(self.sd[p + ".fc1.weight"])[:, :, 0, 0]  # [S, C]
            w2 = _np(self.sd[p + ".fc2.weight"])[:, :, 0, 0]  # [C, S]
            self._w[key] = (self.pack.add(w1), self.pack.add(_np(self.sd[p + ".fc1.bias"])),
                            self.pack.add(w2.T), self.pack.add(_np(self.sd[p + ".fc2.bias"])), w1.shape[0])
        return self._w[key]

    def n_chains(self, B):
        """Independent sub-batches lowered as concurrent chains (stream lanes): SSDLite's layers are
        small, so two chains overlap one chain's latency-bound tail (NMS) and small kernels with the
        other's work.  EDGEDET_SSD_CHAINS overrides (1 = one chain)."""
        n = int(os.environ.get("EDGEDET_SSD_CHAINS", "0")) or self.CHAINS
        return max(1, min(n, ops.MAX_LANES, B // 8 if B >= 16 else 1))

    @staticmethod
    def chain_split(B, n):
        """(first image, images) of each chain: B split as evenly as possible (earlier chains +1)."""
        q, r = divmod(B, n)
        starts = [c * q + min(c, r) for c in range(n)]
        return [(b0, q + (1 if c < r else 0)) for c, b0 in enumerate(starts)]

    def build_plan(self, B, H, W, u8=False, pack_only=False):
        P = Plan(self.pack, self.device or "cpu")
        nch = 1 if pack_only else self.n_chains(B)
        inp = P.buf((B, 3, H, W), torch.uint8 if u8 else torch.float32, name="images")
        shared = {}
        if nch > 1:
            P.fork(nch - 1)
        for c, (b0, bc) in enumerate(self.chain_split(B, nch)):
            if nch > 1:
                P.lane(c)
            self._lower_chain(P, c, b0, bc, B, H, W, inp, shared, nch, pack_only)
            if pack_only:
                return P
        if nch > 1:
            P.join()
        P.input = inp
        P.cls_logits, P.bbox_regression = shared["cls"], shared["reg"]
        P.scores_t, P.boxes = shared["scores_t"], shared["boxes"]
        P.out_box, P.out_score, P.out_label, P.out_count = (shared[k] for k in ("ob", "os", "ol", "oc"))
        P.feats = shared["feats"]
        P.chains = nch
        return P

    def _lower_chain(self, P, c, img0, B, Btot, H, W, inp, shared, nch, pack_only):
        """Lower the forward of images [img0, img0 + B) (B in this chain, Btot in the plan)."""
        NC = self.num_classes
        S = self.SIZE
        sfx = f"#{c}" if nch > 1 else ""
        view = (lambda buf: BufView(buf, img0, B)) if nch > 1 else (lambda buf: buf)
        x = P.buf((B, S, S, 4), name="pre" + sfx)
        src = {2: view(inp)} if inp.dtype == torch.uint8 else {0: view(inp)}
        P.add(Op(ops.PREPROCESS, {0: B, 1: H, 2: W, 3: S, 4: S, 5: S, 6: S}, {**src, 1: x},
                 {0: 0.5, 1: 0.5, 2: 0.5, 3: 0.5, 4: 0.5, 5: 0.5}, name="transform"))
        cur = (x, (B, S, S, 4))

        def conv(cur, prefix, k, stride, act, res=None, in_scale=None, cin_pad=None):
            xb, xs = cur
            w, b, K, Kpad, cin = self._conv_bn(prefix + ".0.weight", prefix + ".1", self.BN_EPS, cin_pad)
            cout = int(self.sd[prefix + ".0.weight"].shape[0])
            Ho = (xs[1] + 2 * ((k - 1) // 2) - k) // stride + 1
            Wo = (xs[2] + 2 * ((k - 1) // 2) - k) // stride + 1
            ys = (B, Ho, Wo, cout)
            y = P.buf(ys, name=prefix + sfx)
            conv_op(P, xb, xs, w, b, cout, k, stride, (k - 1) // 2, act, y, ys, K, Kpad, res=res,
                    in_scale=in_scale, name=prefix)
            return (y, ys)

        def dw(cur, prefix, k, stride, act, se_part=False):
            """Depthwise conv; with se_part it also emits the SE squeeze partial sums (fused)."""
            xb, xs = cur
            w, b, _, _, c = self._conv_bn(prefix + ".0.weight", prefix + ".1", self.BN_EPS)
            pad = (k - 1) // 2
            Ho = (xs[1] + 2 * pad - k) // stride + 1
            Wo = (xs[2] + 2 * pad - k) // stride + 1
            ys = (B, Ho, Wo, xs[3])
            y = P.buf(ys, name=prefix + sfx)
            parts = ops.se_parts(Ho, Wo)
            part = P.buf((B, parts, xs[3]), name=prefix + ".se_partial_sums" + sfx) if se_part else None
            P.add(Op(ops.DWCONV, {0: B, 1: xs[1], 2: xs[2], 3: xs[3], 4: Ho, 5: Wo, 6: k, 7: stride, 8: pad,
                                  9: ops.ACT[act], 10: parts}, {0: xb, 1: w, 2: b, 3: y, 4: part}, name=prefix))
            return (y, ys, (part, parts)) if se_part else (y, ys)

        def se(cur, p):
            """SqueezeExcitation excitation from the partial sums the depthwise conv emitted."""
            xb, xs, (part, parts) = cur
            w1, b1, w2t, b2, sq = self._se(p)
            C = xs[3]
            scale = P.buf((B, C), name=p + ".scale" + sfx)
            hidden = P.buf((B, sq), name=p + ".hidden" + sfx)
            P.add(Op(ops.SE_FC, {0: B, 1: C, 2: sq, 3: xs[1] * xs[2], 4: parts},
                     {0: part, 1: w1, 2: b1, 3: w2t, 4: b2, 5: scale, 6: hidden}, name=p))
            return scale

        def mbfront(cur, pe, pd, k, stride, act):
            """Expand 1x1 + depthwise as one fused op (csrc/layers.hip mbconv_front_kernel), or None
            when the shapes do not fit it."""
            xb, xs = cur
            w1, b1, _, kpad1, cin = self._conv_bn(pe + ".0.weight", pe + ".1", self.BN_EPS)
            w, b, _, _, c = self._conv_bn(pd + ".0.weight", pd + ".1", self.BN_EPS)
            ipp = ((7 * stride + k) ** 2 + 31) // 32 * 32  # LDS of the kernel (csrc/layers.hip MbGeom)
            lds = 4 * (ipp * (cin + 4) + 32 * (cin + 4) + ipp * 36)
            if not (MBCONV_FUSE and xs[3] == cin and cin % 8 == 0 and c % 8 == 0 and lds <= 160 * 1024):
                return None
            pad = (k - 1) // 2
            Ho = (xs[1] + 2 * pad - k) // stride + 1
            Wo = (xs[2] + 2 * pad - k) // stride + 1
            ys = (B, Ho, Wo, c)
            y = P.buf(ys, name=pd + sfx)
            P.add(Op(ops.DWCONV, {0: B, 1: xs[1], 2: xs[2], 3: c, 4: Ho, 5: Wo, 6: k, 7: stride, 8: pad,
                                  9: ops.ACT[act], 10: 0, 11: cin, 12: kpad1, 13: ops.ACT[act]},
                     {0: xb, 1: w, 2: b, 3: y, 4: None, 5: w1, 6: b1}, name=pe + "+" + pd.rsplit(".", 1)[-1]))
            return (y, ys)

        def mb_block(cur, cnf, pe, pd, pp):
            """The whole block as one MBCONV op (csrc/layers.hip mbconv_kernel)."""
            xb, xs = cur
            cin, k, exp, cout, use_se, act, stride = cnf
            w1, b1, _, kpad1, _ = self._conv_bn(pe + ".0.weight", pe + ".1", self.BN_EPS)
            wd, bd, _, _, _ = self._conv_bn(pd + ".0.weight", pd + ".1", self.BN_EPS)
            w2, b2, _, kpad2, _ = self._conv_bn(pp + ".0.weight", pp + ".1", self.BN_EPS)
            pad = (k - 1) // 2
            Ho = (xs[1] + 2 * pad - k) // stride + 1
            Wo = (xs[2] + 2 * pad - k) // stride + 1
            ys = (B, Ho, Wo, cout)
            y = P.buf(ys, name=pp + sfx)
            P.add(Op(ops.MBCONV, {0: B, 1: xs[1], 2: xs[2], 3: cin, 4: exp, 5: cout, 6: Ho, 7: Wo, 8: k, 9: stride,
                                  10: pad, 11: ops.ACT[act], 12: kpad1, 13: kpad2,
                                  14: int(stride == 1 and cin == cout)},
                     {0: xb, 1: w1, 2: b1, 3: wd, 4: bd, 5: w2, 6: b2, 7: y}, name=base_name(pe)))
            return (y, ys)

        def base_name(pe):
            return pe.rsplit(".", 1)[0]

        def inverted_residual(cur, cnf, base):
            cin, k, exp, cout, use_se, act, stride = cnf
            pe, pd, ps, pp = arch.block_prefixes(cnf, base)
            if MB_BLOCK_FUSE and not pack_only and pe and not use_se and cin <= 32 and cout <= 32:
                return mb_block(cur, cnf, pe, pd, pp)
            y = cur
            fused = mbfront(y, pe, pd, k, stride, act) if pe and not use_se and not pack_only else None
            if fused is not None:
                res = cur[0] if (stride == 1 and cin == cout) else None
                return conv(fused, pp, 1, 1, None, res=res)
            if pe:
                y = conv(y, pe, 1, 1, act)
            y = dw(y, pd, k, stride, act, se_part=use_se)
            scale = se(y, ps) if use_se else None
            res = cur[0] if (stride == 1 and cin == cout) else None
            return conv(y[:2], pp, 1, 1, None, res=res, in_scale=scale)

        cfg = arch.mnv3_blocks(self.reduced_tail)
        first = 0
        if SSD_STEM_FUSE and not pack_only and cfg[0] == (16, 3, 16, 16, False, "RE", 1):
            # features.0.0 + features.0.1 as one op (csrc/layers.hip ssd_stem_kernel)
            w0, b0, _, kpad0, _ = self._conv_bn("backbone.features.0.0.0.weight", "backbone.features.0.0.1",
                                                self.BN_EPS, 4)
            _, pd, _, pp = arch.block_prefixes(cfg[0], "backbone.features.0.1.block")
            wd, bd, _, _, _ = self._conv_bn(pd + ".0.weight", pd + ".1", self.BN_EPS)
            w1, b1, _, kpad1, _ = self._conv_bn(pp + ".0.weight", pp + ".1", self.BN_EPS)
            Ho, Wo = (S - 1) // 2 + 1, (S - 1) // 2 + 1
            ys = (B, Ho, Wo, 16)
            y = P.buf(ys, name="backbone.features.0.1" + sfx)
            P.add(Op(ops.SSD_STEM, {0: B, 1: S, 2: S, 3: Ho, 4: Wo, 5: kpad0, 6: kpad1},
                     {0: x, 1: w0, 2: b0, 3: wd, 4: bd, 5: w1, 6: b1, 7: y}, name="backbone.features.0.0+0.1"))
            cur, first = (y, ys), 1
        else:
            cur = conv(cur, "backbone.features.0.0", 3, 2, "HS", cin_pad=4)
        for i in range(first, 12):
            cur = inverted_residual(cur, cfg[i], f"backbone.features.0.{i + 1}.block")
        _, k, exp, cout, _, act, stride = cfg[12]
        cur = conv(cur, "backbone.features.0.13", 1, 1, act)
        feats = [cur]
        y = dw(cur, "backbone.features.1.0.1", k, stride, act, se_part=True)
        scale = se(y, "backbone.features.1.0.2")
        cur = conv(y[:2], "backbone.features.1.0.3", 1, 1, None, in_scale=scale)
        for i in (13, 14):
            cur = inverted_residual(cur, cfg[i], f"backbone.features.1.{i - 12}.block")
        cur = conv(cur, "backbone.features.1.3", 1, 1, "HS")
        feats.append(cur)
        for e in range(4):
            p = f"backbone.extra.{e}"
            cur = conv(cur, p + ".0", 1, 1, "R6")
            cur = dw(cur, p + ".1", 3, 2, "R6")
            cur = conv(cur, p + ".2", 1, 1, "R6")
            feats.append(cur)

        grids = [(f[1][1], f[1][2]) for f in feats]
        A = sum(h * w * 6 for h, w in grids)
        if "cls" not in shared:
            shared["cls"] = P.buf((Btot, A, NC), name="cls_logits")
            shared["reg"] = P.buf((Btot, A, 4), name="bbox_regression")
            shared["feats"] = [f[0] for f in feats]
        cls, reg = shared["cls"], shared["reg"]
        off = 0
        # the 12 head branches are independent: spread them over 4 stream lanes (one chain only)
        if nch == 1:
            P.fork(3)
        chain = 0
        for i, f in enumerate(feats):
            fb, fs = f
            for name, cols, out in (("classification_head", NC, cls), ("regression_head", 4, reg)):
                p = f"head.{name}.module_list.{i}"
                if nch == 1:
                    P.lane(chain % 4)
                chain += 1
                t = dw(f, p + ".0", 3, 1, "R6")
                w, b, K, Kpad, cin = self._conv_bias(p + ".1.weight", p + ".1.bias")
                cout = 6 * cols
                conv_op(P, t[0], t[1], w, b, cout, 1, 1, 0, None, out, (B, fs[1], fs[2], cout), K, Kpad,
                        y_pstride=cout, y_bstride=A * cols, y_off=img0 * A * cols + off * cols, name=p + ".1" + sfx)
            off += fs[1] * fs[2] * 6
        if nch == 1:
            P.join()
        self.grids = grids
        if pack_only:
            return

        if "anchors" not in shared:
            shared["anchors"] = P.const(anc.ssd_default_boxes(grids, (S, S)), name="anchors")
            shared["scores_t"] = P.buf((Btot, NC, A), name="scores_t")
            shared["boxes"] = P.buf((Btot, A, 4), name="boxes")
            ratio = np.tile(np.asarray([np.float32(W) / np.float32(S), np.float32(H) / np.float32(S)], np.float32),
                            (Btot, 1))
            shared["ratio"] = P.const(ratio, name="ratio")
            shared["ob"] = P.buf((Btot, self.DETS, 4), name="out.boxes")
            shared["os"] = P.buf((Btot, self.DETS), name="out.scores")
            shared["ol"] = P.buf((Btot, self.DETS), torch.int64, name="out.labels")
            shared["oc"] = P.buf((Btot,), torch.int32, name="out.count")
        anchors = shared["anchors"]
        scores_t, boxes = view(shared["scores_t"]), view(shared["boxes"])
        P.add(Op(ops.SSD_SCORES, {0: B, 1: A, 2: NC}, {0: view(cls), 1: view(reg), 2: anchors, 3: scores_t, 4: boxes},
                 {0: S, 1: S}, name="postprocess.scores" + sfx))
        NS, KM = NC - 1, self.TOPK
        ratio_b = view(shared["ratio"])
        out_box, out_score, out_label, out_count = (view(shared[k]) for k in ("ob", "os", "ol", "oc"))
        if self.postprocess == "image" and NS * KM <= self.IMAGE_POOL_MAX and self.DETS <= 1024:
            # class top-k pool + global-order greedy NMS, stopping at DETS kept (csrc/detect.hip)
            pool_key = P.buf((B, NS, KM), torch.int32, name="pool.key" + sfx)
            pool_ref = P.buf((B, NS, KM), torch.int32, name="pool.ref" + sfx)
            P.add(Op(ops.SSD_POSTPROCESS, {0: B, 1: A, 2: NC, 3: KM, 4: self.DETS},
                     {0: scores_t, 1: boxes, 2: pool_key, 3: pool_ref, 4: ratio_b, 5: out_box, 6: out_score,
                      7: out_label, 8: out_count}, {0: self.SCORE_THRESH}, {0: self.NMS_THRESH},
                     name="postprocess.nms" + sfx))
        else:
            rec = [P.buf((B, NS, KM, 4), name="rec.box" + sfx), P.buf((B, NS, KM), name="rec.score" + sfx),
                   P.buf((B, NS, KM), torch.int32, name="rec.tb" + sfx),
                   P.buf((B, NS, KM), torch.int32, name="rec.label" + sfx),
                   P.buf((B, NS), torch.int32, name="rec.count" + sfx)]
            P.add(Op(ops.SSD_CLASS_NMS, {0: B, 1: A, 2: NC, 3: self.TOPK, 4: KM},
                     {0: scores_t, 1: boxes, 2: rec[0], 3: rec[1], 4: rec[2], 5: rec[3], 6: rec[4]},
                     {0: self.SCORE_THRESH}, {0: self.NMS_THRESH}, name="postprocess.class_nms" + sfx))
            P.add(Op(ops.MERGE_TOPK, {0: B, 1: NS, 2: KM, 3: self.DETS},
                     {0: rec[0], 1: rec[1], 2: rec[2], 3: rec[3], 4: rec[4], 5: ratio_b, 6: out_box,
                      7: out_score, 8: out_label, 9: out_count}, name="postprocess.merge" + sfx))


# ====================================================================================== FRCNN
class FasterRCNNFPNv2(_Detector):
    """fasterrcnn_resnet50_fpn_v2."""

    kind = "faster_rcnn"
    BN_EPS = 1e-5
    MEAN = (0.485, 0.456, 0.406)
    STD = (0.229, 0.224, 0.225)
    MIN_SIZE, MAX_SIZE, DIVISIBLE = 800, 1333, 32
    RPN_PRE, RPN_POST, RPN_NMS, RPN_MIN, RPN_SCORE = 1000, 1000, 0.7, 1e-3, 0.0
    BOX_SCORE, BOX_NMS, BOX_DETS, BOX_MIN = 0.05, 0.5, 100, 1e-2
    max_batch = 8

    def table(self):
        return arch.frcnn_table(self.num_classes)

    def _pack_all(self):
        self.build_plan(1, self.MIN_SIZE, self.MIN_SIZE, pack_only=True)

    def _fc6(self):
        key = ("fc6",)
        if key not in self._w:
            w = _np(self.sd["roi_heads.box_head.5.weight"]).astype(np.float32)  # [1024, 256*7*7] (c, h, w)
            w = w.reshape(-1, 256, 7, 7).transpose(0, 2, 3, 1).reshape(w.shape[0], -1)  # -> (h, w, c)
            b = _np(self.sd["roi_heads.box_head.5.bias"]).astype(np.float32)
            wp, K, Kpad, cin = pack_conv_weight(w[:, :, None, None])
            self._w[key] = (self._conv_w(wp), self.pack.add(b), K, Kpad, cin)
        return self._w[key]

    def _predictor(self):
        key = ("pred",)
        if key not in self._w:
            q = "roi_heads.box_predictor."
            w = np.concatenate([_np(self.sd[q + "bbox_pred.weight"]), _np(self.sd[q + "cls_score.weight"])], 0)
            b = np.concatenate([_np(self.sd[q + "bbox_pred.bias"]), _np(self.sd[q + "cls_score.bias"])], 0)
            wp, K, Kpad, cin = pack_conv_weight(w.astype(np.float32)[:, :, None, None])
            self._w[key] = (self._conv_w(wp), self.pack.add(b.astype(np.float32)), K, Kpad, cin)
        return self._w[key]


    def resized_size(self, H, W):
        """[TV] GeneralizedRCNNTransform resize (detect.py:78): the scale is a float32
        tensor op, `min(800. / min_f32, 1333. / max_f32)` with `float / Tensor` = `reciprocal(t) * x`;
        the sizes are `floor(side * float(scale))` in double (`recompute_scale_factor=True`)."""
        f32 = np.float32
        a = f32(f32(1.0) / f32(min(H, W))) * f32(self.MIN_SIZE)
        b = f32(f32(1.0) / f32(max(H, W))) * f32(self.MAX_SIZE)
        scale = float(min(a, b))
        return int(math.floor(H * scale)), int(math.floor(W * scale))

    def _lower_body(self, P, B, H, W, u8=False):
        """GeneralizedRCNNTransform + ResNet-50 body (shared with RetinaNet): returns the input buffer,
        the sizes, the conv / maxpool emitters and C2..C5."""
        Ho, Wo = self.resized_size(H, W)
        Hp = (Ho + self.DIVISIBLE - 1) // self.DIVISIBLE * self.DIVISIBLE
        Wp = (Wo + self.DIVISIBLE - 1) // self.DIVISIBLE * self.DIVISIBLE
        inp = P.buf((B, 3, H, W), torch.uint8 if u8 else torch.float32, name="images")
        x = P.buf((B, Hp, Wp, 4), name="pre")
        P.add(Op(ops.PREPROCESS, {0: B, 1: H, 2: W, 3: Ho, 4: Wo, 5: Hp, 6: Wp}, {(2 if u8 else 0): inp, 1: x},
                 {0: self.MEAN[0], 1: self.MEAN[1], 2: self.MEAN[2], 3: self.STD[0], 4: self.STD[1],
                  5: self.STD[2]}, name="transform"))
        cur = (x, (B, Hp, Wp, 4))

        def conv(cur, wkey, bnp, k, stride, act, res=None, res_hw=None, cin_pad=None, bias_key=None, name=None,
                 tile=0, in_scale=None, in_shift=None, in_relu=False, out=None):
            xb, xs = cur
            if bias_key is not None:
                w, b, K, Kpad, cin = self._conv_bias(wkey, bias_key)
            elif bnp is None:
                w, b, K, Kpad, cin = self._conv_nobias(wkey)
            else:
                w, b, K, Kpad, cin = self._conv_bn(wkey, bnp, self.BN_EPS, cin_pad)
            cout = int(self.sd[wkey].shape[0])
            pad = (k - 1) // 2
            Ho_ = (xs[1] + 2 * pad - k) // stride + 1
            Wo_ = (xs[2] + 2 * pad - k) // stride + 1
            ys = (xs[0], Ho_, Wo_, cout)
            if out is not None:  # strided store into a concatenated buffer: (buf, pixel stride, batch stride, off)
                y, yp, yb, yo = out
                conv_op(P, xb, xs, w, b, cout, k, stride, pad, act, y, ys, K, Kpad, res=res, res_hw=res_hw,
                        name=name or wkey, tile=tile, in_scale=in_scale, in_shift=in_shift, in_relu=in_relu,
                        y_pstride=yp, y_bstride=yb, y_off=yo)
                return (y, ys)
            y = P.buf(ys, name=name or wkey)
            conv_op(P, xb, xs, w, b, cout, k, stride, pad, act, y, ys, K, Kpad, res=res, res_hw=res_hw,
                    name=name or wkey, tile=tile, in_scale=in_scale, in_shift=in_shift, in_relu=in_relu)
            return (y, ys)

        def maxpool(cur, k, stride, pad, name):
            xb, xs = cur
            Ho_ = (xs[1] + 2 * pad - k) // stride + 1
            Wo_ = (xs[2] + 2 * pad - k) // stride + 1
            ys = (xs[0], Ho_, Wo_, xs[3])
            y = P.buf(ys, name=name)
            P.add(Op(ops.MAXPOOL, {0: xs[0], 1: xs[1], 2: xs[2], 3: xs[3], 4: Ho_, 5: Wo_, 6: k, 7: stride, 8: pad},
                     {0: xb, 1: y}, name=name))
            return (y, ys)

        # ---- ResNet-50 body
        p = "backbone.body."
        cur = conv(cur, p + "conv1.weight", p + "bn1", 7, 2, "RE", cin_pad=4)
        cur = maxpool(cur, 3, 2, 1, "backbone.body.maxpool")
        cs = []
        for lname, nblk, width, stride in arch.RESNET_LAYERS:
            for bi in range(nblk):
                q = f"{p}{lname}.{bi}."
                s = stride if bi == 0 else 1
                y = conv(cur, q + "conv1.weight", q + "bn1", 1, 1, "RE")
                # deep-K 3x3 convs on small maps (layer3/4 at detection batch sizes) fill the GPU only
                # with split-K (tile 26), which cannot apply the ReLU: conv3 applies it to its input
                m = y[1][0] * ((y[1][1] - 1) // s + 1) * ((y[1][2] - 1) // s + 1)  # output pixels
                defer = SPLITK_DEFER and 9 * width >= 2048 and -(-m // 256) * -(-width // 128) < 200
                y = conv(y, q + "conv2.weight", q + "bn2", 3, s, None if defer else "RE")
                if bi == 0:
                    idn = conv(cur, q + "downsample.0.weight", q + "downsample.1", 1, s, None)
                else:
                    idn = cur
                cur = conv(y, q + "conv3.weight", q + "bn3", 1, 1, "RE", res=idn[0], in_relu=defer)
            cs.append(cur)

        return inp, (Ho, Wo, Hp, Wp), conv, maxpool, cs

    def build_plan(self, B, H, W, u8=False, pack_only=False):
        P = Plan(self.pack, self.device or "cpu")
        NC = self.num_classes
        inp, (Ho, Wo, Hp, Wp), conv, maxpool, cs = self._lower_body(P, B, H, W, u8)

        # ---- FPN (BN, no activations) + LastLevelMaxPool
        f = "backbone.fpn."
        last = conv(cs[3], f + "inner_blocks.3.0.weight", f + "inner_blocks.3.1", 1, 1, None)
        outs = [conv(last, f + "layer_blocks.3.0.weight", f + "layer_blocks.3.1", 3, 1, None)]
        for i in (2, 1, 0):
            last = conv(cs[i], f"{f}inner_blocks.{i}.0.weight", f"{f}inner_blocks.{i}.1", 1, 1, None,
                        res=last[0], res_hw=(last[1][1], last[1][2]))
            outs.insert(0, conv(last, f"{f}layer_blocks.{i}.0.weight", f"{f}layer_blocks.{i}.1", 3, 1, None))
        outs.append(maxpool(outs[-1], 1, 2, 0, "backbone.fpn.extra_blocks.pool"))
        if pack_only:
            for k in ("rpn.head.conv.0.0", "rpn.head.conv.1.0", "rpn.head.cls_logits", "rpn.head.bbox_pred"):
                self._conv_bias(k + ".weight", k + ".bias")
            for i in range(4):
                self._conv_bn(f"roi_heads.box_head.{i}.0.weight", f"roi_heads.box_head.{i}.1", self.BN_EPS)
            self._fc6()
            self._predictor()
            return P

        # ---- RPN head (shared over levels) + proposal filtering
        A = 3
        heads, grids = [], []
        P.fork(3)  # the five RPN head levels are independent
        for lvl, fm in enumerate(outs):
            P.lane(lvl % 4)
            t = conv(fm, "rpn.head.conv.0.0.weight", None, 3, 1, "RE", bias_key="rpn.head.conv.0.0.bias",
                     name=f"rpn.head.conv.0@{lvl}")
            t = conv(t, "rpn.head.conv.1.0.weight", None, 3, 1, "RE", bias_key="rpn.head.conv.1.0.bias",
                     name=f"rpn.head.conv.1@{lvl}")
            # objectness [B, HW*A] (dense: the top-k reads it contiguously) and deltas [B, HW*A, 4]
            o = conv(t, "rpn.head.cls_logits.weight", None, 1, 1, None, bias_key="rpn.head.cls_logits.bias",
                     name=f"rpn.head.cls_logits@{lvl}")
            d = conv(t, "rpn.head.bbox_pred.weight", None, 1, 1, None, bias_key="rpn.head.bbox_pred.bias",
                     name=f"rpn.head.bbox_pred@{lvl}")
            heads.append((o[0], d[0]))
            grids.append((fm[1][1], fm[1][2]))
        P.join()
        anchor_bufs = [P.const(a, name=f"rpn.anchors@{l}") for l, a in enumerate(anc.rpn_anchors(grids, (Hp, Wp)))]
        L = len(outs)
        KM = self.RPN_PRE
        rrec = [P.buf((B, L, KM, 4), name="rpn.rec.box"), P.buf((B, L, KM), name="rpn.rec.score"),
                P.buf((B, L, KM), torch.int32, name="rpn.rec.tb"), P.buf((B, L, KM), torch.int32, name="rpn.rec.lvl"),
                P.buf((B, L), torch.int32, name="rpn.rec.count")]
        pi = {0: B, 1: L, 2: 0, 3: A, 4: self.RPN_PRE, 5: KM}
        pp = {}
        for l in range(L):
            pi[6 + l] = grids[l][0] * grids[l][1] * A
            pp[l] = heads[l][0]
            pp[15 + l] = heads[l][1]
            pp[5 + l] = anchor_bufs[l]
        for j in range(5):
            pp[10 + j] = rrec[j]
        P.add(Op(ops.RPN_LEVEL_NMS, pi, pp, {0: Ho, 1: Wo, 2: self.RPN_MIN, 3: self.RPN_SCORE}, {0: self.RPN_NMS},
                 name="rpn.filter_proposals"))
        R = self.RPN_POST
        props = P.buf((B, R, 4), name="proposals")
        pscore = P.buf((B, R), name="proposal_scores")
        pcount = P.buf((B,), torch.int32, name="proposal_count")
        P.add(Op(ops.MERGE_TOPK, {0: B, 1: L, 2: KM, 3: R},
                 {0: rrec[0], 1: rrec[1], 2: rrec[2], 3: rrec[3], 4: rrec[4], 5: None, 6: props, 7: pscore, 8: None,
                  9: pcount}, name="rpn.post_nms_top_n"))

        # ---- MultiScaleRoIAlign (levels '0'..'3')
        C = 256
        roi = P.buf((B * R, 7, 7, C), name="box_roi_pool")
        ri = {0: 1, 1: B * R, 2: R, 3: B, 4: C, 5: 7, 6: 7, 7: 2, 8: 4, 9: 2, 10: 5}
        rp = {4: props, 5: pcount, 6: roi}
        rf = {}
        for l in range(4):
            fh, fw = outs[l][1][1], outs[l][1][2]
            ri[11 + l], ri[15 + l] = fh, fw
            rp[l] = outs[l][0]
            # MultiScaleRoIAlign._infer_scale: 2 ** round(log2(feat / image)) in float32
            rf[l] = 2.0 ** float(torch.tensor(float(fh) / float(Ho)).log2().round())
        P.add(Op(ops.ROI_ALIGN, ri, rp, rf, name="roi_heads.box_roi_pool"))

        # ---- box head + predictor
        cur = (roi, (B * R, 7, 7, C))
        for i in range(4):
            cur = conv(cur, f"roi_heads.box_head.{i}.0.weight", f"roi_heads.box_head.{i}.1", 3, 1, "RE")
        w, b, K, Kpad, cin = self._fc6()
        fc6 = P.buf((B * R, 1024), name="roi_heads.box_head.5")
        conv_op(P, cur[0], (B * R, 1, 1, 7 * 7 * C), w, b, 1024, 1, 1, 0, "RE", fc6, (B * R, 1, 1, 1024), K, Kpad,
                name="roi_heads.box_head.5")
        w, b, K, Kpad, cin = self._predictor()
        LD = 456
        pred = P.buf((B * R, LD), name="box_predictor")
        conv_op(P, fc6, (B * R, 1, 1, 1024), w, b, 5 * NC, 1, 1, 0, None, pred, (B * R, 1, 1, 5 * NC), K, Kpad,
                y_pstride=LD, y_bstride=LD, name="roi_heads.box_predictor")

        # ---- RoIHeads.postprocess_detections
        scores = P.buf((B, R, NC), name="box_scores")
        bxs = P.buf((B, R, NC, 4), name="box_decoded")
        P.add(Op(ops.BOX_SCORES, {0: LD, 1: B, 2: R, 3: NC, 4: 4 * NC, 5: 0}, {0: pred, 1: props, 2: pcount,
                                                                             3: scores, 4: bxs},
                 {0: Ho, 1: Wo}, name="roi_heads.scores_decode"))
        NS = NC - 1
        brec = [P.buf((B, NS, R, 4), name="box.rec.box"), P.buf((B, NS, R), name="box.rec.score"),
                P.buf((B, NS, R), torch.int32, name="box.rec.tb"), P.buf((B, NS, R), torch.int32, name="box.rec.lbl"),
                P.buf((B, NS), torch.int32, name="box.rec.count")]
        P.add(Op(ops.BOX_CLASS_NMS, {0: B, 1: R, 2: NC, 3: R},
                 {0: scores, 1: bxs, 2: pcount, 3: brec[0], 4: brec[1], 5: brec[2], 6: brec[3], 7: brec[4]},
                 {0: self.BOX_SCORE, 1: self.BOX_MIN}, {0: self.BOX_NMS}, name="roi_heads.class_nms"))
        ratio = np.tile(np.asarray([np.float32(W) / np.float32(Wo), np.float32(H) / np.float32(Ho)], np.float32),
                        (B, 1))
        ratio_b = P.const(ratio, name="ratio")
        N = self.BOX_DETS
        P.out_box = P.buf((B, N, 4), name="out.boxes")
        P.out_score = P.buf((B, N), name="out.scores")
        P.out_label = P.buf((B, N), torch.int64, name="out.labels")
        P.out_count = P.buf((B,), torch.int32, name="out.count")
        P.add(Op(ops.MERGE_TOPK, {0: B, 1: NS, 2: R, 3: N},
                 {0: brec[0], 1: brec[1], 2: brec[2], 3: brec[3], 4: brec[4], 5: ratio_b, 6: P.out_box,
                  7: P.out_score, 8: P.out_label, 9: P.out_count}, name="roi_heads.detections_per_img"))
        P.input = inp
        P.feats = [o[0] for o in outs]
        P.rpn_heads = heads  # per level (objectness [B,H,W,3], deltas [B,H,W,12]): the parity tests' RPN inputs
        P.proposals, P.proposal_count = props, pcount
        P.box_features = roi
        P.pred = pred
        P.box_scores, P.box_decoded = scores, bxs
        P.resized = (Ho, Wo, Hp, Wp)
        return P


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
    GN_GROUPS, GN_EPS = 32, 1e-5
    A = arch.RETINA_ANCHORS
    SELECT_CHUNK = 1 << 16  # flat (anchor, class) indices per first-stage select workgroup

    def table(self):
        return arch.retinanet_table(self.num_classes)

    def _gn(self, p):
        key = ("gn", p)
        if key not in self._w:
            self._w[key] = (self.pack.add(_np(self.sd[p + ".weight"])), self.pack.add(_np(self.sd[p + ".bias"])))
        return self._w[key]

    def build_plan(self, B, H, W, u8=False, pack_only=False):
        P = Plan(self.pack, self.device or "cpu")
        K, A = self.num_classes, self.A
        inp, (Ho, Wo, Hp, Wp), conv, maxpool, cs = self._lower_body(P, B, H, W, u8)
        f = "backbone.fpn."
        c3, c4, c5 = cs[1], cs[2], cs[3]
        last = conv(c5, f + "inner_blocks.2.0.weight", None, 1, 1, None, bias_key=f + "inner_blocks.2.0.bias")
        outs = [conv(last, f + "layer_blocks.2.0.weight", None, 3, 1, None, bias_key=f + "layer_blocks.2.0.bias")]
        for i, c in ((1, c4), (0, c3)):
            last = conv(c, f"{f}inner_blocks.{i}.0.weight", None, 1, 1, None, bias_key=f"{f}inner_blocks.{i}.0.bias",
                        res=last[0], res_hw=(last[1][1], last[1][2]))
            outs.insert(0, conv(last, f"{f}layer_blocks.{i}.0.weight", None, 3, 1, None,
                                bias_key=f"{f}layer_blocks.{i}.0.bias"))
        p6 = conv(c5, f + "extra_blocks.p6.weight", None, 3, 2, None, bias_key=f + "extra_blocks.p6.bias")
        p7 = conv(p6, f + "extra_blocks.p7.weight", None, 3, 2, None, bias_key=f + "extra_blocks.p7.bias",
                  in_relu=True)
        outs += [p6, p7]
        branches = (("classification_head", "cls_logits", K), ("regression_head", "bbox_reg", 4))
        if pack_only:
            for br, last_name, _ in branches:
                for i in range(4):
                    self._conv_nobias(f"head.{br}.conv.{i}.0.weight")
                    self._gn(f"head.{br}.conv.{i}.1")
                self._conv_bias(f"head.{br}.{last_name}.weight", f"head.{br}.{last_name}.bias")
            return P

        grids = [(o[1][1], o[1][2]) for o in outs]
        na = [gh * gw * A for gh, gw in grids]
        a0 = [int(v) for v in np.concatenate([[0], np.cumsum(na)[:-1]])]
        Atot = int(sum(na))
        cls = P.buf((B, Atot, K), name="head.cls_logits")
        reg = P.buf((B, Atot, 4), name="head.bbox_regression")
        C = 256
        P.fork(3)  # the five levels' head towers are independent
        for lvl, fm in enumerate(outs):
            P.lane(lvl % 4)
            hw = fm[1][1] * fm[1][2]
            for br, last_name, kk in branches:
                dst = cls if kk == K else reg
                t, sc, sh = fm, None, None
                for i in range(4):
                    q = f"head.{br}.conv.{i}."
                    t = conv(t, q + "0.weight", None, 3, 1, None, in_scale=sc, in_shift=sh, in_relu=i > 0,
                             name=f"{q}0@{lvl}")
                    gamma, beta = self._gn(q + "1")
                    sc = P.buf((B, C), name=f"{q}1.scale@{lvl}")
                    sh = P.buf((B, C), name=f"{q}1.shift@{lvl}")
                    P.add(Op(ops.GN_STATS, {0: B, 1: hw, 2: C, 3: self.GN_GROUPS},
                             {0: t[0], 1: gamma, 2: beta, 3: sc, 4: sh}, {0: self.GN_EPS}, name=f"{q}1@{lvl}"))
                conv(t, f"head.{br}.{last_name}.weight", None, 3, 1, None, bias_key=f"head.{br}.{last_name}.bias",
                     in_scale=sc, in_shift=sh, in_relu=True, out=(dst, A * kk, Atot * kk, a0[lvl] * kk),
                     name=f"head.{br}.{last_name}@{lvl}")
        P.join()
        anchors = P.const(np.concatenate(anc.retina_anchors(grids, (Hp, Wp)), 0), name="anchors")

        # ---- RetinaNet.postprocess_detections
        L, KM = len(outs), self.TOPK
        lrec = [P.buf((B, L, KM, 4), name="retina.cand.box"), P.buf((B, L, KM), name="retina.cand.score"),
                P.buf((B, L, KM), torch.int32, name="retina.cand.tb"),
                P.buf((B, L, KM), torch.int32, name="retina.cand.label"),
                P.buf((B, L), torch.int32, name="retina.cand.count")]
        CH = self.SELECT_CHUNK
        nchunk = max(-(-n * K // CH) for n in na)
        ck = P.buf((B, L, nchunk, 1024), torch.int32, name="retina.chunk.key")
        ci = P.buf((B, L, nchunk, 1024), torch.int32, name="retina.chunk.idx")
        cc = P.buf((B, L, nchunk), torch.int32, name="retina.chunk.count")
        si = {0: B, 1: L, 2: Atot, 3: K, 4: self.TOPK, 5: KM, 16: CH, 17: nchunk}
        for l in range(L):
            si[6 + l], si[11 + l] = a0[l], na[l]
        P.add(Op(ops.RETINA_SELECT, si, {0: cls, 1: reg, 2: anchors, 3: lrec[0], 4: lrec[1], 5: lrec[2],
                                         6: lrec[3], 7: lrec[4], 8: ck, 9: ci, 10: cc},
                 {0: Ho, 1: Wo, 2: self.SCORE}, name="retina.select_topk"))
        N = self.DETS
        crec = [P.buf((B, K, N, 4), name="retina.kept.box"), P.buf((B, K, N), name="retina.kept.score"),
                P.buf((B, K, N), torch.int32, name="retina.kept.tb"), P.buf((B, K, N), torch.int32, name="retina.kept.lbl"),
                P.buf((B, K), torch.int32, name="retina.kept.count")]
        P.add(Op(ops.RETINA_CLASS_NMS, {0: B, 1: L, 2: KM, 3: K, 4: N},
                 {0: lrec[0], 1: lrec[1], 2: lrec[2], 3: lrec[3], 4: lrec[4], 5: crec[0], 6: crec[1], 7: crec[2],
                  8: crec[3], 9: crec[4]}, d={0: self.NMS}, name="retina.batched_nms"))
        ratio = np.tile(np.asarray([np.float32(W) / np.float32(Wo), np.float32(H) / np.float32(Ho)], np.float32),
                        (B, 1))
        ratio_b = P.const(ratio, name="ratio")
        P.out_box = P.buf((B, N, 4), name="out.boxes")
        P.out_score = P.buf((B, N), name="out.scores")
        P.out_label = P.buf((B, N), torch.int64, name="out.labels")
        P.out_count = P.buf((B,), torch.int32, name="out.count")
        P.add(Op(ops.MERGE_TOPK, {0: B, 1: K, 2: N, 3: N},
                 {0: crec[0], 1: crec[1], 2: crec[2], 3: crec[3], 4: crec[4], 5: ratio_b, 6: P.out_box,
                  7: P.out_score, 8: P.out_label, 9: P.out_count}, name="retina.detections_per_img"))
        P.input = inp
        P.feats = [o[0] for o in outs]
        P.cls_logits, P.bbox_regression = cls, reg
        P.cand_count = lrec[4]
        P.level_anchors = na  # anchors per level in the concatenated head outputs (parity tests)
        P.resized = (Ho, Wo, Hp, Wp)
        return P


# ====================================================================================== factories
def ssdlite320_mobilenet_v3_large(weights=None, num_classes=91, reduced_tail=True, state_dict=None, seed=0):
    """Builder mirroring torchvision's (detect.py:24,26).  ``weights="DEFAULT"`` would download COCO
    weights, impossible offline: pass ``state_dict=`` (e.g. torch.load(--model-path)) or get seeded
    synthetic weights (edgeml_amd.synthetic) in their place."""
    from . import synthetic
    if state_dict is None:
        state_dict = synthetic.synthetic_state_dict("ssd", num_classes, reduced_tail, seed=seed)
    return SSDLite320(state_dict, num_classes, reduced_tail)


def fasterrcnn_resnet50_fpn_v2(weights=None, num_classes=91, state_dict=None, seed=0):
    """Builder mirroring torchvision's (detect.py:30,32); see ssdlite320_mobilenet_v3_large."""
    from . import synthetic
    if state_dict is None:
        state_dict = synthetic.synthetic_state_dict("faster_rcnn", num_classes, seed=seed)
    return FasterRCNNFPNv2(state_dict, num_classes)


def retinanet_resnet50_fpn_v2(weights=None, num_classes=91, state_dict=None, seed=0):
    """Builder mirroring torchvision's (detect.py:36,38); see ssdlite320_mobilenet_v3_large."""
    from . import synthetic
    if state_dict is None:
        state_dict = synthetic.synthetic_state_dict("retinanet", num_classes, seed=seed)
    return RetinaNetFPNv2(state_dict, num_classes)
