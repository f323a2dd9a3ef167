"""Benchmark of the detection-output hot path (BASELINE.json metric, configs[1] / configs[2]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model ssd|frcnn|both] [--no-cpu]

A step = one forward of the detector over one batch of synthetic 640x640 images already resident in
HBM as the decoded uint8 images the detect CLI hands the engine (read_image's output, detect.py:57; the
/255 of detect.py:58 runs in the device transform, bit-identical to the host's float path; --input f32
keeps the model contract's float images instead) (/255 -> preprocess -> backbone -> heads -> decode ->
NMS -> final top-k), replayed from a captured
hipGraph, plus the D2H copy of the batch's detections (counts, boxes, scores, labels) into pinned
host memory.  The steps rotate over the model's INFLIGHT independent plan instances
(SSDLite 4, FRCNN 2: the counts the detect CLI's run_batches keeps on the device); the SSD rate at
the other count is reported beside it ("alt_inflight").  N=1 workload: SSDLite320-MobileNetV3 at batch 32 (configs[1]); FRCNN-R50-FPN-v2 at
batch 8 (configs[2]) is measured beside it and reported under "frcnn".  For N>1 the script is
launched by torch.distributed.run: one process per GPU, each replays its own batch (weak scaling:
images are independent, no collective on the data path); the timed region is bracketed by a
barrier + device sync and the max over ranks is taken.

Extra objects on the JSON line:
  roofline      the dominant kernel of the SSD step (the dominant family by solo device time, its largest
                launch): algorithmic bytes or flops per launch / its average launch time IN THE RUNNING
                PIPELINE (the kernel's own start / end stamps on the GPU clock, written into a probe slot
                in every instance's captured graph: pipeline_launch_ms); the same launch timed alone
                with HIP events is reported beside it (launch_ms_solo / frac_solo)
  cpu_baseline  the CPU oracle (a restatement of the reference's torchvision CPU path, detect.py's
                batch=1 loop) timed on a bounded sample on this host, rank 0 only
  end_to_end    uint8 host images -> detect.py's .npy rows: pinned staging, H2D of the bytes, forward,
                D2H, row formatting (model.run_batches, the CLI's path; JPEG decode excluded)
  orie          the metric's "ORIE max-abs-diff vs ref": ORIE of the engine's SSDLite/FRCNN rows (GPU
                reward) against ORIE of the CPU oracle's rows (oracle consumer) on a small sample
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
SSD_BYTES_PER_IMG = 87.1e6   # algorithmic HBM bytes per SSDLite image
FP32_MFMA_PEAK_TFS = 157.3   # dense fp32 MFMA (= fp32 vector peak)


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # one rank per GPU over RCCL; EDGEDET_DIST_BACKEND=gloo with more ranks than GPUs rehearses
        # the multi-rank logic on a one-GPU box (ranks share the device)
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dist.init_process_group(os.environ.get("EDGEDET_DIST_BACKEND", "nccl"))
        return dist, dist.get_rank(), world
    torch.cuda.set_device(0)
    return None, 0, 1


def d2h_buffers(plan):
    """Pinned host buffers for one instance's detections (count, boxes, scores, labels)."""
    return [(t, torch.empty(tuple(t.shape), dtype=t.dtype, pin_memory=True))
            for t in (plan.out_count.tensor(), plan.out_box.tensor(), plan.out_score.tensor(),
                      plan.out_label.tensor())]


def step(plan, stream, d2h):
    plan.replay(stream)
    with torch.cuda.stream(stream):
        for dev, host in d2h:
            host.copy_(dev, non_blocking=True)


TIMING = {}  # how the last timed_steps call measured (reported on the JSON line)
SETTLE_S = float(os.environ.get("EDGEDET_BENCH_SETTLE", "0.5"))  # untimed device warm-up before the warmup passes (s)


def timed_steps(plan, stream, steps, warmup, dist, extra=()):
    """Seconds for `steps` whole-batch passes (forward graph + D2H of the detections) in steady state.

    With `extra` = [(plan, stream), ...] the passes rotate over independent plan instances (own arena,
    own graph, own pinned output buffers) on their own streams, so batch k+1's first convolutions
    overlap batch k's low-occupancy NMS tail; every pass is still a complete forward of its own batch,
    and each instance's passes stay ordered on its stream.

    Steady state (round 4): a completion event is recorded on the instance's stream after each pass's
    D2H.  The pipeline is NOT drained between the warmup and the timed passes, so the timed region
    starts full, as in a long run, with no fill or drain latency in the denominator; the host keeps at
    most 2n passes outstanding throughout (settle, warmup and timed passes alike).  The interval runs
    between two completions of the SAME instance: from a warmup pass j0 to the last timed pass, j0
    chosen r = (-K) mod n passes before the last warmup pass so that K + r is a multiple of the n
    instances; between two completions of one instance the pipeline is in the same phase, so the
    interval holds (K + r) / n cycles, and the time returned is that interval scaled by K / (K + r).
    Concurrent instances can finish in bursts (the three FRCNN plans finish within a few ms of each
    other every ~68 ms, profiles/r4d_trace_frcnn.jsonl), so an interval between completions of
    different instances would count part of a burst for free.  Two earlier forms read too high on
    FRCNN after the SSD run (443 and 538 img/s against ~360, profiles/r4c_bench_driver_bias.json): the
    timed passes were issued all at once, and two of the three instances' streams shared a hardware
    queue, so the third instance ran ahead alone inside the window (profiles/r4d_trace_both.jsonl);
    the issue discipline and fresh per-model streams (main) remove both.  Every instance was primed
    when it was captured (graph uploaded and replayed, plan.capture), and the warmup covers each
    instance at least once.  The ranks start together (barrier + device sync before the warmup) and
    end together (device sync + barrier after the last pass); the max over ranks is taken.  After the K
    timed passes 2n more passes are issued untimed (a full pipeline at the end of the window too, as at
    its start).  The host wall clock of the K timed passes (from the first timed issue to the last timed
    pass's completion) is kept in TIMING."""
    lanes = [(p, s, d2h_buffers(p)) for p, s in [(plan, stream)] + list(extra)]
    n = len(lanes)
    warm = max(warmup, n)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    # settle: untimed passes for SETTLE_S of wall time before the warmup, issued like the timed ones
    # (round robin, never drained: the host waits only for the pass 2n back, so the instances keep the
    # staggered phases of a long run instead of starting in lockstep) -- the clocks and the overlap the
    # timed passes see are a long run's (profiles/r4a_bench_driver.json: 1.67 ms/step over 20 steps
    # right after an idle host phase, against 1.38 in a 750-step run).  Settle, warmup and timed
    # passes share one issue discipline (issue): at most 2n passes outstanding.  Issued all at once,
    # an instance whose stream had no backlog ran ahead of the others inside the timed window and the
    # interval measured it alone (profiles/r4d_trace_both.jsonl).
    ring = []  # completion events of the outstanding passes, oldest first

    def issue(k, timing=False):  # pass k round robin; at most 2n passes outstanding before it
        while len(ring) >= 2 * n:
            ring.pop(0).synchronize()
        p_, s_, d_ = lanes[k % n]
        step(p_, s_, d_)
        e = torch.cuda.Event(enable_timing=timing)
        e.record(s_)
        ring.append(e)
        return e

    t_settle, settled = time.perf_counter(), 0
    while time.perf_counter() - t_settle < SETTLE_S or settled < 2 * n:
        issue(settled)
        settled += 1
    r = (-steps) % n  # warm >= n > r: the interval's first completion is a warmup pass
    for i in range(warm):
        e = issue(settled + i, timing=i == warm - 1 - r)
        if i == warm - 1 - r:
            mark = e
    done = []
    t0 = time.perf_counter()
    for i in range(steps):
        done.append(issue(settled + warm + i, timing=True))
    # tail: 2n more passes, untimed, so the last timed passes complete under the contention of the
    # passes behind them, as every pass of a long run does.  Without them the pipeline drains at the
    # end of the window: the last passes run with nothing queued behind them and finish early, which
    # read a 20-pass window 1-3 % above the steady rate (profiles/r5c_bias.txt; a 3,000-pass trace is
    # flat, and its 20-pass windows scatter by 0.8 %).
    for i in range(2 * n):
        issue(settled + warm + steps + i)
    done[-1].synchronize()
    wall = time.perf_counter() - t0
    for _, s, _ in lanes:
        s.synchronize()
    torch.cuda.synchronize()
    el = mark.elapsed_time(done[-1]) / 1e3 * steps / (steps + r)
    if os.environ.get("EDGEDET_BENCH_TRACE"):  # per-pass completion times (timing investigation)
        with open(os.environ["EDGEDET_BENCH_TRACE"], "a") as fh:
            fh.write(json.dumps({"n": n, "r": r, "warm": warm, "settled": settled,
                                 "streams": [int(s_.cuda_stream) for _, s_, _ in lanes],
                                 "pass_lane": [(settled + warm + i) % n for i in range(steps)],
                                 "done_ms": [round(mark.elapsed_time(e), 3) for e in done]}) + "\n")
    if dist:
        dist.barrier()
        t = torch.tensor([el, wall], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, wall = (float(v) for v in t.tolist())
    TIMING.clear()
    TIMING.update({"method": "steady state: HIP completion events after each pass's D2H, pipeline kept full "
                             "across the start and the end (2n untimed tail passes); interval between two "
                             "completions of the same instance (K + r passes, r = (-K) mod instances), "
                             "scaled to K",
                   "device_s": round(el, 6), "interval_passes": steps + r, "wall_s": round(wall, 6),
                   "warmup_passes": warm, "settle_passes": settled, "instances": n})
    return el


def end_to_end(m, B, batches, seed):
    """uint8 host images -> the .npy rows detect.py writes, through model.run_batches as the detect
    CLI runs it: each batch is a pinned uint8 [B,3,640,640] buffer (the CLI's decode pool writes the
    decoded images straight into one), uploaded as bytes, /255 on the device, forward, D2H of the
    detections, rows by fmt.format_batch (byte-identical to detect.py:79-103), two batches in flight.
    JPEG decode is excluded (the CLI's thread pool; tools/pipeline_bench.py times it)."""
    from edgeml_amd import fmt, synthetic
    imgs = synthetic.make_batch_u8(B, 640, 640, seed=seed).pin_memory()
    work = [(k, imgs) for k in range(batches)]
    for _ in m.run_batches(work[:m.INFLIGHT + 1], raw=True):  # builds and captures every slot's plan
        pass
    torch.cuda.synchronize()
    n, t0 = 0, time.perf_counter()
    for _, cnt, box, score, label in m.run_batches(work, raw=True):
        n += len(fmt.format_batch(box, score, label, cnt, 640, 640))
    el = time.perf_counter() - t0
    # the PCIe ceiling of this path: pinned uint8 batch -> device, alone
    dev = torch.empty(imgs.shape, dtype=imgs.dtype, device="cuda")
    dev.copy_(imgs, non_blocking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(10):
        dev.copy_(imgs, non_blocking=True)
    torch.cuda.synchronize()
    h2d = 10 * imgs.numel() / (time.perf_counter() - t1) / 1e9
    return {"value": round(n / el, 2), "unit": "images/s", "images": n, "batch": B,
            "h2d_GBps": round(h2d, 1), "h2d_bound_images_s": round(h2d * 1e9 / (imgs.numel() / B), 1),
            "path": "pinned uint8 host images -> H2D (bytes) -> forward -> D2H -> .npy rows "
                    "(no JPEG decode, no file write)"}


def fill_input(plan, B, seed):
    """The plan's input batch: the decoded uint8 images (u8 plans: read_image's output, detect.py:57,
    divided by 255 in the device transform) or the model contract's float images."""
    from edgeml_amd import synthetic
    src = synthetic.make_batch_u8(B, 640, 640, seed=seed) if plan.u8 else synthetic.make_batch(B, 640, 640, seed=seed)
    plan.input.tensor().copy_(src.cuda())


def inflight_instances(m, B, n, seed, u8=True):
    """n-1 more independent plans of the same (model, B, 640, 640), inputs filled like the first."""
    out = []
    for k in range(1, n):
        p = m.build_plan(B, 640, 640, u8).finalize()
        fill_input(p, B, seed + k)
        s = torch.cuda.Stream()
        p.capture(s)
        out.append((p, s))
    return out


# ------------------------------------------------------------------------------ per-op costs
BF16X6_PEAK_TFS = 157.3 * 16 / 6  # dense bf16 MFMA (16x the fp32 rate) / six partial products

CONV_TILES = {  # tile id (csrc/conv.hip conv_launch) -> kernel, BM, BN, threads (0 BM = waves of 64-row pw)
    1: ("conv_mfma_kernel", 128, 32, 256), 2: ("conv_mfma_kernel", 128, 64, 256),
    3: ("conv_mfma_kernel", 128, 128, 256), 4: ("conv_mfma_kernel", 256, 128, 512),
    5: ("conv_mfma_kernel", 64, 64, 256), 6: ("conv_mfma_kernel", 32, 32, 64),
    10: ("pw_mfma_kernel", 256, 64, 256), 11: ("pw_mfma_kernel", 512, 32, 256), 12: ("pw_mfma_kernel", 128, 64, 256),
    15: ("pw_mfma_kernel", 256, 32, 256), 13: ("pw_splitk_kernel", 32, 32, 256), 14: ("pw_splitk_kernel", 32, 64, 256),
    16: ("pw_splitk_kernel", 32, 32, 512), 17: ("pw_splitk_kernel", 32, 64, 512),
    21: ("conv_x6_kernel", 64, 64, 256), 22: ("conv_x6_kernel", 128, 64, 256), 23: ("conv_x6_kernel", 128, 128, 256), 24: ("conv_x6_kernel", 256, 128, 512),
    25: ("conv_x6b_kernel", 256, 128, 512), 27: ("conv_x6_kernel", 128, 64, 512), 28: ("conv_x6_kernel", 128, 128, 512),
    29: ("conv_x6b_kernel", 128, 128, 512), 30: ("conv_x6b_kernel", 128, 128, 512),
    31: ("conv_x6b_kernel", 64, 128, 512), 32: ("conv_x6b_kernel", 64, 128, 512),
    38: ("conv_x6b_kernel", 128, 64, 512), 39: ("conv_x6b_kernel", 128, 256, 512),
}


def conv_tile(op_record):
    """The kernel variant libedgedet runs for this CONV record (edgedet_conv_tile)."""
    import ctypes
    from edgeml_amd import ops as O
    t = O.lib().edgedet_conv_tile(op_record.ctypes.data_as(ctypes.c_void_p))
    if t < 0:
        O.check(t)
    return t


def conv_grid(op, rec):
    """(kernel name, workgroups, threads per workgroup, fp32-equivalent MFMA peak) of a CONV record."""
    i = op.i
    M, Cout = i[0] * i[4] * i[5], i[6]
    name, bm, bn, nt = CONV_TILES[conv_tile(rec)]
    wg = -(-M // bm) * -(-Cout // bn)
    return name, wg, nt, (BF16X6_PEAK_TFS if name.startswith("conv_x6") else FP32_MFMA_PEAK_TFS)


def op_work(op):
    """(family, algorithmic flops, algorithmic HBM bytes) of one plan op: every input read once,
    every output written once (SURVEY.md §8d byte model)."""
    from edgeml_amd import ops as O
    i = op.i
    k = op.kind
    if k == O.CONV:
        B, H, W, Cin, Ho, Wo, Cout, KH, KW = (i[j] for j in range(9))
        M = B * Ho * Wo
        flops = 2.0 * M * Cout * KH * KW * Cin
        byts = 4.0 * (B * H * W * Cin + Cout * KH * KW * Cin + M * Cout)
        if op.p.get(4) is not None:
            byts += 4.0 * M * Cout
        return "conv", flops, byts
    if k == O.DWCONV:
        B, H, W, C, Ho, Wo, K = (i[j] for j in range(7))
        return "dwconv", 2.0 * B * Ho * Wo * C * K * K, 4.0 * (B * H * W * C + B * Ho * Wo * C + C * K * K)
    if k == O.SSD_STEM:  # stem conv 3x3 s2 (4 -> 16) + depthwise 3x3 + projection 16 -> 16 + residual
        B, H, W, Ho, Wo = (i[j] for j in range(5))
        H0, W0 = i[7], i[8]
        if H0:  # the transform folded in: the source image in (uint8 or float), no NHWC4 intermediate
            src = B * 3 * H0 * W0 * (1 if op.p.get(9) is not None else 4)
            return "stem", 2.0 * B * Ho * Wo * 16 * (36 + 9 + 16), float(src) + 4.0 * B * Ho * Wo * 16
        return "stem", 2.0 * B * Ho * Wo * 16 * (36 + 9 + 16), 4.0 * (B * H * W * 4 + B * Ho * Wo * 16)
    if k == O.PREPROCESS:
        B, H, W, Ho, Wo, Hp, Wp = (i[j] for j in range(7))
        return "preprocess", 0.0, 4.0 * (B * 3 * H * W + B * Hp * Wp * 4)
    if k == O.CHANNEL_MEAN:
        return "se_squeeze", float(i[0] * i[1] * i[2]), 4.0 * i[0] * i[1] * i[2]
    if k == O.SE_FC:
        return "se_fc", 4.0 * i[0] * i[1] * i[2], 4.0 * (2 * i[1] * i[2] + i[0] * ((i[4] or O.SE_PARTS) + 1) * i[1] + 2 * i[0] * i[2])
    if k == O.MAXPOOL:
        B, H, W, C, Ho, Wo = (i[j] for j in range(6))
        return "maxpool", 0.0, 4.0 * (B * H * W * C + B * Ho * Wo * C)
    if k == O.SSD_SCORES:
        B, A, NC = i[0], i[1], i[2]
        return "ssd_scores", 0.0, 4.0 * (2 * B * A * NC + 2 * B * A * 4 + A * 4)
    if k == O.SSD_CLASS_NMS:
        B, A, NC = i[0], i[1], i[2]
        return "class_nms", 0.0, 4.0 * (B * NC * A + B * A * 4)
    if k == O.SSD_POSTPROCESS:
        B, A, NC, KM = i[0], i[1], i[2], i[3]
        return "ssd_nms", 0.0, 4.0 * (B * NC * A + B * A * 4 + 2 * 2 * B * (NC - 1) * KM)
    if k == O.MERGE_TOPK:
        return "merge_topk", 0.0, 4.0 * i[0] * i[1] * i[2] * 7
    if k == O.RPN_LEVEL_NMS:
        n = sum(i[6 + l] for l in range(i[1]))
        return "rpn_nms", 0.0, 4.0 * i[0] * n * 5
    if k == O.ROI_ALIGN:
        return "roi_align", 0.0, 4.0 * 2 * i[1] * i[5] * i[6] * i[4]
    if k == O.BOX_SCORES:
        return "box_scores", 0.0, 4.0 * i[1] * i[2] * (i[0] + 5 * i[3])
    if k == O.BOX_CLASS_NMS:
        return "class_nms", 0.0, 4.0 * i[0] * i[1] * i[2] * 5
    if k == O.GN_STATS:
        return "group_norm", 0.0, 4.0 * i[0] * i[1] * i[2]
    if k == O.RETINA_SELECT:
        n = sum(i[11 + l] for l in range(i[1]))
        return "retina_select", 0.0, 4.0 * i[0] * n * (i[3] + 4)
    if k == O.RETINA_CLASS_NMS:
        return "retina_nms", 0.0, 4.0 * i[0] * i[1] * i[2] * 7
    if k == O.MBCONV:  # expand 1x1 + depthwise KxK + project 1x1 (+ residual): block input in, output out
        B, H, W, Cin, Cexp, Cout, Ho, Wo, K = (i[j] for j in range(9))
        fl = 2.0 * B * (H * W * Cin * Cexp + Ho * Wo * Cexp * (K * K + Cout))
        return "mbconv", fl, 4.0 * (B * H * W * Cin + B * Ho * Wo * Cout + Cexp * (Cin + K * K + Cout + 2) + Cout)
    if k in (O.FORK, O.JOIN, O.WAIT, O.GROUP):
        return "lanes", 0.0, 0.0
    if k == O.MEMSET:  # zeroing the output of a split-K conv
        return "conv", 0.0, float(i[0])
    return f"kind{k}", 0.0, 0.0


def group_members(plan, k):
    """Indices of the records a GROUP record at k issues as one launch."""
    return list(range(k + 1, k + 1 + int(plan.ops[k].i[0])))


def per_op_times(plan, stream, reps=20):
    """Average device time of each launch of the plan, run alone between HIP events on `stream`: an
    op per record, a GROUP record with its members as the one grouped launch they are (the time is
    attributed to the GROUP record, its members get 0)."""
    import ctypes
    from edgeml_amd import ops as O
    L = O.lib()
    recs = plan.records.copy()
    recs["i"][:, O.LANE_FIELD] = 0  # time every launch alone on the timed stream
    sh = O.stream_handle(stream)
    res = [0.0] * len(recs)
    k = 0
    with torch.cuda.stream(stream):
        while k < len(recs):
            kind = recs[k]["kind"]
            if kind in (O.FORK, O.JOIN, O.WAIT):
                k += 1
                continue
            n = 1 + (int(recs[k]["i"][0]) if kind == O.GROUP else 0)
            ptr = recs[k:k + n].ctypes.data_as(ctypes.c_void_p)
            O.check(L.edgedet_plan_run(ptr, n, sh))
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                L.edgedet_plan_run(ptr, n, sh)
            e1.record(stream)
            e1.synchronize()
            res[k] = e0.elapsed_time(e1) / reps
            k += n
    return res


OP_DUMP = {}


def unit_work(plan, k):
    """(family, flops, bytes) of the launch at record k: one op, or a GROUP's members summed."""
    from edgeml_amd import ops as O
    op = plan.ops[k]
    if op.kind != O.GROUP:
        return op_work(op)
    ws = [op_work(plan.ops[j]) for j in group_members(plan, k)]
    return ws[0][0], sum(w[1] for w in ws), sum(w[2] for w in ws)


def roofline_for(plan, stream, step_ms, model=""):
    """Dominant kernel family of the step (by measured device time) and its longest launch, priced
    against the roof that binds it (max of flops / the MFMA peak and bytes / HBM peak).  A grouped
    launch (EDGEDET_OP_GROUP) is one launch: its members' work summed, its kernel the grouped one."""
    from edgeml_amd import ops as O
    times = per_op_times(plan, stream)
    in_group = set()
    for k, op in enumerate(plan.ops):
        if op.kind == O.GROUP:
            in_group.update(group_members(plan, k))
    units = [k for k, op in enumerate(plan.ops) if k not in in_group and op.kind not in (O.FORK, O.JOIN, O.WAIT)]
    OP_DUMP[model] = [{"name": op.name, "family": op_work(op)[0] if op.kind != O.GROUP else "group",
                       "ms": round(t, 5), "flops": op_work(op)[1], "bytes": op_work(op)[2],
                       "in_group": k in in_group,
                       "tile": conv_tile(plan.records[k:k + 1]) if op.kind == O.CONV else None}
                      for k, (op, t) in enumerate(zip(plan.ops, times))]
    fam = {}
    for k in units:
        name = unit_work(plan, k)[0]
        fam[name] = fam.get(name, 0.0) + times[k]
    dom = max(fam, key=fam.get)
    # the family's largest launch by algorithmic work (first in plan order among equal shapes, so
    # the choice does not flip between identical layers from run to run and the committed PMC
    # summary of the same launch applies); its measured time prices it
    k = max((j for j in units if unit_work(plan, j)[0] == dom), key=lambda j: (unit_work(plan, j)[1], unit_work(plan, j)[2]))
    op, t = plan.ops[k], times[k]
    name, flops, byts = unit_work(plan, k)
    kname, peak_tf = {"dwconv": "dwconv_kernel"}.get(name, name), FP32_MFMA_PEAK_TFS
    grouped = op.kind == O.GROUP
    if name == "conv":
        if grouped:
            wg, peak_tf = 0, FP32_MFMA_PEAK_TFS
            for j in group_members(plan, k):
                kn, w_, nt, peak_tf = conv_grid(plan.ops[j], plan.records[j:j + 1])
                wg += w_
            kname = kn.replace("conv_x6b_kernel", "conv_x6b_group_kernel")
        else:
            kname, wg, nt, peak_tf = conv_grid(op, plan.records[k:k + 1])
    t_f = flops / (peak_tf * 1e12)
    t_b = byts / (HBM_PEAK_GBS * 1e9)
    out = {"kernel": kname, "launch": op.name, "members": len(group_members(plan, k)) if grouped else 1,
           "launch_ms": round(t, 4), "algorithmic_flops": flops, "algorithmic_bytes": byts,
           "family_ms": {f: round(v, 4) for f, v in sorted(fam.items(), key=lambda kv: -kv[1])},
           "sum_ops_ms": round(sum(times), 3), "step_ms": round(step_ms, 3), "launches": launch_count(plan)}
    if name == "conv":
        out["grid_wg"], out["wg_threads"] = wg, nt
        if kname.startswith("conv_x6"):
            out["peak_basis"] = "dense bf16 MFMA 2516.6 TFLOP/s / 6 bf16 products per fp32 product"
    if t_f >= t_b:
        ach = flops / (t * 1e-3) / 1e12
        out.update({"bound": "mfma", "achieved": round(ach, 2), "peak": round(peak_tf, 1), "unit": "TFLOP/s",
                    "frac": round(ach / peak_tf, 4)})
    else:
        ach = byts / (t * 1e-3) / 1e9
        out.update({"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4)})
    out["traffic"] = None
    out["record"] = k
    return out


def attach_pipeline(roof, instances, steps):
    """The roofline launch timed in the running pipeline (pipeline_launch_ms): `launch_ms`, `achieved`
    and `frac` become the in-pipeline figures (the kernel-trace average of the same launch is what
    they are checked against, profiles/); the solo figures stay beside them as *_solo."""
    res = pipeline_launch_ms(instances, roof["record"], steps)
    if res is None:
        roof["frac_in_pipeline"] = None
        return
    ms, nlaunch, ips = res
    work = roof["algorithmic_flops"] if roof["bound"] == "mfma" else roof["algorithmic_bytes"]
    scale = 1e12 if roof["bound"] == "mfma" else 1e9
    roof["launch_ms_solo"], roof["achieved_solo"], roof["frac_solo"] = roof["launch_ms"], roof["achieved"], roof["frac"]
    ach = work / (ms * 1e-3) / scale
    roof.update({"launch_ms": round(ms, 4), "achieved": round(ach, 2), "frac": round(ach / roof["peak"], 4),
                 "frac_in_pipeline": round(ach / roof["peak"], 4),
                 "contention": "inclusive: launch_ms / achieved / frac are the launch's span inside the running "
                               "pipeline, CU time held by the other chains' kernels included (what the kernel "
                               "trace of the pipeline averages); the kernel alone against its roof is *_solo",
                 "timing": f"workgroup 0's start to the last workgroup's end on the GPU's 100 MHz clock, written by "
                           f"the kernel into a probe slot, {nlaunch} launches over {steps} pipelined passes of "
                           f"{len(instances)} instances ({ips:.1f} img/s with the probes); *_solo: the launch "
                           f"alone, HIP events around 20 back-to-back replays",
                 "stretch_vs_solo": round(ms / roof["launch_ms_solo"], 3)})


def _probe_records(recs, k, slot_ptr):
    """The plan's records with the launch at record k (a GROUP record: its members, the one grouped
    launch) carrying a timing-probe slot (CONV p9, csrc/kernels.hpp ConvParams::stamp); nothing else
    changes (no extra record: the slot needs no reset between launches)."""
    from edgeml_amd import ops as O
    end = k + 1 + (int(recs[k]["i"][0]) if recs[k]["kind"] == O.GROUP else 0)
    out = np.ascontiguousarray(recs.copy())
    for r in out[k:end]:
        if r["kind"] == O.CONV:
            r["p"][9] = slot_ptr
    return out


def pipeline_launch_ms(instances, k, steps):
    """Average duration (ms) of the launch at record k in the RUNNING pipeline.  Every instance's plan is
    captured again with a timing-probe slot on that launch (_probe_records; the same records otherwise)
    and primed like plan.capture; the bf16x6 kernels write workgroup 0's start and the last workgroup's
    end on the GPU's 100 MHz constant clock into the slot (s_memrealtime, vector atomics), and a 16-byte
    D2H copy after each pass's detections brings it to pinned host memory (two host buffers per
    instance, alternating, so a buffer is read after the ring has waited for its pass, two cycles
    back).  Settle and passes are issued exactly as timed_steps issues them (round robin, at most 2n
    outstanding, completion event after each pass's D2H).  The span includes the time the launch's
    workgroups wait for CU slots held by the kernels of the other chains / instances running beside
    it: what a kernel trace of the pipeline shows, and what the solo timing of per_op_times leaves
    out.  (HIP events recorded inside a captured graph do not time: hipEventElapsedTime refuses them
    on this ROCm.)  Returns (mean ms, launches timed, img/s of these passes), or None when the
    launch's kernel does not write the probe (only the bf16x6 conv tiles do)."""
    import ctypes
    from edgeml_amd import ops as O
    L = O.lib()
    n = len(instances)
    slots = []
    for p, s in instances:
        dev = torch.zeros(2, dtype=torch.int64, device="cuda")
        host = torch.zeros((2, 2), dtype=torch.int64, pin_memory=True)
        recs = _probe_records(p.records, k, dev.data_ptr())
        g = ctypes.c_void_p()
        O.check(L.edgedet_graph_create(recs.ctypes.data_as(ctypes.c_void_p), len(recs), O.stream_handle(s),
                                       ctypes.byref(g)))
        for _ in range(2):  # prime, as plan.capture does
            O.check(L.edgedet_graph_launch(g, O.stream_handle(s)))
        slots.append((p, s, d2h_buffers(p), g, dev, host, [None, None]))
    torch.cuda.synchronize()
    ring, ticks = [], []

    def read(host, v):
        st, en = int(host[v, 0]), int(host[v, 1])
        return en - st if st and en > st else None

    def issue(j, keep):
        while len(ring) >= 2 * n:
            ring.pop(0).synchronize()
        p, s, d2h, g, dev, host, used = slots[j % n]
        v = (j // n) % 2
        if used[v] is True:  # this buffer's pass (2n passes back) has completed and was a timed one
            ticks.append(read(host, v))
        O.check(L.edgedet_graph_launch(g, O.stream_handle(s)))
        with torch.cuda.stream(s):
            for d, h in d2h:
                h.copy_(d, non_blocking=True)
            host[v].copy_(dev, non_blocking=True)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(s)
        ring.append(ev)
        used[v] = keep  # readings of settle passes are never averaged
        return ev
    t0, j = time.perf_counter(), 0
    while time.perf_counter() - t0 < SETTLE_S or j < 4 * n:  # settle, as timed_steps
        issue(j, False)
        j += 1
    first = issue(j, True)
    for j2 in range(j + 1, j + 1 + steps):
        last = issue(j2, True)
    torch.cuda.synchronize()
    for _, _, _, _, _, host, used in slots:
        for v in range(2):
            if used[v] is True:
                ticks.append(read(host, v))
    ips = steps * instances[0][0].B / (first.elapsed_time(last) / 1e3)
    for sl in slots:
        L.edgedet_graph_destroy(sl[3])
    if not ticks or any(t is None for t in ticks):
        return None
    return float(np.mean(ticks)) * 1e-5, len(ticks), ips  # 100 MHz ticks -> ms


def launch_count(plan):
    """Kernel launches per forward: every record but FORK / JOIN / WAIT, a GROUP's members as one
    (records that issue two kernels -- the SSD post-process (class selection + image NMS), the
    chunked RPN filter, an SE excitation wider than the fused kernel takes, a pre-split conv -- counted
    as two)."""
    from edgeml_amd import ops as O
    n, k = 0, 0
    while k < len(plan.ops):
        op = plan.ops[k]
        if op.kind == O.GROUP:
            n += 1
            k += 1 + int(op.i[0])
            continue
        if op.kind in (O.FORK, O.JOIN, O.WAIT):
            pass
        elif op.kind == O.SSD_POSTPROCESS:
            n += 2
        elif op.kind == O.RPN_LEVEL_NMS:
            n += 2 if op.p.get(20) is not None else 1  # chunked top-k: chunk select + level kernel
        elif op.kind == O.SE_FC:
            n += 1 if op.i[1] * op.i[2] <= 8192 else 2
        elif op.kind == O.CONV and op.p.get(8) is not None and conv_tile(plan.records[k:k + 1]) == 25:
            n += 2
        else:
            n += 1
        k += 1
    return {"records": len(plan.ops), "kernel_launches": n}


def attach_traffic(roof, model):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_<model>.json, produced by tools/pmc_summary.py from separate FETCH_SIZE and
    WRITE_SIZE passes, gfx950 FETCH_SIZE x2 correction applied there); None if absent or stale."""
    path = os.path.join(ROOT, "profiles", f"pmc_{model}.json")
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return
    # "#k" names the k-th batch chain's copy of a layer: the chains split the batch evenly, so
    # every copy has the same shape and grid and one PMC summary covers them all
    same = lambda a: (a or "").split("#")[0]
    kernel_ok = not (pmc.get("kernel") and roof.get("kernel")) or pmc["kernel"] == roof["kernel"]
    if same(pmc.get("launch")) == same(roof.get("launch")) and pmc.get("grid_wg") == roof.get("grid_wg") and kernel_ok:
        roof["traffic"] = pmc.get("hbm_bytes_per_launch")
        roof["traffic_source"] = os.path.relpath(path, ROOT)


# ------------------------------------------------------------------------------ CPU baseline
def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


G5 = os.path.join(ROOT, "tests", "golden", "g5_orie_f64.npz")  # float64 ground truth (make_orie_f64.py)


def _f64_truth(n):
    """The float64 detector files of G5 for the leg's n images ({"weak"/"strong": [rows]}) and the
    per-image input checksums they were made from; None if absent or too short."""
    try:
        z = np.load(G5)
    except OSError:
        return None
    if len(z["image_sums"]) < n:
        return None
    out = {"sums": z["image_sums"][:n]}
    for tag in ("weak", "strong"):
        cnt = z[tag + "_f64_count"]
        off = np.concatenate([[0], np.cumsum(cnt)])
        out[tag] = [z[tag + "_f64_rows"][off[i]:off[i + 1]] for i in range(n)]
    return out


def orie_vs_ref(n=48, E=None):
    """ORIE of the engine's files vs ORIE of the CPU oracle's files on n synthetic 640x640 images
    (SSDLite weak, FRCNN strong), E = n - 1 so every image is in every ensemble, as in config 4
    (E = 1000 over 5,000).  Three sets of detect.py files for the same images:
      engine    the HIP engine (batch=1 per image), through the product consumer (GPU reward) for
                the metric's ORIE max-abs-diff;
      oracle    the CPU oracle in float32 (its batch=1 forwards are timed on the way: they are the
                FRCNN cpu_baseline), through the oracle consumer (pinned to the reference's G2);
      f64       the same oracle with every conv / linear / BN / activation in float64 and the head
                outputs rounded to float32 before the reference's float32 post-processing
                (tests/golden/g5_orie_f64.npz, made by tests/golden/make_orie_f64.py from the same
                seeded inputs; the input checksums are verified here): the exact-arithmetic detector
                both float32 implementations approximate.
    Pseudo ground truth for all three = the f64 strong detector's confident boxes (conf >= 0.3).
    Reported: max |ORIE(engine) - ORIE(oracle)| (the metric); ORIE(engine) - ORIE(f64) beside
    ORIE(oracle) - ORIE(f64), all three through the oracle consumer; and identity-paired file
    differences (tools/rowpair.py: rows paired by class and IoU >= 0.99, paired |dconf| / |dbox|,
    unpaired counts) for each pair of sets and detector."""
    import tempfile
    import warnings
    from edgeml_amd import fmt, models, reward, synthetic
    from oracle import orie
    from oracle.frcnn import FasterRCNNOracle
    from oracle.ssdlite import SSDLiteOracle
    from edgeml_amd.distributed import usable_cpus
    from tools import rowpair
    warnings.filterwarnings("ignore")
    torch.set_num_threads(usable_cpus())
    E = n - 1 if E is None else E
    cpu_s = {"weak": 0.0, "strong": 0.0}
    truth = _f64_truth(n)
    sd_w, sd_s = synthetic.synthetic_state_dict("ssd", 91, True), synthetic.synthetic_state_dict("faster_rcnn", 91)
    eng = {"weak": models.SSDLite320(sd_w, 91, True).to("cuda"), "strong": models.FasterRCNNFPNv2(sd_s, 91).to("cuda")}
    ref = {"weak": SSDLiteOracle(sd_w, 91, True), "strong": FasterRCNNOracle(sd_s, 91)}
    sets = ("eng", "ref", "f64")
    with tempfile.TemporaryDirectory() as td:
        d = lambda *p: os.path.join(td, *p)  # noqa: E731
        for sub in [s_ + "_" + t for s_ in sets for t in ("weak", "strong")] + ["labels"]:
            os.makedirs(d(sub))
        for i in range(n):
            img = synthetic.make_batch(1, 640, 640, seed=7000 + i)
            if truth is not None and float(img.double().sum()) != float(truth["sums"][i]):
                truth = None  # regenerated inputs differ from G5's: no f64 leg
            name = f"{i:012d}.png"
            for tag in ("weak", "strong"):
                p = eng[tag](img.cuda())[0]
                fmt.save_npy(d("eng_" + tag), name, fmt.format_detections(
                    p["boxes"].cpu().numpy(), p["scores"].cpu().numpy(), p["labels"].cpu().numpy(), 640, 640))
                t0 = time.perf_counter()
                q = ref[tag]([img[0]])[0]
                if i:  # image 0 warms the oracle up
                    cpu_s[tag] += time.perf_counter() - t0
                rows = fmt.format_detections(q["boxes"].numpy(), q["scores"].numpy(), q["labels"].numpy(), 640, 640)
                fmt.save_npy(d("ref_" + tag), name, rows)
        have_f64 = truth is not None
        for i in range(n):
            name = f"{i:012d}.png"
            if have_f64:
                for tag in ("weak", "strong"):
                    fmt.save_npy(d("f64_" + tag), name, truth[tag][i])
            src = truth["strong"][i] if have_f64 else np.load(d("ref_strong", name[:-4] + ".npy"))
            with open(d("labels", name[:-4] + ".txt"), "w") as f:
                for r in src[src[:, 5] >= 0.3]:
                    f.write(" ".join([str(int(r[0]))] + [repr(float(v)) for v in r[1:5]]) + "\n")
        names = [f"{i:012d}" for i in range(n)]
        load = lambda side, tag: (lambda nm: np.load(d(side + "_" + tag, nm + ".npy")))  # noqa: E731
        files = {}
        for a_, b_ in (("eng", "ref"), ("eng", "f64"), ("ref", "f64")):
            if "f64" in (a_, b_) and not have_f64:
                continue
            files[f"{a_}_vs_{b_}"] = {tag: rowpair.compare_dirs(names, load(a_, tag), load(b_, tag))
                                      for tag in ("weak", "strong")}
        wd, sd, lab = reward.set_data(d("eng_weak"), d("eng_strong"), d("labels"))
        got = reward.compute_orie_all(wd, sd, lab, E, seed=1000)  # engine files, product (GPU) consumer
        cons = {s_: orie.orie_all(d(s_ + "_weak"), d(s_ + "_strong"), d("labels"), E, seed=1000)
                for s_ in sets if s_ != "f64" or have_f64}  # every set through the oracle consumer
    want = cons["ref"]
    dd = np.abs(got - want)
    out = {"max_abs_diff": float(dd.max()), "images": n, "num_ensemble": E,
           "images_differing": int(np.count_nonzero(dd)), "nonzero_ref": int(np.count_nonzero(want)),
           "consumer_check_max_abs": float(np.abs(got - cons["eng"]).max()),
           "files_paired": files}
    if have_f64:
        t = cons["f64"]
        de, do = np.abs(cons["eng"] - t), np.abs(cons["ref"] - t)
        out["vs_f64"] = {"engine_max_abs": float(de.max()), "oracle_f32_max_abs": float(do.max()),
                         "engine_images_differing": int(np.count_nonzero(de)),
                         "oracle_f32_images_differing": int(np.count_nonzero(do)),
                         "engine_mean_abs": float(de.mean()), "oracle_f32_mean_abs": float(do.mean()),
                         "truth": "tests/golden/g5_orie_f64.npz (oracle forward in float64, heads rounded to "
                                  "float32, float32 post-processing)"}
    else:
        out["vs_f64"] = None
    frcnn_cpu = {"value": round((n - 1) / cpu_s["strong"], 3), "unit": "images/s", "cores": torch.get_num_threads(),
                 "kind": "port", "host_cores": os.cpu_count(), "host_cpu": _cpu_model(),
                 "sample": f"{n - 1} synthetic 640x640 images, batch=1 ({cpu_s['strong']:.1f}s), frcnn CPU oracle "
                           f"(PyTorch-CPU + C restatement of the torchvision eval path), the orie leg's strong pass"}
    return out, frcnn_cpu


def cpu_baseline(kind, budget_s=15.0):
    """The CPU oracle (restated reference path) on a bounded sample, batch=1 like detect.py."""
    from edgeml_amd import synthetic
    from oracle.frcnn import FasterRCNNOracle
    from oracle.ssdlite import SSDLiteOracle
    from edgeml_amd.distributed import usable_cpus
    torch.set_num_threads(usable_cpus())
    if kind == "ssd":
        m = SSDLiteOracle(synthetic.synthetic_state_dict("ssd", 91, True), 91, True)
    else:
        m = FasterRCNNOracle(synthetic.synthetic_state_dict("faster_rcnn", 91), 91)
    n, t0 = 0, time.perf_counter()
    m(list(synthetic.make_batch(1, 640, 640, seed=999)))  # warm-up
    t0 = time.perf_counter()
    while True:
        m(list(synthetic.make_batch(1, 640, 640, seed=1000 + n)))
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 200:
            break
    return {"value": round(n / el, 3), "unit": "images/s", "cores": torch.get_num_threads(), "kind": "port",
            "host_cores": os.cpu_count(), "host_cpu": _cpu_model(),
            "sample": f"{n} synthetic 640x640 images, batch=1 ({el:.1f}s), {kind} CPU oracle "
                      f"(PyTorch-CPU + C restatement of the torchvision eval path)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=750)  # about 1 s of timed SSD work
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="both", choices=["ssd", "frcnn", "retinanet", "both", "all"])
    ap.add_argument("--retina-batch", type=int, default=8)
    ap.add_argument("--ssd-batch", type=int, default=32)
    ap.add_argument("--frcnn-batch", type=int, default=8)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--inflight", type=int, default=0,
                    help="independent plan instances the steps rotate over (batches in flight per GPU); "
                         "0 = the model's INFLIGHT, the count the detect CLI's run_batches keeps in flight")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-alt", action="store_true", help="skip the SSD rate at the other in-flight count")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--dump-ops", default="", help="write the per-op device times of each model to this JSON")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host uint8 -> rows) rates")
    ap.add_argument("--diagnostic", action="store_true",
                    help="allow EDGEDET_DIAG_SKIP (diagnostic builds only); the line is marked and is not a result")
    ap.add_argument("--e2e-batches", type=int, default=40)
    ap.add_argument("--input", default="u8", choices=["u8", "f32"],
                    help="what the step's input batch in HBM holds: the decoded uint8 images (the detect CLI's "
                         "engine input; /255 in the device transform, bit-identical to the host's float path) "
                         "or the model contract's float images")
    args = ap.parse_args()
    u8 = args.input == "u8"
    # EDGEDET_DIAG_SKIP (honoured only by a -DEDGEDET_DIAG build, libedgedet_diag.so) leaves op families
    # out: wrong results, so a measurement under it is never a product number
    if os.environ.get("EDGEDET_DIAG_SKIP") and not args.diagnostic:
        sys.exit("bench.py: EDGEDET_DIAG_SKIP is set (a diagnostic that skips work, wrong results); "
                 "refusing to measure without --diagnostic")

    dist, rank, world = dist_setup(args.gpus)
    from edgeml_amd import models, synthetic
    from edgeml_amd import plan as plan_mod
    out = {}
    if args.model in ("ssd", "both", "all"):
        B = args.ssd_batch
        # fresh streams per model, created together with the other instances' (inflight_instances):
        # consecutive streams land on distinct hardware queues; instances of a model placed on streams
        # that share a queue are serialised against each other (an FRCNN run after the SSD one had two
        # of its three instances on one queue: profiles/r4d_trace_both.jsonl)
        stream = torch.cuda.Stream()
        m = models.ssdlite320_mobilenet_v3_large().to("cuda")
        plan = m.plan(B, 640, 640, u8)
        fill_input(plan, B, 100 * rank)
        plan.capture(stream)
        nin = args.inflight or m.INFLIGHT
        extra = inflight_instances(m, B, nin, 100 * rank, u8)
        el = timed_steps(plan, stream, args.steps, args.warmup, dist, extra)
        out["ssd"] = {"value": world * B * args.steps / el, "ms_per_step": 1e3 * el / args.steps, "batch": B,
                      "inflight": nin, "dets_per_img": float(plan.out_count.tensor().float().mean().item()),
                      "timing": dict(TIMING)}
        if rank == 0 and not args.no_roofline:
            out["ssd"]["roofline"] = roofline_for(plan, stream, 1e3 * el / args.steps, "ssd")
            attach_pipeline(out["ssd"]["roofline"], [(plan, stream)] + extra, max(args.steps, 40 * nin))
            attach_traffic(out["ssd"]["roofline"], "ssd")
        # SURVEY §8(d)'s binding roof for C2: 87.1 MB of algorithmic HBM traffic per image with the fp32
        # input image (4.92 MB); a uint8 input batch reads 1.23 MB of it instead
        bpi = SSD_BYTES_PER_IMG - (3 * 640 * 640 * 3 if u8 else 0)
        gbs = bpi * out["ssd"]["value"] / world / 1e9
        out["ssd"]["step_hbm"] = {"bytes_per_img": bpi, "achieved_GBps": round(gbs, 1),
                                  "peak_GBps": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4)}
        if not args.no_alt:  # the other in-flight count, same plans (reported beside the headline)
            alt = 2 if nin != 2 else 4
            more = inflight_instances(m, B, alt - nin + 1, 100 * rank + 7, u8) if alt > nin else []
            el2 = timed_steps(plan, stream, args.steps, args.warmup, dist, (extra + more)[:alt - 1])
            del more
            out["ssd"]["alt_inflight"] = {"inflight": alt, "value": round(world * B * args.steps / el2, 2)}
        del extra
        del plan
        m.plans.clear()
        if rank == 0 and not args.no_e2e:
            out["ssd"]["end_to_end"] = end_to_end(m, B, args.e2e_batches, 100 * rank)
            m.plans.clear()
            m._slots.clear()
    if args.model in ("retinanet", "all"):
        B = args.retina_batch
        # fresh streams per model, created together with the other instances' (inflight_instances):
        # consecutive streams land on distinct hardware queues; instances of a model placed on streams
        # that share a queue are serialised against each other (an FRCNN run after the SSD one had two
        # of its three instances on one queue: profiles/r4d_trace_both.jsonl)
        stream = torch.cuda.Stream()
        m = models.retinanet_resnet50_fpn_v2().to("cuda")
        plan = m.plan(B, 640, 640, u8)
        fill_input(plan, B, 100 * rank + 70)
        plan.capture(stream)
        steps = max(20, args.steps // 10)
        extra = inflight_instances(m, B, args.inflight or m.INFLIGHT, 100 * rank + 70, u8)
        el = timed_steps(plan, stream, steps, max(2, args.warmup // 4), dist, extra)
        out["retinanet"] = {"value": world * B * steps / el, "ms_per_step": 1e3 * el / steps, "batch": B,
                            "dets_per_img": float(plan.out_count.tensor().float().mean().item())}
        if rank == 0 and not args.no_roofline:
            out["retinanet"]["roofline"] = roofline_for(plan, stream, 1e3 * el / steps, "retinanet")
            attach_pipeline(out["retinanet"]["roofline"], [(plan, stream)] + extra, max(steps, 8 * len(extra) + 8))
        del extra
        del plan
    if args.model in ("frcnn", "both", "all"):
        B = args.frcnn_batch
        # fresh streams per model, created together with the other instances' (inflight_instances):
        # consecutive streams land on distinct hardware queues; instances of a model placed on streams
        # that share a queue are serialised against each other (an FRCNN run after the SSD one had two
        # of its three instances on one queue: profiles/r4d_trace_both.jsonl)
        stream = torch.cuda.Stream()
        m = models.fasterrcnn_resnet50_fpn_v2().to("cuda")
        plan = m.plan(B, 640, 640, u8)
        fill_input(plan, B, 100 * rank + 50)
        plan.capture(stream)
        extra = inflight_instances(m, B, args.inflight or m.INFLIGHT, 100 * rank + 50, u8)
        steps = max(20, args.steps // 10)  # FRCNN steps are ~20x SSD's: at least 20 (about half a second)
        el = timed_steps(plan, stream, steps, max(2, args.warmup // 4), dist, extra)
        timing = dict(TIMING)
        R = float(plan.proposal_count.tensor().float().mean().item())
        gflop = 2 * (151.45e9 + 128.92e6 * R) / 1e9
        out["frcnn"] = {"value": world * B * steps / el, "ms_per_step": 1e3 * el / steps, "batch": B,
                        "proposals_per_img": R, "dets_per_img": float(plan.out_count.tensor().float().mean().item()),
                        "tflops_model": round(gflop * B * steps / el / 1e3 / world, 2), "timing": timing}
        if rank == 0 and not args.no_roofline:
            out["frcnn"]["roofline"] = roofline_for(plan, stream, 1e3 * el / steps, "frcnn")
            attach_pipeline(out["frcnn"]["roofline"], [(plan, stream)] + extra, max(steps, 8 * len(extra) + 8))
            attach_traffic(out["frcnn"]["roofline"], "frcnn")
        del extra
        del plan
        m.plans.clear()
        if rank == 0 and not args.no_e2e:
            out["frcnn"]["end_to_end"] = end_to_end(m, B, max(4, args.e2e_batches // 4), 100 * rank + 50)
            m.plans.clear()
            m._slots.clear()
    if rank == 0 and args.dump_ops:
        with open(args.dump_ops, "w") as f:
            json.dump(OP_DUMP, f, indent=0)
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    primary = "ssd" if "ssd" in out else ("frcnn" if "frcnn" in out else "retinanet")
    p = out[primary]
    line = {
        "metric": "images/sec/GPU at 640x640 (SSDLite & FRCNN-R50); ORIE max-abs-diff vs ref",
        "value": round(p["value"], 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(p["ms_per_step"], 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": {"ssd": "ssdlite320_mobilenet_v3_large b=%d 640x640 (configs[1])",
                                "frcnn": "fasterrcnn_resnet50_fpn_v2 b=%d 640x640 (configs[2])",
                                "retinanet": "retinanet_resnet50_fpn_v2 b=%d 640x640"}[primary] % p["batch"],
                   "global_batch": p["batch"] * world, "parallelism": f"dp{world}",
                   "batches_in_flight": p.get("inflight", args.inflight),
                   "input": ("uint8 decoded images in HBM (read_image, detect.py:57); /255 in the device transform"
                             if u8 else "float32 images in HBM (the model contract, detect.py:58)"),
                   "conv_math": plan_mod.CONV_MATH,
                   "weights": "seeded synthetic (COCO weights need a download)"},
    }
    if "frcnn" in out and primary == "ssd":
        f = out["frcnn"]
        line["frcnn"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in f.items()
                         if k not in ("roofline", "end_to_end")}
        if "end_to_end" in f:
            line["frcnn"]["end_to_end"] = f["end_to_end"]
        if "roofline" in f:
            line["frcnn"]["roofline"] = f["roofline"]
    if "retinanet" in out and primary != "retinanet":
        f = out["retinanet"]
        line["retinanet"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in f.items()}
    if "roofline" in p:
        line["roofline"] = p["roofline"]
    if os.environ.get("EDGEDET_DIAG_SKIP"):
        line["diagnostic"] = "EDGEDET_DIAG_SKIP=%s: op families skipped, NOT a result" % os.environ["EDGEDET_DIAG_SKIP"]
    line["dets_per_img"] = p.get("dets_per_img")
    if "end_to_end" in p:
        line["end_to_end"] = p["end_to_end"]
    for k in ("step_hbm", "alt_inflight", "timing"):
        if k in p:
            line[k] = p[k]
    if not args.no_cpu:
        line["orie"], frcnn_cpu = orie_vs_ref()
        line["cpu_baseline"] = cpu_baseline(primary, args.cpu_budget)
        if "frcnn" in out and primary == "ssd":
            line["frcnn"]["cpu_baseline"] = frcnn_cpu
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
