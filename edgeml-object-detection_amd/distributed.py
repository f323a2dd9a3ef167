"""One process per GPU: contiguous shards of the sorted image list and a gather of the output rows.

SURVEY.md §8e: images are independent, so the ranks split sorted(os.listdir(img_dir)) (detect.py:64)
with no collective on the data path.  The detect CLI shards at BATCH granularity: every rank forms
the single-process run's list of size-grouped batches (size_batches) and takes a contiguous block of
it (batch_shard), so each image runs in exactly the batch it would run in on one GPU and its output
bits do not depend on the GPU count (the conv tile table is keyed on the batch size).  The reward CLI
shards target images as contiguous blocks (shard).  The only exchange is the final gather of the per-image (n_i, 6) float64 rows to rank 0,
which writes every file (single writer): an all_gather of per-rank row counts, then an all_gather of
the packed rows padded to the largest rank (``torch.distributed``; backend "nccl" = RCCL over xGMI on
the MI355X node, "gloo" in the CPU tests).
"""
import os

import numpy as np
import torch
import torch.distributed as dist


def ensure_initialized():
    """Join the process group torchrun describes (WORLD_SIZE > 1 in the environment), once.

    Backend: "nccl" (RCCL over xGMI) when a GPU is visible, "gloo" otherwise; EDGEDET_DIST_BACKEND
    overrides (the multi-process GPU tests run two gloo ranks on one card).  With nccl each rank
    binds its LOCAL_RANK's device before the group is created.  Returns (rank, world)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and dist.is_available() and not dist.is_initialized():
        backend = os.environ.get("EDGEDET_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(device_index())
        dist.init_process_group(backend)
    return rank_world()


def device_index():
    """This rank's GPU: LOCAL_RANK, wrapped onto the visible devices (ranks may share a card)."""
    n = torch.cuda.device_count()
    return local_rank() % n if n else 0


def rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def usable_cpus():
    """CPU cores this process may actually use: the affinity mask, further limited by a cgroup v2
    CPU quota (cpu.max) when one is set.  os.cpu_count() reports the whole host, which on a shared
    GPU box is many times the share a job gets, so thread pools are sized by this instead."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def local_rank():
    return int(os.environ.get("LOCAL_RANK", 0))


def shard_bounds(n, rank, world):
    return rank * n // world, (rank + 1) * n // world


def shard(items, rank, world):
    lo, hi = shard_bounds(len(items), rank, world)
    return list(items)[lo:hi]


def size_batches(sizes, batch):
    """The single-process detect run's batches (detect.py:64-66 order, batched): images grouped by
    (H, W) in order of first appearance, each group cut into chunks of at most `batch` in sorted-name
    order.  sizes: [(H, W)] per image of the sorted list -> [[image index, ...], ...]."""
    groups = {}
    for i, hw in enumerate(sizes):
        groups.setdefault(tuple(hw), []).append(i)
    return [idx[k:k + batch] for idx in groups.values() for k in range(0, len(idx), batch)]


def batch_shard(chunks, rank, world, cost=None):
    """A contiguous block of the batch list for `rank`, balanced by work: batch j goes to rank
    floor((W_j + w_j / 2) * world / W), where w_j = cost(batch j), W_j = the cost of the batches before
    it and W the total (the batch's midpoint decides, so every rank's work is within one batch of
    W / world).  cost=None counts images; the detect CLI passes the model's per-batch work (FRCNN /
    RetinaNet: batch size x resized padded pixels, which vary up to 1.5x with the source size; SSDLite
    resizes everything to 320 x 320, so its work is the image count).  Every batch lands on exactly
    one rank, unchanged, so per-image results equal the world-1 run's bit for bit."""
    w = [float(cost(c) if cost is not None else len(c)) for c in chunks]
    total = sum(w)
    out, start = [], 0.0
    for c, wc in zip(chunks, w):
        r = int((start + 0.5 * wc) * world // total) if total > 0 else 0
        if min(world - 1, r) == rank:
            out.append(c)
        start += wc
    return out


def gather_rows(results, my_names, all_names, rank, world, device=None, shards=None):
    """results: {name: (n,6) float64} for this rank's shard -> {name: rows} for every image on rank 0.
    shards: the names of every rank's shard in its processing order (all ranks pass the same list);
    None means the contiguous blocks of `all_names` that shard() gives."""
    if world == 1:
        return results
    if not dist.is_initialized():
        raise RuntimeError("gather_rows needs an initialised torch.distributed process group")
    backend = dist.get_backend()
    dev = device or (torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu"))
    counts = np.asarray([results[n].shape[0] for n in my_names], dtype=np.int64)
    rows = np.concatenate([results[n].reshape(-1, 6) for n in my_names], 0) if my_names else np.zeros((0, 6))
    meta = torch.tensor([len(my_names), rows.shape[0]], dtype=torch.int64, device=dev)
    metas = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta)
    metas = [m.cpu().tolist() for m in metas]
    max_imgs = max(m[0] for m in metas)
    max_rows = max(m[1] for m in metas)
    c = torch.zeros(max(max_imgs, 1), dtype=torch.int64, device=dev)
    c[:len(counts)] = torch.from_numpy(counts).to(dev)
    r = torch.zeros((max(max_rows, 1), 6), dtype=torch.float64, device=dev)
    r[:rows.shape[0]] = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.float64)).to(dev)
    cs = [torch.zeros_like(c) for _ in range(world)]
    rs = [torch.zeros_like(r) for _ in range(world)]
    dist.all_gather(cs, c)
    dist.all_gather(rs, r)
    if rank != 0:
        return None
    out = {}
    for k in range(world):
        if shards is None:
            lo, hi = shard_bounds(len(all_names), k, world)
            names = all_names[lo:hi]
        else:
            names = shards[k]
        cnt = cs[k].cpu().numpy()[:len(names)]
        rr = rs[k].cpu().numpy()
        pos = 0
        for name, n in zip(names, cnt):
            out[name] = rr[pos:pos + n].copy().reshape(int(n), 6)
            pos += int(n)
    return out


def gather_values(vals, my_idx, n, rank, world, device=None):
    """Per-image float64 values of this rank's contiguous shard (my_idx) -> the full [n] array on rank 0
    (reward.py: every rank computes the ORIE of its shard of target images)."""
    if world == 1:
        return np.asarray(vals, np.float64)
    backend = dist.get_backend()
    dev = device or (torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu"))
    width = max(shard_bounds(n, k, world)[1] - shard_bounds(n, k, world)[0] for k in range(world))
    buf = torch.zeros(max(width, 1), dtype=torch.float64, device=dev)
    buf[:len(my_idx)] = torch.from_numpy(np.asarray(vals, np.float64)).to(dev)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    if rank != 0:
        return None
    out = np.zeros(n)
    for k in range(world):
        lo, hi = shard_bounds(n, k, world)
        out[lo:hi] = bufs[k].cpu().numpy()[:hi - lo]
    return out
