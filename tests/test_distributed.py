"""World-size-2 gloo tests of the sharding and the output-row gather."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows_for(name):
    rs = np.random.RandomState(int(name) % 97)
    n = int(name) % 4  # includes empty (0,6) outputs
    return rs.rand(n, 6)


def _worker(rank, world, port, names, q, batched=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from edgeml_amd import distributed as D
    shards = None
    if batched:  # the detect CLI's batch-granular shards: two sizes, batches of 3
        sizes = [(480, 640) if int(n) % 3 else (427, 640) for n in names]
        chunks = D.size_batches(sizes, 3)
        shards = [[names[i] for c in D.batch_shard(chunks, r, world) for i in c] for r in range(world)]
        mine = shards[rank]
    else:
        mine = D.shard(names, rank, world)
    res = {n: _rows_for(n) for n in mine}
    out = D.gather_rows(res, mine, names, rank, world, shards=shards)
    if rank == 0:
        q.put({k: v.tolist() for k, v in out.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_shard_is_contiguous_partition():
    from edgeml_amd import distributed as D
    names = [f"{i:012d}.jpg" for i in range(103)]
    for world in (1, 2, 3, 8):
        parts = [D.shard(names, r, world) for r in range(world)]
        assert sum(parts, []) == names
        assert max(map(len, parts)) - min(map(len, parts)) <= 1


def test_size_batches_and_batch_shard():
    """Batch-granular shards: every rank's batches are the world-1 batches, unchanged, in a
    contiguous block of the world-1 order, balanced by image count."""
    from edgeml_amd import distributed as D
    rs = np.random.RandomState(0)
    pool = [(480, 640), (640, 480), (427, 640), (612, 612)]
    for n, batch in ((103, 8), (5000, 32), (7, 32), (40, 1), (0, 4)):
        sizes = [pool[k] for k in rs.randint(0, 4, n)]
        chunks = D.size_batches(sizes, batch)
        assert sorted(i for c in chunks for i in c) == list(range(n))
        for c in chunks:
            assert len(c) <= batch and len({sizes[i] for i in c}) == 1 and c == sorted(c)
        for world in (1, 2, 3, 8):
            parts = [D.batch_shard(chunks, r, world) for r in range(world)]
            assert sum(parts, []) == chunks  # contiguous blocks, world-1 order, batches unchanged
            if n >= world * batch * 4:
                load = [sum(map(len, p)) for p in parts]
                assert max(load) - min(load) <= 2 * batch


def test_batch_shard_balances_frcnn_work_on_coco_sizes():
    """A 5,000-image COCO-size list at world 8 with the FRCNN batches of the detect CLI: balanced by
    the model's batch work (batch x resized padded pixels, models.FasterRCNNFPNv2.batch_work), every
    rank's work is within one batch of the ideal share; the world-1 batches are unchanged and the
    blocks contiguous.  Balancing by image count instead leaves a larger spread on the same list."""
    from edgeml_amd import distributed as D
    from edgeml_amd.models import FasterRCNNFPNv2
    m = object.__new__(FasterRCNNFPNv2)  # batch_work needs only the class's transform constants
    rs = np.random.RandomState(1)
    # COCO val2017's common shapes (640 on the long side, portrait and landscape), mixed by frequency
    pool = [(480, 640), (427, 640), (640, 480), (425, 640), (640, 427), (424, 640), (428, 640),
            (612, 612), (500, 375), (375, 500), (333, 500), (640, 640), (360, 640), (640, 360)]
    p = np.array([20, 14, 9, 8, 6, 5, 5, 3, 3, 3, 3, 3, 2, 2], float)
    sizes = [pool[k] for k in rs.choice(len(pool), 5000, p=p / p.sum())]
    batch, world = m.max_batch, 8
    chunks = D.size_batches(sizes, batch)
    work = lambda c: m.batch_work(len(c), *sizes[c[0]])  # noqa: E731
    parts = [D.batch_shard(chunks, r, world, work) for r in range(world)]
    assert sum(parts, []) == chunks
    load = [sum(work(c) for c in part) for part in parts]
    ideal, wmax = sum(load) / world, max(work(c) for c in chunks)
    assert all(abs(x - ideal) <= wmax for x in load), (load, ideal, wmax)
    by_count = [sum(work(c) for c in D.batch_shard(chunks, r, world)) for r in range(world)]
    assert max(load) - min(load) <= max(by_count) - min(by_count)


@pytest.mark.parametrize("n,batched", [(7, False), (1, False), (11, True)])
def test_gather_rows_world2(n, batched):
    names = [f"{i:06d}" for i in range(n)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, names, q, batched)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(got) == names
    for k in names:
        np.testing.assert_array_equal(np.asarray(got[k]).reshape(-1, 6), _rows_for(k))


def _values_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from edgeml_amd import distributed as D
    mine = D.shard(list(range(n)), rank, world)
    out = D.gather_values(np.asarray(mine, np.float64) * 1.5, mine, n, rank, world)
    if rank == 0:
        q.put(out.tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [0, 1, 7])
def test_gather_values_world2(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_values_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert got == [1.5 * i for i in range(n)]


def _init_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), EDGEDET_DIST_BACKEND="gloo")
    from edgeml_amd import distributed as D
    r, w = D.ensure_initialized()
    r2, w2 = D.ensure_initialized()  # idempotent
    out = D.gather_values(np.asarray([10.0 * r]), [r], world, r, w)
    if r == 0:
        q.put((r, w, r2, w2, dist.get_backend(), out.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_ensure_initialized_joins_torchrun_group():
    """The CLIs (detect.main, reward.main, pipeline.main) join the group torchrun's environment
    describes; gloo when no GPU is visible."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_init_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == (0, 2, 0, 2, "gloo", [0.0, 10.0])


def test_ensure_initialized_single_process_is_noop(monkeypatch):
    from edgeml_amd import distributed as D
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert D.ensure_initialized() == (0, 1)
    assert not dist.is_initialized()
