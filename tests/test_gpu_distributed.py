"""The multi-GPU entry points as torchrun runs them, on one card.

Two ranks started with torchrun's environment (WORLD_SIZE=2, RANK, LOCAL_RANK, MASTER_*) run the
real ``detect.main`` (SSDLite weak, FRCNN strong) and ``reward.main``: each rank detects its
contiguous shard of the sorted image list (detect.py:64), rank 0 gathers the rows and writes every
file, then each rank evaluates its block of target images and rank 0 gathers the ORIE values
(reward.py:78-92).  Both ranks share cuda:0 over the gloo backend (the box has one GPU; on an
8-GPU node the same code binds LOCAL_RANK's device and uses nccl = RCCL).  Every output file must
be byte-identical to a single-process run.  Per-image results depend on the batch an image runs
in (the conv tile choice is keyed on the batch size), so detect shards at batch granularity
(distributed.size_batches / batch_shard): each rank runs a contiguous block of exactly the batches
the single-process run forms.  The cases use the CLI's default --batch (SSD 32, FRCNN 8) on ragged,
mixed-size sets, plus a forced small batch that splits a size group across the ranks.
"""
import os
import socket
import tempfile
import warnings

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_cli(img, lab, work, E, batch):
    import torch.distributed as dist
    from edgeml_amd import detect, reward
    for stage, model in (("weak", "ssd"), ("strong", "faster_rcnn")):
        extra = ["--batch", str(batch)] if batch else []  # 0: the CLI default (model.max_batch)
        detect.main(detect.getargs([img, os.path.join(work, stage), "--model", model, *extra]))
        if dist.is_initialized():
            dist.barrier()  # rank 0 has written every file before any rank reads them
    reward.main(reward.getargs([os.path.join(work, "weak"), os.path.join(work, "strong"), lab,
                                os.path.join(work, "reward"), "--num-ensemble", str(E), "--seed", "7"]))


def _rank(rank, world, port, img, lab, work, E, batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), EDGEDET_DIST_BACKEND="gloo")
    warnings.filterwarnings("ignore")
    try:
        _run_cli(img, lab, work, E, batch)
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # report, then fail the rank
        q.put((rank, repr(e)))
        raise


@pytest.mark.parametrize("n,batch,sizes", [
    (13, 0, [(480, 640), (427, 640)]),     # default batch, two size groups of ragged length
    (21, 0, [(480, 640), (640, 640)]),     # default batch: FRCNN's 8 cuts each group into 8 + rest
    (9, 2, [(480, 640), (375, 500)]),      # small batches: a size group straddles the ranks
])
def test_detect_and_reward_world2_equal_world1(n, batch, sizes):
    from edgeml_amd import synthetic
    warnings.filterwarnings("ignore")
    E = 4
    with tempfile.TemporaryDirectory() as td:
        img, lab = os.path.join(td, "imgs"), os.path.join(td, "labels")
        synthetic.make_dataset(img, n, seed=5, label_dir=lab, sizes=sizes)
        one, two = os.path.join(td, "w1"), os.path.join(td, "w2")
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_rank, args=(r, 2, port, img, lab, two, E, batch, q)) for r in range(2)]
        for p in procs:
            p.start()
        status = dict(q.get(timeout=300) for _ in procs)
        for p in procs:
            p.join(timeout=120)
        assert status == {0: "ok", 1: "ok"}, status
        assert all(p.exitcode == 0 for p in procs)
        _run_cli(img, lab, one, E, batch)  # single process (no WORLD_SIZE in this environment)
        for stage in ("weak", "strong"):
            a, b = sorted(os.listdir(os.path.join(one, stage))), sorted(os.listdir(os.path.join(two, stage)))
            assert a == b == [f"{i:012d}.npy" for i in range(n)]
            for f in a:
                with open(os.path.join(one, stage, f), "rb") as x, open(os.path.join(two, stage, f), "rb") as y:
                    assert x.read() == y.read(), (stage, f)
        with np.load(os.path.join(one, "reward", f"orie{E}.npz")) as z1, \
                np.load(os.path.join(two, "reward", f"orie{E}.npz")) as z2:
            np.testing.assert_array_equal(z1["reward"], z2["reward"])
            assert z1["reward"].shape == (n,)
