"""BASELINE configs[3] beyond a miniature: the config-4 pipeline as torchrun runs it.

100 synthetic COCO-size JPEGs (the four COCO sizes of synthetic.COCO_SIZES, the tools/config4_full.py
recipe at JPEG quality 90) with seeded YOLO labels go through ``edgeml_amd.pipeline`` -- SSDLite weak
files, FRCNN strong files (each rank a contiguous, work-balanced block of the single-process run's
size-grouped batches; rows gathered to rank 0, which writes), then ORIE with every image in every
ensemble (E = 99) -- at world 2 over gloo on the one card, and once in this process at world 1.
Every file must be byte-identical between the two runs, and the outputs must satisfy the reference's
file contract (detect.py:83-105, reward.py:86-92): one (N, 6) float64 file per image, rows in
descending confidence (torchvision's score-descending output order), YOLO labels in 0..79, boxes
normalised inside the image, one finite ORIE per image.
"""
import os
import socket
import tempfile
import warnings

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, E = 100, 99


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pipeline(img, lab, work):
    from edgeml_amd import pipeline
    pipeline.main(pipeline.getargs([img, lab, work, "--num-ensemble", str(E), "--seed", "3"]))


def _rank(rank, world, port, img, lab, work, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), EDGEDET_DIST_BACKEND="gloo")
    warnings.filterwarnings("ignore")
    try:
        _pipeline(img, lab, work)
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # report, then fail the rank
        q.put((rank, repr(e)))
        raise


def test_config4_pipeline_world2_equals_world1_on_100_coco_size_jpegs():
    from edgeml_amd import synthetic
    warnings.filterwarnings("ignore")
    with tempfile.TemporaryDirectory() as td:
        img, lab = os.path.join(td, "imgs"), os.path.join(td, "labels")
        synthetic.make_dataset(img, N, seed=11, label_dir=lab, ext=".jpg")
        from PIL import Image
        sizes = set()
        for f in sorted(os.listdir(img)):
            with Image.open(os.path.join(img, f)) as im:
                sizes.add(im.size[::-1])
        assert sizes == set(synthetic.COCO_SIZES)  # every COCO size group: FRCNN plans of four shapes
        one, two = os.path.join(td, "w1"), os.path.join(td, "w2")
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_rank, args=(r, 2, port, img, lab, two, q)) for r in range(2)]
        for p in procs:
            p.start()
        status = dict(q.get(timeout=400) for _ in procs)
        for p in procs:
            p.join(timeout=120)
        assert status == {0: "ok", 1: "ok"}, status
        assert all(p.exitcode == 0 for p in procs)
        _pipeline(img, lab, one)  # single process (no WORLD_SIZE in this environment)
        names = [f"{i:012d}" for i in range(N)]
        for stage in ("weak", "strong"):
            a, b = sorted(os.listdir(os.path.join(one, stage))), sorted(os.listdir(os.path.join(two, stage)))
            assert a == b == [n + ".npy" for n in names], stage
            total = 0
            for f in a:
                with open(os.path.join(one, stage, f), "rb") as x, open(os.path.join(two, stage, f), "rb") as y:
                    assert x.read() == y.read(), (stage, f)
                r = np.load(os.path.join(one, stage, f))
                assert r.dtype == np.float64 and r.ndim == 2 and r.shape[1] == 6, (stage, f, r.shape)
                total += len(r)
                if len(r):
                    assert np.all(np.diff(r[:, 5]) <= 0), (stage, f)          # descending confidence
                    assert np.all(r[:, 0] == np.round(r[:, 0])) and r[:, 0].min() >= 0 and r[:, 0].max() <= 79
                    # normalised boxes inside the image, up to the float32 rounding of the rescale
                    # (orig / resized ratio) and of the division by W / H (detect.py:94-100)
                    assert np.all((r[:, 1:5] >= 0) & (r[:, 1:5] <= 1 + 1e-6)), (stage, f)
                    assert np.all((r[:, 5] > 0) & (r[:, 5] <= 1)), (stage, f)
            assert total > 10 * N, (stage, total)  # detections, not empty files
        with np.load(os.path.join(one, "reward", f"orie{E}.npz")) as z1, \
                np.load(os.path.join(two, "reward", f"orie{E}.npz")) as z2:
            np.testing.assert_array_equal(z1["reward"], z2["reward"])
            assert z1["reward"].shape == (N,) and np.all(np.isfinite(z1["reward"]))
            assert np.count_nonzero(z1["reward"]) > N // 2
