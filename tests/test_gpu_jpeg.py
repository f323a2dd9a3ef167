"""The device JPEG reconstruction (csrc/jpeg.hip jpeg_idct_kernel + jpeg_color_kernel) byte-exact
against the reference decoder (PIL's libjpeg-turbo; torchvision.io.read_image(..., RGB) of
detect.py:55-58 decodes with libjpeg the same way), batched as the detect CLI batches: images of one
size, packets of different sizes and block counts in one launch."""
import io

import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu


def _case(h, w, seed, **kw):
    from edgeml_amd import synthetic
    img = Image.fromarray(synthetic.make_scene(seed, h, w).transpose(1, 2, 0))
    if kw.pop("gray", False):
        img = img.convert("L")
    b = io.BytesIO()
    img.save(b, "JPEG", **kw)
    data = b.getvalue()
    with Image.open(io.BytesIO(data)) as im:
        ref = np.asarray(im.convert("RGB")).transpose(2, 0, 1)
    return data, ref


@pytest.mark.parametrize("h,w,kws", [
    (480, 640, [dict(quality=75), dict(quality=95), dict(quality=40, optimize=True), dict(quality=75, subsampling=0)]),
    (427, 640, [dict(quality=75, subsampling=1), dict(quality=80, restart_marker_blocks=5), dict(quality=70, gray=True)]),
    (101, 67, [dict(quality=30), dict(quality=100, subsampling=0)]),
])
def test_gpu_decode_batch_byte_exact(h, w, kws):
    from edgeml_amd import jpeg
    cases = [_case(h, w, 10 * i + h, **dict(k)) for i, k in enumerate(kws)]
    pks = []
    for data, _ in cases:
        pk, hw = jpeg.packet(data)
        assert pk is not None and hw == (h, w)
        pks.append(pk)
    out = torch.zeros((len(pks), 3, h, w), dtype=torch.uint8, device="cuda")
    dec = jpeg.BatchDecoder("cuda")
    for _ in range(2):  # the second call reuses the staging / scratch buffers
        out.zero_()
        dec.decode(pks, out)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for b, (_, ref) in enumerate(cases):
            np.testing.assert_array_equal(got[b], ref)


def test_gpu_decode_synthetic_coco_set(tmp_path):
    """The synthetic COCO-sized JPEG set of the pipeline benches, batched by size."""
    from edgeml_amd import jpeg, synthetic
    names = synthetic.make_dataset(str(tmp_path), 24, seed=9, ext=".jpg")
    by = {}
    for n in names:
        data = (tmp_path / (n + ".jpg")).read_bytes()
        pk, hw = jpeg.packet(data)
        with Image.open(io.BytesIO(data)) as im:
            ref = np.asarray(im.convert("RGB")).transpose(2, 0, 1)
        by.setdefault(hw, []).append((pk, ref))
    dec = jpeg.BatchDecoder("cuda")
    for (h, w), items in by.items():
        out = torch.empty((len(items), 3, h, w), dtype=torch.uint8, device="cuda")
        dec.decode([p for p, _ in items], out)
        torch.cuda.synchronize()
        for b, (_, ref) in enumerate(items):
            np.testing.assert_array_equal(out[b].cpu().numpy(), ref)


def test_detect_cli_gpu_decode_equals_host_decode(tmp_path):
    """The detect CLI with the device JPEG path (default) writes byte-identical .npy files to the
    all-host decode (--decode host): mixed sizes, a ragged batch, and a PNG among the JPEGs (its
    batch falls back to the host decoder)."""
    import os
    from edgeml_amd import detect, synthetic
    img = tmp_path / "imgs"
    names = synthetic.make_dataset(str(img), 11, seed=4, ext=".jpg", sizes=[(480, 640), (427, 640)])
    synthetic.make_dataset(str(tmp_path / "png"), 1, seed=8, ext=".png", sizes=[(480, 640)])
    os.replace(tmp_path / "png" / "000000000000.png", img / "zz_extra.png")
    outs = {}
    for mode in ("gpu", "host"):
        d = tmp_path / mode
        detect.main(detect.getargs([str(img), str(d), "--decode", mode]))
        outs[mode] = d
    files = sorted(os.listdir(outs["gpu"]))
    assert files == sorted(os.listdir(outs["host"])) and len(files) == len(names) + 1
    for f in files:
        assert (outs["gpu"] / f).read_bytes() == (outs["host"] / f).read_bytes(), f
