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


def _corrupt_scan_copy(src, dst):
    """Copy a baseline JPEG with bytes of its entropy-coded scan overwritten so that the device path's
    entropy decoder rejects it (edgedet_jpeg_packet raises) while PIL/libjpeg still decodes it."""
    from edgeml_amd import jpeg, ops
    data = bytearray(src.read_bytes())
    sos = data.index(b"\xff\xda")
    start = sos + 2 + int.from_bytes(data[sos + 2:sos + 4], "big")
    rs = np.random.RandomState(0)
    for _ in range(200):
        d = bytearray(data)
        at = int(rs.randint(start + 64, len(d) - 256))
        d[at:at + 24] = bytes(int(v) for v in rs.randint(0, 255, 24))  # no 0xFF: no new markers
        try:
            jpeg.packet(bytes(d))
            continue  # still parses: try another spot
        except ops.EdgeDetError:
            pass
        try:
            with Image.open(io.BytesIO(bytes(d))) as im:
                im.convert("RGB").load()
        except Exception:
            continue
        dst.write_bytes(bytes(d))
        return
    raise AssertionError("no corruption found that the device decoder rejects and PIL decodes")


def test_detect_cli_gpu_decode_equals_host_decode(tmp_path):
    """The detect CLI with the device JPEG path (default) writes byte-identical .npy files to the
    all-host decode (--decode host): mixed sizes, a ragged batch, and a PNG among the JPEGs (its
    batch falls back to the host decoder)."""
    import os
    from edgeml_amd import detect, synthetic
    img = tmp_path / "imgs"
    names = synthetic.make_dataset(str(img), 11, seed=4, ext=".jpg", sizes=[(480, 640), (427, 640)])
    synthetic.make_dataset(str(tmp_path / "png"), 2, seed=8, ext=".png", sizes=[(480, 640)])
    os.replace(tmp_path / "png" / "000000000000.png", img / "zz_extra.png")
    # a PNG saved under a .jpg name (read_image picks the format from the magic bytes) and a JPEG
    # whose scan the device path's entropy decoder rejects (libjpeg warns and still decodes): their
    # batches fall back to the host decoder instead of failing the run
    os.replace(tmp_path / "png" / "000000000001.png", img / "zz_png_named.jpg")
    _corrupt_scan_copy(img / (names[0] + ".jpg"), img / "zz_corrupt.jpg")
    outs = {}
    for mode in ("gpu", "host"):
        d = tmp_path / mode
        detect.main(detect.getargs([str(img), str(d), "--decode", mode]))
        outs[mode] = d
    files = sorted(os.listdir(outs["gpu"]))
    assert files == sorted(os.listdir(outs["host"])) and len(files) == len(names) + 3
    for f in files:
        assert (outs["gpu"] / f).read_bytes() == (outs["host"] / f).read_bytes(), f
