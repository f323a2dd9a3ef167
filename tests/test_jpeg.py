"""Baseline-JPEG ingest (csrc/jpeg.hip; SURVEY §8(f) row 4, detect.py:55-58) on the CPU: the host
entropy decoder's packets, reconstructed by the host checker that shares its integer arithmetic with the
device kernels (csrc/jpeg_core.hpp), are byte-identical to the reference decoder's RGB image (PIL's
libjpeg-turbo, the decode torchvision.io.read_image(..., RGB) performs with libjpeg), over qualities,
chroma samplings, odd sizes, optimised Huffman tables, restart intervals and grayscale.  Unsupported
files (progressive) are reported, not mis-decoded.  tests/test_gpu_jpeg.py checks the device path."""
import io

import numpy as np
import pytest
from PIL import Image

from edgeml_amd import jpeg, synthetic


def _encode(img, **kw):
    b = io.BytesIO()
    img.save(b, "JPEG", **kw)
    return b.getvalue()


def _ref(data):
    with Image.open(io.BytesIO(data)) as im:
        return np.asarray(im.convert("RGB")).transpose(2, 0, 1)


def _scene(h, w, seed):
    return Image.fromarray(synthetic.make_scene(seed, h, w).transpose(1, 2, 0))


CASES = [
    dict(h=480, w=640, quality=75),                     # PIL default: 4:2:0
    dict(h=427, w=640, quality=90, subsampling=0),      # 4:4:4
    dict(h=375, w=500, quality=60, subsampling=1),      # 4:2:2
    dict(h=333, w=501, quality=95),                     # odd width, 4:2:0
    dict(h=101, w=67, quality=30),                      # MCU-ragged on both axes
    dict(h=612, w=612, quality=85, optimize=True),      # optimised Huffman tables
    dict(h=240, w=320, quality=75, restart_marker_blocks=7),
    dict(h=241, w=333, quality=50, restart_marker_rows=1, subsampling=1),
    dict(h=200, w=300, quality=100, subsampling=0),     # quality 100: large coefficients
    dict(h=17, w=9, quality=75),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(str(c[k]) for k in ("h", "w")) + f"q{c['quality']}")
def test_host_reconstruction_is_byte_exact(case):
    c = dict(case)
    h, w = c.pop("h"), c.pop("w")
    data = _encode(_scene(h, w, h * 7 + w), **c)
    pk, hw = jpeg.packet(data)
    assert pk is not None, hw
    assert hw == (h, w)
    np.testing.assert_array_equal(jpeg.reconstruct_host(pk, hw), _ref(data))


@pytest.mark.parametrize("h,w", [(480, 640), (99, 131)])
def test_grayscale(h, w):
    img = _scene(h, w, 3).convert("L")
    data = _encode(img, quality=80)
    pk, hw = jpeg.packet(data)
    assert pk is not None
    np.testing.assert_array_equal(jpeg.reconstruct_host(pk, hw), _ref(data))


def test_noise_image_all_coefficients():
    """Uniform noise: almost every coefficient nonzero (the dense extreme of the packet format)."""
    rs = np.random.RandomState(0)
    img = Image.fromarray(rs.randint(0, 256, (128, 192, 3), dtype=np.uint8))
    data = _encode(img, quality=98, subsampling=0)
    pk, hw = jpeg.packet(data)
    np.testing.assert_array_equal(jpeg.reconstruct_host(pk, hw), _ref(data))


def test_unsupported_and_corrupt():
    data = _encode(_scene(120, 160, 1), quality=75, progressive=True)
    pk, why = jpeg.packet(data)
    assert pk is None and "progressive" in why
    from edgeml_amd import ops
    with pytest.raises(ops.EdgeDetError):
        jpeg.packet(b"\x89PNG\r\n\x1a\n" + bytes(100))


def test_packets_of_the_synthetic_dataset(tmp_path):
    """The COCO-shaped synthetic JPEG set the pipeline benches use (synthetic.make_dataset)."""
    names = synthetic.make_dataset(str(tmp_path), 6, seed=2, ext=".jpg")
    for n in names:
        data = (tmp_path / (n + ".jpg")).read_bytes()
        pk, hw = jpeg.packet(data)
        np.testing.assert_array_equal(jpeg.reconstruct_host(pk, hw), _ref(data))


def test_image_dims_match_pil_headers(tmp_path):
    """edgedet_image_dims (the detect CLI's batch sizing, csrc/jpeg.hip) against PIL's Image.open(path).size
    over baseline / progressive / grayscale JPEGs, one with an EXIF block holding a JPEG thumbnail, PNG,
    and files it must leave to the caller (BMP, not an image, missing)."""
    import ctypes
    from edgeml_amd import detect, ops
    rs = np.random.RandomState(3)
    paths = []
    for k, (h, w) in enumerate([(480, 640), (37, 1001), (1, 1), (640, 427)]):
        im = Image.fromarray(rs.randint(0, 255, (h, w, 3), dtype=np.uint8))
        p = tmp_path / f"b{k}.jpg"
        im.save(p, quality=85)
        paths.append(p)
    im = Image.fromarray(rs.randint(0, 255, (300, 200, 3), dtype=np.uint8))
    im.save(tmp_path / "prog.jpg", progressive=True)
    im.convert("L").save(tmp_path / "gray.jpg")
    thumb = io.BytesIO()
    Image.fromarray(rs.randint(0, 255, (64, 96, 3), dtype=np.uint8)).save(thumb, "JPEG")
    exif = Image.Exif()
    exif[0x0112] = 6  # orientation (not applied by read_image nor by PIL's size)
    big = Image.fromarray(rs.randint(0, 255, (123, 456, 3), dtype=np.uint8))
    big.save(tmp_path / "exif.jpg", exif=exif.tobytes() + b"\0" * 16 + thumb.getvalue())
    im.save(tmp_path / "img.png")
    im.save(tmp_path / "img.bmp")
    (tmp_path / "text.jpg").write_bytes(b"not an image at all")
    paths += [tmp_path / n for n in ("prog.jpg", "gray.jpg", "exif.jpg", "img.png", "img.bmp", "text.jpg", "missing.jpg")]
    hw = np.full((len(paths), 2), -1, np.int32)
    arr = (ctypes.c_char_p * len(paths))(*[bytes(str(p), "utf-8") for p in paths])
    found = ops.lib().edgedet_image_dims(ctypes.cast(arr, ctypes.c_void_p), len(paths), hw.ctypes.data, 2)
    assert found == len(paths) - 3
    for p, (h, w) in zip(paths, hw):
        if p.suffix == ".bmp" or p.name in ("text.jpg", "missing.jpg"):
            assert (h, w) == (0, 0), p
        else:
            assert (h, w) == detect._image_size(str(p)), p


def test_batch_packets_equal_per_file_packets(tmp_path):
    """edgedet_jpeg_batch_packets (the detect CLI's one-call batch entropy decode) lays out exactly the
    per-file packets of edgedet_jpeg_packet behind its offset table, for several thread counts, with a
    first guess too small (the retry path); unsupported and corrupt files come back as None / an error."""
    from edgeml_amd import ops
    rs = np.random.RandomState(4)
    paths = []
    for k in range(7):
        p = tmp_path / f"{k}.jpg"
        p.write_bytes(_encode(_scene(96, 128, 10 + k), quality=int(rs.randint(40, 100)),
                              subsampling=int(rs.randint(0, 3))))
        paths.append(str(p))
    want = [jpeg.packet(open(p, "rb").read())[0] for p in paths]
    for threads in (1, 3, 0):
        pb = jpeg.batch_packets(paths, threads, pinned=False)
        assert pb.hw == (96, 128) and len(pb) == len(paths)
        buf = pb.buf.numpy()
        offs = buf[:8 * len(paths)].view(np.int64)
        assert (offs % 256 == 0).all() and pb.span <= buf.size
        for o, w in zip(offs, want):
            np.testing.assert_array_equal(buf[o:o + w.size], w)
        assert pb.plane_bytes == max(jpeg.plane_bytes(w) for w in want)
    # a buffer too small: the call reports the span it needs and writes nothing past cap
    import ctypes
    arr = (ctypes.c_char_p * 3)(*[p.encode() for p in paths[:3]])
    hw, planes = np.zeros((3, 2), np.int32), ctypes.c_int64(0)
    small = np.full(300, 7, np.uint8)
    need = ops.lib().edgedet_jpeg_batch_packets(ctypes.cast(arr, ctypes.c_void_p), 3, small.ctypes.data, 256,
                                                hw.ctypes.data, ctypes.byref(planes), 2)
    assert need > 256 and (small[256:] == 7).all()
    full = np.zeros(need, np.uint8)
    assert ops.lib().edgedet_jpeg_batch_packets(ctypes.cast(arr, ctypes.c_void_p), 3, full.ctypes.data, need,
                                                hw.ctypes.data, ctypes.byref(planes), 2) == need
    for o, w in zip(full[:24].view(np.int64), want[:3]):
        np.testing.assert_array_equal(full[o:o + w.size], w)
    prog = tmp_path / "prog.jpg"
    prog.write_bytes(_encode(_scene(96, 128, 1), progressive=True))
    assert jpeg.batch_packets(paths[:2] + [str(prog)], 2, pinned=False) is None
    other = tmp_path / "other.jpg"
    other.write_bytes(_encode(_scene(64, 128, 1)))
    assert jpeg.batch_packets(paths[:2] + [str(other)], 2, pinned=False) is None  # sizes differ
    # files the decoder rejects make the batch "unsupported" (decoded on the host, as read_image
    # would): malformed headers, a PNG saved under a .jpg name, corrupt entropy data
    bad = tmp_path / "bad.jpg"
    bad.write_bytes(b"\xff\xd8\xff\xdb" + bytes(40))
    assert jpeg.batch_packets(paths[:2] + [str(bad)], 2, pinned=False) is None
    png = tmp_path / "png.jpg"
    _scene(96, 128, 3).save(png, format="PNG")
    assert jpeg.batch_packets(paths[:2] + [str(png)], 2, pinned=False) is None
    assert "rejected" in ops.lib().edgedet_last_error().decode()
    with pytest.raises(ops.EdgeDetError):
        jpeg.batch_packets([str(tmp_path / "missing.jpg")], 1, pinned=False)
