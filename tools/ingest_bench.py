"""Image ingest of the detect CLI (detect.py:55-58 read_image) on one GPU: N synthetic COCO-sized JPEGs
through edgeml_amd.detect (SSDLite, the weak stage of config 4) with the device JPEG path
(--decode gpu: Huffman on the host threads, IDCT / upsampling / colour on the GPU) and with the host
decoder (--decode host, PIL), timed end to end (files -> .npy files), outputs compared byte for byte;
plus the entropy-decode rate of the host threads alone.

    python tools/ingest_bench.py [--n 2000] [--quality 90]
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--quality", type=int, default=90)
    a = ap.parse_args()
    from config4_full import _make
    from edgeml_amd import detect, jpeg
    from edgeml_amd.distributed import usable_cpus
    td = tempfile.mkdtemp()
    img, lab = os.path.join(td, "imgs"), os.path.join(td, "labels")
    os.makedirs(img)
    os.makedirs(lab)
    step = 250
    with cf.ProcessPoolExecutor(min(16, usable_cpus())) as ex:
        list(ex.map(_make, [(img, lab, lo, min(lo + step, a.n), 1) for lo in range(0, a.n, step)]))
    print(f"wrote {a.n} JPEGs", flush=True)
    paths = sorted(os.path.join(img, f) for f in os.listdir(img))
    datas = [open(p, "rb").read() for p in paths]
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(usable_cpus()) as ex:
        pks = list(ex.map(lambda d: jpeg.packet(d)[0], datas))
    t_ent = time.perf_counter() - t0
    nnz_bytes = sum(p.size for p in pks)
    out = {"images": a.n, "threads": usable_cpus(), "entropy_decode_images_s": round(a.n / t_ent, 1),
           "packet_MB_per_image": round(nnz_bytes / a.n / 1e6, 3),
           "jpeg_MB_per_image": round(sum(len(d) for d in datas) / a.n / 1e6, 3)}
    res = {}
    for mode in ("gpu", "host", "gpu"):  # gpu twice: the first includes plan building / capture
        d = os.path.join(td, f"out_{mode}")
        t0 = time.perf_counter()
        detect.main(detect.getargs([img, d, "--decode", mode]))
        res[mode] = (time.perf_counter() - t0, d)
        print(mode, round(res[mode][0], 2), "s", flush=True)
    same = all(open(os.path.join(res["gpu"][1], f), "rb").read() == open(os.path.join(res["host"][1], f), "rb").read()
               for f in os.listdir(res["host"][1]))
    out.update({"detect_ssd_gpu_decode_images_s": round(a.n / res["gpu"][0], 1),
                "detect_ssd_host_decode_images_s": round(a.n / res["host"][0], 1),
                "files_byte_identical": same})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
