"""Build an A/B variant of libedgedet.so with extra -D flags into build/variants/lib_<name>.so
(load it with EDGEDET_LIB=...).  python tools/build_variant.py NAME -DX6_PF=2 ..."""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "edgeml-object-detection_amd"))
import build as B  # noqa: E402

name, extra = sys.argv[1], sys.argv[2:]
od = os.path.join(ROOT, "build", "variants", name)
os.makedirs(od, exist_ok=True)
B.write_tile_table(od)


def cc(src):
    obj = os.path.join(od, os.path.basename(src)[:-4] + ".o")
    r = subprocess.run([B.hipcc(), *B.FLAGS, *extra, "-I", od, "-c", src, "-o", obj], capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    return obj


with cf.ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(cc, B.sources()))
out = os.path.join(ROOT, "build", "variants", f"lib_{name}.so")
subprocess.run([B.hipcc(), "-shared", f"--offload-arch={B.ARCH}", *objs, "-o", out], check=True)
print(out)
