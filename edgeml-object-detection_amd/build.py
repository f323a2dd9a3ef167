"""Build libedgedet.so (every HIP kernel + the native plan executor) for gfx950, in-tree.

    python -m edgeml_amd.build        (or edgeml_amd.build.build())

Each csrc/*.hip is compiled with hipcc --offload-arch=gfx950 in parallel, then linked into
edgeml-object-detection_amd/libedgedet.so.  -ffp-contract=off keeps every float op of the
box/NMS/RoIAlign arithmetic individually rounded, as in the reference's scalar CPU kernels.
"""
import concurrent.futures as cf
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libedgedet.so")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
# Per-file flags.  conv.hip: no SLP vectorisation, so the stage-sum adds and the operand split stay
# scalar v_fmac_f32 / v_sub_f32: beside MFMAs a packed f32 op costs about three scalar ones
# (MI355X_MICROARCH.md, 'price of one filler beside MFMAs').
FILE_FLAGS = {"conv.hip": ["-fno-slp-vectorize"]}


def hipcc():
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: libedgedet.so cannot be built")


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


TILES_JSON = os.path.join(HERE, "data", "conv_tiles_gfx950.json")


def _deps():
    return sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hpp")] + [
        os.path.join(os.path.dirname(HERE), "include", "edgedet.h"), TILES_JSON]


def write_tile_table(objdir):
    """The tuned conv tile table (data/conv_tiles_gfx950.json, also read by plan.py) as a C++
    initializer list for the native lowering (csrc/lower.hip)."""
    import json
    with open(TILES_JSON) as f:
        tiles = json.load(f).get("tiles", {})
    path = os.path.join(objdir, "conv_tiles_gfx950.inc")
    body = "".join(f'{{"{k}", {int(v)}}},\n' for k, v in sorted(tiles.items()))
    if not os.path.exists(path) or open(path).read() != body:
        with open(path, "w") as f:
            f.write(body)


def up_to_date():
    if not os.path.exists(LIB) or not os.path.exists(os.path.join(os.path.dirname(HERE), "tools", "native_host")):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in _deps())


DIAG_LIB = os.path.join(HERE, "libedgedet_diag.so")


def build(force=False, verbose=False, jobs=8, diag=False, variant=None, defines=(), extra_flags=(), only=()):
    """diag=True: libedgedet_diag.so with -DEDGEDET_DIAG (the EDGEDET_DIAG_SKIP op-family skips of
    csrc/exec.hip, wrong results; load it with EDGEDET_LIB, tools/gpu_skip.sh).  variant="name" with
    defines=("NMS_PROFILE", ...): libedgedet_<name>.so built with those -D flags (diagnostic builds,
    loaded with EDGEDET_LIB); extra_flags: further hipcc flags of such a variant (A/B builds); only:
    the csrc files a variant compiles, the product's objects (build/) standing in for the rest.
    Never the product."""
    if variant:
        diag = True
    lib = os.path.join(HERE, f"libedgedet_{variant}.so") if variant else (DIAG_LIB if diag else LIB)
    if not force and not diag and up_to_date():
        return LIB
    cc = hipcc()
    objdir = os.path.join(HERE, f"build_{variant}" if variant else ("build_diag" if diag else "build"))
    os.makedirs(objdir, exist_ok=True)
    write_tile_table(objdir)

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src)[:-4] + ".o")
        dflags = [f"-D{d}" for d in defines] + list(extra_flags) if variant else (["-DEDGEDET_DIAG"] if diag else [])
        cmd = [cc, *FLAGS, *FILE_FLAGS.get(os.path.basename(src), []), *dflags, "-I", objdir, "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        if verbose and r.stderr:
            print(r.stderr)
        return obj

    def obj_of(src):
        if variant and only and os.path.basename(src) not in only:
            return os.path.join(HERE, "build", os.path.basename(src)[:-4] + ".o")
        return compile_one(src)

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(obj_of, sources()))
    tmp = lib + ".tmp"
    r = subprocess.run([cc, "-shared", f"--offload-arch={ARCH}", *objs, "-o", tmp], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, lib)
    if not diag:
        build_native_host(cc)
    return lib


HOST_SRC = os.path.join(os.path.dirname(HERE), "tools", "native_host.cpp")
HOST_BIN = os.path.join(os.path.dirname(HERE), "tools", "native_host")


def build_native_host(cc=None):
    """tools/native_host: a C++ program (no Python) that runs a detector through the model-level
    C-ABI, linked against the in-tree libedgedet.so (rpath relative to the binary)."""
    if not os.path.exists(HOST_SRC):
        return None
    cc = cc or hipcc()
    cmd = [cc, "-O2", "-std=c++17", HOST_SRC, "-I", os.path.join(os.path.dirname(HERE), "include"), "-L", HERE,
           "-ledgedet", "-Wl,-rpath,$ORIGIN/../edgeml-object-detection_amd", "-o", HOST_BIN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native_host build failed:\n{r.stderr}")
    return HOST_BIN


if __name__ == "__main__":
    import sys
    print(build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv))
