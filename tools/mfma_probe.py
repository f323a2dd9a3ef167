"""Rounding behaviour of the gfx950 matrix instructions (tools/mfma_probe.hip; diagnostic, needs a GPU).

    python tools/mfma_probe.py

Prints, per instruction, C' - 1 in units of 2^-24 for the experiments of tools/mfma_probe.hip:
  c_rne_pos   RNE +2 / truncation 0        c_rne_neg  RNE -1 / toward zero or -inf -2
  in_group    exact-then-RNE +4 / per-product truncation to the group's largest 0
  cross_group exact-then-RNE +2 / truncated 0
  many_small  1.0 plus (K-1) x 2^-25 (exact (K-1)/2)
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tools", "libmfma_probe.so")
KINDS = {0: ("16x16x32 bf16", 32), 1: ("32x32x16 bf16", 16), 2: ("16x16x16 bf16_1k", 16), 3: ("32x32x8 bf16_1k", 8),
         5: ("16x16x4 f32", 4), 6: ("32x32x2 f32", 2)}
EXPS = ("c_rne_pos", "c_rne_neg", "in_group", "cross_group", "many_small")


def main():
    src = os.path.join(ROOT, "tools", "mfma_probe.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", SO])
    lib = ctypes.CDLL(SO)
    out = (ctypes.c_float * 5)()
    for kind, (name, K) in KINDS.items():
        assert lib.mfma_probe(kind, out) == 0
        vals = [(v - 1.0) / 2.0 ** -24 for v in out]
        print(f"{name:18s} K={K:2d}: " + "  ".join(f"{e} {v:+.2f}" for e, v in zip(EXPS, vals)) +
              f"  (many_small exact {(K - 1) / 2:+.2f})", flush=True)


if __name__ == "__main__":
    main()
