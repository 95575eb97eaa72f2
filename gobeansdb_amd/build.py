"""Build libqlzx.so in-tree with hipcc for gfx950 (no JIT cache, travels with the repo)."""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libqlzx.so")
ARCH = os.environ.get("QLZX_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    srcs = glob.glob(os.path.join(CSRC, "*")) + [os.path.join(ROOT, "include", "qlzx.h")]
    return any(os.path.getmtime(s) > t for s in srcs)


PROF_OUT = os.path.join(HERE, "libqlzx_prof.so")


def _compile(out: str, extra: list[str], verbose: bool) -> None:
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-Wno-unused-parameter", *extra,
           "-I", os.path.join(ROOT, "include"), "-o", out + ".tmp",
           os.path.join(CSRC, "qlzx_api.hip")]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)


def build(force: bool = False, verbose: bool = False, profile: bool = False) -> str:
    """libqlzx.so (release) and, with profile=True, libqlzx_prof.so (phase stamps)."""
    if force or _stale():
        _compile(OUT, [], verbose)
    if profile:
        _compile(PROF_OUT, ["-DQLZX_PROFILE", "-DQLZX_SP_WAVES_PER_EU=1"], verbose)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, profile="--profile" in sys.argv))
