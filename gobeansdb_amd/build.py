"""Build libqlzx.so in-tree with hipcc for gfx950 (no JIT cache, travels with the repo)."""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libqlzx.so")
ARCH = os.environ.get("QLZX_ARCH", "gfx950")


def source_hash() -> str:
    """sha256 (first 16 hex digits) of every csrc/* file, include/qlzx.h and this build script
    (its compile flags, scheduler strategy and split layout), by name and content, plus the target
    arch: compiled into the library (qlzx_info: "src <hash>"), so a binary is tied to the sources
    and the way they were compiled."""
    h = hashlib.sha256()
    h.update(("arch=" + ARCH + "\0").encode())
    srcs = sorted(glob.glob(os.path.join(CSRC, "*"))) + [os.path.join(ROOT, "include", "qlzx.h"),
                                                         os.path.abspath(__file__)]
    for s in srcs:
        if os.path.isfile(s):
            h.update(os.path.relpath(s, ROOT).encode() + b"\0")
            with open(s, "rb") as f:
                h.update(f.read())
    return h.hexdigest()[:16]


def embedded_hash(path: str = OUT) -> str | None:
    """The source hash compiled into a built library (None if absent)."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    i = data.find(b"qlzx-src-hash:")
    return data[i + 14:i + 30].decode() if i >= 0 else None


def _stale() -> bool:
    return embedded_hash(OUT) != source_hash()


PROF_OUT = os.path.join(HERE, "libqlzx_prof.so")


# K1 (k_dec_parse6) and K2 without its CRC prologue (k_dec_chunk4<false>) are compiled in a
# translation unit of their own with this machine-scheduler strategy (csrc/qlzx_k2.hip;
# profiles/r05_sched_strategy_ab.txt)
K2_SCHED = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)


def _compile(out: str, extra: list[str], verbose: bool, split: bool = True) -> None:
    # --offload-compress: the gfx950 code object is stored zstd-compressed (1.1 MB instead of
    # 3.8 MB; the HIP runtime inflates it at load)
    base = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "--offload-compress", "-Wall",
            "-Wno-unused-function", "-Wno-unused-parameter", "-I", os.path.join(ROOT, "include")]
    api = [f"-DQLZX_SRC_HASH=\"{source_hash()}\"", *extra]
    if not split:  # one translation unit (the profile build: its stamps need qlzx_api.hip's g_prof)
        _run([*base, "-shared", *api, "-o", out + ".tmp", os.path.join(CSRC, "qlzx_api.hip")], verbose)
    else:
        oa, ok2 = out + ".api.o", out + ".k2.o"
        _run([*base, "-c", *api, "-DQLZX_SPLIT_K2=1", "-DQLZX_SPLIT_K1=1", "-o", oa, os.path.join(CSRC, "qlzx_api.hip")],
             verbose)
        _run([*base, "-c", "-DQLZX_SPLIT_K1=1", *extra, *K2_SCHED, "-o", ok2, os.path.join(CSRC, "qlzx_k2.hip")],
             verbose)
        _run(["hipcc", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", out + ".tmp", oa, ok2], verbose)
        for f in (oa, ok2):
            os.remove(f)
    os.replace(out + ".tmp", out)


def build(force: bool = False, verbose: bool = False, profile: bool = False) -> str:
    """libqlzx.so (release) and, with profile=True, libqlzx_prof.so (phase stamps)."""
    if force or _stale():
        _compile(OUT, [], verbose)
    if profile:
        _compile(PROF_OUT, ["-DQLZX_PROFILE", "-DQLZX_SP_WAVES_PER_EU=1"], verbose, split=False)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, profile="--profile" in sys.argv))
