"""In-tree build of librc2dgi.so (HIP kernels + C ABI) for gfx950 with hipcc.

The library lands next to this file so that it travels with the repository snapshot to
the GPU box (built ``.so`` files are git-ignored but not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "librc2dgi.so")
SOURCES = ["rc2dgi_kernels.hip", "rc2dgi_rc_f32a.hip", "rc2dgi_rc_f32b.hip", "rc2dgi_rc_f32c.hip", "rc2dgi_rc_f16.hip",
           "rc2dgi_rc_u8.hip", "rc2dgi_rc_top.hip", "rc2dgi_rc_chain.hip", "rc2dgi_capi.cpp", "rc2dgi_shard.cpp", "rc2dgi_paint.hip"]
HEADERS = ["rc2dgi_device.h", "rc2dgi_kernels.h", "rc2dgi_rc.h", "rc2dgi_shard.h", "rc2dgi_paint.h"]
ARCH = os.environ.get("RC2DGI_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: each a*b+c in the kernels is two IEEE roundings, exactly as the GLSL
# expressions they restate; the GL lerp's fused multiply-add is written as fmaf explicitly.
# -disable-promote-alloca-to-lds: per-thread staging arrays stay in VGPRs (the AMDGPU
# promote-alloca pass would otherwise move them to LDS and serialise the staging loads).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result", "-mllvm", "-disable-promote-alloca-to-lds"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build librc2dgi.so)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "rc2dgi.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, extra=(), out: str = LIB) -> str:
    """extra: additional compiler flags (diagnostic builds go to a different `out`).  Every
    translation unit compiles in its own hipcc process (the k_rc_level variant families are
    separate units), then one link."""
    if not force and out == LIB and not _stale():
        return LIB
    from concurrent.futures import ThreadPoolExecutor

    objdir = os.path.join(ROOT, "build", "obj", os.path.basename(out).replace(".so", ""))
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    base = [hipcc()] + FLAGS + list(extra) + ["-I", os.path.join(ROOT, "include")]

    def compile_one(src):
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        cmd = base + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr[-4000:]}")
        return obj

    jobs = int(os.environ.get("MAX_JOBS", "0")) or min(len(SOURCES), os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    link = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    import sys

    if len(sys.argv) > 1 and sys.argv[1] == "diag":
        # timing-only ablation build: march capped at N iterations (WRONG results by design)
        n = sys.argv[2] if len(sys.argv) > 2 else "6"
        print(build(force=True, verbose=True, extra=[f"-DRC2DGI_DIAG_MAX_ITERS={n}"],
                    out=os.path.join(ROOT, "build", "diag", f"librc2dgi_diag{n}.so")))
    elif len(sys.argv) > 1 and sys.argv[1] == "nomerge":
        # timing-only ablation build: RC levels without the upper-cascade staging and merge (WRONG results)
        print(build(force=True, verbose=True, extra=["-DRC2DGI_DIAG_NOMERGE"], out=os.path.join(ROOT, "build", "diag", "librc2dgi_nomerge.so")))
    elif len(sys.argv) > 2 and sys.argv[1] == "exp":
        # A/B build of an experiment: build/ab/librc2dgi_<name>.so with the flags given (scripts/ab_lib.sh)
        print(build(force=True, verbose=True, extra=sys.argv[3:],
                    out=os.path.join(ROOT, "build", "ab", f"librc2dgi_{sys.argv[2]}.so")))
    elif len(sys.argv) > 1 and sys.argv[1] == "timing":
        # diagnostic build: k_rc_level wave-lifetime split by section (s_memtime; scripts/rc_timing.py)
        print(build(force=True, verbose=True, extra=["-DRC2DGI_DIAG_TIMING"] + sys.argv[2:],
                    out=os.path.join(ROOT, "build", "diag", "librc2dgi_timing.so")))
    elif len(sys.argv) > 1 and sys.argv[1] == "stats":
        # diagnostic build: march statistics per level (rc2dgi_diag_stats; atomics, slower)
        print(build(force=True, verbose=True, extra=["-DRC2DGI_DIAG_STATS"], out=os.path.join(ROOT, "build", "diag", "librc2dgi_stats.so")))
    else:
        print(build(force=True, verbose=True))
