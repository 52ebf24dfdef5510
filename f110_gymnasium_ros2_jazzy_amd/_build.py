"""Build libf110.so (HIP for gfx950) in-tree with hipcc.

The shared library carries the C ABI of include/f110.h.  It is built next to
this file so it travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libf110.so")
SOURCES = ["f110_kernels.hip", "f110_opponent.hip", "f110_reward.hip", "f110_replay.hip", "f110_adam.hip", "f110_ddpg.hip", "f110_gemm.hip",
           "f110_capi.cpp",
           "f110_replay_capi.cpp"]
HEADERS = ["f110_device.h", "f110_internal.h", "f110_sincos_table.h"]
ARCH = os.environ.get("F110_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: the reference (Python/Numba) never fuses a*b+c; hipcc
# would by default, which changes the last bit of scans and dynamics.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
         f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function", "-fvisibility=hidden"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: libf110.so cannot be built (no HIP toolchain)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(REPO, "include", "f110.h"),
                                                                  os.path.join(REPO, "include", "f110_debug.h"),
                                                                  __file__]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    tmp = LIB + ".tmp"
    cmd = [hipcc()] + FLAGS + [os.path.join(CSRC, f) for f in SOURCES] + ["-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd, cwd=REPO)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
