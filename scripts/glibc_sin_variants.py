"""Host-only: the reference's float64 sin / cos (np.sin / np.cos, i.e. glibc's
libm here: equal to math.sin on every sampled argument) is not one rounding.
glibc picks its sin / cos by CPU at load time (an FMA build and an SSE2 build
of the same source); the two differ on a fraction of arguments, and each
differs from the correctly rounded value (cr_sincos, f110_host_sincos) on
more.  Runs a child interpreter per glibc variant (GLIBC_TUNABLES masks the
FMA / AVX2 hardware capabilities for the second) and prints one JSON line.

    python scripts/glibc_sin_variants.py
"""
import ctypes
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 400_000
CHILD = r"""
import math, sys, numpy as np
x = np.random.default_rng(3).uniform(-8, 8, %d)
s = np.array([math.sin(v) for v in x]); c = np.array([math.cos(v) for v in x])
assert np.array_equal(s, np.sin(x)) and np.array_equal(c, np.cos(x))
np.save(sys.argv[1], np.stack([s, c]))
""" % N


def variant(path, tunables):
    env = dict(os.environ)
    if tunables:
        env["GLIBC_TUNABLES"] = tunables
    subprocess.run([sys.executable, "-c", CHILD, path], env=env, check=True)
    return np.load(path)


def main():
    sys.path.insert(0, REPO)
    from f110_gymnasium_ros2_jazzy_amd import _lib
    L = _lib.load()
    x = np.random.default_rng(3).uniform(-8, 8, N)
    s, c = np.empty_like(x), np.empty_like(x)
    p = ctypes.c_void_p
    L.f110_host_sincos(x.ctypes.data_as(p), x.size, s.ctypes.data_as(p), c.ctypes.data_as(p))
    with tempfile.TemporaryDirectory() as d:
        fma = variant(os.path.join(d, "fma.npy"), None)
        sse2 = variant(os.path.join(d, "sse2.npy"), "glibc.cpu.hwcaps=-AVX2,-FMA,-FMA4,-AVX")
    libc = ctypes.CDLL("libc.so.6").gnu_get_libc_version
    libc.restype = ctypes.c_char_p
    print(json.dumps({
        "glibc": libc().decode(), "args": N, "range": [-8, 8],
        "fma_vs_sse2": {"sin": int((fma[0] != sse2[0]).sum()), "cos": int((fma[1] != sse2[1]).sum())},
        "fma_vs_correctly_rounded": {"sin": int((fma[0] != s).sum()), "cos": int((fma[1] != c).sum())},
        "sse2_vs_correctly_rounded": {"sin": int((sse2[0] != s).sum()), "cos": int((sse2[1] != c).sum())},
    }))


if __name__ == "__main__":
    main()
