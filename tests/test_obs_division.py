"""k_rays_fxs's obs-entry division (f110_kernels.hip obs_scan_value_fast):
F110Env._pack_flat_obs divides the clipped float32 scan by lidar_max in
float32 (f110_env.py:557-560).  The kernel computes q = v * y, r = fma(-q,
lm, v), q' = fma(r, y, q) with y = RN(1 / lm) (obs_reciprocal,
f110_internal.h) and takes the IEEE divide for v < 2^-60 or lm outside
[2^-30, 2^30].  Here the same formula, compiled with gcc (fmaf is correctly
rounded), is compared with the IEEE divide for EVERY float32 v in
[2^-60, lm] at the reference's lidar_max = 30 (f110_env.py:156), and on a
strided sweep for other lidar_max values at the edges of the fast range."""
import os
import shutil
import subprocess
import tempfile

import pytest

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
int main(int argc, char **argv) {
    float lm = strtof(argv[1], 0);
    uint32_t stride = (uint32_t)strtoul(argv[2], 0, 10);
    volatile float lv = lm;
    float y = 1.0f / lv;  /* obs_reciprocal */
    uint32_t lo, hi;
    float lo_f = 0x1p-60f;
    memcpy(&lo, &lo_f, 4);
    memcpy(&hi, &lm, 4);
    unsigned long long n = 0, bad = 0;
    for (uint32_t u = lo; u <= hi && u >= lo; u += stride) {
        float v;
        memcpy(&v, &u, 4);
        float q = v * y;
        float q2 = fmaf(fmaf(-q, lm, v), y, q);
        float ex = v / lv;
        if (memcmp(&q2, &ex, 4)) ++bad;
        ++n;
    }
    printf("%llu %llu\n", n, bad);
    return 0;
}
"""


@pytest.fixture(scope="module")
def divcheck():
    cc = shutil.which("gcc")
    if not cc:
        pytest.skip("gcc not available")
    d = tempfile.mkdtemp()
    src, exe = os.path.join(d, "div.c"), os.path.join(d, "div")
    with open(src, "w") as f:
        f.write(SRC)
    subprocess.run([cc, "-O2", "-ffp-contract=off", "-o", exe, src, "-lm"], check=True)
    yield exe
    shutil.rmtree(d, ignore_errors=True)


def _run(exe, lm, stride):
    out = subprocess.run([exe, repr(lm), str(stride)], check=True, capture_output=True, text=True).stdout.split()
    return int(out[0]), int(out[1])


def test_obs_division_exhaustive_reference_lidar_max(divcheck):
    n, bad = _run(divcheck, 30.0, 1)  # every float32 in [2^-60, 30]
    assert n > 5 * 10**8 and bad == 0


@pytest.mark.parametrize("lm", [2.0 ** -30, 1e-3, 0.1, 1.0, 10.0, 12345.678, 1e6, 2.0 ** 30])
def test_obs_division_other_lidar_max(divcheck, lm):
    n, bad = _run(divcheck, lm, 97)
    assert n > 10**6 and bad == 0
