"""libf110.so host-side checks (no GPU): the library loads, exports every
symbol include/f110.h declares, and its host paths (EDT, lookup tables,
beam-index runs, argument validation) match the golden vectors / oracle."""
import ctypes
import hashlib
import os
import re

import numpy as np
import pytest

from conftest import MAPS, REPO, golden


@pytest.fixture(scope="module")
def L():
    from f110_gymnasium_ros2_jazzy_amd import _lib
    return _lib.load()


def declared_symbols():
    names = []
    for h in os.listdir(os.path.join(REPO, "include")):
        if h.endswith(".h"):
            txt = open(os.path.join(REPO, "include", h)).read()
            names += re.findall(r"F110_API\s+[\w\s\*]*?\b(f110_\w+)\s*\(", txt)
    return sorted(set(names))


def test_exports_every_declared_symbol(L):
    names = declared_symbols()
    assert len(names) >= 17
    for n in names:
        assert hasattr(L, n), f"libf110.so does not export {n}"
    from f110_gymnasium_ros2_jazzy_amd import _lib
    assert sorted(_lib.EXPORTS) == names


def test_abi_and_defaults(L):
    from f110_gymnasium_ros2_jazzy_amd import _lib
    assert L.f110_abi_version() == 3
    p = _lib.default_params().as_dict()
    # F110Env default params (f110_env.py:132-156)
    assert p["v_min"] == 1e-8 and p["a_max"] == 9.51 and p["sv_max"] == 3.2 and p["lidar_max"] == 30.0
    c = _lib.default_config()
    assert (c.n_agents, c.n_beams, c.theta_dis, c.integrator) == (2, 1080, 2000, 1)
    assert (c.fov, c.eps, c.max_range, c.time_step, c.ttc_thresh) == (4.7, 1e-4, 30.0, 0.01, 0.005)


def test_host_tables(L):
    from f110_gymnasium_ros2_jazzy_amd import _lib
    t = golden("tables.npz")
    p = _lib.default_params()
    s, c, a, bc, sd = (np.empty(2000), np.empty(2000), np.empty(1080), np.empty(1080), np.empty(1080))
    L.f110_host_tables(2000, 1080, 4.7, ctypes.byref(p), *(x.ctypes.data for x in (s, c, a, bc, sd)))
    assert np.array_equal(s, t["sines"]) and np.array_equal(c, t["cosines"])
    assert np.array_equal(a, t["scan_angles"]) and np.array_equal(bc, t["beam_cosines"])
    assert np.array_equal(sd, t["side_distances"])


@pytest.mark.parametrize("m", ["Spielberg_map", "straight_corridor", "Shanghai_map"])
def test_edt_matches_scipy_golden(L, m):
    from f110_gymnasium_ros2_jazzy_amd.maps import load_map
    e = golden(f"edt_{m}.npz")
    tm = load_map(os.path.join(MAPS, m + ".yaml"))
    k = tm.ensure_edt()
    assert hashlib.sha256(k.tobytes()).hexdigest() == e["k_sha256"].item().decode()
    assert hashlib.sha256(tm.dt().tobytes()).hexdigest() == e["dt_sha256"].item().decode()


def test_edt_edge_cases(L, oracle_mod):
    from f110_gymnasium_ros2_jazzy_amd.maps import edt_k
    rng = np.random.default_rng(3)
    for shape, p in [((1, 1), 0.0), ((1, 7), 0.5), ((9, 1), 0.5), ((37, 53), 0.9), ((64, 64), 0.999),
                     ((128, 96), 0.5)]:
        free = (rng.random(shape) < p).astype(np.uint8)
        free.flat[rng.integers(free.size)] = 0   # at least one occupied cell
        assert np.array_equal(edt_k(free), oracle_mod.edt_k(free))
    from f110_gymnasium_ros2_jazzy_amd import F110Error
    with pytest.raises(F110Error):
        edt_k(np.ones((4, 4), np.uint8))    # no occupied cell: EDT undefined


def _seq_indices(yaw, fov, td, nb):
    """get_scan's beam index, sequential (laser_models.py:167-184)."""
    inc = td * (fov / (nb - 1)) / (2. * np.pi)
    t = td * (yaw - fov / 2.) / (2. * np.pi)
    t = np.fmod(t, td)
    while t < 0:
        t += td
    out = np.empty(nb)
    for i in range(nb):
        out[i] = t
        t += inc
        while t >= td:
            t -= td
    return out


def test_beam_index_runs_spielberg_config(L, oracle_scanners):
    sc = oracle_scanners("Spielberg_map")
    rng = np.random.default_rng(0)
    yaws = np.concatenate([rng.uniform(-20, 20, 3000), np.linspace(-np.pi, np.pi, 1001),
                           [0.0, 2.35, -2.35, 2.35 + 2 * np.pi, 1e-300, -1e-300, 4.7 / 2, 1e6]])
    out = np.empty(1080)
    for y in yaws:
        n = L.f110_host_beam_indices(float(y), 4.7, 2000, 1080, out.ctypes.data)
        assert 0 < n <= 80
        assert np.array_equal(out, sc.beam_indices(y)), y


@pytest.mark.parametrize("fov,td,nb", [(6.2, 2000, 1080), (3.14159, 2000, 271), (4.7, 1000, 1080),
                                       (0.5, 2000, 64), (4.7, 4096, 2160), (6.28, 360, 3),
                                       (4.7, 7, 1080), (4.7, 2, 1080), (6.2, 100, 2048), (4.7, 2000, 65536)])
def test_beam_index_runs_other_configs(L, fov, td, nb):
    """Runs against the sequential accumulation; small theta_dis (indices below 1 over a large part
    of the scan) and fine scans included: there the runs cover binades below 1 too."""
    rng = np.random.default_rng(1)
    out = np.empty(nb)
    for y in rng.uniform(-10, 10, 200 if nb <= 4096 else 20):
        n = L.f110_host_beam_indices(float(y), fov, td, nb, out.ctypes.data)
        assert 0 < n <= 80
        assert np.array_equal(out, _seq_indices(y, fov, td, nb))


@pytest.mark.parametrize("fov,td,nb", [(4.7, 2000, 1080), (6.2, 2000, 1080), (3.14159, 2000, 271),
                                       (4.7, 1000, 1080), (0.5, 2000, 64), (4.7, 4096, 2160), (6.28, 360, 3),
                                       (4.7, 3, 1080), (1.0, 7, 1081)])
def test_beam_runs_fast_builder_agrees(L, fov, td, nb):
    """k_agents' run builder (approximate quotient + exact fixups) gives build_beam_runs' runs."""
    rng = np.random.default_rng(2)
    yaws = np.concatenate([rng.uniform(-20, 20, 2000), np.linspace(-np.pi, np.pi, 501), [0.0, 2.35, -2.35, 1e-300]])
    for y in yaws:
        assert L.f110_host_beam_runs_agree(float(y), fov, td, nb) == 1, (y, fov, td, nb)


def test_sincos_fast_path_matches_cr_sincos(L):
    """The branch-free common case of cr_sincos (k_agents) gives cr_sincos's bits wherever it
    claims to apply, and claims it for almost every argument."""
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.uniform(-8, 8, 400000), rng.uniform(-0.42, 0.42, 200000),
                        rng.uniform(-3000, 3000, 100000), 10.0 ** rng.uniform(-300, 5.9, 50000),
                        [0.0, -0.0, np.pi / 4, -np.pi / 4, 1048575.9, 1048576.0, 1e300, np.inf, -np.inf, np.nan,
                         5e-324, -5e-324]])
    n = x.size
    s0, c0 = np.empty(n), np.empty(n)
    s1, c1 = np.empty(n), np.empty(n)
    ok = np.zeros(n, np.uint8)
    L.f110_host_sincos(x.ctypes.data, n, s0.ctypes.data, c0.ctypes.data)
    L.f110_host_sincos_fast(x.ctypes.data, n, s1.ctypes.data, c1.ctypes.data, ok.ctypes.data)
    m = ok.astype(bool)
    assert np.array_equal(s1[m].view(np.uint64), s0[m].view(np.uint64))
    assert np.array_equal(c1[m].view(np.uint64), c0[m].view(np.uint64))
    assert not m[-7:-2].any() and m[-12] and m[-11]  # 2^20, 1e300, +-inf, NaN fall back; +-0 do not
    assert m.mean() > 0.995


def _tan_cr(x):
    """tan(x) correctly rounded to double: 40-digit sin / cos series (|x| < 3.2)."""
    from decimal import Decimal, getcontext
    getcontext().prec = 40
    d = Decimal(float(x))  # exact
    s, c, term, k = Decimal(0), Decimal(0), Decimal(1), 0
    while True:  # term = x^k / k!
        if k % 4 == 0: c += term
        elif k % 4 == 1: s += term
        elif k % 4 == 2: c -= term
        else: s -= term
        k += 1
        term = term * d / k
        if abs(term) < Decimal(10) ** -38:
            break
    return float(s / c)


def test_tan_cos_fast_is_correctly_rounded(L):
    """k_agents' tan (one table evaluation with the cos): the correctly rounded tan where it
    claims certainty, cr_sincos's cos where it claims that, both for nearly every argument."""
    rng = np.random.default_rng(4)
    x = np.concatenate([rng.uniform(-0.42, 0.42, 3000), rng.uniform(-3.1, 3.1, 1000), 10.0 ** rng.uniform(-12, -1, 300),
                        [0.0, -0.0, 0.4189, -0.4189, 1.0, np.pi / 4]])
    n = x.size
    t, c = np.empty(n), np.empty(n)
    okt, okc = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
    L.f110_host_tan_cos_fast(x.ctypes.data, n, t.ctypes.data, c.ctypes.data, okt.ctypes.data, okc.ctypes.data)
    s0, c0 = np.empty(n), np.empty(n)
    L.f110_host_sincos(x.ctypes.data, n, s0.ctypes.data, c0.ctypes.data)
    mc = okc.astype(bool)
    assert np.array_equal(c[mc].view(np.uint64), c0[mc].view(np.uint64))
    mt = okt.astype(bool)
    assert mt.mean() > 0.99 and mc.mean() > 0.99
    ref = np.array([_tan_cr(v) if v != 0.0 else v for v in x[mt]])  # tan(+-0) = +-0
    assert np.array_equal(t[mt].view(np.uint64), ref.view(np.uint64))
    assert np.signbit(t[-5]) and not np.signbit(t[-6])  # tan(-0) = -0
    # the reference's libm tan agrees on all but a fraction of a percent
    assert np.mean(t[mt] != np.tan(x[mt])) < 0.01


def test_create_validates_without_gpu(L):
    """No GPU here: f110_create must fail loudly (no CPU fallback)."""
    from f110_gymnasium_ros2_jazzy_amd import _lib
    p = _lib.default_params()
    c = _lib.default_config()
    k = np.zeros((4, 4), np.uint32)
    origin = (ctypes.c_double * 3)(0, 0, 0)
    ctx = ctypes.c_void_p()
    c.n_agents = 9
    rc = L.f110_create(ctypes.byref(ctx), 0, ctypes.byref(c), ctypes.byref(p), k.ctypes.data, 4, 4, 0.05,
                       origin, None, 0)
    assert rc == -1 and b"n_agents" in L.f110_last_error()
    c.n_agents = 2
    c.fov = 7.0
    rc = L.f110_create(ctypes.byref(ctx), 0, ctypes.byref(c), ctypes.byref(p), k.ctypes.data, 4, 4, 0.05,
                       origin, None, 0)
    assert rc == -1
    # a scan so fine against theta_dis that its beam-index runs could overflow the 80-run table
    # (f110_device.h max_beam_runs): rejected before any device call
    c.fov, c.theta_dis, c.n_beams = 0.001, 2, 2048
    rc = L.f110_create(ctypes.byref(ctx), 0, ctypes.byref(c), ctypes.byref(p), k.ctypes.data, 4, 4, 0.05,
                       origin, None, 0)
    assert rc == -1 and b"beam-index runs" in L.f110_last_error()
    c.fov, c.theta_dis, c.n_beams = 4.7, 2000, 1080
    rc = L.f110_create(ctypes.byref(ctx), 0, ctypes.byref(c), ctypes.byref(p), k.ctypes.data, 4, 4, 0.05,
                       origin, None, 0)
    import torch
    if not torch.cuda.is_available():
        assert rc == -4 and ctx.value is None      # F110_E_NODEVICE
    elif rc == 0:
        L.f110_destroy(ctx)


def test_batchsim_refuses_cpu():
    import torch
    from f110_gymnasium_ros2_jazzy_amd import F110Error
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(F110Error):
        BatchSim("Spielberg_map", n_envs=1, n_agents=1)


def _boundary_points(H, W, res, origin, rng):
    """Points whose map-frame coordinates sit on / next to cell boundaries
    (including x_rot/res rounding up to W or H), off-map and non-finite ones,
    mapped back to the world frame through the origin pose."""
    xs = []
    for n, lim in ((W, W), (H, H)):
        k = np.arange(0, lim + 1, dtype=np.float64) * res
        v = np.concatenate([k, np.nextafter(k, -np.inf), np.nextafter(k, np.inf),
                            np.nextafter(np.nextafter(k, -np.inf), -np.inf), rng.uniform(-res, lim * res + res, 64)])
        xs.append(v)
    xr = rng.choice(xs[0], 4000)
    yr = rng.choice(xs[1], 4000)
    # also pair every x boundary with a y boundary row near the top / bottom
    xr = np.concatenate([xr, xs[0], xs[0], [np.nan, np.inf, -np.inf, 0.0]])
    yr = np.concatenate([yr, np.full(xs[0].size, np.nextafter(H * res, 0)), np.zeros(xs[0].size),
                         [0.0, 0.0, 0.0, np.nan]])
    c, s = np.cos(origin[2]), np.sin(origin[2])
    # world = origin + R(yaw) [xr, yr]  (inverse of xy_2_rc's rotation; exactness is not needed:
    # the three mappings are compared with each other on the same world points)
    with np.errstate(invalid="ignore"):
        x = origin[0] + c * xr - s * yr
        y = origin[1] + s * xr + c * yr
    if origin[2] == 0.0:
        x, y = origin[0] + xr, origin[1] + yr
    return np.ascontiguousarray(np.stack([x, y], 1))


@pytest.mark.parametrize("H,W,res,origin,roundup", [
    (2000, 2000, 0.05, (-78.21853769831466, -44.37590462453829, 0.0), False),   # Spielberg
    (13, 7, 0.05, (-0.3, -0.2, 0.0), False),                                      # H, W not multiples of 4
    (8, 12, 0.1, (0.0, 0.0, 0.0), False),                                         # multiples of 4 (tile edge)
    (64, 40, 0.05, (-1.0, -1.0, 0.3), False),                                     # rotated origin
    (33, 17, 0.07, (2.0, -3.0, -1.2), False),
    # fl(v/res) == W (or H) for v = nextafter(W*res, 0): 17, 34, 39, 68 at res 0.05 / 0.1,
    # 9 and 13 at 0.07; H = 68 is a multiple of 4 (the row past the last tile row)
    (68, 17, 0.05, (0.0, 0.0, 0.0), True),
    (39, 34, 0.1, (0.0, 0.0, 0.0), True),
    (13, 9, 0.07, (0.0, 0.0, 0.0), True),
])
def test_cell_mappings_agree_on_boundaries(H, W, res, origin, roundup):
    """The ray kernel's tiled, fast-quotient cell mapping equals xy_2_rc's
    IEEE int(x_rot/res) row-major read (laser_models.py:55-104), including
    quotients that round up to W or H and off-map / NaN points."""
    import ctypes
    from f110_gymnasium_ros2_jazzy_amd import _lib
    L = _lib.load(build_if_missing=False)
    rng = np.random.default_rng(H * 1000 + W)
    xy = _boundary_points(H, W, res, origin, rng)
    out = np.empty((xy.shape[0], 3), np.int64)
    org = (ctypes.c_double * 3)(*origin)
    assert L.f110_host_cell_index(H, W, res, org, xy.ctypes.data, xy.shape[0], out.ctypes.data) == 0
    assert np.array_equal(out[:, 0], out[:, 1])
    assert np.array_equal(out[:, 0], out[:, 2])
    assert out.min() >= 0 and out.max() <= H * W - 1
    assert (out[:, 0] == H * W - 1).any() and (out[:, 0] < H * W - 1).sum() > 1000
    if roundup:  # map frame == world frame: the round-up case must be present
        x, y = xy[:, 0], xy[:, 1]
        with np.errstate(invalid="ignore"):
            up = ((x < W * res) & (x >= 0) & (np.floor(x / res) == W)) | ((y < H * res) & (y >= 0) & (np.floor(y / res) == H))
        assert up.any()


def test_window_ranges_contain_window_beams():
    """k_post_multi visits only the beam ranges window_beam_ranges returns;
    every beam whose angle lies in the box window must be inside them."""
    import ctypes
    from f110_gymnasium_ros2_jazzy_amd import _lib
    L = _lib.load(build_if_missing=False)
    rng = np.random.default_rng(7)
    for fov, B in ((4.7, 1080), (2 * np.pi - 0.01, 720), (1.0, 64), (4.7, 541)):
        ang = np.empty(B)
        L.f110_host_tables(2000, B, fov, ctypes.byref(_lib.default_params()), None, None,
                           ang.ctypes.data, None, None)
        for _ in range(3000):
            yaw = rng.uniform(-50, 50)
            center = rng.uniform(-10, 10)
            half = rng.choice([rng.uniform(1e-5, 0.05), rng.uniform(0.05, 1.5), rng.uniform(1.5, 3.14)])
            out = np.empty(4, np.int32)
            L.f110_host_window_ranges(yaw, fov, B, center, half, out.ctypes.data)
            d = yaw + ang - center
            d = d - 2 * np.pi * np.rint(d / (2 * np.pi))
            inside = np.nonzero(np.abs(d) <= half)[0]
            covered = ((inside >= out[0]) & (inside <= out[1])) | ((inside >= out[2]) & (inside <= out[3]))
            assert covered.all(), (fov, B, yaw, center, half, out, inside[~covered])


def test_np_float32_sincos_matches_numpy():
    """The device's float32 start_rot trig (f110_device.h np_sincosf,
    F110Env.reset with float32 options, f110_env.py:448-451) against the
    installed NumPy's float32 np.cos / np.sin, bit for bit: yaw range, wider
    arguments, quadrant boundaries, signed zeros, NaN."""
    import ctypes
    from f110_gymnasium_ros2_jazzy_amd import _lib
    L = _lib.load()
    rng = np.random.default_rng(3)
    xs = [rng.uniform(-np.pi, np.pi, 400_000), rng.uniform(-200, 200, 200_000),
          (np.arange(-64, 65) * np.pi / 4), np.array([0.0, -0.0, np.pi, -np.pi, 1e-30, -1e-30])]
    x = np.concatenate(xs).astype(np.float32)
    x = np.concatenate([x, np.nextafter(x[-129 - 6:-6], np.float32(np.inf)), np.array([np.nan], np.float32)])
    for op, ref in ((1, np.cos), (0, np.sin)):
        out = np.empty_like(x)
        L.f110_host_np_sincosf(x.ctypes.data_as(ctypes.c_void_p), x.size, op, out.ctypes.data_as(ctypes.c_void_p))
        want = ref(x)
        same = (out == want) | (np.isnan(out) & np.isnan(want))
        assert same.all(), (op, x[~same][:5], out[~same][:5], want[~same][:5])


def _dec_sincos(v):
    """sin and cos of the double v to ~55 digits (Taylor series after reduction
    by a 100-digit 2 pi): the correctly rounded double is float() of it."""
    from decimal import Decimal, getcontext
    getcontext().prec = 60
    pi = Decimal("3.14159265358979323846264338327950288419716939937510582097494459230781640628620899862803")
    x = Decimal(float(v))
    r = x - (x / (2 * pi)).to_integral_value() * 2 * pi
    out = []
    for t, k in ((r, 1), (Decimal(1), 0)):
        acc = Decimal(0)
        while abs(t) > Decimal(10) ** -58:
            acc += t
            t = -t * r * r / ((k + 1) * (k + 2))
            k += 2
        out.append(float(acc))
    return out


def test_cr_sincos_matches_numpy():
    """f110_device.h cr_sincos (the ray_cast beam direction, box vertices,
    dynamics and start_rot sin / cos, double-double + one rounding) against
    NumPy's float64 np.sin / np.cos (glibc here), the reference's own trig:
    bit-exact but on a small rest (< 0.3 % of arguments over scan / yaw
    ranges), and on a sample of that rest cr_sincos is the correctly rounded
    value (checked to 55 digits), i.e. the rest is glibc's own last-ulp error.
    Signed zeros, NaN and |x| >= 2^20 (library fallback) too."""
    import ctypes
    from f110_gymnasium_ros2_jazzy_amd import _lib
    L = _lib.load()
    rng = np.random.default_rng(17)
    x = np.concatenate([rng.uniform(-8, 8, 600_000), rng.uniform(-1e-3, 1e-3, 50_000),
                        np.arange(-64, 65) * (np.pi / 4), np.array([0.0, -0.0, 1e-300, 2.0 ** 20, 1e7])])
    s, c = np.empty_like(x), np.empty_like(x)
    L.f110_host_sincos(x.ctypes.data_as(ctypes.c_void_p), x.size, s.ctypes.data_as(ctypes.c_void_p),
                       c.ctypes.data_as(ctypes.c_void_p))
    for got, ref, name in ((s, np.sin(x), "sin"), (c, np.cos(x), "cos")):
        bad = np.flatnonzero(got != ref)
        assert bad.size < 0.003 * x.size, (name, bad.size)
        for i in bad[:: max(1, bad.size // 40)]:
            want = _dec_sincos(x[i])[0 if name == "sin" else 1]
            assert got[i] == want, (name, x[i], got[i], ref[i], want)
    assert np.signbit(s[x.size - 4]) and s[x.size - 4] == 0.0 and c[x.size - 4] == 1.0  # sin(-0.0) = -0.0
    xn = np.array([np.nan, np.inf])
    sn, cn = np.empty_like(xn), np.empty_like(xn)
    L.f110_host_sincos(xn.ctypes.data_as(ctypes.c_void_p), 2, sn.ctypes.data_as(ctypes.c_void_p),
                       cn.ctypes.data_as(ctypes.c_void_p))
    assert np.isnan(sn).all() and np.isnan(cn).all()


def test_cr_sincos_table_equals_series():
    """cr_sincos's table path (sin / cos of i/64 plus short series, taken
    where its rounding is certain) gives the same bits as the double-double
    series alone (f110_host_sincos_series) on uniform, scan-grid, tiny,
    large, table-cell-edge and near-quadrant arguments."""
    import ctypes
    from f110_gymnasium_ros2_jazzy_amd import _lib
    L = _lib.load()
    rng = np.random.default_rng(29)
    x = np.concatenate([
        rng.uniform(-2 * np.pi, 2 * np.pi, 1_500_000), rng.uniform(-1e5, 1e5, 300_000),
        np.exp(rng.uniform(np.log(1e-300), 0.0, 300_000)) * rng.choice([-1.0, 1.0], 300_000),
        ((-2.35 + np.arange(1080) * (4.7 / 1079))[None, :] + rng.uniform(-np.pi, np.pi, (300, 1))).ravel(),
        ((np.arange(-60, 60)[:, None] + 0.5) / 64 + np.arange(-100, 101)[None, :] * 2.0 ** -52).ravel(),
        ((np.arange(-40000, 40000) * (np.pi / 2))[:, None] * (1 + np.arange(-3, 4)[None, :] * 2.0 ** -52)).ravel(),
    ])
    out = [np.empty_like(x) for _ in range(4)]
    p = [a.ctypes.data_as(ctypes.c_void_p) for a in [x] + out]
    L.f110_host_sincos(p[0], x.size, p[1], p[2])
    L.f110_host_sincos_series(p[0], x.size, p[3], p[4])
    assert np.array_equal(out[0].view(np.int64), out[2].view(np.int64))
    assert np.array_equal(out[1].view(np.int64), out[3].view(np.int64))


@pytest.mark.parametrize("H,W,pad",[(7, 5, 3), (40, 33, 12), (1, 1, 1), (16, 15, 0)])
def test_host_map_tables(L, H, W, pad):
    """The fixed-point kernels' EDT tables as f110_create builds them
    (f110_host_map_table, the same host code): the row-major table (rows of
    W + 1 rounded up to 16 cells, dt[-1,-1] in the padding column / row, a 0.0
    zero cell after the last row) and the padded one (pad cells of dt[-1,-1]
    on every side, rows of 511 mod 512 cells, the zero cell after the last
    row), checked cell by cell against a NumPy construction."""
    rng = np.random.default_rng(H * 100 + W)
    k = rng.integers(0, 50, (H, W)).astype(np.uint32)
    res = 0.05
    dt = res * np.sqrt(k.astype(np.float64))
    meta = np.zeros(3, np.int64)
    for kind in (0, 1):
        n = L.f110_host_map_table(k.ctypes.data, H, W, res, kind, pad, None, 0, meta.ctypes.data)
        rows, cols, zero = (int(v) for v in meta)
        if kind == 1 and pad == 0:
            assert n == 0 and zero == -1  # no padded table without padding
            continue
        out = np.full(n, np.nan)
        assert L.f110_host_map_table(k.ctypes.data, H, W, res, kind, pad, out.ctypes.data, n, meta.ctypes.data) == n
        assert n == rows * cols + 16 and zero == rows * cols * 8
        ref = np.full(rows * cols + 16, dt[-1, -1])
        grid = ref[:rows * cols].reshape(rows, cols)
        if kind == 0:
            assert cols % 16 == 0 and cols >= W + 1 and rows == H + 1
            grid[:H, :W] = dt
        else:
            assert cols % 512 == 511 and cols >= W + 2 * pad + 1 and rows == H + 2 * pad
            grid[pad:pad + H, pad:pad + W] = dt
        ref[rows * cols] = 0.0
        assert np.array_equal(out, ref)
