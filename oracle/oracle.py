"""NumPy front-end for the C oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY — the parity checker.  Imported by tests/,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg; never by
the product package.  See f110_oracle.c for the reference file:line each
restated function follows.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# F110_ORACLE_LIB: an alternate build of the same source (scripts/sanitize.sh: ASan/UBSan)
LIB_PATH = os.environ.get("F110_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")

_D = ctypes.POINTER(ctypes.c_double)
_I32 = ctypes.POINTER(ctypes.c_int32)
_U32 = ctypes.POINTER(ctypes.c_uint32)
_U8 = ctypes.POINTER(ctypes.c_uint8)


class Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in
                ("mu", "C_Sf", "C_Sr", "lf", "lr", "h", "m", "I", "s_min", "s_max", "sv_min",
                 "sv_max", "v_switch", "a_max", "v_min", "v_max", "width", "length")]


class Scanner(ctypes.Structure):
    _fields_ = [("H", ctypes.c_int32), ("W", ctypes.c_int32), ("theta_dis", ctypes.c_int32),
                ("num_beams", ctypes.c_int32), ("res", ctypes.c_double), ("orig_x", ctypes.c_double),
                ("orig_y", ctypes.c_double), ("orig_c", ctypes.c_double), ("orig_s", ctypes.c_double),
                ("fov", ctypes.c_double), ("eps", ctypes.c_double), ("max_range", ctypes.c_double),
                ("theta_index_increment", ctypes.c_double), ("dt", _D), ("sines", _D), ("cosines", _D)]


class Sim(ctypes.Structure):
    _fields_ = [("sc", ctypes.POINTER(Scanner)), ("p", ctypes.POINTER(Params)), ("angles", _D),
                ("beam_cos", _D), ("side", _D), ("dt", ctypes.c_double), ("lidar_dist", ctypes.c_double),
                ("ttc_thresh", ctypes.c_double), ("n_agents", ctypes.c_int32), ("integrator", ctypes.c_int32),
                ("noise_std", ctypes.c_double), ("noise_seed", ctypes.c_uint64), ("step_no", ctypes.c_uint64)]


DEFAULT_PARAMS = {'mu': 1.0489, 'C_Sf': 4.718, 'C_Sr': 5.4562, 'lf': 0.15875, 'lr': 0.17145,
                  'h': 0.074, 'm': 3.74, 'I': 0.04712, 's_min': -0.4189, 's_max': 0.4189,
                  'sv_min': -3.2, 'sv_max': 3.2, 'v_switch': 7.319, 'a_max': 9.51,
                  'v_min': 0.00000001, 'v_max': 20.0, 'width': 0.31, 'length': 0.58}

_lib = None


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "f110_oracle.c")
    if os.environ.get("F110_ORACLE_LIB"):
        return LIB_PATH  # prebuilt by its own recipe
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE, "-B", "liboracle.so"])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.or_edt_k.argtypes = [_U8, ctypes.c_int, ctypes.c_int, _U32]
        L.or_edt_k.restype = ctypes.c_int
        L.or_scan_tables.argtypes = [ctypes.c_int, _D, _D]
        L.or_beam_tables.argtypes = [ctypes.c_int] + [ctypes.c_double] * 4 + [_D, _D, _D]
        L.or_get_scan.argtypes = [ctypes.POINTER(Scanner), _D, _D, _I32, _I32]
        L.or_scan_batch.argtypes = [ctypes.POINTER(Scanner), _D, ctypes.c_int64, _D, _I32, _I32, ctypes.c_int]
        L.or_beam_indices.argtypes = [ctypes.POINTER(Scanner), ctypes.c_double, _D]
        L.or_vehicle_dynamics_st.argtypes = [_D, _D, ctypes.POINTER(Params), _D]
        L.or_vehicle_dynamics_ks.argtypes = [_D, _D, ctypes.POINTER(Params), _D]
        L.or_pid.argtypes = [ctypes.c_double] * 8 + [_D]
        L.or_update_pose.argtypes = [_D, _D, _I32, ctypes.c_double, ctypes.c_double, ctypes.POINTER(Params),
                                     ctypes.c_double, ctypes.c_int]
        L.or_check_ttc.argtypes = [_D, ctypes.c_int, ctypes.c_double, _D, _D, ctypes.c_double]
        L.or_check_ttc.restype = ctypes.c_int
        L.or_get_vertices.argtypes = [_D, ctypes.c_double, ctypes.c_double, _D]
        L.or_collision.argtypes = [_D, _D]
        L.or_collision.restype = ctypes.c_int
        L.or_collision_multiple.argtypes = [_D, ctypes.c_int, _D, _D]
        L.or_ray_cast.argtypes = [_D, _D, _D, ctypes.c_int, _D]
        L.or_sim_step.argtypes = [ctypes.POINTER(Sim), ctypes.c_int64, _D, _D, _I32, _D, _D, _D, ctypes.c_int]
        L.or_sim_reset.argtypes = [ctypes.c_int64, _D, _D, _I32, _D]
        L.or_gap_follow.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_int32, ctypes.c_double,
                                    ctypes.c_double, _D, _I32]
        _lib = L
    return _lib


_HOOK_KEEP = []


def set_device_trig(on: bool = True):
    """Residue attribution only: route the oracle's sin / cos at
    the sites the device evaluates with its correctly rounded cr_sincos
    through libf110's host copy of it (f110_host_sincos); off restores glibc
    (the reference's).  The scan tables stay glibc's either way."""
    L = lib()
    if not hasattr(L, "_hooked"):
        L.or_set_sincos_hook.argtypes = [ctypes.c_void_p]
        L.or_set_sincos_hook.restype = None
        L._hooked = True
    if not on:
        L.or_set_sincos_hook(None)
        return
    from f110_gymnasium_ros2_jazzy_amd import _lib as F
    fn = F.load().f110_host_sincos
    _HOOK_KEEP[:] = [fn]
    L.or_set_sincos_hook(ctypes.cast(fn, ctypes.c_void_p))


class device_trig:
    """Context manager: set_device_trig(True) inside, glibc again after."""

    def __enter__(self):
        set_device_trig(True)
        return self

    def __exit__(self, *exc):
        set_device_trig(False)
        return False


def _p(a, t=_D):
    return a.ctypes.data_as(t)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def make_params(d=None) -> Params:
    d = dict(DEFAULT_PARAMS, **(d or {}))
    return Params(**{k: float(d[k]) for k, _ in Params._fields_})


# ------------------------------------------------------------------ EDT ----
def edt_k(free_mask: np.ndarray) -> np.ndarray:
    fm = np.ascontiguousarray(free_mask, dtype=np.uint8)
    H, W = fm.shape
    k = np.empty((H, W), np.uint32)
    rc = lib().or_edt_k(_p(fm, _U8), H, W, _p(k, _U32))
    if rc != 0:
        raise ValueError(f"or_edt_k failed ({rc})")
    return k


def scan_tables(theta_dis=2000):
    s = np.empty(theta_dis)
    c = np.empty(theta_dis)
    lib().or_scan_tables(theta_dis, _p(s), _p(c))
    return s, c


def beam_tables(nb=1080, fov=4.7, params=None):
    d = dict(DEFAULT_PARAMS, **(params or {}))
    a, c, s = np.empty(nb), np.empty(nb), np.empty(nb)
    lib().or_beam_tables(nb, fov, d["width"], d["lf"], d["lr"], _p(a), _p(c), _p(s))
    return a, c, s


class OracleScanner:
    """ScanSimulator2D (laser_models.py:348-457) restated: noise-free scans."""

    def __init__(self, free_mask, res, origin, num_beams=1080, fov=4.7, eps=0.0001, theta_dis=2000,
                 max_range=30.0):
        self.k = edt_k(free_mask)
        self.H, self.W = self.k.shape
        self.dt = _f64(res * np.sqrt(self.k.astype(np.float64)))
        self.sines, self.cosines = scan_tables(theta_dis)
        self.num_beams = num_beams
        angle_increment = fov / (num_beams - 1)
        tii = theta_dis * angle_increment / (2. * np.pi)
        self.sc = Scanner(H=self.H, W=self.W, theta_dis=theta_dis, num_beams=num_beams, res=float(res),
                          orig_x=float(origin[0]), orig_y=float(origin[1]), orig_c=float(np.cos(origin[2])),
                          orig_s=float(np.sin(origin[2])), fov=float(fov), eps=float(eps),
                          max_range=float(max_range), theta_index_increment=float(tii),
                          dt=_p(self.dt), sines=_p(self.sines), cosines=_p(self.cosines))

    def scan(self, poses, with_probe=False, threads=1):
        poses = _f64(np.atleast_2d(poses))
        M = poses.shape[0]
        out = np.empty((M, self.num_beams))
        look = np.empty((M, self.num_beams), np.int32) if with_probe else None
        rc = np.empty((M, self.num_beams, 2), np.int32) if with_probe else None
        lib().or_scan_batch(ctypes.byref(self.sc), _p(poses), M, _p(out),
                            _p(look, _I32) if with_probe else None, _p(rc, _I32) if with_probe else None,
                            threads)
        return (out, look, rc) if with_probe else out

    def beam_indices(self, yaw):
        out = np.empty(self.num_beams)
        lib().or_beam_indices(ctypes.byref(self.sc), float(yaw), _p(out))
        return out


# ------------------------------------------------------------- dynamics ----
def vehicle_dynamics_st(x, u, params: Params):
    f = np.empty(7)
    lib().or_vehicle_dynamics_st(_p(_f64(x)), _p(_f64(u)), ctypes.byref(params), _p(f))
    return f


def vehicle_dynamics_ks(x, u, params: Params):
    f = np.empty(5)
    lib().or_vehicle_dynamics_ks(_p(_f64(x)), _p(_f64(u)), ctypes.byref(params), _p(f))
    return f


def pid(speed, steer, cur_speed, cur_steer, max_sv, max_a, max_v, min_v):
    out = np.empty(2)
    lib().or_pid(speed, steer, cur_speed, cur_steer, max_sv, max_a, max_v, min_v, _p(out))
    return out[0], out[1]


def update_pose(state, buf, cnt, steer, vel, params: Params, dt=0.01, integrator=1):
    """In-place on state (7,), buf (2,), cnt (1,) int32 arrays."""
    lib().or_update_pose(_p(state), _p(buf), _p(cnt, _I32), float(steer), float(vel), ctypes.byref(params),
                         float(dt), int(integrator))


def check_ttc(scan, vel, beam_cos, side, thresh=0.005):
    scan = _f64(scan)
    return bool(lib().or_check_ttc(_p(scan), scan.shape[0], float(vel), _p(_f64(beam_cos)), _p(_f64(side)),
                                   float(thresh)))


def get_vertices(pose, length, width):
    v = np.empty((4, 2))
    lib().or_get_vertices(_p(_f64(pose)), float(length), float(width), _p(v))
    return v


def collision(v1, v2):
    return bool(lib().or_collision(_p(_f64(v1)), _p(_f64(v2))))


def collision_multiple(verts):
    verts = _f64(verts)
    n = verts.shape[0]
    c, i = np.empty(n), np.empty(n)
    lib().or_collision_multiple(_p(verts), n, _p(c), _p(i))
    return c, i


def ray_cast(pose, scan, angles, vertices):
    scan = _f64(scan).copy()
    angles = _f64(angles)
    lib().or_ray_cast(_p(_f64(pose)), _p(scan), _p(angles), angles.shape[0], _p(_f64(vertices)))
    return scan


# ------------------------------------------------------------ simulator ----
class OracleSim:
    """Simulator.step / reset (base_classes.py:464-643) for E independent
    envs of A agents, noise-free.  State layout AoS [E*A][7]."""

    def __init__(self, scanner: OracleScanner, n_envs, n_agents, params=None, dt=0.01, lidar_dist=0.0,
                 integrator=1, ttc_thresh=0.005):
        self.scanner = scanner
        self.E, self.A = n_envs, n_agents
        self.params = make_params(params)
        self.angles, self.beam_cos, self.side = beam_tables(scanner.num_beams, scanner.sc.fov, params)
        self.state = np.zeros((n_envs * n_agents, 7))
        self.buf = np.zeros((n_envs * n_agents, 2))
        self.cnt = np.zeros(n_envs * n_agents, np.int32)
        self.sim = Sim(sc=ctypes.pointer(scanner.sc), p=ctypes.pointer(self.params), angles=_p(self.angles),
                       beam_cos=_p(self.beam_cos), side=_p(self.side), dt=float(dt),
                       lidar_dist=float(lidar_dist), ttc_thresh=float(ttc_thresh), n_agents=n_agents,
                       integrator=integrator)

    def reset(self, poses):
        poses = _f64(poses).reshape(self.E * self.A, 3)
        lib().or_sim_reset(self.E * self.A, _p(self.state), _p(self.buf), _p(self.cnt, _I32), _p(poses))

    def set_noise(self, std: float, seed: int = 0):
        """Host-drawn scan noise (timing baseline only; parity runs keep 0)."""
        self.sim.noise_std = float(std)
        self.sim.noise_seed = int(seed) & 0xFFFFFFFFFFFFFFFF

    def step(self, actions, threads=1):
        self.sim.step_no += 1
        actions = _f64(actions).reshape(self.E * self.A, 2)
        scans = np.empty((self.E * self.A, self.scanner.num_beams))
        cols = np.empty(self.E * self.A)
        lib().or_sim_step(ctypes.byref(self.sim), self.E, _p(self.state), _p(self.buf), _p(self.cnt, _I32),
                          _p(actions), _p(scans), _p(cols), threads)
        return scans.reshape(self.E, self.A, -1), cols.reshape(self.E, self.A)


# ------------------------------------------------------------------ map ----
def gap_follow_action(scan, angle_min=-np.pi / 2, angle_increment=np.pi / 1080):
    """gap_follow.py:44-58 on one float32 scan -> (action f64 [2], gap (start, end))."""
    s = np.ascontiguousarray(scan, dtype=np.float32)
    act = np.empty(2)
    gap = np.empty(2, np.int32)
    lib().or_gap_follow(s.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), s.shape[0], angle_min, angle_increment,
                        _p(act), _p(gap, _I32))
    return act, gap


class LapOracle:
    """F110Env's lap bookkeeping (_check_done, f110_env.py:310-352, with the
    start state of reset, :444-451), restated in NumPy for the checker: start
    zone 2 m either side of the ego start line, toggles on entering / leaving
    it (squared distance <= 0.1), lap_counts = toggles // 2, lap_times frozen
    at the fourth toggle, done on the ego's collision or every car's fourth
    toggle.  float32 reset poses keep the reference's dtype behaviour (float32
    start poses and start_rot, float64 arithmetic after the upcast)."""

    def __init__(self, poses, ego_idx=0):
        poses = np.asarray(poses)
        n = poses.shape[0]
        self.ego_idx = ego_idx
        self.start_xs, self.start_ys = poses[:, 0], poses[:, 1]
        th = poses[ego_idx, 2]
        self.start_rot = np.array([[np.cos(-th), -np.sin(-th)], [np.sin(-th), np.cos(-th)]])
        self.near_starts = np.array([True] * n)
        self.toggle_list = np.zeros((n,))
        self.lap_counts = np.zeros((n,))
        self.lap_times = np.zeros((n,))

    def check_done(self, poses_x, poses_y, collisions, current_time):
        left_t = right_t = 2
        dx = np.array(poses_x) - self.start_xs
        dy = np.array(poses_y) - self.start_ys
        delta_pt = np.dot(self.start_rot, np.stack((dx, dy), axis=0))
        temp_y = delta_pt[1, :]
        beyond_left = temp_y > left_t
        beyond_right = temp_y < -right_t
        temp_y[beyond_left] -= left_t
        temp_y[beyond_right] = -right_t - temp_y[beyond_right]
        temp_y[np.invert(np.logical_or(beyond_left, beyond_right))] = 0
        closes = (delta_pt[0, :] ** 2 + temp_y ** 2) <= 0.1
        for i in range(len(closes)):
            if closes[i] and not self.near_starts[i]:
                self.near_starts[i] = True
                self.toggle_list[i] += 1
            elif not closes[i] and self.near_starts[i]:
                self.near_starts[i] = False
                self.toggle_list[i] += 1
            self.lap_counts[i] = self.toggle_list[i] // 2
            if self.toggle_list[i] < 4:
                self.lap_times[i] = current_time
        done = collisions[self.ego_idx] or np.all(self.toggle_list >= 4)
        return bool(done), self.toggle_list >= 4


def load_map(yaml_path, map_ext=".png"):
    """ScanSimulator2D.set_map (laser_models.py:383-427) restated:
    PIL load -> FLIP_TOP_BOTTOM -> (<=128 -> occupied) ; returns
    (free_mask uint8 [H,W], resolution, origin[3])."""
    import yaml
    from PIL import Image
    img_path = os.path.splitext(yaml_path)[0] + map_ext
    img = np.array(Image.open(img_path).transpose(Image.FLIP_TOP_BOTTOM)).astype(np.float64)
    free = (img > 128.).astype(np.uint8)
    with open(yaml_path) as f:
        meta = yaml.safe_load(f)
    return free, float(meta["resolution"]), [float(v) for v in meta["origin"]]
