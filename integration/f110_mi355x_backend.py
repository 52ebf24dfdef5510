"""MI355X backend for the reference's f110_gym: the ctypes binding a
maintainer adds next to ``f110_gym/envs/base_classes.py``.

It binds ``libf110.so`` (``include/f110.h``) with ctypes only; it does not
import this repository's Python package.  It provides drop-ins for the two
reference classes the per-step hot path runs through:

  Simulator        base_classes.py:464-643  (__init__, set_map, update_params,
                                             reset, step -> observation dict)
  ScanSimulator2D  laser_models.py:349-460  (__init__, set_map, scan, get_increment)

Both keep the reference's argument meaning, return types and error
behaviour (ValueError for a scan before set_map or a wrong pose count,
IndexError for an out-of-range agent index).  Scan noise is the reference's
own stream: a ``np.random.default_rng(seed)`` re-created at every reset, one
``rng.normal(0, 0.01, num_beams)`` draw per step shared by all cars
(base_classes.py:119,204; laser_models.py:450-452), handed to the device
through ``f110_set_scan_noise``.

Device memory is held in torch tensors (the reference's RL stack already
depends on torch); every libf110 call takes their ``data_ptr()``.  There is
no CPU fallback: without a gfx950 device ``f110_create`` fails and the error
is raised.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

_LIB_PATH = os.environ.get("LIBF110", "libf110.so")

_P = ctypes.c_void_p
_i32, _i64, _u64, _f64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double


class f110_params(ctypes.Structure):
    _fields_ = [(k, _f64) for k in ("mu", "C_Sf", "C_Sr", "lf", "lr", "h", "m", "I", "s_min", "s_max", "sv_min",
                                    "sv_max", "v_switch", "a_max", "v_min", "v_max", "width", "length",
                                    "lidar_max")]


class f110_config(ctypes.Structure):
    _fields_ = [("n_envs", _i32), ("n_agents", _i32), ("n_beams", _i32), ("theta_dis", _i32),
                ("integrator", _i32), ("ego_idx", _i32), ("autoreset", _i32), ("_pad", _i32),
                ("fov", _f64), ("eps", _f64), ("max_range", _f64), ("time_step", _f64), ("lidar_dist", _f64),
                ("ttc_thresh", _f64), ("noise_std", _f64), ("env_offset", _i64), ("seed", _u64)]


class f110_outputs(ctypes.Structure):
    _fields_ = [(k, _P) for k in ("obs", "scans", "scans_f64", "collisions", "terminated", "was_reset",
                                  "lap_times", "lap_counts", "sim_time")] + [("obs_stride", _i64)]


_lib = None


def lib():
    """Load libf110.so once and declare the entry points used here."""
    global _lib
    if _lib is None:
        L = ctypes.CDLL(_LIB_PATH)
        L.f110_last_error.restype = ctypes.c_char_p
        L.f110_default_params.argtypes = [ctypes.POINTER(f110_params)]
        L.f110_default_config.argtypes = [ctypes.POINTER(f110_config)]
        L.f110_edt_k.argtypes = [_P, _i32, _i32, _P]
        L.f110_create.argtypes = [ctypes.POINTER(_P), _i32, ctypes.POINTER(f110_config),
                                  ctypes.POINTER(f110_params), _P, _i32, _i32, _f64, ctypes.POINTER(_f64), _P, _i32]
        L.f110_destroy.argtypes = [_P]
        L.f110_step.argtypes = [_P, _P, _i32, ctypes.POINTER(f110_outputs), _P]
        L.f110_get_state.argtypes = [_P, _P, _P, _P, _P]
        L.f110_set_state.argtypes = [_P, _P, _P, _P, _P]
        L.f110_scan_batch.argtypes = [_P, _P, _i64, _P, _P, _P, _P]
        L.f110_set_params.argtypes = [_P, ctypes.POINTER(f110_params), _i32, _P]
        L.f110_set_scan_noise.argtypes = [_P, _P]
        if L.f110_abi_version() != 3:  # include/f110.h F110_ABI_VERSION
            raise RuntimeError("libf110.so ABI version mismatch")
        _lib = L
    return _lib


def _check(rc, what):
    if rc < 0:
        raise RuntimeError(f"{what}: {lib().f110_last_error().decode()} ({rc})")


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _load_map(map_path, map_ext):
    """ScanSimulator2D.set_map (laser_models.py:383-427): flip, threshold at 128,
    resolution and origin from the yaml.  Returns (free mask, resolution, origin)."""
    import yaml
    from PIL import Image
    with open(map_path) as f:
        meta = yaml.safe_load(f)
    img_path = os.path.splitext(map_path)[0] + map_ext
    img = np.array(Image.open(img_path).transpose(Image.FLIP_TOP_BOTTOM)).astype(np.float64)
    free = np.ascontiguousarray((img > 128.).astype(np.uint8))
    return free, float(meta["resolution"]), [float(v) for v in meta["origin"]]


def _params_struct(params, base=None):
    p = f110_params()
    if base is not None:
        ctypes.pointer(p)[0] = base
    else:
        lib().f110_default_params(ctypes.byref(p))
    for k, _ in p._fields_:
        if k in params:
            setattr(p, k, float(params[k]))
    return p


class _Context:
    """One libf110 context: a map plus n_agents cars of one environment."""

    def __init__(self, map_path, map_ext, n_agents, params, num_beams=1080, fov=4.7, eps=0.0001, theta_dis=2000,
                 max_range=30.0, time_step=0.01, integrator=1, ego_idx=0, lidar_dist=0.0, seed=12345):
        L = lib()
        if not torch.cuda.is_available():
            raise RuntimeError("libf110 needs a gfx950 device (no CPU fallback)")
        free, res, origin = _load_map(map_path, map_ext)
        H, W = free.shape
        k = np.empty((H, W), np.uint32)
        _check(L.f110_edt_k(free.ctypes.data, H, W, k.ctypes.data), "f110_edt_k")  # get_dt, laser_models.py:40
        cfg = f110_config()
        L.f110_default_config(ctypes.byref(cfg))
        cfg.n_envs, cfg.n_agents, cfg.n_beams, cfg.theta_dis = 1, n_agents, num_beams, theta_dis
        cfg.integrator, cfg.ego_idx = int(getattr(integrator, "value", integrator)), ego_idx
        cfg.fov, cfg.eps, cfg.max_range, cfg.time_step, cfg.lidar_dist = fov, eps, max_range, time_step, lidar_dist
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        cfg.noise_std = 0.0  # noise comes only from the caller's rng (f110_set_scan_noise)
        self.params = _params_struct(params)
        self.ctx = _P()
        dev = torch.cuda.current_device()
        _check(L.f110_create(ctypes.byref(self.ctx), dev, ctypes.byref(cfg), ctypes.byref(self.params),
                             k.ctypes.data, H, W, res, (_f64 * 3)(*origin), None, 0), "f110_create")
        self.A, self.B = n_agents, num_beams
        self.dev = torch.device("cuda", dev)

    def close(self):
        if self.ctx:
            torch.cuda.synchronize(self.dev)
            lib().f110_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ScanSimulator2D:
    """Drop-in for laser_models.ScanSimulator2D (laser_models.py:349-460)."""

    def __init__(self, num_beams, fov, eps=0.0001, theta_dis=2000, max_range=30.0):
        self.num_beams, self.fov, self.eps, self.theta_dis, self.max_range = num_beams, fov, eps, theta_dis, max_range
        self.angle_increment = self.fov / (self.num_beams - 1)
        self._ctx = None

    def set_map(self, map_path, map_ext):
        if self._ctx is not None:
            self._ctx.close()
        self._ctx = _Context(map_path, map_ext, 1, {}, self.num_beams, self.fov, self.eps, self.theta_dis,
                             self.max_range)
        return True

    def scan_batch(self, poses):
        """get_scan for M poses [M, 3] in one launch -> [M, num_beams] (numpy f64)."""
        if self._ctx is None:
            raise ValueError('Map is not set for scan simulator.')
        p = torch.as_tensor(np.asarray(poses, np.float64).reshape(-1, 3), device=self._ctx.dev).contiguous()
        out = torch.empty(p.shape[0], self.num_beams, dtype=torch.float64, device=self._ctx.dev)
        _check(lib().f110_scan_batch(self._ctx.ctx, _ptr(p), p.shape[0], _ptr(out), None, None, _stream()),
               "f110_scan_batch")
        return out.cpu().numpy()

    def scan(self, pose, rng, std_dev=0.01):
        """laser_models.py:429-454: ranges of one pose, plus rng.normal noise."""
        scan = self.scan_batch(np.asarray(pose, np.float64)[None])[0]
        if rng is not None:
            scan += rng.normal(0., std_dev, size=self.num_beams)
        return scan

    def get_increment(self):
        return self.angle_increment


class Simulator:
    """Drop-in for base_classes.Simulator (base_classes.py:464-643).

    ``scan_noise`` (extension, default True = the reference) turns the
    per-car scan noise off for noise-free comparisons."""

    def __init__(self, params, num_agents, seed, time_step=0.01, ego_idx=0, integrator=1, lidar_dist=0.0,
                 scan_noise=True):
        self.num_agents, self.seed, self.time_step, self.ego_idx = num_agents, seed, time_step, ego_idx
        self.params, self.integrator, self.lidar_dist = params, integrator, lidar_dist
        self.scan_noise = scan_noise
        self.agent_poses = np.empty((self.num_agents, 3))
        self.collisions = np.zeros((self.num_agents,))
        self._ctx = None
        self._rng = None
        self._agent_params = [None] * num_agents

    def set_map(self, map_path, map_ext):
        old = self._ctx
        state = None
        if old is not None:  # the reference's cars keep their state across set_map
            state = self._get_state()
        self._ctx = _Context(map_path, map_ext, self.num_agents, self.params, time_step=self.time_step,
                             integrator=self.integrator, ego_idx=self.ego_idx, lidar_dist=self.lidar_dist,
                             seed=self.seed)
        for i, p in enumerate(self._agent_params):
            if p is not None:
                self.update_params(p, agent_idx=i)
        self._noise = torch.zeros(1, self._ctx.B, dtype=torch.float64, device=self._ctx.dev)
        _check(lib().f110_set_scan_noise(self._ctx.ctx, _ptr(self._noise) if self.scan_noise else None),
               "f110_set_scan_noise")
        self._outs_scans = torch.empty(1, self.num_agents, self._ctx.B, dtype=torch.float64, device=self._ctx.dev)
        self._outs_cols = torch.empty(1, self.num_agents, dtype=torch.uint8, device=self._ctx.dev)
        self._outs = f110_outputs(scans_f64=_ptr(self._outs_scans), collisions=_ptr(self._outs_cols))
        if state is not None:
            self._set_state(*state)
        if old is not None:
            old.close()

    def update_params(self, params, agent_idx=-1):
        if agent_idx >= self.num_agents:
            raise IndexError('Index given is out of bounds for list of agents.')
        if self._ctx is None:
            raise ValueError("set_map before update_params")
        p = _params_struct(params, self._ctx.params)
        _check(lib().f110_set_params(self._ctx.ctx, ctypes.byref(p), int(agent_idx), _stream()), "f110_set_params")
        for i in range(self.num_agents):
            if agent_idx < 0 or i == agent_idx:
                self._agent_params[i] = dict(params)

    def _get_state(self):
        A = self.num_agents
        st = torch.empty(7, A, dtype=torch.float64, device=self._ctx.dev)
        sb = torch.empty(2, A, dtype=torch.float64, device=self._ctx.dev)
        sc = torch.empty(A, dtype=torch.int32, device=self._ctx.dev)
        _check(lib().f110_get_state(self._ctx.ctx, _ptr(st), _ptr(sb), _ptr(sc), _stream()), "f110_get_state")
        return st, sb, sc

    def _set_state(self, st, sb, sc):
        _check(lib().f110_set_state(self._ctx.ctx, _ptr(st), _ptr(sb), _ptr(sc), _stream()), "f110_set_state")

    def reset(self, poses):
        """Simulator.reset -> RaceCar.reset per car (base_classes.py:183-204):
        state = (x, y, 0, 0, yaw, 0, 0), empty steer buffer, fresh scan rng."""
        poses = np.asarray(poses)
        if poses.shape[0] != self.num_agents:
            raise ValueError('Number of poses for reset does not match number of agents.')
        st = np.zeros((7, self.num_agents))
        st[0], st[1], st[4] = poses[:, 0], poses[:, 1], poses[:, 2]
        dev = self._ctx.dev
        self._set_state(torch.as_tensor(st, device=dev).contiguous(),
                        torch.zeros(2, self.num_agents, dtype=torch.float64, device=dev),
                        torch.zeros(self.num_agents, dtype=torch.int32, device=dev))
        self._rng = np.random.default_rng(seed=self.seed)

    def step(self, control_inputs):
        """Simulator.step (base_classes.py:566-625) -> observation dict."""
        if self._rng is None:
            raise RuntimeError("reset the simulator before step")
        if self.scan_noise:
            n = self._rng.normal(0., 0.01, size=self._ctx.B)
            self._noise.copy_(torch.from_numpy(n).view(1, -1))
        a = torch.as_tensor(np.asarray(control_inputs, np.float64).reshape(1, self.num_agents, 2),
                            device=self._ctx.dev).contiguous()
        _check(lib().f110_step(self._ctx.ctx, _ptr(a), 1, ctypes.byref(self._outs), _stream()), "f110_step")
        st = self._get_state()[0].cpu().numpy()           # [7, A]
        scans = self._outs_scans[0].cpu().numpy()
        self.collisions = self._outs_cols[0].cpu().numpy().astype(np.float64)
        self.agent_poses = np.stack([st[0], st[1], st[4]], 1)
        A = self.num_agents
        return {'ego_idx': self.ego_idx,
                'scans': [scans[i] for i in range(A)],
                'poses_x': [st[0, i] for i in range(A)],
                'poses_y': [st[1, i] for i in range(A)],
                'poses_theta': [st[4, i] for i in range(A)],
                'linear_vels_x': [st[3, i] for i in range(A)],
                'linear_vels_y': [0. for _ in range(A)],
                'ang_vels_z': [st[5, i] for i in range(A)],
                'collisions': self.collisions}
