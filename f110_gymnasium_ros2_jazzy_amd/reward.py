"""The training reward on the device.

Mirrors rl_training/utils/track_progress.py:CenterlineProgress (:5-110) and
rl_training/utils/rewards.py:CenterlineSafetyProgressReward (:185-355), which
train_ddpg.py evaluates on the host for every next_obs
(``rew = reward_fn(next_obs)``, :176).  Here the reward of every env of a
batch is one wave of libf110's ``f110_reward``; the per-env progress state
stays on the device.

    track = CenterlineTrack.from_csv(".../Spielberg_map.csv")
    reward_fn = BatchedCenterlineReward(n_envs, dt=0.01, progress=track, w_prog=5.0, ...)
    reward_fn.reset()                       # all envs (or reset(env_mask))
    r = reward_fn(obs)                      # obs: float32 [n_envs, obs_len] cuda -> float64 [n_envs]

Same kwargs and defaults as the reference class; ``progress=None`` selects
the reference's Euclidean fallback (_ProgFallback, rewards.py:72-84).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def load_centerline_csv(path: str):
    """(xy [n, 2], w_right [n] | None, w_left [n] | None) parsed the way
    CenterlineProgress.__init__ parses the file (pandas.read_csv, column
    names stripped of blanks and '#', track_progress.py:18-27)."""
    try:
        import pandas as pd
    except ImportError as exc:  # pragma: no cover - pandas is in the image
        raise ImportError("load_centerline_csv needs pandas (the reference's parser)") from exc
    df = pd.read_csv(path)
    df.columns = [c.strip().lstrip("#").strip() for c in df.columns]
    if not {"x_m", "y_m"}.issubset(df.columns):
        raise ValueError(f"CSV must have x_m,y_m; has {df.columns}")
    xy = df[["x_m", "y_m"]].to_numpy(dtype=float)
    if len(xy) < 2:
        raise ValueError("Need at least 2 centerline points")
    if {"w_tr_right_m", "w_tr_left_m"}.issubset(df.columns):
        return xy, df["w_tr_right_m"].to_numpy(dtype=float), df["w_tr_left_m"].to_numpy(dtype=float)
    return xy, None, None


class CenterlineTrack:
    """CenterlineProgress's arrays (xy, s, tan, nrm, mid, widths, L) in device
    memory (f110_track).  ``device=None`` keeps the host arrays only."""

    def __init__(self, xy, w_right=None, w_left=None, closed: bool = True, device=0):
        self.L_lib = _lib.load()
        self.xy = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 2)
        self.n = self.xy.shape[0]
        self.closed = bool(closed)
        self.wR = None if w_right is None else np.ascontiguousarray(w_right, dtype=np.float64)
        self.wL = None if w_left is None else np.ascontiguousarray(w_left, dtype=np.float64)
        if (self.wR is None) != (self.wL is None):
            raise ValueError("give both lane widths or neither")
        dev = -1 if device is None else (torch.device(device).index if not isinstance(device, int) else device)
        self.device = None if device is None else torch.device("cuda", dev or 0)
        h = ctypes.c_void_p()
        _lib.check(self.L_lib.f110_track_create(
            ctypes.byref(h), -1 if device is None else int(dev or 0), self.xy.ctypes.data,
            None if self.wR is None else self.wR.ctypes.data, None if self.wL is None else self.wL.ctypes.data,
            self.n, int(self.closed)), "f110_track_create")
        self.handle = h
        self.s = np.empty(self.n)
        self.tan = np.empty((self.n - 1, 2))
        self.nrm = np.empty((self.n - 1, 2))
        self.mid = np.empty((self.n - 1, 2))
        self.L = self.L_lib.f110_track_arrays(h, self.s.ctypes.data, self.tan.ctypes.data, self.nrm.ctypes.data,
                                              self.mid.ctypes.data)
        self.has_widths = self.wR is not None

    @classmethod
    def from_csv(cls, path: str, closed: bool = True, device=0) -> "CenterlineTrack":
        xy, wr, wl = load_centerline_csv(path)
        return cls(xy, wr, wl, closed=closed, device=device)

    def close(self):
        if getattr(self, "handle", None):
            self.L_lib.f110_track_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BatchedCenterlineReward:
    """CenterlineSafetyProgressReward for n_envs envs at once (one state per env)."""

    def __init__(self, n_envs: int, dt: float, progress: CenterlineTrack | None, w_prog: float = 1.2,
                 forward_sign: float = +1.0, alive_bonus: float = 0.02, w_rel_lead: float = 0.0,
                 lead_clip: float = 5.0, w_lat: float = 0.35, lat_cap: float = 4.0, default_half_width: float = 1.5,
                 lidar_max: float = 1.0, near_wall_dist: float = 0.35 / 30.0, w_wall: float = 1.0,
                 wall_quantile: float = 0.05, opp_safe_dist: float = 0.7, w_opp: float = 0.8,
                 ego_crash_penalty: float = 50.0, opp_crash_bonus: float = 50.0, grace_steps_wall: int = 25,
                 grace_steps_opp: int = 25, device=0, num_beams: int = 1080):
        self.L_lib = _lib.load()
        p = _lib.F110RewardParams()
        self.L_lib.f110_default_reward_params(ctypes.byref(p))
        for k, v in dict(dt=dt, w_prog=w_prog, forward_sign=forward_sign, alive_bonus=alive_bonus,
                         w_rel_lead=w_rel_lead, lead_clip=lead_clip, w_lat=w_lat, lat_cap=lat_cap,
                         default_half_width=default_half_width, lidar_max=lidar_max, near_wall_dist=near_wall_dist,
                         w_wall=w_wall, wall_quantile=wall_quantile, opp_safe_dist=opp_safe_dist, w_opp=w_opp,
                         ego_crash_penalty=ego_crash_penalty, opp_crash_bonus=opp_crash_bonus).items():
            setattr(p, k, float(v))
        p.grace_steps_wall, p.grace_steps_opp = int(grace_steps_wall), int(grace_steps_opp)
        p.use_progress = 0 if progress is None else 1
        if progress is not None and progress.device is None:
            raise ValueError("progress must be a device CenterlineTrack")
        self.params = p
        self.progress = progress
        self.n_envs = int(n_envs)
        self.num_beams = int(num_beams)
        dev = torch.device(device if not isinstance(device, int) else f"cuda:{device}")
        if dev.type != "cuda" or not torch.cuda.is_available():
            raise _lib.F110Error("BatchedCenterlineReward runs on a HIP device only (no CPU path)")
        self.device = dev
        self.state = torch.zeros(self.n_envs, _lib.REWARD_STATE_BYTES, dtype=torch.uint8, device=dev)
        self.rewards = torch.zeros(self.n_envs, dtype=torch.float64, device=dev)

    def reset(self, env_mask=None):
        """reward_fn.reset() (rewards.py:255-257) for every env or the masked ones."""
        if env_mask is None:
            self.state.zero_()
        else:
            m = torch.as_tensor(env_mask, device=self.device).bool()
            self.state[m] = 0

    def __call__(self, obs, reset_mask=None):
        """Rewards [n_envs] float64 (device) for the flat observations
        [n_envs, obs_len] (float32, device).  Envs in ``reset_mask`` are reset
        instead and get 0 (an autoresetting vector env's reset observation)."""
        o = torch.as_tensor(obs, device=self.device)
        if o.dtype != torch.float32:
            o = o.to(torch.float32)
        o = o.reshape(self.n_envs, -1).contiguous()
        m = None
        if reset_mask is not None:
            m = torch.as_tensor(reset_mask, device=self.device).reshape(-1)
            m = m.view(torch.uint8) if m.dtype == torch.bool and m.is_contiguous() else m.to(torch.uint8).contiguous()
        self._keep = (o, m)
        s = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(self.L_lib.f110_reward(
            self.progress.handle if self.progress is not None else None, ctypes.byref(self.params),
            ctypes.c_void_p(o.data_ptr()), self.n_envs, o.shape[1], self.num_beams,
            ctypes.c_void_p(self.state.data_ptr()), ctypes.c_void_p(m.data_ptr()) if m is not None else None,
            ctypes.c_void_p(self.rewards.data_ptr()), ctypes.c_void_p(s)), "f110_reward")
        return self.rewards
