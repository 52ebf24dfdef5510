"""BatchSim: n_envs x n_agents F1TENTH cars stepped on one MI355X.

Thin Python owner of a libf110 context: device memory for inputs/outputs is
PyTorch-ROCm tensors; every per-step call enqueues one HIP kernel on the
current torch stream through the C ABI (include/f110.h).  Semantics are the
reference's Simulator.step / F110Env.step (base_classes.py:566-625,
f110_env.py:371-421) for every env at once.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .maps import TrackMap, load_map


@dataclass
class StepOut:
    obs: torch.Tensor          # [E, B + 4A] f32
    scans: torch.Tensor        # [E, A, B] f32
    collisions: torch.Tensor   # [E, A] u8
    terminated: torch.Tensor   # [E] u8
    was_reset: torch.Tensor    # [E] u8
    lap_times: torch.Tensor    # [E, A] f32
    lap_counts: torch.Tensor   # [E, A] f32
    sim_time: torch.Tensor     # [E] f64
    scans_f64: torch.Tensor = None  # [E, A, B] f64 (optional)


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class BatchSim:
    """Batched simulator on one device.

    Args mirror F110Env kwargs (f110_env.py:104-186) plus ``n_envs``.
    ``autoreset`` + ``spawn_poses`` [S, A, 3] enable device-side resets of
    terminated envs at their next step.
    """

    def __init__(self, track: TrackMap | str = "Spielberg_map", n_envs: int = 1, n_agents: int = 2,
                 params: dict | None = None, device: int | str | torch.device = 0, seed: int = 42,
                 timestep: float = 0.01, integrator: int = _lib.INTEGRATOR_RK4, ego_idx: int = 0,
                 lidar_dist: float = 0.0, num_beams: int = 1080, fov: float = 4.7, noise_std: float = 0.01,
                 autoreset: bool = False, spawn_poses: np.ndarray | None = None, env_offset: int = 0,
                 keep_f64_scans: bool = False, map_ext: str = ".png"):
        if isinstance(track, str):
            track = load_map(track, map_ext)
        self.track = track
        dev = torch.device(device if not isinstance(device, int) else f"cuda:{device}")
        if dev.type != "cuda":
            raise _lib.F110Error("BatchSim runs on a HIP device only (no CPU path)")
        if not torch.cuda.is_available():
            raise _lib.F110Error("no HIP device visible: libf110 has no CPU fallback")
        self.device = dev
        self.L = _lib.load()
        p = _lib.default_params()
        for k, v in (params or {}).items():
            if hasattr(p, k):
                setattr(p, k, float(v))
        self.params = p
        c = _lib.default_config()
        c.n_envs, c.n_agents, c.n_beams = int(n_envs), int(n_agents), int(num_beams)
        c.integrator, c.ego_idx, c.autoreset = int(integrator), int(ego_idx), int(bool(autoreset))
        c.fov, c.time_step, c.lidar_dist, c.noise_std = float(fov), float(timestep), float(lidar_dist), \
            float(noise_std)
        c.max_range = 30.0  # ScanSimulator2D default (laser_models.py:360); lidar_max only scales obs
        c.env_offset, c.seed = int(env_offset), int(seed) & 0xFFFFFFFFFFFFFFFF
        self.cfg = c
        self.E, self.A, self.B = c.n_envs, c.n_agents, c.n_beams
        k = np.ascontiguousarray(track.ensure_edt())
        origin = (ctypes.c_double * 3)(*track.origin)
        spawn = None
        n_spawn = 0
        if spawn_poses is not None:
            spawn = np.ascontiguousarray(spawn_poses, dtype=np.float64)
            if spawn.ndim != 3 or spawn.shape[1] != self.A or spawn.shape[2] != 3:
                raise ValueError("spawn_poses must be [S, n_agents, 3]")
            n_spawn = spawn.shape[0]
        self._spawn = spawn
        torch.cuda.set_device(dev)
        ctx = ctypes.c_void_p()
        _lib.check(self.L.f110_create(ctypes.byref(ctx), dev.index or 0, ctypes.byref(c), ctypes.byref(p),
                                      k.ctypes.data, track.height, track.width, track.resolution, origin,
                                      spawn.ctypes.data if spawn is not None else None, n_spawn), "f110_create")
        self.ctx = ctx
        self.reset_dtype = np.float64  # f110_set_reset_dtype: the context's default
        E, A, B = self.E, self.A, self.B
        kw = dict(device=dev)
        # obs rows padded to a 128-B multiple (1088 floats for A = 1, packed
        # 1088 already for A = 2): the ray kernel's 64-beam obs stores then
        # cover whole cache lines; out.obs is the [E, B + 4A] view
        self.obs_stride = (B + 4 * A + 31) // 32 * 32
        self._obs_buf = torch.empty(E, self.obs_stride, dtype=torch.float32, **kw)
        self.out = StepOut(
            obs=self._obs_buf[:, :B + 4 * A],
            scans=torch.empty(E, A, B, dtype=torch.float32, **kw),
            collisions=torch.zeros(E, A, dtype=torch.uint8, **kw),
            terminated=torch.zeros(E, dtype=torch.uint8, **kw),
            was_reset=torch.zeros(E, dtype=torch.uint8, **kw),
            lap_times=torch.zeros(E, A, dtype=torch.float32, **kw),
            lap_counts=torch.zeros(E, A, dtype=torch.float32, **kw),
            sim_time=torch.zeros(E, dtype=torch.float64, **kw),
            scans_f64=torch.empty(E, A, B, dtype=torch.float64, **kw) if keep_f64_scans else None,
        )
        self._outs = _lib.F110Outputs(
            obs=self.out.obs.data_ptr(), scans=self.out.scans.data_ptr(),
            scans_f64=self.out.scans_f64.data_ptr() if keep_f64_scans else None,
            collisions=self.out.collisions.data_ptr(), terminated=self.out.terminated.data_ptr(),
            was_reset=self.out.was_reset.data_ptr(), lap_times=self.out.lap_times.data_ptr(),
            lap_counts=self.out.lap_counts.data_ptr(), sim_time=self.out.sim_time.data_ptr(),
            obs_stride=self.obs_stride)
        self._outs_min = _lib.F110Outputs(
            obs=self.out.obs.data_ptr(), collisions=self.out.collisions.data_ptr(),
            terminated=self.out.terminated.data_ptr(), obs_stride=self.obs_stride)

    # ------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def reset(self, poses, env_mask=None) -> StepOut:
        """F110Env.reset for the envs in ``env_mask`` (all if None).
        poses: [E, A, 3] (or [A, 3] broadcast to every env)."""
        p = torch.as_tensor(poses, dtype=torch.float64, device=self.device)
        if p.dim() == 2:
            p = p.unsqueeze(0).expand(self.E, self.A, 3)
        if tuple(p.shape) != (self.E, self.A, 3):
            raise ValueError(f"poses must be [{self.E}, {self.A}, 3]; got {tuple(p.shape)} "
                             "(Number of poses for reset does not match number of agents.)")
        p = p.contiguous()
        m = None
        if env_mask is not None:
            m = torch.as_tensor(env_mask, device=self.device).to(torch.uint8).contiguous()
        self._keep = (p, m)
        _lib.check(self.L.f110_reset(self.ctx, _ptr(p), _ptr(m), ctypes.byref(self._outs), self._stream()),
                   "f110_reset")
        return self.out

    def step(self, actions, minimal_outputs: bool = False, obs_out=None) -> StepOut:
        """actions: [E, A, 2] (steer, velocity); float32 or float64 tensor/array
        (float64 keeps Simulator.step's full-precision control inputs).
        obs_out: a float32 [E, n_beams + 4A] tensor (unit column stride) that
        receives this step's observations instead of ``out.obs`` (which then
        keeps the previous ones): a trainer's own next_obs buffer, no copy."""
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype not in (torch.float32, torch.float64):
            a = a.to(torch.float32)
        if a.dim() == 2 and self.E == 1:
            a = a.unsqueeze(0)
        if tuple(a.shape) != (self.E, self.A, 2):
            raise ValueError(f"actions must be [{self.E}, {self.A}, 2]; got {tuple(a.shape)}")
        a = a.contiguous()
        self._keep_a = a
        outs = self._outs_min if minimal_outputs else self._outs
        if obs_out is not None:
            B = self.out.obs.shape[1]
            if (obs_out.dtype != torch.float32 or obs_out.device != self.device or tuple(obs_out.shape) != (self.E, B)
                    or obs_out.stride(1) != 1 or obs_out.stride(0) < B):
                raise ValueError(f"obs_out must be a float32 [{self.E}, {B}] tensor on {self.device}, unit column stride")
            o = _lib.F110Outputs()
            ctypes.pointer(o)[0] = outs
            o.obs, o.obs_stride = obs_out.data_ptr(), obs_out.stride(0)
            outs = o
        dt = _lib.F64 if a.dtype == torch.float64 else _lib.F32
        _lib.check(self.L.f110_step(self.ctx, _ptr(a), dt, ctypes.byref(outs), self._stream()), "f110_step")
        return self.out

    def step_n(self, actions, minimal_outputs: bool = False) -> StepOut:
        """n consecutive steps with resident actions [n, E, A, 2] (f110_step_n:
        n three-launch steps, no host work in between); the outputs hold the
        last step's values."""
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype not in (torch.float32, torch.float64):
            a = a.to(torch.float32)
        if a.dim() != 4 or tuple(a.shape[1:]) != (self.E, self.A, 2):
            raise ValueError(f"actions must be [n, {self.E}, {self.A}, 2]; got {tuple(a.shape)}")
        a = a.contiguous()
        self._keep_a = a
        outs = self._outs_min if minimal_outputs else self._outs
        dt = _lib.F64 if a.dtype == torch.float64 else _lib.F32
        _lib.check(self.L.f110_step_n(self.ctx, _ptr(a), dt, int(a.shape[0]), 0, ctypes.byref(outs), self._stream()),
                   "f110_step_n")
        return self.out

    def update_params(self, params: dict, agent_idx: int = -1):
        """Simulator.update_params (base_classes.py:527-546) for every env."""
        p = _lib.F110Params()
        ctypes.pointer(p)[0] = self.params
        for k, _ in p._fields_:
            if k in params:
                setattr(p, k, float(params[k]))
        _lib.check(self.L.f110_set_params(self.ctx, ctypes.byref(p), int(agent_idx), self._stream()),
                   "f110_set_params")

    def set_scan_noise(self, noise):
        """Caller-supplied scan noise for the following step/reset calls
        (f110_set_scan_noise): a device f64 tensor [E, B] that the caller
        refills before each call; ``None`` returns to the device stream."""
        if noise is None:
            self._noise = None
            _lib.check(self.L.f110_set_scan_noise(self.ctx, None), "f110_set_scan_noise")
            return
        if not (isinstance(noise, torch.Tensor) and noise.device == self.device and noise.dtype == torch.float64
                and tuple(noise.shape) == (self.E, self.B) and noise.is_contiguous()):
            raise ValueError(f"noise must be a contiguous float64 [{self.E}, {self.B}] tensor on {self.device}")
        self._noise = noise
        _lib.check(self.L.f110_set_scan_noise(self.ctx, _ptr(noise)), "f110_set_scan_noise")

    def get_state(self):
        """(state [7, E*A] f64, steer_buf [2, E*A] f64, steer_cnt [E*A] i32) — SoA."""
        EA = self.E * self.A
        st = torch.empty(7, EA, dtype=torch.float64, device=self.device)
        sb = torch.empty(2, EA, dtype=torch.float64, device=self.device)
        sc = torch.empty(EA, dtype=torch.int32, device=self.device)
        _lib.check(self.L.f110_get_state(self.ctx, _ptr(st), _ptr(sb), _ptr(sc), self._stream()), "f110_get_state")
        return st, sb, sc

    def lap_state(self):
        """(start_rot [2, E] f64, toggles [E, A] i32): F110Env's start_rot and
        toggle_list as the device holds them (f110_get_lap_state)."""
        rot = torch.empty(2, self.E, dtype=torch.float64, device=self.device)
        tog = torch.empty(self.E * self.A, dtype=torch.int32, device=self.device)
        _lib.check(self.L.f110_get_lap_state(self.ctx, _ptr(rot), _ptr(tog), self._stream()), "f110_get_lap_state")
        return rot, tog.reshape(self.E, self.A)

    def set_state(self, state=None, steer_buf=None, steer_cnt=None):
        EA = self.E * self.A
        st = None if state is None else torch.as_tensor(state, dtype=torch.float64, device=self.device).reshape(7, EA).contiguous()
        sb = None if steer_buf is None else torch.as_tensor(steer_buf, dtype=torch.float64, device=self.device).reshape(2, EA).contiguous()
        sc = None if steer_cnt is None else torch.as_tensor(steer_cnt, dtype=torch.int32, device=self.device).reshape(EA).contiguous()
        self._keep_s = (st, sb, sc)
        _lib.check(self.L.f110_set_state(self.ctx, _ptr(st), _ptr(sb), _ptr(sc), self._stream()), "f110_set_state")

    def agent_states(self) -> torch.Tensor:
        """[E, A, 7] f64 copy of the state (AoS view for consumers)."""
        st, _, _ = self.get_state()
        return st.t().reshape(self.E, self.A, 7)

    def scan_batch(self, poses, probe: bool = False):
        """ScanSimulator2D.scan with rng=None for arbitrary poses [M, 3]."""
        p = torch.as_tensor(poses, dtype=torch.float64, device=self.device).reshape(-1, 3).contiguous()
        M = p.shape[0]
        scans = torch.empty(M, self.B, dtype=torch.float64, device=self.device)
        look = torch.empty(M, self.B, dtype=torch.int32, device=self.device) if probe else None
        rc = torch.empty(M, self.B, 2, dtype=torch.int32, device=self.device) if probe else None
        _lib.check(self.L.f110_scan_batch(self.ctx, _ptr(p), M, _ptr(scans), _ptr(look), _ptr(rc), self._stream()),
                   "f110_scan_batch")
        return (scans, look, rc) if probe else scans

    def dynamics_batch(self, x, u) -> torch.Tensor:
        x = torch.as_tensor(x, dtype=torch.float64, device=self.device).reshape(-1, 7).contiguous()
        u = torch.as_tensor(u, dtype=torch.float64, device=self.device).reshape(-1, 2).contiguous()
        f = torch.empty_like(x)
        _lib.check(self.L.f110_dynamics_batch(self.ctx, _ptr(x), _ptr(u), _ptr(f), x.shape[0], self._stream()),
                   "f110_dynamics_batch")
        return f

    def dynamics_ks_batch(self, x, u) -> torch.Tensor:
        """vehicle_dynamics_ks (dynamic_models.py:90-121) for kinematic states [M, 5]."""
        x = torch.as_tensor(x, dtype=torch.float64, device=self.device).reshape(-1, 5).contiguous()
        u = torch.as_tensor(u, dtype=torch.float64, device=self.device).reshape(-1, 2).contiguous()
        f = torch.empty_like(x)
        _lib.check(self.L.f110_dynamics_ks_batch(self.ctx, _ptr(x), _ptr(u), _ptr(f), x.shape[0], self._stream()),
                   "f110_dynamics_ks_batch")
        return f

    def read_counters(self):
        lk, rays = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(self.L.f110_read_counters(self.ctx, ctypes.byref(lk), ctypes.byref(rays), self._stream()),
                   "f110_read_counters")
        return lk.value, rays.value

    def set_simt(self, on: bool = True):
        """Counting on / off (f110_debug_set_simt; off by default): the fixed-point ray loops count their
        lane slots, and k_rays_fxs (the default ray kernel) counts lookups and rays only while it is on."""
        _lib.check(self.L.f110_debug_set_simt(self.ctx, int(bool(on))), "f110_debug_set_simt")

    def set_handoff_check(self, mode: int):
        """Hand-off mask check (f110_debug_set_handoff_check): bit 0 NaN-poisons the hand-off buffer
        before each ray launch and counts k_post_multi's reads outside the mask (read_counter(6));
        bit 1 turns the mask off (every chunk stored).  Debug only."""
        _lib.check(self.L.f110_debug_set_handoff_check(self.ctx, int(mode)), "f110_debug_set_handoff_check")

    def read_simt(self):
        """(loop lookups, lane slots) of the fixed-point ray loops since the
        last counter reset (f110_debug_read_simt); their ratio is the loop's SIMT
        efficiency, None when the ray kernel keeps no lane-slot count."""
        lk, sl = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(self.L.f110_debug_read_simt(self.ctx, ctypes.byref(lk), ctypes.byref(sl), self._stream()),
                   "f110_debug_read_simt")
        return lk.value, sl.value

    def read_counter(self, idx: int) -> int:
        """Diagnostic counter idx summed over its lines (f110_debug_read_counter)."""
        v = ctypes.c_uint64()
        _lib.check(self.L.f110_debug_read_counter(self.ctx, int(idx), ctypes.byref(v), self._stream()), "f110_debug_read_counter")
        return v.value

    def reset_counters(self):
        _lib.check(self.L.f110_reset_counters(self.ctx, self._stream()), "f110_reset_counters")

    def profile_begin(self, max_steps: int):
        """Time each kernel of the next max_steps step/reset calls (HIP events)."""
        _lib.check(self.L.f110_profile_begin(self.ctx, int(max_steps)), "f110_profile_begin")

    def profile_stamps(self, ref_event, max_steps: int = 4096) -> np.ndarray:
        """Before profile_end: [steps, 6] ms after ref_event (a torch.cuda.Event with timing, recorded
        before the profiled steps) of each step's k_agents / ray kernel / k_post begin and end
        (f110_debug_profile_stamps)."""
        n = int(max_steps)
        buf = np.zeros((n, 6), np.float64)
        got = ctypes.c_int32()
        _lib.check(self.L.f110_debug_profile_stamps(self.ctx, ctypes.c_void_p(ref_event.cuda_event), buf.ctypes.data,
                                                    n, ctypes.byref(got)), "f110_debug_profile_stamps")
        return buf[:got.value]

    def profile_end(self) -> dict:
        ms = (ctypes.c_double * 3)()
        n = ctypes.c_int32()
        _lib.check(self.L.f110_profile_end(self.ctx, ms, ctypes.byref(n)), "f110_profile_end")
        k = max(n.value, 1)
        return {"steps": n.value, "k_agents_ms": ms[0] / k, "k_rays_ms": ms[1] / k, "k_post_ms": ms[2] / k}

    def set_reset_dtype(self, dtype):
        """F110Env.reset semantics for the following resets and autoresets
        (f110_set_reset_dtype): float32 options round the poses to float32
        and give start_rot NumPy's float32 cos / sin (f110_env.py:448-451)."""
        try:  # a NumPy dtype / type, or a dtype name
            f32 = np.dtype(dtype) == np.float32
        except TypeError:  # a torch dtype
            f32 = np.dtype(str(dtype).replace("torch.", "")) == np.float32
        _lib.check(self.L.f110_set_reset_dtype(self.ctx, _lib.F32 if f32 else _lib.F64), "f110_set_reset_dtype")
        self.reset_dtype = np.float32 if f32 else np.float64

    @property
    def ray_kernel(self) -> int:
        """The ray kernel this context launches (f110_debug_ray_kernel: 3 = the fixed-point kernels)."""
        return _lib.check(self.L.f110_debug_ray_kernel(self.ctx), "f110_debug_ray_kernel")

    @property
    def ray_lanes(self) -> int:
        """Rays per lane of the fixed-point ray kernel (f110_debug_ray_lanes: 1 = k_rays_fx, 2 = k_rays_fxn / fxs)."""
        return _lib.check(self.L.f110_debug_ray_lanes(self.ctx), "f110_debug_ray_lanes")

    def set_ray_lanes(self, n: int):
        """Rays per lane, 1 or 2 (f110_debug_set_ray_lanes; before the first reset / step)."""
        _lib.check(self.L.f110_debug_set_ray_lanes(self.ctx, int(n)), "f110_debug_set_ray_lanes")

    def set_ray_refill(self, waves: int):
        """k_rays_fxs's waves per car (0: k_rays_fxn), with the padded EDT and heavy-first off
        (f110_debug_set_ray_refill)."""
        _lib.check(self.L.f110_debug_set_ray_refill(self.ctx, int(waves)), "f110_debug_set_ray_refill")

    @property
    def ray_refill(self) -> int:
        """k_rays_fxs's waves per car for unmasked steps (f110_debug_ray_refill), 0 when k_rays_fxn /
        k_rays_fx trace this context's rays."""
        return _lib.check(self.L.f110_debug_ray_refill(self.ctx), "f110_debug_ray_refill")

    def disable_heavy_first(self):
        """Heavy-first ray dispatch off for good (f110_debug_disable_heavy_first; results unchanged)."""
        _lib.check(self.L.f110_debug_disable_heavy_first(self.ctx), "f110_debug_disable_heavy_first")

    def close(self):
        if getattr(self, "ctx", None):
            torch.cuda.synchronize(self.device)
            self.L.f110_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
