"""ctypes binding of libf110.so (the C ABI in include/f110.h).

Loads the in-tree library; there is no CPU fallback: if the library or a
gfx950 device is missing, the calls fail loudly with the library's error.
"""
from __future__ import annotations

import ctypes
import os

from . import _build

_P = ctypes.c_void_p
_D = ctypes.POINTER(ctypes.c_double)


class F110Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in
                ("mu", "C_Sf", "C_Sr", "lf", "lr", "h", "m", "I", "s_min", "s_max", "sv_min", "sv_max",
                 "v_switch", "a_max", "v_min", "v_max", "width", "length", "lidar_max")]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class F110Config(ctypes.Structure):
    _fields_ = [("n_envs", ctypes.c_int32), ("n_agents", ctypes.c_int32), ("n_beams", ctypes.c_int32),
                ("theta_dis", ctypes.c_int32), ("integrator", ctypes.c_int32), ("ego_idx", ctypes.c_int32),
                ("autoreset", ctypes.c_int32), ("_pad", ctypes.c_int32), ("fov", ctypes.c_double),
                ("eps", ctypes.c_double), ("max_range", ctypes.c_double), ("time_step", ctypes.c_double),
                ("lidar_dist", ctypes.c_double), ("ttc_thresh", ctypes.c_double),
                ("noise_std", ctypes.c_double), ("env_offset", ctypes.c_int64), ("seed", ctypes.c_uint64)]


class F110Outputs(ctypes.Structure):
    _fields_ = [("obs", _P), ("scans", _P), ("scans_f64", _P), ("collisions", _P), ("terminated", _P),
                ("was_reset", _P), ("lap_times", _P), ("lap_counts", _P), ("sim_time", _P),
                ("obs_stride", ctypes.c_int64)]


class F110RewardParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in
                ("dt", "w_prog", "forward_sign", "alive_bonus", "w_rel_lead", "lead_clip", "w_lat", "lat_cap",
                 "default_half_width", "lidar_max", "near_wall_dist", "w_wall", "wall_quantile", "opp_safe_dist",
                 "w_opp", "ego_crash_penalty", "opp_crash_bonus", "beta")] + \
               [(n, ctypes.c_int32) for n in ("grace_steps_wall", "grace_steps_opp", "auto_flip_steps",
                                             "use_progress")]


class F110GemmOp(ctypes.Structure):  # f110_gemm_op
    _fields_ = [(n, _P) for n in ("A", "B", "bias", "amask", "omask", "x2", "w2", "C")] + \
               [(n, ctypes.c_int32) for n in ("N", "K", "lda", "ldb", "ldc", "ldx2", "ldw2", "nx2", "relu", "nn")]


class F110WgradOp(ctypes.Structure):  # f110_wgrad_op
    _fields_ = [(n, _P) for n in ("G", "gmask", "X", "dW", "db")] + \
               [(n, ctypes.c_int32) for n in ("N", "KX", "ldg", "ldx", "ldw")]


REWARD_STATE_BYTES = 8 * 12 + 4 * 4   # f110_reward_state

ABI_VERSION = 3  # include/f110.h F110_ABI_VERSION
F32 = 0
F64 = 1
INTEGRATOR_RK4 = 1
INTEGRATOR_EULER = 2

EXPORTS = [
    "f110_abi_version", "f110_last_error", "f110_default_params", "f110_default_config", "f110_edt_k",
    "f110_create", "f110_destroy", "f110_reset", "f110_step", "f110_get_state", "f110_set_state",
    "f110_scan_batch", "f110_dynamics_batch", "f110_read_counters", "f110_reset_counters", "f110_debug_read_simt", "f110_debug_set_simt", "f110_debug_set_handoff_check", "f110_debug_profile_stamps", "f110_host_beam_runs_agree", "f110_host_sincos_fast", "f110_host_tan_cos_fast",
    "f110_profile_begin", "f110_profile_end", "f110_host_tables", "f110_host_beam_indices",
    "f110_set_scan_noise", "f110_set_params", "f110_host_cell_index", "f110_gap_follow",
    "f110_host_window_ranges", "f110_track_create", "f110_track_destroy", "f110_track_arrays",
    "f110_default_reward_params", "f110_reward", "f110_replay_create", "f110_replay_destroy", "f110_replay_add", "f110_replay_add_env",
    "f110_replay_sample", "f110_replay_update_priorities", "f110_replay_length", "f110_replay_arrays",
    "f110_debug_wave_trace", "f110_debug_set_ray_gate", "f110_debug_disable_heavy_first", "f110_debug_ray_kernel", "f110_debug_ray_lanes", "f110_debug_ray_refill", "f110_debug_set_ray_refill", "f110_debug_read_counter", "f110_step_n", "f110_debug_set_ray_lanes", "f110_set_reset_dtype", "f110_set_device_share", "f110_host_np_sincosf", "f110_host_sincos", "f110_host_sincos_series", "f110_host_map_table", "f110_get_lap_state",
    "f110_dynamics_ks_batch", "f110_collision_batch", "f110_collision_multiple", "f110_adam_step", "f110_ddpg_scratch_floats", "f110_ddpg_actor_head", "f110_ddpg_actor_explore",
    "f110_ddpg_actor_head_bwd", "f110_ddpg_td_target", "f110_ddpg_critic_loss", "f110_ddpg_critic_loss_bwd",
    "f110_ddpg_q_mean", "f110_ddpg_q_mean_bwd", "f110_ddpg_relu_bwd_scratch_floats", "f110_ddpg_relu_bwd",
    "f110_learner_gemm", "f110_learner_wgrad_scratch_floats", "f110_learner_wgrad", "f110_learner_wgrad_loss",
    "f110_ddpg_critic_step", "f110_ddpg_q_mean_step", "f110_ddpg_row_blocks",
]

_lib = None


class F110Error(RuntimeError):
    pass


class _Missing:
    """An entry point an older A/B build (F110_LIB) does not export."""

    def __init__(self, name):
        self.name, self.argtypes, self.restype = name, None, None

    def __call__(self, *a):
        raise F110Error(f"{self.name}: not exported by this (alternate) build")


def lib_path() -> str:
    return _build.LIB


def load(build_if_missing: bool = True):
    """Load libf110.so (building it with hipcc if it is missing/stale)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("F110_LIB") or _build.LIB  # F110_LIB: an alternate build (A/B runs)
    if build_if_missing and path == _build.LIB:
        try:
            _build.build()
        except Exception as exc:  # pragma: no cover - toolchain missing
            if not os.path.exists(path):
                raise F110Error(f"libf110.so is missing and could not be built: {exc}") from exc
    if not os.path.exists(path):
        raise F110Error(f"libf110.so not found at {path}; run f110_gymnasium_ros2_jazzy_amd._build.build()")
    try:  # share torch's HIP runtime (same SONAME) when torch is present
        import torch  # noqa: F401
    except Exception:
        pass
    L = ctypes.CDLL(path)
    alternate = path != _build.LIB
    if alternate:  # an older build for A/B (ABI 2): its diagnostics under their pre-f110_debug_ names
        for name in EXPORTS:
            old = name.replace("f110_debug_", "f110_")
            if name.startswith("f110_debug_") and not hasattr(L, name) and hasattr(L, old):
                setattr(L, name, getattr(L, old))
            elif not hasattr(L, name):  # newer than that build: fails when called
                setattr(L, name, _Missing(name))
    i32, i64, u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    L.f110_abi_version.restype = ctypes.c_int
    L.f110_last_error.restype = ctypes.c_char_p
    L.f110_default_params.argtypes = [ctypes.POINTER(F110Params)]
    L.f110_default_config.argtypes = [ctypes.POINTER(F110Config)]
    L.f110_edt_k.argtypes = [_P, i32, i32, _P]
    L.f110_create.argtypes = [ctypes.POINTER(_P), i32, ctypes.POINTER(F110Config), ctypes.POINTER(F110Params),
                              _P, i32, i32, ctypes.c_double, _D, _P, i32]
    L.f110_destroy.argtypes = [_P]
    L.f110_reset.argtypes = [_P, _P, _P, ctypes.POINTER(F110Outputs), _P]
    L.f110_step.argtypes = [_P, _P, i32, ctypes.POINTER(F110Outputs), _P]
    L.f110_get_state.argtypes = [_P, _P, _P, _P, _P]
    L.f110_set_state.argtypes = [_P, _P, _P, _P, _P]
    L.f110_scan_batch.argtypes = [_P, _P, i64, _P, _P, _P, _P]
    L.f110_dynamics_batch.argtypes = [_P, _P, _P, _P, i64, _P]
    L.f110_dynamics_ks_batch.argtypes = [_P, _P, _P, _P, i64, _P]
    L.f110_collision_batch.argtypes = [_P, _P, i64, _P, _P]
    L.f110_collision_multiple.argtypes = [_P, i64, ctypes.c_int32, _P, _P, _P]
    L.f110_read_counters.argtypes = [_P, ctypes.POINTER(u64), ctypes.POINTER(u64), _P]
    L.f110_reset_counters.argtypes = [_P, _P]
    L.f110_debug_read_simt.argtypes = [_P, ctypes.POINTER(u64), ctypes.POINTER(u64), _P]
    L.f110_debug_set_simt.argtypes = [_P, ctypes.c_int32]
    L.f110_debug_set_handoff_check.argtypes = [_P, ctypes.c_int32]
    L.f110_host_beam_runs_agree.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int32, ctypes.c_int32]
    L.f110_host_sincos_fast.argtypes = [_P, i64, _P, _P, _P]
    L.f110_host_tan_cos_fast.argtypes = [_P, i64, _P, _P, _P, _P]
    L.f110_debug_profile_stamps.argtypes = [_P, _P, _P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
    L.f110_set_scan_noise.argtypes = [_P, _P]
    L.f110_host_window_ranges.argtypes = [ctypes.c_double, ctypes.c_double, i32, ctypes.c_double, ctypes.c_double,
                                          _P]
    L.f110_host_window_ranges.restype = None
    L.f110_track_create.argtypes = [ctypes.POINTER(_P), i32, _P, _P, _P, i32, i32]
    L.f110_track_destroy.argtypes = [_P]
    L.f110_track_arrays.argtypes = [_P, _P, _P, _P, _P]
    L.f110_track_arrays.restype = ctypes.c_double
    L.f110_default_reward_params.argtypes = [ctypes.POINTER(F110RewardParams)]
    L.f110_default_reward_params.restype = None
    L.f110_reward.argtypes = [_P, ctypes.POINTER(F110RewardParams), _P, i64, i32, i32, _P, _P, _P, _P]
    L.f110_gap_follow.argtypes = [_P, i64, i64, i32, ctypes.c_double, ctypes.c_double, _P, i64, _P, _P]
    L.f110_host_cell_index.argtypes = [i32, i32, ctypes.c_double, _D, _P, i64, _P]
    L.f110_set_params.argtypes = [_P, ctypes.POINTER(F110Params), i32, _P]
    L.f110_profile_begin.argtypes = [_P, i32]
    L.f110_profile_end.argtypes = [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32)]
    L.f110_host_tables.argtypes = [i32, i32, ctypes.c_double, ctypes.POINTER(F110Params), _P, _P, _P, _P, _P]
    L.f110_host_beam_indices.argtypes = [ctypes.c_double, ctypes.c_double, i32, i32, _P]
    L.f110_host_beam_indices.restype = ctypes.c_int
    L.f110_replay_create.argtypes = [ctypes.POINTER(_P), i32, i64, i32, i32, i32, i64, ctypes.c_double,
                                     ctypes.c_double, u64]
    L.f110_replay_destroy.argtypes = [_P]
    L.f110_replay_add.argtypes = [_P, _P, i64, _P, i64, _P, _P, i64, _P, _P, _P, i64, _P]
    L.f110_replay_add_env.argtypes = [_P, _P, i64, _P, i64, _P, _P, i64, _P, _P, i64, _P]
    L.f110_replay_sample.argtypes = [_P, i32, ctypes.c_double, _P, _P, _P, _P, _P, _P, _P, _P]
    L.f110_replay_update_priorities.argtypes = [_P, _P, _P, i64, i32, ctypes.c_float, _P]
    L.f110_replay_length.argtypes = [_P, ctypes.POINTER(i64), ctypes.POINTER(i64), _P]
    L.f110_replay_arrays.argtypes = [_P] + [ctypes.POINTER(_P)] * 6
    L.f110_debug_wave_trace.argtypes = [_P, i32, _P, i64, ctypes.POINTER(i64), _P]
    L.f110_debug_set_ray_gate.argtypes = [_P, _P, _P]
    L.f110_debug_disable_heavy_first.argtypes = [_P]
    L.f110_debug_ray_kernel.argtypes = [_P]
    L.f110_debug_ray_lanes.argtypes = [_P]
    L.f110_debug_ray_refill.argtypes = [_P]
    L.f110_debug_set_ray_refill.argtypes = [_P, ctypes.c_int32]
    L.f110_step_n.argtypes = [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, _P, _P]
    L.f110_debug_read_counter.argtypes = [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64), _P]
    L.f110_debug_set_ray_lanes.argtypes = [_P, ctypes.c_int32]
    if hasattr(L, "f110_set_device_share") or not alternate:
        L.f110_set_device_share.argtypes = [_P, i64, i32]
    L.f110_set_reset_dtype.argtypes = [_P, ctypes.c_int32]
    L.f110_get_lap_state.argtypes = [_P, _P, _P, _P]
    L.f110_host_np_sincosf.argtypes = [_P, i64, ctypes.c_int32, _P]
    L.f110_host_np_sincosf.restype = None
    L.f110_host_sincos.argtypes = [_P, i64, _P, _P]
    L.f110_host_sincos.restype = None
    L.f110_host_sincos_series.argtypes = [_P, i64, _P, _P]
    L.f110_host_sincos_series.restype = None
    L.f110_host_map_table.argtypes = [_P, i32, i32, ctypes.c_double, i32, i32, _P, i64, _P]
    L.f110_host_map_table.restype = ctypes.c_int64
    L.f110_adam_step.argtypes = [_P, _P, _P, _P, i64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, _P, _P, ctypes.c_double, _P]
    f32 = ctypes.c_float
    L.f110_ddpg_scratch_floats.argtypes = [i32, i32, i32]
    L.f110_ddpg_actor_head.argtypes = [_P] * 5 + [i32] * 3 + [_P] * 3
    L.f110_ddpg_actor_explore.argtypes = [_P] * 5 + [i32] * 3 + [_P, _P, ctypes.c_double, ctypes.c_double, _P, _P,
                                                                  ctypes.c_uint64, _P, i64, _P]
    L.f110_ddpg_actor_head_bwd.argtypes = [_P] * 5 + [i32] * 3 + [_P] * 6
    L.f110_ddpg_td_target.argtypes = [_P] * 5 + [f32, i32, i32, _P, _P]
    L.f110_ddpg_critic_loss.argtypes = [_P] * 5 + [i32] * 2 + [_P] * 4
    L.f110_ddpg_critic_loss_bwd.argtypes = [_P] * 5 + [i32] * 2 + [_P] * 6
    L.f110_ddpg_q_mean.argtypes = [_P] * 3 + [f32, i32, i32] + [_P] * 3
    L.f110_ddpg_q_mean_bwd.argtypes = [_P] * 3 + [f32, i32, i32] + [_P] * 6
    L.f110_ddpg_relu_bwd_scratch_floats.argtypes = [i32, i32]
    L.f110_ddpg_relu_bwd.argtypes = [_P, _P, i32, i32, _P, _P, _P, _P]
    L.f110_learner_gemm.argtypes = [ctypes.POINTER(F110GemmOp), i32, i32, _P]
    L.f110_learner_wgrad_scratch_floats.argtypes = [ctypes.POINTER(F110WgradOp), i32, i32]
    L.f110_learner_wgrad.argtypes = [ctypes.POINTER(F110WgradOp), i32, i32, _P, _P]
    L.f110_learner_wgrad_loss.argtypes = [ctypes.POINTER(F110WgradOp), i32, i32, _P, _P, i32, f32, _P, _P]
    L.f110_ddpg_critic_step.argtypes = [_P] * 5 + [f32] + [_P] * 5 + [i32, i32] + [_P] * 6
    L.f110_ddpg_q_mean_step.argtypes = [_P] * 4 + [f32, i32, i32] + [_P] * 4
    L.f110_ddpg_row_blocks.argtypes = [i32]
    L.f110_ddpg_row_blocks.restype = i32
    for name in EXPORTS:
        if alternate and not hasattr(L, name):
            continue
        if name not in ("f110_abi_version", "f110_last_error", "f110_default_params", "f110_default_config",
                        "f110_host_np_sincosf", "f110_host_sincos", "f110_host_sincos_series",
                        "f110_host_tables", "f110_host_window_ranges", "f110_track_arrays",
                        "f110_default_reward_params", "f110_ddpg_scratch_floats",
                        "f110_ddpg_relu_bwd_scratch_floats", "f110_learner_wgrad_scratch_floats"):
            getattr(L, name).restype = ctypes.c_int
    L.f110_ddpg_scratch_floats.restype = i64
    L.f110_ddpg_relu_bwd_scratch_floats.restype = i64
    L.f110_learner_wgrad_scratch_floats.restype = i64
    if L.f110_abi_version() != ABI_VERSION and not (alternate and L.f110_abi_version() == 2):
        raise F110Error(f"libf110.so ABI version mismatch ({L.f110_abi_version()} != {ABI_VERSION})")
    _lib = L
    return L


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        msg = load().f110_last_error()
        raise F110Error(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


def default_params() -> F110Params:
    p = F110Params()
    load().f110_default_params(ctypes.byref(p))
    return p


def default_config() -> F110Config:
    c = F110Config()
    load().f110_default_config(ctypes.byref(c))
    return c
