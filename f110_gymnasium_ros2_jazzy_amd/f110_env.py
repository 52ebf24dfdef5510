"""F110Env: drop-in for f110_gym.envs.F110Env (f110_env.py:55-602) on MI355X.

Same constructor kwargs and defaults (f110_env.py:104-186), same
``reset(seed, options=poses) -> (obs, info)`` and
``step(action) -> (obs, reward, terminated, truncated, info)`` contract, the
same 1088-float flat observation, the same ``info`` keys, ``timestep``
attribute and ``close()``, so rl_training/train_ddpg.py runs unchanged.

The physics + lidar + collision step runs on the GPU (one env of a
BatchSim), and so does the reference's lap bookkeeping (_check_done,
f110_env.py:310-352): the device epilogue (k_post_*'s env_epilogue) keeps the
start poses, start_rot, toggles, lap times / counts and terminated, with the
reference's dtype behaviour for float32 ``options`` (f110_set_reset_dtype:
float32 poses and NumPy's float32 start_rot).  The facade reads them back;
there is no second (host) implementation of the lap logic.

Scan noise is the reference's own stream: every RaceCar re-creates
``np.random.default_rng(seed)`` at reset and ScanSimulator2D.scan adds
``rng.normal(0, 0.01, num_beams)`` after the clamp (base_classes.py:119,204,
laser_models.py:450-452).  All cars share the seed, so they draw the same
vector; the facade draws it once per step on the host and hands it to the
device (f110_set_scan_noise), so noisy trajectories match the reference.
``noise_std`` (extension kwarg) scales it; 0 turns it off.  The batched
F110VectorEnv uses the device Philox stream instead (same law).

Differences, by design:
  * render() is not provided (visualisation is out of scope; the DDPG
    script never calls it).
"""
from __future__ import annotations

import os

import numpy as np

try:  # gymnasium is optional: the env works without it (no registry)
    import gymnasium as _gym
    from gymnasium import spaces as _spaces
    _EnvBase = _gym.Env
except Exception:  # pragma: no cover - exercised where gymnasium is absent
    _gym = None
    _spaces = None
    _EnvBase = object

from . import _lib

DEFAULT_PARAMS = {'mu': 1.0489, 'C_Sf': 4.718, 'C_Sr': 5.4562, 'lf': 0.15875, 'lr': 0.17145, 'h': 0.074,
                  'm': 3.74, 'I': 0.04712, 's_min': -0.4189, 's_max': 0.4189, 'sv_min': -3.2, 'sv_max': 3.2,
                  'v_switch': 7.319, 'a_max': 9.51, 'v_min': 0.00000001, 'v_max': 20.0, 'width': 0.31,
                  'length': 0.58, 'lidar_max': 30.0}


class Integrator:
    """Mirror of base_classes.Integrator (base_classes.py:40-42)."""
    RK4 = _lib.INTEGRATOR_RK4
    Euler = _lib.INTEGRATOR_EULER


class _Box:
    """Minimal stand-in for gymnasium.spaces.Box when gymnasium is absent."""

    def __init__(self, low, high, dtype=np.float32):
        self.low = np.asarray(low, dtype)
        self.high = np.asarray(high, dtype)
        self.shape = self.low.shape
        self.dtype = np.dtype(dtype)

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        return rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))


def _box(low, high):
    if _spaces is not None:
        return _spaces.Box(low=low, high=high, dtype=np.float32)
    return _Box(low, high, np.float32)


def _integrator_code(v):
    if isinstance(v, (int, np.integer)):
        return int(v)
    name = getattr(v, "name", str(v))
    if "RK4" in name:
        return _lib.INTEGRATOR_RK4
    if "Euler" in name:
        return _lib.INTEGRATOR_EULER
    raise SyntaxError(f"Invalid Integrator Specified. Provided {name}. Please choose RK4 or Euler")


class F110Env(_EnvBase):
    metadata = {'render_modes': ['human', 'human_fast'], 'render_fps': 30}

    def __init__(self, **kwargs):
        from .maps import load_map
        from .sim import BatchSim

        self.conf = kwargs.get('conf')
        self.seed = kwargs.get('seed', 42)
        if 'map_dir' in kwargs and 'map' in kwargs:
            self.map_dir = kwargs['map_dir']
            self.map_name = kwargs['map']
            self.map_path = self.map_dir + self.map_name + '.yaml'
        else:
            # the reference falls back to a bundled 'vegas' map; ours bundles Spielberg
            self.map_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'maps') + os.sep
            self.map_name = kwargs.get('map', 'Spielberg_map')
            self.map_path = self.map_dir + self.map_name + '.yaml'
        self.map_ext = kwargs.get('map_ext', '.png')
        self.params = dict(kwargs.get('params', DEFAULT_PARAMS))
        self.num_agents = kwargs.get('num_agents', 2)
        self.timestep = kwargs.get('timestep', 0.01)
        self.ego_idx = kwargs.get('ego_idx', 0)
        self.integrator = kwargs.get('integrator', Integrator.RK4)
        self.lidar_dist = kwargs.get('lidar_dist', 0.0)
        self.render_mode = kwargs.get('render_mode')
        self.noise_std = float(kwargs.get('noise_std', 0.01))
        device = kwargs.get('device', 0)

        self.start_thresh = 0.1
        self.poses_x, self.poses_y, self.poses_theta = [], [], []
        self.collisions = np.zeros((self.num_agents,))
        self.lidar_max = self.params["lidar_max"]
        self.near_start = True
        self.num_toggles = 0
        self.lap_times = np.zeros((self.num_agents,))
        self.lap_counts = np.zeros((self.num_agents,))
        self.current_time = 0.0
        self.near_starts = np.array([True] * self.num_agents)
        self.toggle_list = np.zeros((self.num_agents,))
        self.start_xs = np.zeros((self.num_agents,))
        self.start_ys = np.zeros((self.num_agents,))
        self.start_thetas = np.zeros((self.num_agents,))
        self.start_rot = np.eye(2)

        self.track = load_map(self.map_path, self.map_ext)
        self.sim = BatchSim(self.track, n_envs=1, n_agents=self.num_agents, params=self.params, device=device,
                            seed=self.seed, timestep=self.timestep, integrator=_integrator_code(self.integrator),
                            ego_idx=self.ego_idx, lidar_dist=self.lidar_dist, noise_std=self.noise_std,
                            keep_f64_scans=True)
        self._scan_rng = None
        self._agent_params = [None] * self.num_agents
        self._noise = None
        if self.noise_std > 0.0:
            import torch
            self._noise = torch.zeros(1, self.sim.B, dtype=torch.float64, device=self.sim.device)
            self.sim.set_scan_noise(self._noise)

        self.resolution = self.track.resolution
        self.x0, self.y0 = self.track.origin[0], self.track.origin[1]
        self.x_min, self.x_max, self.y_min, self.y_max = self.track.bounds
        low = np.array([self.params['s_min'], self.params['v_min']], dtype=np.float32)
        high = np.array([self.params['s_max'], self.params['v_max']], dtype=np.float32)
        self.action_space = _box(np.tile(low, (self.num_agents, 1)), np.tile(high, (self.num_agents, 1)))
        B = self.sim.B
        olow = np.array([0.0] * B + [self.x_min, self.y_min, -np.pi, 0.0] * self.num_agents, dtype=np.float32)
        ohigh = np.array([1.0] * B + [self.x_max, self.y_max, np.pi, 1.0] * self.num_agents, dtype=np.float32)
        self.observation_space = _box(olow, ohigh)
        self.render_obs = None

    # ------------------------------------------------------------------
    def _check_done(self, out):
        """Lap toggles + ego collision (f110_env.py:310-352) as the device's step epilogue computed
        them: terminated, lap times / counts (f110_outputs) and the toggles (f110_get_lap_state).
        The reference's attributes mirror them (toggle_list and lap_counts as float64, lap_times
        as the float32 values the reference reports in its info)."""
        _, tog = self.sim.lap_state()
        self.toggle_list = tog[0].cpu().numpy().astype(np.float64)
        self.lap_counts = out.lap_counts[0].cpu().numpy().astype(np.float64)
        self.lap_times = out.lap_times[0].cpu().numpy().astype(np.float64)
        return bool(out.terminated[0].item()), self.toggle_list >= 4

    def _obs_dict(self, out):
        """Simulator.step's observation dict (base_classes.py:607-625) from device outputs."""
        st = self.sim.agent_states()[0].cpu().numpy()          # [A, 7] f64
        scans64 = out.scans_f64[0].cpu().numpy()               # [A, B] f64
        cols = out.collisions[0].cpu().numpy().astype(np.float64)
        return {
            'ego_idx': self.ego_idx,
            'scans': [scans64[i] for i in range(self.num_agents)],
            'poses_x': [st[i, 0] for i in range(self.num_agents)],
            'poses_y': [st[i, 1] for i in range(self.num_agents)],
            'poses_theta': [st[i, 4] for i in range(self.num_agents)],
            'linear_vels_x': [st[i, 3] for i in range(self.num_agents)],
            'linear_vels_y': [0. for _ in range(self.num_agents)],
            'ang_vels_z': [st[i, 5] for i in range(self.num_agents)],
            'collisions': cols,
        }, out.obs[0].cpu().numpy()

    def _finish_step(self, out):
        obs_dict, flat = self._obs_dict(out)
        terminated, toggle_list = self._check_done(out)
        obs_dict['lap_times'] = self.lap_times.astype(np.float32)
        obs_dict['lap_counts'] = self.lap_counts.astype(np.float32)
        F110Env.current_obs = obs_dict
        self.render_obs = {k: obs_dict[k] for k in ('ego_idx', 'poses_x', 'poses_y', 'poses_theta', 'lap_times',
                                                    'lap_counts', 'scans')}
        reward = self.timestep
        self.current_time = self.current_time + self.timestep
        self.poses_x = obs_dict['poses_x']
        self.poses_y = obs_dict['poses_y']
        self.poses_theta = obs_dict['poses_theta']
        self.collisions = obs_dict['collisions']
        info = self._build_info(obs_dict)
        info["checkpoint_done"] = toggle_list
        return flat, reward, terminated, False, info

    def _build_info(self, obs_dict):
        return {
            "ego_idx": int(obs_dict["ego_idx"]),
            "poses_x": np.asarray(obs_dict["poses_x"], dtype=np.float32),
            "poses_y": np.asarray(obs_dict["poses_y"], dtype=np.float32),
            "poses_theta": np.asarray(obs_dict["poses_theta"], dtype=np.float32),
            "linear_vels_x": np.asarray(obs_dict["linear_vels_x"], dtype=np.float32),
            "linear_vels_y": np.asarray(obs_dict["linear_vels_y"], dtype=np.float32),
            "ang_vels_z": np.asarray(obs_dict["ang_vels_z"], dtype=np.float32),
            "collisions": np.asarray(obs_dict["collisions"], dtype=np.int8),
            "lap_times": self.lap_times.astype(np.float32),
            "lap_counts": self.lap_counts.astype(np.float32),
            "scans": [np.asarray(s, dtype=np.float32) for s in obs_dict["scans"]],
            "checkpoint_done": getattr(self, "toggle_list", None),
            "time": float(self.current_time),
        }

    def _draw_noise(self):
        """This step's ScanSimulator2D.scan noise (laser_models.py:450-452)."""
        if self._noise is not None:
            import torch
            n = self._scan_rng.normal(0., self.noise_std, size=self.sim.B)
            self._noise.copy_(torch.from_numpy(n).view(1, -1))

    # ------------------------------------------------------------------
    def step(self, action):
        """F110Env.step (f110_env.py:371-421); action [num_agents, 2] (steer, velocity)."""
        if self._noise is not None and self._scan_rng is None:
            raise RuntimeError("call reset() before step()")  # the reference's cars lack scan_rng too
        a = np.asarray(action)
        if a.dtype not in (np.float32, np.float64):
            a = a.astype(np.float32)
        self._draw_noise()
        out = self.sim.step(a.reshape(1, self.num_agents, 2))
        return self._finish_step(out)

    def reset(self, seed=None, options=None):
        """F110Env.reset (f110_env.py:425-472): options = poses [num_agents, 3]."""
        poses = options
        if poses is None:
            raise ValueError("reset(options=poses) requires the start poses [num_agents, 3]")
        poses = np.asarray(poses)
        if poses.shape[0] != self.num_agents:
            raise ValueError('Number of poses for reset does not match number of agents.')
        self.current_time = 0.0
        self.collisions = np.zeros((self.num_agents,))
        self.num_toggles = 0
        self.near_start = True
        self.near_starts = np.array([True] * self.num_agents)
        self.toggle_list = np.zeros((self.num_agents,))
        self.start_xs = poses[:, 0]
        self.start_ys = poses[:, 1]
        self.start_thetas = poses[:, 2]
        th = self.start_thetas[self.ego_idx]
        self.start_rot = np.array([[np.cos(-th), -np.sin(-th)], [np.sin(-th), np.cos(-th)]])
        # the device's lap bookkeeping takes the options' dtype (float32 poses: float32 start poses and
        # start_rot, as NumPy computes them in the reference, f110_env.py:444-451)
        dt = np.float32 if poses.dtype == np.float32 else np.float64
        if self.sim.reset_dtype != dt:
            self.sim.set_reset_dtype(dt)
        # device: RaceCar.reset for every car + the reference's zero-action step (f110_env.py:457)
        self._scan_rng = np.random.default_rng(seed=self.seed)  # RaceCar.reset, base_classes.py:204
        self._draw_noise()
        out = self.sim.reset(np.asarray(poses, dtype=np.float64).reshape(1, self.num_agents, 3))
        obs_flat, _, _, _, info = self._finish_step(out)
        return obs_flat, info

    def update_map(self, map_path, map_ext):
        """F110Env.update_map (f110_env.py:474-485): new map, cars keep their state.
        The device context is rebuilt for the new EDT; state and steer buffers
        are carried over (the reference's RaceCars keep theirs too)."""
        from .maps import load_map
        from .sim import BatchSim
        track = load_map(map_path, map_ext)
        state = self.sim.get_state()
        old = self.sim
        self.sim = BatchSim(track, n_envs=1, n_agents=self.num_agents, params=self.params, device=old.device,
                            seed=self.seed, timestep=self.timestep, integrator=_integrator_code(self.integrator),
                            ego_idx=self.ego_idx, lidar_dist=self.lidar_dist, noise_std=self.noise_std,
                            keep_f64_scans=True)
        for i, p in enumerate(self._agent_params):
            if p is not None:
                self.sim.update_params(p, agent_idx=i)
        self.sim.set_state(*state)
        if self._noise is not None:
            self.sim.set_scan_noise(self._noise)
        old.close()
        self.track = track
        self.map_path = map_path

    def update_params(self, params, index=-1):
        """F110Env.update_params (f110_env.py:487-498) -> Simulator.update_params:
        the car's dynamics and its agent ray_cast box use the new params; GJK,
        TTC side distances and the obs lidar_max keep the construction params,
        as in the reference (base_classes.py:223, :562, :122-158)."""
        if not (index < self.num_agents):
            raise IndexError('Index given is out of bounds for list of agents.')
        self.sim.update_params(params, agent_idx=index)
        for i in range(self.num_agents):
            if index < 0 or i == index:
                self._agent_params[i] = dict(params)

    def add_render_callback(self, callback_func):
        pass

    def render(self, mode='human'):
        raise NotImplementedError("rendering is out of scope of the MI355X simulator")

    def close(self):
        if getattr(self, "sim", None) is not None:
            self.sim.close()
            self.sim = None

    @property
    def unwrapped(self):
        return self
