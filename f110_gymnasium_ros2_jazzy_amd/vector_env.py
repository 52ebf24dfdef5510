"""F110VectorEnv: N F1TENTH envs stepped as one batch on one GPU.

Gymnasium-1.x vector surface (``reset(seed, options) -> (obs, infos)``,
``step(actions) -> (obs, rewards, terminations, truncations, infos)``,
``num_envs``, ``single_observation_space``, ``single_action_space``) with
observations and infos kept as device tensors (``as_numpy=True`` converts).

Per env the semantics are F110Env's (f110_env.py:371-472): reward = timestep,
terminated = ego collision or 4 lap toggles, truncated = False, flat obs =
[agent-0 scan / lidar_max, (x, y, yaw, collision) per agent].  Autoreset is
the gymnasium NEXT_STEP mode and runs on the device: the step after an env
terminates resets it to a pose drawn from ``spawn_poses`` (and performs the
reference's zero-action reset step); that step's reward is 0.

``reward_fn`` (a reward.BatchedCenterlineReward) replaces the timestep
reward with the training reward train_ddpg.py computes per step, evaluated on
the device; autoreset steps reset its state and are rewarded 0.

``opponent="gap_follow"`` drives agent ``opponent_idx`` with the reference's
rule-based opponent (gap_follow.py) on the device, as train_ddpg.py:168 does
on the host: its action for step t comes from its own float32 scan of step
t-1 (or of the reset).  ``step`` then takes the other agents' actions
([N, 2] for two agents) and ``infos["opponent_actions"]`` shows the
opponent's.

Multi-GPU: give each rank its block of envs (distributed.shard_range) and
``env_offset`` = the block's first global id; RNG streams are keyed by global
env id, so results do not depend on the GPU count.
"""
from __future__ import annotations

import numpy as np
import torch

from .f110_env import DEFAULT_PARAMS, _box
from .maps import centerline_spawns, load_map
from .sim import BatchSim


class F110VectorEnv:
    metadata = {"autoreset_mode": "NextStep", "render_modes": []}

    def __init__(self, num_envs: int, map: str = "Spielberg_map", map_ext: str = ".png", num_agents: int = 1,
                 params: dict | None = None, seed: int = 42, timestep: float = 0.01, device=0,
                 spawn_poses: np.ndarray | None = None, noise_std: float = 0.01, env_offset: int = 0,
                 ego_idx: int = 0, as_numpy: bool = False, autoreset: bool = True, opponent: str | None = None,
                 opponent_idx: int = 1, reward_fn=None, infos: str = "full", options_dtype=np.float32, **kwargs):
        self.num_envs = int(num_envs)
        self.num_agents = int(num_agents)
        self.params = dict(params or DEFAULT_PARAMS)
        self.timestep = timestep
        self.as_numpy = as_numpy
        self.track = load_map(map, map_ext)
        if spawn_poses is None:
            spawn_poses = centerline_spawns(map.replace("_map", ""), self.num_agents)
        self.spawn_poses = np.ascontiguousarray(spawn_poses, dtype=np.float64)
        self.sim = BatchSim(self.track, n_envs=self.num_envs, n_agents=self.num_agents, params=self.params,
                            device=device, seed=seed, timestep=timestep, ego_idx=ego_idx, noise_std=noise_std,
                            autoreset=autoreset, spawn_poses=self.spawn_poses, env_offset=env_offset, **kwargs)
        self.device = self.sim.device
        # F110Env.reset computes start_rot in the dtype of its options
        # (f110_env.py:448-451): autoresets and option-less resets follow
        # options_dtype (train_ddpg passes float32 poses); an explicit
        # reset(options=...) follows that array's dtype
        self.options_dtype = np.dtype(options_dtype)
        self.sim.set_reset_dtype(self.options_dtype)
        B, A = self.sim.B, self.num_agents
        x_min, x_max, y_min, y_max = self.track.bounds
        self.single_observation_space = _box(
            np.array([0.0] * B + [x_min, y_min, -np.pi, 0.0] * A, np.float32),
            np.array([1.0] * B + [x_max, y_max, np.pi, 1.0] * A, np.float32))
        low = np.array([self.params["s_min"], self.params["v_min"]], np.float32)
        high = np.array([self.params["s_max"], self.params["v_max"]], np.float32)
        self.single_action_space = _box(np.tile(low, (A, 1)), np.tile(high, (A, 1)))
        self._rng = np.random.default_rng(seed)
        self.opponent = opponent
        self.opponent_idx = int(opponent_idx)
        # reward_fn: a BatchedCenterlineReward (reward.py) evaluated on the device
        # from every step's observations, as train_ddpg.py:176 does per env
        self.reward_fn = reward_fn
        # infos="minimal": only "reset" (+ "opponent_actions"), no per-step copies
        # of the scans and poses (the batched trainer reads nothing else)
        if infos not in ("full", "minimal"):
            raise ValueError("infos must be 'full' or 'minimal'")
        self.infos_mode = infos
        if reward_fn is not None and reward_fn.n_envs != self.num_envs:
            raise ValueError("reward_fn must be built for num_envs envs")
        if opponent is not None:
            if opponent != "gap_follow":
                raise ValueError(f"unknown opponent policy {opponent!r} (supported: 'gap_follow')")
            if not (0 <= self.opponent_idx < A) or A < 2:
                raise ValueError("opponent needs num_agents >= 2 and 0 <= opponent_idx < num_agents")
            self._act = torch.zeros(self.num_envs, A, 2, dtype=torch.float32, device=self.device)
            self._others = [i for i in range(A) if i != self.opponent_idx]
            # a contiguous run of caller-driven agents is written with a slice
            # copy (one strided copy kernel) instead of an index_put
            o = self._others
            self._others_sl = slice(o[0], o[-1] + 1) if o and o == list(range(o[0], o[-1] + 1)) else o

    def _opponent_next(self, out):
        """Next step's opponent action from this step's scans (train_ddpg.py:168)."""
        if self.opponent is not None:
            from .opponent import gap_follow
            gap_follow(out.scans[:, self.opponent_idx], out=self._act[:, self.opponent_idx])

    # ------------------------------------------------------------------
    def _infos(self, out):
        if self.infos_mode == "minimal":
            infos = {"reset": out.was_reset.bool()}
            if self.opponent is not None:
                infos["opponent_actions"] = self._act[:, self.opponent_idx]
            return {k: v.cpu().numpy() for k, v in infos.items()} if self.as_numpy else infos
        st = self.sim.agent_states()  # [E, A, 7]
        infos = {
            "poses_x": st[..., 0].float(), "poses_y": st[..., 1].float(), "poses_theta": st[..., 4].float(),
            "linear_vels_x": st[..., 3].float(), "ang_vels_z": st[..., 5].float(),
            "collisions": out.collisions.to(torch.int8), "lap_times": out.lap_times.clone(),
            "lap_counts": out.lap_counts.clone(), "scans": out.scans.clone(), "time": out.sim_time.clone(),
            "reset": out.was_reset.bool(),
        }
        if self.opponent is not None:
            infos["opponent_actions"] = self._act[:, self.opponent_idx].clone()
        if self.as_numpy:
            infos = {k: v.cpu().numpy() for k, v in infos.items()}
        return infos

    def reset(self, seed=None, options=None):
        """options: poses [N, A, 3] (or [A, 3] for every env); default: spawn table draws."""
        if seed is not None:
            self._rng = np.random.default_rng(seed)
        if options is None:
            idx = self._rng.integers(0, self.spawn_poses.shape[0], self.num_envs)
            options = self.spawn_poses[idx].astype(self.options_dtype)
        dt = options.dtype if hasattr(options, "dtype") else np.asarray(options).dtype
        self.sim.set_reset_dtype(dt)
        out = self.sim.reset(options)
        self.sim.set_reset_dtype(self.options_dtype)  # the device autoresets
        self._opponent_next(out)
        if self.reward_fn is not None:
            self.reward_fn.reset()
        obs = out.obs.clone()
        return (obs.cpu().numpy() if self.as_numpy else obs), self._infos(out)

    def step(self, actions):
        a = torch.as_tensor(actions, device=self.device)
        if self.opponent is not None:
            if a.dim() == 2:
                a = a.reshape(self.num_envs, len(self._others), 2)
            if a.shape[1] == self.num_agents:
                a = a[:, self._others_sl]
            self._act[:, self._others_sl] = a
            a = self._act
        elif a.dim() == 2 and self.num_agents == 1:
            a = a.unsqueeze(1)
        out = self.sim.step(a)
        self._opponent_next(out)
        if self.reward_fn is not None:  # reset envs: reward_fn.reset(), reward 0 (the u8 flags as they are)
            rewards = self.reward_fn(out.obs, reset_mask=out.was_reset).clone()
        else:
            rewards = torch.where(out.was_reset.bool(), torch.zeros((), dtype=torch.float64, device=self.device),
                                  torch.full((), self.timestep, dtype=torch.float64, device=self.device))
        term = out.terminated.bool()
        trunc = torch.zeros_like(term)
        obs = out.obs.clone()
        if self.as_numpy:
            return (obs.cpu().numpy(), rewards.cpu().numpy(), term.cpu().numpy(), trunc.cpu().numpy(),
                    self._infos(out))
        return obs, rewards, term, trunc, self._infos(out)

    def agent_actions(self):
        """The learning agent's rows of the action buffer the next step reads
        ([N, 2] view), or None (no opponent, or several learning agents): a
        policy may write its actions here (DDPGLearner.choose_action(out=...))
        and pass the same view to step_transition(), which then copies nothing."""
        if self.opponent is None or len(self._others) != 1:
            return None
        return self._act[:, self._others[0]]

    def step_transition(self, actions, obs_out=None):
        """step() for a trainer on the device: (next_obs copy [N, obs_dim],
        rewards float64 [N], terminated uint8 [N], was_reset uint8 [N]).  The
        rewards and flags are the simulator's / reward function's own buffers
        (no clone, no dtype conversion): valid until the next step.  obs_out:
        a preallocated [N, obs_dim] float32 tensor to copy next_obs into (a
        captured step graph's fixed buffer) instead of a new one."""
        if self.as_numpy:
            raise ValueError("step_transition: device tensors only (as_numpy=False)")
        a = torch.as_tensor(actions, device=self.device)
        if self.opponent is not None:
            dst = self.agent_actions()
            if dst is None or a.data_ptr() != dst.data_ptr() or a.stride() != dst.stride():
                self._act[:, self._others_sl] = a.reshape(self.num_envs, len(self._others), 2)
            a = self._act
        elif a.dim() == 2 and self.num_agents == 1:
            a = a.unsqueeze(1)
        out = self.sim.step(a, obs_out=obs_out)  # the simulator writes obs_out itself (no copy)
        obs = out.obs if obs_out is None else obs_out
        self._opponent_next(out)
        if self.reward_fn is not None:
            rewards = self.reward_fn(obs, reset_mask=out.was_reset)
        else:
            rewards = torch.where(out.was_reset.bool(), torch.zeros((), dtype=torch.float64, device=self.device),
                                  torch.full((), self.timestep, dtype=torch.float64, device=self.device))
        return (obs.clone() if obs_out is None else obs_out), rewards, out.terminated, out.was_reset

    def close(self):
        if getattr(self, "sim", None) is not None:
            self.sim.close()
            self.sim = None
