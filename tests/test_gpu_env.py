"""F110Env facade and F110VectorEnv on the GPU vs the reference F110Env
trace (tests/golden/env_2agent.npz, reference run with noise disabled)."""
import os

import numpy as np
import pytest
import torch

from conftest import MAPS, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env(gpu):
    from f110_gym.envs import F110Env
    e = F110Env(map_dir=MAPS + os.sep, map="Spielberg_map", map_ext=".png", num_agents=2, noise_std=0.0)
    yield e
    e.close()


def test_f110env_matches_reference_trace(env, nonexact_budget):
    d = golden("env_2agent.npz")
    nonexact = 0
    obs, info = env.reset(options=d["reset_poses"])
    assert obs.dtype == np.float32 and obs.shape == (1088,)
    np.testing.assert_allclose(obs, d["obs"][0], rtol=1e-6, atol=1e-6)
    assert info["time"] == d["info_time"][0]
    for t in range(d["actions"].shape[0]):
        obs, r, term, trunc, info = env.step(d["actions"][t])
        np.testing.assert_allclose(obs, d["obs"][t + 1], rtol=1e-5, atol=1e-5)
        nonexact += int(np.sum(obs != d["obs"][t + 1]))
        assert r == d["reward"][t] and term == d["terminated"][t] and trunc == d["truncated"][t]
        for k in ("poses_x", "poses_y", "poses_theta", "linear_vels_x", "linear_vels_y", "ang_vels_z"):
            np.testing.assert_allclose(info[k], d["info_" + k][t + 1], rtol=1e-5, atol=1e-5)
        assert np.array_equal(info["collisions"], d["info_collisions"][t + 1])
        assert np.array_equal(info["lap_counts"], d["info_lap_counts"][t + 1])
        np.testing.assert_allclose(info["lap_times"], d["info_lap_times"][t + 1], rtol=1e-6)
        assert np.array_equal(info["checkpoint_done"], d["info_checkpoint_done"][t + 1])
        assert abs(info["time"] - d["info_time"][t + 1]) < 1e-12
        np.testing.assert_allclose(np.stack(info["scans"]), d["info_scans"][t + 1], rtol=1e-5, atol=1e-5)
    assert env.unwrapped.timestep == 0.01
    nonexact_budget("env_2agent_obs", nonexact)


def test_f110env_api_surface(env):
    assert env.action_space.shape == (2, 2)
    assert env.observation_space.shape == (1088,)
    with pytest.raises(ValueError):
        env.reset(options=np.zeros((3, 3), np.float32))


def test_vector_env_autoreset_next_step(gpu):
    from f110_gymnasium_ros2_jazzy_amd.vector_env import F110VectorEnv
    N = 64
    venv = F110VectorEnv(N, num_agents=1, seed=3)
    obs, info = venv.reset(seed=3)
    assert obs.shape == (N, 1084) and obs.device.type == "cuda"
    crash = torch.tensor([0.4189, 20.0], device="cuda").expand(N, 2)
    prev_term = torch.zeros(N, dtype=torch.bool, device="cuda")
    seen = 0
    for t in range(300):
        obs, rew, term, trunc, info = venv.step(crash)
        assert torch.equal(info["reset"], prev_term)        # NEXT_STEP autoreset
        assert torch.all(rew[info["reset"]] == 0) and torch.all(rew[~info["reset"]] == 0.01)
        assert not trunc.any()
        seen += int(info["reset"].sum())
        prev_term = term
    assert seen > 0
    venv.close()


def test_vector_env_numpy_two_agents(gpu):
    from f110_gymnasium_ros2_jazzy_amd.vector_env import F110VectorEnv
    venv = F110VectorEnv(8, num_agents=2, as_numpy=True, seed=1)
    obs, info = venv.reset()
    assert isinstance(obs, np.ndarray) and obs.shape == (8, 1088)
    a = np.zeros((8, 2, 2), np.float32)
    a[..., 1] = 3.0
    obs, rew, term, trunc, info = venv.step(a)
    assert rew.shape == (8,) and term.dtype == bool and info["scans"].shape == (8, 2, 1080)
    venv.close()


def _replay(env, d):
    """Drive the facade through a recorded reference run (resets marked by
    is_reset) and compare every call's outputs; returns the number of obs
    entries that are not bit-exact (ray_cast beams only)."""
    nonexact = 0
    for t in range(d["obs"].shape[0]):
        if d["is_reset"][t]:
            obs, info = env.reset(options=d["reset_poses"])
        else:
            obs, r, term, trunc, info = env.step(d["actions"][t])
            assert r == d["reward"][t] and term == d["terminated"][t] and trunc == d["truncated"][t]
        np.testing.assert_allclose(obs, d["obs"][t], rtol=1e-5, atol=1e-5)
        nonexact += int(np.sum(obs != d["obs"][t]))
        for k in ("poses_x", "poses_y", "poses_theta", "linear_vels_x", "ang_vels_z"):
            np.testing.assert_allclose(info[k], d["info_" + k][t], rtol=1e-5, atol=1e-5)
        assert np.array_equal(info["collisions"], d["info_collisions"][t])
        assert np.array_equal(info["lap_counts"], d["info_lap_counts"][t])
        np.testing.assert_allclose(np.stack(info["scans"]), d["info_scans"][t], rtol=1e-5, atol=1e-5)
    return nonexact


def test_f110env_reference_noise_stream(gpu, nonexact_budget):
    """Noise on (the reference default): the facade replays the reference's
    per-car default_rng(seed) draws, so noisy scans match the reference run,
    including the generator restart at the second reset."""
    from f110_gym.envs import F110Env
    d = golden("env_2agent_noise.npz")
    env = F110Env(map_dir=MAPS + os.sep, map="Spielberg_map", map_ext=".png", num_agents=2, seed=int(d["seed"]))
    try:
        nonexact_budget("env_2agent_noise_obs", _replay(env, d))
    finally:
        env.close()


def test_f110env_update_params_per_agent(gpu, nonexact_budget):
    """update_params(p, index=0) before reset: agent 0's dynamics and the box
    it ray-casts agent 1 with use p; GJK keeps the construction params."""
    from f110_gym.envs import F110Env
    d = golden("env_2agent_params.npz")
    p1 = {str(k): float(v) for k, v in zip(d["params1_keys"], d["params1"])}
    env = F110Env(map_dir=MAPS + os.sep, map="Spielberg_map", map_ext=".png", num_agents=2, noise_std=0.0)
    try:
        with pytest.raises(IndexError):
            env.update_params(p1, index=2)
        env.update_params(p1, index=0)
        nonexact_budget("env_2agent_params_obs", _replay(env, d))
    finally:
        env.close()


def test_f110env_update_map_keeps_state(gpu):
    """update_map swaps the EDT; the cars keep their state (f110_env.py:474-485)."""
    from f110_gym.envs import F110Env
    env = F110Env(map_dir=MAPS + os.sep, map="Spielberg_map", map_ext=".png", num_agents=1, noise_std=0.0)
    try:
        d = golden("env_2agent.npz")
        env.reset(options=d["reset_poses"][:1])
        for _ in range(5):
            obs, *_ , info = env.step(np.array([[0.0, 5.0]], np.float32))
        before = env.sim.agent_states().cpu().numpy()
        env.update_map(os.path.join(MAPS, "straight_corridor.yaml"), ".png")
        assert np.array_equal(env.sim.agent_states().cpu().numpy(), before)
        obs2, *_ = env.step(np.array([[0.0, 5.0]], np.float32))
        assert not np.array_equal(obs2[:1080], obs[:1080])   # new walls
    finally:
        env.close()


@pytest.mark.parametrize("options_dtype", ["float32", "auto"])
def test_vector_env_float32_lap_boundary(gpu, options_dtype):
    """The batched VectorEnv's device lap logic with float32 reset options
    (train_ddpg's dtype) against a reference F110Env episode
    (tests/golden/env_lap_f32.npz): both cars circle through their start
    zones, the toggles pass 4 and the episode terminates on laps.  start_rot
    is NumPy's float32 cos / sin of the float32 yaw and np.dot's fma rows
    (f110_env.py:330, 448-451): lap counts, lap times, collisions and
    terminated equal the reference at every step.  "auto": the dtype comes
    from the options array itself; "float32": the env's options_dtype."""
    from f110_gymnasium_ros2_jazzy_amd.vector_env import F110VectorEnv
    d = golden("env_lap_f32.npz")
    kw = {"options_dtype": np.float64} if options_dtype == "auto" else {}
    env = F110VectorEnv(1, num_agents=2, noise_std=0.0, autoreset=False, device=gpu, **kw)
    try:
        obs, info = env.reset(options=d["reset_poses"][None])
        rot, _ = env.sim.lap_state()
        sr = d["start_rot"].astype(np.float64)   # the reference's float32 matrix
        assert np.array_equal(rot[:, 0].cpu().numpy(), [sr[0, 0], sr[1, 0]])
        T = d["terminated"].shape[0]
        for t in range(T):
            if t:
                obs, r, term, trunc, info = env.step(d["actions"][None])
                assert bool(term[0]) == bool(d["terminated"][t]), t
            _, tog = env.sim.lap_state()
            assert np.array_equal(tog[0].cpu().numpy(), d["toggles"][t].astype(np.int32)), t
            assert np.array_equal(info["lap_counts"][0].cpu().numpy(), d["lap_counts"][t].astype(np.float32)), t
            assert np.array_equal(info["lap_times"][0].cpu().numpy(), d["lap_times"][t].astype(np.float32)), t
            assert np.array_equal(info["collisions"][0].cpu().numpy(), d["collisions"][t].astype(np.int8)), t
        assert bool(term[0]) and d["lap_counts"][-1].min() >= 2
    finally:
        env.close()


def test_f110env_float32_lap_boundary(gpu):
    """The facade's _check_done reads the device epilogue (terminated, lap
    times / counts, toggles): with float32 reset options (train_ddpg's dtype)
    it follows the reference F110Env episode of tests/golden/env_lap_f32.npz
    through both cars' start-zone crossings to the lap termination, step by
    step (terminated, lap_counts, lap_times, checkpoint_done, collisions)."""
    from f110_gym.envs import F110Env
    d = golden("env_lap_f32.npz")
    env = F110Env(map_dir=MAPS + os.sep, map="Spielberg_map", map_ext=".png", num_agents=2, noise_std=0.0)
    try:
        poses = d["reset_poses"]
        assert poses.dtype == np.float32
        obs, info = env.reset(options=poses)
        for t in range(d["terminated"].shape[0]):
            if t:
                obs, r, term, trunc, info = env.step(d["actions"])
                assert term == bool(d["terminated"][t]), t
            assert np.array_equal(info["lap_counts"], d["lap_counts"][t].astype(np.float32)), t
            assert np.array_equal(info["lap_times"], d["lap_times"][t].astype(np.float32)), t
            assert np.array_equal(info["checkpoint_done"], d["toggles"][t] >= 4), t
            assert np.array_equal(info["collisions"], d["collisions"][t].astype(np.int8)), t
            assert np.array_equal(env.toggle_list, d["toggles"][t].astype(np.float64)), t
        assert term and d["lap_counts"][-1].min() >= 2
    finally:
        env.close()
