"""Device gap_follow_action (f110_gap_follow) vs the reference
(tests/golden/gap_follow.npz, env_gapfollow.npz) and the C oracle."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def test_gap_follow_golden(gpu):
    from f110_gymnasium_ros2_jazzy_amd.opponent import gap_follow
    d = golden("gap_follow.npz")
    s = torch.as_tensor(d["scans"], device="cuda")
    act, gaps = gap_follow(s, return_gaps=True)
    assert np.array_equal(gaps.cpu().numpy(), d["gaps"])
    assert np.array_equal(act.cpu().numpy(), d["actions"].astype(np.float32))


def _structured_scans(rng, M, B=1080):
    s = rng.uniform(0.0, 6.0, (M, B)).astype(np.float32)
    for m in range(M):
        for _ in range(rng.integers(0, 8)):
            a = rng.integers(0, B)
            s[m, a:a + rng.integers(1, 200)] = rng.uniform(0.0, 0.7)
    s[rng.random((M, B)) < 0.01] = 0.5
    return s


def test_gap_follow_random_vs_oracle(gpu, oracle_mod):
    from f110_gymnasium_ros2_jazzy_amd.opponent import gap_follow
    rng = np.random.default_rng(5)
    for B in (1080, 541, 64, 7):
        s = _structured_scans(rng, 257, B)
        act, gaps = gap_follow(torch.as_tensor(s, device="cuda"), angle_increment=np.pi / B, return_gaps=True)
        act, gaps = act.cpu().numpy(), gaps.cpu().numpy()
        for m in range(s.shape[0]):
            a, g = oracle_mod.gap_follow_action(s[m], angle_increment=np.pi / B)
            assert np.array_equal(gaps[m], g), (B, m)
            assert np.array_equal(act[m], a.astype(np.float32)), (B, m)


def test_gap_follow_strided_views(gpu, oracle_mod):
    """Agent 1's scans inside [E, A, B] in, agent 1's slot of [E, A, 2] out."""
    from f110_gymnasium_ros2_jazzy_amd.opponent import gap_follow
    rng = np.random.default_rng(6)
    E, A, B = 33, 3, 1080
    s = torch.as_tensor(_structured_scans(rng, E * A).reshape(E, A, B), device="cuda")
    acts = torch.full((E, A, 2), -7.0, device="cuda")
    gap_follow(s[:, 1], out=acts[:, 1])
    a = acts.cpu().numpy()
    assert np.all(a[:, [0, 2]] == -7.0)
    for e in range(E):
        ref, _ = oracle_mod.gap_follow_action(s[e, 1].cpu().numpy())
        assert np.array_equal(a[e, 1], ref.astype(np.float32))


def test_vector_env_gapfollow_loop_matches_reference(gpu):
    """train_ddpg.py's loop (:150-174) with the opponent on the device: one env,
    noise off, the recorded ego actions -> the reference's opponent actions
    and observations."""
    from f110_gymnasium_ros2_jazzy_amd.vector_env import F110VectorEnv
    d = golden("env_gapfollow.npz")
    venv = F110VectorEnv(1, num_agents=2, noise_std=0.0, opponent="gap_follow", autoreset=False)
    try:
        obs, info = venv.reset(options=d["reset_poses"].astype(np.float64)[None])
        np.testing.assert_allclose(obs.cpu().numpy()[0], d["obs"][0], rtol=1e-6, atol=1e-6)
        for t in range(d["ego_actions"].shape[0]):
            opp = info["opponent_actions"].cpu().numpy()[0]
            np.testing.assert_allclose(opp, d["opp_actions"][t], rtol=1e-6, atol=1e-6)
            obs, rew, term, trunc, info = venv.step(torch.as_tensor(d["ego_actions"][t][None], device="cuda"))
            np.testing.assert_allclose(obs.cpu().numpy()[0], d["obs"][t + 1], rtol=1e-5, atol=1e-5)
            assert bool(term[0]) == bool(d["terminated"][t])
    finally:
        venv.close()
