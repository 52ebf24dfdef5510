"""The CPU restatement of the PER buffer (oracle/replay_oracle.py) against
the reference buffer's own recorded state (tests/golden/per.npz), and the
DDPG learner's update against the reference DDPGAgent (tests/golden/ddpg.npz,
CPU torch; the DDPG learner is f110_gymnasium_ros2_jazzy_amd/ddpg.py)."""
import numpy as np
import pytest
import torch

from conftest import golden


def replay_ops(d):
    """Yield (op, arg) of the recorded sequence; arg: add priority (op 1),
    sample index (op 2), update index (op 3)."""
    s = u = 0
    for t, op in enumerate(d["ops"]):
        if op == 1:
            slot = d["next_idx"][t - 1] if t else 0
            yield t, op, float(d["prio"][t][slot])
        elif op == 2:
            yield t, op, s
            s += 1
        elif op == 3:
            yield t, op, u
            u += 1
        else:
            yield t, op, None


def test_per_oracle_matches_reference_buffer():
    from replay_oracle import PEROracle
    d = golden("per.npz")
    o = PEROracle(16, 5, alpha=0.6)
    betas = [0.4, 0.4, 0.7, 0.4, 0.4, 0.4, 0.4]
    for t, op, arg in replay_ops(d):
        if op == 0:
            o.add()
        elif op == 1:
            o.add(priority=arg)
        elif op == 2:
            n = o.length
            np.testing.assert_array_equal(o.sampling_probs(), d["sample_probs"][arg][:n])
            idx = d["sample_idx"][arg]
            idx = idx[idx >= 0]
            np.testing.assert_array_equal(o.weights(idx, betas[arg]), d["sample_w"][arg][:idx.size])
        else:
            idx = d["upd_idx"][arg]
            o.update_priorities(idx[idx >= 0], d["upd_val"][arg][idx >= 0])
        np.testing.assert_array_equal(o.prio, d["prio"][t], err_msg=f"op {t}")
        assert (o.length, o.next_idx) == (d["length"][t], d["next_idx"][t])


def test_per_sampling_statistics_fixture():
    """The reference's own draws follow successive sampling without
    replacement: first position ~ p (chi-square), batch members distinct."""
    d = golden("per.npz")
    n = int(d["stat_draws"])
    exp = n * d["stat_probs"]
    chi2 = float(np.sum((d["stat_first"] - exp) ** 2 / exp))
    assert chi2 < 39 + 6 * np.sqrt(2 * 39)  # 39 dof, ~6 sigma
    assert d["stat_incl"].sum() == n * int(d["stat_batch"])


# ---------------------------------------------------------------- DDPG ----
def _load_state(net, d, prefix):
    sd = {k: torch.from_numpy(np.asarray(d[f"{prefix}/{k}"])) for k in net.state_dict().keys()}
    net.load_state_dict(sd)


def _learner(device="cpu"):
    from f110_gymnasium_ros2_jazzy_amd.ddpg import DDPGLearner
    return DDPGLearner(obs_dim=12, act_dim=2, action_low=[-0.4189, 0.0], action_high=[0.4189, 20.0], gamma=0.99,
                       tau=0.005, actor_lr=1e-4, critic_lr=1e-3, seed=42, device=device, replay=None)


def test_ddpg_init_matches_reference_seed():
    """DDPGAgent(seed=42): torch.manual_seed then Actor, Critic, targets in
    that order (agent.py:176-184) -> the same initial weights."""
    d = golden("ddpg.npz")
    ln = _learner()
    for name, net in (("actor", ln.actor), ("critic", ln.critic), ("actor", ln.actor_target),
                      ("critic", ln.critic_target)):
        for k, v in net.state_dict().items():
            if k in ("action_low", "action_high"):
                continue
            np.testing.assert_array_equal(v.numpy(), d[f"init/{name}/{k}"], err_msg=f"{name}.{k}")


def test_ddpg_update_matches_reference_replay():
    """Three DDPGAgent.replay() steps (agent.py:242-348) on the recorded
    batches: losses, TD priorities and all four networks."""
    d = golden("ddpg.npz")
    ln = _learner()
    S, A, R, S2, D = (torch.from_numpy(np.asarray(d[k])) for k in ("S", "A", "R", "S2", "D"))
    for step in range(3):
        idx = torch.from_numpy(d["idx"][step])
        w = torch.from_numpy(d["w"][step])
        st = ln.update(S[idx], A[idx], R[idx], S2[idx], D[idx].float(), w)
        cl, al, td = float(st["critic_loss"]), float(st["actor_loss"]), st["td"]
        np.testing.assert_allclose([cl, al], d["losses"][step][:2], rtol=1e-6)
        pr = ln.td_priorities(td, 1e-5).numpy()
        np.testing.assert_allclose(float(np.mean(pr)), d["losses"][step][2], rtol=1e-6)
        np.testing.assert_allclose(pr, d["prios"][step][d["idx"][step]], rtol=1e-6)
    for name, net in (("actor", ln.actor), ("critic", ln.critic), ("actor_target", ln.actor_target),
                      ("critic_target", ln.critic_target)):
        for k, v in net.state_dict().items():
            if k in ("action_low", "action_high"):
                continue
            np.testing.assert_allclose(v.numpy(), d[f"final/{name}/{k}"], rtol=1e-5, atol=1e-7,
                                       err_msg=f"{name}.{k}")
