"""The fused learner heads (csrc/f110_ddpg.hip via ddpg_heads.py) against the
plain torch modules they replace (rl_training/DDPG/agent.py:56-61, :93-97,
:302-331): forward values and every parameter gradient of the critic and
actor updates, fp32 (fused dot products: rounding-level differences, rtol
1e-5)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _nets(seed, obs_dim=1088, act_dim=2):
    from f110_gymnasium_ros2_jazzy_amd.ddpg import Actor, Critic
    torch.manual_seed(seed)
    a = Actor(obs_dim, act_dim, [-0.4189, 0.0], [0.4189, 20.0]).cuda()
    c = Critic(obs_dim, act_dim).cuda()
    with torch.no_grad():  # non-trivial output layers (the reference inits them near 0)
        a.fc3.weight.normal_(0, 0.2)
        a.fc3.bias.normal_(0, 0.1)
        c.q.weight.normal_(0, 0.2)
        c.q.bias.normal_(0, 0.1)
    return a, c


def _close(x, y, what):
    """fp32 rounding of a reordered 128-term sum: a few ulps of the tensor's
    scale (td = y - q cancels, so the absolute bar follows max |ref|)."""
    x, y = x.detach().cpu().numpy(), y.detach().cpu().numpy()
    np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-5 * float(np.abs(y).max()) + 1e-9, err_msg=what)


@pytest.mark.parametrize("B", [4096, 333])
def test_fused_heads_match_torch(gpu, monkeypatch, B):
    import f110_gymnasium_ros2_jazzy_amd.ddpg as D
    g = torch.Generator(device="cuda").manual_seed(B)
    s = torch.rand(B, 1088, device="cuda", generator=g)
    ns = torch.rand(B, 1088, device="cuda", generator=g)
    act = torch.rand(B, 2, device="cuda", generator=g)
    r = torch.randn(B, 1, device="cuda", generator=g)
    d = (torch.rand(B, 1, device="cuda", generator=g) < 0.1).float()
    w = torch.rand(B, 1, device="cuda", generator=g)
    out = {}
    for fused in (False, True):
        monkeypatch.setattr(D, "FUSED", fused)
        a, c = _nets(3)
        with torch.no_grad():
            a_next = a(ns)
            if fused:
                from f110_gymnasium_ros2_jazzy_amd.ddpg_heads import td_target
                y = td_target(c.hidden(ns, a_next), c.q.weight, c.q.bias, r, d, 0.99)
            else:
                y = r + 0.99 * (1.0 - d) * c(ns, a_next)
        if fused:
            from f110_gymnasium_ros2_jazzy_amd.ddpg_heads import critic_loss, q_mean
            closs, td = critic_loss(c.hidden(s, act), c.q.weight, c.q.bias, y, w)
        else:
            td = y - c(s, act)
            closs = (w * td ** 2).mean()
        closs.backward()
        cgrads = [p.grad.clone() for p in c.parameters()]
        for p in c.parameters():
            p.requires_grad_(False)
        if fused:
            aloss = q_mean(c.hidden(s, a(s)), c.q.weight, c.q.bias, -1.0)
        else:
            aloss = -c(s, a(s)).mean()
        aloss.backward()
        agrads = [p.grad.clone() for p in a.parameters()]
        out[fused] = (a_next, y, td.detach(), closs.detach(), cgrads, aloss.detach(), agrads)
    ref, got = out[False], out[True]
    for k, name in enumerate(["a_next", "target_y", "td", "critic_loss"]):
        _close(got[k], ref[k], name)
    for i, (x, y) in enumerate(zip(got[4], ref[4])):
        _close(x, y, f"critic grad {i}")
    _close(got[5], ref[5], "actor_loss")
    for i, (x, y) in enumerate(zip(got[6], ref[6])):
        _close(x, y, f"actor grad {i}")


def test_fused_heads_reject_bad_shapes(gpu):
    from f110_gymnasium_ros2_jazzy_amd import _lib
    from f110_gymnasium_ros2_jazzy_amd.ddpg_heads import q_mean
    h = torch.zeros(8, 300, device="cuda")  # K > 255
    with pytest.raises(_lib.F110Error):
        q_mean(h, torch.zeros(1, 300, device="cuda"), torch.zeros(1, device="cuda"))
    with pytest.raises(_lib.F110Error):
        q_mean(torch.zeros(8, 16), torch.zeros(1, 16), torch.zeros(1))  # CPU tensors
