"""Device PER buffer (f110_replay_*) and the DDPG learner on the GPU, against
the reference buffer's recorded state (tests/golden/per.npz), the CPU
restatement (oracle/replay_oracle.py) and the reference DDPGAgent
(tests/golden/ddpg.npz)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def _rb(cap, batch, D=8, A=2, **kw):
    from f110_gymnasium_ros2_jazzy_amd.replay import DeviceReplayBuffer
    return DeviceReplayBuffer(buffer_size=cap, batch_size=batch, obs_dim=D, act_dim=A, device=0, **kw)


def _rows(n, D=8, A=2, base=0.0):
    v = torch.arange(n, dtype=torch.float32, device="cuda")[:, None] + base
    return v.expand(n, D).contiguous(), v.expand(n, A).contiguous() * 2, v[:, 0] * 3, v.expand(n, D) + 0.5


def test_replay_follows_reference_sequence(gpu):
    from replay_oracle import PEROracle
    from test_oracle_replay import replay_ops
    d = golden("per.npz")
    rb = _rb(16, 5)
    o = PEROracle(16, 5, alpha=0.6)
    betas = [0.4, 0.4, 0.7, 0.4, 0.4, 0.4, 0.4]
    for t, op, arg in replay_ops(d):
        if op in (0, 1):
            s, a, r, s2 = _rows(1, base=float(t))
            rb.add(s, a, r, s2, torch.zeros(1, device="cuda"), priority=None if op == 0 else [arg])
            o.add(None if op == 0 else arg)
        elif op == 2:
            idx, batch, w = rb.sample(beta=betas[arg])
            idx = idx.cpu().numpy()
            assert ((idx >= 0) & (idx < o.length)).all()
            if o.length >= 5:
                assert len(set(idx.tolist())) == 5  # without replacement
            np.testing.assert_allclose(w.cpu().numpy(), o.weights(idx, betas[arg]), rtol=2e-6)
            st = rb.arrays(("states",))["states"].cpu().numpy()
            np.testing.assert_array_equal(batch["states"].cpu().numpy(), st[idx])
        else:  # the reference's own update (indices and raw priorities)
            idx = d["upd_idx"][arg]
            vals = d["upd_val"][arg][idx >= 0]
            idx = idx[idx >= 0]
            rb.update_priorities(idx, vals)
            o.update_priorities(idx, vals)
        np.testing.assert_array_equal(rb.priorities().cpu().numpy(), d["prio"][t], err_msg=f"op {t}")
        assert len(rb) == d["length"][t]
    rb.close()


def test_replay_sampling_distribution(gpu):
    """40 rows with the fixture's priorities, 20000 draws of 6 without
    replacement: every batch is 6 distinct rows in index order, and the
    per-row inclusion counts agree with the reference's own rng.choice
    counts (same distribution of the sampled set)."""
    d = golden("per.npz")
    n_draws, B = int(d["stat_draws"]), int(d["stat_batch"])
    rb = _rb(40, B, seed=123)
    s, a, r, s2 = _rows(40)
    rb.add(s, a, r, s2, priority=torch.as_tensor(d["stat_prio"]))
    incl = torch.zeros(40, dtype=torch.int64, device="cuda")
    ones = torch.ones(B, dtype=torch.int64, device="cuda")
    ordered = torch.ones((), dtype=torch.bool, device="cuda")
    for _ in range(n_draws):
        idx, _, _ = rb.sample(beta=0.4, gather=False)
        incl.index_add_(0, idx, ones)
        ordered &= (idx[1:] > idx[:-1]).all()
    assert bool(ordered)  # distinct and ascending
    incl = incl.cpu().numpy()
    assert incl.sum() == n_draws * B and (incl <= n_draws).all()
    ref = d["stat_incl"]
    z = np.abs(incl - ref) / np.sqrt(incl + ref + 1.0)
    assert z.max() < 5.0, (incl, ref)
    rb.close()


def test_replay_masked_add_and_gather(gpu):
    D, A = 1088, 2
    rb = _rb(100, 32, D=D, A=A, max_add=64)
    g = torch.Generator(device="cuda").manual_seed(0)
    S = torch.rand(60, D, device="cuda", generator=g)
    S2 = torch.rand(60, D, device="cuda", generator=g)
    Ac = torch.rand(60, A, device="cuda", generator=g)
    R = torch.rand(60, device="cuda", generator=g)
    done = torch.rand(60, device="cuda", generator=g) < 0.3
    mask = torch.rand(60, device="cuda", generator=g) < 0.7
    rb.add(S, Ac, R, S2, done, mask=mask)
    rb.add(S, Ac, R, S2, done, mask=mask)     # wraps the 100-row ring
    keep = torch.cat([mask.nonzero()[:, 0]] * 2)
    k = keep.numel()
    assert len(rb) == min(k, 100)
    arr = rb.arrays()
    slots = torch.arange(k, device="cuda") % 100
    last = {int(s): i for i, s in enumerate(slots.tolist())}  # later rows overwrite earlier ones
    rows = keep[torch.tensor([last[s] for s in range(min(k, 100))], device="cuda")]
    torch.testing.assert_close(arr["states"][:len(rows)], S[rows], rtol=0, atol=0)
    torch.testing.assert_close(arr["next_states"][:len(rows)], S2[rows], rtol=0, atol=0)
    torch.testing.assert_close(arr["actions"][:len(rows)], Ac[rows], rtol=0, atol=0)
    torch.testing.assert_close(arr["dones"][:len(rows)], done[rows].float(), rtol=0, atol=0)
    idx, b, w = rb.sample(0.4)
    torch.testing.assert_close(b["states"], arr["states"][idx], rtol=0, atol=0)
    torch.testing.assert_close(b["rewards"], arr["rewards"][idx], rtol=0, atol=0)
    assert float(w.max()) == 1.0
    rb.close()


def test_replay_full_size(gpu):
    """train_ddpg-sized rows (1088 floats), 2^18 rows, batch 4096: distinct
    indices inside the buffer, weights in (0, 1] with max 1, priority update
    by TD errors (|td| + 1e-5) lands on the sampled rows."""
    from replay_oracle import PEROracle
    cap, B, D = 1 << 18, 4096, 1088
    rb = _rb(cap, B, D=D, max_add=1 << 16)
    g = torch.Generator(device="cuda").manual_seed(1)
    for k in range(5):
        S = torch.rand(1 << 16, D, device="cuda", generator=g)
        rb.add(S, torch.rand(1 << 16, 2, device="cuda", generator=g), torch.rand(1 << 16, device="cuda"), S)
    assert len(rb) == cap
    td = torch.randn(B, device="cuda", generator=g)
    for _ in range(3):
        idx, b, w = rb.sample(0.4)
        rb.update_priorities(idx, td, td_errors=True, add_eps=1e-5)
    i = idx.cpu().numpy()
    assert len(np.unique(i)) == B and i.min() >= 0 and i.max() < cap
    wn = w.cpu().numpy()
    assert wn.max() == 1.0 and (wn > 0).all()
    pr = rb.priorities().cpu().numpy()
    np.testing.assert_array_equal(pr[i], PEROracle.td_priorities(td.cpu().numpy(), 1e-5))
    rb.close()


def test_learner_on_gpu_matches_reference(gpu):
    """The reference DDPGAgent's three replay() steps on the GPU learner
    (hipBLASLt GEMMs, fused Adam): losses within 1e-4 relative, weights
    within 2e-6 absolute of the reference's CPU result."""
    from f110_gymnasium_ros2_jazzy_amd.ddpg import DDPGLearner
    d = golden("ddpg.npz")
    ln = DDPGLearner(obs_dim=12, act_dim=2, action_low=[-0.4189, 0.0], action_high=[0.4189, 20.0], seed=42,
                     device="cuda:0", replay=None)
    S, A, R, S2, Dn = (torch.from_numpy(np.asarray(d[k])).cuda() for k in ("S", "A", "R", "S2", "D"))
    for step in range(3):
        idx = torch.from_numpy(d["idx"][step]).cuda()
        w = torch.from_numpy(d["w"][step]).cuda()
        st = ln.update(S[idx], A[idx], R[idx], S2[idx], Dn[idx].float(), w)
        np.testing.assert_allclose([float(st["critic_loss"]), float(st["actor_loss"])], d["losses"][step][:2],
                                   rtol=1e-4)
    for name, net in (("actor", ln.actor), ("critic", ln.critic), ("actor_target", ln.actor_target),
                      ("critic_target", ln.critic_target)):
        for k, v in net.state_dict().items():
            if k in ("action_low", "action_high"):
                continue
            np.testing.assert_allclose(v.cpu().numpy(), d[f"final/{name}/{k}"], rtol=1e-4, atol=2e-6,
                                       err_msg=f"{name}.{k}")


@pytest.mark.parametrize("M,D", [(4096, 1088), (333, 64), (64, 12)])
def test_explicit_update_matches_autograd(gpu, monkeypatch, M, D):
    """learner_fused.ExplicitUpdate (the learner GEMMs, no autograd) against
    the autograd learner on the same weights and batch: losses (rtol 1e-4),
    the critic's and the actor's flat gradient buckets after one update
    (|diff| <= 1e-4 |g| + 1e-5 max|g|, fp32 summation-order noise) and the
    policy's actions; then two more updates: losses still within 1e-4."""
    import f110_gymnasium_ros2_jazzy_amd.ddpg as Dd
    g = torch.Generator(device="cuda").manual_seed(M + D)
    S = torch.randn(M, D, device="cuda", generator=g)
    A = torch.rand(M, 2, device="cuda", generator=g) * torch.tensor([0.8378, 20.0], device="cuda") - \
        torch.tensor([0.4189, 0.0], device="cuda")
    R = torch.randn(M, device="cuda", generator=g)
    S2 = S + 0.1 * torch.randn(M, D, device="cuda", generator=g)
    Dn = (torch.rand(M, device="cuda", generator=g) < 0.1).float()
    W = torch.rand(M, device="cuda", generator=g) + 0.5
    runs = []
    for explicit in (True, False):
        monkeypatch.setattr(Dd, "EXPLICIT", explicit)
        ln = Dd.DDPGLearner(obs_dim=D, act_dim=2, action_low=[-0.4189, 0.0], action_high=[0.4189, 20.0], seed=1,
                            device="cuda:0", replay=None)
        assert (ln.explicit is not None) == explicit
        losses = []
        st = ln.update(S, A, R, S2, Dn, W)
        losses.append((float(st["critic_loss"]), float(st["actor_loss"])))
        grads = (ln.critic_grads.flat.clone(), ln.actor_grads.flat.clone(), st["td"].clone())
        pol = ln.choose_action(S[:100], training=False).clone()
        for _ in range(2):
            st = ln.update(S, A, R, S2, Dn, W)
            losses.append((float(st["critic_loss"]), float(st["actor_loss"])))
        runs.append((losses, grads, pol))
    np.testing.assert_allclose(runs[0][0], runs[1][0], rtol=1e-4)
    for x, y in zip(runs[0][1], runs[1][1]):
        tol = 1e-4 * y.abs() + 1e-5 * y.abs().max()
        assert bool(((x - y).abs() <= tol).all()), float(((x - y).abs() / tol).max())
    torch.testing.assert_close(runs[0][2], runs[1][2], rtol=1e-5, atol=1e-6)


def test_vector_trainer_loop(gpu):
    """The batched train_ddpg loop: 256 two-agent envs, gap-follow opponent,
    device reward, replay, learner updates after a 5-step warm-up."""
    from f110_gymnasium_ros2_jazzy_amd.train import VectorTrainer
    tr = VectorTrainer(256, batch_size=256, memory_size=4096, warmup_steps=5, seed=3)
    stored = 0
    for _ in range(30):
        tr.step()
        stored += int((tr.env.sim.out.was_reset == 0).sum())
    assert len(tr.agent.memory) == min(stored, 4096)
    st = tr.last
    assert st is not None and torch.isfinite(st["critic_loss"]) and torch.isfinite(st["actor_loss"])
    assert tr.agent.global_step == 25
    for p in tr.agent.actor.parameters():
        assert torch.isfinite(p).all()
    tr.close()


def test_learner_graphs_match_eager(gpu):
    """replay() as HIP-graph replays (graphs=True: 3 eager warm-up updates,
    then captured phases) follows the eager learner: same PER draws (device
    Philox counter), same losses and weights within fp32 tolerance."""
    from f110_gymnasium_ros2_jazzy_amd.ddpg import DDPGLearner
    g = torch.Generator(device="cuda").manual_seed(5)
    D = 64
    S = torch.randn(512, D, device="cuda", generator=g)
    A = torch.rand(512, 2, device="cuda", generator=g) * torch.tensor([0.8378, 20.0], device="cuda") - \
        torch.tensor([0.4189, 0.0], device="cuda")
    R = torch.randn(512, device="cuda", generator=g)
    S2 = S + 0.1 * torch.randn(512, D, device="cuda", generator=g)
    Dn = torch.rand(512, device="cuda", generator=g) < 0.1
    runs = []
    for graphs in (False, True):
        ln = DDPGLearner(obs_dim=D, act_dim=2, action_low=[-0.4189, 0.0], action_high=[0.4189, 20.0], seed=3,
                         device="cuda:0", memory_size=1024, batch_size=128, graphs=graphs)
        ln.remember(S, A, R, S2, Dn)
        losses = []
        for _ in range(8):
            st = ln.replay()
            losses.append((float(st["critic_loss"]), float(st["actor_loss"])))
        runs.append((losses, [p.detach().clone() for p in ln.actor.parameters()],
                     ln.memory.priorities().clone()))
        ln.memory.close()
    np.testing.assert_allclose(runs[0][0], runs[1][0], rtol=1e-4)
    for a, b in zip(runs[0][1], runs[1][1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(runs[0][2], runs[1][2], rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("n", [5000, 345_000])
def test_flat_adam_matches_torch_adam(gpu, n):
    """f110_adam_step over a flat buffer == torch.optim.Adam's single-tensor
    update (agent.py:187-188) on CPU, five steps, float32 tolerance; its fused
    soft target update == target.lerp_(param, tau) after each step.  2 blocks,
    and the critic's size (337 blocks taking tickets: the step counter advances
    once per launch and the ticket word is re-armed to 0)."""
    import ctypes
    from f110_gymnasium_ros2_jazzy_amd import _lib
    L = _lib.load()
    g = torch.Generator().manual_seed(0)
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) * 10 ** (k - 2) for k in range(5)]
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=1e-3)
    dev = p0.cuda()
    m, v = torch.zeros_like(dev), torch.zeros_like(dev)
    state = torch.zeros(2, dtype=torch.int64, device="cuda")
    tgt_ref = torch.randn(n, generator=g)
    tgt = tgt_ref.cuda()
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for gr in grads:
        ref.grad = gr.clone()
        opt.step()
        with torch.no_grad():
            tgt_ref.lerp_(ref, 0.005)
        gd = gr.cuda()
        _lib.check(L.f110_adam_step(vp(dev), vp(m), vp(v), vp(gd), dev.numel(), 1e-3, 0.9, 0.999, 1e-8, vp(state),
                                    vp(tgt), 0.005, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "adam")
        torch.cuda.synchronize()
        assert int(state[1]) == 0
    assert int(state[0]) == 5
    torch.testing.assert_close(tgt.cpu(), tgt_ref, rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(dev.cpu(), ref.detach(), rtol=2e-6, atol=1e-7)
    # CPU lerp may fuse: an ulp or two of (1 - beta1) * g, which is all of m where m cancels to ~0
    atol = 4 * torch.finfo(torch.float32).eps * 0.1 * max(float(gr.abs().max()) for gr in grads)
    torch.testing.assert_close(m.cpu(), opt.state[ref]["exp_avg"], rtol=1e-5, atol=max(atol, 1e-7))


def test_replay_add_env_matches_add(gpu):
    """add_env (f110_replay_add_env: float64 rewards, uint8 terminated and
    was_reset as the simulator writes them, reset rows skipped) stores the
    same rows, in the same ring slots, as add() with the torch conversions
    train_ddpg used (rew.to(float32), mask = ~reset); strided action rows."""
    D, A = 1088, 2
    g = torch.Generator(device="cuda").manual_seed(4)
    S = torch.rand(90, D, device="cuda", generator=g)
    S2 = torch.rand(90, D, device="cuda", generator=g)
    act_rows = torch.rand(90, 2, A, device="cuda", generator=g)  # [env, agent, 2]: agent 1's rows are strided
    Ac = act_rows[:, 1]
    R64 = torch.randn(90, device="cuda", generator=g, dtype=torch.float64) * 3.0
    term = (torch.rand(90, device="cuda", generator=g) < 0.3).to(torch.uint8)
    reset = (torch.rand(90, device="cuda", generator=g) < 0.25).to(torch.uint8)
    ra, rb = _rb(128, 32, D=D, A=A, max_add=64), _rb(128, 32, D=D, A=A, max_add=64)
    for _ in range(2):  # the second pass wraps the ring
        ra.add(S, Ac, R64.to(torch.float32), S2, term.bool(), mask=~reset.bool())
        rb.add_env(S, Ac, R64, S2, term, reset)
    assert len(ra) == len(rb)
    xa, xb = ra.arrays(), rb.arrays()
    for k in xa:
        torch.testing.assert_close(xb[k], xa[k], rtol=0, atol=0, msg=k)
    ra.close()
    rb.close()


def test_actor_explore_head(gpu):
    """f110_ddpg_actor_explore (choose_action(training=True) on the explicit
    path): sigma = 0 gives the actor head's actions clipped to the bounds;
    sigma > 0 adds N(0, sigma^2) noise (mean / std of act - actor over 65536
    x 2 draws within 4 standard errors, the two outputs uncorrelated), the
    result inside [low, high], written into a strided view; the same (sigma,
    call index) repeats, the next call index draws anew; the launch writes the
    decayed (sigma, call + 1) pair, and choose_action's host mirror follows it."""
    from f110_gymnasium_ros2_jazzy_amd.ddpg import DDPGLearner
    ln = DDPGLearner(obs_dim=64, act_dim=2, action_low=[-0.4189, 0.0], action_high=[0.4189, 20.0], seed=9,
                     device="cuda:0", replay=None, noise_sigma_start=0.2, noise_sigma_min=0.02, noise_decay=0.9)
    if ln.explicit is None:
        pytest.skip("explicit learner path not supported here")
    M = 65536
    g = torch.Generator(device="cuda").manual_seed(2)
    S = torch.randn(M, 64, device="cuda", generator=g) * 0.1
    base = ln.choose_action(S, training=False).clone()
    lo, hi = ln._low32, ln._high32
    buf = torch.full((M, 3, 2), float("nan"), device="cuda")
    out = buf[:, 1]
    ex = ln.explicit

    def st(sigma, call):
        return torch.tensor([sigma, float(call)], dtype=torch.float64, device="cuda")

    nxt = torch.zeros(2, dtype=torch.float64, device="cuda")
    a0 = ex.policy(ln.actor, S, explore=(st(0.0, 0), nxt, 0.5, 0.01, lo, hi, 7, out))
    assert a0.data_ptr() == out.data_ptr()
    torch.testing.assert_close(a0, torch.minimum(torch.maximum(base, lo), hi), rtol=0, atol=0)
    assert bool(torch.isnan(buf[:, 0]).all()) and bool(torch.isnan(buf[:, 2]).all())  # nothing else written
    assert nxt.tolist() == [0.01, 1.0]  # max(0 * 0.5, 0.01), call + 1
    sigma = 1e-3  # small enough that almost no row reaches a bound
    a1 = ex.policy(ln.actor, S, explore=(st(sigma, 5), nxt, 0.5, 0.0, lo, hi, 7, None)).clone()
    assert nxt.tolist() == [sigma * 0.5, 6.0]
    a1b = ex.policy(ln.actor, S, explore=(st(sigma, 5), nxt, 0.5, 0.0, lo, hi, 7, None)).clone()
    a2 = ex.policy(ln.actor, S, explore=(st(sigma, 6), nxt, 0.5, 0.0, lo, hi, 7, None)).clone()
    torch.testing.assert_close(a1, a1b, rtol=0, atol=0)
    assert not torch.equal(a1, a2)
    assert bool(((a1 >= lo) & (a1 <= hi)).all())
    inside = ((base > lo + 10 * sigma) & (base < hi - 10 * sigma)).all(1)
    n = (a1 - base)[inside].double() / sigma
    assert n.shape[0] > M // 2
    se = 1.0 / n.shape[0] ** 0.5
    assert float(n.mean(0).abs().max()) < 4 * se
    assert float((n.std(0) - 1.0).abs().max()) < 4 * se * 0.75 + 0.01
    assert abs(float((n[:, 0] * n[:, 1]).mean())) < 4 * se
    # choose_action: the device pair and the host mirror decay together
    for k in range(3):
        ln.choose_action(S[:256], training=True)
        torch.cuda.synchronize()
        dev = ln._noise_state[ln._noise_slot].tolist()
        assert dev == [ln.sigma, float(ln._noise_calls)] and ln._noise_calls == k + 1
    sg = 0.2
    for _ in range(3):
        sg = max(sg * 0.9, 0.02)
    assert ln.sigma == sg
    # a single observation (1-D) keeps the reference's [act_dim] shape, also into a 1-D out
    a_1d = ln.choose_action(S[7], training=False)
    assert a_1d.shape == (2,)
    torch.testing.assert_close(a_1d, base[7], rtol=0, atol=0)
    o1 = torch.empty(2, device="cuda")
    assert ln.choose_action(S[7], training=False, out=o1) is o1 and torch.equal(o1, base[7])
    assert ln.choose_action(S[7], training=True).shape == (2,)


def test_trainer_step_graphs_match_eager(gpu, monkeypatch):
    """VectorTrainer's whole-step graphs (two captured vector steps, even / odd,
    replayed after the learner's eager warm-up updates) against the same loop
    run eagerly (F110_STEP_GRAPH=0): after 14 steps the actor / critic weights,
    the replay ring, the noise state and the last losses are bit-identical, and
    so are the losses after 13 steps (an even-parity replay: each parity's
    graph keeps its own loss outputs)."""
    from f110_gymnasium_ros2_jazzy_amd.train import VectorTrainer
    runs = []
    l13 = []
    for flag in ("1", "0"):
        monkeypatch.setenv("F110_STEP_GRAPH", flag)
        tr = VectorTrainer(256, batch_size=256, memory_size=4096, warmup_steps=3, seed=11)
        for _ in range(13):
            tr.step()
        l13.append((float(tr.last["critic_loss"]), float(tr.last["actor_loss"])))
        tr.step()
        torch.cuda.synchronize()
        assert (tr._sg[0] is not None and tr._sg[1] is not None) == (flag == "1")
        ag = tr.agent
        params = [p.detach().clone() for p in list(ag.actor.parameters()) + list(ag.critic.parameters())]
        n = len(ag.memory)  # rows past the length were never written
        ring = {k: v[:n].clone() for k, v in ag.memory.arrays().items()}
        runs.append((params, ring, float(tr.last["critic_loss"]), float(tr.last["actor_loss"]), ag.sigma,
                     ag._noise_calls, tr.obs.clone(), len(ag.memory), ag.global_step))
        tr.close()
    (pa, ra, ca, aa, sa, na, oa, la, ga), (pb, rb_, cb, ab, sb, nb, ob, lb, gb) = runs
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)
    for k in ra:
        assert torch.equal(ra[k], rb_[k]), k
    assert (ca, aa, sa, na, la, ga) == (cb, ab, sb, nb, lb, gb)
    assert torch.equal(oa, ob)
    assert l13[0] == l13[1]
