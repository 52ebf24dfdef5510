"""BASELINE.json's GPU configurations at their own sizes (SURVEY §8 config
shorthand): C3 65 536 single-agent envs, C4 8192 envs x 2 agents, C5 the
batched train_ddpg loop at its per-GPU share (32 768 / 8 = 4096 two-agent
envs).  Size-independent properties at full size, plus an oracle-compared
sample stepped in lock-step (base_classes.py:566-625 Simulator.step)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _actions(gen, E, A, device):
    a = torch.rand(E, A, 2, device=device, generator=gen, dtype=torch.float32)
    a[..., 0] = a[..., 0] * 0.8378 - 0.4189   # steer in [-0.4189, 0.4189]
    a[..., 1] *= 20.0                          # speed in [0, 20] (ddpg_config.yaml:19-20)
    return a


def test_c3_65536_single_agent(tracks, gpu, oracle_scanners):
    """C3 on one GPU: 65 536 single-agent envs (the metric's configuration),
    noise off, autoreset on, 20 random-action steps.  Every range in
    [0, 30], every lookup counted (rays == steps x envs x beams, mean lookups
    per ray in the measured band), obs finite; a 512-env sample of the last
    step's scans bit-exact against the oracle scanner at the cars' post-step
    poses (cars whose TTC fired are skipped: their yaw was zeroed after the
    scan, base_classes.py:246-249)."""
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    E, T = 65536, 20
    sp = centerline_spawns("Spielberg", 1)
    sim = BatchSim(tracks("Spielberg_map"), n_envs=E, n_agents=1, device=gpu, noise_std=0.0, autoreset=True,
                   spawn_poses=sp, keep_f64_scans=True)
    assert sim.ray_kernel == 3
    rng = np.random.default_rng(65536)
    sim.set_simt(True)  # k_rays_fxs counts lookups / rays while counting is on
    sim.reset(sp[rng.integers(0, sp.shape[0], E)])
    sim.reset_counters()
    g = torch.Generator(device=gpu)
    g.manual_seed(33)
    for _ in range(T):
        out = sim.step(_actions(g, E, 1, gpu))
    torch.cuda.synchronize()
    s = out.scans_f64
    assert bool(((s >= 0) & (s <= 30)).all())
    assert bool(torch.isfinite(out.obs).all())
    assert bool(((out.obs[:, :1080] >= 0) & (out.obs[:, :1080] <= 1)).all())
    lk, rays = sim.read_counters()
    assert rays == T * E * 1080
    assert 4.0 < lk / rays < 15.0
    idx = rng.choice(E, 512, replace=False)
    ok = out.collisions[idx, 0].cpu().numpy() == 0
    st = sim.agent_states()[idx, 0].cpu().numpy()[ok]
    ref = oracle_scanners("Spielberg_map").scan(np.stack([st[:, 0], st[:, 1], st[:, 4]], 1))
    assert ok.sum() > 400
    assert np.array_equal(s[idx, 0].cpu().numpy()[ok], ref)
    sim.close()


def test_c2_4096_single_agent(tracks, gpu, oracle_scanners):
    """C2: 4096 single-agent envs on one GPU, stepped by the bench's own runner
    for that size (bench.auto_streams: StreamShards, 4 unjoined sub-shards)
    AND by one context, 20 random-action steps with autoreset (noise off).
    The two runners agree bit for bit (obs, f64 scans, states, lookup
    counts); every range in [0, 30], mean lookups per ray in the measured
    band; a 512-env sample of the last step's scans bit-exact against the
    oracle scanner at the cars' post-step poses (TTC-fired cars skipped)."""
    import bench
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards
    E, T = 4096, 20
    S = bench.auto_streams(E, 1)
    assert S == 4
    sp = centerline_spawns("Spielberg", 1)
    kw = dict(n_agents=1, device=gpu, noise_std=0.0, autoreset=True, spawn_poses=sp, keep_f64_scans=True)
    shards = StreamShards(tracks("Spielberg_map"), n_envs=E, n_streams=S, **kw)
    one = BatchSim(tracks("Spielberg_map"), n_envs=E, **kw)
    rng = np.random.default_rng(4096)
    p0 = sp[rng.integers(0, sp.shape[0], E)]
    shards.set_simt(True)  # k_rays_fxs counts lookups / rays while counting is on
    one.set_simt(True)
    shards.reset(p0)
    one.reset(p0)
    shards.reset_counters()
    one.reset_counters()
    g = torch.Generator(device=gpu)
    g.manual_seed(22)
    acts = torch.stack([_actions(g, E, 1, gpu) for _ in range(T)])
    for t in range(T):
        shards.step(acts[t], minimal_outputs=False)
        out = one.step(acts[t])
    shards.join()
    torch.cuda.synchronize()
    assert torch.equal(shards.obs, out.obs)
    assert torch.equal(torch.cat([sm.out.scans_f64 for sm in shards.sims]), out.scans_f64)
    assert torch.equal(torch.cat([sm.agent_states() for sm in shards.sims]), one.agent_states())
    lk, rays = one.read_counters()
    assert shards.read_counters() == (lk, rays)
    assert rays == T * E * 1080 and 4.0 < lk / rays < 15.0
    s = out.scans_f64
    assert bool(((s >= 0) & (s <= 30)).all()) and bool(torch.isfinite(out.obs).all())
    idx = rng.choice(E, 512, replace=False)
    ok = out.collisions[idx, 0].cpu().numpy() == 0
    st = one.agent_states()[idx, 0].cpu().numpy()[ok]
    ref = oracle_scanners("Spielberg_map").scan(np.stack([st[:, 0], st[:, 1], st[:, 4]], 1))
    assert ok.sum() > 400
    assert np.array_equal(s[idx, 0].cpu().numpy()[ok], ref)
    shards.close()
    one.close()


def test_c4_8192x2_lockstep_sample(tracks, gpu, oracle_scanners, nonexact_budget):
    """C4: 8192 envs x 2 agents on one GPU, 20 random-action steps (noise
    off, no autoreset).  The first 256 envs are stepped by the oracle in
    lock-step with the same actions (the oracle's state re-synced to the
    device's after each step, so ulp-level trig differences do not
    accumulate): states within 1e-10, collisions equal, scans bit-exact but
    for agent ray_cast beams (recorded budget).  The sample holds GJK
    overlaps (opponents spawned 1-3 centerline points apart) and agent
    occlusions (10-30 points apart), both asserted present."""
    import oracle as O
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    E, A, S, T = 8192, 2, 256, 20
    cl = centerline_spawns("Spielberg", 1)[:, 0]
    rng = np.random.default_rng(8192)
    n = cl.shape[0]
    i0 = rng.integers(0, n, E)
    gap = np.where(np.arange(E) % 2 == 0, rng.integers(1, 4, E), rng.integers(10, 31, E))
    poses = np.stack([cl[i0], cl[(i0 + gap) % n]], 1)
    sim = BatchSim(tracks("Spielberg_map"), n_envs=E, n_agents=A, device=gpu, noise_std=0.0, keep_f64_scans=True)
    sim.set_handoff_check(1)  # hand-off buffer NaN-poisoned per step, reads outside the mask counted
    sim.reset_counters()
    ref = O.OracleSim(oracle_scanners("Spielberg_map"), S, A)
    # residue attribution: the oracle with the device's correctly rounded sin / cos
    refd = O.OracleSim(oracle_scanners("Spielberg_map"), S, A)
    sim.reset(poses)
    ref.reset(poses[:S])
    rs, rc = ref.step(np.zeros((S, A, 2)))
    with O.device_trig():
        refd.reset(poses[:S])
        rd, _ = refd.step(np.zeros((S, A, 2)))
    g = torch.Generator(device=gpu)
    g.manual_seed(44)
    nonexact = nonexact_d = gjk = occluded = 0
    clean = BatchSim(tracks("Spielberg_map"), n_envs=S, n_agents=1, device=gpu, noise_std=0.0)
    for t in range(T + 1):
        if t:
            act = _actions(g, E, A, gpu)
            out = sim.step(act)
            rs, rc = ref.step(act[:S].double().cpu().numpy())
            with O.device_trig():
                rd, _ = refd.step(act[:S].double().cpu().numpy())
        else:
            out = sim.out
        torch.cuda.synchronize()
        st = sim.agent_states().cpu().numpy()
        np.testing.assert_allclose(st[:S].reshape(S * A, 7), ref.state, rtol=1e-10, atol=1e-10)
        sc = out.scans_f64[:S].cpu().numpy()
        np.testing.assert_allclose(sc, rs, rtol=1e-9, atol=1e-9)
        nonexact += int(np.sum(sc != rs))
        nonexact_d += int(np.sum(sc != rd))
        col = out.collisions[:S].cpu().numpy()
        assert np.array_equal(col, rc.astype(np.uint8)), t
        gjk += int(col.all(1).sum())
        # occlusion: agent 0's scan shorter than the map-only scan at the same pose
        p0 = st[:S, 0]
        bare = clean.scan_batch(np.stack([p0[:, 0], p0[:, 1], p0[:, 4]], 1)).cpu().numpy()
        live = col[:, 0] == 0  # a TTC response zeroes the yaw after the scan
        occluded += int(np.sum(sc[live, 0] < bare[live]))
        ref.state[:] = st[:S].reshape(S * A, 7)
        refd.state[:] = ref.state
        # the rest of the batch: ranges in [0, 30], obs finite
        full = out.scans_f64
        assert bool(((full >= 0) & (full <= 30)).all()) and bool(torch.isfinite(out.obs).all())
    assert gjk > 0 and occluded > 0, (gjk, occluded)
    assert sim.read_counter(6) == 0, "k_post_multi read hand-off beams outside the mask"
    nonexact_budget("c4_8192x2_sample256_20steps", nonexact)
    nonexact_budget("c4_8192x2_sample256_20steps/device_trig_oracle", nonexact_d)
    clean.close()
    sim.close()


def test_c5_vector_trainer_4096(gpu):
    """C5's per-GPU share of the batched train_ddpg loop: 4096 two-agent envs
    (gap-follow opponent, device reward, PER replay, one learner update of
    4096 rows per vector step after a 3-step warm-up), 8 vector steps.
    Losses finite, weights finite and moved, and a re-run from the same seeds
    reproduces every loss and weight bit for bit."""
    from f110_gymnasium_ros2_jazzy_amd.train import VectorTrainer
    runs = []
    for _ in range(2):
        tr = VectorTrainer(4096, batch_size=4096, memory_size=1 << 16, warmup_steps=3, seed=5)
        w0 = [p.detach().clone() for p in tr.agent.actor.parameters()]
        losses = []
        for _ in range(8):
            tr.step()
            if tr.last is not None:
                losses.append((float(tr.last["critic_loss"]), float(tr.last["actor_loss"])))
        torch.cuda.synchronize()
        assert tr.agent.global_step == 5 and len(losses) == 5
        assert all(np.isfinite(c) and np.isfinite(a) for c, a in losses)
        actor = [p.detach().clone() for p in tr.agent.actor.parameters()]
        critic = [p.detach().clone() for p in tr.agent.critic.parameters()]
        assert all(bool(torch.isfinite(p).all()) for p in actor + critic)
        assert any(not torch.equal(a, b) for a, b in zip(actor, w0))
        runs.append((losses, actor, critic))
        tr.close()
    (l0, a0, c0), (l1, a1, c1) = runs
    assert l0 == l1
    assert all(torch.equal(x, y) for x, y in zip(a0 + c0, a1 + c1))
