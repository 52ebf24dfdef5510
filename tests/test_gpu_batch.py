"""GPU batch semantics: env independence, global-id RNG keying (sharding
invariance), scan-noise statistics, autoreset, full-size properties."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _spawns(A=1):
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    return centerline_spawns("Spielberg", A)


def _sim(tracks, gpu, **kw):
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    return BatchSim(tracks("Spielberg_map"), device=gpu, **kw)


def test_env_independence_and_shard_invariance(tracks, gpu):
    """A 2-way split of 32 envs (env_offset) reproduces the 32-env run bit for
    bit, noise and autoreset included: trajectories do not depend on how the
    batch is sharded over GPUs."""
    E, A = 32, 1
    sp = _spawns(A)
    rng = np.random.default_rng(5)
    poses = sp[rng.integers(0, sp.shape[0], E)]
    acts = np.stack([rng.uniform(-0.4189, 0.4189, (40, E, A)), rng.uniform(0, 20, (40, E, A))], -1).astype(np.float32)
    full = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=9)
    halves = [_sim(tracks, gpu, n_envs=E // 2, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=9,
                   env_offset=h * (E // 2)) for h in range(2)]
    full.reset(poses)
    for h in range(2):
        halves[h].reset(poses[h * 16:(h + 1) * 16])
    for t in range(40):
        of = full.step(acts[t]).obs.cpu().numpy()
        oh = np.concatenate([halves[h].step(acts[t, h * 16:(h + 1) * 16]).obs.cpu().numpy() for h in range(2)])
        assert np.array_equal(of, oh), t


def test_noise_statistics(tracks, gpu):
    """Scan noise (laser_models.py:450-452): N(0, 0.01) added after the clamp,
    identical for every agent of an env (all RaceCars share the seed,
    base_classes.py:119,204), restarted at reset, different across envs."""
    E, A = 16, 2
    sp = _spawns(A)[::300][:E]
    clean = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.0, keep_f64_scans=True)
    noisy = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.01, keep_f64_scans=True, seed=42)
    zero = np.zeros((E, A, 2), np.float32)
    n1 = noisy.reset(sp).scans_f64.cpu().numpy() - clean.reset(sp).scans_f64.cpu().numpy()
    # agents share the stream; ray_cast occlusion only lowers ranges -> compare unoccluded beams
    same = np.abs(n1[:, 0] - n1[:, 1]) < 1e-12
    assert same.mean() > 0.9
    assert abs(n1.mean()) < 5e-4 and abs(n1.std() - 0.01) < 5e-4
    # beams b and b + 64 of a 128-beam block take the two outputs of one Box-Muller draw: uncorrelated
    blk = n1[:, 0, :1024].reshape(E, 8, 2, 64)
    lo, hi = blk[:, :, 0].ravel(), blk[:, :, 1].ravel()
    ok = (np.abs(lo) < 0.1) & (np.abs(hi) < 0.1)  # noise is cut at 5.8 sigma; drop occluded beams
    assert ok.mean() > 0.95
    assert abs(np.corrcoef(lo[ok], hi[ok])[0, 1]) < 0.05
    assert abs(np.corrcoef(lo[ok] ** 2, hi[ok] ** 2)[0, 1]) < 0.05
    assert not np.allclose(n1[0, 0], n1[1, 0])     # different envs, different streams
    n2 = noisy.step(zero).scans_f64.cpu().numpy() - clean.step(zero).scans_f64.cpu().numpy()
    assert not np.allclose(n1[:, 0], n2[:, 0])     # next step, next draw
    n3 = noisy.reset(sp).scans_f64.cpu().numpy() - clean.reset(sp).scans_f64.cpu().numpy()
    assert np.array_equal(n1, n3)                  # re-seeded at reset


def test_autoreset(tracks, gpu):
    """A terminated env (ego collision) is reset at its next step from the
    spawn table; the reset step ignores the action (F110Env.reset semantics)."""
    E, A = 8, 1
    sp = _spawns(A)
    sim = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.0, autoreset=True, spawn_poses=sp)
    sim.reset(sp[:E * 50:50])
    crash = np.tile([[[0.4189, 20.0]]], (E, 1, 1)).astype(np.float32)
    seen_term = np.zeros(E, bool)
    seen_reset_after = np.zeros(E, bool)
    prev_term = np.zeros(E, bool)
    for t in range(400):
        out = sim.step(crash)
        term = out.terminated.cpu().numpy().astype(bool)
        was = out.was_reset.cpu().numpy().astype(bool)
        assert np.array_equal(was, prev_term)   # reset happens exactly one step after termination
        if was.any():
            st = sim.agent_states().cpu().numpy()[was, 0]
            assert np.all(np.abs(st[:, 3]) < 1.0)  # fresh car: speed ~0 after the zero step
            assert np.allclose(out.sim_time.cpu().numpy()[was], 0.01)
            seen_reset_after |= was
        seen_term |= term
        prev_term = term
    assert seen_term.all() and seen_reset_after.all()


def test_full_size_properties(tracks, gpu):
    """BASELINE-size shard (8192 envs): ranges in [0, 30] (noise-free),
    lookups/ray in the expected band, obs finite, sample bit-exact vs oracle."""
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    import oracle as O
    E = 8192
    sp = _spawns(1)
    sim = BatchSim(tracks("Spielberg_map"), n_envs=E, n_agents=1, device=gpu, noise_std=0.0, autoreset=True,
                   spawn_poses=sp, keep_f64_scans=True)
    rng = np.random.default_rng(1)
    sim.reset(sp[rng.integers(0, sp.shape[0], E)])
    sim.set_simt(True)  # k_rays_fxs counts lookups / rays while counting is on
    sim.reset_counters()
    g = torch.Generator(device=gpu)
    g.manual_seed(3)
    for _ in range(50):
        a = torch.rand(E, 1, 2, device=gpu, generator=g)
        a[..., 0] = a[..., 0] * 0.8378 - 0.4189
        a[..., 1] *= 20
        out = sim.step(a)
    torch.cuda.synchronize()
    s = out.scans_f64
    assert bool(((s >= 0) & (s <= 30)).all())
    assert bool(torch.isfinite(out.obs).all())
    lk, rays = sim.read_counters()
    assert rays == 50 * E * 1080
    assert 4.0 < lk / rays < 15.0
    ok = out.collisions[:512, 0].cpu().numpy() == 0   # TTC zeroes yaw after the scan
    st = sim.agent_states()[:512, 0].cpu().numpy()[ok]
    poses = np.stack([st[:, 0], st[:, 1], st[:, 4]], 1)
    ref = O.OracleScanner(tracks("Spielberg_map").free_mask, tracks("Spielberg_map").resolution,
                          tracks("Spielberg_map").origin).scan(poses)
    assert ok.sum() > 100
    assert np.array_equal(s[:512, 0].cpu().numpy()[ok], ref)


@pytest.mark.parametrize("A", [1, 2])
def test_ray_kernel_dispatch_variants_identical(tracks, gpu, monkeypatch, A):
    """The ray-kernel dispatches (F110_RAY_KERNEL: 1 k_rays_tiled in flat ray
    order, 2 tiled chunked in descending chunk order, 3 the fixed-point
    kernels -- the default -- with 1 ray per lane (k_rays_fx) and 2
    (k_rays_fxn on the padded table, or, F110_FX_PAD=0, the clamped one))
    give bit-identical steps: scans, obs, collisions, states, with noise,
    autoreset and a masked reset."""
    E = 300  # not a multiple of 4 cars per chunked block
    sp = _spawns(A)
    rng = np.random.default_rng(7)
    poses = sp[rng.integers(0, sp.shape[0], E)]
    acts = np.stack([rng.uniform(-0.4189, 0.4189, (30, E, A)), rng.uniform(0, 20, (30, E, A))], -1).astype(np.float32)
    mask = rng.random(E) < 0.5
    outs = []
    for k, lanes, pad in (("1", 1, "1"), ("2", 1, "1"), ("3", 1, "1"), ("3", 2, "1"), ("3", 2, "0")):
        monkeypatch.setenv("F110_RAY_KERNEL", k)
        monkeypatch.setenv("F110_FX_PAD", pad)  # k_rays_fxn on the padded table (1) or the clamped one (0)
        sim = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=4,
                   keep_f64_scans=True)
        assert sim.ray_kernel == int(k)
        if k == "3":
            sim.set_ray_lanes(lanes)
        sim.reset(poses)
        rec = []
        for t in range(30):
            if t == 15:
                o = sim.reset(poses[::-1].copy(), env_mask=mask)
            else:
                o = sim.step(acts[t])
            rec.append((o.scans_f64.clone(), o.obs.clone(), o.collisions.clone(), sim.agent_states().clone()))
        torch.cuda.synchronize()
        outs.append(rec)
        sim.close()
    for rec in outs[1:]:
        for t, (a, b) in enumerate(zip(outs[0], rec)):
            for x, y in zip(a, b):
                assert torch.equal(x, y), f"step {t}"


@pytest.mark.parametrize("lanes,refill", [(1, 0), (2, 0), (2, 1)])
def test_stream_shards_match_single_context(tracks, gpu, lanes, refill):
    """streams.StreamShards (bench.py's default timed runner): 4 sub-shards on
    4 dedicated-queue streams, never joined between steps, end bit-identical
    to one context stepping all envs (noise and autoreset on; the actions are
    resident before the loop, as in the bench), with the sub-shards' map
    tables shared and 1 or 2 rays per lane (f110_debug_set_ray_lanes), and with
    k_rays_fxs switched on per sub-shard (f110_debug_set_ray_refill)."""
    from f110_gymnasium_ros2_jazzy_amd import _lib
    from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards
    E, A, T = 256, 1, 60
    sp = _spawns(A)
    rng = np.random.default_rng(11)
    poses = sp[rng.integers(0, sp.shape[0], E)]
    acts = torch.tensor(np.stack([rng.uniform(-0.4189, 0.4189, (T, E, A)), rng.uniform(0, 20, (T, E, A))], -1),
                        dtype=torch.float32, device=gpu)
    full = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=9)
    sh = StreamShards(tracks("Spielberg_map"), n_envs=E, n_streams=4, ray_lanes=lanes, refill=refill,
                      n_agents=A, device=gpu, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=9)
    assert all(sm.ray_lanes == lanes for sm in sh.sims)
    assert all(sm.ray_refill == refill for sm in sh.sims)  # f110_debug_set_ray_refill (k_rays_fxs + padded EDT)
    full.set_simt(True)  # k_rays_fxs counts lookups / rays while counting is on
    sh.set_simt(True)
    full.reset(poses)
    sh.reset(poses)
    with pytest.raises(RuntimeError, match="before the first"):
        _lib.check(sh.sims[0].L.f110_debug_set_ray_lanes(sh.sims[0].ctx, 1), "f110_debug_set_ray_lanes")
    for t in range(T):
        full.step(acts[t], minimal_outputs=True)
        sh.step(acts[t], minimal_outputs=True)
    assert torch.equal(sh.obs, full.out.obs)
    assert sh.read_counters() == full.read_counters()
    sh.close()


@pytest.mark.parametrize("caller", ["null", "torch_stream"])
def test_stream_shards_policy_loop(tracks, gpu, caller):
    """A policy-style loop on StreamShards: actions drawn with torch.rand on
    the caller's stream every step (then freed), obs read (torch.cat on the
    caller's stream) every step.  On the legacy null stream the ordering is
    implicit; on a torch stream step() orders the sub-streams after it and
    holds the action tensor until their kernels are done.  Either way every
    per-step obs equals one BatchSim's, bit for bit."""
    import contextlib
    from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards
    ctx = torch.cuda.stream(torch.cuda.Stream(device=gpu)) if caller == "torch_stream" else contextlib.nullcontext()
    with ctx:
        _policy_loop(tracks, gpu, StreamShards)


def _policy_loop(tracks, gpu, StreamShards):
    E, A, T = 512, 1, 40
    sp = _spawns(A)
    rng = np.random.default_rng(12)
    poses = sp[rng.integers(0, sp.shape[0], E)]
    full = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=3)
    sh = StreamShards(tracks("Spielberg_map"), n_envs=E, n_streams=2,
                      n_agents=A, device=gpu, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=3)
    full.reset(poses)
    sh.reset(poses)
    g = torch.Generator(device=gpu)
    g.manual_seed(5)
    for t in range(T):
        a = torch.rand(E, A, 2, device=gpu, generator=g)
        a[..., 0] = a[..., 0] * 0.8378 - 0.4189
        a[..., 1] *= 20
        o_sh = sh.step(a) or sh.obs          # the obs of THIS step (join + cat on the caller's stream)
        o_full = full.step(a.clone()).obs.clone()
        del a                                 # freed on the caller's stream while the sub-streams may still read it
        junk = torch.full((E, A, 2), float("nan"), device=gpu)  # would land in the freed block
        assert torch.equal(o_sh, o_full), f"step {t}"
        del junk
    sh.close()
    sh.close()  # idempotent


def test_stream_shards_broadcast_reset(tracks, gpu):
    """StreamShards.reset accepts BatchSim's broadcast [A, 3] pose."""
    from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards
    E, A = 64, 2
    sp = _spawns(A)
    sh = StreamShards(tracks("Spielberg_map"), n_envs=E, n_streams=2, n_agents=A, device=gpu, noise_std=0.0)
    full = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.0)
    sh.reset(sp[100])
    full.reset(sp[100])
    assert torch.equal(sh.obs, full.out.obs)
    sh.close()


@pytest.mark.parametrize("beams,A", [(64, 1), (333, 2), (2048, 1), (1080, 3)])
def test_rays_per_lane_identical_across_beam_counts(tracks, gpu, beams, A):
    """k_rays_fxn (2 rays per lane) against k_rays_fx (1) for scan sizes whose
    64-beam chunks do not pair evenly (1, 6, 32 chunks; 17 with three agents):
    scans, obs, collisions and states bit-identical over 25 noisy steps with
    autoreset and a masked reset."""
    E = 96
    sp = _spawns(A)
    rng = np.random.default_rng(beams)
    poses = sp[rng.integers(0, sp.shape[0], E)]
    acts = np.stack([rng.uniform(-0.4189, 0.4189, (25, E, A)), rng.uniform(0, 20, (25, E, A))], -1).astype(np.float32)
    mask = rng.random(E) < 0.5
    outs = []
    for lanes in (1, 2):
        sim = _sim(tracks, gpu, n_envs=E, n_agents=A, num_beams=beams, noise_std=0.01, autoreset=True,
                   spawn_poses=sp, seed=9, keep_f64_scans=True)
        sim.set_ray_lanes(lanes)
        assert sim.ray_kernel == 3 and sim.ray_lanes == lanes
        sim.reset(poses)
        rec = []
        for t in range(25):
            o = sim.reset(poses[::-1].copy(), env_mask=mask) if t == 12 else sim.step(acts[t])
            rec.append((o.scans_f64.clone(), o.obs.clone(), o.collisions.clone(), sim.agent_states().clone()))
        torch.cuda.synchronize()
        outs.append(rec)
        sim.close()
    for rec in outs[1:]:
        for t, (a, b) in enumerate(zip(outs[0], rec)):
            for x, y in zip(a, b):
                assert torch.equal(x, y), f"step {t}"


@pytest.mark.parametrize("lanes,refill,shared", [(1, 0, False), (2, 0, False), (2, 1, False), (2, 1, True)])
def test_simt_counters(tracks, gpu, lanes, refill, shared):
    """f110_debug_set_simt / f110_debug_read_simt: the fixed-point loops count the lane
    slots of the gathers they issue (64 per wave-level gather: trip count x
    rays per lane, or k_rays_fxs's trips x 2 slots, closed slots included);
    loop lookups = all lookups less the first lookup of each ray (k_agents'),
    and never exceed the slots.  k_rays_fxs also counts its other vector loads
    (counter 3: the arms' theta-table loads, TTC tables, guard-band re-gathers,
    run searches).  A context sharing the device (f110_set_device_share with
    two contexts) runs the kernel with the theta table in LDS: each wave counts
    its share of its block's LDS copy, and fewer than one load per arm plus the
    shares; alone, at least one load per arm."""
    from f110_gymnasium_ros2_jazzy_amd import _lib
    E, A = 512, 1
    sp = _spawns(A)
    rng = np.random.default_rng(3)
    sim = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=2)
    if shared:
        _lib.check(sim.L.f110_set_device_share(sim.ctx, 2 * E * A, 2), "f110_set_device_share")
    sim.set_ray_lanes(lanes)
    sim.set_ray_refill(refill)
    assert sim.ray_kernel == 3 and sim.ray_lanes == lanes and sim.ray_refill == refill
    sim.reset(sp[rng.integers(0, sp.shape[0], E)])
    sim.set_simt(True)
    sim.reset_counters()
    for t in range(5):
        sim.step(np.stack([rng.uniform(-0.4, 0.4, (E, A)), rng.uniform(0, 20, (E, A))], -1).astype(np.float32))
    lookups, rays = sim.read_counters()
    loop, slots = sim.read_simt()
    assert rays == 5 * E * A * sim.B
    assert loop == lookups - rays
    assert 0 < loop <= slots
    assert 0.2 < loop / slots <= 1.0
    other = sim.read_counter(3)
    nch = (sim.B + 63) // 64
    if refill and shared:
        waves = E * A * refill  # refill = waves per car here (set_ray_refill)
        share = -(-2000 // 512)  # theta_dis entries over a block's 512 threads
        assert 5 * waves * share <= other < 5 * waves * share + 5 * E * A * nch
    elif refill:  # one load per arm, at most one TTC table load per chunk, the run searches
        assert 5 * E * A * nch <= other < 5 * E * A * (2 * nch + 8)
    sim.set_simt(False)
    sim.step(np.zeros((E, A, 2), np.float32))
    assert sim.read_simt()[1] == slots  # off: no lane slots added
    sim.close()


@pytest.mark.parametrize("A,beams", [(1, 1080), (2, 1080), (1, 333), (1, 64)])
def test_refill_kernel_identical(tracks, gpu, monkeypatch, A, beams):
    """k_rays_fxs (f110_debug_set_ray_refill: one wave per car, two chunk slots, a
    slot refilled with the car's next chunk as soon as its chunk ends; 1 and
    3 waves per car) against k_rays_fxn's adjacent pairs on the clamped and
    the padded table: scans, obs, collisions and states bit-identical over 25
    noisy steps with autoreset and a masked reset (which runs k_rays_fxn), for
    17, 6 and 1 chunks per car; the counters (lookups, rays) equal."""
    E = 200
    sp = _spawns(A)
    rng = np.random.default_rng(beams + A)
    poses = sp[rng.integers(0, sp.shape[0], E)]
    acts = np.stack([rng.uniform(-0.4189, 0.4189, (25, E, A)), rng.uniform(0, 20, (25, E, A))], -1).astype(np.float32)
    mask = rng.random(E) < 0.5
    outs, ctrs = [], []
    for refill, pad in ((0, "0"), (0, "1"), (1, "1"), (3, "1")):
        monkeypatch.setenv("F110_FX_PAD", pad)
        sim = _sim(tracks, gpu, n_envs=E, n_agents=A, num_beams=beams, noise_std=0.01, autoreset=True,
                   spawn_poses=sp, seed=6, keep_f64_scans=True)
        sim.set_ray_lanes(2)
        sim.set_ray_refill(refill)
        sim.set_simt(True)  # k_rays_fxs counts lookups / rays while counting is on
        assert sim.ray_refill == min(refill, (beams + 63) // 64)
        sim.reset(poses)
        sim.reset_counters()
        rec = []
        for t in range(25):
            o = sim.reset(poses[::-1].copy(), env_mask=mask) if t == 12 else sim.step(acts[t])
            rec.append((o.scans_f64.clone(), o.obs.clone(), o.collisions.clone(), sim.agent_states().clone()))
        torch.cuda.synchronize()
        outs.append(rec)
        ctrs.append(sim.read_counters())
        sim.close()
    for k in range(1, len(outs)):
        assert ctrs[0] == ctrs[k]
        for t, (a, b) in enumerate(zip(outs[0], outs[k])):
            for x, y in zip(a, b):
                assert torch.equal(x, y), f"step {t}"


def test_step_n_matches_single_steps(tracks, gpu):
    """f110_step_n (n resident steps, no host work in between) equals n
    f110_step calls: obs, scans, states and counters bit-identical, f32 and
    f64 action blocks."""
    E, A, T = 203, 1, 11
    sp = _spawns(A)
    rng = np.random.default_rng(21)
    poses = sp[rng.integers(0, sp.shape[0], E)]
    acts = np.stack([rng.uniform(-0.4189, 0.4189, (T, E, A)), rng.uniform(0, 20, (T, E, A))], -1)
    for dt in (np.float32, np.float64):
        a = torch.from_numpy(acts.astype(dt)).to(gpu)
        runs = []
        for n_call in (False, True):
            sim = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=9,
                       keep_f64_scans=True)
            sim.set_simt(True)  # k_rays_fxs counts lookups / rays while counting is on
            sim.reset(poses)
            sim.reset_counters()
            if n_call:
                o = sim.step_n(a)
            else:
                for t in range(T):
                    o = sim.step(a[t])
            torch.cuda.synchronize()
            runs.append((o.obs.clone(), o.scans_f64.clone(), sim.agent_states().clone(), sim.read_counters()))
            sim.close()
        for x, y in zip(runs[0][:3], runs[1][:3]):
            assert torch.equal(x, y)
        assert runs[0][3] == runs[1][3]


@pytest.mark.parametrize("A", [1, 2])
def test_counting_build_identical(tracks, gpu, A):
    """k_rays_fxs's counting build (f110_debug_set_simt on: lookups, rays, lane
    slots) and its uncounted build (the default: no per-trip bookkeeping) step
    the same bits (obs, f64 scans, states, collisions over 20 noisy steps with
    autoreset); the uncounted build adds nothing to the counters."""
    E, T = 384, 20
    sp = _spawns(A)
    rng = np.random.default_rng(77 + A)
    poses = sp[rng.integers(0, sp.shape[0], E)]
    acts = np.stack([rng.uniform(-0.4189, 0.4189, (T, E, A)), rng.uniform(0, 20, (T, E, A))], -1).astype(np.float32)
    runs = []
    for counting in (False, True):
        sim = _sim(tracks, gpu, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=5,
                   keep_f64_scans=True)
        assert sim.ray_kernel == 3 and sim.ray_refill > 0  # k_rays_fxs
        sim.set_simt(counting)
        sim.reset(poses)
        sim.reset_counters()
        rec = []
        for t in range(T):
            o = sim.step(acts[t])
            rec.append((o.obs.clone(), o.scans_f64.clone(), o.collisions.clone(), sim.agent_states().clone()))
        torch.cuda.synchronize()
        lk, rays = sim.read_counters()
        if counting:
            assert rays == T * E * A * sim.B and lk > 4 * rays
        else:
            assert (lk, rays) == (0, 0)
        runs.append(rec)
        sim.close()
    for t, (a, b) in enumerate(zip(*runs)):
        for x, y in zip(a, b):
            assert torch.equal(x, y), f"step {t}"
