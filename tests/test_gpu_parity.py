"""GPU parity: libf110 kernels (through the C ABI) vs the golden vectors and
the CPU oracle.  Bars: bit-exact scans, lookup counts and hit cells;
dynamics within 1e-12 relative (ocml vs glibc transcendentals differ by an
ulp; north star allows 1e-5)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

PKEYS = ["mu", "C_Sf", "C_Sr", "lf", "lr", "h", "m", "I", "s_min", "s_max", "sv_min", "sv_max", "v_switch",
         "a_max", "v_min", "v_max"]


@pytest.fixture(scope="module")
def sims(gpu, tracks):
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    cache = {}

    def get(map_name, E=1, A=1, **kw):
        key = (map_name, E, A, repr(sorted(kw.items())))
        if key not in cache:
            kw.setdefault("noise_std", 0.0)
            cache[key] = BatchSim(tracks(map_name), n_envs=E, n_agents=A, device=gpu, keep_f64_scans=True, **kw)
        return cache[key]
    return get


@pytest.mark.parametrize("m", ["Spielberg_map", "straight_corridor", "Shanghai_map"])
def test_scan_batch_golden(sims, m):
    g = golden(f"scans_{m}.npz")
    sim = sims(m)
    scans = sim.scan_batch(g["poses"]).cpu().numpy()
    assert np.array_equal(scans, g["scans"])
    s2, look, rc = sim.scan_batch(g["poses"], probe=True)
    assert np.array_equal(s2.cpu().numpy(), g["scans"])
    assert np.array_equal(look.cpu().numpy(), g["lookups"])
    assert np.array_equal(rc.cpu().numpy(), g["hit_rc"])


@pytest.fixture(scope="module")
def rotated(gpu, tracks):
    """Spielberg with map-origin yaw 0.35 rad (the rotated-map kernel variants)."""
    import dataclasses
    g = golden("scans_Spielberg_rot.npz")
    return dataclasses.replace(tracks("Spielberg_map"), origin=tuple(float(v) for v in g["origin"])), g


def test_scan_batch_rotated_origin_golden(rotated, gpu):
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    tm, g = rotated
    sim = BatchSim(tm, n_envs=1, n_agents=1, device=gpu, noise_std=0.0, keep_f64_scans=True)
    s2, look, rc = sim.scan_batch(g["poses"], probe=True)
    assert np.array_equal(s2.cpu().numpy(), g["scans"])
    assert np.array_equal(look.cpu().numpy(), g["lookups"])
    assert np.array_equal(rc.cpu().numpy(), g["hit_rc"])
    sim.close()


@pytest.mark.parametrize("A", [1, 2])
def test_step_rotated_origin_vs_oracle(rotated, gpu, oracle_mod, monkeypatch, A):
    """Steps on the rotated map through every ray-kernel dispatch (tiled flat,
    tiled chunked: the ROT=true instantiations): each step's
    scans equal the oracle scanner's at the poses the step produced."""
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    import os
    from conftest import MAPS
    tm, g = rotated
    free, res, _ = oracle_mod.load_map(os.path.join(MAPS, "Spielberg_map.yaml"))
    osc = oracle_mod.OracleScanner(free, res, g["origin"])
    E = 48
    rng = np.random.default_rng(5)
    base = g["poses"][:20]
    poses = np.repeat(base[rng.integers(0, 20, E)][:, None, :], A, 1)
    poses[:, 1:, 0] += 0.8  # the other car 0.8 m along x
    acts = np.stack([rng.uniform(-0.4189, 0.4189, (6, E, A)), rng.uniform(0, 8, (6, E, A))], -1).astype(np.float32)
    outs = []
    for k in ("1", "2", "3"):  # 3 (the fixed-point kernels) falls back to 2 on a rotated map
        monkeypatch.setenv("F110_RAY_KERNEL", k)
        sim = BatchSim(tm, n_envs=E, n_agents=A, device=gpu, noise_std=0.0, keep_f64_scans=True)
        sim.reset(poses.reshape(E, A, 3))
        rec = []
        for t in range(6):
            o = sim.step(acts[t])
            st = sim.agent_states().cpu().numpy().reshape(E * A, 7)
            rec.append((o.scans_f64.cpu().numpy().reshape(E * A, -1), st))
        outs.append(rec)
        sim.close()
    for rec in outs[1:]:
        for (a, sa), (b, sb) in zip(outs[0], rec):
            assert np.array_equal(a, b) and np.array_equal(sa, sb)
    if A == 1:  # single agent: the step scan is exactly the scan at the new pose
        for sc, st in outs[0]:
            ref = osc.scan(np.stack([st[:, 0], st[:, 1], st[:, 4]], 1))
            live = st[:, 3] != 0  # TTC-collided cars have yaw zeroed after their scan
            assert live.sum() > E // 2
            assert np.array_equal(sc[live], ref[live])


@pytest.mark.parametrize("td,B", [(7, 1080), (100, 2048), (3, 333)])
def test_small_theta_dis_vs_oracle(gpu, tracks, oracle_mod, monkeypatch, td, B):
    """ScanSimulator2D's theta_dis (laser_models.py:360, the C-ABI's f110_config.theta_dis)
    small enough that the beam indices spend a large part of the scan below 1: the beam-index
    runs then cover the binades below 1 (before, every such beam was a run of its own and a
    scan could exceed the 80-run table).  scan_batch and steps through k_rays_fxs, k_rays_fxn
    and the tiled kernel (F110_RAY_KERNEL=1) against the oracle scanner with the same
    theta_dis, poses with yaws all round the circle."""
    import os
    from conftest import MAPS
    from f110_gymnasium_ros2_jazzy_amd import _lib
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    free, res, org = oracle_mod.load_map(os.path.join(MAPS, "Spielberg_map.yaml"))
    osc = oracle_mod.OracleScanner(free, res, org, num_beams=B, theta_dis=td)
    base_cfg = _lib.default_config

    def cfg():
        c = base_cfg()
        c.theta_dis = td
        return c
    monkeypatch.setattr(_lib, "default_config", cfg)
    E = 96
    rng = np.random.default_rng(td)
    sp = centerline_spawns("Spielberg", 1)
    poses = sp[rng.integers(0, sp.shape[0], E)].copy()
    poses[:, 0, 2] = rng.uniform(-np.pi, np.pi, E)
    acts = np.stack([rng.uniform(-0.4189, 0.4189, (4, E, 1)), rng.uniform(0, 3, (4, E, 1))], -1).astype(np.float32)
    outs = []
    for kern, refill in (("3", None), ("3", 0), ("1", None)):
        monkeypatch.setenv("F110_RAY_KERNEL", kern)
        sim = BatchSim(tracks("Spielberg_map"), n_envs=E, n_agents=1, device=gpu, noise_std=0.0, num_beams=B,
                       keep_f64_scans=True)
        assert sim.cfg.theta_dis == td
        if refill is not None:
            sim.set_ray_refill(refill)
        if kern == "3":
            assert sim.ray_kernel == 3 and (sim.ray_refill > 0) == (refill is None)
        got = sim.scan_batch(poses[:, 0]).cpu().numpy()
        assert np.array_equal(got, osc.scan(poses[:, 0]))
        rec = [sim.reset(poses).scans_f64.cpu().numpy()[:, 0]]
        sts = [poses[:, 0].copy()]
        for t in range(4):
            o = sim.step(acts[t])
            rec.append(o.scans_f64.cpu().numpy()[:, 0])
            st = sim.agent_states().cpu().numpy()[:, 0]
            sts.append(np.stack([st[:, 0], st[:, 1], st[:, 4]], 1))
        outs.append(rec)
        sim.close()
        for sc, p in zip(rec, sts):
            live = p[:, 2] != 0  # TTC-collided cars have yaw zeroed after their scan
            assert live.sum() > E // 2
            assert np.array_equal(sc[live], osc.scan(p)[live])
    for rec in outs[1:]:
        for a, b in zip(outs[0], rec):
            assert np.array_equal(a, b)


def test_scan_batch_random_poses_vs_oracle(sims, oracle_scanners):
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    sp = centerline_spawns("Spielberg", 1)[:, 0]
    rng = np.random.default_rng(7)
    idx = rng.integers(0, sp.shape[0], 600)
    poses = sp[idx] + np.stack([rng.normal(0, .3, 600), rng.normal(0, .3, 600), rng.normal(0, 1.0, 600)], 1)
    # edge cases: inside walls, off the map, far yaw
    poses = np.concatenate([poses, [[-200, -200, 0.1], [0, 0, 1e6], [0, 0, -1e-300], [30.0, 100.0, 3.0]]])
    sim = sims("Spielberg_map")
    got = sim.scan_batch(poses).cpu().numpy()
    ref = oracle_scanners("Spielberg_map").scan(poses)
    assert np.array_equal(got, ref)


def test_dynamics_golden(sims):
    d = golden("dynamics.npz")
    sim = sims("Spielberg_map", params=dict(zip(PKEYS, d["params"])))
    F = sim.dynamics_batch(d["X"], d["U"]).cpu().numpy()
    np.testing.assert_allclose(F, d["F"], rtol=1e-12, atol=1e-13)
    simk = sims("Spielberg_map", params=dict(zip(PKEYS, d["kat_params"])))
    fk = simk.dynamics_batch(d["kat_x_st"][None], d["kat_u"][None]).cpu().numpy()[0]
    np.testing.assert_allclose(fk, d["kat_f_st"], rtol=1e-12, atol=1e-15)
    assert np.max(np.abs(fk - d["kat_f_st_gt"])) < 5e-8   # dynamic_models.py:278, 7 places


def _resync_trace(sim, d):
    """Replay a Simulator.step trace with the device state re-synced to the
    reference state before every step (compares single steps)."""
    A = d["poses"].shape[0]
    T = d["actions"].shape[0]
    st0 = np.zeros((A, 7))
    st0[:, 0], st0[:, 1], st0[:, 4] = d["poses"][:, 0], d["poses"][:, 1], d["poses"][:, 2]
    worst_state, scan_exact, nonexact = 0.0, 0, 0
    for t in range(T):
        prev = st0 if t == 0 else d["states"][t - 1]
        buf = np.zeros((2, A))
        cnt = np.full(A, min(t, 2), np.int32)
        if t >= 1:
            buf[0] = d["actions"][t - 1][:, 0]
        if t >= 2:
            buf[1] = d["actions"][t - 2][:, 0]
        sim.set_state(prev.T.copy(), buf, cnt)
        out = sim.step(d["actions"][t][None])          # float64, like Simulator.step's inputs
        st = sim.agent_states().cpu().numpy()[0]
        worst_state = max(worst_state, float(np.max(np.abs(st - d["states"][t]) / np.maximum(1.0, np.abs(d["states"][t])))))
        scans = out.scans_f64.cpu().numpy()[0]
        if np.array_equal(scans, d["scans"][t]):
            scan_exact += 1
        else:
            # only beams re-cast onto another car may differ: ray_cast's cos/sin
            # (ocml vs glibc, 1 ulp) amplified by near-parallel beam/edge
            # intersections; bound well inside the north star's 1e-5
            np.testing.assert_allclose(scans, d["scans"][t], rtol=1e-9, atol=1e-9)
            nonexact += int(np.sum(scans != d["scans"][t]))
        assert np.array_equal(out.collisions.cpu().numpy()[0], d["collisions"][t].astype(np.uint8)), t
    return worst_state, scan_exact, T, nonexact


@pytest.mark.parametrize("tag", ["1agent", "1agent_crash", "2agent", "2agent_overlap", "3agent", "corridor",
                                 "1agent_euler", "2agent_euler"])
def test_simulator_traces(sims, tag, nonexact_budget):
    """Reference Simulator.step traces, RK4 and (the *_euler fixtures) the
    Euler integrator of update_pose (base_classes.py:376-396)."""
    d = golden(f"sim_{tag}.npz")
    A = d["poses"].shape[0]
    kw = {"integrator": int(d["integrator"])} if "integrator" in d and int(d["integrator"]) != 1 else {}
    sim = sims(d["map_name"].item().decode(), 1, A, **kw)
    worst, exact, T, nonexact = _resync_trace(sim, d)
    assert worst < 1e-12, worst
    if A == 1:
        assert exact == T, f"only {exact}/{T} steps bit-exact"
    nonexact_budget(f"sim_trace/{tag}", nonexact)


def test_free_running_trace_matches(sims):
    """No re-sync: the whole 120-step crash trajectory (incl. TTC zeroing)."""
    d = golden("sim_1agent_crash.npz")
    sim = sims("Spielberg_map", 1, 1)
    st = np.zeros((7, 1))
    st[0, 0], st[1, 0], st[4, 0] = d["poses"][0]
    sim.set_state(st, np.zeros((2, 1)), np.zeros(1, np.int32))
    for t in range(d["actions"].shape[0]):
        out = sim.step(d["actions"][t][None])
        s = sim.agent_states().cpu().numpy()[0]
        np.testing.assert_allclose(s, d["states"][t], rtol=1e-12, atol=1e-12)
        assert np.array_equal(out.collisions.cpu().numpy()[0], d["collisions"][t].astype(np.uint8))


def test_batch_matches_oracle_multi_env(sims, oracle_scanners, nonexact_budget):
    """64 envs x 2 agents, random actions, 20 steps vs the oracle (F110Env
    reset semantics: reset + one zero-action step)."""
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    import oracle as O
    E, A = 64, 2
    sp = centerline_spawns("Spielberg", A, gap=20)
    rng = np.random.default_rng(11)
    poses = sp[rng.integers(0, sp.shape[0], E)]
    sim = sims("Spielberg_map", E, A)
    ref = O.OracleSim(oracle_scanners("Spielberg_map"), E, A)
    sim.reset(poses)
    ref.reset(poses)
    rs, rc = ref.step(np.zeros((E, A, 2)))
    np.testing.assert_allclose(sim.out.scans_f64.cpu().numpy(), rs, rtol=1e-9, atol=1e-9)
    nonexact = int(np.sum(sim.out.scans_f64.cpu().numpy() != rs))
    for t in range(20):
        act = np.stack([rng.uniform(-0.4189, 0.4189, (E, A)), rng.uniform(0, 20, (E, A))], -1).astype(np.float32)
        out = sim.step(act)
        rs, rc = ref.step(act.astype(np.float64))
        st = sim.agent_states().cpu().numpy().reshape(E * A, 7)
        np.testing.assert_allclose(st, ref.state, rtol=1e-10, atol=1e-10)
        g = out.scans_f64.cpu().numpy()
        np.testing.assert_allclose(g, rs, rtol=1e-9, atol=1e-9)
        nonexact += int(np.sum(g != rs))
        ref.state[:] = st      # keep the two in lock-step (ulp-level trig differences)
        np.testing.assert_array_equal(out.collisions.cpu().numpy(), rc.astype(np.uint8))
    nonexact_budget("multi_env_64x2_20steps", nonexact)


def test_obs_packing(sims):
    """_pack_flat_obs (f110_env.py:552-584): scan of agent 0, f32 /30, poses."""
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    E, A = 8, 2
    sp = centerline_spawns("Spielberg", A, gap=30)[::600][:E]
    sim = sims("Spielberg_map", E, A)
    out = sim.reset(sp)
    for _ in range(3):
        out = sim.step(np.tile([[[0.1, 5.0], [-0.1, 4.0]]], (E, 1, 1)).astype(np.float32))
    obs = out.obs.cpu().numpy()
    scans = out.scans_f64.cpu().numpy()
    lidar = np.clip(np.nan_to_num(scans[:, 0].astype(np.float32), nan=30., posinf=30., neginf=0.), 0.0, 30.0) / 30.0
    assert obs.shape == (E, 1080 + 8)
    assert np.array_equal(obs[:, :1080], lidar)
    st = sim.agent_states().cpu().numpy()
    wrap = lambda a: ((a + np.pi) % (2 * np.pi)) - np.pi  # noqa: E731
    for a in range(A):
        assert np.array_equal(obs[:, 1080 + 4 * a + 0], st[:, a, 0].astype(np.float32))
        assert np.array_equal(obs[:, 1080 + 4 * a + 1], st[:, a, 1].astype(np.float32))
        assert np.array_equal(obs[:, 1080 + 4 * a + 2], np.array([wrap(float(v)) for v in st[:, a, 4]], np.float32))
        assert np.array_equal(obs[:, 1080 + 4 * a + 3], out.collisions.cpu().numpy()[:, a].astype(np.float32))


def _adversarial_poses(rng, E, A, sp):
    """Per env: agent 0 on the centerline; the others behind it (where
    get_blocked_view_indices spans most of the scan), beside it, touching or
    overlapping it, or exactly on the extension of one of its edge lines."""
    W, L = 0.31, 0.58
    out = np.zeros((E, A, 3))
    for e in range(E):
        x, y, th = sp[rng.integers(0, sp.shape[0]), 0]
        out[e, 0] = (x, y, th)
        c, s = np.cos(th), np.sin(th)
        for a in range(1, A):
            kind = rng.integers(0, 6)
            if kind == 0:    # behind, 0.5 - 3 m
                dx, dy, dth = -rng.uniform(0.5, 3.0), rng.uniform(-0.5, 0.5), rng.normal(0, 0.3)
            elif kind == 1:  # beside
                dx, dy, dth = rng.uniform(-0.5, 0.5), rng.choice([-1, 1]) * rng.uniform(0.35, 1.5), rng.normal(0, 0.5)
            elif kind == 2:  # touching / overlapping
                dx, dy, dth = rng.uniform(-0.7, 0.7), rng.uniform(-0.35, 0.35), rng.uniform(-np.pi, np.pi)
            elif kind == 3:  # agent 0's scan origin on the line of the other car's side edge
                dx, dy, dth = rng.uniform(0.8, 3.0), W / 2, 0.0
            elif kind == 4:  # ... or of its rear edge (car rotated 90 degrees)
                dx, dy, dth = rng.uniform(0.8, 3.0), L / 2, np.pi / 2
            else:            # ahead
                dx, dy, dth = rng.uniform(0.6, 4.0), rng.uniform(-0.6, 0.6), rng.normal(0, 0.3)
            out[e, a] = (x + c * dx - s * dy, y + s * dx + c * dy, th + dth)
    return out


@pytest.mark.parametrize("A,B,fov,ld", [(1, 2, 4.7, 0.0), (1, 3, 4.7, 0.0), (1, 63, 4.7, 0.0), (1, 4096, 4.7, 0.0),
                                        (2, 2, 4.7, 0.0), (2, 3, 4.7, 0.0), (2, 63, 4.7, 0.0), (2, 4096, 4.7, 0.0),
                                        (8, 333, 4.7, 0.0), (1, 1080, 4.7, 0.275), (2, 1080, 6.2, 0.275),
                                        (2, 720, 1.0, -0.1), (1, 256, 0.05, 0.0)])
def test_beam_counts_lockstep_vs_oracle(sims, oracle_mod, A, B, fov, ld):
    """Scan configurations away from the default (ScanSimulator2D(num_beams, fov),
    laser_models.py:360; RaceCar's lidar_dist, base_classes.py:420-422): two and three beams (one
    64-beam chunk, mostly idle), 63, and 4096 (past the fixed-point kernels' 2048: the tiled
    kernel over 64 chunks); eight agents; the scan origin ahead of / behind the car; a wide, a
    narrow and a very narrow fov.  Adversarial opponent poses, 4 steps in lock-step with the
    oracle: scans and collisions bit-exact against the oracle with the device's correctly
    rounded sin / cos, within 1e-9 of the glibc one; no hand-off read outside the
    mask."""
    import os
    from conftest import MAPS
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    O = oracle_mod
    E = 48
    rng = np.random.default_rng(B * 10 + A)
    poses = _adversarial_poses(rng, E, A, centerline_spawns("Spielberg", 1))
    free, res, org = O.load_map(os.path.join(MAPS, "Spielberg_map.yaml"))
    osc = O.OracleScanner(free, res, org, num_beams=B, fov=fov)
    sim = sims("Spielberg_map", E, A, num_beams=B, fov=fov, lidar_dist=ld)
    if B > 2048:
        assert sim.ray_kernel == 1
    if A > 1:
        sim.set_handoff_check(1)
    sim.reset_counters()
    ref, refd = O.OracleSim(osc, E, A, lidar_dist=ld), O.OracleSim(osc, E, A, lidar_dist=ld)
    sim.reset(poses)
    ref.reset(poses)
    rs, rc = ref.step(np.zeros((E, A, 2)))
    with O.device_trig():
        refd.reset(poses)
        rd, _ = refd.step(np.zeros((E, A, 2)))
    for t in range(4):
        g = sim.out.scans_f64.cpu().numpy()
        assert g.shape == (E, A, B)
        assert np.array_equal(g, rd), f"step {t}"
        np.testing.assert_allclose(g, rs, rtol=1e-9, atol=1e-9)
        np.testing.assert_array_equal(sim.out.collisions.cpu().numpy(), rc.astype(np.uint8))
        act = np.stack([rng.uniform(-0.3, 0.3, (E, A)), rng.uniform(0, 5, (E, A))], -1)
        ref.state[:] = sim.agent_states().cpu().numpy().reshape(E * A, 7)
        refd.state[:] = ref.state
        sim.step(act)
        rs, rc = ref.step(act)
        with O.device_trig():
            rd, _ = refd.step(act)
    if A > 1:
        assert sim.read_counter(6) == 0, "k_post_multi read hand-off beams outside the mask"
        sim.set_handoff_check(0)


@pytest.mark.parametrize("A", [2, 3])
def test_agent_ray_cast_adversarial_vs_oracle(sims, oracle_scanners, A, nonexact_budget):
    """Agent ray_cast (base_classes.py:206-227, laser_models.py:318-346) with
    opponents behind / beside / touching / on edge-line extensions: the device
    beam-window filter must not change a single range."""
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    import oracle as O
    E = 256
    rng = np.random.default_rng(100 + A)
    poses = _adversarial_poses(rng, E, A, centerline_spawns("Spielberg", 1))
    sim = sims("Spielberg_map", E, A)
    sim.set_handoff_check(1)  # hand-off buffer NaN-poisoned per step, reads outside the mask counted
    sim.reset_counters()
    ref = O.OracleSim(oracle_scanners("Spielberg_map"), E, A)
    # residue attribution: the same oracle with the device's correctly rounded
    # sin / cos in place of glibc's at the sites the device computes them
    refd = O.OracleSim(oracle_scanners("Spielberg_map"), E, A)
    sim.reset(poses)
    ref.reset(poses)
    rs, rc = ref.step(np.zeros((E, A, 2)))
    with O.device_trig():
        refd.reset(poses)
        rd, _ = refd.step(np.zeros((E, A, 2)))
    nonexact = nonexact_d = 0
    for t in range(4):
        g = sim.out.scans_f64.cpu().numpy()
        np.testing.assert_allclose(g, rs, rtol=1e-9, atol=1e-9)
        nonexact += int(np.sum(g != rs))
        nonexact_d += int(np.sum(g != rd))
        np.testing.assert_array_equal(sim.out.collisions.cpu().numpy(), rc.astype(np.uint8))
        act = np.stack([rng.uniform(-0.2, 0.2, (E, A)), rng.uniform(0, 3, (E, A))], -1)
        ref.state[:] = sim.agent_states().cpu().numpy().reshape(E * A, 7)
        refd.state[:] = ref.state
        sim.step(act)
        rs, rc = ref.step(act)
        with O.device_trig():
            rd, _ = refd.step(act)
    assert sim.read_counter(6) == 0, "k_post_multi read hand-off beams outside the mask"
    sim.set_handoff_check(0)
    nonexact_budget(f"ray_cast_adversarial_A{A}", nonexact)
    nonexact_budget(f"ray_cast_adversarial_A{A}/device_trig_oracle", nonexact_d)


@pytest.mark.parametrize("kernel,lanes,pad,refill", [
    ("2", 1, "1", 0), ("3", 1, "1", 0), ("3", 2, "0", 0), ("3", 2, "1", 0), ("3", 2, "1", 1), ("3", 2, "1", 3)])
def test_fixed_point_cell_index_adversarial_vs_oracle(gpu, tracks, oracle_scanners, monkeypatch, kernel, lanes, pad,
                                                      refill):
    """The fixed-point cell index (F110_RAY_KERNEL=3, the default) against
    the oracle's IEEE xy_2_rc (laser_models.py:55-104) where it is hardest:
    scan origins exactly on cell edges and corners with the beam whose table
    direction is exactly (1, 0) (every lookup of that ray then sits on a row
    edge: the guard-band path), origins just inside / outside the map edges
    looking out (clamped into the row-major padding), and origins far off the
    map (dt[-1, -1] steps; the cars whose rays could leave t's binade take
    fx_step).  Scans must be bit-exact for every kernel: k_rays_tiled
    (kernel 2), k_rays_fx (1 ray per lane), k_rays_fxn (2, on the clamped
    table or, F110_FX_PAD=1, the padded one: 2^24 binade, u24 offsets, no
    clamp; origins 1-20 cells outside the map edges straddle its per-car
    test, the fast loop up to 6 cells out, the IEEE loop beyond) and
    k_rays_fxs (f110_debug_set_ray_refill: 1 or 3 waves per car, kFxsBase
    offsets on the padded table)."""
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    monkeypatch.setenv("F110_RAY_KERNEL", kernel)
    monkeypatch.setenv("F110_FX_PAD", pad)
    tm = tracks("Spielberg_map")
    ox, oy, _ = tm.origin
    res = tm.resolution
    H, W = tm.free_mask.shape
    rng = np.random.default_rng(11)
    sp = _spawns_for(tm)
    fov, td = 4.7, 2000
    yaw_x = fov / 2 + 0.5 * 2 * np.pi / td   # beam 0 has theta index 0.5 -> (cos, sin) = (1, 0) exactly
    poses = []
    for i in range(96):  # on-track origins snapped to a row edge / a column edge / a corner
        x, y, _ = sp[rng.integers(0, sp.shape[0])]
        r = np.floor((y - oy) / res)
        c = np.floor((x - ox) / res)
        if i % 3 == 0:
            y = oy + r * res
        elif i % 3 == 1:
            x = ox + c * res
        else:
            x, y = ox + c * res, oy + r * res
        poses.append((x, y, yaw_x + (0.0 if i % 2 == 0 else rng.normal(0, 1e-3))))
    for i in range(32):  # near the four map edges, looking out
        side = i % 4
        t = rng.uniform(0.1, 0.9)
        eps = [0.0, 1e-12, 1e-9, 1e-6][(i // 4) % 4] * (1 if i % 8 < 4 else -1)
        if side == 0:
            poses.append((ox + eps, oy + t * H * res, np.pi))
        elif side == 1:
            poses.append((ox + W * res + eps, oy + t * H * res, 0.0))
        elif side == 2:
            poses.append((ox + t * W * res, oy + eps, -np.pi / 2))
        else:
            poses.append((ox + t * W * res, oy + H * res + eps, np.pi / 2))
    for i in range(16):  # far off the map
        poses.append((ox - 5.0 - 100.0 * i, oy + rng.uniform(-50, 150), rng.uniform(-np.pi, np.pi)))
    for k in (1, 5, 6, 7, 8, 20):  # k cells outside each edge, looking in and along (the padded loop's per-car test)
        t = rng.uniform(0.2, 0.8)
        poses.append((ox - k * res + 1e-7, oy + t * H * res, rng.uniform(-1.0, 1.0)))
        poses.append((ox + (W + k) * res - 1e-7, oy + t * H * res, np.pi + rng.uniform(-1.0, 1.0)))
        poses.append((ox + t * W * res, oy - k * res + 1e-7, np.pi / 2 + rng.uniform(-1.0, 1.0)))
        poses.append((ox + t * W * res, oy + (H + k) * res - 1e-7, -np.pi / 2 + rng.uniform(-1.0, 1.0)))
    for i in range(8):  # beyond 2^21 cells: t leaves its binade (the per-car check sends these to fx_step)
        far = (2.0e5, -2.0e5, 1.0e7, -3.0e8)[i % 4]
        poses.append((ox + far if i < 4 else ox + 10.0, oy + (far if i >= 4 else 10.0), rng.uniform(-np.pi, np.pi)))
    poses = np.asarray(poses, np.float64)
    E = poses.shape[0]
    sim = BatchSim(tm, n_envs=E, n_agents=1, device=gpu, noise_std=0.0, keep_f64_scans=True)
    assert sim.ray_kernel == int(kernel)  # no silent fallback on this axis-aligned map
    if kernel == "3":
        sim.set_ray_lanes(lanes)
        sim.set_ray_refill(refill)
    assert sim.ray_refill == refill
    out = sim.reset(poses[:, None, :])
    torch.cuda.synchronize()
    st = sim.agent_states().cpu().numpy().reshape(E, 7)
    got = out.scans_f64.cpu().numpy().reshape(E, -1)
    ref = oracle_scanners("Spielberg_map").scan(np.stack([st[:, 0], st[:, 1], st[:, 4]], 1))
    sim.close()
    bad = np.flatnonzero(~np.all(got == ref, axis=1))
    assert bad.size == 0, f"poses {bad[:8]} differ from the oracle"


def _spawns_for(tm):
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    return centerline_spawns("Spielberg", 1)[:, 0]


def _rk4_device(f, x, dt, n):
    for _ in range(n):
        k1 = f(x)
        k2 = f(x + dt * (k1 / 2))
        k3 = f(x + dt * (k2 / 2))
        k4 = f(x + dt * k3)
        x = x + dt * (1 / 6) * (k1 + 2 * k2 + 2 * k3 + k4)
    return x


def test_dynamics_zeroinit_kats(gpu, tracks):
    """The reference's DynamicsTest.test_zeroinit_{roll,dec,acc,rollleft}
    (dynamic_models.py:281-423) through the device right-hand sides
    (f110_dynamics_batch: vehicle_dynamics_st, f110_dynamics_ks_batch:
    vehicle_dynamics_ks) with DynamicsTest's vehicle params: zero initial
    state, the four inputs integrated together (4 rows) for 1 s at dt 1e-4
    (RK4; the reference uses odeint on the same time grid).  End states within
    the reference's 1e-2 of its ground truth; the rolling car stays exactly
    at rest, as the reference asserts with == (:310-311)."""
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    d = golden("dynamics_kat.npz")
    sim = BatchSim(tracks("Spielberg_map"), n_envs=1, n_agents=1, device=gpu, noise_std=0.0,
                   params=dict(zip(PKEYS, d["params"])))
    u = torch.as_tensor(d["u"], device=gpu)
    n, dt = int(d["n_steps"]), float(d["dt"])
    st = _rk4_device(lambda x: sim.dynamics_batch(x, u), torch.zeros(4, 7, dtype=torch.float64, device=gpu), dt, n)
    ks = _rk4_device(lambda x: sim.dynamics_ks_batch(x, u), torch.zeros(4, 5, dtype=torch.float64, device=gpu), dt, n)
    st, ks = st.cpu().numpy(), ks.cpu().numpy()
    sim.close()
    assert np.all(np.abs(st - d["gt_st"]) < 1e-2), st
    assert np.all(np.abs(ks - d["gt_ks"]) < 1e-2), ks
    # and against scipy odeint on the reference's own func_ST / func_KS (the fixture's cross-check)
    assert np.all(np.abs(st - d["odeint_st"]) < 1e-3) and np.all(np.abs(ks - d["odeint_ks"]) < 1e-3)
    roll = list(d["names"]).index("roll")
    assert np.all(st[roll] == 0.0) and np.all(ks[roll] == 0.0)


def test_collision_batch_golden(gpu):
    """f110_collision_batch (collision_models.py:113, GJK) on 3000 car-box
    pairs of the reference fixture (coincident centres and equal headings
    included), and f110_collision_multiple (collision_models.py:184-212) on
    the reference's own KAT CollisionTests.test_multiple_collisions (:313-324,
    7 perturbed bodies: collisions [1,1,1,1,1,1,0], idx [5,5,5,5,5,4,-1]) and
    on 200 clustered sets of 2..6 cars."""
    from f110_gymnasium_ros2_jazzy_amd.collision import collision_batch, collision_multiple
    d = golden("collision.npz")
    got = collision_batch(d["verts_a"], d["verts_b"], device=gpu).cpu().numpy()
    assert np.array_equal(got, d["overlap"])
    c, i = collision_multiple(d["kat_vertices"], device=gpu)
    assert np.array_equal(c.cpu().numpy(), d["kat_expected_collisions"])
    assert np.array_equal(i.cpu().numpy(), d["kat_expected_idx"])
    assert np.array_equal(c.cpu().numpy(), d["kat_collisions"]) and np.array_equal(i.cpu().numpy(), d["kat_idx"])
    counts = d["mb_count"]
    for k in np.unique(counts):
        sel = np.flatnonzero(counts == k)
        cc, ii = collision_multiple(d["mb_vertices"][sel, :k], device=gpu)
        assert np.array_equal(cc.cpu().numpy(), d["mb_collisions"][sel, :k])
        assert np.array_equal(ii.cpu().numpy(), d["mb_idx"][sel, :k])
    # empty batch is a no-op
    assert collision_batch(np.zeros((0, 4, 2)), np.zeros((0, 4, 2)), device=gpu).numel() == 0
