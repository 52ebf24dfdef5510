"""Hand-off mask coverage (multi-agent step).

k_agents' handoff_chunks marks, in f32, the 64-beam chunks of each car's
scan that k_post_multi's agent ray_cast may read (get_blocked_view_indices,
laser_models.py:282-315, seen from the car's yaw or, after a TTC response,
from yaw 0: base_classes.py:206-227, :246-249); the ray kernel stores only
those chunks into the f64 hand-off buffer.  A chunk the mask missed would be
read stale.  These tests run the masked step with the hand-off buffer
NaN-poisoned before every ray launch and k_post_multi counting each read of a
beam outside the mask (f110_debug_set_handoff_check mode 1), beside an
identical context with the mask off (mode 2): every output must be the same
bits and the miss counter 0.  The poses are the mask's hard cases: opponent
vertices 1-2 cm from the scan origin, vertex bearings within 2e-2 rad of the
+-pi wrap, bearings whose nearest beam sits exactly on the 3-beam margin of a
chunk edge (and half a beam either side), and cars whose TTC fires (yaw-0
recompute); the oracle checks the same steps (1e-9, ray_cast trig residue).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

W_CAR, L_CAR = 0.31, 0.58
FOV, B = 4.7, 1080
INCR = FOV / (B - 1)
# get_vertices' order (collision_models.py:250-259): rl, rr, fr, fl
VX = np.array([-L_CAR / 2, -L_CAR / 2, L_CAR / 2, L_CAR / 2])
VY = np.array([W_CAR / 2, -W_CAR / 2, -W_CAR / 2, W_CAR / 2])


def _center_for_vertex(px, py, thj, q):
    """The opponent pose whose box vertex q lies at (px, py) for yaw thj."""
    c, s = np.cos(thj), np.sin(thj)
    return px - (c * VX[q] - s * VY[q]), py - (s * VX[q] + c * VY[q])


def _wall_pose(scanner, cl, rng):
    """A centerline point turned towards a side wall, moved so that the wall
    is 0.35-0.75 m ahead (a car at 20 m/s then fires its TTC within a step)."""
    for _ in range(100):
        x, y, th = cl[rng.integers(0, cl.shape[0])]
        th = th + rng.choice([-1.0, 1.0]) * np.pi / 2 + rng.normal(0.0, 0.2)
        fwd = scanner.scan(np.array([[x, y, th]]))[0, B // 2]
        d = fwd - rng.uniform(0.35, 0.75)
        if 0.0 < d < 5.0:
            return x + d * np.cos(th), y + d * np.sin(th), th
    raise AssertionError("no wall pose found")


def _hard_poses(scanner, cl, rng, E, A):
    """Per env: car 0 on the centerline (kind 3: facing a wall); each opponent
    placed by one of the mask's hard cases relative to car 0."""
    poses = np.zeros((E, A, 3))
    kinds = np.zeros(E, np.int64)
    for e in range(E):
        kind = e % 4
        kinds[e] = kind
        if kind == 3:
            x, y, th = _wall_pose(scanner, cl, rng)
        else:
            x, y, th = cl[rng.integers(0, cl.shape[0])]
        poses[e, 0] = (x, y, th)
        for j in range(1, A):
            thj = rng.uniform(-np.pi, np.pi)
            q = int(rng.integers(0, 4))
            if kind == 0:    # a vertex 1-2 cm from the scan origin
                r, phi = rng.uniform(0.01, 0.02), rng.uniform(-np.pi, np.pi)
            elif kind == 1:  # a vertex bearing within 2e-2 rad of the +-pi wrap (behind the car)
                r, phi = rng.uniform(0.3, 3.0), th + np.pi + rng.uniform(-0.02, 0.02)
            elif kind == 2:  # nearest beam on the 3-beam margin of a chunk edge, or half a beam off it
                m = int(rng.integers(1, 17))
                k = 64 * m + 3 if rng.integers(0, 2) else 64 * m - 4
                k = min(max(k + rng.choice([-0.5, 0.0, 0.5]) + rng.choice([-1e-7, 0.0, 1e-7]), 0.0), B - 1.0)
                r, phi = rng.uniform(0.4, 4.0), th + (k * INCR - FOV / 2)
            else:            # the TTC car's opponent: anywhere 1-3 m around it
                r, phi = rng.uniform(1.0, 3.0), rng.uniform(-np.pi, np.pi)
            cx, cy = _center_for_vertex(x + r * np.cos(phi), y + r * np.sin(phi), thj, q)
            poses[e, j] = (cx, cy, thj)
    return poses, kinds


def _same_bits(x, y):
    a, b = np.ascontiguousarray(x.cpu().numpy()), np.ascontiguousarray(y.cpu().numpy())
    return a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("A", [2, 4])
def test_handoff_mask_hard_cases_bit_identical(tracks, gpu, oracle_scanners, A):
    import oracle as O
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    E, T = 1000 if A == 2 else 250, 6  # E * A not a multiple of 64: k_agents' padding threads
    scanner = oracle_scanners("Spielberg_map")
    rng = np.random.default_rng(7000 + A)
    cl = centerline_spawns("Spielberg", 1)[:, 0]
    poses, kinds = _hard_poses(scanner, cl, rng, E, A)
    kw = dict(n_envs=E, n_agents=A, device=gpu, noise_std=0.0, keep_f64_scans=True)
    masked = BatchSim(tracks("Spielberg_map"), **kw)
    plain = BatchSim(tracks("Spielberg_map"), **kw)
    masked.set_handoff_check(1)  # poison + count misses
    plain.set_handoff_check(2)   # every chunk stored
    masked.reset_counters()
    ref = O.OracleSim(scanner, E, A)
    masked.reset(poses)
    plain.reset(poses)
    ref.reset(poses)
    rs, rc = ref.step(np.zeros((E, A, 2)))
    # the TTC group's car 0 at 20 m/s towards its wall
    st = masked.agent_states().cpu().numpy()
    ttc_env = kinds == 3
    st[ttc_env, 0, 3] = 20.0
    state = torch.from_numpy(np.ascontiguousarray(st.reshape(E * A, 7).T))
    masked.set_state(state)
    plain.set_state(state)
    ttc_hits = 0
    for t in range(T + 1):
        if t:
            act = np.zeros((E, A, 2))
            act[..., 0] = rng.uniform(-0.05, 0.05, (E, A))
            act[ttc_env, 0, 1] = 20.0
            ref.state[:] = masked.agent_states().cpu().numpy().reshape(E * A, 7)
            masked.step(act)
            plain.step(act)
            rs, rc = ref.step(act)
        torch.cuda.synchronize()
        for name in ("scans_f64", "obs", "collisions", "terminated"):
            assert _same_bits(getattr(masked.out, name), getattr(plain.out, name)), (t, name)
        assert _same_bits(masked.agent_states(), plain.agent_states()), t
        g = masked.out.scans_f64.cpu().numpy()
        assert np.isfinite(g).all(), t
        np.testing.assert_allclose(g, rs, rtol=1e-9, atol=1e-9)
        col = masked.out.collisions.cpu().numpy()
        assert np.array_equal(col, rc.astype(np.uint8)), t
        if t:
            ttc_hits += int(col[ttc_env, 0].sum())
    misses = masked.read_counter(6)
    assert misses == 0, f"{misses} k_post_multi reads outside the hand-off mask"
    assert ttc_hits > 0, "no TTC response in the TTC group (yaw-0 recompute not exercised)"
    masked.close()
    plain.close()


def test_handoff_check_counts_a_forced_miss(tracks, gpu):
    """The miss counter is live: with the mask forced empty (every hand-off
    store skipped) a two-agent step with an opponent in view must count
    misses and read the NaN poison."""
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    E, A = 64, 2
    sp = centerline_spawns("Spielberg", A, gap=10)
    sim = BatchSim(tracks("Spielberg_map"), n_envs=E, n_agents=A, device=gpu, noise_std=0.0, keep_f64_scans=True)
    sim.set_handoff_check(1 | 4)  # bit 2: an empty mask (test of the check itself)
    sim.reset_counters()
    sim.reset(sp[np.arange(E) * 37 % sp.shape[0]])
    torch.cuda.synchronize()
    assert sim.read_counter(6) > 0
    sim.set_handoff_check(0)
    sim.close()
