"""Generate the golden fixtures under tests/golden/ from the upstream reference.

TEST INFRASTRUCTURE ONLY.  Run in the build container (it needs
/root/reference; the GPU box never runs this):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Every fixture is *data* produced by executing the reference's own functions
(loaded by ``_refload``) on seeded inputs: inputs and expected outputs only.
Reference functions exercised (file:line under
f110_gymnasium/gym/f110_gym/envs/):

  laser_models.py   ScanSimulator2D.__init__:360, set_map:383, get_dt:40,
                    get_scan:148, trace_ray:106, xy_2_rc:55, check_ttc_jit:188,
                    ray_cast:318, get_blocked_view_indices:282, get_range:249
  dynamic_models.py vehicle_dynamics_st:123, vehicle_dynamics_ks:90, pid:178,
                    DynamicsTest.test_derivatives:255 (reference KAT)
  collision_models.py get_vertices:237, collision:113, collision_multiple:184,
                    CollisionTests:271 (reference KAT)
  base_classes.py   RaceCar.__init__:69 (beam tables), update_pose:256,
                    Simulator.step:566, reset:627
  f110_env.py       F110Env.reset:425, step:371, _pack_flat_obs:552,
                    _build_info:586, _check_done:310
"""
from __future__ import annotations

import hashlib
import os
import sys

sys.dont_write_bytecode = True
import numpy as np  # noqa: E402
from scipy.ndimage import distance_transform_edt  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refload  # noqa: E402

REPO = os.path.dirname(os.path.dirname(HERE))
MAPS = os.path.join(REPO, "f110_gymnasium_ros2_jazzy_amd", "maps")
REF = _refload.REF_ROOT

dm, lm, cm, bc = _refload.load_all()

DEFAULT_PARAMS = {'mu': 1.0489, 'C_Sf': 4.718, 'C_Sr': 5.4562, 'lf': 0.15875, 'lr': 0.17145,
                  'h': 0.074, 'm': 3.74, 'I': 0.04712, 's_min': -0.4189, 's_max': 0.4189,
                  'sv_min': -3.2, 'sv_max': 3.2, 'v_switch': 7.319, 'a_max': 9.51,
                  'v_min': 0.00000001, 'v_max': 20.0, 'width': 0.31, 'length': 0.58,
                  'lidar_max': 30.0}
PKEYS = ['mu', 'C_Sf', 'C_Sr', 'lf', 'lr', 'h', 'm', 'I', 's_min', 's_max', 'sv_min',
         'sv_max', 'v_switch', 'a_max', 'v_min', 'v_max']


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {name}: {os.path.getsize(path)/1024:.1f} KiB")


def scan_sim(map_name):
    s = lm.ScanSimulator2D(1080, 4.7)
    s.set_map(os.path.join(MAPS, map_name + ".yaml"), ".png")
    return s


# ---------------------------------------------------------------- tables ----
def gen_tables():
    s = lm.ScanSimulator2D(1080, 4.7)
    bc.RaceCar.scan_simulator = None
    car = bc.RaceCar(DEFAULT_PARAMS, 12345, time_step=0.01, integrator=bc.Integrator.RK4)
    save("tables.npz", sines=s.sines, cosines=s.cosines,
         angle_increment=np.float64(s.angle_increment),
         theta_index_increment=np.float64(s.theta_index_increment),
         scan_angles=bc.RaceCar.scan_angles.copy(), beam_cosines=bc.RaceCar.cosines.copy(),
         side_distances=bc.RaceCar.side_distances.copy())
    del car


# ------------------------------------------------------------------- EDT ----
def gen_edt(map_name, rng):
    s = scan_sim(map_name)
    bitmap = s.map_img
    inds = distance_transform_edt(bitmap, return_distances=False, return_indices=True)
    H, W = bitmap.shape
    rr, cc = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    k = ((inds[0] - rr).astype(np.int64) ** 2 + (inds[1] - cc).astype(np.int64) ** 2).astype(np.uint32)
    recon = s.map_resolution * np.sqrt(k.astype(np.float64))
    exact = bool(np.array_equal(recon, s.dt))
    assert exact, f"res*sqrt(k) != dt on {map_name}"
    n = 4000
    sr = rng.integers(0, H, n)
    sc = rng.integers(0, W, n)
    out = dict(H=np.int64(H), W=np.int64(W), res=np.float64(s.map_resolution),
               origin=np.array(s.origin, dtype=np.float64),
               occupied=np.int64((bitmap == 0).sum()),
               k_sha256=np.bytes_(hashlib.sha256(np.ascontiguousarray(k).tobytes()).hexdigest()),
               dt_sha256=np.bytes_(hashlib.sha256(np.ascontiguousarray(s.dt).tobytes()).hexdigest()),
               k_max=np.int64(k.max()), spot_r=sr, spot_c=sc, spot_k=k[sr, sc], spot_dt=s.dt[sr, sc],
               dt_last=np.float64(s.dt[-1, -1]))
    if H * W <= 200_000:
        out["k_full"] = k
    save(f"edt_{map_name}.npz", **out)
    return s


# ----------------------------------------------------------------- scans ----
class RayProbe:
    """Counts EDT lookups per ray and records the last (r, c) of each ray by
    wrapping the module-level xy_2_rc / trace_ray that get_scan resolves at
    call time (laser_models.py:102,177)."""

    def __init__(self):
        self.orig_xy = lm.xy_2_rc
        self.orig_trace = lm.trace_ray
        self.count = 0
        self.last = (0, 0)
        self.counts, self.lasts = [], []

    def __enter__(self):
        def xy(*a):
            r = self.orig_xy(*a)
            self.count += 1
            self.last = r
            return r

        def tr(*a):
            self.count = 0
            d = self.orig_trace(*a)
            self.counts.append(self.count)
            self.lasts.append(self.last)
            return d

        lm.xy_2_rc, lm.trace_ray = xy, tr
        return self

    def __exit__(self, *exc):
        lm.xy_2_rc, lm.trace_ray = self.orig_xy, self.orig_trace


def centerline():
    path = os.path.join(REF, "tools/Raceline-Optimization/inputs/tracks/Spielberg_map.csv")
    pts = np.loadtxt(path, delimiter=",", comments="#")
    return pts


def gen_scans(map_name, s, poses):
    scans, counts, rcs = [], [], []
    for p in poses:
        with RayProbe() as pr:
            sc = s.scan(np.asarray(p, dtype=np.float64), None)
        scans.append(sc)
        counts.append(pr.counts)
        rcs.append(pr.lasts)
    save(f"scans_{map_name}.npz", poses=np.asarray(poses, np.float64), scans=np.asarray(scans),
         lookups=np.asarray(counts, np.int32), hit_rc=np.asarray(rcs, np.int32))


def spielberg_poses(rng, cl):
    n = cl.shape[0]
    poses = []
    for i in rng.choice(n, 24, replace=False):
        j = (i + 3) % n
        th = np.arctan2(cl[j, 1] - cl[i, 1], cl[j, 0] - cl[i, 0])
        poses.append([cl[i, 0] + rng.uniform(-0.2, 0.2), cl[i, 1] + rng.uniform(-0.2, 0.2),
                      th + rng.uniform(-0.2, 0.2)])
    poses += [[0.0, 0.0, 0.0],            # the reference's own test pose (laser_models.py:564)
              [0.5, 0.0, -1.0],           # ScanTests pose family (laser_models.py:478)
              [cl[5, 0], cl[5, 1], 10.0],  # theta far outside [-pi, pi] -> fmod/while wrap
              [cl[9, 0], cl[9, 1], -7.5],
              [-200.0, -200.0, 0.3],      # outside the map: every lookup reads dt[-1,-1]
              [-84.85359914210505 + 0.01, -36.30299725862132 + 0.01, 0.0],  # map corner
              [cl[100, 0], cl[100, 1], 4.7 / 2.0],  # theta_index starts exactly at 0
              ]
    return poses


def corridor_poses(s, rng):
    free = np.argwhere(s.map_img > 0)
    pick = free[rng.choice(len(free), 8, replace=False)]
    poses = []
    for r, c in pick:
        xr = (c + 0.5) * s.map_resolution
        yr = (r + 0.5) * s.map_resolution
        # invert xy_2_rc's rotation (laser_models.py:75-76)
        xt = xr * s.orig_c - yr * s.orig_s
        yt = xr * s.orig_s + yr * s.orig_c
        poses.append([xt + s.orig_x, yt + s.orig_y, rng.uniform(-np.pi, np.pi)])
    poses.append([s.orig_x, s.orig_y, 0.1])
    return poses


ROT_YAW = 0.35


def gen_scans_rotated(rng):
    """Spielberg with a map-origin yaw of 0.35 rad (every bundled map has yaw
    0): xy_2_rc's rotation (laser_models.py:75-76) on the reference's own
    ScanSimulator2D, origin fields overridden after set_map."""
    s = scan_sim("Spielberg_map")
    s.orig_c, s.orig_s = np.cos(ROT_YAW), np.sin(ROT_YAW)
    free = np.argwhere(s.map_img > 0)
    pick = free[rng.choice(len(free), 20, replace=False)]
    poses = []
    for r, c in pick:
        xr = (c + rng.uniform(0.05, 0.95)) * s.map_resolution
        yr = (r + rng.uniform(0.05, 0.95)) * s.map_resolution
        xt = xr * s.orig_c - yr * s.orig_s
        yt = xr * s.orig_s + yr * s.orig_c
        poses.append([xt + s.orig_x, yt + s.orig_y, rng.uniform(-np.pi, np.pi)])
    poses += [[s.orig_x, s.orig_y, 0.2], [-300.0, 10.0, 0.0], [s.orig_x + 1.0, s.orig_y - 0.5, 2.5]]
    scans, counts, rcs = [], [], []
    for p in poses:
        with RayProbe() as pr:
            sc = s.scan(np.asarray(p, dtype=np.float64), None)
        scans.append(sc)
        counts.append(pr.counts)
        rcs.append(pr.lasts)
    save("scans_Spielberg_rot.npz", poses=np.asarray(poses, np.float64), scans=np.asarray(scans),
         lookups=np.asarray(counts, np.int32), hit_rc=np.asarray(rcs, np.int32),
         origin=np.array([s.orig_x, s.orig_y, ROT_YAW]))


# -------------------------------------------------------------- dynamics ----
def gen_dynamics(rng):
    P = [DEFAULT_PARAMS[k] for k in PKEYS]
    n = 3000
    X = np.empty((n, 7))
    X[:, 0] = rng.uniform(-50, 50, n)
    X[:, 1] = rng.uniform(-50, 50, n)
    X[:, 2] = rng.uniform(-0.5, 0.5, n)
    X[:, 3] = np.where(rng.random(n) < 0.3, rng.uniform(-0.6, 0.6, n), rng.uniform(-5, 21, n))
    X[:, 4] = rng.uniform(-4, 4, n)
    X[:, 5] = rng.uniform(-3, 3, n)
    X[:, 6] = rng.uniform(-0.5, 0.5, n)
    U = np.stack([rng.uniform(-4, 4, n), rng.uniform(-12, 12, n)], axis=1)
    # hit constraint edges exactly
    X[:20, 2] = DEFAULT_PARAMS['s_max']
    X[20:40, 2] = DEFAULT_PARAMS['s_min']
    X[40:60, 3] = DEFAULT_PARAMS['v_max']
    X[60:80, 3] = DEFAULT_PARAMS['v_min']
    X[80:100, 3] = 0.5
    F = np.stack([dm.vehicle_dynamics_st(X[i], U[i], *P) for i in range(n)])

    # pid (dynamic_models.py:178); includes the v_min=1e-8 braking sign quirk
    m = 2000
    Q = np.stack([rng.uniform(-5, 21, m), rng.uniform(-0.5, 0.5, m),
                  rng.uniform(-5, 21, m), rng.uniform(-0.5, 0.5, m)], axis=1)
    Q[:50, 1] = Q[:50, 3] + rng.uniform(-1e-4, 1e-4, 50)   # |steer_diff| ~ 1e-4 boundary
    Q[50:80, 2] = 0.0
    pid_out = np.array([dm.pid(q[0], q[1], q[2], q[3], DEFAULT_PARAMS['sv_max'], DEFAULT_PARAMS['a_max'],
                               DEFAULT_PARAMS['v_max'], DEFAULT_PARAMS['v_min']) for q in Q])

    # reference KAT (dynamic_models.py:231-266)
    t = dm.DynamicsTest()
    t.setUp()
    kat_params = np.array([t.mu, t.C_Sf, t.C_Sr, t.lf, t.lr, t.h, t.m, t.I, t.s_min, t.s_max,
                           t.sv_min, t.sv_max, t.v_switch, t.a_max, t.v_min, t.v_max])
    x_ks = np.array([3.9579422297936526, 0.0391650102771405, 0.0378491427211811,
                     16.3546957860883566, 0.0294717351052816])
    x_st = np.array([2.0233348142065677, 0.0041907137716636, 0.0197545248559617,
                     15.7216236334290116, 0.0025857914776859, 0.0529001056654038,
                     0.0033012170610298])
    u_kat = np.array([0.15, 0.63 * 9.81])
    f_st_kat = dm.vehicle_dynamics_st(x_st, u_kat, *kat_params)
    f_ks_kat = dm.vehicle_dynamics_ks(x_ks, u_kat, *kat_params)
    f_st_gt = np.array([15.7213512030862397, 0.0925527979719355, 0.1500000000000000,
                        5.3536773276413925, 0.0529001056654038, 0.6435589397748606,
                        0.0313297971641291])
    f_ks_gt = np.array([16.3475935934250209, 0.4819314886013121, 0.1500000000000000,
                        5.1464424102339752, 0.2401426578627629])
    save("dynamics.npz", params=np.array(P), X=X, U=U, F=F, pid_in=Q, pid_out=pid_out,
         kat_params=kat_params, kat_x_st=x_st, kat_x_ks=x_ks, kat_u=u_kat,
         kat_f_st=f_st_kat, kat_f_ks=f_ks_kat, kat_f_st_gt=f_st_gt, kat_f_ks_gt=f_ks_gt)


# ------------------------------------------------------------ collision ----
def gen_collision(rng):
    # reference KAT: CollisionTests.test_multiple_collisions with its legacy seed
    t = cm.CollisionTests()
    t.setUp()   # np.random.seed(1234)
    v1 = t.vertices1
    bodies = [v1 + np.random.normal(size=v1.shape) / 100. for _ in range(6)] + [v1 + 10.]
    allv = np.stack(bodies)
    cols, idx = cm.collision_multiple(allv)

    # car rectangles at random nearby poses
    n = 3000
    L, Wd = DEFAULT_PARAMS['length'], DEFAULT_PARAMS['width']
    pa = np.stack([rng.uniform(-5, 5, n), rng.uniform(-5, 5, n), rng.uniform(-4, 4, n)], 1)
    pb = pa + np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(-4, 4, n)], 1)
    pb[:30] = pa[:30]                          # coincident centres: d == 0 branch
    pb[30:60, 2] = pa[30:60, 2]
    va = np.stack([cm.get_vertices(p, L, Wd) for p in pa])
    vb = np.stack([cm.get_vertices(p, L, Wd) for p in pb])
    res = np.array([cm.collision(va[i].copy(), vb[i].copy()) for i in range(n)])

    # multi-body: 3..6 cars clustered
    mb_v, mb_c, mb_i, mb_n = [], [], [], []
    for _ in range(200):
        k = int(rng.integers(2, 7))
        pp = np.stack([rng.uniform(-0.8, 0.8, k), rng.uniform(-0.8, 0.8, k), rng.uniform(-4, 4, k)], 1)
        vv = np.stack([cm.get_vertices(p, L, Wd) for p in pp])
        c, ix = cm.collision_multiple(vv)
        pad = np.full((6, 4, 2), np.nan)
        pad[:k] = vv
        mb_v.append(pad)
        mb_c.append(np.pad(c, (0, 6 - k)))
        mb_i.append(np.pad(ix, (0, 6 - k), constant_values=-9))
        mb_n.append(k)
    save("collision.npz", kat_vertices=allv, kat_collisions=cols, kat_idx=idx,
         kat_expected_collisions=np.array([1., 1., 1., 1., 1., 1., 0.]),
         kat_expected_idx=np.array([5., 5., 5., 5., 5., 4., -1.]),
         poses_a=pa, poses_b=pb, verts_a=va, verts_b=vb, overlap=res.astype(np.uint8),
         mb_vertices=np.stack(mb_v), mb_collisions=np.stack(mb_c), mb_idx=np.stack(mb_i),
         mb_count=np.array(mb_n))


def gen_raycast_ttc(rng):
    tables = np.load(os.path.join(HERE, "tables.npz"))
    ang = tables["scan_angles"]
    L, Wd = DEFAULT_PARAMS['length'], DEFAULT_PARAMS['width']
    n = 200
    poses = np.stack([rng.uniform(-3, 3, n), rng.uniform(-3, 3, n), rng.uniform(-4, 4, n)], 1)
    opp = poses[:, :2] + np.stack([rng.uniform(-4, 4, n), rng.uniform(-4, 4, n)], 1)
    opp = np.concatenate([opp, rng.uniform(-4, 4, (n, 1))], 1)
    # ranges quantised to 1/1024 m keep the fixture compressible; the
    # reference consumed exactly these float64 values
    scans_in = np.round(rng.uniform(0.2, 30.0, (n, ang.shape[0])) * 1024.0) / 1024.0
    scans_in[:100] = 30.0
    out = []
    for i in range(n):
        v = cm.get_vertices(opp[i], L, Wd)
        out.append(lm.ray_cast(poses[i].copy(), scans_in[i].copy(), ang, v))
    # the reference's own example case (laser_models.py:636-648)
    ex_ang = np.linspace(-2.35, 2.35, num=1080)
    ex_v = np.asarray([[4, 11.], [5, 5], [9, 9], [10, 10]])
    ex_out = lm.ray_cast(np.array([0., 0., -1.]), 100. * np.ones(1080), ex_ang, ex_v)

    # TTC (laser_models.py:188)
    m = 400
    vel = rng.uniform(-6, 20, m)
    vel[:40] = 0.0
    tscans = np.round(rng.uniform(0.0, 3.0, (m, ang.shape[0])) * 1024.0) / 1024.0
    tscans[100:200] += 1.0
    tscans[200:260] = np.round(rng.uniform(0.4, 0.5, (60, ang.shape[0])) * 1024.0) / 1024.0
    ttc = np.array([lm.check_ttc_jit(tscans[i], vel[i], ang, tables["beam_cosines"],
                                     tables["side_distances"], 0.005) for i in range(m)])
    save("raycast_ttc.npz", poses=poses, opp_poses=opp, scans_in=scans_in, scans_out=np.asarray(out),
         ex_angles=ex_ang, ex_vertices=ex_v, ex_out=ex_out,
         ttc_vel=vel, ttc_scans=tscans, ttc_out=ttc.astype(np.uint8))


# ------------------------------------------------------------- simulator ----
def gen_sim(map_name, tag, poses, n_steps, rng, action_fn=None, integrator=None):
    bc.RaceCar.scan_simulator = None
    A = len(poses)
    sim = bc.Simulator(DEFAULT_PARAMS, A, 12345, time_step=0.01,
                       integrator=bc.Integrator.RK4 if integrator is None else integrator)
    sim.set_map(os.path.join(MAPS, map_name + ".yaml"), ".png")
    sim.reset(np.asarray(poses, np.float64))
    for ag in sim.agents:
        ag.scan_rng = None                      # noise-free parity (SURVEY §7 "Noise parity")
    acts, scans, states, cols, bufs = [], [], [], [], []
    for t in range(n_steps):
        if action_fn is None:
            a = np.stack([rng.uniform(-0.4189, 0.4189, A), rng.uniform(0.0, 20.0, A)], 1)
        else:
            a = action_fn(t, A)
        obs = sim.step(a)
        acts.append(a)
        scans.append(np.stack(obs['scans']))
        states.append(np.stack([ag.state.copy() for ag in sim.agents]))
        cols.append(np.asarray(obs['collisions'], np.float64).copy())
    save(f"sim_{tag}.npz", map_name=np.bytes_(map_name), poses=np.asarray(poses, np.float64),
         integrator=np.int32(2 if integrator is bc.Integrator.Euler else 1),  # base_classes.Integrator value
         actions=np.asarray(acts), scans=np.asarray(scans), states=np.asarray(states),
         collisions=np.asarray(cols))


def gen_euler(cl):
    """Simulator.step traces with the Euler integrator (base_classes.py:376-396,
    RaceCar's own default, :69): one agent on the track and a 2-agent pair."""
    rng = np.random.default_rng(4242)

    def ahead(i, d):
        j = (i + 3) % cl.shape[0]
        th = np.arctan2(cl[j, 1] - cl[i, 1], cl[j, 0] - cl[i, 0])
        k = (i + d) % cl.shape[0]
        return [cl[i, 0], cl[i, 1], th], [cl[k, 0], cl[k, 1], th]

    gen_sim("Spielberg_map", "1agent_euler", [ahead(1500, 25)[0]], 80, rng, integrator=bc.Integrator.Euler)
    gen_sim("Spielberg_map", "2agent_euler", list(ahead(2600, 20)), 60, rng, integrator=bc.Integrator.Euler)


def gen_dynamics_kat():
    """The reference's zero-initial-state KATs (DynamicsTest.test_zeroinit_*,
    dynamic_models.py:281-423): DynamicsTest's vehicle params, the four inputs,
    the ground-truth end states held in the reference test (data) and, as a
    cross-check, scipy odeint's end states of the reference's func_ST /
    func_KS exactly as the test integrates them (t = arange(0, 1, 1e-4))."""
    from scipy.integrate import odeint
    t = dm.DynamicsTest()
    t.setUp()
    P = (t.mu, t.C_Sf, t.C_Sr, t.lf, t.lr, t.h, t.m, t.I, t.s_min, t.s_max, t.sv_min, t.sv_max, t.v_switch,
         t.a_max, t.v_min, t.v_max)
    g = 9.81
    names = ["roll", "dec", "acc", "rollleft"]
    U = np.array([[0., 0.], [0., -0.7 * g], [0.15, 0.63 * g], [0.15, 0.]])
    gt_st = np.array([[0.] * 7,
                      [-3.4335000000000013, 0., 0., -6.8670000000000018, 0., 0., 0.],
                      [3.0731976046859715, 0.2869835398304389, 0.1500000000000000, 6.1802999999999999,
                       0.1097747074946325, 0.3248268063223301, 0.0697547542798040],
                      [0., 0., 0.15, 0., 0., 0., 0.]])
    gt_ks = np.array([[0.] * 5,
                      [-3.4335000000000013, 0., 0., -6.8670000000000018, 0.],
                      [3.0845676868494927, 0.1484249221523042, 0.1500000000000000, 6.1803000000000017,
                       0.1203664469224163],
                      [0., 0., 0.15, 0., 0.]])
    tt = np.arange(0., 1., 1e-4)
    end_st, end_ks = [], []
    for u in U:
        end_st.append(odeint(dm.func_ST, np.zeros(7), tt, args=(u,) + P)[-1])
        end_ks.append(odeint(dm.func_KS, np.zeros(5), tt, args=(u,) + P)[-1])
    end_st, end_ks = np.asarray(end_st), np.asarray(end_ks)
    assert np.all(np.abs(end_st - gt_st) < 1e-2) and np.all(np.abs(end_ks - gt_ks) < 1e-2)
    save("dynamics_kat.npz", names=np.array(names), params=np.array(P), u=U, t=tt[-1:], dt=np.float64(1e-4),
         n_steps=np.int64(tt.size - 1), gt_st=gt_st, gt_ks=gt_ks, odeint_st=end_st, odeint_ks=end_ks)


def gen_update_pose(rng, cl):
    """RaceCar.update_pose trajectories (base_classes.py:256): steer delay, pid,
    RK4, clamps, yaw wrap, NaN guards.  Several regimes: random, hard braking
    (exercises the v_min=1e-8 pid quirk), slow (KS branch), reversing."""
    bc.RaceCar.scan_simulator = None
    car = bc.RaceCar(DEFAULT_PARAMS, 12345, time_step=0.01, integrator=bc.Integrator.RK4)
    car.set_map(os.path.join(MAPS, "Spielberg_map.yaml"), ".png")
    trajs_a, trajs_s = [], []
    T = 150
    for mode in range(6):
        i = int(rng.integers(0, cl.shape[0]))
        car.reset(np.array([cl[i, 0], cl[i, 1], rng.uniform(-np.pi, np.pi)]))
        car.scan_rng = None
        if mode == 0:
            a = np.stack([rng.uniform(-0.4189, 0.4189, T), rng.uniform(0, 20, T)], 1)
        elif mode == 1:
            a = np.stack([rng.uniform(-0.4189, 0.4189, T), np.where(np.arange(T) < 60, 15.0, 0.0)], 1)
        elif mode == 2:
            a = np.stack([rng.uniform(-0.4189, 0.4189, T), rng.uniform(0, 0.4, T)], 1)
        elif mode == 3:
            a = np.stack([np.full(T, 0.4189), rng.uniform(-5, 5, T)], 1)
        elif mode == 4:
            a = np.stack([rng.uniform(-1.0, 1.0, T), rng.uniform(-20, 25, T)], 1)
        else:
            a = np.stack([np.sin(np.arange(T) / 7.0) * 0.4, np.full(T, 8.0)], 1)
        st = [car.state.copy()]
        for t in range(T):
            car.update_pose(a[t, 0], a[t, 1])
            st.append(car.state.copy())
        trajs_a.append(a)
        trajs_s.append(np.asarray(st))
    save("update_pose.npz", actions=np.asarray(trajs_a), states=np.asarray(trajs_s))


def gen_env(rng, cl):
    """F110Env (2 agents) reset + steps, noise disabled by re-patching
    RaceCar.reset (base_classes.py:183-204 re-seeds scan_rng)."""
    f110_env = _refload.load_env()
    bc.RaceCar.scan_simulator = None
    orig_reset = bc.RaceCar.reset

    def reset_no_noise(self, pose):
        orig_reset(self, pose)
        self.scan_rng = None

    bc.RaceCar.reset = reset_no_noise
    try:
        env = f110_env.F110Env(map_dir=MAPS + "/", map="Spielberg_map", map_ext=".png", num_agents=2)
        i = 400
        j = (i + 3) % cl.shape[0]
        th = float(np.arctan2(cl[j, 1] - cl[i, 1], cl[j, 0] - cl[i, 0]))
        k = i + 30
        poses = np.array([[cl[i, 0], cl[i, 1], th], [cl[k, 0], cl[k, 1], th]], np.float32)
        obs0, info0 = env.reset(options=poses)
        T = 60
        acts = np.stack([np.stack([rng.uniform(-0.4189, 0.4189, 2), rng.uniform(0, 20, 2)], 1)
                         for _ in range(T)]).astype(np.float32)
        obs, rew, term, trunc, keys = [obs0], [], [], [], {}
        infos = [info0]
        for t in range(T):
            o, r, te, tr, inf = env.step(acts[t])
            obs.append(o)
            rew.append(r)
            term.append(te)
            trunc.append(tr)
            infos.append(inf)
        for key in ["poses_x", "poses_y", "poses_theta", "linear_vels_x", "linear_vels_y",
                    "ang_vels_z", "collisions", "lap_times", "lap_counts", "checkpoint_done"]:
            keys["info_" + key] = np.asarray([np.asarray(inf[key]) for inf in infos])
        keys["info_time"] = np.asarray([inf["time"] for inf in infos])
        keys["info_scans"] = np.asarray([np.stack(inf["scans"]) for inf in infos]).astype(np.float32)
        save("env_2agent.npz", reset_poses=poses, actions=acts, obs=np.asarray(obs),
             reward=np.asarray(rew), terminated=np.asarray(term), truncated=np.asarray(trunc), **keys)
    finally:
        bc.RaceCar.reset = orig_reset


def _record_env(env, segments):
    """Run F110Env through segments [(reset_poses, actions[T, A, 2]), ...] and
    return the per-call obs / reward / flags / info arrays (reset calls
    included, in call order; `is_reset` marks them)."""
    obs, rew, term, trunc, infos, is_reset, acts = [], [], [], [], [], [], []
    A = segments[0][0].shape[0]
    for poses, seg_acts in segments:
        o, inf = env.reset(options=poses)
        obs.append(o); infos.append(inf); rew.append(0.0); term.append(False); trunc.append(False)
        is_reset.append(True); acts.append(np.zeros((A, 2), np.float32))
        for a in seg_acts:
            o, r, te, tr, inf = env.step(a)
            obs.append(o); infos.append(inf); rew.append(r); term.append(te); trunc.append(tr)
            is_reset.append(False); acts.append(a)
    keys = {}
    for key in ["poses_x", "poses_y", "poses_theta", "linear_vels_x", "linear_vels_y",
                "ang_vels_z", "collisions", "lap_times", "lap_counts", "checkpoint_done"]:
        keys["info_" + key] = np.asarray([np.asarray(inf[key]) for inf in infos])
    keys["info_time"] = np.asarray([inf["time"] for inf in infos])
    keys["info_scans"] = np.asarray([np.stack(inf["scans"]) for inf in infos]).astype(np.float32)
    return dict(actions=np.asarray(acts), is_reset=np.asarray(is_reset), obs=np.asarray(obs),
                reward=np.asarray(rew), terminated=np.asarray(term), truncated=np.asarray(trunc), **keys)


def _track_poses(cl, i, gap):
    j = (i + 3) % cl.shape[0]
    th = float(np.arctan2(cl[j, 1] - cl[i, 1], cl[j, 0] - cl[i, 0]))
    k = (i + gap) % cl.shape[0]
    return np.array([[cl[i, 0], cl[i, 1], th], [cl[k, 0], cl[k, 1], th]], np.float32)


def gen_env_lap_f32(cl, max_steps=1500):
    """F110Env (2 agents, noise off) reset with float32 options -- train_ddpg's
    dtype -- whose cars each drive full-lock circles (radius ~0.74 m) in an
    open free area of the Spielberg map (> 12 m from any wall) through their
    start zones: the lap toggles (_check_done, f110_env.py:310-352, with the
    float32 start_rot of f110_env.py:448-451) count past 4 for both cars and
    the episode terminates on laps.  Records toggles, lap counts / times,
    terminated and collisions per step."""
    sys.path.insert(0, REPO)
    from f110_gymnasium_ros2_jazzy_amd.maps import load_map
    tm = load_map("Spielberg_map")
    tm.ensure_edt()
    dt = tm.resolution * np.sqrt(tm.edt_k.astype(np.float64))
    rr, cc = np.nonzero(dt > 12.0)
    k = int(np.random.default_rng(0).integers(0, rr.size))
    x = tm.origin[0] + (cc[k] + 0.5) * tm.resolution
    y = tm.origin[1] + (rr[k] + 0.5) * tm.resolution
    poses = np.array([[x, y, 0.3], [x, y - 3.0, 0.3]], np.float32)
    f110_env = _refload.load_env()
    bc.RaceCar.scan_simulator = None
    orig_reset = bc.RaceCar.reset

    def reset_no_noise(self, pose):
        orig_reset(self, pose)
        self.scan_rng = None

    bc.RaceCar.reset = reset_no_noise
    try:
        env = f110_env.F110Env(map_dir=MAPS + "/", map="Spielberg_map", map_ext=".png", num_agents=2)
        obs, info = env.reset(options=poses)
        acts = np.array([[0.4189, 1.5], [0.4189, 1.3]], np.float32)
        tog, laps, times, term, cols = [env.toggle_list.copy()], [np.asarray(info["lap_counts"]).copy()], \
            [np.asarray(info["lap_times"]).copy()], [False], [np.asarray(info["collisions"]).copy()]
        start_rot = env.start_rot.copy()
        for t in range(max_steps):
            o, r, te, tr, inf = env.step(acts)
            tog.append(env.toggle_list.copy())
            laps.append(np.asarray(inf["lap_counts"]).copy())
            times.append(np.asarray(inf["lap_times"]).copy())
            term.append(bool(te))
            cols.append(np.asarray(inf["collisions"]).copy())
            if te:
                break
        assert term[-1] and not np.any(np.asarray(cols)) and np.all(tog[-1] >= 4)
        save("env_lap_f32.npz", reset_poses=poses, actions=acts, start_rot=start_rot,
             toggles=np.asarray(tog), lap_counts=np.asarray(laps), lap_times=np.asarray(times),
             terminated=np.asarray(term), collisions=np.asarray(cols))
    finally:
        bc.RaceCar.reset = orig_reset


def gen_env_noise(cl):
    """F110Env (2 agents) with the reference's own scan noise: every RaceCar
    re-creates default_rng(seed) at reset (base_classes.py:204) and scan adds
    rng.normal(0, 0.01, 1080) (laser_models.py:450-452).  Two episodes: the
    second reset must restart the generators."""
    rng = np.random.default_rng(777)
    f110_env = _refload.load_env()
    bc.RaceCar.scan_simulator = None
    env = f110_env.F110Env(map_dir=MAPS + "/", map="Spielberg_map", map_ext=".png", num_agents=2, seed=1234)
    poses = _track_poses(cl, 900, 12)
    segs = []
    for T in (40, 20):
        segs.append((poses, np.stack([np.stack([rng.uniform(-0.4189, 0.4189, 2), rng.uniform(0, 20, 2)], 1)
                                      for _ in range(T)]).astype(np.float32)))
    rec = _record_env(env, segs)
    save("env_2agent_noise.npz", reset_poses=poses, seed=np.int64(1234), **rec)


def gen_env_params(cl):
    """F110Env.update_params(params, index=0) (f110_env.py:487-498): agent 0 (behind)
    gets its own mass/geometry and sees agent 1 through its own box size; noise off (scan_rng=None after reset).  The
    cars start 8 centerline points apart so each sees the other (agent
    ray_cast uses the observer's length/width, base_classes.py:223)."""
    rng = np.random.default_rng(778)
    f110_env = _refload.load_env()
    bc.RaceCar.scan_simulator = None
    orig_reset = bc.RaceCar.reset

    def reset_no_noise(self, pose):
        orig_reset(self, pose)
        self.scan_rng = None

    bc.RaceCar.reset = reset_no_noise
    try:
        env = f110_env.F110Env(map_dir=MAPS + "/", map="Spielberg_map", map_ext=".png", num_agents=2)
        p1 = dict(DEFAULT_PARAMS, m=4.5, I=0.06, length=0.75, width=0.42, mu=0.9, v_max=15.0)
        env.update_params(p1, index=0)
        poses = _track_poses(cl, 1500, 14)
        acts = np.stack([np.stack([rng.uniform(-0.2, 0.2, 2), rng.uniform(2, 12, 2)], 1)
                         for _ in range(50)]).astype(np.float32)
        rec = _record_env(env, [(poses, acts)])
        save("env_2agent_params.npz", reset_poses=poses, params1=np.array([p1[k] for k in sorted(p1)]),
             params1_keys=np.array(sorted(p1)), **rec)
    finally:
        bc.RaceCar.reset = orig_reset


def gen_gap_follow():
    """rl_training/utils/gap_follow.py:gap_follow_action on float32 scans, as
    train_ddpg.py:168 calls it on info["scans"][1]: recorded F110Env scans
    (noise-free and noisy) plus edge cases (no gap, ties, bubble at either
    end, values on the 0.5 / 3.0 thresholds)."""
    gf = _refload.load_path("gap_follow", "rl_training/utils/gap_follow.py")
    rng = np.random.default_rng(779)
    scans = []
    for f in ("env_2agent.npz", "env_2agent_noise.npz", "env_2agent_params.npz"):
        d = np.load(os.path.join(HERE, f))
        scans += list(d["info_scans"][::3, 1]) + list(d["info_scans"][::15, 0])
    B = 1080
    z = np.zeros(B, np.float32)
    scans.append(z)                                            # no gap -> (0, B-1)
    scans.append(np.full(B, 10.0, np.float32))                 # all beyond max_distance
    scans.append(np.full(B, 0.5, np.float32))                  # exactly on the gap threshold
    two = np.full(B, 2.0, np.float32); two[300:310] = 0.1; two[700:710] = 0.1
    scans.append(two)                                          # equal gaps -> first maximal wins
    e0 = np.full(B, 4.0, np.float32); e0[0] = 0.05
    scans.append(e0)                                           # closest point at beam 0
    e1 = np.full(B, 4.0, np.float32); e1[-1] = 0.05
    scans.append(e1)                                           # closest point at the last beam
    tie = np.full(B, 4.0, np.float32); tie[100] = 0.2; tie[900] = 0.2
    scans.append(tie)                                          # argmin tie -> first index
    for _ in range(40):
        s = rng.uniform(0.0, 5.0, B).astype(np.float32)
        k = rng.integers(1, 6)
        for _ in range(k):
            a = rng.integers(0, B)
            s[a:a + rng.integers(1, 120)] = rng.uniform(0.0, 0.6)
        scans.append(s)
    for _ in range(10):                                        # values near 3.0 and 0.5 in f32
        s = rng.choice(np.array([0.5, 0.49999997, 0.50000006, 3.0, 2.9999998, 3.0000002, 1.0], np.float32), B)
        scans.append(s.astype(np.float32))
    scans = np.stack(scans).astype(np.float32)
    acts, gaps, proc = [], [], []
    for s in scans:
        acts.append(gf.gap_follow_action(s))
        p = gf.create_bubble(gf.preprocess_lidar(s))
        proc.append(p)
        gaps.append(gf.find_max_gap(p))
    save("gap_follow.npz", scans=scans, actions=np.asarray(acts), gaps=np.asarray(gaps, np.int64),
         processed16=np.asarray(proc[:16]))


def gen_env_gapfollow(cl):
    """train_ddpg.py's loop (:150-174) with noise off: agent 1 is driven by
    gap_follow_action(info["scans"][1]) of the previous call, agent 0 by
    recorded random actions (float32)."""
    gf = _refload.load_path("gap_follow", "rl_training/utils/gap_follow.py")
    rng = np.random.default_rng(780)
    f110_env = _refload.load_env()
    bc.RaceCar.scan_simulator = None
    orig_reset = bc.RaceCar.reset

    def reset_no_noise(self, pose):
        orig_reset(self, pose)
        self.scan_rng = None

    bc.RaceCar.reset = reset_no_noise
    try:
        env = f110_env.F110Env(map_dir=MAPS + "/", map="Spielberg_map", map_ext=".png", num_agents=2)
        poses = _track_poses(cl, 2100, 25)
        obs, info = env.reset(options=poses)
        T = 80
        ego = np.stack([np.stack([rng.uniform(-0.3, 0.3), rng.uniform(3, 9)]) for _ in range(T)]).astype(np.float32)
        obs_l, opp_l, term_l, scans_l = [obs], [], [], [np.stack(info["scans"])]
        for t in range(T):
            opp = gf.gap_follow_action(info["scans"][1]).astype(np.float32)
            obs, r, term, trunc, info = env.step(np.stack([ego[t], opp], axis=0).astype(np.float32))
            obs_l.append(obs); opp_l.append(opp); term_l.append(term); scans_l.append(np.stack(info["scans"]))
        save("env_gapfollow.npz", reset_poses=poses, ego_actions=ego, opp_actions=np.asarray(opp_l),
             obs=np.asarray(obs_l), terminated=np.asarray(term_l), info_scans=np.asarray(scans_l))
    finally:
        bc.RaceCar.reset = orig_reset


from make_golden_configs import REWARD_CONFIGS  # noqa: E402


def gen_reward(cl):
    """CenterlineSafetyProgressReward (rl_training/utils/rewards.py:185-355) over
    CenterlineProgress (track_progress.py:5-110) on the Spielberg centerline,
    fed the F110Env observations of three episodes (noise off; both cars
    driven by gap_follow_action, the ego's steering perturbed), as
    train_ddpg.py:150-185 calls it: reward_fn.reset() before each episode,
    reward_fn(next_obs) after every step."""
    gf = _refload.load_path("gap_follow", "rl_training/utils/gap_follow.py")
    tp = _refload.load_path("track_progress", "rl_training/utils/track_progress.py")
    rw = _refload.load_path("rewards", "rl_training/utils/rewards.py")
    csv = os.path.join(REF, "tools", "Raceline-Optimization", "inputs", "tracks", "Spielberg_map.csv")
    P = tp.CenterlineProgress(csv, closed=True)
    rng = np.random.default_rng(781)
    f110_env = _refload.load_env()
    bc.RaceCar.scan_simulator = None
    orig_reset = bc.RaceCar.reset

    def reset_no_noise(self, pose):
        orig_reset(self, pose)
        self.scan_rng = None

    bc.RaceCar.reset = reset_no_noise
    try:
        env = f110_env.F110Env(map_dir=MAPS + "/", map="Spielberg_map", map_ext=".png", num_agents=2)
        fns = {k: rw.CenterlineSafetyProgressReward(dt=0.01, progress=P, **v) for k, v in REWARD_CONFIGS.items()}
        obs_l, ep_l, rew = [], [], {k: [] for k in fns}
        starts = [(600, 30, 200), (2500, 20, 240), (4100, 45, 220)]
        for ep, (i, gap, T) in enumerate(starts):
            poses = _track_poses(cl, i, gap)
            for f in fns.values():
                f.reset()
            obs, info = env.reset(options=poses)
            for t in range(T):
                ego = gf.gap_follow_action(info["scans"][0]).astype(np.float32)
                ego[0] += np.float32(rng.normal(0, 0.08))
                ego[1] = np.float32(ego[1] * 1.6)
                opp = gf.gap_follow_action(info["scans"][1]).astype(np.float32)
                obs, _, term, trunc, info = env.step(np.stack([ego, opp]).astype(np.float32))
                obs_l.append(obs)
                ep_l.append(ep)
                for k, f in fns.items():
                    rew[k].append(float(f(obs)))
                if term:
                    break
        save("reward.npz", obs=np.asarray(obs_l, np.float32), episode=np.asarray(ep_l, np.int32),
             **{"reward_" + k: np.asarray(v) for k, v in rew.items()},
             config_names=np.array(list(REWARD_CONFIGS)),
             track_xy=P.xy, track_s=P.s, track_tan=P.tan, track_nrm=P.nrm, track_mid=P.mid, track_wR=P.wR,
             track_wL=P.wL, track_L=np.float64(P.L))
    finally:
        bc.RaceCar.reset = orig_reset


def gen_noise():
    """Noise semantics of ScanSimulator2D.scan (laser_models.py:450-452) with the
    per-agent default_rng(seed) re-seeded at reset (base_classes.py:119,204):
    we record the reference noise draws so the tests can check mean/std and
    the "same stream for every agent" property statistically."""
    r1 = np.random.default_rng(seed=42)
    r2 = np.random.default_rng(seed=42)
    n1 = np.stack([r1.normal(0., 0.01, size=1080) for _ in range(50)])
    n2 = np.stack([r2.normal(0., 0.01, size=1080) for _ in range(50)])
    save("noise.npz", agent0=n1, agent1=n2)


def main():
    rng = np.random.default_rng(20250824)
    cl = centerline()
    np.savez_compressed(os.path.join(MAPS, "Spielberg_centerline.npz"), xy=cl[:, :2].astype(np.float64),
                        w_right=cl[:, 2], w_left=cl[:, 3])
    print("wrote maps/Spielberg_centerline.npz")
    gen_tables()
    s_sp = gen_edt("Spielberg_map", rng)
    s_co = gen_edt("straight_corridor", rng)
    s_sh = gen_edt("Shanghai_map", rng)
    gen_scans("Spielberg_map", s_sp, spielberg_poses(rng, cl))
    gen_scans("straight_corridor", s_co, corridor_poses(s_co, rng))
    gen_scans("Shanghai_map", s_sh, [[0.0, 0.0, 0.0], [3.0, 0.5, 0.0], [1.0, 0.2, 0.1], [-2.0, 0.0, 3.0]])
    gen_dynamics(rng)
    gen_collision(rng)
    gen_raycast_ttc(rng)
    gen_update_pose(rng, cl)

    def ahead(i, d):
        j = (i + 3) % cl.shape[0]
        th = np.arctan2(cl[j, 1] - cl[i, 1], cl[j, 0] - cl[i, 0])
        k = (i + d) % cl.shape[0]
        return [cl[i, 0], cl[i, 1], th], [cl[k, 0], cl[k, 1], th]

    p0, p1 = ahead(1200, 25)
    gen_sim("Spielberg_map", "1agent", [p0], 80, rng)
    gen_sim("Spielberg_map", "1agent_crash", [ahead(700, 1)[0]], 120, rng,
            action_fn=lambda t, A: np.tile([[0.4189, 18.0]], (A, 1)))
    gen_sim("Spielberg_map", "2agent", list(ahead(2500, 25)), 60, rng)
    gen_sim("Spielberg_map", "2agent_overlap", list(ahead(3000, 5)), 30, rng)
    a0, a1 = ahead(4000, 30)
    _, a2 = ahead(4000, 60)
    gen_sim("Spielberg_map", "3agent", [a0, a1, a2], 40, rng)
    gen_sim("straight_corridor", "corridor", [[-0.5, 0.2, 0.0]], 40, rng,
            action_fn=lambda t, A: np.tile([[0.05, 12.0]], (A, 1)))
    gen_env(rng, cl)
    gen_noise()
    gen_env_noise(cl)
    gen_env_params(cl)
    gen_gap_follow()
    gen_env_gapfollow(cl)
    gen_reward(cl)
    gen_scans_rotated(np.random.default_rng(35))
    gen_euler(cl)
    gen_dynamics_kat()
    gen_env_lap_f32(cl)


if __name__ == "__main__":
    if len(sys.argv) > 1:  # regenerate selected fixtures only, e.g. `make_golden.py env_noise env_params`
        _cl = centerline()
        for name in sys.argv[1:]:
            {"env_noise": lambda c: gen_env_noise(c), "env_params": lambda c: gen_env_params(c),
             "gap_follow": lambda c: gen_gap_follow(), "env_gapfollow": gen_env_gapfollow,
             "reward": gen_reward, "euler": gen_euler, "lap_f32": gen_env_lap_f32, "dyn_kat": lambda c: gen_dynamics_kat(),
             "scans_rot": lambda c: gen_scans_rotated(np.random.default_rng(35))}[name](_cl)
    else:
        main()
