"""The reference-side ctypes binding (integration/f110_mi355x_backend.py)
driven exactly like the reference drives base_classes.Simulator and
ScanSimulator2D, against the reference's recorded outputs
(tests/golden/sim_*.npz, scans_*.npz from make_golden.py)."""
import os
import sys

import numpy as np
import pytest

from conftest import MAPS, golden

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_PARAMS = {'mu': 1.0489, 'C_Sf': 4.718, 'C_Sr': 5.4562, 'lf': 0.15875, 'lr': 0.17145, 'h': 0.074,
                  'm': 3.74, 'I': 0.04712, 's_min': -0.4189, 's_max': 0.4189, 'sv_min': -3.2, 'sv_max': 3.2,
                  'v_switch': 7.319, 'a_max': 9.51, 'v_min': 0.00000001, 'v_max': 20.0, 'width': 0.31,
                  'length': 0.58}


@pytest.fixture(scope="module")
def backend():
    from f110_gymnasium_ros2_jazzy_amd import _build
    os.environ["LIBF110"] = _build.LIB
    sys.path.insert(0, os.path.join(REPO, "integration"))
    import f110_mi355x_backend as b
    return b


def test_binding_declares_abi(backend):
    """CPU: the stub loads libf110.so and every entry point it declares exists."""
    L = backend.lib()
    for name in ("f110_create", "f110_step", "f110_scan_batch", "f110_set_params", "f110_set_scan_noise",
                 "f110_get_state", "f110_set_state", "f110_edt_k"):
        assert hasattr(L, name)
    sim = backend.ScanSimulator2D(1080, 4.7)
    with pytest.raises(ValueError):
        sim.scan(np.zeros(3), None)          # laser_models.py:445-446


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["1agent", "1agent_crash", "2agent", "2agent_overlap", "3agent", "corridor"])
def test_simulator_stub_replays_reference_trace(gpu, backend, tag):
    """Free-running Simulator(params, A, 12345).reset(poses); step(actions[t]) as
    make_golden.gen_sim ran the reference (noise off there: scan_noise=False)."""
    d = golden(f"sim_{tag}.npz")
    A = d["poses"].shape[0]
    sim = backend.Simulator(DEFAULT_PARAMS, A, 12345, time_step=0.01, integrator=1, scan_noise=False)
    sim.set_map(os.path.join(MAPS, d["map_name"].item().decode() + ".yaml"), ".png")
    with pytest.raises(ValueError):
        sim.reset(np.zeros((A + 1, 3)))
    sim.reset(d["poses"])
    for t in range(d["actions"].shape[0]):
        obs = sim.step(d["actions"][t])
        st = np.stack([obs["poses_x"], obs["poses_y"], obs["poses_theta"], obs["linear_vels_x"],
                       obs["ang_vels_z"]], 1)
        ref = d["states"][t][:, [0, 1, 4, 3, 5]]
        np.testing.assert_allclose(st, ref, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(np.stack(obs["scans"]), d["scans"][t], rtol=1e-9, atol=1e-9)
        assert np.array_equal(obs["collisions"], d["collisions"][t])
    sim._ctx.close()


@pytest.mark.gpu
def test_scan_simulator_stub_with_rng(gpu, backend):
    """ScanSimulator2D.scan(pose, rng): ranges bit-exact, plus the caller's
    rng.normal(0, 0.01, 1080) draws (laser_models.py:450-452)."""
    d = golden("scans_Spielberg_map.npz")
    s = backend.ScanSimulator2D(1080, 4.7)
    s.set_map(os.path.join(MAPS, "Spielberg_map.yaml"), ".png")
    assert s.get_increment() == 4.7 / 1079
    assert np.array_equal(s.scan_batch(d["poses"]), d["scans"])
    rng, ref_rng = np.random.default_rng(12345), np.random.default_rng(12345)
    for i in range(3):
        got = s.scan(d["poses"][i], rng)
        assert np.array_equal(got, d["scans"][i] + ref_rng.normal(0., 0.01, size=1080))
    s._ctx.close()
