"""Host-side (CPU) checks: the oracle's lap bookkeeping (_check_done,
f110_env.py:310-352; the device epilogue is checked against the same traces
in tests/test_gpu_env.py) replayed against the reference traces, env-shard
arithmetic, the f110_gym drop-in package, and a gloo world_size-2 run of the
sharding + timing reduction bench.py uses."""
import os
import socket

import numpy as np
import pytest

from conftest import golden


def test_check_done_replay():
    """Feed the reference's per-step poses/collisions through the oracle's
    _check_done and compare terminated / lap counters / checkpoint flags."""
    import oracle as O
    d = golden("env_2agent.npz")
    lap = O.LapOracle(d["reset_poses"], ego_idx=0)
    current_time = 0.0
    T = d["info_poses_x"].shape[0]
    for t in range(T):
        current_time = current_time + 0.01
        # the reference keeps float64 poses; the f32 info copies differ from
        # them by < 1e-6 m, far from the 0.1 m^2 zone boundary here
        term, cp = lap.check_done(list(d["info_poses_x"][t].astype(np.float64)),
                                  list(d["info_poses_y"][t].astype(np.float64)),
                                  d["info_collisions"][t].astype(np.float64), current_time)
        if t:
            assert term == bool(d["terminated"][t - 1])
        assert np.array_equal(cp, d["info_checkpoint_done"][t])
        assert np.array_equal(lap.lap_counts.astype(np.float32), d["info_lap_counts"][t])


def test_shard_range():
    from f110_gymnasium_ros2_jazzy_amd.distributed import shard_range
    for total, world in [(65536, 8), (10, 3), (7, 7), (5, 8)]:
        shards = [shard_range(total, world, r) for r in range(world)]
        assert sum(s.count for s in shards) == total
        assert shards[0].offset == 0
        for a, b in zip(shards, shards[1:]):
            assert b.offset == a.offset + a.count
        assert max(s.count for s in shards) - min(s.count for s in shards) <= 1
    assert shard_range(65536, 8, 3).offset == 3 * 8192


def test_f110_gym_package_imports():
    import f110_gym
    from f110_gym.envs import F110Env, Integrator
    assert F110Env.__name__ == "F110Env" and Integrator.RK4 == 1
    try:
        import gymnasium  # noqa: F401
    except Exception:
        pytest.skip("gymnasium not installed: registry not available")
    from gymnasium.envs.registration import registry
    assert "f110-v0" in registry


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from f110_gymnasium_ros2_jazzy_amd import distributed as D
    D.init(backend="gloo")
    sh = D.shard_range(16, world, rank)
    t = D.max_over_ranks(0.5 + rank)        # bench.py: max over ranks of the timed region
    n = D.sum_over_ranks(sh.count * 10)     # total env-steps of the job
    D.barrier()
    q.put((rank, sh.offset, sh.count, t, n))
    dist.destroy_process_group()


def test_gloo_world2_sharding_and_reductions():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert [r[1] for r in res] == [0, 8] and [r[2] for r in res] == [8, 8]
    assert all(r[3] == 1.5 for r in res) and all(r[4] == 160 for r in res)


def test_stream_shards_rejects_uneven_split():
    """streams.StreamShards splits the shard into equal contiguous sub-shards
    (bench.py --streams); an uneven split is refused before any device work."""
    import pytest
    from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards
    with pytest.raises(ValueError):
        StreamShards(None, n_envs=10, n_streams=3)
    with pytest.raises(ValueError):
        StreamShards(None, n_envs=8, n_streams=0)
