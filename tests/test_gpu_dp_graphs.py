"""Config 5's data-parallel step graphs (train.VectorTrainer on several ranks):
two gloo ranks on the one GPU, each stepping its half of the envs, run the
same loop with the per-step HIP graphs (three graphs per parity, the two
gradient-bucket all-reduces eager between them) and eagerly
(F110_STEP_GRAPH=0).  Weights, losses, replay length and the noise state
are bit-identical between the two modes on every rank, and the ranks hold
the same weights (rl_training/DDPG/agent.py:242-348 batched; the reference
learner is single-process)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS = 13  # ends on an even-parity replay (steps 4.. are graphed: both parities replay)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), F110_SAME_DEVICE="1")
    try:
        import torch as T
        from f110_gymnasium_ros2_jazzy_amd import distributed as D
        from f110_gymnasium_ros2_jazzy_amd.train import VectorTrainer
        D.init(backend="gloo")
        T.cuda.set_device(0)
        shard = D.shard_range(256 * world, world, rank)
        out = {}
        for flag in ("1", "0"):
            os.environ["F110_STEP_GRAPH"] = flag
            tr = VectorTrainer(shard.count, batch_size=128, memory_size=4096, warmup_steps=3, seed=11,
                               env_offset=shard.offset, rank_seed=rank)
            losses = []
            for _ in range(STEPS):
                tr.step()
                if tr.last is not None:
                    losses.append((float(tr.last["critic_loss"]), float(tr.last["actor_loss"])))
            T.cuda.synchronize()
            ag = tr.agent
            graphed = tr._sg[0] is not None and tr._sg[1] is not None
            params = np.concatenate([p.detach().reshape(-1).cpu().numpy() for p in
                                     list(ag.actor.parameters()) + list(ag.critic.parameters())])
            out[flag] = dict(graphed=graphed, params=params, losses=losses, sigma=ag.sigma, calls=ag._noise_calls,
                             n=len(ag.memory), ngraphs=len(tr._sg[0][0]) if graphed else 0)
            tr.close()
        q.put((rank, out))
        D.shutdown()
    except Exception as exc:  # report, do not hang the parent
        import traceback
        q.put((rank, {"error": repr(exc), "tb": traceback.format_exc()}))


def test_dp_step_graphs_match_eager_two_ranks(gpu):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in ps)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in (0, 1):
        assert "error" not in res[r], res[r].get("tb")
        g, e = res[r]["1"], res[r]["0"]
        assert g["graphed"] and not e["graphed"]
        assert g["ngraphs"] == 3  # split at the two all-reduces
        assert np.array_equal(g["params"], e["params"])
        assert g["losses"] == e["losses"]
        assert (g["sigma"], g["calls"], g["n"]) == (e["sigma"], e["calls"], e["n"])
    assert np.array_equal(res[0]["1"]["params"], res[1]["1"]["params"])  # the ranks agree
