"""Data-parallel DDPG learner on CPU: two gloo ranks with half a batch each
end every update with the weights of one process on the whole batch (the
gradient bucket all-reduce of ddpg.GradBucket)."""
import os
import socket

import numpy as np
import torch

from conftest import golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _learner():
    from f110_gymnasium_ros2_jazzy_amd.ddpg import DDPGLearner
    return DDPGLearner(obs_dim=12, act_dim=2, action_low=[-0.4189, 0.0], action_high=[0.4189, 20.0], seed=42,
                       device="cpu", replay=None)


def _batches():
    d = golden("ddpg.npz")
    S, A, R, S2, D = (torch.from_numpy(np.asarray(d[k])) for k in ("S", "A", "R", "S2", "D"))
    g = torch.Generator().manual_seed(0)
    out = []
    for _ in range(4):
        idx = torch.randperm(S.shape[0], generator=g)[:32]
        w = torch.rand(32, generator=g)
        out.append((S[idx], A[idx], R[idx], S2[idx], D[idx].float(), w))
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from f110_gymnasium_ros2_jazzy_amd import distributed as D
    D.init(backend="gloo")
    ln = _learner()
    half = 32 // world
    for b in _batches():
        ln.update(*(t[rank * half:(rank + 1) * half] for t in b))
    q.put((rank, {k: v.numpy().copy() for k, v in ln.actor.state_dict().items()},
           {k: v.numpy().copy() for k, v in ln.critic_target.state_dict().items()}))  # numpy: no fd sharing
    D.shutdown()


def test_gloo_world2_matches_single_process_update():
    import multiprocessing as mp
    torch.set_num_threads(1)
    ref = _learner()
    for b in _batches():
        ref.update(*b)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=180) for _ in ps), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for _, actor, critic_t in res:
        for k, v in ref.actor.state_dict().items():
            np.testing.assert_allclose(actor[k], v.numpy(), rtol=1e-5, atol=1e-7)
        for k, v in ref.critic_target.state_dict().items():
            np.testing.assert_allclose(critic_t[k], v.numpy(), rtol=1e-5, atol=1e-7)
    for k in res[0][1]:  # the ranks hold identical weights
        assert np.array_equal(res[0][1][k], res[1][1][k])
