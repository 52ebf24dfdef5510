"""The RCCL path on the GPU box: torch.distributed's "nccl" backend (RCCL on ROCm) initialised the
way bench.py / distributed.init do it (device_id bound, then the all-reduce self-check), run with
one rank (a one-GPU box cannot hold two RCCL ranks: one rank per device).  Checks that the
communicator comes up in this image and that an all-reduce of a DDPG-sized fp32 gradient bucket
(the critic's flat bucket, GradBucket.reduce's sum then scale) returns the bucket itself.  Runs in
a child process with its own time limit, so a hung communicator cannot take the test session."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import os, sys, json
    sys.path.insert(0, os.environ["REPO"])
    import torch, torch.distributed as dist
    from f110_gymnasium_ros2_jazzy_amd import distributed as D
    torch.cuda.set_device(0)
    dist.init_process_group(backend="nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    D.self_check()
    g = torch.Generator(device="cuda"); g.manual_seed(0)
    n = 1084 * 256 + 256 + 258 * 256 + 256 + 256 * 1 + 1  # ~ the critic's flat bucket
    flat = torch.randn(n, generator=g, device="cuda", dtype=torch.float32)
    ref = flat.clone()
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    flat.mul_(1.0 / dist.get_world_size())
    torch.cuda.synchronize()
    ok = bool(torch.equal(flat, ref))
    print(json.dumps({"backend": dist.get_backend(), "world": dist.get_world_size(), "n": n, "equal": ok,
                      "desc": D.describe()}))
    dist.destroy_process_group()
""")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_world1_self_check_and_bucket_allreduce():
    env = dict(os.environ, REPO=REPO, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    import json
    d = json.loads(line)
    assert d["backend"] == "nccl" and d["world"] == 1
    assert d["equal"], d
