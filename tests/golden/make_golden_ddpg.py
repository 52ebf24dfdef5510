"""Golden fixtures for the DDPG learner and its prioritized replay buffer.

TEST INFRASTRUCTURE ONLY.  Run in the build container (needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ddpg.py

Executes the reference's own classes, loaded by file path (no copy):
  rl_training/DDPG/replay_buffer.py  PrioritizedExperienceReplayBuffer :6-135
  rl_training/DDPG/agent.py          Actor :25, Critic :64, DDPGAgent :105
                                     (remember :223, replay :242, _soft_update :373)
and records inputs and outputs only:

  per.npz   one buffer (size 16, batch 5) driven through adds (with and
            without priority), a with-replacement sample, updates holding
            NaN / inf / negative / duplicate entries, a wrap of the ring and a
            without-replacement sample: the priority array, length and ring
            pointer after every operation, each sample's idxs / weights /
            sampling probabilities.
            Plus sampling statistics: 20000 draws of sample() (batch 6) from a
            40-row buffer with fixed priorities -> per-index inclusion counts
            and first-position counts.
  ddpg.npz  a DDPGAgent (obs_dim 12, train_ddpg's hyper-parameters): its
            initial actor / critic weights, a filled memory, and three replay()
            steps -- the sampled idxs and IS weights of each, the returned
            losses, the priorities after each update, and all four networks'
            weights after the last one.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

sys.dont_write_bytecode = True
import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("F110_REFERENCE_ROOT", "/root/reference")
DDPG_DIR = os.path.join(REF, "rl_training", "DDPG")


def load_ddpg():
    pkg = types.ModuleType("_ref_DDPG")
    pkg.__path__ = [DDPG_DIR]
    sys.modules["_ref_DDPG"] = pkg
    mods = {}
    for name in ("replay_buffer", "agent"):
        spec = importlib.util.spec_from_file_location(f"_ref_DDPG.{name}", os.path.join(DDPG_DIR, name + ".py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[spec.name] = mod
        spec.loader.exec_module(mod)
        mods[name] = mod
    return mods["replay_buffer"], mods["agent"]


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {name}: {os.path.getsize(path) / 1024:.1f} KiB")


def gen_per(rbm):
    PER = rbm.PrioritizedExperienceReplayBuffer
    rb = PER(buffer_size=16, batch_size=5, alpha=0.6)
    ops, prio, length, nxt = [], [], [], []
    samples = {"idx": [], "w": [], "probs": [], "op": []}
    upd_idx, upd_val = [], []

    def record(op):
        ops.append(op)
        prio.append(rb._buffer["priority"].copy())
        length.append(rb._length)
        nxt.append(rb._next_idx)

    def sample(beta):
        idxs, _, w = rb.sample(beta=beta)
        ps = rb._buffer["priority"][: rb._length]
        pa = np.power(ps + rb._eps, rb._alpha, dtype=np.float64)
        samples["idx"].append(np.pad(idxs, (0, 5 - len(idxs)), constant_values=-1))
        samples["w"].append(w)
        samples["probs"].append(np.pad(pa / pa.sum(), (0, 16 - len(pa))))
        samples["op"].append(len(ops))
        record(2)

    def update(idxs, vals):
        rb.update_priorities(np.asarray(idxs), np.asarray(vals, dtype=np.float32))
        upd_idx.append(np.pad(np.asarray(idxs, np.int64), (0, 5 - len(idxs)), constant_values=-1))
        upd_val.append(np.pad(np.asarray(vals, np.float32), (0, 5 - len(vals))))
        record(3)

    for _ in range(3):
        rb.add(object())
        record(0)
    sample(0.4)                                    # len 3 < batch 5: replace=True
    update([0, 2, 0, 1, 2], [0.5, np.nan, 3.0, -1.0, 2.5])  # duplicates: last wins; -1 -> 1e-8; NaN -> 1e-6
    for k in range(20):                            # wraps the 16-slot ring
        if k % 7 == 3:
            rb.add(object(), priority=0.25 * k)
        else:
            rb.add(object())
        record(1 if k % 7 == 3 else 0)
    sample(0.4)                                    # without replacement
    update(list(samples["idx"][-1][:5]), [1e39, 0.0, 7.5, np.inf, 0.125])  # f32 inf -> clip to max
    sample(0.7)
    rng = np.random.default_rng(5)
    for _ in range(4):
        rb.add(object())
        record(0)
        idxs = samples["idx"][-1][:5]
        update(list(idxs), list(rng.exponential(1.0, 5)))
        sample(0.4)

    # sampling statistics on a fixed 40-row buffer
    st = PER(buffer_size=40, batch_size=6, alpha=0.6, seed=7)
    pr = np.random.default_rng(3).lognormal(0.0, 1.0, 40).astype(np.float32)
    for i in range(40):
        st.add(object(), priority=float(pr[i]))
    incl = np.zeros(40, np.int64)
    first = np.zeros(40, np.int64)
    n_draws = 20000
    for _ in range(n_draws):
        idxs, _, _ = st.sample(beta=0.4)
        incl[idxs] += 1
        first[idxs[0]] += 1
    ps = st._buffer["priority"][:40]
    pa = np.power(ps + st._eps, st._alpha, dtype=np.float64)
    save("per.npz", ops=np.array(ops), prio=np.stack(prio), length=np.array(length), next_idx=np.array(nxt),
         sample_idx=np.stack(samples["idx"]), sample_w=np.stack(samples["w"]), sample_probs=np.stack(samples["probs"]),
         sample_op=np.array(samples["op"]), upd_idx=np.stack(upd_idx), upd_val=np.stack(upd_val),
         stat_prio=ps.copy(), stat_probs=pa / pa.sum(), stat_incl=incl, stat_first=first,
         stat_draws=np.int64(n_draws), stat_batch=np.int64(6))


def _state(net):
    return {k: v.detach().cpu().numpy().copy() for k, v in net.state_dict().items()}


def gen_ddpg(agm):
    obs_dim, act_dim = 12, 2
    low = np.array([-0.4189, 0.0], np.float32)
    high = np.array([0.4189, 20.0], np.float32)
    # train_ddpg.py:80-108 with ddpg_config.yaml's hyper-parameters, smaller memory / batch
    agent = agm.DDPGAgent(state_size=obs_dim, action_size=act_dim, path="/tmp/_ddpg_golden", agent_id=0,
                          action_low=low, action_high=high, gamma=0.99, tau=0.005, actor_lr=1e-4, critic_lr=1e-3,
                          memory_size=64, batch_size=16, alpha=0.6, beta=0.4, priority_epsilon=1e-5,
                          noise_type="gaussian", noise_sigma_start=0.2, noise_sigma_min=0.02, noise_decay=0.9995,
                          seed=42)
    out = {}
    for name, net in (("actor", agent.actor), ("critic", agent.critic)):
        for k, v in _state(net).items():
            out[f"init/{name}/{k}"] = v
    rng = np.random.default_rng(11)
    N = 48
    S = rng.normal(0.0, 1.0, (N, obs_dim)).astype(np.float32)
    A = np.stack([rng.uniform(low[0], high[0], N), rng.uniform(low[1], high[1], N)], 1).astype(np.float32)
    R = rng.normal(0.0, 2.0, N).astype(np.float32)
    S2 = (S + rng.normal(0.0, 0.1, (N, obs_dim))).astype(np.float32)
    D = rng.random(N) < 0.15
    for i in range(N):
        agent.remember(S[i], A[i], float(R[i]), S2[i], bool(D[i]))
    out.update(S=S, A=A, R=R, S2=S2, D=D.astype(np.uint8))
    orig = agent.memory.sample
    rec = []

    def sample(beta=0.4):
        idxs, exps, w = orig(beta=beta)
        rec.append((np.asarray(idxs).copy(), np.asarray(w).copy()))
        return idxs, exps, w

    agent.memory.sample = sample
    losses, prios = [], []
    for _ in range(3):
        st = agent.replay()
        losses.append([st["critic_loss"], st["actor_loss"], st["mean_td_abs"]])
        prios.append(agent.memory._buffer["priority"][:N].copy())
    out["idx"] = np.stack([r[0] for r in rec])
    out["w"] = np.stack([r[1] for r in rec])
    out["losses"] = np.array(losses)
    out["prios"] = np.stack(prios)
    for name, net in (("actor", agent.actor), ("critic", agent.critic), ("actor_target", agent.actor_target),
                      ("critic_target", agent.critic_target)):
        for k, v in _state(net).items():
            out[f"final/{name}/{k}"] = v
    save("ddpg.npz", **out)


def main():
    rbm, agm = load_ddpg()
    gen_per(rbm)
    gen_ddpg(agm)


if __name__ == "__main__":
    main()
