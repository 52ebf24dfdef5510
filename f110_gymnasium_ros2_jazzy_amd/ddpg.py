"""Data-parallel DDPG learner on PyTorch-ROCm.

Mirrors rl_training/DDPG/agent.py: ``Actor`` (:25-62) and ``Critic``
(:64-97) are the reference's networks (same layers, initialisation and seed
order), and ``DDPGLearner`` is ``DDPGAgent`` (:105-460) for batches of
envs on one GPU per rank:

  remember      agent.py:223   -> DeviceReplayBuffer.add (batched, masked)
  replay        agent.py:242   -> PER sample on the device, critic step, actor
                                  step, priority update, soft target update
  choose_action agent.py:350   -> actor + GaussianActionNoise (:507-539) on the
                                  device for [N, obs_dim] observations
  save_model / load_model      -> same checkpoint keys (weights_only loads)

Data parallelism: one process per GPU (torch.distributed, backend "nccl" =
RCCL over xGMI).  Every rank samples its own replay shard; after a backward
pass the gradients of a network are packed into ONE flat fp32 bucket and
all-reduced in a single collective (critic: 156 289 floats, actor: 156 162
floats at obs_dim 1088), then the optimizer step.  The critic's all-reduce must finish before the actor's
forward (the actor loss reads the updated critic), so the two buckets are two
collectives.  Ranks start from rank 0's weights and stay identical.
"""
from __future__ import annotations

import os
from typing import Sequence

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

# On a HIP device the networks' hidden layers run as GEMMs with the bias and
# ReLU fused into the BLAS epilogue (torch._addmm_activation: the same values
# as relu(linear(x))) and their output layers as the fused learner heads of
# ddpg_heads.py.  F110_DDPG_FUSED=0 keeps the plain torch modules (A/B runs).
FUSED = os.environ.get("F110_DDPG_FUSED", "1") != "0"
# The GPU learner's update runs without autograd (learner_fused.py: grouped
# fp32 matrix-core GEMMs with fused epilogues, gradients written straight into
# the flat buckets).  F110_DDPG_EXPLICIT=0 keeps the autograd path (A/B runs).
EXPLICIT = os.environ.get("F110_DDPG_EXPLICIT", "1") != "0"


# The learner's GEMM choices at batch 4096 (torch TunableOp, tuned on MI355X
# over hipBLASLt and rocBLAS solutions: tuning/tunableop_gfx950.csv, read-only).
# At C5's batch the learner update went 0.545 -> 0.486 ms.
# F110_TUNABLEOP=0 keeps torch's default heuristics.
TUNED_GEMMS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "tunableop_gfx950.csv")


def enable_tuned_gemms(device: torch.device) -> bool:
    """Load the shipped TunableOp results once (no tuning, no file writes).
    TunableOp validates the file against this torch / HIP / hipBLASLt / arch and
    ignores it on a mismatch; shapes not in the file keep the defaults.  The
    process-wide switch stays as the caller had it: `TunedGemms` turns it on
    only around the learner's own GEMMs."""
    if os.environ.get("F110_TUNABLEOP", "1") == "0" or device.type != "cuda" or not os.path.exists(TUNED_GEMMS):
        return False
    import torch.cuda.tunable as tunable
    if "gfx950" not in torch.cuda.get_device_properties(device).gcnArchName:
        return False
    with TunedGemms(True):
        if hasattr(tunable, "record_untuned_enable"):
            tunable.record_untuned_enable(False)
        tunable.set_filename(TUNED_GEMMS)
        return bool(tunable.read_file(TUNED_GEMMS))


class TunedGemms:
    """Context: TunableOp on (lookups only, tuning off) for the learner's
    GEMMs, then the caller's previous state back, so other models in the
    process keep their own GEMM dispatch."""

    def __init__(self, on: bool):
        self.on = bool(on)
        self._prev = None

    def __enter__(self):
        if self.on:
            import torch.cuda.tunable as tunable
            self._prev = (tunable.is_enabled(), tunable.tuning_is_enabled())
            tunable.enable(True)
            tunable.tuning_enable(False)
        return self

    def __exit__(self, *exc):
        if self._prev is not None:
            import torch.cuda.tunable as tunable
            tunable.tuning_enable(self._prev[1])
            tunable.enable(self._prev[0])
            self._prev = None
        return False


def _fused(x: torch.Tensor) -> bool:
    return FUSED and x.is_cuda


class _LinearReLU(torch.autograd.Function):
    """relu(x W^T + b) with the ReLU in the GEMM epilogue; backward as
    autograd does it for relu(linear): threshold on the result, two GEMMs
    and a bias sum (only the ones whose inputs need a gradient)."""

    @staticmethod
    def forward(ctx, x, W, b):
        y = torch._addmm_activation(b, x, W.t())
        ctx.save_for_backward(x, W, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W, y = ctx.saved_tensors
        nx, nw, nb = ctx.needs_input_grad
        from .ddpg_heads import relu_bwd
        gz, db = relu_bwd(gy, y, nb)  # one HIP pass: threshold_backward + the bias gradient's column sums
        return (gz.mm(W) if nx else None, gz.t().mm(x) if nw else None, db)


def _linear_relu(lin: nn.Linear, x: torch.Tensor) -> torch.Tensor:
    return _LinearReLU.apply(x, lin.weight, lin.bias)


class Actor(nn.Module):
    """agent.py:25-62: obs -> 128 -> 128 -> act_dim, tanh scaled to [low, high]."""

    def __init__(self, obs_dim, act_dim, action_low: Sequence[float], action_high: Sequence[float]):
        super().__init__()
        self.fc1 = nn.Linear(obs_dim, 128)
        self.fc2 = nn.Linear(128, 128)
        self.fc3 = nn.Linear(128, act_dim)
        self.register_buffer("action_low", torch.tensor(action_low, dtype=torch.float32))
        self.register_buffer("action_high", torch.tensor(action_high, dtype=torch.float32))
        nn.init.kaiming_uniform_(self.fc1.weight, nonlinearity="relu")  # :41-47
        nn.init.kaiming_uniform_(self.fc2.weight, nonlinearity="relu")
        nn.init.uniform_(self.fc3.weight, -3e-3, 3e-3)
        nn.init.zeros_(self.fc1.bias)
        nn.init.zeros_(self.fc2.bias)
        nn.init.zeros_(self.fc3.bias)

    def forward(self, obs: torch.Tensor) -> torch.Tensor:
        if obs.dim() == 1:
            obs = obs.unsqueeze(0)
        if _fused(obs):
            from .ddpg_heads import actor_head
            x = _linear_relu(self.fc2, _linear_relu(self.fc1, obs))
            return actor_head(x, self.fc3.weight, self.fc3.bias, *self._affine())
        x = F.relu(self.fc1(obs))
        x = F.relu(self.fc2(x))
        t = torch.tanh(self.fc3(x))
        low, high = self.action_low, self.action_high
        return 0.5 * (high - low) * t + 0.5 * (high + low)  # :60-61

    def _affine(self):
        """0.5*(high-low), 0.5*(high+low) as forward computes them (:60-61),
        cached until the bounds change (the learner's eager warm-up fills the
        cache before any graph capture)."""
        low, high = self.action_low, self.action_high
        key = (low.data_ptr(), high.data_ptr(), low._version, high._version)
        if getattr(self, "_aff_key", None) != key:
            self._aff = (0.5 * (high - low), 0.5 * (high + low))
            self._aff_key = key
        return self._aff


class Critic(nn.Module):
    """agent.py:64-97: obs -> 128, concat action -> 128 -> 1."""

    def __init__(self, obs_dim: int, act_dim: int):
        super().__init__()
        self.fcs1 = nn.Linear(obs_dim, 128)
        self.fcs2 = nn.Linear(128 + act_dim, 128)
        self.q = nn.Linear(128, 1)
        nn.init.kaiming_uniform_(self.fcs1.weight, nonlinearity="relu")  # :77-83
        nn.init.kaiming_uniform_(self.fcs2.weight, nonlinearity="relu")
        nn.init.uniform_(self.q.weight, -3e-3, 3e-3)
        nn.init.zeros_(self.fcs1.bias)
        nn.init.zeros_(self.fcs2.bias)
        nn.init.zeros_(self.q.bias)

    def forward(self, obs: torch.Tensor, act: torch.Tensor) -> torch.Tensor:
        if obs.dim() == 1:
            obs = obs.unsqueeze(0)
        if act.dim() == 1:
            act = act.unsqueeze(0)
        return self.q(self.hidden(obs, act))

    def hidden(self, obs: torch.Tensor, act: torch.Tensor) -> torch.Tensor:
        """The input of the q layer (agent.py:93-96)."""
        if _fused(obs):
            z = torch.cat([_linear_relu(self.fcs1, obs), act], dim=-1)
            return _linear_relu(self.fcs2, z)
        z = F.relu(self.fcs1(obs))
        z = torch.cat([z, act], dim=-1)
        return F.relu(self.fcs2(z))


class GradBucket:
    """Gradient all-reduce of one network as ONE flat fp32 bucket.

    Backward writes fresh .grad tensors (set_to_none semantics, no
    accumulate kernels); with more than one rank they are gathered into the
    flat bucket by one cat, all-reduced by RCCL (sum, then one scale) and the
    parameters' .grad become views of the averaged bucket for the optimizer
    step."""

    def __init__(self, module: nn.Module, group=None, always_pack: bool = False):
        self.always_pack = always_pack  # flat-Adam path: the optimizer reads self.flat
        self.params = [p for p in module.parameters()]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        self.group = group
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        self.direct = False  # learner_fused writes the gradients into self.flat itself (no .grad tensors)

    def zero(self):
        for p in self.params:  # optimizer.zero_grad(set_to_none=True) (agent.py:318, :329)
            p.grad = None

    # pack / reduce / unpack: in graph mode pack ends one captured phase,
    # reduce runs eagerly (RCCL) and unpack starts the next captured phase
    def pack(self):
        if self.direct:
            return
        if self.world > 1 or self.always_pack:
            torch.cat([p.grad.reshape(-1) for p in self.params], out=self.flat)

    def reduce(self):
        if self.world > 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
            self.flat.mul_(1.0 / self.world)

    def unpack(self):
        if self.world > 1 and not self.always_pack and not self.direct:
            torch._foreach_copy_([p.grad for p in self.params], self.views)

    def all_reduce(self):
        self.pack()
        self.reduce()
        self.unpack()


def flatten_params(module: nn.Module) -> torch.Tensor:
    """Re-home a module's parameters into ONE flat fp32 buffer (the
    nn.Parameters become views of it) and return the buffer."""
    params = list(module.parameters())
    flat = torch.cat([p.detach().reshape(-1) for p in params]).contiguous()
    off = 0
    for p in params:
        p.data = flat[off:off + p.numel()].view_as(p)
        off += p.numel()
    return flat


class FlatAdam:
    """torch.optim.Adam (agent.py:187-188) over a flat parameter buffer: one
    libf110 f110_adam_step launch per network and step (the step counter lives
    on the device, so it can run inside a HIP graph).  state_dict() /
    load_state_dict() use torch.optim.Adam's per-parameter layout, so
    checkpoints stay interchangeable with the reference agent's."""

    def __init__(self, module: nn.Module, flat: torch.Tensor, lr: float, betas=(0.9, 0.999), eps: float = 1e-8):
        from . import _lib
        self.L = _lib.load()
        self._check = _lib.check
        self.params = list(module.parameters())
        self.flat = flat
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        self.exp_avg = torch.zeros_like(flat)
        self.exp_avg_sq = torch.zeros_like(flat)
        self.state = torch.zeros(2, dtype=torch.int64, device=flat.device)  # [step, scratch]

    def step(self, flat_grad: torch.Tensor, target: torch.Tensor | None = None, tau: float = 0.0):
        """One Adam step; with ``target`` (the target network's flat buffer) its
        soft update target.lerp_(param, tau) follows in the same launch."""
        import ctypes
        s = torch.cuda.current_stream(self.flat.device).cuda_stream
        vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        self._check(self.L.f110_adam_step(vp(self.flat), vp(self.exp_avg), vp(self.exp_avg_sq), vp(flat_grad),
                                          self.flat.numel(), self.lr, self.betas[0], self.betas[1], self.eps,
                                          vp(self.state), vp(target) if target is not None else None, float(tau),
                                          ctypes.c_void_p(s)), "f110_adam_step")

    def _views(self, flat):
        out, off = [], 0
        for p in self.params:
            out.append(flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        return out

    def state_dict(self):
        step = float(self.state[0].item())
        st = {i: {"step": torch.tensor(step), "exp_avg": a.detach().clone(), "exp_avg_sq": b.detach().clone()}
              for i, (a, b) in enumerate(zip(self._views(self.exp_avg), self._views(self.exp_avg_sq)))}
        return {"state": st, "param_groups": [{"lr": self.lr, "betas": self.betas, "eps": self.eps,
                                               "weight_decay": 0, "amsgrad": False,
                                               "params": list(range(len(self.params)))}]}

    def load_state_dict(self, sd):
        with torch.no_grad():
            for i, (a, b) in enumerate(zip(self._views(self.exp_avg), self._views(self.exp_avg_sq))):
                if i in sd["state"]:
                    a.copy_(sd["state"][i]["exp_avg"])
                    b.copy_(sd["state"][i]["exp_avg_sq"])
            steps = [float(v["step"]) for v in sd["state"].values()]
            self.state[0] = int(max(steps)) if steps else 0
        self.lr = float(sd["param_groups"][0].get("lr", self.lr))


class DDPGLearner:
    """DDPGAgent (agent.py:105) for batched envs, one GPU per rank."""

    def __init__(self, obs_dim: int, act_dim: int, action_low, action_high, gamma: float = 0.99, tau: float = 0.005,
                 actor_lr: float = 1e-4, critic_lr: float = 1e-3, memory_size: int = 1 << 20, batch_size: int = 128,
                 alpha: float = 0.6, beta: float = 0.4, priority_epsilon: float = 1e-5,
                 noise_sigma_start: float = 0.2, noise_sigma_min: float = 0.05, noise_decay: float = 0.999,
                 seed: int = 42, device="cuda:0", replay="device", process_group=None, max_add: int | None = None,
                 check_finite: bool = False, path: str | None = None, graphs: bool = False):
        self.device = torch.device(device)
        self.tuned_gemms = enable_tuned_gemms(self.device)
        self.obs_dim, self.act_dim = int(obs_dim), int(act_dim)
        self.action_low = np.asarray(action_low, dtype=np.float32)
        self.action_high = np.asarray(action_high, dtype=np.float32)
        assert self.action_low.shape == (self.act_dim,) and self.action_high.shape == (self.act_dim,)
        self.batch_size = int(batch_size)
        self.gamma, self.tau, self.beta = float(gamma), float(tau), float(beta)
        self.priority_epsilon = float(priority_epsilon)
        self.check_finite = bool(check_finite)
        self.path = path
        # agent.py:176-184: seed, then the four networks in this order, built on
        # the CPU generator so every device (and rank) starts from the same weights
        torch.manual_seed(seed)
        self.actor = Actor(self.obs_dim, self.act_dim, self.action_low, self.action_high)
        self.critic = Critic(self.obs_dim, self.act_dim)
        self.actor_target = Actor(self.obs_dim, self.act_dim, self.action_low, self.action_high)
        self.critic_target = Critic(self.obs_dim, self.act_dim)
        self.actor_target.load_state_dict(self.actor.state_dict())
        self.critic_target.load_state_dict(self.critic.state_dict())
        for net in (self.actor, self.critic, self.actor_target, self.critic_target):
            net.to(self.device)
        self.group = process_group
        self.distributed = dist.is_available() and dist.is_initialized()
        if self.distributed:  # every rank starts from rank 0's weights
            for net in (self.actor, self.critic, self.actor_target, self.critic_target):
                for t in list(net.parameters()) + list(net.buffers()):
                    dist.broadcast(t.data, src=0, group=self.group)
        # On the GPU each network is one flat buffer (parameters are views):
        # its gradient bucket feeds one flat Adam launch and the soft target
        # update is one lerp over the buffers.  The CPU path keeps
        # torch.optim.Adam (the reference's own optimizer, for parity tests).
        self.flat = self.device.type == "cuda"
        if self.flat:
            self._flat = {n: flatten_params(net) for n, net in (("actor", self.actor), ("critic", self.critic),
                                                                 ("actor_target", self.actor_target),
                                                                 ("critic_target", self.critic_target))}
        self.actor_grads = GradBucket(self.actor, self.group, always_pack=self.flat)
        self.critic_grads = GradBucket(self.critic, self.group, always_pack=self.flat)
        self.graphs = bool(graphs) and self.device.type == "cuda" and replay is not None
        self._graphs, self._graph_out, self._eager_left = None, None, 3
        self._side = torch.cuda.Stream(self.device) if self.graphs else None
        if self.flat:
            self.actor_optim = FlatAdam(self.actor, self._flat["actor"], lr=actor_lr)
            self.critic_optim = FlatAdam(self.critic, self._flat["critic"], lr=critic_lr)
            self._online = [self._flat["actor"], self._flat["critic"]]
            self._target = [self._flat["actor_target"], self._flat["critic_target"]]
        else:
            self.actor_optim = torch.optim.Adam(self.actor.parameters(), lr=actor_lr)
            self.critic_optim = torch.optim.Adam(self.critic.parameters(), lr=critic_lr)
            self._online = list(self.actor.parameters()) + list(self.critic.parameters())
            self._target = list(self.actor_target.parameters()) + list(self.critic_target.parameters())
        self.explicit = None
        if self.flat and FUSED and EXPLICIT:
            from .learner_fused import ExplicitUpdate
            if ExplicitUpdate.supported(self):
                self.explicit = ExplicitUpdate(self)
                self.actor_grads.direct = self.critic_grads.direct = True
        self.memory = None
        if replay == "device":
            from .replay import DeviceReplayBuffer
            self.memory = DeviceReplayBuffer(buffer_size=memory_size, batch_size=self.batch_size, alpha=alpha,
                                             seed=seed + 7919 * (dist.get_rank() if self.distributed else 0),
                                             obs_dim=self.obs_dim, act_dim=self.act_dim, device=self.device,
                                             max_add=max_add)
        elif replay is not None:
            self.memory = replay
        # GaussianActionNoise (agent.py:507-539) on the device
        self.sigma = float(noise_sigma_start)
        self.sigma_min, self.noise_decay = float(noise_sigma_min), float(noise_decay)
        self._noise_gen = torch.Generator(device=self.device)
        self._noise_gen.manual_seed(seed)
        self._low = torch.as_tensor(self.action_low, device=self.device)
        self._high = torch.as_tensor(self.action_high, device=self.device)
        # the explicit path draws the noise inside its head launch (f110_ddpg_actor_explore): per rank a
        # key, per call a counter
        self._low32 = self._low.to(torch.float32).contiguous()
        self._high32 = self._high.to(torch.float32).contiguous()
        self._noise_key = (int(seed) * 1000003 + (dist.get_rank() if self.distributed else 0)) & ((1 << 64) - 1)
        self._noise_calls = 0
        # (sigma, call index) on the device in two f64 slots: a call reads slot _noise_slot and writes
        # the decayed pair to the other (so a captured step graph can replay it); the host mirrors the
        # same double arithmetic in self.sigma / self._noise_calls
        self._noise_state = torch.tensor([[self.sigma, 0.0]] * 2, dtype=torch.float64, device=self.device)
        self._noise_slot = 0
        self._noise_dev = (self.sigma, 0)  # what the current slot holds
        self._ready = False
        self.global_step = 0

    # ------------------------------------------------------------------
    def remember(self, state, action, reward, next_state, done, mask=None):
        """agent.py:223-237 for a batch of transitions (rows with mask == 0 skipped)."""
        self.memory.add(state, action, reward, next_state, done, mask=mask)

    def remember_env(self, state, action, reward, next_state, terminated, was_reset):
        """remember() of a vector env's raw outputs (float64 rewards, uint8
        terminated / was_reset flags; reset rows skipped) without torch-side
        conversions (DeviceReplayBuffer.add_env)."""
        self.memory.add_env(state, action, reward, next_state, terminated, was_reset)

    def _finite(self, name, x):  # agent.py:291-296 (host sync; only with check_finite)
        if self.check_finite and not bool(torch.isfinite(x).all()):
            bad = (~torch.isfinite(x)).nonzero(as_tuple=False)[:10].cpu().numpy().tolist()
            raise ValueError(f"Non-finite in {name}; examples idx={bad[:5]}")

    # The update is three phases split at the two gradient all-reduces, so a
    # HIP graph can hold each phase while the RCCL collectives stay eager.
    def _phase_critic(self, states, actions, rewards, next_states, dones, weights):
        """agent.py:302-319: TD target, critic loss, critic backward."""
        r = rewards.reshape(-1, 1)
        d = dones.reshape(-1, 1)
        w = weights.reshape(-1, 1)
        for name, t in (("states", states), ("actions", actions), ("next_states", next_states), ("rewards", r),
                        ("dones", d)):
            self._finite(name, t)
        if self.explicit is not None:  # learner_fused.py: the same graph without autograd
            critic_loss, td = self.explicit.critic(states, actions, r, next_states, d, w)
            self._finite("td", td)
            return critic_loss, td
        fused = _fused(states)
        with torch.no_grad():  # :302-308
            a_next = self.actor_target(next_states)
            if fused:
                from .ddpg_heads import td_target
                ct = self.critic_target
                target_y = td_target(ct.hidden(next_states, a_next), ct.q.weight, ct.q.bias, r, d, self.gamma)
            else:
                q_next = self.critic_target(next_states, a_next)
                target_y = r + self.gamma * (1.0 - d) * q_next
            self._finite("target_y", target_y)
        self.critic_grads.zero()               # :318-319
        if fused:  # :310-316
            from .ddpg_heads import critic_loss as fused_loss
            critic_loss, td = fused_loss(self.critic.hidden(states, actions), self.critic.q.weight,
                                         self.critic.q.bias, target_y, w)
        else:
            q_pred = self.critic(states, actions)  # :310-315
            td = target_y - q_pred
            critic_loss = (w * td ** 2).mean()
        critic_loss.backward()
        return critic_loss.detach(), td.detach()

    def _optim_step(self, optim, bucket, target=None):
        if self.flat:  # the flat path soft-updates the network's target in the same launch (agent.py:340-341)
            optim.step(bucket.flat, target, self.tau)
        else:
            optim.step()

    def _phase_actor(self, states):
        """agent.py:321-331: critic step, actor loss through the frozen critic."""
        self._optim_step(self.critic_optim, self.critic_grads, self._flat["critic_target"] if self.flat else None)
        if self.explicit is not None:
            return self.explicit.actor(states)
        for p in self.critic.parameters():
            p.requires_grad_(False)
        if _fused(states):
            from .ddpg_heads import q_mean
            actor_loss = q_mean(self.critic.hidden(states, self.actor(states)), self.critic.q.weight,
                                self.critic.q.bias, -1.0)
        else:
            actor_loss = -self.critic(states, self.actor(states)).mean()
        self.actor_grads.zero()
        actor_loss.backward()
        for p in self.critic.parameters():
            p.requires_grad_(True)
        return actor_loss.detach()

    def _phase_finish(self):
        """agent.py:331, :340-341: actor step, soft target update."""
        self._optim_step(self.actor_optim, self.actor_grads, self._flat["actor_target"] if self.flat else None)
        if not self.flat:  # (the flat path did both soft updates inside the Adam launches)
            with torch.no_grad():
                for tgt, src in zip(self._target, self._online):
                    tgt.lerp_(src, self.tau)

    def update(self, states, actions, rewards, next_states, dones, weights) -> dict:
        """The learning part of replay() (agent.py:302-343) on one batch:
        critic step, actor step, soft target update.  Returns device tensors
        (critic_loss, actor_loss, td [B])."""
        with TunedGemms(self.tuned_gemms):
            critic_loss, td = self._phase_critic(states, actions, rewards, next_states, dones, weights)
            self.critic_grads.all_reduce()
            actor_loss = self._phase_actor(states)
            self.actor_grads.all_reduce()
            self._phase_finish()
        self.global_step += 1
        return {"critic_loss": critic_loss, "actor_loss": actor_loss, "td": td}

    @staticmethod
    def td_priorities(td: torch.Tensor, priority_epsilon: float) -> torch.Tensor:
        """agent.py:337: new_priorities = |td| + priority_epsilon (float32)."""
        return td.abs().reshape(-1) + priority_epsilon

    def replay(self):
        """agent.py:242-348: None until the memory holds batch_size rows.
        With graphs=True the sample + update + priority update run as HIP
        graph replays (captured after a few eager updates): one launch per
        phase instead of ~150 kernel launches from Python."""
        if not self._ready:  # len() syncs; once full enough it stays so (the ring never shrinks)
            if len(self.memory) < self.batch_size:
                return None
            self._ready = True
        with TunedGemms(self.tuned_gemms):
            if self.graphs:
                return self._replay_graphed()
            return self._replay_eager()

    def _replay_eager(self):
        idxs, b, w = self.memory.sample(beta=self.beta)
        st = self.update(b["states"], b["actions"], b["rewards"], b["next_states"], b["dones"], w)
        self.memory.update_priorities(idxs, st["td"], td_errors=True, add_eps=self.priority_epsilon)
        return st

    def _graph_phases(self):
        """The replay() body as three callables split at the all-reduces."""
        m = self.memory
        out = {}

        def a():
            idxs, b, w = m.sample(beta=self.beta)
            out["critic_loss"], out["td"] = self._phase_critic(b["states"], b["actions"], b["rewards"],
                                                               b["next_states"], b["dones"], w)
            self.critic_grads.pack()

        def b_():
            self.critic_grads.unpack()
            out["actor_loss"] = self._phase_actor(m.batch["states"])
            self.actor_grads.pack()

        def c():
            self.actor_grads.unpack()
            self._phase_finish()
            m.update_priorities(m.idx, out["td"], td_errors=True, add_eps=self.priority_epsilon)
        return (a, b_, c), out

    def _replay_graphed(self):
        cur = torch.cuda.current_stream(self.device)
        if self._graphs is None:
            phases, out = self._graph_phases()
            if self._eager_left > 0:  # warm-up: real updates on a side stream (allocator, optimizer state)
                side = self._side
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    phases[0]()
                    self.critic_grads.reduce()
                    phases[1]()
                    self.actor_grads.reduce()
                    phases[2]()
                cur.wait_stream(side)
                self._eager_left -= 1
                self.global_step += 1
                return dict(out)
            graphs = [torch.cuda.CUDAGraph() for _ in phases]
            pool = torch.cuda.graph_pool_handle()
            for g, ph in zip(graphs, phases):  # capture records, it does not run
                with torch.cuda.graph(g, pool=pool, stream=self._side):
                    ph()
            self._graphs, self._graph_out = graphs, out
        g = self._graphs
        g[0].replay()
        self.critic_grads.reduce()  # eager RCCL between the captured phases
        g[1].replay()
        self.actor_grads.reduce()
        g[2].replay()
        self.global_step += 1
        return self._graph_out

    def choose_action(self, obs, training: bool = True, out: torch.Tensor | None = None) -> torch.Tensor:
        """agent.py:350-370 for obs [N, obs_dim] (or [obs_dim]): actor output,
        plus N(0, sigma^2) noise clipped to [low, high] when training; sigma
        decays once per call (GaussianActionNoise.__call__, :520-539).  On the
        explicit path a training call is one launch after the hidden layers
        (the head draws the noise and clips) and may write into out, a
        [N, act_dim] float32 view with unit column stride (e.g. the env's action rows)."""
        with torch.no_grad(), TunedGemms(self.tuned_gemms):
            o = torch.as_tensor(obs, device=self.device, dtype=torch.float32)
            if self.explicit is not None and training and o.dim() == 2:
                s = self._noise_slot
                if self._noise_dev != (self.sigma, self._noise_calls):  # the host changed sigma: upload it
                    self._noise_state[s, 0] = self.sigma
                    self._noise_state[s, 1] = float(self._noise_calls)
                a = self.explicit.policy(self.actor, o, explore=(
                    self._noise_state[s], self._noise_state[1 - s], self.noise_decay, self.sigma_min, self._low32,
                    self._high32, self._noise_key, out))
                self.noise_advance()
                return a
            if self.explicit is not None:
                a = self.explicit.policy(self.actor, o if o.dim() == 2 else o.unsqueeze(0))
                if o.dim() == 1:  # a single observation keeps agent.py's [act_dim] shape (:368-370)
                    a = a.squeeze(0)
            else:
                a = self.actor(o)
            if training:
                noise = torch.randn(a.shape, generator=self._noise_gen, device=self.device) * self.sigma
                a = torch.clamp(a + noise, self._low, self._high)
                self.sigma = max(self.sigma * self.noise_decay, self.sigma_min)
        if out is not None:
            out.copy_(a)
            return out
        return a

    def noise_advance(self):
        """The host mirror of one explicit training choose_action: the device
        slot flips and the pair decays as f110_ddpg_actor_explore decays it (a
        replayed step graph calls this per replay)."""
        self._noise_calls += 1
        self.sigma = max(self.sigma * self.noise_decay, self.sigma_min)
        self._noise_slot ^= 1
        self._noise_dev = (self.sigma, self._noise_calls)

    def hard_update(self):
        self.actor_target.load_state_dict(self.actor.state_dict())
        self.critic_target.load_state_dict(self.critic.state_dict())

    # ---------------------------------------------------------- checkpoint --
    def save_model(self, filename: str = "ddpg_checkpoint.pt"):
        """agent.py:384-405 (same keys)."""
        os.makedirs(self.path, exist_ok=True)
        torch.save({
            "actor": self.actor.state_dict(), "critic": self.critic.state_dict(),
            "actor_target": self.actor_target.state_dict(), "critic_target": self.critic_target.state_dict(),
            "actor_optim": self.actor_optim.state_dict(), "critic_optim": self.critic_optim.state_dict(),
            "action_low": self.action_low.tolist(), "action_high": self.action_high.tolist(),
            "gamma": self.gamma, "tau": self.tau, "obs_dim": self.obs_dim, "act_dim": self.act_dim,
            "global_step": self.global_step, "torch_version": torch.__version__,
        }, os.path.join(self.path, filename))

    def load_model(self, filename: str = "ddpg_checkpoint.pt") -> bool:
        """agent.py:407-460 with the safe loader only (weights_only=True)."""
        model_path = os.path.join(self.path, filename)
        if not os.path.exists(model_path):
            return False
        ckpt = torch.load(model_path, map_location=self.device, weights_only=True)
        self.actor.load_state_dict(ckpt["actor"], strict=True)
        self.critic.load_state_dict(ckpt["critic"], strict=True)
        self.actor_target.load_state_dict(ckpt.get("actor_target", ckpt["actor"]), strict=False)
        self.critic_target.load_state_dict(ckpt.get("critic_target", ckpt["critic"]), strict=False)
        if "actor_optim" in ckpt:
            self.actor_optim.load_state_dict(ckpt["actor_optim"])
        if "critic_optim" in ckpt:
            self.critic_optim.load_state_dict(ckpt["critic_optim"])
        self.gamma = float(ckpt.get("gamma", self.gamma))
        self.tau = float(ckpt.get("tau", self.tau))
        self.global_step = int(ckpt.get("global_step", 0))
        return True
