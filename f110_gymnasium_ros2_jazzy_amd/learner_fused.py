"""DDPGLearner.update's critic and actor phases on the GPU without autograd
(rl_training/DDPG/agent.py:302-331), every hidden layer on the learner GEMMs
(learner_gemm.py, csrc/f110_gemm.hip) and every output layer on the learner
heads (ddpg_heads.py, csrc/f110_ddpg.hip).

Same mathematics as the autograd graph of the reference's replay(), written
out layer by layer, with these launches merged:
  * the first layers that read one batch run as ONE grouped launch
    (critic phase: actor_target.fc1 and critic_target.fcs1 on next_states
    and critic.fcs1 on states; actor phase: actor.fc1 and the updated
    critic.fcs1 on states);
  * fcs2 reads its input [z, action] as z plus two epilogue columns (no
    torch.cat; agent.py:94);
  * threshold_backward is fused into the producer of each gradient (the
    head's dh, the input-gradient GEMM's output mask), and each bias gradient
    comes out of its weight gradient's launch;
  * every gradient is written straight into the network's flat gradient
    bucket (ddpg.GradBucket), which RCCL all-reduces and FlatAdam reads.
Results match the autograd path to fp32 rounding (different summation
orders); deterministic run to run.  Device tensors only.
"""
from __future__ import annotations

import torch

from . import _lib
from . import learner_gemm as lg
from .ddpg_heads import _p, _scratch, _stream


class ExplicitUpdate:
    H = 128  # hidden width of both networks (agent.py:35-37, :72-74)

    @staticmethod
    def supported(ln) -> bool:
        return ln.device.type == "cuda" and ln.act_dim <= 2 and ln.actor.fc1.out_features == ExplicitUpdate.H \
            and ln.critic.fcs1.out_features == ExplicitUpdate.H

    def __init__(self, ln):
        self.ln = ln
        self.L = _lib.load()
        self.one = torch.ones((), dtype=torch.float32, device=ln.device)  # d loss / d loss
        self.ga = dict(zip([n for n, _ in ln.actor.named_parameters()], ln.actor_grads.views))
        self.gc = dict(zip([n for n, _ in ln.critic.named_parameters()], ln.critic_grads.views))

    def _e(self, M, n=None):
        return torch.empty(M, self.H if n is None else n, dtype=torch.float32, device=self.ln.device)

    @staticmethod
    def _fwd(x, lin, y, x2=None):
        """relu(x W^T [+ x2 W[:, K:]^T] + b) of one Linear as a gemm op."""
        W = lin.weight
        K = x.shape[1]
        nx2 = 0 if x2 is None else x2.shape[1]
        if K + nx2 != W.shape[1]:
            raise _lib.F110Error(f"layer input {K}+{nx2} != weight columns {W.shape[1]}")
        return lg.op(x, W, y, W.shape[0], K, x.stride(0), W.stride(0), y.stride(0), bias=lin.bias, x2=x2,
                     w2=(W, K) if nx2 else None, nx2=nx2, ldx2=x2.stride(0) if nx2 else 0, ldw2=W.stride(0),
                     relu=True)

    def _actor_head(self, actor, h):
        W, b = actor.fc3.weight, actor.fc3.bias
        scale, shift = actor._affine()
        M, K = h.shape
        n = W.shape[0]
        act, t = self._e(M, n), self._e(M, n)
        _lib.check(self.L.f110_ddpg_actor_head(_p(h), _p(W), _p(b), _p(scale), _p(shift), M, K, n, _p(act), _p(t),
                                               _stream(h)), "f110_ddpg_actor_head")
        return act, t

    def critic(self, s, a, r, ns, d, w):
        """agent.py:302-319: TD target, critic loss, its gradients into the
        critic's bucket.  Returns (loss, td [M, 1])."""
        ln, L, H = self.ln, self.L, self.H
        at, ct, cr = ln.actor_target, ln.critic_target, ln.critic
        s, a, ns = s.contiguous(), a.contiguous(), ns.contiguous()
        r, d, w = r.reshape(-1).contiguous(), d.reshape(-1).contiguous(), w.reshape(-1).contiguous()
        M, D = s.shape
        nA = a.shape[1]
        dev = s.device
        h1t, z1t, z1 = self._e(M), self._e(M), self._e(M)
        lg.gemm([self._fwd(ns, at.fc1, h1t), self._fwd(ns, ct.fcs1, z1t), self._fwd(s, cr.fcs1, z1)], M, dev)
        h2t, z2 = self._e(M), self._e(M)
        lg.gemm([self._fwd(h1t, at.fc2, h2t), self._fwd(z1, cr.fcs2, z2, x2=a)], M, dev)
        a_next, _ = self._actor_head(at, h2t)
        z2t = self._e(M)
        lg.gemm([self._fwd(z1t, ct.fcs2, z2t, x2=a_next)], M, dev)
        # one launch: TD target (critic_target's head), td / w td^2 partials (critic's head) and the
        # head's backward: dq and g2 = dq Wq where z2 > 0 (d loss / d fcs2's pre-activation)
        td = self._e(M, 1)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        part = torch.empty(L.f110_ddpg_row_blocks(M), dtype=torch.float32, device=dev)
        dq = self._e(M, 1)
        g2 = self._e(M)
        _lib.check(L.f110_ddpg_critic_step(_p(z2t), _p(ct.q.weight), _p(ct.q.bias), _p(r), _p(d), ln.gamma,
                                           _p(z2), _p(cr.q.weight), _p(cr.q.bias), _p(w), _p(self.one), M, H,
                                           _p(td), _p(g2), _p(z2), _p(dq), _p(part), _stream(s)),
                   "f110_ddpg_critic_step")
        gc = self.gc
        Ws2 = cr.fcs2.weight
        ld2 = Ws2.stride(0)
        g1 = self._e(M)  # d loss / d fcs1's pre-activation: g2 Ws2[:, :H] where z1 > 0
        lg.gemm([lg.op(g2, Ws2, g1, H, H, H, ld2, H, omask=z1, nn=True)], M, dev)
        # the four weight gradients (q, fcs2 and its action columns, fcs1) in one launch; its
        # finishing launch also writes the loss
        lg.wgrad([lg.wop(g2, z1, gc["fcs2.weight"], H, H, H, H, ld2, db=gc["fcs2.bias"]),
                  lg.wop(g2, a, (gc["fcs2.weight"], H), H, nA, H, a.stride(0), ld2),
                  lg.wop(g1, s, gc["fcs1.weight"], H, D, H, s.stride(0), gc["fcs1.weight"].stride(0),
                         db=gc["fcs1.bias"]),
                  lg.wop(dq, z2, gc["q.weight"], 1, H, 1, H, gc["q.weight"].stride(0), db=gc["q.bias"])], M, dev,
                 loss=(part, 1.0, loss))
        return loss, td

    def actor(self, s):
        """agent.py:321-331 after the critic step: actor loss -mean(q) through
        the updated critic, its gradients into the actor's bucket."""
        ln, L, H = self.ln, self.L, self.H
        ac, cr = ln.actor, ln.critic
        s = s.contiguous()
        M, D = s.shape
        dev = s.device
        h1, z1 = self._e(M), self._e(M)
        lg.gemm([self._fwd(s, ac.fc1, h1), self._fwd(s, cr.fcs1, z1)], M, dev)
        h2 = self._e(M)
        lg.gemm([self._fwd(h1, ac.fc2, h2)], M, dev)
        act, t = self._actor_head(ac, h2)
        nA = act.shape[1]
        z2 = self._e(M)
        lg.gemm([self._fwd(z1, cr.fcs2, z2, x2=act)], M, dev)
        st = _stream(s)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        part = torch.empty(L.f110_ddpg_row_blocks(M), dtype=torch.float32, device=dev)
        g2 = self._e(M)  # d loss / d fcs2's pre-activation: (-1 / M) Wq where z2 > 0, with the q partials
        _lib.check(L.f110_ddpg_q_mean_step(_p(z2), _p(cr.q.weight), _p(cr.q.bias), _p(self.one), -1.0, M, H,
                                           _p(g2), _p(z2), _p(part), st), "f110_ddpg_q_mean_step")
        Ws2 = cr.fcs2.weight
        da = self._e(M, nA)  # g2 Ws2[:, H:]
        lg.gemm([lg.op(g2, (Ws2, H), da, nA, H, H, Ws2.stride(0), nA, nn=True)], M, dev)
        ga = self.ga
        scale, _ = ac._affine()
        gh2 = self._e(M)  # d loss / d fc2's pre-activation
        sc = _scratch(L, M, H, nA, s)  # its first M * nA floats: the actor head's dz
        _lib.check(L.f110_ddpg_actor_head_bwd(_p(h2), _p(ac.fc3.weight), _p(t), _p(scale), _p(da), M, H, nA, _p(gh2),
                                              _p(h2), None, None, _p(sc), st), "f110_ddpg_actor_head_bwd")
        gh1 = self._e(M)  # gh2 W2 where h1 > 0
        W2 = ac.fc2.weight
        lg.gemm([lg.op(gh2, W2, gh1, H, H, H, W2.stride(0), H, omask=h1, nn=True)], M, dev)
        dz = sc[:M * nA].view(M, nA)
        # fc2, fc1 and the head's fc3 in one launch; its finishing launch also writes the loss
        lg.wgrad([lg.wop(gh2, h1, ga["fc2.weight"], H, H, H, H, ga["fc2.weight"].stride(0), db=ga["fc2.bias"]),
                  lg.wop(gh1, s, ga["fc1.weight"], H, D, H, s.stride(0), ga["fc1.weight"].stride(0),
                         db=ga["fc1.bias"]),
                  lg.wop(dz, h2, ga["fc3.weight"], nA, H, nA, H, ga["fc3.weight"].stride(0), db=ga["fc3.bias"])],
                 M, dev, loss=(part, -1.0, loss))
        return loss

    def policy(self, actor, obs, explore=None):
        """Actor.forward without autograd (choose_action): fc1, fc2, head.
        explore = (state_in, state_out, decay, sigma_min, low, high, seed, out):
        the head adds sigma * N(0, 1) and clips to [low, high]
        (f110_ddpg_actor_explore; sigma and the call index from the f64 device
        pair state_in, the decayed pair written to state_out), writing the
        actions into out (rows may be strided; None: a new tensor), which is
        returned."""
        obs = obs.contiguous()
        M = obs.shape[0]
        h1, h2 = self._e(M), self._e(M)
        lg.gemm([self._fwd(obs, actor.fc1, h1)], M, obs.device)
        lg.gemm([self._fwd(h1, actor.fc2, h2)], M, obs.device)
        if explore is None:
            return self._actor_head(actor, h2)[0]
        st_in, st_out, decay, sigma_min, low, high, seed, out = explore
        W, b = actor.fc3.weight, actor.fc3.bias
        scale, shift = actor._affine()
        n = W.shape[0]
        if out is None:
            out = self._e(M, n)
        if out.shape != (M, n) or out.stride(1) != 1 or out.dtype != torch.float32:
            raise ValueError("policy: out must be [M, act_dim] float32 with unit column stride")
        _lib.check(self.L.f110_ddpg_actor_explore(_p(h2), _p(W), _p(b), _p(scale), _p(shift), M, h2.shape[1], n,
                                                  _p(st_in), _p(st_out), float(decay), float(sigma_min), _p(low),
                                                  _p(high), int(seed), _p(out), out.stride(0), _stream(h2)),
                   "f110_ddpg_actor_explore")
        return out
