"""Fused DDPG output heads (include/f110.h "learner heads", csrc/f110_ddpg.hip).

The last layer of each DDPG network and what replay() does with it
(rl_training/DDPG/agent.py):

  actor_head   fc3 -> tanh -> 0.5*(high-low)*t + 0.5*(high+low)   (:56-61)
  td_target    r + gamma * (1 - d) * critic_target.q(h)            (:302-308)
  critic_loss  td = y - critic.q(h); mean(w * td**2)               (:310-316)
  q_mean       -mean(critic.q(h))  (the actor loss)                (:321-326)

as torch.autograd.Functions over HIP kernels: one row-parallel launch
forward, a row pass and a deterministic two-pass weight reduction backward,
instead of a skinny GEMM (N = 1 or 2) and 3-10 elementwise launches.  They
run on the caller's current stream and allocate through torch, so a HIP
graph can capture them.  Device tensors only: there is no CPU path here
(DDPG on the CPU uses the plain torch modules)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _scratch(L, B, K, n, like):
    m = L.f110_ddpg_scratch_floats(B, K, n)
    if m < 0:
        raise _lib.F110Error(f"learner head: unsupported shape B={B} K={K} nout={n}")
    return torch.empty(int(m), dtype=torch.float32, device=like.device)


def _check(h, W, b):
    if not (h.is_cuda and W.is_cuda and b.is_cuda):
        raise _lib.F110Error("learner heads run on a HIP device only")
    if h.dtype != torch.float32 or W.dtype != torch.float32:
        raise _lib.F110Error("learner heads are float32")
    if h.dim() != 2 or W.dim() != 2 or h.shape[1] != W.shape[1] or b.numel() != W.shape[0]:
        raise _lib.F110Error(f"learner head shapes: h {tuple(h.shape)} W {tuple(W.shape)} b {tuple(b.shape)}")


class _ActorHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, W, b, scale, shift):
        _check(h, W, b)
        L = _lib.load()
        h, W, b = h.contiguous(), W.contiguous(), b.contiguous()
        B, K = h.shape
        n = W.shape[0]
        act = torch.empty(B, n, dtype=torch.float32, device=h.device)
        t = torch.empty_like(act)
        _lib.check(L.f110_ddpg_actor_head(_p(h), _p(W), _p(b), _p(scale), _p(shift), B, K, n, _p(act), _p(t),
                                          _stream(h)), "f110_ddpg_actor_head")
        ctx.save_for_backward(h, W, t, scale)
        return act

    @staticmethod
    def backward(ctx, dact):
        h, W, t, scale = ctx.saved_tensors
        L = _lib.load()
        B, K = h.shape
        n = W.shape[0]
        nh, nw, nb = ctx.needs_input_grad[:3]
        dh = torch.empty_like(h) if nh else None
        dW = torch.empty_like(W) if nw else None
        db = torch.empty(n, dtype=torch.float32, device=h.device) if nb else None
        dact = dact.contiguous()
        _lib.check(L.f110_ddpg_actor_head_bwd(_p(h), _p(W), _p(t), _p(scale), _p(dact), B, K, n, _p(dh), None,
                                              _p(dW), _p(db), _p(_scratch(L, B, K, n, h)), _stream(h)),
                   "f110_ddpg_actor_head_bwd")
        return dh, dW, db, None, None


class _CriticLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, W, b, y, w):
        _check(h, W, b)
        L = _lib.load()
        h, W, b = h.contiguous(), W.contiguous(), b.contiguous()
        y, w = y.reshape(-1).contiguous(), w.reshape(-1).contiguous()
        B, K = h.shape
        td = torch.empty(B, 1, dtype=torch.float32, device=h.device)
        loss = torch.empty((), dtype=torch.float32, device=h.device)
        _lib.check(L.f110_ddpg_critic_loss(_p(h), _p(W), _p(b), _p(y), _p(w), B, K, _p(td), _p(loss),
                                           _p(_scratch(L, B, K, 1, h)), _stream(h)), "f110_ddpg_critic_loss")
        ctx.save_for_backward(h, W, td, w)
        ctx.mark_non_differentiable(td)
        return loss, td

    @staticmethod
    def backward(ctx, gloss, _gtd):
        h, W, td, w = ctx.saved_tensors
        L = _lib.load()
        B, K = h.shape
        nh, nw, nb = ctx.needs_input_grad[:3]
        dh = torch.empty_like(h) if nh else None
        dW = torch.empty_like(W) if nw else None
        db = torch.empty(1, dtype=torch.float32, device=h.device) if nb else None
        g = gloss.reshape(()).contiguous()
        _lib.check(L.f110_ddpg_critic_loss_bwd(_p(h), _p(W), _p(td), _p(w), _p(g), B, K, _p(dh), None, _p(dW),
                                               _p(db), _p(_scratch(L, B, K, 1, h)), _stream(h)), "f110_ddpg_critic_loss_bwd")
        return dh, dW, db, None, None


class _QMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, W, b, sign):
        _check(h, W, b)
        L = _lib.load()
        h, W, b = h.contiguous(), W.contiguous(), b.contiguous()
        B, K = h.shape
        loss = torch.empty((), dtype=torch.float32, device=h.device)
        _lib.check(L.f110_ddpg_q_mean(_p(h), _p(W), _p(b), float(sign), B, K, _p(loss),
                                      _p(_scratch(L, B, K, 1, h)), _stream(h)), "f110_ddpg_q_mean")
        ctx.save_for_backward(h, W)
        ctx.sign = float(sign)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        h, W = ctx.saved_tensors
        L = _lib.load()
        B, K = h.shape
        nh, nw, nb = ctx.needs_input_grad[:3]
        dh = torch.empty_like(h) if nh else None
        dW = torch.empty_like(W) if nw else None
        db = torch.empty(1, dtype=torch.float32, device=h.device) if nb else None
        g = gloss.reshape(()).contiguous()
        _lib.check(L.f110_ddpg_q_mean_bwd(_p(h), _p(W), _p(g), ctx.sign, B, K, _p(dh), None, _p(dW), _p(db),
                                          _p(_scratch(L, B, K, 1, h)), _stream(h)), "f110_ddpg_q_mean_bwd")
        return dh, dW, db, None


def actor_head(h, W, b, scale, shift):
    """0.5*(high-low) * tanh(h W^T + b) + 0.5*(high+low); scale / shift are
    those two float32 vectors."""
    return _ActorHead.apply(h, W, b, scale, shift)


def critic_loss(h, W, b, y, w):
    """(mean(w * td**2), td) with td = y - (h W^T + b); td [B, 1] is detached."""
    return _CriticLoss.apply(h, W, b, y, w)


def q_mean(h, W, b, sign: float = -1.0):
    """sign * mean(h W^T + b) (sign -1: the actor loss)."""
    return _QMean.apply(h, W, b, sign)


@torch.no_grad()
def td_target(h, W, b, r, d, gamma: float):
    """r + gamma * (1 - d) * (h W^T + b) as [B, 1] (no autograd)."""
    _check(h, W, b)
    L = _lib.load()
    h, W, b = h.contiguous(), W.contiguous(), b.contiguous()
    r, d = r.reshape(-1).contiguous(), d.reshape(-1).contiguous()
    B, K = h.shape
    y = torch.empty(B, 1, dtype=torch.float32, device=h.device)
    _lib.check(L.f110_ddpg_td_target(_p(h), _p(W), _p(b), _p(r), _p(d), float(gamma), B, K, _p(y), _stream(h)),
               "f110_ddpg_td_target")
    return y


def relu_bwd(gy, y, need_db: bool = True):
    """(threshold_backward(gy, y, 0), its column sums or None) in one pass."""
    L = _lib.load()
    gy, y = gy.contiguous(), y.contiguous()
    B, K = y.shape
    gz = torch.empty_like(y)
    db = torch.empty(K, dtype=torch.float32, device=y.device) if need_db else None
    m = L.f110_ddpg_relu_bwd_scratch_floats(B, K)
    if m < 0:
        raise _lib.F110Error(f"relu_bwd: unsupported shape B={B} K={K}")
    scratch = torch.empty(int(m), dtype=torch.float32, device=y.device) if need_db else None
    _lib.check(L.f110_ddpg_relu_bwd(_p(gy), _p(y), B, K, _p(gz), _p(db), _p(scratch), _stream(y)),
               "f110_ddpg_relu_bwd")
    return gz, db
