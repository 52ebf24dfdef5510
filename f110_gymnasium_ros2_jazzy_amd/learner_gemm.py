"""The DDPG learner's hidden-layer GEMMs on the fp32 matrix cores
(include/f110.h "learner GEMMs", csrc/f110_gemm.hip).

`gemm` runs up to four GEMMs that share the batch rows M in one launch, each
C = epi(A' B + x2 w2^T + bias) with B a Linear's weight ([N][K], x W^T) or,
nn=True, the weight itself ([K][N], g W); the epilogue fuses the layer's bias
and ReLU, the critic's action columns of fcs2's input (agent.py:94's
torch.cat) and the threshold_backward masks.  `wgrad` runs up to four
weight / bias gradients dW = G'^T X, db = sum_rows G'.  Both are
deterministic, run on the current torch stream and take their scratch from
torch's allocator, so HIP graphs can capture them.  Operands are given as
(tensor, element offset) pairs or tensors; float32, row-major.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _ptr(x):
    if x is None:
        return None
    t, off = x if isinstance(x, tuple) else (x, 0)
    if t.dtype != torch.float32 or not t.is_cuda:
        raise _lib.F110Error("learner GEMM operands are float32 device tensors")
    return t.data_ptr() + 4 * off


def op(A, B, C, N: int, K: int, lda: int, ldb: int, ldc: int, bias=None, amask=None, omask=None, x2=None, w2=None,
       nx2: int = 0, ldx2: int = 0, ldw2: int = 0, relu: bool = False, nn: bool = False) -> _lib.F110GemmOp:
    """One f110_gemm_op (see include/f110.h)."""
    return _lib.F110GemmOp(_ptr(A), _ptr(B), _ptr(bias), _ptr(amask), _ptr(omask), _ptr(x2), _ptr(w2), _ptr(C),
                           N, K, lda, ldb, ldc, ldx2, ldw2, nx2, 1 if relu else 0, 1 if nn else 0)


def wop(G, X, dW, N: int, KX: int, ldg: int, ldx: int, ldw: int, db=None, gmask=None) -> _lib.F110WgradOp:
    """One f110_wgrad_op (see include/f110.h)."""
    return _lib.F110WgradOp(_ptr(G), _ptr(gmask), _ptr(X), _ptr(dW), _ptr(db), N, KX, ldg, ldx, ldw)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def gemm(ops, M: int, device) -> None:
    L = _lib.load()
    arr = (_lib.F110GemmOp * len(ops))(*ops)
    _lib.check(L.f110_learner_gemm(arr, len(ops), int(M), _stream(device)), "f110_learner_gemm")


def wgrad(ops, M: int, device, loss=None) -> None:
    """f110_learner_wgrad; loss = (partials, sign, out): also *out = sign *
    sum(partials) / M in the finishing launch (f110_learner_wgrad_loss)."""
    L = _lib.load()
    arr = (_lib.F110WgradOp * len(ops))(*ops)
    n = L.f110_learner_wgrad_scratch_floats(arr, len(ops), int(M))
    if n < 0:
        raise _lib.F110Error("f110_learner_wgrad: unsupported shapes")
    scratch = torch.empty(max(int(n), 1), dtype=torch.float32, device=device)
    if loss is None:
        _lib.check(L.f110_learner_wgrad(arr, len(ops), int(M), ctypes.c_void_p(scratch.data_ptr()), _stream(device)),
                   "f110_learner_wgrad")
        return
    part, sign, out = loss
    _lib.check(L.f110_learner_wgrad_loss(arr, len(ops), int(M), ctypes.c_void_p(scratch.data_ptr()),
                                         ctypes.c_void_p(part.data_ptr()), int(part.numel()), float(sign),
                                         ctypes.c_void_p(out.data_ptr()), _stream(device)),
               "f110_learner_wgrad_loss")


def linear(x, W, b=None, relu: bool = True, x2=None, W2=None, omask=None, out=None):
    """relu(x W^T [+ x2 W2^T] + b) for a Linear (W [N][ldw], its first K = x's
    columns; W2 = (W, K) for the trailing action columns): a one-op gemm."""
    M, K = x.shape
    N = W.shape[0]
    y = out if out is not None else torch.empty(M, N, dtype=torch.float32, device=x.device)
    nx2 = 0 if x2 is None else x2.shape[1]
    gemm([op(x, W, y, N, K, x.stride(0), W.stride(0), y.stride(0), bias=b, omask=omask, x2=x2, w2=W2, nx2=nx2,
             ldx2=x2.stride(0) if x2 is not None else 0, ldw2=W.stride(0) if x2 is not None else 0, relu=relu)],
         M, x.device)
    return y
