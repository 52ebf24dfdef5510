"""Batched collision_models on the device (collision_models.py:113-212).

    collision_batch(v1, v2)      -> uint8 [M]   GJK overlap of M vertex pairs
    collision_multiple(verts)    -> (collisions [M, N] f64, idx [M, N] f64)

Vertices are [.., 4, 2] float64 (get_vertices order: rl, rr, fr, fl), host
arrays or tensors; results are device tensors on `device` (cuda:0 default).
The kernels are the GJK of the batched step (f110_device.h gjk_collision)
behind f110_collision_batch / f110_collision_multiple.
"""
from __future__ import annotations

import torch

from . import _lib


def _dev(device):
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


def _ptr(t):
    return t.data_ptr() if t is not None else None


def collision_batch(v1, v2, device=None) -> torch.Tensor:
    """collision(vertices1, vertices2) (collision_models.py:113) for M pairs."""
    dev = _dev(device)
    a = torch.as_tensor(v1, dtype=torch.float64, device=dev).reshape(-1, 4, 2).contiguous()
    b = torch.as_tensor(v2, dtype=torch.float64, device=dev).reshape(-1, 4, 2).contiguous()
    if a.shape != b.shape:
        raise ValueError(f"v1 {tuple(a.shape)} and v2 {tuple(b.shape)} must both be [M, 4, 2]")
    out = torch.empty(a.shape[0], dtype=torch.uint8, device=dev)
    L = _lib.load()
    _lib.check(L.f110_collision_batch(_ptr(a), _ptr(b), a.shape[0], _ptr(out),
                                      torch.cuda.current_stream(dev).cuda_stream), "f110_collision_batch")
    return out


def collision_multiple(verts, device=None):
    """collision_multiple(vertices) (collision_models.py:184) for M sets of N
    bodies ([N, 4, 2] is one set): (collisions, collision_idx), float64 like
    the reference (1./0., partner index or -1.)."""
    dev = _dev(device)
    v = torch.as_tensor(verts, dtype=torch.float64, device=dev)
    single = v.dim() == 3
    if single:
        v = v.unsqueeze(0)
    if v.dim() != 4 or tuple(v.shape[2:]) != (4, 2):
        raise ValueError(f"verts must be [M, N, 4, 2] or [N, 4, 2]; got {tuple(v.shape)}")
    v = v.contiguous()
    M, N = v.shape[0], v.shape[1]
    col = torch.empty(M, N, dtype=torch.float64, device=dev)
    idx = torch.empty(M, N, dtype=torch.float64, device=dev)
    L = _lib.load()
    _lib.check(L.f110_collision_multiple(_ptr(v), M, N, _ptr(col), _ptr(idx),
                                         torch.cuda.current_stream(dev).cuda_stream), "f110_collision_multiple")
    return (col[0], idx[0]) if single else (col, idx)
