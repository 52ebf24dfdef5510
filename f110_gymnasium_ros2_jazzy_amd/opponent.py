"""Rule-based opponent on the device: gap_follow_action
(rl_training/utils/gap_follow.py:3-58) for a batch of float32 scans through
libf110's f110_gap_follow, bit-exact with the reference's NumPy float32
arithmetic.  train_ddpg.py:168 computes it on the host from the previous
step's info["scans"][1]; F110VectorEnv(opponent="gap_follow") keeps that loop
on the GPU.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib

ANGLE_MIN = -math.pi / 2          # gap_follow.py:44 defaults
ANGLE_INCREMENT = math.pi / 1080


def gap_follow(scans: torch.Tensor, out: torch.Tensor | None = None, angle_min: float = ANGLE_MIN,
               angle_increment: float = ANGLE_INCREMENT, return_gaps: bool = False, stream=None):
    """scans: float32 device tensor [M, B] (rows may be strided, e.g.
    ``sim.out.scans[:, 1]``).  Returns actions [M, 2] float32 (steer, speed),
    written into ``out`` if given (rows may be strided), plus the chosen gaps
    [M, 2] int32 when ``return_gaps``."""
    if scans.dim() != 2 or scans.dtype != torch.float32 or scans.device.type != "cuda" or scans.stride(1) != 1:
        raise ValueError("scans must be a float32 cuda tensor [M, B] with unit stride along beams")
    M, B = scans.shape
    if out is None:
        out = torch.empty(M, 2, dtype=torch.float32, device=scans.device)
    if out.shape != (M, 2) or out.dtype != torch.float32 or out.stride(1) != 1 or out.device != scans.device:
        raise ValueError("out must be a float32 [M, 2] tensor on the scans' device with unit column stride")
    gaps = torch.empty(M, 2, dtype=torch.int32, device=scans.device) if return_gaps else None
    L = _lib.load()
    s = stream if stream is not None else torch.cuda.current_stream(scans.device).cuda_stream
    _lib.check(L.f110_gap_follow(ctypes.c_void_p(scans.data_ptr()), M, scans.stride(0) if M > 1 else B, B,
                                 float(angle_min), float(angle_increment), ctypes.c_void_p(out.data_ptr()),
                                 out.stride(0) if M > 1 else 2,
                                 ctypes.c_void_p(gaps.data_ptr()) if gaps is not None else None,
                                 ctypes.c_void_p(s)), "f110_gap_follow")
    return (out, gaps) if return_gaps else out
