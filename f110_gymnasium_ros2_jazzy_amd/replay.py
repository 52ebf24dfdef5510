"""Prioritized experience replay in device memory.

Mirrors rl_training/DDPG/replay_buffer.py:PrioritizedExperienceReplayBuffer
(:6-135) -- same constructor arguments and defaults, ``add`` / ``sample`` /
``update_priorities`` / ``len`` -- for batches of transitions held as device
tensors.  Every call is libf110's ``f110_replay_*`` on the current torch
stream; nothing goes through the host on the per-step path.

    rb = DeviceReplayBuffer(buffer_size=1 << 20, batch_size=4096, obs_dim=1088, act_dim=2, device=0)
    rb.add(obs, act, rew, next_obs, done, mask=~reset)    # [n, 1088], [n, 2], [n], [n, 1088], [n]
    idx, batch, w = rb.sample(beta=0.4)                    # batch: states, actions, rewards, next_states, dones
    rb.update_priorities(idx, td, td_errors=True, add_eps=1e-5)   # |td| + eps (agent.py:337)

Sampling without replacement has the distribution of numpy's
``Generator.choice(replace=False, p=...)`` (an ordered successive sample);
the draws themselves come from a device Philox stream, not PCG64.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())



def _as_u8(t: torch.Tensor) -> torch.Tensor:
    """Flat uint8 flags; a contiguous bool tensor is reinterpreted (no copy)."""
    t = t.reshape(-1)
    if t.dtype == torch.bool and t.is_contiguous():
        return t.view(torch.uint8)
    return t.to(torch.uint8).contiguous()

class DeviceReplayBuffer:
    def __init__(self, buffer_size: int, batch_size: int, alpha: float = 0.6, seed: int = 42,
                 priority_epsilon: float = 1e-6, obs_dim: int = 1088, act_dim: int = 2, device=0,
                 max_add: int | None = None):
        if batch_size <= 0 or buffer_size <= 0:
            raise ValueError("buffer_size and batch_size must be positive")  # replay_buffer.py:26
        dev = torch.device(device if not isinstance(device, int) else f"cuda:{device}")
        if dev.type != "cuda" or not torch.cuda.is_available():
            raise _lib.F110Error("DeviceReplayBuffer runs on a HIP device only (no CPU path)")
        self.device = dev
        self.L = _lib.load()
        self._buffer_size = int(buffer_size)
        self._batch_size = int(batch_size)
        self._alpha = float(alpha)
        self._eps = float(priority_epsilon)
        self.obs_dim, self.act_dim = int(obs_dim), int(act_dim)
        self.max_add = int(max_add or min(self._buffer_size, 1 << 16))
        h = ctypes.c_void_p()
        _lib.check(self.L.f110_replay_create(ctypes.byref(h), dev.index or 0, self._buffer_size, self.obs_dim,
                                             self.act_dim, self._batch_size, self.max_add, self._alpha, self._eps,
                                             int(seed) & 0xFFFFFFFFFFFFFFFF), "f110_replay_create")
        self.handle = h
        kw = dict(device=dev)
        B = self._batch_size
        self.idx = torch.empty(B, dtype=torch.int64, **kw)
        self.weights = torch.empty(B, dtype=torch.float32, **kw)
        self.batch = {
            "states": torch.empty(B, self.obs_dim, dtype=torch.float32, **kw),
            "actions": torch.empty(B, self.act_dim, dtype=torch.float32, **kw),
            "rewards": torch.empty(B, dtype=torch.float32, **kw),
            "next_states": torch.empty(B, self.obs_dim, dtype=torch.float32, **kw),
            "dones": torch.empty(B, dtype=torch.float32, **kw),
        }
        self._added = 0  # host upper bound of len() (masked rows may not be stored)
        self._keep = None

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------
    def __len__(self) -> int:
        """replay_buffer.py:42-43 (waits for the stream)."""
        n = ctypes.c_int64()
        _lib.check(self.L.f110_replay_length(self.handle, ctypes.byref(n), None, self._stream()),
                   "f110_replay_length")
        return int(n.value)

    def add(self, states, actions, rewards, next_states, dones=None, mask=None, priority=None):
        """n add() calls (replay_buffer.py:48-71) in row order, priority = the
        current max (1.0 when empty) or ``priority`` [n].  Rows with mask == 0
        are not stored."""
        s = self._rows(states, self.obs_dim)
        ns = self._rows(next_states, self.obs_dim)
        a = self._rows(actions, self.act_dim)
        n = s.shape[0]
        r = torch.as_tensor(rewards, device=self.device).reshape(-1).to(torch.float32).contiguous()
        d = None if dones is None else _as_u8(torch.as_tensor(dones, device=self.device))
        m = None if mask is None else _as_u8(torch.as_tensor(mask, device=self.device))
        pr = None if priority is None else \
            torch.as_tensor(priority, device=self.device).reshape(-1).to(torch.float32).contiguous()
        if (pr is not None and pr.shape[0] != n) or ns.shape[0] != n or a.shape[0] != n or r.shape[0] != n or (d is not None and d.shape[0] != n) or \
                (m is not None and m.shape[0] != n):
            raise ValueError("add: every input needs the same number of rows")
        self._keep = (s, ns, a, r, d, m, pr)  # alive until the stream has consumed them
        for lo in range(0, n, self.max_add):
            hi = min(n, lo + self.max_add)
            _lib.check(self.L.f110_replay_add(
                self.handle, _p(s[lo:hi]), s.stride(0), _p(a[lo:hi]), a.stride(0), _p(r[lo:hi]), _p(ns[lo:hi]),
                ns.stride(0), _p(None if d is None else d[lo:hi]), _p(None if pr is None else pr[lo:hi]),
                _p(None if m is None else m[lo:hi]), hi - lo,
                self._stream()), "f110_replay_add")
        self._added += n

    def add_env(self, states, actions, rewards, next_states, terminated, was_reset):
        """add() of a vector env's raw step outputs (f110_replay_add_env): rewards
        float64, terminated / was_reset uint8 device tensors as the simulator
        writes them; rows with was_reset != 0 are not stored.  No dtype
        conversions on the torch side."""
        s = self._rows(states, self.obs_dim)
        ns = self._rows(next_states, self.obs_dim)
        a = self._rows(actions, self.act_dim)
        n = s.shape[0]
        r, d, m = rewards.reshape(-1), terminated.reshape(-1), was_reset.reshape(-1)
        if r.dtype != torch.float64 or d.dtype != torch.uint8 or m.dtype != torch.uint8:
            raise TypeError("add_env: rewards float64, terminated and was_reset uint8")
        if not (r.is_contiguous() and d.is_contiguous() and m.is_contiguous()):
            raise ValueError("add_env: contiguous rewards / flags")
        if ns.shape[0] != n or a.shape[0] != n or r.shape[0] != n or d.shape[0] != n or m.shape[0] != n:
            raise ValueError("add_env: every input needs the same number of rows")
        self._keep = (s, ns, a, r, d, m)  # alive until the stream has consumed them
        for lo in range(0, n, self.max_add):
            hi = min(n, lo + self.max_add)
            _lib.check(self.L.f110_replay_add_env(
                self.handle, _p(s[lo:hi]), s.stride(0), _p(a[lo:hi]), a.stride(0), _p(r[lo:hi]), _p(ns[lo:hi]),
                ns.stride(0), _p(d[lo:hi]), _p(m[lo:hi]), hi - lo, self._stream()), "f110_replay_add_env")
        self._added += n

    def _rows(self, x, width):
        t = torch.as_tensor(x, device=self.device)
        if t.dtype != torch.float32:
            t = t.to(torch.float32)
        t = t.reshape(-1, width)
        if t.stride(1) != 1:
            t = t.contiguous()
        return t

    def sample(self, beta: float = 0.4, batch_size: int | None = None, gather: bool = True):
        """replay_buffer.py:76-116: (idxs [B] int64, batch dict or None, weights [B] float32), device
        tensors.  The returned tensors are reused by the next sample()."""
        if self._added == 0:
            raise ValueError("Cannot sample from an empty buffer.")  # :83-84
        B = int(batch_size or self._batch_size)
        if B > self._batch_size:
            raise ValueError("batch_size above the buffer's batch_size")
        b = self.batch
        _lib.check(self.L.f110_replay_sample(
            self.handle, B, float(beta), _p(self.idx), _p(self.weights),
            *((_p(b["states"]), _p(b["actions"]), _p(b["rewards"]), _p(b["next_states"]), _p(b["dones"]))
              if gather else (None,) * 5), self._stream()), "f110_replay_sample")
        if B == self._batch_size:
            return self.idx, (b if gather else None), self.weights
        return self.idx[:B], ({k: v[:B] for k, v in b.items()} if gather else None), self.weights[:B]

    def update_priorities(self, idxs, priorities, td_errors: bool = False, add_eps: float = 0.0):
        """update_priorities(idxs, priorities) (replay_buffer.py:121-135).
        td_errors=True takes TD errors and stores agent.replay's
        |td| + add_eps (agent.py:337) without a separate kernel."""
        i = torch.as_tensor(idxs, device=self.device).reshape(-1).to(torch.int64).contiguous()
        t = torch.as_tensor(priorities, device=self.device).reshape(-1).to(torch.float32).contiguous()
        if i.shape != t.shape:
            raise ValueError("update_priorities: idxs and priorities differ in length")
        self._keep_u = (i, t)
        _lib.check(self.L.f110_replay_update_priorities(self.handle, _p(i), _p(t), i.shape[0], int(bool(td_errors)),
                                                        float(add_eps), self._stream()),
                   "f110_replay_update_priorities")

    # ------------------------------------------------------------------
    def arrays(self, names=("priority", "states", "actions", "rewards", "next_states", "dones")):
        """Device copies of the stored arrays: priority [cap], states / next_states [cap, D],
        actions [cap, A], rewards / dones [cap] (checkpoints, tests)."""
        ptrs = [ctypes.c_void_p() for _ in range(6)]
        _lib.check(self.L.f110_replay_arrays(self.handle, *[ctypes.byref(p) for p in ptrs]), "f110_replay_arrays")
        cap, D, A = self._buffer_size, self.obs_dim, self.act_dim
        shapes = {"priority": (cap,), "states": (cap, D), "actions": (cap, A), "rewards": (cap,),
                  "next_states": (cap, D), "dones": (cap,)}
        order = ["priority", "states", "actions", "rewards", "next_states", "dones"]
        out = {}
        for n in names:
            t = torch.empty(shapes[n], dtype=torch.float32, device=self.device)
            _d2d(t, ptrs[order.index(n)].value, self._stream())
            out[n] = t
        return out

    def priorities(self) -> torch.Tensor:
        return self.arrays(("priority",))["priority"]

    def close(self):
        if getattr(self, "handle", None):
            torch.cuda.synchronize(self.device)
            self.L.f110_replay_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_hip = None


def _d2d(dst: torch.Tensor, src_ptr: int, stream) -> None:
    """hipMemcpyAsync device-to-device from library-owned memory into a tensor."""
    global _hip
    if _hip is None:
        _lib.load()
        _hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime libf110 and torch already share (by SONAME)
        _hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_void_p]
        _hip.hipMemcpyAsync.restype = ctypes.c_int
    rc = _hip.hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src_ptr),
                             dst.numel() * dst.element_size(), 3, stream)  # hipMemcpyDeviceToDevice
    if rc != 0:
        raise _lib.F110Error(f"hipMemcpyAsync failed ({rc})")
