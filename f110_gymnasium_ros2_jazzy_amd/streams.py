"""Sub-shards of one GPU's env batch stepped on concurrent HIP streams.

Envs never interact across env ids, so a GPU's shard of E envs
can be stepped as S contiguous sub-shards, one `BatchSim` context each, on S
streams that are never joined between steps.  Sub-shard s then starts step
t+1 while another is still tracing step t: the latency-bound launches
(k_agents / k_post_single, one thread per car) and the ray kernel's tail
(the few grazing-beam waves) run beside another sub-shard's ray
pass instead of leaving CUs idle.  Results are those of one E-env context:
the RNG streams are keyed by global env id (`env_offset`), so every
sub-shard reproduces its slice of the single-context run bit for bit
(`tests/test_gpu_batch.py::test_stream_shards_match_single_context`).

Each stream is created with a full CU mask (`hipExtStreamCreateWithCUMask`),
which gives it a hardware queue of its own: streams handed out round-robin
from a shared pool can land on one queue, which serialises the sub-shards in
submission order and runs them in lock-step (measured 27-33 M env-steps/s
instead of 41; `scripts/stream_split.py`).

This is a throughput mode for callers whose actions are already resident
(random-action rollouts, the bench): a consumer that reads the obs of step t
before choosing the actions of step t+1 joins every step, which measured
slower than one context (`scripts/stream_split.py --join 1`).
"""
from __future__ import annotations

import collections
import ctypes

import torch

from . import _lib
from .sim import BatchSim

_hip = None


def _hip_lib():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
    return _hip


def dedicated_stream(device: torch.device) -> torch.cuda.ExternalStream:
    """A stream with a hardware queue of its own (full CU mask)."""
    hip = _hip_lib()
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    h = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    return torch.cuda.ExternalStream(h.value, device=device)


class StreamShards:
    """S BatchSim sub-shards of an E-env batch on S dedicated streams.

    `step(actions[E, A, 2])` launches every sub-shard on its own stream and
    returns without joining; `join()` makes the caller's current stream wait
    for all of them (do that before reading `obs`)."""

    def __init__(self, track, n_envs: int, n_streams: int = 2, env_offset: int = 0, heavy_first: bool = False,
                 ray_lanes: int | None = None, refill: int | None = None, **kw):
        if n_streams < 1 or n_envs % n_streams:
            raise ValueError(f"n_envs ({n_envs}) must split evenly into n_streams ({n_streams})")
        self.S = n_streams
        self.E = n_envs
        self.Es = n_envs // n_streams
        self.streams = []
        self.sims = []
        self._inflight = collections.deque()
        self._free_ev = []
        # one explicit device index for the CU-masked streams AND the contexts
        # ('cuda' alone would mean device 0 to BatchSim but the current device
        # to the stream constructor)
        dev = kw.pop("device", None)
        dev = torch.device(f"cuda:{dev}" if isinstance(dev, int) else (dev if dev is not None else "cuda"))
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.n_agents = int(kw.get("n_agents", 2))
        self.streams = [dedicated_stream(self.device) for _ in range(self.S)]
        # the ray kernel for the cars the GPU traces at once (f110_set_device_share applies
        # f110_create's size rules to the device's cars: 8192 envs as 4 x 2048 53.1 vs 47.6 M env-steps/s
        # with 1 vs 2 rays per lane, 32768 as 2 x 16384 69.2 vs 62.6 M with k_rays_fxs);
        # explicit ray_lanes / refill (A/B runs) go through the f110_debug_* knobs instead
        explicit = ray_lanes is not None or refill is not None or heavy_first
        cars = n_envs * self.n_agents
        for s in range(self.S):
            with torch.cuda.stream(self.streams[s]):
                sm = BatchSim(track, n_envs=self.Es, env_offset=env_offset + s * self.Es, device=self.device, **kw)
                if not explicit:
                    _lib.check(sm.L.f110_set_device_share(sm.ctx, cars, self.S), "f110_set_device_share")
                else:
                    lanes = ray_lanes if ray_lanes is not None else (2 if cars >= 12288 else 1)
                    rf = refill if refill is not None else (
                        1 if ((cars >= 32768 or (cars >= 16384 and n_streams >= 4)) and lanes == 2
                              and not heavy_first) else 0)
                    if not heavy_first and (n_streams > 1 or rf):
                        _lib.check(sm.L.f110_debug_disable_heavy_first(sm.ctx), "f110_debug_disable_heavy_first")
                    if sm.ray_kernel == 3:  # the fixed-point kernel (the others trace one ray per lane)
                        _lib.check(sm.L.f110_debug_set_ray_lanes(sm.ctx, int(lanes)), "f110_debug_set_ray_lanes")
                        _lib.check(sm.L.f110_debug_set_ray_refill(sm.ctx, int(rf)), "f110_debug_set_ray_refill")
                self.sims.append(sm)
        self.ray_lanes = self.sims[0].ray_lanes
        # what the contexts actually run (an unsupported map can override the request)
        self.refill = self.sims[0].ray_refill
        self._sl = [slice(s * self.Es, (s + 1) * self.Es) for s in range(self.S)]
        self._handles = [ctypes.c_void_p(st.cuda_stream) for st in self.streams]
        self._fork()

    def _caller(self):
        """The caller's current stream, or None when it is the legacy null
        stream.  The sub-streams are blocking streams (hipExtStreamCreate-
        WithCUMask takes no flags), so null-stream work is ordered against
        them implicitly in both directions: sub-stream kernels start after
        earlier null-stream work (actions drawn there), and later null-stream
        work (obs reads, a reuse of a freed action block) waits for them.
        Recording an event there would also wait for every sub-stream, i.e.
        serialise the sub-shards, so nothing is recorded on it."""
        cur = torch.cuda.current_stream(self.device)
        return None if cur.cuda_stream == 0 else cur

    def _event(self):
        return self._free_ev.pop() if self._free_ev else torch.cuda.Event()

    def _fork(self):
        # whatever the caller's stream produced so far (inputs) precedes every sub-shard's work
        cur = self._caller()
        if cur is None:
            return
        ev = self._event()
        ev.record(cur)
        for st in self.streams:
            st.wait_event(ev)
        self._free_ev.append(ev)  # re-recording later is safe: the waits are already enqueued

    def _hold(self, t):
        """Keep a caller tensor that the sub-streams read alive until their
        kernels are done with it, so the caching allocator cannot hand its
        block to the caller's (non-null) stream while a sub-stream still
        reads it.  One event per sub-stream marks the end of the reads; the
        reference is dropped once they have completed.  (Tensor.record_stream
        on these external streams crashed at hipStreamDestroy.)"""
        if self._caller() is None:
            return
        evs = []
        for st in self.streams:
            ev = self._event()
            ev.record(st)
            evs.append(ev)
        self._inflight.append((t, evs))
        while self._inflight and all(e.query() for e in self._inflight[0][1]):
            self._free_ev.extend(self._inflight.popleft()[1])

    def reset(self, poses):
        p = torch.as_tensor(poses, dtype=torch.float64, device=self.device)
        if p.dim() == 2:  # [A, 3] broadcast to every env (as BatchSim.reset)
            p = p.unsqueeze(0).expand(self.E, p.shape[0], 3)
        if p.shape[0] != self.E:
            raise ValueError(f"poses must be [{self.E}, A, 3] or [A, 3]; got {tuple(p.shape)}")
        self._fork()
        for s in range(self.S):
            with torch.cuda.stream(self.streams[s]):
                self.sims[s].reset(p[self._sl[s]])
        self._hold(p)

    def step(self, actions, minimal_outputs: bool = True):
        """Launch every sub-shard's step on its stream (not joined).  The
        sub-streams first wait for the caller's stream: actions produced there
        (a policy, torch.rand) and any reads of the previous obs queued there
        (`obs`, a torch.cat) are ordered before this step's kernels.

        Sub-shard s reads its rows of the contiguous action tensor by pointer
        offset, and f110_step is called with that sub-shard's stream handle
        directly (no per-sub-shard tensor views or stream switches: at 4096
        envs x 4 sub-shards the submission loop was 80 of the 111 us of a
        step)."""
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype not in (torch.float32, torch.float64):
            a = a.to(torch.float32)
        if tuple(a.shape) != (self.E, self.n_agents, 2):
            raise ValueError(f"actions must be [{self.E}, {self.n_agents}, 2]; got {tuple(a.shape)}")
        a = a.contiguous()
        self._fork()
        dt = _lib.F64 if a.dtype == torch.float64 else _lib.F32
        base, stride = a.data_ptr(), self.Es * self.n_agents * 2 * a.element_size()
        for s, sm in enumerate(self.sims):
            sm._keep_a = a
            outs = sm._outs_min if minimal_outputs else sm._outs
            rc = sm.L.f110_step(sm.ctx, ctypes.c_void_p(base + s * stride), dt, ctypes.byref(outs), self._handles[s])
            if rc < 0:
                _lib.check(rc, "f110_step")
        self._hold(a)

    def join(self):
        cur = self._caller()
        if cur is None:
            return  # the null stream waits for the sub-streams by itself
        for st in self.streams:
            ev = self._event()
            ev.record(st)
            cur.wait_event(ev)
            self._free_ev.append(ev)

    @property
    def obs(self) -> torch.Tensor:
        self.join()
        return torch.cat([sm.out.obs for sm in self.sims], 0)

    def read_counters(self):
        self.join()
        lk = rays = 0
        for sm in self.sims:
            a, b = sm.read_counters()
            lk += a
            rays += b
        return lk, rays

    def set_simt(self, on: bool = True):
        """Counting on / off for every sub-shard (f110_debug_set_simt: k_rays_fxs counts lookups, rays
        and lane slots only while it is on)."""
        for sm in self.sims:
            sm.set_simt(on)

    def reset_counters(self):
        self._fork()
        for s in range(self.S):
            with torch.cuda.stream(self.streams[s]):
                self.sims[s].reset_counters()

    def close(self):
        if not self.streams and not self.sims:
            return
        torch.cuda.synchronize(self.device)
        self._inflight.clear()
        for sm in self.sims:
            sm.close()
        # the contexts' output tensors were allocated under these streams:
        # release them (to the caching allocator) before the streams go away
        self.sims = []
        torch.cuda.synchronize(self.device)
        hip = _hip_lib()
        for st in self.streams:
            hip.hipStreamDestroy(ctypes.c_void_p(st.cuda_stream))
        self.streams = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
