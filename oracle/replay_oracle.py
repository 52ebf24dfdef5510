"""CPU restatement of the prioritized replay buffer — TEST INFRASTRUCTURE ONLY.

Only tests/ use this module, as the checker of libf110's f110_replay_*; the
product path never imports it.  It restates
rl_training/DDPG/replay_buffer.py:PrioritizedExperienceReplayBuffer (:6-135)
in NumPy with the reference's dtypes (float32 priorities, float64 sampling
probabilities, NumPy 2 promotion rules) for everything except the random
draw itself:
  add               :48-71   (priority = current max, clipped, float32)
  sampling_probs    :86-94
  weights(idxs)     :103-113 (IS weights of given indices)
  update_priorities :121-135
Pinned bit-exact on tests/golden/per.npz (the reference object's own
priority arrays, lengths, ring pointers, probabilities and weights).
"""
from __future__ import annotations

import numpy as np


class PEROracle:
    def __init__(self, buffer_size: int, batch_size: int, alpha: float = 0.6, priority_epsilon: float = 1e-6):
        self.size = int(buffer_size)
        self.batch = int(batch_size)
        self.alpha = float(alpha)
        self.eps = float(priority_epsilon)
        self.prio = np.zeros(self.size, np.float32)
        self.length = 0
        self.next_idx = 0

    def add(self, priority=None):
        """replay_buffer.py:48-71 (the experience itself is not modelled)."""
        if priority is None:
            if self.length > 0:
                p0 = float(np.max(self.prio[:self.length]))
                if not np.isfinite(p0) or p0 <= 0.0:
                    p0 = 1.0
            else:
                p0 = 1.0
        else:
            p0 = float(priority)
        self.prio[self.next_idx] = np.float32(np.clip(p0, 1e-8, np.finfo(np.float32).max))
        if self.length < self.size:
            self.length += 1
        self.next_idx = (self.next_idx + 1) % self.size

    def sampling_probs(self) -> np.ndarray:
        """replay_buffer.py:86-94: (p + eps) in float32, ^alpha in float64."""
        ps = self.prio[:self.length]
        pa = np.power(ps + np.float32(self.eps), self.alpha, dtype=np.float64)
        den = pa.sum()
        if den <= 0.0 or not np.isfinite(den):
            return np.full(self.length, 1.0 / self.length)
        return pa / den

    def weights(self, idxs, beta: float) -> np.ndarray:
        """replay_buffer.py:103-113 for the given indices."""
        p = self.sampling_probs()[np.asarray(idxs)]
        with np.errstate(divide="ignore", invalid="ignore"):
            w = np.power(self.length * p, -float(beta), dtype=np.float64)
        m = np.max(w)
        if not np.isfinite(m) or m <= 0.0:
            w = np.ones_like(w)
        else:
            w = w / m
        return w.astype(np.float32)

    def update_priorities(self, idxs, priorities):
        """replay_buffer.py:121-135."""
        pr = np.asarray(priorities, dtype=np.float32).reshape(-1)
        pr = np.clip(pr, 1e-8, np.finfo(np.float32).max)
        pr[~np.isfinite(pr)] = 1e-6
        self.prio[np.asarray(idxs)] = pr

    @staticmethod
    def td_priorities(td, priority_epsilon: float) -> np.ndarray:
        """agent.py:337: |td| (float32) + priority_epsilon -> float32 (NEP 50)."""
        return np.abs(np.asarray(td, np.float32)) + np.float32(priority_epsilon)
