"""Synthetic request traces: Poisson arrivals, 4-tier mix (10/30/40/20 --
the sample mix of the reference docs, `docs/api.md:573-593`, adopted as the
benchmark mix in BASELINE.md).

Tier is produced the way real traffic would produce it:
  * realtime (10 %): content carries a realtime keyword ("emergency", "asap",
    ...), scored by the GPU keyword kernel;
  * high (30 %): content carries a high keyword ("urgent", "critical", ...);
  * normal (40 %): neutral content;
  * low (20 %): neutral content with an explicit client priority of 4.
The neutral vocabulary is checked (tests) to contain none of the default
keyword patterns as a substring.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

from ..models.message import Message

NEUTRAL = (
    "hello please help me write a short summary of the report about the new model release "
    "can you explain this code snippet and tell me how it works in simple words "
    "translate the following paragraph into french thanks a lot for your answer "
    "what is the best way to learn linear algebra for machine learning "
    "draft an email to my team about the project schedule and the next milestone "
    "give me three ideas for dinner tonight with rice beans and vegetables "
    "review my resume and suggest edits to the experience section "
    "compare python and rust for building a web service with high throughput "
    "why does my test fail on the build server but pass on my laptop "
    "describe the history of the printing press in one paragraph"
).split()
REALTIME_KW = ("emergency", "asap", "immediate", "right now")
HIGH_KW = ("urgent", "important", "critical")
TIER_MIX = (0.10, 0.30, 0.40, 0.20)


class Workload:
    def __init__(self, seed: int = 0, min_words: int = 6, max_words: int = 24,
                 mix: Tuple[float, ...] = TIER_MIX, conversations: int = 0):
        self.rng = np.random.default_rng(seed)
        self.seed = seed
        self._serial = 0
        self.min_words, self.max_words = min_words, max_words
        self.mix = np.asarray(mix, dtype=np.float64) / sum(mix)
        self.conversations = conversations
        self._conv_ids = [f"conv-{seed}-{i}" for i in range(conversations)]

    def make(self, n: int) -> List[Message]:
        """n requests; all random draws are vectorised (host cost ~ a few
        microseconds per request, so trace generation never throttles the
        gateway it measures)."""
        if n <= 0:
            return []
        rng = self.rng
        tiers = rng.choice(4, size=n, p=self.mix)
        lens = rng.integers(self.min_words, self.max_words + 1, size=n)
        widx = rng.integers(0, len(NEUTRAL), size=int(lens.sum()))
        kpos = (rng.random(n) * lens).astype(np.int64)
        ksel = rng.integers(0, 1 << 30, size=n)
        capz = rng.random(n) < 0.3
        ques = rng.random(n) < 0.25
        users = rng.integers(0, 1000, size=n)
        convs = rng.integers(0, max(1, self.conversations), size=n)
        words_all = [NEUTRAL[i] for i in widx.tolist()]
        out = []
        off = 0
        base = self._serial
        self._serial += n
        for i in range(n):
            L = int(lens[i])
            words = words_all[off:off + L]
            off += L
            t = tiers[i]
            prio = 0
            if t == 0:
                words[kpos[i]] = REALTIME_KW[ksel[i] % len(REALTIME_KW)]
            elif t == 1:
                words[kpos[i]] = HIGH_KW[ksel[i] % len(HIGH_KW)]
            elif t == 3:
                prio = 4
            if capz[i]:
                words[0] = words[0].capitalize()
            content = " ".join(words) + ("?" if ques[i] else ".")
            conv = self._conv_ids[convs[i]] if self.conversations else ""
            out.append(Message(id=f"{self.seed}-{base + i}", conversation_id=conv,
                               user_id=f"user-{users[i]}", content=content, priority=prio))
        return out


class PoissonArrivals:
    """Arrival clock: ``due(now_s)`` returns how many requests arrived since
    the last call at rate ``rate`` (req/s)."""

    def __init__(self, rate: float, seed: int = 0):
        self.rate = float(rate)
        self.rng = np.random.default_rng(seed + 7919)
        self.t_next: Optional[float] = None

    def reset(self, t0: float, rate: Optional[float] = None) -> None:
        if rate is not None:
            self.rate = float(rate)
        self.t_next = t0 + self.rng.exponential(1.0 / self.rate) if self.rate > 0 else float("inf")

    def due(self, now: float, limit: Optional[int] = None) -> List[float]:
        """Arrival timestamps (s, monotonic) of every request due by ``now``
        (at most ``limit``; the rest stay due for the next call)."""
        if self.t_next is None:
            self.reset(now)
        out = []
        if self.rate <= 0:
            return out
        while self.t_next <= now and (limit is None or len(out) < limit):
            out.append(self.t_next)
            self.t_next += self.rng.exponential(1.0 / self.rate)
        return out
