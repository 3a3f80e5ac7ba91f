"""Simulated-device backend: the engine's host side for real, the GPU as a
clock.

``SimEngine`` runs everything ``BackendEngine`` does on the host -- slots,
continuous batching, chunked prefill, decode gathers, completions at launch,
the ``max_inflight`` run-ahead queue -- but its "forward" computes nothing:
each launched step occupies a simulated device for ``step_ms(T) / speed``
of wall time, steps execute back to back in launch order, and the step's
completion event fires when its simulated end time has passed.  A fleet of
these on the CPU (one process per rank, the real control plane) reproduces
how a multi-GPU job behaves when its GPUs differ in speed -- the lock-step
question a one-GPU box cannot answer (bench.py ``--sim-gpu``).

The cost model is the 8B serving step on one MI355X: GEMM work is quantised
in 256-row M tiles, so ``step_ms(T) = base_ms + tile_ms * ceil(T / 256)``
(41.5 ms at T = 4041 with the defaults, `profiles/r3_bench_1gpu_20steps.json`).
"""
from __future__ import annotations

import time

import torch

from ..models.llama_stub import LlamaConfig
from .engine import BackendEngine

# tiny host-side model shape: only the engine's bookkeeping runs
SIM_MODEL = LlamaConfig(vocab=512, dim=64, layers=1, heads=2, kv_heads=1, ffn=128)


class _SimEvent:
    """End of one simulated step (monotonic ns, or a ``VirtualClock``'s)."""

    __slots__ = ("start_ns", "due_ns", "clock")

    def __init__(self, start_ns: int, due_ns: int, clock=None):
        self.start_ns, self.due_ns, self.clock = start_ns, due_ns, clock

    def query(self) -> bool:
        c = self.clock
        if c is None:
            return time.monotonic_ns() >= self.due_ns
        if c.now_ns() >= self.due_ns:
            return True
        c.poll()                                  # the host's poll interval passes
        return c.now_ns() >= self.due_ns

    def synchronize(self) -> None:
        if self.clock is not None:
            self.clock.advance_to(self.due_ns)
            return
        d = self.due_ns - time.monotonic_ns()
        if d > 0:
            time.sleep(d / 1e9)


class _SimStart:
    """``time_steps`` start marker: device time of the step it opens."""

    @staticmethod
    def elapsed_time(end: _SimEvent) -> float:
        return (end.due_ns - end.start_ns) / 1e6


class SimEngine(BackendEngine):
    def __init__(self, *, speed: float = 1.0, tile_ms: float = 2.5, base_ms: float = 1.5,
                 slots: int = 1536, max_ctx: int = 512, token_budget: int = 4096, max_inflight: int = 2,
                 page=None, gpu_index: int = 0, seed: int = 0, clock=None):
        """``clock``: a ``parallel.comm.VirtualClock`` (deterministic tests:
        the device runs in simulated time); None = wall time."""
        super().__init__(SIM_MODEL, slots=slots, max_ctx=max_ctx, token_budget=token_budget, device="cpu",
                         impl="ref", seed=seed, page=page, gpu_index=gpu_index, max_inflight=max_inflight)
        if speed <= 0:
            raise ValueError("speed must be > 0")
        self.speed = float(speed)
        self.tile_ms, self.base_ms = float(tile_ms), float(base_ms)
        self._dev_free_ns = 0
        self.clock = clock
        self.async_device = True                   # the simulated device runs steps asynchronously
        self.model.forward = self._forward          # the host never computes a forward

    def step_ms(self, T: int) -> float:
        return (self.base_ms + self.tile_ms * -(-int(T) // 256)) / self.speed

    @staticmethod
    def _forward(tok, pos, slot, samp, tiles=None, n_dec=0):
        return torch.zeros(int(samp.shape[0]), dtype=torch.int32)

    def warm_shapes(self, sizes=None) -> int:
        return 0

    def _start_event(self):
        return _SimStart() if self.time_steps else None

    def _now(self) -> int:
        return self.clock.now_ns() if self.clock is not None else time.monotonic_ns()

    def _end_event(self, T: int, timing: bool):
        now = self._now()
        start = max(now, self._dev_free_ns)
        self._dev_free_ns = start + int(self.step_ms(T) * 1e6)
        return _SimEvent(start, self._dev_free_ns, self.clock)

    def device_idle(self) -> bool:
        return self._now() >= self._dev_free_ns
