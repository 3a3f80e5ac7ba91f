"""Native HTTP ingress (``csrc/ingress/http_ingress.cpp``) for the hot route
``POST /api/v1/messages``: C++ epoll threads accept, validate and ack
requests and push the raw bodies into the shared request ring that the GPU
dispatcher (``cli queue-manager``) drains and preprocesses in batches.
Other routes stay on the Python API server (``cli serve`` / ``api-gateway``).
"""
from __future__ import annotations

from typing import Optional, Tuple

from .. import _native


class NativeIngress:
    def __init__(self, port: int = 8080, ring: str = "default", threads: int = 4, host: str = "0.0.0.0",
                 cfg=None, conv_ring: str = "", upstream: Optional[Tuple[str, int]] = None,
                 gateway_compat: bool = False):
        """``cfg`` (optional): attach the config's guard (authentication, RBAC,
        rate limits -- ``api/security.py``) and response envelope.
        ``conv_ring``: ring (name of a ``RingPair``) for messages that carry a
        conversation_id -- drained by the process that owns conversation
        state.  ``upstream``: (host, port) of the Python API server; every
        other route is reverse-proxied to it (one public port).
        ``gateway_compat``: the submit reply also carries the reference
        api-gateway's ``message`` / ``id`` fields (``cli api-gateway``)."""
        self.ring = ring
        self._k = _native.ingress().HttpIngress(int(port), f"llmq-{ring}-req", int(threads), host)
        self.port = int(port)
        if conv_ring:
            self._k.set_conv_ring(f"llmq-{conv_ring}-req")
        if upstream is not None:
            self._k.set_upstream(str(upstream[0]), int(upstream[1]))
        if gateway_compat:
            self._k.set_gateway_compat(True)
        self.guard = None
        if cfg is not None:
            from ..api.security import guard_from_config
            self.guard = guard_from_config(cfg)
            if self.guard is not None:
                self._k.set_guard(self.guard)
            self._k.set_envelope(bool(cfg.server.response_envelope))
            self.set_idle_timeout(getattr(cfg.server, "idle_timeout", 60_000_000_000) / 1e9)

    def set_idle_timeout(self, seconds: float) -> None:
        """Close connections silent for longer than this (idle keep-alives and
        stalled / slowloris senders); 0 = never.  Default 60 s."""
        self._k.set_idle_timeout(float(seconds))

    def set_health(self, ok: bool, reason: str = "") -> None:
        """``GET /health`` on the door answers 503 (with ``reason``) while
        not ok -- the serve loop's stall watchdog drives it."""
        self._k.set_health(bool(ok), str(reason))

    def start(self) -> int:
        """Start listening; returns the bound port (useful with port 0)."""
        self.port = self._k.start()
        return self.port

    def stop(self) -> None:
        self._k.stop()

    def stats(self) -> dict:
        return dict(self._k.stats())
