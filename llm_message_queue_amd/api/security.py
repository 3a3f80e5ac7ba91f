"""Authentication, RBAC and rate limiting for both HTTP front ends.

The reference documents JWT / API-key authentication, RBAC roles and
token-bucket rate limits (`docs/configuration.md:503-537, 732-805`) but its
code has none of them.  Here they are one native object,
``_ingress.Guard`` (``csrc/ingress/guard.h``): the C++ epoll ingress checks
every ``POST /api/v1/messages`` inline, and the FastAPI server calls the same
object from a middleware, so both front ends enforce identical rules.

Everything is off by default (the reference's routes are open):
``security.authentication.method`` = none, ``security.authorization.enabled``
= false, ``loadbalancer.rate_limiting.enabled`` = false.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import time
from typing import Any, Dict, Optional

from .. import _native


def guard_from_config(cfg) -> Optional[Any]:
    """Build the native guard for ``cfg`` (None when nothing is enabled)."""
    sec = cfg.security
    auth, az = sec.authentication, sec.authorization
    rl = cfg.loadbalancer.rate_limiting
    rates = dict(global_rps=0.0, global_burst=0.0, ip_rps=0.0, ip_burst=0.0, user_rps=0.0, user_burst=0.0)
    if rl.enabled:
        rates = dict(global_rps=rl.global_.requests_per_second, global_burst=float(rl.global_.burst_size),
                     ip_rps=rl.per_ip.requests_per_second, ip_burst=float(rl.per_ip.burst_size),
                     user_rps=rl.per_user.requests_per_second, user_burst=float(rl.per_user.burst_size))
    if az.enabled and az.policy != "rbac":
        # the reference documents role-based access (docs/configuration.md:
        # 760-828 there); RBAC is the policy the native guard implements
        raise ValueError(f"security.authorization.policy {az.policy!r}: only 'rbac' is implemented")
    if auth.method == "none" and not az.enabled and not any(v > 0 for k, v in rates.items() if k.endswith("rps")):
        return None
    # /health and /metrics stay public and unthrottled (Guard.permission_for == "")
    g = _native.ingress().Guard(
        method=auth.method, api_key_header=auth.api_key.header_name, api_keys=list(auth.api_key.valid_keys),
        jwt_secret=auth.jwt.secret, jwt_issuer=auth.jwt.issuer, jwt_leeway_s=int(auth.jwt.leeway),
        rbac=bool(az.enabled), roles={k: list(v) for k, v in az.roles.items()}, default_role=az.default_role,
        idle_s=float(max(1, rl.per_ip.window_size)), **rates)
    return g


def _b64(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def issue_token(secret: str, subject: str, role: str = "", ttl_s: int = 24 * 3600,
                issuer: str = "llm-message-queue", now: Optional[int] = None) -> str:
    """HS256 JWT for ``subject`` (``cli token``; tests).  Pure-Python signer,
    verified by the native guard -- the two implementations check each other."""
    now = int(time.time()) if now is None else int(now)
    claims: Dict[str, Any] = {"sub": subject, "iat": now, "exp": now + int(ttl_s)}
    if issuer:
        claims["iss"] = issuer
    if role:
        claims["role"] = role
    head = _b64(json.dumps({"alg": "HS256", "typ": "JWT"}, separators=(",", ":")).encode())
    body = _b64(json.dumps(claims, separators=(",", ":")).encode())
    sig = hmac.new(secret.encode(), f"{head}.{body}".encode(), hashlib.sha256).digest()
    return f"{head}.{body}.{_b64(sig)}"


REDACTED = "***"


def redact_config(d: Dict[str, Any]) -> Dict[str, Any]:
    """Config dict for ``GET /api/v1/config`` with credentials masked."""
    def walk(x, key=""):
        if isinstance(x, dict):
            return {k: walk(v, k) for k, v in x.items()}
        if isinstance(x, list):
            return [REDACTED for _ in x] if key == "valid_keys" else [walk(v) for v in x]
        if key in ("password", "secret") and x:
            return REDACTED
        return x
    return walk(d)
