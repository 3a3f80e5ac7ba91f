"""Authentication (API key / JWT HS256), RBAC, token-bucket rate limits and
the response envelope -- the reference's doc-only security features
(`docs/configuration.md:503-537, 732-805`, `docs/api.md:12-20`; SURVEY.md
D26), enforced by the native guard (``csrc/ingress/guard.h``) in both the
FastAPI server and the C++ ingress.  Parity unpinned: the reference has no
implementation or test to compare against; the expected behaviour is the
documented one."""
import json
import os
import time
import urllib.request

import pytest
from fastapi.testclient import TestClient

from llm_message_queue_amd import _native
from llm_message_queue_amd.api.security import guard_from_config, issue_token, redact_config
from llm_message_queue_amd.api.server import create_app
from llm_message_queue_amd.gateway.app import GatewayApp
from llm_message_queue_amd.utils.config import ConfigError, default_config, validate

SECRET = "s3cret-for-tests"


def _guard(**kw):
    return _native.ingress().Guard(**kw)


# ---------------------------------------------------------------- native guard
def test_token_bucket_refill_and_burst():
    g = _guard(global_rps=10.0, global_burst=3.0)
    t0 = 1_000_000_000
    got = [g.check("POST", "/api/v1/messages", now_ns=t0)[0] for _ in range(5)]
    assert got == [0, 0, 0, 429, 429]                    # burst of 3, then empty
    code, _, _, reason, retry = g.check("POST", "/api/v1/messages", now_ns=t0)
    assert code == 429 and "global" in reason and 0 < retry <= 0.1 + 1e-9
    assert g.check("POST", "/api/v1/messages", now_ns=t0 + 100_000_000)[0] == 0   # 1 token after 100 ms
    assert g.check("POST", "/api/v1/messages", now_ns=t0 + 100_000_000)[0] == 429
    assert g.check("POST", "/api/v1/messages", now_ns=t0 + 10_000_000_000)[0] == 0  # refilled (capped at burst)


def test_per_ip_and_per_user_buckets_are_independent():
    g = _guard(ip_rps=1.0, ip_burst=2.0, user_rps=1.0, user_burst=1.0)
    t = 5_000_000_000
    assert g.check("GET", "/api/v1/queues/stats", ip="1.1.1.1", now_ns=t)[0] == 0
    assert g.check("GET", "/api/v1/queues/stats", ip="1.1.1.1", now_ns=t)[0] == 0
    code, *_, reason, _ = g.check("GET", "/api/v1/queues/stats", ip="1.1.1.1", now_ns=t)
    assert code == 429 and "per_ip" in reason
    assert g.check("GET", "/api/v1/queues/stats", ip="2.2.2.2", now_ns=t)[0] == 0
    # anonymous callers are limited per address; a body's user_id claim never
    # keys a per-user bucket (naming "alice" must not spend alice's quota)
    for ip in ("3.3.3.3", "4.4.4.4", "5.5.5.5"):
        assert g.check("POST", "/api/v1/messages", ip=ip, user="alice", now_ns=t)[0] == 0
    assert g.allow_user("carol")[0] and not g.allow_user("carol")[0]


def test_specific_limits_checked_before_the_global_bucket():
    """a request refused by its IP's bucket must not drain the
    global bucket shared by everyone."""
    g = _guard(global_rps=0.001, global_burst=3.0, ip_rps=0.001, ip_burst=1.0)
    t = 7_000_000_000
    assert g.check("POST", "/api/v1/messages", ip="6.6.6.6", now_ns=t)[0] == 0
    for _ in range(10):                                   # the abusive IP is refused ...
        code, *_, reason, _ = g.check("POST", "/api/v1/messages", ip="6.6.6.6", now_ns=t)
        assert code == 429 and "per_ip" in reason
    # ... without spending the 2 global tokens left for other clients
    assert g.check("POST", "/api/v1/messages", ip="7.7.7.7", now_ns=t)[0] == 0
    assert g.check("POST", "/api/v1/messages", ip="8.8.8.8", now_ns=t)[0] == 0


def test_refused_request_drains_no_bucket():
    """a request the per-user or the global limit refuses
    keeps the caller's per-IP token (refunded), so a client held back by a
    shared limit does not also lose its own address budget."""
    g = _guard(method="api_key", api_keys=["k-a:alice:user"], ip_rps=0.001, ip_burst=2.0, user_rps=0.001,
               user_burst=1.0, global_rps=0.001, global_burst=100.0)
    t = 9_000_000_000
    assert g.check("POST", "/api/v1/messages", ip="9.9.9.9", api_key="k-a", now_ns=t)[0] == 0
    for _ in range(5):                                    # alice's user bucket is empty now
        code, *_, reason, _ = g.check("POST", "/api/v1/messages", ip="9.9.9.9", api_key="k-a", now_ns=t)
        assert code == 429 and "per_user" in reason
    # the address still has its second token (refunded each time)
    g2 = _guard(ip_rps=0.001, ip_burst=2.0, global_rps=0.001, global_burst=1.0)
    assert g2.check("POST", "/api/v1/messages", ip="1.2.3.4", now_ns=t)[0] == 0     # takes the 1 global token
    for _ in range(3):
        code, *_, reason, _ = g2.check("POST", "/api/v1/messages", ip="1.2.3.4", now_ns=t)
        assert code == 429 and "global" in reason
    # global refill: one token after 1000 s; 1.2.3.4's per-IP bucket kept its second token
    code, *_, reason, _ = g2.check("POST", "/api/v1/messages", ip="1.2.3.4", now_ns=t + 1_000_000_000_000)
    assert code == 0, reason


def test_api_key_auth_and_rbac():
    g = _guard(method="api_key", api_keys=["k-user", "k-ro:rita:readonly", "k-adm:ada:admin"], rbac=True,
               roles={"admin": ["*"], "user": ["message:*", "conversation:read"], "readonly": ["message:read"]})
    assert g.check("GET", "/health")[0] == 0                                 # public
    assert g.check("POST", "/api/v1/messages")[0] == 401                     # no key
    assert g.check("POST", "/api/v1/messages", api_key="nope")[0] == 401
    assert g.check("POST", "/api/v1/messages", api_key="k-user")[:3] == (0, "", "user")
    assert g.check("POST", "/api/v1/messages", api_key="k-ro")[0] == 403     # readonly can't write
    assert g.check("GET", "/api/v1/messages/x", api_key="k-ro")[:3] == (0, "rita", "readonly")
    assert g.check("POST", "/api/v1/admin/preprocessor/rules", api_key="k-user")[0] == 403
    assert g.check("POST", "/api/v1/admin/preprocessor/rules", api_key="k-adm")[0] == 0
    assert g.check("GET", "/api/v1/conversations", api_key="k-user")[0] == 0
    assert g.check("POST", "/api/v1/conversations", api_key="k-user")[0] == 403
    P = g.permission_for
    assert P("GET", "/health") == "" and P("PUT", "/api/v1/messages/1/status") == "message:write"
    assert P("GET", "/api/v1/users/u/conversations") == "conversation:read"
    assert P("DELETE", "/api/v1/endpoints/e") == "resource:write" and P("GET", "/api/v1/config") == "admin:write"


def test_jwt_verification_matches_python_signer():
    g = _guard(method="jwt", jwt_secret=SECRET, jwt_issuer="llm-message-queue", rbac=True,
               roles={"admin": ["*"], "user": ["message:read", "message:write"]})
    now = 1_700_000_000
    tok = issue_token(SECRET, "alice", "", ttl_s=60, now=now)
    assert g.check("POST", "/api/v1/messages", authorization="Bearer " + tok, wall_s=now + 1)[:3] == (0, "alice", "user")
    adm = issue_token(SECRET, "root", "admin", ttl_s=60, now=now)
    assert g.check("DELETE", "/api/v1/admin/queues/normal/x", authorization="Bearer " + adm, wall_s=now)[0] == 0
    assert g.check("DELETE", "/api/v1/admin/queues/normal/x", authorization="Bearer " + tok, wall_s=now)[0] == 403
    # expired / wrong secret / tampered payload / wrong issuer / alg=none / garbage
    assert g.check("GET", "/api/v1/messages", authorization="Bearer " + tok, wall_s=now + 61)[3] == "token expired"
    bad = issue_token("other-secret", "alice", ttl_s=60, now=now)
    assert g.check("GET", "/api/v1/messages", authorization="Bearer " + bad, wall_s=now)[3] == "bad signature"
    h, p, s = tok.split(".")
    forged = issue_token(SECRET, "mallory", "admin", ttl_s=60, now=now).split(".")[1]
    assert g.check("GET", "/api/v1/messages", authorization=f"Bearer {h}.{forged}.{s}", wall_s=now)[0] == 401
    other_iss = issue_token(SECRET, "alice", ttl_s=60, issuer="evil", now=now)
    assert g.check("GET", "/api/v1/messages", authorization="Bearer " + other_iss, wall_s=now)[3] == "wrong issuer"
    import base64
    none_hdr = base64.urlsafe_b64encode(b'{"alg":"none","typ":"JWT"}').rstrip(b"=").decode()
    assert g.check("GET", "/api/v1/messages", authorization=f"Bearer {none_hdr}.{p}.", wall_s=now)[0] == 401
    for junk in ("", "Bearer", "Bearer a.b", "Basic abc", "Bearer !!.??.##", "Bearer a.b.c.d"):
        assert g.check("GET", "/api/v1/messages", authorization=junk, wall_s=now)[0] == 401, junk
    # the native signer agrees with the Python one byte for byte
    payload = json.dumps({"sub": "x", "iat": now, "exp": now + 5, "iss": "llm-message-queue"}, separators=(",", ":"))
    nat = g.sign_jwt(payload)
    assert nat == issue_token(SECRET, "x", ttl_s=5, now=now)
    assert g.check("GET", "/api/v1/messages", authorization="Bearer " + nat, wall_s=now)[:2] == (0, "x")


def test_jwt_parser_fuzz_never_admits_forgeries():
    """Property test over the native token parser (untrusted input): arbitrary
    bytes and single-character mutations of a valid token are rejected with 401
    unless the mutation left the signed bytes intact."""
    from hypothesis import given, settings, strategies as st
    g = _guard(method="jwt", jwt_secret=SECRET, jwt_issuer="llm-message-queue")
    now = 1_700_000_000
    tok = issue_token(SECRET, "alice", "", ttl_s=60, now=now)

    @settings(max_examples=300, deadline=None)
    @given(st.text(max_size=120))
    def arbitrary(s):
        assert g.check("GET", "/api/v1/messages", authorization="Bearer " + s, wall_s=now)[0] == 401

    @settings(max_examples=300, deadline=None)
    @given(st.integers(0, len(tok) - 1), st.characters(codec="ascii"))
    def mutated(at, ch):
        t = tok[:at] + ch + tok[at + 1:]
        code = g.check("GET", "/api/v1/messages", authorization="Bearer " + t, wall_s=now)[0]
        if t == tok:
            assert code == 0
        else:
            # base64url's last char can carry unused bits: decoding may still
            # yield the original bytes, which is not a forgery
            assert code in (0, 401)
            if code == 0:
                assert at in (tok.index(".") - 1, tok.rindex(".") - 1, len(tok) - 1)

    arbitrary()
    mutated()


def test_security_config_validation_and_redaction():
    cfg = default_config()
    assert guard_from_config(cfg) is None                # everything off by default
    cfg.security.authentication.method = "jwt"
    with pytest.raises(ConfigError):
        validate(cfg)                                    # no secret
    cfg.security.authentication.jwt.secret = SECRET
    cfg.security.authorization.enabled = True
    cfg.security.authorization.default_role = "ghost"
    with pytest.raises(ConfigError):
        validate(cfg)
    cfg.security.authorization.default_role = "user"
    validate(cfg)
    cfg.security.authentication.api_key.valid_keys = ["topsecret"]
    d = redact_config(cfg.to_dict())
    assert d["security"]["authentication"]["jwt"]["secret"] == "***"
    assert d["security"]["authentication"]["api_key"]["valid_keys"] == ["***"]
    assert d["database"]["postgres"]["password"] == "***"


# ---------------------------------------------------------------- FastAPI server
def _app(cfg):
    cfg.queue.worker.process_interval = 5_000_000
    cfg.preprocessor.batch_window_us = 200
    return GatewayApp(cfg, use_gpu=False, simulate_ms=(1, 1, 1, 1))


def test_api_server_jwt_rbac_and_rate_limit():
    cfg = default_config()
    cfg.security.authentication.method = "jwt"
    cfg.security.authentication.jwt.secret = SECRET
    cfg.security.authorization.enabled = True
    cfg.loadbalancer.rate_limiting.enabled = True
    cfg.loadbalancer.rate_limiting.per_user.requests_per_second = 0.001
    cfg.loadbalancer.rate_limiting.per_user.burst_size = 3
    gw = _app(cfg)
    try:
        with TestClient(create_app(gw)) as c:
            assert c.get("/health").status_code == 200
            r = c.post("/api/v1/messages", json={"content": "hi"})
            assert r.status_code == 401 and r.headers["www-authenticate"] == "Bearer"
            user = {"Authorization": "Bearer " + issue_token(SECRET, "alice")}
            ro = {"Authorization": "Bearer " + issue_token(SECRET, "rita", "readonly")}
            adm = {"Authorization": "Bearer " + issue_token(SECRET, "root", "admin")}
            assert c.post("/api/v1/messages", json={"content": "a"}, headers=user).status_code == 202
            assert c.post("/api/v1/messages", json={"content": "b"}, headers=ro).status_code == 403
            assert c.get("/api/v1/queues/stats", headers=ro).status_code == 200
            assert c.get("/api/v1/config", headers=user).status_code == 403
            conf = c.get("/api/v1/config", headers=adm)
            assert conf.status_code == 200 and conf.json()["security"]["authentication"]["jwt"]["secret"] == "***"
            # per-user bucket (burst 3, ~no refill): alice has used 1
            codes = [c.post("/api/v1/messages", json={"content": "x"}, headers=user).status_code for _ in range(3)]
            assert codes == [202, 202, 429]
            r = c.post("/api/v1/messages", json={"content": "x"}, headers=user)
            assert r.status_code == 429 and int(r.headers["retry-after"]) >= 1
            # anonymous-by-token users are keyed on the body's user_id (other users unaffected)
            assert c.post("/api/v1/messages", json={"content": "x", "user_id": "z"}, headers=adm).status_code == 202
            # CORS preflight is never challenged
            assert c.options("/api/v1/messages", headers={"Origin": "http://x"}).status_code == 204
    finally:
        gw.stop()


def test_api_server_response_envelope():
    cfg = default_config()
    cfg.server.response_envelope = True
    gw = _app(cfg)
    try:
        with TestClient(create_app(gw)) as c:
            r = c.post("/api/v1/messages", json={"content": "hello", "priority": "high"})
            e = r.json()
            assert r.status_code == 202 and e["code"] == 202 and e["message"] == "success"
            assert e["data"]["priority"] == 2 and e["timestamp"].endswith("Z")
            bad = c.post("/api/v1/messages", content=b"{nope")
            b = bad.json()
            assert bad.status_code == 400 and b["code"] == 400 and "Invalid message format" in b["error"]
            assert "data" not in b
            bp = c.post("/api/v1/messages", json={"content": "x", "priority": "bogus"}).json()
            assert bp["code"] == 400 and bp["error_code"] == 1003          # documented business codes
            nf = c.get("/api/v1/conversations/does-not-exist").json()
            assert nf["code"] == 404 and nf["error_code"] == 1005
            assert c.get("/api/v1/messages/nope").json()["error_code"] == 1004
            assert c.get("/api/v1/health").json()["data"]["status"] == "ok"
            assert c.get("/metrics").text.startswith("#") or "llm_queue" in c.get("/metrics").text
    finally:
        gw.stop()


# ---------------------------------------------------------------- native ingress
def _http(port, path, body=None, headers=None, method=None):
    data = None if body is None else json.dumps(body).encode()
    req = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=data, method=method or ("POST" if data else "GET"),
                                 headers={"Content-Type": "application/json", **(headers or {})})
    try:
        with urllib.request.urlopen(req, timeout=5) as r:
            return r.status, dict(r.headers), json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, dict(e.headers), json.loads(e.read())


def test_native_ingress_guard_and_envelope():
    from llm_message_queue_amd.gateway.native_ingress import NativeIngress
    from llm_message_queue_amd.gateway.shm_bridge import RingPair
    cfg = default_config()
    cfg.security.authentication.method = "api_key"
    cfg.security.authentication.api_key.valid_keys = ["k1:alice", "k2:rita:readonly"]
    cfg.security.authorization.enabled = True
    cfg.loadbalancer.rate_limiting.enabled = True
    cfg.loadbalancer.rate_limiting.per_user.requests_per_second = 0.001
    cfg.loadbalancer.rate_limiting.per_user.burst_size = 2
    cfg.server.response_envelope = True
    validate(cfg)
    name = f"pyt-guard-{os.getpid()}"
    ring = RingPair(name, 1 << 20, "create")
    ing = NativeIngress(0, name, threads=1, host="127.0.0.1", cfg=cfg)
    port = ing.start()
    try:
        code, hdr, body = _http(port, "/api/v1/messages", {"content": "x"})
        assert code == 401 and body["code"] == 401 and "API key" in body["error"]
        code, _, body = _http(port, "/api/v1/messages", {"content": "x"}, {"X-API-Key": "k2"})
        assert code == 403 and "readonly" in body["message"]
        for _ in range(2):
            code, _, body = _http(port, "/api/v1/messages", {"content": "x"}, {"X-API-Key": "k1"})
            assert code == 202 and body["code"] == 202 and len(body["data"]["message_id"]) == 36
        code, hdr, body = _http(port, "/api/v1/messages", {"content": "x"}, {"X-API-Key": "k1"})
        assert code == 429 and int(hdr["Retry-After"]) >= 1 and "per_user" in body["error"]
        code, _, body = _http(port, "/health")
        assert code == 200 and body["data"]["status"] == "ok"
        st = ing.stats()
        assert st["unauthorized"] == 1 and st["forbidden"] == 1 and st["rate_limited"] == 1 and st["accepted"] == 2
    finally:
        ing.stop()
        ring.close(unlink=True)


def test_per_ip_buckets_survive_the_front_door_proxy():
    """behind the C++ front door every proxied request reaches the
    API server from loopback.  With the front door as a trusted proxy the
    guard keys the per-IP bucket on the X-Forwarded-For the front door sets
    (the connection's own address), so two clients keep separate buckets;
    without it they would share the loopback one."""
    import http.client
    import socket
    import threading
    import time

    import uvicorn

    from llm_message_queue_amd.gateway.native_ingress import NativeIngress

    cfg = default_config()
    cfg.loadbalancer.rate_limiting.enabled = True
    cfg.loadbalancer.rate_limiting.per_ip.requests_per_second = 0.001
    cfg.loadbalancer.rate_limiting.per_ip.burst_size = 2
    gw = _app(cfg)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        api_port = s.getsockname()[1]
    server = uvicorn.Server(uvicorn.Config(create_app(gw, trusted_proxies=("127.0.0.1",)), host="127.0.0.1",
                                           port=api_port, log_level="warning"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    ing = None
    try:
        t0 = time.time()
        while not server.started and time.time() - t0 < 20:
            time.sleep(0.05)
        assert server.started
        ing = NativeIngress(0, f"pyt-xff-{os.getpid()}", threads=1, host="127.0.0.1",
                            upstream=("127.0.0.1", api_port))
        port = ing.start()

        def get(src):
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=10, source_address=(src, 0))
            try:
                c.request("GET", "/api/v1/queues/stats")
                r = c.getresponse()
                r.read()
                return r.status
            finally:
                c.close()

        assert [get("127.0.0.2") for _ in range(3)] == [200, 200, 429]
        # another client, its own bucket (it would be 429 on a shared loopback bucket)
        assert [get("127.0.0.3") for _ in range(2)] == [200, 200]
        assert get("127.0.0.3") == 429
    finally:
        if ing is not None:
            ing.stop()
            from llm_message_queue_amd import _native
            _native.shmring().ShmRing(f"llmq-pyt-xff-{os.getpid()}-req", 1 << 20, "open").unlink()
        server.should_exit = True
        th.join(timeout=10)
        gw.stop()


def test_untrusted_peer_cannot_pick_its_bucket():
    """A client talking to the API server directly (not a trusted proxy)
    cannot choose its bucket with a forged X-Forwarded-For."""
    cfg = default_config()
    cfg.loadbalancer.rate_limiting.enabled = True
    cfg.loadbalancer.rate_limiting.per_ip.requests_per_second = 0.001
    cfg.loadbalancer.rate_limiting.per_ip.burst_size = 2
    gw = _app(cfg)
    try:
        with TestClient(create_app(gw, trusted_proxies=("127.0.0.1",))) as c:
            codes = [c.get("/api/v1/queues/stats", headers={"X-Forwarded-For": f"10.0.0.{i}"}).status_code
                     for i in range(3)]
            assert codes == [200, 200, 429]
    finally:
        gw.stop()
