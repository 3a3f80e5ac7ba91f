"""gRPC front-end (api/grpc_server.py): unary + streaming submission, watch
until completion, stats/health, the guard on call metadata, and the
checked-in proto schema kept in sync with the runtime descriptors."""
import os
import time

import grpc
import pytest

from llm_message_queue_amd.api.grpc_server import GrpcClient, GrpcServer, pb, proto_source
from llm_message_queue_amd.api.security import issue_token
from llm_message_queue_amd.gateway.app import GatewayApp
from llm_message_queue_amd.utils.config import default_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SECRET = "grpc-test-secret"


def _stack(cfg=None):
    cfg = cfg or default_config()
    cfg.queue.worker.process_interval = 5_000_000
    cfg.preprocessor.batch_window_us = 200
    gw = GatewayApp(cfg, use_gpu=False, simulate_ms=(1, 1, 1, 1))
    srv = GrpcServer(gw, 0, "127.0.0.1", max_workers=8)
    port = srv.start()
    return gw, srv, port


def test_proto_file_matches_runtime_schema():
    with open(os.path.join(ROOT, "proto", "llmq.proto")) as f:
        assert f.read() == proto_source(), "regenerate proto/llmq.proto from grpc_server.proto_source()"
    # wire round trip of the map + repeated fields
    r = pb["SubmitRequest"](content="x", priority=2, metadata={"k": "v"})
    assert pb["SubmitRequest"].FromString(r.SerializeToString()).metadata["k"] == "v"


def test_grpc_submit_watch_stream_and_stats():
    gw, srv, port = _stack()
    cli = GrpcClient(f"127.0.0.1:{port}", gzip=True)
    try:
        assert cli.health().status == "ok"
        r = cli.submit("EMERGENCY: server down", user_id="u1", metadata={"team": "ops"})
        assert r.code == 202 and len(r.message_id) == 36 and r.priority == 1     # preprocessed -> realtime
        states = [m.status for m in cli.watch(r.message_id, timeout_ms=10_000)]
        assert states[-1] == "completed", states
        info = cli.get_message(r.message_id)
        assert info.user_id == "u1" and '"team":"ops"' in info.metadata_json
        r2 = cli.submit("routine", id="client-7", priority_name="low")
        assert r2.message_id == "client-7" and r2.priority == 4
        # bidirectional stream: replies in request order, bad items reported inline
        reqs = [pb["SubmitRequest"](content=f"m{i}", user_id=f"s{i}") for i in range(50)]
        reqs.insert(10, pb["SubmitRequest"](content="bad", priority_name="bogus"))
        replies = list(cli.submit_stream(reqs, timeout=30))
        assert len(replies) == 51
        assert replies[10].code == 400 and "priority" in replies[10].error
        ok = [x for x in replies if x.code == 202]
        assert len(ok) == 50 and len({x.message_id for x in ok}) == 50
        t0 = time.time()
        while time.time() - t0 < 10 and not all(
                (gw.messages.get(x.message_id) and gw.messages.get(x.message_id).status == "completed") for x in ok):
            time.sleep(0.02)
        assert all(gw.messages.get(x.message_id).status == "completed" for x in ok)
        batch = cli.submit_batch([pb["SubmitRequest"](content=f"b{i}", priority=1 + i % 4) for i in range(40)])
        assert [x.priority for x in batch] == [1 + i % 4 for i in range(40)] and all(x.code == 202 for x in batch)
        st = cli.queue_stats()
        assert [t.name for t in st.tiers] == ["realtime", "high", "normal", "low"]
        assert sum(t.completed for t in st.tiers) >= 52
        with pytest.raises(grpc.RpcError) as e:
            cli.get_message("nope")
        assert e.value.code() == grpc.StatusCode.NOT_FOUND
        with pytest.raises(grpc.RpcError) as e:
            cli.submit("x", priority=9)
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        prom = gw.metrics.render().decode()
        assert 'llm_grpc_requests_total{code="OK",method="Submit"}' in prom
        assert 'llm_grpc_requests_total{code="NOT_FOUND",method="GetMessage"}' in prom
        assert 'llm_grpc_requests_total{code="INVALID_ARGUMENT",method="Submit"}' in prom
    finally:
        cli.close()
        srv.stop()
        gw.stop()


def test_grpc_guard_on_metadata():
    cfg = default_config()
    cfg.security.authentication.method = "jwt"
    cfg.security.authentication.jwt.secret = SECRET
    cfg.security.authorization.enabled = True
    cfg.loadbalancer.rate_limiting.enabled = True
    cfg.loadbalancer.rate_limiting.per_user.requests_per_second = 0.001
    cfg.loadbalancer.rate_limiting.per_user.burst_size = 2
    gw, srv, port = _stack(cfg)
    target = f"127.0.0.1:{port}"
    anon = GrpcClient(target)
    user = GrpcClient(target, token=issue_token(SECRET, "alice"))
    ro = GrpcClient(target, token=issue_token(SECRET, "rita", "readonly"))
    try:
        assert anon.health().status == "ok"                      # public
        with pytest.raises(grpc.RpcError) as e:
            anon.submit("hi")
        assert e.value.code() == grpc.StatusCode.UNAUTHENTICATED
        with pytest.raises(grpc.RpcError) as e:
            ro.submit("hi")
        assert e.value.code() == grpc.StatusCode.PERMISSION_DENIED
        assert len(ro.queue_stats().tiers) == 4                  # queue:read is allowed
        assert user.submit("a").code == 202
        assert user.submit("b").code == 202
        with pytest.raises(grpc.RpcError) as e:
            user.submit("c")                                     # per-user burst 2 spent
        assert e.value.code() == grpc.StatusCode.RESOURCE_EXHAUSTED
        md = dict(e.value.trailing_metadata() or ())
        assert int(md["retry-after"]) >= 1
    finally:
        for c in (anon, user, ro):
            c.close()
        srv.stop()
        gw.stop()


def test_grpc_stream_cancel_releases_server_threads():
    """A client that abandons a SubmitStream mid-way must not pin server
    handler threads (the pool has 8 workers; 12 abandoned streams in a row
    would exhaust it if any leaked)."""
    import threading
    gw, srv, port = _stack()
    cli = GrpcClient(f"127.0.0.1:{port}")
    try:
        for k in range(12):
            gate = threading.Event()

            def reqs():
                for i in range(5):
                    yield pb["SubmitRequest"](content=f"c{k}-{i}")
                gate.wait(5)                      # keep the request side open

            call = cli.submit_stream(reqs())
            assert next(call).code == 202
            call.cancel()
            gate.set()
        assert cli.health(timeout=5).status == "ok"
        assert cli.submit("after", timeout=10).code == 202
    finally:
        cli.close()
        srv.stop()
        gw.stop()


def test_grpc_tls(tmp_path):
    import shutil
    import subprocess
    if shutil.which("openssl") is None:
        pytest.skip("openssl CLI not available")
    key, crt = tmp_path / "k.pem", tmp_path / "c.pem"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out", str(crt),
                    "-days", "1", "-subj", "/CN=localhost", "-addext", "subjectAltName=DNS:localhost"],
                   check=True, capture_output=True)
    cfg = default_config()
    cfg.queue.worker.process_interval = 5_000_000
    gw = GatewayApp(cfg, use_gpu=False, simulate_ms=(1, 1, 1, 1))
    srv = GrpcServer(gw, 0, "127.0.0.1", max_workers=4, tls_cert=str(crt), tls_key=str(key))
    port = srv.start()
    sec = GrpcClient(f"localhost:{port}", root_cert=str(crt))
    plain = GrpcClient(f"127.0.0.1:{port}")
    try:
        assert sec.submit("over tls").code == 202
        with pytest.raises(grpc.RpcError) as e:
            plain.health(timeout=3)                       # plaintext client cannot talk to a TLS port
        assert e.value.code() in (grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED)
    finally:
        sec.close()
        plain.close()
        srv.stop()
        gw.stop()
    with pytest.raises(ValueError):
        GrpcServer(gw, 0, tls_cert=str(crt))


def test_grpc_batch_items_charge_rate_limits_individually():
    """A batch cannot bypass the global bucket: each item takes a token."""
    cfg = default_config()
    cfg.security.authentication.method = "jwt"
    cfg.security.authentication.jwt.secret = SECRET
    cfg.loadbalancer.rate_limiting.enabled = True
    cfg.loadbalancer.rate_limiting.global_.requests_per_second = 0.001
    cfg.loadbalancer.rate_limiting.global_.burst_size = 5
    gw, srv, port = _stack(cfg)
    good = GrpcClient(f"127.0.0.1:{port}", token=issue_token(SECRET, "bob"))
    bad = GrpcClient(f"127.0.0.1:{port}", token="not-a-token")
    try:
        out = good.submit_batch([pb["SubmitRequest"](content=f"x{i}") for i in range(10)])
        assert [x.code for x in out].count(202) == 5 and [x.code for x in out].count(429) == 5
        with pytest.raises(grpc.RpcError) as e:
            bad.submit_batch([pb["SubmitRequest"](content="y")])
        assert e.value.code() == grpc.StatusCode.UNAUTHENTICATED
    finally:
        good.close()
        bad.close()
        srv.stop()
        gw.stop()
