"""REST contract tests (reference api/handlers.go routes) on the CPU
monolith (GatewayApp without a GPU: workers + simulated LLM)."""
import time

import pytest
from fastapi.testclient import TestClient

from llm_message_queue_amd.api.server import create_app
from llm_message_queue_amd.gateway.app import GatewayApp
from llm_message_queue_amd.utils.config import default_config


@pytest.fixture(scope="module")
def client():
    cfg = default_config()
    cfg.queue.worker.process_interval = 5_000_000
    cfg.queue.retry.initial_backoff = 10_000_000
    cfg.queue.retry.max_retries = 1
    cfg.conversation.max_context_length = 3
    cfg.preprocessor.batch_window_us = 200
    app = GatewayApp(cfg, use_gpu=False, simulate_ms=(1, 1, 1, 1))
    with TestClient(create_app(app, ["http://ok.example"])) as c:
        c.gw = app
        yield c
    app.stop()


def wait(pred, t=3.0):
    t0 = time.time()
    while time.time() - t0 < t:
        if pred():
            return True
        time.sleep(0.01)
    return False


def test_health_and_metrics(client):
    r = client.get("/health")
    assert r.status_code == 200 and r.json()["status"] == "ok" and r.json()["version"] == "1.0.0"
    client.post("/api/v1/messages", json={"content": "hello metrics"})
    m = client.get("/metrics")
    assert m.status_code == 200 and b"llm_queue_operations_total" in m.content


def test_submit_string_priority_and_get(client):
    r = client.post("/api/v1/messages", json={"content": "please summarise", "priority": "high", "user_id": "u"})
    assert r.status_code == 202, r.text
    body = r.json()
    assert body["priority"] == 2 and isinstance(body["estimated_wait"], int)
    mid = body["message_id"]
    g = client.get(f"/api/v1/messages/{mid}")
    assert g.status_code == 200 and g.json()["id"] == mid
    assert wait(lambda: client.get(f"/api/v1/messages/{mid}").json()["status"] == "completed")
    lst = client.get("/api/v1/messages", params={"user_id": "u"}).json()
    assert lst["total"] >= 1 and any(m["id"] == mid for m in lst["messages"])


def test_keyword_priority_and_analysis(client):
    r = client.post("/api/v1/messages", json={"content": "EMERGENCY the server is down"})
    assert r.status_code == 202 and r.json()["priority"] == 1
    mid = r.json()["message_id"]
    md = client.get(f"/api/v1/messages/{mid}").json()["metadata"]
    assert md["priority_reason"] == "content_keywords" and "analysis" in md and md["analyzed"] is True


def test_bad_bodies(client):
    assert client.post("/api/v1/messages", content=b"{not json").status_code == 400
    assert client.post("/api/v1/messages", json={"content": "x", "priority": "soonish"}).status_code == 400
    assert client.post("/api/v1/conversations", json={}).status_code == 400
    assert client.get("/api/v1/messages/nope").status_code == 404
    # 4 MiB body cap (same as the native ingress): declared or chunked
    big = b'{"content":"' + b"x" * (4 << 20) + b'"}'
    assert client.post("/api/v1/messages", content=big).status_code == 413
    assert client.post("/api/v1/messages", content=iter([big[:1 << 20], big[1 << 20:]])).status_code == 413
    assert client.post("/api/v1/messages", content=iter([b'{"content":', b'"chunked ok"}'])).status_code == 202


def test_chunked_body_cap_reads_incrementally():
    """a huge chunked stream is cut off at the 4 MiB cap, not
    buffered whole before the check (raw ASGI receive, no client in between)."""
    import asyncio
    from llm_message_queue_amd.api.server import ChunkedBodyCap
    pulled, sent, reached = [0], [], []

    async def receive():
        pulled[0] += 1
        return {"type": "http.request", "body": b"x" * (1 << 20), "more_body": pulled[0] < 1000}   # 1 GB

    async def send(msg):
        sent.append(msg)

    async def app(scope, rcv, snd):
        reached.append(True)

    scope = {"type": "http", "method": "POST", "path": "/api/v1/messages",
             "headers": [(b"transfer-encoding", b"chunked")]}
    asyncio.run(ChunkedBodyCap(app)(scope, receive, send))
    assert pulled[0] == 5 and not reached                       # 5 MiB read, then 413
    assert sent[0]["status"] == 413


def test_conversation_flow(client):
    r = client.post("/api/v1/conversations", json={"user_id": "alice", "metadata": {"topic": "t"}})
    assert r.status_code == 201
    cid = r.json()["conversation_id"]
    assert r.json()["state"] == "active"
    for i in range(5):
        a = client.post(f"/api/v1/conversations/{cid}/messages", json={"content": f"turn {i} good", "user_id": "alice"})
        assert a.status_code == 202 and a.json()["conversation_id"] == cid
    c = client.get(f"/api/v1/conversations/{cid}").json()
    assert c["user_id"] == "alice" and len(c["messages"]) == 3 and c["message_count"] == 5
    assert client.put(f"/api/v1/conversations/{cid}/state", json={"state": "completed"}).json() == {"status": "updated"}
    assert client.put("/api/v1/conversations/missing/state", json={"state": "x"}).status_code == 500
    assert client.put(f"/api/v1/conversations/{cid}/state", json={}).status_code == 400
    convs = client.get("/api/v1/users/alice/conversations").json()["conversations"]
    assert [x["id"] for x in convs] == [cid]
    assert client.get("/api/v1/conversations/unknown").status_code == 404        # D19
    assert client.post("/api/v1/conversations/unknown/messages", json={"content": "x"}).status_code == 500
    assert client.get("/api/v1/conversations", params={"user_id": "alice"}).json()["total"] == 1
    up = client.put(f"/api/v1/conversations/{cid}", json={"title": "T", "metadata": {"k": 1}}).json()
    assert up["title"] == "T" and up["metadata"]["k"] == 1


def test_message_into_conversation_via_submit(client):
    r = client.post("/api/v1/messages", json={"content": "hi", "conversation_id": "conv-x", "user_id": "bob"})
    assert r.status_code == 202
    assert client.get("/api/v1/conversations/conv-x").json()["user_id"] == "bob"


def test_queue_stats_and_status(client):
    s = client.get("/api/v1/queues/stats").json()
    assert set(s) >= {"standard", "delayed", "dead_letter", "priority", "workers"}
    assert set(s["standard"]) == {"realtime", "high", "normal", "low"}
    st = client.get("/api/v1/queues/status").json()
    assert [q["name"] for q in st["queues"]] == ["realtime", "high", "normal", "low"]


def test_resources_and_endpoints(client):
    r = client.post("/api/v1/resources", json={"id": "gpu7", "type": "llama3-8b", "capacity": {"gpu": 8}})
    assert r.status_code == 201 and r.json()["resource_id"] == "gpu7"
    assert client.post("/api/v1/resources", json={"id": "gpu7", "type": "x"}).status_code == 500
    assert client.post("/api/v1/resources", json={"type": "x"}).status_code == 400
    assert any(x["id"] == "gpu7" for x in client.get("/api/v1/resources").json()["resources"])
    assert client.get("/api/v1/resources/stats").json()["resources"]["total"] >= 1
    e = client.post("/api/v1/endpoints", json={"id": "ep9", "url": "http://x:1", "type": "llm", "weight": 3,
                                               "response_time": "150ms"})
    assert e.status_code == 201
    eps = client.get("/api/v1/endpoints").json()["endpoints"]
    ep9 = [x for x in eps if x["id"] == "ep9"][0]
    assert ep9["response_time"] == 150_000_000 and ep9["status"] == "healthy"
    assert client.get("/api/v1/endpoints/stats").json()["endpoints"]["total"] >= 2
    assert client.put("/api/v1/endpoints/ep9/status", json={"status": "unhealthy"}).status_code == 200
    assert client.delete("/api/v1/endpoints/ep9").status_code == 200
    assert client.delete("/api/v1/endpoints/ep9").status_code == 404


def test_admin_rules_user_priority_and_dlq(client):
    assert client.post("/api/v1/admin/preprocessor/rules",
                       json={"pattern": "(?i)deadline", "priority": "high"}).status_code == 201
    rules = client.get("/api/v1/admin/preprocessor/rules").json()["rules"]
    assert {"priority": 2, "priority_name": "high", "pattern": "(?i)deadline"} in rules
    assert client.post("/api/v1/messages", json={"content": "the deadline"}).json()["priority"] == 2
    assert client.request("DELETE", "/api/v1/admin/preprocessor/rules",
                          json={"pattern": "(?i)deadline", "priority": 2}).status_code == 200
    assert client.post("/api/v1/admin/preprocessor/user-priorities",
                       json={"user_id": "vip", "priority": "realtime"}).status_code == 200   # D18
    assert client.post("/api/v1/messages", json={"content": "hello", "user_id": "vip"}).json()["priority"] == 1
    # a failing message retries then lands in the DLQ; requeue it by id
    r = client.post("/api/v1/messages", json={"content": "boom", "metadata": {"simulate_error": "x"}})
    mid = r.json()["message_id"]
    dlq = client.gw.factory.dead_letter_queue
    assert wait(lambda: dlq.index_of(mid) >= 0)
    assert any(it["message"]["id"] == mid for it in client.get("/api/v1/admin/dead-letter").json()["items"])
    assert client.post(f"/api/v1/admin/dead-letter/requeue/{mid}").status_code == 200
    assert client.post("/api/v1/admin/dead-letter/requeue/nope").status_code == 404
    assert client.post("/api/v1/admin/dead-letter/requeue-all").json()["status"] == "requeued"
    assert client.delete("/api/v1/admin/queues/bogus/x").status_code == 400
    assert client.delete("/api/v1/admin/queues/standard/nope").status_code == 404


def test_cors(client):
    r = client.options("/api/v1/messages", headers={"Origin": "http://ok.example"})
    assert r.status_code == 204 and r.headers["access-control-allow-origin"] == "http://ok.example"
    r = client.get("/health", headers={"Origin": "http://evil.example"})
    assert "access-control-allow-origin" not in r.headers


def test_config_endpoint_redacts(client):
    d = client.get("/api/v1/config").json()
    assert d["database"]["postgres"]["password"] == "***" and d["queue"]["levels"][0]["name"] == "realtime"


def test_json_metrics_summary(client):
    for i in range(3):
        assert client.post("/api/v1/messages", json={"content": f"metrics json {i}"}).status_code == 202
    r = client.get("/api/v1/metrics")
    assert r.status_code == 200
    d = r.json()
    assert d["requests_total"] >= 3 and "requests_per_second" in d and 0.0 <= d["error_rate"] <= 1.0
    assert set(d["queue_lengths"]) == {"realtime", "high", "normal", "low"}
    assert "dispatch" in d["latency"] and "end_to_end" in d["latency"]


def test_merge_expositions_adds_rank_and_groups_families():
    """The multi-GPU front door's /metrics (gateway/app.py:metrics_exposition):
    every sample gets a ``rank`` label, each family is one block under one
    HELP/TYPE header, and the result parses as Prometheus text."""
    from prometheus_client.parser import text_string_to_metric_families
    from llm_message_queue_amd.utils.metrics import _with_rank, merge_expositions
    assert _with_rank("up 1", 3) == 'up{rank="3"} 1'
    assert _with_rank("up{} 1", 3) == 'up{rank="3"} 1'
    assert _with_rank('x_total{a="b"} 2.0', 0) == 'x_total{rank="0",a="b"} 2.0'
    a = "# HELP x_total X\n# TYPE x_total counter\nx_total{q=\"hi\"} 1.0\n# HELP g G\n# TYPE g gauge\ng 4\n"
    b = "# HELP x_total X\n# TYPE x_total counter\nx_total{q=\"hi\"} 2.0\n# HELP g G\n# TYPE g gauge\ng 5\n"
    txt = merge_expositions({1: b, 0: a}).decode()
    assert txt.count("# TYPE x_total counter") == 1 and txt.count("# TYPE g gauge") == 1
    fams = {f.name: f for f in text_string_to_metric_families(txt)}
    assert sorted((s.labels["rank"], s.value) for s in fams["x"].samples) == [("0", 1.0), ("1", 2.0)]
    assert sorted((s.labels["rank"], s.value) for s in fams["g"].samples) == [("0", 4.0), ("1", 5.0)]
    lines = txt.splitlines()
    assert lines.index("# TYPE g gauge") > max(i for i, l in enumerate(lines) if l.startswith("x_total"))
    assert merge_expositions({}) == b""
