"""Python client SDK (``llm_message_queue_amd.client``) against the REST API
(FastAPI TestClient as the transport): every route family, the envelope
format, API-key auth and error mapping."""
import pytest
from fastapi.testclient import TestClient

from llm_message_queue_amd.api.server import create_app
from llm_message_queue_amd.client import APIError, LLMQueueClient
from llm_message_queue_amd.gateway.app import GatewayApp
from llm_message_queue_amd.utils.config import default_config


def _cfg(**kw):
    cfg = default_config()
    cfg.queue.worker.process_interval = 5_000_000
    cfg.preprocessor.batch_window_us = 200
    for k, v in kw.items():
        obj, attr = k.rsplit("__", 1) if "__" in k else ("", k)
        tgt = cfg
        for part in obj.split("__") if obj else []:
            tgt = getattr(tgt, part)
        setattr(tgt, attr, v)
    return cfg


@pytest.fixture(params=[False, True], ids=["plain", "envelope"])
def client(request):
    cfg = _cfg(server__response_envelope=request.param)
    gw = GatewayApp(cfg, use_gpu=False, simulate_ms=(1, 1, 1, 1))
    with TestClient(create_app(gw)) as tc:
        yield LLMQueueClient("http://testserver/api/v1", session=tc)
    gw.stop()


def test_messages_and_conversations(client):
    assert client.health_check()["status"] == "ok"
    r = client.send_message("", "u1", "EMERGENCY: the database is down", priority=None)
    assert r["priority"] == 1
    m = client.wait_for_status(r["message_id"], "completed", timeout=10)
    assert m["metadata"]["analyzed"]
    assert client.list_messages(user_id="u1")["total"] >= 1
    conv = client.create_conversation("u2", {"topic": "sdk"})
    cid = conv["conversation_id"]
    client.add_conversation_message(cid, "u2", "hello there", priority="high")
    got = client.get_conversation(cid)
    assert got["id"] == cid and got["message_count"] == 1
    client.update_conversation_state(cid, "completed")
    assert any(c["id"] == cid for c in client.user_conversations("u2"))
    with pytest.raises(APIError) as e:
        client.get_conversation("missing")
    assert e.value.status == 404


def test_queues_resources_endpoints_admin(client):
    assert "standard" in client.get_queue_stats() or client.get_queue_stats()
    assert client.get_queue_status()
    client.register_endpoint({"id": "ep-x", "url": "http://x", "type": "llm"})
    assert any(ep["id"] == "ep-x" for ep in client.list_endpoints())
    client.set_endpoint_status("ep-x", "degraded")
    client.remove_endpoint("ep-x")
    client.register_resource({"id": "r1", "name": "gpu-x", "type": "llm", "capacity": {"gpu": 1}})
    assert any(r["id"] == "r1" for r in client.list_resources())
    assert client.resource_stats()
    client.add_priority_rule(2, "(?i)sdk-urgent")
    assert any(r["pattern"] == "(?i)sdk-urgent" for r in client.list_priority_rules())
    client.remove_priority_rule(2, "(?i)sdk-urgent")
    client.set_user_priority("vip", "realtime")
    assert isinstance(client.dead_letters(), list)
    assert client.requeue_all_dead_letters()["count"] == 0
    assert client.get_config()["database"]["postgres"]["password"] == "***"


def test_errors_carry_status_and_business_code():
    cfg = _cfg(server__response_envelope=True)
    cfg.security.authentication.method = "api_key"
    cfg.security.authentication.api_key.valid_keys = ["k1:alice"]
    gw = GatewayApp(cfg, use_gpu=False, simulate_ms=(1, 1, 1, 1))
    try:
        with TestClient(create_app(gw)) as tc:
            anon = LLMQueueClient("http://testserver", session=tc)
            assert anon.health_check()["status"] == "ok"             # public
            with pytest.raises(APIError) as e:
                anon.send_message("", "u", "hi")
            assert e.value.status == 401
            c = LLMQueueClient("http://testserver", session=tc, api_key="k1")
            assert c.send_message("", "u", "hi")["message_id"]
            with pytest.raises(APIError) as e2:
                c.send_message("", "u", "hi", priority="bogus")
            assert e2.value.status == 400 and e2.value.error_code == 1003
            with pytest.raises(APIError) as e3:
                c.get_message("nope")
            assert e3.value.status == 404 and e3.value.error_code == 1004
    finally:
        gw.stop()
