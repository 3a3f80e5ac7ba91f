"""Parity ports of reference tests/loadbalancer_test.go + GPU-aware and fixed-
defect coverage."""
import time

import pytest

from llm_message_queue_amd.backend.slot_page import SlotPage
from llm_message_queue_amd.balancer.load_balancer import (Endpoint, EndpointStatus, LoadBalancer,
                                                          LoadBalancerError)
from llm_message_queue_amd.models.message import Message
from llm_message_queue_amd.utils.config import LoadBalancerConfig

MS = 1_000_000


def lb_with(algorithm, eps, interval=0, **kw):
    kw.setdefault("max_failures", 3)
    lb = LoadBalancer(LoadBalancerConfig(algorithm=algorithm, health_check_interval=interval, **kw), seed=1)
    for e in eps:
        lb.add_endpoint(e)
    return lb


def three(**kw):
    return [Endpoint(id=f"ep{i}", url=f"http://endpoint{i}:8080", name=f"endpoint{i}", type="llm", weight=1,
                     status=EndpointStatus.HEALTHY, max_connections=100, **kw) for i in (1, 2, 3)]


def test_round_robin():
    lb = lb_with("round_robin", three())
    counts = {}
    for _ in range(9):
        ep = lb.get_endpoint(None, "")
        counts[ep.url] = counts.get(ep.url, 0) + 1
    assert counts == {f"http://endpoint{i}:8080": 3 for i in (1, 2, 3)}
    lb.stop()


def test_least_connections():
    eps = three()
    eps[0].connections, eps[1].connections, eps[2].connections = 2, 0, 1
    lb = lb_with("least_connections", eps)
    assert lb.get_endpoint(None, "").id == "ep2"
    assert lb.get_endpoint_stats() is not None


def test_weighted_random():
    eps = three()
    for e, w in zip(eps, (1, 5, 10)):
        e.weight = w
    lb = lb_with("weighted_random", eps)
    counts = {e.id: 0 for e in eps}
    for _ in range(1000):
        ep = lb.get_endpoint(None, "")
        counts[ep.id] += 1
        lb.release_endpoint(ep.id)
    assert counts["ep3"] > counts["ep1"] and counts["ep3"] > counts["ep2"] and counts["ep2"] > counts["ep1"]


def test_adaptive_load():
    eps = three()
    for e, (rt, er) in zip(eps, ((150, 0.1), (50, 0.02), (100, 0.05))):
        e.response_time, e.error_rate = rt * MS, er
    lb = lb_with("adaptive_load", eps, interval=30_000 * MS)
    counts = {}
    for _ in range(20):
        ep = lb.get_endpoint(None, "")
        counts[ep.url] = counts.get(ep.url, 0) + 1
        lb.release_endpoint(ep.id, 50 * MS, False)
    c2 = counts.get("http://endpoint2:8080", 0)
    assert c2 >= counts.get("http://endpoint1:8080", 0) and c2 >= counts.get("http://endpoint3:8080", 0)
    lb.stop()


def test_health_management():
    eps = three()
    eps[1].status = EndpointStatus.UNHEALTHY
    lb = lb_with("round_robin", eps)
    for _ in range(6):
        assert lb.get_endpoint(None, "").url != "http://endpoint2:8080"
    lb.update_endpoint_status("ep2", EndpointStatus.HEALTHY)
    assert any(lb.get_endpoint(None, "").url == "http://endpoint2:8080" for _ in range(9))


def test_add_remove_endpoints():
    lb = lb_with("round_robin", three()[:2])
    assert len(lb.get_all_endpoints()) == 2
    lb.remove_endpoint("ep1")
    assert [e.id for e in lb.get_all_endpoints()] == ["ep2"]
    lb.add_endpoint(Endpoint(id="ep3"))
    lb.add_endpoint(Endpoint(id="ep4"))
    assert len(lb.get_all_endpoints()) == 3
    with pytest.raises(LoadBalancerError):
        lb.add_endpoint(Endpoint(id="ep3"))
    with pytest.raises(LoadBalancerError):
        lb.remove_endpoint("nope")


def test_session_affinity():
    lb = lb_with("round_robin", three())
    first = lb.get_endpoint(None, "session-1")
    for _ in range(5):
        assert lb.get_endpoint(None, "session-1").id == first.id
    assert lb.get_session_count() == 1
    lb.clear_sessions()
    assert lb.get_session_count() == 0


def test_errors_do_not_deadlock():
    """D7: the reference leaks its mutex on these two error paths."""
    lb = lb_with("round_robin", [])
    for _ in range(3):
        with pytest.raises(LoadBalancerError):
            lb.get_endpoint(Message(metadata={"model_type": "nope"}), "")
    eps = three()
    for e in eps:
        e.status = EndpointStatus.UNHEALTHY
        lb.add_endpoint(e)
    for _ in range(3):
        with pytest.raises(LoadBalancerError):
            lb.get_endpoint(None, "")
    lb.update_endpoint_status("ep1", EndpointStatus.HEALTHY)
    assert lb.get_endpoint(None, "").id == "ep1"


def test_model_type_groups():
    a = Endpoint(id="a", type="llm")
    b = Endpoint(id="b", type="embed")
    lb = lb_with("round_robin", [a, b])
    assert lb.get_endpoint(Message(metadata={"model_type": "embed"}), "").id == "b"
    assert lb.get_endpoint(Message(), "").id == "a"
    assert lb.get_endpoint_stats()["endpoints_by_type"] == {"llm": 1, "embed": 1}


def test_session_timeout_and_config():
    lb = lb_with("round_robin", three(), session_timeout=30 * MS)
    e = lb.get_endpoint(None, "s")
    time.sleep(0.08)
    assert lb.get_session_count() == 0      # cleanup loop expired it
    lb.stop()
    lb2 = lb_with("round_robin", three(), enable_session_affinity=False)
    lb2.get_endpoint(None, "s")
    assert lb2.get_session_count() == 0


def test_probe_thresholds():
    ok = {"v": True}
    eps = three()
    for e in eps:
        e.probe = lambda ep: ok["v"]
    lb = lb_with("round_robin", eps, max_failures=2)
    ok["v"] = False
    lb.perform_health_checks()
    assert eps[0].status == EndpointStatus.DEGRADED
    lb.perform_health_checks()
    assert eps[0].status == EndpointStatus.UNHEALTHY
    ok["v"] = True
    lb.perform_health_checks()
    assert eps[0].status == EndpointStatus.DEGRADED
    lb.perform_health_checks()
    assert eps[0].status == EndpointStatus.HEALTHY


def test_gpu_pages_drive_least_connections():
    pages = [SlotPage("pytest-lb", g) for g in range(3)]
    try:
        for g, (act, free, used) in enumerate(((200, 56, 100_000), (10, 246, 200_000), (10, 246, 50_000))):
            pages[g].write_host(act, free, 0, 1)
            pages[g].set_telemetry(used, 288_000, 50)
            pages[g].set_health(True)
        eps = [Endpoint(id=f"gpu{g}", gpu_index=g, page=pages[g], max_connections=256) for g in range(3)]
        lb = lb_with("least_connections", eps)
        # gpu1 and gpu2 tie on slots; gpu2 has more free HBM
        assert lb.get_endpoint(None, "").id == "gpu2"
        assert eps[2].pending == 1
        lb.mark_admitted("gpu2")
        assert eps[2].pending == 0
        st = lb.get_endpoint_stats()
        assert st["total_connections"] == 220
        d = eps[0].to_dict()
        assert d["load"]["active"] == 200 and d["gpu_index"] == 0
        wr = lb_with("weighted_random", [Endpoint(id=f"g{g}", page=pages[g], max_connections=256) for g in range(3)])
        counts = {"g0": 0, "g1": 0, "g2": 0}
        for _ in range(600):
            counts[wr.get_endpoint(None, "").id] += 1
        assert counts["g0"] < counts["g1"] and counts["g0"] < counts["g2"]
    finally:
        for p in pages:
            p.close(unlink=True)


def test_url_endpoints_get_a_real_http_probe():
    """D9: the reference's health check always reported healthy.  An
    endpoint registered with a URL (and no probe of its own) is probed with
    GET <url>/health: a dead URL goes UNHEALTHY after max_failures checks, a
    live one stays HEALTHY; the autoscaler's placeholder replicas (never
    called, as in the reference) are not probed over HTTP."""
    import http.server
    import socket
    import threading
    from llm_message_queue_amd.scheduler.scheduler import _always_healthy

    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            self.send_response(200 if self.path == "/health" else 404)
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = http.server.HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    dead_port = s.getsockname()[1]
    s.close()                                   # nothing listens there any more
    live = Endpoint(id="live", url=f"http://127.0.0.1:{srv.server_port}", type="llm")
    dead = Endpoint(id="dead", url=f"http://127.0.0.1:{dead_port}", type="llm")
    placeholder = Endpoint(id="ph", url="http://llm-processor-9:8080", type="llm")
    placeholder.probe = _always_healthy
    lb = lb_with("round_robin", [live, dead, placeholder], max_failures=2)
    for _ in range(2):
        lb.perform_health_checks()
    assert live.status == EndpointStatus.HEALTHY
    assert dead.status == EndpointStatus.UNHEALTHY
    assert placeholder.status == EndpointStatus.HEALTHY
    srv.shutdown()
    lb.stop()
