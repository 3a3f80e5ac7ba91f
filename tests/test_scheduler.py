"""Scheduler (C12) strategies and ResourceScheduler (C13), incl. the fixed
defects D10-D13."""
import datetime as dt
import time

import pytest

from llm_message_queue_amd.balancer.load_balancer import Endpoint, LoadBalancer
from llm_message_queue_amd.scheduler.resource_scheduler import (RequestQueued, Resource, ResourceError,
                                                                ResourceRequest, ResourceScheduler,
                                                                ResourceSchedulerConfig, ResourceStatus)
from llm_message_queue_amd.scheduler.scheduler import EndpointPool, Scheduler, SchedulerConfig
from llm_message_queue_amd.utils.config import LoadBalancerConfig


def lb():
    return LoadBalancer(LoadBalancerConfig(health_check_interval=0))


def test_dynamic_scale_up_down_and_recommendation():
    l = lb()
    l.add_endpoint(Endpoint(id="endpoint-1"))
    stats = {"realtime": 300, "high": 10, "normal": 0, "low": 0}
    s = Scheduler(SchedulerConfig(), lambda: stats, l)
    assert s.schedule_resources() == "scale_up"
    assert [e.id for e in l.get_all_endpoints()] == ["endpoint-1", "endpoint-2"]
    assert l.get_endpoint_by_id("endpoint-2").url == "http://llm-processor-2:8080"
    assert s.recommendation == "least_connections"
    stats.update(realtime=0, high=0)
    assert s.schedule_resources() == "scale_down"
    assert len(l.get_all_endpoints()) == 1
    assert s.schedule_resources() == "none"           # at min
    assert s.recommendation == "weighted_random"


def test_missing_level_stats_no_crash():
    """D13: the reference nil-derefs when a level queue is absent."""
    s = Scheduler(SchedulerConfig(), lambda: {}, lb())
    s.schedule_resources()


def test_adaptive_business_hours():
    l = lb()
    s = Scheduler(SchedulerConfig(strategy="adaptive", resource_limits={"min_endpoints": 1, "max_endpoints": 4}),
                  lambda: {"normal": 0}, l, clock=lambda: dt.datetime(2025, 9, 3, 10, 0))   # Wednesday 10:00
    s.schedule_resources()
    assert len(l.get_all_endpoints()) == 3             # max - 1
    s.clock = lambda: dt.datetime(2025, 9, 6, 22, 0)   # Saturday night, queue below scale-down
    s.schedule_resources()
    assert len(l.get_all_endpoints()) == 1


def test_hybrid_applies_weights():
    l = lb()
    l.add_endpoint(Endpoint(id="a", response_time=20_000_000))
    l.add_endpoint(Endpoint(id="b", response_time=400_000_000))
    s = Scheduler(SchedulerConfig(strategy="hybrid", resource_limits={"min_endpoints": 1, "max_endpoints": 2}),
                  lambda: {"normal": 50}, l)
    s.schedule_resources()
    assert l.get_endpoint_by_id("a").weight == 5 and l.get_endpoint_by_id("b").weight == 1


def test_gpu_pool_park_and_reactivate():
    l = lb()
    pool = EndpointPool([Endpoint(id=f"gpu{i}", gpu_index=i) for i in range(1, 3)])
    l.add_endpoint(Endpoint(id="gpu0", gpu_index=0))
    stats = {"normal": 1000}
    s = Scheduler(SchedulerConfig(), lambda: stats, l, pool=pool)
    s.schedule_resources()
    s.schedule_resources()
    assert [e.id for e in l.get_all_endpoints()] == ["gpu0", "gpu1", "gpu2"]
    assert s.schedule_resources() == "none"            # pool empty: no fake URLs
    stats["normal"] = 0
    s.schedule_resources()
    assert pool.size() == 1 and len(l.get_all_endpoints()) == 2


def test_scheduler_thread_lifecycle():
    s = Scheduler(SchedulerConfig(monitor_interval=5_000_000), lambda: {}, lb())
    s.start()
    s.start()
    assert s.is_running()
    time.sleep(0.03)
    s.stop()
    assert not s.is_running()


# ---------------------------------------------------------------- ResourceScheduler
def rs(**kw):
    return ResourceScheduler(ResourceSchedulerConfig(**kw), start=False)


def gpu_res(rid, slots=4, hbm=100):
    return Resource(id=rid, type="llama3-8b", capabilities=["bf16"], capacity={"gpu": slots, "memory": hbm})


def test_allocate_lowest_load_and_release_exact():
    s = rs()
    s.register_resource(gpu_res("a"))
    s.register_resource(gpu_res("b"))
    a1 = s.request_resource(ResourceRequest("r1", "llama3-8b", {"gpu": 2, "memory": 50}))
    a2 = s.request_resource(ResourceRequest("r2", "llama3-8b", {"gpu": 1, "memory": 10}))
    assert a1.resource_id != a2.resource_id                      # lowest load wins
    ra = s.get_resource(a1.resource_id)
    assert ra.used == {"gpu": 2, "memory": 50} and abs(ra.load - 0.5) < 1e-9
    assert a1.token.startswith("r1-" + a1.resource_id + "-")
    s.release_resource("r1")
    assert ra.used == {"gpu": 0, "memory": 0} and ra.load == 0.0  # D11: exact accounting
    with pytest.raises(ResourceError):
        s.release_resource("r1")


def test_capabilities_type_and_busy():
    s = rs()
    s.register_resource(gpu_res("a", slots=10))
    with pytest.raises(RequestQueued):
        s.request_resource(ResourceRequest("x", "other-model", {"gpu": 1}))
    with pytest.raises(RequestQueued):
        s.request_resource(ResourceRequest("y", "llama3-8b", {"gpu": 1}, capabilities=["fp4"]))
    s.request_resource(ResourceRequest("z", "llama3-8b", {"gpu": 10, "memory": 100}))
    assert s.get_resource("a").status == ResourceStatus.BUSY


def test_pending_queue_urgency_order_and_timeouts():
    """D10 (queued_at set, no panic) + D12 (more urgent first)."""
    s = rs()
    s.register_resource(gpu_res("a", slots=1))
    s.request_resource(ResourceRequest("hold", "llama3-8b", {"gpu": 1}))
    for rid, prio in (("low", 4), ("rt", 1), ("hi", 2)):
        with pytest.raises(RequestQueued):
            s.request_resource(ResourceRequest(rid, "llama3-8b", {"gpu": 1}, priority=prio, timeout=10**12))
    with pytest.raises(RequestQueued):
        s.request_resource(ResourceRequest("stale", "llama3-8b", {"gpu": 1}, priority=1, timeout=1))
    assert [r.request_id for r in s.pending] == ["rt", "stale", "hi", "low"]
    time.sleep(0.001)
    s.release_resource("hold")                        # frees the slot -> most urgent live request wins
    assert s.get_allocation("rt").resource_id == "a"
    assert [r.request_id for r in s.pending] == ["hi", "low"]   # "stale" timed out


def test_heartbeat_offline_and_expiry():
    s = rs(heartbeat_timeout=10_000_000)
    s.register_resource(gpu_res("a"))
    s.request_resource(ResourceRequest("r", "llama3-8b", {"gpu": 1}, timeout=5_000_000))
    time.sleep(0.02)
    assert s.check_resource_status() == ["a"]
    assert s.check_allocations() == 1
    assert s.get_resource("a").used["gpu"] == 0
    s.heartbeat("a", used={"gpu": 2}, capacity={"gpu": 4})
    r = s.get_resource("a")
    assert r.status == ResourceStatus.AVAILABLE and r.load == pytest.approx(0.25)
    st = s.get_resource_stats()
    assert st["resources"]["total"] == 1 and st["resource_by_type"] == {"llama3-8b": 1}


def test_autoscale_decisions_and_register_gpu():
    events = []
    s = ResourceScheduler(ResourceSchedulerConfig(enable_auto_scaling=True, scale_cooldown=0, max_resources=4),
                          start=False, on_scale=lambda a, l: events.append(a))
    r = s.register_gpu(0, "llama3-8b", slots=8, hbm_total=288 << 30, kv_tokens=8 * 512)
    assert r.capacity["gpu"] == 8 and r.endpoint == "gpu://0"
    s.request_resource(ResourceRequest("a", "llama3-8b", {"gpu": 8, "tokens": 4096, "memory": 200 << 30}))
    assert s.check_auto_scaling() == "scale_up" and events == ["scale_up"]


def test_background_threads_process_pending():
    s = ResourceScheduler(ResourceSchedulerConfig(pending_retry_period=10_000_000, resource_check_period=10_000_000))
    try:
        with pytest.raises(RequestQueued):
            s.request_resource(ResourceRequest("w", "m", {"gpu": 1}))
        s.register_resource(Resource(id="late", type="m", capacity={"gpu": 1}))
        t0 = time.time()
        while s.get_pending_queue_length() and time.time() - t0 < 2:
            time.sleep(0.01)
        assert s.get_allocation("w").resource_id == "late"
    finally:
        s.stop()
