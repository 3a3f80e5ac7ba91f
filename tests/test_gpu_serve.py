"""The serving stack on a real GPU: REST API -> GPU preprocess micro-batches ->
C++ queue -> gateway serve loop -> continuous-batching engine (tiny
Llama-shaped stub through the HIP kernels) -> completion status, metrics,
telemetry and operator health control."""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def served():
    from fastapi.testclient import TestClient

    from llm_message_queue_amd.api.server import create_app
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.backend.slot_page import SlotPage
    from llm_message_queue_amd.balancer.load_balancer import Endpoint
    from llm_message_queue_amd.gateway.app import GatewayApp
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.utils.config import default_config

    cfg = default_config()
    cfg.preprocessor.batch_window_us = 200
    cfg.backend.prompt_tokens = 16
    cfg.backend.gen_tokens = 2
    page = SlotPage("pytest-serve", 0)
    eng = BackendEngine(LlamaConfig.tiny(), slots=32, max_ctx=64, token_budget=256, device="cuda:0", impl="hip",
                        page=page, gpu_index=0)
    app = GatewayApp(cfg, use_gpu=True, engine=eng, start=False)
    app.lb.add_endpoint(Endpoint(id="gpu0", type="llm", gpu_index=0, page=page, max_connections=32))
    app.start_telemetry({0: page})
    app.start()
    with TestClient(create_app(app)) as c:
        c.app_ = app
        yield c
    app.stop()
    page.close(unlink=True)


def wait_status(c, mid, status="completed", t=20.0):
    t0 = time.time()
    while time.time() - t0 < t:
        r = c.get(f"/api/v1/messages/{mid}")
        if r.status_code == 200 and r.json()["status"] == status:
            return True
        time.sleep(0.02)
    return False


def test_rest_to_gpu_backend_completion(served):
    c = served
    ids = []
    for i in range(24):
        body = {"content": ("URGENT: " if i % 3 == 0 else "") + f"please summarise item {i} for me?", "user_id": "u"}
        r = c.post("/api/v1/messages", json=body)
        assert r.status_code == 202, r.text
        ids.append(r.json()["message_id"])
    assert all(wait_status(c, mid) for mid in ids)
    m = c.get(f"/api/v1/messages/{ids[0]}").json()
    assert m["priority"] == 2 and m["metadata"]["analyzed"] and m["metadata"]["contains_question"] == "true"
    assert "ml_priority" in m["metadata"]                         # MFMA classifier ran
    app = c.app_
    assert app.preprocessor.stats["gpu_batches"] >= 1
    assert app.engine.completed_total >= 24
    met = c.get("/metrics").text
    assert "llm_queue_enqueue_to_dispatch_seconds" in met


def test_operator_marks_gpu_unhealthy_and_back(served):
    c = served
    r = c.put("/api/v1/endpoints/gpu0/status", json={"status": "unhealthy"})
    assert r.status_code == 200
    assert not c.app_.gateway.healthy
    mid = c.post("/api/v1/messages", json={"content": "held while the GPU is out", "user_id": "u"}).json()["message_id"]
    time.sleep(0.3)
    assert c.get(f"/api/v1/messages/{mid}").json()["status"] != "completed"
    c.put("/api/v1/endpoints/gpu0/status", json={"status": "healthy"})
    assert wait_status(c, mid)


def test_telemetry_snapshot_or_unavailable(served):
    tel = served.app_.telemetry
    assert tel is not None
    if tel.available:                                   # amd-smi present: real HBM numbers for OUR GPU
        tel.native.poll_once()
        snap = tel.publish()
        mine = [s for s in snap if (tel.gpu_map.get(s["gpu"], s["gpu"]) if tel.gpu_map else s["gpu"]) == 0]
        assert mine and mine[0]["valid"] and mine[0]["hbm_total_mb"] > 100_000, (snap, tel.gpu_map)
        assert served.app_.gateway.healthy              # telemetry of other GPUs never evacuates ours


def test_backend_fault_evacuation_with_steps_in_flight():
    """Launch faults while 2 steps are queued on the GPU: the evacuated
    requests are re-queued and completed, and the steps dropped by the
    evacuation finish before their pinned staging buffers are refilled
    (regression: refilling them under an in-flight H2D fed the kernels
    mismatched descriptors)."""
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.utils.config import default_config

    cfg = default_config()
    cfg.queue.enable_metrics = False
    eng = BackendEngine(LlamaConfig.tiny(), slots=32, max_ctx=64, token_budget=256, device="cuda:0", impl="hip",
                        max_inflight=2)
    gw = Gateway(cfg, engine=eng, use_gpu_preprocess=True, prompt_cap=16, gen_tokens=3)
    gw.submit(Workload(seed=3).make(200))
    faults = 0
    for i in range(400):
        if i % 7 == 3 and faults < 10:
            eng.inject(fail_launch=1)
            faults += 1
        gw.tick()
        if not gw.healthy:
            gw.set_healthy(True)
        if gw.counters["completed"] >= 200:
            break
    torch.cuda.synchronize()
    assert faults >= 3 and gw.counters["evacuated"] > 0
    assert gw.counters["completed"] >= 200, gw.counters


def test_overload_expiry_and_adaptive_lifo_on_gpu():
    """Requests past their deadline are shed to the DLQ, never dispatched;
    with adaptive LIFO the newest requests of an overloaded tier go first."""
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.queue.dead_letter import DeadLetterQueue
    from llm_message_queue_amd.utils.config import default_config

    cfg = default_config()
    cfg.queue.enable_metrics = False
    cfg.queue.adaptive_lifo = True
    cfg.queue.lifo_after = 1_000_000                      # 1 ms
    dlq = DeadLetterQueue()
    eng = BackendEngine(LlamaConfig.tiny(), slots=8, max_ctx=64, token_budget=128, device="cuda:0", impl="hip")
    gw = Gateway(cfg, engine=eng, use_gpu_preprocess=True, prompt_cap=16, gen_tokens=2, dead_letter=dlq)
    msgs = Workload(seed=4).make(64)
    now = time.monotonic_ns()
    for i, m in enumerate(msgs):
        m.timeout = 200_000_000 if i < 16 else 30_000_000_000
        m.arrival_ns = now - (500_000_000 if i < 16 else 0)
    gw.submit(msgs)
    for _ in range(200):
        gw.tick()
        if gw.counters["completed"] + gw.counters["expired"] >= 64:
            break
    torch.cuda.synchronize()
    assert gw.counters["expired"] == 16 and dlq.size() == 16
    assert all(m.status == "timeout" and not m.dispatched_at for m in msgs[:16])
    assert gw.counters["completed"] == 48


def test_async_ingest_matches_sync():
    """Overlapped ingest (launch the preprocess batch, enqueue when its
    kernels finished) produces exactly the synchronous path's messages."""
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.queue.enable_metrics = False
    outs = []
    for mode in ("sync", "async"):
        eng = BackendEngine(LlamaConfig.tiny(), slots=8, max_ctx=64, token_budget=128, device="cuda:0", impl="hip")
        gw = Gateway(cfg, engine=eng, use_gpu_preprocess=True, prompt_cap=16, gen_tokens=2)
        msgs = Workload(seed=9).make(200)
        gw.submit(msgs)
        if mode == "sync":
            gw.ingest()
        else:
            assert gw.ingest_async() and gw.preprocessing() == 200 and gw.pending() == 0
            t0 = time.time()
            while gw.preprocessing() and time.time() - t0 < 10:
                gw.ingest_async()
        assert gw.pending() == 200
        outs.append([(m.priority, m.queue_name, m.metadata.get("word_count"), m.metadata.get("sentiment"),
                      m.metadata.get("contains_question"), m.metadata.get("ml_priority"),
                      tuple(int(x) for x in m.prompt_ids)) for m in msgs])
    assert outs[0] == outs[1]
