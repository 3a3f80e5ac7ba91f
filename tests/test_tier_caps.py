"""Per-tier in-flight caps (``queue.levels[*].max_concurrent``, a dead key in
the reference that acts here).  The reference ships caps that grow toward
the bulk tiers (realtime 100 / high 200 / normal 500 / low 1000); taken
literally they held urgent requests back while less urgent ones were
admitted (one GPU at 5k req/s: high p99 1.7 s vs normal 150 ms).  With
``queue.priority_monotone_caps`` (default) a tier may always hold at least as
many requests in flight as any less urgent tier."""
from llm_message_queue_amd.gateway.router import Gateway


def test_tier_caps_monotone_rule():
    f = Gateway._tier_caps
    assert f([100, 200, 500, 1000], True) == [1000, 1000, 1000, 1000]
    assert f([100, 200, 500, 1000], False) == [100, 200, 500, 1000]
    # capping a bulk tier below the urgent ones keeps working
    assert f([0, 300, 300, 50], True) == [-1, 300, 300, 50]
    assert f([64, 32, 16, 8], True) == [64, 32, 16, 8]
    # an uncapped less urgent tier leaves every more urgent tier uncapped
    assert f([10, 20, 0, 40], True) == [-1, -1, -1, 40]


def _gateway(monotone, caps, slots=64):
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.queue.enable_metrics = False
    cfg.queue.realtime_lane = False
    cfg.queue.priority_monotone_caps = monotone
    for lv, c in zip(sorted(cfg.queue.levels, key=lambda lv: lv.priority), caps):
        lv.max_concurrent = c
    eng = BackendEngine(LlamaConfig.tiny(), slots=slots, max_ctx=64, token_budget=2048, device="cpu", impl="ref")
    return Gateway(cfg, engine=eng, use_gpu_preprocess=False, prompt_cap=8, gen_tokens=2)


def _msgs(prio, n):
    from llm_message_queue_amd.models.message import Message
    return [Message(id=f"p{prio}-{i}", content="hello there", priority=prio, user_id="u") for i in range(n)]


def test_high_tier_not_held_behind_normal_by_its_cap():
    """High (cap 4) and normal (cap 16) both queued deep, 64 slots: literal
    caps admit 4 high and 16 normal; monotone caps (every tier at least low's
    32) admit high first, up to 32, then normal into the rest."""
    for monotone, want in ((False, [0, 4, 16, 0]), (True, [0, 32, 32, 0])):
        gw = _gateway(monotone, [2, 4, 16, 32])
        gw.submit(_msgs(2, 40) + _msgs(3, 40))
        gw.ingest()
        gw.dispatch()
        assert gw.inflight_by_tier.tolist() == want, (monotone, gw.inflight_by_tier)

