"""Serve-loop stall watchdog (``server.stall_dump_after``)."""


def test_stall_watchdog_dumps_stacks_once(capfd):
    """``server.stall_dump_after``: no tick while requests wait -> one error
    log and every thread's stack on stderr (what a hung rank was doing)."""
    import threading
    import time
    from types import SimpleNamespace
    from llm_message_queue_amd.gateway.app import GatewayApp
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.server.stall_dump_after = 200_000_000          # 0.2 s
    logged = []
    gw = SimpleNamespace(counters={"ticks": 7}, pending=lambda: 3, engine=None, rank=0)
    app = SimpleNamespace(gateway=gw, cfg=cfg, _stop=threading.Event(),
                          log=SimpleNamespace(error=lambda msg, **kw: logged.append((msg, kw))))
    th = threading.Thread(target=GatewayApp._stall_watchdog, args=(app,), daemon=True)
    th.start()
    time.sleep(0.8)
    app._stop.set()
    th.join(2)
    assert len(logged) == 1 and logged[0][1]["waiting"] == 3
    assert "_stall_watchdog" in capfd.readouterr().err   # the dump names the watchdog's own frame
