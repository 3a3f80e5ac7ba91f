"""PeerDirectory: rank 0's scatter-gather queries over the node-local shm
rings (gateway/peers.py), both ends in one process."""
import os

import pytest

from llm_message_queue_amd.gateway.peers import PeerDirectory


def _handler_for(rank):
    store = {f"m{rank}": {"id": f"m{rank}", "rank": rank}}

    def handler(op, args):
        if op == "get":
            if args[0] == "boom":
                raise RuntimeError("store unavailable")
            return store.get(args[0])
        if op == "stats":
            if rank == 2:
                raise RuntimeError("stats broke")
            return {"counters": {"dispatched": rank}}
        return None
    return handler


@pytest.fixture
def dirs():
    name = f"pt{os.getpid()}"
    world = 3
    peers = [PeerDirectory(name, r, world, _handler_for(r)) for r in range(1, world)]
    root = PeerDirectory(name, 0, world)
    yield root, peers
    for p in peers:
        p.close()
    root.close(unlink=True)
    for p in peers:
        p.qring.unlink()


def test_first_finds_the_rank_holding_the_message(dirs):
    root, _ = dirs
    assert root.first("get", ["m2"]) == {"id": "m2", "rank": 2}
    assert root.first("get", ["m1"]) == {"id": "m1", "rank": 1}
    assert root.first("get", ["nope"]) is None


def test_a_peer_error_is_no_answer(dirs):
    root, _ = dirs
    # every peer's handler raises: the error dicts come back from ask() but
    # first() must not hand one out as the message
    got = root.ask("get", ["boom"])
    assert set(got) == {1, 2} and all("error" in v for v in got.values())
    assert root.first("get", ["boom"]) is None


def test_ask_collects_every_rank(dirs):
    root, _ = dirs
    got = root.ask("stats", [])
    assert got[1] == {"counters": {"dispatched": 1}}
    assert "error" in got[2]
    with pytest.raises(ValueError):
        root.ask("not-an-op", [])


def test_large_answers_from_every_peer_arrive_paged():
    """7 peers each answering several MiB (more than a reply page
    and, together, far more than any one ring) all arrive whole."""
    name = f"ptbig{os.getpid()}"
    world = 8
    blob = {r: os.urandom(3 << 20) + bytes([r]) for r in range(1, world)}
    peers = [PeerDirectory(name, r, world, lambda op, args, r=r: [r, blob[r]]) for r in range(1, world)]
    root = PeerDirectory(name, 0, world)
    try:
        for _ in range(2):
            got = root.ask("dlq", ["list"], timeout_s=20.0)
            assert sorted(got) == list(range(1, world)) and root.last_missing == []
            for r, v in got.items():
                assert v[0] == r and v[1] == blob[r]
        assert sum(p.dropped for p in peers) == 0
    finally:
        for p in peers:
            p.close()
        root.close(unlink=True)
        for p in peers:
            p.qring.unlink()


def test_a_silent_peer_is_reported_missing_and_its_late_answer_is_discarded():
    name = f"ptslow{os.getpid()}"
    import time
    world = 3
    gate = {"sleep": 0.6}

    def slow(op, args):
        time.sleep(gate["sleep"])
        return "late" if op == "stats" else None

    peers = [PeerDirectory(name, 1, world, lambda op, args: "fast"), PeerDirectory(name, 2, world, slow)]
    root = PeerDirectory(name, 0, world)
    try:
        got = root.ask("stats", [], timeout_s=0.2)
        assert got == {1: "fast"} and root.last_missing == [2] and root.missing_total == 1
        time.sleep(0.8)                       # rank 2's late answer lands in its ring now
        gate["sleep"] = 0.0
        got = root.ask("get", ["x"], timeout_s=2.0)
        assert got == {1: "fast", 2: None} and root.last_missing == []   # the stale "late" is not taken
    finally:
        for p in peers:
            p.close()
        root.close(unlink=True)
        for p in peers:
            p.qring.unlink()
