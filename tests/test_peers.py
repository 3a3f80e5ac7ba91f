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
