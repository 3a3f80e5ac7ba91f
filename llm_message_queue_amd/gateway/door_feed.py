"""A load generator standing in for the native front door (bench.py
``--ingress rank0``): one process, Poisson arrivals of the bench workload,
each written at its arrival time as a TAG_RAW record -- the record the C++
HTTP ingress writes (`csrc/ingress/http_ingress.cpp`: arrival ns, id, JSON
body) -- into ONE shared ring that every rank drains, as `cli serve`'s front
door does (`cli/main.py`: a shared MPMC request ring).

It runs as its own process so the feed never waits for a rank's Python
(the C++ front door never does either): the arrival -> ring hop costs what
it costs in production, and what a rank adds (its pump cadence) shows up in
the bench's ``ingress`` stage.

Control: one line per command on stdin --
  ``rate <req/s> <t0 monotonic s>``   start (or change) the Poisson clock at t0
  ``stop``                            no more arrivals (the ring keeps what it has)
  ``exit``                            quit.
Every command is acknowledged with one line on stdout (``ok <pushed>``)."""
from __future__ import annotations

import argparse
import json
import select
import sys
import time

from .. import _native
from .shm_bridge import TAG_RAW
from .workload import PoissonArrivals, Workload

POOL = 16384


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ring", required=True)
    ap.add_argument("--ring-bytes", type=int, default=256 << 20)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    ring = _native.shmring().ShmRing(a.ring, a.ring_bytes, "open")
    pool = []
    for m in Workload(seed=a.seed).make(POOL):
        body = {"content": m.content, "user_id": m.user_id}
        if m.priority:
            body["priority"] = int(m.priority)
        pool.append(json.dumps(body).encode())
    arr = PoissonArrivals(0.0, seed=a.seed)
    active = False
    serial = pushed = 0
    print("ok 0", flush=True)
    while True:
        # commands (non-blocking while feeding, blocking while idle)
        r, _, _ = select.select([sys.stdin], [], [], 0.0002 if active else 0.5)
        if r:
            line = sys.stdin.readline()
            if not line:
                break
            cmd = line.split()
            if not cmd:
                continue
            if cmd[0] == "rate":
                arr = PoissonArrivals(float(cmd[1]), seed=a.seed + serial)
                arr.reset(float(cmd[2]))
                active = float(cmd[1]) > 0
            elif cmd[0] == "stop":
                active = False
            elif cmd[0] == "exit":
                print(f"ok {pushed}", flush=True)
                break
            print(f"ok {pushed}", flush=True)
        if not active:
            continue
        due = arr.due(time.monotonic())
        if not due:
            continue
        recs = []
        for ts in due:
            body = pool[serial % POOL]
            recs.append(int(ts * 1e9).to_bytes(8, "little", signed=True)
                        + (b"door-%x" % serial).ljust(36, b"\0")
                        + len(body).to_bytes(4, "little") + body)
            serial += 1
        n = ring.push_many(recs, TAG_RAW)
        pushed += n
        if n != len(recs):
            print(f"door_feed: ring full, {len(recs) - n} arrivals dropped", file=sys.stderr, flush=True)
    ring.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
