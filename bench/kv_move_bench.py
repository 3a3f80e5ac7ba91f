"""KV-migration data plane on one MI355X (N11):

  * ``kv_move`` pack / unpack (one HIP launch over all 32 layers: the
    conversation's K/V rows of a slot <-> a packed [L][2][Hkv][n][128]
    buffer) at 32, 300 and 512 tokens -- GB/s of HBM traffic (read + write)
    against the ~6.3 TB/s a streaming copy reaches;
  * the RCCL leg: a world-1 self ``exchange_p2p`` (send + receive on the same
    device, one RCCL group call) swept from 1 to 64 MiB -- what the
    transport costs before any xGMI link is involved (a one-GPU box has no
    peer; the 8-GPU number is the driver's).

Prints one JSON line.  Llama-3-8B KV shape: 32 layers x 8 KV heads x 128,
bf16 = 128 KiB per token."""
import json
import os
import socket
import sys
import time
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

DEV = torch.device("cuda", 0)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters          # ms


def main():
    import torch.distributed as dist
    from llm_message_queue_amd.parallel.comm import TorchComm
    from llm_message_queue_amd.parallel.migration import KVMigrator
    L, H, D, SLOTS, CTX = 32, 8, 128, 64, 512
    cfg = SimpleNamespace(layers=L, kv_heads=H, head_dim=D)
    kc = [torch.randn(SLOTS, H, CTX, D, device=DEV).to(torch.bfloat16) for _ in range(L)]
    vc = [torch.randn(SLOTS, H, CTX, D, device=DEV).to(torch.bfloat16) for _ in range(L)]
    model = SimpleNamespace(cfg=cfg, kcache=kc, vcache=vc, slots=SLOTS, max_ctx=CTX)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=DEV)
    try:
        comm = TorchComm()
        mig = KVMigrator(model, comm)
        out = {"kv_shape": "32 layers x 2 x 8 kv heads x n x 128 bf16 (128 KiB / token)", "kv_move": [],
               "rccl_self_p2p": []}
        default_variant = mig.KV_VARIANT
        variants = [int(v) for v in os.environ.get("KV_VARIANTS", str(default_variant)).split(",")]
        for var in variants:
            mig.KV_VARIANT = var
            for n in (32, 300, 512):
                nbytes = L * 2 * H * n * D * 2
                buf = mig.pack(3, n)
                ms_p = _time(lambda: mig._kv_move(buf, 3, True, torch.cuda.current_stream()), 50)
                ms_u = _time(lambda: mig._kv_move(buf, 7, False, torch.cuda.current_stream()), 50)
                out["kv_move"].append({"variant": var, "tokens": n, "bytes": nbytes,
                                       "pack_us": round(ms_p * 1e3, 2), "unpack_us": round(ms_u * 1e3, 2),
                                       "pack_GBps": round(2 * nbytes / (ms_p * 1e-3) / 1e9, 1),
                                       "unpack_GBps": round(2 * nbytes / (ms_u * 1e-3) / 1e9, 1)})
        # Beyond the 256 MiB Infinity Cache: pack 16
        # different 512-token conversations (64 MiB each) into 16 different
        # buffers in rotation -- 1 GiB read + 1 GiB written per round, so no
        # launch finds its bytes in the cache -- and the same rotation as
        # plain torch copies of 64 MiB buffers (the achievable-copy reference)
        nrot, n = 16, 512
        nbytes = L * 2 * H * n * D * 2
        bufs = [mig.pack(s_, n) for s_ in range(nrot)]
        torch.cuda.synchronize()
        src = [torch.empty(nbytes, dtype=torch.uint8, device=DEV) for _ in range(nrot)]
        dst = [torch.empty_like(x) for x in src]
        rc = {"k": 0}

        def copy_rot():
            k = rc["k"]
            dst[k].copy_(src[k])
            rc["k"] = (k + 1) % nrot
        ms_rc = _time(copy_rot, 4 * nrot)
        out["beyond_cache"] = {"working_set_GiB": round(2 * nrot * nbytes / 2**30, 2), "bytes_per_launch": nbytes,
                               "torch_copy_GBps": round(2 * nbytes / (ms_rc * 1e-3) / 1e9, 1)}
        for var in variants:
            mig.KV_VARIANT = var
            rot = {"k": 0}

            def pack_rot():
                k = rot["k"]
                mig._kv_move(bufs[k], k, True, torch.cuda.current_stream())
                rot["k"] = (k + 1) % nrot
            ms_r = _time(pack_rot, 4 * nrot)
            tag = "" if var == 0 else f"_v{var}"
            out["beyond_cache"][f"kv_move_pack_GBps{tag}"] = round(2 * nbytes / (ms_r * 1e-3) / 1e9, 1)
            out["beyond_cache"][f"kv_move_over_copy{tag}"] = round(ms_rc / ms_r, 3)
        mig.KV_VARIANT = default_variant
        del bufs, src, dst
        # same bytes as one torch copy (reference point for the HBM roofline)
        a = torch.empty(512 * 128 * 1024, dtype=torch.uint8, device=DEV)
        b = torch.empty_like(a)
        ms_c = _time(lambda: b.copy_(a), 50)
        out["torch_copy_64MiB_GBps"] = round(2 * a.numel() / (ms_c * 1e-3) / 1e9, 1)
        comm.warm_data_plane()
        for mib in (1, 2, 4, 8, 16, 32, 64):
            s = torch.ones(mib << 20, dtype=torch.uint8, device=DEV)
            r = torch.empty_like(s)
            for _ in range(3):
                comm.exchange_p2p([(0, s)], [(0, r)])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            it = 20
            for _ in range(it):
                comm.exchange_p2p([(0, s)], [(0, r)])
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / it
            out["rccl_self_p2p"].append({"MiB": mib, "us": round(dt * 1e6, 1),
                                         "GBps": round((mib << 20) / dt / 1e9, 1)})
        assert torch.equal(r, s)
        print(json.dumps(out), flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
