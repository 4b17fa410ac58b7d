"""Dev probe (GPU box): where the in-process shard path loses time against
queued launches.  One configs[1] shard, one context; per variant the wall
time of K steps (median of rounds, one process, one buffer set):
  torch     sqobfs.launch on torch's current stream, one sync at the end
            (bench.py's queued launches)
  ctx       the same on the context's own stream
  ctx_ev    + a torch event (no timing) recorded on the context's stream
            after every launch (what sqobfs_shard_launch adds)
  ticket1/2 sqobfs_shard_launch / wait, 1 or 2 steps in flight
  ticketN0  2 in flight with the context's sync spin 0 (blocking waits)
usage: inproc_probe.py [K] [ROUNDS]"""
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "sing-quic_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import sqobfs  # noqa: E402
import bench  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 50
R = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
kind, n, L, n_psk = bench.CONFIGS["salamander-1m"]
sh = bench.build_shard(torch, dev, kind, n, L, n_psk, 0, 1, "salamander-1m", "dense")
ctx = sqobfs.Context(0)
ctx.unit_packets = sqobfs.unit_packets_for(sh["payload_bytes"], n, False)
kr = sqobfs.Keyring(ctx, kind, sh["psks"])
b = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"], sh["out_off"],
                      sh["out_len"], sh["salt"], sh["psk_id"])
ts = torch.cuda.current_stream(dev)
cs = torch.cuda.ExternalStream(ctx.stream, device=dev)
torch.cuda.synchronize()


def v_torch():
    for _ in range(K):
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, ts.cuda_stream)
    torch.cuda.synchronize()


def v_ctx():
    for _ in range(K):
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, ctx.stream)
    ctx.sync(ctx.stream)


def v_ctx_ev():
    evs = []
    for _ in range(K):
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, ctx.stream)
        e = torch.cuda.Event()
        e.record(cs)
        evs.append(e)
    ctx.sync(ctx.stream)


def tickets(depth, spin):
    def f():
        ctx.set_sync_spin(spin)
        pend = []
        for _ in range(K):
            pend.append(sqobfs.shard_launch([ctx], [kr], sqobfs.OBFUSCATE, [b]))
            if len(pend) >= depth:
                pend.pop(0).wait()
        for t in pend:
            t.wait()
    return f


variants = [("torch", v_torch), ("ctx", v_ctx), ("ctx_ev", v_ctx_ev),
            ("ticket1", tickets(1, 4000)), ("ticket2", tickets(2, 4000)),
            ("ticketN0", tickets(2, 0)), ("ticket3", tickets(3, 4000))]
for _, f in variants:
    f()
res = {nm: [] for nm, _ in variants}
for _ in range(R):
    for nm, f in variants:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        res[nm].append((time.perf_counter() - t0) / K * 1e3)
for nm, _ in variants:
    print(f"{nm:10s} median {statistics.median(res[nm]):.4f} ms/step  all "
          f"{[round(x, 4) for x in res[nm]]}", flush=True)
