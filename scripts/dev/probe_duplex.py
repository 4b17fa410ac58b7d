"""Dev probe (GPU box): the PCIe ceiling of the host-staged e2e path (VERDICT
r5 item 4).  sqobfs_run_host moves a batch as 8 chunks, H2D | kernel | D2H
on 3 streams, so its rate is bounded by what the link carries in both
directions at once.  This times, on page-locked buffers of run_host's sizes
(256K x 1,360-B input slots in, 256K x 1,360-B output slots out, in 8
chunks each):
  h2d      the input chunks alone, one stream
  d2h      the output chunks alone, one stream
  duplex   both at once, on two streams (each direction's own rate and the
           time both take together)
Each case is repeated `reps` times after a warm-up; medians.  Prints one
JSON object.  usage: probe_duplex.py [packets [reps]]"""
import json
import statistics
import sys
import time

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 15
SLOT_IN, SLOT_OUT, CHUNKS = 1360, 1360, 8
nin, nout = n * SLOT_IN, n * SLOT_OUT
dev = torch.device("cuda", 0)
h_in = torch.empty(nin, dtype=torch.uint8, pin_memory=True)
h_out = torch.empty(nout, dtype=torch.uint8, pin_memory=True)
h_in.fill_(7)
d_in = torch.empty(nin, dtype=torch.uint8, device=dev)
d_out = torch.empty(nout, dtype=torch.uint8, device=dev)
d_out.fill_(9)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def chunks(total):
    c = (total + CHUNKS - 1) // CHUNKS
    return [(o, min(c, total - o)) for o in range(0, total, c)]


def h2d(s):
    with torch.cuda.stream(s):
        for o, c in chunks(nin):
            d_in[o:o + c].copy_(h_in[o:o + c], non_blocking=True)


def d2h(s):
    with torch.cuda.stream(s):
        for o, c in chunks(nout):
            h_out[o:o + c].copy_(d_out[o:o + c], non_blocking=True)


def timed(fn):
    out = []
    for _ in range(reps + 2):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        out.append(time.perf_counter() - t0)
    return statistics.median(out[2:])


def duplex_each():
    """each direction's own time while both run (events on each stream)"""
    ts = {"h2d": [], "d2h": [], "both": []}
    for _ in range(reps + 2):
        torch.cuda.synchronize(dev)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        t0 = time.perf_counter()
        e[0].record(s1)
        e[2].record(s2)
        h2d(s1)
        d2h(s2)
        e[1].record(s1)
        e[3].record(s2)
        torch.cuda.synchronize(dev)
        ts["both"].append(time.perf_counter() - t0)
        ts["h2d"].append(e[0].elapsed_time(e[1]) * 1e-3)
        ts["d2h"].append(e[2].elapsed_time(e[3]) * 1e-3)
    return {k: statistics.median(v[2:]) for k, v in ts.items()}


t_h2d = timed(lambda: h2d(s1))
t_d2h = timed(lambda: d2h(s2))
dx = duplex_each()
gb = 1e9
res = {
    "packets": n, "chunks": CHUNKS, "in_bytes": nin, "out_bytes": nout, "reps": reps,
    "h2d_alone_GBps": round(nin / t_h2d / gb, 2),
    "d2h_alone_GBps": round(nout / t_d2h / gb, 2),
    "duplex_h2d_GBps": round(nin / dx["h2d"] / gb, 2),
    "duplex_d2h_GBps": round(nout / dx["d2h"] / gb, 2),
    "duplex_both_ms": round(dx["both"] * 1e3, 3),
    "duplex_total_GBps": round((nin + nout) / dx["both"] / gb, 2),
    # the payload rate a run_host batch of n x 1,350 B could reach if the link
    # were its only limit: both directions' bytes in the duplex time
    "ceiling_payload_GiBps": round(n * 1350 / dx["both"] / 2**30, 3),
}
print(json.dumps(res), flush=True)
