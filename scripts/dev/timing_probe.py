"""Dev probe (GPU box): what the bench's per-kernel timing costs the step.
configs[1] (1M x 1350 B Salamander obfuscate, dense, host salts), one buffer
set, one process; interleaved rounds of STEPS launches each, timed three ways:
  torch2  a torch.cuda.Event pair recorded around every launch (bench.py
          through round 4's first builds): two marker packets per step
  ext     the pair recorded by the launch's own dispatch
          (sqobfs.DispatchEvents / sqobfs_debug_time_next_launch)
  none    launches only
  two     launches only, alternating between two streams (each with its own
          output buffers), so a launch's head may overlap the previous
          one's tail
Prints per mode the wall time per step (sync-bracketed) and the kernel
average where events exist.  usage: timing_probe.py [ROUNDS] [STEPS]"""
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

R = int(sys.argv[1]) if len(sys.argv) > 1 else 5
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda", 0)
n, ln = 1 << 20, 1350
ctx = sqobfs.Context(0)
kr = sqobfs.Keyring(ctx, sqobfs.SALAMANDER, [b"sing-quic-mi355x-bench-psk"])
g = torch.Generator(device=dev)
g.manual_seed(1)
data = torch.randint(0, 256, (n * ln,), generator=g, device=dev, dtype=torch.uint8)
salt = torch.randint(0, 256, (n * 8,), generator=g, device=dev, dtype=torch.uint8)
in_off = torch.arange(n, device=dev, dtype=torch.int64) * ln
out_off = torch.arange(n, device=dev, dtype=torch.int64) * (ln + 8)
lens = torch.full((n,), ln, device=dev, dtype=torch.int32)
out = torch.empty(n * (ln + 8), device=dev, dtype=torch.uint8)
out_len = torch.zeros(n, device=dev, dtype=torch.int32)
b = sqobfs.make_batch(n, data, in_off, lens, out, out_off, out_len, salt)
out2 = torch.empty_like(out)
out_len2 = torch.zeros_like(out_len)
b2 = sqobfs.make_batch(n, data, in_off, lens, out2, out_off, out_len2, salt)
stream = torch.cuda.current_stream(dev)
s = stream.cuda_stream
side = torch.cuda.Stream(dev)
s2 = side.cuda_stream
ctx.unit_packets = sqobfs.unit_packets_for(n * ln, n)

tev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
dev_ev = sqobfs.DispatchEvents(K)


def run(mode):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(K):
        if mode == "torch2":
            tev[i][0].record(stream)
            sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
            tev[i][1].record(stream)
        elif mode == "ext":
            dev_ev.arm(i)
            sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
        elif mode == "two" and i % 2:
            sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b2, s2)
        else:
            sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) / K * 1e6
    if mode == "torch2":
        kern = statistics.mean(e0.elapsed_time(e1) for e0, e1 in tev) * 1e3
    elif mode == "ext":
        kern = statistics.mean(dev_ev.elapsed_ms(i) for i in range(K)) * 1e3
    else:
        kern = float("nan")
    return wall, kern


for _ in range(80):
    sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
torch.cuda.synchronize(dev)
modes = ["torch2", "ext", "none", "two"]
res = {m: [] for m in modes}
for r in range(R):
    for m in (modes if r % 2 == 0 else modes[::-1]):
        res[m].append(run(m))
for m in modes:
    w = statistics.median(x[0] for x in res[m])
    k = statistics.median(x[1] for x in res[m])
    print(f"{m:7s} wall per step {w:7.1f} us   kernel avg {k:7.1f} us   "
          f"walls {[round(x[0], 1) for x in res[m]]}", flush=True)
dev_ev.close()
