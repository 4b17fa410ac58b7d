"""Dev probe (GPU box): is a batch's rate set by its address range?  The
same 1M x 1350 B Salamander batch (1,415 MB of payload each way) with every
packet in a slot of STRIDE bytes, so the batch spans 1M x STRIDE bytes in
and out: 2,048 (4.3 GB in all), 4,096 (8.6 GB), 8,192 (17 GB), 16,384 (34
GB).  No batch flags (the slots' tails are written byte-exact, the same at
every stride), or SQ_STRIDE_FLAGS (8 = SQOBFS_FLAG_OUT_LINES: every output
line written whole, so no stride leaves lines written in part).  Interleaved rounds in one process, 20 timed launches each.
usage: stride_probe.py ROUNDS "STRIDE ..." """
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "sing-quic_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import sqobfs  # noqa: E402
import bench  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
strides = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2048 4096 8192").split()]
dev = torch.device("cuda", 0)
ctx = sqobfs.Context(0)
s = torch.cuda.current_stream(dev).cuda_stream
n, L = 1 << 20, 1350
ctx.unit_packets = 16
runs = []
g = torch.Generator(device=dev)
g.manual_seed(7)
kr = sqobfs.Keyring(ctx, 0, [bench.PSK])
for st in strides:
    # (built here, not by bench.build_shard: that zeroes the slot gaps through
    # index tensors of the gap size, far too large at these strides)
    data = torch.randint(0, 256, (n * st + 128,), generator=g, device=dev, dtype=torch.uint8)
    out = torch.empty(n * st + 128, device=dev, dtype=torch.uint8)
    off = torch.arange(n, device=dev, dtype=torch.int64) * st + 64
    lens = torch.full((n,), L, device=dev, dtype=torch.int32)
    salt = torch.randint(0, 256, (n * 8,), generator=g, device=dev, dtype=torch.uint8)
    out_len = torch.zeros(n, device=dev, dtype=torch.int32)
    b = sqobfs.make_batch(n, data, off + 8, lens, out, off, out_len, salt, None,
                          flags=int(os.environ.get("SQ_STRIDE_FLAGS", "0")))
    runs.append((st, (data, out), kr, b))
alg = 2 * n * L + 16 * n
for st, sh, kr, b in runs:
    for _ in range(40):
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
res = {st: [] for st in strides}
for _ in range(rounds):
    for st, sh, kr, b in runs:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(20)]
        for e0, e1 in ev:
            e0.record()
            sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
            e1.record()
        torch.cuda.synchronize()
        res[st].append(statistics.median(e0.elapsed_time(e1) * 1e3 for e0, e1 in ev))
for st in strides:
    us = statistics.median(res[st])
    print(f"stride {st:6d} span {2 * n * st / 1e9:5.1f} GB  {us:8.1f} us  frac {alg / us / 8e6:.4f}"
          f"  rounds {[round(x, 1) for x in res[st]]}", flush=True)
ctx.close()
