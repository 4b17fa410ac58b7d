"""Dev probe (GPU box): time per launch vs unit size (packets per wavefront)
in ONE process on one buffer set, interleaved rounds, event-free timed
loops (wall clock, sync-bracketed); every unit's output compared byte for
byte with the first's.
usage: unit_probe.py KIND(0 salamander, 1 xplus) DIR(0 obf, 1 deobf) LEN|ragged "PPW list" [ROUNDS]"""
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

kind, direction = int(sys.argv[1]), int(sys.argv[2])
ragged = sys.argv[3] == "ragged"
ppws = [int(x) for x in sys.argv[4].split()]
R = int(sys.argv[5]) if len(sys.argv) > 5 else 5
K = 20
dev = torch.device("cuda", 0)
S = 8 if kind == 0 else 16
n = (1 << 22) if ragged else (1 << 20)
g = torch.Generator(device=dev)
g.manual_seed(4)
if ragged:
    lens = torch.randint(64, 1453, (n,), generator=g, device=dev, dtype=torch.int32)
else:
    lens = torch.full((n,), int(sys.argv[3]), device=dev, dtype=torch.int32)
l64 = lens.to(torch.int64)
in_off = torch.cumsum(l64, 0) - l64
wire_len = (lens + S).to(torch.int32)
w64 = wire_len.to(torch.int64)
out_off = torch.cumsum(w64, 0) - w64
tot, wtot = int(l64.sum()), int(w64.sum())
data = torch.randint(0, 256, (tot + 64,), generator=g, device=dev, dtype=torch.uint8)
salt = torch.randint(0, 256, (n * S,), generator=g, device=dev, dtype=torch.uint8)
wire = torch.zeros(wtot + 64, device=dev, dtype=torch.uint8)
back = torch.zeros(tot + 64, device=dev, dtype=torch.uint8)
out_len = torch.zeros(n, device=dev, dtype=torch.int32)
ctx = sqobfs.Context(0)
kr = sqobfs.Keyring(ctx, kind, [b"sing-quic-mi355x-bench-psk"])
s = torch.cuda.current_stream(dev).cuda_stream
enc = sqobfs.make_batch(n, data, in_off, lens, wire, out_off, out_len, salt)
ctx.unit_packets = sqobfs.unit_packets_for(tot, n)
sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, enc, s)
torch.cuda.synchronize(dev)
if direction == 0:
    b, out = enc, wire
else:
    b, out = sqobfs.make_batch(n, wire, out_off, wire_len, back, in_off, out_len, None), back


def run(ppw, steps):
    ctx.unit_packets = ppw
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        sqobfs.launch(ctx, kr, direction, b, s)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps * 1e6


ref = None
for w in ppws:
    run(w, 30)
    got = out.clone()
    if ref is None:
        ref = got
    assert torch.equal(got, ref), f"ppw {w}: output differs"
res = {w: [] for w in ppws}
for r in range(R):
    for w in (ppws if r % 2 == 0 else ppws[::-1]):
        res[w].append(run(w, K))
print(f"kind {kind} dir {direction} {'ragged' if ragged else sys.argv[3]} n {n}, default unit "
      f"{sqobfs.unit_packets_for(tot, n)}")
for w in ppws:
    print(f"  ppw {w:3d}  median {statistics.median(res[w]):8.1f} us  all {[round(x, 1) for x in res[w]]}",
          flush=True)
