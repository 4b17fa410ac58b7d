"""Minimal driver for profiling the QUIC kernels (rocprofv3 --pmc / kernel
trace): seal + open of 1M short-header packets, one key, `reps` times.
usage: python scripts/quic_prof.py [suite=1] [reps=3]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sing-quic_amd"))
import sqobfs  # noqa: E402

suite = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n, ln = 1 << 20, 1361
dev = torch.device("cuda", 0)
torch.cuda.init()
ctx = sqobfs.Context(0)
kl = 16 if suite else 32
g = torch.Generator(device=dev)
g.manual_seed(1)
data = torch.randint(0, 256, (n * ln,), generator=g, device=dev, dtype=torch.uint8)
data.view(n, ln)[:, 0] = 0x41  # short header, 2-byte packet number at offset 9
pn = torch.arange(n, device=dev, dtype=torch.int64) + 1000
data.view(n, ln)[:, 9] = ((pn >> 8) & 0xFF).to(torch.uint8)
data.view(n, ln)[:, 10] = (pn & 0xFF).to(torch.uint8)
in_off = torch.arange(n, device=dev, dtype=torch.int64) * ln
out_off = torch.arange(n, device=dev, dtype=torch.int64) * (ln + 16)
sealed = torch.zeros(n * (ln + 16), device=dev, dtype=torch.uint8)
opened = torch.zeros(n * ln, device=dev, dtype=torch.uint8)
lens = torch.full((n,), ln, device=dev, dtype=torch.int32)
slens = torch.full((n,), ln + 16, device=dev, dtype=torch.int32)
pno = torch.full((n,), 9, device=dev, dtype=torch.int16)
largest = pn - 1
olen = torch.zeros(n, device=dev, dtype=torch.int32)
olen2 = torch.zeros(n, device=dev, dtype=torch.int32)
key = sqobfs.QuicKey.of(bytes(range(kl)), bytes(12), bytes(range(kl, 2 * kl)))
s = torch.cuda.current_stream(dev).cuda_stream
with sqobfs.QuicKeyring(ctx, [key], suite) as kr:
    bs = sqobfs.quic_batch(n, data, in_off, lens, sealed, out_off, olen, pno, pn)
    bo = sqobfs.quic_batch(n, sealed, out_off, slens, opened, in_off, olen2, pno, largest)
    ts, to = [], []
    for _ in range(reps):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        sqobfs.quic_seal(ctx, kr, bs, s)
        e[1].record()
        sqobfs.quic_open(ctx, kr, bo, s)
        e[2].record()
        torch.cuda.synchronize(dev)
        ts.append(e[0].elapsed_time(e[1]) * 1e3)
        to.append(e[1].elapsed_time(e[2]) * 1e3)
    if reps > 1:
        ts, to = ts[1:], to[1:]
    print(f"seal {sum(ts) / len(ts):.1f} us  open {sum(to) / len(to):.1f} us  "
          f"lib {os.environ.get('SQOBFS_LIB', 'default')}")
ok = bool((olen == ln + 16).all()) and bool((olen2 == ln).all()) and torch.equal(opened, data)
print("quic_prof suite", suite, "round trip ok", ok)
ctx.close()
