"""Dev probe (GPU box): QUIC multi-key kernels vs how the batch's key ids are
ordered.  1M short-header packets (1 + 8-byte DCID + 2-byte pn + 1350 B),
16 keys; key_id patterns: one key (single-key kernel), i mod 16 (every wave
sees all keys), runs of 32 / 1024 packets (one key per wave).  Seal then
open, median of the interleaved rounds, both suites.
usage: quic_keyorder.py [rounds=3]"""
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "sing-quic_amd"))
import sqobfs  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n, payload, nk = 1 << 20, 1350, 16
ln = 11 + payload
dev = torch.device("cuda", 0)
ctx = sqobfs.Context(0)
s = torch.cuda.current_stream(dev).cuda_stream
g = torch.Generator(device=dev)
g.manual_seed(5)
data = torch.randint(0, 256, (n * ln,), generator=g, device=dev, dtype=torch.uint8)
data.view(n, ln)[:, 0] = 0x41
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
i = torch.arange(n, device=dev, dtype=torch.int64)
patterns = {"one key": None, "i mod 16": i % nk, "runs of 32": (i // 32) % nk,
            "runs of 1024": (i // 1024) % nk}


def timed(fn, b, kr, steps=6):
    for _ in range(2):
        fn(ctx, kr, b, s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn(ctx, kr, b, s)
    e1.record()
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / steps * 1e3


for suite in (0, 1):
    kl = 16 if suite else 32
    rng = np.random.Generator(np.random.PCG64(77))
    keys = [sqobfs.QuicKey.of(*(rng.integers(0, 256, m, dtype=np.uint8).tobytes()
                                for m in (kl, 12, kl))) for _ in range(nk)]
    res = {k: {"seal": [], "open": []} for k in patterns}
    with sqobfs.QuicKeyring(ctx, keys[:1], suite) as k1, sqobfs.QuicKeyring(ctx, keys, suite) as km:
        for _ in range(rounds):
            for name, kid in patterns.items():
                kr = k1 if kid is None else km
                kid16 = None if kid is None else kid.to(torch.int16)
                bs = sqobfs.quic_batch(n, data, in_off, lens, sealed, out_off, olen, pno, pn,
                                       key_id=kid16)
                bo = sqobfs.quic_batch(n, sealed, out_off, slens, opened, in_off, olen2, pno,
                                       largest, key_id=kid16)
                res[name]["seal"].append(timed(sqobfs.quic_seal, bs, kr))
                res[name]["open"].append(timed(sqobfs.quic_open, bo, kr))
                ok = bool((olen == ln + 16).all()) and bool((olen2 == ln).all()) and \
                    torch.equal(opened, data)
                assert ok, (suite, name)
    for name in patterns:
        print(f"suite {'aes-128-gcm' if suite else 'chacha20-poly1305':18s} {name:13s} "
              f"seal {statistics.median(res[name]['seal']):8.1f} us  "
              f"open {statistics.median(res[name]['open']):8.1f} us", flush=True)
ctx.close()
