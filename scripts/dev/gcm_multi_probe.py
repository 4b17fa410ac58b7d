"""Dev probe (GPU box): multi-key AES-128-GCM seal / open cost by key layout,
against the single-key kernel, on bench.py --quic's 1M x 1361 B batch (one
process, one buffer set, median of rounds; the time includes the key
grouping's kernels).
  single     no key ids (round keys in the kernarg segment)
  one_id     key ids all 0 (grouped, staged: the staged kernel's own cost)
  blocks16   16 keys in contiguous runs (kid = i * 16 / n)
  mod16      16 keys interleaved (kid = i mod 16, bench.py --quic's case)
  mod16_2k   the same, 2,047-packet launches' worth ungrouped (n < 2,048 is
             never grouped: here the whole batch through the per-packet
             kernel, by a keyring of 1,100 keys -- over the grouping limit)
usage: gcm_multi_probe.py [ROUNDS]"""
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "sing-quic_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import sqobfs  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
n, ln = 1 << 20, 11 + 1350
rng = np.random.Generator(np.random.PCG64(12))
ctx = sqobfs.Context(0)
in_off = torch.arange(n, device=dev, dtype=torch.int64) * ln
out_off = torch.arange(n, device=dev, dtype=torch.int64) * (ln + 16)
g = torch.Generator(device=dev)
g.manual_seed(5)
data = torch.randint(0, 256, (n * ln,), generator=g, device=dev, dtype=torch.uint8)
data.view(n, ln)[:, 0] = 0x41
pn = torch.arange(n, device=dev, dtype=torch.int64) + 1000
data.view(n, ln)[:, 9] = ((pn >> 8) & 0xFF).to(torch.uint8)
data.view(n, ln)[:, 10] = (pn & 0xFF).to(torch.uint8)
sealed = torch.zeros(n * (ln + 16), device=dev, dtype=torch.uint8)
opened = torch.zeros(n * ln, device=dev, dtype=torch.uint8)
lens = torch.full((n,), ln, device=dev, dtype=torch.int32)
slens = torch.full((n,), ln + 16, device=dev, dtype=torch.int32)
pno = torch.full((n,), 9, device=dev, dtype=torch.int16)
olen = torch.zeros(n, device=dev, dtype=torch.int32)
pn_out = torch.zeros(n, device=dev, dtype=torch.int64)
s = torch.cuda.current_stream(dev).cuda_stream
keys = [sqobfs.QuicKey.of(*(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (16, 12, 16)))
        for _ in range(1100)]
ar = torch.arange(n, device=dev, dtype=torch.int64)
layouts = [("single", None, 1), ("one_id", torch.zeros(n, device=dev, dtype=torch.int16), 1),
           ("blocks16", (ar * 16 // n).to(torch.int16), 16), ("mod16", (ar % 16).to(torch.int16), 16),
           ("mod16_ungrouped", (ar % 16).to(torch.int16), 1100)]
krs = {k: sqobfs.QuicKeyring(ctx, keys[:k], sqobfs.QUIC_AES_128_GCM) for k in (1, 16, 1100)}
variants = []
for name, kid, nk in layouts:
    bs = sqobfs.quic_batch(n, data, in_off, lens, sealed, out_off, olen, pno, pn, key_id=kid)
    bo = sqobfs.quic_batch(n, sealed, out_off, slens, opened, in_off, olen, pno, pn - 1, key_id=kid,
                           pn_out=pn_out)
    variants.append((name + "/seal", sqobfs.quic_seal, krs[nk], bs))
    variants.append((name + "/open", sqobfs.quic_open, krs[nk], bo))


def timed(v, steps=5):
    _, fn, kr, b = v
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn(ctx, kr, b, s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps * 1e3


for v in variants:  # (seal before open: open reads the sealed packets)
    timed(v, 2)
res = {v[0]: [] for v in variants}
for _ in range(R):
    for v in variants:
        res[v[0]].append(timed(v))
for v in variants:
    print(f"{v[0]:24s} median {statistics.median(res[v[0]]):8.1f} us  all "
          f"{[round(x, 1) for x in res[v[0]]]}", flush=True)
