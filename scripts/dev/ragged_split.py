"""Dev probe (GPU box): where configs[3]'s ragged batch loses time against
configs[1], in ONE process on one box, interleaved rounds.

Cases (dense wire layout, Salamander, one PSK, as bench.py builds them):
  F16   configs[1]: 1M x 1350 B at its default unit (16 packets per wave)
  R<u>  configs[3]: 4M x U[64,1452] (mean 758) at its default unit (28)
  C<u>  4M x 758 B constant (same mean) at the ragged default unit
  FB16  2,372,000 x 1350 B at 16: configs[1]'s packets with configs[3]'s
        footprint (the same input and output bytes)
  P<u>  1M x 758 B at the ragged unit: configs[3]'s packets per byte with a
        footprint near configs[1]'s
  B<u>  the ragged lengths reordered inside every run of 4096 packets as
        shortest, longest, 2nd shortest, 2nd longest, ...: the same lengths
        and packets per byte, but every unit holds nearly the same bytes
        (R's unit bytes vary ~10 %)
R vs C separates length variance from the per-packet fixed cost (same
packets per byte); FB16 and P vs F16 separate the footprint (address
translation) from the packets per byte.
usage: ragged_split.py DIRECTION ROUNDS lib1.so [lib2.so ...]
Prints per lib and case the median kernel time, ns per KiB of algorithmic
bytes and frac of 8 TB/s; every lib's output of a case is compared with the
first lib's."""
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

direction, rounds = sys.argv[1], int(sys.argv[2])
paths = sys.argv[3:]
dev = torch.device("cuda", 0)
S = 8
PSK = bench.PSK
s = torch.cuda.current_stream(dev).cuda_stream


def shard(lens):
    """Dense wire layout (bench.build_shard's): payload behind S bytes of
    headroom in a wire-sized input slot; outputs back to back."""
    n = lens.numel()
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    l64 = lens.to(torch.int64)
    w = l64 + S
    out_off = torch.cumsum(w, 0) - w + 64
    in_off = out_off + S
    nbytes = int(w.sum().item()) + 256
    data = torch.randint(0, 256, (nbytes,), generator=g, device=dev, dtype=torch.uint8)
    salt = torch.randint(0, 256, (n * S,), generator=g, device=dev, dtype=torch.uint8)
    out = torch.zeros(nbytes, device=dev, dtype=torch.uint8)
    out_len = torch.zeros(n, device=dev, dtype=torch.int32)
    lens32 = lens.to(torch.int32)
    pay = int(l64.sum().item())
    enc = sqobfs.make_batch(n, data, in_off, lens32, out, out_off, out_len, salt)
    alg = 2 * pay + 2 * S * n
    if direction == "obfuscate":
        return dict(n=n, pay=pay, b=enc, out=out, alg=alg, enc=enc)
    back_off = torch.cumsum(l64, 0) - l64 + 64
    back = torch.zeros(pay + 128, device=dev, dtype=torch.uint8)
    dec = sqobfs.make_batch(n, out, out_off, (lens + S).to(torch.int32), back, back_off, out_len,
                            None)
    return dict(n=n, pay=pay, b=dec, out=back, alg=2 * pay + S * n, enc=enc)


g = torch.Generator(device=dev)
g.manual_seed(4)
n4 = 1 << 22
ragged = torch.randint(64, 1453, (n4,), generator=g, device=dev, dtype=torch.int64)
srt = ragged.view(-1, 4096).sort(dim=1).values
bal = torch.stack([srt[:, :2048], srt[:, 2048:].flip(1)], dim=2).reshape(-1)
const = torch.full((n4,), 758, device=dev, dtype=torch.int64)
fixed = torch.full((1 << 20,), 1350, device=dev, dtype=torch.int64)
fbig = torch.full((2372000,), 1350, device=dev, dtype=torch.int64)
p758 = torch.full((1 << 20,), 758, device=dev, dtype=torch.int64)
sqobfs._lib = sqobfs.load(paths[0])
u_r = sqobfs.unit_packets_for(int(ragged.sum().item()), n4)
cases = [("F16", fixed, 0), (f"R{u_r}", ragged, u_r), (f"C{u_r}", const, u_r),
         ("FB16", fbig, 16), (f"P{u_r}", p758, u_r), (f"B{u_r}", bal, u_r)]
if os.environ.get("SPLIT_CASES") == "ladder":
    # the per-byte rate against the batch's packet count, for both lengths
    # (a size ladder: 1M, 2M / 2.37M, 4M packets)
    del ragged, srt, bal, const, fbig
    cases = [("F1M", fixed, 16),
             ("F2.4M", torch.full((2372000,), 1350, device=dev, dtype=torch.int64), 16),
             ("F4M", torch.full((n4,), 1350, device=dev, dtype=torch.int64), 16),
             ("P1M", p758, u_r),
             ("P2M", torch.full((1 << 21,), 758, device=dev, dtype=torch.int64), u_r),
             ("P4M", torch.full((n4,), 758, device=dev, dtype=torch.int64), u_r)]
bufs = {}
for name, lens, u in cases:
    key = id(lens)
    if key not in bufs:
        bufs[key] = shard(lens)
variants = []
for path in paths:
    lib = sqobfs.load(path)
    sqobfs._lib = lib
    ctx = sqobfs.Context(0)
    kr = sqobfs.Keyring(ctx, 0, [PSK])
    variants.append((os.path.basename(path), lib, ctx, kr))
d = sqobfs.OBFUSCATE if direction == "obfuscate" else sqobfs.DEOBFUSCATE


def launch(v, sh, u):
    sqobfs._lib = v[1]
    v[2].unit_packets = u or sqobfs.unit_packets_for(sh["pay"], sh["n"])
    sqobfs.launch(v[2], v[3], d, sh["b"], s)


def timed(v, sh, u, steps=15):
    for _ in range(2):
        launch(v, sh, u)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        launch(v, sh, u)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps * 1e3


# wire made once by the first lib (deobfuscate decodes it); parity of libs
for name, lens, u in cases:
    sh = bufs[id(lens)]
    if d == sqobfs.DEOBFUSCATE:
        sqobfs._lib = variants[0][1]
        variants[0][2].unit_packets = u or 16
        sqobfs.launch(variants[0][2], variants[0][3], sqobfs.OBFUSCATE, sh["enc"], s)
    ref = None
    for v in variants:
        sh["out"].zero_()
        launch(v, sh, u)
        torch.cuda.synchronize()
        if ref is None:
            ref = sh["out"].clone()
        elif not torch.equal(ref, sh["out"]):
            print(f"parity FAIL {name} {v[0]} vs {variants[0][0]}", flush=True)
            sys.exit(1)
    del ref
print("parity of the libs: ok", flush=True)
res = {(v[0], c[0]): [] for v in variants for c in cases}
for r in range(rounds):
    for v in (variants if r % 2 == 0 else variants[::-1]):
        for name, lens, u in cases:
            res[(v[0], name)].append(timed(v, bufs[id(lens)], u))
    print(f"round {r} done", flush=True)
for v in variants:
    for name, lens, u in cases:
        sh = bufs[id(lens)]
        med = statistics.median(res[(v[0], name)])
        print(f"{direction[:3]} {v[0]:22s} {name:5s} n {sh['n']:8d} ppw {u or 16:2d} "
              f"median {med:8.1f} us  {med * 1e3 / (sh['alg'] / 1024):6.2f} ns/KiB  "
              f"frac {sh['alg'] / med / 8e6:.4f}", flush=True)
