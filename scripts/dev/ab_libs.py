"""Dev probe (GPU box): kernel time of several libsqobfs builds in ONE process
on ONE buffer set, interleaved rounds (box and allocation effects cancel).
usage: ab_libs.py CONFIG DIRECTION ROUNDS lib1.so lib2.so ...
Prints per lib the median kernel time and frac of 8 TB/s, and checks every
build's output against the first one's (parity of the variants).
AB_KR=k: k contexts + keyrings per build (keyring tables at k different
addresses; per-instance medians are printed, the build's median is over all).
AB_FLAGS="4,8" with one library: one variant per batch flag set instead
(slotted layouts: SQOBFS_FLAG_OUT_BLOCKS = 4 vs SQOBFS_FLAG_OUT_LINES = 8)."""
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

cfg, direction, rounds = sys.argv[1], sys.argv[2], int(sys.argv[3])
paths = sys.argv[4:]
dev = torch.device("cuda", 0)
kind, n, L, n_psk = bench.CONFIGS[cfg]
n = int(os.environ.get("AB_PACKETS", "0")) or n  # (dev: another batch size)
layout = os.environ.get("AB_LAYOUT", "dense")
sh = bench.build_shard(torch, dev, kind, n, L, n_psk, 0, 1, cfg, layout)
S = sh["S"]
ob = sqobfs.FLAG_OUT_BLOCKS if sh["slotted"] else 0
ob = int(os.environ.get("AB_OB", ob))  # (e.g. 8: SQOBFS_FLAG_OUT_LINES for slot2048)
s = torch.cuda.current_stream(dev).cuda_stream
variants = []
# AB_PPWS="18,20,..." with one library: one variant per unit size instead
ppws = [int(x) for x in os.environ.get("AB_PPWS", "").split(",") if x]
fsets = [int(x) for x in os.environ.get("AB_FLAGS", "").split(",") if x]
specs = [(paths[0], u) for u in ppws] if ppws else [(p, 0) for p in paths]
if fsets:
    specs = [(paths[0], -f - 1) for f in fsets]  # (negative: a flag set, default unit)
specs = specs * int(os.environ.get("AB_KR", "1"))
loaded = {}
for path, u in specs:
    if path not in loaded:
        loaded[path] = sqobfs.load(path)
    sqobfs._lib = loaded[path]
    ctx = sqobfs.Context(0)
    kr = sqobfs.Keyring(ctx, kind, sh["psks"])
    fl = -u - 1 if u < 0 else None
    u = max(u, 0)
    ctx.unit_packets = u or int(os.environ.get("AB_PPW", "0")) or sqobfs.unit_packets_for(
        sh["payload_bytes"], n, n_psk > 1)
    name = f"{path}@ppw{ctx.unit_packets}" if ppws else (f"{path}@flags{fl}" if fsets else path)
    variants.append((name, sqobfs._lib, ctx, kr, fl))
names = list(dict.fromkeys(v[0] for v in variants))
b = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"], sh["out_off"],
                      sh["out_len"], sh["salt"], sh["psk_id"], flags=ob)
d = sqobfs.OBFUSCATE
mk = lambda fl: sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"],  # noqa
                                  sh["out_off"], sh["out_len"], sh["salt"], sh["psk_id"], flags=fl)
alg = 2 * sh["payload_bytes"] + 2 * S * n
outs = []
if direction == "deobfuscate":
    sqobfs._lib = variants[0][1]
    sqobfs.launch(variants[0][2], variants[0][3], sqobfs.OBFUSCATE, b, s)
    wl = (sh["lens"] + S).to(torch.int32)
    lens64 = sh["lens"].to(torch.int64)
    if sh["slotted"]:  # decoded into slots like the input's (as bench.py)
        back_off = sh["in_off"]
        back = torch.zeros_like(sh["data"])
    else:
        back_off = torch.cumsum(lens64, 0) - lens64 + 64
        back = torch.zeros(int(sh["payload_bytes"]) + 128, device=dev, dtype=torch.uint8)
    b = sqobfs.make_batch(n, sh["out"], sh["out_off"], wl, back, back_off, sh["out_len"], None,
                          sh["psk_id"], flags=ob)
    mk = lambda fl: sqobfs.make_batch(n, sh["out"], sh["out_off"], wl, back, back_off,  # noqa
                                      sh["out_len"], None, sh["psk_id"], flags=fl)
    d = sqobfs.DEOBFUSCATE
    alg = 2 * sh["payload_bytes"] + S * n
    outs = [back]
else:
    outs = [sh["out"]]
# per variant: its batch (its own flag set, or the layout's)
variants = [v[:4] + (mk(v[4]) if v[4] is not None else b,) for v in variants]


def timed(v, steps=15):
    sqobfs._lib = v[1]
    for _ in range(2):
        sqobfs.launch(v[2], v[3], d, v[4], s)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for e0, e1 in ev:
        e0.record()
        sqobfs.launch(v[2], v[3], d, v[4], s)
        e1.record()
    torch.cuda.synchronize()
    return sum(e0.elapsed_time(e1) for e0, e1 in ev) / steps * 1e3


# parity of the variants: each one's output equals the first's
ref = cov = None
for v in variants:
    sqobfs._lib = v[1]
    outs[0].zero_()
    sqobfs.launch(v[2], v[3], d, v[4], s)
    torch.cuda.synchronize()
    if ref is None:
        ref = outs[0].clone()
    if ref is not None and fsets and cov is None:
        # (flag variants: only the packets' output bytes are specified)
        cov = torch.zeros_like(ref, dtype=torch.bool)
        offs = (back_off if direction == "deobfuscate" else sh["out_off"]).to(torch.int64)
        olen = (sh["lens"] if direction == "deobfuscate" else sh["lens"] + S).to(torch.int64)
        idx = torch.repeat_interleave(offs, olen) + (
            torch.arange(int(olen.sum().item()), device=dev)
            - torch.repeat_interleave(torch.cumsum(olen, 0) - olen, olen))
        cov[idx] = True
        del idx
    if v is not variants[0]:
        same = (not bool(((ref != outs[0]) & cov).any().item())) if fsets else torch.equal(ref, outs[0])
        print(f"parity {os.path.basename(v[0])} vs {os.path.basename(variants[0][0])}: {same}",
              flush=True)
        if not same and not os.environ.get("AB_NOPARITY"):  # (ablation builds: timing only)
            sys.exit(1)
for v in variants:
    sqobfs._lib = v[1]
    for _ in range(40):
        sqobfs.launch(v[2], v[3], d, v[4], s)
torch.cuda.synchronize()
res = {nm: [] for nm in names}
inst = [[] for _ in variants]
for r in range(rounds):
    for i, v in enumerate(variants):
        t = round(timed(v), 1)
        res[v[0]].append(t)
        inst[i].append(t)
if len(variants) > len(names):
    for i, v in enumerate(variants):
        print(f"  instance {i} {os.path.basename(v[0])}: median {statistics.median(inst[i]):8.1f}",
              flush=True)
for nm in names:
    med = statistics.median(res[nm])
    print(f"{cfg:24s} {direction[:3]} {os.path.basename(nm):24s} median {med:8.1f} us  "
          f"frac {alg / med / 8e6:.4f}  all {res[nm]}", flush=True)
