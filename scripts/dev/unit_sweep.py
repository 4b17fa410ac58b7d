"""Dev probe (GPU box): kernel time vs unit size (packets per wavefront) in
ONE process on ONE buffer set, interleaved rounds, so that box and
allocation effects cancel, after a 60-launch warm-up (the GPU's first
~25 launches of a process run up to 10 % slower).
usage: unit_sweep.py CONFIG "ppw ..." [ROUNDS] [obfuscate|deobfuscate]
Tokens PPW[uU][lP][wW] (e.g. 16u6, 16u4l10240, 16w1) also set
SQOBFS_DEV_U=U, SQOBFS_DEV_LDSPAD=P and SQOBFS_DEV_WPB=W (timing builds with
SQ_DEVVAR: stream step of U blocks per lane, P bytes of extra LDS per
workgroup, W waves per workgroup).  SWEEP_LAYOUT=slot16 runs bench.py's
16-byte-slot layout (SQOBFS_FLAG_OUT_BLOCKS) instead of the dense one."""
import os
import re
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "sing-quic_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import sqobfs  # noqa: E402
import bench  # noqa: E402

cfg = sys.argv[1]
ppws = sys.argv[2].split()
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
deo = len(sys.argv) > 4 and sys.argv[4] == "deobfuscate"
dev = torch.device("cuda", 0)
kind, n, L, n_psk = bench.CONFIGS[cfg]
layout = os.environ.get("SWEEP_LAYOUT", "dense")
sh = bench.build_shard(torch, dev, kind, n, L, n_psk, 0, 1, cfg, layout)
ob = sqobfs.FLAG_OUT_BLOCKS if sh["slotted"] else 0
ctx = sqobfs.Context(0)
kr = sqobfs.Keyring(ctx, kind, sh["psks"])
s = torch.cuda.current_stream(dev).cuda_stream
b = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"], sh["out_off"],
                      sh["out_len"], sh["salt"], sh["psk_id"], flags=ob)
d = sqobfs.OBFUSCATE
alg = 2 * sh["payload_bytes"] + 2 * sh["S"] * n
if deo:
    sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
    wl = (sh["lens"] + sh["S"]).to(torch.int32)
    lens64 = sh["lens"].to(torch.int64)
    if sh["slotted"]:  # decoded payloads into slots like the input's (as bench.py)
        back_off, back = sh["in_off"], torch.zeros_like(sh["data"])
    else:
        back_off = torch.cumsum(lens64, 0) - lens64 + 64
        back = torch.zeros(int(sh["payload_bytes"]) + 128, device=dev, dtype=torch.uint8)
    b = sqobfs.make_batch(n, sh["out"], sh["out_off"], wl, back, back_off, sh["out_len"], None,
                          sh["psk_id"], flags=ob)
    d = sqobfs.DEOBFUSCATE
    alg = 2 * sh["payload_bytes"] + sh["S"] * n


def timed(steps=15):
    for _ in range(2):
        sqobfs.launch(ctx, kr, d, b, s)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for e0, e1 in ev:
        e0.record()
        sqobfs.launch(ctx, kr, d, b, s)
        e1.record()
    torch.cuda.synchronize()
    return sum(e0.elapsed_time(e1) for e0, e1 in ev) / steps * 1e3


res = {w: [] for w in ppws}
for _ in range(60):
    sqobfs.launch(ctx, kr, d, b, s)
torch.cuda.synchronize()
for r in range(rounds):
    for w in ppws:
        m = re.fullmatch(r"(\d+)(?:u(\d+))?(?:l(\d+))?(?:w(\d+))?", w)
        ctx.unit_packets = int(m.group(1))
        os.environ["SQOBFS_DEV_U"] = m.group(2) or "4"
        os.environ["SQOBFS_DEV_LDSPAD"] = m.group(3) or "0"
        os.environ["SQOBFS_DEV_WPB"] = m.group(4) or "0"
        res[w].append(round(timed(), 1))
    print(f"round {r} done", flush=True)
for w in ppws:
    med = statistics.median(res[w])
    print(f"{cfg:24s} {layout} {'deo' if deo else 'obf'} ppw {w:>4s} median {med:8.1f} us  frac {alg / med / 8e6:.3f}  all {res[w]}")
