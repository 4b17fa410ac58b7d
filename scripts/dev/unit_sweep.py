"""Dev probe (GPU box): kernel time vs unit size (packets per wavefront) in
ONE process on ONE buffer set, interleaved rounds, so that box and
allocation effects cancel.  usage: unit_sweep.py CONFIG "ppw ..." [ROUNDS]"""
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

cfg = sys.argv[1]
ppws = [int(x) for x in sys.argv[2].split()]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda", 0)
kind, n, L, n_psk = bench.CONFIGS[cfg]
sh = bench.build_shard(torch, dev, kind, n, L, n_psk, 0, 1, cfg, "dense")
ctx = sqobfs.Context(0)
kr = sqobfs.Keyring(ctx, kind, sh["psks"])
s = torch.cuda.current_stream(dev).cuda_stream
b = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"], sh["out_off"],
                      sh["out_len"], sh["salt"], sh["psk_id"])


def timed(steps=15):
    for _ in range(2):
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for e0, e1 in ev:
        e0.record()
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
        e1.record()
    torch.cuda.synchronize()
    return sum(e0.elapsed_time(e1) for e0, e1 in ev) / steps * 1e3


res = {w: [] for w in ppws}
for r in range(rounds):
    for w in ppws:
        ctx.unit_packets = w
        res[w].append(round(timed(), 1))
    print(f"round {r} done", flush=True)
alg = 2 * sh["payload_bytes"] + 2 * sh["S"] * n
for w in ppws:
    med = statistics.median(res[w])
    print(f"{cfg:24s} ppw {w:3d} median {med:8.1f} us  frac {alg / med / 8e6:.3f}  all {res[w]}")
