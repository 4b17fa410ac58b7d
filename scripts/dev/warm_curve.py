"""Dev probe (GPU box): per-launch kernel time over a long run, per unit
size, in one process (is there a warm-up, and does it depend on the unit
size?).  usage: warm_curve.py CONFIG "ppw ..." [LAUNCHES]"""
import os
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
launches = int(sys.argv[3]) if len(sys.argv) > 3 else 100
dev = torch.device("cuda", 0)
kind, n, L, n_psk = bench.CONFIGS[cfg]
sh = bench.build_shard(torch, dev, kind, n, L, n_psk, 0, 1, cfg, "dense")
ctx = sqobfs.Context(0)
kr = sqobfs.Keyring(ctx, kind, sh["psks"])
s = torch.cuda.current_stream(dev).cuda_stream
b = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"], sh["out_off"],
                      sh["out_len"], sh["salt"], sh["psk_id"])
for w in ppws:
    ctx.unit_packets = w
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(launches)]
    for e0, e1 in ev:
        e0.record()
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
        e1.record()
    torch.cuda.synchronize()
    us = [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
    blocks = [round(sum(us[i:i + 10]) / len(us[i:i + 10]), 1) for i in range(0, launches, 10)]
    print(f"{cfg} ppw {w:3d} per-10 avg us: {blocks}", flush=True)
