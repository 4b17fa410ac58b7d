"""Dev probe (GPU box): does the kernel time depend on where the batch's
buffers land in HBM?  Builds configs[1] once, then times the obfuscation
launch on SETS fresh copies of the input/output buffers (all kept alive),
twice round-robin, 20 launches each (HIP events on the launch stream)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "sing-quic_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import sqobfs  # noqa: E402
import bench  # noqa: E402

SETS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cfg = sys.argv[2] if len(sys.argv) > 2 else "salamander-1m"
layout = sys.argv[3] if len(sys.argv) > 3 else "dense"
flags = {"slot2048": sqobfs.FLAG_OUT_LINES, "slot16": sqobfs.FLAG_OUT_BLOCKS}.get(layout, 0)
dev = torch.device("cuda", 0)
kind, n, L, n_psk = bench.CONFIGS[cfg]
sh = bench.build_shard(torch, dev, kind, n, L, n_psk, 0, 1, cfg, layout)
ctx = sqobfs.Context(0)
kr = sqobfs.Keyring(ctx, kind, sh["psks"])
s = torch.cuda.current_stream(dev).cuda_stream
sets = []
for k in range(SETS):
    data = sh["data"].clone()
    out = torch.zeros_like(sh["out"])
    b = sqobfs.make_batch(n, data, sh["in_off"], sh["lens"], out, sh["out_off"],
                          sh["out_len"], sh["salt"], sh["psk_id"], flags=flags)
    sets.append((data, out, b))


def timed(b, steps=20):
    for _ in range(3):
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for e0, e1 in ev:
        e0.record()
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
        e1.record()
    torch.cuda.synchronize()
    return sum(e0.elapsed_time(e1) for e0, e1 in ev) / steps * 1e3


for rnd in range(2):
    for k, (data, out, b) in enumerate(sets):
        print(f"round {rnd} set {k} in 0x{data.data_ptr():x} out 0x{out.data_ptr():x} "
              f"{timed(b):8.1f} us", flush=True)
