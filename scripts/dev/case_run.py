"""Dev probe (GPU box): one obfuscation case of scripts/dev/ragged_split.py,
launched a few times in a process of its own, so that a `rocprofv3 --pmc`
pass counts that case alone (per-dispatch counters of one batch shape).
usage: case_run.py CASE [LAUNCHES]
CASE: F16 (1M x 1350 B), F4M (4M x 1350), FB16 (2,372,000 x 1350),
      P28 (1M x 758), C28 (4M x 758), R28 (configs[3]: 4M x U[64,1452]),
      F16M (configs[4] on one GPU: 16M x 1350, one PSK)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "sing-quic_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import sqobfs  # noqa: E402
import bench  # noqa: E402

CASES = {"F16": (1 << 20, 1350), "F4M": (1 << 22, 1350), "FB16": (2372000, 1350),
         "P28": (1 << 20, 758), "C28": (1 << 22, 758), "R28": (1 << 22, None),
         "F16M": (1 << 24, 1350)}
case = sys.argv[1]
launches = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n, L = CASES[case]
dev = torch.device("cuda", 0)
sh = bench.build_shard(torch, dev, 0, n, L, 1, 0, 1, "case", "dense", 0)
ctx = sqobfs.Context(0)
ctx.unit_packets = sqobfs.unit_packets_for(int(sh["payload_bytes"]), n)
kr = sqobfs.Keyring(ctx, 0, sh["psks"])
b = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"], sh["out_off"],
                      sh["out_len"], sh["salt"], sh["psk_id"])
s = torch.cuda.current_stream(dev).cuda_stream
for _ in range(launches):
    sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
torch.cuda.synchronize()
print(case, n, L, "unit", ctx.unit_packets, "launches", launches, flush=True)
ctx.close()
