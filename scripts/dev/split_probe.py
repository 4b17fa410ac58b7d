"""Dev probe (GPU box): does a large batch run faster as several back-to-back
launches over slices of it?  Per case (scripts/dev/case_run.py's), on the
same buffers in one process: the whole batch as one launch against K
launches of n/K packets each (the descriptor arrays sliced; host salts),
interleaved over ROUNDS rounds of 20 timed steps (HIP events on the launch
stream around each step), after a 60-launch warm-up.
usage: split_probe.py ROUNDS "K1 K2 ..." [cases ...]"""
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

CASES = {"F16": (1 << 20, 1350), "F4M": (1 << 22, 1350), "FB16": (2372000, 1350),
         "P28": (1 << 20, 758), "C28": (1 << 22, 758), "R28": (1 << 22, None)}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
splits = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1 2 4").split()]
cases = sys.argv[3:] or ["F16", "FB16", "F4M", "C28", "R28"]
dev = torch.device("cuda", 0)
ctx = sqobfs.Context(0)
s = torch.cuda.current_stream(dev).cuda_stream
for case in cases:
    n, L = CASES[case]
    sh = bench.build_shard(torch, dev, 0, n, L, 1, 0, 1, "case", "dense", 0)
    kr = sqobfs.Keyring(ctx, 0, sh["psks"])
    S = sh["S"]
    alg = 2 * int(sh["payload_bytes"]) + 2 * S * n
    ctx.unit_packets = sqobfs.unit_packets_for(int(sh["payload_bytes"]), n)
    batches = {}
    for k in splits:
        cuts = [n * i // k for i in range(k + 1)]
        bl = []
        for a, b in zip(cuts[:-1], cuts[1:]):
            bl.append(sqobfs.make_batch(b - a, sh["data"], sh["in_off"][a:b], sh["lens"][a:b],
                                        sh["out"], sh["out_off"][a:b], sh["out_len"][a:b],
                                        sh["salt"][a * S:b * S], None))
        batches[k] = bl
    for _ in range(60):
        for b in batches[splits[0]]:
            sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
    res = {k: [] for k in splits}
    for _ in range(rounds):
        for k in splits:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(20)]
            for e0, e1 in ev:
                e0.record()
                for b in batches[k]:
                    sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
                e1.record()
            torch.cuda.synchronize()
            res[k].append(statistics.median(e0.elapsed_time(e1) * 1e3 for e0, e1 in ev))
    for k in splits:
        us = statistics.median(res[k])
        print(f"{case:5s} n {n:8d} unit {ctx.unit_packets:2d} split {k:2d} step {us:8.1f} us "
              f"frac {alg / us / 8e6:.4f}  rounds {[round(x, 1) for x in res[k]]}", flush=True)
    del batches, sh, kr
    torch.cuda.empty_cache()
ctx.close()
