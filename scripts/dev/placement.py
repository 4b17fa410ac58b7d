"""Dev probe (GPU box): does the kernel time depend on where the batch's
buffers land in HBM?  Builds configs[1] once per slot stride, then times the
obfuscation (and deobfuscation) launch on SETS fresh copies of the
input/output buffers (all kept alive), twice round-robin over every stride's
sets, 20 launches each (HIP events on the launch stream).
usage: placement.py SETS [config] [layout] [strides, e.g. "2048,1536"]
(strides apply to the slot2048 layout: bench.py --slot-bytes; the Go Slots
geometry is 2,048 B, hop.go:19).  Prints every set's time and, per stride
and direction, the median and the spread over its sets."""
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

SETS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cfg = sys.argv[2] if len(sys.argv) > 2 else "salamander-1m"
layout = sys.argv[3] if len(sys.argv) > 3 else "dense"
strides = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "2048").split(",")]
flags = {"slot2048": sqobfs.FLAG_OUT_LINES, "slot16": sqobfs.FLAG_OUT_BLOCKS}.get(layout, 0)
dev = torch.device("cuda", 0)
kind, n, L, n_psk = bench.CONFIGS[cfg]
ctx = sqobfs.Context(0)
s = torch.cuda.current_stream(dev).cuda_stream
sets = []  # (stride, k, direction, buffers, batch, keyring)
for stride in strides:
    sh = bench.build_shard(torch, dev, kind, n, L, n_psk, 0, 1, cfg, layout, 0, stride)
    kr = sqobfs.Keyring(ctx, kind, sh["psks"])
    S = sh["S"]
    for k in range(SETS):
        data = sh["data"].clone()
        out = torch.zeros_like(sh["out"])
        enc = sqobfs.make_batch(n, data, sh["in_off"], sh["lens"], out, sh["out_off"],
                                sh["out_len"], sh["salt"], sh["psk_id"], flags=flags)
        sets.append((stride, k, sqobfs.OBFUSCATE, (data, out), enc, kr))
        # decode the set's wire into its own input buffer's slots (as bench.py
        # slotted deobfuscate: payloads back in slots like the input's)
        back = torch.zeros_like(data)
        wl = (sh["lens"] + S).to(torch.int32)
        dec = sqobfs.make_batch(n, out, sh["out_off"], wl, back, sh["in_off"], sh["out_len"],
                                None, sh["psk_id"], flags=flags)
        sets.append((stride, k, sqobfs.DEOBFUSCATE, (out, back), dec, kr))


def timed(d, b, kr, steps=20):
    for _ in range(3):
        sqobfs.launch(ctx, kr, d, b, s)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for e0, e1 in ev:
        e0.record()
        sqobfs.launch(ctx, kr, d, b, s)
        e1.record()
    torch.cuda.synchronize()
    return sum(e0.elapsed_time(e1) for e0, e1 in ev) / steps * 1e3


res = {}
for rnd in range(2):
    for stride, k, d, bufs, b, kr in sets:
        t = timed(d, b, kr)
        res.setdefault((stride, d, k), []).append(t)
        print(f"round {rnd} stride {stride} set {k} {'obf' if d == 0 else 'deo'} "
              f"in 0x{bufs[0].data_ptr():x} out 0x{bufs[1].data_ptr():x} {t:8.1f} us", flush=True)
for stride in strides:
    for d in (sqobfs.OBFUSCATE, sqobfs.DEOBFUSCATE):
        per_set = [statistics.median(res[(stride, d, k)]) for k in range(SETS)]
        print(f"stride {stride} {'obfuscate' if d == 0 else 'deobfuscate'}: median "
              f"{statistics.median(per_set):8.1f} us, sets {min(per_set):.1f}-{max(per_set):.1f} "
              f"(spread {100 * (max(per_set) / min(per_set) - 1):.1f} %)", flush=True)
