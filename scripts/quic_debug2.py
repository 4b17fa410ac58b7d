"""Dev: seal single-key batches of packets with payload 0..200 and report
which lengths disagree with the oracle (tag vs body)."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "sing-quic_amd")
import torch; torch.cuda.init()
import numpy as np
import test_gpu_quic as T, sqobfs, oracle_lib as ol
from sqobfs import QuicKey
rng = np.random.Generator(np.random.PCG64(1))
kb = tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (32, 12, 32))
ctx = sqobfs.Context(0)
for multi in (False, True):
    pkts = [bytes([0x41]) + bytes(8) + b"\x00\x07" + rng.integers(0, 256, pl, dtype=np.uint8).tobytes()
            for pl in range(3, 200)]
    out, oo, ol_, _, _ = T.run(ctx, [QuicKey.of(*kb)], True, pkts, [9] * len(pkts), [7] * len(pkts),
                               key_ids=[0] * len(pkts) if multi else None)
    bad = []
    for i, pk in enumerate(pkts):
        want, _ = ol.quic_seal(*kb, 7, pk, 9)
        got = out[int(oo[i]):int(oo[i]) + ol_[i]].tobytes()
        if got != want:
            bad.append((len(pk) - 11, got[:-16] == want[:-16]))
    print("multi", multi, "bad payload lengths (pl, body_ok):", bad[:60])
