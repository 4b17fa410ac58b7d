import sys, json
sys.path.insert(0, "tests"); sys.path.insert(0, "sing-quic_amd")
import torch; torch.cuda.init()
import test_gpu_quic as T, sqobfs
from sqobfs import QuicKey
B = bytes.fromhex
g = json.load(open("tests/golden/quic.json"))["packets"]
ctx = sqobfs.Context(0)
keys = [QuicKey.of(B(v["key"]), B(v["iv"]), B(v["hp"])) for v in g]
pkts = [B(v["packet"]) for v in g]
out, oo, ol_, _, _ = T.run(ctx, keys, True, pkts, [v["pn_offset"] for v in g], [v["pn"] for v in g], key_ids=list(range(len(g))))
for i, v in enumerate(g):
    pkt = pkts[i]; hdr = v["pn_offset"] + (pkt[0] & 3) + 1; pl = len(pkt) - hdr
    got = out[int(oo[i]):int(oo[i]) + ol_[i]].tobytes().hex()
    ok = got == v["protected"]
    body_ok = got[:-32] == v["protected"][:-32]
    print(i, "ok" if ok else "BAD", "body_ok", body_ok, "hdr", hdr, "pl", pl, "nblk", (pl + 63) // 64, "klast", ((pl - 64 * max(0, (pl + 63) // 64 - 1)) + 15) // 16)
