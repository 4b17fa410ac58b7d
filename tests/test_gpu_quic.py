"""QUIC packet protection on the GPU (sqobfs_quic_seal / _open,
AEAD_CHACHA20_POLY1305 + ChaCha20 header protection) against the CPU oracle
and the committed vectors: RFC 9001 Appendix A.5 and OpenSSL-built packets
(tests/golden/quic.json).  Bit-exact on every output byte, including the
bytes around each packet, and on out_len / decoded packet numbers."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import QuicKey

import oracle_lib as ol

pytestmark = pytest.mark.gpu
B = bytes.fromhex
SENT = 0x5A


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    c = sqobfs.Context(0)
    yield c
    c.close()


def _place(sizes, align, gap):
    offs, pos = [], 64
    for sz in sizes:
        offs.append(pos)
        pos = (pos + sz + gap + align - 1) // align * align
    return np.array(offs, np.uint64), pos + 64


def run(ctx, keys, seal, pkts, pn_offsets, pns, key_ids=None, align=1, inplace=False,
        suite=0, pn_out_fill=0, ctx_stream=False):
    """One device batch; returns (out buffer, out offsets, out_len, pn_out).
    ctx_stream: launched on the context's own stream (stream NULL) instead of
    torch's current one."""
    import torch
    dev = torch.device("cuda", 0)
    n = len(pkts)
    grow = 16 if seal else 0
    in_off, end = _place([len(p) + grow for p in pkts], align, 3)
    data = np.full(end, SENT, np.uint8)
    for o, p in zip(in_off, pkts):
        data[int(o):int(o) + len(p)] = np.frombuffer(p, np.uint8)
    if inplace:
        out_off = in_off.copy()
        out = data
    else:
        out_off, oend = _place([len(p) + grow for p in pkts], align, 5)
        out = np.full(oend, SENT, np.uint8)
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa
    d_data = t(data)
    d_out = d_data if inplace else t(out)
    d = dict(in_off=t(in_off), in_len=t(np.array([len(p) for p in pkts], np.uint32)),
             out_off=t(out_off), out_len=t(np.zeros(n, np.uint32)),
             pno=t(np.asarray(pn_offsets, np.uint16)), pn=t(np.asarray(pns, np.uint64)),
             kid=t(None if key_ids is None else np.asarray(key_ids, np.uint16)),
             pn_out=t(np.full(n, pn_out_fill, np.uint64)))
    b = sqobfs.quic_batch(n, d_data, d["in_off"], d["in_len"], d_out, d["out_off"], d["out_len"],
                          d["pno"], d["pn"], d["kid"], d["pn_out"])
    with sqobfs.QuicKeyring(ctx, keys, suite) as kr:
        s = None if ctx_stream else torch.cuda.current_stream(dev).cuda_stream
        (sqobfs.quic_seal if seal else sqobfs.quic_open)(ctx, kr, b, s)
        if ctx_stream:
            ctx.sync()
        torch.cuda.synchronize(dev)
    return (d_out.cpu().numpy(), out_off, d["out_len"].cpu().numpy(), d["pn_out"].cpu().numpy(),
            out)


def test_rfc9001_a5(ctx):
    a5 = __import__("json").load(open(ol.REPO + "/tests/golden/quic.json"))["rfc9001_a5"]
    k = QuicKey.of(B(a5["key"]), B(a5["iv"]), B(a5["hp"]))
    pkt = B(a5["header"] + a5["payload"])
    out, oo, ol_, _, _ = run(ctx, [k], True, [pkt], [a5["pn_offset"]], [a5["pn"]])
    assert ol_[0] == len(pkt) + 16
    assert out[int(oo[0]):int(oo[0]) + ol_[0]].tobytes().hex() == a5["protected"]
    out, oo, ol_, pno, _ = run(ctx, [k], False, [B(a5["protected"])], [a5["pn_offset"]],
                               [a5["pn"] - 1])
    assert ol_[0] == len(pkt) and pno[0] == a5["pn"]
    assert out[int(oo[0]):int(oo[0]) + ol_[0]].tobytes() == pkt


@pytest.mark.parametrize("inplace", [False, True])
def test_golden_packets_one_batch(ctx, golden, inplace):
    """All 40 OpenSSL-built packets (each with its own keys) in one batch."""
    g = golden("quic.json")["packets"]
    keys = [QuicKey.of(B(v["key"]), B(v["iv"]), B(v["hp"])) for v in g]
    pkts = [B(v["packet"]) for v in g]
    out, oo, ol_, _, _ = run(ctx, keys, True, pkts, [v["pn_offset"] for v in g],
                             [v["pn"] for v in g], key_ids=list(range(len(g))), inplace=inplace)
    for i, v in enumerate(g):
        assert ol_[i] == len(pkts[i]) + 16
        assert out[int(oo[i]):int(oo[i]) + ol_[i]].tobytes().hex() == v["protected"], i
    prot = [B(v["protected"]) for v in g]
    out, oo, ol_, pno, _ = run(ctx, keys, False, prot, [v["pn_offset"] for v in g],
                               [v["largest_pn"] for v in g], key_ids=list(range(len(g))),
                               inplace=inplace)
    for i, v in enumerate(g):
        assert ol_[i] == len(pkts[i]) and pno[i] == v["pn"]
        assert out[int(oo[i]):int(oo[i]) + ol_[i]].tobytes() == pkts[i], i


def _random_packets(rng, n, max_payload=1500):
    pkts, pnos, pns = [], [], []
    for i in range(n):
        pn_len = int(rng.integers(1, 5))
        dcid = int(rng.integers(0, 21))
        first = 0x40 | (int(rng.integers(0, 8)) << 2) | (pn_len - 1)
        pn = int(rng.integers(0, 2**40))
        plen = int(rng.integers(4 - pn_len, max_payload))
        pkt = bytes([first]) + rng.integers(0, 256, dcid, dtype=np.uint8).tobytes() + \
            (pn & ((1 << (8 * pn_len)) - 1)).to_bytes(pn_len, "big") + \
            rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        pkts.append(pkt)
        pnos.append(1 + dcid)
        pns.append(pn)
    return pkts, pnos, pns


@pytest.mark.parametrize("align,inplace", [(1, False), (16, False), (1, True)])
def test_ragged_batch_vs_oracle(ctx, align, inplace):
    """Ragged 3000-packet batch, 3 connections, seal then open, every byte
    (sentinels around each packet included) against the oracle."""
    rng = np.random.Generator(np.random.PCG64(400 + align + inplace))
    keys_b = [tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (32, 12, 32))
              for _ in range(3)]
    keys = [QuicKey.of(*kb) for kb in keys_b]
    pkts, pnos, pns = _random_packets(rng, 3000)
    kid = rng.integers(0, 3, len(pkts))
    out, oo, ol_, _, buf = run(ctx, keys, True, pkts, pnos, pns, key_ids=kid, align=align,
                               inplace=inplace)
    ref = buf.copy()
    for i, p in enumerate(pkts):
        prot, r = ol.quic_seal(*keys_b[kid[i]], pns[i], p, pnos[i])
        assert r == len(p) + 16 and ol_[i] == r
        ref[int(oo[i]):int(oo[i]) + r] = np.frombuffer(prot, np.uint8)
    if not inplace:
        assert np.array_equal(out, ref), "seal output differs (or bytes outside packets touched)"
    else:
        for i in range(len(pkts)):
            assert out[int(oo[i]):int(oo[i]) + ol_[i]].tobytes() == \
                ref[int(oo[i]):int(oo[i]) + ol_[i]].tobytes()
    prot = [out[int(oo[i]):int(oo[i]) + ol_[i]].tobytes() for i in range(len(pkts))]
    largest = [max(0, pn - int(rng.integers(1, 100))) for pn in pns]
    out2, oo2, ol2, pno2, _ = run(ctx, keys, False, prot, pnos, largest, key_ids=kid,
                                  align=align, inplace=inplace)
    for i, p in enumerate(pkts):
        assert ol2[i] == len(p) and pno2[i] == pns[i]
        assert out2[int(oo2[i]):int(oo2[i]) + ol2[i]].tobytes() == p


def test_open_rejects_tampering_and_bad_input(ctx):
    rng = np.random.Generator(np.random.PCG64(77))
    kb = tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (32, 12, 32))
    pkts, pnos, pns = _random_packets(rng, 64, 300)
    prot = [ol.quic_seal(*kb, pn, p, o)[0] for p, o, pn in zip(pkts, pnos, pns)]
    bad = []
    for i, q in enumerate(prot):
        q = bytearray(q)
        q[len(q) - 1 - (i % len(q))] ^= 1 << (i % 8)  # one flipped bit anywhere
        bad.append(bytes(q))
    _, _, ol_, _, _ = run(ctx, [QuicKey.of(*kb)], False, bad, pnos, [pn - 1 for pn in pns])
    for i in range(len(bad)):
        want = ol.quic_open(*kb, pns[i] - 1, bad[i], pnos[i])[1]
        assert want < 0
        assert ol_[i] in (sqobfs.QUIC_EAUTH, sqobfs.QUIC_ESHORT), i
        assert (ol_[i] == sqobfs.QUIC_EAUTH) == (want == -2), i
    # too short to sample, and an out-of-range key id
    _, _, ol_, _, _ = run(ctx, [QuicKey.of(*kb)], True, [b"\x40\x01\x02", b"\x43" + bytes(40)],
                          [1, 1], [1, 2], key_ids=[0, 5])
    assert ol_[0] == sqobfs.QUIC_ESHORT and ol_[1] == sqobfs.QUIC_EKEY


@pytest.mark.parametrize("suite", [0, 1])
def test_open_rejects_write_pn_out_zero(ctx, suite):
    """Every rejected packet of an open gets pn_out = 0 (too short, and an
    out-of-range key id), not whatever the buffer held before."""
    rng = np.random.Generator(np.random.PCG64(17 + suite))
    kl = 16 if suite else 32
    kb = tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (kl, 12, kl))
    pkts = [b"\x40\x01\x02", b"\x43" + bytes(60)]
    _, _, ol_, pno_, _ = run(ctx, [QuicKey.of(*kb)], False, pkts, [1, 1], [1, 2], key_ids=[0, 5],
                             suite=suite, pn_out_fill=0xDEADBEEF)
    assert ol_[0] == sqobfs.QUIC_ESHORT and ol_[1] == sqobfs.QUIC_EKEY
    assert list(pno_) == [0, 0]


def test_long_payloads_owner_path(ctx):
    """Payloads either side of the cooperative limit (1,536 B; 2,048 B before),
    walked by the owner lane above it, mixed in one batch with short
    packets."""
    rng = np.random.Generator(np.random.PCG64(991))
    kb = tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (32, 12, 32))
    pkts, pnos, pns = [], [], []
    for plen in [1500, 1535, 1536, 1537, 1538, 1552, 2030, 2047, 2048, 2049, 2050, 2064,
                 3000, 9000, 65, 2, 4000, 1350]:
        pn_len = 2
        pkt = bytes([0x41]) + bytes(8) + (7).to_bytes(pn_len, "big") + \
            rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        pkts.append(pkt)
        pnos.append(9)
        pns.append(7)
    out, oo, ol_, _, _ = run(ctx, [QuicKey.of(*kb)], True, pkts, pnos, pns)
    prot = []
    for i, p in enumerate(pkts):
        want, r = ol.quic_seal(*kb, pns[i], p, pnos[i])
        assert ol_[i] == r == len(p) + 16
        got = out[int(oo[i]):int(oo[i]) + r].tobytes()
        assert got == want, (i, len(p))
        prot.append(got)
    out2, oo2, ol2, pno2, _ = run(ctx, [QuicKey.of(*kb)], False, prot, pnos, [6] * len(prot))
    for i, p in enumerate(pkts):
        assert ol2[i] == len(p) and pno2[i] == 7
        assert out2[int(oo2[i]):int(oo2[i]) + ol2[i]].tobytes() == p
