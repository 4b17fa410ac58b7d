"""QUIC protection (both suites) fused with the Salamander layer on the GPU
(sqobfs_quic_seal_salamander / _open_salamander): Hysteria2's datagram is
salt8 || (protected QUIC packet) ^ BLAKE2b-256(psk || salt8).  Checked byte
for byte against the oracle composition: or_quic_seal (RFC 9001, ChaCha20-
Poly1305) followed by the restated SalamanderPacketConn.WriteTo
(hysteria2/salamander.go:57-70), and on the way in ReadFrom
(salamander.go:42-55) followed by or_quic_open."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import QuicKey

import oracle_lib as ol
from test_gpu_quic import _random_packets, ctx  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu
PSK = b"sing-quic-mi355x-bench-psk"
SENT = 0x5A


def _place(sizes, lead, gap, align=1):
    offs, pos = [], lead
    for sz in sizes:
        offs.append(pos)
        pos = (pos + sz + gap + align - 1) // align * align + lead
    return np.array(offs, np.uint64), pos + 64


def _seal(ctx, keys, kr_o, pkts, pnos, pns, salts, key_ids=None, inplace=False, align=1,  # noqa: F811
          suite=0):
    import torch
    dev = torch.device("cuda", 0)
    n = len(pkts)
    in_off, end = _place([len(p) + 16 for p in pkts], 8, 3, align)
    data = np.full(end, SENT, np.uint8)
    for o, p in zip(in_off, pkts):
        data[int(o):int(o) + len(p)] = np.frombuffer(p, np.uint8)
    if inplace:
        out_off = in_off - 8
        out = data
    else:
        out_off, oend = _place([len(p) + 24 for p in pkts], 0, 5, align)
        out = np.full(oend, SENT, np.uint8)
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa
    d_data = t(data)
    d_out = d_data if inplace else t(out)
    d = dict(in_off=t(in_off), in_len=t(np.array([len(p) for p in pkts], np.uint32)),
             out_off=t(out_off), out_len=t(np.zeros(n, np.uint32)),
             pno=t(np.asarray(pnos, np.uint16)), pn=t(np.asarray(pns, np.uint64)),
             kid=t(None if key_ids is None else np.asarray(key_ids, np.uint16)),
             salt=t(np.frombuffer(b"".join(salts), np.uint8).copy()))
    b = sqobfs.quic_batch(n, d_data, d["in_off"], d["in_len"], d_out, d["out_off"], d["out_len"],
                          d["pno"], d["pn"], d["kid"])
    with sqobfs.QuicKeyring(ctx, keys, suite) as kr:
        s = torch.cuda.current_stream(dev).cuda_stream
        sqobfs.quic_seal_salamander(ctx, kr, kr_o, b, d["salt"], s)
        torch.cuda.synchronize(dev)
    return d_out.cpu().numpy(), out_off, d["out_len"].cpu().numpy(), out


def _open(ctx, keys, kr_o, wires, pnos, largest, key_ids=None, inplace=False,  # noqa: F811
          suite=0):
    import torch
    dev = torch.device("cuda", 0)
    n = len(wires)
    in_off, end = _place([len(w) for w in wires], 0, 3)
    data = np.full(end, SENT, np.uint8)
    for o, w in zip(in_off, wires):
        data[int(o):int(o) + len(w)] = np.frombuffer(w, np.uint8)
    if inplace:
        out_off, out = in_off, data
    else:
        out_off, oend = _place([max(len(w), 1) for w in wires], 0, 5)
        out = np.full(oend, SENT, np.uint8)
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa
    d_data = t(data)
    d_out = d_data if inplace else t(out)
    d = dict(in_off=t(in_off), in_len=t(np.array([len(w) for w in wires], np.uint32)),
             out_off=t(out_off), out_len=t(np.zeros(n, np.uint32)),
             pno=t(np.asarray(pnos, np.uint16)), pn=t(np.asarray(largest, np.uint64)),
             kid=t(None if key_ids is None else np.asarray(key_ids, np.uint16)),
             pn_out=t(np.zeros(n, np.uint64)))
    b = sqobfs.quic_batch(n, d_data, d["in_off"], d["in_len"], d_out, d["out_off"], d["out_len"],
                          d["pno"], d["pn"], d["kid"], d["pn_out"])
    with sqobfs.QuicKeyring(ctx, keys, suite) as kr:
        s = torch.cuda.current_stream(dev).cuda_stream
        sqobfs.quic_open_salamander(ctx, kr, kr_o, b, s)
        torch.cuda.synchronize(dev)
    return d_out.cpu().numpy(), out_off, d["out_len"].cpu().numpy(), d["pn_out"].cpu().numpy()


def _keys(rng, n, suite=0):
    kl = 16 if suite else 32
    kb = [tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (kl, 12, kl))
          for _ in range(n)]
    return kb, [QuicKey.of(*k) for k in kb]


def _want_wire(kb, pkt, pno, pn, salt, suite=0):
    prot, r = ol.quic_seal(*kb, pn, pkt, pno, suite=suite)
    assert r == len(pkt) + 16
    return ol.salamander_write(PSK, salt, prot)[0]


@pytest.mark.parametrize("suite", [0, 1])
@pytest.mark.parametrize("nkeys,inplace", [(1, False), (1, True), (3, False)])
def test_seal_open_ragged_vs_oracle(ctx, nkeys, inplace, suite):  # noqa: F811
    rng = np.random.Generator(np.random.PCG64(500 + nkeys + inplace + 10 * suite))
    kb, keys = _keys(rng, nkeys, suite)
    # (multi-key AES-GCM batches of >= 2,048 packets are grouped by key)
    pkts, pnos, pns = _random_packets(rng, 3200 if nkeys > 1 else 2000)
    salts = [rng.integers(0, 256, 8, dtype=np.uint8).tobytes() for _ in pkts]
    kid = rng.integers(0, nkeys, len(pkts)) if nkeys > 1 else np.zeros(len(pkts), np.int64)
    kid_arg = kid if nkeys > 1 else None
    with sqobfs.Keyring(ctx, sqobfs.SALAMANDER, [PSK]) as kr_o:
        out, oo, olen, buf = _seal(ctx, keys, kr_o, pkts, pnos, pns, salts, kid_arg, inplace,
                                   suite=suite)
        ref = buf.copy()
        wires = []
        for i, p in enumerate(pkts):
            w = _want_wire(kb[kid[i]], p, pnos[i], pns[i], salts[i], suite)
            assert olen[i] == len(p) + 24, i
            ref[int(oo[i]):int(oo[i]) + len(w)] = np.frombuffer(w, np.uint8)
            got = out[int(oo[i]):int(oo[i]) + len(w)].tobytes()
            assert got == w, i
            wires.append(w)
        if not inplace:
            assert np.array_equal(out, ref), "bytes outside the datagrams were touched"
        largest = [max(0, pn - int(rng.integers(1, 100))) for pn in pns]
        out2, oo2, ol2, pno2 = _open(ctx, keys, kr_o, wires, pnos, largest, kid_arg, inplace,
                                     suite=suite)
        for i, p in enumerate(pkts):
            assert ol2[i] == len(p) and pno2[i] == pns[i], i
            assert out2[int(oo2[i]):int(oo2[i]) + len(p)].tobytes() == p, i


@pytest.mark.parametrize("suite", [0, 1])
def test_long_payloads_and_rejects(ctx, suite):  # noqa: F811
    rng = np.random.Generator(np.random.PCG64(77 + suite))
    kb, keys = _keys(rng, 1, suite)
    pkts = [bytes([0x41]) + bytes(8) + (7).to_bytes(2, "big") +
            rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
            for plen in [1535, 1536, 1537, 2047, 2048, 2049, 3000, 9000, 65, 2, 1350]]
    pnos, pns = [9] * len(pkts), [7] * len(pkts)
    salts = [rng.integers(0, 256, 8, dtype=np.uint8).tobytes() for _ in pkts]
    with sqobfs.Keyring(ctx, sqobfs.SALAMANDER, [PSK]) as kr_o:
        out, oo, olen, _ = _seal(ctx, keys, kr_o, pkts, pnos, pns, salts, suite=suite)
        wires = []
        for i, p in enumerate(pkts):
            w = _want_wire(kb[0], p, pnos[i], pns[i], salts[i], suite)
            assert out[int(oo[i]):int(oo[i]) + len(w)].tobytes() == w, len(p)
            wires.append(w)
        out2, oo2, ol2, pno2 = _open(ctx, keys, kr_o, wires, pnos, [6] * len(wires), suite=suite)
        for i, p in enumerate(pkts):
            assert ol2[i] == len(p) and out2[int(oo2[i]):int(oo2[i]) + len(p)].tobytes() == p
        # tampering anywhere (salt, header, payload, tag) and too-short datagrams
        bad = []
        for i, w in enumerate(wires):
            w = bytearray(w)
            w[[0, 9, len(w) // 2, len(w) - 1][i % 4]] ^= 0x10
            bad.append(bytes(w))
        bad += [b"\x01\x02\x03", bytes(8), bytes(20)]
        _, _, ol3, _ = _open(ctx, keys, kr_o, bad, [9] * len(bad), [6] * len(bad), suite=suite)
        for i, w in enumerate(bad):
            plain, n = ol.salamander_read(PSK, w)
            want = ol.quic_open(*kb[0], 6, plain[:n], 9, suite=suite)[1] if len(w) > 8 else -1
            assert want < 0
            if len(w) <= 8:
                assert ol3[i] == sqobfs.QUIC_ESHORT
            else:
                assert (ol3[i] == sqobfs.QUIC_EAUTH) == (want == -2), i
