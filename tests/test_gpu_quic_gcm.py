"""QUIC packet protection with AES-128-GCM on the GPU (sqobfs_quic_seal /
_open on a SQOBFS_QUIC_AES_128_GCM keyring) against the CPU oracle and the
committed vectors: RFC 9001 Appendix A.3 and OpenSSL-built packets
(tests/golden/quic_gcm.json).  Bit-exact on every output byte, including
the bytes around each packet, and on out_len / decoded packet numbers.
Both kernel variants are covered: one key (round keys in the kernarg
segment, GHASH tables in LDS) and per-packet key ids (keyring in global
memory)."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import QuicKey

import oracle_lib as ol
from test_gpu_quic import _random_packets, ctx, run  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu
B = bytes.fromhex
GCM = sqobfs.QUIC_AES_128_GCM


def _keys(rng, n):
    kb = [tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (16, 12, 16))
          for _ in range(n)]
    return kb, [QuicKey.of(*k) for k in kb]


def test_rfc9001_a3(ctx, golden):  # noqa: F811
    g = golden("quic_gcm.json")
    a3, sk = g["rfc9001_a3"], g["rfc9001_a1"]["server"]
    k = QuicKey.of(B(sk["key"]), B(sk["iv"]), B(sk["hp"]))
    pkt = B(a3["header"] + a3["payload"])
    for kid in (None, [0]):
        out, oo, ol_, _, _ = run(ctx, [k], True, [pkt], [a3["pn_offset"]], [a3["pn"]],
                                 key_ids=kid, suite=GCM)
        assert ol_[0] == len(pkt) + 16
        assert out[int(oo[0]):int(oo[0]) + ol_[0]].tobytes().hex() == a3["protected"]
        out, oo, ol_, pno, _ = run(ctx, [k], False, [B(a3["protected"])], [a3["pn_offset"]], [0],
                                   key_ids=kid, suite=GCM)
        assert ol_[0] == len(pkt) and pno[0] == a3["pn"]
        assert out[int(oo[0]):int(oo[0]) + ol_[0]].tobytes() == pkt


@pytest.mark.parametrize("inplace", [False, True])
def test_golden_packets_one_batch(ctx, golden, inplace):  # noqa: F811
    """All 40 OpenSSL-built packets (each with its own keys) in one batch."""
    g = golden("quic_gcm.json")["packets"]
    keys = [QuicKey.of(B(v["key"]), B(v["iv"]), B(v["hp"])) for v in g]
    pkts = [B(v["packet"]) for v in g]
    kid = list(range(len(g)))
    out, oo, ol_, _, _ = run(ctx, keys, True, pkts, [v["pn_offset"] for v in g],
                             [v["pn"] for v in g], key_ids=kid, inplace=inplace, suite=GCM)
    for i, v in enumerate(g):
        assert ol_[i] == len(pkts[i]) + 16
        assert out[int(oo[i]):int(oo[i]) + ol_[i]].tobytes().hex() == v["protected"], i
    prot = [B(v["protected"]) for v in g]
    out, oo, ol_, pno, _ = run(ctx, keys, False, prot, [v["pn_offset"] for v in g],
                               [v["largest_pn"] for v in g], key_ids=kid, inplace=inplace,
                               suite=GCM)
    for i, v in enumerate(g):
        assert ol_[i] == len(pkts[i]) and pno[i] == v["pn"]
        assert out[int(oo[i]):int(oo[i]) + ol_[i]].tobytes() == pkts[i], i


@pytest.mark.parametrize("nkeys,align,inplace", [(1, 1, False), (1, 16, True), (3, 1, False),
                                                 (3, 16, False), (3, 1, True)])
def test_ragged_batch_vs_oracle(ctx, nkeys, align, inplace):  # noqa: F811
    """Ragged 3000-packet batch, seal then open, every byte (sentinels around
    each packet included) against the oracle; one key or three."""
    rng = np.random.Generator(np.random.PCG64(700 + 10 * nkeys + align + inplace))
    kb, keys = _keys(rng, nkeys)
    pkts, pnos, pns = _random_packets(rng, 3000)
    kid = rng.integers(0, nkeys, len(pkts)) if nkeys > 1 else np.zeros(len(pkts), np.int64)
    kid_arg = kid if nkeys > 1 else None
    out, oo, ol_, _, buf = run(ctx, keys, True, pkts, pnos, pns, key_ids=kid_arg, align=align,
                               inplace=inplace, suite=GCM)
    ref = buf.copy()
    for i, p in enumerate(pkts):
        prot, r = ol.quic_seal(*kb[kid[i]], pns[i], p, pnos[i], suite=ol.AES128GCM)
        assert r == len(p) + 16 and ol_[i] == r
        ref[int(oo[i]):int(oo[i]) + r] = np.frombuffer(prot, np.uint8)
    if not inplace:
        assert np.array_equal(out, ref), "seal output differs (or bytes outside packets touched)"
    else:
        for i in range(len(pkts)):
            assert out[int(oo[i]):int(oo[i]) + ol_[i]].tobytes() == \
                ref[int(oo[i]):int(oo[i]) + ol_[i]].tobytes(), i
    prot = [out[int(oo[i]):int(oo[i]) + ol_[i]].tobytes() for i in range(len(pkts))]
    largest = [max(0, pn - int(rng.integers(1, 100))) for pn in pns]
    out2, oo2, ol2, pno2, _ = run(ctx, keys, False, prot, pnos, largest, key_ids=kid_arg,
                                  align=align, inplace=inplace, suite=GCM)
    for i, p in enumerate(pkts):
        assert ol2[i] == len(p) and pno2[i] == pns[i], i
        assert out2[int(oo2[i]):int(oo2[i]) + ol2[i]].tobytes() == p, i


@pytest.mark.parametrize("multi", [False, True])
def test_long_payloads_owner_path(ctx, multi):  # noqa: F811
    """Payloads either side of the cooperative limit (2,048 B)."""
    rng = np.random.Generator(np.random.PCG64(992 + multi))
    kb, keys = _keys(rng, 1)
    pkts = []
    for plen in [2030, 2047, 2048, 2049, 2050, 2064, 3000, 9000, 65, 2, 4000, 1350]:
        pkts.append(bytes([0x41]) + bytes(8) + (7).to_bytes(2, "big") +
                    rng.integers(0, 256, plen, dtype=np.uint8).tobytes())
    pnos, pns = [9] * len(pkts), [7] * len(pkts)
    kid = [0] * len(pkts) if multi else None
    out, oo, ol_, _, _ = run(ctx, keys, True, pkts, pnos, pns, key_ids=kid, suite=GCM)
    prot = []
    for i, p in enumerate(pkts):
        want, r = ol.quic_seal(*kb[0], pns[i], p, pnos[i], suite=ol.AES128GCM)
        assert ol_[i] == r == len(p) + 16
        got = out[int(oo[i]):int(oo[i]) + r].tobytes()
        assert got == want, (i, len(p))
        prot.append(got)
    out2, oo2, ol2, pno2, _ = run(ctx, keys, False, prot, pnos, [6] * len(prot), key_ids=kid,
                                  suite=GCM)
    for i, p in enumerate(pkts):
        assert ol2[i] == len(p) and pno2[i] == 7
        assert out2[int(oo2[i]):int(oo2[i]) + ol2[i]].tobytes() == p


def test_open_rejects_tampering_and_bad_input(ctx):  # noqa: F811
    rng = np.random.Generator(np.random.PCG64(78))
    kb, keys = _keys(rng, 1)
    pkts, pnos, pns = _random_packets(rng, 64, 300)
    prot = [ol.quic_seal(*kb[0], pn, p, o, suite=ol.AES128GCM)[0]
            for p, o, pn in zip(pkts, pnos, pns)]
    bad = []
    for i, q in enumerate(prot):
        q = bytearray(q)
        q[len(q) - 1 - (i % len(q))] ^= 1 << (i % 8)
        bad.append(bytes(q))
    _, _, ol_, _, _ = run(ctx, keys, False, bad, pnos, [pn - 1 for pn in pns], suite=GCM)
    for i in range(len(bad)):
        want = ol.quic_open(*kb[0], pns[i] - 1, bad[i], pnos[i], suite=ol.AES128GCM)[1]
        assert want < 0
        assert ol_[i] in (sqobfs.QUIC_EAUTH, sqobfs.QUIC_ESHORT), i
        assert (ol_[i] == sqobfs.QUIC_EAUTH) == (want == -2), i
    _, _, ol_, _, _ = run(ctx, keys, True, [b"\x40\x01\x02", b"\x43" + bytes(40)], [1, 1], [1, 2],
                          key_ids=[0, 5], suite=GCM)
    assert ol_[0] == sqobfs.QUIC_ESHORT and ol_[1] == sqobfs.QUIC_EKEY


@pytest.mark.parametrize("nkeys,n,inplace", [(16, 20000, False), (4, 8192, True), (1, 4096, False),
                                             (300, 6000, False), (2, 2047, False),
                                             (1100, 3000, False)])
def test_key_grouped_batches(ctx, nkeys, n, inplace):  # noqa: F811
    """Multi-key batches of >= 2,048 packets, <= 1,023 keys and >= 1,024
    packets per key are grouped by key (sq_launch_gcm_group: steps of one
    key each, run on staged keys; invalid ids rejected by the grouping); 300
    keys over 6,000 packets, 2,047 packets and 1,100 keys stay on the
    per-packet kernel.  Random key order, 1 % invalid key ids; seal then open
    against the oracle."""
    rng = np.random.Generator(np.random.PCG64(900 + nkeys + n))
    kb, keys = _keys(rng, nkeys)
    pkts, pnos, pns = _random_packets(rng, n)
    kid = rng.integers(0, nkeys, n)
    bad = rng.random(n) < 0.01
    kid[bad] = nkeys + rng.integers(0, 5, int(bad.sum()))
    out, oo, ol_, _, buf = run(ctx, keys, True, pkts, pnos, pns, key_ids=kid, inplace=inplace,
                               suite=GCM)
    prot = []
    for i, p in enumerate(pkts):
        if bad[i]:
            assert ol_[i] == sqobfs.QUIC_EKEY, i
            prot.append(p + bytes(16))
            continue
        want, r = ol.quic_seal(*kb[kid[i]], pns[i], p, pnos[i], suite=ol.AES128GCM)
        assert ol_[i] == r == len(p) + 16, i
        got = out[int(oo[i]):int(oo[i]) + r].tobytes()
        assert got == want, i
        prot.append(got)
    largest = [max(0, pn - int(rng.integers(1, 100))) for pn in pns]
    out2, oo2, ol2, pno2, _ = run(ctx, keys, False, prot, pnos, largest, key_ids=kid,
                                  inplace=inplace, suite=GCM)
    for i, p in enumerate(pkts):
        if bad[i]:
            assert ol2[i] == sqobfs.QUIC_EKEY and pno2[i] == 0, i
            continue
        assert ol2[i] == len(p) and pno2[i] == pns[i], i
        assert out2[int(oo2[i]):int(oo2[i]) + ol2[i]].tobytes() == p, i


@pytest.mark.parametrize("ctx_stream", [False, True])
def test_ungrouped_fallback_matches_grouped(ctx, ctx_stream):  # noqa: F811
    """The kernel a multi-key batch falls back to when its grouping scratch
    cannot be allocated (forced by sqobfs_debug_gcm_ungrouped) gives the same
    bytes, lengths and packet numbers as the grouped launch.  On the context's
    own stream the grouping scratch is cached and grows: a smaller batch
    first, then a larger one, then the smaller again."""
    rng = np.random.Generator(np.random.PCG64(77))
    kb, keys = _keys(rng, 16)
    for n in (4096, 20000, 4096):
        pkts, pnos, pns = _random_packets(rng, n)
        kid = rng.integers(0, 16, n)
        kid[rng.random(n) < 0.01] = 16  # invalid ids: rejected either way
        res = []
        for ungrouped in (False, True):
            sqobfs.debug_gcm_ungrouped(ungrouped)
            try:
                out, oo, ol_, _, _ = run(ctx, keys, True, pkts, pnos, pns, key_ids=kid,
                                         suite=GCM, ctx_stream=ctx_stream)
                prot = [out[int(oo[i]):int(oo[i]) + int(ol_[i])].tobytes()
                        if ol_[i] == len(p) + 16 else p + bytes(16) for i, p in enumerate(pkts)]
                out2, oo2, ol2, pno2, _ = run(ctx, keys, False, prot, pnos, pns, key_ids=kid,
                                              suite=GCM, ctx_stream=ctx_stream)
            finally:
                sqobfs.debug_gcm_ungrouped(False)
            res.append((prot, ol_.copy(), [out2[int(oo2[i]):int(oo2[i]) + max(0, int(ol2[i]))
                                               ].tobytes() if ol2[i] < 1 << 31 else b""
                                           for i in range(n)], ol2.copy(), pno2.copy()))
        g, u = res
        assert g[0] == u[0] and np.array_equal(g[1], u[1]), n
        assert np.array_equal(g[3], u[3]) and np.array_equal(g[4], u[4]), n
        assert g[2] == u[2], n
        i = int(np.flatnonzero(kid < 16)[0])
        want, r = ol.quic_seal(*kb[kid[i]], pns[i], pkts[i], pnos[i], suite=ol.AES128GCM)
        assert g[0][i] == want and r == len(pkts[i]) + 16
