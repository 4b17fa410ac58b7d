"""Pin the CPU restatement (oracle/oracle.c) before trusting it as the checker.

1. Primitive known-answer tests: RFC 7693 Appendix A (BLAKE2b-512 "abc"),
   FIPS 180-2 SHA-256 examples, hashlib BLAKE2b-256 values.
2. Every committed golden vector (tests/golden/, made by the hashlib-based
   py_oracle) reproduced by the C restatement, byte for byte.
3. Randomised cross-check C vs Python restatement (hypothesis) over payload
   and PSK lengths that cross every block boundary.
The Go reference has no tests/fixtures and cannot be run (no Go toolchain),
so this is where parity is pinned ("Parity").
"""
from __future__ import annotations

import hashlib

import numpy as np
import py_oracle as po
from hypothesis import given, settings
from hypothesis import strategies as st

import oracle_lib as ol

B = bytes.fromhex


def test_blake2b_kats(golden):
    k = golden("kat.json")
    r = k["blake2b512_abc_rfc7693"]
    assert ol.blake2b(B(r["msg"]), 64).hex() == r["digest"]
    for v in k["blake2b256"]:
        assert ol.blake2b(B(v["msg"]), 32).hex() == v["digest"]
        assert hashlib.blake2b(B(v["msg"]), digest_size=32).hexdigest() == v["digest"]


def test_sha256_kats(golden):
    k = golden("kat.json")
    for v in k["sha256_fips180"] + k["sha256"]:
        assert ol.sha256(B(v["msg"])).hex() == v["digest"]
        assert hashlib.sha256(B(v["msg"])).hexdigest() == v["digest"]


def test_survey_examples(golden):
    sal, xp = golden("survey_examples.json")
    assert ol.salamander_key(B(sal["psk"]), B(sal["salt"])).hex() == sal["key"]
    wire, ret = ol.salamander_write(B(sal["psk"]), B(sal["salt"]), B(sal["payload"]))
    assert wire.hex() == sal["wire"] and ret == len(B(sal["payload"]))
    assert sal["wire"] == ("0001020304050607d9e35a28e0017913caa0c3556b6e1d7c41d94eee839e2"
                           "31b1cd585e94895745fd5e350")
    assert ol.xplus_key(B(xp["psk"]), B(xp["salt"])).hex() == xp["key"]
    wire, ret = ol.xplus_write(B(xp["psk"]), B(xp["salt"]), B(xp["payload"]))
    assert wire.hex() == xp["wire"] and ret == len(B(xp["payload"])) + 16


def test_golden_write(golden):
    for name, write, keyf, S in (("salamander_write.json", ol.salamander_write, ol.salamander_key, 8),
                                 ("xplus_write.json", ol.xplus_write, ol.xplus_key, 16)):
        for v in golden(name):
            psk, salt, pay = B(v["psk"]), B(v["salt"]), B(v["payload"])
            assert keyf(psk, salt).hex() == v["key"]
            wire, ret = write(psk, salt, pay)
            assert wire.hex() == v["wire"]
            assert ret == v["write_ret"]


def test_golden_read(golden):
    for v in golden("salamander_read.json"):
        buf, ret = ol.salamander_read(B(v["psk"]), B(v["datagram"]))
        assert buf.hex() == v["buffer_after"] and ret == v["read_ret"]
    for v in golden("xplus_read.json"):
        full = B(v["buffer_full"])
        buf, ret = ol.xplus_read(B(v["psk"]), full, len(B(v["datagram"])))
        assert buf.hex() == v["buffer_after"] and ret == v["read_ret"]


def test_read_quirks():
    psk = b"k"
    # salamander.go:47-49: n <= 8 returned untouched with length n
    for n in range(0, 9):
        d = bytes(range(n))
        assert ol.salamander_read(psk, d) == (d, n)
    # xplus.go:50-52: n < 16 returns 0, untouched
    for n in range(0, 16):
        d = bytes(range(n)) + b"\xaa" * 4
        assert ol.xplus_read(psk, d, n) == (d, 0)


def test_golden_vectorised(golden):
    for v in golden("vectorised.json"):
        bufs = [B(x) for x in v["bufs"]]
        out, panicked = ol.salamander_write_vectorised(B(v["psk"]), B(v["salamander_salt"]), bufs)
        assert panicked == v["salamander_panics"]
        if not panicked:
            assert [o.hex() for o in out] == v["salamander_out"]
        xo = ol.xplus_write_vectorised(B(v["psk"]), B(v["xplus_salt"]), bufs)
        assert [o.hex() for o in xo] == v["xplus_out"]


def test_salamander_line104_only_first_buffer_is_sound():
    """salamander.go:104 indexes key[bufferIndex+index%32]: any second
    non-empty buffer after a non-empty first one panics in Go."""
    _, panicked = ol.salamander_write_vectorised(b"p", bytes(8), [b"x" * 10, b"y"])
    assert panicked
    out, panicked = ol.salamander_write_vectorised(b"p", bytes(8), [b"", b"y" * 40])
    assert not panicked
    assert out[1] == ol.salamander_write(b"p", bytes(8), b"y" * 40)[0][8:]


@settings(max_examples=150, deadline=None)
@given(psk=st.binary(min_size=0, max_size=300), salt8=st.binary(min_size=8, max_size=8),
       salt16=st.binary(min_size=16, max_size=16), pay=st.binary(min_size=0, max_size=200))
def test_c_matches_python_restatement(psk, salt8, salt16, pay):
    assert ol.salamander_write(psk, salt8, pay) == po.salamander_write(psk, salt8, pay)
    assert ol.xplus_write(psk, salt16, pay) == po.xplus_write(psk, salt16, pay)
    wire, _ = po.salamander_write(psk, salt8, pay)
    assert ol.salamander_read(psk, wire) == po.salamander_read(psk, wire)
    wire, _ = po.xplus_write(psk, salt16, pay)
    assert ol.xplus_read(psk, wire + b"\x01\x02", len(wire)) == \
        po.xplus_read(psk, wire + b"\x01\x02", len(wire))


def test_batch_restatement_matches_per_packet():
    """or_batch_run (threaded, used as the CPU baseline) == per-packet calls."""
    import sqobfs
    rng = np.random.Generator(np.random.PCG64(7))
    lens = rng.integers(0, 300, 97)
    pk = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    psks = [b"a" * 5, b"bb" * 70, b""]
    ids = rng.integers(0, 3, 97).astype(np.uint16)
    for kind, S, write in ((0, 8, ol.salamander_write), (1, 16, ol.xplus_write)):
        data, off, ln = sqobfs.pack(pk, align=1)
        salt = rng.integers(0, 256, 97 * S, dtype=np.uint8)
        oo = np.cumsum([0] + [len(p) + S for p in pk[:-1]]).astype(np.uint64)
        out = np.zeros(int(oo[-1]) + len(pk[-1]) + S + 8, np.uint8)
        olen = np.zeros(97, np.uint32)
        hb = sqobfs.HostBatch(data, off, ln, out, oo, olen, salt, ids)
        ol.batch_run(kind, 0, psks, hb, nthreads=4)
        for i, p in enumerate(pk):
            w, _ = write(psks[ids[i]], salt[i * S:(i + 1) * S].tobytes(), p)
            assert out[int(oo[i]):int(oo[i]) + len(w)].tobytes() == w
            assert olen[i] == len(p) + S


def test_chacha20_keystreams(golden):
    """ChaCha20 restatement (device-salt checker) vs RFC 8439 2.3.2 and
    OpenSSL keystreams (tests/golden/make_chacha.py)."""
    g = golden("chacha20.json")
    assert g["streams"][0]["source"].startswith("RFC 8439")
    for v in g["streams"]:
        n = len(v["stream"]) // 2
        assert ol.chacha20_stream(B(v["key"]), B(v["nonce"]), v["counter"], n).hex() == v["stream"]


def test_device_salt_derivation(golden):
    for v in golden("chacha20.json")["device_salts"]:
        got = ol.device_salts(B(v["key"]), v["seq"], v["n"], v["S"])
        assert got.hex() == v["salts"]
        # packet i's salt is bytes [(i % (64/S))*S, +S) of block i // (64/S)
        per = 64 // v["S"]
        nonce = b"sqob" + v["seq"].to_bytes(8, "little")
        for i in (0, v["n"] - 1):
            blk = ol.chacha20_stream(B(v["key"]), nonce, i // per, 64)
            assert got[i * v["S"]:(i + 1) * v["S"]] == blk[(i % per) * v["S"]:(i % per + 1) * v["S"]]


def test_poly1305_and_aead(golden):
    """Poly1305 / AEAD restatement vs RFC 8439 2.5.2 and OpenSSL."""
    g = golden("quic.json")
    for v in g["poly1305"]:
        assert ol.poly1305(B(v["key"]), B(v["msg"])).hex() == v["tag"]
    for v in g["aead"]:
        assert ol.aead_seal(B(v["key"]), B(v["nonce"]), B(v["aad"]), B(v["pt"])).hex() == \
            v["ct_tag"]


def test_quic_packet_protection(golden):
    """QUIC seal / open restatement vs RFC 9001 A.5 and OpenSSL-built
    packets (short and long headers, pn lengths 1-4, minimum-size payloads)."""
    g = golden("quic.json")
    a5 = g["rfc9001_a5"]
    prot, r = ol.quic_seal(B(a5["key"]), B(a5["iv"]), B(a5["hp"]), a5["pn"],
                           B(a5["header"] + a5["payload"]), a5["pn_offset"])
    assert prot.hex() == a5["protected"]
    plain, r, pn = ol.quic_open(B(a5["key"]), B(a5["iv"]), B(a5["hp"]), a5["pn"] - 1,
                                B(a5["protected"]), a5["pn_offset"])
    assert r > 0 and pn == a5["pn"] and plain.hex() == a5["header"] + a5["payload"]
    for v in g["packets"]:
        k, iv, hp = B(v["key"]), B(v["iv"]), B(v["hp"])
        prot, r = ol.quic_seal(k, iv, hp, v["pn"], B(v["packet"]), v["pn_offset"])
        assert prot.hex() == v["protected"]
        plain, r, pn = ol.quic_open(k, iv, hp, v["largest_pn"], prot, v["pn_offset"])
        assert r == len(prot) - 16 and pn == v["pn"] and plain.hex() == v["packet"]
        bad = bytearray(prot)
        bad[-1] ^= 1  # tag bit flip
        assert ol.quic_open(k, iv, hp, v["largest_pn"], bytes(bad), v["pn_offset"])[1] == -2


def test_aes128_and_gcm(golden):
    """AES-128 (FIPS-197) and AES-128-GCM restatements against FIPS-197, the
    GCM specification's test cases and OpenSSL (tests/golden/make_quic_gcm.py)."""
    g = golden("quic_gcm.json")
    for v in g["aes"]:
        assert ol.aes128_encrypt(B(v["key"]), B(v["pt"])).hex() == v["ct"], v["source"]
    for v in g["gcm"]:
        assert ol.gcm_seal(B(v["key"]), B(v["nonce"]), B(v["aad"]), B(v["pt"])).hex() == \
            v["ct_tag"], v["source"]
    # GF(2^128): x * 1 = x (1 is the bit-reflected 0x80..00), commutative
    one = bytes([0x80]) + bytes(15)
    x, y = bytes(range(16)), bytes(range(100, 116))
    assert ol.gf128_mul(x, one) == x
    assert ol.gf128_mul(x, y) == ol.gf128_mul(y, x)


def test_quic_aes_gcm_packet_protection(golden):
    """RFC 9001 A.3 (server Initial, AES-128-GCM) and 40 OpenSSL-built packets:
    seal bit-exact, open round trip with the packet number decoded."""
    g = golden("quic_gcm.json")
    a3, sk = g["rfc9001_a3"], g["rfc9001_a1"]["server"]
    k, iv, hp = B(sk["key"]), B(sk["iv"]), B(sk["hp"])
    pkt = B(a3["header"] + a3["payload"])
    prot, r = ol.quic_seal(k, iv, hp, a3["pn"], pkt, a3["pn_offset"], suite=ol.AES128GCM)
    assert r == len(pkt) + 16 and prot.hex() == a3["protected"]
    back, r, pn = ol.quic_open(k, iv, hp, 0, prot, a3["pn_offset"], suite=ol.AES128GCM)
    assert r == len(pkt) and back == pkt and pn == a3["pn"]
    for v in g["packets"]:
        k, iv, hp = B(v["key"]), B(v["iv"]), B(v["hp"])
        pkt = B(v["packet"])
        prot, r = ol.quic_seal(k, iv, hp, v["pn"], pkt, v["pn_offset"], suite=ol.AES128GCM)
        assert prot.hex() == v["protected"]
        back, r, pn = ol.quic_open(k, iv, hp, v["largest_pn"], prot, v["pn_offset"],
                                   suite=ol.AES128GCM)
        assert r == len(pkt) and back == pkt and pn == v["pn"]
        bad = bytearray(prot)
        bad[-1] ^= 1
        assert ol.quic_open(k, iv, hp, v["largest_pn"], bytes(bad), v["pn_offset"],
                            suite=ol.AES128GCM)[1] == -2
