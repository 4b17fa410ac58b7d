"""The lane-pair ChaCha20 block of the QUIC kernel's owner phases
(sing-quic_amd/csrc/sq_quic.hip chacha20_pair, lane pairs), emulated on the
CPU: lane l holds state columns 0-1, lane l + 32 columns 2-3, and the
diagonal round exchanges 4 words each way (v_permlane32_swap).  The two
halves' outputs must put together the RFC 8439 2.3 block, checked against
the oracle's ChaCha20 (itself pinned by RFC 8439 2.3.2 and OpenSSL in
test_oracle.py).  The GPU kernels that use it are checked bit for bit by
test_gpu_quic*.py."""
from __future__ import annotations

import struct

import numpy as np

import oracle_lib as ol

M = 0xFFFFFFFF


def rotl(x: int, n: int) -> int:
    return ((x << n) | (x >> (32 - n))) & M


def qr(s: list, a: int, b: int, c: int, d: int) -> None:
    s[a] = (s[a] + s[b]) & M; s[d] = rotl(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & M; s[b] = rotl(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b]) & M; s[d] = rotl(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & M; s[b] = rotl(s[b] ^ s[c], 7)


def chacha20_pair(key: list, counter: int, nonce: list) -> tuple:
    """Both lanes of chacha20_pair in lockstep; lane state = [a0, a1, b0,
    b1, c0, c1, d0, d1]; x(v) = the partner lane's v."""
    ins = [[0x61707865, 0x3320646E, key[0], key[1], key[4], key[5], counter, nonce[0]],
           [0x79622D32, 0x6B206574, key[2], key[3], key[6], key[7], nonce[1], nonce[2]]]
    st = [list(ins[0]), list(ins[1])]
    for _ in range(10):
        for s in st:  # column round: local
            qr(s, 0, 2, 4, 6)
            qr(s, 1, 3, 5, 7)
        # diagonalise: b = (b1, x(b0)), c = (x(c0), x(c1)), d = (x(d1), d0)
        new = []
        for h in (0, 1):
            s, o = st[h], st[1 - h]
            new.append([s[0], s[1], s[3], o[2], o[4], o[5], o[7], s[6]])
        st = new
        for s in st:
            qr(s, 0, 2, 4, 6)
            qr(s, 1, 3, 5, 7)
        # back: b = (x(e1), e0), c = (x(f0), x(f1)), d = (g1, x(g0))
        new = []
        for h in (0, 1):
            s, o = st[h], st[1 - h]
            new.append([s[0], s[1], o[3], s[2], o[4], o[5], s[7], o[6]])
        st = new
    return tuple([(v + i) & M for v, i in zip(st[h], ins[h])] for h in (0, 1))


def block_words(lo: list, hi: list) -> list:
    """Reassemble x0..x15 from the low lane's words 0,1,4,5,8,9,12,13 and
    the high lane's 2,3,6,7,10,11,14,15."""
    out = [0] * 16
    for r in range(4):
        out[4 * r + 0], out[4 * r + 1] = lo[2 * r], lo[2 * r + 1]
        out[4 * r + 2], out[4 * r + 3] = hi[2 * r], hi[2 * r + 1]
    return out


def check(key: bytes, counter: int, nonce: bytes, want: bytes | None = None) -> None:
    kw = list(struct.unpack("<8I", key))
    nw = list(struct.unpack("<3I", nonce))
    lo, hi = chacha20_pair(kw, counter, nw)
    got = struct.pack("<16I", *block_words(lo, hi))
    assert got == ol.chacha20_stream(key, nonce, counter, 64)
    if want is not None:
        assert got == want


def test_lanepair_rfc8439_block(golden):
    """RFC 8439 2.3.2's block and the committed keystreams (RFC 8439 and
    OpenSSL, tests/golden/make_chacha.py): the first block of each."""
    check(bytes(range(32)), 1, bytes.fromhex("000000090000004a00000000"))
    streams = golden("chacha20.json")["streams"]
    assert streams[0]["source"].startswith("RFC 8439")
    for v in streams:
        s = bytes.fromhex(v["stream"])
        if len(s) >= 64:
            check(bytes.fromhex(v["key"]), v["counter"], bytes.fromhex(v["nonce"]), s[:64])


def test_lanepair_random_blocks():
    """Random keys, counters (the header-protection sample's first word is
    any 32-bit value) and nonces."""
    rng = np.random.Generator(np.random.PCG64(3232))
    for _ in range(200):
        key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        nonce = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        check(key, int(rng.integers(0, 1 << 32)), nonce)


def test_lanepair_otk_and_mask_words():
    """What the kernel takes from the halves: the Poly1305 key otk[0..8)
    (low lane words 0,1,4,5 + the high lane's 2,3,6,7 over the swap) and
    the mask words 0 and 1 (low lane only)."""
    rng = np.random.Generator(np.random.PCG64(9001))
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    nonce = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    lo, hi = chacha20_pair(list(struct.unpack("<8I", key)), 0, list(struct.unpack("<3I", nonce)))
    otk = [lo[0], lo[1], hi[0], hi[1], lo[2], lo[3], hi[2], hi[3]]
    assert struct.pack("<8I", *otk) == ol.chacha20_stream(key, nonce, 0, 32)
    assert struct.pack("<2I", lo[0], lo[1]) == ol.chacha20_stream(key, nonce, 0, 8)
