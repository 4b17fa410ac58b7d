"""Generate tests/golden/quic_gcm.json: vectors for the TLS_AES_128_GCM_SHA256
QUIC path (AES-128-GCM payload protection + AES header protection, RFC 9001
5.3 / 5.4.3).  Run from the repo root:

    python tests/golden/make_quic_gcm.py

Independent sources only (not oracle/oracle.c, not the GPU kernel):
  * AES-128: FIPS-197 Appendix B and C.1 examples, and OpenSSL (EVP_aes_128_ecb);
  * GCM: McGrew & Viega GCM specification test cases 1-4 (as reproduced in
    NIST's GCM validation examples), and OpenSSL (EVP_aes_128_gcm, ctypes);
  * RFC 9001 Appendix A.1 (Initial keys, re-derived here by HKDF from the
    initial salt and the client's DCID) and A.3 (server Initial packet);
    each literal from those documents is kept only because OpenSSL
    reproduces it here (asserted).
Deterministic: numpy PCG64 with fixed seeds.
"""
from __future__ import annotations

import ctypes
import hashlib
import hmac
import json
import os

import numpy as np

from make_quic import hkdf_expand_label

HERE = os.path.dirname(os.path.abspath(__file__))
B = bytes.fromhex

FIPS197 = [  # (key, plaintext, ciphertext)
    ("000102030405060708090a0b0c0d0e0f", "00112233445566778899aabbccddeeff",
     "69c4e0d86a7b0430d8cdb78070b4c55a"),
    ("2b7e151628aed2a6abf7158809cf4f3c", "3243f6a8885a308d313198a2e0370734",
     "3925841d02dc09fbdc118597196a0b32"),
]
_K3, _IV3 = "feffe9928665731c6d6a8f9467308308", "cafebabefacedbaddecaf888"
_P3 = ("d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a72"
       "1c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b391aafd255")
GCM_CASES = [  # (key, nonce, aad, pt, ct || tag)
    ("00" * 16, "00" * 12, "", "", "58e2fccefa7e3061367f1d57a4e7455a"),
    ("00" * 16, "00" * 12, "", "00" * 16,
     "0388dace60b6a392f328c2b971b2fe78ab6e47d42cec13bdf53a67b21257bddf"),
    (_K3, _IV3, "", _P3,
     "42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e"
     "21d514b25466931c7d8f6a5aac84aa051ba30b396a0aac973d58e091473f5985"
     "4d5c2af327cd64a62cf35abd2ba6fab4"),
    (_K3, _IV3, "feedfacedeadbeeffeedfacedeadbeefabaddad2", _P3[:120],
     "42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e"
     "21d514b25466931c7d8f6a5aac84aa051ba30b396a0aac973d58e091"
     "5bc94fbc3221a5db94fae95ae7121a47"),
]
RFC9001_A1 = {
    "initial_salt": "38762cf7f55934b34d179ae6a4c80cadccbb7f0a",
    "dcid": "8394c8f03e515708",
    "client": {"key": "1f369613dd76d5467730efcbe3b1a22d", "iv": "fa044b2f42a3fd3b46fb255c",
               "hp": "9f50449e04a0e810283a1e9933adedd2"},
    "server": {"key": "cf3a5331653c364c88f0f379b6067e37", "iv": "0ac1493ca1905853b0bba03e",
               "hp": "c206b8d9b9f0f37644430b490eeaa314"},
}
RFC9001_A3 = {
    "header": "c1000000010008f067a5502a4262b50040750001",
    "payload": "02000000000600405a020000560303eefce7f7b37ba1d1632e96677825ddf73988cfc79825"
               "df566dc5430b9a045a1200130100002e00330024001d00209d3c940d89690b84d08a6099"
               "3c144eca684d1081287c834d5311bcf32bb9da1a002b00020304",
    "pn": 1,
    "pn_offset": 18,
    "protected": "cf000000010008f067a5502a4262b5004075c0d95a482cd0991cd25b0aac406a5816b639"
                 "4100f37a1c69797554780bb38cc5a99f5ede4cf73c3ec2493a1839b3dbcba3f6ea46c5b7"
                 "684df3548e7ddeb9c3bf9c73cc3f3bded74b562bfb19fb84022f8ef4cdd93795d77d06ed"
                 "bb7aaf2f58891850abbdca3d20398c276456cbc42158407dd074ee",
}

_L = ctypes.CDLL("libcrypto.so.3")
_L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
_L.EVP_aes_128_gcm.restype = ctypes.c_void_p
_L.EVP_aes_128_ecb.restype = ctypes.c_void_p
_L.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_char_p] * 2
_L.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                 ctypes.c_char_p, ctypes.c_int]
_L.EVP_EncryptFinal_ex.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
_L.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
_L.EVP_CIPHER_CTX_set_padding.argtypes = [ctypes.c_void_p, ctypes.c_int]
_L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]


def aes_ecb(key: bytes, block: bytes) -> bytes:
    c = _L.EVP_CIPHER_CTX_new()
    assert _L.EVP_EncryptInit_ex(c, _L.EVP_aes_128_ecb(), None, key, None) == 1
    _L.EVP_CIPHER_CTX_set_padding(c, 0)
    out, n = ctypes.create_string_buffer(32), ctypes.c_int(0)
    assert _L.EVP_EncryptUpdate(c, out, ctypes.byref(n), block, 16) == 1 and n.value == 16
    _L.EVP_CIPHER_CTX_free(c)
    return out.raw[:16]


def gcm_seal(key: bytes, nonce: bytes, aad: bytes, pt: bytes) -> bytes:
    c = _L.EVP_CIPHER_CTX_new()
    assert _L.EVP_EncryptInit_ex(c, _L.EVP_aes_128_gcm(), None, key, nonce) == 1
    n = ctypes.c_int(0)
    if aad:
        assert _L.EVP_EncryptUpdate(c, None, ctypes.byref(n), aad, len(aad)) == 1
    out = ctypes.create_string_buffer(len(pt) + 16)
    if pt:
        assert _L.EVP_EncryptUpdate(c, out, ctypes.byref(n), pt, len(pt)) == 1
    assert _L.EVP_EncryptFinal_ex(c, out, ctypes.byref(n)) == 1
    tag = ctypes.create_string_buffer(16)
    assert _L.EVP_CIPHER_CTX_ctrl(c, 0x10, 16, tag) == 1  # EVP_CTRL_AEAD_GET_TAG
    _L.EVP_CIPHER_CTX_free(c)
    return out.raw[:len(pt)] + tag.raw


def quic_seal(key, iv, hp, pn, pkt, pn_offset):
    """RFC 9001 5.3 + 5.4.3 with OpenSSL primitives."""
    pn_len = (pkt[0] & 3) + 1
    hdr = pn_offset + pn_len
    nonce = bytes(a ^ b for a, b in zip(iv, pn.to_bytes(12, "big")))
    out = bytearray(pkt[:hdr] + gcm_seal(key, nonce, pkt[:hdr], pkt[hdr:]))
    mask = aes_ecb(hp, bytes(out[pn_offset + 4:pn_offset + 20]))
    out[0] ^= mask[0] & (0x0F if out[0] & 0x80 else 0x1F)
    for i in range(pn_len):
        out[pn_offset + i] ^= mask[1 + i]
    return bytes(out)


def main() -> None:
    for k, p, c in FIPS197:
        assert aes_ecb(B(k), B(p)).hex() == c
    for k, n, a, p, ct in GCM_CASES:
        assert gcm_seal(B(k), B(n), B(a), B(p)).hex() == ct
    a1 = RFC9001_A1
    init = hmac.new(B(a1["initial_salt"]), B(a1["dcid"]), hashlib.sha256).digest()
    for side, label in (("client", b"client in"), ("server", b"server in")):
        sec = hkdf_expand_label(init, label, 32)
        for what, n in (("key", 16), ("iv", 12), ("hp", 16)):
            assert hkdf_expand_label(sec, b"quic " + what.encode(), n).hex() == a1[side][what]
    a3, sk = RFC9001_A3, a1["server"]
    got = quic_seal(B(sk["key"]), B(sk["iv"]), B(sk["hp"]), a3["pn"],
                    B(a3["header"] + a3["payload"]), a3["pn_offset"])
    assert got.hex() == a3["protected"], "OpenSSL disagrees with RFC 9001 A.3"

    rng = np.random.Generator(np.random.PCG64(9003))
    rb = lambda n: rng.integers(0, 256, n, dtype=np.uint8).tobytes()  # noqa: E731
    aes = [{"key": k, "pt": p, "ct": c, "source": "FIPS-197"} for k, p, c in FIPS197]
    for _ in range(8):
        k, p = rb(16), rb(16)
        aes.append({"key": k.hex(), "pt": p.hex(), "ct": aes_ecb(k, p).hex(), "source": "openssl"})
    gcm = [{"key": k, "nonce": n, "aad": a, "pt": p, "ct_tag": ct, "source": "GCM spec"}
           for k, n, a, p, ct in GCM_CASES]
    for aad_n, n in ((0, 1), (1, 15), (12, 17), (16, 64), (21, 65), (33, 127), (7, 1350),
                     (20, 1452), (5, 4000)):
        key, nonce, aad, pt = rb(16), rb(12), rb(aad_n), rb(n)
        gcm.append({"key": key.hex(), "nonce": nonce.hex(), "aad": aad.hex(), "pt": pt.hex(),
                    "ct_tag": gcm_seal(key, nonce, aad, pt).hex(), "source": "openssl"})
    packets = []
    for i in range(40):
        key, iv, hp = rb(16), rb(12), rb(16)
        pn_len = 1 + i % 4
        dcid = int(rng.integers(0, 21))
        long_hdr = i % 5 == 4
        first = (0xC0 if long_hdr else 0x40) | int(rng.integers(0, 16)) << 2 & 0x3C | (pn_len - 1)
        pn_offset = 1 + dcid + (6 if long_hdr else 0)
        pn = int(rng.integers(0, 2**62)) if i % 3 else int(rng.integers(0, 2**16))
        trunc = pn & ((1 << (8 * pn_len)) - 1)
        plen = max(4 - pn_len, int(rng.integers(0, 1500)) if i % 7 else 4 - pn_len)
        pkt = bytes([first]) + rb(pn_offset - 1) + trunc.to_bytes(pn_len, "big") + rb(plen)
        largest = max(0, pn - int(rng.integers(1, 2 ** (8 * pn_len - 2))))
        packets.append({"key": key.hex(), "iv": iv.hex(), "hp": hp.hex(), "pn": pn,
                        "largest_pn": largest, "pn_offset": pn_offset, "packet": pkt.hex(),
                        "protected": quic_seal(key, iv, hp, pn, pkt, pn_offset).hex()})
    out = {"_doc": "QUIC AES-128-GCM packet protection vectors (FIPS-197, GCM spec, RFC 9001 "
                   "A.1/A.3) checked against OpenSSL; see make_quic_gcm.py",
           "rfc9001_a1": a1, "rfc9001_a3": a3, "aes": aes, "gcm": gcm, "packets": packets}
    with open(os.path.join(HERE, "quic_gcm.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote quic_gcm.json:", len(aes), "aes,", len(gcm), "gcm,", len(packets), "packets")


if __name__ == "__main__":
    main()
