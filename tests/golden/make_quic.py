"""Generate tests/golden/quic.json: QUIC packet protection vectors for the
ChaCha20-Poly1305 path.  Run from the repo root:

    python tests/golden/make_quic.py

Independent sources only (not oracle/oracle.c, not the GPU kernel):
  * Poly1305: RFC 8439 section 2.5.2 and `openssl mac POLY1305`;
  * AEAD_CHACHA20_POLY1305: OpenSSL libcrypto (EVP_chacha20_poly1305, ctypes);
  * header protection masks: `openssl enc -chacha20` (RFC 9001 5.4.4);
  * RFC 9001 Appendix A.5 (ChaCha20-Poly1305 short header packet), with its
    key / iv / hp re-derived here by HKDF-Expand-Label (hmac + hashlib).
Deterministic: numpy PCG64 with fixed seeds.
"""
from __future__ import annotations

import ctypes
import hashlib
import hmac
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

RFC9001_A5 = {
    "secret": "9ac312a7f877468ebe69422748ad00a15443f18203a07d6060f688f30f21632b",
    "key": "c6d98ff3441c3fe1b2182094f69caa2ed4b716b65488960a7a984979fb23e1c8",
    "iv": "e0459b3474bdd0e44a41c144",
    "hp": "25a282b9e82f06f21f488917a4fc8f1b73573685608597d0efcb076b0ab7a7a4",
    "pn": 654360564,
    "header": "4200bff4",
    "payload": "01",
    "pn_offset": 1,
    "protected": "4cfe4189655e5cd55c41f69080575d7999c25a5bfb",
}
RFC8439_252 = {"key": "85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b",
               "msg": b"Cryptographic Forum Research Group".hex(),
               "tag": "a8061dc1305136c6c22b8baf0c0127a9"}

_L = ctypes.CDLL("libcrypto.so.3")
_L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
_L.EVP_chacha20_poly1305.restype = ctypes.c_void_p
_L.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_char_p] * 2
_L.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                 ctypes.c_char_p, ctypes.c_int]
_L.EVP_EncryptFinal_ex.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
_L.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
_L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]


def aead_seal(key: bytes, nonce: bytes, aad: bytes, pt: bytes) -> bytes:
    c = _L.EVP_CIPHER_CTX_new()
    assert _L.EVP_EncryptInit_ex(c, _L.EVP_chacha20_poly1305(), None, key, nonce) == 1
    n = ctypes.c_int(0)
    if aad:
        assert _L.EVP_EncryptUpdate(c, None, ctypes.byref(n), aad, len(aad)) == 1
    out = ctypes.create_string_buffer(len(pt) + 1)
    if pt:
        assert _L.EVP_EncryptUpdate(c, out, ctypes.byref(n), pt, len(pt)) == 1
    assert _L.EVP_EncryptFinal_ex(c, out, ctypes.byref(n)) == 1
    tag = ctypes.create_string_buffer(16)
    assert _L.EVP_CIPHER_CTX_ctrl(c, 0x10, 16, tag) == 1  # EVP_CTRL_AEAD_GET_TAG
    _L.EVP_CIPHER_CTX_free(c)
    return out.raw[:len(pt)] + tag.raw


def chacha_mask(hp: bytes, sample: bytes) -> bytes:
    return subprocess.run(["openssl", "enc", "-chacha20", "-K", hp.hex(), "-iv", sample.hex()],
                          input=bytes(5), capture_output=True, check=True).stdout


def poly1305_openssl(key: bytes, msg: bytes) -> bytes:
    path = os.path.join("/tmp", f"sq_poly_{os.getpid()}.bin")
    with open(path, "wb") as f:
        f.write(msg)
    out = subprocess.run(["openssl", "mac", "-macopt", "hexkey:" + key.hex(), "-in", path,
                          "POLY1305"], capture_output=True, check=True, text=True).stdout
    os.unlink(path)
    return bytes.fromhex(out.strip())


def hkdf_expand_label(secret: bytes, label: bytes, length: int) -> bytes:
    full = b"tls13 " + label
    info = length.to_bytes(2, "big") + bytes([len(full)]) + full + b"\x00"
    out, t, i = b"", b"", 1
    while len(out) < length:
        t = hmac.new(secret, t + info + bytes([i]), hashlib.sha256).digest()
        out += t
        i += 1
    return out[:length]


def quic_seal(key, iv, hp, pn, pkt, pn_offset):
    """RFC 9001 5.3 + 5.4 with OpenSSL primitives."""
    pn_len = (pkt[0] & 3) + 1
    hdr = pn_offset + pn_len
    nonce = bytes(a ^ b for a, b in zip(iv, pn.to_bytes(12, "big")))
    body = aead_seal(key, nonce, pkt[:hdr], pkt[hdr:])
    out = bytearray(pkt[:hdr] + body)
    mask = chacha_mask(hp, bytes(out[pn_offset + 4:pn_offset + 20]))
    out[0] ^= mask[0] & (0x0F if out[0] & 0x80 else 0x1F)
    for i in range(pn_len):
        out[pn_offset + i] ^= mask[1 + i]
    return bytes(out)


def main() -> None:
    a5 = dict(RFC9001_A5)
    sec = bytes.fromhex(a5["secret"])
    assert hkdf_expand_label(sec, b"quic key", 32).hex() == a5["key"]
    assert hkdf_expand_label(sec, b"quic iv", 12).hex() == a5["iv"]
    assert hkdf_expand_label(sec, b"quic hp", 32).hex() == a5["hp"]
    got = quic_seal(bytes.fromhex(a5["key"]), bytes.fromhex(a5["iv"]), bytes.fromhex(a5["hp"]),
                    a5["pn"], bytes.fromhex(a5["header"] + a5["payload"]), a5["pn_offset"])
    assert got.hex() == a5["protected"], "OpenSSL disagrees with RFC 9001 A.5"
    assert poly1305_openssl(bytes.fromhex(RFC8439_252["key"]),
                            bytes.fromhex(RFC8439_252["msg"])).hex() == RFC8439_252["tag"]

    rng = np.random.Generator(np.random.PCG64(9001))
    rb = lambda n: rng.integers(0, 256, n, dtype=np.uint8).tobytes()  # noqa: E731
    polys = [dict(RFC8439_252, source="RFC 8439 2.5.2")]
    for n in (0, 1, 15, 16, 17, 63, 64, 65, 300, 1500):
        key, msg = rb(32), rb(n)
        polys.append({"key": key.hex(), "msg": msg.hex(),
                      "tag": poly1305_openssl(key, msg).hex(), "source": "openssl mac"})
    aeads = []
    for aad_n, n in ((0, 0), (1, 0), (12, 1), (16, 16), (21, 63), (33, 64), (7, 1350),
                     (20, 1452), (5, 4000)):
        key, nonce, aad, pt = rb(32), rb(12), rb(aad_n), rb(n)
        aeads.append({"key": key.hex(), "nonce": nonce.hex(), "aad": aad.hex(), "pt": pt.hex(),
                      "ct_tag": aead_seal(key, nonce, aad, pt).hex()})
    packets = []
    for i in range(40):
        key, iv, hp = rb(32), rb(12), rb(32)
        pn_len = 1 + i % 4
        dcid = int(rng.integers(0, 21))
        long_hdr = i % 5 == 4
        first = (0xC0 if long_hdr else 0x40) | int(rng.integers(0, 16)) << 2 & 0x3C | (pn_len - 1)
        pn_offset = 1 + dcid + (6 if long_hdr else 0)
        pn = int(rng.integers(0, 2**62)) if i % 3 else int(rng.integers(0, 2**16))
        trunc = pn & ((1 << (8 * pn_len)) - 1)
        plen = max(4 - pn_len, int(rng.integers(0, 1500)) if i % 7 else 4 - pn_len)
        pkt = bytes([first]) + rb(pn_offset - 1) + trunc.to_bytes(pn_len, "big") + rb(plen)
        # largest received pn close to pn, so the truncated pn decodes uniquely
        largest = max(0, pn - int(rng.integers(1, 2 ** (8 * pn_len - 2))))
        packets.append({"key": key.hex(), "iv": iv.hex(), "hp": hp.hex(), "pn": pn,
                        "largest_pn": largest, "pn_offset": pn_offset, "packet": pkt.hex(),
                        "protected": quic_seal(key, iv, hp, pn, pkt, pn_offset).hex()})
    out = {"_doc": "QUIC ChaCha20-Poly1305 packet protection vectors (RFC 8439, RFC 9001) "
                   "from OpenSSL; see make_quic.py",
           "rfc9001_a5": a5, "poly1305": polys, "aead": aeads, "packets": packets}
    with open(os.path.join(HERE, "quic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote quic.json:", len(polys), "poly1305,", len(aeads), "aead,", len(packets), "packets")


if __name__ == "__main__":
    main()
