"""Generate tests/golden/*.json from the hashlib-based restatement
(oracle/py_oracle.py).  Run from the repo root:

    python tests/golden/make_golden.py

The reference (Go) ships no vectors and cannot run here, so these fixtures are
produced by an independent restatement whose primitives are themselves pinned
by published known-answer tests (kat.json, checked in tests/test_oracle.py).
Deterministic: numpy PCG64 with fixed seeds.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import py_oracle as po  # noqa: E402

PAYLOAD_LENS = [0, 1, 2, 3, 7, 8, 9, 15, 16, 17, 23, 24, 25, 31, 32, 33, 47, 48, 63, 64,
                65, 100, 127, 128, 129, 255, 256, 257, 1200, 1350, 1452, 1500]
# PSK lengths crossing BLAKE2b's 120/128-byte and SHA-256's 39/55/64-byte
# boundaries (the salt and padding then spill into a second block)
PSK_LENS = [0, 1, 8, 26, 38, 39, 40, 47, 48, 55, 56, 63, 64, 65, 103, 104, 119, 120, 121,
            127, 128, 129, 200, 255, 256, 257, 300]


def hx(b: bytes) -> str:
    return b.hex()


def kat() -> dict:
    """Published known answers (RFC 7693 Appendix A; FIPS 180-2 examples)
    plus hashlib values for the BLAKE2b-256 cases the reference uses."""
    return {
        "blake2b512_abc_rfc7693": {
            "msg": hx(b"abc"), "outlen": 64,
            "digest": "ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
                      "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923"},
        "blake2b256": [
            {"msg": hx(m), "digest": hashlib.blake2b(m, digest_size=32).hexdigest()}
            for m in [b"", b"abc", bytes(range(128)), bytes(range(129)), bytes(255 for _ in range(256))]],
        "sha256_fips180": [
            {"msg": hx(b"abc"),
             "digest": "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"},
            {"msg": hx(b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"),
             "digest": "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"},
            {"msg": "", "digest": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"},
        ],
        "sha256": [
            {"msg": hx(m), "digest": hashlib.sha256(m).hexdigest()}
            for m in [bytes(range(55)), bytes(range(56)), bytes(range(64)), bytes(range(119))]],
    }


def survey_examples() -> list[dict]:
    """The two worked examples of SURVEY.md section 0."""
    psk = b"password"
    s8 = bytes(range(8))
    p = b"hello, salamander! 0123456789abcdef"
    wire, _ = po.salamander_write(psk, s8, p)
    s16 = bytes(range(16))
    q = b"hello, xplus! 0123456789abcdefghij"
    wire2, _ = po.xplus_write(psk, s16, q)
    return [
        {"kind": "salamander", "psk": hx(psk), "salt": hx(s8), "payload": hx(p),
         "key": hx(po.salamander_key(psk, s8)), "wire": hx(wire)},
        {"kind": "xplus", "psk": hx(psk), "salt": hx(s16), "payload": hx(q),
         "key": hx(po.xplus_key(psk, s16)), "wire": hx(wire2)},
    ]


def transform_vectors(kind: str, rng: np.random.Generator) -> list[dict]:
    S = 8 if kind == "salamander" else 16
    write = po.salamander_write if kind == "salamander" else po.xplus_write
    keyf = po.salamander_key if kind == "salamander" else po.xplus_key
    out = []
    cases = [(pl, 26) for pl in PAYLOAD_LENS] + [(37, kl) for kl in PSK_LENS] + \
            [(1350, kl) for kl in (0, 39, 40, 121, 128, 300)]
    for L, K in cases:
        psk = rng.integers(0, 256, K, dtype=np.uint8).tobytes()
        salt = rng.integers(0, 256, S, dtype=np.uint8).tobytes()
        pay = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        wire, wret = write(psk, salt, pay)
        out.append({"psk": hx(psk), "salt": hx(salt), "payload": hx(pay),
                    "key": hx(keyf(psk, salt)), "wire": hx(wire), "write_ret": wret})
    return out


def read_vectors(kind: str, rng: np.random.Generator) -> list[dict]:
    """ReadFrom on raw datagrams, including the short-datagram quirks and,
    for XPlus, a read buffer longer than the datagram (xplus.go:55)."""
    S = 8 if kind == "salamander" else 16
    out = []
    psk = b"sing-quic-mi355x-bench-psk"
    for n in [0, 1, 7, 8, 9, 15, 16, 17, 24, 40, 41, 1358, 1216]:
        dgram = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        if kind == "salamander":
            buf, ret = po.salamander_read(psk, dgram)
            out.append({"psk": hx(psk), "datagram": hx(dgram), "cap": n,
                        "buffer_after": hx(buf), "read_ret": ret})
        else:
            for extra in (0, 5, 40):
                cap = n + extra
                full = dgram + rng.integers(0, 256, extra, dtype=np.uint8).tobytes()
                buf, ret = po.xplus_read(psk, full, n)
                out.append({"psk": hx(psk), "datagram": hx(full[:n]), "cap": cap,
                            "buffer_full": hx(full), "buffer_after": hx(buf), "read_ret": ret})
    return out


def vectorised_vectors(rng: np.random.Generator) -> list[dict]:
    """Multi-buffer writes: XPlus's running keystream (xplus.go:108-115) and
    Salamander's literal line-104 behaviour (panics for a second non-empty
    buffer)."""
    psk = b"vectorised-psk"
    out = []
    for lens in ([5], [40], [0, 33], [16, 16], [3, 50, 7], [32, 0, 1]):
        bufs = [rng.integers(0, 256, k, dtype=np.uint8).tobytes() for k in lens]
        s8 = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
        s16 = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        sal, panicked = po.salamander_write_vectorised(psk, s8, bufs)
        xp = po.xplus_write_vectorised(psk, s16, bufs)
        out.append({"psk": hx(psk), "bufs": [hx(b) for b in bufs],
                    "salamander_salt": hx(s8), "salamander_out": [hx(b) for b in sal],
                    "salamander_panics": panicked,
                    "xplus_salt": hx(s16), "xplus_out": [hx(b) for b in xp]})
    return out


def main() -> None:
    rng = np.random.Generator(np.random.PCG64(20260213))
    files = {
        "kat.json": kat(),
        "survey_examples.json": survey_examples(),
        "salamander_write.json": transform_vectors("salamander", rng),
        "xplus_write.json": transform_vectors("xplus", rng),
        "salamander_read.json": read_vectors("salamander", rng),
        "xplus_read.json": read_vectors("xplus", rng),
        "vectorised.json": vectorised_vectors(rng),
    }
    for name, obj in files.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=0, sort_keys=True)
            f.write("\n")
    print("wrote", ", ".join(files))


if __name__ == "__main__":
    main()
