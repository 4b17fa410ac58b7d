"""Generate tests/golden/chacha20.json: ChaCha20 keystream vectors for the
device salt generator (SQOBFS_FLAG_DEVICE_SALT).  Run from the repo root:

    python tests/golden/make_chacha.py

Expected outputs come from OpenSSL's chacha20 (`openssl enc -chacha20`, an
implementation independent of oracle/oracle.c and of the GPU kernel), plus
the published RFC 8439 section 2.3.2 block.  OpenSSL's 16-byte IV is the
32-bit little-endian block counter followed by the 96-bit nonce.
Deterministic: numpy PCG64 with fixed seeds.
"""
from __future__ import annotations

import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# RFC 8439 section 2.3.2: key 00..1f, nonce 000000090000004a00000000, counter 1
RFC8439_232 = ("10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
               "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


def openssl_stream(key: bytes, nonce: bytes, counter0: int, n: int) -> bytes:
    iv = counter0.to_bytes(4, "little") + nonce
    out = subprocess.run(["openssl", "enc", "-chacha20", "-K", key.hex(), "-iv", iv.hex()],
                         input=bytes(n), capture_output=True, check=True).stdout
    assert len(out) == n
    return out


def salt_nonce(seq: int) -> bytes:
    return b"sqob" + seq.to_bytes(8, "little")


def main() -> None:
    rng = np.random.Generator(np.random.PCG64(8439))
    rfc_key = bytes(range(32))
    rfc_nonce = bytes.fromhex("000000090000004a00000000")
    got = openssl_stream(rfc_key, rfc_nonce, 1, 64)
    assert got.hex() == RFC8439_232, "openssl disagrees with RFC 8439 2.3.2"
    streams = [{"key": rfc_key.hex(), "nonce": rfc_nonce.hex(), "counter": 1,
                "stream": RFC8439_232, "source": "RFC 8439 section 2.3.2 (and openssl)"}]
    for n in (1, 7, 63, 64, 65, 200, 1000, 4096):
        key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        nonce = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        ctr = int(rng.integers(0, 2**32 - 200))
        streams.append({"key": key.hex(), "nonce": nonce.hex(), "counter": ctr,
                        "stream": openssl_stream(key, nonce, ctr, n).hex(), "source": "openssl"})
    salts = []
    for S in (8, 16):
        for seq, n in ((0, 1), (0, 100), (1, 100), (2**32 + 5, 37), (2**63 + 1, 64)):
            key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
            salts.append({"S": S, "key": key.hex(), "seq": seq, "n": n,
                          "salts": openssl_stream(key, salt_nonce(seq), 0, n * S).hex()})
    out = {"_doc": "ChaCha20 keystreams (RFC 8439) from openssl; device salts = "
                   "ChaCha20(key, 'sqob' || le64(seq), counter 0)[0:n*S]",
           "streams": streams, "device_salts": salts}
    with open(os.path.join(HERE, "chacha20.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote chacha20.json:", len(streams), "streams,", len(salts), "salt sets")


if __name__ == "__main__":
    main()
