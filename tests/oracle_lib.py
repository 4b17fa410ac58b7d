"""ctypes access to the CPU restatement oracle/liboracle.so (test checker only)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")

SALAMANDER, XPLUS = 0, 1
OBFUSCATE, DEOBFUSCATE = 0, 1


class OrBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("in_", ctypes.c_void_p), ("in_off", ctypes.c_void_p),
                ("in_len", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("out_off", ctypes.c_void_p), ("out_len", ctypes.c_void_p),
                ("salt", ctypes.c_void_p), ("psk_id", ctypes.c_void_p),
                ("in_cap", ctypes.c_void_p)]


class OrPsks(ctypes.Structure):
    _fields_ = [("blob", ctypes.c_void_p), ("off", ctypes.c_void_p), ("len", ctypes.c_void_p),
                ("count", ctypes.c_uint32)]


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
        L = ctypes.CDLL(ORACLE_SO)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.or_blake2b.argtypes = [vp, sz, vp, sz]
        L.or_blake2b256.argtypes = [vp, sz, vp]
        L.or_sha256.argtypes = [vp, sz, vp]
        L.or_salamander_key.argtypes = [vp, sz, vp, vp]
        L.or_xplus_key.argtypes = [vp, sz, vp, vp]
        L.or_salamander_write.argtypes = [vp, sz, vp, vp, sz, vp]
        L.or_salamander_write.restype = ctypes.c_long
        L.or_salamander_read.argtypes = [vp, sz, vp, sz]
        L.or_salamander_read.restype = ctypes.c_long
        L.or_salamander_write_inplace.argtypes = [vp, sz, vp, vp, sz]
        L.or_salamander_write_inplace.restype = ctypes.c_long
        L.or_salamander_write_vectorised.argtypes = [vp, sz, vp, vp, vp, sz]
        L.or_xplus_write.argtypes = [vp, sz, vp, vp, sz, vp]
        L.or_xplus_write.restype = ctypes.c_long
        L.or_xplus_read.argtypes = [vp, sz, vp, sz, sz]
        L.or_xplus_read.restype = ctypes.c_long
        L.or_xplus_write_vectorised.argtypes = [vp, sz, vp, vp, vp, sz]
        L.or_xplus_write_vectorised.restype = None
        L.or_chacha20_block.argtypes = [vp, ctypes.c_uint32, vp, vp]
        L.or_chacha20_block.restype = None
        L.or_chacha20_stream.argtypes = [vp, vp, ctypes.c_uint32, vp, sz]
        L.or_chacha20_stream.restype = None
        L.or_device_salts.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, vp]
        L.or_device_salts.restype = None
        L.or_poly1305.argtypes = [vp, vp, sz, vp]
        L.or_poly1305.restype = None
        L.or_aead_seal.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp]
        L.or_aead_seal.restype = None
        L.or_quic_seal.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, sz, sz, vp]
        L.or_quic_seal.restype = ctypes.c_long
        L.or_quic_open.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, sz, sz, vp,
                                   ctypes.POINTER(ctypes.c_uint64)]
        L.or_quic_open.restype = ctypes.c_long
        L.or_quic_seal_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_uint32, vp, vp,
                                         ctypes.c_int]
        L.or_quic_seal_batch2.argtypes = [ctypes.c_int] + L.or_quic_seal_batch.argtypes
        L.or_quic_seal2.argtypes = [ctypes.c_int] + L.or_quic_seal.argtypes
        L.or_quic_seal2.restype = ctypes.c_long
        L.or_quic_open2.argtypes = [ctypes.c_int] + L.or_quic_open.argtypes
        L.or_quic_open2.restype = ctypes.c_long
        L.or_aes_sbox.argtypes = [ctypes.c_uint8]
        L.or_aes_sbox.restype = ctypes.c_uint8
        L.or_aes128_expand.argtypes = [vp, vp]
        L.or_aes128_expand.restype = None
        L.or_aes128_encrypt.argtypes = [vp, vp, vp]
        L.or_aes128_encrypt.restype = None
        L.or_gf128_mul.argtypes = [vp, vp, vp]
        L.or_gf128_mul.restype = None
        L.or_gcm_crypt.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, ctypes.c_int]
        L.or_gcm_crypt.restype = None
        L.or_batch_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(OrPsks),
                                   ctypes.POINTER(OrBatch), ctypes.c_int]
        L.or_fnv64.argtypes = [vp, sz, ctypes.c_uint64]
        L.or_fnv64.restype = ctypes.c_uint64
        _lib = L
    return _lib


def _buf(b: bytes):
    return ctypes.create_string_buffer(b, max(len(b), 1))


def blake2b(msg: bytes, outlen: int = 32) -> bytes:
    out = ctypes.create_string_buffer(outlen)
    lib().or_blake2b(_buf(msg), len(msg), out, outlen)
    return out.raw


def sha256(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().or_sha256(_buf(msg), len(msg), out)
    return out.raw


def salamander_key(psk: bytes, salt: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().or_salamander_key(_buf(psk), len(psk), _buf(salt), out)
    return out.raw


def xplus_key(psk: bytes, salt: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().or_xplus_key(_buf(psk), len(psk), _buf(salt), out)
    return out.raw


def salamander_write(psk: bytes, salt: bytes, p: bytes) -> tuple[bytes, int]:
    wire = ctypes.create_string_buffer(len(p) + 8)
    r = lib().or_salamander_write(_buf(psk), len(psk), _buf(salt), _buf(p), len(p), wire)
    return wire.raw, r


def salamander_read(psk: bytes, dgram: bytes) -> tuple[bytes, int]:
    b = _buf(dgram)
    r = lib().or_salamander_read(_buf(psk), len(psk), b, len(dgram))
    return b.raw[:len(dgram)], r


def xplus_write(psk: bytes, salt: bytes, p: bytes) -> tuple[bytes, int]:
    wire = ctypes.create_string_buffer(len(p) + 16)
    r = lib().or_xplus_write(_buf(psk), len(psk), _buf(salt), _buf(p), len(p), wire)
    return wire.raw, r


def xplus_read(psk: bytes, full: bytes, n: int) -> tuple[bytes, int]:
    b = _buf(full)
    r = lib().or_xplus_read(_buf(psk), len(psk), b, n, len(full))
    return b.raw[:len(full)], r


def _vectorised(fn, psk: bytes, salt: bytes, bufs: list[bytes]):
    cb = [_buf(x) for x in bufs]
    arr = (ctypes.c_void_p * max(len(cb), 1))(*[ctypes.addressof(c) for c in cb])
    lens = (ctypes.c_size_t * max(len(cb), 1))(*[len(x) for x in bufs])
    r = fn(_buf(psk), len(psk), _buf(salt), arr, lens, len(bufs))
    return [c.raw[:len(x)] for c, x in zip(cb, bufs)], r


def salamander_write_vectorised(psk, salt, bufs):
    out, r = _vectorised(lib().or_salamander_write_vectorised, psk, salt, bufs)
    return out, r != 0


def xplus_write_vectorised(psk, salt, bufs):
    out, _ = _vectorised(lib().or_xplus_write_vectorised, psk, salt, bufs)
    return out


def psk_table(psks: list[bytes]):
    blob = np.frombuffer(b"".join(psks) + b"\0", dtype=np.uint8).copy()
    lens = np.array([len(p) for p in psks], dtype=np.uint32)
    offs = np.zeros(len(psks), dtype=np.uint64)
    if len(psks) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    keep = (blob, offs, lens)
    t = OrPsks(blob.ctypes.data, offs.ctypes.data, lens.ctypes.data, len(psks))
    return t, keep


def batch_run(kind: int, direction: int, psks: list[bytes], hb, nthreads: int = 1) -> None:
    """Run the batch restatement over a sqobfs.HostBatch-shaped object."""
    t, keep = psk_table(psks)

    def p(a):
        return None if a is None else a.ctypes.data

    b = OrBatch(hb.n, p(hb.data), p(hb.in_off), p(hb.in_len), p(hb.out), p(hb.out_off),
                p(hb.out_len), p(hb.salt), p(hb.psk_id), p(hb.in_cap))
    st = lib().or_batch_run(kind, direction, ctypes.byref(t), ctypes.byref(b), nthreads)
    del keep
    if st != 0:
        raise RuntimeError(f"or_batch_run failed: {st}")


def fnv64(a: np.ndarray, h: int = 0) -> int:
    return lib().or_fnv64(a.ctypes.data, a.nbytes, h)


def chacha20_stream(key: bytes, nonce: bytes, counter0: int, n: int) -> bytes:
    """RFC 8439 keystream (n bytes from block counter0), C restatement."""
    assert len(key) == 32 and len(nonce) == 12
    out = ctypes.create_string_buffer(max(n, 1))
    lib().or_chacha20_stream(key, nonce, counter0, out, n)
    return out.raw[:n]


def device_salts(key: bytes, seq: int, n: int, S: int) -> bytes:
    """Salts of one SQOBFS_FLAG_DEVICE_SALT launch (include/sqobfs.h)."""
    assert len(key) == 32
    out = ctypes.create_string_buffer(max(n * S, 1))
    lib().or_device_salts(key, seq, n, S, out)
    return out.raw[:n * S]


def poly1305(key: bytes, msg: bytes) -> bytes:
    tag = ctypes.create_string_buffer(16)
    lib().or_poly1305(key, msg, len(msg), tag)
    return tag.raw


def aead_seal(key: bytes, nonce: bytes, aad: bytes, pt: bytes) -> bytes:
    """ct || tag (RFC 8439 2.8)."""
    ct = ctypes.create_string_buffer(max(len(pt), 1))
    tag = ctypes.create_string_buffer(16)
    lib().or_aead_seal(key, nonce, aad, len(aad), pt, len(pt), ct, tag)
    return ct.raw[:len(pt)] + tag.raw


CHACHA20, AES128GCM = 0, 1  # QUIC suites (oracle.h OR_QUIC_*)


def quic_seal(key: bytes, iv: bytes, hp: bytes, pn: int, pkt: bytes, pn_offset: int,
              suite: int = CHACHA20):
    """(protected packet, return code) -- RFC 9001 5.3/5.4; suite CHACHA20
    (32-byte key/hp) or AES128GCM (16-byte key/hp)."""
    out = ctypes.create_string_buffer(len(pkt) + 16)
    r = lib().or_quic_seal2(suite, key, iv, hp, pn, pkt, len(pkt), pn_offset, out)
    return (out.raw[:r] if r > 0 else b""), r


def quic_open(key: bytes, iv: bytes, hp: bytes, largest_pn: int, pkt: bytes, pn_offset: int,
              suite: int = CHACHA20):
    """(unprotected header || plaintext, return code, decoded pn)."""
    out = ctypes.create_string_buffer(max(len(pkt), 1))
    pn = ctypes.c_uint64(0)
    r = lib().or_quic_open2(suite, key, iv, hp, largest_pn, pkt, len(pkt), pn_offset, out,
                            ctypes.byref(pn))
    return (out.raw[:len(pkt) - 16] if len(pkt) >= 16 else b""), r, pn.value


def aes128_encrypt(key: bytes, block: bytes) -> bytes:
    """FIPS-197 AES-128 of one block."""
    rk = ctypes.create_string_buffer(176)
    out = ctypes.create_string_buffer(16)
    lib().or_aes128_expand(key, rk)
    lib().or_aes128_encrypt(rk, block, out)
    return out.raw


def gf128_mul(x: bytes, y: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().or_gf128_mul(x, y, out)
    return out.raw


def gcm_seal(key: bytes, nonce: bytes, aad: bytes, pt: bytes) -> bytes:
    """ct || tag (SP 800-38D, 96-bit nonce)."""
    ct = ctypes.create_string_buffer(max(len(pt), 1))
    tag = ctypes.create_string_buffer(16)
    lib().or_gcm_crypt(key, nonce, aad, len(aad), pt, len(pt), ct, tag, 0)
    return ct.raw[:len(pt)] + tag.raw
