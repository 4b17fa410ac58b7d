"""Independent Python restatement of sing-quic's obfuscation layer.

TEST INFRASTRUCTURE ONLY -- used to generate tests/golden/ and to cross-check
the C restatement (oracle/oracle.c).  Never imported by the product.

Primitives come from hashlib (BLAKE2b reference implementation, OpenSSL
SHA-256), i.e. from code independent of oracle.c, so agreement between the two
restatements is evidence about both.  Parity with the Go reference itself is
unpinned: the reference ships no tests or vectors and no Go toolchain exists
here or on the GPU box ("Parity").

Citations are /root/reference paths.
"""
from __future__ import annotations

import hashlib

SALAMANDER_SALT = 8  # hysteria2/salamander.go:15
XPLUS_SALT = 16  # hysteria/xplus.go:17


def salamander_key(psk: bytes, salt: bytes) -> bytes:
    """blake2b.Sum256(append(password, salt...)) -- salamander.go:50,61,84,99"""
    assert len(salt) == SALAMANDER_SALT
    return hashlib.blake2b(psk + salt, digest_size=32).digest()


def xplus_key(psk: bytes, salt: bytes) -> bytes:
    """sha256.Sum256(append(key, salt...)) -- xplus.go:54,70,93,107"""
    assert len(salt) == XPLUS_SALT
    return hashlib.sha256(psk + salt).digest()


def _xor_stream(data: bytes, key: bytes) -> bytes:
    return bytes(c ^ key[i % 32] for i, c in enumerate(data))


def salamander_write(psk: bytes, salt: bytes, p: bytes) -> tuple[bytes, int]:
    """SalamanderPacketConn.WriteTo, salamander.go:57-70 -> (wire, return n)"""
    key = salamander_key(psk, salt)
    return salt + _xor_stream(p, key), len(p)


def salamander_read(psk: bytes, p: bytes) -> tuple[bytes, int]:
    """SalamanderPacketConn.ReadFrom, salamander.go:42-55.

    p is exactly the n bytes the socket returned.  Returns (buffer after the
    call, return n).  n <= 8: untouched, returns n (:47-49)."""
    n = len(p)
    if n <= SALAMANDER_SALT:
        return bytes(p), n
    key = salamander_key(psk, p[:SALAMANDER_SALT])
    dec = _xor_stream(p[SALAMANDER_SALT:], key)
    # in place: p[index] = ...; bytes [n-8, n) keep the old tail
    return dec + p[n - SALAMANDER_SALT:], n - SALAMANDER_SALT


def xplus_write(psk: bytes, salt: bytes, p: bytes) -> tuple[bytes, int]:
    """XPlusPacketConn.WriteTo, xplus.go:62-75 -> (wire, return n = len+16)"""
    key = xplus_key(psk, salt)
    return salt + _xor_stream(p, key), len(p) + XPLUS_SALT


def xplus_read(psk: bytes, buf: bytes, n: int) -> tuple[bytes, int]:
    """XPlusPacketConn.ReadFrom, xplus.go:46-60.

    buf is the whole read buffer p (len(p) = cap >= n); the socket wrote n
    bytes.  n < 16: returns 0, untouched.  Otherwise XORs i in [0, cap-16)."""
    if n < XPLUS_SALT:
        return bytes(buf), 0
    key = xplus_key(psk, buf[:XPLUS_SALT])
    cap = len(buf)
    dec = _xor_stream(buf[XPLUS_SALT:cap], key)
    return dec + buf[cap - XPLUS_SALT:], n - XPLUS_SALT


def salamander_write_vectorised(psk: bytes, salt: bytes, bufs: list[bytes]):
    """VectorisedSalamanderPacketConn.WriteVectorisedPacket, salamander.go:95-109,
    literally.  Returns (list of buffers, panicked)."""
    key = salamander_key(psk, salt)
    out = [bytearray(b) for b in bufs]
    buffer_index = 0
    for content in out:
        for index in range(len(content)):
            c = content[index]
            ci = buffer_index + index
            ki = buffer_index + index % 32
            if ki >= 32 or ci >= len(content):
                return [bytes(b) for b in out], True
            content[ci] = c ^ key[ki]
        buffer_index += len(content)
    return [bytes(b) for b in out], False


def xplus_write_vectorised(psk: bytes, salt: bytes, bufs: list[bytes]):
    """VectorisedXPlusConn.WriteVectorisedPacket, xplus.go:100-118."""
    key = xplus_key(psk, salt)
    out, index = [], 0
    for b in bufs:
        nb = bytearray(b)
        for i in range(len(nb)):
            nb[i] ^= key[index % 32]
            index += 1
        out.append(bytes(nb))
    return out
