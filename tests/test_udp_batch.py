"""Batched UDP socket I/O (include/sqobfs.h, sqobfs_udp_recv / _send) on
loopback sockets.  CPU only: these entry points move datagrams, the GPU is
not involved.  They replace the reference's one-syscall-per-datagram
ReadFrom / WriteTo (salamander.go:43,65,88) and hop.go's per-socket recvLoop
(hysteria/hop.go:40-161) with recvmmsg / sendmmsg and multi-socket fan-in."""
from __future__ import annotations

import socket

import numpy as np
import pytest
import sqobfs
from sqobfs import Addr


def _sock(family=socket.AF_INET, host="127.0.0.1"):
    s = socket.socket(family, socket.SOCK_DGRAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    s.bind((host, 0))
    return s


def _recv_all(fds, expect, slot=2048, headroom=0, max_n=4096):
    """Receive until `expect` datagrams arrived (several calls)."""
    slots = np.zeros(max_n * slot, np.uint8)
    got = []
    while len(got) < expect:
        n, ln, fi, addrs = sqobfs.udp_recv(fds, slots, slot, headroom, max_n, 2000)
        assert n > 0, f"timed out after {len(got)} of {expect}"
        for k in range(n):
            base = k * slot + headroom
            got.append((slots[base:base + ln[k]].tobytes(), int(fi[k]), addrs[k].pair()))
    return got


def test_addr_roundtrip():
    a = Addr.of("127.0.0.1", 4433)
    assert a.family == socket.AF_INET and a.pair() == ("127.0.0.1", 4433)
    b = Addr.of("::1", 443)
    assert b.family == socket.AF_INET6 and b.pair() == ("::1", 443)


def test_recv_fan_in_many_sockets():
    """hop.go fan-in: datagrams sent to 4 sockets come back in one batch API,
    each tagged with its socket index and source address."""
    rx = [_sock() for _ in range(4)]
    tx = _sock()
    rng = np.random.Generator(np.random.PCG64(1))
    sent, got = [], []
    for burst in range(15):  # bursts small enough for any socket buffer
        for i in range(40):
            j = int(rng.integers(0, 4))
            d = rng.integers(0, 256, int(rng.integers(1, 1500)), dtype=np.uint8).tobytes()
            tx.sendto(d, rx[j].getsockname())
            sent.append((d, j))
        got += _recv_all([s.fileno() for s in rx], 40)
    assert len(got) == len(sent)
    src = tx.getsockname()
    # per socket, order is preserved (one sender)
    for j in range(4):
        want = [d for d, jj in sent if jj == j]
        have = [d for d, jj, a in got if jj == j]
        assert have == want
    assert all(a == src for _, _, a in got)
    for s in rx + [tx]:
        s.close()


def test_recv_timeout_and_headroom_and_truncation():
    rx, tx = _sock(), _sock()
    slots = np.zeros(8 * 256, np.uint8)
    n, *_ = sqobfs.udp_recv([rx.fileno()], slots, 256, 8, 8, 0)
    assert n == 0  # nothing queued: immediate timeout
    tx.sendto(b"a" * 300, rx.getsockname())  # longer than slot - headroom
    tx.sendto(b"bc", rx.getsockname())
    n, ln, fi, _ = sqobfs.udp_recv([rx.fileno()], slots, 256, 8, 8, 2000)
    if n == 1:  # second datagram not yet queued
        n2, ln2, _, _ = sqobfs.udp_recv([rx.fileno()], slots[256:], 256, 8, 7, 2000)
        ln = np.concatenate([ln, ln2])
        n += n2
    assert n == 2
    assert ln[0] == 248 and slots[8:256].tobytes() == b"a" * 248  # truncated like ReadFrom
    assert ln[1] == 2 and slots[256 + 8:256 + 10].tobytes() == b"bc"
    assert slots[:8].tobytes() == bytes(8)  # headroom untouched
    rx.close()
    tx.close()


@pytest.mark.parametrize("family,host", [(socket.AF_INET, "127.0.0.1"),
                                         (socket.AF_INET6, "::1")])
def test_send_batch(family, host):
    try:
        rx, tx = _sock(family, host), _sock(family, host)
    except OSError:
        pytest.skip(f"no {host} loopback")
    rng = np.random.Generator(np.random.PCG64(2))
    n = 1500  # several sendmmsg chunks
    lens = rng.integers(0, 1400, n).astype(np.uint32)
    base = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
    off = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.uint64)
    if True:
        to = [Addr.of(host, rx.getsockname()[1])] * n
        got = []
        for k0 in range(0, n, 50):  # bursts small enough for any socket buffer
            k1 = min(n, k0 + 50)
            assert sqobfs.udp_send(tx.fileno(), base, off[k0:k1], lens[k0:k1], to[k0:k1]) == k1 - k0
            got += _recv_all([rx.fileno()], k1 - k0)
        for k in range(n):
            assert got[k][0] == base[int(off[k]):int(off[k]) + int(lens[k])].tobytes()
    rx.close()
    tx.close()


def test_bad_arguments():
    slots = np.zeros(64, np.uint8)
    with pytest.raises(sqobfs.SqError):
        sqobfs.udp_recv([], slots, 64, 0, 1, 0)
    with pytest.raises(sqobfs.SqError):
        sqobfs.udp_recv([0], slots, 64, 64, 1, 0)  # headroom >= slot


def test_send_gso_runs_arrive_as_datagrams():
    """sqobfs_udp_send_gso: runs of equal-length datagrams to one address go
    out as UDP_SEGMENT messages; the receiver still sees the original
    datagrams, in order, byte for byte (mixed lengths, shorter run ends,
    two destinations, runs longer than 64 segments)."""
    rx = [_sock(), _sock()]
    tx = _sock()
    rng = np.random.Generator(np.random.PCG64(5))
    pkts, dst = [], []
    for run in range(12):
        L = int(rng.integers(1, 1400))
        cnt = int(rng.integers(1, 90))
        j = run % 2
        for k in range(cnt):
            ln = L if k + 1 < cnt or run % 3 else max(1, L - int(rng.integers(0, L)))
            pkts.append(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
            dst.append(j)
    # send in bursts that fit the receive buffers, read back per socket
    pos = 0
    while pos < len(pkts):
        n = min(100, len(pkts) - pos)
        buf, off, lens = sqobfs.pack(pkts[pos:pos + n], align=1)
        to = [Addr.of(*rx[d].getsockname()) for d in dst[pos:pos + n]]
        try:
            sent = sqobfs.udp_send(tx.fileno(), buf, off, lens, to, gso=True)
        except sqobfs.SqError as e:  # kernel without UDP GSO: nothing to test
            pytest.skip(f"UDP GSO unavailable: {e}")
        assert sent == n
        for d in (0, 1):
            want = [p for p, q in zip(pkts[pos:pos + n], dst[pos:pos + n]) if q == d]
            rx[d].settimeout(2.0)
            got = [rx[d].recv(65536) for _ in want]
            assert got == want
        pos += n
    for s in rx + [tx]:
        s.close()
