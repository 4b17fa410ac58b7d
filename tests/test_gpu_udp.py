"""The obfuscating batched UDP endpoint (sqobfs_udp_conn) on loopback, with
the GPU doing every byte transform.  Checks against the CPU oracle that

  * what the endpoint SENDS is reference wire format: each datagram, decoded
    by the restated SalamanderPacketConn / XPlusPacketConn ReadFrom
    (salamander.go:42-55, xplus.go:46-60), gives back the payload;
  * what it RECEIVES from reference-format senders decodes to exactly what
    the reference's ReadFrom returns, including the short-datagram quirks
    (salamander.go:47-49; xplus.go:50-52);
  * several sockets fan into one batch (hysteria/hop.go:40-161) with each
    datagram tagged by socket and source address.
"""
from __future__ import annotations

import socket

import numpy as np
import pytest
import sqobfs
from sqobfs import SALAMANDER, XPLUS, Addr

import oracle_lib as ol

pytestmark = pytest.mark.gpu

PSK = b"sing-quic-mi355x-bench-psk"


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    c = sqobfs.Context(0)
    yield c
    c.close()


def _sock():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    s.bind(("127.0.0.1", 0))
    return s


def _ref_read(kind, psk, d):
    """The reference ReadFrom on datagram d: (payload, n returned)."""
    if kind == SALAMANDER:
        buf, n = ol.salamander_read(psk, d)
    else:
        buf, n = ol.xplus_read(psk, d + bytes(64), len(d))
    return buf[:n], n


def _read_n(conn, n):
    got = []
    while len(got) < n:
        batch = conn.read(3000)
        assert batch, f"timed out after {len(got)} of {n}"
        got += batch
    return got


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_conn_round_trip_with_fan_in(ctx, kind):
    S = sqobfs.SALT_LEN[kind]
    rng = np.random.Generator(np.random.PCG64(60 + kind))
    srv_socks = [_sock() for _ in range(3)]
    cli_sock = _sock()
    spy = _sock()  # sees raw wire datagrams
    with sqobfs.Keyring(ctx, kind, [PSK]) as kr, \
            sqobfs.UdpConn(ctx, kr, [s.fileno() for s in srv_socks], slots=256) as srv, \
            sqobfs.UdpConn(ctx, kr, [cli_sock.fileno()], slots=256) as cli:
        for burst in range(6):
            pay = [rng.integers(0, 256, int(rng.integers(1, 1400)), dtype=np.uint8).tobytes()
                   for _ in range(40)]
            dst = [int(rng.integers(0, 3)) for _ in pay]
            to = [Addr.of("127.0.0.1", srv_socks[j].getsockname()[1]) for j in dst]
            assert cli.write(0, pay, to) == len(pay)
            got = _read_n(srv, len(pay))
            # per server socket, order is preserved
            for j in range(3):
                want = [p for p, jj in zip(pay, dst) if jj == j]
                have = [q for q, fi, a in got if fi == j]
                assert have == want, f"burst {burst} socket {j}"
            assert all(a.pair() == cli_sock.getsockname() for _, _, a in got)
        # the wire is reference format: decode raw datagrams with the oracle
        pay = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes()
               for L in (0, 1, 7, 8, 9, 31, 32, 33, 1200, 1350, 2048 - S)]
        assert cli.write(0, pay, [Addr.of("127.0.0.1", spy.getsockname()[1])] * len(pay)) == len(pay)
        spy.settimeout(3)
        salts = set()
        for p in pay:
            d, _ = spy.recvfrom(4096)
            assert len(d) == len(p) + S
            q, n = _ref_read(kind, PSK, d)
            if kind == SALAMANDER and len(p) == 0:
                assert (q, n) == (d, 8)  # salamander.go:47-49: an 8-byte datagram reads raw
            else:
                assert n == len(p) and q == p
            salts.add(d[:S])
        assert len(salts) == len(pay)  # device salts differ per packet
    for s in srv_socks + [cli_sock, spy]:
        s.close()


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_conn_reads_reference_senders(ctx, kind):
    """Datagrams made by the restated reference WriteTo (host salts), plus
    short and junk datagrams, decode to what the reference ReadFrom returns."""
    S = sqobfs.SALT_LEN[kind]
    rng = np.random.Generator(np.random.PCG64(70 + kind))
    srv = _sock()
    tx = _sock()
    write = ol.salamander_write if kind == SALAMANDER else ol.xplus_write
    dgrams = []
    for L in list(range(0, 20)) + [int(x) for x in rng.integers(0, 1450, 100)]:
        if L < 20 and L % 3 == 0:  # raw short / junk datagrams
            dgrams.append(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        else:
            salt = rng.integers(0, 256, S, dtype=np.uint8).tobytes()
            pay = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            dgrams.append(write(PSK, salt, pay)[0])
    with sqobfs.Keyring(ctx, kind, [PSK]) as kr, \
            sqobfs.UdpConn(ctx, kr, [srv.fileno()], slots=64) as conn:
        got = []
        for k0 in range(0, len(dgrams), 40):
            chunk = [d for d in dgrams[k0:k0 + 40] if len(d) > 0]  # empty datagrams: skip
            for d in chunk:
                tx.sendto(d, srv.getsockname())
            got += [(q, len(q)) for q, _, _ in _read_n(conn, len(chunk))]
    want = [_ref_read(kind, PSK, d) for d in dgrams if len(d) > 0]
    assert got == want
    srv.close()
    tx.close()


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_conn_offloads_gso_gro(ctx, kind):
    """UDP segmentation offloads on the endpoint: the client sends runs of
    equal-length datagrams as UDP_SEGMENT messages, the server receives
    coalesced datagrams with UDP_GRO and the kernel's batch offsets point
    inside the 64 KiB receive buffers.  Every payload must come back intact
    and in order, and the wire must still be reference format (checked with
    a spy socket and the oracle's ReadFrom)."""
    rng = np.random.Generator(np.random.PCG64(90 + kind))
    srv_sock, cli_sock, spy = _sock(), _sock(), _sock()
    with sqobfs.Keyring(ctx, kind, [PSK]) as kr, \
            sqobfs.UdpConn(ctx, kr, [srv_sock.fileno()], slots=256) as srv, \
            sqobfs.UdpConn(ctx, kr, [cli_sock.fileno()], slots=256) as cli:
        on_tx = cli.set_offload(sqobfs.UDP_TX_GSO)
        on_rx = srv.set_offload(sqobfs.UDP_RX_GRO)
        assert on_tx in (0, sqobfs.UDP_TX_GSO) and on_rx in (0, sqobfs.UDP_RX_GRO)
        to = Addr.of(*srv_sock.getsockname())
        for burst in range(8):
            L = int(rng.integers(20, 1400))
            pay = [rng.integers(0, 256, L if i % 17 else int(rng.integers(1, L + 1)),
                                dtype=np.uint8).tobytes() for i in range(150)]
            assert cli.write(0, pay, [to] * len(pay)) == len(pay)
            got = _read_n(srv, len(pay))
            assert [g[0] for g in got] == pay
        # the wire is still reference format
        pay = [rng.integers(0, 256, 500, dtype=np.uint8).tobytes() for _ in range(10)]
        assert cli.write(0, pay, [Addr.of(*spy.getsockname())] * 10) == 10
        spy.settimeout(2.0)
        for p in pay:
            d = spy.recv(65536)
            assert _ref_read(kind, PSK, d)[0] == p
        # offloads off again: the fixed slot layout is restored
        assert srv.set_offload(0) == 0
        pay = [b"x" * 100, b"y" * 7]
        assert cli.write(0, pay, [to] * 2) == 2
        assert [g[0] for g in _read_n(srv, 2)] == pay
    for s in (srv_sock, cli_sock, spy):
        s.close()


def test_conn_gro_fan_in_mixed_sources(ctx):
    """GRO receive over two server sockets, from a GSO endpoint and from a
    plain reference-format sender at once: every datagram is tagged with its
    socket and source, per-source order holds, and payloads decode exactly."""
    kind = SALAMANDER
    rng = np.random.Generator(np.random.PCG64(123))
    srv = [_sock(), _sock()]
    cli_sock, plain = _sock(), _sock()
    with sqobfs.Keyring(ctx, kind, [PSK]) as kr, \
            sqobfs.UdpConn(ctx, kr, [s.fileno() for s in srv], slots=512) as conn, \
            sqobfs.UdpConn(ctx, kr, [cli_sock.fileno()], slots=256) as cli:
        assert conn.set_offload(sqobfs.UDP_RX_GRO) in (0, sqobfs.UDP_RX_GRO)
        cli.set_offload(sqobfs.UDP_TX_GSO)
        for burst in range(4):
            pay_g = [rng.integers(0, 256, 900, dtype=np.uint8).tobytes() for _ in range(120)]
            to = [Addr.of(*srv[0 if i < 60 else 1].getsockname()) for i in range(120)]
            pay_p = [rng.integers(0, 256, int(rng.integers(1, 1300)), dtype=np.uint8).tobytes()
                     for _ in range(30)]
            assert cli.write(0, pay_g, to) == 120
            for p in pay_p:  # reference WriteTo: salt || payload ^ key
                salt = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
                plain.sendto(ol.salamander_write(PSK, salt, p)[0], srv[1].getsockname())
            got = _read_n(conn, 150)
            by_src = {}
            for payload, fi, addr in got:
                by_src.setdefault((fi, addr.pair()), []).append(payload)
            c = cli_sock.getsockname()
            assert by_src[(0, c)] == pay_g[:60]
            assert by_src[(1, c)] == pay_g[60:]
            assert by_src[(1, plain.getsockname())] == pay_p
    for s in srv + [cli_sock, plain]:
        s.close()


@pytest.mark.parametrize("suite,offload", [(0, 0), (0, 3), (1, 3)])
def test_conn_quic_fused(ctx, suite, offload):
    """Hysteria2's data path through the endpoint: QUIC packets sealed and
    Salamander-obfuscated in one launch, sent (GSO), received (GRO),
    de-obfuscated and opened in one launch.  The wire is checked against the
    oracle composition (or_quic_seal then the restated WriteTo), the
    received packets and packet numbers against the originals."""
    rng = np.random.Generator(np.random.PCG64(300 + 10 * suite + offload))
    kl = 16 if suite else 32
    kb = tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (kl, 12, kl))
    srv_sock, cli_sock, spy = _sock(), _sock(), _sock()
    dcid = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
    pno = 1 + len(dcid)
    with sqobfs.Keyring(ctx, SALAMANDER, [PSK]) as kr, \
            sqobfs.QuicKeyring(ctx, [sqobfs.QuicKey.of(*kb)], suite) as qkr, \
            sqobfs.UdpConn(ctx, kr, [srv_sock.fileno()], slots=256) as srv, \
            sqobfs.UdpConn(ctx, kr, [cli_sock.fileno()], slots=256) as cli:
        cli.set_offload(offload & sqobfs.UDP_TX_GSO)
        srv.set_offload(offload & sqobfs.UDP_RX_GRO)
        to = Addr.of(*srv_sock.getsockname())
        pn0 = 1000
        for burst in range(4):
            L = int(rng.integers(40, 1300))
            pkts = [bytes([0x41]) + dcid + ((pn0 + i) & 0xFFFF).to_bytes(2, "big") +
                    rng.integers(0, 256, L if i % 9 else int(rng.integers(3, L + 1)),
                                 dtype=np.uint8).tobytes() for i in range(100)]
            pns = [pn0 + i for i in range(100)]
            assert cli.write_quic(qkr, 0, pkts, pno, pns, [to] * 100) == 100
            got = []
            while len(got) < 100:
                b = srv.read_quic(qkr, pno, pn0 - 1, 3000)
                assert b, f"timed out after {len(got)}"
                got += b
            assert [g[0] for g in got] == pkts
            assert [g[4] for g in got] == pns
            pn0 += 100
        # the wire: salt || (RFC 9001 protected packet) ^ BLAKE2b(psk || salt)
        pkts = [bytes([0x41]) + dcid + (7).to_bytes(2, "big") + b"\x33" * 200]
        assert cli.write_quic(qkr, 0, pkts, pno, [pn0 + 7], [Addr.of(*spy.getsockname())]) == 1
        spy.settimeout(2.0)
        w = spy.recv(65536)
        assert len(w) == len(pkts[0]) + 24
        plain, n = ol.salamander_read(PSK, w)
        want, r = ol.quic_seal(*kb, pn0 + 7, pkts[0], pno, suite=suite)
        assert plain[:n] == want
    for s in (srv_sock, cli_sock, spy):
        s.close()


def test_conn_quic_reader_and_writer_threads(ctx):
    """One endpoint seals + sends in one thread while another thread receives
    and opens on it (quic-go's send and receive loops, salamander.go:42-70
    called concurrently).  Each direction has its own packet-number arrays:
    every datagram on the wire must be sealed under ITS packet number (a
    shared array would let the reader's largest_pn leak into the writer's
    nonces)."""
    import threading
    rng = np.random.Generator(np.random.PCG64(77))
    kb = tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (32, 12, 32))
    a_sock, b_sock, spy = _sock(), _sock(), _sock()
    dcid = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
    pno = 1 + len(dcid)
    n_bursts, per = 12, 64
    mk = lambda pn, L: (bytes([0x41]) + dcid + (pn & 0xFFFF).to_bytes(2, "big") +  # noqa: E731
                        bytes((pn * 7 + i) & 0xFF for i in range(L)))
    with sqobfs.Keyring(ctx, SALAMANDER, [PSK]) as kr, \
            sqobfs.QuicKeyring(ctx, [sqobfs.QuicKey.of(*kb)], 0) as qkr, \
            sqobfs.UdpConn(ctx, kr, [a_sock.fileno()], slots=256) as a, \
            sqobfs.UdpConn(ctx, kr, [b_sock.fileno()], slots=256) as b:
        to_spy = Addr.of(*spy.getsockname())
        to_a = Addr.of(*a_sock.getsockname())
        sent_pns = []
        rx = []
        errs = []

        def writer():
            try:
                for k in range(n_bursts):
                    pns = [10_000 + k * per + i for i in range(per)]
                    pk = [mk(pn, 300) for pn in pns]
                    assert a.write_quic(qkr, 0, pk, pno, pns, [to_spy] * per) == per
                    sent_pns.extend(pns)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        def reader():
            try:
                while len(rx) < n_bursts * per:
                    got = a.read_quic(qkr, pno, 499, 3000)
                    assert got, f"reader timed out after {len(rx)}"
                    rx.extend(got)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        tw, tr = threading.Thread(target=writer), threading.Thread(target=reader)
        tr.start()
        tw.start()
        for k in range(n_bursts):  # b feeds a's reader meanwhile
            pns = [500 + k * per + i for i in range(per)]
            assert b.write_quic(qkr, 0, [mk(pn, 200) for pn in pns], pno, pns,
                                [to_a] * per) == per
        tw.join(60)
        tr.join(60)
        assert not errs, errs
        assert [g[4] for g in rx] == [500 + i for i in range(n_bursts * per)]
        assert [g[0] for g in rx] == [mk(500 + i, 200) for i in range(n_bursts * per)]
        spy.settimeout(2.0)
        for pn in sent_pns:
            w = spy.recv(65536)
            plain, n = ol.salamander_read(PSK, w)
            want, _ = ol.quic_seal(*kb, pn, mk(pn, 300), pno, suite=0)
            assert plain[:n] == want, f"packet {pn} sealed under another packet number"
    for s in (a_sock, b_sock, spy):
        s.close()


def test_conn_quic_rejects_reported(ctx):
    """write_quic: a packet too short for its packet number and sample is
    not sent; the ones before it are, and the call fails with *sent = its
    index.  read_quic: a datagram that cannot be opened has no packet and
    no packet number."""
    rng = np.random.Generator(np.random.PCG64(78))
    kb = tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (32, 12, 32))
    a_sock, spy, raw = _sock(), _sock(), _sock()
    dcid = bytes(8)
    pno = 9
    good = [bytes([0x41]) + dcid + bytes([0, i]) + bytes(100) for i in range(3)]
    short = bytes([0x41]) + dcid + bytes([0, 9, 1])  # pn_offset + 4 > len: no sample
    with sqobfs.Keyring(ctx, SALAMANDER, [PSK]) as kr, \
            sqobfs.QuicKeyring(ctx, [sqobfs.QuicKey.of(*kb)], 0) as qkr, \
            sqobfs.UdpConn(ctx, kr, [a_sock.fileno()], slots=64) as a:
        with pytest.raises(sqobfs.SqError) as ei:
            a.write_quic(qkr, 0, good[:2] + [short] + good[2:], pno, [0, 1, 2, 3],
                         [Addr.of(*spy.getsockname())] * 4)
        assert ei.value.sent == 2
        spy.settimeout(1.0)
        for i in range(2):
            plain, n = ol.salamander_read(PSK, spy.recv(65536))
            assert plain[:n] == ol.quic_seal(*kb, i, good[i], pno, suite=0)[0]
        with pytest.raises(socket.timeout):
            spy.recv(65536)
        raw.sendto(b"\x07" * 5, a_sock.getsockname())      # shorter than a salt
        raw.sendto(bytes(40), a_sock.getsockname())         # tag cannot match
        got = []
        while len(got) < 2:
            b = a.read_quic(qkr, pno, 0, 3000)
            assert b
            got += b
        for data, code, _, _, pn in got:
            assert data is None and pn is None and code >= 0xFFFFFFF0
    for s in (a_sock, spy, raw):
        s.close()
