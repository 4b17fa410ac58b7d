"""Debug driver: GRO fan-in from a GSO endpoint and a plain sender."""
import os
import socket
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sing-quic_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import sqobfs  # noqa: E402
import oracle_lib as ol  # noqa: E402
from sqobfs import Addr  # noqa: E402

torch.cuda.init()
PSK = b"sing-quic-mi355x-bench-psk"


def sock():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    s.bind(("127.0.0.1", 0))
    return s


ctx = sqobfs.Context(0)
rng = np.random.Generator(np.random.PCG64(123))
srv = [sock(), sock()]
cli_sock, plain = sock(), sock()
nplain = int(sys.argv[1]) if len(sys.argv) > 1 else 30
gro = int(sys.argv[2]) if len(sys.argv) > 2 else 1
with sqobfs.Keyring(ctx, 0, [PSK]) as kr, \
        sqobfs.UdpConn(ctx, kr, [s.fileno() for s in srv], slots=512) as conn, \
        sqobfs.UdpConn(ctx, kr, [cli_sock.fileno()], slots=256) as cli:
    print("offload", conn.set_offload(sqobfs.UDP_RX_GRO * gro), cli.set_offload(sqobfs.UDP_TX_GSO))
    pay_g = [bytes([i]) * 900 for i in range(120)]
    to = [Addr.of(*srv[0 if i < 60 else 1].getsockname()) for i in range(120)]
    pay_p = [bytes([200 + (i % 50)]) * (10 + i) for i in range(nplain)]
    assert cli.write(0, pay_g, to) == 120
    for p in pay_p:
        salt = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
        plain.sendto(ol.salamander_write(PSK, salt, p)[0], srv[1].getsockname())
    got = []
    while len(got) < 120 + nplain:
        b = conn.read(2000)
        print("read batch", len(b))
        if not b:
            break
        got += b
    c = cli_sock.getsockname()
    for payload, fi, addr in got[:200]:
        src = "cli" if addr.pair() == c else "plain"
        print(fi, src, len(payload), payload[:4].hex(), payload[-2:].hex(),
              "uniform" if payload == bytes([payload[0]]) * len(payload) else "MIXED")
ctx.close()
