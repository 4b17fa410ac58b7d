"""Ragged batches whose datagrams lie more than 4 GiB apart within one unit
(a wavefront's packets): the kernel's 32-bit buffer ranges cannot cover such
a unit, so its input windows and its stream take their wide paths (window
blocks re-loaded with 64-bit addresses, the generic stream).  Every output
byte equals the oracle's, as for compact batches.

The host batch is compact; on the device every third datagram's input (or
output) sits GAP bytes further on in the same allocation, so consecutive
datagrams of every unit alternate between two regions 4.5 GiB apart."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import DEOBFUSCATE, OBFUSCATE, SALAMANDER, XPLUS, SALT_LEN

import gpu_harness as gh

pytestmark = pytest.mark.gpu

PSKS = [b"sing-quic-mi355x-bench-psk", b"", b"z" * 200]
GAP = (9 << 29) + 48  # 4.5 GiB + 48: 16-byte phases kept, line phases not


def _far(n: int) -> np.ndarray:
    return (np.arange(n) % 3) == 1


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
@pytest.mark.parametrize("direction", [OBFUSCATE, DEOBFUSCATE])
@pytest.mark.parametrize("side", ["input", "output"])
@pytest.mark.parametrize("multi", [False, True])
def test_unit_spans_over_4gib(kind, direction, side, multi):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    dev = torch.device("cuda", 0)
    rng = np.random.Generator(np.random.PCG64(700 + 8 * kind + 4 * direction + 2 * multi
                                              + (side == "output")))
    n = 3000
    lens = np.concatenate([np.arange(0, 40), rng.integers(0, 1500, n - 40)])
    ids = rng.integers(0, len(PSKS), n) if multi else None
    psks = PSKS if multi else PSKS[:1]
    hb = gh.make_case(rng, kind, direction, lens, psks, psk_ids=ids, in_align=1, out_align=1,
                      gaps=True)
    ref = gh.run_oracle(kind, direction, psks, hb)
    far = _far(n)
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    in_off, out_off = hb.in_off.copy(), hb.out_off.copy()
    if side == "input":
        d_in = torch.empty(GAP + hb.data.size, dtype=torch.uint8, device=dev)
        src = t(hb.data)
        d_in[:hb.data.size] = src
        d_in[GAP:GAP + hb.data.size] = src
        in_off[far] += GAP
        d_out = t(hb.out)
    else:
        d_in = t(hb.data)
        d_out = torch.full((GAP + hb.out.size,), gh.SENTINEL, dtype=torch.uint8, device=dev)
        out_off[far] += GAP
    d_in_off, d_out_off = t(in_off), t(out_off)
    d_len, d_olen = t(hb.in_len), t(hb.out_len)
    b = sqobfs.make_batch(n, d_in, d_in_off, d_len, d_out, d_out_off, d_olen, t(hb.salt),
                          t(hb.psk_id), t(hb.in_cap))
    with sqobfs.Context(0) as ctx, sqobfs.Keyring(ctx, kind, psks) as kr:
        for ppw in (0, 1, 28):  # default, one packet per unit, a wide unit
            ctx.unit_packets = ppw
            d_olen.zero_()
            if side == "output":
                d_out.fill_(gh.SENTINEL)
            sqobfs.launch(ctx, kr, direction, b, torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize(dev)
            got = gh.clone(hb)
            got.out_len[:] = d_olen.cpu().numpy()
            if side == "input":
                got.out[:] = d_out.cpu().numpy()
            else:
                near = d_out[:hb.out.size].cpu().numpy()
                away = d_out[GAP:GAP + hb.out.size].cpu().numpy()
                # the far datagrams' bytes come from the far region, whose
                # other bytes (and the near region's under them) stay sentinel
                assert np.all(away[~_mask(hb, far, kind, direction)] == gh.SENTINEL), \
                    f"ppw={ppw}: far region written outside its datagrams"
                fm = _mask(hb, far, kind, direction)
                assert np.all(near[fm] == gh.SENTINEL), f"ppw={ppw}: far datagram written near"
                got.out[:] = np.where(fm, away, near)
            gh.assert_same(got, ref, f"ppw={ppw} side={side}")
        ctx.unit_packets = 0


def _mask(hb, sel, kind, direction) -> np.ndarray:
    """Output bytes of the selected datagrams (their full output extent)."""
    m = np.zeros(hb.out.size, dtype=bool)
    caps = hb.in_cap if hb.in_cap is not None else hb.in_len
    for i in np.nonzero(sel)[0]:
        o = int(hb.out_off[i])
        m[o:o + gh.out_size(kind, direction, int(hb.in_len[i]), int(caps[i]))] = True
    return m
