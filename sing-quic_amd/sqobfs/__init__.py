"""ctypes binding of libsqobfs.so (include/sqobfs.h) for tests and bench.py.

The product is the C ABI + gfx950 kernels; this module is plumbing.  It
loads the in-tree ``sing-quic_amd/libsqobfs.so`` and raises if it is missing.
Device entry points never fall back to the CPU; the product's CPU path is
explicit (host keyrings, ``cpu_run``, and the packet conn engine's small or
GPU-less batches, include/sqobfs.h).

Names mirror the reference's obfuscation layer:
  hysteria2/salamander.go  -> SALAMANDER, salt 8, BLAKE2b-256
  hysteria/xplus.go        -> XPLUS,      salt 16, SHA-256
"""
from __future__ import annotations

import ctypes
import os
import sys
import re
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
LIB_PATH = os.environ.get("SQOBFS_LIB") or os.path.join(PKG, "libsqobfs.so")
HEADER_PATH = os.path.join(REPO, "include", "sqobfs.h")

SALAMANDER, XPLUS = 0, 1
OBFUSCATE, DEOBFUSCATE = 0, 1
SALT_LEN = {SALAMANDER: 8, XPLUS: 16}
OBFS_TYPE_SALAMANDER = "salamander"  # hysteria2/salamander.go:17

SQ_OK, SQ_EINVAL, SQ_ENOMEM, SQ_EDEVICE, SQ_ENODEV, SQ_EPSK = 0, -1, -2, -3, -4, -5
SQ_ETIMEDOUT, SQ_ECLOSED, SQ_EIO = -6, -7, -8
BAD_PSK = 0xFFFFFFFF
FLAG_OUT_UNINIT = 1  # run_host: bytes between output regions need not be kept
FLAG_DEVICE_SALT = 2  # obfuscate: salts from the GPU's ChaCha20 generator
FLAG_OUT_BLOCKS = 4  # outputs own their 16-byte blocks (slot padding is scratch)
FLAG_OUT_LINES = 8  # ... and their last 128-byte line to its end (no line written in part)


class SqError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: {status} ({strerror(status)})")


class Batch(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("in_", ctypes.c_void_p),
        ("in_off", ctypes.c_void_p),
        ("in_len", ctypes.c_void_p),
        ("out", ctypes.c_void_p),
        ("out_off", ctypes.c_void_p),
        ("out_len", ctypes.c_void_p),
        ("salt", ctypes.c_void_p),
        ("psk_id", ctypes.c_void_p),
        ("in_cap", ctypes.c_void_p),
        ("salt_out", ctypes.c_void_p),
    ]


class Addr(ctypes.Structure):
    """sqobfs_addr: family, port (host order), scope id, 16 address bytes."""
    _fields_ = [("family", ctypes.c_uint16), ("port", ctypes.c_uint16),
                ("scope_id", ctypes.c_uint32), ("addr", ctypes.c_uint8 * 16)]

    @classmethod
    def of(cls, host: str, port: int) -> "Addr":
        import ipaddress
        ip = ipaddress.ip_address(host)
        a = cls()
        a.family = 2 if ip.version == 4 else 10
        a.port = port
        raw = ip.packed
        ctypes.memmove(a.addr, raw, len(raw))
        return a

    def pair(self) -> tuple[str, int]:
        import ipaddress
        raw = bytes(self.addr)
        ip = ipaddress.ip_address(raw[:4] if self.family == 2 else raw)
        return str(ip), int(self.port)


class QuicKey(ctypes.Structure):
    """sqobfs_quic_key: one connection's 1-RTT key, iv, hp."""
    _fields_ = [("key", ctypes.c_uint8 * 32), ("iv", ctypes.c_uint8 * 12),
                ("hp", ctypes.c_uint8 * 32)]

    @classmethod
    def of(cls, key: bytes, iv: bytes, hp: bytes) -> "QuicKey":
        """key / hp: 32 bytes (ChaCha20-Poly1305) or 16 (AES-128-GCM)."""
        assert len(key) in (16, 32) and len(hp) == len(key) and len(iv) == 12
        k = cls()
        ctypes.memmove(k.key, key, len(key))
        ctypes.memmove(k.iv, iv, 12)
        ctypes.memmove(k.hp, hp, len(hp))
        return k


class QuicBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("in_", ctypes.c_void_p),
                ("in_off", ctypes.c_void_p), ("in_len", ctypes.c_void_p),
                ("out", ctypes.c_void_p), ("out_off", ctypes.c_void_p),
                ("out_len", ctypes.c_void_p), ("pn_offset", ctypes.c_void_p),
                ("pn", ctypes.c_void_p), ("key_id", ctypes.c_void_p), ("pn_out", ctypes.c_void_p)]


QUIC_EKEY, QUIC_ESHORT, QUIC_EAUTH = 0xFFFFFFFF, 0xFFFFFFFE, 0xFFFFFFFD
QUIC_CHACHA20_POLY1305, QUIC_AES_128_GCM = 0, 1  # SQOBFS_QUIC_* suites


class UdpView(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint32), ("base", ctypes.c_void_p), ("off", ctypes.c_void_p),
                ("len", ctypes.c_void_p), ("fd_index", ctypes.c_void_p),
                ("from_", ctypes.c_void_p)]


_lib = None


def lib() -> ctypes.CDLL:
    """Load libsqobfs.so (fails loudly: the product has no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `make -C sing-quic_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    _lib = load(LIB_PATH)
    return _lib


def load(path: str) -> ctypes.CDLL:
    """A libsqobfs build at `path` with its prototypes declared (lib() loads
    the in-tree one; dev A/B scripts load timing variants side by side)."""
    # torch (the device-memory plumbing of the tests and the bench) first,
    # where it is installed: its wheel carries its own HIP runtime, which the
    # library then shares; loaded after the library, torch would bring a
    # second runtime that finds no GPU
    if "torch" not in sys.modules:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(path)
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    L.sqobfs_abi_version.restype = i32
    L.sqobfs_strerror.restype = ctypes.c_char_p
    L.sqobfs_strerror.argtypes = [i32]
    L.sqobfs_device_count.argtypes = [ctypes.POINTER(i32)]
    L.sqobfs_open.argtypes = [i32, ctypes.POINTER(vp)]
    L.sqobfs_close.argtypes = [vp]
    L.sqobfs_close.restype = None
    L.sqobfs_stream.argtypes = [vp]
    L.sqobfs_stream.restype = vp
    L.sqobfs_sync.argtypes = [vp, vp]
    L.sqobfs_keyring_create.argtypes = [vp, i32, u32, vp, vp, vp, ctypes.POINTER(vp)]
    L.sqobfs_keyring_destroy.argtypes = [vp]
    L.sqobfs_keyring_destroy.restype = None
    L.sqobfs_keyring_kind.argtypes = [vp]
    L.sqobfs_keyring_count.argtypes = [vp]
    L.sqobfs_keyring_count.restype = u32
    for name in ("sqobfs_salamander_obfuscate", "sqobfs_salamander_deobfuscate",
                 "sqobfs_xplus_obfuscate", "sqobfs_xplus_deobfuscate"):
        getattr(L, name).argtypes = [vp, vp, ctypes.POINTER(Batch), vp]
    L.sqobfs_launch.argtypes = [vp, vp, i32, ctypes.POINTER(Batch), vp]
    L.sqobfs_run_host.argtypes = [vp, vp, i32, ctypes.POINTER(Batch)]
    L.sqobfs_host_alloc.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(vp)]
    L.sqobfs_host_free.argtypes = [vp, vp]
    L.sqobfs_build_info.restype = ctypes.c_char_p
    L.sqobfs_build_info.argtypes = []
    L.sqobfs_host_free.restype = None
    L.sqobfs_host_staging_bytes.argtypes = [vp]
    L.sqobfs_host_staging_bytes.restype = ctypes.c_size_t
    L.sqobfs_debug_fail_chunk.argtypes = [i32]
    L.sqobfs_debug_fail_chunk.restype = None
    L.sqobfs_debug_time_next_launch.argtypes = [vp, vp]
    L.sqobfs_debug_time_next_launch.restype = None
    L.sqobfs_shard_cuts.argtypes = [u32, vp, u32, vp]
    L.sqobfs_run_host_sharded.argtypes = [u32, vp, vp, i32, ctypes.POINTER(Batch)]
    L.sqobfs_shard_run.argtypes = [u32, vp, vp, i32, vp]
    u16p, u32p = ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_uint32)
    L.sqobfs_udp_recv.argtypes = [vp, u32, vp, u32, u32, u32, i32, vp, vp, vp, u32p]
    L.sqobfs_udp_send.argtypes = [i32, vp, vp, vp, vp, u32, u32p]
    L.sqobfs_udp_send_gso.argtypes = [i32, vp, vp, vp, vp, u32, u32p]
    L.sqobfs_udp_conn_set_offload.argtypes = [vp, u32]
    L.sqobfs_udp_conn_write_quic.argtypes = [vp, vp, u32, u32, vp, ctypes.c_uint16, vp, vp, u32p]
    L.sqobfs_udp_conn_read_quic.argtypes = [vp, vp, ctypes.c_uint16, ctypes.c_uint64, i32, vp,
                                            ctypes.POINTER(ctypes.c_void_p)]
    L.sqobfs_udp_conn_set_offload.restype = i32
    L.sqobfs_udp_conn_open.argtypes = [vp, vp, vp, u32, u32, u32, ctypes.POINTER(vp)]
    L.sqobfs_udp_conn_close.argtypes = [vp]
    L.sqobfs_udp_conn_close.restype = None
    L.sqobfs_udp_conn_read.argtypes = [vp, i32, ctypes.POINTER(UdpView)]
    L.sqobfs_udp_conn_tx_payload.argtypes = [vp, u32]
    L.sqobfs_udp_conn_tx_payload.restype = vp
    L.sqobfs_udp_conn_write.argtypes = [vp, u32, u32, vp, vp, u32p]
    L.sqobfs_quic_keyring_create.argtypes = [vp, u32, vp, ctypes.POINTER(vp)]
    L.sqobfs_quic_keyring_create_suite.argtypes = [vp, u32, u32, vp, ctypes.POINTER(vp)]
    L.sqobfs_quic_keyring_destroy.argtypes = [vp]
    L.sqobfs_quic_keyring_destroy.restype = None
    L.sqobfs_quic_seal.argtypes = [vp, vp, ctypes.POINTER(QuicBatch), vp]
    L.sqobfs_quic_open.argtypes = [vp, vp, ctypes.POINTER(QuicBatch), vp]
    L.sqobfs_quic_seal_salamander.argtypes = [vp, vp, vp, ctypes.POINTER(QuicBatch), vp, vp]
    L.sqobfs_quic_open_salamander.argtypes = [vp, vp, vp, ctypes.POINTER(QuicBatch), vp]
    L.sqobfs_salt_key.argtypes = [vp, vp, ctypes.c_uint64]
    L.sqobfs_salt_seq.argtypes = [vp]
    L.sqobfs_salt_seq.restype = ctypes.c_uint64
    L.sqobfs_set_unit_packets.argtypes = [vp, ctypes.c_uint32]
    L.sqobfs_set_unit_packets.restype = ctypes.c_int
    L.sqobfs_unit_packets.argtypes = [vp]
    L.sqobfs_unit_packets.restype = ctypes.c_uint32
    L.sqobfs_unit_packets_for.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int]
    L.sqobfs_unit_packets_for.restype = ctypes.c_uint32
    L.sqobfs_unit_packets_for_kind.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32,
                                               ctypes.c_int]
    L.sqobfs_unit_packets_for_kind.restype = ctypes.c_uint32
    if not hasattr(L, "sqobfs_pconn_open"):
        return L  # an older build (dev A/B against earlier rounds' libraries)
    L.sqobfs_set_sync_spin.argtypes = [vp, u32]
    L.sqobfs_debug_host_allocs.argtypes = []
    L.sqobfs_debug_host_allocs.restype = ctypes.c_int64
    L.sqobfs_pconn_open.argtypes = [vp, vp, i32, vp, ctypes.POINTER(vp)]
    L.sqobfs_pconn_shutdown.argtypes = [vp]
    L.sqobfs_pconn_shutdown.restype = None
    L.sqobfs_pconn_close.argtypes = [vp]
    L.sqobfs_pconn_close.restype = None
    L.sqobfs_pconn_write.argtypes = [vp, vp, u32, vp, ctypes.c_uint64]
    L.sqobfs_pconn_read.argtypes = [vp, vp, u32, u32p, vp, vp]
    L.sqobfs_pconn_set_deadline.argtypes = [vp, u32, ctypes.c_int64]
    L.sqobfs_pconn_rx_push.argtypes = [vp, vp, u32, vp, ctypes.c_uint64]
    L.sqobfs_pconn_rx_fail.argtypes = [vp, i32, i32]
    L.sqobfs_pconn_tx_take.argtypes = [vp, i32, vp]
    L.sqobfs_pconn_tx_done.argtypes = [vp]
    L.sqobfs_pconn_stats_get.argtypes = [vp, vp]
    if not hasattr(L, "sqobfs_cpu_run"):
        return L  # ABI 4
    L.sqobfs_cpu_run.argtypes = [vp, i32, ctypes.POINTER(Batch)]
    L.sqobfs_keyring_release_stream.argtypes = [vp, vp]
    L.sqobfs_debug_keyring_check.argtypes = [vp]
    L.sqobfs_engine_info_get.argtypes = [vp, vp]
    L.sqobfs_engine_set_workers.argtypes = [vp, u32]
    L.sqobfs_engine_trim.argtypes = [vp]
    L.sqobfs_debug_engine_fail.argtypes = [i32, i32]
    L.sqobfs_debug_engine_fail.restype = None
    L.sqobfs_shard_launch.argtypes = [u32, vp, vp, i32, vp, ctypes.POINTER(vp)]
    L.sqobfs_shard_query.argtypes = [vp]
    L.sqobfs_shard_wait.argtypes = [vp]
    if not hasattr(L, "sqobfs_debug_pool_fail"):
        return L  # ABI before round 5
    L.sqobfs_debug_pool_fail.argtypes = [i32]
    L.sqobfs_debug_pool_fail.restype = None
    L.sqobfs_debug_gcm_ungrouped.argtypes = [i32]
    L.sqobfs_debug_gcm_ungrouped.restype = None
    L.sqobfs_engine_set_affinity.argtypes = [vp, i32]
    L.sqobfs_debug_device_pool.argtypes = [vp, ctypes.c_uint64]
    L.sqobfs_debug_device_pool.restype = ctypes.c_uint64
    L.sqobfs_engine_set_group.argtypes = [vp, u32]
    L.sqobfs_debug_engine_hold.argtypes = [i32]
    L.sqobfs_debug_engine_hold.restype = None
    return L


def unit_packets_for(total_bytes: int, n: int, multi_psk: bool = False,
                     kind: int = SALAMANDER) -> int:
    """Unit size (packets per wavefront) for a batch of n packets holding
    total_bytes bytes, for the kind's kernel: sqobfs_unit_packets_for_kind."""
    return lib().sqobfs_unit_packets_for_kind(kind, total_bytes, n, int(multi_psk))


def build_info() -> str:
    return lib().sqobfs_build_info().decode()


def strerror(status: int) -> str:
    try:
        return lib().sqobfs_strerror(status).decode()
    except Exception:  # pragma: no cover - message only
        return "?"


def header_symbols() -> list[str]:
    """Every function declared in include/sqobfs.h."""
    src = open(HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sqobfs_[a-z0-9_]+)\s*\(", src)))


def _check(st: int, what: str) -> None:
    if st != SQ_OK:
        raise SqError(st, what)


def device_count() -> int:
    n = ctypes.c_int(0)
    st = lib().sqobfs_device_count(ctypes.byref(n))
    if st == SQ_ENODEV:
        return 0
    _check(st, "sqobfs_device_count")
    return n.value


def _ptr(a) -> int | None:
    """Address of a numpy array or torch tensor (None passes NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch.Tensor


class Context:
    """One GPU (sqobfs_open)."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib().sqobfs_open(device, ctypes.byref(h)), "sqobfs_open")
        self.handle = h
        self.device = device

    def close(self) -> None:
        if self.handle:
            lib().sqobfs_close(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def stream(self) -> int:
        return lib().sqobfs_stream(self.handle)

    def sync(self, stream: int | None = None) -> None:
        _check(lib().sqobfs_sync(self.handle, stream), "sqobfs_sync")

    @property
    def staging_bytes(self) -> int:
        """Pinned staging held by sqobfs_run_host."""
        return int(lib().sqobfs_host_staging_bytes(self.handle))

    def salt_key(self, key: bytes, next_seq: int = 0) -> None:
        """Deterministic device-salt key and sequence (tests / replay)."""
        assert len(key) == 32
        _check(lib().sqobfs_salt_key(self.handle, key, next_seq), "sqobfs_salt_key")

    @property
    def salt_seq(self) -> int:
        return lib().sqobfs_salt_seq(self.handle)

    def set_sync_spin(self, us: int) -> None:
        """sqobfs_sync polls the stream this long before blocking (opt-in)."""
        _check(lib().sqobfs_set_sync_spin(self.handle, us), "sqobfs_set_sync_spin")

    @property
    def unit_packets(self) -> int:
        """Packets per wavefront of the obfuscation kernel (tuning only)."""
        return lib().sqobfs_unit_packets(self.handle)

    @unit_packets.setter
    def unit_packets(self, packets: int) -> None:
        _check(lib().sqobfs_set_unit_packets(self.handle, packets), "sqobfs_set_unit_packets")


class Keyring:
    """Device copy of the PSK(s): the `password` field of
    SalamanderPacketConn (salamander.go:19-22) / `key` of XPlusPacketConn
    (xplus.go:39-44).  ctx=None makes a host keyring (no GPU: cpu_run and
    packet conns opened without a context)."""

    def __init__(self, ctx: Context | None, kind: int, psks: list[bytes]):
        blob = np.frombuffer(b"".join(psks) + b"\0", dtype=np.uint8).copy()
        lens = np.array([len(p) for p in psks], dtype=np.uint32)
        offs = np.zeros(len(psks), dtype=np.uint64)
        if len(psks) > 1:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        h = ctypes.c_void_p()
        _check(lib().sqobfs_keyring_create(ctx.handle if ctx else None, kind, len(psks), _ptr(blob),
                                           _ptr(offs), _ptr(lens), ctypes.byref(h)),
               "sqobfs_keyring_create")
        self.handle = h
        self.ctx = ctx
        self.kind = kind
        self.count = len(psks)

    def close(self) -> None:
        if self.handle:
            lib().sqobfs_keyring_destroy(self.handle)
            self.handle = None

    def release_stream(self, stream: int) -> None:
        """The caller is about to destroy `stream` (sqobfs_keyring_release_stream)."""
        _check(lib().sqobfs_keyring_release_stream(self.handle, stream),
               "sqobfs_keyring_release_stream")

    def device_check(self) -> int:
        """Entries whose device hash state differs from the host copy."""
        st = lib().sqobfs_debug_keyring_check(self.handle)
        if st < 0:
            raise SqError(st, "sqobfs_debug_keyring_check")
        return st

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def cpu_run(kr: Keyring, direction: int, batch: Batch) -> None:
    """The product's CPU path over a host batch (sqobfs_cpu_run)."""
    _check(lib().sqobfs_cpu_run(kr.handle, direction, ctypes.byref(batch)), "sqobfs_cpu_run")


class EngineInfo(ctypes.Structure):
    _fields_ = [("pconns", ctypes.c_uint32), ("threads", ctypes.c_uint32),
                ("workers", ctypes.c_uint32), ("pool_blocks", ctypes.c_uint32),
                ("pool_bytes", ctypes.c_uint64), ("blocks_in_use", ctypes.c_uint32),
                ("gpu_disabled", ctypes.c_uint32), ("route_bytes", ctypes.c_uint64),
                ("launch_us", ctypes.c_uint32), ("cpu_ns_per_kib", ctypes.c_uint32),
                ("load_permille", ctypes.c_uint32), ("loaded", ctypes.c_uint32),
                ("gpu_host_ns", ctypes.c_uint32), ("cpus", ctypes.c_uint32),
                ("group_max", ctypes.c_uint32), ("launches", ctypes.c_uint64),
                ("group_launches", ctypes.c_uint64), ("group_batches", ctypes.c_uint64),
                ("async_launches", ctypes.c_uint64), ("streams", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


def engine_set_group(ctx: Context | None, max_batches: int) -> None:
    """Most batches of several pconns one engine launch takes (0 = 32, 1 = no
    coalescing; sqobfs_engine_set_group)."""
    _check(lib().sqobfs_engine_set_group(ctx.handle if ctx else None, max_batches),
           "sqobfs_engine_set_group")


def engine_info(ctx: Context | None) -> EngineInfo:
    info = EngineInfo()
    _check(lib().sqobfs_engine_info_get(ctx.handle if ctx else None, ctypes.byref(info)),
           "sqobfs_engine_info_get")
    return info


def make_batch(n, in_, in_off, in_len, out, out_off, out_len, salt=None,
               psk_id=None, in_cap=None, salt_out=None, flags=0) -> Batch:
    """Batch from numpy arrays (host) or torch tensors (device).  The batch
    holds references to them: a launch reads them after this returns, so a
    temporary passed here must not be freed (and its memory reused) before
    the batch is."""
    b = Batch(n, flags, _ptr(in_), _ptr(in_off), _ptr(in_len), _ptr(out), _ptr(out_off),
              _ptr(out_len), _ptr(salt), _ptr(psk_id), _ptr(in_cap), _ptr(salt_out))
    b._keep = (in_, in_off, in_len, out, out_off, out_len, salt, psk_id, in_cap, salt_out)
    return b


def launch(ctx: Context, kr: Keyring, direction: int, batch: Batch,
           stream: int | None = None) -> None:
    """Device-resident launch (async on `stream`)."""
    _check(lib().sqobfs_launch(ctx.handle, kr.handle, direction, ctypes.byref(batch), stream),
           "sqobfs_launch")


def shard_cuts(in_len: np.ndarray, parts: int) -> np.ndarray:
    """sqobfs_shard_cuts: parts + 1 cut points balanced by bytes."""
    ln = np.ascontiguousarray(in_len, dtype=np.uint32)
    cut = np.zeros(parts + 1, dtype=np.uint32)
    _check(lib().sqobfs_shard_cuts(ln.size, _ptr(ln), parts, _ptr(cut)), "sqobfs_shard_cuts")
    return cut


def _handles(objs):
    return (ctypes.c_void_p * len(objs))(*[o.handle for o in objs])


def run_host_sharded(ctxs: list[Context], krs: list[Keyring], direction: int,
                     batch: Batch) -> None:
    """One host batch over several contexts, one host thread per shard."""
    _check(lib().sqobfs_run_host_sharded(len(ctxs), _handles(ctxs), _handles(krs), direction,
                                         ctypes.byref(batch)), "sqobfs_run_host_sharded")


def shard_run(ctxs: list[Context], krs: list[Keyring], direction: int,
              batches: list[Batch]) -> None:
    """Device-resident shards, shard k on ctxs[k]'s GPU; returns when all are done."""
    arr = (Batch * len(batches))(*batches)
    _check(lib().sqobfs_shard_run(len(ctxs), _handles(ctxs), _handles(krs), direction, arr),
           "sqobfs_shard_run")


class ShardTicket:
    """A step of device-resident shards in flight (sqobfs_shard_launch)."""

    def __init__(self, handle):
        self.handle = handle

    def done(self) -> bool:
        st = lib().sqobfs_shard_query(self.handle)
        if st < 0:
            raise SqError(st, "sqobfs_shard_query")
        return st == 1

    def wait(self) -> None:
        if self.handle:
            h, self.handle = self.handle, None
            _check(lib().sqobfs_shard_wait(h), "sqobfs_shard_wait")


def shard_launch(ctxs: list[Context], krs: list[Keyring], direction: int,
                 batches: list[Batch]) -> ShardTicket:
    """Queue shard k on ctxs[k]'s stream; returns at once (wait on the ticket)."""
    arr = (Batch * len(batches))(*batches)
    h = ctypes.c_void_p()
    _check(lib().sqobfs_shard_launch(len(ctxs), _handles(ctxs), _handles(krs), direction, arr,
                                     ctypes.byref(h)), "sqobfs_shard_launch")
    return ShardTicket(h)


def debug_gcm_ungrouped(on: bool) -> None:
    """Multi-key AES-128-GCM launches skip the grouping by key while on (the
    path taken when its scratch cannot be allocated)."""
    lib().sqobfs_debug_gcm_ungrouped(1 if on else 0)


def debug_device_pool(base: int | None, nbytes: int = 0) -> int:
    """Carve keyring tables and grouping scratch from [base, base + nbytes)
    (device memory the caller owns) until called with None; returns the bytes
    carved from the previous region."""
    return int(lib().sqobfs_debug_device_pool(base, nbytes))


def debug_pool_fail(count: int) -> None:
    """The next `count` packet conn engine batch-block allocations fail."""
    lib().sqobfs_debug_pool_fail(count)


def debug_fail_chunk(chunk: int) -> None:
    """Test hook: the next run_host fails (SQ_EDEVICE) at that pipeline chunk."""
    lib().sqobfs_debug_fail_chunk(chunk)


class DispatchEvents:
    """`count` pairs of HIP timing events, each pair recorded by one launch's
    own kernel dispatch (sqobfs_debug_time_next_launch): per-kernel times
    with no marker packets queued between the kernels, as a pair of
    hipEventRecord calls around each launch would.  Used by bench.py."""

    def __init__(self, count: int):
        self._hip = ctypes.CDLL("libamdhip64.so")
        self._hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self._hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float),
                                                  ctypes.c_void_p, ctypes.c_void_p]
        self._hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self.ev = []
        for _ in range(2 * count):
            e = ctypes.c_void_p()
            if self._hip.hipEventCreate(ctypes.byref(e)) != 0:
                self.close()
                raise SqError(-5, "hipEventCreate")
            self.ev.append(e)

    def arm(self, i: int) -> None:
        """The calling thread's next launch records pair i."""
        lib().sqobfs_debug_time_next_launch(self.ev[2 * i], self.ev[2 * i + 1])

    def elapsed_ms(self, i: int) -> float:
        ms = ctypes.c_float()
        st = self._hip.hipEventElapsedTime(ctypes.byref(ms), self.ev[2 * i], self.ev[2 * i + 1])
        if st != 0:
            self._hip.hipGetLastError()  # (HIP keeps the error until read)
            raise SqError(-5, f"hipEventElapsedTime: {st}")
        return ms.value

    def close(self) -> None:
        for e in self.ev:
            self._hip.hipEventDestroy(e)
        self.ev = []


def run_host(ctx: Context, kr: Keyring, direction: int, batch: Batch) -> None:
    """Host-memory batch (synchronous, staged through pinned memory)."""
    _check(lib().sqobfs_run_host(ctx.handle, kr.handle, direction, ctypes.byref(batch)),
           "sqobfs_run_host")


@dataclass
class HostBatch:
    """A ragged batch in host numpy arrays plus its output buffers."""
    data: np.ndarray
    in_off: np.ndarray
    in_len: np.ndarray
    out: np.ndarray
    out_off: np.ndarray
    out_len: np.ndarray
    salt: np.ndarray | None = None
    psk_id: np.ndarray | None = None
    in_cap: np.ndarray | None = None
    flags: int = 0
    salt_out: np.ndarray | None = None

    @property
    def n(self) -> int:
        return int(self.in_len.shape[0])

    def as_batch(self) -> Batch:
        return make_batch(self.n, self.data, self.in_off, self.in_len, self.out,
                          self.out_off, self.out_len, self.salt, self.psk_id, self.in_cap,
                          self.salt_out, self.flags)


class PinnedArray:
    """A uint8 numpy view of page-locked host memory (sqobfs_host_alloc);
    run_host DMAs such buffers directly instead of staging them."""

    def __init__(self, ctx: Context, nbytes: int):
        self._ctx = ctx
        p = ctypes.c_void_p()
        _check(lib().sqobfs_host_alloc(ctx.handle, max(nbytes, 1), ctypes.byref(p)),
               "sqobfs_host_alloc")
        self._p = p
        buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=np.uint8)[:nbytes]

    def free(self) -> None:
        if self._p is not None:
            self.array = None
            lib().sqobfs_host_free(self._ctx.handle, self._p)
            self._p = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.free()


def pack(packets: list[bytes], align: int = 16, lead: int = 0) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Pack byte strings into one buffer at `align`-aligned offsets (+lead)."""
    offs, pos = [], lead
    for p in packets:
        offs.append(pos)
        pos += len(p)
        pos = (pos + align - 1) // align * align + lead if align > 1 else pos
    buf = np.zeros(max(pos, 1) + 64, dtype=np.uint8)
    for o, p in zip(offs, packets):
        buf[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    return (buf, np.array(offs, dtype=np.uint64),
            np.array([len(p) for p in packets], dtype=np.uint32))


# ---------------------------------------------------------------- batched UDP

def udp_recv(fds: list[int], slots: np.ndarray, slot_bytes: int, headroom: int, max_n: int,
             timeout_ms: int):
    """sqobfs_udp_recv: (count, len[count], fd_index[count], [Addr])."""
    fa = np.asarray(fds, dtype=np.int32)
    ln = np.zeros(max_n, np.uint32)
    fi = np.zeros(max_n, np.uint16)
    addrs = (Addr * max_n)()
    cnt = ctypes.c_uint32(0)
    _check(lib().sqobfs_udp_recv(_ptr(fa), len(fds), _ptr(slots), slot_bytes, headroom, max_n,
                                 timeout_ms, _ptr(ln), _ptr(fi), addrs, ctypes.byref(cnt)),
           "sqobfs_udp_recv")
    n = cnt.value
    return n, ln[:n].copy(), fi[:n].copy(), list(addrs)[:n]


UDP_TX_GSO, UDP_RX_GRO = 1, 2  # sqobfs_udp_conn_set_offload flags


def udp_send(fd: int, base: np.ndarray, off, lens, to: list[Addr], gso: bool = False) -> int:
    """sqobfs_udp_send (sendmmsg), or sqobfs_udp_send_gso (UDP_SEGMENT runs)."""
    off = np.asarray(off, dtype=np.uint64)
    lens = np.asarray(lens, dtype=np.uint32)
    arr = (Addr * max(len(to), 1))(*to)
    sent = ctypes.c_uint32(0)
    fn = lib().sqobfs_udp_send_gso if gso else lib().sqobfs_udp_send
    _check(fn(fd, _ptr(base), _ptr(off), _ptr(lens), arr, len(to), ctypes.byref(sent)),
           "sqobfs_udp_send_gso" if gso else "sqobfs_udp_send")
    return sent.value


class UdpConn:
    """sqobfs_udp_conn: an obfuscating batched UDP endpoint over one or more
    sockets (hysteria port hopping fans several into one batch)."""

    def __init__(self, ctx: Context, kr: Keyring, fds: list[int], slots: int = 1024,
                 slot_bytes: int = 2048):
        self._fds = np.asarray(fds, dtype=np.int32)
        h = ctypes.c_void_p()
        _check(lib().sqobfs_udp_conn_open(ctx.handle, kr.handle, _ptr(self._fds), len(fds),
                                          slots, slot_bytes, ctypes.byref(h)),
               "sqobfs_udp_conn_open")
        self.handle = h
        self.slots, self.slot_bytes = slots, slot_bytes
        self.S = SALT_LEN[kr.kind]

    def close(self) -> None:
        if self.handle:
            lib().sqobfs_udp_conn_close(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_offload(self, flags: int) -> int:
        """sqobfs_udp_conn_set_offload: UDP_TX_GSO | UDP_RX_GRO; returns the
        flags in effect."""
        r = lib().sqobfs_udp_conn_set_offload(self.handle, flags)
        _check(min(r, 0), "sqobfs_udp_conn_set_offload")
        return r

    def read(self, timeout_ms: int = 1000):
        """[(payload bytes, fd_index, Addr)] of one received, decoded batch."""
        v = UdpView()
        _check(lib().sqobfs_udp_conn_read(self.handle, timeout_ms, ctypes.byref(v)),
               "sqobfs_udp_conn_read")
        out = []
        if v.count == 0:
            return out
        off = np.ctypeslib.as_array((ctypes.c_uint64 * v.count).from_address(v.off))
        ln = np.ctypeslib.as_array((ctypes.c_uint32 * v.count).from_address(v.len))
        fi = np.ctypeslib.as_array((ctypes.c_uint16 * v.count).from_address(v.fd_index))
        addrs = (Addr * v.count).from_address(v.from_)
        for i in range(v.count):  # copies: the next read reuses the endpoint's arrays
            out.append((ctypes.string_at(v.base + int(off[i]), int(ln[i])), int(fi[i]),
                        Addr.from_buffer_copy(addrs[i])))
        return out

    def write_quic(self, qkr: "QuicKeyring", fd_index: int, packets: list[bytes],
                   pn_offset: int, pns: list[int], to: list[Addr]) -> int:
        """QUIC packets (header || payload) -> one fused seal + Salamander
        launch -> send.  Returns datagrams sent."""
        lens = np.array([len(p) for p in packets], dtype=np.uint32)
        for i, p in enumerate(packets):
            self.tx_payload(i)[:len(p)] = np.frombuffer(p, np.uint8)
        pn = np.asarray(pns, dtype=np.uint64)
        arr = (Addr * max(len(to), 1))(*to)
        sent = ctypes.c_uint32(0)
        st = lib().sqobfs_udp_conn_write_quic(self.handle, qkr.handle, fd_index, len(packets),
                                              _ptr(lens), pn_offset, _ptr(pn), arr,
                                              ctypes.byref(sent))
        if st != SQ_OK:
            e = SqError(st, "sqobfs_udp_conn_write_quic")
            e.sent = sent.value  # datagrams sent before the failing packet
            raise e
        return sent.value

    def read_quic(self, qkr: "QuicKeyring", pn_offset: int, largest_pn: int,
                  timeout_ms: int = 1000):
        """[(packet bytes or None, out_len code, fd_index, Addr, pn)] of one
        received batch, de-obfuscated and opened in one launch."""
        v = UdpView()
        pp = ctypes.c_void_p()
        _check(lib().sqobfs_udp_conn_read_quic(self.handle, qkr.handle, pn_offset, largest_pn,
                                               timeout_ms, ctypes.byref(v), ctypes.byref(pp)),
               "sqobfs_udp_conn_read_quic")
        out = []
        if v.count == 0:
            return out
        off = np.ctypeslib.as_array((ctypes.c_uint64 * v.count).from_address(v.off))
        ln = np.ctypeslib.as_array((ctypes.c_uint32 * v.count).from_address(v.len))
        fi = np.ctypeslib.as_array((ctypes.c_uint16 * v.count).from_address(v.fd_index))
        pn = np.ctypeslib.as_array((ctypes.c_uint64 * v.count).from_address(pp.value))
        addrs = (Addr * v.count).from_address(v.from_)
        for i in range(v.count):
            n = int(ln[i])
            ok = n < 0xFFFFFFF0  # else a SQOBFS_QUIC_E* code: no packet, no number
            data = ctypes.string_at(v.base + int(off[i]), n) if ok else None
            out.append((data, n, int(fi[i]), Addr.from_buffer_copy(addrs[i]),
                        int(pn[i]) if ok else None))
        return out

    def tx_payload(self, i: int) -> np.ndarray:
        p = lib().sqobfs_udp_conn_tx_payload(self.handle, i)
        if not p:
            raise IndexError(i)
        n = self.slot_bytes - self.S
        return np.frombuffer((ctypes.c_uint8 * n).from_address(p), dtype=np.uint8)

    def write(self, fd_index: int, payloads: list[bytes], to: list[Addr]) -> int:
        """Copy payloads into the tx slots, obfuscate (device salts), send."""
        lens = np.array([len(p) for p in payloads], dtype=np.uint32)
        for i, p in enumerate(payloads):
            self.tx_payload(i)[:len(p)] = np.frombuffer(p, np.uint8)
        arr = (Addr * max(len(to), 1))(*to)
        sent = ctypes.c_uint32(0)
        _check(lib().sqobfs_udp_conn_write(self.handle, fd_index, len(payloads), _ptr(lens), arr,
                                           ctypes.byref(sent)), "sqobfs_udp_conn_write")
        return sent.value


# ---------------------------------------------------------------- QUIC

class QuicKeyring:
    """Device copy of per-connection QUIC 1-RTT keys (sqobfs_quic_keyring) of
    one suite: QUIC_CHACHA20_POLY1305 (default) or QUIC_AES_128_GCM."""

    def __init__(self, ctx: Context, keys: list[QuicKey], suite: int = QUIC_CHACHA20_POLY1305):
        arr = (QuicKey * len(keys))(*keys)
        h = ctypes.c_void_p()
        _check(lib().sqobfs_quic_keyring_create_suite(ctx.handle, suite, len(keys), arr,
                                                      ctypes.byref(h)),
               "sqobfs_quic_keyring_create_suite")
        self.suite = suite
        self.handle = h
        self.ctx = ctx
        self.count = len(keys)

    def close(self) -> None:
        if self.handle:
            lib().sqobfs_quic_keyring_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def quic_batch(n, in_, in_off, in_len, out, out_off, out_len, pn_offset, pn, key_id=None,
               pn_out=None) -> QuicBatch:
    b = QuicBatch(n, 0, _ptr(in_), _ptr(in_off), _ptr(in_len), _ptr(out), _ptr(out_off),
                  _ptr(out_len), _ptr(pn_offset), _ptr(pn), _ptr(key_id), _ptr(pn_out))
    b._keep = (in_, in_off, in_len, out, out_off, out_len, pn_offset, pn, key_id, pn_out)  # (make_batch)
    return b


def quic_seal(ctx: Context, kr: QuicKeyring, batch: QuicBatch, stream=None) -> None:
    _check(lib().sqobfs_quic_seal(ctx.handle, kr.handle, ctypes.byref(batch), stream),
           "sqobfs_quic_seal")


def quic_open(ctx: Context, kr: QuicKeyring, batch: QuicBatch, stream=None) -> None:
    _check(lib().sqobfs_quic_open(ctx.handle, kr.handle, ctypes.byref(batch), stream),
           "sqobfs_quic_open")


def quic_seal_salamander(ctx: Context, kr: QuicKeyring, okr: Keyring, batch: QuicBatch, salt,
                         stream=None) -> None:
    """Seal + Salamander obfuscation in one pass (wire = salt || obfs(packet))."""
    _check(lib().sqobfs_quic_seal_salamander(ctx.handle, kr.handle, okr.handle,
                                             ctypes.byref(batch), _ptr(salt), stream),
           "sqobfs_quic_seal_salamander")


def quic_open_salamander(ctx: Context, kr: QuicKeyring, okr: Keyring, batch: QuicBatch,
                         stream=None) -> None:
    """Salamander de-obfuscation + open in one pass."""
    _check(lib().sqobfs_quic_open_salamander(ctx.handle, kr.handle, okr.handle,
                                             ctypes.byref(batch), stream),
           "sqobfs_quic_open_salamander")
