"""The C++ mirror of the reference's PacketConn decorators
(sing-quic_amd/host/packet_conn.*): behaviour checked against the oracle
(tests/cpp/test_packet_conn.cpp) on the GPU and, with no GPU at all, on the
library's CPU path (the constructors do not fail without a device, as the
reference's cannot)."""
from __future__ import annotations

import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "test_packet_conn.cpp")
OUT = os.path.join(REPO, "build", "test_packet_conn")


def _compile() -> str:
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    lib = os.path.join(REPO, "sing-quic_amd")
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(REPO, "include"),
           "-I", os.path.join(lib, "host"), "-I", os.path.join(REPO, "oracle"), SRC,
           "-L", lib, "-lsqobfs", "-L", os.path.join(REPO, "oracle"), "-loracle",
           f"-Wl,-rpath,{lib}", f"-Wl,-rpath,{os.path.join(REPO, 'oracle')}", "-o", OUT]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return OUT


def test_host_mirror_compiles_and_links():
    assert os.path.exists(os.path.join(REPO, "sing-quic_amd", "libsqobfs.so"))
    _compile()


def test_host_mirror_without_a_device():
    """No GPU in this process's view: every transform on the CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present (the -m gpu test covers it)")
    exe = _compile()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


@pytest.mark.gpu
def test_host_mirror_against_oracle():
    exe = _compile()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


CGO_SRC = os.path.join(REPO, "tests", "cpp", "test_cgo_sequence.c")
CGO_OUT = os.path.join(REPO, "build", "test_cgo_sequence")


def _compile_cgo_replay() -> str:
    os.makedirs(os.path.dirname(CGO_OUT), exist_ok=True)
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    lib = os.path.join(REPO, "sing-quic_amd")
    cmd = ["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-I", os.path.join(REPO, "include"),
           "-I", os.path.join(REPO, "oracle"), CGO_SRC, "-L", lib, "-lsqobfs",
           "-L", os.path.join(REPO, "oracle"), "-loracle", f"-Wl,-rpath,{lib}",
           f"-Wl,-rpath,{os.path.join(REPO, 'oracle')}", "-o", CGO_OUT]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return CGO_OUT


def test_cgo_replay_compiles_as_c():
    """The Go binding's call sequence (tests/cpp/test_cgo_sequence.c) is plain
    C against include/sqobfs.h: what cgo sees."""
    _compile_cgo_replay()


@pytest.mark.gpu
def test_cgo_replay_against_oracle():
    exe = _compile_cgo_replay()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout
