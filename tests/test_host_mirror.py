"""The C++ mirror of the reference's PacketConn decorators
(sing-quic_amd/host/packet_conn.*): compiles on CPU; behaviour checked
against the oracle on the GPU (tests/cpp/test_packet_conn.cpp)."""
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


@pytest.mark.gpu
def test_host_mirror_against_oracle():
    exe = _compile()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout
