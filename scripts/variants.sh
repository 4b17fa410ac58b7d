#!/bin/bash
# Build timing variants of libsqobfs.so: scripts/variants.sh name:"-DFLAGS" ...
set -e
cd "$(dirname "$0")/.."
V=${VARDIR:-build/var}; mkdir -p $V
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -Iinclude \
    -Ising-quic_amd/csrc -Ising-quic_amd/host -shared -o $V/lib_$name.so \
    sing-quic_amd/csrc/*.hip sing-quic_amd/host/*.cpp &
done
wait
