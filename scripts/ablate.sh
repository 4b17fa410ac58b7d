#!/bin/bash
# Build timing-only ablation variants of libsqobfs.so into build/ablate/.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ablate
for v in 1 2 3; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSQ_ABLATE=$v -Iinclude \
    -Ising-quic_amd/csrc -shared -o build/ablate/libsqobfs_a$v.so \
    sing-quic_amd/csrc/sq_kernels.hip sing-quic_amd/csrc/sq_api.hip &
done
wait
ls build/ablate
