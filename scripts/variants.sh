#!/bin/bash
# Build timing variants of libsqobfs.so: scripts/variants.sh name:"-DFLAGS" ...
# (the flags go to the HIP sources; the host sources are shared, host-only)
# VARDIR: output directory (default build/ab, which travels to the GPU box).
set -e
cd "$(dirname "$0")/.."
V=${VARDIR:-build/ab}
mkdir -p $V/obj
HOSTCXX=${HOSTCXX:-/opt/rocm/lib/llvm/bin/clang++}
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Ising-quic_amd/csrc -Ising-quic_amd/host"
hobjs=()
for f in sing-quic_amd/host/*.cpp; do
  o=$V/obj/host_$(basename ${f%.cpp}).o
  $HOSTCXX -O3 -std=c++17 -fPIC -Iinclude -Ising-quic_amd/csrc -Ising-quic_amd/host -c $f -o $o &
  hobjs+=($o)
done
wait
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  (
    kobjs=()
    for f in sing-quic_amd/csrc/*.hip; do
      o=$V/obj/${name}_$(basename ${f%.hip}).o
      /opt/rocm/bin/hipcc $HIPFLAGS $flags -c $f -o $o
      kobjs+=($o)
    done
    /opt/rocm/bin/hipcc $HIPFLAGS -shared -o $V/lib_$name.so "${kobjs[@]}" "${hobjs[@]}" -lpthread
  ) &
done
wait
