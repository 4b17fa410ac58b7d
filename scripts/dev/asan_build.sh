#!/bin/bash
# Dev: AddressSanitizer build of the HOST code of libsqobfs (the device code
# is not instrumented: GPU sanitizers are not used on this pool) and of the
# threaded C tests that drive it (packet conn engine, cgo call-sequence
# replay).  Built here on the CPU; run on the GPU box by scripts/dev/asan_run.sh.
set -e
cd "$(dirname "$0")/../.."
O=build/asan; mkdir -p $O
CL=/opt/rocm/llvm/bin/clang
SAN="-fsanitize=address -fno-omit-frame-pointer"
/opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address \
  -Xarch_host -fno-omit-frame-pointer -Iinclude -Ising-quic_amd/csrc -Ising-quic_amd/host \
  -shared -shared-libasan -Wl,-rpath,/opt/rocm/llvm/lib/clang/22/lib/linux -o $O/libsqobfs.so sing-quic_amd/csrc/*.hip sing-quic_amd/host/*.cpp -lpthread
make -s -C oracle
for t in test_pconn test_cgo_sequence; do
  $CL -std=c11 -O1 -g $SAN -shared-libasan -Iinclude -Ioracle tests/cpp/$t.c -L$O -lsqobfs \
    -Loracle -loracle -lpthread -Wl,-rpath,$PWD/$O -Wl,-rpath,$PWD/oracle -Wl,-rpath,/opt/rocm/llvm/lib/clang/22/lib/linux -o $O/$t
done
$CL++ -std=c++17 -O1 -g $SAN -shared-libasan -Iinclude -Ising-quic_amd/host -Ioracle \
  tests/cpp/test_packet_conn.cpp -L$O -lsqobfs -Loracle -loracle -lpthread -Wl,-rpath,$PWD/$O \
  -Wl,-rpath,$PWD/oracle -Wl,-rpath,/opt/rocm/llvm/lib/clang/22/lib/linux -o $O/test_packet_conn
# the latency tool drives the UDP endpoint (sqobfs_udp_conn_*) and the engine
$CL -std=c11 -O1 -g $SAN -shared-libasan -Iinclude sing-quic_amd/tools/lat_bench.c -L$O -lsqobfs \
  -Loracle -loracle -lpthread -Wl,-rpath,$PWD/$O -Wl,-rpath,$PWD/oracle \
  -Wl,-rpath,/opt/rocm/llvm/lib/clang/22/lib/linux -o $O/lat_bench
ls -la $O
