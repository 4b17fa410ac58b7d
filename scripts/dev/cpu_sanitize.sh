#!/usr/bin/env bash
# The packet conn engine (host/pconn.cpp), the CPU path (host/sq_cpu.cpp) and
# the UDP layer (host/udp_batch.cpp) built WITHOUT HIP, over the CPU device
# of tests/cpp/sq_devstub.cpp, and tests/cpp/test_pconn.c run on them under
# AddressSanitizer (+UBSan) and ThreadSanitizer -- in the container, on host
# code only (GPU sanitizers are not available on the GPU pool, and a
# sanitized process that initialises HIP aborted in the ASan runtime's
# device allocator there in round 3).
#
#   scripts/dev/cpu_sanitize.sh [plain|asan|tsan ...]   (default: asan tsan)
#
# Logs: build/san/<variant>.log; the summaries are copied to profiles/r04/asan/.
set -euo pipefail
REPO="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$REPO/build/san"
mkdir -p "$OUT"
make -s -C "$REPO/oracle"
variants=("$@")
[ ${#variants[@]} -eq 0 ] && variants=(asan tsan)
SRCS=("$REPO/sing-quic_amd/host/pconn.cpp" "$REPO/sing-quic_amd/host/sq_cpu.cpp"
      "$REPO/sing-quic_amd/host/udp_batch.cpp" "$REPO/tests/cpp/sq_devstub.cpp")
INC=(-I "$REPO/include" -I "$REPO/sing-quic_amd/csrc" -I "$REPO/sing-quic_amd/host"
     -I "$REPO/oracle")
LLVM=/opt/rocm/lib/llvm/bin
for v in "${variants[@]}"; do
  CXX=g++ CC=gcc
  case "$v" in
    plain) SAN=(-O2) ;;
    asan) SAN=(-O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined
               -fno-sanitize-recover=undefined) ;;
    # clang's TSan runtime: GCC 11's libtsan does not intercept
    # pthread_cond_clockwait (std::condition_variable::wait_for / wait_until
    # with libstdc++ 11), so it reports every timed wait as a double lock
    tsan) SAN=(-O1 -g -fsanitize=thread) CXX=$LLVM/clang++ CC=$LLVM/clang ;;
    *) echo "unknown variant $v" >&2; exit 2 ;;
  esac
  d="$OUT/$v"
  mkdir -p "$d"
  objs=()
  for s in "${SRCS[@]}"; do
    o="$d/$(basename "${s%.*}").o"
    $CXX -std=c++17 -Wall -Wextra "${SAN[@]}" "${INC[@]}" -c "$s" -o "$o"
    objs+=("$o")
  done
  $CC -std=c11 -Wall -Wextra "${SAN[@]}" "${INC[@]}" -c "$REPO/tests/cpp/test_pconn.c" \
    -o "$d/test_pconn.o"
  $CXX "${SAN[@]}" "$d/test_pconn.o" "${objs[@]}" -L "$REPO/oracle" -loracle -lpthread \
    -Wl,-rpath,"$REPO/oracle" -o "$d/test_pconn"
  log="$OUT/$v.log"
  : > "$log"
  for mode in gpu nodev; do
    echo "== $v: test_pconn $mode (CPU device: tests/cpp/sq_devstub.cpp)" | tee -a "$log"
    # halt_on_error: any report fails the run
    ASAN_OPTIONS=detect_leaks=1:halt_on_error=1 TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 \
      timeout -k 10 900 "$d/test_pconn" "$mode" >> "$log" 2>&1
    echo "   exit 0" | tee -a "$log"
  done
done
