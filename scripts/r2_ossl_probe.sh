#!/bin/bash
# GPU box (CPU only): does OpenSSL 3.0's ChaCha20-Poly1305 scale over threads / processes here?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ossl
gcc -O2 -o /tmp/ot scripts/dev/ossl_threads.c -lcrypto -lpthread && gcc -O2 -o /tmp/op scripts/dev/ossl_procs.c -lcrypto || exit 1
for T in 1 4 16; do timeout 60 /tmp/ot 0 $T; timeout 60 /tmp/ot 3 $T; timeout 60 /tmp/op $T; done 2>&1 | tee gpurun_out/ossl/probe.txt
