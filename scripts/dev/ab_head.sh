#!/bin/bash
# Dev (container): build the library of a git revision (default HEAD) in a
# temporary worktree and put it beside the working tree's build as
# build/ablate/{a_<rev>,b_new,c_<rev>,d_new}/libsqobfs.so (two copies each:
# scripts/dev/gcm_ablate_run.sh then times them interleaved on one box).
# usage: scripts/dev/ab_head.sh [rev]
set -e
REPO=$(cd "$(dirname "$0")/../.." && pwd)
REV=${1:-HEAD}
WT=$(mktemp -d /tmp/sqwt.XXXXXX)
git -C "$REPO" worktree add -f "$WT" "$REV" -q
make -s -C "$WT/sing-quic_amd" -j8 2>&1 | grep -v hip-link || true
rm -rf "$REPO/build/ablate"
for d in a_old c_old; do mkdir -p "$REPO/build/ablate/$d"; cp "$WT/sing-quic_amd/libsqobfs.so" "$REPO/build/ablate/$d/"; done
for d in b_new d_new; do mkdir -p "$REPO/build/ablate/$d"; cp "$REPO/sing-quic_amd/libsqobfs.so" "$REPO/build/ablate/$d/"; done
git -C "$REPO" worktree remove --force "$WT"
echo "built $REV vs working tree"
