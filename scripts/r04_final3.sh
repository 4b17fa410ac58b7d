#!/usr/bin/env bash
# round 4, final build with the span-timed bench: every config's kernel trace
# + PMC passes, the default bench line and the table of every config /
# direction / layout (profile_configs.sh all)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 1150 bash scripts/profile_configs.sh r04g all || { echo "profiles rc=$?"; exit 1; }
