#!/usr/bin/env bash
# round 4, final build: configs[4] traces + PMC and the bench table of every
# config / direction / layout (profile_configs.sh part 2)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 1100 bash scripts/profile_configs.sh r04f 2 || { echo "profiles rc=$?"; exit 1; }
