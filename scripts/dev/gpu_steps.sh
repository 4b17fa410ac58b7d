#!/bin/bash
# GPU box: run steps one after another, each under its own time limit;
# a step that fails ordinarily (exit 1-127) is recorded and the next runs,
# but a time limit (124 / 137), an abort (134), a segfault (139) or any
# other signal ends the call there -- nothing more touches the GPU after
# it.  usage: gpu_steps.sh OUTDIR "SECONDS name command..." ...
# Each step's output goes to OUTDIR/<name>.log; OUTDIR/steps.txt records
# the exit codes.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p "$O"
for step in "$@"; do
  read -r secs name cmd <<< "$step"
  timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  echo "$name rc $rc" | tee -a "$O/steps.txt"
  if [ $rc -ge 124 ]; then
    echo "stopping after $name (rc $rc)" | tee -a "$O/steps.txt"
    tail -20 "$O/$name.log"
    exit $rc
  fi
done
