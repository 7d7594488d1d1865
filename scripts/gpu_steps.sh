#!/usr/bin/env bash
# Run GPU steps in order; a pytest failure (exit 1) does not stop the chain,
# any other non-zero exit (timeout, abort, segfault) does.
#   scripts/gpu_steps.sh 'cmd1 > log1' 'cmd2 > log2' ...
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in "$@"; do
  echo "== $step"
  bash -c "$step"
  rc=$?
  echo "rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "FATAL rc=$rc: no further GPU steps"
    exit "$rc"
  fi
done
exit 0
