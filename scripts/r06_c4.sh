#!/usr/bin/env bash
# Config-4 check of the group kernel: its GPU tests, then the panda legs alone
# (1,024 worlds and the 8-GPU shares), then the counter passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p "$OUT"; tag="${1:-r06c4}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_panda.py tests/test_gpu_shard.py -v -s \
  --timeout 200 --timeout-method thread > "$OUT/pytest_c4_$tag.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_c4_$tag.log"; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python scripts/leg_probe.py panda panda/8 > "$OUT/legs_c4_$tag.log" 2>&1
rc=$?; echo "legs rc=$rc"; tail -c 1500 "$OUT/legs_c4_$tag.log"; [ $rc -eq 0 ] || exit $rc
[ "${PMC:-1}" = "1" ] && bash scripts/r06_pmc.sh "$tag"
exit 0
