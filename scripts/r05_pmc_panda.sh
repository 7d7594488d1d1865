#!/usr/bin/env bash
# r05: where config 4's extra L2->memory read bytes come
# from.  Counter passes (one rocprofv3 run each, separate processes) on
# vecenv_pid_group_kernel<9>: FETCH_SIZE at 64 / 256 / 1024 worlds (a constant
# term that does not grow with the world count is not data), the instruction
# and scalar-data requests of the SQC (instruction / scalar caches) to the
# L2, their misses, and the L2's memory read requests by size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05p}
mkdir -p "$OUT"
run() {  # $1 = tag, $2 = worlds, rest = counters
  local tag=$1 w=$2; shift 2
  PANDA_WORLDS=$w timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/pmc_$tag" -o run -- python3 scripts/profile_panda.py > "$OUT/pmc_$tag.log" 2>&1
  local rc=$?
  echo "pass $tag ($w worlds: $*) rc=$rc"
  if [ "$rc" -ne 0 ]; then exit $rc; fi
}
run fetch64 64 FETCH_SIZE
run fetch256 256 FETCH_SIZE
run fetch1024 1024 FETCH_SIZE
run write1024 1024 WRITE_SIZE
run sqc_tc 1024 SQC_TC_INST_REQ SQC_TC_DATA_READ_REQ
run sqc_miss 1024 SQC_ICACHE_MISSES SQC_DCACHE_MISSES
run sqc_tc64 64 SQC_TC_INST_REQ SQC_TC_DATA_READ_REQ
run rdreq 1024 TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B
exit 0
