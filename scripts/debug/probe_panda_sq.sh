# SQ / SQC counters of the config-4 Panda env kernel (instruction-fetch study)
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/probe
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS \
  --kernel-trace --output-format csv -d gpurun_out/probe/panda_sq -o run -- python3 scripts/profile_panda.py > gpurun_out/probe/panda_sq.log 2>&1 || { echo "rc=$?"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQC_ICACHE_MISSES SQC_ICACHE_REQ \
  --kernel-trace --output-format csv -d gpurun_out/probe/step_sq -o run -- python3 scripts/profile_step.py > gpurun_out/probe/step_sq.log 2>&1 || { echo "rc=$?"; exit 1; }
echo ok
