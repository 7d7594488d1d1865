# SQ counters of the config-4 Panda env kernel (group kernel), two passes
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/probe
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d gpurun_out/probe/sq_group -o run -- python3 scripts/profile_panda.py > gpurun_out/probe/sq_group.log 2>&1 || { echo "rc=$?"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/probe/sq2_group -o run -- python3 scripts/profile_panda.py > gpurun_out/probe/sq2_group.log 2>&1 || { echo "rc=$?"; exit 1; }
echo ok
