# SQ counters of the config-4 Panda env kernel, lane vs group kernels
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/probe
for k in group lane; do
  MWSTEP_PANDA_KERNEL=$k timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    --kernel-trace --output-format csv -d gpurun_out/probe/sq_$k -o run -- python3 scripts/profile_panda.py > gpurun_out/probe/sq_$k.log 2>&1 || { echo "rc=$?"; exit 1; }
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/probe/trace_group -o run -- python3 scripts/profile_panda.py > gpurun_out/probe/trace_group.log 2>&1 || { echo "rc=$?"; exit 1; }
echo ok
