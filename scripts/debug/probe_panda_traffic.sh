# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the config-4 Panda env kernel
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/probe
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/probe/panda_$c -o run -- python3 scripts/profile_panda.py > gpurun_out/probe/panda_$c.log 2>&1 || { echo "rc=$?"; exit 1; }
done
python scripts/pmc_summary.py gpurun_out/probe/panda_FETCH_SIZE gpurun_out/probe/panda_WRITE_SIZE gpurun_out/probe/panda_traffic.json --kernel vecenv_pid_group_kernel --task PandaPositionTracking --worlds 1024
