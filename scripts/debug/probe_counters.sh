set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/probe
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/probe/avail.txt 2>&1; echo "list rc=$?"
for W in 256 4096; do
  PANDA_WORLDS=$W timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/probe/fetch_$W -o run -- python3 scripts/profile_panda.py > gpurun_out/probe/fetch_$W.log 2>&1 || { echo "fetch $W rc=$?"; exit 1; }
done
echo ok
