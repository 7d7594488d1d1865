set -u
export TMPDIR=/tmp; OUT=gpurun_out; mkdir -p $OUT
for v in x0 x1 x2; do
  if [ $v = x2 ]; then L=gym-ignition_amd/libmwstep.so; else L=gym-ignition_amd/libmwstep_$v.so; fi
  MWSTEP_LIB=$PWD/$L timeout -k 10 200 python -u -m pytest "tests/test_gpu_group.py" "tests/test_gpu_panda.py::test_panda_vecenv_vs_oracle" -s -q --timeout 150 --timeout-method thread > $OUT/var_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc"; grep -E "max\||vs oracle|passed|failed" $OUT/var_$v.log | tail -6; [ $rc -le 1 ] || exit $rc
  MWSTEP_LIB=$PWD/$L timeout -k 10 120 python scripts/leg_probe.py panda > $OUT/var_leg_$v.log 2>&1 || exit 3
  grep -o '"kernel_us_per_launch": [0-9.]*' $OUT/var_leg_$v.log | head -2
done
