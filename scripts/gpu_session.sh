#!/usr/bin/env bash
# One GPU-box session: gpu tests -> smoke -> bench (driver command) -> phase
# profiles of the wave kernel -> per-env path profile.  Output under
# gpurun_out/<tag>_*.  A pytest failure does not stop the session; a timeout,
# abort or crash does (scripts/gpu_steps.sh).
tag=${1:-r03}
exec scripts/gpu_steps.sh \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1" \
  "timeout -k 10 150 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${tag}_smoke.log 2>&1" \
  "timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err" \
  "MWSTEP_LIB=gym-ignition_amd/libmwstep_prof.so timeout -k 10 120 python scripts/wave_prof.py 64 50 > gpurun_out/${tag}_wave_prof64.log 2>&1" \
  "MWSTEP_LIB=gym-ignition_amd/libmwstep_prof.so timeout -k 10 120 python scripts/wave_prof.py 512 50 > gpurun_out/${tag}_wave_prof512.log 2>&1" \
  "timeout -k 10 120 python scripts/profile_runtime_c1.py 2000 > gpurun_out/${tag}_runtime_prof.log 2>&1"
