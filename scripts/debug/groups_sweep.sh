set -e
for g in 1 2 4 8; do
  timeout -k 10 120 python bench.py --groups $g --steps 2000 --warmup 200 --no-cpu-baseline --no-sweep --no-rollout --no-panda > gpurun_out/grp_c2_$g.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/grp_c2_$g.json')); print('C2 groups=$g', d['value'], d['ms_per_step'])"
done
for g in 1 2 4; do
  timeout -k 10 120 python bench.py --task PandaPositionTracking --worlds 1024 --groups $g --steps 1000 --warmup 100 --no-cpu-baseline --no-sweep --no-rollout --no-panda > gpurun_out/grp_c4_$g.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/grp_c4_$g.json')); print('C4 groups=$g', d['value'], d['ms_per_step'])"
done
