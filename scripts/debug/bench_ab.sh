set -e
for i in 1; do
timeout -k 10 120 python scripts/debug/bench_head.py --steps 2000 --warmup 200 --no-cpu-baseline --no-sweep --no-rollout --no-panda > gpurun_out/bh.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/bh.json')); print('HEAD', d['value'], d['ms_per_step'], d['roofline']['kernel_us_per_launch'])"
timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-sweep --no-rollout --no-panda > gpurun_out/bn.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/bn.json')); print('NEW ', d['value'], d['ms_per_step'], d['roofline']['kernel_us_per_launch'])"
done
for g in 2 4; do
timeout -k 10 120 python bench.py --groups $g --steps 2000 --warmup 200 --no-cpu-baseline --no-sweep --no-rollout --no-panda > gpurun_out/bn.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/bn.json')); print('NEW g=$g', d['value'], d['ms_per_step'], d['roofline']['kernel_us_per_launch'])"
done
