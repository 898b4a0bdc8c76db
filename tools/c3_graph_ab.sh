# c3 / c3fp32 eager vs HIP-graph replay (GPU box)
for c in c3fp32 c3; do for g in "" "--graph"; do timeout -k 10 400 python bench.py --config $c $g --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$c $g', d['value'], d['ms_per_step'])"; done; done
