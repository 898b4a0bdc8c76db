# C2 step time vs the bf16x6 tall-tile epilogue mask (COPENERF_X6_TALL), alternating (GPU box)
for r in 1 2; do for t in 0x18 0x1a 0x1f; do COPENERF_X6_TALL=$t timeout -k 10 300 python bench.py --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('tall $t', d['value'], d['ms_per_step'])"; done; done
