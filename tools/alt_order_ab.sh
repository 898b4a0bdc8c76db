# C2 bench with and without the alternating M-tile order (COPENERF_ALT_ORDER), alternating (GPU box)
for r in 1 2; do for a in 0 1; do COPENERF_ALT_ORDER=$a timeout -k 10 300 python bench.py --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('alt $a', d['value'], d['ms_per_step'])"; done; done
