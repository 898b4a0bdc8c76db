#!/bin/bash
# Same-box A/B of the C2 bench step under environment variants, interleaved REPS times.
#   ARMS="A=COPENERF_X=1;B=COPENERF_X=2" REPS=3 CONFIG=c2 bash tools/env_ab.sh
# Each arm: NAME=VAR=VAL[,VAR=VAL...]; one JSON line per run in gpurun_out/env_ab/res.jsonl
set -eo pipefail
mkdir -p gpurun_out/env_ab
IFS=';' read -ra arms <<< "${ARMS:-base=}"
for rep in $(seq ${REPS:-3}); do
  for arm in "${arms[@]}"; do
    name=${arm%%=*}; spec=${arm#*=}
    envs=()
    IFS=',' read -ra kv <<< "$spec"
    for x in "${kv[@]}"; do [ -n "$x" ] && envs+=("$x"); done
    out=$(env "${envs[@]}" timeout -k 10 300 python bench.py --config ${CONFIG:-c2} --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --timer-steps 1 2>/dev/null | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(json.dumps({'arm': sys.argv[1], 'rep': int(sys.argv[3]), 'value': d['value'], 'ms': d['ms_per_step']}))" "$name" "$out" "$rep" | tee -a gpurun_out/env_ab/res.jsonl
  done
done
