# C2 / c3fp32 bench of two source trees (the committed HEAD exported to ab/head vs the working
# tree), alternating, on one box (GPU box)
for r in 1 2; do for t in ab/head .; do for c in c2 c3fp32; do
  (cd $t && timeout -k 10 300 python bench.py --config $c --no-cpu-baseline 2>/dev/null) | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$t $c', d['value'])"
done; done; done
