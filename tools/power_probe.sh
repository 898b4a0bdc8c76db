#!/bin/bash
# Board power and clocks while the C2 step runs (is the GEMM step at the power cap?): rocm-smi sampled
# every ~0.5 s during a long bench run, idle samples before it.
mkdir -p gpurun_out/pw
(rocm-smi --showpower --showclocks --showtemp > gpurun_out/pw/idle.txt 2>&1 || true)
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 5 --no-cpu-baseline > gpurun_out/pw/bench.json 2> gpurun_out/pw/bench.err &
BP=$!
sleep 20
for i in $(seq 1 30); do (rocm-smi --showpower --showclocks 2>&1 | grep -Ei "power|sclk|fclk|mclk" >> gpurun_out/pw/samples.txt || true); echo "--" >> gpurun_out/pw/samples.txt; sleep 0.5; done
(rocm-smi --showmaxpower > gpurun_out/pw/maxpower.txt 2>&1 || true)
wait $BP
echo "bench rc=$?"
tail -c 200 gpurun_out/pw/bench.json
