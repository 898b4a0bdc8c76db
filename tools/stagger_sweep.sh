# cn_linear bf16x6 epilogue timings vs the workgroup stagger (GPU box)
for st in ${@:-0 2 4 8}; do echo "stagger $st"; COPENERF_STAGGER=$st ONLY=x6 timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | grep -v wgrad; done
