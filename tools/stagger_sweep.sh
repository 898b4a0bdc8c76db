# cn_linear bf16x6 epilogue timings vs the workgroup stagger and the tile choice (GPU box)
for w in 0x1f 0x07; do for st in 0 2 4; do echo "wide $w stagger $st"; COPENERF_WIDE_EPIS=$w COPENERF_STAGGER=$st ONLY=x6 timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | grep -v wgrad; done; done
