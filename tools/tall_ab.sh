# A/B of the bf16x6 tilings (COPENERF_X6_TALL epilogue mask), alternating rounds (GPU box)
for r in 1 2; do for t in 0 0x7f; do echo "== tall $t round $r"; COPENERF_X6_TALL=$t ONLY=x6 timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | grep -v wgrad; done; done
