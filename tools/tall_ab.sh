# A/B of the bf16x6 tile per epilogue (COPENERF_X6_TALL mask: 128x256 tiles), alternating rounds (GPU box)
#   bash tools/tall_ab.sh MASK_A MASK_B
for r in 1 2; do for t in ${1:-0x18} ${2:-0x78}; do echo "== tall $t round $r"; COPENERF_X6_TALL=$t ONLY=x6 timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | grep -v wgrad; done; done
