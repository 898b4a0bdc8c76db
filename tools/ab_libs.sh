# A/B two builds of libcopenerf.so with tools/gemm_bench.py, alternating, 2 rounds (GPU box)
#   bash tools/ab_libs.sh libA.so libB.so [ONLY filter]
for r in 1 2; do for L in "$1" "$2"; do echo "== $L round $r"; COPENERF_LIB=$L ONLY=${3:-x6} timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids; done; done
