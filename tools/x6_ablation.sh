#!/bin/bash
# bf16x6 main-loop ablations (cn_gemm.hip X6_EXP): build here with `build`, run on the GPU box with `run`.
#   0 baseline  1 RNE convert instead of split3 (VALU cost of the split)  2 three products instead of six
#   3 term-0 fragments only (LDS read cost)  4 no A global loads  5 no B loads
R=$(cd "$(dirname "$0")/.." && pwd)
V=${VARIANTS:-"0 1 2 3 4 5"}
FLAG=${FLAG:-X6_EXP}  # X6_EXP (cn_gemm.hip main-loop ablations)
if [ "$1" = build ]; then
  cd $R/cope-nerf_amd/csrc
  for n in $V; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -D$FLAG=$n \
      -o $R/tools/abl/lib_${FLAG}_$n.so cn_abi.hip cn_gemm.hip cn_fields.hip cn_render.hip cn_pack.hip cn_loss.hip &
  done
  wait
else
  for n in $V; do
    echo "== $FLAG=$n"
    COPENERF_LIB=$R/tools/abl/lib_${FLAG}_$n.so ONLY="${ONLY:-x6}" timeout -k 10 120 python3 $R/tools/gemm_bench.py || exit 1
  done
fi
