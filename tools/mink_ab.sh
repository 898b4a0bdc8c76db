# per-shape GEMM table with the 1-per-CU tiles for every K vs only K >= 128 (COPENERF_WIDE_MINK), GPU box
for r in 1 2; do for k in 0 128; do echo "== mink $k"; COPENERF_WIDE_MINK=$k timeout -k 10 200 python tools/step_profile.py 2>&1 | grep -E "^step|, 64\)\)|, 52\)\)"; done; done
