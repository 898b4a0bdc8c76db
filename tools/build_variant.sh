#!/bin/bash
# Build the library with extra hipcc flags into another path (for same-box A/Bs with COPENERF_LIB), then
# restore the default library.   bash tools/build_variant.sh OUT.so -DFLAG=1 ...
set -e
OUT=$1; shift
cd "$(dirname "$0")/.."
COPENERF_HIPCC_EXTRA="$*" python -c "import __graft_entry__ as g; g.build()"
cp cope-nerf_amd/copenerf/libcopenerf.so "$OUT"
cp cope-nerf_amd/copenerf/libcopenerf.so.stamp "$OUT.stamp"
python -c "import __graft_entry__ as g; g.build()"
