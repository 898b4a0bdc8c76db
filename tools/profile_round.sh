#!/bin/bash
# Profile round on the GPU box: for each config, the rocprofv3 kernel-trace stats of a short bench
# run, then the untraced bench line (which reads those stats for its roofline frac), and for c2 the
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate --pmc passes).  Outputs in gpurun_out/prof_TAG/,
# named as profiles/ expects them: TAG_kernel_stats.csv / TAG_bench.json for c2,
# TAG_<config>_kernel_stats.csv / TAG_<config>_bench.json otherwise.
#   bash tools/profile_round.sh TAG [configs...]      (default: c2)
set -eo pipefail
TAG=${1:-cur}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${@:-c2}; do
  n=${TAG}_$c; [ $c = c2 ] && n=$TAG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks_$c -o run --output-format csv -- \
    python3 $R/bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $O/${n}_bench_trace.json
  cp $O/ks_$c/run_kernel_stats.csv $O/${n}_kernel_stats.csv
  # the library build the stats were taken on (bench.py cites stats only for the same build)
  cp $R/cope-nerf_amd/copenerf/libcopenerf.so.stamp $O/${n}_lib_stamp.txt
  # the untraced line reads the stats for its roofline: copy them where bench.py looks first
  cp $O/${n}_kernel_stats.csv $R/profiles/${n}_kernel_stats.csv
  cp $O/${n}_lib_stamp.txt $R/profiles/${n}_lib_stamp.txt
  if [ $c = c2 ]; then
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --timer-steps 1 > /dev/null
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --timer-steps 1 > /dev/null
    python3 $R/tools/pmc_summary.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/${n}_pmc.json
    cp $O/${n}_pmc.json $R/profiles/${n}_pmc.json
    timeout -k 10 300 python3 $R/bench.py > $O/${n}_bench.json
  else
    timeout -k 10 300 python3 $R/bench.py --config $c --no-cpu-baseline > $O/${n}_bench.json
  fi
  python3 -c "import json; d=json.load(open('$O/${n}_bench.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['launch_class'], r['frac'], r['frac_hip_events'])"
done
echo done
