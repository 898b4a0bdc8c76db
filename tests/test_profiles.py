"""The committed measurement record is self-consistent (CPU): every cn_linear launch
class of the newest profiled bench line names (through copenerf.ops' mirror of
cn_linear's tile choice) a kernel present in the rocprofv3 stats of the same run,
and the bench's HIP-event launch time of the dominant kernel agrees with rocprof's
(bench line and kernel stats come from the same profile round, tools/profile_round.sh)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]


def _newest_profiled_run():
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_bench.json")), reverse=True):
        stats = f.replace("_bench.json", "_kernel_stats.csv")
        if os.path.exists(stats):
            return f, stats
    raise AssertionError("no profiles/<tag>_bench.json with a matching _kernel_stats.csv")


def test_launch_classes_name_profiled_kernels():
    from copenerf import ops
    bench_f, stats_f = _newest_profiled_run()
    with open(bench_f) as fh:
        line = json.loads(fh.read().strip().splitlines()[-1])
    with open(stats_f) as fh:
        stats = {r["Name"]: r for r in csv.DictReader(fh)}
    classes = [tuple(k.split("/")) for k in line["kernel_breakdown_ms_per_step"] if k.startswith("linear/")]
    assert classes
    for key in classes:
        assert ops.linear_kernel_symbol(key) in stats, (key, ops.linear_kernel_symbol(key))
    roof = line["roofline"]
    avg_us = float(stats[roof["kernel"]]["AverageNs"]) / 1e3
    assert abs(avg_us - roof["avg_launch_ms"] * 1e3) <= 0.05 * avg_us, (avg_us, roof["avg_launch_ms"])
