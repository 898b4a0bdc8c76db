"""The committed measurement record is self-consistent (CPU): every launch class of the
newest profiled bench line names (cn_linear_kernel_name / cn_wgrad_kernel_name: the
library's own tile choice) a kernel present in the rocprofv3 stats of the same run,
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
    bench_f, stats_f = _newest_profiled_run()
    with open(bench_f) as fh:
        line = json.loads(fh.read().strip().splitlines()[-1])
    with open(stats_f) as fh:
        stats = {r["Name"]: r for r in csv.DictReader(fh)}
    symbols = line.get("kernel_symbols")
    if symbols is not None:  # bench lines from round 3 on carry the library-named symbol of each class
        assert symbols.keys() == line["kernel_breakdown_ms_per_step"].keys()
        for key, sym in symbols.items():
            assert sym in stats, (key, sym)
    roof = line["roofline"]
    assert roof["kernel"] in stats
    avg_us = float(stats[roof["kernel"]]["AverageNs"]) / 1e3
    assert abs(avg_us - roof["avg_launch_ms"] * 1e3) <= 0.05 * avg_us, (avg_us, roof["avg_launch_ms"])
