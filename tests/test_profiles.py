"""The committed measurement record is self-consistent (CPU): every launch class of the
newest profiled bench line names (cn_linear_kernel_name / cn_wgrad_kernel_name: the
library's own tile choice) a kernel present in the rocprofv3 stats of the same run,
and the bench's HIP-event launch time of the dominant kernel agrees with rocprof's
(bench line and kernel stats come from the same profile round, tools/profile_round.sh), and
the line's roofline frac is the one its cited kernel stats give."""
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


def test_roofline_frac_follows_the_cited_kernel_stats():
    """bench.py reports roofline.frac from the committed rocprofv3 average duration of the dominant
    kernel (roofline.frac_source names the file): recomputed here from that file, within 1 %."""
    from bench import BF16_MFMA_PEAK_TFLOPS, HBM_PEAK_GBS, MODE_PEAK_TFLOPS  # noqa: F401
    checked = 0
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*bench*.json"))):
        with open(f) as fh:
            lines = [ln for ln in fh.read().strip().splitlines() if ln.startswith("{")]
        if not lines:
            continue
        line = json.loads(lines[-1])
        roof = line.get("roofline") or {}
        src = roof.get("frac_source", "")
        if not src.endswith("average duration"):
            continue
        path = os.path.join(ROOT, src.split(":")[0])
        with open(path) as fh:
            stats = {r["Name"]: r for r in csv.DictReader(fh)}
        avg_s = float(stats[roof["kernel"]]["AverageNs"]) * 1e-9
        flops = roof["algorithmic_gflop_per_launch"] * 1e9
        nbytes = roof["algorithmic_mb_per_launch"] * 1e6
        mode = {"bf16 MFMA dense": "bf16", "fp32 MFMA dense": "fp32"}.get(roof["peak_basis"].split(";")[0], "bf16x6")
        peak_tf = MODE_PEAK_TFLOPS[mode]
        frac = max(flops / (peak_tf * 1e12), nbytes / (HBM_PEAK_GBS * 1e9)) / avg_s
        assert abs(frac - roof["frac"]) <= 0.01 * roof["frac"], (f, frac, roof["frac"])
        checked += 1
    assert checked >= 1, "no committed bench line cites rocprofv3 stats for its roofline"


def test_cited_kernel_stats_were_recorded_for_the_reported_library():
    """A bench line (round 5 on) that takes its frac from committed kernel stats cites a CSV whose
    _lib_stamp.txt equals the library stamp the line reports."""
    from bench import stats_stamp
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*bench*.json"))):
        with open(f) as fh:
            lines = [ln for ln in fh.read().strip().splitlines() if ln.startswith("{")]
        if not lines:
            continue
        roof = json.loads(lines[-1]).get("roofline") or {}
        if "lib_stamp" not in roof or not roof.get("frac_source", "").endswith("average duration"):
            continue
        csv_path = os.path.join(ROOT, roof["frac_source"].split(":")[0])
        assert stats_stamp(csv_path) == roof["lib_stamp"], f


def test_bench_cites_stats_only_for_the_same_library_build(tmp_path, monkeypatch):
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r9a_kernel_stats.csv").write_text("Name,Calls,TotalDurationNs,AverageNs\nk,2,200,100\n")
    (prof / "r9a_lib_stamp.txt").write_text("aaaa\n")
    (prof / "r9b_kernel_stats.csv").write_text("Name,Calls,TotalDurationNs,AverageNs\nk,2,400,200\n")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.rocprof_launch_ns("k", "c2", "aaaa") == (100.0, os.path.join("profiles", "r9a_kernel_stats.csv"))
    assert bench.rocprof_launch_ns("k", "c2", "bbbb") == (None, None)  # r9b has no stamp, r9a another one
    assert bench.rocprof_launch_ns("k", "c2", None) == (None, None)
