"""Per-kernel table from a tools/pmc_round.sh round: time per step, effective clock
(GRBM_GUI_ACTIVE / 8 / duration), MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over
1024 SIMDs x GPU cycles), wait / issue-stall / active shares of wave cycles, and the
PMC HBM bytes per launch.  Usage: python tools/pmc_table.py gpurun_out/pmc_TAG [steps]"""
import csv
import json
import os
import re
import sys


def short(name):
    m = re.search(r"<([^>]*)>", name)
    return name.split("(")[0].split("<")[0].replace("void ", "") + (f"<{m.group(1)}>" if m else "")


def main(d, steps=None):
    sq = {}
    cur = None
    for l in open(os.path.join(d, "sq_summary.txt")):
        if l.strip() and not l.startswith(" "):
            cur = l.strip()
            sq[cur] = {}
        elif cur:
            m = re.match(r"\s+(\S+)\s+([\d.]+)", l)
            if m:
                sq[cur][m.group(1)] = float(m.group(2))
    stats = list(csv.DictReader(open(os.path.join(d, "ks", "run_kernel_stats.csv"))))
    pmc = json.load(open(os.path.join(d, "pmc.json")))["kernels"]
    bench = json.loads(open(os.path.join(d, "bench_trace.json")).read().strip().splitlines()[-1])
    steps = steps or (bench["steps"] + bench["warmup"] + 1)
    # algorithmic bytes per launch of each kernel symbol (bench.py's launch classes)
    alg = {}
    for cls, sym in bench.get("kernel_symbols", {}).items():
        c = bench.get("roofline_by_class", {}).get(cls, {})
        if "algorithmic_mb_per_launch" in c:
            alg[sym] = c["algorithmic_mb_per_launch"]
    rows = []
    for r in stats:
        k = short(r["Name"])
        b = sq.get(k)
        avg = float(r["AverageNs"])
        tot = float(r["TotalDurationNs"])
        row = {"kernel": r["Name"], "ms_per_step": tot / 1e6 / steps, "avg_us": avg / 1e3, "calls": int(r["Calls"])}
        if b and "GRBM_GUI_ACTIVE" in b:
            cyc = b["GRBM_GUI_ACTIVE"] / 8
            wc = b.get("SQ_WAVE_CYCLES", 0) or 1
            row.update({"clock_ghz": cyc / avg, "mfma_busy": b.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (cyc * 1024),
                        "wait": b.get("SQ_WAIT_ANY", 0) / wc, "issue_stall": b.get("SQ_WAIT_INST_ANY", 0) / wc,
                        "active": b.get("SQ_ACTIVE_INST_ANY", 0) / wc})
        p = pmc.get(r["Name"])
        if p:
            row["hbm_mb_per_launch"] = p["hbm_bytes_per_launch"] / 1e6
            if alg.get(r["Name"]):
                row["algorithmic_mb_per_launch"] = alg[r["Name"]]
                row["pmc_over_algorithmic"] = row["hbm_mb_per_launch"] / alg[r["Name"]]
                row["hbm_tbs"] = row["hbm_mb_per_launch"] / row["avg_us"]
        rows.append(row)
    rows.sort(key=lambda x: -x["ms_per_step"])
    out = ["| kernel | ms/step | avg µs | GHz | MFMA busy | wait | issue stall | PMC MB/launch | algorithmic MB | "
           "PMC / alg. | PMC TB/s |",
           "|---|---|---|---|---|---|---|---|---|---|---|"]
    for x in rows[:16]:
        f = lambda k, fmt: (fmt % x[k]) if k in x else "—"  # noqa: E731
        out.append(f"| `{short(x['kernel'])}` | {x['ms_per_step']:.2f} | {x['avg_us']:.1f} | {f('clock_ghz', '%.2f')} | "
                   f"{f('mfma_busy', '%.3f')} | {f('wait', '%.2f')} | {f('issue_stall', '%.2f')} | "
                   f"{f('hbm_mb_per_launch', '%.0f')} | {f('algorithmic_mb_per_launch', '%.0f')} | "
                   f"{f('pmc_over_algorithmic', '%.2f')} | {f('hbm_tbs', '%.2f')} |")
    print("\n".join(out))
    json.dump(rows, open(os.path.join(d, "kernel_table.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
