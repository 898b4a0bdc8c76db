"""Summarise rocprofv3 SQ counter passes per cn kernel (average over dispatches):
python tools/sq_summary.py gpurun_out/sq/p1_x6/p1_counter_collection.csv ..."""
import csv
import re
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if not name.startswith("void cn::") and not name.startswith("cn::"):
            continue
        m = re.search(r"<([^>]*)>", name)
        key = (name.split("(")[0].split("<")[0].replace("void ", "") + (f"<{m.group(1)}>" if m else ""))
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k)
    wc = avg.get("SQ_WAVE_CYCLES")
    for c in sorted(avg):
        extra = f"  ({avg[c] / wc:6.3f} of wave cycles)" if wc and c.startswith("SQ_") and c != "SQ_WAVE_CYCLES" and "INSTS" not in c else ""
        print(f"   {c:28s} {avg[c]:16.0f}{extra}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back): /8 = GPU cycles
        cyc = avg["GRBM_GUI_ACTIVE"] / 8
        print(f"   GPU cycles (GUI_ACTIVE / 8): {cyc:.0f}; MFMA busy fraction (busy / (cycles * 1024 SIMDs)): "
              f"{avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f}")
