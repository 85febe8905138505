#!/usr/bin/env python3
"""Effective shader clock per kernel from a `rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT` pass
(MI355X_MICROARCH.md 'DVFS give-back': clock ~ GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time).
Usage: python tools/pmc_clock.py gpurun_out/pmc_clk/c_counter_collection.csv profiles/pmc_clock.json
"""
import collections
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    gui = collections.defaultdict(float)
    dur = collections.defaultdict(float)
    n = collections.Counter()
    seen = set()
    for r in rows:
        k = (r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
             .split("(")[0].replace("rbl::", ""))
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            gui[k] += float(r["Counter_Value"])
        if (r["Dispatch_Id"], k) not in seen:
            seen.add((r["Dispatch_Id"], k))
            dur[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            n[k] += 1
    out = {k: {"launches": n[k], "avg_us": round(dur[k] / n[k] / 1e3, 1),
               "clock_ghz": round(gui[k] / 8 / dur[k], 3)}
           for k in sorted(dur, key=lambda k: -dur[k]) if dur[k] > 0 and gui[k] > 0}
    res = {"method": "rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT over `bench.py --steps 1 --warmup 0 "
                     "--no-cpu-baseline --no-ttk`; clock = GRBM_GUI_ACTIVE / 8 / wall",
           "config": {"n": 10_000_000, "b": 32, "workload": "C4a"}, "kernels": out}
    txt = json.dumps(res, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
