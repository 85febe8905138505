#!/usr/bin/env python3
"""Summarise tools/pmc_traffic.sh output into per-kernel HBM bytes per launch.

FETCH_SIZE / WRITE_SIZE are in KB (1024 B).  The calibration probe (tools/pmc_calib.hip)
streams 2 GiB per kernel with 4 / 8 / 16 B per lane; its ratio bytes / counter is the
per-width correction (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of wide streaming reads on
gfx950).  Usage: python tools/pmc_summarize.py gpurun_out/pmc [out.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict

CAL_BYTES = 2 << 30


def load(path):
    rows = list(csv.DictReader(open(path)))
    per = defaultdict(list)
    for r in rows:
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return per


def short(name):
    s = name.replace("void ", "").split("(")[0]
    return s.replace("rbl::", "")


def main():
    d = sys.argv[1]
    out_path = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "-" else None
    # optional: the workload the passes ran (default C4a), e.g. "rmat 10000000 32 38" or
    # "circuit 1585478 16 75" (matrix, n, b, block steps per run)
    wl = sys.argv[3].split() if len(sys.argv) > 3 else ["hashwindow", "10000000", "32", "38"]
    matrix, wn, wb, wm = wl[0], int(wl[1]), int(wl[2]), int(wl[3])
    cf = load(os.path.join(d, "calib_fetch", "c_counter_collection.csv"))
    cw = load(os.path.join(d, "calib_write", "c_counter_collection.csv"))
    cal = {}
    for k, v in cf.items():
        if k.startswith("void k_read"):
            cal["fetch_" + k.split("<")[1].split(">")[0]] = CAL_BYTES / v[0]
    for k, v in cw.items():
        if k.startswith("void k_write"):
            cal["write_" + k.split("<")[1].split(">")[0]] = CAL_BYTES / v[0]
    f = load(os.path.join(d, "fetch", "b_counter_collection.csv"))
    w = load(os.path.join(d, "write", "b_counter_collection.csv"))
    kern = {}
    for k in sorted(set(f) | set(w), key=lambda k: -sum(f.get(k, [0])) - sum(w.get(k, [0]))):
        fv, wv = f.get(k, []), w.get(k, [])
        n = max(len(fv), len(wv))
        kern[short(k)] = {
            "launches": n,
            "fetch_raw_bytes_per_launch": sum(fv) / max(len(fv), 1),
            "write_raw_bytes_per_launch": sum(wv) / max(len(wv), 1),
        }
    fetch_corr = cal.get("fetch_double", 2.0)
    write_corr = cal.get("write_double", 1.0)
    for v in kern.values():
        v["hbm_bytes_per_launch"] = (v["fetch_raw_bytes_per_launch"] * fetch_corr +
                                     v["write_raw_bytes_per_launch"] * write_corr)
    spmm = {k: v for k, v in kern.items() if k.startswith("k_spmm")}
    tot_l = sum(v["launches"] for v in spmm.values())
    spmm_bytes = sum(v["hbm_bytes_per_launch"] * v["launches"] for v in spmm.values()) / max(tot_l, 1)
    # the partial-reorth pair: the Gram and the 64- (b = 32) or 32-column (b = 16) update
    upd = ("k_tsmm44<32, 64,", "k_tsmm44f") if wb == 32 else ("k_tsmm44<16, 32,",)
    reo = {k: v for k, v in kern.items() if k.startswith((f"k_gram44<{wb}, 2",) + upd)}
    # bench.py --steps 1 --warmup 0 runs the job once timed and (since round 6) once more with
    # the stage timers: count the runs by the Gram's launches (len(range(4, m + 1, 2)) per run)
    per_run = len(range(4, wm + 1, 2))
    gl = sum(v["launches"] for k, v in reo.items() if k.startswith(f"k_gram44<{wb}, 2"))
    runs = max(1, round(gl / per_run)) if per_run else 1
    reorth_bytes = sum(v["hbm_bytes_per_launch"] * v["launches"] for v in reo.values()) / runs
    # the kernels measured: the bench line of the FETCH pass names the fusions and the format
    extra = {}
    try:
        with open(os.path.join(d, "fetch.log")) as fh:
            j = json.loads([ln for ln in fh if ln.startswith('{"metric"')][0])
        extra = {"fuse": j["config"].get("fuse", 7),
                 "matrix_format": (j["roofline"].get("matrix_format")
                                   or j["roofline_secondary"].get("matrix_format"))}
    except (OSError, IndexError, KeyError, ValueError):
        pass
    name = {"hashwindow": "C4a (bench.py defaults)", "rmat": "C4b R-MAT (bench.py --matrix rmat)",
            "circuit": "C3 shape (bench.py --matrix circuit --n 1585478 --b 16)"}[matrix]
    res = {
        "config": {"n": wn, "b": wb, **({"matrix": matrix} if matrix != "hashwindow" else {}),
                   "workload": f"{name}, 1 run = {wm} steps", **extra},
        "calibration": cal,
        "correction_used": {"fetch": fetch_corr, "write": write_corr},
        "spmm_hbm_bytes_per_launch": spmm_bytes,
        "reorth_launches": {k: v["launches"] for k, v in reo.items()},
        "part_reorth_hbm_bytes_per_run": reorth_bytes,
        "kernels": kern,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                  "`bench.py --steps 1 --warmup 0`; KB x 1024 x per-width calibration factor "
                  "(tools/pmc_calib.hip, 2 GiB streams)",
    }
    txt = json.dumps(res, indent=1)
    if out_path:
        open(out_path, "w").write(txt + "\n")
    print(json.dumps(cal))
    for k, v in list(kern.items())[:12]:
        print(f"{k:40s} x{v['launches']:4d}  fetch {v['fetch_raw_bytes_per_launch']/1e9:8.3f} GB  "
              f"write {v['write_raw_bytes_per_launch']/1e9:8.3f} GB  hbm {v['hbm_bytes_per_launch']/1e9:8.3f} GB")
    print("spmm bytes/launch", spmm_bytes / 1e9, "part reorth bytes/run", reorth_bytes / 1e9)


if __name__ == "__main__":
    main()
