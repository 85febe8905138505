#!/usr/bin/env python3
"""Per-kernel summary of tools/pmc_groups.sh output: python tools/pmc_groups_summary.py DIR [substr]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(d, "g*", "p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").split("(")[0].replace("rbl::", "")
        if sub in k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, a in agg.items():
    wc = a["SQ_WAVE_CYCLES"] or 1
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md 'DVFS give-back'):
    # per-XCD active cycles = sum / 8; 256 CUs / 1024 SIMDs on the chip
    gui = (a["GRBM_GUI_ACTIVE"] or 8) / 8.0
    print(f"== {k}")
    nonmfma = a["SQ_INSTS_VALU"] - a["SQ_INSTS_MFMA"]
    print("  non-MFMA VALU instructions per MFMA %.3f" % (nonmfma / (a["SQ_INSTS_MFMA"] or 1)))
    print("  per-CU-cycle: LDS busy %.3f  bank-conflict %.3f  MFMA busy/SIMD %.3f  CU busy %.3f" % (
        a["SQ_LDS_IDX_ACTIVE"] / (gui * 256), a["SQ_LDS_BANK_CONFLICT"] / (gui * 256),
        a["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * 1024), a["SQ_BUSY_CU_CYCLES"] / (gui * 256)))
    print("  per-wave-cycle: wait_any %.3f wait_inst_any %.3f active_any %.3f lds %.3f vmem %.3f valu %.3f wait_inst_lds %.3f" % (
        a["SQ_WAIT_ANY"] / wc, a["SQ_WAIT_INST_ANY"] / wc, a["SQ_ACTIVE_INST_ANY"] / wc,
        a["SQ_ACTIVE_INST_LDS"] / wc, a["SQ_ACTIVE_INST_VMEM"] / wc, a["SQ_ACTIVE_INST_VALU"] / wc,
        a["SQ_WAIT_INST_LDS"] / wc))
    print("  insts: lds_load %.3g lds_store %.3g mfma %.3g valu %.3g salu %.3g waves %.3g; lds fifo full data %.3g cmd %.3g unaligned %.3g addrconf %.3g" % (
        a["SQ_INSTS_LDS_LOAD"], a["SQ_INSTS_LDS_STORE"], a["SQ_INSTS_MFMA"], a["SQ_INSTS_VALU"],
        a["SQ_INSTS_SALU"], a["SQ_WAVES"], a["SQ_LDS_DATA_FIFO_FULL"], a["SQ_LDS_CMD_FIFO_FULL"],
        a["SQ_LDS_UNALIGNED_STALL"], a["SQ_LDS_ADDR_CONFLICT"]))
    print("  raw GRBM_GUI_ACTIVE %.4g  LDS_IDX_ACTIVE %.4g  MFMA_BUSY %.4g" % (gui, a["SQ_LDS_IDX_ACTIVE"], a["SQ_VALU_MFMA_BUSY_CYCLES"]))
    if a["FETCH_SIZE"] or a["WRITE_SIZE"]:
        # FETCH_SIZE in KB, x2 for 16-B-per-lane streaming reads on gfx950 (MI355X_MICROARCH.md HBM)
        hit = a["TCC_HIT_sum"] / max(1.0, a["TCC_HIT_sum"] + a["TCC_MISS_sum"])
        print("  memory side: FETCH %.4g GB (x2 calibrated)  WRITE %.4g GB  L2 hit %.3f" % (
            a["FETCH_SIZE"] * 2 * 1024 / 1e9, a["WRITE_SIZE"] * 1024 / 1e9, hit))
