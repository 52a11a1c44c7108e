#!/usr/bin/env python3
"""Fold rocprofv3 SQ counter passes (tools/gpu_pmc_sq.sh, tools/gpu_evidence_r04.sh) per
kernel name: totals, and the wave-cycle split WAIT_ANY (parked on waitcnt / barrier) /
WAIT_INST_ANY (issue stall) / ACTIVE_INST_ANY, per wave; with GRBM_GUI_ACTIVE also the mean
resident waves per CU (SQ_WAVE_CYCLES counts quad-cycles, MI355X_MICROARCH.md: waves =
4 * WAVE_CYCLES / (GUI_ACTIVE / 8 XCDs * 256 CUs)) and VALU-busy = ACTIVE_INST_VALU share of
the wave cycles.  usage: python tools/pmc_sq_report.py gpurun_out/pmcsq"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcsq"
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if not k.startswith("k_"):
        continue
    w = max(c.get("SQ_WAVES", 1), 1)
    wc = max(c.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"{k:12s} waves {w:9.0f}  per wave: VALU {c['SQ_INSTS_VALU'] / w:7.0f} SALU {c['SQ_INSTS_SALU'] / w:6.0f}"
          f" LDS {c['SQ_INSTS_LDS'] / w:6.0f} VMEM rd {c['SQ_INSTS_VMEM_RD'] / w:5.0f} wr {c['SQ_INSTS_VMEM_WR'] / w:5.0f}"
          f" SMEM {c['SQ_INSTS_SMEM'] / w:5.0f} | wave-cycles {wc / w:8.0f}: parked {c['SQ_WAIT_ANY'] / wc:5.1%}"
          f" issue-stall {c['SQ_WAIT_INST_ANY'] / wc:5.1%} active {c['SQ_ACTIVE_INST_ANY'] / wc:5.1%}"
          f" (VALU {c['SQ_ACTIVE_INST_VALU'] / wc:5.1%} LDS {c['SQ_ACTIVE_INST_LDS'] / wc:5.1%}) LDS-stall {c['SQ_WAIT_INST_LDS'] / wc:5.1%}"
          f" bank-conf {c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_ACTIVE_INST_LDS'], 1):5.2f}x"
          + (f" | waves/CU {4 * c['SQ_WAVE_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8 * 256):5.1f}"
             f" (of 32) over {c['GRBM_GUI_ACTIVE'] / 8 / 2.1e3:7.1f} us busy" if c.get("GRBM_GUI_ACTIVE") else ""))
