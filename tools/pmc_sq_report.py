#!/usr/bin/env python3
"""Per-kernel SQ counter report from rocprofv3 --pmc passes (tools/gpu_evidence_r05.sh).

Every ratio is computed from the counters of ONE pass: each pass is a separate run of the
program, so counters of different passes never share a denominator.  The passes are laid out
so that each one carries the denominators its own ratios need (SQ_WAVES, SQ_WAVE_CYCLES and
GRBM_GUI_ACTIVE where waves per CU are reported), and bench.py runs with a fixed amount of
work per pass (--prime-steps) so that passes stay comparable side by side.

Per pass and kernel (counters summed over the kernel's dispatches of that pass):
  * instruction mix (pass with SQ_INSTS_*): instructions per wave, wave-cycles per wave;
  * cycle split (pass with SQ_WAIT_ANY): WAIT_ANY (parked on s_waitcnt / barrier) +
    WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY, each as a share of SQ_WAVE_CYCLES, and
    their sum (MI355X_MICROARCH.md: the three are disjoint and add up to WAVE_CYCLES, so the
    sum must read ~100 %); VALU / LDS active shares; LDS issue stall;
  * LDS (pass with SQ_LDS_IDX_ACTIVE): bank-conflict cycles as a share of LDS-array cycles;
  * waves per CU wherever GRBM_GUI_ACTIVE is in the pass: SQ_WAVE_CYCLES counts quad-cycles,
    GRBM_GUI_ACTIVE is summed over the 8 XCDs, so waves/CU = 4 * WAVE_CYCLES /
    (GUI_ACTIVE / 8 * 256).

usage: python tools/pmc_sq_report.py gpurun_out/pmcsq   (one sub-directory per pass)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load_pass(d):
    tot = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            # k_flow: a solo deep frame (key frame, one workgroup per CU) apart from the batched
            # launches (every resident slot): separate rows by grid size
            if k.startswith("k_flow") and r.get("Grid_Size"):
                k = f"k_flow[grid {int(r['Grid_Size']) // 256}]"
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return tot


def waves_per_cu(c):
    if not c.get("GRBM_GUI_ACTIVE") or "SQ_WAVE_CYCLES" not in c:
        return None
    return 4 * c["SQ_WAVE_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 256)


def report_pass(name, tot):
    lines = []
    kernels = sorted((k for k in tot if k.startswith("k_")), key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0))
    for k in kernels:
        c = tot[k]
        parts = []
        wc = c.get("SQ_WAVE_CYCLES")
        w = c.get("SQ_WAVES")
        if w and "SQ_INSTS_VALU" in c:
            parts.append(f"waves {w:9.0f} per wave: VALU {c['SQ_INSTS_VALU'] / w:7.0f} SALU {c.get('SQ_INSTS_SALU', 0) / w:6.0f}"
                         f" LDS {c.get('SQ_INSTS_LDS', 0) / w:6.0f} VMEM rd {c.get('SQ_INSTS_VMEM_RD', 0) / w:5.0f}"
                         f" wr {c.get('SQ_INSTS_VMEM_WR', 0) / w:5.0f} SMEM {c.get('SQ_INSTS_SMEM', 0) / w:5.0f}"
                         + (f" wave-cycles {4 * wc / w:8.0f}" if wc else ""))
        if wc and "SQ_WAIT_ANY" in c:
            pk, st, ac = c["SQ_WAIT_ANY"] / wc, c.get("SQ_WAIT_INST_ANY", 0) / wc, c.get("SQ_ACTIVE_INST_ANY", 0) / wc
            parts.append(f"parked {pk:5.1%} issue-stall {st:5.1%} active {ac:5.1%} (sum {pk + st + ac:6.1%};"
                         f" VALU {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:5.1%} LDS {c.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.1%}"
                         f" LDS-issue-stall {c.get('SQ_WAIT_INST_LDS', 0) / wc:5.1%})")
        if c.get("SQ_LDS_IDX_ACTIVE"):
            parts.append(f"LDS bank-conflict cycles {c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:5.1%} of LDS-array cycles"
                         + (f" ({c['SQ_LDS_IDX_ACTIVE'] / w:7.0f} LDS cycles per wave)" if w else ""))
        wpc = waves_per_cu(c)
        if wpc is not None:
            parts.append(f"waves/CU {wpc:5.1f} (of 32) over {c['GRBM_GUI_ACTIVE'] / 8 / 2.1e3:8.1f} us busy")
        if parts:
            lines.append(f"  {k:12s} " + " | ".join(parts))
    return [f"[{name}]"] + lines


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcsq"
    passes = sorted(p for p in glob.glob(os.path.join(d, "*")) if os.path.isdir(p))
    out = []
    for p in passes:
        tot = load_pass(p)
        if tot:
            out += report_pass(os.path.basename(p), tot)
    print("\n".join(out))


if __name__ == "__main__":
    main()
