#!/usr/bin/env python3
"""Instruction-class counts and resources of kernels in a hipcc -S assembly file.
usage: python3 tools/isa_stats.py file.s kernel [kernel ...]"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    for name in sys.argv[2:]:
        i = s.index(f"\n{name}:")
        j = s.find(".Lfunc_end", i)
        body = s[i:j]
        print(f"{name}: {body.count(chr(10))} lines")
        for pat in ["flat_load", "flat_store", "global_load", "global_store", "global_atomic", "ds_read", "ds_write",
                    "s_waitcnt vmcnt(0)", "scratch_", "buffer_", "s_barrier"]:
            print(f"  {pat:20s} {body.count(pat)}")
        k = s.find(f".name:           {name}\n")
        blk = s[s.rfind("- .args:", 0, k):k + 800]
        for key in [".vgpr_count", ".sgpr_count", ".group_segment_fixed_size", ".private_segment_fixed_size"]:
            pat = re.escape(key) + r":\s+(\d+)"
            print(f"  {key:30s} {re.findall(pat, blk)}")


if __name__ == "__main__":
    main()
