#!/usr/bin/env python3
"""Register / spill / LDS summary per kernel from a hipcc --save-temps .s
(AMDGPU metadata block). usage: kernel_regs.py file.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
md = s[s.rfind("amdhsa.kernels:"):]
for blk in re.split(r"\n  - \.", md)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or pat not in name.group(1):
        continue
    f = {k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
         for k in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                   "private_segment_fixed_size", "group_segment_fixed_size")}
    print(name.group(1), " ".join(f"{k}={v}" for k, v in f.items()))
