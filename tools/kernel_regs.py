#!/usr/bin/env python3
"""VGPR / spill / scratch of the split-K kernels in the built gfx950 assembly (build/rr_sk-*.s, -save-temps).
    python tools/kernel_regs.py [filter-prefix ...]   e.g. "8, 2, 16" for the headline int8 screen"""
import glob
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
f = glob.glob(os.path.join(HERE, "rag-serving-system_amd", "build", "rr_sk-hip-amdgcn-amd-amdhsa-gfx950.s"))[0]
txt = open(f).read()
items = re.findall(r"\.agpr_count:\s+(\d+).*?\.name:\s+(\S+).*?\.private_segment_fixed_size:\s+(\d+).*?"
                   r"\.vgpr_count:\s+(\d+)\s+\.vgpr_spill_count:\s+(\d+)", txt, re.S)
names = subprocess.run(["c++filt"], input="\n".join(i[1] for i in items), capture_output=True, text=True).stdout.split("\n")
for (agpr, _, priv, vg, sp), d in zip(items, names):
    m = re.search(r"sk_score_kernel<(.*)>\(", d)
    if not m:
        continue
    args = m.group(1)
    if len(sys.argv) > 1 and not any(args.startswith(p) for p in sys.argv[1:]):
        continue
    print(f"<{args}> vgpr {vg} agpr {agpr} spill {sp} scratch {priv}")
