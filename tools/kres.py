#!/usr/bin/env python3
"""Per-kernel resources from a gfx950 .s (make asm): VGPRs, AGPRs, spills, LDS, SGPRs.
Usage: kres.py FILE.s [substring]"""
import re
import sys

txt = open(sys.argv[1]).read()
meta = txt[txt.find("amdhsa.kernels:"):]
match = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n  - ", meta)[1:]:
    kv = dict(re.findall(r"^\s*\.(\w+):\s+(\S+)", blk, re.M))
    name = kv.get("name", "?")
    if match in name:
        print(f"{kv.get('vgpr_count'):>4} vgpr {kv.get('agpr_count'):>3} agpr "
              f"{kv.get('vgpr_spill_count'):>3} spill {int(kv.get('group_segment_fixed_size', 0)):>7} lds "
              f"{kv.get('sgpr_count'):>4} sgpr  {name[:110]}")
