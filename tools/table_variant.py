#!/usr/bin/env python3
"""Write a copy of the committed tile table with some entries replaced (step-level A/B of tile
choices inside the graph). Diagnostics only.

    python tools/table_variant.py OUT.json RULE [RULE ...]
    RULE = n,h,cin,cout,k,res_q=cfg   (a field '*' matches anything)"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd", "smpq", "data", "tiles_gfx950.json")
doc = json.load(open(SRC))
changed = 0
for rule in sys.argv[2:]:
    pat, cfg = rule.split("=")
    pat = pat.split(",")
    for key in doc["tiles"]:
        f = key.split("|")
        if f[0] == "stem_s2d":
            continue
        fields = [f[0], f[1], f[3], f[4], f[5], f[14]]
        if all(p == "*" or p == v for p, v in zip(pat, fields)):
            doc["tiles"][key] = int(cfg)
            changed += 1
json.dump(doc, open(sys.argv[1], "w"), indent=1)
print("%s: %d entries changed" % (sys.argv[1], changed))
