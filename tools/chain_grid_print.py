#!/usr/bin/env python3
"""Print the band rescoring's timeline per CBV2_OPT_RESCORE_GRID from chain_lab.py lines."""
import json
import sys

for line in open(sys.argv[1]):
    d = json.loads(line)
    t = d["timeline_us_from_bmax_start"]
    print(d["grid"], d["p50_us"], t.get("band_rescore_select:first_wg_start"), t.get("band_rescore_select:last_wg_end"),
          t.get("band_rescore_select:select_start"), t.get("band_rescore_select:select_end"))
