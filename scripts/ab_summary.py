#!/usr/bin/env python
"""Summarise an r04_ab_c5.sh directory (bench --config c5 per setting and
round) into one JSON: scoring / DP ms, fractions, parity per setting.
usage: ab_summary.py DIR OUT_JSON LABEL1 LABEL2 ..."""
import glob
import json
import os
import sys

d, out, labels = sys.argv[1], sys.argv[2], sys.argv[3:]
res = {"source": d, "settings": {}}
for i, lab in enumerate(labels, 1):
    rows = []
    for f in sorted(glob.glob(os.path.join(d, f"c5_{i}_*.json"))):
        try:
            j = json.load(open(f))
        except ValueError:
            continue
        rows.append({"round": int(f.rsplit("_", 1)[1].split(".")[0]), "score_ms": j["score_ms"], "dp_ms": j["dp_ms"],
                     "score_frac_of_8tbs": j["roofline"]["frac"], "parity_bitexact": j["parity"]["bitexact"]})
    res["settings"][lab] = rows
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
