#!/usr/bin/env python
"""One-screen summary of a bench.py JSON line (scripts/session.sh bench)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print("c4" if d.get("config", {}).get("workload") == "c4" else d.get("config", {}).get("workload"),
      {k: d.get(k) for k in ("value", "ms_per_step", "dp_ms", "score_ms")}, "frac", r.get("frac"))
s = d.get("secondary")
if s:
    print("c5", {k: s.get(k) for k in ("value", "dp_ms", "score_ms")}, "frac", s.get("roofline", {}).get("frac"),
          "traffic", s.get("roofline", {}).get("traffic"))
e = d.get("e2e")
if e:
    print("e2e", {k: e.get(k) for k in ("clusters_per_s", "consensus_equals_template", "same_as_python_stage_machine")},
          "pinned", (e.get("pinned") or {}).get("ratio_to_unpinned"))
c3 = d.get("c3")
if c3:
    ps = c3.get("per_stage", {})
    print("c3", c3.get("native_seconds_per_run"), c3.get("same_as_python_stage_machine"),
          {k: round(v.get("dp_gcups", 0), 1) for k, v in ps.items()})
print("parity", d.get("parity"))
