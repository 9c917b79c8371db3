#!/usr/bin/env python3
"""Tabulate every bench log's team placement trials by trial index and
member count: which trials collapsed (frac or copy
below 0.5 of the member count's median) and at which index.  Reads the
round-3..6 N=1 lines under profiles/ (the old key roofline_team_by_members
with `placements`, the round-6 key team_by_members with `trials`).
Not part of the product.
    python tools/placement_table.py > profiles/r06_placement_table.json"""
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def trials_of(line):
    by = line.get("team_by_members") or line.get("roofline_team_by_members") or {}
    for P, rec in by.items():
        if not isinstance(rec, dict):
            continue
        tr = rec.get("trials") or rec.get("placements") or []
        for i, t in enumerate(tr):
            yield P, i, t.get("frac"), t.get("copy_frac"), t.get("label")


rows = []
for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "r0[3-6]_bench*.log"))):
    try:
        lines = [json.loads(l) for l in open(p) if l.startswith("{")]
    except (OSError, ValueError):
        continue
    for line in lines[-1:]:
        got = list(trials_of(line))
        for P in sorted({g[0] for g in got}):
            fr = sorted(g[2] for g in got if g[0] == P and g[2] is not None)
            cp = sorted(g[3] for g in got if g[0] == P and g[3] is not None)
            if not fr:
                continue
            fm, cm = fr[len(fr) // 2], (cp[len(cp) // 2] if cp else None)
            for (q, i, f, c, lab) in got:
                if q != P:
                    continue
                rows.append({"log": os.path.basename(p), "members": int(P), "trial": i,
                             "frac": f, "copy_frac": c, "label": lab,
                             "collapse": bool((f is not None and f < 0.5 * fm) or
                                              (c is not None and cm and c < 0.5 * cm))})
summary = {}
for r in rows:
    k = f"trial{r['trial']}"
    s = summary.setdefault(k, {"trials": 0, "collapses": 0})
    s["trials"] += 1
    s["collapses"] += r["collapse"]
print(json.dumps({"by_trial_index": summary, "collapses": [r for r in rows if r["collapse"]],
                  "rows": len(rows)}, indent=1))
