#!/bin/bash
# one-lease in-process A/B of team-kernel variants at 6 and 8 members
# (tools/build_ab.sh builds them; tools/ab must not be gpurun-ignored)
set -e
mkdir -p gpurun_out/r05
for v in ${AB_VARIANTS:-g4 occ4 occ3 occ2}; do
  timeout -k 10 240 python3 -u tools/team_inproc_ab.py tools/ab/$v/libosgpu_reduce.so ${AB_P:-6,8} ${AB_TRIALS:-4} \
      > gpurun_out/r05/ab_$v.jsonl
  python3 - "$v" <<'P'
import json,sys,statistics as s
v=sys.argv[1]; rows=[json.loads(l) for l in open(f'gpurun_out/r05/ab_{v}.jsonl')]
for P in sorted({r['P'] for r in rows}):
    x=[r['b_over_a'] for r in rows if r['P']==P]; a=[r['a_of_copy'] for r in rows if r['P']==P]; b=[r['b_of_copy'] for r in rows if r['P']==P]
    print(v,P,'B/A mean %.3f min %.3f max %.3f | A/copy %.3f B/copy %.3f same %s'%(s.mean(x),min(x),max(x),s.median(a),s.median(b),all(r['same_result'] for r in rows)))
P
done
