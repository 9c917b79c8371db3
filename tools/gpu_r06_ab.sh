#!/bin/bash
# Round-6 in-process A/B of team-kernel variants (tools/ab/<name>, built by
# tools/build_ab.sh) against the shipped library, on the same allocations.
#   AB_VARIANTS="g2:2,3,4 g4:4" bash tools/gpu_r06_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in ${AB_VARIANTS}; do
  v=${spec%%:*}; ps=${spec#*:}
  echo "== $v P=$ps"
  timeout -k 10 ${AB_TIMEOUT:-240} python -u tools/${AB_TOOL:-team_inproc_ab.py} tools/ab/$v/libosgpu_reduce.so $ps ${AB_TRIALS:-4} \
      > gpurun_out/ab_$v.jsonl 2> gpurun_out/ab_$v.err
  rc=$?
  echo "== $v rc=$rc"; tail -3 gpurun_out/ab_$v.err
  if [ $rc -ne 0 ]; then exit $rc; fi
  python - gpurun_out/ab_$v.jsonl <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    r.setdefault("a_of_copy", r["a_frac"] / r["copy_frac"])
    r.setdefault("b_of_copy", r["b_frac"] / r["copy_frac"])
    r.setdefault("same_result", r.get("same_output"))
    by[r.get("P", r.get("K"))].append(r)
for P, rs in sorted(by.items()):
    med = lambda k: sorted(x[k] for x in rs)[len(rs) // 2]
    print(f"  P/K={P} n={len(rs)} a_frac={med('a_frac'):.3f} b_frac={med('b_frac'):.3f} "
          f"a_of_copy={med('a_of_copy'):.3f} b_of_copy={med('b_of_copy'):.3f} "
          f"b/a={med('b_over_a'):.3f} min_b/a={min(x['b_over_a'] for x in rs):.3f} "
          f"same={all(x['same_result'] for x in rs)}")
PY
done
echo "all variants done"
