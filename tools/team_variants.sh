#!/bin/bash
# team-kernel variants (tools/build_variants.sh) against the shipped build,
# one box, interleaved: team_type_sweep.py for a few types at P = 4 and 8
mkdir -p gpurun_out
for rep in 1 2; do
for v in shipped ${TV_VARIANTS:-u4442 u4441 u4482 u4484 u4422}; do
  if [ $v = shipped ]; then lib=""; else lib=tools/variants/$v/libosgpu_reduce.so; fi
  OSGPU_LIB_PATH=$lib TT_TYPES=${TT_TYPES:-double,int,complexf} TT_PS=${TT_PS:-4,8} timeout -k 10 200 python -u tools/team_type_sweep.py > gpurun_out/tts_$v.log 2>&1 || exit 1
  sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" gpurun_out/team_type_sweep.jsonl >> gpurun_out/team_variants.jsonl
  rm gpurun_out/team_type_sweep.jsonl
done
done
