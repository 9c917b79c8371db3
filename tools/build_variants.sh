#!/bin/bash
# Build libosgpu_reduce variants with different per-lane unroll depths
# (OSGPU_U_K2/K4/K8) into tools/variants/ for tools/variant_sweep.py.
#   VARIANTS="421 442 444" tools/build_variants.sh   (digits: U for K<=2, K<=4, K<=8)
#   a fourth digit sets OSGPU_TEAM_G8 (team kernel above 4 PEs: vectors in
#   flight per input per round) and a fifth OSGPU_TEAM_U8 (vectors per input
#   per lane; default = the fourth digit), e.g. "44824"; G8 must divide U8
#   (team.hip static_assert)
set -e
cd "$(dirname "$0")/../test-resilient-osss-ucx_amd/csrc"
make -s -j8
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math"
TAGS=${VARIANTS:-"421 442 422 441 842"}
for t in $TAGS; do
  a=${t:0:1}; b=${t:1:1}; c=${t:2:1}; g=${t:3:1}; u=${t:4:1}
  u=${u:-$g}
  d=../../tools/variants/u$t; mkdir -p $d
  X="-DOSGPU_U_K2=$a -DOSGPU_U_K4=$b -DOSGPU_U_K8=$c ${g:+-DOSGPU_TEAM_G8=$g -DOSGPU_TEAM_U8=$u}"
  /opt/rocm/bin/hipcc $FL $X -c combine.hip -o $d/combine.o &
  /opt/rocm/bin/hipcc $FL $X -c team.hip -o $d/team.o &
done
wait
OTHERS="fused.o verify.o longdouble.o copy.o runtime.o heap.o shmem_reduce.o shmem_collect.o"
for t in $TAGS; do
  d=../../tools/variants/u$t
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libosgpu_reduce.so \
      $d/combine.o $d/team.o $OTHERS -lrccl -ldl -lpthread
done
ls ../../tools/variants/*/libosgpu_reduce.so
