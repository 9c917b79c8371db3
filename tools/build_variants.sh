#!/bin/bash
# Build libosgpu_reduce variants with different per-lane unroll depths
# (OSGPU_U_K2/K4/K8) into tools/variants/ for tools/variant_sweep.py.
set -e
cd "$(dirname "$0")/../test-resilient-osss-ucx_amd/csrc"
make -s -j8
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math"
for v in "4 2 1" "4 4 2" "4 2 2" "4 4 1" "8 4 2"; do
  set -- $v
  tag="u$1$2$3"; d=../../tools/variants/$tag; mkdir -p $d
  /opt/rocm/bin/hipcc $FL -DOSGPU_U_K2=$1 -DOSGPU_U_K4=$2 -DOSGPU_U_K8=$3 -c combine.hip -o $d/combine.o &
  /opt/rocm/bin/hipcc $FL -DOSGPU_U_K2=$1 -DOSGPU_U_K4=$2 -DOSGPU_U_K8=$3 -c team.hip -o $d/team.o &
done
wait
for v in "4 2 1" "4 4 2" "4 2 2" "4 4 1" "8 4 2"; do
  set -- $v; tag="u$1$2$3"; d=../../tools/variants/$tag
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libosgpu_reduce.so $d/combine.o $d/team.o longdouble.o shmem_reduce.o -lrccl -ldl -lpthread
done
ls ../../tools/variants/*/libosgpu_reduce.so
