#!/bin/bash
# Build libosgpu_reduce variants into tools/ab/<name>/ for one-lease A/B runs
# (tools/ab is gpurun-ignored by default: the calling script lists it).
# Builds in a scratch copy of csrc/, so the in-tree library and objects are
# never touched (a GPU call may be snapshotting the tree meanwhile).
#   tools/build_ab.sh name "-DFLAG=1 -DOTHER=2" [name2 "flags2" ...]
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
W=$(mktemp -d /tmp/osgpu_ab.XXXXXX)
mkdir -p "$W/test-resilient-osss-ucx_amd" "$W/include"
cp -r "$ROOT/test-resilient-osss-ucx_amd/csrc" "$W/test-resilient-osss-ucx_amd/"
cp "$ROOT/include/osgpu_reduce.h" "$W/include/"
cd "$W/test-resilient-osss-ucx_amd/csrc"
make -s -j8
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math"
while [ $# -ge 2 ]; do
  name=$1; X=$2; shift 2
  d=$ROOT/tools/ab/$name; mkdir -p $d
  # AB_FILES: the sources the flags affect (default all four kernel files);
  # the others are linked from the scratch build unchanged
  for f in ${AB_FILES:-combine team fused longdouble}; do
    /opt/rocm/bin/hipcc $FL $X -c $f.hip -o $d/$f.o &
  done
  wait
  for f in combine team fused longdouble; do [ -f $d/$f.o ] || cp $f.o $d/$f.o; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libosgpu_reduce.so \
      $d/combine.o $d/team.o $d/fused.o verify.o $d/longdouble.o copy.o host_fold.o runtime.o heap.o \
      shmem_reduce.o shmem_collect.o -lrccl -ldl -lpthread
  rm -f $d/*.o
  echo "built tools/ab/$name"
done
rm -rf "$W"
