#!/bin/bash
# The product library with its HOST code (runtime.cpp, heap.cpp,
# shmem_reduce.cpp, shmem_collect.cpp: barriers, heaps and their sockets, the
# VMM mappings, dispatch) built under UndefinedBehaviorSanitizer (gcc,
# aborting on the first report), linked with the tree's unchanged device
# objects, into tools/ubsan/libosgpu_reduce.so.  No device code is
# instrumented (GPU sanitizers are not available on the GPU pool).  Run the
# GPU suite against it:
#   OSGPU_LIB_PATH=$PWD/tools/ubsan/libosgpu_reduce.so \
#   UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 python -m pytest tests -m gpu
# (profiles/r03_ubsan_gpu_suite.txt).  Not part of the product.
set -e
cd "$(dirname "$0")/../test-resilient-osss-ucx_amd/csrc"
make -s -j8
out=../../tools/ubsan
mkdir -p $out
BID=$(cat $(ls *.hip *.cpp *.hpp | sort) ../../include/osgpu_reduce.h | sha256sum | cut -c1-16)
for f in runtime heap shmem_reduce shmem_collect; do
  g++ -O1 -g -std=c++17 -fPIC -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
      -fsanitize=undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer \
      -DOSGPU_BUILD_ID="\"$BID\"" -c $f.cpp -o $out/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libosgpu_reduce.so \
    combine.o team.o fused.o verify.o longdouble.o copy.o \
    $out/runtime.o $out/heap.o $out/shmem_reduce.o $out/shmem_collect.o \
    -lrccl -ldl -lpthread -lubsan
rm -f $out/*.o
ls -l $out/libosgpu_reduce.so
