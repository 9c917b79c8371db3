#!/bin/bash
# combine A/B at 5-8 inputs: shipped (register form above 4) vs LDS form U = 2 / 4.  Not product.
set -e
O=gpurun_out/r05; mkdir -p $O
AB_N=$((32<<20)) timeout -k 10 500 python tools/combine_inproc_ab.py tools/ab/clds8u2/libosgpu_reduce.so 5,8 4 > $O/cab_k8u2.jsonl
AB_N=$((32<<20)) timeout -k 10 500 python tools/combine_inproc_ab.py tools/ab/clds8u4/libosgpu_reduce.so 5,8 4 > $O/cab_k8u4.jsonl
