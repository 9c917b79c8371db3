#!/bin/bash
# in-process A/B at 3-4 members: shipped (LDS form, U = 4) vs LDS U = 2, second box.  Not product.
set -e
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python tools/team_inproc_ab.py tools/ab/ldsu2/libosgpu_reduce.so 3,4 10 > $O/ab_ldsu2_b2.jsonl
