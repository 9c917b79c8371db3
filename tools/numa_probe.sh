#!/bin/bash
# in-process A/B at 5-8 members: shipped register form (U = 4, G = 2) vs U = 2 (G = 2, 1).  Not product.
set -e
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python tools/team_inproc_ab.py tools/ab/u8g2/libosgpu_reduce.so 5,8 6 > $O/ab_u8g2.jsonl
timeout -k 10 600 python tools/team_inproc_ab.py tools/ab/u8g1/libosgpu_reduce.so 5,8 6 > $O/ab_u8g1.jsonl
