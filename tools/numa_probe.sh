#!/bin/bash
# in-process A/B at 2 members: shipped (register form) vs the LDS form with U = 2, types and ops.  Not product.
set -e
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python tools/team_inproc_ab.py tools/ab/lds2u2/libosgpu_reduce.so 2 10 > $O/ab_lds2u2_b2.jsonl
AB_CASES="float:sum,float:prod,double:max,int:sum,long:xor,short:min,complexf:prod,complexd:sum,complexd:prod" timeout -k 10 600 python tools/team_inproc_ab.py tools/ab/lds2u2/libosgpu_reduce.so 2 3 > $O/ab_lds2u2_types.jsonl
