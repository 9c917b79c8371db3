"""VALU / SALU / s_nop count of every basic block of a kernel's ISA with more
than 150 VALU instructions (a straight-line round of 7 soft adds), in
program order.  usage: count_rounds.py KERNEL.s"""
import re
import sys

blocks, cur = [], None
for line in open(sys.argv[1]).read().splitlines():
    t = line.strip()
    m = re.match(r'^(\.LBB\d+_\d+):', t)
    if m:
        if cur and cur[1] > 150:
            blocks.append(cur)
        cur = [m.group(1), 0, 0, 0]
        continue
    if cur is None:
        cur = ["entry", 0, 0, 0]
    if t.startswith('v_'):
        cur[1] += 1
    elif t.startswith('s_nop'):
        cur[3] += 1
    elif t.startswith('s_'):
        cur[2] += 1
if cur and cur[1] > 150:
    blocks.append(cur)
for b, v, s_, n in blocks:
    print(f"{b}: VALU {v} SALU {s_} nop {n}")
