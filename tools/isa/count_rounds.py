import re,sys
# VALU / SALU per straight-line round: blocks that start at a "%Flow" label
# and end at the next s_cbranch, keeping those with > 200 VALU (a full round)
lines=open(sys.argv[1]).read().splitlines()
rounds=[];cur=None
for l in lines:
    if re.match(r'^\.LBB\d+_\d+:.*%Flow',l): cur=[0,0,0]; continue
    if cur is None: continue
    t=l.strip()
    if t.startswith('s_cbranch'):
        if cur[0]>150: rounds.append(cur)
        cur=None; continue
    if t.startswith('v_'): cur[0]+=1
    elif t.startswith('s_nop'): cur[2]+=1
    elif t.startswith('s_'): cur[1]+=1
print("rounds",len(rounds),"VALU per round",[r[0] for r in rounds],"SALU",[r[1] for r in rounds],"nop",[r[2] for r in rounds])
