"""Block-split policy simulator: replays a JSON trace into 64-slot blocks (tombstones kept,
as in the tracker) and counts blocks under several cut-point policies.
Usage: python tools/blocksim.py friendsforever_flat sveltecomponent"""
import sys, gzip, json, random
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
import golden_data as G
def sim(txns, policy):
    blocks=[[]]  # each item: [visible]
    def find(p):  # block idx, slot of visible index p
        acc=0
        for bi,b in enumerate(blocks):
            v=sum(b)
            if acc+v>p:
                k=p-acc
                for si,x in enumerate(b):
                    if x:
                        if k==0: return bi,si
                        k-=1
            acc+=v
        raise Exception
    def insert(pos,n):
        if pos==0: bi,s=0,0
        else:
            bi,s=find(pos-1); s+=1
        for _ in range(n):
            b=blocks[bi]
            if len(b)==64:
                c = policy(s)
                nb=b[c:]; del b[c:]
                blocks.insert(bi+1,nb)
                if s>c or c==64: bi+=1; s-=c
            blocks[bi].insert(s,1); s+=1
    def delete(pos,n):
        for _ in range(n):
            bi,s=find(pos); blocks[bi][s]=0
    for t in txns:
        for p,d,ins in t['patches']:
            if d: delete(p,d)
            if ins: insert(p,len(ins))
    return len(blocks), sum(len(b) for b in blocks)
pols={'mid':lambda s:32,'cursor':lambda s:s,'cursor>=48':lambda s: s if s>=48 else 32,'clamp16':lambda s:min(max(s,16),48)}
for name in sys.argv[1:]:
    t=G.trace(name)
    for pn,pf in pols.items():
        nb,items=sim(t['txns'],pf)
        print(name,pn,nb,items, f"fill={items/nb:.1f}")
