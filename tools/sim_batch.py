#!/usr/bin/env python3
"""Batch boundaries that the batch rule's token conditions alone force on a merge sequence (an upper
bound on batch sizes: the count rules are ignored).  usage: tools/sim_batch.py tests/golden/scale/train_C3.json.gz"""
import gzip,json,sys
d=json.load(gzip.open(sys.argv[1]))
M=[(bytes.fromhex(a),bytes.fromhex(b)) for a,b in d['merges']]
def sim(relaxed, cap=16):
    existing=set(bytes([i]) for i in range(256))
    i=0; trips=0; ends={}
    while i<len(M):
        L=set();R=set();T=set();new=set();k=0
        while i<len(M) and k<cap:
            a,b=M[i]
            if a==b and k>0: ends['a=b']=ends.get('a=b',0)+1; break
            if (a in new or b in new) and k>0: ends['fresh']=ends.get('fresh',0)+1; break
            if (a+b in existing or a+b in new) and k>0: ends['dup']=ends.get('dup',0)+1; break
            if k>0:
                if relaxed:
                    if a in R or b in L or a==b: ends['clash']=ends.get('clash',0)+1; break
                else:
                    if a in T or b in T: ends['clash']=ends.get('clash',0)+1; break
            L.add(a);R.add(b);T.add(a);T.add(b);new.add(a+b);k+=1;i+=1
            if a==b: break
        if k==cap: ends['cap']=ends.get('cap',0)+1
        existing|=new; trips+=1
    return trips, ends
for r in (False,True):
    for cap in (16,32):
        t,e=sim(r,cap); print('relaxed' if r else 'strict', cap, t, len(M)/t, e)
