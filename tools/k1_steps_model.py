"""K1 step-chain model (tools only): replays the step chains of k_dec_parse4/6 (a control word,
or a literal run plus the match that ends it plus a second match whose first byte is in the same
dword) over 64 oracle-compressed 16 KiB text blocks, and counts the wave's step iterations
(1) with every lane in the same 32-B round, looping until its slowest lane is done (round 4),
and (2) with per-lane rings and a budget of K steps per iteration (round 5).
usage: python tools/k1_steps_model.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O
def tlen(b):
    ty=(b&3)+(1 if (b&127)==3 else 0)
    return ((0x32110>>(4*ty))&15)
def steps_of(c):
    hdr = 9 if c[0]&2 else 3
    csize=len(c); ip=hdr; cwr=1; out=[]
    while True:
        gb = cwr==1
        rem=csize-ip
        run=(cwr & -cwr).bit_length()-1
        run=min(run,rem)
        q=ip+run; rest=cwr>>run
        hasm = (not gb) and rest!=1 and (rest&1) and q<csize
        end = ip + (4 if gb else 1) > csize
        if end: break
        need = q + (4 if gb else 1)
        if gb:
            cw=int.from_bytes(c[ip:ip+4],'little'); out.append((need, ip+4)); ip+=4; cwr=cw; continue
        e=tlen(c[q]) if hasm else 0
        w_has2 = hasm and e<3 and ((rest>>1)&1) and (rest>>1)!=1 and q+e+1<csize
        ncwr = rest >> (2 if w_has2 else (1 if hasm else 0))
        nip = q + (e+1 if hasm else 0)
        if w_has2:
            e2=tlen(c[q+e+1]); nip += e2+1
        out.append((max(need, q+e+2 if w_has2 else need), nip))
        if not hasm and rest==1:  # group exhausted by literals
            ip=q; cwr=1; 
            continue
        ip=nip; cwr=ncwr
        if ip>=csize: break
    return out
blocks=[O.compress(O.gen_text(7,i,16384)) for i in range(64)]
seqs=[steps_of(c) for c in blocks]
print("steps per block", np.mean([len(s) for s in seqs]), "csize", np.mean([len(c) for c in blocks]))
def cur(seqs, R=32):
    pos=[0]*64; it=0; r=0
    while any(p<len(s) for p,s in zip(pos,seqs)):
        lim=(r+1)*R; mx=0
        for l,s in enumerate(seqs):
            k=0
            while pos[l]<len(s) and s[pos[l]][0]<=lim: pos[l]+=1; k+=1
            mx=max(mx,k)
        it+=mx+1; r+=1   # +1: the iteration that finds nothing landed (go=false)
    return it, r
print("current: step-iterations, rounds", cur(seqs))
def new(seqs, K, R=32, S=4):
    """round 5 (k_dec_parse6): per iteration a lane stores the rounds it loaded in the previous
    iteration, loads up to two more the ring has room for, then takes up to K steps; the wave
    pays the largest step count among its lanes in that iteration."""
    n = len(seqs)
    pos, ip = [0] * n, [0] * n
    rl, ri, pend = [0] * n, [0] * n, [0] * n
    wave_steps = iters = 0
    while any(p < len(s) for p, s in zip(pos, seqs)):
        iters += 1
        mx = 0
        for l, s in enumerate(seqs):
            rl[l] += pend[l]
            cap = ip[l] // R + S - 1
            k = 0
            while k < 2 and ri[l] + k <= cap:
                k += 1
            pend[l] = k
            ri[l] += k
            lim = rl[l] * R
            k = 0
            while k < K and pos[l] < len(s) and s[pos[l]][0] <= lim:
                ip[l] = s[pos[l]][1]
                pos[l] += 1
                k += 1
            mx = max(mx, k)
        wave_steps += max(mx, 1)
    return wave_steps, iters


for K in (6, 10, 16):
    print("K", K, "wave step iterations, iterations", new(seqs, K))
