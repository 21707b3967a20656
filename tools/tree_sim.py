#!/usr/bin/env python3
"""Tree-schedule simulation of the leaf kernel over the C2 corpus (sampled
tiles): tasks and wave-compressions per level in a tile, now and with the
in-tile tree capped at level 4 for 17..128-chunk messages (their upper levels
merged by a finish kernel, one lane per message). Measurement aid for
DESIGN.md section 8."""
import sys, numpy as np
sys.path.insert(0,'/root/repo')
import bench
n=1000000
sizes, keys, _ = bench.files_of("c2", 0, n)
lens = bench.S.cas_msg_len(sizes).astype(np.int64)
C = np.maximum(1, (lens + 1023)//1024)
S = np.concatenate([[0], np.cumsum(C)[:-1]])
T=1024
def fl2(x): return int(x).bit_length()-1
def node_level(j, c, s, cap=99):
    if c <= 1: return 0
    a = (j & -j).bit_length()-1 if j else 63
    b = min(fl2(c-j), fl2(c-1))
    return min(a, b, fl2(T - s), cap)
import collections
ntiles = int((S[-1]+C[-1]+T-1)//T)
sample_tiles = range(0, ntiles, 97)   # sample
tot = collections.Counter(); waves = collections.Counter()
tot_cap = collections.Counter(); waves_cap = collections.Counter(); fin_parents = 0; fin_msgs=0
for t in sample_tiles:
    tb = t*T
    lo = np.searchsorted(S, tb, 'right')-1
    hi = np.searchsorted(S, tb+T, 'left')
    per = collections.Counter(); per_cap = collections.Counter()
    for m in range(max(lo,0), hi):
        s0, c = int(S[m]), int(C[m])
        capped = 16 < c <= 128
        for g in range(max(s0, tb), min(s0+c, tb+T)):
            j = g - s0; s = g - tb
            K = node_level(j, c, s)
            for k in range(1, K+1): per[k]+=1
            Kc = node_level(j, c, s, 4 if capped else 99)
            for k in range(1, Kc+1): per_cap[k]+=1
        if c > 1 and s0 >= tb and s0 + c <= tb + T:
            # spine: binary decomposition parts
            parts = bin(c).count('1')
            if c & (c-1) == 0:
                per[fl2(c)] += 1
                if not capped: per_cap[fl2(c)] += 1
            else:
                rem = c; part = rem & -rem; rem -= part
                while rem:
                    part = rem & -rem
                    per[fl2(part)+1] += 1
                    if not capped: per_cap[fl2(part)+1] += 1
                    rem -= part
            if capped:
                # finish: merge of capped nodes: (#nodes - 1) parents
                j=0; nn=0
                while j < c:
                    k = node_level(j, c, (s0+j)-tb, 4); j += 1<<k; nn+=1
                fin_parents += nn-1; fin_msgs += 1
    for k,v in per.items(): tot[k]+=v; waves[k]+= -(-v//64)
    for k,v in per_cap.items(): tot_cap[k]+=v; waves_cap[k]+= -(-v//64)
nt=len(sample_tiles)
print("per tile, current: tasks", {k: round(tot[k]/nt,1) for k in sorted(tot)}, "waves", {k: round(waves[k]/nt,2) for k in sorted(waves)})
print("per tile, capped : tasks", {k: round(tot_cap[k]/nt,1) for k in sorted(tot_cap)}, "waves", {k: round(waves_cap[k]/nt,2) for k in sorted(waves_cap)})
w_cur = sum(waves.values())/nt; w_cap = sum(waves_cap.values())/nt
print("tree wave-compressions per tile: current", round(w_cur,2), "capped", round(w_cap,2), "finish parents per tile", round(fin_parents/nt,1), "-> finish wave-compressions", round(fin_parents/nt/64,2))
leaf_wave_comp = 1024*16.4/64
print("leaf wave-compressions per tile ~", leaf_wave_comp, "saving frac", round((w_cur - w_cap - fin_parents/nt/64)/ (leaf_wave_comp + w_cur),4))
