"""LDS bank-conflict model of k_conv_i8's A-fragment reads (profiles/r5/conv/README.md).

ds_read_b128 serves a wave in four 16-lane groups ({0-3,12-15,20-27},
{4-11,16-19,28-31}, +32); a group costs as many cycles as the most lanes it
puts on one 16-byte (4-bank) quad of the 64-bank LDS.  Lane (m, g) of k-step
s reads chunk e = perm[s][g]: input row m + e // 3 (plane stride q quads),
column block e % 3 (+ the wave's block).  For each stride, searches every
partition of the 12 chunks into 3 ordered 4-tuples for the fewest cycles.

    python tools/lds_conflict_model.py 6 7 10 14
"""
from collections import Counter
import itertools, sys
groups=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
groups += [[l+32 for l in g] for g in groups]
def run(q):
    def tuple_cost(t):
        tot=0
        for r0 in (0,4,8,12):
          for wave in range(4):
            for gr in groups:
                c=Counter()
                for l in gr:
                    m=l&15; g=l>>4; e=t[g]
                    r=m+e//3+r0; col=e%3+wave
                    c[(r*q+col)%16]+=1
                tot+=max(c.values())
        return tot
    best_of={}
    for t in itertools.permutations(range(12),4):
        k=frozenset(t); c=tuple_cost(t)
        if k not in best_of or c<best_of[k][0]: best_of[k]=(c,t)
    best=(10**9,None)
    for a in itertools.combinations(range(1,12),3):
        s1=frozenset((0,)+a); rest=sorted(set(range(12))-s1)
        for b in itertools.combinations(rest[1:],3):
            s2=frozenset((rest[0],)+b); s3=frozenset(set(rest)-s2)
            c=best_of[s1][0]+best_of[s2][0]+best_of[s3][0]
            if c<best[0]: best=(c,(best_of[s1][1],best_of[s2][1],best_of[s3][1]))
    cur=tuple_cost((0,1,2,3))+tuple_cost((4,5,6,7))+tuple_cost((8,9,10,11))
    print(q*16, "best", best, "current-order", cur, "ideal", 3*4*4*4, flush=True)
for q in map(int, sys.argv[1:]): run(q)
