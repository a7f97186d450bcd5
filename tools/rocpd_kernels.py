"""Per-kernel median durations (and the gap before each k_tbatch_init) from a rocprofv3 rocpd database:
    python tools/rocpd_kernels.py gpurun_out/<call>/prof_d/run_results.db"""
import sqlite3, sys, numpy as np, collections
db=sqlite3.connect(sys.argv[1])
ks=db.execute("select start,end,name from kernels order by start").fetchall()
d=collections.defaultdict(list)
for s,e,n in ks: d[n[:50]].append(e-s)
for n,v in d.items(): print("%-50s n=%d med=%.0f" % (n, len(v), np.median(v)))
ev=sorted(ks)
gaps=[]
for i in range(1,len(ev)):
    if 'init' in ev[i][2]: gaps.append(ev[i][0]-ev[i-1][1])
print("gap before init median", np.median(gaps) if gaps else None)
