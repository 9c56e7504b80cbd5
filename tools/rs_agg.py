"""Aggregate RS_STATS lines (k_match_resolve_spec walk statistics) from stdin."""
import sys
import numpy as np
rows = []
for ln in sys.stdin:
    p = ln.split()
    if len(p) >= 15 and p[0] == "RS":
        rows.append([int(p[i]) for i in (4, 6, 8, 10, 12, 14)])
a = np.array(rows)
if len(a):
    n = len(a)
    print(f"units {n}  n1 {a[:,0].mean():.0f} n2 {a[:,1].mean():.0f} feas {a[:,2].mean():.0f} "
          f"chunks {a[:,3].mean():.1f} rounds {a[:,4].mean():.1f} (max {a[:,4].max()}) hard {a[:,5].mean():.2f}")
