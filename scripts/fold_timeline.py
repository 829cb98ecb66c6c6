#!/usr/bin/env python3
"""Per-kernel timeline (durations and gaps) of the last two path-counter folds
in a rocprofv3 --kernel-trace CSV: fold_timeline.py p_kernel_trace.csv"""
import csv,sys,re
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
def nm(r):
    n=r['Kernel_Name']
    m=re.search(r'(k_\w+|__amd_\w+)',n)
    return m.group(1) if m else n[:30]
idx=[i for i,r in enumerate(rows) if nm(r) in ('k_fold_hist1','k_fold_p1')]
for i in idx[-2:]:
    seq=[];j=i
    while j<len(rows) and (('fold' in nm(rows[j])) or 'scan' in nm(rows[j]) or 'fill' in nm(rows[j])):
        seq.append(rows[j]); j+=1
    t0=int(seq[0]['Start_Timestamp']); prev=t0
    for r in seq:
        s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
        print(f"{nm(r):26s} gap {(s-prev)/1e3:7.1f} us  dur {(e-s)/1e3:8.1f} us")
        prev=e
    print(f"total {(prev-t0)/1e3:.1f} us\n")
