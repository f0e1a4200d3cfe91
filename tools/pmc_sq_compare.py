#!/usr/bin/env python3
"""Developer script: wave-cycle ratios (wait, VALU) and SALU:VALU of the stripe kernels from the
SQ counter passes of tools/pmc_bench_sq.sh, for two recorded runs side by side."""
import csv, glob, statistics, re
from collections import defaultdict
def load(files):
    v=defaultdict(lambda: defaultdict(list))
    for f in files:
        acc=defaultdict(float); nm={}
        for r in csv.DictReader(open(f)):
            k=(r['Dispatch_Id'],r['Counter_Name']); acc[k]+=float(r['Counter_Value']); nm[r['Dispatch_Id']]=r['Kernel_Name']
        for (dsp,c),x in acc.items(): v[nm[dsp]][c].append(x)
    return v
def short(k):
    m=re.search(r'(rs_\w+<[^>]*>|rs_\w+)', k); return m.group(1) if m else None
for label, files in [('v14', glob.glob('profiles/r01/pmc_sq_v14/*.csv')), ('v17', glob.glob('profiles/r01/pmc_sq_v17/*.csv'))]:
    v=load(files)
    for k,c in sorted(v.items()):
        s=short(k)
        if not s or 'targets' in s: continue
        m={n:statistics.median(x) for n,x in c.items()}
        out=[label, s]
        if 'SQ_WAVE_CYCLES' in m: out+=['wait/wave %.2f'%(m['SQ_WAIT_ANY']/m['SQ_WAVE_CYCLES']), 'valu/wave %.2f'%(m['SQ_ACTIVE_INST_VALU']/m['SQ_WAVE_CYCLES'])]
        if 'SQ_INSTS_SALU' in m: out+=['SALU:VALU %.2f'%(m['SQ_INSTS_SALU']/m['SQ_INSTS_VALU']), 'VALU insts %.3g'%m['SQ_INSTS_VALU'], 'LDS bank conf %.3g'%m['SQ_LDS_BANK_CONFLICT']]
        print(*out)
