"""Mean idle gap before each kernel (previous kernel's end -> this kernel's start) in a rocprofv3
kernel trace, over consecutive pairs on the trace's timeline.  Usage: gaps.py DIR [DIR ...]"""
import collections, csv, glob, gzip, os, sys

for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, '**', '*kernel_trace.csv*'), recursive=True)[0]
    op = gzip.open if f.endswith('.gz') else open
    rows = sorted(csv.DictReader(op(f, 'rt')), key=lambda r: int(r['Start_Timestamp']))
    gaps = collections.defaultdict(list)
    for a, b in zip(rows, rows[1:]):
        g = (int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1000
        if 0 <= g < 50:
            key = a['Kernel_Name'].split('(')[0].replace('void ', '')[-18:] + ' -> ' + b['Kernel_Name'].split('(')[0].replace('void ', '')[-18:]
            gaps[key].append(g)
    print(d)
    for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))[:8]:
        v.sort()
        print(f'   {k:42s} n={len(v):4d} median={v[len(v)//2]:6.2f} us')
