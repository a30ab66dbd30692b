"""Instruction mix per kernel from a hipcc -save-temps device .s file (dev aid)."""
import re, sys
txt = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2] if len(sys.argv) > 2 else ''
cur = None; counts = {}
for l in txt:
    m = re.match(r'^(_Z\S+):\s*(;|$)', l)
    if m:
        cur = m.group(1); counts[cur] = dict(n=0, fma=0, mfma=0, barrier=0, ds=0, glob=0, scratch=0, branch=0); continue
    if cur and l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;'):
        c = counts[cur]; c['n'] += 1
        if 'v_fma_f64' in l: c['fma'] += 1
        if 'v_mfma' in l: c['mfma'] += 1
        if 's_barrier' in l: c['barrier'] += 1
        if '\tds_' in l: c['ds'] += 1
        if 'global_load' in l: c['glob'] += 1
        if 'scratch_' in l: c['scratch'] += 1
        if 's_cbranch' in l: c['branch'] += 1
    if l.startswith('.Lfunc_end'): cur = None
for k, v in counts.items():
    if pat in k: print(k[:60], v)
