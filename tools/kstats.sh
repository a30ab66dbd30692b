#!/bin/bash
# Register/LDS/occupancy per kernel + instruction mix (dev aid).  Usage: tools/kstats.sh kernels.hip [name-filter]
SRC=$1; PAT=${2:-}
D=$(mktemp -d)
cd /root/repo/a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I/opt/rocm/include -I/root/repo/include -c $SRC -save-temps=obj -o $D/k.o -Rpass-analysis=kernel-resource-usage 2> $D/remarks.txt
python3 - "$D" "$PAT" <<'PY'
import re, sys, glob
D, pat = sys.argv[1], sys.argv[2]
cur = None; res = {}
for line in open(f"{D}/remarks.txt"):
    m = re.search(r'Function Name: (\S+)', line)
    if m: cur = m.group(1); res[cur] = {}; continue
    m = re.search(r'remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)', line)
    if m and cur: res[cur][m.group(1).strip()] = int(m.group(2))
s = glob.glob(f"{D}/*gfx950.s")[0]
txt = open(s).read().split('\n'); cur = None; mix = {}
for l in txt:
    m = re.match(r'^(_Z\S+):\s*(;|$)', l)
    if m: cur = m.group(1); mix[cur] = dict(n=0, fma=0, mfma=0, bar=0, ds=0, glob=0); continue
    if l.startswith('.Lfunc_end'): cur = None
    if cur and l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;'):
        c = mix[cur]; c['n'] += 1
        for k, t in (('fma', 'v_fma_f64'), ('mfma', 'v_mfma'), ('bar', 's_barrier'), ('ds', '\tds_'), ('glob', 'global_load')):
            if t in l: c[k] += 1
for k, v in res.items():
    if pat not in k: continue
    print(f"{k[:44]:44s} vgpr={v.get('VGPRs')} agpr={v.get('AGPRs')} occ={v.get('Occupancy')} lds={v.get('LDS Size')} spill={v.get('VGPRs Spill')} scratch={v.get('ScratchSize')} {mix.get(k, {})}")
PY
rm -rf $D
