#!/bin/bash
# Per-kernel register / LDS / scratch usage of libtmhpvsim's kernels (compile-only, CPU)
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I include -c \
  --cuda-device-only -Rpass-analysis=kernel-resource-usage tmhpvsim_amd/csrc/tmh_engine.hip -o /tmp/res.o "$@" 2>&1 |
python3 -c "
import re,sys,subprocess
cur=None; row={}
out=[]
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m:
        if cur: out.append((cur,row))
        cur=m.group(1); row={}; continue
    m=re.search(r'remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|TotalSGPRs|LDS Size \[bytes/block\]|VGPRs Spill|SGPRs Spill): (\d+)',l)
    if m and cur: row[m.group(1).split()[0]+('Spill' if 'Spill' in m.group(1) else '')]=m.group(2)
if cur: out.append((cur,row))
names=subprocess.run(['c++filt'],input='\n'.join(c for c,_ in out),capture_output=True,text=True).stdout.split('\n')
for (c,r),nm in zip(out,names):
    nm=nm.replace('(anonymous namespace)::','').split('(')[0]
    print(f'{nm[:44]:44s} ' + ' '.join(f'{k}={v}' for k,v in r.items()))
"
