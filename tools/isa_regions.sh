#!/bin/bash
# Instruction counts per step-loop region of a kernel (tools only): builds
# librhmc with -DRHMC_MARKS (s_setprio markers in rhmc_k1step.hpp) into
# /tmp/isa and splits the disassembly at the markers.  usage: isa_regions.sh NAME_SUBSTRING
cd /root/repo/hmc-stellar-toy-model_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -DRHMC_MARKS ${EXTRA:-} -c -o /tmp/isa/mark.o csrc/rhmc_kernels.hip 2>&1 | grep error
mkdir -p /tmp/isa; cd /tmp/isa
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=mark.o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=km.co 2>/dev/null || { /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o libmark.so mark.o; /opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=fatm.bin libmark.so; /opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=fatm.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=km.co; }
/opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 km.co > km.s
python3 - "$1" <<'PY'
import re,sys
from collections import Counter
funcs={};cur=None
for line in open('km.s'):
    m=re.match(r"^[0-9a-f]+ <(\S+)>:",line)
    if m: cur=m.group(1); funcs[cur]=[]; continue
    if cur and line.strip(): funcs[cur].append(line.split('//')[0].strip())
k=[k for k in funcs if sys.argv[1] in k][0]
v=funcs[k]
open('m.s','w').write('\n'.join(v))
seg='start'; counts={}
for l in v:
    op=l.split()[0] if l else ''
    if op=='s_setprio':
        seg=l; counts.setdefault(seg,Counter()); continue
    c=counts.setdefault(seg,Counter())
    for p,n in (('v_','valu'),('s_','salu'),('ds_','lds')):
        if op.startswith(p): c[n]+=1
    if op.startswith('s_cbranch') or op.startswith('s_branch'): c['br']+=1
for s,c in counts.items(): print(s, dict(c))
PY
