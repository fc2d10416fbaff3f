#!/usr/bin/env python3
"""Static instruction histogram of one kernel of the built librhmc.so (tools
only): the whole kernel and its largest loop (the step loop).
usage: python tools/isa_hist.py KERNEL_SUBSTRING [LIB]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
sub = sys.argv[1]
lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "..", "hmc-stellar-toy-model_amd", "librhmc.so")
with tempfile.TemporaryDirectory() as t:
    subprocess.run([LLVM + "/llvm-objcopy", "--dump-section=.hip_fatbin=%s/f" % t, lib], check=True)
    subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=%s/f" % t,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=%s/k" % t], check=True)
    asm = subprocess.run([LLVM + "/llvm-objdump", "-d", "--mcpu=gfx950", t + "/k"], check=True,
                         capture_output=True, text=True).stdout
cur, body = None, []
for l in asm.splitlines():
    m = re.match(r"^[0-9a-f]+ <(.*)>:", l)
    if m:
        if cur and sub in cur:
            break
        cur, body = m.group(1), []
        continue
    t = l.strip()
    m = re.search(r"//\s*([0-9A-F]+):", t)
    if t and m:
        body.append((int(m.group(1), 16), t.split("//")[0].strip()))
print(cur)
addr = {a: i for i, (a, _) in enumerate(body)}
loops = []
for i, (a, t) in enumerate(body):
    if t.startswith("s_cbranch") or t.startswith("s_branch"):
        off = int(t.split()[1])
        off = off - 65536 if off >= 32768 else off
        tgt = addr.get(a + 4 + 4 * off)
        if tgt is not None and tgt < i:
            loops.append((i - tgt, tgt, i))
big = max(loops)
for name, (lo, hi) in (("kernel", (0, len(body) - 1)), ("largest loop", (big[1], big[2]))):
    ins = [t.split()[0] for _, t in body[lo:hi + 1]]
    c = collections.Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print("%s: %d instructions, %d VALU, %d accvgpr, %d ds_, %d s_" % (
        name, len(ins), valu, sum(v for k, v in c.items() if "accvgpr" in k),
        sum(v for k, v in c.items() if k.startswith("ds_")),
        sum(v for k, v in c.items() if k.startswith("s_"))))
    if name == "largest loop":
        print("  " + ", ".join("%s %d" % kv for kv in c.most_common(24)))
