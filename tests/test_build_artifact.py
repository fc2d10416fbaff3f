"""CPU checks of the shipped librhmc.so code object (gfx950): the hot leapfrog
kernels must not touch scratch memory (register spills turn the VALU-bound
loop into a memory-bound one — a one-step `hipcc -shared` build once did)."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import PKG_DIR

LLVM = "/opt/rocm/lib/llvm/bin"


def _disassemble(tmp_path):
    so = os.path.join(PKG_DIR, "librhmc.so")
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
    if not all(os.path.exists(t) for t in tools) or not os.path.exists(so):
        pytest.skip("ROCm llvm tools or librhmc.so not available")
    fat, co = str(tmp_path / "fat.bin"), str(tmp_path / "k.co")
    subprocess.run([tools[0], "--dump-section=.hip_fatbin=" + fat, so], check=True)
    subprocess.run([tools[1], "--unbundle", "--type=o", "--input=" + fat,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
    out = subprocess.run([tools[2], "-d", "--mcpu=gfx950", co], check=True,
                         capture_output=True, text=True).stdout
    funcs, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
        elif cur:
            funcs[cur].append(line)
    return funcs


def test_gfx950_code_object_present_and_hot_kernels_spill_free(tmp_path):
    funcs = _disassemble(tmp_path)
    leap = [f for f in funcs if "leapfrog" in f or "integrate_k1" in f]
    assert any("leapfrog_k1_tiledr" in f for f in leap)
    assert any("leapfrog_k1_tiledl" in f for f in leap)
    assert any("leapfrog_pk" in f for f in leap) and any("leapfrog_kr" in f for f in leap)
    assert sum("integrate_k1_tiledr" in f for f in leap) == 18   # 3 images x 2 DT x 3 solvers
    assert any("leapfrog_win_kernel" in f for f in leap)
    # superseded families are gone (round 3)
    assert not any("leapfrog_k1_tiled<" in f or "leapfrog_k1_tiled2" in f or
                   "leapfrog_k1_tiledw" in f or "leapfrog_tiledk_kernel" in f for f in funcs)
    for name in leap:
        if "win_kernel" in name:
            continue        # windowed kernel: a few scratch words from exp/pow (measured, small)
        n = sum("scratch_" in l for l in funcs[name])
        assert n == 0, "%s uses scratch (%d instructions)" % (name, n)
