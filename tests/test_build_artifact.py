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
    fat = str(tmp_path / "fat.bin")
    subprocess.run([tools[0], "--dump-section=.hip_fatbin=" + fat, so], check=True)
    # one offload bundle per translation unit (csrc/rhmc_kernels.hip and
    # csrc/rhmc_dense_ilp.hip), concatenated by the linker
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    assert starts, "no offload bundle in .hip_fatbin"
    funcs = {}
    for i, st in enumerate(starts):
        part, co = str(tmp_path / ("b%d.bin" % i)), str(tmp_path / ("k%d.co" % i))
        open(part, "wb").write(data[st:starts[i + 1] if i + 1 < len(starts) else len(data)])
        subprocess.run([tools[1], "--unbundle", "--type=o", "--input=" + part,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
        out = subprocess.run([tools[2], "-d", "--mcpu=gfx950", co], check=True,
                             capture_output=True, text=True).stdout
        cur = None
        for line in out.splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
            if m:
                cur = m.group(1)
                assert cur not in funcs, "kernel in two code objects: " + cur
                funcs[cur] = []
            elif cur:
                funcs[cur].append(line)
    return funcs


# Scratch budgets: every kernel of the library gets 0 scratch instructions
# except these (pattern on the demangled name -> the most allowed, and where
# they sit).  Counted in the gfx950 code object (static instructions).
SCRATCH_BUDGET = [
    # the fused multi-star MH iteration (C3's MH, K <= 10): kernel arguments
    # spilled in the prologue and reloaded in the momentum-draw block before
    # the step loop — 6 stores + 4 loads per lane per launch (one launch = one
    # MH iteration of n_steps leapfrog steps), none inside the step loop
    (r"mh_pk_iter<", 10),
    # one-wave-per-chain windowed kernels (WinG, any image; the K > 64
    # fallback off 32/48-px images): a few words around exp / pow
    (r"_win_kernel<rhmc::WinG, \d+(, \d+)?>", 11),
    # four register slots (K 129 - 256) of the dense kernel on 32/48-px
    # images: the fourth slot's state does not fit (BASELINE's configs and the
    # reference's drivers, K <= 120, use slots 1 - 2, which are scratch-free)
    (r"(leapfrog|energy|gradient|hmc_random)_win_kernel<rhmc::DenseG<\d+>, 4>", 43),
    (r"integrate_win_kernel<rhmc::DenseG<\d+>, \d, 4>", 54),
    # K > 256 (8 / 16 register slots, factor tables in global memory): the
    # completeness path past LDS-sized tables; 8 or 16 stars' state per lane
    # does not fit the register file and spills (no BASELINE config or
    # reference driver runs it: the reference's drivers stop at 120 stars)
    (r"_win_kernel<rhmc::WinGG, (\d, )?(2|4|8|16)>", 1300),
]


def _demangle(names):
    filt = shutil.which("c++filt")
    if not filt:
        pytest.skip("c++filt not available")
    out = subprocess.run([filt], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.splitlines()
    return dict(zip(names, out))


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
    dem = _demangle(list(funcs))
    used = set()
    for name, body in funcs.items():
        n = sum("scratch_" in l for l in body)
        d = dem[name]
        allowed = 0
        for i, (pat, cap) in enumerate(SCRATCH_BUDGET):
            if re.search(pat, d):
                allowed = cap
                used.add(i)
                break
        assert n <= allowed, "%s uses scratch (%d instructions, budget %d)" % (d, n, allowed)
    # every budget entry still names kernels of the library
    assert used == set(range(len(SCRATCH_BUDGET))), used


def test_production_kernels_scratch_free(tmp_path):
    """The kernels BASELINE's configurations and the reference's own drivers
    run are all scratch-free: the one-star register-window / lane-group /
    fused-MH kernels, the pixel-major and multi-star register-window
    kernels, the dense kernel's slots 1 - 2 (K <= 128), the energies and
    the MH begin / end kernels."""
    funcs = _disassemble(tmp_path)
    dem = _demangle(list(funcs))
    must = [r"leapfrog_k1_tiledr<", r"leapfrog_k1_tiledl<", r"mh_k1_tiledr<", r"energy_k1_tiledr<",
            r"leapfrog_pk<", r"leapfrog_kr<", r"_win_kernel<rhmc::DenseG<\d+>, [12]>",
            r"integrate_win_kernel<rhmc::DenseG<\d+>, \d, [12]>", r"mh_begin", r"mh_end",
            r"energy_win_kernel<rhmc::WinEG"]
    for pat in must:
        hits = [n for n in funcs if re.search(pat, dem[n])]
        assert hits, pat
        for n in hits:
            k = sum("scratch_" in l for l in funcs[n])
            assert k == 0, "%s: %d scratch instructions" % (dem[n], k)
