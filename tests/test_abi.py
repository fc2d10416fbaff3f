"""CPU-only checks of the C-ABI library: it loads, exports every symbol that
include/rhmc.h declares, and its structs match the header."""
import ctypes
import os
import re

from conftest import ROOT


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "rhmc.h")).read()
    return sorted(set(re.findall(r"\b(rhmc_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from rhmc_amd import capi
    declared = _header_functions()
    assert declared, "no declarations parsed"
    missing = [s for s in declared if not hasattr(capi.lib(), s)]
    assert not missing, missing
    assert sorted(capi.EXPORTS) == declared


def test_abi_version_and_params_layout():
    from rhmc_amd import capi
    assert capi.abi_version() == capi.ABI_VERSION == 4
    # 16 doubles + 4 int32 = 144 bytes, no padding
    assert ctypes.sizeof(capi.RhmcParams) == 16 * 8 + 4 * 4
    assert ctypes.sizeof(capi.MhSchedule) == 2 * 8 + 2 * 4


def test_device_count_without_gpu_is_safe():
    from rhmc_amd import capi
    assert capi.device_count() >= 0


def test_no_cpu_fallback_in_product_package():
    """The product package must never import the oracle (test infrastructure)."""
    pkg = os.path.join(ROOT, "hmc-stellar-toy-model_amd", "rhmc_amd")
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            src = open(os.path.join(pkg, fn)).read()
            assert "oracle" not in src.replace("oracle/", ""), fn
