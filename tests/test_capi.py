"""The C-ABI library builds, loads without a GPU, exports every symbol include/wab.h declares,
and its ctypes mirrors have the C layout (no compute calls here: those are -m gpu)."""
import ctypes
import math
import os
import re
import subprocess

import pytest

from wab_gym_amd import _lib
from wab_gym_amd.options import WabConfig

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "wab.h")
HEADERS = [HEADER, os.path.join(REPO, "include", "wab_torus.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(wab2?_[a-z_]+)\s*\(", src))
    return sorted(names)


def test_header_declares_the_boundary():
    names = declared_functions()
    assert set(names) == set(_lib.EXPORTED), names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libwab_hip.so not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in declared_functions() if n not in syms]
    assert not missing, missing


def test_product_library_is_not_a_diagnostic_build():
    """csrc/wab_build_guard.h: the product build refuses the diagnostic macros, a diagnostic
    build must say so, and the product library does not export wab_diagnostic_build."""
    guard = os.path.join(REPO, "wab_gym_amd", "csrc", "wab_build_guard.h")

    def compiles(*defs):
        r = subprocess.run(["g++", "-fsyntax-only", "-x", "c++", "-include", guard, "-"] + list(defs),
                           input="int main() { return 0; }\n", capture_output=True, text=True)
        return r.returncode == 0

    assert compiles("-DWAB_PRODUCT_BUILD")
    for macro in ("WAB_STAMPS", "WAB2_STAMPS", "WAB_ROLL_FLOOR=1", "WAB_WIDE_ROLL_FLOOR=1",
                  "WAB2_ABLATE=2", "WAB_ONLY_WAVE=0"):
        assert not compiles("-DWAB_PRODUCT_BUILD", "-D" + macro), macro
        assert not compiles("-D" + macro), macro
        assert not compiles("-DWAB_PRODUCT_BUILD", "-DWAB_DIAGNOSTIC_BUILD", "-D" + macro), macro
        assert compiles("-DWAB_DIAGNOSTIC_BUILD", "-D" + macro), macro
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libwab_hip.so not built")
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert "wab_diagnostic_build" not in out


def test_library_loads_and_reports_abi():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libwab_hip.so not built")
    L = _lib.load()
    assert L.wab_abi_version() == _lib.ABI_VERSION
    cfg = WabConfig(gatherer_only=0, lookout_only=1)
    assert L.wab_num_actions(ctypes.addressof(cfg)) == 5
    cfg.lookout_only = 0
    assert L.wab_num_actions(ctypes.addressof(cfg)) == 6


def test_ctypes_layout_matches_c(tmp_path):
    prog = tmp_path / "layout.c"
    fields = [f for f, _ in WabConfig._fields_]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HEADER, "int main(void){",
             'printf("%zu\\n", sizeof(wab_config));']
    lines += ['printf("%%zu\\n", offsetof(wab_config, %s));' % f for f in fields]
    lines += ['printf("%zu %zu\\n", sizeof(wab_obs), sizeof(wab_counters));', "return 0;}"]
    prog.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(prog)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(WabConfig)
    for i, f in enumerate(fields):
        assert int(out[1 + i]) == getattr(WabConfig, f).offset, f
    assert int(out[-2]) == ctypes.sizeof(_lib.WabObs)
    assert int(out[-1]) == ctypes.sizeof(_lib.WabCounters)


# (bush_power, max_berries): the defaults, every golden / parity option set, and edge cases
THRESHOLD_CASES = [(100, 200), (60, 200), (20, 200), (400, 200), (20, 1), (2.5, 7), (1, 255),
                   (400, 50), (100, 255), (1, 1), (0.5, 3), (100, 0)]


@pytest.mark.parametrize("power,mx", THRESHOLD_CASES)
def test_c_bush_thresholds_equal_numpy_table(power, mx):
    """wab_bush_thresholds (C, libm) == options.bush_thresholds (the reference's numpy
    expression, wab_env.py:631-635): a C caller can build wab_config without Python."""
    import numpy as np

    from wab_gym_amd.options import bush_thresholds

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libwab_hip.so not built")
    L = _lib.load()
    out = np.zeros(max(mx, 1), np.uint64)
    assert L.wab_bush_thresholds(float(power), mx, out.ctypes.data) == 0
    c, ref = out[:mx].astype(np.int64), bush_thresholds(power, mx).astype(np.int64)
    # Equal, except where numpy's vectorised float64 pow (this numpy 2.2) is one ulp below
    # libm's pow at the last draw before the boundary: the C table then starts one draw (2^-53)
    # earlier.  The reference's pinned numpy 1.19 evaluates np.power with libm's pow, so there
    # the C table is the reference's; the default options (100, 200) agree exactly.
    for k in np.nonzero(c != ref)[0]:
        U = int(c[k])
        assert U == ref[k] - 1, (k, U, ref[k])
        u = U * 2.0 ** -53
        assert round(math.pow(u, power) * mx) >= k + 1 > np.round(np.power(np.array([u]), float(power))[0] * mx)
    assert np.count_nonzero(c != ref) <= 2
    if (power, mx) in ((100, 200), (60, 200), (400, 200), (2.5, 7), (1, 255)):
        assert np.array_equal(c, ref)


def test_c_bush_thresholds_rejects_bad_arguments():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libwab_hip.so not built")
    L = _lib.load()
    assert L.wab_bush_thresholds(100.0, 256, None) == -1
    assert L.wab_bush_thresholds(float("nan"), 10, None) == -1
    assert L.wab_bush_thresholds(100.0, 10, None) == -1


def test_torus_config_layout_matches_c(tmp_path):
    """wab_torus.h's wab2_config and wab2_counters against their ctypes mirrors."""
    from wab_gym_amd.torus_options import Wab2Config

    fields = [f for f, _ in Wab2Config._fields_]
    hdr = os.path.join(REPO, "include", "wab_torus.h")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % hdr, "int main(void){",
             'printf("%zu\\n", sizeof(wab2_config));']
    lines += ['printf("%%zu\\n", offsetof(wab2_config, %s));' % f for f in fields]
    lines += ['printf("%zu\\n", sizeof(wab2_counters));', "return 0;}"]
    prog = tmp_path / "layout2.c"
    prog.write_text("\n".join(lines))
    exe = tmp_path / "layout2"
    subprocess.run(["gcc", "-o", str(exe), str(prog)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(Wab2Config)
    for i, f in enumerate(fields):
        assert int(out[1 + i]) == getattr(Wab2Config, f).offset, f
    assert int(out[-1]) == ctypes.sizeof(_lib.Wab2Counters)


def test_torus_record_size_and_validation_on_host():
    """wab2_record_size is host-only: round_up(24 + 2N + NB, 16); invalid options -> -1."""
    from wab_gym_amd.torus_options import make_config, record_size

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libwab_hip.so not built")
    L = _lib.load()
    assert L.wab2_abi_version() == _lib.ABI2_VERSION
    for counts in ((1, 8, 16), (3, 4, 9), (2, 6, 10), (1, 3, 5), (8, 0, 24), (0, 0, 1)):
        cfg, _ = make_config(32, 32, *counts)
        assert L.wab2_record_size(ctypes.addressof(cfg)) == record_size(sum(counts), counts[2])
    assert record_size(25, 16) == 96
    cfg, _ = make_config(32, 32, 1, 8, 16)
    cfg.num_ostriches = 9
    assert L.wab2_record_size(ctypes.addressof(cfg)) == -1
    assert b"ostriches" in L.wab2_last_error()
    cfg.num_ostriches, cfg.width = 1, 128
    assert L.wab2_record_size(ctypes.addressof(cfg)) == -1
    cfg.width = 32
    for f in ("lookout_view_radius", "gatherer_view_radius", "wolf_view_radius"):
        setattr(cfg, f, (1 << 20) + 1)  # C callers get the host wrapper's cap too (int32 view math)
        assert L.wab2_record_size(ctypes.addressof(cfg)) == -1, f
        assert b"radii" in L.wab2_last_error()
        setattr(cfg, f, 1 << 20)
        assert L.wab2_record_size(ctypes.addressof(cfg)) == 96, f
