"""The C-ABI library builds, loads without a GPU, exports every symbol include/wab.h declares,
and its ctypes mirrors have the C layout (no compute calls here: those are -m gpu)."""
import ctypes
import os
import re
import subprocess

import pytest

from wab_gym_amd import _lib
from wab_gym_amd.options import WabConfig

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "wab.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(wab_[a-z_]+)\s*\(", src)))


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
