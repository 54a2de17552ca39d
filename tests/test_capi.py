"""CPU: the C-ABI library builds for gfx950, loads, and exports every symbol include/bprmf.h
declares.  No compute call is made here (no GPU in the build container)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared():
    names = set()
    for h in ("bprmf.h", "ncf.h", "mf.h", "bprfm.h", "sgns.h"):
        with open(os.path.join(ROOT, "include", h)) as f:
            src = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
        names |= set(re.findall(r"\b((?:bprmf|ncf|mf|bprfm|sgns)_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_library_exports_every_declared_symbol(rl):
    lib = rl.build()
    L = ctypes.CDLL(lib)
    names = _declared()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python binding covers the same set
    assert set(names) == set(rl._lib.SIGNATURES), set(names) ^ set(rl._lib.SIGNATURES)


def test_library_is_gfx950_code_object(rl):
    lib = rl.build()
    with open(lib, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_no_gpu_fails_loudly(rl):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises((rl.BprmfError, ValueError, RuntimeError)):
        rl.BPRMF(10, 10, 8)


def test_config_layout_matches_header(rl):
    # int64,int64,int32,float,float,int32,int32,float,uint64,int32,int32,int32,int32[4]
    assert ctypes.sizeof(rl._lib.Config) == 8 + 8 + 4 + 4 + 4 + 4 + 4 + 4 + 8 + 4 + 4 + 4 + 16 + 4
    assert ctypes.sizeof(rl._lib.Stats) == 32
    # int64 x2, int32 x5, float x5, uint64 (offset 56), int32, int32[4] -> 84, padded to 88
    assert ctypes.sizeof(rl._lib.NcfConfig) == 88
    assert rl._lib.NcfConfig.seed.offset == 56
    # int64 x2, int32 x4, double[4] x2 (offset 32, 64), double x2 (lr_yj, reg_yj) -> 112
    from importlib import import_module
    mf = import_module("recommend-lib_amd.mf")
    assert ctypes.sizeof(mf.MfConfig) == 112 and mf.MfConfig.lr.offset == 32
    assert mf.MfConfig.lr_yj.offset == 96 and mf.MfConfig.reg_yj.offset == 104
    assert ctypes.sizeof(mf.MfStats) == 24


def test_config_offsets_match_the_c_header(rl, tmp_path):
    """Every bprmf_config / bprmf_stats field at the offset a C compiler gives it (include/bprmf.h
    compiled with gcc here), so a field added on one side only cannot go unnoticed."""
    import shutil
    import subprocess
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = [f for f, _ in rl._lib.Config._fields_]
    st = [f for f, _ in rl._lib.Stats._fields_]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "bprmf.h"', "int main(void) {",
             '  printf("config %zu\\n", sizeof(bprmf_config));', '  printf("stats %zu\\n", sizeof(bprmf_stats));']
    lines += [f'  printf("c.{f} %zu\\n", offsetof(bprmf_config, {f}));' for f in cfg]
    lines += [f'  printf("s.{f} %zu\\n", offsetof(bprmf_stats, {f}));' for f in st]
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)],
                   check=True, capture_output=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], check=True, capture_output=True,
                                                 text=True).stdout.splitlines())
    assert int(got["config"]) == ctypes.sizeof(rl._lib.Config)
    assert int(got["stats"]) == ctypes.sizeof(rl._lib.Stats)
    for f in cfg:
        assert int(got[f"c.{f}"]) == getattr(rl._lib.Config, f).offset, f
    for f in st:
        assert int(got[f"s.{f}"]) == getattr(rl._lib.Stats, f).offset, f
