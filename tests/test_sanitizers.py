"""CPU: the host C/C++ under AddressSanitizer + UndefinedBehaviorSanitizer.

tests/sanitize/Makefile builds ASan + UBSan variants of the host ingestion of libbprmf_amd
(csrc/ingest.cpp + csrc/status.cpp: the restatement of util/data_loader.py:27-146,444-548) and of
the C oracles (oracle/bpr_cpu.c, oracle/mf_cpu.c), and of the host-only planning logic of the
handle and its sharded runner (csrc/host_plan.cpp, driven by tests/sanitize/host_plan_check.cpp).
This test runs the CPU suites that drive them
in a child pytest with libasan preloaded (Python itself is not instrumented), the ingestion loaded
from the sanitizer build (BPRMF_DIAG_LIB) and the oracles from theirs (BPRMF_ORACLE_LIB_DIR).
Any ASan report or UBSan finding aborts the child (-fno-sanitize-recover, halt_on_error), so the
test fails on the first one.  Leak checking is off: the interpreter's own allocations at exit are
not ours."""
import os
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = os.path.join(HERE, "sanitize")
OUT = os.path.join(SAN, "_build")
SUITES = ["tests/test_ingest.py", "tests/test_oracle.py", "tests/test_mf_oracle.py",
          "tests/test_svdpp_oracle.py"]


def _libasan():
    r = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if r.returncode == 0 and os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def san_build():
    if not shutil.which("gcc") or not shutil.which("g++") or not _libasan():
        pytest.skip("gcc with libasan is needed for the sanitizer build")
    r = subprocess.run(["make", "-s", "-C", SAN], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return OUT


def _env(out):
    env = dict(os.environ)
    pre = env.get("LD_PRELOAD", "")
    env["LD_PRELOAD"] = _libasan() + (":" + pre if pre else "")  # ASan's runtime goes first
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["BPRMF_DIAG_LIB"] = os.path.join(out, "libbprmf_host_asan.so")
    env["BPRMF_ORACLE_LIB_DIR"] = out
    env["OMP_NUM_THREADS"] = "4"
    return env


def test_sanitizer_build_is_instrumented(san_build):
    """The variants really carry ASan: their dynamic symbols reference the ASan runtime."""
    for name in ("libbprmf_host_asan.so", "liboracle_bpr.so", "liboracle_mf.so"):
        r = subprocess.run(["nm", "-D", os.path.join(san_build, name)], capture_output=True, text=True)
        assert "__asan_" in r.stdout, name
        assert "__ubsan_" in r.stdout, name


def test_host_plan_clean_under_asan_ubsan(san_build):
    """The handle's and the sharded runner's host-only planning code (csrc/host_plan.cpp: shard
    positive lists, runner geometry, exchange capacity, IPC blob comparison) under ASan + UBSan,
    every result checked against a restatement (tests/sanitize/host_plan_check.cpp)."""
    exe = os.path.join(san_build, "host_plan_check")
    r = subprocess.run(["nm", exe], capture_output=True, text=True)
    assert "__asan_" in r.stdout and "__ubsan_" in r.stdout
    r = subprocess.run([exe], env=_env(san_build), capture_output=True, text=True, timeout=600)
    log = r.stdout[-4000:] + r.stderr[-4000:]
    assert "AddressSanitizer" not in log and "runtime error:" not in log, log
    assert r.returncode == 0 and "host_plan_check: ok" in r.stdout, log


@pytest.mark.parametrize("suite", SUITES)
def test_cpu_suite_clean_under_asan_ubsan(san_build, suite):
    cmd = [sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider",
           "-o", "addopts=", suite]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(san_build), capture_output=True, text=True,
                       timeout=900)
    log = r.stdout[-6000:] + r.stderr[-6000:]
    assert "AddressSanitizer" not in log and "runtime error:" not in log, log
    assert r.returncode == 0, log
    assert " passed" in r.stdout, log
