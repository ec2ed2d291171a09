"""Host sanitizer runs (SURVEY.md §5 sanitizer row; GPU ASan is not available
on the pool, so the host code is what runs instrumented): the CPU tests that
exercise each native host library, re-run in a child process against its
AddressSanitizer + UBSan build with the matching runtime preloaded --
  * the oracle (gcc, oracle/build/liboracle_asan.so),
  * the CBOR slicer (gcc, lib/libouro_pack_asan.so: csrc/pack.cpp alone),
  * the kernels' lane routines compiled for the host with the bound tracker
    (clang via hipcc, lib/libouro_devhost_asan.so),
  * the product's host path -- host_path.hip, host_fast.h, the task pool --
    behind a test-only shim (clang via hipcc, lib/libouro_hostpath_asan.so).
Any sanitizer report fails the test (UBSan is built non-recoverable)."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ouroboros-network_amd")


def _gcc_asan():
    r = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def _clang_asan():
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


def _run(preload, env_extra, tests):
    env = dict(os.environ)
    env.update(env_extra)
    env["LD_PRELOAD"] = preload
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1"
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu",
                        "-p", "no:cacheprovider", *tests], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert " passed" in out, out[-2000:]  # not everything skipped
    return out


def _make(target_dir, target):
    subprocess.run(["make", "-s", "-C", target_dir, target], check=True, stdout=subprocess.DEVNULL)


@pytest.mark.skipif(_gcc_asan() is None, reason="gcc libasan not installed")
def test_oracle_under_asan_ubsan():
    _make(os.path.join(ROOT, "oracle"), "asan")
    _run(_gcc_asan(), {"OURO_ORACLE_LIB": os.path.join(ROOT, "oracle", "build", "liboracle_asan.so")},
         ["tests/test_oracle.py", "tests/test_nonce.py", "tests/test_leader.py",
          "tests/test_byron.py", "tests/test_shard.py"])


@pytest.mark.skipif(_gcc_asan() is None, reason="gcc libasan not installed")
def test_cbor_slicer_under_asan_ubsan():
    _make(PKG, "lib/libouro_pack_asan.so")
    _run(_gcc_asan(), {"OURO_PACK_LIB": os.path.join(PKG, "lib", "libouro_pack_asan.so")},
         ["tests/test_pack.py", "tests/test_pack_byron.py"])


@pytest.mark.skipif(_clang_asan() is None, reason="clang ASan runtime not in the ROCm llvm")
def test_lane_routines_under_asan_ubsan():
    _make(PKG, "lib/libouro_devhost_asan.so")  # prebuilt by __graft_entry__.build()
    _run(_clang_asan(), {"OURO_DEVHOST_LIB": os.path.join(PKG, "lib", "libouro_devhost_asan.so")},
         ["tests/test_devcode_host.py"])


@pytest.mark.skipif(_clang_asan() is None, reason="clang ASan runtime not in the ROCm llvm")
def test_host_path_under_asan_ubsan():
    _make(PKG, "lib/libouro_hostpath_asan.so")
    _run(_clang_asan(),
         {"OURO_HOSTPATH_ASAN_LIB": os.path.join(PKG, "lib", "libouro_hostpath_asan.so")},
         ["tests/test_hostpath_asan.py"])
