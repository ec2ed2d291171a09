"""The C-ABI boundary (CPU-only): the product library loads, exports every
symbol include/*.h declares, and the Python mirror types every one of them.
No compute calls are made here; on a host without a GPU the library must
report an error -- never "valid".
"""
import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_verify.so")


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(ouro_[a-z0-9_]+)\s*\(", text):
            syms.add(m.group(1))
    return syms


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("ouro_ed25519_verify", "ouro_vrf03_verify", "ouro_vrf03_proof_to_hash",
              "ouro_sum6kes_verify", "ouro_ed25519_verify_batch", "ouro_vrf03_verify_batch",
              "ouro_sum6kes_verify_batch", "ouro_tpraos_verify_batch",
              "ouro_tpraos_verify_batch_device"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build the library first (__graft_entry__.build())"
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_mirror_types_every_symbol():
    from ouroboros_network_amd import _native

    assert set(_native.SIGNATURES) == declared_symbols()


def test_struct_layout_matches_header():
    """ouro_tpraos_batch field order/size as the C header declares it."""
    from ouroboros_network_amd import _native

    text = open(os.path.join(ROOT, "include", "ouro_verify.h")).read()
    body = text[text.index("typedef struct ouro_tpraos_batch"):text.index("} ouro_tpraos_batch;")]
    names = re.findall(r"\*?\s*\b([a-z_]+);", body)
    assert [f[0] for f in _native.TPraosBatch._fields_] == names
    assert ctypes.sizeof(_native.TPraosBatch) == 21 * 8


def test_struct_offsets_match_the_c_compiler(tmp_path):
    """Every member's offset as gcc lays out the C header = the ctypes mirror's
    (and the oracle's orc_tpraos_batch, which tests hand the same struct)."""
    import subprocess

    from ouroboros_network_amd import _native

    names = [f[0] for f in _native.TPraosBatch._fields_]
    src = tmp_path / "off.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "ouro_verify.h"\n'
        '#include "oracle.h"\nint main(void){\n'
        'printf("%zu %zu\\n", sizeof(ouro_tpraos_batch), sizeof(orc_tpraos_batch));\n'
        + "".join(f'printf("%zu %zu\\n", offsetof(ouro_tpraos_batch, {n}), '
                  f'offsetof(orc_tpraos_batch, {n}));\n' for n in names)
        + "return 0;}\n")
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
                    str(src), "-o", str(exe)], check=True)
    rows = [tuple(map(int, ln.split())) for ln in
            subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
            if ln]
    assert rows[0] == (ctypes.sizeof(_native.TPraosBatch),) * 2
    for (name, _), (c_off, orc_off) in zip(_native.TPraosBatch._fields_, rows[1:]):
        assert getattr(_native.TPraosBatch, name).offset == c_off == orc_off, name


def test_byron_batch_offsets_match_the_c_compiler(tmp_path):
    """ouro_byron_batch as gcc lays it out = the ctypes mirror."""
    import subprocess

    from ouroboros_network_amd import _native

    names = [f[0] for f in _native.ByronBatch._fields_]
    src = tmp_path / "boff.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "ouro_verify.h"\nint main(void){\n'
        'printf("%zu\\n", sizeof(ouro_byron_batch));\n'
        + "".join(f'printf("%zu\\n", offsetof(ouro_byron_batch, {n}));\n' for n in names)
        + "return 0;}\n")
    exe = tmp_path / "boff"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    rows = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True,
                                            text=True).stdout.split()]
    assert rows[0] == ctypes.sizeof(_native.ByronBatch) == 9 * 8
    for (name, _), off in zip(_native.ByronBatch._fields_, rows[1:]):
        assert getattr(_native.ByronBatch, name).offset == off, name


SHIM = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_vrf_shim.so")
SODIUM_SHIM = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_sodium_shim.so")


def test_vrf_names_only_in_the_opt_in_shim():
    """crypto_vrf_ietfdraft03_{verify,proof_to_hash} and crypto_vrf_{verify,
    proof_to_hash} -- the cardano-crypto-praos names PraosVRF binds -- come
    from the separate lib/libouro_vrf_shim.so a maintainer links on purpose
    (INTEGRATION.md §1), never from the product library, so linking the
    product cannot take over the fork's symbols by accident."""
    import subprocess

    from ouroboros_network_amd import _native

    syms = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True,
                          text=True).stdout
    shim = subprocess.run(["nm", "-D", "--defined-only", SHIM], check=True, capture_output=True,
                          text=True).stdout
    for name in _native.VRF_ALIASES:
        assert f" {name}\n" not in syms, name
        assert f" T {name}\n" in shim, name
    text = open(os.path.join(ROOT, "include", "ouro_verify.h")).read()
    for name in _native.VRF_ALIASES:
        assert name in text
    # libsodium's Ed25519 verify: only from its own opt-in shim
    sod = subprocess.run(["nm", "-D", "--defined-only", SODIUM_SHIM], check=True,
                         capture_output=True, text=True).stdout
    assert " crypto_sign_ed25519_verify_detached\n" not in syms
    assert " T crypto_sign_ed25519_verify_detached\n" in sod
    assert "crypto_sign_ed25519_verify_detached" in text


_SHIM_CALL = """
import ctypes, sys
ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL)
shim = ctypes.CDLL(sys.argv[2])
out = ctypes.create_string_buffer(64)
if sys.argv[3] == "vrf":
    print(shim.crypto_vrf_ietfdraft03_verify(out, bytes(32), bytes(80), b"x", 1), flush=True)
else:
    print(shim.crypto_sign_ed25519_verify_detached(bytes(64), b"x", 1, bytes(32)), flush=True)
"""


@pytest.mark.parametrize("which", ["vrf", "sodium"])
@pytest.mark.parametrize("mode", ["default", "invalid"])
def test_shim_never_reports_a_device_error_as_an_invalid_proof(mode, which):
    """PraosVRF reads any nonzero as 'invalid proof'.  With no device the
    product's GPU route returns an error code; the shim must abort (default)
    rather than pass it on, or return -1 only when OURO_SHIM_ON_ERROR=invalid
    says so.  (Single items run on the host path by default since round 4;
    OURO_SINGLE_ITEM=gpu sends them to the -- here absent -- device.)"""
    import subprocess
    import sys

    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    env = dict(os.environ)
    env.pop("OURO_SHIM_ON_ERROR", None)
    env["OURO_SINGLE_ITEM"] = "gpu"
    if mode == "invalid":
        env["OURO_SHIM_ON_ERROR"] = "invalid"
    r = subprocess.run([sys.executable, "-c", _SHIM_CALL, LIB,
                        SHIM if which == "vrf" else SODIUM_SHIM, which],
                       capture_output=True, text=True, env=env, timeout=120)
    if mode == "default":
        assert r.returncode == -6, (r.returncode, r.stdout, r.stderr)  # SIGABRT
        assert "aborting rather than reporting a valid proof as invalid" in r.stderr
    else:
        assert r.returncode == 0 and r.stdout.strip() == "-1", (r.stdout, r.stderr)


def test_no_device_is_an_error_not_an_accept():
    """A batch call with no device returns OURO_ENODEV -- not a device error,
    so nothing is recomputed on the host path behind the caller's back -- and
    leaves the verdicts untouched."""
    import numpy as np
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = ctypes.CDLL(LIB)
    P = ctypes.c_void_p
    lib.ouro_ed25519_verify_batch.argtypes = [ctypes.c_size_t, P, P, P, P, P, P]
    off = np.zeros(1, np.uint64)
    ln = np.zeros(1, np.uint32)
    v = np.full(1, 7, np.uint8)
    rc = lib.ouro_ed25519_verify_batch(1, bytes(32), bytes(64), b"\0", off.ctypes.data,
                                       ln.ctypes.data, v.ctypes.data)
    assert rc == -4 and v[0] == 7  # OURO_ENODEV
    single, recomputed = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    lib.ouro_debug_host_path(ctypes.byref(single), ctypes.byref(recomputed))
    assert recomputed.value == 0


def test_missing_library_fails_loudly(tmp_path):
    from ouroboros_network_amd import _native

    with pytest.raises(_native.NativeUnavailable):
        _native._lib_saved = _native._lib
        _native._lib = None
        try:
            _native.load(str(tmp_path / "nope.so"))
        finally:
            _native._lib = _native._lib_saved


def test_kes_period_saturation_keeps_word_semantics():
    """kes.periods_u32: the reference's SumKES path choice (t >= half: go right,
    t -= half) restated over unbounded ints picks the same leaf for t and for
    min(t, 2^32 - 1), for every Word-sized t."""
    import numpy as np

    from ouroboros_network_amd.kes import periods_u32

    def leaf(t):
        idx = 0
        for k in range(6, 0, -1):
            half = 1 << (k - 1)
            if t >= half:
                idx, t = idx + half, t - half
        return idx

    ts = [0, 1, 31, 32, 62, 63, 64, 65, 1000, (1 << 32) - 1, 1 << 32, (1 << 63) + 5, (1 << 64) - 1]
    sat = periods_u32(ts)
    assert sat.dtype == np.uint32
    assert [leaf(t) for t in ts] == [leaf(int(s)) for s in sat]
    assert list(periods_u32(np.array(ts, np.uint64))) == list(sat)
    with pytest.raises(ValueError):
        periods_u32([3, -1])


def test_header_batch_saturates_kes_t():
    """HeaderBatch coerces kes_t through kes.periods_u32 (no silent uint32 wrap)."""
    import numpy as np

    from ouroboros_network_amd.tpraos import HeaderBatch

    n = 3
    z = lambda w: np.zeros((n, w), np.uint8)  # noqa: E731
    hb = HeaderBatch(issuer_vk=z(32), vrf_vk=z(32), eta_proof=z(80), leader_proof=z(80),
                     eta_alpha=z(32), leader_alpha=z(32), hot_vk=z(32),
                     ocert_counter=np.zeros(n, np.uint64), ocert_kes_period=np.zeros(n, np.uint64),
                     ocert_sigma=z(64), kes_t=np.array([5, 1 << 32, (1 << 64) - 1], np.uint64),
                     kes_sig=z(448), body=np.zeros(1, np.uint8), body_off=np.zeros(n, np.uint64),
                     body_len=np.zeros(n, np.uint32))
    assert hb.kes_t.dtype == np.uint32
    assert list(hb.kes_t) == [5, 0xFFFFFFFF, 0xFFFFFFFF]
    assert list(hb.slice(1, 3).kes_t) == [0xFFFFFFFF, 0xFFFFFFFF]


def test_no_getenv_on_call_paths():
    """the library reads its environment switches once
    (csrc/knobs.cpp, on first use or ouro_debug_reload_knobs) -- no other
    translation unit of the product calls getenv, so no call path reads the
    environment (a setenv racing a getenv is undefined behaviour, and a stray
    variable could switch kernels between calls).  numa.cpp's sysfs root and
    the task pool's size are read once at their first use (function-local
    statics), the opt-in shims' error mode once per process."""
    csrc = os.path.join(ROOT, "ouroboros-network_amd", "csrc")
    product = ["kernels.hip", "kernels_lat.hip", "host_path.hip", "pack.cpp"]
    for f in product:
        text = re.sub(r"//[^\n]*", "", open(os.path.join(csrc, f)).read())
        assert "getenv" not in text, f"{f} calls getenv"
    knobs = open(os.path.join(csrc, "knobs.cpp")).read()
    assert len(set(re.findall(r"\"(OURO_[A-Z_0-9]+)\"", knobs))) >= 25
    # the split kernels (rejected A/B) are not selectable in the product
    kern = open(os.path.join(csrc, "kernels.hip")).read()
    body = kern[kern.index("bool split_launch()"):]
    body = body[:body.index("\n}\n")]
    assert "#if OURO_TEST_HOOKS" in body


def test_knobs_read_once_and_on_reload(tmp_path):
    """A switch changed after the library's first call is NOT seen until
    ouro_debug_reload_knobs: OURO_SINGLE_ITEM=gpu routes single items to the
    (here absent) device -- an error -- only after the reload."""
    import subprocess
    import sys

    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the device route would succeed")
    code = r"""
import ctypes, os, sys
sys.path.insert(0, %r)
from ouroboros_network_amd import _native
lib = _native.load()
sys.path.insert(0, %r)
import oracle_ffi as O
pk, sig, msg = O.synth_ed25519(1, first=5)
args = (sig[0].ctypes.data, msg[0].ctypes.data, 32, pk[0].ctypes.data)
assert lib.ouro_ed25519_verify(*args) == 0
os.environ["OURO_SINGLE_ITEM"] = "gpu"
assert lib.ouro_ed25519_verify(*args) == 0      # not re-read
lib.ouro_debug_reload_knobs()
assert lib.ouro_ed25519_verify(*args) != 0      # the device route, no device here
del os.environ["OURO_SINGLE_ITEM"]
lib.ouro_debug_reload_knobs()
assert lib.ouro_ed25519_verify(*args) == 0
print("ok")
""" % (ROOT, os.path.join(ROOT, "tests"))
    env = {k: v for k, v in os.environ.items() if not k.startswith("OURO_")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
