import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: larger CPU-side cases")
    config.addinivalue_line("markers", "device_error: forces device errors (the host recompute "
                            "path is expected to run); needs the test-hook build")
    config.addinivalue_line("markers", "hooks: needs the test-hook build of the library "
                            "(lib/libouro_verify_test.so; tests/test_gpu_hooks.py runs these)")


@pytest.fixture(autouse=True)
def _hook_tests_need_the_test_build(request):
    """The product library compiles no test hooks (OURO_TEST_HOOKS): tests that
    inject device errors or poison plan records run only where the test build
    is loaded -- in the child process tests/test_gpu_hooks.py starts."""
    if request.node.get_closest_marker("device_error") is None and \
            request.node.get_closest_marker("hooks") is None:
        return
    from ouroboros_network_amd import _native

    if not _native.test_hooks():
        pytest.skip("needs the test-hook build (run by tests/test_gpu_hooks.py)")


def _reload_knobs():
    from ouroboros_network_amd import _native

    _native.reload_knobs()


@pytest.fixture
def monkeypatch():
    """pytest's monkeypatch, whose environment changes the library sees: it
    reads its switches once (csrc/knobs.h) and is told to re-read them after
    every setenv / delenv and after the undo."""
    mp = pytest.MonkeyPatch()
    setenv, delenv = mp.setenv, mp.delenv

    def _setenv(name, value, prepend=None):
        setenv(name, value, prepend)
        _reload_knobs()

    def _delenv(name, raising=True):
        delenv(name, raising)
        _reload_knobs()

    mp.setenv, mp.delenv = _setenv, _delenv
    yield mp
    mp.undo()
    _reload_knobs()


def _recomputed(lib):
    import ctypes

    a, b = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    lib.ouro_debug_host_path(ctypes.byref(a), ctypes.byref(b))
    return b.value


@pytest.fixture(autouse=True)
def _no_silent_host_recompute(request):
    """A GPU test must pass on the GPU: the library recomputes a host-buffer
    batch on its host path after a device error (include/ouro_verify.h), so
    every `gpu` test not marked `device_error` fails if that happened while
    it ran -- a device fault can never hide behind correct host verdicts."""
    if request.node.get_closest_marker("gpu") is None or \
            request.node.get_closest_marker("device_error") is not None:
        yield
        return
    from ouroboros_network_amd import _native

    before = _recomputed(_native._lib) if _native._lib is not None else 0
    yield
    if _native._lib is not None:
        after = _recomputed(_native._lib)
        assert after == before, f"{after - before} batch(es) were recomputed on the host " \
                                "path after a device error during a GPU test"


@pytest.fixture(scope="session")
def kats():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library on a real device; fails loudly (no skip) when the
    HIP library is missing on a GPU run.  torch is initialised first: its
    wheel bundles its own libamdhip64, and whichever HIP runtime a process
    loads first is the one both then share (same soname) -- torch's must win
    for torch.cuda to see the GPU."""
    import torch

    torch.cuda.init()
    import ouroboros_network_amd as ona

    lib = ona._native.load()
    return lib


@pytest.fixture
def small_chunks():
    """The pipeline cut into many chunks: `set(CHUNK=..., SLOTS=..., RAMP=...)`
    sets OURO_CBOR_* and has the library re-read its switches (knobs.h)."""
    from ouroboros_network_amd import _native

    saved = {k: os.environ.get(k) for k in ("OURO_CBOR_CHUNK", "OURO_CBOR_SLOTS",
                                             "OURO_CBOR_RAMP")}

    def set_(**kw):
        for k, v in kw.items():
            os.environ["OURO_CBOR_" + k] = str(v)
        _native.reload_knobs()

    yield set_
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    _native.reload_knobs()
