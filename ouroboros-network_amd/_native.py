"""ctypes binding of the C-ABI product library ``lib/libouro_verify.so``.

The library is the drop-in boundary (``include/ouro_verify.h``); this module is
the Python host's view of it.  There is deliberately no fallback: if the HIP
library is missing or cannot load, every call raises ``NativeUnavailable``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import sys
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# OURO_VERIFY_LIB overrides the library (A/B runs of build variants, tools/ab_variants.py)
LIB_PATH = os.environ.get("OURO_VERIFY_LIB") or os.path.join(_HERE, "lib", "libouro_verify.so")

OURO_OK = 0
OURO_INVALID = -1
OURO_EDEVICE = -2
OURO_EINVAL = -3
OURO_ENODEV = -4

HDR_OCERT_OK = 0x01
HDR_KES_OK = 0x02
HDR_VRF_ETA_OK = 0x04
HDR_VRF_LEADER_OK = 0x08
HDR_ETA_CLAIM_OK = 0x10
HDR_LEADER_CLAIM_OK = 0x20
HDR_ALL_OK = 0x0F      # ref2020: every proof and signature valid
HDR_STRICT_OK = 0x3F   # strict: and both claimed outputs equal the computed ones
HDR_ETA_S_UNREDUCED = 0x40     # the proof's s is not below L
HDR_LEADER_S_UNREDUCED = 0x80
HDR_S_UNREDUCED = 0xC0
VRF_STRICT_S = 0x1             # ouro_vrf03_verify_batch_flags: reject s >= L

LEADER_NO = 0
LEADER_YES = 1
LEADER_BADARG = 0xFF


class NativeUnavailable(RuntimeError):
    """The gfx950 library is not built or cannot be loaded."""


class DeviceError(RuntimeError):
    """A batch could not be verified (HIP/runtime failure).  Never 'valid'."""


class TPraosBatch(ctypes.Structure):
    """Mirror of ``ouro_tpraos_batch`` (include/ouro_verify.h)."""

    _fields_ = [
        ("n", ctypes.c_size_t),
        ("issuer_vk", ctypes.c_void_p),
        ("vrf_vk", ctypes.c_void_p),
        ("eta_proof", ctypes.c_void_p),
        ("leader_proof", ctypes.c_void_p),
        ("eta_alpha", ctypes.c_void_p),
        ("leader_alpha", ctypes.c_void_p),
        ("hot_vk", ctypes.c_void_p),
        ("ocert_counter", ctypes.c_void_p),
        ("ocert_kes_period", ctypes.c_void_p),
        ("ocert_sigma", ctypes.c_void_p),
        ("kes_t", ctypes.c_void_p),
        ("kes_sig", ctypes.c_void_p),
        ("body", ctypes.c_void_p),
        ("body_off", ctypes.c_void_p),
        ("body_len", ctypes.c_void_p),
        # optional (NULL = not used)
        ("eta_output", ctypes.c_void_p),
        ("leader_output", ctypes.c_void_p),
        ("slot", ctypes.c_void_p),
        ("epoch_nonce", ctypes.c_void_p),
        ("eta_nonce", ctypes.c_void_p),
    ]


class ByronBatch(ctypes.Structure):
    """Mirror of ``ouro_byron_batch`` (include/ouro_verify.h)."""

    _fields_ = [("n", ctypes.c_size_t)] + [
        (f, ctypes.c_void_p) for f in ("pk", "sig", "msg", "msg_off", "msg_len", "genesis_vk",
                                       "delegate_vk", "magic")]


# every symbol include/ouro_verify.h (the boundary) and include/ouro_verify_debug.h
# (diagnostics) declare, with its ctypes signature
_P = ctypes.c_void_p
_SZ = ctypes.c_size_t
_I = ctypes.c_int
_ULL = ctypes.c_ulonglong
SIGNATURES = {
    "ouro_set_device": (_I, [_I]),
    "ouro_last_error": (ctypes.c_char_p, []),
    "ouro_ed25519_verify": (_I, [_P, _P, _ULL, _P]),
    "ouro_byron_ed25519_verify": (_I, [_P, _SZ, _P, _P]),
    "ouro_vrf03_verify": (_I, [_P, _P, _P, _P, _ULL]),
    "ouro_vrf03_proof_to_hash": (_I, [_P, _P]),
    "ouro_sum6kes_verify": (_I, [_P, ctypes.c_uint, _P, _ULL, _P]),
    "ouro_ed25519_verify_batch": (_I, [_SZ, _P, _P, _P, _P, _P, _P]),
    "ouro_byron_ed25519_verify_batch": (_I, [_SZ, _P, _P, _P, _P, _P, _P]),
    "ouro_byron_dlg_cert_message": (_SZ, [_P, ctypes.c_uint32, _P, ctypes.c_uint64]),
    "ouro_byron_dlg_cert_verify": (_I, [ctypes.c_uint32, _P, _P, ctypes.c_uint64, _P]),
    "ouro_byron_dlg_cert_verify_batch": (_I, [_SZ, ctypes.c_uint32, _P, _P, _P, _P, _P]),
    "ouro_vrf03_verify_batch": (_I, [_SZ, _P, _P, _P, _P, _P, _P, _P]),
    "ouro_vrf03_verify_batch_flags": (_I, [_SZ, _P, _P, _P, _P, _P, _P, _P, ctypes.c_uint32]),
    "ouro_vrf03_verify_batch_device_flags": (_I, [_P, _SZ, _P, _P, _P, _P, _P, _P, _P,
                                                  ctypes.c_uint32]),
    "ouro_debug_host_path": (_I, [_P, _P]),
    "ouro_ed25519_verify_batch_host": (_I, [_SZ, _P, _P, _P, _P, _P, _P]),
    "ouro_byron_ed25519_verify_batch_host": (_I, [_SZ, _P, _P, _P, _P, _P, _P]),
    "ouro_vrf03_verify_batch_host": (_I, [_SZ, _P, _P, _P, _P, _P, _P, _P, ctypes.c_uint32]),
    "ouro_sum6kes_verify_batch_host": (_I, [_SZ, _P, _P, _P, _P, _P, _P, _P]),
    "ouro_tpraos_verify_batch_host": (_I, [ctypes.POINTER(TPraosBatch), _P, _P, _P]),
    "ouro_leader_check_batch_host": (_I, [_SZ, _P, _P, _P, ctypes.c_int64, ctypes.c_uint64, _I,
                                          _P]),
    "ouro_debug_contexts": (_I, [_I, _P, _P]),
    "ouro_debug_lat_stamps": (_I, [_P]),
    "ouro_debug_clock_stamps": (_I, [_P, _I]),
    "ouro_debug_plan_timing": (_I, [_P, _P, _P, _P]),
    "ouro_device_numa_node": (_I, [_I]),
    "ouro_bind_thread_to_device": (_I, [_I]),
    "ouro_debug_multi_workers": (_I, [_P, _P, _P, _I]),
    "ouro_debug_numa_bind_pci": (_I, [ctypes.c_char_p, _P]),
    "ouro_debug_thread_cpus": (_I, [_P, _I]),
    "ouro_integrity_verify_cbor": (_I, [_P, _SZ, _P, _P, _SZ, ctypes.c_uint64, _P, _P]),
    "ouro_tpraos_verify_cbor": (_I, [_P, _SZ, _P, _P, _SZ, ctypes.c_uint64, _P, _P, _P, _P, _P,
                                     _P, _P, _P]),
    "ouro_debug_cbor_stats": (_I, [_P]),
    "ouro_tpraos_verify_cbor_multi": (_I, [_P, _I, _P, _SZ, _P, _P, _SZ, ctypes.c_uint64, _P, _P,
                                           _P, _P, _P, _P, _P, _P]),
    "ouro_integrity_verify_cbor_multi": (_I, [_P, _I, _P, _SZ, _P, _P, _SZ, ctypes.c_uint64, _P,
                                              _P]),
    "ouro_byron_verify_cbor_multi": (_I, [_P, _I, _P, _SZ, _P, _P, _SZ, ctypes.c_int64, _P, _P]),
    "ouro_debug_test_hooks": (_I, []),
    "ouro_debug_reload_knobs": (None, []),
    "ouro_integrity_verify_cbor_device": (_I, [_P, _P, _SZ, _P, _P, _SZ, ctypes.c_uint64, _P,
                                               _SZ, _P, _P]),
    "ouro_sum6kes_verify_batch": (_I, [_SZ, _P, _P, _P, _P, _P, _P, _P]),
    "ouro_tpraos_verify_batch": (_I, [ctypes.POINTER(TPraosBatch), _P, _P, _P]),
    "ouro_ed25519_verify_batch_device": (_I, [_P, _SZ, _P, _P, _P, _P, _P, _P]),
    "ouro_byron_ed25519_verify_batch_device": (_I, [_P, _SZ, _P, _P, _P, _P, _P, _P]),
    "ouro_vrf03_verify_batch_device": (_I, [_P, _SZ, _P, _P, _P, _P, _P, _P, _P]),
    "ouro_sum6kes_verify_batch_device": (_I, [_P, _SZ, _P, _P, _P, _P, _P, _P, _P]),
    "ouro_tpraos_verify_batch_device": (_I, [_P, ctypes.POINTER(TPraosBatch), _P, _P, _P]),
    "ouro_tpraos_verify_batch_lowlat": (_I, [ctypes.POINTER(TPraosBatch), _P, _P, _P]),
    "ouro_tpraos_plan_create": (_P, [_SZ, _SZ]),
    "ouro_tpraos_plan_run": (_I, [_P, ctypes.POINTER(TPraosBatch), _P, _P, _P]),
    "ouro_tpraos_plan_destroy": (None, [_P]),
    "ouro_device_count": (_I, []),
    "ouro_tpraos_verify_batch_multi": (_I, [ctypes.POINTER(TPraosBatch), _P, _I, _P, _P, _P]),
    "ouro_tpraos_plan_submit": (_I, [_P, ctypes.POINTER(TPraosBatch)]),
    "ouro_tpraos_plan_wait": (_I, [_P, _P, _P, _P]),
    "ouro_leader_check_batch": (_I, [_SZ, _P, _P, _P, ctypes.c_int64, ctypes.c_uint64, _I, _P]),
    "ouro_leader_check_batch_device": (_I, [_P, _SZ, _P, _P, _P, ctypes.c_int64, ctypes.c_uint64,
                                            _I, _P]),
    "ouro_nonce_fold": (_I, [_SZ, _P, _P, ctypes.c_uint64, ctypes.c_uint64, _P, _P, _P]),
    "ouro_tpraos_pack_bytes": (_SZ, [_SZ]),
    "ouro_tpraos_pack_cbor": (_I, [_P, _SZ, _P, _P, _SZ, ctypes.c_uint64, _P, _SZ,
                                   ctypes.POINTER(TPraosBatch), _P, _P, _P, _I]),
    "ouro_byron_pack_bytes": (_SZ, [_SZ, _P]),
    "ouro_byron_pack_cbor": (_I, [_P, _SZ, _P, _P, _SZ, ctypes.c_int64, _P, _SZ,
                                  ctypes.POINTER(ByronBatch), _P, _I]),
    "ouro_byron_verify_cbor": (_I, [_P, _SZ, _P, _P, _SZ, ctypes.c_int64, _P, _P]),
    "ouro_tpraos_pack_cbor_device": (_I, [_P, _P, _SZ, _P, _P, _SZ, ctypes.c_uint64, _P, _SZ,
                                          ctypes.POINTER(TPraosBatch), _P, _P, _P]),
}

# the cardano-crypto-praos names the OPT-IN shim exports (lib/libouro_vrf_shim.so,
# csrc/vrf_shim.cpp); the product library itself does not
SHIM_PATH = os.path.join(_HERE, "lib", "libouro_vrf_shim.so")
VRF_ALIASES = {
    "crypto_vrf_ietfdraft03_verify": (_I, [_P, _P, _P, _P, _ULL]),
    "crypto_vrf_ietfdraft03_proof_to_hash": (_I, [_P, _P]),
    "crypto_vrf_verify": (_I, [_P, _P, _P, _P, _ULL]),
    "crypto_vrf_proof_to_hash": (_I, [_P, _P]),
}

_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and type the product library; raise if unavailable."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NativeUnavailable(
                f"{path} is not built; run `make -C ouroboros-network_amd` "
                "(or __graft_entry__.build())")
        # PyTorch wheels bundle their own libamdhip64 under the same soname as
        # ROCm's: whichever a process loads first is the one both use, and
        # torch.cuda only finds the GPU with its own.  So when torch is
        # installed, load it before this library (a no-op if already loaded).
        if "torch" not in sys.modules:
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        try:
            lib = ctypes.CDLL(path)
        except OSError as e:  # pragma: no cover - depends on the image
            raise NativeUnavailable(f"cannot load {path}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


_shim = None


def load_shim(path: str = SHIM_PATH) -> ctypes.CDLL:
    """The opt-in crypto_vrf_* link shim (loads the product library first)."""
    global _shim
    load()
    with _lock:
        if _shim is None:
            if not os.path.exists(path):
                raise NativeUnavailable(f"{path} is not built")
            lib = ctypes.CDLL(path)
            for name, (res, args) in VRF_ALIASES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _shim = lib
        return _shim


# the test-hook build of the same library (tests/test_gpu_hooks.py loads it in a
# child process through OURO_VERIFY_LIB)
TEST_LIB_PATH = os.path.join(_HERE, "lib", "libouro_verify_test.so")


def test_hooks() -> bool:
    """True when the loaded library is the test-hook build (OURO_TEST_HOOKS)."""
    return bool(load().ouro_debug_test_hooks())


def reload_knobs() -> None:
    """Re-read the library's environment switches (csrc/knobs.h): the library
    reads them once and never on a call path, so a process that changes one
    calls this afterwards (ouro_debug_reload_knobs)."""
    if _lib is not None:
        _lib.ouro_debug_reload_knobs()


@contextlib.contextmanager
def knob_env(**env):
    """Set environment switches (None = unset) for a block, the library
    re-reading them on entry and exit."""
    saved = {k: os.environ.get(k) for k in env}
    try:
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v)
        reload_knobs()
        yield
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        reload_knobs()


def check(rc: int, what: str) -> int:
    """Map a batch return code to an exception; 0 passes through."""
    if rc == OURO_OK:
        return rc
    msg = load().ouro_last_error()
    msg = msg.decode() if msg else ""
    if rc == OURO_EINVAL:
        raise ValueError(f"{what}: invalid arguments ({msg})")
    if rc == OURO_ENODEV:
        raise NativeUnavailable(f"{what}: no gfx950 device ({msg})")
    raise DeviceError(f"{what}: device error {rc} ({msg})")
