"""ouroboros-network_amd -- MI355X-native batch verifier for the Ouroboros
Praos/TPraos header-crypto hot path (Ed25519DSIGN, Sum6KES, PraosVRF draft-03)
and the Byron PBFT block signature (ByronDSIGN).

Importable as ``ouroboros_network_amd`` (repo-root symlink).  The compute path
is the gfx950 library ``lib/libouro_verify.so`` behind the C ABI in
``include/ouro_verify.h``; there is no CPU fallback.
"""
from . import _native
from ._native import DeviceError, NativeUnavailable
from .byron import (ByronDSIGN, dlg_cert_message, pack_byron_cbor, parse_byron_header,
                    verify_byron_cbor, verify_byron_headers, verify_delegation_certs)
from .dsign import Ed25519DSIGN
from .header import verify_headers_cbor, verify_integrity_cbor
from .kes import Sum6KES, kes_period
from .tpraos import HeaderBatch, first_invalid, verify_headers, verify_headers_multi
from .vrf import PraosVRF

__all__ = [
    "ByronDSIGN",
    "DeviceError",
    "Ed25519DSIGN",
    "HeaderBatch",
    "NativeUnavailable",
    "PraosVRF",
    "Sum6KES",
    "first_invalid",
    "kes_period",
    "dlg_cert_message",
    "pack_byron_cbor",
    "parse_byron_header",
    "verify_byron_cbor",
    "verify_byron_headers",
    "verify_delegation_certs",
    "verify_headers",
    "verify_headers_cbor",
    "verify_headers_multi",
    "verify_integrity_cbor",
]


def library_path() -> str:
    return _native.LIB_PATH
