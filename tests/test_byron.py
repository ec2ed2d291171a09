"""ByronDSIGN host side (CPU): the Byron header slicer and signTag assembly
against the reference's golden Byron header, and the oracle's donna-style
acceptance rules on the golden signature and the edge
cases where they differ from libsodium's."""
import numpy as np
import pytest

import oracle_ffi as O
from edge_cases import L, ed25519_edge_cases


def test_golden_byron_header_slices_to_the_signed_message(kats):
    from ouroboros_network_amd.byron import parse_byron_header

    b = kats["byron"]
    h = parse_byron_header(bytes.fromhex(b["raw"]))
    assert h.magic == b["magic"] == 55550001
    assert h.message("header").hex() == b["msg"]
    assert h.delegate_xpub[:32].hex() == b["pk"]
    assert h.sig.hex() == b["sig"]
    assert h.to_sign[0] == 0x85  # ToSign is a 5-element CBOR list


def test_sign_tag_layout():
    from ouroboros_network_amd.byron import cbor_uint, sign_tag_block

    assert cbor_uint(0) == b"\x00" and cbor_uint(23) == b"\x17"
    assert cbor_uint(24) == b"\x18\x18" and cbor_uint(764824073) == b"\x1a\x2d\x96\x4a\x09"
    assert cbor_uint(2**32) == b"\x1b" + (2**32).to_bytes(8, "big")
    tag = sign_tag_block(764824073, bytes(range(64)))
    assert tag == b"01" + bytes(range(64)) + b"\x09\x1a\x2d\x96\x4a\x09"
    with pytest.raises(ValueError):
        sign_tag_block(1, bytes(32))


def test_non_delegated_and_truncated_headers_are_rejected(kats):
    from ouroboros_network_amd.byron import parse_byron_header
    from ouroboros_network_amd.header import CBORError

    raw = bytes.fromhex(kats["byron"]["raw"])
    with pytest.raises(CBORError):
        parse_byron_header(raw[:100])
    with pytest.raises(CBORError):
        parse_byron_header(bytes.fromhex(kats["headers"][0]["raw"]))


def test_oracle_accepts_golden_byron_signature(kats):
    b = kats["byron"]
    sig, msg, pk = bytes.fromhex(b["sig"]), bytes.fromhex(b["msg"]), bytes.fromhex(b["pk"])
    assert O.ed25519_verify_byron(sig, msg, pk)
    assert O.ed25519_verify(sig, msg, pk)  # an honest signature passes both rule sets
    bad = bytearray(msg)
    bad[-1] ^= 1
    assert not O.ed25519_verify_byron(sig, bytes(bad), pk)


def test_byron_rules_differ_from_libsodium_where_expected():
    cases = ed25519_edge_cases()
    pk, sig, msg = cases[0]
    R, S = sig[:32], int.from_bytes(sig[32:], "little")
    assert S + L < 2**253
    s_plus_l = R + (S + L).to_bytes(32, "little")
    assert O.ed25519_verify_byron(s_plus_l, msg, pk)       # donna: S is only bit-checked
    assert not O.ed25519_verify(s_plus_l, msg, pk)         # libsodium: S >= L rejected
    top = R + (S | (1 << 253)).to_bytes(32, "little")
    assert not O.ed25519_verify_byron(top, msg, pk)
    ident = (1).to_bytes(32, "little")
    # the identity-key forgery: donna-style acceptance has no small-order check
    assert O.ed25519_verify_byron(ident + bytes(32), msg, ident)
    assert not O.ed25519_verify(ident + bytes(32), msg, ident)
    verdicts = np.array([O.ed25519_verify_byron(s, m, p) for p, s, m in cases])
    assert verdicts.any() and not verdicts.all()


def test_protocol_magic_is_required_and_the_configured_one_is_used(kats):
    """the sign tag's magic is the node's configured
    ProtocolMagicId (Byron/Ledger/PBFT.hs:43-45, DSIGN.hs:111), never
    silently the peer's header field.  No default; HEADER_MAGIC only by name.
    A header whose magic field differs from the configured magic is rejected
    (host path: no GPU needed)."""
    from ouroboros_network_amd import byron as B

    b = kats["byron"]
    h = B.parse_byron_header(bytes.fromhex(b["raw"]))
    raw = bytes.fromhex(b["raw"])
    with pytest.raises(ValueError):
        B.pack_byron_cbor([raw], None)
    with pytest.raises(TypeError):
        B.verify_byron_cbor([raw])  # pylint: disable=no-value-for-parameter
    with pytest.raises(ValueError):
        h.message(None)
    with pytest.raises(ValueError):
        B.pack_byron_cbor([raw], "peer")
    assert h.message(b["magic"]) == h.message(B.HEADER_MAGIC)  # golden: field == configured
    mainnet = 764824073
    assert h.magic != mainnet
    ok = B.ByronDSIGN.verify_batch([h.delegate_xpub[:32]] * 2,
                                   [h.message(b["magic"]), h.message(mainnet)], [h.sig] * 2,
                                   host=True)
    assert ok.tolist() == [True, False]
    packed = B.pack_byron_cbor([raw], mainnet)
    assert packed.message(0) == h.message(mainnet)
