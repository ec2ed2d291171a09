"""The C header slicer (include/ouro_verify.h ouro_tpraos_pack_cbor,
csrc/pack.cpp) against the Python one (header.parse_header + header.pack) on
the reference's golden headers and on every single-byte corruption and every
truncation of them: the same headers accepted, bit-identical arrays for the
accepted ones (body compared through its spans: the C slicer points into the
raw buffer instead of copying).  Host-only: no GPU."""
import json
import os

import numpy as np
import pytest

from ouroboros_network_amd import header as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPKP = 129600

FIELDS = ["issuer_vk", "vrf_vk", "eta_proof", "leader_proof", "hot_vk", "ocert_counter",
          "ocert_kes_period", "ocert_sigma", "kes_t", "kes_sig", "eta_output", "leader_output"]


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        return [bytes.fromhex(h["raw"]) for h in json.load(f)["headers"]]


def py_pack(raws, spkp=SPKP):
    """Python slicer; None for a header it rejects (any exception)."""
    out = []
    for r in raws:
        try:
            h = H.parse_header(r)
            b = H.pack([h], [b"\0" * 32], [b"\0" * 32], slots_per_kes_period=spkp)
            out.append((h, b))
        except Exception:  # noqa: BLE001 - any rejection counts
            out.append(None)
    return out


def c_pack(raws, spkp=SPKP, nthreads=1):
    n = len(raws)
    z = np.zeros((n, 32), np.uint8)
    return H.pack_cbor(raws, slots_per_kes_period=spkp, eta_alpha=z, leader_alpha=z,
                       nthreads=nthreads)


def assert_same(raws, py, pk):
    b = pk.batch
    for i, (r, p) in enumerate(zip(raws, py)):
        if p is None:
            assert pk.status[i] != H.PACK_OK, f"header {i}: C accepts what Python rejects"
            for f in FIELDS:
                assert not np.any(getattr(b, f)[i]), f"rejected header {i}: {f} not zeroed"
            assert b.body_len[i] == 0
            continue
        assert pk.status[i] == H.PACK_OK, f"header {i}: C rejects ({pk.status[i]}) what Python accepts"
        h, pb = p
        for f in FIELDS:
            assert np.array_equal(getattr(b, f)[i], getattr(pb, f)[0]), f"header {i}: {f}"
        o, ln = int(b.body_off[i]), int(b.body_len[i])
        assert bytes(b.body[o:o + ln]) == h.body
        assert pk.slot[i] == h.slot and pk.era[i] == h.era


def test_golden_headers_match_python(golden):
    pk = c_pack(golden)
    assert (pk.status == H.PACK_OK).all()
    assert_same(golden, py_pack(golden), pk)
    assert list(pk.era) == [1, 1, 1, 2, 1, 2, 3]


def test_every_byte_corruption_matches_python(golden):
    raws = []
    for g in golden[:2]:  # one unwrapped, one HFC-wrapped
        for pos in range(len(g)):
            for x in (0x01, 0x20, 0x80, 0xFF):
                m = bytearray(g)
                m[pos] ^= x
                raws.append(bytes(m))
    pk = c_pack(raws, nthreads=4)
    py = py_pack(raws)
    assert_same(raws, py, pk)
    # the corruptions exercise both outcomes and several rejection classes
    assert 0 < int((pk.status == H.PACK_OK).sum()) < len(raws)
    # (a single byte can no longer give ESIZE: a field of another length moves
    # the end of [header_body, kes_sig] off the payload's end, which the
    # reference rejects as CBOR first; test_cbor_in_cbor_bounds_as_the_reference
    # makes a consistent one)
    assert {H.PACK_ECBOR, H.PACK_ESHAPE} <= set(pk.status.tolist())


def test_every_truncation_rejected(golden):
    for g in golden[:2]:
        raws = [g[:k] for k in range(len(g))]
        pk = c_pack(raws)
        assert (pk.status != H.PACK_OK).all()
        assert_same(raws, py_pack(raws), pk)


def _cbor_in_cbor_cases(g):
    """Headers the reference's CBOR-in-CBOR decoding rejects
    (ouroboros-network/src/Ouroboros/Network/Block.hs:509-514): payload
    length not matching [header_body, kes_sig], trailing bytes inside the
    payload or after the header, an indefinite byte string."""
    at = g.index(bytes.fromhex("d81859")) + 3      # the 2-byte payload length
    ln = int.from_bytes(g[at:at + 2], "big")
    pre, payload = g[:at], g[at + 2:]
    assert len(payload) == ln
    enc = lambda n: n.to_bytes(2, "big")  # noqa: E731
    out = {
        "length_minus_1": pre + enc(ln - 1) + payload,
        "length_plus_1": pre + enc(ln + 1) + payload,
        "trailing_in_payload": pre + enc(ln + 1) + payload + b"\x00",
        "trailing_after_header": g + b"\x00",
        "trailing_after_header_ff": g + b"\xff\xff",
        # the payload as an indefinite byte string of one chunk
        "indefinite_bytes": pre[:-1] + b"\x5f" + b"\x59" + enc(ln) + payload + b"\xff",
    }
    return out


def _short_eta_proof(g):
    """A well-formed header whose eta proof has 79 bytes (the payload length
    adjusted): CBOR fine, a crypto field of the wrong size (ESIZE)."""
    at = g.index(bytes.fromhex("d81859")) + 3
    ln = int.from_bytes(g[at:at + 2], "big")
    payload = g[at + 2:]
    e = payload.index(b"\x58\x40")          # the eta certificate's output
    q = e + 2 + 64                           # its proof's head
    assert payload[q:q + 2] == b"\x58\x50"
    payload = payload[:q] + b"\x58\x4f" + payload[q + 2:q + 2 + 79] + payload[q + 2 + 80:]
    return g[:at] + (ln - 1).to_bytes(2, "big") + payload


def test_cbor_in_cbor_bounds_as_the_reference(golden):
    """the slicers parse the tag-24 payload alone and reject what
    the reference's decoder rejects -- Python, host C and (tests/test_gpu_pack)
    device C alike."""
    for g in (golden[0], golden[3]):  # unwrapped, HFC-wrapped
        cases = _cbor_in_cbor_cases(g)
        raws = list(cases.values())
        py = py_pack(raws)
        for name, p in zip(cases, py):
            assert p is None, f"Python accepts {name}"
        pk = c_pack(raws)
        for name, st in zip(cases, pk.status):
            assert st != H.PACK_OK, f"C accepts {name}"
        assert_same(raws, py, pk)
        short = _short_eta_proof(g)
        assert py_pack([short]) == [None]
        assert c_pack([short]).status[0] == H.PACK_ESIZE


def test_byron_era_and_wrappers(golden):
    g = golden[0]  # N2N v1: #6.24(...)
    wrapped = [b"\x82\x00" + g, b"\x82\x05" + g, b"\x82\x18\x2a" + g]
    pk = c_pack(wrapped)
    assert pk.status.tolist() == [H.PACK_EBYRON, H.PACK_OK, H.PACK_OK]
    assert pk.era.tolist()[1:] == [5, 42]
    assert_same(wrapped, py_pack(wrapped), pk)


def test_threads_and_spans_inside_one_buffer(golden):
    rng = np.random.default_rng(7)
    raws = [golden[int(k)] for k in rng.integers(0, len(golden), 9000)]
    # a shared buffer with junk between headers and absolute offsets
    parts, off, ln, at = [], [], [], 0
    for r in raws:
        pad = bytes(rng.integers(0, 256, int(rng.integers(0, 5)), dtype=np.uint8))
        parts += [pad, r]
        off.append(at + len(pad))
        ln.append(len(r))
        at += len(pad) + len(r)
    buf = b"".join(parts)
    z = np.zeros((len(raws), 32), np.uint8)
    one = H.pack_cbor((buf, off, ln), eta_alpha=z, leader_alpha=z, nthreads=1)
    many = H.pack_cbor((buf, off, ln), eta_alpha=z, leader_alpha=z, nthreads=3)
    assert (one.status == 0).all() and (many.status == 0).all()
    for f in FIELDS + ["body_off", "body_len"]:
        assert np.array_equal(getattr(one.batch, f), getattr(many.batch, f)), f
    for i in (0, 1, 4500, 8999):
        o, n = int(one.batch.body_off[i]), int(one.batch.body_len[i])
        assert buf[o:o + n] == H.parse_header(raws[i]).body


def test_kes_t_saturates_like_python(golden):
    # slots_per_kes_period = 1: kes_t = slot - c0 (a large Word), saturated
    pk = c_pack(golden[:1], spkp=1)
    py = py_pack(golden[:1], spkp=1)
    assert pk.batch.kes_t[0] == py[0][1].kes_t[0]


def test_bad_arguments_are_einval(golden):
    from ouroboros_network_amd import _native
    with pytest.raises(ValueError):
        H.pack_cbor((golden[0], [0], [len(golden[0]) + 1]), seeds=True)  # span past the end
    with pytest.raises(ValueError):
        H.pack_cbor((golden[0], [2 ** 64 - 1], [4]), seeds=True)         # wrapping offset
    lib = _native.load()
    out = _native.TPraosBatch()
    import ctypes
    assert lib.ouro_tpraos_pack_cbor(None, 0, None, None, 0, 0, None, 0, ctypes.byref(out),
                                     None, None, None, 0) == _native.OURO_EINVAL
    st = (ctypes.c_uint8 * 1)()
    small = (ctypes.c_uint8 * 16)()
    buf = (ctypes.c_uint8 * len(golden[0])).from_buffer_copy(golden[0])
    offs = (ctypes.c_uint64 * 1)(0)
    lens = (ctypes.c_uint32 * 1)(len(golden[0]))
    assert lib.ouro_tpraos_pack_cbor(buf, len(golden[0]), offs, lens, 1, SPKP, small, 16,
                                     ctypes.byref(out), None, None, st, 0) == _native.OURO_EINVAL


def test_empty_batch():
    pk = H.pack_cbor([], seeds=True)
    assert len(pk.batch) == 0 and pk.status.size == 0
