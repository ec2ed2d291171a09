"""GPU parity at BASELINE.json's full sizes (configs[3]: 1,048,576 headers on
one GPU; configs[1] / configs[2]: 1M VRF proofs / Sum6KES signatures; the
metric's Ed25519 leg: 1M signatures) through size-independent properties,
plus a bit-exact oracle sample.

1/8 of the device-synthesised headers get one byte incremented
(applyCorruption-style, ouroboros-consensus-test/src/Test/Util/Corruption.hs)
in exactly one of the four signed objects, so each header's verdict is known
without the oracle: the corrupted check's bit is cleared and only that one.
The VRF outputs of the header kernel equal those of the standalone VRF kernel
(and are zero where the proof fails).  A random sample of 2,048 headers is
compared with the CPU oracle bit for bit (verdicts and both 64-byte outputs).
"""
import os
import sys

import numpy as np
import pytest

import oracle_ffi as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ge_l(s):
    """Rows of 32-byte little-endian scalars that are >= L (vectorised)."""
    L = (2**252 + 27742317777372353535851937790883648493).to_bytes(32, "little")
    gt = np.zeros(s.shape[0], bool)
    eq = np.ones(s.shape[0], bool)
    for b in range(31, -1, -1):
        gt |= eq & (s[:, b] > L[b])
        eq &= s[:, b] == L[b]
    return gt | eq


def _s_unreduced_bits(se, sl):
    return (_ge_l(se) * 0x40 | _ge_l(sl) * 0x80).astype(np.uint8)


def test_full_size_batch_with_corruptions():
    import ctypes

    import torch

    sys.path.insert(0, ROOT)
    import bench
    from ouroboros_network_amd import _native

    dev = torch.device("cuda:0")
    n = 1 << 20
    t, _ = bench.synth_headers(n, 1024, dev)
    g = torch.Generator().manual_seed(20261016)
    # (field, row width, verdict bits the corruption must clear): signatures
    # and proofs, and -- SURVEY.md §8(d)'s pk | sig | msg | proof | alpha --
    # the keys (the hot key is both the OCert's message and the KES root),
    # the VRF inputs, the OCert counter / KES period (the OCert's message) and
    # the header body (the KES message)
    fields = [("ocert_sigma", 64, 0x01), ("kes_sig", 448, 0x02), ("eta_proof", 80, 0x04),
              ("leader_proof", 80, 0x08), ("issuer_vk", 32, 0x01), ("hot_vk", 32, 0x03),
              ("vrf_vk", 32, 0x0C), ("eta_alpha", 32, 0x04), ("leader_alpha", 32, 0x08),
              ("ocert_counter", 8, 0x01), ("ocert_kes_period", 8, 0x01), ("body", 544, 0x02)]
    pick = torch.randint(0, 8, (n,), generator=g) == 0
    which = torch.randint(0, len(fields), (n,), generator=g)
    expect = torch.full((n,), 15, dtype=torch.uint8)
    for k, (name, w, bit) in enumerate(fields):
        rows = torch.nonzero(pick & (which == k)).squeeze(1)
        cols = torch.randint(0, w, (rows.numel(),), generator=g)
        view = t[name].view(n, w)
        view[rows.to(dev), cols.to(dev)] += 1
        expect[rows] = 15 ^ bit
    # a corrupted byte of a proof's s can lift it to s >= L: the header then
    # also carries that proof's OURO_HDR_*_S_UNREDUCED bit (include/ouro_verify.h)
    expect |= torch.from_numpy(_s_unreduced_bits(t["eta_proof"].view(n, 80)[:, 48:].cpu().numpy(),
                                                 t["leader_proof"].view(n, 80)[:, 48:].cpu().numpy()))
    hdr = bench.DeviceHeaders(t, n, dev)
    st = torch.cuda.current_stream()
    hdr.launch(st)
    torch.cuda.synchronize()
    verdict = hdr.verdict.cpu()
    assert torch.equal(verdict, expect), int((verdict != expect).sum())

    # header-kernel eta outputs == standalone VRF kernel outputs (0 where invalid)
    v = _native.load()
    off = torch.arange(n, dtype=torch.int64, device=dev) * 32
    ln = torch.full((n,), 32, dtype=torch.int32, device=dev)
    beta = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    rc = v.ouro_vrf03_verify_batch_device(ctypes.c_void_p(st.cuda_stream), n,
                                           t["vrf_vk"].data_ptr(), t["eta_proof"].data_ptr(),
                                           t["eta_alpha"].data_ptr(), off.data_ptr(),
                                           ln.data_ptr(), beta.data_ptr(), ok.data_ptr())
    _native.check(rc, "vrf batch")
    torch.cuda.synchronize()
    assert torch.equal(ok.cpu(), ((expect & 0x04) != 0).to(torch.uint8))
    assert int((expect & 0xC0 != 0).sum()) > 0  # the s >= L corner did occur
    assert torch.equal(beta, hdr.beta_eta)

    # bit-exact oracle comparison on a random sample
    rng = np.random.default_rng(5)
    sample = np.sort(rng.choice(n, 2048, replace=False))
    hb = hdr.host_sample(n).rows(sample)
    wv, wbe, wbl = O.tpraos_verify_batch(hb, threads=min(16, os.cpu_count() or 1))
    np.testing.assert_array_equal(verdict.numpy()[sample], wv)
    be = hdr.beta_eta.cpu().numpy().reshape(n, 64)[sample]
    bl = hdr.beta_leader.cpu().numpy().reshape(n, 64)[sample]
    np.testing.assert_array_equal(be, wbe)
    np.testing.assert_array_equal(bl, wbl)

    # the same 1M headers from pageable host memory through the host-buffer
    # ABI (two-stream chunked pipeline) give the device path's results
    from ouroboros_network_amd.tpraos import verify_headers

    hv, hbe, hbl = verify_headers(hdr.host_sample(n))
    np.testing.assert_array_equal(hv, verdict.numpy())
    np.testing.assert_array_equal(hbe.reshape(-1), hdr.beta_eta.cpu().numpy())
    np.testing.assert_array_equal(hbl.reshape(-1), hdr.beta_leader.cpu().numpy())


def test_full_size_kes_batch_with_corruptions():
    """configs[2] at its full size: 1,048,576 Sum6KES signatures (the headers'
    hot keys, periods, bodies and KES signatures) through the standalone
    kernel, 1/8 of them with one byte of the signature, the key or the body
    incremented (each then fails), and a random sample of 1,024 against the
    CPU oracle one by one."""
    import ctypes

    import torch

    sys.path.insert(0, ROOT)
    import bench
    from ouroboros_network_amd import _native

    dev = torch.device("cuda:0")
    n = 1 << 20
    t, blen = bench.synth_headers(n, 1024, dev)
    g = torch.Generator().manual_seed(20261017)
    pick = torch.randint(0, 8, (n,), generator=g) == 0
    which = torch.randint(0, 3, (n,), generator=g)
    expect = torch.ones(n, dtype=torch.uint8)
    for k, (name, w) in enumerate((("kes_sig", 448), ("hot_vk", 32), ("body", blen))):
        rows = torch.nonzero(pick & (which == k)).squeeze(1)
        cols = torch.randint(0, w, (rows.numel(),), generator=g)
        t[name].view(n, w)[rows.to(dev), cols.to(dev)] += 1
        expect[rows] = 0
    v = _native.load()
    st = torch.cuda.current_stream()
    ver = torch.zeros(n, dtype=torch.uint8, device=dev)
    rc = v.ouro_sum6kes_verify_batch_device(ctypes.c_void_p(st.cuda_stream), n,
                                             *[t[k].data_ptr() for k in (
                                                 "hot_vk", "kes_t", "body", "body_off",
                                                 "body_len", "kes_sig")], ver.data_ptr())
    _native.check(rc, "kes batch")
    torch.cuda.synchronize()
    got = ver.cpu()
    assert torch.equal(got, expect), int((got != expect).sum())
    rng = np.random.default_rng(6)
    vk = t["hot_vk"].cpu().numpy().reshape(n, 32)
    kt = t["kes_t"].cpu().numpy().view(np.uint32)
    body = t["body"].cpu().numpy().reshape(n, blen)
    sig = t["kes_sig"].cpu().numpy().reshape(n, 448)
    for i in rng.choice(n, 1024, replace=False):
        want = O.kes_verify(vk[i].tobytes(), int(kt[i]), body[i].tobytes(), sig[i].tobytes())
        assert bool(got[i]) == want, i


def test_full_size_vrf_batch_with_corruptions():
    """configs[1] at its full size: 1,048,576 VRF proofs (the headers' eta
    proofs under their VRF keys and alphas) through the standalone kernel, 1/8
    of them with one byte of the proof, the key or alpha incremented (each then
    fails).  Valid rows' outputs equal the header kernel's eta outputs of the
    uncorrupted batch, failed rows' are zero, and a random sample of 1,024 is
    compared with the CPU oracle (verdict and 64-byte output)."""
    import ctypes

    import torch

    sys.path.insert(0, ROOT)
    import bench
    from ouroboros_network_amd import _native

    dev = torch.device("cuda:0")
    n = 1 << 20
    t, _ = bench.synth_headers(n, 1024, dev)
    v = _native.load()
    st = torch.cuda.current_stream()
    S = ctypes.c_void_p(st.cuda_stream)
    hdr = bench.DeviceHeaders(t, n, dev)
    hdr.launch(st)
    torch.cuda.synchronize()
    hv, be = hdr.verdict.clone(), hdr.beta_eta.clone()
    del hdr
    g = torch.Generator().manual_seed(20261018)
    pick = torch.randint(0, 8, (n,), generator=g) == 0
    which = torch.randint(0, 3, (n,), generator=g)
    expect = torch.ones(n, dtype=torch.uint8)
    for k, (name, w) in enumerate((("eta_proof", 80), ("vrf_vk", 32), ("eta_alpha", 32))):
        rows = torch.nonzero(pick & (which == k)).squeeze(1)
        cols = torch.randint(0, w, (rows.numel(),), generator=g)
        t[name].view(n, w)[rows.to(dev), cols.to(dev)] += 1
        expect[rows] = 0
    a_off = torch.arange(n, dtype=torch.int64, device=dev) * 32
    a_len = torch.full((n,), 32, dtype=torch.int32, device=dev)
    beta = torch.full((n * 64,), 0xAA, dtype=torch.uint8, device=dev)
    ver = torch.zeros(n, dtype=torch.uint8, device=dev)
    rc = v.ouro_vrf03_verify_batch_device(S, n, t["vrf_vk"].data_ptr(), t["eta_proof"].data_ptr(),
                                          t["eta_alpha"].data_ptr(), a_off.data_ptr(),
                                          a_len.data_ptr(), beta.data_ptr(), ver.data_ptr())
    _native.check(rc, "vrf batch")
    torch.cuda.synchronize()
    assert ((hv.cpu() & 15) == 15).all()
    got = ver.cpu()
    assert torch.equal(got, expect), int((got != expect).sum())
    b = beta.view(n, 64).cpu()
    ok = expect.bool()
    assert torch.equal(b[ok], be.view(n, 64).cpu()[ok])
    assert not b[~ok].any()
    rng = np.random.default_rng(7)
    vk = t["vrf_vk"].cpu().numpy().reshape(n, 32)
    pf = t["eta_proof"].cpu().numpy().reshape(n, 80)
    al = t["eta_alpha"].cpu().numpy().reshape(n, 32)
    bn = b.numpy()
    for i in rng.choice(n, 1024, replace=False):
        want = O.vrf_verify(vk[i].tobytes(), pf[i].tobytes(), al[i].tobytes())
        assert bool(got[i]) == (want is not None), i
        assert bn[i].tobytes() == (want or bytes(64)), i


def test_full_size_ed25519_batch_with_corruptions():
    """BASELINE's "Ed25519 ver/s" at the bench's size: 1,048,576 device-
    synthesised signatures over 32-byte messages, 1/8 with one byte of the key,
    the signature or the message incremented (each then fails libsodium's
    rules), the verdicts known in advance, and a random sample of 1,024
    compared with the CPU oracle."""
    import ctypes

    import torch

    sys.path.insert(0, ROOT)
    import bench
    from ouroboros_network_amd import _native

    dev = torch.device("cuda:0")
    n = 1 << 20
    syn = ctypes.CDLL(bench.SYNTH_SO)
    syn.ouro_synth_ed25519.argtypes = [ctypes.c_size_t, ctypes.c_uint64] + [ctypes.c_void_p] * 3
    u8 = dict(dtype=torch.uint8, device=dev)
    pk, sig, msg = torch.empty(n * 32, **u8), torch.empty(n * 64, **u8), torch.empty(n * 32, **u8)
    assert syn.ouro_synth_ed25519(n, 77, pk.data_ptr(), sig.data_ptr(), msg.data_ptr()) == 0
    g = torch.Generator().manual_seed(20261019)
    pick = torch.randint(0, 8, (n,), generator=g) == 0
    which = torch.randint(0, 3, (n,), generator=g)
    expect = torch.ones(n, dtype=torch.uint8)
    for k, (x, w) in enumerate(((pk, 32), (sig, 64), (msg, 32))):
        rows = torch.nonzero(pick & (which == k)).squeeze(1)
        cols = torch.randint(0, w, (rows.numel(),), generator=g)
        x.view(n, w)[rows.to(dev), cols.to(dev)] += 1
        expect[rows] = 0
    off = torch.arange(n, dtype=torch.int64, device=dev) * 32
    ln = torch.full((n,), 32, dtype=torch.int32, device=dev)
    ver = torch.full((n,), 7, **u8)
    st = torch.cuda.current_stream()
    rc = _native.load().ouro_ed25519_verify_batch_device(
        ctypes.c_void_p(st.cuda_stream), n, pk.data_ptr(), sig.data_ptr(), msg.data_ptr(),
        off.data_ptr(), ln.data_ptr(), ver.data_ptr())
    _native.check(rc, "ed25519 batch")
    torch.cuda.synchronize()
    got = ver.cpu()
    assert torch.equal(got, expect), int((got != expect).sum())
    rng = np.random.default_rng(8)
    P = pk.cpu().numpy().reshape(n, 32)
    G = sig.cpu().numpy().reshape(n, 64)
    M = msg.cpu().numpy().reshape(n, 32)
    for i in rng.choice(n, 1024, replace=False):
        assert bool(got[i]) == O.ed25519_verify(G[i].tobytes(), M[i].tobytes(), P[i].tobytes()), i
