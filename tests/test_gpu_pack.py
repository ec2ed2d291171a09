"""Raw wire CBOR -> verdicts on the GPU: headers sliced
by the C slicer (ouro_tpraos_pack_cbor) give the verdicts and outputs of the
Python-sliced batch and of the oracle; synthesised raw headers (keys, VRF
certificates with their real outputs, opcerts, KES over the encoded body) are
all valid end to end, and corruptions of their wire bytes are judged like the
oracle judges the same sliced batch."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ffi as O  # noqa: E402

pytestmark = pytest.mark.gpu


def test_golden_raw_headers_through_the_c_slicer(gpu_lib, kats):
    from ouroboros_network_amd import header as H
    from ouroboros_network_amd import verify_headers

    hs = kats["headers"]
    raws = [bytes.fromhex(h["raw"]) for h in hs]
    ea = np.array([list(bytes.fromhex(h["eta_alpha"])) for h in hs], np.uint8)
    la = np.array([list(bytes.fromhex(h["leader_alpha"])) for h in hs], np.uint8)
    pk = H.pack_cbor(raws, slots_per_kes_period=100, eta_alpha=ea, leader_alpha=la)
    assert (pk.status == H.PACK_OK).all()
    verdict, be, bl = verify_headers(pk.batch)
    ref = H.pack([H.parse_header(r) for r in raws], [bytes(a) for a in ea], [bytes(a) for a in la],
                 slots_per_kes_period=100)
    rv, rbe, rbl = verify_headers(ref)
    np.testing.assert_array_equal(verdict, rv)
    np.testing.assert_array_equal(be, rbe)
    np.testing.assert_array_equal(bl, rbl)
    for h, v in zip(hs, verdict):
        assert int(v) & 0x0F == h["expect_verdict"], h["name"]


def test_synthesised_raw_headers_end_to_end(gpu_lib):
    import torch

    import bench
    from ouroboros_network_amd import header as H
    from ouroboros_network_amd import verify_headers

    n = 2048
    dev = torch.device("cuda", 0)
    t, raw, rl = bench.synth_raw_headers(n, 64, dev)
    rawh = raw.cpu().numpy()
    off = np.arange(n, dtype=np.uint64) * rl
    ln = np.full(n, rl, np.uint32)
    host = {k: v.cpu().numpy() for k, v in t.items()}
    ea = host["eta_alpha"].reshape(n, 32)
    la = host["leader_alpha"].reshape(n, 32)
    pk = H.pack_cbor((rawh, off, ln), eta_alpha=ea, leader_alpha=la, nthreads=2)
    assert (pk.status == H.PACK_OK).all()
    b = pk.batch
    for k, w in (("issuer_vk", 32), ("vrf_vk", 32), ("eta_proof", 80), ("leader_proof", 80),
                 ("hot_vk", 32), ("ocert_sigma", 64)):
        np.testing.assert_array_equal(getattr(b, k), host[k].reshape(n, w), k)
    np.testing.assert_array_equal(b.kes_t, host["kes_t"].view(np.uint32))
    assert not b.ocert_counter.any() and not b.ocert_kes_period.any()
    verdict, be, bl = verify_headers(b)
    assert (verdict == 0x3F).all()  # every check, claimed outputs = computed
    np.testing.assert_array_equal(be, b.eta_output)
    np.testing.assert_array_equal(bl, b.leader_output)

    # wire corruptions: a byte in each of the body, the KES signature and a
    # claimed output; verdicts equal the oracle's on the sliced batch
    rng = np.random.default_rng(11)
    tmpl, offs = bench.raw_template()
    o = dict(zip(bench.RAW_OFFSET_NAMES, offs))
    bad = rawh.copy().reshape(n, rl)
    rows = rng.choice(n, 96, replace=False)
    for k, r in enumerate(rows):
        lo, hi = [(o["body"], o["body"] + o["body_len"]), (o["sig"], o["sig"] + 448),
                  (o["eta_out"], o["eta_out"] + 64)][k % 3]
        bad[r, int(rng.integers(lo, hi))] ^= 1 << int(rng.integers(0, 8))
    pk2 = H.pack_cbor((bad.reshape(-1), off, ln), eta_alpha=ea, leader_alpha=la)
    sel = np.sort(rows)
    v2, be2, bl2 = verify_headers(pk2.batch)
    wv, wbe, wbl = O.tpraos_verify_batch(_rows(pk2.batch, sel))
    np.testing.assert_array_equal(v2[sel], wv)
    np.testing.assert_array_equal(be2[sel], wbe)
    np.testing.assert_array_equal(bl2[sel], wbl)
    assert (v2[np.setdiff1d(np.arange(n), sel)] == 0x3F).all()
    assert (v2[sel] != 0x3F).all()  # every corruption is caught by some check


def _rows(batch, sel):
    """The headers `sel` of a batch as a new HeaderBatch (for the oracle)."""
    from ouroboros_network_amd.tpraos import HeaderBatch

    def pick(a):
        return None if a is None else a[sel]

    bodies = [bytes(batch.body[int(batch.body_off[i]):int(batch.body_off[i]) + int(batch.body_len[i])])
              for i in sel]
    lens = np.array([len(x) for x in bodies], np.uint32)
    offs = np.zeros(len(sel), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return HeaderBatch(
        issuer_vk=pick(batch.issuer_vk), vrf_vk=pick(batch.vrf_vk), eta_proof=pick(batch.eta_proof),
        leader_proof=pick(batch.leader_proof), eta_alpha=pick(batch.eta_alpha),
        leader_alpha=pick(batch.leader_alpha), hot_vk=pick(batch.hot_vk),
        ocert_counter=pick(batch.ocert_counter), ocert_kes_period=pick(batch.ocert_kes_period),
        ocert_sigma=pick(batch.ocert_sigma), kes_t=pick(batch.kes_t), kes_sig=pick(batch.kes_sig),
        body=np.frombuffer(b"".join(bodies), np.uint8), body_off=offs, body_len=lens,
        eta_output=pick(batch.eta_output), leader_output=pick(batch.leader_output))


def _device_pack(raw_bytes: bytes, off, ln, spkp=129600):
    """ouro_tpraos_pack_cbor_device on a device copy of the buffers; returns
    (host views of the arena arrays as a dict, status, slot, era)."""
    import ctypes

    import torch

    from ouroboros_network_amd import _native

    lib = _native.load()
    dev = torch.device("cuda", 0)
    n = len(off)
    raw = torch.frombuffer(bytearray(raw_bytes), dtype=torch.uint8).to(dev)
    doff = torch.tensor(np.asarray(off, np.int64), device=dev)
    dlen = torch.tensor(np.asarray(ln, np.int32), device=dev)
    nb = int(lib.ouro_tpraos_pack_bytes(n))
    arena = torch.zeros(nb, dtype=torch.uint8, device=dev)
    status = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    slot = torch.zeros(n, dtype=torch.int64, device=dev)
    era = torch.zeros(n, dtype=torch.uint8, device=dev)
    out = _native.TPraosBatch()
    st = torch.cuda.current_stream()
    rc = lib.ouro_tpraos_pack_cbor_device(ctypes.c_void_p(st.cuda_stream), raw.data_ptr(), raw.numel(),
                                          doff.data_ptr(), dlen.data_ptr(), n, spkp, arena.data_ptr(),
                                          nb, ctypes.byref(out), slot.data_ptr(), era.data_ptr(),
                                          status.data_ptr())
    assert rc == 0, rc
    torch.cuda.synchronize()
    host = arena.cpu().numpy()
    base = arena.data_ptr()

    def view(addr, dt, w):
        cnt = n * (w or 1) * np.dtype(dt).itemsize
        a = host[addr - base: addr - base + cnt].view(dt)
        return a.reshape(n, w) if w else a

    f = {"issuer_vk": view(out.issuer_vk, np.uint8, 32), "vrf_vk": view(out.vrf_vk, np.uint8, 32),
         "eta_proof": view(out.eta_proof, np.uint8, 80),
         "leader_proof": view(out.leader_proof, np.uint8, 80),
         "hot_vk": view(out.hot_vk, np.uint8, 32),
         "ocert_counter": view(out.ocert_counter, np.uint64, None),
         "ocert_kes_period": view(out.ocert_kes_period, np.uint64, None),
         "ocert_sigma": view(out.ocert_sigma, np.uint8, 64), "kes_t": view(out.kes_t, np.uint32, None),
         "kes_sig": view(out.kes_sig, np.uint8, 448), "body_off": view(out.body_off, np.uint64, None),
         "body_len": view(out.body_len, np.uint32, None),
         "eta_output": view(out.eta_output, np.uint8, 64),
         "leader_output": view(out.leader_output, np.uint8, 64)}
    assert out.body == raw.data_ptr()
    return f, status.cpu().numpy(), slot.cpu().numpy().view(np.uint64), era.cpu().numpy()


def test_device_slicer_matches_host_slicer(gpu_lib, kats):
    """The device slicer (same cbor.h code) against the host one on the golden
    headers, every single-byte corruption of two of them, truncations, and
    spans outside the buffer (device status OURO_PACK_ESPAN)."""
    from ouroboros_network_amd import header as H

    golden = [bytes.fromhex(h["raw"]) for h in kats["headers"]]
    raws = list(golden)
    for g in golden[:2]:
        for pos in range(len(g)):
            for x in (0x01, 0x80, 0xFF):
                m = bytearray(g)
                m[pos] ^= x
                raws.append(bytes(m))
        raws += [g[:k] for k in range(0, len(g), 7)]
    # CBOR-in-CBOR bounds: rejected alike on host and device
    import test_pack as TP

    for g in (golden[0], golden[3]):
        raws += list(TP._cbor_in_cbor_cases(g).values()) + [TP._short_eta_proof(g)]
    ln = np.array([len(r) for r in raws], np.uint32)
    off = np.zeros(len(raws), np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    buf = b"".join(raws)
    z = np.zeros((len(raws), 32), np.uint8)
    hp = H.pack_cbor((buf, off, ln), eta_alpha=z, leader_alpha=z)
    dev, status, slot, era = _device_pack(buf, off, ln)
    np.testing.assert_array_equal(status, hp.status)
    assert 0 < int((status == 0).sum()) < len(raws)
    for k, v in dev.items():
        np.testing.assert_array_equal(v, getattr(hp.batch, k), k)
    np.testing.assert_array_equal(slot, hp.slot)
    np.testing.assert_array_equal(era, hp.era)
    # spans outside the buffer: rejected per header, neighbours unaffected
    off2, ln2 = off[:3].copy(), ln[:3].copy()
    off2[1] = len(buf) - 10
    ln2[2] = len(buf) + 1
    _, st2, _, _ = _device_pack(buf, off2, ln2)
    assert st2.tolist() == [H.PACK_OK, H.PACK_ESPAN, H.PACK_ESPAN]


def test_raw_headers_sliced_and_verified_on_device(gpu_lib):
    """Synthetic raw headers in HBM -> device slicer -> header kernel, all on
    one stream: every header valid, results equal to the host-sliced path."""
    import ctypes

    import torch

    import bench
    from ouroboros_network_amd import _native

    lib = _native.load()
    n = 4096
    dev = torch.device("cuda", 0)
    t, raw, rl = bench.synth_raw_headers(n, 64, dev)
    off = torch.arange(n, dtype=torch.int64, device=dev) * rl
    ln = torch.full((n,), rl, dtype=torch.int32, device=dev)
    nb = int(lib.ouro_tpraos_pack_bytes(n))
    arena = torch.zeros(nb, dtype=torch.uint8, device=dev)
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    out = _native.TPraosBatch()
    st = torch.cuda.current_stream()
    S = ctypes.c_void_p(st.cuda_stream)
    assert lib.ouro_tpraos_pack_cbor_device(S, raw.data_ptr(), raw.numel(), off.data_ptr(),
                                            ln.data_ptr(), n, 129600, arena.data_ptr(), nb,
                                            ctypes.byref(out), None, None, status.data_ptr()) == 0
    out.eta_alpha = t["eta_alpha"].data_ptr()
    out.leader_alpha = t["leader_alpha"].data_ptr()
    v = torch.zeros(n, dtype=torch.uint8, device=dev)
    be = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    bl = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    assert lib.ouro_tpraos_verify_batch_device(S, ctypes.byref(out), v.data_ptr(), be.data_ptr(),
                                               bl.data_ptr()) == 0
    torch.cuda.synchronize()
    assert (status.cpu() == 0).all()
    assert (v.cpu() == 0x3F).all()
