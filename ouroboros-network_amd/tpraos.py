"""TPraos header-crypto batch -- the crypto subset of ``SL.updateChainDepState``.

Reference path: ``TPraos.updateChainDepState``
(ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:433-442)
-> ledger-specs PRTCL -> OVERLAY (two ``verifyCertified`` on
``mkSeed seedEta slot eta0`` / ``mkSeed seedL slot eta0``) and OCERT
(``verifySignedDSIGN coldVk (OCertSignable hotVk n c0) sigma`` then
``verifySignedKES hotVk t bhbody kesSig``).  The sequential fold that consumes
the verdicts (nonce evolution, counters, first-failure stop) stays on the host.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, fields
from typing import Optional

import numpy as np

from . import _native
from ._pack import ptr
from .kes import periods_u32

HDR_OCERT_OK = _native.HDR_OCERT_OK
HDR_KES_OK = _native.HDR_KES_OK
HDR_VRF_ETA_OK = _native.HDR_VRF_ETA_OK
HDR_VRF_LEADER_OK = _native.HDR_VRF_LEADER_OK
HDR_ETA_CLAIM_OK = _native.HDR_ETA_CLAIM_OK
HDR_LEADER_CLAIM_OK = _native.HDR_LEADER_CLAIM_OK
HDR_ALL_OK = _native.HDR_ALL_OK
HDR_STRICT_OK = _native.HDR_STRICT_OK
HDR_ETA_S_UNREDUCED = _native.HDR_ETA_S_UNREDUCED
HDR_LEADER_S_UNREDUCED = _native.HDR_LEADER_S_UNREDUCED
HDR_S_UNREDUCED = _native.HDR_S_UNREDUCED

# field name -> (dtype, row width or None for scalars)
LAYOUT = {
    "issuer_vk": (np.uint8, 32),
    "vrf_vk": (np.uint8, 32),
    "eta_proof": (np.uint8, 80),
    "leader_proof": (np.uint8, 80),
    "eta_alpha": (np.uint8, 32),
    "leader_alpha": (np.uint8, 32),
    "hot_vk": (np.uint8, 32),
    "ocert_counter": (np.uint64, None),
    "ocert_kes_period": (np.uint64, None),
    "ocert_sigma": (np.uint8, 64),
    "kes_t": (np.uint32, None),
    "kes_sig": (np.uint8, 448),
    "body": (np.uint8, None),
    "body_off": (np.uint64, None),
    "body_len": (np.uint32, None),
    # optional members (None = not used; include/ouro_verify.h)
    "eta_output": (np.uint8, 64),
    "leader_output": (np.uint8, 64),
    "slot": (np.uint64, None),
    "epoch_nonce": (np.uint8, None),
}
OPTIONAL = ("eta_output", "leader_output", "slot", "epoch_nonce")
# per-batch (not per-header) members
SHARED = ("body", "epoch_nonce")


@dataclass
class HeaderBatch:
    """Structure-of-arrays batch of TPraos headers (host numpy arrays).

    The optional members follow include/ouro_verify.h: ``eta_output`` /
    ``leader_output`` are the header's claimed certifiedOutputs (enabling the
    HDR_*_CLAIM_OK bits); ``slot`` (+ ``epoch_nonce``, 32 bytes or None for
    NeutralNonce) makes the device derive the VRF inputs with mkSeed, and the
    alphas may then be None."""

    issuer_vk: np.ndarray
    vrf_vk: np.ndarray
    eta_proof: np.ndarray
    leader_proof: np.ndarray
    eta_alpha: Optional[np.ndarray]
    leader_alpha: Optional[np.ndarray]
    hot_vk: np.ndarray
    ocert_counter: np.ndarray
    ocert_kes_period: np.ndarray
    ocert_sigma: np.ndarray
    kes_t: np.ndarray
    kes_sig: np.ndarray
    body: np.ndarray
    body_off: np.ndarray
    body_len: np.ndarray
    eta_output: Optional[np.ndarray] = None
    leader_output: Optional[np.ndarray] = None
    slot: Optional[np.ndarray] = None
    epoch_nonce: Optional[np.ndarray] = None

    def __post_init__(self):
        for f in fields(self):
            v = getattr(self, f.name)
            if v is None:
                if f.name in OPTIONAL or (f.name in ("eta_alpha", "leader_alpha")
                                          and self.slot is not None):
                    continue
                raise ValueError(f"{f.name}: required (the alphas only without slots)")
            dt, w = LAYOUT[f.name]
            if f.name == "kes_t":
                # a Word period saturates (kes.periods_u32), never wraps
                a = periods_u32(np.asarray(v).ravel())
            else:
                a = np.ascontiguousarray(v, dtype=dt)
            if w is not None:
                a = a.reshape(-1, w)
            elif f.name != "body":
                a = a.reshape(-1)
            setattr(self, f.name, a)
        n = len(self)
        for f in fields(self):
            v = getattr(self, f.name)
            if f.name not in SHARED and v is not None and v.shape[0] != n:
                raise ValueError(f"{f.name}: expected {n} rows")
        if self.epoch_nonce is not None and self.epoch_nonce.size != 32:
            raise ValueError("epoch_nonce: 32 bytes (or None for NeutralNonce)")
        # checked in Python ints: a uint64 off + len must not wrap past the check
        if n and max(int(o) + int(ln) for o, ln in zip(self.body_off, self.body_len)) \
                > self.body.size:
            raise ValueError("body_off/body_len address bytes beyond body")

    def __len__(self) -> int:
        return self.issuer_vk.shape[0]

    def _rows(self, sel) -> "HeaderBatch":
        kw = {}
        for f in fields(self):
            v = getattr(self, f.name)
            kw[f.name] = v if (f.name in SHARED or v is None) else v[sel]
        return HeaderBatch(**kw)

    def slice(self, lo: int, hi: int) -> "HeaderBatch":
        """Rows [lo, hi) sharing the body buffer (offsets are absolute)."""
        return self._rows(slice(lo, hi))

    def rows(self, idx) -> "HeaderBatch":
        """The given rows (any order), sharing the body buffer."""
        return self._rows(np.asarray(idx, dtype=np.int64))

    def with_(self, **kw) -> "HeaderBatch":
        """A copy with some members replaced (e.g. claimed outputs, slots)."""
        cur = {f.name: getattr(self, f.name) for f in fields(self)}
        cur.update(kw)
        return HeaderBatch(**cur)

    def c_struct(self, eta_nonce: Optional[np.ndarray] = None) -> _native.TPraosBatch:
        s = _native.TPraosBatch()
        s.n = len(self)
        for f in fields(self):
            v = getattr(self, f.name)
            setattr(s, f.name, ptr(v) if v is not None else None)
        s.eta_nonce = ptr(eta_nonce) if eta_nonce is not None else None
        return s


def _outputs(n: int, nonce: bool):
    return (np.zeros(n, dtype=np.uint8), np.zeros((n, 64), dtype=np.uint8),
            np.zeros((n, 64), dtype=np.uint8), np.zeros((n, 32), np.uint8) if nonce else None)


def verify_headers(batch: HeaderBatch, nonce: bool = False):
    """Verify every header; returns (verdict bits u8, beta_eta (n,64),
    beta_leader (n,64)), and with nonce=True also eta_nonce (n,32): the
    mkNonceFromOutputVRF values the nonce fold consumes (nonce_fold)."""
    n = len(batch)
    verdict, be, bl, en = _outputs(n, nonce)
    if n:
        s = batch.c_struct(en)
        rc = _native.load().ouro_tpraos_verify_batch(ctypes.byref(s), ptr(verdict), ptr(be), ptr(bl))
        _native.check(rc, "ouro_tpraos_verify_batch")
    return (verdict, be, bl, en) if nonce else (verdict, be, bl)


def verify_headers_host(batch: HeaderBatch, nonce: bool = False):
    """verify_headers on the library's host path (ouro_tpraos_verify_batch_host:
    the kernels' lane routines on the CPU threads); same results."""
    n = len(batch)
    verdict, be, bl, en = _outputs(n, nonce)
    if n:
        s = batch.c_struct(en)
        rc = _native.load().ouro_tpraos_verify_batch_host(ctypes.byref(s), ptr(verdict), ptr(be),
                                                          ptr(bl))
        _native.check(rc, "ouro_tpraos_verify_batch_host")
    return (verdict, be, bl, en) if nonce else (verdict, be, bl)


def nonce_fold(eta_nonce: np.ndarray, slot: np.ndarray, first_slot_next_epoch: int,
               stability_window: int, eta_v: Optional[bytes], eta_c: Optional[bytes]):
    """The host-side UPDN fold over headers already verified (ouro_nonce_fold):
    returns the new (eta_v, eta_c), None standing for NeutralNonce."""
    en = np.ascontiguousarray(eta_nonce, np.uint8).reshape(-1, 32)
    sl = np.ascontiguousarray(slot, np.uint64).reshape(-1)
    if sl.size != en.shape[0]:
        raise ValueError("one slot per eta_nonce")
    v = np.frombuffer(eta_v or bytes(32), np.uint8).copy()
    c = np.frombuffer(eta_c or bytes(32), np.uint8).copy()
    neutral = (ctypes.c_int * 2)(int(eta_v is None), int(eta_c is None))
    rc = _native.load().ouro_nonce_fold(en.shape[0], ptr(en), ptr(sl), first_slot_next_epoch,
                                        stability_window, ptr(v), ptr(c), neutral)
    _native.check(rc, "ouro_nonce_fold")
    return (None if neutral[0] else v.tobytes()), (None if neutral[1] else c.tobytes())


def verify_headers_multi(batch: HeaderBatch, devices=None, nonce: bool = False):
    """verify_headers over several GPUs of this process (contiguous shards,
    one worker thread per shard; devices=None: every visible device)."""
    n = len(batch)
    verdict, be, bl, en = _outputs(n, nonce)
    if n:
        s = batch.c_struct(en)
        if devices is None:
            dv, nd = None, 0
        else:
            dv = np.ascontiguousarray(devices, dtype=np.int32)
            nd = int(dv.size)
        rc = _native.load().ouro_tpraos_verify_batch_multi(
            ctypes.byref(s), ptr(dv) if dv is not None else None, nd, ptr(verdict), ptr(be),
            ptr(bl))
        _native.check(rc, "ouro_tpraos_verify_batch_multi")
    return (verdict, be, bl, en) if nonce else (verdict, be, bl)


def verify_headers_lowlat(batch: HeaderBatch, nonce: bool = False):
    """Same results as verify_headers; eight lanes per header (small batches)."""
    n = len(batch)
    verdict, be, bl, en = _outputs(n, nonce)
    if n:
        s = batch.c_struct(en)
        rc = _native.load().ouro_tpraos_verify_batch_lowlat(ctypes.byref(s), ptr(verdict), ptr(be),
                                                            ptr(bl))
        _native.check(rc, "ouro_tpraos_verify_batch_lowlat")
    return (verdict, be, bl, en) if nonce else (verdict, be, bl)


class HeaderPlan:
    """A plan (pinned staging, the latency kernel's launch fixed at create)
    for repeated batches of <= max_headers (the ChainSync small-batch path,
    BASELINE.json configs[4]); include/ouro_verify.h ouro_tpraos_plan_*."""

    def __init__(self, max_headers: int = 64, max_body_bytes: int = 64 * 1400):
        self._lib = _native.load()
        self._p = self._lib.ouro_tpraos_plan_create(max_headers, max_body_bytes)
        if not self._p:
            msg = self._lib.ouro_last_error()
            raise _native.DeviceError(f"plan create failed: {msg.decode() if msg else ''}")
        self.max_headers = max_headers

    def run(self, batch: HeaderBatch, out=None, nonce: bool = False):
        """Verify one batch synchronously; out = (verdict, beta_eta,
        beta_leader[, eta_nonce]) buffers to fill, or None to allocate."""
        n = len(batch)
        if out is None:
            out = _outputs(n, nonce)
            out = out if nonce else out[:3]
        s = batch.c_struct(out[3] if len(out) > 3 else None)
        rc = self._lib.ouro_tpraos_plan_run(self._p, ctypes.byref(s), ptr(out[0]), ptr(out[1]),
                                            ptr(out[2]))
        _native.check(rc, "ouro_tpraos_plan_run")
        return out

    def submit(self, batch: HeaderBatch, nonce: bool = False) -> None:
        """Start a batch and return at once (ouro_tpraos_plan_submit); the
        batch's arrays may be reused immediately.  With nonce=True, wait()
        also returns the batch's eta_nonce rows."""
        self._nonce = np.zeros((len(batch), 32), np.uint8) if nonce else None
        s = batch.c_struct(self._nonce)
        _native.check(self._lib.ouro_tpraos_plan_submit(self._p, ctypes.byref(s)),
                      "ouro_tpraos_plan_submit")
        self._pending = len(batch)

    def wait(self, out=None):
        """Results of the submitted batch (ouro_tpraos_plan_wait)."""
        n = getattr(self, "_pending", 0)
        if out is None:
            out = (np.zeros(n, np.uint8), np.zeros((n, 64), np.uint8), np.zeros((n, 64), np.uint8))
        rc = self._lib.ouro_tpraos_plan_wait(self._p, ptr(out[0]), ptr(out[1]), ptr(out[2]))
        _native.check(rc, "ouro_tpraos_plan_wait")
        self._pending = 0
        nonce, self._nonce = getattr(self, "_nonce", None), None
        return tuple(out) + (nonce,) if nonce is not None else out

    def close(self):
        if self._p:
            self._lib.ouro_tpraos_plan_destroy(self._p)
            self._p = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass


def first_invalid(verdict: np.ndarray, required: int = HDR_ALL_OK,
                  s_mode: str = "reduce") -> Optional[int]:
    """Index of the first header failing any required CRYPTO check (HDR_ALL_OK
    for the reference's ref2020 semantics, HDR_STRICT_OK to also demand the
    claimed VRF outputs; s_mode="strict" also rejects a VRF proof whose s is
    not below L, the HDR_*_S_UNREDUCED bits) -- where the reference's sequential
    HeaderStateHistory fold stops as far as the crypto goes.

    The verdict bits cover the signatures and proofs only.  The host fold must
    still apply the OCERT rule's non-crypto checks itself: the KES window
    (c0 <= kesPeriod(slot) < c0 + maxKESEvo; kes_t is only clamped at 0 like
    Integrity.hs:38-44), the operational-certificate counter, the VRF key hash
    against the pool's registration, and the leader threshold
    (leader.check_leader_value on the CLAIMED leader output)."""
    if s_mode not in ("reduce", "strict"):
        raise ValueError("s_mode: reduce or strict")
    bad = (verdict & required) != required
    if s_mode == "strict":
        bad |= (verdict & HDR_S_UNREDUCED) != 0
    bad = np.nonzero(bad)[0]
    return int(bad[0]) if bad.size else None


# ---- device-resident batches (torch tensors on a HIP device) -----------------

class DeviceHeaderBatch:
    """The same SoA held as torch uint8/int tensors in HBM."""

    def __init__(self, host: HeaderBatch, device):
        import torch

        self.n = len(host)
        self.t = {}
        for f in fields(host):
            a = getattr(host, f.name)
            if a is None:
                continue
            self.t[f.name] = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)
                                              ).to(device)
        self.verdict = torch.zeros(self.n, dtype=torch.uint8, device=device)
        self.beta_eta = torch.zeros(self.n * 64, dtype=torch.uint8, device=device)
        self.beta_leader = torch.zeros(self.n * 64, dtype=torch.uint8, device=device)
        self._s = _native.TPraosBatch()
        self._s.n = self.n
        for name, ten in self.t.items():
            setattr(self._s, name, ten.data_ptr())

    def launch(self, stream_handle: int) -> None:
        """Enqueue the header kernel on `stream_handle` (a hipStream_t as int)."""
        rc = _native.load().ouro_tpraos_verify_batch_device(
            ctypes.c_void_p(stream_handle), ctypes.byref(self._s), self.verdict.data_ptr(),
            self.beta_eta.data_ptr(), self.beta_leader.data_ptr())
        _native.check(rc, "ouro_tpraos_verify_batch_device")
