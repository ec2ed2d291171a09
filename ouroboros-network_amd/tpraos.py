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
from typing import Optional, Tuple

import numpy as np

from . import _native
from ._pack import ptr
from .kes import periods_u32

HDR_OCERT_OK = _native.HDR_OCERT_OK
HDR_KES_OK = _native.HDR_KES_OK
HDR_VRF_ETA_OK = _native.HDR_VRF_ETA_OK
HDR_VRF_LEADER_OK = _native.HDR_VRF_LEADER_OK
HDR_ALL_OK = _native.HDR_ALL_OK

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
}


@dataclass
class HeaderBatch:
    """Structure-of-arrays batch of TPraos headers (host numpy arrays)."""

    issuer_vk: np.ndarray
    vrf_vk: np.ndarray
    eta_proof: np.ndarray
    leader_proof: np.ndarray
    eta_alpha: np.ndarray
    leader_alpha: np.ndarray
    hot_vk: np.ndarray
    ocert_counter: np.ndarray
    ocert_kes_period: np.ndarray
    ocert_sigma: np.ndarray
    kes_t: np.ndarray
    kes_sig: np.ndarray
    body: np.ndarray
    body_off: np.ndarray
    body_len: np.ndarray

    def __post_init__(self):
        for f in fields(self):
            dt, w = LAYOUT[f.name]
            if f.name == "kes_t":
                # a Word period saturates (kes.periods_u32), never wraps
                a = periods_u32(np.asarray(getattr(self, f.name)).ravel())
            else:
                a = np.ascontiguousarray(getattr(self, f.name), dtype=dt)
            if w is not None:
                a = a.reshape(-1, w)
            setattr(self, f.name, a)
        n = len(self)
        for f in fields(self):
            if f.name != "body" and getattr(self, f.name).shape[0] != n:
                raise ValueError(f"{f.name}: expected {n} rows")
        if n and int((self.body_off + self.body_len).max()) > self.body.size:
            raise ValueError("body_off/body_len address bytes beyond body")

    def __len__(self) -> int:
        return self.issuer_vk.shape[0]

    def slice(self, lo: int, hi: int) -> "HeaderBatch":
        """Rows [lo, hi) sharing the body buffer (offsets are absolute)."""
        kw = {f.name: getattr(self, f.name)[lo:hi] for f in fields(self) if f.name != "body"}
        return HeaderBatch(body=self.body, **kw)

    def rows(self, idx) -> "HeaderBatch":
        """The given rows (any order), sharing the body buffer."""
        idx = np.asarray(idx, dtype=np.int64)
        kw = {f.name: getattr(self, f.name)[idx] for f in fields(self) if f.name != "body"}
        return HeaderBatch(body=self.body, **kw)

    def c_struct(self) -> _native.TPraosBatch:
        s = _native.TPraosBatch()
        s.n = len(self)
        for f in fields(self):
            setattr(s, f.name, ptr(getattr(self, f.name)))
        return s


def verify_headers(batch: HeaderBatch) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Verify every header; returns (verdict bits u8, beta_eta (n,64), beta_leader (n,64))."""
    n = len(batch)
    verdict = np.zeros(n, dtype=np.uint8)
    be = np.zeros((n, 64), dtype=np.uint8)
    bl = np.zeros((n, 64), dtype=np.uint8)
    if n:
        s = batch.c_struct()
        rc = _native.load().ouro_tpraos_verify_batch(ctypes.byref(s), ptr(verdict), ptr(be), ptr(bl))
        _native.check(rc, "ouro_tpraos_verify_batch")
    return verdict, be, bl


def verify_headers_multi(batch: HeaderBatch, devices=None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """verify_headers over several GPUs of this process (contiguous shards,
    one worker thread per shard; devices=None: every visible device)."""
    n = len(batch)
    verdict = np.zeros(n, dtype=np.uint8)
    be = np.zeros((n, 64), dtype=np.uint8)
    bl = np.zeros((n, 64), dtype=np.uint8)
    if n:
        s = batch.c_struct()
        if devices is None:
            dv, nd = None, 0
        else:
            dv = np.ascontiguousarray(devices, dtype=np.int32)
            nd = int(dv.size)
        rc = _native.load().ouro_tpraos_verify_batch_multi(
            ctypes.byref(s), ptr(dv) if dv is not None else None, nd, ptr(verdict), ptr(be),
            ptr(bl))
        _native.check(rc, "ouro_tpraos_verify_batch_multi")
    return verdict, be, bl


def verify_headers_lowlat(batch: HeaderBatch) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Same results as verify_headers; eight lanes per header (small batches)."""
    n = len(batch)
    verdict = np.zeros(n, dtype=np.uint8)
    be = np.zeros((n, 64), dtype=np.uint8)
    bl = np.zeros((n, 64), dtype=np.uint8)
    if n:
        s = batch.c_struct()
        rc = _native.load().ouro_tpraos_verify_batch_lowlat(ctypes.byref(s), ptr(verdict), ptr(be),
                                                            ptr(bl))
        _native.check(rc, "ouro_tpraos_verify_batch_lowlat")
    return verdict, be, bl


class HeaderPlan:
    """A captured hipGraph plan for repeated batches of <= max_headers
    (the ChainSync small-batch path, BASELINE.json configs[4])."""

    def __init__(self, max_headers: int = 64, max_body_bytes: int = 64 * 1400):
        self._lib = _native.load()
        self._p = self._lib.ouro_tpraos_plan_create(max_headers, max_body_bytes)
        if not self._p:
            msg = self._lib.ouro_last_error()
            raise _native.DeviceError(f"plan create failed: {msg.decode() if msg else ''}")
        self.max_headers = max_headers

    def run(self, batch: HeaderBatch, out=None):
        n = len(batch)
        if out is None:
            out = (np.zeros(n, np.uint8), np.zeros((n, 64), np.uint8), np.zeros((n, 64), np.uint8))
        s = batch.c_struct()
        rc = self._lib.ouro_tpraos_plan_run(self._p, ctypes.byref(s), ptr(out[0]), ptr(out[1]),
                                            ptr(out[2]))
        _native.check(rc, "ouro_tpraos_plan_run")
        return out

    def submit(self, batch: HeaderBatch) -> None:
        """Start a batch and return at once (ouro_tpraos_plan_submit); the
        batch's arrays may be reused immediately."""
        s = batch.c_struct()
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
        return out

    def close(self):
        if self._p:
            self._lib.ouro_tpraos_plan_destroy(self._p)
            self._p = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass


def first_invalid(verdict: np.ndarray, required: int = HDR_ALL_OK) -> Optional[int]:
    """Index of the first header failing any required check -- where the
    reference's sequential HeaderStateHistory fold stops."""
    bad = np.nonzero((verdict & required) != required)[0]
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
