"""Concurrent C callers of the ABI (tests/c/concurrency.c): 8 pthreads mixing
single-item calls (ouro_ed25519_verify, crypto_vrf_ietfdraft03_verify,
ouro_sum6kes_verify, crypto_vrf_proof_to_hash) with batch calls, every result
checked against the oracle -- the header's "thread-safe and reentrant"
promise, under the reference's one-thread-per-peer calling pattern
(ouroboros-consensus/src/Ouroboros/Consensus/Network/NodeToNode.hs:173-176)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "build", "concurrency")

pytestmark = pytest.mark.gpu


def test_eight_threads_mixed_calls(gpu_lib):
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "c")], check=True)
    r = subprocess.run([EXE, "8", "30"], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.split() == ["ok", str(8 * 30)]
