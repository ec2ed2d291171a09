/*
 * tpraos.c -- crypto subset of SL.updateChainDepState for one TPraos header.
 * TEST INFRASTRUCTURE ONLY.
 *
 * Reached in the reference via TPraos.updateChainDepState
 * (ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:433-442)
 * -> ledger-specs PRTCL/OVERLAY/OCERT:
 *   OCERT:   verifySignedDSIGN coldVk (OCertSignable hotVk n c0) sigma
 *            (message = hotVk || BE64(n) || BE64(c0))
 *            verifySignedKES hotVk t bhbody kesSig
 *   OVERLAY: verifyCertified vrfVk (mkSeed seedEta slot eta0) etaCert
 *            verifyCertified vrfVk (mkSeed seedL   slot eta0) leaderCert
 *   PRTCL:   eta = mkNonceFromOutputVRF (certifiedOutput etaCert) for UPDN
 * Claimed outputs: the reference's verifyCertified checks the proof only and
 * uses the header's certifiedOutput downstream (leader check at
 * Shelley/Protocol.hs:484-486, chain selection at Shelley/Ledger/TPraos.hs:40,
 * the nonce); the CLAIM bits say whether it equals the computed output.
 * The non-crypto checks (counters, KES window, VRF key hash, leader threshold)
 * are outside the hot path and not restated here.
 */
#include "internal.h"
#include <string.h>

static void be64(uint8_t *p, uint64_t v) {
  for (int i = 7; i >= 0; i--) { p[i] = (uint8_t)v; v >>= 8; }
}

void orc_mk_nonce_from_number(uint8_t out[32], uint64_t k) {
  uint8_t b[8];
  be64(b, k);
  orc_blake2b_256(out, b, 8);
}

void orc_mk_seed(uint8_t out[32], const uint8_t *uc, uint64_t slot, const uint8_t *eta0) {
  uint8_t m[40];
  be64(m, slot);
  if (eta0) memcpy(m + 8, eta0, 32);
  orc_blake2b_256(out, m, eta0 ? 40 : 8);
  if (uc)
    for (int k = 0; k < 32; k++) out[k] ^= uc[k];
}

void orc_tpraos_verify_one(const orc_tpraos_batch *b, size_t i, uint8_t *verdict,
                           uint8_t beta_eta[64], uint8_t beta_leader[64]) {
  uint8_t v = 0;
  uint8_t msg[48];
  memcpy(msg, b->hot_vk + 32 * i, 32);
  be64(msg + 32, b->ocert_counter[i]);
  be64(msg + 40, b->ocert_kes_period[i]);
  if (orc_ed25519_verify(b->ocert_sigma + 64 * i, msg, 48, b->issuer_vk + 32 * i) == 0)
    v |= ORC_HDR_OCERT_OK;
  if (orc_sum6kes_verify(b->hot_vk + 32 * i, b->kes_t[i], b->body + b->body_off[i],
                         b->body_len[i], b->kes_sig + ORC_KES_SIGBYTES * i) == 0)
    v |= ORC_HDR_KES_OK;
  /* OVERLAY's VRF inputs: mkSeed seedEta / seedL slot eta0, seedEta =
   * mkNonceFromNumber 0, seedL = mkNonceFromNumber 1 (ledger-specs
   * BlockChain.hs), or the caller's alphas */
  uint8_t ae[32], al[32];
  if (b->slot) {
    uint8_t se[32], sl[32];
    orc_mk_nonce_from_number(se, 0);
    orc_mk_nonce_from_number(sl, 1);
    orc_mk_seed(ae, se, b->slot[i], b->epoch_nonce);
    orc_mk_seed(al, sl, b->slot[i], b->epoch_nonce);
  } else {
    memcpy(ae, b->eta_alpha + 32 * i, 32);
    memcpy(al, b->leader_alpha + 32 * i, 32);
  }
  memset(beta_eta, 0, 64);
  memset(beta_leader, 0, 64);
  if (orc_vrf03_verify(beta_eta, b->vrf_vk + 32 * i, b->eta_proof + 80 * i, ae, 32) == 0) {
    v |= ORC_HDR_VRF_ETA_OK;
    if (b->eta_output && memcmp(b->eta_output + 64 * i, beta_eta, 64) == 0)
      v |= ORC_HDR_ETA_CLAIM_OK;
  }
  if (orc_vrf03_verify(beta_leader, b->vrf_vk + 32 * i, b->leader_proof + 80 * i, al, 32) == 0) {
    v |= ORC_HDR_VRF_LEADER_OK;
    if (b->leader_output && memcmp(b->leader_output + 64 * i, beta_leader, 64) == 0)
      v |= ORC_HDR_LEADER_CLAIM_OK;
  }
  /* PRTCL: eta = mkNonceFromOutputVRF (certifiedOutput bheaderEta) -- the
   * CLAIMED output -- = Blake2b-256 of its 64 bytes; without claimed outputs,
   * of the computed one */
  if (b->eta_nonce)
    orc_blake2b_256(b->eta_nonce + 32 * i, b->eta_output ? b->eta_output + 64 * i : beta_eta, 64);
  /* App. B.3 flag: s not reduced mod L, whatever the verdict */
  if (!sc_is_canonical(b->eta_proof + 80 * i + 48)) v |= ORC_HDR_ETA_S_UNREDUCED;
  if (!sc_is_canonical(b->leader_proof + 80 * i + 48)) v |= ORC_HDR_LEADER_S_UNREDUCED;
  *verdict = v;
}
