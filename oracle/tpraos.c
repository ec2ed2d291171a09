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
 * The non-crypto checks (counters, KES window, VRF key hash, leader threshold)
 * are outside the hot path and not restated here.
 */
#include "internal.h"
#include <string.h>

static void be64(uint8_t *p, uint64_t v) {
  for (int i = 7; i >= 0; i--) { p[i] = (uint8_t)v; v >>= 8; }
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
  memset(beta_eta, 0, 64);
  memset(beta_leader, 0, 64);
  if (orc_vrf03_verify(beta_eta, b->vrf_vk + 32 * i, b->eta_proof + 80 * i,
                       b->eta_alpha + 32 * i, 32) == 0)
    v |= ORC_HDR_VRF_ETA_OK;
  if (orc_vrf03_verify(beta_leader, b->vrf_vk + 32 * i, b->leader_proof + 80 * i,
                       b->leader_alpha + 32 * i, 32) == 0)
    v |= ORC_HDR_VRF_LEADER_OK;
  *verdict = v;
}
