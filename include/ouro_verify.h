/*
 * ouro_verify.h -- C-ABI drop-in boundary of the MI355X (gfx950) batch verifier
 * for the Ouroboros Praos/TPraos header-crypto hot path.
 *
 * The reference (dizgotti/ouroboros-network) reaches this arithmetic through
 * cardano-crypto-class / cardano-crypto-praos, whose Haskell instances bind C
 * symbols with `foreign import ccall`.  Each entry point below
 * names the reference interface it replaces.  Plain pointers and sizes only;
 * no HIP or torch types cross this boundary.
 *
 * Semantics shared by every call:
 *   - Return 0 = valid / OURO_OK, -1 = invalid (single-item calls), or a
 *     negative OURO_E* status for a call that could not run.  A device or
 *     runtime failure NEVER reports "valid" without a verification: a
 *     host-buffer call (single item, ouro_*_batch, header batches, plans)
 *     whose device run fails is recomputed on the library's host path -- the
 *     same lane routines the kernels run, compiled for the CPU -- and returns
 *     OURO_OK with those verdicts (ouro_last_error then says what failed);
 *     with OURO_ON_DEVICE_ERROR=fail in the environment it returns
 *     OURO_EDEVICE instead and leaves the verdicts untouched.  Device-pointer
 *     calls (*_batch_device) cannot be recomputed on the host and return
 *     OURO_EDEVICE.
 *   - Verdict bytes carry several bits: test them with masks, e.g.
 *     (v & OURO_HDR_ALL_OK) == OURO_HDR_ALL_OK, never with equality (a valid
 *     header may also carry OURO_HDR_*_CLAIM_OK or OURO_HDR_*_S_UNREDUCED).
 *   - The caller owns every buffer; nothing is retained after return.
 *   - All calls are thread-safe and reentrant: each calling thread gets its own
 *     HIP stream and staging buffers on the current device, borrowed from a
 *     per-device pool and returned when the thread exits (threads that come
 *     and go reuse them; nothing leaks per thread).
 *   - Byte layouts are the raw encodings of cardano-crypto-class:
 *     VerKeyDSIGN/VerKeyVRF/VerKeyKES 32 B, SigDSIGN 64 B, CertVRF (proof) 80 B,
 *     OutputVRF 64 B, SigKES (Sum6KES Ed25519DSIGN Blake2b_256) 448 B.
 */
#ifndef OURO_VERIFY_H
#define OURO_VERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OURO_OK 0
#define OURO_INVALID (-1)
#define OURO_EDEVICE (-2) /* HIP/runtime error; nothing was verified      */
#define OURO_EINVAL (-3)  /* bad arguments (NULL with n > 0, sizes, ...)  */
#define OURO_ENODEV (-4)  /* no usable gfx950 device                      */

/* Per-header verdict bits (ouro_tpraos_verify_batch). */
#define OURO_HDR_OCERT_OK 0x01u      /* Ed25519 over OCertSignable            */
#define OURO_HDR_KES_OK 0x02u        /* Sum6KES over the header body          */
#define OURO_HDR_VRF_ETA_OK 0x04u    /* nonce VRF proof                       */
#define OURO_HDR_VRF_LEADER_OK 0x08u /* leader VRF proof                      */
/* The header's claimed certifiedOutput equals the output computed from the
 * proof (set only when the proof verified and the batch carries the claimed
 * outputs).  The reference ("ref2020") accepts on the proof alone and then
 * uses the CLAIMED output downstream: the leader check
 * (ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:484-486,
 * SL.checkLeaderValue (VRF.certifiedOutput certNat)), the nonce update and the
 * chain-selection tiebreak (.../Shelley/Ledger/TPraos.hs:40).  "strict"
 * callers require these bits too (OURO_HDR_STRICT_OK). */
#define OURO_HDR_ETA_CLAIM_OK 0x10u
#define OURO_HDR_LEADER_CLAIM_OK 0x20u
#define OURO_HDR_ALL_OK 0x0fu    /* ref2020: every proof / signature valid    */
#define OURO_HDR_STRICT_OK 0x3fu /* strict: and both claimed outputs correct  */
/* Test verdicts with MASKS, never equality: valid(v) = (v & OURO_HDR_ALL_OK)
 * == OURO_HDR_ALL_OK, strict(v) = (v & OURO_HDR_STRICT_OK) == OURO_HDR_STRICT_OK
 * (a valid header may carry further bits, e.g. OURO_HDR_*_S_UNREDUCED). */
/* The VRF proof's s is NOT below L (set from the proof bytes alone, whatever
 * the verdict).  Draft-03 leaves s's range to the implementation; this
 * library, like the libsodium fork as SURVEY.md App. B.3 recalls it, reduces
 * s mod L and accepts (the default; parity of that choice is unpinned: no
 * reference fixture has s >= L).  A caller that must reject unreduced s
 * ("strict s") requires these bits CLEAR:
 *   valid_strict_s(v) = (v & (OURO_HDR_ALL_OK | OURO_HDR_S_UNREDUCED))
 *                       == OURO_HDR_ALL_OK */
#define OURO_HDR_ETA_S_UNREDUCED 0x40u
#define OURO_HDR_LEADER_S_UNREDUCED 0x80u
#define OURO_HDR_S_UNREDUCED 0xc0u

/* ------------------------------------------------------------------ setup */

/* Select the HIP device used by the calling thread (default: current device).
 * Returns OURO_OK or OURO_ENODEV. */
int ouro_set_device(int device);

/* Human-readable last error of the calling thread ("" if none). */
const char *ouro_last_error(void);

/* ----------------------------------------- single item (ABI-identical) --- */

/* Replaces libsodium 1.0.18 crypto_sign_ed25519_verify_detached, the symbol
 * cardano-crypto-class Ed25519DSIGN.verifyDSIGN binds (callers
 * ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:435 via
 * the OCERT rule, ouroboros-consensus-cardano/src/Ouroboros/Consensus/Cardano/
 * CanHardFork.hs:360).  0 = valid, -1 = invalid, <= -2 = error. */
int ouro_ed25519_verify(const unsigned char *sig, const unsigned char *m,
                        unsigned long long mlen, const unsigned char *pk);

/* Replaces the donna-derived Ed25519 verify of cardano-crypto
 * (cardano_crypto_ed25519_sign_open(m, mlen, pk, sig) [recalled], argument
 * order kept) that ByronDSIGN.verifyDSIGN reaches through verifySignatureRaw
 * (ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Crypto/DSIGN.hs:110-113;
 * callers ouroboros-consensus/src/Ouroboros/Consensus/Protocol/PBFT.hs:332 and
 * ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Ledger/Integrity.hs:32-35).
 * pk = the first 32 bytes of the 64-byte XPub; m = signTag || signable bytes.
 * Acceptance differs from ouro_ed25519_verify: rejects only
 * sig[63] & 0xE0 and an undecodable A -- no S < L, canonicity or small-order
 * checks.  0 = valid, -1 = invalid, <= -2 = error. */
int ouro_byron_ed25519_verify(const unsigned char *m, size_t mlen, const unsigned char *pk,
                              const unsigned char *sig);

/* Replaces crypto_vrf_ietfdraft03_verify (cardano-crypto-praos, bound by
 * PraosVRF.verifyVRF / verifyCertified; caller: OVERLAY vrfChecks via
 * Shelley/Protocol.hs:435).  On success writes the 64-byte output. */
int ouro_vrf03_verify(unsigned char *output, const unsigned char *pk,
                      const unsigned char *proof, const unsigned char *msg,
                      unsigned long long msglen);

/* Replaces crypto_vrf_ietfdraft03_proof_to_hash (VRF.certifiedOutput,
 * Shelley/Ledger/TPraos.hs:40).  Does not verify the proof. */
int ouro_vrf03_proof_to_hash(unsigned char *output, const unsigned char *proof);

/* Routing of single items.  The single-item calls above run on the library's
 * HOST path (the kernels' own lane routines compiled for the CPU; round 4):
 * one GPU round trip (H2D, one wave, D2H) costs about 220 us for Ed25519 and
 * 420 us for a VRF proof on MI355X, the host path about 1.5x libsodium's
 * ~32 us per Ed25519 on one core (bench.py "single_item" has both routes).
 * OURO_SINGLE_ITEM=gpu in the environment sends them to the device instead.
 * Windows of headers (ChainSync's 64-300, ouro_tpraos_plan_*) and bulk
 * batches (ouro_*_batch) are what the GPU path is for.  The names the
 * reference's Haskell binds are NOT exported by this library; two OPT-IN link
 * shims provide them, with these exact signatures, for a maintainer who
 * wants the drop-in by link order instead of a Haskell edit:
 *   lib/libouro_vrf_shim.so (PraosVRF's foreign imports; the version-less
 *   names are the fork's aliases of draft-03):
 *     int crypto_vrf_ietfdraft03_verify(unsigned char *output, const unsigned char *pk,
 *                                       const unsigned char *proof, const unsigned char *m,
 *                                       unsigned long long mlen);
 *     int crypto_vrf_ietfdraft03_proof_to_hash(unsigned char *output,
 *                                              const unsigned char *proof);
 *     int crypto_vrf_verify(...);         same as crypto_vrf_ietfdraft03_verify
 *     int crypto_vrf_proof_to_hash(...);  same as crypto_vrf_ietfdraft03_proof_to_hash
 *   lib/libouro_sodium_shim.so (Ed25519DSIGN.verifyDSIGN's libsodium symbol):
 *     int crypto_sign_ed25519_verify_detached(const unsigned char *sig,
 *                                             const unsigned char *m,
 *                                             unsigned long long mlen,
 *                                             const unsigned char *pk);
 * Those names follow libsodium's convention (any nonzero = invalid), so a
 * device error must not be passed through: the shims abort with the error on
 * stderr by default, or return -1 with OURO_SHIM_ON_ERROR=invalid. */

/* Replaces SumKES.verifyKES (Sum6KES Ed25519DSIGN Blake2b_256), called via
 * SL.verifySignedKES at ouroboros-consensus-shelley/src/Ouroboros/Consensus/
 * Shelley/Ledger/Integrity.hs:27.  t = KES period relative to the opcert.
 * The reference's Period is a 64-bit Word; every t >= 63 selects leaf 63, so
 * callers saturate larger periods at 2^32 - 1 (kes.py periods_u32). */
int ouro_sum6kes_verify(const unsigned char *vk, unsigned int t, const unsigned char *m,
                        unsigned long long mlen, const unsigned char *sig);

/* --------------------------------------------- batch, host buffers ------ */
/* H2D + kernel + D2H on the calling thread's stream; blocks until done.
 * Messages are addressed by (offset, length) into one buffer.
 * verdict[i] = 1 (valid) / 0 (invalid). */

int ouro_ed25519_verify_batch(size_t n, const uint8_t *pk /* n x 32 */,
                              const uint8_t *sig /* n x 64 */, const uint8_t *msg,
                              const uint64_t *msg_off, const uint32_t *msg_len,
                              uint8_t *verdict);

/* ByronDSIGN acceptance (see ouro_byron_ed25519_verify), pk = XPub[0:32] */
int ouro_byron_ed25519_verify_batch(size_t n, const uint8_t *pk /* n x 32 */,
                                    const uint8_t *sig /* n x 64 */, const uint8_t *msg,
                                    const uint64_t *msg_off, const uint32_t *msg_len,
                                    uint8_t *verdict);

/* beta[i] = 64-byte output on success, zeros otherwise */
int ouro_vrf03_verify_batch(size_t n, const uint8_t *pk /* n x 32 */,
                            const uint8_t *proof /* n x 80 */, const uint8_t *alpha,
                            const uint64_t *alpha_off, const uint32_t *alpha_len,
                            uint8_t *beta /* n x 64 */, uint8_t *verdict);
/* The same with option flags: OURO_VRF_STRICT_S rejects a proof whose s is
 * not below L (verdict 0, beta zeroed) instead of reducing it (the default,
 * see OURO_HDR_S_UNREDUCED). */
#define OURO_VRF_STRICT_S 0x1u
int ouro_vrf03_verify_batch_flags(size_t n, const uint8_t *pk, const uint8_t *proof,
                                  const uint8_t *alpha, const uint64_t *alpha_off,
                                  const uint32_t *alpha_len, uint8_t *beta, uint8_t *verdict,
                                  uint32_t flags);

int ouro_sum6kes_verify_batch(size_t n, const uint8_t *vk /* n x 32 */,
                              const uint32_t *t, const uint8_t *msg, const uint64_t *msg_off,
                              const uint32_t *msg_len, const uint8_t *sig /* n x 448 */,
                              uint8_t *verdict);

/* The crypto subset of SL.updateChainDepState for a batch of TPraos headers,
 * reached in the reference via TPraos.updateChainDepState
 * (ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:433-442):
 * OCERT (Ed25519 over hotVk || BE64(counter) || BE64(kesPeriod), then Sum6KES
 * over the raw header body) and OVERLAY (the eta and leader VRFs over
 * mkSeed seedEta/seedL slot eta0).  Structure-of-arrays, one entry per header.
 *
 * The first 16 members are required (eta_alpha / leader_alpha only when
 * `slot` is NULL).  The last five are optional -- NULL = not used; a caller
 * that zero-initialises the struct gets the round-1 behaviour:
 *   eta_output / leader_output: the header's claimed certifiedOutputs (the
 *     first element of bheaderEta / bheaderL); enables the *_CLAIM_OK bits.
 *   slot + epoch_nonce: the VRF inputs are derived on the device exactly as
 *     the OVERLAY rule does (Shelley/Protocol.hs:409-410, ledger-specs mkSeed):
 *       alpha = Blake2b-256(BE64(slot) || eta0) XOR seed,
 *       seedEta = Blake2b-256(BE64(0)), seedL = Blake2b-256(BE64(1))
 *     (mkNonceFromNumber 0 / 1); epoch_nonce = NULL is NeutralNonce (nothing
 *     appended after the slot).  eta_alpha / leader_alpha are then ignored.
 *     One eta0 per call: a window that crosses an epoch boundary is split.
 *   eta_nonce (OUTPUT, n x 32): mkNonceFromOutputVRF of the eta output the
 *     nonce update consumes = Blake2b-256(claimed eta output) when
 *     eta_output is given (the reference's choice), else of the computed
 *     beta_eta.  ouro_nonce_fold folds these into eta_v / eta_c. */
typedef struct ouro_tpraos_batch {
  size_t n;
  const uint8_t *issuer_vk;        /* n x 32  bheaderVk (cold key)            */
  const uint8_t *vrf_vk;           /* n x 32  bheaderVrfVk                    */
  const uint8_t *eta_proof;        /* n x 80  bheaderEta proof                */
  const uint8_t *leader_proof;     /* n x 80  bheaderL proof                  */
  const uint8_t *eta_alpha;        /* n x 32  mkSeed seedEta slot eta0        */
  const uint8_t *leader_alpha;     /* n x 32  mkSeed seedL   slot eta0        */
  const uint8_t *hot_vk;           /* n x 32  ocertVkHot (Sum6KES root)       */
  const uint64_t *ocert_counter;   /* n       ocertN                          */
  const uint64_t *ocert_kes_period;/* n       ocertKESPeriod (c0)             */
  const uint8_t *ocert_sigma;      /* n x 64  ocertSigma                      */
  const uint32_t *kes_t;           /* n       kesPeriod(slot) - c0, clamped   */
  const uint8_t *kes_sig;          /* n x 448 header KES signature            */
  const uint8_t *body;             /* concatenated raw header-body CBOR       */
  const uint64_t *body_off;        /* n                                       */
  const uint32_t *body_len;        /* n                                       */
  /* optional (NULL = not used) */
  const uint8_t *eta_output;       /* n x 64  claimed certifiedOutput (eta)   */
  const uint8_t *leader_output;    /* n x 64  claimed certifiedOutput (leader)*/
  const uint64_t *slot;            /* n       bheaderSlotNo: seeds on device  */
  const uint8_t *epoch_nonce;      /* 32      eta0 (NULL: NeutralNonce)       */
  uint8_t *eta_nonce;              /* n x 32  OUT: Blake2b-256(eta output)    */
} ouro_tpraos_batch;

/* verdict[i] = OURO_HDR_* bits; beta_eta / beta_leader (n x 64, may be NULL)
 * receive the computed VRF outputs (zeros where a proof fails). */
int ouro_tpraos_verify_batch(const ouro_tpraos_batch *b, uint8_t *verdict,
                             uint8_t *beta_eta, uint8_t *beta_leader);

/* Raw header CBOR -> the SoA above.  Replaces the
 * per-header decode the reference runs on every header ChainSync receives
 * (ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Ledger/Block.hs:216-217,
 * the Annotator keeping the raw header_body bytes; N2N wrapping at
 * .../Shelley/Node/Serialisation.hs:88-90) with one host call per batch.
 * Header i is raw[off[i] .. off[i] + len[i]) as it came off the wire:
 *   #6.24(bytes .cbor [header_body, kes_sig])             (N2N v1), or
 *   [era, #6.24(bytes .cbor [header_body, kes_sig])]      (Cardano HFC, era >= 1)
 * header_body = [blockNo, slot, prevHash, issuerVk, vrfVk, [etaOut, etaProof],
 * [leaderOut, leaderProof], bodySize, bodyHash, hotVk, counter, kesPeriod,
 * sigma, protMajor, protMinor] (ouroboros-network/test/messages.cddl:27-34).
 * The fixed-size fields are copied into `arena` (ouro_tpraos_pack_bytes(n)
 * bytes, any alignment) and *out's required members and eta_output /
 * leader_output (the claimed outputs) are pointed at them; body = raw and
 * body_off / body_len are the header_body spans inside raw (the KES message,
 * not copied); kes_t = kesPeriod(slot) - kesPeriod, clamped at 0 and saturated
 * at 2^32 - 1 (Integrity.hs:38-44).  eta_alpha / leader_alpha / slot /
 * epoch_nonce / eta_nonce are left to the caller (set out->slot = slot and
 * epoch_nonce to have the device derive the VRF inputs).  slot / era (n
 * each, may be NULL) receive bheaderSlotNo and the HFC era (1 if unwrapped).
 * status[i] = OURO_PACK_*; a rejected header's rows are zero (every verdict
 * bit then fails).  nthreads <= 0: one per hardware thread (at least 4096
 * headers each).  Host-only.  Returns OURO_OK, or OURO_EINVAL for bad
 * arguments (a span outside raw_bytes, a short arena, NULLs). */
#define OURO_PACK_OK 0u
#define OURO_PACK_ECBOR 1u  /* malformed or truncated CBOR                    */
#define OURO_PACK_ESHAPE 2u /* not the header shape (tag 24, [body, sig], 15
                               fields, [output, proof] certs, uint/bytes types) */
#define OURO_PACK_ESIZE 3u  /* a fixed-size crypto field has the wrong length  */
#define OURO_PACK_EBYRON 4u /* HFC era 0: a Byron header, not TPraos          */
#define OURO_PACK_ESPAN 5u  /* (device slicer) span outside raw_bytes          */
#define OURO_PACK_EBB 6u    /* (Byron slicer) an epoch-boundary header: PBFT
                               checks no signature on it (PBFT.hs:327-328)     */
#define OURO_PACK_ESHELLEY 7u /* (Byron slicer) HFC era >= 1: not a Byron header */
size_t ouro_tpraos_pack_bytes(size_t n);
int ouro_tpraos_pack_cbor(const uint8_t *raw, size_t raw_bytes, const uint64_t *off,
                          const uint32_t *len, size_t n, uint64_t slots_per_kes_period,
                          void *arena, size_t arena_bytes, ouro_tpraos_batch *out,
                          uint64_t *slot, uint8_t *era, uint8_t *status, int nthreads);
/* The same slicer on the GPU, one lane per header, for raw headers already in
 * device memory (raw, off, len, arena, slot, era, status: device pointers;
 * slot / era may be NULL): enqueued on `stream` and returns at once; *out
 * receives device pointers into the arena, ready for
 * ouro_tpraos_verify_batch_device on the same stream.  A span outside
 * raw_bytes is per-header status OURO_PACK_ESPAN.  Same parse code as the
 * host slicer (csrc/cbor.h); tests/test_gpu_pack.py checks the two agree. */
int ouro_tpraos_pack_cbor_device(void *stream, const uint8_t *raw, size_t raw_bytes,
                                 const uint64_t *off, const uint32_t *len, size_t n,
                                 uint64_t slots_per_kes_period, void *arena, size_t arena_bytes,
                                 ouro_tpraos_batch *out, uint64_t *slot, uint8_t *era,
                                 uint8_t *status);

/* Storage integrity, KES only, straight from raw header CBOR: replaces
 * verifyHeaderIntegrity (ouroboros-consensus-shelley/src/Ouroboros/Consensus/
 * Shelley/Ledger/Integrity.hs:20-44) as the storage layer runs it on every
 * block -- the VolatileDB parser at open
 * (ouroboros-consensus/src/Ouroboros/Consensus/Storage/VolatileDB/Impl/Parser.hs:66-85)
 * and ImmutableDB chunk validation
 * (.../Storage/ImmutableDB/Impl/Validation.hs:358-365).  Headers as for
 * ouro_tpraos_pack_cbor; verdict[i] = 1 iff header i slices (status
 * OURO_PACK_OK) and its Sum6KES signature verifies over the raw header body
 * under the opcert's hot key at t = kesPeriod(slot) - c0 (0 when the slot's
 * period is below c0; Integrity.hs:38-44).  Host buffers (pageable is fine),
 * synchronous; runs on the raw-CBOR pipeline described at
 * ouro_tpraos_verify_cbor (a device error recomputes on the host path).
 * OURO_EINVAL for a span outside raw_bytes, NULLs or a zero period. */
int ouro_integrity_verify_cbor(const uint8_t *raw, size_t raw_bytes, const uint64_t *off,
                               const uint32_t *len, size_t n, uint64_t slots_per_kes_period,
                               uint8_t *status, uint8_t *verdict);
/* Raw TPraos headers in host memory -> the full header check in ONE call:
 * the crypto of TPraos.updateChainDepState (ouroboros-consensus-shelley/src/
 * Ouroboros/Consensus/Shelley/Protocol.hs:433-442) over every header of a
 * batch the caller holds as the raw bytes it received or stored -- ChainSync
 * windows (ouroboros-consensus/src/Ouroboros/Consensus/MiniProtocol/ChainSync/
 * Client.hs:792) and ChainDB's re-validation of a stored chain suffix
 * (.../Storage/ChainDB/Impl/LgrDB.hs:350-368).  Headers as for
 * ouro_tpraos_pack_cbor (raw may be pageable, any offsets and order).
 * VRF inputs: eta_alpha / leader_alpha (n x 32 each) when both are given,
 * otherwise derived on the device from each header's slot as the OVERLAY rule
 * does (mkSeed seedEta / seedL slot eta0, see ouro_tpraos_batch), with
 * epoch_nonce = eta0 (32 B; NULL = NeutralNonce; one eta0 per call).  The
 * headers' claimed certifiedOutputs are compared (OURO_HDR_*_CLAIM_OK).
 * Outputs: status[i] = OURO_PACK_*; verdict[i] = OURO_HDR_* bits, 0 for a
 * header that does not slice; beta_eta / beta_leader (n x 64) and eta_nonce
 * (n x 32, Blake2b-256 of the claimed eta output) may be NULL.
 * How it runs: the batch is cut into chunks of whole headers; the library's
 * worker pool gathers each chunk's spans into pinned, NUMA-local staging,
 * and per chunk one stream uploads the raw bytes, runs the device slicer
 * and the header kernel and copies the results back, several chunks in
 * flight so the host copies and PCIe hide behind the kernels
 * (OURO_CBOR_CHUNK headers per chunk, default 65536; OURO_CBOR_SLOTS chunks
 * in flight, default 6 -- 4 for ouro_integrity_verify_cbor --, at most 8;
 * OURO_CBOR_COPY_THREADS gather threads, default 8).  Synchronous; a device error recomputes the batch on the host
 * path.  OURO_EINVAL for a span outside raw_bytes, NULLs, a zero period or
 * only one of the two alpha arrays.
 * Footprint: the pipeline's buffers belong to the calling
 * thread's pooled context and are kept for its next call -- per slot pinned
 * staging of ~1.125 x the chunk's raw bytes, device buffers for the raw
 * bytes, the slicer's arena and the results, and the kernel's scratch; at the
 * default 65,536-header chunk of ~1 KB headers about 75 MB pinned and 180 MB
 * of device memory per slot in use (6 slots for headers, 4 for integrity),
 * once per context that has made such a call.  OURO_CBOR_CHUNK and
 * OURO_CBOR_SLOTS shrink it. */
int ouro_tpraos_verify_cbor(const uint8_t *raw, size_t raw_bytes, const uint64_t *off,
                            const uint32_t *len, size_t n, uint64_t slots_per_kes_period,
                            const uint8_t *epoch_nonce, const uint8_t *eta_alpha,
                            const uint8_t *leader_alpha, uint8_t *status, uint8_t *verdict,
                            uint8_t *beta_eta, uint8_t *beta_leader, uint8_t *eta_nonce);
/* The same on raw headers already in device memory (device pointers; arena
 * of ouro_tpraos_pack_bytes(n) bytes): the device slicer and the Sum6KES
 * kernel enqueued on `stream`, not synchronised.  A rejected header's row is
 * zeroed by the slicer, so its verdict is 0. */
int ouro_integrity_verify_cbor_device(void *stream, const uint8_t *raw, size_t raw_bytes,
                                      const uint64_t *off, const uint32_t *len, size_t n,
                                      uint64_t slots_per_kes_period, void *arena,
                                      size_t arena_bytes, uint8_t *status, uint8_t *verdict);

/* Raw Byron header CBOR -> the inputs of its PBFT block-signature check
 * (SURVEY.md §8(f) row 4).  Replaces the per-header decode + message assembly
 * in front of ByronDSIGN.verifyDSIGN: Byron/Ledger/PBFT.hs:47-73 builds
 * PBftFields and recoverSignedBytes from the decoded header, PBFT.hs:332-337
 * verifies them (caller: ChainSync's validateHeader; Integrity.hs:32-35 from
 * storage).  Header i is raw[off[i] .. off[i] + len[i]) in any of the forms
 * the reference sends (Byron/Node/Serialisation.hs:87-101, 197-210):
 *   #6.24(bytes .cbor [kind, header])                      Byron / Cardano N2N v1
 *   [[kind, size], #6.24(bytes .cbor header)]              Byron N2N v2
 *   [0, [[kind, size], #6.24(bytes .cbor header)]]         Cardano N2N v2+
 * kind 1 = regular, 0 = epoch boundary (status OURO_PACK_EBB: no signature,
 * fields unchecked).  For a regular header the batch receives pk =
 * delegateXPub[0:32] (pbftIssuer), sig, genesis_vk = the delegation
 * certificate's issuer XPub (pbftGenKey), delegate_vk, the header's
 * protocol magic, and the signed message
 *   "01" || genesis_vk || 0x09 || CBOR(magic) || 0x85 || prevHash || bodyProof
 *   || slotId || difficulty || extraData                    (raw field bytes)
 * at msg + msg_off[i] (msg_len[i] bytes), magic = protocol_magic (the node's
 * ProtocolMagicId, mkByronContextDSIGN at Byron/Ledger/PBFT.hs:43-44) or,
 * for protocol_magic = -1, each header's own field.  The arena holds all of
 * it: ouro_byron_pack_bytes(n, len) bytes, any alignment.  status[i] =
 * OURO_PACK_* (OK, ECBOR, ESHAPE, ESIZE, EBB, ESHELLEY); rows of other
 * statuses are zero with msg_len 0.  nthreads as for ouro_tpraos_pack_cbor.
 * Host-only.  OURO_EINVAL for a span outside raw_bytes, a short arena, a
 * protocol_magic outside -1 .. 2^32 - 1, NULLs. */
typedef struct {
  size_t n;
  const uint8_t *pk;          /* n x 32  delegate XPub[0:32]                  */
  const uint8_t *sig;         /* n x 64  block signature                      */
  const uint8_t *msg;         /* signed messages                              */
  const uint64_t *msg_off;    /* n       offsets into msg                     */
  const uint32_t *msg_len;    /* n                                            */
  const uint8_t *genesis_vk;  /* n x 64  delegation certificate issuer XPub   */
  const uint8_t *delegate_vk; /* n x 64  delegate XPub                        */
  const uint64_t *magic;      /* n       the header's protocolMagic field     */
} ouro_byron_batch;
size_t ouro_byron_pack_bytes(size_t n, const uint32_t *len);
int ouro_byron_pack_cbor(const uint8_t *raw, size_t raw_bytes, const uint64_t *off,
                         const uint32_t *len, size_t n, int64_t protocol_magic, void *arena,
                         size_t arena_bytes, ouro_byron_batch *out, uint8_t *status,
                         int nthreads);
/* Raw Byron headers -> verdicts in one call: ouro_byron_pack_cbor, then the
 * ByronDSIGN batch verify of the packed rows on the calling thread's stream.
 * verdict[i] = 1 for a regular header whose block signature verifies and for
 * an epoch-boundary header (PBftValidateBoundary checks nothing), else 0;
 * status[i] as above.  The delegation lookup and the signing-window
 * threshold (PBFT.hs:344-357) stay with the caller: they are ledger state,
 * not crypto. */
int ouro_byron_verify_cbor(const uint8_t *raw, size_t raw_bytes, const uint64_t *off,
                           const uint32_t *len, size_t n, int64_t protocol_magic,
                           uint8_t *status, uint8_t *verdict);
/* (How ouro_byron_verify_cbor runs, since round 6: on the raw-CBOR pipeline
 * of ouro_tpraos_verify_cbor -- chunks gathered into pinned NUMA-local
 * staging, the device Byron slicer (the same cbor_byron.h parse as
 * ouro_byron_pack_cbor) and the ByronDSIGN Ed25519 kernel per chunk, 5
 * chunks in flight; a device error recomputes the batch on the host path.
 * OURO_EINVAL as for ouro_byron_pack_cbor.) */

/* Byron heavyweight delegation certificates (the "Byron delegation" use of
 * DSIGN in the north star): a certificate (epoch, issuer XPub, delegate XPub,
 * signature) -- cardano-ledger-byron's Delegation.Certificate [ext], the
 * reference's PBftDelegationCert (ouroboros-consensus-byron/src/Ouroboros/
 * Consensus/Byron/Protocol.hs:30) and the mempool's ByronDlg payload
 * (.../Byron/Ledger/Mempool.hs:90), whose signature the ledger checks under
 * the issuer's key with the SignCertificate tag.  Signed bytes, pinned on the
 * certificate inside the reference's golden Byron header
 * (tests/test_byron_cert.py):
 *   0x0a || CBOR(protocol_magic) || CBOR bytes("00" || delegate XPub || CBOR(epoch))
 * Key = issuer XPub[0:32]; ByronDSIGN acceptance (ouro_byron_ed25519_verify).
 * _message writes those bytes (at most OURO_BYRON_DLG_MSG_MAX) and returns
 * their length (0 for NULL arguments); _verify is one certificate on the
 * host path (0 / -1 / <= -2 as ouro_byron_ed25519_verify); _verify_batch
 * builds the n messages and runs ouro_byron_ed25519_verify_batch
 * (verdict[i] = 1 / 0). */
#define OURO_BYRON_DLG_MSG_MAX 96
size_t ouro_byron_dlg_cert_message(uint8_t *out, uint32_t protocol_magic,
                                   const uint8_t *delegate_xpub /* 64 */, uint64_t epoch);
int ouro_byron_dlg_cert_verify(uint32_t protocol_magic, const uint8_t *issuer_xpub /* 64 */,
                               const uint8_t *delegate_xpub /* 64 */, uint64_t epoch,
                               const uint8_t *sig /* 64 */);
int ouro_byron_dlg_cert_verify_batch(size_t n, uint32_t protocol_magic,
                                     const uint8_t *issuer_xpub /* n x 64 */,
                                     const uint8_t *delegate_xpub /* n x 64 */,
                                     const uint64_t *epoch, const uint8_t *sig /* n x 64 */,
                                     uint8_t *verdict);

/* The host-side UPDN fold (ledger-specs; the per-header step of
 * SL.updateChainDepState after the crypto): for i = 0..n-1
 *   eta_v <- eta_v (*) eta_nonce[i]
 *   eta_c <- eta_v            if slot[i] + stability_window < first_slot_next_epoch
 *            (unchanged)      otherwise
 * with a (*) b = Blake2b-256(a || b) (Nonce composition; the 32-byte values are
 * Nonce hashes).  The caller stops at the first invalid header itself (pass
 * n = that index).  eta_v / eta_c are updated in place (32 B each);
 * is_neutral[0..1] (may be NULL) say eta_v / eta_c start as NeutralNonce and
 * receive whether they still are.  Host-only, no device.  Returns OURO_OK. */
int ouro_nonce_fold(size_t n, const uint8_t *eta_nonce, const uint64_t *slot,
                    uint64_t first_slot_next_epoch, uint64_t stability_window,
                    uint8_t *eta_v, uint8_t *eta_c, int *is_neutral);

/* Latency-oriented variant for small batches (ChainSync windows of up to 300
 * pipelined headers, ouroboros-network/src/Ouroboros/Network/NodeToNode.hs:197-200):
 * the checks of a header run on eight lanes concurrently (each VRF's
 * V = [s]H - [c]Gamma split over two), then one finish pass.  Same verdicts and outputs as ouro_tpraos_verify_batch. */
int ouro_tpraos_verify_batch_lowlat(const ouro_tpraos_batch *b, uint8_t *verdict,
                                    uint8_t *beta_eta, uint8_t *beta_leader);

/* One process, several GPUs: the batch is cut into
 * contiguous shards, shard k verified on devices[k] (devices = NULL: every
 * visible device) by a persistent worker thread -- one per (device, k-th
 * listing of that device) -- with its own streams and pinned staging (the
 * pipelined path of ouro_tpraos_verify_batch), writing straight into the
 * caller's buffers (no collective is needed inside one process).  A device
 * may be listed more than once (two pipelines on one GPU).  The workers are
 * pooled per device: a call borrows one per shard and returns it when every
 * shard has finished, so concurrent callers (ChainSync windows beside
 * ChainDB's suffix re-validation) run at once on workers of their own --
 * nothing is serialised process-wide since round 6.  The first shard error
 * is returned after every shard has finished (a shard's device error is
 * recomputed on the host path like any host-buffer batch).  Same results as
 * ouro_tpraos_verify_batch. */
int ouro_device_count(void);
/* NUMA placement (each GPU's pinned staging NUMA-local).
 * ouro_device_numa_node: the node of the device's PCI function in sysfs
 * (-1 unknown; OURO_ENODEV for a bad index).  ouro_bind_thread_to_device:
 * restricts the calling thread to that node's CPUs (within the process's
 * cpuset) and prefers its memory, so the pinned staging the thread allocates
 * afterwards lands there; returns the node or -1 (left alone).  The workers of
 * ouro_tpraos_verify_batch_multi bind themselves to their device's node; all
 * pinned staging is allocated with hipHostMallocNumaUser (the allocating
 * thread's policy).  ouro_debug_multi_workers: per worker its device, node and
 * the CPUs it is bound to (0 = unbound; declared in ouro_verify_debug.h). */
int ouro_device_numa_node(int device);
int ouro_bind_thread_to_device(int device);
int ouro_tpraos_verify_batch_multi(const ouro_tpraos_batch *b, const int *devices, int ndev,
                                   uint8_t *verdict, uint8_t *beta_eta, uint8_t *beta_leader);
/* The raw-CBOR entries over several GPUs of one process -- what the bulk
 * callers of an 8-GPU node hold: ChainDB's re-validation of a stored suffix
 * (ouroboros-consensus/src/Ouroboros/Consensus/Storage/ChainDB/Impl/
 * LgrDB.hs:350-368) and ImmutableDB / VolatileDB integrity
 * (.../Storage/ImmutableDB/Impl/Validation.hs:358-365,
 * .../Storage/VolatileDB/Impl/Parser.hs:66-85).  Arguments and results as
 * ouro_tpraos_verify_cbor / ouro_integrity_verify_cbor /
 * ouro_byron_verify_cbor, plus the device list (NULL: every visible
 * device; a device may be listed more than once).  Headers are cut into
 * contiguous shards of ceil(n / ndev), shard k runs the one-device pipeline
 * (chunks, pinned NUMA-local staging, several chunks in flight) on a pooled
 * worker of devices[k] bound to that GPU's NUMA node, and writes straight into
 * the caller's buffers.  Every span is checked before any shard starts
 * (OURO_EINVAL); OURO_ENODEV for a device index outside the visible ones. */
int ouro_tpraos_verify_cbor_multi(const int *devices, int ndev, const uint8_t *raw,
                                  size_t raw_bytes, const uint64_t *off, const uint32_t *len,
                                  size_t n, uint64_t slots_per_kes_period,
                                  const uint8_t *epoch_nonce, const uint8_t *eta_alpha,
                                  const uint8_t *leader_alpha, uint8_t *status, uint8_t *verdict,
                                  uint8_t *beta_eta, uint8_t *beta_leader, uint8_t *eta_nonce);
int ouro_integrity_verify_cbor_multi(const int *devices, int ndev, const uint8_t *raw,
                                     size_t raw_bytes, const uint64_t *off, const uint32_t *len,
                                     size_t n, uint64_t slots_per_kes_period, uint8_t *status,
                                     uint8_t *verdict);
int ouro_byron_verify_cbor_multi(const int *devices, int ndev, const uint8_t *raw,
                                 size_t raw_bytes, const uint64_t *off, const uint32_t *len,
                                 size_t n, int64_t protocol_magic, uint8_t *status,
                                 uint8_t *verdict);

/* A plan for repeated fixed-capacity batches: pinned staging, device buffers
 * and the latency kernel's launch shape fixed at create; each run issues the
 * window's input copy kernel and the fused latency kernel on the plan's own
 * stream (OURO_PLAN_GRAPH=1 at create: replayed from one captured hipGraph
 * instead).  A plan is used by one thread at a time; any n <= max_headers per
 * run. */
typedef struct ouro_tpraos_plan ouro_tpraos_plan;
ouro_tpraos_plan *ouro_tpraos_plan_create(size_t max_headers, size_t max_body_bytes);
int ouro_tpraos_plan_run(ouro_tpraos_plan *plan, const ouro_tpraos_batch *b, uint8_t *verdict,
                         uint8_t *beta_eta, uint8_t *beta_leader);
void ouro_tpraos_plan_destroy(ouro_tpraos_plan *plan);

/* Asynchronous form of ouro_tpraos_plan_run for pipelined ChainSync windows
 * (SURVEY.md §8(b) "Async": a client keeps up to 300 headers in flight,
 * ouroboros-network/src/Ouroboros/Network/NodeToNode.hs:197-200, and
 * validates each window as its headers arrive,
 * ouroboros-consensus/src/Ouroboros/Consensus/MiniProtocol/ChainSync/Client.hs:792).
 * submit copies the batch into the plan's pinned staging and launches its
 * kernels, returning at once (the caller's input buffers are free again on
 * return); wait blocks until that batch's results are in the caller's buffers.
 * One batch in flight per plan: a second submit before wait, or a wait with
 * nothing submitted, returns OURO_EINVAL.  Several plans = several windows in
 * flight, each on its own stream. */
int ouro_tpraos_plan_submit(ouro_tpraos_plan *plan, const ouro_tpraos_batch *b);
int ouro_tpraos_plan_wait(ouro_tpraos_plan *plan, uint8_t *verdict, uint8_t *beta_eta,
                          uint8_t *beta_leader);

/* (A plan's latency kernel counts each header's finished checks in
 * per-header arrival counters tagged with the launch's generation -- a new
 * one per submit -- so a counter an earlier launch left mid-count, one that
 * never completed, is never counted again; tests/test_gpu_claims.py checks it
 * through a test hook reached only from the environment.) */

/* ------------------------------------------------------- host path ----- */
/* The same batches on the library's host path, explicitly: the kernels' own
 * lane routines compiled for the CPU (csrc/host_path.hip), the batch split
 * over host threads (OURO_HOST_THREADS caps them; default the CPUs the
 * process may run on, at most 64).  Same arguments, verdicts and outputs as
 * the calls without _host; no device is touched.  For nodes without a GPU,
 * for callers that keep small batches on the CPU, and the path the device
 * calls recompute on after a device error. */
int ouro_ed25519_verify_batch_host(size_t n, const uint8_t *pk, const uint8_t *sig,
                                   const uint8_t *msg, const uint64_t *msg_off,
                                   const uint32_t *msg_len, uint8_t *verdict);
int ouro_byron_ed25519_verify_batch_host(size_t n, const uint8_t *pk, const uint8_t *sig,
                                         const uint8_t *msg, const uint64_t *msg_off,
                                         const uint32_t *msg_len, uint8_t *verdict);
int ouro_vrf03_verify_batch_host(size_t n, const uint8_t *pk, const uint8_t *proof,
                                 const uint8_t *alpha, const uint64_t *alpha_off,
                                 const uint32_t *alpha_len, uint8_t *beta, uint8_t *verdict,
                                 uint32_t flags);
int ouro_sum6kes_verify_batch_host(size_t n, const uint8_t *vk, const uint32_t *t,
                                   const uint8_t *msg, const uint64_t *msg_off,
                                   const uint32_t *msg_len, const uint8_t *sig, uint8_t *verdict);
int ouro_tpraos_verify_batch_host(const ouro_tpraos_batch *b, uint8_t *verdict,
                                  uint8_t *beta_eta, uint8_t *beta_leader);
int ouro_leader_check_batch_host(size_t n, const uint8_t *beta, const uint64_t *sigma_num,
                                 const uint64_t *sigma_den, int64_t act_log_hi,
                                 uint64_t act_log_lo, int f_is_one, uint8_t *verdict);

/* ---------------------------------------------- leader threshold ----- */
/* ledger-specs checkLeaderValue (shelley-spec-ledger BlockChain.hs), called by
 * meetsLeaderThreshold, ouroboros-consensus-shelley/src/Ouroboros/Consensus/
 * Shelley/Protocol.hs:473-491: is the leader VRF output beta (64 B) below
 * 1 - (1 - f)^sigma, decided with shelley-spec-non-integral's taylorExpCmp in
 * 34-digit fixed point.  sigma = sigma_num[i] / sigma_den[i] (the pool's
 * relative stake, 0 <= sigma <= 1); f is given as its ActiveSlotCoeff fields:
 * unActiveSlotLog (a signed 128-bit integer, act_log_hi:act_log_lo; the
 * reference precomputes it from f) and whether f is exactly 1.
 * verdict[i] = OURO_LEADER_YES / OURO_LEADER_NO, or OURO_LEADER_BADARG when
 * sigma or unActiveSlotLog is outside the supported domain
 * (-8 * 10^34 <= unActiveSlotLog <= 0, i.e. f <= 1 - e^-8). */
#define OURO_LEADER_NO 0u
#define OURO_LEADER_YES 1u
#define OURO_LEADER_BADARG 0xffu
int ouro_leader_check_batch(size_t n, const uint8_t *beta, const uint64_t *sigma_num,
                            const uint64_t *sigma_den, int64_t act_log_hi,
                            uint64_t act_log_lo, int f_is_one, uint8_t *verdict);

/* ----------------------------------- batch, device-resident buffers ----- */
/* Same kernels on caller-owned device memory, enqueued on `stream` (a
 * hipStream_t; NULL = HIP's default stream) and NOT synchronised: the caller
 * orders its own copies/events around them.  `msg_off`/`msg_len` etc. are
 * device pointers too.  Used by bench.py (inputs resident in HBM) and by
 * pipelined callers that overlap H2D of the next window with this one. */

int ouro_ed25519_verify_batch_device(void *stream, size_t n, const uint8_t *pk,
                                     const uint8_t *sig, const uint8_t *msg,
                                     const uint64_t *msg_off, const uint32_t *msg_len,
                                     uint8_t *verdict);
int ouro_byron_ed25519_verify_batch_device(void *stream, size_t n, const uint8_t *pk,
                                           const uint8_t *sig, const uint8_t *msg,
                                           const uint64_t *msg_off, const uint32_t *msg_len,
                                           uint8_t *verdict);
int ouro_vrf03_verify_batch_device(void *stream, size_t n, const uint8_t *pk,
                                   const uint8_t *proof, const uint8_t *alpha,
                                   const uint64_t *alpha_off, const uint32_t *alpha_len,
                                   uint8_t *beta, uint8_t *verdict);
int ouro_vrf03_verify_batch_device_flags(void *stream, size_t n, const uint8_t *pk,
                                         const uint8_t *proof, const uint8_t *alpha,
                                         const uint64_t *alpha_off, const uint32_t *alpha_len,
                                         uint8_t *beta, uint8_t *verdict, uint32_t flags);
int ouro_sum6kes_verify_batch_device(void *stream, size_t n, const uint8_t *vk,
                                     const uint32_t *t, const uint8_t *msg,
                                     const uint64_t *msg_off, const uint32_t *msg_len,
                                     const uint8_t *sig, uint8_t *verdict);
/* `b` is a host struct whose pointers are device pointers */
int ouro_tpraos_verify_batch_device(void *stream, const ouro_tpraos_batch *b,
                                    uint8_t *verdict, uint8_t *beta_eta,
                                    uint8_t *beta_leader);
int ouro_leader_check_batch_device(void *stream, size_t n, const uint8_t *beta,
                                   const uint64_t *sigma_num, const uint64_t *sigma_den,
                                   int64_t act_log_hi, uint64_t act_log_lo, int f_is_one,
                                   uint8_t *verdict);

#ifdef __cplusplus
}
#endif
#endif /* OURO_VERIFY_H */
