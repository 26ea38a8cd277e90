/*
 * bls381.h -- C ABI of the MI355X (gfx950) BLS12-381 engine.
 *
 * Drop-in boundary for the reference's BLS path: every entry point below is
 * what `test_libs/pyspec/eth2spec/utils/bls.py` (reference) would bind through
 * ctypes in place of `from py_ecc import bls` (bls.py:1).  The Python mirror of
 * that module is consensus-specs_amd/bls381_amd/bls.py; the binding a
 * maintainer would add to the reference is shown in INTEGRATION.md.
 *
 * Conventions
 *   - Plain pointers and sizes only; the caller owns every buffer.
 *   - Pubkeys are 48-byte compressed G1, signatures 96-byte compressed G2
 *     (specs/bls_signature.md:36-64).  Messages are `msg_len` bytes (the spec's
 *     message_hash is Bytes32; py_ecc hashes any length, so 0..BLS381_MSG_MAX is accepted).
 *   - `dom8` is the 8-byte serialisation of the spec's uint64 `domain`
 *     (hash_to_G2, bls_signature.md:76-77).  The int -> bytes step is done by
 *     the caller so the byte order has one switch.
 *   - Return codes: >= 0 success (verdicts 1/0), < 0 error (BLS381_E*).
 *   - Host-pointer entry points copy to/from the device internally.  The
 *     `_device` variants take device pointers and a hipStream_t (as void*).
 *   - There is no CPU fallback: without a usable gfx950 device every call
 *     returns BLS381_ENODEV.
 */
#ifndef BLS381_H
#define BLS381_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BLS381_OK 0
#define BLS381_EINVAL_POINT (-1) /* an input point encoding is invalid (aggregate raises ValueError) */
#define BLS381_EARG (-2)         /* bad argument (NULL, length) */
#define BLS381_ENODEV (-3)       /* no HIP device / kernels not loadable */
#define BLS381_EHIP (-4)         /* HIP runtime error */
#define BLS381_MSG_MAX (1u << 20) /* message bytes per call (hash_to_G2 streams the message) */

/* Subgroup policy of the verify paths (DESIGN.md "Subgroup policy").
 *   PYECC (default): the checks py_ecc 1.7.0 makes, which the reference calls
 *     (bls.py:24-31): decoding and the on-curve test only.  Torsion of order
 *     prime to r in a pubkey leaves the verdict unchanged, and a signature with
 *     no G2 component whose Miller loop degenerates gives False -- both as py_ecc.
 *   STRICT: every pubkey and signature must also lie in G1 / G2, the spec's
 *     "valid G1/G2 point" (specs/bls_signature.md:135-136,143-144).
 * Aggregation never checks subgroups (py_ecc's aggregate_* do not). */
#define BLS381_POLICY_PYECC 0
#define BLS381_POLICY_STRICT 1

/* ---- runtime ----------------------------------------------------------- */
/* Number of visible HIP devices (0 if none). */
int bls381_device_count(void);
/* Select the device used by subsequent calls from this thread and create its
 * context (stream, workspace).  Idempotent. */
int bls381_init(int device);
/* Create the contexts of devices 0 .. n_devices-1 (SURVEY §8(b)'s bls381_init(n_devices);
 * a process driving several GPUs then selects one per thread with bls381_init). */
int bls381_init_devices(int n_devices);
void bls381_shutdown(void);
/* Last HIP error string of this thread (static storage). */
const char* bls381_last_error(void);
/* Process-wide subgroup policy (BLS381_POLICY_*), read when a call is queued.
 * Returns 0, or BLS381_EARG for an unknown policy.  Needs no device. */
int bls381_set_subgroup_policy(int policy);
int bls381_get_subgroup_policy(void);
/* Policy override for calls queued from the calling thread only (-1 clears it and the
 * thread follows the process-wide policy again).  The Python shim (bls.py) scopes each
 * verify with its module switch this way, so it neither rewrites the process-wide policy
 * that other front ends read nor races with other threads.  Returns 0 or BLS381_EARG. */
int bls381_set_thread_subgroup_policy(int policy);
/* The policy calls queued from this thread use (the override if set). */
int bls381_get_thread_subgroup_policy(void);
/* Kernel-time accounting (HIP events on the launch stream) for bench.py. */
int bls381_profile_enable(int on);
int bls381_profile_read(char* json_out, size_t cap);

/* ---- eth2spec.utils.bls drop-ins (reference bls.py:24-46) -------------- */

/* bls_verify (bls.py:24-26; bls_signature.md:131-137).  1 = valid, 0 = invalid
 * (including undecodable inputs, as py_ecc's except-clause returns False). */
int bls381_verify(const uint8_t pk[48], const uint8_t* msg, size_t msg_len,
                  const uint8_t sig[96], const uint8_t dom8[8]);

/* bls_verify_multiple (bls.py:29-31; bls_signature.md:139-146).  n pubkeys and
 * n messages of msg_len bytes each; pubkeys sharing a message are aggregated
 * first (py_ecc grouping) and one final exponentiation decides the call. */
int bls381_verify_multiple(size_t n, const uint8_t* pks, const uint8_t* msgs, size_t msg_len,
                           const uint8_t sig[96], const uint8_t dom8[8]);

/* bls_aggregate_pubkeys (bls.py:34-36): sum of n G1 points; n == 0 -> infinity.
 * Returns BLS381_EINVAL_POINT if any input does not decode. */
int bls381_aggregate_pubkeys(size_t n, const uint8_t* pks, uint8_t out[48]);

/* bls_aggregate_signatures (bls.py:39-41): sum of n G2 points. */
int bls381_aggregate_signatures(size_t n, const uint8_t* sigs, uint8_t out[96]);
/* SURVEY §8(b)'s names for the two aggregations (same behaviour). */
int bls381_aggregate_g1(size_t n, const uint8_t* pks, uint8_t out[48]);
int bls381_aggregate_g2(size_t n, const uint8_t* sigs, uint8_t out[96]);

/* bls_sign (bls.py:44-46): [sk] hash_to_G2(msg, domain); sk 32-byte big-endian. */
int bls381_sign(const uint8_t* msg, size_t msg_len, const uint8_t sk[32], const uint8_t dom8[8],
                uint8_t out[96]);

/* py_ecc bls.privtopub (test_generators/bls/main.py:114; helpers/keys.py:5). */
int bls381_privtopub(const uint8_t sk[32], uint8_t out[48]);

/* Batched sign / privtopub over n items (32-byte messages, 32-byte big-endian
 * secret keys, per-item dom8) -- used to build synthetic verify batches. */
int bls381_sign_batch(size_t n, const uint8_t* msgs32, const uint8_t* sks, const uint8_t* dom8s, uint8_t* out96);
int bls381_privtopub_batch(size_t n, const uint8_t* sks, uint8_t* out48);

/* hash_to_G2 (bls_signature.md:74-87; main.py:71,84): compressed (96 B) and
 * normalised affine x_re,x_im,y_re,y_im (4 x 48 B big-endian).  Either output may be NULL. */
int bls381_hash_to_g2(const uint8_t* msg, size_t msg_len, const uint8_t dom8[8],
                      uint8_t out_compressed[96], uint8_t out_affine[192]);

/* py_ecc's un-normalised projective triple for hash_to_G2 (main.py:56-72,
 * msg_hash_g2_uncompressed vectors): X,Y,Z each (re, im), 6 x 48 B big-endian.
 * n messages of 32 bytes with per-message dom8. */
int bls381_hash_to_g2_pyecc_projective(size_t n, const uint8_t* msgs32, const uint8_t* dom8s,
                                       uint8_t* out288);

/* ---- batched entry points (the throughput path) ------------------------ */

/* n independent bls_verify calls: verdicts_out[i] = 1/0. */
int bls381_verify_batch(size_t n, const uint8_t* pks, const uint8_t* msgs32, const uint8_t* sigs,
                        const uint8_t* dom8s, uint8_t* verdicts_out);

/* Device-resident variant: all pointers are device memory, stream = hipStream_t
 * (NULL = the HIP null stream, i.e. torch's default stream; work is queued, not synchronised).
 * `workspace` must hold bls381_verify_batch_workspace_size(n) bytes. */
size_t bls381_verify_batch_workspace_size(size_t n);
int bls381_verify_batch_device(size_t n, const uint8_t* d_pks, const uint8_t* d_msgs32,
                               const uint8_t* d_sigs, const uint8_t* d_dom8s, uint8_t* d_verdicts,
                               void* d_workspace, void* stream);

/* Opt-in randomized batch verification of n independent bls_verify items (the
 * north star's "batched Miller loops share a single final exponentiation"; SURVEY
 * §7 "Verdict semantics under batching").  Items go in sub-batches of `batch`
 * (even, 2 <= batch <= 32768; otherwise BLS381_EARG, and the workspace size is 0); a
 * sub-batch passes when
 *     prod_i e(H(m_i), [r_i] pk_i) * e(sum_i [r_i] sig_i, -g1) == 1,
 * r_i = k0 + mu k1 mod r, mu = -x^2, (k1, k0) = the first 8 bytes of
 * SHA-256(seed || i) as two 32-bit words (seed: 32 caller-chosen random bytes; 2^64
 * distinct weights, applied through the endomorphisms sigma / -psi^2: [r_i] pk_i as a joint
 * 32-bit multiplication, sum_i [r_i] sig_i as one bucket multi-scalar multiplication per
 * sub-batch), with one final exponentiation.  Items of a passing sub-batch are
 * valid (a wrong one slips through with probability <= 2^-63); every item of a failing sub-batch,
 * and every item whose signature is outside G2, is re-verified alone by the
 * default pipeline, so verdicts are the per-item ones.  The device form takes
 * device buffers, runs synchronously (the re-verification needs the sub-batch
 * results on the host) and, when stats != NULL, stores [items accepted in passing
 * sub-batches, items verified one by one, failed sub-batches]. */
int bls381_verify_batch_randomized(size_t n, const uint8_t* pks, const uint8_t* msgs32, const uint8_t* sigs,
                                   const uint8_t* dom8s, const uint8_t seed[32], size_t batch,
                                   uint8_t* verdicts_out);
size_t bls381_verify_batch_randomized_workspace_size(size_t n, size_t batch);
int bls381_verify_batch_randomized_device(size_t n, const uint8_t* d_pks, const uint8_t* d_msgs32,
                                          const uint8_t* d_sigs, const uint8_t* d_dom8s, const uint8_t seed[32],
                                          size_t batch, uint8_t* d_verdicts, void* d_workspace, void* stream,
                                          uint64_t* stats);

/* Committee aggregation (config C3/C4): n_groups groups, group g = pubkeys
 * [offsets[g], offsets[g+1]).  out48 receives n_groups compressed sums; status[g]
 * is 0, or BLS381_EINVAL_POINT when a member does not decode. */
int bls381_aggregate_pubkeys_batch(size_t n_groups, const uint32_t* offsets, const uint8_t* pks,
                                   uint8_t* out48, int32_t* status);
size_t bls381_aggregate_pubkeys_batch_workspace_size(size_t n_groups, size_t n_pks);
/* h_offsets is a HOST array (n_groups + 1 entries): the grouping plan is built on the host. */
int bls381_aggregate_pubkeys_batch_device(size_t n_groups, const uint32_t* h_offsets, size_t n_pks,
                                          const uint8_t* d_pks, uint8_t* d_out48, int32_t* d_status,
                                          void* d_workspace, void* stream);

/* n_calls independent bls_verify_multiple calls: call c
 * owns pubkeys/messages [call_off[c], call_off[c+1]) (host offsets, n_calls+1
 * entries), signature sigs[c] (96 B) and dom8s[c] (8 B).  verdicts[c] = 1/0. */
int bls381_verify_multiple_batch(size_t n_calls, const uint32_t* call_off, const uint8_t* pks,
                                 const uint8_t* msgs, size_t msg_len, const uint8_t* sigs, const uint8_t* dom8s,
                                 uint8_t* verdicts);

/* Device-resident form (C3: the committee aggregates never leave HBM).  Pubkeys
 * (d_pks, 48 B each, numbered like the messages), signatures (d_sigs, 96 B per
 * call) and domains (d_dom8s) are device memory; the call offsets and the
 * messages stay on the HOST (h_call_off, h_msgs): they decide the per-message
 * grouping plan, and the messages are copied with it.  d_verdicts[c] = 1/0.  Work
 * is queued on `stream` (hipStream_t; NULL = the null stream), not synchronised.
 * The workspace must hold bls381_verify_multiple_batch_workspace_size bytes. */
size_t bls381_verify_multiple_batch_workspace_size(size_t n_calls, size_t n_pks, size_t msg_len);
int bls381_verify_multiple_batch_device(size_t n_calls, const uint32_t* h_call_off, const uint8_t* h_msgs,
                                        size_t msg_len, const uint8_t* d_pks, const uint8_t* d_sigs,
                                        const uint8_t* d_dom8s, uint8_t* d_verdicts, void* d_workspace,
                                        void* stream);

/* Batched validate_indexed_attestation (reference 0_beacon-chain.md:1023-1026):
 *   bls_verify_multiple(pubkeys=[bls_aggregate_pubkeys(group) for group in call c],
 *                       message_hashes=[one message per group], signature, domain)
 * in one call, with the aggregation fused in: call c owns groups
 * [h_call_group_off[c], h_call_group_off[c+1]); group g owns the member keys
 * d_pks[h_group_key_off[g] .. h_group_key_off[g+1]) (48 B each, device memory, in
 * group order) and message h_group_msgs[g] (msg_len bytes, host).  The members' sum
 * runs beside hash_to_G2 instead of before it.  An empty group is the infinite
 * aggregate (its pairing is 1); groups of one call with equal messages are merged, as
 * py_ecc's verify_multiple does.  Divergence: an undecodable member key makes the
 * verdict 0 where bls_aggregate_pubkeys would raise.  Queued on `stream`, not
 * synchronised; the workspace must hold bls381_verify_multiple_grouped_workspace_size. */
size_t bls381_verify_multiple_grouped_workspace_size(size_t n_calls, size_t n_groups, size_t n_pks,
                                                     size_t msg_len);
int bls381_verify_multiple_grouped_device(size_t n_calls, const uint32_t* h_call_group_off, size_t n_groups,
                                          const uint32_t* h_group_key_off, const uint8_t* h_group_msgs,
                                          size_t msg_len, const uint8_t* d_pks, const uint8_t* d_sigs,
                                          const uint8_t* d_dom8s, uint8_t* d_verdicts, void* d_workspace,
                                          void* stream);

/* ---- multi-GPU partial products --------------------------- */
/* Miller-loop product of one shard of a bls_verify_multiple call: pairs
 * (hash_to_G2(msg_g), group_pubkey_g) for the messages in this shard, plus
 * (sig, -g1) when include_sig != 0.  out576 = Fp12 in the engine's tower
 * (a0..b2, each re||im, 48-byte big-endian).  Returns 0, or 1 when an input
 * fails to decode / fails a subgroup check (the call's verdict is then False). */
int bls381_miller_partial(size_t n, const uint8_t* pks, const uint8_t* msgs, size_t msg_len,
                          const uint8_t sig[96], int include_sig, const uint8_t dom8[8],
                          uint8_t out576[576]);
/* Multiply k partial products and run one final exponentiation: 1 / 0. */
int bls381_final_verify(size_t k, const uint8_t* parts576);

/* ---- native multi-GPU over RCCL: one process per GPU -------- */
/* A communicator lives inside the library (RCCL opened with dlopen on first
 * use).  Rank 0 makes a 128-byte id, the launcher hands it to every rank (any
 * channel: bls381_amd/comm.py uses TCP), each rank calls bls381_comm_init on the
 * device it selected with bls381_init.  No PyTorch anywhere. */
int bls381_comm_unique_id(uint8_t out[128]);
int bls381_comm_init(int nranks, int rank, const uint8_t uid[128]);
/* Path of the RCCL shared object the library uses (an RCCL the process already loaded,
 * e.g. PyTorch's, is preferred over a fresh dlopen; needs no device).  0, or ENODEV. */
int bls381_comm_rccl_path(char* out, size_t cap);
/* One process plays all nranks ranks on its own GPU: the same partition and
 * rank-0 combination, the all-gather a device copy (RCCL refuses two ranks on
 * one GPU; this is how a one-GPU box runs the N-rank protocol). */
int bls381_comm_init_virtual(int nranks);
int bls381_comm_size(void);   /* 0 without a communicator */
int bls381_comm_rank(void);   /* -1 without a communicator */
void bls381_comm_destroy(void);
/* Collective bls_verify_multiple (every rank passes the same call): distinct
 * message k goes to rank k mod nranks (its pubkey group never straddles ranks),
 * rank 0 adds (sig, -g1); each rank's Miller product (576 B, zero if a member is
 * invalid) is all-gathered over RCCL and rank 0 multiplies them and runs the one
 * final exponentiation of the call (py_ecc's single-FE semantics,
 * 1_custody-game.md:409); the verdict is broadcast.  Returns 1 / 0 on every rank. */
int bls381_verify_multiple_sharded(size_t n, const uint8_t* pks, const uint8_t* msgs, size_t msg_len,
                                   const uint8_t sig[96], const uint8_t dom8[8]);
/* Collective bls_aggregate_pubkeys: contiguous pubkey ranges per rank, compressed
 * partials all-gathered and summed on rank 0, broadcast.  Returns 0 or
 * BLS381_EINVAL_POINT (any rank's invalid encoding) on every rank. */
int bls381_aggregate_pubkeys_sharded(size_t n, const uint8_t* pks, uint8_t out[48]);
/* Device-resident form: this rank's n_local keys (its contiguous range of the call, in rank
 * order; a virtual communicator takes the whole call) are already in HBM at d_pks; every rank
 * receives the aggregate in d_out48 and the status (0 or BLS381_EINVAL_POINT) in d_status[0],
 * queued on `stream` with no host copy and no synchronisation.  Replaces the host-buffer form's
 * PCIe copies for callers whose keys are device-resident (bls.py:34-36 aggregate_pubkeys,
 * SURVEY.md §8e).  Returns 0 or a launch / RCCL error code. */
size_t bls381_aggregate_pubkeys_sharded_device_workspace_size(size_t n_local);
int bls381_aggregate_pubkeys_sharded_device(size_t n_local, const uint8_t* d_pks, uint8_t* d_out48,
                                            int32_t* d_status, void* d_workspace, void* stream);
/* Independent verify_multiple calls, contiguous call ranges per rank (a call's
 * final exponentiation is never split); every rank receives all verdicts. */
int bls381_verify_multiple_batch_sharded(size_t n_calls, const uint32_t* call_off, const uint8_t* pks,
                                         const uint8_t* msgs, size_t msg_len, const uint8_t* sigs,
                                         const uint8_t* dom8s, uint8_t* verdicts);

/* ---- device-resident pubkey registry ---------------- */
/* Decoded validator pubkeys kept in HBM, so committee aggregation reads each
 * member's point instead of decompressing it (the per-key Fp square root that
 * dominates bls_aggregate_pubkeys).  The reference indexes pubkeys through
 * state.validator_registry (specs/core/0_beacon-chain.md:1025-1026, the
 * get_attesting_indices -> bls_aggregate_pubkeys call of
 * validate_indexed_attestation); aggregation over the registry returns the same
 * bytes as bls_aggregate_pubkeys over the members' encodings (bls.py:34-36).
 * Entries are appended in order: entry e is the e-th key ever added (the
 * validator index when keys are added in registry order).  One registry belongs
 * to the device current at creation. */
typedef struct bls381_registry bls381_registry;
int bls381_registry_create(size_t capacity, bls381_registry** out);
void bls381_registry_destroy(bls381_registry* reg);
size_t bls381_registry_size(const bls381_registry* reg);
/* Append n keys as entries [size, size+n).  entry_out[i] (may be NULL) is the
 * entry that now holds key i's bytes (its own, or an earlier duplicate's), or
 * -1 when key i does not decode.  Returns the number of keys that do not decode. */
int bls381_registry_add(bls381_registry* reg, size_t n, const uint8_t* pks48, int32_t* entry_out);
/* Content-addressed lookup: entry_out[i] = entry holding key i's bytes, or -1.
 * Returns the number of hits. */
int bls381_registry_lookup(bls381_registry* reg, size_t n, const uint8_t* pks48, int32_t* entry_out);
/* Group g = entries indices[offsets[g] .. offsets[g+1]); status as for
 * bls381_aggregate_pubkeys_batch (an undecodable or out-of-range entry makes
 * its group BLS381_EINVAL_POINT). */
int bls381_registry_aggregate_indices(bls381_registry* reg, size_t n_groups, const uint32_t* offsets,
                                      const uint32_t* indices, uint8_t* out48, int32_t* status);
/* Same contract as bls381_aggregate_pubkeys_batch: members found in the
 * registry are read from it, the others are decoded from their bytes. */
int bls381_registry_aggregate_pubkeys_batch(bls381_registry* reg, size_t n_groups, const uint32_t* offsets,
                                            const uint8_t* pks, uint8_t* out48, int32_t* status);
size_t bls381_registry_aggregate_workspace_size(size_t n_groups, size_t n_idx);
/* Device-pointer form of bls381_registry_aggregate_indices (h_offsets on the host). */
int bls381_registry_aggregate_indices_device(bls381_registry* reg, size_t n_groups, const uint32_t* h_offsets,
                                             size_t n_idx, const uint32_t* d_indices, uint8_t* d_out48,
                                             int32_t* d_status, void* d_workspace, void* stream);

/* bls381_verify_multiple_grouped_device with the member keys given as registry entries
 * (d_entries: one uint32 entry per member, in group order; the reference's
 * state.validator_registry[i].pubkey, 0_beacon-chain.md:1025-1026): the committee sums
 * add decoded registry points instead of decoding every member.  An entry past the
 * registry's end, or one holding an undecodable key, makes the verdict 0.  Workspace:
 * bls381_verify_multiple_grouped_workspace_size. */
int bls381_registry_verify_multiple_grouped_device(bls381_registry* reg, size_t n_calls,
                                                   const uint32_t* h_call_group_off, size_t n_groups,
                                                   const uint32_t* h_group_key_off, const uint8_t* h_group_msgs,
                                                   size_t msg_len, const uint32_t* d_entries, const uint8_t* d_sigs,
                                                   const uint8_t* d_dom8s, uint8_t* d_verdicts, void* d_workspace,
                                                   void* stream);

/* ---- SSZ roots: the message_hash producer ---------- */
/* hash_tree_root / signing_root of n serialized fixed-size SSZ items
 * (test_libs/pyspec/eth2spec/utils/ssz/ssz_impl.py:143-163, merkle_minimal.py
 * merkleize_chunks).  `prog` is the item type compiled by bls381_amd/ssz.py:
 * words {1, off, len} push bytes [off, off+len) zero-padded to a 32-byte chunk
 * (len <= 32); {2, k} merkleizes the top k chunks (zero-padded to a power of
 * two) into one.  The program must leave exactly one chunk, read only inside
 * the item, and fit 512 words / 64 chunks, else BLS381_EARG.  roots32 receives
 * n x 32 bytes. */
int bls381_ssz_root_batch(size_t n, const uint8_t* items, size_t item_size, const uint32_t* prog,
                          uint32_t prog_len, uint8_t* roots32);
size_t bls381_ssz_root_workspace_size(void);
/* Device form: item i at d_items + i * stride (stride >= item_size); h_prog on the host. */
int bls381_ssz_root_batch_device(size_t n, const uint8_t* d_items, size_t stride, size_t item_size,
                                 const uint32_t* h_prog, uint32_t prog_len, uint8_t* d_roots32,
                                 void* d_workspace, void* stream);
/* process_deposit's proof-of-possession check over n serialized DepositData
 * (184 B each: pubkey, withdrawal_credentials, amount, signature;
 * 0_beacon-chain.md:394-403): verdicts[i] = bls_verify(pubkey,
 * signing_root(deposit.data), signature, domain) (0_beacon-chain.md:1755-1758),
 * the signing roots computed on the device and fed straight to the verify
 * pipeline. */
int bls381_verify_deposits(size_t n, const uint8_t* deposit_data, const uint8_t* dom8s, uint8_t* verdicts);
size_t bls381_verify_deposits_workspace_size(size_t n);
int bls381_verify_deposits_device(size_t n, const uint8_t* d_deposit_data, const uint8_t* d_dom8s,
                                  uint8_t* d_verdicts, void* d_workspace, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* BLS381_H */
