/*
 * ntcrypto.h -- C ABI of the MI355X (gfx950) crypto backend for Narwhal/Tusk.
 *
 * Drop-in boundary: the reference's `crypto` crate (crypto/src/lib.rs) keeps
 * its public Rust surface; its FFI binds these symbols.
 *
 *   nt_sha512_trunc32            replaces  Digest(Sha512::digest(&batch)[..32])
 *                                          worker/src/processor.rs:38,
 *                                          worker/src/batch_maker.rs:124-128 (benchmark hash),
 *                                          primary/src/messages.rs:70-84 (Header::digest),
 *                                          :145-153 (Vote::digest), :226-234 (Certificate::digest)
 *   nt_ed25519_verify_strict     replaces  Signature::verify -> dalek verify_strict
 *                                          crypto/src/lib.rs:200-204
 *   nt_ed25519_verify_batch_groups replaces Signature::verify_batch -> dalek verify_batch
 *                                          crypto/src/lib.rs:206-219, called once per
 *                                          certificate by Certificate::verify
 *                                          primary/src/messages.rs:189-215
 *   nt_ed25519_sign_batch /      batch form of Signature::new / generate_keypair
 *   nt_ed25519_keypair_batch               crypto/src/lib.rs:163-191 (NOT constant time:
 *                                          corpus generation and tests only)
 *
 * Conventions
 *   - Host entry points take caller-owned host memory, borrowed for the call;
 *     the library stages it into its own device buffers and keeps no pointer.
 *   - Calls are synchronous.  Verdicts are data (bitmaps), never errors.
 *   - Bitmaps: bit i of byte i/8 (LSB first) = item i; 1 = accept.
 *   - Return 0 on success, < 0 on failure (NT_E*).  A caller must never turn a
 *     negative return into "reject"; there is NO CPU fallback inside this
 *     library: without a usable gfx950 device nt_init fails with NT_ENODEV.
 *   - Thread-safe: calls on one context may come from several threads.  Each
 *     device entry has NT_SLOTS (default 2) execution slots -- own streams,
 *     workspace and staging -- and a call takes a free one, so a long call (a
 *     batch of digests) does not block a concurrent short one (a certificate
 *     batch): small calls prefer the extra slot, whose single stream has the
 *     highest priority; bulk calls the entry's own slot.
 *   - Multi-GPU: host entry points shard items by contiguous index ranges
 *     over the context's devices (certificates are never split); no
 *     collective, results gathered on the host.
 *   - nt_dev_* entry points take DEVICE pointers on device `dev` of the
 *     context and a hipStream_t (NULL = HIP's NULL stream), and only
 *     enqueue work; message buffers come with their byte size and the
 *     kernels never read outside it.  Word-typed buffers (pk, sig, seed, out) must be 16-byte
 *     aligned; message data may have any alignment.
 */
#ifndef NTCRYPTO_H
#define NTCRYPTO_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NT_OK 0
#define NT_EINVAL (-1)
#define NT_EHIP (-2)
#define NT_ENOMEM (-3)
#define NT_ENODEV (-4)

#define NT_MODE_STRICT 0       /* dalek verify_strict */
#define NT_MODE_COFACTORLESS 1 /* per-entry rule of dalek verify_batch */
/* Key-cache entry points only: per signature, bit 31 of key_idx set = strict
 * (Header/Vote::verify), clear = cofactorless (Certificate::verify's votes), so a
 * drained batch of headers, votes and certificate votes is one launch. */
#define NT_MODE_MIXED 2
#define NT_KEY_STRICT_BIT 0x80000000u

typedef struct nt_ctx nt_ctx;

/* num_gpus: 0 = all visible devices, k > 0 = the first k, -1 = CPU only
 * (unsupported: returns NT_ENODEV -- this library has no CPU path). */
int nt_init(nt_ctx **out, int num_gpus);
/* One specific device ordinal (used by one-process-per-GPU launchers). */
int nt_init_device(nt_ctx **out, int device_ordinal);
/* An explicit list of device ordinals; repeats are allowed (each entry gets
 * its own streams, workspace and staging), which lets the multi-device
 * sharding of the host entry points be exercised on a single GPU. */
int nt_init_devices(nt_ctx **out, const int *ordinals, int n);
void nt_free(nt_ctx *ctx);
int nt_num_devices(const nt_ctx *ctx);
const char *nt_strerror(int code);
/* Library / build identification, e.g. "ntcrypto 0.1 gfx950". */
const char *nt_version(void);

/* ---- device memory (lazy, budgeted) -----------------------------------
 * The reference runs every primary and every worker as its own process
 * (node/src/main.rs:101-133); a worker only hashes (worker/src/processor.rs:38).
 * So nt_init allocates nothing large: a context that only digests holds
 * streams and grow-only staging.  The first call that verifies or signs on a
 * device entry builds the wide comb of B there (shared by every context of
 * the process on that ordinal and width) and, for the verify kernel, the [k]A
 * workspace (~1.5 GB per execution slot that verifies).  The comb's width is
 * the widest that fits: 24-bit digits (11 additions per [s]B, 11.8 GB) when
 * the context's budget allows it and the device keeps 4 GB free beside it,
 * else 20-bit digits (13 additions, 872 MB); NT_BCOMB_BITS=24|20 forces one.
 * A key set (nt_keyset_create) or the key registry (nt_set_key_cache) reserves
 * its key combs against the same budget after the comb of B: 21 / 20 / 18 /
 * 16-bit digits, the widest that fits.
 *
 * nt_set_hbm_budget: bytes of such TABLES (comb of B + key combs) the context
 * may hold per device entry; 0 = no cap (the device's free memory decides).
 * Default: the NT_HBM_BUDGET environment variable at nt_init (bytes, or with a
 * K / M / G suffix).  Applies to the tables built after the call; NT_ENOMEM
 * when not even the narrowest width fits.
 *
 * nt_memory_info(ctx, dev, out8): what device entry `dev` of THIS context holds:
 *   out8[0] comb of B digit width (0 = not built yet)   out8[1] its bytes
 *   out8[2] key-comb bytes of live key sets             out8[3] verify workspaces
 *   out8[4] key-cache stashes + sort scratch            out8[5] other device staging
 *   out8[6] the budget (0 = none)                       out8[7] table bytes held against it */
int nt_set_hbm_budget(nt_ctx *ctx, uint64_t bytes_per_device);
int nt_memory_info(nt_ctx *ctx, int dev, uint64_t *out8);

/* SHA-512 truncated to 32 bytes of n independent messages packed in `data`
 * (message i = data[off[i] .. off[i] + len[i])).  out32: n * 32 bytes. */
int nt_sha512_trunc32(nt_ctx *ctx, const uint8_t *data, const uint64_t *off, const uint64_t *len,
                      uint64_t n, uint8_t *out32);

/* dalek verify_strict for n (pk, sig, msg) triples.  pk32: n*32, sig64: n*64 (R || s),
 * message i = msg[off[i] .. off[i] + len[i]).  out_bitmap: ceil(n/8) bytes. */
int nt_ed25519_verify_strict(nt_ctx *ctx, const uint8_t *pk32, const uint8_t *sig64,
                             const uint8_t *msg, const uint64_t *off, const uint64_t *len,
                             uint64_t n, uint8_t *out_bitmap);

/* Narwhal verify_batch semantics for G certificates at once: group g has cnt[g]
 * (pk, sig) pairs starting at index first[g], all over the 32-byte msg32[g].
 * out_group_bitmap: ceil(G/8) bytes; out_sig_bitmap (nullable): one bit per
 * pair, sized for max(first[g] + cnt[g]) pairs.  Empty group -> accept. */
int nt_ed25519_verify_batch_groups(nt_ctx *ctx, const uint8_t *pk32, const uint8_t *sig64,
                                   const uint64_t *first, const uint32_t *cnt,
                                   const uint8_t *msg32, uint64_t G, uint8_t *out_group_bitmap,
                                   uint8_t *out_sig_bitmap);

/* Keygen (seed -> pk) and RFC 8032 signing of message i with seed i.
 * sig64 may be NULL (keygen only).  Not constant time. */
int nt_ed25519_sign_batch(nt_ctx *ctx, const uint8_t *seed32, const uint8_t *msg,
                          const uint64_t *off, const uint64_t *len, uint64_t n, uint8_t *pk32,
                          uint8_t *sig64);
int nt_ed25519_keypair_batch(nt_ctx *ctx, const uint8_t *seed32, uint64_t n, uint8_t *pk32);

/* ---- committee key cache ------------------------------
 * A keyset holds, on every device of the context, per-key comb tables
 * (the wide comb of -A: 21-bit digits of the scalar reduced to |k| <= L/2,
 * 12 x 1048641 affine niels entries plus the key's [L](-A) = 1.61 GB per key
 * -- 161 GB for n = 100 -- when every device can hold them with 1/8 of its
 * HBM to spare and the context's HBM budget allows, else 20-bit digits, 13 x
 * 524289 entries = 872 MB per key, else 18-bit digits, 15 x 131073 = 252 MB,
 * else 16-bit digits, 16 x 32769 = 67 MB; NT_KEYSET_COMB_BITS=16|18|20|21
 * forces one) plus each key's raw
 * encoding and decode / small-order flags, so verification against a static
 * committee (config/src/lib.rs:140-143) needs no decompression of A and no
 * doublings.  Keys are addressed by index (the caller's committee order);
 * an index >= nkeys means "not a committee key" and verifies as reject.
 * Keys that do not decode are accepted into the set and always reject, as
 * PublicKey::from_bytes would (crypto/src/lib.rs:202,216).
 * Lifetime: free every keyset before its context; an nt_committee built on a
 * keyset keeps the keyset's device tables alive, so the keyset handle may be
 * freed before the committee. */
typedef struct nt_keyset nt_keyset;
int nt_keyset_create(nt_ctx *ctx, const uint8_t *pk32, uint32_t nkeys, nt_keyset **out);
void nt_keyset_free(nt_keyset *ks);
/* flags of key i: bit 0 = decodes, bit 1 = small order */
int nt_keyset_flags(const nt_keyset *ks, uint32_t i, uint32_t *flags);
/* comb digit width of the set (16, 18, 20 or 21) and its device bytes per device */
int nt_keyset_info(const nt_keyset *ks, uint32_t *comb_bits, uint64_t *bytes_per_device);
int nt_ed25519_verify_keyset(nt_ctx *ctx, const nt_keyset *ks, int mode, const uint32_t *key_idx,
                             const uint8_t *sig64, const uint8_t *msg, const uint64_t *off,
                             const uint64_t *len, uint64_t n, uint8_t *out_bitmap);
int nt_ed25519_verify_batch_groups_keyset(nt_ctx *ctx, const nt_keyset *ks, const uint32_t *key_idx,
                                          const uint8_t *sig64, const uint64_t *first,
                                          const uint32_t *cnt, const uint8_t *msg32, uint64_t G,
                                          uint8_t *out_group_bitmap, uint8_t *out_sig_bitmap);

/* ---- key registry: the committee key cache behind the plain entry points --
 * The reference's crate binds Signature::verify / verify_batch with raw
 * PublicKeys (crypto/src/lib.rs:200-219): no committee handle crosses it.  With
 * a registry enabled, nt_ed25519_verify_strict and
 * nt_ed25519_verify_batch_groups look every 32-byte key up in it (a host-side
 * index, before the keys cross PCIe: a registered key travels as a 4-byte
 * index); registered keys verify through the key-cache kernel, the others
 * through the uncached kernel in the same call, same verdicts either way.  A
 * key that misses is counted, and after `admit_after` sightings (>= 1) a
 * background thread builds its key combs on every device entry (on a
 * low-priority stream of its own) and publishes it: later calls find it.
 * Every key the reference passes to these calls is a committee member
 * (primary/src/messages.rs:86-100, 155-163, 189-215) and the committee is
 * static (config/src/lib.rs:140-143), so the registry holds at most max_keys
 * keys and never evicts; keys that do not decode are never admitted (they
 * reject either way).  Its comb width is chosen at the first admission for
 * max_keys keys, as for a key set (21 / 20 / 18 / 16 bits, against the
 * context's HBM budget); its tables are allocated then, not before.
 *
 * nt_set_key_cache: max_keys in [1, NT_KEY_CACHE_MAX], 0 = off (the default;
 * NT_KEY_CACHE=<max_keys>[:<admit_after>] in the environment at nt_init sets
 * it).  Call it before the context's verify calls, not concurrently with them.
 * nt_key_cache_add: admit these keys now (waits for their tables).
 * nt_key_cache_sync: wait until every queued admission is published; returns
 * the registry's error (NT_ENOMEM: its tables did not fit, it admits no more).
 * nt_key_cache_info out12: keys, max_keys, comb bits, device bytes per device
 * entry (0 before the first admission), lookups that hit, lookups that missed,
 * keys admitted, keys refused (do not decode / tables failed), admissions
 * pending, -error, microseconds the admission thread spent allocating tables
 * and building combs (the allocation waits for the driver to clear memory
 * another table just freed: DESIGN.md §6.5). */
#define NT_KEY_CACHE_MAX 4095u
int nt_set_key_cache(nt_ctx *ctx, uint32_t max_keys, uint32_t admit_after);
int nt_key_cache_add(nt_ctx *ctx, const uint8_t *pk32, uint32_t n);
int nt_key_cache_sync(nt_ctx *ctx);
int nt_key_cache_info(const nt_ctx *ctx, uint64_t *out12);

/* ---- certificate ingestion from wire bytes --------------
 * The primary's receiver deserializes every PrimaryMessage with bincode
 * (primary/src/primary.rs:225-244) before Core::sanitize_certificate
 * (core.rs:339-346) runs Certificate::verify (messages.rs:189-215).  These
 * entry points take the message bytes as they arrived, copy them to the
 * device as-is and parse, check and verify them there: one SHA-512 launch
 * (header ids and certificate digests), one NT_MODE_MIXED key-cache launch
 * (the header signature strict, the votes cofactorless) and a group AND per
 * chunk of messages, chunks pipelined so the PCIe copy of one overlaps the
 * kernels of the previous one.
 *
 * nt_committee: the committee of a keyset (key i = keyset key i): stake per
 * key, its worker ids (worker_ids[worker_first[i] .. worker_first[i + 1]),
 * any order) and the quorum threshold (config/src/lib.rs:168-173:
 * 2 * total_stake / 3 + 1).  The keyset's keys ARE the committee's
 * authorities (Committee::authorities, config/src/lib.rs:140-143): build it
 * from exactly those keys.  Certificate::genesis(committee) has one
 * certificate per authority (primary/src/messages.rs:175-187), so a round-0
 * certificate with the zero header id whose author is a keyset key is
 * genesis, whatever that key's stake -- as in the reference.  Keys are
 * looked up by their canonical base64 text (crypto/src/lib.rs:73-79,103-112),
 * as the reference's serde does.  Free the committee before its context. */
typedef struct nt_committee nt_committee;
int nt_committee_create(nt_ctx *ctx, const nt_keyset *ks, const uint32_t *stake, const uint64_t *worker_first,
                        const uint32_t *worker_ids, uint32_t quorum, nt_committee **out);
void nt_committee_free(nt_committee *cm);
/* primary::DagError codes of out_code (host/narwhal.hpp; error.rs variants) */
#define NT_DAG_OK 0
#define NT_DAG_INVALID_SIGNATURE 1
#define NT_DAG_INVALID_HEADER_ID 2
#define NT_DAG_MALFORMED_HEADER 3
#define NT_DAG_UNKNOWN_AUTHORITY 4
#define NT_DAG_AUTHORITY_REUSE 5
#define NT_DAG_REQUIRES_QUORUM 6
#define NT_DAG_TOO_OLD 7
/* a message this path does not decide: not a Certificate, not in canonical
 * form (map / set entries out of order, a key string that is not a committee
 * key's canonical base64 text), malformed or truncated -- the caller runs its
 * host decoder on it (the C++ mirror: Core::ingest) */
#define NT_DAG_HOST 0xff
/* message i = data[off[i] .. off[i] + len[i]); out_code: n bytes.  Inputs in
 * nt_host_alloc memory are DMA'd straight from it. */
int nt_certificates_ingest(nt_ctx *ctx, const nt_committee *cm, const uint8_t *data, const uint64_t *off,
                           const uint64_t *len, uint64_t n, uint64_t gc_round, uint8_t *out_code);

/* ---- small-call path (SURVEY.md H3, §8(b) "CPU-fallback threshold") ------
 * The reference calls verify once per header / vote, verify_batch once per
 * certificate (primary/src/core.rs:349-411) and hashes one ~508 KB batch per
 * Processor call (worker/src/processor.rs:36-38).  A GPU call that small costs
 * a launch plus one lane's serial chain (a lone 508,052-B digest 16.8 ms on
 * MI355X; a lone verify ~1.5 ms) -- more than the host needs.  With
 * NT_SMALL_AUTO the host entry points run calls whose estimated host time is
 * below their estimated GPU time on `threads` host threads, with the SAME
 * arithmetic compiled for the host (csrc/cpu_lane.cpp; not the oracle); with
 * NT_SMALL_ALWAYS every host entry point does (tests).  Default NT_SMALL_OFF:
 * everything on the GPU.  The nt_dev_* entry points always run on the GPU.
 * A context still requires a gfx950 device: this is a latency path, not a
 * fallback.  threads <= 0: min(16, hardware threads). */
#define NT_SMALL_OFF 0
#define NT_SMALL_AUTO 1
#define NT_SMALL_ALWAYS 2
int nt_set_small_call_path(nt_ctx *ctx, int mode, int threads);
/* Host entry-point calls served on host threads / on the GPU so far. */
int nt_call_counts(const nt_ctx *ctx, uint64_t *host_calls, uint64_t *gpu_calls);
/* The cost model AUTO routes by.  The first nt_set_small_call_path that enables
 * the path calibrates it on this context: the host lane's verify_strict time
 * and SHA-512 rate on one thread, the pool wake-up on `threads` threads, and
 * the GPU floors from real calls (a one-signature verify, a 64-byte and a
 * 1 MiB digest); NT_SMALL_* environment variables override single fields.
 * out10 = cpu_verify_us, gpu_verify_us, cpu_sha_mbs, gpu_lane_mbs, gpu_call_us,
 * pcie_gbs, spawn_us, threads, calibrated (0/1), gpu_keyset_us.  A verify call
 * of n signatures runs on the host iff ceil(n / T) * cpu_verify_us + (T > 1 ?
 * spawn_us : 0) < the GPU floor of the kernel it would run (T = min(threads,
 * n)): gpu_keyset_us (a one-signature call through the key-cache kernel, timed
 * on a one-key 16-bit key set) for key-set calls and registry calls whose keys
 * all hit, gpu_verify_us (the uncached kernel) otherwise; a digest call iff
 * max(longest, total / T) / cpu_sha_mbs + (T > 1 ? spawn_us : 0) < gpu_call_us
 * + longest / gpu_lane_mbs + total / (1000 pcie_gbs) (bytes, microseconds;
 * csrc/small_model.hpp). */
int nt_small_call_model(const nt_ctx *ctx, double *out10);

/* ---- pinned host buffers ---------------------------------------------
 * Page-locked host memory for callers that stage large batches themselves
 * (the primary's wire ingestion).  Inputs that lie in such a buffer are
 * copied to the device by DMA straight from it: the host entry points skip
 * their own staging copy (for certificate groups: when the groups' signatures
 * and keys are also densely packed, first[g + 1] == first[g] + cnt[g]).
 * No reference counterpart: the reference's Rust callers own ordinary Vecs.
 * Returns NULL when no device / no memory. */
void *nt_host_alloc(uint64_t bytes);
void nt_host_free(void *p);

/* ---- device-resident entry points (enqueue only) ----------------------
 * `stream` is the caller's hipStream_t; NULL is HIP's NULL stream, as for any
 * HIP call (round 4 read NULL as "the library's stream").  The calls order
 * their launches after earlier work on `stream` only: inputs produced on
 * another stream must be complete (an event `stream` waits on, or a
 * synchronize) before the call.
 *
 * Message buffers come with their byte size (msg_bytes / data_bytes): item i
 * reads d_msg[d_off[i] .. d_off[i] + d_len[i]) only when that slice lies inside
 * [0, msg_bytes).  An item whose slice does not is never read -- a verification
 * rejects it, signing writes an all-zero signature, SHA-512 writes a zero
 * digest and adds 1 to *d_bad (a device counter the caller zeroes; NULL = not
 * counted).  So an offset read before its producer wrote it (round 4's fault
 * r04e: a wild offset from a cross-stream race) cannot fault the card.
 *
 * nt_dev_stream returns device entry `dev`'s two compute streams (which = 0 /
 * 1), the streams the host entry points pipeline on: non-blocking, ordered
 * against no other stream (NT_STREAMS=mask: each on a hardware queue of its
 * own, but then BLOCKING, i.e. ordered against the NULL stream).  Batches
 * enqueued back to back overlap only if their streams sit on different
 * hardware queues (HIP multiplexes a process's streams over GPU_MAX_HW_QUEUES
 * queues per priority); a caller pipelining device-API batches may alternate
 * between these two or two of its own. */
int nt_dev_stream(nt_ctx *ctx, int dev, int which, void **out);
int nt_dev_sha512_trunc32(nt_ctx *ctx, int dev, void *stream, const uint8_t *d_data, uint64_t data_bytes,
                          const uint64_t *d_off, const uint64_t *d_len, uint64_t n, uint32_t *d_bad,
                          uint8_t *d_out32);
/* The same digests when the caller knows an upper bound of the lengths
 * (headers, votes, certificate digests): max_len only selects the kernel --
 * below 16 KB the one-lane kernel, which holds no LDS, so it never waits
 * behind a key-cache launch of another stream.  Any length is
 * still hashed correctly whatever max_len says. */
int nt_dev_sha512_trunc32_bounded(nt_ctx *ctx, int dev, void *stream, const uint8_t *d_data,
                                  uint64_t data_bytes, const uint64_t *d_off, const uint64_t *d_len, uint64_t n,
                                  uint64_t max_len, uint32_t *d_bad, uint8_t *d_out32);
/* d_out_words: ceil(n/64) little-endian 64-bit bitmap words.  Successive calls
 * alternate between the device entry's two [k]A workspaces (each ordered by
 * its own event), so batches enqueued back to back on two different streams
 * overlap: the next batch's waves fill the SIMDs the previous batch's last
 * round leaves idle.  Calls on one stream run in stream order. */
int nt_dev_ed25519_verify(nt_ctx *ctx, int dev, void *stream, int mode, const uint8_t *d_pk32,
                          const uint8_t *d_sig64, const uint8_t *d_msg, uint64_t msg_bytes,
                          const uint64_t *d_off, const uint64_t *d_len, uint64_t n, uint64_t *d_out_words);
int nt_dev_group_and(nt_ctx *ctx, int dev, void *stream, const uint64_t *d_first,
                     const uint32_t *d_cnt, uint64_t G, const uint64_t *d_sig_words,
                     uint64_t *d_group_words);
int nt_dev_ed25519_verify_keyset(nt_ctx *ctx, const nt_keyset *ks, int dev, void *stream, int mode,
                                 const uint32_t *d_key_idx, const uint8_t *d_sig64, const uint8_t *d_msg,
                                 uint64_t msg_bytes, const uint64_t *d_off, const uint64_t *d_len, uint64_t n,
                                 uint64_t *d_out_words);
/* Diagnostics (no reference counterpart): the shader clock of device entry
 * `dev` under a fixed integer-multiply load enqueued on `stream` -- every CU
 * runs `iters` x 64 dependent-pair v_mad_u64_u32 per lane for ~1-2 ms while
 * each wave reads the shader-clock and the constant-rate wall-clock counters at
 * its start and end.  out2 (device memory, 2 x uint64, written by the kernel):
 * summed shader-clock cycles and summed wall-clock ticks over the waves; their
 * ratio x the wall clock's rate (*wall_khz) is the effective clock.  bench.py
 * brackets its timed regions with it. */
int nt_dev_clock_probe(nt_ctx *ctx, int dev, void *stream, uint32_t iters, uint64_t *d_out2, uint64_t *wall_khz);

/* The key-cache verification of n signatures that also ANDs their verdicts per
 * certificate: group g = signatures [d_first[g], d_first[g] + d_cnt[g]) of the
 * call (d_first non-decreasing; a signature may belong to no group, e.g. a
 * header signature of a NT_MODE_MIXED call), bit g of d_group_words (ceil(G/64)
 * words) = every one accepted; an empty group accepts.  The groups' AND and the
 * verdict words are written by the key-cache kernel itself (one launch chain:
 * init, key sort, kernel -- no verdict-pack or group-AND launch after it), so a
 * pipelined caller's next step waits for nothing but this call.  The device
 * form of nt_ed25519_verify_batch_groups_keyset (Certificate::verify,
 * primary/src/messages.rs:189-215). */
int nt_dev_ed25519_verify_keyset_groups(nt_ctx *ctx, const nt_keyset *ks, int dev, void *stream, int mode,
                                        const uint32_t *d_key_idx, const uint8_t *d_sig64, const uint8_t *d_msg,
                                        uint64_t msg_bytes, const uint64_t *d_off, const uint64_t *d_len, uint64_t n,
                                        const uint64_t *d_first, const uint32_t *d_cnt, uint64_t G,
                                        uint64_t *d_out_words, uint64_t *d_group_words);

/* d_sig64 may be NULL (keygen only; d_msg, d_off, d_len ignored). */
int nt_dev_ed25519_sign(nt_ctx *ctx, int dev, void *stream, const uint8_t *d_seed32, const uint8_t *d_msg,
                        uint64_t msg_bytes, const uint64_t *d_off, const uint64_t *d_len, uint64_t n,
                        uint8_t *d_pk32, uint8_t *d_sig64);

#ifdef __cplusplus
}
#endif
#endif /* NTCRYPTO_H */
