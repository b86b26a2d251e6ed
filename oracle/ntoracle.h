/*
 * ntoracle.h -- CPU restatement of the Narwhal/Tusk crypto hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity CHECKER for the
 * gfx950 HIP backend (narwhal-tusk_amd/csrc).  Only tests/, the smoke() entry
 * in __graft_entry__.py and the cpu_baseline leg of bench.py may load it.
 * It is never linked into, called by, or used as a fallback for the product
 * library (libntcrypto.so).
 *
 * What it restates (the reference's arithmetic lives in the third-party crate
 * ed25519-dalek 1.0.1 [features=batch] -> curve25519-dalek 3.x (u64 backend),
 * sha2 0.9; pinned at /root/reference/crypto/Cargo.toml:10, none vendored):
 *   - SHA-512 (FIPS 180-4) and the truncate-to-32 `Digest`
 *       worker/src/processor.rs:38, primary/src/messages.rs:70-84,145-153,226-234
 *   - Signature::verify  -> dalek verify_strict      crypto/src/lib.rs:200-204
 *   - Signature::verify_batch -> dalek verify_batch  crypto/src/lib.rs:206-219
 *     with the deterministic accept rule of SURVEY.md Appendix A.3
 *   - Signature::new -> dalek Keypair::sign (RFC 8032)  crypto/src/lib.rs:185-191
 *   - generate_keypair (32-byte seed -> (pk, seed||pk))  crypto/src/lib.rs:163-175
 *   - rand 0.7 StdRng (= ChaCha20, 20 rounds) keystream used by the reference's
 *     test fixture keys()                     crypto/src/tests/crypto_tests.rs:26-29
 *
 * Parity pinning: SHA-512 against Python hashlib; verify_strict / sign /
 * keygen against libsodium 1.0.18 via the
 * committed fixtures in tests/golden/ (generator: tests/golden/make_golden.py).
 * verify_batch's nondeterministic set is documented in DESIGN.md §Oracle.
 */
#ifndef NTORACLE_H
#define NTORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- SHA-512 -------------------------------------------------------------- */
void ntor_sha512(const uint8_t *msg, uint64_t len, uint8_t out64[64]);
/* n independent messages packed in `data` at byte offsets off[i], lengths len[i];
 * writes n*32 bytes (first 32 bytes of each SHA-512).  nthreads<=0 -> 1. */
void ntor_sha512_trunc32_many(const uint8_t *data, const uint64_t *off, const uint64_t *len,
                              uint64_t n, uint8_t *out32, int nthreads);

/* ---- ChaCha20 keystream (rand_chacha 0.2 / rand 0.7 StdRng layout) ---------- */
void ntor_chacha20_keystream(const uint8_t key32[32], uint64_t stream_id, uint64_t counter,
                             uint8_t *out, uint64_t len);

/* ---- Ed25519 (dalek semantics) --------------------------------------------- */
/* seed (32) -> public key (32). */
void ntor_ed25519_pubkey(const uint8_t seed32[32], uint8_t pk32[32]);
/* RFC 8032 deterministic signature with keypair (seed, pk); pk is hashed as given. */
void ntor_ed25519_sign(const uint8_t seed32[32], const uint8_t pk32[32], const uint8_t *msg,
                       uint64_t len, uint8_t sig64[64]);
/* dalek PublicKey::verify_strict + crypto::Signature::verify: 1 = accept, 0 = reject. */
int ntor_ed25519_verify_strict(const uint8_t pk32[32], const uint8_t sig64[64], const uint8_t *msg,
                               uint64_t len);
/* One signature under the cofactorless batch rule (A.2 without the small-order step). */
int ntor_ed25519_verify_cofactorless(const uint8_t pk32[32], const uint8_t sig64[64],
                                     const uint8_t *msg, uint64_t len);
/* crypto::Signature::verify_batch over `cnt` (pk, sig) pairs, one shared message.
 * Returns 1 = Ok, 0 = Err.  Empty input -> 1. */
int ntor_ed25519_verify_batch(const uint8_t *pk32, const uint8_t *sig64, uint64_t cnt,
                              const uint8_t *msg, uint64_t len);
/* Bulk forms (OpenMP-free pthreads pool; nthreads<=0 -> 1), same layouts as the C ABI. */
void ntor_ed25519_verify_strict_many(const uint8_t *pk32, const uint8_t *sig64, const uint8_t *msg,
                                     const uint64_t *off, const uint64_t *len, uint64_t n,
                                     uint8_t *out_bitmap, int nthreads);
void ntor_ed25519_verify_batch_groups(const uint8_t *pk32, const uint8_t *sig64,
                                      const uint64_t *first, const uint32_t *cnt,
                                      const uint8_t *msg32, uint64_t G, uint8_t *out_group_bitmap,
                                      uint8_t *out_sig_bitmap, int nthreads);

/* CPU BASELINE ONLY (bench.py config 3): dalek's verify_batch as dalek computes
 * it -- random 128-bit z_i (ChaCha20 keyed by zkey), one Straus/NAF-5 vartime
 * multiscalar multiplication -- and Certificate::verify's signature + digest
 * work over G certificates (header preimages at hoff/hlen in hdr, ids G*32,
 * author keys hpk G*32, header signatures G*64, certificate digest preimages
 * cpre G*72, votes vpk/vsig from first[g], cnt[g]).  out: 1 byte per certificate. */
int ntor_ed25519_verify_batch_dalek(const uint8_t *pk32, const uint8_t *sig64, uint64_t cnt,
                                    const uint8_t *msg, uint64_t len, const uint8_t zkey[32]);
void ntor_certificates_verify_many(const uint8_t *hdr, const uint64_t *hoff, const uint64_t *hlen,
                                   const uint8_t *ids, const uint8_t *hpk, const uint8_t *hsig,
                                   const uint8_t *cpre, const uint8_t *vpk, const uint8_t *vsig,
                                   const uint64_t *first, const uint32_t *cnt, uint64_t G, uint8_t *out,
                                   int nthreads);

/* Diagnostics used by the corpus generator (tests only). */
/* 1 if the 32 bytes decode as a point under dalek decompress rules. */
int ntor_point_decodes(const uint8_t p32[32]);
/* 1 if decodes and [8]P == identity. */
int ntor_point_is_small_order(const uint8_t p32[32]);
/* 1 if decodes and [L]P != identity (point has a torsion component). */
int ntor_point_has_torsion(const uint8_t p32[32]);
/* Classify a (pk, sig, msg) triple for the dalek verify_batch rule:
 * 0 = deterministic reject, 1 = deterministic accept,
 * 2 = dalek's randomized batch decision is NOT deterministic for this entry
 *     (residual has no prime-order part but a nonzero torsion part, or the
 *      equation holds and A has a torsion component).  See DESIGN.md. */
int ntor_ed25519_batch_class(const uint8_t pk32[32], const uint8_t sig64[64], const uint8_t *msg,
                             uint64_t len);
/* scalar helpers (little-endian 32 bytes) */
void ntor_sc_reduce64(const uint8_t in64[64], uint8_t out32[32]);
int ntor_sc_is_canonical(const uint8_t s32[32]);
/* point helpers on compressed encodings (canonical outputs) */
int ntor_point_add(const uint8_t p32[32], const uint8_t q32[32], uint8_t out32[32]);
int ntor_point_scalarmul(const uint8_t p32[32], const uint8_t s32[32], uint8_t out32[32]);
void ntor_basepoint_mul(const uint8_t s32[32], uint8_t out32[32]);
/* The 8 torsion points E[8], canonical encodings, index i = [i]T8 for a fixed
 * generator T8 of order 8. */
void ntor_torsion_point(int i, uint8_t out32[32]);

/* External CPU comparator (bench.py cpu_baseline): libsodium crypto_sign_verify_detached
 * over n signatures on nthreads threads, library dlopen'ed from libpath; -1 if absent. */
int ntor_sodium_verify_many(const char *libpath, const uint8_t *pk32, const uint8_t *sig64, const uint8_t *msg,
                            const uint64_t *off, const uint64_t *len, uint64_t n, int nthreads, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
