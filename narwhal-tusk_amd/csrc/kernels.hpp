// kernels.hpp -- host-side launchers of the k_*.hip kernels (used by ntcrypto.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ks_plan.hpp"
#include "nt_common.hpp"

namespace nt {

// Every launcher that reads caller messages takes the byte size of the message
// buffer (msg_bytes / data_bytes): items whose slice lies outside it are never
// read (nt_common.hpp msg_slice) -- rejected by verification and signing, a
// zero digest counted in *d_bad (nullable) by SHA-512.
// max_len: an upper bound of the messages' lengths when the caller knows one
// (it selects the kernel; any length is still hashed correctly)
hipError_t launch_sha512_trunc32(const uint8_t* d_data, uint64_t data_bytes, const uint64_t* d_off,
                                 const uint64_t* d_len, uint64_t n, uint8_t* d_out32, hipStream_t s,
                                 uint64_t max_len = ~0ull, uint32_t* d_bad = nullptr);
hipError_t launch_verify(int mode, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                         uint64_t msg_bytes, const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                         const uint32_t* d_combB, int bbits, void* d_ws, uint32_t ws_slots, uint64_t* d_out_words,
                         hipStream_t s, int per_lane = 0);
hipError_t launch_group_and(const uint64_t* d_first, const uint32_t* d_cnt, uint64_t G,
                            const uint64_t* d_sig_words, uint64_t* d_group_words, hipStream_t s);
// off[first[g] + q] = 32 g, len = 32 for q < cnt[g] (groups' 32-byte messages)
hipError_t launch_group_msgs(const uint64_t* d_first, const uint32_t* d_cnt, uint64_t G, uint64_t* d_off,
                             uint64_t* d_len, hipStream_t s);
hipError_t launch_sign(const uint8_t* d_seed, const uint8_t* d_msg, uint64_t msg_bytes, const uint64_t* d_off,
                       const uint64_t* d_len, uint64_t n, const uint32_t* d_combB, int bbits, uint8_t* d_pk,
                       uint8_t* d_sig, uint32_t max_blocks, hipStream_t s);
// wide combs with `bits`-bit digits (a key-comb width, or kBCombBits for B; kBCombFallback = kKeyCombWide).
// bbits below: the digit width of the comb of B d_combB was built with (kBCombBits / kBCombFallback).
hipError_t launch_wcomb_build(int bits, const uint32_t* d_enc, uint32_t nkeys, int negate, uint32_t* d_comb,
                              uint32_t* d_meta, uint32_t* d_bases, uint32_t* d_tmp, uint32_t batch,
                              hipStream_t s);
// Groups (optional, G > 0): the launch also ANDs the verdicts of each group of
// signatures [d_gfirst[g], d_gfirst[g] + d_gcnt[g]) (d_gfirst non-decreasing)
// into bit g of d_group_words -- inside the kernel's epilogue (KsVerdict,
// kernels_common.hpp), no k_group_and launch.
hipError_t launch_verify_keyset(int mode, int key_bits, const uint32_t* d_key_idx, const uint8_t* d_sig, const uint8_t* d_msg,
                                uint64_t msg_bytes, const uint64_t* d_off, const uint64_t* d_len, uint64_t n, const uint32_t* d_meta,
                                const uint32_t* d_enc, const uint32_t* d_combA, uint32_t nkeys,
                                const uint32_t* d_combB, int bbits, void* d_stash, void* d_sort, uint64_t* d_out_words,
                                uint32_t cus, hipStream_t s, const uint64_t* d_gfirst = nullptr,
                                const uint32_t* d_gcnt = nullptr, uint64_t G = 0, uint64_t* d_group_words = nullptr);
// scratch of launch_verify_keyset: the chunk counter and the key-grouped order (d_sort, required)
size_t keyset_sort_bytes(uint64_t n);
// the plan of one key-cache launch over n signatures on a device of `cus` CUs (ks_plan.hpp;
// NT_KEYSET_WAVES = 1 (streamed) / 2 / 3 forces the waves per SIMD, NT_KEYSET_PER_LANE caps the rows per chunk)
KsPlan keyset_plan(uint64_t n, uint32_t cus);
// signatures one full round of the launch covers (host-side chunk sizing)
uint64_t keyset_round_sigs(uint32_t cus);
// signatures per lane of a launch_verify: per_lane 0 = the build's default (kVPer, 2);
// 1 = one per lane (half the launch latency; host entry points' short chunks)
int verify_per_lane_for(int per_lane);
uint64_t verify_grid(uint64_t n, uint32_t ws_slots, int per_lane = 0);  // blocks of a launch_verify
uint64_t verify_round_sigs(uint32_t cus, int per_lane = 0);
uint32_t keyset_per_lane();
// per-wave stash of a launch over n signatures (d_stash above)
size_t keyset_stash_bytes(uint64_t n, uint32_t cus);
size_t wcomb_bytes_per_key(int bits);
size_t wcomb_bases_bytes_per_key(int bits);
size_t wcomb_fill_tmp_bytes_per_key(int bits);
uint32_t wcomb_fill_batch(int bits);  // keys per k_wcomb_fill launch
size_t ws_bytes_per_slot();
int verify_occupancy();  // waves per SIMD of the selected verify kernel variant
// diagnostics: d_out2[0] / d_out2[1] = summed shader-clock cycles / 100 MHz ticks of a fixed multiply load
hipError_t launch_clock_probe(uint32_t iters, uint32_t cus, uint64_t* d_out2, hipStream_t s);

// ---- certificate ingestion on the device (k_ingest.hip, ingest_gpu.cpp) ----
// Committee tables of an nt_committee on one device.
struct CertCommittee {
  const uint32_t* enc;        // [nkeys][12]: canonical base64 text of the key (44 chars) + 4 zero bytes
  const uint64_t* slot_head;  // [1 << sbits]: first 8 characters of the key in the slot
  const uint32_t* slot_idx;   // [1 << sbits]: key index, 0xffffffff = empty (open addressing)
  const uint32_t* stake;      // [nkeys]
  const uint32_t* wfirst;     // [nkeys + 1]: key k's workers are wids[wfirst[k] .. wfirst[k + 1]), sorted
  const uint32_t* wids;
  const uint32_t* raw;        // [nkeys][8]: the raw 32-byte keys (the keyset's encodings)
  uint32_t nkeys, sbits, quorum;
};
// One chunk of n messages: inputs, per-message state, launch buffers, outputs.
struct CertBufs {
  const uint8_t* wire;   // message bytes (64 bytes of readable slack on both sides)
  const uint64_t* moff;  // message i = wire[moff[i] .. moff[i] + mlen[i])
  const uint64_t* mlen;
  uint64_t n;
  uint64_t* round;       // k_cert_parse
  uint32_t *author, *np, *nq, *nv, *flags, *plen;
  uint64_t *vbase, *pbase;  // k_cert_scan (n + 1 entries)
  uint8_t* mbase;        // [claimed ids 32 n][digests 64 n][certificate preimages 72 n][header preimages]
  uint64_t pre_off;      // offset of the header preimages in mbase
  uint32_t* keys;        // n + V key-cache launch entries: key index (| strict bit), signature, message
  uint4* sigs;
  uint64_t *smoff, *smlen;
  uint64_t *soff, *slen;   // 2 n SHA-512 inputs (offsets into mbase)
  uint64_t* gfirst;        // n vote groups
  uint32_t* gcnt;
  uint32_t *verr, *weight;
  const uint64_t* sig_words;  // verdict words of the key-cache launch
  const uint64_t* grp_words;  // group AND words
  uint8_t* code;              // per message: primary::DagError, 0xff = host decoder
};
hipError_t launch_cert_parse(const CertCommittee& c, const CertBufs& b, hipStream_t s);
hipError_t launch_cert_scan(const CertBufs& b, hipStream_t s);
hipError_t launch_cert_scatter(const CertCommittee& c, const CertBufs& b, hipStream_t s);
hipError_t launch_cert_verdict(const CertCommittee& c, const CertBufs& b, uint64_t gc_round, hipStream_t s);

}  // namespace nt
