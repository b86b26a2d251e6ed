// kernels.hpp -- host-side launchers of the k_*.hip kernels (used by ntcrypto.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ks_plan.hpp"
#include "nt_common.hpp"

namespace nt {

hipError_t launch_sha512_trunc32(const uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_len,
                                 uint64_t n, uint8_t* d_out32, hipStream_t s);
hipError_t launch_verify(int mode, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                         const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                         const uint32_t* d_combB, void* d_ws, uint32_t ws_slots, uint64_t* d_out_words,
                         hipStream_t s);
hipError_t launch_group_and(const uint64_t* d_first, const uint32_t* d_cnt, uint64_t G,
                            const uint64_t* d_sig_words, uint64_t* d_group_words, hipStream_t s);
// off[first[g] + q] = 32 g, len = 32 for q < cnt[g] (groups' 32-byte messages)
hipError_t launch_group_msgs(const uint64_t* d_first, const uint32_t* d_cnt, uint64_t G, uint64_t* d_off,
                             uint64_t* d_len, hipStream_t s);
hipError_t launch_sign(const uint8_t* d_seed, const uint8_t* d_msg, const uint64_t* d_off,
                       const uint64_t* d_len, uint64_t n, const uint32_t* d_combB, uint8_t* d_pk,
                       uint8_t* d_sig, uint32_t max_blocks, hipStream_t s);
// wide combs with `bits`-bit digits (kKeyCombWide or kKeyCombNarrow)
hipError_t launch_wcomb_build(int bits, const uint32_t* d_enc, uint32_t nkeys, int negate, uint32_t* d_comb,
                              uint32_t* d_meta, uint32_t* d_bases, uint32_t* d_tmp, uint32_t batch,
                              hipStream_t s);
hipError_t launch_verify_keyset(int mode, int key_bits, const uint32_t* d_key_idx, const uint8_t* d_sig, const uint8_t* d_msg,
                                const uint64_t* d_off, const uint64_t* d_len, uint64_t n, const uint32_t* d_meta,
                                const uint32_t* d_enc, const uint32_t* d_combA, uint32_t nkeys,
                                const uint32_t* d_combB, void* d_stash, void* d_sort, uint64_t* d_out_words,
                                uint32_t cus, hipStream_t s);
// scratch of launch_verify_keyset: the chunk counter and the key-grouped order (d_sort, required)
size_t keyset_sort_bytes(uint64_t n);
// the plan of one key-cache launch over n signatures on a device of `cus` CUs (ks_plan.hpp;
// NT_KEYSET_WAVES = 2 / 3 forces the waves per SIMD, NT_KEYSET_PER_LANE caps the rows per chunk)
KsPlan keyset_plan(uint64_t n, uint32_t cus);
// signatures one full round of the launch covers (host-side chunk sizing)
uint64_t keyset_round_sigs(uint32_t cus);
uint64_t verify_grid(uint64_t n, uint32_t ws_slots);  // blocks of a launch_verify
uint64_t verify_round_sigs(uint32_t cus);
uint32_t keyset_per_lane();
// per-wave stash of a launch over n signatures (d_stash above)
size_t keyset_stash_bytes(uint64_t n, uint32_t cus);
size_t wcomb_bytes_per_key(int bits);
size_t wcomb_bases_bytes_per_key(int bits);
size_t wcomb_fill_tmp_bytes_per_key(int bits);
uint32_t wcomb_fill_batch(int bits);  // keys per k_wcomb_fill launch
int bcomb_bits();                     // digit width of the base-point comb
size_t ws_bytes_per_slot();
int verify_occupancy();  // waves per SIMD of the selected verify kernel variant

}  // namespace nt
