/*
 * balloon_ref.c — Balloon hashing over BLAKE3 (TEST INFRASTRUCTURE ONLY, see oracle.h).
 *
 * Why it is here: the reference's only in-repo BLAKE3 known answers are in
 * crates/crypto/src/keys/hashing.rs — DERIVE_B3_EXPECTED (:210-213, one-block inputs) and
 * HASH_B3BALLOON_EXPECTED / HASH_B3BALLOON_WITH_SECRET_EXPECTED (:180-208): the password
 * hash `Balloon::<blake3::Hasher>` (hashing.rs:95-114) with params s_cost = 131,072 / 262,144
 * / 524,288, t_cost 2, p_cost 1 (:58-65), password "password" (:130), salt 0xFF x 16
 * (:138-141), secret 0x55 x 18 (:143-146).  Those runs feed BLAKE3 millions of streamed
 * multi-piece inputs of 48-106 bytes (one and two 64-B blocks with CHUNK_START/CHUNK_END in
 * different blocks), so they pin the chunk-internal block chaining that the one-block
 * derive_key vector does not.
 *
 * The algorithm is the Balloon construction of Boneh, Corrigan-Gibbs and Schechter
 * (ePrint 2016/027, §3.1) as the `balloon-hash` 0.4.0 crate (Cargo.lock:920-928) applies it
 * to a `Digest`: a buffer of s_cost 32-B blocks; cnt a u64 counter hashed little-endian in
 * front of every block hash; delta = 3 dependencies per block; `other` = the little-endian
 * integer of hash(cnt, salt[, secret], idx_block) mod s_cost, idx_block = hash(le64 t, le64
 * m, le64 i); the output is the last block.  The optional secret enters the first block's
 * hash (after the salt) and the `other` index hashes only — which of the hashes take it is
 * the one thing the paper leaves to the implementation, and the reference's
 * WITH_SECRET KATs single it out: of the 64 combinations of placing it in each hash, exactly
 * this one reproduces them.  Restated from the paper and the KATs (the crate's source is not
 * vendored in the reference): tests/test_oracle.py reproduces all six KATs.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static void le64(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
}

/* BLAKE3 of the concatenation of up to 5 pieces (== Hasher::update per piece) */
static void h5(uint8_t out[32], const uint8_t* a, size_t la, const uint8_t* b, size_t lb,
               const uint8_t* c, size_t lc, const uint8_t* d, size_t ld, const uint8_t* e,
               size_t le) {
  uint8_t buf[512];
  size_t n = 0;
  const uint8_t* p[5] = {a, b, c, d, e};
  const size_t l[5] = {la, lb, lc, ld, le};
  for (int i = 0; i < 5; i++)
    if (l[i]) { memcpy(buf + n, p[i], l[i]); n += l[i]; }
  orc_blake3(buf, n, out, 32);
}

int orc_balloon_blake3(const uint8_t* pwd, size_t pwd_len, const uint8_t* salt, size_t salt_len,
                       const uint8_t* secret, size_t secret_len, uint64_t s_cost, uint64_t t_cost,
                       uint8_t out[32]) {
  if (s_cost == 0 || pwd_len + salt_len + secret_len + 8 > 512 || salt_len + secret_len > 400)
    return -1;
  uint8_t(*buf)[32] = malloc(s_cost * 32);
  if (!buf) return -1;
  uint64_t cnt = 0;
  uint8_t c8[8];
  /* 1. expand: buf[0] = H(cnt++, pwd, salt[, secret]); buf[m] = H(cnt++, buf[m-1]) */
  le64(c8, cnt++);
  h5(buf[0], c8, 8, pwd, pwd_len, salt, salt_len, secret, secret_len, NULL, 0);
  for (uint64_t m = 1; m < s_cost; m++) {
    le64(c8, cnt++);
    h5(buf[m], c8, 8, buf[m - 1], 32, NULL, 0, NULL, 0, NULL, 0);
  }
  /* 2. mix */
  for (uint64_t t = 0; t < t_cost; t++) {
    for (uint64_t m = 0; m < s_cost; m++) {
      const uint8_t* prev = buf[m ? m - 1 : s_cost - 1];
      le64(c8, cnt++);
      h5(buf[m], c8, 8, prev, 32, buf[m], 32, NULL, 0, NULL, 0);
      for (uint64_t i = 0; i < 3; i++) {
        uint8_t ints[24], idx[32], oth[32];
        le64(ints, t);
        le64(ints + 8, m);
        le64(ints + 16, i);
        orc_blake3(ints, 24, idx, 32);
        le64(c8, cnt++);
        h5(oth, c8, 8, salt, salt_len, secret, secret_len, idx, 32, NULL, 0);
        /* the 256-bit little-endian integer mod s_cost */
        uint64_t r = 0;
        for (int k = 31; k >= 0; k--) r = (uint64_t)(((__uint128_t)r << 8 | oth[k]) % s_cost);
        le64(c8, cnt++);
        h5(buf[m], c8, 8, buf[m], 32, buf[r], 32, NULL, 0, NULL, 0);
      }
    }
  }
  memcpy(out, buf[s_cost - 1], 32);
  free(buf);
  return 0;
}
