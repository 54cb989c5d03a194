// Request-digest kernels: one byte string per lane.
//  * Blake2b-512 (RFC 7693, unkeyed, 64-byte output): digest() at
//    src/message.rs:209-212 (blake2 0.10.6, Cargo.lock:369-375), the value
//    PrePrepare::validate_digest recomputes (src/message.rs:139-145).
//  * SHA-256 (FIPS 180-4): the request digest named by BASELINE.json north_star.
// Inputs are packed variable-length strings; lanes with different lengths
// diverge only in their block-loop trip count.
#pragma once
#include "sha512.h"

namespace pbft {

__host__ __device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

// little-endian u64 at byte offset o of a string of length len (zero past the end)
__host__ __device__ __forceinline__ uint64_t le64_masked(const uint8_t* m, uint64_t len, uint64_t o) {
  uint32_t lo = 0, hi = 0;
  if (o < len) lo = load_u32_unaligned(m + o);
  if (o + 4 < len) hi = load_u32_unaligned(m + o + 4);
  if (o + 4 > len) lo = (o >= len) ? 0u : (lo & ((1u << (8 * (len - o))) - 1u));
  if (o + 8 > len) hi = (o + 4 >= len) ? 0u : (hi & ((1u << (8 * (len - o - 4))) - 1u));
  return ((uint64_t)hi << 32) | lo;
}

__host__ __device__ __forceinline__ void blake2b_compress(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
  const uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                          0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                          0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  const uint8_t SIG[12][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
  uint64_t v[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[8 + i] = IV[i]; }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
#define B2G(a, b, c, d, x, y)          \
  v[a] = v[a] + v[b] + (x);            \
  v[d] = rotr64(v[d] ^ v[a], 32);      \
  v[c] = v[c] + v[d];                  \
  v[b] = rotr64(v[b] ^ v[c], 24);      \
  v[a] = v[a] + v[b] + (y);            \
  v[d] = rotr64(v[d] ^ v[a], 16);      \
  v[c] = v[c] + v[d];                  \
  v[b] = rotr64(v[b] ^ v[c], 63);
#pragma unroll
  for (int r = 0; r < 12; ++r) {
    B2G(0, 4, 8, 12, m[SIG[r][0]], m[SIG[r][1]]);
    B2G(1, 5, 9, 13, m[SIG[r][2]], m[SIG[r][3]]);
    B2G(2, 6, 10, 14, m[SIG[r][4]], m[SIG[r][5]]);
    B2G(3, 7, 11, 15, m[SIG[r][6]], m[SIG[r][7]]);
    B2G(0, 5, 10, 15, m[SIG[r][8]], m[SIG[r][9]]);
    B2G(1, 6, 11, 12, m[SIG[r][10]], m[SIG[r][11]]);
    B2G(2, 7, 8, 13, m[SIG[r][12]], m[SIG[r][13]]);
    B2G(3, 4, 9, 14, m[SIG[r][14]], m[SIG[r][15]]);
  }
#undef B2G
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[8 + i];
}

// Blake2b-512 of m[0..len); out: 64 bytes
__host__ __device__ __forceinline__ void blake2b512(uint8_t out[64], const uint8_t* m, uint64_t len) {
  uint64_t h[8] = {0x6a09e667f3bcc908ULL ^ 0x01010040ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  const uint64_t nblocks = len == 0 ? 1 : (len + 127) / 128;
  for (uint64_t b = 0; b < nblocks; ++b) {
    uint64_t mw[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) mw[j] = le64_masked(m, len, 128 * b + 8 * j);
    const bool last = b == nblocks - 1;
    const uint64_t t = last ? len : 128 * (b + 1);
    blake2b_compress(h, mw, t, last);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(h[i] >> (8 * j));
}

__host__ __device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// SHA-256 of m[0..len); out: 32 bytes
__host__ __device__ __forceinline__ void sha256(uint8_t out[32], const uint8_t* m, uint64_t len) {
  const uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t H[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint64_t nblocks = (len + 9 + 63) / 64;
  for (uint64_t b = 0; b < nblocks; ++b) {
    uint32_t W[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t o = 64 * b + 4 * j;
      uint32_t w = 0;
      if (o < len) w = load_u32_unaligned(m + o);
      if (o + 4 > len) w = (o >= len) ? 0u : (w & ((1u << (8 * (len - o))) - 1u));
      if (o <= len && len < o + 4) w |= 0x80u << (8 * (len - o));
      W[j] = bswap32(w);
    }
    if (b == nblocks - 1) {
      W[14] = (uint32_t)((len * 8) >> 32);
      W[15] = (uint32_t)(len * 8);
    }
    uint32_t a = H[0], bb = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      uint32_t w;
      if (t < 16) {
        w = W[t];
      } else {
        const uint32_t w15 = W[(t - 15) & 15], w2 = W[(t - 2) & 15];
        const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
        const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
        w = W[t & 15] + s0 + W[(t - 7) & 15] + s1;
        W[t & 15] = w;
      }
      const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t T1 = h + S1 + ch + K[t] + w;
      const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
      const uint32_t mj = (a & bb) ^ (c & (a ^ bb));
      const uint32_t T2 = S0 + mj;
      h = g; g = f; f = e; e = d + T1; d = c; c = bb; bb = a; a = T1 + T2;
    }
    H[0] += a; H[1] += bb; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(H[i] >> (24 - 8 * j));
}

}  // namespace pbft
