// SHA-512 (FIPS 180-4) for one lane, specialised for the Ed25519 challenge
// hash k = SHA-512(R || A || M) of ed25519-dalek 1.0.1 verify_strict (sha2 0.9.9,
// Cargo.lock:2784-2787).  R and A are 32 bytes each (4 big-endian words);
// M is fetched from HBM as aligned dwords and re-aligned per lane, so the
// message layout in memory can have any byte stride.
#pragma once
#include "fe25519.h"

namespace pbft {

// 64-bit rotate: two v_alignbit_b32 on gfx950 (the generic form lowers to
// 2 x 64-bit shifts + 2 ORs).  n is a compile-time constant at every call site.
__host__ __device__ __forceinline__ uint64_t ror64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t nlo, nhi;
  if (n < 32) {
    nlo = __builtin_amdgcn_alignbit(hi, lo, n);
    nhi = __builtin_amdgcn_alignbit(lo, hi, n);
  } else {
    nlo = __builtin_amdgcn_alignbit(lo, hi, n - 32);
    nhi = __builtin_amdgcn_alignbit(hi, lo, n - 32);
  }
  return ((uint64_t)nhi << 32) | nlo;
#else
  return (x >> n) | (x << (64 - n));
#endif
}
// 3-input VOP3 logic on gfx950: one v_bitop3_b32 instead of two or three VOP2 ops (LLVM keeps the VOP2
// pairs on its own).  Sigma functions XOR three rotations (table 0x96); Maj is table 0xE8.
__host__ __device__ __forceinline__ uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));  // gfx950 has no v_xor3
  return r;
#else
  return a ^ b ^ c;
#endif
}
__host__ __device__ __forceinline__ uint32_t maj32(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return (a & b) | (c & (a | b));
#endif
}
__host__ __device__ __forceinline__ uint32_t ab32(uint32_t hi, uint32_t lo, int n) {  // (hi:lo) >> n, low word
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, n);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> n);
#endif
}
#define LO32(x) ((uint32_t)(x))
#define HI32(x) ((uint32_t)((x) >> 32))
// pack two halves as a register pair (a bitcast, not shift + or: LLVM would turn "(h << 32) | l" into an add
// and re-associate it with the round's 64-bit additions, doubling them)
__host__ __device__ __forceinline__ uint64_t MK64(uint32_t h, uint32_t l) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 v = {l, h};
  return __builtin_bit_cast(uint64_t, v);
#else
  return ((uint64_t)h << 32) | l;
#endif
}
// Sigma1(e) = ror14 ^ ror18 ^ ror41, Sigma0(a) = ror28 ^ ror34 ^ ror39 (ror41 = ror(9) of the swapped halves...)
__host__ __device__ __forceinline__ uint64_t big_sigma1(uint64_t x) {
  const uint32_t l = LO32(x), h = HI32(x);
  return MK64(xor3_32(ab32(l, h, 14), ab32(l, h, 18), ab32(h, l, 9)),
              xor3_32(ab32(h, l, 14), ab32(h, l, 18), ab32(l, h, 9)));
}
__host__ __device__ __forceinline__ uint64_t big_sigma0(uint64_t x) {
  const uint32_t l = LO32(x), h = HI32(x);
  return MK64(xor3_32(ab32(l, h, 28), ab32(h, l, 2), ab32(h, l, 7)),
              xor3_32(ab32(h, l, 28), ab32(l, h, 2), ab32(l, h, 7)));
}
// sigma0(w) = ror1 ^ ror8 ^ (w >> 7), sigma1(w) = ror19 ^ ror61 ^ (w >> 6)
__host__ __device__ __forceinline__ uint64_t small_sigma0(uint64_t x) {
  const uint32_t l = LO32(x), h = HI32(x);
  return MK64(xor3_32(ab32(l, h, 1), ab32(l, h, 8), h >> 7), xor3_32(ab32(h, l, 1), ab32(h, l, 8), ab32(h, l, 7)));
}
__host__ __device__ __forceinline__ uint64_t small_sigma1(uint64_t x) {
  const uint32_t l = LO32(x), h = HI32(x);
  return MK64(xor3_32(ab32(l, h, 19), ab32(h, l, 29), h >> 6), xor3_32(ab32(h, l, 19), ab32(l, h, 29), ab32(h, l, 6)));
}
__host__ __device__ __forceinline__ uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) {
  return MK64(maj32(HI32(a), HI32(b), HI32(c)), maj32(LO32(a), LO32(b), LO32(c)));
}

__host__ __device__ __forceinline__ uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

#define SHA512_K_TABLE                                                                                       \
  {0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,               \
   0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,               \
   0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,               \
   0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,               \
   0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,               \
   0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,               \
   0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,               \
   0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,               \
   0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,               \
   0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,               \
   0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,               \
   0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,               \
   0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,               \
   0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,               \
   0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,               \
   0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,               \
   0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,               \
   0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,               \
   0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,               \
   0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL}

__host__ __device__ __forceinline__ void sha512_init(uint64_t H[8]) {
  H[0] = 0x6a09e667f3bcc908ULL; H[1] = 0xbb67ae8584caa73bULL; H[2] = 0x3c6ef372fe94f82bULL;
  H[3] = 0xa54ff53a5f1d36f1ULL; H[4] = 0x510e527fade682d1ULL; H[5] = 0x9b05688c2b3e6c1fULL;
  H[6] = 0x1f83d9abfb41bd6bULL; H[7] = 0x5be0cd19137e2179ULL;
}

#if defined(__HIP_DEVICE_COMPILE__)
__constant__ static const uint64_t SHA512_K[80] = SHA512_K_TABLE;
#endif

// One compression; W holds the 16 big-endian message words of the block.
// The 80 rounds run as 5 iterations of a 16-round unrolled body: the message
// schedule indices (t mod 16) and the a..h renaming (16 = 0 mod 8) stay
// compile-time constants while the code stays ~5x smaller than a full unroll
// (instruction-cache footprint); K[t] is a wave-uniform scalar load.
__host__ __device__ __forceinline__ void sha512_round(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d,
                                                      uint64_t& e, uint64_t& f, uint64_t& g, uint64_t& h,
                                                      uint64_t k, uint64_t w) {
  const uint64_t S1 = big_sigma1(e);
  const uint64_t ch = (e & f) ^ (~e & g);
  const uint64_t T1 = h + S1 + ch + k + w;
  const uint64_t S0 = big_sigma0(a);
  const uint64_t mj = maj64(a, b, c);
  h = g; g = f; f = e; e = d + T1; d = c; c = b; b = a; a = T1 + S0 + mj;
}

// PEEL: the first 16 schedule rounds are unrolled too, for a final block whose
// words are mostly compile-time constants (the padding of a fixed-length
// message): the zero and constant words then fold out of the schedule
// (~150 instructions fewer for the 2nd block of the 149-byte R || A || M).
template <bool PEEL = false>
__host__ __device__ __forceinline__ void sha512_compress(uint64_t H[8], uint64_t W[16]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t* K = SHA512_K;
#else
  const uint64_t K[80] = SHA512_K_TABLE;
#endif
  uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
  for (int j = 0; j < 16; ++j) sha512_round(a, b, c, d, e, f, g, h, K[j], W[j]);
  auto sched16 = [&](int t0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t w15 = W[(j + 1) & 15], w2 = W[(j + 14) & 15];
      const uint64_t s0 = small_sigma0(w15);
      const uint64_t s1 = small_sigma1(w2);
      W[j] = W[j] + s0 + W[(j + 9) & 15] + s1;
      sha512_round(a, b, c, d, e, f, g, h, K[t0 + j], W[j]);
    }
  };
  int t0 = 16;
  if constexpr (PEEL) {
    sched16(16);
    t0 = 32;
  }
#pragma nounroll
  for (; t0 < 80; t0 += 16) sched16(t0);
  H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

// 4 message bytes starting at an arbitrary byte address (little-endian u32).
// Reads the two aligned dwords that cover them.
__host__ __device__ __forceinline__ uint32_t load_u32_unaligned(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8u;
  const uint32_t lo = q[0];
  const uint32_t hi = sh ? q[1] : 0u;
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
}

// Big-endian 64-bit word j (j >= 0) of the padded stream M || 0x80 || 0...,
// without the length field.  LEN < 0 means the length is the runtime `len`.
__host__ __device__ __forceinline__ uint64_t msg_word(const uint8_t* m, int len, int j) {
  const int o = 8 * j;
  uint32_t w0 = 0, w1 = 0;
  if (o < len) w0 = load_u32_unaligned(m + o);
  if (o + 4 < len) w1 = load_u32_unaligned(m + o + 4);
  // mask bytes >= len and insert the 0x80 terminator at byte `len`
  const int r0 = len - o, r1 = len - o - 4;
  if (r0 < 4) w0 = (r0 <= 0) ? 0u : (w0 & ((1u << (8 * r0)) - 1u));
  if (r0 >= 0 && r0 < 4) w0 |= 0x80u << (8 * r0);
  if (r1 < 4) w1 = (r1 <= 0) ? 0u : (w1 & ((1u << (8 * r1)) - 1u));
  if (r1 >= 0 && r1 < 4) w1 |= 0x80u << (8 * r1);
  return ((uint64_t)bswap32(w0) << 32) | bswap32(w1);
}

// SHA-512(pre || M) where pre is NPRE (32 or 64) bytes held in registers as
// little-endian words and M is fetched from memory.  out: 16 LE words of the
// digest read as a little-endian 512-bit integer (Scalar::from_hash input).
template <int NPRE, int LEN>
__host__ __device__ __forceinline__ void sha512_pre(uint32_t out[16], const uint32_t pre[NPRE / 4],
                                                    const uint8_t* m, int len_rt) {
  static_assert(NPRE == 32 || NPRE == 64, "prefix is 32 or 64 bytes");
  constexpr int NW = NPRE / 8;  // prefix words (64-bit)
  const int len = LEN >= 0 ? LEN : len_rt;
  uint64_t H[8];
  sha512_init(H);
  const int total = NPRE + len;
  const int nblocks = (total + 17 + 127) / 128;
  uint64_t W[16];
#pragma unroll
  for (int t = 0; t < NW; ++t) W[t] = ((uint64_t)bswap32(pre[2 * t]) << 32) | bswap32(pre[2 * t + 1]);
#pragma unroll
  for (int t = NW; t < 16; ++t) W[t] = msg_word(m, len, t - NW);
  if (nblocks == 1) {
    W[14] = 0;
    W[15] = (uint64_t)total * 8u;
  }
  sha512_compress(H, W);
  for (int b = 1; b < nblocks; ++b) {
#pragma unroll
    for (int t = 0; t < 16; ++t) W[t] = msg_word(m, len, 16 * b - NW + t);
    if (b == nblocks - 1) {
      W[14] = 0;
      W[15] = (uint64_t)total * 8u;
      if constexpr (LEN >= 0) {  // fixed length: the last block's padding words are constants
        sha512_compress<true>(H, W);
        continue;
      }
    }
    sha512_compress(H, W);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    out[2 * i] = bswap32((uint32_t)(H[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)H[i]);
  }
}

// k-hash: SHA-512(R || A || M), r and a as 8 LE words each.
template <int LEN>
__host__ __device__ __forceinline__ void sha512_ram(uint32_t out[16], const uint32_t r[8], const uint32_t a[8],
                                                    const uint8_t* m, int len_rt) {
  uint32_t pre[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { pre[i] = r[i]; pre[8 + i] = a[i]; }
  sha512_pre<64, LEN>(out, pre, m, len_rt);
}

// ---- the signed envelope's share of the hash, once per envelope -------------------------------
// For the 85-byte envelope, R || A || M is 149 bytes: block 2 holds only M[64..84], the 0x80
// terminator and the length, so its message schedule W[16..79] is a function of the ENVELOPE alone.
// In a PBFT round every envelope is signed by all n replicas (the votes form, include/pbft_verify.h
// pbft_verify_votes): env_sched computes W[t] + K[t], t = 16..79, once per envelope (512 B), and the
// per-signature hash reads them instead of expanding the schedule -- the same SHA-512, ~1.3k fewer
// VALU instructions per signature.
#define SHA_ENV_WORDS 64  // W[t] + K[t] for t = 16 .. 79
#ifndef PBFT_SALU_SCHED
#define PBFT_SALU_SCHED 1  // A/B: 0 = no wave-uniform scalar schedule
#endif
__host__ __device__ __forceinline__ void sha512_env_block2(uint64_t W[16], const uint8_t* m) {
  // bytes 128 .. 148 of R || A || M = M[64 .. 84]; then 0x80, zeros, the 128-bit length 149 * 8
#pragma unroll
  for (int t = 0; t < 16; ++t) W[t] = t < 3 ? msg_word(m, 85, 8 + t) : 0u;
  W[15] = 149u * 8u;
}
__host__ __device__ __forceinline__ void sha512_env_sched(uint64_t wk[SHA_ENV_WORDS], const uint8_t* m) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t* K = SHA512_K;
#else
  const uint64_t K[80] = SHA512_K_TABLE;
#endif
  uint64_t W[16];
  sha512_env_block2(W, m);
#pragma unroll
  for (int t = 16; t < 80; ++t) {
    const int j = t & 15;
    W[j] = W[j] + small_sigma0(W[(j + 1) & 15]) + W[(j + 9) & 15] + small_sigma1(W[(j + 14) & 15]);
    wk[t - 16] = W[j] + K[t];
  }
}
// SHA-512(R || A || M) for an 85-byte M.  Block 2 (M[64..84] + padding) needs its message schedule
// W[16..79], a function of the envelope alone, which comes
//  * from the SCALAR unit when every lane of the wave signs the same envelope (a round's signatures are
//    grouped by envelope, n replicas each): the schedule is computed once per wave in SGPRs, beside the
//    other waves' VALU work, and enters each round as a scalar operand;
//  * else from wk (the votes form's per-envelope table, env_sched_kernel), if given;
//  * else per lane, as sha512_compress does.
// Same hash in every case (host harness: test_sha512_ram_envelope_schedule; GPU: golden + round tests).
__host__ __device__ __forceinline__ uint64_t rotr64_s(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
__host__ __device__ __forceinline__ void sha512_ram85(uint32_t out[16], const uint32_t r[8], const uint32_t a[8],
                                                      const uint8_t* m, const uint64_t* __restrict__ wk) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t* K = SHA512_K;
#else
  const uint64_t K[80] = SHA512_K_TABLE;
#endif
  uint64_t H[8];
  sha512_init(H);
  uint64_t W[16];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    W[t] = ((uint64_t)bswap32(r[2 * t]) << 32) | bswap32(r[2 * t + 1]);
    W[4 + t] = ((uint64_t)bswap32(a[2 * t]) << 32) | bswap32(a[2 * t + 1]);
  }
#pragma unroll
  for (int t = 8; t < 16; ++t) W[t] = msg_word(m, 85, t - 8);
  sha512_compress(H, W);
  sha512_env_block2(W, m);
  uint64_t a_ = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
  for (int j = 0; j < 16; ++j) sha512_round(a_, b, c, d, e, f, g, h, K[j], W[j]);
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t w0l = (uint32_t)__builtin_amdgcn_readfirstlane((int)LO32(W[0]));
  const uint32_t w0h = (uint32_t)__builtin_amdgcn_readfirstlane((int)HI32(W[0]));
  const uint32_t w1l = (uint32_t)__builtin_amdgcn_readfirstlane((int)LO32(W[1]));
  const uint32_t w1h = (uint32_t)__builtin_amdgcn_readfirstlane((int)HI32(W[1]));
  const uint32_t w2l = (uint32_t)__builtin_amdgcn_readfirstlane((int)LO32(W[2]));
  const uint32_t w2h = (uint32_t)__builtin_amdgcn_readfirstlane((int)HI32(W[2]));
  const bool same = LO32(W[0]) == w0l && HI32(W[0]) == w0h && LO32(W[1]) == w1l && HI32(W[1]) == w1h &&
                    LO32(W[2]) == w2l && HI32(W[2]) == w2h;
  if (PBFT_SALU_SCHED && __all(same)) {
    // wave-uniform schedule: plain 64-bit shifts (s_lshr_b64 / s_lshl_b64 / s_or_b64 on the SALU)
    uint64_t Ws[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) Ws[t] = 0;
    Ws[0] = ((uint64_t)w0h << 32) | w0l;
    Ws[1] = ((uint64_t)w1h << 32) | w1l;
    Ws[2] = ((uint64_t)w2h << 32) | w2l;
    Ws[15] = 149u * 8u;
#pragma nounroll
    for (int t0 = 16; t0 < 80; t0 += 16) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint64_t x15 = Ws[(j + 1) & 15], x2 = Ws[(j + 14) & 15];
        const uint64_t s0 = rotr64_s(x15, 1) ^ rotr64_s(x15, 8) ^ (x15 >> 7);
        const uint64_t s1 = rotr64_s(x2, 19) ^ rotr64_s(x2, 61) ^ (x2 >> 6);
        Ws[j] = Ws[j] + s0 + Ws[(j + 9) & 15] + s1;
        sha512_round(a_, b, c, d, e, f, g, h, 0u, Ws[j] + K[t0 + j]);
      }
    }
  } else
#endif
  if (wk) {
#pragma nounroll
    for (int t0 = 0; t0 < SHA_ENV_WORDS; t0 += 16) {
      uint64_t kw[16];
#if defined(__HIP_DEVICE_COMPILE__)
      const uint4* p4 = (const uint4*)(wk + t0);  // rows are 512-B aligned: 8 x 16-B loads per 16 rounds
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint4 v = p4[q];
        kw[2 * q] = MK64(v.y, v.x);
        kw[2 * q + 1] = MK64(v.w, v.z);
      }
#else
#pragma unroll
      for (int j = 0; j < 16; ++j) kw[j] = wk[t0 + j];
#endif
#pragma unroll
      for (int j = 0; j < 16; ++j) sha512_round(a_, b, c, d, e, f, g, h, 0u, kw[j]);  // T1 = h + S1 + ch + (K + W)
    }
  } else {
#pragma nounroll
    for (int t0 = 16; t0 < 80; t0 += 16) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        W[j] = W[j] + small_sigma0(W[(j + 1) & 15]) + W[(j + 9) & 15] + small_sigma1(W[(j + 14) & 15]);
        sha512_round(a_, b, c, d, e, f, g, h, K[t0 + j], W[j]);
      }
    }
  }
  H[0] += a_; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    out[2 * i] = bswap32((uint32_t)(H[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)H[i]);
  }
}
// the votes form's entry point (kept for the host harness): the per-envelope table
__host__ __device__ __forceinline__ void sha512_ram_env(uint32_t out[16], const uint32_t r[8], const uint32_t a[8],
                                                        const uint8_t* m, const uint64_t* __restrict__ wk) {
  sha512_ram85(out, r, a, m, wk);
}

}  // namespace pbft
