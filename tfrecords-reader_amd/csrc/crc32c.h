// crc32c.h — CRC-32C (Castagnoli, reflected poly 0x82F63B78) algebra shared by host and device.
//
// The TFRecord framing (tensorflow/core/lib/io/record_writer) stores masked CRC-32C of the 8
// length bytes and of the payload. The reference never computes them; the build
// reports them as verdicts.
//
// Notation: U(c, M) is the table-driven reflected update of state c over bytes M with no final
// inversion. U is affine: U(c, M) = U(c, 0^|M|) ^ U(0, M), and U(c, 0^k) = c (x) x^(8k) mod P,
// where (x) is GF(2) polynomial multiplication in the reflected representation (bit 31 = x^0).
// Full CRC: crc(M) = ~U(~0, M); for |M| >= 4, U(~0, M) = U(0, M') with the first 4 bytes of M
// inverted. This is what lets a wavefront split a payload into 16-byte chunks, CRC each chunk
// from a zero state and recombine them with shift operators.
#pragma once
#include <stdint.h>

#ifndef TFRG_HD
#if defined(__HIPCC__)
#define TFRG_HD __host__ __device__
#else
#define TFRG_HD
#endif
#endif

namespace tfrg {

constexpr uint32_t kCrcPoly = 0x82F63B78u;
constexpr uint32_t kCrcMaskDelta = 0xa282ead8u;

TFRG_HD constexpr uint32_t crc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kCrcMaskDelta; }

// reflected GF(2) product a (x) b mod P
TFRG_HD inline uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma nounroll
  for (int i = 0; i < 32; ++i) {  // (a loop: the device kernels call it off their hot paths)
    p ^= (0u - ((a >> 31) & 1u)) & b;  // coefficient of x^i in a (bit 31 - i)
    a <<= 1;
    b = (b >> 1) ^ (kCrcPoly & (0u - (b & 1u)));  // b *= x
  }
  return p;
}

// x^(8n) mod P by square-and-multiply (x^0 is 0x80000000 in the reflected representation).
TFRG_HD inline uint32_t gf_xpow8(uint64_t n) {
  uint32_t result = 0x80000000u;
  uint32_t sq = 0x00800000u;  // x^8
  while (n) {
    if (n & 1) result = gf_mul(result, sq);
    sq = gf_mul(sq, sq);
    n >>= 1;
  }
  return result;
}

// base^e mod P (reflected).
TFRG_HD inline uint32_t gf_pow(uint32_t base, uint64_t e) {
  uint32_t result = 0x80000000u;
  while (e) {
    if (e & 1) result = gf_mul(result, base);
    base = gf_mul(base, base);
    e >>= 1;
  }
  return result;
}

// P has a unit constant term, so x is invertible: P = x*Q + 1  =>  x^-1 = Q = (P - 1) / x.
// In the normal representation Q = (0x1EDC6F41 >> 1) | 1 << 31 = 0x8F6E37A0; reflected below.
constexpr uint32_t kXInverse = 0x05EC76F1u;  // bit-reverse of 0x8F6E37A0

// x^(-8z): undoes z trailing zero bytes appended to a message.
TFRG_HD inline uint32_t gf_xpow8_inv(uint64_t z) { return gf_pow(kXInverse, 8 * z); }

// Byte tables T[j][v] = U(0, v followed by j zero bytes) (T[0] is the classic byte table): the
// first 4 are the slice-by-4 set, 8 slice-by-8, all 16 the slice-by-16 set (one independent
// lookup per byte of a 16-byte chunk).
struct CrcTables {
  uint32_t t[16][256];
};

inline void crc_make_tables(CrcTables* T) {
  for (uint32_t v = 0; v < 256; ++v) {
    uint32_t c = v;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kCrcPoly & (0u - (c & 1u)));
    T->t[0][v] = c;
  }
  for (uint32_t v = 0; v < 256; ++v) {
    uint32_t c = T->t[0][v];
    for (int j = 1; j < 16; ++j) {
      c = (c >> 8) ^ T->t[0][c & 0xff];
      T->t[j][v] = c;
    }
  }
}

// Tables for multiplying a state by a constant K: (c (x) K) = xor_j M[j][(c >> 8j) & 0xff],
// M[j][v] = (v << 8j) (x) K.
inline void crc_make_mul_tables(uint32_t K, uint32_t M[4][256]) {
  for (int j = 0; j < 4; ++j)
    for (uint32_t v = 0; v < 256; ++v) M[j][v] = gf_mul(v << (8 * j), K);
}

// Serial reference update (host): U(c, p[0..n))
inline uint32_t crc_update_bytes(const CrcTables& T, uint32_t c, const uint8_t* p, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) c = T.t[0][(c ^ p[i]) & 0xff] ^ (c >> 8);
  return c;
}

}  // namespace tfrg
