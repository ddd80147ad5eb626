// GF(2) folding tables for the reflected CRC-32 register (host side).
//
// The ICRC is zlib's CRC-32 (reflected polynomial 0xEDB88320) of
// FF x 8 || masked frame (datenlord/roce-sim src/roce.py:204-218).  With the
// register convention of zlib ("r = T[(r ^ b) & 0xff] ^ (r >> 8)"), processing
// one zero bit is the linear map r -> (r >> 1) ^ (r & 1 ? P : 0), i.e.
// multiplication by x modulo the CRC polynomial in the bit-reflected basis.
// Everything the kernels do is built from that map:
//
//   Mul(m)       = x^m mod P as a 32 x 32 bit-matrix (m may be negative: x is
//                  invertible because P has a constant term),
//   table set    = four 256-entry tables Tab[k][b] = Mul(m)(b << 8k), so that
//                  Mul(m)(r) = Tab[0][r & 255] ^ Tab[1][r >> 8 & 255]
//                            ^ Tab[2][r >> 16 & 255] ^ Tab[3][r >> 24].
//
// Processing a dword w then z zero bytes from register r gives
// Mul(32 + 8z)(r ^ w); Mul(32) is zlib's slice-by-4 and is checked against a
// byte-wise CRC in self_test().
#pragma once

#include <array>
#include <cstdint>

namespace ricrc {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr uint32_t kSeedRegister = 0xDEBB20E3u;  // register after FF x 8 from ~0

struct Mat {
  std::array<uint32_t, 32> col{};  // col[b] = image of basis vector (1 << b)
  uint32_t apply(uint32_t v) const {
    uint32_t r = 0;
    for (int b = 0; b < 32; ++b)
      if (v >> b & 1u) r ^= col[b];
    return r;
  }
  Mat compose(const Mat& rhs) const {  // (*this) o rhs
    Mat o;
    for (int b = 0; b < 32; ++b) o.col[b] = apply(rhs.col[b]);
    return o;
  }
};

inline uint32_t mul_x(uint32_t r) { return (r >> 1) ^ ((r & 1u) ? kPoly : 0u); }
inline uint32_t mul_xinv(uint32_t r) {
  uint32_t top = r >> 31;  // bit 31 of mul_x's output is the dropped lsb
  return ((r ^ (top ? kPoly : 0u)) << 1) | top;
}

inline Mat identity() {
  Mat m;
  for (int b = 0; b < 32; ++b) m.col[b] = 1u << b;
  return m;
}

inline Mat mul_power(long long m) {
  Mat base;
  for (int b = 0; b < 32; ++b) base.col[b] = (m >= 0) ? mul_x(1u << b) : mul_xinv(1u << b);
  unsigned long long e = (m >= 0) ? (unsigned long long)m : (unsigned long long)(-m);
  Mat acc = identity();
  while (e) {
    if (e & 1ull) acc = acc.compose(base);
    base = base.compose(base);
    e >>= 1;
  }
  return acc;
}

// Tab[k][b] = Mul(m)(b << 8k), flattened [k * 256 + b].
inline void table_set(long long m, uint32_t* out1024) {
  Mat M = mul_power(m);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) out1024[k * 256 + b] = M.apply(b << (8 * k));
}

inline uint32_t apply_set(const uint32_t* t, uint32_t r) {
  return t[r & 255] ^ t[256 + (r >> 8 & 255)] ^ t[512 + (r >> 16 & 255)] ^ t[768 + (r >> 24)];
}

// Host-side consistency check of the table algebra (runs once per context):
// slice-by-4 from Mul(32) must equal a byte-wise CRC, and Mul(m) o Mul(-m) = I.
inline bool self_test() {
  uint32_t t[1024];
  table_set(32, t);
  uint32_t r1 = 0x12345678u, r2 = r1;
  const uint32_t words[3] = {0xDEADBEEFu, 0x00000000u, 0x89ABCDEFu};
  for (uint32_t w : words) {
    r1 = apply_set(t, r1 ^ w);
    for (int byte = 0; byte < 4; ++byte) {
      r2 ^= (w >> (8 * byte)) & 255u;
      for (int i = 0; i < 8; ++i) r2 = mul_x(r2);
    }
  }
  if (r1 != r2) return false;
  Mat a = mul_power(2048).compose(mul_power(-2048));
  for (int b = 0; b < 32; ++b)
    if (a.col[b] != (1u << b)) return false;
  return true;
}

}  // namespace ricrc
