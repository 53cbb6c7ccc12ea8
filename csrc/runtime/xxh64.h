// XXH64 (public algorithm by Yann Collet), used for every identifier digest.
// Must agree with igaming_platform_amd/utils/hashing.py (tests cross-check both).
#pragma once
#include <cstdint>
#include <cstring>
#include <string_view>

namespace igp {

constexpr uint64_t XP1 = 0x9E3779B185EBCA87ULL, XP2 = 0xC2B2AE3D27D4EB4FULL,
                   XP3 = 0x165667B19E3779F9ULL, XP4 = 0x85EBCA77C2B2AE63ULL,
                   XP5 = 0x27D4EB2F165667C5ULL;

constexpr uint64_t SEED_ACCOUNT = 0x41434354, SEED_DEVICE = 0x44455649,
                   SEED_FINGERPRINT = 0x46505249, SEED_IP = 0x49504144, SEED_EMAIL = 0x454D4149;

inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return v; }
inline uint32_t rd32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
inline uint64_t xround(uint64_t acc, uint64_t lane) { acc += lane * XP2; acc = rotl64(acc, 31); return acc * XP1; }
inline uint64_t xmerge(uint64_t acc, uint64_t v) { acc ^= xround(0, v); return acc * XP1 + XP4; }

inline uint64_t xxh64(const void* data, size_t len, uint64_t seed) {
  const uint8_t* p = (const uint8_t*)data;
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    const uint8_t* lim = end - 32;
    do {
      v1 = xround(v1, rd64(p)); v2 = xround(v2, rd64(p + 8));
      v3 = xround(v3, rd64(p + 16)); v4 = xround(v4, rd64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xmerge(h, v1); h = xmerge(h, v2); h = xmerge(h, v3); h = xmerge(h, v4);
  } else {
    h = seed + XP5;
  }
  h += uint64_t(len);
  while (p + 8 <= end) { h ^= xround(0, rd64(p)); h = rotl64(h, 27) * XP1 + XP4; p += 8; }
  if (p + 4 <= end) { h ^= uint64_t(rd32(p)) * XP1; h = rotl64(h, 23) * XP2 + XP3; p += 4; }
  while (p < end) { h ^= uint64_t(*p) * XP5; h = rotl64(h, 11) * XP1; ++p; }
  h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32;
  return h;
}

// Identifier digest: 0 = absent (empty string); a real 0 digest maps to 1.
inline uint64_t id_hash(std::string_view s, uint64_t seed) {
  if (s.empty()) return 0;
  uint64_t h = xxh64(s.data(), s.size(), seed);
  return h ? h : 1;
}

}  // namespace igp
