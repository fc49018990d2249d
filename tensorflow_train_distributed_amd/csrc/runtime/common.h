// Shared helpers for the host-side native runtime (libttd_rt.so).
//
// Everything in this library is exported through a flat C ABI (`extern "C"`,
// prefix `ttd_`) and loaded from Python with ctypes, so the library has no
// dependency on the Python or PyTorch headers and builds in seconds with g++.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#define TTD_EXPORT extern "C" __attribute__((visibility("default")))

namespace ttd {

// ---- crc32c (Castagnoli), see crc32c.cc ---------------------------------
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
inline uint32_t crc32c_value(const void* data, size_t n) { return crc32c_extend(0, data, n); }
// The "masked" form used by TFRecord framing and TensorBundle entries.
inline uint32_t crc32c_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }
inline uint32_t crc32c_unmask(uint32_t m) {
  uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}

// ---- little-endian / varint encoding (protobuf + leveldb wire format) ------
inline void put_fixed32(std::string* d, uint32_t v) {
  char b[4];
  std::memcpy(b, &v, 4);
  d->append(b, 4);
}
inline void put_fixed64(std::string* d, uint64_t v) {
  char b[8];
  std::memcpy(b, &v, 8);
  d->append(b, 8);
}
inline void put_varint64(std::string* d, uint64_t v) {
  while (v >= 0x80) {
    d->push_back(static_cast<char>((v & 0x7f) | 0x80));
    v >>= 7;
  }
  d->push_back(static_cast<char>(v));
}
inline void put_varint32(std::string* d, uint32_t v) { put_varint64(d, v); }
inline uint32_t get_fixed32(const char* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t get_fixed64(const char* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
// Returns pointer past the varint or nullptr on malformed input.
inline const char* get_varint64(const char* p, const char* limit, uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift <= 63 && p < limit; shift += 7) {
    uint64_t byte = static_cast<unsigned char>(*p++);
    r |= (byte & 0x7f) << shift;
    if (!(byte & 0x80)) {
      *v = r;
      return p;
    }
  }
  return nullptr;
}

// Thread-local last-error string exposed as ttd_last_error().
void set_error(const std::string& msg);

}  // namespace ttd
