// CRC-32C (Castagnoli polynomial 0x82F63B78), used by the TFRecord/Event framing and
// by TensorBundle V2 entries (the reference triggers both via
// MonitoredTrainingSession's CheckpointSaverHook / SummarySaverHook,
// /root/reference/distribute_training.py:209-215).
//
// Uses the SSE4.2 `crc32` instruction when the CPU has it (8 bytes per instruction),
// otherwise a slicing-by-8 table implementation.
#include "common.h"

#include <mutex>
#if defined(__x86_64__)
#include <cpuid.h>
#endif

namespace ttd {
namespace {

uint32_t g_table[8][256];
std::once_flag g_once;
bool g_have_sse42 = false;

void init_tables() {
  const uint32_t poly = 0x82F63B78u;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
    g_table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = g_table[0][i];
    for (int t = 1; t < 8; ++t) {
      c = g_table[0][c & 0xff] ^ (c >> 8);
      g_table[t][i] = c;
    }
  }
#if defined(__x86_64__)
  unsigned a, b, c, d;
  if (__get_cpuid(1, &a, &b, &c, &d)) g_have_sse42 = (c & bit_SSE4_2) != 0;
#endif
}

uint32_t extend_sw(uint32_t crc, const unsigned char* p, size_t n) {
  uint32_t c = crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = g_table[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    --n;
  }
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    w ^= c;
    c = g_table[7][w & 0xff] ^ g_table[6][(w >> 8) & 0xff] ^ g_table[5][(w >> 16) & 0xff] ^
        g_table[4][(w >> 24) & 0xff] ^ g_table[3][(w >> 32) & 0xff] ^ g_table[2][(w >> 40) & 0xff] ^
        g_table[1][(w >> 48) & 0xff] ^ g_table[0][w >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = g_table[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return c;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t extend_hw(uint32_t crc, const unsigned char* p, size_t n) {
  uint64_t c = crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = __builtin_ia32_crc32qi(static_cast<uint32_t>(c), *p++);
    --n;
  }
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    c = __builtin_ia32_crc32di(c, w);
    p += 8;
    n -= 8;
  }
  while (n--) c = __builtin_ia32_crc32qi(static_cast<uint32_t>(c), *p++);
  return static_cast<uint32_t>(c);
}
#endif

}  // namespace

uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  std::call_once(g_once, init_tables);
  const auto* p = static_cast<const unsigned char*>(data);
  uint32_t c = crc ^ 0xffffffffu;
#if defined(__x86_64__)
  if (g_have_sse42) return extend_hw(c, p, n) ^ 0xffffffffu;
#endif
  return extend_sw(c, p, n) ^ 0xffffffffu;
}

namespace {
thread_local std::string g_last_error;
}
void set_error(const std::string& msg) { g_last_error = msg; }

}  // namespace ttd

TTD_EXPORT const char* ttd_last_error() { return ttd::g_last_error.c_str(); }
TTD_EXPORT uint32_t ttd_crc32c_extend(uint32_t crc, const void* data, size_t n) {
  return ttd::crc32c_extend(crc, data, n);
}
TTD_EXPORT uint32_t ttd_crc32c_mask(uint32_t c) { return ttd::crc32c_mask(c); }
TTD_EXPORT uint32_t ttd_crc32c_unmask(uint32_t c) { return ttd::crc32c_unmask(c); }
