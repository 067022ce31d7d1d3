// Host-side utilities of liblcn.so that sit on the hot path's I/O boundary.
//
// lcn_crc32c: CRC-32C (Castagnoli), the checksum of TensorFlow's tensor-bundle
// checkpoints (tensor data, BundleEntryProto.crc32c) and of the LevelDB table
// blocks of their .index file.  tf.train.Saver writes those files in the
// reference (models_att.py:256-260, 321-322) and the reference restores them
// (:457-461); lcn_amd/tf_bundle.py reads and writes the same format without
// TensorFlow and calls this for the checksums (86 MB of Adam state per save
// at F = 64, L = 3: too slow for a pure-Python CRC).
//
// Semantics of leveldb/TensorFlow crc32c::Extend(crc, data, n): `crc` is the
// unmasked CRC of the preceding bytes (0 for none).  The x86 crc32 instruction
// computes exactly this polynomial; a slicing-by-8 table is the fallback.
#include <stdint.h>
#include <string.h>

#include "../../include/lcn.h"

namespace {

uint32_t g_tab[8][256];
bool g_init = false;

void init_tables() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    g_tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) g_tab[t][i] = (g_tab[t - 1][i] >> 8) ^ g_tab[0][g_tab[t - 1][i] & 0xff];
  g_init = true;
}

uint32_t crc_soft(uint32_t l, const uint8_t* p, int64_t n) {
  if (!g_init) init_tables();
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    v ^= l;
    l = g_tab[7][v & 0xff] ^ g_tab[6][(v >> 8) & 0xff] ^ g_tab[5][(v >> 16) & 0xff] ^
        g_tab[4][(v >> 24) & 0xff] ^ g_tab[3][(v >> 32) & 0xff] ^ g_tab[2][(v >> 40) & 0xff] ^
        g_tab[1][(v >> 48) & 0xff] ^ g_tab[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n-- > 0) l = (l >> 8) ^ g_tab[0][(l ^ *p++) & 0xff];
  return l;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc_hw(uint32_t l, const uint8_t* p, int64_t n) {
  uint64_t l64 = l;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    l64 = __builtin_ia32_crc32di(l64, v);
    p += 8;
    n -= 8;
  }
  uint32_t l32 = (uint32_t)l64;
  while (n-- > 0) l32 = __builtin_ia32_crc32qi(l32, *p++);
  return l32;
}
#endif

}  // namespace

extern "C" uint32_t lcn_crc32c(uint32_t crc, const void* data, int64_t n) {
  const uint8_t* p = (const uint8_t*)data;
  uint32_t l = crc ^ 0xffffffffu;
  if (n > 0 && p) {
#if defined(__x86_64__)
    if (__builtin_cpu_supports("sse4.2")) l = crc_hw(l, p, n);
    else l = crc_soft(l, p, n);
#else
    l = crc_soft(l, p, n);
#endif
  }
  return l ^ 0xffffffffu;
}
