// Host build of the GPU inflate core (tmlibrary_amd/csrc/inflate_core.h) for
// tests/test_inflate_host.py: the same decode code, run lane by lane on the
// CPU, so its output can be compared with zlib byte for byte without a GPU.
//   inflate_host TABLE BLOB RAW_BYTES OUT STATUS
// TABLE: tmh_zchunk records; BLOB: the compressed bytes; writes RAW_BYTES of
// decompressed output and one int32 status per chunk.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static inline uint32_t bitrev32(uint32_t x) {
  x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
  x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
  x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
  x = ((x >> 8) & 0x00FF00FFu) | ((x & 0x00FF00FFu) << 8);
  return (x >> 16) | (x << 16);
}
#define TMH_ZDEV static inline
#define TMH_ZHD static inline
#define TMH_ZCONST static const
#define TMH_ZBITREV32(x) bitrev32(x)
#define __restrict__
#define TMH_ZGLOBAL
#define TMH_ZKEEP(v) (void)(v)
#define TMH_ZBFE(x, n) ((n) ? ((x) & (0xFFFFFFFFu >> (32 - (n)))) : 0u)
#define TMH_ZLD16(p, a, b, c, d) \
  do {                           \
    uint32_t v_[4];              \
    memcpy(v_, (p), 16);         \
    (a) = v_[0];                 \
    (b) = v_[1];                 \
    (c) = v_[2];                 \
    (d) = v_[3];                 \
  } while (0)
#define TMH_ZLDS16(p, a, b, c, d)          \
  do {                                     \
    const uint32_t v_[4] = {(a), (b), (c), (d)}; \
    memcpy((p), v_, 16);                   \
  } while (0)
#define TMH_ZANY(pred) (pred)
#define TMH_ZST8(p, a, b)                                    \
  do {                                                       \
    const uint32_t v8_[2] = {(uint32_t)(a), (uint32_t)(b)};  \
    memcpy((p), v8_, 8);                                     \
  } while (0)
#include "../tmlibrary_amd/csrc/inflate_core.h"

static std::vector<uint8_t> slurp(const char* p) {
  FILE* f = fopen(p, "rb");
  if (!f) exit(2);
  std::vector<uint8_t> v;
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
  fclose(f);
  return v;
}

int main(int argc, char** argv) {
  if (argc != 6) return 2;
  const std::vector<uint8_t> tab = slurp(argv[1]), blob = slurp(argv[2]);
  const long long raw_bytes = atoll(argv[3]);
  const size_t n = tab.size() / sizeof(tmh_zchunk);
  std::vector<uint8_t> out((size_t)raw_bytes + 1, 0);
  std::vector<int32_t> st(n, 0);
  static tmh::ZShared<> z;
  for (int i = 0; i < 30; ++i) {  // the kernel's per-workgroup copy of the code tables
    if (i < 29) z.ltab[i] = tmh::kLenCode[i];
    z.dtab[i] = tmh::kDistCode[i];
  }
  std::vector<tmh_zchunk> cs(n);
  int64_t raw_max = 0;
  for (size_t i = 0; i < n; ++i) {
    memcpy(&cs[i], tab.data() + i * sizeof(tmh_zchunk), sizeof(tmh_zchunk));
    if (cs[i].raw_len > raw_max) raw_max = cs[i].raw_len;
  }
  const int64_t mw = tmh::match_words(raw_max);
  std::vector<uint32_t> ml((size_t)(mw * (int64_t)n + 2), 0);
  for (size_t i = 0; i < n; ++i)  // phase 1, lane by lane
    st[i] = tmh::inflate_tokens(blob.data(), (int64_t)blob.size(), cs[i], out.data(), raw_bytes,
                                ml.data() + i * mw, tmh::match_cap(mw), z, (int)(i % tmh::kZW));
  for (size_t i = 0; i < n; ++i)  // phase 2
    if (st[i] == 0 && cs[i].raw_off >= 0 && cs[i].raw_off + cs[i].raw_len <= raw_bytes)
      st[i] = tmh::resolve_matches(out.data() + cs[i].raw_off, cs[i].raw_len, ml.data() + i * mw);
  FILE* fo = fopen(argv[4], "wb");
  fwrite(out.data(), 1, (size_t)raw_bytes, fo);
  fclose(fo);
  FILE* fs = fopen(argv[5], "wb");
  fwrite(st.data(), 4, n, fs);
  fclose(fs);
  return 0;
}
