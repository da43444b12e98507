// Deflate decode of one zlib stream per GPU lane: the core of k_inflate
// (inflate_kernels.hip), kept free of HIP headers so the same code also
// builds for the host (tests/inflate_host.cpp: the decoder checked
// byte-for-byte against zlib on CPU).  See inflate_kernels.hip.
#pragma once

#include <cstdint>

#include "../../include/tmhip.h"

#ifndef TMH_ZDEV
#define TMH_ZDEV __device__ __forceinline__
#define TMH_ZHD __host__ __device__ __forceinline__
#define TMH_ZCONST __constant__
#define TMH_ZBITREV32(x) __builtin_bitreverse32(x)
#endif
#ifndef TMH_ZPROF
#define TMH_ZPROF 0  // 1: per-chunk decode counters in the match list's head (tools/inflate_prof.py)
#endif
#ifndef TMH_ZCLOCK
#define TMH_ZCLOCK() __builtin_readcyclecounter()
#endif
#ifndef TMH_ZST8
#define TMH_ZST8(p, a, b)                                            \
  do {                                                               \
    typedef uint32_t Z8_ __attribute__((ext_vector_type(2)));       \
    *reinterpret_cast<Z8_*>(p) = Z8_{(uint32_t)(a), (uint32_t)(b)};  \
  } while (0)
#endif
#ifndef TMH_ZKEEP
// an empty asm that "uses and redefines" v: the compiler cannot sink the
// computation of v into a branch
#define TMH_ZKEEP(v) __asm__ volatile("" : "+v"(v))
#endif
#ifndef TMH_ZBFE
// the low n bits of x (0 <= n <= 31): one v_bfe_u32
#define TMH_ZBFE(x, n) __builtin_amdgcn_ubfe((x), 0u, (unsigned)(n))
#endif
#ifndef TMH_ZLD16
// one 16-byte load from a 16-byte aligned p into four dwords
#define TMH_ZLD16(p, a, b, c, d)                                        \
  do {                                                                  \
    typedef uint32_t W4_ __attribute__((ext_vector_type(4)));          \
    const W4_ v_ = *reinterpret_cast<const W4_*>(p);                    \
    (a) = v_.x;                                                         \
    (b) = v_.y;                                                         \
    (c) = v_.z;                                                         \
    (d) = v_.w;                                                         \
  } while (0)
#endif
#ifndef TMH_ZLDS16
// one 16-byte LDS store to a 16-byte aligned p
#define TMH_ZLDS16(p, a, b, c, d)                                       \
  do {                                                                  \
    typedef uint32_t W4s_ __attribute__((ext_vector_type(4)));         \
    *reinterpret_cast<W4s_*>(p) = W4s_{(a), (b), (c), (d)};            \
  } while (0)
#define TMH_ZANY(pred) (__builtin_amdgcn_ballot_w64(pred) != 0)
#endif
#ifndef TMH_ZGLOBAL
// the output pointers in the global address space: a generic (flat) store
// also counts against the LDS wait counter, so every table lookup after it
// would wait for the store to reach memory
#define TMH_ZGLOBAL __attribute__((address_space(1)))
#endif

namespace tmh {

namespace {

constexpr int kZW = 64;  // lanes of a wave; a workgroup runs W <= kZW streams (one per lane)

// LDS layout: u16 arrays [n][W], W = the streams of a workgroup
constexpr int kLsym = 288, kDsym = 32, kLens = 320;
// first-level tables: the codes of at most kLFast (literal/length) or kDFast
// (distance) bits decode with one lookup of the peeked bits (entry = symbol
// | length << 12, 0 = a longer code: the canonical search below)
constexpr int kLFast = 9, kDFast = 6;
// Per lane, the next bytes of its stream in LDS (a ring of kRing dwords; rows
// padded to kRingStride, 16-byte aligned, so lanes at different positions
// fall in different banks)
constexpr int kRing = 32, kRingStride = 36, kRingLow = 4;
template <int W = kZW>
struct ZShared {
  static constexpr int kW = W;
  alignas(16) uint32_t ring[W][kRingStride];
  uint32_t ltab[29], dtab[30];  // kLenCode / kDistCode, shared by the workgroup
  uint16_t lfast[1 << kLFast][W];
  uint16_t dfast[1 << kDFast][W];
  uint16_t llim[16][W];   // left-justified limit of code length l (index 1..15)
  uint16_t lbase[16][W];  // symbol index base of code length l (mod 2^16)
  uint16_t lsym[kLsym][W];
  uint16_t dlim[16][W];
  uint16_t dbase[16][W];
  uint16_t dsym[kDsym][W];
  uint16_t tmp[16][W];    // table build: counts, then offsets
  uint8_t lens[kLens][W]; // code lengths of a dynamic block
};

// status codes (tmhip.h TMH_Z_*)
constexpr int kZOk = 0, kZHeader = 1, kZBlockType = 2, kZCode = 3, kZDist = 4, kZOverflow = 5,
              kZInput = 6, kZAdler = 7, kZSize = 8, kZStored = 9, kZTable = 10;

// The bit buffer, fed from the lane's ring in LDS.  The ring is topped up
// for all lanes of the wave at once (ring_top_up, at the top of every
// iteration of the decode loop, when any lane runs low): up to eight 16-byte
// loads per lane in flight together, one memory round trip for the whole
// wave every ~80 symbols.  A lane waiting alone on its own loads stalled the
// wave once per few symbols (a load in flight across iterations is waited
// for at the loop's back edge by the compiler's register copies, and a
// synchronous window load is a round trip per window per lane).  The ring
// running dry inside an iteration (long block headers) falls back to one
// synchronous 16-byte load (ring_load_unit).
struct Bits {
  uint64_t bb;     // bit buffer (LSB first)
  int nb;          // valid bits
  uint32_t head;   // dwords taken from the ring
  uint32_t fill;   // dwords put into the ring (a multiple of 4)
  int64_t p;       // byte offset in src of the ring's next 16 bytes (16-byte aligned)
  int64_t end;     // src bytes (loads at or past it read 0)
#if TMH_ZPROF
  uint32_t slow;  // codes decoded by the canonical search
  uint32_t priv;  // synchronous 16-byte units (ring ran dry)
  uint32_t tops;  // top-ups that loaded
#endif
};

// the aligned dword at byte p; bytes at or past `end` (the buffer's size) read 0
TMH_ZDEV uint32_t ld32(const uint8_t* src, int64_t p, int64_t end) {
  if (p + 4 <= end) return *reinterpret_cast<const uint32_t*>(src + p);
  uint32_t v = 0;
  for (int i = 0; i < 4; ++i)
    if (p + i < end) v |= (uint32_t)src[p + i] << (8 * i);
  return v;
}

// one 16-byte unit of the stream into the ring, synchronously
template <int W>
TMH_ZDEV void ring_load_unit(const uint8_t* src, Bits& b, ZShared<W>& z, int lane) {
  uint32_t a0, a1, a2, a3;
  if (b.p + 16 <= b.end) {
    TMH_ZLD16(src + b.p, a0, a1, a2, a3);
  } else {
    a0 = ld32(src, b.p, b.end);
    a1 = ld32(src, b.p + 4, b.end);
    a2 = ld32(src, b.p + 8, b.end);
    a3 = ld32(src, b.p + 12, b.end);
  }
  TMH_ZLDS16(&z.ring[lane][b.fill % kRing], a0, a1, a2, a3);
  b.fill += 4;
  b.p += 16;
#if TMH_ZPROF
  b.priv += 1;
#endif
}

// Called by every active lane of the wave at the same point: if any lane has
// fewer than kRingLow dwords left, every lane fills its ring's free 16-byte
// units that lie wholly inside the buffer (the loads first, then the LDS
// stores; the buffer's last partial unit, and zeros past it, come through
// ring_load_unit), so the data loop's refills never find the ring empty.
template <int W>
TMH_ZDEV void ring_top_up(const uint8_t* src, Bits& b, ZShared<W>& z, int lane) {
  if (!TMH_ZANY(b.fill - b.head < (uint32_t)kRingLow)) return;
  const int64_t in_buf = b.end - b.p >= 16 ? (b.end - b.p) >> 4 : 0;  // whole units left
  const int room = (int)((kRing - (b.fill - b.head)) >> 2);
  const int k = room < in_buf ? room : (int)in_buf;
  if (k > 0) {
    // eight loads in one block (units past k re-read unit k - 1: no branches,
    // no partly-defined registers), then the k stores
    uint32_t v[8][4];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      TMH_ZLD16(src + b.p + 16 * (u < k ? u : k - 1), v[u][0], v[u][1], v[u][2], v[u][3]);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (u < k)
        TMH_ZLDS16(&z.ring[lane][(b.fill + 4 * u) % kRing], v[u][0], v[u][1], v[u][2], v[u][3]);
    b.fill += 4 * k;
#if TMH_ZPROF
    b.tops += 1;
#endif
    b.p += 16 * k;
  }
  // at the buffer's end: the last partial unit, then zeros, one unit at a time
  while (b.fill - b.head < (uint32_t)kRingLow) ring_load_unit<W>(src, b, z, lane);
}

template <int W>
TMH_ZDEV uint32_t next_dword(const uint8_t* src, Bits& b, ZShared<W>& z, int lane) {
  if (b.head == b.fill) ring_load_unit<W>(src, b, z, lane);
  const uint32_t v = z.ring[lane][b.head % kRing];
  b.head += 1;
  return v;
}

template <int W>
TMH_ZDEV void refill(Bits& b, const uint8_t* src, ZShared<W>& z, int lane) {
  if (b.nb <= 32) {
    b.bb |= (uint64_t)next_dword<W>(src, b, z, lane) << b.nb;
    b.nb += 32;
  }
}

// refill for the data loop, where the ring is known to hold the dwords
// (ring_top_up leaves at least kRingLow, an iteration takes at most two):
// no branch, the ring's next dword read whether it is needed or not
template <int W>
TMH_ZDEV void refill_ring(Bits& b, ZShared<W>& z, int lane) {
  uint32_t v = z.ring[lane][b.head % kRing];
  TMH_ZKEEP(v);  // the read stays unconditional: no exec-mask branch (-2.5%, r4zbf)
  const bool need = b.nb <= 32;
  b.bb |= need ? (uint64_t)v << b.nb : 0ull;
  b.nb += need ? 32 : 0;
  b.head += need ? 1u : 0u;
}

// stream bits consumed: loaded from src_off on, less what the ring and the buffer hold
TMH_ZDEV int64_t consumed_bits(const Bits& b, int64_t src_off) {
  return (b.p - src_off) * 8 - (int64_t)(b.fill - b.head) * 32 - b.nb;
}

template <int W>
TMH_ZDEV uint32_t take(Bits& b, int n) {  // n <= 16 and <= the bits in the buffer
  const uint32_t v = TMH_ZBFE((uint32_t)b.bb, n);
  b.bb >>= n;
  b.nb -= n;
  return v;
}

template <int W>
TMH_ZDEV uint32_t getb(Bits& b, const uint8_t* src, ZShared<W>& z, int lane, int n) {
  refill<W>(b, src, z, lane);
  const uint32_t v = TMH_ZBFE((uint32_t)b.bb, n);  // n <= 16
  b.bb >>= n;
  b.nb -= n;
  return v;
}

// Canonical Huffman decode.  A code of at most FB bits is one lookup of the
// next FB stream bits in `fast`; a longer one: v = the next 15 bits in code
// order (bit-reversed peek), the code length is the smallest l with v <
// lim[l] (lim non-decreasing), found by binary search.  Returns -1 for a code
// the table does not hold.
template <int FB, int W, bool RingSafe = false>
TMH_ZDEV int hdecode(Bits& b, const uint8_t* src, ZShared<W>& z, uint16_t (*fast)[W],
                     uint16_t (*lim)[W], uint16_t (*base)[W], uint16_t (*sym)[W], int nsym,
                     int lane) {
  if (RingSafe) refill_ring<W>(b, z, lane);
  else refill<W>(b, src, z, lane);
  const uint32_t e = fast[(uint32_t)b.bb & ((1u << FB) - 1u)][lane];
  if (e >> 12) {
    const int len = (int)(e >> 12);
    b.bb >>= len;
    b.nb -= len;
    return (int)(e & 0x1FFu);
  }
#if TMH_ZPROF
  b.slow += 1;
#endif
  const uint32_t v = TMH_ZBITREV32((uint32_t)b.bb) >> 17;
  int l = 0;  // largest l with lim[l] <= v (lim[0] = 0)
#pragma unroll
  for (int step = 8; step >= 1; step >>= 1)
    if (l + step <= 15 && v >= (uint32_t)lim[l + step][lane]) l += step;
  const int len = l + 1;
  if (len > 15) return -1;
  const uint32_t code = v >> (15 - len);
  b.bb >>= len;
  b.nb -= len;
  // in range for every code hbuild accepted; clamped so no input can index past the table
  const uint32_t i = (uint16_t)(base[len][lane] + code);
  return sym[i < (uint32_t)nsym ? i : (uint32_t)nsym - 1u][lane];
}

// Canonical tables from n code lengths (lens column of this lane, or the
// fixed code), with the first-level table of the codes of at most FB bits;
// returns false for an over-subscribed code.
template <int FB, int W>
TMH_ZDEV bool hbuild(ZShared<W>& z, int lane, const uint8_t (*lens)[W], int off, int n,
                     uint16_t (*fast)[W], uint16_t (*lim)[W], uint16_t (*base)[W],
                     uint16_t (*sym)[W]) {
  for (int i = 0; i < (1 << FB); ++i) fast[i][lane] = 0;
  for (int l = 0; l < 16; ++l) z.tmp[l][lane] = 0;
  for (int s = 0; s < n; ++s) {
    const int l = lens[off + s][lane];
    if (l) z.tmp[l][lane] += 1;
  }
  uint32_t code = 0, offs = 0;
  for (int l = 1; l < 16; ++l) {
    const uint32_t cnt = z.tmp[l][lane];
    base[l][lane] = (uint16_t)(offs - code);
    code += cnt;
    if (code > (1u << l)) return false;
    lim[l][lane] = (uint16_t)(code << (15 - l));
    z.tmp[l][lane] = (uint16_t)offs;
    offs += cnt;
    code <<= 1;
  }
  for (int s = 0; s < n; ++s) {
    const int l = lens[off + s][lane];
    if (l) {
      const int i = z.tmp[l][lane];
      sym[i][lane] = (uint16_t)s;
      z.tmp[l][lane] = (uint16_t)(i + 1);
      if (l <= FB) {  // its canonical code, stream bit order: every FB-bit peek starting with it
        const uint32_t code = (uint16_t)(i - base[l][lane]);
        const uint32_t rev = TMH_ZBITREV32(code) >> (32 - l);
        const uint16_t ent = (uint16_t)(s | (l << 12));
        for (uint32_t k = rev; k < (1u << FB); k += 1u << l) fast[k][lane] = ent;
      }
    }
  }
  return true;
}

// RFC 1951 3.2.5: length / distance symbol -> base | extra bits << 16 (copied
// into each workgroup's LDS: one lookup beat the arithmetic, 39.0 vs 40.4 ms
// per 128 sites, profiles/r4/ab_inflate_ml8_ltab_r4zv.txt)
TMH_ZCONST uint32_t kLenCode[29] = {
    3,  4,  5,  6,  7,  8,  9,  10, 11 | 1 << 16, 13 | 1 << 16, 15 | 1 << 16, 17 | 1 << 16,
    19 | 2 << 16, 23 | 2 << 16, 27 | 2 << 16, 31 | 2 << 16, 35 | 3 << 16, 43 | 3 << 16,
    51 | 3 << 16, 59 | 3 << 16, 67 | 4 << 16, 83 | 4 << 16, 99 | 4 << 16, 115 | 4 << 16,
    131 | 5 << 16, 163 | 5 << 16, 195 | 5 << 16, 227 | 5 << 16, 258};
TMH_ZCONST uint32_t kDistCode[30] = {
    1, 2, 3, 4, 5 | 1 << 16, 7 | 1 << 16, 9 | 2 << 16, 13 | 2 << 16, 17 | 3 << 16, 25 | 3 << 16,
    33 | 4 << 16, 49 | 4 << 16, 65 | 5 << 16, 97 | 5 << 16, 129 | 6 << 16, 193 | 6 << 16,
    257 | 7 << 16, 385 | 7 << 16, 513 | 8 << 16, 769 | 8 << 16, 1025 | 9 << 16, 1537 | 9 << 16,
    2049 | 10 << 16, 3073 | 10 << 16, 4097 | 11 << 16, 6145 | 11 << 16, 8193 | 12 << 16,
    12289 | 12 << 16, 16385 | 13 << 16, 24577 | 13 << 16};
TMH_ZCONST uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum : int { kStBlock = 0, kStData = 1, kStStored = 2, kStTrailer = 3, kStDone = 4 };


// Per chunk, the match list the decode leaves for the resolver (scratch,
// 32-bit words, 16-byte aligned): [0] matches, [1] the stream's Adler-32
// (big-endian value), [2..15] unused (TMH_ZPROF counters), then from word
// kMlHead per match (output
// position, length | distance << 9), one 8-byte store per match.
// A match needs at least 3 output bytes, so raw_len / 3 + 2 entries always fit.
constexpr int kMlHead = 16;
TMH_ZHD int64_t match_words(int64_t raw_max) {
  return (kMlHead + 2 * (raw_max / 3 + 2) + 3) & ~int64_t(3);
}
TMH_ZHD int64_t match_cap(int64_t mw) { return (mw - kMlHead) / 2; }


// Phase 1 of a chunk (one zlib stream): Huffman-decode every symbol, write
// the literal (and stored) bytes at their output positions, and append each
// back-reference to the chunk's match list `ml` (match_words above) instead
// of copying it -- so no step of the lane's serial decode waits on a load of
// earlier output.  Returns the TMH_Z_* status (Adler-32 is checked once the
// matches are resolved: resolve_matches / k_resolve_matches).
template <int W>
TMH_ZDEV int inflate_tokens(const uint8_t* __restrict__ src, int64_t src_bytes,
                            const tmh_zchunk& c, uint8_t* __restrict__ dst, int64_t dst_bytes,
                            uint32_t* __restrict__ ml, int ml_cap,
                            ZShared<W>& z, int lane) {
  int err = kZOk;
  if (c.src_off < 0 || c.src_len < 0 || c.src_off + c.src_len > src_bytes || c.raw_off < 0 ||
      c.raw_len < 0 || c.raw_off + c.raw_len > dst_bytes) {
    return kZInput;
  }
  TMH_ZGLOBAL uint8_t* out = (TMH_ZGLOBAL uint8_t*)(dst + c.raw_off);
  const int olen = (int)c.raw_len;  // < 2^31 (tmh_inflate_device checks raw_max)
  ml[0] = 0u;
  if (c.flags & 1) {  // the HDF5 filter was skipped: raw bytes, nothing to check
    if (c.src_len != c.raw_len) return kZSize;
    for (int i = 0; i < olen; ++i) out[i] = src[c.src_off + i];
    ml[1] = 0xFFFFFFFFu;  // no Adler-32 to check
    return kZOk;
  }
  Bits b;
  {
    b.end = src_bytes;  // loads past the stream's own bytes read the next stream's
    b.p = c.src_off & ~15ll;  // (harmless: the consumed-bit count is checked), never past the buffer
    b.head = 0;
    b.fill = 0;
    ring_load_unit<W>(src, b, z, lane);
    b.head = (uint32_t)((c.src_off >> 2) & 3);
    const int sh = (int)(c.src_off & 3) * 8;
    b.bb = (uint64_t)next_dword<W>(src, b, z, lane) >> sh;
    b.nb = 32 - sh;
  }
  const int64_t in_bits = (int64_t)c.src_len * 8;
  // loads running this far past the stream mean a corrupt stream (checked per
  // symbol on the ring's load position; exactly at the trailer)
  const int64_t p_limit = c.src_off + c.src_len + 256;
  // zlib header (RFC 1950): CM = 8, CINFO <= 7, FCHECK, no preset dictionary
  const uint32_t cmf = getb<W>(b, src, z, lane, 8), flg = getb<W>(b, src, z, lane, 8);
  if ((cmf & 15u) != 8u || (cmf >> 4) > 7u || ((cmf << 8) | flg) % 31u != 0u || (flg & 0x20u))
    err = kZHeader;
  int o = 0;   // output bytes (literals written, matches listed)
  int nm = 0;  // matches listed
  int state = err ? kStDone : kStBlock;
  int last = 0;
  int stored_left = 0;
#if TMH_ZPROF
  b.slow = 0;
  b.priv = 0;
  b.tops = 0;
  uint64_t pc_sym = 0, pc_runs = 0, pc_data = 0, pc_hdr = 0, pc_hcyc = 0;
  const uint64_t tstart = TMH_ZCLOCK();
#endif
  while (state != kStDone) {
#if TMH_ZPROF
    const uint64_t t0 = TMH_ZCLOCK();
    const int st0 = state;
#endif
    if (consumed_bits(b, c.src_off) > in_bits + 64) {  // ran far past the stream: corrupt
      err = kZInput;
      break;
    }
    if (state == kStData) {
      // The data path as a loop of its own: every active lane decodes
      // symbols until any lane leaves its block (end-of-block or an error),
      // with the stream ring topped up for the wave and branch-free refills
#if TMH_ZPROF
      const uint64_t td = TMH_ZCLOCK();
      pc_runs += 1;
#endif
      do {
        ring_top_up<W>(src, b, z, lane);
        int ecode = 0;
        const int s = hdecode<kLFast, W, true>(b, src, z, z.lfast, z.llim, z.lbase, z.lsym, kLsym,
                                               lane);
        if (s < 256) {
          if (s < 0) ecode = kZCode;
          else if (o >= olen) ecode = kZOverflow;
          else out[o++] = (uint8_t)s;
        } else if (s == 256) {
          state = last ? kStTrailer : kStBlock;
        } else {
          const int li = s - 257 < 29 ? s - 257 : 28;
          // <= 15 + 5 bits since the refill: no refill before the length's extra bits
          const uint32_t le = z.ltab[li];  // base | extra bits << 16
          const int len = (int)(le & 0xFFFFu) + (int)take<W>(b, (int)(le >> 16));
          const int ds = hdecode<kDFast, W, true>(b, src, z, z.dfast, z.dlim, z.dbase, z.dsym,
                                                  kDsym, lane);
          const int dsc = ds >= 0 && ds < 30 ? ds : 0;
          const uint32_t de = z.dtab[dsc];
          const int dist = (int)(de & 0xFFFFu) + (int)take<W>(b, (int)(de >> 16));
          ecode = (s - 257 >= 29 || ds < 0 || ds >= 30) ? kZCode
                  : dist > o                              ? kZDist
                  : (o + len > olen || nm >= ml_cap)      ? kZOverflow
                                                          : kZOk;
          if (ecode == kZOk) {
            const uint32_t e = (uint32_t)len | ((uint32_t)dist << 9);
            TMH_ZST8(ml + kMlHead + 2 * nm, o, e);  // one 8-byte store per match
            ++nm;
            o += len;
          }
        }
        if (b.p > p_limit) ecode = kZInput;  // ran far past the stream: corrupt
        if (ecode) {
          err = ecode;
          state = kStDone;
        }
#if TMH_ZPROF
        pc_sym += 1;
#endif
      } while (!TMH_ZANY(state != kStData));
#if TMH_ZPROF
      pc_data += TMH_ZCLOCK() - td;
#endif
      if (err) break;
    } else if (state == kStBlock) {
      last = (int)getb<W>(b, src, z, lane, 1);
      const uint32_t type = getb<W>(b, src, z, lane, 2);
      if (type == 0) {  // stored: byte-align, LEN, NLEN
        const int drop = b.nb & 7;
        b.bb >>= drop;
        b.nb -= drop;
  
        const uint32_t len = getb<W>(b, src, z, lane, 16), nlen = getb<W>(b, src, z, lane, 16);
        if ((len ^ nlen) != 0xFFFFu) {
          err = kZStored;
          break;
        }
        stored_left = len;
        state = kStStored;
      } else if (type == 1) {  // fixed Huffman code
        for (int s = 0; s < 288; ++s)
          z.lens[s][lane] = (uint8_t)(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8);
        for (int s = 0; s < 32; ++s) z.lens[288 + s][lane] = 5;
        if (!hbuild<kLFast, W>(z, lane, z.lens, 0, 288, z.lfast, z.llim, z.lbase, z.lsym) ||
            !hbuild<kDFast, W>(z, lane, z.lens, 288, 32, z.dfast, z.dlim, z.dbase, z.dsym)) {
          err = kZTable;
          break;
        }
        state = kStData;
      } else if (type == 2) {  // dynamic: code-length code, then the two codes' lengths
        const int hlit = (int)getb<W>(b, src, z, lane, 5) + 257, hdist = (int)getb<W>(b, src, z, lane, 5) + 1;
        const int hclen = (int)getb<W>(b, src, z, lane, 4) + 4;
        if (hlit > 286 || hdist > 30) {
          err = kZTable;
          break;
        }
        for (int i = 0; i < 19; ++i) z.lens[i][lane] = 0;
        for (int i = 0; i < hclen; ++i) z.lens[kClOrder[i]][lane] = (uint8_t)getb<W>(b, src, z, lane, 3);
        // the code-length code lives in the distance tables until the real ones are built
        if (!hbuild<kDFast, W>(z, lane, z.lens, 0, 19, z.dfast, z.dlim, z.dbase, z.dsym)) {
          err = kZTable;
          break;
        }
        int n = 0;
        const int total = hlit + hdist;
        while (n < total) {
          const int s = hdecode<kDFast, W>(b, src, z, z.dfast, z.dlim, z.dbase, z.dsym, kDsym, lane);
          if (s < 0) {
            err = kZCode;
            break;
          }
          int rep = 0, val = 0;
          if (s < 16) {
            z.lens[n++][lane] = (uint8_t)s;
            continue;
          } else if (s == 16) {
            if (n == 0) {
              err = kZTable;
              break;
            }
            val = z.lens[n - 1][lane];
            rep = 3 + (int)getb<W>(b, src, z, lane, 2);
          } else if (s == 17) {
            rep = 3 + (int)getb<W>(b, src, z, lane, 3);
          } else {
            rep = 11 + (int)getb<W>(b, src, z, lane, 7);
          }
          if (n + rep > total) {
            err = kZTable;
            break;
          }
          for (int i = 0; i < rep; ++i) z.lens[n++][lane] = (uint8_t)val;
        }
        if (err) break;
        if (z.lens[256][lane] == 0 ||  // no end-of-block code
            !hbuild<kLFast, W>(z, lane, z.lens, 0, hlit, z.lfast, z.llim, z.lbase, z.lsym) ||
            !hbuild<kDFast, W>(z, lane, z.lens, hlit, hdist, z.dfast, z.dlim, z.dbase, z.dsym)) {
          err = kZTable;
          break;
        }
        state = kStData;
      } else {
        err = kZBlockType;
        break;
      }
    } else if (state == kStStored) {
      if (stored_left == 0) {
        state = last ? kStTrailer : kStBlock;
        continue;
      }
      if (o >= olen) {
        err = kZOverflow;
        break;
      }
      out[o++] = (uint8_t)getb<W>(b, src, z, lane, 8);
      --stored_left;
    } else {  // trailer: byte-align, Adler-32 big-endian
      const int drop = b.nb & 7;
      b.bb >>= drop;
      b.nb -= drop;

      uint32_t want = 0;
      for (int i = 0; i < 4; ++i) want = (want << 8) | getb<W>(b, src, z, lane, 8);
      ml[1] = want;
      if (o != olen) err = kZSize;
      else if (consumed_bits(b, c.src_off) > in_bits) err = kZInput;
      state = kStDone;
    }
#if TMH_ZPROF
    if (st0 == kStBlock) {
      pc_hdr += 1;
      pc_hcyc += TMH_ZCLOCK() - t0;
    }
#endif
  }
#if TMH_ZPROF
  ml[2] = (uint32_t)pc_sym;                            // symbols decoded in the data loop
  ml[3] = (uint32_t)((TMH_ZCLOCK() - tstart) >> 8);   // cycles of the whole stream
  ml[4] = b.slow;
  ml[5] = (uint32_t)(pc_data >> 8);  // cycles in the data loop
  ml[6] = (uint32_t)(pc_hcyc >> 8);  // cycles in block headers
  ml[7] = (uint32_t)pc_runs;         // entries into the data loop
  ml[8] = b.priv;
  ml[9] = b.tops;
  ml[10] = (uint32_t)pc_hdr;
#endif
  ml[0] = (uint32_t)nm;
  return err;
}

// Adler-32 of n bytes from partial sums: a = 1 + sum x_i, b = n + sum (n - i) x_i.
TMH_ZHD uint32_t adler_from_sums(uint64_t sa, uint64_t sb, int64_t n) {
  const uint64_t a = (1u + sa % 65521u) % 65521u;
  const uint64_t b = ((uint64_t)(n % 65521) + sb % 65521u) % 65521u;
  return (uint32_t)((b << 16) | a);
}

// Phase 2 on the host (tests/inflate_host.cpp): the matches in order, then
// the Adler-32 check.  The device resolves the same list with a wave per
// chunk (k_resolve_matches).
inline int resolve_matches(uint8_t* out, int64_t olen, const uint32_t* ml) {
  const int64_t nm = ml[0];
  for (int64_t m = 0; m < nm; ++m) {
    const int64_t o = ml[kMlHead + 2 * m];
    const uint32_t e = ml[kMlHead + 2 * m + 1];
    const int len = (int)(e & 511u), dist = (int)(e >> 9);
    for (int i = 0; i < len; ++i) out[o + i] = out[o - dist + i];
  }
  if (ml[1] == 0xFFFFFFFFu) return kZOk;  // stored chunk
  uint64_t sa = 0, sb = 0;
  for (int64_t i = 0; i < olen; ++i) {
    sa += out[i];
    sb += (uint64_t)(olen - i) * out[i];
    if ((i & 0xFFFFF) == 0xFFFFF) {
      sa %= 65521u;
      sb %= 65521u;
    }
  }
  return adler_from_sums(sa, sb, olen) == ml[1] ? kZOk : kZAdler;
}


}  // namespace

}  // namespace tmh
