// GPU inflate of HDF5 gzip chunks (gfx950 / MI355X) -- the site-image input
// path of the corilla job.
//
// Reference: tmlib/models/file.py:322-351 (ChannelImageFile.get) and
// tmlib/readers.py:367-389 (DatasetReader.read): h5py reads the gzip-filtered
// /array dataset, i.e. libhdf5's deflate filter runs zlib's inflate on every
// chunk (files written by tmlib/models/file.py:353-363 / writers.py:384-387).
// Each HDF5 chunk is an independent zlib stream (RFC 1950 header, RFC 1951
// deflate blocks, Adler-32 trailer), so a batch of sites is thousands of
// independent streams: here one LANE decodes one stream, 64 streams per
// wave, in two kernels.  Phase 1 (k_inflate_tokens) is the serial Huffman
// decode: literal bytes go straight to their output positions and every
// back-reference is only listed -- a lane copying its matches itself waited
// one memory round trip per match, and with 64 lanes per wave some lane had
// a match in nearly every step (3.6 GB/s for 128 sites,
// profiles/r4/bench_inflate_*_r4g.json).  Phase 2 (k_resolve_matches) is
// one wave per chunk copying its matches in order, 64 at a time.
// Host cores then only move compressed bytes (raw chunks read straight from
// the files, libtmh5) and the PCIe link carries compressed data.
//
// Per lane (LDS, interleaved [index][lane] so the 64 lanes' table reads fall
// in different banks): the literal/length and distance codes as canonical
// Huffman tables -- left-justified limit per code length, symbol base per
// length, symbols in code order -- decoded by a 4-step binary search over the
// 15 code lengths on the bit-reversed 15-bit peek; the dynamic block header's
// code lengths; a count/offset scratch for the table build.  The lane's loop
// is a flat state machine (one deflate symbol, or one whole block header, per
// iteration) so lanes at different points of their streams stay converged
// on the symbol path; the bit buffer's next dword is loaded one refill
// ahead.  Output bytes go to the chunk's region of a raw buffer.  Adler-32
// is checked like zlib's inflate, in phase 2.
// tmh_place_chunks_device then moves each chunk's rows into [image][H][W]
// (edge chunks carry padding past the dataset extent).
#include <cstring>

#include "common.h"
#include "inflate_core.h"

namespace tmh {

// Phase 1: one lane per chunk (inflate_core.h inflate_tokens), W chunks per
// workgroup (a wave with W active lanes).
template <int W>
__global__ __launch_bounds__(W) void k_inflate_tokens(
    const uint8_t* __restrict__ src, int64_t src_bytes, const tmh_zchunk* __restrict__ chunks,
    int64_t n_chunks, uint8_t* __restrict__ dst, int64_t dst_bytes, uint32_t* __restrict__ ml_all,
    int64_t mw, int32_t* __restrict__ status) {
  __shared__ ZShared<W> z;
  const int lane = threadIdx.x;
  for (int i = lane; i < 30; i += W) {
    if (i < 29) z.ltab[i] = kLenCode[i];
    z.dtab[i] = kDistCode[i];
  }
  __syncthreads();
  const int64_t ci = (int64_t)blockIdx.x * W + lane;
  if (ci >= n_chunks) return;
  status[ci] = inflate_tokens<W>(src, src_bytes, chunks[ci], dst, dst_bytes, ml_all + ci * mw,
                                 match_cap(mw), z, lane);
}

__device__ __forceinline__ uint32_t wave_excl_min(uint32_t v, int lane) {
  uint32_t incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, off, 64);
    if (lane >= off) incl = y < incl ? y : incl;
  }
  const uint32_t ex = (uint32_t)__shfl_up((int)incl, 1, 64);
  return lane == 0 ? 0xFFFFFFFFu : ex;
}

// Phase 2: one wave per chunk resolves its match list in order, 64 matches
// at a time.  A match's source lies before its own position; in a round,
// every pending match whose source ends before the first still-pending
// destination of the earlier lanes copies (a copy that overlaps itself,
// distance < length, runs byte by byte in its lane, in order), so each round
// makes progress and a batch usually needs one or two rounds -- one memory
// round trip per 64 matches instead of one per match.  Then the chunk's
// Adler-32 from its bytes (a = 1 + sum x_i, b = n + sum (n - i) x_i, a wave
// reduction) against the stream's trailer.
__global__ __launch_bounds__(kZW) void k_resolve_matches(const tmh_zchunk* __restrict__ chunks,
                                                         uint8_t* __restrict__ dst,
                                                         const uint32_t* __restrict__ ml_all,
                                                         int64_t mw, int32_t* __restrict__ status) {
  const int64_t ci = blockIdx.x;
  const int lane = threadIdx.x;
  if (status[ci] != 0) return;  // phase 1 failed: nothing to resolve (uniform)
  const tmh_zchunk c = chunks[ci];
  uint8_t* out = dst + c.raw_off;
  const int64_t olen = c.raw_len;
  const uint32_t* ml = ml_all + ci * mw;
  const int64_t nm = ml[0];
  const uint32_t want = ml[1];
  for (int64_t base = 0; base < nm; base += kZW) {
    const int64_t i = base + lane;
    const bool act = i < nm;
    const uint2 oe = act ? reinterpret_cast<const uint2*>(ml + kMlHead)[i] : make_uint2(0u, 0u);
    const uint32_t o = oe.x, e = oe.y;
    const uint32_t len = e & 511u, d = e >> 9;
    const uint32_t src_end = o - d + (len < d ? len : d);  // source bytes before its own output
    bool todo = act;
    while (__builtin_amdgcn_ballot_w64(todo)) {
      const uint32_t fu = wave_excl_min(todo ? o : 0xFFFFFFFFu, lane);
      const bool go = todo && src_end <= fu;
      if (go) {
        uint8_t* to = out + o;
        const uint8_t* from = out + o - d;
        if (d >= len) {  // the loads of up to 8 bytes together, then the stores
          for (uint32_t k = 0; k < len; k += 8) {
            uint8_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = k + j < len ? from[k + j] : 0;
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (k + j < len) to[k + j] = v[j];
          }
        } else {
          for (uint32_t k = 0; k < len; ++k) to[k] = from[k];
        }
      }
      // this round's stores before the next round's loads (other lanes)
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      todo = todo && !go;
    }
  }
  if (want == 0xFFFFFFFFu) return;  // a stored chunk (filter skipped): no checksum
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  uint64_t sa = 0, sb = 0;
  int64_t k = 0;
  for (int64_t j = lane; j < olen; j += kZW) {
    const uint32_t x = out[j];
    sa += x;
    sb += (uint64_t)(olen - j) * x;
    if (++k == 65536) {
      sa %= 65521u;
      sb %= 65521u;
      k = 0;
    }
  }
  sa %= 65521u;
  sb %= 65521u;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sa += (uint64_t)__shfl_xor((long long)sa, off, 64);
    sb += (uint64_t)__shfl_xor((long long)sb, off, 64);
  }
  if (lane == 0 && adler_from_sums(sa, sb, olen) != want) status[ci] = kZAdler;
}

// ---------------------------------------------------------------------------
// The whole-wave decode: one WAVE per zlib stream, all 64 lanes decoding.
//
// A lane-per-stream decode leaves each wave instruction serving a handful of
// streams (W = 8: the per-stream tables fill LDS at ~16k resident streams,
// and a wave's lanes diverge over literal / match / long-code paths), so
// phase 1 was issue-bound at ~270 instructions per symbol and wave
// (DESIGN.md §9.4).  Here a wave owns one stream and decodes it
// SPECULATIVELY: in each round lane k decodes a whole token (literal, match
// with its extra bits and distance, or end-of-block) as if one started at
// bit bp + k; a scalar walk from lane 0 along the tokens' lengths then marks
// the lanes that are real token starts (~8 per round on microscopy data) and
// the marked tokens are emitted at once -- literal bytes at their prefix-sum
// offsets, matches appended to the chunk's match list.  Block headers
// (dynamic code lengths, table builds), stored-block headers and the trailer
// run on lane 0 with the lane-per-stream code of inflate_core.h (one table
// set per wave), stored bytes are copied by the whole wave.  The same wave
// then resolves its matches (k_resolve_matches' rounds) and checks the
// Adler-32: one kernel instead of two.
// ---------------------------------------------------------------------------

constexpr int kWRing = 128;  // dwords of the stream staged in LDS per wave (a ring)

template <int NW>
struct ZWaves {
  ZShared<1> z[NW];                   // lane 0's tables, bit buffer ring, scratch
  uint32_t ring[NW][kWRing];          // the stream's next dwords for the whole wave
};

// Resolve one chunk's match list in order, 64 matches at a time, then check
// its Adler-32 (see k_resolve_matches); every lane of the wave calls it.
__device__ __forceinline__ int32_t resolve_wave(uint8_t* __restrict__ out, int64_t olen,
                                                const uint32_t* __restrict__ ml, int lane) {
  const int64_t nm = ml[0];
  const uint32_t want = ml[1];
  for (int64_t base = 0; base < nm; base += kZW) {
    const int64_t i = base + lane;
    const bool act = i < nm;
    const uint2 oe = act ? reinterpret_cast<const uint2*>(ml + kMlHead)[i] : make_uint2(0u, 0u);
    const uint32_t o = oe.x, e = oe.y;
    const uint32_t len = e & 511u, d = e >> 9;
    const uint32_t src_end = o - d + (len < d ? len : d);
    bool todo = act;
    while (__builtin_amdgcn_ballot_w64(todo)) {
      const uint32_t fu = wave_excl_min(todo ? o : 0xFFFFFFFFu, lane);
      const bool go = todo && src_end <= fu;
      if (go) {
        uint8_t* to = out + o;
        const uint8_t* from = out + o - d;
        if (d >= len) {
          for (uint32_t k = 0; k < len; k += 8) {
            uint8_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = k + j < len ? from[k + j] : 0;
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (k + j < len) to[k + j] = v[j];
          }
        } else {
          for (uint32_t k = 0; k < len; ++k) to[k] = from[k];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      todo = todo && !go;
    }
  }
  if (want == 0xFFFFFFFFu) return kZOk;  // a stored chunk (filter skipped): no checksum
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  uint64_t sa = 0, sb = 0;
  int64_t k = 0;
  for (int64_t j = lane; j < olen; j += kZW) {
    const uint32_t x = out[j];
    sa += x;
    sb += (uint64_t)(olen - j) * x;
    if (++k == 65536) {
      sa %= 65521u;
      sb %= 65521u;
      k = 0;
    }
  }
  sa %= 65521u;
  sb %= 65521u;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sa += (uint64_t)__shfl_xor((long long)sa, off, 64);
    sb += (uint64_t)__shfl_xor((long long)sb, off, 64);
  }
  return adler_from_sums(sa, sb, olen) == want ? kZOk : kZAdler;
}

// lane 0's bit buffer starting at absolute bit `bit` of the stream (bits
// counted from byte `base`)
__device__ __forceinline__ void bits_at(Bits& b, const uint8_t* src, int64_t src_bytes,
                                        int64_t base, int64_t bit, ZShared<1>& z) {
  const int64_t byte = base + (bit >> 3);
  b.end = src_bytes;
  b.p = byte & ~15ll;
  b.head = 0;
  b.fill = 0;
  ring_load_unit<1>(src, b, z, 0);
  b.head = (uint32_t)((byte >> 2) & 3);
  const int sh = (int)(byte & 3) * 8 + (int)(bit & 7);
  b.bb = (uint64_t)next_dword<1>(src, b, z, 0) >> sh;
  b.nb = 32 - sh;
}

enum : uint32_t { kTokLit = 0, kTokMatch = 1, kTokEob = 2, kTokBad = 3 };

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_inflate_wave(
    const uint8_t* __restrict__ src, int64_t src_bytes, const tmh_zchunk* __restrict__ chunks,
    int64_t n_chunks, uint8_t* __restrict__ dst, int64_t dst_bytes, uint32_t* __restrict__ ml_all,
    int64_t mw, int32_t* __restrict__ status) {
  __shared__ ZWaves<NW> zw;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  ZShared<1>& z = zw.z[wv];
  uint32_t* wr = zw.ring[wv];
  if (lane < 30) {
    if (lane < 29) z.ltab[lane] = kLenCode[lane];
    z.dtab[lane] = kDistCode[lane];
  }
  const int64_t ci = (int64_t)blockIdx.x * NW + wv;
  if (ci >= n_chunks) return;  // (uniform per wave; no workgroup barrier below)
  const tmh_zchunk c = chunks[ci];
  uint32_t* ml = ml_all + ci * mw;
  const int ml_cap = match_cap(mw);
  if (c.src_off < 0 || c.src_len < 0 || c.src_off + c.src_len > src_bytes || c.raw_off < 0 ||
      c.raw_len < 0 || c.raw_off + c.raw_len > dst_bytes) {
    if (lane == 0) status[ci] = kZInput;
    return;
  }
  uint8_t* out = dst + c.raw_off;
  const int olen = (int)c.raw_len;
  if (c.flags & 1) {  // the HDF5 filter was skipped: raw bytes, nothing to check
    if (c.src_len != c.raw_len) {
      if (lane == 0) status[ci] = kZSize;
      return;
    }
    for (int i = lane; i < olen; i += 64) out[i] = src[c.src_off + i];
    if (lane == 0) status[ci] = kZOk;
    return;
  }
  const int64_t base = c.src_off & ~3ll;  // bit positions count from this byte
  const int64_t in_end = (c.src_off - base + c.src_len) * 8;  // the stream's end, in those bits
  // the wave ring: stream dwords [whi - kWRing, whi) sit at slot index % kWRing
  int64_t whi = 0;
  auto refill = [&]() {  // the next 64 dwords, one per lane (uniform call)
    const int64_t p = base + 4 * (whi + lane);
    wr[(whi + lane) % kWRing] = ld32(src, p, src_bytes);
    whi += 64;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  };
  int64_t bp = (c.src_off - base) * 8;  // next unconsumed bit
  int err = kZOk;
  int state = kStBlock;
  int last = 0;
  int o = 0, nm = 0;
  uint32_t want = 0;
  // zlib header (RFC 1950) on lane 0
  if (lane == 0) {
    Bits b;
    bits_at(b, src, src_bytes, base, bp, z);
    const uint32_t cmf = getb<1>(b, src, z, 0, 8), flg = getb<1>(b, src, z, 0, 8);
    if ((cmf & 15u) != 8u || (cmf >> 4) > 7u || ((cmf << 8) | flg) % 31u != 0u || (flg & 0x20u))
      err = kZHeader;
  }
  err = __builtin_amdgcn_readfirstlane(err);
  bp += 16;
  if (err) state = kStDone;
  while (state != kStDone) {
    if (state == kStBlock || state == kStTrailer) {
      // lane 0: block header / trailer with the lane-per-stream code
      int st2 = state, l2 = last, e2 = 0, stored = -1;
      int64_t bp2 = bp;
      if (lane == 0) {
        Bits b;
        bits_at(b, src, src_bytes, base, bp, z);
        if (state == kStTrailer) {
          const int drop = b.nb & 7;
          b.bb >>= drop;
          b.nb -= drop;
          uint32_t w = 0;
          for (int i = 0; i < 4; ++i) w = (w << 8) | getb<1>(b, src, z, 0, 8);
          want = w;
          st2 = kStDone;
        } else {
          l2 = (int)getb<1>(b, src, z, 0, 1);
          const uint32_t type = getb<1>(b, src, z, 0, 2);
          if (type == 0) {  // stored: byte-align, LEN, NLEN; the wave copies the bytes
            const int drop = b.nb & 7;
            b.bb >>= drop;
            b.nb -= drop;
            const uint32_t len = getb<1>(b, src, z, 0, 16), nlen = getb<1>(b, src, z, 0, 16);
            if ((len ^ nlen) != 0xFFFFu) e2 = kZStored;
            stored = (int)len;
            st2 = kStStored;
          } else if (type == 1) {  // fixed Huffman code
            for (int s2 = 0; s2 < 288; ++s2)
              z.lens[s2][0] = (uint8_t)(s2 < 144 ? 8 : s2 < 256 ? 9 : s2 < 280 ? 7 : 8);
            for (int s2 = 0; s2 < 32; ++s2) z.lens[288 + s2][0] = 5;
            if (!hbuild<kLFast, 1>(z, 0, z.lens, 0, 288, z.lfast, z.llim, z.lbase, z.lsym) ||
                !hbuild<kDFast, 1>(z, 0, z.lens, 288, 32, z.dfast, z.dlim, z.dbase, z.dsym))
              e2 = kZTable;
            st2 = kStData;
          } else if (type == 2) {  // dynamic
            const int hlit = (int)getb<1>(b, src, z, 0, 5) + 257;
            const int hdist = (int)getb<1>(b, src, z, 0, 5) + 1;
            const int hclen = (int)getb<1>(b, src, z, 0, 4) + 4;
            if (hlit > 286 || hdist > 30) e2 = kZTable;
            if (!e2) {
              for (int i = 0; i < 19; ++i) z.lens[i][0] = 0;
              for (int i = 0; i < hclen; ++i) z.lens[kClOrder[i]][0] = (uint8_t)getb<1>(b, src, z, 0, 3);
              if (!hbuild<kDFast, 1>(z, 0, z.lens, 0, 19, z.dfast, z.dlim, z.dbase, z.dsym)) e2 = kZTable;
            }
            int n = 0;
            const int total = hlit + hdist;
            while (!e2 && n < total) {
              const int s2 = hdecode<kDFast, 1>(b, src, z, z.dfast, z.dlim, z.dbase, z.dsym, kDsym, 0);
              if (s2 < 0) {
                e2 = kZCode;
                break;
              }
              int rep = 0, val = 0;
              if (s2 < 16) {
                z.lens[n++][0] = (uint8_t)s2;
                continue;
              } else if (s2 == 16) {
                if (n == 0) {
                  e2 = kZTable;
                  break;
                }
                val = z.lens[n - 1][0];
                rep = 3 + (int)getb<1>(b, src, z, 0, 2);
              } else if (s2 == 17) {
                rep = 3 + (int)getb<1>(b, src, z, 0, 3);
              } else {
                rep = 11 + (int)getb<1>(b, src, z, 0, 7);
              }
              if (n + rep > total) {
                e2 = kZTable;
                break;
              }
              for (int i = 0; i < rep; ++i) z.lens[n++][0] = (uint8_t)val;
            }
            if (!e2 && (z.lens[256][0] == 0 ||
                        !hbuild<kLFast, 1>(z, 0, z.lens, 0, hlit, z.lfast, z.llim, z.lbase, z.lsym) ||
                        !hbuild<kDFast, 1>(z, 0, z.lens, hlit, hdist, z.dfast, z.dlim, z.dbase, z.dsym)))
              e2 = kZTable;
            st2 = kStData;
          } else {
            e2 = kZBlockType;
          }
        }
        bp2 = consumed_bits(b, base);
      }
      err = __builtin_amdgcn_readfirstlane(e2);
      state = __builtin_amdgcn_readfirstlane(st2);
      last = __builtin_amdgcn_readfirstlane(l2);
      stored = __builtin_amdgcn_readfirstlane(stored);
      want = __builtin_amdgcn_readfirstlane(want);
      bp = (int64_t)__builtin_amdgcn_readfirstlane((uint32_t)bp2);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // lane 0's tables, for every lane
      if (err) break;
      if (bp > in_end + 64) {  // ran far past the stream: corrupt
        err = kZInput;
        break;
      }
      if (state == kStDone) {  // after the trailer
        if (o != olen) err = kZSize;
        else if (bp > in_end) err = kZInput;
        break;
      }
      if (state == kStStored) {
        const int64_t sb = base + (bp >> 3);  // byte aligned
        if (o + stored > olen) {
          err = kZOverflow;
          break;
        }
        if (sb + stored > c.src_off + c.src_len) {
          err = kZInput;
          break;
        }
        for (int i = lane; i < stored; i += 64) out[o + i] = src[sb + i];
        o += stored;
        bp += (int64_t)stored * 8;
        state = last ? kStTrailer : kStBlock;
        continue;
      }
      // the data path from bp: restart the wave ring at bp's dword
      whi = bp >> 5;
      refill();
      refill();
      continue;
    }
    // kStData: speculative rounds until the end-of-block token
    while (true) {
      if (whi - (bp >> 5) < 8) refill();
      const int64_t bl = bp + lane;
      const uint32_t di = (uint32_t)(bl >> 5), sh = (uint32_t)(bl & 31);
      const uint32_t d0 = wr[di % kWRing], d1 = wr[(di + 1) % kWRing], d2 = wr[(di + 2) % kWRing];
      uint64_t w = (((uint64_t)d1 << 32) | d0) >> sh;
      if (sh) w |= (uint64_t)d2 << (64 - sh);
      // the literal/length symbol
      int sym, cl;
      {
        const uint32_t e = z.lfast[(uint32_t)w & ((1u << kLFast) - 1u)][0];
        if (e >> 12) {
          cl = (int)(e >> 12);
          sym = (int)(e & 0x1FFu);
        } else {
          const uint32_t v = __builtin_bitreverse32((uint32_t)w) >> 17;
          int l = 0;
#pragma unroll
          for (int step = 8; step >= 1; step >>= 1)
            if (l + step <= 15 && v >= (uint32_t)z.llim[l + step][0]) l += step;
          cl = l + 1;
          if (cl > 15) {
            sym = -1;
          } else {
            const uint32_t i = (uint16_t)(z.lbase[cl][0] + (v >> (15 - cl)));
            sym = z.lsym[i < (uint32_t)kLsym ? i : (uint32_t)kLsym - 1u][0];
          }
        }
      }
      uint32_t kind, tl = (uint32_t)cl, mlen = 0, mdist = 0;
      if (sym < 0) {
        kind = kTokBad;
      } else if (sym < 256) {
        kind = kTokLit;
      } else if (sym == 256) {
        kind = kTokEob;
      } else if (sym - 257 >= 29) {
        kind = kTokBad;
      } else {
        const uint32_t le = z.ltab[sym - 257];
        const uint32_t lx = le >> 16;
        mlen = (le & 0xFFFFu) + TMH_ZBFE((uint32_t)(w >> cl), lx);
        const uint64_t w2 = w >> (cl + lx);
        int ds, dl;
        const uint32_t e = z.dfast[(uint32_t)w2 & ((1u << kDFast) - 1u)][0];
        if (e >> 12) {
          dl = (int)(e >> 12);
          ds = (int)(e & 0x1FFu);
        } else {
          const uint32_t v = __builtin_bitreverse32((uint32_t)w2) >> 17;
          int l = 0;
#pragma unroll
          for (int step = 8; step >= 1; step >>= 1)
            if (l + step <= 15 && v >= (uint32_t)z.dlim[l + step][0]) l += step;
          dl = l + 1;
          if (dl > 15) {
            ds = -1;
          } else {
            const uint32_t i = (uint16_t)(z.dbase[dl][0] + (v >> (15 - dl)));
            ds = z.dsym[i < (uint32_t)kDsym ? i : (uint32_t)kDsym - 1u][0];
          }
        }
        if (ds < 0 || ds >= 30) {
          kind = kTokBad;
        } else {
          const uint32_t de = z.dtab[ds];
          const uint32_t dx = de >> 16;
          mdist = (de & 0xFFFFu) + TMH_ZBFE((uint32_t)(w2 >> dl), dx);
          tl = (uint32_t)cl + lx + (uint32_t)dl + dx;
          kind = kTokMatch;
        }
      }
      const uint32_t tok = tl | (kind << 8);
      // the real token starts: a scalar walk from lane 0 along the lengths
      uint64_t mask = 0;
      uint32_t p = 0, stop = kTokLit;
      while (p < 64) {
        const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)tok, (int)p);
        const uint32_t k2 = t >> 8;
        if (k2 == kTokBad) {
          stop = kTokBad;
          break;
        }
        mask |= 1ull << p;
        p += t & 255u;
        if (k2 == kTokEob) {
          stop = kTokEob;
          break;
        }
      }
      if (stop == kTokBad) {
        err = kZCode;
        break;
      }
      const bool on = (mask >> lane) & 1ull;
      const bool lit = on && kind == kTokLit, mat = on && kind == kTokMatch;
      const uint64_t mmask = __builtin_amdgcn_ballot_w64(mat);
      uint32_t excl, total;
      if (!mmask) {  // literals only: one byte each
        excl = (uint32_t)__builtin_popcountll(mask & ((1ull << lane) - 1ull));
        total = (uint32_t)__builtin_popcountll(mask) - (stop == kTokEob ? 1u : 0u);
      } else {
        const uint32_t nb = lit ? 1u : (mat ? mlen : 0u);
        uint32_t incl = nb;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const uint32_t y = (uint32_t)__shfl_up((int)incl, off, 64);
          if (lane >= off) incl += y;
        }
        excl = incl - nb;
        total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      }
      const int nmat = __builtin_popcountll(mmask);
      bool bad = false;
      if (o + (int)total > olen || nm + nmat > ml_cap) {
        err = kZOverflow;
        break;
      }
      if (mat && mdist > (uint32_t)o + excl) bad = true;
      if (__builtin_amdgcn_ballot_w64(bad)) {
        err = kZDist;
        break;
      }
      if (lit) out[o + excl] = (uint8_t)sym;
      if (mat) {
        const int mi = nm + (int)__builtin_popcountll(mmask & ((1ull << lane) - 1ull));
        TMH_ZST8(ml + kMlHead + 2 * mi, (uint32_t)o + excl, mlen | (mdist << 9));
      }
      o += (int)total;
      nm += nmat;
      bp += p;
      if (bp > in_end + 64) {
        err = kZInput;
        break;
      }
      if (stop == kTokEob) {
        state = last ? kStTrailer : kStBlock;
        break;
      }
    }
    if (err) break;
  }
  if (lane == 0) {
    ml[0] = (uint32_t)nm;
    ml[1] = want;
  }
  if (err) {
    if (lane == 0) status[ci] = err;
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the literal bytes and the list
  const int32_t r = resolve_wave(out, olen, ml, lane);
  if (lane == 0) status[ci] = r;
}

// Chunk i's raw bytes (chunk_rows x chunk_cols elements, row-major) into
// image c.image of [*][height][width] at (row0, col0), clipped to the
// dataset's extent.  Workgroups of 256 threads, up to 64 per chunk, 16-byte
// copies where the row segments allow, else per byte.
__global__ __launch_bounds__(256) void k_place_chunks(const uint8_t* __restrict__ raw,
                                                      const tmh_zchunk* __restrict__ chunks,
                                                      int64_t n_chunks, int height, int width,
                                                      int esize, int chunk_rows, int chunk_cols,
                                                      uint8_t* __restrict__ images) {
  const int64_t ci = blockIdx.x;
  if (ci >= n_chunks) return;
  const tmh_zchunk c = chunks[ci];
  const int rows = min(chunk_rows, height - c.row0);
  const int cols = min(chunk_cols, width - c.col0);
  if (rows <= 0 || cols <= 0) return;
  const int64_t rb = (int64_t)cols * esize;                       // bytes per placed row
  const int64_t sstride = (int64_t)chunk_cols * esize;             // raw row stride
  const int64_t dstride = (int64_t)width * esize;
  const uint8_t* s = raw + c.raw_off;
  uint8_t* d = images + (c.image * height + c.row0) * dstride + (int64_t)c.col0 * esize;
  const bool v16 = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0 &&
                   (rb & 15) == 0 && (sstride & 15) == 0 && (dstride & 15) == 0;
  // the chunk's (row, 16-byte column) pairs spread over every thread of the
  // grid's y blocks (rows of a 160-column chunk are 20 vectors: a block per
  // row left 236 of 256 threads idle)
  const int64_t step = (int64_t)gridDim.y * 256;
  if (v16) {
    const int64_t per_row = rb / 16;
    for (int64_t t = (int64_t)blockIdx.y * 256 + threadIdx.x; t < rows * per_row; t += step) {
      const int64_t r = t / per_row, q = t - r * per_row;
      reinterpret_cast<uint4*>(d + r * dstride)[q] = reinterpret_cast<const uint4*>(s + r * sstride)[q];
    }
  } else {
    for (int64_t t = (int64_t)blockIdx.y * 256 + threadIdx.x; t < rows * rb; t += step) {
      const int64_t r = t / rb, q = t - r * rb;
      d[r * dstride + q] = s[r * sstride + q];
    }
  }
}

int64_t inflate_scratch_bytes(int64_t n_chunks, int64_t raw_max) {
  return n_chunks * match_words(raw_max) * 4;
}

// The decode form: "lane" (default: one lane per stream, two kernels) or
// "wave" (one wave per stream, speculative tokens, resolve + Adler-32 in the
// same kernel).  The wave form measured slower on the site images' 32 KB
// streams: 68.4 against 35.2 + 4.6 ms per 128 sites (one 64-bit window per
// round covers ~7 literal tokens of near-incompressible data, and each
// round's chain walk is a serial readlane chain; profiles/r5/
// bench_inflate_modes_r5i.json).  TMH_INFLATE_MODE selects one.
static bool inflate_wave_mode() {
  if (const char* e = getenv("TMH_INFLATE_MODE")) return strcmp(e, "wave") == 0;
  return false;
}

// Streams per phase-1 workgroup.  A lane's decode is a serial chain of
// dependent LDS lookups and ALU steps, so a wave of few lanes is as fast per
// symbol as a full one while its divergence (block headers, long codes, the
// literal and match paths) is paid for fewer lanes; LDS (~2.5 KB per stream)
// caps the streams resident at once at ~16k.  W = 8 (two to four waves per
// SIMD when a launch fills the chip) measured fastest at 128 and 384 sites
// per launch (profiles/r4/bench_inflate_*_r4n.json).  TMH_INFLATE_LANES =
// 4|8|16|32|64 overrides it.
static int inflate_lanes() {
  if (const char* e = getenv("TMH_INFLATE_LANES")) {
    const int w = atoi(e);
    if (w == 4 || w == 8 || w == 16 || w == 32 || w == 64) return w;
  }
  return 8;
}

template <int W>
static void launch_tokens(const uint8_t* src, int64_t src_bytes, const tmh_zchunk* chunks,
                          int64_t n_chunks, uint8_t* dst, int64_t dst_bytes, uint32_t* scratch,
                          int64_t mw, int32_t* status, hipStream_t s) {
  hipLaunchKernelGGL(k_inflate_tokens<W>, dim3((unsigned)cdiv(n_chunks, W)), dim3(W), 0, s, src,
                     src_bytes, chunks, n_chunks, dst, dst_bytes, scratch, mw, status);
}

void launch_inflate(const uint8_t* src, int64_t src_bytes, const tmh_zchunk* chunks,
                    int64_t n_chunks, int64_t raw_max, uint8_t* dst, int64_t dst_bytes,
                    uint32_t* scratch, int32_t* status, hipStream_t s) {
  if (n_chunks <= 0) return;
  const int64_t mw = match_words(raw_max);
  if (inflate_wave_mode()) {
    ProfScope prof("inflate", s);
    constexpr int NW = 4;  // waves (streams) per workgroup
    hipLaunchKernelGGL(k_inflate_wave<NW>, dim3((unsigned)cdiv(n_chunks, NW)), dim3(64 * NW), 0,
                       s, src, src_bytes, chunks, n_chunks, dst, dst_bytes, scratch, mw, status);
    TMH_HIP(hipGetLastError());
    return;
  }
  {
    ProfScope prof("inflate", s);
    switch (inflate_lanes()) {
      case 4: launch_tokens<4>(src, src_bytes, chunks, n_chunks, dst, dst_bytes, scratch, mw, status, s); break;
      case 8: launch_tokens<8>(src, src_bytes, chunks, n_chunks, dst, dst_bytes, scratch, mw, status, s); break;
      case 16: launch_tokens<16>(src, src_bytes, chunks, n_chunks, dst, dst_bytes, scratch, mw, status, s); break;
      case 32: launch_tokens<32>(src, src_bytes, chunks, n_chunks, dst, dst_bytes, scratch, mw, status, s); break;
      default: launch_tokens<64>(src, src_bytes, chunks, n_chunks, dst, dst_bytes, scratch, mw, status, s); break;
    }
  }
  {
    ProfScope prof("inflate_matches", s);
    hipLaunchKernelGGL(k_resolve_matches, dim3((unsigned)n_chunks), dim3(kZW), 0, s, chunks, dst,
                       scratch, mw, status);
  }
  TMH_HIP(hipGetLastError());
}

void launch_place_chunks(const uint8_t* raw, const tmh_zchunk* chunks, int64_t n_chunks,
                         int height, int width, int esize, int chunk_rows, int chunk_cols,
                         uint8_t* images, hipStream_t s) {
  if (n_chunks <= 0) return;
  ProfScope prof("place_chunks", s);
  // ~one 16-byte vector per thread: y blocks of 256 threads per chunk
  const int64_t vecs = ((int64_t)chunk_rows * chunk_cols * esize + 15) / 16;
  const unsigned ry = (unsigned)std::min<int64_t>(64, std::max<int64_t>(1, cdiv(vecs, 256)));
  hipLaunchKernelGGL(k_place_chunks, dim3((unsigned)n_chunks, ry), dim3(256), 0, s, raw, chunks,
                     n_chunks, height, width, esize, chunk_rows, chunk_cols, images);
  TMH_HIP(hipGetLastError());
}

}  // namespace tmh
