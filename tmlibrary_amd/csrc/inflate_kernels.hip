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

// (Round 5's whole-wave decode -- one wave per stream, speculative tokens --
// measured slower on the site images' 32 KB streams, 68.4 against 35.2 + 4.6
// ms per 128 sites, profiles/r5/bench_inflate_modes_r5i.json; removed in
// round 6, see git history.)

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
