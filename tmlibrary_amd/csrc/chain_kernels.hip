// illuminati post-correct chain (gfx950 / MI355X): SURVEY.md §8(f) rank 3.
//
// Reference: tmlib/workflow/illuminati/api.py:396-405 takes every corrected
// site through
//   image.correct(stats)            tmlib/image.py:633-670
//        .align(crop=False)         tmlib/image.py:345-454  (shift + zero pad)
//        .clip(clip_min, clip_max)  tmlib/image.py:570-597
//        .scale(clip_min, clip_max) tmlib/image.py:493-568  (uint16 -> uint8 LUT)
// before cutting pyramid tiles.  k_chain_u8 does all four in one pass that
// reads the uint16 site (2 B/px) and writes the uint8 tile source (1 B/px).
//
// align is a window copy: the host evaluates the reference's numpy slicing
// into (src_r0, src_c0, dst_r0, dst_c0, rows, cols); output pixels outside
// the destination window are 0, which clip/scale map to scale8(clip_min) = 0.
//
// scale is the reference's LUT
//   zeros(lo) | linspace(0, 255, hi - lo).astype(uint16) | 255 * ones(65536 - hi)
// evaluated per pixel the way numpy builds it: entry lo + i is
// trunc(double(i) * (255.0 / (n - 1))) with n = hi - lo, except the last one
// (i = n - 1), which linspace sets to exactly 255, and n = 1 (a lone 0).  One
// f64 multiply, bit-identical to the table (pinned exhaustively against the
// reference's LUTs, tests/golden/map_uint8.npz).
#include "common.h"

namespace tmh {

__device__ __forceinline__ uint32_t scale8(uint32_t v, int lo, int hi, double step) {
  if (v < (uint32_t)lo) return 0u;
  if (v >= (uint32_t)hi) return 255u;
  const int n = hi - lo, i = (int)v - lo;
  if (n == 1) return 0u;
  if (i == n - 1) return 255u;
  return (uint32_t)((double)i * step);  // x in [0, 255): trunc == astype(uint16)
}

__device__ __forceinline__ bool in_window(int r, int c, const tmh_window& w) {
  return (unsigned)(r - w.dst_r0) < (unsigned)w.rows && (unsigned)(c - w.dst_c0) < (unsigned)w.cols;
}

// align (any dtype): out[n][oh][ow], window per site
template <typename T>
__global__ void k_align(const T* __restrict__ in, T* __restrict__ out, int H, int W, int oh, int ow,
                        const tmh_window* __restrict__ win) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t s = blockIdx.y;
  if (i >= (int64_t)oh * ow) return;
  const tmh_window w = win[s];
  const int r = (int)(i / ow), c = (int)(i % ow);
  T v = (T)0;
  if (in_window(r, c, w))
    v = in[s * (int64_t)H * W + (int64_t)(r - w.dst_r0 + w.src_r0) * W + (c - w.dst_c0 + w.src_c0)];
  out[s * (int64_t)oh * ow + i] = v;
}

__global__ void k_map_u8(const uint16_t* __restrict__ in, uint8_t* __restrict__ out, int64_t n,
                         int lo, int hi, double step) {  // no clip: the LUT's zeros / 255 tails
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = (uint8_t)scale8(in[i], lo, hi, step);
}

// Clip to [lo, hi] then the reference LUT, branch-free: T = n - 1 for
// n = hi - lo > 1 (linspace's end point and v = hi give 255), T = 1 for n = 1.
__device__ __forceinline__ uint32_t clip_scale8(uint32_t v16, int lo, int hi, int T, double step) {
  const uint32_t v = min(max(v16, (uint32_t)lo), (uint32_t)hi);
  const uint32_t i = v - (uint32_t)lo;
  return i >= (uint32_t)T ? 255u : (uint32_t)((double)i * step);
}

// one pixel px (site s, source index p) of the packed-f32 correction; m =
// mconst2 (M' hi, M' lo, zf, T): beyond T the pixel is flagged for the f64
// refinement (common.h, k_fix_chain)
template <bool LOG>
__device__ __forceinline__ uint32_t correct16(uint32_t px, float mu, float a, const float4 m,
                                              int64_t s, int64_t p, const FixList& fl) {
  float L = (float)px;
  if (LOG) L = __builtin_amdgcn_logf(__builtin_fmaxf(L, m.z));
  const float t = fmaf(L - mu, a, m.x);
  float o = LOG ? __builtin_amdgcn_exp2f(t) : t;
  if (__builtin_fabsf(o) >= m.w) fix_push(fl, s, p);
  o = __builtin_fminf(o, 2147418112.0f);  // >= 2^31, inf, NaN -> low half 0 (x86 astype)
  if (!LOG) o = __builtin_fmaxf(o, -2147483648.0f);
  return (uint32_t)(int32_t)o & 0xFFFFu;
}

// Source-driven fused chain (W % 8 == 0): one thread = 8 consecutive SOURCE
// pixels, their coefficients loaded once and reused for every site of its
// part (blockIdx.y = site part).  align is a flat shift per site, off =
// (dst_r0 - src_r0) * W + (dst_c0 - src_c0): source pixel p lands at p + off,
// a bijection onto [off, npx + off), and source pixels outside the window land
// outside the destination window (they write the padding value, 0 scaled).
// The 8 result bytes of thread i go to [8i + off, 8i + off + 8); unless off
// is a multiple of the 128-B line they are staged in LDS per workgroup and
// stored as line-aligned 16-B chunks.  k_chain_fill pads [0, off) / [npx + off,
// npx), the only destinations no source pixel reaches.
// n < 8 bytes of v (low first) at the 8-aligned address p: dword, short, byte
// pieces, each naturally aligned
__device__ __forceinline__ void store_head(uint8_t* p, uint64_t v, int n) {
  if (n & 4) {
    *reinterpret_cast<uint32_t*>(p) = (uint32_t)v;
    p += 4;
    v >>= 32;
  }
  if (n & 2) {
    *reinterpret_cast<uint16_t*>(p) = (uint16_t)v;
    p += 2;
    v >>= 16;
  }
  if (n & 1) *p = (uint8_t)v;
}

// the low n < 8 bytes of v ending just below the 8-aligned address end
__device__ __forceinline__ void store_tail(uint8_t* end, uint64_t v, int n) {
  uint8_t* p = end - n;
  if (n & 1) {
    *p = (uint8_t)v;
    p += 1;
    v >>= 8;
  }
  if (n & 2) {
    *reinterpret_cast<uint16_t*>(p) = (uint16_t)v;
    p += 2;
    v >>= 16;
  }
  if (n & 4) *reinterpret_cast<uint32_t*>(p) = (uint32_t)v;
}

// blockIdx -> tile with XCD x (= blockIdx % 8, the dispatch round-robin)
// owning tiles [x*q + min(x, r), ...) of n = 8q + r: a bijection on [0, n)
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t n) {
  const int64_t q = n / 8, r = n % 8, x = b % 8, k = b / 8;
  return x * q + (x < r ? x : r) + k;
}

typedef float f32x2c_t __attribute__((ext_vector_type(2)));
constexpr int kChainDepth = 4;

// streamed-once site loads: non-temporal
__device__ __forceinline__ uint4 ld_nt16(const uint4* p) {
  typedef unsigned int u32x4n_t __attribute__((ext_vector_type(4)));
  const u32x4n_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4n_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// LUT 0: clip + scale in f64 arithmetic; 1: the reference's uint8 table for
// the clipped range [lo, hi] staged in LDS (hi - lo + 1 bytes), one ds_read_u8
// per pixel after the clip; 2: clip and table for every 16-bit value (64 KB,
// copied from lut8, k_chain_lut8), indexed by the cast's low half directly --
// the pass is VALU-bound (~24 ops + 2 transcendentals per pixel), and this
// drops the clip's max/min and the index subtract.  NT threads per workgroup.
template <bool LOG, int LUT, int NT = 256>
__global__ __launch_bounds__(NT) void k_chain_u8(const uint16_t* __restrict__ in,
                                                  uint8_t* __restrict__ out, int H, int W,
                                                  int64_t n_sites, int64_t per,
                                                  const float2* __restrict__ coef_lin,
                                                  const float4* __restrict__ mconst2,
                                                  FixList fl,
                                                  const tmh_window* __restrict__ win, int lo,
                                                  int hi, int T, double step,
                                                  const uint8_t* __restrict__ lut8) {
  extern __shared__ __attribute__((aligned(16))) uint8_t slut[];
  if (LUT == 1) {
    for (int i = threadIdx.x; i <= hi - lo; i += NT)
      slut[i] = (uint8_t)(i >= T ? 255u : (uint32_t)((double)i * step));
    __syncthreads();
  } else if (LUT == 2) {
    for (int i = threadIdx.x; i < 65536 / 16; i += NT)
      reinterpret_cast<uint4*>(slut)[i] = reinterpret_cast<const uint4*>(lut8)[i];
    __syncthreads();
  }
  const int64_t npx = (int64_t)H * W;
  const int64_t ngroups = npx >> 3;
  // XCD-aware tile order: workgroups go round-robin over the 8 XCDs, so give
  // XCD x a contiguous run of tiles -- neighbouring tiles' shifted outputs
  // share a 128-B line at their seam, and a seam inside one XCD's L2 merges
  // instead of leaving two partial lines to write back.
  const int64_t tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t g = tile * NT + threadIdx.x;
  const bool live = g < ngroups;
  const int lane = threadIdx.x & 63;
  const bool top_lane = threadIdx.x == NT - 1 || g + 1 >= ngroups;  // no upper neighbour run
  __shared__ uint64_t edge[NT / 64];
  __shared__ __attribute__((aligned(16))) uint8_t stage[NT * 8 + 256];
  const int64_t p0 = (live ? g : 0) * 8;
  const int r = (int)(p0 / W), c0 = (int)(p0 % W);
  const float4 m = mconst2[0];
  const f32x2c_t M = {m.x, m.x};
  f32x2c_t mu[4], a[4];
  {
    const float4* cf = reinterpret_cast<const float4*>(coef_lin + p0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v0 = live ? cf[k] : make_float4(0.f, 1.f, 0.f, 1.f);
      mu[k] = (f32x2c_t){v0.x, v0.z};
      a[k] = (f32x2c_t){v0.y, v0.w};
    }
  }
  const int64_t s0 = (int64_t)blockIdx.y * per;
  const int64_t s1 = s0 + per < n_sites ? s0 + per : n_sites;
  const uint4* src = reinterpret_cast<const uint4*>(in) + (live ? g : 0);
  // kChainDepth sites' loads in flight ahead of the one being processed
  uint4 q[kChainDepth];
#pragma unroll
  for (int k = 0; k < kChainDepth; ++k)
    q[k] = live && s0 + k < s1 ? ld_nt16(src + (s0 + k) * ngroups) : make_uint4(0, 0, 0, 0);
  for (int64_t s = s0; s < s1; ++s) {
    const uint4 cur = q[0];
#pragma unroll
    for (int k = 0; k + 1 < kChainDepth; ++k) q[k] = q[k + 1];
    q[kChainDepth - 1] = live && s + kChainDepth < s1 ? ld_nt16(src + (s + kChainDepth) * ngroups)
                                                      : make_uint4(0, 0, 0, 0);
    const tmh_window w = win[s];  // uniform: scalar loads
    const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
    f32x2c_t t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      t[k].x = (float)(wd[k] & 0xFFFFu);
      t[k].y = (float)(wd[k] >> 16);
    }
    if (LOG) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        t[k].x = __builtin_amdgcn_logf(__builtin_fmaxf(t[k].x, m.z));
        t[k].y = __builtin_amdgcn_logf(__builtin_fmaxf(t[k].y, m.z));
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = __builtin_elementwise_fma(t[k] - mu[k], a[k], M);
    uint32_t o[8];
    float mx = 0.0f;  // largest |result| of the 8 pixels: one compare against T per 8
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float x = LOG ? __builtin_amdgcn_exp2f(t[k][h]) : t[k][h];
        mx = __builtin_fmaxf(mx, __builtin_fabsf(x));
        x = __builtin_fminf(x, 2147418112.0f);  // >= 2^31, inf, NaN -> low half 0 (x86)
        if (!LOG) x = __builtin_fmaxf(x, -2147483648.0f);
        const uint32_t v16 = (uint32_t)(int32_t)x & 0xFFFFu;
        if (LUT == 2) {
          o[2 * k + h] = slut[v16];
        } else {
          const uint32_t v = min(max(v16, (uint32_t)lo), (uint32_t)hi);  // np.clip
          o[2 * k + h] = LUT ? (uint32_t)slut[v - (uint32_t)lo]
                             : (v - (uint32_t)lo >= (uint32_t)T ? 255u
                                                                : (uint32_t)((double)(v - lo) * step));
        }
      }
    }
    // rare: a pixel beyond the f32 bound flags its group of 8 for the f64
    // refinement (common.h; f64 is the reference value for all 8)
    if (mx >= m.w && live) fix_push8(fl, 0xFFu, s, p0);
    // pixels outside the source window write the padding value: 0 after
    // clip/scale (clip(0) = lo, the table's first entry is 0)
    const int cs = c0 - w.src_c0;
    int jlo = -cs < 0 ? 0 : (-cs > 8 ? 8 : -cs);
    int jhi = w.cols - cs < 0 ? 0 : (w.cols - cs > 8 ? 8 : w.cols - cs);
    if ((unsigned)(r - w.src_r0) >= (unsigned)w.rows) jhi = 0;
    const uint64_t keep = jhi > jlo ? ((~0ull >> (8 * (8 - (jhi - jlo)))) << (8 * jlo)) : 0ull;
    const uint32_t lo4 = (o[0] | (o[1] << 8) | (o[2] << 16) | (o[3] << 24)) & (uint32_t)keep;
    const uint32_t hi4 = (o[4] | (o[5] << 8) | (o[6] << 16) | (o[7] << 24)) & (uint32_t)(keep >> 32);
    const uint64_t v8 = ((uint64_t)hi4 << 32) | lo4;
    const int64_t off = (int64_t)(w.dst_r0 - w.src_r0) * W + (w.dst_c0 - w.src_c0);
    const int64_t D = p0 + off;  // destination of byte 0
    const int rr = (int)(off & 7);  // uniform
    uint8_t* o8 = out + s * npx;
    if ((off & 127) == 0) {  // line-aligned destination: direct stores
      if (live && D >= 0 && D < npx) *reinterpret_cast<uint64_t*>(o8 + D) = v8;
      continue;
    }
    // Otherwise the workgroup's 2,048 output bytes [o0, o0 + 2048) are staged
    // in LDS and leave as whole 16-B chunks of 128-B lines: a shifted run
    // written lane by lane would split every wave's store across one more,
    // partial line on each side.  Runs are first made 8-byte aligned with the
    // upper neighbour's bytes (wave shuffle, LDS slot across waves).
    const int wv = threadIdx.x >> 6;
    if (lane == 0) edge[wv] = v8;
    const uint32_t nlo = (uint32_t)__shfl_down((int)lo4, 1, 64);
    const uint32_t nhi = (uint32_t)__shfl_down((int)hi4, 1, 64);
    __syncthreads();  // (1) edge slots written; the previous site's stage is drained
    uint64_t n8 = ((uint64_t)nhi << 32) | nlo;
    if (lane == 63 && wv < NT / 64 - 1) n8 = edge[wv + 1];
    const int64_t o0 = tile * NT * 8 + off;  // destination of thread 0's byte 0
    const int64_t L0 = o0 >= 0 ? (o0 & ~(int64_t)127) : -((-o0 + 127) & ~(int64_t)127);
    if (!live) {
      // no run (past the last group): nothing to stage
    } else if (rr == 0) {
      *reinterpret_cast<uint64_t*>(stage + (D - L0)) = v8;
    } else {
      const int64_t A = D - rr + 8;  // aligned word holding our bytes [8 - rr, 8)
      if (!top_lane) {
        *reinterpret_cast<uint64_t*>(stage + (A - L0)) = (v8 >> (8 * (8 - rr))) | (n8 << (8 * rr));
      } else {
        for (int b = 8 - rr; b < 8; ++b) stage[D + b - L0] = (uint8_t)(v8 >> (8 * b));
      }
      if (threadIdx.x == 0)
        for (int b = 0; b < 8 - rr; ++b) stage[D + b - L0] = (uint8_t)(v8 >> (8 * b));
    }
    __syncthreads();  // (2) stage complete
    // valid destination bytes of this workgroup: [o0, o0 + 2048) within the
    // site (the last workgroup may own fewer groups)
    const int64_t wg_bytes = (ngroups - tile * NT < NT ? ngroups - tile * NT : NT) * 8;
    const int64_t v0 = o0 > 0 ? o0 : 0;
    const int64_t v1 = o0 + wg_bytes < npx ? o0 + wg_bytes : npx;
    const int64_t c = L0 + 16 * (int64_t)threadIdx.x;  // this thread's 16-B chunk
    if (c + 16 <= v1 && c >= v0) {
      *reinterpret_cast<uint4*>(o8 + c) = *reinterpret_cast<const uint4*>(stage + (c - L0));
    } else if (c < v1 && c + 16 > v0) {
      for (int b = 0; b < 16; ++b)
        if (c + b >= v0 && c + b < v1) o8[c + b] = stage[c + b - L0];
    }
  }
}

// The production chain pass: k_chain_u8's 16-bit-table form with its VALU
// trimmed (the pass is VALU-bound: ~24 issue slots per pixel, two of them
// quarter-rate transcendentals).
//  * no queue of site loads (below);
//  * a group flagged when its max |o| passes the f32 error bound of its
//    largest a, |o| (K1 a_max8 + K2) >= 1 (the fused pass's per-pixel rule,
//    fcorrect8, with the group's largest a), and k_fix_chain refines only the
//    pixels beyond their own bound (the launch-wide T = 1 / (K1 a_max + K2)
//    with whole groups refined ran 0.30 ms of f64 fixups per 3,456 bench
//    sites);
//  * no min/max before the cast: every |o| >= 1 / K2 (< 2^18) fails its own
//    f32 bound and is refined in f64; k_fix_chain refines only the pixels
//    beyond their own bound and keeps the streamed byte of the others, whose
//    |o| < 0.998 / K2 < 2^18 -- there v_cvt_i32_f32 truncates exactly as the
//    x86 cast does, so no clamp is needed; NaN converts to 0 on both;
//  * ZADD: a zero pixel's floor as x + zf instead of max(x, zf) -- two pixels
//    per v_pk_add_f32; exact for zf < 2^-25 (x >= 1 plus zf rounds to x);
//  * the table bytes packed with v_perm (3 per 4 bytes) instead of shifts,
//    ors and a masking bitop;
//  * the align window's byte mask only for threads whose 8 pixels are not all
//    inside it (a divergent branch: whole waves skip it).
template <bool LOG, bool ZADD, int NT, bool PF = false, bool GB = true, bool SEAM = false>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2 * NT / 256))) void k_chain_u8t(const uint16_t* __restrict__ in,
                                                   uint8_t* __restrict__ out, int H, int W,
                                                   int64_t n_sites, int64_t per,
                                                   const float2* __restrict__ coef_lin,
                                                   const float4* __restrict__ mconst2, FixList fl,
                                                   const tmh_window* __restrict__ win,
                                                   const uint8_t* __restrict__ lut8) {
  extern __shared__ __attribute__((aligned(16))) uint8_t slut[];
  for (int i = threadIdx.x; i < 65536 / 16; i += NT)
    reinterpret_cast<uint4*>(slut)[i] = reinterpret_cast<const uint4*>(lut8)[i];
  __syncthreads();
  const int64_t npx = (int64_t)H * W;
  const int64_t ngroups = npx >> 3;
  const int64_t tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t g = tile * NT + threadIdx.x;
  const bool live = g < ngroups;
  const int lane = threadIdx.x & 63;
  const bool top_lane = threadIdx.x == NT - 1 || g + 1 >= ngroups;
  // SEAM: only the 128-B lines two waves share are staged (two sets, one
  // barrier per site); otherwise the whole workgroup's bytes (k_chain_u8's
  // staging, two barriers per site)
  constexpr int kSeams = NT / 64 + 1;  // seam s = line L0 + 512 s
  __shared__ uint64_t edge[SEAM ? 1 : NT / 64];
  __shared__ __attribute__((aligned(16))) uint8_t stage[SEAM ? 2 * kSeams * 128 : NT * 8 + 256];
  const int64_t p0 = (live ? g : 0) * 8;
  const int r = (int)(p0 / W), c0 = (int)(p0 % W);
  const float4 m = mconst2[0];
  const f32x2c_t M = {m.x, m.x};
  const f32x2c_t Z = {m.z, m.z};
  f32x2c_t mu[4], a[4];
  float thr;  // this thread's flag threshold on max |o| (below)
  {
    const float4* cf = reinterpret_cast<const float4*>(coef_lin + p0);
    float am = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v0 = live ? cf[k] : make_float4(0.f, 1.f, 0.f, 1.f);
      mu[k] = (f32x2c_t){v0.x, v0.z};
      a[k] = (f32x2c_t){v0.y, v0.w};
      am = __builtin_fmaxf(am, __builtin_fmaxf(__builtin_fabsf(v0.y), __builtin_fabsf(v0.w)));
    }
    // the fused pass's per-pixel bound |o| (K1 a + K2) >= 0.998 (fcorrect8),
    // taken with the largest a of the thread's 8 pixels: max |o| >= thr flags
    // the group (a superset of the pixels the per-pixel bound flags)
    constexpr float K1 = (float)(kRefineK1 * 1.002), K2 = (float)(kRefineK2 * 1.002);
    thr = 0.998f / __builtin_fmaf(am, K1, K2);
  }
  const int64_t s0 = (int64_t)blockIdx.y * per;
  const int64_t s1 = s0 + per < n_sites ? s0 + per : n_sites;
  const uint4* src = reinterpret_cast<const uint4*>(in) + (live ? g : 0);

  auto site = [&](const uint4 cur, const int64_t s) {
    const tmh_window w = win[s];  // uniform: scalar loads
    const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
    f32x2c_t t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      t[k].x = (float)(wd[k] & 0xFFFFu);
      t[k].y = (float)(wd[k] >> 16);
    }
    if (LOG) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (ZADD) {
          t[k] += Z;
        } else {
          t[k].x = __builtin_fmaxf(t[k].x, m.z);
          t[k].y = __builtin_fmaxf(t[k].y, m.z);
        }
        t[k].x = __builtin_amdgcn_logf(t[k].x);
        t[k].y = __builtin_amdgcn_logf(t[k].y);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = __builtin_elementwise_fma(t[k] - mu[k], a[k], M);
    float mx = 0.0f;  // largest |result| of the 8 pixels (v_max3 with |.| modifiers)
    uint32_t o[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float x = LOG ? __builtin_amdgcn_exp2f(t[k][h]) : t[k][h];
        mx = __builtin_fmaxf(mx, __builtin_fabsf(x));
        o[2 * k + h] = slut[(uint32_t)(int32_t)x & 0xFFFFu];
      }
    }
    // bytes (o0, o1, o2, o3): v_perm pairs, then the pairs' low halves -- in
    // the loads' basic block, where the compiler knows the bytes are
    // zero-extended (sunk past the branch below it masks each byte first)
    uint32_t lo4 = __builtin_amdgcn_perm(__builtin_amdgcn_perm(o[3], o[2], 0x0c0c0400u),
                                         __builtin_amdgcn_perm(o[1], o[0], 0x0c0c0400u), 0x05040100u);
    uint32_t hi4 = __builtin_amdgcn_perm(__builtin_amdgcn_perm(o[7], o[6], 0x0c0c0400u),
                                         __builtin_amdgcn_perm(o[5], o[4], 0x0c0c0400u), 0x05040100u);
    asm volatile("" : "+v"(lo4), "+v"(hi4));  // keeps the packing here (no code is emitted)
    if (mx >= (GB ? thr : m.w) && live) fix_push8(fl, 0xFFu, s, p0);
    // pixels outside the source window write the padding value (0 after
    // clip/scale); only threads with a pixel outside build the byte mask
    const int cs = c0 - w.src_c0;
    const bool inside = w.cols >= 8 && (unsigned)(r - w.src_r0) < (unsigned)w.rows &&
                        (unsigned)cs <= (unsigned)(w.cols - 8);
    if (!inside) {
      int jlo = -cs < 0 ? 0 : (-cs > 8 ? 8 : -cs);
      int jhi = w.cols - cs < 0 ? 0 : (w.cols - cs > 8 ? 8 : w.cols - cs);
      if ((unsigned)(r - w.src_r0) >= (unsigned)w.rows) jhi = 0;
      const uint64_t keep = jhi > jlo ? ((~0ull >> (8 * (8 - (jhi - jlo)))) << (8 * jlo)) : 0ull;
      lo4 &= (uint32_t)keep;
      hi4 &= (uint32_t)(keep >> 32);
    }
    const uint64_t v8 = ((uint64_t)hi4 << 32) | lo4;
    // byte offsets inside one site fit in 32 bits (the launch checks npx < 2^30)
    const int n32 = (int)npx;
    const int off = (w.dst_r0 - w.src_r0) * W + (w.dst_c0 - w.src_c0);  // uniform
    const int D = (int)p0 + off;  // destination of byte 0
    const int rr = off & 7;       // uniform
    uint8_t* o8 = out + s * npx;
    // the destinations no source pixel reaches -- [0, off) for off > 0,
    // [npx + off, npx) for off < 0, all outside the destination window -- take
    // the padding value, written by the site part's first / last workgroup
    // (k_chain_fill's job for k_chain_u8)
    if ((off > 0 && tile == 0) || (off < 0 && tile == (int64_t)gridDim.x - 1)) {
      const int b0 = off > 0 ? 0 : n32 + off, b1 = off > 0 ? off : n32;
      const uint8_t pad = slut[0];
#pragma unroll 1
      for (int b = b0 + (int)threadIdx.x; b < b1; b += NT) o8[b] = pad;
    }
    if ((off & 127) == 0) {  // line-aligned destination: direct stores
      if (live && (unsigned)D < (unsigned)n32) *reinterpret_cast<uint64_t*>(o8 + D) = v8;
      return;
    }
    if (SEAM) {
      // A wave's 512 output bytes [o0 + 512 w, +512) fully cover the three
      // lines L0 + 512 w + 128 k (k = 1..3): its lanes store their aligned
      // 8-byte words there directly.  The lines L0 + 512 s (s = 0..16) are
      // shared with the neighbouring wave (or workgroup): their words and the
      // partial words at the waves' edges go to an LDS copy of those lines,
      // stored after one barrier as whole 16-B chunks.
      const int o0 = (int)(tile * NT * 8) + off;  // uniform
      const int L0 = o0 & ~127;
      uint8_t* seam = stage + (int)(s & 1) * (kSeams * 128);
      const uint32_t nlo = (uint32_t)__shfl_down((int)lo4, 1, 64);
      const uint32_t nhi = (uint32_t)__shfl_down((int)hi4, 1, 64);
      const uint64_t n8 = ((uint64_t)nhi << 32) | nlo;
      const bool wtop = lane == 63 || g + 1 >= ngroups;  // no upper neighbour in the wave
      if (live) {
        const int X = rr == 0 ? D : D - rr + 8;  // the aligned word this lane completes
        const int r = X - L0;
        const bool in_seam = (r & 511) < 128;
        uint8_t* sp = seam + (r >> 9) * 128 + (r & 127);
        if (rr == 0 || !wtop) {  // a whole word: ours, or our [8 - rr, 8) + the upper lane's [0, 8 - rr)
          const uint64_t v = rr == 0 ? v8 : (v8 >> (8 * (8 - rr))) | (n8 << (8 * rr));
          if (in_seam)
            *reinterpret_cast<uint64_t*>(sp) = v;
          else if ((unsigned)X < (unsigned)n32)
            *reinterpret_cast<uint64_t*>(o8 + X) = v;
        } else {  // the wave's top lane: only our bytes of that word
          if (in_seam)
            store_head(sp, v8 >> (8 * (8 - rr)), rr);
          else if ((unsigned)X < (unsigned)n32)
            store_head(o8 + X, v8 >> (8 * (8 - rr)), rr);
        }
        if (rr != 0 && lane == 0) {  // our bytes [0, 8 - rr): the top of word X - 8, a seam line
          const int q = X - 8 - L0;
          store_tail(seam + (q >> 9) * 128 + (q & 127) + 8, v8, 8 - rr);
        }
      }
      __syncthreads();  // seam lines complete (the other set was read before it)
      const int wg_bytes = (int)((ngroups - tile * NT < NT ? ngroups - tile * NT : NT) * 8);
      const int v0 = o0 > 0 ? o0 : 0;
      const int v1 = o0 + wg_bytes < n32 ? o0 + wg_bytes : n32;
      if ((int)threadIdx.x < kSeams * 8) {
        const int sl = threadIdx.x >> 3, ch = threadIdx.x & 7;
        const int c = L0 + 512 * sl + 16 * ch;
        const uint8_t* src8 = seam + sl * 128 + 16 * ch;
        if (c + 16 <= v1 && c >= v0) {
          *reinterpret_cast<uint4*>(o8 + c) = *reinterpret_cast<const uint4*>(src8);
        } else if (c < v1 && c + 16 > v0) {
          for (int b = 0; b < 16; ++b)
            if (c + b >= v0 && c + b < v1) o8[c + b] = src8[b];
        }
      }
      return;
    }
    // as k_chain_u8: the workgroup's output bytes staged in LDS and stored as
    // whole 16-B chunks of 128-B lines (runs first made 8-byte aligned with the
    // upper neighbour's bytes: wave shuffle, LDS slot across waves)
    const int wv = threadIdx.x >> 6;
    if (lane == 0) edge[wv] = v8;
    const uint32_t nlo = (uint32_t)__shfl_down((int)lo4, 1, 64);
    const uint32_t nhi = (uint32_t)__shfl_down((int)hi4, 1, 64);
    __syncthreads();  // (1) edge slots written; the previous site's stage is drained
    uint64_t n8 = ((uint64_t)nhi << 32) | nlo;
    if (lane == 63 && wv < NT / 64 - 1) n8 = edge[wv + 1];
    const int o0 = (int)(tile * NT * 8) + off;  // uniform: destination of thread 0's byte 0
    const int L0 = o0 & ~127;                   // its line (floor, also for o0 < 0)
    if (!live) {
      // past the last group: nothing to stage
    } else if (rr == 0) {
      *reinterpret_cast<uint64_t*>(stage + (D - L0)) = v8;
    } else {
      const int A = D - rr + 8;  // aligned word holding our bytes [8 - rr, 8)
      if (!top_lane) {
        *reinterpret_cast<uint64_t*>(stage + (A - L0)) = (v8 >> (8 * (8 - rr))) | (n8 << (8 * rr));
      } else {
        for (int b = 8 - rr; b < 8; ++b) stage[D + b - L0] = (uint8_t)(v8 >> (8 * b));
      }
      if (threadIdx.x == 0)
        for (int b = 0; b < 8 - rr; ++b) stage[D + b - L0] = (uint8_t)(v8 >> (8 * b));
    }
    __syncthreads();  // (2) stage complete
    // valid destination bytes of this workgroup: [v0, v1) (uniform)
    const int wg_bytes = (int)((ngroups - tile * NT < NT ? ngroups - tile * NT : NT) * 8);
    const int v0 = o0 > 0 ? o0 : 0;
    const int v1 = o0 + wg_bytes < n32 ? o0 + wg_bytes : n32;
    const int c = L0 + 16 * (int)threadIdx.x;  // this thread's 16-B chunk
    if (c + 16 <= v1 && c >= v0) {
      *reinterpret_cast<uint4*>(o8 + c) = *reinterpret_cast<const uint4*>(stage + (c - L0));
    } else if (c < v1 && c + 16 > v0) {
      for (int b = 0; b < 16; ++b)
        if (c + b >= v0 && c + b < v1) o8[c + b] = stage[c + b - L0];
    }
  };

  // one site's load, then its processing: k_chain_u8's queue of kChainDepth
  // loads compiled to a full wait for the load just issued (a conditional load
  // in the loop), i.e. this same order, plus 16 register moves per site; the
  // 32 waves of a CU hide the latency.  (A pipeline that really keeps loads in
  // flight across sites ran slower for this shape: 19.4 vs 14.5 ms,
  // profiles/r3/mb_chain_pipeline_r3n.txt.)
  if (PF) {  // the next site's load issued before this site's processing
    if (s0 >= s1) return;
    uint4 nxt = ld_nt16(src + s0 * ngroups);
    for (int64_t s = s0; s < s1; ++s) {
      const uint4 cur = nxt;
      nxt = ld_nt16(src + (s + 1 < s1 ? s + 1 : s) * ngroups);  // unconditional
      site(cur, s);
    }
  } else {
    for (int64_t s = s0; s < s1; ++s)
      site(live ? ld_nt16(src + s * ngroups) : make_uint4(0, 0, 0, 0), s);
  }
}

// The 16-bit clip + scale table of k_chain_u8<LUT = 2>: entry v = scale8(clip(v)).
__global__ void k_chain_lut8(uint8_t* __restrict__ lut8, int lo, int hi, int T, double step) {
  const int v = (int)blockIdx.x * 256 + threadIdx.x;
  if (v < 65536) lut8[v] = (uint8_t)clip_scale8((uint32_t)v, lo, hi, T, step);
}

// The destinations no source pixel reaches: [0, off) for off > 0, [npx + off,
// npx) for off < 0 (all outside the destination window).
__global__ void k_chain_fill(uint8_t* __restrict__ out, int H, int W,
                             const tmh_window* __restrict__ win, int lo, int hi, int T,
                             double step) {
  const int64_t npx = (int64_t)H * W;
  const int64_t s = blockIdx.y;
  const tmh_window w = win[s];
  const int64_t off = (int64_t)(w.dst_r0 - w.src_r0) * W + (w.dst_c0 - w.src_c0);
  const int64_t b0 = off > 0 ? 0 : npx + off, b1 = off > 0 ? off : npx;
  const uint8_t pad = (uint8_t)clip_scale8(0u, lo, hi, T, step);
  for (int64_t i = b0 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < b1;
       i += (int64_t)gridDim.x * 256)
    out[s * npx + i] = pad;
}

// Any width: one thread per output pixel.
template <bool LOG>
__global__ __launch_bounds__(256) void k_chain_u8_scalar(const uint16_t* __restrict__ in,
                                                          uint8_t* __restrict__ out, int H, int W,
                                                          int64_t n_sites,
                                                          const float2* __restrict__ coef_lin,
                                                          const float4* __restrict__ mconst2,
                                                          FixList fl,
                                                          const tmh_window* __restrict__ win,
                                                          int lo, int hi, int T, double step) {
  const int64_t npx = (int64_t)H * W;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npx) return;
  const int r = (int)(i / W), c = (int)(i % W);
  const float4 m = mconst2[0];
  for (int64_t s = 0; s < n_sites; ++s) {
    const tmh_window w = win[s];
    uint32_t v = clip_scale8(0u, lo, hi, T, step);
    if (in_window(r, c, w)) {
      const int64_t p = (int64_t)(r - w.dst_r0 + w.src_r0) * W + (c - w.dst_c0 + w.src_c0);
      const float2 k = coef_lin[p];
      v = clip_scale8(correct16<LOG>(in[s * npx + p], k.x, k.y, m, s, p, fl), lo, hi, T, step);
    }
    out[s * npx + i] = (uint8_t)v;
  }
}

// f64 refinement of the chain pixels the pass flagged (FixList, common.h;
// source pixels): the corrected value -> clip -> scale, written at the pixel's
// aligned destination; pixels outside the source window were written as
// padding and are left alone.  Overflowed list: every source pixel.
// A pixel of a flagged group whose f32 value (recomputed with the streaming
// kernels' own instructions) lies within its error bound |o| (K1 a + K2) <
// 0.998 keeps the byte the streaming kernel wrote; the others are refined.
template <bool LOG>
__global__ __launch_bounds__(256) void k_fix_chain(const uint16_t* __restrict__ in,
                                                   uint8_t* __restrict__ out, int H, int W,
                                                   int64_t n_sites, FixList fl,
                                                   const double2* __restrict__ c64,
                                                   const RefineConst* __restrict__ rc,
                                                   const tmh_window* __restrict__ win, int lo,
                                                   int hi, int T, double step,
                                                   const float2* __restrict__ coef_lin,
                                                   const float4* __restrict__ mconst2) {
  const int64_t npx = (int64_t)H * W;
  const unsigned int n = *fl.n;
  const bool all = n > fl.cap;
  const int64_t total = all ? n_sites * ((npx + 7) / 8) : (int64_t)n;
  if (total == 0) return;
  const RefineConst k = *rc;
  // one thread per (entry, pixel): the 8 lanes of an entry read its pixels
  // and coefficients together, and the rare f64 refinements spread over lanes
  for (int64_t it = (int64_t)blockIdx.x * 256 + threadIdx.x; it < total * 8;
       it += (int64_t)gridDim.x * 256) {
    const int64_t i = it >> 3;
    const int j = (int)(it & 7);
    int64_t s, p0;
    uint32_t mask;
    fix_entry(fl, all, i, npx, s, p0, mask);
    {
      const int64_t p = p0 + j;
      if (!((mask >> j) & 1u) || p >= npx) continue;
      const tmh_window w = win[s];
      const int r = (int)(p / W), c = (int)(p - (int64_t)r * W);
      if ((unsigned)(r - w.src_r0) >= (unsigned)w.rows ||
          (unsigned)(c - w.src_c0) >= (unsigned)w.cols)
        continue;
      const uint16_t px = in[s * npx + p];
      {  // the streaming kernels' f32 value and its bound
        constexpr float K1 = (float)(kRefineK1 * 1.002), K2 = (float)(kRefineK2 * 1.002);
        const float4 m = mconst2[0];
        const float2 cf = coef_lin[p];
        float L = (float)px;
        if (LOG) L = __builtin_amdgcn_logf(__builtin_fmaxf(L, m.z));
        const float t = __builtin_fmaf(L - cf.x, cf.y, m.x);
        const float o = LOG ? __builtin_amdgcn_exp2f(t) : t;
        if (__builtin_fabsf(o) * __builtin_fmaf(cf.y, K1, K2) < 0.998f) continue;
      }
      const double2 q = c64[p];
      const uint32_t v16 =
          (uint32_t)correct_ref_f64<LOG>(px, q.x, q.y, k.S, k.M, k.zero_log10) & 0xFFFFu;
      const int64_t d = (int64_t)(r - w.src_r0 + w.dst_r0) * W + (c - w.src_c0 + w.dst_c0);
      out[s * npx + d] = (uint8_t)clip_scale8(v16, lo, hi, T, step);
    }
  }
}

double scale_step(int lo, int hi) { return hi - lo > 1 ? 255.0 / (double)(hi - lo - 1) : 0.0; }

void launch_align(const void* in, void* out, int elem_bytes, int64_t n_sites, int H, int W, int oh,
                  int ow, const tmh_window* d_win, hipStream_t s) {
  if (n_sites <= 0 || (int64_t)oh * ow == 0) return;
  const dim3 grid((unsigned)cdiv((int64_t)oh * ow, 256), (unsigned)n_sites);
  if (elem_bytes == 2)
    hipLaunchKernelGGL(k_align<uint16_t>, grid, dim3(256), 0, s, (const uint16_t*)in,
                       (uint16_t*)out, H, W, oh, ow, d_win);
  else
    hipLaunchKernelGGL(k_align<uint8_t>, grid, dim3(256), 0, s, (const uint8_t*)in, (uint8_t*)out,
                       H, W, oh, ow, d_win);
  TMH_HIP(hipGetLastError());
}

void launch_map_u8(const uint16_t* in, uint8_t* out, int64_t n, int lo, int hi, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_map_u8, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, in, out, n, lo, hi,
                     scale_step(lo, hi));
  TMH_HIP(hipGetLastError());
}

void launch_chain_u8(const uint16_t* in, uint8_t* out, int H, int W, int64_t n_sites,
                     const float2* coef_lin, const float4* mconst2, const FixList& fl,
                     const double2* coef64, const RefineConst* rc, int log_transform,
                     const tmh_window* d_win, int lo, int hi, uint8_t* lut8, hipStream_t s,
                     double zero_log10) {
  if (n_sites <= 0) return;
  ProfScope prof("chain", s);
  const int64_t npx = (int64_t)H * W;
  const double step = scale_step(lo, hi);
  const int T = hi - lo > 1 ? hi - lo - 1 : 1;
  const bool vec = (W & 7) == 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(out) & 7) == 0 && npx < ((int64_t)1 << 30);
  if (vec) {
    // site parts even out the dispatch rounds (each thread streams its part)
    const int64_t parts = n_sites >= 64 ? 8 : 1;
    const int64_t per = cdiv(n_sites, parts);
    const int lut_bytes = hi - lo + 1;
    const bool lut = lut_bytes <= 16384;  // else three f64 ops per pixel
    const size_t shm = lut ? (size_t)((lut_bytes + 15) & ~15) : 0;
#define TMH_CHAIN(L_, U_, NT_, SHM_, LUT8_)                                                      \
  hipLaunchKernelGGL((k_chain_u8<L_, U_, NT_>),                                                  \
                     dim3((unsigned)cdiv(npx >> 3, NT_), (unsigned)cdiv(n_sites, per)), dim3(NT_), \
                     SHM_, s, in, out, H, W, n_sites, per, coef_lin, mconst2, fl, d_win, lo, hi, T,  \
                     step, LUT8_)
    if (lut8) {
      // the whole 16-bit table: 1,024-thread workgroups (two per CU with the
      // 64 KB table; smaller ones copy it too often: 256 threads ran 37 ms,
      // 512 21.6, 1,024 14.6 against 15.0 for the clipped-range table,
      // profiles/r2/mb_chain_lut64_r2lt.txt)
      hipLaunchKernelGGL(k_chain_lut8, dim3(256), dim3(256), 0, s, lut8, lo, hi, T, step);
      // 16 site parts: 3,456 sites of 2160x2560 ran 12.49 ms against 12.77
      // with 8 (tools/mb/mb_chain.hip)
      const int64_t tparts = n_sites >= 128 ? 16 : parts, tper = cdiv(n_sites, tparts);
      const dim3 grid((unsigned)cdiv(npx >> 3, 1024), (unsigned)cdiv(n_sites, tper));
#define TMH_CHAIN_T(L_, Z_)                                                                      \
  hipLaunchKernelGGL((k_chain_u8t<L_, Z_, 1024, true, true, true>), grid, dim3(1024), 65536, s, \
                     in, out, H, W, n_sites, tper, coef_lin, mconst2, fl, d_win, lut8)
      // zf = 10**zero_log10 below 2^-25 (~2.98e-8): the floor as an add is exact
      if (!log_transform) TMH_CHAIN_T(false, false);
      else if (zero_log10 <= -8.0) TMH_CHAIN_T(true, true);
      else TMH_CHAIN_T(true, false);
#undef TMH_CHAIN_T
    } else {
      if (log_transform) {
        if (lut) TMH_CHAIN(true, 1, 256, shm, nullptr); else TMH_CHAIN(true, 0, 256, shm, nullptr);
      } else {
        if (lut) TMH_CHAIN(false, 1, 256, shm, nullptr); else TMH_CHAIN(false, 0, 256, shm, nullptr);
      }
      hipLaunchKernelGGL(k_chain_fill, dim3(64, (unsigned)n_sites), dim3(256), 0, s, out, H, W,
                         d_win, lo, hi, T, step);
    }
#undef TMH_CHAIN
  } else {
    const dim3 grid((unsigned)cdiv(npx, 256));
    if (log_transform)
      hipLaunchKernelGGL(k_chain_u8_scalar<true>, grid, dim3(256), 0, s, in, out, H, W, n_sites,
                         coef_lin, mconst2, fl, d_win, lo, hi, T, step);
    else
      hipLaunchKernelGGL(k_chain_u8_scalar<false>, grid, dim3(256), 0, s, in, out, H, W, n_sites,
                         coef_lin, mconst2, fl, d_win, lo, hi, T, step);
  }
  if (log_transform)
    hipLaunchKernelGGL(k_fix_chain<true>, dim3(2048), dim3(256), 0, s, in, out, H, W, n_sites, fl,
                       coef64, rc, d_win, lo, hi, T, step, coef_lin, mconst2);
  else
    hipLaunchKernelGGL(k_fix_chain<false>, dim3(2048), dim3(256), 0, s, in, out, H, W, n_sites,
                       fl, coef64, rc, d_win, lo, hi, T, step, coef_lin, mconst2);
  TMH_HIP(hipGetLastError());
}

}  // namespace tmh
