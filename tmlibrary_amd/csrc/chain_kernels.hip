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
                         int lo, int hi, double step) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = (uint8_t)scale8(in[i], lo, hi, step);
}

// u16 words K..K+7 of the 16 packed in d[8]
template <int K>
__device__ __forceinline__ void words8(const uint32_t (&d)[8], uint32_t (&px)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int q = K + j;
    px[j] = (q & 1) ? (d[q >> 1] >> 16) : (d[q >> 1] & 0xFFFFu);
  }
}

// correct one pixel (log2 domain, as the fused correct pass; image.py:599-631)
// -> x86 uint16 cast -> clip -> scale
template <bool LOG>
__device__ __forceinline__ uint32_t chain1(uint32_t px, float2 k, float mh, float zf, int lo,
                                           int hi, double step) {
  float L = (float)px;
  if (LOG) L = __builtin_amdgcn_logf(__builtin_fmaxf(L, zf));
  const float t = fmaf(L - k.x, k.y, mh);
  float o = LOG ? __builtin_amdgcn_exp2f(t) : t;
  o = __builtin_fminf(o, 2147418112.0f);  // >= 2^31, inf, NaN -> low half 0 (x86 astype)
  if (!LOG) o = __builtin_fmaxf(o, -2147483648.0f);
  uint32_t v = (uint32_t)(int32_t)o & 0xFFFFu;
  v = v < (uint32_t)lo ? (uint32_t)lo : (v > (uint32_t)hi ? (uint32_t)hi : v);
  return scale8(v, lo, hi, step);
}

// Fused chain, one thread = 8 consecutive output pixels of a row (W % 8 == 0),
// walking the sites of the launch.  Per site the source of the 8 pixels is a
// uniformly shifted run: two aligned 16-B buffer loads (out-of-range reads
// return 0) cover it and a uniform funnel shift picks the 8 values; the
// per-pixel (mean*log2(10), mean(std)/std) coefficients at the source
// positions are 8-B loads from the linear plane (L2-resident neighbourhood).
template <bool LOG>
__global__ __launch_bounds__(256) void k_chain_u8(const uint16_t* __restrict__ in,
                                                   uint8_t* __restrict__ out, int H, int W,
                                                   int64_t n_sites,
                                                   const float2* __restrict__ coef_lin,
                                                   const float4* __restrict__ mconst2,
                                                   const tmh_window* __restrict__ win, int lo,
                                                   int hi, double step) {
  const int64_t npx = (int64_t)H * W;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (npx >> 3)) return;
  const int r = (int)((g * 8) / W), c0 = (int)((g * 8) % W);
  const float4 m = mconst2[0];
  const uint32_t pad = scale8((uint32_t)lo, lo, hi, step);  // clip(0) = lo
  for (int64_t s = 0; s < n_sites; ++s) {
    const tmh_window w = win[s];  // uniform: scalar loads
    uint32_t o[8];
    const bool row_in = (unsigned)(r - w.dst_r0) < (unsigned)w.rows;
    const int dc = w.src_c0 - w.dst_c0;
    if (row_in && c0 - w.dst_c0 >= 0 && c0 + 7 - w.dst_c0 < w.cols) {
      // whole run inside the window
      const int sr = r - w.dst_r0 + w.src_r0;
      const int64_t p = (int64_t)sr * W + c0 + dc;  // first source pixel
      const int64_t a = p & ~(int64_t)7;
      const int k = (int)(p - a);  // uniform per site
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(in + s * npx), 0, (int)(npx * 2), 0x00020000);
      typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
      const u32x4_t v0 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(a * 2), 0, 0);
      const u32x4_t v1 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(a * 2) + 16, 0, 0);
      const uint32_t d[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      uint32_t px[8];
      switch (k) {  // uniform: one scalar branch per site
        case 0: words8<0>(d, px); break;
        case 1: words8<1>(d, px); break;
        case 2: words8<2>(d, px); break;
        case 3: words8<3>(d, px); break;
        case 4: words8<4>(d, px); break;
        case 5: words8<5>(d, px); break;
        case 6: words8<6>(d, px); break;
        default: words8<7>(d, px); break;
      }
      const float2* cf = coef_lin + p;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = chain1<LOG>(px[j], cf[j], m.x, m.z, lo, hi, step);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        if (row_in && in_window(r, c, w)) {
          const int64_t p = (int64_t)(r - w.dst_r0 + w.src_r0) * W + (c + dc);
          o[j] = chain1<LOG>(in[s * npx + p], coef_lin[p], m.x, m.z, lo, hi, step);
        } else {
          o[j] = pad;
        }
      }
    }
    uint2 packed = make_uint2(o[0] | (o[1] << 8) | (o[2] << 16) | (o[3] << 24),
                              o[4] | (o[5] << 8) | (o[6] << 16) | (o[7] << 24));
    reinterpret_cast<uint2*>(out + s * npx)[g] = packed;
  }
}

// Any width: one thread per output pixel.
template <bool LOG>
__global__ __launch_bounds__(256) void k_chain_u8_scalar(const uint16_t* __restrict__ in,
                                                          uint8_t* __restrict__ out, int H, int W,
                                                          int64_t n_sites,
                                                          const float2* __restrict__ coef_lin,
                                                          const float4* __restrict__ mconst2,
                                                          const tmh_window* __restrict__ win,
                                                          int lo, int hi, double step) {
  const int64_t npx = (int64_t)H * W;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npx) return;
  const int r = (int)(i / W), c = (int)(i % W);
  const float4 m = mconst2[0];
  for (int64_t s = 0; s < n_sites; ++s) {
    const tmh_window w = win[s];
    uint32_t v = scale8((uint32_t)lo, lo, hi, step);
    if (in_window(r, c, w)) {
      const int64_t p = (int64_t)(r - w.dst_r0 + w.src_r0) * W + (c - w.dst_c0 + w.src_c0);
      v = chain1<LOG>(in[s * npx + p], coef_lin[p], m.x, m.z, lo, hi, step);
    }
    out[s * npx + i] = (uint8_t)v;
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
                     const float2* coef_lin, const float4* mconst2, int log_transform,
                     const tmh_window* d_win, int lo, int hi, hipStream_t s) {
  if (n_sites <= 0) return;
  ProfScope prof("chain", s);
  const int64_t npx = (int64_t)H * W;
  const double step = scale_step(lo, hi);
  const bool vec = (W & 7) == 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(out) & 7) == 0 && npx * 2 < (int64_t)1 << 31;
  if (vec) {
    const dim3 grid((unsigned)cdiv(npx >> 3, 256));
    if (log_transform)
      hipLaunchKernelGGL(k_chain_u8<true>, grid, dim3(256), 0, s, in, out, H, W, n_sites, coef_lin,
                         mconst2, d_win, lo, hi, step);
    else
      hipLaunchKernelGGL(k_chain_u8<false>, grid, dim3(256), 0, s, in, out, H, W, n_sites,
                         coef_lin, mconst2, d_win, lo, hi, step);
  } else {
    const dim3 grid((unsigned)cdiv(npx, 256));
    if (log_transform)
      hipLaunchKernelGGL(k_chain_u8_scalar<true>, grid, dim3(256), 0, s, in, out, H, W, n_sites,
                         coef_lin, mconst2, d_win, lo, hi, step);
    else
      hipLaunchKernelGGL(k_chain_u8_scalar<false>, grid, dim3(256), 0, s, in, out, H, W, n_sites,
                         coef_lin, mconst2, d_win, lo, hi, step);
  }
  TMH_HIP(hipGetLastError());
}

}  // namespace tmh
