// Fused correct + per-site histogram pass (gfx950 / MI355X).
//
// The job reads every site twice at minimum: once for the Welford statistics
// (pixel-major, mean/M2 in registers across all sites) and once for the
// correction (which needs the finished, smoothed statistics).  The per-site
// intensity percentiles (stats.py:76) need nothing but the raw pixels, so
// their histograms are built from the correction's read instead of a pass of
// their own: HBM traffic is then the algorithmic 2 + 4 B/px per site.
//
// Layout of the work: the image is cut into kBands pixel bands; XCD x owns
// bands {x, x+8} and walks (band, site) units band-major from its own queue,
// so a band's correction coefficients (f32 mean, f32 mean(std)/std: 8 B/px,
// 2.76 MB at 2160x2560) stay resident in that XCD's 4 MB L2 while the sites
// stream through.  A workgroup corrects one unit, histograms its raw pixels in
// LDS, and adds the non-zero counts to the site's global histogram with
// contiguous-lane atomics.  Idle XCDs steal from other queues (placement is
// a speed choice only; every unit is processed exactly once).
#include <cstdlib>

#include "common.h"

namespace tmh {

constexpr int kBandsPerXcd = 2;  // default; TMH_FUSED_BANDS overrides (experiments)
constexpr int kFThreads = 1024;
constexpr int kFLut = 4000;  // float2 LDS LUT: 131,072 (bins) + 32,000 + small <= 160 KiB
constexpr float kLog2_10f = 3.32192809488736234787f;

__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7;
}

__device__ __noinline__ float2 fused_log_slow(uint32_t u) {
  const double L = log10((double)u);
  const float hi = (float)L;
  return make_float2(hi, (float)(L - (double)hi));
}

template <bool LOG>
__device__ __forceinline__ uint32_t fcorrect(float Lh, float Ll, float mu, float a, float mh,
                                             float ml, int clip_lo, int clip_hi) {
  const float d = (Lh - mu) + Ll;                  // (img - mean)
  const float t = fmaf(d, a, mh) + ml;             // * mean(std)/std + mean(mean)
  const float o = LOG ? exp2f(t * kLog2_10f) : t;  // 10 ** t
  const int32_t iv = (o >= -2147483648.0f && o < 2147483648.0f) ? (int32_t)o : INT32_MIN;
  uint32_t r = (uint32_t)iv & 0xFFFFu;             // x86 astype(uint16)
  if (clip_lo >= 0) {
    r = r < (uint32_t)clip_lo ? (uint32_t)clip_lo : r;
    r = r > (uint32_t)clip_hi ? (uint32_t)clip_hi : r;
  }
  return r;
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld_px(const uint4* p) {
  if (NT) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *p;
}

template <bool NT>
__device__ __forceinline__ void st_px(uint4* p, uint4 v) {
  if (NT) {
    const u32x4_t w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(p));
  } else {
    *p = v;
  }
}

template <bool LOG, bool NT>
__global__ __launch_bounds__(kFThreads) void k_correct_hist(
    const uint16_t* __restrict__ in, uint16_t* __restrict__ out, int64_t npx, int64_t n_sites,
    const float2* __restrict__ coef2, const float2* __restrict__ lut,
    const float2* __restrict__ mconst, int clip_lo, int clip_hi, uint32_t* __restrict__ hist,
    int* __restrict__ queues, int bands_per_xcd) {
  __shared__ __attribute__((aligned(16))) uint32_t bins[kLdsBins];
  __shared__ float2 slut[kFLut];
  __shared__ int unit_sh;
  const int tid = threadIdx.x;
  for (int i = tid; i < kLdsBins / 4; i += kFThreads)
    reinterpret_cast<uint4*>(bins)[i] = make_uint4(0u, 0u, 0u, 0u);
  if (LOG)
    for (int i = tid; i < kFLut; i += kFThreads) slut[i] = lut[i];
  __syncthreads();

  const float2 m = mconst[0];
  const int64_t ngroups = npx >> 3;
  const int n_bands = 8 * bands_per_xcd;
  const int64_t units_per_queue = bands_per_xcd * n_sites;  // bands x, x+8, ...
  const uint4* src = reinterpret_cast<const uint4*>(in);
  uint4* dst = reinterpret_cast<uint4*>(out);
  const float4* cf = reinterpret_cast<const float4*>(coef2);  // 2 px per float4

  int q = xcc_id(), exhausted = 0;
  while (exhausted < 8) {
    if (tid == 0) unit_sh = atomicAdd(&queues[q], 1);
    __syncthreads();
    const int u = unit_sh;
    __syncthreads();
    if (u >= units_per_queue) {  // this queue is drained: steal from the next
      q = (q + 1) & 7;
      ++exhausted;
      continue;
    }
    exhausted = 0;
    const int band = q + 8 * (u / (int)n_sites);
    const int64_t s = u % n_sites;
    const int64_t g0 = band * ngroups / n_bands, g1 = (band + 1) * ngroups / n_bands;
    const uint4* sp = src + s * ngroups;
    uint4* dp = dst + s * ngroups;
    uint32_t* hs = hist + s * (int64_t)kBins;

    auto process = [&](const uint4 v, const float4 c0, const float4 c1, const float4 c2,
                       const float4 c3) -> uint4 {
      const uint32_t px[8] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16,
                              v.z & 0xFFFFu, v.z >> 16, v.w & 0xFFFFu, v.w >> 16};
      const float mu[8] = {c0.x, c0.z, c1.x, c1.z, c2.x, c2.z, c3.x, c3.z};
      const float a[8] = {c0.y, c0.w, c1.y, c1.w, c2.y, c2.w, c3.y, c3.w};
      uint32_t mx = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        mx = px[k] > mx ? px[k] : mx;
        atomicAdd(&bins[px[k] & (kLdsBins - 1)], px[k] < (uint32_t)kLdsBins);
      }
      float2 l[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        l[k] = LOG ? slut[px[k] < (uint32_t)kFLut ? px[k] : 0u] : make_float2((float)px[k], 0.f);
      if (mx >= (uint32_t)kFLut) {  // rare: beyond the LDS LUT and/or the LDS bins
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (LOG && px[k] >= (uint32_t)kFLut) l[k] = fused_log_slow(px[k]);
          if (px[k] >= (uint32_t)kLdsBins) atomicAdd(&hs[px[k]], 1u);
        }
      }
      uint32_t o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        o[k] = fcorrect<LOG>(l[k].x, l[k].y, mu[k], a[k], m.x, m.y, clip_lo, clip_hi);
      return make_uint4(o[0] | (o[1] << 16), o[2] | (o[3] << 16), o[4] | (o[5] << 16),
                        o[6] | (o[7] << 16));
    };

    // two-stage pipeline over the unit's pixel groups
    int64_t g = g0 + tid;
    uint4 v = make_uint4(0, 0, 0, 0);
    float4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    if (g < g1) {
      v = ld_px<NT>(sp + g);
      c0 = cf[g * 4]; c1 = cf[g * 4 + 1]; c2 = cf[g * 4 + 2]; c3 = cf[g * 4 + 3];
    }
    while (g < g1) {
      const int64_t gn = g + kFThreads;
      uint4 vn = make_uint4(0, 0, 0, 0);
      float4 n0 = {}, n1 = {}, n2 = {}, n3 = {};
      if (gn < g1) {
        vn = ld_px<NT>(sp + gn);
        n0 = cf[gn * 4]; n1 = cf[gn * 4 + 1]; n2 = cf[gn * 4 + 2]; n3 = cf[gn * 4 + 3];
      }
      st_px<NT>(dp + g, process(v, c0, c1, c2, c3));
      v = vn; c0 = n0; c1 = n1; c2 = n2; c3 = n3;
      g = gn;
    }
    // fold this unit's histogram into the site's (contiguous lanes -> bins)
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < kLdsBins / kFThreads; ++j) {
      const int b = j * kFThreads + tid;
      const uint32_t c = bins[b];
      if (c) {
        atomicAdd(&hs[b], c);
        bins[b] = 0u;
      }
    }
    __syncthreads();
  }
}

void launch_correct_hist(const uint16_t* in, uint16_t* out, int64_t npx, int64_t n_sites,
                         const float2* coef2, const float2* lut, const float2* mconst,
                         int log_transform, int clip_lo, int clip_hi, uint32_t* hist,
                         int* queues, int n_wg, hipStream_t s) {
  if (n_sites <= 0) return;
  ProfScope prof("correct_hist", s);
  static const int bpx = [] {
    const char* e = getenv("TMH_FUSED_BANDS");
    const int v = e ? atoi(e) : kBandsPerXcd;
    return v >= 1 && v <= 16 ? v : kBandsPerXcd;
  }();
  static const bool nt = [] {
    const char* e = getenv("TMH_FUSED_NT");
    return e ? atoi(e) != 0 : true;
  }();
  TMH_HIP(hipMemsetAsync(queues, 0, 8 * sizeof(int), s));
#define TMH_LAUNCH_CH(L_, N_)                                                                 \
  hipLaunchKernelGGL((k_correct_hist<L_, N_>), dim3(n_wg), dim3(kFThreads), 0, s, in, out, npx, \
                     n_sites, coef2, lut, mconst, clip_lo, clip_hi, hist, queues, bpx)
  if (log_transform && nt) TMH_LAUNCH_CH(true, true);
  else if (log_transform) TMH_LAUNCH_CH(true, false);
  else if (nt) TMH_LAUNCH_CH(false, true);
  else TMH_LAUNCH_CH(false, false);
#undef TMH_LAUNCH_CH
  TMH_HIP(hipGetLastError());
}

// coef2[i] = (f32 mean, f32 mean(std)/std): the compact per-pixel form the
// fused pass keeps L2-resident (|mean| rounding adds <= 0.023*a DN at 65535)
__global__ void k_coeffs2(const double* __restrict__ mean, const double* __restrict__ std,
                          const double* __restrict__ sums, int64_t npx,
                          float2* __restrict__ coef2) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npx) return;
  const double S = sums[0] / (double)npx;
  coef2[i] = make_float2((float)mean[i], (float)(S / std[i]));
}

void launch_coeffs2(const double* mean, const double* std, const double* sums, int64_t npx,
                    float2* coef2, hipStream_t s) {
  hipLaunchKernelGGL(k_coeffs2, dim3((unsigned)cdiv(npx, 256)), dim3(256), 0, s, mean, std, sums,
                     npx, coef2);
  TMH_HIP(hipGetLastError());
}

}  // namespace tmh
