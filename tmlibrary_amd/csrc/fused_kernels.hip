// Fused correct + per-site histogram pass (gfx950 / MI355X).
//
// The job reads every site twice at minimum: once for the Welford statistics
// (pixel-major, mean/M2 in registers across all sites) and once for the
// correction (which needs the finished, smoothed statistics).  The per-site
// intensity percentiles (stats.py:76) need nothing but the raw pixels, so
// their histograms are built from the correction's read instead of a pass of
// their own: HBM traffic is then the algorithmic 2 + 4 B/px per site.
//
// Layout of the work: the image is cut into 8 * bands_per_xcd pixel bands;
// XCD x owns bands {x, x+8, ...} and walks (band, site-group) units
// band-major from its own queue, so a band's correction coefficients (8 B/px:
// 2.76 MB per band at 2160x2560 and 2 bands per XCD) stay resident in that
// XCD's 4 MB L2 while the sites stream through.  A unit is SPU sites of one
// band: each lane loads its 8 pixels' coefficients once and applies them to
// the SPU sites, so the L2 coefficient traffic is 8/SPU B/px.  Each site of
// the unit histograms its raw pixels into its own LDS slice (values below
// kLdsBins/SPU; larger values go straight to the global histogram), and at
// the end of the unit the slices are added to the sites' global histograms
// with contiguous-lane atomics, only up to the largest value the unit saw.
// Idle XCDs steal from other queues (placement is a speed choice only; every
// unit is processed exactly once).
//
// Arithmetic (ChannelImage._correct_illumination, tmlib/image.py:599-631), in
// the log2 domain so 10**t is one v_exp_f32:
//   t2 = (log2(img) - mean*log2(10)) * mean(std)/std + mean(mean)*log2(10)
//   out = astype_uint16_x86(2**t2)
// log2 is v_log_f32 (<= 1 ulp: <= 0.1 DN at 65535); mean*log2(10) and
// mean(std)/std are f32 (mean's rounding adds <= 0.05*a DN at 65535); zero
// pixels take the reference's log10(1e-10) = -10.  Parity bar: +-1 DN.
#include <cstdlib>

#include "common.h"

namespace tmh {

constexpr int kBandsPerXcd = 2;  // default; TMH_FUSED_BANDS overrides (experiments)
constexpr int kFThreads = 1024;
constexpr double kLog2_10 = 3.32192809488736234787;

__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7;
}

template <bool LOG>
__device__ __forceinline__ uint32_t fcorrect(uint32_t px, float mu, float a, float mh, float ml,
                                             float zero_l, int clip_lo, int clip_hi) {
  float L;
  if (LOG)
    L = px ? __builtin_amdgcn_logf((float)px) : zero_l;  // v_log_f32
  else
    L = (float)px;
  const float t = fmaf(L - mu, a, mh) + ml;
  const float o = LOG ? __builtin_amdgcn_exp2f(t) : t;  // v_exp_f32
  const int32_t iv = (o >= -2147483648.0f && o < 2147483648.0f) ? (int32_t)o : INT32_MIN;
  uint32_t r = (uint32_t)iv & 0xFFFFu;  // x86 astype(uint16)
  if (clip_lo >= 0) {
    r = r < (uint32_t)clip_lo ? (uint32_t)clip_lo : r;
    r = r > (uint32_t)clip_hi ? (uint32_t)clip_hi : r;
  }
  return r;
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void st_nt(uint4* p, uint4 v) {
  const u32x4_t w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(p));
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

// ABL: development ablations (tools/mb), 0 in production: 1 = no histogram,
// 2 = constant coefficients, 8 = no flush
template <bool LOG, int SPU, int ABL = 0>
__global__ __launch_bounds__(kFThreads) void k_correct_hist(
    const uint16_t* __restrict__ in, uint16_t* __restrict__ out, int64_t npx, int64_t n_sites,
    const float2* __restrict__ coef2, const float4* __restrict__ mconst2, int clip_lo,
    int clip_hi, uint32_t* __restrict__ hist, int* __restrict__ queues, int bands_per_xcd) {
  constexpr int BINS = kLdsBins / SPU;
  __shared__ __attribute__((aligned(16))) uint32_t bins[kLdsBins];
  __shared__ int unit_sh;
  __shared__ uint32_t top_sh[SPU];
  const int tid = threadIdx.x;
  for (int i = tid; i < kLdsBins / 4; i += kFThreads)
    reinterpret_cast<uint4*>(bins)[i] = make_uint4(0u, 0u, 0u, 0u);

  const float4 m = mconst2[0];
  const int64_t ngroups = npx >> 3;
  const int n_bands = 8 * bands_per_xcd;
  const int64_t n_groups_s = (n_sites + SPU - 1) / SPU;
  const int64_t units_per_queue = bands_per_xcd * n_groups_s;
  const uint4* src = reinterpret_cast<const uint4*>(in);
  uint4* dst = reinterpret_cast<uint4*>(out);
  // coefficient planes: plane k holds pixels 8g+2k, 8g+2k+1 of group g, so each
  // of a lane's four coefficient loads is one contiguous 1 KiB per wave
  const float4* cf = reinterpret_cast<const float4*>(coef2);
  const float4 cc = make_float4(2.5f, 1.1f, 2.4f, 0.9f);

  int q = xcc_id(), exhausted = 0;
  while (exhausted < 8) {
    if (tid == 0) unit_sh = atomicAdd(&queues[q], 1);
    if (tid < SPU) top_sh[tid] = 0u;
    __syncthreads();
    const int u = unit_sh;
    __syncthreads();
    if (u >= units_per_queue) {  // this queue is drained: steal from the next
      q = (q + 1) & 7;
      ++exhausted;
      continue;
    }
    exhausted = 0;
    const int band = q + 8 * (int)(u / n_groups_s);
    const int64_t s0 = (u % n_groups_s) * SPU;
    const int ns = (int)(n_sites - s0 < SPU ? n_sites - s0 : SPU);
    const int64_t g0 = band * ngroups / n_bands, g1 = (band + 1) * ngroups / n_bands;
    const uint4* sp = src + s0 * ngroups;
    uint4* dp = dst + s0 * ngroups;
    uint32_t* hs = hist + s0 * (int64_t)kBins;
    uint32_t top[SPU];
#pragma unroll
    for (int k = 0; k < SPU; ++k) top[k] = 0u;

    auto process = [&](const uint4 v, const int k, const float4 c0, const float4 c1,
                       const float4 c2, const float4 c3) -> uint4 {
      const uint32_t px[8] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16,
                              v.z & 0xFFFFu, v.z >> 16, v.w & 0xFFFFu, v.w >> 16};
      const float mu[8] = {c0.x, c0.z, c1.x, c1.z, c2.x, c2.z, c3.x, c3.z};
      const float a[8] = {c0.y, c0.w, c1.y, c1.w, c2.y, c2.w, c3.y, c3.w};
      uint32_t mx = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mx = px[j] > mx ? px[j] : mx;
        if (!(ABL & 1)) atomicAdd(&bins[k * BINS + (px[j] & (BINS - 1))], px[j] < (uint32_t)BINS);
      }
      top[k] = mx > top[k] ? mx : top[k];
      if (!(ABL & 1) && mx >= (uint32_t)BINS) {  // rare: beyond this site's LDS slice
        uint32_t* h = hs + k * (int64_t)kBins;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (px[j] >= (uint32_t)BINS) atomicAdd(&h[px[j]], 1u);
      }
      uint32_t o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = fcorrect<LOG>(px[j], mu[j], a[j], m.x, m.y, m.z, clip_lo, clip_hi);
      return make_uint4(o[0] | (o[1] << 16), o[2] | (o[3] << 16), o[4] | (o[5] << 16),
                        o[6] | (o[7] << 16));
    };

    // two-stage pipeline over the unit's pixel groups
    int64_t g = g0 + tid;
    uint4 v[SPU];
    float4 c0 = cc, c1 = cc, c2 = cc, c3 = cc;
#pragma unroll
    for (int k = 0; k < SPU; ++k) v[k] = make_uint4(0, 0, 0, 0);
    if (g < g1) {
#pragma unroll
      for (int k = 0; k < SPU; ++k)
        if (k < ns) v[k] = ld_nt(sp + k * ngroups + g);
      if (!(ABL & 2)) {
        c0 = cf[g]; c1 = cf[ngroups + g]; c2 = cf[2 * ngroups + g]; c3 = cf[3 * ngroups + g];
      }
    }
    while (g < g1) {
      const int64_t gn = g + kFThreads;
      uint4 vn[SPU];
      float4 n0 = cc, n1 = cc, n2 = cc, n3 = cc;
#pragma unroll
      for (int k = 0; k < SPU; ++k) vn[k] = make_uint4(0, 0, 0, 0);
      if (gn < g1) {
#pragma unroll
        for (int k = 0; k < SPU; ++k)
          if (k < ns) vn[k] = ld_nt(sp + k * ngroups + gn);
        if (!(ABL & 2)) {
          n0 = cf[gn]; n1 = cf[ngroups + gn]; n2 = cf[2 * ngroups + gn]; n3 = cf[3 * ngroups + gn];
        }
      }
#pragma unroll
      for (int k = 0; k < SPU; ++k)
        if (k < ns) st_nt(dp + k * ngroups + g, process(v[k], k, c0, c1, c2, c3));
#pragma unroll
      for (int k = 0; k < SPU; ++k) v[k] = vn[k];
      c0 = n0; c1 = n1; c2 = n2; c3 = n3;
      g = gn;
    }
    // largest value per site in this unit bounds the bins worth flushing
#pragma unroll
    for (int k = 0; k < SPU; ++k) {
      const uint32_t t = wave_max(top[k]);
      if ((tid & 63) == 0) atomicMax(&top_sh[k], t);
    }
    __syncthreads();
    if (ABL & 9) continue;
    // fold this unit's slices into the sites' histograms (contiguous lanes -> bins)
#pragma unroll
    for (int k = 0; k < SPU; ++k) {
      if (k >= ns) break;
      const uint32_t t = top_sh[k];
      const int lim = (int)(t < (uint32_t)BINS ? t : (uint32_t)BINS - 1);
      uint32_t* h = hs + k * (int64_t)kBins;
      for (int b = tid; b <= lim; b += kFThreads) {
        const uint32_t c = bins[k * BINS + b];
        if (c) {
          atomicAdd(&h[b], c);
          bins[k * BINS + b] = 0u;
        }
      }
    }
    __syncthreads();
  }
}

static int fused_spu() {
  static const int v = [] {
    const char* e = getenv("TMH_FUSED_SPU");
    const int x = e ? atoi(e) : 2;
    return (x == 1 || x == 2 || x == 4) ? x : 2;
  }();
  return v;
}

void launch_correct_hist(const uint16_t* in, uint16_t* out, int64_t npx, int64_t n_sites,
                         const float2* coef2, const float4* mconst2, int log_transform,
                         int clip_lo, int clip_hi, uint32_t* hist, int* queues, int n_wg,
                         hipStream_t s) {
  if (n_sites <= 0) return;
  ProfScope prof("correct_hist", s);
  static const int bpx = [] {
    const char* e = getenv("TMH_FUSED_BANDS");
    const int v = e ? atoi(e) : kBandsPerXcd;
    return v >= 1 && v <= 16 ? v : kBandsPerXcd;
  }();
  TMH_HIP(hipMemsetAsync(queues, 0, 8 * sizeof(int), s));
#define TMH_LAUNCH_CH(L_, S_)                                                                  \
  hipLaunchKernelGGL((k_correct_hist<L_, S_>), dim3(n_wg), dim3(kFThreads), 0, s, in, out, npx, \
                     n_sites, coef2, mconst2, clip_lo, clip_hi, hist, queues, bpx)
  const int spu = fused_spu();
  if (log_transform) {
    if (spu == 1) TMH_LAUNCH_CH(true, 1);
    else if (spu == 2) TMH_LAUNCH_CH(true, 2);
    else TMH_LAUNCH_CH(true, 4);
  } else {
    if (spu == 1) TMH_LAUNCH_CH(false, 1);
    else if (spu == 2) TMH_LAUNCH_CH(false, 2);
    else TMH_LAUNCH_CH(false, 4);
  }
#undef TMH_LAUNCH_CH
  TMH_HIP(hipGetLastError());
}

// coef2 = (f32 mean [*log2(10) when log], f32 mean(std)/std) per pixel: the
// compact form the fused pass keeps L2-resident.  For npx % 8 == 0 (the only
// case the fused pass runs) pixel 8g+j is stored in plane j/2 at float2 index
// (j/2)*2*ngroups + 2g + j%2.  mconst2 = (M' hi, M' lo, zero pixel value, 0)
// with M' = mean(mean) [*log2(10)].
__global__ void k_coeffs2(const double* __restrict__ mean, const double* __restrict__ std,
                          const double* __restrict__ sums, int64_t npx, int log_transform,
                          double zero_log10, float2* __restrict__ coef2,
                          float4* __restrict__ mconst2) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const double K = log_transform ? kLog2_10 : 1.0;
  if (i == 0) {
    const double M = sums[1] / (double)npx * K;
    const float mh = (float)M;
    mconst2[0] = make_float4(mh, (float)(M - (double)mh), (float)(zero_log10 * kLog2_10), 0.f);
  }
  if (i >= npx) return;
  const double S = sums[0] / (double)npx;
  int64_t o = i;
  if ((npx & 7) == 0) {
    const int64_t g = i >> 3, j = i & 7;
    o = (j >> 1) * (npx >> 2) + 2 * g + (j & 1);
  }
  coef2[o] = make_float2((float)(mean[i] * K), (float)(S / std[i]));
}

void launch_coeffs2(const double* mean, const double* std, const double* sums, int64_t npx,
                    int log_transform, double zero_log10, float2* coef2, float4* mconst2,
                    hipStream_t s) {
  hipLaunchKernelGGL(k_coeffs2, dim3((unsigned)cdiv(npx, 256)), dim3(256), 0, s, mean, std, sums,
                     npx, log_transform, zero_log10, coef2, mconst2);
  TMH_HIP(hipGetLastError());
}

}  // namespace tmh
