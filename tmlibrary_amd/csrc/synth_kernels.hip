// Synthetic site images in HBM (SURVEY.md §8(d) distribution), integer-exact.
//
// The bench's 3,456-site input is generated on the device, and its results
// have to be checked against the CPU oracle on the SAME pixels.  So the
// generator uses no device transcendental at all: every pixel is a counter
// hash (splitmix64) of (seed, channel, site, pixel) mapped through integer
// tables that the host builds with IEEE +-*/, exp and log only (glibc, the
// same calls numpy/CPython make), and integer arithmetic on the device.
// tmlibrary_amd/synth.py restates it in numpy bit for bit (synth_exact_host);
// tmh_synth_tables exports the tables so a CPU test pins the two builds.
//
// Per pixel p of site s (all uint64, wrapping):
//   z1 = splitmix64(key ^ splitmix64(s) ^ p),  z2 = splitmix64(z1)
//   LOGNORMAL(mu):  ill  = ey[y] * ex[x]                      (vignetting, 2^30 = 1)
//                   v16  = 1600 + (ill * LN16[z1 >> 52] >> 30) + NZ16[(z1 >> 40) & 4095]
//                   v    = clamp((v16 + 8) >> 4, 0, 65535)      (1/16-DN fixed point)
//                   z2 >> 40 < 1678 -> 0;  >= 2^24 - 1678 -> 65535  (0.01 % each)
//   UNIFORM:        v = z2 >> 48
// LN16[i] = round(16 exp(mu + 0.6 z_i)), NZ16[i] = round(80 z_i), z_i the
// standard-normal quantile at (i + 0.5) / 4096 (Acklam's rational form), i.e.
// v ~ 100 + illum * LogNormal(mu, 0.6) + N(0, 5) as in SURVEY.md §8(d).
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "common.h"

namespace tmh {

namespace {

constexpr int kSynthTab = 4096;

double acklam_ndtri(double p) {
#pragma clang fp contract(off)
  static const double a[6] = {-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
                              1.383577518672690e+02,  -3.066479806614716e+01, 2.506628277459239e+00};
  static const double b[5] = {-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
                              6.680131188771972e+01,  -1.328068155288572e+01};
  static const double c[6] = {-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
                              -2.549732539343734e+00, 4.374664141464968e+00,  2.938163982698783e+00};
  static const double d[4] = {7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
                              3.754408661907416e+00};
  const double plow = 0.02425;
  if (p < plow) {
    const double q = std::sqrt(-2.0 * std::log(p));
    const double num = ((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5];
    const double den = (((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1.0;
    return num / den;
  }
  if (p > 1.0 - plow) {
    const double q = std::sqrt(-2.0 * std::log(1.0 - p));
    const double num = ((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5];
    const double den = (((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1.0;
    return -(num / den);
  }
  const double q = p - 0.5;
  const double r = q * q;
  const double num = (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q;
  const double den = ((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1.0;
  return num / den;
}

double dist_mu(int dist) { return dist == TMH_SYNTH_BRIGHT ? 8.5 : 6.0; }

void build_tables(int dist, int H, int W, int32_t* ln, int32_t* nz, int32_t* ey, int32_t* ex) {
#pragma clang fp contract(off)
  const double mu = dist_mu(dist);
  for (int i = 0; i < kSynthTab; ++i) {
    const double z = acklam_ndtri(((double)i + 0.5) / (double)kSynthTab);
    const double e = std::exp(mu + 0.6 * z);
    ln[i] = (int32_t)std::floor(16.0 * e + 0.5);
    nz[i] = (int32_t)std::floor(80.0 * z + 0.5);
  }
  auto axis = [](int n, int32_t* t) {
#pragma clang fp contract(off)
    const double c = ((double)n - 1.0) / 2.0;
    const double h = std::fmax((double)n / 2.0, 1.0);
    for (int i = 0; i < n; ++i) {
      const double f = ((double)i - c) / h;
      t[i] = (int32_t)std::floor(32768.0 * std::exp(-0.75 * (f * f)) + 0.5);
    }
  };
  axis(H, ey);
  axis(W, ex);
}

struct SynthDev {
  int32_t* p = nullptr;  // [ln 4096 | nz 4096 | ey H | ex W]
};
std::mutex g_synth_mu;
std::map<std::tuple<int, int, int, int>, SynthDev> g_synth;

const int32_t* synth_tables_dev(int dist, int H, int W) {
  int dev = 0;
  TMH_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_synth_mu);
  const auto key = std::make_tuple(dev, dist, H, W);
  auto it = g_synth.find(key);
  if (it != g_synth.end()) return it->second.p;
  std::vector<int32_t> t((size_t)2 * kSynthTab + H + W);
  build_tables(dist, H, W, t.data(), t.data() + kSynthTab, t.data() + 2 * kSynthTab,
               t.data() + 2 * kSynthTab + H);
  SynthDev d;
  TMH_HIP(hipMalloc(&d.p, t.size() * 4));
  TMH_HIP(hipMemcpy(d.p, t.data(), t.size() * 4, hipMemcpyHostToDevice));
  g_synth[key] = d;
  return d.p;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint32_t synth_px(uint64_t base, uint64_t p, int y, int x, int dist,
                                             const int32_t* __restrict__ tab, int H) {
  const uint64_t z1 = splitmix64(base ^ p);
  const uint64_t z2 = splitmix64(z1);
  if (dist == TMH_SYNTH_UNIFORM) return (uint32_t)(z2 >> 48);
  const int32_t* ln = tab;
  const int32_t* nz = tab + kSynthTab;
  const int32_t* ey = tab + 2 * kSynthTab;
  const int32_t* ex = ey + H;
  const uint64_t ill = (uint64_t)ey[y] * (uint64_t)ex[x];
  const int64_t prod = (int64_t)((ill * (uint64_t)ln[z1 >> 52]) >> 30);
  const int64_t v16 = 1600 + prod + nz[(z1 >> 40) & 4095u];
  int64_t v = (v16 + 8) >> 4;
  v = v < 0 ? 0 : (v > 65535 ? 65535 : v);
  const uint32_t u3 = (uint32_t)(z2 >> 40);
  if (u3 < 1678u) v = 0;
  if (u3 >= 16777216u - 1678u) v = 65535;
  return (uint32_t)v;
}

// thread = 8 consecutive pixels of one site (one 16-B store when npx % 8 == 0)
__global__ __launch_bounds__(256) void k_synth(uint16_t* __restrict__ out, int H, int W,
                                               uint64_t key, int64_t first_site, int dist,
                                               const int32_t* __restrict__ tab, int vec) {
  const int64_t npx = (int64_t)H * W;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t s = blockIdx.y;
  const int64_t p0 = g * 8;
  if (p0 >= npx) return;
  const uint64_t base = key ^ splitmix64((uint64_t)(first_site + s));
  uint16_t* o = out + s * npx;
  int y = (int)(p0 / W), x = (int)(p0 % W);
  uint32_t v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] = (p0 + k < npx) ? synth_px(base, (uint64_t)(p0 + k), y, x, dist, tab, H) : 0u;
    if (++x == W) {
      x = 0;
      ++y;
    }
  }
  if (vec) {
    *reinterpret_cast<uint4*>(o + p0) =
        make_uint4(v[0] | v[1] << 16, v[2] | v[3] << 16, v[4] | v[5] << 16, v[6] | v[7] << 16);
  } else {
    for (int k = 0; k < 8 && p0 + k < npx; ++k) o[p0 + k] = (uint16_t)v[k];
  }
}

// Box probe (bench support): the box's own stream rate for a pass's bytes,
// so a bench line can tell a slow box from a slow kernel.  WRITE: every
// site's 16-byte groups read and written to its output block (the fused
// pass's 2 + 2 B/px); else read only (the Welford pass's 2 B/px).
// Non-temporal loads and stores, as the passes move them.  Two shapes:
//   k_box_probe       persistent, grid-strided over each block of sites in
//                     turn, four groups in flight per thread;
//   k_box_probe_flat  one group per thread, one launch per block (a
//                     workgroup streams 4 KB and leaves).
// Workgroup 0's first thread stamps the shader clock (clock64) and the
// constant 100 MHz clock (wall_clock64) at its start and end: clk[0..3].
typedef unsigned int probe_u32x4 __attribute__((ext_vector_type(4)));

template <bool WRITE>
__global__ __launch_bounds__(256) void k_box_probe(const uint16_t* const* __restrict__ in_blocks,
                                                   uint16_t* const* __restrict__ out_blocks,
                                                   int shift, int64_t n_sites, int64_t npx,
                                                   unsigned long long* __restrict__ clk,
                                                   unsigned int* __restrict__ sink) {
  typedef probe_u32x4 u32x4;
  const bool stamp = blockIdx.x == 0 && threadIdx.x == 0;
  if (stamp) {
    clk[0] = clock64();
    clk[1] = wall_clock64();
  }
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t per_block = (int64_t)1 << shift;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (int64_t b = 0; b * per_block < n_sites; ++b) {
    const int64_t ns = n_sites - b * per_block < per_block ? n_sites - b * per_block : per_block;
    const int64_t n = ns * (npx >> 3);  // 16-byte groups of the block
    const u32x4* src = reinterpret_cast<const u32x4*>(in_blocks[b]);
    u32x4* dst = WRITE ? reinterpret_cast<u32x4*>(out_blocks[b]) : nullptr;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
      u32x4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(src + i + k * stride);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (WRITE)
          __builtin_nontemporal_store(v[k], dst + i + k * stride);
        else
          acc ^= v[k];
      }
    }
    for (; i < n; i += stride) {
      const u32x4 v = __builtin_nontemporal_load(src + i);
      if (WRITE)
        __builtin_nontemporal_store(v, dst + i);
      else
        acc ^= v;
    }
  }
  if (!WRITE && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[0] = acc.x;  // keeps the loads
  if (stamp) {
    clk[2] = clock64();
    clk[3] = wall_clock64();
  }
}

template <bool WRITE>
__global__ __launch_bounds__(256) void k_box_probe_flat(const uint16_t* __restrict__ in,
                                                        uint16_t* __restrict__ out, int64_t n,
                                                        unsigned int* __restrict__ sink) {
  typedef probe_u32x4 u32x4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in) + i);
  if (WRITE)
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out) + i);
  else if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u)
    sink[0] = v.x;
}

}  // namespace

void launch_box_probe(const uint16_t* const* in_blocks, uint16_t* const* out_blocks, int shift,
                      int64_t n_sites, int64_t npx, int write, unsigned long long* clk,
                      unsigned int* sink, int n_cus, hipStream_t s) {
  const dim3 grid((unsigned)(n_cus * 8));  // 2,048 threads per CU, 4 loads each in flight
  if (write)
    hipLaunchKernelGGL(k_box_probe<true>, grid, dim3(256), 0, s, in_blocks, out_blocks, shift,
                       n_sites, npx, clk, sink);
  else
    hipLaunchKernelGGL(k_box_probe<false>, grid, dim3(256), 0, s, in_blocks, out_blocks, shift,
                       n_sites, npx, clk, sink);
  TMH_HIP(hipGetLastError());
}

void launch_box_probe_flat(const uint16_t* in, uint16_t* out, int64_t n_sites, int64_t npx,
                           int write, unsigned int* sink, hipStream_t s) {
  const int64_t n = n_sites * (npx >> 3);
  if (n <= 0) return;
  const dim3 grid((unsigned)cdiv(n, 256));
  if (write)
    hipLaunchKernelGGL(k_box_probe_flat<true>, grid, dim3(256), 0, s, in, out, n, sink);
  else
    hipLaunchKernelGGL(k_box_probe_flat<false>, grid, dim3(256), 0, s, in, out, n, sink);
  TMH_HIP(hipGetLastError());
}

void synth_tables_host(int dist, int H, int W, int32_t* ln, int32_t* nz, int32_t* ey, int32_t* ex) {
  build_tables(dist, H, W, ln, nz, ey, ex);
}

void launch_synth(uint16_t* out, int64_t n_sites, int H, int W, uint64_t seed, int channel,
                  int64_t first_site, int dist, hipStream_t s) {
  const int64_t npx = (int64_t)H * W;
  const int32_t* tab = synth_tables_dev(dist, H, W);
  const uint64_t key = seed * 0x100000001B3ull ^ ((uint64_t)channel << 56);
  const int vec = (npx & 7) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  for (int64_t s0 = 0; s0 < n_sites; s0 += 65535) {
    const int64_t ns = (n_sites - s0 < 65535) ? n_sites - s0 : 65535;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)cdiv(cdiv(npx, 8), 256), (unsigned)ns), dim3(256),
                       0, s, out + s0 * npx, H, W, key, first_site + s0, dist, tab, vec);
  }
  TMH_HIP(hipGetLastError());
}

}  // namespace tmh
