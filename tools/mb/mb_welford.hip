// Microbenchmark (development tool, not shipped): the Welford pass's read
// pattern.  Each thread owns PX consecutive pixels and walks the sites of its
// part (site-strided reads, as k_welford_vec8); variants change the pixels per
// thread, the number of site parts (parts run one after another in dispatch
// order) and the site depth in flight, against a contiguous grid-stride read
// of the same bytes and the production launch.
// Usage: mb_welford [n_sites=3456] [reps=3] [dist=0 standard|1 bright|2 uniform]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../tmlibrary_amd/csrc/common.h"
#include "../../tmlibrary_amd/csrc/stats_kernels.hip"
#include "../../tmlibrary_amd/csrc/synth_kernels.hip"

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));        \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

namespace tmh {
ProfScope::ProfScope(const char* n, hipStream_t s) : name_(n), s_(s), slot_(nullptr) {}
ProfScope::~ProfScope() {}
}  // namespace tmh
using namespace tmh;
typedef unsigned int u32x4w __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4w ldnt(const uint4* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4w*>(p));
}

// site-strided loads only: thread = V x 16 B (8V px) per site, D sites per stage (2 stages)
template <int V, int D>
__global__ __launch_bounds__(256) void k_wf_loads(const uint16_t* __restrict__ sites, int64_t npx,
                                                  int64_t n_total, int64_t per,
                                                  uint32_t* __restrict__ sink) {
  const int64_t ng = npx >> 3;                   // 16-B groups per site
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t * V >= ng) return;
  const int64_t s0 = (int64_t)blockIdx.y * per;
  const int64_t ns = n_total - s0 < per ? n_total - s0 : per;
  // lane's V groups: strided by the wave's width so each load instruction
  // reads 1 KB contiguous per wave
  const int64_t wbase = (t / 64) * 64 * V + (t % 64);
  const uint4* src = reinterpret_cast<const uint4*>(sites) + s0 * ng + wbase;
  uint32_t acc = 0;
  const int64_t last = ns - 1;
  u32x4w cur[D][V], nxt[D][V];
#pragma unroll
  for (int k = 0; k < D; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) cur[k][v] = ldnt(src + (k < last ? k : last) * ng + v * 64);
  for (int64_t s = 0; s < ns; s += D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int64_t u = s + D + k < last ? s + D + k : last;
#pragma unroll
      for (int v = 0; v < V; ++v) nxt[k][v] = ldnt(src + u * ng + v * 64);
    }
#pragma unroll
    for (int k = 0; k < D; ++k)
#pragma unroll
      for (int v = 0; v < V; ++v) acc ^= cur[k][v].x ^ cur[k][v].y ^ cur[k][v].z ^ cur[k][v].w;
#pragma unroll
    for (int k = 0; k < D; ++k)
#pragma unroll
      for (int v = 0; v < V; ++v) cur[k][v] = nxt[k][v];
  }
  if (acc == 0x9u) sink[0] = acc;
}

// Welford body ablations (one part, no merge): 0 = production math (LDS LUT,
// rare-value series, 3 f64 ops / px), 1 = no LUT ((double)u), 2 = LUT only
// (f64 sum of x), 3 = integer sum of the raw values
template <int MODE>
__global__ __launch_bounds__(256) void k_wf_abl(const uint16_t* __restrict__ sites, int64_t npx,
                                                int64_t n_sites, const double* __restrict__ lut,
                                                double* __restrict__ out) {
  __shared__ double slut[kWfLut], sinv[kWfLut];
  fill_wf_tables<1>(lut, slut, sinv, 256);
  __syncthreads();
  uint32_t wc = 0;
  const int64_t ng = npx >> 3;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= ng) return;
  const uint4* src = reinterpret_cast<const uint4*>(sites) + g;
  const int64_t last = n_sites - 1;
  uint4 cur[4], nxt[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) cur[k] = ld_site<true>(src + (k < last ? k : last) * ng);
  double K[8], s1[8], s2[8];
  uint32_t isum = 0;
  xform8<true, 1>(cur[0], slut, sinv, K, wc, wc);
#pragma unroll
  for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.0;
  for (int64_t s = 0; s < n_sites; s += 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t t = s + 4 + k;
      nxt[k] = ld_site<true>(src + (t < last ? t : last) * ng);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (s + k < n_sites) {
        const uint4 v = cur[k];
        if (MODE == 3) {
          isum += (v.x & 0xFFFF) + (v.x >> 16) + (v.y & 0xFFFF) + (v.y >> 16) + (v.z & 0xFFFF) +
                  (v.z >> 16) + (v.w & 0xFFFF) + (v.w >> 16);
          continue;
        }
        double x[8];
        if (MODE == 1) {
          const uint32_t u[8] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16,
                                 v.z & 0xFFFFu, v.z >> 16, v.w & 0xFFFFu, v.w >> 16};
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = (double)u[j];
        } else {
          xform8<true, 1>(v, slut, sinv, x, wc, wc);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (MODE == 2) {
            s1[j] += x[j];
          } else {
            const double d = x[j] - K[j];
            s1[j] += d;
            s2[j] = fma(d, d, s2[j]);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
  }
  double r = (double)isum;
#pragma unroll
  for (int j = 0; j < 8; ++j) r += s1[j] + s2[j];
  if (r == 1.2345 + wc) out[g] = r;
}

// full Welford math, variants: G sites per pipeline stage, KF (shift K kept in
// f32), WPS launch-bound waves per SIMD
template <int G, bool KF, int WPS>
__global__ __launch_bounds__(256, WPS) void k_wf_var(const uint16_t* __restrict__ sites, int64_t npx,
                                                     int64_t n_sites, const double* __restrict__ lut,
                                                     double* __restrict__ out) {
  __shared__ double slut[kWfLut], sinv[kWfLut];
  fill_wf_tables<1>(lut, slut, sinv, 256);
  __syncthreads();
  uint32_t wc = 0;
  const int64_t ng = npx >> 3;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= ng) return;
  const uint4* src = reinterpret_cast<const uint4*>(sites) + g;
  const int64_t last = n_sites - 1;
  uint4 cur[G], nxt[G];
#pragma unroll
  for (int k = 0; k < G; ++k) cur[k] = ld_site<true>(src + (k < last ? k : last) * ng);
  double K[8], s1[8], s2[8];
  float Kf[8];
  xform8<true, 1>(cur[0], slut, sinv, K, wc, wc);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s1[k] = s2[k] = 0.0;
    Kf[k] = (float)K[k];
  }
  for (int64_t s = 0; s < n_sites; s += G) {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int64_t t = s + G + k;
      nxt[k] = ld_site<true>(src + (t < last ? t : last) * ng);
    }
#pragma unroll
    for (int k = 0; k < G; ++k) {
      if (s + k < n_sites) {
        double x[8];
        xform8<true, 1>(cur[k], slut, sinv, x, wc, wc);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const double d = x[j] - (KF ? (double)Kf[j] : K[j]);
          s1[j] += d;
          s2[j] = fma(d, d, s2[j]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < G; ++k) cur[k] = nxt[k];
  }
  double r = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r += s1[j] + s2[j];
  if (r == 1.2345 + wc) out[g] = r;
}

// f32 packed arithmetic variant: LUT as (hi, lo) f32 pairs, d = (x_hi - K_hi) +
// (x_lo - K_lo) in f32, 16-site f32 block sums folded into f64
typedef float f2_t __attribute__((ext_vector_type(2)));
template <int G, int BLK>
__global__ __launch_bounds__(256) void k_wf_f32(const uint16_t* __restrict__ sites, int64_t npx,
                                                int64_t n_sites, const double* __restrict__ lut,
                                                double* __restrict__ out) {
  __shared__ float2 slut2[kWfLut];
  for (int i = threadIdx.x; i < kWfLut; i += 256) {
    const double x = lut[i];
    const float hi = (float)x;
    slut2[i] = make_float2(hi, (float)(x - (double)hi));
  }
  __syncthreads();
  const int64_t ng = npx >> 3;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= ng) return;
  const uint4* src = reinterpret_cast<const uint4*>(sites) + g;
  const int64_t last = n_sites - 1;
  uint4 cur[G], nxt[G];
#pragma unroll
  for (int k = 0; k < G; ++k) cur[k] = ld_site<true>(src + (k < last ? k : last) * ng);
  f2_t Kh[4], Kl[4];
  {
    const uint4 v = cur[0];
    const uint32_t u[8] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16,
                           v.z & 0xFFFFu, v.z >> 16, v.w & 0xFFFFu, v.w >> 16};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float2 a = slut2[u[2 * p] & 4095u], b = slut2[u[2 * p + 1] & 4095u];
      Kh[p] = (f2_t){a.x, b.x};
      Kl[p] = (f2_t){a.y, b.y};
    }
  }
  double s1[8], s2[8];
  f2_t f1[4], f2[4];
#pragma unroll
  for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.0;
#pragma unroll
  for (int p = 0; p < 4; ++p) f1[p] = f2[p] = (f2_t){0.f, 0.f};
  int blk = 0;
  for (int64_t s = 0; s < n_sites; s += G) {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int64_t t = s + G + k;
      nxt[k] = ld_site<true>(src + (t < last ? t : last) * ng);
    }
#pragma unroll
    for (int k = 0; k < G; ++k) {
      if (s + k < n_sites) {
        const uint4 v = cur[k];
        const uint32_t u[8] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16,
                               v.z & 0xFFFFu, v.z >> 16, v.w & 0xFFFFu, v.w >> 16};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const float2 a = slut2[u[2 * p] & 4095u], b = slut2[u[2 * p + 1] & 4095u];
          const f2_t d = ((f2_t){a.x, b.x} - Kh[p]) + ((f2_t){a.y, b.y} - Kl[p]);
          f1[p] += d;
          f2[p] = __builtin_elementwise_fma(d, d, f2[p]);
        }
      }
    }
    blk += G;
    if (blk >= BLK) {
      blk = 0;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        s1[2 * p] += f1[p].x; s1[2 * p + 1] += f1[p].y;
        s2[2 * p] += f2[p].x; s2[2 * p + 1] += f2[p].y;
        f1[p] = f2[p] = (f2_t){0.f, 0.f};
      }
    }
#pragma unroll
    for (int k = 0; k < G; ++k) cur[k] = nxt[k];
  }
  double r = 0.0;
#pragma unroll
  for (int p = 0; p < 4; ++p) r += f1[p].x + f2[p].y;
#pragma unroll
  for (int j = 0; j < 8; ++j) r += s1[j] + s2[j];
  if (r == 1.2345) out[g] = r;
}

template <int U>
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ p, int64_t n,
                                              uint32_t* __restrict__ sink) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += U * stride) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t j = i + k * stride;
      if (j < n) {
        const u32x4w v = ldnt(p + j);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
  }
  if (acc == 0x9u) sink[0] = acc;
}

static int run(int argc, char** argv) {
  const int64_t S = argc > 1 ? atoll(argv[1]) : 3456;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  const int H = 2160, W = 2560;
  const int64_t npx = (int64_t)H * W, ng = npx / 8;
  const int64_t bytes = S * npx * 2;
  uint16_t* in;
  CK(hipMalloc(&in, bytes));
  const int dist = argc > 3 ? atoi(argv[3]) : 0;
  launch_synth(in, S, H, W, 12345, 0, 0, dist, 0);  // the bench's sites
  CK(hipDeviceSynchronize());
  uint32_t* sink;
  CK(hipMalloc(&sink, 64));
  double *mean, *m2, *lut, *rn, *part;
  CK(hipMalloc(&mean, npx * 8));
  CK(hipMalloc(&m2, npx * 8));
  CK(hipMalloc(&lut, 65536 * 8));
  CK(hipMalloc(&rn, S * 8));
  CK(hipMalloc(&part, 8 * npx * 8));
  {
    std::vector<double> l(65536);
    for (int i = 0; i < 65536; ++i) l[i] = i ? std::log10((double)i) : 0.0;
    CK(hipMemcpy(lut, l.data(), 65536 * 8, hipMemcpyHostToDevice));
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto time = [&](const char* name, auto&& launch) {
    launch();
    CK(hipDeviceSynchronize());
    float tot = 0.f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      tot += ms;
    }
    const double ms = tot / reps;
    printf("%-40s %8.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9,
           100.0 * bytes / (ms * 1e-3) / 8e12);
  };
  time("read contiguous nt u4 grid2048", [&] {
    hipLaunchKernelGGL((k_read<4>), dim3(2048), dim3(256), 0, 0, (const uint4*)in, bytes / 16, sink);
  });
  auto loads = [&](const char* nm, auto vtag, auto dtag, int parts) {
    constexpr int V = decltype(vtag)::value, D = decltype(dtag)::value;
    const int64_t per = (S + parts - 1) / parts;
    const dim3 grid((unsigned)((ng / V + 255) / 256), (unsigned)parts);
    char full[96];
    snprintf(full, sizeof full, "%s V%d D%d parts%d (%u WGs)", nm, V, D, parts, grid.x * grid.y);
    time(full, [&] {
      hipLaunchKernelGGL((k_wf_loads<V, D>), grid, dim3(256), 0, 0, in, npx, S, per, sink);
    });
  };
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  for (int parts : {1, 3, 8, 24})
    loads("loads", I1(), I4(), parts);
  loads("loads", I1(), I8(), 3);
  loads("loads", I1(), I2(), 3);
  loads("loads", I2(), I4(), 3);
  loads("loads", I2(), I2(), 3);
  loads("loads", I4(), I2(), 3);
  loads("loads", I2(), I4(), 8);
  const dim3 ag((unsigned)((ng + 255) / 256));
  time("wf abl 0: production math, 1 part", [&] { hipLaunchKernelGGL((k_wf_abl<0>), ag, dim3(256), 0, 0, in, npx, S, lut, mean); });
  time("wf abl 1: no LUT", [&] { hipLaunchKernelGGL((k_wf_abl<1>), ag, dim3(256), 0, 0, in, npx, S, lut, mean); });
  time("wf abl 2: LUT + f64 sum", [&] { hipLaunchKernelGGL((k_wf_abl<2>), ag, dim3(256), 0, 0, in, npx, S, lut, mean); });
  time("wf abl 3: integer sum", [&] { hipLaunchKernelGGL((k_wf_abl<3>), ag, dim3(256), 0, 0, in, npx, S, lut, mean); });
  auto var = [&](const char* nm, auto gt, auto kt, auto wt) {
    constexpr int G = decltype(gt)::value, WPS = decltype(wt)::value;
    constexpr bool KF = decltype(kt)::value;
    time(nm, [&] { hipLaunchKernelGGL((k_wf_var<G, KF, WPS>), ag, dim3(256), 0, 0, in, npx, S, lut, mean); });
  };
  using B0 = std::integral_constant<bool, false>;
  using B1 = std::integral_constant<bool, true>;
  using W1 = std::integral_constant<int, 1>;
  using W5 = std::integral_constant<int, 5>;
  using W6 = std::integral_constant<int, 6>;
  var("wf var G4 K64", I4(), B0(), W1());
  var("wf var G4 Kf32", I4(), B1(), W1());
  var("wf var G2 K64", I2(), B0(), W1());
  var("wf var G2 Kf32", I2(), B1(), W1());
  var("wf var G2 Kf32 wps5", I2(), B1(), W5());
  var("wf var G2 Kf32 wps6", I2(), B1(), W6());
  var("wf var G4 Kf32 wps5", I4(), B1(), W5());
  var("wf var G1 Kf32 wps6", I1(), B1(), W6());
  static const char* shapes[9] = {"256 thr, Newton rcp", "256 thr, LDS rcp", "512 thr, Newton rcp",
                                  "512 thr, LDS rcp", "256 thr, f32 small term", "512 thr, f32 small term"};
  for (int shape = 0; shape < 9; ++shape)
    for (int f : {1, 3}) {
      char nm[80];
      snprintf(nm, sizeof nm, "welford shape %d (%s) parts %d", shape, shapes[shape], f);
      time(nm, [&] {
        launch_welford(in, npx, S, 0, rn, mean, m2, lut, 1, part, 8 * npx, f, nullptr, 0, 0, shape);
      });
    }
  time("wf f32 G2 blk16", [&] { hipLaunchKernelGGL((k_wf_f32<2, 16>), ag, dim3(256), 0, 0, in, npx, S, lut, mean); });
  time("wf f32 G2 blk32", [&] { hipLaunchKernelGGL((k_wf_f32<2, 32>), ag, dim3(256), 0, 0, in, npx, S, lut, mean); });
  time("wf f32 G4 blk16", [&] { hipLaunchKernelGGL((k_wf_f32<4, 16>), ag, dim3(256), 0, 0, in, npx, S, lut, mean); });
  unsigned int* probe;
  CK(hipMalloc(&probe, 4));
  for (int r = 0; r < 2; ++r) {
    time("welford production (parts 1)", [&] {
      launch_welford(in, npx, S, 0, rn, mean, m2, lut, 1, part, 8 * npx, 1, nullptr, 0, 0);
    });
    time("welford bright form (16,384-entry LUT, 3 parts)", [&] {
      launch_welford(in, npx, S, 0, rn, mean, m2, lut, 1, part, 8 * npx, 0, nullptr, 1, 0);
    });
  }
  return 0;
}

// a library check or HIP call that fails throws tmh::Error: print its message
// (which names the failing call) instead of dying in std::terminate
int main(int argc, char** argv) {
  try {
    return run(argc, argv);
  } catch (const tmh::Error& e) {
    fprintf(stderr, "tmh::Error %d: %s\n", e.code, e.msg.c_str());
    return 1;
  }
}
