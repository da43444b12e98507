// Microbenchmark (development tool, not shipped): does the fused pass's work
// shape -- persistent workgroups, each streaming SPU whole-band site streams
// -- cost the ~1 ms it trails a one-element-per-thread copy of the same bytes?
// Copies S sites (u16 in -> out, plus the L2-resident coefficient loads of the
// fused pass) with teams of T workgroups sharing each (band, site group) unit:
// member m of a team takes the unit's 16-B groups m*NT + tid + i*T*NT, so the
// chip has n_teams*SPU concurrent site streams instead of G*SPU.  ORDER 0 =
// units band-major (as production), 1 = site-major.
// Usage: mb_shape [n_sites=3456] [reps=3] [dist=0 standard|1 bright] [quick=0]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../tmlibrary_amd/csrc/common.h"
#include "../../tmlibrary_amd/csrc/fused_kernels.hip"
#include "../../tmlibrary_amd/csrc/synth_kernels.hip"

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));        \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

namespace tmh {  // no per-kernel event timing in this tool
ProfScope::ProfScope(const char* n, hipStream_t s) : name_(n), s_(s), slot_(nullptr) {}
ProfScope::~ProfScope() {}
}  // namespace tmh

using namespace tmh;
typedef unsigned int u32x4m __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy1(const u32x4m* __restrict__ a, u32x4m* __restrict__ c,
                                               int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) c[i] = a[i];
}

template <int SPU, int NT, int ORDER, bool COEF>
__global__ __launch_bounds__(NT) void k_team(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                             int64_t npx, int64_t n_sites, const float4* __restrict__ coef,
                                             int T, int n_bands) {
  const int n_teams = (int)gridDim.x / T;
  const int team = (int)blockIdx.x % n_teams, mem = (int)blockIdx.x / n_teams;
  const int ngroups = (int)(npx >> 3);
  const int site_bytes = (int)(npx * 2);
  const int n_sg = (int)((n_sites + SPU - 1) / SPU);
  const int n_units = n_sg * n_bands;
  const __amdgpu_buffer_rsrc_t rcf =
      __builtin_amdgcn_make_buffer_rsrc((void*)coef, 0, (int)(npx * 8), 0x00020000);
  const int step = T * NT;
  for (int u = team; u < n_units; u += n_teams) {
    const int band = ORDER == 0 ? u / n_sg : u % n_bands;
    const int sg = ORDER == 0 ? u % n_sg : u / n_bands;
    const int64_t s0 = (int64_t)sg * SPU;
    const int ns = (int)(n_sites - s0 < SPU ? n_sites - s0 : SPU);
    const int g0 = (int)((int64_t)band * ngroups / n_bands);
    const int g1 = (int)((int64_t)(band + 1) * ngroups / n_bands);
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void*)(in + s0 * npx), 0, ns * site_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rout =
        __builtin_amdgcn_make_buffer_rsrc((void*)(out + s0 * npx), 0, ns * site_bytes, 0x00020000);
    auto load = [&](int g, u32x4m (&v)[SPU], u32x4m& c) {
#pragma unroll
      for (int k = 0; k < SPU; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rin, g * 16, k * site_bytes, 2);
      c = u32x4m{0, 0, 0, 0};
      if (COEF) {
#pragma unroll
        for (int p = 0; p < 4; ++p) c ^= __builtin_amdgcn_raw_buffer_load_b128(rcf, g * 16, p * ngroups * 16, 0);
      }
    };
    int g = g0 + mem * NT + (int)threadIdx.x;
    u32x4m v[SPU], c;
    if (g < g1) load(g, v, c);
    while (g < g1) {
      const int gn = g + step;
      u32x4m vn[SPU], cn;
      if (gn < g1) load(gn, vn, cn);
#pragma unroll
      for (int k = 0; k < SPU; ++k)
        if (k < ns) __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ (c & 1u), rout, g * 16, k * site_bytes, 2);
#pragma unroll
      for (int k = 0; k < SPU; ++k) v[k] = vn[k];
      c = cn;
      g = gn;
    }
  }
}

static int run(int argc, char** argv) {
  const int64_t S = argc > 1 ? atoll(argv[1]) : 3456;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  const int H = 2160, W = 2560;
  const int64_t npx = (int64_t)H * W;
  const int64_t bytes = S * npx * 2;
  uint16_t *in, *out;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, bytes));
  const int dist = argc > 3 ? atoi(argv[3]) : 0;
  const int quick = argc > 4 ? atoi(argv[4]) : 0;  // 1: configuration x band sweep + bright breakdown
  launch_synth(in, S, H, W, 12345, 0, 0, dist, 0);
  CK(hipDeviceSynchronize());
  float4 *coef, *mconst2;
  uint32_t* hist;
  unsigned long long *rmask, *fe;
  unsigned int* fn;
  CK(hipMalloc(&coef, npx * 8));
  CK(hipMalloc(&mconst2, 16));
  CK(hipMalloc(&hist, (size_t)S * 65536 * 4));
  CK(hipMalloc(&rmask, S * 8));
  CK(hipMalloc(&fe, (size_t)1 << 23));
  CK(hipMalloc(&fn, 4));
  {
    std::vector<float> c(npx * 2);
    for (int64_t i = 0; i < npx * 2; ++i) c[i] = (i & 2) ? 1.02f : 8.3f;
    CK(hipMemcpy(coef, c.data(), npx * 8, hipMemcpyHostToDevice));
    const float m[4] = {8.2f, 0.0f, 1e-10f, 3.0e38f};
    CK(hipMemcpy(mconst2, m, 16, hipMemcpyHostToDevice));
  }
  CK(hipMemset(hist, 0, (size_t)S * 65536 * 4));
  CK(hipMemset(rmask, 0, S * 8));
  unsigned long long* wide;
  CK(hipMalloc(&wide, 16));
  CK(hipMemset(wide, 0, 16));
  int* queues;  // per-XCD unit counters + round-mask union (zeroed before every launch)
  CK(hipMalloc(&queues, kFusedQueueInts * sizeof(int)));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const FixList fl{fe, fn, (unsigned)(((size_t)1 << 23) / 8)};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double cb = 2.0 * bytes;
  auto time = [&](const char* name, auto&& launch) {
    launch();
    CK(hipDeviceSynchronize());
    float tot = 0.f, best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      tot += ms;
      best = ms < best ? ms : best;
    }
    printf("%-44s %8.3f ms (best %8.3f) %7.1f GB/s %5.1f%%\n", name, tot / reps, best,
           cb / (tot / reps * 1e-3) / 1e9, 100.0 * cb / (tot / reps * 1e-3) / 8e12);
    fflush(stdout);
  };
  const int64_t n16 = bytes / 16;
  time("copy1 (one per thread)", [&] {
    hipLaunchKernelGGL(k_copy1, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, 0, (const u32x4m*)in,
                       (u32x4m*)out, n16);
  });
  int nb = kFusedBands;
  auto fused = [&](auto abl_tag) {
    constexpr int ABL = decltype(abl_tag)::value;
    CK(hipMemsetAsync(fn, 0, 4, 0));
    CK(hipMemsetAsync(queues, 0, kFusedQueueInts * sizeof(int), 0));
    hipLaunchKernelGGL((k_correct_hist<true, false, 4, ABL, 512, 16384>), dim3(cus * 2), dim3(512), 0, 0,
                       in, out, npx, S, coef, mconst2, fl, -1, -1, hist, rmask, nb, queues,
                       nullptr, 0ull, 0ull, 0ull, 0ull, SiteTab{}, InPassFin{});
  };
  char nm[96];
  for (int b : {16, 8, 12, 24, 32, 64}) {
    nb = b;
    snprintf(nm, sizeof nm, "fused prod (ABL 0) bands %d", b);
    time(nm, [&] { fused(std::integral_constant<int, 0>()); });
  }
  nb = kFusedBands;
  auto fcfg = [&](const char* nm2, auto spu_t, auto nt_t, auto lb_t, int grid) {
    constexpr int SPU_ = decltype(spu_t)::value, NT_ = decltype(nt_t)::value, LB_ = decltype(lb_t)::value;
    time(nm2, [&] {
      CK(hipMemsetAsync(fn, 0, 4, 0));
      CK(hipMemsetAsync(queues, 0, kFusedQueueInts * sizeof(int), 0));
      hipLaunchKernelGGL((k_correct_hist<true, false, SPU_, 0, NT_, LB_>), dim3(grid), dim3(NT_), 0, 0,
                         in, out, npx, S, coef, mconst2, fl, -1, -1, hist, rmask, nb, queues, nullptr, 0ull, 0ull, 0ull, 0ull, SiteTab{}, InPassFin{});
    });
  };
  using C8 = std::integral_constant<int, 8>;
  using C4 = std::integral_constant<int, 4>;
  using T256 = std::integral_constant<int, 256>;
  using T512 = std::integral_constant<int, 512>;
  using T1024 = std::integral_constant<int, 1024>;
  using L8k = std::integral_constant<int, 8192>;
  using L16k = std::integral_constant<int, 16384>;
  using L32k = std::integral_constant<int, 32768>;
  using C2 = std::integral_constant<int, 2>;
  for (int b : {16, 8, 4, 2}) {
    nb = b;
    snprintf(nm, sizeof nm, "cfg (2,1024,32768) [wide] bands %d", b);
    fcfg(nm, C2(), T1024(), L32k(), cus);
    snprintf(nm, sizeof nm, "cfg (4,512,16384) [narrow] bands %d", b);
    fcfg(nm, C4(), T512(), L16k(), 2 * cus);
  }
  nb = kFusedBands;
  if (quick == 2 || quick) {
    // where the wide configuration's time goes (bright data): the same launch
    // without histogram (ABL 1), without the per-unit flush (ABL 8), and the
    // four-site shape without histogram
    auto fabl = [&](const char* nm2, auto spu_t, auto nt_t, auto lb_t, auto abl_t, int grid, int bands) {
      constexpr int SPU_ = decltype(spu_t)::value, NT_ = decltype(nt_t)::value,
                    LB_ = decltype(lb_t)::value, ABL_ = decltype(abl_t)::value;
      time(nm2, [&] {
        CK(hipMemsetAsync(fn, 0, 4, 0));
        CK(hipMemsetAsync(queues, 0, kFusedQueueInts * sizeof(int), 0));
        hipLaunchKernelGGL((k_correct_hist<true, false, SPU_, ABL_, NT_, LB_>), dim3(grid), dim3(NT_), 0, 0,
                           in, out, npx, S, coef, mconst2, fl, -1, -1, hist, rmask, bands, queues, nullptr,
                           0ull, 0ull, 0ull, 0ull, SiteTab{}, InPassFin{});
      });
    };
    using A0 = std::integral_constant<int, 0>;
    using A1 = std::integral_constant<int, 1>;
    using A8 = std::integral_constant<int, 8>;
    fabl("wide (2,1024,32768) b8 ABL0", C2(), T1024(), L32k(), A0(), cus, 8);
    fabl("wide (2,1024,32768) b8 ABL1 no hist", C2(), T1024(), L32k(), A1(), cus, 8);
    fabl("wide (2,1024,32768) b8 ABL8 no flush", C2(), T1024(), L32k(), A8(), cus, 8);
    fabl("four (4,1024,32768) b16 ABL1 no hist", C4(), T1024(), L32k(), A1(), cus, 16);
    fabl("four (4,1024,32768) b8 ABL1 no hist", C4(), T1024(), L32k(), A1(), cus, 8);
    fabl("narrow (4,512,16384) b16 ABL1 no hist", C4(), T512(), L16k(), A1(), 2 * cus, 16);
    printf("done\n");
    return 0;
  }
  fcfg("cfg (8,512,32768) grid cus", C8(), T512(), L32k(), cus);
  fcfg("cfg (8,1024,32768) grid cus", C8(), T1024(), L32k(), cus);
  fcfg("cfg (4,512,16384) grid 2cus [prod]", C4(), T512(), L16k(), 2 * cus);
  fcfg("cfg (4,256,16384) grid 2cus", C4(), T256(), L16k(), 2 * cus);
  fcfg("cfg (4,256,8192) grid 4cus [2048 bins]", C4(), T256(), L8k(), 4 * cus);
  fcfg("cfg (8,1024,32768) grid cus again", C8(), T1024(), L32k(), cus);
  time("fused no hist (ABL 1)", [&] { fused(std::integral_constant<int, 1>()); });
  time("fused no hist, const coef (ABL 3)", [&] { fused(std::integral_constant<int, 3>()); });
  time("fused no flush (ABL 8)", [&] { fused(std::integral_constant<int, 8>()); });
  time("fused no arith (ABL 32)", [&] { fused(std::integral_constant<int, 32>()); });
  time("fused no arith no hist (ABL 33)", [&] { fused(std::integral_constant<int, 33>()); });
  time("fused auto (narrow runs, wide exits)", [&] {
    CK(hipMemsetAsync(fn, 0, 4, 0));
    launch_correct_hist(in, out, npx, S, (const float2*)coef, mconst2, fl, 1, -1, -1, hist, rmask,
                        queues, cus, kFusedNarrow, 0);
  });
  for (int cfg = 0; cfg < kFusedConfigs; ++cfg) {
    snprintf(nm, sizeof nm, "fused cfg %d (%d,%d,%d)", cfg, kFusedCfgs[cfg].spu,
             kFusedCfgs[cfg].threads, kFusedCfgs[cfg].lds_bins);
    time(nm, [&] {
      CK(hipMemsetAsync(fn, 0, 4, 0));
      launch_correct_hist(in, out, npx, S, (const float2*)coef, mconst2, fl, 1, -1, -1, hist, rmask,
                          queues, cus, cfg, 0);
    });
  }
#define TEAM(SPU_, NT_, ORD_, COEF_, G_, T_, NB_)                                                   \
  snprintf(nm, sizeof nm, "team spu%d nt%d ord%d coef%d G%d T%d bands%d", SPU_, NT_, ORD_, (int)COEF_, \
           G_, T_, NB_);                                                                           \
  time(nm, [&] {                                                                                   \
    hipLaunchKernelGGL((k_team<SPU_, NT_, ORD_, COEF_>), dim3(G_), dim3(NT_), 0, 0, in, out, npx, S, \
                       coef, T_, NB_);                                                             \
  });
  const int G2 = cus * 2;
  TEAM(4, 512, 0, true, G2, 1, 16)
  TEAM(4, 512, 0, false, G2, 1, 16)
  TEAM(4, 512, 1, true, G2, 1, 16)
  TEAM(4, 512, 0, true, G2, 16, 16)
  time("fused prod (ABL 0) again", [&] { fused(std::integral_constant<int, 0>()); });
  time("copy1 again", [&] {
    hipLaunchKernelGGL(k_copy1, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, 0, (const u32x4m*)in,
                       (u32x4m*)out, n16);
  });
  printf("done\n");
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
