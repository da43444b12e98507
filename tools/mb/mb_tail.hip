// Microbenchmark (development tool, not shipped): the percentile tail of the
// fused job -- histogram finalize (order statistics from the per-site
// histograms) and the ordered percentile sum -- with ablations, against the
// pure store / load streams of the same order-statistic bytes.
// Histograms come from one production fused pass over the bench's generator.
// Usage: mb_tail [n_sites=3456] [reps=5] [dist=0 standard|1 bright|2 uniform]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../tmlibrary_amd/csrc/common.h"
#include "../../tmlibrary_amd/csrc/fused_kernels.hip"
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

// pure 16-B store stream over the order-statistic buffer
__global__ __launch_bounds__(256) void k_store(uint4* __restrict__ p, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
    p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

// pure 16-B load stream (sink)
__global__ __launch_bounds__(256) void k_load(const uint4* __restrict__ p, int64_t n16,
                                              uint32_t* __restrict__ sink) {
  uint32_t a = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
    const uint4 v = p[i];
    a ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (a == 0x12345u) sink[0] = a;
}

// k_pct_acc with a deeper site pipeline (U sites in flight per thread)
template <int U>
__global__ __launch_bounds__(256) void k_pct_acc_u(const uint32_t* __restrict__ vlh, int64_t n_sites,
                                                   int64_t tstride, int Q,
                                                   const double* __restrict__ gamma,
                                                   double* __restrict__ acc) {
  const int q = (int)blockIdx.x * 256 + threadIdx.x;
  if (q >= Q) return;
  const double g = gamma[q];
  double a = acc[q];
  const uint32_t* p = vlh + (int64_t)(q / kOsTile) * tstride + (q % kOsTile);
  const int64_t last = n_sites - 1;
  uint32_t v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) v[k] = p[(k < last ? k : last) * kOsTile];
  for (int64_t s = 0; s < n_sites; s += U) {
    uint32_t vn[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t u = s + U + k < last ? s + U + k : last;
      vn[k] = p[u * kOsTile];
    }
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (s + k < n_sites) a = add_nc(a, lerp_np(v[k] & 0xFFFFu, v[k] >> 16, g));
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = vn[k];
  }
  acc[q] = a;
}

static int run(int argc, char** argv) {
  const int64_t S = argc > 1 ? atoll(argv[1]) : 3456;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int dist = argc > 3 ? atoi(argv[3]) : 0;
  const int H = 2160, W = 2560;
  const int64_t npx = (int64_t)H * W;
  const int Q = 100000;
  uint16_t *in, *out;
  CK(hipMalloc(&in, S * npx * 2));
  CK(hipMalloc(&out, S * npx * 2));
  launch_synth(in, S, H, W, 12345, 0, 0, dist, 0);
  float4 *coef, *mconst2;
  uint32_t* hist;
  unsigned long long *rmask, *fe, *pooled, *parts;
  unsigned int* fn;
  uint32_t* sink;
  CK(hipMalloc(&coef, npx * 8));
  CK(hipMalloc(&mconst2, 16));
  CK(hipMalloc(&hist, (size_t)S * kBins * 4));
  CK(hipMalloc(&rmask, S * 8));
  CK(hipMalloc(&fe, (size_t)1 << 23));
  CK(hipMalloc(&fn, 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&pooled, kBins * 8));
  CK(hipMalloc(&parts, 16 * kBins * 8));
  CK(hipMemset(parts, 0, 16 * kBins * 8));
  {
    std::vector<float> c(npx * 2);
    for (int64_t i = 0; i < npx * 2; ++i) c[i] = (i & 2) ? 1.02f : 8.3f;
    CK(hipMemcpy(coef, c.data(), npx * 8, hipMemcpyHostToDevice));
    const float m[4] = {8.2f, 0.0f, 1e-10f, 3.0e38f};
    CK(hipMemcpy(mconst2, m, 16, hipMemcpyHostToDevice));
  }
  CK(hipMemset(hist, 0, (size_t)S * kBins * 4));
  CK(hipMemset(rmask, 0, S * 8));
  CK(hipMemset(fn, 0, 4));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const FixList fl{fe, fn, (unsigned)(((size_t)1 << 23) / 8)};
  int* queues;  // per-XCD unit counters + round-mask union
  CK(hipMalloc(&queues, kFusedQueueInts * sizeof(int)));
  launch_correct_hist(in, out, npx, S, (const float2*)coef, mconst2, fl, 1, -1, -1, hist, rmask,
                      queues, cus, dist == 0 ? kFusedNarrow : kFusedWide, 0, 0);
  CK(hipDeviceSynchronize());
  {
    std::vector<unsigned long long> rm(S);
    CK(hipMemcpy(rm.data(), rmask, S * 8, hipMemcpyDeviceToHost));
    double tot = 0;
    for (auto r : rm) tot += __builtin_popcountll(r);
    printf("sites %ld, rounds per site %.2f\n", (long)S, tot / S);
  }
  // quantile tables (timing only: not numpy's exact rounding)
  std::vector<int32_t> lo(Q), hi(Q);
  std::vector<double> gm(Q);
  for (int i = 0; i < Q; ++i) {
    const double vi = (double)(npx - 1) * ((100.0 * i / (Q - 1)) / 100.0);
    lo[i] = (int32_t)vi;
    hi[i] = std::min<int64_t>(lo[i] + 1, npx - 1);
    gm[i] = vi - lo[i];
  }
  int32_t *qlo, *qhi;
  double *gamma, *acc;
  CK(hipMalloc(&qlo, Q * 4));
  CK(hipMalloc(&qhi, Q * 4));
  CK(hipMalloc(&gamma, Q * 8));
  CK(hipMalloc(&acc, Q * 8));
  CK(hipMemcpy(qlo, lo.data(), Q * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(qhi, hi.data(), Q * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(gamma, gm.data(), Q * 8, hipMemcpyHostToDevice));
  CK(hipMemset(acc, 0, Q * 8));
  const int64_t tiles = os_tiles(Q);
  uint32_t* vlh;
  const size_t os_bytes = (size_t)S * tiles * kOsTile * 4;
  CK(hipMalloc(&vlh, os_bytes));
  int64_t* zeros;
  CK(hipMalloc(&zeros, S * 8));
  QPos qp{qlo, qhi, Q, (double)(Q - 1) / (npx - 1), (int32_t)(npx - 1), 1, S * kOsTile};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto time = [&](const char* name, double bytes, auto&& launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, tot = 0.f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
      tot += ms;
    }
    printf("%-40s %8.3f ms (best %7.3f)", name, tot / reps, best);
    if (bytes > 0) printf("  %7.1f GB/s", bytes / (tot / reps * 1e-3) / 1e9);
    printf("\n");
  };
  const double osb = (double)S * Q * 4;
  time("store stream (order-stat bytes)", osb, [&] {
    hipLaunchKernelGGL(k_store, dim3(4096), dim3(256), 0, 0, (uint4*)vlh, (int64_t)(os_bytes / 16));
  });
  time("load stream (order-stat bytes)", osb, [&] {
    hipLaunchKernelGGL(k_load, dim3(4096), dim3(256), 0, 0, (const uint4*)vlh, (int64_t)(os_bytes / 16), sink);
  });
  auto fin = [&](auto kern, int nt) {
    return [&, kern, nt] {
      hipLaunchKernelGGL(kern, dim3((unsigned)S), dim3(nt), 0, 0, hist, rmask, 0, qp, vlh, parts, 16,
                         zeros, (uint32_t*)nullptr, (const unsigned long long*)nullptr, 0ull);
    };
  };
  time("hfin 1024 (no reset)", osb, fin(k_hist_finalize<8, 1024>, 1024));
  time("hfin 1024 no output", 0, fin(k_hist_finalize<9, 1024>, 1024));
  time("hfin 1024 no pooled", osb, fin(k_hist_finalize<12, 1024>, 1024));
  time("hfin 1024 scan only", 0, fin(k_hist_finalize<13, 1024>, 1024));
  time("hfin 256 (no reset)", osb, fin(k_hist_finalize<8, 256>, 256));
  time("pct_acc prod", osb, [&] { launch_pct_accumulate(vlh, S, S, Q, gamma, acc, 0); });
  time("pct_acc U32", osb, [&] {
    hipLaunchKernelGGL(k_pct_acc_u<32>, dim3((unsigned)cdiv(Q, 256)), dim3(256), 0, 0, vlh, S,
                       S * kOsTile, Q, gamma, acc);
  });
  CK(hipDeviceSynchronize());
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
