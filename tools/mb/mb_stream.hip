// Microbenchmark (development tool, not shipped): what streaming shape lets a
// pass over the bench's buffers reach the box's copy / read rate?  Round 6's
// box probe found one-16-B-per-thread launches copying the 3,456 sites at
// 6.6 TB/s where a persistent grid-strided copy reached 5.9 and the fused pass
// 5.8 (profiles/r6/bench_quick_r6b.json).  Same layout as bench.py: the sites
// in one buffer, the outputs in 64-site blocks.  Every variant is timed
// (HIP events, reps launches after one warm-up) on the same buffers:
//   copy  flat          one 16-B group per thread, one launch per block
//         grid4         persistent grid-stride, 4 groups in flight per thread
//         queueK        persistent, each workgroup takes the next K x 4 KB
//                       chunk from one atomic counter (address order)
//         fusedA        the production k_correct_hist schedule with ablation
//                       A (33: no histogram, no arithmetic; 1: no histogram;
//                       32: no arithmetic; 0: the real pass)
//   read  flat, welford (production), wfread (its access shape, no compute)
// Usage: mb_stream [n_sites=3456] [reps=3] [dist=0 standard | 1 bright]
// (bright: the packed configuration's ablations -- cfg 5, rare lists on --
// beside the copies)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
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

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_flat_copy(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                                   int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), c + i);
}

__global__ __launch_bounds__(256) void k_flat_read(const u32x4* __restrict__ a, int64_t n,
                                                   unsigned* sink) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const u32x4 v = __builtin_nontemporal_load(a + i);
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u) sink[0] = v.x;
}

// flat, but workgroup k copies 4 KB chunk (k / S) of site k % S: every site
// in flight at once (the dispatcher's order, scattered addresses)
__global__ __launch_bounds__(256) void k_flat_scatter(const u32x4* __restrict__ in,
                                                      u32x4* const* __restrict__ out, int shift,
                                                      int64_t S, int64_t ng) {
  const int64_t k = blockIdx.x;
  const int64_t site = k % S, chunk = k / S;
  const int64_t g = chunk * 256 + threadIdx.x;
  if (g >= ng) return;
  const u32x4 v = __builtin_nontemporal_load(in + site * ng + g);
  u32x4* o = out[site >> shift] + (site & ((1 << shift) - 1)) * ng + g;
  __builtin_nontemporal_store(v, o);
}

// flat, each thread two consecutive 16-B groups (512-B runs per wave... 8 KB per workgroup)
__global__ __launch_bounds__(256) void k_flat_copy2(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                                    int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
  if (i + 1 < n) {
    const u32x4 x = __builtin_nontemporal_load(a + i), y = __builtin_nontemporal_load(a + i + 1);
    __builtin_nontemporal_store(x, c + i);
    __builtin_nontemporal_store(y, c + i + 1);
  } else if (i < n) {
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), c + i);
  }
}

// flat with K consecutive 4 KB chunks per workgroup (thread t: groups t,
// t + 256, ...; U loads in flight): how long-lived may a workgroup be?
template <int K, int U>
__global__ __launch_bounds__(256) void k_flatk_copy(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                                    int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 256 * K + threadIdx.x;
#pragma unroll 1
  for (int k = 0; k < K; k += U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)(k + u) * 256;
      if (i < n) v[u] = __builtin_nontemporal_load(a + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)(k + u) * 256;
      if (i < n) __builtin_nontemporal_store(v[u], c + i);
    }
  }
}

// persistent grid-stride, one group per iteration
__global__ __launch_bounds__(256) void k_grid1_copy(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                                    int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), c + i);
}

// persistent, chunks of K x 4 KB in address order from one counter; the
// chunk's block: in / out tables of nb blocks of per_blk groups (16 B)
template <int K>
__global__ __launch_bounds__(256) void k_queue_copy(const u32x4* const* __restrict__ in,
                                                    u32x4* const* __restrict__ out,
                                                    int64_t per_blk, int64_t total,
                                                    int* __restrict__ ctr) {
  __shared__ int c_sh;
  const int64_t chunk = 256 * K;  // groups per chunk
  const int64_t nchunks = (total + chunk - 1) / chunk;
  for (;;) {
    if (threadIdx.x == 0) c_sh = atomicAdd(ctr, 1);
    __syncthreads();
    const int64_t c = __builtin_amdgcn_readfirstlane(c_sh);
    __syncthreads();
    if (c >= nchunks) break;
    const int64_t g0 = c * chunk;
    const int64_t b = g0 / per_blk, o = g0 - b * per_blk;  // chunks never straddle blocks
    const u32x4* src = in[b] + o;
    u32x4* dst = out[b] + o;
    const int64_t lim = per_blk - o < chunk ? per_blk - o : chunk;
    u32x4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = k * 256 + threadIdx.x;
      if (i < lim) v[k] = __builtin_nontemporal_load(src + i);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = k * 256 + threadIdx.x;
      if (i < lim) __builtin_nontemporal_store(v[k], dst + i);
    }
  }
}

// the Welford pass's access shape without its arithmetic: thread = 16-B group,
// all sites in order, two sites in flight
__global__ __launch_bounds__(256) void k_wf_read(const u32x4* __restrict__ sites, int64_t ngroups,
                                                 int n_sites, unsigned* sink) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= ngroups) return;
  u32x4 acc = {0, 0, 0, 0};
  for (int s = 0; s < n_sites; s += 2) {
    const u32x4 a = __builtin_nontemporal_load(sites + (int64_t)s * ngroups + g);
    const u32x4 b = __builtin_nontemporal_load(sites + (int64_t)(s + 1 < n_sites ? s + 1 : s) * ngroups + g);
    acc ^= a ^ b;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[0] = acc.x;
}

int main(int argc, char** argv) {
  try {
    const int64_t S = argc > 1 ? atoll(argv[1]) : 3456;
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    const int dist = argc > 3 ? atoi(argv[3]) : 0;
    const int H = 2160, W = 2560, B = 64, shift = 6;
    const int64_t npx = (int64_t)H * W, ng = npx / 8;
    const size_t bytes = (size_t)S * npx * 2;
    const int nblk = (int)((S + B - 1) / B);
    uint16_t* in;
    CK(hipMalloc(&in, bytes));
    launch_synth(in, S, H, W, 12345, 0, 0, dist, 0);
    std::vector<uint16_t*> ib(nblk), ob(nblk);
    for (int k = 0; k < nblk; ++k) {
      ib[k] = in + (size_t)k * B * npx;
      CK(hipMalloc(&ob[k], (size_t)B * npx * 2));
    }
    uint16_t **tin, **tout;
    CK(hipMalloc(&tin, nblk * sizeof(void*)));
    CK(hipMalloc(&tout, nblk * sizeof(void*)));
    CK(hipMemcpy(tin, ib.data(), nblk * sizeof(void*), hipMemcpyHostToDevice));
    CK(hipMemcpy(tout, ob.data(), nblk * sizeof(void*), hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    SiteTab tab;
    tab.in = tin;
    tab.out = tout;
    tab.shift = shift;
    float4 *coef, *mconst2;
    uint32_t* hist;
    unsigned long long *rmask, *fe;
    unsigned int *fn, *sink;
    int *queues, *ctr;
    CK(hipMalloc(&coef, npx * 8));
    CK(hipMalloc(&mconst2, 16));
    CK(hipMalloc(&hist, (size_t)S * kBins * 4));
    CK(hipMalloc(&rmask, S * 8));
    CK(hipMalloc(&fe, (size_t)1 << 23));
    CK(hipMalloc(&fn, 4));
    CK(hipMalloc(&sink, 4));
    CK(hipMalloc(&queues, kFusedQueueInts * sizeof(int)));
    CK(hipMalloc(&ctr, 4));
    uint16_t* rare_v;
    unsigned int* rare_n;
    const unsigned int rare_cap = 65536;
    CK(hipMalloc(&rare_v, (size_t)S * rare_cap * 2));
    CK(hipMalloc(&rare_n, (size_t)S * 4));
    {
      // (c, a) planes of a plausible correction: c = 0.02 * log2 10, a = 1.02
      std::vector<float> c(npx * 2);
      for (int64_t i = 0; i < npx * 2; ++i) c[i] = (i & 2) ? 1.02f : 0.066f;
      CK(hipMemcpy(coef, c.data(), npx * 8, hipMemcpyHostToDevice));
      const float m[4] = {8.2f, 0.0f, 1e-10f, 3.0e38f};
      CK(hipMemcpy(mconst2, m, 16, hipMemcpyHostToDevice));
    }
    CK(hipMemset(hist, 0, (size_t)S * kBins * 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const FixList fl{fe, fn, (unsigned)(((size_t)1 << 23) / 8)};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](const char* name, double nbytes, auto&& launch) {
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
        tot += ms;
        best = ms < best ? ms : best;
      }
      printf("%-22s avg %8.3f ms  min %8.3f ms  %6.0f GB/s\n", name, tot / reps, best,
             nbytes / (tot / reps * 1e6));
      fflush(stdout);
    };
    const double cbytes = 2.0 * bytes, rbytes = (double)bytes;
    const int64_t per_blk = (int64_t)B * ng;
    auto fused = [&](auto kern, int n_wg_mult, int bands, int nt = 512) {
      CK(hipMemsetAsync(fn, 0, 4, 0));
      CK(hipMemsetAsync(rmask, 0, S * 8, 0));
      CK(hipMemsetAsync(queues, 0, kFusedQueueInts * sizeof(int), 0));
      FusedJobs J{};
      J.n = 1;
      J.j[0] = FusedJob{nullptr, nullptr, S, coef, mconst2, fl, hist, rmask,
                        reinterpret_cast<unsigned long long*>(queues + 8), tab, RareList{}};
      hipLaunchKernelGGL(kern, dim3(cus * n_wg_mult), dim3(nt), 0, 0, J, npx, -1, -1, bands,
                         queues);
    };
    // the packed configuration (cfg 5: 4 sites, 1,024 threads, u16 counters,
    // rare lists), as abi.hip launches it for bright jobs
    auto fusedp = [&](auto kern, int bands) {
      CK(hipMemsetAsync(fn, 0, 4, 0));
      CK(hipMemsetAsync(rmask, 0, S * 8, 0));
      CK(hipMemsetAsync(queues, 0, kFusedQueueInts * sizeof(int), 0));
      CK(hipMemsetAsync(rare_n, 0, (size_t)S * 4, 0));
      FusedJobs J{};
      J.n = 1;
      J.j[0] = FusedJob{nullptr, nullptr, S, coef, mconst2, fl, hist, rmask,
                        reinterpret_cast<unsigned long long*>(queues + 8), tab,
                        RareList{rare_v, rare_n, rare_cap}};
      hipLaunchKernelGGL(kern, dim3(cus), dim3(1024), 0, 0, J, npx, -1, -1, bands, queues);
    };
    if (dist == 1) {
      for (int pass = 0; pass < 2; ++pass) {
        printf("-- bright pass %d\n", pass);
        time("copy flat", cbytes, [&] {
          for (int k = 0; k < nblk; ++k) {
            const int64_t n = std::min<int64_t>(B, S - (int64_t)k * B) * ng;
            hipLaunchKernelGGL(k_flat_copy, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0,
                               (const u32x4*)ib[k], (u32x4*)ob[k], n);
          }
        });
        time("copy grid4", cbytes, [&] {
          launch_box_probe(tin, tout, shift, S, npx, 1, (unsigned long long*)fe, sink, cus, 0);
        });
        time("packed abl33 (copy)", cbytes,
             [&] { fusedp(k_correct_hist<true, false, 4, 33, 1024, 65536, true>, 8); });
        time("packed abl1 (no hist)", cbytes,
             [&] { fusedp(k_correct_hist<true, false, 4, 1, 1024, 65536, true>, 8); });
        time("packed abl32 (no arith)", cbytes,
             [&] { fusedp(k_correct_hist<true, false, 4, 32, 1024, 65536, true>, 8); });
        time("packed abl0 (real)", cbytes,
             [&] { fusedp(k_correct_hist<true, false, 4, 0, 1024, 65536, true>, 8); });
        time("packed abl0 16 bands", cbytes,
             [&] { fusedp(k_correct_hist<true, false, 4, 0, 1024, 65536, true>, 16); });
        time("packed abl8 (no flush)", cbytes,
             [&] { fusedp(k_correct_hist<true, false, 4, 8, 1024, 65536, true>, 8); });
        time("packed abl64 (no rare path)", cbytes,
             [&] { fusedp(k_correct_hist<true, false, 4, 64, 1024, 65536, true>, 8); });
        time("packed abl96 (no rare, no arith)", cbytes,
             [&] { fusedp(k_correct_hist<true, false, 4, 96, 1024, 65536, true>, 8); });
      }
      printf("done\n");
      return 0;
    }
    for (int pass = 0; pass < 2; ++pass) {  // twice: the order of the variants should not matter
      printf("-- pass %d\n", pass);
      time("copy flat", cbytes, [&] {
        for (int k = 0; k < nblk; ++k) {
          const int64_t n = std::min<int64_t>(B, S - (int64_t)k * B) * ng;
          hipLaunchKernelGGL(k_flat_copy, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0,
                             (const u32x4*)ib[k], (u32x4*)ob[k], n);
        }
      });
      time("copy grid4", cbytes, [&] {
        launch_box_probe(tin, tout, shift, S, npx, 1, (unsigned long long*)fe, sink, cus, 0);
      });
      time("fused abl33 (copy)", cbytes, [&] {
        fused(k_correct_hist<true, false, 4, 33, 512, 16384, false>, 2, 16);
      });
      time("fused abl1 (no hist)", cbytes, [&] {
        fused(k_correct_hist<true, false, 4, 1, 512, 16384, false>, 2, 16);
      });
      time("fused abl32 (no arith)", cbytes, [&] {
        fused(k_correct_hist<true, false, 4, 32, 512, 16384, false>, 2, 16);
      });
      time("fused abl0 (real)", cbytes, [&] {
        fused(k_correct_hist<true, false, 4, 0, 512, 16384, false>, 2, 16);
      });
      time("fused abl33 64 bands", cbytes, [&] {
        fused(k_correct_hist<true, false, 4, 33, 512, 16384, false>, 2, 64);
      });
      time("copy flat scattered", cbytes, [&] {
        hipLaunchKernelGGL(k_flat_scatter, dim3((unsigned)(S * ((ng + 255) / 256))), dim3(256), 0, 0,
                           (const u32x4*)in, (u32x4* const*)tout, shift, S, ng);
      });
      auto flatk = [&](const char* name, auto kern, int K) {
        time(name, cbytes, [&] {
          for (int k = 0; k < nblk; ++k) {
            const int64_t n = std::min<int64_t>(B, S - (int64_t)k * B) * ng;
            hipLaunchKernelGGL(kern, dim3((unsigned)((n + 256 * K - 1) / (256 * K))), dim3(256), 0, 0,
                               (const u32x4*)ib[k], (u32x4*)ob[k], n);
          }
        });
      };
      flatk("copy flatK4 U1", k_flatk_copy<4, 1>, 4);
      flatk("copy flatK16 U1", k_flatk_copy<16, 1>, 16);
      flatk("copy flatK16 U4", k_flatk_copy<16, 4>, 16);
      flatk("copy flatK256 U1", k_flatk_copy<256, 1>, 256);
      flatk("copy flatK256 U4", k_flatk_copy<256, 4>, 256);
      time("copy grid1 (per block)", cbytes, [&] {
        for (int k = 0; k < nblk; ++k) {
          const int64_t n = std::min<int64_t>(B, S - (int64_t)k * B) * ng;
          hipLaunchKernelGGL(k_grid1_copy, dim3(cus * 8), dim3(256), 0, 0, (const u32x4*)ib[k],
                             (u32x4*)ob[k], n);
        }
      });
      time("fused abl33 cfg1 4x1024", cbytes, [&] {
        fused(k_correct_hist<true, false, 4, 33, 1024, 32768, false>, 1, 16, 1024);
      });
      time("read flat", rbytes, [&] {
        hipLaunchKernelGGL(k_flat_read, dim3((unsigned)((S * ng + 255) / 256)), dim3(256), 0, 0,
                           (const u32x4*)in, S * ng, sink);
      });
      time("read wfshape", rbytes, [&] {
        hipLaunchKernelGGL(k_wf_read, dim3((unsigned)((ng + 255) / 256)), dim3(256), 0, 0,
                           (const u32x4*)in, ng, (int)S, sink);
      });
    }
    printf("done\n");
  } catch (const tmh::Error& e) {
    fprintf(stderr, "tmh::Error %d: %s\n", e.code, e.msg.c_str());
    return 1;
  }
  return 0;
}
