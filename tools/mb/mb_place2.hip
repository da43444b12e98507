// Microbenchmark (development tool, not shipped): which buffer of a pair sets
// the fused pass's speed, and does a blocked site layout average it out?
// Round 2 found the fused pass running 12.8-14.7 ms on different (input,
// output) pairs of 38 GB buffers in one process (profiles/r2/mb_place_r2pl.txt).
// Here, in one process:
//   1. NB contiguous site buffers: the fused pass and a plain copy kernel on
//      every ordered (input, output) pair, a read-only and a write-only pass
//      on every buffer -- the matrix says whether the input, the output or
//      the pair decides;
//   2. the same sites in a blocked layout (blocks of B sites, input and
//      output blocks allocated alternately) through the production fused
//      pass's SiteTab path, for several B.
// Usage: mb_place2 [n_sites=3456] [n_buffers=4] [reps=2] [blocks="16,64"]
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

__global__ __launch_bounds__(256) void k_copy1(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                               int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) c[i] = a[i];
}

__global__ __launch_bounds__(256) void k_write1(u32x4* __restrict__ c, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) c[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

__global__ __launch_bounds__(256) void k_read1(const u32x4* __restrict__ a, int64_t n,
                                               unsigned* sink) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const u32x4 v = a[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u) sink[0] = v.x;
}

int main(int argc, char** argv) {
  try {
    const int64_t S = argc > 1 ? atoll(argv[1]) : 3456;
    const int NB = argc > 2 ? atoi(argv[2]) : 4;
    const int reps = argc > 3 ? atoi(argv[3]) : 2;
    std::vector<int> blocks;
    {
      std::string b = argc > 4 ? argv[4] : "16,64";
      size_t p = 0;
      while (p < b.size()) {
        const size_t q = b.find(',', p);
        blocks.push_back(atoi(b.substr(p, q - p).c_str()));
        if (q == std::string::npos) break;
        p = q + 1;
      }
    }
    const int H = 2160, W = 2560;
    const int64_t npx = (int64_t)H * W;
    const size_t bytes = (size_t)S * npx * 2;
    const int64_t n16 = (int64_t)(bytes / 16);
    std::vector<uint16_t*> buf(NB);
    for (int i = 0; i < NB; ++i) {
      CK(hipMalloc(&buf[i], bytes));
      launch_synth(buf[i], S, H, W, 12345, 0, 0, 0, 0);
      printf("buffer %d at %p\n", i, (void*)buf[i]);
    }
    CK(hipDeviceSynchronize());
    float4 *coef, *mconst2;
    uint32_t* hist;
    unsigned long long *rmask, *fe;
    unsigned int *fn, *sink;
    int* queues;
    CK(hipMalloc(&coef, npx * 8));
    CK(hipMalloc(&mconst2, 16));
    CK(hipMalloc(&hist, (size_t)S * kBins * 4));
    CK(hipMalloc(&rmask, S * 8));
    CK(hipMalloc(&fe, (size_t)1 << 23));
    CK(hipMalloc(&fn, 4));
    CK(hipMalloc(&sink, 4));
    CK(hipMalloc(&queues, kFusedQueueInts * sizeof(int)));
    {
      std::vector<float> c(npx * 2);
      for (int64_t i = 0; i < npx * 2; ++i) c[i] = (i & 2) ? 1.02f : 8.3f;
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
    auto time = [&](auto&& launch) {
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
      return tot / reps;
    };
    auto fused = [&](const uint16_t* in, uint16_t* out, const SiteTab& tab) {
      return time([&] {
        CK(hipMemsetAsync(fn, 0, 4, 0));
        CK(hipMemsetAsync(rmask, 0, S * 8, 0));
        launch_correct_hist(in, out, npx, S, (const float2*)coef, mconst2, fl, 1, -1, -1, hist,
                            rmask, queues, cus, kFusedNarrow, 0, 0, tab);
      });
    };
    double *mean, *m2, *lut, *rn, *part;
    unsigned long long* wide;
    CK(hipMalloc(&mean, npx * 8));
    CK(hipMalloc(&m2, npx * 8));
    CK(hipMalloc(&lut, 65536 * 8));
    CK(hipMalloc(&rn, S * 8));
    CK(hipMalloc(&part, 8 * npx * 8));
    CK(hipMalloc(&wide, 16));
    {
      std::vector<double> l(65536);
      for (int i = 0; i < 65536; ++i) l[i] = i ? std::log10((double)i) : 0.0;
      CK(hipMemcpy(lut, l.data(), 65536 * 8, hipMemcpyHostToDevice));
    }
    auto welford = [&](const uint16_t* in, const SiteTab& tab) {
      return time([&] {
        launch_welford(in, npx, S, 0, rn, mean, m2, lut, 1, part, 8 * npx, 1, wide, 0, 0, -1,
                       tab);
      });
    };
    const unsigned g16 = (unsigned)((n16 + 255) / 256);
    for (int i = 0; i < NB; ++i) {
      const float r = time([&] {
        hipLaunchKernelGGL(k_read1, dim3(g16), dim3(256), 0, 0, (const u32x4*)buf[i], n16, sink);
      });
      printf("read  %d: %8.3f ms  %.0f GB/s\n", i, r, bytes / (r * 1e6));
    }
    printf("fused matrix (row = input, column = output), ms\n");
    for (int i = 0; i < NB; ++i) {
      printf("in %d:", i);
      for (int o = 0; o < NB; ++o)
        printf(" %8.3f", i == o ? 0.0f : fused(buf[i], buf[o], SiteTab{}));
      printf("\n");
      fflush(stdout);
    }
    printf("copy matrix (row = input, column = output), ms\n");
    for (int i = 0; i < NB; ++i) {
      printf("in %d:", i);
      for (int o = 0; o < NB; ++o)
        printf(" %8.3f", i == o ? 0.0f : time([&] {
          hipLaunchKernelGGL(k_copy1, dim3(g16), dim3(256), 0, 0, (const u32x4*)buf[i],
                             (u32x4*)buf[o], n16);
        }));
      printf("\n");
      fflush(stdout);
    }
    for (int i = 0; i < NB; ++i) {
      const float r = time([&] {
        hipLaunchKernelGGL(k_write1, dim3(g16), dim3(256), 0, 0, (u32x4*)buf[i], n16);
      });
      printf("write %d: %8.3f ms  %.0f GB/s\n", i, r, bytes / (r * 1e6));
    }
    // free two contiguous buffers' worth for the blocked layouts
    for (int i = 2; i < NB; ++i) CK(hipFree(buf[i]));
    for (int i = 0; i < 2; ++i) launch_synth(buf[i], S, H, W, 12345, 0, 0, 0, 0);  // after the writes
    for (int B : blocks) {
      const int nblk = (int)((S + B - 1) / B);
      int shift = 0;
      while ((1 << shift) < B) ++shift;
      std::vector<uint16_t*> ib(nblk), ob(nblk);
      for (int k = 0; k < nblk; ++k) {  // input and output blocks alternately
        CK(hipMalloc(&ib[k], (size_t)B * npx * 2));
        CK(hipMalloc(&ob[k], (size_t)B * npx * 2));
        const int64_t n = std::min<int64_t>(B, S - (int64_t)k * B);
        launch_synth(ib[k], n, H, W, 12345, 0, (int64_t)k * B, 0, 0);
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
      printf("blocked B=%d (%d blocks):", 1 << shift, nblk);
      for (int r = 0; r < 3; ++r) printf(" %8.3f", fused(nullptr, nullptr, tab));
      printf("   contiguous 0->1: %8.3f  1->0: %8.3f\n", fused(buf[0], buf[1], SiteTab{}),
             fused(buf[1], buf[0], SiteTab{}));
      printf("  welford blocked:");
      for (int r = 0; r < 3; ++r) printf(" %8.3f", welford(nullptr, tab));
      printf("   contiguous 0: %8.3f  1: %8.3f\n", welford(buf[0], SiteTab{}),
             welford(buf[1], SiteTab{}));
      fflush(stdout);
      for (int k = 0; k < nblk; ++k) {
        CK(hipFree(ib[k]));
        CK(hipFree(ob[k]));
      }
      CK(hipFree(tin));
      CK(hipFree(tout));
    }
    {  // the blocked code path over ONE contiguous buffer: code cost vs placement
      const int B = 64, nblk = (int)((S + B - 1) / B);
      std::vector<uint16_t*> ib(nblk);
      for (int k = 0; k < nblk; ++k) ib[k] = buf[0] + (size_t)k * B * npx;
      uint16_t** tin;
      CK(hipMalloc(&tin, nblk * sizeof(void*)));
      CK(hipMemcpy(tin, ib.data(), nblk * sizeof(void*), hipMemcpyHostToDevice));
      SiteTab tab;
      tab.in = tin;
      tab.out = nullptr;
      tab.shift = 6;
      printf("welford, blocked path over contiguous buffer 0:");
      for (int r = 0; r < 3; ++r) printf(" %8.3f", welford(nullptr, tab));
      printf("   contiguous path: %8.3f %8.3f\n", welford(buf[0], SiteTab{}),
             welford(buf[0], SiteTab{}));
    }
    printf("done\n");
  } catch (const tmh::Error& e) {
    fprintf(stderr, "tmh::Error %d: %s\n", e.code, e.msg.c_str());
    return 1;
  }
  return 0;
}
