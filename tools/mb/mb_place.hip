// Microbenchmark (development tool, not shipped): does the fused pass's speed
// depend on where its 76 GB of sites and outputs sit in HBM?  Successive
// bench processes on one box ran the fused pass at 13.5 and 14.4 ms in
// alternation with the same library (profiles/r2/ab_forkfix_r2fx.jsonl).
// Here one process allocates NB site-sized buffers (38 GB each at the bench
// size), fills the first with the bench's sites and copies it to the others,
// then times the production fused pass (narrow configuration) and the
// Welford pass for several (input, output) buffer pairs.  (Round 2 also ran
// the fused pass with each unit's band walk rotated by a hash of the unit, to
// de-synchronise the concurrent streams' offsets: no better on any pair,
// profiles/r2/mb_place_rot_r2pl.txt.)
// Usage: mb_place [n_sites=3456] [n_buffers=6] [reps=3] [mode=0] [fill=0]
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

static int run(int argc, char** argv) {
  const int64_t S = argc > 1 ? atoll(argv[1]) : 3456;
  const int NB = argc > 2 ? atoi(argv[2]) : 6;
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  const int H = 2160, W = 2560;
  const int64_t npx = (int64_t)H * W;
  const size_t bytes = (size_t)S * npx * 2;
  // mode 0: hipMalloc; 1: hipExtMallocWithFlags(hipDeviceMallocContiguous);
  // 2: alternating (even buffers plain, odd contiguous)
  const int mode = argc > 4 ? atoi(argv[4]) : 0;
  std::vector<uint16_t*> buf(NB);
  for (int i = 0; i < NB; ++i) {
    const bool contig = mode == 1 || (mode == 2 && (i & 1));
    // + 64 MB of slack: the output offset sweep below writes at buf + delta
    if (contig)
      CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&buf[i]), bytes + (64 << 20),
                               hipDeviceMallocContiguous));
    else
      CK(hipMalloc(&buf[i], bytes + (64 << 20)));
    printf("buffer %d at %p%s\n", i, (void*)buf[i], contig ? " (contiguous)" : "");
  }
  // fill: buffer 0 by the generator kernel, the others by device copies
  // (fill=1: every buffer by the generator kernel)
  const int fill = argc > 5 ? atoi(argv[5]) : 0;
  launch_synth(buf[0], S, H, W, 12345, 0, 0, 0, 0);
  for (int i = 1; i < NB; ++i) {
    if (fill == 1)
      launch_synth(buf[i], S, H, W, 12345, 0, 0, 0, 0);
    else
      CK(hipMemcpy(buf[i], buf[0], bytes, hipMemcpyDeviceToDevice));
  }
  CK(hipDeviceSynchronize());
  float4 *coef, *mconst2;
  uint32_t* hist;
  unsigned long long *rmask, *fe, *wide;
  unsigned int* fn;
  int* queues;
  double *mean, *m2, *lut, *rn, *part;
  CK(hipMalloc(&coef, npx * 8));
  CK(hipMalloc(&mconst2, 16));
  CK(hipMalloc(&hist, (size_t)S * kBins * 4));
  CK(hipMalloc(&rmask, S * 8));
  CK(hipMalloc(&fe, (size_t)1 << 23));
  CK(hipMalloc(&fn, 4));
  CK(hipMalloc(&wide, 16));
  CK(hipMalloc(&queues, kFusedQueueInts * sizeof(int)));
  CK(hipMalloc(&mean, npx * 8));
  CK(hipMalloc(&m2, npx * 8));
  CK(hipMalloc(&lut, 65536 * 8));
  CK(hipMalloc(&rn, S * 8));
  CK(hipMalloc(&part, 8 * npx * 8));
  {
    std::vector<float> c(npx * 2);
    for (int64_t i = 0; i < npx * 2; ++i) c[i] = (i & 2) ? 1.02f : 8.3f;
    CK(hipMemcpy(coef, c.data(), npx * 8, hipMemcpyHostToDevice));
    const float m[4] = {8.2f, 0.0f, 1e-10f, 3.0e38f};
    CK(hipMemcpy(mconst2, m, 16, hipMemcpyHostToDevice));
    std::vector<double> l(65536);
    for (int i = 0; i < 65536; ++i) l[i] = i ? std::log10((double)i) : 0.0;
    CK(hipMemcpy(lut, l.data(), 65536 * 8, hipMemcpyHostToDevice));
  }
  CK(hipMemset(hist, 0, (size_t)S * kBins * 4));
  CK(hipMemset(rmask, 0, S * 8));
  CK(hipMemset(wide, 0, 16));
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
  auto fused = [&](int i, int o) {
    return time([&] {
      CK(hipMemsetAsync(fn, 0, 4, 0));
      // zero-maintained slab: the production finalize resets it; here a memset
      CK(hipMemsetAsync(rmask, 0, S * 8, 0));
      launch_correct_hist(buf[i], buf[o], npx, S, (const float2*)coef, mconst2, fl, 1, -1, -1, hist,
                          rmask, queues, cus, kFusedNarrow, 0, 0);
    });
  };
  // output written at buf[o] + delta bytes: does the read/write address
  // relation matter?
  auto fused_at = [&](int i, int o, size_t delta) {
    return time([&] {
      CK(hipMemsetAsync(fn, 0, 4, 0));
      CK(hipMemsetAsync(rmask, 0, S * 8, 0));
      launch_correct_hist(buf[i], reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(buf[o]) + delta),
                          npx, S, (const float2*)coef, mconst2, fl, 1, -1, -1, hist, rmask, queues,
                          cus, kFusedNarrow, 0, 0);
    });
  };
  auto welford = [&](int i) {
    return time([&] {
      launch_welford(buf[i], npx, S, 0, rn, mean, m2, lut, 1, part, 8 * npx, 1, wide, 0, 0);
    });
  };
  for (int i = 0; i < NB; ++i) printf("welford on buffer %d: %8.3f ms\n", i, welford(i));
  for (int pass = 0; pass < 2; ++pass)
    for (int i = 0; i < NB; ++i) {
      const int o = (i + 1) % NB;
      printf("fused in %d -> out %d: %8.3f ms\n", i, o, fused(i, o));
      fflush(stdout);
    }
  printf("fused in 0 -> out 0 (in place): %8.3f ms\n", fused(0, 0));
  const size_t deltas[] = {0, 4096, 65536, 1u << 20, (2u << 20) + 4096, 16u << 20, 48u << 20};
  for (int i = 0; i < NB; ++i) {
    const int o = (i + 1) % NB;
    printf("fused in %d -> out %d + delta:", i, o);
    for (size_t d : deltas) printf(" %zu:%.3f", d, fused_at(i, o, d));
    printf("\n");
    fflush(stdout);
  }
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
