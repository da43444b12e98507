// Microbenchmark (development tool, not shipped): the illuminati chain pass
// (correct -> align -> clip -> scale u8, 3 B/px), per-site shifts as
// bench.py's extra, with a device checksum of the uint8 output.  (Round 2
// measured a variant staging SB = 2 / 4 sites per barrier pair: 17.65 / 16.74
// ms vs 15.36 for one site, identical checksums: profiles/r2/mb_chain_r2zf.txt.)
// Round 3: k_chain_u8t (the production form, VALU trimmed) against
// k_chain_u8's 64 KB-table form, same checksum expected.
// Usage: mb_chain [n_sites=3456] [reps=3]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../tmlibrary_amd/csrc/common.h"
#include "../../tmlibrary_amd/csrc/chain_kernels.hip"
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

__global__ void k_sum(const uint8_t* __restrict__ p, int64_t n, unsigned long long* out) {
  unsigned long long t = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    t += (unsigned long long)p[i] * (unsigned long long)((i % 65521) + 1);
  atomicAdd(out, t);
}

static int run(int argc, char** argv) {
  const int64_t S = argc > 1 ? atoll(argv[1]) : 3456;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  const int H = 2160, W = 2560;
  const int64_t npx = (int64_t)H * W;
  uint16_t* in;
  uint8_t* out;
  CK(hipMalloc(&in, S * npx * 2));
  CK(hipMalloc(&out, S * npx));
  launch_synth(in, S, H, W, 12345, 0, 0, 0, 0);
  float2* clin;
  float4* mc2;
  unsigned long long *fe, *sum;
  unsigned int* fn;
  tmh_window* dw;
  CK(hipMalloc(&clin, npx * 8));
  CK(hipMalloc(&mc2, 16));
  CK(hipMalloc(&fe, (size_t)1 << 23));
  CK(hipMalloc(&fn, 4));
  CK(hipMalloc(&sum, 8));
  CK(hipMalloc(&dw, S * sizeof(tmh_window)));
  {
    std::vector<float> c(npx * 2);
    for (int64_t i = 0; i < npx; ++i) {
      c[2 * i] = 8.3f + 0.1f * (float)((i * 7) % 13) / 13.0f;  // mu * log2(10)
      c[2 * i + 1] = 1.0f + 0.05f * (float)((i * 5) % 11) / 11.0f;  // mean(std) / std
    }
    CK(hipMemcpy(clin, c.data(), npx * 8, hipMemcpyHostToDevice));
    const float m[4] = {8.2f, 0.0f, 1e-10f, 3.0e38f};  // T huge: nothing flagged
    CK(hipMemcpy(mc2, m, 16, hipMemcpyHostToDevice));
    std::vector<tmh_window> w(S);
    for (int64_t i = 0; i < S; ++i) {
      const int dy = (int)(i % 7) - 3, dx = (int)(i % 9) - 4;
      w[i].src_r0 = 3 - dy; w[i].src_c0 = 4 - dx; w[i].dst_r0 = 3; w[i].dst_c0 = 4;
      w[i].rows = H - 6; w[i].cols = W - 8;
    }
    CK(hipMemcpy(dw, w.data(), S * sizeof(tmh_window), hipMemcpyHostToDevice));
  }
  const FixList fl{fe, fn, (unsigned)(((size_t)1 << 23) / 8)};
  const int lo = 110, hi = 4000;
  const double step = scale_step(lo, hi);
  const int T = hi - lo - 1;
  const int64_t parts = 8, per = (S + parts - 1) / parts;
  const dim3 grid((unsigned)((npx / 8 + 255) / 256), (unsigned)((S + per - 1) / per));
  const size_t shm = (size_t)((hi - lo + 1 + 15) & ~15);
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
    CK(hipMemset(out, 0, S * npx));
    launch();
    CK(hipMemset(sum, 0, 8));
    hipLaunchKernelGGL(k_sum, dim3(4096), dim3(256), 0, 0, out, S * npx, sum);
    unsigned long long h = 0;
    CK(hipMemcpy(&h, sum, 8, hipMemcpyDeviceToHost));
    const double ms = tot / reps, bytes = 3.0 * S * npx;
    printf("%-30s %8.3f ms %7.1f GB/s %5.1f%%  checksum %llu\n", name, ms, bytes / (ms * 1e-3) / 1e9,
           100.0 * bytes / (ms * 1e-3) / 8e12, h);
    fflush(stdout);
  };
  uint8_t* lut8;
  CK(hipMalloc(&lut8, 65536));
  hipLaunchKernelGGL(k_chain_lut8, dim3(256), dim3(256), 0, 0, lut8, lo, hi, T, step);
  auto full = [&](const char* nm, auto nt_tag) {
    constexpr int NT = decltype(nt_tag)::value;
    const dim3 g((unsigned)((npx / 8 + NT - 1) / NT), grid.y);
    time(nm, [&] {
      CK(hipMemsetAsync(fn, 0, 4, 0));
      hipLaunchKernelGGL((k_chain_u8<true, 2, NT>), g, dim3(NT), 65536, 0, in, out, H, W, S, per,
                         clin, mc2, fl, dw, lo, hi, T, step, lut8);
    });
  };
  auto trimmed = [&](const char* nm, auto z_tag, auto pf_tag, int64_t prt, auto gb_tag) {
    constexpr bool Z = decltype(z_tag)::value, PF = decltype(pf_tag)::value;
    constexpr bool GB = decltype(gb_tag)::value;
    const int64_t pp = (S + prt - 1) / prt;
    const dim3 g((unsigned)((npx / 8 + 1023) / 1024), (unsigned)((S + pp - 1) / pp));
    time(nm, [&] {
      CK(hipMemsetAsync(fn, 0, 4, 0));
      hipLaunchKernelGGL((k_chain_u8t<true, Z, 1024, PF, GB>), g, dim3(1024), 65536, 0, in, out, H, W,
                         S, pp, clin, mc2, fl, dw, lut8);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  auto seamed = [&](const char* nm, auto seam_tag) {
    constexpr bool SM = decltype(seam_tag)::value;
    const int64_t pp = (S + 15) / 16;
    const dim3 g((unsigned)((npx / 8 + 1023) / 1024), (unsigned)((S + pp - 1) / pp));
    time(nm, [&] {
      CK(hipMemsetAsync(fn, 0, 4, 0));
      hipLaunchKernelGGL((k_chain_u8t<true, true, 1024, true, true, SM>), g, dim3(1024), 65536, 0,
                         in, out, H, W, S, pp, clin, mc2, fl, dw, lut8);
    });
  };
  for (int r = 0; r < 3; ++r) {
    seamed("stage whole workgroup (2 barriers)", F_());
    seamed("stage seam lines only (1 barrier)", T_());
  }
  // (Measured and removed: 960- and 896-thread workgroups with a
  // double-buffered stage and one barrier per site -- the only shapes whose
  // two stages fit beside the 64 KB table at two workgroups per CU: 12.68 /
  // 17.04 ms against 12.06 for 1,024 threads with two barriers per site;
  // profiles/r3/mb_chain_stage_db_r3z6.txt.)
  for (int r = 0; r < 2; ++r) {
    full("chain k_chain_u8 64 KB, NT 1024", std::integral_constant<int, 1024>());
    trimmed("chain k_chain_u8t (zf add)", T_(), F_(), 8, T_());
    trimmed("chain k_chain_u8t (zf max)", F_(), F_(), 8, T_());
    trimmed("chain k_chain_u8t prefetch", T_(), T_(), 8, T_());
    trimmed("chain k_chain_u8t 6 parts", T_(), F_(), 6, T_());
    trimmed("chain k_chain_u8t 12 parts", T_(), F_(), 12, T_());
    trimmed("chain k_chain_u8t 16 parts", T_(), F_(), 16, T_());
    trimmed("chain k_chain_u8t pf 16 parts", T_(), T_(), 16, T_());
    trimmed("chain k_chain_u8t pf 24 parts", T_(), T_(), 24, T_());
    trimmed("chain k_chain_u8t pf 32 parts", T_(), T_(), 32, T_());
    trimmed("chain k_chain_u8t pf 16, launch T", T_(), T_(), 16, F_());
  }
  {  // realistic flags: T from the coefficients (a_max 1.05 except 64 columns at a = 40)
    std::vector<float> c(npx * 2);
    for (int64_t i = 0; i < npx; ++i) {
      c[2 * i] = 8.3f + 0.1f * (float)((i * 7) % 13) / 13.0f;
      c[2 * i + 1] = (i % W) >= 1000 && (i % W) < 1064 ? 40.0f : 1.0f + 0.05f * (float)((i * 5) % 11) / 11.0f;
    }
    CK(hipMemcpy(clin, c.data(), npx * 8, hipMemcpyHostToDevice));
    const float T = (float)(1.0 / (6.7e-6 * 40.0 + 4.2e-6));
    const float m[4] = {8.2f, 0.0f, 1e-10f, T};
    CK(hipMemcpy(mc2, m, 16, hipMemcpyHostToDevice));
    unsigned int nf = 0;
    for (int r = 0; r < 2; ++r) {
      trimmed("FLAGS k_chain_u8t pf 16, group bound", T_(), T_(), 16, T_());
      CK(hipMemcpy(&nf, fn, 4, hipMemcpyDeviceToHost));
      printf("   flagged groups %u\n", nf);
      trimmed("FLAGS k_chain_u8t pf 16, launch T", T_(), T_(), 16, F_());
      CK(hipMemcpy(&nf, fn, 4, hipMemcpyDeviceToHost));
      printf("   flagged groups %u\n", nf);
    }
  }
  {  // ablation: every site unshifted (line-aligned destination: no LDS staging, no barriers)
    std::vector<tmh_window> w0(S);
    for (int64_t i = 0; i < S; ++i) w0[i] = tmh_window{0, 0, 0, 0, H, W};
    CK(hipMemcpy(dw, w0.data(), S * sizeof(tmh_window), hipMemcpyHostToDevice));
    trimmed("ABLATION unshifted k_chain_u8t pf 16", T_(), T_(), 16, T_());
    full("ABLATION unshifted k_chain_u8 1024", std::integral_constant<int, 1024>());
    std::vector<tmh_window> w(S);
    for (int64_t i = 0; i < S; ++i) {
      const int dy = (int)(i % 7) - 3, dx = (int)(i % 9) - 4;
      w[i].src_r0 = 3 - dy; w[i].src_c0 = 4 - dx; w[i].dst_r0 = 3; w[i].dst_c0 = 4;
      w[i].rows = H - 6; w[i].cols = W - 8;
    }
    CK(hipMemcpy(dw, w.data(), S * sizeof(tmh_window), hipMemcpyHostToDevice));
  }
  for (int r = 0; r < 1; ++r) {
    time("chain (clipped-range table)", [&] {
      CK(hipMemsetAsync(fn, 0, 4, 0));
      hipLaunchKernelGGL((k_chain_u8<true, 1>), grid, dim3(256), shm, 0, in, out, H, W, S, per,
                         clin, mc2, fl, dw, lo, hi, T, step, nullptr);
    });
    full("chain 64 KB table, NT 256", std::integral_constant<int, 256>());
    full("chain 64 KB table, NT 512", std::integral_constant<int, 512>());
    full("chain 64 KB table, NT 1024", std::integral_constant<int, 1024>());
  }
  // VALU-bound check: the same pass without the log / exp (two transcendental
  // ops per pixel; different output, same bytes)
  time("chain without log/exp (LOG=false)", [&] {
    CK(hipMemsetAsync(fn, 0, 4, 0));
    hipLaunchKernelGGL((k_chain_u8<false, 1>), grid, dim3(256), shm, 0, in, out, H, W, S, per,
                       clin, mc2, fl, dw, lo, hi, T, step, nullptr);
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
