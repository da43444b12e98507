// Microbenchmark (development tool, not shipped): the sigma-5 one-pass
// smoothing of a job's planes (apply_kernels.hip).  k_smooth_2d (16 rows per
// workgroup, every input row read 2R + 16 times per 16 rows, 41 LDS reads per
// axis-1 output) against k_smooth_2d_blk (18 axis-1 outputs per thread), on
// NP = 2 and 8 planes of 2160 x 2560:
// half mean planes, half M2 planes read as std (finalize-on-read).  Every
// form's outputs and tile partials must equal k_smooth_2d's bit for bit.
// Usage: mb_smooth [reps=20]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../tmlibrary_amd/csrc/common.h"
#include "../../tmlibrary_amd/csrc/apply_kernels.hip"

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

static std::vector<double> taps5() {  // abi.hip gaussian_taps(5)
  const int lw = 20;
  std::vector<double> w(2 * lw + 1, 0.0);
  w[lw] = 1.0;
  double sum = 1.0;
  for (int ii = 1; ii <= lw; ++ii) {
    const double t = std::exp(-0.5 * (double)(ii * ii) / 25.0);
    w[lw + ii] = t;
    w[lw - ii] = t;
    sum += 2.0 * t;
  }
  for (auto& x : w) x /= sum;
  return w;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const int H = 2160, W = 2560;
  const int64_t npx = (int64_t)H * W;
  const int nt = (int)(cdiv(W, kSumTW) * cdiv(H, kSumTH));
  const auto w = taps5();
  double* dw;
  CK(hipMalloc(&dw, w.size() * 8));
  CK(hipMemcpy(dw, w.data(), w.size() * 8, hipMemcpyHostToDevice));
  const int NPMAX = 8;
  std::vector<double*> in(NPMAX), out(NPMAX), ref(NPMAX), ps(NPMAX), pm(NPMAX), psr(NPMAX),
      pmr(NPMAX);
  std::mt19937_64 rng(7);
  std::vector<double> h(npx);
  for (int p = 0; p < NPMAX; ++p) {
    const bool std_plane = p & 1;
    std::uniform_real_distribution<double> d(std_plane ? 10.0 : 2.0, std_plane ? 400.0 : 4.0);
    for (auto& x : h) x = d(rng);
    if (p == 3) h[12345] = 0.0;  // a zero std somewhere
    CK(hipMalloc(&in[p], npx * 8));
    CK(hipMemcpy(in[p], h.data(), npx * 8, hipMemcpyHostToDevice));
    for (double** b : {&out[p], &ref[p]}) CK(hipMalloc(b, npx * 8));
    for (double** b : {&ps[p], &pm[p], &psr[p], &pmr[p]}) CK(hipMalloc(b, nt * 8));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Form {
    const char* name;
    int id;
  };
  const Form forms[] = {{"2d (round 5)", 0}, {"blk (shipped)", 1}};
  bool all_ok = true;
  for (int np : {2, 8}) {
    auto planes = [&](bool is_ref) {
      SmPlanes a{};
      for (int p = 0; p < np; ++p) {
        a.in[p] = in[p];
        a.out[p] = is_ref ? ref[p] : out[p];
        a.sq[p] = (p & 1) ? 3455.0 : 0.0;
        a.psum[p] = is_ref ? psr[p] : ps[p];
        a.pmin[p] = (p & 1) ? (is_ref ? pmr[p] : pm[p]) : nullptr;
      }
      return a;
    };
    for (const Form& f : forms) {
      const bool is_ref = f.id == 0;
      const SmPlanes a = planes(is_ref);
      auto launch = [&] {
        const unsigned gx = (unsigned)cdiv(W, kSumTW);
        const dim3 g(gx, (unsigned)cdiv(H, kSumTH), (unsigned)np);
        if (f.id == 0)
          hipLaunchKernelGGL((k_smooth_2d<kSumTH, 20>), g, dim3(256), 0, 0, a, H, W, dw);
        else
          hipLaunchKernelGGL(k_smooth_2d_blk, g, dim3(256), 0, 0, a, H, W, dw);
      };
      launch();
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      bool ok = true;
      if (!is_ref) {
        std::vector<double> A(npx), B(npx), pa(nt), pb(nt);
        for (int p = 0; p < np && ok; ++p) {
          CK(hipMemcpy(A.data(), out[p], npx * 8, hipMemcpyDeviceToHost));
          CK(hipMemcpy(B.data(), ref[p], npx * 8, hipMemcpyDeviceToHost));
          ok = ok && memcmp(A.data(), B.data(), npx * 8) == 0;
          CK(hipMemcpy(pa.data(), ps[p], nt * 8, hipMemcpyDeviceToHost));
          CK(hipMemcpy(pb.data(), psr[p], nt * 8, hipMemcpyDeviceToHost));
          ok = ok && memcmp(pa.data(), pb.data(), nt * 8) == 0;
          if (p & 1) {
            CK(hipMemcpy(pa.data(), pm[p], nt * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(pb.data(), pmr[p], nt * 8, hipMemcpyDeviceToHost));
            ok = ok && memcmp(pa.data(), pb.data(), nt * 8) == 0;
          }
        }
      }
      all_ok = all_ok && ok;
      printf("np %d  %-16s avg %8.4f ms  %s\n", np, f.name, ms / reps,
             is_ref ? "(reference)" : (ok ? "bit-identical" : "MISMATCH"));
      fflush(stdout);
    }
  }
  printf(all_ok ? "ALL OK\n" : "SOME FORMS MISMATCH\n");
  return all_ok ? 0 : 1;
}
