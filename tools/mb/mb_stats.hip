// Microbenchmarks for the stats/apply kernels (development tool, not shipped).
//
// Builds against the production kernels (launch_* from libtmhip sources) and
// adds ablation variants to find each kernel's limiter:
//   stream_read / copy        HBM roofline of this access pattern
//   hist_* variants           loads only / LDS atomics only / production
//   welford variants          production
// Usage: mb_stats [n_sites] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#include "../../tmlibrary_amd/csrc/common.h"
#include "../../tmlibrary_amd/csrc/fused_kernels.hip"
#include "../../tmlibrary_amd/csrc/stats_kernels.hip"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

using namespace tmh;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void mb_st_nt(uint4* p, uint4 v) {
  u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

__global__ __launch_bounds__(256) void k_stream_read(const uint4* __restrict__ p, int64_t n,
                                                     uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ p, uint4* __restrict__ q,
                                              int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    q[i] = p[i];
}

// copy variants: U loads in flight per thread, NT = nontemporal stores
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy_u(const uint4* __restrict__ p, uint4* __restrict__ q,
                                                int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += U * stride) {
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = (i + k * stride < n) ? p[i + k * stride] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + k * stride < n) {
        if (NT) mb_st_nt(q + i + k * stride, v[k]);
        else q[i + k * stride] = v[k];
      }
  }
}

// pixel-major copy (the correct kernel's pattern): thread = 8 px, loop sites
template <bool NT>
__global__ __launch_bounds__(256) void k_copy_pm(const uint4* __restrict__ p, uint4* __restrict__ q,
                                                 int64_t ngroups, int64_t n_sites) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= ngroups) return;
  for (int64_t s = 0; s < n_sites; s += 4) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (s + k < n_sites) ? p[(s + k) * ngroups + g] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (s + k < n_sites) {
        if (NT) mb_st_nt(q + (s + k) * ngroups + g, v[k]);
        else q[(s + k) * ngroups + g] = v[k];
      }
  }
}


// block-contiguous copy: one 1024-thread WG streams `chunk` uint4s in order
template <int U, bool NT>
__global__ __launch_bounds__(1024) void k_copy_blk(const uint4* __restrict__ p, uint4* __restrict__ q,
                                                   int64_t chunk, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * chunk;
  const int64_t end = base + chunk < n ? base + chunk : n;
  for (int64_t i = base + threadIdx.x; i < end; i += U * 1024) {
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = (i + k * 1024 < end) ? p[i + k * 1024] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + k * 1024 < end) {
        if (NT) mb_st_nt(q + i + k * 1024, v[k]);
        else q[i + k * 1024] = v[k];
      }
  }
}

// block-contiguous read
template <int U>
__global__ __launch_bounds__(1024) void k_read_blk(const uint4* __restrict__ p, int64_t chunk,
                                                   int64_t n, uint32_t* __restrict__ sink) {
  const int64_t base = (int64_t)blockIdx.x * chunk;
  const int64_t end = base + chunk < n ? base + chunk : n;
  uint32_t acc = 0;
  for (int64_t i = base + threadIdx.x; i < end; i += U * 1024) {
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = (i + k * 1024 < end) ? p[i + k * 1024] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < U; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// welford over a site chunk (grid.y = chunks), partial states per chunk
__global__ __launch_bounds__(256) void k_wf_split(const uint16_t* __restrict__ sites, int64_t npx,
                                                  int64_t n_sites, const double* __restrict__ rn,
                                                  double* __restrict__ mean, double* __restrict__ m2,
                                                  const double* __restrict__ lut) {
  __shared__ double slut[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) slut[i] = lut[i];
  __syncthreads();
  const int64_t ngroups = npx >> 3;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= ngroups) return;
  const int64_t s0 = n_sites * blockIdx.y / gridDim.y, s1 = n_sites * (blockIdx.y + 1) / gridDim.y;
  double mu[8], q[8];
  for (int k = 0; k < 8; ++k) { mu[k] = 0; q[k] = 0; }
  const uint4* src = reinterpret_cast<const uint4*>(sites) + g;
  const int64_t last = s1 - 1;
  uint4 cur[4], nxt[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) cur[k] = src[(s0 + k < last ? s0 + k : last) * ngroups];
  for (int64_t s = s0; s < s1; s += 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) { const int64_t t = s + 4 + k; nxt[k] = src[(t < last ? t : last) * ngroups]; }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (s + k >= s1) continue;
      const double r = rn[s + k - s0];
      const uint32_t w[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
      uint32_t mx = 0;
      double x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t u = (j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xFFFF);
        mx = u > mx ? u : mx;
        x[j] = slut[u & 4095];
      }
      if (mx >= 4096) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t u = (j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xFFFF);
          if (u >= 4096) x[j] = log10((double)u);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const double d = x[j] - mu[j];
        mu[j] = fma(d, r, mu[j]);
        q[j] = fma(d, x[j] - mu[j], q[j]);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
  }
  double* om = mean + blockIdx.y * npx;
  double* oq = m2 + blockIdx.y * npx;
  for (int k = 0; k < 8; ++k) { om[g * 8 + k] = mu[k]; oq[g * 8 + k] = q[k]; }
}


// production-shaped Welford variants: RARE=0 drops the >=4032 fix-up (timing
// only), GROUP sites per pipeline stage, WPS min waves/SIMD launch bound
template <int GROUP, bool RARE, int WPS>
__global__ __launch_bounds__(256, WPS) void k_wf_var(const uint16_t* __restrict__ sites, int64_t npx,
                                                     int64_t n_sites, const double* __restrict__ rn,
                                                     double* __restrict__ mean, double* __restrict__ m2,
                                                     const double* __restrict__ lut) {
  constexpr int LUTN = 4032;
  __shared__ double slut[LUTN];
  for (int i = threadIdx.x; i < LUTN; i += 256) slut[i] = lut[i];
  __syncthreads();
  const int64_t ngroups = npx >> 3;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= ngroups) return;
  double mu[8], q[8];
  for (int k = 0; k < 8; ++k) { mu[k] = mean[g * 8 + k]; q[k] = m2[g * 8 + k]; }
  const uint4* src = reinterpret_cast<const uint4*>(sites) + g;
  const int64_t last = n_sites - 1;
  uint4 cur[GROUP], nxt[GROUP];
#pragma unroll
  for (int k = 0; k < GROUP; ++k) cur[k] = src[(k < last ? k : last) * ngroups];
  for (int64_t s = 0; s < n_sites; s += GROUP) {
#pragma unroll
    for (int k = 0; k < GROUP; ++k) { const int64_t t = s + GROUP + k; nxt[k] = src[(t < last ? t : last) * ngroups]; }
#pragma unroll
    for (int k = 0; k < GROUP; ++k) {
      if (s + k >= n_sites) continue;
      const double r = rn[s + k];
      const uint32_t w[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
      uint32_t u[8], mx = 0;
      double x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        u[j] = (j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xFFFF);
        mx = u[j] > mx ? u[j] : mx;
        x[j] = slut[u[j] < (uint32_t)LUTN ? u[j] : 0u];
      }
      if (RARE && mx >= (uint32_t)LUTN) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (u[j] >= (uint32_t)LUTN) x[j] = log10((double)u[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const double d = x[j] - mu[j];
        mu[j] = fma(d, r, mu[j]);
        q[j] = fma(d, x[j] - mu[j], q[j]);
      }
    }
#pragma unroll
    for (int k = 0; k < GROUP; ++k) cur[k] = nxt[k];
  }
  for (int k = 0; k < 8; ++k) { mean[g * 8 + k] = mu[k]; m2[g * 8 + k] = q[k]; }
}

// welford ablation: MODE 0 = production math, 1 = x = (double)u (no LUT),
// 2 = LUT gather + plain sum (no Welford), 3 = loads + int sum only
template <int MODE>
__global__ __launch_bounds__(256) void k_wf_abl(const uint16_t* __restrict__ sites, int64_t npx,
                                                int64_t n_sites, const double* __restrict__ rn,
                                                double* __restrict__ mean, double* __restrict__ m2,
                                                const double* __restrict__ lut) {
  __shared__ double slut[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) slut[i] = lut[i];
  __syncthreads();
  const int64_t ngroups = npx >> 3;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= ngroups) return;
  double mu[8], q[8];
  for (int k = 0; k < 8; ++k) { mu[k] = mean[g * 8 + k]; q[k] = m2[g * 8 + k]; }
  const uint4* src = reinterpret_cast<const uint4*>(sites) + g;
  const int64_t last = n_sites - 1;
  uint4 cur[4], nxt[4];
  uint32_t isum = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) cur[k] = src[(k < last ? k : last) * ngroups];
  for (int64_t s = 0; s < n_sites; s += 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) { const int64_t t = s + 4 + k; nxt[k] = src[(t < last ? t : last) * ngroups]; }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (s + k >= n_sites) continue;
      const double r = rn[s + k];
      const uint32_t w[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t u = (j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xFFFF);
        if (MODE == 3) { isum += u; continue; }
        double x = (MODE == 1) ? (double)u : slut[u & 4095];
        if (MODE == 2) { mu[j] += x; continue; }
        const double d = x - mu[j];
        mu[j] = fma(d, r, mu[j]);
        q[j] = fma(d, x - mu[j], q[j]);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
  }
  for (int k = 0; k < 8; ++k) { mean[g * 8 + k] = mu[k] + isum; m2[g * 8 + k] = q[k]; }
}

// hist ablation: MODE 0 = loads + integer sum only, 1 = LDS atomics (no hi branch),
// 2 = LDS atomics with 8 loads in flight
template <int MODE>
__global__ __launch_bounds__(1024) void k_hist_abl(const uint16_t* __restrict__ sites, int64_t npx,
                                                   uint32_t* __restrict__ sink) {
  __shared__ uint32_t bins[32768];
  const int tid = threadIdx.x;
  for (int i = tid; i < 32768; i += 1024) bins[i] = 0;
  __syncthreads();
  const uint4* src = reinterpret_cast<const uint4*>(sites + blockIdx.x * npx);
  const int64_t n16 = npx >> 3;
  uint32_t acc = 0;
  constexpr int U = MODE == 2 ? 8 : 4;
  for (int64_t i = tid; i < n16; i += U * 1024) {
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = (i + k * 1024 < n16) ? src[i + k * 1024] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (MODE == 0) {
          acc += (w[j] & 0xFFFF) + (w[j] >> 16);
        } else {
          atomicAdd(&bins[(w[j] & 0xFFFF) & 32767], 1u);
          atomicAdd(&bins[(w[j] >> 16) & 32767], 1u);
        }
      }
    }
  }
  __syncthreads();
  if (MODE != 0) acc = bins[tid];
  if (acc == 0x12345678u) sink[0] = acc;
}

struct Timer {
  hipEvent_t a, b;
  Timer() {
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
  }
  void start() { CK(hipEventRecord(a, 0)); }
  float stop() {
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
  }
};

int main(int argc, char** argv) {
  const int64_t S = argc > 1 ? atoll(argv[1]) : 512;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  const int H = 2160, W = 2560;
  const int64_t npx = (int64_t)H * W;
  const double site_gb = npx * 2 / 1e9;
  uint16_t *sites, *out;
  CK(hipMalloc(&sites, S * npx * 2));
  CK(hipMalloc(&out, S * npx * 2));
  uint32_t* sink;
  CK(hipMalloc(&sink, 64));
  launch_synth(sites, S, H, W, 12345, 0, 0, 0);
  CK(hipDeviceSynchronize());
  Timer t;
  auto report = [&](const char* name, float ms, double gb) {
    printf("%-28s %9.3f ms  %8.1f GB/s  %6.1f%% of 8 TB/s  %9.0f sites/s\n", name, ms, gb / (ms * 1e-3),
           100.0 * gb / (ms * 1e-3) / 8000.0, S / (ms * 1e-3));
  };
  const int64_t n16 = S * npx / 8;
  for (int r = 0; r < reps; ++r) {
    t.start();
    hipLaunchKernelGGL(k_stream_read, dim3(8192), dim3(256), 0, 0, (const uint4*)sites, n16, sink);
    report("stream_read (2 B/px)", t.stop(), S * site_gb);
    t.start();
    hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, (const uint4*)sites, (uint4*)out, n16);
    report("copy (4 B/px)", t.stop(), 2 * S * site_gb);
  }
  for (int r = 0; r < reps; ++r) {
    t.start();
    hipLaunchKernelGGL((k_copy_u<4, false>), dim3(8192), dim3(256), 0, 0, (const uint4*)sites, (uint4*)out, n16);
    report("copy u4", t.stop(), 2 * S * site_gb);
    t.start();
    hipLaunchKernelGGL((k_copy_u<4, true>), dim3(8192), dim3(256), 0, 0, (const uint4*)sites, (uint4*)out, n16);
    report("copy u4 nt-store", t.stop(), 2 * S * site_gb);
    t.start();
    hipLaunchKernelGGL((k_copy_u<1, true>), dim3(8192), dim3(256), 0, 0, (const uint4*)sites, (uint4*)out, n16);
    report("copy u1 nt-store", t.stop(), 2 * S * site_gb);
    t.start();
    hipLaunchKernelGGL((k_copy_u<4, false>), dim3(2048), dim3(256), 0, 0, (const uint4*)sites, (uint4*)out, n16);
    report("copy u4 grid2048", t.stop(), 2 * S * site_gb);
    const int64_t ng = npx / 8;
    t.start();
    hipLaunchKernelGGL(k_copy_pm<false>, dim3((unsigned)cdiv(ng, 256)), dim3(256), 0, 0, (const uint4*)sites, (uint4*)out, ng, S);
    report("copy pixel-major", t.stop(), 2 * S * site_gb);
    t.start();
    hipLaunchKernelGGL(k_copy_pm<true>, dim3((unsigned)cdiv(ng, 256)), dim3(256), 0, 0, (const uint4*)sites, (uint4*)out, ng, S);
    report("copy pixel-major nt", t.stop(), 2 * S * site_gb);
  }

  if (getenv("MB_COPY")) {
    const int64_t site16 = npx / 8;
    for (int r = 0; r < reps; ++r) {
      t.start();
      hipLaunchKernelGGL((k_read_blk<4>), dim3((unsigned)cdiv(n16, site16)), dim3(1024), 0, 0, (const uint4*)sites, site16, n16, sink);
      report("read blk site u4", t.stop(), S * site_gb);
      t.start();
      hipLaunchKernelGGL((k_read_blk<4>), dim3((unsigned)cdiv(n16, site16 / 16)), dim3(1024), 0, 0, (const uint4*)sites, site16 / 16, n16, sink);
      report("read blk site/16 u4", t.stop(), S * site_gb);
      t.start();
      hipLaunchKernelGGL((k_copy_blk<4, false>), dim3((unsigned)cdiv(n16, site16)), dim3(1024), 0, 0, (const uint4*)sites, (uint4*)out, site16, n16);
      report("copy blk site u4", t.stop(), 2 * S * site_gb);
      t.start();
      hipLaunchKernelGGL((k_copy_blk<4, true>), dim3((unsigned)cdiv(n16, site16)), dim3(1024), 0, 0, (const uint4*)sites, (uint4*)out, site16, n16);
      report("copy blk site u4 nt", t.stop(), 2 * S * site_gb);
      t.start();
      hipLaunchKernelGGL((k_copy_blk<2, true>), dim3((unsigned)cdiv(n16, site16)), dim3(1024), 0, 0, (const uint4*)sites, (uint4*)out, site16, n16);
      report("copy blk site u2 nt", t.stop(), 2 * S * site_gb);
      t.start();
      hipLaunchKernelGGL((k_copy_blk<8, true>), dim3((unsigned)cdiv(n16, site16)), dim3(1024), 0, 0, (const uint4*)sites, (uint4*)out, site16, n16);
      report("copy blk site u8 nt", t.stop(), 2 * S * site_gb);
      t.start();
      hipLaunchKernelGGL((k_copy_blk<4, true>), dim3((unsigned)cdiv(n16, site16 / 16)), dim3(1024), 0, 0, (const uint4*)sites, (uint4*)out, site16 / 16, n16);
      report("copy blk site/16 u4 nt", t.stop(), 2 * S * site_gb);
      t.start();
      hipLaunchKernelGGL((k_copy_blk<4, true>), dim3((unsigned)cdiv(n16, 65536)), dim3(1024), 0, 0, (const uint4*)sites, (uint4*)out, 65536, n16);
      report("copy blk 1MB u4 nt", t.stop(), 2 * S * site_gb);
      t.start();
      hipLaunchKernelGGL((k_copy_blk<4, false>), dim3((unsigned)cdiv(n16, 65536)), dim3(1024), 0, 0, (const uint4*)sites, (uint4*)out, 65536, n16);
      report("copy blk 1MB u4", t.stop(), 2 * S * site_gb);
    }
    double *pm, *pq, *rn2, *lut2;
    CK(hipMalloc(&pm, 16 * npx * 8));
    CK(hipMalloc(&pq, 16 * npx * 8));
    CK(hipMalloc(&rn2, S * 8));
    CK(hipMalloc(&lut2, 65536 * 8));
    CK(hipMemset(rn2, 0, S * 8));
    CK(hipMemset(lut2, 0, 65536 * 8));
    for (int r = 0; r < reps; ++r) {
      for (int c : {1, 2, 4, 8, 16}) {
        t.start();
        hipLaunchKernelGGL(k_wf_split, dim3((unsigned)cdiv(npx / 8, 256), c), dim3(256), 0, 0, sites, npx, S, rn2, pm, pq, lut2);
        char nm[64];
        snprintf(nm, sizeof nm, "welford split %d", c);
        report(nm, t.stop(), S * site_gb);
      }
    }
  }
  // Infinity-cache probe: re-read a buffer that fits (128 MB) vs one that doesn't
  for (int64_t mb : {64, 128, 200, 512, 4096}) {
    const int64_t n = mb * (1 << 20) / 16;
    if (n > n16) break;
    hipLaunchKernelGGL(k_stream_read, dim3(8192), dim3(256), 0, 0, (const uint4*)sites, n, sink);
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
      t.start();
      hipLaunchKernelGGL(k_stream_read, dim3(8192), dim3(256), 0, 0, (const uint4*)sites, n, sink);
      best = std::min(best, t.stop());
    }
    printf("re-read %5ld MB: %8.1f GB/s\n", (long)mb, n * 16 / (best * 1e-3) / 1e9);
  }
  // welford (production)
  double *mean, *m2, *lut, *rn;
  CK(hipMalloc(&rn, S * 8));
  CK(hipMalloc(&mean, npx * 8));
  CK(hipMalloc(&m2, npx * 8));
  CK(hipMalloc(&lut, 65536 * 8));
  std::vector<double> hl(65536);
  for (int v = 0; v < 65536; ++v) hl[v] = v ? log10((double)v) : 0.0;
  CK(hipMemcpy(lut, hl.data(), 65536 * 8, hipMemcpyHostToDevice));
  double* wpart;
  CK(hipMalloc(&wpart, 8 * npx * 8));
  for (int split = 0; split < 2; ++split) {
    for (int r = 0; r < reps; ++r) {
      CK(hipMemset(mean, 0, npx * 8));
      CK(hipMemset(m2, 0, npx * 8));
      t.start();
      launch_welford(sites, npx, S, 0, rn, mean, m2, lut, 1, split ? wpart : nullptr,
                     split ? (size_t)8 * npx : 0, 0);
      report(split ? "welford (prod, site parts)" : "welford (one part)", t.stop(), S * site_gb);
    }
  }

  {  // non-temporal site loads A/B (one part, same grid as production's parts)
    const int64_t ng = npx >> 3;
    const int64_t per = cdiv(S, 3);
    const dim3 grid((unsigned)cdiv(ng, 256), 3);
    WfMerge mg{1.0 / S, 1.0, 0.0, 1};
    for (int v = 0; v < 2; ++v)
      for (int r = 0; r < reps; ++r) {
        t.start();
        if (v)
          hipLaunchKernelGGL((k_welford_vec8<true, true>), grid, dim3(256), 0, 0, sites, npx, S, per,
                             mg, mean, m2, lut, wpart);
        else
          hipLaunchKernelGGL((k_welford_vec8<true, false>), grid, dim3(256), 0, 0, sites, npx, S,
                             per, mg, mean, m2, lut, wpart);
        report(v ? "welford kernel 3 parts, nt loads" : "welford kernel 3 parts, plain loads",
               t.stop(), S * site_gb);
      }
  }
  if (getenv("MB_WF")) {
    const dim3 gr((unsigned)cdiv(npx / 8, 256));
    auto runw = [&](auto kern, const char* name) {
      for (int r = 0; r < reps; ++r) {
        t.start();
        hipLaunchKernelGGL(kern, gr, dim3(256), 0, 0, sites, npx, S, rn, mean, m2, lut);
        report(name, t.stop(), S * site_gb);
      }
    };
    runw(k_wf_var<4, true, 1>, "wfvar g4 rare");
    runw(k_wf_var<4, false, 1>, "wfvar g4 norare");
    runw(k_wf_var<2, true, 1>, "wfvar g2 rare");
    runw(k_wf_var<4, true, 5>, "wfvar g4 rare wps5");
    runw(k_wf_var<2, true, 6>, "wfvar g2 rare wps6");
    runw(k_wf_var<8, true, 1>, "wfvar g8 rare");
  }
  for (int r = 0; r < reps; ++r) {
    const dim3 gr((unsigned)cdiv(npx / 8, 256));
    t.start();
    hipLaunchKernelGGL(k_wf_abl<0>, gr, dim3(256), 0, 0, sites, npx, S, rn, mean, m2, lut);
    report("welford abl: full", t.stop(), S * site_gb);
    t.start();
    hipLaunchKernelGGL(k_wf_abl<1>, gr, dim3(256), 0, 0, sites, npx, S, rn, mean, m2, lut);
    report("welford abl: no LUT", t.stop(), S * site_gb);
    t.start();
    hipLaunchKernelGGL(k_wf_abl<2>, gr, dim3(256), 0, 0, sites, npx, S, rn, mean, m2, lut);
    report("welford abl: LUT+sum", t.stop(), S * site_gb);
    t.start();
    hipLaunchKernelGGL(k_wf_abl<3>, gr, dim3(256), 0, 0, sites, npx, S, rn, mean, m2, lut);
    report("welford abl: loads only", t.stop(), S * site_gb);
  }
  // hist ablations
  for (int r = 0; r < reps; ++r) {
    t.start();
    hipLaunchKernelGGL(k_hist_abl<0>, dim3(S), dim3(1024), 0, 0, sites, npx, sink);
    report("hist: loads only", t.stop(), S * site_gb);
    t.start();
    hipLaunchKernelGGL(k_hist_abl<1>, dim3(S), dim3(1024), 0, 0, sites, npx, sink);
    report("hist: lds atomics", t.stop(), S * site_gb);
    t.start();
    hipLaunchKernelGGL(k_hist_abl<2>, dim3(S), dim3(1024), 0, 0, sites, npx, sink);
    report("hist: lds atomics, 8 ld", t.stop(), S * site_gb);
  }
  // hist production
  const int Q = 100000;
  uint32_t* hist_hi;
  CK(hipMalloc(&hist_hi, S * kHiBins * 4));
  CK(hipMemset(hist_hi, 0, S * kHiBins * 4));
  int32_t *qlo, *qhi;
  CK(hipMalloc(&qlo, Q * 4));
  CK(hipMalloc(&qhi, Q * 4));
  std::vector<int32_t> lo(Q), hi(Q);
  for (int i = 0; i < Q; ++i) {
    const double vi = (double)(npx - 1) * ((100.0 * i / (Q - 1)) / 100.0);
    lo[i] = (int32_t)vi;
    hi[i] = std::min<int64_t>(lo[i] + 1, npx - 1);
  }
  CK(hipMemcpy(qlo, lo.data(), Q * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(qhi, hi.data(), Q * 4, hipMemcpyHostToDevice));
  uint32_t* vlh;
  CK(hipMalloc(&vlh, S * Q * 4));
  unsigned long long* pooled;
  CK(hipMalloc(&pooled, 65536 * 8));
  int64_t* zeros;
  CK(hipMalloc(&zeros, S * 8));
  for (int r = 0; r < reps; ++r) {
    t.start();
    QPos qp{qlo, qhi, Q, (double)(Q - 1) / (npx - 1), (int32_t)(npx - 1), 1};
    launch_hist_scatter(sites, npx, S, hist_hi, qp, vlh, pooled, zeros, nullptr, 0);
    report("hist (prod)", t.stop(), S * site_gb);
  }
  // correct (production) with dummy stats
  float4* coef;
  float2 *clut, *mconst;
  double* sums;
  CK(hipMalloc(&coef, npx * 16));
  CK(hipMalloc(&clut, 65536 * 8));
  CK(hipMalloc(&mconst, 8));
  CK(hipMalloc(&sums, 16));
  launch_finalize(mean, m2, S, npx, nullptr, m2, 0);
  launch_build_corr_lut(clut, 1, -10.0, 0);
  std::vector<double> hs = {1.0 * npx, 2.5 * npx};
  CK(hipMemcpy(sums, hs.data(), 16, hipMemcpyHostToDevice));
  launch_coeffs(mean, m2, sums, npx, coef, mconst, 0);
  for (int r = 0; r < reps; ++r) {
    t.start();
    launch_correct_u16(sites, out, npx, S, coef, clut, mconst, 1, -1, -1, 0);
    report("correct (prod)", t.stop(), 2 * S * site_gb);
  }
  // illuminati chain (correct -> align -> clip -> scale u8), 3 B/px
  if (!getenv("MB_NO_CHAIN")) {
    float2* clin;
    float4* mc2;
    float2* c2;
    uint8_t* o8;
    tmh_window* dw;
    CK(hipMalloc(&clin, npx * 8));
    CK(hipMalloc(&c2, npx * 8));
    CK(hipMalloc(&mc2, 16));
    CK(hipMalloc(&o8, S * npx));
    CK(hipMalloc(&dw, S * sizeof(tmh_window)));
    launch_coeffs2(mean, m2, sums, npx, 1, -10.0, c2, mc2, clin, 0);
    auto run_chain = [&](int shift_mode, int lo, int hi, const char* name) {
      std::vector<tmh_window> w(S);
      for (int64_t i = 0; i < S; ++i) {
        int dy = shift_mode ? (int)(i % 7) - 3 : 0, dx = shift_mode ? (int)(i % 9) - 4 : 0;
        if (shift_mode == 2) dx = 0;             // row shifts only: aligned destinations
        if (shift_mode == 3) dy = 0;             // column shifts only
        // residues 3,3,4,4 (bottom, top, right, left) as align_window computes them
        w[i].src_r0 = 3 - dy; w[i].src_c0 = 4 - dx; w[i].dst_r0 = 3; w[i].dst_c0 = 4;
        w[i].rows = H - 6; w[i].cols = W - 8;
      }
      CK(hipMemcpy(dw, w.data(), S * sizeof(tmh_window), hipMemcpyHostToDevice));
      for (int r = 0; r < reps; ++r) {
        t.start();
        launch_chain_u8(sites, o8, H, W, S, clin, mc2, 1, dw, lo, hi, 0);
        report(name, t.stop(), 1.5 * S * site_gb);
      }
    };
    run_chain(1, 110, 4000, "chain: shifts, LUT");
    run_chain(0, 110, 4000, "chain: no shift, LUT");
    run_chain(1, 110, 40000, "chain: shifts, f64 scale");
    run_chain(2, 110, 4000, "chain: row shifts only");
    run_chain(3, 110, 4000, "chain: col shifts only");
    CK(hipFree(clin)); CK(hipFree(c2)); CK(hipFree(mc2)); CK(hipFree(o8)); CK(hipFree(dw));
  }
  // fused correct+hist ablations (persistent, 1 WG per CU)
  {
    int n_cu = 0;
    CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
    float2* coef2;
    float4* mconst2;
    uint32_t* hist;
    int* queues;
    unsigned long long* rmask;
    CK(hipMalloc(&rmask, S * 8));
    CK(hipMemset(rmask, 0, S * 8));
    CK(hipMalloc(&coef2, npx * 8));
    CK(hipMalloc(&mconst2, 16));
    CK(hipMalloc(&hist, S * kBins * 4));
    CK(hipMalloc(&queues, 64));
    CK(hipMemset(hist, 0, S * kBins * 4));
    launch_coeffs2(mean, m2, sums, npx, 1, -10.0, coef2, mconst2, nullptr, 0);
    const int bpx = getenv("MB_BANDS") ? atoi(getenv("MB_BANDS")) : 2;
    auto run = [&](auto kern, int nt, const char* name) {
      for (int r = 0; r < reps; ++r) {
        CK(hipMemset(queues, 0, 64));
        t.start();
        hipLaunchKernelGGL(kern, dim3(n_cu * (1024 / nt)), dim3(nt), 0, 0, sites, out, npx, S, (const float4*)coef2,
                           mconst2, -1, -1, hist, rmask, queues, bpx);
        report(name, t.stop(), 2 * S * site_gb);
      }
    };
    run(k_correct_hist<true, false, 2, 0, 1024, 32768>, 1024, "fused spu2 t1024: full");
    run(k_correct_hist<true, false, 4, 0, 1024, 32768>, 1024, "fused spu4 t1024: full");
    run(k_correct_hist<true, false, 2, 0, 512, 16384>, 512, "fused spu2 t512: full");
    run(k_correct_hist<true, false, 4, 0, 512, 16384>, 512, "fused spu4 t512: full");
    run(k_correct_hist<true, false, 8, 0, 1024, 32768>, 1024, "fused spu8 t1024: full");
    run(k_correct_hist<true, false, 8, 3, 1024, 32768>, 1024, "fused spu8 t1024: math only");
    run(k_correct_hist<true, false, 4, 0, 256, 8192>, 256, "fused spu4 t256: full");
    run(k_correct_hist<true, false, 8, 0, 512, 32768>, 512, "fused spu8 t512 lds128k: full");
    run(k_correct_hist<true, false, 8, 3, 512, 32768>, 512, "fused spu8 t512 lds128k: math only");
    run(k_correct_hist<true, false, 4, 8, 1024, 32768>, 1024, "fused spu4 t1024: no flush");
    run(k_correct_hist<true, false, 4, 1, 1024, 32768>, 1024, "fused spu4 t1024: no hist");
    run(k_correct_hist<true, false, 4, 2, 1024, 32768>, 1024, "fused spu4 t1024: const coef");
    run(k_correct_hist<true, false, 4, 3, 1024, 32768>, 1024, "fused spu4 t1024: math only");
    run(k_correct_hist<true, false, 4, 3, 512, 16384>, 512, "fused spu4 t512: math only");
    run(k_correct_hist<true, false, 2, 3, 512, 16384>, 512, "fused spu2 t512: math only");
    // one clean fused pass -> exact per-site histograms in `hist`
    CK(hipMemset(hist, 0, S * kBins * 4));
    CK(hipMemset(queues, 0, 64));
    hipLaunchKernelGGL((k_correct_hist<true, false, 4, 0, 512, 16384>), dim3(n_cu * 2), dim3(512), 0, 0,
                       sites, out, npx, S, (const float4*)coef2, mconst2, -1, -1, hist, rmask, queues, bpx);
    QPos qa{qlo, qhi, Q, (double)(Q - 1) / (npx - 1), (int32_t)(npx - 1), 1};
    unsigned long long* parts;
    CK(hipMalloc(&parts, 16 * 65536 * 8));
    CK(hipMemset(parts, 0, 16 * 65536 * 8));
    auto runf = [&](auto kern, const char* name) {
      for (int r = 0; r < reps; ++r) {
        t.start();
        hipLaunchKernelGGL(kern, dim3((unsigned)S), dim3(1024), 0, 0, hist, rmask, 4, qa, vlh, parts, 16,
                           zeros, (uint32_t*)nullptr);
        report(name, t.stop(), 0.0);
      }
    };
    runf(k_hist_finalize<8>, "hfin: full (no reset)");
    runf(k_hist_finalize<9>, "hfin: no output");
    runf(k_hist_finalize<13>, "hfin: scan only");
    runf(k_hist_finalize<12>, "hfin: no pooled");
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
