// Microbenchmark (development tool, not shipped): HBM copy / write / read
// ceilings on this box by buffer size and kernel shape -- is the fused
// correct pass's ~5.4 TB/s (uint16 in -> out, 38 GB each way) the copy
// ceiling of the part, or of the shape?
// Usage: mb_copy [reps=5]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));        \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// one element per thread (BabelStream shape)
__global__ __launch_bounds__(256) void k_copy1(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                               int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) c[i] = a[i];
}

// grid-stride, U loads in flight; NT = nontemporal stores
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copyu(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                               int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + k * stride < n) v[k] = a[i + k * stride];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + k * stride < n) {
        if (NT)
          __builtin_nontemporal_store(v[k], c + i + k * stride);
        else
          c[i + k * stride] = v[k];
      }
  }
}

// each workgroup copies one contiguous chunk of CH elements (4 in flight)
template <int CH>
__global__ __launch_bounds__(256) void k_copy_chunk(const u32x4* __restrict__ a,
                                                    u32x4* __restrict__ c, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * CH;
  for (int64_t j = threadIdx.x; j < CH; j += 4 * 256) {
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (j + k * 256 < CH && base + j + k * 256 < n) v[k] = a[base + j + k * 256];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (j + k * 256 < CH && base + j + k * 256 < n) c[base + j + k * 256] = v[k];
  }
}

__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ c, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    c[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, int64_t n,
                                              unsigned* sink) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  unsigned acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const u32x4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x1234567u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  const size_t max_bytes = (size_t)38 << 30;
  u32x4 *a, *c;
  unsigned* sink;
  CK(hipMalloc(&a, max_bytes));
  CK(hipMalloc(&c, max_bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 1, max_bytes));
  CK(hipMemset(c, 0, max_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](const char* name, double bytes, auto&& launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("%-36s %9.3f ms  %7.1f GB/s  %5.1f%%\n", name, best, bytes / (best * 1e-3) / 1e9,
           100.0 * bytes / (best * 1e-3) / 8e12);
  };
  for (size_t gb : {1, 4, 16, 38}) {
    const int64_t n = (int64_t)((gb << 30) / 16);
    char nm[80];
    printf("-- %zu GB per buffer\n", gb);
    snprintf(nm, sizeof nm, "read grid8192");
    time(nm, (double)n * 16, [&] { hipLaunchKernelGGL(k_read, dim3(8192), dim3(256), 0, 0, a, n, sink); });
    snprintf(nm, sizeof nm, "write grid8192");
    time(nm, (double)n * 16, [&] { hipLaunchKernelGGL(k_write, dim3(8192), dim3(256), 0, 0, c, n); });
    snprintf(nm, sizeof nm, "copy1 (one per thread)");
    time(nm, 2.0 * n * 16, [&] {
      hipLaunchKernelGGL(k_copy1, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, a, c, n);
    });
    for (int g : {2048, 8192, 32768}) {
      snprintf(nm, sizeof nm, "copyu4 grid%d", g);
      time(nm, 2.0 * n * 16, [&] { hipLaunchKernelGGL((k_copyu<4, false>), dim3(g), dim3(256), 0, 0, a, c, n); });
      snprintf(nm, sizeof nm, "copyu4 nt grid%d", g);
      time(nm, 2.0 * n * 16, [&] { hipLaunchKernelGGL((k_copyu<4, true>), dim3(g), dim3(256), 0, 0, a, c, n); });
    }
    snprintf(nm, sizeof nm, "copyu8 grid8192");
    time(nm, 2.0 * n * 16, [&] { hipLaunchKernelGGL((k_copyu<8, false>), dim3(8192), dim3(256), 0, 0, a, c, n); });
    snprintf(nm, sizeof nm, "copy chunk 64 KB");
    time(nm, 2.0 * n * 16, [&] {
      hipLaunchKernelGGL((k_copy_chunk<4096>), dim3((unsigned)((n + 4095) / 4096)), dim3(256), 0, 0, a, c, n);
    });
    snprintf(nm, sizeof nm, "copy chunk 1 MB");
    time(nm, 2.0 * n * 16, [&] {
      hipLaunchKernelGGL((k_copy_chunk<65536>), dim3((unsigned)((n + 65535) / 65536)), dim3(256), 0, 0, a, c, n);
    });
    snprintf(nm, sizeof nm, "hipMemcpyAsync D2D");
    time(nm, 2.0 * n * 16, [&] { CK(hipMemcpyAsync(c, a, (size_t)n * 16, hipMemcpyDeviceToDevice, 0)); });
  }
  printf("done\n");
  return 0;
}
