// Apply-step kernels for gfx950 (MI355X).
//
// Reference: tmlib/image.py
//   287-311 / 1172-1193  smoothing (mahotas.gaussian_filter, 'reflect', f64)
//   599-631              ChannelImage._correct_illumination
//   570-597              ChannelImage.clip
//
// Correction is pixel-major: each thread owns 8 pixels, loads their
// per-pixel coefficients once and walks the sites, so HBM sees 2 B/px read
// + 2 B/px written per site.  The log10 of the input comes from an f32
// hi/lo LUT (|err| ~1e-14) staged in LDS, the affine step runs in f32
// keeping (L - mean) exact to ~1e-7, and 10**t is one v_exp_f32: |rel err|
// < 1e-6, i.e. < 0.07 DN at 65535 (tolerance +-1 DN).
#include <cstdlib>

#include "common.h"

namespace tmh {

// ---------------------------------------------------------------------------
// separable Gaussian, 'reflect' border (d c b a | a b c d | d c b a)
// ---------------------------------------------------------------------------

__device__ __forceinline__ int reflect_idx(int i, int n) {
  if ((unsigned)i < (unsigned)n) return i;  // inside: no integer division
  if (n == 1) return 0;
  const int p = 2 * n;
  i %= p;
  if (i < 0) i += p;
  return (i < n) ? i : p - 1 - i;
}

// Planes of one launch (gridDim.z = the planes): the mean and std planes of
// one job -- or of several jobs (tmh_job_planes_multi_device: a rank's
// channels) -- are smoothed by the same launches, instead of a launch per
// plane (each ~0.035 ms at 2160x2560: launch and tail dominated).  A plane
// with sq[z] != 0 is read through the statistics finalize (stats.py:94-112):
// sqrt(in / sq) -- in = M2, sq = n - 1 -- or NaN (sq < 0: n < 2), the same
// expression k_finalize evaluates, so the std plane is never written out.
struct SmPlanes {
  const double* in[kMaxPlanes];
  double* out[kMaxPlanes];
  double sq[kMaxPlanes];
  // optional (k_smooth_2d): the plane's partial sums per coefficient tile
  // (kSumTH x kSumTW outputs, tile = blockIdx.y * gridDim.x + blockIdx.x) and
  // its smallest positive value per tile -- the coefficient step's np.mean
  // and refinement bound without a pass of their own (k_tile_sums computes
  // the same partials from a plane in memory)
  double* psum[kMaxPlanes];
  double* pmin[kMaxPlanes];
};

__device__ __forceinline__ double block_sum256(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  return red[0];
}

__device__ __forceinline__ double block_min256(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = fmin(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  return red[0];
}

// A thread's column of a coefficient tile, summed in row order, then the
// tile's 256 threads (idle ones adding 0) in a fixed tree: the partition and
// order k_smooth_2d's fused sums and k_tile_sums share, so the sums do not
// depend on which of the two made them.
__device__ __forceinline__ void tile_partials(double sum, double mn, double* psum, double* pmin,
                                              double* red) {
  const int tile = blockIdx.y * gridDim.x + blockIdx.x;
  const double t = block_sum256(sum, red);
  if (threadIdx.x == 0) psum[tile] = t;
  if (pmin) {
    __syncthreads();
    const double m = block_min256(mn, red);
    if (threadIdx.x == 0) pmin[tile] = m;
  }
}

__device__ __forceinline__ double sm_in(const SmPlanes& pl, const double* __restrict__ in, int64_t i) {
  const double v = in[i];
  const double q = pl.sq[blockIdx.z];
  if (q == 0.0) return v;
  return q > 0.0 ? sqrt(v / q) : __builtin_nan("");
}

// axis 0 (rows of the plane vary): out[y][x] = sum_j w[j] in[refl(y+j-r)][x]
__global__ __launch_bounds__(256) void k_smooth_axis0(const SmPlanes pl, int H, int W,
                                                      const double* __restrict__ w, int r) {
  const double* __restrict__ in = pl.in[blockIdx.z];
  double* __restrict__ out = pl.out[blockIdx.z];
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= W) return;
  double acc = 0.0;
  for (int j = -r; j <= r; ++j) acc = fma(w[j + r], in[(int64_t)reflect_idx(y + j, H) * W + x], acc);
  out[(int64_t)y * W + x] = acc;
}

// axis 0 for a compile-time radius: each thread produces T consecutive rows
// of one column from T + 2R loads (register accumulators, taps added in the
// same order as k_smooth_axis0 -> bit-identical results), instead of 2R + 1
// loads per output.
template <int T, int R>
__global__ __launch_bounds__(256) void k_smooth_axis0_strip(const SmPlanes pl, int H, int W,
                                                            const double* __restrict__ w) {
  const double* __restrict__ in = pl.in[blockIdx.z];
  double* __restrict__ out = pl.out[blockIdx.z];
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y0 = blockIdx.y * T;
  if (x >= W) return;
  double acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = 0.0;
#pragma unroll
  for (int u = 0; u < T + 2 * R; ++u) {
    const double v = in[(int64_t)reflect_idx(y0 + u - R, H) * W + x];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int k = u - t;
      if (k >= 0 && k <= 2 * R) acc[t] = fma(w[k], v, acc[t]);
    }
  }
#pragma unroll
  for (int t = 0; t < T; ++t)
    if (y0 + t < H) out[(int64_t)(y0 + t) * W + x] = acc[t];
}

// axis 1 (along a row), row segment + halo staged in LDS
constexpr int kSmTile = 256;
constexpr int kSmMaxR = 128;
__global__ __launch_bounds__(256) void k_smooth_axis1(const SmPlanes pl, int H, int W,
                                                      const double* __restrict__ w, int r) {
  __shared__ double tile[kSmTile + 2 * kSmMaxR];
  const double* __restrict__ in = pl.in[blockIdx.z];
  double* __restrict__ out = pl.out[blockIdx.z];
  const int x0 = blockIdx.x * kSmTile;
  const int y = blockIdx.y;
  const double* row = in + (int64_t)y * W;
  for (int i = threadIdx.x; i < kSmTile + 2 * r; i += 256) tile[i] = row[reflect_idx(x0 - r + i, W)];
  __syncthreads();
  const int x = x0 + threadIdx.x;
  if (x >= W) return;
  double acc = 0.0;
  for (int j = 0; j <= 2 * r; ++j) acc = fma(w[j], tile[threadIdx.x + j], acc);
  out[(int64_t)y * W + x] = acc;
}

__global__ __launch_bounds__(256) void k_smooth_axis1_wide(const SmPlanes pl, int H, int W,
                                                           const double* __restrict__ w, int r) {
  const double* __restrict__ in = pl.in[blockIdx.z];
  double* __restrict__ out = pl.out[blockIdx.z];
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= W) return;
  const double* row = in + (int64_t)y * W;
  double acc = 0.0;
  for (int j = -r; j <= r; ++j) acc = fma(w[j + r], row[reflect_idx(x + j, W)], acc);
  out[(int64_t)y * W + x] = acc;
}

// Both axes in one pass for a compile-time radius: a workgroup owns TW =
// 256 - 2R output columns x TH rows; its 256 threads first run the axis-0
// taps down the tile's TW + 2R columns (halo columns are the reflected
// columns, as the axis-1 pass reads them), keep the TH x 256 results in LDS,
// then each thread runs the axis-1 taps along one output column.  Every tap
// is added in the same order as k_smooth_axis0(_strip) then k_smooth_axis1,
// so the result is bit-identical, without the intermediate plane's HBM
// write and read (2 x 44 MB per plane at 2160 x 2560).
template <int TH, int R>
__global__ __launch_bounds__(256) void k_smooth_2d(const SmPlanes pl, int H, int W,
                                                   const double* __restrict__ w) {
  constexpr int CW = 256, TW = CW - 2 * R;
  __shared__ double vt[TH][CW];
  const double* __restrict__ in = pl.in[blockIdx.z];
  double* __restrict__ out = pl.out[blockIdx.z];
  const int x0 = blockIdx.x * TW, y0 = blockIdx.y * TH;
  {
    const int x = reflect_idx(x0 - R + (int)threadIdx.x, W);
    double acc[TH];
#pragma unroll
    for (int t = 0; t < TH; ++t) acc[t] = 0.0;
#pragma unroll
    for (int u = 0; u < TH + 2 * R; ++u) {
      const double v = sm_in(pl, in, (int64_t)reflect_idx(y0 + u - R, H) * W + x);
#pragma unroll
      for (int t = 0; t < TH; ++t) {
        const int k = u - t;
        if (k >= 0 && k <= 2 * R) acc[t] = fma(w[k], v, acc[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < TH; ++t) vt[t][threadIdx.x] = acc[t];
  }
  __syncthreads();
  const int x = x0 + (int)threadIdx.x;
  double sum = 0.0, mn = __builtin_inf();
  if ((int)threadIdx.x < TW && x < W) {
#pragma unroll 4
    for (int t = 0; t < TH; ++t) {
      if (y0 + t >= H) break;
      double a = 0.0;
#pragma unroll
      for (int j = 0; j <= 2 * R; ++j) a = fma(w[j], vt[t][threadIdx.x + j], a);
      out[(int64_t)(y0 + t) * W + x] = a;
      sum += a;
      if (a > 0.0 && a < mn) mn = a;  // NaN fails both; +inf never below mn
    }
  }
  double* ps = pl.psum[blockIdx.z];
  if (ps) {  // uniform per workgroup
    __shared__ double red[256];
    tile_partials(sum, mn, ps, pl.pmin[blockIdx.z], red);
  }
}

static_assert(kSumTW == 256 - 2 * 20, "coefficient tiles are the sigma-5 smoothing's tiles");

// block_sum256's tree (red[i] += red[i + o], o = 128, 64, ..., 1) and the
// matching min, with two LDS exchanges and in-wave shuffles instead of eight
// barriers each: the same additions of the same operands, so the same sum.
// red: 2 x (128 + 64) doubles.  Thread 0 writes the tile's partials.
__device__ __forceinline__ void tile_partials_wave(double s, double m, double* red, double* ps,
                                                   double* pm) {
  const int t = threadIdx.x;
  double* rs1 = red;
  double* rm1 = red + 128;
  double* rs2 = red + 256;
  double* rm2 = red + 320;
  if (t >= 128) {
    rs1[t - 128] = s;
    rm1[t - 128] = m;
  }
  __syncthreads();
  if (t < 128) {
    s += rs1[t];
    m = fmin(m, rm1[t]);
    if (t >= 64) {
      rs2[t - 64] = s;
      rm2[t - 64] = m;
    }
  }
  __syncthreads();
  if (t < 64) {
    s += rs2[t];
    m = fmin(m, rm2[t]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s += __shfl_down(s, o, 64);
      m = fmin(m, __shfl_down(m, o, 64));
    }
    if (t == 0) {
      *ps = s;
      if (pm) *pm = m;
    }
  }
}

template <bool STD>
__device__ __forceinline__ double sm_xf(double v, double q) {
  if (!STD) return v;
  return q > 0.0 ? sqrt(v / q) : __builtin_nan("");
}

// Both axes in one pass, axis 1 register-blocked (sigma 5, R = 20): the
// production form.  A workgroup owns one coefficient tile, kSumTW output
// columns x 16 rows.  Axis 0 as k_smooth_2d: each of the 256 threads runs one
// input column (the tile's 216 plus the reflected 2R halo) over the tile's
// 16 + 2R input rows into 16 register accumulators.  Axis 1 differs: a thread
// runs 18 consecutive outputs of one row from 58 LDS reads (k_smooth_2d: one
// output from 41 reads, a serial chain of 41 FMAs per output), i.e. 18
// independent chains; the outputs go back through LDS for coalesced stores
// and the tile's column sums.  Every output's taps are added in k_smooth_2d's
// order (axis 0 k = 0..2R, then axis 1 j = 0..2R, each from 0.0) and the tile
// partials in tile_partials' tree: bit-identical outputs and partials
// (tools/mb/mb_smooth.hip checks both; 0.086-0.091 vs 0.147 ms for a job's
// two planes, 0.32 vs 0.60 ms for four jobs' eight,
// profiles/r6/mb_smooth_r6s4.txt).  Rows rolled through the registers from one
// 16-row chunk to the next (each input row read once per workgroup) measured
// slower at every depth (56 live accumulators: half the occupancy;
// mb_smooth_variants_r6s3.txt).
constexpr int kVtS = 257;  // LDS row stride in doubles (odd: rows land on different banks)
template <bool STD>
__device__ __forceinline__ void smooth2d_blk_body(const double* __restrict__ in,
                                                  double* __restrict__ out, double q,
                                                  const double* __restrict__ w, double* ps,
                                                  double* pm, int H, int W, double* vt,
                                                  double* red) {
  constexpr int R = 20, K = 2 * R + 1, CH = kSumTH, OX = 18, NG = kSumTW / OX;
  static_assert(CH == 16 && NG * OX == kSumTW && NG * CH <= 256, "axis-1 work split");
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * kSumTW, y0 = blockIdx.y * CH;
  // One reflection: -n <= i < 2n.  The launcher asks H, W > R, so i >= -R
  // holds; indices past n - 1 + R feed no output inside the plane (the
  // tile's last threads and rows on narrow or short planes), so they are
  // clamped there first -- every load stays inside the plane.
  auto refl = [](int i, int n) {
    i = i < n + R - 1 ? i : n + R - 1;
    return i < 0 ? -1 - i : (i >= n ? 2 * n - 1 - i : i);
  };
  const double* __restrict__ col = in + refl(x0 - R + tid, W);
  // the taps are symmetric bit for bit (abi.hip gaussian_taps writes w[R + i]
  // and w[R - i] from one value): 21 scalar registers' worth, not 41
  double wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[k <= R ? k : 2 * R - k];
  {  // axis 0: input rows y0 - R .. y0 + CH + R - 1 of this column
    double acc[CH], v[CH + 2 * R];
#pragma unroll
    for (int t = 0; t < CH; ++t) acc[t] = 0.0;
#pragma unroll
    for (int u = 0; u < CH + 2 * R; ++u) v[u] = col[(int64_t)refl(y0 - R + u, H) * W];
#pragma unroll
    for (int u = 0; u < CH + 2 * R; ++u) {
      const double x = sm_xf<STD>(v[u], q);
#pragma unroll
      for (int t = 0; t < CH; ++t)
        if (u - t >= 0 && u - t <= 2 * R) acc[t] = fma(wk[u - t], x, acc[t]);
    }
#pragma unroll
    for (int r = 0; r < CH; ++r) vt[r * kVtS + tid] = acc[r];
  }
  __syncthreads();
  const int r1 = tid & (CH - 1), g1 = tid >> 4;  // axis-1 item: row r1, columns 18 g1 ..
  const bool act1 = g1 < NG;
  double o[OX];
  if (act1) {
    const double* row = vt + r1 * kVtS + OX * g1;
#pragma unroll
    for (int i = 0; i < OX; ++i) o[i] = 0.0;
#pragma unroll
    for (int j = 0; j < OX + 2 * R; ++j) {
      const double v = row[j];
#pragma unroll
      for (int i = (j > 2 * R ? j - 2 * R : 0); i <= (j < OX - 1 ? j : OX - 1); ++i)
        o[i] = fma(wk[j - i], v, o[i]);
    }
  }
  __syncthreads();
  if (act1) {
#pragma unroll
    for (int i = 0; i < OX; ++i) vt[r1 * kVtS + OX * g1 + i] = o[i];
  }
  __syncthreads();
  const int x = x0 + tid;
  double sum = 0.0, mn = __builtin_inf();
  if (tid < kSumTW && x < W) {
#pragma unroll
    for (int r = 0; r < CH; ++r) {
      if (y0 + r >= H) break;
      const double a = vt[r * kVtS + tid];
      out[(int64_t)(y0 + r) * W + x] = a;
      sum += a;
      if (a > 0.0 && a < mn) mn = a;  // NaN fails both; +inf never below mn
    }
  }
  if (ps) {  // uniform per workgroup
    const int tile = blockIdx.y * gridDim.x + blockIdx.x;
    tile_partials_wave(sum, mn, red, ps + tile, pm ? pm + tile : nullptr);
  }
}

__global__ __launch_bounds__(256) void k_smooth_2d_blk(const SmPlanes pl, int H, int W,
                                                       const double* __restrict__ w) {
  __shared__ double vt[kSumTH * kVtS];
  __shared__ double red[384];
  const int z = blockIdx.z;
  const double q = pl.sq[z];
  if (q == 0.0)
    smooth2d_blk_body<false>(pl.in[z], pl.out[z], q, w, pl.psum[z], pl.pmin[z], H, W, vt, red);
  else
    smooth2d_blk_body<true>(pl.in[z], pl.out[z], q, w, pl.psum[z], pl.pmin[z], H, W, vt, red);
}

// The coefficient tiles' partial sums (and smallest positive values) of
// planes in memory, in k_smooth_2d's partition and order.
__global__ __launch_bounds__(256) void k_tile_sums(const SmPlanes pl, int H, int W) {
  __shared__ double red[256];
  const double* __restrict__ in = pl.in[blockIdx.z];
  const int x = blockIdx.x * kSumTW + (int)threadIdx.x, y0 = blockIdx.y * kSumTH;
  double sum = 0.0, mn = __builtin_inf();
  if ((int)threadIdx.x < kSumTW && x < W) {
    for (int t = 0; t < kSumTH; ++t) {
      if (y0 + t >= H) break;
      const double a = in[(int64_t)(y0 + t) * W + x];
      sum += a;
      if (a > 0.0 && a < mn) mn = a;
    }
  }
  tile_partials(sum, mn, pl.psum[blockIdx.z], pl.pmin[blockIdx.z], red);
}

int coef_tiles(int H, int W) { return (int)(cdiv(W, kSumTW) * cdiv(H, kSumTH)); }

// np planes: in[k] -> tmp[k] (axis 0) -> out[k] (axis 1); sq[k] != 0: plane k
// is read as a finalized std (SmPlanes), which needs the one-pass form
// (radius 20) -- the caller finalizes into a plane of its own otherwise
void launch_smooth_planes(const double* const* in, double* const* out, double* const* tmp,
                          const double* sq, int np, int H, int W, const double* d_w, int radius,
                          hipStream_t s, double* const* psum, double* const* pmin) {
  ProfScope prof("smooth", s);
  if (np <= 0) return;
  auto planes = [&](const double* const* a, double* const* b) {
    SmPlanes p{};
    for (int k = 0; k < np; ++k) {
      p.in[k] = a[k];
      p.out[k] = b[k];
      p.sq[k] = sq ? sq[k] : 0.0;
    }
    return p;
  };
  if (radius == 20 && W >= 2 * radius + 1 && !getenv("TMH_SMOOTH_2PASS")) {
    // sigma = 5, the reference's default (image.py:1172): one pass, both
    // axes, the coefficient tiles' sums as the outputs are written
    SmPlanes a = planes(in, out);
    for (int k = 0; k < np && psum; ++k) {
      a.psum[k] = psum[k];
      a.pmin[k] = pmin ? pmin[k] : nullptr;
    }
    // k_smooth_2d_blk needs H, W > R (one reflection); TMH_SMOOTH_FORM=0 picks
    // the round-5 form (A/B)
    static const bool blk = [] {
      const char* e = getenv("TMH_SMOOTH_FORM");
      return !(e && atoi(e) == 0);
    }();
    const dim3 g((unsigned)cdiv(W, kSumTW), (unsigned)cdiv(H, kSumTH), (unsigned)np);
    if (blk && H > 20)
      hipLaunchKernelGGL(k_smooth_2d_blk, g, dim3(256), 0, s, a, H, W, d_w);
    else
      hipLaunchKernelGGL((k_smooth_2d<kSumTH, 20>), g, dim3(256), 0, s, a, H, W, d_w);
    TMH_HIP(hipGetLastError());
    return;
  }
  for (int k = 0; k < np; ++k)
    if (sq && sq[k] != 0.0) throw Error{TMH_EINVAL, "finalize-on-read smoothing needs sigma 5"};
  const SmPlanes a0 = planes(in, tmp), a1 = planes(tmp, out);
  const dim3 grid((unsigned)cdiv(W, 256), (unsigned)H, (unsigned)np);
  if (radius == 20) {  // sigma = 5, the reference's default (image.py:1172)
    // 16 rows per thread: 1,350 workgroups per plane at 2160x2560 (8 / 32 measured slower)
    const dim3 g2((unsigned)cdiv(W, 256), (unsigned)cdiv(H, 16), (unsigned)np);
    hipLaunchKernelGGL((k_smooth_axis0_strip<16, 20>), g2, dim3(256), 0, s, a0, H, W, d_w);
  } else {
    hipLaunchKernelGGL(k_smooth_axis0, grid, dim3(256), 0, s, a0, H, W, d_w, radius);
  }
  if (radius <= kSmMaxR)
    hipLaunchKernelGGL(k_smooth_axis1, dim3((unsigned)cdiv(W, kSmTile), (unsigned)H, (unsigned)np),
                       dim3(256), 0, s, a1, H, W, d_w, radius);
  else
    hipLaunchKernelGGL(k_smooth_axis1_wide, grid, dim3(256), 0, s, a1, H, W, d_w, radius);
  if (psum) launch_tile_sums(out, psum, pmin, np, H, W, s);
  TMH_HIP(hipGetLastError());
}

void launch_tile_sums(const double* const* x, double* const* psum, double* const* pmin, int np,
                      int H, int W, hipStream_t s) {
  if (np <= 0) return;
  SmPlanes p{};
  for (int k = 0; k < np; ++k) {
    p.in[k] = x[k];
    p.psum[k] = psum[k];
    p.pmin[k] = pmin ? pmin[k] : nullptr;
  }
  const dim3 g((unsigned)cdiv(W, kSumTW), (unsigned)cdiv(H, kSumTH), (unsigned)np);
  hipLaunchKernelGGL(k_tile_sums, g, dim3(256), 0, s, p, H, W);
  TMH_HIP(hipGetLastError());
}

void launch_smooth(const double* in, double* out, double* tmp, int H, int W, const double* d_w,
                   int radius, hipStream_t s) {
  launch_smooth_planes(&in, &out, &tmp, nullptr, 1, H, W, d_w, radius, s, nullptr, nullptr);
}

void launch_smooth2(const double* in0, const double* in1, double* out0, double* out1,
                    double* tmp0, double* tmp1, int H, int W, const double* d_w, int radius,
                    hipStream_t s) {
  const double* in[2] = {in0, in1};
  double* out[2] = {out0, out1};
  double* tmp[2] = {tmp0, tmp1};
  launch_smooth_planes(in, out, tmp, nullptr, 2, H, W, d_w, radius, s, nullptr, nullptr);
}

// ---------------------------------------------------------------------------
// correction coefficients
// ---------------------------------------------------------------------------

// LUT of the correct-path transform of every uint16 value as an f32 hi/lo pair:
// log: v==0 -> log10(1e-10) (image.py:624-626), else log10(v); no log: v.
__global__ void k_build_corr_lut(float2* __restrict__ lut, int log_transform, double zero_log10) {
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v >= kBins) return;
  double L = (double)v;
  if (log_transform) L = (v == 0) ? zero_log10 : log10((double)v);
  const float hi = (float)L;
  lut[v] = make_float2(hi, (float)(L - (double)hi));
}

void launch_build_corr_lut(float2* lut, int log_transform, double zero_log10, hipStream_t s) {
  hipLaunchKernelGGL(k_build_corr_lut, dim3(kBins / 256), dim3(256), 0, s, lut, log_transform,
                     zero_log10);
  TMH_HIP(hipGetLastError());
}

constexpr double kLog2_10d = 3.32192809488736234787;

// Every coefficient form of one (mean, std) pair, one thread per pixel i
// (blockIdx.y = job, CoefJobs):
//   coef[i]    = (mean hi, mean lo, a = mean(std)/std, 0)      LUT path
//   coef2      = (c, a) as f32, a rounded first and c = (M - mean * a) [* log2
//                10] from it in f64 (M = np.mean(mean)), so the fused pass's
//                t2 = log2(x) * a + c is one fma; for npx % 8 == 0 pixel 8g+j
//                in plane j/2 as float4 (c_2p, c_2p+1, a_2p, a_2p+1) at g: one
//                16-B load gives a pixel pair its packed-f32 operands
//   coef_lin[i] = (mean [* log2 10], a) in pixel order (the chain's shifted
//                gathers)
//   coef64[i]  = (mean, std) in f64 (the refinement, common.h)
__global__ void k_coeffs_all(const CoefJobs J, int64_t npx) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npx) return;
  const int j = blockIdx.y;
  const double S = J.sums[j][0] / (double)npx;  // np.mean(std)
  const double mu = J.mean[j][i], sd = J.std[j][i];
  const double a = S / sd;
  const float mh = (float)mu;
  if (J.coef[j]) J.coef[j][i] = make_float4(mh, (float)(mu - (double)mh), (float)a, 0.0f);
  const double K = J.log_transform[j] ? kLog2_10d : 1.0;
  int64_t om = 2 * i, oa = 2 * i + 1;
  if ((npx & 7) == 0) {
    const int64_t g = i >> 3, jj = i & 7;
    const int64_t base = (jj >> 1) * (npx >> 1) + 4 * g + (jj & 1);
    om = base;
    oa = base + 2;
  }
  const float mu2 = (float)(mu * K), af = (float)a;
  const double M = J.sums[j][1] / (double)npx;  // np.mean(mean)
  float* coef2 = reinterpret_cast<float*>(J.coef2[j]);
  coef2[om] = (float)((M - mu * (double)af) * K);
  coef2[oa] = af;
  if (J.coef_lin[j]) J.coef_lin[j][i] = make_float2(mu2, af);
  J.coef64[j][i] = make_double2(mu, sd);
}

// The LUT path's coef and the chain's coef_lin from coef64 and the sums, for
// a corrector whose coefficient update skipped them (the fused job path needs
// only coef2 / coef64): the same values k_coeffs_all writes.
__global__ void k_coeffs_forms(const double2* __restrict__ coef64, const double* __restrict__ sums,
                               int64_t npx, int log_transform, float4* __restrict__ coef,
                               float2* __restrict__ coef_lin) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npx) return;
  const double S = sums[0] / (double)npx;
  const double2 ms = coef64[i];
  const double mu = ms.x, a = S / ms.y;
  const float mh = (float)mu;
  coef[i] = make_float4(mh, (float)(mu - (double)mh), (float)a, 0.0f);
  const double K = log_transform ? kLog2_10d : 1.0;
  coef_lin[i] = make_float2((float)(mu * K), (float)a);
}

void launch_coeffs_forms(const double2* coef64, const double* sums, int64_t npx, int log_transform,
                         float4* coef, float2* coef_lin, hipStream_t s) {
  hipLaunchKernelGGL(k_coeffs_forms, dim3((unsigned)cdiv(npx, 256)), dim3(256), 0, s, coef64, sums,
                     npx, log_transform, coef, coef_lin);
  TMH_HIP(hipGetLastError());
}

// Per job (blockIdx.x): the planes' sums from the coefficient tiles'
// partials -- sums[0] = sum(std), sums[1] = sum(mean), sums[2] = the smallest
// positive std (np.mean(std), np.mean(mean) of image.py:627; each a fixed
// order, deterministic) -- then the launch constants: mconst = (M hi, M lo,
// T, 0) (LUT path), mconst2 = (M' hi, M' lo, 10**zero_log10 as f32 (a zero
// pixel's floor), T) with M' = M [* log2 10], and the refinement constants;
// a_max = S / (smallest positive std), T rounded down to f32.
__global__ __launch_bounds__(256) void k_sums_const(const CoefJobs J, int n, int64_t npx) {
  __shared__ double red[256];
  const int j = blockIdx.x;
  const double* p = J.partial[j];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) acc += p[i];
  const double s_std = block_sum256(acc, red);
  __syncthreads();
  acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) acc += p[n + i];
  const double s_mean = block_sum256(acc, red);
  __syncthreads();
  double mn = __builtin_inf();
  for (int i = threadIdx.x; i < n; i += 256) mn = fmin(mn, p[2 * n + i]);
  const double s_min = block_min256(mn, red);
  if (threadIdx.x != 0) return;
  double* sums = J.sums[j];
  sums[0] = s_std;
  sums[1] = s_mean;
  sums[2] = s_min;
  const double S = s_std / (double)npx, M = s_mean / (double)npx;
  double am = fabs(S / s_min);  // s_min = +inf (no positive std): 0
  if (!(am <= 1.7976931348623157e308)) am = 0.0;  // S inf/NaN: every pixel is inf/NaN anyway
  const double T = 1.0 / (kRefineK1 * am + kRefineK2);
  float Tf = (float)T;
  if ((double)Tf > T) Tf = __uint_as_float(__float_as_uint(Tf) - 1u);  // T > 0: one f32 step down
  const float mh = (float)M;
  J.mconst[j][0] = make_float4(mh, (float)(M - (double)mh), Tf, 0.0f);
  const double M2 = M * (J.log_transform[j] ? kLog2_10d : 1.0);
  const float m2h = (float)M2;
  J.mconst2[j][0] = make_float4(m2h, (float)(M2 - (double)m2h), (float)exp10(J.zero_log10[j]), Tf);
  J.rc[j][0] = RefineConst{S, M, J.zero_log10[j], (double)Tf};
}

// The jobs' tile partials (unless the smoothing already wrote them), their
// sums and launch constants, then every coefficient form: one to three
// launches for all jobs.  J.partial[j] holds 3 x coef_tiles(H, W) doubles:
// std sums, mean sums, std minima.
void launch_coeffs_jobs(const CoefJobs& J, int n_jobs, int H, int W, bool partials_ready,
                        hipStream_t s) {
  if (n_jobs <= 0) return;
  const int nt = coef_tiles(H, W);
  const int64_t npx = (int64_t)H * W;
  if (!partials_ready) {
    const double* x[kMaxPlanes];
    double* ps[kMaxPlanes];
    double* pm[kMaxPlanes];
    for (int j = 0; j < n_jobs; ++j) {
      x[2 * j] = J.std[j];
      ps[2 * j] = J.partial[j];
      pm[2 * j] = J.partial[j] + 2 * nt;
      x[2 * j + 1] = J.mean[j];
      ps[2 * j + 1] = J.partial[j] + nt;
      pm[2 * j + 1] = nullptr;
    }
    launch_tile_sums(x, ps, pm, 2 * n_jobs, H, W, s);
  }
  hipLaunchKernelGGL(k_sums_const, dim3(n_jobs), dim3(256), 0, s, J, nt, npx);
  hipLaunchKernelGGL(k_coeffs_all, dim3((unsigned)cdiv(npx, 256), n_jobs), dim3(256), 0, s, J, npx);
  TMH_HIP(hipGetLastError());
}

// The f64 refinement of the pixels a correct launch flagged (FixList,
// common.h), written as the launch would (low BITS bits, clip).  If the list
// overflowed, every pixel of the launch is recomputed in f64.
template <bool LOG, typename T, int BITS>
__device__ __forceinline__ void fix_correct_body(const T* __restrict__ in, T* __restrict__ out,
                                                 int64_t npx, int64_t n_sites, const FixList& fl,
                                                 const double2* __restrict__ c64,
                                                 const RefineConst* __restrict__ rc, int clip_lo,
                                                 int clip_hi, const SiteTab& tab) {
  const unsigned int n = *fl.n;
  const bool all = n > fl.cap;
  const int64_t total = all ? n_sites * ((npx + 7) / 8) : (int64_t)n;
  if (total == 0) return;
  const RefineConst k = *rc;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    int64_t s, p0;
    uint32_t mask;
    fix_entry(fl, all, i, npx, s, p0, mask);
    const T* si = in + s * npx;
    T* so = out + s * npx;
    if (tab.in) {  // blocked layout (u16 launches only)
      const int64_t b = site_block(tab, s), o = site_in_block(tab, s) * npx;
      si = reinterpret_cast<const T*>(tab.in[b]) + o;
      so = reinterpret_cast<T*>(tab.out[b]) + o;
    }
    for (int j = 0; j < 8; ++j) {
      const int64_t p = p0 + j;
      if (!((mask >> j) & 1u) || p >= npx) continue;
      const double2 q = c64[p];
      uint32_t r =
          (uint32_t)correct_ref_f64<LOG>(si[p], q.x, q.y, k.S, k.M, k.zero_log10) &
          ((1u << BITS) - 1u);
      if (clip_lo >= 0) {
        r = r < (uint32_t)clip_lo ? (uint32_t)clip_lo : r;
        r = r > (uint32_t)clip_hi ? (uint32_t)clip_hi : r;
      }
      so[p] = (T)r;
    }
  }
}

template <bool LOG, typename T, int BITS>
__global__ __launch_bounds__(256) void k_fix_correct(const T* __restrict__ in, T* __restrict__ out,
                                                     int64_t npx, int64_t n_sites, FixList fl,
                                                     const double2* __restrict__ c64,
                                                     const RefineConst* __restrict__ rc,
                                                     int clip_lo, int clip_hi, const SiteTab tab) {
  fix_correct_body<LOG, T, BITS>(in, out, npx, n_sites, fl, c64, rc, clip_lo, clip_hi, tab);
}

// Several jobs' fixups in one launch (blockIdx.y = job, uint16 sites), each
// job's Welford wide counters reset on the way (FixJob::wide, may be null)
template <bool LOG>
__global__ __launch_bounds__(256) void k_fix_correct_jobs(const FixJobs J, int64_t npx, int clip_lo,
                                                          int clip_hi) {
  const FixJob& f = J.j[blockIdx.y];
  if (f.wide && blockIdx.x == 0 && threadIdx.x < 2) f.wide[threadIdx.x] = 0ull;
  fix_correct_body<LOG, uint16_t, 16>(f.in, f.out, npx, f.n_sites, f.fl, f.c64, f.rc, clip_lo,
                                      clip_hi, f.tab);
}

void launch_fix_correct_jobs(const FixJobs& J, int64_t npx, int log_transform, int clip_lo,
                             int clip_hi, hipStream_t s) {
  if (J.n <= 0) return;
  const dim3 grid(512, (unsigned)J.n), block(256);
  if (log_transform)
    hipLaunchKernelGGL(k_fix_correct_jobs<true>, grid, block, 0, s, J, npx, clip_lo, clip_hi);
  else
    hipLaunchKernelGGL(k_fix_correct_jobs<false>, grid, block, 0, s, J, npx, clip_lo, clip_hi);
  TMH_HIP(hipGetLastError());
}

void launch_fix_correct(const void* in, void* out, int elem_bytes, int64_t npx, int64_t n_sites,
                        const FixList& fl, const double2* coef64, const RefineConst* rc,
                        int log_transform, int clip_lo, int clip_hi, hipStream_t s,
                        const SiteTab& tab) {
  if (n_sites <= 0) return;
  const dim3 grid(512), block(256);
  TMH_CHECK(!tab.in || elem_bytes == 2, TMH_EINVAL, "blocked layouts are uint16 only");
  if (elem_bytes == 2) {
    auto i16 = static_cast<const uint16_t*>(in);
    auto o16 = static_cast<uint16_t*>(out);
    if (log_transform)
      hipLaunchKernelGGL((k_fix_correct<true, uint16_t, 16>), grid, block, 0, s, i16, o16, npx,
                         n_sites, fl, coef64, rc, clip_lo, clip_hi, tab);
    else
      hipLaunchKernelGGL((k_fix_correct<false, uint16_t, 16>), grid, block, 0, s, i16, o16, npx,
                         n_sites, fl, coef64, rc, clip_lo, clip_hi, tab);
  } else {
    auto i8 = static_cast<const uint8_t*>(in);
    auto o8 = static_cast<uint8_t*>(out);
    if (log_transform)
      hipLaunchKernelGGL((k_fix_correct<true, uint8_t, 8>), grid, block, 0, s, i8, o8, npx, n_sites,
                         fl, coef64, rc, clip_lo, clip_hi, tab);
    else
      hipLaunchKernelGGL((k_fix_correct<false, uint8_t, 8>), grid, block, 0, s, i8, o8, npx,
                         n_sites, fl, coef64, rc, clip_lo, clip_hi, tab);
  }
  TMH_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// fused correct (+ clip)
// ---------------------------------------------------------------------------

constexpr float kLog2_10 = 3.32192809488736234787f;

// correct-path log10 of a value >= kLutLds as an f32 hi/lo pair (out of line:
// rare for microscopy data, and a global LUT load in the pixel loop would make
// the compiler wait for the prefetched sites)
__device__ __noinline__ float2 corr_log_slow(uint32_t u) {
  const double L = log10((double)u);
  const float hi = (float)L;
  return make_float2(hi, (float)(L - (double)hi));
}

// the correction of one pixel u (pixel index p) given its log10 (hi, lo) (or
// value) L; m = mconst (M hi, M lo, T, 0)
// (site s): a result beyond the f32 error bound T = m.z is flagged for the
// f64 refinement (common.h)
template <bool LOG, int BITS>
__device__ __forceinline__ uint32_t correct_l(float Lh, float Ll, const float4 c, const float4 m,
                                              int64_t s, int64_t p, const FixList& fl,
                                              int clip_lo, int clip_hi) {
  const float d = (Lh - c.x) + (Ll - c.y);        // (img - mean)
  const float t = fmaf(d, c.z, m.x) + m.y;         // * mean(std)/std + mean(mean)
  const float o = LOG ? exp2f(t * kLog2_10) : t;   // 10 ** t
  if (__builtin_fabsf(o) >= m.z) fix_push(fl, s, p);
  // numpy float64 -> uint astype on x86: trunc to int32 (out of range/NaN ->
  // INT32_MIN), keep the low bits (image.py:631)
  const int32_t iv = (o >= -2147483648.0f && o < 2147483648.0f) ? (int32_t)o : INT32_MIN;
  uint32_t r = (uint32_t)iv & ((1u << BITS) - 1u);
  if (clip_lo >= 0) {
    r = r < (uint32_t)clip_lo ? (uint32_t)clip_lo : r;
    r = r > (uint32_t)clip_hi ? (uint32_t)clip_hi : r;
  }
  return r;
}

template <bool LOG, int BITS>
__device__ __forceinline__ uint32_t correct1(uint32_t u, const float4 c, const float2* slut,
                                             const float4 m, int64_t s, int64_t p,
                                             const FixList& fl, int clip_lo, int clip_hi) {
  float2 l;
  if (LOG) {
    l = slut[u < (uint32_t)kLutLds ? u : 0u];
    if (u >= (uint32_t)kLutLds) l = corr_log_slow(u);
  } else {
    l = make_float2((float)u, 0.0f);
  }
  return correct_l<LOG, BITS>(l.x, l.y, c, m, s, p, fl, clip_lo, clip_hi);
}

// streamed-once site data: non-temporal loads / stores
typedef unsigned int u32x4a_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt_u4(const uint4* p) {
  const u32x4a_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4a_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt_u4(uint4* p, uint4 v) {
  const u32x4a_t w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4a_t*>(p));
}

constexpr int kCorrThreads = 256;
constexpr int kCorrGroup = 4;  // sites per pipeline stage (two stages in flight)

template <bool LOG>
__global__ __launch_bounds__(kCorrThreads) void k_correct_u16_vec8(
    const uint16_t* __restrict__ in, uint16_t* __restrict__ out, int64_t npx, int64_t n_sites,
    const float4* __restrict__ coef, const float2* __restrict__ lut,
    const float4* __restrict__ mconst, FixList fl, int clip_lo, int clip_hi) {
  __shared__ float2 slut[kLutLds];
  if (LOG)
    for (int i = threadIdx.x; i < kLutLds; i += kCorrThreads) slut[i] = lut[i];
  __syncthreads();
  const int64_t ngroups = npx >> 3;
  const int64_t g = (int64_t)blockIdx.x * kCorrThreads + threadIdx.x;
  if (g >= ngroups) return;
  const float4 m = mconst[0];
  float4 c[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) c[k] = coef[g * 8 + k];
  const uint4* src = reinterpret_cast<const uint4*>(in) + g;
  uint4* dst = reinterpret_cast<uint4*>(out) + g;
  auto one = [&](const uint4 v, const int64_t site) -> uint4 {
    const uint32_t u[8] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16,
                           v.z & 0xFFFFu, v.z >> 16, v.w & 0xFFFFu, v.w >> 16};
    float2 l[8];
    if (LOG) {
      // one branch per 8 pixels: LDS LUT for all, then patch the rare big ones
      uint32_t mx = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        mx = u[k] > mx ? u[k] : mx;
        l[k] = slut[u[k] < (uint32_t)kLutLds ? u[k] : 0u];
      }
      if (mx >= (uint32_t)kLutLds) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (u[k] >= (uint32_t)kLutLds) l[k] = corr_log_slow(u[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) l[k] = make_float2((float)u[k], 0.0f);
    }
    uint32_t o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      o[k] = correct_l<LOG, 16>(l[k].x, l[k].y, c[k], m, site, g * 8 + k, fl, clip_lo, clip_hi);
    return make_uint4(o[0] | (o[1] << 16), o[2] | (o[3] << 16), o[4] | (o[5] << 16),
                      o[6] | (o[7] << 16));
  };
  const int64_t last = n_sites - 1;
  uint4 cur[kCorrGroup], nxt[kCorrGroup];
#pragma unroll
  for (int k = 0; k < kCorrGroup; ++k) cur[k] = ld_nt_u4(src + (k < last ? k : last) * ngroups);
  for (int64_t s = 0; s < n_sites; s += kCorrGroup) {
#pragma unroll
    for (int k = 0; k < kCorrGroup; ++k) {
      const int64_t t = s + kCorrGroup + k;
      nxt[k] = ld_nt_u4(src + (t < last ? t : last) * ngroups);
    }
#pragma unroll
    for (int k = 0; k < kCorrGroup; ++k)
      if (s + k < n_sites) st_nt_u4(dst + (s + k) * ngroups, one(cur[k], s + k));
#pragma unroll
    for (int k = 0; k < kCorrGroup; ++k) cur[k] = nxt[k];
  }
}

template <bool LOG, typename T, int BITS>
__global__ __launch_bounds__(kCorrThreads) void k_correct_scalar(
    const T* __restrict__ in, T* __restrict__ out, int64_t npx, int64_t n_sites,
    const float4* __restrict__ coef, const float2* __restrict__ lut,
    const float4* __restrict__ mconst, FixList fl, int clip_lo, int clip_hi) {
  __shared__ float2 slut[kLutLds];
  if (LOG)
    for (int i = threadIdx.x; i < kLutLds; i += kCorrThreads) slut[i] = lut[i];
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * kCorrThreads + threadIdx.x;
  if (p >= npx) return;
  const float4 m = mconst[0];
  const float4 c = coef[p];
  for (int64_t s = 0; s < n_sites; ++s)
    out[s * npx + p] =
        (T)correct1<LOG, BITS>(in[s * npx + p], c, slut, m, s, p, fl, clip_lo, clip_hi);
}

void launch_correct_u16(const uint16_t* in, uint16_t* out, int64_t npx, int64_t n_sites,
                        const float4* coef, const float2* lut, const float4* mconst,
                        const FixList& fl, int log_transform, int clip_lo, int clip_hi,
                        hipStream_t s) {
  if (n_sites <= 0) return;
  ProfScope prof("correct", s);
  const bool vec = (npx & 7) == 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (vec) {
    const dim3 grid((unsigned)cdiv(npx >> 3, kCorrThreads));
    if (log_transform)
      hipLaunchKernelGGL(k_correct_u16_vec8<true>, grid, dim3(kCorrThreads), 0, s, in, out, npx,
                         n_sites, coef, lut, mconst, fl, clip_lo, clip_hi);
    else
      hipLaunchKernelGGL(k_correct_u16_vec8<false>, grid, dim3(kCorrThreads), 0, s, in, out, npx,
                         n_sites, coef, lut, mconst, fl, clip_lo, clip_hi);
  } else {
    const dim3 grid((unsigned)cdiv(npx, kCorrThreads));
    if (log_transform)
      hipLaunchKernelGGL((k_correct_scalar<true, uint16_t, 16>), grid, dim3(kCorrThreads), 0, s, in,
                         out, npx, n_sites, coef, lut, mconst, fl, clip_lo, clip_hi);
    else
      hipLaunchKernelGGL((k_correct_scalar<false, uint16_t, 16>), grid, dim3(kCorrThreads), 0, s,
                         in, out, npx, n_sites, coef, lut, mconst, fl, clip_lo, clip_hi);
  }
  TMH_HIP(hipGetLastError());
}

void launch_correct_u8(const uint8_t* in, uint8_t* out, int64_t npx, int64_t n_sites,
                       const float4* coef, const float2* lut, const float4* mconst,
                       const FixList& fl, int log_transform, int clip_lo, int clip_hi,
                       hipStream_t s) {
  if (n_sites <= 0) return;
  ProfScope prof("correct_u8", s);
  const dim3 grid((unsigned)cdiv(npx, kCorrThreads));
  if (log_transform)
    hipLaunchKernelGGL((k_correct_scalar<true, uint8_t, 8>), grid, dim3(kCorrThreads), 0, s, in,
                       out, npx, n_sites, coef, lut, mconst, fl, clip_lo, clip_hi);
  else
    hipLaunchKernelGGL((k_correct_scalar<false, uint8_t, 8>), grid, dim3(kCorrThreads), 0, s, in,
                       out, npx, n_sites, coef, lut, mconst, fl, clip_lo, clip_hi);
  TMH_HIP(hipGetLastError());
}

__global__ void k_clip_u16(const uint16_t* __restrict__ in, uint16_t* __restrict__ out, int64_t n,
                           int lo, int hi) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int v = in[i];
  v = v < lo ? lo : v;
  v = v > hi ? hi : v;
  out[i] = (uint16_t)v;
}

void launch_clip_u16(const uint16_t* in, uint16_t* out, int64_t n, int lo, int hi, hipStream_t s) {
  hipLaunchKernelGGL(k_clip_u16, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, in, out, n, lo, hi);
  TMH_HIP(hipGetLastError());
}

}  // namespace tmh
