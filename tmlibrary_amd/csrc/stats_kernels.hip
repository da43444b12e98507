// Illumination-statistics kernels for gfx950 (MI355X).
//
// Reference: tmlib/workflow/corilla/stats.py:64-121 (OnlineStatistics.update,
// var/mean/std/percentiles).  Two passes over the resident site images:
//
//   k_welford_*      pixel-major: each thread owns 8 pixels and walks the
//                    sites in order, keeping (mean, M2) in f64 registers
//                    (stats.py:89-92) — state is read/written once per launch,
//                    so HBM traffic is the 2 B/px of the sites.  log10 comes
//                    from the host-numpy LUT (stats.py:79-85), first 4096
//                    entries staged in LDS.
//   k_hist_scatter   site-major: one 1024-thread workgroup per site builds the
//                    exact 65,536-bin histogram (bins < 32768 in LDS, the rest
//                    with global atomics into a zero-maintained per-site
//                    slab), scans it, and scatters the value at every
//                    percentile's previous/next sorted position (np.percentile
//                    linear, stats.py:76) as u16.
//   k_pct_acc        thread per quantile: folds each site's interpolated
//                    percentile into the f64 accumulator in SITE ORDER, without
//                    FMA, so the sum is bit-identical to the reference's
//                    sequential `_percentiles +=`.
#include <algorithm>

#include "common.h"
#include "hist_tail.h"

namespace tmh {

// ---------------------------------------------------------------------------
// Welford
// ---------------------------------------------------------------------------

// x = stats transform of one pixel value.  LOG: np.log10 with 0 -> 0 from the
// host-numpy LUT for values < kWfLut (LDS, bit-identical to numpy).  Larger
// values (bright sites) use the same LUT on their top bits:
//   u = 16 a + r,  a = u >> 4 in [256, 4096),
//   log10(u) = log10(a) + log10(16) + log1p(t) / ln 10,  t = r / (16 a) < 1/256.
// INV 0 / 1: 1/(16 a) in f64 (Newton step / LDS table) and a 5-term f64 series
// (truncation below 3e-16 absolute), ~12 f64 ops.  INV 2 (production): the
// small term log1p(t) / ln 10 <= 1.6e-3 in f32 -- rcp, three-term series
// (truncation <= t^4/4 / ln 10 < 5e-11), f32 rounding < 2e-10 absolute -- then
// one f64 add: a value >= 4,096 is within 3e-10 of numpy's log10 (1e-10
// relative, against the 1e-6 bar on mean and std), at a fraction of the
// VALU cost -- bright sites (most values >= 4,096) made the f64 form's pass
// VALU-bound (17.7 ms vs 6.0 on standard sites, profiles/r2/ab_finalize_sr_r2y.jsonl).
constexpr double kInvLn10 = 0.43429448190325182765;
constexpr double kLog10_16 = 1.2041199826559247809;
constexpr int kWfInvScalar = 2;  // rare-value form of the odd-shape (per-pixel) pass
// 1/(16 a): INV = 1 from the LDS table, INV = 0 by v_rcp_f32 plus one f64
// Newton step (relative error ~1e-14: t then carries < 1e-17 absolute)
template <int INV>
__device__ __forceinline__ double recip16(uint32_t a, const double* sinv) {
  if (INV == 1) return sinv[a];
  const double d = (double)(a << 4);
  const double r0 = (double)__builtin_amdgcn_rcpf((float)(a << 4));
  return fma(r0, fma(-d, r0, 1.0), r0);
}
template <int INV>
__device__ __forceinline__ double log10_big(uint32_t u, const double* slut, const double* sinv) {
  const uint32_t a = u >> 4;
  if (INV == 2) {
    constexpr float c1 = (float)kInvLn10, c2 = (float)(-0.5 * kInvLn10),
                    c3 = (float)(kInvLn10 / 3.0);
    const float t = (float)(u & 15u) * __builtin_amdgcn_rcpf((float)(a << 4));
    const float c = t * __builtin_fmaf(t, __builtin_fmaf(t, c3, c2), c1);
    return slut[a] + (kLog10_16 + (double)c);
  }
  const double t = (double)(u & 15u) * recip16<INV>(a, sinv);
  const double series =
      t * (kInvLn10 +
           t * (-0.5 * kInvLn10 + t * (kInvLn10 / 3.0 + t * (-0.25 * kInvLn10 + t * (0.2 * kInvLn10)))));
  return (slut[a] + kLog10_16) + series;
}

// LUT entries staged in LDS: the 4,096 values below 2^12 (32 KB) and, with
// INV = 1, the 4,096 reciprocals 1/(16 a) (32 KB more), so a site's 8 pixels
// need the rare path exactly when one of their 16-bit words has a bit >= 12
// set (one OR/AND over the four packed words).
constexpr int kWfLut = 4096;

// The fill issues up to 8 of a thread's loads before its LDS stores (one L2
// round trip per 8 entries instead of one per entry: a 1,024-thread bright
// workgroup, alone on its CU, waits out its whole fill).
template <int INV, int LUTN = kWfLut>
__device__ __forceinline__ void fill_wf_tables(const double* __restrict__ lut, double* slut,
                                               double* sinv, int nt) {
  constexpr int U = 8;
  for (int i0 = threadIdx.x; i0 < LUTN; i0 += U * nt) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * nt;
      v[u] = i < LUTN ? lut[i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * nt;
      if (i < LUTN) slut[i] = v[u];
      if (INV == 1 && i < kWfLut) sinv[i] = i ? 1.0 / (16.0 * (double)i) : 0.0;
    }
  }
}

// Bright sites: the host LUT's first kWfLutBright entries (160 KB of LDS less
// the pass's two counters and reciprocal slot, one 1,024-thread workgroup per
// CU) -- values below it take the exact table like the standard pass's values
// below 4,096, and only the bright pixels above it the log10_big path (with
// 4,096 entries most bright pixels took it: the pass was VALU-bound, 11.3-12.3
// ms against 6.0 on standard sites).  A wave runs that path for a pixel slot
// when any of its 64 lanes needs it: at 16,384 entries (round 3-6) ~1.5% of the
// bright values did, i.e. most slots of most waves; at 20,472 about half as
// many.  Not a power of two: indices are clamped (v_pk_min_u16), not masked.
constexpr int kWfLutBright = 20472;
constexpr int kWfThreadsBright = 1024;

template <bool LOG>
__device__ __forceinline__ double xform(uint32_t u, const double* slut) {
  if (!LOG) return (double)u;
  double x = slut[u & (uint32_t)(kWfLut - 1)];
  if (u >= (uint32_t)kWfLut) x = log10_big<kWfInvScalar>(u, slut, nullptr);
  return x;
}

__device__ __forceinline__ void welford1(double x, double rn, double& mu, double& m2) {
  const double d = x - mu;
  mu = fma(d, rn, mu);          // mean + delta / n
  m2 = fma(d, x - mu, m2);      // M2 + delta * (x - mean_new)
}

// Production shape of the vec8 pass: threads per workgroup and the
// reciprocal source (tools/mb/mb_welford.hip compares the four shapes on
// standard and bright sites; profiles/r2/mb_welford_shapes_*.txt).
constexpr int kWfThreads = 256;
constexpr int kWfInv = 2;
constexpr int kWfScalarThreads = 256;
constexpr int kWfGroup = 2;  // sites per pipeline stage (two stages in flight)
constexpr int kWfMaxParts = 4;

// 1/n for the sites of one launch (uniform per site: read with scalar loads)
__global__ void k_rn_table(double* __restrict__ rn, int64_t n0, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) rn[i] = 1.0 / (double)(n0 + i + 1);
}

// LDS byte offsets of a packed word's two table entries (8-B entries): the
// caller brings both halves' indices into the table (one v_and with the
// 4,096-entry mask, or one v_pk_min_u16 clamp for the bright table), then one
// SDWA shift per half selects and scales it -- three VALU ops per word where
// the compiler's shift-and-mask pairs took four (the standard pass issues 2
// such ops per pixel beside its 3 f64 ops).  `three` is a VGPR holding 3 (an
// SDWA shift amount is a register operand).
__device__ __forceinline__ void lut_offsets(uint32_t m, uint32_t three, uint32_t& lo,
                                            uint32_t& hi) {
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
      "src1_sel:WORD_0"
      : "=v"(lo)
      : "v"(three), "v"(m));
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
      "src1_sel:WORD_1"
      : "=v"(hi)
      : "v"(three), "v"(m));
}
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t w, uint32_t c2) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2_t, w),
                                                                __builtin_bit_cast(u16x2_t, c2)));
}
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2_t, a),
                                                                __builtin_bit_cast(u16x2_t, b)));
}
__device__ __forceinline__ double lds_at(const double* base, uint32_t byte_off) {
  return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + byte_off);
}

// Stats transform of eight pixels: LDS LUT gather of each value's table
// index (the low 12 bits, or for the bright table the value clamped to it),
// then -- only when a word has a value past the table -- those slots
// recomputed with log10_big (wc counts the groups with a value >= 4,096, xc
// those with a value >= 16,384: diagnostics since round 5).  The inner loop is VALU-issue bound (3 f64 ops per
// pixel), so the integer work per pixel is kept to the gather address.
template <bool LOG, int INV, int LUTN = kWfLut>
__device__ __forceinline__ void xform8(const uint4 v, const double* slut, const double* sinv,
                                       double (&x)[8], uint32_t& wc, uint32_t& xc) {
  const uint32_t u[8] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16,
                         v.z & 0xFFFFu, v.z >> 16, v.w & 0xFFFFu, v.w >> 16};
  const uint32_t any = v.x | v.y | v.z | v.w;
  const bool wide = (any & 0xF000F000u) != 0;
  constexpr bool kPow2 = (LUTN & (LUTN - 1)) == 0;
  constexpr uint32_t kIdx = LUTN - 1;
  if (LOG) {  // the table entries of every pixel (index masked or clamped)
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
    const uint32_t three = 3u;
    constexpr uint32_t kIdx2 = kIdx * 0x00010001u;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      uint32_t lo, hi;
      lut_offsets(kPow2 ? wd[p] & kIdx2 : pk_min_u16(wd[p], kIdx2), three, lo, hi);
      x[2 * p] = lds_at(slut, lo);
      x[2 * p + 1] = lds_at(slut, hi);
    }
  }
  if (LOG && LUTN == kWfLutBright) {  // exact below kWfLutBright
    wc += wide ? 1u : 0u;
    xc += (any & 0xC000C000u) ? 1u : 0u;  // a value >= 16,384
    const uint32_t mx = pk_max_u16(pk_max_u16(v.x, v.y), pk_max_u16(v.z, v.w));
    if ((mx & 0xFFFFu) > kIdx || (mx >> 16) > kIdx) {  // a value beyond the table
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (u[k] > kIdx) x[k] = log10_big<INV>(u[k], slut, sinv);
    }
  } else if (LOG) {
    if (wide) {
      ++wc;
      xc += (any & 0xC000C000u) ? 1u : 0u;  // a value >= 16,384
      // per pixel: on standard data ~7 % of wave-steps have one lane with
      // one such value, and a branch-free pass over all eight cost 0.2 ms
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (u[k] > kIdx) x[k] = log10_big<INV>(u[k], slut, sinv);
    }
  } else {
    wc += wide ? 1u : 0u;
    xc += (any & 0xC000C000u) ? 1u : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = (double)u[k];
  }
}

// Launch-level constants of the shifted-sum pass (host-computed f64)
struct WfMerge {
  double inv_nl;  // 1 / sites of this launch
  double w_new;   // nl / (n0 + nl)
  double w_cross; // n0 * nl / (n0 + nl)
  int first;      // n0 == 0: no previous state to merge
};

// Welford over the launch's sites as shifted sums (stats.py:86-92 restated):
// per pixel K = x of the launch's first site, S1 = sum(x - K), S2 = sum((x - K)^2)
// -- three f64 ops per pixel-site instead of Welford's four, no 1/n per site.
// At the end (mean_l, M2_l) = (K + S1/nl, S2 - S1^2/nl) is merged into the
// running (mean, M2) with Chan's pairwise formula.  K is one of the samples,
// so (mean_l - K)^2 <= (nl - 1) var and the cancellation in S2 - S1^2/nl
// costs at most a factor nl of f64 precision (~1e-12 relative at 3456 sites,
// against the 1e-6 bar); a constant pixel gives exactly 0.
// blockIdx.y = site part: part p covers sites [p * per, min((p + 1) * per, n));
// with more than one part each writes its (mean_l, M2_l) to `part` planes and
// k_wf_merge_parts folds them in part order.
// site loads: NTL = non-temporal (streamed once, kept out of L2's way)
template <bool NTL>
__device__ __forceinline__ uint4 ld_site(const uint4* p) {
  if (!NTL) return *p;
  typedef unsigned int u32x4w_t __attribute__((ext_vector_type(4)));
  const u32x4w_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4w_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// A site pointer read from a block table is a generic pointer: the compiler
// then emits flat loads (slower than global loads, and counted on both the
// vector-memory and LDS counters).  Site loads through a global-address-space
// pointer stay global_load.
typedef unsigned int u32x4g_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4g_t gsite_t;
__device__ __forceinline__ gsite_t* to_global(const void* p) { return (gsite_t*)p; }
template <bool NTL>
__device__ __forceinline__ uint4 ld_site(gsite_t* p) {
  const u32x4g_t v = NTL ? __builtin_nontemporal_load(p) : *p;
  return make_uint4(v.x, v.y, v.z, v.w);
}

// BLK: blocked site layout (common.h SiteTab): site t of the launch is site
// t & (2^shift - 1) of block t >> shift; the block base is re-read (one scalar
// load) only when the walk enters a new block.
template <bool LOG, bool NTL, int NT, int INV, bool BLK = false, int G = kWfGroup,
          int LUTN = kWfLut>
__global__ __launch_bounds__(NT) void k_welford_vec8(
    const uint16_t* __restrict__ sites, int64_t npx, int64_t n_total, int64_t per,
    const WfMerge mg, double* __restrict__ mean, double* __restrict__ m2,
    const double* __restrict__ lut, double* __restrict__ part,
    unsigned long long* __restrict__ wide, const SiteTab tab) {
  const int parts = (int)gridDim.y;
  __shared__ double slut[LUTN], sinv[INV == 1 ? kWfLut : 1];
  __shared__ uint32_t wide_sh[2];
  if (LOG) fill_wf_tables<INV, LUTN>(lut, slut, sinv, NT);
  if (threadIdx.x < 2) wide_sh[threadIdx.x] = 0u;
  __syncthreads();
  const int64_t ngroups = npx >> 3;
  const int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (g >= ngroups) return;

  const int64_t s_begin = (int64_t)blockIdx.y * per;
  const int64_t n_sites = n_total - s_begin < per ? n_total - s_begin : per;
  const uint4* src = reinterpret_cast<const uint4*>(sites) + s_begin * ngroups + g;
  const int64_t last = n_sites - 1;
  // BLK: a running (uniform) site base -- t advances by 0 or 1 per call; one
  // scalar load of the next block's base where the walk enters a block
  int64_t bt = 0;
  const uint4* bbase = nullptr;
  if (BLK)
    bbase = reinterpret_cast<const uint4*>(tab.in[s_begin >> tab.shift]) +
            (s_begin & ((1ll << tab.shift) - 1)) * ngroups;
  auto site = [&](int64_t t) -> gsite_t* {  // t: site of this part, non-decreasing
    if (!BLK) return to_global(src + t * ngroups);
    if (t != bt) {
      bt = t;
      const int64_t gs = s_begin + t;
      if (gs & ((1ll << tab.shift) - 1))
        bbase += ngroups;
      else
        bbase = reinterpret_cast<const uint4*>(tab.in[gs >> tab.shift]);
    }
    return to_global(bbase + g);
  };
  // two-stage pipeline: the next group's loads are in flight while the
  // current group is folded in (tail loads clamp to the last site: harmless)
  uint4 cur[G], nxt[G];
#pragma unroll
  for (int k = 0; k < G; ++k) cur[k] = ld_site<NTL>(site(k < last ? k : last));
  double K[8], s1[8], s2[8];
  uint32_t wc = 0, xc = 0;  // this thread's groups with a value >= 4,096 / >= 16,384
  xform8<LOG, INV, LUTN>(cur[0], slut, sinv, K, wc, xc);
  wc = xc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.0;
  // 32-bit site counters: the per-site bounds test is then one scalar compare
  // (gfx9 has no 64-bit scalar less-than; an int64 test costs two VALU ops
  // per site in a VALU-issue-bound loop)
  const int ns = (int)n_sites;
  // stage of G sites starting at s: the next stage's loads are issued first;
  // two register sets used in turn (no copy of the next set into the current)
  auto fold = [&](const uint4 (&v)[G], int s) {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      if (s + k < ns) {
        double x[8];
        xform8<LOG, INV, LUTN>(v[k], slut, sinv, x, wc, xc);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const double d = x[j] - K[j];
          s1[j] += d;
          s2[j] = fma(d, d, s2[j]);
        }
      }
    }
  };
  auto issue = [&](uint4 (&v)[G], int s) {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int t = s + k;
      v[k] = ld_site<NTL>(site(t < (int)last ? t : (int)last));
    }
  };
  for (int s = 0; s < ns; s += 2 * G) {
    issue(nxt, s + G);
    fold(cur, s);
    if (s + G >= ns) break;
    issue(cur, s + 2 * G);
    fold(nxt, s + G);
  }

  if (wide) {  // one global add per counter and workgroup (thread 0's group always exists)
    if (wc) atomicAdd(&wide_sh[0], wc);
    if (xc) atomicAdd(&wide_sh[1], xc);
    __syncthreads();
    if (threadIdx.x == 0 && wide_sh[0]) atomicAdd(wide, (unsigned long long)wide_sh[0]);
    if (threadIdx.x == 0 && wide_sh[1]) atomicAdd(wide + 1, (unsigned long long)wide_sh[1]);
  }

  if (parts > 1) {  // partial (mean_l, M2_l) of this part
    const double inv = 1.0 / (double)n_sites;
    double2* pm = reinterpret_cast<double2*>(part + (2 * blockIdx.y) * npx) + g * 4;
    double2* pq = reinterpret_cast<double2*>(part + (2 * blockIdx.y + 1) * npx) + g * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int j = 2 * k + i;
        a[i] = K[j] + s1[j] * inv;
        b[i] = fmax(s2[j] - s1[j] * (s1[j] * inv), 0.0);
      }
      pm[k] = make_double2(a[0], a[1]);
      pq[k] = make_double2(b[0], b[1]);
    }
    return;
  }
  double2* om = reinterpret_cast<double2*>(mean) + g * 4;
  double2* oq = reinterpret_cast<double2*>(m2) + g * 4;
  double mu[8], q[8];
  if (!mg.first) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double2 a = om[k], b = oq[k];
      mu[2 * k] = a.x; mu[2 * k + 1] = a.y;
      q[2 * k] = b.x; q[2 * k + 1] = b.y;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const double ml = K[j] + s1[j] * mg.inv_nl;
    const double m2l = fmax(s2[j] - s1[j] * (s1[j] * mg.inv_nl), 0.0);
    if (mg.first) {
      mu[j] = ml;
      q[j] = m2l;
    } else {
      const double d = ml - mu[j];
      mu[j] = fma(d, mg.w_new, mu[j]);
      q[j] = q[j] + m2l + d * d * mg.w_cross;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    om[k] = make_double2(mu[2 * k], mu[2 * k + 1]);
    oq[k] = make_double2(q[2 * k], q[2 * k + 1]);
  }
}

struct WfParts {
  double cnt[kWfMaxParts];  // sites per part
  int n;                    // parts
};

// Fold the parts' (mean_l, M2_l) in part order (Chan's pairwise combine),
// then into the running state (n0 sites before this launch).
__global__ void k_wf_merge_parts(const double* __restrict__ part, int64_t npx, const WfParts pc,
                                 double n0, double* __restrict__ mean, double* __restrict__ m2) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npx) return;
  double na = pc.cnt[0], ma = part[i], qa = part[npx + i];
  for (int p = 1; p < pc.n; ++p) {
    const double nb = pc.cnt[p], mb = part[(2 * p) * npx + i], qb = part[(2 * p + 1) * npx + i];
    const double n = na + nb, d = mb - ma;
    ma = fma(d, nb / n, ma);
    qa = qa + qb + d * d * (na * nb / n);
    na = n;
  }
  if (n0 > 0) {
    const double n = n0 + na, d = ma - mean[i];
    mean[i] = fma(d, na / n, mean[i]);
    m2[i] = m2[i] + qa + d * d * (n0 * na / n);
  } else {
    mean[i] = ma;
    m2[i] = qa;
  }
}

// Any shape (npx % 8 != 0 leaves sites unaligned for 16-B loads): 1 px/thread.
template <bool LOG>
__global__ __launch_bounds__(kWfScalarThreads) void k_welford_scalar(
    const uint16_t* __restrict__ sites, int64_t npx, int64_t n_sites,
    const double* __restrict__ rn, double* __restrict__ mean, double* __restrict__ m2,
    const double* __restrict__ lut) {
  __shared__ double slut[kWfLut];
  if (LOG) fill_wf_tables<0>(lut, slut, nullptr, kWfScalarThreads);
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * kWfScalarThreads + threadIdx.x;
  if (p >= npx) return;
  double mu = mean[p], q = m2[p];
  for (int64_t s = 0; s < n_sites; ++s)
    welford1(xform<LOG>(sites[s * npx + p], slut), rn[s], mu, q);
  mean[p] = mu;
  m2[p] = q;
}

// Site parts for one launch.  Each thread streams every site of its part;
// splitting the sites into f parts gives f times the workgroups (shorter
// dispatch tail) for one extra pass over 16*f B/px of partial state plus a
// merge.  Measured at 2160x2560 x 3,456 sites with the issue-trimmed loop
// (tools/mb/mb_welford.hip, profiles/r2/mb_welford_r2f.txt): 1 part 5.85 ms,
// 2 parts 5.98, 3 parts 6.00, 4 parts 6.18 -- so a launch is one part unless
// forced (tmh_stats_set_option TMH_OPT_WELFORD_PARTS, for tests), where the
// split is possible.
static int welford_parts(int64_t n_sites, int64_t npx, size_t part_cap, int forced) {
  auto fits = [&](int f) {
    return f >= 1 && f <= kWfMaxParts && (f == 1 || ((size_t)2 * f * npx <= part_cap &&
                                                    n_sites >= (int64_t)f * 32));
  };
  return forced && fits(forced) ? forced : 1;
}

template <int NT, int INV, int G = kWfGroup, int LUTN = kWfLut>
static void launch_welford_vec8(const uint16_t* sites, int64_t npx, int64_t n_sites, int64_t per,
                                int f, const WfMerge& mg, double* mean, double* m2,
                                const double* lut, int log_transform, double* part,
                                unsigned long long* wide, hipStream_t s,
                                const SiteTab& tab = SiteTab{}) {
  const dim3 grid((unsigned)cdiv(npx >> 3, NT), (unsigned)f);
  // site loads are non-temporal (streamed once; regular loads measured
  // 6.60-6.75 vs 6.19-6.34 ms at job level, profiles/r1/ab_welford_ntl.txt)
#define TMH_WF(L_, B_)                                                                           \
  hipLaunchKernelGGL((k_welford_vec8<L_, true, NT, INV, B_, G, LUTN>), grid, dim3(NT), 0, s,     \
                     sites, npx, n_sites, per, mg, mean, m2, lut, part, wide, tab)
  if (tab.in) {
    if (log_transform)
      TMH_WF(true, true);
    else
      TMH_WF(false, true);
  } else {
    if (log_transform)
      TMH_WF(true, false);
    else
      TMH_WF(false, false);
  }
#undef TMH_WF
}

// Site probe of a job (tmh_stats' automatic choices, abi.hip): of kProbeGroups
// 8-pixel groups spread over the launch's first min(n, kProbeSites) sites, how
// many hold a value >= 4,096 (out[1]) and >= 16,384 (out[2]); out[0] = the
// groups sampled.  One workgroup, every load in flight at once (one DRAM
// latency).  The host reads the counts and launches only the Welford pass and
// the fused configuration they call for: no candidate launch that waits for
// LDS behind another job's kernels just to exit (round 4: the idle packed
// fused candidate averaged 1.58 ms on the corrected-pass stream,
// profiles/r4/rocprof_kernel_stats_synthetic_r4fin3.csv).
constexpr int kProbeGroups = 16384;
constexpr int kProbeSites = 64;
constexpr int kWfBrightParts = 3;
__global__ __launch_bounds__(1024) void k_site_probe(const uint16_t* __restrict__ sites,
                                                     int64_t ngroups, int n_probe,
                                                     unsigned int* __restrict__ out,
                                                     const SiteTab tab) {
  __shared__ unsigned int cnt[2];
  if (threadIdx.x < 2) cnt[threadIdx.x] = 0u;
  __syncthreads();
  // sample j: site j % n_probe, its (j / n_probe)-th of R positions spread
  // over the site
  const int R = (kProbeGroups + n_probe - 1) / n_probe;
  uint4 v[kProbeGroups / 1024];
#pragma unroll
  for (int k = 0; k < kProbeGroups / 1024; ++k) {
    const int j = (int)threadIdx.x + 1024 * k;
    const int st = j % n_probe;
    const int64_t g = (int64_t)(j / n_probe) * ngroups / R;
    const uint16_t* base =
        tab.in ? tab.in[site_block(tab, st)] + site_in_block(tab, st) * ngroups * 8
               : sites + (int64_t)st * ngroups * 8;
    v[k] = reinterpret_cast<const uint4*>(base)[g];
  }
  unsigned int w = 0u, x = 0u;
#pragma unroll
  for (int k = 0; k < kProbeGroups / 1024; ++k) {
    const uint32_t any = v[k].x | v[k].y | v[k].z | v[k].w;
    w += (any & 0xF000F000u) ? 1u : 0u;
    x += (any & 0xC000C000u) ? 1u : 0u;
  }
  if (w) atomicAdd(&cnt[0], w);
  if (x) atomicAdd(&cnt[1], x);
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = (unsigned int)kProbeGroups;
    out[1] = cnt[0];
    out[2] = cnt[1];
  }
}

void launch_site_probe(const uint16_t* sites, int64_t npx, int64_t n_sites, unsigned int* out,
                       hipStream_t s, const SiteTab& tab) {
  const int np = (int)std::min<int64_t>(n_sites, kProbeSites);
  hipLaunchKernelGGL(k_site_probe, dim3(1), dim3(1024), 0, s, sites, npx >> 3, np, out, tab);
  TMH_HIP(hipGetLastError());
}

// shape = -1: production (kWfThreads, kWfInv); 0..8: (256|512 threads) x
// (f64 Newton | f64 LDS-table reciprocal | f32 small term) x pipeline depth,
// for the microbenchmark.  bright (production shape, log transform, no forced
// split): the host's site probe found bright sites -- the 16,384-entry LUT
// pass in kWfBrightParts site parts (the log10 pass is VALU-bound there:
// three times the workgroups even the dispatch rounds, 11.3 vs 12.4 ms with
// the 4,096-entry pass, profiles/r2/mb_welford_bright_r2za.txt; the 16,384
// entries 8.0 vs 11.4 ms, profiles/r3/ab_welford_bright16k_bright_r3m.jsonl).
void launch_welford(const uint16_t* sites, int64_t npx, int64_t n_sites, int64_t n0, double* rn,
                    double* mean, double* m2, const double* lut, int log_transform,
                    double* part, size_t part_cap, int forced_parts,
                    unsigned long long* wide, int bright, hipStream_t s, int shape,
                    const SiteTab& tab) {
  if (n_sites <= 0) return;
  // (a blocked layout is checked by the caller: npx % 8 == 0, 16-B aligned blocks)
  const bool vec = tab.in || ((npx & 7) == 0 && (reinterpret_cast<uintptr_t>(sites) & 15) == 0);
  if (vec) {
    int f = part ? welford_parts(n_sites, npx, part_cap, forced_parts) : 1;
    const bool bpass = bright > 0 && part && !forced_parts && log_transform && shape < 0 &&
                       welford_parts(n_sites, npx, part_cap, kWfBrightParts) == kWfBrightParts;
    if (bpass) f = kWfBrightParts;
    const int64_t per = cdiv(n_sites, f);
    const double nl = (double)n_sites, n = (double)(n0 + n_sites);
    const WfMerge mg{1.0 / nl, nl / n, (double)n0 * nl / n, n0 == 0};
    ProfScope prof("welford", s);  // the pass (and its part merge) only
    switch (shape) {
      case 0: launch_welford_vec8<256, 0>(sites, npx, n_sites, per, f, mg, mean, m2, lut, log_transform, part, wide, s); break;
      case 1: launch_welford_vec8<256, 1>(sites, npx, n_sites, per, f, mg, mean, m2, lut, log_transform, part, wide, s); break;
      case 2: launch_welford_vec8<512, 0>(sites, npx, n_sites, per, f, mg, mean, m2, lut, log_transform, part, wide, s); break;
      case 3: launch_welford_vec8<512, 1>(sites, npx, n_sites, per, f, mg, mean, m2, lut, log_transform, part, wide, s); break;
      case 4: launch_welford_vec8<256, 2>(sites, npx, n_sites, per, f, mg, mean, m2, lut, log_transform, part, wide, s); break;
      case 5: launch_welford_vec8<512, 2>(sites, npx, n_sites, per, f, mg, mean, m2, lut, log_transform, part, wide, s); break;
      // pipeline depth: sites per stage (two stages in flight)
      case 6: launch_welford_vec8<256, 2, 3>(sites, npx, n_sites, per, f, mg, mean, m2, lut, log_transform, part, wide, s); break;
      case 7: launch_welford_vec8<256, 2, 4>(sites, npx, n_sites, per, f, mg, mean, m2, lut, log_transform, part, wide, s); break;
      case 8: launch_welford_vec8<512, 2, 4>(sites, npx, n_sites, per, f, mg, mean, m2, lut, log_transform, part, wide, s); break;
      default:
        if (bpass)
          launch_welford_vec8<kWfThreadsBright, kWfInv, kWfGroup, kWfLutBright>(
              sites, npx, n_sites, per, f, mg, mean, m2, lut, log_transform, part, wide, s, tab);
        else
          launch_welford_vec8<kWfThreads, kWfInv>(sites, npx, n_sites, per, f, mg, mean, m2, lut,
                                                  log_transform, part, wide, s, tab);
        break;
    }
    if (f > 1) {
      WfParts pc{};
      pc.n = f;
      for (int p = 0; p < f; ++p)
        pc.cnt[p] = (double)std::min<int64_t>(per, n_sites - (int64_t)p * per);
      hipLaunchKernelGGL(k_wf_merge_parts, dim3((unsigned)cdiv(npx, 256)), dim3(256), 0, s, part,
                         npx, pc, (double)n0, mean, m2);
    }
  } else {  // the per-pixel Welford of odd shapes reads 1/n per site
    const dim3 grid((unsigned)cdiv(npx, kWfScalarThreads));
    hipLaunchKernelGGL(k_rn_table, dim3((unsigned)cdiv(n_sites, 256)), dim3(256), 0, s, rn, n0,
                       n_sites);
    if (log_transform)
      hipLaunchKernelGGL(k_welford_scalar<true>, grid, dim3(kWfScalarThreads), 0, s, sites, npx,
                         n_sites, rn, mean, m2, lut);
    else
      hipLaunchKernelGGL(k_welford_scalar<false>, grid, dim3(kWfScalarThreads), 0, s, sites, npx,
                         n_sites, rn, mean, m2, lut);
  }
  TMH_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// per-site histogram + percentile order statistics
// ---------------------------------------------------------------------------

// High values (>= kLdsBins) are rare in microscopy data: they go to global
// atomics in a per-site slab; the LDS add for them is a harmless +0 so the
// common path has no per-pixel branch.
__device__ __forceinline__ void count_hi(uint32_t u, uint32_t* himask, uint32_t* __restrict__ hhi) {
  if (u >= (uint32_t)kLdsBins) {
    const uint32_t h = u - kLdsBins;
    atomicAdd(&hhi[h], 1u);
    atomicOr(&himask[h >> 11], 1u << ((h >> 6) & 31u));
  }
}

__device__ __forceinline__ void count8(const uint4 v, uint32_t* bins, uint32_t* himask,
                                       uint32_t* __restrict__ hhi) {
  const uint32_t u[8] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16,
                         v.z & 0xFFFFu, v.z >> 16, v.w & 0xFFFFu, v.w >> 16};
  const uint32_t any_hi = (v.x | v.y | v.z | v.w) & 0x80008000u;  // kLdsBins == 32768
#pragma unroll
  for (int k = 0; k < 8; ++k) atomicAdd(&bins[u[k] & (kLdsBins - 1)], u[k] < (uint32_t)kLdsBins);
  if (any_hi) {
#pragma unroll
    for (int k = 0; k < 8; ++k) count_hi(u[k], himask, hhi);
  }
}


// Walk the 65,536 bins in 64 rounds of 1024 consecutive bins, thread t
// owning bin 1024*j + t: reads are conflict-free/coalesced, and the dense part
// of a microscopy histogram (a few thousand adjacent values) is spread over
// every thread.  count(b) returns the site's count of value b.  Counts are
// fetched kTailChunk rounds at a time (the next chunk's loads in flight while
// the current one is scanned) and rounds that are empty for the whole
// workgroup are skipped, so a typical microscopy site (values < ~10,000 plus
// saturation) scans ~12 rounds.  `cmask` is 3 words of LDS (chunk masks,
// triple-buffered), `starts` 2 x 1024 int32 of LDS (per-bin inclusive prefix
// ranks, double-buffered by round).  done(b, c) is called once per bin
// after its count has been used (e.g. to reset it).
// ABL (development ablations, tools/mb; 0 in production): 1 = no order-
// statistic output, 4 = no pooled histogram adds
template <int ABL = 0, int kTailChunk = kTailChunkDefault, typename CountFn, typename DoneFn>
__device__ __forceinline__ void hist_tail(CountFn count, DoneFn done, int64_t s, const QPos& p,
                                          uint32_t* __restrict__ vlh_all,
                                          unsigned long long* __restrict__ pooled,
                                          int64_t* __restrict__ zero_counts,
                                          uint32_t* __restrict__ site_hist, uint32_t* slots,
                                          uint32_t* cmask, int32_t* starts) {
  const int tid = threadIdx.x;
  uint32_t* vlh = vlh_all + s * (int64_t)kOsTile;  // this site's column of the tiles
  const bool vec16 = (p.Q & 7) == 0;
  int64_t base = 0;          // exclusive rank of the current round's first bin
  int nscan = 0;
  uint32_t cn[kTailChunk];
#pragma unroll
  for (int k = 0; k < kTailChunk; ++k) cn[k] = count((uint32_t)k * kHistThreads + tid);
  for (int jc = 0; jc < kBins / kHistThreads; jc += kTailChunk) {
    uint32_t c[kTailChunk];
#pragma unroll
    for (int k = 0; k < kTailChunk; ++k) c[k] = cn[k];
    if (jc + kTailChunk < kBins / kHistThreads) {
#pragma unroll
      for (int k = 0; k < kTailChunk; ++k)
        cn[k] = count((uint32_t)(jc + kTailChunk + k) * kHistThreads + tid);
    }
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < kTailChunk; ++k) m |= (c[k] != 0u ? 1u : 0u) << k;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m |= (uint32_t)__shfl_xor((int)m, off, 64);
    const int slot = (jc / kTailChunk) % 3;
    if (tid == 0) cmask[(slot + 1) % 3] = 0u;
    if ((tid & 63) == 0 && m) atomicOr(&cmask[slot], m);
    __syncthreads();
    const uint32_t mask = cmask[slot];
#pragma unroll
    for (int k = 0; k < kTailChunk; ++k) {
      const uint32_t b = (uint32_t)(jc + k) * kHistThreads + tid;
      if (site_hist) site_hist[s * kBins + b] = c[k];
      if (b == 0 && zero_counts) zero_counts[s] = c[k];
      done(b, c[k]);
      if (!((mask >> k) & 1u)) continue;  // uniform: no counts in this round
      uint32_t total;
      const int64_t r = base + block_exscan(c[k], slots, nscan, &total);
      int32_t* R = starts + (nscan & 1) * kHistThreads;
      ++nscan;
      const int64_t r0 = base;
      base += total;
      if (c[k] && !(ABL & 4)) atomicAdd(&pooled[b], (unsigned long long)c[k]);
      if (ABL & 1) continue;
      R[tid] = (int32_t)(r + c[k]);
      __syncthreads();  // R visible; the other R buffer is rewritten only after the next scan
      fill_groups(R, r0, base, (uint32_t)(jc + k) * kHistThreads, p, vlh, vec16);
    }
  }
}


__global__ __launch_bounds__(kHistThreads) void k_hist_scatter(
    const uint16_t* __restrict__ sites, int64_t npx, int vec, uint32_t* __restrict__ hist_hi,
    const QPos p, uint32_t* __restrict__ vlh_all,
    unsigned long long* __restrict__ pooled, int64_t* __restrict__ zero_counts,
    uint32_t* __restrict__ site_hist) {
  __shared__ __attribute__((aligned(16))) uint32_t bins[kLdsBins];
  __shared__ uint32_t himask[16];
  __shared__ uint32_t slots[32];
  __shared__ uint32_t cmask[3];
  __shared__ int32_t starts[2 * kHistThreads];
  const int tid = threadIdx.x;
  const int64_t s = blockIdx.x;

  for (int i = tid; i < kLdsBins / 4; i += kHistThreads)
    reinterpret_cast<uint4*>(bins)[i] = make_uint4(0u, 0u, 0u, 0u);
  if (tid < 16) himask[tid] = 0u;
  if (tid < 3) cmask[tid] = 0u;
  __syncthreads();

  const uint16_t* site = sites + s * npx;
  uint32_t* hhi = hist_hi + s * (int64_t)kHiBins;
  if (vec) {
    const uint4* src = reinterpret_cast<const uint4*>(site);
    const int64_t n16 = npx >> 3;
    int64_t i = tid;
    for (; i + 3 * kHistThreads < n16; i += 4 * kHistThreads) {
      const uint4 v0 = ld_site<true>(src + i), v1 = ld_site<true>(src + i + kHistThreads),
                  v2 = ld_site<true>(src + i + 2 * kHistThreads),
                  v3 = ld_site<true>(src + i + 3 * kHistThreads);
      count8(v0, bins, himask, hhi);
      count8(v1, bins, himask, hhi);
      count8(v2, bins, himask, hhi);
      count8(v3, bins, himask, hhi);
    }
    for (; i < n16; i += kHistThreads) count8(ld_site<true>(src + i), bins, himask, hhi);
  } else {
    for (int64_t i = tid; i < npx; i += kHistThreads) {
      const uint32_t u = site[i];
      atomicAdd(&bins[u & (kLdsBins - 1)], u < (uint32_t)kLdsBins);
      count_hi(u, himask, hhi);
    }
  }
  // __syncthreads() orders LDS only: the global atomics into the slab must
  // have been performed before other waves swap the slab out below.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  hist_tail(
      [&](uint32_t b) -> uint32_t {
        if (b < (uint32_t)kLdsBins) return bins[b];
        const uint32_t h = b - kLdsBins;
        return ((himask[h >> 11] >> ((h >> 6) & 31u)) & 1u) ? atomicExch(&hhi[h], 0u) : 0u;
      },
      [](uint32_t, uint32_t) {},
      s, p, vlh_all, pooled, zero_counts, site_hist, slots, cmask, starts);
}

// Per-site histogram (65,536 counts, exact) -> order statistics, written from
// a complete histogram held in global memory (zero-maintained: every count is
// read and reset), e.g. accumulated by the fused correct+histogram pass.
// ABL 8: counts are not reset (re-runnable).  NT threads per site (1024, or
// 256: one workgroup fits beside the fused pass's two on a CU -- VGPRs <= 64).
// rmask (may be NULL: every round is read): per site, the 1,024-bin rounds
// at or above dense_rounds that hold counts; the others are known empty and
// are not read (a microscopy site touches a handful of the 64).  The mask is
// zero-maintained like the counts.
// super-round width of the finalize: 8 rounds (8,192 bins, 32 KB of ranks
// per buffer) for the 1,024-thread form, 1 for the narrow side-stream form.
// Round 6: 8 instead of 4 -- bright sites (45 of 64 rounds in use) scan in 6
// super-rounds instead of 12: bright job 136.1k / 136.7k vs 135.5k / 134.5k,
// standard 166.9k / 165.4k vs 166.5k / 166.6k, same box ABBA
// (profiles/r6/ab_finalize_sr8_*_r6g.jsonl).
template <int NT>
struct FinSR {
  static constexpr int value = NT >= 1024 ? 8 : 1;
};

template <int ABL, int NT>
__device__ __forceinline__ void hist_finalize_site(
    int64_t s, uint32_t* __restrict__ hist, unsigned long long* __restrict__ rmask,
    int dense_rounds, const QPos& p, uint32_t* __restrict__ vlh_all,
    unsigned long long* __restrict__ pooled, int n_pooled, int64_t* __restrict__ zero_counts,
    uint32_t* __restrict__ site_hist) {
  constexpr int SR = FinSR<NT>::value;
  __shared__ uint32_t slots[32];
  __shared__ int32_t starts[2 * SR * kRound];
  const unsigned long long rm = rmask ? rmask[s] : ~0ull;
  __syncthreads();
  if (rmask && !(ABL & 8) && threadIdx.x == 0) rmask[s] = 0ull;  // every thread has read it
  uint32_t* h = hist + s * (int64_t)kBins;
  // sites spread their pooled-histogram adds over n_pooled copies (fewer
  // same-address atomic collisions); k_pooled_fold sums the copies
  unsigned long long* pl = pooled ? pooled + (int64_t)(s % n_pooled) * kBins : nullptr;
  const unsigned long long dense = dense_rounds >= 64 ? ~0ull : ((1ull << dense_rounds) - 1ull);
  hist_tail_rounds<ABL & 7, NT, SR>(
      dense | rm, [&](uint32_t b) -> uint32_t { return h[b]; },
      [&](uint32_t b, uint32_t c) {
        if (!(ABL & 8) && c) h[b] = 0u;
      },
      s, p, vlh_all, pl, zero_counts, site_hist, slots, starts);
}

template <int ABL = 0, int NT = kHistThreads>
__global__ __launch_bounds__(NT, 8) void k_hist_finalize(
    uint32_t* __restrict__ hist, unsigned long long* __restrict__ rmask, int dense_rounds,
    const QPos p, uint32_t* __restrict__ vlh_all,
    unsigned long long* __restrict__ pooled, int n_pooled,
    int64_t* __restrict__ zero_counts, uint32_t* __restrict__ site_hist,
    const unsigned long long* __restrict__ wide = nullptr, unsigned long long xthr = 0) {
  // a very wide launch: k_hist_site_u16 has written this site's outputs
  if (wide && __builtin_nontemporal_load(wide + 1) >= xthr) return;
  hist_finalize_site<ABL, NT>(blockIdx.x, hist, rmask, dense_rounds, p, vlh_all, pooled, n_pooled,
                              zero_counts, site_hist);
}

// Several jobs' finalize in one launch (blockIdx.y = job): each site's order
// statistics from its job's histogram slab and round mask (the pooled
// histograms come from the column sum)
__global__ __launch_bounds__(kHistThreads, 8) void k_hist_finalize_jobs(const TailJobs J) {
  const TailJob& t = J.j[blockIdx.y];
  if ((int64_t)blockIdx.x >= t.n_sites) return;  // uniform per workgroup
  hist_finalize_site<0, kHistThreads>(blockIdx.x, t.hist, t.rmask, 0, t.qp, t.vlh, nullptr, 1,
                                      t.zero_counts, t.site_hist);
}

// Pooled histogram of a fused launch's sites without per-site atomics:
// pooled[b] += sum over the sites of hist[s][b], read only where site s's
// round mask names b's 1,024-bin round (the other rounds are known empty).
// Thread = bin, blockIdx.y = a chunk of kColSites sites: coalesced 1 KB rows,
// one 64-bit atomic per bin and chunk.  Runs before k_hist_finalize, which
// reads and resets the same counts; on bright sites (45 of 64 rounds in use)
// this replaced ~30,000 per-site atomics per site in the finalize (1.2 ms of
// its 2.4 ms at 3,456 sites: profiles/r2/mb_tail_bright_r2y.txt).
constexpr int kColSites = 32;
__device__ __forceinline__ void pooled_colsum_chunk(const uint32_t* __restrict__ hist,
                                                    const unsigned long long* __restrict__ rmask,
                                                    const unsigned long long* __restrict__ rm_all,
                                                    int64_t n_sites,
                                                    unsigned long long* __restrict__ pooled) {
  static_assert(kColSites <= 256, "one mask per thread");
  __shared__ uint32_t use[kColSites];  // per site of the chunk: this round holds counts
  __shared__ int any;
  const int b = (int)blockIdx.x * 256 + threadIdx.x;
  const int round = (int)blockIdx.x >> 2;  // 256 bins per workgroup, 4 workgroups per round
  // rounds no site of the launch uses (the fused pass's union of the masks)
  if (rm_all && !((*rm_all >> round) & 1ull)) return;
  const int64_t s0 = (int64_t)blockIdx.y * kColSites;
  const int ns = (int)(n_sites - s0 < kColSites ? n_sites - s0 : kColSites);
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  if ((int)threadIdx.x < kColSites) {
    const uint32_t u = (int)threadIdx.x < ns ? (uint32_t)((rmask[s0 + threadIdx.x] >> round) & 1ull) : 0u;
    use[threadIdx.x] = u;
    if (u) any = 1;
  }
  __syncthreads();
  if (!any) return;  // uniform: no site of the chunk uses this round
  const uint32_t* h = hist + s0 * kBins + b;
  unsigned long long t = 0;
#pragma unroll 16
  for (int s = 0; s < ns; ++s)
    if (use[s]) t += h[(int64_t)s * kBins];
  if (t) atomicAdd(&pooled[b], t);
}

__global__ __launch_bounds__(256) void k_pooled_colsum(const uint32_t* __restrict__ hist,
                                                       const unsigned long long* __restrict__ rmask,
                                                       const unsigned long long* __restrict__ rm_all,
                                                       int64_t n_sites,
                                                       unsigned long long* __restrict__ pooled) {
  pooled_colsum_chunk(hist, rmask, rm_all, n_sites, pooled);
}

// blockIdx.z = job (TailJobs)
__global__ __launch_bounds__(256) void k_pooled_colsum_jobs(const TailJobs J) {
  const TailJob& t = J.j[blockIdx.z];
  if ((int64_t)blockIdx.y * kColSites >= t.n_sites) return;  // uniform per workgroup
  pooled_colsum_chunk(t.hist, t.rmask, t.rm_all, t.n_sites, t.pooled);
}

// Several fused jobs' histogram tails (pooled column sums, then every site's
// order statistics) in two launches
void launch_hist_finalize_jobs(const TailJobs& J, hipStream_t s) {
  if (J.n <= 0) return;
  ProfScope prof("hist_finalize", s);
  int64_t nmax = 0;
  for (int j = 0; j < J.n; ++j) nmax = std::max(nmax, J.j[j].n_sites);
  if (nmax <= 0) return;
  hipLaunchKernelGGL(k_pooled_colsum_jobs,
                     dim3(kBins / 256, (unsigned)cdiv(nmax, kColSites), (unsigned)J.n), dim3(256), 0,
                     s, J);
  hipLaunchKernelGGL(k_hist_finalize_jobs, dim3((unsigned)nmax, (unsigned)J.n), dim3(kHistThreads),
                     0, s, J);
  TMH_HIP(hipGetLastError());
}

// pooled[b] += sum of the copies; copies reset to zero (zero-maintained)
__global__ void k_pooled_fold(unsigned long long* __restrict__ pooled,
                              unsigned long long* __restrict__ parts, int n_parts,
                              const unsigned long long* __restrict__ wide = nullptr,
                              unsigned long long xthr = 0) {
  if (wide && __builtin_nontemporal_load(wide + 1) < xthr) return;  // nothing was added
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= kBins) return;
  unsigned long long t = 0;
  for (int i = 0; i < n_parts; ++i) {
    t += parts[(int64_t)i * kBins + b];
    parts[(int64_t)i * kBins + b] = 0ull;
  }
  pooled[b] += t;
}

void launch_pooled_colsum(const uint32_t* hist, const unsigned long long* rmask,
                          const unsigned long long* rm_all, int64_t n_sites,
                          unsigned long long* pooled, hipStream_t s) {
  if (n_sites <= 0) return;
  hipLaunchKernelGGL(k_pooled_colsum, dim3(kBins / 256, (unsigned)cdiv(n_sites, kColSites)),
                     dim3(256), 0, s, hist, rmask, rm_all, n_sites, pooled);
  TMH_HIP(hipGetLastError());
}

void launch_hist_finalize(uint32_t* hist, unsigned long long* rmask, int dense_rounds,
                          int64_t n_sites, const QPos& p, uint32_t* vlh, int64_t vlh_ld,
                          unsigned long long* pooled,
                          unsigned long long* pooled_parts, int n_parts, int64_t* zero_counts,
                          uint32_t* site_hist, hipStream_t s, bool narrow,
                          const unsigned long long* rm_all, const unsigned long long* wide,
                          unsigned long long xthr) {
  if (n_sites <= 0) return;
  ProfScope prof(narrow ? "hist_finalize_side" : "hist_finalize", s);
  QPos pp = p;
  pp.tstride = vlh_ld * kOsTile;
  // with a round mask the pooled histogram is a column sum ahead of the
  // finalize; without one, the finalize adds into pooled copies, then folded
  const bool colsum = rmask != nullptr && dense_rounds == 0;
  if (colsum)
    hipLaunchKernelGGL(k_pooled_colsum, dim3(kBins / 256, (unsigned)cdiv(n_sites, kColSites)),
                       dim3(256), 0, s, hist, rmask, rm_all, n_sites, pooled);
  unsigned long long* fin_pooled = colsum ? nullptr : pooled_parts;
  if (narrow)
    hipLaunchKernelGGL((k_hist_finalize<0, 256>), dim3((unsigned)n_sites), dim3(256), 0, s, hist,
                       rmask, dense_rounds, pp, vlh, fin_pooled, n_parts, zero_counts, site_hist,
                       wide, xthr);
  else
    hipLaunchKernelGGL((k_hist_finalize<0, kHistThreads>), dim3((unsigned)n_sites),
                       dim3(kHistThreads), 0, s, hist, rmask, dense_rounds, pp, vlh, fin_pooled,
                       n_parts, zero_counts, site_hist, wide, xthr);
  if (!colsum)
    hipLaunchKernelGGL(k_pooled_fold, dim3(kBins / 256), dim3(256), 0, s, pooled, pooled_parts,
                       n_parts);
  TMH_HIP(hipGetLastError());
}

// Very wide sites (a third or more of the 8-pixel groups hold a value >=
// 16,384, e.g. uniform 16-bit data): the per-site LDS slices of the fused pass
// would send most pixels to global atomics (uniform sites ran the fused pass
// at ~0.5 s for 3,456 sites), so the fused pass runs without its histogram
// and this kernel builds each site's exact 65,536-bin histogram in LDS as u16
// pairs (128 KB: value v in word v >> 1, half v & 1) from one more read of the
// site, then scans it into order statistics as k_hist_finalize does.  A half
// never wraps: the add that takes it to kU16Spill (seen in the returned old
// word -- exactly one add sees kU16Spill - 1 each time) takes kU16Spill back
// out of it and adds kU16Spill to the site's zero-maintained global slab,
// whose 1,024-bin round is flagged; the scan adds (and resets) the slab's
// counts of the flagged rounds.  Until that subtract lands other adds keep
// landing on the half, so it is kept far below 65,535: 49,151 adds of
// headroom, against at most 16 waves x 15 x 64 = 15,360 LDS adds the
// workgroup has outstanding at once.  (Spilling at the wrap itself raced: a carry
// into the upper half, not yet undone, could make an add to the upper half
// see -- and spill -- a wrap that was not there.)  Launched when the job's
// site probe finds very wide sites (wide == null), or gated on a count.
constexpr int kU16Threads = 1024;
constexpr uint32_t kU16Spill = 0x4000u;
__global__ __launch_bounds__(kU16Threads) void k_hist_site_u16(
    const uint16_t* __restrict__ sites, int64_t npx, int64_t n_sites,
    uint32_t* __restrict__ slab, const QPos p,
    uint32_t* __restrict__ vlh_all, unsigned long long* __restrict__ pooled, int n_pooled,
    int64_t* __restrict__ zero_counts, uint32_t* __restrict__ site_hist,
    const unsigned long long* __restrict__ wide, unsigned long long xthr, const SiteTab tab) {
  if (wide && __builtin_nontemporal_load(wide + 1) < xthr) return;  // uniform: not very wide
  constexpr int SR = 2;  // 2,048-bin super-rounds: 16 KB of ranks beside the 128 KB histogram
  __shared__ __attribute__((aligned(16))) uint32_t w16[kBins / 2];
  __shared__ uint32_t slots[32];
  __shared__ int32_t starts[2 * SR * kRound];
  __shared__ unsigned long long ovf;  // rounds with counts in the slab
  const int tid = threadIdx.x;
  // persistent over the sites (one workgroup per CU fits): a launch that is
  // not very wide costs one small grid, not one workgroup per site
  for (int64_t s = blockIdx.x; s < n_sites; s += gridDim.x) {
  __syncthreads();  // the previous site's scan is done with the LDS
  for (int i = tid; i < kBins / 8; i += kU16Threads)
    reinterpret_cast<uint4*>(w16)[i] = make_uint4(0u, 0u, 0u, 0u);
  if (tid == 0) ovf = 0ull;
  __syncthreads();
  uint32_t* hs = slab + s * (int64_t)kBins;
  auto add = [&](uint32_t u) {
    const uint32_t sh = (u & 1u) << 4;
    const uint32_t old = atomicAdd(&w16[u >> 1], 1u << sh);
    if (((old >> sh) & 0xFFFFu) == kU16Spill - 1u) {  // this add took the half to kU16Spill: rare
      atomicSub(&w16[u >> 1], kU16Spill << sh);
      atomicAdd(&hs[u], kU16Spill);
      atomicOr(&ovf, 1ull << (u >> 10));
    }
  };
  gsite_t* src = to_global(
      tab.in ? tab.in[site_block(tab, s)] + site_in_block(tab, s) * npx : sites + s * npx);
  const int64_t n16 = npx >> 3;
  int64_t i = tid;
  for (; i + 3 * kU16Threads < n16; i += 4 * kU16Threads) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = ld_site<true>(src + i + k * kU16Threads);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t wd[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        add(wd[q] & 0xFFFFu);
        add(wd[q] >> 16);
      }
    }
  }
  for (; i < n16; i += kU16Threads) {
    const uint4 v = ld_site<true>(src + i);
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      add(wd[q] & 0xFFFFu);
      add(wd[q] >> 16);
    }
  }
  // the slab atomics must have been performed before the scan reads the slab
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long ov = ovf;
  unsigned long long* pl = pooled + (int64_t)(blockIdx.x % n_pooled) * kBins;
  hist_tail_rounds<0, kU16Threads, SR>(
      ~0ull,
      [&](uint32_t b) -> uint32_t {
        uint32_t c = (w16[b >> 1] >> ((b & 1u) << 4)) & 0xFFFFu;
        if ((ov >> (b >> 10)) & 1ull) {
          const uint32_t g = hs[b];
          if (g) {
            hs[b] = 0u;  // zero-maintained
            c += g;
          }
        }
        return c;
      },
      [](uint32_t, uint32_t) {}, s, p, vlh_all, pl, zero_counts, site_hist, slots, starts);
  }
}

void launch_hist_site_u16(const uint16_t* sites, int64_t npx, int64_t n_sites, uint32_t* slab,
                          const QPos& p, uint32_t* vlh, int64_t vlh_ld,
                          unsigned long long* pooled, unsigned long long* pooled_parts,
                          int n_parts, int64_t* zero_counts, uint32_t* site_hist,
                          const unsigned long long* wide, unsigned long long xthr, hipStream_t s,
                          const SiteTab& tab) {
  if (n_sites <= 0) return;
  ProfScope prof("hist_u16", s);
  QPos pp = p;
  pp.tstride = vlh_ld * kOsTile;
  int dev = 0, cus = 256;
  TMH_HIP(hipGetDevice(&dev));
  TMH_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const unsigned grid = (unsigned)std::min<int64_t>(n_sites, cus);
  hipLaunchKernelGGL(k_hist_site_u16, dim3(grid), dim3(kU16Threads), 0, s, sites, npx, n_sites,
                     slab, pp, vlh, pooled_parts, n_parts, zero_counts, site_hist, wide, xthr, tab);
  hipLaunchKernelGGL(k_pooled_fold, dim3(kBins / 256), dim3(256), 0, s, pooled, pooled_parts,
                     n_parts, wide, xthr);
  TMH_HIP(hipGetLastError());
}

void launch_hist_scatter(const uint16_t* sites, int64_t npx, int64_t n_sites, uint32_t* hist_hi,
                         const QPos& p, uint32_t* vlh, int64_t vlh_ld, unsigned long long* pooled,
                         int64_t* zero_counts, uint32_t* site_hist, hipStream_t s) {
  if (n_sites <= 0) return;
  ProfScope prof("hist", s);
  const int vec = ((npx & 7) == 0 && (reinterpret_cast<uintptr_t>(sites) & 15) == 0) ? 1 : 0;
  QPos pp = p;
  pp.tstride = vlh_ld * kOsTile;
  hipLaunchKernelGGL(k_hist_scatter, dim3((unsigned)n_sites), dim3(kHistThreads), 0, s, sites, npx,
                     vec, hist_hi, pp, vlh, pooled, zero_counts, site_hist);
  TMH_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// sequential percentile accumulation
// ---------------------------------------------------------------------------

// numpy 2.2.6 _lerp on the two order statistics, f64, no contraction:
//   a + (b-a)*g, or b - (b-a)*(1-g) where g >= 0.5.  Plain operators under a
// scoped fp-contract(off) (built with -ffp-contract=fast-honor-pragmas); the
// HIP __dmul_rn/__dadd_rn helpers are header code compiled with contraction
// on and would still fuse into one v_fma_f64 (1-ulp drift vs numpy).
__device__ __forceinline__ double lerp_np(uint32_t a, uint32_t b, double g) {
#pragma clang fp contract(off)
  const double d = (double)(b - a);
  return (g >= 0.5) ? (double)b - d * (1.0 - g) : (double)a + d * g;
}

__device__ __forceinline__ double add_nc(double x, double y) {
#pragma clang fp contract(off)
  return x + y;
}

constexpr int kPctThreads = 256;
constexpr int kPctUnroll = 16;

// Quantiles [q_begin, q_begin + Q) of the quantile-tiled order statistics of
// n_sites sites (vlh: the first site's column, tstride words between tiles;
// acc points at the range's first quantile: a sub-range is one launch of the
// pipelined rank chain).  Thread = quantile: one u32 load per site -- a
// workgroup's 256 quantiles are one tile, so it streams contiguous 1 KB runs,
// site after site -- the lerp off the critical path, and only the f64 add (no
// contraction) on the in-order dependency chain.
template <bool NTL>
__global__ __launch_bounds__(kPctThreads) void k_pct_acc(const uint32_t* __restrict__ vlh,
                                                          int64_t n_sites, int64_t tstride,
                                                          int q_begin, int Q,
                                                          const double* __restrict__ gamma,
                                                          double* __restrict__ acc,
                                                          const unsigned long long* __restrict__ xw,
                                                          unsigned long long xthr) {
  // xw: run only for a very wide launch (the compact-CDF fold serves the rest)
  if (xw && __builtin_nontemporal_load(xw + 1) < xthr) return;
  const int t = (int)blockIdx.x * kPctThreads + threadIdx.x;
  if (t >= Q) return;
  const int q = q_begin + t;
  const double g = gamma[q];
  double a = acc[t];
  const uint32_t* p = vlh + (int64_t)(q / kOsTile) * tstride + (q % kOsTile);
  constexpr int64_t ld = kOsTile;
  // software pipeline over two register sets used alternately (no copies
  // between them: a copy of a pending load makes the compiler wait for every
  // load in flight): the next kPctUnroll sites' loads are in flight while the
  // current ones are folded in (tail loads clamp to the last site)
  const int64_t last = n_sites - 1;
  auto ld1 = [&](int64_t u) -> uint32_t {
    u = u < last ? u : last;
    return NTL ? __builtin_nontemporal_load(p + u * ld) : p[u * ld];
  };
  uint32_t va[kPctUnroll], vb[kPctUnroll];
#pragma unroll
  for (int k = 0; k < kPctUnroll; ++k) va[k] = ld1(k);
  for (int64_t s = 0; s < n_sites; s += 2 * kPctUnroll) {
#pragma unroll
    for (int k = 0; k < kPctUnroll; ++k) vb[k] = ld1(s + kPctUnroll + k);
#pragma unroll
    for (int k = 0; k < kPctUnroll; ++k)
      if (s + k < n_sites) a = add_nc(a, lerp_np(va[k] & 0xFFFFu, va[k] >> 16, g));
#pragma unroll
    for (int k = 0; k < kPctUnroll; ++k) va[k] = ld1(s + 2 * kPctUnroll + k);
#pragma unroll
    for (int k = 0; k < kPctUnroll; ++k)
      if (s + kPctUnroll + k < n_sites) a = add_nc(a, lerp_np(vb[k] & 0xFFFFu, vb[k] >> 16, g));
  }
  acc[t] = a;
}

void launch_pct_accumulate(const uint32_t* vlh, int64_t n_sites, int64_t vlh_ld, int Q,
                           const double* gamma, double* acc, hipStream_t s) {
  launch_pct_accumulate_range(vlh, n_sites, vlh_ld, 0, Q, gamma, acc, s);
}

void launch_pct_accumulate_range(const uint32_t* vlh, int64_t n_sites, int64_t vlh_ld, int q_begin,
                                 int q_count, const double* gamma, double* acc, hipStream_t s,
                                 const unsigned long long* only_xwide, unsigned long long xthr) {
  if (n_sites <= 0 || q_count <= 0) return;
  ProfScope prof("pct_acc", s);
  // Regular (not non-temporal) loads of the order statistics.  PROVISIONAL:
  // the kernel itself runs 5% slower with them, and the +1.7% job throughput
  // measured for this choice (profiles/r1/ab_pct_ntl.txt) is within the
  // run-to-run spread of one build (profiles/r1/noise_same_build.txt).
  hipLaunchKernelGGL(k_pct_acc<false>, dim3((unsigned)cdiv(q_count, kPctThreads)),
                     dim3(kPctThreads), 0, s, vlh, n_sites, vlh_ld * kOsTile, q_begin, q_count,
                     gamma, acc, only_xwide, xthr);
  TMH_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// finalize (stats.py:94-112) and multi-rank merge
// ---------------------------------------------------------------------------

__global__ void k_finalize(const double* __restrict__ mean, const double* __restrict__ m2, int64_t n,
                           int64_t npx, double* __restrict__ out_mean, double* __restrict__ out_std) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npx) return;
  if (out_mean) out_mean[i] = mean[i];
  if (out_std) out_std[i] = (n < 2) ? __builtin_nan("") : sqrt(m2[i] / (double)(n - 1));
}

__global__ void k_variance(const double* __restrict__ m2, int64_t n, int64_t npx,
                           double* __restrict__ out_var) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npx) return;
  out_var[i] = (n < 2) ? __builtin_nan("") : m2[i] / (double)(n - 1);
}

void launch_variance(const double* m2, int64_t n, int64_t npx, double* out_var, hipStream_t s) {
  hipLaunchKernelGGL(k_variance, dim3((unsigned)cdiv(npx, 256)), dim3(256), 0, s, m2, n, npx,
                     out_var);
  TMH_HIP(hipGetLastError());
}

void launch_finalize(const double* mean, const double* m2, int64_t n, int64_t npx, double* out_mean,
                     double* out_std, hipStream_t s) {
  ProfScope prof("finalize", s);
  hipLaunchKernelGGL(k_finalize, dim3((unsigned)cdiv(npx, 256)), dim3(256), 0, s, mean, m2, n, npx,
                     out_mean, out_std);
  TMH_HIP(hipGetLastError());
}

__global__ void k_merge1(const double* __restrict__ mean, double nr, int64_t npx,
                         double* __restrict__ nmean) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < npx) nmean[i] = nr * mean[i];
}

// Chan et al. pairwise combine, expressed as two sums so that one RCCL
// all-reduce per quantity merges any number of ranks:
//   mean = sum_r n_r mean_r / n,  M2 = sum_r [M2_r + n_r (mean_r - mean)^2]
__global__ void k_merge2(double* __restrict__ mean, const double* __restrict__ m2, double nr,
                         const double* __restrict__ sum_nmean, double n_total, int64_t npx,
                         double* __restrict__ m2c) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npx) return;
  const double mu = sum_nmean[i] / n_total;
  const double d = mean[i] - mu;
  m2c[i] = m2[i] + nr * d * d;
  mean[i] = mu;
}

void launch_merge1(const double* mean, int64_t n, int64_t npx, double* nmean, hipStream_t s) {
  hipLaunchKernelGGL(k_merge1, dim3((unsigned)cdiv(npx, 256)), dim3(256), 0, s, mean, (double)n,
                     npx, nmean);
  TMH_HIP(hipGetLastError());
}

void launch_merge2(double* mean, const double* m2, int64_t n_r, const double* sum_nmean,
                   int64_t n_total, int64_t npx, double* m2c, hipStream_t s) {
  hipLaunchKernelGGL(k_merge2, dim3((unsigned)cdiv(npx, 256)), dim3(256), 0, s, mean, m2,
                     (double)n_r, sum_nmean, (double)n_total, npx, m2c);
  TMH_HIP(hipGetLastError());
}

// Zero several u64/f64 arrays in one launch (a job reset: mean, M2, the
// percentile accumulator, the pooled histogram, the wide-group counters) --
// one kernel instead of a fill launch per array.
__global__ void k_zero_u64(const ZeroList z) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int k = 0; k < z.n; ++k) {
    unsigned long long* p = z.p[k];
    const int64_t n = z.count[k];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = 0ull;
  }
}

void launch_zero_u64(const ZeroList& z, hipStream_t s) {
  int64_t total = 0;
  for (int k = 0; k < z.n; ++k) total += z.count[k];
  if (!total) return;
  const unsigned g = (unsigned)std::min<int64_t>(cdiv(total, 256 * 4), 2048);
  hipLaunchKernelGGL(k_zero_u64, dim3(g), dim3(256), 0, s, z);
  TMH_HIP(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_zero_u32(const ZeroList32 z) {
  for (int k = 0; k < z.n; ++k)
    for (int i = threadIdx.x; i < z.count[k]; i += 256) z.p[k][i] = 0u;
}

void launch_zero_u32(const ZeroList32& z, hipStream_t s) {
  if (z.n == 0) return;
  hipLaunchKernelGGL(k_zero_u32, dim3(1), dim3(256), 0, s, z);
  TMH_HIP(hipGetLastError());
}

__global__ void k_copy_f64(const double* __restrict__ src, double* __restrict__ dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

void launch_copy_f64(const double* src, double* dst, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_copy_f64, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, src, dst, n);
  TMH_HIP(hipGetLastError());
}

}  // namespace tmh
