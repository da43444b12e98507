// Shared definitions for libtmhip (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/tmhip.h"

namespace tmh {

// error plumbing --------------------------------------------------------------
void set_error(const std::string& msg);

struct Error {
  int code;
  std::string msg;
};

#define TMH_HIP(expr)                                                                    \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw ::tmh::Error{TMH_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)}; \
  } while (0)

#define TMH_CHECK(cond, code, msg)                         \
  do {                                                     \
    if (!(cond)) throw ::tmh::Error{(code), (msg)};        \
  } while (0)

// kernel timing (bench/roofline support) ----------------------------------------
// When enabled, every launch of a named kernel is bracketed by a pair of HIP
// events on the stream it runs on; tmh_profile_read sums their durations.
struct ProfScope {
  ProfScope(const char* name, hipStream_t s);
  ~ProfScope();
  const char* name_;
  hipStream_t s_;
  void* slot_;
};

// histogram geometry ------------------------------------------------------------
constexpr int kBins = 65536;      // all uint16 values
constexpr int kLdsBins = 32768;   // bins [0, kLdsBins) counted in LDS (u32)
constexpr int kHiBins = kBins - kLdsBins;  // counted with global atomics
constexpr int kHistThreads = 1024;
constexpr int kBinsPerThread = kBins / kHistThreads;  // 64

// log10 LUT entries staged in LDS by the per-pixel kernels (f64 / f32x2): 32 KB
constexpr int kLutLds = 4096;

// quantile positions (np.percentile 'linear' previous/next sorted positions)
struct QPos {
  const int32_t* lo;  // [Q] previous sorted positions (tables uploaded by the caller)
  const int32_t* hi;  // [Q] next sorted positions
  int Q;
  double scale;  // (Q - 1) / (n - 1): the quantile at a sorted position, up to rounding
  int32_t last;  // n - 1
  int hi_next;   // hi[q] == min(lo[q] + 1, n - 1) for every q: hi is not read
  int64_t tstride;  // order statistics: words between quantile tiles (sites x kOsTile)
};

// Order statistics (per site and quantile, u32 previous | next << 16) are
// stored quantile-tiled, [Q / kOsTile][site][kOsTile]: the ordered percentile
// sum (one thread per quantile, sites in order) then reads a contiguous 1 KB
// run per site per workgroup instead of 1 KB every Q words.  A buffer with
// room for C sites has tile stride C * kOsTile words.
constexpr int kOsTile = 256;
__host__ __device__ inline int64_t os_tiles(int64_t Q) { return (Q + kOsTile - 1) / kOsTile; }

// ---------------------------------------------------------------------------
// f64 refinement of the f32 correction
// ---------------------------------------------------------------------------
// The correct kernels compute 10**t in f32 (log2 domain).  Their result o
// carries a relative error below kRefineK1 * a + kRefineK2 (a = mean(std)/std
// of the pixel; v_log/v_exp 1 ulp, f32 coefficients, fma roundings: derived
// in DESIGN.md §3), so |o_f32 - o_f64| < 1 -- and the truncated uint16 is
// within 1 DN of the reference -- wherever |o| < T = 1 / (K1 * a_max + K2),
// a_max the image's largest finite a.  Pixels with |o| >= T (saturated pixels
// in dim corners: corrected values up to ~1e6 that numpy wraps modulo 2^16)
// are appended to a fixup list by the streaming kernel, and a small kernel
// after it recomputes them in f64, op for op as the reference does.  (Doing
// the f64 work inline would make every streaming kernel reserve its
// registers: the chain pass fell from 8 to 5 waves per SIMD.)
constexpr double kRefineK1 = 6.7e-6;
constexpr double kRefineK2 = 4.2e-6;

// per corrector, device memory: np.mean(std), np.mean(mean) (image.py:627),
// np.log10(1e-10) (the zero pixels' log), T (as double)
struct RefineConst {
  double S, M, zero_log10, T;
};

// pixels to refine, one entry per group of up to 8 consecutive pixels:
// e[i] = site << 40 | mask << 32 | p0 (bit j of mask: pixel p0 + j), for
// i < min(*n, cap); *n > cap means the list overflowed and the fixup
// recomputes every pixel in f64.  (A launch covers < 2^24 sites.)
struct FixList {
  unsigned long long* e;
  unsigned int* n;
  unsigned int cap;
};

__device__ __forceinline__ unsigned long long fix_code8(uint32_t mask, int64_t site, int64_t p0) {
  return ((unsigned long long)site << 40) | ((unsigned long long)(mask & 0xFFu) << 32) |
         (unsigned long long)(uint32_t)p0;
}

__device__ __forceinline__ void fix_push8(const FixList& fl, uint32_t mask, int64_t site, int64_t p0) {
  const unsigned int i = atomicAdd(fl.n, 1u);
  if (i < fl.cap) fl.e[i] = fix_code8(mask, site, p0);
}

__device__ __forceinline__ void fix_push(const FixList& fl, int64_t site, int64_t px) {
  fix_push8(fl, 1u, site, px);
}

// entry i of the list (or, overflowed, the i-th group of 8 pixels)
__device__ __forceinline__ void fix_entry(const FixList& fl, bool all, int64_t i, int64_t npx,
                                          int64_t& site, int64_t& p0, uint32_t& mask) {
  if (all) {
    const int64_t gps = (npx + 7) / 8;  // groups per site
    site = i / gps;
    p0 = (i - site * gps) * 8;
    mask = 0xFFu;
  } else {
    const unsigned long long e = fl.e[i];
    site = (int64_t)(e >> 40);
    mask = (uint32_t)(e >> 32) & 0xFFu;
    p0 = (int64_t)(e & 0xFFFFFFFFull);
  }
}

// ChannelImage._correct_illumination (tmlib/image.py:619-631) of one pixel in
// f64, one rounding per numpy operation; returns the int32 numpy's x86
// astype truncates to (NaN, +-inf, out of range -> INT32_MIN).
template <bool LOG>
__device__ __forceinline__ int32_t correct_ref_f64(uint32_t x, double mean, double std, double S,
                                                   double M, double zero_log10) {
#pragma clang fp contract(off)
  double v = (double)x;
  if (LOG) v = (x == 0u) ? zero_log10 : log10(v);  // img[img == 0] = 1e-10; log10
  double t = (v - mean) / std;
  t = t * S;
  t = t + M;
  if (LOG) t = exp10(t);  // 10 ** img
  return (t > -2147483649.0 && t < 2147483648.0) ? (int32_t)t : INT32_MIN;
}

// launches (defined in the .hip files) -------------------------------------------
// part: optional scratch of part_cap doubles for site-split launches (null: one part)
// forced_parts: 0 = pick the site split automatically, 1..4 = that many parts
// Blocked site layout: the sites of a launch live in blocks of 1 << shift
// consecutive sites each (device arrays of block base pointers; in == null:
// one contiguous run at the launch's in / out pointers).  A block holds a
// multiple of every configuration's sites per unit (shift >= 2).
struct SiteTab {
  const uint16_t* const* in = nullptr;
  uint16_t* const* out = nullptr;
  int shift = 0;
};

// Values beyond the packed fused configuration's LDS slices (>= 16,384 on
// bright sites): appended per site as u16 (staged in LDS, one reservation per
// site and unit) instead of one global atomic each (~61 B of HBM traffic per
// atomic, profiles/r4/abl_rare_atomics_r4ab.jsonl); k_rare_count folds each
// site's list into its histogram.  cnt[s] counts every append; entries past
// cap took the global atomic instead.  v == null: atomics only.
struct RareList {
  uint16_t* v = nullptr;      // site s: v[s * cap, s * cap + min(cnt[s], cap))
  unsigned int* cnt = nullptr;
  unsigned int cap = 0;
};
constexpr int kRareLo = 16384;  // the packed configuration's slice size

// site s of a launch in its layout (contiguous at base, or blocked)
__device__ __forceinline__ int64_t site_block(const SiteTab& t, int64_t s) { return s >> t.shift; }
__device__ __forceinline__ int64_t site_in_block(const SiteTab& t, int64_t s) {
  return s & ((1ll << t.shift) - 1);
}

// bright: 1 = the host's site probe found bright sites (the 16,384-entry LUT
// pass in three site parts where the launch allows), 0 = standard
void launch_welford(const uint16_t* sites, int64_t npx, int64_t n_sites, int64_t n0, double* rn,
                    double* mean, double* m2, const double* lut, int log_transform,
                    double* part, size_t part_cap, int forced_parts,
                    unsigned long long* wide, int bright, hipStream_t s, int shape = -1,
                    const SiteTab& tab = SiteTab{});
// Site probe: out[0] = 8-pixel groups sampled (kProbeGroups, spread over the
// launch's first <= 64 sites), out[1] / out[2] = those holding a value >=
// 4,096 / >= 16,384 (device words; the caller copies them to the host)
void launch_site_probe(const uint16_t* sites, int64_t npx, int64_t n_sites, unsigned int* out,
                       hipStream_t s, const SiteTab& tab = SiteTab{});
// vlh: the order statistics of the launch's first site (buffer + site *
// kOsTile) in a buffer with room for vlh_ld sites (kOsTile layout above)
void launch_hist_scatter(const uint16_t* sites, int64_t npx, int64_t n_sites, uint32_t* hist_hi,
                         const QPos& p, uint32_t* vlh, int64_t vlh_ld, unsigned long long* pooled,
                         int64_t* zero_counts, uint32_t* site_hist, hipStream_t s);
void launch_hist_finalize(uint32_t* hist, unsigned long long* rmask, int dense_rounds,
                          int64_t n_sites, const QPos& p, uint32_t* vlh, int64_t vlh_ld,
                          unsigned long long* pooled,
                          unsigned long long* pooled_parts, int n_parts, int64_t* zero_counts,
                          uint32_t* site_hist, hipStream_t s, bool narrow = false,
                          const unsigned long long* rm_all = nullptr,
                          const unsigned long long* wide = nullptr, unsigned long long xthr = 0);
// very wide launches: the exact per-site histogram in LDS as u16 pairs from
// one more read of the sites, scanned into order statistics (wide == null:
// unconditionally; else only when wide[1] >= xthr)
void launch_hist_site_u16(const uint16_t* sites, int64_t npx, int64_t n_sites, uint32_t* slab,
                          const QPos& p, uint32_t* vlh, int64_t vlh_ld,
                          unsigned long long* pooled, unsigned long long* pooled_parts,
                          int n_parts, int64_t* zero_counts, uint32_t* site_hist,
                          const unsigned long long* wide, unsigned long long xthr, hipStream_t s,
                          const SiteTab& tab = SiteTab{});
void launch_pct_accumulate(const uint32_t* vlh, int64_t n_sites, int64_t vlh_ld, int Q,
                           const double* gamma, double* acc, hipStream_t s);
// quantiles [q_begin, q_begin + q_count) only; acc points at the range
void launch_pct_accumulate_range(const uint32_t* vlh, int64_t n_sites, int64_t vlh_ld, int q_begin,
                                 int q_count, const double* gamma, double* acc, hipStream_t s,
                                 const unsigned long long* only_xwide = nullptr,
                                 unsigned long long xthr = 0);
// pooled[b] += sum over the sites of hist[s][b] for the rounds rmask names
// (rm_all: the launch-wide union of the masks, or null)
void launch_pooled_colsum(const uint32_t* hist, const unsigned long long* rmask,
                          const unsigned long long* rm_all, int64_t n_sites,
                          unsigned long long* pooled, hipStream_t s);
void launch_finalize(const double* mean, const double* m2, int64_t n, int64_t npx, double* out_mean,
                     double* out_std, hipStream_t s);
// var = M2 / (n - 1), NaN where n < 2 (stats.py:94-102)
void launch_variance(const double* m2, int64_t n, int64_t npx, double* out_var, hipStream_t s);
void launch_merge1(const double* mean, int64_t n, int64_t npx, double* nmean, hipStream_t s);
void launch_merge2(double* mean, const double* m2, int64_t n_r, const double* sum_nmean,
                   int64_t n_total, int64_t npx, double* m2c, hipStream_t s);
void launch_copy_f64(const double* src, double* dst, int64_t n, hipStream_t s);
struct ZeroList {
  unsigned long long* p[8];
  int64_t count[8];  // u64 elements
  int n = 0;
  void add(void* ptr, int64_t elems) {
    p[n] = static_cast<unsigned long long*>(ptr);
    count[n++] = elems;
  }
};
void launch_zero_u64(const ZeroList& z, hipStream_t s);
// Small u32 arrays zeroed in one launch (a multi-job corrected pass's
// per-job fixup counters and unit queues: one kernel, not a fill per array)
struct ZeroList32 {
  unsigned int* p[16];
  int count[16];  // u32 elements
  int n = 0;
  void add(void* ptr, int elems) {
    p[n] = static_cast<unsigned int*>(ptr);
    count[n++] = elems;
  }
};
void launch_zero_u32(const ZeroList32& z, hipStream_t s);

constexpr int kMaxJobs = 8;          // jobs (a rank's channels) of one multi-job launch
// Several fused jobs' histogram tails (same image size)
struct TailJob {
  uint32_t* hist;                  // the job's histogram slab (zero-maintained)
  unsigned long long* rmask;       // per site: rounds holding counts (zero-maintained)
  const unsigned long long* rm_all;  // the union of the masks
  QPos qp;                         // the handle's quantile table (tstride set)
  uint32_t* vlh;                   // order statistics of the job's first site
  unsigned long long* pooled;
  int64_t* zero_counts;
  uint32_t* site_hist;             // may be null
  int64_t n_sites;
};
struct TailJobs {
  TailJob j[kMaxJobs];
  int n;
};
void launch_hist_finalize_jobs(const TailJobs& J, hipStream_t s);
constexpr int kMaxPlanes = 2 * kMaxJobs;
void launch_smooth(const double* in, double* out, double* tmp, int H, int W, const double* d_w,
                   int radius, hipStream_t s);
// np <= kMaxPlanes planes; sq (may be null): per plane 0 = read as is, else
// the plane is M2 read as the finalized std sqrt(M2 / sq) (sq = n - 1; < 0:
// NaN), sigma 5 only
// psum / pmin (may be null): per plane the coefficient tiles' partial sums
// and smallest positive values (k_tile_sums' partition), written as the
// sigma-5 pass stores its outputs, or by k_tile_sums after the two-pass form
void launch_smooth_planes(const double* const* in, double* const* out, double* const* tmp,
                          const double* sq, int np, int H, int W, const double* d_w, int radius,
                          hipStream_t s, double* const* psum, double* const* pmin);
// Coefficient tiles: kSumTH rows x kSumTW columns of a plane (the sigma-5
// smoothing's workgroup tile); a plane's sums are fixed-order sums of its
// tiles' partials (deterministic, whichever kernel made them)
constexpr int kSumTH = 16, kSumTW = 216;
int coef_tiles(int H, int W);
void launch_tile_sums(const double* const* x, double* const* psum, double* const* pmin, int np,
                      int H, int W, hipStream_t s);
void launch_smooth2(const double* in0, const double* in1, double* out0, double* out1,
                    double* tmp0, double* tmp1, int H, int W, const double* d_w, int radius,
                    hipStream_t s);
void launch_build_corr_lut(float2* lut, int log_transform, double zero_log10, hipStream_t s);
// Per job (a corrector) of a coefficient launch: its (smoothed) mean / std
// planes, the reduction scratch (3 x n_partial) and sums (sum(std),
// sum(mean), min positive std), and every coefficient form (coef / coef_lin
// null: left out, launch_coeffs_forms makes them when needed; apply_kernels.hip
// k_coeffs_all: coef (LUT path, mconst = (M hi, M lo, T, 0)), coef2 / coef_lin
// / mconst2 (packed log2-domain path, fused_kernels.hip), coef64 (f64 (mean,
// std) for the refinement) and rc (RefineConst)).
struct CoefJobs {
  const double* mean[kMaxJobs];
  const double* std[kMaxJobs];
  double* partial[kMaxJobs];
  double* sums[kMaxJobs];
  float4* coef[kMaxJobs];
  float2* coef2[kMaxJobs];
  float2* coef_lin[kMaxJobs];
  double2* coef64[kMaxJobs];
  float4* mconst[kMaxJobs];
  float4* mconst2[kMaxJobs];
  RefineConst* rc[kMaxJobs];
  int log_transform[kMaxJobs];
  double zero_log10[kMaxJobs];
};
// partials_ready: J.partial already holds the tiles' sums (the smoothing wrote them)
void launch_coeffs_jobs(const CoefJobs& J, int n_jobs, int H, int W, bool partials_ready,
                        hipStream_t s);
// coef (LUT path) and coef_lin (chain) from coef64 + sums, for a job whose
// coefficient launch left them out (CoefJobs entries null)
void launch_coeffs_forms(const double2* coef64, const double* sums, int64_t npx, int log_transform,
                         float4* coef, float2* coef_lin, hipStream_t s);
// Refinement of the pixels a correct launch flagged (fl), written into out
// (u16 or u8 of in's type; clip as the launch); launched on the same stream.
void launch_fix_correct(const void* in, void* out, int elem_bytes, int64_t npx, int64_t n_sites,
                        const FixList& fl, const double2* coef64, const RefineConst* rc,
                        int log_transform, int clip_lo, int clip_hi, hipStream_t s,
                        const SiteTab& tab = SiteTab{});
// Several uint16 jobs' fixups in one launch (the multi-job fused pass)
struct FixJob {
  const uint16_t* in;
  uint16_t* out;
  int64_t n_sites;
  FixList fl;
  const double2* c64;
  const RefineConst* rc;
  SiteTab tab;
  unsigned long long* wide;  // the job's Welford wide counters to reset, or null
};
struct FixJobs {
  FixJob j[kMaxJobs];
  int n;
};
void launch_fix_correct_jobs(const FixJobs& J, int64_t npx, int log_transform, int clip_lo,
                             int clip_hi, hipStream_t s);
void launch_correct_u16(const uint16_t* in, uint16_t* out, int64_t npx, int64_t n_sites,
                        const float4* coef, const float2* lut, const float4* mconst,
                        const FixList& fl, int log_transform, int clip_lo, int clip_hi,
                        hipStream_t s);
void launch_correct_u8(const uint8_t* in, uint8_t* out, int64_t npx, int64_t n_sites,
                       const float4* coef, const float2* lut, const float4* mconst,
                       const FixList& fl, int log_transform, int clip_lo, int clip_hi,
                       hipStream_t s);
// fused pass configurations (fused_kernels.hip kFusedCfgs).  kFusedAuto picks
// per job on the host from the site probe: kFusedNarrow (four sites per unit,
// 4,096-bin slices) unless at least kWideFrac of the probed pixel groups hold
// a value >= 4,096, then kFusedWide: four sites, 16,384 bins
// each as u16 counters packed two sites to a word (round 3: 15.95-16.11 ms
// on 3,456 bright sites against 17.67-17.75 for configuration 0's two sites
// x 16,384 u32 bins, profiles/r3/ab_fused_packed_bright_r3z20.jsonl; round 2:
// configuration 0 18.6 ms against 22.4 for one site x 32,768 bins and 231 ms
// narrow, profiles/r2/mb_fused_bright_r2f.txt).
constexpr int kFusedConfigs = 6;
constexpr int kFusedQueueInts = 16;  // fused pass scratch: 8 unit counters + 64-bit round union
constexpr int kFusedAuto = -1;
constexpr int kFusedNarrow = 3;
constexpr int kFusedWide = 5;
constexpr double kWideFrac = 0.02;
// very wide: a third of the 8-pixel groups hold a value >= 16,384 (~5% of the
// pixels beyond the wide configuration's slices: from there its global atomics
// cost more than one more read of the sites); the fused pass then runs without
// its histogram and k_hist_site_u16 builds the histograms
constexpr double kXWideFrac = 0.33;
// the Welford pass's bright form: >= kBrightFrac of the probed groups hold a
// value >= 4,096
constexpr double kBrightFrac = 0.10;
// the fused pass without its histogram (very wide sites: k_hist_site_u16
// builds the histograms)
constexpr int kFusedNoHist = 100;
// cfg: 0 .. kFusedConfigs - 1 or kFusedNoHist -- exactly one launch; bands:
// pixel bands of the unit sweep (0: the configuration's, more for a short
// launch -- fused_kernels.hip fused_bands)
void launch_correct_hist(const uint16_t* in, uint16_t* out, int64_t npx, int64_t n_sites,
                         const float2* coef2, const float4* mconst2, const FixList& fl,
                         int log_transform, int clip_lo, int clip_hi, uint32_t* hist,
                         unsigned long long* rmask, int* queues, int n_wg, int cfg, int bands,
                         hipStream_t s, const SiteTab& tab = SiteTab{},
                         const RareList& rl = RareList{});
// One fused pass over several jobs (a rank's channels, same image size,
// configuration and transform): job j's units follow job j-1's in one sweep,
// each unit with its own job's sites, coefficients, histograms, round masks
// and fixup list.  uni: the job's round-mask union (its corrector's
// queues + 8, zeroed by the caller); queues: the launch's unit counters.
struct FusedJob {
  const uint16_t* in;
  uint16_t* out;
  int64_t n_sites;
  const float4* coef;     // coef2 as float4 planes
  const float4* mconst2;
  FixList fl;
  uint32_t* hist;
  unsigned long long* rmask;
  unsigned long long* uni;
  SiteTab tab;
  RareList rl;
};
struct FusedJobs {
  FusedJob j[kMaxJobs];
  int n;
};
void launch_correct_hist_jobs(const FusedJobs& J, int64_t npx, int log_transform, int clip_lo,
                              int clip_hi, int* queues, int n_wg, int cfg, int bands,
                              hipStream_t s);
// after launch_correct_hist with a RareList: each site's list into its
// histogram (hist + s * kBins), on the same stream
void launch_rare_count(const RareList& rl, uint32_t* hist, int64_t n_sites, hipStream_t s);
// illuminati chain (chain_kernels.hip)
void launch_align(const void* in, void* out, int elem_bytes, int64_t n_sites, int H, int W, int oh,
                  int ow, const tmh_window* d_win, hipStream_t s);
void launch_map_u8(const uint16_t* in, uint8_t* out, int64_t n, int lo, int hi, hipStream_t s);
// (launches its own fixup kernel after the chain pass; lut8: 64 KB of device
// scratch for the 16-bit clip + scale table, or null for the clipped-range one)
void launch_chain_u8(const uint16_t* in, uint8_t* out, int H, int W, int64_t n_sites,
                     const float2* coef_lin, const float4* mconst2, const FixList& fl,
                     const double2* coef64, const RefineConst* rc, int log_transform,
                     const tmh_window* d_win, int lo, int hi, uint8_t* lut8, hipStream_t s,
                     double zero_log10 = -10.0);
// site-image input (inflate_kernels.hip)
int64_t inflate_scratch_bytes(int64_t n_chunks, int64_t raw_max);
void launch_inflate(const uint8_t* src, int64_t src_bytes, const tmh_zchunk* chunks,
                    int64_t n_chunks, int64_t raw_max, uint8_t* dst, int64_t dst_bytes,
                    uint32_t* scratch, int32_t* status, hipStream_t s);
void launch_place_chunks(const uint8_t* raw, const tmh_zchunk* chunks, int64_t n_chunks,
                         int height, int width, int esize, int chunk_rows, int chunk_cols,
                         uint8_t* images, hipStream_t s);
void launch_clip_u16(const uint16_t* in, uint16_t* out, int64_t n, int lo, int hi, hipStream_t s);
void launch_synth(uint16_t* out, int64_t n_sites, int H, int W, uint64_t seed, int channel,
                  int64_t first_site, int dist, hipStream_t s);
void synth_tables_host(int dist, int H, int W, int32_t* ln, int32_t* nz, int32_t* ey, int32_t* ex);
// box probe (bench support, synth_kernels.hip): write = copy the sites to the
// output blocks, else read them; clk[4] = (clock64, wall_clock64) at workgroup
// 0's start and end
void launch_box_probe(const uint16_t* const* in_blocks, uint16_t* const* out_blocks, int shift,
                      int64_t n_sites, int64_t npx, int write, unsigned long long* clk,
                      unsigned int* sink, int n_cus, hipStream_t s);
// the flat shape: one 16-byte group per thread over one contiguous run of sites
void launch_box_probe_flat(const uint16_t* in, uint16_t* out, int64_t n_sites, int64_t npx,
                           int write, unsigned int* sink, hipStream_t s);

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace tmh
