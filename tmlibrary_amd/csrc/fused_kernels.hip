// Fused correct + per-site histogram pass (gfx950 / MI355X).
//
// The job reads every site twice at minimum: once for the Welford statistics
// (pixel-major, mean/M2 in registers across all sites) and once for the
// correction (which needs the finished, smoothed statistics).  The per-site
// intensity percentiles (stats.py:76) need nothing but the raw pixels, so
// their histograms are built from the correction's read instead of a pass of
// their own: HBM traffic is then the algorithmic 2 + 4 B/px per site.
//
// Layout of the work: the image is cut into n_bands = 16 pixel bands, and a
// unit is SPU sites of one band.  XCD x owns bands 2x and 2x+1 and deals
// their units band-major from its own counter (its L2 holds the coefficients
// of the band it is on -- 8 B/px: 2.76 MB per band at 2160x2560 -- while the
// site groups of every job of the launch stream through, the XCDs an eighth
// of the site groups apart), stealing from the next XCD's counter once its
// own is drained.
// Same-box job A/B (profiles/r2/ab_fused_sched_r2pqr.txt, ab_fused_dyn_r2zd.jsonl):
// this deal against round 1's per-XCD queues that each owned two whole bands,
// 13.8 vs 14.3 ms on one box, 14.5 vs 14.7 on another; against the same
// sweep dealt statically, +0.8% job throughput with one channel and +1.6%
// with four channels sharing the GPU (a static deal cannot rebalance when
// kernels co-run); every XCD on the same band ran 15.5 ms.  Each lane loads
// its 8 pixels' coefficients once per group and applies them to the SPU sites
// (L2 coefficient traffic 8/SPU B/px).  Each site of the unit histograms its
// raw pixels into its own LDS slice (values below kLdsBins/SPU; larger values
// go straight to the global histogram), and at the end of the unit the slices
// are added to the sites' global histograms with contiguous-lane atomics.
//
// Arithmetic (ChannelImage._correct_illumination, tmlib/image.py:599-631), in
// the log2 domain so 10**t is one v_exp_f32:
//   t2 = (log2(img) - mean*log2(10)) * a + mean(mean)*log2(10),  a = mean(std)/std
//      = log2(img) * a + c,  c = (mean(mean) - mean*a)*log2(10)  (per pixel, f32)
//   out = astype_uint16_x86(2**t2)
// log2 is v_log_f32 (<= 1 ulp: <= 0.1 DN at 65535); a and c are f32 (c's
// rounding adds <= 0.05*a DN at 65535); zero pixels take the reference's
// log10(1e-10) = -10.  Parity bar: +-1 DN.
#include "common.h"

namespace tmh {

constexpr int kFusedBands = 16;  // pixel bands of the unit sweep
// cache policy bits of the site loads and corrected stores (2: streamed,
// non-temporal); overridable at build time for A/B builds
#ifndef TMH_FUSED_LOAD_AUX
#define TMH_FUSED_LOAD_AUX 2
#endif
#ifndef TMH_FUSED_STORE_AUX
#define TMH_FUSED_STORE_AUX 2
#endif
constexpr int kFusedLoadAux = TMH_FUSED_LOAD_AUX, kFusedStoreAux = TMH_FUSED_STORE_AUX;

// A pointer every lane holds the same value of, moved to scalar registers: a
// buffer resource built from a pointer loaded with a vector load (a block
// table entry) would otherwise live in VGPRs, and the compiler wraps every
// buffer load and store that uses it in a waterfall loop.
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7;
}

typedef float f32x2_t __attribute__((ext_vector_type(2)));

// The f32 error bound (common.h): |o| (K1 a + K2) < 1 keeps the truncated
// value within 1 DN of the f64 one; K1, K2 carry a 0.2% margin for the f32
// evaluation of the bound itself.
constexpr float kBoundK1 = (float)(kRefineK1 * 1.002), kBoundK2 = (float)(kRefineK2 * 1.002);

// The bound factor K1 a + K2 of a pixel group's largest a (monotone in a, so
// no pixel of the group has a larger one): computed once per group for all
// the unit's sites.  NaN a's drop out of the max (their pixels are not
// flagged, as before).
__device__ __forceinline__ float group_bound(const float4 (&k)[4]) {
  float am = __builtin_fmaxf(__builtin_fmaxf(k[0].z, k[0].w), __builtin_fmaxf(k[1].z, k[1].w));
  am = __builtin_fmaxf(am, __builtin_fmaxf(__builtin_fmaxf(k[2].z, k[2].w),
                                           __builtin_fmaxf(k[3].z, k[3].w)));
  return __builtin_fmaf(am, kBoundK1, kBoundK2);
}

// Eight pixels (four packed u16 words) -> their corrected u16 values packed
// the same way.  k[p] = (c_lo, c_hi, a_lo, a_hi) of word p's two pixels, c =
// (M - mean * a) [* log2 10] with a already rounded to f32 (k_coeffs_all), so
//   t2 = log2(x) * a + c
// is one v_pk_fma_f32 per pair (the reference's (log x - mean) * a + M with
// one rounding of c instead of the rounded mean, the subtraction and the
// rounded M: the error stays within the bound below).  Each stage is issued
// for all four pairs before the next so dependent packed ops do not stall on
// their one-pass hazard.  A zero pixel takes log2(zf), zf = 10**zero_log10 as
// f32 (1e-10f: v_log_f32 is within 1 ulp of the reference's log10(1e-10) =
// -10, scaled): one v_max instead of a compare + select.  The caller keeps zf
// in [FLT_MIN, 1].  Returns the mask of the pixels whose f32 result may be
// more than 1 DN off (their own error bound): the caller flags them for the
// f64 refinement (common.h) -- rare, saturated pixels in dim corners.  The
// common path tests the group once: its largest |o| against bmax (the group's
// largest bound factor, group_bound); only a group that passes that test
// (the return value) has its pixels' own bounds evaluated, by the caller
// (far_mask, inside a branch that also stages the fixups, so the compiler
// cannot if-convert the per-pixel work into the common path).
template <bool LOG, bool CLIP>
__device__ __forceinline__ bool fcorrect8(const uint32_t (&w)[4], const float4 (&k)[4], float zf,
                                          float bmax, uint32_t clip_lo2, uint32_t clip_hi2,
                                          uint32_t (&r)[4], float (&o)[8]) {
  f32x2_t t[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    t[p].x = (float)(w[p] & 0xFFFFu);
    t[p].y = (float)(w[p] >> 16);
  }
  if (LOG) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      t[p].x = __builtin_amdgcn_logf(__builtin_fmaxf(t[p].x, zf));  // v_log_f32
      t[p].y = __builtin_amdgcn_logf(__builtin_fmaxf(t[p].y, zf));
    }
  }
#pragma unroll
  for (int p = 0; p < 4; ++p)
    t[p] = __builtin_elementwise_fma(t[p], (f32x2_t){k[p].z, k[p].w}, (f32x2_t){k[p].x, k[p].y});
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    o[2 * p] = LOG ? __builtin_amdgcn_exp2f(t[p].x) : t[p].x;  // v_exp_f32
    o[2 * p + 1] = LOG ? __builtin_amdgcn_exp2f(t[p].y) : t[p].y;
  }
  auto mag = [](float v) { return LOG ? v : __builtin_fabsf(v); };  // log: o = 2**t >= 0 (or NaN)
  float mx = __builtin_fmaxf(mag(o[0]), mag(o[1]));
#pragma unroll
  for (int j = 2; j < 8; ++j) mx = __builtin_fmaxf(mx, mag(o[j]));
  // No clamp before the cast: an unflagged |o| is below 1 / K2 < 2^18, where
  // v_cvt_i32_f32 truncates exactly as the reference's x86 cast does, and a
  // flagged pixel's value is rewritten by the f64 refinement (every |o| >=
  // 1 / K2, +-inf included, is flagged; NaN -- never flagged -- converts to 0,
  // the low half of the reference's INT32_MIN).
  int32_t iv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) iv[j] = (int32_t)o[j];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    r[p] = __builtin_amdgcn_perm((uint32_t)iv[2 * p + 1], (uint32_t)iv[2 * p], 0x05040100u);
    if (CLIP) {  // np.clip on the wrapped uint16 values, both halves at once
      typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
      u16x2_t v = __builtin_bit_cast(u16x2_t, r[p]);
      v = __builtin_elementwise_min(__builtin_elementwise_max(v, __builtin_bit_cast(u16x2_t, clip_lo2)),
                                    __builtin_bit_cast(u16x2_t, clip_hi2));
      r[p] = __builtin_bit_cast(uint32_t, v);
    }
  }
  return mx * bmax >= 0.998f;
}

// The pixels of a flagged group beyond their own f32 bound (bit j: pixel j)
__device__ __forceinline__ uint32_t far_mask(const float4 (&k)[4], const float (&o)[8]) {
  uint32_t far = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float b0 = __builtin_fmaf(k[p].z, kBoundK1, kBoundK2);
    const float b1 = __builtin_fmaf(k[p].w, kBoundK1, kBoundK2);
    far |= (__builtin_fabsf(o[2 * p]) * b0 >= 0.998f ? 1u : 0u) << (2 * p);
    far |= (__builtin_fabsf(o[2 * p + 1]) * b1 >= 0.998f ? 2u : 0u) << (2 * p);
  }
  return far;
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void st_nt(uint4* p, uint4 v) {
  const u32x4_t w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(p));
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

// ABL: development ablations (tools/mb), 0 in production: 1 = no histogram,
// 2 = constant coefficients, 8 = no flush, 32 = no arithmetic, 64 = values
// beyond the slices not staged (the rare path's loop skipped).
// NT threads per workgroup, LB LDS bins per workgroup (split into SPU slices
// of BINS counters plus one overflow counter each: a pixel >= BINS adds to the
// overflow counter -- never read -- and to its global bin, so the common path
// is one v_min + one ds_add per pixel).
// Each workgroup issues its next unit's first loads before it flushes the
// current unit's histogram slices, so the flush (LDS scan + global atomics +
// barriers) runs with the next unit's pixels already in flight.
// PK (packed): the LDS counters are u16 halves of 32-bit words -- sites 2j
// and 2j+1 share word array j (one ds_add of 1 or 0x10000 per pixel, no
// extra VALU), so four sites get 16,384 bins each in 128 KB.  A half can
// wrap only if one value fills more than 65,535 pixels of a site's band, so
// every unit's flush first sums each site's counters (plus the site's
// pixels that took the global path) against the band's pixel count; a site
// whose sum falls short is recounted from its pixels with global atomics
// instead of flushed.
template <bool LOG, bool CLIP, int SPU, int ABL, int NT, int LB, bool PK = false>
__global__ __launch_bounds__(NT, (LB * 4 > 80 * 1024 && NT <= 512) ? 2 : 4) void k_correct_hist(
    const FusedJobs J, int64_t npx, int clip_lo, int clip_hi, int n_bands,
    int* __restrict__ queues) {
  constexpr int BINS = LB / SPU;
  constexpr int SLICE = BINS + 1;
  constexpr int NSL = PK ? SPU / 2 : SPU;  // word arrays (PK: two sites per array)
  constexpr uint32_t HIMASK = (0xFFFFu & ~(uint32_t)(BINS - 1)) * 0x00010001u;
  static_assert((BINS & (BINS - 1)) == 0, "slice size must be a power of two");
  static_assert(!PK || (SPU % 2 == 0 && BINS <= 16384), "packed: site pairs, u16 headroom");
  __shared__ __attribute__((aligned(16))) uint32_t bins[NSL * SLICE];
  __shared__ uint32_t pk_red[PK ? NT / 64 : 1][PK ? SPU : 1];  // packed: per-wave site sums
  static_assert(!PK || BINS == kRareLo, "rare lists start at the packed slice size");
  // packed with a rare list: the unit's values beyond the slices, per site
  constexpr int kRareSh = PK ? 3072 : 1;  // the rest of the 160 KB of LDS (r4: 1,024)
  __shared__ uint16_t rstage[PK ? SPU : 1][kRareSh];
  __shared__ unsigned int rcnt[PK ? SPU : 1], rbase[PK ? SPU : 1];
  uint32_t rare[SPU];  // packed: this thread's pixels of the unit beyond the slices (list or atomic)
#pragma unroll
  for (int k = 0; k < SPU; ++k) rare[k] = 0u;
  // per site of the unit: the 1,024-bin rounds holding counts (the rare
  // global adds and, at the flush, the slice's non-empty rounds); two sets,
  // alternating by unit, so one is published while the next unit fills the
  // other.  k_hist_finalize reads exactly these rounds.
  __shared__ unsigned long long rm_sh[2][SPU];
  // f64 fixups: the pixel groups a unit flags are staged in LDS (two sets,
  // alternating by unit like rm_sh) and appended to the global list by wave 0
  // after the unit's flush.  (A global atomic with a return value in the pixel
  // loop makes the compiler wait, wherever it is taken, for every load in
  // flight -- the next stage's included.)
  constexpr int kFixSh = 256;
  __shared__ unsigned long long fix_sh[2][kFixSh];
  __shared__ unsigned int fix_cnt[2];
  const int tid = threadIdx.x;
  for (int i = tid; i < NSL * SLICE; i += NT) bins[i] = 0u;
  if (tid < 2 * SPU) rm_sh[tid / SPU][tid % SPU] = 0ull;
  if (PK && tid < SPU) rcnt[tid] = 0u;
  if (tid < 2) fix_cnt[tid] = 0u;
  __syncthreads();

  const uint32_t clo2 = (uint32_t)clip_lo * 0x00010001u, chi2 = (uint32_t)clip_hi * 0x00010001u;
  const int ngroups = (int)(npx >> 3);
  const int site_bytes = (int)(npx * 2);
  int n_groups_all = 0;  // every job's site groups
  for (int j = 0; j < J.n; ++j) n_groups_all += (int)((J.j[j].n_sites + SPU - 1) / SPU);
  const int n_units = n_bands * n_groups_all;
  const float4 cc = make_float4(2.5f, 2.4f, 1.1f, 0.9f);

  // Unit order: XCD x deals the units i = x + 8 j from its own counter
  // (queues[x]), stealing from the next queue once its own is drained, and
  // owns the bands [x * n_bands / 8, (x + 1) * n_bands / 8): its j-th unit is
  // band x * n_bands / 8 + j / G, site group (j + x * (G / 8)) % G of the G
  // site groups of every job of the launch (job after job).  So each XCD's L2
  // holds one band of coefficients at a time and reads each job's band once
  // per launch (round 5's sweep walked every XCD over every band: a
  // multi-job launch re-read each job's 44 MB of coefficient planes once per
  // XCD, ~1.4 GB per 4 x 432-site step), and the XCDs stay G/8 site groups
  // apart: with every XCD on the same or neighbouring site groups (different
  // bands of the same sites at once) the single-job pass ran 4% slower
  // (profiles/r6/ab_fused_sweep_xcd_bands_r6j.jsonl).  The next unit is
  // grabbed while the current one streams.
  __shared__ int unit_sh;
  int q = xcc_id(), exhausted = 0;
  auto grab = [&]() -> int {
    while (exhausted < 8) {
      if (tid == 0) unit_sh = atomicAdd(&queues[q], 1);
      __syncthreads();
      const int j = __builtin_amdgcn_readfirstlane(unit_sh);
      __syncthreads();
      const int i = q + 8 * j;
      if (i < n_units) {
        exhausted = 0;
        return i;
      }
      q = (q + 1) & 7;  // this queue is drained: steal from the next
      ++exhausted;
    }
    return -1;
  };
  struct Unit {
    int job, g0, g1, ns;
    int64_t s0;
    __amdgpu_buffer_rsrc_t rin, rout;  // the unit's SPU sites; loads past ns read 0
    // coefficient planes: plane k holds (mu, mu, a, a) of pixels 8g+2k,
    // 8g+2k+1 of group g, so each of a lane's four coefficient loads is one
    // contiguous 1 KiB per wave
    __amdgpu_buffer_rsrc_t rcf;
  };
  auto decode = [&](int i) -> Unit {
    Unit r;
    const int j8 = i >> 3;
    const int band = (i & 7) * (n_bands >> 3) + j8 / n_groups_all;
    int job = 0, grp = (j8 + (i & 7) * (n_groups_all >> 3)) % n_groups_all;
    for (;; ++job) {  // the unit's job (uniform: every lane the same)
      const int n_groups_s = (int)((J.j[job].n_sites + SPU - 1) / SPU);
      if (job + 1 >= J.n || grp < n_groups_s) break;
      grp -= n_groups_s;
    }
    const FusedJob& jb = J.j[job];
    r.job = job;
    r.s0 = (int64_t)grp * SPU;
    r.ns = (int)(jb.n_sites - r.s0 < SPU ? jb.n_sites - r.s0 : SPU);
    r.g0 = (int)((int64_t)band * ngroups / n_bands);
    r.g1 = (int)((int64_t)(band + 1) * ngroups / n_bands);
    const uint16_t* ib = jb.in + r.s0 * npx;
    uint16_t* ob = jb.out + r.s0 * npx;
    if (jb.tab.in) {  // blocked layout: the unit's sites lie inside one block
      const int64_t b = site_block(jb.tab, r.s0), o = site_in_block(jb.tab, r.s0) * npx;
      ib = jb.tab.in[b] + o;
      ob = jb.tab.out[b] + o;
    }
    r.rin = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(ib), 0, r.ns * site_bytes,
                                              0x00020000);
    r.rout = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(ob), 0, r.ns * site_bytes,
                                               0x00020000);
    r.rcf = __builtin_amdgcn_make_buffer_rsrc((void*)jb.coef, 0, (int)(npx * 8), 0x00020000);
    return r;
  };
  // a lane whose group lies past the unit's band loads from past the buffers'
  // ends: raw buffer loads there return 0 without touching memory, so every
  // load of the pixel loop is unconditional and the compiler's wait before a
  // stage counts exactly the loads issued after it
  constexpr int kOOB = 0x7FFFFF00;
  auto load = [&](const Unit& un, int g, uint4 (&v)[SPU], float4 (&c)[4]) {
    const int off = g < un.g1 ? g * 16 : kOOB;
#pragma unroll
    for (int k = 0; k < SPU; ++k) {
      // (a site past a partial unit's last: its own out-of-range offset)
      const u32x4_t w = __builtin_amdgcn_raw_buffer_load_b128(un.rin, k < un.ns ? off : kOOB,
                                                              k * site_bytes, kFusedLoadAux);
      v[k] = make_uint4(w.x, w.y, w.z, w.w);
    }
    if (!(ABL & 2)) {
#pragma unroll
      for (int p = 0; p < 4; ++p)
        c[p] = __builtin_bit_cast(float4,
                                  __builtin_amdgcn_raw_buffer_load_b128(un.rcf, off, p * ngroups * 16, 0));
    }
  };

  uint4 vA[SPU], vB[SPU];
  float4 cA[4] = {cc, cc, cc, cc}, cB[4] = {cc, cc, cc, cc};
#pragma unroll
  for (int k = 0; k < SPU; ++k) vA[k] = vB[k] = make_uint4(0, 0, 0, 0);
  bool pre = false;  // v/c already hold this unit's first group (loaded by the previous unit)
  int cur = grab(), par = 0;
  while (cur >= 0) {
    unsigned long long* rm = rm_sh[par];
    const int nxt = grab();
    const Unit un = decode(cur);
    Unit nu = un;
    if (nxt >= 0) nu = decode(nxt);
    const FusedJob& jb = J.j[un.job];
    const float4 m = jb.mconst2[0];
    const FixList fl = jb.fl;
    const RareList rl = jb.rl;
    const bool rlist = PK && rl.v != nullptr;
    uint32_t* hs = jb.hist + un.s0 * (int64_t)kBins;

    auto process = [&](const uint4 w, const int k, const float4 (&cf)[4], const float bmax,
                       const int g, const bool ok) -> u32x4_t {
      const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
      if (!(ABL & 1) && ok) {
        uint32_t* sl = bins + (PK ? k >> 1 : k) * SLICE;
        const uint32_t inc = PK && (k & 1) ? 0x10000u : 1u;  // compile-time per site
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const uint32_t lo = wd[p] & 0xFFFFu, hi = wd[p] >> 16;
          atomicAdd(&sl[lo < (uint32_t)BINS ? lo : (uint32_t)BINS], inc);
          atomicAdd(&sl[hi < (uint32_t)BINS ? hi : (uint32_t)BINS], inc);
        }
        if ((w.x | w.y | w.z | w.w) & HIMASK) {  // rare: beyond this site's LDS slice
          uint32_t* h = hs + k * (int64_t)kBins;
          unsigned long long rounds = 0ull;  // 1,024-bin rounds this site touches
          // the lane's rare halves as a bit mask (bit 2p + j: half j of word p),
          // then one iteration per rare half: a wave runs max-popcount
          // iterations (~1-2 on bright sites) instead of eight masked sections
          uint32_t msk = 0u;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const uint32_t t = wd[p] & HIMASK;
            msk |= ((t & 0xFFFFu) ? 1u : 0u) << (2 * p);
            msk |= ((t >> 16) ? 2u : 0u) << (2 * p);
          }
          if (PK) rare[k] += __builtin_popcount(msk);
          if (ABL & 64) msk = 0u;  // (ablation: counted for the wrap check, not staged)
          while (msk) {
            const uint32_t b = __builtin_ctz(msk);
            msk &= msk - 1u;
            const uint32_t p = b >> 1;
            const uint32_t word = p == 0 ? wd[0] : p == 1 ? wd[1] : p == 2 ? wd[2] : wd[3];
            const uint32_t v = (word >> ((b & 1u) << 4)) & 0xFFFFu;
            bool staged = false;
            if (rlist) {
              const unsigned int i = atomicAdd(&rcnt[k], 1u);  // LDS
              if (i < (unsigned int)kRareSh) {
                rstage[k][i] = (uint16_t)v;
                staged = true;
              }
            }
            if (!staged) atomicAdd(&h[v], 1u);
            rounds |= 1ull << (v >> 10);
          }
          atomicOr(&rm[k], rounds);  // LDS: published once per unit
        }
      }
      uint32_t o[4];
      if (ABL & 32) {  // no arithmetic: the pixels pass through (coefficients kept live)
        const u32x4_t r = {w.x ^ (__float_as_uint(cf[0].x) & 1u), w.y ^ (__float_as_uint(cf[1].y) & 1u),
                           w.z ^ (__float_as_uint(cf[2].z) & 1u), w.w ^ (__float_as_uint(cf[3].w) & 1u)};
        return r;
      }
      float of[8];
      if (fcorrect8<LOG, CLIP>(wd, cf, m.z, bmax, clo2, chi2, o, of) && ok) {  // rare
        const uint32_t far = far_mask(cf, of);
        if (far) {
          const unsigned int i = atomicAdd(&fix_cnt[par], 1u);
          if (i < (unsigned int)kFixSh)
            fix_sh[par][i] = fix_code8(far, un.s0 + k, (int64_t)g * 8);
          else
            fix_push8(fl, far, un.s0 + k, (int64_t)g * 8);  // rare: the unit's LDS set is full
        }
      }
      const u32x4_t r = {o[0], o[1], o[2], o[3]};
      return r;
    };

    // two stages (A, B) over the unit's pixel groups, a uniform number of
    // steps; A holds the unit's first group when the previous unit loaded it.
    // Every stage issues all SPU stores, a lane past the band or a site past
    // a partial unit's last with an out-of-range offset (dropped): with the
    // stores under a branch, a path that skips them issues fewer memory
    // operations, and the compiler's wait at the loop head was s_waitcnt
    // vmcnt(0) (loads and the previous stores drained) instead of vmcnt(4).
    // Measured neutral (12.82 vs 12.83 ms, profiles/r6/mb_stream_r6e/f.txt).
    auto stage = [&](const uint4 (&v)[SPU], const float4 (&cf)[4], int g) {
      const bool live = g < un.g1;
      const float bmax = group_bound(cf);  // once per group for the unit's sites
#pragma unroll
      for (int k = 0; k < SPU; ++k) {
        const bool ok = live && k < un.ns;
        __builtin_amdgcn_raw_buffer_store_b128(process(v[k], k, cf, bmax, g, ok), un.rout,
                                               ok ? g * 16 : kOOB, k * site_bytes,
                                               kFusedStoreAux);
      }
    };
    const int iters = (un.g1 - un.g0 + NT - 1) / NT;
    int g = un.g0 + tid;
    if (!pre) load(un, g, vA, cA);
    pre = false;
    for (int it = 0; it < iters; it += 2) {
      load(un, g + NT, vB, cB);
      stage(vA, cA, g);
      g += NT;
      if (it + 1 >= iters) break;
      load(un, g + NT, vA, cA);
      stage(vB, cB, g);
      g += NT;
    }
    // the next unit's first group is in flight during this unit's flush
    if (nxt >= 0) {
      load(nu, nu.g0 + tid, vA, cA);
      pre = true;
    }
    cur = nxt;
    if (ABL & 9) continue;
    __syncthreads();
    if (PK) {
      // the check: each site's counters (a wrapped half comes up 65,536
      // short) plus its global-path pixels against the band's pixel count
      uint32_t sum[SPU];
#pragma unroll
      for (int k = 0; k < SPU; ++k) sum[k] = rare[k];
#pragma unroll
      for (int j = 0; j < NSL; ++j) {
#pragma unroll 4
        for (int b = tid; b < BINS; b += NT) {
          const uint32_t w = bins[j * SLICE + b];
          sum[2 * j] += w & 0xFFFFu;
          sum[2 * j + 1] += w >> 16;
        }
      }
      if (rlist) {  // the unit's staged rare values to their sites' lists
        if (tid < SPU) {
          const unsigned int n = rcnt[tid] < (unsigned int)kRareSh ? rcnt[tid] : kRareSh;
          rbase[tid] = (tid < un.ns && n) ? atomicAdd(&rl.cnt[un.s0 + tid], n) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < SPU; ++k) {
          const unsigned int n = rcnt[k] < (unsigned int)kRareSh ? rcnt[k] : kRareSh;
          if (k >= un.ns) break;
          uint16_t* dst = rl.v + (un.s0 + k) * (int64_t)rl.cap;
          for (unsigned int i = tid; i < n; i += NT) {
            const unsigned int j = rbase[k] + i;
            const uint16_t v = rstage[k][i];
            if (j < rl.cap)
              dst[j] = v;
            else
              atomicAdd(&hs[k * (int64_t)kBins + v], 1u);  // past the list's capacity
          }
        }
        __syncthreads();
        if (tid < SPU) rcnt[tid] = 0u;
      }
      const int wv = tid >> 6;
#pragma unroll
      for (int k = 0; k < SPU; ++k) {
        uint32_t v = sum[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
        if ((tid & 63) == 0) pk_red[wv][k] = v;
        rare[k] = 0u;
      }
      __syncthreads();
      const uint32_t band_px = (uint32_t)(un.g1 - un.g0) * 8u;
      uint32_t bad = 0;  // sites whose counters wrapped
#pragma unroll
      for (int k = 0; k < SPU; ++k) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) t += pk_red[w][k];
        if (k < un.ns && t != band_px) bad |= 1u << k;
      }
#pragma unroll
      for (int j = 0; j < NSL; ++j) {
        uint32_t* h0 = hs + (2 * j) * (int64_t)kBins;
        uint32_t* h1 = hs + (2 * j + 1) * (int64_t)kBins;
        const bool ok0 = 2 * j < un.ns && !((bad >> (2 * j)) & 1u);
        const bool ok1 = 2 * j + 1 < un.ns && !((bad >> (2 * j + 1)) & 1u);
        unsigned long long lm0 = 0ull, lm1 = 0ull;
#pragma unroll 4
        for (int b = tid; b < BINS; b += NT) {
          const uint32_t w = bins[j * SLICE + b];
          if (w) {
            const uint32_t c0 = w & 0xFFFFu, c1 = w >> 16;
            if (c0 && ok0) {
              atomicAdd(&h0[b], c0);
              lm0 |= 1ull << (b >> 10);
            }
            if (c1 && ok1) {
              atomicAdd(&h1[b], c1);
              lm1 |= 1ull << (b >> 10);
            }
            bins[j * SLICE + b] = 0u;
          }
        }
        if (lm0) atomicOr(&rm[2 * j], lm0);
        if (lm1) atomicOr(&rm[2 * j + 1], lm1);
      }
      if (bad) {  // rare: recount those sites' band pixels below BINS exactly
        const uint16_t* ib = jb.in + un.s0 * npx;
        if (jb.tab.in) ib = jb.tab.in[site_block(jb.tab, un.s0)] + site_in_block(jb.tab, un.s0) * npx;
        for (int k = 0; k < SPU; ++k) {
          if (!((bad >> k) & 1u)) continue;
          uint32_t* h = hs + k * (int64_t)kBins;
          const uint16_t* src = ib + k * npx;
          unsigned long long lm = 0ull;
          for (int64_t i = (int64_t)un.g0 * 8 + tid; i < (int64_t)un.g1 * 8; i += NT) {
            const uint32_t v = src[i];
            if (v < (uint32_t)BINS) {
              atomicAdd(&h[v], 1u);
              lm |= 1ull << (v >> 10);
            }
          }
          if (lm) atomicOr(&rm[k], lm);
        }
      }
    } else {
    // fold this unit's slices into the sites' histograms (contiguous lanes ->
    // bins); the overflow counters are left to wrap, they are never read
#pragma unroll
    for (int k = 0; k < SPU; ++k) {
      if (k >= un.ns) break;
      uint32_t* h = hs + k * (int64_t)kBins;
      unsigned long long lm = 0ull;  // this thread's non-empty rounds
#pragma unroll 4
      for (int b = tid; b < BINS; b += NT) {
        const uint32_t cnt = bins[k * SLICE + b];
        if (cnt) {
          atomicAdd(&h[b], cnt);
          bins[k * SLICE + b] = 0u;
          lm |= 1ull << (b >> 10);
        }
      }
      if (lm) atomicOr(&rm[k], lm);
    }
    }
    __syncthreads();
    // publish the unit's round masks; the next unit fills the other set, and
    // this one is not touched again before the next unit's first barrier
    if (tid < un.ns) {
      const unsigned long long r = rm[tid];
      if (r) {
        atomicOr(&jb.rmask[un.s0 + tid], r);
        atomicOr(jb.uni, r);  // the job's union
      }
      rm[tid] = 0ull;
    }
    // append the unit's staged fixups (wave 0; the set is next written two
    // units on, after barriers wave 0 reaches only when done here)
    if (tid < 64) {
      const unsigned int nf = fix_cnt[par] < (unsigned int)kFixSh ? fix_cnt[par] : kFixSh;
      if (nf) {
        unsigned int base = 0u;
        if (tid == 0) base = atomicAdd(fl.n, nf);
        base = __builtin_amdgcn_readfirstlane(base);
        for (unsigned int i = tid; i < nf; i += 64)
          if (base + i < fl.cap) fl.e[base + i] = fix_sh[par][i];
      }
      if (tid == 0) fix_cnt[par] = 0u;
    }
    par ^= 1;
  }
}

// (sites per unit, threads, LDS bins) of the fused pass, selected per handle
// (tmh_stats_set_option, TMH_OPT_FUSED_CONFIG) or automatically per job
// (kFusedAuto: kFusedNarrow, or kFusedWide when the sites are bright).
// bands: pixel bands of the unit sweep -- 8 for the wide configuration, whose
// 16,384-bin slices flush more counts per unit (fewer, longer units: 17.3 vs
// 17.95 ms on bright sites, profiles/r2/mb_shape_bright_r2x.txt), 16 otherwise.
struct FusedCfg {
  int spu, threads, lds_bins, bands;
  bool packed;  // u16 counters, two sites per word (k_correct_hist PK)
};
constexpr FusedCfg kFusedCfgs[kFusedConfigs] = {{2, 1024, 32768, 8, false},
                                                {4, 1024, 32768, kFusedBands, false},
                                                {2, 512, 16384, kFusedBands, false},
                                                {4, 512, 16384, kFusedBands, false},
                                                {1, 1024, 32768, kFusedBands, false},
                                                {4, 1024, 65536, 8, true}};
template <int K>
struct FusedCfgCheck {
  static_assert((kFusedCfgs[K].lds_bins / kFusedCfgs[K].spu) % 1024 == 0,
                "LDS slices must cover whole 1,024-bin rounds");
  static constexpr bool ok = true;
};
static_assert(FusedCfgCheck<0>::ok && FusedCfgCheck<1>::ok && FusedCfgCheck<2>::ok &&
              FusedCfgCheck<3>::ok && FusedCfgCheck<4>::ok && FusedCfgCheck<5>::ok, "");

// Pixel bands of a launch: the configuration's, doubled (up to 64) while the
// launch has fewer than 8 units per workgroup -- a short launch (a rank's
// 432-site share of a channel at N = 8: 108 site groups x 16 bands over 512
// workgroups) otherwise ends with most workgroups idle for a unit's time.
// bands > 0: that many (TMH_OPT_FUSED_BANDS).
static int fused_bands(int cfg_bands, int64_t n_sites, int spu, int64_t n_wgs, int bands) {
  if (bands > 0) return bands;
  int b = cfg_bands;
  const int64_t groups = (n_sites + spu - 1) / spu;
  while (b < 64 && groups * b < 8 * n_wgs) b *= 2;
  return b;
}

static void launch_correct_hist_cfg(const FusedJobs& J, int64_t npx, int log_transform,
                                    int clip_lo, int clip_hi, int* queues, int n_wg, int cfg,
                                    int bands_opt, hipStream_t s) {
  int64_t n_sites = 0;  // the bands see the launch's site groups, every job's
#define TMH_LAUNCH_CH(L_, K_, A_)                                                                \
  {                                                                                              \
    constexpr FusedCfg c = kFusedCfgs[K_];                                                       \
    const dim3 grid(n_wg * (1024 / c.threads));                                                  \
    for (int j = 0; j < J.n; ++j) n_sites += (J.j[j].n_sites + c.spu - 1) / c.spu * c.spu;      \
    const int nbands = fused_bands(c.bands, n_sites, c.spu, grid.x, bands_opt);                  \
    FusedJobs Jc = J;                                                                            \
    if (!c.packed)                                                                               \
      for (int j = 0; j < J.n; ++j) Jc.j[j].rl = RareList{};                                     \
    if (clip_lo >= 0)                                                                            \
      hipLaunchKernelGGL((k_correct_hist<L_, true, c.spu, A_, c.threads, c.lds_bins, c.packed>), \
                         grid, dim3(c.threads), 0, s, Jc, npx, clip_lo, clip_hi, nbands, queues); \
    else                                                                                         \
      hipLaunchKernelGGL((k_correct_hist<L_, false, c.spu, A_, c.threads, c.lds_bins, c.packed>), \
                         grid, dim3(c.threads), 0, s, Jc, npx, clip_lo, clip_hi, nbands, queues); \
  }
#define TMH_LAUNCH_CFG(L_)                                     \
  switch (cfg) {                                               \
    case 0: TMH_LAUNCH_CH(L_, 0, 0) break;                     \
    case 1: TMH_LAUNCH_CH(L_, 1, 0) break;                     \
    case 2: TMH_LAUNCH_CH(L_, 2, 0) break;                     \
    case 3: TMH_LAUNCH_CH(L_, 3, 0) break;                     \
    case 5: TMH_LAUNCH_CH(L_, 5, 0) break;                     \
    case kFusedNoHist: TMH_LAUNCH_CH(L_, kFusedNarrow, 1) break; \
    default: TMH_LAUNCH_CH(L_, 4, 0) break;                    \
  }
  if (log_transform) {
    TMH_LAUNCH_CFG(true);
  } else {
    TMH_LAUNCH_CFG(false);
  }
#undef TMH_LAUNCH_CFG
#undef TMH_LAUNCH_CH
  TMH_HIP(hipGetLastError());
}

// One launch of configuration cfg (chosen by the caller: abi.hip picks it per
// job from the host-read site probe, so no losing configuration is queued).
// The round masks name every non-empty round whatever the configuration, so
// the histogram finalize is the same.  The "correct_hist" timing bracket
// holds the kernel alone (the scratch reset is outside it), so the bench's
// per-launch rate is the pass's own.
void launch_correct_hist(const uint16_t* in, uint16_t* out, int64_t npx, int64_t n_sites,
                         const float2* coef2, const float4* mconst2, const FixList& fl,
                         int log_transform, int clip_lo, int clip_hi, uint32_t* hist,
                         unsigned long long* rmask, int* queues, int n_wg, int cfg, int bands,
                         hipStream_t s, const SiteTab& tab, const RareList& rl) {
  if (n_sites <= 0) return;
  // queues[0..8): per-XCD unit counters; queues[8..10): the union of the
  // sites' round masks (read by the pooled column sum)
  TMH_HIP(hipMemsetAsync(queues, 0, kFusedQueueInts * sizeof(int), s));
  FusedJobs J{};
  J.n = 1;
  J.j[0] = FusedJob{in, out, n_sites, reinterpret_cast<const float4*>(coef2), mconst2, fl, hist,
                    rmask, reinterpret_cast<unsigned long long*>(queues + 8), tab, rl};
  ProfScope prof("correct_hist", s);
  launch_correct_hist_cfg(J, npx, log_transform, clip_lo, clip_hi, queues, n_wg, cfg, bands, s);
}

// Several jobs in one launch (the caller zeroed queues and every job's uni).
void launch_correct_hist_jobs(const FusedJobs& J, int64_t npx, int log_transform, int clip_lo,
                              int clip_hi, int* queues, int n_wg, int cfg, int bands,
                              hipStream_t s) {
  if (J.n <= 0) return;
  ProfScope prof("correct_hist", s);
  launch_correct_hist_cfg(J, npx, log_transform, clip_lo, clip_hi, queues, n_wg, cfg, bands, s);
}

// Each site's rare list into its histogram: one workgroup per site, the
// values [kRareLo, 65536) counted in LDS in two halves of 24,576 bins, then
// added to the site's bins (the fused pass has finished: plain adds).  The
// fused pass already marked the rounds these values touch.
constexpr int kRareHalf = (65536 - kRareLo) / 2;
__global__ __launch_bounds__(1024) void k_rare_count(const RareList rl, uint32_t* __restrict__ hist,
                                                     int64_t n_sites) {
  __shared__ uint32_t c[kRareHalf];
  for (int64_t site = blockIdx.x; site < n_sites; site += gridDim.x) {  // uniform per workgroup
  const unsigned int cnt = rl.cnt[site];
  const unsigned int n = cnt < rl.cap ? cnt : rl.cap;
  if (n == 0u) continue;
  const uint16_t* v = rl.v + site * (int64_t)rl.cap;
  uint32_t* h = hist + site * (int64_t)kBins;
  for (int half = 0; half < 2; ++half) {
    const uint32_t lo = (uint32_t)kRareLo + (uint32_t)half * kRareHalf;
    for (int i = threadIdx.x; i < kRareHalf; i += 1024) c[i] = 0u;
    __syncthreads();
    for (unsigned int i = threadIdx.x; i < n; i += 1024) {
      const uint32_t u = (uint32_t)v[i] - lo;
      if (u < (uint32_t)kRareHalf) atomicAdd(&c[u], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kRareHalf; i += 1024)
      if (c[i]) h[lo + i] += c[i];
    __syncthreads();
  }
  }
}

void launch_rare_count(const RareList& rl, uint32_t* hist, int64_t n_sites, hipStream_t s) {
  if (n_sites <= 0 || !rl.v) return;
  const unsigned grid = (unsigned)(n_sites < 256 ? n_sites : 256);  // one workgroup per CU (96 KB LDS)
  hipLaunchKernelGGL(k_rare_count, dim3(grid), dim3(1024), 0, s, rl, hist, n_sites);
  TMH_HIP(hipGetLastError());
}

}  // namespace tmh
