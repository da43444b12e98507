// Order statistics of one site's histogram (np.percentile 'linear' previous /
// next sorted values, tmlib/workflow/corilla/stats.py:75-76) written from its
// counts: shared by the standalone finalize kernels (stats_kernels.hip) and
// the fused pass's in-pass finalize (fused_kernels.hip).
#pragma once

#include "common.h"

namespace tmh {

// Exclusive scan of one value per thread over an NT-thread workgroup.
// `slots` holds 2 x 16 wave totals (double-buffered by the parity of the
// caller's scan counter, so one barrier per scan suffices).  Returns the
// exclusive prefix; *total = sum.
template <int NT>
__device__ __forceinline__ uint32_t block_exscan_t(uint32_t c, uint32_t* slots, int round,
                                                   uint32_t* total) {
  static_assert(NT % 64 == 0 && NT <= 1024, "whole waves, at most 16");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t incl = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  uint32_t* ws = slots + (round & 1) * 16;
  if (lane == 63) ws[wid] = incl;
  __syncthreads();
  uint32_t woff = 0, all = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const uint32_t t = ws[w];
    woff += (w < wid) ? t : 0u;
    all += t;
  }
  *total = all;
  return woff + incl - c;
}

__device__ __forceinline__ uint32_t block_exscan(uint32_t c, uint32_t* slots, int round,
                                                 uint32_t* total) {
  return block_exscan_t<kHistThreads>(c, slots, round, total);
}

constexpr int kRound = 1024;  // histogram bins per round of the scans

constexpr int kTailChunkDefault = 8;  // rounds whose counts are loaded together
// Advance (t, Rt = R[t]) to the first index >= t with R[index] > x (R: LEN
// non-decreasing inclusive prefix ranks in LDS; the caller guarantees
// R[t - 1] <= x < R[LEN - 1]).  Consecutive quantile positions mostly stay in
// one bin (no LDS read: Rt is cached) or step to the next (one read); the
// rest finish with a binary search over (t+1, 1023].
template <int LEN = kRound>
__device__ __forceinline__ void advance_rank(const int32_t* R, int& t, int32_t& Rt, int32_t x) {
  if (Rt > x) return;
  const int32_t r1 = R[t + 1];
  if (r1 > x) {
    ++t;
    Rt = r1;
    return;
  }
  int lo = t + 1, hi = LEN - 1;  // R[lo] <= x < R[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (R[mid] > x)
      hi = mid;
    else
      lo = mid;
  }
  t = hi;
  Rt = R[hi];
}

// One round's order statistics.  R[t] = inclusive prefix rank of the round's
// bin t (value bin0 + t); the round owns the sorted positions [r0, r1).
// Quantile-centric: each thread takes groups of 8 quantiles, reads their
// previous positions from the (L2-resident) table -- the next group's
// positions are loaded while the current group is resolved -- keeps the ones
// inside [r0, r1), and finds each owning bin by advancing through R from the
// previous quantile's bin (one binary search per group).  The next position
// is min(prev + 1, n - 1) for every q in [0, 100] (np.percentile 'linear'):
// when it is still inside the previous statistic's bin (R[bin] > prev + 1,
// nearly always) the next statistic is the same value and needs no search; a
// general next table is read only if the caller's differs.  Each group is
// written as one 32-B store of interleaved (previous, next) values (2-B
// stores where a group straddles the round's ends).  The round's quantile
// range is [r0 * scale, r1 * scale] up to rounding (and one position's worth
// of quantiles), so the groups scanned carry a margin and the position test
// decides membership exactly.
template <int NT = kHistThreads, int LEN = kRound>
__device__ __forceinline__ void fill_groups(const int32_t* R, int64_t r0, int64_t r1,
                                            uint32_t bin0, const QPos& p,
                                            uint32_t* __restrict__ vlh, bool vec16) {
  const int64_t m = (int64_t)p.scale + 3;  // scale > 1 when Q exceeds the pixel count
  int64_t qa = (int64_t)((double)r0 * p.scale) - m;
  int64_t qb = (int64_t)((double)r1 * p.scale) + m;
  qa = qa < 0 ? 0 : qa;
  qb = qb > p.Q ? p.Q : qb;
  if (qa >= qb) return;
  const int64_t g0 = qa >> 3, g1 = (qb - 1) >> 3;
  const bool tab16 = vec16;  // tables are 16-B aligned rows when Q % 8 == 0 (hipMalloc base)
  const int32_t a = (int32_t)r0, b = (int32_t)r1;
  auto positions = [&](int64_t q0, int32_t (&pl)[8]) {
    if (tab16 && q0 + 8 <= p.Q) {
      const int4 a0 = reinterpret_cast<const int4*>(p.lo + q0)[0];
      const int4 a1 = reinterpret_cast<const int4*>(p.lo + q0)[1];
      pl[0] = a0.x; pl[1] = a0.y; pl[2] = a0.z; pl[3] = a0.w;
      pl[4] = a1.x; pl[5] = a1.y; pl[6] = a1.z; pl[7] = a1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) pl[j] = q0 + j < p.Q ? p.lo[q0 + j] : INT32_MAX;
    }
  };
  int64_t g = g0 + (int64_t)threadIdx.x;
  int32_t pn[8];
  if (g <= g1) positions(g << 3, pn);
  for (; g <= g1; g += NT) {
    const int64_t q0 = g << 3;
    int32_t pl[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) pl[j] = pn[j];
    if (g + NT <= g1) positions((g + NT) << 3, pn);  // in flight while this group resolves
    int tl = 0, th = 0;
    int32_t Rl = R[0], Rh = Rl;
    uint32_t ol[4] = {0u, 0u, 0u, 0u}, oh[4] = {0u, 0u, 0u, 0u};
    uint32_t ml = 0, mh = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int32_t pj = pl[j];
      const bool mine = pj >= a && pj < b;
      if (mine) {
        advance_rank<LEN>(R, tl, Rl, pj);
        ol[j >> 1] |= (bin0 + (uint32_t)tl) << (16 * (j & 1));
        ml |= 1u << j;
      }
      const int32_t hj = p.hi_next ? (pj < p.last ? pj + 1 : pj)
                                   : (q0 + j < p.Q ? p.hi[q0 + j] : INT32_MAX);
      if (p.hi_next && mine && hj < Rl) {  // next position in the same bin
        oh[j >> 1] |= (bin0 + (uint32_t)tl) << (16 * (j & 1));
        mh |= 1u << j;
      } else if (hj >= a && hj < b) {
        if (th < tl) {
          th = tl;
          Rh = Rl;
        }
        advance_rank<LEN>(R, th, Rh, hj);
        oh[j >> 1] |= (bin0 + (uint32_t)th) << (16 * (j & 1));
        mh |= 1u << j;
      }
    }
    // interleaved (previous, next) order statistics: one u32 per quantile,
    // a group of 8 is contiguous inside one quantile tile
    uint32_t* og = vlh + (q0 / kOsTile) * p.tstride + (q0 % kOsTile);
    if (vec16 && ml == 0xFFu && mh == 0xFFu) {
      uint4* dst = reinterpret_cast<uint4*>(og);
      dst[0] = make_uint4(__builtin_amdgcn_perm(oh[0], ol[0], 0x05040100u),
                          __builtin_amdgcn_perm(oh[0], ol[0], 0x07060302u),
                          __builtin_amdgcn_perm(oh[1], ol[1], 0x05040100u),
                          __builtin_amdgcn_perm(oh[1], ol[1], 0x07060302u));
      dst[1] = make_uint4(__builtin_amdgcn_perm(oh[2], ol[2], 0x05040100u),
                          __builtin_amdgcn_perm(oh[2], ol[2], 0x07060302u),
                          __builtin_amdgcn_perm(oh[3], ol[3], 0x05040100u),
                          __builtin_amdgcn_perm(oh[3], ol[3], 0x07060302u));
    } else if (ml | mh) {  // a round edge: write the halves this round owns
      uint16_t* h16 = reinterpret_cast<uint16_t*>(og);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if ((ml >> j) & 1u) h16[2 * j] = (uint16_t)(ol[j >> 1] >> (16 * (j & 1)));
        if ((mh >> j) & 1u) h16[2 * j + 1] = (uint16_t)(oh[j >> 1] >> (16 * (j & 1)));
      }
    }
  }
}

// hist_tail for a histogram whose possibly non-empty 1,024-bin rounds are
// known up front (need: bit j = round j): only those rounds are loaded, and
// they are scanned SR rounds at a time (a super-round of SR * 1,024 bins: one
// block scan and one rank table per super-round that holds any needed round,
// bins of the rounds not needed taken as 0 without a load) -- BPT = SR *
// 1024 / NT consecutive bins per thread, the next super-round's counts in
// flight while the current one is scanned -- instead of walking all 64
// rounds.  Same outputs as hist_tail (site_hist rows are zero-filled for the
// rounds not visited).  NT = 256, SR = 1 is the narrow form that fits beside
// the fused pass's workgroups on a CU.  starts: 2 * SR * 1024 int32 of LDS.
template <int ABL, int NT, int SR, typename CountFn, typename DoneFn>
__device__ __forceinline__ void hist_tail_rounds(unsigned long long need, CountFn count,
                                                 DoneFn done, int64_t s, const QPos& p,
                                                 uint32_t* __restrict__ vlh_all,
                                                 unsigned long long* __restrict__ pooled,
                                                 int64_t* __restrict__ zero_counts,
                                                 uint32_t* __restrict__ site_hist,
                                                 uint32_t* slots, int32_t* starts) {
  constexpr int LEN = SR * kRound;
  constexpr int BPT = LEN / NT;
  static_assert(BPT >= 1 && kRound % BPT == 0, "a thread's bins lie inside one round");
  const int tid = threadIdx.x;
  uint32_t* vlh = vlh_all + s * (int64_t)kOsTile;  // this site's column of the tiles
  const bool vec16 = (p.Q & 7) == 0;
  if (site_hist) {  // debug/parity copy: the rounds not visited are empty
    for (int j = 0; j < kBins / kRound; ++j)
      if (!((need >> j) & 1ull))
        for (int i = tid; i < kRound; i += NT) site_hist[s * kBins + (uint32_t)(j * kRound + i)] = 0u;
  }
  unsigned long long sneed = 0ull;  // super-rounds holding a needed round
#pragma unroll
  for (int k = 0; k < kBins / LEN; ++k)
    if ((need >> (k * SR)) & ((SR == 64 ? 0ull : (1ull << SR)) - 1ull)) sneed |= 1ull << k;
  // bin 0 lies in super-round 0: a site whose masks skip it has no zeros
  if (zero_counts && tid == 0 && !(sneed & 1ull)) zero_counts[s] = 0;
  // this thread's bins lie in round (k * SR + tid * BPT / kRound) of super-round k
  auto load = [&](int k, uint32_t (&c)[BPT]) {
    const uint32_t b0 = (uint32_t)k * LEN + tid * BPT;
    const bool live = (need >> (b0 / kRound)) & 1ull;
#pragma unroll
    for (int i = 0; i < BPT; ++i) c[i] = live ? count(b0 + i) : 0u;
  };
  int64_t base = 0;  // exclusive rank of the current super-round's first bin
  int nscan = 0;
  uint32_t cn[BPT];
  if (sneed) load(__builtin_ctzll(sneed), cn);
  while (sneed) {
    const int k = __builtin_ctzll(sneed);
    sneed &= sneed - 1ull;
    uint32_t c[BPT], inc[BPT];
#pragma unroll
    for (int i = 0; i < BPT; ++i) c[i] = cn[i];
    if (sneed) load(__builtin_ctzll(sneed), cn);
    const uint32_t b0 = (uint32_t)k * LEN + tid * BPT;
    const bool live = (need >> (b0 / kRound)) & 1ull;
    uint32_t run = 0;
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      run += c[i];
      inc[i] = run;  // inclusive prefix inside the thread's bins
      const uint32_t b = b0 + i;
      if (live) {
        if (site_hist) site_hist[s * kBins + b] = c[i];
        done(b, c[i]);
      }
      if (b == 0 && zero_counts) zero_counts[s] = c[i];
    }
    uint32_t total;
    // slots and R are double-buffered by scan parity: every scan flips it
    const int64_t r = base + block_exscan_t<NT>(run, slots, nscan, &total);
    int32_t* R = starts + (nscan & 1) * LEN;
    ++nscan;
    if (total == 0) continue;  // uniform: an empty super-round
    const int64_t r0 = base;
    base += total;
#pragma unroll
    for (int i = 0; i < BPT; ++i)
      if (c[i] && !(ABL & 4) && pooled) atomicAdd(&pooled[b0 + i], (unsigned long long)c[i]);
    if (ABL & 1) continue;
#pragma unroll
    for (int i = 0; i < BPT; ++i) R[tid * BPT + i] = (int32_t)(r + inc[i]);
    __syncthreads();  // R visible; the other R buffer is rewritten only after the next scan
    fill_groups<NT, LEN>(R, r0, base, (uint32_t)k * LEN, p, vlh, vec16);
  }
}

}  // namespace tmh
