// C-ABI of libtmhip.so (include/tmhip.h): handles, device memory, launches.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"

namespace tmh {

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

template <typename F>
static int guard(F&& f) {
  try {
    f();
    return TMH_OK;
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_error("host allocation failed");
    return TMH_ENOMEM;
  } catch (...) {
    set_error("unknown error");
    return TMH_EDEVICE;
  }
}

// ---------------------------------------------------------------------------
// per-kernel event timing
// ---------------------------------------------------------------------------
struct ProfSlot {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  double total_ms = 0.0;
  int64_t launches = 0;
};
static std::mutex g_prof_mu;
static bool g_prof_on = false;
static std::map<std::string, ProfSlot> g_prof;

ProfScope::ProfScope(const char* name, hipStream_t s) : name_(name), s_(s), slot_(nullptr) {
  if (!g_prof_on) return;
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
  (void)hipEventRecord(a, s);
  std::lock_guard<std::mutex> lk(g_prof_mu);
  auto& slot = g_prof[name];
  slot.pending.emplace_back(a, b);
  slot_ = &slot;
}

ProfScope::~ProfScope() {
  if (!slot_) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  auto* slot = static_cast<ProfSlot*>(slot_);
  (void)hipEventRecord(slot->pending.back().second, s_);
}

static void prof_drain(ProfSlot& slot) {
  for (auto& p : slot.pending) {
    float ms = 0.f;
    (void)hipEventSynchronize(p.second);
    if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) slot.total_ms += ms;
    slot.launches += 1;
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  slot.pending.clear();
}

// ---------------------------------------------------------------------------
// device buffers
// ---------------------------------------------------------------------------
template <typename T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  void alloc(size_t count, bool zero = false) {
    release();
    if (count == 0) return;
    if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) {
      p = nullptr;
      throw Error{TMH_ENOMEM, "hipMalloc of " + std::to_string(count * sizeof(T)) + " bytes failed"};
    }
    n = count;
    if (zero) {
      // null-stream memset: our launches run on non-blocking streams, so wait
      TMH_HIP(hipMemset(p, 0, count * sizeof(T)));
      TMH_HIP(hipDeviceSynchronize());
    }
  }
  void ensure(size_t count, bool zero = false) {
    if (count > n) alloc(count, zero);
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  ~DBuf() { release(); }
};

// ---------------------------------------------------------------------------
// host staging of the host-buffer entry points (tmh_stats_update,
// tmh_correct_u16): two device slots and two pinned host slots per direction,
// copy streams separate from the compute stream, so the copies of chunk k
// overlap the kernels (and, for correct, the opposite-direction copy) of
// chunk k-1 instead of alternating copy -> kernel -> synchronize.
// ---------------------------------------------------------------------------
struct PinBuf {
  void* p = nullptr;
  size_t n = 0;
  void ensure(size_t bytes) {
    if (bytes <= n) return;
    release();
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      throw Error{TMH_ENOMEM, "hipHostMalloc of " + std::to_string(bytes) + " bytes failed"};
    }
    n = bytes;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
  ~PinBuf() { release(); }
};

// memcpy between pageable and pinned host memory, split over up to max_t
// threads (TMH_OPT_COPY_THREADS, default 8): one thread moves <= 30 GB/s and
// much less into a fresh (unfaulted) numpy output, below a PCIe 5 x16 link.
static void par_copy(void* dst, const void* src, size_t bytes, int max_t) {
  const size_t min_part = (size_t)4 << 20;
  size_t nt = std::min<size_t>((size_t)std::max(1, max_t), std::max<size_t>(1, bytes / min_part));
  nt = std::min<size_t>(nt, std::max(1u, std::thread::hardware_concurrency()));
  if (nt <= 1) {
    std::memcpy(dst, src, bytes);
    return;
  }
  const size_t part = ((bytes + nt - 1) / nt + 63) & ~(size_t)63;
  std::vector<std::thread> ts;
  for (size_t i = 1; i < nt; ++i) {
    const size_t b = i * part;
    if (b >= bytes) break;
    const size_t e = std::min(bytes, b + part);
    ts.emplace_back([=] { std::memcpy((char*)dst + b, (const char*)src + b, e - b); });
  }
  std::memcpy(dst, src, std::min(bytes, part));
  for (auto& t : ts) t.join();
}

// Staging of the host-buffer entry points (TMH_OPT_HOST_STAGING).  Measured
// on MI355X boxes (tools/diag_host.py, bench extras.host_path): the runtime's
// own pageable H2D path already reaches ~56 GB/s, above a pinned bounce fed by
// 8 host threads, so by default inputs go straight from the caller's buffer;
// outputs land in pinned slots and are copied out by several threads, which
// also spreads the first-touch page faults of a fresh numpy output.
// 0: everything direct; 1: inputs through pinned slots too; 2 (default).
constexpr int kStagingDirect = 0, kStagingPinnedIn = 1, kStagingPinnedOut = 2;

struct HostOpts {
  int copy_threads = 8;
  int staging = kStagingPinnedOut;
  bool set(int option, int value) {
    if (option == TMH_OPT_COPY_THREADS) {
      TMH_CHECK(value >= 1 && value <= 64, TMH_EINVAL, "copy threads must be 1..64");
      copy_threads = value;
      return true;
    }
    if (option == TMH_OPT_HOST_STAGING) {
      TMH_CHECK(value >= 0 && value <= 2, TMH_EINVAL, "host staging must be 0, 1 or 2");
      staging = value;
      return true;
    }
    return false;
  }
};

struct HostPipe {
  PinBuf in[2], out[2];
  hipStream_t h2d = nullptr, d2h = nullptr;
  hipEvent_t ev_in[2]{}, ev_kern[2]{}, ev_done[2]{};
  bool busy[2] = {false, false};
  int64_t s0[2] = {0, 0}, ns[2] = {0, 0};
  void init() {
    if (h2d) return;
    TMH_HIP(hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking));
    TMH_HIP(hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
      TMH_HIP(hipEventCreateWithFlags(&ev_in[i], hipEventDisableTiming));
      TMH_HIP(hipEventCreateWithFlags(&ev_kern[i], hipEventDisableTiming));
      TMH_HIP(hipEventCreateWithFlags(&ev_done[i], hipEventDisableTiming));
    }
  }
  // after an error mid-call: let queued work finish, forget the chunks (their
  // host destinations belong to the failed call)
  void abandon(hipStream_t compute) {
    if (h2d) (void)hipStreamSynchronize(h2d);
    if (d2h) (void)hipStreamSynchronize(d2h);
    if (compute) (void)hipStreamSynchronize(compute);
    busy[0] = busy[1] = false;
  }
  ~HostPipe() {
    if (!h2d) return;
    (void)hipStreamSynchronize(h2d);
    (void)hipStreamSynchronize(d2h);
    for (int i = 0; i < 2; ++i) {
      (void)hipEventDestroy(ev_in[i]);
      (void)hipEventDestroy(ev_kern[i]);
      (void)hipEventDestroy(ev_done[i]);
    }
    (void)hipStreamDestroy(h2d);
    (void)hipStreamDestroy(d2h);
  }
};

}  // namespace tmh

using namespace tmh;

struct tmh_stats {
  int device = 0;
  int H = 0, W = 0;
  int64_t npx = 0;
  int Q = 0;
  double scale = 0.0;
  unsigned flags = 0;
  int64_t batch_cap = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;   // histogram pass runs here, concurrent with Welford
  // the fused pass's histogram tail when the pass runs on another stream
  // (correct_hist_dev).  (At the lowest priority, with the caller's streams
  // above it, a two-jobs-in-flight bench ran 4-6% slower: profiles/r4/
  // ab_jobs_in_flight_priority_r4y.txt.)
  hipStream_t tail = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;  // ordering against a caller's stream
  // work on other streams the handle's stream must wait for, joined lazily
  // (hstream): a wait enqueued at once would sit in the stream's hardware
  // queue ahead of unrelated work of every stream sharing that queue until
  // the awaited pass had finished
  static constexpr int kJoins = 8;
  hipEvent_t join_ev[kJoins]{};
  hipStream_t join_s[kJoins]{};  // one entry per stream: a later record supersedes
  int join_n = 0;
  int fused_cfg = kFusedAuto;     // TMH_OPT_FUSED_CONFIG (-1: per launch, on the device)
  int wf_parts = 0;               // TMH_OPT_WELFORD_PARTS (0: automatic)
  HostOpts host;                  // TMH_OPT_COPY_THREADS / TMH_OPT_HOST_STAGING
  bool hist_dirty = false;        // a fused launch may have left counts / round masks behind
  int64_t n = 0;              // sites accumulated (Welford count)
  int64_t n_deferred = 0;     // sites whose order statistics are stored
  int64_t last_batch = 0;
  int64_t pending = 0;        // Welford-updated sites whose histograms are still to come
  DBuf<unsigned long long> wide;  // pixel groups with a value >= 4,096 / >= 16,384 in the pending sites
  // The job's site probe (k_site_probe, first Welford launch after a reset):
  // 8-pixel groups sampled, those with a value >= 4,096, >= 16,384.  The host
  // reads the counts once per job and launches only the Welford pass and the
  // fused configuration they call for (stats_choice).
  DBuf<unsigned int> probe;
  unsigned int* probe_host = nullptr;  // pinned copy
  hipEvent_t ev_probe = nullptr;
  bool probed = false;
  bool probe_queued = false;  // tmh_stats_probe_device: launched, not yet read
  unsigned int probe_cnt[3] = {0u, 0u, 0u};
  int64_t wide_sites = 0;         // sites that count covers
  bool pct_sum_external = false;
  DBuf<double> mean, m2, lut_log, gamma, acc, tmp_mean, tmp_std, rn;
  DBuf<double> wf_part;  // partial (mean, M2) planes of site-split Welford launches
  DBuf<int32_t> q_lo, q_hi;
  DBuf<unsigned long long> pooled, pooled_parts;  // parts: kPooledParts zero-maintained copies
  DBuf<uint32_t> hist_hi, site_hist, hist_full;
  DBuf<unsigned long long> hist_rmask;  // per site: touched high rounds of hist_full
  DBuf<uint16_t> rare_v;                // fused pass, packed configuration: per-site rare lists
  DBuf<unsigned int> rare_n;
  QPos qp{};
  DBuf<uint16_t> stage;  // two device slots of batch_cap sites
  HostPipe pipe;
  DBuf<uint32_t> vlh;  // order statistics (previous | next << 16), quantile-tiled (common.h)
  int64_t vlh_cap = 0;   // deferred mode: sites the tiles have room for
  int64_t vlh_ld = 0;    // tile stride in sites of the current contents
  DBuf<int64_t> zeros;
};

struct tmh_corrector {
  int device = 0;
  int H = 0, W = 0;
  int64_t npx = 0;
  int log_transform = 1;
  double zero_log10 = -10.0;
  hipStream_t stream = nullptr;
  DBuf<float4> coef, mconst, mconst2;
  DBuf<float2> lut, coef2, coef_lin;
  DBuf<double2> coef64;              // f64 (mean, std): the refinement's operands
  DBuf<RefineConst> rc;
  DBuf<unsigned long long> fix_e;    // pixels flagged for the f64 refinement (common.h)
  DBuf<unsigned int> fix_n;
  DBuf<tmh_window> win;  // per-site alignment windows of the chain pass
  DBuf<uint8_t> lut8;    // the chain pass's 16-bit clip + scale table (64 KB)
  int n_wg = 256;
  int bands = 0;     // TMH_OPT_FUSED_BANDS (0: automatic)
  bool forms_stale = false;  // coef / coef_lin not made since the last coefficient update
  DBuf<int> queues;  // fused pass: per-XCD unit counters (dynamic deal)
  DBuf<double> sums, partial;
  DBuf<uint16_t> stage_in, stage_out;
  DBuf<uint8_t> stage8_in, stage8_out;
  HostPipe pipe;
  HostOpts host;  // TMH_OPT_COPY_THREADS / TMH_OPT_HOST_STAGING
  // a histogram tail still reading queues (round masks) on a statistics
  // handle's stream (correct_hist_dev, cross-stream calls)
  hipEvent_t ev_tail = nullptr;
  bool tail_pending = false;
};

static hipStream_t pick(hipStream_t own, void* s) { return s ? (hipStream_t)s : own; }

// The handle's stream for new work: first it waits for the work on other
// streams joined since its last use (defer_join).
static hipStream_t hstream(tmh_stats* h) {
  for (int i = 0; i < h->join_n; ++i) TMH_HIP(hipStreamWaitEvent(h->stream, h->join_ev[i], 0));
  h->join_n = 0;
  return h->stream;
}

// The stream of an entry point: the caller's, or the handle's (joins first).
static hipStream_t hpick(tmh_stats* h, void* stream) {
  return stream ? (hipStream_t)stream : hstream(h);
}

// The handle's stream must wait for the work queued on s so far: recorded
// now, waited for when the handle's stream is next used (or by the next
// cross-stream call, directly).  One entry per stream.
static void defer_join(tmh_stats* h, hipStream_t s) {
  int i = 0;
  while (i < h->join_n && h->join_s[i] != s) ++i;
  if (i == tmh_stats::kJoins) {  // full: join them now
    hstream(h);
    i = 0;
  }
  hipEvent_t& e = h->join_ev[i];
  if (!e) TMH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  TMH_HIP(hipEventRecord(e, s));
  h->join_s[i] = s;
  if (i == h->join_n) ++h->join_n;
}

// Stream contract of the statistics entry points that take a stream
// (include/tmhip.h): on another stream than the handle's, the work runs after
// everything queued on the handle's stream (and the work joined to it), and
// the handle's stream waits for it before any later work on the handle.
// Nothing is queued on the handle's stream here: s waits for the joined
// work's events itself.
static void cross_begin(tmh_stats* h, hipStream_t s) {
  if (s == h->stream) {
    hstream(h);
    return;
  }
  TMH_HIP(hipEventRecord(h->ev_in, h->stream));
  TMH_HIP(hipStreamWaitEvent(s, h->ev_in, 0));
  for (int i = 0; i < h->join_n; ++i)
    if (h->join_s[i] != s) TMH_HIP(hipStreamWaitEvent(s, h->join_ev[i], 0));
}
static void cross_end(tmh_stats* h, hipStream_t s) {
  if (s == h->stream) return;
  defer_join(h, s);
}

constexpr int kPooledParts = 16;

extern "C" {

int tmh_abi_version(void) { return TMH_ABI_VERSION; }
const char* tmh_last_error(void) { return g_last_error.c_str(); }

int tmh_device_count(int* n) {
  return guard([&] {
    TMH_CHECK(n, TMH_EINVAL, "n is NULL");
    TMH_HIP(hipGetDeviceCount(n));
  });
}

int tmh_set_device(int device) { return guard([&] { TMH_HIP(hipSetDevice(device)); }); }

int tmh_synchronize(void* stream) {
  return guard([&] {
    if (stream)
      TMH_HIP(hipStreamSynchronize((hipStream_t)stream));
    else
      TMH_HIP(hipDeviceSynchronize());
  });
}

// ---------------------------------------------------------------------------
// stats
// ---------------------------------------------------------------------------

// words of order statistics for n sites (quantile tiles of kOsTile)
static size_t os_words(const tmh_stats* h, int64_t n_sites) {
  return (size_t)n_sites * (size_t)os_tiles(h->Q) * kOsTile;
}

static void stats_reserve_sites(tmh_stats* h, int64_t n_sites) {
  // growing frees buffers earlier launches may still be using
  const bool grow = (size_t)n_sites * kHiBins > h->hist_hi.n || (size_t)n_sites > h->zeros.n ||
                    ((h->flags & 2u) && (size_t)n_sites * kBins > h->site_hist.n) ||
                    (!(h->flags & TMH_STATS_DEFERRED_PCT) && os_words(h, n_sites) > h->vlh.n);
  if (grow) {
    TMH_HIP(hipStreamSynchronize(hstream(h)));
    TMH_HIP(hipStreamSynchronize(h->side));
  }
  // per-site slabs: hist_hi stays all-zero between launches (the kernel
  // resets what it touched), so it is zeroed only when (re)allocated.
  if ((size_t)n_sites * kHiBins > h->hist_hi.n) h->hist_hi.alloc((size_t)n_sites * kHiBins, true);
  h->zeros.ensure((size_t)n_sites);
  if (h->flags & 2u) h->site_hist.ensure((size_t)n_sites * kBins);
  if (!(h->flags & TMH_STATS_DEFERRED_PCT)) {
    h->vlh.ensure(os_words(h, n_sites));
  }
}

// Deferred mode keeps every site's order statistics: room for n_deferred +
// extra sites, growing geometrically; the tiles' stride is the capacity, so a
// growth re-lays the stored sites out (one 2-D copy: a row per tile).
static void stats_grow_deferred(tmh_stats* h, int64_t extra) {
  const int64_t need = h->n_deferred + extra;
  if (need <= h->vlh_cap) {
    h->vlh_ld = h->vlh_cap;
    return;
  }
  const int64_t cap = std::max(need, 2 * h->vlh_cap);
  DBuf<uint32_t> nb;
  nb.alloc(os_words(h, cap));
  if (h->n_deferred) {
    const size_t row = (size_t)kOsTile * 4;
    TMH_HIP(hipMemcpy2DAsync(nb.p, (size_t)cap * row, h->vlh.p, (size_t)h->vlh_cap * row,
                             (size_t)h->n_deferred * row, (size_t)os_tiles(h->Q),
                             hipMemcpyDeviceToDevice, hstream(h)));
  }
  TMH_HIP(hipStreamSynchronize(hstream(h)));
  TMH_HIP(hipStreamSynchronize(h->side));
  std::swap(h->vlh.p, nb.p);
  std::swap(h->vlh.n, nb.n);
  h->vlh_cap = cap;
  h->vlh_ld = cap;
}

int tmh_stats_create(int height, int width, int n_quantiles, const int64_t* q_lo,
                     const int64_t* q_hi, const double* q_gamma, const double* lut_log10,
                     int batch_capacity, unsigned flags, tmh_stats** out) {
  return guard([&] {
    TMH_CHECK(out, TMH_EINVAL, "out is NULL");
    TMH_CHECK(height > 0 && width > 0, TMH_EINVAL, "image dimensions must be positive");
    const int64_t npx = (int64_t)height * width;
    TMH_CHECK(npx < (int64_t(1) << 31), TMH_EINVAL, "images must have fewer than 2^31 pixels");
    TMH_CHECK(n_quantiles > 0 && q_lo && q_hi && q_gamma && lut_log10, TMH_EINVAL,
              "quantile tables and LUT are required");
    auto* h = new tmh_stats();
    try {
      TMH_HIP(hipGetDevice(&h->device));
      h->H = height;
      h->W = width;
      h->npx = npx;
      h->Q = n_quantiles;
      h->scale = (npx > 1) ? (double)(n_quantiles - 1) / (double)(npx - 1) : 0.0;
      h->flags = flags;
      h->batch_cap = std::min(4096, batch_capacity > 0 ? batch_capacity : 1);
      TMH_HIP(hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking));
      TMH_HIP(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));

      TMH_HIP(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
      TMH_HIP(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
      TMH_HIP(hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming));
      TMH_HIP(hipEventCreateWithFlags(&h->ev_out, hipEventDisableTiming));
      h->stream = h->own_stream;
      h->mean.alloc(npx, true);
      h->m2.alloc(npx, true);
      h->wf_part.alloc((size_t)8 * npx);
      h->wide.alloc(2, true);  // groups with a value >= 4,096 / >= 16,384
      h->probe.alloc(3);
      TMH_HIP(hipHostMalloc((void**)&h->probe_host, 4 * sizeof(unsigned int), hipHostMallocDefault));
      TMH_HIP(hipEventCreateWithFlags(&h->ev_probe, hipEventDisableTiming));
      h->acc.alloc(n_quantiles, true);
      h->pooled.alloc(kBins, true);
      h->lut_log.alloc(kBins);
      h->gamma.alloc(n_quantiles);
      h->q_lo.alloc(n_quantiles);
      h->q_hi.alloc(n_quantiles);
      std::vector<int32_t> lo(n_quantiles), hi(n_quantiles);
      for (int i = 0; i < n_quantiles; ++i) {
        TMH_CHECK(q_lo[i] >= 0 && q_lo[i] < npx && q_hi[i] >= q_lo[i] && q_hi[i] < npx, TMH_EINVAL,
                  "quantile positions out of range");
        TMH_CHECK(i == 0 || (q_lo[i] >= q_lo[i - 1] && q_hi[i] >= q_hi[i - 1]), TMH_EINVAL,
                  "quantile positions must be non-decreasing");
        lo[i] = (int32_t)q_lo[i];
        hi[i] = (int32_t)q_hi[i];
      }
      TMH_HIP(hipMemcpy(h->q_lo.p, lo.data(), lo.size() * 4, hipMemcpyHostToDevice));
      TMH_HIP(hipMemcpy(h->q_hi.p, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
      TMH_HIP(hipMemcpy(h->gamma.p, q_gamma, (size_t)n_quantiles * 8, hipMemcpyHostToDevice));
      TMH_HIP(hipMemcpy(h->lut_log.p, lut_log10, (size_t)kBins * 8, hipMemcpyHostToDevice));
      h->pooled_parts.alloc((size_t)kPooledParts * kBins, true);
      h->qp.lo = h->q_lo.p;
      h->qp.hi = h->q_hi.p;
      h->qp.Q = n_quantiles;
      h->qp.scale = h->scale;
      h->qp.last = (int32_t)(npx - 1);
      h->qp.hi_next = 1;
      for (int i = 0; i < n_quantiles; ++i)
        if (hi[i] != std::min<int32_t>(lo[i] + 1, (int32_t)(npx - 1))) h->qp.hi_next = 0;
    } catch (...) {
      tmh_stats_destroy(h);
      throw;
    }
    *out = h;
  });
}

void tmh_stats_destroy(tmh_stats* h) {
  if (!h) return;
  for (int i = 0; i < h->join_n; ++i) (void)hipEventSynchronize(h->join_ev[i]);
  if (h->own_stream) (void)hipStreamSynchronize(h->own_stream);
  if (h->stream && h->stream != h->own_stream) (void)hipStreamSynchronize(h->stream);
  hipStream_t s = h->own_stream, side = h->side, tail = h->tail;
  if (side) (void)hipStreamSynchronize(side);
  if (tail) (void)hipStreamSynchronize(tail);
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->ev_in) (void)hipEventDestroy(h->ev_in);
  if (h->ev_out) (void)hipEventDestroy(h->ev_out);
  if (h->ev_probe) (void)hipEventDestroy(h->ev_probe);
  for (hipEvent_t e : h->join_ev)
    if (e) (void)hipEventDestroy(e);
  if (h->probe_host) (void)hipHostFree(h->probe_host);
  delete h;
  if (s) (void)hipStreamDestroy(s);
  if (side) (void)hipStreamDestroy(side);
  if (tail) (void)hipStreamDestroy(tail);
}

int tmh_stats_set_stream(tmh_stats* h, void* stream) {
  return guard([&] {
    TMH_CHECK(h, TMH_EINVAL, "handle is NULL");
    h->stream = stream ? (hipStream_t)stream : h->own_stream;
  });
}

int tmh_stats_set_option(tmh_stats* h, int option, int value) {
  return guard([&] {
    TMH_CHECK(h, TMH_EINVAL, "handle is NULL");
    switch (option) {
      case TMH_OPT_FUSED_CONFIG:
        TMH_CHECK((value >= kFusedAuto && value < kFusedConfigs) || value == kFusedNoHist,
                  TMH_EINVAL, "fused configuration out of range");
        h->fused_cfg = value;
        break;
      case TMH_OPT_WELFORD_PARTS:
        TMH_CHECK(value >= 0 && value <= 4, TMH_EINVAL, "Welford parts must be 0..4");
        h->wf_parts = value;
        break;
      default:
        if (!h->host.set(option, value)) throw Error{TMH_EINVAL, "unknown option"};
    }
  });
}

int tmh_stats_reset(tmh_stats* h) {
  return guard([&] {
    TMH_CHECK(h, TMH_EINVAL, "handle is NULL");
    if (h->hist_dirty) {  // an interrupted fused launch: restore the zero-maintained slabs
      TMH_HIP(hipDeviceSynchronize());  // it may have been queued on any stream
      if (h->hist_full.n)
        TMH_HIP(hipMemsetAsync(h->hist_full.p, 0, h->hist_full.n * 4, hstream(h)));
      if (h->hist_rmask.n)
        TMH_HIP(hipMemsetAsync(h->hist_rmask.p, 0, h->hist_rmask.n * 8, hstream(h)));
      TMH_HIP(hipMemsetAsync(h->pooled_parts.p, 0, h->pooled_parts.n * 8, hstream(h)));
      h->hist_dirty = false;
    }
    ZeroList z;  // one launch for the job's fresh state
    z.add(h->mean.p, h->npx);
    z.add(h->m2.p, h->npx);
    z.add(h->acc.p, h->Q);
    z.add(h->pooled.p, kBins);
    z.add(h->wide.p, 2);
    launch_zero_u64(z, hstream(h));
    h->wide_sites = 0;
    h->n = 0;
    h->n_deferred = 0;
    h->last_batch = 0;
    h->pending = 0;
    h->pct_sum_external = false;
    if (h->probe_queued) TMH_HIP(hipEventSynchronize(h->ev_probe));  // its buffers are reused
    h->probed = false;  // the next job probes its own sites
    h->probe_queued = false;
  });
}

// The job's site probe, once per job (first call after a reset): one small
// kernel on s, its three counts copied to pinned memory, and the host waits
// for them -- a wait for the probe itself plus whatever s had queued before
// it.  Nothing is probed when every automatic choice is forced off.
static void stats_probe(tmh_stats* h, const uint16_t* d, int64_t ns, const SiteTab& tab,
                        hipStream_t s) {
  if (h->probed || (ns <= 0 && !h->probe_queued)) return;
  if (!h->probe_queued) {
    launch_site_probe(d, h->npx, ns, h->probe.p, s, tab);
    TMH_HIP(hipMemcpyAsync(h->probe_host, h->probe.p, 3 * sizeof(unsigned int),
                           hipMemcpyDeviceToHost, s));
    TMH_HIP(hipEventRecord(h->ev_probe, s));
  }
  TMH_HIP(hipEventSynchronize(h->ev_probe));
  for (int i = 0; i < 3; ++i) h->probe_cnt[i] = h->probe_host[i];
  h->probed = true;
  h->probe_queued = false;
}

// The probe queued ahead of the job's Welford launch (tmh_stats_probe_device):
// stats_probe then only waits for it.
static void stats_probe_queue(tmh_stats* h, const uint16_t* d, int64_t ns, const SiteTab& tab,
                              hipStream_t s) {
  if (h->probed || h->probe_queued || ns <= 0) return;
  launch_site_probe(d, h->npx, ns, h->probe.p, s, tab);
  TMH_HIP(hipMemcpyAsync(h->probe_host, h->probe.p, 3 * sizeof(unsigned int),
                         hipMemcpyDeviceToHost, s));
  TMH_HIP(hipEventRecord(h->ev_probe, s));
  h->probe_queued = true;
}

// The automatic choices from the probe (a job not probed: standard).
static bool probe_bright(const tmh_stats* h) {
  return h->probed && (double)h->probe_cnt[1] >= kBrightFrac * (double)h->probe_cnt[0];
}
static int probe_fused_cfg(const tmh_stats* h) {
  if (h->fused_cfg != kFusedAuto) return h->fused_cfg;
  if (!h->probed) return kFusedNarrow;
  const double g = (double)h->probe_cnt[0];
  if ((double)h->probe_cnt[2] >= kXWideFrac * g) return kFusedNoHist;
  if ((double)h->probe_cnt[1] >= kWideFrac * g) return kFusedWide;
  return kFusedNarrow;
}

static void stats_update_dev(tmh_stats* h, const uint16_t* d, int64_t ns, int log_transform,
                             hipStream_t s) {
  if (ns <= 0) return;
  if ((size_t)ns > h->rn.n) {
    TMH_HIP(hipStreamSynchronize(s));
    h->rn.alloc((size_t)ns);
  }
  // Both passes only read the sites: run the histogram/percentile pass on a
  // side stream concurrently with the Welford pass (fork/join by events).
  const bool serial = (h->flags & TMH_STATS_SERIAL) != 0;
  hipStream_t hs = serial ? s : h->side;
  const int64_t chunk = 4096;
  stats_reserve_sites(h, std::min(chunk, ns));  // (re)allocate before forking
  if (h->flags & TMH_STATS_DEFERRED_PCT) stats_grow_deferred(h, ns);
  // the bright Welford form needs a three-part split (>= 96 sites): only then
  // is the probe worth its host wait
  const bool vec = (h->npx & 7) == 0 && (reinterpret_cast<uintptr_t>(d) & 15) == 0;
  if (vec && log_transform && h->wf_parts == 0 && ns >= 96) stats_probe(h, d, ns, SiteTab{}, s);
  if (!serial) {
    TMH_HIP(hipEventRecord(h->ev_fork, s));
    TMH_HIP(hipStreamWaitEvent(hs, h->ev_fork, 0));
  }
  launch_welford(d, h->npx, ns, h->n, h->rn.p, h->mean.p, h->m2.p, h->lut_log.p,
                 log_transform, h->wf_part.p, h->wf_part.n, h->wf_parts, nullptr,
                 probe_bright(h) ? 1 : 0, s);
  // order statistics, in chunks so the per-site slabs stay bounded
  for (int64_t c0 = 0; c0 < ns; c0 += chunk) {
    const int64_t nc = std::min(chunk, ns - c0);
    const bool deferred = (h->flags & TMH_STATS_DEFERRED_PCT) != 0;
    uint32_t* vlh = h->vlh.p + (deferred ? (size_t)h->n_deferred * kOsTile : 0);
    const int64_t ld = deferred ? h->vlh_cap : nc;
    launch_hist_scatter(d + c0 * h->npx, h->npx, nc, h->hist_hi.p, h->qp, vlh, ld, h->pooled.p,
                        h->zeros.p, (h->flags & 2u) ? h->site_hist.p : nullptr, hs);
    if (deferred)
      h->n_deferred += nc;
    else
      launch_pct_accumulate(vlh, nc, ld, h->Q, h->gamma.p, h->acc.p, hs);
    h->vlh_ld = ld;
    h->last_batch = nc;
  }
  if (!serial) {
    TMH_HIP(hipEventRecord(h->ev_join, hs));
    TMH_HIP(hipStreamWaitEvent(s, h->ev_join, 0));
  }
  h->n += ns;
}

static void stats_welford_dev(tmh_stats* h, const uint16_t* dev_sites, int64_t n_sites,
                              int log_transform, void* stream, const SiteTab& tab) {
  hipStream_t s = hpick(h, stream);
  cross_begin(h, s);
  if ((size_t)n_sites > h->rn.n) {
    TMH_HIP(hipStreamSynchronize(s));
    h->rn.alloc((size_t)n_sites);
  }
  // the probe serves the fused pass's configuration and the Welford form
  const bool vec = tab.in || ((h->npx & 7) == 0 && (reinterpret_cast<uintptr_t>(dev_sites) & 15) == 0);
  if (vec && (h->fused_cfg == kFusedAuto || (log_transform && h->wf_parts == 0)))
    stats_probe(h, dev_sites, n_sites, tab, s);
  launch_welford(dev_sites, h->npx, n_sites, h->n, h->rn.p, h->mean.p, h->m2.p, h->lut_log.p,
                 log_transform, h->wf_part.p, h->wf_part.n, h->wf_parts, h->wide.p,
                 probe_bright(h) ? 1 : 0, s, -1, tab);
  if ((h->npx & 7) == 0) h->wide_sites += n_sites;
  h->n += n_sites;
  h->pending += n_sites;
  cross_end(h, s);
}

static SiteTab blocked_tab(const uint16_t* const* dev_in_blocks, uint16_t* const* dev_out_blocks,
                          int block_shift, int64_t npx);

int tmh_stats_probe_device(tmh_stats* h, const uint16_t* dev_sites, int64_t n_sites,
                           void* stream) {
  return guard([&] {
    TMH_CHECK(h && (dev_sites || n_sites == 0) && n_sites >= 0, TMH_EINVAL, "bad arguments");
    if ((h->npx & 7) || (reinterpret_cast<uintptr_t>(dev_sites) & 15)) return;  // no vector path
    // ordered after stream's work only (include/tmhip.h): the counts go to the host
    stats_probe_queue(h, dev_sites, n_sites, SiteTab{}, hpick(h, stream));
  });
}

int tmh_stats_probe_blocks_device(tmh_stats* h, const uint16_t* const* dev_blocks, int block_shift,
                                  int64_t n_sites, void* stream) {
  return guard([&] {
    TMH_CHECK(h && n_sites >= 0, TMH_EINVAL, "bad arguments");
    const SiteTab tab = blocked_tab(dev_blocks, nullptr, block_shift, h->npx);
    stats_probe_queue(h, nullptr, n_sites, tab, hpick(h, stream));
  });
}

int tmh_stats_update_welford_device(tmh_stats* h, const uint16_t* dev_sites, int64_t n_sites,
                                    int log_transform, void* stream) {
  return guard([&] {
    TMH_CHECK(h && (dev_sites || n_sites == 0) && n_sites >= 0, TMH_EINVAL, "bad arguments");
    stats_welford_dev(h, dev_sites, n_sites, log_transform, stream, SiteTab{});
  });
}

// a blocked site layout's table (include/tmhip.h): checked as far as the host can
static SiteTab blocked_tab(const uint16_t* const* dev_in_blocks, uint16_t* const* dev_out_blocks,
                           int block_shift, int64_t npx) {
  TMH_CHECK(dev_in_blocks, TMH_EINVAL, "block table is NULL");
  TMH_CHECK(block_shift >= 2 && block_shift <= 24, TMH_EINVAL, "block_shift must be 2..24");
  TMH_CHECK((npx & 7) == 0, TMH_EINVAL,
            "blocked site layouts need height * width divisible by 8 (16-byte pixel groups)");
  SiteTab t;
  t.in = dev_in_blocks;
  t.out = dev_out_blocks;
  t.shift = block_shift;
  return t;
}

int tmh_stats_update_welford_blocks_device(tmh_stats* h, const uint16_t* const* dev_blocks,
                                           int block_shift, int64_t n_sites, int log_transform,
                                           void* stream) {
  return guard([&] {
    TMH_CHECK(h && n_sites >= 0, TMH_EINVAL, "bad arguments");
    if (n_sites == 0) return;
    stats_welford_dev(h, nullptr, n_sites, log_transform, stream,
                      blocked_tab(dev_blocks, nullptr, block_shift, h->npx));
  });
}

int tmh_stats_update_device(tmh_stats* h, const uint16_t* dev_sites, int64_t n_sites,
                            int log_transform, void* stream) {
  return guard([&] {
    TMH_CHECK(h && (dev_sites || n_sites == 0) && n_sites >= 0, TMH_EINVAL, "bad arguments");
    const hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    stats_update_dev(h, dev_sites, n_sites, log_transform, s);
    cross_end(h, s);
  });
}

int tmh_stats_zero_counts(tmh_stats* h, int64_t* host_out, int64_t n, void* stream) {
  return guard([&] {
    TMH_CHECK(h && (host_out || n == 0) && n >= 0, TMH_EINVAL, "bad arguments");
    TMH_CHECK(n <= h->last_batch && (size_t)n <= h->zeros.n, TMH_EINVAL,
              "more sites than the last update held");
    if (n == 0) return;
    hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    TMH_HIP(hipMemcpyAsync(host_out, h->zeros.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
    cross_end(h, s);  // a later update (on any stream) writes h->zeros after this copy
  });
}

int tmh_stats_update(tmh_stats* h, const uint16_t* host_sites, int64_t n_sites, int log_transform,
                     int64_t* zero_counts_out) {
  return guard([&] {
    TMH_CHECK(h && (host_sites || n_sites == 0) && n_sites >= 0, TMH_EINVAL, "bad arguments");
    if (n_sites == 0) return;
    HostPipe& p = h->pipe;
    const int64_t per = h->batch_cap;
    const size_t slot_px = (size_t)per * h->npx;
    if (2 * slot_px > h->stage.n) {
      TMH_HIP(hipStreamSynchronize(hstream(h)));
      h->stage.ensure(2 * slot_px);
    }
    p.init();
    const bool pinned = h->host.staging == kStagingPinnedIn;
    // retire chunk k-2 of this slot: its H2D, kernels and zero-count copy
    auto retire = [&](int slot) {
      if (!p.busy[slot]) return;
      TMH_HIP(hipEventSynchronize(p.ev_done[slot]));
      if (zero_counts_out)
        std::memcpy(zero_counts_out + p.s0[slot], p.out[slot].p, (size_t)p.ns[slot] * 8);
      p.busy[slot] = false;
    };
    int64_t k = 0;
    try {
      for (int64_t s0 = 0; s0 < n_sites; s0 += per, ++k) {
        const int slot = (int)(k & 1);
        const int64_t ns = std::min<int64_t>(per, n_sites - s0);
        const size_t bytes = (size_t)ns * h->npx * 2;
        retire(slot);
        p.out[slot].ensure((size_t)per * 8);
        const void* src = host_sites + s0 * h->npx;
        if (pinned) {
          p.in[slot].ensure(slot_px * 2);
          par_copy(p.in[slot].p, src, bytes, h->host.copy_threads);
          src = p.in[slot].p;
        }
        uint16_t* dev = h->stage.p + (size_t)slot * slot_px;
        TMH_HIP(hipMemcpyAsync(dev, src, bytes, hipMemcpyHostToDevice, p.h2d));
        TMH_HIP(hipEventRecord(p.ev_in[slot], p.h2d));
        TMH_HIP(hipStreamWaitEvent(hstream(h), p.ev_in[slot], 0));
        stats_update_dev(h, dev, ns, log_transform, hstream(h));
        if (zero_counts_out)
          TMH_HIP(hipMemcpyAsync(p.out[slot].p, h->zeros.p, (size_t)ns * 8, hipMemcpyDeviceToHost,
                                 hstream(h)));
        TMH_HIP(hipEventRecord(p.ev_done[slot], hstream(h)));
        p.busy[slot] = true;
        p.s0[slot] = s0;
        p.ns[slot] = ns;
      }
      retire((int)(k & 1));
      retire((int)((k + 1) & 1));
    } catch (...) {
      p.abandon(hstream(h));
      throw;
    }
  });
}

static void stats_pct_sum_device(tmh_stats* h) {
  if ((h->flags & TMH_STATS_DEFERRED_PCT) && !h->pct_sum_external) {
    TMH_HIP(hipMemsetAsync(h->acc.p, 0, (size_t)h->Q * 8, hstream(h)));
    launch_pct_accumulate(h->vlh.p, h->n_deferred, h->vlh_cap, h->Q, h->gamma.p, h->acc.p,
                          hstream(h));
  }
}

int tmh_stats_finalize(tmh_stats* h, int64_t* n, double* mean, double* std, double* pct_sum,
                       uint64_t* hist) {
  return guard([&] {
    TMH_CHECK(h, TMH_EINVAL, "handle is NULL");
    if (n) *n = h->n;
    if (mean || std) {
      h->tmp_std.ensure(h->npx);
      launch_finalize(h->mean.p, h->m2.p, h->n, h->npx, nullptr, h->tmp_std.p, hstream(h));
      if (mean)
        TMH_HIP(hipMemcpyAsync(mean, h->mean.p, h->npx * 8, hipMemcpyDeviceToHost, hstream(h)));
      if (std)
        TMH_HIP(hipMemcpyAsync(std, h->tmp_std.p, h->npx * 8, hipMemcpyDeviceToHost, hstream(h)));
    }
    if (pct_sum) {
      stats_pct_sum_device(h);
      TMH_HIP(hipMemcpyAsync(pct_sum, h->acc.p, (size_t)h->Q * 8, hipMemcpyDeviceToHost, hstream(h)));
    }
    if (hist)
      TMH_HIP(hipMemcpyAsync(hist, h->pooled.p, (size_t)kBins * 8, hipMemcpyDeviceToHost, hstream(h)));
    TMH_HIP(hipStreamSynchronize(hstream(h)));
  });
}

int tmh_stats_finalize_device(tmh_stats* h, double* dev_mean, double* dev_std, void* stream) {
  return guard([&] {
    TMH_CHECK(h, TMH_EINVAL, "handle is NULL");
    const hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    launch_finalize(h->mean.p, h->m2.p, h->n, h->npx, dev_mean, dev_std, s);
    cross_end(h, s);
  });
}

int tmh_stats_variance(tmh_stats* h, double* host_var) {
  return guard([&] {
    TMH_CHECK(h && host_var, TMH_EINVAL, "bad arguments");
    h->tmp_std.ensure(h->npx);
    launch_variance(h->m2.p, h->n, h->npx, h->tmp_std.p, hstream(h));
    TMH_HIP(hipMemcpyAsync(host_var, h->tmp_std.p, h->npx * 8, hipMemcpyDeviceToHost, hstream(h)));
    TMH_HIP(hipStreamSynchronize(hstream(h)));
  });
}

int tmh_stats_job_choice(tmh_stats* h, uint32_t* probe_counts, int* welford_bright,
                         int* fused_cfg) {
  return guard([&] {
    TMH_CHECK(h, TMH_EINVAL, "handle is NULL");
    if (probe_counts)
      for (int i = 0; i < 3; ++i) probe_counts[i] = h->probed ? h->probe_cnt[i] : 0u;
    if (welford_bright) *welford_bright = h->probed ? (probe_bright(h) ? 1 : 0) : -1;
    if (fused_cfg) {
      const int c = probe_fused_cfg(h);
      *fused_cfg = c == kFusedNoHist ? TMH_FUSED_NO_HIST : c;
    }
  });
}

int tmh_stats_wide_groups(tmh_stats* h, uint64_t* groups_out, int64_t* sites_out) {
  return guard([&] {
    TMH_CHECK(h && groups_out, TMH_EINVAL, "bad arguments");
    unsigned long long w = 0;
    TMH_HIP(hipMemcpyAsync(&w, h->wide.p, 8, hipMemcpyDeviceToHost, hstream(h)));
    TMH_HIP(hipStreamSynchronize(hstream(h)));
    *groups_out = w;
    if (sites_out) *sites_out = h->wide_sites;
  });
}

int tmh_stats_get_hist_device(tmh_stats* h, uint64_t* dev_hist, void* stream) {
  return guard([&] {
    TMH_CHECK(h && dev_hist, TMH_EINVAL, "bad arguments");
    const hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    TMH_HIP(hipMemcpyAsync(dev_hist, h->pooled.p, (size_t)kBins * 8, hipMemcpyDeviceToDevice, s));
    cross_end(h, s);
  });
}

int tmh_stats_set_hist_device(tmh_stats* h, const uint64_t* dev_hist, void* stream) {
  return guard([&] {
    TMH_CHECK(h && dev_hist, TMH_EINVAL, "bad arguments");
    const hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    TMH_HIP(hipMemcpyAsync(h->pooled.p, dev_hist, (size_t)kBins * 8, hipMemcpyDeviceToDevice, s));
    cross_end(h, s);
  });
}

int tmh_stats_site_histogram(tmh_stats* h, int64_t site, uint32_t* host_hist) {
  return guard([&] {
    TMH_CHECK(h && host_hist, TMH_EINVAL, "bad arguments");
    TMH_CHECK(h->flags & 2u, TMH_ESTATE, "handle was created without TMH_STATS_KEEP_SITE_HIST (2)");
    TMH_CHECK(site >= 0 && site < h->last_batch, TMH_EINVAL, "site outside the last batch");
    TMH_HIP(hipMemcpyAsync(host_hist, h->site_hist.p + (size_t)site * kBins, (size_t)kBins * 4,
                           hipMemcpyDeviceToHost, hstream(h)));
    TMH_HIP(hipStreamSynchronize(hstream(h)));
  });
}

int tmh_stats_site_order_stats(tmh_stats* h, int64_t site, uint16_t* host_vlo, uint16_t* host_vhi) {
  return guard([&] {
    TMH_CHECK(h && host_vlo && host_vhi, TMH_EINVAL, "bad arguments");
    const bool deferred = h->flags & TMH_STATS_DEFERRED_PCT;
    const int64_t avail = deferred ? h->n_deferred : h->last_batch;
    TMH_CHECK(site >= 0 && site < avail, TMH_EINVAL, "site not available");
    // one site's column of every quantile tile
    const size_t row = (size_t)kOsTile * 4;
    std::vector<uint32_t> w((size_t)os_tiles(h->Q) * kOsTile);
    TMH_HIP(hipMemcpy2DAsync(w.data(), row, h->vlh.p + (size_t)site * kOsTile,
                             (size_t)h->vlh_ld * row, row, (size_t)os_tiles(h->Q),
                             hipMemcpyDeviceToHost, hstream(h)));
    TMH_HIP(hipStreamSynchronize(hstream(h)));
    for (int64_t q = 0; q < h->Q; ++q) {
      host_vlo[q] = (uint16_t)(w[q] & 0xFFFFu);
      host_vhi[q] = (uint16_t)(w[q] >> 16);
    }
    TMH_HIP(hipStreamSynchronize(hstream(h)));
  });
}

int tmh_stats_get_n(tmh_stats* h, int64_t* n) {
  return guard([&] {
    TMH_CHECK(h && n, TMH_EINVAL, "bad arguments");
    *n = h->n;
  });
}

int tmh_stats_set_n(tmh_stats* h, int64_t n) {
  return guard([&] {
    TMH_CHECK(h && n >= 0, TMH_EINVAL, "bad arguments");
    h->n = n;
  });
}

int tmh_stats_merge_stage1(tmh_stats* h, double* dev_nmean, void* stream) {
  return guard([&] {
    TMH_CHECK(h && dev_nmean, TMH_EINVAL, "bad arguments");
    const hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    launch_merge1(h->mean.p, h->n, h->npx, dev_nmean, s);
    cross_end(h, s);
  });
}

int tmh_stats_merge_stage2(tmh_stats* h, const double* dev_sum_nmean, int64_t n_total,
                           double* dev_m2c, void* stream) {
  return guard([&] {
    TMH_CHECK(h && dev_sum_nmean && dev_m2c && n_total > 0, TMH_EINVAL, "bad arguments");
    const hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    launch_merge2(h->mean.p, h->m2.p, h->n, dev_sum_nmean, n_total, h->npx, dev_m2c, s);
    cross_end(h, s);
  });
}

int tmh_stats_merge_stage3(tmh_stats* h, int64_t n_total, const double* dev_sum_m2c, void* stream) {
  return guard([&] {
    TMH_CHECK(h && dev_sum_m2c && n_total >= 0, TMH_EINVAL, "bad arguments");
    const hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    launch_copy_f64(dev_sum_m2c, h->m2.p, h->npx, s);
    cross_end(h, s);
    h->n = n_total;
  });
}

int tmh_stats_pct_accumulate(tmh_stats* h, double* dev_acc, void* stream) {
  return guard([&] {
    TMH_CHECK(h && dev_acc, TMH_EINVAL, "bad arguments");
    TMH_CHECK(h->flags & TMH_STATS_DEFERRED_PCT, TMH_ESTATE,
              "percentile chain needs a TMH_STATS_DEFERRED_PCT handle");
    const hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    launch_pct_accumulate(h->vlh.p, h->n_deferred, h->vlh_cap, h->Q, h->gamma.p, dev_acc, s);
    cross_end(h, s);
  });
}

int tmh_stats_pct_accumulate_range(tmh_stats* h, double* dev_acc_range, int q_begin, int q_count,
                                   void* stream) {
  return guard([&] {
    TMH_CHECK(h && dev_acc_range, TMH_EINVAL, "bad arguments");
    TMH_CHECK(h->flags & TMH_STATS_DEFERRED_PCT, TMH_ESTATE,
              "percentile chain needs a TMH_STATS_DEFERRED_PCT handle");
    TMH_CHECK(q_begin >= 0 && q_count >= 0 && (int64_t)q_begin + q_count <= h->Q, TMH_EINVAL,
              "quantile range out of bounds");
    const hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    launch_pct_accumulate_range(h->vlh.p, h->n_deferred, h->vlh_cap, q_begin, q_count, h->gamma.p,
                                dev_acc_range, s);
    cross_end(h, s);
  });
}

int tmh_stats_set_pct_sum(tmh_stats* h, const double* dev_acc, void* stream) {
  return guard([&] {
    TMH_CHECK(h && dev_acc, TMH_EINVAL, "bad arguments");
    const hipStream_t s = hpick(h, stream);
    cross_begin(h, s);
    launch_copy_f64(dev_acc, h->acc.p, h->Q, s);
    cross_end(h, s);
    h->pct_sum_external = true;
  });
}

int tmh_stats_get_pct_sum_device(tmh_stats* h, double* dev_acc, void* stream) {
  return guard([&] {
    TMH_CHECK(h && dev_acc, TMH_EINVAL, "bad arguments");
    hipStream_t s = hpick(h, stream);
    const bool cross = s != h->stream;
    cross_begin(h, s);  // after the handle's queued work, and the handle waits for the copy
    if ((h->flags & TMH_STATS_DEFERRED_PCT) && !h->pct_sum_external) {
      TMH_HIP(hipMemsetAsync(dev_acc, 0, (size_t)h->Q * 8, s));
      launch_pct_accumulate(h->vlh.p, h->n_deferred, h->vlh_cap, h->Q, h->gamma.p, dev_acc, s);
    } else {
      TMH_HIP(hipMemcpyAsync(dev_acc, h->acc.p, (size_t)h->Q * 8, hipMemcpyDeviceToDevice, s));
    }
    if (cross) defer_join(h, s);
  });
}

// ---------------------------------------------------------------------------
// smoothing
// ---------------------------------------------------------------------------

static std::vector<double> gaussian_taps(double sigma) {
  // mahotas 1.4.3 gaussian_filter1d (order 0): radius int(4 sd + 0.5)
  const int lw = (int)(4.0 * sigma + 0.5);
  std::vector<double> w(2 * lw + 1, 0.0);
  w[lw] = 1.0;
  double sum = 1.0;
  const double sd2 = sigma * sigma;
  for (int ii = 1; ii <= lw; ++ii) {
    const double t = std::exp(-0.5 * (double)(ii * ii) / sd2);
    w[lw + ii] = t;
    w[lw - ii] = t;
    sum += 2.0 * t;
  }
  for (auto& x : w) x /= sum;
  return w;
}

// taps per sigma, uploaded once (no allocation or sync on later calls)
static std::mutex g_taps_mu;
static std::map<double, std::pair<double*, int>> g_taps;

static std::pair<double*, int> taps_for(double sigma) {
  std::lock_guard<std::mutex> lk(g_taps_mu);
  auto it = g_taps.find(sigma);
  if (it != g_taps.end()) return it->second;
  const auto w = gaussian_taps(sigma);
  double* d = nullptr;
  TMH_HIP(hipMalloc(&d, w.size() * 8));
  TMH_HIP(hipMemcpy(d, w.data(), w.size() * 8, hipMemcpyHostToDevice));
  auto v = std::make_pair(d, (int)(w.size() / 2));
  g_taps[sigma] = v;
  return v;
}

int tmh_smooth_f64_device(const double* dev_in, double* dev_out, double* dev_tmp, int height,
                          int width, double sigma, void* stream) {
  return guard([&] {
    TMH_CHECK(dev_in && dev_out && dev_tmp && height > 0 && width > 0, TMH_EINVAL, "bad arguments");
    TMH_CHECK(sigma >= 0.125, TMH_EINVAL, "sigma must be >= 0.125");
    TMH_CHECK(dev_tmp != dev_in && dev_tmp != dev_out, TMH_EINVAL, "dev_tmp must be a third buffer");
    const auto t = taps_for(sigma);
    launch_smooth(dev_in, dev_out, dev_tmp, height, width, t.first, t.second, (hipStream_t)stream);
  });
}

int tmh_smooth2_f64_device(const double* dev_in0, const double* dev_in1, double* dev_out0,
                           double* dev_out1, double* dev_tmp0, double* dev_tmp1, int height,
                           int width, double sigma, void* stream) {
  return guard([&] {
    TMH_CHECK(dev_in0 && dev_in1 && dev_out0 && dev_out1 && dev_tmp0 && dev_tmp1 && height > 0 &&
                  width > 0,
              TMH_EINVAL, "bad arguments");
    TMH_CHECK(sigma >= 0.125, TMH_EINVAL, "sigma must be >= 0.125");
    const double* ins[2] = {dev_in0, dev_in1};
    const double* outs[2] = {dev_out0, dev_out1};
    for (const double* t : {(const double*)dev_tmp0, (const double*)dev_tmp1})
      for (int k = 0; k < 2; ++k)
        TMH_CHECK(t != ins[k] && t != outs[k], TMH_EINVAL, "dev_tmp0/1 must be buffers of their own");
    TMH_CHECK(dev_tmp0 != dev_tmp1, TMH_EINVAL, "dev_tmp0 and dev_tmp1 must differ");
    TMH_CHECK(dev_out0 != dev_out1, TMH_EINVAL, "dev_out0 and dev_out1 must differ");
    const auto t = taps_for(sigma);
    launch_smooth2(dev_in0, dev_in1, dev_out0, dev_out1, dev_tmp0, dev_tmp1, height, width,
                   t.first, t.second, (hipStream_t)stream);
  });
}

int tmh_smooth_f64(const double* host_in, double* host_out, int height, int width, double sigma) {
  return guard([&] {
    TMH_CHECK(host_in && host_out && height > 0 && width > 0, TMH_EINVAL, "bad arguments");
    const size_t npx = (size_t)height * width;
    DBuf<double> a, b, t;
    a.alloc(npx);
    b.alloc(npx);
    t.alloc(npx);
    TMH_HIP(hipMemcpy(a.p, host_in, npx * 8, hipMemcpyHostToDevice));
    int rc = tmh_smooth_f64_device(a.p, b.p, t.p, height, width, sigma, nullptr);
    if (rc) throw Error{rc, g_last_error};
    TMH_HIP(hipDeviceSynchronize());
    TMH_HIP(hipMemcpy(host_out, b.p, npx * 8, hipMemcpyDeviceToHost));
  });
}

// ---------------------------------------------------------------------------
// correction
// ---------------------------------------------------------------------------

static void coef_job(CoefJobs& J, int k, tmh_corrector* c, const double* d_mean,
                     const double* d_std) {
  J.mean[k] = d_mean;
  J.std[k] = d_std;
  J.partial[k] = c->partial.p;
  J.sums[k] = c->sums.p;
  // the LUT path's coef and the chain's coef_lin are made when a call needs
  // them (corrector_forms): the fused job path reads only coef2 and coef64
  // (24 of the 48 B/px the full set writes)
  J.coef[k] = nullptr;
  J.coef2[k] = c->coef2.p;
  J.coef_lin[k] = nullptr;
  c->forms_stale = true;
  J.coef64[k] = c->coef64.p;
  J.mconst[k] = c->mconst.p;
  J.mconst2[k] = c->mconst2.p;
  J.rc[k] = c->rc.p;
  J.log_transform[k] = c->log_transform;
  J.zero_log10[k] = c->zero_log10;
}

// coef / coef_lin for the calls that read them, from the last update
static void corrector_forms(tmh_corrector* c, hipStream_t s) {
  if (!c->forms_stale) return;
  launch_coeffs_forms(c->coef64.p, c->sums.p, c->npx, c->log_transform, c->coef.p, c->coef_lin.p, s);
  c->forms_stale = false;
}

static void corrector_coeffs(tmh_corrector* c, const double* d_mean, const double* d_std,
                             hipStream_t s) {
  ProfScope prof("coeffs", s);
  CoefJobs J{};
  coef_job(J, 0, c, d_mean, d_std);
  launch_coeffs_jobs(J, 1, c->H, c->W, false, s);
}

static void corrector_init(tmh_corrector* c, const double* d_mean, const double* d_std) {
  c->sums.alloc(3);
  c->partial.alloc(3 * (size_t)coef_tiles(c->H, c->W));
  c->coef.alloc(c->npx);
  c->coef2.alloc(c->npx);
  c->coef_lin.alloc(c->npx);
  c->coef64.alloc(c->npx);
  c->mconst.alloc(1);
  c->mconst2.alloc(1);
  c->rc.alloc(1);
  c->fix_n.alloc(1, true);
  TMH_HIP(hipDeviceGetAttribute(&c->n_wg, hipDeviceAttributeMultiprocessorCount, c->device));
  c->queues.alloc(kFusedQueueInts, true);
  corrector_coeffs(c, d_mean, d_std, c->stream);
}

// The refinement list of one correct launch over n_sites sites on stream s:
// capacity for 1/1024 of the launch's pixels (an overflow makes the fixup
// recompute every pixel in f64: slow but exact), count reset on s.  One
// launch at a time per corrector (the list is reused).
static FixList corrector_fixlist(tmh_corrector* c, int64_t n_sites, hipStream_t s,
                                 bool reset = true) {
  TMH_CHECK(n_sites < ((int64_t)1 << 24), TMH_EINVAL, "at most 2^24 - 1 sites per correct call");
  const int64_t want = std::min<int64_t>(std::max<int64_t>((int64_t)1 << 20, n_sites * c->npx / 1024),
                                         (int64_t)1 << 30);
  if ((size_t)want > c->fix_e.n) {
    TMH_HIP(hipDeviceSynchronize());  // the list may be in use on any stream
    c->fix_e.alloc((size_t)want);
  }
  if (reset) TMH_HIP(hipMemsetAsync(c->fix_n.p, 0, sizeof(unsigned int), s));
  return FixList{c->fix_e.p, c->fix_n.p, (unsigned int)c->fix_e.n};
}

int tmh_corrector_create_device(const double* dev_mean, const double* dev_std, int height,
                                int width, int log_transform, double zero_log10, void* stream,
                                tmh_corrector** out) {
  return guard([&] {
    TMH_CHECK(out && dev_mean && dev_std && height > 0 && width > 0, TMH_EINVAL, "bad arguments");
    auto* c = new tmh_corrector();
    try {
      TMH_HIP(hipGetDevice(&c->device));
      c->H = height;
      c->W = width;
      c->npx = (int64_t)height * width;
      c->log_transform = log_transform ? 1 : 0;
      c->zero_log10 = zero_log10;
      c->stream = (hipStream_t)stream;
      c->lut.alloc(kBins);
      launch_build_corr_lut(c->lut.p, c->log_transform, zero_log10, c->stream);
      corrector_init(c, dev_mean, dev_std);
    } catch (...) {
      delete c;
      throw;
    }
    *out = c;
  });
}

int tmh_corrector_create(const double* host_mean, const double* host_std, int height, int width,
                         int log_transform, double zero_log10, tmh_corrector** out) {
  return guard([&] {
    TMH_CHECK(out && host_mean && host_std && height > 0 && width > 0, TMH_EINVAL, "bad arguments");
    const size_t npx = (size_t)height * width;
    DBuf<double> m, s;
    m.alloc(npx);
    s.alloc(npx);
    TMH_HIP(hipMemcpy(m.p, host_mean, npx * 8, hipMemcpyHostToDevice));
    TMH_HIP(hipMemcpy(s.p, host_std, npx * 8, hipMemcpyHostToDevice));
    int rc = tmh_corrector_create_device(m.p, s.p, height, width, log_transform, zero_log10, nullptr,
                                         out);
    if (rc) throw Error{rc, g_last_error};
    TMH_HIP(hipDeviceSynchronize());
  });
}

void tmh_corrector_destroy(tmh_corrector* c) {
  if (!c) return;
  (void)hipStreamSynchronize(c->stream);
  if (c->ev_tail) {
    (void)hipEventSynchronize(c->ev_tail);
    (void)hipEventDestroy(c->ev_tail);
  }
  delete c;
}

int tmh_corrector_set_option(tmh_corrector* c, int option, int value) {
  return guard([&] {
    TMH_CHECK(c, TMH_EINVAL, "corrector is NULL");
    if (option == TMH_OPT_FUSED_BANDS) {
      TMH_CHECK(value == 0 || value == 8 || value == 16 || value == 32 || value == 64, TMH_EINVAL,
                "fused bands must be 0 (automatic), 8, 16, 32 or 64");
      c->bands = value;
      return;
    }
    if (option == TMH_OPT_FUSED_CUS) {
      int cus = 256;
      TMH_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
      TMH_CHECK(value >= 0 && value <= cus, TMH_EINVAL, "fused CUs must be 0..CU count");
      c->n_wg = value ? value : cus;
      return;
    }
    if (!c->host.set(option, value)) throw Error{TMH_EINVAL, "unknown corrector option"};
  });
}

int tmh_corrector_update_device(tmh_corrector* c, const double* dev_mean, const double* dev_std,
                                void* stream) {
  return guard([&] {
    TMH_CHECK(c && dev_mean && dev_std, TMH_EINVAL, "bad arguments");
    corrector_coeffs(c, dev_mean, dev_std, pick(c->stream, stream));
  });
}

int tmh_corrector_update_multi_device(tmh_corrector* const* cs, int n, const double* const* dev_mean,
                                      const double* const* dev_std, void* stream) {
  return guard([&] {
    TMH_CHECK(cs && dev_mean && dev_std && n >= 1 && n <= kMaxJobs, TMH_EINVAL,
              "bad arguments (1 <= n <= 8 correctors)");
    CoefJobs J{};
    for (int k = 0; k < n; ++k) {
      TMH_CHECK(cs[k] && dev_mean[k] && dev_std[k], TMH_EINVAL, "bad arguments");
      TMH_CHECK(cs[k]->npx == cs[0]->npx, TMH_EINVAL, "correctors of different image sizes");
      coef_job(J, k, cs[k], dev_mean[k], dev_std[k]);
    }
    for (int k = 0; k < n; ++k)
      TMH_CHECK(cs[k]->H == cs[0]->H && cs[k]->W == cs[0]->W, TMH_EINVAL,
                "correctors of different image shapes");
    const hipStream_t s = pick(cs[0]->stream, stream);
    ProfScope prof("coeffs", s);
    launch_coeffs_jobs(J, n, cs[0]->H, cs[0]->W, false, s);
  });
}

int tmh_job_planes_multi_device(tmh_stats* const* hs, tmh_corrector* const* cs, int n,
                                double* const* dev_mean, double* const* dev_std,
                                double* const* dev_smean, double* const* dev_sstd, double sigma,
                                void* stream) {
  return guard([&] {
    TMH_CHECK(hs && cs && dev_smean && dev_sstd && n >= 1 && n <= kMaxJobs, TMH_EINVAL,
              "bad arguments (1 <= n <= 8 jobs)");
    TMH_CHECK(sigma >= 0.125, TMH_EINVAL, "sigma must be >= 0.125");
    for (int k = 0; k < n; ++k) {
      TMH_CHECK(hs[k] && cs[k] && dev_smean[k] && dev_sstd[k], TMH_EINVAL, "bad arguments");
      TMH_CHECK(hs[k]->H == hs[0]->H && hs[k]->W == hs[0]->W && cs[k]->npx == hs[0]->npx,
                TMH_EINVAL, "jobs of different image sizes");
      // (every check before the first cross_begin / launch: a rejected call
      // leaves nothing queued that reads scratch freed on the way out)
      TMH_CHECK(cs[k]->H == hs[0]->H && cs[k]->W == hs[0]->W, TMH_EINVAL,
                "jobs of different image shapes");
      TMH_CHECK(dev_smean[k] != dev_sstd[k], TMH_EINVAL, "smoothed planes must differ");
      for (int j = 0; j < k; ++j)
        TMH_CHECK(hs[j] != hs[k] && cs[j] != cs[k], TMH_EINVAL, "a handle listed twice");
    }
    const int H = hs[0]->H, W = hs[0]->W;
    const int64_t npx = hs[0]->npx;
    const hipStream_t s = pick(hs[0]->stream, stream);
    for (int k = 0; k < n; ++k) cross_begin(hs[k], s);
    // stats.py:94-112 as asked for (the unsmoothed planes: what the
    // illumstats file keeps); the smoothing reads the handles' state itself
    for (int k = 0; k < n; ++k) {
      const bool m = dev_mean && dev_mean[k], d = dev_std && dev_std[k];
      if (m || d)
        launch_finalize(hs[k]->mean.p, hs[k]->m2.p, hs[k]->n, npx, m ? dev_mean[k] : nullptr,
                        d ? dev_std[k] : nullptr, s);
    }
    // IllumstatsContainer.smooth (image.py:1172-1193), every job's mean and
    // std in one launch; the std planes finalized as they are read
    const auto t = taps_for(sigma);
    const double* in[kMaxPlanes];
    double* out[kMaxPlanes];
    double sq[kMaxPlanes];
    DBuf<double> scratch;
    const bool onepass = t.second == 20 && W >= 41 && !getenv("TMH_SMOOTH_2PASS");
    if (!onepass) scratch.alloc((size_t)3 * n * npx);  // finalized std + axis-0 temps
    double* tmp[kMaxPlanes];
    for (int k = 0; k < n; ++k) {
      tmh_stats* h = hs[k];
      in[2 * k] = h->mean.p;
      out[2 * k] = dev_smean[k];
      sq[2 * k] = 0.0;
      out[2 * k + 1] = dev_sstd[k];
      if (onepass) {
        in[2 * k + 1] = h->m2.p;
        sq[2 * k + 1] = h->n >= 2 ? (double)(h->n - 1) : -1.0;
      } else {
        double* sd = scratch.p + (size_t)(3 * k) * npx;
        launch_finalize(h->mean.p, h->m2.p, h->n, npx, nullptr, sd, s);
        in[2 * k + 1] = sd;
        sq[2 * k + 1] = 0.0;
        tmp[2 * k] = scratch.p + (size_t)(3 * k + 1) * npx;
        tmp[2 * k + 1] = scratch.p + (size_t)(3 * k + 2) * npx;
      }
    }
    // the coefficient tiles' sums of the smoothed planes come with them
    // (psum / pmin: std sums, mean sums, std minima in each corrector's
    // partial buffer)
    const int nt = coef_tiles(H, W);
    double* psum[kMaxPlanes];
    double* pmin[kMaxPlanes];
    for (int k = 0; k < n; ++k) {
      psum[2 * k] = cs[k]->partial.p + nt;  // mean
      pmin[2 * k] = nullptr;
      psum[2 * k + 1] = cs[k]->partial.p;  // std
      pmin[2 * k + 1] = cs[k]->partial.p + 2 * nt;
    }
    launch_smooth_planes(in, out, onepass ? out : tmp, sq, 2 * n, H, W, t.first, t.second, s,
                         psum, pmin);
    // the correctors' coefficients (image.py:599-631) from the smoothed planes
    CoefJobs J{};
    for (int k = 0; k < n; ++k) coef_job(J, k, cs[k], dev_smean[k], dev_sstd[k]);
    {
      ProfScope prof("coeffs", s);
      launch_coeffs_jobs(J, n, H, W, true, s);
    }
    for (int k = 0; k < n; ++k) cross_end(hs[k], s);
    if (!onepass) TMH_HIP(hipStreamSynchronize(s));  // the scratch is freed on return
  });
}

int tmh_corrector_means(tmh_corrector* c, double* mean_of_std, double* mean_of_mean) {
  return guard([&] {
    TMH_CHECK(c, TMH_EINVAL, "corrector is NULL");
    double sums[2];
    TMH_HIP(hipStreamSynchronize(c->stream));
    TMH_HIP(hipMemcpy(sums, c->sums.p, 16, hipMemcpyDeviceToHost));
    if (mean_of_std) *mean_of_std = sums[0] / (double)c->npx;
    if (mean_of_mean) *mean_of_mean = sums[1] / (double)c->npx;
  });
}

static void check_clip(int lo, int hi, int maxv) {
  if (lo < 0) return;
  TMH_CHECK(lo <= maxv && hi >= 0 && hi <= maxv, TMH_EINVAL, "clip bounds out of range");
}

int tmh_correct_u16_device(tmh_corrector* c, const uint16_t* dev_in, uint16_t* dev_out,
                           int64_t n_sites, int clip_lo, int clip_hi, void* stream) {
  return guard([&] {
    TMH_CHECK(c && (dev_in && dev_out || n_sites == 0) && n_sites >= 0, TMH_EINVAL, "bad arguments");
    check_clip(clip_lo, clip_hi, 65535);
    hipStream_t s = pick(c->stream, stream);
    const FixList fl = corrector_fixlist(c, n_sites, s);
    corrector_forms(c, s);
    launch_correct_u16(dev_in, dev_out, c->npx, n_sites, c->coef.p, c->lut.p, c->mconst.p, fl,
                       c->log_transform, clip_lo, clip_hi, s);
    launch_fix_correct(dev_in, dev_out, 2, c->npx, n_sites, fl, c->coef64.p, c->rc.p,
                       c->log_transform, clip_lo, clip_hi, s);
  });
}

int tmh_correct_u16(tmh_corrector* c, const uint16_t* host_in, uint16_t* host_out, int64_t n_sites,
                    int clip_lo, int clip_hi) {
  return guard([&] {
    TMH_CHECK(c && (host_in && host_out || n_sites == 0) && n_sites >= 0, TMH_EINVAL,
              "bad arguments");
    check_clip(clip_lo, clip_hi, 65535);
    if (n_sites == 0) return;
    // chunks of <= 16 sites (~177 MB at 2160x2560), two slots per direction
    const int64_t step =
        std::max<int64_t>(1, std::min<int64_t>({16, n_sites, ((int64_t)192 << 20) / (c->npx * 2)}));
    const size_t slot_px = (size_t)step * c->npx;
    if (2 * slot_px > c->stage_in.n) {
      TMH_HIP(hipStreamSynchronize(c->stream));
      c->stage_in.ensure(2 * slot_px);
      c->stage_out.ensure(2 * slot_px);
    }
    HostPipe& p = c->pipe;
    p.init();
    const bool pinned_in = c->host.staging == kStagingPinnedIn,
               pinned_out = c->host.staging != kStagingDirect;
    auto retire = [&](int slot) {
      if (!p.busy[slot]) return;
      TMH_HIP(hipEventSynchronize(p.ev_done[slot]));
      if (pinned_out)
        par_copy(host_out + p.s0[slot] * c->npx, p.out[slot].p, (size_t)p.ns[slot] * c->npx * 2,
                 c->host.copy_threads);
      p.busy[slot] = false;
    };
    int64_t k = 0;
    try {
      for (int64_t s0 = 0; s0 < n_sites; s0 += step, ++k) {
        const int slot = (int)(k & 1);
        const int64_t ns = std::min(step, n_sites - s0);
        const size_t bytes = (size_t)ns * c->npx * 2;
        retire(slot);  // chunk k-2: output copied out, both slot buffers free
        const void* src = host_in + s0 * c->npx;
        void* dst = host_out + s0 * c->npx;
        if (pinned_in) {
          p.in[slot].ensure(slot_px * 2);
          par_copy(p.in[slot].p, src, bytes, c->host.copy_threads);
          src = p.in[slot].p;
        }
        if (pinned_out) {
          p.out[slot].ensure(slot_px * 2);
          dst = p.out[slot].p;
        }
        uint16_t* din = c->stage_in.p + (size_t)slot * slot_px;
        uint16_t* dout = c->stage_out.p + (size_t)slot * slot_px;
        TMH_HIP(hipMemcpyAsync(din, src, bytes, hipMemcpyHostToDevice, p.h2d));
        TMH_HIP(hipEventRecord(p.ev_in[slot], p.h2d));
        TMH_HIP(hipStreamWaitEvent(c->stream, p.ev_in[slot], 0));
        const FixList fl = corrector_fixlist(c, ns, c->stream);
        corrector_forms(c, c->stream);
        launch_correct_u16(din, dout, c->npx, ns, c->coef.p, c->lut.p, c->mconst.p, fl,
                           c->log_transform, clip_lo, clip_hi, c->stream);
        launch_fix_correct(din, dout, 2, c->npx, ns, fl, c->coef64.p, c->rc.p, c->log_transform,
                           clip_lo, clip_hi, c->stream);
        TMH_HIP(hipEventRecord(p.ev_kern[slot], c->stream));
        TMH_HIP(hipStreamWaitEvent(p.d2h, p.ev_kern[slot], 0));
        TMH_HIP(hipMemcpyAsync(dst, dout, bytes, hipMemcpyDeviceToHost, p.d2h));
        TMH_HIP(hipEventRecord(p.ev_done[slot], p.d2h));
        p.busy[slot] = true;
        p.s0[slot] = s0;
        p.ns[slot] = ns;
      }
      retire((int)(k & 1));
      retire((int)((k + 1) & 1));
    } catch (...) {
      p.abandon(c->stream);
      throw;
    }
  });
}

int tmh_correct_u8(tmh_corrector* c, const uint8_t* host_in, uint8_t* host_out, int64_t n_sites,
                   int clip_lo, int clip_hi) {
  return guard([&] {
    TMH_CHECK(c && (host_in && host_out || n_sites == 0) && n_sites >= 0, TMH_EINVAL,
              "bad arguments");
    check_clip(clip_lo, clip_hi, 255);
    const size_t bytes = (size_t)n_sites * c->npx;
    if (!bytes) return;
    c->stage8_in.ensure(bytes);
    c->stage8_out.ensure(bytes);
    TMH_HIP(hipMemcpyAsync(c->stage8_in.p, host_in, bytes, hipMemcpyHostToDevice, c->stream));
    const FixList fl = corrector_fixlist(c, n_sites, c->stream);
    corrector_forms(c, c->stream);
    launch_correct_u8(c->stage8_in.p, c->stage8_out.p, c->npx, n_sites, c->coef.p, c->lut.p,
                      c->mconst.p, fl, c->log_transform, clip_lo, clip_hi, c->stream);
    launch_fix_correct(c->stage8_in.p, c->stage8_out.p, 1, c->npx, n_sites, fl, c->coef64.p,
                       c->rc.p, c->log_transform, clip_lo, clip_hi, c->stream);
    TMH_HIP(hipMemcpyAsync(host_out, c->stage8_out.p, bytes, hipMemcpyDeviceToHost, c->stream));
    TMH_HIP(hipStreamSynchronize(c->stream));
  });
}

// One job's fused pass (correct + per-site histograms, then the histogram
// tail), in three steps so several jobs can share the launch in between
// (tmh_correct_u16_hist_multi_device): fused_prepare -> launch -> fused_finish.
struct FusedPass {
  tmh_corrector* c;
  tmh_stats* h;
  const uint16_t* in;
  uint16_t* out;
  int64_t n;
  SiteTab tab;
  hipStream_t s;
  bool cross;
  int clip_lo, clip_hi;
  int cfg;
  RareList rl;
  FixList fl;
  uint32_t* vlh;
  int64_t ld;
  uint32_t* sh;
};

// the fused pass floors zero pixels at 10**zero_log10 in f32 and reads 8-pixel
// groups: false = the two-pass path for odd shapes
static bool fused_vec(const tmh_corrector* c, const tmh_stats* h, const uint16_t* dev_in,
                      const uint16_t* dev_out, const SiteTab& tab) {
  const bool zl_ok = !c->log_transform || (c->zero_log10 >= -37.0 && c->zero_log10 <= 0.0);
  const bool vec = zl_ok && (h->npx & 7) == 0 &&
                   (tab.in || ((reinterpret_cast<uintptr_t>(dev_in) & 15) == 0 &&
                               (reinterpret_cast<uintptr_t>(dev_out) & 15) == 0));
  TMH_CHECK(vec || !tab.in, TMH_EINVAL,
            "a blocked site layout needs the fused pass (zero_log10 in [-37, 0])");
  return vec;
}

static void fused_check(const tmh_corrector* c, const tmh_stats* h, int64_t n_sites) {
  TMH_CHECK(c->npx == h->npx, TMH_EINVAL, "corrector and statistics image sizes differ");
  TMH_CHECK(n_sites <= h->pending, TMH_ESTATE,
            "more sites than were passed to tmh_stats_update_welford_device");
}

// Stream contract (include/tmhip.h): the job's launches run on s, after
// everything already queued on the statistics handle's stream (and after the
// corrector's pending tail, which still reads its round masks).
static bool fused_begin(tmh_corrector* c, tmh_stats* h, hipStream_t s) {
  const bool cross = s != h->stream;
  cross_begin(h, s);
  if (c->tail_pending) {
    TMH_HIP(hipStreamWaitEvent(s, c->ev_tail, 0));
    c->tail_pending = false;
  }
  return cross;
}

// buffers, rare lists, fixup list and the configuration of one job's pass
// (batched: the caller zeroes the fixup counter with its other jobs')
static void fused_prepare(FusedPass& p, bool batched = false) {
  tmh_stats* h = p.h;
  tmh_corrector* c = p.c;
  const int64_t n_sites = p.n;
  hipStream_t s = p.s;
  // rare lists (RareList, common.h) for the packed configuration
  if (h->fused_cfg == kFusedAuto) stats_probe(h, p.in, n_sites, p.tab, s);
  const bool rl_on = probe_fused_cfg(h) == kFusedWide;
  const unsigned int rl_cap =
      (unsigned int)std::min<int64_t>(65536, std::max<int64_t>(1024, h->npx / 64));
  const bool grow = (size_t)n_sites * kBins > h->hist_full.n || (size_t)n_sites > h->zeros.n ||
                    (size_t)n_sites > h->hist_rmask.n ||
                    (rl_on && ((size_t)n_sites * rl_cap > h->rare_v.n ||
                               (size_t)n_sites > h->rare_n.n)) ||
                    ((h->flags & 2u) && (size_t)n_sites * kBins > h->site_hist.n) ||
                    (!(h->flags & TMH_STATS_DEFERRED_PCT) && os_words(h, n_sites) > h->vlh.n);
  if (grow) {
    TMH_HIP(hipStreamSynchronize(s));
    TMH_HIP(hipStreamSynchronize(hstream(h)));
    TMH_HIP(hipStreamSynchronize(h->side));
  }
  if ((size_t)n_sites * kBins > h->hist_full.n) h->hist_full.alloc((size_t)n_sites * kBins, true);
  if ((size_t)n_sites > h->hist_rmask.n) h->hist_rmask.alloc((size_t)n_sites, true);
  p.rl = RareList{};
  if (rl_on) {
    h->rare_v.ensure((size_t)n_sites * rl_cap);
    h->rare_n.ensure((size_t)n_sites);
    TMH_HIP(hipMemsetAsync(h->rare_n.p, 0, (size_t)n_sites * sizeof(unsigned int), s));
    p.rl = RareList{h->rare_v.p, h->rare_n.p, rl_cap};
  }
  h->zeros.ensure((size_t)n_sites);
  if (h->flags & 2u) h->site_hist.ensure((size_t)n_sites * kBins);
  if (h->flags & TMH_STATS_DEFERRED_PCT) {
    stats_grow_deferred(h, n_sites);
    p.vlh = h->vlh.p + (size_t)h->n_deferred * kOsTile;
    p.ld = h->vlh_cap;
  } else {
    h->vlh.ensure(os_words(h, n_sites));
    p.vlh = h->vlh.p;
    p.ld = n_sites;
  }
  h->vlh_ld = p.ld;
  // the histogram slab and round masks are zero-maintained: the fused pass
  // fills them and k_hist_finalize resets what it read; if anything fails in
  // between, tmh_stats_reset clears them (hist_dirty)
  h->hist_dirty = true;
  p.sh = (h->flags & 2u) ? h->site_hist.p : nullptr;
  // one configuration, chosen on the host from the job's site probe (probed
  // at the Welford launch, or above for a job whose Welford pass did not)
  p.cfg = probe_fused_cfg(h);
  p.fl = corrector_fixlist(c, n_sites, s, !batched);
}

// what follows the job's fused launch up to its histogram tail: rare lists,
// f64 fixups and the very wide configuration's histograms.  fixed: the caller
// launched the fixups (and the wide counters' reset) for several jobs at once.
static void fused_post(FusedPass& p, bool fixed) {
  tmh_stats* h = p.h;
  tmh_corrector* c = p.c;
  const int64_t n_sites = p.n;
  hipStream_t s = p.s;
  if (p.cfg == kFusedWide) launch_rare_count(p.rl, h->hist_full.p, n_sites, s);
  if (!fixed)
    launch_fix_correct(p.in, p.out, 2, c->npx, n_sites, p.fl, c->coef64.p, c->rc.p,
                       c->log_transform, p.clip_lo, p.clip_hi, s, p.tab);
  if (p.cfg == kFusedNoHist)  // the histograms from one more read of the sites
    launch_hist_site_u16(p.in, h->npx, n_sites, h->hist_full.p, h->qp, p.vlh, p.ld, h->pooled.p,
                         h->pooled_parts.p, kPooledParts, h->zeros.p, p.sh, nullptr, 0, s, p.tab);
  // the Welford pass's diagnostic wide counts restart with the next batch
  // (reset here on s, before any later Welford launch on the handle)
  if (h->pending - n_sites == 0) {
    if (!fixed) TMH_HIP(hipMemsetAsync(h->wide.p, 0, 16, s));
    h->wide_sites = 0;
  }
}

// The histogram tail (order statistics, percentile sums) reads only the
// handle's buffers: called on another stream than the handle's, it runs on
// the handle's tail stream (the handle's stream waits for it), so s is free
// as soon as the corrected sites are written (a caller pipelining jobs
// starts the next one's Welford pass under this one's tail).
static hipStream_t fused_tail_stream(const FusedPass& p) {
  tmh_stats* h = p.h;
  if (!p.cross) return p.s;
  if (!h->tail) {  // created on first use: every stream takes a hardware queue slot
    TMH_HIP(hipStreamCreateWithFlags(&h->tail, hipStreamNonBlocking));
  }
  TMH_HIP(hipEventRecord(h->ev_out, p.s));
  TMH_HIP(hipStreamWaitEvent(h->tail, h->ev_out, 0));
  return h->tail;
}

// the tail's percentile sums and the handle's bookkeeping; ts: the stream
// the job's order statistics were queued on
static void fused_tail_end(FusedPass& p, hipStream_t ts) {
  tmh_stats* h = p.h;
  tmh_corrector* c = p.c;
  const int64_t n_sites = p.n;
  if (!(h->flags & TMH_STATS_DEFERRED_PCT))
    launch_pct_accumulate(p.vlh, n_sites, p.ld, h->Q, h->gamma.p, h->acc.p, ts);
  h->hist_dirty = false;
  if (h->flags & TMH_STATS_DEFERRED_PCT) h->n_deferred += n_sites;
  h->last_batch = n_sites;
  h->pending -= n_sites;
  if (p.cross) {  // the handle's later work, and this corrector's next pass, after the tail
    defer_join(h, ts);
    if (!c->ev_tail) TMH_HIP(hipEventCreateWithFlags(&c->ev_tail, hipEventDisableTiming));
    TMH_HIP(hipEventRecord(c->ev_tail, ts));
    c->tail_pending = true;
  }
}

// one job's histogram tail, on its handle's tail stream (or s)
static void fused_tail(FusedPass& p) {
  hipStream_t ts = fused_tail_stream(p);
  tmh_stats* h = p.h;
  if (p.cfg != kFusedNoHist)  // (very wide: k_hist_site_u16 wrote the order statistics)
    launch_hist_finalize(h->hist_full.p, h->hist_rmask.p, 0, p.n, h->qp, p.vlh, p.ld, h->pooled.p,
                         h->pooled_parts.p, kPooledParts, h->zeros.p, p.sh, ts, false,
                         reinterpret_cast<const unsigned long long*>(p.c->queues.p + 8));
  fused_tail_end(p, ts);
}

static void fused_finish(FusedPass& p) {
  fused_post(p, false);
  fused_tail(p);
}

static void correct_hist_dev(tmh_corrector* c, tmh_stats* h, const uint16_t* dev_in,
                             uint16_t* dev_out, int64_t n_sites, int clip_lo, int clip_hi,
                             void* stream, const SiteTab& tab) {
  {
    fused_check(c, h, n_sites);
    check_clip(clip_lo, clip_hi, 65535);
    if (n_sites == 0) return;
    hipStream_t s = pick(c->stream, stream);
    const bool vec = fused_vec(c, h, dev_in, dev_out, tab);
    const bool cross = fused_begin(c, h, s);
    if (vec) {
      FusedPass p{c, h, dev_in, dev_out, n_sites, tab, s, cross, clip_lo, clip_hi};
      fused_prepare(p);
      launch_correct_hist(dev_in, dev_out, c->npx, n_sites, c->coef2.p, c->mconst2.p, p.fl,
                          c->log_transform, clip_lo, clip_hi, h->hist_full.p, h->hist_rmask.p,
                          c->queues.p, c->n_wg, p.cfg, c->bands, s, tab, p.rl);
      fused_finish(p);
      return;
    }
    const int64_t chunk = 4096;  // odd shapes: correct and histogram in two passes
    for (int64_t c0 = 0; c0 < n_sites; c0 += chunk) {
      const int64_t nc = std::min(chunk, n_sites - c0);
      const uint16_t* din = dev_in + c0 * h->npx;
      uint16_t* dout = dev_out + c0 * h->npx;
      // per-site buffers (growing frees memory earlier launches may still use)
      const bool grow = (size_t)nc > h->zeros.n ||
                        ((h->flags & 2u) && (size_t)nc * kBins > h->site_hist.n) ||
                        (!(h->flags & TMH_STATS_DEFERRED_PCT) && os_words(h, nc) > h->vlh.n);
      if (grow) {
        TMH_HIP(hipStreamSynchronize(s));
        TMH_HIP(hipStreamSynchronize(hstream(h)));
        TMH_HIP(hipStreamSynchronize(h->side));
      }
      h->zeros.ensure((size_t)nc);
      if (h->flags & 2u) h->site_hist.ensure((size_t)nc * kBins);
      uint32_t* vlh;
      int64_t ld;
      if (h->flags & TMH_STATS_DEFERRED_PCT) {
        stats_grow_deferred(h, nc);
        vlh = h->vlh.p + (size_t)h->n_deferred * kOsTile;
        ld = h->vlh_cap;
      } else {
        h->vlh.ensure(os_words(h, nc));
        vlh = h->vlh.p;
        ld = nc;
      }
      h->vlh_ld = ld;
      stats_reserve_sites(h, nc);
      const FixList fl = corrector_fixlist(c, nc, s);
      corrector_forms(c, s);
      launch_correct_u16(din, dout, c->npx, nc, c->coef.p, c->lut.p, c->mconst.p, fl,
                         c->log_transform, clip_lo, clip_hi, s);
      launch_fix_correct(din, dout, 2, c->npx, nc, fl, c->coef64.p, c->rc.p, c->log_transform,
                         clip_lo, clip_hi, s);
      launch_hist_scatter(din, h->npx, nc, h->hist_hi.p, h->qp, vlh, ld, h->pooled.p, h->zeros.p,
                          (h->flags & 2u) ? h->site_hist.p : nullptr, s);
      if (h->flags & TMH_STATS_DEFERRED_PCT)
        h->n_deferred += nc;
      else
        launch_pct_accumulate(vlh, nc, ld, h->Q, h->gamma.p, h->acc.p, s);
      h->last_batch = nc;
      h->pending -= nc;
    }
    if (h->pending == 0 && h->wide_sites) {
      TMH_HIP(hipMemsetAsync(h->wide.p, 0, 16, s));
      h->wide_sites = 0;
    }
    if (cross) defer_join(h, s);
  }
}

int tmh_correct_u16_hist_device(tmh_corrector* c, tmh_stats* h, const uint16_t* dev_in,
                                uint16_t* dev_out, int64_t n_sites, int clip_lo, int clip_hi,
                                void* stream) {
  return guard([&] {
    TMH_CHECK(c && h && (dev_in && dev_out || n_sites == 0) && n_sites >= 0, TMH_EINVAL,
              "bad arguments");
    // the pass re-reads its input after storing outputs (f64 fixups, packed
    // counter recounts): input and output must not overlap
    TMH_CHECK(n_sites == 0 || dev_in + n_sites * h->npx <= dev_out ||
                  dev_out + n_sites * h->npx <= dev_in,
              TMH_EINVAL, "input and output sites must not overlap");
    correct_hist_dev(c, h, dev_in, dev_out, n_sites, clip_lo, clip_hi, stream, SiteTab{});
  });
}

int tmh_correct_u16_hist_blocks_device(tmh_corrector* c, tmh_stats* h,
                                       const uint16_t* const* dev_in_blocks,
                                       uint16_t* const* dev_out_blocks, int block_shift,
                                       int64_t n_sites, int clip_lo, int clip_hi, void* stream) {
  return guard([&] {
    TMH_CHECK(c && h && n_sites >= 0 && dev_out_blocks, TMH_EINVAL, "bad arguments");
    TMH_CHECK(dev_in_blocks != (const uint16_t* const*)dev_out_blocks, TMH_EINVAL,
              "input and output block tables must differ");
    const SiteTab tab = blocked_tab(dev_in_blocks, dev_out_blocks, block_shift, h->npx);
    correct_hist_dev(c, h, nullptr, nullptr, n_sites, clip_lo, clip_hi, stream, tab);
  });
}

// Several jobs' fused passes in ONE launch (a rank's channels): a short job's
// launch ends with most workgroups idle for a unit's time and starts with the
// pipeline filling; one sweep over every job's units pays that once.  Jobs
// whose configuration differs from the first's, or that need the two-pass
// path, run their own passes on the same stream; results are the per-job
// calls' in every case.
static void correct_hist_multi(tmh_corrector* const* cs, tmh_stats* const* hs, int n_jobs,
                               const uint16_t* const* ins, uint16_t* const* outs,
                               const SiteTab* tabs, const int64_t* n_sites, int clip_lo,
                               int clip_hi, void* stream) {
  TMH_CHECK(cs && hs && n_sites && n_jobs >= 1 && n_jobs <= kMaxJobs, TMH_EINVAL,
            "bad arguments (1 to 8 jobs)");
  check_clip(clip_lo, clip_hi, 65535);
  for (int j = 0; j < n_jobs; ++j) {
    TMH_CHECK(cs[j] && hs[j] && n_sites[j] >= 0, TMH_EINVAL, "bad arguments");
    fused_check(cs[j], hs[j], n_sites[j]);
    TMH_CHECK(cs[j]->npx == cs[0]->npx && cs[j]->log_transform == cs[0]->log_transform,
              TMH_EINVAL, "the jobs of one call need the same image size and transform");
    for (int k = 0; k < j; ++k)
      TMH_CHECK(cs[k] != cs[j] && hs[k] != hs[j], TMH_EINVAL,
                "each job needs its own corrector and statistics handle");
  }
  hipStream_t s = pick(cs[0]->stream, stream);
  bool all_vec = true;
  for (int j = 0; j < n_jobs; ++j)
    all_vec = all_vec && fused_vec(cs[j], hs[j], ins ? ins[j] : nullptr,
                                   outs ? outs[j] : nullptr, tabs[j]);
  if (!all_vec) {
    for (int j = 0; j < n_jobs; ++j)
      correct_hist_dev(cs[j], hs[j], ins ? ins[j] : nullptr, outs ? outs[j] : nullptr, n_sites[j],
                       clip_lo, clip_hi, s, tabs[j]);
    return;
  }
  FusedPass p[kMaxJobs];
  int np = 0;
  for (int j = 0; j < n_jobs; ++j) {
    if (n_sites[j] == 0) continue;
    const bool cross = fused_begin(cs[j], hs[j], s);
    p[np] = FusedPass{cs[j], hs[j], ins ? ins[j] : nullptr, outs ? outs[j] : nullptr, n_sites[j],
                      tabs[j], s, cross, clip_lo, clip_hi};
    fused_prepare(p[np], true);
    ++np;
  }
  if (np == 0) return;
  // every job's fixup counter, and the unit queues of the jobs sharing the
  // first job's launch, zeroed by one kernel (a fill per array cost ~10 us
  // each on the pass stream, 8 of them ahead of a four-job launch)
  ZeroList32 Z;
  for (int j = 0; j < np; ++j) {
    Z.add(p[j].c->fix_n.p, 1);
    if (p[j].cfg == p[0].cfg) Z.add(p[j].c->queues.p, kFusedQueueInts);
  }
  launch_zero_u32(Z, s);
  FusedJobs J{};
  for (int j = 0; j < np; ++j) {
    if (p[j].cfg != p[0].cfg) {  // its own launch
      tmh_corrector* c = p[j].c;
      launch_correct_hist(p[j].in, p[j].out, c->npx, p[j].n, c->coef2.p, c->mconst2.p, p[j].fl,
                          c->log_transform, clip_lo, clip_hi, p[j].h->hist_full.p,
                          p[j].h->hist_rmask.p, c->queues.p, c->n_wg, p[j].cfg, c->bands, s,
                          p[j].tab, p[j].rl);
      continue;
    }
    tmh_corrector* c = p[j].c;
    // the launch's unit counters are the first job's queues[0..8); every
    // job's round-mask union is its own corrector's queues + 8 (zeroed above)
    J.j[J.n++] = FusedJob{p[j].in, p[j].out, p[j].n,
                          reinterpret_cast<const float4*>(c->coef2.p), c->mconst2.p, p[j].fl,
                          p[j].h->hist_full.p, p[j].h->hist_rmask.p,
                          reinterpret_cast<unsigned long long*>(c->queues.p + 8), p[j].tab,
                          p[j].rl};
  }
  tmh_corrector* c0 = p[0].c;
  launch_correct_hist_jobs(J, c0->npx, c0->log_transform, clip_lo, clip_hi, c0->queues.p, c0->n_wg,
                           p[0].cfg, c0->bands, s);
  // every job's fixups (and Welford wide-counter reset) in one launch
  FixJobs F{};
  for (int j = 0; j < np; ++j) {
    tmh_corrector* c = p[j].c;
    F.j[F.n++] = FixJob{p[j].in, p[j].out, p[j].n, p[j].fl, c->coef64.p, c->rc.p, p[j].tab,
                        p[j].h->pending - p[j].n == 0 ? p[j].h->wide.p : nullptr};
  }
  launch_fix_correct_jobs(F, c0->npx, c0->log_transform, clip_lo, clip_hi, s);
  for (int j = 0; j < np; ++j) fused_post(p[j], true);
  // every job's histogram tail (column sums, order statistics) in two
  // launches on one stream: the first job's tail stream when the jobs run
  // off their handles' streams, else s
  bool same_cross = true;
  for (int j = 1; j < np; ++j) same_cross = same_cross && p[j].cross == p[0].cross;
  if (!same_cross) {  // mixed: per-job tails
    for (int j = 0; j < np; ++j) fused_tail(p[j]);
    return;
  }
  hipStream_t ts = fused_tail_stream(p[0]);
  TailJobs T{};
  for (int j = 0; j < np; ++j) {
    if (p[j].cfg == kFusedNoHist) continue;  // its order statistics are written
    tmh_stats* h = p[j].h;
    QPos qp = h->qp;
    qp.tstride = p[j].ld * kOsTile;
    T.j[T.n++] = TailJob{h->hist_full.p, h->hist_rmask.p,
                         reinterpret_cast<const unsigned long long*>(p[j].c->queues.p + 8), qp,
                         p[j].vlh, h->pooled.p, h->zeros.p, p[j].sh, p[j].n};
  }
  launch_hist_finalize_jobs(T, ts);
  for (int j = 0; j < np; ++j) fused_tail_end(p[j], ts);
}

int tmh_correct_u16_hist_multi_device(tmh_corrector* const* correctors, tmh_stats* const* handles,
                                      int n_jobs, const uint16_t* const* dev_in,
                                      uint16_t* const* dev_out, const int64_t* n_sites,
                                      int clip_lo, int clip_hi, void* stream) {
  return guard([&] {
    TMH_CHECK(dev_in && dev_out && n_jobs >= 1 && n_jobs <= kMaxJobs && n_sites, TMH_EINVAL,
              "bad arguments");
    SiteTab tabs[kMaxJobs];
    for (int j = 0; j < n_jobs; ++j) {
      TMH_CHECK(n_sites[j] >= 0 && (n_sites[j] == 0 || (dev_in[j] && dev_out[j])), TMH_EINVAL,
                "bad arguments");
      const int64_t npx = handles && handles[j] ? handles[j]->npx : 0;
      TMH_CHECK(n_sites[j] == 0 || dev_in[j] + n_sites[j] * npx <= dev_out[j] ||
                    dev_out[j] + n_sites[j] * npx <= dev_in[j],
                TMH_EINVAL, "input and output sites must not overlap");
    }
    correct_hist_multi(correctors, handles, n_jobs, dev_in, dev_out, tabs, n_sites, clip_lo,
                       clip_hi, stream);
  });
}

int tmh_correct_u16_hist_multi_blocks_device(tmh_corrector* const* correctors,
                                             tmh_stats* const* handles, int n_jobs,
                                             const uint16_t* const* const* dev_in_blocks,
                                             uint16_t* const* const* dev_out_blocks,
                                             int block_shift, const int64_t* n_sites, int clip_lo,
                                             int clip_hi, void* stream) {
  return guard([&] {
    TMH_CHECK(dev_in_blocks && dev_out_blocks && handles && n_jobs >= 1 && n_jobs <= kMaxJobs,
              TMH_EINVAL, "bad arguments");
    SiteTab tabs[kMaxJobs];
    for (int j = 0; j < n_jobs; ++j) {
      TMH_CHECK(handles[j] && dev_out_blocks[j], TMH_EINVAL, "bad arguments");
      TMH_CHECK(dev_in_blocks[j] != (const uint16_t* const*)dev_out_blocks[j], TMH_EINVAL,
                "input and output block tables must differ");
      tabs[j] = blocked_tab(dev_in_blocks[j], dev_out_blocks[j], block_shift, handles[j]->npx);
    }
    correct_hist_multi(correctors, handles, n_jobs, nullptr, nullptr, tabs, n_sites, clip_lo,
                       clip_hi, stream);
  });
}

// ---------------------------------------------------------------------------
// illuminati chain: align / scale / fused correct->align->clip->scale
// ---------------------------------------------------------------------------

static void check_windows(const tmh_window* w, int64_t n, int H, int W, int oh, int ow) {
  for (int64_t i = 0; i < n; ++i) {
    const tmh_window& x = w[i];
    TMH_CHECK(x.rows >= 0 && x.cols >= 0, TMH_EINVAL, "alignment window has negative extent");
    if (x.rows == 0 || x.cols == 0) continue;
    TMH_CHECK(x.src_r0 >= 0 && x.src_c0 >= 0 && x.src_r0 + x.rows <= H && x.src_c0 + x.cols <= W,
              TMH_EINVAL, "alignment window leaves the source image");
    TMH_CHECK(x.dst_r0 >= 0 && x.dst_c0 >= 0 && x.dst_r0 + x.rows <= oh && x.dst_c0 + x.cols <= ow,
              TMH_EINVAL, "alignment window leaves the output image");
  }
}

static void check_scale(int lo, int hi) {
  TMH_CHECK(lo >= 0 && lo < 65536 && hi >= 0 && hi < 65536, TMH_EINVAL,
            "scale bounds must be in the range [0, 65535]");
  TMH_CHECK(lo < hi, TMH_EINVAL, "\"lower_bound\" must be smaller than \"upper_bound\"");
}

int tmh_align(const void* host_in, void* host_out, int elem_bytes, int64_t n_sites, int height,
              int width, const tmh_window* windows, int out_height, int out_width) {
  return guard([&] {
    TMH_CHECK((elem_bytes == 1 || elem_bytes == 2) && n_sites >= 0 && height > 0 && width > 0 &&
                  out_height >= 0 && out_width >= 0 && (windows || n_sites == 0) &&
                  ((host_in && host_out) || n_sites == 0),
              TMH_EINVAL, "bad arguments");
    check_windows(windows, n_sites, height, width, out_height, out_width);
    if (n_sites == 0) return;
    const size_t in_b = (size_t)n_sites * height * width * elem_bytes;
    const size_t out_b = (size_t)n_sites * out_height * out_width * elem_bytes;
    DBuf<uint8_t> a, b;
    DBuf<tmh_window> w;
    a.alloc(in_b);
    b.alloc(std::max<size_t>(out_b, 1));
    w.alloc((size_t)n_sites);
    TMH_HIP(hipMemcpy(a.p, host_in, in_b, hipMemcpyHostToDevice));
    TMH_HIP(hipMemcpy(w.p, windows, (size_t)n_sites * sizeof(tmh_window), hipMemcpyHostToDevice));
    launch_align(a.p, b.p, elem_bytes, n_sites, height, width, out_height, out_width, w.p, nullptr);
    TMH_HIP(hipDeviceSynchronize());
    if (out_b) TMH_HIP(hipMemcpy(host_out, b.p, out_b, hipMemcpyDeviceToHost));
  });
}

int tmh_map_u16_to_u8(const uint16_t* host_in, uint8_t* host_out, int64_t n, int lower,
                      int upper) {
  return guard([&] {
    TMH_CHECK(n >= 0 && ((host_in && host_out) || n == 0), TMH_EINVAL, "bad arguments");
    check_scale(lower, upper);
    if (n == 0) return;
    DBuf<uint16_t> a;
    DBuf<uint8_t> b;
    a.alloc((size_t)n);
    b.alloc((size_t)n);
    TMH_HIP(hipMemcpy(a.p, host_in, (size_t)n * 2, hipMemcpyHostToDevice));
    launch_map_u8(a.p, b.p, n, lower, upper, nullptr);
    TMH_HIP(hipDeviceSynchronize());
    TMH_HIP(hipMemcpy(host_out, b.p, (size_t)n, hipMemcpyDeviceToHost));
  });
}

int tmh_correct_chain_u8_device(tmh_corrector* c, const uint16_t* dev_in, uint8_t* dev_out,
                                int64_t n_sites, const tmh_window* host_windows, int clip_lo,
                                int clip_hi, void* stream) {
  return guard([&] {
    TMH_CHECK(c && n_sites >= 0 && ((dev_in && dev_out && host_windows) || n_sites == 0),
              TMH_EINVAL, "bad arguments");
    check_scale(clip_lo, clip_hi);
    check_windows(host_windows, n_sites, c->H, c->W, c->H, c->W);
    TMH_CHECK(!c->log_transform || (c->zero_log10 >= -37.0 && c->zero_log10 <= 0.0), TMH_EINVAL,
              "the chain pass needs zero_log10 in [-37, 0]");
    if (n_sites == 0) return;
    hipStream_t s = pick(c->stream, stream);
    if ((size_t)n_sites > c->win.n) {
      TMH_HIP(hipStreamSynchronize(s));
      c->win.alloc((size_t)n_sites);
    }
    TMH_HIP(hipMemcpyAsync(c->win.p, host_windows, (size_t)n_sites * sizeof(tmh_window),
                           hipMemcpyHostToDevice, s));
    const FixList fl = corrector_fixlist(c, n_sites, s);
    if (!c->lut8.n) c->lut8.alloc(65536);
    corrector_forms(c, s);
    launch_chain_u8(dev_in, dev_out, c->H, c->W, n_sites, c->coef_lin.p, c->mconst2.p, fl,
                    c->coef64.p, c->rc.p, c->log_transform, c->win.p, clip_lo, clip_hi,
                    c->lut8.p, s, c->zero_log10);
    TMH_HIP(hipStreamSynchronize(s));  // the window buffer is reused by the next call
  });
}

int tmh_correct_chain_u8(tmh_corrector* c, const uint16_t* host_in, uint8_t* host_out,
                         int64_t n_sites, const tmh_window* host_windows, int clip_lo,
                         int clip_hi) {
  return guard([&] {
    TMH_CHECK(c && n_sites >= 0 && ((host_in && host_out && host_windows) || n_sites == 0),
              TMH_EINVAL, "bad arguments");
    if (n_sites == 0) return;
    const size_t npx = (size_t)c->npx;
    DBuf<uint16_t> a;
    DBuf<uint8_t> b;
    a.alloc((size_t)n_sites * npx);
    b.alloc((size_t)n_sites * npx);
    TMH_HIP(hipMemcpyAsync(a.p, host_in, (size_t)n_sites * npx * 2, hipMemcpyHostToDevice,
                           c->stream));
    int rc = tmh_correct_chain_u8_device(c, a.p, b.p, n_sites, host_windows, clip_lo, clip_hi,
                                         nullptr);
    if (rc) throw Error{rc, g_last_error};
    TMH_HIP(hipMemcpy(host_out, b.p, (size_t)n_sites * npx, hipMemcpyDeviceToHost));
  });
}

int tmh_clip_u16(const uint16_t* host_in, uint16_t* host_out, int64_t n, int lo, int hi) {
  return guard([&] {
    TMH_CHECK((host_in && host_out) || n == 0, TMH_EINVAL, "bad arguments");
    TMH_CHECK(lo >= 0 && lo <= 65535 && hi >= 0 && hi <= 65535, TMH_EINVAL, "clip bounds out of range");
    if (n == 0) return;
    DBuf<uint16_t> a, b;
    a.alloc(n);
    b.alloc(n);
    TMH_HIP(hipMemcpy(a.p, host_in, (size_t)n * 2, hipMemcpyHostToDevice));
    launch_clip_u16(a.p, b.p, n, lo, hi, nullptr);
    TMH_HIP(hipMemcpy(host_out, b.p, (size_t)n * 2, hipMemcpyDeviceToHost));
  });
}

// ---------------------------------------------------------------------------
// misc
// ---------------------------------------------------------------------------

int tmh_synth_sites_device(uint16_t* dev_out, int64_t n_sites, int height, int width, uint64_t seed,
                           int channel, int64_t first_site, int distribution, void* stream) {
  return guard([&] {
    TMH_CHECK(dev_out && n_sites >= 0 && height > 0 && width > 0 && first_site >= 0, TMH_EINVAL,
              "bad arguments");
    TMH_CHECK(distribution >= TMH_SYNTH_STANDARD && distribution <= TMH_SYNTH_UNIFORM, TMH_EINVAL,
              "unknown distribution");
    if (n_sites == 0) return;
    launch_synth(dev_out, n_sites, height, width, seed, channel, first_site, distribution,
                 (hipStream_t)stream);
  });
}

int tmh_box_probe_device(const uint16_t* const* dev_in_blocks, uint16_t* const* dev_out_blocks,
                         int block_shift, int64_t n_sites, int height, int width, int mode,
                         int reps, void* stream, double* ms_out, double* sclk_mhz_out) {
  return guard([&] {
    TMH_CHECK(dev_in_blocks && n_sites > 0 && n_sites < (int64_t(1) << 24) && height > 0 &&
                  width > 0 && ((int64_t)height * width) % 8 == 0 && block_shift >= 0 &&
                  block_shift <= 24 && mode >= 0 && mode <= 3 && reps > 0 && ms_out,
              TMH_EINVAL, "bad arguments");
    const bool write = (mode & 1) == 0, flat = mode >= 2;
    TMH_CHECK(!write || dev_out_blocks, TMH_EINVAL, "the copy probe needs output blocks");
    const hipStream_t s = (hipStream_t)stream;
    int dev = 0, cus = 0;
    TMH_HIP(hipGetDevice(&dev));
    TMH_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DBuf<unsigned long long> clk;
    DBuf<unsigned int> sink;
    clk.alloc(4);
    sink.alloc(1);
    hipEvent_t e0, e1;
    TMH_HIP(hipEventCreate(&e0));
    TMH_HIP(hipEventCreate(&e1));
    const int64_t npx = (int64_t)height * width;
    const int64_t per = (int64_t)1 << block_shift, nb = (n_sites + per - 1) / per;
    std::vector<const uint16_t*> hin;
    std::vector<uint16_t*> hout;
    if (flat) {  // the flat shape launches per block: the block pointers on the host
      hin.resize(nb);
      TMH_HIP(hipMemcpy(hin.data(), dev_in_blocks, nb * sizeof(void*), hipMemcpyDeviceToHost));
      if (write) {
        hout.resize(nb);
        TMH_HIP(hipMemcpy(hout.data(), dev_out_blocks, nb * sizeof(void*), hipMemcpyDeviceToHost));
      }
    }
    TMH_HIP(hipMemsetAsync(clk.p, 0, 4 * sizeof(unsigned long long), s));
    float ms = 0.0f;
    try {
      TMH_HIP(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r) {
        if (!flat) {
          launch_box_probe(dev_in_blocks, const_cast<uint16_t* const*>(dev_out_blocks),
                           block_shift, n_sites, npx, write, clk.p, sink.p, cus, s);
          continue;
        }
        for (int64_t b = 0; b < nb; ++b)
          launch_box_probe_flat(hin[b], write ? hout[b] : nullptr,
                                std::min<int64_t>(per, n_sites - b * per), npx, write, sink.p, s);
      }
      TMH_HIP(hipEventRecord(e1, s));
      TMH_HIP(hipEventSynchronize(e1));
      TMH_HIP(hipEventElapsedTime(&ms, e0, e1));
    } catch (...) {
      (void)hipStreamSynchronize(s);  // no launch left using clk / sink as they unwind
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      throw;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *ms_out = (double)ms / reps;
    if (sclk_mhz_out) {
      unsigned long long t[4];
      TMH_HIP(hipMemcpy(t, clk.p, sizeof(t), hipMemcpyDeviceToHost));
      *sclk_mhz_out = t[3] > t[1] ? 100.0 * (double)(t[2] - t[0]) / (double)(t[3] - t[1]) : 0.0;
    }
  });
}

int tmh_synth_tables(int distribution, int height, int width, int32_t* ln16, int32_t* nz16,
                     int32_t* ey, int32_t* ex) {
  return guard([&] {
    TMH_CHECK(ln16 && nz16 && ey && ex && height > 0 && width > 0, TMH_EINVAL, "bad arguments");
    TMH_CHECK(distribution >= TMH_SYNTH_STANDARD && distribution <= TMH_SYNTH_UNIFORM, TMH_EINVAL,
              "unknown distribution");
    synth_tables_host(distribution, height, width, ln16, nz16, ey, ex);
  });
}

int64_t tmh_inflate_scratch_bytes(int64_t n_chunks, int64_t raw_max) {
  return n_chunks > 0 && raw_max >= 0 ? inflate_scratch_bytes(n_chunks, raw_max) : 0;
}

int tmh_inflate_device(const uint8_t* dev_src, int64_t src_bytes, const tmh_zchunk* dev_chunks,
                       int64_t n_chunks, int64_t raw_max, uint8_t* dev_raw, int64_t raw_bytes,
                       void* dev_scratch, int64_t scratch_bytes, int32_t* dev_status,
                       void* stream) {
  return guard([&] {
    TMH_CHECK(n_chunks >= 0 && src_bytes >= 0 && raw_bytes >= 0 && raw_max >= 0, TMH_EINVAL,
              "bad sizes");
    if (n_chunks == 0) return;
    TMH_CHECK(dev_src && dev_chunks && dev_raw && dev_status && dev_scratch, TMH_EINVAL,
              "bad arguments");
    TMH_CHECK(raw_max < (int64_t(1) << 31), TMH_EINVAL, "chunks must hold fewer than 2^31 bytes");
    TMH_CHECK(scratch_bytes >= inflate_scratch_bytes(n_chunks, raw_max), TMH_EINVAL,
              "scratch smaller than tmh_inflate_scratch_bytes");
    TMH_CHECK((reinterpret_cast<uintptr_t>(dev_scratch) & 15) == 0, TMH_EINVAL,
              "scratch must be 16-byte aligned");
    launch_inflate(dev_src, src_bytes, dev_chunks, n_chunks, raw_max, dev_raw, raw_bytes,
                   static_cast<uint32_t*>(dev_scratch), dev_status, (hipStream_t)stream);
  });
}

int tmh_place_chunks_device(const uint8_t* dev_raw, const tmh_zchunk* dev_chunks, int64_t n_chunks,
                            int height, int width, int elem_bytes, int chunk_rows, int chunk_cols,
                            void* dev_images, void* stream) {
  return guard([&] {
    TMH_CHECK(n_chunks >= 0 && height > 0 && width > 0 && chunk_rows > 0 && chunk_cols > 0 &&
                  (elem_bytes == 1 || elem_bytes == 2 || elem_bytes == 4 || elem_bytes == 8),
              TMH_EINVAL, "bad geometry");
    if (n_chunks == 0) return;
    TMH_CHECK(dev_raw && dev_chunks && dev_images, TMH_EINVAL, "bad arguments");
    launch_place_chunks(dev_raw, dev_chunks, n_chunks, height, width, elem_bytes, chunk_rows,
                        chunk_cols, static_cast<uint8_t*>(dev_images), (hipStream_t)stream);
  });
}

int tmh_malloc_device(void** dev_ptr, size_t bytes) {
  return guard([&] {
    TMH_CHECK(dev_ptr, TMH_EINVAL, "dev_ptr is NULL");
    if (hipMalloc(dev_ptr, bytes) != hipSuccess) {
      *dev_ptr = nullptr;
      throw Error{TMH_ENOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed"};
    }
  });
}

int tmh_free_device(void* dev_ptr) { return guard([&] { TMH_HIP(hipFree(dev_ptr)); }); }

int tmh_memcpy(void* dst, const void* src, size_t bytes, int kind, void* stream) {
  return guard([&] {
    TMH_CHECK(kind >= 0 && kind <= 2, TMH_EINVAL, "kind must be 0 (h2d), 1 (d2h) or 2 (d2d)");
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                          : kind == 1 ? hipMemcpyDeviceToHost
                                      : hipMemcpyDeviceToDevice;
    TMH_HIP(hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)stream));
    TMH_HIP(hipStreamSynchronize((hipStream_t)stream));
  });
}

int tmh_profile_enable(int on) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof_on = on != 0;
  return TMH_OK;
}

int tmh_profile_read(const char* kernel, double* total_ms, int64_t* launches) {
  return guard([&] {
    TMH_CHECK(kernel && total_ms && launches, TMH_EINVAL, "bad arguments");
    std::lock_guard<std::mutex> lk(g_prof_mu);
    auto it = g_prof.find(kernel);
    if (it == g_prof.end()) {
      *total_ms = 0.0;
      *launches = 0;
      return;
    }
    prof_drain(it->second);
    *total_ms = it->second.total_ms;
    *launches = it->second.launches;
  });
}

int tmh_profile_reset(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& kv : g_prof) {
    prof_drain(kv.second);
    kv.second.total_ms = 0.0;
    kv.second.launches = 0;
  }
  return TMH_OK;
}

}  // extern "C"
