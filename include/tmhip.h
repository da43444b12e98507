/*
 * tmhip.h — C-ABI of libtmhip.so, the MI355X (gfx950) implementation of
 * TmLibrary's corilla illumination-statistics path and its apply step.
 *
 * The reference (scottberry/TmLibrary) is pure Python and has no FFI; these
 * entry points are the boundary its Python classes would bind through
 * ctypes.  Each function names the reference interface it replaces.
 *
 * Conventions
 *   - Every int-returning function returns 0 on success and a negative
 *     errno-style code on failure; tmh_last_error() holds a thread-local
 *     message for the last failure on the calling thread.
 *   - "host" pointers are plain CPU memory owned by the caller; "dev"
 *     pointers are device (HBM) memory on the handle's device, owned by the
 *     caller unless stated otherwise.
 *   - stream arguments are hipStream_t passed as void*; NULL means the
 *     handle's own stream.  Host-pointer calls are synchronous on return.
 *   - A handle is not thread-safe; distinct handles may be used from
 *     distinct threads.  No callbacks.
 *   - Sites are contiguous [n_sites][height][width] uint16 images in site
 *     order (the order of batch['channel_image_files_ids'],
 *     tmlib/workflow/corilla/api.py:125-136).
 */
#ifndef TMHIP_H
#define TMHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMH_ABI_VERSION 4

#define TMH_OK 0
#define TMH_EINVAL (-22)  /* bad argument: maps to ValueError / TypeError */
#define TMH_ENOMEM (-12)  /* device or host allocation failed             */
#define TMH_EDEVICE (-5)  /* HIP runtime error                            */
#define TMH_ESTATE (-71)  /* call not valid in the handle's state         */

/* ---- library ---------------------------------------------------------- */
int tmh_abi_version(void);
const char* tmh_last_error(void);
int tmh_device_count(int* n);
int tmh_set_device(int device);
int tmh_synchronize(void* stream);

/* ---- illumination statistics ------------------------------------------
 * Replaces tmlib/workflow/corilla/stats.py:35-121 (OnlineStatistics):
 *   __init__(image_dimensions, decimals)  -> tmh_stats_create
 *   update(image, log_transform)           -> tmh_stats_update[_device]
 *   mean / std / var / percentiles         -> tmh_stats_finalize[_device]
 *
 * n_quantiles = 10**(decimals+2).  q_lo/q_hi/q_gamma are numpy 2.2.6's
 * linear-percentile sorted positions and weights for an image of
 * height*width pixels (previous/next index after the above/below-bound
 * substitution, gamma = virtual - previous), computed on the host so they
 * are bit-identical to np.percentile (stats.py:76).
 * lut_log10[65536] is the stats log transform of every uint16 value
 * (np.log10 with 0 -> 0, stats.py:79-85), built by the host's numpy.
 * batch_capacity is the number of sites the handle stages per launch for
 * host-pointer updates (device updates of any size are processed in
 * place).  flags: TMH_STATS_DEFERRED_PCT keeps every site's order
 * statistics on the device instead of folding them into the accumulator at
 * each update (needed for the multi-GPU percentile chain).
 */
typedef struct tmh_stats tmh_stats;

#define TMH_STATS_DEFERRED_PCT 1u
#define TMH_STATS_KEEP_SITE_HIST 2u /* keep per-site histograms (debug/parity) */
#define TMH_STATS_SERIAL 4u         /* no side stream: histogram after Welford */

int tmh_stats_create(int height, int width, int n_quantiles, const int64_t* q_lo,
                     const int64_t* q_hi, const double* q_gamma, const double* lut_log10,
                     int batch_capacity, unsigned flags, tmh_stats** out);
void tmh_stats_destroy(tmh_stats* h);
int tmh_stats_set_stream(tmh_stats* h, void* stream);
/* Start a new job on the handle (stats.py:53-62 state).  Also restores the
 * handle's zero-maintained histogram slabs if a fused pass was interrupted. */
int tmh_stats_reset(tmh_stats* h);

/* Options of a handle (results never depend on them).  The automatic
 * choices below come from the job's SITE PROBE: at the first Welford launch
 * after tmh_stats_reset, one small kernel samples 16,384 8-pixel groups
 * spread over the launch's first <= 64 sites, and the host waits for its
 * three counts (groups sampled, holding a value >= 4,096, >= 16,384) --
 * so that launch returns only once the probe has run on its stream.  Only
 * the chosen kernels are queued.  The choice assumes the first <= 64 sites
 * stand for the job: a job whose first sites are dark and later sites very
 * wide runs the narrow configurations, its wide values taking their global-
 * atomic path -- results identical, the pass slower (uniform 16-bit sites
 * that way: ~0.5 s per 3,456 sites, against ~36 ms chosen right;
 * test_gpu_parity.py dark_prefix_wide_tail).  Force a configuration
 * (TMH_OPT_FUSED_CONFIG) for such jobs.
 *   TMH_OPT_FUSED_CONFIG   0..5: (sites per unit, threads, LDS bins) of the
 *                          fused correct+histogram pass = (2, 1024, 32768),
 *                          (4, 1024, 32768), (2, 512, 16384), (4, 512, 16384),
 *                          (1, 1024, 32768), (4, 1024, 65536 u16 counters
 *                          packed two sites to a word).  -1 (default): from
 *                          the probe -- 3; or 5 when >= 2% of the probed
 *                          groups hold a value >= 4,096; or, when >= 33% hold
 *                          a value >= 16,384 ("very wide" sites, e.g. uniform
 *                          16-bit data), the pass runs without its histogram
 *                          and a per-site u16-pair LDS histogram pass (one
 *                          more read) builds them; 100 forces that form.
 *   TMH_OPT_WELFORD_PARTS  0 (default): automatic -- with the log transform,
 *                          a launch of >= 96 sites whose job probe found >=
 *                          10% of the groups holding a value >= 4,096 (bright
 *                          sites: the log10 pass is VALU-bound) runs the
 *                          16,384-entry LUT pass in 3 site parts (merged in
 *                          order), else one part; 1..4: that many parts where
 *                          the launch has >= 32 sites a part
 *   TMH_OPT_COPY_THREADS   1..64 (default 8): host threads of the pageable <->
 *                          pinned copies of the host-buffer entry points
 *   TMH_OPT_HOST_STAGING   host-buffer entry points: 0 = the caller's buffers
 *                          go straight to the copy engines; 1 = inputs AND
 *                          outputs through pinned slots; 2 (default) =
 *                          outputs only (the pageable H2D path is as fast as
 *                          a pinned bounce; a pinned D2H slot copied out by
 *                          several threads spreads a fresh output's faults) */
#define TMH_OPT_FUSED_CONFIG 1
#define TMH_OPT_WELFORD_PARTS 2
/* 3, 6 and 7 were TMH_OPT_TAIL_CHUNKS / TMH_OPT_PCT_TAIL / TMH_OPT_FUSED_EPOCHS
 * (percentile-tail variants measured slower than the default, removed) */
#define TMH_OPT_COPY_THREADS 4
#define TMH_OPT_HOST_STAGING 5
int tmh_stats_set_option(tmh_stats* h, int option, int value);

/* update(image) for a run of sites.  zero_counts_out (host, n_sites, may be
 * NULL): per-site number of zero pixels, for the 'image contains zero
 * values' warning (stats.py:81-82).  Host sites move in chunks of the
 * handle's batch capacity through two device slots on a copy stream, so
 * chunk k's H2D overlaps chunk k-1's kernels; returns when all are done. */
int tmh_stats_update(tmh_stats* h, const uint16_t* host_sites, int64_t n_sites,
                     int log_transform, int64_t* zero_counts_out);
/* Stream contract of the device update entry points: on another stream than
 * the handle's, the work runs after everything already queued on the
 * handle's stream, and the handle's stream waits for it before any later work
 * on the handle (finalize, merge, ...), so results read on the handle's
 * stream are complete.  The wait is queued with the handle's next work (a
 * wait queued at once would hold up every stream sharing the handle stream's
 * hardware queue until the awaited pass ended): work a caller queues on the
 * handle's stream itself, outside this library, is not ordered after it --
 * order such work against the caller's stream, or synchronise. */
int tmh_stats_update_device(tmh_stats* h, const uint16_t* dev_sites, int64_t n_sites,
                            int log_transform, void* stream);
/* Per-site zero-pixel counts of the LAST CHUNK of the last update call: the
 * call's sites in chunks of 4,096, so for a call of <= 4,096 sites these are
 * its sites' counts (n <= that chunk's size, else TMH_EINVAL).  Copied to
 * host_out on `stream` after the handle's queued work (asynchronous for
 * pinned host_out). */
int tmh_stats_zero_counts(tmh_stats* h, int64_t* host_out, int64_t n, void* stream);

/* Split job pipeline (one read of the sites per pass):
 *   tmh_stats_update_welford_device  Welford only; the sites' percentile
 *                                    contributions are left pending
 *   tmh_correct_u16_hist_device      (below) corrects the SAME sites, in the
 *                                    same order, and builds their histograms
 *                                    from that read, completing the pending
 *                                    percentile state.
 * Results are identical to tmh_stats_update_device + tmh_correct_u16_device. */
int tmh_stats_update_welford_device(tmh_stats* h, const uint16_t* dev_sites, int64_t n_sites,
                                    int log_transform, void* stream);

/* The job's site probe (see the options above), queued now on `stream`
 * without waiting for it: the first Welford launch of the job then only
 * waits for the probe's counts.  A caller running several jobs on several
 * streams (a rank's channels) queues every job's probe first, so that no
 * launch waits for another job's kernels to drain before its probe can run.
 * Optional: a job not probed this way is probed by its first Welford launch.
 * Stream: the probe reads only the sites and its counts go to the host, so
 * it is ordered after `stream`'s queued work alone (the sites must be ready
 * there; NULL: the handle's stream) and nothing of the handle waits for it:
 * on a stream of its own it runs as soon as the sites are, whatever the
 * handle still has queued (the previous job's merges and tails).  Call it
 * after tmh_stats_reset. */
int tmh_stats_probe_device(tmh_stats* h, const uint16_t* dev_sites, int64_t n_sites,
                           void* stream);
int tmh_stats_probe_blocks_device(tmh_stats* h, const uint16_t* const* dev_blocks, int block_shift,
                                  int64_t n_sites, void* stream);

/* Blocked site layout (device entry points below): the n_sites sites, in
 * site order, live in blocks of 2^block_shift consecutive sites (2 <= shift
 * <= 24; the last block may be partial), block b at dev_blocks[b] -- a DEVICE
 * array of device pointers, 16-byte aligned (hipMalloc's are), owned by the
 * caller.  Sites that arrive one file at a time need not be copied into one
 * allocation, and a job's 38 GB of sites and outputs spread over many
 * allocations: the fused pass's speed depended on which 38 GB buffer held its
 * output (12.8-15.2 ms on one box; blocks of 4-64 sites allocated in- and
 * output alternately ran 13.1 on every draw).  Results are
 * identical to the contiguous entry points.  Needs height*width % 8 == 0. */
int tmh_stats_update_welford_blocks_device(tmh_stats* h, const uint16_t* const* dev_blocks,
                                           int block_shift, int64_t n_sites, int log_transform,
                                           void* stream);

/* Host copies of the results; any output may be NULL.
 *   n            sites accumulated (stats.py:89)
 *   mean, std    [height*width] f64; std is NaN where n < 2 (stats.py:94-112)
 *   pct_sum      [n_quantiles] f64 running sum of per-site percentiles in
 *                site order (stats.py:76); values = int(pct_sum / n)
 *   hist         [65536] u64 pooled per-site histogram (sum over sites) */
int tmh_stats_finalize(tmh_stats* h, int64_t* n, double* mean, double* std, double* pct_sum,
                       uint64_t* hist);
/* Device form: writes mean/std planes into caller device buffers. */
int tmh_stats_finalize_device(tmh_stats* h, double* dev_mean, double* dev_std, void* stream);
/* var = M2 / (n - 1), NaN everywhere when n < 2 (stats.py:94-102), host copy. */
int tmh_stats_variance(tmh_stats* h, double* host_var);
/* Pixel groups (8 consecutive pixels of one site) holding a value >= 4,096
 * in the sites passed to tmh_stats_update_welford_device since the last fused
 * pass consumed them (synchronous; diagnostics: the automatic fused
 * configuration compares it with 2% of the groups).  sites_out may be NULL. */
int tmh_stats_wide_groups(tmh_stats* h, uint64_t* groups_out, int64_t* sites_out);
/* The current job's site probe and the automatic choices it made (see the
 * options above): probe_counts[3] = groups sampled, groups with a value >=
 * 4,096, >= 16,384 (zeros before the probe ran); welford_bright = 1 / 0, -1
 * if the job has not been probed; fused_cfg = the configuration the fused
 * pass runs (0..5, or TMH_FUSED_NO_HIST).  Any output may be NULL. */
#define TMH_FUSED_NO_HIST 100
int tmh_stats_job_choice(tmh_stats* h, uint32_t* probe_counts, int* welford_bright,
                         int* fused_cfg);
/* Per-site histogram of the most recent update batch (debug/parity). */
int tmh_stats_site_histogram(tmh_stats* h, int64_t site_in_last_batch, uint32_t* host_hist);
/* Order statistics at every quantile's previous/next sorted position for one
 * site (last batch; any stored site in deferred mode) — debug/parity. */
int tmh_stats_site_order_stats(tmh_stats* h, int64_t site, uint16_t* host_vlo,
                               uint16_t* host_vhi);

/* ---- multi-GPU merge (one process per GPU; collectives done by the caller
 * over RCCL on the device buffers these functions fill/consume).  Every
 * entry point below that takes a stream follows the updates' stream
 * contract: on another stream than the handle's it runs after the handle's
 * queued work and the handle's stream waits for it (so one stream can merge
 * several handles -- a rank's channels -- with batched collectives). ---- */
int tmh_stats_get_n(tmh_stats* h, int64_t* n);
/* The reference's plain attribute OnlineStatistics.n (stats.py:53): the count
 * later Welford updates continue from and percentiles / var divide by. */
int tmh_stats_set_n(tmh_stats* h, int64_t n);
/* dev_nmean = n_r * mean_r (input of all_reduce(sum)) */
int tmh_stats_merge_stage1(tmh_stats* h, double* dev_nmean, void* stream);
/* mean = dev_sum_nmean / n_total; dev_m2c = M2_r + n_r * (mean_r - mean)^2 */
int tmh_stats_merge_stage2(tmh_stats* h, const double* dev_sum_nmean, int64_t n_total,
                           double* dev_m2c, void* stream);
/* Adopt the merged state: n = n_total, mean from stage 2, M2 = dev_sum_m2c. */
int tmh_stats_merge_stage3(tmh_stats* h, int64_t n_total, const double* dev_sum_m2c,
                           void* stream);
/* Percentile chain: dev_acc[n_quantiles] += each local site's percentiles,
 * in local site order (deferred mode).  Rank r runs this on the accumulator
 * received from rank r-1, keeping the reference's sequential summation. */
int tmh_stats_pct_accumulate(tmh_stats* h, double* dev_acc, void* stream);
/* Same for quantiles [q_begin, q_begin + q_count) only; dev_acc_range points at
 * the range's first element.  Lets the rank chain run as a pipeline over
 * quantile chunks (rank r adds chunk c while rank r-1 adds chunk c+1); each
 * quantile still sees every rank's sites in order (bit-exact). */
int tmh_stats_pct_accumulate_range(tmh_stats* h, double* dev_acc_range, int q_begin, int q_count,
                                   void* stream);
int tmh_stats_set_pct_sum(tmh_stats* h, const double* dev_acc, void* stream);
/* Device copy of the percentile sums (what tmh_stats_finalize's pct_sum
 * returns; deferred mode: summed in site order first unless a chain result
 * was installed), ordered on `stream` -- lets a pipelined caller keep a job's
 * results before the handle is reused, without a host synchronisation. */
int tmh_stats_get_pct_sum_device(tmh_stats* h, double* dev_acc, void* stream);
/* Pooled 65,536-bin u64 histogram out of / into the handle (device buffers):
 * the histogram merge is get -> all_reduce(sum) -> set.  Sums of counts are
 * exact, so any reduction order gives the same bins. */
int tmh_stats_get_hist_device(tmh_stats* h, uint64_t* dev_hist, void* stream);
int tmh_stats_set_hist_device(tmh_stats* h, const uint64_t* dev_hist, void* stream);

/* ---- smoothing -----------------------------------------------------------
 * Replaces tmlib/image.py:287-311 Image.smooth -> mahotas.gaussian_filter
 * (image.py:303) as used by IllumstatsContainer.smooth (image.py:1172-1193):
 * separable Gaussian, radius int(4*sigma+0.5), normalised taps, 'reflect'
 * border, float64, axis 0 then axis 1.  in == out is allowed. */
int tmh_smooth_f64(const double* host_in, double* host_out, int height, int width, double sigma);
int tmh_smooth_f64_device(const double* dev_in, double* dev_out, double* dev_tmp, int height,
                          int width, double sigma, void* stream);
/* The same for two planes (a job's mean and std, image.py:1185-1186) in one
 * launch per axis; bit-identical to two tmh_smooth_f64_device calls.
 * dev_tmp0 / dev_tmp1: scratch planes of their own. */
int tmh_smooth2_f64_device(const double* dev_in0, const double* dev_in1, double* dev_out0,
                           double* dev_out1, double* dev_tmp0, double* dev_tmp1, int height,
                           int width, double sigma, void* stream);

/* ---- correction ------------------------------------------------------------
 * Replaces tmlib/image.py:599-631 ChannelImage._correct_illumination,
 * image.py:633-670 correct, and image.py:570-597 clip.
 * A corrector holds the per-pixel affine form of the correction for one
 * (mean, std) pair:  log: out = 10**(a*log10(x) + b), a = mean(std)/std,
 * b = mean(mean) - mean*a, x==0 -> log10(1e-10);  no log: out = a*x + b.
 * lut_zero_log10 = np.log10(1e-10) from the host numpy.  The float result is
 * cast with the x86 astype rule (trunc to int32, low bits) and optionally
 * clipped to [clip_lo, clip_hi] (clip_lo < 0: no clip). */
/* One site's alignment window (Image.align, tmlib/image.py:345-454): output
 * pixel (r, c) with 0 <= r - dst_r0 < rows and 0 <= c - dst_c0 < cols takes
 * input pixel (r - dst_r0 + src_r0, c - dst_c0 + src_c0); every other output
 * pixel is 0.  The host evaluates the reference's numpy slicing into it. */
typedef struct tmh_window {
  int32_t src_r0, src_c0, dst_r0, dst_c0, rows, cols;
} tmh_window;

typedef struct tmh_corrector tmh_corrector;

int tmh_corrector_create(const double* host_mean, const double* host_std, int height, int width,
                         int log_transform, double zero_log10, tmh_corrector** out);
int tmh_corrector_create_device(const double* dev_mean, const double* dev_std, int height,
                                int width, int log_transform, double zero_log10, void* stream,
                                tmh_corrector** out);
void tmh_corrector_destroy(tmh_corrector* c);
/* Recompute the coefficients in place from new device planes (no allocation,
 * no synchronisation): one corrector serves every job of the same shape. */
int tmh_corrector_update_device(tmh_corrector* c, const double* dev_mean, const double* dev_std,
                                void* stream);
/* Options of a corrector: TMH_OPT_COPY_THREADS, TMH_OPT_HOST_STAGING (see
 * tmh_stats_set_option), and TMH_OPT_FUSED_CUS: the fused correct+histogram
 * pass's persistent grid spans this many CUs' worth of workgroups (0 or the
 * CU count, default: all) -- fewer leave room for other streams' kernels
 * (several channel jobs sharing a GPU).  Results never depend on them. */
#define TMH_OPT_FUSED_CUS 8
/* TMH_OPT_FUSED_BANDS: pixel bands of the fused pass's unit sweep, 0
 * (default: the configuration's, doubled up to 64 while a launch has fewer
 * than 8 units per workgroup -- short launches, e.g. a rank's 432-site share
 * of a channel at N = 8), or 8 / 16 / 32 / 64. */
#define TMH_OPT_FUSED_BANDS 9
int tmh_corrector_set_option(tmh_corrector* c, int option, int value);
/* The two global means (np.mean(std), np.mean(mean), image.py:627). */
int tmh_corrector_means(tmh_corrector* c, double* mean_of_std, double* mean_of_mean);
/* tmh_corrector_update_device for n <= 8 correctors (a rank's channels) in
 * one launch per kernel (the plane sums, every coefficient form, the launch
 * constants), on `stream` (NULL: the first corrector's); results identical
 * to n separate calls. */
int tmh_corrector_update_multi_device(tmh_corrector* const* cs, int n, const double* const* dev_mean,
                                      const double* const* dev_std, void* stream);
/* The planes step of n <= 8 jobs at once (a rank's channels, configs[2]/[3];
 * reference: one corilla job per channel, tmlib/workflow/corilla/api.py:64-105):
 * per job k, statistics finalize (stats.py:94-112) -> IllumstatsContainer
 * smoothing of mean and std (image.py:1172-1193, sigma) -> corrector k's
 * coefficients from the smoothed planes (image.py:599-631).  One launch per
 * kernel for all jobs: the smoothing reads each handle's mean and M2 and
 * finalizes std as it reads it (sigma 5; other sigmas finalize into scratch
 * first), then the coefficient launches of tmh_corrector_update_multi_device.
 * dev_smean / dev_sstd [n]: the smoothed planes (device, f64 [height*width]);
 * dev_mean / dev_std (may be NULL, or hold NULL entries): the unsmoothed
 * planes, written only where asked for.  Runs on `stream` (NULL: the first
 * handle's) after everything queued on every handle's stream, and every
 * handle's stream waits for it.  Results identical to finalize + smooth2 +
 * corrector update per job. */
int tmh_job_planes_multi_device(tmh_stats* const* hs, tmh_corrector* const* cs, int n,
                                double* const* dev_mean, double* const* dev_std,
                                double* const* dev_smean, double* const* dev_sstd, double sigma,
                                void* stream);
/* Host buffers: chunks of <= 16 sites, H2D / kernel / D2H on three streams
 * with two device and two pinned output slots (TMH_OPT_HOST_STAGING).  Returns when host_out is
 * complete; host_out must not overlap host_in. */
int tmh_correct_u16(tmh_corrector* c, const uint16_t* host_in, uint16_t* host_out,
                    int64_t n_sites, int clip_lo, int clip_hi);
int tmh_correct_u16_device(tmh_corrector* c, const uint16_t* dev_in, uint16_t* dev_out,
                           int64_t n_sites, int clip_lo, int clip_hi, void* stream);
/* Correct n_sites pending sites of h and fold their histograms/percentiles
 * into h (see tmh_stats_update_welford_device).  Stream contract: the work
 * runs on `stream` (NULL: the corrector's stream), ordered after everything
 * already queued on h's stream, and h's stream waits for it before any later
 * work on h -- the two handles may live on different streams.  On another
 * stream than h's, the histogram tail (per-site order statistics, percentile
 * sums) runs on a stream of h's own, which h's stream waits for:
 * `stream` is free once the corrected sites are written, so a caller can
 * start its next job under this one's tail.
 * dev_in and
 * dev_out must not overlap (the pass re-reads its input after storing
 * outputs: f64 fixups, packed-counter recounts; overlapping runs are
 * rejected with TMH_EINVAL, and the block entry point's tables must name
 * separate blocks). */
int tmh_correct_u16_hist_device(tmh_corrector* c, tmh_stats* h, const uint16_t* dev_in,
                                uint16_t* dev_out, int64_t n_sites, int clip_lo, int clip_hi,
                                void* stream);
/* The same on the blocked layout (see tmh_stats_update_welford_blocks_device):
 * input and output block tables with the same block_shift; the correction's
 * zero_log10 must lie in [-37, 0] (the fused pass). */
int tmh_correct_u16_hist_blocks_device(tmh_corrector* c, tmh_stats* h,
                                       const uint16_t* const* dev_in_blocks,
                                       uint16_t* const* dev_out_blocks, int block_shift,
                                       int64_t n_sites, int clip_lo, int clip_hi, void* stream);
/* n <= 8 jobs' tmh_correct_u16_hist_device (the same image size and
 * transform, each job its own corrector and statistics handle, n_sites[k]
 * pending sites of handle k) in ONE fused launch when their configurations
 * agree (a rank's channels: a short job's launch otherwise pays the pass's
 * fill and drain on its own); a job whose configuration differs, or which
 * needs the two-pass path, gets its own launch on the same stream.  Runs on
 * `stream` (NULL: the first corrector's); the stream contract of the
 * single-job call holds for every job (each after its handle's queued work,
 * each handle's stream after its job's tail).  Results identical to the
 * per-job calls. */
int tmh_correct_u16_hist_multi_device(tmh_corrector* const* cs, tmh_stats* const* hs, int n,
                                      const uint16_t* const* dev_in, uint16_t* const* dev_out,
                                      const int64_t* n_sites, int clip_lo, int clip_hi,
                                      void* stream);
/* The same on the blocked layout: per job an input and an output block table
 * (device arrays of block pointers), one block_shift for all. */
int tmh_correct_u16_hist_multi_blocks_device(tmh_corrector* const* cs, tmh_stats* const* hs,
                                             int n, const uint16_t* const* const* dev_in_blocks,
                                             uint16_t* const* const* dev_out_blocks,
                                             int block_shift, const int64_t* n_sites, int clip_lo,
                                             int clip_hi, void* stream);
int tmh_correct_u8(tmh_corrector* c, const uint8_t* host_in, uint8_t* host_out, int64_t n_sites,
                   int clip_lo, int clip_hi);
/* ---- illuminati chain ------------------------------
 * Image.align (tmlib/image.py:412-454) of n_sites images [n][height][width] of
 * elem_bytes 1 (uint8) or 2 (uint16) into [n][out_height][out_width]: crop=True
 * gives out = window extent, crop=False out = input size, zero padded. */
int tmh_align(const void* host_in, void* host_out, int elem_bytes, int64_t n_sites, int height,
              int width, const tmh_window* windows, int out_height, int out_width);
/* ChannelImage._map_to_uint8 (tmlib/image.py:493-531) with explicit bounds
 * (0 <= lower < upper <= 65535): the reference's numpy LUT, bit-exact. */
int tmh_map_u16_to_u8(const uint16_t* host_in, uint8_t* host_out, int64_t n, int lower,
                      int upper);
/* illuminati/api.py:396-405 in one pass: correct (this corrector's statistics)
 * -> align(crop=False) with each site's window -> clip(clip_lo, clip_hi) ->
 * scale(clip_lo, clip_hi) to uint8.  Corrected values within +-1 DN of the
 * reference before the clip/scale (the +-1 DN bar of the correction). */
int tmh_correct_chain_u8_device(tmh_corrector* c, const uint16_t* dev_in, uint8_t* dev_out,
                                int64_t n_sites, const tmh_window* host_windows, int clip_lo,
                                int clip_hi, void* stream);
int tmh_correct_chain_u8(tmh_corrector* c, const uint16_t* host_in, uint8_t* host_out,
                         int64_t n_sites, const tmh_window* host_windows, int clip_lo,
                         int clip_hi);

/* ChannelImage.clip alone (image.py:589), u16. */
int tmh_clip_u16(const uint16_t* host_in, uint16_t* host_out, int64_t n, int lo, int hi);

/* ---- synthetic input (imextract stand-in for benchmarks) -----------------
 * Sites [first_site, first_site + n_sites) of (seed, channel), generated in
 * HBM with integer arithmetic only, so tmlibrary_amd/synth.py
 * (synth_exact_host) reproduces every pixel bit for bit on the host and the
 * bench's full-size results can be checked against the CPU oracle.
 * distribution: TMH_SYNTH_STANDARD  100 + vignetting * LogNormal(6, 0.6) + N(0, 5)
 *               TMH_SYNTH_BRIGHT    the same with LogNormal(8.5, 0.6) (median ~5,000)
 *               TMH_SYNTH_UNIFORM   uniform 0..65535
 * (STANDARD / BRIGHT also carry 0.01 % zeros and 0.01 % saturated pixels.) */
#define TMH_SYNTH_STANDARD 0
#define TMH_SYNTH_BRIGHT 1
#define TMH_SYNTH_UNIFORM 2
int tmh_synth_sites_device(uint16_t* dev_out, int64_t n_sites, int height, int width,
                           uint64_t seed, int channel, int64_t first_site, int distribution,
                           void* stream);
/* The generator's integer tables (host only, no GPU needed): ln16/nz16
 * [4096] (lognormal and noise quantiles in 1/16 DN), ey[height], ex[width]
 * (vignetting factors, 2^15 = 1). */
int tmh_synth_tables(int distribution, int height, int width, int32_t* ln16, int32_t* nz16,
                     int32_t* ey, int32_t* ex);

/* ---- box probe (bench support; no reference counterpart) ------------------
 * The box's own stream rates for the two passes' bytes, so a bench line can
 * tell a slow box from a slow kernel: even modes copy -- read every site's 2
 * B/px and write them to its output block (the fused correct+histogram pass's
 * bytes) --, odd modes read every site once (the Welford pass's); 16-byte
 * non-temporal loads and stores as the passes move them, over the caller's
 * blocked layout (device block tables as in
 * tmh_stats_update_welford_blocks_device; shift 24 with one entry: one
 * contiguous run; dev_out_blocks unused when reading).  Modes 0 / 1: one
 * persistent grid-strided launch; 2 / 3: one thread per 16 bytes, one launch
 * per block.  reps repetitions on `stream`; ms_out = their average (HIP
 * events), sclk_mhz_out (may be NULL) = the shader clock during the last
 * persistent launch (clock64 ticks per 100 MHz wall_clock64 tick in
 * workgroup 0; 0 for modes 2 / 3).  Synchronous.  The copy modes overwrite
 * the output blocks with the sites: probe before the outputs are produced or
 * after they have been checked. */
int tmh_box_probe_device(const uint16_t* const* dev_in_blocks, uint16_t* const* dev_out_blocks,
                         int block_shift, int64_t n_sites, int height, int width, int mode,
                         int reps, void* stream, double* ms_out, double* sclk_mhz_out);

/* ---- site-image input: GPU inflate of HDF5 gzip chunks ------------------
 * Replaces the deflate filter libhdf5 runs under h5py for every chunk of a
 * ChannelImageFile's /array (tmlib/models/file.py:322-351,
 * tmlib/readers.py:367-389; written by file.py:353-363, writers.py:384-387):
 * each chunk is an independent zlib stream (RFC 1950/1951), decoded by one
 * GPU lane.  The compressed chunks of many files (libtmh5's
 * tmh5_read_raw_chunks fills the same table layout) sit in one device
 * buffer; tmh_inflate_device writes chunk i's raw_len decompressed bytes at
 * dev_raw + raw_off and its status (TMH_Z_*; 0 = ok) -- byte-identical to
 * zlib's inflate, Adler-32 checked.  tmh_place_chunks_device then copies
 * every chunk's rows into dev_images[image][height][width] (elem_bytes per
 * element), clipping edge chunks to the dataset's extent. */
#define TMH_ZCHUNK_STORED 1 /* the deflate filter was skipped: raw bytes stored */
typedef struct tmh_zchunk {
  int64_t src_off;    /* the chunk's zlib stream in the compressed buffer */
  int64_t src_len;
  int64_t raw_off;    /* its decompressed bytes in the raw buffer */
  int64_t raw_len;    /* chunk_rows * chunk_cols * elem_bytes */
  int64_t image;      /* destination image of tmh_place_chunks_device */
  int32_t row0, col0; /* chunk origin in the image, elements */
  int32_t flags;      /* TMH_ZCHUNK_STORED */
  int32_t reserved;
} tmh_zchunk;
#define TMH_Z_OK 0
#define TMH_Z_HEADER 1     /* not a zlib stream (CM/CINFO/FCHECK/FDICT) */
#define TMH_Z_BLOCKTYPE 2  /* deflate block type 3 */
#define TMH_Z_CODE 3       /* a code the block's Huffman tables do not hold */
#define TMH_Z_DIST 4       /* a back-reference before the start of the chunk */
#define TMH_Z_OVERFLOW 5   /* more than raw_len bytes */
#define TMH_Z_INPUT 6      /* ran past the chunk's bytes / bad offsets */
#define TMH_Z_ADLER 7      /* Adler-32 mismatch */
#define TMH_Z_SIZE 8       /* fewer than raw_len bytes */
#define TMH_Z_STORED 9     /* stored block LEN / NLEN mismatch */
#define TMH_Z_TABLE 10     /* invalid code lengths (over-subscribed, no end code) */
/* Two kernels: each lane Huffman-decodes one chunk, writing its literal bytes
 * and listing its back-references in dev_scratch (no lane waits on a load of
 * earlier output); then one wave per chunk resolves the list in order, 64
 * matches at a time, and checks the Adler-32.  raw_max: the largest raw_len
 * of the table; dev_scratch: at least tmh_inflate_scratch_bytes(n_chunks,
 * raw_max) bytes, 16-byte aligned.  TMH_INFLATE_LANES (4..64, env) sets the
 * streams per phase-1 workgroup (default: from n_chunks and the CU count). */
int64_t tmh_inflate_scratch_bytes(int64_t n_chunks, int64_t raw_max);
int tmh_inflate_device(const uint8_t* dev_src, int64_t src_bytes, const tmh_zchunk* dev_chunks,
                       int64_t n_chunks, int64_t raw_max, uint8_t* dev_raw, int64_t raw_bytes,
                       void* dev_scratch, int64_t scratch_bytes, int32_t* dev_status,
                       void* stream);
int tmh_place_chunks_device(const uint8_t* dev_raw, const tmh_zchunk* dev_chunks, int64_t n_chunks,
                            int height, int width, int elem_bytes, int chunk_rows, int chunk_cols,
                            void* dev_images, void* stream);

/* ---- device memory helpers for callers without another allocator -------- */
int tmh_malloc_device(void** dev_ptr, size_t bytes);
int tmh_free_device(void* dev_ptr);
int tmh_memcpy(void* dst, const void* src, size_t bytes, int kind /*0 h2d,1 d2h,2 d2d*/,
               void* stream);

/* ---- timing of the most recent launches (bench/roofline support) ---------
 * Per-kernel event timing on the handle's stream, enabled by flag. */
int tmh_profile_enable(int on);
int tmh_profile_read(const char* kernel, double* total_ms, int64_t* launches);
int tmh_profile_reset(void);

#ifdef __cplusplus
}
#endif
#endif /* TMHIP_H */
