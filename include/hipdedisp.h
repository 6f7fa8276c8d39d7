/*
 * hipdedisp.h — C ABI of libhipdedisp.so, the MI355X dedispersion engine that
 * replaces the two `prepsubband` invocations of the PALFA search loop.
 *
 * Reference interface being replaced (pipeline2.0, read as text):
 *   lib/python/PALFA2_presto_search.py:506-511  stage 1: prepsubband -sub -subdm S -downsamp ds
 *                                                 -nsub 96 -mask M -o tmp/subbands/<base> <raw>
 *   lib/python/PALFA2_presto_search.py:514-520  stage 2: prepsubband -lodm L -dmstep D -numdms n
 *                                                 -downsamp 1 -nsub 96 -numout choose_N(N/ds)
 *                                                 -o tmp/<base> tmp/subbands/<base>_DM<S>.sub[0-9]*
 *   lib/python/PALFA2_presto_search.py:522-529  use_subbands=False variant (raw -> .dat directly)
 *   lib/python/PALFA2_presto_search.py:95-139   timed_execute: non-zero status -> PrestoError
 *
 * The reference crosses this boundary as a shell command + files; the ABI below is the
 * in-process equivalent.  Conventions:
 *   - every call returns int: HD_OK (0) or a negative HD_E_* code; no exceptions cross;
 *   - hd_last_error(ctx) returns the message of the last failure on that context
 *     (ctx == NULL: last failure of a call that had no context, e.g. hd_open);
 *   - plain C types only; all host buffers are caller-owned and are not retained past
 *     the call that receives them (hd_push_raw copies synchronously into device memory);
 *   - a context is bound to one HIP device and one stream and is NOT thread-safe; use one
 *     context per host thread (contexts on different devices run concurrently);
 *   - channel index c is ascending-frequency order (after the PSRFITS band flip) everywhere
 *     except raw bytes, which stay in file order.
 */
#ifndef HIPDEDISP_H
#define HIPDEDISP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Only the hd_* entry points are exported (the library builds with -fvisibility=hidden). */
#define HD_API __attribute__((visibility("default")))

#define HD_OK        0
#define HD_E_INVAL  -1   /* bad argument / inconsistent shapes          */
#define HD_E_NODEV  -2   /* no HIP device / device index out of range   */
#define HD_E_HIP    -3   /* HIP runtime error (message has the detail)  */
#define HD_E_NOMEM  -4   /* device or host allocation failed            */
#define HD_E_STATE  -5   /* call out of order (e.g. no raw data yet)    */
#define HD_E_IO     -6   /* file I/O failed                             */

/* Subband sample storage (PRESTO writes .subNN as 16-bit ints; f32 keeps them exact). */
#define HD_SUB_I16   0
#define HD_SUB_F32   1
/* Downsampling of subbands: sum of ds samples, or their mean (prepsubband's get_data
 * divides the ds-sample sum by -downsamp [PRESTO-ext]; the default). */
#define HD_DS_SUM    0
#define HD_DS_MEAN   1
/* Padding of a DM series from its length N/ds up to numout. */
#define HD_PAD_MEAN  0   /* per-DM mean of the series' data samples (double sum, cast to f32) */
#define HD_PAD_ZERO  1
#define HD_PAD_DM0   2   /* prepsubband: the running mean of the FIRST DM's data samples,
                            for every DM [PRESTO-ext] (the default); computed as the exact
                            mean (integer sums for int16 subbands), cast to f32          */
/* int16 subband rounding. */
#define HD_ROUND_PRESTO  0   /* prepsubband's (short)(x + 0.5) as x86-64 evaluates it: the
                                double x + 0.5 truncated to int32, low 16 bits (default)  */
#define HD_ROUND_NEAREST 1   /* nearest, ties away from zero, saturated                    */

typedef struct hd_ctx  hd_ctx;
typedef struct hd_plan hd_plan;

/* Observation, as read from the PSRFITS headers
 * (reference: lib/python/formats/psrfits.py:116-134, 210-220, 272-314). */
typedef struct {
    int32_t   nchan;     /* NCHAN                                                   */
    int32_t   nbits;     /* NBITS: 4, 8 or 16                                       */
    int32_t   npol;      /* NPOL (only 1 supported: summed polarisations)          */
    int32_t   flip;      /* 1: raw channels are in descending frequency (need_flipband) */
    double    dt;        /* TBIN, seconds                                           */
    double    lofreq;    /* MHz, centre of the lowest-frequency channel             */
    double    df;        /* MHz, channel width, > 0                                 */
    int64_t   N;         /* spectra in the observation                              */
    int32_t   nsblk;     /* NSBLK, spectra per PSRFITS row                          */
    int32_t   _pad0;
    double    voverc;    /* average barycentric v/c; 0 == prepsubband -nobary      */
} hd_obs;

/* PRESTO-semantics switches.  Defaults: hd_opts_default(). */
typedef struct {
    int32_t   sub_dtype;       /* HD_SUB_I16 (default) | HD_SUB_F32                      */
    int32_t   ds_mode;         /* HD_DS_MEAN (default) | HD_DS_SUM                       */
    int32_t   pad_mode;        /* HD_PAD_DM0 (default) | HD_PAD_MEAN | HD_PAD_ZERO       */
    int32_t   nibble_hi_first; /* 4-bit: first sample in the high nibble (default 1)     */
    int32_t   be16;            /* 16-bit samples big-endian as stored in FITS (default 1)*/
    int32_t   inf_roundtrip;   /* subband-level freq/dt pass through "%.12g"/"%.15g" text,
                                  as they do through the .sub.inf file (default 1)        */
    float     clip_sigma;      /* PRESTO clip_times threshold on each raw read block (obs
                                  nsblk spectra); 6.0 = prepsubband's default -clip, which
                                  the reference's commands leave on; 0 = -noclip           */
    int32_t   sub_round;       /* HD_ROUND_PRESTO (default) | HD_ROUND_NEAREST           */
} hd_opts;

/* One prepsubband pass: stage-1 subbanding at subdm + stage-2 sweep over numdms DMs. */
typedef struct {
    double    subdm;     /* -subdm                                      */
    double    lodm;      /* stage-2 -lodm (value of the "%.2f" argument) */
    double    dmstep;    /* stage-2 -dmstep                             */
    int32_t   numdms;    /* stage-2 -numdms                             */
    int32_t   nsub;      /* -nsub (nchan % nsub == 0)                   */
    int32_t   ds;        /* stage-1 -downsamp (stage 2 runs at -downsamp 1) */
    int32_t   flags;     /* HD_PASS_* below                             */
    int64_t   numout;    /* stage-2 -numout; 0 == N/ds (no padding)     */
} hd_pass;

/* hd_pass.flags: the observation IS the subband file set (stage-2-only prepsubband run on
 * .subNN input): nsub == nchan, ds == 1, and lofreq/df/dt are taken as read from the
 * .sub.inf, without re-deriving them.  Only hd_set_subbands + hd_run_dedisp apply.      */
#define HD_PASS_SUB_INPUT 1

/* Synthetic PALFA-like beam description for hd_synth_* (SURVEY.md §8d). */
#define HD_SYNTH_MAX_PSR 8
typedef struct {
    uint64_t  seed;
    float     base_level;      /* mean level of a channel (digitiser units)      */
    float     bandpass_slope;  /* fractional level change across the band        */
    float     noise_sigma;     /* per-channel noise sigma (digitiser units)      */
    int32_t   npsr;            /* periodic sources in psr_* below                */
    int32_t   nspulse;         /* single pulses in sp_* below                    */
    double    psr_period[HD_SYNTH_MAX_PSR];  /* s   */
    double    psr_dm[HD_SYNTH_MAX_PSR];
    double    psr_width[HD_SYNTH_MAX_PSR];   /* s   */
    float     psr_amp[HD_SYNTH_MAX_PSR];     /* digitiser units per channel */
    double    sp_time[HD_SYNTH_MAX_PSR];     /* s, arrival time at the top of the band */
    double    sp_dm[HD_SYNTH_MAX_PSR];
    double    sp_width[HD_SYNTH_MAX_PSR];
    float     sp_amp[HD_SYNTH_MAX_PSR];
    int32_t   rfi_nchan;       /* persistent narrowband RFI channels (ascending index list) */
    int32_t   rfi_chan[8];
    float     rfi_amp;
    float     burst_frac;      /* fraction of (interval, channel) cells with bursty RFI */
    int32_t   burst_len;       /* samples per bursty interval                   */
    float     burst_amp;
    float     spike_frac;      /* fraction of spectra carrying a zero-DM broadband spike */
    float     spike_amp;
} hd_synth;

/* ---- library / context -------------------------------------------------------- */
HD_API const char* hd_version(void);
HD_API void        hd_opts_default(hd_opts* opts);
HD_API void        hd_synth_default(hd_synth* s);
HD_API int         hd_device_count(int* n);
/* device = HD_HOST_ONLY: a context bound to no device (its device entry points fail with
 * HD_E_HIP); it exists for tests of the context life cycle on machines without a GPU.     */
#define HD_HOST_ONLY (-1)
HD_API int         hd_open(int device, hd_ctx** out);
/* Releases everything the context holds.  After a device fault (a sticky HIP error such as
 * an illegal memory access, seen by any earlier call on the context) the device is unusable
 * for the rest of the process: hd_close then makes NO device call (HIP's teardown calls on a
 * faulted device can abort the process), releases the host side only and returns HD_E_HIP,
 * so the caller's failure path (PrestoError -> the job pool's retry,
 * lib/python/job.py:140-165) still runs.  hd_plan_destroy behaves the same way.            */
HD_API int         hd_close(hd_ctx* ctx);
/* Test hook: mark the context faulted as a sticky HIP error would (no device call).        */
HD_API int         hd_debug_fault(hd_ctx* ctx);
HD_API const char* hd_last_error(const hd_ctx* ctx);
HD_API int         hd_sync(hd_ctx* ctx);
/* Streams for stage 2 (default 1).  With 2, consecutive hd_run_dedisp calls alternate
 * between two HIP streams, so one pass's last tiles share the GPU with the next pass's
 * first ones (no launch tail); stage 1 and hd_set_subbands wait for the second stream's
 * passes, hd_sync waits for both.  With 3, every hd_run_dedisp runs on the second
 * stream behind the stage 1 issued before it, and stage 1 waits only for the last stage-2
 * passes of the plans it rewrites: the next DDplan stage's stage 1 overlaps this stage's
 * stage 2.  Per-plan device times (hd_plan_last_ms) then include the time a kernel shared
 * the GPU with others.                                                                  */
HD_API int         hd_set_streams(hd_ctx* ctx, int32_t n);
/* Declare the raw block changed outside the library (e.g. written in place through a device
 * pointer): derived layouts (the channel-major copy the 8-bit stage-1 fill reads, built once
 * per raw block inside the first stage-1 launch) are rebuilt by the next stage-1 launch.  */
HD_API int         hd_touch_raw(hd_ctx* ctx);

/* Observation + switches.  The device raw block (N * nchan * nbits/8 bytes) is allocated
 * on the first hd_push_raw / hd_synth_device. */
HD_API int hd_set_obs(hd_ctx* ctx, const hd_obs* obs, const hd_opts* opts);
/* Per-raw-channel DAT_SCL / DAT_OFFS / DAT_WTS (file channel order); NULL = identity.
 * Value = ((raw * scl) + offs) * wts, as PSRFITS defines.                         */
HD_API int hd_set_chan_calib(hd_ctx* ctx, const float* scl, const float* offs, const float* wts);
/* rfifind mask (reference :482-490 makes it, stage 1 reads it with -mask) as PRESTO's
 * read_mask leaves it: mask[numint][nchan] = the interval's channel list (1 = listed,
 * ascending-frequency channels), zapint[numint] = 1 for intervals in zap_ints (NULL: a row
 * listing every channel counts as one), dtint = seconds per interval as stored in the file
 * (<= 0: ptsperint * dt).  Applied per raw read block (obs nsblk spectra) with check_mask's
 * rule [PRESTO-ext]: the union of the lists of the block's first and last interval, or
 * every channel when either is a zap_int.  padvals[nchan] = initial pad values (rfifind
 * .stats, hd_stats_padvals; NULL = 0); with clipping on, clip_times replaces them block by
 * block with its running channel levels.  mask == NULL clears the mask.                */
HD_API int hd_set_mask(hd_ctx* ctx, const uint8_t* mask, int32_t numint, int32_t ptsperint,
                       double dtint, const uint8_t* zapint, const float* padvals);
/* determine_padvals [PRESTO-ext]: pad values from an rfifind .stats file's interval
 * averages dataavg[numint][numchan] -- per channel, the avg_var mean of the middle 80 % of
 * its sorted interval averages.  Host-only.                                            */
HD_API int hd_stats_padvals(const float* dataavg, int32_t numint, int32_t numchan, float* padvals);
/* Cleaning state of the current raw block (computed by the next stage-1 launch, or now):
 * pad[nblk][nchan] pad values in force per read block, clipped[N] (1 = spectrum replaced
 * by clip_times), zap[nblk][nchan] zapped channels per block; any may be NULL.  *nclipped
 * receives the number of clipped spectra (may be NULL).  nblk = ceil(N / nsblk).        */
HD_API int hd_get_clean(hd_ctx* ctx, float* pad, uint8_t* clipped, uint8_t* zap, int64_t* nclipped);
/* Copy nspectra raw spectra (file layout, rows of nchan*nbits/8 bytes) to device
 * spectra [start, start + nspectra).  Host memory may be pageable or pinned.       */
HD_API int hd_push_raw(hd_ctx* ctx, const void* spectra, int64_t start, int64_t nspectra);
/* Streaming PSRFITS ingest (north_star (b); replaces the whole-file read PRESTO's
 * prepsubband does through psrfits.c before the loops of
 * lib/python/PALFA2_presto_search.py:506-511).  Reads the DATA column of rows
 * [row0, row0 + nrows) of one SUBINT binary table straight from the file into two pinned
 * host buffers in turn (pread), each handed to the device with hipMemcpyAsync on the
 * context's stream, so the disk read of block k+1 overlaps the PCIe copy of block k.
 * The DATA column must hold whole spectra (npol 1: col_bytes = nsblk*nchan*nbits/8);
 * spectra land at device spectra [start, ...).  Optional stats: seconds spent in pread,
 * seconds for the whole call (both may be NULL).                                      */
typedef struct {
    int64_t table_offset;   /* byte offset of the table's first row in the file          */
    int64_t row_bytes;      /* NAXIS1                                                      */
    int64_t col_offset;     /* byte offset of the DATA column inside a row                 */
    int64_t col_bytes;      /* DATA bytes per row                                          */
    int64_t row0, nrows;    /* rows to read                                                */
    int64_t block_bytes;    /* pinned block size (0: 32 MiB; at least one row)             */
} hd_rows_src;
HD_API int hd_push_raw_file(hd_ctx* ctx, const char* path, const hd_rows_src* src, int64_t start,
                            double* io_seconds, double* total_seconds);
/* Mock ingest in-stream (replaces `combine_mocks <s0> <s1> -o <base>` + `fitsdelrow
 * <base>_0001.fits[SUBINT] 1 7`, lib/python/datafile.py:494-508): rows of one band's file
 * whose spectra are spec_bytes long; bytes [src_offset, src_offset + nbytes) of each land at
 * bytes [dst_offset, dst_offset + nbytes) of device spectrum start + k (the merged row), so
 * the two halves fill their channel ranges of one raw block with no merged file written.
 * src->row0 = 7 skips the rows fitsdelrow deletes.                                        */
HD_API int hd_push_raw_file_band(hd_ctx* ctx, const char* path, const hd_rows_src* src, int64_t start,
                                 int64_t spec_bytes, int64_t src_offset, int64_t dst_offset, int64_t nbytes,
                                 double* io_seconds, double* total_seconds);
/* Spectra [start, start + count) of the raw block set to byte_value in every byte: the
 * padding between PSRFITS files that start later than the previous one ends
 * (lib/python/formats/psrfits.py:272-280).                                                */
HD_API int hd_fill_raw(hd_ctx* ctx, int64_t start, int64_t count, int32_t byte_value);
/* Overlapped ingest of the next beam (BASELINE configs[4]: the 7 beams of an ALFA pointing,
 * one beam per job as queue_managers/pbs.py:67 runs them): hd_prefetch_raw_file / _band /
 * hd_prefetch_fill queue the work of hd_push_raw_file / _band / hd_fill_raw for the NEXT
 * beam into the context's second raw slot and return at once -- a reader thread preads into
 * pinned blocks of its own and copies on a stream of its own while the current beam computes.
 * hd_swap_raw waits for the queued reads (not for compute), orders the context's streams after
 * their copies and makes the prefetched block current; the previous block becomes the next
 * prefetch target, reused only after the work already queued on it.  Same hd_set_obs for both
 * beams (a new hd_set_obs drops the prefetch).  *io_seconds: pread time, *total_seconds:
 * first queued job to the swap.  HD_E_STATE when nothing was prefetched; a read or copy error
 * of any queued job is returned here.                                                      */
HD_API int hd_prefetch_raw_file(hd_ctx* ctx, const char* path, const hd_rows_src* src, int64_t start);
HD_API int hd_prefetch_raw_file_band(hd_ctx* ctx, const char* path, const hd_rows_src* src, int64_t start,
                                     int64_t spec_bytes, int64_t src_offset, int64_t dst_offset, int64_t nbytes);
HD_API int hd_prefetch_fill(hd_ctx* ctx, int64_t start, int64_t count, int32_t byte_value);
HD_API int hd_swap_raw(hd_ctx* ctx, double* io_seconds, double* total_seconds);
/* Fill the device raw block with the synthetic beam (bit-identical to hd_synth_host). */
HD_API int hd_synth_device(hd_ctx* ctx, const hd_synth* s);
/* Host generator: spectra [start, start+count) of the same beam into out (file layout).
 * Needs only the observation geometry; usable without a GPU.                        */
HD_API int hd_synth_host(const hd_obs* obs, const hd_synth* s, int64_t start, int64_t count,
                  void* out);

/* Copy device spectra [start, start+count) back to host (file layout). */
HD_API int hd_get_raw(hd_ctx* ctx, void* out, int64_t start, int64_t count);
/* Multi-GPU (hipdedisp.sharding): raw spectra already in device memory of the context's
 * GPU -- e.g. a block another rank broadcast over RCCL -- in / out, device-to-device.      */
HD_API int hd_push_raw_device(hd_ctx* ctx, const void* dev_spectra, int64_t start, int64_t nspectra);
HD_API int hd_get_raw_device(hd_ctx* ctx, void* dev_out, int64_t start, int64_t count);
/* Multi-GPU time slices (hipdedisp.sharding.TimeSlices): the context (after hd_set_obs with
 * obs.N = the slice's spectra) holds spectra [t0, t0 + N) of an observation of n_total
 * spectra; t0 is a multiple of nsblk.  Read blocks and mask intervals count from the
 * observation's start and hd_synth_device generates the observation's spectra t0.. .
 * (0, 0) returns to a whole observation.  Clears the mask-block and clip state.           */
HD_API int hd_set_slice(hd_ctx* ctx, int64_t t0, int64_t n_total);
/* clip_times across slices: its running statistics carry from block to block over the
 * whole observation, so every slice contributes the per-block statistics of the read
 * blocks it owns and every slice then runs the recurrence over all blocks before its end.
 * Layout of `stats` (host or device memory of this context's GPU; the observation's
 * ceil(n_total / nsblk) rows of nchan + 3 doubles: bavg, bstd, numgood, chansum[nchan]):
 * hd_clip_stats writes the rows of this slice's first nown blocks (global rows t0/nsblk ..)
 * and leaves the others alone, so a zero-filled buffer summed over the slices (an all-reduce)
 * is complete; hd_clip_set_stats reads rows [0, t0/nsblk + nblk) and finishes clip_times
 * for this slice (no-ops when clipping is off).                                            */
HD_API int hd_clip_stats(hd_ctx* ctx, int64_t nown, double* stats);
HD_API int hd_clip_set_stats(hd_ctx* ctx, const double* stats);

/* ---- passes --------------------------------------------------------------------- */
/* Host-only: the integer tables and subband-level parameters a plan would use, without
 * a device (chan_delays[nchan], dm_offsets[numdms*nsub]; any output may be NULL).     */
HD_API int hd_plan_tables(const hd_obs* obs, const hd_opts* opts, const hd_pass* pass,
                   int32_t* chan_delays, int32_t* dm_offsets,
                   double* sub_lofreq, double* sub_chanwid, double* sub_dt);
/* Host-only extent check of the stage-2 kernels that copy global memory into LDS in whole
 * 1 KiB DMA pieces (k_stage2_ring, k_stage2_pair, k_stage2_rw, k_stage2_qp): for each such
 * kernel the plan would build and each buffer it copies from, `reach` = bytes from the
 * buffer's start to the end of the furthest piece any workgroup issues (derived from the
 * same tile, window and piece counts the kernels use) and `size` = the bytes hd_plan_create
 * allocates.  hd_plan_create fails with HD_E_INVAL when any reach exceeds its size, and
 * sizes each offset table's zero tail from this reach (no fixed slack).  out[cap] receives
 * the records, *n their count (HD_E_NOMEM when more than cap; out may be NULL with cap 0 to
 * count).  kernel = the hd_plan_set_variant stage-2 number (5 ring, 6 / 7 pair with 1 / 2
 * pairs per chunk, 8 register windows, 9 quarter-layout pairs); ppc = the pairs per chunk
 * the offsets table serves (k_stage2_qp keeps one table per 4, 3, 2).                     */
#define HD_EXT_SUBBANDS 0     /* the int16 subband block [nsub][sub_stride]            */
#define HD_EXT_OFFSETS  1     /* the per-chunk LDS offset table                        */
typedef struct {
    int32_t kernel;
    int32_t region;      /* HD_EXT_*                                                     */
    int32_t ppc;
    int32_t _pad0;
    int64_t reach;       /* bytes, exclusive                                             */
    int64_t size;        /* bytes allocated                                              */
} hd_extent;
HD_API int hd_plan_extents(const hd_obs* obs, const hd_opts* opts, const hd_pass* pass,
                           hd_extent* out, int32_t cap, int32_t* n);
HD_API int hd_plan_create(hd_ctx* ctx, const hd_pass* pass, hd_plan** out);
HD_API int hd_plan_destroy(hd_plan* plan);
/* Integer delay tables: chan_delays[nchan] (stage-1 idispdt, samples at dt) and
 * dm_offsets[numdms*nsub] (stage-2 offsets, samples at dt*ds).  Either may be NULL. */
HD_API int hd_plan_get_delays(const hd_plan* plan, int32_t* chan_delays, int32_t* dm_offsets);
/* Subband-level parameters as written to (and read back from) the .sub.inf file.   */
HD_API int hd_plan_sub_params(const hd_plan* plan, double* sub_lofreq, double* sub_chanwid,
                       double* sub_dt, int64_t* nds);
/* Stage 1: raw (+calib, mask) -> nsub subbands of N/ds samples, kept on device.     */
HD_API int hd_run_subband(hd_plan* plan);
/* Stage 1 for several passes of one DDplan stage (same nsub and ds, same context) with a
 * single read of the raw block per 32 passes.  Device time of each launch is attributed to
 * the first plan of its group of 32 (hd_plan_last_ms of the others reports 0).        */
HD_API int hd_run_subband_multi(hd_plan** plans, int32_t n);
/* Subbands device <-> host, layout [nsub][N/ds] of int16 or f32 (opts.sub_dtype).   */
HD_API int hd_get_subbands(hd_plan* plan, void* host);
/* Samples [t0, t0+count) of every subband, host layout [nsub][count] (t0+count <= N/ds). */
HD_API int hd_get_subbands_window(hd_plan* plan, int64_t t0, int64_t count, void* host);
HD_API int hd_set_subbands(hd_plan* plan, const void* host);
/* Stage 2: subbands -> numdms series of numout f32 samples.  host_out [numdms][numout]
 * receives them when non-NULL; otherwise they stay resident on the device.          */
HD_API int hd_run_dedisp(hd_plan* plan, float* host_out);
/* Stage 2 of several passes (the reference's per-pass prepsubband calls of one DDplan stage,
 * PALFA2_presto_search.py:512-529), series left on the device: passes that take the pair
 * kernel with the same geometry (one DDplan stage) share ONE launch of up to 28 passes, so the
 * tail of one pass's persistent workgroups overlaps the next pass instead of idling the GPU;
 * any other plan runs as hd_run_dedisp(plan, NULL).  Results are identical to per-plan runs.
 * Device time of a shared launch is attributed to its first plan (hd_plan_last_ms of the
 * others reports 0; hd_plan_launch_passes tells which plan led how many passes).        */
HD_API int hd_run_dedisp_multi(hd_plan* const* plans, int32_t n);
/* Passes carried by the last stage-2 launch this plan led: 1 for hd_run_dedisp, n for the
 * first plan of a shared launch, 0 for a plan whose stage 2 ran inside another's.         */
HD_API int hd_plan_launch_passes(const hd_plan* plan, int32_t* npass);
/* Samples [t0, t0+count) of DMs [dm0, dm0+ndm) of the device-resident series of the last
 * hd_run_dedisp, host layout [ndm][count] (t0+count <= numout).                        */
HD_API int hd_get_series(hd_plan* plan, int32_t dm0, int32_t ndm, int64_t t0, int64_t count, float* host);
/* Exact (double) sum of the device series samples [t0, t0+count) of DM dm (int16 subbands:
 * integer-valued samples, so the order of the sum does not matter), and a fill of samples
 * [t0, numout) of every DM with value -- the padding of a time-sliced pass, whose value
 * (prepsubband's first-DM mean) is the observation's, not the slice's.                 */
HD_API int hd_series_sum(hd_plan* plan, int32_t dm, int64_t t0, int64_t count, double* sum);
/* hd_series_sum of n plans (one context) at once: sums[i] = the sum over samples
 * [t0[i], t0[i]+count[i]) of DM dm of plans[i] -- the same doubles, one device wait.     */
HD_API int hd_series_sum_multi(hd_plan* const* plans, int32_t n, int32_t dm, const int64_t* t0, const int64_t* count,
                               double* sums);
HD_API int hd_series_fill(hd_plan* plan, int64_t t0, float value);

/* ---- in-library collectives (RCCL over xGMI) for a time-sliced beam -------------------
 * The two exchanges of hipdedisp.sharding.TimeSlices without torch.distributed, for a caller
 * of the C ABI (librccl is loaded at run time on first use).  Rank 0 makes the 128-byte id,
 * the caller hands it to every rank by any means (MPI, a file, a socket), every rank calls
 * hd_comm_init with its own context (collective).  hd_slice_exchange_clip replaces the
 * hd_clip_stats -> all-reduce -> hd_clip_set_stats sequence (nown = this slice's own read
 * blocks, nblk_total = the beam's); hd_comm_allreduce_sum_f64 sums n doubles in place over
 * the ranks (host or device memory) -- the padding sums of hd_series_sum_multi.           */
HD_API int hd_comm_unique_id(uint8_t* id);
HD_API int hd_comm_init(hd_ctx* ctx, const uint8_t* id, int32_t rank, int32_t world);
HD_API int hd_comm_allreduce_sum_f64(hd_ctx* ctx, double* buf, int64_t n);
HD_API int hd_slice_exchange_clip(hd_ctx* ctx, int64_t nown, int64_t nblk_total);
HD_API int hd_comm_destroy(hd_ctx* ctx);

/* ---- barycentric output (prepsubband without -nobary) ---------------------------------
 * The reference's stage-2 command passes no -nobary (PALFA2_presto_search.py:514-520), so
 * PRESTO resamples every DM series to the solar-system barycentre [PRESTO-ext]: from a TEMPO
 * table of topocentric times topo[n] and their barycentric times bary[n] (MJD, spaced tdt
 * seconds -- what presto.barycenter returns, the call the reference makes in get_baryv,
 * :43-57) it lists the output bins where one bin is added (value > 0: a padding sample
 * before topocentric sample v) or removed (value < 0: topocentric sample -v dropped), in
 * units of the output sample time dsdt.  hd_bary_diffbins restates that list (host only,
 * no device); *ndiff receives the count (HD_E_INVAL when it exceeds cap, diffbins holding the
 * first cap).  hd_plan_set_bary makes the plan's stage 2 write the barycentred series
 * (numout samples; added bins and the tail take the plan's padding value, hd_opts.pad_mode);
 * ndiff = 0 (or diffbins NULL) turns it off.  Not for time-sliced plans (HD_E_INVAL).
 * Setting the list the plan already holds returns at once (no wait on queued work).
 * hd_plan_data_end: the samples of real data at the head of the output -- min(N/ds, numout),
 * or, barycentred, where the last data segment ends (prepsubband's datawrote after the
 * added and removed bins): the .inf on/off pair is [0, n-1], [numout-1, numout-1] when
 * n < numout, and hd_single_pulse's border-case prune uses the same boundary.            */
HD_API int hd_bary_diffbins(const double* topo, const double* bary, int32_t n, double tdt, double dsdt,
                            int32_t* diffbins, int32_t cap, int32_t* ndiff);
HD_API int hd_plan_set_bary(hd_plan* plan, const int32_t* diffbins, int32_t ndiff);
HD_API int hd_plan_data_end(const hd_plan* plan, int64_t* n);
/* The .dat output path (replaces the files prepsubband leaves in the tempdir,
 * PALFA2_presto_search.py:514-520, 532-537): queue the device-resident series of the last
 * hd_run_dedisp of this plan to paths[numdms] -- raw little-endian float32, numout samples,
 * no header.  Chunks are copied device->host into pinned buffers on a copy stream ordered
 * after the plan's stage 2 (so later kernels keep running) and written by a pool of writer
 * threads.  wait = 0 returns once everything is queued; wait = 1 also waits for the files.
 * A later hd_run_dedisp of the plan is ordered after its queued copies.                */
HD_API int hd_write_series(hd_plan* plan, const char* const* paths, int32_t wait);
/* Wait for every queued write of the context; *write_seconds / *bytes (may be NULL): the
 * writer threads' cumulative busy seconds and bytes written since hd_open.  Returns the
 * first I/O error of the writes (HD_E_IO) if any.                                       */
HD_API int hd_wait_writes(hd_ctx* ctx, double* write_seconds, int64_t* bytes);
/* Device-time of the last hd_run_subband / hd_run_dedisp of this plan, ms.  A multi-pass
 * call (hd_run_subband_multi / hd_run_dedisp_multi) charges its whole launch to its first
 * plan; the other plans it carried report 0 for that stage (one event pair per launch).  */
HD_API int hd_plan_last_ms(const hd_plan* plan, float* ms_subband, float* ms_dedisp);
/* Name of the stage-2 kernel the last hd_run_dedisp of this plan launched, as rocprofv3
 * prints it without namespace and arguments (e.g. "k_stage2_qp<5, 3, 4, true, false>": every
 * template argument: for the pair kernels the non-negative-subband flag, then the profiling
 * build flag, false unless probe bits are set): lets a benchmark key its roofline and PMC
 * counters by kernel.  NUL-terminated in name[cap].   */
HD_API int hd_plan_kernel(const hd_plan* plan, char* name, int32_t cap);
/* Kernel variants: (s1 << 8) | s2.  s2: 0 auto, 1 direct, 2 LDS-tiled (4 waves x 256 samples),
 * 3 wide LDS tiles (up to 16 waves share one window), 4 two workgroups per CU, 5 LDS-DMA
 * ring, 6 ring over subband-pair partials (the auto choice when 2*max|subband| <= 32767 is
 * known on the host: 8/4-bit data without calibration, or uploaded int16 subbands; forcing
 * it otherwise fails in hd_run_dedisp with HD_E_INVAL); s1: 0 auto, 1 direct
 * (one thread per subband sample, for cross-checks), 2 float tiled multi-pass, 3 8-bit
 * integer tiled multi-pass (8-bit data without calibration only; HD_E_INVAL otherwise).
 * Bits 16-23 are profiling probes that skip parts of the tiled kernels (results are then
 * invalid; never set them in production): 1 skip the sums, 2 skip the LDS fill, 4 skip
 * the stage-2 stores, 8 skip the stage-2 expand, 32 skip the stage-1 fixup's block-boundary
 * items, 64 skip its clipped-spectrum items; 128 (valid results, for cross-checks) runs the
 * fixup with the generic per-cell kernel instead of the 8-bit LDS-window one; 16 (valid
 * results) keeps k_stage1_q8 at one summing wave per subband (its spare waves idle).  Bits 24-25 schedule the pair kernel's
 * tiles: 0 or 1 persistent workgroups (one per CU, each over a contiguous tile range; the
 * default), 2 one workgroup per tile.  s2 = 7: the pair kernel with two subband pairs per
 * chunk (half the chunks per tile; HD_E_INVAL when its LDS does not fit). */
HD_API int hd_plan_set_variant(hd_plan* plan, int32_t variant);

/* ---- rfifind statistics -------------------------------------------------------------
 * The numeric part of `rfifind -time T -o <base> <files>` (lib/python/PALFA2_presto_search.py:
 * 482-490) on the raw block in HBM [PRESTO-ext]: for every whole interval of ptsperint spectra
 * and every channel (ascending frequency), the samples as rfifind reads them (clip_times per
 * hd_opts, no mask -- call before hd_set_mask), their mean and standard deviation (variance
 * over n - 1) and the largest power of the interval's real FFT over bins 1 .. ptsperint/2 - 1
 * normalised by ptsperint * variance.  Outputs float [N / ptsperint][nchan].  The mask and
 * .stats files are made from these by hipdedisp/rfifind.py.                                */
HD_API int hd_rfifind_stats(hd_ctx* ctx, int32_t ptsperint, float* dataavg, float* datastd, float* datapow);

/* ---- single-pulse search on the device-resident series -------------------------------
 * Replaces the per-.dat `single_pulse_search.py -p -m maxwidth -t threshold <dat>` of
 * lib/python/PALFA2_presto_search.py:539-546 (maxwidth 0.1 s, threshold 5.0:
 * lib/python/config/searching_example.py:13-15) for the numout-sample series of a
 * plan's last hd_run_dedisp: per 1000-sample block a linear detrend and a trimmed std,
 * per DM the bad blocks, then every boxcar value above threshold is a hit.  The
 * candidate pruning of the script (prune_related1/2, border cases) runs on the hits in
 * hipdedisp/single_pulse.py.                                                              */
typedef struct {
    int32_t dm;        /* DM index in the plan                                         */
    int32_t bin;       /* sample                                                       */
    int32_t widx;      /* index into the widths of hd_sp_widths (0: width 1)            */
    int32_t pad;
    double sigma;      /* boxcar value of the normalised series (the candidate's sigma) */
} hd_sp_hit;
/* Boxcar widths the script searches: 1, then 2,3,4,6,9,14,20,30,45,70,100,150,220,300
 * while width * dt <= maxwidth.  widths[16]; *n = count.                              */
HD_API int hd_sp_widths(double dt, double maxwidth, int32_t* widths, int32_t* n);
/* The script's candidates of the plan's series into hits[cap], sorted by (dm, bin, widx):
 * device hits above threshold outside bad blocks, prune_related1 per width (a stronger hit
 * of that width within width/2 bins removes it; equal: the later one stays), then on the
 * host prune_related2 across widths and, for padded series, prune_border_cases.  *nhits =
 * the count; when the device hits exceed cap nothing is copied, *nhits is that number and
 * HD_E_NOMEM is returned (call again with room).  bad_blocks[numdms * nblocks] (may be
 * NULL): 1 = block not searched; *nblocks (may be NULL) = floor(numout / 1000).  A series
 * of fewer than 8000 samples gives no candidates.                                        */
HD_API int hd_single_pulse(hd_plan* plan, double dt, double maxwidth, double threshold, hd_sp_hit* hits,
                           int64_t cap, int64_t* nhits, uint8_t* bad_blocks, int64_t* nblocks);
/* hd_single_pulse in two halves, so the device search of later plans runs while the host
 * prunes this one's hits: _launch queues the device half on the plan's stream (its series
 * must stay unchanged until the collect) and returns; _collect waits for that plan's device
 * half only (copies on a context stream of their own) and then behaves as hd_single_pulse,
 * HD_E_NOMEM included (the search stays collectable: call again with room).  A launch again
 * before the collect replaces the pending search.  hd_single_pulse = _launch + _collect.   */
HD_API int hd_single_pulse_launch(hd_plan* plan, double dt, double maxwidth, double threshold);
HD_API int hd_single_pulse_collect(hd_plan* plan, hd_sp_hit* hits, int64_t cap, int64_t* nhits, uint8_t* bad_blocks,
                                   int64_t* nblocks);
/* The host half of hd_single_pulse on caller-supplied hits (any order, n of them, DMs
 * 0..ndm-1, widths[nw] of hd_sp_widths): grouped by DM, each DM's list in bin order (widths
 * ascending among equal bins), prune_related2 and -- when numout > nds -- the border cases
 * of single_pulse_search.py; the kept hits are compacted to the front, *nkept of them.
 * Host only (no device).                                                                  */
HD_API int hd_sp_prune(hd_sp_hit* hits, int64_t n, int32_t ndm, const int32_t* widths, int32_t nw, int64_t nds,
                       int64_t numout, int64_t* nkept);

/* ---- realfft, zapbirds, rednoise on the device-resident series -----------------------
 * Replace `realfft <dat>; zapbirds -zap -zapfile <zaplist> -baryv <v> <fft>; rednoise <fft>`
 * per .dat (lib/python/PALFA2_presto_search.py:548-558) [PRESTO-ext, restated; parity with
 * PRESTO unpinned].  The spectra stay in HBM with the plan ([numdms][numout/2] complex,
 * PRESTO's packed .fft layout: bin 0 = (DC, Nyquist)); hd_get_fft copies them out.       */
/* Forward real FFT (no normalisation) of the numout samples of every DM series (after
 * hd_run_dedisp; numout even).  The hipFFT plan and spectra buffer belong to the context,
 * one per series geometry (numout, numdms, stride), so consecutive passes of a DDplan stage
 * reuse them: a later hd_realfft of another plan of the same geometry takes the buffer over,
 * and hd_zapbirds / hd_rednoise / hd_get_fft of the earlier plan then fail with HD_E_STATE. */
HD_API int hd_realfft(hd_plan* plan);
/* Build the hipFFT plan and spectra buffer of this plan's geometry now (no transform; the
 * plan need not have run): rocFFT compiles its kernels for a new size, seconds per geometry,
 * which a caller moves off its timed path by preparing each DDplan stage's geometry once.  */
HD_API int hd_fft_prepare(hd_plan* plan);
/* Bin ranges [lo, hi) zapped for birdies lobins[i] .. hibins[i] (frequency * T, the
 * zaplist's freq -+ width/2): lo = floor(lobin), hi = ceil(hibin), clamped to
 * [1, numbins), empty ones dropped, sorted and merged where they overlap or touch; the
 * median window [wlo, lo) u [hi, whi) spans side = min(max(50, hi - lo), 2048) bins either
 * side (clamped).  rng4[4 * k] = {lo, hi, wlo, whi}; cap = room in ranges; *nr = count
 * (HD_E_NOMEM when more than cap).  Host only.                                           */
HD_API int hd_zap_ranges(const double* lobins, const double* hibins, int32_t nbirds, int64_t numbins,
                         int32_t* rng4, int32_t cap, int32_t* nr);
/* zapbirds -zap: every merged range's bins set to (sqrt(median / ln 2), 0), the median
 * (element (n-1)/2 of the sorted powers) over its window in the un-zapped spectrum.        */
HD_API int hd_zapbirds(hd_plan* plan, const double* lobins, const double* hibins, int32_t nbirds);
/* rednoise's blocks over bins 1 .. numbins - 1: from o = 1, width w(f) = startwidth +
 * floor((endwidth - startwidth) * ln(1 + f) / ln(1 + endfreq)) at f = o / T Hz below
 * endfreq, endwidth from there (the last block cut at numbins).  boff[nblk + 1] offsets
 * (cap = room for offsets), *nblk = count; endwidth <= 128.  Host only.                   */
HD_API int hd_rednoise_blocks(int64_t numbins, double T, int32_t startwidth, int32_t endwidth, double endfreq,
                              int32_t* boff, int32_t cap, int32_t* nblk);
/* rednoise: each block's median power m_j (lower median); bin i scaled by 1/sqrt(m(i)/ln 2),
 * m linear between the block centres o_j + (w_j - 1)/2 (flat outside them; m <= 0 gives 0);
 * bin 0 = (1, 0).  T = numout * dt of the series (s); PRESTO's defaults are 6, 100, 6.0.  */
HD_API int hd_rednoise(hd_plan* plan, int32_t startwidth, int32_t endwidth, double endfreq, double T);
/* Spectra of DM series dm0 .. dm0 + ndm - 1: out[ndm][numout] floats (numout/2 complex).  */
HD_API int hd_get_fft(hd_plan* plan, int32_t dm0, int32_t ndm, float* out);

#ifdef __cplusplus
}
#endif
#endif /* HIPDEDISP_H */
