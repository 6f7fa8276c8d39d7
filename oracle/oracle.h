/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of PRESTO prepsubband's
 * two-stage arithmetic, used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker.  The product (libhipdedisp.so) never links it.
 *
 * PARITY STATUS: the arithmetic lives in PRESTO (github.com/scottransom/presto, no
 * pinned version; reference README:13-15), which is absent from /root/reference and
 * from this image.  The reference holds no tests or fixtures that pin prepsubband's
 * numbers.  This oracle is therefore pinned by
 *   (1) the reference's own plan code, run to produce tests/golden/ddplan_ref.json;
 *   (2) analytic known-answer tests (impulses, constants, clipping) in tests/test_oracle.py;
 *   (3) an independent numpy restatement (oracle/oracle_np.py) that must agree bit for bit.
 * Against PRESTO itself it is "parity unpinned"; each PRESTO-derived rule below is
 * tagged [PRESTO-ext], names the PRESTO function it restates from memory, and has a
 * switch in or_opts where PRESTO versions are known to differ.
 *
 * Per-block model (PRESTO reads raw data one PSRFITS subint = nsblk spectra at a time,
 * backend_common.c read_psrdata [PRESTO-ext]).  For raw block b:
 *   1. decode (unpack, DAT_SCL/OFFS/WTS, band flip) -> X[t][c], ascending frequency;
 *   2. check_mask(b*nsblk*dt, nsblk*dt) -> zapped channel set of the block, or ALL when
 *      the block touches an interval in zap_ints (mask.c check_mask: the union of the
 *      block's first and last interval only);
 *   3. if clip_sigma > 0 and the block is not ALL-zapped: clip_times(X, ..., padvals)
 *      (clipping.c): zero-DM series, block median, "good" spectra within 0.7..1.3 x median,
 *      their mean/std (avg_var, AS 52) and per-channel means, 30-block running averages;
 *      spectra with |zdm - running_avg| > clip_sigma * running_std are replaced by the
 *      running channel averages, which also become the pad values (good_chan_levels);
 *   4. zapped channels of the block := padvals (as updated by step 3).
 * Spectra past N read as the last block's pad values.
 */
#ifndef HD_ORACLE_H
#define HD_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int32_t nchan, nbits, npol, flip;
    double  dt, lofreq, df;
    int64_t N;
    int32_t nsblk, _pad0;
    double  voverc;
} or_obs;   /* same field meaning as hd_obs (include/hipdedisp.h) */

typedef struct {
    int32_t sub_dtype;        /* 0 int16, 1 f32                                        */
    int32_t ds_mode;          /* 0 sum, 1 mean (prepsubband get_data: ftmp / downsamp)  */
    int32_t pad_mode;         /* 0 per-DM mean, 1 zero, 2 first-DM running mean (PRESTO) */
    int32_t nibble_hi_first;
    int32_t be16;
    int32_t inf_roundtrip;
    float   clip_sigma;       /* 0: -noclip                                             */
    int32_t sub_round;        /* 0 PRESTO (short)(x + 0.5) (x86 cvttsd2si, low 16 bits);
                                 1 nearest, ties away, saturated                       */
} or_opts;

/* rfifind mask as PRESTO's read_mask leaves it [PRESTO-ext, mask.c] */
typedef struct {
    const uint8_t* chans;     /* [numint][nchan], 1 = channel in the interval's list     */
    const uint8_t* zapint;    /* [numint], 1 = interval in zap_ints; NULL: a row listing
                                 every channel counts as a zap_int                       */
    int32_t numint, ptsperint;
    double  dtint;            /* seconds per interval as stored; <= 0: ptsperint * dt    */
} or_mask;

/* ---- PRESTO src/dispersion.c restated [PRESTO-ext] ---- */
double  or_delay_from_dm(double dm, double freq_emitted);
double  or_doppler(double freq_observed, double voverc);
int64_t or_nearest_long(double x);
void    or_dedisp_delays(int numchan, double dm, double lofreq, double chanwidth,
                         double voverc, double* delays);
void    or_subband_delays(int numchan, int numsubbands, double dm, double lofreq,
                          double chanwidth, double voverc, double* delays);
void    or_subband_search_delays(int numchan, int numsubbands, double dm, double lofreq,
                                 double chanwidth, double voverc, double* delays);

/* ---- integer tables ---- */
void or_chan_delays(const or_obs* obs, int nsub, double subdm, int32_t* idispdt);
void or_sub_params(const or_obs* obs, const or_opts* opts, int nsub, int ds,
                   double* sub_lofreq, double* sub_chanwid, double* sub_dt);
void or_dm_offsets(const or_obs* obs, const or_opts* opts, int nsub, int ds,
                   double lodm, double dmstep, int numdms, int32_t* off);
/* offsets from subband-level (lofreq, chanwidth, dt) as read from a .sub.inf */
void or_dm_offsets_sub(int nsub, double lof, double bw, double dsdt, double voverc,
                       double lodm, double dmstep, int numdms, int32_t* off);

/* ---- per-block cleaning (steps 2-4 above) ----
 * blocks of blk spectra, nblk = ceil(N / blk).
 * or_check_mask_blocks: zap[nblk][nchan] and allzap[nblk] from the mask (mask.c check_mask).
 * or_clip_prepare: pad[nblk][nchan] = pad values in force for block b (after its clip),
 *   clipped[N] = 1 for spectra clip_times replaced; returns the number clipped, or -1.
 *   padvals0 = initial pad values (determine_padvals; NULL = 0). */
void    or_check_mask_blocks(const or_obs* obs, const or_mask* mask, int blk, int nblk,
                             uint8_t* zap, uint8_t* allzap);
int64_t or_clip_prepare(const or_obs* obs, const or_opts* opts, const uint8_t* raw,
                        const float* scl, const float* offs, const float* wts,
                        const uint8_t* allzap, const float* padvals0, int blk, int nblk,
                        float* pad, uint8_t* clipped);
/* The same clip_times split at a time slice's exchange (hd_clip_stats / hd_clip_set_stats):
 * or_clip_rows writes the rows {avg, std, numgood, chansum[nchan]} of global read blocks
 * [b0, b0 + nrows) from raw = spectra b0*blk.. of the observation (obs->N its full length);
 * or_clip_finish runs the recurrence over the summed table of all nblk rows and flags the
 * spectra [t0, t0 + n) that raw holds.  or_clip_prepare == rows over all blocks + finish. */
int     or_clip_rows(const or_obs* obs, const or_opts* opts, const uint8_t* raw, const float* scl,
                     const float* offs, const float* wts, const uint8_t* allzap, int blk, int64_t b0,
                     int64_t nrows, double* rows);
int64_t or_clip_finish(const or_obs* obs, const or_opts* opts, const uint8_t* raw, const float* scl,
                       const float* offs, const float* wts, const uint8_t* allzap, const float* padvals0,
                       int blk, int nblk, const double* table, int64_t t0, int64_t n, float* pad,
                       uint8_t* clipped);

/* ---- stage 1: raw -> subbands, output samples [t0, t0+count) of every subband ----
 * out: [nsub][out_stride] int16 or f32 (opts->sub_dtype); column index = t - t0.
 * scl/offs/wts: per raw channel or NULL.  Cleaning: zap [nblk][nchan] or NULL,
 * pad [nblk][nchan] or NULL (0), clipped [N] or NULL; blocks of blk spectra. */
int or_stage1(const or_obs* obs, const or_opts* opts, const uint8_t* raw,
              const float* scl, const float* offs, const float* wts,
              const uint8_t* zap, const float* pad, const uint8_t* clipped, int blk, int nblk,
              int nsub, int ds, const int32_t* idispdt,
              int64_t t0, int64_t count, void* out, int64_t out_stride);

/* ---- stage 2: subbands -> DM series, samples [t0, t0+count) ----
 * sub: [nsub][sub_stride] with nds valid samples; reads past nds are 0.
 * out: [numdms][out_stride] f32; column index = t - t0.  Padding is not applied here. */
int or_stage2(const void* sub, int sub_dtype, int64_t nds, int64_t sub_stride, int nsub,
              const int32_t* off, int numdms, int64_t t0, int64_t count,
              float* out, int64_t out_stride);

/* Padding of full series [numdms][numout] whose first nds samples are data. */
void or_pad(float* out, int numdms, int64_t nds, int64_t numout, int pad_mode);

/* determine_padvals [PRESTO-ext, mask.c]: per channel, the mean (avg_var) of the middle
 * 80 % of its sorted interval averages from rfifind's .stats (dataavg [numint][numchan]). */
void or_stats_padvals(const float* dataavg, int numint, int numchan, float* padvals);

int or_num_threads(void);

#ifdef __cplusplus
}
#endif
#endif
