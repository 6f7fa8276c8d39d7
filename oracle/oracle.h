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
 *   (2) analytic known-answer tests (impulses, constants) in tests/test_oracle.py;
 *   (3) an independent numpy restatement (oracle/oracle_np.py) that must agree bit for bit.
 * Against PRESTO itself it is "parity unpinned"; each PRESTO-derived rule below is
 * tagged [PRESTO-ext] and has a switch in or_opts.
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
    int32_t sub_dtype;        /* 0 int16, 1 f32              */
    int32_t ds_mode;          /* 0 sum, 1 mean               */
    int32_t pad_mode;         /* 0 mean, 1 zero              */
    int32_t nibble_hi_first;
    int32_t be16;
    int32_t inf_roundtrip;
    float   clip_sigma;
    int32_t _pad0;
} or_opts;

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

/* ---- stage 1: raw -> subbands, output samples [t0, t0+count) of every subband ----
 * out: [nsub][out_stride] int16 or f32 (opts->sub_dtype); column index = t - t0.
 * scl/offs/wts: per raw channel or NULL; mask [numint][nchan] or NULL; padvals or NULL. */
int or_stage1(const or_obs* obs, const or_opts* opts, const uint8_t* raw,
              const float* scl, const float* offs, const float* wts,
              const uint8_t* mask, int numint, int ptsperint, const float* padvals,
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

/* Whole pass, full length: convenience for tests. */
int or_run_pass(const or_obs* obs, const or_opts* opts, const uint8_t* raw,
                const float* scl, const float* offs, const float* wts,
                const uint8_t* mask, int numint, int ptsperint, const float* padvals,
                double subdm, double lodm, double dmstep, int numdms, int nsub, int ds,
                int64_t numout, void* sub_out /* [nsub][N/ds] or NULL */,
                float* dat_out /* [numdms][numout] */);

int or_num_threads(void);

#ifdef __cplusplus
}
#endif
#endif
