/*
 * prepsubband_oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h for the parity status and
 * the per-block model).
 *
 * A plain-C restatement of what PRESTO `prepsubband` computes for the two calls that
 * PALFA2_presto_search.search_job() makes per DDplan pass
 * (reference lib/python/PALFA2_presto_search.py:506-520).  It is the checker for the
 * HIP engine and, built with OpenMP, the CPU baseline timed by bench.py.  It is never
 * linked into libhipdedisp.so.
 *
 * Data flow (mirrors PRESTO's block pipeline: raw block -> float block -> mask / clip ->
 * subbands -> downsample -> .subNN int16; then .subNN -> per-DM float sums):
 *   stage 1  sub[s][t'] = Q( D( sum_{k<ds} ( sum_{c in s} X'(t'*ds + k + idispdt[c], c) ) ) )
 *            X'(t, c) = pad[b][c] if spectrum t was clipped or (b, c) is zapped, else
 *                       ((raw * scl) + offs) * wts (channel c ascending); b = t / blk;
 *                       t >= N reads pad[nblk-1][c]
 *            D        = / ds (mean, prepsubband get_data) or identity (sum)
 *            Q        = (short)(x + 0.5) as x86 evaluates it, or nearest-saturated (sub_round)
 *   stage 2  out[d][t] = sum_{s=0}^{nsub-1} sub[s][t + off[d][s]]   (sub past N/ds = 0)
 *            then pad [N/ds, numout) (first-DM running mean, per-DM mean or 0).
 * Every float sum is accumulated in float32 in ascending channel / subband / k order,
 * starting from 0.0f, with FP contraction disabled (Makefile: -ffp-contract=off).
 */
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------- */
/* PRESTO src/dispersion.c, restated [PRESTO-ext]                                   */
/* ------------------------------------------------------------------------------- */

/* delay in seconds for DM (pc cm^-3) at emitted frequency (MHz) */
double or_delay_from_dm(double dm, double freq_emitted)
{
    return dm / (0.000241 * freq_emitted * freq_emitted);
}

/* emitted frequency for an observer moving with radial velocity voverc */
double or_doppler(double freq_observed, double voverc)
{
    return freq_observed * (1.0 + voverc);
}

/* PRESTO NEAREST_LONG: (long)(x < 0 ? ceil(x - 0.5) : floor(x + 0.5)) */
int64_t or_nearest_long(double x)
{
    return (int64_t)(x < 0 ? ceil(x - 0.5) : floor(x + 0.5));
}

void or_dedisp_delays(int numchan, double dm, double lofreq, double chanwidth,
                      double voverc, double* delays)
{
    for (int ii = 0; ii < numchan; ii++)
        delays[ii] = or_delay_from_dm(dm, or_doppler(lofreq + ii * chanwidth, voverc));
}

/* delays of each subband's highest channel */
void or_subband_delays(int numchan, int numsubbands, double dm, double lofreq,
                       double chanwidth, double voverc, double* delays)
{
    int chan_per_subband = numchan / numsubbands;
    double subbandwidth = chanwidth * chan_per_subband;
    double losubhifreq = lofreq + subbandwidth - chanwidth;
    or_dedisp_delays(numsubbands, dm, losubhifreq, subbandwidth, voverc, delays);
}

/* per-channel delays relative to the top channel of the channel's subband */
void or_subband_search_delays(int numchan, int numsubbands, double dm, double lofreq,
                              double chanwidth, double voverc, double* delays)
{
    int cps = numchan / numsubbands;
    double* sub = (double*)malloc(sizeof(double) * numsubbands);
    or_dedisp_delays(numchan, dm, lofreq, chanwidth, voverc, delays);
    or_subband_delays(numchan, numsubbands, dm, lofreq, chanwidth, voverc, sub);
    for (int ii = 0, jj = 0; ii < numsubbands; ii++)
        for (int kk = 0; kk < cps; kk++, jj++) delays[jj] -= sub[ii];
    free(sub);
}

/* ------------------------------------------------------------------------------- */
/* integer tables                                                                   */
/* ------------------------------------------------------------------------------- */

/* stage-1 idispdt: NEAREST_LONG(subband_search_delays(subdm) / dt) */
void or_chan_delays(const or_obs* obs, int nsub, double subdm, int32_t* idispdt)
{
    double* d = (double*)malloc(sizeof(double) * obs->nchan);
    or_subband_search_delays(obs->nchan, nsub, subdm, obs->lofreq, obs->df, obs->voverc, d);
    for (int c = 0; c < obs->nchan; c++) idispdt[c] = (int32_t)or_nearest_long(d[c] / obs->dt);
    free(d);
}

static double roundtrip(double v, const char* fmt)
{
    char buf[64];
    snprintf(buf, sizeof buf, fmt, v);
    return strtod(buf, NULL);
}

/* Subband-level lofreq / channel width / dt that stage 2 reads from the .sub.inf.
 * lofreq = top channel of the lowest subband (where stage 1 aligned it) [PRESTO-ext]. */
void or_sub_params(const or_obs* obs, const or_opts* opts, int nsub, int ds,
                   double* sub_lofreq, double* sub_chanwid, double* sub_dt)
{
    int cps = obs->nchan / nsub;
    double subbw = obs->df * cps;
    double lof = obs->lofreq + subbw - obs->df;
    double dt = obs->dt * ds;
    if (opts->inf_roundtrip) {
        lof = roundtrip(lof, "%.12g");
        subbw = roundtrip(subbw, "%.12g");
        dt = roundtrip(dt, "%.15g");
    }
    *sub_lofreq = lof;
    *sub_chanwid = subbw;
    *sub_dt = dt;
}

/* stage-2 offsets: NEAREST_LONG((subband_delays(DM_d)[s] - [nsub-1]) / dsdt), with the
 * .sub.inf treated as an nsub-channel observation (PRESTO reads it that way). */
void or_dm_offsets_sub(int nsub, double lof, double bw, double dsdt, double voverc,
                       double lodm, double dmstep, int numdms, int32_t* off)
{
    double* d = (double*)malloc(sizeof(double) * nsub);
    for (int ii = 0; ii < numdms; ii++) {
        double dm = lodm + ii * dmstep;
        or_subband_delays(nsub, nsub, dm, lof, bw, voverc, d);
        double top = d[nsub - 1];
        for (int s = 0; s < nsub; s++)
            off[(int64_t)ii * nsub + s] = (int32_t)or_nearest_long((d[s] - top) / dsdt);
    }
    free(d);
}

void or_dm_offsets(const or_obs* obs, const or_opts* opts, int nsub, int ds,
                   double lodm, double dmstep, int numdms, int32_t* off)
{
    double lof, bw, dsdt;
    or_sub_params(obs, opts, nsub, ds, &lof, &bw, &dsdt);
    or_dm_offsets_sub(nsub, lof, bw, dsdt, obs->voverc, lodm, dmstep, numdms, off);
}

/* ------------------------------------------------------------------------------- */
/* raw decode                                                                       */
/* ------------------------------------------------------------------------------- */

static inline float raw_sample(const or_obs* o, const or_opts* op, const uint8_t* row, int rc)
{
    switch (o->nbits) {
    case 8:
        return (float)row[rc];
    case 4: {
        uint8_t b = row[rc >> 1];
        int first = ((rc & 1) == 0);
        int hi = op->nibble_hi_first ? first : !first;
        return (float)(hi ? (b >> 4) : (b & 15));
    }
    case 16: {
        const uint8_t* p = row + 2 * rc;
        uint16_t u = op->be16 ? (uint16_t)((p[0] << 8) | p[1]) : (uint16_t)((p[1] << 8) | p[0]);
        return (float)(int16_t)u;
    }
    default:
        return 0.0f;
    }
}

/* one raw spectrum -> decoded, calibrated f[nchan] in ascending-frequency order */
static void decode_row(const or_obs* o, const or_opts* op, const uint8_t* row,
                       const float* scl, const float* offs, const float* wts, float* f)
{
    const int n = o->nchan;
    if (o->nbits == 8) {
        if (o->flip) for (int c = 0; c < n; c++) f[c] = (float)row[n - 1 - c];
        else for (int c = 0; c < n; c++) f[c] = (float)row[c];
    } else {
        for (int c = 0; c < n; c++) f[c] = raw_sample(o, op, row, o->flip ? n - 1 - c : c);
    }
    if (scl || offs || wts)
        for (int c = 0; c < n; c++) {
            const int rc = o->flip ? n - 1 - c : c;
            float x = f[c];
            if (scl) x = x * scl[rc];
            if (offs) x = x + offs[rc];
            if (wts) x = x * wts[rc];
            f[c] = x;
        }
}

/* ------------------------------------------------------------------------------- */
/* rfifind mask per read block [PRESTO-ext, mask.c check_mask]                      */
/* ------------------------------------------------------------------------------- */

void or_check_mask_blocks(const or_obs* obs, const or_mask* m, int blk, int nblk,
                          uint8_t* zap, uint8_t* allzap)
{
    const int nchan = obs->nchan;
    memset(zap, 0, (size_t)nblk * nchan);
    memset(allzap, 0, (size_t)nblk);
    if (!m || !m->chans || m->numint <= 0) return;
    const double dtint = m->dtint > 0 ? m->dtint : m->ptsperint * obs->dt;
    const double duration = blk * obs->dt;               /* time_per_subint */
    for (int b = 0; b < nblk; b++) {
        const double starttime = (double)((int64_t)b * blk) * obs->dt;
        const double endtime = starttime + duration;
        int lo = (int)(starttime / dtint), hi = (int)(endtime / dtint);
        /* PRESTO indexes the interval tables with these; past the last interval they are
         * clamped here (rfifind's numint = ceil(N / ptsperint) makes hi == numint only
         * for the final block) */
        if (lo > m->numint - 1) lo = m->numint - 1;
        if (hi > m->numint - 1) hi = m->numint - 1;
        int all = 0;
        for (int k = 0; k < 2 && !all; k++) {
            const int iv = k ? hi : lo;
            const uint8_t* row = m->chans + (int64_t)iv * nchan;
            if (m->zapint) {
                all = m->zapint[iv] != 0;
            } else {
                int n = 0;
                for (int c = 0; c < nchan; c++) n += row[c] != 0;
                all = n == nchan;
            }
        }
        if (all) {
            allzap[b] = 1;
            memset(zap + (int64_t)b * nchan, 1, (size_t)nchan);
            continue;
        }
        for (int c = 0; c < nchan; c++)
            zap[(int64_t)b * nchan + c] = (m->chans[(int64_t)lo * nchan + c] | m->chans[(int64_t)hi * nchan + c]) != 0;
    }
}

/* ------------------------------------------------------------------------------- */
/* clip_times and its statistics helpers [PRESTO-ext, clipping.c / misc]           */
/* ------------------------------------------------------------------------------- */

/* Devillard's quick_select (Numerical Recipes 8.5), as PRESTO's median(): the element of
 * rank (n - 1) / 2 of arr (arr is permuted). */
static float quick_select(float* arr, int n)
{
    int low = 0, high = n - 1, median = (low + high) / 2, middle, ll, hh;
    float t;
#define SWAPF(a, b) { t = (a); (a) = (b); (b) = t; }
    for (;;) {
        if (high <= low) return arr[median];
        if (high == low + 1) {
            if (arr[low] > arr[high]) SWAPF(arr[low], arr[high]);
            return arr[median];
        }
        middle = (low + high) / 2;
        if (arr[middle] > arr[high]) SWAPF(arr[middle], arr[high]);
        if (arr[low] > arr[high]) SWAPF(arr[low], arr[high]);
        if (arr[middle] > arr[low]) SWAPF(arr[middle], arr[low]);
        SWAPF(arr[middle], arr[low + 1]);
        ll = low + 1;
        hh = high;
        for (;;) {
            do ll++; while (arr[low] > arr[ll]);
            do hh--; while (arr[hh] > arr[low]);
            if (hh < ll) break;
            SWAPF(arr[ll], arr[hh]);
        }
        SWAPF(arr[low], arr[hh]);
        if (hh <= median) low = ll;
        if (hh >= median) high = hh - 1;
    }
#undef SWAPF
}

/* avg_var: mean and (n-1)-normalised variance of a float vector, AS 52 one-pass update */
static void avg_var(const float* x, int n, double* mean, double* var)
{
    double an = 0.0, an1 = 0.0, dx;
    *mean = (double)x[0];
    *var = 0.0;
    for (int i = 1; i < n; i++) {
        an = (double)(i + 1);
        an1 = (double)i;
        dx = ((double)x[i] - *mean) / an;
        *var += an * an1 * dx * dx;
        *mean += dx;
    }
    if (n > 1) *var /= an1;
}

#define BLOCKSTOAVG 30

typedef struct {
    float running_avg, running_std;
    int blocksread;
    float* chan_running_avg;
} clipstate;

/* clip_times(rawdata [ptsperblk][numchan], ..., good_chan_levels), split in two so the
 * oracle can run the per-block statistics of many blocks in parallel (OpenMP) and only the
 * running-average recurrence in block order; the arithmetic is PRESTO's, step for step.
 *
 * Part 1 (no state): the zero-DM series, its median, the "good" points within 0.7..1.3 x
 * the median, their avg_var mean and std and the per-channel sums of the good spectra. */
typedef struct {
    int numgood;
    double avg, std;
} blockstat;

static void clip_block_stats(const float* rawdata, int ptsperblk, int numchan, float* zero_dm_block,
                             blockstat* bs, double* chan_avg_temp)
{
    float* median_temp = (float*)malloc(sizeof(float) * ptsperblk);
    for (int ii = 0; ii < ptsperblk; ii++) {
        zero_dm_block[ii] = 0.0f;
        for (int jj = 0; jj < numchan; jj++) zero_dm_block[ii] += rawdata[(int64_t)ii * numchan + jj];
        median_temp[ii] = zero_dm_block[ii];
    }
    const float current_med = quick_select(median_temp, ptsperblk);
    const float lo_cutoff = 0.7 * current_med;
    const float hi_cutoff = 1.3 * current_med;
    int numgoodpts = 0;
    for (int jj = 0; jj < numchan; jj++) chan_avg_temp[jj] = 0.0;
    for (int ii = 0; ii < ptsperblk; ii++) {
        if (zero_dm_block[ii] > lo_cutoff && zero_dm_block[ii] < hi_cutoff) {
            median_temp[numgoodpts] = zero_dm_block[ii];
            for (int jj = 0; jj < numchan; jj++) chan_avg_temp[jj] += rawdata[(int64_t)ii * numchan + jj];
            numgoodpts++;
        }
    }
    bs->numgood = numgoodpts;
    bs->avg = bs->std = 0.0;
    if (numgoodpts >= 1) {
        double var;
        avg_var(median_temp, numgoodpts, &bs->avg, &var);
        bs->std = sqrt(var);
    }
    /* chan_avg_temp keeps the SUMS here: the exchange rows of a time-sliced beam carry them,
     * and clip_finish divides by numgood exactly where clip_times does */
    free(median_temp);
}

/* Part 2 (block order): the BLOCKSTOAVG-block running averages, good_chan_levels, and the
 * spectra beyond clip_sigma * running_std flagged for replacement by the channel levels. */
static int clip_update(const float* zero_dm_block, int ptsperblk, int numchan, float clip_sigma,
                       const blockstat* bs, const double* chan_avg_block, float* good_chan_levels,
                       clipstate* st, uint8_t* flags)
{
    double current_avg, current_std;
    const double* chan_avg_temp = chan_avg_block;
    double* fallback = NULL;
    if (bs->numgood < 1) {
        current_avg = st->running_avg;
        current_std = st->running_std;
        fallback = (double*)malloc(sizeof(double) * numchan);
        for (int jj = 0; jj < numchan; jj++) fallback[jj] = st->chan_running_avg[jj];
        chan_avg_temp = fallback;
    } else {
        current_avg = bs->avg;
        current_std = bs->std;
    }
    if (st->blocksread) {
        st->running_avg = (st->running_avg * (BLOCKSTOAVG - 1) + current_avg) / BLOCKSTOAVG;
        st->running_std = (st->running_std * (BLOCKSTOAVG - 1) + current_std) / BLOCKSTOAVG;
        for (int ii = 0; ii < numchan; ii++)
            st->chan_running_avg[ii] = (st->chan_running_avg[ii] * (BLOCKSTOAVG - 1) + chan_avg_temp[ii]) / BLOCKSTOAVG;
    } else {
        st->running_avg = current_avg;
        st->running_std = current_std;
        for (int ii = 0; ii < numchan; ii++) st->chan_running_avg[ii] = chan_avg_temp[ii];
    }
    for (int ii = 0; ii < numchan; ii++) good_chan_levels[ii] = st->chan_running_avg[ii];
    const float trigger = clip_sigma * st->running_std;
    int clipped = 0;
    for (int ii = 0; ii < ptsperblk; ii++)
        if (fabs(zero_dm_block[ii] - st->running_avg) > trigger) {
            flags[ii] = 1;      /* clip_times replaces the spectrum by chan_running_avg */
            clipped++;
        }
    st->blocksread++;
    free(fallback);
    return clipped;
}

static void zero_dm(const float* rawdata, int ptsperblk, int numchan, float* zero_dm_block)
{
    for (int ii = 0; ii < ptsperblk; ii++) {
        zero_dm_block[ii] = 0.0f;
        for (int jj = 0; jj < numchan; jj++) zero_dm_block[ii] += rawdata[(int64_t)ii * numchan + jj];
    }
}

/* Exchange rows of clip_times' per-block statistics (the layout of hd_clip_stats): for the
 * global read blocks [b0, b0 + nrows), row r = {avg, std, numgood, chansum[nchan]} (zeros for
 * a block whose every channel is masked).  raw holds the observation's spectra from
 * t0 = b0 * blk on (a time slice's own rows); obs->N is the whole observation's length.   */
/* The rows, and (zdm_out != NULL) each block's zero-DM series into zdm_out[(b - b0) * blk + i]
 * from the same decode: the whole-beam path keeps it, so every block is decoded once, as
 * prepsubband's read loop does. */
static int clip_rows_z(const or_obs* obs, const or_opts* opts, const uint8_t* raw, const float* scl,
                       const float* offs, const float* wts, const uint8_t* allzap, int blk, int64_t b0,
                       int64_t nrows, double* rows, float* zdm_out)
{
    const int nchan = obs->nchan;
    const int64_t nblk = (obs->N + blk - 1) / blk;
    if (blk <= 0 || b0 < 0 || nrows < 0 || b0 + nrows > nblk) return -1;
    memset(rows, 0, sizeof(double) * (size_t)nrows * (nchan + 3));
    const int64_t rowbytes = (int64_t)nchan * obs->nbits / 8;
#pragma omp parallel
    {
        float* X = (float*)malloc(sizeof(float) * (size_t)blk * nchan);
        float* zdm = (float*)malloc(sizeof(float) * (size_t)blk);
#pragma omp for schedule(dynamic, 1)
        for (int64_t r = 0; r < nrows; r++) {
            const int64_t b = b0 + r;
            if (allzap && allzap[b]) continue;
            const int64_t t0 = b * blk;
            const int nb = (int)((t0 + blk <= obs->N) ? blk : obs->N - t0);
            for (int ii = 0; ii < nb; ii++)
                decode_row(obs, opts, raw + (t0 - b0 * blk + ii) * rowbytes, scl, offs, wts, X + (int64_t)ii * nchan);
            blockstat bs;
            double* row = rows + r * (nchan + 3);
            clip_block_stats(X, nb, nchan, zdm, &bs, row + 3);
            row[0] = bs.avg;
            row[1] = bs.std;
            row[2] = (double)bs.numgood;
            if (zdm_out) memcpy(zdm_out + r * blk, zdm, sizeof(float) * (size_t)nb);
        }
        free(zdm);
        free(X);
    }
    return 0;
}

int or_clip_rows(const or_obs* obs, const or_opts* opts, const uint8_t* raw, const float* scl, const float* offs,
                 const float* wts, const uint8_t* allzap, int blk, int64_t b0, int64_t nrows, double* rows)
{
    return clip_rows_z(obs, opts, raw, scl, offs, wts, allzap, blk, b0, nrows, rows, NULL);
}

/* clip_times' block-order recurrence over the exchange rows table[nblk][nchan + 3] of the
 * whole observation: pad[nblk][nchan] (the channel levels in force per block) and the
 * clipped flags of spectra [t0, t0 + n) of raw (which holds those spectra; t0 a multiple of
 * blk).  Returns the number of clipped spectra among them.                                */
/* zdm_all != NULL: the zero-DM series of spectra [t0, t0 + n) already computed (the rows'
 * decode); else each of those blocks is decoded here (a time slice's restatement). */
static int64_t clip_finish_z(const or_obs* obs, const or_opts* opts, const uint8_t* raw, const float* scl,
                             const float* offs, const float* wts, const uint8_t* allzap, const float* padvals0,
                             int blk, int nblk, const double* table, int64_t t0, int64_t n, float* pad,
                             uint8_t* clipped, const float* zdm_all)
{
    const int nchan = obs->nchan;
    if (blk <= 0 || nblk != (int)((obs->N + blk - 1) / blk) || t0 % blk || t0 < 0 || t0 + n > obs->N) return -1;
    memset(clipped, 0, (size_t)n);
    float* padvals = (float*)calloc((size_t)nchan, sizeof(float));
    if (padvals0) memcpy(padvals, padvals0, sizeof(float) * nchan);
    const int clip = opts->clip_sigma > 0.0f;
    const int64_t rowbytes = (int64_t)nchan * obs->nbits / 8;
    float* X = zdm_all ? NULL : (float*)malloc(sizeof(float) * (size_t)blk * nchan);
    float* zdm = (float*)malloc(sizeof(float) * (size_t)blk);
    uint8_t* scratch = (uint8_t*)malloc((size_t)blk);
    double* cat = (double*)malloc(sizeof(double) * nchan);
    clipstate st = {0.0f, 0.0f, 0, (float*)calloc((size_t)nchan, sizeof(float))};
    int64_t total = 0;
    for (int b = 0; b < nblk; b++) {
        const int64_t s0 = (int64_t)b * blk;
        const int nb = (int)((s0 + blk <= obs->N) ? blk : obs->N - s0);
        const int mine = s0 >= t0 && s0 < t0 + n;
        if (clip && !(allzap && allzap[b])) {
            const double* row = table + (int64_t)b * (nchan + 3);
            blockstat bs = {(int)row[2], row[0], row[1]};
            for (int jj = 0; jj < nchan; jj++) cat[jj] = bs.numgood >= 1 ? row[3 + jj] / bs.numgood : row[3 + jj];
            uint8_t* flags = scratch;
            const float* z = zdm;
            memset(scratch, 0, (size_t)blk);
            if (mine) {
                if (zdm_all) {
                    z = zdm_all + (s0 - t0);
                } else {
                    for (int ii = 0; ii < nb; ii++)
                        decode_row(obs, opts, raw + (s0 - t0 + ii) * rowbytes, scl, offs, wts, X + (int64_t)ii * nchan);
                    zero_dm(X, nb, nchan, zdm);
                }
                flags = clipped + (s0 - t0);
            } else {
                for (int ii = 0; ii < nb; ii++) zdm[ii] = st.running_avg;   /* flags of other slices: unused */
            }
            const int k = clip_update(z, nb, nchan, opts->clip_sigma, &bs, cat, padvals, &st, flags);
            if (mine) total += k;
        }
        memcpy(pad + (int64_t)b * nchan, padvals, sizeof(float) * nchan);
    }
    free(st.chan_running_avg);
    free(cat);
    free(scratch);
    free(zdm);
    free(X);
    free(padvals);
    return total;
}

int64_t or_clip_finish(const or_obs* obs, const or_opts* opts, const uint8_t* raw, const float* scl,
                       const float* offs, const float* wts, const uint8_t* allzap, const float* padvals0, int blk,
                       int nblk, const double* table, int64_t t0, int64_t n, float* pad, uint8_t* clipped)
{
    return clip_finish_z(obs, opts, raw, scl, offs, wts, allzap, padvals0, blk, nblk, table, t0, n, pad, clipped,
                         NULL);
}

int64_t or_clip_prepare(const or_obs* obs, const or_opts* opts, const uint8_t* raw,
                        const float* scl, const float* offs, const float* wts,
                        const uint8_t* allzap, const float* padvals0, int blk, int nblk,
                        float* pad, uint8_t* clipped)
{
    /* the reference's -sub command leaves prepsubband's default clip on; a block whose
     * every channel is masked is neither clipped nor counted (read_psrdata).  The whole beam:
     * one decode per block (the rows' pass keeps the zero-DM series for the recurrence). */
    if (blk <= 0 || nblk != (int)((obs->N + blk - 1) / blk)) return -1;
    double* table = NULL;
    float* zdm = NULL;
    if (opts->clip_sigma > 0.0f) {
        table = (double*)malloc(sizeof(double) * (size_t)nblk * (obs->nchan + 3));
        zdm = (float*)malloc(sizeof(float) * (size_t)nblk * blk);
        clip_rows_z(obs, opts, raw, scl, offs, wts, allzap, blk, 0, nblk, table, zdm);
    }
    const int64_t total = clip_finish_z(obs, opts, raw, scl, offs, wts, allzap, padvals0, blk, nblk, table, 0,
                                        obs->N, pad, clipped, zdm);
    free(zdm);
    free(table);
    return total;
}

/* ------------------------------------------------------------------------------- */
/* stage 1                                                                          */
/* ------------------------------------------------------------------------------- */

/* prepsubband writes subbands as `subsdata[jj][ii] = (short)(infloat + 0.5)` [PRESTO-ext]:
 * double x + 0.5 truncated to int32 (cvttsd2si; out of range -> 0x80000000), low 16 bits. */
static inline int16_t presto_short(float x)
{
    const double y = (double)x + 0.5;
    int32_t i = (y > -2147483649.0 && y < 2147483648.0) ? (int32_t)y : INT32_MIN;
    return (int16_t)(uint16_t)(uint32_t)i;
}

static inline int16_t nearest_i16(float x)
{
    int64_t v = or_nearest_long((double)x);
    if (v > 32767) v = 32767;
    if (v < -32768) v = -32768;
    return (int16_t)v;
}

int or_stage1(const or_obs* obs, const or_opts* opts, const uint8_t* raw,
              const float* scl, const float* offs, const float* wts,
              const uint8_t* zap, const float* pad, const uint8_t* clipped, int blk, int nblk,
              int nsub, int ds, const int32_t* idispdt,
              int64_t t0, int64_t count, void* out, int64_t out_stride)
{
    const int nchan = obs->nchan;
    if (nsub <= 0 || nchan % nsub || ds <= 0 || obs->npol != 1) return -1;
    if ((zap || pad || clipped) && (blk <= 0 || nblk != (int)((obs->N + blk - 1) / blk))) return -1;
    const int cps = nchan / nsub;
    int maxd = 0;
    for (int c = 0; c < nchan; c++) if (idispdt[c] > maxd) maxd = idispdt[c];
    const int64_t bo = ds >= 8192 ? 1 : 8192 / ds;            /* output samples per block */
    const int64_t nblocks = (count + bo - 1) / bo;

#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t b = 0; b < nblocks; b++) {
        const int64_t tb0 = t0 + b * bo;
        const int64_t nb = (tb0 + bo <= t0 + count) ? bo : (t0 + count - tb0);
        const int64_t nr = nb * ds + maxd;
        float* fb = (float*)malloc(sizeof(float) * nr * nchan);
        /* raw -> cleaned float block (ascending-frequency channels), like read_psrdata */
        for (int64_t r = 0; r < nr; r++) {
            const int64_t t = tb0 * ds + r;
            float* f = fb + r * nchan;
            int64_t rb = blk > 0 ? t / blk : 0;
            if (rb > nblk - 1) rb = nblk - 1;
            const float* prow = pad ? pad + rb * nchan : NULL;
            if (t >= obs->N || (clipped && clipped[t])) {
                for (int c = 0; c < nchan; c++) f[c] = prow ? prow[c] : 0.0f;
                continue;
            }
            const uint8_t* zrow = zap ? zap + rb * nchan : NULL;
            decode_row(obs, opts, raw + t * ((int64_t)nchan * obs->nbits / 8), scl, offs, wts, f);
            if (zrow)
                for (int c = 0; c < nchan; c++)
                    if (zrow[c]) f[c] = prow ? prow[c] : 0.0f;
        }
        /* channel -> subband delay-and-sum at subdm (dedisp_subbands), then downsample */
        for (int64_t j = 0; j < nb; j++) {
            for (int s = 0; s < nsub; s++) {
                float acc = 0.0f;
                for (int k = 0; k < ds; k++) {
                    float sk = 0.0f;
                    for (int cc = 0; cc < cps; cc++) {
                        const int c = s * cps + cc;
                        sk += fb[(j * ds + k + idispdt[c]) * nchan + c];
                    }
                    acc += sk;
                }
                if (opts->ds_mode == 1) acc = acc / (float)ds;
                const int64_t col = tb0 + j - t0;
                if (opts->sub_dtype == 0)
                    ((int16_t*)out)[(int64_t)s * out_stride + col] =
                        opts->sub_round == 0 ? presto_short(acc) : nearest_i16(acc);
                else
                    ((float*)out)[(int64_t)s * out_stride + col] = acc;
            }
        }
        free(fb);
    }
    return 0;
}

/* ------------------------------------------------------------------------------- */
/* stage 2                                                                          */
/* ------------------------------------------------------------------------------- */

int or_stage2(const void* sub, int sub_dtype, int64_t nds, int64_t sub_stride, int nsub,
              const int32_t* off, int numdms, int64_t t0, int64_t count,
              float* out, int64_t out_stride)
{
    if (count <= 0) return 0;
#pragma omp parallel for schedule(dynamic, 1)
    for (int d = 0; d < numdms; d++) {
        float* o = out + (int64_t)d * out_stride;
        for (int64_t t = 0; t < count; t++) o[t] = 0.0f;
        for (int s = 0; s < nsub; s++) {
            const int64_t base = t0 + off[(int64_t)d * nsub + s];   /* input index of o[0] */
            int64_t n = nds - base;                                   /* valid inputs        */
            if (n > count) n = count;
            if (n < 0) n = 0;
            if (sub_dtype == 0) {
                const int16_t* x = (const int16_t*)sub + (int64_t)s * sub_stride + base;
                for (int64_t t = 0; t < n; t++) o[t] += (float)x[t];
            } else {
                const float* x = (const float*)sub + (int64_t)s * sub_stride + base;
                for (int64_t t = 0; t < n; t++) o[t] += x[t];
            }
            for (int64_t t = n; t < count; t++) o[t] += 0.0f;   /* past the end: zeros */
        }
    }
    return 0;
}

/* prepsubband pads [N/ds, numout) with `avg`, the one-pass running mean (update_stats)
 * of the FIRST DM's written samples, for every DM [PRESTO-ext] (pad_mode 2); pad_mode 0 is
 * a per-DM mean (double sum), 1 zeros. */
void or_pad(float* out, int numdms, int64_t nds, int64_t numout, int pad_mode)
{
    if (numout <= nds) return;
    float v0 = 0.0f;
    if (pad_mode == 2 && nds > 0) {
        double avg = 0.0;
        for (int64_t n = 0; n < nds; n++) {
            const double x = out[n];
            const double dev = x - avg;
            avg += dev / (n + 1.0);
        }
        v0 = (float)avg;
    }
    for (int d = 0; d < numdms; d++) {
        float* o = out + (int64_t)d * numout;
        float v = v0;
        if (pad_mode == 0 && nds > 0) {
            double sum = 0.0;
            for (int64_t t = 0; t < nds; t++) sum += (double)o[t];
            v = (float)(sum / (double)nds);
        }
        for (int64_t t = nds; t < numout; t++) o[t] = v;
    }
}

/* ------------------------------------------------------------------------------- */
/* rfifind .stats -> pad values [PRESTO-ext, mask.c determine_padvals]              */
/* ------------------------------------------------------------------------------- */

static int cmp_float(const void* a, const void* b)
{
    const float x = *(const float*)a, y = *(const float*)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

/* calc_avgmedstd(arr, numarr, 0.8, step): mean of the middle `fraction` of the sorted
 * strided values (avg_var), returned as float */
void or_stats_padvals(const float* dataavg, int numint, int numchan, float* padvals)
{
    const float fraction = 0.8f;
    float* tmp = (float*)malloc(sizeof(float) * (numint > 0 ? numint : 1));
    for (int c = 0; c < numchan; c++) {
        const int len = (int)(numint * fraction + 0.5);
        const int start = (numint - len) / 2;
        for (int ii = 0; ii < numint; ii++) tmp[ii] = dataavg[(int64_t)ii * numchan + c];
        qsort(tmp, (size_t)numint, sizeof(float), cmp_float);
        double avg = 0.0, var = 0.0;
        if (len > 0) avg_var(tmp + start, len, &avg, &var);
        padvals[c] = (float)avg;
    }
    free(tmp);
}

int or_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
