/*
 * prepsubband_oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h for the parity status).
 *
 * A plain-C restatement of what PRESTO `prepsubband` computes for the two calls that
 * PALFA2_presto_search.search_job() makes per DDplan pass
 * (reference lib/python/PALFA2_presto_search.py:506-520).  It is the checker for the
 * HIP engine and, built with OpenMP, the CPU baseline timed by bench.py.  It is never
 * linked into libhipdedisp.so.
 *
 * Data flow (mirrors PRESTO's block pipeline: raw block -> float block -> subbands ->
 * downsample -> .subNN int16; then .subNN -> per-DM float sums):
 *   stage 1  sub[s][t'] = Q( sum_{k<ds} ( sum_{c in s} X(t'*ds + k + idispdt[c], c) ) )
 *            X(t, c)  = ((raw * scl) + offs) * wts   for channel c (ascending freq),
 *                       padvals[c] if (t / ptsperint, c) is zapped in the mask or t >= N
 *            Q        = nearest integer, ties away from zero, saturated to int16
 *                       (HD_SUB_I16), or identity (HD_SUB_F32); /ds first if ds_mode=mean
 *   stage 2  out[d][t] = sum_{s=0}^{nsub-1} sub[s][t + off[d][s]]   (sub past N/ds = 0)
 *            then pad [N/ds, numout) with the series mean (or 0).
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
/* stage 1                                                                          */
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

static inline int16_t quant_i16(float x)
{
    int64_t v = or_nearest_long((double)x);
    if (v > 32767) v = 32767;
    if (v < -32768) v = -32768;
    return (int16_t)v;
}

int or_stage1(const or_obs* obs, const or_opts* opts, const uint8_t* raw,
              const float* scl, const float* offs, const float* wts,
              const uint8_t* mask, int numint, int ptsperint, const float* padvals,
              int nsub, int ds, const int32_t* idispdt,
              int64_t t0, int64_t count, void* out, int64_t out_stride)
{
    const int nchan = obs->nchan;
    if (nsub <= 0 || nchan % nsub || ds <= 0 || obs->npol != 1) return -1;
    const int cps = nchan / nsub;
    const int64_t rowbytes = (int64_t)nchan * obs->nbits / 8;
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
        /* raw -> float block (ascending-frequency channels), like read_psrdata */
        for (int64_t r = 0; r < nr; r++) {
            const int64_t t = tb0 * ds + r;
            float* f = fb + r * nchan;
            if (t >= obs->N) {
                for (int c = 0; c < nchan; c++) f[c] = padvals ? padvals[c] : 0.0f;
                continue;
            }
            const uint8_t* row = raw + t * rowbytes;
            const uint8_t* mrow = NULL;
            if (mask && ptsperint > 0) {
                int64_t iv = t / ptsperint;
                if (iv < numint) mrow = mask + iv * nchan;
            }
            for (int c = 0; c < nchan; c++) {
                const int rc = obs->flip ? nchan - 1 - c : c;
                float x = raw_sample(obs, opts, row, rc);
                if (scl) x = x * scl[rc];
                if (offs) x = x + offs[rc];
                if (wts) x = x * wts[rc];
                if (mrow && mrow[c]) x = padvals ? padvals[c] : 0.0f;
                f[c] = x;
            }
        }
        /* channel -> subband delay-and-sum at subdm, then downsample */
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
                    ((int16_t*)out)[(int64_t)s * out_stride + col] = quant_i16(acc);
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

void or_pad(float* out, int numdms, int64_t nds, int64_t numout, int pad_mode)
{
    if (numout <= nds) return;
    for (int d = 0; d < numdms; d++) {
        float* o = out + (int64_t)d * numout;
        float v = 0.0f;
        if (pad_mode == 0 && nds > 0) {
            double sum = 0.0;
            for (int64_t t = 0; t < nds; t++) sum += (double)o[t];
            v = (float)(sum / (double)nds);
        }
        for (int64_t t = nds; t < numout; t++) o[t] = v;
    }
}

int or_run_pass(const or_obs* obs, const or_opts* opts, const uint8_t* raw,
                const float* scl, const float* offs, const float* wts,
                const uint8_t* mask, int numint, int ptsperint, const float* padvals,
                double subdm, double lodm, double dmstep, int numdms, int nsub, int ds,
                int64_t numout, void* sub_out, float* dat_out)
{
    const int64_t nds = obs->N / ds;
    if (numout <= 0) numout = nds;
    int32_t* idd = (int32_t*)malloc(sizeof(int32_t) * obs->nchan);
    int32_t* off = (int32_t*)malloc(sizeof(int32_t) * (size_t)numdms * nsub);
    const size_t esz = opts->sub_dtype == 0 ? 2 : 4;
    void* sub = sub_out ? sub_out : malloc(esz * (size_t)nsub * (size_t)(nds > 0 ? nds : 1));
    or_chan_delays(obs, nsub, subdm, idd);
    or_dm_offsets(obs, opts, nsub, ds, lodm, dmstep, numdms, off);
    int rc = or_stage1(obs, opts, raw, scl, offs, wts, mask, numint, ptsperint, padvals,
                       nsub, ds, idd, 0, nds, sub, nds);
    if (rc == 0) {
        const int64_t n = numout < nds ? numout : nds;
        rc = or_stage2(sub, opts->sub_dtype, nds, nds, nsub, off, numdms, 0, n, dat_out, numout);
        or_pad(dat_out, numdms, nds, numout, opts->pad_mode);
    }
    if (!sub_out) free(sub);
    free(idd);
    free(off);
    return rc;
}

int or_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
