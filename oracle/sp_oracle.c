/* sp_oracle.c — TEST INFRASTRUCTURE ONLY (never linked into the product): CPU restatement
 * of the numeric core of PRESTO's single_pulse_search.py [PRESTO-ext; parity with PRESTO
 * unpinned: the script is not in this image], as the reference runs it on every .dat
 * (lib/python/PALFA2_presto_search.py:539-546, -m 0.1 -t 5.0 from
 * lib/python/config/searching_example.py:13-15).
 *
 *   blocks of detrendlen = 1000 over roundN = floor(N/1000)*1000 samples:
 *     least-squares line removed, std = sqrt(sum of squares of the sorted middle 95 %
 *     / (0.95*1000)) * 1.148;
 *   per DM: sort the stds, locut/hicut at the largest jumps of the lower/upper halves,
 *     pseudo-median and population std of [locut, hicut), bad = outside +-4 std;
 *   normalised data (bad blocks 0) over the first numchunks*8000 samples (0 beyond);
 *   hits: every boxcar value (1/sqrt(w) kernel at PRESTO's offsets) above threshold;
 *   sp_prune_related1: the script's prune_related1 greedy walk, literally (quadratic; the
 *     device uses the O(n) form it reduces to).
 *
 * The summation orders are the ones hd_sp.hip defines (64 lane partials over the block's
 * samples 16l..16l+15, then a xor butterfly; per 8000-sample chunk a prefix over 256
 * segments of 33 window samples), so the GPU's doubles are reproduced exactly.
 * Build: oracle/Makefile (-ffp-contract=off).                                           */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SP_BLOCK 1000
#define SP_CHUNK 8000
#define SP_HALO 224
#define SP_SEG 33
#define SP_WIN (256 * SP_SEG)

typedef struct {
    int32_t dm, bin, widx, pad;
    double sigma;
} sp_hit;

static double butterfly(double* p)
{
    double q[64];
    for (int m = 32; m >= 1; m >>= 1) {
        for (int l = 0; l < 64; l++) q[l] = p[l] + p[l ^ m];
        memcpy(p, q, sizeof(q));
    }
    return p[0];
}

static int cmp_f(const void* a, const void* b)
{
    const float x = *(const float*)a, y = *(const float*)b;
    return x < y ? -1 : x > y ? 1 : 0;
}

static int cmp_d(const void* a, const void* b)
{
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y ? 1 : 0;
}

/* coef[(dm*nblocks + b)*4 + {mean, slope, std, bad}] for one series */
static void block_coefs(const float* x, int nblocks, double* coef)
{
    float v[1024];
    double p[64], p2[64];
    for (int b = 0; b < nblocks; b++) {
        const float* xb = x + (int64_t)b * SP_BLOCK;
        for (int l = 0; l < 64; l++) {
            double s = 0.0, st = 0.0;
            for (int r = 0; r < 16; r++) {
                const int i = 16 * l + r;
                if (i < SP_BLOCK) {
                    s += (double)xb[i];
                    st += ((double)i - 499.5) * (double)xb[i];
                }
            }
            p[l] = s;
            p2[l] = st;
        }
        const double mean = butterfly(p) / (double)SP_BLOCK;
        const double slope = butterfly(p2) / 83333250.0;
        for (int i = 0; i < SP_BLOCK; i++) v[i] = (float)((double)xb[i] - (mean + slope * ((double)i - 499.5)));
        qsort(v, SP_BLOCK, sizeof(float), cmp_f);
        for (int l = 0; l < 64; l++) {
            double q = 0.0;
            for (int r = 0; r < 16; r++) {
                const int i = 16 * l + r;
                if (i >= SP_BLOCK / 40 && i < SP_BLOCK - SP_BLOCK / 40) q += (double)v[i] * (double)v[i];
            }
            p[l] = q;
        }
        const double q = butterfly(p);
        double* cf = coef + (int64_t)b * 4;
        cf[0] = mean;
        cf[1] = slope;
        cf[2] = sqrt(q / (0.95 * SP_BLOCK)) * 1.148;
        cf[3] = 0.0;
    }
    if (nblocks < 2) return;
    /* bad blocks (Python 2 integer division as in the script) */
    double* srt = (double*)malloc(sizeof(double) * nblocks);
    for (int b = 0; b < nblocks; b++) srt[b] = coef[(int64_t)b * 4 + 2];
    qsort(srt, nblocks, sizeof(double), cmp_d);
    const int nb = nblocks, h = nb / 2;
    int locut = 1, am = 0;
    double best = -INFINITY;
    for (int i = 0; i < h; i++)
        if (srt[i + 1] - srt[i] > best) { best = srt[i + 1] - srt[i]; locut = i + 1; }
    best = -INFINITY;
    for (int i = h; i + 1 < nb; i++)
        if (srt[i + 1] - srt[i] > best) { best = srt[i + 1] - srt[i]; am = i - h; }
    const int hicut = am + h - 2;
    if (hicut > locut) {
        double m = 0.0, var = 0.0;
        for (int i = locut; i < hicut; i++) m += srt[i];
        m /= (double)(hicut - locut);
        for (int i = locut; i < hicut; i++) var += (srt[i] - m) * (srt[i] - m);
        const double sd = sqrt(var / (double)(hicut - locut));
        const double med = srt[(locut + hicut) / 2];
        const double lo = med - 4.0 * sd, hi = med + 4.0 * sd;
        for (int b = 0; b < nblocks; b++) {
            double* cf = coef + (int64_t)b * 4;
            if (cf[2] < lo || cf[2] > hi) {
                cf[2] = med;
                cf[3] = 1.0;
            }
        }
    }
    free(srt);
}

static float norm_at(const float* x, const double* coef, int64_t i, int64_t ls)
{
    if (i < 0 || i >= ls) return 0.0f;
    const int64_t b = i / SP_BLOCK;
    const double* c = coef + b * 4;
    if (c[3] != 0.0 || c[2] == 0.0) return 0.0f;
    const double t = (double)(i - b * SP_BLOCK) - 499.5;
    const float d = (float)((double)x[i] - (c[0] + c[1] * t));
    return (float)((double)d / c[2]);
}

/* Hits of ndm series x[dm*stride + t], t < n, unsorted into hits[cap]; returns the count
 * (hits past cap are counted, not stored).  bad[dm*nblocks + b] (may be NULL). */
int64_t sp_oracle_hits(const float* x, int64_t stride, int ndm, int64_t n, const int32_t* widths, int nwidths,
                       double threshold, sp_hit* hits, int64_t cap, uint8_t* bad)
{
    const int nblocks = (int)(n / SP_BLOCK);
    const int64_t ls = (int64_t)nblocks * SP_BLOCK / SP_CHUNK * SP_CHUNK;
    double rsw[16];
    for (int i = 0; i < nwidths; i++) rsw[i] = 1.0 / sqrt((double)widths[i]);
    double* coef = (double*)malloc(sizeof(double) * 4 * (nblocks > 0 ? nblocks : 1));
    double* P = (double*)malloc(sizeof(double) * (SP_WIN + 1));
    double tot[256];
    int64_t cnt = 0;
    for (int dm = 0; dm < ndm; dm++) {
        const float* xs = x + (int64_t)dm * stride;
        block_coefs(xs, nblocks, coef);
        if (bad)
            for (int b = 0; b < nblocks; b++) bad[(int64_t)dm * nblocks + b] = coef[(int64_t)b * 4 + 3] != 0.0;
        for (int64_t ch = 0; ch < ls / SP_CHUNK; ch++) {
            const int64_t w0 = ch * SP_CHUNK - SP_HALO;
            for (int t = 0; t < 256; t++) {
                double run = 0.0;
                for (int j = 0; j < SP_SEG; j++) {
                    run += (double)norm_at(xs, coef, w0 + t * SP_SEG + j, ls);
                    P[t * SP_SEG + j + 1] = run;              /* local prefix for now */
                }
                tot[t] = run;
            }
            double base = 0.0;
            for (int t = 0; t < 256; t++) {
                const double nb = base + tot[t];
                tot[t] = base;
                base = nb;
            }
            P[0] = 0.0;
            for (int t = 0; t < 256; t++)
                for (int j = 0; j < SP_SEG; j++) P[t * SP_SEG + j + 1] = tot[t] + P[t * SP_SEG + j + 1];
            for (int o = 0; o < SP_CHUNK; o++) {
                const int64_t i = ch * SP_CHUNK + o;
                const int k = o + SP_HALO;
                for (int wi = 0; wi < nwidths; wi++) {
                    const int w = widths[wi];
                    double s;
                    if (w == 1) {
                        s = (double)norm_at(xs, coef, i, ls);
                    } else {
                        const int lo = k - w / 2, hi = k + ((w & 1) ? w / 2 : w / 2 - 1) + 1;
                        s = (P[hi] - P[lo]) * rsw[wi];
                    }
                    if (s > threshold) {
                        if (cnt < cap) {
                            hits[cnt].dm = dm;
                            hits[cnt].bin = (int32_t)i;
                            hits[cnt].widx = wi;
                            hits[cnt].pad = 0;
                            hits[cnt].sigma = s;
                        }
                        cnt++;
                    }
                }
            }
        }
    }
    free(P);
    free(coef);
    return cnt;
}

/* prune_related1(hibins, hivals, downfact) of single_pulse_search.py, step for step:
 *   for ii in range(len-1): skip removed ii; for jj > ii: break when |bin_jj - bin_ii| >
 *   downfact/2 (integer); skip removed jj; remove jj if val_ii > val_jj, else remove ii.
 * bins ascending; removed[n] receives 1 for every removed entry.                          */
void sp_prune_related1(const int32_t* bins, const double* vals, int64_t n, int downfact, uint8_t* removed)
{
    memset(removed, 0, (size_t)n);
    const int half = downfact / 2;
    for (int64_t ii = 0; ii + 1 < n; ii++) {
        if (removed[ii]) continue;
        for (int64_t jj = ii + 1; jj < n; jj++) {
            const int gap = bins[jj] - bins[ii];
            if ((gap < 0 ? -gap : gap) > half) break;
            if (removed[jj]) continue;
            if (vals[ii] > vals[jj]) removed[jj] = 1;
            else removed[ii] = 1;
        }
    }
}
