/* TEST INFRASTRUCTURE ONLY: a driver that runs every entry point of the C oracle
 * (prepsubband_oracle.c, sp_oracle.c) on small synthetic inputs -- 8/4/16-bit, flipped and
 * not, masked, clipped, downsampled, padded, plus the single-pulse hits -- so the oracle can
 * be built and run under AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle
 * selftest`, tests/test_oracle_sanitize.py).  Exit status 0 = clean run. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
    int32_t dm, bin, widx, pad;
    double sigma;
} sp_hit;
int64_t sp_oracle_hits(const float* x, int64_t stride, int ndm, int64_t n, const int32_t* widths, int nwidths,
                       double threshold, sp_hit* hits, int64_t cap, uint8_t* bad);

static uint32_t rng = 12345u;
static uint32_t rnd(void)
{
    rng = rng * 1664525u + 1013904223u;
    return rng >> 8;
}

static int run_case(int nbits, int flip, int ds, int sub_dtype, double clip, int masked)
{
    or_obs obs = {0};
    obs.nchan = 64;
    obs.nbits = nbits;
    obs.npol = 1;
    obs.flip = flip;
    obs.dt = 6.5476e-5;
    obs.lofreq = 1214.0;
    obs.df = 5.0;
    obs.N = 4096 + 37;
    obs.nsblk = 512;
    or_opts opts = {0};
    opts.sub_dtype = sub_dtype;
    opts.ds_mode = 1;
    opts.pad_mode = 2;
    opts.nibble_hi_first = 1;
    opts.be16 = 1;
    opts.clip_sigma = (float)clip;
    const int rowbytes = obs.nchan * nbits / 8;
    uint8_t* raw = malloc((size_t)obs.N * rowbytes);
    for (int64_t i = 0; i < obs.N * rowbytes; i++) raw[i] = (uint8_t)(rnd() & (nbits == 4 ? 0x77 : 0x7f));
    for (int k = 0; k < 6; k++) memset(raw + (int64_t)(rnd() % obs.N) * rowbytes, 0xff, rowbytes);   /* spikes */
    const int blk = obs.nsblk, nblk = (int)((obs.N + blk - 1) / blk);
    uint8_t* zap = calloc((size_t)nblk * obs.nchan, 1);
    uint8_t* allzap = calloc(nblk, 1);
    if (masked) {
        const int numint = 3, pts = 1400;
        uint8_t* chans = calloc((size_t)numint * obs.nchan, 1);
        chans[5] = chans[obs.nchan + 9] = chans[2 * obs.nchan + 5] = 1;
        or_mask m = {chans, NULL, numint, pts, 0.0};
        or_check_mask_blocks(&obs, &m, blk, nblk, zap, allzap);
        free(chans);
    }
    float* pad = calloc((size_t)nblk * obs.nchan, sizeof(float));
    uint8_t* clipped = calloc(obs.N, 1);
    float padv[64];
    for (int c = 0; c < 64; c++) padv[c] = 20.0f + 0.25f * c;
    const int64_t nc = or_clip_prepare(&obs, &opts, raw, NULL, NULL, NULL, allzap, padv, blk, nblk, pad, clipped);
    if (nc < 0) return 1;
    const int nsub = 16;
    int32_t idd[64];
    or_chan_delays(&obs, nsub, 120.0, idd);
    const int64_t nds = obs.N / ds;
    const size_t el = sub_dtype == 0 ? 2 : 4;
    void* sub = calloc((size_t)nsub * nds, el);
    if (or_stage1(&obs, &opts, raw, NULL, NULL, NULL, zap, pad, clipped, blk, nblk, nsub, ds, idd, 0, nds, sub, nds))
        return 2;
    const int numdms = 8;
    int32_t* off = malloc(sizeof(int32_t) * numdms * nsub);
    or_dm_offsets(&obs, &opts, nsub, ds, 100.0, 5.0, numdms, off);
    const int64_t numout = nds + 100;
    float* out = calloc((size_t)numdms * numout, sizeof(float));
    if (or_stage2(sub, sub_dtype, nds, nds, nsub, off, numdms, 0, nds, out, numout)) return 3;
    or_pad(out, numdms, nds, numout, opts.pad_mode);
    float stats[3 * 64], pv[64];
    for (int i = 0; i < 3 * 64; i++) stats[i] = (float)(rnd() % 1000) * 0.1f;
    or_stats_padvals(stats, 3, 64, pv);
    free(raw); free(zap); free(allzap); free(pad); free(clipped); free(sub); free(off); free(out);
    return 0;
}

static int run_sp(void)
{
    const int ndm = 2;
    const int64_t n = 17000;
    float* x = malloc(sizeof(float) * ndm * n);
    for (int64_t i = 0; i < ndm * n; i++) x[i] = (float)((int)(rnd() % 2001) - 1000) * 1e-3f;
    for (int k = 0; k < 20; k++) x[rnd() % (ndm * n)] += 9.0f;
    const int32_t widths[] = {1, 2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150, 220, 300};
    sp_hit hits[4096];
    uint8_t bad[64];
    const int64_t nh = sp_oracle_hits(x, n, ndm, n, widths, 15, 5.0, hits, 4096, bad);
    free(x);
    return nh < 0 ? 4 : 0;
}

int main(void)
{
    const int nbits[] = {8, 4, 16};
    int rc = 0;
    for (int b = 0; b < 3 && !rc; b++)
        for (int flip = 0; flip < 2 && !rc; flip++)
            for (int ds = 1; ds <= 3 && !rc; ds += 2) {
                rc = run_case(nbits[b], flip, ds, 0, 6.0, 1);
                if (!rc) rc = run_case(nbits[b], flip, ds, 1, 0.0, 0);
            }
    if (!rc) rc = run_sp();
    printf(rc ? "oracle selftest FAILED (%d)\n" : "oracle selftest ok\n", rc);
    return rc;
}
