// hd_sp.hip — single-pulse search on the device-resident DM series of a pass: PRESTO's
// single_pulse_search.py, which the reference runs on every .dat the pass writes
// (`single_pulse_search.py -p -m maxwidth -t threshold <dat>`,
// lib/python/PALFA2_presto_search.py:539-546; maxwidth 0.1 s, threshold 5.0 from
// lib/python/config/searching_example.py:13-15).  [PRESTO-ext] restated:
//   * the first roundN = floor(N / 1000) * 1000 samples, in blocks of detrendlen = 1000:
//     each block linearly detrended (least-squares line, scipy.signal.detrend), its std
//     taken over the middle 95 % of its sorted detrended values, times 1.148;
//   * per DM, blocks whose std lies 4 sigma off the pseudo-median of the sorted stds
//     (locut/hicut split) are bad: not searched and zeroed;
//   * the data divided by its block std, then boxcars of the downfactors <= maxwidth
//     (1, 2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150, 220, 300 samples, kernel
//     1/sqrt(w) at PRESTO's offsets) over the first numchunks * 8000 samples (zero beyond);
//     a value above threshold outside the bad blocks is a hit;
//   * prune_related1 per (chunk, width > 1) exactly as the script's greedy walk, in the O(n)
//     form it reduces to: in bin order a hit is a "pivot" unless the
//     last pivot lies within h = w/2 bins and is strictly stronger; a pivot survives when
//     the next pivot is more than h bins later (or there is none).  One lane walks one
//     (chunk, width) over a bitmask of its above-threshold bins (made by wave ballots, one
//     lane per bin, so the prefix-sum reads are bank-conflict free).  Splitting the walk into
//     independent runs (a hit more than h bins after the previous one starts a new run) over
//     the 64 lanes measured slower: a bright pulse is one run of thousands of hits, still
//     walked by one lane, and the lanes' second pass for the zip costs more than it saves;
//   * the script's bad-block test after the walk: survivor m is paired with the block of the
//     m-th UNPRUNED hit (`zip(hibins, hivals, hiblocks)` with hiblocks taken before
//     prune_related1); width-1 hits are tested against their own block.
// The survivors go to the host (hd_api.hip) for prune_related2 and the border cases.
// Arithmetic is double with a fixed summation order (lane partials in index order, then a
// xor butterfly over the 64 lanes; per-chunk prefix sums over 256 segments of 34 samples),
// so oracle/sp_oracle.c reproduces every value bit for bit; PRESTO's float32 FFT
// convolution is replaced by exact window sums (no circular wrap of windows wider than its
// 96-sample chunk overlap).
#include <stdlib.h>

#include "hd_internal.h"

namespace hd {

constexpr int kSpBlock = 1000;               // detrendlen
constexpr int kSpChunk = 8000;               // chunklen
constexpr int kSpHalo = 224;                 // >= max downfact / 2 + 1 (a boxcar's reach)
constexpr int kSpSeg = 33;                   // prefix-sum segment per thread
constexpr int kSpWin = 256 * kSpSeg;         // kSpChunk + 2 * kSpHalo = 8448
constexpr int kSpWords = kSpChunk / 32;      // hit bitmask words per (chunk, width)
constexpr int kSpRound = 8;                  // widths per round (bitmask LDS: 8 KB), walked by lanes 0-1 of each wave

__device__ __forceinline__ double wave_sum_f64(double v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// ---- per (DM, block): detrend line and trimmed std ------------------------------------
// One wave per block; lane l holds samples 16l .. 16l+15 of it (the last 24 slots are +inf
// pads for the sort).  coef[(dm * nblocks + b) * 4 + {0,1,2}] = mean, slope, std.
__global__ __launch_bounds__(256) void k_sp_blocks(const float* __restrict__ x, int64_t stride, int32_t ndm,
                                                   int32_t nblocks, double* __restrict__ coef)
{
    const int lane = threadIdx.x & 63;
    const int64_t gb = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gb >= (int64_t)ndm * nblocks) return;                 // whole waves leave; no barriers below
    const int dm = (int)(gb / nblocks), b = (int)(gb - (int64_t)dm * nblocks);
    const float* xb = x + (int64_t)dm * stride + (int64_t)b * kSpBlock;
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int i = 16 * lane + r;
        v[r] = i < kSpBlock ? xb[i] : 0.0f;
    }
    // least-squares line: t centred at 499.5, S_tt = L (L^2 - 1) / 12 exactly
    double s = 0.0, st = 0.0;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int i = 16 * lane + r;
        if (i < kSpBlock) {
            s += (double)v[r];
            st += ((double)i - 499.5) * (double)v[r];
        }
    }
    s = wave_sum_f64(s);
    st = wave_sum_f64(st);
    const double mean = s / (double)kSpBlock;
    const double slope = st / 83333250.0;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int i = 16 * lane + r;
        v[r] = i < kSpBlock ? (float)((double)v[r] - (mean + slope * ((double)i - 499.5))) : __builtin_inff();
    }
    // bitonic sort of the 1024 slots (element 16l + r in lane l, register r)
    for (int k = 2; k <= 1024; k <<= 1) {
        for (int j = k >> 1; j >= 16; j >>= 1) {              // partner in lane l ^ (j / 16)
            const int lm = j >> 4;
            const bool asc = ((16 * lane) & k) == 0, lower = (lane & lm) == 0;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const float o = __shfl_xor(v[r], lm, 64);
                v[r] = (asc == lower) ? fminf(v[r], o) : fmaxf(v[r], o);
            }
        }
        for (int j = (k >> 1) < 8 ? (k >> 1) : 8; j >= 1; j >>= 1) {   // partner in this lane
#pragma unroll
            for (int r = 0; r < 16; r++) {
                if (r & j) continue;
                const int p = r | j;
                const bool asc = ((16 * lane + r) & k) == 0;
                const float a = v[r], c = v[p];
                const float lo = fminf(a, c), hi = fmaxf(a, c);
                v[r] = asc ? lo : hi;
                v[p] = asc ? hi : lo;
            }
        }
    }
    double q = 0.0;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int i = 16 * lane + r;
        if (i >= kSpBlock / 40 && i < kSpBlock - kSpBlock / 40) q += (double)v[r] * (double)v[r];
    }
    q = wave_sum_f64(q);
    if (lane == 0) {
        double* cf = coef + gb * 4;
        cf[0] = mean;
        cf[1] = slope;
        cf[2] = sqrt(q / (0.95 * kSpBlock)) * 1.148;
        cf[3] = 0.0;
    }
}

// ---- per DM: bad blocks from the sorted stds ------------------------------------------
// One 1024-thread workgroup per DM: bitonic sort of the stds (+inf pads to a power of two,
// <= kSpMaxBlocks), then locut / hicut / pseudo-median / population std as the reference
// script computes them (Python 2 integer division), sequentially in index order; bad
// blocks get coef[3] = 1 and the median as their std.
constexpr int kSpMaxBlocks = 8192;

__global__ __launch_bounds__(1024) void k_sp_robust(double* __restrict__ coef, int32_t nblocks)
{
    __shared__ double srt[kSpMaxBlocks];
    __shared__ double lim[3];                                  // lo, hi, median
    double* cf = coef + (int64_t)blockIdx.x * nblocks * 4;
    int n2 = 1;
    while (n2 < nblocks) n2 <<= 1;
    for (int i = threadIdx.x; i < n2; i += blockDim.x) srt[i] = i < nblocks ? cf[(int64_t)i * 4 + 2] : __builtin_inf();
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n2; i += blockDim.x) {
                const int l = i ^ j;
                if (l > i) {
                    const double a = srt[i], c = srt[l];
                    const bool up = (i & k) == 0;
                    if (up ? a > c : a < c) {
                        srt[i] = c;
                        srt[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    if (threadIdx.x == 0) {
        const int nb = nblocks, h = nb / 2;
        int locut = 1, hicut = 0;
        double best = -__builtin_inf();
        for (int i = 0; i < h; i++) {
            const double d = srt[i + 1] - srt[i];
            if (d > best) { best = d; locut = i + 1; }
        }
        best = -__builtin_inf();
        int am = 0;
        for (int i = h; i + 1 < nb; i++) {
            const double d = srt[i + 1] - srt[i];
            if (d > best) { best = d; am = i - h; }
        }
        hicut = am + h - 2;
        const int lo = locut, hi = hicut;
        double lo_std = __builtin_nan(""), hi_std = __builtin_nan(""), med = 0.0;
        if (nb >= 2 && hi > lo) {
            double m = 0.0;
            for (int i = lo; i < hi; i++) m += srt[i];
            m /= (double)(hi - lo);
            double var = 0.0;
            for (int i = lo; i < hi; i++) var += (srt[i] - m) * (srt[i] - m);
            const double sd = sqrt(var / (double)(hi - lo));
            med = srt[(lo + hi) / 2];
            lo_std = med - 4.0 * sd;
            hi_std = med + 4.0 * sd;
        }
        lim[0] = lo_std;
        lim[1] = hi_std;
        lim[2] = med;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nblocks; i += blockDim.x) {
        const double s = cf[(int64_t)i * 4 + 2];
        if (s < lim[0] || s > lim[1]) {                        // NaN limits: nothing is bad
            cf[(int64_t)i * 4 + 2] = lim[2];
            cf[(int64_t)i * 4 + 3] = 1.0;
        }
    }
}

// ---- per (DM, chunk): boxcar hits -----------------------------------------------------
// Normalised sample i: 0 outside [0, ls) and in bad blocks, else
// y = (float)((double)d / std), d = (float)(x - (mean + slope * (t - 499.5))), t = i mod 1000
// (std 0: y = 0).
__device__ __forceinline__ float sp_norm(const float* xs, const double* cf, int64_t i, int64_t ls)
{
    if (i < 0 || i >= ls) return 0.0f;
    const int64_t b = i / kSpBlock;
    const double* c = cf + b * 4;
    if (c[3] != 0.0 || c[2] == 0.0) return 0.0f;
    const double t = (double)(i - b * kSpBlock) - 499.5;
    const float d = (float)((double)xs[i] - (c[0] + c[1] * t));
    return (float)((double)d / c[2]);
}

struct SpArgs {
    const float* x;
    int64_t stride;
    int32_t ndm, nchunks, nwidths;
    int64_t ls;                                  // searched samples: nchunks * 8000
    int32_t nblocks;
    const double* coef;
    double threshold;
    int32_t widths[16];
    double rsw[16];                              // 1 / sqrt(width), host-computed
    hd_sp_hit* hits;
    unsigned long long* count;
    int64_t cap;
    int32_t probe;                               // profiling (HD_SP_PROBE): 1 no walk, 2 no width-1, 4 no bitmask
};

__device__ __forceinline__ void sp_emit(const SpArgs& a, int dm, int64_t bin, int wi, double s)
{
    const unsigned long long slot = atomicAdd(a.count, 1ull);
    if ((int64_t)slot < a.cap) {
        hd_sp_hit h;
        h.dm = dm;
        h.bin = (int32_t)bin;
        h.widx = wi;
        h.pad = 0;
        h.sigma = s;
        a.hits[slot] = h;
    }
}

__global__ __launch_bounds__(256) void k_sp_hits(SpArgs a)
{
    __shared__ double P[kSpWin + 1];
    __shared__ double tot[257];
    __shared__ uint32_t bits[kSpRound][kSpWords];
    const int dm = blockIdx.x / a.nchunks, ch = blockIdx.x - dm * a.nchunks;
    const float* xs = a.x + (int64_t)dm * a.stride;
    const double* cf = a.coef + (int64_t)dm * a.nblocks * 4;
    const int64_t w0 = (int64_t)ch * kSpChunk - kSpHalo;     // sample of window element 0
    const int64_t c0 = (int64_t)ch * kSpChunk;               // first bin of the chunk
    const int tid = threadIdx.x;
    const int wv = tid >> 6, ln = tid & 63;
    double loc[kSpSeg];
    double run = 0.0;
#pragma unroll
    for (int j = 0; j < kSpSeg; j++) {
        run += (double)sp_norm(xs, cf, w0 + tid * kSpSeg + j, a.ls);
        loc[j] = run;
    }
    tot[tid] = run;
    __syncthreads();
    if (tid == 0) {                                           // exclusive scan of the segment totals
        double base = 0.0;
        for (int t = 0; t < 256; t++) {
            const double nb = base + tot[t];
            tot[t] = base;
            base = nb;
        }
        P[0] = 0.0;
    }
    __syncthreads();
    const double base = tot[tid];
#pragma unroll
    for (int j = 0; j < kSpSeg; j++) P[tid * kSpSeg + j + 1] = base + loc[j];
    __syncthreads();
    // boxcar value (width index wi > 0) at chunk bin o
    auto boxcar = [&](int wi, int o) -> double {
        const int w = a.widths[wi];
        const int k = o + kSpHalo;
        const int lo = k - w / 2, hi = k + ((w & 1) ? w / 2 : w / 2 - 1) + 1;
        return (P[hi] - P[lo]) * a.rsw[wi];
    };
    auto bad = [&](int o) { return cf[((c0 + o) / kSpBlock) * 4 + 3] != 0.0; };
    // width 1: every value above threshold outside the bad blocks (no prune_related1)
    for (int o = tid; o < kSpChunk && !(a.probe & 2); o += 256) {
        if (bad(o)) continue;
        const double s = (double)sp_norm(xs, cf, c0 + o, a.ls);
        if (s > a.threshold) sp_emit(a, dm, c0 + o, 0, s);
    }
    for (int r0 = 1; r0 < a.nwidths; r0 += kSpRound) {
        const int nr = min(kSpRound, a.nwidths - r0);
        // the above-threshold bins of widths r0 .. r0+nr-1 (bad blocks included: the script
        // prunes before it looks at blocks): lane = bin, one ballot per 64 bins (consecutive
        // lanes read consecutive P entries: no bank conflicts)
        for (int t = wv; t < nr * (kSpChunk / 64); t += 4) {
            const int j = t / (kSpChunk / 64), q = t - j * (kSpChunk / 64);
            const bool hit = !(a.probe & 4) && boxcar(r0 + j, 64 * q + ln) > a.threshold;
            const uint64_t m = __ballot(hit);
            if (ln == 0) {
                bits[j][2 * q] = (uint32_t)m;
                bits[j][2 * q + 1] = (uint32_t)(m >> 32);
            }
        }
        __syncthreads();
        // prune_related1: width r0 + j walked by lane j >> 2 of wave j & 3
        const int j = wv + 4 * ln;
        if (ln < 2 && j < nr && !(a.probe & 1)) {
            const int wi = r0 + j;
            const int h = a.widths[wi] / 2;
            const uint32_t* bm = bits[j];
            int lpb = 0, zw = 0;
            double lpx = 0.0;
            bool have = false;
            uint32_t zm = bm[0];
            auto survivor = [&](int b, double x) {
                while (zm == 0) zm = bm[++zw];                // the m-th unpruned hit (m <= current)
                const int hb = 32 * zw + __builtin_ctz(zm);
                zm &= zm - 1;
                if (!bad(hb)) sp_emit(a, dm, c0 + b, wi, x);
            };
            // the hits in bin order, their boxcar values read kSpLook hits ahead of the walk
            // (a dense run is thousands of hits: the walk must not wait for each value's LDS
            // reads in turn)
            int rw = 0;
            uint32_t rm = bm[0];
            auto next_bit = [&]() -> int {
                while (!rm && rw < kSpWords - 1) rm = bm[++rw];
                if (!rm) return -1;
                const int b = 32 * rw + __builtin_ctz(rm);
                rm &= rm - 1;
                return b;
            };
            constexpr int kSpLook = 4;
            int qb[kSpLook];
            double qx[kSpLook];
#pragma unroll
            for (int k = 0; k < kSpLook; k++) {
                qb[k] = next_bit();
                qx[k] = qb[k] >= 0 ? boxcar(wi, qb[k]) : 0.0;
            }
            while (qb[0] >= 0) {
                const int b = qb[0];
                const double x = qx[0];
#pragma unroll
                for (int k = 0; k + 1 < kSpLook; k++) {
                    qb[k] = qb[k + 1];
                    qx[k] = qx[k + 1];
                }
                qb[kSpLook - 1] = next_bit();
                qx[kSpLook - 1] = qb[kSpLook - 1] >= 0 ? boxcar(wi, qb[kSpLook - 1]) : 0.0;
                if (have && b - lpb <= h && lpx > x) continue;         // removed by the last pivot
                if (have && b - lpb > h) survivor(lpb, lpx);           // else the new pivot removes it
                lpb = b;
                lpx = x;
                have = true;
            }
            if (have) survivor(lpb, lpx);
        }
        __syncthreads();
    }
}

// The bad-block flags as bytes (the host needs ndm * nblocks bytes, not the 32-byte records).
__global__ __launch_bounds__(256) void k_sp_badflags(const double* __restrict__ coef, int64_t n, uint8_t* __restrict__ bad)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) bad[i] = coef[4 * i + 3] != 0.0;
}

hipError_t launch_sp_badflags(const double* coef, int64_t n, uint8_t* bad, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sp_badflags, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, coef, n, bad);
    return hipGetLastError();
}

int sp_max_blocks() { return kSpMaxBlocks; }

hipError_t launch_sp_blocks(const float* x, int64_t stride, int ndm, int nblocks, double* coef, hipStream_t st)
{
    const int64_t nw = (int64_t)ndm * nblocks;
    if (nw <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sp_blocks, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, st, x, stride, ndm, nblocks, coef);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (nblocks > kSpMaxBlocks) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_sp_robust, dim3((unsigned)ndm), dim3(1024), 0, st, coef, nblocks);
    return hipGetLastError();
}

hipError_t launch_sp_hits(const float* x, int64_t stride, int ndm, int nblocks, const double* coef, int64_t ls,
                          const int32_t* widths, const double* rsw, int nwidths, double threshold, hd_sp_hit* hits,
                          unsigned long long* count, int64_t cap, hipStream_t st)
{
    SpArgs a{};
    a.x = x;
    a.stride = stride;
    a.ndm = ndm;
    a.nchunks = (int32_t)(ls / kSpChunk);
    a.ls = ls;
    a.nblocks = nblocks;
    a.coef = coef;
    a.threshold = threshold;
    a.nwidths = nwidths;
    if (nwidths < 1 || nwidths > 16) return hipErrorInvalidValue;
    for (int i = 0; i < nwidths; i++) {
        if (widths[i] < 1 || widths[i] / 2 + 1 > kSpHalo) return hipErrorInvalidValue;
        a.widths[i] = widths[i];
        a.rsw[i] = rsw[i];
    }
    a.hits = hits;
    a.count = count;
    a.cap = cap;
    a.probe = getenv("HD_SP_PROBE") ? atoi(getenv("HD_SP_PROBE")) : 0;
    if (a.nchunks <= 0 || ndm <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sp_hits, dim3((unsigned)(ndm * a.nchunks)), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace hd
