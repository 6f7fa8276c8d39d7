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
// widths per round = waves per workgroup (one wave walks each): 16 waves take the 14
// widths > 1 of the 0.1-s downfactors in one round (4 waves: four rounds)
constexpr int kSpSegW = 4;                   // bitmask words (128 bins) per lane segment of a walk

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
    // bitonic sort of the 1024 slots (element 16l + r in lane l, register r), fully unrolled,
    // on order-preserving int keys (integer min / max / med3: no NaN canonicalisation).
    // Merges of size k < 16 lie inside a lane, their directions fixed per register.  From
    // k = 16 on, a lane's direction is one bit of its index: a descending lane holds its keys
    // complemented, so every in-lane compare-exchange is ascending (min to the lower slot);
    // across lanes the lower lane takes med3(v, o, INT_MIN) = min, the upper med3(v, o,
    // INT_MAX) = max.  The sorted values are those of any sort (-0 before +0 here; equal
    // squares either way), so the sum below is unchanged.
    int32_t key[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int32_t bb = __float_as_int(v[r]);
        key[r] = bb ^ ((bb >> 31) & 0x7FFFFFFF);
    }
#pragma unroll
    for (int lk = 1; lk <= 3; lk++) {
        const int k = 1 << lk;
#pragma unroll
        for (int lj = lk - 1; lj >= 0; lj--) {
            const int j = 1 << lj;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                if (r & j) continue;
                const int p = r | j;
                const int32_t lo = min(key[r], key[p]), hi = max(key[r], key[p]);
                const bool asc = (r & k) == 0;
                key[r] = asc ? lo : hi;
                key[p] = asc ? hi : lo;
            }
        }
    }
    int32_t cpl = 0;                                           // current complement mask
#pragma unroll
    for (int lk = 4; lk <= 10; lk++) {
        const int k = 1 << lk;
        const int32_t want = ((16 * lane) & k) ? -1 : 0;
        const int32_t flip = want ^ cpl;
        cpl = want;
#pragma unroll
        for (int r = 0; r < 16; r++) key[r] ^= flip;
#pragma unroll
        for (int lj = lk - 1; lj >= 4; lj--) {                // partner in lane l ^ (j / 16)
            const int lm = 1 << (lj - 4);
            const int32_t bound = (lane & lm) ? 0x7FFFFFFF : (int32_t)0x80000000;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int32_t o = __shfl_xor(key[r], lm, 64);
                int32_t m3;
                asm("v_med3_i32 %0, %1, %2, %3" : "=v"(m3) : "v"(key[r]), "v"(o), "v"(bound));
                key[r] = m3;
            }
        }
#pragma unroll
        for (int lj = 3; lj >= 0; lj--) {                     // partner in this lane
            const int j = 1 << lj;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                if (r & j) continue;
                const int p = r | j;
                const int32_t lo = min(key[r], key[p]), hi = max(key[r], key[p]);
                key[r] = lo;
                key[p] = hi;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 16; r++) v[r] = __int_as_float(key[r] ^ ((key[r] >> 31) & 0x7FFFFFFF));
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
    // bitonic sort of kSpMaxBlocks slots (+inf past nblocks) on order-preserving int64 keys,
    // thread t owning slots 8t .. 8t+7 in registers: merges of j < 8 inside a thread, j < 512
    // across the lanes of a wave (shuffles), only j >= 512 through LDS (10 barrier pairs instead
    // of a barrier per stage); the sorted values equal any sort's
    static_assert(kSpMaxBlocks == 8192, "k_sp_robust sorts 8192 slots with 1024 threads");
    const int tid = threadIdx.x, lane = tid & 63;
    int64_t* skey = (int64_t*)srt;
    int64_t x[8];
    auto dkey = [](double d) {
        const int64_t bb = __double_as_longlong(d);
        return bb ^ ((bb >> 63) & 0x7FFFFFFFFFFFFFFFll);
    };
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const int i = 8 * tid + r;
        x[r] = dkey(i < nblocks ? cf[(int64_t)i * 4 + 2] : __builtin_inf());
    }
#pragma unroll
    for (int lk = 1; lk <= 13; lk++) {
        const int k = 1 << lk;
#pragma unroll
        for (int lj = lk - 1; lj >= 0; lj--) {
            const int j = 1 << lj;
            if (j >= 512) {                                  // partner in another wave: via LDS
#pragma unroll
                for (int r = 0; r < 8; r++) skey[8 * tid + r] = x[r];
                __syncthreads();
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const int i = 8 * tid + r;
                    const int64_t o = skey[i ^ j];
                    const bool asc = (i & k) == 0, lower = (i & j) == 0;
                    x[r] = asc == lower ? min(x[r], o) : max(x[r], o);
                }
                __syncthreads();
            } else if (j >= 8) {                             // partner in lane ^ (j / 8)
                const int lm = j >> 3;
                const bool lower = (lane & lm) == 0;
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const int64_t o = __shfl_xor(x[r], lm, 64);
                    const bool asc = ((8 * tid + r) & k) == 0;
                    x[r] = asc == lower ? min(x[r], o) : max(x[r], o);
                }
            } else {                                         // partner in this thread
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    if (r & j) continue;
                    const int q = r | j;
                    const int64_t lo = min(x[r], x[q]), hi = max(x[r], x[q]);
                    const bool asc = ((8 * tid + r) & k) == 0;
                    x[r] = asc ? lo : hi;
                    x[q] = asc ? hi : lo;
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 8; r++)
        srt[8 * tid + r] = __longlong_as_double(x[r] ^ ((x[r] >> 63) & 0x7FFFFFFFFFFFFFFFll));
    __syncthreads();
    // (the scans and sums below stay sequential in index order, as the oracle's; their LDS
    // reads go 16 at a time so the chains wait on their double ops, not on a round trip each)
    if (threadIdx.x == 0) {
        const int nb = nblocks, h = nb / 2;
        int locut = 1, hicut = 0;
        double best = -__builtin_inf();
        auto scan16 = [&](int i0, int i1, int base, int& arg) {   // first max of srt[i+1]-srt[i]
            for (int i = i0; i < i1; i += 16) {
                double v[17];
#pragma unroll
                for (int k = 0; k < 17; k++) v[k] = i + k < nb ? srt[i + k] : 0.0;
#pragma unroll
                for (int k = 0; k < 16; k++)
                    if (i + k < i1) {
                        const double d = v[k + 1] - v[k];
                        if (d > best) { best = d; arg = i + k - base; }
                    }
            }
        };
        scan16(0, h, -1, locut);                              // locut = i + 1
        best = -__builtin_inf();
        int am = 0;
        scan16(h, nb - 1, h, am);                             // am = i - h
        hicut = am + h - 2;
        const int lo = locut, hi = hicut;
        double lo_std = __builtin_nan(""), hi_std = __builtin_nan(""), med = 0.0;
        if (nb >= 2 && hi > lo) {
            double m = 0.0;
            for (int i = lo; i < hi; i += 16) {
                double v[16];
#pragma unroll
                for (int k = 0; k < 16; k++) v[k] = i + k < hi ? srt[i + k] : 0.0;
#pragma unroll
                for (int k = 0; k < 16; k++)
                    if (i + k < hi) m += v[k];
            }
            m /= (double)(hi - lo);
            double var = 0.0;
            for (int i = lo; i < hi; i += 16) {
                double v[16];
#pragma unroll
                for (int k = 0; k < 16; k++) v[k] = i + k < hi ? srt[i + k] : 0.0;
#pragma unroll
                for (int k = 0; k < 16; k++)
                    if (i + k < hi) var += (v[k] - m) * (v[k] - m);
            }
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
    int32_t probe;                               // profiling (HD_SP_PROBE): 1 no walk, 2 no width-1, 4 no bitmask,
                                                 // 8 no true chain, 16 no emission of the walk's survivors
    uint32_t* stats;                             // profiling (HD_SP_STATS): kSpStats words per workgroup, or null
};
// HD_SP_STATS words: 0-6 wall clock (100 MHz) at the phase ends (normalise, prefix, bitmask,
// spec walk, true chain, emission; round 1 for the last four); 7 sum over widths of the
// busiest lane's walk steps, 8 of its batch loads; 9 true-chain pivots, 10 true-chain ballot
// steps, 11 hits, 12 merges, 13 width of the slowest spec wave, 14 its ticks
constexpr int kSpStats = 16;

// The width-1 hits of the active lanes: one counter atomic per wave (a bright pulse gives
// thousands of hits per chunk; one global atomic each serialised the whole grid on one address)
__device__ __forceinline__ void sp_emit_wave(const SpArgs& a, int dm, int64_t bin, bool hit, double s)
{
    const uint64_t hm = __ballot(hit);
    if (!hm) return;                                           // (uniform)
    const int ln = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
    unsigned long long base = 0;
    if (ln == leader) base = atomicAdd(a.count, (unsigned long long)__popcll(hm));
    base = __shfl(base, leader, 64);
    if (!hit) return;
    const unsigned long long slot = base + (unsigned long long)__popcll(hm & ((1ull << ln) - 1ull));
    if ((int64_t)slot < a.cap) {
        hd_sp_hit h;
        h.dm = dm;
        h.bin = (int32_t)bin;
        h.widx = 0;
        h.pad = 0;
        h.sigma = s;
        a.hits[slot] = h;
    }
}

template <int NW, bool STATS>
__global__ __launch_bounds__(NW * 64) void k_sp_hits(SpArgs a)
{
    constexpr int kSpRound = NW;
    __shared__ double P[kSpWin + 1];
    __shared__ uint32_t bits[kSpRound][kSpWords];
    // the walk's per-width state (its space also holds the segment totals of the prefix sum):
    // spec[w]: pivots of the lanes' speculative walks; emt[w]: pivots whose next pivot is a gap
    // (or none) -- the walk emits them when they are on the true path -- and the true path's
    // pivots off the speculative walks; exit / merge / hit-count prefix per lane segment
    struct WalkLds {
        uint32_t spec[kSpRound][kSpWords];
        uint32_t emt[kSpRound][kSpWords];
        int16_t exitb[kSpRound][64], merge[kSpRound][64], hpre[kSpRound][65];
    };
    __shared__ __attribute__((aligned(16))) char wl_raw[sizeof(WalkLds) > 257 * 8 ? sizeof(WalkLds) : 257 * 8];
    double* tot = (double*)wl_raw;
    WalkLds& W = *(WalkLds*)wl_raw;
    const int dm = blockIdx.x / a.nchunks, ch = blockIdx.x - dm * a.nchunks;
    const float* xs = a.x + (int64_t)dm * a.stride;
    const double* cf = a.coef + (int64_t)dm * a.nblocks * 4;
    const int64_t w0 = (int64_t)ch * kSpChunk - kSpHalo;     // sample of window element 0
    const int64_t c0 = (int64_t)ch * kSpChunk;               // first bin of the chunk
    const int tid = threadIdx.x;
    const int wv = tid >> 6, ln = tid & 63;
    uint32_t* const sst = STATS ? a.stats + (int64_t)blockIdx.x * kSpStats : nullptr;
    const uint64_t t_start = STATS ? wall_clock64() : 0;
    auto stamp = [&](int k) {
        if (sst && tid == 0) sst[k] = (uint32_t)(wall_clock64() - t_start);
    };
    // the normalised samples of the window (detrended by the block's line, over its std; 0 in
    // bad blocks and past the searched length), staged as doubles in P[e + 1]; width 1 is
    // tested on the spot: every value above threshold outside the bad blocks is a hit (no
    // prune_related1), so the chunk's samples are not read and normalised a second time
    // (the window's <= 10 blocks' coefficients staged in LDS and every sample load issued
    // before the arithmetic: the loop no longer waits on two dependent global loads per step)
    __shared__ double cfs[12][4];
    const int64_t wlo = w0 > 0 ? w0 : 0, whi = w0 + kSpWin < a.ls ? w0 + kSpWin : a.ls;
    const int64_t bl0 = wlo / kSpBlock;
    const int nbk = whi > wlo ? (int)((whi - 1) / kSpBlock - bl0 + 1) : 0;
    if (tid < nbk * 4) cfs[tid >> 2][tid & 3] = cf[(bl0 + (tid >> 2)) * 4 + (tid & 3)];
    constexpr int NI = (kSpWin + NW * 64 - 1) / (NW * 64);
    float xv[NI];
#pragma unroll
    for (int it = 0; it < NI; it++) {
        const int e = tid + it * NW * 64;
        const int64_t i = w0 + e;
        xv[it] = e < kSpWin && i >= 0 && i < a.ls ? xs[i] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < NI; it++) {
        const int e = tid + it * NW * 64;
        if (e >= kSpWin) continue;
        const int64_t i = w0 + e;
        float v = 0.0f;
        bool isbad = false;
        if (i >= 0 && i < a.ls) {
            const int64_t b = i / kSpBlock;
            const double* c = cfs[b - bl0];
            isbad = c[3] != 0.0;
            if (!isbad && c[2] != 0.0) {
                const double t = (double)(i - b * kSpBlock) - 499.5;
                const float d = (float)((double)xv[it] - (c[0] + c[1] * t));
                v = (float)((double)d / c[2]);
            }
        }
        P[e + 1] = (double)v;
        const int o = e - kSpHalo;
        sp_emit_wave(a, dm, c0 + o, o >= 0 && o < kSpChunk && !isbad && !(a.probe & 2) && (double)v > a.threshold,
                     (double)v);
    }
    __syncthreads();
    // running sums over 256 segments of kSpSeg samples (the oracle's order), in place
    if (tid < 256) {
        double run = 0.0;
#pragma unroll
        for (int j = 0; j < kSpSeg; j++) {
            run += P[tid * kSpSeg + j + 1];
            P[tid * kSpSeg + j + 1] = run;
        }
        tot[tid] = run;
    }
    __syncthreads();
    if (tid == 0) {                                           // exclusive scan of the segment totals
        // (in order, as before; the totals are read 16 at a time so the chain waits only
        // on its double adds, not on an LDS round trip per segment)
        double base = 0.0;
        for (int t0 = 0; t0 < 256; t0 += 16) {
            double v[16];
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = tot[t0 + k];
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const double nb = base + v[k];
                v[k] = base;
                base = nb;
            }
#pragma unroll
            for (int k = 0; k < 16; k++) tot[t0 + k] = v[k];
        }
        P[0] = 0.0;
    }
    stamp(0);
    __syncthreads();
    if (tid < 256) {
        const double base = tot[tid];
#pragma unroll
        for (int j = 0; j < kSpSeg; j++) P[tid * kSpSeg + j + 1] = base + P[tid * kSpSeg + j + 1];
    }
    __syncthreads();
    stamp(1);
    // boxcar value (width index wi > 0) at chunk bin o
    auto boxcar = [&](int wi, int o) -> double {
        const int w = a.widths[wi];
        const int k = o + kSpHalo;
        const int lo = k - w / 2, hi = k + ((w & 1) ? w / 2 : w / 2 - 1) + 1;
        return (P[hi] - P[lo]) * a.rsw[wi];
    };
    // the bad flags of the chunk's 8 blocks, one bit each (every wave, once)
    const uint64_t badm = __ballot(ln < kSpChunk / kSpBlock && cf[(c0 / kSpBlock + ln) * 4 + 3] != 0.0);
    for (int r0 = 1; r0 < a.nwidths; r0 += kSpRound) {
        const int nr = min(kSpRound, a.nwidths - r0);
        // the above-threshold bins of widths r0 .. r0+nr-1 (bad blocks included: the script
        // prunes before it looks at blocks): lane = bin, one ballot per 64 bins (consecutive
        // lanes read consecutive P entries: no bank conflicts)
        // Wave wv takes the contiguous items [t0, t1) of the nr x 125 (width, 64 bins): at most
        // two widths, whose parameters it loads once, and four boxcars' LDS reads in flight
        // before their ballots (was: every 16th item, the width and scale reloaded per item and
        // each compare waiting on its own two reads).  The boxcar values are the same doubles.
        uint32_t nhit_wv = 0;                                 // (HD_SP_STATS)
        constexpr int kQ = kSpChunk / 64;
        const int t1 = (wv + 1) * nr * kQ / NW;
        for (int t = wv * nr * kQ / NW; t < t1;) {
            const int j = t / kQ;
            const int te = min(t1, (j + 1) * kQ);
            const int w = a.widths[r0 + j];
            const double rs = a.rsw[r0 + j];
            const int dlo = kSpHalo - w / 2, dhi = kSpHalo + ((w & 1) ? w / 2 : w / 2 - 1) + 1;
            auto put = [&](int q, double v) {
                const uint64_t m = __ballot(!(a.probe & 4) && v > a.threshold);
                if (ln == 0) {
                    bits[j][2 * q] = (uint32_t)m;
                    bits[j][2 * q + 1] = (uint32_t)(m >> 32);
                }
                nhit_wv += (uint32_t)__popcll(m);
            };
            for (; t + 4 <= te; t += 4) {
                const int o = 64 * (t - j * kQ) + ln;
                double v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) v[u] = (P[o + 64 * u + dhi] - P[o + 64 * u + dlo]) * rs;
#pragma unroll
                for (int u = 0; u < 4; u++) put(t - j * kQ + u, v[u]);
            }
            for (; t < te; t++) {
                const int o = 64 * (t - j * kQ) + ln;
                put(t - j * kQ, (P[o + dhi] - P[o + dlo]) * rs);
            }
        }
        if (sst && ln == 0 && nhit_wv) atomicAdd(sst + 11, nhit_wv);
        __syncthreads();
        if (r0 == 1) stamp(2);
        // prune_related1 of width r0 + wv, by wave wv.  The script's walk is a chain through a
        // function of the pivot alone: next(p) = the first hit q > p with q - p > h or
        // x_q >= x_p (hits between are dropped), and p is kept when that step is a gap (or p is
        // the last pivot).  Each lane walks its 128-bin segment speculatively from the
        // segment's first hit; one lane then follows the true chain, which coincides with a
        // segment's speculative chain from the first pivot they share (merge), walking only the
        // pivots before it; the kept pivots are emitted in order, paired with the hits of the
        // unpruned list at the same index (the script's zip quirk) for the bad-block test.
        const int jw = wv;
        const bool walk = jw < nr && !(a.probe & 1);
        const int wi = r0 + jw;
        const int h = walk ? a.widths[wi] / 2 : 0;
        const uint32_t* bm = bits[walk ? jw : 0];
        uint64_t segmask = 0;                                 // lane segments holding hits (spec phase)
        auto nexthit = [&](int b) -> int {                    // first hit bin > b, or -1
            int w = (b + 1) >> 5;
            if (w >= kSpWords) return -1;
            const uint32_t m = bm[w] & (~0u << ((b + 1) & 31));
            if (m) return 32 * w + __builtin_ctz(m);
            const int sg = w / kSpSegW;
            for (int ww = w + 1; ww < min(kSpSegW * (sg + 1), kSpWords); ww++)
                if (bm[ww]) return 32 * ww + __builtin_ctz(bm[ww]);
            const uint64_t rest = sg + 1 < 64 ? segmask >> (sg + 1) : 0ull;   // empty segments skipped
            if (!rest) return -1;
            for (int ww = kSpSegW * (sg + 1 + __builtin_ctzll(rest));; ww++)
                if (bm[ww]) return 32 * ww + __builtin_ctz(bm[ww]);
        };
        auto nextword = [&](int w) -> int {                   // first word > w holding hits, or -1
            const int sg = w / kSpSegW;
            for (int ww = w + 1; ww < min(kSpSegW * (sg + 1), kSpWords); ww++)
                if (bm[ww]) return ww;
            const uint64_t rest = sg + 1 < 64 ? segmask >> (sg + 1) : 0ull;
            if (!rest) return -1;
            for (int ww = kSpSegW * (sg + 1 + __builtin_ctzll(rest));; ww++)
                if (bm[ww]) return ww;
        };
        // The lane streams through the hits after its segment's first hit in bin order, eight
        // per iteration (their boxcars read together), each tested against the current pivot,
        // which moves to the first one that qualifies; the remaining hits of the batch are then
        // tested against the new pivot.  One flat loop: the wave's trip count is the longest
        // lane's batch count (a next-pivot search nested in a loop over pivots made it the sum
        // over steps of the slowest lane's search).  Pivot / kept bits: bin - 128 * lane.
        int n_step = 0, n_batch = 0;                          // (HD_SP_STATS)
        const int sw0 = ln * kSpSegW;                             // this lane's words
        const uint64_t t_spec = STATS ? wall_clock64() : 0;
        if (walk) {
            uint64_t sp_lo = 0, sp_hi = 0, em_lo = 0, em_hi = 0;
            const int segbeg = 32 * sw0, segend = 32 * (sw0 + kSpSegW);
            auto setbit = [&](uint64_t& lo, uint64_t& hi, int b) {
                const int r = b - segbeg;
                if (r < 64) lo |= 1ull << r;
                else hi |= 1ull << (r - 64);
            };
            int ex = -1, nh = 0;
            int p = -1;
#pragma unroll
            for (int k = 0; k < kSpSegW; k++) {
                const uint32_t m = sw0 + k < kSpWords ? bm[sw0 + k] : 0u;
                nh += __builtin_popcount(m);
                if (p < 0 && m) p = 32 * (sw0 + k) + __builtin_ctz(m);
            }
            segmask = __ballot(nh > 0);
            bool act = p >= 0;
            double px = 0.0;
            int w = 0;
            uint32_t m = 0;
            if (act) {
                px = boxcar(wi, p);
                setbit(sp_lo, sp_hi, p);
                w = (p + 1) >> 5;
                if (w < kSpWords) {
                    m = bm[w] & (~0u << ((p + 1) & 31));
                } else {
                    setbit(em_lo, em_hi, p);                  // the last bin: no next pivot
                    act = false;
                }
            }
            while (act) {
                if (!m) {
                    w = nextword(w);
                    if (w < 0) {                              // no hit after p: p is kept
                        setbit(em_lo, em_hi, p);
                        act = false;
                        break;
                    }
                    m = bm[w];
                }
                int cq[8];
                double cx[8];
                int n = 0;
                n_batch++;
#pragma unroll
                for (int k = 0; k < 8; k++)
                    if (m) {
                        cq[k] = 32 * w + __builtin_ctz(m);
                        m &= m - 1;
                        n = k + 1;
                    }
#pragma unroll
                for (int k = 0; k < 8; k++)
                    if (k < n) cx[k] = boxcar(wi, cq[k]);
#pragma unroll
                for (int k = 0; k < 8; k++)
                    if (act && k < n) {
                        const int q = cq[k];
                        if (q - p > h || cx[k] >= px) {
                            n_step++;
                            if (q - p > h) setbit(em_lo, em_hi, p);
                            p = q;
                            px = cx[k];
                            if (p >= segend) {
                                ex = p;
                                act = false;
                            } else {
                                setbit(sp_lo, sp_hi, p);
                            }
                        }
                    }
            }
            const uint32_t sp[kSpSegW] = {(uint32_t)sp_lo, (uint32_t)(sp_lo >> 32), (uint32_t)sp_hi,
                                          (uint32_t)(sp_hi >> 32)};
            const uint32_t em[kSpSegW] = {(uint32_t)em_lo, (uint32_t)(em_lo >> 32), (uint32_t)em_hi,
                                          (uint32_t)(em_hi >> 32)};
#pragma unroll
            for (int k = 0; k < kSpSegW; k++)
                if (sw0 + k < kSpWords) {
                    W.spec[jw][sw0 + k] = sp[k];
                    W.emt[jw][sw0 + k] = em[k];
                }
            W.exitb[jw][ln] = (int16_t)ex;
            W.merge[jw][ln] = (int16_t)32767;
            // exclusive prefix of the segments' hit counts (the zip quirk's rank lookup)
            int inc = nh;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(inc, o, 64);
                if (ln >= o) inc += t;
            }
            W.hpre[jw][ln + 1] = (int16_t)inc;
            if (ln == 0) W.hpre[jw][0] = 0;
            if (sst) {
                int ms = n_step, mb = n_batch;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) {
                    ms = max(ms, __shfl_xor(ms, o, 64));
                    mb = max(mb, __shfl_xor(mb, o, 64));
                }
                const uint32_t dt = (uint32_t)(wall_clock64() - t_spec);
                if (ln == 0) {
                    atomicAdd(sst + 7, (uint32_t)ms);
                    atomicAdd(sst + 8, (uint32_t)mb);
                    const uint32_t old = atomicMax(sst + 14, dt);
                    if (dt > old) sst[13] = (uint32_t)a.widths[wi];
                }
            }
        }
        __syncthreads();
        if (r0 == 1) stamp(3);
        // the true chain from the chunk's first hit, walked by the whole wave: each step tests
        // the 64 bins from the first hit after the pivot at once (lane l: bin start + l; the
        // first qualifying hit by ballot), so a step that skips a dense stretch of h bins costs
        // h / 64 LDS round trips instead of h / 8 (one lane's batches) -- in a dense falling
        // run the chain hops by h + 1 and never meets the lanes' speculative chains
        if (walk && !(a.probe & 8)) {                             // (probe 8: profiling only)
            uint32_t n_true = 0, n_merge = 0, n_ballot = 0;       // (HD_SP_STATS)
            int p = nexthit(-1);
            double px = p >= 0 ? boxcar(wi, p) : 0.0;
            while (p >= 0) {
                const int sg = p >> 7;
                n_true++;
                if ((W.spec[jw][p >> 5] >> (p & 31)) & 1u) {      // on the segment's chain from here
                    n_merge++;
                    if (ln == 0) W.merge[jw][sg] = (int16_t)p;
                    p = W.exitb[jw][sg];
                    if (p >= 0) px = boxcar(wi, p);
                    continue;
                }
                int q = -1;
                double qx = 0.0;
                for (int start = nexthit(p); start >= 0;) {
                    const int b = start + ln;
                    const bool ishit = b < kSpChunk && ((bm[b >> 5] >> (b & 31)) & 1u);
                    double xb = 0.0;
                    bool qual = false;
                    if (ishit) {
                        xb = boxcar(wi, b);
                        qual = b - p > h || xb >= px;
                    }
                    const uint64_t qm = __ballot(qual);
                    n_ballot++;
                    if (qm) {
                        const int fl = __ffsll((unsigned long long)qm) - 1;
                        q = start + fl;
                        qx = __shfl(xb, fl, 64);
                        break;
                    }
                    start = start + 63 < kSpChunk ? nexthit(start + 63) : -1;
                }
                if (ln == 0 && (q < 0 || q - p > h)) W.emt[jw][p >> 5] |= 1u << (p & 31);   // not in spec: kept pivot
                p = q;
                px = qx;
            }
            if (sst && ln == 0) {
                atomicAdd(sst + 9, n_true);
                atomicAdd(sst + 10, n_ballot);
                atomicAdd(sst + 12, n_merge);
            }
        }
        __syncthreads();
        if (r0 == 1) stamp(4);
        // emit the kept pivots of this lane's segment in bin order, with their ordinals
        if (walk && !(a.probe & 16)) {                           // (probe 16: profiling only)
            const int mg = W.merge[jw][ln];
            uint32_t kv[kSpSegW];
            int nk = 0;
#pragma unroll
            for (int k = 0; k < kSpSegW; k++) {
                const int w = sw0 + k;
                uint32_t v = 0;
                if (w < kSpWords) {
                    const uint32_t spw = W.spec[jw][w], emw = W.emt[jw][w];
                    // spec pivots at or after the merge bin; plus true pivots off the spec chain
                    const int lo = mg - 32 * w;
                    const uint32_t ge = lo <= 0 ? ~0u : lo >= 32 ? 0u : (~0u << lo);
                    v = (emw & spw & ge) | (emw & ~spw);
                }
                kv[k] = v;
                nk += __builtin_popcount(v);
            }
            int inc = nk;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(inc, o, 64);
                if (ln >= o) inc += t;
            }
            const int16_t* hp = W.hpre[jw];
            // the m-th hit of the unpruned list (its segment by the prefix counts, then its bit)
            auto hitrank = [&](int m) -> int {
                int lo = 0, hi = 63;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (hp[mid] <= m) lo = mid;
                    else hi = mid - 1;
                }
                int r = m - hp[lo];
                for (int kk = 0; kk < kSpSegW; kk++) {
                    const int w = lo * kSpSegW + kk;
                    uint32_t mw = w < kSpWords ? bm[w] : 0u;
                    const int c = __builtin_popcount(mw);
                    if (r >= c) {
                        r -= c;
                        continue;
                    }
                    for (; r > 0; r--) mw &= mw - 1;
                    return 32 * w + __builtin_ctz(mw);
                }
                return 0;
            };
            // kept pivots whose zip-quirk partner lies outside the bad blocks: counted, one
            // atomic per wave reserves their slots, then written in bin order
            // (the lane's kept pivots have consecutive ordinals, so their partners are
            // consecutive hits: the first by rank, each next one the hit after the last)
            const int m0 = inc - nk;                              // ordinal of this lane's first kept pivot
            int ng = 0;
            {
                int hb = -1;
#pragma unroll
                for (int k = 0; k < kSpSegW; k++)
                    for (uint32_t v = kv[k]; v; v &= v - 1) {
                        hb = hb < 0 ? hitrank(m0) : nexthit(hb);
                        ng += !((badm >> (hb / kSpBlock)) & 1ull);
                    }
            }
            int incg = ng;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incg, o, 64);
                if (ln >= o) incg += t;
            }
            const int totg = __shfl(incg, 63, 64);
            unsigned long long base = 0;
            if (ln == 0 && totg > 0) base = atomicAdd(a.count, (unsigned long long)totg);
            base = __shfl(base, 0, 64);
            unsigned long long slot = base + (unsigned long long)(incg - ng);
            int hb = -1;
#pragma unroll
            for (int k = 0; k < kSpSegW; k++)
                for (uint32_t v = kv[k]; v; v &= v - 1) {
                    const int b = 32 * (sw0 + k) + __builtin_ctz(v);
                    hb = hb < 0 ? hitrank(m0) : nexthit(hb);
                    if ((badm >> (hb / kSpBlock)) & 1ull) continue;
                    if ((int64_t)slot < a.cap) {
                        hd_sp_hit r;
                        r.dm = dm;
                        r.bin = (int32_t)(c0 + b);
                        r.widx = wi;
                        r.pad = 0;
                        r.sigma = boxcar(wi, b);
                        a.hits[slot] = r;
                    }
                    slot++;
                }
        }
        __syncthreads();
        if (r0 == 1) stamp(5);
    }
    stamp(6);
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
    // HD_SP_STATS=1 (profiling): per-workgroup phase clocks and walk counters, summarised
    // on stderr after each launch (synchronises the stream)
    static uint32_t* d_stats = nullptr;
    static int64_t stats_n = 0;
    const int64_t nwg = (int64_t)ndm * a.nchunks;
    const bool want_stats = getenv("HD_SP_STATS") && atoi(getenv("HD_SP_STATS"));
    if (want_stats) {
        if (stats_n < nwg) {
            if (d_stats) (void)hipFree(d_stats);
            if (hipMalloc(&d_stats, nwg * kSpStats * 4) != hipSuccess) return hipErrorOutOfMemory;
            stats_n = nwg;
        }
        (void)hipMemsetAsync(d_stats, 0, nwg * kSpStats * 4, st);
        a.stats = d_stats;
    }
    // HD_SP_NW=4 (profiling): the 4-wave workgroup, four rounds of widths
    if (getenv("HD_SP_NW") && atoi(getenv("HD_SP_NW")) == 4)
        hipLaunchKernelGGL((k_sp_hits<4, false>), dim3((unsigned)(ndm * a.nchunks)), dim3(256), 0, st, a);
    else if (want_stats)
        hipLaunchKernelGGL((k_sp_hits<16, true>), dim3((unsigned)(ndm * a.nchunks)), dim3(1024), 0, st, a);
    else
        hipLaunchKernelGGL((k_sp_hits<16, false>), dim3((unsigned)(ndm * a.nchunks)), dim3(1024), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !want_stats) return e;
    static int call = 0;
    uint32_t* h = (uint32_t*)malloc(nwg * kSpStats * 4);
    if (!h) return hipErrorOutOfMemory;
    (void)hipStreamSynchronize(st);
    (void)hipMemcpy(h, d_stats, nwg * kSpStats * 4, hipMemcpyDeviceToHost);
    // phase sums over workgroups and the 6 slowest workgroups
    double ph[7] = {0, 0, 0, 0, 0, 0, 0};
    int64_t top[6] = {-1, -1, -1, -1, -1, -1};
    for (int64_t g = 0; g < nwg; g++) {
        const uint32_t* r = h + g * kSpStats;
        for (int k = 0; k < 7; k++) ph[k] += (double)(r[k] - (k ? r[k - 1] : 0)) * 1e-5;  // ms
        int64_t cur = g;
        for (int k = 0; k < 6 && cur >= 0; k++)
            if (top[k] < 0 || h[top[k] * kSpStats + 6] < h[cur * kSpStats + 6]) {
                const int64_t t = top[k];
                top[k] = cur;
                cur = t;
            }
    }
    fprintf(stderr, "sp_stats call %d ndm %d nchunks %d: workgroup-ms normalise %.1f prefix %.1f bitmask %.1f "
            "spec %.1f true %.1f emit %.1f rest %.1f\n", call, ndm, a.nchunks, ph[0], ph[1], ph[2], ph[3], ph[4], ph[5], ph[6]);
    for (int k = 0; k < 6 && top[k] >= 0; k++) {
        const uint32_t* r = h + top[k] * kSpStats;
        fprintf(stderr, "  wg dm %lld ch %lld: %.3f ms (phases %.3f %.3f %.3f %.3f %.3f %.3f) hits %u steps %u batches %u "
                "true %u ballots %u merges %u slowest spec w %u %.3f ms\n", (long long)(top[k] / a.nchunks),
                (long long)(top[k] % a.nchunks), r[6] * 1e-5, r[0] * 1e-5, (r[1] - r[0]) * 1e-5, (r[2] - r[1]) * 1e-5,
                (r[3] - r[2]) * 1e-5, (r[4] - r[3]) * 1e-5, (r[5] - r[4]) * 1e-5, r[11], r[7], r[8], r[9], r[10], r[12],
                r[13], r[14] * 1e-5);
    }
    call++;
    free(h);
    return hipSuccess;
}

}  // namespace hd
