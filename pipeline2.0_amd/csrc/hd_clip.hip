// hd_clip.hip — PRESTO's time-domain clipping (clip_times) of the raw block on the device,
// and the exact stage-1 fixup of the outputs it changes.
//
// prepsubband runs clip_times (clipping.c [PRESTO-ext]) on every raw read block (one
// PSRFITS subint of blk spectra) that is not fully masked, in order, with state carried
// from block to block; the reference's stage-1 command (PALFA2_presto_search.py:506-511)
// leaves its default -clip 6 on.  Per block b:
//   zdm[t]      = channel-order float fold of the decoded (unmasked) spectrum      k_clip_zdm
//   med         = element (nb-1)/2 of the sorted zdm of the block                   k_clip_block
//   good[t]     = 0.7*med < zdm[t] < 1.3*med; numgood
//   avg, std    = avg_var (AS 52, double) over the good zdm in time order          k_clip_as52
//   chansum[c]  = sum over good t of X[t][c] in time order (double)                 k_clip_chan
//   running avg / std / channel levels over BLOCKSTOAVG = 30 blocks, serial          k_clip_recur
//   clipped[t]  = |zdm[t] - running_avg| > clip_sigma * running_std                 k_clip_flag
// The running channel levels become the pad values (good_chan_levels) of the block and of
// every later block until the next clip; clipped spectra read as those levels.
// Everything but the serial recurrence is data-parallel over spectra, blocks or channels;
// the recurrence is one workgroup walking the blocks with a thread per channel.  All float
// steps follow the C expressions' types and order (no FP contraction), so the statistics
// are bit-identical to the oracle's restatement.
#include "hd_device.h"

#include <algorithm>

namespace hd {

constexpr int kClipMaxBlock = 8192;           // LDS sort capacity (32 KiB of floats)
constexpr int kBlocksToAvg = 30;

int clip_max_block() { return kClipMaxBlock; }

// ---- zero-DM series ----------------------------------------------------------------
// Integer data without calibration: the float fold of <= 2^24 integers is exact in any
// order, so a wave sums a spectrum's bytes with dot products (16 bytes per lane per load).
__global__ __launch_bounds__(256) void k_clip_zdm_u8(RawDesc rd, float* __restrict__ zdm)
{
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= rd.N) return;
    const uint8_t* row = rd.raw + t * rd.rowbytes;
    uint32_t acc = 0;
    for (int o = lane * 16; o < rd.rowbytes; o += 1024) {
        const uint4 v = *(const uint4*)(row + o);
        acc = __builtin_amdgcn_udot4(v.x, 0x01010101u, acc, false);
        acc = __builtin_amdgcn_udot4(v.y, 0x01010101u, acc, false);
        acc = __builtin_amdgcn_udot4(v.z, 0x01010101u, acc, false);
        acc = __builtin_amdgcn_udot4(v.w, 0x01010101u, acc, false);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
    if (lane == 0) zdm[t] = (float)acc;
}

// 4-bit data without calibration: the same with the low and high nibbles of every byte.
__global__ __launch_bounds__(256) void k_clip_zdm_u4(RawDesc rd, float* __restrict__ zdm)
{
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= rd.N) return;
    const uint8_t* row = rd.raw + t * rd.rowbytes;
    uint32_t acc = 0;
    for (int o = lane * 16; o < rd.rowbytes; o += 1024) {
        const uint4 v = *(const uint4*)(row + o);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            acc = __builtin_amdgcn_udot4(w[i] & 0x0F0F0F0Fu, 0x01010101u, acc, false);
            acc = __builtin_amdgcn_udot4((w[i] >> 4) & 0x0F0F0F0Fu, 0x01010101u, acc, false);
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
    if (lane == 0) zdm[t] = (float)acc;
}

// The two int16 samples of a raw dword (low half first), either byte order.
__device__ __forceinline__ void s16_pair(uint32_t w, bool be16, int& lo, int& hi)
{
    if (be16) w = __builtin_amdgcn_perm(0u, w, 0x02030001u);   // swap the bytes of each half
    lo = (int)(int16_t)(w & 0xFFFFu);
    hi = (int)(int16_t)(w >> 16);
}

// 16-bit data without calibration: a wave sums a spectrum's int16 samples as integers (8
// per lane per 16-byte load) together with their magnitudes; when the magnitudes stay under
// 2^24 no partial sum of the channel-order float fold can round, so the integer is that fold
// exactly -- otherwise lane 0 folds the spectrum in channel order as the general kernel does.
__global__ __launch_bounds__(256) void k_clip_zdm_u16(RawDesc rd, float* __restrict__ zdm)
{
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= rd.N) return;
    const uint8_t* row = rd.raw + t * rd.rowbytes;
    int acc = 0, mag = 0;
    for (int o = lane * 16; o < rd.rowbytes; o += 1024) {
        const uint4 v = *(const uint4*)(row + o);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            int lo, hi;
            s16_pair(w[i], rd.be16, lo, hi);
            acc += lo + hi;
            mag += abs(lo) + abs(hi);
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        acc += __shfl_xor(acc, m, 64);
        mag += __shfl_xor(mag, m, 64);
    }
    if (lane == 0) {
        if (mag < (1 << 24)) {
            zdm[t] = (float)acc;
        } else {
            float z = 0.0f;
            for (int c = 0; c < rd.nchan; c++) z += raw_value(rd, t, c);
            zdm[t] = z;
        }
    }
}

// General data: one thread per spectrum folds its channels in ascending-frequency order.
__global__ __launch_bounds__(256) void k_clip_zdm(RawDesc rd, float* __restrict__ zdm)
{
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= rd.N) return;
    float z = 0.0f;
    for (int c = 0; c < rd.nchan; c++) z += raw_value(rd, t, c);
    zdm[t] = z;
}

// ---- per block: median, good points -----------------------------------------------
__global__ __launch_bounds__(1024) void k_clip_block(ClipArgs a)
{
    __shared__ float v[kClipMaxBlock];
    __shared__ int cnt;
    const int b = blockIdx.x;
    const int64_t t0 = (int64_t)b * a.rd.blk;
    const int nb = (int)min((int64_t)a.rd.blk, a.rd.N - t0);
    if (threadIdx.x == 0) cnt = 0;
    int n2 = 1;
    while (n2 < nb) n2 <<= 1;
    for (int i = threadIdx.x; i < n2; i += blockDim.x) v[i] = i < nb ? a.zdm[t0 + i] : __builtin_inff();
    __syncthreads();
    // bitonic sort of n2 floats (ascending)
    for (int k = 2; k <= n2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n2; i += blockDim.x) {
                const int l = i ^ j;
                if (l > i) {
                    const float x = v[i], y = v[l];
                    const bool up = (i & k) == 0;
                    if (up ? x > y : x < y) {
                        v[i] = y;
                        v[l] = x;
                    }
                }
            }
            __syncthreads();
        }
    const float med = v[(nb - 1) / 2];
    const float lo = (float)(0.7 * (double)med), hi = (float)(1.3 * (double)med);
    int mine = 0;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) {
        const float z = a.zdm[t0 + i];
        const uint8_t g = z > lo && z < hi;
        a.good[t0 + i] = g;
        mine += g;
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) mine += __shfl_xor(mine, m, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&cnt, mine);
    __syncthreads();
    if (threadIdx.x == 0) a.numgood[b] = cnt;
}

// ---- per block: avg_var over the good points, in time order (one thread per block) --
__global__ __launch_bounds__(64) void k_clip_as52(ClipArgs a)
{
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= a.rd.nblk) return;
    const int64_t t0 = (int64_t)b * a.rd.blk;
    const int nb = (int)min((int64_t)a.rd.blk, a.rd.N - t0);
    double mean = 0.0, var = 0.0, an1 = 0.0;
    int i = 0;
    for (int k = 0; k < nb; k++) {
        if (!a.good[t0 + k]) continue;
        const double x = (double)a.zdm[t0 + k];
        if (i == 0) {
            mean = x;
        } else {
            const double an = (double)(i + 1);
            an1 = (double)i;
            const double dx = (x - mean) / an;
            var += an * an1 * dx * dx;
            mean += dx;
        }
        i++;
    }
    if (i > 1) var /= an1;
    a.bavg[b] = mean;
    a.bstd[b] = sqrt(var);
}

// ---- per (block, channel): sum of the good spectra, in time order -------------------
// Lanes are consecutive channels of one block, so every spectrum is one coalesced read.
__global__ __launch_bounds__(256) void k_clip_chan(ClipArgs a)
{
    const int nch = a.rd.nchan;
    const int cblocks = (nch + 255) / 256;
    const int b = blockIdx.x / cblocks;
    const int c = (blockIdx.x - b * cblocks) * 256 + threadIdx.x;
    if (c >= nch) return;
    const int64_t t0 = (int64_t)b * a.rd.blk;
    const int nb = (int)min((int64_t)a.rd.blk, a.rd.N - t0);
    double acc = 0.0;
    for (int k = 0; k < nb; k++)
        if (a.good[t0 + k]) acc += (double)raw_value(a.rd, t0 + k, c);
    a.chansum[(int64_t)b * nch + c] = acc;
}

// 8-bit data without calibration: the sums are of integers (exact in any order), so a lane
// keeps four channels' byte sums in integers over dword loads, 8 spectra in flight, with the
// block's good flags staged in LDS; the exact integer is the double the fold would give.
__global__ __launch_bounds__(256) void k_clip_chan_u8(ClipArgs a)
{
    __shared__ uint8_t g[kClipMaxBlock];
    const int nch = a.rd.nchan;
    const int b = blockIdx.x;
    const int64_t t0 = (int64_t)b * a.rd.blk;
    const int nb = (int)min((int64_t)a.rd.blk, a.rd.N - t0);
    for (int i = threadIdx.x; i < nb; i += blockDim.x) g[i] = a.good[t0 + i];
    __syncthreads();
    const int nq = a.rd.rowbytes >> 2;                  // channel quads per spectrum
    for (int q = threadIdx.x; q < nq; q += blockDim.x) {
        uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        const uint8_t* base = a.rd.raw + t0 * a.rd.rowbytes + 4 * q;
        int k = 0;
        for (; k + 8 <= nb; k += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = g[k + u] ? *(const uint32_t*)(base + (int64_t)(k + u) * a.rd.rowbytes) : 0u;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                s0 += v[u] & 0xFFu;
                s1 += (v[u] >> 8) & 0xFFu;
                s2 += (v[u] >> 16) & 0xFFu;
                s3 += v[u] >> 24;
            }
        }
        for (; k < nb; k++) {
            const uint32_t v = g[k] ? *(const uint32_t*)(base + (int64_t)k * a.rd.rowbytes) : 0u;
            s0 += v & 0xFFu;
            s1 += (v >> 8) & 0xFFu;
            s2 += (v >> 16) & 0xFFu;
            s3 += v >> 24;
        }
        const uint32_t sv[4] = {s0, s1, s2, s3};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int rc = 4 * q + i;                   // raw channel -> ascending channel
            const int c = a.rd.flip ? nch - 1 - rc : rc;
            a.chansum[(int64_t)b * nch + c] = (double)sv[i];
        }
    }
}

// 4-bit data without calibration: a lane keeps the eight nibble sums of one raw dword
// (file channels 8q .. 8q+7; channel 2i+j is the first (j = 0) or second nibble of byte i,
// first = high nibble when nibble_hi_first) over the block's good spectra.
__global__ __launch_bounds__(256) void k_clip_chan_u4(ClipArgs a)
{
    __shared__ uint8_t g[kClipMaxBlock];
    const int nch = a.rd.nchan;
    const int b = blockIdx.x;
    const int64_t t0 = (int64_t)b * a.rd.blk;
    const int nb = (int)min((int64_t)a.rd.blk, a.rd.N - t0);
    for (int i = threadIdx.x; i < nb; i += blockDim.x) g[i] = a.good[t0 + i];
    __syncthreads();
    const int nq = a.rd.rowbytes >> 2;                  // 8-channel dwords per spectrum
    for (int q = threadIdx.x; q < nq; q += blockDim.x) {
        uint32_t sh[4] = {0, 0, 0, 0}, sl[4] = {0, 0, 0, 0};   // high / low nibble sums of byte i
        const uint8_t* base = a.rd.raw + t0 * a.rd.rowbytes + 4 * q;
        int k = 0;
        for (; k + 8 <= nb; k += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = g[k + u] ? *(const uint32_t*)(base + (int64_t)(k + u) * a.rd.rowbytes) : 0u;
#pragma unroll
            for (int u = 0; u < 8; u++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    sl[i] += (v[u] >> (8 * i)) & 15u;
                    sh[i] += (v[u] >> (8 * i + 4)) & 15u;
                }
        }
        for (; k < nb; k++) {
            const uint32_t v = g[k] ? *(const uint32_t*)(base + (int64_t)k * a.rd.rowbytes) : 0u;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                sl[i] += (v >> (8 * i)) & 15u;
                sh[i] += (v >> (8 * i + 4)) & 15u;
            }
        }
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int rc = 8 * q + 2 * i + j;       // raw channel -> ascending channel
                const int c = a.rd.flip ? nch - 1 - rc : rc;
                const bool hi = a.rd.nibble_hi_first ? j == 0 : j == 1;
                a.chansum[(int64_t)b * nch + c] = (double)(hi ? sh[i] : sl[i]);
            }
    }
}

// 16-bit data without calibration: a lane keeps the two int16 channels of one raw dword
// over the block's good spectra (|sum| <= 8192 * 32768 < 2^31), exact like the double fold.
__global__ __launch_bounds__(256) void k_clip_chan_u16(ClipArgs a)
{
    __shared__ uint8_t g[kClipMaxBlock];
    const int nch = a.rd.nchan;
    const int b = blockIdx.x;
    const int64_t t0 = (int64_t)b * a.rd.blk;
    const int nb = (int)min((int64_t)a.rd.blk, a.rd.N - t0);
    for (int i = threadIdx.x; i < nb; i += blockDim.x) g[i] = a.good[t0 + i];
    __syncthreads();
    const int nq = a.rd.rowbytes >> 2;                  // channel pairs per spectrum
    const bool be = a.rd.be16;
    for (int q = threadIdx.x; q < nq; q += blockDim.x) {
        int s0 = 0, s1 = 0;
        const uint8_t* base = a.rd.raw + t0 * a.rd.rowbytes + 4 * q;
        int k = 0;
        for (; k + 8 <= nb; k += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = g[k + u] ? *(const uint32_t*)(base + (int64_t)(k + u) * a.rd.rowbytes) : 0u;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                int lo, hi;
                s16_pair(v[u], be, lo, hi);
                s0 += lo;
                s1 += hi;
            }
        }
        for (; k < nb; k++) {
            const uint32_t v = g[k] ? *(const uint32_t*)(base + (int64_t)k * a.rd.rowbytes) : 0u;
            int lo, hi;
            s16_pair(v, be, lo, hi);
            s0 += lo;
            s1 += hi;
        }
        const int sv[2] = {s0, s1};
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int rc = 2 * q + i;                   // raw channel -> ascending channel
            const int c = a.rd.flip ? nch - 1 - rc : rc;
            a.chansum[(int64_t)b * nch + c] = (double)sv[i];
        }
    }
}

// ---- the serial recurrence over blocks (one workgroup, thread = channel) -------------
// One thread per channel, spread over single-wave workgroups on as many CUs: the recurrence
// is serial over blocks and issue-bound in double precision, so one 1024-thread workgroup on
// one CU ran it 16 waves deep on 4 SIMDs.  Every thread carries the (channel-independent)
// running avg / std itself; thread 0 of workgroup 0 publishes them.  The per-block scalars
// are staged in LDS per segment and only the channel sums are global loads (16 blocks
// ahead): 0.85 ms per C2 beam against 2.25 with every input a global load 8 blocks ahead.
constexpr int kRecurSeg = 1024;               // blocks of per-block scalars staged in LDS at a time

__global__ __launch_bounds__(64) void k_clip_recur(ClipArgs a)
{
    // the per-block scalars (numgood, block avg / std, all-zapped) of kRecurSeg blocks at a
    // time in LDS: the chain then reads them at LDS latency; the per-channel sums are the only
    // global loads, U blocks ahead in registers
    __shared__ double s_bav[kRecurSeg], s_bsd[kRecurSeg];
    __shared__ int s_ng[kRecurSeg];
    __shared__ uint8_t s_az[kRecurSeg];
    const int nch = a.rd.nchan;
    const int nblk = a.rd.nblk;
    const float clip_sigma = a.clip_sigma;
    const int nloop = nch > 0 ? nch : 1;
    constexpr int U = 16;                               // chansum loads in flight per thread
    static_assert(kRecurSeg % U == 0, "segment of whole prefetch groups");
    for (int c0 = blockIdx.x * blockDim.x; c0 < nloop; c0 += gridDim.x * blockDim.x) {
        const int c = c0 + threadIdx.x;
        const bool own = c < nch;
        float ravg = 0.0f, rstd = 0.0f, cra = 0.0f;
        float lev = own && a.padvals0 ? a.padvals0[c] : 0.0f;
        int nread = 0;
        double ncsv[U];
        auto fetch = [&](int b0) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int b = min(b0 + u, nblk - 1);
                ncsv[u] = own ? a.chansum[(int64_t)b * nch + c] : 0.0;
            }
        };
        fetch(0);
        for (int s0 = 0; s0 < nblk; s0 += kRecurSeg) {
            const int ns = min(kRecurSeg, nblk - s0);
            __syncthreads();                              // the previous segment is consumed
            for (int i = threadIdx.x; i < ns; i += blockDim.x) {
                s_bav[i] = a.bavg[s0 + i];
                s_bsd[i] = a.bstd[s0 + i];
                s_ng[i] = a.numgood[s0 + i];
                s_az[i] = a.allzap ? a.allzap[s0 + i] : 0;
            }
            __syncthreads();
            for (int g0 = 0; g0 < ns; g0 += U) {
                double csv[U];
#pragma unroll
                for (int u = 0; u < U; u++) csv[u] = ncsv[u];
                if (s0 + g0 + U < nblk) fetch(s0 + g0 + U);
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int bl = g0 + u, b = s0 + bl;
                    if (bl >= ns) continue;                      // (the segment's last group)
                    const bool run = clip_sigma > 0.0f && !s_az[bl];
                    if (run) {
                        const int ng = s_ng[bl];
                        double cur_avg, cur_std, cat;
                        if (ng < 1) {
                            cur_avg = (double)ravg;
                            cur_std = (double)rstd;
                            cat = (double)cra;
                        } else {
                            cur_avg = s_bav[bl];
                            cur_std = s_bsd[bl];
                            cat = csv[u] / (double)ng;
                        }
                        if (nread) {
                            const float r29 = ravg * (float)(kBlocksToAvg - 1);
                            const float s29 = rstd * (float)(kBlocksToAvg - 1);
                            const float c29 = cra * (float)(kBlocksToAvg - 1);
                            ravg = (float)(((double)r29 + cur_avg) / (double)kBlocksToAvg);
                            rstd = (float)(((double)s29 + cur_std) / (double)kBlocksToAvg);
                            cra = (float)(((double)c29 + cat) / (double)kBlocksToAvg);
                        } else {
                            ravg = (float)cur_avg;
                            rstd = (float)cur_std;
                            cra = (float)cat;
                        }
                        lev = cra;
                        nread++;
                    }
                    if (c0 == 0 && threadIdx.x == 0) {          // workgroup 0, thread 0
                        a.doclip[b] = run;
                        a.ravg[b] = ravg;
                        a.trig[b] = clip_sigma * rstd;
                    }
                    if (own) a.pad[(int64_t)b * nch + c] = lev;
                }
            }
        }
    }
}

// ---- clip flags + the event list -------------------------------------------------------
__global__ __launch_bounds__(256) void k_clip_flag(ClipArgs a)
{
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool clip = false;
    if (t < a.rd.N) {
        const int64_t b = blk_of(a.rd, t);
        clip = a.doclip[b] && fabsf(a.zdm[t] - a.ravg[b]) > a.trig[b];
        a.clipped[t] = clip;
    }
    // bit-packed flags (a wave covers 64 rows from a multiple of 64), then a wave-aggregated append
    const uint64_t bal = __ballot(clip);
    const int lane = threadIdx.x & 63;
    if (lane == 0 && t < a.rd.N) *(uint2*)(a.clipbits + (t >> 5)) = make_uint2((uint32_t)bal, (uint32_t)(bal >> 32));
    if (bal) {
        int base = 0;
        if (lane == __ffsll((unsigned long long)bal) - 1) base = atomicAdd(a.nevents, __popcll(bal));
        base = __shfl(base, __ffsll((unsigned long long)bal) - 1, 64);
        if (clip) a.events[base + __popcll(bal & ((1ull << lane) - 1))] = (int32_t)t;
    }
}

// ---- time-sliced contexts: per-block statistics in and out ----------------------------
// Row b of the exchange layout: [bavg, bstd, numgood, chansum[nchan]] (doubles; numgood and
// the 8-bit channel sums are exact integers).
__global__ __launch_bounds__(256) void k_clip_pack(ClipArgs a, double* __restrict__ out, int nown)
{
    const int nch = a.rd.nchan, w = nch + 3;
    const int64_t n = (int64_t)nown * w;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int b = (int)(i / w), k = (int)(i - (int64_t)b * w);
        out[i] = k == 0 ? a.bavg[b] : k == 1 ? a.bstd[b] : k == 2 ? (double)a.numgood[b]
                                                                  : a.chansum[(int64_t)b * nch + k - 3];
    }
}

__global__ __launch_bounds__(256) void k_clip_unpack(ClipArgs g, const double* __restrict__ in)
{
    const int nch = g.rd.nchan, w = nch + 3;
    const int64_t n = (int64_t)g.rd.nblk * w;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int b = (int)(i / w), k = (int)(i - (int64_t)b * w);
        const double v = in[i];
        if (k == 0) g.bavg[b] = v;
        else if (k == 1) g.bstd[b] = v;
        else if (k == 2) g.numgood[b] = (int32_t)v;
        else g.chansum[(int64_t)b * nch + k - 3] = v;
    }
}

static unsigned grid_for(int64_t n)
{
    int64_t nb = (n + 255) / 256;
    return (unsigned)(nb < 1 ? 1 : nb > 4096 ? 4096 : nb);
}

hipError_t launch_clip_pack(const ClipArgs& a, double* out, int nown, hipStream_t st)
{
    if (nown <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_clip_pack, dim3(grid_for((int64_t)nown * (a.rd.nchan + 3))), dim3(256), 0, st, a, out, nown);
    return hipGetLastError();
}

hipError_t launch_clip_unpack(const ClipArgs& g, const double* in, hipStream_t st)
{
    hipLaunchKernelGGL(k_clip_unpack, dim3(grid_for((int64_t)g.rd.nblk * (g.rd.nchan + 3))), dim3(256), 0, st, g, in);
    return hipGetLastError();
}

// the serial recurrence over a.rd.nblk blocks (a's arrays), one wave per 64 channels
hipError_t launch_clip_recur(const ClipArgs& a, hipStream_t st)
{
    const unsigned g = (unsigned)std::max(1, (a.rd.nchan + 63) / 64);
    hipLaunchKernelGGL(k_clip_recur, dim3(g), dim3(64), 0, st, a);
    return hipGetLastError();
}

// clip flags + event list of a's spectra (doclip/ravg/trig indexed by a's blocks)
hipError_t launch_clip_flag(const ClipArgs& a, hipStream_t st)
{
    hipError_t e = hipMemsetAsync(a.nevents, 0, sizeof(int32_t), st);
    if (e != hipSuccess) return e;
    if (a.rd.N <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_clip_flag, dim3((unsigned)((a.rd.N + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError();
}

// per-block statistics of a's spectra (everything before the recurrence)
hipError_t launch_clip_stats(const ClipArgs& a, hipStream_t st, hipEvent_t after_stats)
{
    const RawDesc& rd = a.rd;
    if (rd.N <= 0) return hipSuccess;
    if (rd.blk > kClipMaxBlock) return hipErrorInvalidValue;
    const bool calib = rd.scl || rd.offs || rd.wts;
    if (rd.nbits == 8 && !calib && rd.rowbytes % 16 == 0)
        hipLaunchKernelGGL(k_clip_zdm_u8, dim3((unsigned)((rd.N + 3) / 4)), dim3(256), 0, st, rd, a.zdm);
    else if (rd.nbits == 4 && !calib && rd.rowbytes % 16 == 0)
        hipLaunchKernelGGL(k_clip_zdm_u4, dim3((unsigned)((rd.N + 3) / 4)), dim3(256), 0, st, rd, a.zdm);
    else if (rd.nbits == 16 && !calib && rd.rowbytes % 16 == 0 && rd.blk <= kClipMaxBlock)
        hipLaunchKernelGGL(k_clip_zdm_u16, dim3((unsigned)((rd.N + 3) / 4)), dim3(256), 0, st, rd, a.zdm);
    else
        hipLaunchKernelGGL(k_clip_zdm, dim3((unsigned)((rd.N + 255) / 256)), dim3(256), 0, st, rd, a.zdm);
    // the channel-major copy forks after the channel sums (beside the recurrence); forking it
    // here instead (HD_FORK_EARLY=1), beside the block medians, AS-52 and channel sums too,
    // measured 79.9 vs 78.8 ms per C2 beam: it competes with the channel sums' raw scan
    const bool late = !(getenv("HD_FORK_EARLY") && atoi(getenv("HD_FORK_EARLY")) != 0);
    if (after_stats && !late) {
        const hipError_t e = hipEventRecord(after_stats, st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_clip_block, dim3((unsigned)rd.nblk), dim3(1024), 0, st, a);
    hipLaunchKernelGGL(k_clip_as52, dim3((unsigned)((rd.nblk + 63) / 64)), dim3(64), 0, st, a);
    if (rd.nbits == 8 && !calib && rd.rowbytes % 4 == 0)
        hipLaunchKernelGGL(k_clip_chan_u8, dim3((unsigned)rd.nblk), dim3(256), 0, st, a);
    else if (rd.nbits == 4 && !calib && rd.rowbytes % 4 == 0)
        hipLaunchKernelGGL(k_clip_chan_u4, dim3((unsigned)rd.nblk), dim3(256), 0, st, a);
    else if (rd.nbits == 16 && !calib && rd.rowbytes % 4 == 0)
        hipLaunchKernelGGL(k_clip_chan_u16, dim3((unsigned)rd.nblk), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(k_clip_chan, dim3((unsigned)(rd.nblk * ((rd.nchan + 255) / 256))), dim3(256), 0, st, a);
    if (after_stats && late) {  // the full-chip raw scans are done; the serial recurrence follows
        const hipError_t e = hipEventRecord(after_stats, st);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

hipError_t launch_clip(const ClipArgs& a, hipStream_t st, hipEvent_t after_stats)
{
    if (a.rd.N <= 0) return hipMemsetAsync(a.nevents, 0, sizeof(int32_t), st);
    hipError_t e = launch_clip_stats(a, st, after_stats);
    if (e == hipSuccess) e = launch_clip_recur(a, st);
    if (e == hipSuccess) e = launch_clip_flag(a, st);
    return e;
}

// ------------------------------------------------------------------------------------
// stage-1 fixup
// ------------------------------------------------------------------------------------
// One workgroup per event e, over the launch's passes: the zap rows and pad rows of the (at
// most two) read blocks the event's rows fall in, and each pass's channel delays in turn,
// are staged in LDS.
//  * e < nev: the clipped spectrum r = events[e].  Channel c of subband s reads spectrum r
//    for exactly one output, j = floor((r - d_c) / ds); those outputs (one per distinct j
//    in the subband) are recomputed: at most cps per subband, usually far fewer.
//  * e >= nev (only when `boundaries`): the read-block boundary r = (e - nev + 1) * blk.
//    In subbands with a channel masked in both blocks whose pad values differ, the outputs
//    whose rows contain both r - 1 and r mix the two blocks' pads, which the integer path's
//    per-block constants do not cover; they are recomputed (every other subband was exact).
// Recomputation is the exact per-cell fold of k_stage1_direct; overlapping events write
// identical values.  Index arithmetic is 32-bit (the host checks N < 2^31).

struct FixCtx {
    const int* dly;          // LDS: delays of the pass
    const uint8_t* zap2;     // LDS: [2][nchan] zap rows of blocks b0, b0 + 1
    const float* pad2;       // LDS: [2][nchan] pad rows of blocks b0, b0 + 1
    int b0;                  // first block staged
    int bnd;                 // first spectrum of block b0 + 1
    int lo, hi;              // spectra [lo, hi) are inside the staged blocks
};

__device__ __forceinline__ float fix_cell(const RawDesc& rd, const FixCtx& f, int t, int c)
{
    if (t < f.lo || t >= f.hi) return chan_value(rd, t, c);      // outside the staged blocks
    const int part = t >= f.bnd;
    const bool repl = (rd.clipped && rd.clipped[t]) || f.zap2[part * rd.nchan + c];
    return repl ? f.pad2[part * rd.nchan + c] : raw_value(rd, t, c);
}

// One output (s, j), exactly.  The cells of a k-step are gathered with their loads issued
// together (16 channels at a time, no data-dependent branch between them): a dependent
// chain of one latency per cell would dominate the fixup.
__device__ __forceinline__ int fix_one(const Stage1Multi& a, const FixCtx& f, int p, int s, int j)
{
    const RawDesc& rd = a.rd;
    const int ds = a.ds, cps = a.cps, nch = rd.nchan;
    const bool fast = rd.nbits == 8 && !rd.scl && !rd.offs && !rd.wts;
    float acc = 0.0f;
    for (int k = 0; k < ds; k++) {
        float sk = 0.0f;
        const int tb = j * ds + k;
        for (int c0 = 0; c0 < cps; c0 += 8) {
            float x[8];
            if (fast) {
                uint32_t b[8], cf[8];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int cc = min(c0 + i, cps - 1);
                    const int c = s * cps + cc;
                    const int t = tb + f.dly[c];
                    const int tt = min(t, (int)rd.N - 1);
                    b[i] = rd.raw[(int64_t)tt * rd.rowbytes + (rd.flip ? nch - 1 - c : c)];
                    cf[i] = rd.clipped ? rd.clipped[tt] : 0u;
                }
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int cc = min(c0 + i, cps - 1);
                    const int c = s * cps + cc;
                    const int t = tb + f.dly[c];
                    if (t < f.lo || t >= f.hi) {
                        x[i] = chan_value(rd, t, c);
                    } else {
                        const int part = t >= f.bnd;
                        const bool repl = t >= rd.N || cf[i] || f.zap2[part * nch + c];
                        x[i] = repl ? f.pad2[part * nch + c] : (float)b[i];
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int cc = min(c0 + i, cps - 1);
                    x[i] = fix_cell(rd, f, tb + f.dly[s * cps + cc], s * cps + cc);
                }
            }
            const int n = min(8, cps - c0);
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (i < n) sk += x[i];
        }
        acc += sk;
    }
    if (a.ds_mode == 1) acc = acc / (float)ds;
    if (a.sub_dtype == 0) {
        const int16_t q = to_i16(acc, a.sub_round);
        ((int16_t*)a.out[p])[(int64_t)s * a.ostride[p] + j] = q;
        return q < 0 ? -(int)q : (int)q;
    }
    ((float*)a.out[p])[(int64_t)s * a.ostride[p] + j] = acc;
    return 0;
}

__global__ __launch_bounds__(256) void k_stage1_fixup(Stage1Multi a, const int32_t* __restrict__ events,
                                                     const int32_t* __restrict__ nevents, int boundaries)
{
    // dynamic LDS: delays [nchan] | zap rows [2][nchan] | pad rows [2][nchan] | jlo, cnt [nsub+1]
    extern __shared__ __attribute__((aligned(16))) char fsm[];
    const int nchan = a.rd.nchan, nsub = a.nsub;
    int* dly_s = (int*)fsm;
    float* pad_s = (float*)(dly_s + nchan);
    int* jlo_s = (int*)(pad_s + 2 * nchan);
    int* cnt_s = jlo_s + nsub + 1;
    uint8_t* zap_s = (uint8_t*)(cnt_s + nsub + 1);
    __shared__ int amax_s[kMaxPass];
    __shared__ int dmax_s, wsum[8];
    const int nev = *nevents;
    const int nbound = boundaries ? a.rd.nblk - 1 : 0;
    const int nitems = nev + nbound;
    const int ds = a.ds, cps = a.cps;
    const int nds = (int)a.nds;
    // the delays of every pass reach at most dmax rows: stage the blocks of [r - dmax - ds, ...]
    if (threadIdx.x == 0) dmax_s = 0;
    __syncthreads();
    {
        int m = 0;
        for (int p = 0; p < a.npass; p++)
            for (int c = threadIdx.x; c < nchan; c += blockDim.x) m = max(m, a.dly[p][c]);
        m = wave_max_i32(m);
        if ((threadIdx.x & 63) == 0) atomicMax(&dmax_s, m);
    }
    __syncthreads();
    const int dmax = dmax_s;
    for (int e = blockIdx.x; e < nitems; e += gridDim.x) {
        const bool clip_ev = e < nev;
        const int r = clip_ev ? events[e] : (e - nev + 1) * a.rd.blk;
        FixCtx f;
        f.dly = dly_s;
        f.zap2 = zap_s;
        f.pad2 = pad_s;
        const int b0 = (int)blk_of(a.rd, max(r - dmax - ds, 0));
        f.b0 = b0;
        f.bnd = (b0 + 1) * a.rd.blk;
        f.lo = b0 * a.rd.blk;
        f.hi = b0 + 1 < a.rd.nblk ? (int)min((int64_t)(b0 + 2) * a.rd.blk, a.rd.N) : (int)a.rd.N;
        const int b1 = min(b0 + 1, a.rd.nblk - 1);
        __syncthreads();                                  // the previous event is done with LDS
        for (int c = threadIdx.x; c < nchan; c += blockDim.x) {
            zap_s[c] = zap_at(a.rd, b0, c);
            zap_s[nchan + c] = zap_at(a.rd, b1, c);
            pad_s[c] = pad_at(a.rd, b0, c);
            pad_s[nchan + c] = pad_at(a.rd, b1, c);
        }
        if (threadIdx.x < kMaxPass) amax_s[threadIdx.x] = 0;
        for (int p = 0; p < a.npass; p++) {
            __syncthreads();                              // zap/pad staged; previous pass done with dly_s
            for (int c = threadIdx.x; c < nchan; c += blockDim.x) dly_s[c] = a.dly[p][c];
            __syncthreads();
            int amax = 0;
            if (clip_ev) {
                for (int c = threadIdx.x; c < nchan; c += blockDim.x) {
                    const int s = c / cps;
                    const int jn = r - dly_s[c];
                    if (jn < 0) continue;
                    const int j = jn / ds;
                    if (j >= nds) continue;
                    bool dup = false;                     // an earlier channel already names j
                    for (int c2 = s * cps; c2 < c; c2++) {
                        const int jn2 = r - dly_s[c2];
                        dup |= jn2 >= 0 && jn2 / ds == j;
                    }
                    if (!dup) amax = max(amax, fix_one(a, f, p, s, j));
                }
            } else {
                const int bb = e - nev + 1;               // boundary between blocks bb-1 and bb
                const bool staged = bb - b0 == 1;
                int n = 0;
                const int s = threadIdx.x;                // nsub <= blockDim.x (host check)
                if (s < nsub) {
                    int mind = 1 << 30, maxd = 0;
                    bool need = false;
                    for (int cc = 0; cc < cps; cc++) {
                        const int c = s * cps + cc;
                        mind = min(mind, dly_s[c]);
                        maxd = max(maxd, dly_s[c]);
                        if (staged)
                            need |= zap_s[c] && zap_s[nchan + c] && pad_s[c] != pad_s[nchan + c];
                        else
                            need |= zap_at(a.rd, bb - 1, c) && zap_at(a.rd, bb, c) &&
                                    pad_at(a.rd, bb - 1, c) != pad_at(a.rd, bb, c);
                    }
                    int lo = r - (ds - 1) - maxd, hi = r - 1 - mind;
                    lo = lo <= 0 ? 0 : (lo + ds - 1) / ds;   // ceil for lo > 0
                    hi = hi < 0 ? -1 : min(hi / ds, nds - 1);
                    jlo_s[s] = lo;
                    n = need && hi >= lo ? hi - lo + 1 : 0;
                }
                // exclusive scan of the task counts over the workgroup (wave scans + wave sums)
                const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
                int incl = n;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int v = __shfl_up(incl, d, 64);
                    if (lane >= d) incl += v;
                }
                if (lane == 63) wsum[w] = incl;
                __syncthreads();
                int base = 0;
                for (int k = 0; k < w; k++) base += wsum[k];
                int total = 0;
                for (int k = 0; k < (int)(blockDim.x >> 6); k++) total += wsum[k];
                if (s < nsub) cnt_s[s] = base + incl - n;
                __syncthreads();
                for (int t = threadIdx.x; t < total; t += blockDim.x) {
                    int lo = 0, hi = nsub - 1;            // subband of task t: last s with cnt_s[s] <= t
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (cnt_s[mid] <= t) lo = mid;
                        else hi = mid - 1;
                    }
                    amax = max(amax, fix_one(a, f, p, lo, jlo_s[lo] + (t - cnt_s[lo])));
                }
            }
            if (a.sub_dtype == 0) {
                amax = wave_max_i32(amax);
                if ((threadIdx.x & 63) == 0 && amax > 0) atomicMax(&amax_s[p], amax);
            }
        }
        __syncthreads();
        if (a.sub_dtype == 0 && threadIdx.x < a.npass) publish_max(a.maxabs[threadIdx.x], amax_s[threadIdx.x]);
    }
}

size_t fixup_lds_bytes(const Stage1Multi& a)
{
    return (size_t)a.rd.nchan * 4 + (size_t)2 * a.rd.nchan * 4 + (size_t)2 * (a.nsub + 1) * 4 + (size_t)2 * a.rd.nchan;
}

// ------------------------------------------------------------------------------------
// stage-1 fixup, 8-bit data without calibration: LDS windows from the channel-major copy
// ------------------------------------------------------------------------------------
// The items are those of k_stage1_fixup (clipped spectra, then read-block boundaries), but
// a workgroup takes one (item r, chunk of SG subbands) and first copies the raw window every
// output it may recompute reads -- rows [r - dmax - ds + 1, r + dmax + ds) of the chunk's G
// channels, coalesced 16-byte runs of rawT -- into LDS, with the window's replaced-row flags
// (clipped, or past N), the zap/pad rows of its two read blocks and the chunk's delays of
// every pass.  The exact folds then read only LDS: per output cps*ds LDS bytes instead of as
// many scattered global byte loads (plus a clip-flag load each).
// Window bound: an output j that channel c maps r to (j = floor((r - d_c)/ds)) reads rows
// j*ds + k + d_c' >= r - d_c - ds + 1 >= r - dmax - ds + 1 and <= r - d_c + ds - 1 + dmax;
// a boundary output (rows containing r - 1 and r) stays inside the same bounds.  The host
// only takes this kernel when the window is shorter than a read block (<= 2 blocks staged).
struct Fix8Geom {
    int SG, G, Wp;            // subbands per chunk, channels per chunk, LDS bytes per channel row
    int nchunk, jmax;         // chunks per item; boundary outputs per (pass, subband) at most
};

// The oracle's fold of one output (k outer, channel inner, from 0.0f) over the LDS window,
// for compile-time CPS / DS (the channel loop unrolls): the subband's raw delays dr[] and zap
// bits zb come in registers (the callers load them with the task's other LDS reads), and
// every step's flag, raw byte and pad read issue together, so a task waits for two LDS round
// trips -- delays, then window bytes -- instead of two per channel (branches around the loads).
template <int CPS, int DS, bool FLAGS = true>
__device__ __forceinline__ float fix8_fold_pre(const Stage1Multi& a, const uint8_t* lraw, const uint8_t* flg,
                                               const float* pad, int Wp, int G, int lc0, const int (&dr)[CPS],
                                               uint32_t zb, int trel, int bndrel, int dsr)
{
    // FLAGS = false: no replaced row in the item's window (its flag reads skipped).  The
    // subband's pads of both blocks are read once, not once per step
    const int ds = DS ? DS : dsr;
    float pa[CPS], pb[CPS];
#pragma unroll
    for (int cc = 0; cc < CPS; cc++) {
        pa[cc] = pad[lc0 + cc];
        pb[cc] = pad[G + lc0 + cc];
    }
    float acc = 0.0f;
    // (two steps in flight: their channel sums are independent, only acc is a chain)
#pragma unroll 2
    for (int k = 0; k < ds; k++) {
        uint32_t fb[CPS], rb[CPS];
        float pv[CPS];
#pragma unroll
        for (int cc = 0; cc < CPS; cc++) {
            const int lr = trel + dr[cc] + k;
            fb[cc] = FLAGS ? flg[lr] : 0u;
            rb[cc] = lraw[(lc0 + cc) * Wp + lr];
            pv[cc] = lr >= bndrel ? pb[cc] : pa[cc];
        }
        float sk = 0.0f;
#pragma unroll
        for (int cc = 0; cc < CPS; cc++) {
            const int part = trel + dr[cc] + k >= bndrel ? 16 : 0;
            const bool rep = (fb[cc] | ((zb >> (part + cc)) & 1u)) != 0;
            const float x = rep ? pv[cc] : (float)rb[cc];
            sk += x;
        }
        acc += sk;
    }
    if (a.ds_mode == 1) acc = acc / (float)ds;
    return acc;
}

template <int CPS, int DS>
__device__ __forceinline__ float fix8_fold(const Stage1Multi& a, const uint8_t* lraw, const uint8_t* flg,
                                           const uint8_t* zap, const float* pad, const int16_t* dl, int Wp, int G,
                                           int lc0, int trel, int bndrel, int dsr)
{
    // runtime cps / ds (the templated cases take fix8_fold_pre); trel = j*ds - wlo: window row
    // of (k = 0, delay 0); dl: this pass's delays of the chunk
    const int ds = DS ? DS : dsr, cps = CPS ? CPS : a.cps;
    float acc = 0.0f;
    for (int k = 0; k < ds; k++) {
        float sk = 0.0f;
        for (int cc = 0; cc < cps; cc++) {
            const int lc = lc0 + cc;
            const int lr = trel + k + dl[lc];
            const int part = lr >= bndrel;
            const bool rep = flg[lr] | zap[part * G + lc];
            const float x = rep ? pad[part * G + lc] : (float)lraw[lc * Wp + lr];
            sk += x;
        }
        acc += sk;
    }
    if (a.ds_mode == 1) acc = acc / (float)ds;
    return acc;
}

// DS > 0: compile-time ds; 0: a.ds; -1: per pass (a.pds[p], the fused k_stage1_q8m launch's
// passes of several DDplan stages: one window per item, of the widest stage)
// k_stage1_fix8's window of an item: the chunk's channels' raw bytes (16-byte runs of the
// channel-major copy) and the rows' replaced flags (clipped, or past N)
__device__ __forceinline__ void fix8_window(const Stage1Multi& a, uint8_t* lraw, uint8_t* flg, int G, int Wp, int c0,
                                            int wlo, int N, int nchan, int fprobe, int& anyflag)
{
    if (fprobe & 2) return;
    const int nq = Wp >> 4;
    for (int i = threadIdx.x; i < G * nq; i += blockDim.x) {
        const int lc = i / nq, q = i - lc * nq;
        const int c = c0 + lc;
        const int rc = a.rd.flip ? nchan - 1 - c : c;
        const uint4 v = *(const uint4*)(a.rawT + (int64_t)rc * a.tstride + wlo + 16 * q);
        *(uint4*)(lraw + lc * Wp + 16 * q) = v;
    }
    int fl = 0;
    for (int i = threadIdx.x; i < Wp; i += blockDim.x) {
        const int t = wlo + i;
        flg[i] = t >= N ? 1 : (a.rd.clipped ? a.rd.clipped[t] : 0);
        fl |= flg[i];
    }
    if (__ballot(fl != 0) && (threadIdx.x & 63) == 0) anyflag = 1;
}

// Task i = (pass p, chunk channel lc) of a clipped spectrum r: its output j, unless an earlier
// channel of the subband maps r to the same output.  Delays fall with frequency within a
// subband, so the outputs its channels map r to rise with the channel and equal ones are
// adjacent: only channel lc - 1 can name j first.
__device__ __forceinline__ bool fix8_task(const int16_t* dly, int i, int G, int cps, int DST, int SG, int r, int N,
                                          int nds, int DSt, const int* pds_s, int ds, int& j)
{
    const int p = i / G, lc = i - p * G;
    const int lc0 = lc - lc % cps;
    const int16_t* dl = dly + (p * SG + lc0 / cps) * DST - lc0;          // dl[lc0 .. lc0 + cps)
    const int dsp = DSt > 0 ? DSt : DSt == 0 ? ds : pds_s[p];
    const int ndsp = DSt < 0 ? N / dsp : nds;
    const int jn = r - dl[lc];
    if (jn < 0) return false;
    j = jn / dsp;
    if (j >= ndsp) return false;
    if (lc > lc0) {
        const int jn2 = r - dl[lc - 1];
        if (jn2 >= 0 && jn2 / dsp == j) return false;
    }
    return true;
}

template <int CPS, int DS>
__global__ __launch_bounds__(256) void k_stage1_fix8(Stage1Multi a, Fix8Geom gm, const int32_t* __restrict__ events,
                                                    const int32_t* __restrict__ nevents, int boundaries)
{
    // dynamic LDS: raw [G][Wp] | flags [Wp] | zap [2][G] | pad [2][G] f32 | dly [npass][SG][DST] i16
    //              | lo, cnt [npass][SG] (boundary items)
    extern __shared__ __attribute__((aligned(16))) char fsm[];
    const int G = gm.G, Wp = gm.Wp, SG = gm.SG, npass = a.npass;
    const int cps = CPS ? CPS : a.cps, ds = DS > 0 ? DS : a.ds;   // (DS -1: the largest pass ds)
    uint8_t* lraw = (uint8_t*)fsm;
    uint8_t* flg = lraw + G * Wp;
    float* pad = (float*)(flg + Wp);                      // Wp is a multiple of 16
    uint8_t* zap = (uint8_t*)(pad + 2 * G);
    // a subband's delays start on a 32-byte boundary (DST = 16 slots for the templated cps):
    // packed 20-byte groups made the compiler's merged ds_read_b128 of a task's 10 delays
    // misaligned (SQ_LDS_UNALIGNED_STALL); the runtime-cps kernel keeps the dense layout
    constexpr int DSTC = CPS > 0 ? 16 : 0;
    const int DST = CPS > 0 ? DSTC : cps;
    int16_t* dly = (int16_t*)(zap + ((2 * G + 15) & ~15));
    auto dix = [&](int p, int lc) { return (p * SG + lc / cps) * DST + lc % cps; };
    int* lo_s = (int*)(dly + ((npass * SG * DST + 7) & ~7));
    int* cnt_s = lo_s + npass * SG;
    int* pre_s = cnt_s + npass * SG;                       // [npass * SG + 1] exclusive prefix of cnt_s
    uint16_t* tlist = (uint16_t*)(pre_s + npass * SG + 1);   // [npass * G] clipped-spectrum tasks to fold
    __shared__ int amax_s[kMaxPass];
    __shared__ int needany, anyflag;
    __shared__ int ntask2[2];                             // clipped-spectrum task counts, by item parity
    __shared__ int wsum_s[8];
    __shared__ uint32_t zbm_s[CPS > 0 ? 1024 / (CPS > 0 ? CPS : 1) : 1];   // per subband: zap bits of both blocks
    // per-pass output rows staged once: indexing the kernel argument arrays with a per-lane
    // pass made every task wait for two global loads of the argument block before its store
    __shared__ char* outp_s[kMaxPass];
    __shared__ int64_t ostr_s[kMaxPass];
    __shared__ int pds_s[kMaxPass];
    if (threadIdx.x < npass) {
        outp_s[threadIdx.x] = (char*)a.out[threadIdx.x];
        ostr_s[threadIdx.x] = a.ostride[threadIdx.x];
        pds_s[threadIdx.x] = DS < 0 ? a.pds[threadIdx.x] : ds;
    }
    // a pass's ds and output count
    auto pds = [&](int p) { return DS > 0 ? DS : DS == 0 ? ds : pds_s[p]; };
    const int fprobe = boundaries >> 8;                   // HD_FIX8_PROBE (profiling): 1 no folds, 2 no window
    boundaries &= 1;
    const int nev = *nevents;
    // the grid is a multiple of nchunk: a workgroup keeps one chunk, so its delays of every
    // pass are staged once for all its items
    const int chunk = blockIdx.x % gm.nchunk;
    // boundary items: the host's list of this chunk's boundaries with a channel zapped on both
    // sides (the only ones whose outputs can change), else every boundary
    const bool blist = boundaries && a.fix_blist && a.fix_G == G;
    const int bofs0 = blist ? a.fix_bofs[chunk] : 0;
    const int nbound = !boundaries ? 0 : blist ? a.fix_bofs[chunk + 1] - bofs0 : a.rd.nblk - 1;
    const int nitems = nev + nbound;
    const int N = (int)a.rd.N, nds = (int)a.nds, nchan = a.rd.nchan;
    const int c0 = chunk * G;
    for (int i = threadIdx.x; i < npass * G; i += blockDim.x) {
        const int p = i / G;
        dly[dix(p, i - p * G)] = (int16_t)a.dly[p][c0 + i - p * G];
    }
    // the largest |subband| of every pass over all this workgroup's items, published once
    if (threadIdx.x < kMaxPass) amax_s[threadIdx.x] = 0;
    if (threadIdx.x < 2) ntask2[threadIdx.x] = 0;
    int it = 0;
    for (int e = blockIdx.x / gm.nchunk; e < nitems; e += gridDim.x / gm.nchunk, it++) {
        const bool clip_ev = e < nev;
        const int par = it & 1;
        const int r = clip_ev ? events[e] : (blist ? a.fix_blist[bofs0 + e - nev] : e - nev + 1) * a.rd.blk;
        const int wlo = max(r - a.dmax - ds + 1, 0) & ~15;
        const int b0 = (int)blk_of(a.rd, wlo);
        const int b1 = min(b0 + 1, a.rd.nblk - 1);
        const int bndrel = (b0 + 1) * a.rd.blk - wlo;
        __syncthreads();                                  // the previous item is done with LDS
        if (threadIdx.x == 0) {
            needany = clip_ev;
            anyflag = 0;
            ntask2[par ^ 1] = 0;                          // the next item's count (this one's was cleared before)
        }
        for (int i = threadIdx.x; i < G; i += blockDim.x) {
            zap[i] = zap_at(a.rd, b0, c0 + i);
            zap[G + i] = zap_at(a.rd, b1, c0 + i);
            pad[i] = pad_at(a.rd, b0, c0 + i);
            pad[G + i] = pad_at(a.rd, b1, c0 + i);
        }
        // a clipped spectrum needs every phase: its window, flags, zap bits and task list are all
        // issued in this one phase (no barrier or global round trip between them)
        if (clip_ev) {
            fix8_window(a, lraw, flg, G, Wp, c0, wlo, N, nchan, fprobe, anyflag);
            if constexpr (CPS > 0) {
                for (int i = threadIdx.x; i < SG; i += blockDim.x) {
                    uint32_t zb = 0;                      // bit cc: zapped in block slot 0; 16 + cc: slot 1
#pragma unroll
                    for (int cc = 0; cc < CPS; cc++)
                        zb |= ((uint32_t)zap_at(a.rd, b0, c0 + i * CPS + cc) << cc) |
                              ((uint32_t)zap_at(a.rd, b1, c0 + i * CPS + cc) << (16 + cc));
                    zbm_s[i] = zb;
                }
            }
            if (!(fprobe & 1)) {
                // task (p, lc): the output channel lc maps r to, unless an earlier channel of its
                // subband maps r to the same output.  The tasks that fold are listed first (one
                // LDS atomic per wave), so the folds run on dense lanes (~1 task in 6 folds)
                for (int i0 = 0; i0 < npass * G; i0 += blockDim.x) {
                    const int i = i0 + threadIdx.x;
                    int j = 0;
                    const bool keep = i < npass * G && fix8_task(dly, i, G, cps, DST, SG, r, N, nds, DS, pds_s, ds, j);
                    const uint64_t m = __ballot(keep);
                    if (m) {
                        const int ln = threadIdx.x & 63;
                        int base = 0;
                        if (ln == 0) base = atomicAdd(&ntask2[par], __popcll(m));
                        base = __shfl(base, 0, 64);
                        if (keep) tlist[base + __popcll(m & ((1ull << ln) - 1ull))] = (uint16_t)i;
                    }
                }
            }
        }
        __syncthreads();
        if (!clip_ev) {
            // boundary r between blocks b0 and b1: subbands with a channel masked in both whose
            // pads differ; per pass their outputs whose rows contain r - 1 and r
            for (int i = threadIdx.x; i < npass * SG; i += blockDim.x) {
                const int p = i / SG, sl = i - p * SG;
                int mind = 1 << 30, maxd = 0;
                bool need = false;
                for (int cc = 0; cc < cps; cc++) {
                    const int lc = sl * cps + cc;
                    const int d = dly[dix(p, lc)];
                    mind = min(mind, d);
                    maxd = max(maxd, d);
                    need |= zap[lc] && zap[G + lc] && pad[lc] != pad[G + lc];
                }
                const int dsp = pds(p), ndsp = DS < 0 ? N / dsp : nds;
                int lo = r - (dsp - 1) - maxd, hi = r - 1 - mind;
                lo = lo <= 0 ? 0 : (lo + dsp - 1) / dsp;
                hi = hi < 0 ? -1 : min(hi / dsp, ndsp - 1);
                lo_s[i] = lo;
                cnt_s[i] = need && hi >= lo ? hi - lo + 1 : 0;
                if (cnt_s[i]) needany = 1;
            }
            __syncthreads();
            if (!needany) continue;                       // uniform
        }
        if (!clip_ev) {
            // a boundary that needs outputs redone: the window, flags and zap bits now
            fix8_window(a, lraw, flg, G, Wp, c0, wlo, N, nchan, fprobe, anyflag);
            if constexpr (CPS > 0) {
                for (int i = threadIdx.x; i < SG; i += blockDim.x) {
                    uint32_t zb = 0;                      // bit cc: zapped in block slot 0; 16 + cc: slot 1
#pragma unroll
                    for (int cc = 0; cc < CPS; cc++)
                        zb |= ((uint32_t)zap[i * CPS + cc] << cc) | ((uint32_t)zap[G + i * CPS + cc] << (16 + cc));
                    zbm_s[i] = zb;
                }
            }
            __syncthreads();
        }
        if (fprobe & 1) {
        } else if (clip_ev) {
            const int ntask = ntask2[par];
            for (int t = threadIdx.x; t < ntask; t += blockDim.x) {
                const int i = tlist[t];
                int j = 0;
                (void)fix8_task(dly, i, G, cps, DST, SG, r, N, nds, DS, pds_s, ds, j);
                const int p = i / G, lc = i - p * G;
                const int lc0 = lc - lc % cps;
                const int16_t* dl = dly + dix(p, lc0) - lc0;
                const int dsp = pds(p);
                float acc;
                if constexpr (CPS > 0) {
                    int dr[CPS];
#pragma unroll
                    for (int cc = 0; cc < CPS; cc++) dr[cc] = dl[lc0 + cc];
                    const uint32_t zb = zbm_s[lc0 / CPS];
                    acc = fix8_fold_pre<CPS, (DS > 0 ? DS : 0)>(a, lraw, flg, pad, Wp, G, lc0, dr, zb, j * dsp - wlo,
                                                               bndrel, dsp);
                } else {
                    acc = fix8_fold<CPS, (DS > 0 ? DS : 0)>(a, lraw, flg, zap, pad, dl, Wp, G, lc0, j * dsp - wlo, bndrel,
                                                           dsp);
                }
                const int s = (c0 + lc0) / cps;
                if (a.sub_dtype == 0) {
                    const int16_t q = to_i16(acc, a.sub_round);
                    if (!(fprobe & 4)) ((int16_t*)outp_s[p])[(int64_t)s * ostr_s[p] + j] = q;
                    const int aq = q < 0 ? -(int)q : (int)q;
                    if (aq > 0 && !(fprobe & 8)) atomicMax(&amax_s[p], aq);
                } else {
                    ((float*)outp_s[p])[(int64_t)s * ostr_s[p] + j] = acc;
                }
            }
        } else {
            // the boundary outputs of every (pass, subband) as one dense task range (the
            // (pass, subband, jmax) grid left ~3/4 of the lanes idle): an exclusive prefix of
            // the counts, then each task finds its (pass, subband) by binary search
            const int nps = npass * SG;
            {
                const int per = (nps + (int)blockDim.x - 1) / (int)blockDim.x;
                const int i0 = threadIdx.x * per;
                int sum = 0;
                for (int k = 0; k < per; k++)
                    if (i0 + k < nps) sum += cnt_s[i0 + k];
                int incl = sum;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int t = __shfl_up(incl, o, 64);
                    if ((threadIdx.x & 63) >= o) incl += t;
                }
                const int wv = threadIdx.x >> 6;
                if ((threadIdx.x & 63) == 63) wsum_s[wv] = incl;
                __syncthreads();
                int base = 0;
                for (int w = 0; w < wv; w++) base += wsum_s[w];
                int run = base + incl - sum;
                for (int k = 0; k < per; k++)
                    if (i0 + k < nps) {
                        pre_s[i0 + k] = run;
                        run += cnt_s[i0 + k];
                    }
                if (threadIdx.x == blockDim.x - 1) pre_s[nps] = run;
                __syncthreads();
            }
            const int total = pre_s[nps];
            const bool flags = anyflag != 0;
            for (int t = threadIdx.x; t < total; t += blockDim.x) {
                int lo = 0, hi = nps - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (pre_s[mid] <= t) lo = mid;
                    else hi = mid - 1;
                }
                const int ps = lo, jj = t - pre_s[ps];
                const int p = ps / SG, sl = ps - p * SG;
                const int j = lo_s[ps] + jj;
                const int16_t* dl = dly + dix(p, sl * cps) - sl * cps;
                const int dsp = pds(p);
                float acc;
                if constexpr (CPS > 0) {
                    int dr[CPS];
#pragma unroll
                    for (int cc = 0; cc < CPS; cc++) dr[cc] = dl[sl * CPS + cc];
                    acc = flags ? fix8_fold_pre<CPS, (DS > 0 ? DS : 0), true>(a, lraw, flg, pad, Wp, G, sl * CPS, dr,
                                                                             zbm_s[sl], j * dsp - wlo, bndrel, dsp)
                                : fix8_fold_pre<CPS, (DS > 0 ? DS : 0), false>(a, lraw, flg, pad, Wp, G, sl * CPS, dr,
                                                                              zbm_s[sl], j * dsp - wlo, bndrel, dsp);
                } else {
                    acc = fix8_fold<CPS, (DS > 0 ? DS : 0)>(a, lraw, flg, zap, pad, dl, Wp, G, sl * cps, j * dsp - wlo,
                                                           bndrel, dsp);
                }
                const int s = chunk * SG + sl;
                if (a.sub_dtype == 0) {
                    const int16_t q = to_i16(acc, a.sub_round);
                    if (!(fprobe & 4)) ((int16_t*)outp_s[p])[(int64_t)s * ostr_s[p] + j] = q;
                    const int aq = q < 0 ? -(int)q : (int)q;
                    if (aq > 0 && !(fprobe & 8)) atomicMax(&amax_s[p], aq);
                } else {
                    ((float*)outp_s[p])[(int64_t)s * ostr_s[p] + j] = acc;
                }
            }
        }
    }
    __syncthreads();
    if (a.sub_dtype == 0 && threadIdx.x < npass) publish_max(a.maxabs[threadIdx.x], amax_s[threadIdx.x]);
}

static size_t fix8_lds_bytes(const Stage1Multi& a, const Fix8Geom& g)
{
    const int dst = (a.cps == 8 || a.cps == 10 || a.cps == 16) ? 16 : a.cps;   // k_stage1_fix8's DST
    return (size_t)g.G * g.Wp + g.Wp + (size_t)2 * g.G * 4 + (size_t)((2 * g.G + 15) & ~15) +
           (size_t)2 * ((a.npass * g.SG * dst + 7) & ~7) + (size_t)(3 * a.npass * g.SG + 1) * 4 + (size_t)2 * a.npass * g.G;
}

// LDS budget of one k_stage1_fix8 workgroup: smaller windows per workgroup mean more of
// them in flight on a CU, which this latency-bound kernel wants; measured over the C2 beam's
// stages (profiles/r02_fix8_lds.txt): 24 KiB best, except at ds >= 10 (wide windows) 40 KiB.
static size_t fix8_lds_cap(int ds)
{
    // HD_FIX8_LDS_KB (profiling): the cap in KiB for every ds
    if (getenv("HD_FIX8_LDS_KB")) return (size_t)atoi(getenv("HD_FIX8_LDS_KB")) * 1024;
    // measured per stage of the C2 beam (scripts/ab_fix8_lds.sh, 16/24/32/48 KiB): ds 1 best at
    // 16-24 (1.77 ms), ds 2-3 at 32 (1.33 / 0.84), ds 5-10 at 48 (2.00 / 1.18 / 1.42): wider
    // windows need room for more channels per workgroup
    return (size_t)(ds <= 1 ? 24 : ds <= 3 ? 32 : 48) * 1024;
}

// Geometry for k_stage1_fix8, or false when it does not apply (the generic kernel then runs).
static bool fix8_geom(const Stage1Multi& a, Fix8Geom& g)
{
    if (!a.rawT || (a.rd.nbits != 8 && a.rd.nbits != 4) || a.rd.scl || a.rd.offs || a.rd.wts) return false;
    if (a.dmax > 32767 || a.rd.N >= ((int64_t)1 << 31) - (1 << 24)) return false;
    g.Wp = (2 * a.dmax + 2 * a.ds + 15 + 15) & ~15;       // + alignment of the window start
    if (g.Wp + 16 > a.rd.blk || a.dmax + a.ds + 16 > kRawTPad) return false;
    g.SG = 0;
    for (int sg = a.nsub; sg >= 1; sg--) {
        if (a.nsub % sg) continue;
        const int G = sg * a.cps;
        if (G > 1024) continue;
        Fix8Geom t = g;
        t.SG = sg;
        t.G = G;
        if (fix8_lds_bytes(a, t) <= fix8_lds_cap(a.ds)) {
            g.SG = sg;
            break;
        }
    }
    if (!g.SG) return false;
    g.G = g.SG * a.cps;
    if ((int64_t)a.npass * g.G > 65535) return false;   // (task ids are 16-bit)
    g.nchunk = a.nsub / g.SG;
    int dsmin = a.ds;
    if (a.pass_ds)
        for (int p = 0; p < a.npass; p++) dsmin = std::min(dsmin, (int)a.pds[p]);
    g.jmax = (a.dmax + dsmin - 1) / dsmin + 1;
    return true;
}

int fix8_chunk_channels(const Stage1Multi& a)
{
    Fix8Geom g;
    return !(a.probe & 128) && fix8_geom(a, g) ? g.G : 0;
}

hipError_t launch_stage1_fixup(const Stage1Multi& a, const int32_t* events, const int32_t* nevents, int boundaries,
                               hipStream_t st)
{
    if (a.nds <= 0 || a.npass <= 0) return hipSuccess;
    Fix8Geom g;
    if (!(a.probe & 128) && fix8_geom(a, g)) {           // probe bit 7: the generic kernel
        const unsigned grid = (unsigned)(std::max(1, 4096 / g.nchunk) * g.nchunk);
        const size_t lb = fix8_lds_bytes(a, g);
        // compile-time (cps, ds) for the Mock DDplan's stages (16 bits of zap flags per
        // channel set: cps <= 16), else the runtime kernel
        const void* fn = (const void*)k_stage1_fix8<0, 0>;
#define HD_F8(C, D) if (a.cps == C && a.ds == D) fn = (const void*)k_stage1_fix8<C, D>;
        HD_F8(10, 1) HD_F8(10, 2) HD_F8(10, 3) HD_F8(10, 5) HD_F8(10, 6) HD_F8(10, 10)
        HD_F8(8, 1) HD_F8(16, 1)
#undef HD_F8
        if (a.pass_ds)                                    // several DDplan stages' passes
            fn = a.cps == 10 ? (const void*)k_stage1_fix8<10, -1> : a.cps == 8 ? (const void*)k_stage1_fix8<8, -1>
               : a.cps == 16 ? (const void*)k_stage1_fix8<16, -1> : (const void*)k_stage1_fix8<0, -1>;
        if (lb > 64 * 1024) {
            const hipError_t e = set_max_lds(fn, (int)lb);
            if (e != hipSuccess) return e;
        }
        if (getenv("HD_FIX8_PROBE")) boundaries |= atoi(getenv("HD_FIX8_PROBE")) << 8;
        void* args[] = {(void*)&a, (void*)&g, (void*)&events, (void*)&nevents, (void*)&boundaries};
        return hipLaunchKernel(fn, dim3(grid), dim3(256), args, lb, st);
    }
    if (a.pass_ds) return hipErrorNotSupported;       // (the caller launches per DDplan stage)
    // boundary items scan one subband per thread (nsub <= blockDim); clipped-spectrum items loop
    // over channels, so any nsub (e.g. the nsub = nchan no-subband pass) takes them
    if ((boundaries && a.nsub > 256) || a.rd.N >= ((int64_t)1 << 31) - (1 << 24)) return hipErrorInvalidValue;
    const size_t lds = fixup_lds_bytes(a);
    if (lds > 64 * 1024) return hipErrorInvalidValue;
    // grid-stride over a device-side event count: no host round trip for the count
    hipLaunchKernelGGL(k_stage1_fixup, dim3(4096), dim3(256), lds, st, a, events, nevents, boundaries);
    return hipGetLastError();
}

}  // namespace hd
