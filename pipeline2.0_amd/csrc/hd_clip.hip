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

// ---- the serial recurrence over blocks (one workgroup, thread = channel) -------------
__global__ __launch_bounds__(1024) void k_clip_recur(ClipArgs a)
{
    const int nch = a.rd.nchan;
    const float clip_sigma = a.clip_sigma;
    const int nloop = nch > 0 ? nch : 1;
    for (int c0 = 0; c0 < nloop; c0 += blockDim.x) {
        const int c = c0 + threadIdx.x;
        const bool own = c < nch;
        float ravg = 0.0f, rstd = 0.0f, cra = 0.0f;
        float lev = own && a.padvals0 ? a.padvals0[c] : 0.0f;
        int nread = 0;
        for (int b = 0; b < a.rd.nblk; b++) {
            const bool run = clip_sigma > 0.0f && !(a.allzap && a.allzap[b]);
            if (run) {
                const int ng = a.numgood[b];
                double cur_avg, cur_std, cat;
                if (ng < 1) {
                    cur_avg = (double)ravg;
                    cur_std = (double)rstd;
                    cat = (double)cra;
                } else {
                    cur_avg = a.bavg[b];
                    cur_std = a.bstd[b];
                    cat = own ? a.chansum[(int64_t)b * nch + c] / (double)ng : 0.0;
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
            if (c0 == 0 && threadIdx.x == 0) {
                a.doclip[b] = run;
                a.ravg[b] = ravg;
                a.trig[b] = clip_sigma * rstd;
            }
            if (own) a.pad[(int64_t)b * nch + c] = lev;
        }
    }
}

// ---- clip flags + the event list -------------------------------------------------------
__global__ __launch_bounds__(256) void k_clip_flag(ClipArgs a)
{
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool clip = false;
    if (t < a.rd.N) {
        const int64_t b = t / a.rd.blk;
        clip = a.doclip[b] && fabsf(a.zdm[t] - a.ravg[b]) > a.trig[b];
        a.clipped[t] = clip;
    }
    // wave-aggregated append
    const uint64_t bal = __ballot(clip);
    if (bal) {
        const int lane = threadIdx.x & 63;
        int base = 0;
        if (lane == __ffsll((unsigned long long)bal) - 1) base = atomicAdd(a.nevents, __popcll(bal));
        base = __shfl(base, __ffsll((unsigned long long)bal) - 1, 64);
        if (clip) a.events[base + __popcll(bal & ((1ull << lane) - 1))] = (int32_t)t;
    }
}

hipError_t launch_clip(const ClipArgs& a, hipStream_t st)
{
    const RawDesc& rd = a.rd;
    if (rd.N <= 0) return hipSuccess;
    if (rd.blk > kClipMaxBlock) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(a.nevents, 0, sizeof(int32_t), st);
    if (e != hipSuccess) return e;
    const bool calib = rd.scl || rd.offs || rd.wts;
    if (rd.nbits == 8 && !calib && rd.rowbytes % 16 == 0)
        hipLaunchKernelGGL(k_clip_zdm_u8, dim3((unsigned)((rd.N + 3) / 4)), dim3(256), 0, st, rd, a.zdm);
    else
        hipLaunchKernelGGL(k_clip_zdm, dim3((unsigned)((rd.N + 255) / 256)), dim3(256), 0, st, rd, a.zdm);
    hipLaunchKernelGGL(k_clip_block, dim3((unsigned)rd.nblk), dim3(1024), 0, st, a);
    hipLaunchKernelGGL(k_clip_as52, dim3((unsigned)((rd.nblk + 63) / 64)), dim3(64), 0, st, a);
    hipLaunchKernelGGL(k_clip_chan, dim3((unsigned)(rd.nblk * ((rd.nchan + 255) / 256))), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_clip_recur, dim3(1), dim3(1024), 0, st, a);
    hipLaunchKernelGGL(k_clip_flag, dim3((unsigned)((rd.N + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// stage-1 fixup
// ------------------------------------------------------------------------------------
// Work item = (event e, pass p, subband s), lanes over consecutive subbands.  Event e <
// nev is the clipped spectrum r = events[e]: every output whose rows
// [j*ds + mind_s, j*ds + ds - 1 + maxd_s] contain r is recomputed.  Events past nev are the
// read-block boundaries r = (e - nev + 1) * blk (only when `boundaries`): outputs whose rows
// contain both r - 1 and r, in subbands with a channel masked in either block (the integer
// path's per-block pad constants do not cover them).  Recomputation is the exact per-cell
// fold of k_stage1_direct; overlapping items write identical values.
__global__ __launch_bounds__(256) void k_stage1_fixup(Stage1Multi a, const int32_t* __restrict__ events,
                                                     const int32_t* __restrict__ nevents, int boundaries)
{
    const int nev = *nevents;
    const int nbound = boundaries ? a.rd.nblk - 1 : 0;
    const int64_t per_ev = (int64_t)a.npass * a.nsub;
    const int64_t total = (int64_t)(nev + nbound) * per_ev;
    const int ds = a.ds, cps = a.cps;
    for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < total;
         it += (int64_t)gridDim.x * blockDim.x) {
        const int e = (int)(it / per_ev);
        const int rem = (int)(it - (int64_t)e * per_ev);
        const int p = rem / a.nsub, s = rem - p * a.nsub;
        const int32_t* dly = a.dly[p] + s * cps;
        int mind = 1 << 30, maxd = 0;
        for (int cc = 0; cc < cps; cc++) {
            mind = min(mind, dly[cc]);
            maxd = max(maxd, dly[cc]);
        }
        int64_t jlo, jhi;
        if (e < nev) {
            const int64_t r = events[e];
            jlo = r - (ds - 1) - maxd;
            jhi = r - mind;
        } else {
            const int64_t bb = e - nev + 1;
            const int64_t r = bb * a.rd.blk;
            bool masked = false;
            for (int cc = 0; cc < cps; cc++) {
                const int c = s * cps + cc;
                masked |= zap_at(a.rd, bb - 1, c) || zap_at(a.rd, bb, c);
            }
            if (!masked) continue;
            jlo = r - (ds - 1) - maxd;
            jhi = r - 1 - mind;
        }
        jlo = jlo <= 0 ? 0 : (jlo + ds - 1) / ds;       // ceil for jlo > 0
        jhi = jhi < 0 ? -1 : jhi / ds;
        if (jhi > a.nds - 1) jhi = a.nds - 1;
        int amax = 0;
        for (int64_t j = jlo; j <= jhi; j++) {
            float acc = 0.0f;
            for (int k = 0; k < ds; k++) {
                float sk = 0.0f;
                const int64_t tb = j * ds + k;
                for (int cc = 0; cc < cps; cc++) sk += chan_value(a.rd, tb + dly[cc], s * cps + cc);
                acc += sk;
            }
            if (a.ds_mode == 1) acc = acc / (float)ds;
            if (a.sub_dtype == 0) {
                const int16_t q = to_i16(acc, a.sub_round);
                ((int16_t*)a.out[p])[(int64_t)s * a.ostride[p] + j] = q;
                amax = max(amax, q < 0 ? -(int)q : (int)q);
            } else {
                ((float*)a.out[p])[(int64_t)s * a.ostride[p] + j] = acc;
            }
        }
        if (a.sub_dtype == 0) publish_max(a.maxabs[p], amax);
    }
}

hipError_t launch_stage1_fixup(const Stage1Multi& a, const int32_t* events, const int32_t* nevents, int boundaries,
                               hipStream_t st)
{
    if (a.nds <= 0 || a.npass <= 0) return hipSuccess;
    // grid-stride over a device-side item count: no host round trip for the event count
    hipLaunchKernelGGL(k_stage1_fixup, dim3(2048), dim3(256), 0, st, a, events, nevents, boundaries);
    return hipGetLastError();
}

}  // namespace hd
