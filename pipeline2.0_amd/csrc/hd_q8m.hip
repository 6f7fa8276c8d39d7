// hd_q8m.hip — stage 1 of several DDplan stages in one launch (8-bit integer path).
//
// k_stage1_q8 forms the passes of ONE DDplan stage from a tile whose quarter geometry is tied
// to that stage's downsampling.  Every launch re-reads the channel-major copy of the raw
// block (4 GB) and pays ~0.7-1 ms of per-workgroup setup on its ~10^5 short workgroups
// (profiles/r04_stage1_split.txt: the launch with its fill and sums switched off), and the
// Mock DDplan has five stages with ds >= 2 holding 1-12 passes each.  k_stage1_q8m takes the
// passes of all of them at once: the tile holds 4 quarters of S = 960 raw rows -- a multiple
// of every ds it serves (2, 3, 5, 6, 10 ...) -- so one fill and one setup per workgroup serve
// every pass, each pass summed at its own ds (a compile-time case per ds; lanes past
// 960 / ds outputs per quarter sit out).  The arithmetic per output is k_stage1_q8's: exact
// packed integer sums over the quarter-interleaved LDS tile, the per-read-block pad constants
// of masked channels when the float fold provably rounds the same, else the oracle's float
// fold; clipped spectra and read-block boundaries are recomputed by the per-stage fixup
// launches afterwards, and the tiles past N by the float kernel, exactly as for k_stage1_q8.
#include "hd_device.h"

namespace hd {

constexpr int kQ8mS = 960;                    // raw rows per quarter of the tile
#ifndef Q8M_UNROLL
#define Q8M_UNROLL 4
#endif

bool stage1_q8m_supports_ds(int ds) { return ds == 2 || ds == 3 || ds == 5 || ds == 6 || ds == 10; }

// The DS consecutive dwords of one channel row at LDS byte address addr, as NR = ceil(DS / 2)
// ds_read2_b32 (for odd DS the last read's second dword is past the row's needed range: the
// LDS allocation has 16 bytes of slack).  Inline asm, so the compiler cannot put a wait after
// each read; q8m_wait<N> below waits until at most N LDS operations are outstanding and ties b,
// so no use of b moves above it.
template <int NR>
__device__ __forceinline__ void q8m_rd(uint64_t (&b)[NR], uint32_t addr)
{
#pragma unroll
    for (int r = 0; r < NR; r++)
        asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3" : "=v"(b[r]) : "v"(addr), "i"(2 * r), "i"(2 * r + 1));
}

// The same dwords by ds_read_b64 when the row address is 8-byte aligned (even DS and an even
// channel delay: lanes DS dwords apart then hit all 64 banks once, where the dword pairs of
// ds_read2_b32 are 2-way bank-conflicted)
template <int N, int NB>
__device__ __forceinline__ void q8m_rd64(uint64_t (&b)[NB], uint32_t addr)
{
#pragma unroll
    for (int r = 0; r < N; r++) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(b[r]) : "v"(addr), "i"(8 * r));
}

template <int N, int NR>
__device__ __forceinline__ void q8m_wait(uint64_t (&b)[NR])
{
    if constexpr (NR == 1) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(b[0]) : "i"(N));
    else if constexpr (NR == 2) asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(b[0]), "+v"(b[1]) : "i"(N));
    else if constexpr (NR == 3) asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]) : "i"(N));
    else if constexpr (NR == 4)
        asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) : "i"(N));
    else if constexpr (NR == 5)
        asm volatile("s_waitcnt lgkmcnt(%5)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]) : "i"(N));
    else if constexpr (NR == 6)
        asm volatile("s_waitcnt lgkmcnt(%6)"
                     : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]) : "i"(N));
    else static_assert(NR >= 1 && NR <= 6, "NR");
}

// One pass at compile-time DS over the tile (the body of k_stage1_q8's pass loop, with the
// quarter length S = 960 and ceil(960 / DS / 64) output positions per lane and quarter).
template <int CPS, int DS, bool B64>
__device__ __forceinline__ void q8m_pass(const Stage1Multi& a, int p, int s, int tile, int lane, const uint32_t* lds,
                                         const int (&lrb)[CPS], const int (&dl)[CPS], int dmx, int brow, int brow2,
                                         uint32_t z0, uint32_t z1, uint32_t z2, uint32_t zany, uint32_t zall,
                                         int fz, bool splitfree, double P0, double P1, double P2, bool negpad,
                                         bool intpad, const float* padw, int& amax)
{
    constexpr int S = kQ8mS, JQ = S / DS, M = (JQ + 63) / 64;
    const bool mean = a.ds_mode == 1;
    const int64_t tO0 = (int64_t)tile * (4 * JQ);
    // (opaque lane: keeps the per-DS address arithmetic of all five cases from being hoisted
    //  out of the pass loop, where it would stay live across every pass)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const uint32_t* lbase = lds + ln * DS;
    // this lane's LDS byte address of the tile (the reads below are inline asm)
    const uint32_t lb = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint32_t*)lds) + 4u * (uint32_t)(ln * DS);
    // the per-block pad constants of the channels masked in every block of the tile (see
    // k_stage1_q8): C = DS * P + D/2, integer path while frac(C) keeps clear of 0 and 1
    const int Dh = mean ? DS / 2 : 0;
    int cadd0 = a.sub_dtype == 0 ? Dh : 0, cadd1 = cadd0, cadd2 = cadd0;
    bool intpath = zany == 0;
    if (zany && splitfree && a.sub_dtype == 0) {
        const double half = mean ? 0.5 * DS : 0.5;
        const double C0 = (double)DS * P0 + half, C1 = (double)DS * P1 + half, C2 = (double)DS * P2 + half;
        const double f0 = C0 - floor(C0), f1 = C1 - floor(C1), f2 = C2 - floor(C2);
        const double m0 = fmin(f0, 1.0 - f0), m1 = fmin(f1, 1.0 - f1), m2 = fmin(f2, 1.0 - f2);
        const double cap = mean ? 65535.0 : 32767.0;
        const double eps = a.ptie[p];
        if (!negpad && (intpad || (m0 > eps && m1 > eps && m2 > eps)) &&
            fmax(fmax(C0, C1), C2) + (double)(CPS * DS * 255) <= cap) {
            intpath = true;
            cadd0 = (int)floor(C0);
            cadd1 = (int)floor(C1);
            cadd2 = (int)floor(C2);
        }
    }
    intpath = __builtin_amdgcn_readfirstlane((int)intpath) != 0;
    if (a.probe & 4) intpath = true;                      // (profiling: the float fold never taken)
    cadd0 = __builtin_amdgcn_readfirstlane(cadd0);
    cadd1 = __builtin_amdgcn_readfirstlane(cadd1);
    cadd2 = __builtin_amdgcn_readfirstlane(cadd2);
    if (intpath) {
        // one output position per lane and quarter at a time: two packed accumulators live
        const uint32_t k0c = (uint32_t)cadd0, k1c = (uint32_t)cadd1, k2c = (uint32_t)cadd2;
        const int br1 = brow, br2 = brow2;
        auto kof = [=](int row) { return k0c + (row >= br1 ? k1c - k0c : 0u) + (row >= br2 ? k2c - k1c : 0u); };
        int mx = 0;
#pragma unroll Q8M_UNROLL
        for (int m = 0; m < M; m++) {
            const bool act = (m + 1) * 64 <= JQ || lane + 64 * m < JQ;
            uint32_t ae, ao;
            if (brow >= (1 << 30) || (cadd0 == cadd1 && cadd1 == cadd2)) {   // (uniform: one constant)
                ae = ao = (uint32_t)cadd0 | ((uint32_t)cadd0 << 16);
            } else {
                const int lastrow = (lane + 64 * m) * DS + DS - 1 + dmx;
                ae = kof(lastrow) | (kof(lastrow + 2 * S) << 16);
                ao = kof(lastrow + S) | (kof(lastrow + 3 * S) << 16);
            }
            // lanes past JQ outputs per quarter read a clamped (in-tile) dword, discarded.
            // Channels masked in every block of the tile add zeros (rows zeroed after the fill).
            // Software pipeline over the channels: channel cc + 1's reads are in flight while
            // channel cc is added.
            const int mo = act ? m * 64 * DS : -lane * DS;
            // Odd DS, or B64 off: ds_read2_b32 pairs (at even DS lanes DS dwords apart then
            // 2-way bank-conflict).  B64 (HD_Q8M_B64=1, even DS): DS / 2 + 1 aligned ds_read_b64
            // from the channel's address rounded down to 8 bytes (all 64 banks once); the adds
            // start at the second dword when the channel delay is odd (uniform per channel).
            // No branch may sit between a read and its wait: the compiler resolves a branch with
            // register copies placed before the wait (the asm outputs look ready to it), copies
            // of registers the LDS has not yet written (tests/test_asm_lds.py checks).
            constexpr int NR = (DS + 1) / 2;
            constexpr bool EV = B64 && DS % 2 == 0;
            constexpr int NB = EV ? NR + 1 : NR;
            uint64_t ba[NB], bb[NB];
            auto rd = [&](uint64_t (&b)[NB], int cc) {
                const uint32_t ad = lb + 4u * (uint32_t)(lrb[cc] + dl[cc] + mo);
                if constexpr (EV) q8m_rd64<NB, NB>(b, ad & ~7u);
                else q8m_rd<NR>(b, ad);
            };
            auto adds = [&](const uint64_t (&b)[NB], int off) {
#pragma unroll
                for (int k = 0; k < DS; k++) {
                    const int kk = k + off;
                    const uint32_t x = (kk & 1) ? (uint32_t)(b[kk >> 1] >> 32) : (uint32_t)b[kk >> 1];
                    ae += x & 0x00FF00FFu;
                    ao += __builtin_amdgcn_perm(0u, x, 0x0c030c01u);
                }
            };
            rd(ba, 0);
#pragma unroll
            for (int cc = 0; cc < CPS; cc++) {
                uint64_t (&cur)[NB] = (cc & 1) ? bb : ba;
                uint64_t (&nxt)[NB] = (cc & 1) ? ba : bb;
                if (cc + 1 < CPS) {
                    rd(nxt, cc + 1);
                    q8m_wait<NB, NB>(cur);
                } else {
                    q8m_wait<0, NB>(cur);
                }
                if (EV && (dl[cc] & 1)) adds(cur, 1);
                else adds(cur, 0);
                asm volatile("" : "+v"(ae), "+v"(ao));   // (channel by channel: no add tree over the pass)
            }
            if (!act) continue;
            if (a.probe & 8) {                            // (profiling: sums without the stores)
                mx = max(mx, (int)((ae ^ ao) & 0x7FFFu));
                continue;
            }
            if (a.sub_dtype == 0) {
                if (mean && DS > 1) {
                    const float inv = 1.0f / (float)DS, half = 0.5f / (float)DS;
                    auto divpk = [&](uint32_t v) {
                        // DS = 2: trunc(v * 0.5f + 0.25f) = floor(v / 2) exactly, both halves at once
                        if constexpr (DS == 2) return (v >> 1) & 0x7FFF7FFFu;
                        const uint32_t lo = (uint32_t)((float)(v & 0xFFFFu) * inv + half);
                        const uint32_t hi = (uint32_t)((float)(v >> 16) * inv + half);
                        return lo | (hi << 16);
                    };
                    ae = divpk(ae);
                    ao = divpk(ao);
                }
                int16_t* o = (int16_t*)a.out[p] + (int64_t)s * a.ostride[p] + tO0 + lane + 64 * m;
                __builtin_nontemporal_store((int16_t)(ae & 0xFFFFu), o);     // (non-temporal: as k_stage1_q8)
                __builtin_nontemporal_store((int16_t)(ao & 0xFFFFu), o + JQ);
                __builtin_nontemporal_store((int16_t)(ae >> 16), o + 2 * JQ);
                __builtin_nontemporal_store((int16_t)(ao >> 16), o + 3 * JQ);
                mx = max(mx, (int)max(max(ae & 0xFFFFu, ae >> 16), max(ao & 0xFFFFu, ao >> 16)));
            } else {
                float* o = (float*)a.out[p] + (int64_t)s * a.ostride[p] + tO0 + lane + 64 * m;
                const uint32_t qv[4] = {ae & 0xFFFFu, ao & 0xFFFFu, ae >> 16, ao >> 16};
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    float x = (float)qv[q];
                    if (mean) x = x / (float)DS;
                    o[q * JQ] = x;
                }
            }
        }
        amax = mx;
    } else {
        // the float fold (subbands with a channel masked in some but not all blocks of the tile,
        // near-ties, f32 output): the oracle's order -- per ds step the channels from 0.0f, the
        // integer prefix up to the first masked channel exact, then float adds.  The channels'
        // rows and delays are the integer path's registers; their pads per read block come
        // from the wave's LDS table (padw[bi * 16 + cc]), so nothing extra stays live across
        // the pass loop (the fold had re-derived each channel's delay and pad by dependent
        // global loads: 2.9 of the fused launch's 10.5 ms for 3.8 % of its subband tiles)
        // the channels' LDS rows and delays go to the wave's table too (read back below, so
        // the unrolled fold holds no scalar registers of its own)
        int* chw = (int*)(padw + 48);
        if (lane == 0) {
#pragma unroll
            for (int cc = 0; cc < CPS; cc++) {
                chw[cc] = lrb[cc] + dl[cc];
                chw[16 + cc] = dl[cc];
            }
        }
        asm volatile("" ::: "memory");                    // (as for the pads above)
        __builtin_amdgcn_wave_barrier();
#pragma unroll 1
        for (int m = 0; m < M; m++) {
            if ((m + 1) * 64 > JQ && lane + 64 * m >= JQ) continue;
            float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 1
            for (int k = 0; k < DS; k++) {
                const int t = (lane + 64 * m) * DS + k;    // quarter-relative raw row
                uint32_t xs[CPS];
#pragma unroll
                for (int cc = 0; cc < CPS; cc++) xs[cc] = lbase[chw[cc] + m * 64 * DS + k];
                uint32_t pe = 0, po = 0;
                float sk[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int cc = 0; cc < CPS; cc++) {
                    const uint32_t x = xs[cc];
                    if (cc < fz) {
                        pe += x & 0x00FF00FFu;
                        po += __builtin_amdgcn_perm(0u, x, 0x0c030c01u);
                    } else {
                        if (cc == fz) {
                            sk[0] = (float)(pe & 0xFFFFu);
                            sk[1] = (float)(po & 0xFFFFu);
                            sk[2] = (float)(pe >> 16);
                            sk[3] = (float)(po >> 16);
                        }
                        float v[4] = {(float)(x & 0xFFu), (float)((x >> 8) & 0xFFu), (float)((x >> 16) & 0xFFu),
                                      (float)(x >> 24)};
                        if (zany & (1u << cc)) {
                            const int rr = t + chw[16 + cc];
#pragma unroll
                            for (int q = 0; q < 4; q++) {
                                const int row = rr + q * S;
                                const int bi = row >= brow2 ? 2 : row >= brow ? 1 : 0;
                                const uint32_t zb = bi == 2 ? z2 : bi == 1 ? z1 : z0;
                                if ((zb >> cc) & 1u) v[q] = padw[bi * 16 + cc];
                            }
                        }
#pragma unroll
                        for (int q = 0; q < 4; q++) sk[q] += v[q];
                    }
                }
#pragma unroll
                for (int q = 0; q < 4; q++) acc[q] += sk[q];
            }
            if (mean)
#pragma unroll
                for (int q = 0; q < 4; q++) acc[q] = acc[q] / (float)DS;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int64_t oi = (int64_t)s * a.ostride[p] + tO0 + lane + 64 * m + q * JQ;
                if (a.sub_dtype == 0) {
                    const int16_t v = to_i16(acc[q], a.sub_round);
                    ((int16_t*)a.out[p])[oi] = v;
                    amax = max(amax, v < 0 ? -(int)v : (int)v);
                } else {
                    ((float*)a.out[p])[oi] = acc[q];
                }
            }
        }
    }
}

template <int CPS, bool B64>
__global__ __launch_bounds__(256, 3) void k_stage1_q8m(Stage1Multi a)
{
    constexpr int S = kQ8mS;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint32_t* lds = (uint32_t*)smem;
    const int G = a.sg * CPS;
    const int logical = xcd_remap(blockIdx.x, gridDim.x);
    const int tile = logical / a.ngroups;
    const int g = logical - tile * a.ngroups;
    const int64_t tR0 = (int64_t)tile * (4 * S);
    if (s1_special(a, tR0, 4 * S + a.dmax)) return;     // uniform: the float kernel's SPECIAL launches
    const int K = S + a.dmax;
    const int W = a.W;
    const int c0 = g * G;
    const int rc_lo = a.rd.flip ? a.rd.nchan - c0 - G : c0;

    // ---- fill (k_stage1_q8's channel-major fill): dword kk of channel lc packs rows kk + q*S
    if (!(a.probe & 2)) {
        constexpr int U = 4;
        const int nkb = (K + 15) >> 4;
        const int units = G * nkb;
        const int nthr = blockDim.x;
        const uint8_t* t0p = a.rawT + (int64_t)rc_lo * a.tstride + tR0;
        for (int u0 = threadIdx.x; u0 < units; u0 += U * nthr) {
            uint4 r[U][4];
            int lcs[U], kbs[U];
#pragma unroll
            for (int h = 0; h < U; h++) {
                const int u = min(u0 + h * nthr, units - 1);
                lcs[h] = u / nkb;
                kbs[h] = u - lcs[h] * nkb;
                const uint8_t* sp = t0p + (int64_t)lcs[h] * a.tstride + 16 * kbs[h];
#pragma unroll
                for (int q = 0; q < 4; q++) r[h][q] = *(const uint4*)(sp + (int64_t)q * S);
            }
#pragma unroll
            for (int h = 0; h < U; h++) {
                uint32_t o[16];
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    const uint32_t x0 = w == 0 ? r[h][0].x : w == 1 ? r[h][0].y : w == 2 ? r[h][0].z : r[h][0].w;
                    const uint32_t x1 = w == 0 ? r[h][1].x : w == 1 ? r[h][1].y : w == 2 ? r[h][1].z : r[h][1].w;
                    const uint32_t x2 = w == 0 ? r[h][2].x : w == 1 ? r[h][2].y : w == 2 ? r[h][2].z : r[h][2].w;
                    const uint32_t x3 = w == 0 ? r[h][3].x : w == 1 ? r[h][3].y : w == 2 ? r[h][3].z : r[h][3].w;
                    const uint32_t ab_lo = __builtin_amdgcn_perm(x1, x0, 0x05010400u);
                    const uint32_t ab_hi = __builtin_amdgcn_perm(x1, x0, 0x07030602u);
                    const uint32_t cd_lo = __builtin_amdgcn_perm(x3, x2, 0x05010400u);
                    const uint32_t cd_hi = __builtin_amdgcn_perm(x3, x2, 0x07030602u);
                    o[4 * w + 0] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u);
                    o[4 * w + 1] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u);
                    o[4 * w + 2] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u);
                    o[4 * w + 3] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u);
                }
                uint4* d = (uint4*)(lds + lcs[h] * W + 16 * kbs[h]);
                const int rot = (threadIdx.x >> 1) & 3;
#pragma unroll
                for (int st = 0; st < 4; st++) {
                    const int w = (st + rot) & 3;
                    const uint4 v = w == 0 ? make_uint4(o[0], o[1], o[2], o[3])
                                  : w == 1 ? make_uint4(o[4], o[5], o[6], o[7])
                                  : w == 2 ? make_uint4(o[8], o[9], o[10], o[11])
                                           : make_uint4(o[12], o[13], o[14], o[15]);
                    d[w] = v;
                }
            }
        }
    }
    __shared__ uint8_t zrow[256];
    if (a.rd.zidx) {            // (uniform) channels masked in every block of the tile: rows zeroed
        const int64_t bz = tR0 / a.rd.blk;
        s1_zero_masked_rows(lds, G, W, a.rd, bz, (int)((tR0 + 4 * S + a.dmax - 1) / a.rd.blk - bz) + 1, c0, zrow);
    } else {
        __syncthreads();
    }

    // ---- per-wave subband state (k_stage1_q8): wave w serves subband w / wps and the passes
    //      p = w % wps (mod wps); the tile may straddle two read-block boundaries
    const int wps = (a.probe & 16) || a.sg >= 4 ? 1 : 4 / a.sg;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sl = wv / wps, pw = wv - sl * wps;
    const int lane = threadIdx.x & 63;
    int brow = 1 << 30, brow2 = 1 << 30;
    const int64_t b0 = tR0 / a.rd.blk;
    {
        const int64_t b = (b0 + 1) * a.rd.blk - tR0;
        if (b < 4 * S + a.dmax) brow = (int)b;
        if (b + a.rd.blk < 4 * S + a.dmax) brow2 = (int)(b + a.rd.blk);
    }
    if (sl >= a.sg) return;
    const int s = g * a.sg + sl;
    const int cl0 = sl * CPS;
    int lrb[CPS];
    float pad0[CPS], pad1[CPS], pad2[CPS];
    uint32_t z0 = 0, z1 = 0, z2 = 0;
    const int64_t b1 = brow < (1 << 30) ? b0 + 1 : b0;
    const int64_t b2 = brow2 < (1 << 30) ? b0 + 2 : b1;
#pragma unroll
    for (int cc = 0; cc < CPS; cc++) {
        const int c = c0 + cl0 + cc;
        const int lr = a.rd.flip ? G - 1 - (cl0 + cc) : cl0 + cc;
        lrb[cc] = lr * W;
        pad0[cc] = pad_at(a.rd, b0, c);
        pad1[cc] = pad_at(a.rd, b1, c);
        pad2[cc] = pad_at(a.rd, b2, c);
        if (zap_at(a.rd, b0, c)) z0 |= 1u << cc;
        if (zap_at(a.rd, b1, c)) z1 |= 1u << cc;
        if (zap_at(a.rd, b2, c)) z2 |= 1u << cc;
    }
    z0 = __builtin_amdgcn_readfirstlane(z0);
    z1 = __builtin_amdgcn_readfirstlane(z1);
    z2 = __builtin_amdgcn_readfirstlane(z2);
    const uint32_t zany = z0 | z1 | z2, zall = z0 & z1 & z2, zsplit = (z0 ^ z1) | (z1 ^ z2);
    const int fz = zany ? __builtin_ctz(zany) : CPS;
    // the masked-in-every-block channels' pad sums (their ds-independent part)
    double P0 = 0.0, P1 = 0.0, P2 = 0.0;
    bool negpad = false, intpad = true;
#pragma unroll
    for (int cc = 0; cc < CPS; cc++)
        if (zall & (1u << cc)) {
            P0 += (double)pad0[cc];
            P1 += (double)pad1[cc];
            P2 += (double)pad2[cc];
            negpad |= pad0[cc] < 0.0f || pad1[cc] < 0.0f || pad2[cc] < 0.0f;
            intpad &= pad0[cc] == floorf(pad0[cc]) && pad1[cc] == floorf(pad1[cc]) && pad2[cc] == floorf(pad2[cc]);
        }
    const bool splitfree = zsplit == 0;
    // the float fold's pads: this wave's table [read block slot 0..2][channel] (written and read
    // by the wave itself, so no barrier)
    __shared__ float padtab[4][3 * 16 + 32];              // (<= 4 waves per workgroup; + rows, delays)
    float* padw = padtab[wv];
    if (lane < 3 * CPS) {
        const int bi = lane / CPS, cc = lane - bi * CPS;
        padw[bi * 16 + cc] = pad_at(a.rd, bi == 0 ? b0 : bi == 1 ? b1 : b2, c0 + cl0 + cc);
    }
    // (other lanes of the wave read these: keep every later LDS access after the writes -- the
    // compiler, seeing no write in a reading lane's own program, could otherwise hoist its read)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    int pmax = 0;
    const int npass = (a.probe & 1) ? 0 : a.npass;
    for (int p = pw; p < npass; p += wps) {
        int dl[CPS];
        sload_i32<CPS>(a.dly[p] + c0 + cl0, dl);          // (scalar loads: see k_stage1_q8)
        int dmx = 0;
#pragma unroll
        for (int cc = 0; cc < CPS; cc++) dmx = max(dmx, dl[cc]);
        int amax = 0;
        const int ds = a.pds[p];
#define HD_Q8M_CASE(D)                                                                                        \
        case D:                                                                                               \
            q8m_pass<CPS, D, B64>(a, p, s, tile, lane, lds, lrb, dl, dmx, brow, brow2, z0, z1, z2, zany, zall, fz, \
                                  splitfree, P0, P1, P2, negpad, intpad, padw, amax);                       \
            break;
        switch (ds) {
            HD_Q8M_CASE(2)
            HD_Q8M_CASE(3)
            HD_Q8M_CASE(5)
            HD_Q8M_CASE(6)
            HD_Q8M_CASE(10)
        default: break;
        }
#undef HD_Q8M_CASE
        if (a.sub_dtype == 0) {
            amax = wave_max_full(amax);
            pmax = lane == p ? amax : pmax;
        }
    }
    if (a.sub_dtype == 0 && lane < a.npass) publish_max(a.maxabs[lane], pmax);
}

size_t stage1_q8m_lds_bytes(const Stage1Multi& a) { return (size_t)a.sg * a.cps * a.W * 4 + 16; }   // (+ read slack)

hipError_t launch_stage1_q8m(const Stage1Multi& a, hipStream_t st)
{
    if (a.npass <= 0 || a.ntiles <= 0) return hipSuccess;
    const size_t lds = stage1_q8m_lds_bytes(a);
    const void* fn = nullptr;
    // HD_Q8M_B64=1 (A/B): the even-ds reads as aligned ds_read_b64 (bank-conflict free, one more
    // read and a branch per channel)
    static const bool b64 = getenv("HD_Q8M_B64") && atoi(getenv("HD_Q8M_B64")) != 0;
    if (a.cps == 10) fn = b64 ? (const void*)k_stage1_q8m<10, true> : (const void*)k_stage1_q8m<10, false>;
    else if (a.cps == 8) fn = b64 ? (const void*)k_stage1_q8m<8, true> : (const void*)k_stage1_q8m<8, false>;
    else if (a.cps == 16) fn = b64 ? (const void*)k_stage1_q8m<16, true> : (const void*)k_stage1_q8m<16, false>;
    else return hipErrorInvalidValue;
    {
        const hipError_t e = set_max_lds(fn, (int)std::max<size_t>(lds, 64 * 1024));
        if (e != hipSuccess) return e;
    }
    const dim3 block((unsigned)(64 * (a.sg < 4 ? 4 : a.sg))), grid((unsigned)(a.ntiles * a.ngroups));
    void* args[] = {(void*)&a};
    return hipLaunchKernel(fn, grid, block, args, lds, st);
}

int stage1_q8m_quarter_rows() { return kQ8mS; }

}  // namespace hd
