// hd_stage2.hip — CDNA4 (gfx950) stage-2 kernels of the dedispersion engine: int16 (or f32)
// subbands -> DM series (prepsubband -lodm/-dmstep/-numdms; reference
// PALFA2_presto_search.py:514-520).  k_stage2_pair (the default), k_stage2_ring and the
// cross-check variants (direct, lds, wide, wide2).  Split from hd_kernels.hip (stage 1 and the
// helpers) so the two halves compile in parallel.
#include "hd_device.h"

namespace hd {

// ------------------------------------------------------------------------------------
// stage 2, direct
// ------------------------------------------------------------------------------------

__device__ __forceinline__ double block_sum_f64(double v, double* red /* [4] */)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) r = ((red[0] + red[1]) + red[2]) + red[3];
    return r;
}

__global__ __launch_bounds__(256) void k_stage2_direct(Stage2Args a)
{
    __shared__ double red[4];
    const int d = blockIdx.y;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int32_t* off = a.off + (int64_t)d * a.nsub;
    float acc = 0.0f;
    if (t < a.nvalid) {
        if (a.sub_dtype == 0) {
            const int16_t* sub = (const int16_t*)a.sub;
            for (int s = 0; s < a.nsub; s++) {
                const int64_t idx = t + off[s];
                const float v = idx < a.nds ? (float)sub[(int64_t)s * a.sub_stride + idx] : 0.0f;
                acc += v;
            }
        } else {
            const float* sub = (const float*)a.sub;
            for (int s = 0; s < a.nsub; s++) {
                const int64_t idx = t + off[s];
                const float v = idx < a.nds ? sub[(int64_t)s * a.sub_stride + idx] : 0.0f;
                acc += v;
            }
        }
        a.out[(int64_t)d * a.out_stride + t] = acc;
    }
    if (a.partial) {
        const double tot = block_sum_f64(t < a.nvalid ? (double)acc : 0.0, red);
        if (threadIdx.x == 0) a.partial[(int64_t)d * a.ntiles + blockIdx.x] = tot;
    }
}

hipError_t launch_stage2_direct(const Stage2Args& a, hipStream_t st)
{
    if (a.nvalid <= 0) return hipSuccess;
    dim3 grid((unsigned)((a.nvalid + 255) / 256), (unsigned)a.numdms);
    hipLaunchKernelGGL(k_stage2_direct, grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// stage 2, LDS-tiled (int16 subbands)
// ------------------------------------------------------------------------------------
//
// Workgroup = 4 waves = one tile of 256 output samples x (4*Q) DMs.  Lane l owns the 4
// consecutive samples t0+4l .. t0+4l+3; wave w owns DMs d0+wQ .. d0+wQ+Q-1.
// Subbands are staged SC at a time.  For subband s the workgroup needs samples
// [t0+omin_s, t0+256+omax_s+3]; LDS keeps 4 copies of that window, copy j shifted by j
// samples, so the 4 samples at any offset o start 8-byte aligned in copy (o-omin)&3.
// boff[yblk][s][q'] (host table) is that byte offset, and lane l adds 8*l.

constexpr int kTT = 256;   // output samples per workgroup
constexpr int kSC = 8;     // subbands per LDS stage

typedef short short2v __attribute__((ext_vector_type(2)));


template <int Q>
__global__ __launch_bounds__(256) void k_stage2_lds(Stage2Args a, const int32_t* __restrict__ boff)
{
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    int16_t* lds = (int16_t*)lds_raw;

    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t t0 = (int64_t)tile * kTT;
    const int yb = blockIdx.y;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int dpb = a.dms_per_blk;
    const int dblk0 = yb * dpb;
    const int ws = a.wstride;
    const int16_t* sub = (const int16_t*)a.sub;
    const int32_t* omin = a.omin + (int64_t)yb * a.nsub;
    const int32_t* bo = boff + (int64_t)yb * a.nsub * dpb + wave * Q;

    int maxabs = *a.maxabs;
    maxabs = maxabs < 1 ? 1 : maxabs;
    int G = 32767 / maxabs;
    G = G < 1 ? 1 : (G > 64 ? 64 : G);
    G = __builtin_amdgcn_readfirstlane(G);

    int acc32[Q][4];
    short2v acc16[Q][2];
#pragma unroll
    for (int q = 0; q < Q; q++) {
#pragma unroll
        for (int j = 0; j < 4; j++) acc32[q][j] = 0;
        acc16[q][0] = short2v{0, 0};
        acc16[q][1] = short2v{0, 0};
    }
    int gcount = 0;
    const uint32_t lane_byte = (uint32_t)lane * 8u;

    // The wave's LDS offsets for a whole chunk (kSC subbands x Q DMs) are fetched with one
    // vector load per register before the fill, and read back with v_readlane inside the
    // accumulate loop: no scalar-memory wait sits between the LDS reads.
    constexpr int NR = (kSC * Q + 63) / 64;
    for (int sc0 = 0; sc0 < a.nsub; sc0 += kSC) {
        const int nsc = (a.nsub - sc0) < kSC ? (a.nsub - sc0) : kSC;
        int voff[NR];
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const int e = r * 64 + lane;
            const int sl = e / Q, q = e - (e / Q) * Q;
            voff[r] = (sl < nsc) ? bo[(int64_t)(sc0 + sl) * dpb + q] : 0;
        }
        __syncthreads();
        // ---- fill: thread unit u writes positions 4u..4u+3 of all 4 shifted copies
        //      (copy j, position i = window element i + j) from 4 aligned dword loads:
        //      elements g0-p .. g0-p+7 with g0 = window start + 4u, p = g0 & 1 (uniform
        //      per subband), then v_alignbit for odd element offsets, one ds_write_b64 per copy.
        const int units = ws >> 2;
        for (int sl = 0; sl < nsc; sl++) {
            const int s = sc0 + sl;
            const int64_t wbeg = t0 + omin[s];
            const int p = (int)(wbeg & 1);
            const int16_t* srow = sub + (int64_t)s * a.sub_stride;
            uint2* dst0 = (uint2*)(lds + (sl * 4) * ws);
            for (int u = threadIdx.x; u < units; u += 256) {
                const int64_t g0 = wbeg + 4 * u;
                uint32_t D[4];
                if (g0 - p + 8 <= a.nds) {
                    const uint32_t* src = (const uint32_t*)(srow + (g0 - p));
#pragma unroll
                    for (int i = 0; i < 4; i++) D[i] = src[i];
                } else {   // past the end of the subbands: zeros
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int64_t e0 = g0 - p + 2 * i;
                        const uint32_t lo = e0 < a.nds ? (uint16_t)srow[e0] : 0u;
                        const uint32_t hi = e0 + 1 < a.nds ? (uint16_t)srow[e0 + 1] : 0u;
                        D[i] = lo | (hi << 16);
                    }
                }
                // copy j needs elements j..j+3 of g0, i.e. D-space halves (p+j) .. (p+j+3)
#define HD_PAIR(h) (((h) & 1) ? __builtin_amdgcn_alignbit(D[((h) + 1) >> 1], D[(h) >> 1], 16) : D[(h) >> 1])
                if (p == 0) {
                    dst0[u] = make_uint2(HD_PAIR(0), HD_PAIR(2));
                    dst0[(ws >> 2) + u] = make_uint2(HD_PAIR(1), HD_PAIR(3));
                    dst0[2 * (ws >> 2) + u] = make_uint2(HD_PAIR(2), HD_PAIR(4));
                    dst0[3 * (ws >> 2) + u] = make_uint2(HD_PAIR(3), HD_PAIR(5));
                } else {
                    dst0[u] = make_uint2(HD_PAIR(1), HD_PAIR(3));
                    dst0[(ws >> 2) + u] = make_uint2(HD_PAIR(2), HD_PAIR(4));
                    dst0[2 * (ws >> 2) + u] = make_uint2(HD_PAIR(3), HD_PAIR(5));
                    dst0[3 * (ws >> 2) + u] = make_uint2(HD_PAIR(4), HD_PAIR(6));
                }
#undef HD_PAIR
            }
        }
        __syncthreads();
        // ---- accumulate
#pragma unroll
        for (int sl = 0; sl < kSC; sl++) {
            if (sl >= nsc) break;
#pragma unroll
            for (int q = 0; q < Q; q++) {
                const int e = sl * Q + q;
                const uint32_t addr = (uint32_t)__builtin_amdgcn_readlane(voff[e >> 6], e & 63) + lane_byte;
                const uint2 v = *(const uint2*)(lds_raw + addr);
                acc16[q][0] += __builtin_bit_cast(short2v, v.x);
                acc16[q][1] += __builtin_bit_cast(short2v, v.y);
            }
            if (++gcount == G) {
                gcount = 0;
#pragma unroll
                for (int q = 0; q < Q; q++) {
                    acc32[q][0] += acc16[q][0].x;
                    acc32[q][1] += acc16[q][0].y;
                    acc32[q][2] += acc16[q][1].x;
                    acc32[q][3] += acc16[q][1].y;
                    acc16[q][0] = short2v{0, 0};
                    acc16[q][1] = short2v{0, 0};
                }
            }
        }
    }
    // ---- finish, store, per-tile partial sums
    const int64_t tl = t0 + 4 * lane;
#pragma unroll
    for (int q = 0; q < Q; q++) {
        acc32[q][0] += acc16[q][0].x;
        acc32[q][1] += acc16[q][0].y;
        acc32[q][2] += acc16[q][1].x;
        acc32[q][3] += acc16[q][1].y;
        const int d = dblk0 + wave * Q + q;
        if (d < a.numdms && d < dblk0 + dpb) {
            float* o = a.out + (int64_t)d * a.out_stride + tl;
            int64_t part = 0;
            if (tl + 3 < a.nvalid) {
                *(float4*)o = make_float4((float)acc32[q][0], (float)acc32[q][1], (float)acc32[q][2],
                                          (float)acc32[q][3]);
                part = (int64_t)acc32[q][0] + acc32[q][1] + acc32[q][2] + acc32[q][3];
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (tl + j < a.nvalid) {
                        o[j] = (float)acc32[q][j];
                        part += acc32[q][j];
                    }
            }
            if (a.partial) {
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) part += __shfl_xor(part, m, 64);
                if (lane == 0) a.partial[(int64_t)d * a.ntiles + tile] = (double)part;
            }
        }
    }
}

template <int Q>
static hipError_t launch_lds_q(const Stage2Args& a, const int32_t* boff, int nyblk, hipStream_t st)
{
    const unsigned ntiles = (unsigned)((a.nvalid + kTT - 1) / kTT);
    const size_t lds = (size_t)kSC * 4 * a.wstride * sizeof(int16_t);
    hipLaunchKernelGGL(k_stage2_lds<Q>, dim3(ntiles, (unsigned)nyblk), dim3(256), lds, st, a, boff);
    return hipGetLastError();
}

// boff is passed through Stage2Args.off for this variant (host-built [nyblk][nsub][4Q]).
hipError_t launch_stage2_lds(const Stage2Args& a, int q, hipStream_t st)
{
    if (a.nvalid <= 0) return hipSuccess;
    const int nyblk = (a.numdms + a.dms_per_blk - 1) / a.dms_per_blk;
    switch (q) {
    case 8: return launch_lds_q<8>(a, a.off, nyblk, st);
    case 16: return launch_lds_q<16>(a, a.off, nyblk, st);
    case 19: return launch_lds_q<19>(a, a.off, nyblk, st);
    case 24: return launch_lds_q<24>(a, a.off, nyblk, st);
    default: return hipErrorInvalidValue;
    }
}

// ------------------------------------------------------------------------------------
// stage 2, wide LDS tiles (int16 subbands)
// ------------------------------------------------------------------------------------
//
// Workgroup = NW <= 16 waves; wave w owns DMs w*Q .. w*Q+Q-1 of the y-block and all waves
// share one tile of T = 256*R output samples, so every subband window staged in LDS (the
// same 4 shifted copies as k_stage2_lds) serves NW*Q DMs -- up to 80, a whole PALFA pass.
// Lane l owns samples t0 + 256r + 4l + i (r < R, i < 4): for one (subband, DM) its R
// ds_read_b64 share one address at immediate offsets 512r, so the per-pair address work
// (v_readlane of the host-built byte offset + v_add) is paid once per R reads.  The reads
// are issued by inline asm one (subband, DM) step ahead of their use, with an explicit
// lgkmcnt wait: hipcc would otherwise fuse them into ds_read2st64_b64 (8 LDS cycles
// instead of 2 x 2) and wait for each one right after issuing it.  Subbands are staged sc
// (<= kSC2) at a time into one of two LDS buffers: chunk c+1's global loads are issued
// before chunk c is accumulated and written to the other buffer after it (one barrier per
// chunk).  Accumulation is packed int16 widened to int32 every G subbands, as above.

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

template <int R>
__device__ __forceinline__ void lds_read_r(uint64_t (&b)[R], uint32_t addr)
{
#pragma unroll
    for (int r = 0; r < R; r++) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(b[r]) : "v"(addr), "i"(512 * r));
}

template <int R>
__device__ __forceinline__ void lds_wait_keep(uint64_t (&b)[R])
{
    // wait until at most R LDS operations are outstanding (the next step's reads): the reads
    // into b are then complete; b is an in/out operand so its uses stay after the wait
    if constexpr (R == 3) asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]));
    else if constexpr (R == 4) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]));
    else if constexpr (R == 2) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(b[0]), "+v"(b[1]));
    else static_assert(R == 2 || R == 3 || R == 4, "R");
}

template <int R>
__device__ __forceinline__ void lds_wait_all(uint64_t (&b)[R])
{
    if constexpr (R == 3) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]));
    else if constexpr (R == 4) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]));
    else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b[0]), "+v"(b[1]));
}


// wait until at most N LDS operations are outstanding; b (the buffer about to be consumed)
// is an in/out operand so its uses stay after the wait
template <int N, int R>
__device__ __forceinline__ void lds_wait_n(uint64_t (&b)[R])
{
    if constexpr (R == 2) asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(b[0]), "+v"(b[1]) : "i"(N));
    else if constexpr (R == 3) asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]) : "i"(N));
    else if constexpr (R == 4)
        asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) : "i"(N));
    else static_assert(R >= 2 && R <= 4, "R");
}

// LDS read lookahead of the ring kernel (in (subband, DM) steps): as deep as the 128-VGPR
// budget of 4 waves per SIMD allows next to the Q*R*6 accumulator registers
template <int Q, int R>
constexpr int ring_la()
{
    const int spare = 128 - 26 - Q * R * 6;
    const int la = spare / (2 * R) - 1;
    return la < 1 ? 1 : (la > 3 ? 3 : la);
}

template <int Q, int R, int SC>
__global__ __launch_bounds__(1024) void k_stage2_wide(Stage2Args a, const int32_t* __restrict__ boff)
{
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    int16_t* lds = (int16_t*)lds_raw;
    constexpr int T = 256 * R;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t t0 = (int64_t)tile * T;
    const int yb = blockIdx.y;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nthr = blockDim.x;
    const int dpb = a.dms_per_blk;
    const int dblk0 = yb * dpb;
    const int ws = a.wstride;        // elements per shifted copy (multiple of 4)
    const int upw = ws >> 2;         // fill units (4 window positions) per subband
    constexpr int sc = SC;           // subbands per chunk (nsub % SC == 0: every chunk is full)
    const int16_t* sub = (const int16_t*)a.sub;
    const int32_t* omin = a.omin + (int64_t)yb * a.nsub;
    const int32_t* bo = boff + (int64_t)yb * a.nsub * dpb + wave * Q;
    const int nchunk = (a.nsub + sc - 1) / sc;

    int maxabs = *a.maxabs;
    maxabs = maxabs < 1 ? 1 : maxabs;
    int G = 32767 / maxabs;
    G = G < 1 ? 1 : (G > 64 ? 64 : G);
    G = __builtin_amdgcn_readfirstlane(G);

    int acc32[Q][R][4];
    short2v acc16[Q][R][2];
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int r = 0; r < R; r++) {
#pragma unroll
            for (int j = 0; j < 4; j++) acc32[q][r][j] = 0;
            acc16[q][r][0] = short2v{0, 0};
            acc16[q][r][1] = short2v{0, 0};
        }
    int gcount = 0;
    const uint32_t lane_byte = (uint32_t)lane * 8u;

    // fill unit u = sl * upw + uu of a chunk: 4 window positions of subband sl, from 8
    // subband samples (4 dwords); the first kUMax units of a thread are prefetched
    int usl[kUMax], uuu[kUMax];
#pragma unroll
    for (int i = 0; i < kUMax; i++) {
        const int u = threadIdx.x + i * nthr;
        usl[i] = u / upw;
        uuu[i] = u - usl[i] * upw;
    }
    auto load_unit = [&](int s, int uu, uint32_t* D) -> int {
        const int64_t wbeg = t0 + omin[s];
        const int p = (int)(wbeg & 1);
        const int16_t* srow = sub + (int64_t)s * a.sub_stride;
        const int64_t e0 = wbeg + 4 * uu - p;
        if (e0 + 8 <= a.nds) {   // one dwordx4 load (4-byte aligned: e0 is even)
            const u32x4a4 v = *(const u32x4a4*)(srow + e0);
            D[0] = v.x;
            D[1] = v.y;
            D[2] = v.z;
            D[3] = v.w;
        } else {   // past the end of the subbands: zeros
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int64_t e = e0 + 2 * j;
                const uint32_t lo = e < a.nds ? (uint16_t)srow[e] : 0u;
                const uint32_t hi = e + 1 < a.nds ? (uint16_t)srow[e + 1] : 0u;
                D[j] = lo | (hi << 16);
            }
        }
        return p;
    };
    auto store_unit = [&](int16_t* buf, int sl, int u, const uint32_t* Di, int p) {
        uint2* dst0 = (uint2*)(buf + (sl * 4) * ws);
#define HD_PAIR(h) (((h) & 1) ? __builtin_amdgcn_alignbit(Di[((h) + 1) >> 1], Di[(h) >> 1], 16) : Di[(h) >> 1])
        if (p == 0) {
            dst0[u] = make_uint2(HD_PAIR(0), HD_PAIR(2));
            dst0[upw + u] = make_uint2(HD_PAIR(1), HD_PAIR(3));
            dst0[2 * upw + u] = make_uint2(HD_PAIR(2), HD_PAIR(4));
            dst0[3 * upw + u] = make_uint2(HD_PAIR(3), HD_PAIR(5));
        } else {
            dst0[u] = make_uint2(HD_PAIR(1), HD_PAIR(3));
            dst0[upw + u] = make_uint2(HD_PAIR(2), HD_PAIR(4));
            dst0[2 * upw + u] = make_uint2(HD_PAIR(3), HD_PAIR(5));
            dst0[3 * upw + u] = make_uint2(HD_PAIR(4), HD_PAIR(6));
        }
#undef HD_PAIR
    };
    uint32_t D[kUMax][4];
    int pbit = 0;
    auto fetch = [&](int c) {
        const int s0 = c * sc;
        const int nsc = min(sc, a.nsub - s0);
        pbit = 0;
#pragma unroll
        for (int i = 0; i < kUMax; i++)
            if (usl[i] < nsc) pbit |= load_unit(s0 + usl[i], uuu[i], D[i]) << i;
    };
    auto put_buf = [&](int c, int b) {
        const int s0 = c * sc;
        const int nsc = min(sc, a.nsub - s0);
        int16_t* buf = lds + b * (sc * 4 * ws);
#pragma unroll
        for (int i = 0; i < kUMax; i++)
            if (usl[i] < nsc) store_unit(buf, usl[i], uuu[i], D[i], (pbit >> i) & 1);
        // units beyond the prefetched ones (wide windows only): synchronous
        for (int u = threadIdx.x + kUMax * nthr; u < nsc * upw; u += nthr) {
            const int sl = u / upw, uu = u - (u / upw) * upw;
            uint32_t E[4];
            const int p = load_unit(s0 + sl, uu, E);
            store_unit(buf, sl, uu, E, p);
        }
    };
    // the chunk's (subband, DM) byte offsets: entry e = sl*Q + q in lane e&63 of voff[e>>6]
    constexpr int NR = (SC * Q + 63) / 64;
    auto load_voff = [&](int c, int (&v)[NR]) {
        const int s0 = c * sc;
        const int nsc = min(sc, a.nsub - s0);
#pragma unroll
        for (int i = 0; i < NR; i++) {
            const int e = i * 64 + lane;
            const int sl = e / Q, q = e - (e / Q) * Q;
            v[i] = (sl < nsc) ? bo[(int64_t)(s0 + sl) * dpb + q] : 0;
        }
    };

    int voff[NR], voff_nxt[NR];
    load_voff(0, voff);
    fetch(0);
    put_buf(0, 0);
    __syncthreads();
    for (int c = 0; c < nchunk; c++) {
        // next chunk's loads, unconditionally (the last iteration re-loads the last chunk
        // into the idle buffer): a branch around them would make the compiler drain vmcnt
        // before the accumulation instead of after it
        const int cn = min(c + 1, nchunk - 1);
        load_voff(cn, voff_nxt);
        if (!(a.probe & 2)) fetch(cn);
        constexpr int nsteps = SC * Q;   // (subband, DM) steps of a chunk; straight-line code,
                                         // so the in-flight read registers are never copied
        uint64_t b0[R], b1[R];
        if (!(a.probe & 1)) {
        lds_read_r<R>(b0, (uint32_t)__builtin_amdgcn_readlane(voff[0], 0) + lane_byte);
#pragma unroll
        for (int e = 0; e < nsteps; e++) {
            {
                uint64_t (&cur)[R] = (e & 1) ? b1 : b0;
                uint64_t (&nxt)[R] = (e & 1) ? b0 : b1;
                if (e + 1 < nsteps) {
                    const int e1 = e + 1;
                    lds_read_r<R>(nxt, (uint32_t)__builtin_amdgcn_readlane(voff[e1 >> 6], e1 & 63) + lane_byte);
                    lds_wait_keep<R>(cur);
                } else {
                    lds_wait_all<R>(cur);
                }
                const int q = e % Q;
#pragma unroll
                for (int r = 0; r < R; r++) {
                    acc16[q][r][0] += __builtin_bit_cast(short2v, (uint32_t)cur[r]);
                    acc16[q][r][1] += __builtin_bit_cast(short2v, (uint32_t)(cur[r] >> 32));
                }
                if (q == Q - 1 && ++gcount == G) {
                    gcount = 0;
#pragma unroll
                    for (int qq = 0; qq < Q; qq++)
#pragma unroll
                        for (int r = 0; r < R; r++) {
                            acc32[qq][r][0] += acc16[qq][r][0].x;
                            acc32[qq][r][1] += acc16[qq][r][0].y;
                            acc32[qq][r][2] += acc16[qq][r][1].x;
                            acc32[qq][r][3] += acc16[qq][r][1].y;
                            acc16[qq][r][0] = short2v{0, 0};
                            acc16[qq][r][1] = short2v{0, 0};
                        }
                }
            }
        }
        }
        if (!(a.probe & 2)) put_buf(cn, (c + 1) & 1);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NR; i++) voff[i] = voff_nxt[i];
    }

    // ---- finish, store, per-tile partial sums
#pragma unroll
    for (int q = 0; q < Q; q++) {
        const int dl = wave * Q + q;
        const int d = dblk0 + dl;
        const bool dv = dl < dpb && d < a.numdms;
        int64_t part = 0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            acc32[q][r][0] += acc16[q][r][0].x;
            acc32[q][r][1] += acc16[q][r][0].y;
            acc32[q][r][2] += acc16[q][r][1].x;
            acc32[q][r][3] += acc16[q][r][1].y;
            const int64_t tl = t0 + 256 * r + 4 * lane;
            if (dv && !(a.probe & 4)) {
                float* o = a.out + (int64_t)d * a.out_stride + tl;
                if (tl + 3 < a.nvalid) {
                    *(float4*)o = make_float4((float)acc32[q][r][0], (float)acc32[q][r][1], (float)acc32[q][r][2],
                                              (float)acc32[q][r][3]);
                    part += (int64_t)acc32[q][r][0] + acc32[q][r][1] + acc32[q][r][2] + acc32[q][r][3];
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (tl + j < a.nvalid) {
                            o[j] = (float)acc32[q][r][j];
                            part += acc32[q][r][j];
                        }
                }
            }
        }
        if (dv && a.partial) {
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) part += __shfl_xor(part, m, 64);
            if (lane == 0) a.partial[(int64_t)d * a.ntiles + tile] = (double)part;
        }
    }
}

#define HD_WIDE_QR(X) X(5, 3) X(4, 4) X(3, 4) X(2, 4)
// ring: every (Q, R) keeps its accumulators, two read buffers and the loop addresses in 128
// VGPRs without spilling (Q=4 takes R=3: at R=4 the loop spilled to scratch)
#define HD_RING_QR(X) X(5, 3) X(5, 2) X(4, 3) X(3, 4) X(2, 4)

// ------------------------------------------------------------------------------------
// stage 2, wide tiles fed by an LDS-DMA staging ring
// ------------------------------------------------------------------------------------
//
// As k_stage2_wide (16 waves x Q DMs share a tile of T = 256*R samples; asm-pipelined LDS
// reads), but each 4-subband chunk's raw windows and (subband, DM) offsets are copied
// global -> LDS by LDS-DMA (global_load_lds_dwordx4, inline asm so hipcc neither waits for
// it nor drains it at barriers) into a ring of NS staging slots, NS-3 chunks ahead of
// their expansion.  No register holds data in flight -- the accumulators keep their VGPRs --
// and the global latency is covered by two chunks of accumulation.  Iteration c: DMA of
// chunk c+NS-1 (one 1 KiB piece per loader wave); expand chunk c+1 (staging -> the 4 shifted
// copies); accumulate chunk c; wait for this wave's DMA of chunk c+2; one barrier.
// Subband rows carry a zero tail (plan allocation), so windows never need bounds checks.

template <int R>
__device__ __forceinline__ void ring_wait_vm()
{
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kRingNS - 3) : "memory");
}

__device__ __forceinline__ void ring_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

// The same with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset
// (saddr form): one VGPR per lane instead of a 64-bit pointer kept live across the loop.
__device__ __forceinline__ void dma16s(const void* sbase, uint32_t voff, uint32_t lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds_dst)
                 : "memory");
}

template <int Q, int R>
__global__ __launch_bounds__(1024) void k_stage2_ring(Stage2Args a, const int32_t* __restrict__ boff)
{
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    constexpr int SC = kRingSC, NS = kRingNS, T = 256 * R;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t t0 = (int64_t)tile * T;
    const int yb = blockIdx.y;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nthr = blockDim.x;
    const int dpb = a.dms_per_blk;
    const int dblk0 = yb * dpb;
    const int ws = a.wstride;
    const int upw = ws >> 2;
    const int npw = a.ring_npw;                       // 1 KiB DMA pieces per window
    const int nbp = a.ring_nbp;                       // pieces of a chunk's offset block
    const int slot_bytes = (SC * npw + nbp) * 1024;
    const int omin_bytes = (a.nsub * 4 + 15) & ~15;
    // LDS: [omin: nsub ints][NS staging slots][2 x SC x 4 copies x ws int16]
    int32_t* lomin = (int32_t*)lds_raw;
    const uint32_t ring0 = (uint32_t)omin_bytes;
    const uint32_t exp0 = ring0 + (uint32_t)(NS * slot_bytes);
    const uint32_t lane_byte = exp0 + (uint32_t)lane * 8u;   // host offsets are relative to exp0
    const int16_t* sub = (const int16_t*)a.sub;
    const int32_t* bo_g = boff + (int64_t)yb * a.nsub * dpb;
    const int nchunk = a.nsub / SC;

    for (int i = threadIdx.x; i < a.nsub; i += nthr) lomin[i] = a.omin[(int64_t)yb * a.nsub + i];
    __syncthreads();

    int maxabs = *a.maxabs;
    maxabs = maxabs < 1 ? 1 : maxabs;
    int G = 32767 / maxabs;
    G = G < 1 ? 1 : (G > 64 ? 64 : G);
    G = __builtin_amdgcn_readfirstlane(G);

    int acc32[Q][R][4];
    short2v acc16[Q][R][2];
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int r = 0; r < R; r++) {
#pragma unroll
            for (int j = 0; j < 4; j++) acc32[q][r][j] = 0;
            acc16[q][r][0] = short2v{0, 0};
            acc16[q][r][1] = short2v{0, 0};
        }
    int gcount = 0;
    const bool loader = wave < SC * npw + nbp;

    // one DMA piece per loader wave per chunk (chunks past the end re-load the last one into
    // a consumed slot, so every loader wave issues exactly one DMA per iteration)
    auto dma = [&](int cc) {
        if (!loader) return;
        const int c2 = min(cc, nchunk - 1);
        const int s0 = c2 * SC;
        const uint32_t slot = ring0 + (uint32_t)((cc % NS) * slot_bytes);
        if (wave < SC * npw) {
            const int sl = wave / npw, pc = wave - (wave / npw) * npw;
            const int s = s0 + sl;
            const int om = __builtin_amdgcn_readfirstlane(lomin[s]);
            const int64_t e0 = t0 + om - (om & 1);
            const char* src = (const char*)(sub + (int64_t)s * a.sub_stride + e0) + pc * 1024;
            dma16s(src, (uint32_t)lane * 16u, slot + (uint32_t)((sl * npw + pc) * 1024));
        } else {
            const int bp = wave - SC * npw;
            const char* src = (const char*)(bo_g + (int64_t)s0 * dpb) + bp * 1024;
            dma16s(src, (uint32_t)lane * 16u, slot + (uint32_t)((SC * npw + bp) * 1024));
        }
    };
    // staging slot of chunk cc -> its 4 shifted copies in expanded buffer cc & 1
    auto expand = [&](int cc) {
        const char* slot = lds_raw + ring0 + (cc % NS) * slot_bytes;
        int16_t* buf = (int16_t*)(lds_raw + exp0) + (cc & 1) * (SC * 4 * ws);
        for (int u = threadIdx.x; u < SC * upw; u += nthr) {
            const int sl = u / upw, uu = u - (u / upw) * upw;
            const uint2 lo = *(const uint2*)(slot + sl * npw * 1024 + uu * 8);
            const uint2 hi = *(const uint2*)(slot + sl * npw * 1024 + uu * 8 + 8);
            const uint32_t Di[4] = {lo.x, lo.y, hi.x, hi.y};
            const int p = lomin[cc * SC + sl] & 1;
            uint2* dst0 = (uint2*)(buf + (sl * 4) * ws);
#define HD_PAIR(h) (((h) & 1) ? __builtin_amdgcn_alignbit(Di[((h) + 1) >> 1], Di[(h) >> 1], 16) : Di[(h) >> 1])
            if (p == 0) {
                dst0[uu] = make_uint2(HD_PAIR(0), HD_PAIR(2));
                dst0[upw + uu] = make_uint2(HD_PAIR(1), HD_PAIR(3));
                dst0[2 * upw + uu] = make_uint2(HD_PAIR(2), HD_PAIR(4));
                dst0[3 * upw + uu] = make_uint2(HD_PAIR(3), HD_PAIR(5));
            } else {
                dst0[uu] = make_uint2(HD_PAIR(1), HD_PAIR(3));
                dst0[upw + uu] = make_uint2(HD_PAIR(2), HD_PAIR(4));
                dst0[2 * upw + uu] = make_uint2(HD_PAIR(3), HD_PAIR(5));
                dst0[3 * upw + uu] = make_uint2(HD_PAIR(4), HD_PAIR(6));
            }
#undef HD_PAIR
        }
    };

    // prologue: chunks 0 .. NS-2 in flight; chunks 0 and 1 landed; chunk 0 expanded
#pragma unroll
    for (int cc = 0; cc < NS - 1; cc++) dma(cc);
    ring_wait_vm<R>();
    ring_barrier();
    expand(0);
    ring_barrier();

    for (int c = 0; c < nchunk; c++) {
        if (!(a.probe & 2)) dma(c + NS - 1);   // probe 2: no window DMA after the prologue
        if (c + 1 < nchunk && !(a.probe & 8)) expand(c + 1);
        // this chunk's (subband, DM) byte offsets: entry e = sl*Q + q in lane e
        const int32_t* sboff = (const int32_t*)(lds_raw + ring0 + (c % NS) * slot_bytes + SC * npw * 1024);
        const int esl = lane / Q, eq = lane - (lane / Q) * Q;
        const int voff = esl < SC ? sboff[esl * dpb + wave * Q + eq] : 0;
        if (!(a.probe & 1)) {
            // (subband, DM) steps of this chunk; the reads of step e+LA are issued before
            // step e's sums, so LA steps of R reads stay in flight per wave
            constexpr int nsteps = SC * Q, LA = ring_la<Q, R>();
            uint64_t bb[LA + 1][R];
#pragma unroll
            for (int e = 0; e < LA; e++)
                lds_read_r<R>(bb[e], (uint32_t)__builtin_amdgcn_readlane(voff, e) + lane_byte);
#pragma unroll
            for (int e = 0; e < nsteps; e++) {
                uint64_t (&cur)[R] = bb[e % (LA + 1)];
                if (e + LA < nsteps) {
                    lds_read_r<R>(bb[(e + LA) % (LA + 1)],
                                  (uint32_t)__builtin_amdgcn_readlane(voff, e + LA) + lane_byte);
                    lds_wait_n<LA * R>(cur);
                } else if (e + 3 == nsteps && LA >= 2) {
                    lds_wait_n<2 * R>(cur);
                } else if (e + 2 == nsteps && LA >= 1) {
                    lds_wait_n<R>(cur);
                } else {
                    lds_wait_n<0>(cur);
                }
                const int q = e % Q;
#pragma unroll
                for (int r = 0; r < R; r++) {
                    acc16[q][r][0] += __builtin_bit_cast(short2v, (uint32_t)cur[r]);
                    acc16[q][r][1] += __builtin_bit_cast(short2v, (uint32_t)(cur[r] >> 32));
                }
                if (q == Q - 1 && ++gcount == G) {
                    gcount = 0;
#pragma unroll
                    for (int qq = 0; qq < Q; qq++)
#pragma unroll
                        for (int r = 0; r < R; r++) {
                            acc32[qq][r][0] += acc16[qq][r][0].x;
                            acc32[qq][r][1] += acc16[qq][r][0].y;
                            acc32[qq][r][2] += acc16[qq][r][1].x;
                            acc32[qq][r][3] += acc16[qq][r][1].y;
                            acc16[qq][r][0] = short2v{0, 0};
                            acc16[qq][r][1] = short2v{0, 0};
                        }
                }
            }
        }
        ring_wait_vm<R>();
        ring_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the workgroup ends

#pragma unroll
    for (int q = 0; q < Q; q++) {
        const int dl = wave * Q + q;
        const int d = dblk0 + dl;
        const bool dv = dl < dpb && d < a.numdms;
        int64_t part = 0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            acc32[q][r][0] += acc16[q][r][0].x;
            acc32[q][r][1] += acc16[q][r][0].y;
            acc32[q][r][2] += acc16[q][r][1].x;
            acc32[q][r][3] += acc16[q][r][1].y;
            const int64_t tl = t0 + 256 * r + 4 * lane;
            if (dv && !(a.probe & 4)) {
                float* o = a.out + (int64_t)d * a.out_stride + tl;
                if (tl + 3 < a.nvalid) {
                    *(float4*)o = make_float4((float)acc32[q][r][0], (float)acc32[q][r][1], (float)acc32[q][r][2],
                                              (float)acc32[q][r][3]);
                    part += (int64_t)acc32[q][r][0] + acc32[q][r][1] + acc32[q][r][2] + acc32[q][r][3];
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (tl + j < a.nvalid) {
                            o[j] = (float)acc32[q][r][j];
                            part += acc32[q][r][j];
                        }
                }
            }
        }
        if (dv && a.partial) {
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) part += __shfl_xor(part, m, 64);
            if (lane == 0) a.partial[(int64_t)d * a.ntiles + tile] = (double)part;
        }
    }
}

size_t stage2_ring_lds_bytes(int wstride, int npw, int nbp, int nsub)
{
    return (size_t)((nsub * 4 + 15) & ~15) + (size_t)kRingNS * (kRingSC * npw + nbp) * 1024 +
           (size_t)2 * kRingSC * 4 * wstride * 2;
}

template <int Q, int R>
static hipError_t launch_ring_qr(const Stage2Args& a, int nyblk, hipStream_t st)
{
    {
        const hipError_t e = set_max_lds((const void*)k_stage2_ring<Q, R>, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    const unsigned ntiles = (unsigned)((a.nvalid + 256 * R - 1) / (256 * R));
    hipLaunchKernelGGL((k_stage2_ring<Q, R>), dim3(ntiles, (unsigned)nyblk), dim3(1024),
                       stage2_ring_lds_bytes(a.wstride, a.ring_npw, a.ring_nbp, a.nsub), st, a, a.off);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Pair variant (default where the subband bound allows it): the ring above, one subband PAIR
// (s0, s1) per chunk.  For every DM d of the y-block, out[d] takes
//   sub[s0][t + off[d][s0]] + sub[s1][t + off[d][s1]] = P_u[t + off[d][s0] - base0],
//   P_u[i] = sub[s0][base0 + i] + sub[s1][base0 + r_u + i],  r_u = off[d][s1] - off[d][s0],
// and a pass's 76 DMs take only 2-6 distinct r_u per pair (host table).  The expand step
// forms each P_u once per tile (in its 4 shifted copies) and every DM then reads ONE window
// per pair instead of two: half the LDS reads and half the packed adds of the ring, at the
// price of U/2 (mean ~1.5) times the expand writes.  All sums are exact integers (int16
// subbands, |P_u| <= 2 * max|subband| <= 32767 by the host's static bound, packed-int16
// groups widened to int32 before they can wrap), so the result is bit-identical.
// Staging slot of a chunk: [s0 window: npw KiB][s1 window: npw KiB][offsets: nbp KiB];
// expanded buffer: 2 (chunk parity) x umax patterns x 4 copies x ws int16.

__device__ __forceinline__ void load8_shift(const uint32_t* w32, int x, uint32_t (&o)[4])
{
    // o = int16 elements x .. x+7 of the staging window (any parity), as 4 packed pairs
    const uint32_t* q = w32 + (x >> 1);
    const uint32_t sh = (uint32_t)(x & 1) * 16u;
    uint32_t w[5];
#pragma unroll
    for (int m = 0; m < 5; m++) w[m] = q[m];
#pragma unroll
    for (int m = 0; m < 4; m++) o[m] = __builtin_amdgcn_alignbit(w[m + 1], w[m], sh);
}

// The same 8 elements from two 8-byte-aligned ds_read_b64 and one ds_read_b32 (the five
// ds_read_b32 above, 8 bytes apart across lanes, run 2-way bank-conflicted): the first dword
// x >> 1 is even (b64, b64, b32) or odd (b32, b64, b64); its parity is uniform per window.
__device__ __forceinline__ void load8_shift64(const uint32_t* w32, int x, uint32_t (&o)[4])
{
    const int j = x >> 1;
    const uint32_t sh = (uint32_t)(x & 1) * 16u;
    uint32_t w[5];
    if ((j & 1) == 0) {
        const uint2 p = *(const uint2*)(w32 + j);
        const uint2 q = *(const uint2*)(w32 + j + 2);
        w[0] = p.x;
        w[1] = p.y;
        w[2] = q.x;
        w[3] = q.y;
        w[4] = w32[j + 4];
    } else {
        w[0] = w32[j];
        const uint2 p = *(const uint2*)(w32 + j + 1);
        const uint2 q = *(const uint2*)(w32 + j + 3);
        w[1] = p.x;
        w[2] = p.y;
        w[3] = q.x;
        w[4] = q.y;
    }
#pragma unroll
    for (int m = 0; m < 4; m++) o[m] = __builtin_amdgcn_alignbit(w[m + 1], w[m], sh);
}

// Twelve int16 elements x .. x+11 of a staging window (any parity) as 6 packed pairs, from
// three reads of the 7 dwords j = x >> 1 .. j + 6: one ds_read_b128 at the 16-byte-aligned
// dword, one ds_read_b64 and one ds_read_b32 around it (the split depends on j & 3, uniform per
// window).  Lanes 16 bytes apart (8-element items) keep the b128 reads conflict-free.
__device__ __forceinline__ void load12_shift(const uint32_t* w32, int x, uint32_t (&o)[6])
{
    const int j = x >> 1;
    const uint32_t sh = (uint32_t)(x & 1) * 16u;
    uint32_t w[7];
    switch (j & 3) {
    case 0: {
        const uint4 a = *(const uint4*)(w32 + j);
        const uint2 b = *(const uint2*)(w32 + j + 4);
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = w32[j + 6];
        break;
    }
    case 1: {
        const uint2 b = *(const uint2*)(w32 + j + 1);
        const uint4 a = *(const uint4*)(w32 + j + 3);
        w[0] = w32[j]; w[1] = b.x; w[2] = b.y; w[3] = a.x; w[4] = a.y; w[5] = a.z; w[6] = a.w;
        break;
    }
    case 2: {
        const uint2 b = *(const uint2*)(w32 + j);
        const uint4 a = *(const uint4*)(w32 + j + 2);
        w[0] = b.x; w[1] = b.y; w[2] = a.x; w[3] = a.y; w[4] = a.z; w[5] = a.w; w[6] = w32[j + 6];
        break;
    }
    default: {
        const uint4 a = *(const uint4*)(w32 + j + 1);
        const uint2 b = *(const uint2*)(w32 + j + 5);
        w[0] = w32[j]; w[1] = a.x; w[2] = a.y; w[3] = a.z; w[4] = a.w; w[5] = b.x; w[6] = b.y;
        break;
    }
    }
#pragma unroll
    for (int m = 0; m < 6; m++) o[m] = __builtin_amdgcn_alignbit(w[m + 1], w[m], sh);
}

// PRB: profiling build of the kernel (a.probe bits switch phases off); the production
// instantiation (PRB = false) carries no probe tests
template <int Q, int R, int PPC, bool NN, bool PRB>
__global__ __launch_bounds__(1024) void k_stage2_pair(Stage2Args a, S2Multi m)
{
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    // the pass of this workgroup: blockIdx.y = pass * nyblk + y-block (one launch may carry
    // every pass of a DDplan stage; their per-pass buffers and table geometry come from m)
    const int pi = (int)blockIdx.y / m.nyblk;
    const S2Pass& P = m.p[pi];
    const int32_t* __restrict__ boff = P.off;
    // PPC subband pairs per chunk: two halve the chunks (barriers, DMA/offset bookkeeping) per
    // tile; their staging ring has one slot less (4) so the doubled expanded buffers fit
    constexpr int NS = PPC == 2 ? 4 : kRingNS, T = 256 * R;
    // one tile per workgroup (nwg == 0), or a persistent workgroup over a contiguous tile
    // range whose chunks (tile, pair) form one stream through the DMA ring, so the table
    // load, ring prologue and launch of the next tile overlap the current one
    int tb, ntl;
    if (a.nwg == 0) {
        tb = xcd_remap(blockIdx.x, gridDim.x);
        ntl = 1;
    } else {
        const int nt = (int)((a.nvalid + T - 1) / T);
        tb = (int)((int64_t)blockIdx.x * nt / gridDim.x);
        ntl = (int)((int64_t)(blockIdx.x + 1) * nt / gridDim.x) - tb;
    }
    const int yb = (int)blockIdx.y - pi * m.nyblk;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nthr = blockDim.x;
    const int dpb = a.dms_per_blk;
    const int dblk0 = yb * dpb;
    const int ws = P.ws;
    const int npw = P.npw;                       // 1 KiB DMA pieces per window
    const int nbp = P.nbp;                       // pieces of a chunk's offset block
    const int umax = P.umax;
    const int slot_bytes = (2 * PPC * npw + nbp) * 1024;
    const int npair = a.nsub >> 1;
    const int tab_bytes = npair * kPairTab * 4;
    int32_t* ltab = (int32_t*)lds_raw;
    const uint32_t ring0 = (uint32_t)tab_bytes;
    const uint32_t exp0 = ring0 + (uint32_t)(NS * slot_bytes);
    const uint32_t lane_byte = exp0 + (uint32_t)lane * 8u;   // host offsets are relative to exp0
    const int16_t* sub = (const int16_t*)P.sub;
    const int32_t* bo_g = boff + (int64_t)yb * npair * dpb;
    const int nchunk = npair / PPC;

    for (int i = threadIdx.x; i < npair * kPairTab; i += nthr) ltab[i] = P.ptab[(int64_t)yb * npair * kPairTab + i];
    __syncthreads();

    int maxabs = *P.maxabs;
    maxabs = maxabs < 1 ? 1 : maxabs;
    // pairs per packed-16-bit group: signed halves hold |sum| <= 32767; with subbands known
    // non-negative (host) the halves are unsigned and hold sums <= 65535 (twice the group)
    constexpr bool nonneg = NN;                        // (a runtime switch here spills registers)
    int G = (nonneg ? 65535 : 32767) / (2 * maxabs);
    G = G < 1 ? 1 : (G > 64 ? 64 : G);
    G = __builtin_amdgcn_readfirstlane(G);

    int acc32[Q][R][4];
    short2v acc16[Q][R][2];
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int r = 0; r < R; r++) {
#pragma unroll
            for (int j = 0; j < 4; j++) acc32[q][r][j] = 0;
            acc16[q][r][0] = short2v{0, 0};
            acc16[q][r][1] = short2v{0, 0};
        }
    int gcount = 0;
    const bool loader = wave < 2 * PPC * npw + nbp;
    // packed 16-bit group -> int32 accumulators (zero- or sign-extended halves)
    auto widen = [&]() {
#pragma unroll
        for (int qq = 0; qq < Q; qq++)
#pragma unroll
            for (int r = 0; r < R; r++) {
                if (nonneg) {
                    const uint32_t lo = __builtin_bit_cast(uint32_t, acc16[qq][r][0]);
                    const uint32_t hi = __builtin_bit_cast(uint32_t, acc16[qq][r][1]);
                    acc32[qq][r][0] += (int)(lo & 0xFFFFu);
                    acc32[qq][r][1] += (int)(lo >> 16);
                    acc32[qq][r][2] += (int)(hi & 0xFFFFu);
                    acc32[qq][r][3] += (int)(hi >> 16);
                } else {
                    acc32[qq][r][0] += acc16[qq][r][0].x;
                    acc32[qq][r][1] += acc16[qq][r][0].y;
                    acc32[qq][r][2] += acc16[qq][r][1].x;
                    acc32[qq][r][3] += acc16[qq][r][1].y;
                }
                acc16[qq][r][0] = short2v{0, 0};
                acc16[qq][r][1] = short2v{0, 0};
            }
    };

    const int ntot = ntl * nchunk;
    int dchunk = 0, dtile = 0, dcount = 0;             // source chunk of the next DMA (clamped at the end)
    auto dma = [&](int cc) {
        const int c2 = dchunk;
        const int64_t t0 = (int64_t)(tb + dtile) * T;
        if (dcount + 1 < ntot) {
            dcount++;
            if (++dchunk == nchunk) { dchunk = 0; dtile++; }
        }
        if (!loader) return;
        const uint32_t slot = ring0 + (uint32_t)((cc % NS) * slot_bytes);
        if (wave < 2 * PPC * npw) {
            const int sl = wave / npw, pc = wave - sl * npw;      // window sl: pair sl / 2, side sl % 2
            const int pr = PPC * c2 + (sl >> 1);
            const int s = 2 * pr + (sl & 1);
            const int b = __builtin_amdgcn_readfirstlane(ltab[pr * kPairTab + (sl & 1)]);   // base0 | b1
            const int64_t e0 = t0 + b - (b & 1);
            const char* src = (const char*)(sub + (int64_t)s * P.sub_stride + e0) + pc * 1024;
            dma16s(src, (uint32_t)lane * 16u, slot + (uint32_t)((sl * npw + pc) * 1024));
        } else {
            const int bp = wave - 2 * PPC * npw;
            const char* src = (const char*)(bo_g + (int64_t)PPC * c2 * dpb) + bp * 1024;
            dma16s(src, (uint32_t)lane * 16u, slot + (uint32_t)((2 * PPC * npw + bp) * 1024));
        }
    };
    // staging slot of chunk cc -> the 4 shifted copies of each pattern partial of its pairs,
    // expanded buffers (cc & 1) * PPC + k
    auto expand = [&](int cc, int chk) {
        const char* slot = lds_raw + ring0 + (cc % NS) * slot_bytes;
        // item = 8 elements of every copy (ws is a multiple of 8: 16-byte stores); the items of
        // the chunk's PPC pairs form one index range over the workgroup's threads, so no thread
        // does two while others idle (a pair has U * ws / 8 ~ 400 items for 1024 threads)
        const int up8 = ws >> 3;
        const int n0 = ltab[(PPC * chk) * kPairTab + 2] * up8;
        const int nall = PPC == 2 ? n0 + ltab[(PPC * chk + 1) * kPairTab + 2] * up8 : n0;
        for (int idx = threadIdx.x; idx < nall; idx += nthr) {
            const int k = PPC == 2 && idx >= n0 ? 1 : 0;
            const uint32_t* S0 = (const uint32_t*)(slot + (2 * k) * npw * 1024);
            const uint32_t* S1 = (const uint32_t*)(slot + (2 * k + 1) * npw * 1024);
            const int32_t* pt = ltab + (PPC * chk + k) * kPairTab;
            const int k0 = pt[0] & 1;
            int16_t* buf = (int16_t*)(lds_raw + exp0) + ((cc & 1) * PPC + k) * (umax * 4 * ws);
            {
                int u = 0, uu = idx - (k ? n0 : 0);
#pragma unroll
                for (int m = 1; m < kPairUMax; m++)
                    if (uu >= up8) { uu -= up8; u++; }
                uint32_t A[6], B[6], P[6];
                load12_shift(S0, k0 + 8 * uu, A);
                load12_shift(S1, pt[3 + u] + 8 * uu, B);
#pragma unroll
                for (int m = 0; m < 6; m++)
                    P[m] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2v, A[m]) + __builtin_bit_cast(short2v, B[m]));
                uint4* dst0 = (uint4*)(buf + (u * 4) * ws);
                const uint32_t h1 = __builtin_amdgcn_alignbit(P[1], P[0], 16);
                const uint32_t h3 = __builtin_amdgcn_alignbit(P[2], P[1], 16);
                const uint32_t h5 = __builtin_amdgcn_alignbit(P[3], P[2], 16);
                const uint32_t h7 = __builtin_amdgcn_alignbit(P[4], P[3], 16);
                const uint32_t h9 = __builtin_amdgcn_alignbit(P[5], P[4], 16);
                dst0[uu] = make_uint4(P[0], P[1], P[2], P[3]);
                dst0[up8 + uu] = make_uint4(h1, h3, h5, h7);
                dst0[2 * up8 + uu] = make_uint4(P[1], P[2], P[3], P[4]);
                dst0[3 * up8 + uu] = make_uint4(h3, h5, h7, h9);
            }
        }
    };

    auto flush = [&](int tile) {
        const int64_t t0 = (int64_t)tile * T;
        widen();
    #pragma unroll
        for (int q = 0; q < Q; q++) {
            const int dl = wave * Q + q;
            const int d = dblk0 + dl;
            const bool dv = dl < dpb && d < a.numdms;
            int64_t part = 0;
    #pragma unroll
            for (int r = 0; r < R; r++) {
                const int64_t tl = t0 + 256 * r + 4 * lane;
                if (dv && !(PRB && (a.probe & 4))) {
                    float* o = P.out + (int64_t)d * a.out_stride + tl;
                    if (tl + 3 < a.nvalid) {
                        *(float4*)o = make_float4((float)acc32[q][r][0], (float)acc32[q][r][1], (float)acc32[q][r][2],
                                                  (float)acc32[q][r][3]);
                        part += (int64_t)acc32[q][r][0] + acc32[q][r][1] + acc32[q][r][2] + acc32[q][r][3];
                    } else {
    #pragma unroll
                        for (int j = 0; j < 4; j++)
                            if (tl + j < a.nvalid) {
                                o[j] = (float)acc32[q][r][j];
                                part += acc32[q][r][j];
                            }
                    }
                }
            }
            if (dv && P.partial && (a.partial_ndm == 0 || d < a.partial_ndm)) {   // (uniform per wave)
    #pragma unroll
                for (int m = 32; m >= 1; m >>= 1) part += __shfl_xor(part, m, 64);
                if (lane == 0) P.partial[(int64_t)d * a.ntiles + tile] = (double)part;
            }
        }
        gcount = 0;
#pragma unroll
        for (int q = 0; q < Q; q++)
#pragma unroll
            for (int r = 0; r < R; r++) {
#pragma unroll
                for (int j = 0; j < 4; j++) acc32[q][r][j] = 0;
                acc16[q][r][0] = short2v{0, 0};
                acc16[q][r][1] = short2v{0, 0};
            }
    };

#pragma unroll
    for (int cc = 0; cc < NS - 1; cc++) dma(cc);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NS - 3) : "memory");
    ring_barrier();
    expand(0, 0);
    ring_barrier();

    int chk = 0, ktile = 0;                            // chunk (within the tile) and tile of chunk c
    for (int c = 0; c < ntot; c++) {
        if (!(PRB && (a.probe & 2))) dma(c + NS - 1);   // probe 2: no window DMA after the prologue
        const int chn = chk + 1 == nchunk ? 0 : chk + 1;
        if (c + 1 < ntot && !(PRB && (a.probe & 8))) expand(c + 1, chn);
        // this chunk's per-DM byte offsets: pair k, DM entry q in lane q of voff[k]
        const int32_t* sboff = (const int32_t*)(lds_raw + ring0 + (c % NS) * slot_bytes + 2 * PPC * npw * 1024);
        int voff[PPC];
#pragma unroll
        for (int k = 0; k < PPC; k++) voff[k] = lane < Q ? sboff[k * dpb + wave * Q + lane] : 0;
        if (!(PRB && (a.probe & 1))) {
            constexpr int nsteps = PPC * Q, LA0 = ring_la<Q, R>() < Q - 1 ? ring_la<Q, R>() : Q - 1, LA = LA0;
            uint64_t bb[LA + 1][R];
#pragma unroll
            for (int e = 0; e < LA; e++)
                lds_read_r<R>(bb[e], (uint32_t)__builtin_amdgcn_readlane(voff[e / Q], e % Q) + lane_byte);
#pragma unroll
            for (int e = 0; e < nsteps; e++) {
                uint64_t (&cur)[R] = bb[e % (LA + 1)];
                if (e + LA < nsteps) {
                    lds_read_r<R>(bb[(e + LA) % (LA + 1)],
                                  (uint32_t)__builtin_amdgcn_readlane(voff[(e + LA) / Q], (e + LA) % Q) + lane_byte);
                    lds_wait_n<LA * R>(cur);
                } else if (e + 3 == nsteps && LA >= 2) {
                    lds_wait_n<2 * R>(cur);
                } else if (e + 2 == nsteps && LA >= 1) {
                    lds_wait_n<R>(cur);
                } else {
                    lds_wait_n<0>(cur);
                }
                const int q = e % Q;
#pragma unroll
                for (int r = 0; r < R; r++) {
                    acc16[q][r][0] += __builtin_bit_cast(short2v, (uint32_t)cur[r]);
                    acc16[q][r][1] += __builtin_bit_cast(short2v, (uint32_t)(cur[r] >> 32));
                }
                if (q == Q - 1 && ++gcount == G) {                // one pair done: widen every G pairs
                    gcount = 0;
                    widen();
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NS - 3) : "memory");
        ring_barrier();
        // tile done: its stores go out after this chunk's DMA wait, so they do not hold it up
        if (chk == nchunk - 1) flush(tb + ktile++);
        chk = chn;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the workgroup ends

}


// ---- register-window pair kernel ---------------------------------------------------------
// acc[i] += element (k + i) of the lane's 24-element window w (12 dwords, 2 int16 each),
// i = 0..11, for a wave-uniform shift k = 0..10: a jump into one of 11 straight-line cases
// of 12 SDWA adds (word selects fixed per case), so the accumulators and the window stay in
// fixed registers and nothing is moved.  The words are sign-extended (sext): the partials
// are int16 (|P| <= 32767 by the host's bound), negative for signed subbands.  jc = the case's byte offset from Lpc: 12 + 100 * k
// (the three instructions after s_getpc_b64 are 12 bytes; a case is 12 x 8-byte SDWA adds +
// a 4-byte s_branch).  The host table carries jc; the kernel clamps k before it gets here.
__device__ __forceinline__ void rw_add12(int (&A)[12], const uint32_t (&w)[12], uint32_t jc)
{
    asm volatile(
        "s_getpc_b64 s[98:99]\n"
        "Lpc_%=:\n\t"
        "s_add_u32 s98, s98, %24\n\t"
        "s_addc_u32 s99, s99, 0\n\t"
        "s_setpc_b64 s[98:99]\n"
        "L0_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%12) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %1, %1, sext(%12) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %2, %2, sext(%13) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %3, %3, sext(%13) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %4, %4, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %5, %5, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %6, %6, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %7, %7, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %8, %8, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %9, %9, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %10, %10, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %11, %11, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "s_branch Lend_%=\n\t"
        "L1_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%12) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %1, %1, sext(%13) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %2, %2, sext(%13) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %3, %3, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %4, %4, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %5, %5, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %6, %6, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %7, %7, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %8, %8, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %9, %9, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %10, %10, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %11, %11, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "s_branch Lend_%=\n\t"
        "L2_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%13) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %1, %1, sext(%13) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %2, %2, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %3, %3, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %4, %4, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %5, %5, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %6, %6, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %7, %7, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %8, %8, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %9, %9, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %10, %10, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %11, %11, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "s_branch Lend_%=\n\t"
        "L3_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%13) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %1, %1, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %2, %2, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %3, %3, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %4, %4, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %5, %5, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %6, %6, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %7, %7, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %8, %8, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %9, %9, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %10, %10, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %11, %11, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "s_branch Lend_%=\n\t"
        "L4_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %1, %1, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %2, %2, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %3, %3, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %4, %4, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %5, %5, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %6, %6, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %7, %7, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %8, %8, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %9, %9, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %10, %10, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %11, %11, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "s_branch Lend_%=\n\t"
        "L5_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%14) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %1, %1, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %2, %2, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %3, %3, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %4, %4, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %5, %5, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %6, %6, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %7, %7, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %8, %8, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %9, %9, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %10, %10, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %11, %11, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "s_branch Lend_%=\n\t"
        "L6_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %1, %1, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %2, %2, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %3, %3, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %4, %4, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %5, %5, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %6, %6, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %7, %7, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %8, %8, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %9, %9, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %10, %10, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %11, %11, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "s_branch Lend_%=\n\t"
        "L7_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%15) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %1, %1, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %2, %2, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %3, %3, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %4, %4, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %5, %5, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %6, %6, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %7, %7, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %8, %8, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %9, %9, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %10, %10, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %11, %11, sext(%21) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "s_branch Lend_%=\n\t"
        "L8_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %1, %1, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %2, %2, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %3, %3, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %4, %4, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %5, %5, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %6, %6, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %7, %7, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %8, %8, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %9, %9, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %10, %10, sext(%21) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %11, %11, sext(%21) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "s_branch Lend_%=\n\t"
        "L9_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%16) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %1, %1, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %2, %2, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %3, %3, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %4, %4, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %5, %5, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %6, %6, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %7, %7, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %8, %8, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %9, %9, sext(%21) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %10, %10, sext(%21) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %11, %11, sext(%22) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "s_branch Lend_%=\n\t"
        "L10_%=:\n\t"
        "v_add_u32_sdwa %0, %0, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %1, %1, sext(%17) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %2, %2, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %3, %3, sext(%18) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %4, %4, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %5, %5, sext(%19) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %6, %6, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %7, %7, sext(%20) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %8, %8, sext(%21) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %9, %9, sext(%21) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_add_u32_sdwa %10, %10, sext(%22) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %11, %11, sext(%22) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "s_branch Lend_%=\n\t"
        "Lend_%=:"
        : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]), "+v"(A[4]), "+v"(A[5]), "+v"(A[6]), "+v"(A[7]),
          "+v"(A[8]), "+v"(A[9]), "+v"(A[10]), "+v"(A[11])
        : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]), "v"(w[8]),
          "v"(w[9]), "v"(w[10]), "v"(w[11]), "s"(jc)
        : "s98", "s99", "scc");
}

// Register-window pair kernel (k_stage2_rw).  The pair partials P_u of each subband pair are
// formed once per tile in ONE copy (not four shifted ones), and each wave reads, per pair, a
// 24-element window per lane that serves all of its Q DMs: lane l owns the 12 contiguous
// output samples 12l .. 12l+11 of a 768-sample tile, so a DM whose pattern offset lies
// within 10 elements of the window base takes its 12 values out of the lane's registers
// (rw_add12: a jump to the case of its shift, 12 SDWA adds) instead of three LDS reads of its
// own.  One window load (6 ds_read_b64) serves ~4 DMs; the expand writes a quarter of the
// bytes.  8 waves x Q DMs per workgroup, <= 80 KiB of LDS and <= 128 VGPRs, so two
// workgroups share a CU and one's barriers and DMA waits overlap the other's work.
// Host tables (rw_tables): per (y-block, pair) {base0, b1, U, k1[U]} as the pair kernel;
// per (y-block, chunk) a 256-int block DMA'd with the chunk: [pair k][DM] jump codes
// 12 + 100 * shift, then [pair k][wave] {reload mask, window byte offsets (<= 5)} (8 ints).
constexpr int kRwNW = 8, kRwNS = 4, kRwPPC = 2, kRwT = 768, kRwBlk = 256;

__device__ __forceinline__ void rw_load_win(uint32_t (&w)[12], uint32_t addr)
{
    uint64_t b[6];
#pragma unroll
    for (int j = 0; j < 6; j++) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(b[j]) : "v"(addr), "i"(8 * j));
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]));
#pragma unroll
    for (int j = 0; j < 6; j++) {
        w[2 * j] = (uint32_t)b[j];
        w[2 * j + 1] = (uint32_t)(b[j] >> 32);
    }
}

// Wait until only this wave's pieces of the most recent chunk (mine per chunk) may still be
// in flight: the chunk before it has landed (and every store issued before).
__device__ __forceinline__ void rw_wait_vm(int mine)
{
    if (mine >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (mine == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (mine == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int Q>
__global__ __launch_bounds__(512, 4) void k_stage2_rw(Stage2Args a, S2Multi m)
{
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    constexpr int NS = kRwNS, PPC = kRwPPC, T = kRwT, NW = kRwNW;
    const int pi = (int)blockIdx.y / m.nyblk;
    const S2Pass& P = m.p[pi];
    int tb, ntl;
    if (a.nwg == 0) {
        tb = xcd_remap(blockIdx.x, gridDim.x);
        ntl = 1;
    } else {
        const int nt = (int)((a.nvalid + T - 1) / T);
        tb = (int)((int64_t)blockIdx.x * nt / gridDim.x);
        ntl = (int)((int64_t)(blockIdx.x + 1) * nt / gridDim.x) - tb;
    }
    const int yb = (int)blockIdx.y - pi * m.nyblk;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int nthr = 64 * NW;
    constexpr int dpb = NW * Q;
    const int dblk0 = yb * dpb;
    const int ws = P.ws;
    const int npw = P.npw;
    const int umax = P.umax;
    const int nwin = 2 * PPC * npw;                       // window pieces of a chunk
    const int slot_bytes = (nwin + 1) * 1024;
    const int npair = a.nsub >> 1;
    const int nchunk = npair / PPC;
    int32_t* ltab = (int32_t*)lds_raw;
    const uint32_t ring0 = (uint32_t)(npair * kPairTab * 4);
    const uint32_t exp0 = ring0 + (uint32_t)(NS * slot_bytes);
    const int16_t* sub = (const int16_t*)P.sub;
    const int32_t* bo_g = P.off + (int64_t)yb * nchunk * kRwBlk;

    for (int i = threadIdx.x; i < npair * kPairTab; i += nthr) ltab[i] = P.ptab[(int64_t)yb * npair * kPairTab + i];
    __syncthreads();

    int acc[Q][12];
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int i = 0; i < 12; i++) acc[q][i] = 0;

    const int ntot = ntl * nchunk;
    int dchunk = 0, dtile = 0, dcount = 0;
    auto dma = [&](int cc) {
        const int c2 = dchunk;
        const int64_t t0 = (int64_t)(tb + dtile) * T;
        if (dcount + 1 < ntot) {
            dcount++;
            if (++dchunk == nchunk) { dchunk = 0; dtile++; }
        }
        const uint32_t slot = ring0 + (uint32_t)((cc % NS) * slot_bytes);
        for (int pc = wave; pc <= nwin; pc += NW) {
            if (pc < nwin) {
                const int sl = pc / npw, pw = pc - sl * npw;      // window sl: pair sl / 2, side sl % 2
                const int pr = PPC * c2 + (sl >> 1);
                const int s = 2 * pr + (sl & 1);
                const int b = __builtin_amdgcn_readfirstlane(ltab[pr * kPairTab + (sl & 1)]);
                const int64_t e0 = t0 + b - (b & 1);
                const char* src = (const char*)(sub + (int64_t)s * P.sub_stride + e0) + pw * 1024;
                dma16s(src, (uint32_t)lane * 16u, slot + (uint32_t)(pc * 1024));
            } else {
                dma16s((const char*)(bo_g + (int64_t)c2 * kRwBlk), (uint32_t)lane * 16u, slot + (uint32_t)(pc * 1024));
            }
        }
    };
    // staging slot of chunk cc -> one copy of each pattern partial of its pairs, buffers
    // ((cc & 1) * PPC + k) x umax patterns x ws elements
    auto expand = [&](int cc, int chk) {
        const char* slot = lds_raw + ring0 + (cc % NS) * slot_bytes;
#pragma unroll
        for (int k = 0; k < PPC; k++) {
            const uint32_t* S0 = (const uint32_t*)(slot + (2 * k) * npw * 1024);
            const uint32_t* S1 = (const uint32_t*)(slot + (2 * k + 1) * npw * 1024);
            const int32_t* pt = ltab + (PPC * chk + k) * kPairTab;
            const int k0 = pt[0] & 1;
            const int U = pt[2];
            int16_t* buf = (int16_t*)(lds_raw + exp0) + ((cc & 1) * PPC + k) * (umax * ws);
            const int up8 = ws >> 3;
            for (int idx = threadIdx.x; idx < U * up8; idx += nthr) {
                int u = 0, uu = idx;
#pragma unroll
                for (int mm = 1; mm < kPairUMax; mm++)
                    if (uu >= up8) { uu -= up8; u++; }
                uint32_t A[4], B[4];
                load8_shift64(S0, k0 + 8 * uu, A);
                load8_shift64(S1, pt[3 + u] + 8 * uu, B);
                uint32_t Pv[4];
#pragma unroll
                for (int mm = 0; mm < 4; mm++)
                    Pv[mm] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2v, A[mm]) + __builtin_bit_cast(short2v, B[mm]));
                *(uint4*)(buf + u * ws + 8 * uu) = make_uint4(Pv[0], Pv[1], Pv[2], Pv[3]);
            }
        }
    };
    auto flush = [&](int tile) {
        const int64_t t0 = (int64_t)tile * T;
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const int dl = wave * Q + q;
            const int d = dblk0 + dl;
            const bool dv = d < a.numdms;
            int64_t part = 0;
            if (dv && !(a.probe & 4)) {
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    const int64_t tl = t0 + 12 * lane + 4 * j;
                    float* o = P.out + (int64_t)d * a.out_stride + tl;
                    if (tl + 3 < a.nvalid) {
                        *(float4*)o = make_float4((float)acc[q][4 * j], (float)acc[q][4 * j + 1], (float)acc[q][4 * j + 2],
                                                  (float)acc[q][4 * j + 3]);
                        part += (int64_t)acc[q][4 * j] + acc[q][4 * j + 1] + acc[q][4 * j + 2] + acc[q][4 * j + 3];
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; i++)
                            if (tl + i < a.nvalid) {
                                o[i] = (float)acc[q][4 * j + i];
                                part += acc[q][4 * j + i];
                            }
                    }
                }
            }
            if (dv && P.partial && (a.partial_ndm == 0 || d < a.partial_ndm)) {   // (uniform per wave)
#pragma unroll
                for (int mm = 32; mm >= 1; mm >>= 1) part += __shfl_xor(part, mm, 64);
                if (lane == 0) P.partial[(int64_t)d * a.ntiles + tile] = (double)part;
            }
#pragma unroll
            for (int i = 0; i < 12; i++) acc[q][i] = 0;
        }
    };

    // this wave's DMA pieces per chunk (nwin + 1 pieces over NW waves)
    const int mine = wave <= nwin ? (nwin - wave) / NW + 1 : 0;
#pragma unroll
    for (int cc = 0; cc < NS - 1; cc++) dma(cc);
    rw_wait_vm(mine);
    ring_barrier();
    expand(0, 0);
    ring_barrier();

    int chk = 0, ktile = 0;
    for (int c = 0; c < ntot; c++) {
        if (!(a.probe & 2)) dma(c + NS - 1);
        const int chn = chk + 1 == nchunk ? 0 : chk + 1;
        if (c + 1 < ntot && !(a.probe & 8)) expand(c + 1, chn);
        if (!(a.probe & 1)) {
            const int32_t* sb = (const int32_t*)(lds_raw + ring0 + (c % NS) * slot_bytes + nwin * 1024);
#pragma unroll
            for (int k = 0; k < PPC; k++) {
                const int jcv = lane < Q ? sb[k * dpb + wave * Q + lane] : 0;
                const int rec = lane < 8 ? sb[PPC * dpb + (k * NW + wave) * 8 + lane] : 0;
                const uint32_t mask = (uint32_t)__builtin_amdgcn_readlane(rec, 0);
                uint32_t w[12];
                rw_load_win(w, exp0 + (uint32_t)__builtin_amdgcn_readlane(rec, 1) + 24u * (uint32_t)lane);
                int nwn = 2;
#pragma unroll
                for (int q = 0; q < Q; q++) {
                    if (q > 0 && ((mask >> q) & 1u)) {
                        rw_load_win(w, exp0 + (uint32_t)__builtin_amdgcn_readlane(rec, nwn) + 24u * (uint32_t)lane);
                        nwn = nwn < 5 ? nwn + 1 : 5;
                    }
                    const uint32_t jc = min((uint32_t)__builtin_amdgcn_readlane(jcv, q), 1012u);
                    rw_add12(acc[q], w, jc);
                }
            }
        }
        rw_wait_vm(a.probe & 2 ? 0 : mine);
        ring_barrier();
        if (chk == nchunk - 1) flush(tb + ktile++);
        chk = chn;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

size_t stage2_rw_lds_bytes(int ws, int npw, int nsub, int umax)
{
    return (size_t)(nsub / 2) * kPairTab * 4 + (size_t)kRwNS * (2 * kRwPPC * npw + 1) * 1024 +
           (size_t)2 * kRwPPC * umax * ws * 2;
}

template <int Q>
static hipError_t launch_rw_q(const Stage2Args& a, const S2Multi& m, int nyblk, hipStream_t st)
{
    {
        const hipError_t e = set_max_lds((const void*)k_stage2_rw<Q>, 80 * 1024);
        if (e != hipSuccess) return e;
    }
    const unsigned ntiles = (unsigned)((a.nvalid + kRwT - 1) / kRwT);
    const unsigned nx = a.nwg > 0 && (unsigned)a.nwg < ntiles ? (unsigned)a.nwg : ntiles;
    Stage2Args b = a;
    if (nx == ntiles) b.nwg = 0;
    size_t lds = 0;
    for (int i = 0; i < m.npass; i++)
        lds = std::max(lds, stage2_rw_lds_bytes(m.p[i].ws, m.p[i].npw, a.nsub, m.p[i].umax));
    if (lds > 80 * 1024) return hipErrorInvalidValue;
    S2Multi mm = m;
    mm.nyblk = nyblk;
    hipLaunchKernelGGL((k_stage2_rw<Q>), dim3(nx, (unsigned)(nyblk * m.npass)), dim3(64 * kRwNW), lds, st, b, mm);
    return hipGetLastError();
}

hipError_t launch_stage2_rw_multi(const Stage2Args& a, const S2Multi& m, int q, hipStream_t st)
{
    if (a.nvalid <= 0 || m.npass <= 0) return hipSuccess;
    if (m.npass > kS2MaxPass || a.dms_per_blk != kRwNW * q) return hipErrorInvalidValue;
    const int nyblk = (a.numdms + a.dms_per_blk - 1) / a.dms_per_blk;
    switch (q) {
    case 1: return launch_rw_q<1>(a, m, nyblk, st);
    case 2: return launch_rw_q<2>(a, m, nyblk, st);
    case 3: return launch_rw_q<3>(a, m, nyblk, st);
    case 4: return launch_rw_q<4>(a, m, nyblk, st);
    case 5: return launch_rw_q<5>(a, m, nyblk, st);
    default: return hipErrorInvalidValue;
    }
}

size_t stage2_pair_lds_bytes(int wstride, int npw, int nbp, int nsub, int umax, int ppc)
{
    const int ns = ppc == 2 ? 4 : kRingNS;
    return (size_t)(nsub / 2) * kPairTab * 4 + (size_t)ns * (2 * ppc * npw + nbp) * 1024 +
           (size_t)2 * ppc * umax * 4 * wstride * 2;
}

template <int Q, int R, int PPC, bool NN, bool PRB>
static hipError_t launch_pair_qrpn(const Stage2Args& a, const S2Multi& m, int nyblk, hipStream_t st)
{
    {
        const hipError_t e = set_max_lds((const void*)k_stage2_pair<Q, R, PPC, NN, PRB>, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    const unsigned ntiles = (unsigned)((a.nvalid + 256 * R - 1) / (256 * R));
    const unsigned nx = a.nwg > 0 && (unsigned)a.nwg < ntiles ? (unsigned)a.nwg : ntiles;
    Stage2Args b = a;
    if (nx == ntiles) b.nwg = 0;
    size_t lds = 0;
    for (int i = 0; i < m.npass; i++)
        lds = std::max(lds, stage2_pair_lds_bytes(m.p[i].ws, m.p[i].npw, m.p[i].nbp, a.nsub, m.p[i].umax, PPC));
    S2Multi mm = m;
    mm.nyblk = nyblk;
    hipLaunchKernelGGL((k_stage2_pair<Q, R, PPC, NN, PRB>), dim3(nx, (unsigned)(nyblk * m.npass)), dim3(1024), lds, st, b,
                       mm);
    return hipGetLastError();
}

// non-negative subbands (host-known): unsigned packed halves, twice the group (probe 64 keeps
// the signed kernel for A/B)
template <int Q, int R, int PPC>
static hipError_t launch_pair_qrp(const Stage2Args& a, const S2Multi& m, int nyblk, hipStream_t st)
{
    const bool prb = (a.probe & 15) != 0;
    if (a.nonneg && !(a.probe & 64))
        return prb ? launch_pair_qrpn<Q, R, PPC, true, true>(a, m, nyblk, st)
                   : launch_pair_qrpn<Q, R, PPC, true, false>(a, m, nyblk, st);
    return prb ? launch_pair_qrpn<Q, R, PPC, false, true>(a, m, nyblk, st)
               : launch_pair_qrpn<Q, R, PPC, false, false>(a, m, nyblk, st);
}

// Two workgroups per CU: 8 waves x Q DMs (<= 40) per workgroup, one LDS window buffer, no
// register prefetch.  While one workgroup waits for its chunk's loads and barriers, the other
// accumulates; the subband windows of a tile are filled once per 40-DM y-block.
template <int Q, int R, int SC>
__global__ __launch_bounds__(512, 2) void k_stage2_wide2(Stage2Args a, const int32_t* __restrict__ boff)
{
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    int16_t* lds = (int16_t*)lds_raw;
    constexpr int T = 256 * R;
    constexpr int UM = 4;                       // fill units per thread per chunk (host check)
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t t0 = (int64_t)tile * T;
    const int yb = blockIdx.y;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nthr = blockDim.x;
    const int dpb = a.dms_per_blk;
    const int dblk0 = yb * dpb;
    const int ws = a.wstride;
    const int upw = ws >> 2;
    const int16_t* sub = (const int16_t*)a.sub;
    const int32_t* bo = boff + (int64_t)yb * a.nsub * dpb + wave * Q;
    const int nchunk = a.nsub / SC;
    int32_t* lomin = (int32_t*)(lds_raw + (size_t)SC * 4 * ws * 2);
    for (int i = threadIdx.x; i < a.nsub; i += nthr) lomin[i] = a.omin[(int64_t)yb * a.nsub + i];

    int maxabs = *a.maxabs;
    maxabs = maxabs < 1 ? 1 : maxabs;
    int G = 32767 / maxabs;
    G = G < 1 ? 1 : (G > 64 ? 64 : G);
    G = __builtin_amdgcn_readfirstlane(G);

    int acc32[Q][R][4];
    short2v acc16[Q][R][2];
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int r = 0; r < R; r++) {
#pragma unroll
            for (int j = 0; j < 4; j++) acc32[q][r][j] = 0;
            acc16[q][r][0] = short2v{0, 0};
            acc16[q][r][1] = short2v{0, 0};
        }
    int gcount = 0;
    const uint32_t lane_byte = (uint32_t)lane * 8u;
    constexpr int NR = (SC * Q + 63) / 64;
    __syncthreads();

    for (int c = 0; c < nchunk; c++) {
        const int s0 = c * SC;
        int voff[NR];
#pragma unroll
        for (int i = 0; i < NR; i++) {
            const int e = i * 64 + lane;
            const int sl = e / Q, q = e - (e / Q) * Q;
            voff[i] = (sl < SC) ? bo[(int64_t)(s0 + sl) * dpb + q] : 0;
        }
        // ---- fill: UM units per thread per round, all loads first, then the 4 shifted copies
        for (int ub = 0; ub < SC * upw && !(a.probe & 2); ub += UM * nthr) {
            uint32_t D[UM][4];
            int pb[UM], usl[UM], uuu[UM];
#pragma unroll
            for (int i = 0; i < UM; i++) {
                const int u = ub + threadIdx.x + i * nthr;
                usl[i] = u < SC * upw ? u / upw : SC;
                uuu[i] = u - usl[i] * upw;
                pb[i] = 0;
                if (usl[i] < SC) {
                    const int s = s0 + usl[i];
                    const int64_t wbeg = t0 + lomin[s];
                    const int p = (int)(wbeg & 1);
                    pb[i] = p;
                    const int16_t* srow = sub + (int64_t)s * a.sub_stride;
                    const int64_t e0 = wbeg + 4 * uuu[i] - p;
                    if (e0 + 8 <= a.nds) {
                        const u32x4a4 v = *(const u32x4a4*)(srow + e0);
                        D[i][0] = v.x;
                        D[i][1] = v.y;
                        D[i][2] = v.z;
                        D[i][3] = v.w;
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const int64_t e = e0 + 2 * j;
                            const uint32_t lo = e < a.nds ? (uint16_t)srow[e] : 0u;
                            const uint32_t hi = e + 1 < a.nds ? (uint16_t)srow[e + 1] : 0u;
                            D[i][j] = lo | (hi << 16);
                        }
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < UM; i++) {
                if (usl[i] < SC) {
                    uint2* dst0 = (uint2*)(lds + (usl[i] * 4) * ws);
                    const int u = uuu[i];
                    const uint32_t* Di = D[i];
#define HD_PAIR(h) (((h) & 1) ? __builtin_amdgcn_alignbit(Di[((h) + 1) >> 1], Di[(h) >> 1], 16) : Di[(h) >> 1])
                    if (pb[i] == 0) {
                        dst0[u] = make_uint2(HD_PAIR(0), HD_PAIR(2));
                        dst0[upw + u] = make_uint2(HD_PAIR(1), HD_PAIR(3));
                        dst0[2 * upw + u] = make_uint2(HD_PAIR(2), HD_PAIR(4));
                        dst0[3 * upw + u] = make_uint2(HD_PAIR(3), HD_PAIR(5));
                    } else {
                        dst0[u] = make_uint2(HD_PAIR(1), HD_PAIR(3));
                        dst0[upw + u] = make_uint2(HD_PAIR(2), HD_PAIR(4));
                        dst0[2 * upw + u] = make_uint2(HD_PAIR(3), HD_PAIR(5));
                        dst0[3 * upw + u] = make_uint2(HD_PAIR(4), HD_PAIR(6));
                    }
#undef HD_PAIR
                }
            }
        }
        __syncthreads();
        if (!(a.probe & 1)) {
            constexpr int nsteps = SC * Q;
            uint64_t b0[R], b1[R];
            lds_read_r<R>(b0, (uint32_t)__builtin_amdgcn_readlane(voff[0], 0) + lane_byte);
#pragma unroll
            for (int e = 0; e < nsteps; e++) {
                uint64_t (&cur)[R] = (e & 1) ? b1 : b0;
                uint64_t (&nxt)[R] = (e & 1) ? b0 : b1;
                if (e + 1 < nsteps) {
                    const int e1 = e + 1;
                    lds_read_r<R>(nxt, (uint32_t)__builtin_amdgcn_readlane(voff[e1 >> 6], e1 & 63) + lane_byte);
                    lds_wait_keep<R>(cur);
                } else {
                    lds_wait_all<R>(cur);
                }
                const int q = e % Q;
#pragma unroll
                for (int r = 0; r < R; r++) {
                    acc16[q][r][0] += __builtin_bit_cast(short2v, (uint32_t)cur[r]);
                    acc16[q][r][1] += __builtin_bit_cast(short2v, (uint32_t)(cur[r] >> 32));
                }
                if (q == Q - 1 && ++gcount == G) {
                    gcount = 0;
#pragma unroll
                    for (int qq = 0; qq < Q; qq++)
#pragma unroll
                        for (int r = 0; r < R; r++) {
                            acc32[qq][r][0] += acc16[qq][r][0].x;
                            acc32[qq][r][1] += acc16[qq][r][0].y;
                            acc32[qq][r][2] += acc16[qq][r][1].x;
                            acc32[qq][r][3] += acc16[qq][r][1].y;
                            acc16[qq][r][0] = short2v{0, 0};
                            acc16[qq][r][1] = short2v{0, 0};
                        }
                }
            }
        }
        __syncthreads();
    }

#pragma unroll
    for (int q = 0; q < Q; q++) {
        const int dl = wave * Q + q;
        const int d = dblk0 + dl;
        const bool dv = dl < dpb && d < a.numdms;
        int64_t part = 0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            acc32[q][r][0] += acc16[q][r][0].x;
            acc32[q][r][1] += acc16[q][r][0].y;
            acc32[q][r][2] += acc16[q][r][1].x;
            acc32[q][r][3] += acc16[q][r][1].y;
            const int64_t tl = t0 + 256 * r + 4 * lane;
            if (dv && !(a.probe & 4)) {
                float* o = a.out + (int64_t)d * a.out_stride + tl;
                if (tl + 3 < a.nvalid) {
                    *(float4*)o = make_float4((float)acc32[q][r][0], (float)acc32[q][r][1], (float)acc32[q][r][2],
                                              (float)acc32[q][r][3]);
                    part += (int64_t)acc32[q][r][0] + acc32[q][r][1] + acc32[q][r][2] + acc32[q][r][3];
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (tl + j < a.nvalid) {
                            o[j] = (float)acc32[q][r][j];
                            part += acc32[q][r][j];
                        }
                }
            }
        }
        if (dv && a.partial) {
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) part += __shfl_xor(part, m, 64);
            if (lane == 0) a.partial[(int64_t)d * a.ntiles + tile] = (double)part;
        }
    }
}

size_t stage2_wide2_lds_bytes(int wstride, int sc, int nsub) { return (size_t)sc * 4 * wstride * 2 + (size_t)nsub * 4; }

template <int Q, int R, int SC>
static hipError_t launch_wide2_qrs(const Stage2Args& a, int nw, int nyblk, hipStream_t st)
{
    {
        const hipError_t e = set_max_lds((const void*)k_stage2_wide2<Q, R, SC>, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    const unsigned ntiles = (unsigned)((a.nvalid + 256 * R - 1) / (256 * R));
    hipLaunchKernelGGL((k_stage2_wide2<Q, R, SC>), dim3(ntiles, (unsigned)nyblk), dim3((unsigned)(64 * nw)),
                       stage2_wide2_lds_bytes(a.wstride, SC, a.nsub), st, a, a.off);
    return hipGetLastError();
}

hipError_t launch_stage2_wide2(const Stage2Args& a, int q, int r, int nw, hipStream_t st)
{
    if (a.nvalid <= 0) return hipSuccess;
    const int nyblk = (a.numdms + a.dms_per_blk - 1) / a.dms_per_blk;
#define HD_W2(QQ, RR)                                                                   \
    if (q == QQ && r == RR) {                                                           \
        if (a.sc == 8) return launch_wide2_qrs<QQ, RR, 8>(a, nw, nyblk, st);            \
        if (a.sc == 4) return launch_wide2_qrs<QQ, RR, 4>(a, nw, nyblk, st);            \
    }
    HD_WIDE_QR(HD_W2)
#undef HD_W2
    return hipErrorInvalidValue;
}

// ring variant: 16 waves (nw is fixed by the host to 16 whenever the ring applies)
hipError_t launch_stage2_ring(const Stage2Args& a, int q, int r, hipStream_t st)
{
    if (a.nvalid <= 0) return hipSuccess;
    const int nyblk = (a.numdms + a.dms_per_blk - 1) / a.dms_per_blk;
#define HD_RL(QQ, RR) if (q == QQ && r == RR) return launch_ring_qr<QQ, RR>(a, nyblk, st);
    HD_RING_QR(HD_RL)
#undef HD_RL
    return hipErrorInvalidValue;
}

S2Pass stage2_pass_of(const Stage2Args& a)
{
    S2Pass p{};
    p.sub = a.sub;
    p.ptab = a.ptab;
    p.off = a.off;
    p.maxabs = a.maxabs;
    p.out = a.out;
    p.partial = a.partial;
    p.sub_stride = a.sub_stride;
    p.ws = a.wstride;
    p.npw = a.ring_npw;
    p.nbp = a.ring_nbp;
    p.umax = a.umax;
    p.setb = a.qp_setb;
    return p;
}

hipError_t launch_stage2_pair(const Stage2Args& a, int q, int r, int ppc, hipStream_t st)
{
    S2Multi m{};
    m.npass = 1;
    m.p[0] = stage2_pass_of(a);
    return launch_stage2_pair_multi(a, m, q, r, ppc, st);
}

hipError_t launch_stage2_pair_multi(const Stage2Args& a, const S2Multi& m, int q, int r, int ppc, hipStream_t st)
{
    if (a.nvalid <= 0 || m.npass <= 0) return hipSuccess;
    if (ppc != 1 && ppc != 2) return hipErrorInvalidValue;
    if (m.npass > kS2MaxPass) return hipErrorInvalidValue;
    const int nyblk = (a.numdms + a.dms_per_blk - 1) / a.dms_per_blk;
#define HD_PL(QQ, RR)                                                                             \
    if (q == QQ && r == RR)                                                                       \
        return ppc == 2 ? launch_pair_qrp<QQ, RR, 2>(a, m, nyblk, st) : launch_pair_qrp<QQ, RR, 1>(a, m, nyblk, st);
    HD_RING_QR(HD_PL)
#undef HD_PL
    return hipErrorInvalidValue;
}

bool stage2_pair_supports(int q, int r) { return stage2_ring_supports(q, r); }

bool stage2_ring_supports(int q, int r)
{
#define HD_RS(QQ, RR) if (q == QQ && r == RR) return true;
    HD_RING_QR(HD_RS)
#undef HD_RS
    return false;
}

size_t stage2_wide_lds_bytes(int wstride, int sc) { return (size_t)2 * sc * 4 * wstride * sizeof(int16_t); }

template <int Q, int R, int SC>
static hipError_t launch_wide_qrs(const Stage2Args& a, int nw, int nyblk, hipStream_t st)
{
    {
        const hipError_t e = set_max_lds((const void*)k_stage2_wide<Q, R, SC>, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    const unsigned ntiles = (unsigned)((a.nvalid + 256 * R - 1) / (256 * R));
    hipLaunchKernelGGL((k_stage2_wide<Q, R, SC>), dim3(ntiles, (unsigned)nyblk), dim3((unsigned)(64 * nw)),
                       stage2_wide_lds_bytes(a.wstride, SC), st, a, a.off);
    return hipGetLastError();
}

template <int Q, int R>
static hipError_t launch_wide_qr(const Stage2Args& a, int nw, int nyblk, hipStream_t st)
{
    if (a.sc == 8) return launch_wide_qrs<Q, R, 8>(a, nw, nyblk, st);
    if (a.sc == 4) return launch_wide_qrs<Q, R, 4>(a, nw, nyblk, st);
    return hipErrorInvalidValue;
}


bool stage2_wide_supports(int q, int r)
{
#define HD_WS(QQ, RR) if (q == QQ && r == RR) return true;
    HD_WIDE_QR(HD_WS)
#undef HD_WS
    return false;
}

// boff is passed through Stage2Args.off (host-built [nyblk][nsub][nw*Q] byte offsets).
hipError_t launch_stage2_wide(const Stage2Args& a, int q, int r, int nw, hipStream_t st)
{
    if (a.nvalid <= 0) return hipSuccess;
    const int nyblk = (a.numdms + a.dms_per_blk - 1) / a.dms_per_blk;
#define HD_WL(QQ, RR) if (q == QQ && r == RR) return launch_wide_qr<QQ, RR>(a, nw, nyblk, st);
    HD_WIDE_QR(HD_WL)
#undef HD_WL
    return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------
// Quarter-layout pair kernel (k_stage2_qp, round 5).  The pair partials of k_stage2_pair,
// P_u[x] = sub[s0][base0 + x] + sub[s1][base0 + r_u + x], stored ONCE per tile in a
// quarter-interleaved layout instead of four shifted copies: entry e of pattern u holds the
// four int16 P_u[e], P_u[e + S], P_u[e + 2S], P_u[e + 3S] (8 bytes; tile T = 4 S samples,
// S = 64 RQ).  A DM whose pair offset is o then reads entries o + lane + 64 m (m < RQ) with one
// aligned ds_read_b64 each for ANY o -- four output samples (one per quarter) per read, as
// before -- but the expand writes 8 (S + span) bytes per pattern instead of 8 (T + span)
// (2.5x fewer LDS write cycles, the cost that dominated it), and a pattern's buffer is 2.5x
// smaller, so a chunk carries PPC = 3 or 4 pairs (fewer barriers) in the same 160 KiB.
// Per pair the entries cover only that pair's own DM sweep (S + span_k, not the plan's
// widest), which trims the expand of the high-frequency pairs.
// The staging windows stay plain (LDS-DMA of the subband rows); the expand reads 4 elements
// of each quarter (two aligned ds_read_b64 + a dword select + v_alignbit), adds the pair,
// and transposes the four quarters into entries with v_perm (two ds_write_b128 per item).
// Output lane l, read m, quarter j is sample t0 + j S + 64 m + l: dword stores, 256 bytes
// contiguous per wave-instruction.
// Table per (y-block, pair): [0] base0, [1] b1, [2] U, [3..3+U) k1[u], [9] E_k (entries,
// multiple of 4), [kQpPb + 4 - PPC] pb_k: the byte offset of the pair's U_k x E_k entries inside
// its chunk's buffer set (the chunk's pairs packed one after another, so a set holds the
// chunk's own patterns, not PPC x the plan's largest U x the largest E).  Offsets block per
// chunk: int32 LDS byte offsets from the expanded area, [pair k][DM slot] = (chunk & 1) * setb
// + pb_k + (u E_k + o2) * 8 (the host keeps one such table per pairs-per-chunk a launch may
// take; setb = the largest set over the chunks, per pairs-per-chunk).

// 4 int16 elements x .. x+3 of a staging window (any x) as 2 packed pairs: two aligned
// ds_read_b64 cover dwords (x>>1 & ~1) .. +3, a select picks the 3 that hold them.
__device__ __forceinline__ void qp_load4(const uint32_t* w32, int x, uint32_t& o0, uint32_t& o1)
{
    const int dw = x >> 1;
    const uint2 a = *(const uint2*)(w32 + (dw & ~1));
    const uint2 b = *(const uint2*)(w32 + (dw & ~1) + 2);
    const bool odd = dw & 1;
    const uint32_t w0 = odd ? a.y : a.x, w1 = odd ? b.x : a.y, w2 = odd ? b.y : b.x;
    const uint32_t sh = (uint32_t)(x & 1) * 16u;
    o0 = __builtin_amdgcn_alignbit(w1, w0, sh);
    o1 = __builtin_amdgcn_alignbit(w2, w1, sh);
}

template <int PPC>
constexpr int qp_ns() { return PPC >= 4 ? 3 : 4; }

// 16 waves per workgroup x Q = 4..5 DMs (4 waves per SIMD, 128 VGPRs).  (An 8-wave x 8..10 DM
// variant with 256 VGPRs was tried in round 5: the compiler spills its accumulators beyond one
// step of LDS read lookahead, which removed its point, and it was dropped.)
template <int Q>
constexpr int qp_nw() { return Q >= 6 ? 12 : 16; }

// LDS read lookahead of the sums (steps of RQ reads) in the VGPRs left beside the accumulators:
// one step fits beside the 90 accumulator registers
template <int Q, int RQ>
constexpr int qp_la() { return Q >= 6 ? 2 : 1; }

template <int Q, int RQ, int PPC, bool NN, bool PRB, int NS, bool SY>
__global__ __launch_bounds__(qp_nw<Q>() * 64) void k_stage2_qp(Stage2Args a, S2Multi m)
{
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    const int pi = (int)blockIdx.y / m.nyblk;
    const S2Pass& P = m.p[pi];
    constexpr int S = 64 * RQ, T = 4 * S, NW = qp_nw<Q>();
    static_assert(NS >= 3 && NS <= 4 && (!SY || NS == 3), "NS");
    int tb, ntl;
    if (a.nwg == 0) {
        tb = xcd_remap(blockIdx.x, gridDim.x);
        ntl = 1;
    } else {
        const int nt = (int)((a.nvalid + T - 1) / T);
        tb = (int)((int64_t)blockIdx.x * nt / gridDim.x);
        ntl = (int)((int64_t)(blockIdx.x + 1) * nt / gridDim.x) - tb;
    }
    const int yb = (int)blockIdx.y - pi * m.nyblk;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nthr = blockDim.x;
    const int dpb = a.dms_per_blk;
    const int dblk0 = yb * dpb;
    const int setb = P.setb;                     // bytes of one expanded buffer set (PPC pairs' patterns)
    const int npw = P.npw;                       // 1 KiB DMA pieces per window
    const int nbp = P.nbp;                       // pieces of a chunk's offset block
    const int npiece = 2 * PPC * npw + nbp;      // DMA pieces per chunk (<= 32: two per wave)
    const int pw = (npiece - wave + NW - 1) / NW;  // this wave's pieces per chunk: 0 .. 3
    const int slot_bytes = npiece * 1024;
    const int npair = a.nsub >> 1;
    const int tab_bytes = npair * kPairTab * 4;
    int32_t* ltab = (int32_t*)lds_raw;
    const uint32_t ring0 = (uint32_t)tab_bytes;
    const uint32_t exp0 = ring0 + (uint32_t)(NS * slot_bytes);
    const uint32_t lane_byte = exp0 + (uint32_t)lane * 8u;
    const int16_t* sub = (const int16_t*)P.sub;
    const int32_t* bo_g = P.off + (int64_t)yb * npair * dpb;
    const int nchunk = npair / PPC;

    for (int i = threadIdx.x; i < npair * kPairTab; i += nthr) ltab[i] = P.ptab[(int64_t)yb * npair * kPairTab + i];
    // SY: the two progress counters past the three expanded sets (see the SY loop below)
    uint32_t* ctr = (uint32_t*)(lds_raw + exp0 + 3 * setb);
    if (SY && threadIdx.x < 2) ctr[threadIdx.x] = 0;
    __syncthreads();

    int maxabs = *P.maxabs;
    maxabs = maxabs < 1 ? 1 : maxabs;
    const bool small_part = (int64_t)a.nsub * maxabs * (RQ * 4) * 32 < ((int64_t)1 << 31);
    int G = (NN ? 65535 : 32767) / (2 * maxabs);
    G = G < 1 ? 1 : (G > 64 ? 64 : G);
    G = __builtin_amdgcn_readfirstlane(G);

    int acc32[Q][RQ][4];
    short2v acc16[Q][RQ][2];
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int r = 0; r < RQ; r++) {
#pragma unroll
            for (int j = 0; j < 4; j++) acc32[q][r][j] = 0;
            acc16[q][r][0] = short2v{0, 0};
            acc16[q][r][1] = short2v{0, 0};
        }
    int gcount = 0;
    auto widen = [&]() {
#pragma unroll
        for (int qq = 0; qq < Q; qq++)
#pragma unroll
            for (int r = 0; r < RQ; r++) {
                if (NN) {
                    const uint32_t lo = __builtin_bit_cast(uint32_t, acc16[qq][r][0]);
                    const uint32_t hi = __builtin_bit_cast(uint32_t, acc16[qq][r][1]);
                    acc32[qq][r][0] += (int)(lo & 0xFFFFu);
                    acc32[qq][r][1] += (int)(lo >> 16);
                    acc32[qq][r][2] += (int)(hi & 0xFFFFu);
                    acc32[qq][r][3] += (int)(hi >> 16);
                } else {
                    acc32[qq][r][0] += acc16[qq][r][0].x;
                    acc32[qq][r][1] += acc16[qq][r][0].y;
                    acc32[qq][r][2] += acc16[qq][r][1].x;
                    acc32[qq][r][3] += acc16[qq][r][1].y;
                }
                acc16[qq][r][0] = short2v{0, 0};
                acc16[qq][r][1] = short2v{0, 0};
            }
    };

    const int ntot = ntl * nchunk;
    int dchunk = 0, dtile = 0, dcount = 0;
    // the DMA of one chunk: piece pc of the chunk from wave pc % 16 (pc / 16: its second piece)
    auto dma = [&](int cc) {
        const int c2 = dchunk;
        const int64_t t0 = (int64_t)(tb + dtile) * T;
        if (dcount + 1 < ntot) {
            dcount++;
            if (++dchunk == nchunk) { dchunk = 0; dtile++; }
        }
        const uint32_t slot = ring0 + (uint32_t)((cc % NS) * slot_bytes);
        for (int pc = wave; pc < npiece; pc += NW) {
            if (pc < 2 * PPC * npw) {
                const int win = pc / npw, pcs = pc - win * npw;      // window win: pair win / 2, side win % 2
                const int pr = PPC * c2 + (win >> 1);
                const int s = 2 * pr + (win & 1);
                const int b = __builtin_amdgcn_readfirstlane(ltab[pr * kPairTab + (win & 1)]);
                const int64_t e0 = t0 + b - (b & 1);
                const char* src = (const char*)(sub + (int64_t)s * P.sub_stride + e0) + pcs * 1024;
                dma16s(src, (uint32_t)lane * 16u, slot + (uint32_t)(pc * 1024));
            } else {
                const int bp = pc - 2 * PPC * npw;
                const char* src = (const char*)(bo_g + (int64_t)PPC * c2 * dpb) + bp * 1024;
                dma16s(src, (uint32_t)lane * 16u, slot + (uint32_t)(pc * 1024));
            }
        }
    };
    // wait until the next chunk's DMA is in LDS: at most DL chunks of this wave's pieces newer
    // than it (and nothing older: series stores included) outstanding.  (Issuing each chunk's
    // DMA one iteration earlier, with the offsets read into a register before the slot is
    // reused, measured slower: 34.3 vs 33.3 ms of stage 2 per beam.)
    constexpr int DL = NS - 3;
    auto wait_ring = [&]() {
        if constexpr (DL == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            if (pw >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * DL) : "memory");
            else if (pw == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * DL) : "memory");
            else if (pw == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(DL) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    };
    // staging slot of chunk cc -> quarter entries of every pattern of its PPC pairs.
    // Item (pair k, entry group g): entries 4g .. 4g+3 of each of the pair's U patterns.
    auto expand = [&](int cc, int chk) {
        const char* slot = lds_raw + ring0 + (cc % NS) * slot_bytes;
        int nk[PPC + 1];
        nk[0] = 0;
#pragma unroll
        for (int k = 0; k < PPC; k++) {
            const int32_t* pt = ltab + (PPC * chk + k) * kPairTab;
            nk[k + 1] = nk[k] + pt[2] * (pt[9] >> 2);
        }
        // item (pair k, pattern u, entry group g): entries 4g .. 4g+3 of pattern u
        for (int idx = threadIdx.x; idx < nk[PPC]; idx += nthr) {
            int k = 0;
#pragma unroll
            for (int kk = 1; kk < PPC; kk++)
                if (idx >= nk[kk]) k = kk;
            const int32_t* pt = ltab + (PPC * chk + k) * kPairTab;
            const int ng = pt[9] >> 2;
            int g = idx - nk[k], u = 0;
#pragma unroll
            for (int uu = 1; uu < kPairUMax; uu++)
                if (g >= ng) { g -= ng; u++; }
            const uint32_t* S0 = (const uint32_t*)(slot + (2 * k) * npw * 1024);
            const uint32_t* S1 = (const uint32_t*)(slot + (2 * k + 1) * npw * 1024);
            const int x0 = 4 * g + (pt[0] & 1), x1 = 4 * g + pt[3 + u];
            uint32_t Pq[4][2];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint32_t a0, a1, b0, b1;
                qp_load4(S0, x0 + j * S, a0, a1);
                qp_load4(S1, x1 + j * S, b0, b1);
                Pq[j][0] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2v, a0) + __builtin_bit_cast(short2v, b0));
                Pq[j][1] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2v, a1) + __builtin_bit_cast(short2v, b1));
            }
            // entry i = (q0, q1 | q2, q3) of element i: the low halves of a pair-dword are element 2h
            constexpr uint32_t LO = 0x05040100u, HI = 0x07060302u;
            uint4* d = (uint4*)(lds_raw + exp0 + (SY ? cc % 3 : cc & 1) * setb + pt[kQpPb + 4 - PPC]) + ((u * pt[9] + 4 * g) >> 1);
            d[0] = make_uint4(__builtin_amdgcn_perm(Pq[1][0], Pq[0][0], LO), __builtin_amdgcn_perm(Pq[3][0], Pq[2][0], LO),
                              __builtin_amdgcn_perm(Pq[1][0], Pq[0][0], HI), __builtin_amdgcn_perm(Pq[3][0], Pq[2][0], HI));
            d[1] = make_uint4(__builtin_amdgcn_perm(Pq[1][1], Pq[0][1], LO), __builtin_amdgcn_perm(Pq[3][1], Pq[2][1], LO),
                              __builtin_amdgcn_perm(Pq[1][1], Pq[0][1], HI), __builtin_amdgcn_perm(Pq[3][1], Pq[2][1], HI));
        }
    };

    auto flush = [&](int tile) {
        const int64_t t0 = (int64_t)tile * T;
        widen();
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const int dl = wave * Q + q;
            const int d = dblk0 + dl;
            const bool dv = dl < dpb && d < a.numdms;
            int64_t part = 0;
            if (dv && !(PRB && (a.probe & 4))) {
                float* o = P.out + (int64_t)d * a.out_stride + t0 + lane;
                if (t0 + T <= a.nvalid) {
#pragma unroll
                    for (int r = 0; r < RQ; r++)
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            o[j * S + 64 * r] = (float)acc32[q][r][j];
                            part += acc32[q][r][j];
                        }
                } else {
#pragma unroll
                    for (int r = 0; r < RQ; r++)
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            if (t0 + j * S + 64 * r + lane < a.nvalid) {
                                o[j * S + 64 * r] = (float)acc32[q][r][j];
                                part += acc32[q][r][j];
                            }
                }
            }
            if (dv && P.partial && (a.partial_ndm == 0 || d < a.partial_ndm)) {   // (uniform per wave)
                // (uniform) a lane's partial is at most RQ * 4 series values of |v| <= nsub *
                // max|subband|: when 32 of them fit int32, the DPP sum; else the int64 butterfly
                if (small_part) {
                    part = wave_sum_i32_small((int)part);
                } else {
#pragma unroll
                    for (int mm = 32; mm >= 1; mm >>= 1) part += __shfl_xor(part, mm, 64);
                }
                if (lane == 0) P.partial[(int64_t)d * a.ntiles + tile] = (double)part;
            }
        }
        gcount = 0;
#pragma unroll
        for (int q = 0; q < Q; q++)
#pragma unroll
            for (int r = 0; r < RQ; r++) {
#pragma unroll
                for (int j = 0; j < 4; j++) acc32[q][r][j] = 0;
                acc16[q][r][0] = short2v{0, 0};
                acc16[q][r][1] = short2v{0, 0};
            }
    };

    // this chunk's (pair, DM) byte offsets in ONE register: lane k * Q + q holds pair k, DM q
    auto read_voff = [&](int cc) {
        const int32_t* sboff = (const int32_t*)(lds_raw + ring0 + (cc % NS) * slot_bytes + 2 * PPC * npw * 1024);
        return lane < PPC * Q ? sboff[(lane / Q) * dpb + wave * Q + lane % Q] : 0;
    };
    // The offsets table places pair k of a tile's chunk chk in expanded buffer set (chk & 1),
    // while expand() writes the workgroup's running chunk c into set (c & 1): with an odd chunk
    // count per tile they differ on every other tile a persistent workgroup takes, so the sums
    // shift the table's offsets by one buffer set there (uniform, one scalar per chunk).
    const uint32_t set_bytes = (uint32_t)setb;
    // diagnostics: shader-clock stamps of each phase (PRB builds with a.stamps set), kept in the
    // LDS past the expanded sets and copied out at the end
    const bool stamping = PRB && a.stamps && blockIdx.x < kStampWG && blockIdx.y == 0;
    uint32_t* lst = (uint32_t*)(lds_raw + exp0 + (SY ? 3 * setb + 16 : 2 * setb));
    auto stamp = [&](int c, int ph) {
        if (stamping && c < kStampChunks) {
            const uint32_t t = (uint32_t)clock64();
            if (lane == 0) lst[(wave * kStampChunks + c) * kStampPh + ph] = t;
        }
    };
    // the sums of chunk c: PPC x Q steps of RQ aligned ds_read_b64 from the chunk's buffer set
    auto sums = [&](const int voff, const uint32_t lane_c) {
        if (!(PRB && (a.probe & 1))) {
            constexpr int nsteps = PPC * Q, LA = qp_la<Q, RQ>() < nsteps - 1 ? qp_la<Q, RQ>() : nsteps - 1;
            uint64_t bb[LA + 1][RQ];
#pragma unroll
            for (int e = 0; e < LA; e++)
                lds_read_r<RQ>(bb[e], (uint32_t)__builtin_amdgcn_readlane(voff, e) + lane_c);
#pragma unroll
            for (int e = 0; e < nsteps; e++) {
                uint64_t (&cur)[RQ] = bb[e % (LA + 1)];
                if (e + LA < nsteps) {
                    lds_read_r<RQ>(bb[(e + LA) % (LA + 1)],
                                   (uint32_t)__builtin_amdgcn_readlane(voff, e + LA) + lane_c);
                    lds_wait_n<LA * RQ>(cur);
                } else if (e + 4 == nsteps && LA >= 3) {
                    lds_wait_n<3 * RQ>(cur);
                } else if (e + 3 == nsteps && LA >= 2) {
                    lds_wait_n<2 * RQ>(cur);
                } else if (e + 2 == nsteps && LA >= 1) {
                    lds_wait_n<RQ>(cur);
                } else {
                    lds_wait_n<0>(cur);
                }
                const int q = e % Q;
#pragma unroll
                for (int r = 0; r < RQ; r++) {
                    acc16[q][r][0] += __builtin_bit_cast(short2v, (uint32_t)cur[r]);
                    acc16[q][r][1] += __builtin_bit_cast(short2v, (uint32_t)(cur[r] >> 32));
                }
                if (q == Q - 1 && ++gcount == G) {
                    gcount = 0;
                    widen();
                }
            }
        }
    };

    if constexpr (!SY) {
    // prologue: chunks 0 and 1 in LDS (chunk 1 is expanded in iteration 0)
#pragma unroll
    for (int cc = 0; cc < NS - 1; cc++) dma(cc);
    wait_ring();
    ring_barrier();
    expand(0, 0);
    ring_barrier();

        int chk = 0, ktile = 0;
        for (int c = 0; c < ntot; c++) {
            stamp(c, 0);
            if (!(PRB && (a.probe & 2))) dma(c + NS - 1);
            stamp(c, 1);
            const int chn = chk + 1 == nchunk ? 0 : chk + 1;
            // the expand at raised wave priority: every wave's sums of the next chunk wait on
            // the slowest wave's expand at the barrier (stage 2 33.15-33.19 -> 32.68-32.89 ms
            // per beam; the sums at raised priority instead: 33.9-34.0, profiles/r06_ab_qp_prio.txt)
            __builtin_amdgcn_s_setprio(2);
            if (c + 1 < ntot && !(PRB && (a.probe & 8))) expand(c + 1, chn);
            __builtin_amdgcn_s_setprio(0);
            stamp(c, 2);
            const int voff = read_voff(c);
            sums(voff, lane_byte + (((c ^ chk) & 1) ? ((c & 1) ? set_bytes : 0u - set_bytes) : 0u));
            stamp(c, 3);
            wait_ring();
            stamp(c, 4);
            ring_barrier();
            if (chk == nchunk - 1) {
                flush(tb + ktile++);
                stamp(c, 5);
            }
            chk = chn;
        }
    } else {
        // Barrier-free variant (HD_QP_SYNC=1): three expanded sets, so a wave may expand chunk
        // c + 1 while slower waves still sum chunk c - 1, and two LDS progress counters in place
        // of the per-chunk barrier.  ctr[0] gets +1 per wave and iteration once its share of
        // chunk c + 1 is expanded (its offsets read) and its DMA pieces of chunk c + 2 have
        // landed; ctr[1] gets +1 once its sums of chunk c are done.  Iteration c waits for
        // ctr[0] >= NW (c + 1): chunk c fully expanded (the set its sums read), chunk c + 1 in
        // LDS (the slot its expand reads) and slot c % 3 free for the DMA of chunk c + 3; and for
        // ctr[1] >= NW (c - 1): set (c + 1) % 3 (chunk c - 2's) no longer read.  A wave thus
        // runs up to one iteration ahead of the slowest instead of waiting at a barrier.
        auto signal = [&](int i) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_fetch_add(ctr + i, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        };
        bool stalled = false;
        auto wait_ge = [&](int i, uint32_t target) {
            // bounded (about 0.1 s): a broken count ends the kernel with wrong sums, not a hang
            for (int n = 0; n < (1 << 22) && !stalled; n++) {
                const uint32_t v = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)(ctr + i));
                if (v >= target) {
                    asm volatile("" ::: "memory");
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            stalled = true;
        };
        dma(0);
        dma(1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ring_barrier();
        if (!(PRB && (a.probe & 8))) expand(0, 0);
        int voff_cur = read_voff(0);
        dma(2);
        signal(0);
        int chk = 0, ktile = 0, c3 = 0;
        for (int c = 0; c < ntot; c++) {
            stamp(c, 0);
            wait_ge(0, (uint32_t)(NW * (c + 1)));
            if (c >= 1) wait_ge(1, (uint32_t)(NW * (c - 1)));
            stamp(c, 1);
            const int chn = chk + 1 == nchunk ? 0 : chk + 1;
            int voff_next = 0;
            if (c + 1 < ntot) {
                if (!(PRB && (a.probe & 8))) expand(c + 1, chn);
                voff_next = read_voff(c + 1);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA pieces of chunk c + 2
            signal(0);
            stamp(c, 2);
            if (c + 3 < ntot && !(PRB && (a.probe & 2))) dma(c + 3);
            // the table's set (chk & 1) -> the running set c % 3
            sums(voff_cur, lane_byte + (uint32_t)c3 * set_bytes - (uint32_t)(chk & 1) * set_bytes);
            stamp(c, 3);
            signal(1);
            stamp(c, 4);
            if (chk == nchunk - 1) {
                flush(tb + ktile++);
                stamp(c, 5);
            }
            chk = chn;
            voff_cur = voff_next;
            c3 = c3 == 2 ? 0 : c3 + 1;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the workgroup ends
    if (stamping) {
        __syncthreads();
        const int n = NW * kStampChunks * kStampPh;
        for (int i = threadIdx.x; i < n; i += nthr) a.stamps[(int64_t)blockIdx.x * n + i] = lst[i];
    }
}

size_t stage2_qp_lds_bytes(int setb, int npw, int nbp, int nsub, int ppc, int ns, bool sy)
{
    if (ns <= 0) ns = ppc >= 4 ? 3 : 4;
    if (sy) ns = 3;
    return (size_t)(nsub / 2) * kPairTab * 4 + (size_t)ns * (2 * ppc * npw + nbp) * 1024 + (size_t)(sy ? 3 : 2) * setb +
           (sy ? 16 : 0);
}

// Staging slots of a launch: 4 (a chunk's DMA may land while the next two chunks compute) where
// the LDS allows it at 4 pairs per chunk and HD_QP_NS=4 asks for it (A/B); else 3 at 4 pairs
// per chunk, 4 below.
int stage2_qp_ns(const S2Multi& m, int nsub, int ppc)
{
    if (stage2_qp_sync(m, nsub, ppc)) return 3;
    if (ppc < 4) return 4;
    static const int want = [] {
        const char* e = getenv("HD_QP_NS");
        return e ? atoi(e) : 3;
    }();
    if (want != 4) return 3;
    for (int i = 0; i < m.npass; i++)
        if (stage2_qp_lds_bytes(m.p[i].setb, m.p[i].npw, m.p[i].nbp, nsub, ppc, 4) > 160 * 1024) return 3;
    return 4;
}

// The barrier-free variant (HD_QP_SYNC=1, A/B) where its third buffer set fits the LDS
bool stage2_qp_sync(const S2Multi& m, int nsub, int ppc)
{
    static const bool want = getenv("HD_QP_SYNC") && atoi(getenv("HD_QP_SYNC")) != 0;
    if (!want) return false;
    for (int i = 0; i < m.npass; i++)
        if (stage2_qp_lds_bytes(m.p[i].setb, m.p[i].npw, m.p[i].nbp, nsub, ppc, 3, true) > 160 * 1024) return false;
    return true;
}

template <int Q, int RQ, int PPC, bool NN, bool PRB, int NS, bool SY>
static hipError_t launch_qp_n(const Stage2Args& a, const S2Multi& m, int nyblk, hipStream_t st)
{
    {
        const hipError_t e = set_max_lds((const void*)k_stage2_qp<Q, RQ, PPC, NN, PRB, NS, SY>, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    const unsigned ntiles = (unsigned)((a.nvalid + 256 * RQ - 1) / (256 * RQ));
    const unsigned nx = a.nwg > 0 && (unsigned)a.nwg < ntiles ? (unsigned)a.nwg : ntiles;
    Stage2Args b = a;
    if (nx == ntiles) b.nwg = 0;
    size_t lds = 0;
    for (int i = 0; i < m.npass; i++) {
        if (2 * PPC * m.p[i].npw + m.p[i].nbp > 32) return hipErrorInvalidValue;
        if (m.p[i].setb <= 0 || m.p[i].setb % 32) return hipErrorInvalidValue;
        lds = std::max(lds, stage2_qp_lds_bytes(m.p[i].setb, m.p[i].npw, m.p[i].nbp, a.nsub, PPC, NS, SY));
    }
    if (PRB && a.stamps) lds += (size_t)qp_nw<Q>() * kStampChunks * kStampPh * 4;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    S2Multi mm = m;
    mm.nyblk = nyblk;
    hipLaunchKernelGGL((k_stage2_qp<Q, RQ, PPC, NN, PRB, NS, SY>), dim3(nx, (unsigned)(nyblk * m.npass)),
                       dim3(qp_nw<Q>() * 64), lds, st, b, mm);
    return hipGetLastError();
}

template <int Q, int RQ, int PPC, int NS, bool SY>
static hipError_t launch_qp_s(const Stage2Args& a, const S2Multi& m, int nyblk, hipStream_t st)
{
    const bool prb = (a.probe & 15) != 0 || a.stamps;
    if (a.nonneg && !(a.probe & 64))
        return prb ? launch_qp_n<Q, RQ, PPC, true, true, NS, SY>(a, m, nyblk, st)
                   : launch_qp_n<Q, RQ, PPC, true, false, NS, SY>(a, m, nyblk, st);
    return prb ? launch_qp_n<Q, RQ, PPC, false, true, NS, SY>(a, m, nyblk, st)
               : launch_qp_n<Q, RQ, PPC, false, false, NS, SY>(a, m, nyblk, st);
}

template <int Q, int RQ, int PPC>
static hipError_t launch_qp_p(const Stage2Args& a, const S2Multi& m, int nyblk, hipStream_t st)
{
    if (stage2_qp_sync(m, a.nsub, PPC)) return launch_qp_s<Q, RQ, PPC, 3, true>(a, m, nyblk, st);
    if constexpr (PPC >= 4) {
        if (stage2_qp_ns(m, a.nsub, PPC) == 4) return launch_qp_s<Q, RQ, PPC, 4, false>(a, m, nyblk, st);
        return launch_qp_s<Q, RQ, PPC, 3, false>(a, m, nyblk, st);
    } else {
        return launch_qp_s<Q, RQ, PPC, 4, false>(a, m, nyblk, st);
    }
}

#define HD_QP_QR(X) X(5, 3) X(4, 3) X(7, 3) X(6, 3)

bool stage2_qp_supports(int q, int r)
{
#define HD_QS(QQ, RR) if (q == QQ && r == RR) return true;
    HD_QP_QR(HD_QS)
#undef HD_QS
    return false;
}

hipError_t launch_stage2_qp_multi(const Stage2Args& a, const S2Multi& m, int q, int r, int ppc, hipStream_t st)
{
    if (a.nvalid <= 0 || m.npass <= 0) return hipSuccess;
    if (m.npass > kS2MaxPass) return hipErrorInvalidValue;
    const int nyblk = (a.numdms + a.dms_per_blk - 1) / a.dms_per_blk;
#define HD_QL(QQ, RR)                                                                         \
    if (q == QQ && r == RR) {                                                                 \
        if (ppc == 4) return launch_qp_p<QQ, RR, 4>(a, m, nyblk, st);                         \
        if (ppc == 3) return launch_qp_p<QQ, RR, 3>(a, m, nyblk, st);                         \
        if (ppc == 2) return launch_qp_p<QQ, RR, 2>(a, m, nyblk, st);                         \
        return hipErrorInvalidValue;                                                          \
    }
    HD_QP_QR(HD_QL)
#undef HD_QL
    return hipErrorInvalidValue;
}
#undef HD_QP_QR

}  // namespace hd
