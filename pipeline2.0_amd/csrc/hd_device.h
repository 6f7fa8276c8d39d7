// hd_device.h — device helpers shared by the stage-1 kernels (hd_kernels.hip) and the
// clip/fixup kernels (hd_clip.hip): raw decode, the per-block cleaning lookups, the
// subband rounding rules and small wave utilities.
#pragma once
#include "hd_internal.h"

namespace hd {

__device__ __forceinline__ float raw_value(const RawDesc& rd, int64_t t, int c)
{
    const int rc = rd.flip ? rd.nchan - 1 - c : c;
    const uint8_t* row = rd.raw + t * rd.rowbytes;
    float x;
    if (rd.nbits == 8) {
        x = (float)row[rc];
    } else if (rd.nbits == 4) {
        const uint8_t b = row[rc >> 1];
        const bool first = (rc & 1) == 0;
        const bool hi = rd.nibble_hi_first ? first : !first;
        x = (float)(hi ? (b >> 4) : (b & 15));
    } else {
        const uint8_t* p = row + 2 * rc;
        const uint16_t u = rd.be16 ? (uint16_t)((p[0] << 8) | p[1]) : (uint16_t)((p[1] << 8) | p[0]);
        x = (float)(int16_t)u;
    }
    if (rd.scl) x = x * rd.scl[rc];
    if (rd.offs) x = x + rd.offs[rc];
    if (rd.wts) x = x * rd.wts[rc];
    return x;
}

// read block of spectrum t (spectra past N belong to the last block)
__device__ __host__ __forceinline__ int64_t blk_of(const RawDesc& rd, int64_t t)
{
    const int64_t b = rd.blk_shift >= 0 ? (t >> rd.blk_shift)
                                        : (t < 0x7fffffff ? (int64_t)((int32_t)t / rd.blk) : t / rd.blk);
    return b < rd.nblk ? b : rd.nblk - 1;
}

// Per-block lookups.  A block index past the last block is the last block (blk_of's rule:
// rows past N belong to it): callers derive b0 + 1 / b0 + 2 for tiles that may run past N,
// and an unclamped zidx read there had taken a stray row index into zrows and faulted.
__device__ __forceinline__ int64_t blk_clamp(const RawDesc& rd, int64_t b) { return b < rd.nblk ? b : rd.nblk - 1; }

__device__ __forceinline__ float pad_at(const RawDesc& rd, int64_t b, int c)
{
    return rd.pad ? rd.pad[blk_clamp(rd, b) * rd.pad_stride + c] : 0.0f;
}

__device__ __forceinline__ bool zap_at(const RawDesc& rd, int64_t b, int c)
{
    return rd.zidx && rd.zrows[(int64_t)rd.zidx[blk_clamp(rd, b)] * rd.nchan + c];
}

// The cleaned sample X'(t, c) of the per-block model (oracle/oracle.h), exactly.
__device__ __forceinline__ float chan_value(const RawDesc& rd, int64_t t, int c)
{
    const int64_t b = blk_of(rd, t);
    if (t >= rd.N || (rd.clipped && rd.clipped[t]) || zap_at(rd, b, c)) return pad_at(rd, b, c);
    return raw_value(rd, t, c);
}

// PRESTO NEAREST_LONG, saturated to int16 (sub_round = 1).
// Evaluated in float, exactly: for a float x, (double)x +- 0.5 is exact, so floor/ceil of
// it is trunc(x) stepped by one when the (exact) fraction x - trunc(x) reaches +-0.5.
__device__ __forceinline__ int16_t quant_i16(float x)
{
    const float t = truncf(x);
    const float f = x - t;
    float r = x >= 0.0f ? (f >= 0.5f ? t + 1.0f : t) : (f <= -0.5f ? t - 1.0f : t);
    r = fminf(fmaxf(r, -32768.0f), 32767.0f);
    return (int16_t)(int)r;
}

// prepsubband's `(short)(infloat + 0.5)` as x86-64 evaluates it (sub_round = 0): the double
// x + 0.5 truncated to int32 (cvttsd2si; out of range -> 0x80000000), low 16 bits kept.
__device__ __forceinline__ int16_t presto_short(float x)
{
    const double y = (double)x + 0.5;
    const int32_t i = (y > -2147483649.0 && y < 2147483648.0) ? (int32_t)y : (int32_t)0x80000000u;
    return (int16_t)(uint16_t)(uint32_t)i;
}

__device__ __forceinline__ int16_t to_i16(float x, int sub_round)
{
    return sub_round == 0 ? presto_short(x) : quant_i16(x);
}

// Blocks b, b+8, b+16, ... share an XCD (round-robin dispatch; speed only, never
// correctness): give each XCD a contiguous range of logical block ids (bijective).
// A tile is "special" when it is the last one (reads past the end of the data) or its
// rows straddle a masked read-block boundary.  The hot kernel (SPECIAL = false) skips those
// tiles and runs only the CLEAN / FAST paths, which keeps its register footprint at two
// 8-wave workgroups per CU; the few special tiles (host-built list) get a second launch.
__device__ __host__ __forceinline__ bool s1_special(const Stage1Multi& a, int64_t tR0, int rows)
{
    if (tR0 + rows > a.rd.N) return true;
    if (a.rd.zidx) {
        const int64_t b0 = tR0 / a.rd.blk, b1 = (tR0 + rows - 1) / a.rd.blk;
        if (b1 > b0 + a.two_ok) return true;   // the integer path takes two- (ds >= 10: three-) block tiles
    }
    return false;
}

__device__ __forceinline__ int xcd_remap(int b, int nb)
{
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

__device__ __forceinline__ int wave_max_i32(int v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = max(v, __shfl_xor(v, m, 64));
    return v;
}

// The same maximum, wave-uniform, by DPP steps inside the VALU (quad permutes, row mirrors,
// row broadcasts 15 / 31) instead of six dependent ds_bpermute round trips.  Every lane of the
// wave must be active (EXEC all ones): the stage-1 pass loops, once per pass.
__device__ __forceinline__ int wave_max_full(int v)
{
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));    // quad_perm [1,0,3,2]
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));    // quad_perm [2,3,0,1]
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false));   // row_half_mirror
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false));   // row_mirror
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x142, 0xA, 0xF, false));   // row_bcast:15 -> rows 1, 3
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x143, 0xC, 0xF, false));   // row_bcast:31 -> rows 2, 3
    return __builtin_amdgcn_readlane(v, 63);
}

// The exact sum over the wave of int v, by DPP steps inside the VALU (quad permutes, row
// mirrors, row broadcast 15) and two lane reads, instead of six dependent ds_bpermute round
// trips of an int64.  The caller guarantees every partial fits int32: |v| * 32 < 2^31.  Every
// lane of the wave must be active (EXEC all ones).
__device__ __forceinline__ int64_t wave_sum_i32_small(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]: quad sums
    v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);  // row_half_mirror: 8-lane sums
    v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);  // row_mirror: row sums
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    return (int64_t)__builtin_amdgcn_readlane(v, 31) + (int64_t)__builtin_amdgcn_readlane(v, 63);
}

// Raise *addr to v.  Every wave of a pass targets the same word, and same-address atomics
// serialise at the memory side, so read first (a stale value only costs an extra atomic;
// atomicMax is monotone, so the result is exact) and publish only a new maximum.
__device__ __forceinline__ void publish_max(int32_t* addr, int v)
{
    if (v <= 0) return;
    const int cur = __hip_atomic_load(addr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v > cur) atomicMax(addr, v);
}

// Stage-1 tiles (k_stage1_q8 / k_stage1_q8m): the LDS rows of channels masked in every read
// block the tile touches (b0 .. b0 + nb - 1) are zeroed after the fill, so the integer sums
// add every channel without a per-channel mask (those channels' pads are in the per-block
// constants; the float folds replace their values by the pads).  LDS row r holds channel
// c0 + r (c0 + G - 1 - r on a flipped band), W dwords (a multiple of 4).  Every thread of the
// block calls it; the first barrier is the fill's.
__device__ __forceinline__ void s1_zero_masked_rows(uint32_t* lds, int G, int W, const RawDesc& rd, int64_t b0, int nb,
                                                    int c0, uint8_t* zrow)
{
    bool zf = false;
    if ((int)threadIdx.x < G) {
        const int r = threadIdx.x;
        const int c = c0 + (rd.flip ? G - 1 - r : r);
        zf = rd.zidx != nullptr;
        // blocks past the last one are the last one (as blk_of has it): a tile that runs past N
        // must not index zidx beyond nblk -- an unclamped read there took a stray row index
        // from whatever followed the table and faulted in the zrows lookup
        const int64_t bl = min(b0 + (int64_t)nb - 1, (int64_t)rd.nblk - 1);
        for (int64_t b = b0; b <= bl && zf; b++) zf = zap_at(rd, b, c);
        zrow[r] = zf;
    }
    if (!__syncthreads_or(zf)) return;
    const int w4 = W >> 2;
    for (int i = threadIdx.x; i < G * w4; i += blockDim.x) {
        const int r = i / w4;
        if (zrow[r]) ((uint4*)(lds + (size_t)r * W))[i - r * w4] = make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();
}

// N consecutive ints of a wave-uniform, read-only table (a pass's channel delays) through the
// scalar cache: s_load is counted by lgkmcnt, so waiting for it never waits for the wave's
// outstanding global stores (a vector load of the same words is counted by vmcnt with them).
template <int N>
__device__ __forceinline__ void sload_i32(const int32_t* p, int (&v)[N])
{
    typedef const int32_t __attribute__((address_space(4))) cint32;
    const cint32* q = (const cint32*)p;
#pragma unroll
    for (int i = 0; i < N; i++) v[i] = q[i];
}

}  // namespace hd
