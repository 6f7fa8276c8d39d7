// hd_kernels.hip — CDNA4 (gfx950) stage-1 kernels of the dedispersion engine and helpers.
//
//   k_stage1_direct  raw PSRFITS block -> nsub subbands at subdm, downsampled, int16/f32
//                    (prepsubband -sub; reference PALFA2_presto_search.py:506-511)
//   k_stage1_tiled   the same over an LDS raw tile, every pass of a DDplan stage per launch
//   k_stage1_q8      8-bit (and unpacked 4-bit) integer path over the channel-major copy
//   k_raw_transpose  raw rows -> channel-major bytes (rawT)
//   k_pad            first-DM (prepsubband) or per-DM mean (reduction of per-tile partials,
//                    exact for int16 subbands) fill of samples [N/ds, numout)
//   k_synth          synthetic beam, bit-identical to the host generator
// The stage-2 kernels (subbands -> DM series) are in hd_stage2.hip.
//
// Arithmetic contract with the oracle (oracle/prepsubband_oracle.c): float sums in the
// same order from 0.0f, no FP contraction (built with -ffp-contract=off), correctly
// rounded division; int16 subbands make every stage-2 sum an exact integer, so any
// summation order (including the packed int16 one) is bit-identical.
#include "hd_device.h"

#include <algorithm>
#include <map>
#include <mutex>

namespace hd {

// The dynamic-LDS limit is a per-device property of a kernel: remember per (kernel,
// device) what was granted, so contexts on several GPUs in one process each get it.
hipError_t set_max_lds(const void* fn, int bytes)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, int> granted;
    std::lock_guard<std::mutex> lock(mu);
    int& have = granted[{fn, dev}];
    if (have >= bytes) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) have = bytes;
    return e;
}

// ------------------------------------------------------------------------------------
// stage 1
// ------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_stage1_direct(Stage1Args a)
{
    const int s = blockIdx.y;
    const int64_t tp = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = tp < a.nds;
    int amax = 0;
    if (valid) {
        float acc = 0.0f;
        for (int k = 0; k < a.ds; k++) {
            float sk = 0.0f;
            const int64_t tb = tp * a.ds + k;
            for (int cc = 0; cc < a.cps; cc++) {
                const int c = s * a.cps + cc;
                sk += chan_value(a.rd, tb + a.idispdt[c], c);
            }
            acc += sk;
        }
        if (a.ds_mode == 1) acc = acc / (float)a.ds;
        if (a.sub_dtype == 0) {
            const int16_t q = to_i16(acc, a.sub_round);
            ((int16_t*)a.out)[(int64_t)s * a.out_stride + tp] = q;
            amax = q < 0 ? -(int)q : (int)q;
        } else {
            ((float*)a.out)[(int64_t)s * a.out_stride + tp] = acc;
        }
    }
    if (a.sub_dtype == 0 && a.maxabs) {
        amax = wave_max_i32(amax);
        if ((threadIdx.x & 63) == 0) publish_max(a.maxabs, amax);
    }
}

hipError_t launch_stage1_direct(const Stage1Args& a, hipStream_t st)
{
    if (a.nds <= 0) return hipSuccess;
    dim3 grid((unsigned)((a.nds + 255) / 256), (unsigned)a.nsub);
    hipLaunchKernelGGL(k_stage1_direct, grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// stage 1, tiled + multi-pass
// ------------------------------------------------------------------------------------
//
// Workgroup = 64*sg threads = one time tile of `to` output samples x sg subbands
// (G = sg*cps channels, contiguous in the raw row for either band order).
//  fill : raw rows [to*ds*tile, +to*ds+dmax) of the group's G channels are copied verbatim
//         into LDS (16/8/4-byte global loads, dword LDS stores, row stride rs with an odd
//         dword count so the per-row byte reads below are bank-conflict-free at ds = 1);
//  form : wave w owns subband sl = w, so its CPS channel delays, calibration and zap flags
//         are wave-uniform registers; lane l owns outputs l, l+64, ...  For every pass the
//         decoded samples are summed in the oracle's order (k outer, channel inner, from
//         0.0f), quantised and stored coalesced.
// Mask: zap sets and pad values are per read block (blk spectra, PRESTO's subint).  A tile
// inside one block has, per channel, either zapped samples for the whole tile (the block's
// constant pad value: one add) or none: mode FAST.  Tiles that straddle one block boundary
// (mode TWO: per-row select between the two blocks' flags and pads), tiles over >= 3 blocks
// (mode GEN: per-row block table) and the last tile (reads past the end = the last block's
// pad) take per-sample paths.  Clipped spectra are not handled here: the fixup kernel
// (hd_clip.hip) recomputes every output they touch.

constexpr int kModeFast = 0, kModeTwo = 1, kModeGen = 2, kModeClean = 3;

template <int NBITS>
__device__ __forceinline__ float lds_decode(const uint8_t* p, int lrc, int nibble_hi_first, int be16)
{
    if (NBITS == 8) {
        return (float)p[0];
    } else if (NBITS == 4) {
        const uint8_t b = p[0];
        const bool first = (lrc & 1) == 0;
        const bool hi = nibble_hi_first ? first : !first;
        return (float)(hi ? (b >> 4) : (b & 15));
    } else {
        const uint16_t w = *(const uint16_t*)p;   // file bytes p[0], p[1]
        const uint16_t u = be16 ? (uint16_t)((w << 8) | (w >> 8)) : w;
        return (float)(int16_t)u;
    }
}

// Per-channel, wave-uniform state of one subband for one pass.
template <int CPS>
struct SubState {
    int off[CPS];      // LDS byte offset of (row 0 + delay, channel) for this channel
    int dly[CPS];      // channel delay (rows)
    float scl[CPS], offs[CPS], wts[CPS];
    float pad0[CPS], pad1[CPS];   // pad values of the tile's first / second block
    int zap[CPS];      // FAST: 1 = whole tile zapped;  TWO: bit0 first block, bit1 second;
                       // GEN: the channel index (per-row lookups)
};

// One decoded, calibrated, masked sample of channel cc at tile row jrow + k (+ delay).
template <int NBITS, int CPS, bool CALIB, int MODE, bool TAIL>
__device__ __forceinline__ float s1_sample(const Stage1Multi& a, const uint8_t* rowp, const SubState<CPS>& st,
                                          const int* livr, int c_first, int brow, int rows_valid, int jk, int cc)
{
    // branch-free: every sample is read and decoded, then selected
    float x = lds_decode<NBITS>(rowp + st.off[cc], c_first + cc, a.rd.nibble_hi_first, a.rd.be16);
    // keep the read unconditional: otherwise hipcc sinks it under a uniform
    // branch on the zap flag and splits the channel loop into CPS basic blocks
    if (MODE != kModeClean) asm volatile("" : "+v"(x));
    if (CALIB) {
        x = x * st.scl[cc];
        x = x + st.offs[cc];
        x = x * st.wts[cc];
    }
    if (MODE == kModeFast) {
        x = st.zap[cc] ? st.pad0[cc] : x;
    } else if (MODE == kModeTwo) {
        const int row = jk + st.dly[cc];
        const bool second = row >= brow;
        x = (st.zap[cc] & (second ? 2 : 1)) ? (second ? st.pad1[cc] : st.pad0[cc]) : x;
    } else if (MODE == kModeGen) {
        const int row = jk + st.dly[cc];
        const int lv = livr[row];
        const int b = lv & 0x3FFFFFFF;
        const int c = st.zap[cc];
        if ((TAIL && row >= rows_valid) || (lv >> 30) || zap_at(a.rd, b, c)) x = pad_at(a.rd, b, c);
    }   // kModeClean: no mask logic at all
    return x;
}

template <int NBITS, int CPS, bool CALIB, int MODE, bool TAIL>
__device__ __forceinline__ void form_outputs(const Stage1Multi& a, const uint8_t* lraw, const SubState<CPS>& st,
                                             const int* livr, int c_first, int brow, int rows_valid,
                                             int64_t tO0, int lane, int s, int p, int& amax, int ds, int to, int64_t nds)
{
    // Two outputs per lane per iteration (j, j+64): two independent add chains for ILP.
    // Uniform trip count; only the last iteration can diverge.  (ds, to, nds: the launch's, or
    // the pass's own in a SPECIAL launch over several DDplan stages, a.pass_ds)
    const int jmax = (int)min((int64_t)to, nds - tO0);
    for (int j0 = lane; j0 < jmax; j0 += 128) {
        const bool has1 = j0 + 64 < jmax;
        const int j1 = has1 ? j0 + 64 : j0;          // duplicate work, result discarded
        const int jr0 = j0 * ds, jr1 = j1 * ds;
        float acc0 = 0.0f, acc1 = 0.0f;
        for (int k = 0; k < ds; k++) {
            const uint8_t* rp0 = lraw + (jr0 + k) * a.rs;
            const uint8_t* rp1 = lraw + (jr1 + k) * a.rs;
            float sk0 = 0.0f, sk1 = 0.0f;
#pragma unroll
            for (int cc = 0; cc < CPS; cc++) {
                sk0 += s1_sample<NBITS, CPS, CALIB, MODE, TAIL>(a, rp0, st, livr, c_first, brow, rows_valid, jr0 + k, cc);
                sk1 += s1_sample<NBITS, CPS, CALIB, MODE, TAIL>(a, rp1, st, livr, c_first, brow, rows_valid, jr1 + k, cc);
            }
            acc0 += sk0;
            acc1 += sk1;
        }
        if (a.ds_mode == 1) {
            acc0 = acc0 / (float)ds;
            acc1 = acc1 / (float)ds;
        }
        const int64_t tp0 = tO0 + j0, tp1 = tO0 + j1;
        if (a.sub_dtype == 0) {
            const int16_t q0 = to_i16(acc0, a.sub_round), q1 = to_i16(acc1, a.sub_round);
            int16_t* o = (int16_t*)a.out[p] + (int64_t)s * a.ostride[p];
            o[tp0] = q0;
            amax = max(amax, q0 < 0 ? -(int)q0 : (int)q0);
            if (has1) {
                o[tp1] = q1;
                amax = max(amax, q1 < 0 ? -(int)q1 : (int)q1);
            }
        } else {
            float* o = (float*)a.out[p] + (int64_t)s * a.ostride[p];
            o[tp0] = acc0;
            if (has1) o[tp1] = acc1;
        }
    }
}

template <int NBITS, int CPS, bool CALIB, int VW, bool SPECIAL>
__global__ __launch_bounds__(512, SPECIAL ? 1 : 4)   // hot: 2 x 8-wave WGs per CU -> <= 128 VGPRs
void k_stage1_tiled(Stage1Multi a, const int* __restrict__ special_tiles)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int G = a.sg * CPS;
    const int logical = xcd_remap(blockIdx.x, gridDim.x);
    const int ti = logical / a.ngroups;
    const int g = logical - ti * a.ngroups;
    const int tile = SPECIAL ? special_tiles[ti] : ti;
    const int64_t tO0 = (int64_t)tile * a.to;
    const int64_t tR0 = tO0 * a.ds;
    const int rows = a.to * a.ds + a.dmax;
    if (!SPECIAL && s1_special(a, tR0, rows)) return;      // uniform: handled by the second launch
    const int c0 = g * G;
    const int rc_lo = a.rd.flip ? a.rd.nchan - c0 - G : c0;
    const int gbytes = G * NBITS / 8;
    const int64_t boff = (int64_t)rc_lo * NBITS / 8;
    uint8_t* lraw = (uint8_t*)smem;
    int* livr = (int*)(smem + ((rows * a.rs + 15) & ~15));

    // ---- tile mode (uniform)
    const int rows_valid = (int)min(a.rd.N - tR0, (int64_t)rows);
    const bool tail = rows_valid < rows;
    int mode = kModeFast;
    const int64_t b0 = blk_of(a.rd, tR0);
    int brow = rows;
    if (a.rd.zidx) {
        const int64_t b_last = (tR0 + rows - 1) / a.rd.blk;
        brow = (int)min((b0 + 1) * a.rd.blk - tR0, (int64_t)rows);
        mode = b_last == b0 ? kModeFast : (b_last == b0 + 1 ? kModeTwo : kModeGen);
    }
    if (SPECIAL && tail) mode = kModeGen;          // rows past N read the last block's pads
    // the special tiles of the 8-bit integer path replace clipped spectra themselves (that
    // path has no separate fixup launch): GEN mode, bit 30 of the row table = clipped
    const bool sp_clip = SPECIAL && a.qfix && a.rd.clipped;
    if (sp_clip) mode = kModeGen;
    if (SPECIAL && mode == kModeGen)
        for (int r = threadIdx.x; r < rows; r += blockDim.x) {
            const int64_t t = tR0 + r;
            livr[r] = (int)blk_of(a.rd, t) | (sp_clip && t < a.rd.N && a.rd.clipped[t] ? (1 << 30) : 0);
        }

    // ---- fill: VW-byte global loads, dword LDS stores
    {
        const int vpr = gbytes / VW;                 // vectors per row
        const int nthr = blockDim.x;
        int r = threadIdx.x / vpr, w = threadIdx.x - (threadIdx.x / vpr) * vpr;
        const int dr = nthr / vpr, dw = nthr - dr * vpr;
        for (; r < rows; r += dr) {
            const int64_t t = tR0 + r;
            uint32_t v[VW / 4];
#pragma unroll
            for (int i = 0; i < VW / 4; i++) v[i] = 0;
            if (t < a.rd.N) {
                const uint8_t* src = a.rd.raw + t * a.rd.rowbytes + boff + VW * w;
                if constexpr (VW == 16) {
                    const uint4 x = *(const uint4*)src;
                    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
                } else {
                    v[0] = *(const uint32_t*)src;
                }
            }
            uint32_t* dst = (uint32_t*)(lraw + r * a.rs + VW * w);
#pragma unroll
            for (int i = 0; i < VW / 4; i++) dst[i] = v[i];
            w += dw;
            if (w >= vpr) { w -= vpr; r++; }
        }
    }
    __syncthreads();

    const int sl = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave = subband
    const int lane = threadIdx.x & 63;
    const int s = g * a.sg + sl;
    const int cl0 = sl * CPS;
    SubState<CPS> st;
    int any_zap = 0;
#pragma unroll
    for (int cc = 0; cc < CPS; cc++) {
        const int c = c0 + cl0 + cc;
        const int rc = a.rd.flip ? a.rd.nchan - 1 - c : c;
        if (CALIB) {
            st.scl[cc] = a.rd.scl ? a.rd.scl[rc] : 1.0f;
            st.offs[cc] = a.rd.offs ? a.rd.offs[rc] : 0.0f;
            st.wts[cc] = a.rd.wts ? a.rd.wts[rc] : 1.0f;
        }
        st.pad0[cc] = pad_at(a.rd, b0, c);
        st.pad1[cc] = pad_at(a.rd, min(b0 + 1, (int64_t)a.rd.nblk - 1), c);
        int z = 0;
        if (mode == kModeGen) {
            z = c;   // GEN mode looks the mask up per row; keep the channel index here
            any_zap = 1;
        } else if (a.rd.zidx) {
            const int z0 = zap_at(a.rd, b0, c);
            const int z1 = mode == kModeTwo && zap_at(a.rd, b0 + 1, c);
            z = mode == kModeFast ? z0 : (z0 ? 1 : 0) | (z1 ? 2 : 0);
            any_zap |= z;
        }
        st.zap[cc] = z;
    }
    const int lrc0 = a.rd.flip ? G - 1 - cl0 : cl0;   // local raw index of channel cc=0
    int pmax = 0;                                      // lane p: max |subband| of pass p
    // a SPECIAL grid with y > 1 gives every pass its own workgroup (few special tiles: the
    // passes would otherwise run back to back in a handful of workgroups)
    const int p_lo = SPECIAL && gridDim.y > 1 ? (int)blockIdx.y : 0;
    const int p_hi = SPECIAL && gridDim.y > 1 ? (int)blockIdx.y + 1 : a.npass;
    for (int p = p_lo; p < p_hi; p++) {
#pragma unroll
        for (int cc = 0; cc < CPS; cc++) {
            const int lrc = a.rd.flip ? lrc0 - cc : lrc0 + cc;
            st.dly[cc] = a.dly[p][c0 + cl0 + cc];
            st.off[cc] = st.dly[cc] * a.rs + lrc * NBITS / 8;
        }
        // a SPECIAL launch over the passes of several DDplan stages (the fused k_stage1_q8m
        // call's special tiles, a.pass_ds): the tile is 4 S raw rows for every pass (a.to *
        // a.ds), each pass forms its own to = 4 S / ds outputs of it
        const bool pds = SPECIAL && a.pass_ds;
        const int dsp = pds ? a.pds[p] : a.ds;
        const int top = pds ? a.to * a.ds / dsp : a.to;
        const int64_t ndsp = pds ? a.rd.N / dsp : a.nds;
        const int64_t tO0 = (int64_t)tile * top;
        int amax = 0;
        if (!SPECIAL) {
            // (a tile over two read blocks stays here when the launch allows it, a.two_ok)
            if (!any_zap)
                form_outputs<NBITS, CPS, CALIB, kModeClean, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax, dsp, top, ndsp);
            else if (mode == kModeTwo)
                form_outputs<NBITS, CPS, CALIB, kModeTwo, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax, dsp, top, ndsp);
            else
                form_outputs<NBITS, CPS, CALIB, kModeFast, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax, dsp, top, ndsp);
        } else if (!tail) {
            if (mode == kModeFast)
                form_outputs<NBITS, CPS, CALIB, kModeFast, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax, dsp, top, ndsp);
            else if (mode == kModeTwo)
                form_outputs<NBITS, CPS, CALIB, kModeTwo, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax, dsp, top, ndsp);
            else
                form_outputs<NBITS, CPS, CALIB, kModeGen, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax, dsp, top, ndsp);
        } else {
            form_outputs<NBITS, CPS, CALIB, kModeGen, true>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax, dsp, top, ndsp);
        }
        if (a.sub_dtype == 0) {
            amax = wave_max_i32(amax);
            pmax = lane == p ? amax : pmax;
        }
    }
    // one publication per pass at the end: a load-tested atomic inside the pass loop would
    // make the wave wait for all of its outstanding stores every pass
    if (a.sub_dtype == 0 && lane < a.npass) publish_max(a.maxabs[lane], pmax);
}

size_t stage1_tiled_lds_bytes(const Stage1Multi& a)
{
    const int rows = a.to * a.ds + a.dmax;
    size_t b = ((size_t)rows * a.rs + 15) & ~(size_t)15;
    b += (size_t)rows * sizeof(int);     // GEN-mode row -> interval table
    return b;
}

int stage1_special_tiles(const Stage1Multi& a, int* out)
{
    int n = 0;
    const int rows = a.to * a.ds + a.dmax;
    for (int t = 0; t < a.ntiles; t++) {
        const int64_t tR0 = (int64_t)t * a.to * a.ds;
        const bool sp = s1_special(a, tR0, rows);
        if (sp) {
            if (out) out[n] = t;
            n++;
        }
    }
    return n;
}

template <int NBITS, int CPS, bool CALIB>
static hipError_t launch_s1(const Stage1Multi& a, int vw, size_t lds, const int* special, int nspecial,
                            bool special_only, hipStream_t st)
{
    const dim3 block((unsigned)(64 * a.sg));
    // special tiles are few (the last tile; tiles over >= 3 read blocks): split them by pass
    // unless they already fill the chip
    const unsigned split = nspecial * a.ngroups < 2048 ? (unsigned)a.npass : 1u;
    const dim3 grid((unsigned)(a.ntiles * a.ngroups)), grid_sp((unsigned)(nspecial * a.ngroups), split);
    if (vw == 16) {
        if (!special_only)
            hipLaunchKernelGGL((k_stage1_tiled<NBITS, CPS, CALIB, 16, false>), grid, block, lds, st, a, special);
        if (nspecial)
            hipLaunchKernelGGL((k_stage1_tiled<NBITS, CPS, CALIB, 16, true>), grid_sp, block, lds, st, a, special);
    } else {
        if (!special_only)
            hipLaunchKernelGGL((k_stage1_tiled<NBITS, CPS, CALIB, 4, false>), grid, block, lds, st, a, special);
        if (nspecial)
            hipLaunchKernelGGL((k_stage1_tiled<NBITS, CPS, CALIB, 4, true>), grid_sp, block, lds, st, a, special);
    }
    return hipGetLastError();
}

template <int NBITS, int CPS, bool CALIB>
static hipError_t set_lds_cps(int bytes)
{
    const void* fns[4] = {(const void*)k_stage1_tiled<NBITS, CPS, CALIB, 16, false>,
                          (const void*)k_stage1_tiled<NBITS, CPS, CALIB, 16, true>,
                          (const void*)k_stage1_tiled<NBITS, CPS, CALIB, 4, false>,
                          (const void*)k_stage1_tiled<NBITS, CPS, CALIB, 4, true>};
    for (const void* f : fns) {
        hipError_t e = set_max_lds(f, bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

#define HD_S1_FOR_CPS(X) X(10) X(8) X(16) X(1)

bool stage1_tiled_supports_cps(int cps) { return cps == 10 || cps == 8 || cps == 16 || cps == 1; }

hipError_t stage1_tiled_set_lds_limit(size_t bytes)
{
    hipError_t e = hipSuccess;
    const int b = (int)bytes;
#define HD_SET(C)                                                                 \
    if (e == hipSuccess) e = set_lds_cps<8, C, false>(b);                          \
    if (e == hipSuccess) e = set_lds_cps<8, C, true>(b);                           \
    if (e == hipSuccess) e = set_lds_cps<4, C, false>(b);                          \
    if (e == hipSuccess) e = set_lds_cps<4, C, true>(b);                           \
    if (e == hipSuccess) e = set_lds_cps<16, C, false>(b);                         \
    if (e == hipSuccess) e = set_lds_cps<16, C, true>(b);
    HD_S1_FOR_CPS(HD_SET)
#undef HD_SET
    return e;
}

hipError_t launch_stage1_tiled(const Stage1Multi& a, int vw, const int* special, int nspecial, bool special_only,
                               hipStream_t st)
{
    if (a.nds <= 0 || a.npass <= 0) return hipSuccess;
    const size_t lds = stage1_tiled_lds_bytes(a);
    const bool calib = a.rd.scl || a.rd.offs || a.rd.wts;
#define HD_DISPATCH(C)                                                                                      \
    if (a.cps == C) {                                                                                       \
        switch (a.rd.nbits) {                                                                               \
        case 8: return calib ? launch_s1<8, C, true>(a, vw, lds, special, nspecial, special_only, st)                      \
                             : launch_s1<8, C, false>(a, vw, lds, special, nspecial, special_only, st);                    \
        case 4: return calib ? launch_s1<4, C, true>(a, vw, lds, special, nspecial, special_only, st)                      \
                             : launch_s1<4, C, false>(a, vw, lds, special, nspecial, special_only, st);                    \
        case 16: return calib ? launch_s1<16, C, true>(a, vw, lds, special, nspecial, special_only, st)                    \
                              : launch_s1<16, C, false>(a, vw, lds, special, nspecial, special_only, st);                  \
        default: return hipErrorInvalidValue;                                                               \
        }                                                                                                   \
    }
    HD_S1_FOR_CPS(HD_DISPATCH)
#undef HD_DISPATCH
    return hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------
// stage 1, 8-bit integer path (quarter-interleaved LDS tile)
// ------------------------------------------------------------------------------------
//
// For 8-bit data without calibration every stage-1 sum is a sum of small integers, exact
// in float32, so an integer summation in any order is bit-identical to the oracle's
// float fold.  The tile of a workgroup (sg subbands = G = sg*CPS channels) holds, per
// channel, K = S + dmax dwords; dword k packs the bytes of raw rows k, k+S, k+2S, k+3S
// (one per "quarter" of the tile).  Any delay d then reads whole, aligned dwords: the
// lane that owns quarter-position j reads dword j*DS + k + d and gets 4 samples, one per
// quarter, with one ds_read_b32.  Bytes are widened into two packed u16 accumulators
// (quarters 0/2 and 1/3; the host guarantees CPS*DS*255 < 32768, so no half can carry):
// ~3 VALU per 4 channel-samples instead of ~2 per sample on the float path.
// Subbands with masked channels in the tile (rfifind FAST mode) take an exact path: the
// integer prefix up to the first zapped channel, then the oracle's float fold.  Tiles
// straddling a mask interval boundary, and the last tile, are left to the float kernel
// above (its SPECIAL launch over the same tiles).

template <int DS, int MO = 0>
struct Q8Geom {
    static constexpr int M = MO ? MO : DS == 1 ? 4 : DS == 2 ? 2 : 1;   // outputs per lane per quarter
    static constexpr int JQ = 64 * M;                          // outputs per quarter
    static constexpr int S = JQ * DS;                          // dwords (raw rows) per quarter
    static constexpr bool THREE = DS >= 10;                    // 4S + dmax may exceed a 2048-row block
};

// HD_Q8_M1 (profiling): outputs per lane per quarter at ds 1 (4, or 2: half the tile, about
// 5 instead of 3 workgroups per CU)
int q8_m1()
{
    static int m = -1;
    if (m < 0) m = getenv("HD_Q8_M1") && atoi(getenv("HD_Q8_M1")) == 2 ? 2 : 4;
    return m;
}

int stage1_q8_quarter_rows(int ds)
{
    switch (ds) {
    case 1: return q8_m1() == 2 ? Q8Geom<1, 2>::S : Q8Geom<1>::S;
    case 2: return Q8Geom<2>::S;
    case 3: return Q8Geom<3>::S;
    case 5: return Q8Geom<5>::S;
    case 6: return Q8Geom<6>::S;
    case 10: return Q8Geom<10>::S;
    default: return 0;
    }
}

// Store the 4 quarter outputs of quarter-position j: integral -> the exact packed sums qv
// (each already holding its pad constant, see k_stage1_q8), else the float folds qf.
template <int DS, int MO>
__device__ __forceinline__ void q8_store(const Stage1Multi& a, int p, int s, int64_t tO0, int j,
                                         const uint32_t* qv, const float* qf, bool integral, int& amax)
{
    constexpr int JQ = Q8Geom<DS, MO>::JQ;
    if (a.sub_dtype == 0) {
        int16_t* o = (int16_t*)a.out[p] + (int64_t)s * a.ostride[p] + tO0 + j;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int16_t v;
            if (integral) v = (int16_t)(a.ds_mode == 1 ? qv[q] / (uint32_t)DS : qv[q]);   // < 32768 (host check)
            else v = to_i16(qf[q], a.sub_round);
            o[q * JQ] = v;
            amax = max(amax, v < 0 ? -(int)v : (int)v);
        }
    } else {
        float* o = (float*)a.out[p] + (int64_t)s * a.ostride[p] + tO0 + j;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            float x = integral ? (float)qv[q] : qf[q];
            if (integral && a.ds_mode == 1) x = x / (float)DS;
            o[q * JQ] = x;
        }
    }
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Waves per subband in k_stage1_q8's summing phase: the block has max(4, sg) waves (the fill
// wants at least 4); with sg < 4 the spare waves take a share of the passes (probe bit 4 of
// hd_plan_set_variant's probe byte, value 16: one wave per subband, the spare waves idle).
__host__ __device__ __forceinline__ int q8_waves_per_subband(const Stage1Multi& a)
{
    return (a.probe & 16) ? 1 : a.sg >= 4 ? (a.wps2 ? 2 : 1) : 4 / a.sg;
}

template <int CPS, int DS, int VB, int MO = 0>
__global__ __launch_bounds__(512) void k_stage1_q8(Stage1Multi a)
{
    constexpr bool THREE = Q8Geom<DS, MO>::THREE;
    using Gm = Q8Geom<DS, MO>;
    constexpr int M = Gm::M, JQ = Gm::JQ, S = Gm::S;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint32_t* lds = (uint32_t*)smem;
    const int G = a.sg * CPS;
    const int logical = xcd_remap(blockIdx.x, gridDim.x);
    const int tile = logical / a.ngroups;
    const int g = logical - tile * a.ngroups;
    const int64_t tO0 = (int64_t)tile * (4 * JQ);
    const int64_t tR0 = tO0 * DS;
    if (s1_special(a, tR0, 4 * S + a.dmax)) return;     // uniform: the float kernel's SPECIAL launch
    const int K = S + a.dmax;
    const int W = a.W;
    const int c0 = g * G;
    const int rc_lo = a.rd.flip ? a.rd.nchan - c0 - G : c0;
    const int64_t rb = a.rd.rowbytes;

    // ---- fill: unit = (row k, VB-byte chunk): raw rows k + qS (q < 4) -> VB channel dwords;
    //      U units per iteration, all their row loads issued before the first is used (the
    //      fill is latency-bound: a CU needs tens of KB of loads in flight)
    if (!(a.probe & 2) && a.rawT) {
        // channel-major raw (k_raw_transpose8): unit = (local channel lc, 16-row block kb);
        // the 4 quarter runs of a channel are contiguous bytes, so each lane loads 16 B per
        // quarter and a wave's loads are 1-KiB coalesced runs (the row-major fill below uses G
        // of every 960-B row: 3-7x more L2->L1 traffic than bytes kept, and 4-8x the loads).
        // Same LDS image: dword kk of channel lc packs rows kk + q*S (q = 0..3).
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
                const int u = min(u0 + h * nthr, units - 1);     // duplicate (idempotent) tail unit
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
                    // 4x4 byte transpose: dword j = row 16kb+4w+j of quarters q = 0..3
                    const uint32_t ab_lo = __builtin_amdgcn_perm(x1, x0, 0x05010400u);
                    const uint32_t ab_hi = __builtin_amdgcn_perm(x1, x0, 0x07030602u);
                    const uint32_t cd_lo = __builtin_amdgcn_perm(x3, x2, 0x05010400u);
                    const uint32_t cd_hi = __builtin_amdgcn_perm(x3, x2, 0x07030602u);
                    o[4 * w + 0] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u);
                    o[4 * w + 1] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u);
                    o[4 * w + 2] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u);
                    o[4 * w + 3] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u);
                }
                // the unit's 16 dwords are contiguous (W is a multiple of 16): four 16-byte
                // stores, the lanes of an 8-lane store group staggered over the four chunks
                // (lanes are 64 B apart, so chunk w of every lane would share 2 of the 8
                // bank quads: 4-way conflicts; staggered, the 8 lanes hit 8 distinct quads)
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
    } else if (!(a.probe & 2)) {
        constexpr int U = 32 / VB;
        const uint8_t* src0 = a.rd.raw + tR0 * rb + rc_lo;
        const int NCH = G / VB;
        const int units = K * NCH;
        const int nthr = blockDim.x;
        for (int u0 = threadIdx.x; u0 < units; u0 += U * nthr) {
            uint32_t r[U][4][VB / 4];
            int kk[U], cc[U];
#pragma unroll
            for (int h = 0; h < U; h++) {
                const int u = min(u0 + h * nthr, units - 1);     // duplicate (idempotent) tail unit
                kk[h] = u / NCH;
                cc[h] = u - kk[h] * NCH;
                const uint8_t* sp = src0 + (int64_t)kk[h] * rb + cc[h] * VB;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint8_t* sq = sp + (int64_t)q * S * rb;
                    if constexpr (VB == 8) {
                        const uint2 v = *(const uint2*)sq;
                        r[h][q][0] = v.x;
                        r[h][q][1] = v.y;
                    } else {
                        r[h][q][0] = *(const uint32_t*)sq;
                    }
                }
            }
#pragma unroll
            for (int h = 0; h < U; h++)
#pragma unroll
                for (int i = 0; i < VB / 4; i++) {
                    // 4x4 byte transpose: dword j of the output = channel 4i+j of rows q = 0..3
                    const uint32_t ab_lo = __builtin_amdgcn_perm(r[h][1][i], r[h][0][i], 0x05010400u);
                    const uint32_t ab_hi = __builtin_amdgcn_perm(r[h][1][i], r[h][0][i], 0x07030602u);
                    const uint32_t cd_lo = __builtin_amdgcn_perm(r[h][3][i], r[h][2][i], 0x05010400u);
                    const uint32_t cd_hi = __builtin_amdgcn_perm(r[h][3][i], r[h][2][i], 0x07030602u);
                    uint32_t* d = lds + (cc[h] * VB + 4 * i) * W + kk[h];
                    d[0] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u);
                    d[W] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u);
                    d[2 * W] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u);
                    d[3 * W] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u);
                }
        }
    }
    // in-kernel fixup state (qfix): [clip bits of the tile's rows][pads [3][G]][zap bits [G]]
    const int rows_t = 4 * S + a.dmax;
    const int nwc = (rows_t + 31) >> 5;
    uint32_t* cflag = lds + G * W;
    float* fpad = (float*)(cflag + nwc);
    uint8_t* fzb = (uint8_t*)(fpad + 3 * G);
    __shared__ int amax_fix[kMaxPass];
    __shared__ uint8_t fneed[8];                          // per subband: bit b = boundary b needs outputs redone
    constexpr int kCRow = 64;                             // clipped rows listed per tile (more: word scan)
    __shared__ int crow[kCRow], ncrow;
    if (threadIdx.x == 0) ncrow = 0;                      // (ordered by the barrier below)
    int anyclip = 0;
    if (a.qfix) {
        // the tile's clip flags: one coalesced word per thread from the bit-packed copy (tR0 is a
        // multiple of 256 and tR0 + rows_t <= N on a non-special tile)
        for (int w = threadIdx.x; w < nwc; w += blockDim.x) {
            uint32_t bits = a.rd.clipbits ? a.rd.clipbits[(tR0 >> 5) + w] : 0u;
            const int rem = rows_t - 32 * w;
            if (rem < 32) bits &= (1u << rem) - 1u;
            cflag[w] = bits;
            anyclip |= bits != 0;
        }
        if (threadIdx.x < kMaxPass) amax_fix[threadIdx.x] = 0;
        if (threadIdx.x < 8) fneed[threadIdx.x] = 0;
    }
    anyclip = __syncthreads_or(anyclip);
    __shared__ uint8_t zrow[256];
    if (a.rd.zidx) {                                      // (uniform) channels masked in every block: rows zeroed
        const int64_t bz = tR0 / a.rd.blk;
        s1_zero_masked_rows(lds, G, W, a.rd, bz, (int)((tR0 + 4 * S + a.dmax - 1) / a.rd.blk - bz) + 1, c0, zrow);
    }

    // ---- per-wave subband state: wave w serves subband w / wps and passes p = w % wps (mod
    //      wps), so every wave of the block (at least 4) sums: sg = 2 gives 2 waves per
    //      subband instead of 2 summing waves and 2 that only fill
    const int wps = q8_waves_per_subband(a);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sl = wv / wps, pw = wv - sl * wps;
    const int lane = threadIdx.x & 63;
    // brow / brow2: the tile's read-block boundaries (tile-relative rows), uniform per workgroup
    int brow = 1 << 30, brow2 = 1 << 30;
    const int64_t b0 = tR0 / a.rd.blk;
    {
        const int64_t b = (b0 + 1) * a.rd.blk - tR0;
        if (b < 4 * S + a.dmax) brow = (int)b;
        if (THREE && b + a.rd.blk < 4 * S + a.dmax) brow2 = (int)(b + a.rd.blk);
    }
    const bool mean = a.ds_mode == 1;
    if (sl < a.sg) {                                      // waves past sg only filled
    const int s = g * a.sg + sl;
    const int cl0 = sl * CPS;
    int lrb[CPS];
    float pad0[CPS], pad1[CPS], pad2[THREE ? CPS : 1];
    // read blocks: the tile lies in block b0, or straddles b0 | b0+1 at row brow (and, for
    // THREE, b0+1 | b0+2 at row brow2: the 2560-row tiles of ds >= 6 outgrow a 2048-row block)
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
        if (THREE) pad2[cc] = pad_at(a.rd, b2, c);
        if (zap_at(a.rd, b0, c)) z0 |= 1u << cc;
        if (zap_at(a.rd, b1, c)) z1 |= 1u << cc;
        if (THREE && zap_at(a.rd, b2, c)) z2 |= 1u << cc;
    }
    z0 = __builtin_amdgcn_readfirstlane(z0);
    z1 = __builtin_amdgcn_readfirstlane(z1);
    if (!THREE) z2 = z1;
    z2 = __builtin_amdgcn_readfirstlane(z2);
    const uint32_t zany = z0 | z1 | z2, zall = z0 & z1 & z2, zsplit = (z0 ^ z1) | (z1 ^ z2);
    const int fz = zany ? __builtin_ctz(zany) : CPS;      // first channel off the integer path
    const uint32_t* lbase = lds + lane * DS;
    // Masked channels without a float fold.  With int16 output, a subband whose masked
    // channels are the same in both blocks of the tile outputs Q(D(F)), F = the oracle's float
    // fold of integers and pad values, D = /DS (mean) or identity (sum), Q = floor(x + 1/2)
    // (F >= 0).  The exact sum is R = I + DS*P (I: integer sum of the unmasked channels, P:
    // sum of the masked channels' pads of the block, exact in double) and |F - R| <= the
    // host bound a.tie_eps (which also covers the rounding of /DS), so while frac(C),
    // C = DS*P + D/2 with D = DS (mean) or 1 (sum), stays further than tie_eps from 0 and 1,
    // Q(D(F)) = floor((I + floor(C)) / D): the integer sum plus a per-block constant, then an
    // integer division (floor((n + f)/D) = floor(n/D) for integer n, 0 <= f < 1).  Integer
    // pads make F exact (no margin needed).  Outputs whose rows straddle the block boundary
    // mix both blocks' pads: when those differ (clipping on) the fixup kernel recomputes
    // them.  Near-ties, split channels (masked in one block only), negative pads and f32
    // output with masked channels take the exact float fold below.
    const int Dh = mean ? DS / 2 : 0;                     // floor(D/2) for D = DS or 1
    int cadd0 = a.sub_dtype == 0 ? Dh : 0, cadd1 = cadd0, cadd2 = cadd0;
    bool intpath = zany == 0;
    if (zany && zsplit == 0 && a.sub_dtype == 0) {
        double P0 = 0.0, P1 = 0.0, P2 = 0.0;
        bool neg = false, integral = true;
#pragma unroll
        for (int cc = 0; cc < CPS; cc++)
            if (zall & (1u << cc)) {
                const float p2 = THREE ? pad2[cc] : pad1[cc];
                P0 += (double)pad0[cc];
                P1 += (double)pad1[cc];
                P2 += (double)p2;
                neg |= pad0[cc] < 0.0f || pad1[cc] < 0.0f || p2 < 0.0f;
                integral &= pad0[cc] == floorf(pad0[cc]) && pad1[cc] == floorf(pad1[cc]) && p2 == floorf(p2);
            }
        const double half = mean ? 0.5 * DS : 0.5;
        const double C0 = (double)DS * P0 + half, C1 = (double)DS * P1 + half, C2 = (double)DS * P2 + half;
        const double f0 = C0 - floor(C0), f1 = C1 - floor(C1), f2 = C2 - floor(C2);
        const double m0 = fmin(f0, 1.0 - f0), m1 = fmin(f1, 1.0 - f1), m2 = fmin(f2, 1.0 - f2);
        const double cap = mean ? 65535.0 : 32767.0;
        if (!neg && (integral || (m0 > a.tie_eps && m1 > a.tie_eps && m2 > a.tie_eps)) &&
            fmax(fmax(C0, C1), C2) + (double)(CPS * DS * 255) <= cap) {
            intpath = true;
            cadd0 = (int)floor(C0);
            cadd1 = (int)floor(C1);
            cadd2 = (int)floor(C2);
        }
    }
    intpath = __builtin_amdgcn_readfirstlane((int)intpath) != 0;
    cadd0 = __builtin_amdgcn_readfirstlane(cadd0);
    cadd1 = __builtin_amdgcn_readfirstlane(cadd1);
    cadd2 = __builtin_amdgcn_readfirstlane(cadd2);
    if (a.qfix && pw == 0) {
        // the fixup phase below folds single outputs of any subband of the tile: its channels'
        // pads and zap flags per block slot; and whether the integer path's per-block
        // constants are wrong for outputs straddling a boundary (a channel masked in both
        // blocks whose pads differ)
        if (lane < CPS) {
            const int cc = lane, lc = cl0 + cc;
            float q0 = pad0[0], q1 = pad1[0], q2 = THREE ? pad2[0] : pad1[0];
#pragma unroll
            for (int k = 1; k < CPS; k++)
                if (cc == k) {
                    q0 = pad0[k];
                    q1 = pad1[k];
                    q2 = THREE ? pad2[k] : pad1[k];
                }
            fpad[lc] = q0;
            fpad[G + lc] = q1;
            fpad[2 * G + lc] = q2;
            fzb[lc] = (uint8_t)(((z0 >> cc) & 1u) | (((z1 >> cc) & 1u) << 1) | (((z2 >> cc) & 1u) << 2));
        }
        if (lane == 0 && intpath) {
            uint8_t nd = 0;
#pragma unroll
            for (int cc = 0; cc < CPS; cc++)
                if (zall & (1u << cc)) {
                    if (brow < (1 << 30) && pad0[cc] != pad1[cc]) nd |= 1;
                    if (THREE && brow2 < (1 << 30) && pad1[cc] != pad2[THREE ? cc : 0]) nd |= 2;
                }
            fneed[sl] = nd;
        }
    }
    // channel delays of pass p live in lanes 0..CPS-1 of vd; pass p+1's are loaded while
    // pass p is formed, so no global-load latency sits at the head of a pass
    // (unconditional, clamped loads: a branch around them would cost a vmcnt(0) drain)
    int pmax = 0;                                         // lane p: max |subband| of pass p

    const int npass = (a.probe & 1) ? 0 : a.npass;
    for (int p = pw; p < npass; p += wps) {
        // the pass's channel delays through the scalar cache (a vector load here would make
        // the loop head wait for the previous pass's output stores as well)
        int dl[CPS];
        sload_i32<CPS>(a.dly[p] + c0 + cl0, dl);
        int dmx = 0;
#pragma unroll
        for (int cc = 0; cc < CPS; cc++) dmx = max(dmx, dl[cc]);
        int amax = 0;
        if (intpath) {
            uint32_t ae[M], ao[M];
            // uniform: the tile lies in one read block, or every block's constant is the same
            // (no channel of the subband masked in every block: the constant is D/2)
            if (brow >= (1 << 30) || (cadd0 == cadd1 && cadd1 == cadd2)) {
                const uint32_t kk = (uint32_t)cadd0 | ((uint32_t)cadd0 << 16);
#pragma unroll
                for (int m = 0; m < M; m++) ae[m] = ao[m] = kk;
            } else {
#pragma unroll
                for (int m = 0; m < M; m++) {
                    // quarter q of output j: the constant of the block its last row lies in
                    const int lastrow = (lane + 64 * m) * DS + DS - 1 + dmx;
                    const uint32_t k0c = (uint32_t)cadd0, k1c = (uint32_t)cadd1, k2c = (uint32_t)cadd2;
                    const int br1 = brow, br2 = brow2;
                    // arithmetic select (a ?: chain becomes a scratch lookup table at ds >= 10)
                    auto kof = [=](int row) {
                        return k0c + (row >= br1 ? k1c - k0c : 0u) + (THREE && row >= br2 ? k2c - k1c : 0u);
                    };
                    const uint32_t k0 = kof(lastrow), k1 = kof(lastrow + S), k2 = kof(lastrow + 2 * S),
                                   k3 = kof(lastrow + 3 * S);
                    ae[m] = k0 | (k2 << 16);
                    ao[m] = k1 | (k3 << 16);
                }
            }
            // the channel sums, branch-free so every LDS read of the pass can be in flight
            // before the first add; channels masked in every block of the tile add zeros (their
            // rows were zeroed after the fill, their pads are in the constants).  All reads of
            // a group of channels first (a scheduling barrier keeps the compiler from
            // interleaving a wait after every read pair), then the adds.
            {
                constexpr int PER = M * DS, CG = PER * CPS <= 40 ? CPS : (40 / PER < 1 ? 1 : 40 / PER);
#pragma unroll
                for (int c0g = 0; c0g < CPS; c0g += CG) {
                    uint32_t xs[CG * PER];
#pragma unroll
                    for (int cc = 0; cc < CG; cc++) {
                        const uint32_t* b = lbase + lrb[min(c0g + cc, CPS - 1)] + dl[min(c0g + cc, CPS - 1)];
#pragma unroll
                        for (int m = 0; m < M; m++)
#pragma unroll
                            for (int k = 0; k < DS; k++) xs[cc * PER + m * DS + k] = b[m * 64 * DS + k];
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int cc = 0; cc < CG; cc++) {
                        if (c0g + cc >= CPS) break;
#pragma unroll
                        for (int m = 0; m < M; m++)
#pragma unroll
                            for (int k = 0; k < DS; k++) {
                                const uint32_t x = xs[cc * PER + m * DS + k];
                                ae[m] += x & 0x00FF00FFu;                              // quarters 0, 2
                                ao[m] += __builtin_amdgcn_perm(0u, x, 0x0c030c01u);    // quarters 1, 3
                            }
                    }
                }
            }
            if (a.sub_dtype == 0) {
                // int16 outputs, stored from the packed halves; mean mode divides each 16-bit
                // half by DS exactly (v = kD + r < 2^16: v * fl(1/D) + 0.5/D stays within
                // 0.5/D - 2^-7 of k + (r + 0.5)/D, so truncation gives k)
                if (mean && DS > 1) {
                    const float inv = 1.0f / (float)DS, half = 0.5f / (float)DS;
                    auto divpk = [&](uint32_t v) {
                        // DS = 2: trunc(v * 0.5f + 0.25f) = floor(v / 2) exactly, both halves at once
                        if constexpr (DS == 2) return (v >> 1) & 0x7FFF7FFFu;
                        const uint32_t lo = (uint32_t)((float)(v & 0xFFFFu) * inv + half);
                        const uint32_t hi = (uint32_t)((float)(v >> 16) * inv + half);
                        return lo | (hi << 16);
                    };
#pragma unroll
                    for (int m = 0; m < M; m++) {
                        ae[m] = divpk(ae[m]);
                        ao[m] = divpk(ao[m]);
                    }
                }
                u16x2 mx = {0, 0};
                int16_t* o = (int16_t*)a.out[p] + (int64_t)s * a.ostride[p] + tO0 + lane;
#pragma unroll
                for (int m = 0; m < M; m++) {
                    if (a.probe & 8) {                        // (profiling: sums without the stores)
                        mx = __builtin_elementwise_max(mx, __builtin_bit_cast(u16x2, ae[m] ^ ao[m]));
                        continue;
                    }
                    // non-temporal: the 22.5 GB of subbands per beam are not re-read before
                    // they leave the caches (stage 1 23.4-23.5 vs 23.7-23.9 ms per beam,
                    // profiles/r06_ab_nt_stores.txt)
                    __builtin_nontemporal_store((int16_t)(ae[m] & 0xFFFFu), o + 64 * m);
                    __builtin_nontemporal_store((int16_t)(ao[m] & 0xFFFFu), o + 64 * m + JQ);
                    __builtin_nontemporal_store((int16_t)(ae[m] >> 16), o + 64 * m + 2 * JQ);
                    __builtin_nontemporal_store((int16_t)(ao[m] >> 16), o + 64 * m + 3 * JQ);
                    mx = __builtin_elementwise_max(mx, __builtin_bit_cast(u16x2, ae[m]));
                    mx = __builtin_elementwise_max(mx, __builtin_bit_cast(u16x2, ao[m]));
                }
                amax = max((int)mx.x, (int)mx.y);
            } else {
#pragma unroll
                for (int m = 0; m < M; m++) {
                    const uint32_t qv[4] = {ae[m] & 0xFFFFu, ao[m] & 0xFFFFu, ae[m] >> 16, ao[m] >> 16};
                    q8_store<DS, MO>(a, p, s, tO0, lane + 64 * m, qv, nullptr, true, amax);
                }
            }
        } else {
#pragma unroll
            for (int m = 0; m < M; m++) {
                float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int k = 0; k < DS; k++) {
                    // oracle order: sk folds the channels from 0.0f; integer (exact) until the
                    // first masked channel, then the float fold
                    const int t = (lane + 64 * m) * DS + k;    // quarter-relative raw row
                    uint32_t pe = 0, po = 0;
                    f32x2 sk01 = {0.0f, 0.0f}, sk23 = {0.0f, 0.0f};   // quarters (0,1), (2,3): v_pk_add_f32
#pragma unroll
                    for (int cc = 0; cc < CPS; cc++) {
                        const uint32_t x = lbase[lrb[cc] + dl[cc] + m * 64 * DS + k];
                        if (cc < fz) {
                            pe += x & 0x00FF00FFu;
                            po += __builtin_amdgcn_perm(0u, x, 0x0c030c01u);
                        } else {
                            if (cc == fz) {
                                sk01 = f32x2{(float)(pe & 0xFFFFu), (float)(po & 0xFFFFu)};
                                sk23 = f32x2{(float)(pe >> 16), (float)(po >> 16)};
                            }
                            f32x2 v01 = {(float)(x & 0xFFu), (float)((x >> 8) & 0xFFu)};
                            f32x2 v23 = {(float)((x >> 16) & 0xFFu), (float)(x >> 24)};
                            if (zany & (1u << cc)) {   // masked in some block: per-row block
                                const int rr = t + dl[cc];
                                const bool za = (z0 >> cc) & 1, zb = (z1 >> cc) & 1, zc = (z2 >> cc) & 1;
                                auto cl = [&](int row, float x) {
                                    if (!THREE || row < brow2) {
                                        const bool h = row >= brow;
                                        if (h ? zb : za) x = h ? pad1[cc] : pad0[cc];
                                    } else if (zc) {
                                        x = pad2[THREE ? cc : 0];
                                    }
                                    return x;
                                };
                                v01.x = cl(rr, v01.x);
                                v01.y = cl(rr + S, v01.y);
                                v23.x = cl(rr + 2 * S, v23.x);
                                v23.y = cl(rr + 3 * S, v23.y);
                            }
                            sk01 += v01;
                            sk23 += v23;
                        }
                    }
                    acc[0] += sk01.x;
                    acc[1] += sk01.y;
                    acc[2] += sk23.x;
                    acc[3] += sk23.y;
                }
                if (mean)
#pragma unroll
                    for (int q = 0; q < 4; q++) acc[q] = acc[q] / (float)DS;
                q8_store<DS, MO>(a, p, s, tO0, lane + 64 * m, nullptr, acc, false, amax);
            }
        }
        if (a.sub_dtype == 0) {
            amax = wave_max_full(amax);
            pmax = lane == p ? amax : pmax;
        }
    }
    if (a.sub_dtype == 0 && lane < a.npass) publish_max(a.maxabs[lane], pmax);
    }                                                     // per-wave section

    if (!a.qfix || (!anyclip && brow >= (1 << 30))) return;   // uniform: nothing to redo
    // ---- fixup phase: every output of the tile that a clipped spectrum touches, and (integer
    //      path) every output whose rows straddle a read-block boundary where a masked
    //      channel's pads differ, recomputed as the oracle's exact float fold from the tile
    //      still in LDS.  Tasks are spread over all threads with their pass index per lane.
    //      Ordering: this wave's integer stores have landed in L2 before the barrier, so the
    //      fixup store of the same element (from any wave of the workgroup) lands after them.
    // the tile's clipped rows as a list (any order: every task is independent)
    for (int w = threadIdx.x; w < nwc; w += blockDim.x) {
        uint32_t bits = cflag[w];
        if (!bits) continue;
        int at = atomicAdd(&ncrow, __builtin_popcount(bits));
        for (; bits && at < kCRow; bits &= bits - 1) crow[at++] = 32 * w + __builtin_ctz(bits);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int nthr = blockDim.x;
    auto fold_store = [&](int p, int sl2, int jt, const int* dd) {
        const int q = jt / JQ, jq = jt - q * JQ;
        float acc = 0.0f;
#pragma unroll 1
        for (int k = 0; k < DS; k++) {   // rolled: an unrolled DS x CPS fold costs the hot loop VGPRs
            float sk = 0.0f;
#pragma unroll
            for (int cc = 0; cc < CPS; cc++) {
                const int lc = sl2 * CPS + cc;
                const int lr = a.rd.flip ? G - 1 - lc : lc;
                const int row = jt * DS + k + dd[cc];                    // tile-relative raw row
                const uint32_t wd = lds[lr * W + jq * DS + k + dd[cc]];
                const float xb = (float)((wd >> (8 * q)) & 0xFFu);
                const int slot = row < brow ? 0 : (!THREE || row < brow2) ? 1 : 2;
                const bool rep = ((cflag[row >> 5] >> (row & 31)) & 1u) || ((fzb[lc] >> slot) & 1u);
                sk += rep ? fpad[slot * G + lc] : xb;
            }
            acc += sk;
        }
        if (mean) acc = acc / (float)DS;
        const int s2 = g * a.sg + sl2;
        if (a.sub_dtype == 0) {
            const int16_t v = to_i16(acc, a.sub_round);
            ((int16_t*)a.out[p])[(int64_t)s2 * a.ostride[p] + tO0 + jt] = v;
            const int av = v < 0 ? -(int)v : (int)v;
            if (av > 0) atomicMax(&amax_fix[p], av);
        } else {
            ((float*)a.out[p])[(int64_t)s2 * a.ostride[p] + tO0 + jt] = acc;
        }
    };
    const int np = (a.probe & 1) ? 0 : a.npass;
    // clipped spectra: tasks (pass, clipped row, channel of the tile): the output channel c
    // maps the clipped row to, unless channel c - 1 of its subband maps it to the same output
    // (delays fall with frequency, so equal outputs are adjacent).  Rows from the list, or per
    // flag word (uniform loop) when the tile has more than kCRow of them.
    const int ncr = ncrow;
    const bool listed = ncr <= kCRow;
    for (int w = 0; w < (listed ? 1 : nwc); w++) {
        const uint32_t word = listed ? 0u : cflag[w];
        if (!listed && !word) continue;
        const int nb = listed ? ncr : __builtin_popcount(word);
        const int ntask = np * nb * G;
        for (int t = threadIdx.x; t < ntask; t += nthr) {
            const int p = t / (nb * G), r2 = t - p * (nb * G);
            const int i = r2 / G, lc = r2 - i * G;
            int R;
            if (listed) {
                R = crow[i];
            } else {
                uint32_t wb = word;
                for (int k = 0; k < i; k++) wb &= wb - 1;
                R = 32 * w + __builtin_ctz(wb);
            }
            const int sl2 = lc / CPS, cc = lc - sl2 * CPS;
            const int32_t* dp = a.dly[p] + c0 + sl2 * CPS;
            const int jn = R - dp[cc];
            if (jn < 0) continue;
            const int jt = jn / DS;
            if (jt >= 4 * JQ) continue;
            if (cc > 0) {
                const int jp = R - dp[cc - 1];
                if (jp >= 0 && jp / DS == jt) continue;
            }
            int dd[CPS];
#pragma unroll
            for (int k = 0; k < CPS; k++) dd[k] = dp[k];
            fold_store(p, sl2, jt, dd);
        }
    }
    // read-block boundaries: the outputs whose rows hold both B - 1 and B
#pragma unroll
    for (int bi = 0; bi < (THREE ? 2 : 1); bi++) {
        const int B = bi == 0 ? brow : brow2;
        if (B >= (1 << 30)) continue;
        uint32_t anyneed = 0;
        for (int k = 0; k < a.sg; k++) anyneed |= fneed[k];
        if (!((anyneed >> bi) & 1u)) continue;
        const int JB = (a.dmax + DS - 1) / DS + 2;
        const int ntask = np * a.sg * JB;
        for (int t = threadIdx.x; t < ntask; t += nthr) {
            const int p = t / (a.sg * JB), r2 = t - p * (a.sg * JB);
            const int sl2 = r2 / JB, jj = r2 - sl2 * JB;
            if (!((fneed[sl2] >> bi) & 1u)) continue;
            const int32_t* dp = a.dly[p] + c0 + sl2 * CPS;
            int dd[CPS], mind = 1 << 30, maxd = 0;
#pragma unroll
            for (int k = 0; k < CPS; k++) {
                dd[k] = dp[k];
                mind = min(mind, dd[k]);
                maxd = max(maxd, dd[k]);
            }
            int lo = B - (DS - 1) - maxd, hi = B - 1 - mind;
            lo = lo <= 0 ? 0 : (lo + DS - 1) / DS;
            hi = hi < 0 ? -1 : min(hi / DS, 4 * JQ - 1);
            const int jt = lo + jj;
            if (jt > hi) continue;
            fold_store(p, sl2, jt, dd);
        }
    }
    __syncthreads();
    if (a.sub_dtype == 0 && threadIdx.x < np) publish_max(a.maxabs[threadIdx.x], amax_fix[threadIdx.x]);
}

size_t stage1_q8_lds_bytes(const Stage1Multi& a)
{
    size_t b = (size_t)a.sg * a.cps * a.W * 4;
    if (a.qfix) {
        const int rows = 4 * stage1_q8_quarter_rows(a.ds) + a.dmax;
        const int G = a.sg * a.cps;
        b += (size_t)((rows + 31) >> 5) * 4 + (size_t)3 * G * 4 + (size_t)((G + 15) & ~15);
    }
    return b;
}

template <int CPS, int DS>
static hipError_t launch_q8_ds(const Stage1Multi& a, int vb, size_t lds, hipStream_t st)
{
    // at least 4 waves fill the tile (the fill is latency-bound); waves past sg then leave
    const dim3 block((unsigned)(64 * (a.sg < 4 ? 4 : a.sg) * (a.sg >= 4 && a.wps2 ? 2 : 1))),
        grid((unsigned)(a.ntiles * a.ngroups));
    if (DS == 1 && q8_m1() == 2) {
        if (vb == 8) hipLaunchKernelGGL((k_stage1_q8<CPS, DS, 8, 2>), grid, block, lds, st, a);
        else hipLaunchKernelGGL((k_stage1_q8<CPS, DS, 4, 2>), grid, block, lds, st, a);
    } else if (vb == 8) hipLaunchKernelGGL((k_stage1_q8<CPS, DS, 8>), grid, block, lds, st, a);
    else hipLaunchKernelGGL((k_stage1_q8<CPS, DS, 4>), grid, block, lds, st, a);
    return hipGetLastError();
}

template <int CPS, int DS>
static hipError_t set_lds_q8_ds(int bytes)
{
    hipError_t e = set_max_lds((const void*)k_stage1_q8<CPS, DS, 8>, bytes);
    if (e == hipSuccess) e = set_max_lds((const void*)k_stage1_q8<CPS, DS, 4>, bytes);
    if (DS == 1 && e == hipSuccess) e = set_max_lds((const void*)k_stage1_q8<CPS, DS, 8, 2>, bytes);
    if (DS == 1 && e == hipSuccess) e = set_max_lds((const void*)k_stage1_q8<CPS, DS, 4, 2>, bytes);
    return e;
}

#define HD_Q8_FOR_CPS(X) X(10) X(8) X(16)
#define HD_Q8_FOR_DS(C, X) X(C, 1) X(C, 2) X(C, 3) X(C, 5) X(C, 6) X(C, 10)

bool stage1_q8_supports(int cps, int ds)
{
    return (cps == 10 || cps == 8 || cps == 16) && stage1_q8_quarter_rows(ds) > 0 && cps * ds * 255 < 32768;
}

hipError_t stage1_q8_set_lds_limit(size_t bytes)
{
    hipError_t e = hipSuccess;
    const int b = (int)bytes;
#define HD_SETQ(C, D) \
    if (e == hipSuccess) e = set_lds_q8_ds<C, D>(b);
#define HD_SETQC(C) HD_Q8_FOR_DS(C, HD_SETQ)
    HD_Q8_FOR_CPS(HD_SETQC)
#undef HD_SETQC
#undef HD_SETQ
    return e;
}

hipError_t launch_stage1_q8(const Stage1Multi& a, int vb, hipStream_t st)
{
    if (a.nds <= 0 || a.npass <= 0 || a.ntiles <= 0) return hipSuccess;
    const size_t lds = stage1_q8_lds_bytes(a);
#define HD_LQ(C, D) \
    if (a.cps == C && a.ds == D) return launch_q8_ds<C, D>(a, vb, lds, st);
#define HD_LQC(C) HD_Q8_FOR_DS(C, HD_LQ)
    HD_Q8_FOR_CPS(HD_LQC)
#undef HD_LQC
#undef HD_LQ
    return hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------
// channel-major copy of an 8- or 4-bit raw block (k_stage1_q8's and k_stage1_fix8's source)
// ------------------------------------------------------------------------------------
// Tile = 128 rows x 128 channels: coalesced row reads into LDS, then per thread 4x4 byte
// transposes of 4 rows x 4 channels and 128-B channel runs out.  rawT[c][t] = raw[t][c] as one
// byte per sample: 4-bit data is unpacked on the way into LDS (file channel 2k is the high
// nibble of byte k when nibble_hi_first, as raw_value decodes it), so the 8-bit integer
// stage-1 path runs 4-bit beams (PALFA's production format) unchanged.  The kRawTPad bytes
// after N in every channel row are zeroed by the host allocation.
template <int NB>
__global__ __launch_bounds__(256) void k_raw_transpose(const uint8_t* __restrict__ raw, int64_t N, int32_t nchan,
                                                      int nibble_hi_first, uint8_t* __restrict__ rawT, int64_t tstride)
{
    __shared__ uint32_t tile[128][33];
    // 1-D grid, XCD-aware: workgroup L runs on XCD L % 8; its s-th workgroup there takes
    // channel tile s % nct of time block (s / nct) * 8 + L % 8, so the nct channel tiles of
    // one time block run back to back on one XCD.  Raw rows are 960 B (64-B aligned), so
    // half the 128-B row pieces straddle two cache lines, which the neighbouring channel
    // tile then finds in that XCD's L2 instead of fetching from HBM again.
    const int nct = (nchan + 127) >> 7;
    const int xcd = blockIdx.x & 7, sl = blockIdx.x >> 3;
    const int64_t tb = (int64_t)(sl / nct) * 8 + xcd;
    if (tb * 128 >= N) return;
    const int64_t t0 = tb * 128;
    const int c0 = (sl % nct) * 128;
    const int rb = nchan * NB / 8;                          // bytes per raw row
    const int ncw = min(128, nchan - c0) >> 2;              // 8-bit channel dwords in this tile
    if constexpr (NB == 8) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int idx = threadIdx.x + 256 * k;
            const int row = idx >> 5, col = idx & 31;
            uint32_t v = 0;
            if (t0 + row < N && col < ncw) v = *(const uint32_t*)(raw + (t0 + row) * rb + c0 + 4 * col);
            tile[row][col] = v;
        }
    } else {
        // one raw dword = 8 channels: H = high nibbles, L = low nibbles of its 4 bytes; the
        // output bytes interleave them in file-channel order (first nibble first)
        const uint32_t s0 = 0x05010400u, s1 = 0x07030602u;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int idx = threadIdx.x + 256 * k;
            const int row = idx >> 4, col = idx & 15;
            uint32_t v = 0;
            if (t0 + row < N && 2 * col < ncw) v = *(const uint32_t*)(raw + (t0 + row) * rb + c0 / 2 + 4 * col);
            const uint32_t H = (v >> 4) & 0x0F0F0F0Fu, L = v & 0x0F0F0F0Fu;
            const uint32_t F = nibble_hi_first ? H : L, Sd = nibble_hi_first ? L : H;
            tile[row][2 * col] = __builtin_amdgcn_perm(Sd, F, s0);
            tile[row][2 * col + 1] = __builtin_amdgcn_perm(Sd, F, s1);
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int b = threadIdx.x + 256 * k;
        const int rbk = b & 31, cb = b >> 5;                // rows 4rbk..4rbk+3, channels 4cb..4cb+3
        if (cb >= ncw) continue;
        const uint32_t r0 = tile[4 * rbk][cb], r1 = tile[4 * rbk + 1][cb], r2 = tile[4 * rbk + 2][cb],
                       r3 = tile[4 * rbk + 3][cb];
        const uint32_t ab_lo = __builtin_amdgcn_perm(r1, r0, 0x05010400u);
        const uint32_t ab_hi = __builtin_amdgcn_perm(r1, r0, 0x07030602u);
        const uint32_t cd_lo = __builtin_amdgcn_perm(r3, r2, 0x05010400u);
        const uint32_t cd_hi = __builtin_amdgcn_perm(r3, r2, 0x07030602u);
        const uint32_t o4[4] = {__builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u),
                                __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u),
                                __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u),
                                __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u)};
        const int64_t t = t0 + 4 * rbk;
        if (t < N) {
#pragma unroll
            for (int i = 0; i < 4; i++) *(uint32_t*)(rawT + (int64_t)(c0 + 4 * cb + i) * tstride + t) = o4[i];
        }
    }
}

hipError_t launch_raw_transpose(const uint8_t* raw, int64_t N, int32_t nchan, int nbits, int nibble_hi_first,
                                uint8_t* rawT, int64_t tstride, hipStream_t st)
{
    if (nchan % (nbits == 4 ? 8 : 4) || N % 4 || (nbits != 8 && nbits != 4)) return hipErrorInvalidValue;
    const int64_t ntb8 = ((N + 127) / 128 + 7) / 8 * 8;          // time blocks, padded to the 8 XCDs
    const int64_t nwg = ntb8 * ((nchan + 127) / 128);
    if (nwg > 0x7fffffffLL) return hipErrorInvalidValue;
    if (nbits == 8)
        hipLaunchKernelGGL(k_raw_transpose<8>, dim3((unsigned)nwg), dim3(256), 0, st, raw, N, nchan, nibble_hi_first,
                           rawT, tstride);
    else
        hipLaunchKernelGGL(k_raw_transpose<4>, dim3((unsigned)nwg), dim3(256), 0, st, raw, N, nchan, nibble_hi_first,
                           rawT, tstride);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// padding
// ------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_pad(float* out, int64_t out_stride, int64_t nds, int64_t numout,
                                            const double* partial, int ntiles, int pad_mode)
{
    __shared__ double red[256];
    __shared__ float padv;
    const int d = blockIdx.x;
    // HD_PAD_DM0: every DM takes the first DM's mean (prepsubband's one `avg`)
    const int dsrc = pad_mode == 2 ? 0 : d;
    double s = 0.0;
    if (pad_mode != 1 && partial)
        for (int i = threadIdx.x; i < ntiles; i += 256) s += partial[(int64_t)dsrc * ntiles + i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w >= 1; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) padv = (pad_mode != 1 && nds > 0) ? (float)(red[0] / (double)nds) : 0.0f;
    __syncthreads();
    const float v = padv;
    for (int64_t t = nds + threadIdx.x; t < numout; t += 256) out[(int64_t)d * out_stride + t] = v;
}

hipError_t launch_pad(float* out, int64_t out_stride, int numdms, int64_t nds, int64_t numout,
                      const double* partial, int ntiles, int pad_mode, hipStream_t st)
{
    if (numout <= nds || numdms <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pad, dim3((unsigned)numdms), dim3(256), 0, st, out, out_stride, nds, numout,
                       partial, ntiles, pad_mode);
    return hipGetLastError();
}

// ---- barycentric output: padding values, then the segments of the barycentred series ----
__global__ __launch_bounds__(256) void k_padvals(const double* partial, int ntiles, int64_t nds, int pad_mode,
                                                float* padv)
{
    __shared__ double red[256];
    const int d = blockIdx.x;
    const int dsrc = pad_mode == 2 ? 0 : d;                 // as k_pad
    double s = 0.0;
    if (pad_mode != 1 && partial)
        for (int i = threadIdx.x; i < ntiles; i += 256) s += partial[(int64_t)dsrc * ntiles + i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w >= 1; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) padv[d] = (pad_mode != 1 && nds > 0 && partial) ? (float)(red[0] / (double)nds) : 0.0f;
}

// One workgroup per (2048 output samples, DM): each sample finds its segment {out0, src0, len}
// (binary search over the segment starts staged in LDS in pieces of kBarySegLds), then copies
// topo[src0 + j - out0] or writes the padding value.  Reads are contiguous within a segment.
constexpr int kBarySegLds = 2048;
__global__ __launch_bounds__(256) void k_bary(const float* __restrict__ topo, float* __restrict__ out, int64_t stride,
                                             int64_t numout, const int32_t* __restrict__ seg, int nseg,
                                             const float* __restrict__ padv)
{
    __shared__ int32_t s_out0[kBarySegLds];
    __shared__ int lo_s, hi_s;
    const int d = blockIdx.y;
    const int64_t j0 = (int64_t)blockIdx.x * 2048;
    const int64_t j1 = j0 + 2048 < numout ? j0 + 2048 : numout;
    if (threadIdx.x == 0) {
        // segments overlapping [j0, j1): first = last k with out0[k] <= j0
        int lo = 0, hi = nseg - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (seg[3 * mid] <= j0) lo = mid;
            else hi = mid - 1;
        }
        int last = lo;
        while (last + 1 < nseg && seg[3 * (last + 1)] < j1) last++;
        lo_s = lo;
        hi_s = last;
    }
    __syncthreads();
    const int k0 = lo_s, nk = hi_s - lo_s + 1;
    const float pv = padv[d];
    const float* tp = topo + (int64_t)d * stride;
    float* op = out + (int64_t)d * stride;
    if (nk == 1) {                                            // uniform: one segment
        const int64_t o0 = seg[3 * k0], s0 = seg[3 * k0 + 1];
        for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) op[j] = s0 < 0 ? pv : tp[s0 + (j - o0)];
        return;
    }
    for (int i = threadIdx.x; i < nk && i < kBarySegLds; i += 256) s_out0[i] = seg[3 * (k0 + i)];
    __syncthreads();
    const int nl = nk < kBarySegLds ? nk : kBarySegLds;
    for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) {
        int lo = 0, hi = nl - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_out0[mid] <= j) lo = mid;
            else hi = mid - 1;
        }
        int k = k0 + lo;
        while (k + 1 < nseg && seg[3 * (k + 1)] <= j) k++;     // beyond the staged piece (rare)
        const int64_t o0 = seg[3 * k], s0 = seg[3 * k + 1];
        op[j] = s0 < 0 ? pv : tp[s0 + (j - o0)];
    }
}

hipError_t launch_bary(const float* topo, float* out, int64_t stride, int numdms, int64_t numout, const int32_t* seg,
                       int nseg, const double* partial, int ntiles, int64_t nds, int pad_mode, float* padv,
                       hipStream_t st)
{
    if (numdms <= 0 || numout <= 0 || nseg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_padvals, dim3((unsigned)numdms), dim3(256), 0, st, partial, ntiles, nds, pad_mode, padv);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bary, dim3((unsigned)((numout + 2047) / 2048), (unsigned)numdms), dim3(256), 0, st, topo, out,
                       stride, numout, seg, nseg, padv);
    return hipGetLastError();
}

// ---- series sums and fills (time-sliced passes: the padding value is the observation's) --
__global__ __launch_bounds__(256) void k_series_sum(const float* __restrict__ x, int64_t n, double* __restrict__ part)
{
    __shared__ double red[256];
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc += (double)x[i];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w >= 1; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

hipError_t launch_series_sum(const float* x, int64_t n, double* part, int nparts, hipStream_t st)
{
    hipLaunchKernelGGL(k_series_sum, dim3((unsigned)nparts), dim3(256), 0, st, x, n, part);
    return hipGetLastError();
}

__global__ __launch_bounds__(64) void k_zero_list(ZeroList z, int n)
{
    if ((int)threadIdx.x < n) *z.p[threadIdx.x] = 0;
}

hipError_t launch_zero_list(const ZeroList& z, int n, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    if (n > kMaxPass) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_zero_list, dim3(1), dim3(64), 0, st, z, n);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_series_fill(float* out, int64_t out_stride, int64_t t0, int64_t t1, float v)
{
    float* o = out + (int64_t)blockIdx.y * out_stride;
    for (int64_t t = t0 + (int64_t)blockIdx.x * 256 + threadIdx.x; t < t1; t += (int64_t)gridDim.x * 256) o[t] = v;
}

hipError_t launch_series_fill(float* out, int64_t out_stride, int numdms, int64_t t0, int64_t t1, float v, hipStream_t st)
{
    if (t1 <= t0 || numdms <= 0) return hipSuccess;
    const int64_t nb = std::min<int64_t>((t1 - t0 + 255) / 256, 1024);
    hipLaunchKernelGGL(k_series_fill, dim3((unsigned)nb, (unsigned)numdms), dim3(256), 0, st, out, out_stride, t0, t1, v);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// synthetic beam
// ------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_synth(uint8_t* raw, int64_t N, int32_t rowbytes,
                                              const hd_synth_tab* __restrict__ tb, int64_t t0)
{
    const int32_t *base_q4, *noise_mul, *rfi_flag;
    const int64_t *psr_delay, *sp_delay;
    hd_synth_arrays(tb, &base_q4, &noise_mul, &rfi_flag, &psr_delay, &sp_delay);
    const int64_t total = N * rowbytes;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t t = i / rowbytes;
        const int32_t b = (int32_t)(i - t * rowbytes);
        raw[i] = hd_synth_byte(tb, base_q4, noise_mul, rfi_flag, psr_delay, sp_delay, t0 + t, b);
    }
}

hipError_t launch_synth(uint8_t* raw, int64_t N, int32_t rowbytes, const hd_synth_tab* tab_dev, int64_t t0,
                        hipStream_t st)
{
    const int64_t total = N * rowbytes;
    int64_t nb = (total + 255) / 256;
    if (nb > 256 * 64) nb = 256 * 64;
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)nb), dim3(256), 0, st, raw, N, rowbytes, tab_dev, t0);
    return hipGetLastError();
}

}  // namespace hd
