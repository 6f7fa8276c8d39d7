// hd_kernels.hip — CDNA4 (gfx950) kernels of the dedispersion engine.
//
//   k_stage1_direct  raw PSRFITS block -> nsub subbands at subdm, downsampled, int16/f32
//                    (prepsubband -sub; reference PALFA2_presto_search.py:506-511)
//   k_stage2_direct  subbands -> numdms DM series, one output per thread, global reads
//   k_stage2_lds     same result; LDS-tiled: 4 shifted copies of each subband window so
//                    every lane reads 4 consecutive samples with one aligned ds_read_b64,
//                    packed int16 accumulation (v_pk_add_u16) widened to int32 every G
//                    subbands (G from the pass's max |subband|, so no wrap is possible)
//                    (prepsubband -lodm/-dmstep/-numdms; PALFA2_presto_search.py:514-520)
//   k_pad            first-DM (prepsubband) or per-DM mean (reduction of per-tile partials,
//                    exact for int16 subbands) fill of samples [N/ds, numout)
//   k_synth          synthetic beam, bit-identical to the host generator
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
                                             int64_t tO0, int lane, int s, int p, int& amax)
{
    // Two outputs per lane per iteration (j, j+64): two independent add chains for ILP.
    // Uniform trip count; only the last iteration can diverge.
    const int jmax = (int)min((int64_t)a.to, a.nds - tO0);
    for (int j0 = lane; j0 < jmax; j0 += 128) {
        const bool has1 = j0 + 64 < jmax;
        const int j1 = has1 ? j0 + 64 : j0;          // duplicate work, result discarded
        const int jr0 = j0 * a.ds, jr1 = j1 * a.ds;
        float acc0 = 0.0f, acc1 = 0.0f;
        for (int k = 0; k < a.ds; k++) {
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
            acc0 = acc0 / (float)a.ds;
            acc1 = acc1 / (float)a.ds;
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
        int amax = 0;
        if (!SPECIAL) {
            if (!any_zap)
                form_outputs<NBITS, CPS, CALIB, kModeClean, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax);
            else
                form_outputs<NBITS, CPS, CALIB, kModeFast, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax);
        } else if (!tail) {
            if (mode == kModeFast)
                form_outputs<NBITS, CPS, CALIB, kModeFast, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax);
            else if (mode == kModeTwo)
                form_outputs<NBITS, CPS, CALIB, kModeTwo, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax);
            else
                form_outputs<NBITS, CPS, CALIB, kModeGen, false>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax);
        } else {
            form_outputs<NBITS, CPS, CALIB, kModeGen, true>(a, lraw, st, livr, lrc0, brow, rows_valid, tO0, lane, s, p, amax);
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

template <int DS>
struct Q8Geom {
    static constexpr int M = DS == 1 ? 4 : DS == 2 ? 2 : 1;   // outputs per lane per quarter
    static constexpr int JQ = 64 * M;                          // outputs per quarter
    static constexpr int S = JQ * DS;                          // dwords (raw rows) per quarter
    static constexpr bool THREE = DS >= 10;                    // 4S + dmax may exceed a 2048-row block
};

int stage1_q8_quarter_rows(int ds)
{
    switch (ds) {
    case 1: return Q8Geom<1>::S;
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
template <int DS>
__device__ __forceinline__ void q8_store(const Stage1Multi& a, int p, int s, int64_t tO0, int j,
                                         const uint32_t* qv, const float* qf, bool integral, int& amax)
{
    constexpr int JQ = Q8Geom<DS>::JQ;
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
    return (a.probe & 16) || a.sg >= 4 ? 1 : 4 / a.sg;
}

template <int CPS, int DS, int VB>
__global__ __launch_bounds__(256) void k_stage1_q8(Stage1Multi a)
{
    constexpr bool THREE = Q8Geom<DS>::THREE;
    using Gm = Q8Geom<DS>;
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
    if (a.qfix) {
        for (int w = threadIdx.x; w < nwc; w += blockDim.x) {
            uint32_t bits = 0;
            if (a.rd.clipped)
                for (int b = 0; b < 32; b++) {
                    const int r = 32 * w + b;
                    if (r < rows_t && a.rd.clipped[tR0 + r]) bits |= 1u << b;
                }
            cflag[w] = bits;
        }
        if (threadIdx.x < kMaxPass) amax_fix[threadIdx.x] = 0;
        if (threadIdx.x < 8) fneed[threadIdx.x] = 0;
    }
    __syncthreads();

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
    const int dlane = c0 + cl0 + min(lane, CPS - 1);
    int vd = a.dly[min(pw, a.npass - 1)][dlane];
    int pmax = 0;                                         // lane p: max |subband| of pass p

    const int npass = (a.probe & 1) ? 0 : a.npass;
    for (int p = pw; p < npass; p += wps) {
        const int vd_next = a.dly[min(p + wps, a.npass - 1)][dlane];
        int dl[CPS];
        int dmx = 0;
#pragma unroll
        for (int cc = 0; cc < CPS; cc++) {
            dl[cc] = __builtin_amdgcn_readlane(vd, cc);
            dmx = max(dmx, dl[cc]);
        }
        int amax = 0;
        if (intpath) {
            uint32_t ae[M], ao[M];
            if (brow >= (1 << 30)) {                   // uniform: the tile lies in one read block
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
            // before the first add; channels masked in every block of the tile (their pads are
            // in the constants) are ANDed away by a uniform mask
            if (zall == 0) {
                // all reads of a group of channels first (a scheduling barrier keeps the
                // compiler from interleaving a wait after every read pair), then the adds
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
            } else {
#pragma unroll
                for (int cc = 0; cc < CPS; cc++) {
                    const uint32_t keep = ((zall >> cc) & 1u) ? 0u : 0xFFFFFFFFu;
                    const uint32_t* b = lbase + lrb[cc] + dl[cc];
#pragma unroll
                    for (int m = 0; m < M; m++)
#pragma unroll
                        for (int k = 0; k < DS; k++) {
                            const uint32_t x = b[m * 64 * DS + k] & keep;
                            ae[m] += x & 0x00FF00FFu;
                            ao[m] += __builtin_amdgcn_perm(0u, x, 0x0c030c01u);
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
                    o[64 * m] = (int16_t)(ae[m] & 0xFFFFu);
                    o[64 * m + JQ] = (int16_t)(ao[m] & 0xFFFFu);
                    o[64 * m + 2 * JQ] = (int16_t)(ae[m] >> 16);
                    o[64 * m + 3 * JQ] = (int16_t)(ao[m] >> 16);
                    mx = __builtin_elementwise_max(mx, __builtin_bit_cast(u16x2, ae[m]));
                    mx = __builtin_elementwise_max(mx, __builtin_bit_cast(u16x2, ao[m]));
                }
                amax = max((int)mx.x, (int)mx.y);
            } else {
#pragma unroll
                for (int m = 0; m < M; m++) {
                    const uint32_t qv[4] = {ae[m] & 0xFFFFu, ao[m] & 0xFFFFu, ae[m] >> 16, ao[m] >> 16};
                    q8_store<DS>(a, p, s, tO0, lane + 64 * m, qv, nullptr, true, amax);
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
                q8_store<DS>(a, p, s, tO0, lane + 64 * m, nullptr, acc, false, amax);
            }
        }
        if (a.sub_dtype == 0) {
            amax = wave_max_i32(amax);
            pmax = lane == p ? amax : pmax;
        }
        vd = vd_next;
    }
    if (a.sub_dtype == 0 && lane < a.npass) publish_max(a.maxabs[lane], pmax);
    }                                                     // per-wave section

    if (!a.qfix) return;                                  // uniform
    // ---- fixup phase: every output of the tile that a clipped spectrum touches, and (integer
    //      path) every output whose rows straddle a read-block boundary where a masked
    //      channel's pads differ, recomputed as the oracle's exact float fold from the tile
    //      still in LDS.  Tasks are spread over all threads with their pass index per lane.
    //      Ordering: this wave's integer stores have landed in L2 before the barrier, so the
    //      fixup store of the same element (from any wave of the workgroup) lands after them.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int nthr = blockDim.x;
    auto fold_store = [&](int p, int sl2, int jt, const int* dd) {
        const int q = jt / JQ, jq = jt - q * JQ;
        float acc = 0.0f;
        for (int k = 0; k < DS; k++) {
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
    // clipped spectra: per flag word (uniform loop), tasks (pass, set bit, channel of the
    // tile): the output channel c maps the clipped row to, unless channel c - 1 of its subband
    // maps it to the same output (delays fall with frequency, so equal outputs are adjacent)
    for (int w = 0; w < nwc; w++) {
        const uint32_t word = cflag[w];
        if (!word) continue;
        const int nb = __builtin_popcount(word);
        const int ntask = np * nb * G;
        for (int t = threadIdx.x; t < ntask; t += nthr) {
            const int p = t / (nb * G), r2 = t - p * (nb * G);
            const int i = r2 / G, lc = r2 - i * G;
            uint32_t wb = word;
            for (int k = 0; k < i; k++) wb &= wb - 1;
            const int R = 32 * w + __builtin_ctz(wb);
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
    const dim3 block((unsigned)(64 * (a.sg < 4 ? 4 : a.sg))), grid((unsigned)(a.ntiles * a.ngroups));
    if (vb == 8) hipLaunchKernelGGL((k_stage1_q8<CPS, DS, 8>), grid, block, lds, st, a);
    else hipLaunchKernelGGL((k_stage1_q8<CPS, DS, 4>), grid, block, lds, st, a);
    return hipGetLastError();
}

template <int CPS, int DS>
static hipError_t set_lds_q8_ds(int bytes)
{
    hipError_t e = set_max_lds((const void*)k_stage1_q8<CPS, DS, 8>, bytes);
    if (e == hipSuccess) e = set_max_lds((const void*)k_stage1_q8<CPS, DS, 4>, bytes);
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

template <int Q, int R, int PPC>
__global__ __launch_bounds__(1024) void k_stage2_pair(Stage2Args a, const int32_t* __restrict__ boff)
{
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
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
    const int umax = a.umax;
    const int slot_bytes = (2 * PPC * npw + nbp) * 1024;
    const int npair = a.nsub >> 1;
    const int tab_bytes = npair * kPairTab * 4;
    int32_t* ltab = (int32_t*)lds_raw;
    const uint32_t ring0 = (uint32_t)tab_bytes;
    const uint32_t exp0 = ring0 + (uint32_t)(NS * slot_bytes);
    const uint32_t lane_byte = exp0 + (uint32_t)lane * 8u;   // host offsets are relative to exp0
    const int16_t* sub = (const int16_t*)a.sub;
    const int32_t* bo_g = boff + (int64_t)yb * npair * dpb;
    const int nchunk = npair / PPC;

    for (int i = threadIdx.x; i < npair * kPairTab; i += nthr) ltab[i] = a.ptab[(int64_t)yb * npair * kPairTab + i];
    __syncthreads();

    int maxabs = *a.maxabs;
    maxabs = maxabs < 1 ? 1 : maxabs;
    int G = 32767 / (2 * maxabs);                      // pairs per packed-int16 group
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
            const char* src = (const char*)(sub + (int64_t)s * a.sub_stride + e0) + pc * 1024;
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
#pragma unroll
        for (int k = 0; k < PPC; k++) {
            const uint32_t* S0 = (const uint32_t*)(slot + (2 * k) * npw * 1024);
            const uint32_t* S1 = (const uint32_t*)(slot + (2 * k + 1) * npw * 1024);
            const int32_t* pt = ltab + (PPC * chk + k) * kPairTab;
            const int k0 = pt[0] & 1;
            const int U = pt[2];
            int16_t* buf = (int16_t*)(lds_raw + exp0) + ((cc & 1) * PPC + k) * (umax * 4 * ws);
            for (int idx = threadIdx.x; idx < U * upw; idx += nthr) {
                int u = 0, uu = idx;
#pragma unroll
                for (int m = 1; m < kPairUMax; m++)
                    if (uu >= upw) { uu -= upw; u++; }
                uint32_t A[4], B[4], P[4];
                load8_shift(S0, k0 + 4 * uu, A);
                load8_shift(S1, pt[3 + u] + 4 * uu, B);
#pragma unroll
                for (int m = 0; m < 4; m++)
                    P[m] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2v, A[m]) + __builtin_bit_cast(short2v, B[m]));
                uint2* dst0 = (uint2*)(buf + (u * 4) * ws);
                const uint32_t h1 = __builtin_amdgcn_alignbit(P[1], P[0], 16);
                const uint32_t h3 = __builtin_amdgcn_alignbit(P[2], P[1], 16);
                const uint32_t h5 = __builtin_amdgcn_alignbit(P[3], P[2], 16);
                dst0[uu] = make_uint2(P[0], P[1]);
                dst0[upw + uu] = make_uint2(h1, h3);
                dst0[2 * upw + uu] = make_uint2(P[1], P[2]);
                dst0[3 * upw + uu] = make_uint2(h3, h5);
            }
        }
    };

    auto flush = [&](int tile) {
        const int64_t t0 = (int64_t)tile * T;
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
        if (!(a.probe & 2)) dma(c + NS - 1);   // probe 2: no window DMA after the prologue
        const int chn = chk + 1 == nchunk ? 0 : chk + 1;
        if (c + 1 < ntot && !(a.probe & 8)) expand(c + 1, chn);
        // this chunk's per-DM byte offsets: pair k, DM entry q in lane q of voff[k]
        const int32_t* sboff = (const int32_t*)(lds_raw + ring0 + (c % NS) * slot_bytes + 2 * PPC * npw * 1024);
        int voff[PPC];
#pragma unroll
        for (int k = 0; k < PPC; k++) voff[k] = lane < Q ? sboff[k * dpb + wave * Q + lane] : 0;
        if (!(a.probe & 1)) {
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
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NS - 3) : "memory");
        ring_barrier();
        // tile done: its stores go out after this chunk's DMA wait, so they do not hold it up
        if (chk == nchunk - 1) flush(tb + ktile++);
        chk = chn;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the workgroup ends

}

size_t stage2_pair_lds_bytes(int wstride, int npw, int nbp, int nsub, int umax, int ppc)
{
    const int ns = ppc == 2 ? 4 : kRingNS;
    return (size_t)(nsub / 2) * kPairTab * 4 + (size_t)ns * (2 * ppc * npw + nbp) * 1024 +
           (size_t)2 * ppc * umax * 4 * wstride * 2;
}

template <int Q, int R, int PPC>
static hipError_t launch_pair_qrp(const Stage2Args& a, int nyblk, hipStream_t st)
{
    {
        const hipError_t e = set_max_lds((const void*)k_stage2_pair<Q, R, PPC>, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    const unsigned ntiles = (unsigned)((a.nvalid + 256 * R - 1) / (256 * R));
    const unsigned nx = a.nwg > 0 && (unsigned)a.nwg < ntiles ? (unsigned)a.nwg : ntiles;
    Stage2Args b = a;
    if (nx == ntiles) b.nwg = 0;
    hipLaunchKernelGGL((k_stage2_pair<Q, R, PPC>), dim3(nx, (unsigned)nyblk), dim3(1024),
                       stage2_pair_lds_bytes(a.wstride, a.ring_npw, a.ring_nbp, a.nsub, a.umax, PPC), st, b, a.off);
    return hipGetLastError();
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

hipError_t launch_stage2_pair(const Stage2Args& a, int q, int r, int ppc, hipStream_t st)
{
    if (a.nvalid <= 0) return hipSuccess;
    if (ppc != 1 && ppc != 2) return hipErrorInvalidValue;
    const int nyblk = (a.numdms + a.dms_per_blk - 1) / a.dms_per_blk;
#define HD_PL(QQ, RR)                                                                             \
    if (q == QQ && r == RR)                                                                       \
        return ppc == 2 ? launch_pair_qrp<QQ, RR, 2>(a, nyblk, st) : launch_pair_qrp<QQ, RR, 1>(a, nyblk, st);
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
