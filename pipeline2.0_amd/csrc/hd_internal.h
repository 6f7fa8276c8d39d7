// hd_internal.h — internal types shared by the C-ABI layer (hd_api.hip) and the
// kernel launchers (hd_kernels.hip).  Nothing here crosses the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hd_synth_core.h"
#include "../../include/hipdedisp.h"

namespace hd {

// Raw-sample decode parameters for stage 1 (all device pointers).  The raw block is read
// in blocks of `blk` spectra (PRESTO's read unit, one PSRFITS subint): per block, an rfifind
// zap row (mask.c check_mask of the block) and the pad values in force (clip_times' running
// channel levels when clipping, else the initial pad values); spectra clip_times replaced
// read as the block's pad values, and spectra past N as the last block's.
struct RawDesc {
    const uint8_t* raw;       // [N][rowbytes], file layout
    int64_t N;
    int32_t rowbytes, nchan, nbits, flip, nibble_hi_first, be16;
    const float* scl;         // per raw channel or nullptr
    const float* offs;
    const float* wts;
    int32_t blk, nblk;        // read blocks: nblk = ceil(N / blk)
    int32_t blk_shift;        // log2(blk) when blk is a power of two, else -1
    const int32_t* zidx;      // [nblk] row of zrows zapped in the block, or nullptr (no mask)
    const uint8_t* zrows;     // [rows][nchan] ascending channels, 1 = zapped
    const float* pad;         // [nblk][nchan] (pad_stride = nchan) or [1][nchan] (stride 0), or nullptr (0)
    int32_t pad_stride;
    const uint8_t* clipped;   // [N] 1 = spectrum replaced by clip_times, or nullptr
    const uint32_t* clipbits; // the same flags bit-packed: bit t % 32 of word t / 32 (with clipped)
};

struct Stage1Args {
    RawDesc rd;
    const int32_t* idispdt;   // [nchan]
    int32_t nsub, cps, ds, ds_mode, sub_dtype, sub_round, maxdelay;
    int64_t nds;              // output samples per subband
    int64_t out_stride;       // elements
    void* out;                // [nsub][out_stride]
    int32_t* maxabs;          // device int: max |subband value| (i16 path), atomicMax
};

// Tiled stage 1 over up to kMaxPass passes that share nsub and ds (one DDplan stage):
// every workgroup copies a raw tile (sg subbands x (to*ds + dmax) spectra) into LDS once
// and forms the subbands of all its passes from it.
constexpr int kMaxPass = 32;
struct Stage1Multi {
    RawDesc rd;
    int32_t npass;
    int32_t nsub, cps, ds, ds_mode, sub_dtype, sub_round;
    int64_t nds, out_stride;
    int32_t sg;               // subbands per workgroup (block = 64*sg threads)
    int32_t to;               // output samples per tile
    int32_t dmax;             // max channel delay over the passes
    int32_t rs;               // LDS bytes per raw row (multiple of 4, odd dword count)
    int32_t W;                // 8-bit integer path: LDS dwords per channel row (>= S + dmax)
    int32_t two_ok;           // read-block boundaries a non-special tile may straddle (0, 1; q8 ds >= 10: 2)
    int32_t probe;            // profiling only: bit0 skip subband formation, bit1 skip fill
    int32_t qfix;             // 8-bit integer path: recompute clipped-spectrum / read-block-boundary
                              // outputs inside k_stage1_q8 (no separate fixup launch)
    double tie_eps;           // 8-bit integer path: margin the rounding of a masked subband's pad
                              // constant needs (float-fold error, plus the /ds rounding in mean mode)
    int32_t ntiles, ngroups;
    int32_t pass_ds;                // k_stage1_fix8 / SPECIAL k_stage1_tiled: 1 = per-pass ds in pds[]
    int32_t wps2;                   // k_stage1_q8 with sg >= 4: 2 waves per subband (8-wave blocks)
    int32_t pds[kMaxPass];          // k_stage1_q8m / pass_ds: per-pass downsampling
    double ptie[kMaxPass];          // k_stage1_q8m: per-pass tie_eps (its ds)
    const int32_t* dly[kMaxPass];   // per-pass idispdt [nchan]
    void* out[kMaxPass];            // per-pass subbands [nsub][out_stride]
    int32_t* maxabs[kMaxPass];      // per-pass max |subband|
    int64_t ostride[kMaxPass];      // per-pass subband row stride (elements; rows carry a zero tail)
    // 8-bit integer path: channel-major copy of the raw block ([nchan][tstride] bytes, file
    // channel order, zero tail) or nullptr (row-major fill from rd.raw)
    const uint8_t* rawT;
    int64_t tstride;
    // k_stage1_fix8 boundary items (host list): per chunk of fix_G channels, the read-block
    // boundaries bb (blocks bb-1, bb) where a channel of the chunk is zapped in both blocks --
    // fix_blist[fix_bofs[k] .. fix_bofs[k+1]); nullptr: every boundary is tried
    const int32_t* fix_blist;
    const int32_t* fix_bofs;
    int32_t fix_G;
};
// channels per k_stage1_fix8 chunk for these arguments (0: that kernel does not apply)
int fix8_chunk_channels(const Stage1Multi& a);

struct Stage2Args {
    const void* sub;          // [nsub][sub_stride]
    int32_t sub_dtype, nsub, numdms;
    int32_t nwg;              // pair variant: workgroups along x (0 = one per tile; else persistent, contiguous tile ranges)
    int64_t nds, sub_stride;
    int64_t nvalid;           // min(nds, numout): samples computed
    const int32_t* off;       // [numdms][nsub]
    float* out;               // [numdms][out_stride]
    int64_t out_stride;
    double* partial;          // [numdms][ntiles] per-tile sums (for mean padding) or nullptr
    int32_t ntiles, tile;     // tiles over [0, nvalid) of `tile` samples
    const int32_t* maxabs;    // device int (i16 path) for the packed-accumulation group size
    // LDS-tiled variant
    const int32_t* omin;      // [nyblk][nsub] min offset of the y-block's DMs
    int32_t wstride;          // LDS window stride (elements) per copy
    int32_t dms_per_blk;      // DMs per y-block
    int32_t sc;               // wide variant: subbands per LDS chunk
    int32_t ring_npw, ring_nbp;   // ring variant: 1 KiB DMA pieces per window / per offset block
    int32_t probe;            // profiling only: bit0 skip accumulation, bit1 skip fill, bit2 skip stores
    // pair variant: per (y-block, subband pair) {base0, b1, U, k1[0..U)} (kPairTab ints) and
    // the largest U of the plan (expanded copies per pair = 4*umax)
    const int32_t* ptab;
    int32_t umax;
    int32_t nonneg;           // pair variant: every subband value is >= 0 (unsigned packed halves)
    int32_t qp_setb;          // k_stage2_qp: bytes of one expanded buffer set at the launch's pairs per chunk
    int32_t partial_ndm;      // k_stage2_qp: DMs whose per-tile sums the padding reads (0: all; 1: HD_PAD_DM0)
    uint32_t* stamps;         // k_stage2_qp diagnostics (HD_S2_STAMPS): per-phase shader-clock stamps, or null
};
// k_stage2_qp phase stamps: workgroups x < kStampWG of y 0, each wave's first kStampChunks chunks,
// kStampPh stamps per chunk (iteration start, DMA issued, expand issued, sums done, ring wait
// done; the flush's end in slot 5 of a tile's last chunk)
constexpr int kStampWG = 8, kStampChunks = 32, kStampPh = 6;

hipError_t launch_stage1_direct(const Stage1Args& a, hipStream_t st);
size_t stage1_tiled_lds_bytes(const Stage1Multi& a);
int stage1_special_tiles(const Stage1Multi& a, int* out);
hipError_t launch_stage1_tiled(const Stage1Multi& a, int vw, const int* special, int nspecial, bool special_only,
                               hipStream_t st);
int stage1_q8_quarter_rows(int ds);
bool stage1_q8_supports(int cps, int ds);
size_t stage1_q8_lds_bytes(const Stage1Multi& a);
hipError_t stage1_q8_set_lds_limit(size_t bytes);
hipError_t launch_stage1_q8(const Stage1Multi& a, int vb, hipStream_t st);
bool stage1_tiled_supports_cps(int cps);
// several DDplan stages' passes in one launch (hd_q8m.hip): quarter rows 960, ds | 960
bool stage1_q8m_supports_ds(int ds);
int stage1_q8m_quarter_rows();
size_t stage1_q8m_lds_bytes(const Stage1Multi& a);
hipError_t launch_stage1_q8m(const Stage1Multi& a, hipStream_t st);
hipError_t stage1_tiled_set_lds_limit(size_t bytes);
// wide stage-2 tiles: at most kSC2 subbands staged per chunk, kUMax prefetched fill units
// per thread per chunk, at most kWideWaves waves per workgroup
constexpr int kSC2 = 8;
constexpr int kUMax = 2;
constexpr int kWideWaves = 16;
size_t stage2_wide_lds_bytes(int wstride, int sc);
bool stage2_wide_supports(int q, int r);
bool stage2_ring_supports(int q, int r);
hipError_t launch_stage2_wide(const Stage2Args& a, int q, int r, int nw, hipStream_t st);
size_t stage2_wide2_lds_bytes(int wstride, int sc, int nsub);
constexpr int kRingSC = 4, kRingNS = 5;   // ring variant: subbands per chunk, staging slots
size_t stage2_ring_lds_bytes(int wstride, int npw, int nbp, int nsub);
hipError_t launch_stage2_ring(const Stage2Args& a, int q, int r, hipStream_t st);
constexpr int kPairUMax = 6, kPairTab = 16;   // pair variant: patterns per pair, table ints per pair
// k_stage2_qp pair table: [9] entries per pattern E_k, [kQpPb + 4 - q] the byte offset of the
// pair's patterns inside its chunk's buffer set when a launch takes q pairs per chunk
constexpr int kQpPb = 10;
size_t stage2_pair_lds_bytes(int wstride, int npw, int nbp, int nsub, int umax, int ppc);
bool stage2_pair_supports(int q, int r);
// Per-pass buffers and table geometry of one pass in a pair launch.  One launch may carry up
// to kS2MaxPass passes that share everything else in Stage2Args (nsub, numdms, nvalid, ntiles,
// out_stride, dms_per_blk, nonneg, probe): every pass of a DDplan stage.
struct S2Pass {
    const void* sub;
    const int32_t* ptab;
    const int32_t* off;
    const int32_t* maxabs;
    float* out;
    double* partial;
    int64_t sub_stride;
    int32_t ws, npw, nbp, umax;
    int32_t setb, _pad1;      // k_stage2_qp: bytes of one expanded buffer set (the launch's ppc)
};
constexpr int kS2MaxPass = 28;
struct S2Multi {
    int32_t npass, nyblk;     // nyblk: set by the launcher
    S2Pass p[kS2MaxPass];
};
S2Pass stage2_pass_of(const Stage2Args& a);
hipError_t launch_stage2_pair(const Stage2Args& a, int q, int r, int ppc, hipStream_t st);
// register-window pair kernel (k_stage2_rw): 8 waves x q DMs per workgroup, 768-sample tiles,
// two workgroups per CU; per-chunk table blocks of kRwBlock ints
constexpr int kRwWaves = 8, kRwBlock = 256, kRwTile = 768, kRwMaxWin = 5;
size_t stage2_rw_lds_bytes(int ws, int npw, int nsub, int umax);
hipError_t launch_stage2_rw_multi(const Stage2Args& a, const S2Multi& m, int q, hipStream_t st);
hipError_t launch_stage2_pair_multi(const Stage2Args& a, const S2Multi& m, int q, int r, int ppc, hipStream_t st);
// quarter-layout pair kernel (k_stage2_qp): ws = entries per pattern buffer, ppc 2..4 pairs per chunk
size_t stage2_qp_lds_bytes(int setb, int npw, int nbp, int nsub, int ppc, int ns = 0,
                           bool sync = false);   // ns 0: the default
int stage2_qp_ns(const struct S2Multi& m, int nsub, int ppc);   // staging slots a launch takes
bool stage2_qp_sync(const struct S2Multi& m, int nsub, int ppc);   // the barrier-free variant (A/B)
bool stage2_qp_supports(int q, int r);
hipError_t launch_stage2_qp_multi(const Stage2Args& a, const S2Multi& m, int q, int r, int ppc, hipStream_t st);
hipError_t launch_stage2_wide2(const Stage2Args& a, int q, int r, int nw, hipStream_t st);
hipError_t launch_stage2_direct(const Stage2Args& a, hipStream_t st);
hipError_t launch_stage2_lds(const Stage2Args& a, int q, hipStream_t st);
hipError_t launch_pad(float* out, int64_t out_stride, int numdms, int64_t nds, int64_t numout,
                      const double* partial, int ntiles, int pad_mode, hipStream_t st);
hipError_t launch_series_sum(const float* x, int64_t n, double* part, int nparts, hipStream_t st);
// zero the int32 at each of n (<= kMaxPass) addresses: one launch for a stage-1 call's
// per-plan max|subband| words instead of n memsets
struct ZeroList {
    int32_t* p[kMaxPass];
};
hipError_t launch_zero_list(const ZeroList& z, int n, hipStream_t st);
hipError_t launch_series_fill(float* out, int64_t out_stride, int numdms, int64_t t0, int64_t t1, float v,
                              hipStream_t st);

// ---- PRESTO clip_times on the device (hd_clip.hip) ----
// Scratch of one raw block's clip statistics; device pointers, sized by the host.
struct ClipArgs {
    RawDesc rd;               // rd.clipped / rd.pad are outputs here
    float clip_sigma;
    const uint8_t* allzap;    // [nblk] block fully masked (clip_times skipped), or nullptr
    const float* padvals0;    // [nchan] initial pad values (determine_padvals) or nullptr (0)
    float* zdm;               // [N] zero-DM series (channel-order float fold)
    uint8_t* good;            // [N] within 0.7..1.3 x the block median
    int32_t* numgood;         // [nblk]
    double* bavg;             // [nblk] avg_var mean of the good points
    double* bstd;             // [nblk] sqrt(avg_var variance)
    double* chansum;          // [nblk][nchan] sum of the good spectra per channel
    float* ravg;              // [nblk] running_avg after the block
    float* trig;              // [nblk] clip_sigma * running_std after the block
    int32_t* doclip;          // [nblk] clip_times ran on the block
    uint8_t* clipped;         // [N] out
    uint32_t* clipbits;       // [2 * ceil(N / 64)] out: clipped, bit-packed
    float* pad;               // [nblk][nchan] out: pad values in force for the block
    int32_t* events;          // [N] out: clipped spectra (any order)
    int32_t* nevents;         // device counter
};
int clip_max_block();
hipError_t launch_clip(const ClipArgs& a, hipStream_t st, hipEvent_t after_stats = nullptr);   // = stats + recur + flag
hipError_t launch_clip_stats(const ClipArgs& a, hipStream_t st, hipEvent_t after_stats = nullptr);
hipError_t launch_clip_recur(const ClipArgs& a, hipStream_t st);
hipError_t launch_clip_flag(const ClipArgs& a, hipStream_t st);
// time-sliced contexts: rows [bavg, bstd, numgood, chansum[nchan]] of the first nown blocks
// out; a global block range in (g.rd.nblk rows into g's arrays)
hipError_t launch_clip_pack(const ClipArgs& a, double* out, int nown, hipStream_t st);
hipError_t launch_clip_unpack(const ClipArgs& g, const double* in, hipStream_t st);
// Exact recomputation of the stage-1 outputs a clipped spectrum (events) or a read-block
// boundary with changing pad values (the 8-bit integer path's straddling outputs) touches.
hipError_t launch_stage1_fixup(const Stage1Multi& a, const int32_t* events, const int32_t* nevents,
                               int boundaries, hipStream_t st);
// single-pulse search (hd_sp.hip): per-block detrend/std + per-DM bad blocks -> coef
// [ndm][nblocks][4] (mean, slope, std, bad); boxcar hits above threshold
int sp_max_blocks();
hipError_t launch_sp_badflags(const double* coef, int64_t n, uint8_t* bad, hipStream_t st);
hipError_t launch_sp_blocks(const float* x, int64_t stride, int ndm, int nblocks, double* coef, hipStream_t st);
hipError_t launch_sp_hits(const float* x, int64_t stride, int ndm, int nblocks, const double* coef, int64_t ls,
                          const int32_t* widths, const double* rsw, int nwidths, double threshold, hd_sp_hit* hits,
                          unsigned long long* count, int64_t cap, hipStream_t st);
// rfifind statistics (hd_rfi.hip): per interval and channel mean, std, max normalised power
hipError_t set_max_lds(const void* fn, int bytes);
// barycentric output: padding values (as k_pad) then the segments {out0, src0 | -1, len}
hipError_t launch_bary(const float* topo, float* out, int64_t stride, int numdms, int64_t numout, const int32_t* seg,
                       int nseg, const double* partial, int ntiles, int64_t nds, int pad_mode, float* padv,
                       hipStream_t st);
hipError_t rfi_stats(const RawDesc& rd, const uint8_t* rawT, int64_t tstride, int ptsperint, int numint, float* avg,
                     float* sd, float* pw, hipStream_t st);
// realfft / zapbirds / rednoise of a plan's series (hd_fft.hip)
struct FftState;
FftState* fft_state_new();
void fft_state_free(FftState* s);
hipError_t fft_begin(FftState* s, hipStream_t st);
hipError_t fft_end(FftState* s, hipStream_t st);
float2* fft_buffer(FftState* s);
const void* fft_owner(const FftState* s);
void fft_set_owner(FftState* s, const void* owner);
hipError_t fft_prepare(FftState* s, int64_t xstride, int64_t n, int ndm);
hipError_t fft_series(FftState* s, const float* x, int64_t xstride, int64_t n, int ndm, hipStream_t st);
hipError_t fft_zap(FftState* s, const int32_t* rng4, int nr, hipStream_t st);
hipError_t fft_rednoise(FftState* s, const int32_t* boff, const double* cen, int nblk, hipStream_t st);
constexpr int64_t kRawTPad = 65536;   // zero rows after N in each channel-major raw row
hipError_t launch_raw_transpose(const uint8_t* raw, int64_t N, int32_t nchan, int nbits, int nibble_hi_first,
                                uint8_t* rawT, int64_t tstride, hipStream_t st);
hipError_t launch_synth(uint8_t* raw, int64_t N, int32_t rowbytes, const hd_synth_tab* tab_dev, int64_t t0,
                        hipStream_t st);

}  // namespace hd
