// hd_api.hip — C ABI of libhipdedisp.so (declared in include/hipdedisp.h).
//
// Host side of the engine: observation/mask/calibration state, integer delay tables
// (double precision, PRESTO NEAREST_LONG), device buffers, launch sequencing and
// hipEvent timing.  One context = one device + one stream; plans are per DDplan pass.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <map>
#include <memory>
#include <tuple>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "hd_internal.h"
#include "hd_io.h"
#include "../../include/hipdedisp.h"

#define HD_VERSION_STR "hipdedisp 0.1.0 (gfx950)"

// Pinned host blocks of the file ingest: kReaders reader threads x 2 blocks, each guarded by
// the event of the last copy that read it.
constexpr int kReaders = 4;
struct PinSet {
    void* pin[2 * kReaders] = {};
    hipEvent_t ev[2 * kReaders] = {};
    size_t bytes = 0;
    void release()
    {
        for (int b = 0; b < 2 * kReaders; b++) {
            if (ev[b]) (void)hipEventSynchronize(ev[b]);
            if (pin[b]) (void)hipHostFree(pin[b]);
            if (ev[b]) (void)hipEventDestroy(ev[b]);
            pin[b] = nullptr;
            ev[b] = nullptr;
        }
        bytes = 0;
    }
};

struct hd_ctx {
    int device = -1;                   // HD_HOST_ONLY (-1): no device (life-cycle tests)
    int ncu = 256;                     // compute units (persistent stage-2 workgroups)
    // a sticky HIP error (device fault) was seen: the device is unusable for the rest of the
    // process, so teardown makes no device call (hd_close, hd_plan_destroy)
    bool faulted = false;
    std::string fault_msg;
    hipStream_t stream = nullptr;
    std::string err;
    bool have_obs = false;
    hd_obs obs{};
    hd_opts opts{};
    int32_t rowbytes = 0;
    uint8_t* d_raw = nullptr;
    bool raw_ready = false;
    uint8_t* d_rawT = nullptr;         // channel-major copy for the 8-bit stage-1 fill (lazy)
    int64_t rawT_stride = 0;
    bool rawT_valid = false;           // false whenever the raw block changes
    float *d_scl = nullptr, *d_offs = nullptr, *d_wts = nullptr;
    // rfifind mask as given (hd_set_mask) and the initial pad values
    std::vector<uint8_t> h_mask, h_zapint;  // [numint][nchan], [numint]
    int32_t numint = 0, ptsperint = 0;
    double dtint = 0.0;
    float* d_padvals = nullptr;
    std::vector<float> h_padvals;      // host copy (bounds for the integer stage-1 path)
    // per read block (obs.nsblk spectra): check_mask rows, deduplicated (zidx -> zrows)
    int32_t blk = 1, nblk = 1;
    bool blocks_valid = false;
    std::vector<int32_t> h_zidx;       // host copies of zidx / zrows (the fixup's boundary lists)
    std::vector<uint8_t> h_zrows;
    std::map<int, std::pair<int32_t*, int32_t*>> fixb;   // per fixup chunk width G: device {list, offsets}
    int32_t* d_zidx = nullptr;
    uint8_t* d_zrows = nullptr;
    uint8_t* d_allzap = nullptr;
    // clip_times state of the current raw block (hd_clip.hip), rebuilt when the raw block,
    // mask, pad values or calibration change
    bool clip_valid = false;
    struct ClipBufs {
        float* zdm = nullptr;
        uint8_t *good = nullptr, *clipped = nullptr;
        uint32_t* clipbits = nullptr;       // clipped, bit-packed (k_stage1_q8's in-kernel fixup)
        int32_t *numgood = nullptr, *doclip = nullptr, *events = nullptr, *nevents = nullptr;
        int32_t* nzero = nullptr;           // a device 0 (profiling: a fixup over no clipped spectra)
        double *bavg = nullptr, *bstd = nullptr, *chansum = nullptr;
        float *ravg = nullptr, *trig = nullptr, *pad = nullptr;
        // time-sliced context: the recurrence runs over the observation's blocks [0, g0 + nblk)
        // from exchanged statistics (hd_clip_set_stats) into these global arrays
        bool stats_valid = false;           // this slice's per-block statistics are computed
        int32_t *numgood_g = nullptr, *doclip_g = nullptr;
        double *bavg_g = nullptr, *bstd_g = nullptr, *chansum_g = nullptr, *xbuf = nullptr;
        float *ravg_g = nullptr, *trig_g = nullptr, *pad_g = nullptr;
        uint8_t* allzap_g = nullptr;
    } clip;
    // time slice (hd_set_slice): the context holds spectra [slice_t0, slice_t0 + obs.N) of an
    // observation of slice_total spectra (0: the whole observation)
    int64_t slice_t0 = 0, slice_total = 0;
    size_t lds_attr_set = 64 * 1024;   // dynamic-LDS limit already granted to the tiled kernels
    size_t lds_attr_q8 = 64 * 1024;    // ... and to the 8-bit integer stage-1 kernels
    struct SpecialList {               // stage-1 special-tile list per tile geometry (device)
        int to, ds, dmax, ntiles, two_ok, n;
        int* d;
    };
    std::vector<SpecialList> special_cache;
    double* d_partial = nullptr;    // shared per-tile partial sums
    size_t partial_bytes = 0;
    // single-pulse search: the host half's copy stream, pinned staging of the hits / flags
    // D2H, and the largest device hit count seen (the next plans' first list size)
    // in-library collectives (hd_comm_*): an RCCL communicator, its rank / size, a device
    // scratch for host buffers and the slice clip-statistics table
    void* comm = nullptr;
    int32_t comm_rank = 0, comm_world = 0;
    double* d_comm = nullptr;
    size_t comm_bytes = 0;
    hipStream_t ssp = nullptr;
    std::vector<struct SpBufs*> sp_free, sp_all;   // search buffer sets (free / every one made)
    void* sp_pin = nullptr;
    size_t sp_pin_bytes = 0;
    int64_t sp_cap_hint = 1 << 16;
    double* d_sum_parts = nullptr;  // hd_series_sum partials
    double* d_sum_parts_multi = nullptr;   // hd_series_sum_multi partials [n][512]
    size_t sum_parts_bytes = 0;
    // streaming ingest (hd_push_raw_file): pinned host blocks of the reader threads
    PinSet pins;
    // stage 2 alternates between the main stream and stream2, so one pass's last tiles and
    // the next pass's first ones share the GPU (no tail between launches).  ev_fork orders
    // stream2 after the main stream's work so far; ev_join (after each stream2 pass) orders
    // main-stream work that rewrites subbands after it; each stream has its own partials.
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // the channel-major raw copy runs on saux beside clip_times' latency-bound kernels
    // (AS-52 per block, the serial 30-block recurrence): ev_aux0 orders it after the main
    // stream's work so far, stage 1 waits for ev_aux1
    hipStream_t saux = nullptr;
    hipEvent_t ev_aux0 = nullptr, ev_aux1 = nullptr;
    bool aux_pending = false;
    bool s2_pending = false;
    bool dual = false;              // hd_set_streams(ctx, 2 or 3)
    bool s2all = false;             // hd_set_streams(ctx, 3): every stage-2 pass on stream2
    uint32_t dd_count = 0;
    double* d_partial2 = nullptr;
    size_t partial_bytes2 = 0;
    hd::Writer* writer = nullptr;   // .dat output path (hd_io.hip), opened on first use
    // realfft state per series geometry (numout, numdms, stride): hipFFT plan + spectra
    // buffer, shared by the plans of that geometry -- each pass's hd_realfft takes it over
    // (the owner), so a beam builds 6 hipFFT plans, not 57
    std::map<std::tuple<int64_t, int, int64_t>, hd::FftState*> fft_cache;
    // overlapped ingest of the next beam (hd_prefetch_*, hd_swap_raw): a second raw slot filled
    // by a reader thread through its own pinned blocks on its own copy stream
    struct Prefetch;
    Prefetch* pf = nullptr;
    // diagnostics (HD_S2_STAMPS=<file>): k_stage2_qp phase stamps of the last launch, written
    // to the file by hd_sync
    uint32_t* d_stamps = nullptr;
    bool stamps_pending = false;
};

struct PfJob {
    bool fill = false;
    std::string path;
    hd_rows_src src{};
    int64_t start = 0, sb = 0, soff = 0, doff = 0, nb = 0, count = 0;
    int32_t byte_value = 0;
};

struct hd_ctx::Prefetch {
    uint8_t* d_next = nullptr;       // the idle raw slot
    hipStream_t st = nullptr;        // copy stream
    hipEvent_t ev_free = nullptr;    // recorded at a swap: the work queued on the old block
    hipEvent_t ev_done = nullptr;    // recorded at a swap: the prefetch copies
    bool wait_free = false;          // the next queued job first waits for ev_free
    PinSet pins;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<PfJob> q;
    bool busy = false, stop = false, any = false;
    int err = 0;
    std::string errmsg;
    double io = 0.0, t0 = 0.0;       // pread seconds, steady-clock seconds of the first job
};

// main-stream work from here on runs after every stage-2 pass queued on stream2
static hipError_t join_stream2(hd_ctx* c)
{
    if (!c->s2_pending) return hipSuccess;
    c->s2_pending = false;
    return hipStreamWaitEvent(c->stream, c->ev_join, 0);
}

static hipError_t sync_all(hd_ctx* c)
{
    hipError_t e = hipStreamSynchronize(c->stream);
    for (hipStream_t o : {c->stream2, c->saux})
        if (o) {
            const hipError_t e2 = hipStreamSynchronize(o);
            if (e == hipSuccess) e = e2;
        }
    c->s2_pending = false;
    c->aux_pending = false;
    return e;
}

// The start / end events of a stage-2 launch.  A multi-pass launch (hd_run_dedisp_multi)
// records one pair for all the passes it carries, and every plan's dd_cur points at it: one
// event per plan after the launch had cost the command processor ~5 us each, ~0.3 ms of idle
// GPU after a 28-pass stage.  Shared ownership keeps a pair valid while any plan refers to it;
// a later record into it by its owner only moves the end later (a conservative wait).
struct DdEv {
    hipEvent_t e[2] = {nullptr, nullptr};
    ~DdEv()
    {
        for (hipEvent_t x : e)
            if (x) (void)hipEventDestroy(x);
    }
};

struct hd_plan {
    hd_ctx* ctx = nullptr;
    hd_pass pass{};
    char s2name[64] = {0};          // stage-2 kernel of the last hd_run_dedisp (hd_plan_kernel)
    int32_t s2passes = 1;           // passes the last stage-2 launch this plan led carried (0: it
                                    // ran inside another plan's launch, hd_run_dedisp_multi)
    int64_t nds = 0, numout = 0, nvalid = 0;
    int64_t sub_stride = 0, out_stride = 0;
    double sub_lofreq = 0, sub_chanwid = 0, sub_dt = 0;
    std::vector<int32_t> idispdt, off;
    int32_t maxdelay = 0;
    int32_t* d_idispdt = nullptr;
    int32_t* d_off = nullptr;
    int32_t* d_maxabs = nullptr;
    // LDS-variant tables
    int32_t q = 0, dpb = 0, nyblk = 0, wstride = 0;
    bool lds_ok = false;
    int32_t* d_omin = nullptr;
    int32_t* d_boff = nullptr;
    // wide-tile variant tables: [0] k_stage2_wide (16 waves, double-buffered), [1] k_stage2_wide2
    // (8 waves, two workgroups per CU)
    struct Wide {
        bool ok = false;
        int32_t q = 0, r = 0, nw = 0, dpb = 0, ws = 0, sc = 0, npw = 0, nbp = 0;
        int32_t umax = 0;               // [3] only: largest pattern count of a subband pair
        int32_t setb[3] = {0, 0, 0};    // [6]: bytes of one expanded buffer set at 4, 3, 2 pairs per chunk
        int32_t* d_omin = nullptr;      // [3]: the pair table (kPairTab ints per y-block and pair)
        int32_t* d_boff = nullptr;
        int32_t* d_boffp[3] = {nullptr, nullptr, nullptr};   // [6]: the offsets for 4, 3, 2 pairs per chunk
    } wide[7];                      // [2]: k_stage2_ring (16 waves, LDS-DMA staging ring);
                                    // [3]: k_stage2_pair (the ring over subband-pair partials),
                                    // [4]: the same with two pairs per chunk (half the chunks),
                                    // [5]: k_stage2_rw (register windows, one copy, 2 WGs per CU),
                                    // [6]: k_stage2_qp (quarter-layout pair partials; sc = pairs per chunk)
    bool sub_nonneg = false;        // every subband value >= 0 (known on the host with sub_bound)
    int32_t sub_bound = -1;         // bound on |subband| known on the host (-1: none), set when
                                    // the subbands are formed or uploaded (pair variant gate)
    int32_t variant = 0;
    float* d_out = nullptr;
    void* d_sub = nullptr;          // this pass's subbands [nsub][sub_stride]
    size_t sub_bytes = 0;
    bool sub_valid = false;
    int32_t s1_variant = 0;         // stage 1: 0 auto, 1 direct, 2 float tiled, 3 8-bit integer
    int32_t probe = 0;              // profiling switches (hd_plan_set_variant bits 16-23)
    int32_t pair_persist = 0;       // hd_plan_set_variant bits 24-25 (pair kernel tile scheduling)
    hipEvent_t ev[2] = {nullptr, nullptr};   // stage 1: start, end (recorded by the call's first plan)
    std::shared_ptr<DdEv> dd_own, dd_cur;    // stage 2: this plan's pair; the pair ending its last stage 2
    hipEvent_t ev_copy = nullptr;   // after the writer's copies of this plan's series
    bool copy_pending = false;
    bool ran_sub = false, ran_dd = false;
    hipStream_t dd_stream = nullptr;  // stream of the last hd_run_dedisp (dd_end() marks the end)
    hd::FftState* fft = nullptr;    // realfft state (hd_fft.hip, from hd_ctx::fft_cache)
    bool ran_fft = false;
    // barycentric output (hd_plan_set_bary): stage 2 writes the topocentric series to d_topo,
    // then k_bary copies its segments to d_out; d_bseg [nbseg][3] = {out0, src0 (-1: padding),
    // len}; d_padv [numdms] the padding values
    int32_t nbseg = 0;
    bool bary_adds = false;         // some bin is added (the padding value is needed)
    int64_t data_end = -1;          // samples of real data in the output (-1: nvalid; barycentred:
                                    // the end of the last data segment, PRESTO's datawrote)
    std::vector<int32_t> bary_diff; // the diffbins the segments were built from
    int32_t* d_bseg = nullptr;
    float* d_topo = nullptr;
    float* d_padv = nullptr;
    struct SpPlan* sp = nullptr;    // single-pulse search state (hd_single_pulse_launch / _collect)
};

static hipEvent_t dd_start(const hd_plan* p) { return p->dd_cur ? p->dd_cur->e[0] : nullptr; }
static hipEvent_t dd_end(const hd_plan* p) { return p->dd_cur ? p->dd_cur->e[1] : nullptr; }

// Device buffers of one single-pulse search in flight (block coefficients, hit list, hit
// count, bad flags) and the event after its device half: a context pool, taken by a launch
// and given back by its collect, so a pipeline of k searches allocates k sets once.
struct SpBufs {
    double* d_coef = nullptr;
    size_t coef_bytes = 0;
    hd_sp_hit* d_hits = nullptr;
    int64_t cap = 0;
    unsigned long long* d_count = nullptr;
    uint8_t* d_bad = nullptr;
    size_t bad_bytes = 0;
    hipEvent_t ev = nullptr;
};

// A plan's single-pulse search in flight: the device half (block statistics, boxcar hits,
// prune_related1, bad flags) launched on the plan's stream and marked by b->ev; the host half
// (copies, prune_related2, border cases) waits for that event only, on the context's ssp
// stream, so the device half of later plans keeps running while this plan's hits are pruned.
struct SpPlan {
    SpBufs* b = nullptr;
    hipStream_t st = nullptr;
    bool pending = false;
    int32_t widths[16] = {0};
    double rsw[16] = {0};
    int32_t nw = 0;
    double threshold = 0;
    int64_t nblocks = 0, ls = 0;
};

static thread_local std::string g_err;
extern "C" int hd_comm_destroy(hd_ctx* c);
static void clear_special_cache(hd_ctx* c);
static void sp_bufs_free(SpBufs* b);

static int fail(hd_ctx* ctx, int code, const char* fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    g_err = buf;
    return code;
}

// HIP errors after which the device context is unusable (a kernel faulted): later runtime
// calls return them again, and some teardown calls on such a device abort the process.
static bool hip_sticky(hipError_t e)
{
    switch (e) {
    case hipErrorIllegalAddress:
    case hipErrorLaunchFailure:
    case hipErrorAssert:
    case hipErrorLaunchTimeOut:
    case hipErrorECCNotCorrectable:
        return true;
    default:
        return false;
    }
}

static void note_hip_error(hd_ctx* c, hipError_t e, const char* what)
{
    if (c && hip_sticky(e) && !c->faulted) {
        c->faulted = true;
        c->fault_msg = std::string(what) + ": " + hipGetErrorString(e);
    }
}

#define HIPCHK(ctx, expr)                                                                          \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            note_hip_error((ctx), e_, #expr);                                                      \
            return fail((ctx), HD_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),    \
                        __FILE__, __LINE__);                                                       \
        }                                                                                          \
    } while (0)

static void dfree(void* p)
{
    if (p) (void)hipFree(p);
}

// ---------------------------------------------------------------------------------------
// delay tables (PRESTO src/dispersion.c semantics; the oracle restates the same rules)
// ---------------------------------------------------------------------------------------
static double delay_from_dm(double dm, double f) { return dm / (0.000241 * f * f); }
static double doppler(double f, double v) { return f * (1.0 + v); }
static int64_t nearest_long(double x) { return (int64_t)(x < 0 ? ceil(x - 0.5) : floor(x + 0.5)); }

static void dedisp_delays(int n, double dm, double lof, double cw, double v, double* out)
{
    for (int i = 0; i < n; i++) out[i] = delay_from_dm(dm, doppler(lof + i * cw, v));
}
static void subband_delays(int nchan, int nsub, double dm, double lof, double cw, double v, double* out)
{
    const int cps = nchan / nsub;
    const double sbw = cw * cps;
    const double losubhi = lof + sbw - cw;
    dedisp_delays(nsub, dm, losubhi, sbw, v, out);
}

static double text_roundtrip(double v, const char* fmt)
{
    char buf[64];
    snprintf(buf, sizeof buf, fmt, v);
    return strtod(buf, nullptr);
}

static size_t round_up(size_t x, size_t m) { return (x + m - 1) / m * m; }

// ---------------------------------------------------------------------------------------
// library / context
// ---------------------------------------------------------------------------------------
extern "C" const char* hd_version(void) { return HD_VERSION_STR; }

extern "C" void hd_opts_default(hd_opts* o)
{
    if (!o) return;
    memset(o, 0, sizeof *o);
    o->sub_dtype = HD_SUB_I16;
    o->ds_mode = HD_DS_MEAN;
    o->pad_mode = HD_PAD_DM0;
    o->nibble_hi_first = 1;
    o->be16 = 1;
    o->inf_roundtrip = 1;
    o->clip_sigma = 6.0f;
    o->sub_round = HD_ROUND_PRESTO;
}

extern "C" int hd_device_count(int* n)
{
    if (!n) return fail(nullptr, HD_E_INVAL, "hd_device_count: n is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = (e == hipSuccess) ? c : 0;
    return HD_OK;
}

extern "C" int hd_open(int device, hd_ctx** out)
{
    if (!out) return fail(nullptr, HD_E_INVAL, "hd_open: out is NULL");
    *out = nullptr;
    if (device == HD_HOST_ONLY) {      // no device: streams, events and buffers stay NULL
        *out = new hd_ctx();
        return HD_OK;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(nullptr, HD_E_NODEV, "hd_open: no HIP device available");
    if (device < 0 || device >= n)
        return fail(nullptr, HD_E_NODEV, "hd_open: device %d out of range (have %d)", device, n);
    hd_ctx* c = new hd_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->saux, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_aux0, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_aux1, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return fail(nullptr, HD_E_HIP, "hd_open: cannot initialise device %d", device);
    }
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0) c->ncu = ncu;
    *out = c;
    return HD_OK;
}

static void free_blocks(hd_ctx* c)
{
    for (auto& kv : c->fixb) {
        dfree(kv.second.first);
        dfree(kv.second.second);
    }
    c->fixb.clear();
    c->h_zidx.clear();
    c->h_zrows.clear();
    dfree(c->d_zidx); c->d_zidx = nullptr;
    dfree(c->d_zrows); c->d_zrows = nullptr;
    dfree(c->d_allzap); c->d_allzap = nullptr;
    c->blocks_valid = false;
    c->clip_valid = false;
    c->clip.stats_valid = false;
}

static void free_clip(hd_ctx* c)
{
    hd_ctx::ClipBufs& b = c->clip;
    for (void* p : {(void*)b.zdm, (void*)b.good, (void*)b.clipped, (void*)b.clipbits, (void*)b.numgood, (void*)b.doclip,
                    (void*)b.events, (void*)b.nevents, (void*)b.nzero, (void*)b.bavg, (void*)b.bstd, (void*)b.chansum,
                    (void*)b.ravg, (void*)b.trig, (void*)b.pad, (void*)b.numgood_g, (void*)b.doclip_g,
                    (void*)b.bavg_g, (void*)b.bstd_g, (void*)b.chansum_g, (void*)b.xbuf, (void*)b.ravg_g,
                    (void*)b.trig_g, (void*)b.pad_g, (void*)b.allzap_g})
        dfree(p);
    b = hd_ctx::ClipBufs{};
    c->clip_valid = false;
    c->clip.stats_valid = false;
}

static void pf_stop(hd_ctx* c);
static void pf_abandon(hd_ctx* c);

static void free_obs_buffers(hd_ctx* c)
{
    pf_stop(c);                        // the prefetched block has the old geometry
    dfree(c->d_raw); c->d_raw = nullptr;
    dfree(c->d_rawT); c->d_rawT = nullptr;
    c->rawT_valid = false;
    dfree(c->d_scl); c->d_scl = nullptr;
    dfree(c->d_offs); c->d_offs = nullptr;
    dfree(c->d_wts); c->d_wts = nullptr;
    dfree(c->d_padvals); c->d_padvals = nullptr;
    c->h_padvals.clear();
    c->h_mask.clear();
    c->h_zapint.clear();
    free_blocks(c);
    free_clip(c);
    clear_special_cache(c);
    c->raw_ready = false;
    c->numint = c->ptsperint = 0;
    c->dtint = 0.0;
}

// Teardown of a context whose device faulted (or that never had one): host threads and
// host memory only.  Device buffers, streams, events, pinned blocks and hipFFT plans are
// left to the process exit -- the runtime's own teardown calls on a faulted device are what
// aborted the process in round 5 (hd_close after an illegal memory access).
static int close_without_device(hd_ctx* c)
{
    const bool had = c->faulted;
    const std::string msg = c->fault_msg;
    if (c->writer) {
        hd::writer_abandon(c->writer);
        c->writer = nullptr;
    }
    if (c->pf) pf_abandon(c);
    for (SpBufs* b : c->sp_all) delete b;
    c->sp_all.clear();
    c->sp_free.clear();
    c->special_cache.clear();
    c->fft_cache.clear();
    delete c;
    if (!had) return HD_OK;
    return fail(nullptr, HD_E_HIP, "hd_close: the device faulted earlier (%s); device memory is left to the process exit",
                msg.c_str());
}

extern "C" int hd_close(hd_ctx* c)
{
    if (!c) return HD_OK;
    if (c->device == HD_HOST_ONLY || c->faulted) return close_without_device(c);
    (void)hipSetDevice(c->device);
    {
        const hipError_t e = sync_all(c);
        note_hip_error(c, e, "hd_close: stream synchronize");
        if (c->faulted) return close_without_device(c);
    }
    if (c->writer) {
        std::string e;
        (void)hd::writer_wait(c->writer, e, nullptr, nullptr);
        hd::writer_close(c->writer);
        c->writer = nullptr;
    }
    free_obs_buffers(c);
    dfree(c->d_partial);
    dfree(c->d_partial2);
    (void)hd_comm_destroy(c);
    if (c->sp_pin) (void)hipHostFree(c->sp_pin);
    for (SpBufs* b : c->sp_all) sp_bufs_free(b);
    c->sp_all.clear();
    c->sp_free.clear();
    if (c->ssp) (void)hipStreamDestroy(c->ssp);
    dfree(c->d_sum_parts);
    dfree(c->d_sum_parts_multi);
    dfree(c->d_stamps);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_aux0) (void)hipEventDestroy(c->ev_aux0);
    if (c->ev_aux1) (void)hipEventDestroy(c->ev_aux1);
    if (c->saux) (void)hipStreamDestroy(c->saux);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    c->pins.release();
    clear_special_cache(c);
    for (auto& kv : c->fft_cache) hd::fft_state_free(kv.second);
    c->fft_cache.clear();
    (void)hipStreamDestroy(c->stream);
    delete c;
    return HD_OK;
}

extern "C" int hd_debug_fault(hd_ctx* c)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_debug_fault: NULL context");
    c->faulted = true;
    c->fault_msg = "hd_debug_fault";
    return HD_OK;
}

extern "C" int hd_set_streams(hd_ctx* c, int32_t n)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_set_streams: NULL context");
    if (n < 1 || n > 3) return fail(c, HD_E_INVAL, "hd_set_streams: n must be 1, 2 or 3");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, sync_all(c));
    c->dual = n >= 2;
    c->s2all = n == 3;
    c->dd_count = 0;
    return HD_OK;
}

extern "C" int hd_touch_raw(hd_ctx* c)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_touch_raw: NULL context");
    c->rawT_valid = false;
    c->clip_valid = false;
    c->clip.stats_valid = false;
    return HD_OK;
}

// Channel-major one-byte-per-sample copy of the 8- or 4-bit raw block for k_stage1_q8's and
// k_stage1_fix8's fills, rebuilt on the stream (and charged to the stage-1 launch that needs
// it) once per raw block.  nullptr when it does not apply (8-bit data then fills from the
// row-major block; 4-bit data takes the float tiled kernel).
static bool alloc_rawT(hd_ctx* c, int dmax)
{
    const int nb = c->obs.nbits;
    if ((nb != 8 && nb != 4) || c->obs.nchan % (nb == 4 ? 8 : 4) || c->obs.N % 4 || (int64_t)dmax + 8 > hd::kRawTPad)
        return false;
    if (!c->d_rawT) {
        const int64_t stride = (int64_t)round_up((size_t)(c->obs.N + hd::kRawTPad), 256);
        const size_t bytes = (size_t)stride * c->obs.nchan;
        if (hipMalloc(&c->d_rawT, bytes) != hipSuccess) {
            c->d_rawT = nullptr;
            (void)hipGetLastError();
            return false;                // no room: row-major fill
        }
        if (hipMemsetAsync(c->d_rawT, 0, bytes, c->stream) != hipSuccess) {
            dfree(c->d_rawT);
            c->d_rawT = nullptr;
            return false;
        }
        c->rawT_stride = stride;
        c->rawT_valid = false;
    }
    return true;
}

static const uint8_t* ensure_rawT(hd_ctx* c, int dmax, bool aux = false, bool forked = false)
{
    if (!alloc_rawT(c, dmax)) return nullptr;
    const int nb = c->obs.nbits;
    if (!c->rawT_valid) {
        hipStream_t st = c->stream;
        if (aux) {
            // on saux after ev_aux0: recorded here (the main stream's work so far) or, when
            // forked, by clip_times after its full-chip statistics kernels
            if (!forked && hipEventRecord(c->ev_aux0, c->stream) != hipSuccess) return nullptr;
            if (hipStreamWaitEvent(c->saux, c->ev_aux0, 0) != hipSuccess) return nullptr;
            st = c->saux;
        }
        if (hd::launch_raw_transpose(c->d_raw, c->obs.N, c->obs.nchan, nb, c->opts.nibble_hi_first, c->d_rawT,
                                     c->rawT_stride, st) != hipSuccess)
            return nullptr;
        if (aux) {
            if (hipEventRecord(c->ev_aux1, c->saux) != hipSuccess) return nullptr;
            c->aux_pending = true;
        }
        c->rawT_valid = true;
    }
    return c->d_rawT;
}

// the main stream waits for a channel-major copy still running on saux
static hipError_t join_aux(hd_ctx* c)
{
    if (!c->aux_pending) return hipSuccess;
    c->aux_pending = false;
    return hipStreamWaitEvent(c->stream, c->ev_aux1, 0);
}

extern "C" const char* hd_last_error(const hd_ctx* c) { return c ? c->err.c_str() : g_err.c_str(); }

static size_t stamps_bytes() { return (size_t)hd::kStampWG * 16 * hd::kStampChunks * hd::kStampPh * 4; }

// k_stage2_qp phase stamps (diagnostics): the device buffer when HD_S2_STAMPS names a file
static uint32_t* stamps_buf(hd_ctx* c)
{
    const char* path = getenv("HD_S2_STAMPS");
    if (!path || !*path) return nullptr;
    if (!c->d_stamps && hipMalloc(&c->d_stamps, stamps_bytes()) != hipSuccess) c->d_stamps = nullptr;
    if (c->d_stamps) c->stamps_pending = true;
    return c->d_stamps;
}

extern "C" int hd_sync(hd_ctx* c)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_sync: NULL context");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, sync_all(c));
    if (c->stamps_pending) {
        c->stamps_pending = false;
        std::vector<uint32_t> h(stamps_bytes() / 4);
        HIPCHK(c, hipMemcpy(h.data(), c->d_stamps, stamps_bytes(), hipMemcpyDeviceToHost));
        if (FILE* f = fopen(getenv("HD_S2_STAMPS"), "wb")) {
            (void)fwrite(h.data(), 4, h.size(), f);
            fclose(f);
        }
    }
    return HD_OK;
}

static int check_obs(hd_ctx* c, const hd_obs* o)
{
    if (!o) return fail(c, HD_E_INVAL, "obs is NULL");
    if (o->nchan <= 0) return fail(c, HD_E_INVAL, "nchan must be > 0 (got %d)", o->nchan);
    if (o->nbits != 4 && o->nbits != 8 && o->nbits != 16)
        return fail(c, HD_E_INVAL, "nbits must be 4, 8 or 16 (got %d)", o->nbits);
    if (o->npol != 1) return fail(c, HD_E_INVAL, "only npol == 1 (summed polarisations) is supported (got %d)", o->npol);
    if (((int64_t)o->nchan * o->nbits) % 8) return fail(c, HD_E_INVAL, "nchan*nbits must be a whole number of bytes");
    if (o->N <= 0) return fail(c, HD_E_INVAL, "N must be > 0");
    if (!(o->dt > 0) || !(o->df > 0) || !(o->lofreq > 0))
        return fail(c, HD_E_INVAL, "dt, df and lofreq must be > 0");
    return HD_OK;
}

extern "C" int hd_set_obs(hd_ctx* c, const hd_obs* o, const hd_opts* opts)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_set_obs: NULL context");
    int rc = check_obs(c, o);
    if (rc) return rc;
    hd_opts op;
    if (opts) op = *opts; else hd_opts_default(&op);
    if (op.sub_dtype != HD_SUB_I16 && op.sub_dtype != HD_SUB_F32) return fail(c, HD_E_INVAL, "bad sub_dtype");
    if (op.ds_mode != HD_DS_SUM && op.ds_mode != HD_DS_MEAN) return fail(c, HD_E_INVAL, "bad ds_mode");
    if (op.pad_mode != HD_PAD_MEAN && op.pad_mode != HD_PAD_ZERO && op.pad_mode != HD_PAD_DM0)
        return fail(c, HD_E_INVAL, "bad pad_mode");
    if (op.sub_round != HD_ROUND_PRESTO && op.sub_round != HD_ROUND_NEAREST) return fail(c, HD_E_INVAL, "bad sub_round");
    if (!(op.clip_sigma >= 0.0f) || !std::isfinite(op.clip_sigma))
        return fail(c, HD_E_INVAL, "clip_sigma must be finite and >= 0 (0 = -noclip)");
    if (op.clip_sigma > 0.0f && o->nsblk > hd::clip_max_block())
        return fail(c, HD_E_INVAL, "clipping needs nsblk <= %d (got %d)", hd::clip_max_block(), o->nsblk);
    if (c->device != HD_HOST_ONLY) {
        HIPCHK(c, hipSetDevice(c->device));
        HIPCHK(c, sync_all(c));
        free_obs_buffers(c);
    }
    c->obs = *o;
    c->opts = op;
    c->rowbytes = (int32_t)((int64_t)o->nchan * o->nbits / 8);
    c->blk = (int32_t)std::min<int64_t>(o->nsblk > 0 ? o->nsblk : o->N, o->N);
    c->nblk = (int32_t)((o->N + c->blk - 1) / c->blk);
    c->slice_t0 = c->slice_total = 0;
    c->have_obs = true;
    return HD_OK;
}

extern "C" int hd_set_slice(hd_ctx* c, int64_t t0, int64_t n_total)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_set_slice: NULL context");
    if (!c->have_obs) return fail(c, HD_E_STATE, "hd_set_slice before hd_set_obs");
    if (n_total == 0 && t0 == 0) {
        c->slice_t0 = c->slice_total = 0;
    } else {
        const int64_t blk = c->obs.nsblk > 0 ? c->obs.nsblk : 0;
        if (blk <= 0 || t0 < 0 || t0 % blk || t0 + c->obs.N > n_total)
            return fail(c, HD_E_INVAL, "hd_set_slice: need 0 <= t0, t0 %% nsblk == 0 and t0 + N <= n_total "
                        "(t0 %lld, N %lld, n_total %lld, nsblk %lld)", (long long)t0, (long long)c->obs.N,
                        (long long)n_total, (long long)blk);
        if (c->blk != blk) return fail(c, HD_E_INVAL, "hd_set_slice: the slice is shorter than one read block");
        c->slice_t0 = t0;
        c->slice_total = n_total;
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, sync_all(c));
    free_blocks(c);
    free_clip(c);
    clear_special_cache(c);
    return HD_OK;
}

static int ensure_raw(hd_ctx* c)
{
    if (c->d_raw) return HD_OK;
    const size_t bytes = (size_t)c->obs.N * c->rowbytes;
    if (hipMalloc(&c->d_raw, bytes) != hipSuccess) {
        c->d_raw = nullptr;
        return fail(c, HD_E_NOMEM, "cannot allocate %zu bytes of raw data", bytes);
    }
    return HD_OK;
}

static int upload(hd_ctx* c, float** dst, const float* src, size_t n)
{
    dfree(*dst);
    *dst = nullptr;
    if (!src) return HD_OK;
    HIPCHK(c, hipMalloc(dst, n * sizeof(float)));
    HIPCHK(c, hipMemcpy(*dst, src, n * sizeof(float), hipMemcpyHostToDevice));
    return HD_OK;
}

extern "C" int hd_set_chan_calib(hd_ctx* c, const float* scl, const float* offs, const float* wts)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_set_chan_calib: NULL context");
    if (!c->have_obs) return fail(c, HD_E_STATE, "hd_set_chan_calib before hd_set_obs");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int rc;
    if ((rc = upload(c, &c->d_scl, scl, c->obs.nchan))) return rc;
    if ((rc = upload(c, &c->d_offs, offs, c->obs.nchan))) return rc;
    if ((rc = upload(c, &c->d_wts, wts, c->obs.nchan))) return rc;
    c->clip_valid = false;
    c->clip.stats_valid = false;
    return HD_OK;
}

extern "C" int hd_set_mask(hd_ctx* c, const uint8_t* mask, int32_t numint, int32_t ptsperint, double dtint,
                           const uint8_t* zapint, const float* padvals)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_set_mask: NULL context");
    if (!c->have_obs) return fail(c, HD_E_STATE, "hd_set_mask before hd_set_obs");
    if (mask && (numint <= 0 || ptsperint <= 0))
        return fail(c, HD_E_INVAL, "hd_set_mask: numint and ptsperint must be > 0");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, sync_all(c));
    free_blocks(c);
    clear_special_cache(c);
    c->h_mask.clear();
    c->h_zapint.clear();
    c->numint = c->ptsperint = 0;
    c->dtint = 0.0;
    if (mask) {
        const size_t n = (size_t)numint * c->obs.nchan;
        c->h_mask.assign(mask, mask + n);
        if (zapint) {
            c->h_zapint.assign(zapint, zapint + numint);
        } else {   // a row listing every channel stands for a zap_int
            c->h_zapint.assign((size_t)numint, 0);
            for (int32_t i = 0; i < numint; i++) {
                int32_t k = 0;
                for (int32_t ch = 0; ch < c->obs.nchan; ch++) k += mask[(size_t)i * c->obs.nchan + ch] != 0;
                c->h_zapint[i] = k == c->obs.nchan;
            }
        }
        c->numint = numint;
        c->ptsperint = ptsperint;
        c->dtint = dtint > 0 ? dtint : ptsperint * c->obs.dt;
    }
    if (padvals) c->h_padvals.assign(padvals, padvals + c->obs.nchan);
    else c->h_padvals.clear();
    return upload(c, &c->d_padvals, padvals, c->obs.nchan);
}

extern "C" int hd_stats_padvals(const float* dataavg, int32_t numint, int32_t numchan, float* padvals)
{
    if (!dataavg || !padvals || numint <= 0 || numchan <= 0)
        return fail(nullptr, HD_E_INVAL, "hd_stats_padvals: bad arguments");
    // determine_padvals -> calc_avgmedstd(..., 0.8, numchan, ...) per channel [PRESTO-ext]:
    // the middle `fraction` of the sorted interval averages, their avg_var (AS 52) mean
    const float fraction = 0.8f;
    const int len = (int)(numint * fraction + 0.5);
    const int start = (numint - len) / 2;
    std::vector<float> v((size_t)numint);
    for (int32_t ch = 0; ch < numchan; ch++) {
        for (int32_t i = 0; i < numint; i++) v[i] = dataavg[(size_t)i * numchan + ch];
        std::sort(v.begin(), v.end());
        double mean = 0.0;
        if (len > 0) {
            mean = (double)v[start];
            for (int i = 1; i < len; i++) mean += ((double)v[start + i] - mean) / (double)(i + 1);
        }
        padvals[ch] = (float)mean;
    }
    return HD_OK;
}

extern "C" int hd_push_raw(hd_ctx* c, const void* spectra, int64_t start, int64_t n)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_push_raw: NULL context");
    if (!c->have_obs) return fail(c, HD_E_STATE, "hd_push_raw before hd_set_obs");
    if (!spectra || start < 0 || n < 0 || start + n > c->obs.N)
        return fail(c, HD_E_INVAL, "hd_push_raw: range [%lld, %lld) outside [0, %lld)", (long long)start,
                    (long long)(start + n), (long long)c->obs.N);
    HIPCHK(c, hipSetDevice(c->device));
    int rc = ensure_raw(c);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_raw + (size_t)start * c->rowbytes, spectra, (size_t)n * c->rowbytes,
                             hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->raw_ready = true;
    c->rawT_valid = false;
    c->clip_valid = false;
    c->clip.stats_valid = false;
    return HD_OK;
}

// Streaming PSRFITS ingest: pread of the DATA column of row blocks into two pinned host
// buffers in turn, each followed by hipMemcpyAsync on the context stream; before a buffer is
// refilled its previous copy is waited for (its event), so reading block k+1 from the file
// overlaps the PCIe copy of block k.
static int read_full(int fd, void* dst, size_t n, off_t off)
{
    char* p = (char*)dst;
    while (n) {
        const ssize_t got = pread(fd, p, n, off);
        if (got <= 0) return -1;
        p += got;
        n -= (size_t)got;
        off += got;
    }
    return 0;
}

// Rows of a PSRFITS table to device spectra: kReaders threads, each with two pinned host blocks,
// take blocks of rows in turn (block k: thread k % kReaders); a thread's pread of its next block
// overlaps the copy of its previous one (each block is guarded by the event of the last copy
// that read it; a never-recorded event is complete), and the threads' preads run in parallel
// (one thread reads tmpfs at ~10 GB/s).  Spectra of the file are sb bytes: bytes
// [soff, soff + nb) of each go to bytes [doff, doff + nb) of device spectrum start + k (sb ==
// rb, soff = doff = 0, nb = sb: whole spectra).  Returns 0, HD_E_IO or HD_E_HIP; copies may
// still be in flight on st.
static int rows_to_device(int device, uint8_t* d_raw, int64_t rb, hipStream_t st, PinSet& ps, const char* path,
                          const hd_rows_src* src, int64_t start, int64_t sb, int64_t soff, int64_t doff, int64_t nb,
                          double& io)
{
    using clk = std::chrono::steady_clock;
    const int64_t spr = src->col_bytes / sb;   // spectra per row (NSBLK)
    const size_t want = src->block_bytes > 0 ? (size_t)src->block_bytes : (size_t)32 << 20;
    const int64_t rows_blk = std::max<int64_t>(1, (int64_t)(want / (size_t)src->col_bytes));
    const size_t blk_bytes = (size_t)rows_blk * (size_t)src->col_bytes;
    const int64_t nblocks = (src->nrows + rows_blk - 1) / rows_blk;
    const int nthr = (int)std::min<int64_t>(kReaders, std::max<int64_t>(nblocks, 1));
    if (ps.bytes < blk_bytes) {
        ps.release();
        for (int b = 0; b < 2 * kReaders; b++)
            if (hipHostMalloc(&ps.pin[b], blk_bytes, hipHostMallocDefault) != hipSuccess) return HD_E_HIP;
        ps.bytes = blk_bytes;
    }
    for (int b = 0; b < 2 * kReaders; b++)
        if (!ps.ev[b] && hipEventCreateWithFlags(&ps.ev[b], hipEventDisableTiming) != hipSuccess) return HD_E_HIP;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return HD_E_IO;
    std::atomic<int> err{0};
    std::vector<double> tio((size_t)nthr, 0.0);
    auto reader = [&](int t) {
        if (t > 0 && hipSetDevice(device) != hipSuccess) {
            err = HD_E_HIP;
            return;
        }
        for (int64_t k = t, i = 0; k < nblocks && !err.load(); k += nthr, i++) {
            const int b = 2 * t + (int)(i & 1);
            const int64_t r = k * rows_blk;
            const int64_t nr = std::min(rows_blk, src->nrows - r);
            if (hipEventSynchronize(ps.ev[b]) != hipSuccess) { err = HD_E_HIP; break; }
            const auto t0 = clk::now();
            char* dst = (char*)ps.pin[b];
            bool bad = false;
            if (src->col_offset == 0 && src->col_bytes == src->row_bytes) {
                bad = read_full(fd, dst, (size_t)(nr * src->col_bytes),
                                (off_t)(src->table_offset + (src->row0 + r) * src->row_bytes)) != 0;
            } else {
                for (int64_t q = 0; q < nr && !bad; q++)
                    bad = read_full(fd, dst + q * src->col_bytes, (size_t)src->col_bytes,
                                    (off_t)(src->table_offset + (src->row0 + r + q) * src->row_bytes + src->col_offset)) != 0;
            }
            tio[t] += std::chrono::duration<double>(clk::now() - t0).count();
            if (bad) { err = HD_E_IO; break; }
            const hipError_t ce =
                (sb == rb && nb == rb)
                    ? hipMemcpyAsync(d_raw + (size_t)(start + r * spr) * rb, dst, (size_t)(nr * src->col_bytes),
                                     hipMemcpyHostToDevice, st)
                    : hipMemcpy2DAsync(d_raw + (size_t)(start + r * spr) * rb + doff, (size_t)rb, dst + soff,
                                       (size_t)sb, (size_t)nb, (size_t)(nr * spr), hipMemcpyHostToDevice, st);
            if (ce != hipSuccess || hipEventRecord(ps.ev[b], st) != hipSuccess) { err = HD_E_HIP; break; }
        }
    };
    std::vector<std::thread> helpers;
    for (int t = 1; t < nthr; t++) helpers.emplace_back(reader, t);
    reader(0);
    for (auto& h : helpers) h.join();
    close(fd);
    double m = 0.0;                            // pread time: the busiest reader's
    for (double v : tio) m = std::max(m, v);
    io += m;
    return err.load();
}

// Argument checks shared by the synchronous and the prefetching file ingest.
static int check_rows_src(hd_ctx* c, const char* what, const char* path, const hd_rows_src* src, int64_t start,
                          int64_t sb, int64_t soff, int64_t doff, int64_t nb)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "%s: NULL context", what);
    if (!c->have_obs) return fail(c, HD_E_STATE, "%s before hd_set_obs", what);
    if (!path || !src) return fail(c, HD_E_INVAL, "%s: NULL argument", what);
    const int64_t rb = c->rowbytes;
    if (sb <= 0 || src->col_bytes <= 0 || src->col_bytes % sb || src->row_bytes < src->col_offset + src->col_bytes ||
        src->row0 < 0 || src->nrows < 0 || src->table_offset < 0)
        return fail(c, HD_E_INVAL, "%s: DATA column of %lld bytes is not whole spectra of %lld bytes "
                    "(or bad row geometry)", what, (long long)src->col_bytes, (long long)sb);
    if (soff < 0 || nb <= 0 || soff + nb > sb || doff < 0 || doff + nb > rb)
        return fail(c, HD_E_INVAL, "%s: bytes [%lld, %lld) of %lld-byte spectra into [%lld, %lld) "
                    "of %lld-byte spectra", what, (long long)soff, (long long)(soff + nb), (long long)sb, (long long)doff,
                    (long long)(doff + nb), (long long)rb);
    const int64_t spr = src->col_bytes / sb;
    if (start < 0 || start + src->nrows * spr > c->obs.N)
        return fail(c, HD_E_INVAL, "%s: spectra [%lld, %lld) outside [0, %lld)", what, (long long)start,
                    (long long)(start + src->nrows * spr), (long long)c->obs.N);
    return HD_OK;
}

static int push_raw_file_impl(hd_ctx* c, const char* path, const hd_rows_src* src, int64_t start, int64_t sb,
                              int64_t soff, int64_t doff, int64_t nb, double* io_seconds, double* total_seconds)
{
    using clk = std::chrono::steady_clock;
    const auto t_all = clk::now();
    int rc = check_rows_src(c, "hd_push_raw_file", path, src, start, sb, soff, doff, nb);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    rc = ensure_raw(c);
    if (rc) return rc;
    double io = 0.0;
    const int err = rows_to_device(c->device, c->d_raw, c->rowbytes, c->stream, c->pins, path, src, start, sb, soff,
                                   doff, nb, io);
    const hipError_t se = hipStreamSynchronize(c->stream);
    if (err == HD_E_IO) return fail(c, HD_E_IO, "hd_push_raw_file: cannot read %s", path);
    if (err || se != hipSuccess) return fail(c, HD_E_HIP, "hd_push_raw_file: HIP copy failed");
    c->raw_ready = true;
    c->rawT_valid = false;
    c->clip_valid = false;
    c->clip.stats_valid = false;
    if (io_seconds) *io_seconds = io;
    if (total_seconds) *total_seconds = std::chrono::duration<double>(clk::now() - t_all).count();
    return HD_OK;
}

// ---- overlapped ingest of the next beam ------------------------------------------------
static double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void pf_worker(hd_ctx* c, int device)
{
    hd_ctx::Prefetch* pf = c->pf;
    (void)hipSetDevice(device);
    const int64_t rb = c->rowbytes;
    for (;;) {
        PfJob j;
        {
            std::unique_lock<std::mutex> lk(pf->mu);
            pf->cv.wait(lk, [&] { return pf->stop || !pf->q.empty(); });
            if (pf->q.empty()) return;               // stop with nothing queued
            j = pf->q.front();
            pf->q.pop_front();
            pf->busy = true;
        }
        int err = 0;
        double io = 0.0;
        bool skip;
        {
            std::lock_guard<std::mutex> lk(pf->mu);
            skip = pf->err != 0;                     // after a failure only drain the queue
        }
        if (!skip) {
            if (j.fill) {
                if (j.count && hipMemsetAsync(pf->d_next + (size_t)j.start * rb, j.byte_value, (size_t)j.count * rb,
                                              pf->st) != hipSuccess)
                    err = HD_E_HIP;
            } else {
                err = rows_to_device(device, pf->d_next, rb, pf->st, pf->pins, j.path.c_str(), &j.src, j.start, j.sb,
                                     j.soff, j.doff, j.nb, io);
            }
        }
        {
            std::lock_guard<std::mutex> lk(pf->mu);
            pf->io += io;
            if (err && !pf->err) {
                pf->err = err;
                pf->errmsg = err == HD_E_IO ? "hd_prefetch_raw_file: cannot read " + j.path
                                            : std::string("hd_prefetch: HIP copy failed");
            }
            pf->busy = false;
        }
        pf->cv.notify_all();
    }
}

static void pf_stop(hd_ctx* c)
{
    hd_ctx::Prefetch* pf = c->pf;
    if (!pf) return;
    {
        std::lock_guard<std::mutex> lk(pf->mu);
        pf->stop = true;
        pf->q.clear();
    }
    pf->cv.notify_all();
    if (pf->th.joinable()) pf->th.join();
    if (pf->st) (void)hipStreamSynchronize(pf->st);
    dfree(pf->d_next);
    pf->pins.release();
    if (pf->ev_free) (void)hipEventDestroy(pf->ev_free);
    if (pf->ev_done) (void)hipEventDestroy(pf->ev_done);
    if (pf->st) (void)hipStreamDestroy(pf->st);
    delete pf;
    c->pf = nullptr;
}

// After a device fault: the reader thread stopped, nothing on the device released.
static void pf_abandon(hd_ctx* c)
{
    hd_ctx::Prefetch* pf = c->pf;
    if (!pf) return;
    {
        std::lock_guard<std::mutex> lk(pf->mu);
        pf->stop = true;
        pf->q.clear();
    }
    pf->cv.notify_all();
    if (pf->th.joinable()) pf->th.join();
    delete pf;
    c->pf = nullptr;
}

static int pf_queue(hd_ctx* c, PfJob&& j)
{
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->pf) {
        c->pf = new hd_ctx::Prefetch();
        hd_ctx::Prefetch* pf = c->pf;
        const size_t bytes = (size_t)c->obs.N * c->rowbytes;
        if (hipMalloc(&pf->d_next, bytes) != hipSuccess) {
            pf->d_next = nullptr;
            pf_stop(c);
            return fail(c, HD_E_NOMEM, "cannot allocate %zu bytes for the prefetched raw block", bytes);
        }
        if (hipStreamCreateWithFlags(&pf->st, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&pf->ev_free, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&pf->ev_done, hipEventDisableTiming) != hipSuccess) {
            pf_stop(c);
            return fail(c, HD_E_HIP, "hd_prefetch: cannot create the copy stream");
        }
        pf->th = std::thread(pf_worker, c, c->device);
    }
    hd_ctx::Prefetch* pf = c->pf;
    std::lock_guard<std::mutex> lk(pf->mu);
    if (pf->wait_free) {                             // the slot still holds the previous beam
        HIPCHK(c, hipStreamWaitEvent(pf->st, pf->ev_free, 0));
        pf->wait_free = false;
    }
    if (!pf->any) {
        pf->any = true;
        pf->t0 = now_s();
        pf->io = 0.0;
    }
    pf->q.push_back(std::move(j));
    pf->cv.notify_all();
    return HD_OK;
}

extern "C" int hd_prefetch_raw_file(hd_ctx* c, const char* path, const hd_rows_src* src, int64_t start)
{
    const int64_t rb = c ? c->rowbytes : 0;
    int rc = check_rows_src(c, "hd_prefetch_raw_file", path, src, start, rb, 0, 0, rb);
    if (rc) return rc;
    PfJob j;
    j.path = path;
    j.src = *src;
    j.start = start;
    j.sb = j.nb = rb;
    return pf_queue(c, std::move(j));
}

extern "C" int hd_prefetch_raw_file_band(hd_ctx* c, const char* path, const hd_rows_src* src, int64_t start,
                                         int64_t spec_bytes, int64_t src_offset, int64_t dst_offset, int64_t nbytes)
{
    int rc = check_rows_src(c, "hd_prefetch_raw_file_band", path, src, start, spec_bytes, src_offset, dst_offset,
                            nbytes);
    if (rc) return rc;
    PfJob j;
    j.path = path;
    j.src = *src;
    j.start = start;
    j.sb = spec_bytes;
    j.soff = src_offset;
    j.doff = dst_offset;
    j.nb = nbytes;
    return pf_queue(c, std::move(j));
}

extern "C" int hd_prefetch_fill(hd_ctx* c, int64_t start, int64_t count, int32_t byte_value)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_prefetch_fill: NULL context");
    if (!c->have_obs) return fail(c, HD_E_STATE, "hd_prefetch_fill before hd_set_obs");
    if (start < 0 || count < 0 || start + count > c->obs.N || byte_value < 0 || byte_value > 255)
        return fail(c, HD_E_INVAL, "hd_prefetch_fill: spectra [%lld, %lld) outside [0, %lld) or bad value",
                    (long long)start, (long long)(start + count), (long long)c->obs.N);
    PfJob j;
    j.fill = true;
    j.start = start;
    j.count = count;
    j.byte_value = byte_value;
    return pf_queue(c, std::move(j));
}

extern "C" int hd_swap_raw(hd_ctx* c, double* io_seconds, double* total_seconds)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_swap_raw: NULL context");
    hd_ctx::Prefetch* pf = c->pf;
    if (!pf || !pf->any) return fail(c, HD_E_STATE, "hd_swap_raw: nothing prefetched");
    HIPCHK(c, hipSetDevice(c->device));
    int err;
    std::string msg;
    double io, t0;
    {
        std::unique_lock<std::mutex> lk(pf->mu);
        pf->cv.wait(lk, [&] { return pf->q.empty() && !pf->busy; });
        err = pf->err;
        msg = pf->errmsg;
        io = pf->io;
        t0 = pf->t0;
        pf->err = 0;
        pf->errmsg.clear();
        pf->any = false;
    }
    if (err) {
        (void)hipStreamSynchronize(pf->st);
        return fail(c, err, "%s", msg.c_str());
    }
    // the context's streams run after the copies; the old block is free once the work queued
    // on it so far is done (the next prefetch into it waits for ev_free)
    HIPCHK(c, hipEventRecord(pf->ev_done, pf->st));
    HIPCHK(c, join_stream2(c));
    HIPCHK(c, join_aux(c));
    HIPCHK(c, hipEventRecord(pf->ev_free, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream, pf->ev_done, 0));
    {
        std::lock_guard<std::mutex> lk(pf->mu);
        pf->wait_free = true;
    }
    if (!c->d_raw) {
        const size_t bytes = (size_t)c->obs.N * c->rowbytes;
        if (hipMalloc(&c->d_raw, bytes) != hipSuccess) {
            c->d_raw = nullptr;
            return fail(c, HD_E_NOMEM, "cannot allocate %zu bytes of raw data", bytes);
        }
    }
    std::swap(c->d_raw, pf->d_next);
    c->raw_ready = true;
    c->rawT_valid = false;
    c->clip_valid = false;
    c->clip.stats_valid = false;
    if (io_seconds) *io_seconds = io;
    if (total_seconds) *total_seconds = now_s() - t0;
    return HD_OK;
}

extern "C" int hd_push_raw_file(hd_ctx* c, const char* path, const hd_rows_src* src, int64_t start,
                                double* io_seconds, double* total_seconds)
{
    const int64_t rb = c ? c->rowbytes : 0;
    return push_raw_file_impl(c, path, src, start, rb, 0, 0, rb, io_seconds, total_seconds);
}

extern "C" int hd_push_raw_file_band(hd_ctx* c, const char* path, const hd_rows_src* src, int64_t start,
                                     int64_t spec_bytes, int64_t src_offset, int64_t dst_offset, int64_t nbytes,
                                     double* io_seconds, double* total_seconds)
{
    return push_raw_file_impl(c, path, src, start, spec_bytes, src_offset, dst_offset, nbytes, io_seconds,
                              total_seconds);
}

extern "C" int hd_fill_raw(hd_ctx* c, int64_t start, int64_t count, int32_t byte_value)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_fill_raw: NULL context");
    if (!c->have_obs) return fail(c, HD_E_STATE, "hd_fill_raw before hd_set_obs");
    if (start < 0 || count < 0 || start + count > c->obs.N || byte_value < 0 || byte_value > 255)
        return fail(c, HD_E_INVAL, "hd_fill_raw: spectra [%lld, %lld) outside [0, %lld) or bad value",
                    (long long)start, (long long)(start + count), (long long)c->obs.N);
    HIPCHK(c, hipSetDevice(c->device));
    int rc = ensure_raw(c);
    if (rc) return rc;
    if (count) {
        HIPCHK(c, hipMemsetAsync(c->d_raw + (size_t)start * c->rowbytes, byte_value, (size_t)count * c->rowbytes,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    c->raw_ready = true;
    c->rawT_valid = false;
    c->clip_valid = false;
    c->clip.stats_valid = false;
    return HD_OK;
}

// Device-resident raw spectra (multi-GPU: the block another rank broadcast over RCCL).
extern "C" int hd_push_raw_device(hd_ctx* c, const void* dev_spectra, int64_t start, int64_t n)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_push_raw_device: NULL context");
    if (!c->have_obs) return fail(c, HD_E_STATE, "hd_push_raw_device before hd_set_obs");
    if (!dev_spectra || start < 0 || n < 0 || start + n > c->obs.N)
        return fail(c, HD_E_INVAL, "hd_push_raw_device: range [%lld, %lld) outside [0, %lld)", (long long)start,
                    (long long)(start + n), (long long)c->obs.N);
    HIPCHK(c, hipSetDevice(c->device));
    int rc = ensure_raw(c);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_raw + (size_t)start * c->rowbytes, dev_spectra, (size_t)n * c->rowbytes,
                             hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->raw_ready = true;
    c->rawT_valid = false;
    c->clip_valid = false;
    c->clip.stats_valid = false;
    return HD_OK;
}

extern "C" int hd_get_raw_device(hd_ctx* c, void* dev_out, int64_t start, int64_t n)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_get_raw_device: NULL context");
    if (!c->raw_ready || !c->d_raw) return fail(c, HD_E_STATE, "hd_get_raw_device: no raw data");
    if (!dev_out || start < 0 || n < 0 || start + n > c->obs.N) return fail(c, HD_E_INVAL, "hd_get_raw_device: bad range");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(dev_out, c->d_raw + (size_t)start * c->rowbytes, (size_t)n * c->rowbytes,
                             hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return HD_OK;
}

// Device -> pageable host copies: drain the stream first, then a blocking copy.  (An async
// copy into pageable memory is staged by the runtime; draining first keeps every read after
// the kernels that wrote the data whatever the staging does.)
static hipError_t d2h_2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
                         hipStream_t st)
{
    hipError_t e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = hipMemcpy2D(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToHost);
    return e;
}

static hipError_t d2h(void* dst, const void* src, size_t bytes, hipStream_t st)
{
    return d2h_2d(dst, bytes, src, bytes, bytes, 1, st);
}

extern "C" int hd_get_raw(hd_ctx* c, void* out, int64_t start, int64_t n)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_get_raw: NULL context");
    if (!c->raw_ready || !c->d_raw) return fail(c, HD_E_STATE, "hd_get_raw: no raw data");
    if (!out || start < 0 || n < 0 || start + n > c->obs.N) return fail(c, HD_E_INVAL, "hd_get_raw: bad range");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, d2h(out, c->d_raw + (size_t)start * c->rowbytes, (size_t)n * c->rowbytes, c->stream));
    return HD_OK;
}

// ---------------------------------------------------------------------------------------
// synthetic beam
// ---------------------------------------------------------------------------------------
extern "C" void hd_synth_default(hd_synth* s)
{
    if (!s) return;
    memset(s, 0, sizeof *s);
    s->seed = 20261015ull;
    s->base_level = 96.0f;
    s->bandpass_slope = 0.25f;
    s->noise_sigma = 12.0f;
    s->npsr = 3;
    s->psr_period[0] = 0.0046;  s->psr_dm[0] = 71.0;  s->psr_width[0] = 0.0004; s->psr_amp[0] = 4.0f;
    s->psr_period[1] = 0.253;   s->psr_dm[1] = 217.3; s->psr_width[1] = 0.008;  s->psr_amp[1] = 3.0f;
    s->psr_period[2] = 1.2;     s->psr_dm[2] = 612.0; s->psr_width[2] = 0.03;   s->psr_amp[2] = 3.0f;
    s->nspulse = 1;
    s->sp_time[0] = 1.5; s->sp_dm[0] = 350.0; s->sp_width[0] = 0.002; s->sp_amp[0] = 20.0f;
    s->rfi_nchan = 3;
    s->rfi_chan[0] = 101; s->rfi_chan[1] = 460; s->rfi_chan[2] = 777;
    s->rfi_amp = 30.0f;
    s->burst_frac = 0.01f;
    s->burst_len = 4096;
    s->burst_amp = 25.0f;
    s->spike_frac = 0.0005f;
    s->spike_amp = 15.0f;
}

static int64_t fp16(double x) { return (int64_t)llround(x * 65536.0); }
static uint32_t thresh32(double p)
{
    if (!(p > 0)) return 0;
    if (p >= 1) return 0xFFFFFFFFu;
    return (uint32_t)(p * 4294967296.0);
}

static int build_synth_table(const hd_obs* o, const hd_synth* s, std::vector<uint8_t>& buf, std::string& err)
{
    if (s->npsr < 0 || s->npsr > HD_SYNTH_MAX_PSR || s->nspulse < 0 || s->nspulse > HD_SYNTH_MAX_PSR ||
        s->rfi_nchan < 0 || s->rfi_nchan > 8) {
        err = "synth: bad source counts";
        return HD_E_INVAL;
    }
    const int nchan = o->nchan;
    buf.assign(hd_synth_tab_bytes(nchan, s->npsr, s->nspulse), 0);
    hd_synth_tab* tb = (hd_synth_tab*)buf.data();
    tb->nchan = nchan;
    tb->nbits = o->nbits;
    tb->flip = o->flip;
    tb->npsr = s->npsr;
    tb->nsp = s->nspulse;
    tb->burst_len = s->burst_len;
    tb->N = o->N;
    tb->seed = s->seed;
    if (o->nbits == 16) { tb->maxv = 32767; tb->minv = -32768; }
    else { tb->maxv = (1 << o->nbits) - 1; tb->minv = 0; }
    tb->burst_thresh = thresh32(s->burst_frac);
    tb->spike_thresh = thresh32(s->spike_frac);
    tb->burst_q4 = (int32_t)lround(16.0 * s->burst_amp);
    tb->spike_q4 = (int32_t)lround(16.0 * s->spike_amp);
    tb->rfi_q4 = (int32_t)lround(16.0 * s->rfi_amp);
    const double ftop = o->lofreq + (nchan - 1) * o->df;
    for (int p = 0; p < s->npsr; p++) {
        tb->psr_amp_q4[p] = (int32_t)lround(16.0 * s->psr_amp[p]);
        tb->psr_period_fp[p] = std::max<int64_t>(1, fp16(s->psr_period[p] / o->dt));
        tb->psr_width_fp[p] = fp16(s->psr_width[p] / o->dt);
    }
    for (int p = 0; p < s->nspulse; p++) {
        tb->sp_amp_q4[p] = (int32_t)lround(16.0 * s->sp_amp[p]);
        tb->sp_t0_fp[p] = fp16(s->sp_time[p] / o->dt);
        tb->sp_width_fp[p] = fp16(s->sp_width[p] / o->dt);
    }
    const int32_t *cb, *cn, *cr;
    const int64_t *pd, *sd;
    hd_synth_arrays(tb, &cb, &cn, &cr, &pd, &sd);
    int32_t* base_q4 = (int32_t*)cb;
    int32_t* noise_mul = (int32_t*)cn;
    int32_t* rfi = (int32_t*)cr;
    int64_t* psr_delay = (int64_t*)pd;
    int64_t* sp_delay = (int64_t*)sd;
    for (int c = 0; c < nchan; c++) {
        const double x = nchan > 1 ? (double)c / (nchan - 1) - 0.5 : 0.0;
        base_q4[c] = (int32_t)lround(16.0 * s->base_level * (1.0 + s->bandpass_slope * x));
        noise_mul[c] = (int32_t)lround(s->noise_sigma / 147.8 * 4096.0);
        rfi[c] = 0;
        const double f = o->lofreq + c * o->df;
        for (int p = 0; p < s->npsr; p++)
            psr_delay[(size_t)p * nchan + c] =
                fp16((delay_from_dm(s->psr_dm[p], f) - delay_from_dm(s->psr_dm[p], ftop)) / o->dt);
        for (int p = 0; p < s->nspulse; p++)
            sp_delay[(size_t)p * nchan + c] =
                fp16((delay_from_dm(s->sp_dm[p], f) - delay_from_dm(s->sp_dm[p], ftop)) / o->dt);
    }
    for (int i = 0; i < s->rfi_nchan; i++)
        if (s->rfi_chan[i] >= 0 && s->rfi_chan[i] < nchan) rfi[s->rfi_chan[i]] = 1;
    return HD_OK;
}

extern "C" int hd_synth_host(const hd_obs* o, const hd_synth* s, int64_t start, int64_t count, void* out)
{
    int rc = check_obs(nullptr, o);
    if (rc) return rc;
    if (!s || !out || start < 0 || count < 0 || start + count > o->N)
        return fail(nullptr, HD_E_INVAL, "hd_synth_host: bad arguments");
    std::vector<uint8_t> buf;
    std::string err;
    if ((rc = build_synth_table(o, s, buf, err))) return fail(nullptr, rc, "%s", err.c_str());
    const hd_synth_tab* tb = (const hd_synth_tab*)buf.data();
    const int32_t *cb, *cn, *cr;
    const int64_t *pd, *sd;
    hd_synth_arrays(tb, &cb, &cn, &cr, &pd, &sd);
    const int32_t rowbytes = (int32_t)((int64_t)o->nchan * o->nbits / 8);
    uint8_t* dst = (uint8_t*)out;
    unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (count < 4096) nth = 1;
    std::vector<std::thread> th;
    for (unsigned k = 0; k < nth; k++) {
        th.emplace_back([=]() {
            const int64_t a = count * k / nth, b = count * (k + 1) / nth;
            for (int64_t t = a; t < b; t++)
                for (int32_t by = 0; by < rowbytes; by++)
                    dst[t * rowbytes + by] = hd_synth_byte(tb, cb, cn, cr, pd, sd, start + t, by);
        });
    }
    for (auto& x : th) x.join();
    return HD_OK;
}

extern "C" int hd_synth_device(hd_ctx* c, const hd_synth* s)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_synth_device: NULL context");
    if (!c->have_obs) return fail(c, HD_E_STATE, "hd_synth_device before hd_set_obs");
    if (!s) return fail(c, HD_E_INVAL, "hd_synth_device: synth is NULL");
    std::vector<uint8_t> buf;
    std::string err;
    hd_obs whole = c->obs;                     // a time slice holds spectra [t0, t0 + N) of the beam
    if (c->slice_total) whole.N = c->slice_total;
    int rc = build_synth_table(&whole, s, buf, err);
    if (rc) return fail(c, rc, "%s", err.c_str());
    HIPCHK(c, hipSetDevice(c->device));
    if ((rc = ensure_raw(c))) return rc;
    void* d_tab = nullptr;
    HIPCHK(c, hipMalloc(&d_tab, buf.size()));
    HIPCHK(c, hipMemcpy(d_tab, buf.data(), buf.size(), hipMemcpyHostToDevice));
    hipError_t e = hd::launch_synth(c->d_raw, c->obs.N, c->rowbytes, (const hd_synth_tab*)d_tab, c->slice_t0,
                                    c->stream);
    hipError_t e2 = hipStreamSynchronize(c->stream);
    (void)hipFree(d_tab);
    if (e != hipSuccess || e2 != hipSuccess)
        return fail(c, HD_E_HIP, "synth kernel failed: %s", hipGetErrorString(e != hipSuccess ? e : e2));
    c->raw_ready = true;
    c->rawT_valid = false;
    c->clip_valid = false;
    c->clip.stats_valid = false;
    return HD_OK;
}

// ---------------------------------------------------------------------------------------
// plans
// ---------------------------------------------------------------------------------------
static const int kTT = 256, kSC = 8;

static void plan_free(hd_plan* p)
{
    dfree(p->d_idispdt);
    dfree(p->d_off);
    dfree(p->d_maxabs);
    dfree(p->d_omin);
    dfree(p->d_boff);
    for (auto& w : p->wide) {
        dfree(w.d_omin);
        dfree(w.d_boff);
        for (auto& q : w.d_boffp) dfree(q);
    }
    dfree(p->d_out);
    dfree(p->d_sub);
    dfree(p->d_bseg);
    dfree(p->d_topo);
    dfree(p->d_padv);
    if (p->fft && hd::fft_owner(p->fft) == p) hd::fft_set_owner(p->fft, nullptr);   // the context owns it
    p->fft = nullptr;
    for (auto& e : p->ev)
        if (e) (void)hipEventDestroy(e);
    p->dd_cur.reset();
    p->dd_own.reset();
    if (p->ev_copy) (void)hipEventDestroy(p->ev_copy);
    if (p->sp) {
        if (p->sp->b) {                               // a search never collected: its buffers back
            (void)hipEventSynchronize(p->sp->b->ev);
            p->ctx->sp_free.push_back(p->sp->b);
        }
        delete p->sp;
        p->sp = nullptr;
    }
}

struct Tables {
    std::vector<int32_t> idispdt, off;
    int32_t maxdelay = 0;
    double lof = 0, sbw = 0, sdt = 0;
};

// Validation + integer tables for one pass (shared by hd_plan_create and hd_plan_tables).
static int compute_tables(hd_ctx* c, const hd_obs& o, const hd_opts& opts, const hd_pass* ps, Tables& T)
{
    if (ps->nsub <= 0 || o.nchan % ps->nsub)
        return fail(c, HD_E_INVAL, "nsub (%d) must divide nchan (%d)", ps->nsub, o.nchan);
    if (ps->ds < 1) return fail(c, HD_E_INVAL, "ds must be >= 1");
    if (ps->numdms < 1) return fail(c, HD_E_INVAL, "numdms must be >= 1");
    if (ps->subdm < 0 || ps->lodm < 0 || ps->lodm + (ps->numdms - 1) * ps->dmstep < 0)
        return fail(c, HD_E_INVAL, "negative DMs are not supported");
    if (ps->numout < 0) return fail(c, HD_E_INVAL, "numout must be >= 0");
    const bool sub_input = (ps->flags & HD_PASS_SUB_INPUT) != 0;
    if (sub_input && (ps->nsub != o.nchan || ps->ds != 1))
        return fail(c, HD_E_INVAL, "HD_PASS_SUB_INPUT needs nsub == nchan (%d) and ds == 1", o.nchan);
    const int nchan = o.nchan, nsub = ps->nsub, cps = nchan / nsub;

    // stage-1 channel delays at subdm (subband_search_delays / dt)
    std::vector<double> d(nchan), sd(nsub);
    dedisp_delays(nchan, ps->subdm, o.lofreq, o.df, o.voverc, d.data());
    subband_delays(nchan, nsub, ps->subdm, o.lofreq, o.df, o.voverc, sd.data());
    T.idispdt.assign(nchan, 0);
    T.maxdelay = 0;
    if (!sub_input)
        for (int s = 0, ch = 0; s < nsub; s++)
            for (int k = 0; k < cps; k++, ch++) {
                T.idispdt[ch] = (int32_t)nearest_long((d[ch] - sd[s]) / o.dt);
                T.maxdelay = std::max(T.maxdelay, T.idispdt[ch]);
            }

    // subband-level parameters as carried by the .sub.inf
    double lof = o.lofreq + o.df * cps - o.df, sbw = o.df * cps, sdt = o.dt * ps->ds;
    if (sub_input) {   // the .sub.inf values, as read
        lof = o.lofreq;
        sbw = o.df;
        sdt = o.dt;
    } else if (opts.inf_roundtrip) {
        lof = text_roundtrip(lof, "%.12g");
        sbw = text_roundtrip(sbw, "%.12g");
        sdt = text_roundtrip(sdt, "%.15g");
    }
    T.lof = lof;
    T.sbw = sbw;
    T.sdt = sdt;

    // stage-2 offsets
    T.off.resize((size_t)ps->numdms * nsub);
    for (int i = 0; i < ps->numdms; i++) {
        const double dm = ps->lodm + i * ps->dmstep;
        subband_delays(nsub, nsub, dm, lof, sbw, o.voverc, sd.data());
        const double top = sd[nsub - 1];
        for (int s = 0; s < nsub; s++) T.off[(size_t)i * nsub + s] = (int32_t)nearest_long((sd[s] - top) / sdt);
    }
    return HD_OK;
}

extern "C" int hd_plan_tables(const hd_obs* o, const hd_opts* opts, const hd_pass* ps, int32_t* chan_delays,
                              int32_t* dm_offsets, double* sub_lofreq, double* sub_chanwid, double* sub_dt)
{
    int rc = check_obs(nullptr, o);
    if (rc) return rc;
    if (!ps) return fail(nullptr, HD_E_INVAL, "hd_plan_tables: pass is NULL");
    hd_opts op;
    if (opts) op = *opts; else hd_opts_default(&op);
    Tables T;
    if ((rc = compute_tables(nullptr, *o, op, ps, T))) return rc;
    if (chan_delays) memcpy(chan_delays, T.idispdt.data(), sizeof(int32_t) * T.idispdt.size());
    if (dm_offsets) memcpy(dm_offsets, T.off.data(), sizeof(int32_t) * T.off.size());
    if (sub_lofreq) *sub_lofreq = T.lof;
    if (sub_chanwid) *sub_chanwid = T.sbw;
    if (sub_dt) *sub_dt = T.sdt;
    return HD_OK;
}

// Tables of a wide-tile stage-2 variant: y-blocks of up to nwmax*5 DMs (nw waves x Q DMs),
// T = 256*R samples per tile, windows of ws elements per shifted copy, sc subbands per chunk;
// boff[yb][s][k] = LDS byte offset of DM k's 4 samples for subband s (lane 0).
static void wide_tables(hd_plan* p, int nwmax, bool dbuf, bool i16, hd_plan::Wide& w, std::vector<int32_t>& omin,
                        std::vector<int32_t>& boff, bool ring = false)
{
    const int nsub = p->pass.nsub, numdms = p->pass.numdms;
    int nyb = (numdms + 5 * nwmax - 1) / (5 * nwmax);
    const int per = (numdms + nyb - 1) / nyb;
    const int qneed = (per + nwmax - 1) / nwmax;
    int Q = 2, R = 4;
    if (qneed > 4) { Q = 5; R = 3; }
    else if (qneed > 3) { Q = 4; R = ring ? 3 : 4; }
    else if (qneed > 2) { Q = 3; R = 4; }
    const int nw = ring ? 16 : (per + Q - 1) / Q;   // the ring needs all 16 waves as DMA loaders
    const int dpb = nw * Q;
    nyb = (numdms + dpb - 1) / dpb;
    omin.assign((size_t)nyb * nsub, 0);
    int32_t span = 0;
    for (int yb = 0; yb < nyb; yb++)
        for (int s = 0; s < nsub; s++) {
            int32_t lo = INT32_MAX, hi = INT32_MIN;
            for (int k = 0; k < dpb; k++) {
                const int dm = std::min(yb * dpb + k, numdms - 1);
                const int32_t v = p->off[(size_t)dm * nsub + s];
                lo = std::min(lo, v);
                hi = std::max(hi, v);
            }
            omin[(size_t)yb * nsub + s] = lo;
            span = std::max(span, hi - lo);
        }
    const int ws = (int)round_up((size_t)(256 * R + span + 4), 4);
    int sc = 0;
    int npw = 0, nbp = 0;
    if (ring) {   // 4-subband chunks, every loader piece from one of the 16 waves, LDS fits
        npw = (int)((((size_t)ws + 8) * 2 + 1023) / 1024);
        nbp = (int)(((size_t)hd::kRingSC * dpb * 4 + 1023) / 1024);
        if (nsub % hd::kRingSC == 0 && nw == 16 && hd::kRingSC * npw + nbp <= 16 &&
            hd::stage2_ring_lds_bytes(ws, npw, nbp, nsub) <= 160 * 1024)
            sc = hd::kRingSC;
    }
    for (int pass = 0; pass < 2 && !sc && !ring; pass++)
        for (int cand : {8, 4}) {
            if (nsub % cand) continue;
            const size_t lds = dbuf ? hd::stage2_wide_lds_bytes(ws, cand) : hd::stage2_wide2_lds_bytes(ws, cand, nsub);
            const bool fits = lds <= (size_t)(dbuf || pass ? 160 : 80) * 1024;
            const bool units = !dbuf || (size_t)cand * (ws / 4) <= (size_t)hd::kUMax * nw * 64;
            // double-buffered: prefer chunks whose fill units are all prefetched (the overflow is
            // filled synchronously)
            if (fits && (units || pass)) { sc = cand; break; }
        }
    w = hd_plan::Wide{};
    w.ok = i16 && nw <= nwmax && (ring ? hd::stage2_ring_supports(Q, R) : hd::stage2_wide_supports(Q, R)) && sc > 0;
    if (!w.ok) return;
    w.q = Q;
    w.r = R;
    w.nw = nw;
    w.dpb = dpb;
    w.ws = ws;
    w.sc = sc;
    w.npw = npw;
    w.nbp = nbp;
    boff.resize((size_t)nyb * nsub * dpb);   // (the ring's DMA tail: stage2_host_tables)
    for (int yb = 0; yb < nyb; yb++)
        for (int s = 0; s < nsub; s++)
            for (int k = 0; k < dpb; k++) {
                const int dm = std::min(yb * dpb + k, numdms - 1);
                const int32_t o2 = p->off[(size_t)dm * nsub + s] - omin[(size_t)yb * nsub + s];
                const int32_t buf = dbuf ? (s / sc) & 1 : 0, sl = s % sc;
                boff[((size_t)yb * nsub + s) * dpb + k] = (((buf * sc + sl) * 4 + (o2 & 3)) * ws + (o2 & ~3)) * 2;
            }
}

// Tables of the pair variant (k_stage2_pair): the ring's y-blocks (16 waves x Q DMs), one
// subband pair (2c, 2c+1) per chunk.  Per y-block and pair: the distinct relative offsets
// r = off[d][2c+1] - off[d][2c] of the block's DMs (sorted; at most kPairUMax, else the
// variant does not apply), base0 = min off[d][2c], b1 = base0 + min r, and the S1 staging
// index k1[u] = r_u - min r + (b1 & 1) of pattern u.  boff[yb][c][k] = LDS byte offset
// (from the expanded area) of DM k's 4 samples: buffer (c & 1), pattern u(k), copy o2 & 3.
static void pair_tables(hd_plan* p, bool i16, int ppc, hd_plan::Wide& w, std::vector<int32_t>& ptab,
                        std::vector<int32_t>& boff)
{
    w = hd_plan::Wide{};
    const int nsub = p->pass.nsub, numdms = p->pass.numdms;
    const int nw = 16;
    // chunks of ppc pairs; an even chunk count per tile keeps the expanded-buffer parity of a
    // pair the same in every tile (the tables below fix it per pair)
    if (!i16 || nsub % (4 * ppc) || numdms < 1) return;
    int nyb = (numdms + 5 * nw - 1) / (5 * nw);
    const int per = (numdms + nyb - 1) / nyb;
    const int qneed = (per + nw - 1) / nw;
    int Q = 2, R = 4;
    if (qneed > 4) { Q = 5; R = 3; }
    else if (qneed > 3) { Q = 4; R = 3; }
    else if (qneed > 2) { Q = 3; R = 4; }
    const int dpb = nw * Q;
    nyb = (numdms + dpb - 1) / dpb;
    const int npair = nsub / 2;
    ptab.assign((size_t)nyb * npair * hd::kPairTab, 0);
    std::vector<std::vector<int32_t>> rs((size_t)nyb * npair);
    int32_t span0 = 0, k1max = 0;
    int umax = 0;
    auto dmof = [&](int yb, int k) { return std::min(yb * dpb + k, numdms - 1); };
    for (int yb = 0; yb < nyb; yb++)
        for (int c = 0; c < npair; c++) {
            const int s0 = 2 * c, s1 = s0 + 1;
            int32_t lo = INT32_MAX, hi = INT32_MIN;
            std::vector<int32_t>& r = rs[(size_t)yb * npair + c];
            for (int k = 0; k < dpb; k++) {
                const int dm = dmof(yb, k);
                const int32_t o0 = p->off[(size_t)dm * nsub + s0], o1 = p->off[(size_t)dm * nsub + s1];
                lo = std::min(lo, o0);
                hi = std::max(hi, o0);
                r.push_back(o1 - o0);
            }
            std::sort(r.begin(), r.end());
            r.erase(std::unique(r.begin(), r.end()), r.end());
            if ((int)r.size() > hd::kPairUMax) return;
            const int32_t b1 = lo + r[0];
            int32_t* t = &ptab[((size_t)yb * npair + c) * hd::kPairTab];
            t[0] = lo;
            t[1] = b1;
            t[2] = (int32_t)r.size();
            for (size_t u = 0; u < r.size(); u++) {
                t[3 + u] = r[u] - r[0] + (b1 & 1);
                k1max = std::max(k1max, t[3 + u]);
            }
            span0 = std::max(span0, hi - lo);
            umax = std::max(umax, (int)r.size());
        }
    // a multiple of 8 elements: the expand stores 8-element (16-byte) pieces of each copy
    const int ws = (int)round_up((size_t)(256 * R + span0 + 4), 8);
    const int npw = (int)((((size_t)ws + 14 + k1max) * 2 + 1023) / 1024);
    const int nbp = (int)(((size_t)ppc * dpb * 4 + 1023) / 1024);
    if (2 * ppc * npw + nbp > nw || hd::stage2_pair_lds_bytes(ws, npw, nbp, nsub, umax, ppc) > 160 * 1024 ||
        !hd::stage2_pair_supports(Q, R))
        return;
    boff.assign((size_t)nyb * npair * dpb, 0);   // (the DMA tail: stage2_host_tables)
    for (int yb = 0; yb < nyb; yb++)
        for (int c = 0; c < npair; c++) {
            const std::vector<int32_t>& r = rs[(size_t)yb * npair + c];
            const int32_t base0 = ptab[((size_t)yb * npair + c) * hd::kPairTab];
            for (int k = 0; k < dpb; k++) {
                const int dm = dmof(yb, k);
                const int32_t o0 = p->off[(size_t)dm * nsub + 2 * c], o1 = p->off[(size_t)dm * nsub + 2 * c + 1];
                const int u = (int)(std::lower_bound(r.begin(), r.end(), o1 - o0) - r.begin());
                const int32_t o2 = o0 - base0;
                const int buf = ((c / ppc) & 1) * ppc + c % ppc;   // expanded buffer of pair c
                boff[((size_t)yb * npair + c) * dpb + k] = (((buf * umax + u) * 4 + (o2 & 3)) * ws + (o2 & ~3)) * 2;
            }
        }
    w.ok = true;
    w.q = Q;
    w.r = R;
    w.nw = nw;
    w.dpb = dpb;
    w.ws = ws;
    w.sc = 2;
    w.npw = npw;
    w.nbp = nbp;
    w.umax = umax;
}

// The quarter-layout pair kernel as the auto stage-2 choice (HD_S2_QP=0 keeps the four-copy
// pair kernel, for A/B): measured in the bench context 62.4 vs 67.1 ms per C2 beam, stage 2
// 32.9 vs 37.5 ms (k_stage2_qp<5,3,4> 5.55 vs k_stage2_pair<5,3,2> 6.35 ms per stage-0 launch;
// scripts/r5_ab.sh, profiles/r05_ab_qp.txt).
static bool qp_auto()
{
    static const int v = [] {
        const char* e = getenv("HD_S2_QP");
        return e ? atoi(e) : 1;
    }();
    return v != 0;
}

// Tables of the quarter-layout pair kernel (k_stage2_qp): y-blocks of 16 waves x Q DMs (Q 4
// or 5), tiles of T = 4 S = 768 samples, ppc pairs per chunk.  Per (y-block, pair) the pair
// kernel's {base0, b1, U, k1[U]} and [9] E_k = the pair's entries per pattern (S + its own
// DM sweep, a multiple of 4).  boff[yb][c][k] = LDS byte offset (from the expanded area) of
// DM k's entry 0: buffer ((c / ppc) & 1) * ppc + c % ppc, pattern u(k), entry o2 = o0 - base0.
static void qp_tables(hd_plan* p, bool i16, hd_plan::Wide& w, std::vector<int32_t>& ptab, std::vector<int32_t>& boff,
                      std::vector<int32_t> (&boffp)[3])
{
    w = hd_plan::Wide{};
    constexpr int RQ = 3, S = 64 * RQ, T = 4 * S;
    // 16 waves x Q = 4..5 DMs (128 VGPRs: one step of LDS read lookahead), or (HD_QP_W12=1, A/B)
    // 12 waves x Q = 6..7 DMs (168 VGPRs: two steps)
    static const bool w12 = getenv("HD_QP_W12") && atoi(getenv("HD_QP_W12")) != 0;
    const int NW = w12 ? 12 : 16, qlo = w12 ? 6 : 4, qhi = w12 ? 7 : 5;
    const int nsub = p->pass.nsub, numdms = p->pass.numdms;
    if (!i16 || nsub % 2 || numdms < 1) return;
    int nyb = (numdms + qhi * NW - 1) / (qhi * NW);
    const int per = (numdms + nyb - 1) / nyb;
    const int Q = (per + NW - 1) / NW > qlo ? qhi : qlo;
    const int dpb = NW * Q;
    nyb = (numdms + dpb - 1) / dpb;
    const int npair = nsub / 2;
    ptab.assign((size_t)nyb * npair * hd::kPairTab, 0);
    std::vector<std::vector<int32_t>> rs((size_t)nyb * npair);
    int32_t Emax = 0, k1max = 0;
    int umax = 0;
    auto dmof = [&](int yb, int k) { return std::min(yb * dpb + k, numdms - 1); };
    for (int yb = 0; yb < nyb; yb++)
        for (int c = 0; c < npair; c++) {
            int32_t lo = INT32_MAX, hi = INT32_MIN;
            std::vector<int32_t>& r = rs[(size_t)yb * npair + c];
            for (int k = 0; k < dpb; k++) {
                const int dm = dmof(yb, k);
                const int32_t o0 = p->off[(size_t)dm * nsub + 2 * c], o1 = p->off[(size_t)dm * nsub + 2 * c + 1];
                lo = std::min(lo, o0);
                hi = std::max(hi, o0);
                r.push_back(o1 - o0);
            }
            std::sort(r.begin(), r.end());
            r.erase(std::unique(r.begin(), r.end()), r.end());
            if ((int)r.size() > hd::kPairUMax) return;
            const int32_t b1 = lo + r[0];
            int32_t* t = &ptab[((size_t)yb * npair + c) * hd::kPairTab];
            t[0] = lo;
            t[1] = b1;
            t[2] = (int32_t)r.size();
            for (size_t u = 0; u < r.size(); u++) {
                t[3 + u] = r[u] - r[0] + (b1 & 1);
                k1max = std::max(k1max, t[3 + u]);
            }
            t[9] = (int32_t)round_up((size_t)(S + hi - lo), 4);
            Emax = std::max(Emax, t[9]);
            umax = std::max(umax, (int)r.size());
        }
    // the chunk's pairs packed in its buffer set, per pairs-per-chunk q dividing the pair count:
    // pair c at byte pb_q(c) = the U x E bytes of the chunk's pairs before it; the set is the
    // largest chunk's (every chunk of every y-block)
    int32_t setb[3] = {0, 0, 0};
    for (int qi = 0; qi < 3; qi++) {
        const int q = 4 - qi;
        if (npair % q) continue;
        for (int yb = 0; yb < nyb; yb++)
            for (int ch = 0; ch < npair / q; ch++) {
                int32_t run = 0;
                for (int k = 0; k < q; k++) {
                    int32_t* t = &ptab[((size_t)yb * npair + q * ch + k) * hd::kPairTab];
                    t[hd::kQpPb + qi] = run;
                    run += t[2] * t[9] * 8;
                }
                setb[qi] = std::max(setb[qi], (int32_t)round_up((size_t)run, 32));
            }
    }
    // the expand reads staging elements up to 4 g + 3 S + k + 7 < E + 3 S + k1max + 8
    // the most pairs per chunk (4, 3, 2 dividing the pair count) whose LDS fits; a shared launch
    // takes the smallest of its passes' (the offset block per chunk is sized for 4 pairs)
    const int npw = (int)((((size_t)Emax + 3 * S + k1max + 8) * 2 + 1023) / 1024);
    const int nbp = (int)(((size_t)4 * dpb * 4 + 1023) / 1024);
    int ppc = 0;
    static const int ppc_cap = getenv("HD_QP_PPC") ? atoi(getenv("HD_QP_PPC")) : 4;   // (A/B)
    for (int cand : {4, 3, 2})
        if (cand <= ppc_cap && (nsub / 2) % cand == 0 && 2 * cand * npw + nbp <= 32 &&
            hd::stage2_qp_lds_bytes(setb[4 - cand], npw, nbp, nsub, cand) <= 160 * 1024) {
            ppc = cand;
            break;
        }
    if (getenv("HD_QP_INFO"))
        fprintf(stderr, "qp_tables: nsub %d numdms %d Q %d ppc %d npw %d nbp %d setb %d/%d/%d lds %zu\n", nsub, numdms,
                Q, ppc, npw, nbp, setb[0], setb[1], setb[2],
                ppc ? hd::stage2_qp_lds_bytes(setb[4 - ppc], npw, nbp, nsub, ppc) : (size_t)0);
    if (!ppc || !hd::stage2_qp_supports(Q, RQ) || (size_t)npw * 512 > 4096) return;
    // one offsets table per pairs-per-chunk a shared launch may take (ppc and every smaller
    // candidate dividing the pair count): set (c / q) & 1, pair c at pb_q(c)
    for (int qi = 0; qi < 3; qi++) {
        const int q = 4 - qi;
        std::vector<int32_t>& bo = boffp[qi];
        bo.clear();
        if (q > ppc || (nsub / 2) % q) continue;
        bo.assign((size_t)nyb * npair * dpb, 0);   // (the DMA tail: stage2_host_tables)
        for (int yb = 0; yb < nyb; yb++)
            for (int c = 0; c < npair; c++) {
                const std::vector<int32_t>& r = rs[(size_t)yb * npair + c];
                const int32_t base0 = ptab[((size_t)yb * npair + c) * hd::kPairTab];
                const int32_t* t = &ptab[((size_t)yb * npair + c) * hd::kPairTab];
                const int64_t set0 = (int64_t)((c / q) & 1) * setb[qi] + t[hd::kQpPb + qi];
                for (int k = 0; k < dpb; k++) {
                    const int dm = dmof(yb, k);
                    const int32_t o0 = p->off[(size_t)dm * nsub + 2 * c], o1 = p->off[(size_t)dm * nsub + 2 * c + 1];
                    const int u = (int)(std::lower_bound(r.begin(), r.end(), o1 - o0) - r.begin());
                    bo[((size_t)yb * npair + c) * dpb + k] = (int32_t)(set0 + ((int64_t)u * t[9] + (o0 - base0)) * 8);
                }
            }
    }
    boff = boffp[4 - ppc];
    (void)T;
    w.ok = true;
    w.q = Q;
    w.r = RQ;                      // 256 * r = the tile (ntiles, partial sums)
    w.nw = NW;
    w.dpb = dpb;
    w.ws = Emax;
    w.sc = ppc;
    w.npw = npw;
    w.nbp = nbp;
    w.umax = umax;
    for (int qi = 0; qi < 3; qi++) w.setb[qi] = setb[qi];
}

// Tables of the register-window pair kernel (k_stage2_rw): y-blocks of 8 waves x Q DMs, two
// pairs per chunk, 768-sample tiles (lane l: samples 12l .. 12l+11).  Per (y-block, pair) the
// pair kernel's {base0, b1, U, k1[U]} over the block's DMs.  Per (y-block, chunk) one block of
// kRwBlock ints: [pair k][DM slot] the jump code 12 + 100 * shift of the DM's 12 values in
// its wave's current window, then [pair k][wave] {reload mask, window byte offsets} (8 ints): a wave
// loads a window (24 elements per lane, 8-byte aligned) at its first DM and again at each DM
// of the mask whose pattern buffer or offset leaves the current one (> 10 elements on).
// Window offsets are LDS bytes from the expanded area: buffer ((chunk & 1) * 2 + k) x umax
// patterns x ws elements; element i of pattern u = P_u[i], tile sample 0 at offset base0.
static void rw_tables(hd_plan* p, bool i16, hd_plan::Wide& w, std::vector<int32_t>& ptab, std::vector<int32_t>& blk)
{
    w = hd_plan::Wide{};
    constexpr int NW = hd::kRwWaves, PPC = 2;
    const int nsub = p->pass.nsub, numdms = p->pass.numdms;
    if (!i16 || nsub % (4 * PPC) || numdms < 1) return;
    int nyb = (numdms + 5 * NW - 1) / (5 * NW);
    const int per = (numdms + nyb - 1) / nyb;
    const int Q = (per + NW - 1) / NW;                    // 1..5
    const int dpb = NW * Q;
    nyb = (numdms + dpb - 1) / dpb;
    const int npair = nsub / 2, nchunk = npair / PPC;
    if (PPC * dpb + PPC * NW * 8 > hd::kRwBlock) return;
    auto dmof = [&](int yb, int k) { return std::min(yb * dpb + k, numdms - 1); };
    ptab.assign((size_t)nyb * npair * hd::kPairTab, 0);
    std::vector<std::vector<int32_t>> rs((size_t)nyb * npair);
    int32_t span0 = 0, k1max = 0;
    int umax = 0;
    for (int yb = 0; yb < nyb; yb++)
        for (int c = 0; c < npair; c++) {
            int32_t lo = INT32_MAX, hi = INT32_MIN;
            std::vector<int32_t>& r = rs[(size_t)yb * npair + c];
            for (int k = 0; k < dpb; k++) {
                const int dm = dmof(yb, k);
                const int32_t o0 = p->off[(size_t)dm * nsub + 2 * c], o1 = p->off[(size_t)dm * nsub + 2 * c + 1];
                lo = std::min(lo, o0);
                hi = std::max(hi, o0);
                r.push_back(o1 - o0);
            }
            std::sort(r.begin(), r.end());
            r.erase(std::unique(r.begin(), r.end()), r.end());
            if ((int)r.size() > hd::kPairUMax) return;
            const int32_t b1 = lo + r[0];
            int32_t* t = &ptab[((size_t)yb * npair + c) * hd::kPairTab];
            t[0] = lo;
            t[1] = b1;
            t[2] = (int32_t)r.size();
            for (size_t u = 0; u < r.size(); u++) {
                t[3 + u] = r[u] - r[0] + (b1 & 1);
                k1max = std::max(k1max, t[3 + u]);
            }
            span0 = std::max(span0, hi - lo);
            umax = std::max(umax, (int)r.size());
        }
    // a lane's window reaches element (o & ~3) + 12 * 63 + 23 <= span0 + 779; 8-element items
    const int ws = (int)round_up((size_t)span0 + 780, 8);
    // the expand's 8-element loads read the staging window up to element k1 + ws + 1
    const int npw = (int)((((size_t)ws + 16 + k1max) * 2 + 1023) / 1024);
    if (hd::stage2_rw_lds_bytes(ws, npw, nsub, umax) > 80 * 1024) return;
    blk.assign((size_t)nyb * nchunk * hd::kRwBlock, 0);
    for (int yb = 0; yb < nyb; yb++)
        for (int ch = 0; ch < nchunk; ch++) {
            int32_t* b = &blk[((size_t)yb * nchunk + ch) * hd::kRwBlock];
            for (int k = 0; k < PPC; k++) {
                const int c = PPC * ch + k;
                const std::vector<int32_t>& r = rs[(size_t)yb * npair + c];
                const int32_t base0 = ptab[((size_t)yb * npair + c) * hd::kPairTab];
                const int buf = (ch & 1) * PPC + k;
                for (int wv = 0; wv < NW; wv++) {
                    int32_t* rec = b + PPC * dpb + (k * NW + wv) * 8;
                    int64_t wb = -1;
                    int nwin = 0;
                    for (int q = 0; q < Q; q++) {
                        const int dm = dmof(yb, wv * Q + q);
                        const int32_t o0 = p->off[(size_t)dm * nsub + 2 * c], o1 = p->off[(size_t)dm * nsub + 2 * c + 1];
                        const int u = (int)(std::lower_bound(r.begin(), r.end(), o1 - o0) - r.begin());
                        const int64_t a = 2 * ((int64_t)(buf * umax + u) * ws + (o0 - base0));
                        if (q == 0 || a < wb || a - wb > 20) {
                            if (nwin == hd::kRwMaxWin) return;    // (a wave spanning more windows: not this kernel)
                            wb = a & ~(int64_t)7;
                            if (q > 0) rec[0] |= 1 << q;
                            rec[1 + nwin++] = (int32_t)wb;
                        }
                        b[k * dpb + wv * Q + q] = 12 + 100 * (int32_t)((a - wb) / 2);
                    }
                }
            }
        }
    w.ok = true;
    w.q = Q;
    w.r = 3;                       // 256 * r = the 768-sample tile (ntiles / partial sums)
    w.nw = NW;
    w.dpb = dpb;
    w.ws = ws;
    w.sc = 2;
    w.npw = npw;
    w.nbp = 1;
    w.umax = umax;
}

// Subbands formed by stage 1 on the device are >= 0 when the samples are unsigned integers
// (<= 8 bits, no calibration) and every pad value is >= 0: mask pads from the .stats file
// (h_padvals) and clip_times' running channel means (means of unsigned samples).
static bool stage1_sub_nonneg(const hd_ctx* c)
{
    if (c->d_scl || c->d_offs || c->d_wts || c->obs.nbits > 8) return false;
    for (float v : c->h_padvals)
        if (!(v >= 0.0f)) return false;
    return true;
}

// Static bound on |subband| for subbands formed by stage 1 on the device (-1: none): integer
// samples of <= 8 bits, no calibration, int16 sums of cps*ds samples or pad values.
static int32_t stage1_sub_bound(const hd_ctx* c, const hd_plan* p)
{
    if (c->opts.sub_dtype != HD_SUB_I16 || c->d_scl || c->d_offs || c->d_wts || c->obs.nbits > 8) return -1;
    double amax = (double)((1 << c->obs.nbits) - 1);
    for (float v : c->h_padvals) amax = std::max(amax, std::fabs((double)v));
    const int cps = (c->obs.nchan + p->pass.nsub - 1) / p->pass.nsub;
    const double b = std::ceil((double)cps * (c->opts.ds_mode == HD_DS_SUM ? p->pass.ds : 1) * amax) + 1.0;
    return b > 32767.0 ? 32767 : (int32_t)b;
}

// Lengths, strides and the integer tables of a plan (host only; hd_plan_create, hd_plan_extents).
static void plan_geometry(hd_plan* p, const hd_obs& o, const hd_pass* ps, Tables& T)
{
    p->pass = *ps;
    p->nds = o.N / ps->ds;
    p->numout = ps->numout > 0 ? ps->numout : p->nds;
    p->nvalid = std::min(p->nds, p->numout);
    int32_t maxoff = 0;
    for (int32_t v : T.off) maxoff = std::max(maxoff, v);
    // zero tail after N/ds: stage-2 windows (tile + offsets + DMA pieces) may read into it;
    // stage2_extents proves every window's last piece ends inside the block
    p->sub_stride = (int64_t)round_up((size_t)std::max<int64_t>(p->nds, 1) + (size_t)maxoff + 4096, 64);
    p->out_stride = (int64_t)round_up((size_t)p->numout, 64);
    p->idispdt = std::move(T.idispdt);
    p->off = std::move(T.off);
    p->maxdelay = T.maxdelay;
    p->sub_lofreq = T.lof;
    p->sub_chanwid = T.sbw;
    p->sub_dt = T.sdt;
}

// The host half of a plan's stage-2 variant tables: [k] the pair / window tables (womin) and
// offset tables (wboff) of p->wide[k], qpb the k_stage2_qp offsets for 4 / 3 / 2 pairs per
// chunk, and the DMA extents of every kernel that copies whole pieces (stage2_extents).
struct S2Host {
    std::vector<int32_t> womin[7], wboff[7], qpb[3];
    std::vector<hd_extent> ext;
};

// The furthest byte each whole-piece DMA of the stage-2 kernels can touch, per variant and
// buffer, from the same tile / window / piece numbers the kernels use:
//   windows: subband s's row + (t0 + b - (b & 1)) elements, then npw pieces of 1 KiB, with
//            t0 <= (ntiles - 1) T (the last tile any workgroup takes, persistent or not) and b
//            the window base of s in its y-block: the ring's omin (k_stage2_ring,
//            hd_stage2.hip:657-663), the pair table's base0 / b1 (k_stage2_pair :1018-1025,
//            k_stage2_rw :1449-1457, k_stage2_qp :2124-2131);
//   offsets: the table + (y-block, first row of the chunk) ints, then nbp pieces (ring
//            :664-667, pair :1026-1029, qp :2132-2135 -- sized for 4 pairs whatever the
//            launch's pairs per chunk), the register-window kernel one 1 KiB block (:1459).
// Each offset table gets exactly the zero tail its reach needs.
static void stage2_extents(const hd_plan* p, S2Host& h)
{
    const int nsub = p->pass.nsub, npair = nsub / 2, numdms = p->pass.numdms;
    const int64_t sub_bytes = (int64_t)2 * nsub * p->sub_stride;
    h.ext.clear();
    auto table = [&](int kernel, int ppc, std::vector<int32_t>& tab, int64_t reach) {
        const size_t need = (size_t)((reach + 3) / 4);
        if (tab.size() < need) tab.resize(need, 0);
        h.ext.push_back(hd_extent{kernel, HD_EXT_OFFSETS, ppc, 0, reach, (int64_t)(4 * tab.size())});
    };
    for (int k = 2; k <= 6; k++) {
        const hd_plan::Wide& w = p->wide[k];
        if (!w.ok || p->nvalid <= 0) continue;
        const int64_t T = 256 * (int64_t)w.r, ntiles = (p->nvalid + T - 1) / T, t0max = (ntiles - 1) * T;
        const int nyb = (numdms + w.dpb - 1) / w.dpb, dpb = w.dpb;
        int64_t sreach = 0;
        auto window = [&](int s, int32_t b) {
            sreach = std::max(sreach, ((int64_t)s * p->sub_stride + t0max + b - (b & 1)) * 2 + (int64_t)w.npw * 1024);
        };
        for (int yb = 0; yb < nyb; yb++) {
            if (k == 2) {
                for (int s = 0; s < nsub; s++) window(s, h.womin[2][(size_t)yb * nsub + s]);
            } else {
                for (int pr = 0; pr < npair; pr++)
                    for (int side = 0; side < 2; side++)
                        window(2 * pr + side, h.womin[k][((size_t)yb * npair + pr) * hd::kPairTab + side]);
            }
        }
        h.ext.push_back(hd_extent{k + 3, HD_EXT_SUBBANDS, k == 2 ? 0 : k == 3 ? 1 : k == 6 ? w.sc : 2, 0, sreach, sub_bytes});
        const int64_t nbp = (int64_t)w.nbp * 1024;
        if (k == 2) {
            const int nch = nsub / hd::kRingSC;
            table(5, 0, h.wboff[2], ((int64_t)(nyb - 1) * nsub * dpb + (int64_t)(nch - 1) * hd::kRingSC * dpb) * 4 + nbp);
        } else if (k == 3 || k == 4) {
            const int ppc = k == 3 ? 1 : 2;
            table(k + 3, ppc, h.wboff[k], ((int64_t)(nyb - 1) * npair * dpb + (int64_t)(npair / ppc - 1) * ppc * dpb) * 4 + nbp);
        } else if (k == 5) {
            const int nch = npair / 2;
            table(8, 2, h.wboff[5], ((int64_t)(nyb - 1) * nch + nch - 1) * hd::kRwBlock * 4 + 1024);
        } else {
            for (int qi = 0; qi < 3; qi++) {
                const int q = 4 - qi;
                if (h.qpb[qi].empty()) continue;
                table(9, q, h.qpb[qi], ((int64_t)(nyb - 1) * npair * dpb + (int64_t)(npair / q - 1) * q * dpb) * 4 + nbp);
            }
            h.wboff[6] = h.qpb[4 - w.sc];
        }
    }
}

static void stage2_host_tables(hd_plan* p, bool i16, S2Host& h)
{
    for (int k = 0; k < 3; k++)
        wide_tables(p, k == 1 ? 8 : 16, k != 1, i16, p->wide[k], h.womin[k], h.wboff[k], k == 2);
    pair_tables(p, i16, 1, p->wide[3], h.womin[3], h.wboff[3]);
    pair_tables(p, i16, 2, p->wide[4], h.womin[4], h.wboff[4]);
    rw_tables(p, i16, p->wide[5], h.womin[5], h.wboff[5]);
    qp_tables(p, i16, p->wide[6], h.womin[6], h.wboff[6], h.qpb);
    // the plain-load wide kernels ([0], [1]) read their tables exactly; a small tail anyway
    for (int k = 0; k < 2; k++)
        if (p->wide[k].ok) h.wboff[k].resize(h.wboff[k].size() + 256, 0);
    stage2_extents(p, h);
}

extern "C" int hd_plan_extents(const hd_obs* o, const hd_opts* opts, const hd_pass* ps, hd_extent* out, int32_t cap,
                               int32_t* n)
{
    int rc = check_obs(nullptr, o);
    if (rc) return rc;
    if (!ps || !n) return fail(nullptr, HD_E_INVAL, "hd_plan_extents: NULL argument");
    if (cap < 0 || (cap > 0 && !out)) return fail(nullptr, HD_E_INVAL, "hd_plan_extents: bad output buffer");
    hd_opts op;
    if (opts) op = *opts; else hd_opts_default(&op);
    Tables T;
    if ((rc = compute_tables(nullptr, *o, op, ps, T))) return rc;
    if (o->N / ps->ds < 1) return fail(nullptr, HD_E_INVAL, "hd_plan_extents: no sample at -downsamp %d", ps->ds);
    hd_plan p;
    plan_geometry(&p, *o, ps, T);
    S2Host h;
    stage2_host_tables(&p, op.sub_dtype == HD_SUB_I16, h);
    *n = (int32_t)h.ext.size();
    if ((int32_t)h.ext.size() > cap && cap > 0)
        return fail(nullptr, HD_E_NOMEM, "hd_plan_extents: %d records, room for %d", *n, cap);
    for (size_t i = 0; i < h.ext.size() && (int32_t)i < cap; i++) out[i] = h.ext[i];
    return HD_OK;
}

extern "C" int hd_plan_create(hd_ctx* c, const hd_pass* ps, hd_plan** out)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_plan_create: NULL context");
    if (!ps || !out) return fail(c, HD_E_INVAL, "hd_plan_create: NULL argument");
    *out = nullptr;
    if (!c->have_obs) return fail(c, HD_E_STATE, "hd_plan_create before hd_set_obs");
    const hd_obs& o = c->obs;
    Tables T;
    int rc0 = compute_tables(c, o, c->opts, ps, T);
    if (rc0) return rc0;
    if (o.N / ps->ds < 1)
        return fail(c, HD_E_INVAL, "hd_plan_create: %lld spectra give no sample at -downsamp %d", (long long)o.N, ps->ds);

    hd_plan* p = new hd_plan();
    p->ctx = c;
    plan_geometry(p, o, ps, T);
    const int nchan = o.nchan, nsub = ps->nsub;

    // LDS-variant tables
    const int need = (ps->numdms + 3) / 4;
    p->q = need <= 8 ? 8 : need <= 16 ? 16 : need <= 19 ? 19 : 24;
    p->dpb = 4 * p->q;
    p->nyblk = (ps->numdms + p->dpb - 1) / p->dpb;
    std::vector<int32_t> omin((size_t)p->nyblk * nsub), boff((size_t)p->nyblk * nsub * p->dpb);
    int32_t maxspan = 0;
    for (int yb = 0; yb < p->nyblk; yb++)
        for (int s = 0; s < nsub; s++) {
            int32_t lo = INT32_MAX, hi = INT32_MIN;
            for (int k = 0; k < p->dpb; k++) {
                const int dm = std::min(yb * p->dpb + k, ps->numdms - 1);
                const int32_t v = p->off[(size_t)dm * nsub + s];
                lo = std::min(lo, v);
                hi = std::max(hi, v);
            }
            omin[(size_t)yb * nsub + s] = lo;
            maxspan = std::max(maxspan, hi - lo);
        }
    p->wstride = (int32_t)round_up((size_t)(kTT + maxspan + 4), 4);
    const size_t lds_bytes = (size_t)kSC * 4 * p->wstride * sizeof(int16_t);
    p->lds_ok = (c->opts.sub_dtype == HD_SUB_I16) && lds_bytes <= 64 * 1024;
    for (int yb = 0; yb < p->nyblk; yb++)
        for (int s = 0; s < nsub; s++)
            for (int k = 0; k < p->dpb; k++) {
                const int dm = std::min(yb * p->dpb + k, ps->numdms - 1);
                const int32_t o2 = p->off[(size_t)dm * nsub + s] - omin[(size_t)yb * nsub + s];
                const int32_t sl = s % kSC;
                boff[((size_t)yb * nsub + s) * p->dpb + k] = ((sl * 4 + (o2 & 3)) * p->wstride + (o2 & ~3)) * 2;
            }

    S2Host h;
    stage2_host_tables(p, c->opts.sub_dtype == HD_SUB_I16, h);
    for (const hd_extent& x : h.ext)
        if (x.reach > x.size) {
            const int rc = fail(c, HD_E_INVAL, "hd_plan_create: stage-2 variant %d's DMA reaches byte %lld of a %lld-byte %s "
                                "(internal geometry error)", x.kernel, (long long)x.reach, (long long)x.size,
                                x.region == HD_EXT_SUBBANDS ? "subband block" : "offset table");
            plan_free(p);
            delete p;
            return rc;
        }
    std::vector<int32_t>(&womin)[7] = h.womin;
    std::vector<int32_t>(&wboff)[7] = h.wboff;
    std::vector<int32_t>(&qpb)[3] = h.qpb;
    if (c->device == HD_HOST_ONLY) {   // host tables only (life-cycle tests): nothing on a device
        *out = p;
        return HD_OK;
    }
    int rc = HD_OK;
    hipError_t e = hipSetDevice(c->device);
    for (int k = 0; k < 7 && e == hipSuccess; k++) {
        hd_plan::Wide& w = p->wide[k];
        if (!w.ok) continue;
        e = hipMalloc(&w.d_omin, sizeof(int32_t) * womin[k].size());
        if (e == hipSuccess) e = hipMemcpy(w.d_omin, womin[k].data(), sizeof(int32_t) * womin[k].size(), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMalloc(&w.d_boff, sizeof(int32_t) * wboff[k].size());
        if (e == hipSuccess) e = hipMemcpy(w.d_boff, wboff[k].data(), sizeof(int32_t) * wboff[k].size(), hipMemcpyHostToDevice);
    }
    for (int qi = 0; qi < 3 && e == hipSuccess && p->wide[6].ok; qi++) {
        if (qpb[qi].empty()) continue;
        e = hipMalloc(&p->wide[6].d_boffp[qi], sizeof(int32_t) * qpb[qi].size());
        if (e == hipSuccess)
            e = hipMemcpy(p->wide[6].d_boffp[qi], qpb[qi].data(), sizeof(int32_t) * qpb[qi].size(), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipMalloc(&p->d_idispdt, sizeof(int32_t) * nchan);
    if (e == hipSuccess) e = hipMemcpy(p->d_idispdt, p->idispdt.data(), sizeof(int32_t) * nchan, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_off, sizeof(int32_t) * p->off.size());
    if (e == hipSuccess) e = hipMemcpy(p->d_off, p->off.data(), sizeof(int32_t) * p->off.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_maxabs, sizeof(int32_t));
    if (e == hipSuccess) e = hipMemset(p->d_maxabs, 0, sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&p->d_omin, sizeof(int32_t) * omin.size());
    if (e == hipSuccess) e = hipMemcpy(p->d_omin, omin.data(), sizeof(int32_t) * omin.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_boff, sizeof(int32_t) * boff.size());
    if (e == hipSuccess) e = hipMemcpy(p->d_boff, boff.data(), sizeof(int32_t) * boff.size(), hipMemcpyHostToDevice);
    for (int i = 0; i < 2 && e == hipSuccess; i++) e = hipEventCreate(&p->ev[i]);
    if (e == hipSuccess) {
        p->dd_own = std::make_shared<DdEv>();
        p->dd_cur = p->dd_own;
        for (int i = 0; i < 2 && e == hipSuccess; i++) e = hipEventCreate(&p->dd_own->e[i]);
    }
    if (e != hipSuccess) {
        rc = fail(c, HD_E_HIP, "hd_plan_create: %s", hipGetErrorString(e));
        plan_free(p);
        delete p;
        return rc;
    }
    *out = p;
    return HD_OK;
}

extern "C" int hd_plan_destroy(hd_plan* p)
{
    if (!p) return HD_OK;
    hd_ctx* c = p->ctx;
    if (c->device == HD_HOST_ONLY || c->faulted) {
        // no device call (see hd_close): host state only; device buffers and events stay
        if (p->dd_own) p->dd_own->e[0] = p->dd_own->e[1] = nullptr;
        if (p->dd_cur) p->dd_cur->e[0] = p->dd_cur->e[1] = nullptr;
        delete p->sp;                 // (its buffer set belongs to the context's sp_all)
        if (p->fft && hd::fft_owner(p->fft) == p) hd::fft_set_owner(p->fft, nullptr);
        delete p;
        if (!c->faulted) return HD_OK;
        return fail(c, HD_E_HIP, "hd_plan_destroy: the device faulted earlier (%s); device memory is left to the process exit",
                    c->fault_msg.c_str());
    }
    (void)hipSetDevice(c->device);
    (void)sync_all(c);
    if (p->copy_pending && c->writer) (void)hipEventSynchronize(p->ev_copy);   // copies read p->d_out
    plan_free(p);
    delete p;
    return HD_OK;
}

extern "C" int hd_plan_get_delays(const hd_plan* p, int32_t* chan_delays, int32_t* dm_offsets)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_plan_get_delays: NULL plan");
    if (chan_delays) memcpy(chan_delays, p->idispdt.data(), sizeof(int32_t) * p->idispdt.size());
    if (dm_offsets) memcpy(dm_offsets, p->off.data(), sizeof(int32_t) * p->off.size());
    return HD_OK;
}

extern "C" int hd_plan_sub_params(const hd_plan* p, double* lof, double* cw, double* dt, int64_t* nds)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_plan_sub_params: NULL plan");
    if (lof) *lof = p->sub_lofreq;
    if (cw) *cw = p->sub_chanwid;
    if (dt) *dt = p->sub_dt;
    if (nds) *nds = p->nds;
    return HD_OK;
}

extern "C" int hd_plan_set_variant(hd_plan* p, int32_t v)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_plan_set_variant: NULL plan");
    // bits 0-7: stage-2 variant (0 auto, 1 direct, 2 LDS, 3 wide LDS); bits 8-15: stage-1 (0 auto, 1 direct,
    // 2 float tiled, 3 8-bit integer tiled)
    const int32_t v1 = (v >> 8) & 0xFF;
    p->probe = (v >> 16) & 0xFF;     // profiling only (results invalid): see hipdedisp.h
    p->pair_persist = (v >> 24) & 0x3;   // pair kernel: 0/1 persistent workgroups (default), 2 one per tile
    v &= 0xFF;
    if (v < 0 || v > 9 || v1 > 3) return fail(p->ctx, HD_E_INVAL, "variant must be (s1<<8)|s2 with s1 in 0..3, s2 in 0..9");
    p->s1_variant = v1;
    if (v == 2 && !p->lds_ok) return fail(p->ctx, HD_E_INVAL, "LDS variant unavailable for this plan (needs int16 subbands and a window that fits 64 KiB)");
    if ((v == 3 && !p->wide[0].ok) || (v == 4 && !p->wide[1].ok) || (v == 5 && !p->wide[2].ok) ||
        (v == 6 && !p->wide[3].ok) || (v == 7 && !p->wide[4].ok) || (v == 8 && !p->wide[5].ok) ||
        (v == 9 && !p->wide[6].ok))
        return fail(p->ctx, HD_E_INVAL, "wide-tile variant unavailable for this plan (needs int16 subbands and a window that fits LDS)");
    p->variant = v;
    return HD_OK;
}

static size_t sub_elem(const hd_ctx* c) { return c->opts.sub_dtype == HD_SUB_I16 ? 2 : 4; }

// Each plan owns its subband block (so one launch can form the subbands of many passes).
static int ensure_sub(hd_ctx* c, hd_plan* p)
{
    const size_t need = sub_elem(c) * (size_t)p->pass.nsub * (size_t)p->sub_stride;
    if (p->d_sub && p->sub_bytes >= need) return HD_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dfree(p->d_sub);
    p->d_sub = nullptr;
    p->sub_bytes = 0;
    if (hipMalloc(&p->d_sub, need) != hipSuccess) {
        p->d_sub = nullptr;
        return fail(c, HD_E_NOMEM, "cannot allocate %zu bytes of subbands", need);
    }
    HIPCHK(c, hipMemsetAsync(p->d_sub, 0, need, c->stream));   // the zero tail of every row
    p->sub_bytes = need;
    return HD_OK;
}

static hd::RawDesc raw_desc(const hd_ctx* c)
{
    hd::RawDesc rd{};
    rd.raw = c->d_raw;
    rd.N = c->obs.N;
    rd.rowbytes = c->rowbytes;
    rd.nchan = c->obs.nchan;
    rd.nbits = c->obs.nbits;
    rd.flip = c->obs.flip;
    rd.nibble_hi_first = c->opts.nibble_hi_first;
    rd.be16 = c->opts.be16;
    rd.scl = c->d_scl;
    rd.offs = c->d_offs;
    rd.wts = c->d_wts;
    rd.blk = c->blk;
    rd.nblk = c->nblk;
    rd.blk_shift = (c->blk & (c->blk - 1)) ? -1 : __builtin_ctz((unsigned)c->blk);
    rd.zidx = c->d_zidx;
    rd.zrows = c->d_zrows;
    const bool clip = c->opts.clip_sigma > 0.0f && c->clip_valid;
    const float* cpad = c->slice_total ? c->clip.pad_g + (c->slice_t0 / c->blk) * (int64_t)c->obs.nchan : c->clip.pad;
    rd.pad = clip ? cpad : c->d_padvals;
    rd.pad_stride = clip ? c->obs.nchan : 0;
    rd.clipped = clip ? c->clip.clipped : nullptr;
    rd.clipbits = clip ? c->clip.clipbits : nullptr;
    return rd;
}

// k_stage1_fix8's boundary items, per chunk of G channels: the boundaries bb (read blocks bb-1
// and bb) where some channel of the chunk is zapped in both blocks -- the only ones whose
// outputs the fixup may change (it still checks that the two pads differ).  Built once per G
// from the host copy of the block masks; with a mask the bench beam's ~2,047 boundaries x 96
// chunks shrink to the chunks of its persistently masked channels.
static void fix8_bounds(hd_ctx* c, hd::Stage1Multi& m)
{
    m.fix_blist = m.fix_bofs = nullptr;
    m.fix_G = 0;
    if (!m.rd.zidx || c->h_zidx.empty() || getenv("HD_FIX8_ALLB")) return;
    const int G = hd::fix8_chunk_channels(m);
    const int nchan = c->obs.nchan, nblk = (int)c->h_zidx.size();
    if (G <= 0 || nchan % G) return;
    auto it = c->fixb.find(G);
    if (it == c->fixb.end()) {
        const int nchunk = nchan / G;
        std::vector<int32_t> ofs((size_t)nchunk + 1, 0), list;
        for (int k = 0; k < nchunk; k++) {
            ofs[k] = (int32_t)list.size();
            for (int bb = 1; bb < nblk; bb++) {
                const uint8_t* za = &c->h_zrows[(size_t)c->h_zidx[bb - 1] * nchan + (size_t)k * G];
                const uint8_t* zb = &c->h_zrows[(size_t)c->h_zidx[bb] * nchan + (size_t)k * G];
                for (int i = 0; i < G; i++)
                    if (za[i] && zb[i]) {
                        list.push_back(bb);
                        break;
                    }
            }
        }
        ofs[nchunk] = (int32_t)list.size();
        int32_t *dl = nullptr, *dofs = nullptr;
        if (hipMalloc(&dl, sizeof(int32_t) * std::max<size_t>(list.size(), 1)) != hipSuccess ||
            hipMalloc(&dofs, sizeof(int32_t) * ofs.size()) != hipSuccess ||
            (list.size() && hipMemcpy(dl, list.data(), sizeof(int32_t) * list.size(), hipMemcpyHostToDevice) != hipSuccess) ||
            hipMemcpy(dofs, ofs.data(), sizeof(int32_t) * ofs.size(), hipMemcpyHostToDevice) != hipSuccess) {
            dfree(dl);
            dfree(dofs);
            (void)hipGetLastError();
            return;                      // (every boundary is tried: correct, slower)
        }
        it = c->fixb.emplace(G, std::make_pair(dl, dofs)).first;
    }
    m.fix_blist = it->second.first;
    m.fix_bofs = it->second.second;
    m.fix_G = G;
}

// check_mask per read block [PRESTO-ext, mask.c]: block b spans [b*blk*dt, b*blk*dt +
// blk*dt); its zapped channels are the union of the lists of the intervals holding its
// start and end time (clamped to the last interval), or all channels when either is a
// zap_int.  Identical rows are uploaded once (zidx -> zrows).
static int ensure_blocks(hd_ctx* c)
{
    if (c->blocks_valid) return HD_OK;
    free_blocks(c);
    const int nchan = c->obs.nchan, nblk = c->nblk;
    const int64_t g0 = c->slice_t0 / c->blk;          // global index of local block 0 (time slices)
    std::vector<uint8_t> allzap((size_t)nblk, 0);
    if (c->slice_total && !c->h_mask.empty()) {
        // the clip recurrence of a slice walks every block of the observation before it
        std::vector<uint8_t> ag((size_t)(g0 + nblk), 0);
        for (int64_t b = 0; b < g0 + nblk; b++) {
            const double st = (double)(b * c->blk) * c->obs.dt, en = st + c->blk * c->obs.dt;
            const int lo = std::min((int)(st / c->dtint), c->numint - 1);
            const int hi = std::min((int)(en / c->dtint), c->numint - 1);
            ag[(size_t)b] = c->h_zapint[lo] || c->h_zapint[hi];
        }
        dfree(c->clip.allzap_g);
        c->clip.allzap_g = nullptr;
        HIPCHK(c, hipMalloc(&c->clip.allzap_g, ag.size()));
        HIPCHK(c, hipMemcpy(c->clip.allzap_g, ag.data(), ag.size(), hipMemcpyHostToDevice));
    }
    if (!c->h_mask.empty()) {
        std::vector<int32_t> zidx((size_t)nblk);
        std::vector<uint8_t> rows;
        std::map<int64_t, int32_t> seen;     // (lo, hi) or all -> row
        const double duration = c->blk * c->obs.dt;
        for (int32_t b = 0; b < nblk; b++) {
            const double starttime = (double)((g0 + b) * c->blk) * c->obs.dt;
            const double endtime = starttime + duration;
            const int lo = std::min((int)(starttime / c->dtint), c->numint - 1);
            const int hi = std::min((int)(endtime / c->dtint), c->numint - 1);
            const bool all = c->h_zapint[lo] || c->h_zapint[hi];
            allzap[b] = all;
            const int64_t key = all ? -1 : (int64_t)lo * c->numint + hi;
            auto it = seen.find(key);
            if (it != seen.end()) {
                zidx[b] = it->second;
                continue;
            }
            const int32_t r = (int32_t)seen.size();
            seen[key] = r;
            zidx[b] = r;
            rows.resize((size_t)(r + 1) * nchan);
            uint8_t* dst = &rows[(size_t)r * nchan];
            for (int ch = 0; ch < nchan; ch++)
                dst[ch] = all || c->h_mask[(size_t)lo * nchan + ch] || c->h_mask[(size_t)hi * nchan + ch];
        }
        c->h_zidx = zidx;
        c->h_zrows = rows;
        HIPCHK(c, hipMalloc(&c->d_zidx, sizeof(int32_t) * zidx.size()));
        HIPCHK(c, hipMemcpy(c->d_zidx, zidx.data(), sizeof(int32_t) * zidx.size(), hipMemcpyHostToDevice));
        HIPCHK(c, hipMalloc(&c->d_zrows, rows.size()));
        HIPCHK(c, hipMemcpy(c->d_zrows, rows.data(), rows.size(), hipMemcpyHostToDevice));
    }
    HIPCHK(c, hipMalloc(&c->d_allzap, allzap.size()));
    HIPCHK(c, hipMemcpy(c->d_allzap, allzap.data(), allzap.size(), hipMemcpyHostToDevice));
    c->blocks_valid = true;
    c->clip_valid = false;
    c->clip.stats_valid = false;
    return HD_OK;
}

// clip_times over the raw block (hd_clip.hip), queued on the context stream; its device
// time is charged to the stage-1 launch that needs it.
static int alloc_clip(hd_ctx* c);
static hd::ClipArgs clip_args(hd_ctx* c);

static int ensure_clip(hd_ctx* c, hipEvent_t after_stats = nullptr)
{
    if (!(c->opts.clip_sigma > 0.0f) || c->clip_valid) return HD_OK;
    if (c->slice_total)
        return fail(c, HD_E_STATE, "time-sliced context: clip_times needs the observation's per-block statistics "
                    "(hd_clip_stats on every slice, then hd_clip_set_stats) before stage 1");
    int rc = alloc_clip(c);
    if (rc) return rc;
    HIPCHK(c, hd::launch_clip(clip_args(c), c->stream, after_stats));
    c->clip_valid = true;
    return HD_OK;
}

static int alloc_clip(hd_ctx* c)
{
    int rc = ensure_blocks(c);
    if (rc) return rc;
    hd_ctx::ClipBufs& b = c->clip;
    const size_t N = (size_t)c->obs.N, nb = (size_t)c->nblk, nch = (size_t)c->obs.nchan;
    if (!b.zdm) {
        hipError_t e = hipSuccess;
        auto al = [&](void** p, size_t bytes) {
            if (e == hipSuccess) e = hipMalloc(p, bytes);
        };
        al((void**)&b.zdm, N * 4);
        al((void**)&b.good, N);
        al((void**)&b.clipped, N);
        al((void**)&b.clipbits, (N + 63) / 64 * 8);
        al((void**)&b.events, N * 4);
        al((void**)&b.nevents, 4);
        al((void**)&b.nzero, 4);
        al((void**)&b.numgood, nb * 4);
        al((void**)&b.doclip, nb * 4);
        al((void**)&b.bavg, nb * 8);
        al((void**)&b.bstd, nb * 8);
        al((void**)&b.ravg, nb * 4);
        al((void**)&b.trig, nb * 4);
        al((void**)&b.chansum, nb * nch * 8);
        al((void**)&b.pad, nb * nch * 4);
        if (e != hipSuccess) {
            free_clip(c);
            return fail(c, HD_E_NOMEM, "cannot allocate the clip_times state: %s", hipGetErrorString(e));
        }
        HIPCHK(c, hipMemset(b.nzero, 0, 4));
    }
    if (c->slice_total && !b.numgood_g) {
        const size_t ng = (size_t)(c->slice_t0 / c->blk + c->nblk);
        hipError_t e = hipSuccess;
        auto al = [&](void** p, size_t bytes) {
            if (e == hipSuccess) e = hipMalloc(p, bytes);
        };
        al((void**)&b.numgood_g, ng * 4);
        al((void**)&b.doclip_g, ng * 4);
        al((void**)&b.bavg_g, ng * 8);
        al((void**)&b.bstd_g, ng * 8);
        al((void**)&b.ravg_g, ng * 4);
        al((void**)&b.trig_g, ng * 4);
        al((void**)&b.chansum_g, ng * nch * 8);
        al((void**)&b.pad_g, ng * nch * 4);
        al((void**)&b.xbuf, ng * (nch + 3) * 8);
        if (e != hipSuccess) {
            free_clip(c);
            return fail(c, HD_E_NOMEM, "cannot allocate the sliced clip_times state: %s", hipGetErrorString(e));
        }
    }
    return HD_OK;
}

// the context's own (local) clip arguments
static hd::ClipArgs clip_args(hd_ctx* c)
{
    hd_ctx::ClipBufs& b = c->clip;
    hd::ClipArgs a{};
    a.rd = raw_desc(c);
    a.clip_sigma = c->opts.clip_sigma;
    a.allzap = c->d_allzap;
    a.padvals0 = c->d_padvals;
    a.zdm = b.zdm;
    a.good = b.good;
    a.numgood = b.numgood;
    a.bavg = b.bavg;
    a.bstd = b.bstd;
    a.chansum = b.chansum;
    a.ravg = b.ravg;
    a.trig = b.trig;
    a.doclip = b.doclip;
    a.clipped = b.clipped;
    a.clipbits = b.clipbits;
    a.pad = b.pad;
    a.events = b.events;
    a.nevents = b.nevents;
    return a;
}

// ---- time-sliced contexts: clip_times across slices ----------------------------------
extern "C" int hd_clip_stats(hd_ctx* c, int64_t nown, double* stats)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_clip_stats: NULL context");
    if (!c->slice_total) return fail(c, HD_E_STATE, "hd_clip_stats: the context is not a time slice (hd_set_slice)");
    if (!(c->opts.clip_sigma > 0.0f)) return HD_OK;
    if (!c->raw_ready) return fail(c, HD_E_STATE, "hd_clip_stats: no raw data");
    if (nown < 0 || nown > c->nblk || !stats) return fail(c, HD_E_INVAL, "hd_clip_stats: nown must be in [0, %d]", c->nblk);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, join_stream2(c));
    int rc = alloc_clip(c);
    if (rc) return rc;
    hd::ClipArgs a = clip_args(c);
    if (!c->clip.stats_valid) {
        HIPCHK(c, hd::launch_clip_stats(a, c->stream));
        c->clip.stats_valid = true;
    }
    const size_t w = (size_t)c->obs.nchan + 3;
    HIPCHK(c, hd::launch_clip_pack(a, c->clip.xbuf, (int)nown, c->stream));
    // on the context stream, then a wait: a device-to-device hipMemcpy on the null stream may
    // return before it lands and is not ordered with this non-blocking stream -- with a device
    // table (hd_slice_exchange_clip) the all-reduce and hd_clip_set_stats's copy then raced it
    // and read partly unwritten rows (bench --comm hd: mass clipping, 4 s per beam)
    HIPCHK(c, hipMemcpyAsync(stats + (size_t)(c->slice_t0 / c->blk) * w, c->clip.xbuf, (size_t)nown * w * 8,
                             hipMemcpyDefault, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return HD_OK;
}

extern "C" int hd_clip_set_stats(hd_ctx* c, const double* stats)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_clip_set_stats: NULL context");
    if (!c->slice_total) return fail(c, HD_E_STATE, "hd_clip_set_stats: the context is not a time slice");
    if (!(c->opts.clip_sigma > 0.0f)) return HD_OK;
    if (!c->raw_ready) return fail(c, HD_E_STATE, "hd_clip_set_stats: no raw data");
    if (!stats) return fail(c, HD_E_INVAL, "hd_clip_set_stats: stats is NULL");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, join_stream2(c));
    int rc = alloc_clip(c);
    if (rc) return rc;
    hd_ctx::ClipBufs& b = c->clip;
    const int64_t g0 = c->slice_t0 / c->blk, ng = g0 + c->nblk, nch = c->obs.nchan;
    const size_t w = (size_t)nch + 3;
    hd::ClipArgs a = clip_args(c);
    if (!b.stats_valid) {                       // this slice's own zero-DM series and good flags
        HIPCHK(c, hd::launch_clip_stats(a, c->stream));
        b.stats_valid = true;
    }
    HIPCHK(c, hipMemcpyAsync(b.xbuf, stats, (size_t)ng * w * 8, hipMemcpyDefault, c->stream));
    hd::ClipArgs g = a;                         // the observation's blocks [0, ng)
    g.rd.nblk = (int32_t)ng;
    g.numgood = b.numgood_g;
    g.bavg = b.bavg_g;
    g.bstd = b.bstd_g;
    g.chansum = b.chansum_g;
    g.allzap = c->h_mask.empty() ? nullptr : b.allzap_g;
    g.doclip = b.doclip_g;
    g.ravg = b.ravg_g;
    g.trig = b.trig_g;
    g.pad = b.pad_g;
    HIPCHK(c, hd::launch_clip_unpack(g, b.xbuf, c->stream));
    HIPCHK(c, hd::launch_clip_recur(g, c->stream));
    a.doclip = b.doclip_g + g0;                 // this slice's spectra against its blocks' state
    a.ravg = b.ravg_g + g0;
    a.trig = b.trig_g + g0;
    HIPCHK(c, hd::launch_clip_flag(a, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->clip_valid = true;
    return HD_OK;
}

extern "C" int hd_get_clean(hd_ctx* c, float* pad, uint8_t* clipped, uint8_t* zap, int64_t* nclipped)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_get_clean: NULL context");
    if (!c->have_obs) return fail(c, HD_E_STATE, "hd_get_clean before hd_set_obs");
    const bool clip = c->opts.clip_sigma > 0.0f;
    if (clip && !c->raw_ready) return fail(c, HD_E_STATE, "hd_get_clean: no raw data");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, join_stream2(c));
    int rc = ensure_blocks(c);
    if (rc) return rc;
    if ((rc = ensure_clip(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const size_t nb = (size_t)c->nblk, nch = (size_t)c->obs.nchan;
    if (pad) {
        if (clip) {
            const float* src = c->slice_total ? c->clip.pad_g + (c->slice_t0 / c->blk) * nch : c->clip.pad;
            HIPCHK(c, hipMemcpy(pad, src, nb * nch * 4, hipMemcpyDeviceToHost));
        } else {
            for (size_t b = 0; b < nb; b++)
                for (size_t ch = 0; ch < nch; ch++) pad[b * nch + ch] = c->h_padvals.empty() ? 0.0f : c->h_padvals[ch];
        }
    }
    if (clipped) {
        if (clip) HIPCHK(c, hipMemcpy(clipped, c->clip.clipped, (size_t)c->obs.N, hipMemcpyDeviceToHost));
        else memset(clipped, 0, (size_t)c->obs.N);
    }
    if (zap) {
        if (c->d_zidx) {
            std::vector<int32_t> zidx(nb);
            HIPCHK(c, hipMemcpy(zidx.data(), c->d_zidx, nb * 4, hipMemcpyDeviceToHost));
            int32_t nrow = 0;
            for (int32_t v : zidx) nrow = std::max(nrow, v + 1);
            std::vector<uint8_t> rows((size_t)nrow * nch);
            HIPCHK(c, hipMemcpy(rows.data(), c->d_zrows, rows.size(), hipMemcpyDeviceToHost));
            for (size_t b = 0; b < nb; b++) memcpy(zap + b * nch, &rows[(size_t)zidx[b] * nch], nch);
        } else {
            memset(zap, 0, nb * nch);
        }
    }
    if (nclipped) {
        int32_t n = 0;
        if (clip) HIPCHK(c, hipMemcpy(&n, c->clip.nevents, 4, hipMemcpyDeviceToHost));
        *nclipped = n;
    }
    return HD_OK;
}

// Tiling of the multi-pass stage-1 kernel: sg subbands per workgroup (64*sg threads),
// `to` outputs per tile, within an LDS budget (64 KiB when that still gives long tiles,
// up to 160 KiB for strongly downsampled / high-DM passes).
static bool stage1_tiling(const hd_ctx* c, int nsub, int ds, int dmax, hd::Stage1Multi& a, int& vw)
{
    const int nbits = c->obs.nbits, nchan = c->obs.nchan, cps = nchan / nsub;
    if (c->rowbytes % 4 || !hd::stage1_tiled_supports_cps(cps)) return false;
    int sg = 0;
    // HD_S1T_SG / HD_S1T_KB (profiling): at most this many subbands per workgroup / the first
    // LDS budget (KiB) tried
    const int sgcap = getenv("HD_S1T_SG") ? atoi(getenv("HD_S1T_SG")) : 8;
    const size_t kb0 = getenv("HD_S1T_KB") ? (size_t)atoi(getenv("HD_S1T_KB")) : 64;
    for (int cand : {8, 4, 2, 1})
        if (cand <= sgcap && nsub % cand == 0 && ((int64_t)cand * cps * nbits) % 32 == 0) { sg = cand; break; }
    if (!sg) return false;
    const int G = sg * cps;
    const int gbytes = G * nbits / 8;
    vw = 4;
    for (int cand : {16}) {
        // every group's byte offset (g*G or nchan-(g+1)*G channels) and the row pitch must align
        if (gbytes % cand == 0 && c->rowbytes % cand == 0 && ((int64_t)nchan * nbits / 8) % cand == 0) { vw = cand; break; }
    }
    int rs = (gbytes + 3) & ~3;
    if (((rs / 4) & 1) == 0) rs += 4;
    int to = 0;
    for (size_t budget : {kb0 * 1024, (size_t)96 * 1024, (size_t)156 * 1024}) {
        if (budget < kb0 * 1024) continue;
        const int64_t rows_max = (int64_t)((budget - 64) / (size_t)(rs + 4));
        to = (int)std::min<int64_t>(2048, (rows_max - dmax) / ds);
        if (to >= 256) break;
    }
    if (to < 32) return false;
    a.sg = sg;
    a.to = to;
    a.rs = rs;
    a.dmax = dmax;
    a.ngroups = nsub / sg;
    return true;
}

// Float tiled kernel over tiles of a fixed `to` (the 8-bit integer path's special tiles):
// the widest channel group whose LDS tile fits 160 KiB.
static bool stage1_tiling_fixed(const hd_ctx* c, int nsub, int ds, int dmax, int to, hd::Stage1Multi& a, int& vw)
{
    const int nbits = c->obs.nbits, nchan = c->obs.nchan, cps = nchan / nsub;
    if (c->rowbytes % 4 || !hd::stage1_tiled_supports_cps(cps)) return false;
    for (int cand : {8, 4, 2, 1}) {
        if (nsub % cand || ((int64_t)cand * cps * nbits) % 32) continue;
        const int gbytes = cand * cps * nbits / 8;
        int rs = (gbytes + 3) & ~3;
        if (((rs / 4) & 1) == 0) rs += 4;
        hd::Stage1Multi t = a;
        t.sg = cand;
        t.to = to;
        t.rs = rs;
        t.ds = ds;
        t.dmax = dmax;
        if (hd::stage1_tiled_lds_bytes(t) > 160 * 1024) continue;
        vw = (gbytes % 16 == 0 && c->rowbytes % 16 == 0) ? 16 : 4;
        a.sg = cand;
        a.rs = rs;
        a.ngroups = nsub / cand;
        return true;
    }
    return false;
}

// 8-bit integer path (k_stage1_q8): sg subbands per workgroup, quarter geometry fixed by ds;
// the first sg in {4, 2, 1} whose LDS tile fits 64 KiB (two or more workgroups per CU),
// else the smallest tile that fits 160 KiB.
static bool stage1_q8_tiling(const hd_ctx* c, int nsub, int ds, int dmax, hd::Stage1Multi& a, int& vb)
{
    const int nchan = c->obs.nchan, cps = nchan / nsub;
    // 8-bit data, or 4-bit data through its unpacked channel-major copy (the fill then never
    // reads the packed rows)
    if ((c->obs.nbits != 8 && c->obs.nbits != 4) || c->d_scl || c->d_offs || c->d_wts) return false;
    if (!hd::stage1_q8_supports(cps, ds)) return false;
    const int S = hd::stage1_q8_quarter_rows(ds);
    const int W = S + ((dmax + 15) & ~15);            // whole 16-row fill units (16-byte LDS stores)
    int sg = 0, v = 0;
    size_t best = 0;
    // HD_Q8_SG_CAP (profiling): at most this many subbands per workgroup
    const int sgcap = getenv("HD_Q8_SG_CAP") ? atoi(getenv("HD_Q8_SG_CAP")) : 4;
    for (int cand : {4, 2, 1}) {
        if (nsub % cand || (cand > sgcap && cand > 1)) continue;
        const int G = cand * cps;
        const int cv = (G % 8 == 0 && nchan % 8 == 0) ? 8 : (G % 4 == 0 && nchan % 4 == 0) ? 4 : 0;
        if (!cv) continue;
        const size_t lds = (size_t)G * W * 4;
        if (lds > 160 * 1024) continue;
        // the most subbands whose tile leaves room for 3 workgroups per CU: at ds 2 the
        // 4-subband tile (56 KiB, 2 per CU) measured 5.19 ms per 12-pass launch against 4.30 at
        // 2 subbands; at ds 1 and 3 (48 KiB, 3 per CU) 4 subbands stay faster (8.06 vs 8.26,
        // 2.60 vs 3.45 ms; HD_Q8_SG_CAP=2, scripts/ab_bench.sh)
        if (3 * lds <= 160 * 1024) {
            sg = cand;
            v = cv;
            break;
        }
        if (!sg || lds < best) {
            sg = cand;
            v = cv;
            best = lds;
        }
    }
    if (!sg) return false;
    a.sg = sg;
    a.to = 4 * S / ds;
    a.dmax = dmax;
    a.W = W;
    a.rs = 0;
    a.two_ok = ds >= 10 ? 2 : 1;                      // read blocks past the first a tile may span
    // bound on the rounding of the oracle's float fold (CPS channel adds per ds step, then
    // ds adds of the steps) for sums of 8-bit samples and pad values: each add errs by at most
    // half an ulp of its result; ulps are over-estimated 2x by taking 2^(floor(log2 x) - 22)
    {
        double maxpad = 255.0;
        for (float v : c->h_padvals) maxpad = std::max(maxpad, (double)fabsf(v));
        const double smax = cps * maxpad, amax = ds * smax;
        auto ulp2 = [](double x) { return ldexp(1.0, (int)floor(log2(x)) - 22); };
        a.tie_eps = ds * cps * 0.5 * ulp2(smax) + ds * 0.5 * ulp2(amax);
        // mean mode: x = fl(F / ds) errs by half an ulp of F/ds, i.e. ds/2 ulps in C's units
        if (c->opts.ds_mode == HD_DS_MEAN) a.tie_eps += ds * 0.5 * ulp2(smax);
    }
    a.ngroups = nsub / sg;
    vb = v;
    return true;
}

// Host-built list of a launch's special tiles (last tile / interval-straddling), on device.
// The list depends only on the tile geometry and the mask, so it is built and uploaded once
// per geometry (synchronous copy) and cached on the context until the mask or obs change.
static int special_tiles(hd_ctx* c, const hd::Stage1Multi& m, int** d_sp, int* nsp_out)
{
    *d_sp = nullptr;
    *nsp_out = 0;
    for (const auto& e : c->special_cache)
        if (e.to == m.to && e.ds == m.ds && e.dmax == m.dmax && e.ntiles == m.ntiles && e.two_ok == m.two_ok) {
            *d_sp = e.d;
            *nsp_out = e.n;
            return HD_OK;
        }
    const int nsp = hd::stage1_special_tiles(m, nullptr);
    hd_ctx::SpecialList e{m.to, m.ds, m.dmax, m.ntiles, m.two_ok, nsp, nullptr};
    if (nsp) {
        std::vector<int> h(nsp);
        hd::stage1_special_tiles(m, h.data());
        HIPCHK(c, hipMalloc(&e.d, sizeof(int) * nsp));
        HIPCHK(c, hipMemcpy(e.d, h.data(), sizeof(int) * nsp, hipMemcpyHostToDevice));
    }
    c->special_cache.push_back(e);
    *d_sp = e.d;
    *nsp_out = nsp;
    return HD_OK;
}

// The same list cut into q sub-tiles per tile (tile t -> t q .. t q + q - 1: ALL of them, since
// the integer kernel skipped the whole tile), for a float launch of to / q outputs per tile:
// q times the workgroups on a q-th of the rows each (the few special tiles' float folds are
// latency-bound).  Cached beside the plain lists (key: to < 0).
static int special_subtiles(hd_ctx* c, const hd::Stage1Multi& m, int q, int** d_sp, int* nsp_out)
{
    *d_sp = nullptr;
    *nsp_out = 0;
    const int key = -(m.to / q);
    for (const auto& e : c->special_cache)
        if (e.to == key && e.ds == m.ds && e.dmax == m.dmax && e.ntiles == m.ntiles * q && e.two_ok == m.two_ok) {
            *d_sp = e.d;
            *nsp_out = e.n;
            return HD_OK;
        }
    const int nsp = hd::stage1_special_tiles(m, nullptr);
    std::vector<int> h(nsp), sub;
    if (nsp) hd::stage1_special_tiles(m, h.data());
    const int64_t rows_sub = (int64_t)(m.to / q) * m.ds;
    for (int t : h)
        for (int k = 0; k < q; k++)
            if ((int64_t)(t * q + k) * rows_sub < c->obs.N) sub.push_back(t * q + k);   // (rows past N: no output)
    hd_ctx::SpecialList e{key, m.ds, m.dmax, m.ntiles * q, m.two_ok, (int)sub.size(), nullptr};
    if (!sub.empty()) {
        HIPCHK(c, hipMalloc(&e.d, sizeof(int) * sub.size()));
        HIPCHK(c, hipMemcpy(e.d, sub.data(), sizeof(int) * sub.size(), hipMemcpyHostToDevice));
    }
    c->special_cache.push_back(e);
    *d_sp = e.d;
    *nsp_out = e.n;
    return HD_OK;
}

static void clear_special_cache(hd_ctx* c)
{
    if (!c->special_cache.empty()) (void)hipStreamSynchronize(c->stream);
    for (auto& e : c->special_cache) dfree(e.d);
    c->special_cache.clear();
}

static int run_subband_chunk(hd_ctx* c, hd_plan** plans, int n)
{
    hd_plan* p0 = plans[0];
    int dmax = 0;
    for (int i = 0; i < n; i++) dmax = std::max(dmax, plans[i]->maxdelay);
    hd::Stage1Multi m{};
    int vw = 4, vb = 4;
    const int v1 = p0->s1_variant;
    const bool q8 = (v1 == 0 || v1 == 3) && stage1_q8_tiling(c, p0->pass.nsub, p0->pass.ds, dmax, m, vb) &&
                    (c->obs.nbits == 8 || (!(p0->probe & 4) && alloc_rawT(c, dmax)));
    if (v1 == 3 && !q8)
        return fail(c, HD_E_INVAL, "stage-1 variant 3 (8-bit integer path) does not apply to this pass");
    const bool tiled = !q8 && (v1 == 0 || v1 == 2) && stage1_tiling(c, p0->pass.nsub, p0->pass.ds, dmax, m, vw);
    int rc0 = ensure_blocks(c);
    if (rc0) return rc0;
    {
        hd::ZeroList z{};
        for (int i = 0; i < n; i++) z.p[i] = plans[i]->d_maxabs;
        HIPCHK(c, hd::launch_zero_list(z, n, c->stream));
    }
    HIPCHK(c, hipEventRecord(p0->ev[0], c->stream));
    // the channel-major copy (once per raw block) on saux, beside clip_times' serial 30-block
    // recurrence (one workgroup): forked after clip_times' full-chip statistics kernels, or
    // now when there is no clipping to run
    const bool want_rawT = q8 && !(p0->probe & 4);   // probe bit 2: row-major fill
    const bool clip_runs = c->opts.clip_sigma > 0.0f && !c->clip_valid;
    const bool fork_clip = want_rawT && clip_runs && !c->rawT_valid && alloc_rawT(c, dmax);
    const uint8_t* rawT = want_rawT && !fork_clip ? ensure_rawT(c, dmax, true) : nullptr;
    rc0 = ensure_clip(c, fork_clip ? c->ev_aux0 : nullptr);   // once per raw block, charged to this launch
    if (fork_clip && !rc0) rawT = ensure_rawT(c, dmax, true, true);
    const hipError_t ej = join_aux(c);               // (also on failure: nothing may outlive the call)
    if (rc0) return rc0;
    HIPCHK(c, ej);
    const bool clip = c->opts.clip_sigma > 0.0f;
    if (q8) {
        m.probe = p0->probe;
        // clipped-spectrum and block-boundary outputs: the separate fixup kernel (k_stage1_fix8)
        // by default; HD_QFIX=1 in the environment recomputes them inside k_stage1_q8 instead
        // (measured 36.5 vs 34.4 ms of stage 1 per C2 beam: the in-kernel fixup's store drain and
        // barrier cost every tile, and nearly every tile holds a clipped spectrum; probe bits
        // 5-7 also select the separate kernels)
        const bool env_qfix = getenv("HD_QFIX") && atoi(getenv("HD_QFIX")) != 0;
        m.qfix = clip && env_qfix && !(p0->probe & (32 | 64 | 128)) ? 1 : 0;
        // HD_Q8_WPS2=1: 8-wave blocks at sg = 4, two waves per subband splitting the passes
        m.wps2 = getenv("HD_Q8_WPS2") && atoi(getenv("HD_Q8_WPS2")) != 0 && !m.qfix ? 1 : 0;
        m.rd = raw_desc(c);
        m.rawT = rawT;
        if (!m.rawT && c->obs.nbits != 8) return fail(c, HD_E_HIP, "stage 1: 4-bit channel-major copy failed");
        m.tstride = c->rawT_stride;
        m.npass = n;
        m.nsub = p0->pass.nsub;
        m.cps = c->obs.nchan / p0->pass.nsub;
        m.ds = p0->pass.ds;
        m.ds_mode = c->opts.ds_mode;
        m.sub_dtype = c->opts.sub_dtype;
        m.sub_round = c->opts.sub_round;
        m.nds = p0->nds;
        m.out_stride = p0->sub_stride;
        m.ntiles = (int)((p0->nds + m.to - 1) / m.to);
        for (int i = 0; i < n; i++) {
            m.dly[i] = plans[i]->d_idispdt;
            m.out[i] = plans[i]->d_sub;
            m.maxabs[i] = plans[i]->d_maxabs;
            m.ostride[i] = plans[i]->sub_stride;
        }
        int nsp = 0, *d_sp = nullptr;
        int rc = special_tiles(c, m, &d_sp, &nsp);
        if (rc) return rc;
        const size_t lds = hd::stage1_q8_lds_bytes(m);
        if (lds > c->lds_attr_q8) {
            HIPCHK(c, hd::stage1_q8_set_lds_limit(lds));
            c->lds_attr_q8 = lds;
        }
        HIPCHK(c, hd::launch_stage1_q8(m, vb, c->stream));
        if (nsp) {
            hd::Stage1Multi f = m;
            int fvw = 4;
            if (!stage1_tiling_fixed(c, m.nsub, m.ds, dmax, m.to, f, fvw))
                return fail(c, HD_E_INVAL, "stage 1: no float tiling for the integer path's special tiles");
            const size_t flds = hd::stage1_tiled_lds_bytes(f);
            if (flds > c->lds_attr_set) {
                HIPCHK(c, hd::stage1_tiled_set_lds_limit(flds));
                c->lds_attr_set = flds;
            }
            HIPCHK(c, hd::launch_stage1_tiled(f, fvw, d_sp, nsp, true, c->stream));
        }
        // clipped spectra, and the block-boundary outputs of the per-block pad constants, when
        // k_stage1_q8 did not redo them itself (probe bits 5/6 skip the boundary /
        // clipped-spectrum items: profiling only)
        if (m.qfix) {
        } else if (clip && !(p0->probe & 64)) {
            fix8_bounds(c, m);
            HIPCHK(c, hd::launch_stage1_fixup(m, c->clip.events, c->clip.nevents,
                                              m.rd.zidx != nullptr && !(p0->probe & 32), c->stream));
        } else if (clip && !(p0->probe & 32) && m.rd.zidx) {
            fix8_bounds(c, m);
            HIPCHK(c, hd::launch_stage1_fixup(m, c->clip.events, c->clip.nzero, 1, c->stream));
        }
    } else if (tiled) {
        m.rd = raw_desc(c);
        m.npass = n;
        m.nsub = p0->pass.nsub;
        m.cps = c->obs.nchan / p0->pass.nsub;
        m.ds = p0->pass.ds;
        m.ds_mode = c->opts.ds_mode;
        m.sub_dtype = c->opts.sub_dtype;
        m.sub_round = c->opts.sub_round;
        m.nds = p0->nds;
        m.out_stride = p0->sub_stride;
        // tiles over two read blocks stay in the main launch (per-row pads and zap bits of
        // the two blocks, kModeTwo); only tiles over three or more take the special launch
        // (HD_S1_TWO=0: every block-straddling tile special, as before)
        m.two_ok = getenv("HD_S1_TWO") && atoi(getenv("HD_S1_TWO")) == 0 ? 0 : 1;
        m.ntiles = (int)((p0->nds + m.to - 1) / m.to);
        for (int i = 0; i < n; i++) {
            m.dly[i] = plans[i]->d_idispdt;
            m.out[i] = plans[i]->d_sub;
            m.maxabs[i] = plans[i]->d_maxabs;
            m.ostride[i] = plans[i]->sub_stride;
        }
        const size_t lds = hd::stage1_tiled_lds_bytes(m);
        if (lds > c->lds_attr_set) {
            HIPCHK(c, hd::stage1_tiled_set_lds_limit(lds));
            c->lds_attr_set = lds;
        }
        int nsp = 0, *d_sp = nullptr;
        int rc = special_tiles(c, m, &d_sp, &nsp);
        if (rc) return rc;
        HIPCHK(c, hd::launch_stage1_tiled(m, vw, d_sp, nsp, false, c->stream));
        if (clip) HIPCHK(c, hd::launch_stage1_fixup(m, c->clip.events, c->clip.nevents, 0, c->stream));
    } else {   // one thread per subband sample, every cleaning rule per cell (no fixup needed)
        for (int i = 0; i < n; i++) {
            hd_plan* p = plans[i];
            hd::Stage1Args a{};
            a.rd = raw_desc(c);
            a.idispdt = p->d_idispdt;
            a.nsub = p->pass.nsub;
            a.cps = c->obs.nchan / p->pass.nsub;
            a.ds = p->pass.ds;
            a.ds_mode = c->opts.ds_mode;
            a.sub_dtype = c->opts.sub_dtype;
            a.sub_round = c->opts.sub_round;
            a.maxdelay = p->maxdelay;
            a.nds = p->nds;
            a.out_stride = p->sub_stride;
            a.out = p->d_sub;
            a.maxabs = p->d_maxabs;
            HIPCHK(c, hd::launch_stage1_direct(a, c->stream));
        }
    }
    HIPCHK(c, hipEventRecord(p0->ev[1], c->stream));
    for (int i = 0; i < n; i++) {
        plans[i]->sub_valid = true;
        plans[i]->sub_bound = stage1_sub_bound(c, plans[i]);
        plans[i]->sub_nonneg = plans[i]->sub_bound >= 0 && stage1_sub_nonneg(c);
        plans[i]->ran_sub = (i == 0);   // the launch's time is attributed to its first plan
    }
    return HD_OK;
}

// tie_eps of the 8-bit integer path at downsampling ds (stage1_q8_tiling's bound)
static double q8_tie_eps(const hd_ctx* c, int cps, int ds)
{
    double maxpad = 255.0;
    for (float v : c->h_padvals) maxpad = std::max(maxpad, (double)fabsf(v));
    const double smax = cps * maxpad, amax = ds * smax;
    auto ulp2 = [](double x) { return ldexp(1.0, (int)floor(log2(x)) - 22); };
    double e = ds * cps * 0.5 * ulp2(smax) + ds * 0.5 * ulp2(amax);
    if (c->opts.ds_mode == HD_DS_MEAN) e += ds * 0.5 * ulp2(smax);
    return e;
}

// Whether these plans (several DDplan stages, ds >= 2) can share one k_stage1_q8m launch.
static bool q8m_ok(const hd_ctx* c, hd_plan* const* plans, int n)
{
    if (n < 2 || n > hd::kMaxPass || (getenv("HD_Q8M") && atoi(getenv("HD_Q8M")) == 0)) return false;
    if ((c->obs.nbits != 8 && c->obs.nbits != 4) || c->d_scl || c->d_offs || c->d_wts) return false;
    if (getenv("HD_QFIX") && atoi(getenv("HD_QFIX")) != 0) return false;
    const int nsub = plans[0]->pass.nsub, cps = c->obs.nchan / nsub;
    int nds = 0, ds0 = plans[0]->pass.ds;
    for (int i = 0; i < n; i++) {
        const hd_plan* p = plans[i];
        if (p->pass.nsub != nsub || (p->s1_variant != 0 && p->s1_variant != 3)) return false;
        if (p->probe && (i > 0 || (p->probe & ~(1 | 2 | 4 | 8 | 32 | 64)))) return false;   // q8m's probe bits, on plans[0]
        if (!hd::stage1_q8m_supports_ds(p->pass.ds) || !hd::stage1_q8_supports(cps, p->pass.ds)) return false;
        if (p->pass.ds != ds0) nds = 1;
    }
    return nds > 0 && (cps == 8 || cps == 10 || cps == 16);
}

// Stage 1 of several DDplan stages in one launch (k_stage1_q8m), then per stage its special
// tiles (float kernel) and fixups, as run_subband_chunk does for one stage.  Returns 1 when
// the fused tile does not fit (the caller then runs the stages one by one).
static int run_subband_fused(hd_ctx* c, hd_plan** plans, int n)
{
    hd_plan* p0 = plans[0];
    const int nsub = p0->pass.nsub, cps = c->obs.nchan / nsub;
    int dmax = 0;
    for (int i = 0; i < n; i++) dmax = std::max(dmax, plans[i]->maxdelay);
    const int S = hd::stage1_q8m_quarter_rows();
    hd::Stage1Multi m{};
    m.sg = 1;
    m.W = S + ((dmax + 15) & ~15);
    m.cps = cps;
    if (hd::stage1_q8m_lds_bytes(m) > 160 * 1024) return 1;     // 1: does not apply (per-stage launches)
    // every DDplan stage's special tiles need a float tiling; check them all before anything
    // is launched, so a miss falls back to the per-stage launches with nothing half-formed
    for (int i0 = 0; i0 < n;) {
        int i1 = i0;
        while (i1 < n && plans[i1]->pass.ds == plans[i0]->pass.ds) i1++;
        const int ds = plans[i0]->pass.ds;
        hd::Stage1Multi t{};
        int tvw = 4;
        if (!stage1_tiling_fixed(c, nsub, ds, dmax, 4 * S / ds, t, tvw)) return 1;
        i0 = i1;
    }
    if (!alloc_rawT(c, dmax)) return 1;                          // (the fill reads the channel-major copy)
    int rc0 = ensure_blocks(c);
    if (rc0) return rc0;
    {
        hd::ZeroList z{};
        for (int i = 0; i < n; i++) z.p[i] = plans[i]->d_maxabs;
        HIPCHK(c, hd::launch_zero_list(z, n, c->stream));
    }
    HIPCHK(c, hipEventRecord(p0->ev[0], c->stream));
    const bool clip_runs = c->opts.clip_sigma > 0.0f && !c->clip_valid;
    const bool fork_clip = clip_runs && !c->rawT_valid && alloc_rawT(c, dmax);
    const uint8_t* rawT = !fork_clip ? ensure_rawT(c, dmax, true) : nullptr;
    rc0 = ensure_clip(c, fork_clip ? c->ev_aux0 : nullptr);
    if (fork_clip && !rc0) rawT = ensure_rawT(c, dmax, true, true);
    const hipError_t ej = join_aux(c);
    if (rc0) return rc0;
    HIPCHK(c, ej);
    if (!rawT) return fail(c, HD_E_HIP, "stage 1: channel-major copy failed");
    const bool clip = c->opts.clip_sigma > 0.0f;
    m.rd = raw_desc(c);
    m.rawT = rawT;
    m.tstride = c->rawT_stride;
    m.npass = n;
    m.nsub = nsub;
    m.cps = cps;
    m.ds = 1;                                     // tiles of 4 * S raw rows (special-tile list)
    m.to = 4 * S;
    m.ds_mode = c->opts.ds_mode;
    m.sub_dtype = c->opts.sub_dtype;
    m.sub_round = c->opts.sub_round;
    m.dmax = dmax;
    m.two_ok = 2;
    m.ngroups = nsub;
    m.ntiles = (int)((c->obs.N + 4 * S - 1) / (4 * S));
    m.nds = c->obs.N;
    m.out_stride = p0->sub_stride;
    for (int i = 0; i < n; i++) {
        m.dly[i] = plans[i]->d_idispdt;
        m.out[i] = plans[i]->d_sub;
        m.maxabs[i] = plans[i]->d_maxabs;
        m.ostride[i] = plans[i]->sub_stride;
        m.pds[i] = plans[i]->pass.ds;
        m.ptie[i] = q8_tie_eps(c, cps, plans[i]->pass.ds);
    }
    int nsp = 0, *d_sp = nullptr;
    int rc = special_tiles(c, m, &d_sp, &nsp);
    if (rc) return rc;
    {
        hd::Stage1Multi mp = m;
        mp.probe = p0->probe & (1 | 2 | 4 | 8);    // profiling (results invalid): skip sums / fill / float folds / stores
        HIPCHK(c, hd::launch_stage1_q8m(mp, c->stream));
    }
    // the special tiles on the float kernel: every pass in ONE launch (per-pass ds, a.pass_ds;
    // the tile is 4 S raw rows whatever the ds), or (HD_S1_SPMERGE=0) one launch per DDplan stage
    static const bool sp_merge = !(getenv("HD_S1_SPMERGE") && atoi(getenv("HD_S1_SPMERGE")) == 0);
    if (nsp && sp_merge) {
        // in quarter sub-tiles (S raw rows, S / ds outputs of every pass; S = 960 is a multiple
        // of every ds the fused launch takes)
        hd::Stage1Multi f = m;
        int fvw = 4, *d_sub = nullptr, nsub_t = 0;
        f.pass_ds = 1;
        if (!stage1_tiling_fixed(c, nsub, 1, dmax, S, f, fvw))
            return fail(c, HD_E_INVAL, "stage 1: no float tiling for the fused launch's special tiles");
        f.to = S;
        f.ntiles = 4 * m.ntiles;
        rc = special_subtiles(c, m, 4, &d_sub, &nsub_t);
        if (rc) return rc;
        const size_t flds = hd::stage1_tiled_lds_bytes(f);
        if (flds > c->lds_attr_set) {
            HIPCHK(c, hd::stage1_tiled_set_lds_limit(flds));
            c->lds_attr_set = flds;
        }
        if (nsub_t) HIPCHK(c, hd::launch_stage1_tiled(f, fvw, d_sub, nsub_t, true, c->stream));
    }
    // per DDplan stage (ds): the fixup groups (and the special tiles when not merged)
    std::vector<hd::Stage1Multi> groups;
    for (int i0 = 0; i0 < n;) {
        int i1 = i0;
        while (i1 < n && plans[i1]->pass.ds == plans[i0]->pass.ds) i1++;
        hd::Stage1Multi g = m;
        const int ds = plans[i0]->pass.ds;
        g.ds = ds;
        g.npass = i1 - i0;
        g.nds = plans[i0]->nds;
        g.out_stride = plans[i0]->sub_stride;
        g.dmax = 0;
        for (int i = i0; i < i1; i++) {
            const int k = i - i0;
            g.dly[k] = plans[i]->d_idispdt;
            g.out[k] = plans[i]->d_sub;
            g.maxabs[k] = plans[i]->d_maxabs;
            g.ostride[k] = plans[i]->sub_stride;
            g.dmax = std::max(g.dmax, plans[i]->maxdelay);
        }
        if (nsp && !sp_merge) {
            hd::Stage1Multi f = g;
            int fvw = 4;
            f.dmax = dmax;                            // the fused tiles' rows: 4 S + dmax
            f.to = 4 * S / ds;                        // (tile t: outputs from t * to, raw rows from t * 4 S)
            if (!stage1_tiling_fixed(c, nsub, ds, dmax, 4 * S / ds, f, fvw))   // checked above, before any launch
                return fail(c, HD_E_INVAL, "stage 1: no float tiling for the fused launch's special tiles (ds %d)", ds);
            f.ntiles = m.ntiles;
            const size_t flds = hd::stage1_tiled_lds_bytes(f);
            if (flds > c->lds_attr_set) {
                HIPCHK(c, hd::stage1_tiled_set_lds_limit(flds));
                c->lds_attr_set = flds;
            }
            HIPCHK(c, hd::launch_stage1_tiled(f, fvw, d_sp, nsp, true, c->stream));
        }
        groups.push_back(g);
        i0 = i1;
    }
    // the clipped-spectrum and block-boundary outputs of every pass in one k_stage1_fix8 launch
    // (per-pass ds: one raw window per item for all the stages), else per DDplan stage
    if (clip && !(p0->probe & (32 | 64))) {       // (probe bits 5-6: fixups skipped, profiling)
        hd::Stage1Multi fx = m;
        fx.ds = 0;
        for (int i = 0; i < n; i++) fx.ds = std::max(fx.ds, (int)m.pds[i]);
        fx.pass_ds = 1;
        fx.nds = c->obs.N / fx.ds;
        const bool env_off = getenv("HD_FIX8M") && atoi(getenv("HD_FIX8M")) == 0;
        fix8_bounds(c, fx);
        const hipError_t e = env_off ? hipErrorNotSupported
                                     : hd::launch_stage1_fixup(fx, c->clip.events, c->clip.nevents, fx.rd.zidx != nullptr,
                                                               c->stream);
        if (e == hipErrorNotSupported) {
            for (auto g : groups) {
                fix8_bounds(c, g);
                HIPCHK(c, hd::launch_stage1_fixup(g, c->clip.events, c->clip.nevents, g.rd.zidx != nullptr, c->stream));
            }
        } else {
            HIPCHK(c, e);
        }
    }
    HIPCHK(c, hipEventRecord(p0->ev[1], c->stream));
    for (int i = 0; i < n; i++) {
        plans[i]->sub_valid = true;
        plans[i]->sub_bound = stage1_sub_bound(c, plans[i]);
        plans[i]->sub_nonneg = plans[i]->sub_bound >= 0 && stage1_sub_nonneg(c);
        plans[i]->ran_sub = (i == 0);
    }
    return HD_OK;
}

extern "C" int hd_run_subband_multi(hd_plan** plans, int32_t n)
{
    if (!plans || n < 1 || !plans[0]) return fail(nullptr, HD_E_INVAL, "hd_run_subband_multi: no plans");
    hd_ctx* c = plans[0]->ctx;
    for (int i = 0; i < n; i++) {
        hd_plan* p = plans[i];
        if (!p) return fail(c, HD_E_INVAL, "hd_run_subband_multi: plan %d is NULL", i);
        if (p->ctx != c) return fail(c, HD_E_INVAL, "hd_run_subband_multi: plans from different contexts");
        if (p->pass.nsub != plans[0]->pass.nsub)
            return fail(c, HD_E_INVAL, "hd_run_subband_multi: plans must share nsub");
        if (p->pass.flags & HD_PASS_SUB_INPUT)
            return fail(c, HD_E_STATE, "hd_run_subband: a HD_PASS_SUB_INPUT plan takes hd_set_subbands");
    }
    if (!c->raw_ready) return fail(c, HD_E_STATE, "hd_run_subband: no raw data (hd_push_raw / hd_synth_device)");
    HIPCHK(c, hipSetDevice(c->device));
    if (c->s2all) {
        // stage 2 runs on stream2 behind stage 1: only these plans' own last stage-2 passes
        // must be done before their subbands are rewritten (the next DDplan stage's stage 1
        // overlaps the current stage's stage 2)
        for (int i = 0; i < n; i++)
            if (plans[i]->ran_dd && plans[i]->dd_stream == c->stream2)
                HIPCHK(c, hipStreamWaitEvent(c->stream, dd_end(plans[i]), 0));
    } else {
        HIPCHK(c, join_stream2(c));      // a stage-2 pass on stream2 may still read these subbands
    }
    for (int i = 0; i < n; i++) {
        int rc = ensure_sub(c, plans[i]);
        if (rc) return rc;
    }
    // plans ordered by ds (stable): the stages of a mixed call run in ascending ds
    std::vector<hd_plan*> v(plans, plans + n);
    std::stable_sort(v.begin(), v.end(), [](const hd_plan* x, const hd_plan* y) { return x->pass.ds < y->pass.ds; });
    // the passes of several DDplan stages with ds >= 2: one fused launch when they qualify
    const int cps = c->obs.nchan / plans[0]->pass.nsub;
    std::vector<hd_plan*> fz, rest;
    for (hd_plan* p : v)
        (hd::stage1_q8m_supports_ds(p->pass.ds) && hd::stage1_q8_supports(cps, p->pass.ds) ? fz : rest).push_back(p);
    if (q8m_ok(c, fz.data(), (int)fz.size())) {
        const int rc = run_subband_fused(c, fz.data(), (int)fz.size());
        if (rc < 0) return rc;
        if (rc == HD_OK) fz.clear();
    }
    rest.insert(rest.end(), fz.begin(), fz.end());
    std::stable_sort(rest.begin(), rest.end(), [](const hd_plan* x, const hd_plan* y) { return x->pass.ds < y->pass.ds; });
    for (int a0 = 0; a0 < (int)rest.size();) {
        int a1 = a0;
        while (a1 < (int)rest.size() && rest[a1]->pass.ds == rest[a0]->pass.ds && a1 - a0 < hd::kMaxPass) a1++;
        int rc = run_subband_chunk(c, rest.data() + a0, a1 - a0);
        if (rc) return rc;
        a0 = a1;
    }
    return HD_OK;
}

extern "C" int hd_run_subband(hd_plan* p)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_run_subband: NULL plan");
    return hd_run_subband_multi(&p, 1);
}

extern "C" int hd_get_subbands(hd_plan* p, void* host)
{
    if (!p || !host) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_get_subbands: NULL argument");
    hd_ctx* c = p->ctx;
    if (!p->sub_valid) return fail(c, HD_E_STATE, "hd_get_subbands: no subbands formed for this plan yet");
    const size_t es = sub_elem(c);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, d2h_2d(host, es * p->nds, p->d_sub, es * p->sub_stride, es * p->nds, p->pass.nsub, c->stream));
    return HD_OK;
}

extern "C" int hd_get_subbands_window(hd_plan* p, int64_t t0, int64_t count, void* host)
{
    if (!p || !host) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_get_subbands_window: NULL argument");
    hd_ctx* c = p->ctx;
    if (!p->sub_valid) return fail(c, HD_E_STATE, "hd_get_subbands_window: no subbands formed for this plan yet");
    if (t0 < 0 || count < 0 || t0 + count > p->nds)
        return fail(c, HD_E_INVAL, "hd_get_subbands_window: [%lld, %lld) outside [0, %lld)", (long long)t0,
                    (long long)(t0 + count), (long long)p->nds);
    if (count == 0) return HD_OK;
    const size_t es = sub_elem(c);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, d2h_2d(host, es * count, (const char*)p->d_sub + es * t0, es * p->sub_stride, es * count,
                     p->pass.nsub, c->stream));
    return HD_OK;
}

extern "C" int hd_get_series(hd_plan* p, int32_t dm0, int32_t ndm, int64_t t0, int64_t count, float* host)
{
    if (!p || !host) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_get_series: NULL argument");
    hd_ctx* c = p->ctx;
    if (!p->ran_dd || !p->d_out) return fail(c, HD_E_STATE, "hd_get_series: run hd_run_dedisp first");
    if (dm0 < 0 || ndm < 0 || dm0 + ndm > p->pass.numdms || t0 < 0 || count < 0 || t0 + count > p->numout)
        return fail(c, HD_E_INVAL, "hd_get_series: window outside [%d DMs] x [0, %lld)", p->pass.numdms,
                    (long long)p->numout);
    if (count == 0 || ndm == 0) return HD_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, d2h_2d(host, sizeof(float) * count, p->d_out + (size_t)dm0 * p->out_stride + t0,
                     sizeof(float) * p->out_stride, sizeof(float) * count, ndm, p->dd_stream));
    return HD_OK;
}

// ---- rfifind statistics (hd_rfi.hip; PALFA2_presto_search.py:482-490) ----------------------
extern "C" int hd_rfifind_stats(hd_ctx* c, int32_t ptsperint, float* dataavg, float* datastd, float* datapow)
{
    if (!c || !dataavg || !datastd || !datapow) return fail(c, HD_E_INVAL, "hd_rfifind_stats: NULL argument");
    if (!c->raw_ready) return fail(c, HD_E_STATE, "hd_rfifind_stats: no raw data (hd_push_raw / hd_synth_device)");
    if (!c->h_mask.empty()) return fail(c, HD_E_STATE, "hd_rfifind_stats: rfifind reads the data before any mask");
    if (c->slice_total) return fail(c, HD_E_STATE, "hd_rfifind_stats: not on a time-sliced context");
    if (ptsperint < 4 || ptsperint % 2) return fail(c, HD_E_INVAL, "hd_rfifind_stats: ptsperint must be even, >= 4");
    const int64_t numint = c->obs.N / ptsperint;
    if (numint < 1) return fail(c, HD_E_INVAL, "hd_rfifind_stats: fewer than ptsperint spectra");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, join_stream2(c));
    int rc = ensure_clip(c);                         // rfifind's own clip_times (no mask yet)
    if (rc) return rc;
    const uint8_t* rawT = ensure_rawT(c, 0);         // one byte per sample for 8/4-bit data
    if (c->d_scl || c->d_offs || c->d_wts) rawT = nullptr;   // calibrated: the generic decode
    const size_t n = (size_t)numint * c->obs.nchan;
    float* d = nullptr;
    HIPCHK(c, hipMalloc(&d, sizeof(float) * 3 * n));
    hipError_t e = hd::rfi_stats(raw_desc(c), rawT, c->rawT_stride, ptsperint, (int)numint, d, d + n, d + 2 * n,
                                 c->stream);
    if (e == hipSuccess) e = hipMemcpy(dataavg, d, sizeof(float) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(datastd, d + n, sizeof(float) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(datapow, d + 2 * n, sizeof(float) * n, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    HIPCHK(c, e);
    return HD_OK;
}

// ---- single-pulse search (hd_sp.hip; replaces single_pulse_search.py per .dat,
//      PALFA2_presto_search.py:539-546) ----------------------------------------------------
static const int32_t kSpDownfacts[] = {2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150, 220, 300};

extern "C" int hd_sp_widths(double dt, double maxwidth, int32_t* widths, int32_t* n)
{
    if (!widths || !n || !(dt > 0.0)) return fail(nullptr, HD_E_INVAL, "hd_sp_widths: bad argument");
    int k = 0;
    widths[k++] = 1;
    for (int32_t w : kSpDownfacts)
        if ((double)w * dt <= maxwidth) widths[k++] = w;
    *n = k;
    return HD_OK;
}

// Wall time of hd_single_pulse's phases (device search + count, copies, host pruning),
// summed over the process and printed at exit when HD_SP_TIMING is set (profiling only).
struct SpTimer {
    static double acc[3];
    static int calls;
    bool on;
    std::chrono::steady_clock::time_point t;
    SpTimer() : on(getenv("HD_SP_TIMING") != nullptr), t(std::chrono::steady_clock::now())
    {
        static bool reg = false;
        if (on && !reg) {
            reg = true;
            atexit([] {
                fprintf(stderr, "hd_single_pulse: %d calls, device+count %.1f ms, copies %.1f ms, prune %.1f ms\n",
                        calls, acc[0], acc[1], acc[2]);
            });
        }
        if (on) calls++;
    }
    void mark(int k)
    {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        acc[k] += std::chrono::duration<double, std::milli>(n - t).count();
        t = n;
    }
};
double SpTimer::acc[3] = {0, 0, 0};
int SpTimer::calls = 0;

// Hits grouped by DM (src -> dst, any order within a DM): per-thread counts, offsets, then
// per-thread scatters over up to 16 host threads; dstart[ndm + 1] receives the group starts.
static void sp_group_by_dm(const hd_sp_hit* src, int64_t n, int ndm, hd_sp_hit* dst, std::vector<int64_t>& dstart)
{
    const int nth = n < 65536 ? 1 : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<int64_t> cnt((size_t)nth * ndm, 0);
    auto range = [&](int t, int64_t& a, int64_t& b) {
        a = n * t / nth;
        b = n * (t + 1) / nth;
    };
    auto par = [&](auto&& fn) {
        if (nth == 1) {
            fn(0);
            return;
        }
        std::vector<std::thread> th;
        for (int t = 0; t < nth; t++) th.emplace_back(fn, t);
        for (auto& x : th) x.join();
    };
    par([&](int t) {
        int64_t a, b;
        range(t, a, b);
        int64_t* c = cnt.data() + (size_t)t * ndm;
        for (int64_t i = a; i < b; i++) c[src[i].dm]++;
    });
    dstart.assign((size_t)ndm + 1, 0);
    int64_t run = 0;
    for (int d = 0; d < ndm; d++) {
        dstart[(size_t)d] = run;
        for (int t = 0; t < nth; t++) {
            const int64_t k = cnt[(size_t)t * ndm + d];
            cnt[(size_t)t * ndm + d] = run;
            run += k;
        }
    }
    dstart[(size_t)ndm] = run;
    par([&](int t) {
        int64_t a, b;
        range(t, a, b);
        int64_t* o = cnt.data() + (size_t)t * ndm;
        for (int64_t i = a; i < b; i++) dst[o[src[i].dm]++] = src[i];
    });
}

// One DM's hits in (bin, width) order: an LSD radix sort on bin << 4 | widx (8-bit digits,
// passes up to the key's highest digit) for larger lists, std::sort for short or odd ones.
static void sp_sort_hits(hd_sp_hit* h, int64_t n)
{
    auto cmp = [](const hd_sp_hit& x, const hd_sp_hit& y) { return x.bin != y.bin ? x.bin < y.bin : x.widx < y.widx; };
    uint32_t kmax = 0;
    bool ok = n >= 512;
    for (int64_t i = 0; i < n && ok; i++) {
        ok = h[i].bin >= 0 && h[i].bin < (1 << 27) && h[i].widx >= 0 && h[i].widx < 16;
        kmax = std::max(kmax, ((uint32_t)h[i].bin << 4) | (uint32_t)h[i].widx);
    }
    if (!ok) {
        std::sort(h, h + n, cmp);
        return;
    }
    std::vector<hd_sp_hit> tmp((size_t)n);
    hd_sp_hit *a = h, *b = tmp.data();
    for (int shift = 0; shift < 32 && (kmax >> shift) != 0; shift += 8) {
        int64_t pos[256] = {0};
        for (int64_t i = 0; i < n; i++) pos[((((uint32_t)a[i].bin << 4) | (uint32_t)a[i].widx) >> shift) & 255]++;
        int64_t run = 0;
        for (int d = 0; d < 256; d++) {
            const int64_t c = pos[d];
            pos[d] = run;
            run += c;
        }
        for (int64_t i = 0; i < n; i++) b[pos[((((uint32_t)a[i].bin << 4) | (uint32_t)a[i].widx) >> shift) & 255]++] = a[i];
        std::swap(a, b);
    }
    if (a != h) std::copy(a, a + n, h);
}

// prune_related2 (the script's greedy walk across widths) and, for padded series,
// prune_border_cases, on one DM's hits sorted by (bin, width) in place; returns the kept count.
// The walk's inner loop visits, for pivot i, every later hit within max(downfact)/2 bins; a
// pair acts only when its gap is <= max(w_i/2, w_j/2, 1), and for a fixed i the pairs act
// independently (each sets gone[j] or gone[i], and the loop reads only gone[j]), so the
// relevant j are taken as the contiguous run within max(w_i/2, 1) plus, per wider width
// class k, that class's hits within widths[k]/2 -- the same set, fewer visits.
static int64_t sp_prune_dm(hd_sp_hit* h, int64_t n, const int32_t* widths, int nw, int64_t nds, int64_t numout)
{
    sp_sort_hits(h, n);
    std::vector<char> gone((size_t)n, 0);
    const int reach = nw > 1 ? widths[nw - 1] / 2 : 0;
    std::vector<std::vector<int32_t>> cls((size_t)nw);
    for (int64_t i = 0; i < n; i++) cls[(size_t)h[i].widx].push_back((int32_t)i);
    auto act = [&](int64_t i, int64_t j) {
        if (gone[j]) return;
        if (h[i].sigma > h[j].sigma) gone[j] = 1;
        else gone[i] = 1;
    };
    for (int64_t i = 0; i + 1 < n; i++) {
        if (gone[i]) continue;
        const int bi = h[i].bin;
        const int own = std::max(widths[h[i].widx] / 2, 1);
        const int run = std::min(own, reach);
        int64_t j = i + 1;
        for (; j < n && h[j].bin - bi <= run; j++) act(i, j);
        for (int k = 0; k < nw; k++) {
            const int lim = std::min(widths[k] / 2, reach);
            if (lim <= run) continue;
            const std::vector<int32_t>& L = cls[(size_t)k];
            auto it = std::upper_bound(L.begin(), L.end(), bi + run,
                                       [&](int v, int32_t idx) { return v < h[idx].bin; });
            for (; it != L.end() && h[*it].bin - bi <= lim; ++it) act(i, *it);
        }
    }
    if (numout > nds) {
        const int64_t off = nds - 1, on = numout - 1;
        for (int64_t i = n - 1; i >= 0; i--) {
            if (gone[i]) continue;                        // the script walks the pruned list
            const int64_t lo = h[i].bin - widths[h[i].widx] / 2, hi = h[i].bin + widths[h[i].widx] / 2;
            if (hi < off) break;
            if (hi > off && lo < on) gone[i] = 1;
        }
    }
    int64_t k = 0;
    for (int64_t i = 0; i < n; i++)
        if (!gone[i]) h[k++] = h[i];
    return k;
}

// Every DM's group [dstart[d], dstart[d+1]) pruned (DMs over up to 16 host threads), the
// kept hits compacted to the front in DM order; returns their count.
static int64_t sp_prune_groups(hd_sp_hit* hits, const std::vector<int64_t>& dstart, int ndm, const int32_t* widths,
                               int nw, int64_t nds, int64_t numout)
{
    std::vector<int64_t> kept((size_t)ndm, 0);
    auto one = [&](int d) {
        kept[(size_t)d] = sp_prune_dm(hits + dstart[d], dstart[d + 1] - dstart[d], widths, nw, nds, numout);
    };
    const unsigned nth = std::max(1u, std::min({16u, std::thread::hardware_concurrency(), (unsigned)ndm}));
    if (nth <= 1 || dstart[ndm] < 4096) {
        for (int d = 0; d < ndm; d++) one(d);
    } else {
        std::vector<std::thread> th;
        std::atomic<int> next{0};
        for (unsigned t = 0; t < nth; t++)
            th.emplace_back([&]() {
                for (int d = next++; d < ndm; d = next++) one(d);
            });
        for (auto& t : th) t.join();
    }
    int64_t out = 0;
    for (int d = 0; d < ndm; d++) {
        if (out != dstart[d]) memmove(hits + out, hits + dstart[d], sizeof(hd_sp_hit) * (size_t)kept[(size_t)d]);
        out += kept[(size_t)d];
    }
    return out;
}

extern "C" int hd_sp_prune(hd_sp_hit* hits, int64_t n, int32_t ndm, const int32_t* widths, int32_t nw, int64_t nds,
                           int64_t numout, int64_t* nkept)
{
    if ((n > 0 && !hits) || !widths || !nkept || nw < 1 || nw > 16 || ndm < 1 || n < 0)
        return fail(nullptr, HD_E_INVAL, "hd_sp_prune: bad argument");
    for (int64_t i = 0; i < n; i++)
        if (hits[i].dm < 0 || hits[i].dm >= ndm || hits[i].widx < 0 || hits[i].widx >= nw)
            return fail(nullptr, HD_E_INVAL, "hd_sp_prune: hit %lld has dm %d / widx %d out of range", (long long)i,
                        (int)hits[i].dm, (int)hits[i].widx);
    std::vector<int64_t> dstart;
    {
        std::vector<hd_sp_hit> tmp(hits, hits + n);
        sp_group_by_dm(tmp.data(), n, ndm, hits, dstart);
    }
    *nkept = sp_prune_groups(hits, dstart, ndm, widths, nw, nds, numout);
    return HD_OK;
}

static void sp_bufs_free(SpBufs* b)
{
    dfree(b->d_coef);
    dfree(b->d_hits);
    dfree(b->d_count);
    dfree(b->d_bad);
    if (b->ev) (void)hipEventDestroy(b->ev);
    delete b;
}

// The device half into the search's buffers (hit list sized cap), marked by b->ev.
static int sp_launch_device(hd_ctx* c, hd_plan* p, SpPlan* sp, int64_t cap)
{
    const int ndm = p->pass.numdms;
    SpBufs* b = sp->b;
    if (b->cap < cap) {
        HIPCHK(c, hipStreamSynchronize(sp->st));
        dfree(b->d_hits);
        b->d_hits = nullptr;
        b->cap = 0;
        HIPCHK(c, hipMalloc(&b->d_hits, sizeof(hd_sp_hit) * (size_t)cap));
        b->cap = cap;
    }
    HIPCHK(c, hipMemsetAsync(b->d_count, 0, sizeof(unsigned long long), sp->st));
    if (sp->nblocks > 0) {
        HIPCHK(c, hd::launch_sp_blocks(p->d_out, p->out_stride, ndm, (int)sp->nblocks, b->d_coef, sp->st));
        HIPCHK(c, hd::launch_sp_hits(p->d_out, p->out_stride, ndm, (int)sp->nblocks, b->d_coef, sp->ls, sp->widths,
                                     sp->rsw, sp->nw, sp->threshold, b->d_hits, b->d_count, b->cap, sp->st));
        HIPCHK(c, hd::launch_sp_badflags(b->d_coef, (int64_t)ndm * sp->nblocks, b->d_bad, sp->st));
    }
    HIPCHK(c, hipEventRecord(b->ev, sp->st));
    return HD_OK;
}

extern "C" int hd_single_pulse_launch(hd_plan* p, double dt, double maxwidth, double threshold)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_single_pulse_launch: NULL plan");
    hd_ctx* c = p->ctx;
    if (!p->ran_dd || !p->d_out) return fail(c, HD_E_STATE, "hd_single_pulse: run hd_run_dedisp first");
    int32_t widths[16], nw = 0;
    int rc = hd_sp_widths(dt, maxwidth, widths, &nw);
    if (rc) return fail(c, rc, "hd_single_pulse: dt must be > 0");
    const int ndm = p->pass.numdms;
    const int64_t nblocks = p->numout / 1000;                  // roundN / detrendlen
    if (nblocks > hd::sp_max_blocks())
        return fail(c, HD_E_INVAL, "hd_single_pulse: %lld blocks > %d", (long long)nblocks, hd::sp_max_blocks());
    HIPCHK(c, hipSetDevice(c->device));
    if (!p->sp) p->sp = new SpPlan();
    SpPlan* sp = p->sp;
    if (!c->ssp) HIPCHK(c, hipStreamCreateWithFlags(&c->ssp, hipStreamNonBlocking));
    if (sp->b) {
        HIPCHK(c, hipEventSynchronize(sp->b->ev));            // a relaunch before its collect
    } else if (!c->sp_free.empty()) {
        sp->b = c->sp_free.back();
        c->sp_free.pop_back();
    } else {
        SpBufs* b = new SpBufs();
        c->sp_all.push_back(b);
        sp->b = b;
        HIPCHK(c, hipEventCreateWithFlags(&b->ev, hipEventDisableTiming));
        HIPCHK(c, hipMalloc(&b->d_count, sizeof(unsigned long long)));
    }
    SpBufs* b = sp->b;
    sp->st = p->dd_stream ? p->dd_stream : c->stream;
    sp->nw = nw;
    for (int i = 0; i < nw; i++) {
        sp->widths[i] = widths[i];
        sp->rsw[i] = 1.0 / std::sqrt((double)widths[i]);
    }
    sp->threshold = threshold;
    sp->nblocks = nblocks;
    sp->ls = nblocks * 1000 / 8000 * 8000;                     // numchunks * chunklen
    const size_t cbytes = sizeof(double) * 4 * (size_t)std::max<int64_t>(1, (int64_t)ndm * nblocks);
    const size_t bbytes = (size_t)std::max<int64_t>(1, (int64_t)ndm * nblocks);
    if (b->coef_bytes < cbytes || b->bad_bytes < bbytes) {
        HIPCHK(c, hipStreamSynchronize(sp->st));
        dfree(b->d_coef);
        dfree(b->d_bad);
        b->d_coef = nullptr;
        b->d_bad = nullptr;
        b->coef_bytes = b->bad_bytes = 0;
        HIPCHK(c, hipMalloc(&b->d_coef, cbytes));
        HIPCHK(c, hipMalloc(&b->d_bad, bbytes));
        b->coef_bytes = cbytes;
        b->bad_bytes = bbytes;
    }
    rc = sp_launch_device(c, p, sp, std::max(b->cap, c->sp_cap_hint));
    if (rc) return rc;
    sp->pending = true;
    return HD_OK;
}

// pinned staging of at least `need` bytes (the host half runs one plan at a time)
static int sp_pin(hd_ctx* c, size_t need)
{
    if (need <= c->sp_pin_bytes) return HD_OK;
    if (c->sp_pin) HIPCHK(c, hipHostFree(c->sp_pin));
    c->sp_pin = nullptr;
    c->sp_pin_bytes = 0;
    HIPCHK(c, hipHostMalloc(&c->sp_pin, need + need / 4, hipHostMallocDefault));
    c->sp_pin_bytes = need + need / 4;
    return HD_OK;
}

extern "C" int hd_single_pulse_collect(hd_plan* p, hd_sp_hit* hits, int64_t cap, int64_t* nhits, uint8_t* bad_blocks,
                                       int64_t* nblocks_out)
{
    if (!p || !nhits || (cap > 0 && !hits)) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_single_pulse: NULL argument");
    hd_ctx* c = p->ctx;
    SpPlan* sp = p->sp;
    if (!sp || !sp->pending || !sp->b) return fail(c, HD_E_STATE, "hd_single_pulse_collect: no search launched on this plan");
    SpBufs* b = sp->b;
    HIPCHK(c, hipSetDevice(c->device));
    SpTimer tm;                                                // HD_SP_TIMING=1 (profiling)
    const int ndm = p->pass.numdms;
    if (nblocks_out) *nblocks_out = sp->nblocks;
    int rc = sp_pin(c, 64);
    if (rc) return rc;
    // the count, on the copy stream after the plan's device half only
    HIPCHK(c, hipStreamWaitEvent(c->ssp, b->ev, 0));
    HIPCHK(c, hipMemcpyAsync(c->sp_pin, b->d_count, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->ssp));
    HIPCHK(c, hipStreamSynchronize(c->ssp));
    unsigned long long cnt = *(const unsigned long long*)c->sp_pin;
    tm.mark(0);
    if ((int64_t)cnt > b->cap) {
        // the device list overflowed: grow it to the count and search again (once per size)
        const int64_t ncap = (int64_t)cnt + (int64_t)cnt / 4;
        c->sp_cap_hint = std::max(c->sp_cap_hint, ncap);
        rc = sp_launch_device(c, p, sp, ncap);
        if (rc) return rc;
        HIPCHK(c, hipStreamWaitEvent(c->ssp, b->ev, 0));
        HIPCHK(c, hipMemcpyAsync(c->sp_pin, b->d_count, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->ssp));
        HIPCHK(c, hipStreamSynchronize(c->ssp));
        cnt = *(const unsigned long long*)c->sp_pin;
    }
    // the bad-block flags as bytes (device-packed), and the hits, through the pinned block
    // (pageable copies of a few MB cost milliseconds per pass)
    const size_t nbad = bad_blocks && sp->nblocks > 0 ? (size_t)ndm * sp->nblocks : 0;
    *nhits = (int64_t)cnt;
    const bool fits = (int64_t)cnt <= cap;
    const size_t hbytes = fits ? sizeof(hd_sp_hit) * cnt : 0;
    rc = sp_pin(c, std::max(hbytes, nbad));
    if (rc) return rc;
    if (nbad) {
        HIPCHK(c, hipMemcpyAsync(c->sp_pin, b->d_bad, nbad, hipMemcpyDeviceToHost, c->ssp));
        HIPCHK(c, hipStreamSynchronize(c->ssp));
        memcpy(bad_blocks, c->sp_pin, nbad);
    }
    if (!fits)                                                 // (still pending: call again with room)
        return fail(c, HD_E_NOMEM, "hd_single_pulse: %llu hits > capacity %lld (call again with room)", cnt,
                    (long long)cap);
    if (cnt) {
        HIPCHK(c, hipMemcpyAsync(c->sp_pin, b->d_hits, hbytes, hipMemcpyDeviceToHost, c->ssp));
        HIPCHK(c, hipStreamSynchronize(c->ssp));
    }
    sp->pending = false;                                       // the buffers go back to the pool
    c->sp_free.push_back(b);
    sp->b = nullptr;
    if (!cnt) return HD_OK;
    const hd_sp_hit* src = (const hd_sp_hit*)c->sp_pin;
    tm.mark(1);
    // per DM (in parallel): the script's dm_candlist order -- by bin, widths in increasing
    // order among equal bins (width-1 hits appended first, every downfactor's bisect.insort
    // after equals) -- then prune_related2 (its greedy walk, literally) and prune_border_cases
    // (padded series: data ends at dend - 1, padding runs to numout - 1 -- the .inf on/off pair)
    // grouped by DM straight from the pinned block into the caller's buffer
    std::vector<int64_t> dstart;
    sp_group_by_dm(src, (int64_t)cnt, ndm, hits, dstart);
    // barycentred series: the data end where the last data segment ends (hd_plan_data_end)
    const int64_t dend = p->data_end >= 0 ? p->data_end : p->nvalid;
    const int64_t out = sp_prune_groups(hits, dstart, ndm, sp->widths, sp->nw, dend, p->numout);
    *nhits = out;
    tm.mark(2);
    return HD_OK;
}

extern "C" int hd_single_pulse(hd_plan* p, double dt, double maxwidth, double threshold, hd_sp_hit* hits,
                               int64_t cap, int64_t* nhits, uint8_t* bad_blocks, int64_t* nblocks_out)
{
    if (!p || !nhits || (cap > 0 && !hits)) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_single_pulse: NULL argument");
    const int rc = hd_single_pulse_launch(p, dt, maxwidth, threshold);
    if (rc) return rc;
    return hd_single_pulse_collect(p, hits, cap, nhits, bad_blocks, nblocks_out);
}

extern "C" int hd_series_sum(hd_plan* p, int32_t dm, int64_t t0, int64_t count, double* sum)
{
    if (!p || !sum) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_series_sum: NULL argument");
    hd_ctx* c = p->ctx;
    if (!p->ran_dd || !p->d_out) return fail(c, HD_E_STATE, "hd_series_sum: run hd_run_dedisp first");
    if (dm < 0 || dm >= p->pass.numdms || t0 < 0 || count < 0 || t0 + count > p->numout)
        return fail(c, HD_E_INVAL, "hd_series_sum: window outside [%d DMs] x [0, %lld)", p->pass.numdms,
                    (long long)p->numout);
    *sum = 0.0;
    if (count == 0) return HD_OK;
    HIPCHK(c, hipSetDevice(c->device));
    constexpr int kParts = 512;
    // partials in a context buffer (no stream-ordered pool), the stage-2 stream drained
    // before and after, and a blocking copy into the host vector
    if (!c->d_sum_parts) HIPCHK(c, hipMalloc(&c->d_sum_parts, kParts * sizeof(double)));
    HIPCHK(c, hipStreamSynchronize(p->dd_stream));
    HIPCHK(c, hd::launch_series_sum(p->d_out + (size_t)dm * p->out_stride + t0, count, c->d_sum_parts, kParts,
                                    p->dd_stream));
    HIPCHK(c, hipStreamSynchronize(p->dd_stream));
    std::vector<double> h(kParts);
    HIPCHK(c, d2h(h.data(), c->d_sum_parts, kParts * sizeof(double), p->dd_stream));
    double acc = 0.0;
    for (double v : h) acc += v;
    *sum = acc;
    return HD_OK;
}

extern "C" int hd_series_sum_multi(hd_plan* const* plans, int32_t n, int32_t dm, const int64_t* t0, const int64_t* count,
                                   double* sums)
{
    if (n < 0 || (n > 0 && (!plans || !t0 || !count || !sums)))
        return fail(nullptr, HD_E_INVAL, "hd_series_sum_multi: bad argument");
    if (n == 0) return HD_OK;
    hd_ctx* c = plans[0] ? plans[0]->ctx : nullptr;
    for (int i = 0; i < n; i++) {
        const hd_plan* p = plans[i];
        if (!p || p->ctx != c) return fail(c, HD_E_INVAL, "hd_series_sum_multi: plan %d is NULL or of another context", i);
        if (!p->ran_dd || !p->d_out) return fail(c, HD_E_STATE, "hd_series_sum_multi: plan %d: run hd_run_dedisp first", i);
        if (dm < 0 || dm >= p->pass.numdms || t0[i] < 0 || count[i] < 0 || t0[i] + count[i] > p->numout)
            return fail(c, HD_E_INVAL, "hd_series_sum_multi: plan %d: window outside [%d DMs] x [0, %lld)", i,
                        p->pass.numdms, (long long)p->numout);
    }
    HIPCHK(c, hipSetDevice(c->device));
    // hd_series_sum's partials (512 per series, summed on the host in index order: the same
    // doubles), every series' kernel queued on the main stream behind that plan's stage 2,
    // then one copy and one wait for all of them
    constexpr int kParts = 512;
    const size_t need = (size_t)n * kParts * sizeof(double);
    if (c->sum_parts_bytes < need) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        dfree(c->d_sum_parts_multi);
        c->d_sum_parts_multi = nullptr;
        c->sum_parts_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_sum_parts_multi, need));
        c->sum_parts_bytes = need;
    }
    HIPCHK(c, hipMemsetAsync(c->d_sum_parts_multi, 0, need, c->stream));
    for (int i = 0; i < n; i++) {
        hd_plan* p = plans[i];
        if (count[i] == 0) continue;
        if (p->dd_stream && p->dd_stream != c->stream) HIPCHK(c, hipStreamWaitEvent(c->stream, dd_end(p), 0));
        HIPCHK(c, hd::launch_series_sum(p->d_out + (size_t)dm * p->out_stride + t0[i], count[i],
                                        c->d_sum_parts_multi + (size_t)i * kParts, kParts, c->stream));
    }
    std::vector<double> h((size_t)n * kParts);
    HIPCHK(c, d2h(h.data(), c->d_sum_parts_multi, need, c->stream));
    for (int i = 0; i < n; i++) {
        double acc = 0.0;
        for (int k = 0; k < kParts; k++) acc += h[(size_t)i * kParts + k];
        sums[i] = count[i] ? acc : 0.0;
    }
    return HD_OK;
}

extern "C" int hd_series_fill(hd_plan* p, int64_t t0, float value)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_series_fill: NULL plan");
    hd_ctx* c = p->ctx;
    if (!p->ran_dd || !p->d_out) return fail(c, HD_E_STATE, "hd_series_fill: run hd_run_dedisp first");
    if (t0 < 0 || t0 > p->numout) return fail(c, HD_E_INVAL, "hd_series_fill: t0 outside [0, %lld]", (long long)p->numout);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hd::launch_series_fill(p->d_out, p->out_stride, p->pass.numdms, t0, p->numout, value, p->dd_stream));
    p->dd_cur = p->dd_own;           // (a pair this plan shared with a multi launch's other passes stays theirs)
    HIPCHK(c, hipEventRecord(dd_end(p), p->dd_stream));   // the series' end: hd_write_series copies after it
    return HD_OK;
}

extern "C" int hd_set_subbands(hd_plan* p, const void* host)
{
    if (!p || !host) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_set_subbands: NULL argument");
    hd_ctx* c = p->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, join_stream2(c));
    int rc = ensure_sub(c, p);
    if (rc) return rc;
    const size_t es = sub_elem(c);
    HIPCHK(c, hipMemcpy2DAsync(p->d_sub, es * p->sub_stride, host, es * p->nds, es * p->nds, p->pass.nsub,
                               hipMemcpyHostToDevice, c->stream));
    if (c->opts.sub_dtype == HD_SUB_I16) {
        int32_t m = 0;
        const int16_t* h = (const int16_t*)host;
        const size_t n = (size_t)p->pass.nsub * p->nds;
        bool neg = false;
        for (size_t i = 0; i < n; i++) {
            m = std::max(m, h[i] < 0 ? -(int32_t)h[i] : (int32_t)h[i]);
            neg |= h[i] < 0;
        }
        HIPCHK(c, hipMemcpyAsync(p->d_maxabs, &m, sizeof m, hipMemcpyHostToDevice, c->stream));
        p->sub_bound = m;
        p->sub_nonneg = !neg;
    } else {
        p->sub_bound = -1;
        p->sub_nonneg = false;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    p->sub_valid = true;
    return HD_OK;
}

// ---- barycentric output ---------------------------------------------------------------
// prepsubband's add/remove-bin list [PRESTO-ext, restated; reference call site
// PALFA2_presto_search.py:514-520, which passes no -nobary]: the barycentric minus topocentric
// time of each table point, relative to the first point, in output bins; wherever its nearest
// integer changes between points ii-1 and ii, one bin per half-bin crossing, at the output
// bin the crossing interpolates to (NEAREST_LONG(LININTERP(...)) of the crossing point
// between the two points' bin positions); negative when the difference falls (bins removed).
static long nearest_long_c(double x) { return x < 0.0 ? (long)(x - 0.5) : (long)(x + 0.5); }

extern "C" int hd_bary_diffbins(const double* topo, const double* bary, int32_t n, double tdt, double dsdt,
                                int32_t* diffbins, int32_t cap, int32_t* ndiff)
{
    if (!topo || !bary || !ndiff || (cap > 0 && !diffbins)) return fail(nullptr, HD_E_INVAL, "hd_bary_diffbins: NULL argument");
    if (n < 2 || !(tdt > 0.0) || !(dsdt > 0.0)) return fail(nullptr, HD_E_INVAL, "hd_bary_diffbins: need n >= 2, tdt > 0, dsdt > 0");
    std::vector<double> b((size_t)n);
    const double d0 = bary[0] - topo[0];
    for (int i = 0; i < n; i++) b[i] = ((bary[i] - topo[i]) - d0) * 86400.0 / dsdt;
    int32_t cnt = 0;
    long oldbin = 0;
    for (int ii = 1; ii < n; ii++) {
        const long currentbin = nearest_long_c(b[ii]);
        if (currentbin == oldbin) continue;
        double calcpt, lobin, hibin;
        if (currentbin > 0) {
            calcpt = (double)oldbin + 0.5;
            lobin = (ii - 1) * tdt / dsdt;
            hibin = ii * tdt / dsdt;
        } else {
            calcpt = (double)oldbin - 0.5;
            lobin = -((ii - 1) * tdt / dsdt);
            hibin = -(ii * tdt / dsdt);
        }
        while (std::fabs(calcpt) < std::fabs(b[ii])) {
            const double y = (calcpt - b[ii - 1]) * (hibin - lobin) / (b[ii] - b[ii - 1]) + lobin;
            const long v = nearest_long_c(y);
            if (cnt < cap) diffbins[cnt] = (int32_t)v;
            cnt++;
            calcpt = currentbin > 0 ? calcpt + 1.0 : calcpt - 1.0;
        }
        oldbin = currentbin;
    }
    *ndiff = cnt;
    if (cnt > cap) return fail(nullptr, HD_E_INVAL, "hd_bary_diffbins: %d bins > cap %d", (int)cnt, (int)cap);
    return HD_OK;
}

// Segments of the barycentred series from the diffbins, applied in PRESTO's order while the
// topocentric samples [0, nvalid) are written: the samples before |v|, then one padding sample
// (v > 0) or sample |v| skipped (v < 0); the rest, then padding to numout.
static void bary_segments(const int32_t* dv, int32_t nd, int64_t nvalid, int64_t numout, std::vector<int32_t>& seg,
                          bool& adds, int64_t& data_end)
{
    seg.clear();
    adds = false;
    data_end = 0;
    int64_t out = 0, src = 0;
    auto put = [&](int64_t s, int64_t len) {
        len = std::min<int64_t>(len, numout - out);
        if (len <= 0) return;
        if (s >= 0) data_end = out + len;                     // end of the last data segment
        const size_t k = seg.size();
        if (s < 0 && k >= 3 && seg[k - 2] < 0) {              // merge padding runs
            seg[k - 1] += (int32_t)len;
        } else {
            seg.push_back((int32_t)out);
            seg.push_back((int32_t)s);
            seg.push_back((int32_t)len);
        }
        if (s < 0) adds = true;
        out += len;
    };
    for (int32_t i = 0; i < nd && out < numout; i++) {
        const int64_t p = dv[i] < 0 ? -(int64_t)dv[i] : (int64_t)dv[i];
        if (p >= nvalid) break;
        put(src, p - src);
        src = p;
        if (dv[i] > 0) put(-1, 1);
        else src = p + 1;
    }
    put(src, nvalid - src);
    put(-1, numout - out);
}

extern "C" int hd_plan_set_bary(hd_plan* p, const int32_t* diffbins, int32_t ndiff)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_plan_set_bary: NULL plan");
    hd_ctx* c = p->ctx;
    if (ndiff < 0) return fail(c, HD_E_INVAL, "hd_plan_set_bary: bad diffbins");
    if (!diffbins) ndiff = 0;              // header contract: ndiff = 0 or diffbins NULL turns it off
    // unchanged settings (the same list, or topocentric again): nothing to do, and no wait
    // on the plan's queued work (run_pass sets the table on every pass)
    if (ndiff == (int32_t)p->bary_diff.size() && (ndiff == 0 ? p->nbseg == 0 : p->nbseg > 0) &&
        std::equal(p->bary_diff.begin(), p->bary_diff.end(), diffbins ? diffbins : p->bary_diff.data()))
        return HD_OK;
    if (ndiff > 0) {
        if (c->slice_total > 0) return fail(c, HD_E_INVAL, "hd_plan_set_bary: not for a time-sliced context");
        for (int32_t i = 1; i < ndiff; i++)
            if (std::abs((int64_t)diffbins[i]) < std::abs((int64_t)diffbins[i - 1]))
                return fail(c, HD_E_INVAL, "hd_plan_set_bary: |diffbins| must not decrease (entry %d)", (int)i);
        if (p->numout >= ((int64_t)1 << 31)) return fail(c, HD_E_INVAL, "hd_plan_set_bary: numout >= 2^31");
    }
    HIPCHK(c, hipSetDevice(c->device));
    // the old segment table may still be read by this plan's queued stage 2 / k_bary, and its
    // series by the writer: wait for exactly those (dd_end ends the plan's last hd_run_dedisp)
    if (p->ran_dd && dd_end(p)) HIPCHK(c, hipEventSynchronize(dd_end(p)));
    if (p->copy_pending && c->writer) HIPCHK(c, hipEventSynchronize(p->ev_copy));
    dfree(p->d_bseg);
    p->d_bseg = nullptr;
    p->nbseg = 0;
    p->bary_diff.clear();
    p->data_end = -1;
    p->ran_dd = false;                 // the device series no longer match the settings
    if (ndiff == 0) {
        dfree(p->d_topo);
        p->d_topo = nullptr;
        return HD_OK;
    }
    std::vector<int32_t> seg;
    bary_segments(diffbins, ndiff, p->nvalid, p->numout, seg, p->bary_adds, p->data_end);
    const size_t bytes = sizeof(int32_t) * seg.size();
    HIPCHK(c, hipMalloc(&p->d_bseg, std::max<size_t>(bytes, 16)));
    // a pageable source: the copy has completed when the call returns, so seg may go
    if (bytes) HIPCHK(c, hipMemcpyAsync(p->d_bseg, seg.data(), bytes, hipMemcpyHostToDevice, c->stream));
    if (bytes) HIPCHK(c, hipStreamSynchronize(c->stream));
    p->nbseg = (int32_t)(seg.size() / 3);
    p->bary_diff.assign(diffbins, diffbins + ndiff);
    if (!p->d_padv) HIPCHK(c, hipMalloc(&p->d_padv, sizeof(float) * (size_t)std::max(p->pass.numdms, 1)));
    return HD_OK;
}

extern "C" int hd_plan_data_end(const hd_plan* p, int64_t* n)
{
    if (!p || !n) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_plan_data_end: NULL argument");
    *n = p->data_end >= 0 ? p->data_end : p->nvalid;
    return HD_OK;
}

extern "C" int hd_run_dedisp(hd_plan* p, float* host_out)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_run_dedisp: NULL plan");
    hd_ctx* c = p->ctx;
    if (!p->sub_valid) return fail(c, HD_E_STATE, "hd_run_dedisp: run hd_run_subband (or hd_set_subbands) for this plan first");
    HIPCHK(c, hipSetDevice(c->device));
    if (!p->d_out) {
        const size_t bytes = sizeof(float) * (size_t)p->pass.numdms * p->out_stride;
        if (hipMalloc(&p->d_out, bytes) != hipSuccess) {
            p->d_out = nullptr;
            return fail(c, HD_E_NOMEM, "cannot allocate %zu bytes of DM series", bytes);
        }
    }
    const bool bary = p->nbseg > 0;
    if (bary && !p->d_topo) {
        const size_t bytes = sizeof(float) * (size_t)p->pass.numdms * p->out_stride;
        if (hipMalloc(&p->d_topo, bytes) != hipSuccess) {
            p->d_topo = nullptr;
            return fail(c, HD_E_NOMEM, "cannot allocate %zu bytes of topocentric DM series", bytes);
        }
    }
    // barycentric output: the padding value is needed for added bins and the tail
    const bool pad = bary || p->numout > p->nds;
    // alternate streams between passes (see hd_ctx::stream2); a plan re-run on the other
    // stream first waits for its previous run, which wrote the same series
    const bool alt = c->dual && (c->s2all || (c->dd_count++ & 1u) != 0);
    hipStream_t st = alt ? c->stream2 : c->stream;
    if (alt) {
        HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
        HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_fork, 0));
    }
    if (p->ran_dd && p->dd_stream != st) HIPCHK(c, hipStreamWaitEvent(st, dd_end(p), 0));
    if (p->copy_pending) {            // the writer may still be copying the previous series
        HIPCHK(c, hipStreamWaitEvent(st, p->ev_copy, 0));
        p->copy_pending = false;
    }
    // pair partials need |sub[s0] + sub[s1]| <= 32767 (packed int16), known on the host
    const bool pair_bound = p->sub_bound >= 0 && 2 * p->sub_bound <= 32767;
    const bool pair_ok = p->wide[3].ok && pair_bound;
    if ((p->variant == 6 && !pair_ok) || (p->variant == 7 && !(p->wide[4].ok && pair_bound)) ||
        (p->variant == 8 && !(p->wide[5].ok && pair_bound)) || (p->variant == 9 && !(p->wide[6].ok && pair_bound)))
        return fail(c, HD_E_INVAL, "hd_run_dedisp: pair variant needs 2 * max|subband| <= 32767 known on the host "
                    "(bound %d)", (int)p->sub_bound);
    int wk = -1;                       // wide variant in use (index into p->wide), or -1
    if (p->variant >= 3) wk = p->variant - 3;
    else if (p->variant == 0) {
        // auto: pair partials where they measured faster than the ring (full-resolution passes
        // of >= 72 DMs: 1.31 vs 1.39 ms per Mock stage-0 pass; at ds >= 2 or 64 DMs the extra
        // expand work outweighs the halved sums, profiles/r01_stage2_variants.txt)
        const bool pair_auto = pair_ok && p->pass.ds == 1 && p->pass.numdms >= 72;
        // two pairs per chunk beat the ring and the one-pair kernel at every Mock DDplan
        // stage (profiles/r02_stage2_variants.txt: 1.10 / 0.56 / 0.42 / 0.27 / 0.22 / 0.17 ms
        // vs the ring's 1.42 / 0.60 / 0.53 / 0.33 / 0.27 / 0.20)
        const bool pair2_auto = p->wide[4].ok && pair_bound;
        // (the register-window kernel, variant 8, measured slower at every DDplan stage: 1.63 vs
        // 1.07 ms per stage-0 pass, profiles/r04_stage2_rw_probe.txt -- not an auto choice)
        const bool qp = p->wide[6].ok && pair_bound && qp_auto();
        wk = qp ? 6 : pair2_auto ? 4 : pair_auto ? 3 : p->wide[2].ok ? 2 : p->wide[0].ok ? 0 : (p->wide[1].ok ? 1 : -1);
    }
    const bool use_wide = wk >= 0;
    const bool use_lds = !use_wide && (p->variant == 2 || (p->variant == 0 && p->lds_ok));
    const int tile = use_wide ? 256 * p->wide[wk].r : kTT;
    const int ntiles = (int)((p->nvalid + tile - 1) / tile);
    double* partial = nullptr;
    if (pad && c->opts.pad_mode != HD_PAD_ZERO) {
        const size_t need = sizeof(double) * (size_t)p->pass.numdms * std::max(ntiles, 1);
        double*& buf = alt ? c->d_partial2 : c->d_partial;
        size_t& have = alt ? c->partial_bytes2 : c->partial_bytes;
        if (have < need) {
            HIPCHK(c, hipStreamSynchronize(st));
            dfree(buf);
            buf = nullptr;
            have = 0;
            HIPCHK(c, hipMalloc(&buf, need));
            have = need;
        }
        partial = buf;
    }
    hd::Stage2Args a{};
    a.sub = p->d_sub;
    a.sub_dtype = c->opts.sub_dtype;
    a.nsub = p->pass.nsub;
    a.numdms = p->pass.numdms;
    a.nds = p->nds;
    a.sub_stride = p->sub_stride;
    a.nvalid = p->nvalid;
    a.out = bary ? p->d_topo : p->d_out;
    a.out_stride = p->out_stride;
    a.partial = partial;
    a.partial_ndm = c->opts.pad_mode == HD_PAD_DM0 ? 1 : 0;   // the padding reads DM 0's sums only
    a.ntiles = ntiles;
    a.tile = tile;
    a.maxabs = p->d_maxabs;
    a.omin = p->d_omin;
    a.wstride = p->wstride;
    a.dms_per_blk = p->dpb;
    p->dd_cur = p->dd_own;
    HIPCHK(c, hipEventRecord(dd_start(p), st));
    if (use_wide) {
        const hd_plan::Wide& w = p->wide[wk];
        a.off = w.d_boff;
        a.omin = w.d_omin;
        a.wstride = w.ws;
        a.dms_per_blk = w.dpb;
        a.sc = w.sc;
        a.probe = p->probe;
        a.ring_npw = w.npw;
        a.ring_nbp = w.nbp;
        a.ptab = w.d_omin;
        a.umax = w.umax;
        a.nonneg = p->sub_nonneg ? 1 : 0;
        a.qp_setb = wk == 6 ? w.setb[4 - w.sc] : 0;
        a.stamps = wk == 6 ? stamps_buf(c) : nullptr;
        a.nwg = p->pair_persist != 2 ? c->ncu : 0;   // persistent by default (measured 1.29 vs 1.36 ms, stage-0 pass)
        if (wk == 0) HIPCHK(c, hd::launch_stage2_wide(a, w.q, w.r, w.nw, st));
        else if (wk == 1) HIPCHK(c, hd::launch_stage2_wide2(a, w.q, w.r, w.nw, st));
        else if (wk == 2) HIPCHK(c, hd::launch_stage2_ring(a, w.q, w.r, st));
        int qp_ns = 0;
        bool qp_sy = false;
        if (wk == 5 || wk == 6) {
            hd::S2Multi m{};
            m.npass = 1;
            m.p[0] = hd::stage2_pass_of(a);
            if (wk == 5) HIPCHK(c, hd::launch_stage2_rw_multi(a, m, w.q, st));
            else {
                qp_ns = hd::stage2_qp_ns(m, a.nsub, w.sc);
                qp_sy = hd::stage2_qp_sync(m, a.nsub, w.sc);
                HIPCHK(c, hd::launch_stage2_qp_multi(a, m, w.q, w.r, w.sc, st));
            }
        } else if (wk > 2) HIPCHK(c, hd::launch_stage2_pair(a, w.q, w.r, wk == 4 ? 2 : 1, st));
        // the names rocprofv3 prints (template arguments as the compiler spells them)
        if (wk == 0) snprintf(p->s2name, sizeof(p->s2name), "k_stage2_wide<%d, %d, %d>", w.q, w.r, w.sc);
        else if (wk == 1) snprintf(p->s2name, sizeof(p->s2name), "k_stage2_wide2<%d, %d, %d>", w.q, w.r, w.sc);
        else if (wk == 2) snprintf(p->s2name, sizeof(p->s2name), "k_stage2_ring<%d, %d>", w.q, w.r);
        else if (wk == 5) snprintf(p->s2name, sizeof(p->s2name), "k_stage2_rw<%d>", w.q);
        else if (wk == 6) snprintf(p->s2name, sizeof(p->s2name), "k_stage2_qp<%d, %d, %d, %s, %s, %d, %s>", w.q, w.r, w.sc,
                                   a.nonneg && !(p->probe & 64) ? "true" : "false", (p->probe & 15) ? "true" : "false",
                                   qp_ns, qp_sy ? "true" : "false");
        else snprintf(p->s2name, sizeof(p->s2name), "k_stage2_pair<%d, %d, %d, %s, %s>", w.q, w.r, wk == 4 ? 2 : 1,
                      a.nonneg && !(p->probe & 64) ? "true" : "false", (p->probe & 15) ? "true" : "false");
    } else if (use_lds) {
        a.off = p->d_boff;
        HIPCHK(c, hd::launch_stage2_lds(a, p->q, st));
        snprintf(p->s2name, sizeof(p->s2name), "k_stage2_lds<%d>", p->q);
    } else {
        a.off = p->d_off;
        HIPCHK(c, hd::launch_stage2_direct(a, st));
        snprintf(p->s2name, sizeof(p->s2name), "k_stage2_direct");
    }
    if (bary)
        HIPCHK(c, hd::launch_bary(p->d_topo, p->d_out, p->out_stride, p->pass.numdms, p->numout, p->d_bseg, p->nbseg,
                                  partial, ntiles, p->nds, c->opts.pad_mode, p->d_padv, st));
    else if (pad)
        HIPCHK(c, hd::launch_pad(p->d_out, p->out_stride, p->pass.numdms, p->nds, p->numout, partial, ntiles,
                                 c->opts.pad_mode, st));
    HIPCHK(c, hipEventRecord(dd_end(p), st));
    if (alt) {
        HIPCHK(c, hipEventRecord(c->ev_join, st));
        c->s2_pending = true;
    }
    p->ran_dd = true;
    p->dd_stream = st;
    p->s2passes = 1;
    if (host_out) {
        HIPCHK(c, d2h_2d(host_out, sizeof(float) * p->numout, p->d_out, sizeof(float) * p->out_stride,
                         sizeof(float) * p->numout, p->pass.numdms, st));
    }
    return HD_OK;
}

// ---- stage 2 of several passes in one launch ---------------------------------------------
// A plan joins a multi-pass launch when it takes the two-pairs-per-chunk pair kernel (auto or
// variant 7) on the topocentric grid; plans with the same kernel and geometry (one DDplan
// stage) share a launch of at most kS2MaxPass passes, the rest run one by one.
// The kernel a plan takes in a shared launch: 5 (k_stage2_rw: variant 8), 4 (the
// two-pairs-per-chunk pair kernel: auto or variant 7), or -1 (alone).
static int dedisp_multi_kernel(const hd_plan* p)
{
    const bool pair_bound = p->sub_bound >= 0 && 2 * p->sub_bound <= 32767;
    if (!p->sub_valid || !pair_bound || p->nbseg != 0 || p->pair_persist == 2) return -1;
    if (p->variant == 8 && p->wide[5].ok) return 5;
    if ((p->variant == 9 || (p->variant == 0 && qp_auto())) && p->wide[6].ok) return 6;
    if ((p->variant == 0 || p->variant == 7) && p->wide[4].ok) return 4;
    return -1;
}

static bool dedisp_multi_ok(const hd_plan* p) { return dedisp_multi_kernel(p) >= 0; }

static bool dedisp_same_group(const hd_plan* a, const hd_plan* b)
{
    const int ka = dedisp_multi_kernel(a);
    if (ka != dedisp_multi_kernel(b)) return false;
    const hd_plan::Wide &x = a->wide[ka], &y = b->wide[ka];
    return a->ctx == b->ctx && x.q == y.q && x.r == y.r && x.dpb == y.dpb && (ka == 6 || x.sc == y.sc) &&
           a->pass.numdms == b->pass.numdms &&
           a->pass.nsub == b->pass.nsub && a->nds == b->nds && a->nvalid == b->nvalid && a->numout == b->numout &&
           a->out_stride == b->out_stride && a->sub_nonneg == b->sub_nonneg && a->probe == b->probe;
}

static int run_dedisp_group(hd_ctx* c, hd_plan* const* g, int n)
{
    hd_plan* p0 = g[0];
    const int wk = dedisp_multi_kernel(p0);
    const hd_plan::Wide& w0 = p0->wide[wk];
    // hd_set_streams(2 or 3): the shared launch runs on stream2, so the main stream goes on
    // to the next DDplan stage's stage 1 (other plans' subbands) beside it
    const bool alt = c->dual;
    hipStream_t st = alt ? c->stream2 : c->stream;
    if (alt) {
        HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
        HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_fork, 0));
    } else {
        HIPCHK(c, join_stream2(c));
    }
    for (int i = 0; i < n; i++) {
        hd_plan* p = g[i];
        if (!p->d_out) {
            const size_t bytes = sizeof(float) * (size_t)p->pass.numdms * p->out_stride;
            if (hipMalloc(&p->d_out, bytes) != hipSuccess) {
                p->d_out = nullptr;
                return fail(c, HD_E_NOMEM, "cannot allocate %zu bytes of DM series", bytes);
            }
        }
        if (p->ran_dd && p->dd_stream != st) HIPCHK(c, hipStreamWaitEvent(st, dd_end(p), 0));
        if (p->copy_pending) {
            HIPCHK(c, hipStreamWaitEvent(st, p->ev_copy, 0));
            p->copy_pending = false;
        }
    }
    const bool pad = p0->numout > p0->nds;
    const int tile = 256 * w0.r;
    const int ntiles = (int)((p0->nvalid + tile - 1) / tile);
    const size_t per = (size_t)p0->pass.numdms * std::max(ntiles, 1);
    double* partial = nullptr;
    if (pad && c->opts.pad_mode != HD_PAD_ZERO) {
        const size_t need = sizeof(double) * per * n;
        double*& buf = alt ? c->d_partial2 : c->d_partial;
        size_t& have = alt ? c->partial_bytes2 : c->partial_bytes;
        if (have < need) {
            HIPCHK(c, hipStreamSynchronize(st));
            dfree(buf);
            buf = nullptr;
            have = 0;
            HIPCHK(c, hipMalloc(&buf, need));
            have = need;
        }
        partial = buf;
    }
    hd::Stage2Args a{};
    a.sub = p0->d_sub;
    a.sub_dtype = c->opts.sub_dtype;
    a.nsub = p0->pass.nsub;
    a.numdms = p0->pass.numdms;
    a.nds = p0->nds;
    a.sub_stride = p0->sub_stride;
    a.nvalid = p0->nvalid;
    a.out = p0->d_out;
    a.out_stride = p0->out_stride;
    a.partial = partial;
    a.partial_ndm = c->opts.pad_mode == HD_PAD_DM0 ? 1 : 0;   // the padding reads DM 0's sums only
    a.ntiles = ntiles;
    a.tile = tile;
    a.maxabs = p0->d_maxabs;
    a.off = w0.d_boff;
    a.omin = w0.d_omin;
    a.wstride = w0.ws;
    a.dms_per_blk = w0.dpb;
    a.sc = w0.sc;
    a.probe = p0->probe;
    a.ring_npw = w0.npw;
    a.ring_nbp = w0.nbp;
    a.ptab = w0.d_omin;
    a.umax = w0.umax;
    a.nonneg = p0->sub_nonneg ? 1 : 0;
    a.nwg = c->ncu;
    a.stamps = wk == 6 ? stamps_buf(c) : nullptr;
    hd::S2Multi m{};
    m.npass = n;
    int ppc6 = 4;                       // k_stage2_qp: the smallest pairs-per-chunk of the passes
    for (int i = 0; i < n; i++) ppc6 = std::min(ppc6, (int)g[i]->wide[wk].sc);
    for (int i = 0; i < n; i++) {
        const hd_plan* p = g[i];
        const hd_plan::Wide& w = p->wide[wk];
        hd::S2Pass& q = m.p[i];
        q.sub = p->d_sub;
        q.ptab = w.d_omin;
        q.off = wk == 6 ? w.d_boffp[4 - ppc6] : w.d_boff;
        q.maxabs = p->d_maxabs;
        q.out = p->d_out;
        q.partial = partial ? partial + per * i : nullptr;
        q.sub_stride = p->sub_stride;
        q.ws = w.ws;
        q.npw = w.npw;
        q.nbp = w.nbp;
        q.umax = w.umax;
        q.setb = wk == 6 ? w.setb[4 - ppc6] : 0;
    }
    p0->dd_cur = p0->dd_own;
    HIPCHK(c, hipEventRecord(dd_start(p0), st));
    const int qp_ns = wk == 6 ? hd::stage2_qp_ns(m, a.nsub, ppc6) : 0;
    const bool qp_sy = wk == 6 && hd::stage2_qp_sync(m, a.nsub, ppc6);
    if (wk == 5) HIPCHK(c, hd::launch_stage2_rw_multi(a, m, w0.q, st));
    else if (wk == 6) HIPCHK(c, hd::launch_stage2_qp_multi(a, m, w0.q, w0.r, ppc6, st));
    else HIPCHK(c, hd::launch_stage2_pair_multi(a, m, w0.q, w0.r, 2, st));
    if (pad)
        for (int i = 0; i < n; i++)
            HIPCHK(c, hd::launch_pad(g[i]->d_out, g[i]->out_stride, g[i]->pass.numdms, g[i]->nds, g[i]->numout,
                                     m.p[i].partial, ntiles, c->opts.pad_mode, st));
    HIPCHK(c, hipEventRecord(dd_end(p0), st));       // one pair for every pass of the launch
    for (int i = 0; i < n; i++) {
        hd_plan* p = g[i];
        p->dd_cur = p0->dd_own;
        p->ran_dd = true;
        p->dd_stream = st;
        p->s2passes = i == 0 ? n : 0;
        if (wk == 5) snprintf(p->s2name, sizeof(p->s2name), "k_stage2_rw<%d>", w0.q);
        else if (wk == 6) snprintf(p->s2name, sizeof(p->s2name), "k_stage2_qp<%d, %d, %d, %s, %s, %d, %s>", w0.q, w0.r, ppc6,
                                   a.nonneg && !(a.probe & 64) ? "true" : "false", (a.probe & 15) ? "true" : "false",
                                   qp_ns, qp_sy ? "true" : "false");
        else snprintf(p->s2name, sizeof(p->s2name), "k_stage2_pair<%d, %d, 2, %s, %s>", w0.q, w0.r,
                      a.nonneg && !(a.probe & 64) ? "true" : "false", (a.probe & 15) ? "true" : "false");
    }
    if (alt) {
        HIPCHK(c, hipEventRecord(c->ev_join, st));
        c->s2_pending = true;
    }
    return HD_OK;
}

extern "C" int hd_run_dedisp_multi(hd_plan* const* plans, int32_t n)
{
    if (!plans || n <= 0) return fail(nullptr, HD_E_INVAL, "hd_run_dedisp_multi: need n >= 1 plans");
    for (int32_t i = 0; i < n; i++)
        if (!plans[i]) return fail(nullptr, HD_E_INVAL, "hd_run_dedisp_multi: plan %d is NULL", (int)i);
    hd_ctx* c = plans[0]->ctx;
    for (int32_t i = 1; i < n; i++)
        if (plans[i]->ctx != c) return fail(c, HD_E_INVAL, "hd_run_dedisp_multi: plans of different contexts");
    for (int32_t i = 0; i < n; i++)
        for (int32_t j = 0; j < i; j++)
            if (plans[i] == plans[j]) return fail(c, HD_E_INVAL, "hd_run_dedisp_multi: plan %d repeated", (int)i);
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<bool> done((size_t)n, false);
    for (int32_t i = 0; i < n; i++) {
        if (done[i]) continue;
        if (!dedisp_multi_ok(plans[i]) || getenv("HD_DD_SINGLE")) {
            const int rc = hd_run_dedisp(plans[i], nullptr);
            if (rc) return rc;
            done[i] = true;
            continue;
        }
        std::vector<hd_plan*> g;
        for (int32_t j = i; j < n && (int)g.size() < hd::kS2MaxPass; j++)
            if (!done[j] && dedisp_multi_ok(plans[j]) && dedisp_same_group(plans[i], plans[j])) {
                g.push_back(plans[j]);
                done[j] = true;
            }
        const int rc = run_dedisp_group(c, g.data(), (int)g.size());
        if (rc) return rc;
    }
    return HD_OK;
}

extern "C" int hd_plan_launch_passes(const hd_plan* p, int32_t* npass)
{
    if (!p || !npass) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_plan_launch_passes: NULL argument");
    if (!p->ran_dd) return fail(p->ctx, HD_E_STATE, "hd_plan_launch_passes: run hd_run_dedisp first");
    *npass = p->s2passes;
    return HD_OK;
}

extern "C" int hd_write_series(hd_plan* p, const char* const* paths, int32_t wait)
{
    if (!p || !paths) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_write_series: NULL argument");
    hd_ctx* c = p->ctx;
    if (!p->ran_dd || !p->d_out) return fail(c, HD_E_STATE, "hd_write_series: run hd_run_dedisp first");
    for (int d = 0; d < p->pass.numdms; d++)
        if (!paths[d]) return fail(c, HD_E_INVAL, "hd_write_series: path %d is NULL", d);
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->writer) HIPCHK(c, hd::writer_open(&c->writer, c->device));
    if (!p->ev_copy) HIPCHK(c, hipEventCreateWithFlags(&p->ev_copy, hipEventDisableTiming));
    std::string err;
    int rc = hd::writer_series(c->writer, dd_end(p), p->d_out, p->out_stride, p->pass.numdms, p->numout, paths, err);
    // even after a failure part-way (a file that cannot be created, a copy that fails), the
    // chunks queued before it keep copying from p->d_out: a later hd_run_dedisp of this plan
    // must wait for them, so the copy event is recorded whatever rc is
    {
        const hipError_t e = hipEventRecord(p->ev_copy, hd::writer_stream(c->writer));
        if (e == hipSuccess) p->copy_pending = true;
        if (e != hipSuccess && rc == 0) HIPCHK(c, e);
    }
    if (rc) return fail(c, rc, "hd_write_series: %s", err.c_str());
    if (wait) return hd_wait_writes(c, nullptr, nullptr);
    return HD_OK;
}

extern "C" int hd_wait_writes(hd_ctx* c, double* write_seconds, int64_t* bytes)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_wait_writes: NULL context");
    if (write_seconds) *write_seconds = 0.0;
    if (bytes) *bytes = 0;
    if (!c->writer) return HD_OK;
    std::string err;
    if (hd::writer_wait(c->writer, err, write_seconds, bytes)) return fail(c, HD_E_IO, "hd_wait_writes: %s", err.c_str());
    return HD_OK;
}

extern "C" int hd_plan_last_ms(const hd_plan* p, float* ms_sub, float* ms_dd)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_plan_last_ms: NULL plan");
    hd_ctx* c = p->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    if (ms_sub) {
        *ms_sub = 0.0f;
        if (p->ran_sub) {
            HIPCHK(c, hipEventSynchronize(p->ev[1]));
            HIPCHK(c, hipEventElapsedTime(ms_sub, p->ev[0], p->ev[1]));
        }
    }
    if (ms_dd) {
        *ms_dd = 0.0f;
        if (p->ran_dd) {
            HIPCHK(c, hipEventSynchronize(dd_end(p)));
            if (p->s2passes > 0) HIPCHK(c, hipEventElapsedTime(ms_dd, dd_start(p), dd_end(p)));
        }
    }
    return HD_OK;
}

// ---- realfft / zapbirds / rednoise (hd_fft.hip; replace the per-.dat PRESTO commands of
//      PALFA2_presto_search.py:548-558) ---------------------------------------------------
extern "C" int hd_plan_kernel(const hd_plan* p, char* name, int32_t cap)
{
    if (!p || !name || cap < 1) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_plan_kernel: bad argument");
    if (!p->ran_dd) return fail(p->ctx, HD_E_STATE, "hd_plan_kernel: run hd_run_dedisp first");
    snprintf(name, (size_t)cap, "%s", p->s2name);
    return HD_OK;
}

extern "C" int hd_realfft(hd_plan* p)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_realfft: NULL plan");
    hd_ctx* c = p->ctx;
    if (!p->ran_dd || !p->d_out) return fail(c, HD_E_STATE, "hd_realfft: run hd_run_dedisp first");
    if (p->numout < 4 || p->numout % 2) return fail(c, HD_E_INVAL, "hd_realfft: numout %lld must be even, >= 4",
                                                    (long long)p->numout);
    if (p->out_stride > INT32_MAX) return fail(c, HD_E_INVAL, "hd_realfft: series stride beyond 2^31");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t st = p->dd_stream ? p->dd_stream : c->stream;
    const auto key = std::make_tuple(p->numout, p->pass.numdms, p->out_stride);
    hd::FftState*& st_fft = c->fft_cache[key];
    if (!st_fft) st_fft = hd::fft_state_new();
    p->fft = st_fft;
    hd::fft_set_owner(p->fft, nullptr);            // (a failed transform leaves no owner)
    HIPCHK(c, hd::fft_series(p->fft, p->d_out, p->out_stride, p->numout, p->pass.numdms, st));
    hd::fft_set_owner(p->fft, p);
    p->ran_fft = true;
    return HD_OK;
}

extern "C" int hd_fft_prepare(hd_plan* p)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_fft_prepare: NULL plan");
    hd_ctx* c = p->ctx;
    if (p->numout < 4 || p->numout % 2) return fail(c, HD_E_INVAL, "hd_fft_prepare: numout %lld must be even, >= 4",
                                                    (long long)p->numout);
    if (p->out_stride > INT32_MAX) return fail(c, HD_E_INVAL, "hd_fft_prepare: series stride beyond 2^31");
    HIPCHK(c, hipSetDevice(c->device));
    const auto key = std::make_tuple(p->numout, p->pass.numdms, p->out_stride);
    hd::FftState*& st_fft = c->fft_cache[key];
    if (!st_fft) st_fft = hd::fft_state_new();
    HIPCHK(c, hd::fft_prepare(st_fft, p->out_stride, p->numout, p->pass.numdms));
    return HD_OK;
}

extern "C" int hd_zap_ranges(const double* lobins, const double* hibins, int32_t n, int64_t numbins, int32_t* rng4,
                             int32_t cap, int32_t* nr)
{
    if (!nr || n < 0 || (n > 0 && (!lobins || !hibins)) || (cap > 0 && !rng4) || numbins < 2)
        return fail(nullptr, HD_E_INVAL, "hd_zap_ranges: bad argument");
    std::vector<std::pair<int64_t, int64_t>> r;
    for (int32_t i = 0; i < n; i++) {
        if (!(lobins[i] <= hibins[i])) continue;
        int64_t lo = (int64_t)std::floor(lobins[i]), hi = (int64_t)std::ceil(hibins[i]);
        lo = std::max<int64_t>(lo, 1);
        hi = std::min<int64_t>(hi, numbins);
        if (lo < hi) r.emplace_back(lo, hi);
    }
    std::sort(r.begin(), r.end());
    std::vector<std::pair<int64_t, int64_t>> m;
    for (auto& x : r) {
        if (!m.empty() && x.first <= m.back().second) m.back().second = std::max(m.back().second, x.second);
        else m.push_back(x);
    }
    *nr = (int32_t)m.size();
    if ((int64_t)m.size() > cap) return fail(nullptr, HD_E_NOMEM, "hd_zap_ranges: %zu ranges > cap %d", m.size(), cap);
    for (size_t k = 0; k < m.size(); k++) {
        const int64_t lo = m[k].first, hi = m[k].second;
        const int64_t side = std::min<int64_t>(std::max<int64_t>(50, hi - lo), 2048);
        rng4[4 * k + 0] = (int32_t)lo;
        rng4[4 * k + 1] = (int32_t)hi;
        rng4[4 * k + 2] = (int32_t)std::max<int64_t>(1, lo - side);
        rng4[4 * k + 3] = (int32_t)std::min<int64_t>(numbins, hi + side);
    }
    return HD_OK;
}

extern "C" int hd_zapbirds(hd_plan* p, const double* lobins, const double* hibins, int32_t n)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_zapbirds: NULL plan");
    hd_ctx* c = p->ctx;
    if (!p->ran_fft) return fail(c, HD_E_STATE, "hd_zapbirds: run hd_realfft first");
    if (hd::fft_owner(p->fft) != p)
        return fail(c, HD_E_STATE, "hd_zapbirds: the spectra were replaced by another plan's hd_realfft (same geometry)");
    const int64_t nb = p->numout / 2;
    if (nb > INT32_MAX) return fail(c, HD_E_INVAL, "hd_zapbirds: spectrum beyond 2^31 bins");
    int32_t nr = 0;
    int rc = hd_zap_ranges(lobins, hibins, n, nb, nullptr, 0, &nr);
    if (rc && rc != HD_E_NOMEM) return fail(c, rc, "hd_zapbirds: %s", g_err.c_str());
    std::vector<int32_t> rng((size_t)4 * std::max(nr, 1));
    rc = hd_zap_ranges(lobins, hibins, n, nb, rng.data(), nr, &nr);
    if (rc) return fail(c, rc, "hd_zapbirds: %s", g_err.c_str());
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t st = p->dd_stream ? p->dd_stream : c->stream;
    HIPCHK(c, hd::fft_zap(p->fft, rng.data(), nr, st));
    return HD_OK;
}

extern "C" int hd_rednoise_blocks(int64_t numbins, double T, int32_t startwidth, int32_t endwidth, double endfreq,
                                  int32_t* boff, int32_t cap, int32_t* nblk)
{
    if (!nblk || numbins < 2 || !(T > 0.0) || startwidth < 1 || endwidth < startwidth || endwidth > 128 ||
        !(endfreq > 0.0) || (cap > 0 && !boff) || numbins > INT32_MAX)
        return fail(nullptr, HD_E_INVAL, "hd_rednoise_blocks: bad argument");
    const double lg = std::log(1.0 + endfreq);
    int64_t o = 1;
    int32_t k = 0;
    while (o < numbins) {
        const double f = (double)o / T;
        int64_t w = endwidth;
        if (f < endfreq) w = startwidth + (int64_t)std::floor((double)(endwidth - startwidth) * std::log(1.0 + f) / lg);
        if (k < cap) boff[k] = (int32_t)o;
        k++;
        o = std::min(numbins, o + w);
    }
    if (k < cap) boff[k] = (int32_t)numbins;
    *nblk = k;
    if (k + 1 > cap) return fail(nullptr, HD_E_NOMEM, "hd_rednoise_blocks: %d offsets > cap %d", k + 1, cap);
    return HD_OK;
}

extern "C" int hd_rednoise(hd_plan* p, int32_t startwidth, int32_t endwidth, double endfreq, double T)
{
    if (!p) return fail(nullptr, HD_E_INVAL, "hd_rednoise: NULL plan");
    hd_ctx* c = p->ctx;
    if (!p->ran_fft) return fail(c, HD_E_STATE, "hd_rednoise: run hd_realfft first");
    if (hd::fft_owner(p->fft) != p)
        return fail(c, HD_E_STATE, "hd_rednoise: the spectra were replaced by another plan's hd_realfft (same geometry)");
    const int64_t nb = p->numout / 2;
    int32_t nblk = 0;
    int rc = hd_rednoise_blocks(nb, T, startwidth, endwidth, endfreq, nullptr, 0, &nblk);
    if (rc && rc != HD_E_NOMEM) return fail(c, rc, "hd_rednoise: %s", g_err.c_str());
    std::vector<int32_t> boff((size_t)nblk + 1);
    rc = hd_rednoise_blocks(nb, T, startwidth, endwidth, endfreq, boff.data(), nblk + 1, &nblk);
    if (rc) return fail(c, rc, "hd_rednoise: %s", g_err.c_str());
    std::vector<double> cen((size_t)nblk);
    for (int32_t j = 0; j < nblk; j++) cen[j] = (double)boff[j] + (double)(boff[j + 1] - boff[j] - 1) / 2.0;
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t st = p->dd_stream ? p->dd_stream : c->stream;
    HIPCHK(c, hd::fft_rednoise(p->fft, boff.data(), cen.data(), nblk, st));
    return HD_OK;
}

extern "C" int hd_get_fft(hd_plan* p, int32_t dm0, int32_t ndm, float* out)
{
    if (!p || !out) return fail(p ? p->ctx : nullptr, HD_E_INVAL, "hd_get_fft: NULL argument");
    hd_ctx* c = p->ctx;
    if (!p->ran_fft) return fail(c, HD_E_STATE, "hd_get_fft: run hd_realfft first");
    if (hd::fft_owner(p->fft) != p)
        return fail(c, HD_E_STATE, "hd_get_fft: the spectra were replaced by another plan's hd_realfft (same geometry)");
    if (dm0 < 0 || ndm < 1 || dm0 + ndm > p->pass.numdms) return fail(c, HD_E_INVAL, "hd_get_fft: bad DM range");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t st = p->dd_stream ? p->dd_stream : c->stream;
    const int64_t fs = p->numout / 2 + 1;
    HIPCHK(c, hd::fft_begin(p->fft, st));          // after the last op on the shared spectra
    HIPCHK(c, d2h_2d(out, sizeof(float) * p->numout, hd::fft_buffer(p->fft) + (size_t)dm0 * fs,
                     sizeof(float2) * fs, sizeof(float) * p->numout, ndm, st));
    HIPCHK(c, hd::fft_end(p->fft, st));
    return HD_OK;
}

// ---- in-library collectives: RCCL over xGMI, loaded at run time ------------------------
// librccl is dlopen'ed on first use (a process that already holds one -- torch's -- gets that
// one back by soname), so the library has no link-time RCCL dependency and a caller that
// never makes a communicator never loads it.  The types come from the ROCm header.
namespace {
struct RcclApi {
    bool ok = false;
    std::string err;
    ncclResult_t (*get_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    const char* (*errstr)(ncclResult_t) = nullptr;
};
const RcclApi& rccl()
{
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        // The RCCL must run on the HIP runtime this library runs on.  A process can hold two:
        // torch's wheel ships its own libamdhip64/librccl, and when this library is loaded
        // before torch, torch maps a second HIP runtime and its librccl.so.1 -- which a plain
        // dlopen("librccl.so.1") then returns (soname match), an RCCL whose runtime knows
        // neither our device buffers nor our streams (bench --comm hd measured 3.9 s per beam
        // that way).  So load librccl from OUR runtime's directory, by path, and check it.
        hipError_t (*const ours)(int*) = hipGetDeviceCount;    // a runtime entry point, as bound for us
        Dl_info di{};
        std::string rtdir;
        if (dladdr((void*)ours, &di) && di.dli_fname) {
            rtdir = di.dli_fname;
            rtdir = rtdir.substr(0, rtdir.find_last_of('/') + 1);
        }
        // HD_TEST_NO_RCCL=1 (CPU tests) takes the not-found path without touching the loader
        if (!getenv("HD_TEST_NO_RCCL")) {
            for (const char* n : {"librccl.so.1", "librccl.so"})
                if (!rtdir.empty() && (h = dlopen((rtdir + n).c_str(), RTLD_NOW | RTLD_LOCAL))) break;
            if (!h)
                for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
                    if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        }
        if (!h) {
            // dlerror() clears the message it returns: read it once
            const char* de = getenv("HD_TEST_NO_RCCL") ? nullptr : dlerror();
            api.err = de ? de : "librccl not found";
            return;
        }
        // the HIP runtime the loaded RCCL resolves against must be ours
        void* their = dlsym(h, "hipGetDeviceCount");
        Dl_info dr{};
        if (their && their != (void*)ours) {
            std::string rp = dladdr(their, &dr) && dr.dli_fname ? dr.dli_fname : "?";
            api.err = "librccl in this process runs on another HIP runtime (" + rp + ", this library: " +
                      (di.dli_fname ? std::string(di.dli_fname) : std::string("?")) +
                      "); load libhipdedisp after torch, or use torch.distributed for the exchanges";
            return;
        }
        api.get_id = (decltype(api.get_id))dlsym(h, "ncclGetUniqueId");
        api.init_rank = (decltype(api.init_rank))dlsym(h, "ncclCommInitRank");
        api.all_reduce = (decltype(api.all_reduce))dlsym(h, "ncclAllReduce");
        api.destroy = (decltype(api.destroy))dlsym(h, "ncclCommDestroy");
        api.errstr = (decltype(api.errstr))dlsym(h, "ncclGetErrorString");
        api.ok = api.get_id && api.init_rank && api.all_reduce && api.destroy && api.errstr;
        if (!api.ok) api.err = "librccl lacks the nccl* entry points";
    });
    return api;
}
}  // namespace

#define RCCLCHK(c, x)                                                                                        \
    do {                                                                                                    \
        const ncclResult_t r_ = (x);                                                                        \
        if (r_ != ncclSuccess) return fail((c), HD_E_HIP, "%s failed: %s", #x, rccl().errstr(r_));          \
    } while (0)

extern "C" int hd_comm_unique_id(uint8_t* id)
{
    if (!id) return fail(nullptr, HD_E_INVAL, "hd_comm_unique_id: NULL id");
    const RcclApi& r = rccl();
    if (!r.ok) return fail(nullptr, HD_E_HIP, "hd_comm_unique_id: %s", r.err.c_str());
    ncclUniqueId u;
    RCCLCHK(nullptr, r.get_id(&u));
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return HD_OK;
}

extern "C" int hd_comm_init(hd_ctx* c, const uint8_t* id, int32_t rank, int32_t world)
{
    if (!c || !id) return fail(c, HD_E_INVAL, "hd_comm_init: NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return fail(c, HD_E_INVAL, "hd_comm_init: rank %d of %d", rank, world);
    if (c->comm) return fail(c, HD_E_STATE, "hd_comm_init: the context already has a communicator");
    const RcclApi& r = rccl();
    if (!r.ok) return fail(c, HD_E_HIP, "hd_comm_init: %s", r.err.c_str());
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t comm = nullptr;
    RCCLCHK(c, r.init_rank(&comm, world, u, rank));       // collective: every rank of the id
    c->comm = comm;
    c->comm_rank = rank;
    c->comm_world = world;
    return HD_OK;
}

static int comm_scratch(hd_ctx* c, size_t bytes)
{
    if (c->comm_bytes >= bytes) return HD_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dfree(c->d_comm);
    c->d_comm = nullptr;
    c->comm_bytes = 0;
    HIPCHK(c, hipMalloc(&c->d_comm, bytes));
    c->comm_bytes = bytes;
    return HD_OK;
}

extern "C" int hd_comm_allreduce_sum_f64(hd_ctx* c, double* buf, int64_t n)
{
    if (!c || (n > 0 && !buf) || n < 0) return fail(c, HD_E_INVAL, "hd_comm_allreduce_sum_f64: bad argument");
    if (!c->comm) return fail(c, HD_E_STATE, "hd_comm_allreduce_sum_f64: no communicator (hd_comm_init)");
    if (n == 0) return HD_OK;
    HIPCHK(c, hipSetDevice(c->device));
    hipPointerAttribute_t at{};
    const bool dev = hipPointerGetAttributes(&at, buf) == hipSuccess && at.type == hipMemoryTypeDevice;
    (void)hipGetLastError();
    double* d = buf;
    const size_t bytes = (size_t)n * sizeof(double);
    if (!dev) {
        int rc = comm_scratch(c, bytes);
        if (rc) return rc;
        d = c->d_comm;
        HIPCHK(c, hipMemcpyAsync(d, buf, bytes, hipMemcpyHostToDevice, c->stream));
    }
    RCCLCHK(c, rccl().all_reduce(d, d, (size_t)n, ncclFloat64, ncclSum, (ncclComm_t)c->comm, c->stream));
    if (!dev) HIPCHK(c, hipMemcpyAsync(buf, d, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return HD_OK;
}

extern "C" int hd_slice_exchange_clip(hd_ctx* c, int64_t nown, int64_t nblk_total)
{
    if (!c) return fail(nullptr, HD_E_INVAL, "hd_slice_exchange_clip: NULL context");
    if (!c->comm) return fail(c, HD_E_STATE, "hd_slice_exchange_clip: no communicator (hd_comm_init)");
    if (!(c->opts.clip_sigma > 0.0f)) return HD_OK;
    if (nblk_total < 1 || nown < 0) return fail(c, HD_E_INVAL, "hd_slice_exchange_clip: bad block counts");
    // hd_clip_stats writes rows up to slice_t0/blk + nown and hd_clip_set_stats reads rows up
    // to slice_t0/blk + nblk of the [nblk_total] table
    if (nown > c->nblk || nblk_total < c->slice_t0 / c->blk + c->nblk)
        return fail(c, HD_E_INVAL, "hd_slice_exchange_clip: nown %lld > %d blocks, or nblk_total %lld < %lld",
                    (long long)nown, c->nblk, (long long)nblk_total, (long long)(c->slice_t0 / c->blk + c->nblk));
    HIPCHK(c, hipSetDevice(c->device));
    // the beam's [nblk_total][nchan + 3] statistics table on the device: this slice's own
    // rows (hd_clip_stats), summed over the ranks, then clip_times finished (hd_clip_set_stats)
    const size_t n = (size_t)nblk_total * ((size_t)c->obs.nchan + 3);
    int rc = comm_scratch(c, n * sizeof(double));
    if (rc) return rc;
    HIPCHK(c, hipMemsetAsync(c->d_comm, 0, n * sizeof(double), c->stream));
    rc = hd_clip_stats(c, nown, c->d_comm);
    if (rc) return rc;
    rc = hd_comm_allreduce_sum_f64(c, c->d_comm, (int64_t)n);
    if (rc) return rc;
    return hd_clip_set_stats(c, c->d_comm);
}

extern "C" int hd_comm_destroy(hd_ctx* c)
{
    if (!c) return HD_OK;
    if (c->comm) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        (void)rccl().destroy((ncclComm_t)c->comm);
        c->comm = nullptr;
    }
    dfree(c->d_comm);
    c->d_comm = nullptr;
    c->comm_bytes = 0;
    c->comm_rank = c->comm_world = 0;
    return HD_OK;
}
