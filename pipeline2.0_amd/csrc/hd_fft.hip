// hd_fft.hip — the FFT, birdie zapping and de-reddening of a pass's device-resident DM series:
// what the reference runs on every .dat after the single-pulse search
// (lib/python/PALFA2_presto_search.py:548-558):
//     realfft <dat>;  zapbirds -zap -zapfile <zaplist> -baryv <v> <fft>;  rednoise <fft>
// [PRESTO-ext, parity with PRESTO unpinned: none of the three is in this image] restated:
//   * realfft: the forward real FFT of the numout samples (hipFFT R2C, float32, no
//     normalisation), stored as PRESTO's packed .fft: numout/2 complex bins, bin 0 holding
//     (DC, Nyquist) as its (real, imaginary) parts;
//   * zapbirds: the host turns the zaplist into bin ranges [lo, hi) (merged where they touch);
//     each range's bins are set to (sqrt(median / ln 2), 0), the median (the lower one, element
//     (n - 1) / 2 of the sorted values) taken over the powers of up to kZapSide bins on either
//     side of the range in the un-zapped spectrum (all ranges see the same input, so the
//     result does not depend on their order);
//   * rednoise: bins 1 .. numout/2 - 1 in consecutive blocks whose widths the host lays out
//     (growing from startwidth to endwidth bins at endfreq); each block's median power; every
//     bin scaled by 1 / sqrt(m / ln 2), m the median linearly interpolated between the block
//     centres (held flat before the first and after the last); bin 0 becomes (1, 0).
// Powers and scales are double, with no fused multiply-adds, so oracle/fft_oracle.py gives
// the zap and rednoise outputs bit for bit from the same FFT.
#include <hipfft/hipfft.h>

#include "hd_internal.h"

#pragma clang fp contract(off)

namespace hd {

constexpr int kZapMaxWin = 4096;     // values per zap median (both sides together)
constexpr double kLn2 = 0.69314718055994530942;

__device__ __forceinline__ double bin_power(float2 z)
{
    return (double)z.x * (double)z.x + (double)z.y * (double)z.y;   // each product exact
}

// PRESTO packing: bin 0 = (DC, Nyquist).  One thread per DM series.
__global__ void k_fft_pack(float2* __restrict__ F, int64_t fstride, int64_t nb, int ndm)
{
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= ndm) return;
    float2* f = F + (int64_t)d * fstride;
    f[0].y = f[nb].x;
}

// Bitonic sort of n (a power of two, <= kZapMaxWin) doubles in LDS by the whole workgroup.
__device__ void lds_bitonic(double* v, int n)
{
    for (int k = 2; k <= n; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                const int l = i ^ j;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    const double a = v[i], b = v[l];
                    if ((a > b) == up) {
                        v[i] = b;
                        v[l] = a;
                    }
                }
            }
            __syncthreads();
        }
}

// Median of the window around zap range b of series blockIdx.y: ranges [lo, hi) and window
// [wlo, lo) u [hi, whi) (int4 {lo, hi, wlo, whi}).
__global__ __launch_bounds__(256) void k_zap_median(const float2* __restrict__ F, int64_t fstride,
                                                    const int4* __restrict__ rng, double* __restrict__ med, int nr)
{
    __shared__ double v[kZapMaxWin];
    const int4 r = rng[blockIdx.x];
    const float2* f = F + (int64_t)blockIdx.y * fstride;
    const int nl = r.x - r.z, n = nl + (r.w - r.y);
    int np = 64;
    while (np < n) np <<= 1;
    for (int i = threadIdx.x; i < np; i += blockDim.x)
        v[i] = i < n ? bin_power(f[i < nl ? r.z + i : r.y + (i - nl)]) : __builtin_inf();
    __syncthreads();
    lds_bitonic(v, np);
    if (threadIdx.x == 0) med[(int64_t)blockIdx.y * nr + blockIdx.x] = n > 0 ? v[(n - 1) / 2] : 0.0;
}

__global__ __launch_bounds__(256) void k_zap_apply(float2* __restrict__ F, int64_t fstride,
                                                   const int4* __restrict__ rng, const double* __restrict__ med, int nr)
{
    const int4 r = rng[blockIdx.x];
    float2* f = F + (int64_t)blockIdx.y * fstride;
    const float a = (float)sqrt(med[(int64_t)blockIdx.y * nr + blockIdx.x] / kLn2);
    for (int i = r.x + threadIdx.x; i < r.y; i += blockDim.x) f[i] = make_float2(a, 0.0f);
}

// One wave per (block, series): the lower median of the block's powers (width <= 128): a
// bitonic sort of 128 slots (+inf past the block) held two per lane (slot lane + 64 h),
// cross-lane steps by __shfl_xor; the median is slot (n - 1) / 2.
__global__ __launch_bounds__(256) void k_red_median(const float2* __restrict__ F, int64_t fstride,
                                                    const int32_t* __restrict__ boff, int nblk, int ndm,
                                                    double* __restrict__ med)
{
    const int lane = threadIdx.x & 63;
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int d = blockIdx.y;
    if (j >= nblk) return;
    const int o = boff[j], n = boff[j + 1] - o;
    const float2* f = F + (int64_t)d * fstride + o;
    double v0 = lane < n ? bin_power(f[lane]) : __builtin_inf();
    double v1 = lane + 64 < n ? bin_power(f[lane + 64]) : __builtin_inf();
#pragma unroll
    for (int k = 2; k <= 128; k <<= 1) {
#pragma unroll
        for (int s = k >> 1; s > 0; s >>= 1) {
            if (s == 64) {                                   // partner: the same lane's other slot
                const bool up = (lane & k) == 0;             // k == 128: always ascending
                const double lo = fmin(v0, v1), hi = fmax(v0, v1);
                v0 = up ? lo : hi;
                v1 = up ? hi : lo;
            } else {
                const bool first = (lane & s) == 0;
                const bool up0 = (lane & k) == 0, up1 = ((lane + 64) & k) == 0;
                const double p0 = __shfl_xor(v0, s, 64), p1 = __shfl_xor(v1, s, 64);
                v0 = (first == up0) ? fmin(v0, p0) : fmax(v0, p0);
                v1 = (first == up1) ? fmin(v1, p1) : fmax(v1, p1);
            }
        }
    }
    const int k = (n - 1) / 2;
    if (lane == (k & 63)) med[(int64_t)d * nblk + j] = k < 64 ? v0 : v1;
}

// Block j (blockIdx.x, <= 128 bins) of series blockIdx.y: each bin scaled by
// 1 / sqrt(m / ln 2), m interpolated between the medians of the neighbouring block centres
// cen[] (double).  Block 0's workgroup also sets bin 0 to (1, 0).
__global__ __launch_bounds__(128) void k_red_scale(float2* __restrict__ F, int64_t fstride,
                                                   const int32_t* __restrict__ boff, const double* __restrict__ cen,
                                                   int nblk, int ndm, const double* __restrict__ med)
{
    const int j = blockIdx.x;
    const int o = boff[j], n = boff[j + 1] - o;
    const int t = threadIdx.x;
    const int i = o + t;
    const double c = cen[j];
    const bool left = (double)i < c;
    const int ja = left ? j - 1 : j, jb = left ? j : j + 1;
    {
        const int d = blockIdx.y;
        float2* f = F + (int64_t)d * fstride;
        if (j == 0 && t == 0) f[0] = make_float2(1.0f, 0.0f);
        if (t >= n) return;
        const double* m = med + (int64_t)d * nblk;
        double mi;
        if (ja < 0) mi = m[0];
        else if (jb >= nblk) mi = m[nblk - 1];
        else mi = m[ja] + (m[jb] - m[ja]) * (((double)i - cen[ja]) / (cen[jb] - cen[ja]));
        const float2 z = f[i];
        if (mi > 0.0) {
            const double s = 1.0 / sqrt(mi / kLn2);
            f[i] = make_float2((float)((double)z.x * s), (float)((double)z.y * s));
        } else {
            f[i] = make_float2(0.0f, 0.0f);
        }
    }
}

// ---- host side --------------------------------------------------------------------------

struct FftState {
    const void* owner = nullptr;    // the plan whose spectra d_fft holds (hd_api.hip)
    hipfftHandle plan = 0;
    bool have_plan = false;
    int64_t n = 0;
    int ndm = 0;
    float2* d_fft = nullptr;        // [ndm][n/2 + 1]
    int4* d_rng = nullptr;
    double* d_med = nullptr;
    int32_t* d_boff = nullptr;
    double* d_cen = nullptr;
    size_t rng_cap = 0, med_cap = 0, boff_cap = 0, cen_cap = 0;
    // plans of the same geometry share this state from different stage-2 streams: every op
    // on it waits for the last one's event and records its own (fft_begin / fft_end)
    hipEvent_t done = nullptr;
    bool pending = false;
};

FftState* fft_state_new() { return new FftState(); }

void fft_state_free(FftState* s)
{
    if (!s) return;
    if (s->pending) (void)hipEventSynchronize(s->done);
    if (s->done) (void)hipEventDestroy(s->done);
    if (s->have_plan) hipfftDestroy(s->plan);
    (void)hipFree(s->d_fft);
    (void)hipFree(s->d_rng);
    (void)hipFree(s->d_med);
    (void)hipFree(s->d_boff);
    (void)hipFree(s->d_cen);
    delete s;
}

float2* fft_buffer(FftState* s) { return s ? s->d_fft : nullptr; }
const void* fft_owner(const FftState* s) { return s ? s->owner : nullptr; }
void fft_set_owner(FftState* s, const void* owner)
{
    if (s) s->owner = owner;
}

// Order work on the shared state after the previous op (whatever its stream) / record its end.
hipError_t fft_begin(FftState* s, hipStream_t st)
{
    if (!s->done) {
        hipError_t e = hipEventCreateWithFlags(&s->done, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    return s->pending ? hipStreamWaitEvent(st, s->done, 0) : hipSuccess;
}

hipError_t fft_end(FftState* s, hipStream_t st)
{
    hipError_t e = hipEventRecord(s->done, st);
    s->pending = e == hipSuccess;
    return e;
}

// the hipFFT plan and spectra buffer of a geometry (rocFFT builds its kernels here: seconds
// for a new size, so hd_fft_prepare can run it ahead of the timed path)
hipError_t fft_prepare(FftState* s, int64_t xstride, int64_t n, int ndm)
{
    if (n < 4 || (n & 1) || ndm < 1) return hipErrorInvalidValue;
    if (s->n == n && s->ndm == ndm && s->d_fft) return hipSuccess;
    if (s->pending) {
        const hipError_t e = hipEventSynchronize(s->done);
        if (e != hipSuccess) return e;
        s->pending = false;
    }
    const int64_t fs = n / 2 + 1;
    if (s->have_plan) hipfftDestroy(s->plan);
    s->have_plan = false;
    (void)hipFree(s->d_fft);
    s->d_fft = nullptr;
    hipError_t e = hipMalloc(&s->d_fft, sizeof(float2) * (size_t)fs * ndm);
    if (e != hipSuccess) return e;
    int nn = (int)n;
    int inembed = (int)xstride, onembed = (int)fs;
    if (hipfftPlanMany(&s->plan, 1, &nn, &inembed, 1, (int)xstride, &onembed, 1, (int)fs, HIPFFT_R2C, ndm) !=
        HIPFFT_SUCCESS)
        return hipErrorUnknown;
    s->have_plan = true;
    s->n = n;
    s->ndm = ndm;
    return hipSuccess;
}

hipError_t fft_series(FftState* s, const float* x, int64_t xstride, int64_t n, int ndm, hipStream_t st)
{
    if (n < 4 || (n & 1) || ndm < 1) return hipErrorInvalidValue;
    {
        hipError_t e = fft_begin(s, st);
        if (e != hipSuccess) return e;
    }
    const int64_t fs = n / 2 + 1;
    {
        hipError_t e = fft_prepare(s, xstride, n, ndm);
        if (e != hipSuccess) return e;
    }
    if (hipfftSetStream(s->plan, st) != HIPFFT_SUCCESS ||
        hipfftExecR2C(s->plan, (hipfftReal*)x, (hipfftComplex*)s->d_fft) != HIPFFT_SUCCESS)
        return hipErrorUnknown;
    hipLaunchKernelGGL(k_fft_pack, dim3((ndm + 63) / 64), dim3(64), 0, st, s->d_fft, fs, n / 2, ndm);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? fft_end(s, st) : e;
}

template <class T>
static hipError_t grow(T** p, size_t* cap, size_t n, hipStream_t st)
{
    if (*cap >= n) return hipSuccess;
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    e = hipMalloc(p, sizeof(T) * n);
    if (e == hipSuccess) *cap = n;
    return e;
}

hipError_t fft_zap(FftState* s, const int32_t* rng4, int nr, hipStream_t st)
{
    if (!s->d_fft) return hipErrorInvalidValue;
    if (nr == 0) return hipSuccess;
    hipError_t e = fft_begin(s, st);
    if (e == hipSuccess) e = grow(&s->d_rng, &s->rng_cap, (size_t)nr, st);
    if (e == hipSuccess) e = grow(&s->d_med, &s->med_cap, (size_t)nr * s->ndm, st);
    if (e == hipSuccess) e = hipMemcpyAsync(s->d_rng, rng4, sizeof(int4) * nr, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);     // rng4 is the caller's (pageable) memory
    if (e != hipSuccess) return e;
    const int64_t fs = s->n / 2 + 1;
    hipLaunchKernelGGL(k_zap_median, dim3(nr, s->ndm), dim3(256), 0, st, s->d_fft, fs, s->d_rng, s->d_med, nr);
    hipLaunchKernelGGL(k_zap_apply, dim3(nr, s->ndm), dim3(256), 0, st, s->d_fft, fs, s->d_rng, s->d_med, nr);
    e = hipGetLastError();
    return e == hipSuccess ? fft_end(s, st) : e;
}

hipError_t fft_rednoise(FftState* s, const int32_t* boff, const double* cen, int nblk, hipStream_t st)
{
    if (!s->d_fft || nblk < 1) return hipErrorInvalidValue;
    hipError_t e = fft_begin(s, st);
    if (e == hipSuccess) e = grow(&s->d_boff, &s->boff_cap, (size_t)nblk + 1, st);
    if (e == hipSuccess) e = grow(&s->d_cen, &s->cen_cap, (size_t)nblk, st);
    if (e == hipSuccess) e = grow(&s->d_med, &s->med_cap, (size_t)nblk * s->ndm, st);
    if (e == hipSuccess) e = hipMemcpyAsync(s->d_boff, boff, sizeof(int32_t) * (nblk + 1), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(s->d_cen, cen, sizeof(double) * nblk, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    const int64_t fs = s->n / 2 + 1;
    hipLaunchKernelGGL(k_red_median, dim3((nblk + 3) / 4, s->ndm), dim3(256), 0, st, s->d_fft, fs, s->d_boff, nblk,
                       s->ndm, s->d_med);
    hipLaunchKernelGGL(k_red_scale, dim3(nblk, s->ndm), dim3(128), 0, st, s->d_fft, fs, s->d_boff, s->d_cen, nblk,
                       s->ndm, s->d_med);
    e = hipGetLastError();
    return e == hipSuccess ? fft_end(s, st) : e;
}

}  // namespace hd
