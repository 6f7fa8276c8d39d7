// hd_rfi.hip — rfifind's per-interval statistics on the device-resident raw block: the step
// just before the hot path (lib/python/PALFA2_presto_search.py:482-490,
// `rfifind -time <rfifind_chunk_time> -o <base> <files>`), whose .mask / .stats feed stage 1.
// [PRESTO-ext] restated (rfifind.c): for every interval of ptsperint spectra and every
// channel, the samples as rfifind reads them (clip_times applied, no mask yet), their mean
// and standard deviation (avg_var: two passes, the variance over n - 1), and the largest
// power of the interval's real FFT, bins 1 .. ptsperint/2 - 1, normalised by
// ptsperint * variance.  The mask decisions over these [numint][nchan] arrays are host work
// (hipdedisp/rfifind.py).  Sums are double in a fixed order (64 lane partials over samples
// l, l + 64, ..., then a xor butterfly) so oracle/rfifind_oracle.py reproduces the means and
// standard deviations exactly; the FFT is hipFFT (float32).
#include <hipfft/hipfft.h>

#include "hd_device.h"

#pragma clang fp contract(off)   // products and sums rounded separately, as the oracle does

namespace hd {

__device__ __forceinline__ double rfi_wave_sum(double v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// One wave per channel of interval t0 / n + blockIdx.y: the samples (float, into
// x[y][c][n] for the FFT), their mean and standard deviation into avg/sd/var [y][nchan].
// rawT (8/4-bit without calibration: one byte per sample, channel-major) or the generic
// decode; clipped spectra read as the block's pads.
__global__ __launch_bounds__(256) void k_rfi_chan(RawDesc rd, const uint8_t* __restrict__ rawT, int64_t tstride,
                                                  int64_t t0, int32_t n, float* __restrict__ x, float* __restrict__ avg,
                                                  float* __restrict__ sd, double* __restrict__ var_out)
{
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= rd.nchan) return;
    const int64_t cell = (int64_t)blockIdx.y * rd.nchan + c;
    t0 += (int64_t)blockIdx.y * n;
    const int rc = rd.flip ? rd.nchan - 1 - c : c;
    float* xc = x + cell * n;
    double s = 0.0;
    for (int i = lane; i < n; i += 64) {
        const int64_t t = t0 + i;
        float v;
        if (rd.clipped && rd.clipped[t]) v = pad_at(rd, blk_of(rd, t), c);
        else if (rawT) v = (float)rawT[(int64_t)rc * tstride + t];
        else v = raw_value(rd, t, c);
        xc[i] = v;
        s += (double)v;
    }
    s = rfi_wave_sum(s);
    const double mean = s / (double)n;
    double q = 0.0;
    for (int i = lane; i < n; i += 64) {
        const double d = (double)xc[i] - mean;
        q += d * d;
    }
    q = rfi_wave_sum(q);
    if (lane == 0) {
        const double var = n > 1 ? q / (double)(n - 1) : 0.0;
        avg[cell] = (float)mean;
        sd[cell] = (float)sqrt(var);
        var_out[cell] = var;
    }
}

// One wave per channel: max over bins 1 .. n/2 - 1 of |X_k|^2 / (n * var) (var 0: norm 1).
__global__ __launch_bounds__(256) void k_rfi_maxpow(const float2* __restrict__ X, int32_t n, int32_t nchan,
                                                    const double* __restrict__ var, float* __restrict__ pw)
{
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nchan) return;
    const int64_t cell = (int64_t)blockIdx.y * nchan + c;
    const float2* Xc = X + cell * (n / 2 + 1);
    double norm = var[cell] * (double)n;
    if (!(norm > 0.0)) norm = 1.0;
    const float fn = (float)norm;
    float m = 0.0f;
    for (int k = 1 + lane; k < n / 2; k += 64) {
        const float2 z = Xc[k];
        m = fmaxf(m, (z.x * z.x + z.y * z.y) / fn);
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) m = fmaxf(m, __shfl_xor(m, s, 64));
    if (lane == 0) pw[cell] = m;
}

// rfifind statistics of the intervals [0, numint) into avg/sd/pw [numint][nchan] (device),
// kRfiBatch intervals per launch (nchan * kRfiBatch waves, one batched R2C plan).
constexpr int kRfiBatch = 16;

hipError_t rfi_stats(const RawDesc& rd, const uint8_t* rawT, int64_t tstride, int ptsperint, int numint, float* avg,
                     float* sd, float* pw, hipStream_t st)
{
    if (ptsperint < 4 || (ptsperint & 1) || numint < 1) return hipErrorInvalidValue;
    const int nch = rd.nchan;
    const int kb = numint < kRfiBatch ? numint : kRfiBatch;
    const size_t cells = (size_t)nch * kb;
    float* x = nullptr;
    float2* X = nullptr;
    double* var = nullptr;
    hipError_t e = hipMalloc(&x, sizeof(float) * cells * ptsperint);
    if (e == hipSuccess) e = hipMalloc(&X, sizeof(float2) * cells * (ptsperint / 2 + 1));
    if (e == hipSuccess) e = hipMalloc(&var, sizeof(double) * cells);
    hipfftHandle plans[2] = {0, 0};
    int have = 0;
    const int tail = numint % kb;
    for (int k = 0; k < (tail ? 2 : 1) && e == hipSuccess; k++) {
        int nn = ptsperint;
        const int batch = nch * (k ? tail : kb);
        if (hipfftPlanMany(&plans[k], 1, &nn, nullptr, 1, ptsperint, nullptr, 1, ptsperint / 2 + 1, HIPFFT_R2C,
                           batch) != HIPFFT_SUCCESS)
            e = hipErrorUnknown;
        else if (have++, hipfftSetStream(plans[k], st) != HIPFFT_SUCCESS)
            e = hipErrorUnknown;
    }
    const unsigned grid = (unsigned)((nch + 3) / 4);
    for (int ii = 0; ii < numint && e == hipSuccess; ii += kb) {
        const int m = numint - ii < kb ? numint - ii : kb;
        const size_t o = (size_t)ii * nch;
        hipLaunchKernelGGL(k_rfi_chan, dim3(grid, m), dim3(256), 0, st, rd, rawT, tstride, (int64_t)ii * ptsperint,
                           ptsperint, x, avg + o, sd + o, var);
        e = hipGetLastError();
        if (e == hipSuccess &&
            hipfftExecR2C(plans[m == kb ? 0 : 1], (hipfftReal*)x, (hipfftComplex*)X) != HIPFFT_SUCCESS)
            e = hipErrorUnknown;
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_rfi_maxpow, dim3(grid, m), dim3(256), 0, st, X, ptsperint, nch, var, pw + o);
            e = hipGetLastError();
        }
    }
    const hipError_t es = hipStreamSynchronize(st);   // the scratch buffers are freed below
    if (e == hipSuccess) e = es;
    for (int k = 0; k < have; k++) hipfftDestroy(plans[k]);
    if (x) (void)hipFree(x);
    if (X) (void)hipFree(X);
    if (var) (void)hipFree(var);
    return e;
}

}  // namespace hd
