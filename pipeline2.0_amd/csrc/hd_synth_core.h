// hd_synth_core.h — synthetic PALFA-like beam generator shared by host and device.
//
// Integer-only arithmetic: the host (hd_synth_host) and device (hd_synth_device)
// builds of these functions produce identical bytes, which lets the tests feed the
// same beam to the GPU engine and to the CPU oracle without copying 4 GB back.
//
// Model: per-channel Gaussian-like noise around a sloped bandpass,
// dispersed periodic pulsars and single pulses (delay law dm / (0.000241 f^2) s,
// relative to the top of the band), persistent narrowband RFI channels, bursty
// (interval, channel) RFI cells and zero-DM broadband spikes; quantised to NBITS.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define HD_HD __host__ __device__ __forceinline__
#else
#define HD_HD static inline
#endif

#define HD_SYNTH_MAXPSR 8

// Host-precomputed tables. Fixed-point conventions: levels in 1/16 digitiser units
// ("q4"), times in 1/65536 sample ("fp16").
struct hd_synth_tab {
    int32_t  nchan, nbits, flip, npsr, nsp, burst_len;
    int64_t  N;
    uint64_t seed;
    int32_t  maxv, minv;          // quantiser range
    uint32_t burst_thresh;        // P(burst cell) * 2^32
    uint32_t spike_thresh;        // P(spike spectrum) * 2^32
    int32_t  burst_q4, spike_q4, rfi_q4;
    int32_t  psr_amp_q4[HD_SYNTH_MAXPSR];
    int64_t  psr_period_fp[HD_SYNTH_MAXPSR];
    int64_t  psr_width_fp[HD_SYNTH_MAXPSR];
    int32_t  sp_amp_q4[HD_SYNTH_MAXPSR];
    int64_t  sp_t0_fp[HD_SYNTH_MAXPSR];
    int64_t  sp_width_fp[HD_SYNTH_MAXPSR];
    // per-channel arrays (ascending frequency), stored after the struct:
    //   int32 base_q4[nchan], int32 noise_mul[nchan], int32 rfi_flag[nchan],
    //   int64 psr_delay_fp[npsr][nchan], int64 sp_delay_fp[nsp][nchan]
};

HD_HD uint64_t hd_mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

HD_HD uint32_t hd_hash(uint64_t seed, uint64_t stream, uint64_t x)
{
    return (uint32_t)(hd_mix64(x * 0x9E3779B97F4A7C15ull + hd_mix64(seed ^ (stream << 56))) >> 32);
}

// Sum of four uniform bytes minus 510: mean 0, sigma ~147.8, range +-510.
HD_HD int32_t hd_gauss4(uint32_t h)
{
    return (int32_t)(h & 0xFF) + (int32_t)((h >> 8) & 0xFF) + (int32_t)((h >> 16) & 0xFF) +
           (int32_t)(h >> 24) - 510;
}

HD_HD int64_t hd_floordiv(int64_t a, int64_t b)   // b > 0
{
    int64_t q = a / b;
    return (q * b > a) ? q - 1 : q;
}

// Sample value (ascending channel c, spectrum t), already clamped to the quantiser range.
HD_HD int32_t hd_synth_sample(const hd_synth_tab* tb, const int32_t* base_q4,
                              const int32_t* noise_mul, const int32_t* rfi_flag,
                              const int64_t* psr_delay, const int64_t* sp_delay,
                              int64_t t, int32_t c)
{
    const uint64_t idx = (uint64_t)t * (uint64_t)tb->nchan + (uint64_t)c;
    int64_t v = base_q4[c] + (((int64_t)hd_gauss4(hd_hash(tb->seed, 1, idx)) * noise_mul[c]) >> 8);
    const int64_t tfp = t << 16;
    for (int p = 0; p < tb->npsr; p++) {
        const int64_t ph = tfp - psr_delay[(int64_t)p * tb->nchan + c];
        const int64_t r = ph - hd_floordiv(ph, tb->psr_period_fp[p]) * tb->psr_period_fp[p];
        if (r < tb->psr_width_fp[p]) v += tb->psr_amp_q4[p];
    }
    for (int p = 0; p < tb->nsp; p++) {
        const int64_t ph = tfp - sp_delay[(int64_t)p * tb->nchan + c] - tb->sp_t0_fp[p];
        if (ph >= 0 && ph < tb->sp_width_fp[p]) v += tb->sp_amp_q4[p];
    }
    if (rfi_flag[c])
        v += tb->rfi_q4 + (((int64_t)hd_gauss4(hd_hash(tb->seed, 2, idx)) * tb->rfi_q4) >> 9);
    if (tb->burst_len > 0 && hd_hash(tb->seed, 3, (uint64_t)(t / tb->burst_len) * tb->nchan + c) < tb->burst_thresh)
        v += tb->burst_q4;
    if (hd_hash(tb->seed, 4, (uint64_t)t) < tb->spike_thresh) v += tb->spike_q4;
    int64_t q = (v + 8) >> 4;   // nearest, ties up
    if (q > tb->maxv) q = tb->maxv;
    if (q < tb->minv) q = tb->minv;
    return (int32_t)q;
}

// Pointers to the per-channel arrays that follow the table.
HD_HD void hd_synth_arrays(const hd_synth_tab* tb, const int32_t** base_q4, const int32_t** noise_mul,
                           const int32_t** rfi_flag, const int64_t** psr_delay, const int64_t** sp_delay)
{
    const char* p = (const char*)tb + ((sizeof(hd_synth_tab) + 15) & ~(size_t)15);
    *base_q4 = (const int32_t*)p;
    *noise_mul = *base_q4 + tb->nchan;
    *rfi_flag = *noise_mul + tb->nchan;
    size_t off = (size_t)3 * tb->nchan * sizeof(int32_t);
    off = (off + 15) & ~(size_t)15;
    *psr_delay = (const int64_t*)(p + off);
    *sp_delay = *psr_delay + (size_t)tb->npsr * tb->nchan;
}

HD_HD size_t hd_synth_tab_bytes(int nchan, int npsr, int nsp)
{
    size_t head = (sizeof(hd_synth_tab) + 15) & ~(size_t)15;
    size_t a = ((size_t)3 * nchan * sizeof(int32_t) + 15) & ~(size_t)15;
    return head + a + (size_t)(npsr + nsp) * nchan * sizeof(int64_t);
}

// Write byte `b` of spectrum t's row (file layout: raw channel order, 4-bit high nibble
// first, 16-bit big-endian).
HD_HD uint8_t hd_synth_byte(const hd_synth_tab* tb, const int32_t* base_q4, const int32_t* noise_mul,
                            const int32_t* rfi_flag, const int64_t* psr_delay, const int64_t* sp_delay,
                            int64_t t, int32_t b)
{
    const int32_t nchan = tb->nchan;
    if (tb->nbits == 8) {
        const int32_t c = tb->flip ? nchan - 1 - b : b;
        return (uint8_t)hd_synth_sample(tb, base_q4, noise_mul, rfi_flag, psr_delay, sp_delay, t, c);
    } else if (tb->nbits == 4) {
        const int32_t rc0 = 2 * b, rc1 = 2 * b + 1;
        const int32_t c0 = tb->flip ? nchan - 1 - rc0 : rc0;
        const int32_t c1 = tb->flip ? nchan - 1 - rc1 : rc1;
        const int32_t v0 = hd_synth_sample(tb, base_q4, noise_mul, rfi_flag, psr_delay, sp_delay, t, c0);
        const int32_t v1 = hd_synth_sample(tb, base_q4, noise_mul, rfi_flag, psr_delay, sp_delay, t, c1);
        return (uint8_t)((v0 << 4) | (v1 & 15));
    } else {  // 16-bit, big-endian signed
        const int32_t rc = b >> 1;
        const int32_t c = tb->flip ? nchan - 1 - rc : rc;
        const uint16_t u = (uint16_t)(int16_t)hd_synth_sample(tb, base_q4, noise_mul, rfi_flag, psr_delay, sp_delay, t, c);
        return (b & 1) ? (uint8_t)(u & 0xFF) : (uint8_t)(u >> 8);
    }
}
