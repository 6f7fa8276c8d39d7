// Probe: are ds_read_b64 / ds_read_b128 at 2-, 4- and 8-byte (mis)aligned LDS addresses
// correct on gfx950 under the driver's SH_MEM_CONFIG, and what do they cost?
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_align_bench lds_align_bench.hip
// Output: per (width, byte shift): mismatches, ns per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int LDS_ELEMS = 16384;    // int16 elements (32 KiB)

// correctness: every lane reads width W at element index 4*lane + sh (+ a per-iteration offset)
template <int W>
__global__ __launch_bounds__(256) void k_check(int sh, int* bad)
{
    __shared__ __attribute__((aligned(16))) uint16_t s[LDS_ELEMS];
    for (int i = threadIdx.x; i < LDS_ELEMS; i += blockDim.x) s[i] = (uint16_t)(i * 7 + 3);
    __syncthreads();
    const int lane = threadIdx.x;
    int nb = 0;
    for (int it = 0; it < 8; it++) {
        const int e = (W / 2) * lane + sh + it * 37;
        const uint32_t addr = (uint32_t)(uintptr_t)(s) + 2u * (uint32_t)e;
        if constexpr (W == 8) {
            uint64_t v;
            asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
            for (int k = 0; k < 4; k++)
                if ((uint16_t)(v >> (16 * k)) != (uint16_t)((e + k) * 7 + 3)) nb++;
        } else {
            uint32_t v0, v1, v2, v3;
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            u4 v;
            asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
            v0 = v.x; v1 = v.y; v2 = v.z; v3 = v.w;
            const uint32_t w[4] = {v0, v1, v2, v3};
            for (int k = 0; k < 8; k++)
                if ((uint16_t)(w[k >> 1] >> (16 * (k & 1))) != (uint16_t)((e + k) * 7 + 3)) nb++;
        }
    }
    if (nb) atomicAdd(bad, nb);
}

// throughput: 16 independent reads per iteration, all at shift sh, per-iteration base moves
template <int W>
__global__ __launch_bounds__(256) void k_speed(int sh, int iters, uint32_t* out)
{
    __shared__ __attribute__((aligned(16))) uint16_t s[LDS_ELEMS];
    for (int i = threadIdx.x; i < LDS_ELEMS; i += blockDim.x) s[i] = (uint16_t)i;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t base = (uint32_t)(uintptr_t)(s) + 2u * (uint32_t)((W / 2) * lane + sh);
    uint32_t acc = 0;
    for (int it = 0; it < iters; it++) {
        const uint32_t a = base + (uint32_t)((it & 7) * 1024);
        if constexpr (W == 8) {
            uint64_t v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[k]) : "v"(a), "i"(k * 1024));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int k = 0; k < 8; k++) acc ^= (uint32_t)v[k] ^ (uint32_t)(v[k] >> 32);
        } else {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            u4 v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v[k]) : "v"(a), "i"(k * 1024));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int k = 0; k < 8; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// ds_read2_b32 of two consecutive dwords (8 bytes per lane, lanes 8 bytes apart) at element
// shift sh (even: 4-byte aligned, what the instruction needs)
__global__ __launch_bounds__(256) void k_check2(int sh, int* bad)
{
    __shared__ __attribute__((aligned(16))) uint16_t s[LDS_ELEMS];
    for (int i = threadIdx.x; i < LDS_ELEMS; i += blockDim.x) s[i] = (uint16_t)(i * 7 + 3);
    __syncthreads();
    const int lane = threadIdx.x;
    int nb = 0;
    for (int it = 0; it < 8; it++) {
        const int e = 4 * lane + sh + it * 38;
        const uint32_t addr = (uint32_t)(uintptr_t)(s) + 2u * (uint32_t)e;
        uint64_t v;
        asm volatile("ds_read2_b32 %0, %1 offset0:0 offset1:1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
        for (int k = 0; k < 4; k++)
            if ((uint16_t)(v >> (16 * k)) != (uint16_t)((e + k) * 7 + 3)) nb++;
    }
    if (nb) atomicAdd(bad, nb);
}

__global__ __launch_bounds__(256) void k_speed2(int sh, int iters, uint32_t* out)
{
    __shared__ __attribute__((aligned(16))) uint16_t s[LDS_ELEMS];
    for (int i = threadIdx.x; i < LDS_ELEMS; i += blockDim.x) s[i] = (uint16_t)i;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t base = (uint32_t)(uintptr_t)(s) + 2u * (uint32_t)(4 * lane + sh);
    uint32_t acc = 0;
    for (int it = 0; it < iters; it++) {
        const uint32_t a = base + (uint32_t)((it & 7) * 1024);
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++)
            asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3" : "=v"(v[k]) : "v"(a), "i"(k * 32), "i"(k * 32 + 1));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 8; k++) acc ^= (uint32_t)v[k] ^ (uint32_t)(v[k] >> 32);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

static int run2(int* dbad, uint32_t* dout, int nblk)
{
    for (int sh = 0; sh < 4; sh += 2) {
        CK(hipMemset(dbad, 0, 4));
        hipLaunchKernelGGL(k_check2, dim3(1), dim3(64), 0, 0, sh, dbad);
        CK(hipDeviceSynchronize());
        int bad = 0;
        CK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
        const int iters = 4096;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        hipLaunchKernelGGL(k_speed2, dim3(nblk), dim3(256), 0, 0, sh, iters, dout);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_speed2, dim3(nblk), dim3(256), 0, 0, sh, iters, dout);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double winst_per_cu = (double)nblk / 256.0 * 4.0 * iters * 8.0;
        const double bytes = (double)nblk * 256 * iters * 8 * 8;
        printf("ds_read2_b32 (8 B/lane) shift %d B: mismatches %d, %.3f ms, %.2f ns per wave-instr per CU, %.1f TB/s LDS\n",
               2 * sh, bad, ms, ms * 1e6 / winst_per_cu, bytes / (ms * 1e-3) / 1e12);
    }
    return 0;
}

template <int W>
static int run(int* dbad, uint32_t* dout, int nblk)
{
    for (int sh = 0; sh < (W == 8 ? 4 : 8); sh++) {
        CK(hipMemset(dbad, 0, 4));
        hipLaunchKernelGGL(k_check<W>, dim3(1), dim3(64), 0, 0, sh, dbad);
        CK(hipDeviceSynchronize());
        int bad = 0;
        CK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
        const int iters = 4096;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        hipLaunchKernelGGL(k_speed<W>, dim3(nblk), dim3(256), 0, 0, sh, iters, dout);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_speed<W>, dim3(nblk), dim3(256), 0, 0, sh, iters, dout);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        // wave-instructions per CU: (nblk/256 CUs) * 4 waves * iters * 8
        const double winst_per_cu = (double)nblk / 256.0 * 4.0 * iters * 8.0;
        const double bytes = (double)nblk * 256 * iters * 8 * W;
        printf("ds_read_b%d shift %d B: mismatches %d, %.3f ms, %.2f ns per wave-instr per CU, %.1f TB/s LDS\n",
               W * 8, 2 * sh, bad, ms, ms * 1e6 / winst_per_cu, bytes / (ms * 1e-3) / 1e12);
    }
    return 0;
}

int main()
{
    int* dbad;
    uint32_t* dout;
    const int nblk = 256 * 8;
    CK(hipMalloc(&dbad, 4));
    CK(hipMalloc(&dout, (size_t)nblk * 256 * 4));
    if (run<8>(dbad, dout, nblk)) return 1;
    if (run<16>(dbad, dout, nblk)) return 1;
    if (run2(dbad, dout, nblk)) return 1;
    return 0;
}
