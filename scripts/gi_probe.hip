// Probe (GPU box, profiling aid): GPR-indexed register windows on gfx950.  A wave loads a
// 24-element int16 window per lane (lane l at element 8l) into v[100:111], forms the
// one-element-shifted dwords v[112:121] (v_alignbit), and adds, per DM, the 8 elements at a
// wave-uniform shift k (0..13) into 4 packed accumulators with s_set_gpr_idx_on + v_add_u32
// (VOP2, SRC0 indexed by M0: index (k & 1) * 12 + (k >> 1)).  Checks every lane against the
// host and times a loop of it.   hipcc --offload-arch=gfx950 -O3 -o gi_probe gi_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

template <int Q>
__global__ __launch_bounds__(512, 4) void k_gi(const uint16_t* __restrict__ src, const uint32_t* __restrict__ ks,
                                               uint32_t* __restrict__ out, int iters)
{
    __shared__ __attribute__((aligned(16))) uint16_t lds[64 * 8 + 64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 64 * 8 + 64; i += blockDim.x) lds[i] = src[i];
    __syncthreads();
    uint32_t acc[Q][4];
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[q][j] = 0;
    uint32_t idx[Q];
#pragma unroll
    for (int q = 0; q < Q; q++) {
        const uint32_t k = ks[(wave * Q + q) % 14];
        idx[q] = __builtin_amdgcn_readfirstlane((k & 1) * 12 + (k >> 1));
    }
    const uint32_t addr = 16u * (uint32_t)lane;      // lds is the kernel's only LDS allocation: offset 0
    for (int it = 0; it < iters; it++) {
        asm volatile(
            "ds_read_b64 v[100:101], %20 offset:0\n\t"
            "ds_read_b64 v[102:103], %20 offset:8\n\t"
            "ds_read_b64 v[104:105], %20 offset:16\n\t"
            "ds_read_b64 v[106:107], %20 offset:24\n\t"
            "ds_read_b64 v[108:109], %20 offset:32\n\t"
            "ds_read_b64 v[110:111], %20 offset:40\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"
            "v_alignbit_b32 v112, v101, v100, 16\n\t"
            "v_alignbit_b32 v113, v102, v101, 16\n\t"
            "v_alignbit_b32 v114, v103, v102, 16\n\t"
            "v_alignbit_b32 v115, v104, v103, 16\n\t"
            "v_alignbit_b32 v116, v105, v104, 16\n\t"
            "v_alignbit_b32 v117, v106, v105, 16\n\t"
            "v_alignbit_b32 v118, v107, v106, 16\n\t"
            "v_alignbit_b32 v119, v108, v107, 16\n\t"
            "v_alignbit_b32 v120, v109, v108, 16\n\t"
            "v_alignbit_b32 v121, v110, v109, 16\n\t"
            "s_set_gpr_idx_on %21, gpr_idx(SRC0)\n\t"
            "v_add_u32_e32 %0, v100, %0\n\t"
            "v_add_u32_e32 %1, v101, %1\n\t"
            "v_add_u32_e32 %2, v102, %2\n\t"
            "v_add_u32_e32 %3, v103, %3\n\t"
            "s_set_gpr_idx_idx %22\n\t"
            "v_add_u32_e32 %4, v100, %4\n\t"
            "v_add_u32_e32 %5, v101, %5\n\t"
            "v_add_u32_e32 %6, v102, %6\n\t"
            "v_add_u32_e32 %7, v103, %7\n\t"
            "s_set_gpr_idx_idx %23\n\t"
            "v_add_u32_e32 %8, v100, %8\n\t"
            "v_add_u32_e32 %9, v101, %9\n\t"
            "v_add_u32_e32 %10, v102, %10\n\t"
            "v_add_u32_e32 %11, v103, %11\n\t"
            "s_set_gpr_idx_idx %24\n\t"
            "v_add_u32_e32 %12, v100, %12\n\t"
            "v_add_u32_e32 %13, v101, %13\n\t"
            "v_add_u32_e32 %14, v102, %14\n\t"
            "v_add_u32_e32 %15, v103, %15\n\t"
            "s_set_gpr_idx_idx %25\n\t"
            "v_add_u32_e32 %16, v100, %16\n\t"
            "v_add_u32_e32 %17, v101, %17\n\t"
            "v_add_u32_e32 %18, v102, %18\n\t"
            "v_add_u32_e32 %19, v103, %19\n\t"
            "s_set_gpr_idx_off"
            : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[0][2]), "+v"(acc[0][3]), "+v"(acc[1][0]), "+v"(acc[1][1]),
              "+v"(acc[1][2]), "+v"(acc[1][3]), "+v"(acc[2][0]), "+v"(acc[2][1]), "+v"(acc[2][2]), "+v"(acc[2][3]),
              "+v"(acc[3][0]), "+v"(acc[3][1]), "+v"(acc[3][2]), "+v"(acc[3][3]), "+v"(acc[4][0]), "+v"(acc[4][1]),
              "+v"(acc[4][2]), "+v"(acc[4][3])
            : "v"(addr), "s"(idx[0]), "s"(idx[1]), "s"(idx[2]), "s"(idx[3]), "s"(idx[4])
            : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112",
              "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121");
    }
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int j = 0; j < 4; j++) out[((size_t)blockIdx.x * 512 + threadIdx.x) * (Q * 4) + q * 4 + j] = acc[q][j];
}

int main()
{
    const int n = 64 * 8 + 64;
    std::vector<uint16_t> h(n);
    for (int i = 0; i < n; i++) h[i] = (uint16_t)((i * 37 + 11) % 200);
    std::vector<uint32_t> ks(14);
    for (int i = 0; i < 14; i++) ks[i] = (uint32_t)((i * 5) % 14);
    uint16_t* d;
    uint32_t *dk, *dout;
    const int nblk = 512, Q = 5;
    hipMalloc(&d, n * 2);
    hipMalloc(&dk, 14 * 4);
    hipMalloc(&dout, (size_t)nblk * 512 * Q * 4 * 4);
    hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice);
    hipMemcpy(dk, ks.data(), 14 * 4, hipMemcpyHostToDevice);
    int bad = 0;
    for (int iters : {1, 3}) {
        hipLaunchKernelGGL(k_gi<5>, dim3(nblk), dim3(512), 0, 0, d, dk, dout, iters);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
        std::vector<uint32_t> o((size_t)nblk * 512 * Q * 4);
        hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
        for (int b = 0; b < nblk && bad < 10; b++)
            for (int t = 0; t < 512; t++) {
                const int lane = t & 63, wave = t >> 6;
                for (int q = 0; q < Q; q++) {
                    const uint32_t k = ks[(wave * Q + q) % 14];
                    for (int j = 0; j < 4; j++) {
                        const int e = 8 * lane + k + 2 * j;
                        const uint32_t want = (uint32_t)iters * ((uint32_t)h[e] | ((uint32_t)h[e + 1] << 16));
                        const uint32_t got = o[((size_t)b * 512 + t) * (Q * 4) + q * 4 + j];
                        if (got != want && bad++ < 10)
                            printf("mismatch blk %d t %d q %d j %d k %u: got %08x want %08x\n", b, t, q, j, k, got, want);
                    }
                }
            }
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 2000;
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_gi<5>, dim3(nblk), dim3(512), 0, 0, d, dk, dout, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double dmsub = (double)nblk * 8 * Q * iters;      // (DM, window) items
    printf("%s: %d mismatches; %.3f ms for %.3g DM-subband items of 8 samples: %.3f ns per item per CU-equivalent\n",
           bad ? "FAIL" : "OK", bad, ms, dmsub, ms * 1e6 / dmsub * 256);
    return bad ? 1 : 0;
}
