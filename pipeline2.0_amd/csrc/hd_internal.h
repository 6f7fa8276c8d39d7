// hd_internal.h — internal types shared by the C-ABI layer (hd_api.hip) and the
// kernel launchers (hd_kernels.hip).  Nothing here crosses the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hd_synth_core.h"

namespace hd {

// Raw-sample decode parameters for stage 1 (all device pointers).
struct RawDesc {
    const uint8_t* raw;       // [N][rowbytes], file layout
    int64_t N;
    int32_t rowbytes, nchan, nbits, flip, nibble_hi_first, be16;
    const float* scl;         // per raw channel or nullptr
    const float* offs;
    const float* wts;
    const uint8_t* mask;      // [numint][nchan] ascending channels or nullptr
    int32_t numint, ptsperint;
    const float* padvals;     // per ascending channel or nullptr
};

struct Stage1Args {
    RawDesc rd;
    const int32_t* idispdt;   // [nchan]
    int32_t nsub, cps, ds, ds_mode, sub_dtype, maxdelay;
    int64_t nds;              // output samples per subband
    int64_t out_stride;       // elements
    void* out;                // [nsub][out_stride]
    int32_t* maxabs;          // device int: max |subband value| (i16 path), atomicMax
};

struct Stage2Args {
    const void* sub;          // [nsub][sub_stride]
    int32_t sub_dtype, nsub, numdms, _pad;
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
};

hipError_t launch_stage1_direct(const Stage1Args& a, hipStream_t st);
hipError_t launch_stage2_direct(const Stage2Args& a, hipStream_t st);
hipError_t launch_stage2_lds(const Stage2Args& a, int q, hipStream_t st);
hipError_t launch_pad(float* out, int64_t out_stride, int numdms, int64_t nds, int64_t numout,
                      const double* partial, int ntiles, int pad_mode, hipStream_t st);
hipError_t launch_synth(uint8_t* raw, int64_t N, int32_t rowbytes, const hd_synth_tab* tab_dev,
                        hipStream_t st);

}  // namespace hd
