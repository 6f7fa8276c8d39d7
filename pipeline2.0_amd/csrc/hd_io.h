// hd_io.h — the asynchronous .dat writer (hd_io.hip) used by hd_write_series.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace hd {

struct Writer;
hipError_t writer_open(Writer** out, int device);
void writer_close(Writer* w);
void writer_abandon(Writer* w);   // device faulted: threads stopped, host memory only
hipStream_t writer_stream(Writer* w);
// Queue numdms series [numdms][out_stride] (numout samples each) to paths[d], after `after`.
int writer_series(Writer* w, hipEvent_t after, const float* d_out, int64_t out_stride, int numdms, int64_t numout,
                  const char* const* paths, std::string& err);
// Wait for every queued chunk; first I/O error (if any) in err; cumulative writer-thread
// seconds and bytes since the writer was opened.
int writer_wait(Writer* w, std::string& err, double* write_seconds, int64_t* bytes);

}  // namespace hd
