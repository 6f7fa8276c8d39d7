// hd_io.hip — the .dat output path (host code): device series -> pinned staging buffers on
// a copy stream -> a pool of writer threads -> files.
//
// The reference leaves every pass's 76 (or 64) DM series as `<base>_DM<dm>.dat` in its
// /dev/shm tempdir (PALFA2_presto_search.py:463-464, 514-520), where the per-DM tools read
// them (:532-606).  hd_write_series queues one plan's series: chunks of up to kChunk bytes
// are copied device->host into pinned buffers on the context's copy stream (ordered after
// the plan's last stage-2 launch by an event, so the next pass's kernels keep running on
// the compute stream), and writer threads pwrite() each chunk once its copy event has
// completed, then recycle the buffer.  A file is closed by whichever thread writes its last
// chunk.  hd_wait_writes drains everything and reports the first I/O error.
#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hd_io.h"

namespace hd {

namespace {
constexpr size_t kChunk = (size_t)16 << 20;    // bytes per staging buffer (one 2^22-sample series)
constexpr int kBuffers = 16;
constexpr int kThreads = 8;

struct File {
    int fd;
    std::atomic<int> left;                       // chunks not yet written
    std::string path;
};

struct Task {
    int buf;
    File* file;
    off_t off;
    size_t bytes;
};
}  // namespace

struct Writer {
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<void*> bufs;
    std::vector<hipEvent_t> evs;
    std::deque<int> free_bufs;
    std::deque<Task> queue;
    std::mutex mu;
    std::condition_variable cv_task, cv_free, cv_idle;
    int inflight = 0;                            // tasks queued or being written
    bool stop = false;
    std::string err;
    std::vector<std::thread> threads;
    std::atomic<int64_t> bytes{0};
    std::atomic<int64_t> write_ns{0};

    void run()
    {
        (void)hipSetDevice(device);
        for (;;) {
            Task t;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_task.wait(lk, [&] { return stop || !queue.empty(); });
                if (queue.empty()) return;
                t = queue.front();
                queue.pop_front();
            }
            const auto t0 = std::chrono::steady_clock::now();
            std::string e;
            if (hipEventSynchronize(evs[t.buf]) != hipSuccess) e = "device-to-host copy failed";
            const char* p = (const char*)bufs[t.buf];
            size_t n = t.bytes;
            off_t off = t.off;
            while (e.empty() && n) {
                const ssize_t w = pwrite(t.file->fd, p, n, off);
                if (w <= 0) {
                    e = "write to " + t.file->path + " failed";
                    break;
                }
                p += w;
                n -= (size_t)w;
                off += w;
            }
            if (t.file->left.fetch_sub(1) == 1) {
                if (close(t.file->fd) && e.empty()) e = "close of " + t.file->path + " failed";
                delete t.file;
            }
            bytes += (int64_t)t.bytes;
            write_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
            std::lock_guard<std::mutex> lk(mu);
            if (!e.empty() && err.empty()) err = e;
            free_bufs.push_back(t.buf);
            cv_free.notify_one();
            if (--inflight == 0) cv_idle.notify_all();
        }
    }
};

hipError_t writer_open(Writer** out, int device)
{
    *out = nullptr;
    Writer* w = new Writer();
    w->device = device;
    hipError_t e = hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking);
    for (int i = 0; i < kBuffers && e == hipSuccess; i++) {
        void* b = nullptr;
        hipEvent_t ev = nullptr;
        e = hipHostMalloc(&b, kChunk, hipHostMallocDefault);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (b) w->bufs.push_back(b);
        if (ev) w->evs.push_back(ev);
        w->free_bufs.push_back(i);
    }
    if (e != hipSuccess) {
        writer_close(w);
        return e;
    }
    for (int i = 0; i < kThreads; i++) w->threads.emplace_back([w] { w->run(); });
    *out = w;
    return hipSuccess;
}

hipStream_t writer_stream(Writer* w) { return w->stream; }

void writer_close(Writer* w)
{
    if (!w) return;
    {
        std::lock_guard<std::mutex> lk(w->mu);
        w->stop = true;
    }
    w->cv_task.notify_all();
    for (auto& t : w->threads) t.join();
    for (void* b : w->bufs) (void)hipHostFree(b);
    for (hipEvent_t ev : w->evs) (void)hipEventDestroy(ev);
    if (w->stream) (void)hipStreamDestroy(w->stream);
    delete w;
}

// After a device fault: stop the threads (queued chunks are dropped; a thread inside a
// hipEventSynchronize gets the fault's error back) and free the host side only.
void writer_abandon(Writer* w)
{
    if (!w) return;
    {
        std::lock_guard<std::mutex> lk(w->mu);
        w->stop = true;
        for (const Task& t : w->queue)
            if (t.file->left.fetch_sub(1) == 1) {
                close(t.file->fd);
                delete t.file;
            }
        w->queue.clear();
    }
    w->cv_task.notify_all();
    for (auto& t : w->threads) t.join();
    delete w;
}

int writer_series(Writer* w, hipEvent_t after, const float* d_out, int64_t out_stride, int numdms, int64_t numout,
                  const char* const* paths, std::string& err)
{
    if (hipStreamWaitEvent(w->stream, after, 0) != hipSuccess) {
        err = "hipStreamWaitEvent failed";
        return -3;
    }
    const size_t total = sizeof(float) * (size_t)numout;
    const int nchunk = total ? (int)((total + kChunk - 1) / kChunk) : 0;
    for (int d = 0; d < numdms; d++) {
        const int fd = open(paths[d], O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd < 0) {
            err = std::string("cannot create ") + paths[d];
            return -6;
        }
        if (nchunk == 0) {
            close(fd);
            continue;
        }
        File* f = new File{fd, {nchunk}, paths[d]};
        for (int k = 0; k < nchunk; k++) {
            const size_t off = (size_t)k * kChunk, n = std::min(kChunk, total - off);
            int b;
            {
                std::unique_lock<std::mutex> lk(w->mu);
                w->cv_free.wait(lk, [&] { return !w->free_bufs.empty(); });
                b = w->free_bufs.front();
                w->free_bufs.pop_front();
            }
            const char* src = (const char*)(d_out + (size_t)d * out_stride) + off;
            hipError_t e = hipMemcpyAsync(w->bufs[b], src, n, hipMemcpyDeviceToHost, w->stream);
            if (e == hipSuccess) e = hipEventRecord(w->evs[b], w->stream);
            std::lock_guard<std::mutex> lk(w->mu);
            if (e != hipSuccess) {
                // chunks of this file already queued still write (and close it when last)
                w->free_bufs.push_back(b);
                if (f->left.fetch_sub(nchunk - k) == nchunk - k) {
                    close(fd);
                    delete f;
                }
                err = std::string("device-to-host copy failed: ") + hipGetErrorString(e);
                return -3;
            }
            w->queue.push_back(Task{b, f, (off_t)off, n});
            w->inflight++;
            w->cv_task.notify_one();
        }
    }
    return 0;
}

int writer_wait(Writer* w, std::string& err, double* write_seconds, int64_t* bytes)
{
    std::unique_lock<std::mutex> lk(w->mu);
    w->cv_idle.wait(lk, [&] { return w->inflight == 0; });
    if (write_seconds) *write_seconds = (double)w->write_ns.load() * 1e-9;
    if (bytes) *bytes = w->bytes.load();
    if (!w->err.empty()) {
        err = w->err;
        w->err.clear();
        return -6;
    }
    return 0;
}

}  // namespace hd
