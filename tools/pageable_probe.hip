// pageable_probe.hip — host<->HBM copies from PAGEABLE memory, the case the
// single-object C-ABI calls (chip_encode / chip_decode / chip_scrub) see when
// the Rust crate hands them a &[u8]: the runtime's own pageable path on the
// same buffer every time vs a new buffer every time, against a pipelined copy
// through a small pinned staging ring (CPU memcpy of piece j+1 overlapping the
// DMA of piece j).  Calibration tool (not product code).
//   pageable_probe [MiB=34] [buffers=16] [piece_MiB=4]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <sys/mman.h>

#include <thread>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const size_t n = (argc > 1 ? atoll(argv[1]) : 34) << 20;
    const int nb = argc > 2 ? atoi(argv[2]) : 16;
    const size_t piece = (argc > 3 ? atoll(argv[3]) : 4) << 20;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    void *dev;
    CK(hipMalloc(&dev, n));
    std::vector<uint8_t *> bufs(nb);
    for (auto &b : bufs) {
        b = static_cast<uint8_t *>(malloc(n));
        memset(b, 1, n);
    }
    const int R = 4;  // staging ring
    uint8_t *stage;
    CK(hipHostMalloc(reinterpret_cast<void **>(&stage), R * piece, hipHostMallocDefault));
    std::vector<hipEvent_t> ev(R);
    for (size_t i = 0; i < ev.size(); ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));

    auto h2d_runtime = [&](uint8_t *src) {
        CK(hipMemcpyAsync(dev, src, n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    };
    auto d2h_runtime = [&](uint8_t *dst) {
        CK(hipMemcpyAsync(dst, dev, n, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    };
    auto h2d_staged = [&](uint8_t *src) {
        size_t j = 0;
        for (size_t off = 0; off < n; off += piece, ++j) {
            const size_t len = std::min(piece, n - off);
            uint8_t *st = stage + (j % R) * piece;
            if (j >= R) CK(hipEventSynchronize(ev[j % R]));  // ring slot free again
            memcpy(st, src + off, len);
            CK(hipMemcpyAsync(static_cast<uint8_t *>(dev) + off, st, len, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(ev[j % R], s));
        }
        CK(hipStreamSynchronize(s));
    };
    auto d2h_staged = [&](uint8_t *dst) {
        const size_t np = (n + piece - 1) / piece;
        auto issue = [&](size_t j) {
            const size_t off = j * piece, len = std::min(piece, n - off);
            CK(hipMemcpyAsync(stage + (j % R) * piece, static_cast<uint8_t *>(dev) + off, len,
                              hipMemcpyDeviceToHost, s));
            CK(hipEventRecord(ev[j % R], s));
        };
        for (size_t j = 0; j < std::min<size_t>(R, np); ++j) issue(j);
        for (size_t j = 0; j < np; ++j) {
            CK(hipEventSynchronize(ev[j % R]));
            const size_t off = j * piece, len = std::min(piece, n - off);
            memcpy(dst + off, stage + (j % R) * piece, len);
            if (j + R < np) issue(j + R);
        }
    };
    auto populate = [&](uint8_t *p, size_t len) {  // MADV_POPULATE_WRITE (Linux 5.14) on whole pages
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        const uintptr_t lo = a & ~uintptr_t(4095), hi = (a + len + 4095) & ~uintptr_t(4095);
        return madvise(reinterpret_cast<void *>(lo), hi - lo, 23);
    };
    auto d2h_staged_mt = [&](uint8_t *dst, int th) {  // staged, each piece's memcpy split over th threads
        const size_t np = (n + piece - 1) / piece;
        auto issue = [&](size_t j) {
            const size_t off = j * piece, len = std::min(piece, n - off);
            CK(hipMemcpyAsync(stage + (j % R) * piece, static_cast<uint8_t *>(dev) + off, len,
                              hipMemcpyDeviceToHost, s));
            CK(hipEventRecord(ev[j % R], s));
        };
        for (size_t j = 0; j < std::min<size_t>(R, np); ++j) issue(j);
        for (size_t j = 0; j < np; ++j) {
            CK(hipEventSynchronize(ev[j % R]));
            const size_t off = j * piece, len = std::min(piece, n - off);
            std::vector<std::thread> ws;
            const size_t part = (len / th + 4095) & ~size_t(4095);
            for (int t = 0; t < th; ++t) {
                const size_t o = t * part;
                if (o >= len) break;
                ws.emplace_back([&, o] { memcpy(dst + off + o, stage + (j % R) * piece + o, std::min(part, len - o)); });
            }
            for (auto &w : ws) w.join();
            if (j + R < np) issue(j + R);
        }
    };
    struct T {
        const char *name;
        std::function<void(int)> fn;
    };
    std::vector<uint8_t *> fresh(nb, nullptr);
    std::vector<T> ts = {
        {"H2D runtime, same buffer", [&](int) { h2d_runtime(bufs[0]); }},
        {"H2D runtime, buffer i", [&](int i) { h2d_runtime(bufs[i]); }},
        {"H2D staged, buffer i", [&](int i) { h2d_staged(bufs[i]); }},
        {"D2H runtime, same buffer", [&](int) { d2h_runtime(bufs[0]); }},
        {"D2H runtime, buffer i", [&](int i) { d2h_runtime(bufs[i]); }},
        {"D2H staged, buffer i", [&](int i) { d2h_staged(bufs[i]); }},
        {"D2H runtime, fresh malloc", [&](int i) {
             free(fresh[i]);
             fresh[i] = static_cast<uint8_t *>(malloc(n));
             d2h_runtime(fresh[i]);
         }},
        {"D2H populate+runtime, fresh", [&](int i) {
             free(fresh[i]);
             fresh[i] = static_cast<uint8_t *>(malloc(n));
             if (populate(fresh[i], n)) perror("madvise");
             d2h_runtime(fresh[i]);
         }},
        {"populate only, fresh", [&](int i) {
             free(fresh[i]);
             fresh[i] = static_cast<uint8_t *>(malloc(n));
             if (populate(fresh[i], n)) perror("madvise");
         }},
        {"D2H memset+runtime, fresh", [&](int i) {
             free(fresh[i]);
             fresh[i] = static_cast<uint8_t *>(malloc(n));
             memset(fresh[i], 0, n);
             d2h_runtime(fresh[i]);
         }},
        {"D2H staged x4 thr, fresh", [&](int i) {
             free(fresh[i]);
             fresh[i] = static_cast<uint8_t *>(malloc(n));
             d2h_staged_mt(fresh[i], 4);
         }},
        {"D2H staged x8 thr, fresh", [&](int i) {
             free(fresh[i]);
             fresh[i] = static_cast<uint8_t *>(malloc(n));
             d2h_staged_mt(fresh[i], 8);
         }},
        {"D2H staged x4 thr, buffer i", [&](int i) { d2h_staged_mt(bufs[i], 4); }},
        {"D2H staged, fresh malloc", [&](int i) {
             free(fresh[i]);
             fresh[i] = static_cast<uint8_t *>(malloc(n));
             d2h_staged(fresh[i]);
         }},
    };
    {  // where the fresh-buffer time goes: the free() of a buffer the runtime pinned, or the copy
        std::vector<double> tf, tc;
        for (int rep = 0; rep < 3; ++rep)
            for (int i = 0; i < nb; ++i) {
                double t0 = now();
                free(fresh[i]);
                fresh[i] = static_cast<uint8_t *>(malloc(n));
                tf.push_back(now() - t0);
                t0 = now();
                d2h_runtime(fresh[i]);
                tc.push_back(now() - t0);
            }
        std::sort(tf.begin(), tf.end());
        std::sort(tc.begin(), tc.end());
        printf("runtime D2H fresh: free+malloc median %7.3f ms, copy median %7.3f ms\n", tf[tf.size() / 2] * 1e3,
               tc[tc.size() / 2] * 1e3);
        tf.clear();
        tc.clear();
        for (int rep = 0; rep < 3; ++rep)
            for (int i = 0; i < nb; ++i) {
                double t0 = now();
                free(fresh[i]);
                fresh[i] = static_cast<uint8_t *>(malloc(n));
                tf.push_back(now() - t0);
                t0 = now();
                d2h_staged(fresh[i]);
                tc.push_back(now() - t0);
            }
        std::sort(tf.begin(), tf.end());
        std::sort(tc.begin(), tc.end());
        printf("staged D2H fresh:  free+malloc median %7.3f ms, copy median %7.3f ms\n", tf[tf.size() / 2] * 1e3,
               tc[tc.size() / 2] * 1e3);
    }
    for (auto &t : ts) {
        std::vector<double> d;
        for (int rep = 0; rep < 3; ++rep)
            for (int i = 0; i < nb; ++i) {
                const double t0 = now();
                t.fn(i);
                d.push_back(now() - t0);
            }
        std::sort(d.begin(), d.end());
        const double med = d[d.size() / 2];
        printf("%-28s median %7.3f ms (%6.1f GB/s)  max %7.3f ms\n", t.name, med * 1e3, n / med / 1e9,
               d.back() * 1e3);
    }
    return 0;
}
