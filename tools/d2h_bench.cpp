// d2h_bench.cpp -- device-to-host copy of an NW table (the drop-in nw_fill's
// last step, driver.cpp:22-30 times it) by strategy, on the GPU box:
//   pageable2d  hipMemcpy2D into the caller's pageable buffer (the r02 path)
//   pinned2d    the same into hipHostMalloc memory (the bare pinned D2H time)
//   register    hipHostRegister(caller buffer) + hipMemcpy2D + unregister
//   staged      pinned staging chunks (DMA) + threaded memcpy into the caller buffer
// Usage: d2h_bench <n> [threads] [chunk MB]
//   hipcc -O2 -std=c++17 tools/d2h_bench.cpp -o tools/d2h_bench -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));     \
            std::exit(1);                                                  \
        }                                                                  \
    } while (0)

static void par_copy(char *dst, const char *src, size_t bytes, int threads) {
    std::vector<std::thread> ts;
    const size_t per = (bytes / threads + 4095) & ~(size_t)4095;
    for (int t = 0; t < threads; ++t) {
        const size_t o = (size_t)t * per;
        if (o >= bytes) break;
        const size_t n = std::min(per, bytes - o);
        ts.emplace_back([=] { std::memcpy(dst + o, src + o, n); });
    }
    for (auto &t : ts) t.join();
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 45000;
    const int threads = argc > 2 ? atoi(argv[2]) : 8;
    const size_t chunk = (size_t)(argc > 3 ? atol(argv[3]) : 64) << 20;
    const long cols = n + 1, rows = n + 1, pitch = (cols + 3 + 63) / 64 * 64;
    const size_t w = (size_t)cols * 4, bytes = w * rows;
    std::printf("n=%ld table %.2f GB, pitch %ld, threads %d, chunk %zu MB\n", n, bytes / 1e9, pitch, threads,
                chunk >> 20);
    int32_t *d = nullptr;
    CK(hipMalloc(&d, (size_t)pitch * 4 * rows));
    CK(hipMemset(d, 1, (size_t)pitch * 4 * rows));
    CK(hipDeviceSynchronize());
    // caller buffer as driver.cpp makes it: new int[], touched every 1024 ints
    int32_t *host = new int32_t[(size_t)cols * rows];
    for (size_t i = 0; i < (size_t)cols * rows; i += 1024) host[i] = 0;

    double t0, t1;
    if (argc > 4 && atoi(argv[4]) == 1) {
        // the drop-in's configuration on a caller buffer fresh from the touch loop,
        // twice: cold pages first, then the same buffer again; then a memcpy-only pass
        char *st[3];
        hipEvent_t ev[3];
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        for (int k = 0; k < 3; ++k) {
            CK(hipHostMalloc((void **)&st[k], chunk, hipHostMallocCoherent));
            CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
        }
        const long rpc = std::max<long>(1, (long)(chunk / w));
        const long nch = (rows + rpc - 1) / rpc;
        for (int pass = 0; pass < 2; ++pass) {
            double tdma = 0, tcpy = 0;
            t0 = now();
            auto issue = [&](long c) {
                const long r0 = c * rpc, nr = std::min(rpc, rows - r0);
                CK(hipMemcpy2DAsync(st[c % 3], w, d + r0 * pitch, pitch * 4, w, nr, hipMemcpyDeviceToHost, s));
                CK(hipEventRecord(ev[c % 3], s));
            };
            for (long c = 0; c < std::min<long>(3, nch); ++c) issue(c);
            for (long c = 0; c < nch; ++c) {
                double a0 = now();
                CK(hipEventSynchronize(ev[c % 3]));
                double a1 = now();
                const long r0 = c * rpc, nr = std::min(rpc, rows - r0);
                par_copy((char *)host + (size_t)r0 * w, st[c % 3], (size_t)nr * w, threads);
                double a2 = now();
                tdma += a1 - a0;
                tcpy += a2 - a1;
                if (c + 3 < nch) issue(c + 3);
            }
            t1 = now();
            std::printf("fresh-first pass %d: %.3f s %.1f GB/s (waiting on DMA %.3f s, copying %.3f s)\n", pass,
                        t1 - t0, bytes / (t1 - t0) / 1e9, tdma, tcpy);
        }
        return 0;
    }
    t0 = now();
    CK(hipMemcpy2D(host, w, d, pitch * 4, w, rows, hipMemcpyDeviceToHost));
    t1 = now();
    std::printf("pageable2d  %.3f s  %.1f GB/s\n", t1 - t0, bytes / (t1 - t0) / 1e9);

    {
        int32_t *pin = nullptr;
        t0 = now();
        CK(hipHostMalloc((void **)&pin, bytes, 0));
        t1 = now();
        std::printf("  hipHostMalloc %.3f s\n", t1 - t0);
        for (int it = 0; it < 2; ++it) {
            t0 = now();
            CK(hipMemcpy2D(pin, w, d, pitch * 4, w, rows, hipMemcpyDeviceToHost));
            t1 = now();
            std::printf("pinned2d    %.3f s  %.1f GB/s\n", t1 - t0, bytes / (t1 - t0) / 1e9);
        }
        CK(hipHostFree(pin));
    }
    {
        t0 = now();
        hipError_t e = hipHostRegister(host, bytes, hipHostRegisterDefault);
        t1 = now();
        if (e != hipSuccess) {
            std::printf("register    failed: %s\n", hipGetErrorString(e));
        } else {
            CK(hipMemcpy2D(host, w, d, pitch * 4, w, rows, hipMemcpyDeviceToHost));
            double t2 = now();
            CK(hipHostUnregister(host));
            double t3 = now();
            std::printf("register    %.3f s (register %.3f, copy %.3f = %.1f GB/s, unregister %.3f)\n", t3 - t0,
                        t1 - t0, t2 - t1, bytes / (t2 - t1) / 1e9, t3 - t2);
        }
    }
    struct Flag {
        const char *name;
        unsigned f;
    } flags[] = {{"default", hipHostMallocDefault}, {"noncoherent", hipHostMallocNonCoherent},
                 {"coherent", hipHostMallocCoherent}};
    for (const Flag &fl : flags) {
        // CPU side alone: memcpy out of one pinned chunk into the caller's buffer
        {
            char *pin = nullptr;
            CK(hipHostMalloc((void **)&pin, chunk, fl.f));
            std::memset(pin, 1, chunk);
            for (int th : {8, 16}) {
                const long reps = (long)(bytes / chunk);
                t0 = now();
                for (long r = 0; r < reps; ++r) par_copy((char *)host + (size_t)r * chunk, pin, chunk, th);
                t1 = now();
                std::printf("  %-11s memcpy only, %2d threads: %.1f GB/s\n", fl.name, th,
                            reps * (double)chunk / (t1 - t0) / 1e9);
            }
            CK(hipHostFree(pin));
        }
        for (int th : {8, 16}) {
            for (size_t ck : {chunk / 2, chunk, chunk * 2}) {
                for (int nb : {3, 4}) {
                    std::vector<char *> st(nb);
                    std::vector<hipEvent_t> ev(nb);
                    hipStream_t s;
                    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                    for (int k = 0; k < nb; ++k) {
                        CK(hipHostMalloc((void **)&st[k], ck, fl.f));
                        CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
                    }
                    const long rpc = std::max<long>(1, (long)(ck / w));
                    const long nch = (rows + rpc - 1) / rpc;
                    t0 = now();
                    auto issue = [&](long c) {
                        const long r0 = c * rpc, nr = std::min(rpc, rows - r0);
                        CK(hipMemcpy2DAsync(st[c % nb], w, d + r0 * pitch, pitch * 4, w, nr, hipMemcpyDeviceToHost,
                                            s));
                        CK(hipEventRecord(ev[c % nb], s));
                    };
                    for (long c = 0; c < std::min<long>(nb, nch); ++c) issue(c);
                    for (long c = 0; c < nch; ++c) {
                        CK(hipEventSynchronize(ev[c % nb]));
                        const long r0 = c * rpc, nr = std::min(rpc, rows - r0);
                        par_copy((char *)host + (size_t)r0 * w, st[c % nb], (size_t)nr * w, th);
                        if (c + nb < nch) issue(c + nb);
                    }
                    t1 = now();
                    std::printf("staged %-11s th %2d chunk %4zu MB x%d  %.3f s  %.1f GB/s\n", fl.name, th, ck >> 20,
                                nb, t1 - t0, bytes / (t1 - t0) / 1e9);
                    for (int k = 0; k < nb; ++k) {
                        CK(hipHostFree(st[k]));
                        CK(hipEventDestroy(ev[k]));
                    }
                    CK(hipStreamDestroy(s));
                }
            }
        }
    }
    long bad = 0;
    for (size_t i = 0; i < (size_t)cols * rows; i += 4099)
        if (host[i] != 0x01010101) ++bad;
    std::printf("check: %ld bad samples\n", bad);
    delete[] host;
    CK(hipFree(d));
    return 0;
}
