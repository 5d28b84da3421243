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

    double t0 = now();
    CK(hipMemcpy2D(host, w, d, pitch * 4, w, rows, hipMemcpyDeviceToHost));
    double t1 = now();
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
    for (int nb : {2, 3}) {
        std::vector<char *> st(nb);
        std::vector<hipEvent_t> ev(nb);
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        for (int k = 0; k < nb; ++k) {
            CK(hipHostMalloc((void **)&st[k], chunk, 0));
            CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
        }
        const long rpc = std::max<long>(1, (long)(chunk / w));
        const long nch = (rows + rpc - 1) / rpc;
        t0 = now();
        auto issue = [&](long c) {
            const long r0 = c * rpc, nr = std::min(rpc, rows - r0);
            CK(hipMemcpy2DAsync(st[c % nb], w, d + r0 * pitch, pitch * 4, w, nr, hipMemcpyDeviceToHost, s));
            CK(hipEventRecord(ev[c % nb], s));
        };
        for (long c = 0; c < std::min<long>(nb, nch); ++c) issue(c);
        for (long c = 0; c < nch; ++c) {
            CK(hipEventSynchronize(ev[c % nb]));
            const long r0 = c * rpc, nr = std::min(rpc, rows - r0);
            par_copy((char *)host + (size_t)r0 * w, st[c % nb], (size_t)nr * w, threads);
            if (c + nb < nch) issue(c + nb);
        }
        t1 = now();
        std::printf("staged x%d  %.3f s  %.1f GB/s\n", nb, t1 - t0, bytes / (t1 - t0) / 1e9);
        for (int k = 0; k < nb; ++k) {
            CK(hipHostFree(st[k]));
            CK(hipEventDestroy(ev[k]));
        }
        CK(hipStreamDestroy(s));
    }
    long bad = 0;
    for (size_t i = 0; i < (size_t)cols * rows; i += 4099)
        if (host[i] != 0x01010101) ++bad;
    std::printf("check: %ld bad samples\n", bad);
    delete[] host;
    CK(hipFree(d));
    return 0;
}
