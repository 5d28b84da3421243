// panel_store.hip -- the row-scan panel fill's store side alone at the bench's
// scale (262144 x 262144 int32, 1 MB pitch): 256 workgroups, panel p = columns
// [1024p, 1024p+1024), NS store waves per workgroup, store wave w writes the
// 1 KB piece (w % 4) of rows w/4, w/4 + NS/4, ... (one row per store
// instruction, the fill's pattern), panel p trailing panel p-1 by `lag` rows.
//   hipcc --offload-arch=gfx950 -O3 panel_store.hip -o panel_store
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned v4 __attribute__((ext_vector_type(4)));

template <int NS, int BATCH, bool NT = false>
__global__ __launch_bounds__(64 * NS) void sweep(char *t, long pitchb, long nrows, int lag) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int piece = wave & 3, sub = wave >> 2;
    constexpr int NSUB = NS / 4;
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    const long r0 = ((long)blockIdx.x * lag) % nrows;
    char *base = t + (long)blockIdx.x * 4096 + piece * 1024 + lane * 16;
    // rows in batches of BATCH, batches dealt round robin to the NSUB waves of a piece
    for (long f = (long)sub * BATCH; f < nrows; f += (long)NSUB * BATCH) {
#pragma unroll
        for (int g = 0; g < BATCH; ++g) {
            long row = f + g + r0;
            if (f + g >= nrows) break;
            if (row >= nrows) row -= nrows;
            if constexpr (NT)
                __builtin_nontemporal_store(v, (v4 *)(base + row * pitchb));
            else
                *(v4 *)(base + row * pitchb) = v;
            v.x += 1;
        }
    }
}

template <int NS, int BATCH, bool NT = false>
static void run(char *t, long pitchb, long nrows, int lag) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((sweep<NS, BATCH, NT>), dim3(256), dim3(64 * NS), 0, 0, t, pitchb, nrows, lag);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL((sweep<NS, BATCH, NT>), dim3(256), dim3(64 * NS), 0, 0, t, pitchb, nrows, lag);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 3;
    const double bytes = 262144.0 * 4096.0 / 4.0 * 4.0 * (double)nrows / 262144.0 * 256.0;  // 256 panels x 4 KB x rows
    printf("store waves/CU=%d batch=%d nt=%d lag=%d: %.2f ms  %.0f GB/s\n", NS, BATCH, (int)NT, lag, ms, bytes / (ms * 1e6));
}

int main(int argc, char **argv) {
    // panel_store [pitch slack in int32, default 64] [lags, default 0,9,64,256] [all shapes 0/1]
    const long n = 262144, nrows = n + 1;
    const long slack = argc > 1 ? atol(argv[1]) : 64;
    const long pitch = n + slack;
    const long pitchb = pitch * 4;
    const bool all = argc > 3 ? atoi(argv[3]) != 0 : true;
    char *t = nullptr;
    if (hipMalloc(&t, (size_t)(nrows * pitchb + 4096)) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    printf("pitch %ld (slack %ld)\n", pitch, slack);
    int lags[16], nl = 0;
    if (argc > 2) {
        for (char *q = argv[2]; *q && nl < 16;) {
            lags[nl++] = (int)strtol(q, &q, 10);
            if (*q == ',') ++q;
        }
    } else {
        lags[0] = 0, lags[1] = 9, lags[2] = 64, lags[3] = 256, nl = 4;
    }
    for (int li = 0; li < nl; ++li) {
        const int lag = lags[li];
        if (all) {
            run<4, 1>(t, pitchb, nrows, lag);
            run<4, 8>(t, pitchb, nrows, lag);
            run<12, 8>(t, pitchb, nrows, lag);
        }
        run<8, 8>(t, pitchb, nrows, lag);
        run<8, 8, true>(t, pitchb, nrows, lag);
    }
    (void)hipFree(t);
    return 0;
}
