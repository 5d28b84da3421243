// nw_link.hip -- launch-to-launch flow control between neighbouring bands.
//
// A multi-GPU band sweep (nw_bands.py; the reference's mpi-horz / mpi-vert
// pipelines, src/mpi/mpi-horz.cpp:27-43) enqueues K fills back to back on every
// rank with no host round trip between them.  Launch k uses the halo / feed
// buffer k % 2, so launch k + 2 of the PRODUCER rewrites the buffer launch k of
// the CONSUMER reads.  The consumer therefore signals "consumed through launch
// k" into a word in the producer's memory (peer store over xGMI) after its fill
// k, and the producer's stream waits on that word before fill k + 2.  Both are
// one-lane kernels on the fill's stream: no hipStreamWaitValue (it would park a
// hardware queue) and no host involvement.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_internal.h"

namespace nw {

// A context's control words (nw_capi.cpp nw_ctx::ctrl, 16 words): [0..7] belong
// to one launch (ticket, error code, watchdog site / need / seen -- nw_dev.h
// give_up) and are reset before every launch; [8..11] keep the FIRST failure
// since the host last read the status (code, site, need, seen) and [12] counts
// the failed launches since then; [13] = 1 once the host has read the words
// (the last launch's failure is then not recorded again).  The reset folds the previous launch's words
// into them instead of clearing them, so a watchdog trip in any launch of a
// back-to-back sweep survives the launches after it (nw_ctx_status reads and
// clears them), and a context that has failed POISONS its next launches: their
// error word starts at the recorded failure, so every wait in them gives up at
// once and no halo / feed is published (nw_strips.h / nw_rows.hip publish only
// while the error word is 0) -- a producer that lost its consumer never rewrites
// a buffer the consumer may still be reading.
__global__ __launch_bounds__(64) void nw_ctrl_reset(uint32_t *ctrl) {
    if (threadIdx.x != 0) return;
    // ctrl[13]: the host has read (nw_ctx_status) the previous launch's words already
    const uint32_t code = ctrl[13] != 0u ? 0u : ctrl[1];
    ctrl[13] = 0u;
    if (code != 0u) {
        if (ctrl[8] == 0u) {
            ctrl[9] = ctrl[2];
            ctrl[10] = ctrl[3];
            ctrl[11] = ctrl[4];
            ctrl[8] = code;
        }
        ctrl[12] += 1u;
    }
    for (int k = 0; k < 8; ++k) ctrl[k] = 0u;
    if (ctrl[8] != 0u) {
        ctrl[2] = ctrl[9];
        ctrl[3] = ctrl[10];
        ctrl[4] = ctrl[11];
        ctrl[1] = ctrl[8];
    }
}

// Spin (s_sleep between polls) until word[0] >= value; after `ticks` of
// s_memrealtime (100 MHz) give up and record the failure in word[1] (the host
// reads it with nw_link_status) and, with a context's control words `poison`,
// as that context's failure (code 4, site 20): its next fill then gives up at
// once instead of rewriting the buffer the consumer has not released.
__global__ __launch_bounds__(64) void nw_link_wait(uint32_t *word, uint32_t value, uint64_t ticks,
                                                   uint32_t *poison) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint32_t v = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((int32_t)(v - value) >= 0) return;
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
            __hip_atomic_store(word + 1, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (poison != nullptr && atomicCAS(poison + 8, 0u, 4u) == 0u) {
                poison[9] = 20u << 24;
                poison[10] = value;
                poison[11] = v;
            }
            if (poison != nullptr) atomicAdd(poison + 12, 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

// word[0] = value, a system-scope store (the word may live in a peer GPU's
// memory).  The fill kernel before it on the stream has finished, so every
// halo / feed read of that launch is done.
__global__ __launch_bounds__(64) void nw_link_signal(uint32_t *word, uint32_t value) {
    if (threadIdx.x == 0) __hip_atomic_store(word, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int launch_ctrl_reset(uint32_t *ctrl, void *stream) {
    hipLaunchKernelGGL(nw_ctrl_reset, dim3(1), dim3(64), 0, (hipStream_t)stream, ctrl);
    return (int)hipGetLastError();
}

int launch_link_wait(uint32_t *word, uint32_t value, uint64_t ticks, uint32_t *poison, void *stream) {
    hipLaunchKernelGGL(nw_link_wait, dim3(1), dim3(64), 0, (hipStream_t)stream, word, value, ticks, poison);
    return (int)hipGetLastError();
}

int launch_link_signal(uint32_t *word, uint32_t value, void *stream) {
    hipLaunchKernelGGL(nw_link_signal, dim3(1), dim3(64), 0, (hipStream_t)stream, word, value);
    return (int)hipGetLastError();
}

}  // namespace nw
