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

// Spin (s_sleep between polls) until word[0] >= value; after `ticks` of
// s_memrealtime (100 MHz) give up and record the failure in word[1] (the host
// reads it with nw_link_status).
__global__ __launch_bounds__(64) void nw_link_wait(uint32_t *word, uint32_t value, uint64_t ticks) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint32_t v = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((int32_t)(v - value) >= 0) return;
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
            __hip_atomic_store(word + 1, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

int launch_link_wait(uint32_t *word, uint32_t value, uint64_t ticks, void *stream) {
    hipLaunchKernelGGL(nw_link_wait, dim3(1), dim3(64), 0, (hipStream_t)stream, word, value, ticks);
    return (int)hipGetLastError();
}

int launch_link_signal(uint32_t *word, uint32_t value, void *stream) {
    hipLaunchKernelGGL(nw_link_signal, dim3(1), dim3(64), 0, (hipStream_t)stream, word, value);
    return (int)hipGetLastError();
}

}  // namespace nw
