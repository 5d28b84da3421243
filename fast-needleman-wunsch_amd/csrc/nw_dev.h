// nw_dev.h -- device helpers shared by the gfx950 fill kernels (nw_fill.hip:
// anti-diagonal strips, nw_rows.hip: row-scan panels): the watchdog, the LDS
// counters, the {tag, value} hand-off granules and their bounded waits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "nw_internal.h"

namespace nw {

// s_memrealtime runs at 100 MHz on gfx9: 20 s watchdog for every bounded spin.
// (the bound of every spin: FillArgs::timeout_ticks, 20 s unless nw_params.timeout_ms says otherwise)
constexpr int32_t kDone = 0x7FFFFFFF;  // counter value: "no more waiting on me"
constexpr int32_t kDead = INT32_MIN;   // wait_counter: gave up (watchdog / error word)

// Watchdog diagnosis: the first bounded wait that gives up records where
// (ctrl[1] = error code, ctrl[2] = site << 24 | wave << 16 | LDS/granule word
// offset, ctrl[3] = the value it needed, ctrl[4] = the value it last saw).
__device__ __forceinline__ void give_up(uint32_t *ctrl, uint32_t code, uint32_t site,
                                        const void *p, int64_t need, int64_t seen) {
    if ((threadIdx.x & 63) != 0) return;
    if (atomicCAS(ctrl + 1, 0u, code) == 0u) {
        ctrl[2] = (site << 24) | ((threadIdx.x >> 6) << 16) | ((uint32_t)(uintptr_t)p & 0xFFFFu);
        ctrl[3] = (uint32_t)need;
        ctrl[4] = (uint32_t)seen;
    }
}

// Compiler-only ordering of LDS accesses around the workgroup counters.  One
// wave's LDS instructions execute in order, so a counter store placed after the
// data it publishes (and a data load placed after the counter load that
// allowed it) is ordered for the other waves; the barrier only stops the
// compiler from moving plain loads/stores across the relaxed counter accesses.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }
// Granules are system-scope: the same loads and stores serve a column band's
// feed, which lives in the neighbouring GPU's HBM (written over xGMI).  (Agent
// scope on a single GPU measured no faster, profiles/r04u_gran_agent_ab.txt.)
#define NW_GRAN_SCOPE __HIP_MEMORY_SCOPE_SYSTEM
__device__ __forceinline__ uint64_t gran_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, NW_GRAN_SCOPE);
}
__device__ __forceinline__ uint64_t gran_load(const __attribute__((address_space(1))) uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, NW_GRAN_SCOPE);
}
__device__ __forceinline__ void gran_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, NW_GRAN_SCOPE);
}
__device__ __forceinline__ uint32_t ctrl_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// workgroup counters in LDS (relaxed atomics: plain ds_read/ds_write that the
// compiler may neither cache nor drop)
__device__ __forceinline__ int32_t ctr_load(const int32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void ctr_store(int32_t *p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Slow path of the hand-off: re-poll the granules of one 64-row block until
// those of chunk c (lanes Gc .. Gc+G-1, G rows per chunk) carry `tag` (s_sleep
// between polls).
// Bounded: gives up -- raising the error word -- after `tmo` ticks, or at once
// if another wave already raised it.  Returns the last value read; the caller
// re-checks its tag.
//
// Every loop that polls global memory lives in a __noinline__ function reached
// only on a slow path.  Inlined, such a loop issues an unknown number of vector
// memory operations, after which the compiler can no longer count the prefetch
// loads still in flight and waits for ALL of them (s_waitcnt vmcnt(0)) before
// the next use of any -- once per iteration, on the fast path too.  A call
// drains the counters on the slow path only (the callee's entry waits), so the
// fast path keeps counted vmcnt(N) waits.
//
// The poll is SERIAL: one load in flight, s_sleep 1 between polls.  (Round 4
// measured a pipelined poll -- 4 loads in flight per waiting wave -- SLOWER on the
// same box, profiles/r04c_poll_ab.txt: 256k panels 44.9 -> 48.7 ms, SW 64k strip
// fill 6.3 -> 7.5 ms: the extra loads of every waiting wave compete with the
// fill's own traffic.)  The error word and the watchdog are checked every
// kPollCheck polls only, so a poll is one round trip instead of two and the one
// error word is not re-read by every waiting wave of the chip after each poll
// (round 5, measured neutral on the band, the SW fill and the 256k bench: the
// r05x section of profiles/r05y_poll_sleep.txt).  The loads are global (the
// generic pointer of a noinline callee would make them flat loads).
constexpr uint32_t kPollCheck = 32;
template <int G, int SLEEP>
__device__ __noinline__ uint64_t wait_chunk(const uint64_t *g, uint32_t tag, int c,
                                            uint32_t *ctrl, uint32_t site, uint64_t tmo) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63;
    const bool in_chunk = lane / G == c;
    const __attribute__((address_space(1))) uint64_t *gg = (const __attribute__((address_space(1))) uint64_t *)g;
    for (uint32_t n = 1;; ++n) {
        __builtin_amdgcn_s_sleep(SLEEP);
        const uint64_t v = gran_load(gg);
        if (__all(!in_chunk || (uint32_t)(v >> 32) == tag)) return v;
        if (n % kPollCheck == 0u) {
            if (ctrl_load(ctrl + 1) != 0u) return v;
            if (__builtin_amdgcn_s_memrealtime() - t0 > tmo) {
                give_up(ctrl, 1u, site, g, tag, (int64_t)(v >> 32));
                return v;
            }
        }
    }
}

// Leading G-row chunks of a block whose granules all carry `tag` (0 .. 64/G).
template <int G>
__device__ __forceinline__ int chunks_ready(uint64_t v, uint32_t tag) {
    const uint64_t ok = __ballot((uint32_t)(v >> 32) == tag);
    const int run = ok == ~0ull ? 64 : (int)__builtin_ctzll(~ok);  // leading tagged rows
    return run / G;
}

// Bounded spin until the LDS counter *p reaches `need`; returns the value seen
// (kDead once the watchdog expires).  The loop touches only LDS: a global memory
// access in it would make the compiler drain every store and prefetch the wave
// has in flight (s_waitcnt vmcnt(0)) each time it waits -- for a store wave, the
// whole point of having stores in flight -- and a scalar poll of the error word
// from every wave of the chip at once slows the fill a hundredfold (measured).
// A wave that gives up releases the waves waiting on it anyway: compute_strip
// and store_strip publish kDone on every exit path.
__device__ __noinline__ void wait_expired(uint32_t *ctrl, uint32_t site, const int32_t *p, int32_t need,
                                          int32_t seen) {
    give_up(ctrl, 3u, site, p, need, seen);
}
__device__ __forceinline__ int32_t wait_counter(const int32_t *p, int32_t need, uint32_t *ctrl,
                                             uint32_t site, uint64_t tmo) {
    int32_t v = __builtin_amdgcn_readfirstlane(ctr_load(p));
    if (v >= need) return v;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        __builtin_amdgcn_s_sleep(1);
        v = __builtin_amdgcn_readfirstlane(ctr_load(p));
        if (v >= need) return v;
        // twice the hand-off bound: a partner in the workgroup only stalls behind
        // a hand-off or halo wait, and that wait must be the one that reports
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2 * tmo) break;
    }
    wait_expired(ctrl, site, p, need, v);
    return kDead;
}

// Compile-time loop: f(std::integral_constant<int, U>) for U in [B, E).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// How a cell's substitution score is formed (see nw_fill.hip diag_plus_sub and
// nw_rows.hip sub_score): table lookups (PERM), compares (UNIT / GEN), and the
// Smith-Waterman forms of both.
enum Sub { SUB_PERM = 0, SUB_UNIT = 1, SUB_GEN = 2, SUB_PERM_SW = 3, SUB_GEN_SW = 4 };
template <int MODE> constexpr bool is_sw() { return MODE == SUB_PERM_SW || MODE == SUB_GEN_SW; }

}  // namespace nw
