// stamps.h -- diagnostic in-kernel phase stamps (s_memtime), compiled in only with
// -DSTOMP_STAMPS (a separate diagnostic library, never the benchmarked one).  Thread 0 of
// the selected workgroup records the shader clock at named phase boundaries into a
// per-translation-unit device array; STOMP_STAMP_ACCESSORS(name) defines
// extern "C" stomp_debug_stamps_<name>(int block, unsigned long long* out) to read it.
#pragma once

#include <hip/hip_runtime.h>

#ifdef STOMP_STAMPS
static __device__ unsigned long long g_stamps[256];
static __device__ int g_stamp_block;
#define STAMP(i)                                                                                        \
    do {                                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                                              \
        if (threadIdx.x == 0 && (int)(blockIdx.x + blockIdx.y * gridDim.x) == g_stamp_block) {          \
            unsigned long long _t;                                                                      \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                 \
            g_stamps[(i)] = _t;                                                                         \
        }                                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                                              \
    } while (0)
// the same from whichever workgroup executes it (e.g. the last-arriving one of a launch)
#define STAMP_ANY(i)                                                                                    \
    do {                                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                                              \
        if (threadIdx.x == 0) {                                                                         \
            unsigned long long _t;                                                                      \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                 \
            g_stamps[(i)] = _t;                                                                         \
        }                                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                                              \
    } while (0)
// Per-workgroup residency record: {HW_ID, XCC_ID, start, end} for blocks < 8192, to measure
// how many workgroups of a launch actually share a CU.
static __device__ unsigned long long g_blocks[8192][6];
#define BLOCK_BEGIN()                                                                                   \
    do {                                                                                                \
        if (threadIdx.x == 0 && blockIdx.x < 8192) {                                                    \
            unsigned long long _t;                                                                      \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                  \
            g_blocks[blockIdx.x][0] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);             \
            g_blocks[blockIdx.x][1] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);            \
            g_blocks[blockIdx.x][2] = _t;                                                               \
        }                                                                                               \
    } while (0)
#define BLOCK_END()                                                                                     \
    do {                                                                                                \
        if (threadIdx.x == 0 && blockIdx.x < 8192) {                                                    \
            unsigned long long _t;                                                                      \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                  \
            g_blocks[blockIdx.x][3] = _t;                                                               \
        }                                                                                               \
    } while (0)
// per-block phase mark k (4 or 5): the shader clock when thread 0 passes it
#define BLOCK_MARK(k)                                                                                   \
    do {                                                                                                \
        if (threadIdx.x == 0 && blockIdx.x < 8192) {                                                    \
            unsigned long long _t;                                                                      \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                  \
            g_blocks[blockIdx.x][(k)] = _t;                                                             \
        }                                                                                               \
    } while (0)
#define STOMP_STAMP_ACCESSORS(name)                                                                     \
    extern "C" int stomp_debug_stamps_##name(int block, unsigned long long* out, int reset)            \
    {                                                                                                   \
        if (out) hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps));                      \
        if (reset) {                                                                                    \
            static unsigned long long zero[256];                                                        \
            hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero));                                \
            hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_block), &block, sizeof(int));                          \
        }                                                                                               \
        return 0;                                                                                       \
    }                                                                                                   \
    extern "C" int stomp_debug_blocks_##name(unsigned long long* out)                                  \
    {                                                                                                   \
        return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_blocks), sizeof(g_blocks)) == hipSuccess ? 0 : -1; \
    }
#else
#define STAMP(i) \
    do {         \
    } while (0)
#define STAMP_ANY(i) \
    do {             \
    } while (0)
#define BLOCK_BEGIN() \
    do {              \
    } while (0)
#define BLOCK_END() \
    do {            \
    } while (0)
#define BLOCK_MARK(k) \
    do {              \
    } while (0)
#define STOMP_STAMP_ACCESSORS(name)
#endif
