// sm_common.hpp — gfx950 building blocks shared by the stereo kernels:
// DPP lane exchange within a 16-lane row / across the wave, and widened
// vector loads/stores of small per-lane disparity slices.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smk {

constexpr int kMaxDirs = 8;
constexpr uint32_t kBig = 0x7FFF;  // OpenCV MAX_COST used at d = -1 / d = D

// ----------------------------------------------------------------- DPP ---
enum : int {
    DPP_QP_XOR1 = 0xB1,          // quad_perm [1,0,3,2]
    DPP_QP_XOR2 = 0x4E,          // quad_perm [2,3,0,1]
    DPP_ROW_SHL1 = 0x101,        // lane i <- lane i+1 (within 16-lane row)
    DPP_ROW_SHR1 = 0x111,        // lane i <- lane i-1
    DPP_WAVE_SHL1 = 0x130,       // lane i <- lane i+1 across the wave (lane 63 keeps old)
    DPP_WAVE_SHR1 = 0x138,       // lane i <- lane i-1 across the wave (lane 0 keeps old)
    DPP_ROW_MIRROR = 0x140,      // lane i <- lane 15-i
    DPP_ROW_HALF_MIRROR = 0x141, // lane i <- lane 7-i (per 8-lane half)
    DPP_ROW_BCAST15 = 0x142,     // rows 1..3 <- lane 15 of the previous row
    DPP_ROW_BCAST31 = 0x143      // rows 2..3 <- lane 31
};

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t src)
{
    // bound_ctrl = false: lanes whose source is outside the row keep `old`.
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, CTRL, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t row16_min(uint32_t v)
{
    v = min(v, dpp<DPP_QP_XOR1>(v, v));
    v = min(v, dpp<DPP_QP_XOR2>(v, v));
    v = min(v, dpp<DPP_ROW_HALF_MIRROR>(v, v));
    v = min(v, dpp<DPP_ROW_MIRROR>(v, v));
    return v;
}

template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t old, uint64_t src)
{
    const uint32_t lo = dpp<CTRL>((uint32_t)old, (uint32_t)src);
    const uint32_t hi = dpp<CTRL>((uint32_t)(old >> 32), (uint32_t)(src >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// A "line" is the set of lanes holding one SGM path's D disparities: a
// 16-lane DPP row (4 lines per wave) or the whole wave (1 line per wave).
template <int LANES>
struct Line;

template <>
struct Line<16> {
    // value of the previous / next lane of the line; the first / last lane gets `edge`
    template <typename T>
    static __device__ __forceinline__ T prev(T edge, T v)
    {
        if constexpr (sizeof(T) == 8) return dpp64<DPP_ROW_SHR1>(edge, v);
        else return dpp<DPP_ROW_SHR1>(edge, v);
    }
    template <typename T>
    static __device__ __forceinline__ T next(T edge, T v)
    {
        if constexpr (sizeof(T) == 8) return dpp64<DPP_ROW_SHL1>(edge, v);
        else return dpp<DPP_ROW_SHL1>(edge, v);
    }
    static __device__ __forceinline__ uint32_t min(uint32_t v);
};

template <>
struct Line<64> {
    template <typename T>
    static __device__ __forceinline__ T prev(T edge, T v)
    {
        if constexpr (sizeof(T) == 8) return dpp64<DPP_WAVE_SHR1>(edge, v);
        else return dpp<DPP_WAVE_SHR1>(edge, v);
    }
    template <typename T>
    static __device__ __forceinline__ T next(T edge, T v)
    {
        if constexpr (sizeof(T) == 8) return dpp64<DPP_WAVE_SHL1>(edge, v);
        else return dpp<DPP_WAVE_SHL1>(edge, v);
    }
    static __device__ __forceinline__ uint32_t min(uint32_t v);
};

__device__ __forceinline__ uint32_t row16_or(uint32_t v)
{
    v |= dpp<DPP_QP_XOR1>(v, v);
    v |= dpp<DPP_QP_XOR2>(v, v);
    v |= dpp<DPP_ROW_HALF_MIRROR>(v, v);
    v |= dpp<DPP_ROW_MIRROR>(v, v);
    return v;
}

__device__ __forceinline__ uint32_t Line<16>::min(uint32_t v) { return row16_min(v); }

// whole-wave minimum, returned wave-uniform (SGPR)
__device__ __forceinline__ uint32_t Line<64>::min(uint32_t v)
{
    v = row16_min(v);
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return ::min(::min(a, b), ::min(c, d));
}

// ------------------------------------------------------ vector load/store
template <typename T, int N>
struct Vec {
    T v[N];
};

template <int N, typename T>
__device__ __forceinline__ void load_n(const T* __restrict__ p, uint32_t (&out)[N])
{
    constexpr int BYTES = N * (int)sizeof(T);
    if constexpr (BYTES % 16 == 0) {
#pragma unroll
        for (int c = 0; c < BYTES / 16; c++) {
            uint4 w = reinterpret_cast<const uint4*>(p)[c];
            const T* t = reinterpret_cast<const T*>(&w);
#pragma unroll
            for (int i = 0; i < 16 / (int)sizeof(T); i++) out[c * (16 / sizeof(T)) + i] = t[i];
        }
    } else if constexpr (BYTES % 8 == 0) {
#pragma unroll
        for (int c = 0; c < BYTES / 8; c++) {
            uint2 w = reinterpret_cast<const uint2*>(p)[c];
            const T* t = reinterpret_cast<const T*>(&w);
#pragma unroll
            for (int i = 0; i < 8 / (int)sizeof(T); i++) out[c * (8 / sizeof(T)) + i] = t[i];
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; i++) out[i] = p[i];
    }
}

template <int N, typename T>
__device__ __forceinline__ void store_n(T* __restrict__ p, const uint32_t (&in)[N])
{
    constexpr int BYTES = N * (int)sizeof(T);
    if constexpr (BYTES % 16 == 0) {
#pragma unroll
        for (int c = 0; c < BYTES / 16; c++) {
            uint4 w;
            T* t = reinterpret_cast<T*>(&w);
#pragma unroll
            for (int i = 0; i < 16 / (int)sizeof(T); i++) t[i] = (T)in[c * (16 / sizeof(T)) + i];
            reinterpret_cast<uint4*>(p)[c] = w;
        }
    } else if constexpr (BYTES % 8 == 0) {
#pragma unroll
        for (int c = 0; c < BYTES / 8; c++) {
            uint2 w;
            T* t = reinterpret_cast<T*>(&w);
#pragma unroll
            for (int i = 0; i < 8 / (int)sizeof(T); i++) t[i] = (T)in[c * (8 / sizeof(T)) + i];
            reinterpret_cast<uint2*>(p)[c] = w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; i++) p[i] = (T)in[i];
    }
}

}  // namespace smk
