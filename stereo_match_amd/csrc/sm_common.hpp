// sm_common.hpp — gfx950 building blocks shared by the stereo kernels:
// DPP lane exchange within a 16-lane row / across the wave, and widened
// vector loads/stores of small per-lane disparity slices.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smk {

// WTA tie-break.  MODE_SGBM (5 paths) takes its winner inside OpenCV's CV_SIMD128
// loop (x86 builds): each int16 lane (d mod 8) keeps its first minimum and the lowest
// lane holding the overall minimum wins, so equal minima rank by (d mod 8, d)
// (oracle/sgm_np.py:wta_best).  MODE_HH (8 paths) keeps the first minimum.  The rank
// sits in the low 16 bits of the (S << 16 | rank) min-keys; D <= 256.
__device__ __forceinline__ uint32_t wta_rank(int d, bool lane8)
{
    return lane8 ? ((((uint32_t)d & 7u) << 5) | ((uint32_t)d >> 3)) : (uint32_t)d;
}
__device__ __forceinline__ int wta_unrank(uint32_t r, bool lane8)
{
    return lane8 ? (int)(((r & 31u) << 3) | (r >> 5)) : (int)r;
}

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

// OpenCV's sub-pixel step trunc(((Sm - Sq) * 16 + den) / (2 * den)), den = max(Sm + Sq - 2 minS, 1),
// for Sm, Sq in [minS, minS + 65535]: the quotient lies in [-8, 8] and n, d < 2^24, so the f32
// product n * rcp(d) is within 2.5e-6 of n / d (v_rcp_f32: 1 ulp), closer than any non-integer
// quotient lies to an integer (1 / d >= 3.8e-6); an exact integer quotient may land one below
// (toward zero), which the 24-bit remainder check corrects.  ~8 VALU ops instead of the ~25 of
// the integer division; exhaustive over every (Sm - minS, Sq - minS) pair:
// tools/ubench/subpix_exact.hip.
__device__ __forceinline__ int subpix_step(int Sm, int Sq, int minS)
{
    const int den = max(Sm + Sq - 2 * minS, 1);
    const int n = (Sm - Sq) * 16 + den, d = den * 2;
    int q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));  // v_cvt_i32_f32 truncates
    const int rem = n - __mul24(q, d);
    return q + (rem >= d ? 1 : 0) - (rem <= -d ? 1 : 0);
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t src)
{
    // bound_ctrl = false: lanes whose source is outside the row keep `old`.
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, CTRL, 0xF, 0xF, false);
}

// full permutations (every source lane valid): bound_ctrl lets the compiler
// fuse the DPP move into the consuming VALU op (v_min_u32_dpp ...).
template <int CTRL>
__device__ __forceinline__ uint32_t perm_dpp(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}

__device__ __forceinline__ uint32_t row16_min(uint32_t v)
{
    v = min(v, perm_dpp<DPP_QP_XOR1>(v));
    v = min(v, perm_dpp<DPP_QP_XOR2>(v));
    v = min(v, perm_dpp<DPP_ROW_HALF_MIRROR>(v));
    v = min(v, perm_dpp<DPP_ROW_MIRROR>(v));
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

// 8-lane lines (two per DPP row): row shifts plus a fix-up at the half-row edge
template <>
struct Line<8> {
    template <typename T>
    static __device__ __forceinline__ T prev(T edge, T v)
    {
        T r;
        if constexpr (sizeof(T) == 8) r = dpp64<DPP_ROW_SHR1>(edge, v);
        else r = dpp<DPP_ROW_SHR1>(edge, v);
        return (threadIdx.x & 7) == 0 ? edge : r;
    }
    template <typename T>
    static __device__ __forceinline__ T next(T edge, T v)
    {
        T r;
        if constexpr (sizeof(T) == 8) r = dpp64<DPP_ROW_SHL1>(edge, v);
        else r = dpp<DPP_ROW_SHL1>(edge, v);
        return (threadIdx.x & 7) == 7 ? edge : r;
    }
    static __device__ __forceinline__ uint32_t min(uint32_t v);
};

// 4-lane lines (four per DPP row): row shifts plus a fix-up at the quad edge
template <>
struct Line<4> {
    template <typename T>
    static __device__ __forceinline__ T prev(T edge, T v)
    {
        T r;
        if constexpr (sizeof(T) == 8) r = dpp64<DPP_ROW_SHR1>(edge, v);
        else r = dpp<DPP_ROW_SHR1>(edge, v);
        return (threadIdx.x & 3) == 0 ? edge : r;
    }
    template <typename T>
    static __device__ __forceinline__ T next(T edge, T v)
    {
        T r;
        if constexpr (sizeof(T) == 8) r = dpp64<DPP_ROW_SHL1>(edge, v);
        else r = dpp<DPP_ROW_SHL1>(edge, v);
        return (threadIdx.x & 3) == 3 ? edge : r;
    }
};

// 32-lane lines (two per wave, each spanning two DPP rows): whole-wave shifts (DPP
// wave_shr / wave_shl cross the row boundary inside a line) plus a fix-up at the line edge
// (lane 32 would otherwise read lane 31 of the other line)
template <>
struct Line<32> {
    template <typename T>
    static __device__ __forceinline__ T prev(T edge, T v)
    {
        T r;
        if constexpr (sizeof(T) == 8) r = dpp64<DPP_WAVE_SHR1>(edge, v);
        else r = dpp<DPP_WAVE_SHR1>(edge, v);
        return (threadIdx.x & 31) == 0 ? edge : r;
    }
    template <typename T>
    static __device__ __forceinline__ T next(T edge, T v)
    {
        T r;
        if constexpr (sizeof(T) == 8) r = dpp64<DPP_WAVE_SHL1>(edge, v);
        else r = dpp<DPP_WAVE_SHL1>(edge, v);
        return (threadIdx.x & 31) == 31 ? edge : r;
    }
    static __device__ __forceinline__ uint32_t min(uint32_t v);
};

// gfx950 v_permlane16_swap of v with itself: in rows 0 and 1 (2 and 3) the two results hold
// row 0's and row 1's (row 2's and row 3's) values, one each, in some order, so any
// symmetric combination of the pair (min, max, or, +) combines the two rows of a 32-lane half
template <class F>
__device__ __forceinline__ uint32_t row_pair_combine(uint32_t v, F f)
{
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return f((uint32_t)r[0], (uint32_t)r[1]);
}

__device__ __forceinline__ uint32_t row16_or(uint32_t v)
{
    v |= perm_dpp<DPP_QP_XOR1>(v);
    v |= perm_dpp<DPP_QP_XOR2>(v);
    v |= perm_dpp<DPP_ROW_HALF_MIRROR>(v);
    v |= perm_dpp<DPP_ROW_MIRROR>(v);
    return v;
}

__device__ __forceinline__ uint32_t Line<16>::min(uint32_t v) { return row16_min(v); }

__device__ __forceinline__ uint32_t Line<32>::min(uint32_t v)
{
    return row_pair_combine(row16_min(v), [](uint32_t a, uint32_t b) { return ::min(a, b); });
}

__device__ __forceinline__ uint32_t Line<8>::min(uint32_t v)
{
    v = ::min(v, perm_dpp<DPP_QP_XOR1>(v));
    v = ::min(v, perm_dpp<DPP_QP_XOR2>(v));
    v = ::min(v, perm_dpp<DPP_ROW_HALF_MIRROR>(v));
    return v;
}

// whole-wave minimum, returned wave-uniform (SGPR)
__device__ __forceinline__ uint32_t Line<64>::min(uint32_t v)
{
    v = row16_min(v);
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return ::min(::min(a, b), ::min(c, d));
}

// whole-wave reductions (the result in every lane): 16-lane rows by DPP, then the four rows
__device__ __forceinline__ uint32_t group_min_u32_wave(uint32_t v)
{
    v = row16_min(v);
    // readlane returns int: compare as unsigned (keys use the top bit)
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16),
                   c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return ::min(::min(a, b), ::min(c, d));
}
__device__ __forceinline__ uint32_t group_max_u32_wave(uint32_t v)
{
    v = ::max(v, perm_dpp<DPP_QP_XOR1>(v));
    v = ::max(v, perm_dpp<DPP_QP_XOR2>(v));
    v = ::max(v, perm_dpp<DPP_ROW_HALF_MIRROR>(v));
    v = ::max(v, perm_dpp<DPP_ROW_MIRROR>(v));
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16),
                   c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return ::max(::max(a, b), ::max(c, d));
}
__device__ __forceinline__ uint32_t group_sum_u32_wave(uint32_t v)
{
    v += perm_dpp<DPP_QP_XOR1>(v);
    v += perm_dpp<DPP_QP_XOR2>(v);
    v += perm_dpp<DPP_ROW_HALF_MIRROR>(v);
    v += perm_dpp<DPP_ROW_MIRROR>(v);
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
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


// ---------------------------------------------------------- buffer ops
// Raw buffer descriptors (T8/T20 of the CDNA guide): 32-bit byte offsets,
// hardware range check.  Stores at an offset >= num_records are dropped and
// loads there return 0, which lets every per-step memory op stay
// unconditional (no control-flow merge -> the compiler keeps counted
// vmcnt waits instead of vmcnt(0)).
using rsrc_t = __amdgpu_buffer_rsrc_t;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// out-of-range offset for masked lanes: above every volume a descriptor
// covers (per-pair volumes are limited to kMaxRecords bytes on the host side)
// and far enough below 2^32 that the small per-chunk increments never wrap
constexpr uint32_t kOOB = 0xFFFF0000u;
constexpr uint64_t kMaxRecords = 0xFFFE0000ull;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint64_t bytes)
{
    const uint64_t p = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane((uint32_t)(bytes > kMaxRecords ? kMaxRecords : bytes));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, (int)n, 0x00020000);
}

__device__ __forceinline__ uint64_t bload_u64(rsrc_t r, uint32_t off)
{
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return ((uint64_t)v.y << 32) | v.x;
}

// pack N small values (< 2^(8*sizeof(T))) into little-endian 32-bit words
template <typename T, int N>
__device__ __forceinline__ void pack_words(const uint32_t (&in)[N], uint32_t (&w)[(N * sizeof(T) + 3) / 4])
{
    constexpr int NW = (N * (int)sizeof(T) + 3) / 4;
    if constexpr (sizeof(T) == 4) {  // words already packed (u16 pairs of the packed sweeps)
#pragma unroll
        for (int k = 0; k < NW; k++) w[k] = in[k];
    } else if constexpr (sizeof(T) == 1) {
#pragma unroll
        for (int k = 0; k < NW; k++) {
            const uint32_t a = in[4 * k];
            const uint32_t b = 4 * k + 1 < N ? in[4 * k + 1] : 0u;
            const uint32_t c = 4 * k + 2 < N ? in[4 * k + 2] : 0u;
            const uint32_t d = 4 * k + 3 < N ? in[4 * k + 3] : 0u;
            const uint32_t lo = __builtin_amdgcn_perm(b, a, 0x0c0c0400u);  // [a0, b0, 0, 0]
            const uint32_t hi = __builtin_amdgcn_perm(d, c, 0x0c0c0400u);  // [c0, d0, 0, 0]
            w[k] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);             // [a0, b0, c0, d0]
        }
    } else {
#pragma unroll
        for (int k = 0; k < NW; k++) {
            const uint32_t a = in[2 * k];
            const uint32_t b = 2 * k + 1 < N ? in[2 * k + 1] : 0u;
            w[k] = __builtin_amdgcn_perm(b, a, 0x05040100u);  // [a0, a1, b0, b1]
        }
    }
}

// store N values of T at byte offset `off` (N*sizeof(T) bytes), split in
// naturally aligned chunks of gcd(N*sizeof(T), 16) bytes
// AUX: the buffer instruction's cache-policy operand (0 = default; 2 = nt)
template <typename T, int N, int AUX = 0>
__device__ __forceinline__ void bstore_n(rsrc_t r, uint32_t off, const uint32_t (&in)[N])
{
    constexpr int BYTES = N * (int)sizeof(T);
    constexpr int CH = (BYTES % 16 == 0) ? 16 : (BYTES % 8 == 0) ? 8 : (BYTES % 4 == 0) ? 4 : (BYTES % 2 == 0) ? 2 : 1;
    if constexpr (CH >= 4) {
        uint32_t w[(BYTES + 3) / 4];
        pack_words<T, N>(in, w);
#pragma unroll
        for (int c = 0; c < BYTES / CH; c++) {
            if constexpr (CH == 16) {
                const u32x4 v = {w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]};
                __builtin_amdgcn_raw_buffer_store_b128(v, r, off + 16 * c, 0, AUX);
            } else if constexpr (CH == 8) {
                const u32x2 v = {w[2 * c], w[2 * c + 1]};
                __builtin_amdgcn_raw_buffer_store_b64(v, r, off + 8 * c, 0, AUX);
            } else {
                __builtin_amdgcn_raw_buffer_store_b32(w[c], r, off + 4 * c, 0, AUX);
            }
        }
    } else if constexpr (CH == 2) {
        if constexpr (sizeof(T) == 2) {
#pragma unroll
            for (int i = 0; i < N; i++) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)in[i], r, off + 2 * i, 0, AUX);
        } else {
#pragma unroll
            for (int i = 0; i < N / 2; i++)
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(in[2 * i] | (in[2 * i + 1] << 8)), r, off + 2 * i, 0, AUX);
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; i++) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)in[i], r, off + i, 0, AUX);
    }
}

// load N uint16 (raw words, unpacked later)
template <int N>
struct RawU16 {
    static constexpr int BYTES = 2 * N;
    static constexpr int WORDS = (BYTES + 3) / 4;
    uint32_t w[WORDS];
    __device__ __forceinline__ void load(rsrc_t r, uint32_t off)
    {
        if constexpr (BYTES % 16 == 0) {
#pragma unroll
            for (int c = 0; c < BYTES / 16; c++) {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * c, 0, 0);
                w[4 * c] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
            }
        } else if constexpr (BYTES % 8 == 0) {
#pragma unroll
            for (int c = 0; c < BYTES / 8; c++) {
                const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off + 8 * c, 0, 0);
                w[2 * c] = v.x; w[2 * c + 1] = v.y;
            }
        } else if constexpr (BYTES % 4 == 0) {
#pragma unroll
            for (int c = 0; c < WORDS; c++) w[c] = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * c, 0, 0);
        } else {
#pragma unroll
            for (int c = 0; c < N; c++) {
                const uint32_t h = __builtin_amdgcn_raw_buffer_load_b16(r, off + 2 * c, 0, 0);
                if (c & 1) w[c >> 1] |= h << 16;
                else w[c >> 1] = h;
            }
        }
    }
    __device__ __forceinline__ void unpack(uint32_t (&C)[N]) const
    {
#pragma unroll
        for (int i = 0; i < N; i++) C[i] = (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
    }
};

// NB bytes loaded raw into 32-bit words, in naturally aligned chunks of the
// largest power of two (<= 16) dividing NB
template <int NB>
struct RawBytes {
    static constexpr int WORDS = (NB + 3) / 4;
    static constexpr int CH = (NB % 16 == 0) ? 16 : (NB % 8 == 0) ? 8 : (NB % 4 == 0) ? 4 : (NB % 2 == 0) ? 2 : 1;
    uint32_t w[WORDS];
    template <int AUX = 0>  // cache-policy operand (2 = nt)
    __device__ __forceinline__ void load(rsrc_t r, uint32_t off)
    {
        if constexpr (CH == 16) {
#pragma unroll
            for (int c = 0; c < NB / 16; c++) {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * c, 0, AUX);
                w[4 * c] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
            }
        } else if constexpr (CH == 8) {
#pragma unroll
            for (int c = 0; c < NB / 8; c++) {
                const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off + 8 * c, 0, AUX);
                w[2 * c] = v.x; w[2 * c + 1] = v.y;
            }
        } else if constexpr (CH == 4) {
#pragma unroll
            for (int c = 0; c < NB / 4; c++) w[c] = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * c, 0, AUX);
        } else {
#pragma unroll
            for (int c = 0; c < WORDS; c++) w[c] = 0;
#pragma unroll
            for (int c = 0; c < NB / CH; c++) {
                const uint32_t v = CH == 2 ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, off + 2 * c, 0, AUX)
                                           : (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, off + c, 0, AUX);
                w[(c * CH) / 4] |= v << (8 * ((c * CH) % 4));
            }
        }
    }
    template <typename T>
    __device__ __forceinline__ uint32_t get(int i) const
    {
        constexpr int PER = 4 / (int)sizeof(T);
        return (w[i / PER] >> (8 * sizeof(T) * (i % PER))) & ((1u << (8 * sizeof(T))) - 1u);
    }
};

}  // namespace smk
