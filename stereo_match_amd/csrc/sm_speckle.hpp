// sm_speckle.hpp — cv::filterSpeckles on the GPU (applied by
// StereoSGBM::compute after the 3x3 median when speckleWindowSize > 0,
// reference settings at settings.ini:14-17).  Semantics: oracle/sgm_np.py
// filter_speckles / oracle/sgm_ref.c sgm_ref_filter_speckles: 4-connected
// regions of pixels != newval whose neighbours differ by <= maxdiff; regions
// of <= maxsize pixels become newval.
//
// The region set is the connected components of that graph, so the result
// does not depend on OpenCV's scan order and a parallel labelling reproduces
// it exactly:
//   k_speckle_init   parent[p] = p for valid pixels, -1 otherwise
//   k_speckle_union  each pixel unites with its right / lower neighbour when
//                    the edge exists (lock-free union-find: the larger root is
//                    CAS-linked to the smaller one, so parents only decrease
//                    and every find terminates)
//   k_speckle_count  find (with path halving) + atomicAdd of the region size
//   k_speckle_apply  read-only find; regions of <= maxsize pixels -> newval
// Every loop is bounded by the pixel count, so a logic error cannot hang the
// GPU (it would surface as a parity failure instead).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smk {

struct SpeckleArgs {
    int16_t* img;  // [pair][H][W], filtered in place
    int* parent;   // [pair][H*W]
    int* count;    // [pair][H*W]
    int H, W, newval, maxsize, maxdiff;
};

__device__ inline int sp_load(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Root of x.  HALVE: path halving (parent[x] = grandparent).  Halving can
// overwrite a pointer another thread just compressed to the root with a
// lower ancestor, so after the counting pass roots are found again read-only.
template <bool HALVE>
__device__ inline int sp_find(int* parent, int x, int limit)
{
    for (int it = 0; it < limit; it++) {
        const int px = sp_load(parent + x);
        if (px == x) return x;
        if (!HALVE) {
            x = px;
            continue;
        }
        const int gp = sp_load(parent + px);
        if (gp != px) __hip_atomic_store(parent + x, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        x = gp;
    }
    return x;
}

__device__ inline void sp_unite(int* parent, int a, int b, int limit)
{
    for (int it = 0; it < limit; it++) {
        a = sp_find<true>(parent, a, limit);
        b = sp_find<true>(parent, b, limit);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        int expected = a;
        if (__hip_atomic_compare_exchange_strong(parent + a, &expected, b, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return;
        a = expected;  // a was linked meanwhile: retry from its new parent
    }
}

__global__ void __launch_bounds__(256) k_speckle_init(SpeckleArgs s)
{
    const int n = s.H * s.W;
    const int p = blockIdx.x * 256 + threadIdx.x, pair = blockIdx.y;
    if (p >= n) return;
    const int16_t* img = s.img + (size_t)pair * n;
    s.parent[(size_t)pair * n + p] = img[p] != s.newval ? p : -1;
    s.count[(size_t)pair * n + p] = 0;
}

__global__ void __launch_bounds__(256) k_speckle_union(SpeckleArgs s)
{
    const int n = s.H * s.W;
    const int p = blockIdx.x * 256 + threadIdx.x, pair = blockIdx.y;
    if (p >= n) return;
    const int16_t* img = s.img + (size_t)pair * n;
    int* parent = s.parent + (size_t)pair * n;
    const int v = img[p];
    if (v == s.newval) return;
    const int x = p % s.W, y = p / s.W;
    if (x + 1 < s.W) {
        const int q = img[p + 1];
        if (q != s.newval && abs(v - q) <= s.maxdiff) sp_unite(parent, p, p + 1, n + 1);
    }
    if (y + 1 < s.H) {
        const int q = img[p + s.W];
        if (q != s.newval && abs(v - q) <= s.maxdiff) sp_unite(parent, p, p + s.W, n + 1);
    }
}

__global__ void __launch_bounds__(256) k_speckle_count(SpeckleArgs s)
{
    const int n = s.H * s.W;
    const int p = blockIdx.x * 256 + threadIdx.x, pair = blockIdx.y;
    if (p >= n) return;
    int* parent = s.parent + (size_t)pair * n;
    if (sp_load(parent + p) < 0) return;
    const int r = sp_find<true>(parent, p, n + 1);
    atomicAdd(s.count + (size_t)pair * n + r, 1);
}

__global__ void __launch_bounds__(256) k_speckle_apply(SpeckleArgs s)
{
    const int n = s.H * s.W;
    const int p = blockIdx.x * 256 + threadIdx.x, pair = blockIdx.y;
    if (p >= n) return;
    int* parent = s.parent + (size_t)pair * n;
    if (parent[p] < 0) return;
    const int r = sp_find<false>(parent, p, n + 1);
    if (s.count[(size_t)pair * n + r] <= s.maxsize) s.img[(size_t)pair * n + p] = (int16_t)s.newval;
}

}  // namespace smk
