// sm_reproject.hpp — cv::reprojectImageTo3D on the GPU (the
// reference reprojects the filtered int16 map at disparity_calculation.py:302,
// and float32 disparity/16 in stereo_vision.py:203-209 project_points_3D).
// Semantics: oracle/reproject_np.py.  Per pixel, in float64 with FP
// contraction off:
//   qx = Q01*y + Q03 + Q00*x   (likewise qy, qz, qw with rows 1..3)
//   iW = 1/(qw + Q32*d);  X = (qx + Q02*d)*iW;  Y = (qy + Q12*d)*iW;
//   Z = (qz + Q22*d)*iW, or 10000 when handleMissingValues and d is the map's
//   minimum; stored as float32 xyz.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smk {

struct ReprojArgs {
    const void* disp;  // [img][H][W] int16 or float32
    float* xyz;        // [img][H][W][3]
    double Q[16];
    int H, W, handle_missing;
    const float* min_disp;  // [img] (handle_missing)
};

__device__ inline float disp_value(const int16_t* p, size_t i) { return (float)p[i]; }
__device__ inline float disp_value(const float* p, size_t i) { return p[i]; }

template <typename T>
__global__ void __launch_bounds__(256) k_reproject(ReprojArgs a)
{
#pragma clang fp contract(off)
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, img = blockIdx.z;
    if (x >= a.W) return;
    const size_t npx = (size_t)a.H * a.W;
    const size_t i = img * npx + (size_t)y * a.W + x;
    const double d = (double)disp_value(reinterpret_cast<const T*>(a.disp), i);
    const double* Q = a.Q;
    const double qx = Q[1] * y + Q[3] + Q[0] * x;
    const double qy = Q[5] * y + Q[7] + Q[4] * x;
    const double qz = Q[9] * y + Q[11] + Q[8] * x;
    const double qw = Q[13] * y + Q[15] + Q[12] * x;
    const double iW = 1.0 / (qw + Q[14] * d);
    const double X = (qx + Q[2] * d) * iW;
    const double Y = (qy + Q[6] * d) * iW;
    double Z = (qz + Q[10] * d) * iW;
    if (a.handle_missing) {
        const double md = (double)a.min_disp[img];
        if (fabs(d - md) <= 1.1920928955078125e-07) Z = 10000.0;  // FLT_EPSILON, bigZ
    }
    float* o = a.xyz + 3 * i;
    o[0] = (float)X;
    o[1] = (float)Y;
    o[2] = (float)Z;
}

// per-image minimum (handleMissingValues): order-preserving int key of float
__device__ inline int float_key(float f)
{
    const int b = __float_as_int(f);
    return b >= 0 ? b : b ^ 0x7FFFFFFF;
}
__device__ inline float key_float(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7FFFFFFF); }

template <typename T>
__global__ void __launch_bounds__(256) k_disp_min(const T* disp, int* keys, size_t npx)
{
    const int img = blockIdx.y;
    int m = 0x7FFFFFFF;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < npx; i += (size_t)gridDim.x * 256)
        m = min(m, float_key(disp_value(disp, img * npx + i)));
    for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMin(keys + img, m);
}

__global__ void k_keys_to_float(const int* keys, float* out, int n)
{
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i < n) out[i] = key_float(keys[i]);
}

}  // namespace smk
