// sm_ew.hip — translation unit of the packed horizontal-line kernel (sm_ew.hpp).
#include "sm_ew.hpp"

namespace smk {

namespace {

// ring depth: <= 64 VGPRs.  u16 slices of <= 2 words take 32 slots (sgbm5, 8 KITTI pairs, 32-lane
// lines: 5016 -> 5066 pairs/s); the u8 lines keep 16 (beside the census down sweep a deeper
// ring made the lines slower and the total worse: 6185 -> 5670)
template <typename CT>
constexpr int ew_pf(int words) { return words >= 16 ? 4 : words >= 8 ? 8 : (sizeof(CT) == 2 && words <= 2) ? 32 : 16; }

template <int VL, int NP, typename CT>
hipError_t run_ew(EwArgs a, int npairs, hipStream_t stream)
{
    constexpr int WORDS = RawBytes<2 * NP * (int)sizeof(CT)>::WORDS;
    constexpr int LPW = 64 / VL;
    if (a.wpb < 1 || a.wpb > 4) a.wpb = 4;
    a.nrb = (a.H + a.wpb * LPW - 1) / (a.wpb * LPW);
    hipLaunchKernelGGL((k_ew<VL, NP, CT, CT, ew_pf<CT>(WORDS)>), dim3(2 * a.nrb, npairs), dim3(64 * a.wpb), 0, stream, a);
    return hipGetLastError();
}

template <typename CT>
hipError_t ew_d(int D, int vl, const EwArgs& a, int npairs, hipStream_t stream)
{
    if (D == 128 && vl == 4) return run_ew<4, 16, CT>(a, npairs, stream);
    // latency forms for a few pairs per launch (more lanes per line: less work per lane and
    // step on the serial chain): 16-lane lines for D % 32 == 0, 32-lane lines for D % 64 == 0
    if (vl == 16) {
        switch (D) {
#define EW16(d) \
    case d: return run_ew<16, d / 32, CT>(a, npairs, stream);
            EW16(32) EW16(64) EW16(96) EW16(128) EW16(160) EW16(192) EW16(224) EW16(256)
#undef EW16
        default: return hipErrorInvalidValue;
        }
    }
    if (vl == 64) {  // one line per wave (measurement instances, SM_TUNE_EW_LANES 64)
        switch (D) {
        case 128: return run_ew<64, 1, CT>(a, npairs, stream);
        case 256: return run_ew<64, 2, CT>(a, npairs, stream);
        default: return hipErrorInvalidValue;
        }
    }
    if (vl == 32) {
        switch (D) {
        case 64: return run_ew<32, 1, CT>(a, npairs, stream);
        case 128: return run_ew<32, 2, CT>(a, npairs, stream);
        case 192: return run_ew<32, 3, CT>(a, npairs, stream);
        case 256: return run_ew<32, 4, CT>(a, npairs, stream);
        default: return hipErrorInvalidValue;
        }
    }
    if (vl != 0 && vl != 8) return hipErrorInvalidValue;
    switch (D) {  // 8-lane lines, D / 16 u16 pairs per lane
#define EW8(d) \
    case d: return run_ew<8, d / 16, CT>(a, npairs, stream);
        EW8(16) EW8(32) EW8(48) EW8(64) EW8(80) EW8(96) EW8(112) EW8(128)
        EW8(144) EW8(160) EW8(176) EW8(192) EW8(208) EW8(224) EW8(240) EW8(256)
#undef EW8
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

namespace {

template <int VL, int NP, typename CT>
hipError_t run_patch(const EwPatchArgs& a, int npairs, hipStream_t stream)
{
    // one wave per image row (atomic corrections: per row and direction), four per workgroup
    if (a.atom)
        hipLaunchKernelGGL((k_ew_patch<VL, NP, CT, true>), dim3((2 * a.H + 3) / 4, npairs), dim3(256), 0, stream, a);
    else
        hipLaunchKernelGGL((k_ew_patch<VL, NP, CT, false>), dim3((a.H + 3) / 4, npairs), dim3(256), 0, stream, a);
    return hipGetLastError();
}

template <typename CT>
hipError_t patch_d(int D, const EwPatchArgs& a, int npairs, hipStream_t stream)
{
    switch (D) {  // 16-lane lines where D % 32 == 0, else 8-lane lines (every D % 16 == 0)
#define P16(d) \
    case d: return run_patch<16, d / 32, CT>(a, npairs, stream);
#define P8(d) \
    case d: return run_patch<8, d / 16, CT>(a, npairs, stream);
        P8(16) P16(32) P8(48) P16(64) P8(80) P16(96) P8(112) P16(128)
        P8(144) P16(160) P8(176) P16(192) P8(208) P16(224) P8(240) P16(256)
#undef P16
#undef P8
    default: return hipErrorInvalidValue;
    }
}

template <int VL, int NP, typename CT>
hipError_t run_band_patch(BandPatchArgs a, int npairs, hipStream_t stream)
{
    constexpr int LPW = 64 / VL;
    a.nbx = (3 * a.W1 + 4 * LPW - 1) / (4 * LPW);  // 4 waves of LPW chains per workgroup
    if (a.nband < 2) return hipSuccess;
    hipLaunchKernelGGL((k_band_patch<VL, NP, CT>), dim3(a.nbx, a.nband - 1, npairs), dim3(256), 0, stream, a);
    return hipGetLastError();
}

template <typename CT>
hipError_t band_patch_d(int D, const BandPatchArgs& a, int npairs, hipStream_t stream)
{
    switch (D) {  // the lines of k_ew_patch: 16 lanes where D % 32 == 0, else 8
#define P16(d) \
    case d: return run_band_patch<16, d / 32, CT>(a, npairs, stream);
#define P8(d) \
    case d: return run_band_patch<8, d / 16, CT>(a, npairs, stream);
        P8(16) P16(32) P8(48) P16(64) P8(80) P16(96) P8(112) P16(128)
        P8(144) P16(160) P8(176) P16(192) P8(208) P16(224) P8(240) P16(256)
#undef P16
#undef P8
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t band_patch_launch(int D, int ct_bytes, const BandPatchArgs& a, int npairs, hipStream_t stream)
{
    return ct_bytes == 1 ? band_patch_d<uint8_t>(D, a, npairs, stream) : band_patch_d<uint16_t>(D, a, npairs, stream);
}

hipError_t ew_patch_launch(int D, int ct_bytes, const EwPatchArgs& a, int npairs, hipStream_t stream)
{
    if (a.nwg > patch_max_strips(D)) return hipErrorInvalidValue;
    return ct_bytes == 1 ? patch_d<uint8_t>(D, a, npairs, stream) : patch_d<uint16_t>(D, a, npairs, stream);
}

hipError_t ew_launch(int D, int ct_bytes, int vl, EwArgs a, int npairs, hipStream_t stream)
{
    return ct_bytes == 1 ? ew_d<uint8_t>(D, vl, a, npairs, stream) : ew_d<uint16_t>(D, vl, a, npairs, stream);
}

}  // namespace smk
