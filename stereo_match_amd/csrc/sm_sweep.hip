// sm_sweep.hip — translation unit of the fused-sweep kernels (sm_sweep.hpp):
// instantiates k_sweep for every built (D, cost type, mode) and exposes a
// plain host interface to sm_api.hip, so the units compile in parallel.  Built
// once per (SWEEP_MODE, SWEEP_WIDE): the narrow strips (NCW 7, every D, plus
// k_lr_rows) and the wide strips (wide_ncw, where built).  The k_sweep2 ablation
// (sm_sweep2.hpp) is compiled only into the ablation build (SM_ABLATIONS=1).
#include <algorithm>

#include "sm_sweep.hpp"
#include "sm_sweep_host.hpp"
#ifndef SWEEP_WIDE
#define SWEEP_WIDE 0
#endif
#ifndef SM_ABLATIONS
#define SM_ABLATIONS 0
#endif
#if SM_ABLATIONS
#include "sm_sweep2.hpp"
#endif

namespace smk {

namespace {

// calls f.template run<VL, DPL, CT, SWEEP_MODE>() for the instance serving (D, ct_bytes); this unit
// is compiled once per mode (-DSWEEP_MODE=0/1/2) so the three compile in parallel
template <class F>
hipError_t with_sweep(int D, int ct_bytes, F& f)
{
    return ct_bytes == 1 ? with_d<uint8_t, SWEEP_MODE>(D, f) : with_d<uint16_t, SWEEP_MODE>(D, f);
}

}  // namespace

template <typename CT, int MODE, class F>
hipError_t with_d(int D, F& f)
{
    switch (D) {
        // 8-lane lines up to D = 64, 16-lane lines above (<= 16 disparities per lane)
#define SW8(d) \
    case d: return f.template run<8, d / 8, CT, MODE>();
#define SW16(d) \
    case d: return f.template run<16, d / 16, CT, MODE>();
        SW8(16) SW8(32) SW8(48) SW8(64) SW16(80) SW16(96) SW16(112)
#ifdef SWEEP_VL8_128
        SW8(128)
#else
        SW16(128)
#endif
        SW16(144) SW16(160) SW16(176) SW16(192) SW16(208) SW16(224) SW16(240)
#if SWEEP_WIDE == 1
        // the wide D = 256 instance: 32-lane lines for u8 costs (wide_ncw), none for u16
    case 256:
        if constexpr (sizeof(CT) == 1) return f.template run<32, 8, CT, MODE>();
        else return f.template run<16, 16, CT, MODE>();
#else
        SW16(256)
#endif
#undef SW8
#undef SW16
    default: return hipErrorInvalidValue;
    }
}

namespace {

// compute waves of this unit's instance for (D, CT); 0 = not built here
template <int D, typename CT>
constexpr int unit_ncw()
{
    if constexpr (SWEEP_WIDE == 2) return lat_built(D) ? kLatNcw : 0;
    return SWEEP_WIDE ? wide_ncw(D, (int)sizeof(CT)) : kNarrowNcw;
}

// MODES 3 and 4 (in-kernel E/W lines, then the WTA sweep over their partial) exist only for the
// packed row loops (even DPL), MODE 3 where its line waves and LDS ring fit the workgroup
template <int VL, int DPL, typename CT, int MODE>
constexpr bool unit_built()
{
    constexpr int NCW = unit_ncw<VL * DPL, CT>();
    if constexpr (NCW == 0) return false;
    else if constexpr (MODE < 3) return true;
    else if constexpr (DPL % 2 != 0 || SWEEP_U32) return false;
    else if constexpr (MODE == 3) return LineGeo<VL, DPL, NCW, 3, (int)sizeof(CT)>::BUILT;
    else return true;
}

struct InfoF {
    int device;
    SweepInfo* out;
    template <int VL, int DPL, typename CT, int MODE>
    hipError_t run()
    {
        constexpr int NCW = unit_ncw<VL * DPL, CT>();
        if constexpr (!unit_built<VL, DPL, CT, MODE>()) {
            return hipErrorInvalidValue;
        } else {
            using SG = SweepGeo<VL, DPL, NCW>;
            constexpr int THREADS = sweep_threads<VL, DPL, NCW, MODE>();
            auto kern = k_sweep<VL, DPL, CT, MODE, NCW>;
            static int per_cu = -1;  // per instance (one device type per process)
            if (per_cu < 0) {
                int nb = 0;
                if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, THREADS, 0) != hipSuccess) nb = 0;
                // a wide instance is used only if it runs without scratch and fits a CU
                hipFuncAttributes fa{};
                if (SWEEP_WIDE && (hipFuncGetAttributes(&fa, (const void*)kern) != hipSuccess || fa.localSizeBytes > 0))
                    nb = 0;
                per_cu = SWEEP_WIDE ? nb : std::max(nb, 1);
            }
            if (per_cu < 1) return hipErrorInvalidValue;
            out->cw = SG::CW;
            out->hb = SG::HB;
            out->ngr = SG::SNG;
            out->threads = THREADS;
            out->blocks_per_cu = per_cu;
            out->impl = SWEEP_WIDE == 2 ? 2 : SWEEP_WIDE ? 1 : 0;
            out->dpl = DPL;
            out->ncw = NCW;
            return hipSuccess;
        }
    }
};

struct LaunchF {
    const SweepArgs* a;
    dim3 grid;
    hipStream_t stream;
    template <int VL, int DPL, typename CT, int MODE>
    hipError_t run()
    {
        constexpr int NCW = unit_ncw<VL * DPL, CT>();
        if constexpr (!unit_built<VL, DPL, CT, MODE>()) {
            return hipErrorInvalidValue;
        } else {
            hipLaunchKernelGGL((k_sweep<VL, DPL, CT, MODE, NCW>), grid, dim3(sweep_threads<VL, DPL, NCW, MODE>()), 0,
                               stream, *a);
            return hipGetLastError();
        }
    }
};

#if !SWEEP_WIDE && SM_ABLATIONS && SWEEP_MODE <= 2

// column-per-lane sweeps (sm_sweep2.hpp, a measured ablation): built for u8 (census) costs
// at D = 128; variant = compute waves per workgroup: 3 (16 columns per wave), 6 (8 columns)
constexpr int sw2_pf(int mode) { return mode == 2 ? 2 : 4; }

template <int NW, int CPW, int NP, int MODE>
hipError_t sweep2_run(bool info, int device, SweepInfo* out, const SweepArgs* a, int npairs, hipStream_t stream)
{
    using SG = Sweep2Geo<NW, CPW, NP>;
    auto kern = k_sweep2<NW, CPW, NP, uint8_t, MODE, sw2_pf(MODE)>;
    if (info) {
        static int per_cu = -1;
        if (per_cu < 0) {
            int nb = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, SG::THREADS, 0) != hipSuccess) nb = 1;
            per_cu = nb;
        }
        out->cw = SG::CW;
        out->hb = SG::HB;
        out->ngr = SG::NGR;
        out->threads = SG::THREADS;
        out->blocks_per_cu = per_cu;
        out->impl = NW;
        out->dpl = 128 / 64;
        out->ncw = NW;
        return hipSuccess;
    }
    hipLaunchKernelGGL(kern, dim3(a->nwg, npairs), dim3(SG::THREADS), 0, stream, *a);
    return hipGetLastError();
}

template <int NW, int CPW>
hipError_t sweep2_d(int D, bool info, int device, SweepInfo* out, const SweepArgs* a, int npairs, hipStream_t stream)
{
    constexpr int PARTS = 64 / CPW;
    if (D != 128) return hipErrorInvalidValue;
    return sweep2_run<NW, CPW, 128 / (2 * PARTS), SWEEP_MODE>(info, device, out, a, npairs, stream);
}

hipError_t sweep2(int D, int ct_bytes, int variant, bool info, int device, SweepInfo* out, const SweepArgs* a,
                  int npairs, hipStream_t stream)
{
    if (ct_bytes != 1) return hipErrorInvalidValue;
    switch (variant) {  // 3: 16 columns per wave; 6: 8 columns per wave
    case 3: return sweep2_d<3, 16>(D, info, device, out, a, npairs, stream);
    case 6: return sweep2_d<6, 8>(D, info, device, out, a, npairs, stream);
    default: return hipErrorInvalidValue;
    }
}

#endif  // !SWEEP_WIDE && SM_ABLATIONS && SWEEP_MODE <= 2

}  // namespace

#define SW_CAT2(a, b) a##b
#define SW_CAT(a, b) SW_CAT2(a, b)

#if SWEEP_WIDE == 2
hipError_t SW_CAT(sweep_info_lat_m, SWEEP_MODE)(int D, int ct_bytes, int device, SweepInfo* out)
{
    InfoF f{device, out};
    return with_sweep(D, ct_bytes, f);
}

hipError_t SW_CAT(sweep_launch_lat_m, SWEEP_MODE)(int D, int ct_bytes, const SweepArgs& a, int npairs,
                                                  hipStream_t stream)
{
    LaunchF f{&a, a.xcd_per > 0 ? dim3(8 * a.xcd_per, 1) : dim3(a.nwg * (a.nband > 1 ? a.nband : 1), npairs), stream};
    return with_sweep(D, ct_bytes, f);
}
#elif SWEEP_WIDE
hipError_t SW_CAT(sweep_info_wide_m, SWEEP_MODE)(int D, int ct_bytes, int device, SweepInfo* out)
{
    InfoF f{device, out};
    return with_sweep(D, ct_bytes, f);
}

hipError_t SW_CAT(sweep_launch_wide_m, SWEEP_MODE)(int D, int ct_bytes, const SweepArgs& a, int npairs,
                                                   hipStream_t stream)
{
    LaunchF f{&a, a.xcd_per > 0 ? dim3(8 * a.xcd_per, 1) : dim3(a.nwg * (a.nband > 1 ? a.nband : 1), npairs), stream};
    return with_sweep(D, ct_bytes, f);
}
#else
hipError_t SW_CAT(sweep_info_m, SWEEP_MODE)(int D, int ct_bytes, int variant, int device, SweepInfo* out)
{
#if SM_ABLATIONS && SWEEP_MODE <= 2
    if (variant && sweep2(D, ct_bytes, variant, true, device, out, nullptr, 0, nullptr) == hipSuccess)
        return hipSuccess;
#else
    (void)variant;
#endif
    InfoF f{device, out};
    return with_sweep(D, ct_bytes, f);
}

hipError_t SW_CAT(sweep_launch_m, SWEEP_MODE)(int D, int ct_bytes, int variant, const SweepArgs& a, int npairs,
                                              hipStream_t stream)
{
#if SM_ABLATIONS && SWEEP_MODE <= 2
    if (variant) {
        const hipError_t e = sweep2(D, ct_bytes, variant, false, 0, nullptr, &a, npairs, stream);
        if (e != hipErrorInvalidValue) return e;
    }
#else
    (void)variant;
#endif
    LaunchF f{&a, a.xcd_per > 0 ? dim3(8 * a.xcd_per, 1) : dim3(a.nwg * (a.nband > 1 ? a.nband : 1), npairs), stream};
    return with_sweep(D, ct_bytes, f);
}
#endif

#if SWEEP_MODE == 0 && !SWEEP_WIDE
hipError_t lr_rows_launch(const uint32_t* rec, const uint32_t* nb, int16_t* out, int16_t* wta, int G, int H, int W,
                          int D, int minD, int minX1, int maxX1, int disp12, const uint32_t* guard, hipStream_t stream)
{
    hipLaunchKernelGGL(k_lr_rows, dim3(H, G), dim3(256), (size_t)W * 6 + 16, stream, rec, nb, out, wta, H, W, D, minD,
                       minX1, maxX1, disp12, guard);
    return hipGetLastError();
}
#endif

}  // namespace smk
