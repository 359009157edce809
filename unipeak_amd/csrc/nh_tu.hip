// unipeak_amd/csrc/nh_tu.hip -- one translation unit per window width NH
// (= ceil((bw + 1) / 64) words on each side, 1..8): compiled eight times with
// -DUPK_NH_TU=1..8, so the templated K1 / K3 / K4 kernels of the eight widths
// build in parallel.  Each unit exports the addresses of its kernels; api.hip
// launches them with hipLaunchKernel (kernels.hip holds the code).
#include "kernels.hip"
#include "stats1.hip"

#ifndef UPK_NH_TU
#error "compile with -DUPK_NH_TU=1..8"
#endif

#define UPK_CAT2(a, b) a##b
#define UPK_CAT(a, b) UPK_CAT2(a, b)

namespace upk {

constexpr int kNH = UPK_NH_TU;

template <int POOL, bool ND>
static const void *scan_ptr(bool prof, int mode) {
    if (prof) return (const void *)scan_kernel<kNH, POOL, ND, true, kModeFused>;
    if constexpr (kNH <= 4) {  // (wider kernels stream the fields in kModeScreen already)
        if (mode == kModeScreenF) {
            if constexpr (POOL == 0 && !ND) return (const void *)k1a_fields_kernel<kNH>;  // one track
            return (const void *)scan_kernel<kNH, POOL, ND, false, kModeScreenF>;
        }
    }
    return mode == kModeExact ? (const void *)scan_kernel<kNH, POOL, ND, false, kModeExact>
                              : (const void *)scan_kernel<kNH, POOL, ND, false, kModeScreen>;
}

// K1: the variants the library launches -- K1a (screen: over the chunk-sum
// plane or, without the index, the 2-bit fields), K1b (exact) and the
// profile kernel (PROF, fused) -- for every pool mode and strand layout
const void *UPK_CAT(scan_kernel_nh, UPK_NH_TU)(int pool, bool nd, bool prof, int mode) {
    if (nd) {
        if (pool == 0) return scan_ptr<0, true>(prof, mode);
        if (pool == 1) return scan_ptr<1, true>(prof, mode);
        return scan_ptr<2, true>(prof, mode);
    }
    if (pool == 0) return scan_ptr<0, false>(prof, mode);
    if (pool == 1) return scan_ptr<1, false>(prof, mode);
    return scan_ptr<2, false>(prof, mode);
}

// K3 (one: one pooled directional sample with K1b's peaks, stats1.hip --
// 1: a wave per region, 2: a lane per region)
const void *UPK_CAT(stats_kernel_nh, UPK_NH_TU)(int pool, bool nd, int one) {
    if (one == 2) return (const void *)stats1L_kernel<kNH>;
    if (one) return (const void *)stats1_kernel<kNH>;
    if (nd) {
        if (pool == 0) return (const void *)stats_kernel<kNH, 0, true>;
        if (pool == 1) return (const void *)stats_kernel<kNH, 1, true>;
        return (const void *)stats_kernel<kNH, 2, true>;
    }
    if (pool == 0) return (const void *)stats_kernel<kNH, 0, false>;
    if (pool == 1) return (const void *)stats_kernel<kNH, 1, false>;
    return (const void *)stats_kernel<kNH, 2, false>;
}

// K4
const void *UPK_CAT(shift_kernel_nh, UPK_NH_TU)(int pool) {
    if (pool == 0) return (const void *)shift_kernel<kNH, 0>;
    if (pool == 1) return (const void *)shift_kernel<kNH, 1>;
    return (const void *)shift_kernel<kNH, 2>;
}

}  // namespace upk
