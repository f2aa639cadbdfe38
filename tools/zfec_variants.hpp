// zfec_variants.hpp — the tuner's K1 kernels: any configuration of the
// gf_apply body (carbonado_amd/csrc/zfec_device.hpp documents the
// arguments), each its own kernel, for tools/ only.  The library instantiates
// only the configurations it ships (zfec_kernels.hip: zfec_apply_kernel<K, NG>).
#pragma once

#include "../carbonado_amd/csrc/zfec_device.hpp"

namespace chip {
namespace zf {

template <int K, int NG, int U, int MAP, bool NT, int RO = 0, int WPE = 1, int SB = 0, bool PF = false,
          bool NTL = false, bool TR = false>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(WPE))) void gf_apply_kernel(ApplyArgs a) {
    gf_apply_body<K, NG, U, MAP, NT, RO, WPE, SB, PF, NTL, TR>(a);
}

}  // namespace zf
}  // namespace chip
