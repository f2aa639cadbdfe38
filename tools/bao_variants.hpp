// bao_variants.hpp — the tuner's K3 kernels: every configuration of the
// bao_chunk body (carbonado_amd/csrc/bao_device.hpp documents the arguments)
// as a kernel of its own, and the ChunkKernel mapping run_bao_t launches
// through, for tools/ only.  The library specialises ChunkKernel for the
// configurations it ships (bao_kernels.hip: bao_chunk_kernel_encode, ...).
#pragma once

#include "../carbonado_amd/csrc/bao_device.hpp"

namespace chip {
namespace bao {

template <int MODE, int CPL, bool NTS, int SP = 0, int SU = 1, int SE = 0, int XG = 0, bool DQ = false>
__global__ __launch_bounds__(K3_TPB) void bao_chunk_kernel(ChunkArgs a) {
    bao_chunk_body<MODE, CPL, NTS, SP, SU, SE, XG, DQ>(a);
}

template <int MODE, int CPL, bool NTS, int SP, int SU, int SE, int XG, bool DQ>
struct ChunkKernel {
    static constexpr void (*fn)(ChunkArgs) = bao_chunk_kernel<MODE, CPL, NTS, SP, SU, SE, XG, DQ>;
};

}  // namespace bao
}  // namespace chip
