// hbm_alloc.hip — the library's class-balanced batch-buffer allocator
// (hbm_alloc.hpp has the design notes; chip_device_alloc uses it).
#include "chip_internal.hpp"
#include "hbm_alloc.hpp"

namespace chip {

hipError_t hbm_alloc(uint64_t bytes, void **out) {
    *out = nullptr;
    if (bytes < hbm::MIN_BYTES) return hipErrorInvalidValue;
    return hbm::Allocator::get().alloc(bytes, out);
}

bool hbm_free(void *p) { return hbm::Allocator::get().free(p); }

bool hbm_info(const void *p, uint32_t *classes_found, uint32_t *classes_used, double *seconds) {
    hbm::Allocation a;
    if (!hbm::Allocator::get().info(p, &a)) return false;
    *classes_found = a.classes_found;
    *classes_used = a.classes_used;
    *seconds = a.seconds;
    return true;
}

}  // namespace chip
