// Limits of the device-built wide tree (test infrastructure, built with g++ by
// tests/test_wide_device_rules.py): every child block the build may write (childBase + 8 <= the
// slot cap) must survive the traversal kernels' 24-bit child-base field (ng = base << 8 | slots).
#include <cstdint>
#include <cstdio>

#include "pt_wide_dev.hpp"

int main() {
    const int64_t ns[] = {1, 2, 7, 8, 5000, 1043312, (int64_t)1 << 24, 14680064, 14680071, ((int64_t)1 << 26) - 1};
    for (int64_t n : ns) {
        const uint32_t cap = pt::wideDevSlotCap(n);
        if ((int64_t)cap > pt::kWideMaxSlots || (int64_t)cap > pt::wideDevNodeSlots(n)) {
            std::printf("FAIL cap %u for n %lld\n", cap, (long long)n);
            return 1;
        }
        const uint32_t lastBase = cap >= 8 ? cap - 8 : 0;   // the largest base the build accepts
        const uint32_t ng = (lastBase << 8) | 0xffu;
        if ((ng >> 8) != lastBase) {
            std::printf("FAIL base %u truncated for n %lld\n", lastBase, (long long)n);
            return 1;
        }
    }
    // below the limit the cap is the full slot budget (no scene that fits is refused)
    if (pt::wideDevSlotCap(1043312) != (uint32_t)pt::wideDevNodeSlots(1043312)) return 1;
    std::printf("ok\n");
    return 0;
}
