// okm_testing.cpp — the test hooks of include/orion_kmer_testing.h: one
// process-wide atomic word per knob, -1 = unset (the product default).
#include <atomic>

#include "okm_internal.h"
#include "orion_kmer_testing.h"

namespace okm {
namespace {
std::atomic<int64_t> g_knobs[OKM_TEST_KNOBS] = {};
struct Init {
    Init() {
        for (auto &k : g_knobs) k.store(-1);
    }
} g_init;
}  // namespace

int64_t test_knob(int knob) {
    return knob >= 0 && knob < OKM_TEST_KNOBS ? g_knobs[knob].load(std::memory_order_relaxed) : -1;
}
}  // namespace okm

extern "C" {
void okm_test_set(okm_test_knob knob, int64_t value) {
    if ((int)knob >= 0 && (int)knob < OKM_TEST_KNOBS) okm::g_knobs[knob].store(value < 0 ? -1 : value);
}
int64_t okm_test_get(okm_test_knob knob) { return okm::test_knob((int)knob); }
}
