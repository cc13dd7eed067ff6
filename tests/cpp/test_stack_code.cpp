// Host check of the 4-B traversal stack entry (spt_kernels.h stack_code / stack_t0_lower_bits,
// SPT_BVH_STACK_ENTRY 4): for every code width tb = 1..28 and entry distances t0 >= kTNear (every
// 61st float bit pattern from kTNear's up to +inf), the decoded bound is a float <= t0 (the pop's cull
// `bound > best_t` then implies t0 > best_t: exact traversal), the ref above the code survives, and
// for tb >= 8 the bound is within 2^-(tb - 5) of t0 wherever t0 < 2^22 (the culling stays useful).
#include <cstdio>
#include <cstring>

#include "spt_kernels.h"

static float as_float(uint32_t b) {
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}

int main() {
    using namespace spt;
    uint32_t tnear_bits;
    const float tnear = 0.001f;
    std::memcpy(&tnear_bits, &tnear, 4);
    unsigned long long bad = 0, loose = 0, checked = 0;
    for (uint32_t tb = 1; tb <= 28; ++tb) {
        const StackCode c = stack_code_params(tb);
        const uint32_t ref_max = tb == 28 ? 15u : ((1u << (32 - tb)) - 1u);
        for (uint64_t b = tnear_bits; b <= 0x7f800000u; b += 61u) {
            const uint32_t bits = (uint32_t)b;
            const uint32_t e = (ref_max << tb) | stack_code(bits, c);
            const uint32_t lo = stack_t0_lower_bits(e, c);
            ++checked;
            if ((e >> tb) != ref_max || lo > bits || !(as_float(lo) <= as_float(bits))) ++bad;
            if (tb >= 8 && as_float(bits) < 4194304.0f &&
                (double)as_float(lo) < (double)as_float(bits) * (1.0 - 1.0 / (double)(1u << (tb - 5))))
                ++loose;
        }
    }
    std::printf("stack codes: %llu checked, %llu not a lower bound or ref lost, %llu looser than 2^-(tb-5)\n", checked,
                bad, loose);
    const bool ok = bad == 0 && loose == 0 && bvh_stack_t0_bits(0u) == 28u && bvh_stack_t0_bits((1u << 24) - 1u) == 8u &&
                    bvh_stack_t0_bits(0x7fffffffu) == 1u;
    std::printf(ok ? "PASS\n" : "FAIL\n");
    return ok ? 0 : 1;
}
