// Exhaustive GPU check of spt_device.h's range-restricted helpers against the general routines:
// sqrt_unit(x) == sqrtf(x) for x = 0 and every float in [2^-32, 1] (the random_float range), and
// inv_sqrt_ref(x) == 1.0f / sqrtf(x) for all 2^32 bit patterns (NaNs compared as NaN).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "spt_device.h"

__global__ void k_check_sqrt(uint32_t lo, uint32_t n, unsigned long long* bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = i == 0 ? 0.0f : __uint_as_float(lo + i - 1u);
    if (__float_as_uint(spt::sqrt_unit(x)) != __float_as_uint(sqrtf(x))) atomicAdd(bad, 1ull);
}

__global__ void k_check_inv_sqrt(uint32_t base, unsigned long long* bad) {
    const uint32_t i = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float(i);
    const float a = spt::inv_sqrt_ref(x), b = 1.0f / sqrtf(x);
    const bool same = __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
    if (!same) atomicAdd(bad, 1ull);
}

static int check_inv_sqrt() {
    unsigned long long* bad = nullptr;
    if (hipMalloc(&bad, sizeof(*bad)) != hipSuccess || hipMemset(bad, 0, sizeof(*bad)) != hipSuccess) return 2;
    const uint32_t per = 1u << 28;  // 16 launches of 2^28 inputs
    for (uint32_t k = 0; k < 16u; ++k) k_check_inv_sqrt<<<per / 256u, 256>>>(k * per, bad);
    unsigned long long h = 0;
    if (hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::printf("inv_sqrt_ref: 2^32 inputs, %llu mismatches vs 1.0f / sqrtf\n", h);
    (void)hipFree(bad);
    return h == 0 ? 0 : 1;
}

int main() {
    const int inv_rc = check_inv_sqrt();
    const float lo_f = 2.3283064365386963e-10f;  // 2^-32
    uint32_t lo, hi;
    std::memcpy(&lo, &lo_f, 4);
    const float one = 1.0f;
    std::memcpy(&hi, &one, 4);
    const uint32_t n = hi - lo + 2u;  // 0 plus [2^-32, 1]
    unsigned long long* bad = nullptr;
    if (hipMalloc(&bad, sizeof(*bad)) != hipSuccess || hipMemset(bad, 0, sizeof(*bad)) != hipSuccess) return 2;
    k_check_sqrt<<<(n + 255u) / 256u, 256>>>(lo, n, bad);
    unsigned long long h = 0;
    if (hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::printf("sqrt_unit: %u inputs, %llu mismatches vs sqrtf\n", n, h);
    (void)hipFree(bad);
    const bool ok = h == 0 && inv_rc == 0;
    std::printf(ok ? "PASS\n" : "FAIL\n");
    return ok ? 0 : 1;
}
