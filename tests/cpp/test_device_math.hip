// Exhaustive GPU check of spt_device.h's range-restricted helpers against the general routines:
// sqrt_unit(x) == sqrtf(x) for x = 0 and every float in [2^-32, 1] (the random_float range).
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

int main() {
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
    std::printf(h == 0 ? "PASS\n" : "FAIL\n");
    (void)hipFree(bad);
    return h == 0 ? 0 : 1;
}
