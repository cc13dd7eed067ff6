// GPU check of spt_device.h's range-restricted helpers against the general routines:
// sqrt_unit(x) == sqrtf(x) for x = 0 and every float in [2^-96, 2^96) (exhaustive), inv_sqrt_ref(x)
// == 1.0f / sqrtf(x) for all 2^32 bit patterns (NaNs compared as NaN), and div_ref(n, rcp_ref(s))
// == n / s for EVERY divisor |s| in [2^-40, 2^20) (both signs) against 4 hashed numerators each
// with |n| in [2^-100, 2^50) plus n = s * k (exact quotients), and |div_ref| < 2^-59 for numerators
// below 2^-100 (zero and denormals included): the ranges of the flat loop's fast path; and rr_divide
// == T / max(T) (Russian roulette) on 2^28 hashed throughputs.
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

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// divisor i of the enumeration: exponent -40 + (i >> 23), mantissa i & (2^23 - 1), hashed sign
__global__ void k_check_div(uint32_t base, uint32_t n, unsigned long long* bad, unsigned long long* tiny_bad) {
    const uint32_t i = base + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t sign = hash32(i) & 0x80000000u;
    const float s = __uint_as_float(sign | ((uint32_t)(127 - 40 + (int)(i >> 23)) << 23) | (i & 0x7fffffu));
    const spt::RcpRef r = spt::rcp_ref(s);
    for (uint32_t j = 0; j < 6u; ++j) {
        const uint32_t h = hash32(i * 8u + j + 0x9e3779b9u);
        float x;
        if (j < 4u) {  // |n| in [2^-100, 2^50)
            const uint32_t e = 127u - 100u + (hash32(h) % 150u);
            x = __uint_as_float((h & 0x80000000u) | (e << 23) | (h & 0x7fffffu));
        } else {  // exact quotients: n = s * k for small k
            x = s * (float)((h & 255u) + 1u) * ((j & 1u) ? -1.0f : 1.0f);
        }
        if (__float_as_uint(spt::div_ref(x, r)) != __float_as_uint(x / s)) atomicAdd(bad, 1ull);
        // below 2^-100 (zero and denormals): both quotients stay below 2^-59
        const float tx = __uint_as_float((h & 0x80000000u) | (h % (27u << 23)));
        if (!(fabsf(spt::div_ref(tx, r)) < 0x1p-59f) || !(fabsf(tx / s) < 0x1p-59f)) atomicAdd(tiny_bad, 1ull);
    }
}

// recip_ref == 1.0f / s for every float s (its fast range and the fallback alike; NaN for NaN)
__global__ void k_check_recip(uint32_t base, unsigned long long* bad) {
    const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float s = __uint_as_float(bits);
    const float a = spt::recip_ref(s), b = 1.0f / s;
    if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) atomicAdd(bad, 1ull);
}

static int check_recip() {
    unsigned long long* bad = nullptr;
    if (hipMalloc(&bad, sizeof(*bad)) != hipSuccess || hipMemset(bad, 0, sizeof(*bad)) != hipSuccess) return 2;
    const uint32_t per = 1u << 26;
    for (uint64_t b = 0; b < (1ull << 32); b += per) k_check_recip<<<per / 256u, 256>>>((uint32_t)b, bad);
    unsigned long long h = 0;
    if (hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::printf("recip_ref: all 2^32 inputs, %llu mismatches vs 1.0f / s\n", h);
    (void)hipFree(bad);
    return h == 0 ? 0 : 1;
}

static int check_div() {
    unsigned long long* bad = nullptr;
    if (hipMalloc(&bad, 2 * sizeof(*bad)) != hipSuccess || hipMemset(bad, 0, 2 * sizeof(*bad)) != hipSuccess) return 2;
    const uint32_t n = 60u << 23;  // every divisor magnitude in [2^-40, 2^20)
    const uint32_t per = 1u << 26;
    for (uint32_t b = 0; b < n; b += per) k_check_div<<<per / 256u, 256>>>(b, n, bad, bad + 1);
    unsigned long long h[2] = {0, 0};
    if (hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::printf("div_ref: %u divisors x 6 numerators, %llu mismatches vs n / s; tiny numerators: %llu out of range\n",
                n, h[0], h[1]);
    (void)hipFree(bad);
    return h[0] == 0 && h[1] == 0 ? 0 : 1;
}

// rr_divide (Russian roulette's T / max(T)) == the three plain divisions, for hashed throughputs whose
// components mix ordinary values, exact zeros, tiny values and denormals (the fallback lanes)
__global__ void k_check_rr(uint32_t base, unsigned long long* bad) {
    const uint32_t i = base + blockIdx.x * blockDim.x + threadIdx.x;
    float c[3];
    for (uint32_t k = 0; k < 3u; ++k) {
        const uint32_t h = hash32(i * 4u + k + 0x51ed27u);
        const uint32_t kind = h >> 29;  // 0: zero, 1: below 2^-100 (denormals included), else [2^-60, 1)
        if (kind == 0u) c[k] = 0.0f;
        else if (kind == 1u) c[k] = __uint_as_float(h % (27u << 23));
        else c[k] = __uint_as_float(((127u - 60u + (h % 60u)) << 23) | (hash32(h) & 0x7fffffu));
    }
    const float p = fmaxf(fmaxf(c[0], c[1]), c[2]);
    if (!(p > 0.0f)) return;
    const spt::F3 q = spt::rr_divide(spt::F3{c[0], c[1], c[2]}, p);
    if (__float_as_uint(q.x) != __float_as_uint(c[0] / p) || __float_as_uint(q.y) != __float_as_uint(c[1] / p) ||
        __float_as_uint(q.z) != __float_as_uint(c[2] / p))
        atomicAdd(bad, 1ull);
}

static int check_rr() {
    unsigned long long* bad = nullptr;
    if (hipMalloc(&bad, sizeof(*bad)) != hipSuccess || hipMemset(bad, 0, sizeof(*bad)) != hipSuccess) return 2;
    const uint32_t per = 1u << 26;
    for (uint32_t k = 0; k < 4u; ++k) k_check_rr<<<per / 256u, 256>>>(k * per, bad);
    unsigned long long h = 0;
    if (hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::printf("rr_divide: 2^28 throughputs, %llu mismatches vs T / max(T)\n", h);
    (void)hipFree(bad);
    return h == 0 ? 0 : 1;
}

// primary_dir (sqrt_unit + one refined reciprocal + div_ref where the ranges allow) == the reference's
// sqrtf and three divisions, for every pixel of images of the benchmark and App sizes and odd shapes
__global__ void k_check_primary(uint32_t w, uint32_t h, float inv_w, float inv_h, float aspect,
                                unsigned long long* bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= w * h) return;
    const uint32_t x = i % w, y = i / w;
    const spt::F3 d = spt::primary_dir(x, y, inv_w, inv_h, aspect);
    const float u = (float)x * inv_w;
    const float v = 1.0f - (float)y * inv_h;
    const float uv_x = (u * 2.0f - 1.0f) * aspect;
    const float uv_y = v * 2.0f - 1.0f;
    const float len = sqrtf(uv_x * uv_x + uv_y * uv_y + 1.0f);
    if (__float_as_uint(d.x) != __float_as_uint(uv_x / len) || __float_as_uint(d.y) != __float_as_uint(uv_y / len) ||
        __float_as_uint(d.z) != __float_as_uint(1.0f / len))
        atomicAdd(bad, 1ull);
}

static int check_primary() {
    unsigned long long* bad = nullptr;
    if (hipMalloc(&bad, sizeof(*bad)) != hipSuccess || hipMemset(bad, 0, sizeof(*bad)) != hipSuccess) return 2;
    const uint32_t sizes[][2] = {{1920, 1080}, {3840, 2160}, {512, 512}, {256, 256}, {1280, 720}, {7, 3},
                                 {1, 1}, {65535, 2}, {3, 4097}, {1000, 1},
                                 // extreme aspect ratios: q = uv_x^2 + uv_y^2 + 1 reaches 2^40 and beyond (the
                                 // fast path's gate; the lanes past it take the general routines)
                                 {1u << 20, 1}, {1u << 21, 1}, {1u << 22, 2}};
    unsigned long long px = 0;
    for (const auto& wh : sizes) {
        const uint32_t w = wh[0], h = wh[1];
        // the host's camera constants (spt_capi.hip: 1 / W, 1 / H, W / H in float)
        const float inv_w = 1.0f / (float)w, inv_h = 1.0f / (float)h, aspect = (float)w / (float)h;
        k_check_primary<<<(w * h + 255u) / 256u, 256>>>(w, h, inv_w, inv_h, aspect, bad);
        px += (unsigned long long)w * h;
    }
    unsigned long long hb = 0;
    if (hipMemcpy(&hb, bad, sizeof(hb), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::printf("primary_dir: %llu pixels of 13 image shapes, %llu mismatches vs sqrtf and '/'\n", px, hb);
    (void)hipFree(bad);
    return hb == 0 ? 0 : 1;
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
    const int div_rc = check_div() | check_recip() | check_rr() | check_primary();
    const float lo_f = 0x1p-96f;
    uint32_t lo, hi;
    std::memcpy(&lo, &lo_f, 4);
    const float top = 0x1p96f;
    std::memcpy(&hi, &top, 4);
    const uint32_t n = hi - lo + 1u;  // 0 plus [2^-96, 2^96)
    unsigned long long* bad = nullptr;
    if (hipMalloc(&bad, sizeof(*bad)) != hipSuccess || hipMemset(bad, 0, sizeof(*bad)) != hipSuccess) return 2;
    k_check_sqrt<<<(n + 255u) / 256u, 256>>>(lo, n, bad);
    unsigned long long h = 0;
    if (hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::printf("sqrt_unit: %u inputs, %llu mismatches vs sqrtf\n", n, h);
    (void)hipFree(bad);
    const bool ok = h == 0 && inv_rc == 0 && div_rc == 0;
    std::printf(ok ? "PASS\n" : "FAIL\n");
    return ok ? 0 : 1;
}
