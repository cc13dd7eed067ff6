// spt_device.h — device-side arithmetic of the integrator (gfx950).
//
// Every function restates one piece of render::CPUPathTracer
// (libs/render/src/engines/pathtracer/backends/cpu/CPUPathTracer.cpp) with the exact float
// evaluation order of the reference's Linux build (SURVEY.md §8a "numeric semantics"):
//   - no FMA contraction (the whole library is compiled with -ffp-contract=off),
//   - correctly rounded fp32 '/' and sqrtf (HIP default),
//   - glm formulas: dot = (x*x' + y*y') + z*z', cross = (a.y*b.z - b.y*a.z, ...),
//     normalize(v) = v * (1.0f / sqrtf(dot(v, v))), mix(x, y, a) = x*(1-a) + y*a,
//   - get_random_bounche's unqualified sqrt/cos/sin on float arguments bind to the C double
//     functions under libstdc++, so cos/sin and the products with sinTheta run in fp64.
// oracle/cpu_ref.c restates the same functions on the CPU; tests compare the two bit for bit.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#else  // hiprtc (spt_jit.cpp): no system headers; its runtime header defines the fixed-width types
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::uint64_t uint64_t;
typedef __hip_internal::int32_t int32_t;
#endif

namespace spt {

constexpr float kInf = __builtin_inff();
constexpr uint32_t kMiss = 0xffffffffu;        // RTC_INVALID_GEOMETRY_ID analogue
constexpr float kTNear = 0.001f;               // rayhit.ray.tnear, CPUPathTracer.cpp:221
constexpr float kOriginEps = 1e-4f;            // EPSILON, CPUPathTracer.cpp:277
constexpr float kPiF = 3.14159265358979323846f;  // glm::pi<float>()
constexpr uint32_t kSeedPrime = 982451653u;    // CPUPathTracer.cpp:194
constexpr uint32_t kFlagAbsFloat = 1u;         // SPT_FLAG_ABS_FLOAT

struct F3 {
    float x, y, z;
};

__device__ __forceinline__ float dot3(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ F3 cross3(F3 a, F3 b) {
    return F3{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
__device__ __forceinline__ float sqrt_unit(float x);

// 1.0f / sqrtf(x) as glm::normalize computes it (two correctly rounded operations), bit for bit.
// For x in [2^-96, 2^96) it runs hipcc's own instruction sequences minus the steps that are the
// identity there: sqrtf without its rescaling of x < 2^-96 and its 0/inf pass-through (sqrt_unit),
// and the division 1.0f / s (s in [2^-48, 2^48]) without v_div_scale (no scaling at these
// exponents), the multiply by 1.0 and v_div_fixup (finite, normal quotient). Other x take the
// general routines. 11 VALU operations fewer per call; tests/cpp/test_device_math.hip checks all
// 2^32 inputs against 1.0f / sqrtf(x). SPT_EXPERIMENT_FAST_NORM (measurement-only builds, NOT
// reference numerics: SPT_EXPERIMENT_BUILD must be set too) prices the whole thing with the hardware rsq.
#if (defined(SPT_EXPERIMENT_FAST_NORM) || defined(SPT_EXPERIMENT_FP32_TRIG)) && !defined(SPT_EXPERIMENT_BUILD)
#error "SPT_EXPERIMENT_* flags break parity with the reference: measurement builds only (scripts/build_variant.sh sets SPT_EXPERIMENT_BUILD)"
#endif
__device__ __forceinline__ float inv_sqrt_ref(float x) {
#ifdef SPT_EXPERIMENT_FAST_NORM
    return __builtin_amdgcn_rsqf(x);
#else
    if (__float_as_uint(x) - 0x0f800000u < 0x60000000u - 0x0f800000u) {  // 2^-96 <= x < 2^96
        const float s = sqrt_unit(x);
        const float y0 = __builtin_amdgcn_rcpf(s);
        const float e = __builtin_fmaf(-s, y0, 1.0f);
        const float y1 = __builtin_fmaf(e, y0, y0);  // q0 = 1.0f * y1
        const float r0 = __builtin_fmaf(-s, y1, 1.0f);
        const float q1 = __builtin_fmaf(r0, y1, y1);
        const float r1 = __builtin_fmaf(-s, q1, 1.0f);
        return __builtin_fmaf(r1, y1, q1);  // v_div_fmas without scaling
    }
    return 1.0f / sqrtf(x);
#endif
}
__device__ __forceinline__ F3 normalize3(F3 v) {
    const float inv = inv_sqrt_ref(dot3(v, v));
    return F3{v.x * inv, v.y * inv, v.z * inv};
}

// get_rng_state, CPUPathTracer.cpp:192-195 (frame = m_frameCount + 1 at the call site :61).
__device__ __forceinline__ uint32_t rng_seed(uint32_t x, uint32_t y, uint32_t width, uint32_t frame1) {
    return x + y * width + frame1 * kSeedPrime;
}

// random_float, CPUPathTracer.cpp:294-301. 4294967295.0f rounds to 2^32, so this is exact.
__device__ __forceinline__ float random_float(uint32_t& state) {
    state = state * 747796405u + 2891336453u;
    uint32_t r = ((state >> ((state >> 28) + 4u)) ^ state) * 277803737u;
    r = (r >> 22) ^ r;
    return (float)r / 4294967295.0f;
}

// ---- unscaled correctly rounded division (the flat closest-hit loop's fast path) -------------
// hipcc's fp32 n / s is v_div_scale (x2), the reciprocal refinement, the residual steps,
// v_div_fmas and v_div_fixup. For |s| in [2^-40, 2^20] and |n| in [2^-100, 2^50] the scale steps
// are the identity (reciprocal and quotient normal, exponent difference < 96, numerator exponent
// > 23), v_div_fmas is a plain fma and v_div_fixup passes the finite quotient through, so the
// sequence below returns the same bits. For |n| < 2^-100 (zero included) it returns some
// |q| < 2^-59, and so is the exact quotient: every caller rejects both (t < kTNear).
// tests/cpp/test_device_math.hip compares it with n / s on the GPU.
struct RcpRef {
    float s, y;  // the divisor and its refined reciprocal
};
__device__ __forceinline__ RcpRef rcp_ref(float s) {
    const float y0 = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, y0, 1.0f);
    return RcpRef{s, __builtin_fmaf(e, y0, y0)};
}
__device__ __forceinline__ float div_ref(float n, RcpRef r) {
    const float q0 = n * r.y;
    const float r0 = __builtin_fmaf(-r.s, q0, n);
    const float q1 = __builtin_fmaf(r0, r.y, q0);
    const float r1 = __builtin_fmaf(-r.s, q1, n);
    return __builtin_fmaf(r1, r.y, q1);
}

// 1.0f / s, correctly rounded: for 2^-40 <= |s| < 2^20 one refined reciprocal and div_ref (the
// numerator 1 is in its range), else hipcc's division. Same bits (tests/cpp/test_device_math.hip checks
// every float); 5 VALU and no v_div_scale / v_div_fixup where the range holds. The BVH triangle test's
// 1 / det and the traversal's inverse direction (trav_init).
__device__ __forceinline__ float recip_ref(float s) {
    const uint32_t a = __float_as_uint(s) & 0x7fffffffu;
    if (a - 0x2b800000u < 0x49800000u - 0x2b800000u) return div_ref(1.0f, rcp_ref(s));  // [2^-40, 2^20)
    return 1.0f / s;
}

// Primary ray, CPUPathTracer.cpp:53-73: pinhole at the origin looking down +z. The fast path's gate
// q = uv_x^2 + uv_y^2 + 1 < 2^40 keeps `len` in [1, 2^20], inside div_ref's divisor range [2^-40, 2^20],
// and the numerators are 0, +-1 or in [2^-100, 2^50] in magnitude (checked per lane): then sqrt_unit
// and one refined reciprocal with div_ref give the correctly rounded sqrtf and quotients. Every real
// image passes (|uv_y| <= 1, |uv_x| <= the aspect ratio < 2^19); a lane outside takes the general
// routines. Same bits. Every k_frame and
// wavefront path pays it once (k_paths once per pixel and launch).
__device__ __forceinline__ F3 primary_dir(uint32_t x, uint32_t y, float inv_w, float inv_h, float aspect) {
    const float u = (float)x * inv_w;
    const float v = 1.0f - (float)y * inv_h;
    const float uv_x = (u * 2.0f - 1.0f) * aspect;
    const float uv_y = v * 2.0f - 1.0f;
    const float q = uv_x * uv_x + uv_y * uv_y + 1.0f;
    auto in_range = [](float c) {  // c == +-0, or 2^-100 <= |c| <= 2^50 (on the magnitude's bits)
        const uint32_t a = __float_as_uint(c) & 0x7fffffffu;
        return (a == 0u) | (a - 0x0d800000u <= 0x58800000u - 0x0d800000u);
    };
    if (((q < 0x1p40f) & in_range(uv_x) & in_range(uv_y))) {
        const RcpRef r = rcp_ref(sqrt_unit(q));
        return F3{div_ref(uv_x, r), div_ref(uv_y, r), div_ref(1.0f, r)};
    }
    const float len = sqrtf(q);
    return F3{uv_x / len, uv_y / len, 1.0f / len};
}

// sample_sky, CPUPathTracer.cpp:286-292: glm::mix(horizon, zenith, t).
__device__ __forceinline__ F3 sample_sky(float dir_y, float4 horizon, float4 zenith) {
    const float t = 0.5f * (dir_y + 1.0f);
    const float s = 1.0f - t;
    return F3{horizon.x * s + zenith.x * t, horizon.y * s + zenith.y * t, horizon.z * s + zenith.z * t};
}

// Environment map on the miss path (superset; the reference's SkyBox,
// Scene.h:268-278, has no lookup): an octahedral map of w x h RGBA texels, nearest texel. The
// direction is projected onto the octahedron |x|+|y|+|z| = 1 (y up); the lower hemisphere is folded
// over the diagonals. Only +, -, *, / and fabs: the oracle restates it bit for bit.
__host__ __device__ inline uint32_t octa_texel(float dx, float dy, float dz, uint32_t w, uint32_t h) {
    const float s = (fabsf(dx) + fabsf(dy)) + fabsf(dz);
    float px = dx / s, pz = dz / s;
    if (dy < 0.0f) {
        const float fx = (1.0f - fabsf(pz)) * (px >= 0.0f ? 1.0f : -1.0f);
        const float fz = (1.0f - fabsf(px)) * (pz >= 0.0f ? 1.0f : -1.0f);
        px = fx;
        pz = fz;
    }
    // fmaxf/fminf drop a NaN (zero direction): it maps to texel 0
    const float u = fminf(fmaxf(px * 0.5f + 0.5f, 0.0f), 1.0f);
    const float v = fminf(fmaxf(pz * 0.5f + 0.5f, 0.0f), 1.0f);
    uint32_t ix = (uint32_t)(u * (float)w), iy = (uint32_t)(v * (float)h);
    ix = ix < w ? ix : w - 1u;
    iy = iy < h ? iy : h - 1u;
    return iy * w + ix;
}

// get_random_bounche, CPUPathTracer.cpp:303-326 (cosine-weighted hemisphere around n), split in
// two: the tangent t of the frame (a function of n only, so it can be computed once per primary
// hit and reused for every frame of a pixel) and the random direction around (n, t, n x t).
// (float)sqrt((double)u) == sqrtf(u) exactly for float u (double has > 2*24+2 bits), so the two
// square roots stay fp32; cos/sin and the products with sinTheta are fp64 as in the reference.
__device__ __forceinline__ F3 bounce_tangent(F3 n, uint32_t flags) {
    // `abs(normal.z) < 0.999f`: ::abs(int) under libstdc++ (truncate, then |i| < 0.999 <=> i == 0)
    const bool not_pole = (flags & kFlagAbsFloat) ? (fabsf(n.z) < 0.999f) : ((int)n.z == 0);
    const F3 up = not_pole ? F3{0.0f, 0.0f, 1.0f} : F3{1.0f, 0.0f, 0.0f};
    return normalize3(cross3(up, n));
}

// sin and cos of phi in [0, 2*pi] in fp64 (the reference calls the C double cos/sin here, see
// bounce_dir_frame). Cody-Waite reduction by pi/2 (k <= 4: k * kPio2Hi and phi - k * kPio2Hi are
// exact) and Taylor polynomials to r^15 / r^16 on |r| <= pi/4: truncation < 2^-53, so the result
// is within an ulp or so of the correctly rounded value, like the library routines. What the
// integrator consumes is (float)((double)sinTheta * cos), which agreed with glibc's cos/sin for
// all of 1e8 sampled (u1, u2) pairs. About a third of the fp64 work of the
// general-argument sincos (no large-argument path).
// The coefficients of sincos_2pi's polynomials (sin: [0..6], cos: [7..14]), highest power first.
#define SPT_SINCOS_COEFS                                                                              \
    -1.0 / 1307674368000.0, 1.0 / 6227020800.0, -1.0 / 39916800.0, 1.0 / 362880.0, -1.0 / 5040.0,     \
        1.0 / 120.0, -1.0 / 6.0, 1.0 / 20922789888000.0, -1.0 / 87178291200.0, 1.0 / 479001600.0,     \
        -1.0 / 3628800.0, 1.0 / 40320.0, -1.0 / 720.0, 1.0 / 24.0, -0.5
#ifdef __HIP_DEVICE_COMPILE__
// kSmemCoef: a kernel can only take a double constant as an operand from a register (gfx950 VOP3
// has no literals), so inline each of the 15 coefficients costs a v_mov_b64 per call. Read from this
// table through a pointer the compiler cannot hoist, they arrive by scalar loads (SMEM, no VALU) in
// SGPRs, which the FMAs take as operands directly, and free VGPRs: the BVH k_paths spills less
// (C4 +6 %). The flat k_paths uses the table too since round 3 (its step loop had come to spill the
// hoisted coefficient pairs: +3.9 % on C2). Same values, same FMAs: same bits.
static __constant__ double kSinCosCoef[16] = {SPT_SINCOS_COEFS, 0.0};
#endif
// fma(a, b, c) with c in an SGPR pair, as ONE VOP3 v_fma_f64. Left to itself the compiler picks the
// two-address v_fmac_f64 (dst += a * b) for every Horner step of sincos_2pi, and then has to copy the
// scalar-loaded coefficient into the destination VGPR pair first: two v_mov_b32 per step, 26 per
// sample. The same fused operation, so the same bits.
__device__ __forceinline__ double fma_sc(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
#else
    return __builtin_fma(a, b, c);
#endif
}

template <bool kSmemCoef = false>
__host__ __device__ inline void sincos_2pi(double phi, double& s, double& c) {
    constexpr double kPio2Hi = 1.57079632679489655800e+00;
    constexpr double kPio2Lo = 6.12323399573676603587e-17;
    constexpr double k2OverPi = 6.36619772367581382433e-01;
    constexpr double kInline[16] = {SPT_SINCOS_COEFS, 0.0};
#ifdef __HIP_DEVICE_COMPILE__
    const __attribute__((address_space(4))) double* cf = nullptr;
    if constexpr (kSmemCoef) {
        cf = (const __attribute__((address_space(4))) double*)kSinCosCoef;
        asm volatile("" : "+s"(cf));  // opaque: the loads stay next to their use (no SGPRs held across the loop)
    }
#define SPT_CF(i) (kSmemCoef ? cf[i] : kInline[i])
#else
#define SPT_CF(i) kInline[i]
#endif
    const double k = __builtin_rint(phi * k2OverPi);
    const double r = (phi - k * kPio2Hi) - k * kPio2Lo;
    const double w = r * r;
#if defined(__HIP_DEVICE_COMPILE__)
    // (the scalar-table coefficients as SGPR operands: fma_sc; the first step's C0 * w + C1 reads two
    // coefficients, and a VALU instruction takes one scalar operand, so it stays a plain fma)
#define SPT_HORNER(p, i) (kSmemCoef ? fma_sc(p, w, SPT_CF(i)) : __builtin_fma(p, w, SPT_CF(i)))
#else
#define SPT_HORNER(p, i) __builtin_fma(p, w, SPT_CF(i))
#endif
    double ps = SPT_CF(0);
    ps = __builtin_fma(ps, w, SPT_CF(1));
    ps = SPT_HORNER(ps, 2);
    ps = SPT_HORNER(ps, 3);
    ps = SPT_HORNER(ps, 4);
    ps = SPT_HORNER(ps, 5);
    ps = SPT_HORNER(ps, 6);
    const double sr = __builtin_fma(r * w, ps, r);
    double pc = SPT_CF(7);
    pc = __builtin_fma(pc, w, SPT_CF(8));
    pc = SPT_HORNER(pc, 9);
    pc = SPT_HORNER(pc, 10);
    pc = SPT_HORNER(pc, 11);
    pc = SPT_HORNER(pc, 12);
    pc = SPT_HORNER(pc, 13);
    pc = SPT_HORNER(pc, 14);
#undef SPT_HORNER
    const double cr = __builtin_fma(w, pc, 1.0);
    const int q = ((int)k) & 3;
    const double a = (q & 1) ? cr : sr;  // sin: sr, cr, -sr, -cr
    const double b = (q & 1) ? sr : cr;  // cos: cr, -sr, -cr, sr
    s = (q & 2) ? -a : a;
    c = ((q + 1) & 2) ? -b : b;
#undef SPT_CF
}

// Correctly rounded sqrtf for x = 0 and finite x >= 2^-96: hipcc's sqrtf sequence (hardware
// estimate, then the +-1 ulp residual corrections) without its rescaling of inputs below 2^-96 and
// its 0/inf pass-through, neither of which these inputs reach (sqrt(0): the estimate is 0 and both
// corrections keep it). Used for the random_float range [2^-32, 1] and by inv_sqrt_ref.
__device__ __forceinline__ float sqrt_unit(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    const float r = rm <= 0.0f ? sm : s;
    return rp > 0.0f ? sp : r;
}

template <bool kSmemCoef = false>
__device__ __forceinline__ F3 bounce_dir_frame(F3 n, F3 t, uint32_t& state) {
    const float u1 = random_float(state);
    const float u2 = random_float(state);
    const float cos_t = sqrt_unit(u1);
    const float sin_t = sqrt_unit(1.0f - u1);
    const float phi = 2.0f * kPiF * u2;
#ifdef SPT_EXPERIMENT_FP32_TRIG  // measurement-only build: prices the fp64 trig; NOT reference numerics
    float spf, cpf;
    sincosf(phi, &spf, &cpf);
    const float x = sin_t * cpf;
    const float y = sin_t * spf;
#else
    double sp, cp;
    sincos_2pi<kSmemCoef>((double)phi, sp, cp);
    const float x = (float)((double)sin_t * cp);
    const float y = (float)((double)sin_t * sp);
#endif
    const float z = cos_t;
    const F3 b = cross3(n, t);
    return F3{(x * t.x + y * b.x) + z * n.x, (x * t.y + y * b.y) + z * n.y, (x * t.z + y * b.z) + z * n.z};
}

template <bool kSmemCoef = false>
__device__ __forceinline__ F3 bounce_dir(F3 n, uint32_t& state, uint32_t flags) {
    return bounce_dir_frame<kSmemCoef>(n, bounce_tangent(n, flags), state);
}

// ---- primitive tests (replace rtcIntersect1, CPUPathTracer.cpp:214-227) ----------------------
// Each returns the closest root t >= tmin of the ray against the primitive, or +inf.

// Ray-sphere, sphere.md:170-188 (a = d.d, b = 2 L.d, c = L.L - r^2), near root first.
__device__ __forceinline__ float isect_sphere(float4 s, F3 o, F3 d, float tmin) {
    const float lx = o.x - s.x, ly = o.y - s.y, lz = o.z - s.z;
    const float a = (d.x * d.x + d.y * d.y) + d.z * d.z;
    const float b = 2.0f * ((lx * d.x + ly * d.y) + lz * d.z);
    const float c = ((lx * lx + ly * ly) + lz * lz) - s.w * s.w;
    const float disc = b * b - 4.0f * a * c;
    if (!(disc >= 0.0f)) return kInf;
    const float sq = sqrtf(disc);
    const float two_a = 2.0f * a;
    const float t1 = (-b - sq) / two_a;
    if (t1 >= tmin) return t1;
    const float t2 = (-b + sq) / two_a;
    if (t2 >= tmin) return t2;
    return kInf;
}

// Russian roulette's ray_throughput /= p (CPUPathTracer.cpp:268), p = max(T) > 0: the three correctly
// rounded divisions by p as ONE refined reciprocal and three div_ref when every operand is in div_ref's
// range — p in [2^-40, 2^20], each T component 0 or in [2^-100, 2^50] (components are >= 0; 0 / p gives
// +0 either way) — else hipcc's division (a lane with a tiny component). Same bits; 3 v_div_scale pairs,
// fmas and fixups fewer.
__device__ __forceinline__ F3 rr_divide(F3 T, float p) {
    // the range predicates combined without short-circuits (`|`, `&`): one branch instead of a cascade
    // of five exec-mask branches (SALU)
    auto in_range = [](float c) { return (c == 0.0f) | (c >= 0x1p-100f); };
    const bool p_ok = (p >= 0x1p-40f) & (p <= 0x1p20f);
    if ((p_ok & in_range(T.x) & in_range(T.y) & in_range(T.z))) {
        const RcpRef r = rcp_ref(p);
        return F3{div_ref(T.x, r), div_ref(T.y, r), div_ref(T.z, r)};
    }
    return F3{T.x / p, T.y / p, T.z / p};
}

// isect_sphere for |d| ~ 1 (a = d . d in [0.5, 2], two_a's reciprocal refined once per ray in
// r2a) in a scene that passed fast_division_ok (|center| + radius below 2^28): |-b -+ sq| < 2^31,
// so div_ref gives the same t (or both are below kTNear). sqrt_unit is exact for disc = 0 and disc >= 2^-96; a discriminant in (0, 2^-96)
// sets `redo` (the caller repeats the ray with isect_sphere).
// rr: s.w * s.w, precomputed by the host (scene.cpp prepare_prims, DevPrim b.x): the same product.
__device__ __forceinline__ float isect_sphere_fast(float4 s, float rr, F3 o, F3 d, float a, RcpRef r2a, float tmin,
                                                   bool& redo) {
    const float lx = o.x - s.x, ly = o.y - s.y, lz = o.z - s.z;
    const float b = 2.0f * ((lx * d.x + ly * d.y) + lz * d.z);
    const float c = ((lx * lx + ly * ly) + lz * lz) - rr;
    const float disc = b * b - 4.0f * a * c;
    // (the same predicates as `if (!(disc >= 2^-96)) { redo |= disc > 0; if (disc != 0) miss }`, without
    // the nested branch: lane masks, no exec-mask region)
    redo = redo | ((disc > 0.0f) & (disc < 0x1p-96f));
    if (!((disc >= 0x1p-96f) | (disc == 0.0f))) return kInf;
    const float sq = sqrt_unit(disc);
    const float t1 = div_ref(-b - sq, r2a);
    if (t1 >= tmin) return t1;
    const float t2 = div_ref(-b + sq, r2a);
    if (t2 >= tmin) return t2;
    return kInf;
}

__device__ __forceinline__ float comp(float4 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
__device__ __forceinline__ float comp(F3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

// Parallelogram whose normal lies along axis AX and whose edges lie in the plane (scene.cpp sets
// c.w = AX + 1): the plane is x[AX] = Q[AX], so t = (Q[AX] - o[AX]) / d[AX] (the build's definition
// of the axis-aligned quad; the oracle's isect_quad has the same form). The in-plane test is the
// general one with its exactly-zero terms dropped: each dropped term is a product with a +-0
// component of A or B, so every sum keeps its value except possibly the sign of a zero result,
// compared alike as x + 0.0f. d[AX] = +-0 gives t = +-inf or NaN, rejected as in the general form.
template <int AX>
__device__ __forceinline__ float isect_quad_axis(float4 pa, float4 pb, float4 pc, float4 pd, F3 o, F3 d, float tmin) {
    constexpr int U = AX == 0 ? 1 : 0;  // the two in-plane axes, in the general formula's order
    constexpr int V = AX == 2 ? 1 : 2;
    (void)pb;
    const float t = (comp(pa, AX) - comp(o, AX)) / comp(d, AX);
    if (!(t >= tmin) || t == kInf) return kInf;
    const float hu = (comp(o, U) + t * comp(d, U)) - comp(pa, U);
    const float hv = (comp(o, V) + t * comp(d, V)) - comp(pa, V);
    const float al = hu * comp(pc, U) + hv * comp(pc, V);
    const float be = hu * comp(pd, U) + hv * comp(pd, V);
    const uint32_t ua = __float_as_uint(al + 0.0f), ub = __float_as_uint(be + 0.0f);
    return max(ua, ub) <= 0x3f800000u ? t : kInf;
}

// isect_quad_axis with the unscaled division by d[AX] (its reciprocal refined once per ray in rAX),
// for |d[AX]| in [2^-20, 1.5] in a scene that passed fast_division_ok (coordinates below 2^28, so
// |o| < 2^28 + 1 and |Q[AX] - o[AX]| < 2^30): div_ref's quotient is the exact one (or both are below
// kTNear), and it is finite, so the t == inf test of the general form is dropped.
// The in-plane test runs for every lane (t is finite here): no exec-mask branch.
// kRect: the quad is known to be a rectangle (its group in a shape-specialized kernel, flat_rect_bits):
// the short form without the scalar check.
template <int AX, bool kRect = false>
__device__ __forceinline__ float isect_quad_axis_fast(float4 pa, float4 pc, float4 pd, F3 o, F3 d, RcpRef rAX,
                                                      float tmin) {
    constexpr int U = AX == 0 ? 1 : 0;
    constexpr int V = AX == 2 ? 1 : 2;
    const float t = div_ref(comp(pa, AX) - comp(o, AX), rAX);
    const float hu = (comp(o, U) + t * comp(d, U)) - comp(pa, U);
    const float hv = (comp(o, V) + t * comp(d, V)) - comp(pa, V);
    float al, be;
    // A rectangle whose edges also lie along the axes (a wall of a box: A = (a, 0), B = (0, b) in the
    // plane, every record word wave-uniform, so this is a scalar branch): the two products with a
    // zero component are dropped. hv * (+-0) is +-0 (hv is finite here), so the sum loses at most
    // the sign of a zero result, which x + 0.0f below erases: the same predicate.
    if (kRect || (((__float_as_uint(comp(pc, V)) | __float_as_uint(comp(pd, U))) & 0x7fffffffu) == 0u)) {
        al = hu * comp(pc, U);
        be = hv * comp(pd, V);
    } else {
        al = hu * comp(pc, U) + hv * comp(pc, V);
        be = hu * comp(pd, U) + hv * comp(pd, V);
    }
    const uint32_t ua = __float_as_uint(al + 0.0f), ub = __float_as_uint(be + 0.0f);
    return (t >= tmin && max(ua, ub) <= 0x3f800000u) ? t : kInf;
}

// Parallelogram: a = (Q, D = n.Q), b = (n, -), c = (A, type | axis << 2), d = (B, -) (see scene.h).
__device__ __forceinline__ float isect_quad(float4 pa, float4 pb, float4 pc, float4 pd, F3 o, F3 d,
                                            float tmin) {
    const uint32_t axis = __float_as_uint(pc.w) >> 2;
    if (axis == 1u) return isect_quad_axis<0>(pa, pb, pc, pd, o, d, tmin);
    if (axis == 2u) return isect_quad_axis<1>(pa, pb, pc, pd, o, d, tmin);
    if (axis == 3u) return isect_quad_axis<2>(pa, pb, pc, pd, o, d, tmin);
    const float denom = (pb.x * d.x + pb.y * d.y) + pb.z * d.z;
    const float t = (pa.w - ((pb.x * o.x + pb.y * o.y) + pb.z * o.z)) / denom;
    if (!(t >= tmin) || t == kInf) return kInf;
    const float hx = (o.x + t * d.x) - pa.x;
    const float hy = (o.y + t * d.y) - pa.y;
    const float hz = (o.z + t * d.z) - pa.z;
    const float al = (hx * pc.x + hy * pc.y) + hz * pc.z;
    const float be = (hx * pd.x + hy * pd.y) + hz * pd.z;
    // (al >= 0 && al <= 1 && be >= 0 && be <= 1) on the bit patterns: for x + 0.0f (-0 -> +0),
    // 0 <= x <= 1 <=> bits(x) <= bits(1.0f); negatives, NaN and inf all compare above.
    const uint32_t ua = __float_as_uint(al + 0.0f), ub = __float_as_uint(be + 0.0f);
    return max(ua, ub) <= 0x3f800000u ? t : kInf;
}

// Moller-Trumbore: a = (v0, -), b = (e1, -), c = (e2, -).
__device__ __forceinline__ float isect_tri(float4 pa, float4 pb, float4 pc, F3 o, F3 d, float tmin) {
    const float px = d.y * pc.z - pc.y * d.z;
    const float py = d.z * pc.x - pc.z * d.x;
    const float pz = d.x * pc.y - pc.x * d.y;
    const float det = (pb.x * px + pb.y * py) + pb.z * pz;
    const float inv = recip_ref(det);  // (1.0f / det, the same bits)
    const float tx = o.x - pa.x, ty = o.y - pa.y, tz = o.z - pa.z;
    const float u = ((tx * px + ty * py) + tz * pz) * inv;
    if (!(u >= 0.0f && u <= 1.0f)) return kInf;
    const float qx = ty * pb.z - pb.y * tz;
    const float qy = tz * pb.x - pb.z * tx;
    const float qz = tx * pb.y - pb.x * ty;
    const float v = ((d.x * qx + d.y * qy) + d.z * qz) * inv;
    if (!(v >= 0.0f && u + v <= 1.0f)) return kInf;
    const float t = ((pc.x * qx + pc.y * qy) + pc.z * qz) * inv;
    if (!(t >= tmin) || t == kInf) return kInf;
    return t;
}


// ---- next-event estimation (SPT_FLAG_NEE; superset; oracle ref_light_sample) ----
// Emitter records (scene.cpp build_emitters), 5 float4 each:
//   (base.xyz, 1: triangle | 0: parallelogram), (e1.xyz, area * n_emitters / pi), (e2.xyz, 0),
//   (unit normal.xyz, 0), (emission.rgb, 0);
//   a sphere: (center.xyz, 2), (r, 0, 0, area * n_emitters / pi), 0, 0, (emission.rgb, 0)
constexpr uint32_t kEmitRecs = 5;
constexpr float kShadowFar = 0.999f;  // the shadow ray stops short of the sampled point: t < 0.999 * dist

// Three draws (emitter, u, v) at the offset hit point x with shading normal n and throughput T (after
// the albedo, before Russian roulette): the shadow ray direction w and its tmax, and the estimate
// T * (Le * g) with g = cos_s * cos_l * area * n_emit / (pi * dist^2). False when the point is behind
// either surface (no shadow ray). Correctly rounded sqrtf and '/', no contraction: the oracle's bits.
// kSpheres = false: a table without sphere records (the sphere sample left out of the kernel).
template <bool kSpheres = true>
__device__ __forceinline__ bool light_sample(const float4* __restrict__ emit, uint32_t n_emit, F3 x, F3 n, F3 T,
                                             uint32_t& rng, F3& w, float& tmax, F3& add) {
    const float u0 = random_float(rng);
    const float u1 = random_float(rng);
    const float u2 = random_float(rng);
    uint32_t j = (uint32_t)(u0 * (float)n_emit);
    j = j < n_emit ? j : n_emit - 1u;
    const float4* e = emit + kEmitRecs * j;
    const float4 e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3], e4 = e[4];
    const uint32_t kind = __float_as_uint(e0.w);
    F3 p, nl;
    if (kSpheres && kind == 2u) {
        // a sphere, uniform over its area: the unit normal (sz, s cos phi, s sin phi) from z = 1 - 2 u1,
        // s = sqrt(1 - z^2), phi = 2 pi u2 with bounce_dir's fp64 sincos (glibc's cos / sin, the
        // oracle's), the point center + r * normal
        const float z = 1.0f - 2.0f * u1;
        const float s = sqrt_unit(1.0f - z * z);  // (0, or in [2^-24, 1]: correctly rounded)
        const float phi = 2.0f * kPiF * u2;
        double sp, cp;
        sincos_2pi<true>((double)phi, sp, cp);
        nl = F3{(float)((double)s * cp), (float)((double)s * sp), z};
        p = F3{e0.x + e1.x * nl.x, e0.y + e1.x * nl.y, e0.z + e1.x * nl.z};
    } else {
        float a = u1, b = u2;
        if (kind != 0u) {  // uniform on the triangle
            const float su = sqrtf(u1);
            a = su * (1.0f - u2);
            b = su * u2;
        }
        p = F3{(e0.x + a * e1.x) + b * e2.x, (e0.y + a * e1.y) + b * e2.y, (e0.z + a * e1.z) + b * e2.z};
        nl = F3{e3.x, e3.y, e3.z};
    }
    const F3 v{p.x - x.x, p.y - x.y, p.z - x.z};
    const float d2 = dot3(v, v);
    const float dist = sqrtf(d2);
    const float inv = 1.0f / dist;
    w = F3{v.x * inv, v.y * inv, v.z * inv};
    const float cs = dot3(n, w);
    // a sphere emits towards x from the side x sees: its outside when x is outside (the far side is
    // occluded by the sphere itself), its inside when x is inside (a dome around the scene);
    // parallelograms and triangles from both
    const float dl = dot3(nl, w);
    float cl = fabsf(dl);
    if (kSpheres && kind == 2u) {
        const F3 xc{x.x - e0.x, x.y - e0.y, x.z - e0.z};
        cl = dot3(xc, xc) < e1.x * e1.x ? dl : -dl;
    }
    if (!(cs > 0.0f) || !(cl > 0.0f)) return false;
    const float g = ((cs * cl) * e1.w) / d2;
    tmax = dist * kShadowFar;
    add = F3{T.x * (e4.x * g), T.y * (e4.y * g), T.z * (e4.z * g)};
    return true;
}

__device__ __forceinline__ uint32_t meta_type(float4 pd) { return __float_as_uint(pd.w) & 3u; }
__device__ __forceinline__ uint32_t meta_material(float4 pd) { return __float_as_uint(pd.w) >> 2; }

}  // namespace spt
