// Host build of spt_device.h's sincos_2pi (the device fp64 sin/cos of get_random_bounche's phi)
// checked against glibc's double cos/sin, which the reference calls (CPUPathTracer.cpp:313-316):
// what the integrator consumes is (float)((double)sinTheta * cos(phi)) and the same with sin, so
// those float products must agree for every sampled (u1, u2) pair drawn with the reference RNG.
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "spt_device.h"

int main(int argc, char** argv) {
    const unsigned long long n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 10000000ull;
    unsigned long long bad = 0, ulp_diff = 0;
    uint32_t st = 0x5eedu;
    const float kPi = 3.14159265358979323846f;
    auto rnd = [&st]() {  // random_float, CPUPathTracer.cpp:294-301
        st = st * 747796405u + 2891336453u;
        uint32_t r = ((st >> ((st >> 28) + 4u)) ^ st) * 277803737u;
        r = (r >> 22) ^ r;
        return (float)r / 4294967295.0f;
    };
    for (unsigned long long i = 0; i < n; ++i) {
        const float u1 = rnd(), u2 = rnd();
        const float sin_t = std::sqrt(1.0f - u1);
        const float phi = 2.0f * kPi * u2;
        double s, c;
        spt::sincos_2pi((double)phi, s, c);
        const double gs = std::sin((double)phi), gc = std::cos((double)phi);
        ulp_diff += (s != gs) + (c != gc);
        bad += ((float)((double)sin_t * c) != (float)((double)sin_t * gc)) +
               ((float)((double)sin_t * s) != (float)((double)sin_t * gs));
    }
    // the endpoints of the range: phi = 0 and phi = 2*pi_f (u2 == 1.0f is reachable)
    for (float phi : {0.0f, 2.0f * kPi, kPi, 0.5f * kPi, 1.5f * kPi}) {
        double s, c;
        spt::sincos_2pi((double)phi, s, c);
        bad += ((float)s != (float)std::sin((double)phi)) + ((float)c != (float)std::cos((double)phi));
    }
    std::printf("samples=%llu double-ulp-differences=%llu float-product-mismatches=%llu\n", n, ulp_diff, bad);
    std::printf(bad == 0 ? "PASS\n" : "FAIL\n");
    return bad == 0 ? 0 : 1;
}
