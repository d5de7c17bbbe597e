// Host check of wq::quantize_pack (worldql_server_amd/csrc/wq_device.hpp) against the two functions
// it fuses, coord_clamp_dev and pack_key: keys, regularity, packed key and ext must agree for
// every input. Built and run by tests/test_quantize_pack.py (hipcc, host code only).
#include "wq_device.hpp"
#include <cstdio>
#include <cstring>
#include <cmath>
#include <random>
using namespace wq;
static uint64_t bad = 0, n = 0, nfast = 0;
static void one(uint32_t w, double x, double y, double z, int64_t si) {
    const double sf = (double)si;
    int64_t k0[3] = {coord_clamp_dev(x, sf, si), coord_clamp_dev(y, sf, si), coord_clamp_dev(z, sf, si)};
    uint64_t p0 = 7; uint32_t e0 = 9;
    bool r0 = pack_key(w, k0[0], k0[1], k0[2], sf, &p0, &e0);
    const double c[3] = {x, y, z};
    int64_t k1[3]; uint64_t p1 = 7; uint32_t e1 = 9;
    bool r1 = quantize_pack(w, c, sf, si, k1, &p1, &e1);
    ++n;
    if (r0 != r1 || memcmp(k0, k1, sizeof k0) || p0 != p1 || e0 != e1) {
        if (bad++ < 10) printf("MISMATCH w=%u c=(%.17g,%.17g,%.17g) si=%lld r %d/%d k %lld/%lld %lld/%lld %lld/%lld\n", w, x, y, z,
                               (long long)si, r0, r1, (long long)k0[0], (long long)k1[0], (long long)k0[1], (long long)k1[1], (long long)k0[2], (long long)k1[2]);
    }
}
int main(int argc, char** argv) {
    std::mt19937_64 g(12345);
    const int64_t sizes[] = {1, 2, 3, 7, 16, 17, 100, 1000, 4096, 65535, (1 << 20) + 1, (1 << 29) - 1, 1 << 29, 1ll << 33, (1ll << 40) + 3};
    const double specials[] = {0.0, -0.0, 1e-310, -1e-310, 5e-324, -5e-324, NAN, -NAN, INFINITY, -INFINITY, 1e300, -1e300,
                               9.2233720368547758e18, -9.2233720368547758e18, 134217728.0, -134217728.0, 134217712.0,
                               -134217712.0, 134217727.5, 8388608.0, -8388608.0, 16.0, -16.0, 15.999999999999998, 1.0, -1.0};
    const int NS = sizeof specials / sizeof specials[0];
    for (int64_t si : sizes) {
        const double s = (double)si;
        // grids around the axis limits: multiples, +-1 ulp, +-half
        for (double base : {0.0, 1.0, 8388606.0, 8388607.0, 8388608.0, 8388609.0, 8388610.0, 8388611.0, 1099511627776.0 / s}) {
            for (int sgn : {1, -1})
                for (int dk = -3; dk <= 3; ++dk) {
                    const double m = (base + dk) * s * sgn;
                    for (double v : {m, std::nextafter(m, INFINITY), std::nextafter(m, -INFINITY), m + s / 2, m - s / 2})
                        for (int j = 0; j < NS; ++j) one(3, v, specials[j], m, si), one(16777214u, v, -v, specials[j], si);
                }
        }
        for (int j = 0; j < NS; ++j)
            for (int l = 0; l < NS; ++l) one(1, specials[j], specials[l], specials[(j + l) % NS], si);
        std::uniform_real_distribution<double> u(-1.0, 1.0);
        for (int it = 0; it < 200000; ++it) {
            const double scale = std::ldexp(1.0, (int)(g() % 80) - 10);
            double c[3];
            for (double& v : c) {
                const uint64_t r = g() % 4;
                v = r == 0 ? std::round(u(g) * scale / s) * s : r == 1 ? u(g) * scale : r == 2 ? std::round(u(g) * 1e7) * s : u(g) * 9e6 * s;
            }
            const uint32_t w = (g() % 8 == 0) ? (uint32_t)(16777210u + g() % 8) : (uint32_t)(g() % 1000);
            one(w, c[0], c[1], c[2], si);
        }
    }
    // random bit patterns
    for (int it = 0; it < 2000000; ++it) {
        double c[3];
        for (double& v : c) { uint64_t b = g(); memcpy(&v, &b, 8); }
        one((uint32_t)(g() % 100), c[0], c[1], c[2], sizes[g() % 15]);
    }
    printf("checked %llu, mismatches %llu\n", (unsigned long long)n, (unsigned long long)bad);
    return bad != 0;
}
