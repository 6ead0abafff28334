// Host-side checks of the exactness claims behind the kernels' fast paths
// (compiled and run by tests/test_core_identities.py with hipcc (host code) -ffp-contract=off):
//   dsincos(x) == (dsin(x), dcos(x)) bit for bit;
//   wrapi's conditional add/subtract == the modulo form for every i;
//   upper_bound_guided == upper_bound on sorted CDF rows;
//   (float)((double)x * (1.0 / (double)d)) == x / d for normal-range quotients (tri_test's
//   fp32 replacement of the reference's fp64 island).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "device/mcpt_core.hpp"

using namespace mcpt;

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

int main() {
    std::mt19937_64 g(7);
    long bad = 0;
    // dsincos: random bit patterns in the reduction range, special values, edges
    std::vector<float> xs = {0.f, -0.f, 1e-30f, -1e-30f, 0.785398f, 1.570796f, 3.141593f, 8192.f, -8192.f, 8192.5f,
                             INFINITY, -INFINITY, NAN};
    std::uniform_real_distribution<float> U(-8300.f, 8300.f), S(-7.f, 7.f);
    for (int i = 0; i < 2000000; i++) xs.push_back(i & 1 ? U(g) : S(g));
    for (float x : xs) {
        float s, c;
        dsincos(x, s, c);
        float s1 = dsin(x), c1 = dcos(x);
        bool ok = (bits(s) == bits(s1) || (s != s && s1 != s1)) && (bits(c) == bits(c1) || (c != c && c1 != c1));
        if (!ok && bad++ < 5) std::printf("dsincos %a: %a %a vs %a %a\n", x, s, c, s1, c1);
    }
    // wrapi
    for (int n : {1, 2, 3, 255, 256, 512, 1000}) {
        for (int i = -5 * n - 3; i <= 5 * n + 3; i++) {
            int r = i % n;
            r = r < 0 ? r + n : r;
            if (wrapi(i, n) != r && bad++ < 5) std::printf("wrapi %d %d\n", i, n);
        }
    }
    // upper_bound_guided on sorted rows (with flat runs and a dominant jump)
    std::uniform_real_distribution<float> V(0.f, 1.f);
    for (int t = 0; t < 200; t++) {
        int n = 1 + (int)(g() % 600);
        std::vector<float> a(n);
        float acc = 0.f;
        for (int i = 0; i < n; i++) {
            float w = (g() % 5 == 0) ? 0.f : V(g);
            if (g() % 97 == 0) w *= 1000.f;
            acc += w;
            a[i] = acc;
        }
        for (int i = 0; i < n; i++) a[i] = acc > 0.f ? a[i] / acc : 0.f;
        std::vector<int> guide(kEnvGuide + 1);
        for (int k = 0; k <= kEnvGuide; k++) guide[k] = upper_bound(a.data(), n, (float)k / (float)kEnvGuide);
        for (int q = 0; q < 20000; q++) {
            float val = (float)((double)(uint32_t)g() * 0.00000000023283064365386962890625);
            if (upper_bound_guided(a.data(), guide.data(), val) != upper_bound(a.data(), n, val) && bad++ < 5)
                std::printf("upper_bound_guided n=%d val=%a\n", n, val);
        }
    }
    // fp64 island == fp32 quotient: random significands and exponents, plus all-ones significands
    std::uniform_int_distribution<uint32_t> M(0, 0x7FFFFF);
    std::uniform_int_distribution<int> E(-60, 60);
    long checked = 0;
    for (long q = 0; q < 30000000; q++) {
        uint32_t mx = (q % 7 == 0) ? 0x7FFFFF : M(g), md = (q % 11 == 0) ? 0x7FFFFF : M(g);
        float x = std::ldexp(1.f + (float)mx / 8388608.f, E(g)) * ((g() & 1) ? -1.f : 1.f);
        float d = std::ldexp(1.f + (float)md / 8388608.f, E(g) / 3);
        if (d < 1e-6f) continue;
        float fast = x / d;
        if (fast != 0.f && std::fabs(fast) < 1.17549435e-38f) continue;  // subnormal: fp64 path
        float ref = (float)((double)x * (1.0 / (double)d));
        checked++;
        if (bits(fast) != bits(ref) && bad++ < 5) std::printf("div %a / %a: %a vs %a\n", x, d, fast, ref);
    }
    std::printf("division pairs checked %ld\n", checked);
    std::printf("bad=%ld\n", bad);
    return bad != 0;
}
