// Host-side checks of the exactness claims behind the kernels' fast paths
// (compiled and run by tests/test_core_identities.py with hipcc (host code) -ffp-contract=off):
//   dsincos(x) == (dsin(x), dcos(x)) bit for bit;
//   wrapi's conditional add/subtract == the modulo form for every i;
//   upper_bound_guided == upper_bound on sorted CDF rows;
//   (float)((double)x * (1.0 / (double)d)) == x / d for normal-range quotients (tri_test's
//   fp32 replacement of the reference's fp64 island);
//   quot_fp64(a, y) == a / b whenever it reports success, for y = 1/b off by up to 8 ulp of
//   fp64 (the device's Newton-refined reciprocal is within ~1 ulp), over the full exponent
//   range including overflow to inf and quotients at the subnormal boundary.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "device/mcpt_core.hpp"
#include "kernels.hpp"

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
    // ... and on a row that is NaN throughout (row 0 of every HRDI map: 0 / (denom * 0))
    for (int n : {1, 2, 7, 512}) {
        std::vector<float> a(n, std::nanf(""));
        std::vector<int> guide(kEnvGuide + 1);
        for (int k = 0; k <= kEnvGuide; k++) guide[k] = upper_bound(a.data(), n, (float)k / (float)kEnvGuide);
        for (int q = 0; q < 20000; q++) {
            float val = (float)((double)(uint32_t)g() * 0.00000000023283064365386962890625);
            if ((upper_bound_guided(a.data(), guide.data(), val) != upper_bound(a.data(), n, val) ||
                 upper_bound(a.data(), n, val) != 0) && bad++ < 5)
                std::printf("upper_bound_guided NaN row n=%d val=%a\n", n, val);
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
    // rngf's fp32 form == the reference's (float)((double)d * 2^-32) for every d
    for (uint64_t d = 0; d <= 0xFFFFFFFFull; d += (d < (1ull << 26) ? 1 : 997)) {
        float f = (float)(uint32_t)d * 2.3283064365386962890625e-10f;
        float ref = (float)((double)(uint32_t)d * 0.00000000023283064365386962890625);
        if (bits(f) != bits(ref) && bad++ < 5) std::printf("rngf %llu\n", (unsigned long long)d);
    }
    // shared-reciprocal quotients (Recip / quot3 / tri_test on the device)
    long qchecked = 0, qfallback = 0;
    std::uniform_int_distribution<int> EA(-149, 127), EB(-149, 127), K(-8, 8);
    for (long q = 0; q < 40000000; q++) {
        const int mode = (int)(q % 5);
        uint32_t ma = (q % 7 == 0) ? 0x7FFFFF : M(g), mb = (q % 13 == 0) ? 0x7FFFFF : M(g);
        if (q % 17 == 0) mb = 0;  // power-of-two denominators
        int ea = EA(g), eb;
        if (mode == 0) eb = EB(g);                          // anything (overflow, underflow, subnormal b)
        else if (mode == 1) eb = ea - (int)(g() % 40);      // large quotients
        else if (mode == 2) eb = ea + 100 + (int)(g() % 30); // near the subnormal boundary
        else eb = ea - 20 + (int)(g() % 40);                // the common case
        if (eb < -149 || eb > 127) continue;
        float a = std::ldexp(1.f + (float)ma / 8388608.f, ea), b = std::ldexp(1.f + (float)mb / 8388608.f, eb);
        if (ea < -126) a = std::ldexp((float)(ma | 1), -149);  // subnormal operands
        if (eb < -126) b = std::ldexp((float)(mb | 1), -149);
        if (g() & 1) a = -a;
        if (g() & 1) b = -b;
        if (b == 0.f || !std::isfinite(a) || !std::isfinite(b)) continue;
        double y = 1.0 / (double)b;
        int k = K(g);
        for (int i = 0; i < (k < 0 ? -k : k); i++) y = std::nextafter(y, k < 0 ? 0.0 : 2.0 * y);
        float fast;
        if (!quot_fp64(a, y, fast)) { qfallback++; continue; }
        qchecked++;
        float ref = a / b;
        if (bits(fast) != bits(ref) && bad++ < 5) std::printf("quot %a / %a (k=%d): %a vs %a\n", a, b, k, fast, ref);
    }
    for (float a : {0.f, -0.f, 1.f, -3.f})  // signed zeros
        for (float b : {1.f, -2.f, 1e-40f, -3e38f}) {
            float fast;
            if (quot_fp64(a, 1.0 / (double)b, fast) && bits(fast) != bits(a / b) && bad++ < 5)
                std::printf("quot %a / %a: %a vs %a\n", a, b, fast, a / b);
        }
    std::printf("shared-reciprocal quotients checked %ld (fallback %ld)\n", qchecked, qfallback);
    // hardest cases: a / b = M / 2^25 + 1 / (2^25 B) with M odd (a float rounding midpoint),
    // i.e. |a/b - midpoint| = 1 / (M B) ~ 2^-49 relative, the minimum the argument allows.
    // With y within 2 ulp (the device budget) every one must round right; perturbing y by
    // 2^-45 must break some -- proof that these cases are near the boundary.
    long hard = 0, broken = 0;
    for (long q = 0; hard < 2000000 && q < 40000000; q++) {
        uint32_t B = (uint32_t)(0x800000u | (M(g) | 1u));  // odd 24-bit
        uint32_t inv = B;                                  // inverse of B mod 2^32 (Newton)
        for (int i = 0; i < 5; i++) inv *= 2u - B * inv;
        uint32_t Mv = (0u - inv) & 0x1FFFFFFu;             // M B == -1 (mod 2^25)
        if (!(Mv & 0x1000000u)) continue;                  // M must have 25 bits
        uint64_t num = (uint64_t)Mv * B + 1u;
        if (num & 0x1FFFFFFu) continue;
        uint64_t A = num >> 25;
        if (A < 0x800000u || A > 0xFFFFFFu) continue;
        int e = (int)(g() % 120) - 60;
        float a = std::ldexp((float)A, e), b = std::ldexp((float)B, e);
        hard++;
        for (int k = -2; k <= 2; k++) {
            double y = 1.0 / (double)b;
            for (int i = 0; i < (k < 0 ? -k : k); i++) y = std::nextafter(y, k < 0 ? 0.0 : 2.0 * y);
            float fast;
            if (quot_fp64(a, y, fast) && bits(fast) != bits(a / b) && bad++ < 5)
                std::printf("hard quot %a / %a (k=%d): %a vs %a\n", a, b, k, fast, a / b);
        }
        float wrong;
        quot_fp64(a, (1.0 / (double)b) * (1.0 - std::ldexp(1.0, -45)), wrong);
        if (bits(wrong) != bits(a / b)) broken++;
    }
    std::printf("hard quotients %ld, broken by a 2^-45 reciprocal error %ld\n", hard, broken);
    if (hard < 100000 || broken == 0) { std::printf("hard-case generator ineffective\n"); bad++; }
    // PLOC cluster records (bvh_build.hip): height and interior-node count round-trip for every
    // subtree size of a scene mcpt_scene_upload accepts (< 2^24 triangles: at most 2^24 - 2
    // interior nodes), including the merge of two halves of the largest tree
    {
        using namespace mcpt_dev;
        const uint32_t nmax = (1u << 24) - 2u;
        for (uint32_t c : {0u, 1u, 255u, 256u, (1u << 23) - 1u, 1u << 23, (1u << 23) + 7u, nmax - 1u, nmax}) {
            for (uint32_t h : {0u, 1u, 17u, 254u, 255u, 300u}) {
                const uint32_t p = ploc_pack(h, c);
                if ((ploc_count(p) != c || ploc_height(p) != (h < 255u ? h : 255u)) && bad++ < 5)
                    std::printf("ploc_pack(%u, %u) -> %u %u\n", h, c, ploc_height(p), ploc_count(p));
            }
        }
        const uint32_t a = ploc_pack(30, (nmax - 1u) / 2u), b = ploc_pack(40, nmax - 1u - (nmax - 1u) / 2u);
        const uint32_t m = ploc_merge(a, b);
        if ((ploc_count(m) != nmax || ploc_height(m) != 41u) && bad++ < 5)
            std::printf("ploc_merge: %u %u\n", ploc_height(m), ploc_count(m));
    }
    std::printf("bad=%ld\n", bad);
    return bad != 0;
}
