// mcpt_core.hpp -- MI355X-native numeric core of the wavefront path tracer.
//
// __host__ __device__ so the same arithmetic runs in the gfx950 kernels and in
// the host setup code (env tables).  Every function states the reference line
// it implements (paths relative to /root/reference/CUDA-RayTracer/).  Build
// flags: -ffp-contract=off, no fast-math: each float/double operation is one
// IEEE-754 rounding, so CPU and GPU agree bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MCPT_HD __host__ __device__ inline __attribute__((always_inline))

namespace mcpt {

// cuda_math/dMath.h:8-25
constexpr float K_EPSILON = 1e-6f;
constexpr float K_HUGE = 1e32f;
constexpr float PI_F = 3.14159265358979323846f;
constexpr float TWO_PI_F = 6.28318530717958647692f;
constexpr float PI_2_F = 1.57079632679489661923f;
constexpr float PI_4_F = 0.78539816339744830961f;
constexpr float ONE_PI_F = 0.31830988618379067153f;
constexpr float ONE_2PI_F = 0.15915494309189533576f;
constexpr float ONE_4PI_F = 0.07957747154594766788f;
constexpr float BRDF_EPS = 0.00001f;  // dMaterial.cu:8

MCPT_HD float qnan() { return __builtin_nanf(""); }
MCPT_HD int sign_bit(float x) { return (int)(__builtin_bit_cast(uint32_t, x) >> 31); }
MCPT_HD bool isnan_(float x) { return x != x; }
// IEEE fmax: a NaN operand loses (CUDA fmaxf semantics).
MCPT_HD float fmx(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    return a > b ? a : b;
}

// ---------------------------------------------------------------------------
// Deterministic transcendentals (replace CUDA --use_fast_math sin/cos/asin/
// acos/atan2/pow): cephes single-precision polynomials, one rounding per op.
// ---------------------------------------------------------------------------
constexpr float DP1 = 0.78515625f;
constexpr float DP2 = 2.4187564849853515625e-4f;
constexpr float DP3 = 3.77489497744594108e-8f;
constexpr float FOPI = 1.27323954473516f;

MCPT_HD float sin_poly(float x, float z) {
    float p = -1.9515295891e-4f * z;
    p = p + 8.3321608736e-3f;
    p = p * z;
    p = p - 1.6666654611e-1f;
    p = p * z;
    p = p * x;
    return p + x;
}
MCPT_HD float cos_poly(float z) {
    float p = 2.443315711809948e-5f * z;
    p = p - 1.388731625493765e-3f;
    p = p * z;
    p = p + 4.166664568298827e-2f;
    p = p * z;
    p = p * z;
    float h = 0.5f * z;
    p = p - h;
    return p + 1.0f;
}
MCPT_HD float dsin(float xx) {
    float x = xx;
    int sign = 1;
    if (x != x) return x;
    if (x < 0.f) { x = -x; sign = -1; }
    if (!(x <= 8192.f)) return qnan();
    int j = (int)(FOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { sign = -sign; j -= 4; }
    x = ((x - y * DP1) - y * DP2) - y * DP3;
    float z = x * x;
    float r = (j == 1 || j == 2) ? cos_poly(z) : sin_poly(x, z);
    return sign < 0 ? -r : r;
}
MCPT_HD float dcos(float xx) {
    float x = xx;
    if (x != x) return x;
    if (x < 0.f) x = -x;
    if (!(x <= 8192.f)) return qnan();
    int j = (int)(FOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    int sign = 1;
    if (j > 3) { j -= 4; sign = -sign; }
    if (j > 1) sign = -sign;
    x = ((x - y * DP1) - y * DP2) - y * DP3;
    float z = x * x;
    float r = (j == 1 || j == 2) ? sin_poly(x, z) : cos_poly(z);
    return sign < 0 ? -r : r;
}
// dsin and dcos of one argument with a shared range reduction: bit-identical to
// the two separate calls (same reduction, same polynomials, same sign rules).
MCPT_HD void dsincos(float xx, float& so, float& co) {
    float x = xx;
    if (x != x) { so = x; co = x; return; }
    int ss = 1, cs = 1;
    if (x < 0.f) { x = -x; ss = -1; }
    if (!(x <= 8192.f)) { so = qnan(); co = qnan(); return; }
    int j = (int)(FOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { ss = -ss; cs = -cs; j -= 4; }
    if (j > 1) cs = -cs;
    x = ((x - y * DP1) - y * DP2) - y * DP3;
    float z = x * x;
    const float sp = sin_poly(x, z), cp = cos_poly(z);
    const bool swap = (j == 1 || j == 2);
    const float rs = swap ? cp : sp, rc = swap ? sp : cp;
    so = ss < 0 ? -rs : rs;
    co = cs < 0 ? -rc : rc;
}
MCPT_HD float dasin(float xx) {
    float a, x, z;
    int sign, flag;
    if (xx != xx) return xx;
    if (xx > 0.f) { sign = 1; a = xx; } else { sign = -1; a = -xx; }
    if (a > 1.0f) return qnan();
    if (a < 1.0e-4f) {
        z = a;
    } else {
        if (a > 0.5f) { z = 0.5f * (1.0f - a); x = __builtin_sqrtf(z); flag = 1; }
        else { x = a; z = x * x; flag = 0; }
        float p = 4.2163199048e-2f * z;
        p = p + 2.4181311049e-2f; p = p * z;
        p = p + 4.5470025998e-2f; p = p * z;
        p = p + 7.4953002686e-2f; p = p * z;
        p = p + 1.6666752422e-1f; p = p * z;
        p = p * x;
        z = p + x;
        if (flag) { z = z + z; z = PI_2_F - z; }
    }
    return sign < 0 ? -z : z;
}
MCPT_HD float dacos(float x) {
    if (x != x) return x;
    if (x < -1.0f || x > 1.0f) return qnan();
    if (x < -0.5f) return PI_F - 2.0f * dasin(__builtin_sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * dasin(__builtin_sqrtf(0.5f * (1.0f - x)));
    return PI_2_F - dasin(x);
}
MCPT_HD float datan(float xx) {
    float x, y, z;
    int sign = 1;
    if (xx != xx) return xx;
    x = xx;
    if (xx < 0.f) { sign = -1; x = -xx; }
    if (x > 2.414213562373095f) { y = PI_2_F; x = -(1.0f / x); }
    else if (x > 0.4142135623730950f) { y = PI_4_F; x = (x - 1.0f) / (x + 1.0f); }
    else y = 0.0f;
    z = x * x;
    float p = 8.05374449538e-2f * z;
    p = p - 1.38776856032e-1f; p = p * z;
    p = p + 1.99777106478e-1f; p = p * z;
    p = p - 3.33329491539e-1f; p = p * z;
    p = p * x;
    p = p + x;
    y = y + p;
    return sign < 0 ? -y : y;
}
MCPT_HD float datan2(float y, float x) {
    if (x != x || y != y) return x + y;
    if (x == 0.f) {
        if (y > 0.f) return PI_2_F;
        if (y < 0.f) return -PI_2_F;
        return sign_bit(x) ? (sign_bit(y) ? -PI_F : PI_F) : y;
    }
    if (y == 0.f) return x > 0.f ? y : (sign_bit(y) ? -PI_F : PI_F);
    float w;
    if (x < 0.f) w = (y < 0.f) ? -PI_F : PI_F;
    else w = 0.0f;
    return w + datan(y / x);
}
MCPT_HD float pow5(float x) {  // pow(x, 5.f) in fresnel_schlick (dMaterial.cu:143)
    float x2 = x * x;
    float x4 = x2 * x2;
    return x4 * x;
}

// Assembly markers for the static instruction attribution (-DMCPT_ISA_MARKERS analysis builds of
// the device code, tools/isa_sections.py; nothing otherwise)
#if defined(MCPT_ISA_MARKERS) && defined(__HIP_DEVICE_COMPILE__)
#define MCPT_MARK(name) __asm__ volatile("; MCPT_SEC " name)
#else
#define MCPT_MARK(name) \
    do {                \
    } while (0)
#endif

// ---------------------------------------------------------------------------
// Keyed RNG around lowerbias32 (cuda_math/Random.cu:5-13)
// ---------------------------------------------------------------------------
MCPT_HD uint32_t lowerbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0xa812d533u;
    x ^= x >> 15;
    x *= 0xb278e4adu;
    x ^= x >> 17;
    return x;
}
MCPT_HD uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
MCPT_HD uint32_t rng_key(uint64_t seed, uint32_t pixel, uint32_t sample) {
    uint64_t s = splitmix64((((uint64_t)pixel << 32) | (uint64_t)sample) ^ seed);
    return (uint32_t)(s ^ (s >> 32));
}
// rand_float: rand() * 2^-32 in double, rounded to float (Random.cu:31-35).  The
// double product is exact, so RN32(d * 2^-32) == RN32(d) * 2^-32 (power-of-two
// scale, no underflow): one u32 -> f32 conversion and one exact multiply.
MCPT_HD float rngf(uint32_t key, uint32_t len, uint32_t slot) {
    uint32_t d = lowerbias32(key + (len * 16u + slot) * 0x9E3779B9u);
    return (float)d * 2.3283064365386962890625e-10f;
}
enum : uint32_t {
    SL_GEN_U = 0, SL_GEN_V = 1,
    SL_RR = 0, SL_LIGHT = 1, SL_ENV_U = 2, SL_ENV_V = 3,
    SL_MAT_LOBE = 4, SL_MAT_E0 = 5,
    SL_CONT_LOBE = 10, SL_CONT_E0 = 11
};
struct Rng {
    uint32_t key, len;
    MCPT_HD float operator()(uint32_t slot) const { return rngf(key, len, slot); }
};

// ---------------------------------------------------------------------------
// Quotients with a shared denominator.  The reference divides in IEEE fp32:
// RN32(a / b), which gfx950 expands to ~12 VALU operations per quotient
// (div_scale x2, rcp, 6 fma, div_fmas, div_fixup).  Device code computes one
// fp64 reciprocal y per denominator (hardware estimate + two Newton steps:
// |y - 1/b| <= ~2^-52 |1/b|) and RN32(RN64(a * y)) per quotient, 3 operations.
// Equal to RN32(a / b) for finite nonzero b: the product is within 2^-51
// (relative) of a/b, while a/b with 24-bit significands is never a float
// rounding boundary and stays >= 2^-49 (relative) away from every one (a 25-bit
// midpoint m = a/b would need a = m b with >24 significant bits).  Quotients in
// the subnormal range redo the IEEE division (the conversion's denormal mode is
// not relied on).  tests/native/core_identities.cpp checks quot_fp64 against a/b
// with y perturbed by the reciprocal's error budget.  Host code divides.
// ---------------------------------------------------------------------------
struct Recip { float b; double y; bool ok; };
MCPT_HD bool quot_fp64(float a, double y, float& q) {  // false: redo as a / b
    q = (float)((double)a * y);
    return __builtin_fabsf(q) >= 1.17549435e-38f || a == 0.f;
}
MCPT_HD Recip recip(float b) {
    Recip r{b, 0.0, false};
#if defined(__HIP_DEVICE_COMPILE__)
    r.ok = __builtin_fabsf(b) <= 3.40282347e38f && b != 0.f;
    const double bd = (double)b;
    double y = __builtin_amdgcn_rcp(bd);
    double e = __builtin_fma(-bd, y, 1.0);
    y = __builtin_fma(e, y, y);
    e = __builtin_fma(-bd, y, 1.0);
    r.y = __builtin_fma(e, y, y);
#endif
    return r;
}
// The three quotients of one denominator, with one (rarely taken) branch for the
// whole group: any out-of-range case redoes all three as IEEE divisions.
MCPT_HD void quot3(float a0, float a1, float a2, float b, float& q0, float& q1, float& q2) {
#if defined(__HIP_DEVICE_COMPILE__)
    const Recip r = recip(b);
    bool good = quot_fp64(a0, r.y, q0);
    good = quot_fp64(a1, r.y, q1) && good;
    good = quot_fp64(a2, r.y, q2) && good;
    if (r.ok && good) return;
#endif
    q0 = a0 / b;
    q1 = a1 / b;
    q2 = a2 / b;
}

// ---------------------------------------------------------------------------
// Vec3f (cuda_math/Vector.h): one rounding per component per operator.
// ---------------------------------------------------------------------------
struct V3 { float x, y, z; };
MCPT_HD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
MCPT_HD V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
MCPT_HD V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
MCPT_HD V3 operator*(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
MCPT_HD V3 operator/(V3 a, V3 b) { return V3{a.x / b.x, a.y / b.y, a.z / b.z}; }
MCPT_HD V3 operator*(V3 v, float s) { return V3{s * v.x, s * v.y, s * v.z}; }
MCPT_HD V3 operator/(V3 v, float s) {
    V3 q;
    quot3(v.x, v.y, v.z, s, q.x, q.y, q.z);
    return q;
}
MCPT_HD V3 operator-(V3 v) { return V3{-v.x, -v.y, -v.z}; }
MCPT_HD float dot(V3 a, V3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }  // Vector.h:790
MCPT_HD V3 normalize(V3 v) {                                                      // Vector.h:1077
    float l = __builtin_sqrtf(dot(v, v));
    return (l == 0.f) ? v : v / l;
}
MCPT_HD V3 cross(V3 a, V3 b) {                                                    // Vector.h:1108
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
MCPT_HD V3 reflect(V3 i, V3 n) { return i - (n * 2.f) * dot(n, i); }               // Vector.h:1103
MCPT_HD V3 mix(V3 a, V3 b, float t) { return a * (1.f - t) + b * t; }               // Vector.h:1092
MCPT_HD float luminance(V3 c) {                                                   // Vector.h:1123
    return (float)(0.299 * (double)c.x + 0.587 * (double)c.y + 0.114 * (double)c.z);
}
MCPT_HD V3 ld3(const float* p, int64_t i) { return V3{p[3 * i], p[3 * i + 1], p[3 * i + 2]}; }

// jek::gram_schmidt (Vector.h:1128-1139): component-wise divide quirk kept.
// FIXED (quality mode): the textbook projection
// T = normalize(x - vn (x . vn)) with the normalised normal vn.
template <bool FIXED = false>
MCPT_HD V3 gram_schmidt(V3 v, const Rng& r, uint32_t slot0) {
    float rx = r(slot0 + 0) * 2.f + -1.f;  // rand_float(-1,1): Random.cu:39-42
    float ry = r(slot0 + 1) * 2.f + -1.f;
    float rz = r(slot0 + 2) * 2.f + -1.f;
    V3 x = v3(rx, ry, rz);
    if (FIXED) {
        const V3 vn = normalize(v);
        return normalize(x - vn * dot(x, vn));
    }
    float x_dot_v = dot(x, v);
    V3 vn = normalize(v);
    V3 vn2 = vn * vn;
    x = x - ((v * x_dot_v) / vn2);
    return normalize(x);
}
// sample_spherical_map / _direction (Vector.h:1141-1160).
MCPT_HD void spherical_map(V3 d, float& u, float& v) {
    u = 0.5f + datan2(d.z, d.x) * ONE_2PI_F;
    v = 0.5f - dasin(d.y) * ONE_PI_F;
}
// The two factors of spherical_direction: (sin, cos) of theta (from v) and of phi (from u).
MCPT_HD void spherical_theta(float v, float& st, float& ct) { dsincos(PI_F * v, st, ct); }
MCPT_HD void spherical_phi(float u, float& sp, float& cp) {
    float phi = (float)((double)(2.f * PI_F) * ((double)u - 0.5));  // fp64 island
    dsincos(phi, sp, cp);
}
MCPT_HD V3 spherical_direction(float u, float v) {
    float st, ct, sp, cp;
    spherical_theta(v, st, ct);
    spherical_phi(u, sp, cp);
    V3 n;
    n.x = cp * st;
    n.z = sp * st;
    n.y = ct;
    return n;
}

// ---------------------------------------------------------------------------
// Environment light (EnvironmentLight.cu:10-109, Helpers.cu:15-30).
// ---------------------------------------------------------------------------
struct EnvView {
    int mode;  // 0 Color, 1 HRDI
    float color[3];
    float ls;
    int w, h;
    // RGB32F + pdf, row 0 = top (stbi_loadf, no flip: dTexture.cu:208).  The device copy's
    // alpha plane, which env_L never reads (tex2DLod<float4>(...).xyz, EnvironmentLight.cu:45),
    // holds the pdf table (k_env_pack): a BRDF sample's pdf texel then shares the bilinear
    // taps' lines, and the light's tables are 0.5 MiB smaller for the per-XCD L2.
    const float4* tex;
    const float* marginal_y;  // h
    const float* conds_y;     // h*w
    const float* pdf;         // h*w (readback only: the shading kernels read tex[i].w)
    // Optional search guides (device only, built at upload when the CDFs are
    // sorted): guide_m[k] = upper_bound(marginal_y, h, k / kEnvGuide), k = 0..kEnvGuide,
    // and the same per conditional row at guide_c[y * (kEnvGuide + 1) + k].  16-bit
    // entries (tables up to 65535 wide/high): 256 x 1025 x 2 B = 512 KiB for a 512x256 map.
    const uint16_t* guide_m;
    const uint16_t* guide_c;
    // Optional light-sample tables (device only, HRDI mode, built at upload by
    // k_env_table from these same functions): in either mode env_dir's result is a
    // function of the sampled cell (x, y) alone, and so are env_L and env_pdf at that
    // direction.  Entry (y * (w + 1) + x + 1) = {L.xyz, pdf} for x = -1 .. w-1 (the
    // reference's off-by-one column -1 included); the direction is separable,
    // (cos phi * sin theta, cos theta, sin phi * sin theta), so its factors come from a
    // row table lrow[y] = (sin theta, cos theta) and a column table lcol[x + 1] =
    // (sin phi, cos phi).  [0] reference mode, [1] quality mode.
    const float4* ltab[2];
    const float2* lrow[2];
    const float2* lcol[2];
};
// Bins per guide table.  Each bin is equally likely (val uniform), and a bin holds W / G
// CDF entries on average, so G = 1024 leaves ~0.5 (conditional rows, W = 512) and
// ~0.25 (marginal, H = 256) bisection steps per search: the dependent-load chain of
// env_dir is the guide fetch plus at most a step or two.
constexpr int kEnvGuide = 1024;

MCPT_HD int upper_bound(const float* list, int size, float val) {  // Helpers.cu:15-30
    int middle, left = 0, right = size;
    while (left < right) {
        middle = (right - left) / 2 + left;
        if (val >= list[middle]) left = middle + 1;
        else right = middle;
    }
    if (left < size && list[left] <= val) left++;
    return left;
}
// upper_bound on a sorted list whose answers at the bin edges k / kEnvGuide are
// precomputed: for val in [k/G, (k+1)/G) (exact bin: G is a power of two) the
// answer lies in [guide[k], guide[k+1]] by monotonicity, and the same bisection
// restricted to that range returns it.  val in [0, 1) (rand_float).
template <class G>
MCPT_HD int upper_bound_guided(const float* list, const G* guide, float val) {
    int k = (int)(val * (float)kEnvGuide);
    k = k < 0 ? 0 : (k > kEnvGuide - 1 ? kEnvGuide - 1 : k);
    int left = (int)guide[k], right = (int)guide[k + 1];
    while (left < right) {
        const int middle = (right - left) / 2 + left;
        if (val >= list[middle]) left = middle + 1;
        else right = middle;
    }
    return left;
}
MCPT_HD int wrapi(int i, int n) {  // i mod n in [0, n); one conditional add/subtract covers |i| < 2n
    int r = i < 0 ? i + n : (i >= n ? i - n : i);
    if ((unsigned)r >= (unsigned)n) {
        r = i % n;
        r = r < 0 ? r + n : r;
    }
    return r;
}
MCPT_HD float q8(float a) { return __builtin_floorf(a * 256.f + 0.5f) * (1.0f / 256.f); }
// Software tex2DLod<float4>: linear filter, wrap, normalized coords, 8-bit
// fractional weights like the texture unit (dTexture.cu:265-271).  NaN -> 0.
MCPT_HD V3 tex_bilinear(const float4* tex, int W, int H, float u, float v) {
    if (!(__builtin_fabsf(u) < 65536.f)) u = 0.f;
    if (!(__builtin_fabsf(v) < 65536.f)) v = 0.f;
    float x = u * (float)W - 0.5f;
    float y = v * (float)H - 0.5f;
    float fx = __builtin_floorf(x), fy = __builtin_floorf(y);
    float ax = q8(x - fx), ay = q8(y - fy);
    int i0 = wrapi((int)fx, W), i1 = wrapi((int)fx + 1, W);
    int j0 = wrapi((int)fy, H), j1 = wrapi((int)fy + 1, H);
    float4 t00 = tex[(int64_t)j0 * W + i0], t10 = tex[(int64_t)j0 * W + i1];
    float4 t01 = tex[(int64_t)j1 * W + i0], t11 = tex[(int64_t)j1 * W + i1];
    float bx = 1.f - ax, by = 1.f - ay;
    float w00 = bx * by, w10 = ax * by, w01 = bx * ay, w11 = ax * ay;
    V3 o;
    o.x = ((w00 * t00.x + w10 * t10.x) + w01 * t01.x) + w11 * t11.x;
    o.y = ((w00 * t00.y + w10 * t10.y) + w01 * t01.y) + w11 * t11.y;
    o.z = ((w00 * t00.z + w10 * t10.z) + w01 * t01.z) + w11 * t11.z;
    return o;
}
MCPT_HD V3 env_L(const EnvView& e, V3 wi) {  // EnvironmentLight.cu:34-47
    if (e.mode == 0 || e.tex == nullptr) return v3(e.color[0], e.color[1], e.color[2]) * e.ls;
    float u, v;
    spherical_map(wi, u, v);
    return tex_bilinear(e.tex, e.w, e.h, u, v);
}
// FIXED (quality mode): the pdf is read from the cell the sampler draws from
// ((int)(u W), (int)(v H), clamped) instead of the reference's (u (W-1), v (H-1))
// cell (EnvironmentLight.cu:76), and env_dir samples cell centres with the row /
// column index clamped to the table (the reference's off-by-one can give -1).
template <bool FIXED = false>
MCPT_HD float env_pdf_uv(const EnvView& e, float u, float v) {
    int px, py;
    if (FIXED) {
        const float fx = u * (float)e.w, fy = v * (float)e.h;
        px = (fx == fx && fx >= 0.f) ? (fx < (float)(e.w - 1) ? (int)fx : e.w - 1) : 0;
        py = (fy == fy && fy >= 0.f) ? (fy < (float)(e.h - 1) ? (int)fy : e.h - 1) : 0;
    } else {
        const float fx = u * (float)(unsigned)(e.w - 1), fy = v * (float)(unsigned)(e.h - 1);
        px = (fx == fx && fx >= 0.f && fx < (float)e.w) ? (int)fx : 0;
        py = (fy == fy && fy >= 0.f && fy < (float)e.h) ? (int)fy : 0;
    }
    float pdf = e.tex[(int64_t)py * e.w + px].w;
    float sin_theta = dsin(PI_F * v);
    if (sin_theta == 0.f) return 0.f;
    return pdf * (float)((unsigned)e.w * (unsigned)e.h) / (((2.f * sin_theta) * PI_F) * PI_F);
}
template <bool FIXED = false>
MCPT_HD float env_pdf(const EnvView& e, V3 wi) {  // EnvironmentLight.cu:65-85
    if (e.mode == 0 || e.tex == nullptr) return ONE_4PI_F;
    float u, v;
    spherical_map(wi, u, v);
    return env_pdf_uv<FIXED>(e, u, v);
}
// env_L and env_pdf of one direction sharing its spherical map (same values as the two calls)
template <bool FIXED = false>
MCPT_HD void env_L_pdf(const EnvView& e, V3 wi, V3& L, float& pdf) {
    if (e.mode == 0 || e.tex == nullptr) {
        L = v3(e.color[0], e.color[1], e.color[2]) * e.ls;
        pdf = ONE_4PI_F;
        return;
    }
    float u, v;
    spherical_map(wi, u, v);
    L = tex_bilinear(e.tex, e.w, e.h, u, v);
    pdf = env_pdf_uv<FIXED>(e, u, v);
}
// HRDI sampling, EnvironmentLight.cu:20-29: the cell (x, y) drawn from the marginal and
// conditional CDFs (x can be -1 in reference mode; y < 0 is unreachable).
template <bool FIXED = false>
MCPT_HD void env_cell(const EnvView& e, const Rng& r, int& x, int& y) {
    float ex = r(SL_ENV_U);
    float ey = r(SL_ENV_V);
    if (e.guide_m) {
        y = (int)((float)upper_bound_guided(e.marginal_y, e.guide_m, ey) - 1.f);
        if (y < 0) y = 0;  // unreachable (marginal_y[0] == 0); reference reads row -1
        x = (int)((float)upper_bound_guided(e.conds_y + (int64_t)y * e.w, e.guide_c + y * (kEnvGuide + 1), ex) - 1.f);
    } else {
        y = (int)((float)upper_bound(e.marginal_y, e.h, ey) - 1.f);
        if (y < 0) y = 0;
        x = (int)((float)upper_bound(e.conds_y + (int64_t)y * e.w, e.w, ex) - 1.f);
    }
    if (FIXED) {
        y = y > e.h - 1 ? e.h - 1 : y;
        x = x < 0 ? 0 : (x > e.w - 1 ? e.w - 1 : x);
    }
}
// the direction of a sampled cell (EnvironmentLight.cu:28-31: pixel corner u = x / W)
template <bool FIXED = false>
MCPT_HD float env_cell_u(const EnvView& e, int x) { return FIXED ? ((float)x + 0.5f) / (float)e.w : (float)x / (float)e.w; }
template <bool FIXED = false>
MCPT_HD float env_cell_v(const EnvView& e, int y) { return FIXED ? ((float)y + 0.5f) / (float)e.h : (float)y / (float)e.h; }
template <bool FIXED = false>
MCPT_HD V3 env_cell_dir(const EnvView& e, int x, int y) {
    return spherical_direction(env_cell_u<FIXED>(e, x), env_cell_v<FIXED>(e, y));
}
template <bool FIXED = false>
MCPT_HD V3 env_dir(const EnvView& e, const Rng& r) {  // EnvironmentLight.cu:10-33
    if (e.mode == 0 || e.tex == nullptr) {
        float u = r(SL_ENV_U);
        float v = r(SL_ENV_V);
        return spherical_direction(u, v);
    }
    int x, y;
    env_cell<FIXED>(e, r, x, y);
    return env_cell_dir<FIXED>(e, x, y);
}

// ---------------------------------------------------------------------------
// BRDF (dMaterial.cu), material factors only (dMaterial.cu:10-115).
// ---------------------------------------------------------------------------
struct Mat { V3 base, fresnel; float rough, metal; };
MCPT_HD Mat load_mat(const float* p) {
    Mat m;
    m.base = v3(p[0], p[1], p[2]);
    m.fresnel = v3(p[3], p[4], p[5]);
    m.rough = fmx(p[6], BRDF_EPS);  // get_roughness (dMaterial.cu:54)
    m.metal = p[7];
    return m;
}
MCPT_HD float power_heuristic(float fPdf, float gPdf) {  // dMaterial.cu:134-139
    float f = 1.0f * fPdf, g = 1.0f * gPdf;
    return (f * f) / (f * f + g * g);
}
MCPT_HD V3 fresnel_schlick(V3 f0, V3 v, V3 h) {  // dMaterial.cu:141-144
    float v_dot_h = fmx(dot(v, h), 0.f);
    return f0 + (v3(1.f, 1.f, 1.f) - f0) * pow5(1.f - v_dot_h);
}
MCPT_HD float ndf_ggx_tr(V3 n, V3 h, float r) {  // dMaterial.cu:150-161
    float a = r * r;
    float a2 = a * a;
    float n_dot_h = fmx(dot(n, h), BRDF_EPS);
    float n_dot_h_2 = n_dot_h * n_dot_h;
    float denom = fmx(n_dot_h_2 * (a2 - 1.f) + 1.f, BRDF_EPS);
    return a2 / ((PI_F * denom) * denom);
}
MCPT_HD float g1_schlick_ggx(V3 v, V3 n, float r) {  // dMaterial.cu:205-213
    float a = r * r;
    float k = a / 2.f;
    float n_dot_v = fmx(dot(n, v), BRDF_EPS);
    return n_dot_v / fmx(n_dot_v * (1.f - k) + k, BRDF_EPS);
}
template <bool FIXED = false>
MCPT_HD V3 diff_get_wi(V3 N, const Rng& r, uint32_t s0) {  // dMaterial.cu:232-254
    float e0 = r(s0 + 0);
    float e1 = r(s0 + 1);
    float sinTheta = __builtin_sqrtf(1.f - e0 * e0);
    float phi = (2.f * PI_F) * e1;
    float sp, cp;
    dsincos(phi, sp, cp);
    float x = sinTheta * cp;
    float z = sinTheta * sp;
    V3 T = gram_schmidt<FIXED>(N, r, s0 + 2);
    V3 B = normalize(cross(N, T));
    return normalize((T * x + N * e0) + B * z);
}
MCPT_HD V3 diff_get_f(const Mat& m, V3 n, V3 wi, V3 wo) {  // dMaterial.cu:259-276
    float n_dot_wi = fmx(dot(n, wi), BRDF_EPS);
    V3 f0 = mix(m.fresnel, m.base, m.metal);
    V3 wh = normalize(wo + wi);
    V3 F = fresnel_schlick(f0, wh, wo);
    V3 kD = v3(1.f, 1.f, 1.f) - F;
    kD = kD * (1.f - m.metal);
    return ((kD * m.base) * n_dot_wi) * ONE_PI_F;
}
template <bool FIXED = false>
MCPT_HD V3 spec_get_wi(const Mat& m, V3 N, V3 wo, const Rng& r, uint32_t s0) {  // dMaterial.cu:278-307
    float rr = m.rough;
    float a2 = ((rr * rr) * rr) * rr;
    float e0 = r(s0 + 0);
    float e1 = r(s0 + 1);
    float theta = dacos(__builtin_sqrtf((1.f - e0) / (e0 * (a2 - 1.f) + 1.f)));
    float phi = TWO_PI_F * e1;
    float st, ct, sp, cp;
    dsincos(theta, st, ct);
    dsincos(phi, sp, cp);
    V3 h = v3(st * cp, ct, st * sp);
    V3 T = gram_schmidt<FIXED>(N, r, s0 + 2);
    V3 B = normalize(cross(N, T));
    V3 smp = normalize((T * h.x + N * h.y) + B * h.z);
    return normalize(reflect(-wo, smp));
}
MCPT_HD float spec_get_pdf(const Mat& m, V3 n, V3 wi, V3 wo) {  // dMaterial.cu:308-321
    V3 wh = normalize(wo + wi);
    float wh_dot_n = fmx(dot(wh, n), BRDF_EPS);
    float wo_dot_wh = fmx(dot(wo, wh), BRDF_EPS);
    float D = ndf_ggx_tr(n, wh, m.rough);
    return (D * wh_dot_n) / fmx(4.f * wo_dot_wh, BRDF_EPS);
}
MCPT_HD V3 spec_get_f(const Mat& m, V3 n, V3 wi, V3 wo) {  // dMaterial.cu:322-343
    V3 f0 = mix(m.fresnel, m.base, m.metal);
    V3 wh = normalize(wo + wi);
    float n_dot_wi = fmx(dot(n, wi), BRDF_EPS);
    float n_dot_wo = fmx(dot(n, wo), BRDF_EPS);
    float D = ndf_ggx_tr(n, wh, m.rough);
    float G = g1_schlick_ggx(wi, n, m.rough) * g1_schlick_ggx(wo, n, m.rough);
    V3 F = fresnel_schlick(f0, wh, wo);
    V3 L = (F * (D * G)) * n_dot_wi;
    return L / fmx((4.f * n_dot_wo) * n_dot_wi, BRDF_EPS);
}
MCPT_HD float diff_get_pdf() { return ONE_2PI_F; }  // dMaterial.cu:255-258
MCPT_HD V3 brdf_f(const Mat& m, V3 n, V3 wi, V3 wo) {  // spec_get_f + diff_get_f (wavefront_kernels.cu:326)
    return spec_get_f(m, n, wi, wo) + diff_get_f(m, n, wi, wo);
}
MCPT_HD float brdf_pdf(const Mat& m, V3 n, V3 wi, V3 wo) {  // (diff + spec) * 0.5 (wavefront_kernels.cu:329)
    return (diff_get_pdf() + spec_get_pdf(m, n, wi, wo)) * 0.5f;
}

// Lobe-merged sampler: spec_get_wi (spec) or diff_get_wi (!spec) with their common tail
// -- the phi rotation, the gram_schmidt frame and the frame transform -- written once, so
// a wave whose lanes picked different lobes runs that tail once instead of in both
// branches.  Per lane the operations are exactly those of the function it selects
// (2.f * PI_F == TWO_PI_F; the diffuse "theta" terms are sqrt(1 - e0^2) and e0).
template <bool FIXED = false>
MCPT_HD V3 brdf_sample_wi(const Mat& m, V3 N, V3 wo, const Rng& r, uint32_t s0, bool spec) {
    float e0 = r(s0 + 0);
    float e1 = r(s0 + 1);
    float st, ct;
    if (spec) {
        float rr = m.rough;
        float a2 = ((rr * rr) * rr) * rr;
        float theta = dacos(__builtin_sqrtf((1.f - e0) / (e0 * (a2 - 1.f) + 1.f)));
        dsincos(theta, st, ct);
    } else {
        st = __builtin_sqrtf(1.f - e0 * e0);
        ct = e0;
    }
    float phi = TWO_PI_F * e1;
    float sp, cp;
    dsincos(phi, sp, cp);
    float x = st * cp;
    float z = st * sp;
    V3 T = gram_schmidt<FIXED>(N, r, s0 + 2);
    V3 B = normalize(cross(N, T));
    V3 v = normalize((T * x + N * ct) + B * z);
    if (spec) v = normalize(reflect(-wo, v));
    return v;
}
// brdf_f and brdf_pdf of one direction with their shared terms evaluated once: the half
// vector, f0, D, F and n.wi (same operations and values as the separate calls).
MCPT_HD void brdf_f_pdf(const Mat& m, V3 n, V3 wi, V3 wo, V3& f, float& pdf) {
    V3 wh = normalize(wo + wi);
    V3 f0 = mix(m.fresnel, m.base, m.metal);
    float n_dot_wi = fmx(dot(n, wi), BRDF_EPS);
    float n_dot_wo = fmx(dot(n, wo), BRDF_EPS);
    float D = ndf_ggx_tr(n, wh, m.rough);
    float G = g1_schlick_ggx(wi, n, m.rough) * g1_schlick_ggx(wo, n, m.rough);
    V3 F = fresnel_schlick(f0, wh, wo);
    V3 L = (F * (D * G)) * n_dot_wi;
    V3 fs = L / fmx((4.f * n_dot_wo) * n_dot_wi, BRDF_EPS);    // spec_get_f
    V3 kD = (v3(1.f, 1.f, 1.f) - F) * (1.f - m.metal);
    V3 fd = ((kD * m.base) * n_dot_wi) * ONE_PI_F;            // diff_get_f
    f = fs + fd;
    float wh_dot_n = fmx(dot(wh, n), BRDF_EPS);
    float wo_dot_wh = fmx(dot(wo, wh), BRDF_EPS);
    float ps = (D * wh_dot_n) / fmx(4.f * wo_dot_wh, BRDF_EPS);  // spec_get_pdf
    pdf = (diff_get_pdf() + ps) * 0.5f;
}

// ---------------------------------------------------------------------------
// Camera (Camera.cu:18-45, Sample.cu:129-149).
// ---------------------------------------------------------------------------
struct CamView {
    float ivp[16];  // inverse(proj*view), column-major m[c][r]
    float iv[16];   // inverse(view)
    float lens_radius, focal;
};
MCPT_HD void mat_vec4(const float* m, float v0, float v1, float v2, float v3_, float out[4]) {
    for (int r = 0; r < 4; r++)  // cuda_math/Matrix.h:196-204
        out[r] = m[0 * 4 + r] * v0 + m[1 * 4 + r] * v1 + m[2 * 4 + r] * v2 + m[3 * 4 + r] * v3_;
}
MCPT_HD void concentric_disk(const Rng& r, float& dx, float& dy) {  // Sample.cu:150-172
    float ux = r(SL_GEN_U), uy = r(SL_GEN_V);
    float ox = 2.f * ux - 1.f, oy = 2.f * uy - 1.f;
    if (ox == 0.f && oy == 0.f) { dx = 0.f; dy = 0.f; return; }
    // the two branches' quotients as one division of selected operands (a wave whose lanes take
    // both branches divides once)
    const bool xm = __builtin_fabsf(ox) > __builtin_fabsf(oy);
    const float q = (xm ? oy : ox) / (xm ? ox : oy);
    const float theta = xm ? PI_4_F * q : PI_2_F - PI_4_F * q, rr = xm ? ox : oy;
    float st, ct;
    dsincos(theta, st, ct);
    dx = rr * ct;
    dy = rr * st;
}
// dCamera::gen_ray in two parts.  gen_ray_pixel: everything that depends on the pixel alone (the
// pinhole ray through it: the fp64 NDC island, both unprojections, the direction); k_cam_table
// evaluates it once per pixel of the film.  gen_ray_lens: the per-sample thin-lens part from the
// pixel's focal point (two RNG draws).  gen_ray = the two in sequence, the same operations.
MCPT_HD void gen_ray_pixel(const CamView& c, int W, int H, int xi, int yi, V3& o, V3& d) {
    float x = (float)xi, y = (float)yi;
    float px = (float)(2.f * (((double)x + 0.5) / (double)(float)W) - 1.f);  // fp64 island :21-22
    float py = (float)(1.f - 2.f * (((double)y + 0.5) / (double)(float)H));
    float an[4], af[4];
    mat_vec4(c.ivp, px, py, -1.f, 1.f, an);
    mat_vec4(c.ivp, px, py, 1.f, 1.f, af);
    V3 pNear = v3(an[0], an[1], an[2]) / an[3];
    V3 pFar = v3(af[0], af[1], af[2]) / af[3];
    o = pNear;
    d = normalize(pFar - pNear);
}
MCPT_HD V3 gen_ray_focal(const CamView& c, V3 o, V3 d) { return o + d * c.focal; }  // pFocal (:34)
MCPT_HD void gen_ray_lens(const CamView& c, V3 pFocal, const Rng& r, V3& o, V3& d) {
    float lx, ly;
    concentric_disk(r, lx, ly);
    lx = lx * c.lens_radius;
    ly = ly * c.lens_radius;
    float al[4];
    mat_vec4(c.iv, lx, ly, 0.f, 1.f, al);
    V3 pLens = v3(al[0], al[1], al[2]) / al[3];
    o = pLens;
    d = normalize(pFocal - o);
}
MCPT_HD void gen_ray(const CamView& c, int W, int H, int xi, int yi, const Rng& r, V3& o, V3& d) {
    gen_ray_pixel(c, W, H, xi, yi, o, d);
    if (c.lens_radius > 0.f) gen_ray_lens(c, gen_ray_focal(c, o, d), r, o, d);
}

// ---------------------------------------------------------------------------
// Triangle / box tests (Triangle.cu:9-65, Bounds3f.h:121-153).
// ---------------------------------------------------------------------------
// Moller-Trumbore with TEST_CULL and the fp64 det island.  Returns 1 when the
// line hits the front face; t/u/v are the reference's float values.
MCPT_HD bool tri_test(V3 o, V3 d, V3 p0, V3 e1, V3 e2, float& t, float& u_out, float& v_out) {
    V3 pvec = cross(d, e2);
    float detf = dot(e1, pvec);
    if (detf < K_EPSILON) return false;  // (double)det < (double)1e-6f, same ordering
    V3 tvec = o - p0;
    float u = dot(tvec, pvec);
    if (u < 0.f || u > detf) return false;
    V3 qvec = cross(tvec, e1);
    float v = dot(d, qvec);
    if (v < 0.f || u + v > detf) return false;
    float tf = dot(e2, qvec);
#if defined(__HIP_DEVICE_COMPILE__)
    // The reference's fp64 island (Triangle.cu:35-38) rounds twice: RN32(x * RN64(1/det)).
    // For float x and det that equals the correctly rounded fp32 quotient RN32(x / det):
    // the double product is within ~2^-52 (relative) of x/det, while x/det is never a
    // float rounding midpoint and lies >= ~2^-49 (relative) away from every one (x, det
    // have 24-bit significands, a midpoint has 25), so both round the same way -- and so
    // does quot_fp64 with the Newton-refined reciprocal (see Recip).  Normal range only:
    // a nonzero subnormal quotient takes the reference's fp64 path.
    {
        const Recip r = recip(detf);
        float tq, uq, vq;
        bool good = quot_fp64(tf, r.y, tq);
        good = quot_fp64(u, r.y, uq) && good;
        good = quot_fp64(v, r.y, vq) && good;
        if (r.ok && good) {
            t = tq;
            u_out = uq;
            v_out = vq;
            return true;
        }
    }
#endif
    double inv_det = 1.0 / (double)detf;
    t = (float)((double)tf * inv_det);
    u_out = (float)((double)u * inv_det);
    v_out = (float)((double)v * inv_det);
    return true;
}
// The same test when only t is needed (the traversal keeps the triangle index; the hit
// record is rebuilt from it where it is consumed).  Acceptance does not depend on the
// quotients, and t is the same value: its fast path is taken on its own range check
// alone (u and v no longer send a hit to the fp64 path, which gives the same t anyway).
MCPT_HD bool tri_test_t(V3 o, V3 d, V3 p0, V3 e1, V3 e2, float& t) {
    V3 pvec = cross(d, e2);
    float detf = dot(e1, pvec);
    if (detf < K_EPSILON) return false;
    V3 tvec = o - p0;
    float u = dot(tvec, pvec);
    if (u < 0.f || u > detf) return false;
    V3 qvec = cross(tvec, e1);
    float v = dot(d, qvec);
    if (v < 0.f || u + v > detf) return false;
    float tf = dot(e2, qvec);
#if defined(__HIP_DEVICE_COMPILE__)
    {
        const Recip r = recip(detf);
        float tq;
        if (quot_fp64(tf, r.y, tq) && r.ok) {
            t = tq;
            return true;
        }
    }
#endif
    MCPT_MARK("rare");  // (a subnormal quotient or an out-of-range det: the fp64 island itself)
    t = (float)((double)tf * (1.0 / (double)detf));
    return true;
}

// ---------------------------------------------------------------------------
// Conservative box culling ("the culling bound").  The reference visits
// every box the infinite line crosses (Bounds3f.h:114-153) and keeps the smallest accepted t
// (Triangle.cu:157-202); the traversal skips a box only when no triangle in it can be accepted
// with t >= 0 (behind the origin) or with t <= t_best (beyond the best hit).  Moller-Trumbore's
// fp32 expressions (tri_test) can put the accepted point o + t d away from the triangle when the
// ray grazes it: with det >= 1e-6 as the only guard (Triangle.cu:17-21), the rounding error of
// the four dot-of-cross products bounds the point's distance from the triangle, per axis, by
//   w <= omega_T + beta_T |o - p0|,   beta_T = 28.3 u |e1| |e2| / 1e-6 (|d| <= 1 + 2^-10) + 1.01 u,
//   omega_T = 2.1 u max(|e1|, |e2|)          (u = 2^-24; derivation in DESIGN.md section 5)
// and |o - p0| <= t |d| + sqrt3 w + diam_T, so on the t range the cull decides about
//   w <= W'_T + (beta_T / (1 - sqrt3 beta_T)) |d| t,   W'_T = (omega_T + beta_T diam_T) / (1 - sqrt3 beta_T).
// A box's margin W is the largest W'_T of the triangles under it (+inf when one has sqrt3 beta_T
// >= 1/2: a triangle so large against the det threshold that nothing near it is ever culled); P
// is the scene's largest (1 + 2^-9) beta_T / (1 - sqrt3 beta_T) (|d| <= 1 + 2^-10).  Triangles in an
// axis plane have a bound without the threshold (cull_plane_b).  With iota = max_a |1 / d_a| (1 + 2^-18), a
// box is skipped when
//   behind:  t1 (1 - 2^-18) + W iota < 0      (only if iota P <= 1: the exit axis is not grazing)
//   beyond:  t0 - W iota > t_best (1 + 2^-18 + iota P)     (closest hit only)
// The 2^-18 factors cover every fp32 rounding in the tests themselves (each <= 4u = 2^-22).
constexpr float kCullSlackF = 1.0f + 1.0f / 262144.0f;  // 1 + 2^-18
constexpr float kCullBehindF = 1.0f - 1.0f / 262144.0f;  // 1 - 2^-18
constexpr float kCullNormMax = 1.0f + 1.0f / 512.0f;  // |d|^2 bound of a ray the culls apply to (|d| <= 1 + 2^-10)
constexpr double kCullU = 5.9604644775390625e-08;      // 2^-24
constexpr double kCullSlackD = 1.0 + 1.0 / 262144.0;
// beta_T of a triangle record (e1, e2 as stored: the values tri_test uses)
MCPT_HD double cull_beta(V3 e1, V3 e2) {
    const double n1 = __builtin_sqrt((double)e1.x * e1.x + (double)e1.y * e1.y + (double)e1.z * e1.z);
    const double n2 = __builtin_sqrt((double)e2.x * e2.x + (double)e2.y * e2.y + (double)e2.z * e2.z);
    return 28.3 * kCullU * n1 * n2 / (double)K_EPSILON * (1.0 + 1.0 / 512.0) + 1.01 * kCullU;
}
// true when no box holding the triangle may be culled (sqrt3 beta_T >= 1/2)
MCPT_HD bool cull_unbounded(double beta) { return !(1.7321 * beta * kCullSlackD < 0.5); }
MCPT_HD double cull_norm(V3 e) { return __builtin_sqrt((double)e.x * e.x + (double)e.y * e.y + (double)e.z * e.z); }
// Axis-plane triangles (e1_a = e2_a = 0 for some axis a: walls, floors, the quads of boxes).  The
// products that carry e1_a or e2_a are exact zeros, and each dot-of-cross error is then a multiple
// of the same factor as the exact value: with G = the in-plane cross product of e1 and e2 and S =
// the sum of its two products' magnitudes, |det - d_a G| <= c |d_a| S and |N - tvec_a G| <= c
// |tvec_a| S (c = 5.0001 u), so det >= d_a (|G| - c S) = d_a G' and |tvec_a| <= |N| / G': the
// quotients d_a / det and tvec_a / det are bounded by 1 / G' and |t| / G' without the 1e-6
// threshold.  Carried through R:
//   w <= omega_T + 1.01 u |tvec| + b_T (|tvec| + |t| |d|),   b_T = 15.0003 u |e1| |e2| / G'
// -- a few u for a right-angled half of a quad, where the general bound is unbounded above an
// edge product of ~0.17.  Returns b_T, or 0 when the triangle does not lie in an axis plane or is
// too thin (G' < G / 2: then the general bound applies).
MCPT_HD double cull_plane_b(V3 e1, V3 e2) {
    double a1, a2, c1, c2;  // the in-plane components of e1 and e2
    if (e1.x == 0.f && e2.x == 0.f) {
        a1 = e1.y; c1 = e1.z; a2 = e2.y; c2 = e2.z;
    } else if (e1.y == 0.f && e2.y == 0.f) {
        a1 = e1.z; c1 = e1.x; a2 = e2.z; c2 = e2.x;
    } else if (e1.z == 0.f && e2.z == 0.f) {
        a1 = e1.x; c1 = e1.y; a2 = e2.x; c2 = e2.y;
    } else {
        return 0.0;
    }
    // float x float products are exact in double; one rounding in the difference and the sum
    const double g = __builtin_fabs(a1 * c2 - c1 * a2) * (1.0 - 1.0 / 1099511627776.0);
    const double sg = (__builtin_fabs(a1 * c2) + __builtin_fabs(c1 * a2)) * (1.0 + 1.0 / 1099511627776.0);
    const double gp = g - 5.0002 * kCullU * sg;
    if (!(gp > 0.5 * g)) return 0.0;
    return 15.0003 * kCullU * cull_norm(e1) * cull_norm(e2) * (1.0 + 1e-12) / gp;
}
// W'_T of a triangle record (+inf when unbounded), in double; far: its contribution to P (the
// coefficient of t_best in the far cut).  General triangles: w <= omega + beta |o - p0| with
// |o - p0| <= t |d| + sqrt3 w + diam (header above).  Axis-plane triangles (cull_plane_b): beta =
// (1.01 u + b)(1 + u), and the extra b |t| |d| adds b to the far coefficient.
MCPT_HD double cull_tri_margin(V3 e1, V3 e2, double* far, bool plane = true) {
    const double b = plane ? cull_plane_b(e1, e2) : 0.0;
    const double beta = b > 0.0 ? (1.01 * kCullU + b) * (1.0 + 1.0 / 8388608.0) : cull_beta(e1, e2);
    *far = 0.0;
    if (cull_unbounded(beta)) return __builtin_huge_val();
    const V3 e3 = v3(e2.x - e1.x, e2.y - e1.y, e2.z - e1.z);
    const double n1 = cull_norm(e1), n2 = cull_norm(e2), n3 = cull_norm(e3) * (1.0 + 1e-7);
    const double diam = n1 > n2 ? (n1 > n3 ? n1 : n3) : (n2 > n3 ? n2 : n3);
    const double omega = 2.1 * kCullU * (n1 > n2 ? n1 : n2);
    const double den = 1.0 - 1.7321 * beta * kCullSlackD;
    // |d| <= 1 + 2^-10 turns the t |d| term into t: the (1 + 2^-9) factor
    *far = (b > 0.0 ? beta + b : beta) * (1.0 + 1.0 / 512.0) / den * kCullSlackD * (1.0 + 1.0 / 1048576.0);
    return (omega + beta * diam * (1.0 + 1e-12)) * kCullSlackD / den;
}
MCPT_HD bool cull_tri_unbounded(V3 e1, V3 e2, bool plane = true) {
    double far;
    return !(cull_tri_margin(e1, e2, &far, plane) < __builtin_huge_val());
}
// double -> float rounded up (twice 2^-20 covers the conversion's rounding)
MCPT_HD float cull_to_float_up(double w) {
    if (!(w < 3.0e38)) return __builtin_huge_valf();
    return (float)(w * (1.0 + 1.0 / 1048576.0)) * (1.0f + 1.0f / 1048576.0f);
}

}  // namespace mcpt
