/*
 * mcpt_oracle.c -- scalar C restatement of the MC-Path-Tracer wavefront path.
 *
 * TEST INFRASTRUCTURE ONLY (see mcpt_oracle.h).  Compiled with
 * -O2 -ffp-contract=off and no fast-math so every float/double operation is a
 * single IEEE-754 rounding, in the order the reference source writes it.
 *
 * Reference paths are relative to /root/reference/CUDA-RayTracer/ unless they
 * start with cuda_math/.  Deviations from the reference (all forced by it being
 * non-reproducible or by third-party arithmetic) are marked DEVIATION:
 *   - RNG: clock64()-seeded lowerbias32 (cuda_math/Random.cu:18-25) replaced by
 *     the keyed counter RNG of SURVEY.md Appendix B (same output mixer).
 *   - Transcendentals: CUDA --use_fast_math sin/cos/asin/acos/atan2/pow are
 *     replaced by the deterministic polynomials below (cephes-derived).
 *   - tex2DLod bilinear/wrap (EnvironmentLight.cu:44; dTexture.cu:265-271) is
 *     restated in software with 8-bit fractional weights; NaN coords -> 0.
 *   - Exact-t closest-hit ties are broken by lower triangle index.
 */
#include "mcpt_oracle.h"
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* constants: cuda_math/dMath.h:8-25 (float, as _CONSTANT float)            */
/* ------------------------------------------------------------------------- */
#define K_EPSILON 1e-6f
#define K_HUGE 1e32f
#define PI_F 3.14159265358979323846f
#define TWO_PI_F 6.28318530717958647692f
#define PI_2_F 1.57079632679489661923f
#define PI_4_F 0.78539816339744830961f
#define ONE_PI_F 0.31830988618379067153f   /* M_1_PI  */
#define ONE_2PI_F 0.15915494309189533576f  /* M_1_2PI */
#define ONE_4PI_F 0.07957747154594766788f  /* M_1_4PI */
#define BRDF_EPS 0.00001f                  /* dMaterial.cu:8 */

static float qnan(void) { return __builtin_nanf(""); }

static int sgnbit(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return (int)(u >> 31);
}

/* IEEE fmaxf/fminf semantics (NaN loses), written out so both backends agree. */
static float fmx(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    return a > b ? a : b;
}

/* ------------------------------------------------------------------------- */
/* Deterministic transcendentals (DEVIATION: replace CUDA fast-math).        */
/* Cephes single-precision algorithms, every step one rounding.              */
/* ------------------------------------------------------------------------- */
#define DP1 0.78515625f
#define DP2 2.4187564849853515625e-4f
#define DP3 3.77489497744594108e-8f
#define FOPI 1.27323954473516f

static float sin_poly(float x, float z) {
    float p = -1.9515295891e-4f * z;
    p = p + 8.3321608736e-3f;
    p = p * z;
    p = p - 1.6666654611e-1f;
    p = p * z;
    p = p * x;
    return p + x;
}
static float cos_poly(float z) {
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

float or_sinf(float xx) {
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

float or_cosf(float xx) {
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

float or_asinf(float xx) {
    float a, x, z;
    int sign, flag;
    if (xx != xx) return xx;
    if (xx > 0.f) { sign = 1; a = xx; } else { sign = -1; a = -xx; }
    if (a > 1.0f) return qnan();
    if (a < 1.0e-4f) {
        z = a;
    } else {
        if (a > 0.5f) { z = 0.5f * (1.0f - a); x = sqrtf(z); flag = 1; }
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

float or_acosf(float x) {
    if (x != x) return x;
    if (x < -1.0f || x > 1.0f) return qnan();
    if (x < -0.5f) return PI_F - 2.0f * or_asinf(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * or_asinf(sqrtf(0.5f * (1.0f - x)));
    return PI_2_F - or_asinf(x);
}

static float or_atanf(float xx) {
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

float or_atan2f(float y, float x) {
    if (x != x || y != y) return x + y;
    if (x == 0.f) {
        if (y > 0.f) return PI_2_F;
        if (y < 0.f) return -PI_2_F;
        return sgnbit(x) ? (sgnbit(y) ? -PI_F : PI_F) : y;
    }
    if (y == 0.f) return x > 0.f ? y : (sgnbit(y) ? -PI_F : PI_F);
    float w;
    if (x < 0.f) w = (y < 0.f) ? -PI_F : PI_F;
    else w = 0.0f;
    return w + or_atanf(y / x);
}

/* pow(x, 5.f) of fresnel_schlick (dMaterial.cu:143), as three products. */
static float pow5(float x) {
    float x2 = x * x;
    float x4 = x2 * x2;
    return x4 * x;
}

/* ------------------------------------------------------------------------- */
/* RNG: lowerbias32 verbatim (cuda_math/Random.cu:5-13); keyed per           */
/* SURVEY.md Appendix B (DEVIATION from clock64 seeding, Random.cu:18-25).   */
/* ------------------------------------------------------------------------- */
uint32_t or_lowerbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0xa812d533u;
    x ^= x >> 15;
    x *= 0xb278e4adu;
    x ^= x >> 17;
    return x;
}
uint64_t or_splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint32_t rng_key(uint64_t seed, uint32_t pixel, uint32_t sample) {
    uint64_t s = or_splitmix64((((uint64_t)pixel << 32) | (uint64_t)sample) ^ seed);
    return (uint32_t)(s ^ (s >> 32));
}
/* rand_float(): rand() * 2^-32 in double, rounded to float (Random.cu:31-35). */
static float rngf(uint32_t key, uint32_t len, uint32_t slot) {
    uint32_t d = or_lowerbias32(key + (len * 16u + slot) * 0x9E3779B9u);
    return (float)((double)d * 0.00000000023283064365386962890625);
}
float or_rand(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t len, uint32_t slot) {
    return rngf(rng_key(seed, pixel, sample), len, slot);
}

/* Draw slots. */
enum {
    SL_GEN_U = 0, SL_GEN_V = 1,
    SL_RR = 0, SL_LIGHT = 1, SL_ENV_U = 2, SL_ENV_V = 3,
    SL_MAT_LOBE = 4, SL_MAT_E0 = 5, SL_MAT_GS = 7,
    SL_CONT_LOBE = 10, SL_CONT_E0 = 11, SL_CONT_GS = 13
};

typedef struct { uint32_t key, len; } rng_t;
static float rnd(const rng_t *r, uint32_t slot) { return rngf(r->key, r->len, slot); }

/* ------------------------------------------------------------------------- */
/* Vec3f (cuda_math/Vector.h): every operator one rounding per component.   */
/* ------------------------------------------------------------------------- */
typedef struct { float x, y, z; } v3;
static v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }  /* :597 */
static v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }  /* :709 */
static v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }  /* :373 */
static v3 vdiv(v3 a, v3 b) { return V(a.x / b.x, a.y / b.y, a.z / b.z); }  /* :485 */
static v3 vscale(v3 v, float s) { return V(s * v.x, s * v.y, s * v.z); }   /* :380 */
static v3 vdivs(v3 v, float s) { return V(v.x / s, v.y / s, v.z / s); }    /* :492 */
static v3 vneg(v3 v) { return V(-v.x, -v.y, -v.z); }
static float dot3(v3 a, v3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); } /* :790 */
static v3 normalize3(v3 v) {                                                /* :1077 */
    float l = sqrtf(dot3(v, v));
    return (l == 0.f) ? v : vdivs(v, l);
}
static v3 cross3(v3 a, v3 b) {                                              /* :1108 */
    return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static v3 reflect3(v3 i, v3 n) {                                            /* :1103 */
    return vsub(i, vscale(vscale(n, 2.f), dot3(n, i)));
}
static v3 mix3(v3 a, v3 b, float t) {                                       /* :1092 */
    return vadd(vscale(a, 1.f - t), vscale(b, t));
}
static v3 ld3(const float *p, int64_t i) { return V(p[3 * i], p[3 * i + 1], p[3 * i + 2]); }

/* Matrix4x4 * Vec4, column-major m[c][r] (cuda_math/Matrix.h:196-204). */
static void mat_vec4(const float *m, const float v[4], float out[4]) {
    for (int r = 0; r < 4; r++)
        out[r] = m[0 * 4 + r] * v[0] + m[1 * 4 + r] * v[1] + m[2 * 4 + r] * v[2] + m[3 * 4 + r] * v[3];
}

/* luminance in double (cuda_math/Vector.h:1123-1126). */
static float luminance(v3 c) {
    return (float)(0.299 * (double)c.x + 0.587 * (double)c.y + 0.114 * (double)c.z);
}

/* gram_schmidt (cuda_math/Vector.h:1128-1139): component-wise division quirk.
 * fixed mode: textbook projection normalize(x - vn (x . vn)). */
static v3 gram_schmidt(v3 v, const rng_t *r, uint32_t slot0, int fixed) {
    float rx = rnd(r, slot0 + 0) * 2.f + -1.f; /* rand_float(-1,1): Random.cu:39-42 */
    float ry = rnd(r, slot0 + 1) * 2.f + -1.f;
    float rz = rnd(r, slot0 + 2) * 2.f + -1.f;
    v3 x = V(rx, ry, rz);
    if (fixed) {
        v3 vn = normalize3(v);
        return normalize3(vsub(x, vscale(vn, dot3(x, vn))));
    }
    float x_dot_v = dot3(x, v);
    v3 v_norm = normalize3(v);
    v3 v_norm_2 = vmul(v_norm, v_norm);
    x = vsub(x, vdiv(vscale(v, x_dot_v), v_norm_2));
    return normalize3(x);
}

/* sample_spherical_map / _direction (cuda_math/Vector.h:1141-1160). */
static void spherical_map(v3 d, float *u, float *v) {
    *u = 0.5f + or_atan2f(d.z, d.x) * ONE_2PI_F;
    *v = 0.5f - or_asinf(d.y) * ONE_PI_F;
}
static v3 spherical_direction(float u, float v) {
    float phi = (float)((double)(2.f * PI_F) * ((double)u - 0.5)); /* fp64 island */
    float theta = PI_F * v;
    float st = or_sinf(theta);
    v3 n;
    n.x = or_cosf(phi) * st;
    n.z = or_sinf(phi) * st;
    n.y = or_cosf(theta);
    return n;
}

/* ------------------------------------------------------------------------- */
/* Environment light (EnvironmentLight.cu:10-109, Helpers.cu:15-30).         */
/* ------------------------------------------------------------------------- */
int32_t or_upper_bound(const float *list, int32_t size, float val) {  /* Helpers.cu:15-30 */
    int32_t middle, left = 0, right = size;
    while (left < right) {
        middle = (right - left) / 2 + left;
        if (val >= list[middle]) left = middle + 1;
        else right = middle;
    }
    if (left < size && list[left] <= val) left++;
    return left;
}

/* DEVIATION: software restatement of tex2DLod<float4> (linear filter, wrap,
 * normalized coords; dTexture.cu:265-271).  Fractions are quantised to 8 bits
 * as the CUDA texture unit does; NaN/huge coordinates are treated as 0. */
static int wrapi(int i, int n) { int r = i % n; return r < 0 ? r + n : r; }
static float q8(float a) { return floorf(a * 256.f + 0.5f) * (1.0f / 256.f); }
static v3 tex_bilinear(const float *tex, int W, int H, float u, float v) {
    if (!(fabsf(u) < 65536.f)) u = 0.f;
    if (!(fabsf(v) < 65536.f)) v = 0.f;
    float x = u * (float)W - 0.5f;
    float y = v * (float)H - 0.5f;
    float fx = floorf(x), fy = floorf(y);
    float ax = q8(x - fx), ay = q8(y - fy);
    int i0 = wrapi((int)fx, W), i1 = wrapi((int)fx + 1, W);
    int j0 = wrapi((int)fy, H), j1 = wrapi((int)fy + 1, H);
    const float *t00 = tex + 4 * ((int64_t)j0 * W + i0), *t10 = tex + 4 * ((int64_t)j0 * W + i1);
    const float *t01 = tex + 4 * ((int64_t)j1 * W + i0), *t11 = tex + 4 * ((int64_t)j1 * W + i1);
    float bx = 1.f - ax, by = 1.f - ay;
    float w00 = bx * by, w10 = ax * by, w01 = bx * ay, w11 = ax * ay;
    float o[3];
    for (int c = 0; c < 3; c++) o[c] = ((w00 * t00[c] + w10 * t10[c]) + w01 * t01[c]) + w11 * t11[c];
    return V(o[0], o[1], o[2]);
}
void or_env_fetch(const or_scene *sc, float u, float v, float *rgb) {
    v3 c = tex_bilinear(sc->env_tex, sc->env_w, sc->env_h, u, v);
    rgb[0] = c.x; rgb[1] = c.y; rgb[2] = c.z;
}

/* light table: index 0 = env light, 1.. = directional (Scene.cu:370-388). */
static int light_is_delta(const or_scene *sc, int id) { (void)sc; return id > 0; }

static v3 env_L(const or_scene *sc, v3 wi) {                    /* EnvironmentLight.cu:34-47 */
    if (sc->env_mode == 0 || sc->env_tex == NULL)
        return vscale(V(sc->env_color[0], sc->env_color[1], sc->env_color[2]), sc->env_ls);
    float u, v;
    spherical_map(wi, &u, &v);
    return tex_bilinear(sc->env_tex, sc->env_w, sc->env_h, u, v);
}
static float env_pdf(const or_scene *sc, v3 wi, int fixed) {    /* EnvironmentLight.cu:65-85 */
    if (sc->env_mode == 0 || sc->env_tex == NULL) return ONE_4PI_F;
    float u, v;
    spherical_map(wi, &u, &v);
    int W = sc->env_w, H = sc->env_h;
    int px, py;
    if (fixed) { /* the sampled cell (int)(u W), (int)(v H), clamped */
        float fx = u * (float)W, fy = v * (float)H;
        px = (fx == fx && fx >= 0.f) ? (fx < (float)(W - 1) ? (int)fx : W - 1) : 0;
        py = (fy == fy && fy >= 0.f) ? (fy < (float)(H - 1) ? (int)fy : H - 1) : 0;
    } else {
        float fx = u * (float)(unsigned)(W - 1), fy = v * (float)(unsigned)(H - 1);
        px = (fx == fx && fx >= 0.f && fx < (float)W) ? (int)fx : 0; /* NaN -> 0 (DEVIATION) */
        py = (fy == fy && fy >= 0.f && fy < (float)H) ? (int)fy : 0;
    }
    float pdf = sc->env_pdf[(int64_t)py * W + px];
    float sin_theta = or_sinf(PI_F * v);
    if (sin_theta == 0.f) return 0.f;
    return pdf * (float)((unsigned)W * (unsigned)H) / (((2.f * sin_theta) * PI_F) * PI_F);
}
static v3 env_dir(const or_scene *sc, const rng_t *r, int fixed) { /* EnvironmentLight.cu:10-33 */
    if (sc->env_mode == 0 || sc->env_tex == NULL) {
        float u = rnd(r, SL_ENV_U);
        float v = rnd(r, SL_ENV_V);
        return spherical_direction(u, v);
    }
    float ex = rnd(r, SL_ENV_U);
    float ey = rnd(r, SL_ENV_V);
    int W = sc->env_w, H = sc->env_h;
    int y = (int)((float)or_upper_bound(sc->env_marginal_y, H, ey) - 1.f);
    if (y < 0) y = 0; /* unreachable: marginal_y[0] == 0; reference reads row -1 */
    int x = (int)((float)or_upper_bound(sc->env_conds_y + (int64_t)y * W, W, ex) - 1.f);
    if (fixed) { /* clamped indices, cell centres */
        y = y > H - 1 ? H - 1 : y;
        x = x < 0 ? 0 : (x > W - 1 ? W - 1 : x);
        return spherical_direction(((float)x + 0.5f) / (float)W, ((float)y + 0.5f) / (float)H);
    }
    float u = (float)x / (float)W;
    float v = (float)y / (float)H;
    return spherical_direction(u, v);
}
void or_env_dir(const or_scene *sc, float ex, float ey, float *wi) {
    int W = sc->env_w, H = sc->env_h;
    int y = (int)((float)or_upper_bound(sc->env_marginal_y, H, ey) - 1.f);
    if (y < 0) y = 0;
    int x = (int)((float)or_upper_bound(sc->env_conds_y + (int64_t)y * W, W, ex) - 1.f);
    v3 d = spherical_direction((float)x / (float)W, (float)y / (float)H);
    wi[0] = d.x; wi[1] = d.y; wi[2] = d.z;
}
float or_env_pdf(const or_scene *sc, float dx, float dy, float dz) { return env_pdf(sc, V(dx, dy, dz), 0); }

static void light_dir(const or_scene *sc, int id, const rng_t *r, v3 *wi, int fixed) {
    if (id == 0) *wi = env_dir(sc, r, fixed);
    else *wi = ld3(sc->dir_params + 7 * (id - 1), 0);           /* DirectionalLight.cu:8-11 */
}
static v3 light_L(const or_scene *sc, int id, v3 wi) {
    if (id == 0) return env_L(sc, wi);
    const float *p = sc->dir_params + 7 * (id - 1);             /* DirectionalLight.cu:34 */
    return vscale(V(p[3], p[4], p[5]), p[6]);
}
static float light_pdf(const or_scene *sc, int id, v3 wi, int fixed) {
    if (id == 0) return env_pdf(sc, wi, fixed);
    return 1.f;                                                 /* DirectionalLight.cu:40-43 */
}

/* Env table build (light_initialization_kernels.cu:3-112), serial order. */
void or_env_build(int32_t W, int32_t H, const float *tex, float *marginal_y, float *marginal_p,
                  float *conds_y, float *pdf, float *out_denom) {
    float denom = 0.0f;                                         /* :3-25 */
    for (int j = 0; j < H; j++) {
        float v = (float)j / (float)H;
        float s = or_sinf(PI_F * v);
        for (int i = 0; i < W; i++) {
            float u = (float)i / (float)W;
            float lum = luminance(tex_bilinear(tex, W, H, u, v));
            denom += lum * s;
        }
    }
    for (int j = 0; j < H; j++) {                               /* :27-55 */
        float v = (float)j / (float)H;
        double st = (double)(or_sinf(PI_F * v) / denom);
        float mp = 0.f;
        for (int i = 0; i < W; i++) {
            float u = (float)i / (float)W;
            double lum = (double)luminance(tex_bilinear(tex, W, H, u, v));
            mp = (float)((double)mp + lum * st);
        }
        marginal_p[j] = mp;
        marginal_y[j] = (j != 0) ? mp + marginal_y[j - 1] : mp;
    }
    for (int y = 0; y < H; y++) {                               /* :56-84 */
        float v = (float)y / (float)H;
        float st = or_sinf(PI_F * v);
        float val = st / (denom * marginal_p[y]);
        float *row = conds_y + (int64_t)y * W;
        for (int x = 0; x < W; x++) {
            float u = (float)x / (float)W;
            float lum = luminance(tex_bilinear(tex, W, H, u, v));
            row[x] = lum * val;
            if (x != 0) row[x] = row[x] + row[x - 1];
        }
    }
    for (int y = 0; y < H; y++) {                               /* :85-112 */
        float v = (float)y / (float)H;
        float st = or_sinf(PI_F * v);
        for (int x = 0; x < W; x++) {
            float u = (float)x / (float)W;
            float lum = luminance(tex_bilinear(tex, W, H, u, v));
            pdf[(int64_t)y * W + x] = (lum * st) / denom;
        }
    }
    if (out_denom) *out_denom = denom;
}

/* ------------------------------------------------------------------------- */
/* BRDF (dMaterial.cu).  Material factors only: texture lookups are computed */
/* and discarded in the reference (dMaterial.cu:26,54,81,114).                */
/* ------------------------------------------------------------------------- */
typedef struct { v3 base, fresnel; float rough, metal; } mat_t;
static mat_t load_mat(const or_scene *sc, int id) {
    const float *p = sc->mat_params + 8 * id;
    mat_t m;
    m.base = V(p[0], p[1], p[2]);
    m.fresnel = V(p[3], p[4], p[5]);
    m.rough = fmx(p[6], BRDF_EPS);  /* get_roughness: fmax(factor, eps) :54 */
    m.metal = p[7];
    return m;
}

float or_power_heuristic(float fPdf, float gPdf) {              /* :134-139 */
    float f = 1.0f * fPdf, g = 1.0f * gPdf;
    return (f * f) / (f * f + g * g);
}
static v3 fresnel_schlick(v3 f0, v3 v, v3 h) {                 /* :141-144 */
    float v_dot_h = fmx(dot3(v, h), 0.f);
    return vadd(f0, vscale(vsub(V(1.f, 1.f, 1.f), f0), pow5(1.f - v_dot_h)));
}
static float ndf_ggx_tr(v3 n, v3 h, float r) {                  /* :150-161 */
    float a = r * r;
    float a2 = a * a;
    float n_dot_h = fmx(dot3(n, h), BRDF_EPS);
    float n_dot_h_2 = n_dot_h * n_dot_h;
    float denom = fmx(n_dot_h_2 * (a2 - 1.f) + 1.f, BRDF_EPS);
    return a2 / ((PI_F * denom) * denom);
}
static float g1_schlick_ggx(v3 v, v3 n, float r) {              /* :205-213 */
    float a = r * r;
    float k = a / 2.f;
    float n_dot_v = fmx(dot3(n, v), BRDF_EPS);
    return n_dot_v / fmx(n_dot_v * (1.f - k) + k, BRDF_EPS);
}
static v3 diff_get_wi(v3 N, const rng_t *r, uint32_t s0, int fixed) {       /* :232-254 */
    float e0 = rnd(r, s0 + 0);
    float e1 = rnd(r, s0 + 1);
    float sinTheta = sqrtf(1.f - e0 * e0);
    float phi = (2.f * PI_F) * e1;
    float x = sinTheta * or_cosf(phi);
    float z = sinTheta * or_sinf(phi);
    v3 T = gram_schmidt(N, r, s0 + 2, fixed);
    v3 B = normalize3(cross3(N, T));
    return normalize3(vadd(vadd(vscale(T, x), vscale(N, e0)), vscale(B, z)));
}
static v3 diff_get_f(const mat_t *m, v3 n, v3 wi, v3 wo) {      /* :259-276 */
    float n_dot_wi = fmx(dot3(n, wi), BRDF_EPS);
    v3 f0 = mix3(m->fresnel, m->base, m->metal);
    v3 wh = normalize3(vadd(wo, wi));
    v3 F = fresnel_schlick(f0, wh, wo);
    v3 kD = vsub(V(1.f, 1.f, 1.f), F);
    kD = vscale(kD, 1.f - m->metal);
    return vscale(vscale(vmul(kD, m->base), n_dot_wi), ONE_PI_F);
}
static v3 spec_get_wi(const mat_t *m, v3 N, v3 wo, const rng_t *r, uint32_t s0, int fixed) { /* :278-307 */
    float rr = m->rough;
    float a2 = ((rr * rr) * rr) * rr;
    float e0 = rnd(r, s0 + 0);
    float e1 = rnd(r, s0 + 1);
    float theta = or_acosf(sqrtf((1.f - e0) / (e0 * (a2 - 1.f) + 1.f)));
    float phi = TWO_PI_F * e1;
    float st = or_sinf(theta);
    v3 h = V(st * or_cosf(phi), or_cosf(theta), st * or_sinf(phi));
    v3 T = gram_schmidt(N, r, s0 + 2, fixed);
    v3 B = normalize3(cross3(N, T));
    v3 smp = normalize3(vadd(vadd(vscale(T, h.x), vscale(N, h.y)), vscale(B, h.z)));
    return normalize3(reflect3(vneg(wo), smp));
}
static float spec_get_pdf(const mat_t *m, v3 n, v3 wi, v3 wo) { /* :308-321 */
    v3 wh = normalize3(vadd(wo, wi));
    float wh_dot_n = fmx(dot3(wh, n), BRDF_EPS);
    float wo_dot_wh = fmx(dot3(wo, wh), BRDF_EPS);
    float D = ndf_ggx_tr(n, wh, m->rough);
    return (D * wh_dot_n) / fmx(4.f * wo_dot_wh, BRDF_EPS);
}
static v3 spec_get_f(const mat_t *m, v3 n, v3 wi, v3 wo) {      /* :322-343 */
    v3 f0 = mix3(m->fresnel, m->base, m->metal);
    v3 wh = normalize3(vadd(wo, wi));
    float n_dot_wi = fmx(dot3(n, wi), BRDF_EPS);
    float n_dot_wo = fmx(dot3(n, wo), BRDF_EPS);
    float D = ndf_ggx_tr(n, wh, m->rough);
    float G = g1_schlick_ggx(wi, n, m->rough) * g1_schlick_ggx(wo, n, m->rough);
    v3 F = fresnel_schlick(f0, wh, wo);
    v3 L = vscale(vscale(F, D * G), n_dot_wi);
    return vdivs(L, fmx((4.f * n_dot_wo) * n_dot_wi, BRDF_EPS));
}
static float diff_get_pdf(void) { return ONE_2PI_F; }            /* :255-258 */

void or_brdf_eval(const float *params, const float *n, const float *wi, const float *wo, float *out) {
    mat_t m;
    m.base = V(params[0], params[1], params[2]);
    m.fresnel = V(params[3], params[4], params[5]);
    m.rough = fmx(params[6], BRDF_EPS);
    m.metal = params[7];
    v3 N = V(n[0], n[1], n[2]), WI = V(wi[0], wi[1], wi[2]), WO = V(wo[0], wo[1], wo[2]);
    v3 fs = spec_get_f(&m, N, WI, WO), fd = diff_get_f(&m, N, WI, WO);
    out[0] = fs.x; out[1] = fs.y; out[2] = fs.z;
    out[3] = fd.x; out[4] = fd.y; out[5] = fd.z;
    out[6] = spec_get_pdf(&m, N, WI, WO);
    out[7] = diff_get_pdf();
}

/* ------------------------------------------------------------------------- */
/* Geometry: Triangle.cu:9-117, Bounds3f.h:121-153, Triangle.cu:144-243.     */
/* ------------------------------------------------------------------------- */
typedef struct { v3 o, d; } ray_t;

/* dTriangle::intersect with TEST_CULL (Triangle.cu:9-65); fp64 det island. */
static int tri_intersect(const or_scene *sc, int id, const ray_t *ray, float *uo, float *vo, float *to) {
    v3 p0 = ld3(sc->v0, id), p1 = ld3(sc->v1, id), p2 = ld3(sc->v2, id);
    v3 e1 = vsub(p1, p0), e2 = vsub(p2, p0);
    v3 pvec = cross3(ray->d, e2);
    double det = (double)dot3(e1, pvec);
    if (det < (double)K_EPSILON) return 0;
    v3 tvec = vsub(ray->o, p0);
    float u = dot3(tvec, pvec);
    if ((double)u < 0.0 || (double)u > det) return 0;
    v3 qvec = cross3(tvec, e1);
    float v = dot3(ray->d, qvec);
    if ((double)v < 0.0 || (double)(u + v) > det) return 0;
    float t = dot3(e2, qvec);
    double inv_det = 1.0 / det;
    *uo = (float)((double)u * inv_det);
    *vo = (float)((double)v * inv_det);
    *to = (float)((double)t * inv_det);
    return 1;
}

/* Bounds3f::hit(ray, invDir, dirIsNeg) (Bounds3f.h:121-153): no [0,tmax]
 * clamp, NaN compares false so NaN slabs pass. */
static int box_hit(const or_scene *sc, int n, const ray_t *ray, v3 inv, const int neg[3]) {
    const float *mn = sc->bmin + 3 * (int64_t)n, *mx = sc->bmax + 3 * (int64_t)n;
    float bx0 = neg[0] ? mx[0] : mn[0], bx1 = neg[0] ? mn[0] : mx[0];
    float by0 = neg[1] ? mx[1] : mn[1], by1 = neg[1] ? mn[1] : mx[1];
    float bz0 = neg[2] ? mx[2] : mn[2], bz1 = neg[2] ? mn[2] : mx[2];
    float tmin = (bx0 - ray->o.x) * inv.x;
    float tmax = (bx1 - ray->o.x) * inv.x;
    float tymin = (by0 - ray->o.y) * inv.y;
    float tymax = (by1 - ray->o.y) * inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (bz0 - ray->o.z) * inv.z;
    float tzmax = (bz1 - ray->o.z) * inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    return 1;
}

typedef struct { uint64_t nodes, tris; } trav_stats;

/* DEVIATION (tree independence): in a leaf with several triangles (and in the brute-force mode)
 * a triangle's hit counts only if the line also passes its own bounding box (the vertex union,
 * g_init_BVH_triangle_info, mesh_initialization_kernels.cu:63-83) under the same slab test --
 * exactly the leaf test of BVHAccel's one-triangle leaves, so results do not depend on how a
 * builder grouped triangles.  traversal == 2 is the literal reference rule instead (every leaf
 * primitive tested, no own-box check, exact-t ties to the first visited, Triangle.cu:170-179):
 * tests/test_oracle.py::test_literal_leaf_rule_deviation counts the pixels it changes. */
static int own_box_hit(const or_scene *sc, int id, const ray_t *ray, v3 inv, const int neg[3]) {
    const float *a = sc->v0 + 3 * (int64_t)id, *b = sc->v1 + 3 * (int64_t)id, *c = sc->v2 + 3 * (int64_t)id;
    float mn[3], mx[3];
    for (int k = 0; k < 3; k++) {
        mn[k] = fminf(fminf(a[k], b[k]), c[k]);
        mx[k] = fmaxf(fmaxf(a[k], b[k]), c[k]);
    }
    float bx0 = neg[0] ? mx[0] : mn[0], bx1 = neg[0] ? mn[0] : mx[0];
    float by0 = neg[1] ? mx[1] : mn[1], by1 = neg[1] ? mn[1] : mx[1];
    float bz0 = neg[2] ? mx[2] : mn[2], bz1 = neg[2] ? mn[2] : mx[2];
    float tmin = (bx0 - ray->o.x) * inv.x;
    float tmax = (bx1 - ray->o.x) * inv.x;
    float tymin = (by0 - ray->o.y) * inv.y;
    float tymax = (by1 - ray->o.y) * inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (bz0 - ray->o.z) * inv.z;
    float tzmax = (bz1 - ray->o.z) * inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    return 1;
}
static int tri_key(const or_scene *sc, int id) { return sc->tri_id ? sc->tri_id[id] : id; }

/* intersect() (Triangle.cu:144-203).  Returns winning triangle or -1 and its t.
 * DEVIATION: exact-t ties go to the lower triangle id (order independent). */
static int closest_hit(const or_scene *sc, const ray_t *ray, int traversal, float *tbest, trav_stats *st) {
    float tmin = K_HUGE;
    int best = -1;
    v3 inv = V(1.f / ray->d.x, 1.f / ray->d.y, 1.f / ray->d.z);
    int neg[3] = {inv.x < 0, inv.y < 0, inv.z < 0};
    if (traversal == 1) {
        for (int id = 0; id < sc->ntri; id++) {
            float u, v, t;
            st->tris++;
            if (tri_intersect(sc, id, ray, &u, &v, &t) && !(t < 0.f)) {
                if ((t < tmin || (t == tmin && best >= 0 && tri_key(sc, id) < tri_key(sc, best))) &&
                    own_box_hit(sc, id, ray, inv, neg)) { tmin = t; best = id; }
            }
        }
        *tbest = tmin;
        return best;
    }
    if (sc->nnodes <= 0) { *tbest = tmin; return -1; }
    int stack[128];
    int sp = 0, cur = 0;
    for (;;) {
        st->nodes++;
        if (box_hit(sc, cur, ray, inv, neg)) {
            int np = sc->nprims[cur];
            if (np > 0) {
                for (int i = 0; i < np; ++i) {
                    int id = sc->offset[cur] + i;
                    float u, v, t;
                    st->tris++;
                    if (tri_intersect(sc, id, ray, &u, &v, &t) && !(t < 0.f)) {
                        if (traversal == 2) {  /* literal reference leaf rule: first visited wins */
                            if (t < tmin) { tmin = t; best = id; }
                        } else if ((t < tmin || (t == tmin && best >= 0 && tri_key(sc, id) < tri_key(sc, best))) &&
                                   (np == 1 || own_box_hit(sc, id, ray, inv, neg))) { tmin = t; best = id; }
                    }
                }
                if (sp == 0) break;
                cur = stack[--sp];
            } else {
                if (neg[sc->axis[cur]]) { stack[sp++] = cur + 1; cur = sc->offset[cur]; }
                else { stack[sp++] = sc->offset[cur]; cur = cur + 1; }
            }
        } else {
            if (sp == 0) break;
            cur = stack[--sp];
        }
    }
    *tbest = tmin;
    return best;
}

/* intersect_shadows (Triangle.cu:204-243) with tmin = K_HUGE (Light.cu:12-16). */
static int any_hit(const or_scene *sc, const ray_t *ray, int traversal, trav_stats *st) {
    v3 inv = V(1 / ray->d.x, 1 / ray->d.y, 1 / ray->d.z);
    int neg[3] = {inv.x < 0, inv.y < 0, inv.z < 0};
    if (traversal == 1) {
        for (int id = 0; id < sc->ntri; id++) {
            float u, v, t;
            st->tris++;
            if (tri_intersect(sc, id, ray, &u, &v, &t) && !(t < 0.f) && t < K_HUGE && own_box_hit(sc, id, ray, inv, neg))
                return 1;
        }
        return 0;
    }
    if (sc->nnodes <= 0) return 0;
    int stack[128];
    int sp = 0, cur = 0;
    for (;;) {
        st->nodes++;
        if (box_hit(sc, cur, ray, inv, neg)) {
            int np = sc->nprims[cur];
            if (np > 0) {
                for (int i = 0; i < np; ++i) {
                    int id = sc->offset[cur] + i;
                    float u, v, t;
                    st->tris++;
                    if (tri_intersect(sc, id, ray, &u, &v, &t) && !(t < 0.f) && t < K_HUGE &&
                        (traversal == 2 || np == 1 || own_box_hit(sc, id, ray, inv, neg)))
                        return 1;
                }
                if (sp == 0) break;
                cur = stack[--sp];
            } else {
                if (neg[sc->axis[cur]]) { stack[sp++] = cur + 1; cur = sc->offset[cur]; }
                else { stack[sp++] = sc->offset[cur]; cur = cur + 1; }
            }
        } else {
            if (sp == 0) break;
            cur = stack[--sp];
        }
    }
    return 0;
}

typedef struct {
    v3 position, normal;
    float t;
    int was_found, mat;
} isect_t;

/* dTriangle::hit (Triangle.cu:66-93) for the winner: interpolated normal,
 * normalised twice (second time by the identity transform, :82). */
static isect_t make_isect(const or_scene *sc, const ray_t *ray, int id, float tmin) {
    isect_t is;
    memset(&is, 0, sizeof(is));
    is.t = tmin;
    is.mat = -1;
    if (id < 0) return is;
    float u, v, t;
    tri_intersect(sc, id, ray, &u, &v, &t);
    v3 n0 = ld3(sc->n0, id), n1 = ld3(sc->n1, id), n2 = ld3(sc->n2, id);
    float w = (1.f - u) - v;
    v3 n = vadd(vadd(vscale(n1, u), vscale(n2, v)), vscale(n0, w));
    n = normalize3(n);
    is.normal = normalize3(n);
    is.position = vadd(ray->o, vscale(ray->d, t));
    is.was_found = 1;
    is.mat = sc->mat[id];
    return is;
}

void or_trace_closest(const or_scene *sc, int32_t n, const float *ro, const float *rd, int32_t traversal,
                      float *pos_t, float *nrm_mat, int32_t *tri) {
    for (int32_t i = 0; i < n; i++) {
        ray_t r;
        r.o = ld3(ro, i);
        r.d = ld3(rd, i);
        trav_stats st = {0, 0};
        float tb;
        int id = closest_hit(sc, &r, traversal, &tb, &st);
        isect_t is = make_isect(sc, &r, id, tb);
        pos_t[4 * i + 0] = is.position.x; pos_t[4 * i + 1] = is.position.y;
        pos_t[4 * i + 2] = is.position.z; pos_t[4 * i + 3] = is.t;
        nrm_mat[4 * i + 0] = is.normal.x; nrm_mat[4 * i + 1] = is.normal.y;
        nrm_mat[4 * i + 2] = is.normal.z; nrm_mat[4 * i + 3] = (float)is.mat;
        tri[i] = id >= 0 ? tri_key(sc, id) : -1;
    }
}
void or_trace_any(const or_scene *sc, int32_t n, const float *ro, const float *rd, int32_t traversal,
                  uint8_t *visible) {
    for (int32_t i = 0; i < n; i++) {
        ray_t r;
        r.o = ld3(ro, i);
        r.d = ld3(rd, i);
        trav_stats st = {0, 0};
        visible[i] = (uint8_t)!any_hit(sc, &r, traversal, &st);
    }
}

/* ------------------------------------------------------------------------- */
/* Camera ray generation (Camera.cu:18-45, Sample.cu:129-149).               */
/* ------------------------------------------------------------------------- */
static void concentric_disk(const rng_t *r, float *dx, float *dy) {
    float ux = rnd(r, SL_GEN_U), uy = rnd(r, SL_GEN_V);
    float ox = 2.f * ux - 1.f, oy = 2.f * uy - 1.f;
    if (ox == 0.f && oy == 0.f) { *dx = 0.f; *dy = 0.f; return; }
    float theta, rr;
    if (fabsf(ox) > fabsf(oy)) { rr = ox; theta = PI_4_F * (oy / ox); }
    else { rr = oy; theta = PI_2_F - PI_4_F * (ox / oy); }
    *dx = rr * or_cosf(theta);
    *dy = rr * or_sinf(theta);
}
static ray_t gen_ray(const or_camera *cam, int W, int H, int xi, int yi, const rng_t *r) {
    float x = (float)xi, y = (float)yi;
    float px = (float)(2.f * (((double)x + 0.5) / (double)(float)W) - 1.f); /* fp64 island :21-22 */
    float py = (float)(1.f - 2.f * (((double)y + 0.5) / (double)(float)H));
    float vn[4] = {px, py, -1.f, 1.f}, vf[4] = {px, py, 1.f, 1.f}, an[4], af[4];
    mat_vec4(cam->inv_view_proj, vn, an);
    mat_vec4(cam->inv_view_proj, vf, af);
    v3 pNear = vdivs(V(an[0], an[1], an[2]), an[3]);
    v3 pFar = vdivs(V(af[0], af[1], af[2]), af[3]);
    ray_t ray;
    ray.o = pNear;
    ray.d = normalize3(vsub(pFar, pNear));
    if (cam->lens_radius > 0.f) {
        v3 pFocal = vadd(ray.o, vscale(ray.d, cam->focal));
        float lx, ly;
        concentric_disk(r, &lx, &ly);
        lx = lx * cam->lens_radius;
        ly = ly * cam->lens_radius;
        float vl[4] = {lx, ly, 0.f, 1.f}, al[4];
        mat_vec4(cam->inv_view, vl, al);
        v3 pLens = vdivs(V(al[0], al[1], al[2]), al[3]);
        ray.o = pLens;
        ray.d = normalize3(vsub(pFocal, ray.o));
    }
    return ray;
}
void or_gen_ray(const or_camera *cam, int32_t W, int32_t H, int32_t x, int32_t y, uint64_t seed,
                uint32_t pixel, uint32_t sample, float *o, float *d) {
    rng_t r = {rng_key(seed, pixel, sample), 0};
    ray_t ray = gen_ray(cam, W, H, x, y, &r);
    o[0] = ray.o.x; o[1] = ray.o.y; o[2] = ray.o.z;
    d[0] = ray.d.x; d[1] = ray.d.y; d[2] = ray.d.z;
}

/* ------------------------------------------------------------------------- */
/* Wavefront stages (wavefront_kernels.cu:90-375), Paths (Wavefront.cuh:8-26) */
/* ------------------------------------------------------------------------- */
typedef struct {
    v3 f_light, f_brdf, f_sample, Li_light, Li_brdf, beta;
    float pdf_light[2], pdf_brdf[2], pdf_sample;
    ray_t ray, ray_light;
    uint32_t len, light_id;
    isect_t isect;
    uint8_t dead, visible;
} path_t;

typedef struct {
    const or_scene *sc;
    const or_camera *cam;
    const or_config *cfg;
    int W, H;
    path_t *paths;
    float *Ld;
    uint32_t *samples;
} ctx_t;

typedef struct {
    int32_t *newq, *extq, *shq, *matq;
    int nnew, next, nsh, nmat;
    uint64_t cnt[6];
} queues_t;

static rng_t path_rng(const ctx_t *c, uint32_t pid, uint32_t len) {
    rng_t r;
    r.key = rng_key(c->cfg->seed, pid, c->samples[pid]);
    r.len = len;
    return r;
}

/* wf_logic's MIS combination of the previous vertex's two samples (wavefront_kernels.cu:165-180)
 * as four terms: the light-sample and BRDF-sample contributions f*Li*w/pdf and their conditions
 * (w > 0 && pdf > 0), evaluated exactly as the reference evaluates them, plus the throughput
 * factor f_sample / pdf_sample (:187) and its zero test (:182-185).  The product's material stage
 * stores these terms (nee0 / nee1 / flags, mcpt_path_view) and its logic stage sums them; the
 * stage harness (or_stage_*) is checked field by field against the same functions. */
typedef struct {
    v3 cL, cB, ratio;
    int condL, condB, hasvis, fzero;
} mis_t;

static mis_t mis_terms(const path_t *p, int hasvis) {
    mis_t m;
    float w = or_power_heuristic(p->pdf_light[0], p->pdf_brdf[1]);
    m.cL = vdivs(vscale(vmul(p->f_light, p->Li_light), w), p->pdf_light[0]);
    m.condL = w > 0.f && p->pdf_light[0] > 0.f;
    w = or_power_heuristic(p->pdf_brdf[0], p->pdf_light[1]);
    m.cB = vdivs(vscale(vmul(p->f_brdf, p->Li_brdf), w), p->pdf_brdf[0]);
    m.condB = w > 0.f && p->pdf_brdf[0] > 0.f;
    m.hasvis = hasvis;
    m.ratio = vdivs(p->f_sample, p->pdf_sample);
    m.fzero = (p->f_sample.x == 0.f && p->f_sample.y == 0.f && p->f_sample.z == 0.f) || p->pdf_sample == 0.f;
    return m;
}

/* :168-179.  vl / vb: light-sample / BRDF-sample visibility.  An occluded BRDF sample (or a
 * delta light's absent one) adds +0: the reference's f_brdf = Li_brdf = 0 with pdfs 1 (:311). */
static v3 mis_accumulate(const mis_t *m, int vl, int vb) {
    v3 acc = V(0.f, 0.f, 0.f);
    if (m->condL && vl) acc = vadd(acc, m->cL);
    if (m->hasvis && vb) {
        if (m->condB) acc = vadd(acc, m->cB);
    } else {
        acc = vadd(acc, V(0.f, 0.f, 0.f));
    }
    return acc;
}

/* wf_logic (wavefront_kernels.cu:124-205) for one live path: background at len 1, termination,
 * the MIS sum, throughput update and Russian roulette.  Updates *beta and the film Ld; returns
 * 1 if the path continues. */
static int logic_core(const or_scene *sc, const or_config *cfg, const rng_t *r, uint32_t len, int found, v3 ray_d,
                      v3 *beta_io, const mis_t *m, int vl, int vb, float *Ld) {
    int nmb_lights = 1 + sc->ndir;
    int D = cfg->max_depth;
    v3 beta = *beta_io;
    int terminate = 0;
    if (len == 1 && found) {                                   /* :131-133: Vec3f(0)*beta */
        v3 z = vmul(V(0.f, 0.f, 0.f), beta);
        Ld[0] = Ld[0] + z.x; Ld[1] = Ld[1] + z.y; Ld[2] = Ld[2] + z.z;
    }
    if (len == 1 && !found) {                                  /* :134-139 */
        int nbg = cfg->fixed ? 1 : nmb_lights;                  /* fixed: background once */
        for (int i = 0; i < nbg; i++) {
            v3 Le = vmul(env_L(sc, ray_d), beta);
            Ld[0] = Ld[0] + Le.x; Ld[1] = Ld[1] + Le.y; Ld[2] = Ld[2] + Le.z;
        }
    }
    if (len > (uint32_t)D || !found) terminate = 1;            /* :142-146 */
    if (len > (uint32_t)D) return 0;                           /* :148 */
    if (len > 1) {                                             /* :150-197 */
        v3 acc = mis_accumulate(m, vl, vb);
        v3 add = vmul(acc, beta);
        Ld[0] = Ld[0] + add.x; Ld[1] = Ld[1] + add.y; Ld[2] = Ld[2] + add.z;
        if (m->fzero) return 0;
        *beta_io = vmul(*beta_io, m->ratio);
        if (len > (uint32_t)cfg->rr_depth) {
            if (cfg->fixed) { /* fixed: q from the updated throughput, survivors reweighted */
                float qq = fmx(0.05f, 1.f - beta_io->y);
                if (rnd(r, SL_RR) < qq) return 0;
                *beta_io = vdivs(*beta_io, 1.f - qq);
            } else {
                float qq = fmx(0.05f, 1.f - beta.y);
                if (rnd(r, SL_RR) < qq) return 0;
                /* beta /= 1-q applies to a local and is never stored (:195) */
            }
        }
    }
    return !terminate;
}

/* :207-213: the light choice and the shadow ray of a continuing path. */
static void pick_light(const or_scene *sc, int fixed, const rng_t *r, path_t *p) {
    int nmb_lights = 1 + sc->ndir;
    int l_id = (int)(rnd(r, SL_LIGHT) * (float)(nmb_lights - 0) + (float)0); /* rand_int :48-51 */
    p->light_id = (uint32_t)((l_id == nmb_lights) ? 0 : l_id);
    v3 ldir;
    light_dir(sc, (int)p->light_id, r, &ldir, fixed);
    p->ray_light.o = vadd(p->isect.position, vscale(p->isect.normal, 0.01f));
    p->ray_light.d = ldir;
}

/* wf_logic (wavefront_kernels.cu:90-223) for one pixel. */
static void wf_logic(ctx_t *c, queues_t *q, int x, int y) {
    const or_scene *sc = c->sc;
    int W = c->W;
    if (x >= W - 1 || y >= c->H - 1) return;                   /* :110 */
    uint32_t pid = (uint32_t)y * (uint32_t)W + (uint32_t)x;
    path_t *p = &c->paths[pid];
    int spp = c->cfg->spp;
    float *Ld = c->Ld + 3 * (int64_t)pid;
    if (!p->dead && c->samples[pid] < (uint32_t)spp) {        /* :124 */
        rng_t r = path_rng(c, pid, p->len);
        /* the previous vertex's terms; an occluded BRDF sample already zeroed f_brdf (:311) */
        mis_t m = mis_terms(p, 1);
        if (!logic_core(sc, c->cfg, &r, p->len, p->isect.was_found, p->ray.d, &p->beta, &m, p->visible, 1, Ld)) {
            p->dead = 1;                                       /* :199-204 */
            c->samples[pid]++;
        } else {
            pick_light(sc, c->cfg->fixed, &r, p);
            q->matq[q->nmat++] = (int32_t)pid;
        }
    }
    if (p->dead && c->samples[pid] < (uint32_t)spp)            /* :219-222 */
        q->newq[q->nnew++] = (int32_t)pid;
}

/* wf_generate (wavefront_kernels.cu:225-251). */
static void wf_generate(ctx_t *c, queues_t *q, uint32_t id) {
    int x = (int)(id % (uint32_t)c->W), y = (int)((id / (uint32_t)c->W) % (uint32_t)c->H);
    path_t *p = &c->paths[id];
    rng_t r = path_rng(c, id, 0);
    p->dead = 0;
    p->ray = gen_ray(c->cam, c->W, c->H, x, y, &r);
    p->len = 0;
    p->beta = V(1.f, 1.f, 1.f);
    q->extq[q->next++] = (int32_t)id;
}

/* wf_extend (wavefront_kernels.cu:253-272). */
static void wf_extend(ctx_t *c, queues_t *q, uint32_t id) {
    path_t *p = &c->paths[id];
    trav_stats st = {0, 0};
    float tb;
    int tri = closest_hit(c->sc, &p->ray, c->cfg->traversal, &tb, &st);
    p->isect = make_isect(c->sc, &p->ray, tri, tb);
    p->len++;
    q->cnt[4] += st.nodes;
    q->cnt[5] += st.tris;
}

/* wf_shadow (wavefront_kernels.cu:274-293). */
static void wf_shadow(ctx_t *c, queues_t *q, uint32_t id) {
    path_t *p = &c->paths[id];
    trav_stats st = {0, 0};
    p->visible = (uint8_t)!any_hit(c->sc, &p->ray_light, c->cfg->traversal, &st);
    q->cnt[4] += st.nodes;
    q->cnt[5] += st.tris;
}

/* The BRDF sample of wf_mat_mix (:331-345) as if it were visible: its direction, visibility ray
 * and terms.  has = 0 for a delta light (no BRDF sample is drawn). */
typedef struct {
    int has;
    ray_t vis;
    v3 f_brdf, Li_brdf;
    float pdf_brdf0, pdf_light1;
} brdf_sample_t;

/* wf_mat_mix (wavefront_kernels.cu:295-375) without the inline visibility trace: writes the light
 * sample, the continuation and the next ray into p (BRDF-sample fields at the reference's
 * occluded defaults f = Li = 0, pdfs 1, :311) and returns the BRDF sample in *bs. */
static void mat_mix_core(const or_scene *sc, int fixed, const rng_t *r, path_t *p, brdf_sample_t *bs) {
    v3 f_light, Li_light;
    float pdf_light[2] = {1.f, 1.f}, pdf_brdf[2] = {1.f, 1.f};
    const isect_t *is = &p->isect;
    int light_id = (int)p->light_id;
    v3 light_wi = p->ray_light.d;
    v3 wo = vneg(p->ray.d);
    mat_t m = load_mat(sc, is->mat);
    v3 n = is->normal;                                         /* get_normal :83-115 */
    int delta = light_is_delta(sc, light_id);

    f_light = vadd(spec_get_f(&m, n, light_wi, wo), diff_get_f(&m, n, light_wi, wo)); /* :326 */
    Li_light = light_L(sc, light_id, light_wi);
    float sel = fixed ? 1.f / (float)(1 + sc->ndir) : 1.f;   /* fixed: light-selection pdf 1/N */
    pdf_light[0] = light_pdf(sc, light_id, light_wi, fixed);
    if (fixed) pdf_light[0] = pdf_light[0] * sel;
    pdf_brdf[1] = !delta ? (diff_get_pdf() + spec_get_pdf(&m, n, light_wi, wo)) * 0.5f
                         : (fixed ? 0.f : 1.f);               /* fixed: delta-light MIS weight 1 */
    bs->has = !delta;
    if (!delta) {                                              /* :332-345 */
        v3 wi_brdf = (rnd(r, SL_MAT_LOBE) < 0.5f) ? spec_get_wi(&m, n, wo, r, SL_MAT_E0, fixed)
                                                  : diff_get_wi(n, r, SL_MAT_E0, fixed);
        bs->vis.o = vadd(is->position, vscale(wi_brdf, 0.001f));
        bs->vis.d = wi_brdf;
        bs->f_brdf = vadd(spec_get_f(&m, n, wi_brdf, wo), diff_get_f(&m, n, wi_brdf, wo));
        bs->Li_brdf = light_L(sc, light_id, wi_brdf);
        bs->pdf_brdf0 = (diff_get_pdf() + spec_get_pdf(&m, n, wi_brdf, wo)) * 0.5f;
        bs->pdf_light1 = light_pdf(sc, light_id, wi_brdf, fixed);
        if (fixed) bs->pdf_light1 = bs->pdf_light1 * sel;
    }
    v3 wi_s = (rnd(r, SL_CONT_LOBE) < 0.5f) ? spec_get_wi(&m, n, wo, r, SL_CONT_E0, fixed)  /* :353 */
                                            : diff_get_wi(n, r, SL_CONT_E0, fixed);
    float pdf_s = (diff_get_pdf() + spec_get_pdf(&m, n, wi_s, wo)) * 0.5f;
    v3 f_s = vadd(spec_get_f(&m, n, wi_s, wo), diff_get_f(&m, n, wi_s, wo));
    p->Li_light = Li_light; p->Li_brdf = V(0.f, 0.f, 0.f);
    p->f_light = f_light; p->f_brdf = V(0.f, 0.f, 0.f); p->f_sample = f_s;
    p->pdf_light[0] = pdf_light[0]; p->pdf_light[1] = pdf_light[1];
    p->pdf_brdf[0] = pdf_brdf[0]; p->pdf_brdf[1] = pdf_brdf[1];
    p->pdf_sample = pdf_s;
    p->ray.o = vadd(is->position, vscale(n, 0.001f));         /* :358 */
    p->ray.d = wi_s;
}

/* a visible BRDF sample's terms (:340-343) */
static void apply_brdf_sample(path_t *p, const brdf_sample_t *bs) {
    p->f_brdf = bs->f_brdf;
    p->Li_brdf = bs->Li_brdf;
    p->pdf_brdf[0] = bs->pdf_brdf0;
    p->pdf_light[1] = bs->pdf_light1;
}

/* wf_mat_mix (wavefront_kernels.cu:295-375) with the inline visibility ray. */
static void wf_mat_mix(ctx_t *c, queues_t *q, uint32_t id) {
    path_t *p = &c->paths[id];
    rng_t r = path_rng(c, id, p->len);
    brdf_sample_t bs;
    mat_mix_core(c->sc, c->cfg->fixed, &r, p, &bs);
    if (bs.has) {                                              /* :334-345 */
        trav_stats st = {0, 0};
        int occluded = any_hit(c->sc, &bs.vis, c->cfg->traversal, &st);
        q->cnt[4] += st.nodes;
        q->cnt[5] += st.tris;
        q->cnt[2]++;
        if (!occluded) apply_brdf_sample(p, &bs);
    }
    q->extq[q->next++] = (int32_t)id;
    q->shq[q->nsh++] = (int32_t)id;
}

/* ------------------------------------------------------------------------- */
/* Stage restatements at the product's stage boundary (mcpt_path_view).       */
/* ------------------------------------------------------------------------- */
enum { PF_DEAD = 1u, PF_LEN_SHIFT = 1, PF_CONDL = 1u << 9, PF_CONDB = 1u << 10, PF_FZERO = 1u << 11,
       PF_HASVIS = 1u << 12, PF_SIDX_SHIFT = 13 };

void or_stage_logic(const or_scene *sc, const or_camera *cam, const or_config *cfg, int32_t W, int32_t H,
                    uint32_t *flags, uint32_t *samples, const int32_t *hit_tri, float *ray_o, float *ray_d,
                    float *beta, const float *nee0, const float *nee1, const uint8_t *vis, float *Ld,
                    uint8_t *queued) {
    uint32_t spp = (uint32_t)cfg->spp;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            uint32_t i = (uint32_t)y * (uint32_t)W + (uint32_t)x;
            queued[i] = 0;
            if (x >= W - 1 || y >= H - 1) continue;            /* :110 */
            uint32_t fl = flags[i];
            int dead = (fl & PF_DEAD) != 0;
            uint32_t len = (fl >> PF_LEN_SHIFT) & 0xffu, sidx = fl >> PF_SIDX_SHIFT;
            if (!dead && sidx < spp) {                         /* :124 */
                rng_t r = {rng_key(cfg->seed, i, sidx), len};
                mis_t m;
                m.cL = V(nee0[4 * i], nee0[4 * i + 1], nee0[4 * i + 2]);
                m.cB = V(nee1[4 * i], nee1[4 * i + 1], nee1[4 * i + 2]);
                m.ratio = V(beta[4 * i + 3], nee0[4 * i + 3], nee1[4 * i + 3]);
                m.condL = (fl & PF_CONDL) != 0;
                m.condB = (fl & PF_CONDB) != 0;
                m.hasvis = (fl & PF_HASVIS) != 0;
                m.fzero = (fl & PF_FZERO) != 0;
                v3 b = V(beta[4 * i], beta[4 * i + 1], beta[4 * i + 2]);
                if (len == 1) b = V(1.f, 1.f, 1.f);           /* wf_generate's beta (:245) */
                v3 rd = V(ray_d[3 * i], ray_d[3 * i + 1], ray_d[3 * i + 2]);
                if (!logic_core(sc, cfg, &r, len, hit_tri[i] >= 0, rd, &b, &m, vis[2 * i], vis[2 * i + 1], Ld + 3 * (size_t)i)) {
                    dead = 1;                                  /* :199-204 */
                    samples[i]++;
                } else {
                    beta[4 * i] = b.x; beta[4 * i + 1] = b.y; beta[4 * i + 2] = b.z;
                    queued[i] |= 2;
                }
            }
            if (dead) {
                flags[i] = PF_DEAD;
                if (samples[i] < spp) {                        /* :219-222 + wf_generate (:225-251) */
                    rng_t r0 = {rng_key(cfg->seed, i, samples[i]), 0};
                    ray_t ray = gen_ray(cam, W, H, x, y, &r0);
                    ray_o[3 * i] = ray.o.x; ray_o[3 * i + 1] = ray.o.y; ray_o[3 * i + 2] = ray.o.z;
                    ray_d[3 * i] = ray.d.x; ray_d[3 * i + 1] = ray.d.y; ray_d[3 * i + 2] = ray.d.z;
                    flags[i] = (1u << PF_LEN_SHIFT) | (samples[i] << PF_SIDX_SHIFT);
                    queued[i] |= 1;
                }
            }
        }
}

void or_stage_material(const or_scene *sc, const or_config *cfg, int32_t n, uint32_t *flags, const int32_t *hit_tri,
                       float *ray_o, float *ray_d, float *beta, float *nee0, float *nee1, float *light_o,
                       float *light_d, float *bvis_o, float *bvis_d) {
    for (int32_t i = 0; i < n; i++) {
        uint32_t fl = flags[i];
        uint32_t len = (fl >> PF_LEN_SHIFT) & 0xffu, sidx = fl >> PF_SIDX_SHIFT;
        rng_t r = {rng_key(cfg->seed, (uint32_t)i, sidx), len};
        path_t p;
        memset(&p, 0, sizeof(p));
        p.ray.o = V(ray_o[3 * i], ray_o[3 * i + 1], ray_o[3 * i + 2]);
        p.ray.d = V(ray_d[3 * i], ray_d[3 * i + 1], ray_d[3 * i + 2]);
        p.isect = make_isect(sc, &p.ray, hit_tri[i], K_HUGE);
        pick_light(sc, cfg->fixed, &r, &p);                    /* wf_logic :207-213 */
        brdf_sample_t bs;
        mat_mix_core(sc, cfg->fixed, &r, &p, &bs);
        if (bs.has) apply_brdf_sample(&p, &bs);                /* the terms as if visible */
        mis_t m = mis_terms(&p, bs.has);
        uint32_t nf = (m.fzero ? PF_FZERO : 0u) | (m.condL ? PF_CONDL : 0u) | (bs.has && m.condB ? PF_CONDB : 0u) |
                      (bs.has ? PF_HASVIS : 0u);
        flags[i] = nf | ((len + 1) << PF_LEN_SHIFT) | (sidx << PF_SIDX_SHIFT);
        v3 cB = bs.has ? m.cB : V(0.f, 0.f, 0.f);
        beta[4 * i + 3] = m.ratio.x;
        nee0[4 * i] = m.cL.x; nee0[4 * i + 1] = m.cL.y; nee0[4 * i + 2] = m.cL.z; nee0[4 * i + 3] = m.ratio.y;
        nee1[4 * i] = cB.x; nee1[4 * i + 1] = cB.y; nee1[4 * i + 2] = cB.z; nee1[4 * i + 3] = m.ratio.z;
        ray_o[3 * i] = p.ray.o.x; ray_o[3 * i + 1] = p.ray.o.y; ray_o[3 * i + 2] = p.ray.o.z;
        ray_d[3 * i] = p.ray.d.x; ray_d[3 * i + 1] = p.ray.d.y; ray_d[3 * i + 2] = p.ray.d.z;
        light_o[3 * i] = p.ray_light.o.x; light_o[3 * i + 1] = p.ray_light.o.y; light_o[3 * i + 2] = p.ray_light.o.z;
        light_d[3 * i] = p.ray_light.d.x; light_d[3 * i + 1] = p.ray_light.d.y; light_d[3 * i + 2] = p.ray_light.d.z;
        float qn = qnan();
        v3 vo = bs.has ? bs.vis.o : V(qn, qn, qn), vd = bs.has ? bs.vis.d : V(qn, qn, qn);
        bvis_o[3 * i] = vo.x; bvis_o[3 * i + 1] = vo.y; bvis_o[3 * i + 2] = vo.z;
        bvis_d[3 * i] = vd.x; bvis_d[3 * i + 1] = vd.y; bvis_d[3 * i + 2] = vd.z;
    }
}

/* wavefront_pathtrace (wavefront_kernels.cu:377-442) iterated until the tile
 * is complete.  Stage order logic -> generate -> material -> extend -> shadow. */
static void render_tile(ctx_t *c, queues_t *q, int tx, int ty) {
    int tw = c->cfg->tile_w, th = c->cfg->tile_h;
    int rb = c->cfg->row_begin, re = c->cfg->row_end;
    for (;;) {
        q->nnew = q->next = q->nsh = q->nmat = 0;
        for (int ly = 0; ly < th; ly++) {
            int y = ty * th + ly;
            if (y >= c->H) break;
            if (re > rb && (y < rb || y >= re)) continue;
            for (int lx = 0; lx < tw; lx++) {
                int x = tx * tw + lx;
                if (x >= c->W) break;
                wf_logic(c, q, x, y);
            }
        }
        if (q->nnew == 0 && q->nmat == 0) break;
        q->cnt[3]++;
        for (int i = 0; i < q->nnew; i++) wf_generate(c, q, (uint32_t)q->newq[i]);
        for (int i = 0; i < q->nmat; i++) wf_mat_mix(c, q, (uint32_t)q->matq[i]);
        for (int i = 0; i < q->next; i++) wf_extend(c, q, (uint32_t)q->extq[i]);
        for (int i = 0; i < q->nsh; i++) wf_shadow(c, q, (uint32_t)q->shq[i]);
        q->cnt[0] += (uint64_t)q->next;
        q->cnt[1] += (uint64_t)q->nsh;
    }
}

typedef struct {
    ctx_t *c;
    int ntx, nty;
    int *next_tile;
    pthread_mutex_t *mu;
    uint64_t cnt[6];
} worker_t;

static void *worker_main(void *arg) {
    worker_t *w = (worker_t *)arg;
    int cap = w->c->cfg->tile_w * w->c->cfg->tile_h;
    queues_t q;
    memset(&q, 0, sizeof(q));
    q.newq = (int32_t *)malloc(sizeof(int32_t) * cap);
    q.extq = (int32_t *)malloc(sizeof(int32_t) * cap);
    q.shq = (int32_t *)malloc(sizeof(int32_t) * cap);
    q.matq = (int32_t *)malloc(sizeof(int32_t) * cap);
    for (;;) {
        pthread_mutex_lock(w->mu);
        int t = (*w->next_tile)++;
        pthread_mutex_unlock(w->mu);
        if (t >= w->ntx * w->nty) break;
        const or_config *cf = w->c->cfg;
        if (cf->tile_mod > 0 && ((t % w->ntx) + (t / w->ntx)) % cf->tile_mod != cf->tile_rank) continue;
        render_tile(w->c, &q, t % w->ntx, t / w->ntx);
    }
    for (int i = 0; i < 6; i++) w->cnt[i] = q.cnt[i];
    free(q.newq); free(q.extq); free(q.shq); free(q.matq);
    return NULL;
}

int or_render(const or_scene *sc, const or_camera *cam, const or_config *cfg, int32_t W, int32_t H,
              float *Ld, uint32_t *samples, uint64_t *counters) {
    if (W <= 0 || H <= 0 || cfg->tile_w <= 0 || cfg->tile_h <= 0) return -1;
    ctx_t c;
    c.sc = sc; c.cam = cam; c.cfg = cfg; c.W = W; c.H = H; c.Ld = Ld; c.samples = samples;
    size_t P = (size_t)W * (size_t)H;
    c.paths = (path_t *)calloc(P, sizeof(path_t));
    if (!c.paths) return -2;
    for (size_t i = 0; i < P; i++) {                            /* g_clear_dfilm :55-66 */
        c.paths[i].dead = 1;
        samples[i] = 0;
        Ld[3 * i] = Ld[3 * i + 1] = Ld[3 * i + 2] = 0.f;
    }
    int ntx = (W + cfg->tile_w - 1) / cfg->tile_w, nty = (H + cfg->tile_h - 1) / cfg->tile_h;
    int nthreads = cfg->nthreads > 0 ? cfg->nthreads : 1;
    int next_tile = 0;
    pthread_mutex_t mu;
    pthread_mutex_init(&mu, NULL);
    worker_t *ws = (worker_t *)calloc((size_t)nthreads, sizeof(worker_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int i = 0; i < nthreads; i++) {
        ws[i].c = &c; ws[i].ntx = ntx; ws[i].nty = nty; ws[i].next_tile = &next_tile; ws[i].mu = &mu;
        pthread_create(&th[i], NULL, worker_main, &ws[i]);
    }
    for (int k = 0; k < 6; k++) counters[k] = 0;
    for (int i = 0; i < nthreads; i++) {
        pthread_join(th[i], NULL);
        for (int k = 0; k < 6; k++) counters[k] += ws[i].cnt[k];
    }
    pthread_mutex_destroy(&mu);
    free(ws); free(th); free(c.paths);
    return 0;
}

const char *or_version(void) { return "mcpt-oracle 1 (reference @ JakeKurtz/MC-Path-Tracer v0)"; }
