/*
 * trav_model.c -- TEST INFRASTRUCTURE ONLY: a scalar model of the *product* traversal's box
 * culling, used by tests/test_cull_model.py to check the culling rule against the oracle's
 * reference traversal (mcpt_oracle.c closest_hit / any_hit, which culls nothing, as
 * Triangle.cu:144-243 with Bounds3f.h:121-153 does) on adversarial rays.  Nothing in the
 * product links or calls this file.
 *
 * The reference visits every box the infinite line crosses; the product skips boxes that cannot
 * hold the answer.  Two rules are modelled:
 *   mode 1  the round-3 rule: a box is skipped when it lies behind the origin by more than an
 *           absolute 1e-5 (t1 < -1e-5) or starts beyond (1 + 2^-8) * t_best.  It assumed that
 *           Moller-Trumbore's computed t lies within 2^-8 * t of the box's slab interval, which a
 *           grazing ray breaks;
 *   mode 2  the round-4 rule (kernels.hip cull_*; DESIGN.md section 5 "culling bound"): every box
 *           carries a margin W (position units) that bounds how far the point o + t d of an
 *           accepted hit can lie outside the box, whatever the ray's angle to the triangle, from
 *           the rounding error of the fp32 Moller-Trumbore expressions with the det >= 1e-6
 *           acceptance threshold (Triangle.cu:17-21).  Skip when t1 (1 - 2^-18) + W i < 0 (behind)
 *           or t0 - W i > t_best (1 + 2^-18 + i P) (beyond), i = max |1/d_a| (1 + 2^-18).
 *   mode 6  a round-5 candidate (not in the product): margins from
 *           or_model_set_safe(c) give the triangles the general bound leaves unbounded the margin
 *           of rays with |d . m^| >= c |d| (then det >= |d| (c |m| - 7.0712 u |e1| |e2|), no
 *           threshold needed); a ray within c of any such triangle's plane is traced with no
 *           culling (mode 0), every other ray with mode 2's rule.
 * The margins come from or_model_margins (a restatement of the product's k_cull_margins in C).
 * Visit order: both children of an interior node are tested, the nearer (entry t) is visited
 * first -- the product's order; a sound rule gives the reference's answer in any order.
 * Leaves of several primitives test each triangle under its own box (the product's expansion
 * into one-triangle leaves, runtime.cpp scene_upload), with the triangle's own margin.
 */
#include "mcpt_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define M_EPS 1e-6f
#define M_HUGE 1e32f
#define CULL_SLACK 3.814697265625e-06 /* 2^-18 */

typedef struct { float x, y, z; } mv3;
static mv3 mv(float x, float y, float z) { mv3 r = {x, y, z}; return r; }
static mv3 mld(const float *p, int64_t i) { return mv(p[3 * i], p[3 * i + 1], p[3 * i + 2]); }
static mv3 msub(mv3 a, mv3 b) { return mv(a.x - b.x, a.y - b.y, a.z - b.z); }
static float mdot(mv3 a, mv3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static mv3 mcross(mv3 a, mv3 b) { return mv(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }

/* the oracle's tri_intersect (Triangle.cu:9-65, TEST_CULL, fp64 det island), t only */
static int m_tri(const or_scene *sc, int id, mv3 o, mv3 d, float *to) {
    mv3 p0 = mld(sc->v0, id), p1 = mld(sc->v1, id), p2 = mld(sc->v2, id);
    mv3 e1 = msub(p1, p0), e2 = msub(p2, p0);
    mv3 pvec = mcross(d, e2);
    double det = (double)mdot(e1, pvec);
    if (det < (double)M_EPS) return 0;
    mv3 tvec = msub(o, p0);
    float u = mdot(tvec, pvec);
    if ((double)u < 0.0 || (double)u > det) return 0;
    mv3 qvec = mcross(tvec, e1);
    float v = mdot(d, qvec);
    if ((double)v < 0.0 || (double)(u + v) > det) return 0;
    float t = mdot(e2, qvec);
    *to = (float)((double)t * (1.0 / det));
    return 1;
}

/* ---- margins (the product's k_cull_margins / cull_margin, mcpt_core.hpp) ---------------- */
static const double U24 = 5.9604644775390625e-08; /* 2^-24 */

/* per triangle: beta (coefficient of |tvec|) and omega (absolute term) of the bound
 * |P' - conv(T)|_a <= omega + beta |o - p0| on an accepted hit */
static double nrm(mv3 e) { return sqrt((double)e.x * e.x + (double)e.y * e.y + (double)e.z * e.z); }
static void tri_beta_omega(mv3 e1, mv3 e2, double *beta, double *omega) {
    const double n1 = nrm(e1), n2 = nrm(e2);
    const double alpha = 28.3 * U24 * n1 * n2 / (double)M_EPS;
    *beta = alpha * (1.0 + 1.0 / 512.0) + 1.01 * U24;
    *omega = 2.1 * U24 * (n1 > n2 ? n1 : n2);
}
/* axis-plane triangles (e1_a = e2_a = 0): b_T = 15.0003 u |e1| |e2| / G', G' = |G| - 5.0002 u S
 * with G the in-plane cross product and S its products' magnitudes; the bound is then
 * w <= omega + 1.01 u |tvec| + b_T (|tvec| + |t| |d|), independent of the det threshold.  0 when
 * the triangle is not in an axis plane or G' < G / 2. */
static double plane_b(mv3 e1, mv3 e2) {
    double a1, c1, a2, c2;
    if (e1.x == 0.f && e2.x == 0.f) { a1 = e1.y; c1 = e1.z; a2 = e2.y; c2 = e2.z; }
    else if (e1.y == 0.f && e2.y == 0.f) { a1 = e1.z; c1 = e1.x; a2 = e2.z; c2 = e2.x; }
    else if (e1.z == 0.f && e2.z == 0.f) { a1 = e1.x; c1 = e1.y; a2 = e2.x; c2 = e2.y; }
    else return 0.0;
    const double g = fabs(a1 * c2 - c1 * a2) * (1.0 - 1.0 / 1099511627776.0);
    const double sg = (fabs(a1 * c2) + fabs(c1 * a2)) * (1.0 + 1.0 / 1099511627776.0);
    const double gp = g - 5.0002 * U24 * sg;
    if (!(gp > 0.5 * g)) return 0.0;
    return 15.0003 * U24 * nrm(e1) * nrm(e2) * (1.0 + 1e-12) / gp;
}
/* a triangle's margin W'_T = (omega + beta diam_T) / (1 - sqrt3 beta) (+ slack); +inf when
 * sqrt3 beta >= 1/2 (a triangle so large against the det threshold that no box holding it is
 * ever culled).  A box's margin is the maximum over the triangles it holds.  *far: the
 * triangle's coefficient of t_best in the far cut (P is their maximum). */
static float to_f_up(double w) { return isinf(w) ? INFINITY : (float)(w * (1.0 + 1.0 / 1048576.0)) * (1.0f + 1.0f / 1048576.0f); }
static double g_safe_c = 0.0; /* or_model_set_safe: 0 = the product's margins */
void or_model_set_safe(double c) { g_safe_c = c; }
/* beta of the safe-ray bound: |R_a| / det <= 28.285 u |tvec| |e1| |e2| / K, K = c |m| - 7.0712 u |e1| |e2| */
static double safe_beta(mv3 e1, mv3 e2, double c) {
    const double a[3] = {e1.x, e1.y, e1.z}, b[3] = {e2.x, e2.y, e2.z};
    const double m[3] = {b[1] * a[2] - b[2] * a[1], b[2] * a[0] - b[0] * a[2], b[0] * a[1] - b[1] * a[0]};
    const double mm = sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]) * (1.0 - 1e-12);
    const double k = c * mm - 7.0712 * U24 * nrm(e1) * nrm(e2) * (1.0 + 1e-12);
    if (!(k > 0.0)) return INFINITY;
    return 28.3 * U24 * nrm(e1) * nrm(e2) / k * (1.0 + 1e-9) + 1.01 * U24;
}
static double tri_w_of(const or_scene *sc, int t, double *far) {
    mv3 a = mld(sc->v0, t), b = mld(sc->v1, t), c = mld(sc->v2, t);
    mv3 e1 = msub(b, a), e2 = msub(c, a), e3 = msub(c, b);
    double be, om;
    tri_beta_omega(e1, e2, &be, &om);
    const double pb = plane_b(e1, e2);
    if (pb > 0.0) be = (1.01 * U24 + pb) * (1.0 + 1.0 / 8388608.0);
    *far = 0.0;
    if (!(1.7321 * be * (1.0 + CULL_SLACK) < 0.5) && g_safe_c > 0.0 && pb == 0.0) be = safe_beta(e1, e2, g_safe_c);
    if (!(1.7321 * be * (1.0 + CULL_SLACK) < 0.5)) return INFINITY;
    const double l1 = nrm(e1), l2 = nrm(e2), l3 = nrm(e3) * (1.0 + 1e-7);
    const double diam = l1 > l2 ? (l1 > l3 ? l1 : l3) : (l2 > l3 ? l2 : l3);
    const double den = 1.0 - 1.7321 * be * (1.0 + CULL_SLACK);
    *far = (pb > 0.0 ? be + pb : be) * (1.0 + 1.0 / 512.0) / den * (1.0 + CULL_SLACK) * (1.0 + 1.0 / 1048576.0);
    return (om + be * diam * (1.0 + 1e-12)) * (1.0 + CULL_SLACK) / den;
}

/* node_w[n]: margin of desc node n's box; tri_w[t]: margin of triangle t's own box; *p: the
 * scene's far-cut coefficient P.  contained: 0 when some node box fails to contain its
 * subtree's vertices (the product then culls nothing). */
int32_t or_model_margins(const or_scene *sc, float *node_w, float *tri_w, float *p) {
    const int N = sc->nnodes;
    double *nw = calloc((size_t)(N > 0 ? N : 1), sizeof(double));
    float *lo = malloc(sizeof(float) * 3 * (size_t)(N > 0 ? N : 1)), *hi = malloc(sizeof(float) * 3 * (size_t)(N > 0 ? N : 1));
    double pg = 0.0;
    int contained = 1;
    for (int t = 0; t < sc->ntri; t++) {
        double fc;
        const double w = tri_w_of(sc, t, &fc);
        if (!isinf(w) && fc > pg) pg = fc;
        tri_w[t] = to_f_up(w);
    }
    /* subtree maxima, children before parents: desc nodes are depth-first (children after parent) */
    for (int n = N - 1; n >= 0; n--) {
        if (sc->nprims[n] > 0) {
            double w = 0;
            for (int k = 0; k < 3; k++) { lo[3 * n + k] = INFINITY; hi[3 * n + k] = -INFINITY; }
            for (int i = 0; i < sc->nprims[n]; i++) {
                const int t = sc->offset[n] + i;
                double be;
                const double wt = tri_w_of(sc, t, &be);
                if (!(wt <= w)) w = wt;
                const float *v[3] = {sc->v0 + 3 * (int64_t)t, sc->v1 + 3 * (int64_t)t, sc->v2 + 3 * (int64_t)t};
                for (int j = 0; j < 3; j++)
                    for (int k = 0; k < 3; k++) {
                        lo[3 * n + k] = fminf(lo[3 * n + k], v[j][k]);
                        hi[3 * n + k] = fmaxf(hi[3 * n + k], v[j][k]);
                    }
            }
            nw[n] = w;
        } else {
            const int c0 = n + 1, c1 = sc->offset[n];
            nw[n] = nw[c0] > nw[c1] ? nw[c0] : nw[c1];
            for (int k = 0; k < 3; k++) {
                lo[3 * n + k] = fminf(lo[3 * c0 + k], lo[3 * c1 + k]);
                hi[3 * n + k] = fmaxf(hi[3 * c0 + k], hi[3 * c1 + k]);
            }
        }
        for (int k = 0; k < 3; k++)
            if (lo[3 * n + k] < sc->bmin[3 * n + k] || hi[3 * n + k] > sc->bmax[3 * n + k]) contained = 0;
        node_w[n] = to_f_up(nw[n]);
    }
    *p = (float)pg;
    free(nw); free(lo); free(hi);
    return contained;
}

/* ---- traversal ------------------------------------------------------------------------ */
typedef struct {
    mv3 o, d, inv;
    int fin, neg[3];
    float iota, iota_b;  /* mode >= 2: far / behind scale */
} mray;

/* the product's box test: reference slab decisions (Bounds3f.h:121-153); t0/t1 = entry/exit */
static int m_box(const float *mn, const float *mx, const mray *r, float *t0, float *t1) {
    if (r->fin) {
        const float ax = (mn[0] - r->o.x) * r->inv.x, bx = (mx[0] - r->o.x) * r->inv.x;
        const float ay = (mn[1] - r->o.y) * r->inv.y, by = (mx[1] - r->o.y) * r->inv.y;
        const float az = (mn[2] - r->o.z) * r->inv.z, bz = (mx[2] - r->o.z) * r->inv.z;
        *t0 = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
        *t1 = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
        return *t0 <= *t1;
    }
    float bx0 = r->neg[0] ? mx[0] : mn[0], bx1 = r->neg[0] ? mn[0] : mx[0];
    float by0 = r->neg[1] ? mx[1] : mn[1], by1 = r->neg[1] ? mn[1] : mx[1];
    float bz0 = r->neg[2] ? mx[2] : mn[2], bz1 = r->neg[2] ? mn[2] : mx[2];
    float tmin = (bx0 - r->o.x) * r->inv.x, tmax = (bx1 - r->o.x) * r->inv.x;
    float tymin = (by0 - r->o.y) * r->inv.y, tymax = (by1 - r->o.y) * r->inv.y;
    float tzmin = (bz0 - r->o.z) * r->inv.z, tzmax = (bz1 - r->o.z) * r->inv.z;
    int miss = (tmin > tymax) || (tymin > tmax);
    float a = (tymin > tmin) ? tymin : tmin, b = (tymax < tmax) ? tymax : tmax;
    miss = miss || (a > tzmax) || (tzmin > b);
    *t0 = (tzmin > a) ? tzmin : a;
    *t1 = (tzmax < b) ? tzmax : b;
    return !miss;
}

/* keep (visit) a box whose slab test passed; cut: mode 1 (1 + 2^-8) t_best, mode 2 t_best
 * (1 + 2^-18 + iota P), +inf for any-hit rays.  Returns the entry key used for near-first order. */
static int m_keep(int mode, float t0, float t1, float w, const mray *r, float cut, float *key) {
    if (mode == 1) {
        *key = t0;
        return !(t1 < -1e-5f) && !(t0 > cut);
    }
    if (mode >= 2) {
        const float m = w * r->iota, mb = w * r->iota_b;
        const float e = mode == 4 ? t0 : t0 - m;
        *key = e;
        const int behind = mode == 3 ? t1 < -1e-5f : fmaf(t1, (float)(1.0 - CULL_SLACK), mb) < 0.f;
        return !behind && !(e > cut);
    }
    *key = t0;
    return 1;
}

static int tri_key(const or_scene *sc, int id) { return sc->tri_id ? sc->tri_id[id] : id; }

/* Traversal study (or_model_study): what one m_trace call visits, recorded when g_rec is set */
typedef struct {
    const int32_t *pair_line; /* desc node -> 128-B line of its child pair, or of a multi-triangle
                               * leaf's first expansion pair (the layout under study) */
    int32_t tri_line0;        /* first line of the 48-B triangle records */
    int32_t steps, origin_steps, tris;
    int32_t *lines;
    int64_t n, cap;
} study_rec;
static __thread study_rec *g_rec = NULL;
static void rec_line(int32_t l) {
    if (g_rec->n < g_rec->cap) g_rec->lines[g_rec->n] = l;
    g_rec->n++;
}
static void rec_step(const or_scene *sc, int cur, mv3 o) {
    if (!g_rec) return;
    g_rec->steps++;
    const float *mn = sc->bmin + 3 * (int64_t)cur, *mx = sc->bmax + 3 * (int64_t)cur;
    g_rec->origin_steps += mn[0] <= o.x && o.x <= mx[0] && mn[1] <= o.y && o.y <= mx[1] && mn[2] <= o.z && o.z <= mx[2];
    rec_line(g_rec->pair_line[cur]);
}
static void rec_tri(int id) {
    if (!g_rec) return;
    g_rec->tris++;
    const int64_t b0 = (int64_t)id * 48, b1 = b0 + 47;
    rec_line(g_rec->tri_line0 + (int32_t)(b0 >> 7));
    if ((b1 >> 7) != (b0 >> 7)) rec_line(g_rec->tri_line0 + (int32_t)(b1 >> 7));
}

/* triangle tests of the last or_model_trace call (its rays, both kinds): work counts for the
 * culling variants (single-threaded callers only) */
static uint64_t g_tri_tests = 0;
uint64_t or_model_tri_tests(void) { return g_tri_tests; }

/* Any-hit visiting order under study (or_model_set_any_order; the product visits near-first):
 * 1 the child with the larger box surface first, 2 the far child first */
static int g_any_order = 0;
void or_model_set_any_order(int32_t m) { g_any_order = m; }
static double m_area(const or_scene *sc, int i) {
    const float *mn = sc->bmin + 3 * (int64_t)i, *mx = sc->bmax + 3 * (int64_t)i;
    const double x = fmax(mx[0] - mn[0], 0.0), y = fmax(mx[1] - mn[1], 0.0), z = fmax(mx[2] - mn[2], 0.0);
    return x * y + y * z + z * x;
}
static int m_any_first(const or_scene *sc, const int c[2], const float k2[2]) {
    if (g_any_order == 1) return m_area(sc, c[1]) > m_area(sc, c[0]);
    return k2[1] > k2[0];
}

/* kind 0: closest hit (index, t), kind 1: any hit (1 = occluded) */
static int m_trace(const or_scene *sc, int mode, const float *node_w, const float *tri_w, float pg, mv3 o, mv3 d,
                   int kind, float *tout, uint64_t *nodes) {
    mray r;
    r.o = o;
    r.d = d;
    r.inv = mv(1.f / d.x, 1.f / d.y, 1.f / d.z);
    r.neg[0] = r.inv.x < 0.f; r.neg[1] = r.inv.y < 0.f; r.neg[2] = r.inv.z < 0.f;
    r.fin = fabsf(r.inv.x) < INFINITY && fabsf(r.inv.y) < INFINITY && fabsf(r.inv.z) < INFINITY;
    const float n2 = mdot(d, d);
    r.iota = INFINITY;
    if (r.fin && n2 <= (float)(1.0 + 1.0 / 512.0))
        r.iota = fmaxf(fmaxf(fabsf(r.inv.x), fabsf(r.inv.y)), fabsf(r.inv.z)) * (float)(1.0 + CULL_SLACK);
    /* behind cut: valid only when every direction component is >= P |d| */
    r.iota_b = r.iota * pg <= 1.0f ? r.iota : INFINITY;
    const float cfac = (mode == 2 || mode == 3) ? fmaf(r.iota, pg, (float)(1.0 + CULL_SLACK)) : mode ? 1.0f + 1.0f / 256.0f : INFINITY;
    float best = M_HUGE;
    int bt = -1;
    float cut = kind || mode == 0 ? INFINITY : best * cfac;
    if (sc->nnodes <= 0) { *tout = best; return kind ? 0 : -1; }
    int stack[130];
    float skey[130];
    int sp = 0;
    float t0, t1, key;
    /* root */
    (*nodes)++;
    if (!(m_box(sc->bmin, sc->bmax, &r, &t0, &t1) && m_keep(mode, t0, t1, node_w[0], &r, kind ? INFINITY : cut, &key))) {
        *tout = best;
        return kind ? 0 : -1;
    }
    int cur = 0;
    for (;;) {
        if (sc->nprims[cur] > 0) {
            const int np = sc->nprims[cur];
            if (g_rec && np > 1) rec_line(g_rec->pair_line[cur]);  /* the leaf's expansion pairs */
            for (int i = 0; i < np; i++) {
                const int id = sc->offset[cur] + i;
                if (np > 1) {  /* own box (the product's one-triangle leaves) */
                    float mn[3], mx[3];
                    const float *v[3] = {sc->v0 + 3 * (int64_t)id, sc->v1 + 3 * (int64_t)id, sc->v2 + 3 * (int64_t)id};
                    for (int k = 0; k < 3; k++) {
                        mn[k] = fminf(fminf(v[0][k], v[1][k]), v[2][k]);
                        mx[k] = fmaxf(fmaxf(v[0][k], v[1][k]), v[2][k]);
                    }
                    (*nodes)++;
                    if (!(m_box(mn, mx, &r, &t0, &t1) && m_keep(mode, t0, t1, tri_w[id], &r, cut, &key))) continue;
                }
                float t;
                g_tri_tests++;
                rec_tri(id);
                if (m_tri(sc, id, o, d, &t) && !(t < 0.f)) {
                    if (kind) {
                        if (t < M_HUGE) { *tout = t; return 1; }
                    } else if (t < best || (t == best && bt >= 0 && tri_key(sc, id) < tri_key(sc, bt))) {
                        best = t;
                        bt = id;
                        if (mode) cut = best * cfac;
                    }
                }
            }
        } else {
            const int c[2] = {cur + 1, sc->offset[cur]};
            int h[2];
            rec_step(sc, cur, o);
            float k2[2];
            for (int j = 0; j < 2; j++) {
                (*nodes)++;
                h[j] = m_box(sc->bmin + 3 * (int64_t)c[j], sc->bmax + 3 * (int64_t)c[j], &r, &t0, &t1) &&
                       m_keep(mode, t0, t1, node_w[c[j]], &r, cut, &k2[j]);
            }
            if (h[0] && h[1]) {
                int f = k2[1] < k2[0];
                if (kind && g_any_order) f = m_any_first(sc, c, k2);
                stack[sp] = c[1 - f];
                skey[sp++] = k2[1 - f];
                cur = c[f];
                continue;
            }
            if (h[0] || h[1]) { cur = h[0] ? c[0] : c[1]; continue; }
        }
        /* pop the next entry still in front of the cut */
        cur = -1;
        while (sp > 0) {
            sp--;
            if (skey[sp] > cut) continue;
            cur = stack[sp];
            break;
        }
        if (cur < 0) break;
    }
    *tout = best;
    return kind ? 0 : bt;
}

void or_model_trace(const or_scene *sc, int32_t n, const float *ro, const float *rd, int32_t mode,
                    const float *node_w, const float *tri_w, float p, int32_t *tri, float *t, uint8_t *visible,
                    uint64_t *nodes) {
    uint64_t nn = 0;
    g_tri_tests = 0;
    /* modes 6 / 7: the planes of the triangles the general bound leaves unbounded (n as float, thr) */
    int np = 0;
    float *pl = NULL;
    if (mode == 6 || mode == 7) {
        pl = malloc(sizeof(float) * 4 * (size_t)(sc->ntri > 0 ? sc->ntri : 1));
        for (int t = 0; t < sc->ntri; t++) {
            mv3 p0 = mld(sc->v0, t), e1 = msub(mld(sc->v1, t), p0), e2 = msub(mld(sc->v2, t), p0);
            double be, om;
            tri_beta_omega(e1, e2, &be, &om);
            if (1.7321 * be * (1.0 + CULL_SLACK) < 0.5 || plane_b(e1, e2) > 0.0) continue;
            float nf[3];
            const double a3[3] = {e1.x, e1.y, e1.z}, b3[3] = {e2.x, e2.y, e2.z};
            const double m[3] = {b3[1] * a3[2] - b3[2] * a3[1], b3[2] * a3[0] - b3[0] * a3[2], b3[0] * a3[1] - b3[1] * a3[0]};
            const double mm = sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
            double dn = 0.0, nn2 = 0.0;
            for (int k = 0; k < 3; k++) {
                nf[k] = mm > 0.0 ? (float)(m[k] / mm) : 0.f;
                const double e = (double)nf[k] - (mm > 0.0 ? m[k] / mm : 0.0);
                dn += e * e;
                nn2 += (double)nf[k] * nf[k];
            }
            const double fd = 1.0 + 1.0 / 1024.0;
            const double thr = g_safe_c * fd + fd * (sqrt(dn) * (1.0 + 1e-6) + 1e-30 + 3.0002 * U24 * sqrt(nn2));
            float ft = (float)(thr * (1.0 + 1e-9));
            if ((double)ft < thr) ft = nextafterf(ft, INFINITY);
            pl[4 * np] = nf[0]; pl[4 * np + 1] = nf[1]; pl[4 * np + 2] = nf[2]; pl[4 * np + 3] = mm > 0.0 ? ft : INFINITY;
            np++;
        }
    }
    for (int32_t i = 0; i < n; i++) {
        mv3 o = mld(ro, i), d = mld(rd, i);
        float tb;
        int rmode = mode;
        const float *nw = node_w, *tw = tri_w;
        if (mode == 6 || mode == 7) {
            /* mode 6: unsafe rays (within the threshold of an unbounded triangle's plane) are not
             * culled at all; mode 7 (the product's dual tree): they take the general margins
             * (node_w / tri_w first halves), safe rays the safe-ray margins (second halves) */
            int unsafe = 0;
            for (int k = 0; k < np && !unsafe; k++) {
                const float g = (d.x * pl[4 * k] + d.y * pl[4 * k + 1]) + d.z * pl[4 * k + 2];
                if (!(fabsf(g) >= pl[4 * k + 3])) unsafe = 1;
            }
            rmode = mode == 6 && unsafe ? 0 : 2;
            if (mode == 7 && !unsafe) {
                nw = node_w + (sc->nnodes > 0 ? sc->nnodes : 1);
                tw = tri_w + (sc->ntri > 0 ? sc->ntri : 1);
            }
        }
        const int id = m_trace(sc, rmode, nw, tw, p, o, d, 0, &tb, &nn);
        tri[i] = id >= 0 ? tri_key(sc, id) : -1;
        t[i] = tb;
        visible[i] = (uint8_t)!m_trace(sc, rmode, nw, tw, p, o, d, 1, &tb, &nn);
    }
    free(pl);
    *nodes = nn;
}

/* Round-6 traversal study, analysis only: per ray of `kind` (0 closest, 1 any
 * hit) under rule `mode`, the pair steps, the steps whose node box contains the ray origin, the
 * triangle tests and the outcome (hit / occluded); and the 128-B lines those steps fetch under a
 * node numbering: pair_line[node] for an interior desc node's child pair, tri_line0 + the lines of
 * triangle record id (48 B each).  Lines of ray i: lines[off[i] .. off[i+1]) (truncated at cap;
 * off[n] is the full count). */
void or_model_study(const or_scene *sc, int32_t n, const float *ro, const float *rd, int32_t mode, int32_t kind,
                    const float *node_w, const float *tri_w, float p, const int32_t *pair_line, int32_t tri_line0,
                    int32_t *steps, int32_t *origin_steps, int32_t *tris, uint8_t *hit, int32_t *lines, int64_t cap,
                    int64_t *off) {
    study_rec r;
    memset(&r, 0, sizeof r);
    r.pair_line = pair_line;
    r.tri_line0 = tri_line0;
    r.lines = lines;
    r.cap = cap;
    g_rec = &r;
    uint64_t nn = 0;
    for (int32_t i = 0; i < n; i++) {
        off[i] = r.n;
        r.steps = r.origin_steps = r.tris = 0;
        float tb;
        const int res = m_trace(sc, mode, node_w, tri_w, p, mld(ro, i), mld(rd, i), kind, &tb, &nn);
        steps[i] = r.steps;
        origin_steps[i] = r.origin_steps;
        tris[i] = r.tris;
        hit[i] = (uint8_t)(kind ? res != 0 : res >= 0);
    }
    off[n] = r.n;
    g_rec = NULL;
}

/* Misses of a set-associative LRU cache (sets x ways lines) over the line streams of n rays, the
 * rays taken `batch` at a time and interleaved one access per ray per round (a crude model of the
 * rays in flight on one L2). */
int64_t or_lru_sim(const int32_t *lines, const int64_t *off, int32_t n, int32_t batch, int32_t sets, int32_t ways) {
    int32_t *tag = malloc(sizeof(int32_t) * (size_t)sets * ways);
    uint32_t *age = malloc(sizeof(uint32_t) * (size_t)sets * ways);
    int64_t *cur = malloc(sizeof(int64_t) * (size_t)(batch > 0 ? batch : 1));
    for (int64_t k = 0; k < (int64_t)sets * ways; k++) { tag[k] = -1; age[k] = 0; }
    uint32_t clock = 0;
    int64_t miss = 0;
    for (int32_t b0 = 0; b0 < n; b0 += batch) {
        const int32_t nb = n - b0 < batch ? n - b0 : batch;
        for (int32_t j = 0; j < nb; j++) cur[j] = off[b0 + j];
        int live = 1;
        while (live) {
            live = 0;
            for (int32_t j = 0; j < nb; j++) {
                if (cur[j] >= off[b0 + j + 1]) continue;
                live = 1;
                const int32_t l = lines[cur[j]++];
                const int32_t s = (int32_t)((uint32_t)l % (uint32_t)sets);
                int32_t *tg = tag + (int64_t)s * ways;
                uint32_t *ag = age + (int64_t)s * ways;
                int w = -1, lru = 0;
                for (int k = 0; k < ways; k++) {
                    if (tg[k] == l) { w = k; break; }
                    if (ag[k] < ag[lru]) lru = k;
                }
                if (w < 0) { miss++; w = lru; tg[w] = l; }
                ag[w] = ++clock;
            }
        }
    }
    free(tag);
    free(age);
    free(cur);
    return miss;
}
