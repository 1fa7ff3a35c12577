/*
 * cull_probe.c — diagnostic (never product, never a checker): how much of the reference's
 * BVH work on a scene is spent in nodes whose TIGHT box (the box of the node's triangles,
 * without the reference's FLT_MIN-initialised max bound, DataTypes.h:315) the ray misses by
 * more than a margin.  For each pixel it runs the reference traversal (Utils.h:246-288)
 * twice — as the reference does it, and with "visit iff the reference slab passes AND the
 * ray's line meets tight box (+) margin" — and counts slab and triangle tests of both, plus
 * the number of rays whose result differs (closest t / triangle, occlusion), which must be
 * zero for any sound margin.
 *
 * Margins: a fixed delta, or (delta < 0) the per-triangle bound of DESIGN.md §3 ("Exact cull") —
 * for camera rays computed from the camera origin, for shadow rays from the light and the
 * ray's tmax (per node on a geometric tmax grid, the next grid value above the ray's).
 *
 * Build: gcc -O2 -ffp-contract=off -shared -fPIC -Iinclude tools/cull_probe.c -o tools/bin/libcull_probe.so
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rtx.h"
#include "../gp1_raytracer_2223_amd/csrc/rtx_cull.h"

typedef struct { float x, y, z; } v3;
static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 scale(v3 v, float s) { return mk(v.x * s, v.y * s, v.z * s); }
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x);
}
static inline float smin(float a, float b) { return (b < a) ? b : a; }
static inline float smax(float a, float b) { return (a < b) ? b : a; }
typedef struct { v3 o, d, inv; float tmin, tmax; } ray;
static ray mkray(v3 o, v3 d, float tmin, float tmax) {
    ray r; r.o = o; r.d = d; r.inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z); r.tmin = tmin; r.tmax = tmax;
    return r;
}
static int slab(const float* mn, const float* mx, const ray* r) {
    const float tx1 = (mn[0] - r->o.x) * r->inv.x, tx2 = (mx[0] - r->o.x) * r->inv.x;
    float tMin = smin(tx1, tx2), tMax = smax(tx1, tx2);
    const float ty1 = (mn[1] - r->o.y) * r->inv.y, ty2 = (mx[1] - r->o.y) * r->inv.y;
    tMin = smax(tMin, smin(ty1, ty2)); tMax = smin(tMax, smax(ty1, ty2));
    const float tz1 = (mn[2] - r->o.z) * r->inv.z, tz2 = (mx[2] - r->o.z) * r->inv.z;
    tMin = smax(tMin, smin(tz1, tz2)); tMax = smin(tMax, smax(tz1, tz2));
    return tMax > 0 && tMax >= tMin;
}
/* double test: does the LINE through the ray meet box [mn - dl, mx + dl]? */
static int meets(const double* mn, const double* mx, double dl, const ray* r) {
    const double o[3] = {r->o.x, r->o.y, r->o.z}, d[3] = {r->d.x, r->d.y, r->d.z};
    double t0 = -INFINITY, t1 = INFINITY;
    for (int k = 0; k < 3; ++k) {
        const double lo = mn[k] - dl, hi = mx[k] + dl;
        if (d[k] == 0.0) {
            if (o[k] < lo || o[k] > hi) return 0;
            continue;
        }
        double a = (lo - o[k]) / d[k], b = (hi - o[k]) / d[k];
        if (a > b) { const double x = a; a = b; b = x; }
        if (a > t0) t0 = a;
        if (b < t1) t1 = b;
        if (t0 > t1) return 0;
    }
    return 1;
}
static int tri(v3 v0, v3 v1, v3 v2, v3 n, int cull, const ray* r, int ignore, float* tout) {
    const float cullDot = dot(n, r->d);
    if (fabsf(cullDot) < FLT_EPSILON) return 0;
    if (ignore) {
        if (cull == RTX_CULL_FRONT) cull = RTX_CULL_BACK;
        else if (cull == RTX_CULL_BACK) cull = RTX_CULL_FRONT;
    }
    if (cull == RTX_CULL_FRONT) { if (cullDot < 0) return 0; }
    else if (cull == RTX_CULL_BACK) { if (cullDot > 0) return 0; }
    const v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    const v3 h = cross(r->d, e2);
    const float a = dot(e1, h);
    if (fabsf(a) < FLT_EPSILON) return 0;
    const float ai = 1.f / a;
    const v3 s = sub(r->o, v0);
    const float u = ai * dot(s, h);
    if (u < 0.f || u > 1.f) return 0;
    const v3 q = cross(s, e1);
    const float v = ai * dot(r->d, q);
    if (v < 0.f || (u + v) > 1.f) return 0;
    const float t = ai * dot(e2, q);
    if (t < r->tmin || t >= r->tmax) return 0;
    *tout = t;
    return 1;
}

/* ---------------------------------------------------------------- margins ("Exact cull") */
static const double U = 0x1p-24;
static double gam(int n) { return n * U / (1.0 - n * U); }

typedef struct {
    double v0[3], E1[3], E2[3];   /* float values as doubles */
    double n1E1, n1E2;            /* 1-norms */
    double lE1, lE2, lmax;        /* 2-norms */
    double N[3], lN, nh[3];       /* E1 x E2 (exact in double up to 1 ulp), |N|, unit normal */
} tri_info;

static void tri_setup(tri_info* T, const float* p0, const float* p1, const float* p2) {
    for (int k = 0; k < 3; ++k) {
        T->v0[k] = p0[k];
        T->E1[k] = (double)(p1[k] - p0[k]);   /* fl(v1 - v0), the kernel's stored edge */
        T->E2[k] = (double)(p2[k] - p0[k]);
    }
    T->n1E1 = fabs(T->E1[0]) + fabs(T->E1[1]) + fabs(T->E1[2]);
    T->n1E2 = fabs(T->E2[0]) + fabs(T->E2[1]) + fabs(T->E2[2]);
    T->lE1 = sqrt(T->E1[0] * T->E1[0] + T->E1[1] * T->E1[1] + T->E1[2] * T->E1[2]);
    T->lE2 = sqrt(T->E2[0] * T->E2[0] + T->E2[1] * T->E2[1] + T->E2[2] * T->E2[2]);
    T->lmax = T->lE1 > T->lE2 ? T->lE1 : T->lE2;
    T->N[0] = T->E1[1] * T->E2[2] - T->E1[2] * T->E2[1];
    T->N[1] = T->E1[2] * T->E2[0] - T->E1[0] * T->E2[2];
    T->N[2] = T->E1[0] * T->E2[1] - T->E1[1] * T->E2[0];
    T->lN = sqrt(T->N[0] * T->N[0] + T->N[1] * T->N[1] + T->N[2] * T->N[2]);
    for (int k = 0; k < 3; ++k) T->nh[k] = T->lN > 0 ? T->N[k] / T->lN : 0.0;
}

/* Bound W on the distance between the ray's line and a point X of the triangle (inflated by
 * rho) for any ray the float Möller–Trumbore test accepts (DESIGN.md §3 ("Exact cull")).  sb[k] >= |s~_k|
 * (s~ = fl(o - v0)).  omega bounds the in-plane part of w' = w x d (w: X's offset from the
 * line) and |w . n|; the in-plane part of w itself is omega / |cos theta|, and
 * |cos theta| >= (Dist - omega) / R from an anchor point on the line (camera origin / light)
 * at distance Dist from the plane and parameter distance <= R from X.  +inf if Dist <= omega. */
static double tri_omega(const tri_info* T, const double sb[3]) {
    const double Dinf = 1.0 + 0x1p-20;   /* |d_k| of a normalised float direction */
    double H[3], Q[3];
    for (int k = 0; k < 3; ++k) {
        H[k] = Dinf * (T->n1E2 - fabs(T->E2[k]));
        const int j = (k + 1) % 3, l = (k + 2) % 3;
        Q[k] = sb[j] * fabs(T->E1[l]) + sb[l] * fabs(T->E1[j]);
    }
    double sumE1H = 0, sumSH = 0, sumQ = 0;
    for (int k = 0; k < 3; ++k) {
        sumE1H += fabs(T->E1[k]) * H[k];
        sumSH += sb[k] * H[k];
        sumQ += Q[k];
    }
    const double g5 = gam(5);
    const double Wp = g5 * (sumSH + (1 + 4 * U) * sumE1H);
    const double Wg = g5 * ((1 + 4 * U) * sumE1H + Dinf * sumQ);
    if (T->lN <= 0) return INFINITY;
    return (Wp * T->lE1 + Wg * T->lE2) / T->lN * (1 + 1e-9) / (1 - 0x1p-20);
}
static double tri_W(double omega, double Dist, double R) {
    if (!(Dist > omega)) return INFINITY;
    return omega * R / (Dist - omega) * (1 + 1e-9) + omega;
}

/* camera: s~ = fl(o - v0) is the same for every camera ray */
static double tri_margin_camera(const tri_info* T, const float* o) {
    double sb[3], s2 = 0, sd = 0;
    for (int k = 0; k < 3; ++k) {
        const float sf = o[k] - (float)T->v0[k];
        sb[k] = fabs((double)sf);
        s2 += sb[k] * sb[k];
        sd += (double)sf * T->nh[k];
    }
    const double sn = sqrt(s2);
    const double Dist = fabs(sd) * (1 - 1e-12);   /* distance of o' = v0 + s~ from the plane */
    const double R = sn + (1 + 8 * U) * T->lmax;
    const double W = tri_W(tri_omega(T, sb), Dist, R);
    /* rho: X within the triangle inflated by 12u lmax; o' within u|s~| of o */
    return W + 12 * U * T->lmax + U * sn * 1.000001;
}

/* shadow ray toward light L with tmax <= tm: |s~_k| <= (1+u)(tm' + |L_k - v0_k|) */
static double tri_margin_light(const tri_info* T, const float* L, double tm) {
    const double tmp = tm * (1 + 8 * U);
    double sb[3], s2 = 0, lv2 = 0, ld = 0;
    for (int k = 0; k < 3; ++k) {
        const double lv = (double)L[k] - T->v0[k];
        sb[k] = (1 + U) * (tmp + fabs(lv));
        s2 += sb[k] * sb[k];
        lv2 += lv * lv;
        ld += lv * T->nh[k];
    }
    const double sn = sqrt(s2);
    const double epsL = 1.01 * gam(3) * tmp + U * sn;
    const double Dist = fabs(ld) * (1 - 1e-12) - epsL;
    const double R = sqrt(lv2) + (1 + 8 * U) * T->lmax + epsL;
    const double W = tri_W(tri_omega(T, sb), Dist, R);
    return W + 12 * U * T->lmax + U * sn * 1.000001;
}

/* ---------------------------------------------------------------- traversal */
#define NGRID 48
static double grid_t(int j) { return 0.01 * pow(2.0, j * 0.5); }

typedef struct {
    const rtx_mesh* m;
    double* tmn; double* tmx;   /* tight boxes per node (3 each) */
    double* marg;               /* per node margin (camera), or NULL */
    double* mdt;                /* per node t bound (camera, t~ <= 64), or NULL */
    double* lmarg;              /* per node x grid margins for the current light, or NULL */
    double delta;
    double* cone;               /* per node {axis xyz, K}: every triangle below faces away when a.d > K */
    int use_tight;
    uint64_t slabs, tris;
} walk;

static void tight_rec(walk* w, uint32_t ni) {
    const rtx_bvh_node* nd = &w->m->nodes[ni];
    double* mn = w->tmn + 3 * ni; double* mx = w->tmx + 3 * ni;
    for (int k = 0; k < 3; ++k) { mn[k] = INFINITY; mx[k] = -INFINITY; }
    if (nd->idx_count > 0) {
        for (uint32_t i = 0; i < nd->idx_count; i += 3) {
            const float* p0 = &w->m->positions[3 * w->m->indices[nd->first_idx + i]];
            const float* p1 = &w->m->positions[3 * w->m->indices[nd->first_idx + i + 1]];
            const float* p2 = &w->m->positions[3 * w->m->indices[nd->first_idx + i + 2]];
            for (int k = 0; k < 3; ++k) {
                /* the triangle MT tests: v0, v0 + fl(v1 - v0), v0 + fl(v2 - v0) */
                const double c[3] = {p0[k], (double)p0[k] + (double)(p1[k] - p0[k]),
                                     (double)p0[k] + (double)(p2[k] - p0[k])};
                for (int q = 0; q < 3; ++q) {
                    if (c[q] < mn[k]) mn[k] = c[q];
                    if (c[q] > mx[k]) mx[k] = c[q];
                }
            }
        }
    } else {
        tight_rec(w, nd->left_node);
        tight_rec(w, nd->left_node + 1);
        for (uint32_t c = nd->left_node; c <= nd->left_node + 1; ++c)
            for (int k = 0; k < 3; ++k) {
                if (w->tmn[3 * c + k] < mn[k]) mn[k] = w->tmn[3 * c + k];
                if (w->tmx[3 * c + k] > mx[k]) mx[k] = w->tmx[3 * c + k];
            }
    }
}

/* UNSOUND measurement knob (cull_probe_cap): triangle margins above `g_cap` are clipped to it,
   to price the heavy tail of the margin distribution (mismatches may then appear) */
static double g_cap = INFINITY;
void cull_probe_cap(double cap) { g_cap = cap; }
/* per node margin = max over its triangles (camera: one value; light: NGRID values) */
static void margin_rec(walk* w, uint32_t ni, const float* cam, const float* L) {
    const rtx_bvh_node* nd = &w->m->nodes[ni];
    if (nd->idx_count > 0) {
        if (cam) w->marg[ni] = 0;
        if (cam && w->mdt) w->mdt[ni] = 0;
        if (L) for (int j = 0; j < NGRID; ++j) w->lmarg[(size_t)ni * NGRID + j] = 0;
        for (uint32_t i = 0; i < nd->idx_count; i += 3) {
            tri_info T;
            tri_setup(&T, &w->m->positions[3 * w->m->indices[nd->first_idx + i]],
                      &w->m->positions[3 * w->m->indices[nd->first_idx + i + 1]],
                      &w->m->positions[3 * w->m->indices[nd->first_idx + i + 2]]);
            if (cam) {
                const double g = fmin(tri_margin_camera(&T, cam), g_cap);
                if (!(g <= w->marg[ni])) w->marg[ni] = g;
                if (w->mdt) {
                    rtx_cull_tri Tc;
                    const float* p0 = &w->m->positions[3 * w->m->indices[nd->first_idx + i]];
                    const float* p1 = &w->m->positions[3 * w->m->indices[nd->first_idx + i + 1]];
                    const float* p2 = &w->m->positions[3 * w->m->indices[nd->first_idx + i + 2]];
                    const float e1[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
                    const float e2[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
                    rtx_cull_tri_setup(&Tc, p0, e1, e2);
                    const double dt = rtx_cull_point_bounds(&Tc, cam, 64.0).dt;
                    if (!(dt <= w->mdt[ni])) w->mdt[ni] = dt;
                }
            }
            if (L)
                for (int j = 0; j < NGRID; ++j) {
                    const double g = fmin(tri_margin_light(&T, L, grid_t(j)), g_cap);
                    double* x = &w->lmarg[(size_t)ni * NGRID + j];
                    if (!(g <= *x)) *x = g;
                }
        }
    } else {
        margin_rec(w, nd->left_node, cam, L);
        margin_rec(w, nd->left_node + 1, cam, L);
        const uint32_t a = nd->left_node, b = nd->left_node + 1;
        if (cam) w->marg[ni] = fmax(w->marg[a], w->marg[b]);
        if (cam && w->mdt) w->mdt[ni] = (w->mdt[a] >= w->mdt[b] || w->mdt[a] != w->mdt[a]) ? w->mdt[a] : w->mdt[b];
        if (L)
            for (int j = 0; j < NGRID; ++j)
                w->lmarg[(size_t)ni * NGRID + j] =
                    fmax(w->lmarg[(size_t)a * NGRID + j], w->lmarg[(size_t)b * NGRID + j]);
    }
}

static int g_fixed_grid = -1;   /* >= 0: every shadow ray uses this grid tmax */
static double node_margin(const walk* w, uint32_t ni, const ray* r, int shadow) {
    if (w->delta >= 0) return w->delta;
    if (!shadow) return w->marg[ni];
    if (g_fixed_grid >= 0) return w->lmarg[(size_t)ni * NGRID + g_fixed_grid];
    int j = 0;
    while (j < NGRID - 1 && grid_t(j) < r->tmax) ++j;
    if (grid_t(j) < r->tmax) return INFINITY;
    return w->lmarg[(size_t)ni * NGRID + j];
}

/* entry parameter of the line into box [mn - dl, mx + dl] (+inf: misses) */
static double enter_t(const double* mn, const double* mx, double dl, const ray* r) {
    const double o[3] = {r->o.x, r->o.y, r->o.z}, d[3] = {r->d.x, r->d.y, r->d.z};
    double t0 = -INFINITY, t1 = INFINITY;
    for (int k = 0; k < 3; ++k) {
        const double lo = mn[k] - dl, hi = mx[k] + dl;
        if (d[k] == 0.0) {
            if (o[k] < lo || o[k] > hi) return INFINITY;
            continue;
        }
        double a = (lo - o[k]) / d[k], b = (hi - o[k]) / d[k];
        if (a > b) { const double x = a; a = b; b = x; }
        if (a > t0) t0 = a;
        if (b < t1) t1 = b;
        if (t0 > t1) return INFINITY;
    }
    return t0;
}
/* Normal-cone skip (probe of a DESIGN §9 idea): a back-face-culled mesh rejects a triangle with
   fl(n.d) > 0 (front-face: < 0; shadow rays swap), so a node whose every normal is within theta of
   axis a can be skipped by a ray with a.d > sin(theta + delta) + 1e-6 (delta = 1e-5 covers the
   float dot's error).  g_cone = 1 enables it. */
static int g_cone = 0;
void cull_probe_cone(int on) { g_cone = on; }
static void cone_rec(walk* w, uint32_t ni, uint32_t* first, uint32_t* cnt) {
    const rtx_bvh_node* nd = &w->m->nodes[ni];
    double* c = w->cone + 4 * ni;
    uint32_t f, n;
    if (nd->idx_count > 0) {
        f = nd->first_idx / 3; n = nd->idx_count / 3;
    } else {
        uint32_t f1, n1, f2, n2;
        cone_rec(w, nd->left_node, &f1, &n1);
        cone_rec(w, nd->left_node + 1, &f2, &n2);
        f = f1 < f2 ? f1 : f2; n = (f1 < f2 ? f2 + n2 : f1 + n1) - f;
    }
    *first = f; *cnt = n;
    double a[3] = {0, 0, 0};
    for (uint32_t t = f; t < f + n; ++t)
        for (int k = 0; k < 3; ++k) a[k] += w->m->normals[3 * t + k];
    const double l = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    c[3] = INFINITY;
    if (!(l > 1e-9)) return;
    for (int k = 0; k < 3; ++k) c[k] = a[k] / l;
    double th = 0;
    for (uint32_t t = f; t < f + n; ++t) {
        const float* nn = &w->m->normals[3 * t];
        const double ln = sqrt((double)nn[0] * nn[0] + (double)nn[1] * nn[1] + (double)nn[2] * nn[2]);
        double cs = (c[0] * nn[0] + c[1] * nn[1] + c[2] * nn[2]) / ln;
        if (!(cs == cs)) return;
        if (cs > 1) cs = 1;
        const double x = acos(cs);
        if (x > th) th = x;
    }
    if (th + 1e-5 < 1.5707963) c[3] = sin(th + 1e-5) + 1e-6;
}
static int cone_skip(const walk* w, uint32_t ni, const ray* r, int shadow) {
    if (!g_cone || !w->cone) return 0;
    int cull = w->m->cull_mode;
    if (cull == RTX_CULL_NONE) return 0;
    if (shadow) cull = cull == RTX_CULL_BACK ? RTX_CULL_FRONT : RTX_CULL_BACK;
    const double* c = w->cone + 4 * ni;
    const double ad = c[0] * r->d.x + c[1] * r->d.y + c[2] * r->d.z;
    return cull == RTX_CULL_BACK ? ad > c[3] : -ad > c[3];
}
static int g_ordered = 0;     /* 1: nearest child first + t pruning (closest-hit), 2: also shadow rays ordered */
static double g_tslack = 1e-3;
void cull_probe_ordered(int o, double slack) { g_ordered = o; g_tslack = slack; }

static void visit(walk* w, uint32_t ni, const ray* r, int ignore, int* did, float* bt, int* bi) {
    if (ignore && *did) return;
    const rtx_bvh_node* nd = &w->m->nodes[ni];
    w->slabs++;
    if (!slab(nd->min, nd->max, r)) return;
    if (cone_skip(w, ni, r, ignore)) return;
    if (w->use_tight) {
        const double g = node_margin(w, ni, r, ignore);
        if (isfinite(g) && !meets(w->tmn + 3 * ni, w->tmx + 3 * ni, g, r)) return;
        const double slack = (g_tslack < 0 && w->mdt) ? w->mdt[ni] : g_tslack;
        if (g_ordered && !ignore && isfinite(g) && *bt < 64.f && isfinite(slack) &&
            enter_t(w->tmn + 3 * ni, w->tmx + 3 * ni, g, r) - slack > *bt)
            return;   /* every triangle below would give t > best */
    }
    if (nd->idx_count > 0) {
        for (uint32_t i = 0; i < nd->idx_count; i += 3) {
            const int li = (int)(nd->first_idx + i);
            const rtx_mesh* m = w->m;
            const v3 v0 = ld3(&m->positions[3 * m->indices[li]]);
            const v3 v1 = ld3(&m->positions[3 * m->indices[li + 1]]);
            const v3 v2 = ld3(&m->positions[3 * m->indices[li + 2]]);
            const v3 n = ld3(&m->normals[3 * (li / 3)]);
            float t;
            w->tris++;
            if (tri(v0, v1, v2, n, m->cull_mode, r, ignore, &t)) {
                *did = 1;
                if (ignore) return;
                if (t < *bt || (t == *bt && li < *bi)) { *bt = t; *bi = li; }
            }
        }
    } else {
        uint32_t a = nd->left_node, b = nd->left_node + 1;
        if (w->use_tight && g_ordered && (!ignore || g_ordered == 2)) {
            const double ga = node_margin(w, a, r, ignore), gb = node_margin(w, b, r, ignore);
            const double ta = enter_t(w->tmn + 3 * a, w->tmx + 3 * a, isfinite(ga) ? ga : 0, r);
            const double tb = enter_t(w->tmn + 3 * b, w->tmx + 3 * b, isfinite(gb) ? gb : 0, r);
            if (tb < ta) { const uint32_t x = a; a = b; b = x; }
        }
        visit(w, a, r, ignore, did, bt, bi);
        visit(w, b, r, ignore, did, bt, bi);
    }
}

/* out[0..9]: ref slabs, ref tris, cull slabs, cull tris, mismatching rays, rays,
 *            shadow share of ref slabs, shadow share of cull slabs, shadow ref tris, shadow cull tris
 * delta >= 0: fixed margin; delta < 0: the per-triangle bounds. */
void cull_probe_fixed_grid(int j) { g_fixed_grid = j; }
int cull_probe(const rtx_scene* sc, const rtx_camera* cam, uint32_t W, uint32_t H, uint32_t step, double delta,
               uint64_t* out) {
    memset(out, 0, 10 * sizeof(uint64_t));
    if (sc->n_meshes != 1 || sc->n_lights > 16) return -1;
    const rtx_mesh* m = &sc->meshes[0];
    walk a, b;
    memset(&a, 0, sizeof a);
    a.m = m;
    a.tmn = (double*)malloc(sizeof(double) * 3 * m->n_nodes);
    a.tmx = (double*)malloc(sizeof(double) * 3 * m->n_nodes);
    tight_rec(&a, 0);
    b = a; b.use_tight = delta != 0.0; b.delta = delta;
    if (g_cone) {
        uint32_t f0, n0;
        b.cone = (double*)malloc(sizeof(double) * 4 * m->n_nodes);
        cone_rec(&b, 0, &f0, &n0);
    }
    double* lm[16] = {0};
    if (delta < 0) {
        b.marg = (double*)malloc(sizeof(double) * m->n_nodes);
        b.mdt = (double*)malloc(sizeof(double) * m->n_nodes);
        margin_rec(&b, 0, cam->origin, NULL);
        for (uint32_t li = 0; li < sc->n_lights; ++li) {
            lm[li] = (double*)malloc(sizeof(double) * NGRID * m->n_nodes);
            b.lmarg = lm[li];
            margin_rec(&b, 0, NULL, sc->lights[li].origin);
        }
    }
    const float aspect = (int)W / (float)(int)H;
    for (uint32_t py = 0; py < H; py += step) {
        for (uint32_t px = 0; px < W; px += step) {
            const float cx = (2.f * (((int)px + 0.5f) / W) - 1) * aspect * cam->fov;
            const float cy = (1.f - (2.f * ((int)py + 0.5f) / H)) * cam->fov;
            v3 vd = mk(cam->right[0] * cx + cam->up[0] * cy + cam->forward[0] * 1.f,
                       cam->right[1] * cx + cam->up[1] * cy + cam->forward[1] * 1.f,
                       cam->right[2] * cx + cam->up[2] * cy + cam->forward[2] * 1.f);
            const float mg = sqrtf(vd.x * vd.x + vd.y * vd.y + vd.z * vd.z);
            vd.x /= mg; vd.y /= mg; vd.z /= mg;
            const ray vr = mkray(ld3(cam->origin), vd, 0.0001f, FLT_MAX);
            int da = 0, db = 0, ia = -1, ib = -1;
            float ta = FLT_MAX, tb = FLT_MAX;
            visit(&a, 0, &vr, 0, &da, &ta, &ia);
            visit(&b, 0, &vr, 0, &db, &tb, &ib);
            out[5]++;
            if (da != db || ia != ib || ta != tb) { out[4]++; continue; }
            if (!da) continue;
            /* shadow rays from the mesh hit (planes ignored: the probe looks at the mesh only) */
            const v3 n = ld3(&m->normals[3 * (ia / 3)]);
            const v3 P = add(vr.o, scale(vr.d, ta));
            const v3 oo = add(P, scale(n, 0.0001f));
            const uint64_t sa0 = a.slabs, sb0 = b.slabs, ta0 = a.tris, tb0 = b.tris;
            for (uint32_t li = 0; li < sc->n_lights; ++li) {
                v3 ld = sub(ld3(sc->lights[li].origin), oo);
                const float mag = sqrtf(ld.x * ld.x + ld.y * ld.y + ld.z * ld.z);
                ld.x /= mag; ld.y /= mag; ld.z /= mag;
                const ray sr = mkray(oo, ld, 0.0001f, mag);
                int sa = 0, sb = 0, xa = -1, xb = -1;
                float fa = FLT_MAX, fb = FLT_MAX;
                b.lmarg = lm[li];
                visit(&a, 0, &sr, 1, &sa, &fa, &xa);
                visit(&b, 0, &sr, 1, &sb, &fb, &xb);
                out[5]++;
                if (sa != sb) out[4]++;
            }
            out[6] += a.slabs - sa0;
            out[7] += b.slabs - sb0;
            out[8] += a.tris - ta0;
            out[9] += b.tris - tb0;
        }
    }
    out[0] = a.slabs; out[1] = a.tris; out[2] = b.slabs; out[3] = b.tris;
    free(a.tmn); free(a.tmx); free(b.marg); free(b.mdt); free(b.cone);
    for (int li = 0; li < 16; ++li) free(lm[li]);
    return 0;
}

/* per-triangle margins for the camera and light 0 at tmax tm: for histograms */
int cull_margins(const rtx_scene* sc, const rtx_camera* cam, double tm, double* out_cam, double* out_light) {
    const rtx_mesh* m = &sc->meshes[0];
    for (uint32_t i = 0; i < m->n_indices; i += 3) {
        tri_info T;
        tri_setup(&T, &m->positions[3 * m->indices[i]], &m->positions[3 * m->indices[i + 1]],
                  &m->positions[3 * m->indices[i + 2]]);
        out_cam[i / 3] = tri_margin_camera(&T, cam->origin);
        out_light[i / 3] = tri_margin_light(&T, sc->lights[0].origin, tm);
    }
    return 0;
}

/* Per-pixel cost map of the culled, ordered walk (the product's traversal rules), planes included:
 * for every step-th pixel, the slab + triangle tests of its primary ray (closest of planes and the
 * mesh) and of the shadow rays toward every light from that hit (mesh only; planes are O(1)).
 * out_p / out_s: primary / shadow tests per sampled pixel, row-major (W/step x H/step).
 * A wave's cost is roughly the union of its 64 lanes' visits, between the max and the sum of
 * these per-pixel counts. */
int cull_probe_cost_map(const rtx_scene* sc, const rtx_camera* cam, uint32_t W, uint32_t H, uint32_t step,
                        uint32_t* out_p, uint32_t* out_s) {
    if (sc->n_meshes != 1 || sc->n_lights > 16) return -1;
    const rtx_mesh* m = &sc->meshes[0];
    walk b;
    memset(&b, 0, sizeof b);
    b.m = m;
    b.tmn = (double*)malloc(sizeof(double) * 3 * m->n_nodes);
    b.tmx = (double*)malloc(sizeof(double) * 3 * m->n_nodes);
    tight_rec(&b, 0);
    b.use_tight = 1;
    b.delta = -1;
    b.marg = (double*)malloc(sizeof(double) * m->n_nodes);
    b.mdt = (double*)malloc(sizeof(double) * m->n_nodes);
    margin_rec(&b, 0, cam->origin, NULL);
    double* lm[16] = {0};
    for (uint32_t li = 0; li < sc->n_lights; ++li) {
        lm[li] = (double*)malloc(sizeof(double) * NGRID * m->n_nodes);
        b.lmarg = lm[li];
        margin_rec(&b, 0, NULL, sc->lights[li].origin);
    }
    const float aspect = (int)W / (float)(int)H;
    uint32_t k = 0;
    for (uint32_t py = 0; py < H; py += step) {
        for (uint32_t px = 0; px < W; px += step, ++k) {
            const float cx = (2.f * (((int)px + 0.5f) / W) - 1) * aspect * cam->fov;
            const float cy = (1.f - (2.f * ((int)py + 0.5f) / H)) * cam->fov;
            v3 vd = mk(cam->right[0] * cx + cam->up[0] * cy + cam->forward[0] * 1.f,
                       cam->right[1] * cx + cam->up[1] * cy + cam->forward[1] * 1.f,
                       cam->right[2] * cx + cam->up[2] * cy + cam->forward[2] * 1.f);
            const float mg = sqrtf(vd.x * vd.x + vd.y * vd.y + vd.z * vd.z);
            vd.x /= mg; vd.y /= mg; vd.z /= mg;
            const ray vr = mkray(ld3(cam->origin), vd, 0.0001f, FLT_MAX);
            /* planes first: the scratch t the mesh walk starts from */
            float bt = FLT_MAX;
            v3 nrm = mk(0, 1, 0);
            for (uint32_t i = 0; i < sc->n_planes; ++i) {
                const v3 p0 = ld3(sc->planes[i].origin), pn = ld3(sc->planes[i].normal);
                const float t = dot(sub(p0, vr.o), pn) / dot(vr.d, pn);
                if (t >= vr.tmin && t < vr.tmax && t < bt) { bt = t; nrm = pn; }
            }
            int did = 0, bi = -1;
            const float bt0 = bt;
            b.slabs = b.tris = 0;
            visit(&b, 0, &vr, 0, &did, &bt, &bi);
            out_p[k] = (uint32_t)(b.slabs + b.tris);
            if (bi >= 0 && bt < bt0) nrm = ld3(&m->normals[3 * (bi / 3)]);
            out_s[k] = 0;
            if (bt >= FLT_MAX) continue;
            const v3 P = add(vr.o, scale(vr.d, bt));
            const v3 oo = add(P, scale(nrm, 0.0001f));
            b.slabs = b.tris = 0;
            for (uint32_t li = 0; li < sc->n_lights; ++li) {
                v3 ld = sub(ld3(sc->lights[li].origin), oo);
                const float mag = sqrtf(ld.x * ld.x + ld.y * ld.y + ld.z * ld.z);
                ld.x /= mag; ld.y /= mag; ld.z /= mag;
                const ray sr = mkray(oo, ld, 0.0001f, mag);
                int sd = 0, xi = -1;
                float ft = FLT_MAX;
                b.lmarg = lm[li];
                visit(&b, 0, &sr, 1, &sd, &ft, &xi);
            }
            out_s[k] = (uint32_t)(b.slabs + b.tris);
        }
    }
    free(b.tmn); free(b.tmx); free(b.marg); free(b.mdt);
    for (int li = 0; li < 16; ++li) free(lm[li]);
    return 0;
}

/* Wave-packet coherence (DESIGN §3, 128-ray packets): the reference traversal (no cull) of every
 * pixel's primary ray and its shadow rays, with the visited nodes of each tile of tw x th pixels
 * collected in a bitset: out[0] = sum over tiles of |union of primary visits| (node tests a packet
 * walking the union would make), out[1] = the same for the shadow rays (per light), out[2] =
 * per-ray primary visits summed, out[3] = per-ray shadow visits summed, out[4] = tiles. */
static uint8_t* g_mark = NULL;
static void visit_mark(const rtx_mesh* m, uint32_t ni, const ray* r, int ignore, int* did, float* bt, uint64_t* cnt) {
    if (ignore && *did) return;
    const rtx_bvh_node* nd = &m->nodes[ni];
    ++*cnt;
    g_mark[ni] = 1;
    if (!slab(nd->min, nd->max, r)) return;
    if (nd->idx_count > 0) {
        for (uint32_t i = 0; i < nd->idx_count; i += 3) {
            const int li = (int)(nd->first_idx + i);
            const v3 v0 = ld3(&m->positions[3 * m->indices[li]]);
            const v3 v1 = ld3(&m->positions[3 * m->indices[li + 1]]);
            const v3 v2 = ld3(&m->positions[3 * m->indices[li + 2]]);
            const v3 n = ld3(&m->normals[3 * (li / 3)]);
            float t;
            if (tri(v0, v1, v2, n, m->cull_mode, r, ignore, &t)) {
                *did = 1;
                if (ignore) return;
                if (t < *bt) *bt = t;
            }
        }
    } else {
        visit_mark(m, nd->left_node, r, ignore, did, bt, cnt);
        visit_mark(m, nd->left_node + 1, r, ignore, did, bt, cnt);
    }
}
int cull_probe_packet_union(const rtx_scene* sc, const rtx_camera* cam, uint32_t W, uint32_t H, uint32_t tw,
                            uint32_t th, uint64_t* out) {
    if (sc->n_meshes != 1 || sc->n_lights > 16) return -1;
    const rtx_mesh* m = &sc->meshes[0];
    memset(out, 0, 5 * sizeof(uint64_t));
    uint8_t* um = (uint8_t*)malloc(m->n_nodes);
    g_mark = (uint8_t*)malloc(m->n_nodes);
    const float aspect = (int)W / (float)(int)H;
    for (uint32_t ty = 0; ty + th <= H; ty += th)
        for (uint32_t tx = 0; tx + tw <= W; tx += tw) {
            for (int pass = 0; pass < 1 + (int)sc->n_lights; ++pass) {
                memset(um, 0, m->n_nodes);
                for (uint32_t py = ty; py < ty + th; ++py)
                    for (uint32_t px = tx; px < tx + tw; ++px) {
                        const float cx = (2.f * (((int)px + 0.5f) / W) - 1) * aspect * cam->fov;
                        const float cy = (1.f - (2.f * ((int)py + 0.5f) / H)) * cam->fov;
                        v3 vd = mk(cam->right[0] * cx + cam->up[0] * cy + cam->forward[0] * 1.f,
                                   cam->right[1] * cx + cam->up[1] * cy + cam->forward[1] * 1.f,
                                   cam->right[2] * cx + cam->up[2] * cy + cam->forward[2] * 1.f);
                        const float mg = sqrtf(vd.x * vd.x + vd.y * vd.y + vd.z * vd.z);
                        vd.x /= mg; vd.y /= mg; vd.z /= mg;
                        const ray vr = mkray(ld3(cam->origin), vd, 0.0001f, FLT_MAX);
                        float bt = FLT_MAX;
                        v3 nrm = mk(0, 1, 0);
                        for (uint32_t i = 0; i < sc->n_planes; ++i) {
                            const v3 p0 = ld3(sc->planes[i].origin), pn = ld3(sc->planes[i].normal);
                            const float t = dot(sub(p0, vr.o), pn) / dot(vr.d, pn);
                            if (t >= vr.tmin && t < vr.tmax && t < bt) { bt = t; nrm = pn; }
                        }
                        int did = 0;
                        uint64_t c = 0;
                        memset(g_mark, 0, m->n_nodes);
                        const float bt0 = bt;
                        visit_mark(m, 0, &vr, 0, &did, &bt, &c);
                        if (pass == 0) {
                            out[2] += c;
                            for (uint32_t i = 0; i < m->n_nodes; ++i) um[i] |= g_mark[i];
                            continue;
                        }
                        if (bt >= FLT_MAX) continue;
                        (void)bt0;
                        const v3 P = add(vr.o, scale(vr.d, bt));
                        const v3 oo = add(P, scale(nrm, 0.0001f));
                        const uint32_t li = (uint32_t)pass - 1;
                        v3 ld = sub(ld3(sc->lights[li].origin), oo);
                        const float mag = sqrtf(ld.x * ld.x + ld.y * ld.y + ld.z * ld.z);
                        ld.x /= mag; ld.y /= mag; ld.z /= mag;
                        const ray sr = mkray(oo, ld, 0.0001f, mag);
                        int sd = 0;
                        float ft = FLT_MAX;
                        c = 0;
                        memset(g_mark, 0, m->n_nodes);
                        visit_mark(m, 0, &sr, 1, &sd, &ft, &c);
                        out[3] += c;
                        for (uint32_t i = 0; i < m->n_nodes; ++i) um[i] |= g_mark[i];
                    }
                uint64_t u = 0;
                for (uint32_t i = 0; i < m->n_nodes; ++i) u += um[i];
                out[pass == 0 ? 0 : 1] += u;
            }
            out[4]++;
        }
    free(um);
    free(g_mark);
    g_mark = NULL;
    return 0;
}

/* Shadow-hull skip estimate: per (tile of tw x th pixels, light), the shadow rays' union of reference
 * node visits (as cull_probe_packet_union), and whether the AABB of the tile's shadow origins and
 * the light misses the mesh's tight box grown by `grow` (then no shadow ray of the tile can hit the
 * mesh: the wave could skip that light's mesh walk).  out[0] = shadow union visits, out[1] = those in
 * (tile, light) pairs the hull test skips, out[2] = pairs with a shadow ray, out[3] = pairs skipped. */
int cull_probe_shadow_hull(const rtx_scene* sc, const rtx_camera* cam, uint32_t W, uint32_t H, uint32_t tw,
                           uint32_t th, double grow, uint64_t* out) {
    if (sc->n_meshes != 1 || sc->n_lights > 16) return -1;
    const rtx_mesh* m = &sc->meshes[0];
    memset(out, 0, 4 * sizeof(uint64_t));
    double bmn[3] = {INFINITY, INFINITY, INFINITY}, bmx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < m->n_indices; ++i)
        for (int k = 0; k < 3; ++k) {
            const double v = m->positions[3 * m->indices[i] + k];
            if (v < bmn[k]) bmn[k] = v;
            if (v > bmx[k]) bmx[k] = v;
        }
    uint8_t* um = (uint8_t*)malloc(m->n_nodes);
    g_mark = (uint8_t*)malloc(m->n_nodes);
    const float aspect = (int)W / (float)(int)H;
    const uint32_t npx = tw * th;
    v3* oo = (v3*)malloc(sizeof(v3) * npx);
    int* hit = (int*)malloc(sizeof(int) * npx);
    for (uint32_t ty = 0; ty + th <= H; ty += th)
        for (uint32_t tx = 0; tx + tw <= W; tx += tw) {
            uint32_t q = 0;
            for (uint32_t py = ty; py < ty + th; ++py)
                for (uint32_t px = tx; px < tx + tw; ++px, ++q) {
                    const float cx = (2.f * (((int)px + 0.5f) / W) - 1) * aspect * cam->fov;
                    const float cy = (1.f - (2.f * ((int)py + 0.5f) / H)) * cam->fov;
                    v3 vd = mk(cam->right[0] * cx + cam->up[0] * cy + cam->forward[0] * 1.f,
                               cam->right[1] * cx + cam->up[1] * cy + cam->forward[1] * 1.f,
                               cam->right[2] * cx + cam->up[2] * cy + cam->forward[2] * 1.f);
                    const float mg = sqrtf(vd.x * vd.x + vd.y * vd.y + vd.z * vd.z);
                    vd.x /= mg; vd.y /= mg; vd.z /= mg;
                    const ray vr = mkray(ld3(cam->origin), vd, 0.0001f, FLT_MAX);
                    float bt = FLT_MAX;
                    v3 nrm = mk(0, 1, 0);
                    for (uint32_t i = 0; i < sc->n_planes; ++i) {
                        const v3 p0 = ld3(sc->planes[i].origin), pn = ld3(sc->planes[i].normal);
                        const float t = dot(sub(p0, vr.o), pn) / dot(vr.d, pn);
                        if (t >= vr.tmin && t < vr.tmax && t < bt) { bt = t; nrm = pn; }
                    }
                    int did = 0;
                    uint64_t c = 0;
                    const float bt0 = bt;
                    visit_mark(m, 0, &vr, 0, &did, &bt, &c);
                    hit[q] = bt < FLT_MAX;
                    if (bt < bt0) {   /* the mesh hit's normal: find the triangle again (probe only) */
                        nrm = mk(0, 0, 0);
                        for (uint32_t i = 0; i < m->n_indices; i += 3) {
                            float t;
                            const v3 v0 = ld3(&m->positions[3 * m->indices[i]]);
                            const v3 v1 = ld3(&m->positions[3 * m->indices[i + 1]]);
                            const v3 v2 = ld3(&m->positions[3 * m->indices[i + 2]]);
                            const v3 n = ld3(&m->normals[3 * (i / 3)]);
                            if (tri(v0, v1, v2, n, m->cull_mode, &vr, 0, &t) && t == bt) { nrm = n; break; }
                        }
                    }
                    oo[q] = add(add(vr.o, scale(vr.d, bt)), scale(nrm, 0.0001f));
                }
            for (uint32_t li = 0; li < sc->n_lights; ++li) {
                const v3 L = ld3(sc->lights[li].origin);
                double hmn[3] = {L.x, L.y, L.z}, hmx[3] = {L.x, L.y, L.z};
                int any = 0;
                memset(um, 0, m->n_nodes);
                for (uint32_t k = 0; k < npx; ++k) {
                    if (!hit[k]) continue;
                    any = 1;
                    const double o[3] = {oo[k].x, oo[k].y, oo[k].z};
                    for (int a = 0; a < 3; ++a) { if (o[a] < hmn[a]) hmn[a] = o[a]; if (o[a] > hmx[a]) hmx[a] = o[a]; }
                    v3 ld = sub(L, oo[k]);
                    const float mag = sqrtf(ld.x * ld.x + ld.y * ld.y + ld.z * ld.z);
                    ld.x /= mag; ld.y /= mag; ld.z /= mag;
                    const ray sr = mkray(oo[k], ld, 0.0001f, mag);
                    int sd = 0;
                    float ft = FLT_MAX;
                    uint64_t c = 0;
                    memset(g_mark, 0, m->n_nodes);
                    visit_mark(m, 0, &sr, 1, &sd, &ft, &c);
                    for (uint32_t i = 0; i < m->n_nodes; ++i) um[i] |= g_mark[i];
                }
                if (!any) continue;
                uint64_t u = 0;
                for (uint32_t i = 0; i < m->n_nodes; ++i) u += um[i];
                int miss = 0;
                for (int a = 0; a < 3; ++a) miss |= hmx[a] < bmn[a] - grow || hmn[a] > bmx[a] + grow;
                out[0] += u;
                out[2]++;
                if (miss) { out[1] += u; out[3]++; }
            }
        }
    free(um); free(g_mark); g_mark = NULL; free(oo); free(hit);
    return 0;
}
