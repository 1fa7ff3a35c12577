/*
 * mt_graze_search.c — diagnostic for DESIGN.md §3 ("Exact cull") (never product, never a checker).
 *
 * Question: can the reference's float Möller–Trumbore (Utils.h:109-184, binary32, no FMA)
 * accept a ray whose exact line passes FAR from the triangle?  If it can, a BVH cull that
 * skips a node because the ray misses the node's tight box by a fixed margin is not exact.
 *
 * Search: a Synthetic100k-like sliver triangle (grid step 0.024 x 0.02, height steps up to
 * 0.5); a target point P on the triangle's plane at in-plane distance X outside the triangle;
 * a ray direction d inside the plane, tilted out of it by a tiny angle, and an origin o at
 * distance ~10 before P (the camera's distance).  Count float-MT acceptances and report the
 * largest exact distance (double precision) between the accepted ray's line and the triangle.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../gp1_raytracer_2223_amd/csrc/rtx_cull.h"

typedef struct { float x, y, z; } v3;
static v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 cross(v3 a, v3 b) { return mk(a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x); }

/* HitTest_Triangle with NoCulling: the |normal . d| >= FLT_EPSILON guard (Utils.h:111-112) on the
   face normal normalize(e1 x e2) as TriangleMesh computes it, then Möller–Trumbore (:139-171) */
/* the test's intermediates for an accepted ray (mt_x) */
typedef struct { float a, alpha, beta, t; v3 s; } mt_vals;
static mt_vals g_last;
static int mt(v3 v0, v3 v1, v3 v2, v3 o, v3 d, float tmin, float tmax) {
    const v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    v3 nn = cross(e1, e2);
    const float nm = sqrtf(nn.x * nn.x + nn.y * nn.y + nn.z * nn.z);
    nn.x /= nm; nn.y /= nm; nn.z /= nm;
    if (fabsf(dot(nn, d)) < FLT_EPSILON) return 0;
    const v3 h = cross(d, e2);
    const float a = dot(e1, h);
    if (fabsf(a) < FLT_EPSILON) return 0;
    const float ai = 1.f / a;
    const v3 s = sub(o, v0);
    const float u = ai * dot(s, h);
    if (u < 0.f || u > 1.f) return 0;
    const v3 q = cross(s, e1);
    const float v = ai * dot(d, q);
    if (v < 0.f || (u + v) > 1.f) return 0;
    const float t = ai * dot(e2, q);
    if (t < tmin || t >= tmax) return 0;
    g_last.a = a; g_last.alpha = dot(s, h); g_last.beta = dot(d, q); g_last.t = t; g_last.s = s;
    return 1;
}

/* For the accepted ray of the last mt(): X = v0 + (alpha~/a~) E1 + (beta~/a~) E2, its distance to
   the line through o' = v0 + s~ along d, and t* (the line parameter of the point nearest X). */
static void x_check(v3 v0, v3 v1, v3 v2, v3 d, double* dist_x, double* tstar) {
    const v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    const double U = (double)g_last.alpha / g_last.a, V = (double)g_last.beta / g_last.a;
    const double X[3] = {v0.x + U * e1.x + V * e2.x, v0.y + U * e1.y + V * e2.y, v0.z + U * e1.z + V * e2.z};
    const double O[3] = {(double)v0.x + g_last.s.x, (double)v0.y + g_last.s.y, (double)v0.z + g_last.s.z};
    const double D[3] = {d.x, d.y, d.z};
    const double dd = D[0] * D[0] + D[1] * D[1] + D[2] * D[2];
    const double ts = ((X[0] - O[0]) * D[0] + (X[1] - O[1]) * D[1] + (X[2] - O[2]) * D[2]) / dd;
    double r2 = 0;
    for (int k = 0; k < 3; ++k) {
        const double w = X[k] - (O[k] + ts * D[k]);
        r2 += w * w;
    }
    *dist_x = sqrt(r2);
    *tstar = ts;
}

typedef struct { double x, y, z; } d3;
static d3 D(v3 a) { d3 r = {a.x, a.y, a.z}; return r; }
static d3 dsub(d3 a, d3 b) { d3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static d3 dadd(d3 a, d3 b) { d3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static d3 dsc(d3 a, double s) { d3 r = {a.x * s, a.y * s, a.z * s}; return r; }
static double ddot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static d3 dcross(d3 a, d3 b) { d3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; return r; }
static double dlen(d3 a) { return sqrt(ddot(a, a)); }

/* distance from point p to segment ab */
static double pseg(d3 p, d3 a, d3 b) {
    const d3 ab = dsub(b, a);
    double t = ddot(dsub(p, a), ab) / ddot(ab, ab);
    if (t < 0) t = 0;
    if (t > 1) t = 1;
    return dlen(dsub(p, dadd(a, dsc(ab, t))));
}
/* distance between the line (o, d) and the triangle (sampled: closest point search) */
static double line_tri(d3 o, d3 d, d3 A, d3 B, d3 C) {
    /* the closest point of the line to the triangle lies at the line's closest approach to
       an edge or crosses the interior; sample the line parameter finely around the plane */
    d3 n = dcross(dsub(B, A), dsub(C, A));
    const double nl = dlen(n);
    n = dsc(n, 1.0 / nl);
    double best = 1e300;
    /* closest approach to each edge line segment */
    const d3 P[3] = {A, B, C};
    for (int e = 0; e < 3; ++e) {
        const d3 a = P[e], b = P[(e + 1) % 3];
        /* minimise |o + t d - seg(s)| over t, s by coarse-to-fine 1D search on s */
        double lo = 0, hi = 1;
        for (int it = 0; it < 200; ++it) {
            const double s1 = lo + (hi - lo) / 3, s2 = hi - (hi - lo) / 3;
            const d3 q1 = dadd(a, dsc(dsub(b, a), s1)), q2 = dadd(a, dsc(dsub(b, a), s2));
            const d3 w1 = dsub(q1, o), w2 = dsub(q2, o);
            const double f1 = dlen(dsub(w1, dsc(d, ddot(w1, d) / ddot(d, d))));
            const double f2 = dlen(dsub(w2, dsc(d, ddot(w2, d) / ddot(d, d))));
            if (f1 < f2) hi = s2; else lo = s1;
        }
        const d3 q = dadd(a, dsc(dsub(b, a), 0.5 * (lo + hi)));
        const d3 w = dsub(q, o);
        const double f = dlen(dsub(w, dsc(d, ddot(w, d) / ddot(d, d))));
        if (f < best) best = f;
    }
    /* crossing the interior: exact plane intersection inside => distance 0 */
    const double dn = ddot(d, n);
    if (dn != 0) {
        const double t = ddot(dsub(A, o), n) / dn;
        const d3 X = dadd(o, dsc(d, t));
        const d3 e0 = dsub(B, A), e1 = dsub(C, A), w = dsub(X, A);
        const double d00 = ddot(e0, e0), d01 = ddot(e0, e1), d11 = ddot(e1, e1), d20 = ddot(w, e0), d21 = ddot(w, e1);
        const double den = d00 * d11 - d01 * d01;
        const double v = (d11 * d20 - d01 * d21) / den, u2 = (d00 * d21 - d01 * d20) / den;
        if (v >= 0 && u2 >= 0 && v + u2 <= 1) best = 0;
    }
    (void)pseg;
    return best;
}

static double urand(void) { return (double)rand() / RAND_MAX; }

static double margin_camera(v3 v0, v3 v1, v3 v2, v3 o) {
    const v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    rtx_cull_tri T;
    rtx_cull_tri_setup(&T, &v0.x, &e1.x, &e2.x);
    return rtx_cull_margin_point(&T, &o.x);
}
static double margin_light(v3 v0, v3 v1, v3 v2, v3 L, float tmax) {
    const v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    rtx_cull_tri T;
    rtx_cull_tri_setup(&T, &v0.x, &e1.x, &e2.x);
    return rtx_cull_margin_light(&T, &L.x, tmax);
}

int main(int argc, char** argv) {
    const long trials = argc > 1 ? atol(argv[1]) : 2000000;
    const double size = argc > 2 ? atof(argv[2]) : 1.0;   /* triangle scale */
    const double tilt_decades = argc > 3 ? atof(argv[3]) : 3.0;   /* ray tilt out of the plane: 1e-7 .. 1e(-7+this) */
    srand(12345);
    long acc_far[4] = {0, 0, 0, 0}, acc[4] = {0, 0, 0, 0}, viol = 0, lacc = 0, lviol = 0;
    const double Xs[4] = {0.01, 0.1, 0.5, 2.0};
    double worst[4] = {0, 0, 0, 0}, worst_ratio = 0, worst_lratio = 0, worst_dt = 0;
    for (long it = 0; it < trials; ++it) {
        /* sliver: grid triangle with a steep height step */
        const float x0 = (float)(-3.0 + 6.0 * urand()), z0 = (float)(-1.0 + 4.0 * urand());
        const v3 v0 = mk(x0, (float)(0.3 + 0.5 * size * urand()), z0);
        const v3 v1 = mk(x0, (float)(0.3 + 0.5 * size * urand()), z0 + (float)(0.02 * size));
        const v3 v2 = mk(x0 + (float)(0.024 * size), (float)(0.3 + 0.5 * size * urand()), z0);
        const d3 A = D(v0), B = D(v1), C = D(v2);
        d3 n = dcross(dsub(B, A), dsub(C, A));
        n = dsc(n, 1.0 / dlen(n));
        d3 t1 = dsub(B, A);
        t1 = dsc(t1, 1.0 / dlen(t1));
        const d3 t2 = dcross(n, t1);
        const int k = (int)((it >> 1) % 4);
        const double ang = 2 * M_PI * urand();
        const d3 cen = dsc(dadd(dadd(A, B), C), 1.0 / 3.0);
        const d3 Pt = dadd(cen, dadd(dsc(t1, Xs[k] * cos(ang)), dsc(t2, Xs[k] * sin(ang))));
        const double ang2 = 2 * M_PI * urand();
        const double tilt = pow(10.0, -7.0 + tilt_decades * urand()) * (urand() < 0.5 ? -1 : 1);
        d3 dd = dadd(dadd(dsc(t1, cos(ang2)), dsc(t2, sin(ang2))), dsc(n, tilt));
        dd = dsc(dd, 1.0 / dlen(dd));
        const double off = pow(10.0, -8.0 + 4.0 * urand()) * (urand() < 0.5 ? -1 : 1);
        const double back = 0.5 + 12.0 * urand();
        const d3 Od = dadd(dsub(Pt, dsc(dd, back)), dsc(n, off));
        const v3 o = mk((float)Od.x, (float)Od.y, (float)Od.z);
        if (it & 1) {
            /* camera form: the direction as the reference normalises it */
            v3 d = mk((float)dd.x, (float)dd.y, (float)dd.z);
            const float m = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
            d.x /= m; d.y /= m; d.z /= m;
            if (!mt(v0, v1, v2, o, d, 1e-4f, FLT_MAX)) continue;
            acc[k]++;
            const double dist = line_tri(D(o), D(d), A, B, C);
            const double mg = margin_camera(v0, v1, v2, o);
            if (dist > mg) {
                viol++;
                printf("VIOLATION camera: dist %.6g > margin %.6g\n", dist, mg);
            }
            {   /* the derivation's own quantities: |X - P| <= W and |t~ - t*| <= dt */
                const v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
                rtx_cull_tri T;
                rtx_cull_tri_setup(&T, &v0.x, &e1.x, &e2.x);
                const rtx_cull_bound bd = rtx_cull_point_bounds(&T, &o.x, g_last.t);
                double dx, ts;
                x_check(v0, v1, v2, d, &dx, &ts);
                if (dx > bd.margin || fabs((double)g_last.t - ts) > bd.dt) {
                    viol++;
                    printf("VIOLATION camera X: |X-P| %.6g (W %.6g), |t-t*| %.6g (dt %.6g)\n", dx, bd.margin,
                           fabs((double)g_last.t - ts), bd.dt);
                }
                if (bd.dt > 0 && fabs((double)g_last.t - ts) / bd.dt > worst_dt) worst_dt = fabs((double)g_last.t - ts) / bd.dt;
            }
            if (mg > 0 && dist / mg > worst_ratio) worst_ratio = dist / mg;
            if (dist > worst[k]) {
                worst[k] = dist;
                if (getenv("MT_PRINT"))
                    printf("X %.2f dist %.6g margin %.6g v0 %a %a %a v1 %a %a %a v2 %a %a %a o %a %a %a d %a %a %a\n",
                           Xs[k], dist, mg, v0.x, v0.y, v0.z, v1.x, v1.y, v1.z, v2.x, v2.y, v2.z, o.x, o.y, o.z, d.x,
                           d.y, d.z);
            }
            if (dist > 1e-3) acc_far[k]++;
        } else {
            /* shadow form: a light on the line beyond the target, direction and tmax as
               Renderer.cpp:130-136 computes them */
            const double beyond = 0.1 + 8.0 * urand();
            const d3 Ld = dadd(Pt, dsc(dd, beyond));
            const v3 L = mk((float)Ld.x, (float)Ld.y, (float)Ld.z);
            v3 l = sub(L, o);
            const float mag = sqrtf(l.x * l.x + l.y * l.y + l.z * l.z);
            l.x /= mag; l.y /= mag; l.z /= mag;
            if (!mt(v0, v1, v2, o, l, 1e-4f, mag)) continue;
            lacc++;
            const double dist = line_tri(D(o), D(l), A, B, C);
            const double mg = margin_light(v0, v1, v2, L, mag);
            if (dist > mg) {
                lviol++;
                printf("VIOLATION light: dist %.6g > margin %.6g\n", dist, mg);
            }
            {
                const v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
                rtx_cull_tri T;
                rtx_cull_tri_setup(&T, &v0.x, &e1.x, &e2.x);
                const rtx_cull_bound bd = rtx_cull_light_bounds(&T, &L.x, mag);
                double dx, ts;
                x_check(v0, v1, v2, l, &dx, &ts);
                if (dx > bd.margin || fabs((double)g_last.t - ts) > bd.dt) {
                    lviol++;
                    printf("VIOLATION light X: |X-P| %.6g (W %.6g), |t-t*| %.6g (dt %.6g)\n", dx, bd.margin,
                           fabs((double)g_last.t - ts), bd.dt);
                }
                if (bd.dt > 0 && fabs((double)g_last.t - ts) / bd.dt > worst_dt) worst_dt = fabs((double)g_last.t - ts) / bd.dt;
            }
            if (mg > 0 && dist / mg > worst_lratio) worst_lratio = dist / mg;
        }
    }
    for (int k = 0; k < 4; ++k)
        printf("X %.2f: camera rays accepted %ld, with exact line-triangle distance > 1e-3: %ld; largest distance %.4g\n",
               Xs[k], acc[k], acc_far[k], worst[k]);
    printf("camera: violations %ld, largest distance / margin %.4g\n", viol, worst_ratio);
    printf("shadow: accepted %ld, violations %ld, largest distance / margin %.4g\n", lacc, lviol, worst_lratio);
    printf("t bound: largest |t~ - t*| / dt %.4g\n", worst_dt);
    return (viol || lviol) ? 1 : 0;
}
