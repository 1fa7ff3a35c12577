/* rtx_cull.h — exact pruning bound for the reference's float Möller–Trumbore test.
 *
 * The reference's BVH boxes are inflated by its FLT_MIN-initialised max bound (DataTypes.h:315,
 * SURVEY a15): every box whose triangles lie at negative x (or z) reaches x = 0 (z = 0), so a ray
 * near those planes passes thousands of slab tests for triangles far away.  The render kernel
 * may skip a node the reference would visit only when no triangle below it can be accepted by
 * HitTest_Triangle (Utils.h:109-184) as the reference computes it in binary32 — and a float test
 * can accept a ray whose exact line passes far from the triangle (tools/mt_graze_search.c finds
 * accepted rays 0.36 units from a Synthetic100k-sized triangle).  This header bounds that
 * distance ("Exact cull"):
 *
 *   If HitTest_Triangle accepts (o, d) for the triangle (v0, v0 + E1, v0 + E2) — E1, E2 the
 *   float edges fl(v1 - v0), fl(v2 - v0) it computes — then the line {o + t d} passes within
 *   margin(o, d) of that triangle, where, with u = 2^-24, gamma_n = n u / (1 - n u),
 *   s~ = fl(o - v0), N = E1 x E2, n = N / |N|:
 *     omega  = gamma_5 [ (sum_k (|s~_k| + (1+4u)|E1_k|) H_k) |E1| + ((1+4u) sum_k |E1_k| H_k
 *              + sum_k Q_k) |E2| ] / (|N| (1 - 2^-20)),
 *              H_k = |d_j E2_l| + |d_l E2_j| <= (1+2^-20) (|E2|_1 - |E2_k|),
 *              Q_k = |s~_j E1_l| + |s~_l E1_j|                      ({k, j, l} = {0, 1, 2})
 *     W      = omega + omega R / (Dist - omega)        (+inf unless Dist > omega)
 *     margin = W + 12 u max(|E1|, |E2|) + u |s~|
 *   where Dist is the distance of an anchor point on the line from the triangle's plane and R
 *   bounds the anchor's parameter distance to the accepted point:
 *     camera rays (anchor = the ray origin o' = v0 + s~):  Dist = |s~ . n|, R = |s~| + (1+8u) max|E|
 *     shadow rays toward light L with tmax <= T (anchor = the light, within e_L of the line):
 *       Dist = |(L - v0) . n| - e_L,  R = |L - v0| + (1+8u) max|E| + e_L,
 *       |s~_k| <= (1+u)((1+8u) T + |L_k - v0_k|),  e_L = 1.01 gamma_3 (1+8u) T + u |s~|.
 *
 * Sketch (every step in DESIGN.md §3): the computed u~ = a~^-1 (s~ . h~) and v~ = a~^-1 (d . q~)
 * pass the reference's range tests, so U = alpha~/a~ and V = beta~/a~ lie in the unit simplex
 * widened by 4u and X = v0 + U E1 + V E2 is within 12 u max|E| of the triangle.  Let P be the
 * point of the line nearest X and w = X - P (w . d = 0).  The rounding errors E_a, E_alpha,
 * E_beta of a~, alpha~, beta~ (each <= gamma_5 times the sums above) give exactly
 *     w . (d x E2) = E_alpha - U E_a,      w . (d x E1) = V E_a - E_beta,
 * i.e. w' = w x d has both in-plane dot products with E2 and E1 bounded, so its in-plane part is
 * <= omega |d| and |w . n| <= omega: the line meets the triangle's plane steeply enough that
 * |d . n| >= (Dist - omega) / R, and |w| <= omega (1 + R / (Dist - omega)).  No term divides by
 * the determinant a itself (a grazing ray is bounded through the anchor's distance from the
 * plane instead), which is what makes the bound small for almost every triangle.
 *
 * Written as plain C on doubles (the host probes, tests/ and the device margin kernels share it);
 * every rounding of the double arithmetic is covered by the (1 + 1e-9) factors.
 */
#ifndef RTX_CULL_H
#define RTX_CULL_H

#include <float.h>
#include <math.h>

#if defined(__HIPCC__)
#define RTX_CULL_HD __host__ __device__
#else
#define RTX_CULL_HD
#endif

#define RTX_CULL_U 0x1p-24
/* |d_k| of a normalised float direction, and 1 / |d| for |d| >= 1 - 2^-20 */
#define RTX_CULL_DMAX (1.0 + 0x1p-20)

typedef struct rtx_cull_tri {
    double v0[3], E1[3], E2[3];
    double n1E2;               /* |E2|_1 */
    double lE1, lE2, lmax;     /* 2-norms */
    double lN, nh[3];          /* |E1 x E2| and the unit normal */
    double nerr;               /* bound on the error of nh's direction (radians) */
} rtx_cull_tri;

RTX_CULL_HD static inline double rtx_cull_gamma(int n) { return n * RTX_CULL_U / (1.0 - n * RTX_CULL_U); }

/* v0 and the float edges E1 = fl(v1 - v0), E2 = fl(v2 - v0) the triangle test uses */
RTX_CULL_HD static inline void rtx_cull_tri_setup(rtx_cull_tri* T, const float* v0, const float* e1, const float* e2) {
    for (int k = 0; k < 3; ++k) {
        T->v0[k] = v0[k];
        T->E1[k] = e1[k];
        T->E2[k] = e2[k];
    }
    T->n1E2 = fabs(T->E2[0]) + fabs(T->E2[1]) + fabs(T->E2[2]);
    T->lE1 = sqrt(T->E1[0] * T->E1[0] + T->E1[1] * T->E1[1] + T->E1[2] * T->E1[2]);
    T->lE2 = sqrt(T->E2[0] * T->E2[0] + T->E2[1] * T->E2[1] + T->E2[2] * T->E2[2]);
    T->lmax = T->lE1 > T->lE2 ? T->lE1 : T->lE2;
    /* products of floats are exact in double; each component has one rounding */
    const double N0 = T->E1[1] * T->E2[2] - T->E1[2] * T->E2[1];
    const double N1 = T->E1[2] * T->E2[0] - T->E1[0] * T->E2[2];
    const double N2 = T->E1[0] * T->E2[1] - T->E1[1] * T->E2[0];
    T->lN = sqrt(N0 * N0 + N1 * N1 + N2 * N2);
    const double inv = T->lN > 0 ? 1.0 / T->lN : 0.0;
    T->nh[0] = N0 * inv;
    T->nh[1] = N1 * inv;
    T->nh[2] = N2 * inv;
    /* |N~ - N| <= 2^-52 |E1| |E2| (per component, two roundings of exact products), so the
       direction of nh is off by <= ~4 2^-52 |E1||E2| / |N| plus its own few ulps */
    T->nerr = T->lN > 0 ? 0x1p-48 * (T->lE1 * T->lE2 / T->lN + 1.0) : INFINITY;
}

/* Both bounds of one (anchor, triangle):
 *   margin: the line of any accepted ray passes within `margin` of the triangle (above);
 *   dt:     |t~ - t*| <= dt for any accepted ray whose computed t~ is at most Bt, where t* is the
 *           line parameter of the point nearest to X: t* - tau~/a~ = Y.d / |d|^2
 *           with Y = X - o' - (tau~/a~) d, whose components along d x E2 and d x E1 are those of
 *           w and whose N component is E_tau - (tau~/a~) E_a, so
 *           |t* - tau~/a~| <= (E_tau + Bt' E_a) / (|N| |d| c) + omega / (|d| c^2),
 *           and t~ = fl(fl(1/a~) tau~) is tau~/a~ within 2.01 u t~.
 * Both +inf when no bound closes. */
typedef struct rtx_cull_bound {
    double margin, dt;
} rtx_cull_bound;

RTX_CULL_HD static inline rtx_cull_bound rtx_cull_bounds(const rtx_cull_tri* T, const double* sb, double dist, double R,
                                                        double Bt) {
    rtx_cull_bound b = {INFINITY, INFINITY};
    if (!(T->lN > 0)) return b;
    double sumE1H = 0.0, sumSH = 0.0, sumQ = 0.0, sumE2Q = 0.0;
    for (int k = 0; k < 3; ++k) {
        const int j = (k + 1) % 3, l = (k + 2) % 3;
        const double H = RTX_CULL_DMAX * (T->n1E2 - fabs(T->E2[k]));
        const double Q = sb[j] * fabs(T->E1[l]) + sb[l] * fabs(T->E1[j]);
        sumE1H += fabs(T->E1[k]) * H;
        sumSH += sb[k] * H;
        sumQ += Q;
        sumE2Q += fabs(T->E2[k]) * Q;
    }
    const double g5 = rtx_cull_gamma(5), U = RTX_CULL_U, dlo = 1.0 - 0x1p-20;
    const double Ea = g5 * sumE1H;                                      /* |a~ - a| */
    const double Et = g5 * sumE2Q;                                      /* |tau~ - tau| */
    const double ep = g5 * (sumSH + (1 + 4 * U) * sumE1H);             /* |w . (d x E2)| */
    const double eg = g5 * ((1 + 4 * U) * sumE1H + RTX_CULL_DMAX * sumQ);   /* |w . (d x E1)| */
    const double omega = (ep * T->lE1 + eg * T->lE2) / T->lN * (1.0 + 1e-9) / dlo;
    if (!(dist > omega)) return b;
    const double c = (dist - omega) / R * (1.0 - 1e-12);               /* |cos| of d to the plane, lower bound */
    b.margin = (omega + omega * R / (dist - omega)) * (1.0 + 1e-9);
    const double Btp = Bt * (1.0 + 3 * U);
    b.dt = (2.01 * U * Bt + (Et + Btp * Ea) / (T->lN * dlo * c) + omega / (dlo * c * c)) * (1.0 + 1e-9);
    return b;
}

RTX_CULL_HD static inline double rtx_cull_W(double omega, double dist, double R) {
    if (!(dist > omega)) return INFINITY;
    return (omega + omega * R / (dist - omega)) * (1.0 + 1e-9);
}

/* Camera rays: every ray whose origin is exactly o (any direction); dt for t~ <= Bt. */
RTX_CULL_HD static inline rtx_cull_bound rtx_cull_point_bounds(const rtx_cull_tri* T, const float* o, double Bt) {
    double sb[3], s2 = 0.0, sd = 0.0;
    for (int k = 0; k < 3; ++k) {
        const float sf = o[k] - (float)T->v0[k];   /* fl(o - v0): the test's own s~ */
        sb[k] = fabs((double)sf);
        s2 += sb[k] * sb[k];
        sd += (double)sf * T->nh[k];
    }
    const double sn = sqrt(s2) * (1.0 + 1e-12);
    const double dist = fabs(sd) * (1.0 - 1e-12) - sn * T->nerr;
    const double R = (sn + (1.0 + 8 * RTX_CULL_U) * T->lmax) * (1.0 + 1e-12);
    rtx_cull_bound b = rtx_cull_bounds(T, sb, dist, R, Bt);
    b.margin = (b.margin + 12 * RTX_CULL_U * T->lmax + RTX_CULL_U * sn + 0x1p-100) * (1.0 + 1e-9);
    return b;
}
RTX_CULL_HD static inline double rtx_cull_margin_point(const rtx_cull_tri* T, const float* o) {
    return rtx_cull_point_bounds(T, o, 0.0).margin;
}

/* Shadow rays toward a light at L (origin o, direction fl(fl(L - o) / fl(|fl(L - o)|)),
   Renderer.cpp:130-136) whose tmax = |fl(L - o)| is at most Tmax; dt for t~ <= Tmax. */
RTX_CULL_HD static inline rtx_cull_bound rtx_cull_light_bounds(const rtx_cull_tri* T, const float* L, double Tmax) {
    const double U = RTX_CULL_U, tp = Tmax * (1.0 + 8 * U);
    double sb[3], s2 = 0.0, lv2 = 0.0, ld = 0.0;
    for (int k = 0; k < 3; ++k) {
        const double lv = (double)L[k] - T->v0[k];
        sb[k] = (1.0 + U) * (tp + fabs(lv)) * (1.0 + 1e-12);
        s2 += sb[k] * sb[k];
        lv2 += lv * lv;
        ld += lv * T->nh[k];
    }
    const double sn = sqrt(s2) * (1.0 + 1e-12), lvn = sqrt(lv2) * (1.0 + 1e-12);
    const double eL = 1.01 * rtx_cull_gamma(3) * tp + U * sn;
    const double dist = fabs(ld) * (1.0 - 1e-12) - lvn * T->nerr - eL;
    const double R = (lvn + (1.0 + 8 * U) * T->lmax + eL) * (1.0 + 1e-12);
    rtx_cull_bound b = rtx_cull_bounds(T, sb, dist, R, Tmax);
    b.margin = (b.margin + 12 * U * T->lmax + U * sn + 0x1p-100) * (1.0 + 1e-9);
    return b;
}
RTX_CULL_HD static inline double rtx_cull_margin_light(const rtx_cull_tri* T, const float* L, double Tmax) {
    return rtx_cull_light_bounds(T, L, Tmax).margin;
}

#endif /* RTX_CULL_H */
