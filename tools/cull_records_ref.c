/* cull_records_ref.c — brute-force CPU restatement of the exact cull's records (test checker).
 *
 * The device builds each node slot's record from segment trees of the per-triangle values
 * (rtx_hip.hip: rtx_cull_tris_box, rtx_cull_tris_marg, rtx_cull_nodes).  This file computes the
 * same records the direct way — for every slot, fold every triangle of its range — with the
 * same double-precision operations (rtx_cull.h), so tests/test_gpu_cull.py can require the
 * device records to equal these value for value.  Inputs are what rtx_cull_dump returns.
 * Test infrastructure only: nothing in the product links it.
 *
 * Build: gcc -O2 -ffp-contract=off -fPIC -shared (gp1_raytracer_2223_amd/build.py, tools/bin/).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../gp1_raytracer_2223_amd/csrc/rtx_cull.h"

static float f_rd(double x) {
    float f = (float)x;
    if ((double)f > x) f = nextafterf(f, -INFINITY);
    return f;
}
static float f_ru(double x) {
    float f = (float)x;
    if ((double)f < x) f = nextafterf(f, INFINITY);
    return f;
}
static int in_domain(float x) { return fabsf(x) <= 0x1p40f; }

/* triangle t's box (rtx_cull_tris_box) and (margin, dt) for the anchor (rtx_cull_tris_marg) */
static void tri_values(const float* T, const float* anchor, float* lo, float* hi, float* m, float* dt) {
    const float v0[3] = {T[0], T[1], T[2]}, e1[3] = {T[4], T[5], T[6]}, e2[3] = {T[8], T[9], T[10]};
    int ok = 1;
    for (int k = 0; k < 3; ++k) {
        ok = ok && in_domain(v0[k]) && in_domain(e1[k]) && in_domain(e2[k]);
        const double p = v0[k], q = p + (double)e1[k], r = p + (double)e2[k];
        const double mn = fmin(p, fmin(q, r)), mx = fmax(p, fmax(q, r));
        lo[k] = f_rd(mn - fabs(mn) * 0x1p-40);
        hi[k] = f_ru(mx + fabs(mx) * 0x1p-40);
    }
    if (!ok)
        for (int k = 0; k < 3; ++k) { lo[k] = -INFINITY; hi[k] = INFINITY; }
    rtx_cull_tri tri;
    rtx_cull_tri_setup(&tri, v0, e1, e2);
    const rtx_cull_bound bd = anchor[3] > 0.f ? rtx_cull_light_bounds(&tri, anchor, anchor[3])
                                              : rtx_cull_point_bounds(&tri, anchor, anchor[4]);
    *m = (bd.margin >= 0.0 && bd.margin < 0x1p100) ? f_ru(bd.margin) : INFINITY;
    *dt = (bd.dt >= 0.0 && bd.dt < 0x1p100) ? f_ru(bd.dt) : INFINITY;
}

/* records of every slot (8 floats each, rtx_cull_write's layout) for one anchor; returns 0 */
int cull_records_ref(uint32_t n_slots, uint32_t n_tris, const uint32_t* ranges, const float* nodes,
                     const float* tris, const float* anchor, float ratio, int leaves, float* out) {
    for (uint32_t s = 0; s < n_slots; ++s) {
        const uint32_t x = ranges[2 * s], y = ranges[2 * s + 1];
        int bad = y <= x || y > n_tris;
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY}, m = 0.f, dt = 0.f;
        for (uint32_t t = x; !bad && t < y; ++t) {
            float tl[3], th[3], tm, td;
            tri_values(tris + 16 * (size_t)t, anchor, tl, th, &tm, &td);
            for (int k = 0; k < 3; ++k) {
                lo[k] = fminf(lo[k], tl[k]);
                hi[k] = fmaxf(hi[k], th[k]);
            }
            m = fmaxf(m, tm);
            dt = fmaxf(dt, td);
        }
        for (int k = 0; k < 3; ++k) bad = bad || !(fabsf(lo[k]) < INFINITY) || !(fabsf(hi[k]) < INFINITY);
        if (bad) m = dt = 0.f;
        /* cull_write */
        float cf[3], Ef[3];
        for (int k = 0; k < 3; ++k) {
            const double c = 0.5 * ((double)lo[k] + hi[k]);
            cf[k] = (float)c;
            double E = 0.5 * ((double)hi[k] - lo[k]) + fabs(c - cf[k]) + (double)m;
            E = (E + 0x1p-20 * (E + fabs((double)cf[k]))) * (1.0 + 0x1p-40) + 0x1p-50 * (fabs((double)lo[k]) + fabs((double)hi[k]));
            Ef[k] = (!bad && E < 0x1p100) ? f_ru(E) : INFINITY;
            if (bad || !(E < 0x1p100)) cf[k] = 0.f;
        }
        const float* n0 = nodes + 8 * (size_t)s;
        const float ref[3] = {n0[1] - n0[0], n0[3] - n0[2], n0[5] - n0[4]};
        int worth = 0;
        for (int k = 0; k < 3; ++k) worth = worth || ref[k] > ratio * 2.f * Ef[k];
        uint32_t cnt;
        memcpy(&cnt, n0 + 7, 4);
        if (leaves && cnt == 0u) worth = 0;
        float* r = out + 8 * (size_t)s;
        r[0] = cf[0]; r[1] = cf[1]; r[2] = cf[2]; r[3] = Ef[0];
        r[4] = Ef[1]; r[5] = Ef[2]; r[6] = (bad || !(dt < 0x1p100f)) ? INFINITY : dt;
        const uint32_t w = worth ? 1u : 0u;
        memcpy(r + 7, &w, 4);
    }
    return 0;
}
