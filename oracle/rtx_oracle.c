/*
 * rtx_oracle.c — TEST INFRASTRUCTURE ONLY: the CPU restatement ("port") of the
 * reference's per-pixel render loop, used as the parity checker by tests/, by
 * __graft_entry__.smoke() and as the "port" CPU baseline leg of bench.py.  It is never
 * linked into, loaded by, or called from the product library (librtx_hip.so).
 *
 * Parity of this file is PINNED: tests/test_oracle.py checks it bit-for-bit against the
 * golden frames emitted by the reference's own sources compiled in place
 * (oracle/ref/).
 *
 * Every function restates the reference operation-for-operation in IEEE binary32 with
 * no FMA contraction (build with -O2 -ffp-contract=off; the reference is MSVC
 * /fp:precise on x64 SSE2).  Reference locations are given per function.
 */
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rtx.h"

#define REF_PI 3.14159265358979323846f /* MathHelpers.h:7 */

typedef struct { float x, y, z; } v3;

/* Vector3 operators (source/Vector3.cpp:22-176) */
static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 scale(v3 v, float s) { return mk(v.x * s, v.y * s, v.z * s); } /* :105-108, Vector3.h:58 */
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* :45-48 */
static inline float sqrmag(v3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }   /* :27-30 */
/* Vector3::Cross (:50-54), literally UnitX*a - UnitY*b + UnitZ*c */
static inline v3 cross(v3 v1, v3 v2) {
    const float a = v1.y * v2.z - v1.z * v2.y;
    const float b = v1.x * v2.z - v1.z * v2.x;
    const float c = v1.x * v2.y - v1.y * v2.x;
    const v3 X = mk(1.f * a, 0.f * a, 0.f * a);
    const v3 Y = mk(0.f * b, 1.f * b, 0.f * b);
    const v3 Z = mk(0.f * c, 0.f * c, 1.f * c);
    return add(sub(X, Y), Z);
}
/* Vector3::Normalize (:32-40): divides by the magnitude, returns it */
static inline float normalize(v3* v) {
    const float m = sqrtf(v->x * v->x + v->y * v->y + v->z * v->z);
    v->x /= m; v->y /= m; v->z /= m;
    return m;
}
static inline v3 normalized(v3 v) { normalize(&v); return v; }
/* std::min / std::max exact semantics (NaN handling matters in the slab test) */
static inline float smin(float a, float b) { return (b < a) ? b : a; }
static inline float smax(float a, float b) { return (a < b) ? b : a; }

typedef struct { float r, g, b; } rgb;
static inline rgb mkc(float r, float g, float b) { rgb c = {r, g, b}; return c; }

/* dae::Ray (source/DataTypes.h:539-565) */
typedef struct { v3 o, d, inv; float tmin, tmax; } ray;
static inline ray mkray(v3 o, v3 d, float tmin, float tmax) {
    ray r; r.o = o; r.d = d;
    r.inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
    r.tmin = tmin; r.tmax = tmax;
    return r;
}

/* dae::HitRecord (DataTypes.h:567-575) */
typedef struct { v3 origin, normal; float t; int did_hit; uint8_t mat; } hitrec;
static inline hitrec empty_hit(void) {
    hitrec h; memset(&h, 0, sizeof h); h.t = FLT_MAX; return h;
}

/* Work counters (SURVEY §8(d) cost model) */
enum { C_PIXELS, C_SPHERE, C_PLANE, C_SLAB, C_TRI, C_HIT, C_SHADOW, C_OCCLUDED,
       C_SHADE_BASE, C_SHADE_LAMBERT, C_SHADE_PHONG, C_SHADE_CT, C_NCOUNT };
typedef struct { uint64_t c[C_NCOUNT]; } counters;

/* GeometryUtils::HitTest_Sphere (source/Utils.h:15-72) */
static int hit_sphere(const rtx_sphere* s, const ray* r, hitrec* h, int ignore) {
    const v3 so = ld3(s->origin);
    const v3 ov = sub(so, r->o);
    const float ovs = sqrmag(ov);
    const float proj = dot(r->d, ov);
    const float perp = ovs - proj * proj;
    const float r2 = s->radius * s->radius;
    if (r2 < perp) return 0;
    const float dist = sqrtf(r2 - perp);
    const float t = proj - dist;
    if (t < r->tmin || t > r->tmax) return 0;
    if (ignore) return 1;
    h->did_hit = 1;
    h->mat = s->material;
    h->origin = add(r->o, scale(r->d, t));
    h->normal = sub(h->origin, so);
    h->t = t;
    return 1;
}

/* GeometryUtils::HitTest_Plane (Utils.h:82-98) */
static int hit_plane(const rtx_plane* p, const ray* r, hitrec* h, int ignore) {
    const v3 po = ld3(p->origin), pn = ld3(p->normal);
    const float t = dot(sub(po, r->o), pn) / dot(r->d, pn);
    if (t >= r->tmin && t < r->tmax) {
        if (!ignore) {
            h->did_hit = 1; h->mat = p->material; h->normal = pn;
            h->origin = add(r->o, scale(r->d, t)); h->t = t;
        }
        return 1;
    }
    return 0;
}

/* GeometryUtils::HitTest_Triangle (Utils.h:109-184); shadow rays (ignore) swap
 * front/back culling (:114-127). */
static int hit_triangle(v3 v0, v3 v1, v3 v2, v3 n, int cull, uint8_t mat, const ray* r,
                        hitrec* h, int ignore) {
    const float cullDot = dot(n, r->d);
    if (fabsf(cullDot) < FLT_EPSILON) return 0;
    if (ignore) {
        if (cull == RTX_CULL_FRONT) cull = RTX_CULL_BACK;
        else if (cull == RTX_CULL_BACK) cull = RTX_CULL_FRONT;
    }
    if (cull == RTX_CULL_FRONT) { if (cullDot < 0) return 0; }
    else if (cull == RTX_CULL_BACK) { if (cullDot > 0) return 0; }
    const v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    const v3 hh = cross(r->d, e2);
    const float a = dot(e1, hh);
    if (fabsf(a) < FLT_EPSILON) return 0;
    const float ai = 1.f / a;
    const v3 s = sub(r->o, v0);
    const float u = ai * dot(s, hh);
    if (u < 0.f || u > 1.f) return 0;
    const v3 q = cross(s, e1);
    const float v = ai * dot(r->d, q);
    if (v < 0.f || (u + v) > 1.f) return 0;
    const float t = ai * dot(e2, q);
    if (t < r->tmin || t >= r->tmax) return 0;
    const v3 P = add(r->o, scale(r->d, t));
    if (!ignore) {
        h->mat = mat; h->did_hit = 1; h->normal = n; h->origin = P; h->t = t;
    }
    return 1;
}

/* GeometryUtils::SlabTest_BVH (Utils.h:221-243) */
static int slab(const float* mn, const float* mx, const ray* r) {
    const float tx1 = (mn[0] - r->o.x) * r->inv.x, tx2 = (mx[0] - r->o.x) * r->inv.x;
    float tMin = smin(tx1, tx2), tMax = smax(tx1, tx2);
    const float ty1 = (mn[1] - r->o.y) * r->inv.y, ty2 = (mx[1] - r->o.y) * r->inv.y;
    tMin = smax(tMin, smin(ty1, ty2)); tMax = smin(tMax, smax(ty1, ty2));
    const float tz1 = (mn[2] - r->o.z) * r->inv.z, tz2 = (mx[2] - r->o.z) * r->inv.z;
    tMin = smax(tMin, smin(tz1, tz2)); tMax = smin(tMax, smax(tz1, tz2));
    return tMax > 0 && tMax >= tMin;
}

/* GeometryUtils::IntersectionTest_BVH (Utils.h:246-288): recursive DFS left then
 * right, no ordering, no t pruning; the any-hit return leaves only the current leaf. */
static void bvh_visit(const rtx_mesh* m, uint32_t ni, const ray* r, int* didHit, hitrec* hr,
                      hitrec* cur, int ignore, counters* cnt) {
    const rtx_bvh_node* node = &m->nodes[ni];
    /* Work accounting stops an any-hit query at its first occluder (the algorithmic
     * work of DoesHit); the reference keeps visiting the remaining siblings, which does
     * not change the boolean.  Rendering (cnt == NULL) follows the reference exactly. */
    if (cnt && ignore && *didHit) return;
    if (cnt) cnt->c[C_SLAB]++;
    if (!slab(node->min, node->max, r)) return;
    if (node->idx_count > 0) {
        for (int idx = 0; idx < (int)node->idx_count; idx += 3) {
            const int li = (int)node->first_idx + idx;
            const v3 v0 = ld3(&m->positions[3 * m->indices[li]]);
            const v3 v1 = ld3(&m->positions[3 * m->indices[li + 1]]);
            const v3 v2 = ld3(&m->positions[3 * m->indices[li + 2]]);
            const v3 n = ld3(&m->normals[3 * (li / 3)]);
            if (cnt) cnt->c[C_TRI]++;
            if (hit_triangle(v0, v1, v2, n, m->cull_mode, m->material, r, cur, ignore)) {
                *didHit = 1;
                if (ignore) return;
                if (cur->t < hr->t) *hr = *cur;
            }
        }
    } else {
        bvh_visit(m, node->left_node, r, didHit, hr, cur, ignore, cnt);
        bvh_visit(m, node->left_node + 1, r, didHit, hr, cur, ignore, cnt);
    }
}

/* GeometryUtils::HitTest_TriangleMesh (Utils.h:290-327, BVH defined) */
static int hit_mesh(const rtx_mesh* m, const ray* r, hitrec* hr, int ignore, counters* cnt) {
    hitrec closest = empty_hit();
    int didHit = 0;
    if (m->n_nodes == 0) return 0;
    bvh_visit(m, 0, r, &didHit, hr, &closest, ignore, cnt);
    return didHit;
}

/* Scene::GetClosestHit (source/Scene.cpp:29-66): one shared scratch record. */
static void closest_hit(const rtx_scene* sc, const ray* r, hitrec* closest, counters* cnt) {
    hitrec hr = empty_hit();
    for (uint32_t i = 0; i < sc->n_spheres; ++i) {
        if (cnt) cnt->c[C_SPHERE]++;
        if (hit_sphere(&sc->spheres[i], r, &hr, 0)) {
            if (hr.t < closest->t) { *closest = hr; normalize(&closest->normal); }
        }
    }
    for (uint32_t i = 0; i < sc->n_planes; ++i) {
        if (cnt) cnt->c[C_PLANE]++;
        if (hit_plane(&sc->planes[i], r, &hr, 0)) {
            if (hr.t < closest->t) *closest = hr;
        }
    }
    for (uint32_t i = 0; i < sc->n_meshes; ++i) {
        if (hit_mesh(&sc->meshes[i], r, &hr, 0, cnt)) {
            if (hr.t < closest->t) *closest = hr;
        }
    }
}

/* Scene::DoesHit (Scene.cpp:68-96) */
static int does_hit(const rtx_scene* sc, const ray* r, counters* cnt) {
    hitrec tmp = empty_hit();
    for (uint32_t i = 0; i < sc->n_spheres; ++i) {
        if (cnt) cnt->c[C_SPHERE]++;
        if (hit_sphere(&sc->spheres[i], r, &tmp, 1)) return 1;
    }
    for (uint32_t i = 0; i < sc->n_planes; ++i) {
        if (cnt) cnt->c[C_PLANE]++;
        if (hit_plane(&sc->planes[i], r, &tmp, 1)) return 1;
    }
    for (uint32_t i = 0; i < sc->n_meshes; ++i) {
        hitrec t2 = empty_hit();
        if (hit_mesh(&sc->meshes[i], r, &t2, 1, cnt)) return 1;
    }
    return 0;
}

/* LightUtils (Utils.h:341-369) */
static v3 dir_to_light(const rtx_light* l, v3 p) {
    if (l->type == RTX_LIGHT_POINT || l->type == RTX_LIGHT_DIRECTIONAL) return sub(ld3(l->origin), p);
    return mk(0.f, 0.f, 0.f);
}
static rgb radiance(const rtx_light* l, v3 target) {
    if (l->type == RTX_LIGHT_POINT) {
        const float s = l->intensity / sqrmag(sub(ld3(l->origin), target));
        return mkc(l->color[0] * s, l->color[1] * s, l->color[2] * s);
    }
    if (l->type == RTX_LIGHT_DIRECTIONAL) {
        const float s = l->intensity;
        return mkc(l->color[0] * s, l->color[1] * s, l->color[2] * s);
    }
    return mkc(0.f, 0.f, 0.f);
}

/* BRDF::Lambert (BRDFs.h:14-22): (cd * kd) / PI */
static rgb lambert_f(float kd, const float* cd) {
    return mkc((cd[0] * kd) / REF_PI, (cd[1] * kd) / REF_PI, (cd[2] * kd) / REF_PI);
}
/* BRDF::Phong (BRDFs.h:33-40) */
static float phong(float ks, float ex, v3 l, v3 v, v3 n) {
    const float s = 2.f * smax(dot(n, l), 0.f);
    const v3 refl = sub(l, scale(n, s));
    const float cosa = smax(dot(refl, v), 0.f);
    return ks * powf(cosa, ex);
}
/* BRDF::GeometryFunction_SchlickGGX (BRDFs.h:78-86) */
static float schlick_ggx(v3 n, v3 v, float rough) {
    const float a = rough * rough;
    const float k = ((a + 1.f) * (a + 1.f)) / 8.f;
    const float cd = smax(dot(n, v), 0.f);
    return cd / ((cd * (1.f - k)) + k);
}

/* Material::Shade per subclass (source/Material.h:41-123) */
static rgb shade(const rtx_material* mt, v3 n, v3 l, v3 v, counters* cnt) {
    switch (mt->kind) {
    case RTX_MAT_SOLID_COLOR:
        return mkc(mt->color[0], mt->color[1], mt->color[2]);
    case RTX_MAT_LAMBERT:
        if (cnt) cnt->c[C_SHADE_LAMBERT]++;
        return lambert_f(mt->kd, mt->color);
    case RTX_MAT_LAMBERT_PHONG: {
        if (cnt) { cnt->c[C_SHADE_LAMBERT]++; cnt->c[C_SHADE_PHONG]++; }
        const rgb d = lambert_f(mt->kd, mt->color);
        const float s = phong(mt->ks, mt->exponent, l, v, n);
        return mkc(d.r + s, d.g + s, d.b + s);
    }
    case RTX_MAT_COOK_TORRANCE: {
        if (cnt) cnt->c[C_SHADE_CT]++;
        const v3 h = normalized(add(v, l));
        const int dielectric = (mt->metalness == 0.f);
        const rgb f0 = dielectric ? mkc(0.04f, 0.04f, 0.04f) : mkc(mt->color[0], mt->color[1], mt->color[2]);
        /* FresnelFunction_Schlick (BRDFs.h:49-53) */
        const float p = powf(1.f - smax(dot(h, v), 0.f), 5.f);
        const rgb F = mkc(f0.r + ((1.f - f0.r) * p), f0.g + ((1.f - f0.g) * p), f0.b + ((1.f - f0.b) * p));
        /* NormalDistribution_GGX (BRDFs.h:62-68) */
        const float a = mt->roughness * mt->roughness;
        const float sqrA = a * a;
        const float ndh = smax(dot(n, h), 0.f);
        const float in = (ndh * ndh) * ((a * a) - 1.f) + 1.f;
        const float D = sqrA / (REF_PI * (in * in));
        /* GeometryFunction_Smith (BRDFs.h:96-99) */
        const float G = schlick_ggx(n, v, mt->roughness) * schlick_ggx(n, l, mt->roughness);
        const float den = (4.f * smax(dot(v, n), 0.0001f)) * smax(dot(l, n), 0.0001f);
        const rgb spec = mkc(((F.r * D) * G) / den, ((F.g * D) * G) / den, ((F.b * D) * G) / den);
        const float kd[3] = {dielectric ? 1.f - F.r : 0.f, dielectric ? 1.f - F.g : 0.f,
                             dielectric ? 1.f - F.b : 0.f};
        const rgb diff = mkc((mt->color[0] * kd[0]) / REF_PI, (mt->color[1] * kd[1]) / REF_PI,
                             (mt->color[2] * kd[2]) / REF_PI);
        return mkc(diff.r + spec.r, diff.g + spec.g, diff.b + spec.b);
    }
    default:
        return mkc(0.f, 0.f, 0.f);
    }
}

static inline uint32_t q8(float c) {
    /* static_cast<uint8_t>(c * 255) as g++/x86 compiles it (cvttss2si, low byte) */
    return (uint32_t)(uint8_t)(int32_t)(c * 255);
}

/* Renderer::RenderPixel (source/Renderer.cpp:100-182) */
static void render_pixel(const rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* p,
                         float aspect, uint32_t px, uint32_t py, uint32_t* out_px, float* out_rgb,
                         counters* cnt) {
    const int W = (int)p->width, H = (int)p->height;
    const float cx = (2.f * (((int)px + 0.5f) / W) - 1) * aspect * cam->fov;
    const float cy = (1.f - (2.f * ((int)py + 0.5f) / H)) * cam->fov;
    /* Matrix::TransformVector (Matrix.cpp:35-42), rows right/up/forward */
    v3 vd = mk(cam->right[0] * cx + cam->up[0] * cy + cam->forward[0] * 1.f,
               cam->right[1] * cx + cam->up[1] * cy + cam->forward[1] * 1.f,
               cam->right[2] * cx + cam->up[2] * cy + cam->forward[2] * 1.f);
    normalize(&vd);
    const ray vr = mkray(ld3(cam->origin), vd, 0.0001f, FLT_MAX);
    if (cnt) cnt->c[C_PIXELS]++;

    hitrec ch = empty_hit();
    closest_hit(sc, &vr, &ch, cnt);

    float shadowFactor = 1.f;
    rgb fc = mkc(0.f, 0.f, 0.f);
    if (ch.did_hit) {
        if (cnt) cnt->c[C_HIT]++;
        const v3 oo = add(ch.origin, scale(ch.normal, 0.0001f));
        const v3 negv = mk(-vd.x, -vd.y, -vd.z);
        for (uint32_t li = 0; li < sc->n_lights; ++li) {
            const rtx_light* L = &sc->lights[li];
            v3 ld = dir_to_light(L, oo);
            const float mag = normalize(&ld);
            if (p->shadows_enabled) {
                if (cnt) cnt->c[C_SHADOW]++;
                const ray sr = mkray(oo, ld, 0.0001f, mag);
                if (does_hit(sc, &sr, cnt)) {
                    if (cnt) cnt->c[C_OCCLUDED]++;
                    shadowFactor *= 0.95f;
                    continue;
                }
            }
            if (cnt) cnt->c[C_SHADE_BASE]++;
            switch (p->lighting_mode) {
            case RTX_MODE_COMBINED: {
                const float oa = smax(dot(ch.normal, ld), 0.f);
                const rgb rad = radiance(L, ch.origin);
                const rgb br = shade(&sc->materials[ch.mat], ch.normal, ld, negv, cnt);
                fc.r += (rad.r * oa) * br.r; fc.g += (rad.g * oa) * br.g; fc.b += (rad.b * oa) * br.b;
                break;
            }
            case RTX_MODE_OBSERVED_AREA: {
                const float oa = smax(dot(ch.normal, ld), 0.f);
                fc.r += oa; fc.g += oa; fc.b += oa;
                break;
            }
            case RTX_MODE_RADIANCE: {
                const rgb rad = radiance(L, ch.origin);
                fc.r += rad.r; fc.g += rad.g; fc.b += rad.b;
                break;
            }
            case RTX_MODE_BRDF: {
                const rgb br = shade(&sc->materials[ch.mat], ch.normal, ld, negv, cnt);
                fc.r += br.r; fc.g += br.g; fc.b += br.b;
                break;
            }
            default: break;
            }
        }
        fc.r *= shadowFactor; fc.g *= shadowFactor; fc.b *= shadowFactor;
    }
    /* ColorRGB::MaxToOne (ColorRGB.h:12-17) */
    const float mv = smax(fc.r, smax(fc.g, fc.b));
    if (mv > 1.f) { fc.r /= mv; fc.g /= mv; fc.b /= mv; }
    const size_t o = (size_t)px + (size_t)py * (size_t)W;
    out_px[o] = (q8(fc.r) << p->format.rshift) | (q8(fc.g) << p->format.gshift) |
                (q8(fc.b) << p->format.bshift) | p->format.amask;
    if (out_rgb) { out_rgb[3 * o] = fc.r; out_rgb[3 * o + 1] = fc.g; out_rgb[3 * o + 2] = fc.b; }
}

/* ---- frame driver: Renderer::Render (Renderer.cpp:34-98) over owned stripes ---- */
typedef struct {
    const rtx_scene* sc; const rtx_camera* cam; const rtx_render_params* p;
    uint32_t* out_px; float* out_rgb; float aspect;
    uint32_t n_rows; const uint32_t* rows;   /* owned rows */
    volatile uint32_t next; pthread_mutex_t mu;
    counters total; int count;
} job;

static void* worker(void* arg) {
    job* j = (job*)arg;
    const uint32_t W = j->p->width;
    const uint64_t n = (uint64_t)j->n_rows * W;
    counters local; memset(&local, 0, sizeof local);
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const uint64_t b = j->next;
        j->next = (uint32_t)((b + 1024 < n) ? b + 1024 : n);
        pthread_mutex_unlock(&j->mu);
        if (b >= n) break;
        const uint64_t e = (b + 1024 < n) ? b + 1024 : n;
        for (uint64_t i = b; i < e; ++i) {
            const uint32_t row = j->rows[i / W];
            render_pixel(j->sc, j->cam, j->p, j->aspect, (uint32_t)(i % W), row, j->out_px, j->out_rgb,
                         j->count ? &local : NULL);
        }
    }
    if (j->count) {
        pthread_mutex_lock(&j->mu);
        for (int k = 0; k < C_NCOUNT; ++k) j->total.c[k] += local.c[k];
        pthread_mutex_unlock(&j->mu);
    }
    return NULL;
}

static int run(const rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* p,
               uint32_t* out_px, float* out_rgb, int threads, uint64_t* counts_out) {
    if (!sc || !cam || !p || !out_px || p->width == 0 || p->height == 0) return RTX_E_INVALID;
    if (p->lighting_mode < 0 || p->lighting_mode >= RTX_MODE_COUNT) return RTX_E_INVALID;
    uint32_t* rows = (uint32_t*)malloc(sizeof(uint32_t) * p->height);
    if (!rows) return RTX_E_NOMEM;
    uint32_t nr = 0;
    for (uint32_t y = 0; y < p->height; ++y) {
        if (p->stripe_rows == 0 || p->stripe_step <= 1 ||
            (y / p->stripe_rows) % p->stripe_step == p->stripe_first)
            rows[nr++] = y;
    }
    job j; memset(&j, 0, sizeof j);
    j.sc = sc; j.cam = cam; j.p = p; j.out_px = out_px; j.out_rgb = out_rgb;
    j.aspect = (int)p->width / (float)(int)p->height;  /* Renderer.cpp:30 */
    j.n_rows = nr; j.rows = rows; j.count = counts_out != NULL;
    pthread_mutex_init(&j.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads == 1) {
        worker(&j);
    } else {
        pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
        for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &j);
        for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
        free(th);
    }
    pthread_mutex_destroy(&j.mu);
    if (counts_out) for (int k = 0; k < C_NCOUNT; ++k) counts_out[k] = j.total.c[k];
    free(rows);
    return RTX_OK;
}

/* Render the rows selected by `p` (same stripe semantics as rtx_render). */
int rtx_oracle_render(const rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* p,
                      uint32_t* out_px, float* out_rgb, int threads) {
    return run(sc, cam, p, out_px, out_rgb, threads, NULL);
}

/* Same, and return the SURVEY §8(d) work counters (C_NCOUNT = 12 uint64). */
int rtx_oracle_count(const rtx_scene* sc, const rtx_camera* cam, const rtx_render_params* p,
                     uint32_t* out_px, int threads, uint64_t* counts12) {
    return run(sc, cam, p, out_px, NULL, threads, counts12);
}

/* Single-primitive entry points for known-answer tests against oracle/ref prims. */
int rtx_oracle_hit_sphere(const float* ray8, const float* sph4, int ignore, float* out8) {
    const ray r = mkray(ld3(ray8), ld3(ray8 + 3), ray8[6], ray8[7]);
    rtx_sphere s; memset(&s, 0, sizeof s);
    memcpy(s.origin, sph4, 12); s.radius = sph4[3];
    hitrec h = empty_hit();
    const int hit = hit_sphere(&s, &r, &h, ignore);
    out8[0] = (float)hit; out8[1] = h.t;
    out8[2] = h.origin.x; out8[3] = h.origin.y; out8[4] = h.origin.z;
    out8[5] = h.normal.x; out8[6] = h.normal.y; out8[7] = h.normal.z;
    return hit;
}
int rtx_oracle_hit_plane(const float* ray8, const float* pl6, int ignore, float* out8) {
    const ray r = mkray(ld3(ray8), ld3(ray8 + 3), ray8[6], ray8[7]);
    rtx_plane p; memset(&p, 0, sizeof p);
    memcpy(p.origin, pl6, 12); memcpy(p.normal, pl6 + 3, 12);
    hitrec h = empty_hit();
    const int hit = hit_plane(&p, &r, &h, ignore);
    out8[0] = (float)hit; out8[1] = h.t;
    out8[2] = h.origin.x; out8[3] = h.origin.y; out8[4] = h.origin.z;
    out8[5] = h.normal.x; out8[6] = h.normal.y; out8[7] = h.normal.z;
    return hit;
}
int rtx_oracle_hit_triangle(const float* ray8, const float* tri12, int cull, int ignore, float* out8) {
    const ray r = mkray(ld3(ray8), ld3(ray8 + 3), ray8[6], ray8[7]);
    hitrec h = empty_hit();
    const int hit = hit_triangle(ld3(tri12), ld3(tri12 + 3), ld3(tri12 + 6), ld3(tri12 + 9), cull, 0, &r, &h, ignore);
    out8[0] = (float)hit; out8[1] = h.t;
    out8[2] = h.origin.x; out8[3] = h.origin.y; out8[4] = h.origin.z;
    out8[5] = h.normal.x; out8[6] = h.normal.y; out8[7] = h.normal.z;
    return hit;
}
int rtx_oracle_slab(const float* ray8, const float* aabb6) {
    const ray r = mkray(ld3(ray8), ld3(ray8 + 3), ray8[6], ray8[7]);
    return slab(aabb6, aabb6 + 3, &r);
}
void rtx_oracle_shade(const rtx_material* m, const float* n3, const float* l3, const float* v3_, float* out3) {
    const rgb c = shade(m, ld3(n3), ld3(l3), ld3(v3_), NULL);
    out3[0] = c.r; out3[1] = c.g; out3[2] = c.b;
}
