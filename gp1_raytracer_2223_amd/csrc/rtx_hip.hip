// rtx_hip.hip — MI355X (gfx950) render path behind the C-ABI of include/rtx.h.
//
// One HIP thread per pixel; one wave64 = an 8x8 pixel tile; one 256-thread workgroup =
// 16x16 pixels.  The BVH is traversed by the WAVE, not by the lane: a wave-uniform DFS
// stack of (node, 64-bit lane mask) lives in LDS, node/triangle/sphere/plane/light
// records are fetched once per wave through the scalar unit (s_load into SGPRs: the
// address is wave-uniform), and each lane evaluates its own ray against them under its
// mask bit.  A lane takes part in a node exactly when the reference's per-ray
// recursive DFS (source/Utils.h:246-288) would visit that node for its ray, in the same
// left-then-right order, so closest-hit tie-breaking (strict <) is the reference's.
// Shadow rays use the same packet traversal with __ballot early-out: a lane leaves the
// mask at its first occluder and the wave stops when every lane is occluded.
//
// Numerics: every float operation restates the reference in IEEE binary32 in the same
// order (built with -ffp-contract=off, correctly rounded div/sqrt); powf (Phong,
// Fresnel) is the device libm's and may differ from the host's by an ulp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <type_traits>
#include <array>
#include <vector>

#include "rtx.h"
#include "rtx_diag.h"
#include "rtx_anim.h"
#include "rtx_cull.h"
#include "rtx_fastdiv.h"
#include "rtx_kernels.h"
#include "rtx_variants.h"
#include "rtx_ctx.h"

using namespace rtxd;
using namespace rtxh;

[[maybe_unused]] constexpr int kStampWords = 8;   // + primary-hit time, shadow-walk time (RTX_STAMPS)
// split waves' {sum, max, steps} per (phase, part) in 64 shards by wave index: one address per
// (phase, part) took every split wave's atomics into one L2 channel and slowed the whole frame ~6x
[[maybe_unused]] constexpr int kStampShards = 64;
#if RTX_STAMPS
#define RTX_SPLIT_STAMP()                                                                          \
    if (lane == 0 && F.split_stamps) {                                                             \
        const unsigned long long d_ = __builtin_amdgcn_s_memrealtime() - t_start;                 \
        unsigned long long* x_ =                                                                   \
            F.split_stamps + 3 * (((PHASE - 1) * kMaxParts + part) * kStampShards + widx % kStampShards); \
        atomicAdd(x_, d_);                                                                         \
        atomicMax(x_ + 1, d_);                                                                     \
        atomicAdd(x_ + 2, static_cast<unsigned long long>(cnt.c[kWaveNodeTests] + cnt.c[kWaveTriTests])); \
    }
#else
#define RTX_SPLIT_STAMP()
#endif

#define RTX_PI 3.14159265358979323846f   // MathHelpers.h:7

// ====================================================================== device code
namespace {

__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }  // std::min
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }  // std::max

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ unsigned long long uni64(unsigned long long x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x >> 32));
    return (static_cast<unsigned long long>(hi) << 32) | lo;
}
__device__ __forceinline__ unsigned long long ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Scene records are immutable for a whole launch: they are read through the constant
// address space, so every wave-uniform read is an s_load through the scalar cache.  With
// generic pointers the backend needs a "no clobber" proof for s_load, which any
// side-effecting instruction on the path (s_memtime for the tile costs) defeats, and the
// reads silently become per-lane vector loads.
#define RTX_CONST __attribute__((address_space(4)))
typedef float cf4 __attribute__((ext_vector_type(4)));
typedef int ci4 __attribute__((ext_vector_type(4)));
typedef float cf16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ float4 ldc(const float4* base, uint32_t i) {
    const cf4 v = ((const RTX_CONST cf4*)base)[i];
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int4 ldc(const int4* base, uint32_t i) {
    const ci4 v = ((const RTX_CONST ci4*)base)[i];
    return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t ldc(const uint32_t* base, uint32_t i) {
    return ((const RTX_CONST uint32_t*)base)[i];
}
__device__ __forceinline__ float ldc(const float* base, uint32_t i) { return ((const RTX_CONST float*)base)[i]; }
typedef float cf8 __attribute__((ext_vector_type(8)));
// A wave-uniform value the optimiser cannot see through: a loop counter passed through it
// stays a 32-bit SGPR offset instead of being widened into a 64-bit pointer induction
// (which costs an s_add_u32/s_addc_u32 pair per record).
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
    asm("" : "+s"(x));
    return x;
}
// Records at a BYTE offset: the offset goes into the SGPR-offset field of s_load, so a
// loop over records or a link walk costs no scalar address arithmetic.
__device__ __forceinline__ float4 ldcb16(const void* base, uint32_t off) {
    const cf4 v = *(const RTX_CONST cf4*)((const RTX_CONST char*)base + off);
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int4 ldcb16i(const void* base, uint32_t off) {
    const ci4 v = *(const RTX_CONST ci4*)((const RTX_CONST char*)base + off);
    return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void ldcb32(const void* base, uint32_t off, float4& a, float4& b) {
    const cf8 v = *(const RTX_CONST cf8*)((const RTX_CONST char*)base + off);
    a = make_float4(v[0], v[1], v[2], v[3]);
    b = make_float4(v[4], v[5], v[6], v[7]);
}
// 64-byte record (Tri, NodePair): one s_load_dwordx16
__device__ __forceinline__ void ldcb64(const void* base, uint32_t off, float4& a, float4& b, float4& c, float4& d) {
    const cf16 v = *(const RTX_CONST cf16*)((const RTX_CONST char*)base + off);
    a = make_float4(v[0], v[1], v[2], v[3]);
    b = make_float4(v[4], v[5], v[6], v[7]);
    c = make_float4(v[8], v[9], v[10], v[11]);
    d = make_float4(v[12], v[13], v[14], v[15]);
}

struct Ray {
    float ox, oy, oz, dx, dy, dz, ix, iy, iz, tmin, tmax;
};

// dae::Ray constructor (DataTypes.h:549-564): inversedDir = 1 / dir.  `slow` = lanes whose
// direction is outside the fast reciprocal domain (rcp3_exact); every other lane has a
// finite, non-zero inverse direction — the FAST slab condition.
__device__ __forceinline__ Ray make_ray(float ox, float oy, float oz, float dx, float dy, float dz, float tmin,
                                        float tmax, unsigned long long& slow) {
    Ray r;
    r.ox = ox; r.oy = oy; r.oz = oz; r.dx = dx; r.dy = dy; r.dz = dz;
    slow = rcp3_exact(dx, dy, dz, r.ix, r.iy, r.iz);
    r.tmin = tmin; r.tmax = tmax;
    return r;
}

// HitTest_Sphere (Utils.h:52-66) in two steps, so that the square root (16 VALU when
// correctly rounded) runs only when some lane's ray passes within the radius:
//   sphere_perp: squared distance of the centre from the ray line (reject if r^2 < perp)
//   sphere_t:    t = proj - sqrt(r^2 - perp) and the [tmin, tmax] test
struct SphereProj {
    float proj, perp;
};
__device__ __forceinline__ SphereProj sphere_perp(const float4 s, const Ray& r) {
    const float ovx = s.x - r.ox, ovy = s.y - r.oy, ovz = s.z - r.oz;
    const float ovs = ovx * ovx + ovy * ovy + ovz * ovz;
    const float proj = r.dx * ovx + r.dy * ovy + r.dz * ovz;
    return {proj, ovs - proj * proj};
}
__device__ __forceinline__ float sphere_t(const float4 s, const SphereProj& q) { return q.proj - sqrtf(s.w - q.perp); }

// HitTest_Plane (Utils.h:84-97): t = num / den.  With tmin > 0 (every ray here), a hit
// needs t > 0, i.e. num and den non-zero with the same sign: RN(num/den) carries the exact
// sign of the quotient, 0/x, x/0 and NaN operands all fail t >= tmin.  `plane_cand`
// lets a wave skip the division when no lane can hit.
__device__ __forceinline__ float plane_num(const float4 p0, const float4 p1, const Ray& r) {
    return (p0.x - r.ox) * p1.x + (p0.y - r.oy) * p1.y + (p0.z - r.oz) * p1.z;
}
__device__ __forceinline__ float plane_den(const float4 p1, const Ray& r) {
    return r.dx * p1.x + r.dy * p1.y + r.dz * p1.z;
}
// The room's planes (kSpecRoomPlanes, rtx_kernels.h): plane k's normal is s = +-1 on axis
// A = kRoomAxes[k] and zero elsewhere, its origin finite with |p0| <= 2^64.  For a ray with a
// finite origin every other term of HitTest_Plane's two dot products is a signed zero (p0 - o
// cannot overflow), so the reference's num and den are s * a and s * d with
//   a = p0_A - o_A,   d = d_A
// whenever those are non-zero (x + +-0 = x, inf included), and its t = num / den = a / d (IEEE
// division is sign-symmetric); the same-sign and beyond tests of plane_cand read the same
// signs and magnitudes.  When a or d is zero the quotient is +-0, +-inf or NaN, which fails
// t >= tmin > 0 or t < tmax <= FLT_MAX in both forms whatever the zero's sign; so does a NaN /
// infinite direction component, which leaves d 0, +-inf or NaN here and den NaN in the
// reference (a normalised direction is finite unless its length was 0 or inf).  Same hits,
// same t, 1 VALU instead of 13 before the division.
template <int A>
__device__ __forceinline__ float room_a(const float4 p0, const Ray& r) {
    return A == 0 ? p0.x - r.ox : (A == 1 ? p0.y - r.oy : p0.z - r.oz);
}
template <int A>
__device__ __forceinline__ float room_d(const Ray& r) {
    return A == 0 ? r.dx : (A == 1 ? r.dy : r.dz);
}
template <int A>
__device__ __forceinline__ float room_inv(const Ray& r) {
    return A == 0 ? r.ix : (A == 1 ? r.iy : r.iz);
}
// f(integral_constant<int, k>) for the room's planes k = 0..4, in order
template <class Fn>
__device__ __forceinline__ void for_room_planes(Fn&& f) {
    f(std::integral_constant<int, 0>{});
    f(std::integral_constant<int, 1>{});
    f(std::integral_constant<int, 2>{});
    f(std::integral_constant<int, 3>{});
    f(std::integral_constant<int, 4>{});
}
__device__ __forceinline__ bool finite3(float x, float y, float z) {
    return __builtin_isfinite(x) & __builtin_isfinite(y) & __builtin_isfinite(z);
}
// Shadow rays (finite tmax): only lanes whose num and den have equal sign bits can hit
// (over-inclusive is harmless: it only decides whether the division runs; zeros and NaNs then
// fail the range test on t), and a lane whose exact |num| / |den| exceeds tmax cannot hit either —
// RN(num/den) >= tmax by monotonicity — and one fma tells it exactly: the sign of
// RN(|den| * tmax - |num|) is the sign of the exact value (an underflow to -0 reads as "not
// beyond", and a NaN or inf operand as well; the division then decides).  Walls behind the
// light are the common case, so most waves skip the division.
__device__ __forceinline__ unsigned long long plane_cand(float num, float den, float tmax) {
    const int same = (__float_as_int(num) ^ __float_as_int(den)) >= 0;
    const int beyond = fmaf(fabsf(den), tmax, -fabsf(num)) < 0.f;
    return ballot(same & !beyond);
}

// HitTest_Triangle (Utils.h:109-184), Möller–Trumbore with the reference's cull rules
// (shadow rays swap front/back culling, :114-127).
//
// Written branch-free: every early `return false` of the reference becomes a term whose
// positive value means "reject", folded with v_max_f32 (which ignores NaN exactly as the
// reference's comparisons do: a NaN never rejects).  For binary32 x, y:
//   x < y  <=>  (y - x) > 0   (a non-zero exact difference never rounds to 0 or flips sign)
// so  |c| < EPS <=> EPS-|c| > 0,  u < 0 || u > 1 <=> max(-u, u-1) > 0,
//     v < 0 || (u+v) > 1 <=> max(-v, (u+v)-1) > 0,  t < tmin <=> tmin - t > 0.
// Cross products use the reduced form {a, -b, c}: identical to Vector3::Cross's
// UnitX*a - UnitY*b + UnitZ*c for finite inputs up to the sign of a zero, which none of
// the tests below can observe.  Returns the reject score; accept iff !(score > 0) && !(t >= tmax).
// `cs` is the mesh's cull sign: -1 FrontFaceCulling (reject cullDot < 0), +1
// BackFaceCulling (reject cullDot > 0), 0 NoCulling (the term 0*cullDot never exceeds 0);
// shadow rays pass -cs, which is the reference's front/back swap.
template <bool FAST>
__device__ __forceinline__ float tri_t(const float4 A, const float4 B, const float4 C, float cs, const Ray& r,
                                       float& t) {
    const float cullDot = A.w * r.dx + B.w * r.dy + C.w * r.dz;
    float rej = fmaxf(FLT_EPSILON - fabsf(cullDot), cs * cullDot);
    const float hx = r.dy * C.z - r.dz * C.y;
    const float hy = -(r.dx * C.z - r.dz * C.x);
    const float hz = r.dx * C.y - r.dy * C.x;
    const float a = B.x * hx + B.y * hy + B.z * hz;
    rej = fmaxf(rej, FLT_EPSILON - fabsf(a));
    // RN(1/a): lanes with |a| < EPS are rejected above whatever ai is, so only huge, inf
    // and NaN a need the IEEE sequence (NaN gives NaN either way).  FAST: every direction
    // is finite with |d| < 2 and the scene's |e1||e2| <= 2^56 (DevScene::tri_fast), so
    // |a| <= |e1||d||e2| < 2^60 and rcp_rn is exact without the check.
    float ai = rcp_rn(a);
    if (!FAST && __builtin_expect(fabsf(a) > 0x1p60f, 0)) ai = 1.f / a;
    const float sx = r.ox - A.x, sy = r.oy - A.y, sz = r.oz - A.z;
    const float u = ai * (sx * hx + sy * hy + sz * hz);
    rej = fmaxf(rej, fmaxf(-u, u - 1.f));
    const float qx = sy * B.z - sz * B.y;
    const float qy = -(sx * B.z - sz * B.x);
    const float qz = sx * B.y - sy * B.x;
    const float v = ai * (r.dx * qx + r.dy * qy + r.dz * qz);
    rej = fmaxf(rej, fmaxf(-v, (u + v) - 1.f));
    t = ai * (C.x * qx + C.y * qy + C.z * qz);
    return fmaxf(rej, r.tmin - t);
}

// tri_t with two wave-uniform early exits for the lanes in `act` (the ones whose result is
// used): after the cull test (Utils.h:114-127) and after the u range test (:160-163), the
// rest is skipped when no lane in `act` can still be accepted — the same early returns as
// the reference's, taken per wave.  Returns false (wave-uniform) when the triangle was
// skipped — no lane hits it — else true with the reject score in `rej_out` and t in `t`.
// (A uniform flag rather than a reject value: a phi of the reject compare is carried as a
// lane mask and rebuilt with v_cndmask + v_cmp per triangle.)
// CB (kSpecCullBack): the mesh culls back faces, so cs is +1 for camera rays and -1 for shadow
// rays (ANY) and cs * cullDot is +-cullDot exactly: a source negation instead of a multiply.
template <bool FAST, bool CB = false, bool ANY = false>
__device__ __forceinline__ bool tri_t_wave(const float4 A, const float4 B, const float4 C, float cs, const Ray& r,
                                           unsigned long long act, float& rej_out, float& t) {
    const float cullDot = A.w * r.dx + B.w * r.dy + C.w * r.dz;
    float rej = fmaxf(FLT_EPSILON - fabsf(cullDot), CB ? (ANY ? -cullDot : cullDot) : cs * cullDot);
    if ((ballot(!(rej > 0.f)) & act) == 0) return false;
    const float hx = r.dy * C.z - r.dz * C.y;
    const float hy = -(r.dx * C.z - r.dz * C.x);
    const float hz = r.dx * C.y - r.dy * C.x;
    const float a = B.x * hx + B.y * hy + B.z * hz;
    rej = fmaxf(rej, FLT_EPSILON - fabsf(a));
    float ai = rcp_rn(a);
    if (!FAST && __builtin_expect(fabsf(a) > 0x1p60f, 0)) ai = 1.f / a;
    const float sx = r.ox - A.x, sy = r.oy - A.y, sz = r.oz - A.z;
    const float u = ai * (sx * hx + sy * hy + sz * hz);
    rej = fmaxf(rej, fmaxf(-u, u - 1.f));
    if ((ballot(!(rej > 0.f)) & act) == 0) return false;
    const float qx = sy * B.z - sz * B.y;
    const float qy = -(sx * B.z - sz * B.x);
    const float qz = sx * B.y - sy * B.x;
    const float v = ai * (r.dx * qx + r.dy * qy + r.dz * qz);
    rej = fmaxf(rej, fmaxf(-v, (u + v) - 1.f));
    t = ai * (C.x * qx + C.y * qy + C.z * qz);
    rej_out = fmaxf(rej, r.tmin - t);
    return true;
}

// SlabTest_BVH (Utils.h:221-243).  FAST uses v_min/v_max_f32, which differ from std::min/
// std::max only when an operand is NaN; a NaN slab value needs (box - origin) * inv with
// an infinite inv component, so FAST is taken only when every live lane's inverse
// direction is finite (decided once per ray batch with a ballot).
// Returned as a wave lane mask: one v_cmp per condition straight into SGPRs (a ballot
// of the && would materialise the bool in a VGPR and compare it again).
// Node record (32 B): a = {min.x, max.x, min.y, max.y}, b = {min.z, max.z, link, ntri};
// link and triangle count are adjacent (one 64-bit SGPR pair).  (Packed f32 for the
// (min, max) pairs was measured 15-35 % slower: profiles/r01/ablate_history.md.)
// SLAB selects the formulation (all three give the reference's pass/fail bit):
//   kSlabExact  std::min/std::max restated (NaN-safe), any direction;
//   kSlabFast   v_min/v_max_f32, which differ from std::min/std::max only when an operand
//               is NaN; a NaN slab value needs (box - origin) * inv with an infinite inv
//               component, so it is taken only when every live lane's inverse direction is
//               finite (decided once per ray batch with a ballot);
//   kSlabOct    kSlabFast for a ray batch whose inverse directions have ONE sign per axis
//               (an octant), against the node copy ordered (near, far) for that octant:
//               the near and far planes are known, so min/max of each pair disappears.
// Returned as a wave lane mask: one v_cmp per condition straight into SGPRs (a ballot
// of the && would materialise the bool in a VGPR and compare it again).
enum { kSlabExact = 0, kSlabFast = 1, kSlabOct = 2 };
template <int SLAB>
__device__ __forceinline__ unsigned long long slab_mask(const float4 a, const float4 b, const Ray& r) {
    const float tx1 = (a.x - r.ox) * r.ix, tx2 = (a.y - r.ox) * r.ix;
    const float ty1 = (a.z - r.oy) * r.iy, ty2 = (a.w - r.oy) * r.iy;
    const float tz1 = (b.x - r.oz) * r.iz, tz2 = (b.y - r.oz) * r.iz;
    float tMin, tMax;
    if (SLAB == kSlabOct) {
        // Octant copy: per axis the record holds (near, far) = (lo, hi) where inv > 0 and
        // (hi, lo) where inv < 0, so rounding monotonicity gives t_near <= t_far per axis
        // (the pair's min and max); each value is the reference's own (same operands).
        tMin = fmaxf(fmaxf(fmaxf(tx1, ty1), tz1), 0x1p-149f);
        tMax = fminf(fminf(tx2, ty2), tz2);
        return ballot(tMax >= tMin);
    } else if (SLAB == kSlabFast) {
        tMin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
        tMax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
        // no NaN here: tMax > 0 && tMax >= tMin  <=>  tMax >= max(tMin, smallest denormal)
        // (f32 denormals are kept, .amdhsa_float_denorm_mode_32 = 3): one compare, no s_and
        return ballot(tMax >= fmaxf(tMin, 0x1p-149f));
    } else {
        tMin = smin(tx1, tx2);
        tMax = smax(tx1, tx2);
        tMin = smax(tMin, smin(ty1, ty2));
        tMax = smin(tMax, smax(ty1, ty2));
        tMin = smax(tMin, smin(tz1, tz2));
        tMax = smin(tMax, smax(tz1, tz2));
    }
    return ballot(tMax > 0) & ballot(tMax >= tMin);
}

// Exact cull (rtx_cull.h): a node the reference's slab test passes is skipped for
// a lane when no triangle below can pass HitTest_Triangle for its ray in a way that matters, so
// the visit would change nothing:
//   * the ray's LINE misses the node's tight box widened by the margin rtx_cull.h proves for the
//     ray's anchor (view camera / light): no triangle below can be accepted at all;
//   * closest hit: the line enters that box at n with n - dt > sc_t (dt: rtx_cull.h's bound on
//     |t~ - t*| for t~ <= the anchor's bt, valid while sc_t <= bt): every triangle below that
//     could be accepted has t~ > sc_t, so none replaces the scratch hit (strict <);
//   * shadow ray: n - dt > tmax or f + dt < tmin (f: where the line leaves the box): no accepted
//     t~ lies in [tmin, tmax).
// Record per node slot (same byte offset as the node): {c.x, c.y, c.z, E.x}, {E.y, E.z, dt, flag},
// box = c +- E (E includes the margin and the padding 16u (E + |c|) that covers this test's own
// rounding, so n is at most and f at least the exact entry and exit of the widened box; rounding
// of n - dt etc. is monotone, so each float comparison implies the exact one).  `k` = 16u |o| |inv|
// per axis covers the rounding of (c - o) * inv, or +inf for a lane outside the bound's domain
// (n = -inf, f = +inf: it passes every test).  Lanes of a FAST batch only (finite non-zero inverse
// directions, |inv| <= 2^64).  NaN-safe: max/min ignore a NaN operand (its axis is dropped) and a
// NaN comparison never culls.
struct CullRay {
    const float4* base;   // the anchor's records (null: no cull)
    float kx, ky, kz;
    float bt;             // the anchor's t bound for dt (closest hit: prune only while sc_t <= bt)
};
__device__ __forceinline__ void cull_nf(const float4 a, const float4 b, const Ray& r, const CullRay& q, float& n,
                                        float& f) {
    const float tx = (a.x - r.ox) * r.ix, ty = (a.y - r.oy) * r.iy, tz = (a.z - r.oz) * r.iz;
    const float hx = fmaf(a.w, fabsf(r.ix), q.kx), hy = fmaf(b.x, fabsf(r.iy), q.ky), hz = fmaf(b.y, fabsf(r.iz), q.kz);
    n = fmaxf(fmaxf(tx - hx, ty - hy), tz - hz);
    f = fminf(fminf(tx + hx, ty + hy), tz + hz);
}
// lanes that still have to enter the node whose record is (a, b); n: the entry (child ordering)
template <bool ANY>
__device__ __forceinline__ unsigned long long cull_pass(const float4 a, const float4 b, const Ray& r, const CullRay& q,
                                                        float sc_t, float& n) {
    float f;
    cull_nf(a, b, r, q, n, f);
    const float dt = b.z;
    bool keep = !(n > f);
    if (ANY) keep = keep & !(n - dt > r.tmax) & !(f + dt < r.tmin);
    else keep = keep & !((sc_t <= q.bt) & (n - dt > sc_t));
    return ballot(keep);
}
// 16u |o_k| |inv_k| per axis, or +inf (always pass) for a lane outside the bound's domain:
// |o_k| <= 2^40, |inv_k| <= 2^64 and `ok` (the caller's conditions on the direction and tmax)
__device__ __forceinline__ CullRay cull_ray(const float4* base, const Ray& r, bool ok, float bt) {
    CullRay q;
    q.base = base;
    q.bt = bt;
    ok = ok && fabsf(r.ox) <= 0x1p40f && fabsf(r.oy) <= 0x1p40f && fabsf(r.oz) <= 0x1p40f &&
         fabsf(r.ix) <= 0x1p64f && fabsf(r.iy) <= 0x1p64f && fabsf(r.iz) <= 0x1p64f;
    constexpr float k16u = 0x1p-20f;
    q.kx = ok ? (k16u * fabsf(r.ox)) * fabsf(r.ix) : INFINITY;
    q.ky = ok ? (k16u * fabsf(r.oy)) * fabsf(r.iy) : INFINITY;
    q.kz = ok ? (k16u * fabsf(r.oz)) * fabsf(r.iz) : INFINITY;
    return q;
}

// Octant of a FAST ray batch (every live inverse direction finite and non-zero): bit k set
// when axis k's inverse direction is negative for every lane in `mask` (non-empty), -1
// when the lanes disagree on some axis.  One code per lane from the sign bits, compared
// against the first masked lane's: a few VALU and one compare, no per-axis scalar logic.
__device__ __forceinline__ int batch_octant(const Ray& r, unsigned long long mask) {
    const uint32_t code = (__float_as_uint(r.ix) >> 31) | ((__float_as_uint(r.iy) >> 31) << 1) |
                          ((__float_as_uint(r.iz) >> 31) << 2);
    const uint32_t first = static_cast<uint32_t>(__builtin_ctzll(mask));
    const uint32_t c0 = __builtin_amdgcn_readlane(code, first);
    return (ballot(code == c0) & mask) == mask ? static_cast<int>(c0) : -1;
}
// The mesh record carries its cull sign as float bits (set at upload: -1 FrontFaceCulling,
// +1 BackFaceCulling, 0 NoCulling); shadow rays use the negation, the reference's swap.
__device__ __forceinline__ float cull_sign(int cs_bits, bool shadow) {
    const float cs = __int_as_float(cs_bits);
    return shadow ? -cs : cs;
}

struct alignas(64) NodePair {
    float4 l0, l1, r0, r1;   // left child (a, b) then right child (a, b), see slab_mask
};
// (link, ntri) of a child as one 64-bit value: link low, count high
__device__ __forceinline__ unsigned long long link_ntri(const float4 b) {
    return (static_cast<unsigned long long>(__float_as_uint(b.w)) << 32) | __float_as_uint(b.z);
}

struct Counts {
    uint32_t c[kNumCounters];
};

// Packet traversal of one mesh's BVH by the whole wave.
//
// A node is entered with the mask of lanes whose slab test on it passed; an inner node
// then tests BOTH children (adjacent, one 64-byte scalar load) for those lanes, descends
// into the left child and pushes the right one with its own pass mask.  Each lane thus
// evaluates exactly the slab tests and triangle tests of the reference's recursive DFS
// (Utils.h:246-288), triangles in the same left-to-right order.
//   closest (ANY = false): `sc_t` is the shared scratch HitRecord t of Scene.cpp:31 that
//       IntersectionTest_BVH compares against (Utils.h:270-273); t < sc_t replaces it.
//   any-hit (ANY = true, shadow rays, Scene::DoesHit): a lane leaves at its first
//       occluder; the wave leaves as soon as every lane in `mask` is occluded.
// COUNT: per-lane SURVEY §8(d) work counters, any-hit counted up to the first occluder.
// DFS below one node (link, ntri) that passed its slab test for the lanes in m.
template <bool ANY, bool FAST, bool COUNT>
__device__ void bvh_walk(const DevScene& S, float cs, const Ray& r, uint32_t link, uint32_t ntri, unsigned long long m,
                         unsigned long long mask, uint32_t lane, uint4* stk, unsigned long long* sT, float& sc_t,
                         uint32_t& sc_tri, unsigned long long& live, Counts& cnt, const uint32_t* occ_word = nullptr,
                         uint32_t occ_bit = 0) {
    int sp = 0;
    for (;;) {
        // invariant: the node (link, ntri) passed its slab test exactly for the lanes in m
        if (ntri) {
            if ((COUNT || RTX_STAMPS) && lane == 0) cnt.c[kWaveTriTests] += ntri;
            if (RTX_STAMPS && !COUNT && lane == 0) cnt.c[kTri] += ntri * __popcll(ANY ? (m & live) : m);
            const bool in = (m >> lane) & 1ull;
            for (uint32_t k = 0; k < ntri; ++k) {
                const uint32_t ti = link + k * 64u;   // byte offset of the triangle record
                Tri T;
                ldcb64(S.tris, ti, T.a, T.b, T.c, T.d);
                float t;
                const float rej = tri_t<FAST>(T.a, T.b, T.c, cs, r, t);
                if (ANY) {
                    if (COUNT && ((m & live) >> lane) & 1ull) cnt.c[kTri]++;
                    live &= ~(ballot(!(rej > 0.f)) & ballot(!(t >= r.tmax)) & m);
                } else {
                    if (COUNT && in) cnt.c[kTri]++;
                    const bool u = in & !(rej > 0.f) & !(t >= r.tmax) & (t < sc_t);
                    sc_t = u ? t : sc_t;
                    sc_tri = u ? ti : sc_tri;
                }
            }
            if (ANY && occ_word) {
                // split any-hit: drop the lanes another part has already found occluded
                const uint32_t o = __hip_atomic_load(occ_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                live &= ~ballot((o & occ_bit) != 0u);
            }
            if (ANY && (live & mask) == 0) return;
        } else {
            if ((COUNT || RTX_STAMPS) && lane == 0) cnt.c[kWaveNodeTests]++;
            if (RTX_STAMPS && !COUNT && lane == 0) cnt.c[kSlab] += 2 * __popcll(m);
            NodePair P;
            ldcb64(S.nodes, link, P.l0, P.l1, P.r0, P.r1);
            const unsigned long long ml = slab_mask<FAST ? kSlabFast : kSlabExact>(P.l0, P.l1, r) & m;
            const unsigned long long mr = slab_mask<FAST ? kSlabFast : kSlabExact>(P.r0, P.r1, r) & m;
            const bool in = COUNT && ((m >> lane) & 1ull);
            if (COUNT && in) cnt.c[kSlab]++;               // left child's test
            if (COUNT && !ANY && in) cnt.c[kSlab]++;       // right child's (closest: always reached)
            if (ml) {
                // an opaque copy keeps this test local to the block: a `mr != 0` shared with
                // the test below is hoisted and carried across blocks as a VGPR boolean
                // (s_cselect + v_cndmask + v_cmp per node pair)
                unsigned long long mrl = mr;
                asm("" : "+s"(mrl));
                if (mrl || (COUNT && ANY)) {               // any-hit COUNT: right is counted at pop
                    stk[sp] = make_uint4(__float_as_uint(P.r1.z), __float_as_uint(P.r1.w),
                                         static_cast<uint32_t>(mrl), static_cast<uint32_t>(mrl >> 32));
                    if (COUNT && ANY) sT[sp] = m;
                    ++sp;
                }
                link = __float_as_uint(P.l1.z);
                ntri = __float_as_uint(P.l1.w);
                m = ml;
                continue;
            }
            if (COUNT && ANY && in) cnt.c[kSlab]++;        // right child's test, reached now
            if (mr) {
                link = __float_as_uint(P.r1.z);
                ntri = __float_as_uint(P.r1.w);
                m = mr;
                continue;
            }
        }
        // pop the next pending right child
        for (;;) {
            if (sp == 0) return;
            --sp;
            const uint4 e = stk[sp];
            link = uni(e.x);
            ntri = uni(e.y);
            m = (static_cast<unsigned long long>(uni(e.w)) << 32) | uni(e.z);
            if (ANY) {
                if (COUNT) {
                    const unsigned long long tested = uni64(sT[sp]);
                    if (((tested & live) >> lane) & 1ull) cnt.c[kSlab]++;
                }
                m &= live;
            }
            if (m) break;
        }
    }
}

constexpr int kPlaneCache = 8;   // planes whose shadow-ray numerators are kept in LDS
// bvh_walk without counters, shaped for the scalar unit: one inner loop descends through
// inner nodes with scalar selects (no i1 value crosses a block, so nothing is carried as a
// VGPR boolean or a lane-mask flow variable), a dead end leaves it as an empty "leaf", and
// the pop loop is the only other path.  Same visits, tests and order as bvh_walk.
// `nb` is the node copy the slab form reads (the octant's (near, far) copy for kSlabOct).
// CULL: a child is entered only by the lanes cull_pass keeps, and the walk is ORDERED: the child
// most lanes enter first is walked first.  Shadow rays (RTX_CULL_ORDER_ANY): nearer occluders end
// their lanes sooner, and any-hit is a yes/no that no order changes.  Closest hit: the scratch hit
// is replaced by t < sc_t or, on a tie, by the lower triangle index — the reference's first-found winner whatever the visiting
// order, because left-then-right DFS order is increasing triangle index (the scene has the cull
// only when that holds, upload_scene; the split launches' key minimum rests on the same fact) — so
// nearer subtrees lower sc_t before farther ones are tested and cull_pass prunes those.
// COUNT (the counting variant of the culled walk, rtx_count_work_culled): per lane, the slab,
// exact-cull and triangle tests this walk executes for the lane (a lane in the node's mask is
// tested against both children), in `cp` — the executed work beside the reference's (bvh_walk).
template <bool ANY, int SLAB, bool CB = false, bool CULL = false, bool COUNT = false>
__device__ void bvh_walk_lean(const DevScene& S, const float4* nb, float cs, const Ray& r, uint32_t link,
                              uint32_t ntri, unsigned long long m, unsigned long long mask, uint32_t lane, uint4* stk,
                              float& sc_t, uint32_t& sc_tri, unsigned long long& live, const uint32_t* occ_word,
                              uint32_t occ_bit, const CullRay& cq = CullRay{}, Counts* cp = nullptr) {
    constexpr bool FAST = SLAB != kSlabExact;
    constexpr bool ORD = CULL && (!ANY || RTX_CULL_ORDER_ANY);
    uint32_t sp = 0;
    for (;;) {
        while (ntri == 0) {
            NodePair P;
            ldcb64(nb, link, P.l0, P.l1, P.r0, P.r1);
            // the pair's cull records at the same offset, loaded beside the pair (one memory
            // latency per step, not two: the shadow walk had issued it only after the slab tests)
            [[maybe_unused]] NodePair Q;
            if (CULL) ldcb64(cq.base, link, Q.l0, Q.l1, Q.r0, Q.r1);
            if constexpr (COUNT) {
                if ((m >> lane) & 1ull) cp->c[kSlab] += 2;
                if (lane == 0) cp->c[kWaveNodeTests]++;
            }
            unsigned long long ml = slab_mask<SLAB>(P.l0, P.l1, r) & m;
            unsigned long long mr = slab_mask<SLAB>(P.r0, P.r1, r) & m;
            [[maybe_unused]] bool rfirst = false;
            if (CULL) {
                // only pairs whose records are flagged worth testing (cull_write), and only when
                // some lane entered a child
                if ((__float_as_uint(Q.l1.w) | __float_as_uint(Q.r1.w)) && (ml | mr)) {
                    if constexpr (COUNT) {
                        if ((m >> lane) & 1ull) cp->c[kCullTests] += 2;
                    }
                    float nl, nr;
                    ml &= cull_pass<ANY>(Q.l0, Q.l1, r, cq, sc_t, nl);
                    mr &= cull_pass<ANY>(Q.r0, Q.r1, r, cq, sc_t, nr);
                    if (ORD) {   // right first when most lanes that enter both enter it first
                        const unsigned long long both_m = ml & mr;
                        rfirst = 2 * __popcll(ballot(nr < nl) & both_m) > __popcll(both_m);
                    }
                }
            }
            if (ORD && rfirst) {   // walk the right child first: swap the pair's roles
                const unsigned long long t0 = ml;
                ml = mr;
                mr = t0;
                const float4 t1 = P.l1;
                P.l1 = P.r1;
                P.r1 = t1;
            }
            // next (link, ntri): left, else right, else a dead end taken as an empty leaf
            // (ntri = 1 with m = 0); `both` = mr if the left child is taken too (the right
            // one then waits on the stack).  Written as 64-bit s_cselects on one SCC each:
            // the compiler materialises every `x != 0` as a -1/0 SGPR pair and ANDs them.
            unsigned long long nx, both;
            asm("s_cmp_lg_u64 %[mr], 0\n\t"
                "s_cselect_b64 %[nx], %[lr], %[dead]\n\t"
                "s_cmp_lg_u64 %[ml], 0\n\t"
                "s_cselect_b64 %[nx], %[ll], %[nx]\n\t"
                "s_cselect_b64 %[both], %[mr], 0\n\t"
                "s_cselect_b64 %[m], %[ml], %[mr]"
                : [nx] "=&s"(nx), [both] "=&s"(both), [m] "=&s"(m)
                : [mr] "s"(mr), [ml] "s"(ml), [lr] "s"(link_ntri(P.r1)), [ll] "s"(link_ntri(P.l1)),
                  [dead] "s"(1ull << 32)
                : "scc");
            if (both) {
                stk[sp] = make_uint4(__float_as_uint(P.r1.z), __float_as_uint(P.r1.w), static_cast<uint32_t>(mr),
                                     static_cast<uint32_t>(mr >> 32));
                ++sp;
            }
            link = static_cast<uint32_t>(nx);
            // opaque: a 32-bit s_cmp for the loop test (else it becomes a 64-bit v_cmp on nx)
            ntri = opaque(static_cast<uint32_t>(nx >> 32));
        }
        if (m) {
            const bool in = (m >> lane) & 1ull;
            // split any-hit: the other parts' occlusion bits, read before the leaf's tests so the
            // L2 round trip overlaps them (RTX_OCC_POLL, rtx_variants.h)
            uint32_t occ_pre = 0u;
            if (ANY && RTX_OCC_POLL == 2 && occ_word)
                occ_pre = __hip_atomic_load(occ_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (uint32_t k = 0; k < ntri; ++k) {
                const uint32_t ti = link + k * 64u;
                Tri T;
                ldcb64(S.tris, ti, T.a, T.b, T.c, T.d);
                if constexpr (COUNT) {
                    if (((ANY ? (m & live) : m) >> lane) & 1ull) cp->c[kTri]++;
                    if (lane == 0) cp->c[kWaveTriTests]++;
                }
                float t;
                float rej;
                if (!tri_t_wave<FAST, CB, ANY>(T.a, T.b, T.c, cs, r, ANY ? (m & live) : m, rej, t)) continue;
                if (ANY) {
                    live &= ~(ballot(!(rej > 0.f)) & ballot(!(t >= r.tmax)) & m);
                } else {
                    const bool better = CULL ? ((t < sc_t) | ((t == sc_t) & (ti < sc_tri))) : (t < sc_t);
                    const bool u = in & !(rej > 0.f) & !(t >= r.tmax) & better;
                    sc_t = u ? t : sc_t;
                    sc_tri = u ? ti : sc_tri;
                }
            }
            if (ANY && RTX_OCC_POLL != 0 && occ_word) {
                const uint32_t o = RTX_OCC_POLL == 2
                                       ? occ_pre
                                       : __hip_atomic_load(occ_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                live &= ~ballot((o & occ_bit) != 0u);
            }
            if (ANY && (live & mask) == 0) return;
        }
        for (;;) {
            if (sp == 0) return;
            --sp;
            const uint4 e = stk[sp];
            link = uni(e.x);
            ntri = uni(e.y);
            m = (static_cast<unsigned long long>(uni(e.w)) << 32) | uni(e.z);
            if (ANY) m &= live;
            if (m) break;
        }
    }
}

// SLAB = kSlabOct: `oct` is the batch's octant (batch_octant), else ignored.
// CULL (SLAB != kSlabExact, !COUNT): the exact cull of the anchor `cq` (cull_mask) beside every
// slab test, the root's included.
template <bool ANY, int SLAB, bool COUNT, bool CB = false, bool CULL = false>
__device__ void mesh_traverse(const DevScene& S, const int4 M, const Ray& r, int oct, unsigned long long mask,
                              uint32_t lane, uint4* stk, unsigned long long* sT, float& sc_t, uint32_t& sc_tri,
                              unsigned long long& live, Counts& cnt, const CullRay& cq = CullRay{}) {
    static_assert(!CULL || SLAB != kSlabExact, "the cull runs in FAST batches of the lean walk only");
    constexpr bool FAST = SLAB != kSlabExact;
    if (M.y == 0) return;
    const bool OCT = SLAB == kSlabOct && !COUNT && !RTX_STAMPS_WALK;
    const float4* nb = OCT ? reinterpret_cast<const float4*>(reinterpret_cast<const char*>(S.nodes) +
                                                             static_cast<uint32_t>(oct) * S.oct_bytes)
                           : S.nodes;
    // root (odd global index; every child pair starts at an even one, 64-B aligned)
    float4 b0, b1;
    ldcb32(nb, static_cast<uint32_t>(M.x), b0, b1);   // M.x: the root's byte offset
    [[maybe_unused]] float4 c0, c1;   // the root's cull record, loaded beside it
    if (CULL) ldcb32(cq.base, static_cast<uint32_t>(M.x), c0, c1);
    if (COUNT && ((mask >> lane) & 1ull)) cnt.c[kSlab]++;
    unsigned long long m =
        (OCT ? slab_mask<kSlabOct>(b0, b1, r) : slab_mask<FAST ? kSlabFast : kSlabExact>(b0, b1, r)) & mask;
    if (CULL && m) {
        float n;
        if (__float_as_uint(c1.w)) {
            if (COUNT && ((m >> lane) & 1ull)) cnt.c[kCullTests]++;
            m &= cull_pass<ANY>(c0, c1, r, cq, sc_t, n);
        }
    }
    if (m == 0) return;
    if ((!COUNT || CULL) && !RTX_STAMPS_WALK)
        bvh_walk_lean<ANY, OCT ? kSlabOct : (FAST ? kSlabFast : kSlabExact), CB, CULL, COUNT>(
            S, nb, cull_sign(M.z, ANY), r, __float_as_uint(b1.z), __float_as_uint(b1.w), m, mask, lane, stk, sc_t,
            sc_tri, live, nullptr, 0u, cq, &cnt);
    else
        bvh_walk<ANY, FAST, COUNT>(S, cull_sign(M.z, ANY), r, __float_as_uint(b1.z), __float_as_uint(b1.w), m, mask,
                                   lane, stk, sT, sc_t, sc_tri, live, cnt);
}

// One part of a split traversal: the lanes that reach frontier node E (slab tests of the
// root and of every node on E's path, exactly the tests the full DFS makes on the way
// down), then the DFS of E's subtree.  Parts partition the triangles, so the closest-hit
// result is the minimum of the parts' (t, triangle index) keys — left-then-right DFS
// order is increasing triangle index (checked at upload), which makes the key minimum
// the reference's first-found, strict-< winner — and occlusion is the OR of the parts.
// SLAB = kSlabOct: `oct` is the batch's octant (batch_octant) and the part walks that copy.
// CB: kSpecCullBack (tri_t_wave).
// CULL: as mesh_traverse, on the part's path and below it.
// Returns, when `timed` (motion mode, FrameArgs::part_cost), the duration of the walk below E in
// cycles (0 when no lane reaches E): the part's share of the tile's one-piece cost; else 0.
template <bool ANY, int SLAB, bool CB = false, bool CULL = false>
__device__ unsigned long long part_traverse(const DevScene& S, const int4 E, const Ray& r, int oct,
                                            unsigned long long mask, uint32_t lane, uint4* stk, float& sc_t,
                                            uint32_t& sc_tri, unsigned long long& live, Counts& cnt,
                                            const uint32_t* occ_word = nullptr, uint32_t occ_bit = 0,
                                            const CullRay& cq = CullRay{}, bool timed = false) {
    static_assert(!CULL || SLAB != kSlabExact, "the cull runs in FAST batches only");
    constexpr bool FAST = SLAB != kSlabExact;
    if (E.x < 0) return 0;   // unused entry of a device-animated mesh's reserved frontier
    const int4 M = ldcb16i(S.meshes, static_cast<uint32_t>(E.x) * 16u);
    const float4* nb = SLAB == kSlabOct ? reinterpret_cast<const float4*>(reinterpret_cast<const char*>(S.nodes) +
                                                                          static_cast<uint32_t>(oct) * S.oct_bytes)
                                        : S.nodes;
    float4 b0, b1;
    ldcb32(nb, static_cast<uint32_t>(M.x), b0, b1);   // M.x: the root's byte offset
    [[maybe_unused]] float4 q0, q1;   // cull records loaded beside their nodes (one latency per step)
    if (CULL) ldcb32(cq.base, static_cast<uint32_t>(M.x), q0, q1);
    unsigned long long m = slab_mask<SLAB>(b0, b1, r) & mask;
    if (CULL && m) {
        float n;
        if (__float_as_uint(q1.w)) m &= cull_pass<ANY>(q0, q1, r, cq, sc_t, n);
    }
    uint32_t link = __float_as_uint(b1.z), ntri = __float_as_uint(b1.w);
    const uint32_t path = static_cast<uint32_t>(E.z);
    for (int d = 0; d < E.w && m; ++d) {
        NodePair P;
        ldcb64(nb, link, P.l0, P.l1, P.r0, P.r1);
        const bool right = (path >> d) & 1u;
        if (CULL) ldcb32(cq.base, link + (right ? 32u : 0u), q0, q1);
        const float4 c0 = right ? P.r0 : P.l0, c1 = right ? P.r1 : P.l1;
        m &= slab_mask<SLAB>(c0, c1, r);
        if (CULL) {
            float n;
            if (__float_as_uint(q1.w)) m &= cull_pass<ANY>(q0, q1, r, cq, sc_t, n);
        }
        link = __float_as_uint(c1.z);
        ntri = __float_as_uint(c1.w);
    }
    if (m == 0) return 0;
    // (read unconditionally: a `timed` test here made the compiler version the walk loop)
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (!RTX_STAMPS_WALK)
        bvh_walk_lean<ANY, SLAB, CB, CULL>(S, nb, cull_sign(M.z, ANY), r, link, ntri, m, mask, lane, stk, sc_t,
                                           sc_tri, live, occ_word, occ_bit, cq);
    else
        bvh_walk<ANY, FAST, false>(S, cull_sign(M.z, ANY), r, link, ntri, m, mask, lane, stk, nullptr, sc_t, sc_tri,
                                   live, cnt, occ_word, occ_bit);
    return timed ? __builtin_amdgcn_s_memtime() - t0 : 0ull;   // (timed: the caller's use only)
}

struct RGB {
    float r, g, b;
};

// Material::Shade (Material.h:41-123) via BRDFs.h; m2.yzw holds (rgb*kd)/PI computed on
// the host with the same binary32 operations (BRDF::Lambert, BRDFs.h:14-17).
// KINDS: the material kinds the scene's geometry can hit (kSpecKind* bits, established by the
// host at upload; 0 = any).  Only their branches are compiled; a Lambert-only scene's BRDF is
// the precomputed constant with no dispatch at all.
template <int KINDS = 0>
__device__ __forceinline__ RGB shade(const DevScene& S, uint32_t mi, float nx, float ny, float nz, float lx, float ly,
                                     float lz, float vx, float vy, float vz, Counts& cnt, bool count) {
    constexpr int K = KINDS ? KINDS : kSpecKindAll;
    if (K == kSpecKindLambert) {
        const float4 m2 = ldc(S.materials, 3 * mi + 2);
        if (count) cnt.c[kShadeLambert]++;
        return {m2.y, m2.z, m2.w};
    }
    const float4 m0 = ldc(S.materials, 3 * mi), m1 = ldc(S.materials, 3 * mi + 1), m2 = ldc(S.materials, 3 * mi + 2);
    const int kind = __float_as_int(m0.x);
    RGB c{0.f, 0.f, 0.f};
    if ((K & kSpecKindSolid) && kind == RTX_MAT_SOLID_COLOR) {
        c = {m0.y, m0.z, m0.w};
    } else if ((K & kSpecKindLambert) && kind == RTX_MAT_LAMBERT) {
        if (count) cnt.c[kShadeLambert]++;
        c = {m2.y, m2.z, m2.w};
    } else if ((K & kSpecKindPhong) && kind == RTX_MAT_LAMBERT_PHONG) {
        if (count) { cnt.c[kShadeLambert]++; cnt.c[kShadePhong]++; }
        // BRDF::Phong (BRDFs.h:33-40)
        const float s2 = 2.f * smax(nx * lx + ny * ly + nz * lz, 0.f);
        const float rx = lx - nx * s2, ry = ly - ny * s2, rz = lz - nz * s2;
        const float cosa = smax(rx * vx + ry * vy + rz * vz, 0.f);
        const float spec = m1.y * powf(cosa, m1.z);
        c = {m2.y + spec, m2.z + spec, m2.w + spec};
    } else if ((K & kSpecKindCT) && kind == RTX_MAT_COOK_TORRANCE) {
        if (count) cnt.c[kShadeCT]++;
        float hx = vx + lx, hy = vy + ly, hz = vz + lz;
        const float hm = sqrtf(hx * hx + hy * hy + hz * hz);
        hx = hx / hm; hy = hy / hm; hz = hz / hm;
        const bool dielectric = (m1.w == 0.f);
        const float f0r = dielectric ? 0.04f : m0.y, f0g = dielectric ? 0.04f : m0.z, f0b = dielectric ? 0.04f : m0.w;
        const float p = powf(1.f - smax(hx * vx + hy * vy + hz * vz, 0.f), 5.f);
        const float Fr = f0r + ((1.f - f0r) * p), Fg = f0g + ((1.f - f0g) * p), Fb = f0b + ((1.f - f0b) * p);
        const float rough = m2.x;
        const float a = rough * rough;
        const float sqrA = a * a;
        const float ndh = smax(nx * hx + ny * hy + nz * hz, 0.f);
        const float in = (ndh * ndh) * ((a * a) - 1.f) + 1.f;
        const float D = sqrA / (RTX_PI * (in * in));
        const float k = ((a + 1.f) * (a + 1.f)) / 8.f;
        const float cv = smax(nx * vx + ny * vy + nz * vz, 0.f);
        const float cl = smax(nx * lx + ny * ly + nz * lz, 0.f);
        const float G = (cv / ((cv * (1.f - k)) + k)) * (cl / ((cl * (1.f - k)) + k));
        const float den = (4.f * smax(vx * nx + vy * ny + vz * nz, 0.0001f)) * smax(lx * nx + ly * ny + lz * nz, 0.0001f);
        const float kr = dielectric ? 1.f - Fr : 0.f, kg = dielectric ? 1.f - Fg : 0.f, kb = dielectric ? 1.f - Fb : 0.f;
        c.r = (m0.y * kr) / RTX_PI + ((Fr * D) * G) / den;
        c.g = (m0.z * kg) / RTX_PI + ((Fg * D) * G) / den;
        c.b = (m0.w * kb) / RTX_PI + ((Fb * D) * G) / den;
    }
    return c;
}

// motion mode (FrameArgs::part_cost): a split launch's wave adds the duration of its walk below
// its frontier part (cycles) to its tile's cost, in the tile cost's unit (16 cycles).  The parts'
// walks partition the one-piece walk, so their sum stands for the tile's one-piece cost without
// each part wave's fixed work (ray, planes, the part's path), which would keep a tile that stopped
// being heavy in the split set.
__device__ __forceinline__ void part_cost_add(uint32_t* cost, unsigned long long dt) {
    dt >>= 4;
    atomicAdd(cost, static_cast<uint32_t>(dt < 0xffffffffull ? dt : 0xffffffffull));
}

__device__ __forceinline__ uint32_t q8(float c) {
    // static_cast<uint8_t>(c * 255) as x86 compiles it: cvttss2si then the low byte
    // (NaN and out-of-int32-range values give 0x80000000 -> 0).
    const float x = c * 255;
    if (!(x > -2147483648.f && x < 2147483648.f)) return 0u;
    return static_cast<uint32_t>(static_cast<int32_t>(x)) & 0xffu;
}

}  // namespace

// Renderer::RenderPixel (source/Renderer.cpp:100-182) for a 16x16 tile per workgroup.
//
// PHASE 0 renders every tile except the heavy ones.  A heavy tile (measured cost far above
// the frame's per-slot share, see rtx_reorder_kernel) is rendered by three launches over the
// BVH frontier parts instead, so its serial traversal work is spread over many workgroups:
//   PHASE 1  grid (heavy, parts):          closest hit of one part -> atomicMin of the
//                                          {t bits, triangle} key per pixel
//   PHASE 2  grid (heavy, parts, lights):  shadow ray of one light against one part ->
//                                          atomicOr of the light's occlusion bit
//   PHASE 3  grid (heavy):                 hit record from the key, spheres/planes
//                                          occlusion + the bits, shading, output
// A light-major frame (FrameArgs::lm_*, small launches: a stripe share) replaces PHASE 0 by
//   PHASE 4  grid (tiles):                 PHASE 0 up to the hit record, which it writes
//   PHASE 5  persistent waves over the (tile, light) items: that light's shadow ray from the
//                                          record -> the occluded lanes; the tile's last light wave
//                                          shades every light in order (the occlusion published)
// Every phase recomputes the primary ray and the sphere/plane hits with the same code, so
// all of them see bit-identical values.
// DEEP: the variant for scenes whose BVH is kStackDepth or more levels deep (a DFS stack of
// kStackDepthDeep entries per wave in LDS; fewer waves fit a CU, so it is used only then).
// HSTK (with DEEP): the stacks in HBM instead (DevScene::hstk, any depth: the reference's
// recursion has no limit), for trees kStackDepthDeep or more levels deep.
// SPEC (kSpec* bits, rtx_kernels.h): uniform facts of the scene and frame the host checked at
// launch, compiled in instead of branched on (same operations, so the same pixels; fewer
// uniform branches, selects and registers; constant plane / mesh counts unroll their loops:
// Bunny 74.2 -> 61.2 us with RTX_SPEC_WAVES).
// Occupancy targets of the specialised kernels.  The variants with a constant mesh count ask for
// 8 waves per SIMD: the Lambert-only one then needs 47 VGPRs and 78 SGPRs (8 spilled to VGPR
// lanes, outside the loops), so the SGPR file no longer caps it at 7 waves like the generic
// kernel's 106 SGPRs (Bunny 61.1 -> 60.6 us, Bunny + 8 lights 427 -> 418 us; 10 waves: no gain);
// W4_Optional's variant 231 -> 223 us.  The variant with spheres and meshes stays at 7 (8: +4 %).
// CULLK: the variant with the exact cull (DevScene::cull; launched only for scenes that have the
// records — the code of the cull paths costs the kernel without them registers and 8 %).
#define f_mode (kComb ? RTX_MODE_COMBINED : F.mode)
#define f_shadows (kComb ? 1 : F.shadows)
#define n_sph (kNoSph ? 0u : S.n_spheres)
#define n_pl (kP5 ? 5u : S.n_planes)          // constant trip counts: the plane and mesh loops unroll
#define n_mesh (kNoMesh ? 0u : (kOneMesh ? 1u : S.n_meshes))
// One wave tile of one phase (rtx_render_kernel below dispatches the tiles and describes the phases): `widx` = the
// wave's index in the launch (PHASE 5: its item), `stk` / `sT` its DFS stacks, `pnum` its shadow-ray
// plane numerators in LDS.
// A split wave's duration for the frontier refinement (FrameArgs::part_max), sharded by wave.
template <int PHASE>
__device__ __forceinline__ void part_stat(const FrameArgs& F, uint32_t part, uint32_t widx, uint32_t lane,
                                          unsigned long long t0) {
    if (!F.part_max || lane != 0) return;
    const unsigned long long d = (__builtin_amdgcn_s_memtime() - t0) >> 4;
    atomicMax(F.part_max + ((static_cast<uint32_t>(PHASE) - 1u) * kMaxParts + part) * kPartShards + widx % kPartShards,
              static_cast<uint32_t>(d < 0xffffffffull ? d : 0xffffffffull));
}

template <bool COUNT, int PHASE, bool DEEP, int SPEC, bool HSTK, bool CULLK>
__device__ __forceinline__ void render_tile(const DevScene& S, const FrameArgs& F, uint32_t widx, uint32_t tile,
                                            uint32_t part, uint32_t light, uint4* stk, unsigned long long* sT,
                                            float (*pnum)[64], uint32_t lane) {
    constexpr int kKinds = SPEC & kSpecKindAll;
    constexpr bool kPoint = (SPEC & kSpecPoint) != 0;
    constexpr bool kNoSph = (SPEC & kSpecNoSpheres) != 0, kComb = (SPEC & kSpecCombShadows) != 0;
    constexpr bool kP5 = (SPEC & kSpecFivePlanes) != 0, kOneMesh = (SPEC & kSpecOneMesh) != 0;
    constexpr bool kNoMesh = (SPEC & kSpecNoMesh) != 0;
    constexpr bool kRoom = (SPEC & kSpecRoomPlanes) != 0 && (SPEC & kSpecFivePlanes) != 0;
    constexpr bool kCullBack = (SPEC & kSpecCullBack) != 0 && !COUNT;
#if RTX_STAMPS
    // diagnostic build only: per-wave {start, end, hw_id} in the counters buffer
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_prim = t_start, t_shadow = 0;   // primary hit done; shadow mesh walks
#endif
    if constexpr (HSTK) {   // this wave's stacks in HBM
        stk = S.hstk + static_cast<size_t>(widx) * S.hstk_depth;
        if (COUNT) sT = S.hstkT + static_cast<size_t>(widx) * S.hstk_depth;
    }
    const uint32_t slot = widx * 64u + lane;                 // heavy-pixel slot (PHASE > 0)
    const uint32_t per_view = F.tiles_x * F.tiles_y;
    const uint32_t view = tile / per_view;
    const uint32_t rem = tile - view * per_view;
    const uint32_t bx = rem % F.tiles_x;
    const ViewCam& V = F.cam[view];
    uint32_t gy = rem / F.tiles_x;
    unsigned long long t_block0 = 0;
    if (F.cost || ((PHASE == 1 || PHASE == 2) && F.part_max)) t_block0 = __builtin_amdgcn_s_memtime();
    if (F.groups_per_stripe) {
        // view v owns the stripes s with s % step == (first - v) mod step (rtx.h)
        const uint32_t first = (F.stripe_first + F.stripe_step - view % F.stripe_step) % F.stripe_step;
        const uint32_t k = gy / F.groups_per_stripe, sub = gy % F.groups_per_stripe;
        gy = (first + k * F.stripe_step) * F.groups_per_stripe + sub;
    }
    const int px = static_cast<int>(bx * kWaveTile + (lane & 7u));
    const int py = static_cast<int>(gy * kWaveTile + (lane >> 3));
    const bool valid = px < static_cast<int>(F.width) && py < static_cast<int>(F.height);
    Counts cnt;
    if (COUNT || RTX_STAMPS) for (int k = 0; k < kNumCounters; ++k) cnt.c[k] = 0;
    if (COUNT && valid) cnt.c[kPixels] = 1;

    // ---- primary ray (Renderer.cpp:104-114; Matrix::TransformVector Matrix.cpp:35-42)
    // (px + 0.5f) / W and (2 * (py + 0.5f)) / H as Markstein quotients with the exact
    // reciprocals RN(1/W), RN(1/H) (divided on the host, FrameArgs): numerators in [0.5, 2^17], divisors in
    // [1, 2^16] lie inside div_rn's domain (rtx_fastdiv.h), so each is the IEEE quotient.
    const int W = static_cast<int>(F.width), H = static_cast<int>(F.height);
    const float fW = static_cast<float>(W), fH = static_cast<float>(H);
    const float cx = (2.f * div_rn(px + 0.5f, fW, F.inv_width) - 1) * F.aspect * V.fov;
    const float cy = (1.f - div_rn(2.f * (py + 0.5f), fH, F.inv_height)) * V.fov;
    float dx = V.right[0] * cx + V.up[0] * cy + V.forward[0] * 1.f;
    float dy = V.right[1] * cx + V.up[1] * cy + V.forward[1] * 1.f;
    float dz = V.right[2] * cx + V.up[2] * cy + V.forward[2] * 1.f;
    const float dm = sqrtf(dx * dx + dy * dy + dz * dz);
    div3_exact(dx, dy, dz, dm);   // dx /= dm; ... (Vector3::Normalize)
    unsigned long long vslow;
    const Ray vr = make_ray(V.origin[0], V.origin[1], V.origin[2], dx, dy, dz, 0.0001f, FLT_MAX, vslow);
    const unsigned long long active = ballot(valid);
    // FAST: every active lane's inverse direction finite and non-zero (make_ray's domain)
    const bool fast = (active & vslow) == 0 && S.tri_fast;
    // octant of the wave's primary rays (-1: mixed signs, or no octant copies)
    const int poct = (fast && S.oct_bytes && (PHASE == 0 || PHASE == 4)) ? batch_octant(vr, active) : -1;
    // exact cull of the view's camera anchor (FAST waves; a direction normalised from a magnitude
    // of at least 2^-30 has |d| = 1 +- 3u, which the bound assumes)
    constexpr bool kCull = CULLK && !RTX_STAMPS_WALK;   // (with COUNT: rtx_count_work_culled)
    const bool pcull = kCull && S.cull_stride && fast && (PHASE == 0 || PHASE == 1 || PHASE == 4);
    CullRay pq{};
    if (pcull)
        pq = cull_ray(S.cull + static_cast<size_t>(uni(view)) * (S.cull_stride / 16u), vr, dm >= 0x1p-30f,
                      F.cam[uni(view)].cull_bt);

    // ---- Scene::GetClosestHit (Scene.cpp:29-66)
    float best_t = FLT_MAX, sc_t = FLT_MAX;
    // kind: 0 none, 1 sphere, 2 plane, 3 triangle; best_idx: the record's BYTE offset
    uint32_t best_kind = 0, best_idx = 0;
    // (PHASE 5 reads the hit record PHASE 4 wrote: no closest-hit work)
    for (uint32_t i = 0; i < ((PHASE == 5 || PHASE == 6) ? 0u : n_sph * 16u); i += 16u) {
        const float4 s = ldcb16(S.spheres, opaque(i));
        if (COUNT && valid) cnt.c[kSphere]++;
        const SphereProj q = sphere_perp(s, vr);
        const unsigned long long near = ballot(!(s.w < q.perp)) & active;
        if (!near) continue;
        const float t = sphere_t(s, q);
        const bool h = ((near >> lane) & 1ull) & !(t < vr.tmin) & !(t > vr.tmax);
        sc_t = h ? t : sc_t;
        const bool b = h & (t < best_t);
        best_t = b ? t : best_t;
        best_kind = b ? 1u : best_kind;
        best_idx = b ? i : best_idx;
    }
    // the room's planes as a / d (room_a), for a wave whose ray origins are finite.  The camera
    // numerators come from the host (ViewCam::room_a); in a FAST wave every d is inside div_rn's
    // divisor domain with its RN(1/d) already in the ray, so when the host found the numerators
    // inside theirs too, t = RN(a / d) costs 3 VALU instead of the 11 of IEEE `/`.
    const bool room_p =
        kRoom && PHASE != 5 && PHASE != 6 && !RTX_ABL_PPLANE && (active & ~ballot(finite3(vr.ox, vr.oy, vr.oz))) == 0;
    if (room_p) {
        // the view's record through a readfirstlane'd index: scalar loads (the view index
        // itself stays a VGPR value; making it uniform everywhere measured slower)
        const ViewCam& VU = F.cam[uni(view)];
        const bool mk = fast && VU.room_fast;
        for_room_planes([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int A = kRoomAxes[k];
            float t;
            if (mk) {
                t = div_rn(VU.room_a[k], room_d<A>(vr), room_inv<A>(vr));
            } else {
                float4 p0, p1;
                ldcb32(S.planes, k * 32u, p0, p1);
                t = room_a<A>(p0, vr) / room_d<A>(vr);
            }
            const bool h = valid & (t >= vr.tmin) & (t < vr.tmax);
            sc_t = h ? t : sc_t;
            const bool b = h & (t < best_t);
            best_t = b ? t : best_t;
            best_kind = b ? 2u : best_kind;
            best_idx = b ? static_cast<uint32_t>(k * 32) : best_idx;
        });
    }
    for (uint32_t i = 0; i < ((RTX_ABL_PPLANE || room_p || PHASE == 5 || PHASE == 6) ? 0u : n_pl * 32u); i += 32u) {
        float4 p0, p1;
        ldcb32(S.planes, opaque(i), p0, p1);
        if (COUNT && valid) cnt.c[kPlane]++;
        const float num = plane_num(p0, p1, vr), den = plane_den(p1, vr);
        const float t = num / den;
        const bool h = valid & (t >= vr.tmin) & (t < vr.tmax);
        sc_t = h ? t : sc_t;
        const bool b = h & (t < best_t);
        best_t = b ? t : best_t;
        best_kind = b ? 2u : best_kind;
        best_idx = b ? i : best_idx;
    }
    if (PHASE == 0 || PHASE == 4) {
        for (uint32_t mi = 0; mi < ((RTX_ABL_PMESH) ? 0u : n_mesh); ++mi) {
            const int4 M = ldcb16i(S.meshes, opaque(mi * 16u));
            uint32_t sc_tri = 0;
            unsigned long long unused = 0;
            if (poct >= 0 && pcull)
                mesh_traverse<false, kSlabOct, COUNT, kCullBack, kCull>(S, M, vr, poct, active, lane, stk, sT, sc_t,
                                                                        sc_tri, unused, cnt, pq);
            else if (poct >= 0)
                mesh_traverse<false, kSlabOct, COUNT, kCullBack>(S, M, vr, poct, active, lane, stk, sT, sc_t, sc_tri,
                                                                 unused, cnt);
            else if (fast && pcull)
                mesh_traverse<false, kSlabFast, COUNT, kCullBack, kCull>(S, M, vr, 0, active, lane, stk, sT, sc_t,
                                                                         sc_tri, unused, cnt, pq);
            else if (fast)
                mesh_traverse<false, kSlabFast, COUNT, kCullBack>(S, M, vr, 0, active, lane, stk, sT, sc_t, sc_tri,
                                                                  unused, cnt);
            else
                mesh_traverse<false, kSlabExact, COUNT, kCullBack>(S, M, vr, 0, active, lane, stk, sT, sc_t, sc_tri,
                                                                   unused, cnt);
            if (sc_t < best_t) { best_t = sc_t; best_kind = 3; best_idx = sc_tri; }
        }
#if RTX_STAMPS
        t_prim = __builtin_amdgcn_s_memrealtime();
#endif
    } else if (PHASE == 1) {
        // one frontier part; sc0 = the scratch t the reference enters the meshes with
        const int4 E = ldc(S.parts, part);
        if (RTX_P1_SHARED_T && valid) {
            // the parts that finished before this one already merged their keys: a lane's final t
            // is at most their minimum T, so the walk needs only hits with t <= T (initial scratch t
            // = the next float above T; equal t still compete on the triangle index).  Read at the
            // coherence point (the keys' atomics come from every XCD); a stale key is larger, still
            // a bound.
            const unsigned long long k0 = __hip_atomic_load(&F.hit_key[slot], __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
            const float tb = __uint_as_float(static_cast<uint32_t>(k0 >> 32) + 1u);
            if (k0 != ~0ull && tb < sc_t) sc_t = tb;
        }
        const float sc0 = sc_t;
        uint32_t sc_tri = 0;
        unsigned long long unused = 0;
        const int oct = (fast && S.oct_bytes) ? batch_octant(vr, active) : -1;
        const bool timed = F.part_cost && F.cost;
        unsigned long long wdt;
        if (oct >= 0 && pcull)
            wdt = part_traverse<false, kSlabOct, kCullBack, kCull>(S, E, vr, oct, active, lane, stk, sc_t, sc_tri,
                                                                   unused, cnt, nullptr, 0u, pq, timed);
        else if (oct >= 0)
            wdt = part_traverse<false, kSlabOct, kCullBack>(S, E, vr, oct, active, lane, stk, sc_t, sc_tri, unused,
                                                            cnt, nullptr, 0u, CullRay{}, timed);
        else if (fast && pcull)
            wdt = part_traverse<false, kSlabFast, kCullBack, kCull>(S, E, vr, 0, active, lane, stk, sc_t, sc_tri,
                                                                    unused, cnt, nullptr, 0u, pq, timed);
        else if (fast)
            wdt = part_traverse<false, kSlabFast, kCullBack>(S, E, vr, 0, active, lane, stk, sc_t, sc_tri, unused,
                                                             cnt, nullptr, 0u, CullRay{}, timed);
        else
            wdt = part_traverse<false, kSlabExact, kCullBack>(S, E, vr, 0, active, lane, stk, sc_t, sc_tri, unused,
                                                              cnt, nullptr, 0u, CullRay{}, timed);
        if (valid && sc_t < sc0)   // accepted t >= tmin > 0: the float bits order like the values
            atomicMin(&F.hit_key[slot], (static_cast<unsigned long long>(__float_as_uint(sc_t)) << 32) | sc_tri);
        if (timed && lane == 0 && wdt) part_cost_add(F.cost + tile, wdt);
        part_stat<PHASE>(F, part, widx, lane, t_block0);
        RTX_SPLIT_STAMP();
        return;
    } else if (PHASE == 2 || PHASE == 3) {
        // the minimum over the parts; strict < against the sphere/plane winner, as after
        // every mesh in Scene::GetClosestHit (Scene.cpp:56-63)
        const unsigned long long key = F.hit_key[slot];
        const float T = __uint_as_float(static_cast<uint32_t>(key >> 32));
        if (key != ~0ull && T < best_t) { best_t = T; best_kind = 3; best_idx = static_cast<uint32_t>(key); }
    }

    // ---- hit record (rebuilt from t: ray.origin + t * ray.direction, Utils.h:62-64)
    bool did = best_kind != 0;
    float hx = 0.f, hy = 0.f, hz = 0.f, nx = 0.f, ny = 0.f, nz = 0.f;
    uint32_t mat = 0;
    const size_t lm_slot = 2 * (static_cast<size_t>(tile) * 64u + lane);   // (PHASE 4/5) the pixel's record
    if (PHASE == 5 || PHASE == 6) {   // PHASE 4's record of this pixel (the previous launch: visible)
        const float4 r0 = F.lm_rec[lm_slot], r1 = F.lm_rec[lm_slot + 1];
        hx = r0.x; hy = r0.y; hz = r0.z; nx = r0.w; ny = r1.x; nz = r1.y;
        mat = __float_as_uint(r1.z);
        did = __float_as_uint(r1.w) != 0u;
    } else if (did) {
        hx = vr.ox + vr.dx * best_t; hy = vr.oy + vr.dy * best_t; hz = vr.oz + vr.dz * best_t;
        if (best_kind == 1) {
            const float4 s = ldcb16(S.spheres, best_idx);
            nx = hx - s.x; ny = hy - s.y; nz = hz - s.z;
            const float m = sqrtf(nx * nx + ny * ny + nz * nz);   // closestHit.normal.Normalize()
            div3_exact(nx, ny, nz, m);   // nx /= m; ny /= m; nz /= m
            mat = ldc(S.sphere_mat, best_idx >> 4);
        } else if (best_kind == 2) {
            float4 p0, p1;
            ldcb32(S.planes, best_idx, p0, p1);
            nx = p1.x; ny = p1.y; nz = p1.z;
            mat = __float_as_uint(p0.w);
        } else {
            Tri T;
            ldcb64(S.tris, best_idx, T.a, T.b, T.c, T.d);   // best_idx: byte offset
            nx = T.a.w; ny = T.b.w; nz = T.c.w;
            mat = __float_as_uint(T.d.x);
        }
    }
    if (COUNT && did) cnt.c[kHit]++;
    if (PHASE == 4) {   // light-major: the record for PHASE 5, and this wave's share of the tile's cost
        F.lm_rec[lm_slot] = make_float4(hx, hy, hz, nx);
        F.lm_rec[lm_slot + 1] = make_float4(ny, nz, __uint_as_float(mat), __uint_as_float(did ? 1u : 0u));
        if (F.cost && lane == 0) part_cost_add(F.cost + tile, __builtin_amdgcn_s_memtime() - t_block0);
        return;
    }

    float shadowFactor = 1.f;
    float fr = 0.f, fg = 0.f, fb = 0.f;
    const unsigned long long hitmask = ballot(did);
    unsigned long long lm_occ = 0;   // PHASE 5: the lanes whose shadow ray toward `light` is occluded
    // The reference's light loop (Renderer.cpp:128-176).  Light-major frames run it in two launches:
    // PHASE 5 casts its one light's shadow ray and only records the occluded lanes; PHASE 6 (lm_shade)
    // runs it over every light with each light's occlusion the one PHASE 5 published
    // (FrameArgs::lm_mask), no shadow ray cast.
    constexpr bool lm_shade = PHASE == 6;
    if (hitmask) {
        const uint32_t l_first = (PHASE == 2 || PHASE == 5) ? light : 0u;
        const uint32_t l_end = (PHASE == 2 || PHASE == 5) ? light + 1 : (RTX_ABL_LIGHTS ? 0u : S.n_lights);
        // originOffset = hit.origin + hit.normal * 0.0001f (Renderer.cpp:126)
        const float oox = hx + nx * 0.0001f, ooy = hy + ny * 0.0001f, ooz = hz + nz * 0.0001f;
        const float vx = -dx, vy = -dy, vz = -dz;
        // shadow rays start at originOffset for every light: one finiteness test for all of them
        const bool room_s =
            kRoom && PHASE != 2 && !RTX_ABL_SPLANE && (hitmask & ~ballot(finite3(oox, ooy, ooz))) == 0;
        for (uint32_t li = l_first; li < l_end; ++li) {
            float4 L0, L1;
            ldcb32(S.lights, opaque(li * 32u), L0, L1);
            const int ltype = kPoint ? RTX_LIGHT_POINT : __float_as_int(L0.w);
            const bool known = (ltype == RTX_LIGHT_POINT || ltype == RTX_LIGHT_DIRECTIONAL);
            float lx = known ? L0.x - oox : 0.f, ly = known ? L0.y - ooy : 0.f, lz = known ? L0.z - ooz : 0.f;
            const float mag = sqrtf(lx * lx + ly * ly + lz * lz);
            div3_exact(lx, ly, lz, mag);
            bool occ = false;
            if (lm_shade && f_shadows) {   // PHASE 6: published by the previous launch
                const unsigned long long mk = F.lm_mask[static_cast<size_t>(tile) * F.lm_lights + li];
                occ = did && ((mk >> lane) & 1ull);
            } else if (f_shadows) {
                // Scene::DoesHit (Scene.cpp:68-96) on Ray{originOffset, l, 1e-4, |l|}; `live` =
                // lanes still without an occluder (first hit wins, order irrelevant for a bool)
                unsigned long long sslow;
                const Ray sr = make_ray(oox, ooy, ooz, lx, ly, lz, 0.0001f, mag, sslow);
                unsigned long long live = hitmask;
                const bool sfast = (hitmask & sslow) == 0 && S.tri_fast;
                const int soct =
                    (sfast && S.oct_bytes && (PHASE == 0 || PHASE == 5) && n_mesh) ? batch_octant(sr, hitmask) : -1;
                // exact cull of the light's anchor: lanes with mag <= cull_T[li] (and a direction
                // normalised from at least 2^-30)
                const bool scull = kCull && S.cull_stride && sfast && (PHASE == 0 || PHASE == 2 || PHASE == 5) && n_mesh;
                CullRay sq{};
                if (scull)
                    sq = cull_ray(S.cull + static_cast<size_t>(kMaxViews + li) * (S.cull_stride / 16u), sr,
                                  mag >= 0x1p-30f && mag <= ldc(S.cull_T, li), ldc(S.cull_T, li));
                if (COUNT && did) cnt.c[kShadow]++;
                // (single-condition loops with a separate exit test: a `&& live` loop
                // condition is carried as a VGPR boolean by the compiler)
                for (uint32_t i = 0; i < (PHASE == 2 ? 0u : n_sph * 16u); i += 16u) {
                    const float4 s = ldcb16(S.spheres, opaque(i));
                    if (COUNT && ((live >> lane) & 1ull)) cnt.c[kSphere]++;
                    const SphereProj q = sphere_perp(s, sr);
                    const unsigned long long near = ballot(!(s.w < q.perp)) & live;
                    if (!near) continue;
                    const float t = sphere_t(s, q);
                    live &= ~(near & ballot(!(t < sr.tmin)) & ballot(!(t > sr.tmax)));
                }
                // HitTest_Plane's numerator (p0 - o) . n depends only on the shadow ray's origin,
                // the same originOffset for every light: the first light computes it and keeps it
                // in LDS, the others read it back (same value, bit for bit).  One loop version
                // per case, so no per-plane select.
                const uint32_t np = (RTX_ABL_SPLANE || PHASE == 2 || room_s) ? 0u : n_pl * 32u;
                const bool cache_ok = !COUNT && np <= static_cast<uint32_t>(kPlaneCache) * 32u;
                if (room_s) {   // a / d (room_a): cheaper than the cached numerator
                    for_room_planes([&](auto kc) {
                        constexpr int k = decltype(kc)::value;
                        constexpr int A = kRoomAxes[k];
                        float4 p0, p1;
                        ldcb32(S.planes, k * 32u, p0, p1);
                        const float num = room_a<A>(p0, sr), den = room_d<A>(sr);
                        const unsigned long long cand = plane_cand(num, den, sr.tmax) & live;
                        if (!cand) return;
                        const float t = num / den;
                        live &= ~(ballot(t >= sr.tmin) & ballot(t < sr.tmax) & cand);
                    });
                } else if (cache_ok && li != l_first) {
                    for (uint32_t i = 0; i < np; i += 32u) {
                        float4 p0, p1;
                        ldcb32(S.planes, opaque(i), p0, p1);
                        const float num = pnum[i >> 5][lane];
                        const float den = plane_den(p1, sr);
                        const unsigned long long cand = plane_cand(num, den, sr.tmax) & live;
                        if (!cand) continue;
                        const float t = num / den;
                        live &= ~(ballot(t >= sr.tmin) & ballot(t < sr.tmax) & cand);
                    }
                } else {
                    for (uint32_t i = 0; i < np; i += 32u) {
                        float4 p0, p1;
                        ldcb32(S.planes, opaque(i), p0, p1);
                        if (COUNT && ((live >> lane) & 1ull)) cnt.c[kPlane]++;
                        const float num = plane_num(p0, p1, sr), den = plane_den(p1, sr);
                        if (cache_ok) pnum[i >> 5][lane] = num;
                        const unsigned long long cand = plane_cand(num, den, sr.tmax) & live;
                        if (!cand) continue;   // also taken once no lane is live
                        const float t = num / den;
                        live &= ~(ballot(t >= sr.tmin) & ballot(t < sr.tmax) & cand);
                    }
                }
#if RTX_STAMPS
                const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();
#endif
                for (uint32_t mi = 0; mi < ((RTX_ABL_SMESH || !(PHASE == 0 || PHASE == 5)) ? 0u : n_mesh); ++mi) {
                    if (!live) break;
                    float st = 0.f;
                    uint32_t stri = 0;
                    const int4 M = ldcb16i(S.meshes, opaque(mi * 16u));
                    if (soct >= 0 && scull)
                        mesh_traverse<true, kSlabOct, COUNT, kCullBack, kCull>(S, M, sr, soct, live, lane, stk, sT, st,
                                                                               stri, live, cnt, sq);
                    else if (soct >= 0)
                        mesh_traverse<true, kSlabOct, COUNT, kCullBack>(S, M, sr, soct, live, lane, stk, sT, st, stri,
                                                                        live, cnt);
                    else if (sfast && scull)
                        mesh_traverse<true, kSlabFast, COUNT, kCullBack, kCull>(S, M, sr, 0, live, lane, stk, sT, st,
                                                                                stri, live, cnt, sq);
                    else if (sfast)
                        mesh_traverse<true, kSlabFast, COUNT, kCullBack>(S, M, sr, 0, live, lane, stk, sT, st, stri,
                                                                         live, cnt);
                    else
                        mesh_traverse<true, kSlabExact, COUNT, kCullBack>(S, M, sr, 0, live, lane, stk, sT, st, stri,
                                                                          live, cnt);
                }
#if RTX_STAMPS
                t_shadow += __builtin_amdgcn_s_memrealtime() - ts0;
#endif
                if (PHASE == 2) {
                    const int4 E = ldc(S.parts, part);
                    float st = 0.f;
                    uint32_t stri = 0;
                    const int poct2 = (sfast && S.oct_bytes) ? batch_octant(sr, hitmask) : -1;
                    const bool timed = F.part_cost && F.cost;
                    unsigned long long wdt;
                    if (poct2 >= 0 && scull)
                        wdt = part_traverse<true, kSlabOct, kCullBack, kCull>(S, E, sr, poct2, live, lane, stk, st, stri,
                                                                              live, cnt, &F.occ_bits[slot], 1u << li, sq,
                                                                              timed);
                    else if (poct2 >= 0)
                        wdt = part_traverse<true, kSlabOct, kCullBack>(S, E, sr, poct2, live, lane, stk, st, stri, live,
                                                                       cnt, &F.occ_bits[slot], 1u << li, CullRay{}, timed);
                    else if (sfast && scull)
                        wdt = part_traverse<true, kSlabFast, kCullBack, kCull>(S, E, sr, 0, live, lane, stk, st, stri,
                                                                               live, cnt, &F.occ_bits[slot], 1u << li, sq,
                                                                               timed);
                    else if (sfast)
                        wdt = part_traverse<true, kSlabFast, kCullBack>(S, E, sr, 0, live, lane, stk, st, stri, live, cnt,
                                                                        &F.occ_bits[slot], 1u << li, CullRay{}, timed);
                    else
                        wdt = part_traverse<true, kSlabExact, kCullBack>(S, E, sr, 0, live, lane, stk, st, stri, live,
                                                                         cnt, &F.occ_bits[slot], 1u << li, CullRay{}, timed);
                    if (did && !((live >> lane) & 1ull)) atomicOr(&F.occ_bits[slot], 1u << li);
                    if (timed && lane == 0 && wdt) part_cost_add(F.cost + tile, wdt);
                    continue;
                }
                occ = did & !((live >> lane) & 1ull);
                if (PHASE == 3) occ = occ || (did && ((F.occ_bits[slot] >> li) & 1u));
            }
            if (PHASE == 5) {
                lm_occ = ballot(occ);
                continue;
            }
            if (!did) continue;
            if (occ) {
                if (COUNT) cnt.c[kOccluded]++;
                shadowFactor *= 0.95f;
                continue;
            }
            if (COUNT) cnt.c[kShadeBase]++;
            if (f_mode == RTX_MODE_COMBINED || f_mode == RTX_MODE_RADIANCE) {
                // LightUtils::GetRadiance (Utils.h:355-369) at hit.origin
                float s = 0.f;
                bool any = true;
                if (ltype == RTX_LIGHT_POINT) {
                    const float ex = L0.x - hx, ey = L0.y - hy, ez = L0.z - hz;
                    s = L1.w / (ex * ex + ey * ey + ez * ez);
                } else if (ltype == RTX_LIGHT_DIRECTIONAL) {
                    s = L1.w;
                } else {
                    any = false;
                }
                const float rr = any ? L1.x * s : 0.f, rg = any ? L1.y * s : 0.f, rb = any ? L1.z * s : 0.f;
                if (f_mode == RTX_MODE_RADIANCE) {
                    fr += rr; fg += rg; fb += rb;
                } else {
                    const float oa = smax(nx * lx + ny * ly + nz * lz, 0.f);
                    const RGB br = shade<kKinds>(S, mat, nx, ny, nz, lx, ly, lz, vx, vy, vz, cnt, COUNT);
                    fr += (rr * oa) * br.r; fg += (rg * oa) * br.g; fb += (rb * oa) * br.b;
                }
            } else if (f_mode == RTX_MODE_OBSERVED_AREA) {
                const float oa = smax(nx * lx + ny * ly + nz * lz, 0.f);
                fr += oa; fg += oa; fb += oa;
            } else if (f_mode == RTX_MODE_BRDF) {
                const RGB br = shade<kKinds>(S, mat, nx, ny, nz, lx, ly, lz, vx, vy, vz, cnt, COUNT);
                fr += br.r; fg += br.g; fb += br.b;
            }
        }
        if (did && PHASE != 5) { fr *= shadowFactor; fg *= shadowFactor; fb *= shadowFactor; }
    }
    if (PHASE == 5) {   // the light's occluded lanes for PHASE 6
        if (lane == 0) F.lm_mask[static_cast<size_t>(tile) * F.lm_lights + light] = lm_occ;
        if (F.cost && lane == 0) part_cost_add(F.cost + tile, __builtin_amdgcn_s_memtime() - t_block0);
        return;
    }
    if (PHASE == 2) {
        part_stat<PHASE>(F, part, widx, lane, t_block0);
        RTX_SPLIT_STAMP();
        return;
    }
    if (PHASE == 3) {   // ready for the next frame's split launches
        F.hit_key[slot] = ~0ull;
        F.occ_bits[slot] = 0u;
    }
    // ColorRGB::MaxToOne (ColorRGB.h:12-17)
    const float mv = smax(fr, smax(fg, fb));
    if (mv > 1.f) { fr /= mv; fg /= mv; fb /= mv; }
    if (valid) {
        const size_t o = static_cast<size_t>(view) * F.width * F.height + static_cast<size_t>(py) * F.width +
                         static_cast<size_t>(px);
        F.out_px[o] = (q8(fr) << F.rshift) | (q8(fg) << F.gshift) | (q8(fb) << F.bshift) | F.amask;
        if (F.out_rgb) {
            F.out_rgb[3 * o] = fr; F.out_rgb[3 * o + 1] = fg; F.out_rgb[3 * o + 2] = fb;
        }
    }
    if (PHASE == 0 && F.cost && lane == 0) {   // split tiles keep their one-piece cost
        const unsigned long long dt = (__builtin_amdgcn_s_memtime() - t_block0) >> 4;
        atomicMax(&F.cost[tile], static_cast<uint32_t>(dt < 0xffffffffull ? dt : 0xffffffffull));
    }
    // light-major: the tile's cost is the sum of its waves' (PHASE 4 + every light wave)
    if ((PHASE == 5 || PHASE == 6) && F.cost && lane == 0)
        part_cost_add(F.cost + tile, __builtin_amdgcn_s_memtime() - t_block0);
#if RTX_STAMPS
    if (PHASE == 0 && lane == 0 && F.stamps) {
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        const size_t w = tile;
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        unsigned long long* st = F.stamps + kStampWords * w;
        st[0] = t_start;
        st[1] = t_end;
        st[2] = (static_cast<unsigned long long>(xcc) << 32) | hw;
        st[3] = cnt.c[kWaveNodeTests];
        st[4] = cnt.c[kWaveTriTests];
        st[5] = (static_cast<unsigned long long>(cnt.c[kSlab]) << 32) | cnt.c[kTri];
        st[6] = t_prim - t_start;
        st[7] = t_shadow;
    }
#endif
    if (COUNT) {
        for (int k = 0; k < kNumCounters; ++k)
            if (cnt.c[k]) atomicAdd(&F.counters[k], static_cast<unsigned long long>(cnt.c[k]));
    }
}


template <bool COUNT, int PHASE, bool DEEP = false, int SPEC = 0, bool HSTK = false, bool CULLK = false>
__global__ void __launch_bounds__(kBlockThreads, (DEEP && !HSTK) ? 2
                                                  : ((SPEC & (kSpecOneMesh | kSpecNoMesh))
                                                         ? RTX_SPEC_WAVES
                                                         : (SPEC ? RTX_SPEC_WAVES_PARTIAL : RTX_MIN_WAVES_PER_EU)))
    rtx_render_kernel(const DevScene S, const FrameArgs F) {
    constexpr int kDepth = HSTK ? 1 : (DEEP ? kStackDepthDeep : kStackDepth);
    __shared__ uint4 stkE[kBlockThreads / 64][kDepth];
    __shared__ unsigned long long stkT[(COUNT && !HSTK) ? kBlockThreads / 64 : 1][(COUNT && !HSTK) ? kDepth : 1];
    // per-lane shadow-ray plane numerators, shared by every light (see the light loop)
    __shared__ float pnumS[kBlockThreads / 64][kPlaneCache][64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint4* stk = stkE[wave];
    unsigned long long* sT = stkT[COUNT ? wave : 0];

    // Work unit = one 8x8 wave tile of one view; the waves of a workgroup (one by default,
    // RTX_BLOCK_THREADS) are independent (no barrier) and take consecutive entries of the
    // dispatch order.  The order is a permutation (F.order, null = identity) that
    // rtx_reorder_kernel derives from the previous frame's measured per-tile cost: heavy
    // tiles start first and do not form a tail.  One-wave workgroups free their slot the
    // moment the wave ends (4-wave ones held it until the slowest sibling ended: Bunny
    // -3 %, Synthetic100k -9 %).  Which wave renders a tile never changes a pixel's value.
    const uint32_t b = blockIdx.x;
    uint32_t widx = b * kWavesPerBlock + wave;   // wave index in the launch
    uint32_t tile, part = 0, light = 0;
    // PHASE 4/5: the light-major frame (FrameArgs::lm_*): PHASE 4 = PHASE 0 up to the hit record,
    // PHASE 5 = item (tile, light), the tiles in dispatch order and a tile's lights consecutive
    if (PHASE == 0 || PHASE == 4 || PHASE == 6) {
        if (widx >= F.n_tiles) return;
        tile = F.order ? ldc(F.order, widx) : widx;
        if (F.heavy_flag && ldc(F.heavy_flag, tile)) return;   // rendered by the split launches
    } else if (PHASE == 5) {
        // persistent waves, one per resident wave slot: wave w takes items w, w + NW, w + 2 NW, ... of the
        // cost-ordered list, so every wave gets a share of the heavy items and no per-item workgroup is
        // dispatched (130k one-wave workgroups at 4K / 8 ranks cost more to launch than to run)
        const uint32_t L = F.lm_lights, items = F.n_tiles * L, nw = gridDim.x * kWavesPerBlock;
        for (uint32_t it = uni(widx); it < items; it += nw) {   // (wave-uniform: the light indexes scalar loads)
            const uint32_t k = it / L;
            tile = F.order ? ldc(F.order, k) : k;
            if (F.heavy_flag && ldc(F.heavy_flag, tile)) continue;
            render_tile<COUNT, PHASE, DEEP, SPEC, HSTK, CULLK>(S, F, it, tile, 0u, it - k * L, stk, sT, pnumS[wave],
                                                               lane);
        }
        return;
    } else {
        // grid (heavy tiles / waves per block, parts, lights), tile fastest: every heavy tile's part 0 is
        // dispatched first, the big top-of-tree parts before the small ones.  (Pinning a
        // part to one XCD for L2 locality was measured slower: the heavy parts then load a
        // few XCDs only.)
        if (widx >= F.heavy_n) return;
        part = blockIdx.y;
        light = blockIdx.z;
        tile = ldc(F.heavy_list, widx);
    }
    render_tile<COUNT, PHASE, DEEP, SPEC, HSTK, CULLK>(S, F, widx, tile, part, light, stk, sT, pnumS[wave], lane);
}

#undef f_mode
#undef f_shadows
#undef n_sph
#undef n_pl
#undef n_mesh

template __global__ void rtx_render_kernel<false, 0>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<true, 0>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<false, 1>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<false, 2>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<false, 3>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<false, 0, true>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<true, 0, true>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<false, 0, true, 0, true>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<true, 0, true, 0, true>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<false, 0, false, kSpecVariants[0]>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<false, 0, false, kSpecVariants[1]>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<false, 0, false, kSpecVariants[2]>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<false, 0, false, kSpecVariants[3]>(const DevScene, const FrameArgs);
template __global__ void rtx_render_kernel<false, 0, false, kSpecVariants[4]>(const DevScene, const FrameArgs);
// the exact-cull variants (CULLK): the generic kernel and the mesh variants, all phases
#define RTX_CULL_VARIANTS(P)                                                                                    \
    template __global__ void rtx_render_kernel<false, P, false, 0, false, true>(const DevScene, const FrameArgs); \
    template __global__ void rtx_render_kernel<false, P, false, kSpecVariants[0], false, true>(const DevScene,   \
                                                                                               const FrameArgs); \
    template __global__ void rtx_render_kernel<false, P, false, kSpecVariants[1], false, true>(const DevScene,   \
                                                                                               const FrameArgs); \
    template __global__ void rtx_render_kernel<false, P, false, kSpecVariants[3], false, true>(const DevScene,   \
                                                                                               const FrameArgs); \
    template __global__ void rtx_render_kernel<false, P, false, kSpecVariants[4], false, true>(const DevScene,   \
                                                                                               const FrameArgs);
RTX_CULL_VARIANTS(0)
RTX_CULL_VARIANTS(1)
RTX_CULL_VARIANTS(2)
RTX_CULL_VARIANTS(3)
#undef RTX_CULL_VARIANTS

// Octant copies 1..7 of an uploaded node array from copy 0 (blockIdx.y + 1 = octant k):
// copy k stores (hi, lo) on the axes set in k, the same swap the host applies for small
// arrays (upload_scene).  Zero padding maps to zero padding.  `n2` node records of 32 B per
// copy (padding included), copies `stride` float4 apart.
__global__ void __launch_bounds__(256) rtx_octant_expand(float4* __restrict__ nodes, uint32_t n2, uint32_t stride) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n2) return;
    const uint32_t k = blockIdx.y + 1u;
    const float4 a = nodes[2u * i], b = nodes[2u * i + 1u];
    const bool mx = k & 1u, my = k & 2u, mz = k & 4u;
    float4* dst = nodes + static_cast<size_t>(k) * stride;
    dst[2u * i] = make_float4(mx ? a.y : a.x, mx ? a.x : a.y, my ? a.w : a.z, my ? a.z : a.w);
    dst[2u * i + 1u] = make_float4(mz ? b.y : b.x, mz ? b.x : b.y, b.z, b.w);
}

// ---------------------------------------------------------------- exact cull records
// (rtx_cull.h; DevScene::cull).  Each node slot's record needs, over the node's
// triangle range (contiguous in leaf order: children partition their parent's range), the union
// of the triangles' boxes and, per anchor, the largest margin and dt.  Those range reductions
// run over SEGMENT TREES of the per-triangle values: a perfect binary tree over n = 2^k leaves
// (leaf n + i = triangle i, padding leaves hold the identity; node i = comb(2i, 2i + 1)), so a
// slot's range [x, y) is the combination of at most 2 log2(y - x) tree nodes (cull_tree_query),
// found by one thread in log2(y - x) + 1 dependent steps.  The tree is built in the launch that
// computes the leaves: levels 0-6 across the wave, 7-8 in LDS across the 256-thread workgroup,
// and the levels above by the last workgroup of the tree to arrive (an arrival counter).  Total
// work O(N) for the trees and O(S log N) for S slots; critical path O(log N) — the round-4 kernels
// re-reduced each slot's whole range (the root's wave walked every triangle once per anchor:
// 0.57-1.47 ms for Synthetic100k).  Launches, all on the context stream before the frames:
//   rtx_cull_tris        per triangle: the box of (v0, v0 + E1, v0 + E2), rounded outward (after an
//                        upload), and per (anchor, triangle) rtx_cull.h's (margin, dt); the trees
//   rtx_cull_nodes<BOX>  per node slot: the box (queried after an upload, then kept per context)
//                        widened by the range's largest margin and the kernel test's own padding
//                        -> the anchors' records
// Built before the first frame after an upload (the box, every light's anchor and the frame's
// camera anchors: two launches), then again for a view's camera anchor when a frame's view origin
// is not the one its records were made for.  A NaN, infinite or huge (> 2^40) coordinate anywhere gives +inf (the
// record then always passes: the bound's finite-arithmetic domain, rtx_cull.h).
struct CullAnchors {
    float p[kMaxViews + kMaxCullLights][4];   // xyz: the anchor point; w = 0: camera origin, > 0: light with tmax <= w
    float bt[kMaxViews + kMaxCullLights];     // the t bound of the records' dt (lights: = w)
    uint32_t idx[kMaxViews + kMaxCullLights]; // record copy the anchor writes
    uint32_t n;
};

__device__ __forceinline__ float f_rd(double x) {   // largest float <= x (NaN stays NaN)
    float f = static_cast<float>(x);
    if (static_cast<double>(f) > x) f = nextafterf(f, -INFINITY);
    return f;
}
__device__ __forceinline__ float f_ru(double x) {   // smallest float >= x
    float f = static_cast<float>(x);
    if (static_cast<double>(f) < x) f = nextafterf(f, INFINITY);
    return f;
}
__device__ __forceinline__ bool cull_domain(float x) { return fabsf(x) <= 0x1p40f; }   // false for NaN / inf

// The two kinds of tree values.  Margins and dt are >= 0 or +inf (never NaN: the margin kernel
// maps NaN to +inf), so their identity is 0; box bounds never hold a NaN either (an out-of-domain
// triangle's box is (-inf, +inf)), so min / max are exact folds in any order (only the sign of a
// zero bound can depend on the order, and no record test observes it).
// (CullMD, CullBox: rtx_ctx.h)
__device__ __forceinline__ CullMD cull_ident(CullMD*) { return {0.f, 0.f}; }
__device__ __forceinline__ CullBox cull_ident(CullBox*) {
    return {{INFINITY, INFINITY, INFINITY}, 0.f, {-INFINITY, -INFINITY, -INFINITY}, 0.f};
}
__device__ __forceinline__ CullMD cull_comb(const CullMD& a, const CullMD& b) { return {fmaxf(a.m, b.m), fmaxf(a.dt, b.dt)}; }
__device__ __forceinline__ CullBox cull_comb(const CullBox& a, const CullBox& b) {
    CullBox r;
    for (int k = 0; k < 3; ++k) { r.lo[k] = fminf(a.lo[k], b.lo[k]); r.hi[k] = fmaxf(a.hi[k], b.hi[k]); }
    r.pad0 = r.pad1 = 0.f;
    return r;
}
__device__ __forceinline__ CullMD cull_xor(const CullMD& a, int o) { return {__shfl_xor(a.m, o, 64), __shfl_xor(a.dt, o, 64)}; }
__device__ __forceinline__ CullBox cull_xor(const CullBox& a, int o) {
    CullBox r;
    for (int k = 0; k < 3; ++k) { r.lo[k] = __shfl_xor(a.lo[k], o, 64); r.hi[k] = __shfl_xor(a.hi[k], o, 64); }
    r.pad0 = r.pad1 = 0.f;
    return r;
}

// Write-through (sc1) 8-byte stores and loads of tree values: the workgroup roots are handed to
// the last workgroup INSIDE the launch, across XCDs whose L2s are not coherent.  A plain store
// stays in the writer's L2 (a release fence writes it back, but the reader's L2 may still hold an
// older copy of the line: an acquire invalidates only L1), so the roots are stored write-through
// by the one lane that then adds to the arrival counter after its stores drained, and the last
// workgroup reads them write-through too (MI355X_MICROARCH.md, inter-workgroup visibility: the
// "one lane per storing workgroup, last arriver by the add's value" form).
template <class V>
__device__ __forceinline__ void cull_st_wt(V* p, const V& v) {
    static_assert(sizeof(V) % 8 == 0, "8-byte pieces");
    unsigned long long w[sizeof(V) / 8];
    __builtin_memcpy(w, &v, sizeof(V));
    for (size_t k = 0; k < sizeof(V) / 8; ++k)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(p) + k, w[k], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
template <class V>
__device__ __forceinline__ V cull_ld_wt(const V* p) {
    unsigned long long w[sizeof(V) / 8];
    for (size_t k = 0; k < sizeof(V) / 8; ++k)
        w[k] = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p) + k, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    V v;
    __builtin_memcpy(&v, w, sizeof(V));
    return v;
}

// Leaf i = blockIdx.x * kCullTreeWG + threadIdx.x holds v; writes the tree levels of `t` (2n
// entries, n = gridDim.x * kCullTreeWG).  `arrive`: the tree's arrival counter (0 before the
// launch, 0 again after it); `top_lds` (<= kCullTopLds): the most workgroup roots the last
// workgroup combines in LDS (tests lower it to exercise the global-memory path).  Levels below
// the workgroup roots are read only by later launches (plain stores).
template <class V>
__device__ void cull_tree_build(V v, V* __restrict__ t, uint32_t* arrive, uint32_t top_lds) {
    __shared__ V part[kCullTreeWG / 64];
    __shared__ V top[kCullTopLds / 2];
    __shared__ uint32_t last;
    const uint32_t tid = threadIdx.x, nwg = gridDim.x, n = nwg * kCullTreeWG;
    const uint32_t leaf = n + blockIdx.x * kCullTreeWG + tid;
    t[leaf] = v;
    for (int k = 1; k <= 6; ++k) {   // levels 1-6: butterflies over aligned 2^k lanes
        v = cull_comb(v, cull_xor(v, 1 << (k - 1)));
        if ((tid & ((1u << k) - 1u)) == 0u) t[leaf >> k] = v;
    }
    if ((tid & 63u) == 0u) part[tid >> 6] = v;
    __syncthreads();
    if (tid == 0) {   // levels 7 and 8 (kCullTreeWG = 256 = 4 waves); the root write-through
        const V a = cull_comb(part[0], part[1]), b = cull_comb(part[2], part[3]), r = cull_comb(a, b);
        t[leaf >> 7] = a;
        t[(leaf >> 7) + 1u] = b;
        cull_st_wt(t + (leaf >> 8), r);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the root has left before the arrival
        last = atomicAdd(arrive, 1u) == nwg - 1u ? 1u : 0u;
    }
    __syncthreads();
    if (!last) return;
    // levels above 8: the workgroup roots are nodes [nwg, 2 nwg); node j of a level = comb(2j, 2j + 1)
    if (nwg == 1u) {
        // the workgroup's root is the tree's
    } else if (nwg <= top_lds) {
        for (uint32_t w = tid; w < nwg / 2u; w += kCullTreeWG)
            top[w] = cull_comb(cull_ld_wt(t + nwg + 2u * w), cull_ld_wt(t + nwg + 2u * w + 1u));
        for (uint32_t c = nwg / 2u;; c >>= 1) {   // `top` holds level-nodes [c, 2c)
            __syncthreads();
            for (uint32_t w = tid; w < c; w += kCullTreeWG) t[c + w] = top[w];
            if (c == 1u) break;
            V r[kCullTopLds / 2 / kCullTreeWG];
            uint32_t q = 0;
            for (uint32_t w = tid; w < c / 2u; w += kCullTreeWG) r[q++] = cull_comb(top[2u * w], top[2u * w + 1u]);
            __syncthreads();
            q = 0;
            for (uint32_t w = tid; w < c / 2u; w += kCullTreeWG) top[w] = r[q++];
        }
    } else {   // level by level through memory, every access write-through (this workgroup's own
               // stores are read back by its other waves: past their L1s)
        for (uint32_t c = nwg / 2u; c >= 1u; c >>= 1) {
            for (uint32_t w = tid; w < c; w += kCullTreeWG)
                cull_st_wt(t + c + w, cull_comb(cull_ld_wt(t + 2u * (c + w)), cull_ld_wt(t + 2u * (c + w) + 1u)));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    }
    if (tid == 0) __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
}

// the combination of the leaves [x, y) (x <= y <= n)
template <class V>
__device__ __forceinline__ V cull_tree_query(const V* __restrict__ t, uint32_t n, uint32_t x, uint32_t y) {
    V acc = cull_ident(static_cast<V*>(nullptr));
    for (uint32_t l = x + n, r = y + n; l < r; l >>= 1, r >>= 1) {
        if (l & 1u) acc = cull_comb(acc, t[l++]);
        if (r & 1u) acc = cull_comb(acc, t[--r]);
    }
    return acc;
}

// grid (n / kCullTreeWG, A.n + box): blockIdx.y = j < A.n builds anchor j's (margin, dt) tree at
// trees + 2n j (counter arrive[j]); j = A.n (when `box`) the box tree (counter arrive[kCullMaxAnchors]).
__global__ void __launch_bounds__(kCullTreeWG) rtx_cull_tris(const Tri* __restrict__ tris, uint32_t nt,
                                                             const CullAnchors A, CullMD* __restrict__ trees,
                                                             CullBox* __restrict__ btree, uint32_t* arrive,
                                                             uint32_t top_lds) {
    const uint32_t i = blockIdx.x * kCullTreeWG + threadIdx.x, j = blockIdx.y;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, c = a;
    if (i < nt) { a = tris[i].a; b = tris[i].b; c = tris[i].c; }
    const float v0[3] = {a.x, a.y, a.z}, e1[3] = {b.x, b.y, b.z}, e2[3] = {c.x, c.y, c.z};
    if (j == A.n) {   // the per-triangle box of (v0, v0 + E1, v0 + E2), rounded outward
        CullBox v = cull_ident(static_cast<CullBox*>(nullptr));
        if (i < nt) {
            bool ok = true;
            for (int k = 0; k < 3; ++k) {
                ok = ok && cull_domain(v0[k]) && cull_domain(e1[k]) && cull_domain(e2[k]);
                const double p = v0[k], q = p + static_cast<double>(e1[k]), r = p + static_cast<double>(e2[k]);
                const double mn = fmin(p, fmin(q, r)), mx = fmax(p, fmax(q, r));
                // the double sums are exact unless the exponents differ by > 29: widen by 2^-40 anyway
                v.lo[k] = f_rd(mn - fabs(mn) * 0x1p-40);
                v.hi[k] = f_ru(mx + fabs(mx) * 0x1p-40);
            }
            if (!ok)   // out of the domain: every box holding it passes every ray
                for (int k = 0; k < 3; ++k) { v.lo[k] = -INFINITY; v.hi[k] = INFINITY; }
        }
        cull_tree_build(v, btree, arrive + kCullMaxAnchors, top_lds);
        return;
    }
    CullMD v{0.f, 0.f};
    if (i < nt) {   // anchor j's bound for triangle i (rtx_cull.h), NaN -> inf
        rtx_cull_tri T;
        rtx_cull_tri_setup(&T, v0, e1, e2);
        const float* p = A.p[j];
        const rtx_cull_bound bd = p[3] > 0.f ? rtx_cull_light_bounds(&T, p, p[3]) : rtx_cull_point_bounds(&T, p, A.bt[j]);
        v.m = (bd.margin >= 0.0 && bd.margin < 0x1p100) ? f_ru(bd.margin) : INFINITY;
        v.dt = (bd.dt >= 0.0 && bd.dt < 0x1p100) ? f_ru(bd.dt) : INFINITY;
    }
    cull_tree_build(v, trees + 2ull * gridDim.x * kCullTreeWG * j, arrive + j, top_lds);
}

// Which records the walk tests (CullParams): a box some axis of which the reference's box (node
// copy 0) exceeds `ratio` times — the reference's FLT_MIN-inflated boxes, DataTypes.h:315 — and,
// with `leaves`, only leaf nodes.  Unflagged records are loaded but cost no vector work.
struct CullParams {
    const float4* nodes;   // node copy 0 (reference boxes, {min.x, max.x, min.y, max.y}, {min.z, max.z, link, ntri})
    float ratio;
    uint32_t leaves;
};
// the record of `slot` for anchor copy `a`: tight box [lo, hi] widened by `m` and the padding
// 16u (E + |c|) of cull_mask's rounding (2^-20 = 16u); w of its second half = the test flag
__device__ __forceinline__ void cull_write(float4* __restrict__ cull, uint32_t stride4, uint32_t a, uint32_t slot,
                                           const float* lo, const float* hi, bool bad, float m, float dt,
                                           const CullParams& P) {
    float cf[3], Ef[3];
    for (int k = 0; k < 3; ++k) {
        const double c = 0.5 * (static_cast<double>(lo[k]) + hi[k]);
        cf[k] = static_cast<float>(c);
        double E = 0.5 * (static_cast<double>(hi[k]) - lo[k]) + fabs(c - cf[k]) + static_cast<double>(m);
        E = (E + 0x1p-20 * (E + fabs(static_cast<double>(cf[k])))) * (1.0 + 0x1p-40) +
            0x1p-50 * (fabs(static_cast<double>(lo[k])) + fabs(static_cast<double>(hi[k])));
        Ef[k] = (!bad && E < 0x1p100) ? f_ru(E) : INFINITY;   // NaN and empty boxes pass every ray
        if (bad || !(E < 0x1p100)) cf[k] = 0.f;
    }
    const float4 n0 = P.nodes[2u * slot], n1 = P.nodes[2u * slot + 1u];
    const float ref[3] = {n0.y - n0.x, n0.w - n0.z, n1.y - n1.x};
    bool worth = false;
    for (int k = 0; k < 3; ++k) worth = worth || ref[k] > P.ratio * 2.f * Ef[k];   // false for inf / NaN
    if (P.leaves && __float_as_uint(n1.w) == 0u) worth = false;
    float4* r = cull + static_cast<size_t>(a) * stride4 + 2u * slot;
    r[0] = make_float4(cf[0], cf[1], cf[2], Ef[0]);
    r[1] = make_float4(Ef[1], Ef[2], (bad || !(dt < 0x1p100f)) ? INFINITY : dt, __uint_as_float(worth ? 1u : 0u));
}

// One thread per node slot.  BOX (after an upload): the slot's box from the box tree, kept in `nbox`
// for the camera anchors' later launches; else read from `nbox`.  An empty range (padding slot)
// or a box with an infinite bound (an out-of-domain triangle below) gives the always-pass record.
// (Reducing the box and several anchors' trees in one walk up the levels, their loads issued
// together, measured slower: Synthetic100k camera records 11.2 -> 34.8 us, profiles/r05.)
template <bool BOX>
__global__ void __launch_bounds__(256) rtx_cull_nodes(const uint2* __restrict__ rng, uint32_t nslots, uint32_t ntris,
                                                      uint32_t n, const CullBox* __restrict__ btree,
                                                      CullBox* __restrict__ nbox, const CullMD* __restrict__ trees,
                                                      const CullAnchors A, float4* __restrict__ cull, uint32_t stride4,
                                                      const CullParams P) {
    const uint32_t s = blockIdx.x * 256u + threadIdx.x;
    if (s >= nslots) return;
    const uint2 r = rng[s];
    const bool empty = r.y <= r.x || r.y > ntris;
    CullBox b;
    if (BOX) {
        b = empty ? cull_ident(static_cast<CullBox*>(nullptr)) : cull_tree_query(btree, n, r.x, r.y);
        nbox[s] = b;
    } else {
        b = nbox[s];
    }
    bool bad = empty;
    for (int k = 0; k < 3; ++k) bad = bad || !(fabsf(b.lo[k]) < INFINITY) || !(fabsf(b.hi[k]) < INFINITY);
    for (uint32_t j = 0; j < A.n; ++j) {
        const CullMD md = bad ? CullMD{0.f, 0.f} : cull_tree_query(trees + 2ull * n * j, n, r.x, r.y);
        cull_write(cull, stride4, A.idx[j], s, b.lo, b.hi, bad, md.m, md.dt, P);
    }
}

// Next frames' dispatch order from this frame's per-tile cost: heaviest first, STABLE
// within a cost class so that tiles rendered together stay spatial neighbours (they walk
// the same BVH nodes: scalar-cache locality).  The order is (class, tile index): the same
// permutation a serial counting sort would give, computed by three launches over chunks of
// kSchedChunk tiles (one 256-thread workgroup each):
//   rtx_sched_count    per chunk: class histogram + cost sum (and the saved-cost fix-up)
//   rtx_sched_scan     one workgroup: exclusive prefix of the histograms in (class, chunk)
//                      order, the heavy threshold
//   rtx_sched_scatter  per chunk: every tile's slot = its (class, chunk) base + its rank
//                      among the chunk's tiles of that class; heavy flags / list; clears costs
// It also picks the heavy tiles for split rendering: cost > split_permille/1000 x (total cost /
// min(tiles, concurrent workgroup slots)), i.e. a tile that alone would outlast its share of
// the frame.  `split_slots` = 0 disables splitting, UINT32_MAX forces every tile heavy
// (tests).  Flags and list go to the staging set the host adopts at its next frame.
__device__ __forceinline__ uint32_t cost_class(uint32_t cst) {   // heavier -> smaller class
    const uint32_t lg = cst ? 32u - static_cast<uint32_t>(__builtin_clz(cst)) : 0u;   // 0..32
    const uint32_t half = (cst && lg >= 2) ? ((cst >> (lg - 2)) & 1u) : 0u;
    uint32_t k = 2u * lg + half;                                                     // 0..65
    k = k > 2u * 6u ? k - 2u * 6u : 0u;        // costs below 2^6 (x16 cycles) share a class
    return (kCostBuckets - 1) - (k < kCostBuckets ? k : kCostBuckets - 1);
}

// A tile rendered split this frame has no fresh one-piece cost: it keeps the one it had
// when it was last rendered whole (kept in `saved`) — or, with `parts` (motion mode: the camera
// moves, so that cost goes stale), the sum of its split waves' durations for this frame's sort,
// which lets a tile that stopped being heavy leave the split set (`saved` is left as it was).
__global__ void __launch_bounds__(kReorderThreads) rtx_sched_count(uint32_t* __restrict__ cost, uint32_t n,
                                                                   const uint32_t* __restrict__ was_heavy,
                                                                   uint32_t* __restrict__ saved,
                                                                   uint32_t* __restrict__ hist,
                                                                   unsigned long long* __restrict__ csum,
                                                                   uint32_t nchunks, uint32_t parts,
                                                                   uint32_t* __restrict__ max_cost) {
    __shared__ uint32_t h[kCostBuckets];
    __shared__ unsigned long long tot;
    __shared__ uint32_t mx;
    const uint32_t tid = threadIdx.x, base = blockIdx.x * kSchedChunk;
    if (tid < kCostBuckets) h[tid] = 0;
    if (tid == 0) {
        tot = 0;
        mx = 0;
    }
    __syncthreads();
    unsigned long long my = 0;
    uint32_t my_max = 0;
    for (uint32_t k = 0; k < kSchedChunk / kReorderThreads; ++k) {
        const uint32_t t = base + k * kReorderThreads + tid;   // coalesced; counting ignores order
        if (t >= n) break;
        uint32_t c = cost[t];
        if (was_heavy && was_heavy[t]) {
            // split this frame: static frames sort it by the one-piece cost it had when last
            // rendered whole; motion mode by its part waves' sum (cost[t]), which stands in for this
            // frame only — the saved one-piece cost stays (a part sum leaves out each part wave's
            // fixed work, so it would cost the tile low once motion ends)
            if (!parts) {
                c = saved[t];
                cost[t] = c;
            }
        } else {
            saved[t] = c;
        }
        atomicAdd(&h[cost_class(c)], 1u);
        my += c;
        my_max = c > my_max ? c : my_max;
    }
    atomicAdd(&tot, my);
    atomicMax(&mx, my_max);
    __syncthreads();
    if (tid < kCostBuckets) hist[tid * nchunks + blockIdx.x] = h[tid];
    if (tid == 0) {
        csum[blockIdx.x] = tot;
        atomicMax(max_cost, mx);
    }
}

// Exclusive prefix of hist[class][chunk] in class-major order (in place), the total cost and
// the heavy threshold; zeroes the heavy counter the scatter appends to.
__global__ void __launch_bounds__(kScanThreads) rtx_sched_scan(uint32_t* __restrict__ hist, uint32_t nchunks,
                                                               const unsigned long long* __restrict__ csum, uint32_t n,
                                                               uint32_t split_slots, uint32_t split_permille,
                                                               uint32_t split_min, uint32_t wave_slots,
                                                               unsigned long long* __restrict__ thr_out,
                                                               uint32_t* __restrict__ heavy_n) {
    __shared__ uint32_t part[kScanThreads];
    __shared__ unsigned long long cpart[kScanThreads];
    const uint32_t tid = threadIdx.x;
    const uint32_t len = kCostBuckets * nchunks;
    const uint32_t per = (len + kScanThreads - 1) / kScanThreads;
    const uint32_t lo = tid * per, hi = (lo + per < len) ? lo + per : len;
    uint32_t s = 0;
    for (uint32_t i = lo; i < hi; ++i) s += hist[i];
    unsigned long long cs = 0;
    for (uint32_t i = tid; i < nchunks; i += kScanThreads) cs += csum[i];
    part[tid] = s;
    cpart[tid] = cs;
    __syncthreads();
    for (uint32_t o = 1; o < kScanThreads; o <<= 1) {   // inclusive Hillis-Steele scan
        const uint32_t v = tid >= o ? part[tid - o] : 0u;
        const unsigned long long w = tid >= o ? cpart[tid - o] : 0ull;
        __syncthreads();
        part[tid] += v;
        cpart[tid] += w;
        __syncthreads();
    }
    uint32_t acc = part[tid] - s;   // exclusive
    for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t v = hist[i];
        hist[i] = acc;
        acc += v;
    }
    if (tid == 0) {
        const unsigned long long total = cpart[kScanThreads - 1];
        const bool force = split_slots == 0xffffffffu;
        // (split_min: no tile below it is split, whatever its share of the frame)
        const unsigned long long thr =
            split_slots ? total * split_permille / (1000ull * (n < split_slots ? n : split_slots)) : ~0ull;
        *thr_out = force ? 0ull : (thr > split_min ? thr : static_cast<unsigned long long>(split_min));
        heavy_n[0] = 0;
        // the frame's heaviest tile (rtx_sched_count's maximum, zeroed for the next measurement) and
        // its cost per wave slot, for the in-flight choice (kInflightCritPermille)
        heavy_n[2] = heavy_n[1];
        heavy_n[1] = 0;
        const unsigned long long per = wave_slots ? total / (n < wave_slots ? n : wave_slots) : 0ull;
        heavy_n[3] = static_cast<uint32_t>(per < 0xffffffffull ? per : 0xffffffffull);
    }
}

__global__ void __launch_bounds__(kReorderThreads) rtx_sched_scatter(uint32_t* __restrict__ cost,
                                                                     uint32_t* __restrict__ order, uint32_t n,
                                                                     const uint32_t* __restrict__ hist,
                                                                     uint32_t nchunks,
                                                                     const unsigned long long* __restrict__ thr_in,
                                                                     uint32_t force, uint32_t* __restrict__ heavy_flag,
                                                                     uint32_t* __restrict__ heavy_list,
                                                                     uint32_t* __restrict__ heavy_n) {
    constexpr uint32_t kPer = kSchedChunk / kReorderThreads;   // consecutive tiles per thread
    constexpr uint32_t kSeg = kCostBuckets;   // (class, thread) entries scanned per thread: 32 x 256 / 256
    __shared__ uint32_t cnt[kCostBuckets][kReorderThreads];
    __shared__ uint32_t tsum[kReorderThreads];
    const uint32_t tid = threadIdx.x, base = blockIdx.x * kSchedChunk + tid * kPer;
    uint32_t cls[kPer], cst[kPer];
    for (uint32_t k = 0; k < kCostBuckets; ++k) cnt[k][tid] = 0;
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t t = base + k;
        cst[k] = t < n ? cost[t] : 0u;
        cls[k] = cost_class(cst[k]);
        if (t < n) cnt[cls[k]][tid]++;
    }
    __syncthreads();
    // exclusive scan of cnt flattened in (class, thread) order: thread j scans kSeg
    // consecutive entries, then the per-thread sums are scanned
    uint32_t* flat = &cnt[0][0];
    uint32_t s = 0;
    for (uint32_t i = 0; i < kSeg; ++i) s += flat[tid * kSeg + i];
    tsum[tid] = s;
    __syncthreads();
    for (uint32_t off = 1; off < kReorderThreads; off <<= 1) {
        const uint32_t v = tid >= off ? tsum[tid - off] : 0u;
        __syncthreads();
        tsum[tid] += v;
        __syncthreads();
    }
    uint32_t acc = tsum[tid] - s;
    for (uint32_t i = 0; i < kSeg; ++i) {
        const uint32_t v = flat[tid * kSeg + i];
        flat[tid * kSeg + i] = acc;
        acc += v;
    }
    __syncthreads();
    // slot = global (class, chunk) base + rank within the chunk's class (= flattened prefix
    // minus the prefix at the class's first thread) + rank within the thread
    const unsigned long long thr = *thr_in;
    uint32_t seen[kPer];
    for (uint32_t k = 0; k < kPer; ++k) {
        seen[k] = 0;
        for (uint32_t j = 0; j < k; ++j) seen[k] += cls[j] == cls[k];
    }
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t t = base + k;
        if (t >= n) break;
        const uint32_t c = cls[k];
        order[hist[c * nchunks + blockIdx.x] + (cnt[c][tid] - cnt[c][0]) + seen[k]] = t;
        uint32_t f = 0;
        if (force || cst[k] > thr) {
            const uint32_t h = atomicAdd(heavy_n, 1u);
            if (h < static_cast<uint32_t>(kMaxHeavyTiles)) { heavy_list[h] = t; f = 1; }
        }
        heavy_flag[t] = f;
        cost[t] = 0;
    }
}

// XCD-affine dispatch (RTX_XCD_ORDER=1, rtx_ctx::xcd_order): workgroups are dealt round robin over the 8
// XCDs (MI355X_MICROARCH.md, workgroup dispatch), so positions p and p + 8 of the dispatch order run on
// one XCD.  This pass re-deals the cost order so that position 8k + r holds the k-th tile, in cost order,
// of class r (each view cut into 8 x 8 blocks, block (i, j) in class (i + 3 j) mod 8): each XCD's L2 then
// serves eight blocks' BVH nodes, triangles and cull records instead of the whole screen's.  (One
// compact region per class, a 4 x 2 grid, measured 1.4-2x slower: the in-order round-robin dispatch
// then waits on the XCD of the heaviest region, profiles/r06/xcd_ab.txt.)  Regions hold unequal
// counts; once the smallest is exhausted the remaining tiles follow in cost order.  One workgroup, three
// passes over each thread's consecutive positions (counts, ranks, writes); a permutation, so no pixel
// changes.
#ifndef RTX_XCD_BLOCKS
#define RTX_XCD_BLOCKS 8   // the view cut into B x B blocks, dealt to the 8 classes as a Latin square
#endif
__device__ __forceinline__ uint32_t xcd_region(uint32_t tile, uint32_t tiles_x, uint32_t tiles_y) {
    const uint32_t per_view = tiles_x * tiles_y;
    const uint32_t rem = tile % per_view, bx = rem % tiles_x, gy = rem / tiles_x;
    const uint32_t i = bx * RTX_XCD_BLOCKS / tiles_x, j = gy * RTX_XCD_BLOCKS / tiles_y;
    // every row and column of blocks holds each class (RTX_XCD_BLOCKS = 8) or each class equally often:
    // a compact heavy area (the Bunny, the heightfield's grazing band) spreads over the classes
    return (i + 3u * j) % 8u;
}
__global__ void __launch_bounds__(kScanThreads) rtx_sched_xcd(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                              uint32_t n, uint32_t tiles_x, uint32_t tiles_y) {
    __shared__ uint32_t cnt[8][kScanThreads];
    __shared__ uint32_t ovf[kScanThreads];
    __shared__ uint32_t tot[8];
    const uint32_t tid = threadIdx.x;
    const uint32_t per = (n + kScanThreads - 1) / kScanThreads;
    const uint32_t lo = tid * per < n ? tid * per : n, hi = lo + per < n ? lo + per : n;
    uint32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t p = lo; p < hi; ++p) ++c[xcd_region(in[p], tiles_x, tiles_y)];
    for (int r = 0; r < 8; ++r) cnt[r][tid] = c[r];
    __syncthreads();
    if (tid < 8) {   // exclusive scan of region tid's counts over the threads
        uint32_t acc = 0;
        for (uint32_t t = 0; t < kScanThreads; ++t) {
            const uint32_t v = cnt[tid][t];
            cnt[tid][t] = acc;
            acc += v;
        }
        tot[tid] = acc;
    }
    __syncthreads();
    uint32_t m = tot[0];
    for (int r = 1; r < 8; ++r) m = tot[r] < m ? tot[r] : m;
    uint32_t k[8], o = 0;
    for (int r = 0; r < 8; ++r) k[r] = cnt[r][tid];
    for (uint32_t p = lo; p < hi; ++p) o += k[xcd_region(in[p], tiles_x, tiles_y)]++ >= m ? 1u : 0u;
    ovf[tid] = o;
    __syncthreads();
    if (tid == 0) {   // exclusive scan of the overflow counts
        uint32_t acc = 0;
        for (uint32_t t = 0; t < kScanThreads; ++t) {
            const uint32_t v = ovf[t];
            ovf[t] = acc;
            acc += v;
        }
    }
    __syncthreads();
    for (int r = 0; r < 8; ++r) k[r] = cnt[r][tid];
    o = ovf[tid];
    for (uint32_t p = lo; p < hi; ++p) {
        const uint32_t t = in[p], r = xcd_region(t, tiles_x, tiles_y), kr = k[r]++;
        out[kr < m ? 8u * kr + r : 8u * m + o++] = t;
    }
}

// ====================================================================== host side
// (the context, rtx_ctx, and the frame policies — split tuner, throughput and in-flight choice,
// frontier refinement, deferred join — live in rtx_ctx.h / rtx_policy.hip)

namespace {


inline float4 f4(float x, float y, float z, float w) { return make_float4(x, y, z, w); }
inline float bits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline float bitsi(int32_t i) { float f; std::memcpy(&f, &i, 4); return f; }
inline int32_t bitsi_f(float f) { int32_t i; std::memcpy(&i, &f, 4); return i; }
inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Per device node slot of one mesh's re-laid-out tree, slots [r0, r1): the range of device
// triangles under it (children's slots follow their parent's, so one backward sweep).  `contig`:
// every subtree's leaves hold consecutive triangles in left-then-right order (build_parts'
// condition); `ordered`: every left child's range ends at or before its sibling's starts (the
// ordered walk's, DevScene::cull).  One sweep serves both (an animated loop uploads every frame).
void slot_ranges(const std::vector<float4>& nodes, uint32_t r0, uint32_t r1, std::vector<uint2>& rng, bool& contig,
                 bool& ordered) {
    if (rng.size() < r1) rng.resize(r1, make_uint2(0u, 0u));
    contig = ordered = true;
    for (uint32_t sl = r1; sl-- > r0;) {
        uint32_t link, cnt;
        std::memcpy(&link, &nodes[2 * sl + 1].z, 4);
        std::memcpy(&cnt, &nodes[2 * sl + 1].w, 4);
        if (cnt) {
            rng[sl] = make_uint2(link, link + cnt);
        } else {
            const uint2 l = rng[link], r = rng[link + 1];
            contig = contig && l.y == r.x;
            ordered = ordered && l.y <= r.x;
            rng[sl] = make_uint2(std::min(l.x, r.x), std::max(l.y, r.y));
        }
    }
}

// Frontier of one re-laid-out mesh BVH for split rendering: start from the root and split
// the part with the most triangles until kPartsPerMesh parts (or only leaves) remain.
// Returns false when the tree's left-then-right DFS does not visit the triangles in
// increasing index order (`contig`, slot_ranges) — the property that makes the min-key merge of
// the parts equal to the reference's first-found closest hit — so the scene is rendered unsplit.
bool build_parts(const std::vector<float4>& nodes, uint32_t root, uint32_t mesh, uint32_t target,
                 const std::vector<uint2>& rng, bool contig, std::vector<int4>& parts) {
    if (!contig) return false;
    auto link = [&](uint32_t n) { uint32_t u; std::memcpy(&u, &nodes[2 * n + 1].z, 4); return u; };
    auto ntri = [&](uint32_t n) { uint32_t u; std::memcpy(&u, &nodes[2 * n + 1].w, 4); return u; };
    auto sub = [&](uint32_t n) { return rng[n].y - rng[n].x; };   // triangles under slot n
    struct P { uint32_t node, path, depth; };
    std::vector<P> fr{{root, 0u, 0u}};
    while (fr.size() < target) {
        int best = -1;
        for (size_t k = 0; k < fr.size(); ++k)
            if (!ntri(fr[k].node) && fr[k].depth < 31 && (best < 0 || sub(fr[k].node) > sub(fr[best].node)))
                best = static_cast<int>(k);
        if (best < 0) break;
        const P e = fr[best];
        fr[best] = {link(e.node), e.path, e.depth + 1};
        fr.insert(fr.begin() + best + 1, P{link(e.node) + 1, e.path | (1u << e.depth), e.depth + 1});
    }
    if (const char* ev = std::getenv("RTX_PART_REFINE")) {   // experiment: split the listed parts once more
        std::vector<int> idx;
        for (const char* q = ev; *q;) {
            char* end = nullptr;
            const long v = std::strtol(q, &end, 10);
            if (end == q) break;
            idx.push_back(static_cast<int>(v));
            q = *end ? end + 1 : end;
        }
        std::sort(idx.begin(), idx.end(), std::greater<int>());
        for (int k : idx) {
            if (k < 0 || k >= static_cast<int>(fr.size())) continue;
            const P e = fr[k];
            if (ntri(e.node) || e.depth >= 31) continue;
            fr[k] = {link(e.node), e.path, e.depth + 1};
            fr.insert(fr.begin() + k + 1, P{link(e.node) + 1, e.path | (1u << e.depth), e.depth + 1});
        }
    }
    for (const P& e : fr)
        parts.push_back(make_int4(static_cast<int>(mesh), static_cast<int>(e.node), static_cast<int>(e.path),
                                  static_cast<int>(e.depth)));
    return true;
}

}  // namespace

extern "C" int rtx_abi_version(void) { return RTX_ABI_VERSION; }

namespace {
// Reason for the last failed rtx_create on this thread (rtx_last_error(NULL)).
thread_local std::string g_create_err;

}  // namespace

extern "C" int rtx_create(rtx_ctx** out, int device_id) {
    if (!out) return RTX_E_INVALID;
    *out = nullptr;
    g_create_err.clear();
    rtx_ctx* c = new (std::nothrow) rtx_ctx;
    if (!c) return RTX_E_NOMEM;
    int n = 0;
    const hipError_t ce = hipGetDeviceCount(&n);
    if (ce != hipSuccess || n == 0) {
        g_create_err = std::string("hipGetDeviceCount: ") + (ce != hipSuccess ? hipGetErrorString(ce) : "no device");
        delete c;
        return RTX_E_DEVICE;
    }
    if (device_id < 0 || device_id >= n) {
        g_create_err = "device id out of range";
        delete c;
        return RTX_E_INVALID;
    }
    c->device = device_id;
    // RTX_TILE_ORDER=0 disables cost-ordered tile dispatch (identity order every frame)
    if (const char* e = std::getenv("RTX_TILE_ORDER")) c->sched_enabled = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("RTX_MOTION")) c->motion_off = std::strcmp(e, "0") == 0;
    if (const char* e = std::getenv("RTX_XCD_ORDER")) c->xcd_order = std::strcmp(e, "1") == 0;
    if (const char* e = std::getenv("RTX_THROUGHPUT")) c->throughput_off = std::strcmp(e, "0") == 0;
    if (const char* e = std::getenv("RTX_REFINE")) c->refine_off = std::strcmp(e, "0") == 0;
    if (const char* e = std::getenv("RTX_DEFER_JOIN")) c->join_off = std::strcmp(e, "0") == 0;
    if (const char* e = std::getenv("RTX_DEFER_INFLIGHT")) c->defer_inflight = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("RTX_REFINE_ROUNDS")) c->refine_rounds = static_cast<uint32_t>(std::atoi(e));
    if (const char* e = std::getenv("RTX_REFINE_SPLITS")) c->refine_splits = static_cast<uint32_t>(std::atoi(e));
    if (const char* e = std::getenv("RTX_REFINE_TOP")) c->refine_top = static_cast<uint32_t>(std::atoi(e));
    if (const char* e = std::getenv("RTX_INFLIGHT_CRIT")) {
        const double f = std::atof(e);
        if (f >= 0 && f < 1e6) c->inflight_crit = static_cast<uint32_t>(f * 1000.0);
    }
    if (const char* e = std::getenv("RTX_SCHED_PERIOD"))
        c->sched_period = std::max<uint32_t>(1u, static_cast<uint32_t>(std::strtoul(e, nullptr, 10)));
    // RTX_SPLIT=0 renders heavy tiles in one piece; RTX_SPLIT=force splits every tile
    if (const char* e = std::getenv("RTX_NO_SPEC")) c->no_spec = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("RTX_NO_CULL")) c->no_cull = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("RTX_CULL_RATIO")) {
        const double v = std::atof(e);
        if (v >= 0.0 && v < 1e30) c->cull_ratio = static_cast<float>(v);
    }
    if (const char* e = std::getenv("RTX_CULL_LEAVES")) c->cull_leaves = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("RTX_CULL_ANIMATED")) c->cull_animated = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("RTX_CULL_FAIL")) c->cull_fail_at = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
    if (const char* e = std::getenv("RTX_CULL_TOP_LDS"))
        c->cull_top_lds = std::min<uint32_t>(kCullTopLds, static_cast<uint32_t>(std::strtoul(e, nullptr, 10)));
    if (const char* e = std::getenv("RTX_CULL_MIN_SA")) {
        const double v = std::atof(e);
        if (v >= 0.0 && v < 1e30) c->cull_min_sa = v;
    }
    if (const char* e = std::getenv("RTX_LIGHT_MAJOR"))
        c->lm_mode = std::strcmp(e, "1") == 0 ? 2u : (std::strcmp(e, "auto") == 0 ? 1u : 0u);
    if (const char* e = std::getenv("RTX_LIGHT_MAJOR_TILES")) c->lm_tiles = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
    if (const char* e = std::getenv("RTX_SPLIT")) c->split_mode = std::strcmp(e, "0") == 0 ? 0u : (std::strcmp(e, "force") == 0 ? 2u : 1u);
    if (const char* e = std::getenv("RTX_SPLIT_PARTS")) {
        const int v = std::atoi(e);
        if (v >= 1 && v <= kMaxParts) c->split_parts = static_cast<uint32_t>(v);
    }
    if (const char* e = std::getenv("RTX_SPLIT_FACTOR")) {
        const double f = std::atof(e);
        if (f > 0 && f < 1e6) { c->split_permille = static_cast<uint32_t>(f * 1000.0); c->tune_on = false; }
    }
    if (const char* e = std::getenv("RTX_SPLIT_TUNE")) c->tune_on = c->tune_on && std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("RTX_SPLIT_MIN_US")) {
        const double us = std::atof(e);
        if (us >= 0 && us < 1e6) c->split_min = static_cast<uint32_t>(us * kSplitMinCost / kSplitMinUs);
    }
    const size_t heavy_px = static_cast<size_t>(kMaxHeavyTiles) * 64;   // pixels of the heavy wave tiles
    int cus = 0, lo_prio = 0, hi_prio = 0;
#define RTX_CREATE_TRY(call)                                                             \
    do {                                                                                 \
        const hipError_t e_ = (call);                                                    \
        if (e_ != hipSuccess) {                                                          \
            g_create_err = std::string(#call) + ": " + hipGetErrorString(e_);            \
            rtx_destroy(c);                                                              \
            return RTX_E_DEVICE;                                                         \
        }                                                                                \
    } while (0)
    RTX_CREATE_TRY(hipSetDevice(device_id));
    RTX_CREATE_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    RTX_CREATE_TRY(hipEventCreate(&c->ev0));
    RTX_CREATE_TRY(hipEventCreate(&c->ev1));
    RTX_CREATE_TRY(hipEventCreateWithFlags(&c->ev_heavy, hipEventDisableTiming));
    RTX_CREATE_TRY(hipEventCreateWithFlags(&c->sb[0].done, hipEventDisableTiming));
    RTX_CREATE_TRY(hipEventCreateWithFlags(&c->sb[1].done, hipEventDisableTiming));
    RTX_CREATE_TRY(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    RTX_CREATE_TRY(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    RTX_CREATE_TRY(hipEventCreateWithFlags(&c->ev_frame, hipEventDisableTiming));
    for (auto& e : c->ev_tune) RTX_CREATE_TRY(hipEventCreate(&e));
    for (auto& e : c->ev_win) RTX_CREATE_TRY(hipEventCreate(&e));
    RTX_CREATE_TRY(hipEventCreateWithFlags(&c->ev_refine, hipEventDisableTiming));
    RTX_CREATE_TRY(hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
    if (const char* e = std::getenv("RTX_SPLIT_PRIO"); e && std::strcmp(e, "0") == 0) hi_prio = lo_prio;
    RTX_CREATE_TRY(hipStreamCreateWithPriority(&c->split_stream, hipStreamNonBlocking, hi_prio));
    RTX_CREATE_TRY(hipMalloc(&c->d_counters, sizeof(unsigned long long) * kNumCounters));
    // {heavy tiles, max tile cost (rtx_sched_count), max tile cost, cost per wave slot (rtx_sched_scan)}
    RTX_CREATE_TRY(hipMalloc(&c->d_heavy_n, 16));
    RTX_CREATE_TRY(hipMemset(c->d_heavy_n, 0, 16));
    RTX_CREATE_TRY(hipMalloc(&c->d_thr, 8));
    RTX_CREATE_TRY(hipHostMalloc(&c->h_heavy_n, 16));
    RTX_CREATE_TRY(hipMalloc(&c->d_heavy_list[0], 4 * kMaxHeavyTiles));
    RTX_CREATE_TRY(hipMalloc(&c->d_heavy_list[1], 4 * kMaxHeavyTiles));
    RTX_CREATE_TRY(hipMalloc(&c->d_hit_key, 8 * heavy_px));
    RTX_CREATE_TRY(hipMalloc(&c->d_occ, 4 * heavy_px));
    RTX_CREATE_TRY(hipMemset(c->d_hit_key, 0xff, 8 * heavy_px));
    RTX_CREATE_TRY(hipMemset(c->d_occ, 0, 4 * heavy_px));
    // (null-stream memsets are asynchronous to the host and the context's non-blocking streams do
    // not wait for them: finish them before any launch can read these buffers)
    RTX_CREATE_TRY(hipStreamSynchronize(nullptr));
    RTX_CREATE_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_id));
#undef RTX_CREATE_TRY
    // waves resident at once: 7 per SIMD, 4 SIMDs per CU at the render kernel's occupancy
    c->split_slots = static_cast<uint32_t>(cus > 0 ? cus : 1) * 28u;
    if (!std::getenv("RTX_LIGHT_MAJOR_TILES")) c->lm_tiles = c->split_slots * kLmSlotsPercent / 100u;
    c->lm_waves = static_cast<uint32_t>(cus > 0 ? cus : 1) * 32u;
    *out = c;
    return RTX_OK;
}

extern "C" void rtx_destroy(rtx_ctx* c) {
    if (!c) return;
    frames_forget(c);
    (void)hipSetDevice(c->device);
    if (c->split_stream) (void)hipStreamSynchronize(c->split_stream);   // (a deferred chain, join_pending)
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& B : c->sb) {
        (void)hipFree(B.d);
        (void)hipFree(B.cull);
        if (B.h) (void)hipHostFree(B.h);
        if (B.done) (void)hipEventDestroy(B.done);
    }
    (void)hipFree(c->d_px);
    (void)hipFree(c->d_rgb);
    (void)hipFree(c->d_counters);
    (void)hipFree(c->d_order);
    (void)hipFree(c->d_order_xcd);
    (void)hipFree(c->d_cost);
    (void)hipFree(c->d_saved_cost);
    (void)hipFree(c->d_hist);
    (void)hipFree(c->d_csum);
    (void)hipFree(c->d_thr);
    for (int k = 0; k < 2; ++k) { (void)hipFree(c->d_heavy_flag[k]); (void)hipFree(c->d_heavy_list[k]); }
    (void)hipFree(c->d_heavy_n);
    if (c->h_heavy_n) (void)hipHostFree(c->h_heavy_n);
    (void)hipFree(c->d_hit_key);
    (void)hipFree(c->d_occ);
    (void)hipFree(c->d_lm_rec);
    (void)hipFree(c->d_lm_mask);
    (void)hipFree(c->d_hstk);
    (void)hipFree(c->d_hstkT);
    (void)hipFree(c->d_cull_btree);
    (void)hipFree(c->d_cull_mtree);
    (void)hipFree(c->d_cull_nbox);
    (void)hipFree(c->d_cull_arrive);
    if (c->ev_heavy) (void)hipEventDestroy(c->ev_heavy);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->ev_frame) (void)hipEventDestroy(c->ev_frame);
    for (auto& e : c->ev_tune)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : c->ev_win)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_refine) (void)hipEventDestroy(c->ev_refine);
    (void)hipFree(c->d_part_max);
    if (c->split_stream) {
        (void)hipStreamSynchronize(c->split_stream);
        (void)hipStreamDestroy(c->split_stream);
    }
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

// NULL: why the last rtx_create on this thread failed (empty if it did not).
extern "C" const char* rtx_last_error(const rtx_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

extern "C" int rtx_scene_bytes(const rtx_ctx* c, uint64_t* bytes) {
    if (!c || !bytes) return RTX_E_INVALID;
    *bytes = c->scene_bytes;
    return RTX_OK;
}

namespace {
// Queue the record launches on the context stream: with `boxes` (at upload) the box tree and
// every slot's box, then, for the anchors in A, their margin trees and records.  Grows the
// scratch (after a stream sync: queued launches may still read the old buffers).
int cull_launch(rtx_ctx* c, const CullAnchors& A, bool boxes) {
    const uint32_t nt = c->cull_ntris;
    const uint32_t n = c->cull_n;
    if (c->cull_fail_at && ++c->cull_launches == c->cull_fail_at)   // RTX_CULL_FAIL (tests of the error path)
        return fail(c, RTX_E_NOMEM, "cull records: injected failure (RTX_CULL_FAIL)");
    // the anchors' margin trees: 2n entries per anchor of THIS launch (an upload's first launch has the
    // lights and the views, later ones the views that moved), grown on demand
    const size_t mtree_need = 2 * static_cast<size_t>(n) * std::max<uint32_t>(A.n, 1u);
    if (n > c->cull_tree_cap || mtree_need > c->cull_mtree_cap || c->cull_nslots > c->cull_nbox_cap ||
        !c->d_cull_arrive) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        if (n > c->cull_tree_cap) {
            (void)hipFree(c->d_cull_btree);
            c->d_cull_btree = nullptr;
            c->cull_tree_cap = 0;
            HIP_TRY(c, hipMalloc(&c->d_cull_btree, 2 * static_cast<size_t>(n) * sizeof(CullBox)));
            c->cull_tree_cap = n;
        }
        if (mtree_need > c->cull_mtree_cap) {
            (void)hipFree(c->d_cull_mtree);
            c->d_cull_mtree = nullptr;
            c->cull_mtree_cap = 0;
            HIP_TRY(c, hipMalloc(&c->d_cull_mtree, mtree_need * sizeof(CullMD)));
            c->cull_mtree_cap = mtree_need;
        }
        if (c->cull_nslots > c->cull_nbox_cap) {
            (void)hipFree(c->d_cull_nbox);
            c->d_cull_nbox = nullptr;
            c->cull_nbox_cap = 0;
            HIP_TRY(c, hipMalloc(&c->d_cull_nbox, static_cast<size_t>(c->cull_nslots) * sizeof(CullBox)));
            c->cull_nbox_cap = c->cull_nslots;
        }
        if (!c->d_cull_arrive) {
            HIP_TRY(c, hipMalloc(&c->d_cull_arrive, (kCullMaxAnchors + 1) * sizeof(uint32_t)));
            // on the context stream: a plain hipMemset runs on the null stream, which this
            // non-blocking stream does not wait for (the first tree launch then read whatever the
            // recycled allocation held as its arrival counts)
            HIP_TRY(c, hipMemsetAsync(c->d_cull_arrive, 0, (kCullMaxAnchors + 1) * sizeof(uint32_t), c->stream));
        }
    }
    for (uint32_t j = 0; j < A.n; ++j) {
        for (int k = 0; k < 4; ++k) c->cull_anchor[A.idx[j]][k] = A.p[j][k];
        c->cull_anchor[A.idx[j]][4] = A.bt[j];
    }
    const uint32_t nwg = n / kCullTreeWG, sb = (c->cull_nslots + 255u) / 256u;
    float4* rec = const_cast<float4*>(c->dev.cull);
    const uint32_t stride4 = c->dev.cull_stride / 16u;
    const CullParams P{c->dev.nodes, c->cull_ratio, c->cull_leaves ? 1u : 0u};
    if (A.n || boxes) {
        hipLaunchKernelGGL(rtx_cull_tris, dim3(nwg, A.n + (boxes ? 1u : 0u)), dim3(kCullTreeWG), 0, c->stream,
                           c->dev.tris, nt, A, c->d_cull_mtree, c->d_cull_btree, c->d_cull_arrive, c->cull_top_lds);
        HIP_TRY(c, hipGetLastError());
    }
    if (boxes) {
        hipLaunchKernelGGL(rtx_cull_nodes<true>, dim3(sb), dim3(256), 0, c->stream, c->cull_rng, c->cull_nslots, nt, n,
                           c->d_cull_btree, c->d_cull_nbox, c->d_cull_mtree, A, rec, stride4, P);
    } else if (A.n) {
        hipLaunchKernelGGL(rtx_cull_nodes<false>, dim3(sb), dim3(256), 0, c->stream, c->cull_rng, c->cull_nslots, nt,
                           n, c->d_cull_btree, c->d_cull_nbox, c->d_cull_mtree, A, rec, stride4, P);
    }
    HIP_TRY(c, hipGetLastError());
    return RTX_OK;
}

// At upload: the light anchors (tmax bound T[l]) the first frame's record launches build, with the
// per-triangle boxes (cull_views).
void cull_records(rtx_ctx* c, const std::vector<float>& T, const rtx_light* lights, uint32_t n_lights) {
    c->cull_lights.clear();
    for (uint32_t l = 0; l < n_lights; ++l)
        c->cull_lights.push_back({lights[l].origin[0], lights[l].origin[1], lights[l].origin[2],
                                  T[l] > 0.f ? T[l] : 1.f});   // T = 0: never culled (cull_ray), any bound will do
    c->cull_boxes_pending = true;
}

// Before a frame: after an upload the boxes and the lights' records, and the records of every view
// whose camera origin is not the one its records of the current image were made for (bitwise).
// The records' state (pending boxes, valid views) is committed only once their launches are queued:
// when building them fails (an allocation), the image renders without the cull from then on — the
// unculled walk, the same pixels — instead of a later frame trusting records never written.
int cull_views(rtx_ctx* c, const FrameArgs& F) {
    CullAnchors A{};
    const bool boxes = c->cull_boxes_pending;
    if (boxes) {
        for (size_t l = 0; l < c->cull_lights.size(); ++l) {
            for (int k = 0; k < 4; ++k) A.p[A.n][k] = c->cull_lights[l][k];
            A.bt[A.n] = A.p[A.n][3];
            A.idx[A.n] = static_cast<uint32_t>(kMaxViews + l);
            ++A.n;
        }
    }
    uint32_t valid = c->cull_view_valid;
    for (uint32_t v = 0; v < F.n_views && v < static_cast<uint32_t>(kMaxViews); ++v) {
        const float* o = F.cam[v].origin;
        if ((valid >> v) & 1u && std::memcmp(c->cull_view[v], o, 12) == 0) continue;
        valid |= 1u << v;
        for (int k = 0; k < 3; ++k) A.p[A.n][k] = o[k];
        A.p[A.n][3] = 0.f;
        A.bt[A.n] = F.cam[v].cull_bt;
        A.idx[A.n] = v;
        ++A.n;
    }
    if (A.n == 0 && !boxes) return RTX_OK;
    if (cull_launch(c, A, boxes) != RTX_OK) {   // (c->err says why)
        c->dev.cull = nullptr;
        c->dev.cull_T = nullptr;
        c->dev.cull_stride = 0;
        c->cull_boxes_pending = false;
        c->cull_view_valid = 0;
        ++c->cull_failures;
        (void)hipGetLastError();
        return RTX_OK;
    }
    if (A.n > (boxes ? c->cull_lights.size() : 0u)) ++c->cull_updates;
    for (uint32_t j = 0; j < A.n; ++j)
        if (A.idx[j] < static_cast<uint32_t>(kMaxViews)) std::memcpy(c->cull_view[A.idx[j]], A.p[j], 12);
    c->cull_view_valid = valid;
    c->cull_boxes_pending = false;
    return RTX_OK;
}
}  // namespace

extern "C" int rtx_upload_scene(rtx_ctx* c, const rtx_scene* s) {
    if (c) {   // the upload pattern the cull decision reads (see rtx_ctx::cull_animated)
        c->short_uploads = (c->has_scene && c->renders_since_upload <= 1) ? c->short_uploads + 1 : 0;
        c->renders_since_upload = 0;
        c->upload_motion = c->short_uploads >= 1;
        if (const int rc = join_split(c); rc != RTX_OK) return rc;   // (the last chain reads the current image)
    }
    return upload_scene(c, s, nullptr);
}

namespace rtxh {
int upload_scene(rtx_ctx* c, const rtx_scene* s, UploadLayout* lay) {
    if (!c || !s) return RTX_E_INVALID;
    if ((s->n_spheres && !s->spheres) || (s->n_planes && !s->planes) || (s->n_meshes && !s->meshes) ||
        (s->n_lights && !s->lights) || (s->n_materials && !s->materials))
        return fail(c, RTX_E_INVALID, "null array with non-zero count");
    if (s->n_materials == 0 || s->n_materials > 256) return fail(c, RTX_E_INVALID, "need 1..256 materials");
    const uint32_t nm = s->n_materials;
    std::vector<float4> sph, pl, tri, nodes, lights, mats;
    std::vector<uint32_t> sph_mat;
    std::vector<int4> meshes, parts;
    {
        size_t nt = 0, nn = 0;
        for (uint32_t mi = 0; mi < s->n_meshes; ++mi) { nt += s->meshes[mi].n_indices / 3; nn += s->meshes[mi].n_nodes; }
        tri.reserve(4 * nt);
        nodes.reserve(2 * nn + 4 * s->n_meshes + 4);
    }
    bool split_ok = s->n_lights <= static_cast<uint32_t>(kMaxSplitLights);
    // exact cull (DevScene::cull): host uploads (a device-animated image is rebuilt in place and
    // carries no records), at most kMaxCullLights lights
    bool cull_on = !lay && !c->no_cull && s->n_lights <= static_cast<uint32_t>(kMaxCullLights) &&
                   (c->short_uploads < 2 || c->cull_animated);
    double bmin[3] = {INFINITY, INFINITY, INFINITY}, bmax[3] = {-INFINITY, -INFINITY, -INFINITY};   // mesh vertices
    std::vector<std::pair<uint32_t, uint32_t>> mesh_slots;   // node slots [first, end) of each mesh's tree
    std::vector<uint2> slot_rng;   // per device node slot: its triangles (slot_ranges)
    bool ordered_all = true;
    std::vector<float> tbox;   // per triangle (lo, hi) per axis: the cull's worth estimate below
    std::string worth_sig;
    bool reuse_worth = false;
    if (cull_on) {
        // (not the node count: an animated loop's host rebuilds its trees, whose sizes vary)
        size_t nt = 0;
        for (uint32_t mi = 0; mi < s->n_meshes; ++mi) nt += s->meshes[mi].n_indices / 3;
        worth_sig = std::to_string(s->n_spheres) + "/" + std::to_string(s->n_planes) + "/" + std::to_string(s->n_meshes) +
                    "/" + std::to_string(nt) + "/" + std::to_string(s->n_lights);
        reuse_worth = c->short_uploads >= 1 && c->cull_worth >= 0 && c->cull_worth_age + 1 < kCullWorthReuse &&
                      c->cull_worth_sig == worth_sig;
        if (!reuse_worth) tbox.reserve(6 * nt);
    }
    double max_ee = 0.0;   // max |e1| * |e2| over the triangles (DevScene::tri_fast)
    double max_ee2_lo = 0.0;
    int max_depth = 0;     // deepest BVH node over the meshes (stack variant)
    for (uint32_t i = 0; i < s->n_spheres; ++i) {
        const rtx_sphere& p = s->spheres[i];
        if (p.material >= nm) return fail(c, RTX_E_INVALID, "sphere material out of range");
        sph.push_back(f4(p.origin[0], p.origin[1], p.origin[2], p.radius * p.radius));   // Square(radius)
        sph_mat.push_back(p.material);
    }
    for (uint32_t i = 0; i < s->n_planes; ++i) {
        const rtx_plane& p = s->planes[i];
        if (p.material >= nm) return fail(c, RTX_E_INVALID, "plane material out of range");
        pl.push_back(f4(p.origin[0], p.origin[1], p.origin[2], bits(p.material)));
        pl.push_back(f4(p.normal[0], p.normal[1], p.normal[2], 0.f));
    }
    for (uint32_t mi = 0; mi < s->n_meshes; ++mi) {
        const rtx_mesh& m = s->meshes[mi];
        if (m.material >= nm) return fail(c, RTX_E_INVALID, "mesh material out of range");
        if (m.cull_mode < RTX_CULL_FRONT || m.cull_mode > RTX_CULL_NONE) return fail(c, RTX_E_INVALID, "bad cull mode");
        if (m.n_indices % 3) return fail(c, RTX_E_INVALID, "mesh index count not a multiple of 3");
        const uint32_t tri0 = static_cast<uint32_t>(tri.size() / 4), node0 = static_cast<uint32_t>(nodes.size() / 2);
        const uint32_t ntri = m.n_indices / 3;
        if (ntri && (!m.positions || !m.indices || !m.normals)) return fail(c, RTX_E_INVALID, "mesh arrays missing");
        for (uint32_t k = 0; k < ntri; ++k) {
            const int32_t i0 = m.indices[3 * k], i1 = m.indices[3 * k + 1], i2 = m.indices[3 * k + 2];
            if (i0 < 0 || i1 < 0 || i2 < 0 || static_cast<uint32_t>(i0) >= m.n_positions ||
                static_cast<uint32_t>(i1) >= m.n_positions || static_cast<uint32_t>(i2) >= m.n_positions)
                return fail(c, RTX_E_INVALID, "mesh index out of range");
            const float* v0 = m.positions + 3 * i0;
            const float* v1 = m.positions + 3 * i1;
            const float* v2 = m.positions + 3 * i2;
            const float* n = m.normals + 3 * k;
            // edge1 = v1 - v0, edge2 = v2 - v0 (Utils.h:139-140), same binary32 ops as on device
            const float4 e1 = f4(v1[0] - v0[0], v1[1] - v0[1], v1[2] - v0[2], n[1]);
            const float4 e2 = f4(v2[0] - v0[0], v2[1] - v0[1], v2[2] - v0[2], n[2]);
            tri.push_back(f4(v0[0], v0[1], v0[2], n[0]));
            tri.push_back(e1);
            tri.push_back(e2);
            // |e1| |e2| (two square roots) only for a triangle that can raise the maximum: below
            // max_ee^2 (1 - 2^-40) the product of the roots cannot reach max_ee (their rounding is
            // ~2^-51); NaN always takes the exact path
            const double a2 = double(e1.x) * e1.x + double(e1.y) * e1.y + double(e1.z) * e1.z;
            const double b2 = double(e2.x) * e2.x + double(e2.y) * e2.y + double(e2.z) * e2.z;
            if (!(a2 * b2 < max_ee2_lo)) {
                const double ee = std::sqrt(a2) * std::sqrt(b2);
                max_ee = (ee > max_ee || ee != ee) ? ee : max_ee;   // NaN sticks
                max_ee2_lo = max_ee * max_ee * (1.0 - 0x1p-40);
            }
            tri.push_back(f4(bits(m.material), 0.f, 0.f, 0.f));
            for (int a = 0; a < 3; ++a) {
                const float lo = std::fmin(v0[a], std::fmin(v1[a], v2[a])), hi = std::fmax(v0[a], std::fmax(v1[a], v2[a]));
                bmin[a] = std::fmin(bmin[a], lo);
                bmax[a] = std::fmax(bmax[a], hi);
                if (cull_on && !reuse_worth) { tbox.push_back(lo); tbox.push_back(hi); }
            }
        }
        uint32_t root = 0;
        bool contig_m = true, ordered_m = true;
        if (m.n_nodes) {
            if (!m.nodes) return fail(c, RTX_E_INVALID, "mesh nodes missing");
            // Re-lay the tree out for the device: the root at an odd slot, every child pair
            // (left, left + 1) at an even slot so one 64-B scalar load fetches both boxes.
            // Only the numbering changes; the tree and the left-then-right order do not.  The same
            // walk validates the tree (child indices, cycles) and finds its depth: the deepest DFS
            // stack a wave can need (pending right siblings on a path).
            if ((nodes.size() / 2) % 2 == 0) { nodes.push_back(f4(0, 0, 0, 0)); nodes.push_back(f4(0, 0, 0, 0)); }
            root = static_cast<uint32_t>(nodes.size() / 2);
            struct Work { uint32_t src, dst; int depth; };   // (mesh-local node, device slot, depth)
            std::vector<Work> work;
            work.reserve(64);
            work.push_back({0u, root, 0});
            nodes.resize(nodes.size() + 2);
            int depth = 0;
            size_t visited = 0;
            while (!work.empty()) {
                const Work w = work.back();
                work.pop_back();
                const uint32_t src = w.src, dst = w.dst;
                if (++visited > 4ull * m.n_nodes + 4) return fail(c, RTX_E_INVALID, "BVH has a cycle");
                depth = w.depth > depth ? w.depth : depth;
                const rtx_bvh_node& nd = m.nodes[src];
                uint32_t link, cnt;
                if (nd.idx_count == 0 && (nd.left_node + 1 >= m.n_nodes || nd.left_node == 0))
                    return fail(c, RTX_E_INVALID, "BVH child index out of range");
                if (nd.idx_count > 0) {
                    if (nd.first_idx % 3 || nd.idx_count % 3 || nd.first_idx + nd.idx_count > m.n_indices)
                        return fail(c, RTX_E_INVALID, "BVH leaf range invalid");
                    link = tri0 + nd.first_idx / 3;
                    cnt = nd.idx_count / 3;
                } else {
                    link = static_cast<uint32_t>(nodes.size() / 2);   // even: sizes stay even after the root
                    cnt = 0;
                    nodes.resize(nodes.size() + 4);
                    work.push_back({nd.left_node + 1, link + 1, w.depth + 1});
                    work.push_back({nd.left_node, link, w.depth + 1});
                }
                // device layout: {min.x, max.x, min.y, max.y}, {min.z, max.z, link, ntri} (slab_mask)
                nodes[2 * dst] = f4(nd.min[0], nd.max[0], nd.min[1], nd.max[1]);
                nodes[2 * dst + 1] = f4(nd.min[2], nd.max[2], bits(link), bits(cnt));
            }
            max_depth = std::max(max_depth, depth);
            if (lay) lay->depth[mi] = depth;
            mesh_slots.push_back({root, static_cast<uint32_t>(nodes.size() / 2)});
            slot_ranges(nodes, root, static_cast<uint32_t>(nodes.size() / 2), slot_rng, contig_m, ordered_m);
            ordered_all = ordered_all && ordered_m;
            if (lay && lay->reserve[mi]) {   // slots root .. root + 2T - 1 belong to this mesh
                const size_t want = 2 * (static_cast<size_t>(root) + 2 * static_cast<size_t>(ntri));
                if (nodes.size() < want) nodes.resize(want + (want / 2) % 2 * 2, f4(0, 0, 0, 0));
            }
        }
        if (lay) { lay->tri0[mi] = tri0; lay->root[mi] = root; }
        const float cs = m.cull_mode == RTX_CULL_FRONT ? -1.f : (m.cull_mode == RTX_CULL_BACK ? 1.f : 0.f);
        // {root node byte offset, node count, cull sign bits, material}
        meshes.push_back(make_int4(static_cast<int>(root * 32u), static_cast<int>(m.n_nodes), bitsi_f(cs), m.material));
        (void)node0;
        // ~48 triangles per part at least: finer parts of a small mesh cost more than they spread
        const uint32_t target = std::max(2u, std::min(c->split_parts, ntri / 48u));
        const size_t p0 = parts.size();
        if (m.n_nodes && !build_parts(nodes, root, mi, target, slot_rng, contig_m, parts)) split_ok = false;
        if (lay && lay->reserve[mi]) {   // exactly `target` entries, the unused ones {-1, ...}
            parts.resize(p0 + target, make_int4(-1, 0, 0, 0));
            lay->part0[mi] = static_cast<uint32_t>(p0);
            lay->part_cap[mi] = target;
        }
    }
    if (parts.size() > static_cast<size_t>(kMaxParts)) split_ok = false;
    if (!split_ok) parts.clear();
    // static uploads reserve kMaxParts entries for the frontier refinement (refine_round); meshes
    // with device-rebuild reserves keep theirs exactly
    bool any_reserve = false;
    if (lay)
        for (uint8_t r : lay->reserve) any_reserve = any_reserve || r != 0;
    const size_t n_parts_real = parts.size();
    const bool refinable = split_ok && n_parts_real > 0 && !any_reserve;
    if (refinable) parts.resize(kMaxParts, make_int4(-1, 0, 0, 0));
    // Cull records' inputs: per node slot the range of device triangles under it (leaf order is
    // contiguous within a subtree; children's slots follow their parent's, so one backward sweep)
    // and per light the tmax up to which its shadow rays are culled: 4x the farthest mesh-box
    // corner + 1 (longer rays pass).
    std::vector<uint2> cull_rng;
    std::vector<float> cull_T;
    if (cull_on) {
        cull_on = !tri.empty() && !mesh_slots.empty();
        for (int a = 0; a < 3; ++a) cull_on = cull_on && std::isfinite(bmin[a]) && std::isfinite(bmax[a]);
    }
    if (cull_on) {
        // Worth it?  The surface areas of the reference's boxes over those of the tight boxes,
        // summed over the nodes (the SAH estimate of how many more slab tests the reference's
        // boxes pass): below c->cull_min_sa the records cost more than they save (measured: W4_Bunny
        // 1.19, -11 %; W4_Optional 2.40, +48 %; Synthetic100k 9.26, +182 %; profiles/r04).
        cull_rng = slot_rng;
        cull_rng.resize(nodes.size() / 2, make_uint2(0u, 0u));
        const bool increasing = ordered_all;   // the ordered walk needs left-then-right = increasing index
        if (reuse_worth) {
            ++c->cull_worth_age;
            cull_on = increasing && c->cull_worth == 1;
        } else {
            std::vector<float> nb(6 * (nodes.size() / 2));
            double sa_ref = 0.0, sa_tight = 0.0;
            auto sa = [](double x, double y, double z) { return 2.0 * (x * y + y * z + z * x); };
            for (const auto& [r0, r1] : mesh_slots)
                for (uint32_t sl = r1; sl-- > r0;) {
                    uint32_t link, cnt;
                    std::memcpy(&link, &nodes[2 * sl + 1].z, 4);
                    std::memcpy(&cnt, &nodes[2 * sl + 1].w, 4);
                    float* b = &nb[6 * sl];
                    if (cnt) {
                        for (int a = 0; a < 3; ++a) { b[2 * a] = INFINITY; b[2 * a + 1] = -INFINITY; }
                        for (uint32_t t = link; t < link + cnt && t < tbox.size() / 6; ++t)
                            for (int a = 0; a < 3; ++a) {
                                b[2 * a] = std::fmin(b[2 * a], tbox[6 * t + 2 * a]);
                                b[2 * a + 1] = std::fmax(b[2 * a + 1], tbox[6 * t + 2 * a + 1]);
                            }
                    } else {
                        for (int a = 0; a < 3; ++a) {
                            b[2 * a] = std::fmin(nb[6 * link + 2 * a], nb[6 * (link + 1) + 2 * a]);
                            b[2 * a + 1] = std::fmax(nb[6 * link + 2 * a + 1], nb[6 * (link + 1) + 2 * a + 1]);
                        }
                    }
                    const float4 r0v = nodes[2 * sl], r1v = nodes[2 * sl + 1];
                    sa_ref += sa(double(r0v.y) - r0v.x, double(r0v.w) - r0v.z, double(r1v.y) - r1v.x);
                    sa_tight += sa(std::fmax(double(b[1]) - b[0], 0.0), std::fmax(double(b[3]) - b[2], 0.0),
                                   std::fmax(double(b[5]) - b[4], 0.0));
                }
            const bool worth = sa_ref >= c->cull_min_sa * sa_tight;   // false for NaN
            c->cull_worth = worth ? 1 : 0;
            c->cull_worth_age = 0;
            c->cull_worth_sig = worth_sig;
            cull_on = increasing && worth;
        }
        for (uint32_t i = 0; i < s->n_lights; ++i) {
            double R = 0.0;
            for (int k = 0; k < 8; ++k) {
                const double cx = (k & 1) ? bmax[0] : bmin[0], cy = (k & 2) ? bmax[1] : bmin[1],
                             cz = (k & 4) ? bmax[2] : bmin[2];
                const double dx = s->lights[i].origin[0] - cx, dy = s->lights[i].origin[1] - cy,
                             dz = s->lights[i].origin[2] - cz;
                R = std::fmax(R, std::sqrt(dx * dx + dy * dy + dz * dz));
            }
            const double T = 4.0 * R + 1.0;
            cull_T.push_back(std::isfinite(T) && T < 0x1p60 ? static_cast<float>(T) : 0.f);   // 0: never culled
        }
    }
    // Device links are byte offsets (s_load with an SGPR offset, no address arithmetic):
    // inner node -> its child pair (2 slots x 32 B), leaf -> its first 64-B triangle.
    if (tri.size() * 16 >= (1ull << 32) || nodes.size() * 16 >= (1ull << 32) || sph.size() * 16 >= (1ull << 32) ||
        pl.size() * 16 >= (1ull << 32))
        return fail(c, RTX_E_INVALID, "scene too large for 32-bit record offsets");
    for (size_t n = 0; n < nodes.size(); n += 2) {
        uint32_t link, cnt;
        std::memcpy(&link, &nodes[n + 1].z, 4);
        std::memcpy(&cnt, &nodes[n + 1].w, 4);
        nodes[n + 1].z = bits(cnt ? link * 64u : link * 32u);
    }
    // Octant copies of the node array (DevScene::oct_bytes, slab_mask<kSlabOct>): possible
    // when every box is ordered lo <= hi per axis (no NaN).  The reference's quirky bounds
    // (max initialised with FLT_MIN) stay ordered; an empty box would not.
    // Large trees keep one copy: 8 copies of a multi-MB node array crowd the L2 (Synthetic100k,
    // ~2 MB per copy, is 2.5 % faster without them; W4_Optional, 117 KB, 2.5 % faster with).
    const size_t node_bytes = align256(nodes.size() * 16);
    bool oct_ok = !nodes.empty() && node_bytes <= kOctantMaxNodeBytes && 8 * node_bytes < (1ull << 32);
    for (size_t n = 0; oct_ok && n < nodes.size(); n += 2)
        oct_ok = nodes[n].x <= nodes[n].y && nodes[n].z <= nodes[n].w && nodes[n + 1].x <= nodes[n + 1].y;
    // the node section: 8 octant copies (node_bytes apart, written straight into the
    // staging image below) or the one array
    const size_t node_sec = oct_ok ? 8 * node_bytes : nodes.size() * 16;
    for (uint32_t i = 0; i < s->n_lights; ++i) {
        const rtx_light& l = s->lights[i];
        lights.push_back(f4(l.origin[0], l.origin[1], l.origin[2], bitsi(l.type)));
        lights.push_back(f4(l.color[0], l.color[1], l.color[2], l.intensity));
    }
    for (uint32_t i = 0; i < nm; ++i) {
        const rtx_material& m = s->materials[i];
        // BRDF::Lambert(kd, cd) = (cd * kd) / PI (BRDFs.h:14-17), exact binary32 on host
        const float lr = (m.color[0] * m.kd) / RTX_PI, lg = (m.color[1] * m.kd) / RTX_PI, lb = (m.color[2] * m.kd) / RTX_PI;
        mats.push_back(f4(bitsi(m.kind), m.color[0], m.color[1], m.color[2]));
        mats.push_back(f4(m.kd, m.ks, m.exponent, m.metalness));
        mats.push_back(f4(m.roughness, lr, lg, lb));
    }

    struct Sec { const void* p; size_t n; size_t off; };
    Sec secs[] = {{sph.data(), sph.size() * 16, 0},       {sph_mat.data(), sph_mat.size() * 4, 0},
                  {pl.data(), pl.size() * 16, 0},         {tri.data(), tri.size() * 16, 0},
                  {nullptr, node_sec, 0},
                  {meshes.data(), meshes.size() * 16, 0}, {lights.data(), lights.size() * 16, 0},
                  {mats.data(), mats.size() * 16, 0},     {parts.data(), parts.size() * 16, 0},
                  {cull_rng.data(), cull_rng.size() * 8, 0}, {cull_T.data(), cull_T.size() * 4, 0}};
    size_t total = 0;
    for (auto& x : secs) { x.off = total; total += align256(x.n ? x.n : 16); }
    HIP_TRY(c, hipSetDevice(c->device));
    const int k = c->sb_cur < 0 ? 0 : (c->sb_cur ^ 1);
    rtx_ctx::SceneBuf& B = c->sb[k];
    if (B.pending) {   // frames queued against image k (two uploads ago) must be done with it
        HIP_TRY(c, hipEventSynchronize(B.done));
        B.pending = false;
    }
    if (total > B.cap) {
        (void)hipFree(B.d);
        if (B.h) (void)hipHostFree(B.h);
        B.d = nullptr;
        B.h = nullptr;
        B.cap = 0;
        HIP_TRY(c, hipMalloc(&B.d, total));
        HIP_TRY(c, hipHostMalloc(&B.h, total));
        B.cap = total;
    }
    // cull records: one copy of the node slots per anchor (kMaxViews cameras, then the lights)
    const size_t cull_stride = align256(nodes.size() * 16);
    const size_t cull_bytes = cull_on ? (kMaxViews + static_cast<size_t>(s->n_lights)) * cull_stride : 0;
    if (cull_on && (cull_stride >= (1ull << 32) || 2 * tri.size() >= (1ull << 32))) cull_on = false;
    if (cull_on && cull_bytes > B.cull_cap) {
        (void)hipFree(B.cull);
        B.cull = nullptr;
        B.cull_cap = 0;
        HIP_TRY(c, hipMalloc(&B.cull, cull_bytes));
        B.cull_cap = cull_bytes;
    }
    // Large node arrays send copy 0 only and the device writes copies 1..7 (rtx_octant_expand):
    // 1/8 of the node bytes over PCIe and of the host's staging writes (an upload per animated
    // frame).  Small ones are cheaper as host writes than as one more launch.
    const bool oct_dev = oct_ok && node_bytes >= kOctantDeviceMinBytes;
    // sections in place; only the padding up to the next section is cleared (an upload per
    // animated frame: no full-image memset, no intermediate node image)
    for (size_t i = 0; i < sizeof secs / sizeof secs[0]; ++i) {
        const Sec& x = secs[i];
        const size_t end = i + 1 < sizeof secs / sizeof secs[0] ? secs[i + 1].off : total;
        if (x.p && x.n) std::memcpy(B.h + x.off, x.p, x.n);
        if (!x.p && x.n && oct_ok) {   // octant copy k stores (hi, lo) on the axes set in k
            for (int k = 0; k < (oct_dev ? 1 : 8); ++k) {
                float4* dst = reinterpret_cast<float4*>(B.h + x.off + k * node_bytes);
                const bool mx = k & 1, my = k & 2, mz = k & 4;
                for (size_t n = 0; n < nodes.size(); n += 2) {
                    const float4 a = nodes[n], b = nodes[n + 1];
                    dst[n] = f4(mx ? a.y : a.x, mx ? a.x : a.y, my ? a.w : a.z, my ? a.z : a.w);
                    dst[n + 1] = f4(mz ? b.y : b.x, mz ? b.x : b.y, b.z, b.w);
                }
                std::memset(reinterpret_cast<char*>(dst + nodes.size()), 0, node_bytes - nodes.size() * 16);
            }
        } else if (!x.p && x.n) {
            std::memcpy(B.h + x.off, nodes.data(), x.n);
        }
        std::memset(B.h + x.off + x.n, 0, end - x.off - x.n);
    }
    if (oct_dev) {   // everything but copies 1..7, which the device writes
        const size_t c1 = secs[4].off + node_bytes, c8 = secs[4].off + 8 * node_bytes;
        HIP_TRY(c, hipMemcpyAsync(B.d, B.h, c1, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(B.d + c8, B.h + c8, total - c8, hipMemcpyHostToDevice, c->stream));
        const uint32_t n2 = static_cast<uint32_t>(node_bytes / 32);
        hipLaunchKernelGGL(rtx_octant_expand, dim3((n2 + 255) / 256, 7), dim3(256), 0, c->stream,
                           reinterpret_cast<float4*>(B.d + secs[4].off), n2, static_cast<uint32_t>(node_bytes / 16));
        HIP_TRY(c, hipGetLastError());
    } else {
        HIP_TRY(c, hipMemcpyAsync(B.d, B.h, total, hipMemcpyHostToDevice, c->stream));
    }
    if (c->sb_cur >= 0) {   // every frame queued so far reads the previous image
        rtx_ctx::SceneBuf& O = c->sb[c->sb_cur];
        HIP_TRY(c, hipEventRecord(O.done, c->stream));
        O.pending = true;
    }
    c->sb_cur = k;
    c->scene_bytes = total;
    char* base = B.d;
    DevScene d{};
    d.spheres = reinterpret_cast<const float4*>(base + secs[0].off);
    d.sphere_mat = reinterpret_cast<const uint32_t*>(base + secs[1].off);
    d.planes = reinterpret_cast<const float4*>(base + secs[2].off);
    d.tris = reinterpret_cast<const Tri*>(base + secs[3].off);
    d.nodes = reinterpret_cast<const float4*>(base + secs[4].off);
    d.meshes = reinterpret_cast<const int4*>(base + secs[5].off);
    d.lights = reinterpret_cast<const float4*>(base + secs[6].off);
    d.materials = reinterpret_cast<const float4*>(base + secs[7].off);
    d.parts = reinterpret_cast<const int4*>(base + secs[8].off);
    d.n_parts = static_cast<uint32_t>(n_parts_real);
    d.n_spheres = s->n_spheres; d.n_planes = s->n_planes; d.n_meshes = s->n_meshes;
    d.n_lights = s->n_lights; d.n_materials = nm;
    d.tri_fast = max_ee <= 0x1p56 ? 1u : 0u;
    d.oct_bytes = (oct_ok && !std::getenv("RTX_NO_OCTANT")) ? static_cast<uint32_t>(node_bytes) : 0u;
    d.n_tris = static_cast<uint32_t>(tri.size() / 4); d.n_nodes = static_cast<uint32_t>(nodes.size() / 2);
    if (cull_on) {
        d.cull = B.cull;
        d.cull_T = reinterpret_cast<const float*>(base + secs[10].off);
        d.cull_stride = static_cast<uint32_t>(cull_stride);
        c->cull_rng = reinterpret_cast<const uint2*>(base + secs[9].off);
        c->cull_nslots = d.n_nodes;
        for (int a = 0; a < 3; ++a) { c->cull_bmin[a] = bmin[a]; c->cull_bmax[a] = bmax[a]; }
        c->cull_ntris = d.n_tris;
        c->cull_n = kCullTreeWG;   // the segment trees' leaves: a power of two >= the triangles
        while (c->cull_n < d.n_tris) c->cull_n *= 2u;
    }
    c->cull_view_valid = 0;
    c->dev = d;
    c->cull_boxes_pending = false;
    if (cull_on) cull_records(c, cull_T, s->lights, s->n_lights);   // (built before the first frame)
    // a BVH kStackDepth or more levels deep renders with the deep-stack variant, unsplit;
    // kStackDepthDeep or more with its stacks in HBM
    c->deep_stack = max_depth >= kStackDepth;
    c->hbm_stack = max_depth >= kStackDepthDeep;
    c->max_depth = static_cast<uint32_t>(max_depth);
    {   // uniform facts for the specialised kernels (kSpec*): the material kinds the geometry
        // references, every light a point light, the sphere / plane / mesh counts
        int kinds = 0;
        bool point = true;
        auto kind = [&](uint32_t m) {
            const int k = s->materials[m].kind;
            kinds |= (k >= RTX_MAT_SOLID_COLOR && k <= RTX_MAT_COOK_TORRANCE) ? (1 << k) : kSpecKindAll;
        };
        for (uint32_t i = 0; i < s->n_spheres; ++i) kind(s->spheres[i].material);
        for (uint32_t i = 0; i < s->n_planes; ++i) kind(s->planes[i].material);
        for (uint32_t i = 0; i < s->n_meshes; ++i) kind(s->meshes[i].material);
        for (uint32_t i = 0; i < s->n_lights; ++i) point = point && s->lights[i].type == RTX_LIGHT_POINT;
        bool cull_back = true;   // kSpecCullBack: every mesh culls back faces
        for (uint32_t i = 0; i < s->n_meshes; ++i) cull_back = cull_back && s->meshes[i].cull_mode == RTX_CULL_BACK;
        // the room's planes (kSpecRoomPlanes): normal +-1 on axis kRoomAxes[k], zero elsewhere,
        // origins finite within 2^64
        bool room = s->n_planes == 5;
        for (uint32_t i = 0; room && i < 5; ++i) {
            const rtx_plane& p = s->planes[i];
            for (int a = 0; a < 3; ++a) {
                const float n = p.normal[a], o = p.origin[a];
                room = room && (a == kRoomAxes[i] ? (n == 1.f || n == -1.f) : n == 0.f) && std::isfinite(o) &&
                       std::fabs(o) <= 0x1p64f;
            }
        }
        for (uint32_t i = 0; room && i < 5; ++i) c->room_p0[i] = s->planes[i].origin[kRoomAxes[i]];
        c->scene_spec = kinds | (point ? kSpecPoint : 0) | (s->n_spheres == 0 ? kSpecNoSpheres : 0) |
                        (s->n_planes == 5 ? kSpecFivePlanes : 0) | (s->n_meshes == 1 ? kSpecOneMesh : 0) |
                        (s->n_meshes == 0 ? kSpecNoMesh : 0) | (room ? kSpecRoomPlanes : 0) |
                        (cull_back ? kSpecCullBack : 0);
    }
    c->split_ok = split_ok && !parts.empty() && !c->deep_stack;
    c->refinable = refinable && c->split_ok && !c->refine_off;
    c->h_parts.assign(parts.begin(), parts.begin() + static_cast<std::ptrdiff_t>(n_parts_real));
    c->h_parts_base = c->h_parts;
    c->parts_dev = reinterpret_cast<int4*>(base + secs[8].off);
    c->refine_round = 0;
    c->refine_state = c->refinable ? 0 : 2;
    c->refine_wait = 0;
    c->refine_prev_max = 0;
    c->has_scene = true;
    ++c->scene_gen;
    c->scene_sig = std::to_string(d.n_spheres) + "/" + std::to_string(d.n_planes) + "/" + std::to_string(d.n_meshes) +
                   "/" + std::to_string(d.n_tris) + "/" + std::to_string(d.n_lights) + "/" + std::to_string(nm);
    if (lay) {
        lay->max_ee = max_ee;
        lay->total = total;
        lay->oct_bytes = d.oct_bytes;
        lay->tri_off = secs[3].off;
        lay->node_off = secs[4].off;
        lay->part_off = secs[8].off;
        lay->mesh_off = secs[5].off;
    }
    return RTX_OK;
}
}  // namespace rtxh

namespace {


int prepare(rtx_ctx* c, const rtx_camera* cams, int n_views, const rtx_render_params* p, bool want_rgb, FrameArgs& F,
            dim3& grid) {
    if (!c || !cams || !p) return RTX_E_INVALID;
    if (n_views < 1 || n_views > kMaxViews) return fail(c, RTX_E_INVALID, "n_views must be 1..8");
    if (!c->has_scene) return fail(c, RTX_E_STATE, "no scene uploaded");
    if (p->width == 0 || p->height == 0 || p->width > 65536 || p->height > 65536)
        return fail(c, RTX_E_INVALID, "bad image size");
    if (p->lighting_mode < 0 || p->lighting_mode >= RTX_MODE_COUNT) return fail(c, RTX_E_INVALID, "bad lighting mode");
    if (p->format.rshift > 24 || p->format.gshift > 24 || p->format.bshift > 24)
        return fail(c, RTX_E_INVALID, "bad pixel format");
    const bool striped = p->stripe_rows != 0 && p->stripe_step > 1;
    if (striped && (p->stripe_rows % 16 != 0 || p->stripe_first >= p->stripe_step))
        return fail(c, RTX_E_INVALID, "stripe_rows must be a multiple of 16 and stripe_first < stripe_step");
    const size_t npx = static_cast<size_t>(p->width) * p->height * static_cast<size_t>(n_views);
    HIP_TRY(c, hipSetDevice(c->device));
    if (c->join_pending &&
        !(n_views == c->join_views && c->scene_gen == c->join_gen && c->sb_cur == c->join_sb &&
          std::memcmp(p, &c->join_p, sizeof *p) == 0 &&
          std::memcmp(cams, c->join_cams, sizeof(rtx_camera) * static_cast<size_t>(n_views)) == 0)) {
        const int rc = join_split(c);
        if (rc != RTX_OK) return rc;
    }
    c->join_p = *p;   // this frame's identity, for the next frame's test above
    std::memcpy(c->join_cams, cams, sizeof(rtx_camera) * static_cast<size_t>(n_views));
    c->join_views = n_views;
    c->join_gen = c->scene_gen;
    c->join_sb = c->sb_cur;
    if (npx > c->px_cap) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        (void)hipFree(c->d_px);
        c->d_px = nullptr;
        c->px_cap = 0;
        HIP_TRY(c, hipMalloc(&c->d_px, npx * 4));
        c->px_cap = npx;
    }
    if (want_rgb && npx > c->rgb_cap) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        (void)hipFree(c->d_rgb);
        c->d_rgb = nullptr;
        c->rgb_cap = 0;
        HIP_TRY(c, hipMalloc(&c->d_rgb, npx * 12));
        c->rgb_cap = npx;
    }
    std::memset(&F, 0, sizeof F);
    for (int v = 0; v < n_views; ++v) {
        for (int k = 0; k < 3; ++k) {
            F.cam[v].origin[k] = cams[v].origin[k]; F.cam[v].right[k] = cams[v].right[k];
            F.cam[v].up[k] = cams[v].up[k]; F.cam[v].forward[k] = cams[v].forward[k];
        }
        F.cam[v].fov = cams[v].fov;
        // the camera anchor's t bound (CullRay::bt): 4x the farthest corner of the meshes' box + 1
        if (c->dev.cull_stride) {
            double R = 0.0;
            for (int k = 0; k < 8; ++k) {
                const double dx = cams[v].origin[0] - ((k & 1) ? c->cull_bmax[0] : c->cull_bmin[0]);
                const double dy = cams[v].origin[1] - ((k & 2) ? c->cull_bmax[1] : c->cull_bmin[1]);
                const double dz = cams[v].origin[2] - ((k & 4) ? c->cull_bmax[2] : c->cull_bmin[2]);
                R = std::fmax(R, std::sqrt(dx * dx + dy * dy + dz * dz));
            }
            const double bt = 4.0 * R + 1.0;
            F.cam[v].cull_bt = std::isfinite(bt) && bt < 0x1p60 ? static_cast<float>(bt) : 0.f;   // 0: no pruning
        }
        if (c->scene_spec & kSpecRoomPlanes) {   // the room planes' camera numerators (ViewCam)
            bool ok = true;
            for (int k = 0; k < 5; ++k) {
                const float a = c->room_p0[k] - cams[v].origin[kRoomAxes[k]];
                const float aa = std::fabs(a);
                F.cam[v].room_a[k] = a;
                ok = ok && (a == 0.f || (aa >= 0x1p-60f && aa <= 0x1p60f));
            }
            F.cam[v].room_fast = ok ? 1u : 0u;
        }
    }
    F.n_views = static_cast<uint32_t>(n_views);
    F.aspect = static_cast<int>(p->width) / static_cast<float>(static_cast<int>(p->height));  // Renderer.cpp:30
    F.inv_width = 1.f / static_cast<float>(static_cast<int>(p->width));
    F.inv_height = 1.f / static_cast<float>(static_cast<int>(p->height));
    F.width = p->width; F.height = p->height;
    F.mode = p->lighting_mode; F.shadows = p->shadows_enabled ? 1 : 0;
    F.rshift = p->format.rshift; F.gshift = p->format.gshift; F.bshift = p->format.bshift; F.amask = p->format.amask;
    const uint32_t groups = (p->height + kWaveTile - 1) / kWaveTile;
    uint32_t gy = groups;
    if (striped) {
        // every view owns the same number of stripes only if the stripe count divides
        // evenly; size the grid for the largest owner and let the kernel skip the rest
        const uint32_t gps = p->stripe_rows / kWaveTile;
        const uint32_t nstripes = (groups + gps - 1) / gps;
        const uint32_t owned = (nstripes + p->stripe_step - 1) / p->stripe_step;
        F.groups_per_stripe = gps; F.stripe_first = p->stripe_first; F.stripe_step = p->stripe_step;
        gy = owned * gps;
    }
    F.tiles_x = (p->width + kWaveTile - 1) / kWaveTile;
    F.tiles_y = gy;
    F.out_px = c->d_px;
    F.out_rgb = want_rgb ? c->d_rgb : nullptr;
    F.counters = c->d_counters;
    const uint32_t ntiles = F.tiles_x * gy * static_cast<uint32_t>(n_views);
    F.n_tiles = ntiles;
    const uint32_t nblocks = (ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
    grid = dim3(nblocks, 1, 1);
    // Cost-ordered dispatch (see the kernel): keep one order/cost pair per launch shape.
    if (ntiles > c->sched_cap) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        (void)hipFree(c->d_order);
        (void)hipFree(c->d_order_xcd);
        c->d_order_xcd = nullptr;
        (void)hipFree(c->d_cost);
        for (int k = 0; k < 2; ++k) { (void)hipFree(c->d_heavy_flag[k]); c->d_heavy_flag[k] = nullptr; }
        (void)hipFree(c->d_saved_cost);
        c->d_saved_cost = nullptr;
        (void)hipFree(c->d_hist);
        (void)hipFree(c->d_csum);
        c->d_hist = nullptr;
        c->d_csum = nullptr;
        c->d_order = nullptr;
        c->d_cost = nullptr;
        c->sched_cap = 0;
        HIP_TRY(c, hipMalloc(&c->d_order, ntiles * 4));
        if (c->xcd_order) HIP_TRY(c, hipMalloc(&c->d_order_xcd, ntiles * 4));
        HIP_TRY(c, hipMalloc(&c->d_cost, ntiles * 4));
        for (int k = 0; k < 2; ++k) HIP_TRY(c, hipMalloc(&c->d_heavy_flag[k], ntiles * 4));
        HIP_TRY(c, hipMalloc(&c->d_saved_cost, ntiles * 4));
        const size_t nch = (ntiles + kSchedChunk - 1) / kSchedChunk;
        HIP_TRY(c, hipMalloc(&c->d_hist, nch * kCostBuckets * 4));
        HIP_TRY(c, hipMalloc(&c->d_csum, nch * 8));
        c->sched_cap = ntiles;
        c->sched_key.clear();
    }
    std::string key = std::to_string(p->width) + "x" + std::to_string(p->height) + "v" + std::to_string(n_views) +
                      "s" + std::to_string(p->stripe_rows) + "/" + std::to_string(p->stripe_first) + "/" +
                      std::to_string(p->stripe_step) + "g" + c->scene_sig + "m" +
                      std::to_string(p->lighting_mode) + std::to_string(p->shadows_enabled);
    // Motion mode: a camera differs from the previous frame's (any field), so the tile costs go
    // stale quickly.  For kMotionFrames frames from then on, every frame is measured whose previous
    // measurement has completed (adopted without waiting), and split tiles are costed by their
    // split waves (FrameArgs::part_cost).  Otherwise: one measurement every sched_period frames,
    // adopted at the next frame (one host wait per measurement).
    bool moved = c->prev_views != n_views;
    for (int v = 0; !moved && v < n_views; ++v) {
        const ViewCam &a = F.cam[v], &b = c->prev_cam[v];
        moved = std::memcmp(a.origin, b.origin, 12) || std::memcmp(a.right, b.right, 12) ||
                std::memcmp(a.up, b.up, 12) || std::memcmp(a.forward, b.forward, 12) || a.fov != b.fov;
    }
    std::memcpy(c->prev_cam, F.cam, sizeof(ViewCam) * static_cast<size_t>(n_views));
    c->prev_views = n_views;
    // animated geometry (rtx_ctx::upload_motion), where a stale schedule costs: a scene with split
    // tiles (W4_Optional's F6 loop: GPU wait 0.51 -> 0.43 ms).  Without them the per-frame
    // measurement is the larger cost (W4_Bunny's loop 7-10 % slower, W4_Reference's serial 11 %).
    moved = moved || (c->upload_motion && c->heavy_n > 0);
    c->upload_motion = false;
    if (key != c->sched_key) {   // new shape or scene: identity order, fresh costs, no split
        if (c->heavy_pending) HIP_TRY(c, hipEventSynchronize(c->ev_heavy));
        c->heavy_pending = false;
        c->heavy_n = 0;
        c->sched_key = key;
        c->sched_ready = false;
        c->sched_frame = 0;
        c->motion_left = 0;
        c->max_cost_serial = 0;
        if (c->refinable) {   // a new shape refines from the upload's frontier
            if (c->h_parts.size() != c->h_parts_base.size()) {
                if (const int rc = join_split(c); rc != RTX_OK) return rc;
                c->h_parts = c->h_parts_base;
                HIP_TRY(c, hipMemcpyAsync(c->parts_dev, c->h_parts.data(), c->h_parts.size() * sizeof(int4),
                                          hipMemcpyHostToDevice, c->stream));
                HIP_TRY(c, hipStreamSynchronize(c->stream));
                c->dev.n_parts = static_cast<uint32_t>(c->h_parts.size());
            }
            c->refine_round = 0;
            c->refine_state = 0;
            c->refine_wait = 0;
            c->refine_prev_max = 0;
            c->refine_rec = false;
            c->refine_quiet = kRefineQuiet;
        }
        c->win_state = 0;
        c->win_frames = 0;
        c->win_interval_ms = 0.f;
        if (c->tune_on) {   // a new shape: tune again from the default
            c->split_permille = kSplitPermille;
            c->tune_done = false;
            c->tune_steps = 0;
            c->tune_dir = 0;
            c->tune_step = 1.15f;
            c->tune_best_span = 0.f;
            c->tune_best_permille = 0;
        }
        c->tune_rec = false;
        HIP_TRY(c, hipMemsetAsync(c->d_cost, 0, ntiles * 4, c->stream));
    } else if (moved && !c->motion_off) {
        c->motion_left = kMotionFrames;
    }
    const bool motion = c->motion_left > 0;
    if (motion) --c->motion_left;
    c->frame_motion = motion;
    if (c->heavy_pending) {
        bool ready = true;
        if (motion) {   // no host wait: adopt only a measurement that has completed
            const hipError_t q = hipEventQuery(c->ev_heavy);
            (void)hipGetLastError();   // (a not-ready query is no error for the launches' checks)
            if (q != hipSuccess && q != hipErrorNotReady) HIP_TRY(c, q);
            ready = q == hipSuccess;
        } else {
            // adopt the heavy set the last measured frame selected (one sync per measurement)
            HIP_TRY(c, hipEventSynchronize(c->ev_heavy));
        }
        if (ready) {
            c->heavy_pending = false;
            c->heavy_n = std::min<uint32_t>(c->h_heavy_n[0], kMaxHeavyTiles);
            if (!c->concurrent) c->max_cost_serial = c->h_heavy_n[2];
            c->heavy_cur ^= 1;
            // nothing to balance while no tile is heavy at the default factor (the tuner only
            // raises the factor from there when the split chain is the longer)
            if (c->heavy_n == 0 && c->split_permille == kSplitPermille && c->set_permille[c->heavy_cur] == kSplitPermille)
                c->tune_done = true;
            if (c->tune_rec) {   // the measured frame's timings: complete (they precede ev_heavy)
                c->tune_rec = false;
                float mm = 0.f, ch = 0.f;
                HIP_TRY(c, hipEventElapsedTime(&mm, c->ev_tune[0], c->ev_tune[1]));
                HIP_TRY(c, hipEventElapsedTime(&ch, c->ev_tune[0], c->ev_tune[2]));
                c->tune_main_ms = mm;
                c->tune_chain_ms = ch;
                split_tune(c, mm, ch);
            }
        }
    }
    // throughput mode: other contexts' frames in flight on this device (rtx_ctx::ev_frame; asked only
    // where a tile can be split: the other contexts' event queries are not free in a GPU-bound loop)
    const uint32_t others = (!c->throughput_off && c->tune_on && c->split_ok && (c->heavy_n > 0 || !c->tune_done))
                                ? frames_concurrent(c) : 0u;
    c->concurrent = others > 0;
    // in flight: one piece while the heaviest tile is short next to the split frame (kInflightCritPermille)
    c->frame_onepiece = c->concurrent && c->heavy_n > 0 && inflight_onepiece(c, others + 1);
    const bool split = c->split_mode != 0 && c->split_ok && c->sched_enabled && c->heavy_n > 0 && !c->frame_onepiece;
    F.heavy_flag = split ? c->d_heavy_flag[c->heavy_cur] : nullptr;
    F.part_max = nullptr;
    if (c->refine_state == 1) {
        const int rc = refine_round(c);
        if (rc != RTX_OK) return rc;
    }
    if (c->refine_quiet) --c->refine_quiet;
    if (split && c->refine_state == 0 && !motion && c->renders_since_upload >= kRefineQuiet && c->refine_quiet == 0 &&
        (c->refine_wait == 0 || --c->refine_wait == 0)) {
        if (!c->d_part_max) {
            HIP_TRY(c, hipMalloc(&c->d_part_max, 2ull * kMaxParts * kPartShards * sizeof(uint32_t)));
            c->h_part_max.resize(2ull * kMaxParts * kPartShards);
        }
        HIP_TRY(c, hipMemsetAsync(c->d_part_max, 0, 2ull * kMaxParts * kPartShards * sizeof(uint32_t), c->stream));
        F.part_max = c->d_part_max;
        c->refine_rec = true;
    }
    F.heavy_list = c->d_heavy_list[c->heavy_cur];
    F.heavy_n = split ? c->heavy_n : 0u;
    F.hit_key = c->d_hit_key;
    F.occ_bits = c->d_occ;
    // light-major (FrameArgs::lm_*): a launch small enough that its slowest tiles, not its work, set
    // its time (a few tiles per resident wave slot: a stripe share of a frame), with shadows and 2+
    // lights; the deep-stack variants render one piece
    const uint32_t nl = c->dev.n_lights;
    c->frame_lm = F.shadows && nl >= 2 && nl <= kMaxLmLights && !c->deep_stack && !c->hbm_stack &&
                  (c->lm_mode == 2 || (c->lm_mode == 1 && ntiles <= c->lm_tiles));
    if (c->frame_lm) {
        if (ntiles > c->lm_rec_tiles) {
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            (void)hipFree(c->d_lm_rec);
            c->d_lm_rec = nullptr;
            c->lm_rec_tiles = 0;
            HIP_TRY(c, hipMalloc(&c->d_lm_rec, static_cast<size_t>(ntiles) * 64 * 2 * sizeof(float4)));
            c->lm_rec_tiles = ntiles;
        }
        if (static_cast<size_t>(ntiles) * nl > c->lm_mask_cap) {
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            (void)hipFree(c->d_lm_mask);
            c->d_lm_mask = nullptr;
            c->lm_mask_cap = 0;
            HIP_TRY(c, hipMalloc(&c->d_lm_mask, static_cast<size_t>(ntiles) * nl * 8));
            c->lm_mask_cap = static_cast<size_t>(ntiles) * nl;
        }
        F.lm_lights = nl;
        F.lm_rec = c->d_lm_rec;
        F.lm_mask = c->d_lm_mask;
    }
    // Measure tile costs on the first frame of a shape and then every kSchedPeriod frames;
    // the frames in between reuse the last order and pay nothing for scheduling.
    // while the split threshold is being tuned (a scene with split tiles), every other frame is measured
    const bool tuning = c->tune_on && !c->tune_done && c->heavy_n > 0 && c->split_mode == 1 && c->split_ok && !motion &&
                        !c->concurrent;
    const bool measure = c->sched_enabled && !c->heavy_pending &&
                         (!c->sched_ready || motion || c->sched_frame % (tuning ? 2u : c->sched_period) == 0);
    ++c->sched_frame;
    F.order = (c->sched_enabled && c->sched_ready) ? (c->xcd_order ? c->d_order_xcd : c->d_order) : nullptr;
    F.cost = measure ? c->d_cost : nullptr;
    F.part_cost = (measure && motion) ? 1u : 0u;
    return RTX_OK;
}

// Index into kSpecVariants of the first variant the facts satisfy, -1 for none: every kind the
// scene references is compiled into the variant, and every other fact the variant assumes holds.
int spec_variant(int facts) {
    for (int i = 0; i < static_cast<int>(sizeof kSpecVariants / sizeof kSpecVariants[0]); ++i) {
        const int v = kSpecVariants[i], vk = v & kSpecKindAll, fk = facts & kSpecKindAll;
        if ((fk & ~vk) == 0 && ((v & ~kSpecKindAll) & ~facts) == 0) return i;
    }
    return -1;
}

// The split launches of a frame (PHASE 1-3) in the frame's specialised variant v (-1: generic).
template <int P, bool CU>
void launch_phase_v(int v, dim3 g, hipStream_t s, const DevScene& d, const FrameArgs& F) {
    switch (v) {
    case 0: hipLaunchKernelGGL((rtx_render_kernel<false, P, false, kSpecVariants[0], false, CU>), g, dim3(kBlockThreads), 0, s, d, F); break;
    case 1: hipLaunchKernelGGL((rtx_render_kernel<false, P, false, kSpecVariants[1], false, CU>), g, dim3(kBlockThreads), 0, s, d, F); break;
    case 2: hipLaunchKernelGGL((rtx_render_kernel<false, P, false, kSpecVariants[2]>), g, dim3(kBlockThreads), 0, s, d, F); break;   // (no mesh: nothing to cull)
    case 3: hipLaunchKernelGGL((rtx_render_kernel<false, P, false, kSpecVariants[3], false, CU>), g, dim3(kBlockThreads), 0, s, d, F); break;
    case 4: hipLaunchKernelGGL((rtx_render_kernel<false, P, false, kSpecVariants[4], false, CU>), g, dim3(kBlockThreads), 0, s, d, F); break;
    default: hipLaunchKernelGGL((rtx_render_kernel<false, P, false, 0, false, CU>), g, dim3(kBlockThreads), 0, s, d, F); break;
    }
}
// PHASE P of a frame in the frame's specialised variant v (-1: generic), with the cull variant
// when the scene has cull records
template <int P>
void launch_phase(int v, dim3 g, hipStream_t s, const DevScene& d, const FrameArgs& F) {
    if (d.cull_stride) launch_phase_v<P, true>(v, g, s, d, F);
    else launch_phase_v<P, false>(v, g, s, d, F);
}

// The HBM stacks of the HSTK variant: max_depth + 1 entries for each wave of a launch of
// `groups` workgroups (sized per launch: a wave's index in it selects its stack).
int ensure_hbm_stacks(rtx_ctx* c, uint32_t groups) {
    const size_t depth = static_cast<size_t>(c->max_depth) + 1u;
    const size_t need = static_cast<size_t>(groups) * kWavesPerBlock * depth;
    constexpr size_t kEntryBytes = sizeof(uint4) + sizeof(unsigned long long);
    if (need * kEntryBytes > (size_t(64) << 30))
        return fail(c, RTX_E_UNSUPPORTED, "DFS stacks of a " + std::to_string(c->max_depth) + "-level BVH for this frame exceed 64 GB");
    if (need > c->hstk_entries) {
        (void)hipFree(c->d_hstk);
        (void)hipFree(c->d_hstkT);
        c->d_hstk = nullptr;
        c->d_hstkT = nullptr;
        c->hstk_entries = 0;
        HIP_TRY(c, hipMalloc(&c->d_hstk, need * sizeof(uint4)));
        HIP_TRY(c, hipMalloc(&c->d_hstkT, need * sizeof(unsigned long long)));
        c->hstk_entries = need;
    }
    c->dev.hstk = c->d_hstk;
    c->dev.hstkT = c->d_hstkT;
    c->dev.hstk_depth = static_cast<uint32_t>(depth);
    return RTX_OK;
}

// count: 1 = the reference's traversal counted (the instrumented kernel), 2 = the culled walk's
// executed tests (its counting variant, rtx_count_work_culled; the plain one without records)
int launch(rtx_ctx* c, const FrameArgs& F, dim3 grid, int count) {
    if (grid.x == 0 || grid.y == 0) return RTX_OK;
    // (prepare joined already unless this frame repeats the last one's parameters and cameras)
    const bool inflight_join = c->concurrent && (!c->defer_inflight || c->win_state == 2 || c->win_state == 3);
    if (c->join_pending && (count || F.cost || F.part_max || F.lm_lights || inflight_join || c->hbm_stack ||
                            c->deep_stack || F.heavy_flag != c->join_heavy || F.heavy_n != c->join_heavy_n)) {
        const int rc = join_split(c);
        if (rc != RTX_OK) return rc;
    }
    if (c->hbm_stack) {
        const int rc = ensure_hbm_stacks(c, grid.x);
        if (rc != RTX_OK) return rc;
    }
    if (count) {
        FrameArgs G = F;   // the instrumented variant neither reads nor feeds the schedule
        G.order = nullptr;
        G.cost = nullptr;
        G.heavy_flag = nullptr;
        if (count == 2 && c->dev.cull_stride && !c->hbm_stack && !c->deep_stack) {
            const int rc = cull_views(c, F);   // the views' camera records, as a frame would
            if (rc != RTX_OK) return rc;
            hipLaunchKernelGGL((rtx_render_kernel<true, 0, false, 0, false, true>), grid, dim3(kBlockThreads), 0,
                               c->stream, c->dev, G);
        } else if (c->hbm_stack)
            hipLaunchKernelGGL((rtx_render_kernel<true, 0, true, 0, true>), grid, dim3(kBlockThreads), 0, c->stream, c->dev, G);
        else if (c->deep_stack)
            hipLaunchKernelGGL((rtx_render_kernel<true, 0, true>), grid, dim3(kBlockThreads), 0, c->stream, c->dev, G);
        else
            hipLaunchKernelGGL((rtx_render_kernel<true, 0>), grid, dim3(kBlockThreads), 0, c->stream, c->dev, G);
        HIP_TRY(c, hipGetLastError());
        return RTX_OK;
    }
    ++c->renders_since_upload;
    if (c->dev.cull_stride) {   // the views' camera-anchor cull records, when a camera moved
        const int rc = cull_views(c, F);
        if (rc != RTX_OK) return rc;
    }
    // the first specialised variant whose facts the scene and frame satisfy (kSpecVariants;
    // RTX_NO_SPEC=1 forces the generic kernel); the split launches take it too
    const int facts = c->scene_spec | ((F.mode == RTX_MODE_COMBINED && F.shadows) ? kSpecCombShadows : 0);
    const int v = (c->no_spec || c->deep_stack) ? -1 : spec_variant(facts);
    if (F.heavy_flag) {
        // The heavy tiles, one BVH frontier part per workgroup (see the kernel), on a
        // high-priority stream forked from the frame stream: they share no pixels with the
        // main kernel, so the two run side by side and the join closes the frame.
        const uint32_t nh = (c->heavy_n + kWavesPerBlock - 1) / kWavesPerBlock, np = c->dev.n_parts;   // heavy wave tiles per workgroup
        hipStream_t s2 = c->split_stream;
        // split_tune: static cameras only (a moving one changes the frame under the measurement)
        const bool timed = F.cost && c->tune_on && !c->tune_done && c->split_mode == 1 && !c->frame_motion && !c->concurrent;
        if (timed) HIP_TRY(c, hipEventRecord(c->ev_tune[0], c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_fork, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(s2, c->ev_fork, 0));
        if (!RTX_ABL_CHAIN) {
            launch_phase<1>(v, dim3(nh, np, 1), s2, c->dev, F);
            HIP_TRY(c, hipGetLastError());
            if (F.shadows && c->dev.n_lights) {
                launch_phase<2>(v, dim3(nh, np, c->dev.n_lights), s2, c->dev, F);
                HIP_TRY(c, hipGetLastError());
            }
            launch_phase<3>(v, dim3(nh, 1, 1), s2, c->dev, F);
            HIP_TRY(c, hipGetLastError());
        }
        if (timed) {   // (before ev_join: the frame's completion then implies this event's)
            HIP_TRY(c, hipEventRecord(c->ev_tune[2], s2));
            c->tune_rec = true;
            c->tune_rec_permille = c->set_permille[c->heavy_cur];
        }
        HIP_TRY(c, hipEventRecord(c->ev_join, s2));
    }
    if (c->hbm_stack)   // (the deep variants walk without the cull)
        hipLaunchKernelGGL((rtx_render_kernel<false, 0, true, 0, true>), grid, dim3(kBlockThreads), 0, c->stream, c->dev, F);
    else if (c->deep_stack)
        hipLaunchKernelGGL((rtx_render_kernel<false, 0, true>), grid, dim3(kBlockThreads), 0, c->stream, c->dev, F);
    else if (F.lm_lights) {   // light-major: hit records, then the (tile, light) waves
        launch_phase<4>(v, grid, c->stream, c->dev, F);
        HIP_TRY(c, hipGetLastError());
        // persistent light waves: one per resident wave slot (at most one per item)
        const uint32_t items = F.n_tiles * F.lm_lights, waves = std::min(items, c->lm_waves);
        launch_phase<5>(v, dim3((waves + kWavesPerBlock - 1) / kWavesPerBlock), c->stream, c->dev, F);
        HIP_TRY(c, hipGetLastError());
        launch_phase<6>(v, grid, c->stream, c->dev, F);
    } else if (!(RTX_ABL_MAIN && F.heavy_flag && !F.cost))
        launch_phase<0>(v, grid, c->stream, c->dev, F);
    HIP_TRY(c, hipGetLastError());
    if (F.heavy_flag && c->tune_rec && F.cost) HIP_TRY(c, hipEventRecord(c->ev_tune[1], c->stream));
    if (F.heavy_flag) {
        // a plain repeat of the frame defers the join to the next frame or reader (rtx_ctx::join_pending);
        // a measured, tuned, refined or in-flight one joins now
        if (F.cost || F.part_max || inflight_join || c->join_off || c->tune_rec || c->refine_rec) {
            HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
        } else {
            c->join_pending = true;
            c->join_heavy = F.heavy_flag;
            c->join_heavy_n = F.heavy_n;
        }
    }
    if (F.cost) {
        const uint32_t slots = (c->split_mode == 0 || !c->split_ok) ? 0u
                               : (c->split_mode == 2 ? 0xffffffffu : c->split_slots);
        const int stage = c->heavy_cur ^ 1;
        // (throughput mode: at least kThroughputPermille, see rtx_ctx::ev_frame)
        const uint32_t permille = c->concurrent ? std::max<uint32_t>(c->split_permille, kThroughputPermille)
                                                : c->split_permille;
        c->set_permille[stage] = permille;
        const uint32_t nch = (F.n_tiles + kSchedChunk - 1) / kSchedChunk;
        hipLaunchKernelGGL(rtx_sched_count, dim3(nch), dim3(kReorderThreads), 0, c->stream, F.cost, F.n_tiles,
                           F.heavy_flag, c->d_saved_cost, c->d_hist, c->d_csum, nch, F.part_cost, c->d_heavy_n + 1);
        HIP_TRY(c, hipGetLastError());
        hipLaunchKernelGGL(rtx_sched_scan, dim3(1), dim3(kScanThreads), 0, c->stream, c->d_hist, nch,
                           c->d_csum,
                           F.n_tiles, slots, permille, c->split_min, c->split_slots, c->d_thr, c->d_heavy_n);
        HIP_TRY(c, hipGetLastError());
        hipLaunchKernelGGL(rtx_sched_scatter, dim3(nch), dim3(kReorderThreads), 0, c->stream, F.cost, c->d_order,
                           F.n_tiles, c->d_hist, nch, c->d_thr, slots == 0xffffffffu ? 1u : 0u,
                           c->d_heavy_flag[stage], c->d_heavy_list[stage], c->d_heavy_n);
        HIP_TRY(c, hipGetLastError());
        if (c->xcd_order) {
            hipLaunchKernelGGL(rtx_sched_xcd, dim3(1), dim3(kScanThreads), 0, c->stream, c->d_order, c->d_order_xcd,
                               F.n_tiles, F.tiles_x, F.tiles_y);
            HIP_TRY(c, hipGetLastError());
        }
        HIP_TRY(c, hipMemcpyAsync(c->h_heavy_n, c->d_heavy_n, 16, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_heavy, c->stream));
        c->heavy_pending = true;
        c->sched_ready = true;
    }
    // the frame's end, for other contexts' throughput mode (prepare).  Only a context whose tiles can
    // be split records it: one that has nothing to split (no frontier, or no heavy tile at a converged
    // factor: W4_Bunny) skips the event and the registry's lock on every frame.
    const bool tracked = c->split_ok && c->split_mode != 0 && !(c->heavy_n == 0 && c->tune_done);
    if (c->win_rec >= 0) HIP_TRY(c, hipEventRecord(c->ev_win[c->win_rec], c->stream));
    if (c->refine_rec) {   // the measured frame's end (its chain joined): its part statistics are complete
        HIP_TRY(c, hipEventRecord(c->ev_refine, c->stream));
        c->refine_rec = false;
        c->refine_state = 1;
    }
    if (tracked) {
        HIP_TRY(c, hipEventRecord(c->ev_frame, c->stream));
        if (!c->in_registry) {
            frames_note(c);
            c->in_registry = true;
        }
    } else if (c->in_registry) {
        frames_forget(c);
        c->in_registry = false;
    }
    return RTX_OK;
}

void remember(rtx_ctx* c, const rtx_render_params* p, int n_views, bool rgb) {
    c->last = *p;
    c->last_views = n_views;
    c->last_valid = true;
    c->last_rgb = rgb;
}

}  // namespace

extern "C" int rtx_render_views_async(rtx_ctx* c, const rtx_camera* cams, int n_views, const rtx_render_params* p,
                                      int want_rgb) {
    FrameArgs F;
    dim3 grid;
    int rc = prepare(c, cams, n_views, p, want_rgb != 0, F, grid);
    if (rc != RTX_OK) return rc;
    rc = launch(c, F, grid, 0);
    if (rc != RTX_OK) return rc;
    remember(c, p, n_views, want_rgb != 0);
    return RTX_OK;
}

extern "C" int rtx_render_async(rtx_ctx* c, const rtx_camera* cam, const rtx_render_params* p, int want_rgb) {
    return rtx_render_views_async(c, cam, 1, p, want_rgb);
}

extern "C" int rtx_synchronize(rtx_ctx* c) {
    if (!c) return RTX_E_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    if (const int rc = join_split(c); rc != RTX_OK) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return RTX_OK;
}

namespace {

// Queue the D2H copy of the rows the last render owns (every view) into the caller's
// full-frame host buffers, on the context stream.  A striped frame is one
// hipMemcpy2DAsync per view and plane: `stripe_rows` rows every `stripe_step` stripes
// (row pitch of the 2-D copy = stripe_step stripes), plus the trailing partial stripe.
int queue_owned_copy(rtx_ctx* c, uint32_t* out_px, float* out_rgb) {
    if (!c || !out_px) return RTX_E_INVALID;
    if (!c->last_valid) return fail(c, RTX_E_STATE, "nothing rendered yet");
    if (out_rgb && !c->last_rgb) return fail(c, RTX_E_STATE, "last render did not produce colours");
    const rtx_render_params& p = c->last;
    HIP_TRY(c, hipSetDevice(c->device));
    if (const int rc = join_split(c); rc != RTX_OK) return rc;
    const size_t W = p.width, H = p.height;
    const bool striped = p.stripe_rows != 0 && p.stripe_step > 1;
    for (int v = 0; v < c->last_views; ++v) {
        const size_t base = static_cast<size_t>(v) * W * H;
        if (!striped) {
            HIP_TRY(c, hipMemcpyAsync(out_px + base, c->d_px + base, W * H * 4, hipMemcpyDeviceToHost, c->stream));
            if (out_rgb)
                HIP_TRY(c, hipMemcpyAsync(out_rgb + 3 * base, c->d_rgb + 3 * base, W * H * 12, hipMemcpyDeviceToHost,
                                          c->stream));
            continue;
        }
        const size_t rows = p.stripe_rows, step = p.stripe_step;
        const size_t first = (p.stripe_first + step - static_cast<uint32_t>(v) % step) % step;
        // owned stripes s = first + k*step; the full ones end at or before row H
        size_t n_full = 0;
        if ((first + 1) * rows <= H) n_full = ((H / rows) - 1 - first) / step + 1;
        const size_t last = first + n_full * step;   // next owned stripe (maybe partial or past H)
        struct Plane { char* dst; const char* src; size_t elem; };
        const Plane planes[2] = {{reinterpret_cast<char*>(out_px), reinterpret_cast<const char*>(c->d_px), 4},
                                 {reinterpret_cast<char*>(out_rgb), reinterpret_cast<const char*>(c->d_rgb), 12}};
        for (const Plane& pl : planes) {
            if (!pl.dst) continue;
            const size_t row_b = W * pl.elem, off = (base + first * rows * W) * pl.elem;
            if (n_full)
                HIP_TRY(c, hipMemcpy2DAsync(pl.dst + off, step * rows * row_b, pl.src + off, step * rows * row_b,
                                            rows * row_b, n_full, hipMemcpyDeviceToHost, c->stream));
            if (last * rows < H) {
                const size_t o2 = (base + last * rows * W) * pl.elem;
                HIP_TRY(c, hipMemcpyAsync(pl.dst + o2, pl.src + o2, (H - last * rows) * row_b, hipMemcpyDeviceToHost,
                                          c->stream));
            }
        }
    }
    return RTX_OK;
}

}  // namespace

extern "C" int rtx_download(rtx_ctx* c, uint32_t* out_px, float* out_rgb) {
    const int rc = queue_owned_copy(c, out_px, out_rgb);
    if (rc != RTX_OK) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return RTX_OK;
}

extern "C" int rtx_gather_async(rtx_ctx* c, uint32_t* out_px, float* out_rgb) {
    return queue_owned_copy(c, out_px, out_rgb);
}

extern "C" int rtx_host_register(rtx_ctx* c, void* p, size_t bytes) {
    if (!c || !p || !bytes) return RTX_E_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipHostRegister(p, bytes, hipHostRegisterPortable));
    return RTX_OK;
}

extern "C" int rtx_host_unregister(rtx_ctx* c, void* p) {
    if (!c || !p) return RTX_E_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipHostUnregister(p));
    return RTX_OK;
}

extern "C" int rtx_render(rtx_ctx* c, const rtx_camera* cam, const rtx_render_params* p, uint32_t* out_px,
                          float* out_rgb) {
    if (!out_px) return RTX_E_INVALID;
    int rc = rtx_render_async(c, cam, p, out_rgb != nullptr);
    if (rc != RTX_OK) return rc;
    return rtx_download(c, out_px, out_rgb);
}

extern "C" int rtx_device_buffers(rtx_ctx* c, void** d_px, void** d_rgb) {
    if (!c) return RTX_E_INVALID;
    if (const int rc = join_split(c); rc != RTX_OK) return rc;   // (the caller orders its work after the stream)
    if (d_px) *d_px = c->d_px;
    if (d_rgb) *d_rgb = c->d_rgb;
    return RTX_OK;
}

extern "C" int rtx_time_views(rtx_ctx* c, const rtx_camera* cams, int n_views, const rtx_render_params* p, int iters,
                              float* mean_ms) {
    if (!mean_ms || iters <= 0) return RTX_E_INVALID;
    FrameArgs F;
    dim3 grid;
    // every launch is prepared like a real frame: the first frame of a launch shape measures
    // tile costs, the next ones run in the cost order (and split the heavy tiles) it yields,
    // and every kSchedPeriod-th frame measures again
    int rc = prepare(c, cams, n_views, p, false, F, grid);
    if (rc != RTX_OK) return rc;
    HIP_TRY(c, hipEventRecord(c->ev0, c->stream));
    for (int i = 0; i < iters; ++i) {
        if (i > 0) {
            remember(c, p, n_views, false);
            rc = prepare(c, cams, n_views, p, false, F, grid);
            if (rc != RTX_OK) return rc;
        }
        rc = launch(c, F, grid, false);
        if (rc != RTX_OK) return rc;
    }
    if (const int rc2 = join_split(c); rc2 != RTX_OK) return rc2;   // (the last chain inside the timing)
    HIP_TRY(c, hipEventRecord(c->ev1, c->stream));
    HIP_TRY(c, hipEventSynchronize(c->ev1));
    float ms = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    *mean_ms = ms / static_cast<float>(iters);
    remember(c, p, n_views, false);
    return RTX_OK;
}

extern "C" int rtx_time_frames(rtx_ctx* c, const rtx_camera* cam, const rtx_render_params* p, int iters,
                               float* mean_ms) {
    return rtx_time_views(c, cam, 1, p, iters, mean_ms);
}

// Instrumented variant: the same traversal with per-lane work counters.
namespace {
int count_work(rtx_ctx* c, const rtx_camera* cam, const rtx_render_params* p, uint64_t* counts, int n_counts,
               int mode);
}

extern "C" int rtx_count_work_ex(rtx_ctx* c, const rtx_camera* cam, const rtx_render_params* p, uint64_t* counts,
                                 int n_counts) {
    return count_work(c, cam, p, counts, n_counts, 1);
}

extern "C" int rtx_count_work(rtx_ctx* c, const rtx_camera* cam, const rtx_render_params* p, uint64_t* counts) {
    return count_work(c, cam, p, counts, kModelCounters, 1);
}

extern "C" int rtx_count_work_culled(rtx_ctx* c, const rtx_camera* cam, const rtx_render_params* p, uint64_t* counts,
                                     int n_counts) {
    return count_work(c, cam, p, counts, n_counts, 2);
}

namespace {
// The counters of one render (mode 1: the reference's traversal; 2: the culled walk's executed
// tests), up to kNumCounters values: the kModelCounters of the FLOP model, then the per-wave
// diagnostics and the cull tests.
int count_work(rtx_ctx* c, const rtx_camera* cam, const rtx_render_params* p, uint64_t* counts, int n_counts,
               int mode) {
    if (!counts || n_counts <= 0) return RTX_E_INVALID;
    if (n_counts > kNumCounters) n_counts = kNumCounters;
    FrameArgs F;
    dim3 grid;
    int rc = prepare(c, cam, 1, p, false, F, grid);
    if (rc != RTX_OK) return rc;
    HIP_TRY(c, hipMemsetAsync(c->d_counters, 0, sizeof(unsigned long long) * kNumCounters, c->stream));
    rc = launch(c, F, grid, mode);
    if (rc != RTX_OK) return rc;
    unsigned long long tmp[kNumCounters];
    HIP_TRY(c, hipMemcpyAsync(tmp, c->d_counters, sizeof(unsigned long long) * kNumCounters, hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < n_counts; ++k) counts[k] = tmp[k];
    remember(c, p, 1, false);
    return RTX_OK;
}
}  // namespace

extern "C" int rtx_schedule_state(rtx_ctx* c, uint32_t* order, uint32_t* cost, uint32_t n, uint32_t* n_tiles) {
    if (!c) return RTX_E_INVALID;
    if (n_tiles) *n_tiles = c->sched_ready ? c->sched_cap : 0u;
    if (!c->sched_ready || !order || !cost) return RTX_OK;
    if (n > c->sched_cap) return fail(c, RTX_E_INVALID, "n exceeds the schedule size");
    HIP_TRY(c, hipSetDevice(c->device));
    if (const int rc = join_split(c); rc != RTX_OK) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(order, c->d_order, n * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(cost, c->d_saved_cost, n * 4, hipMemcpyDeviceToHost));
    return RTX_OK;
}

extern "C" int rtx_cull_info(rtx_ctx* c, uint32_t* enabled, uint64_t* camera_updates) {
    if (!c) return RTX_E_INVALID;
    if (enabled) *enabled = c->dev.cull_stride ? 1u : 0u;
    if (camera_updates) *camera_updates = c->cull_updates;
    return RTX_OK;
}

extern "C" int rtx_cull_dump(rtx_ctx* c, uint32_t anchor, uint32_t* n_slots, uint32_t* n_tris, float* anchor_p,
                             float* records, uint32_t* ranges, float* nodes, float* tris) {
    if (!c || anchor >= static_cast<uint32_t>(kMaxViews + kMaxCullLights)) return RTX_E_INVALID;
    if (!c->dev.cull_stride) return fail(c, RTX_E_INVALID, "the uploaded scene has no cull records");
    if (n_slots) *n_slots = c->cull_nslots;
    if (n_tris) *n_tris = c->cull_ntris;
    if (anchor_p) std::memcpy(anchor_p, c->cull_anchor[anchor], sizeof c->cull_anchor[anchor]);
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const size_t ns = c->cull_nslots;
    if (records)
        HIP_TRY(c, hipMemcpy(records, reinterpret_cast<const char*>(c->dev.cull) + static_cast<size_t>(anchor) * c->dev.cull_stride,
                             ns * 32, hipMemcpyDeviceToHost));
    if (ranges) HIP_TRY(c, hipMemcpy(ranges, c->cull_rng, ns * 8, hipMemcpyDeviceToHost));
    if (nodes) HIP_TRY(c, hipMemcpy(nodes, c->dev.nodes, ns * 32, hipMemcpyDeviceToHost));
    if (tris) HIP_TRY(c, hipMemcpy(tris, c->dev.tris, static_cast<size_t>(c->cull_ntris) * 64, hipMemcpyDeviceToHost));
    return RTX_OK;
}

extern "C" int rtx_split_tune_info(rtx_ctx* c, float* factor, float* main_ms, float* chain_ms, uint32_t* done) {
    if (!c) return RTX_E_INVALID;
    if (factor) *factor = static_cast<float>(c->split_permille) / 1000.f;
    if (main_ms) *main_ms = c->tune_main_ms;
    if (chain_ms) *chain_ms = c->tune_chain_ms;
    if (done) *done = (!c->tune_on ? 2u : (c->tune_done ? 1u : 0u));
    return RTX_OK;
}

extern "C" int rtx_inflight_info(rtx_ctx* c, uint32_t* concurrent, uint32_t* onepiece, float* crit,
                                 float* crit_threshold, float* split_interval_ms) {
    if (!c) return RTX_E_INVALID;
    if (split_interval_ms) *split_interval_ms = c->win_interval_ms;
    if (concurrent) *concurrent = c->concurrent ? 1u : 0u;
    if (onepiece) *onepiece = c->frame_onepiece ? 1u : 0u;
    if (crit) *crit = inflight_ratio(c);
    if (crit_threshold) *crit_threshold = static_cast<float>(c->inflight_crit) / 1000.f;
    return RTX_OK;
}

extern "C" int rtx_light_major_info(rtx_ctx* c, uint32_t* last_frame, uint32_t* max_tiles) {
    if (!c) return RTX_E_INVALID;
    if (last_frame) *last_frame = c->frame_lm ? 1u : 0u;
    if (max_tiles) *max_tiles = c->lm_mode == 0 ? 0u : (c->lm_mode == 2 ? 0xffffffffu : c->lm_tiles);
    return RTX_OK;
}

extern "C" int rtx_split_info(rtx_ctx* c, uint32_t* heavy_tiles, uint32_t* parts) {
    if (!c) return RTX_E_INVALID;
    if (c->heavy_pending) {   // a measured frame is in flight: report the set it selects
        HIP_TRY(c, hipSetDevice(c->device));
        HIP_TRY(c, hipEventSynchronize(c->ev_heavy));
    }
    const uint32_t n = c->heavy_pending ? std::min<uint32_t>(c->h_heavy_n[0], kMaxHeavyTiles) : c->heavy_n;
    const bool on = c->split_mode != 0 && c->split_ok && c->sched_enabled;
    if (heavy_tiles) *heavy_tiles = on ? n : 0u;
    if (parts) *parts = c->split_ok ? c->dev.n_parts : 0u;
    return RTX_OK;
}

#if RTX_STAMPS
// Diagnostic build only: render once with per-wave {start, end, hw ids} stamps.
extern "C" int rtx_debug_stamps(rtx_ctx* c, const rtx_camera* cam, const rtx_render_params* p, uint64_t* out,
                                uint64_t capacity, uint64_t* n_waves) {
    FrameArgs F;
    dim3 grid;
    int rc = prepare(c, cam, 1, p, false, F, grid);
    if (rc != RTX_OK) return rc;
    const uint64_t nw = F.n_tiles;   // one record per wave tile
    *n_waves = nw;
    if (kStampWords * nw > capacity) return RTX_E_INVALID;
    if (kStampWords * nw + 6 * kMaxParts > capacity) return RTX_E_INVALID;
    unsigned long long* d = nullptr;
    // + per (phase 1/2, part, shard) {sum, max, steps}, reduced over the shards below
    const size_t words = kStampWords * nw + 6 * kMaxParts * kStampShards;
    HIP_TRY(c, hipMalloc(&d, words * 8));
    HIP_TRY(c, hipMemsetAsync(d, 0, words * 8, c->stream));
    F.stamps = d;
    F.split_stamps = d + kStampWords * nw;
    rc = launch(c, F, grid, false);
    if (rc != RTX_OK) return rc;
    rc = join_split(c);
    if (rc != RTX_OK) return rc;
    HIP_TRY(c, hipMemcpyAsync(out, d, kStampWords * nw * 8, hipMemcpyDeviceToHost, c->stream));
    std::vector<unsigned long long> sh(6 * kMaxParts * kStampShards);
    HIP_TRY(c, hipMemcpyAsync(sh.data(), d + kStampWords * nw, sh.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    (void)hipFree(d);
    for (size_t k = 0; k < 2u * kMaxParts; ++k) {
        unsigned long long sum = 0, mx = 0, steps = 0;
        for (int j = 0; j < kStampShards; ++j) {
            const unsigned long long* x = sh.data() + 3 * (k * kStampShards + j);
            sum += x[0];
            mx = std::max(mx, x[1]);
            steps += x[2];
        }
        out[kStampWords * nw + 3 * k] = sum;
        out[kStampWords * nw + 3 * k + 1] = mx;
        out[kStampWords * nw + 3 * k + 2] = steps;
    }
    return RTX_OK;
}
#endif

// Diagnostics: a copy of the context's current scene image (after its queued work).
extern "C" int rtx_scene_image(rtx_ctx* c, void* out, size_t capacity, size_t* bytes) {
    if (!c || !bytes) return RTX_E_INVALID;
    if (!c->has_scene) return fail(c, RTX_E_STATE, "no scene uploaded");
    *bytes = c->scene_bytes;
    if (!out) return RTX_OK;
    if (capacity < c->scene_bytes) return fail(c, RTX_E_INVALID, "capacity below the image size");
    HIP_TRY(c, hipSetDevice(c->device));
    if (const int rc = join_split(c); rc != RTX_OK) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(out, c->sb[c->sb_cur].d, c->scene_bytes, hipMemcpyDeviceToHost));
    return RTX_OK;
}
