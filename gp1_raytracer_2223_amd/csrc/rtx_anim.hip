// rtx_anim.hip — Scene::Update for animated meshes on the device (see rtx_anim.h).
//
// One 1024-thread workgroup per mesh.  The build tree is grown level by level (one barrier
// per level); each node of a level is handled by one wave:
//   * FindBestSplitPlane (DataTypes.h:398-483): centroid bounds, 8 bins per live axis, the
//     7-plane SAH sweep with the reference's float expressions and quirks (0.3333f
//     centroids, centroid max starting at FLT_MIN, 0 * inf = NaN costs for empty sides);
//   * the partition (DataTypes.h:343-363) as a parallel scatter that lands every triangle
//     exactly where the serial swap loop leaves it (derivation below);
//   * UpdateNodeBounds (:310-321) of both children.
// Every min/max is a fold in the reference's order: each lane folds a contiguous chunk
// in order and lanes are combined left to right, so std::min / std::max's "first
// occurrence wins a tie" is kept (only a signed zero can observe it).  The tree is then
// numbered as the reference's recursion allocates it (children pairs in DFS preorder of the
// splits), and the mesh is written into the scene image in rtx_upload_scene's layout.
// Built with the render library's flags (-ffp-contract=off, correctly rounded div/sqrt).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <type_traits>

#include "rtx_anim.h"
#include "rtx_kernels.h"

namespace rtxa {
namespace {

__device__ __forceinline__ float rmin(float m, float x) { return (x < m) ? x : m; }   // std::min(m, x)
__device__ __forceinline__ float rmax(float m, float x) { return (m < x) ? x : m; }   // std::max(m, x)
__device__ __forceinline__ float fbits(uint32_t u) { return __uint_as_float(u); }

// Matrix::TransformPoint / TransformVector (Matrix.cpp:35-56), m = rows data[0..3] (xyz):
// left-to-right sums of products, no contraction.
__device__ __forceinline__ float3 xform_point(const float* m, float x, float y, float z) {
    return make_float3(m[0] * x + m[3] * y + m[6] * z + m[9], m[1] * x + m[4] * y + m[7] * z + m[10],
                       m[2] * x + m[5] * y + m[8] * z + m[11]);
}
__device__ __forceinline__ float3 xform_vector(const float* m, float x, float y, float z) {
    return make_float3(m[0] * x + m[3] * y + m[6] * z, m[1] * x + m[4] * y + m[7] * z,
                       m[2] * x + m[5] * y + m[8] * z);
}
__device__ __forceinline__ float3 normalized(float3 v) {   // Vector3::Normalized (Vector3.cpp:42-46)
    const float m = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return make_float3(v.x / m, v.y / m, v.z / m);
}
__device__ __forceinline__ float area(const float lo[3], const float hi[3]) {   // AABB::Area
    const float ex = hi[0] - lo[0], ey = hi[1] - lo[1], ez = hi[2] - lo[2];
    return ex * ey + ey * ez + ez * ex;
}

// The build arrays by triangle id and the two permutation buffers, in the workgroup's LDS
// (meshes up to kLdsTris triangles) or in HBM (MeshDev::soa / perm): generic pointers.
template <class S>   // S: the partition scratch type (16-bit in LDS, 32-bit in HBM)
struct Arr {
    float *cx, *cy, *cz;         // centroid (v0 + v1 + v2) * 0.3333f
    float *lx, *ly, *lz;         // triangle box min(min(v0, v1), v2)
    float *hx, *hy, *hz;         //              max(max(v0, v1), v2)
    uint32_t* perm[2];           // build position -> triangle id
    S *lb, *rs, *rk;             // partition scratch: left bigs / right smalls by rank, rank by position
    __device__ float c(int ax, uint32_t id) const { return ax == 0 ? cx[id] : (ax == 1 ? cy[id] : cz[id]); }
};

struct Bounds {
    float l0 = FLT_MAX, l1 = FLT_MAX, l2 = FLT_MAX, h0 = FLT_MIN, h1 = FLT_MIN, h2 = FLT_MIN;
    template <class AR>
    __device__ void grow(const AR& A, uint32_t id) {   // UpdateNodeBounds over one triangle
        l0 = rmin(l0, A.lx[id]); l1 = rmin(l1, A.ly[id]); l2 = rmin(l2, A.lz[id]);
        h0 = rmax(h0, A.hx[id]); h1 = rmax(h1, A.hy[id]); h2 = rmax(h2, A.hz[id]);
    }
    __device__ void store(float mn[3], float mx[3]) const {
        mn[0] = l0; mn[1] = l1; mn[2] = l2; mx[0] = h0; mx[1] = h1; mx[2] = h2;
    }
};

// A team: G consecutive lanes of one wave handle one node (G = 64: the whole wave; G = 16:
// one DPP row, four nodes per wave).  Control flow is uniform within a team (trip counts
// depend only on the node), so team reductions and ballots see every lane of the team.
template <int G>
struct Team {
    static_assert(G == 16 || G == 64, "teams are DPP rows or whole waves");
    uint32_t tl, tb;   // lane within the team, the team's first lane in the wave
    __device__ explicit Team(uint32_t lane) : tl(lane % G), tb(lane - lane % G) {}
    __device__ unsigned long long ballot(bool p) const {
        const unsigned long long b = __ballot(p);
        return G == 64 ? b : (b >> tb) & ((1ull << G) - 1ull);
    }
    __device__ uint32_t below(unsigned long long m) const { return __popcll(m & ((1ull << tl) - 1ull)); }
    // contiguous chunk [s, e) of positions [a, a + n) for this lane: folds stay in order
    __device__ void chunk(uint32_t a, uint32_t n, uint32_t& s, uint32_t& e) const {
        const uint32_t c = (n + G - 1u) / G;
        s = a + min(n, tl * c);
        e = a + min(n, tl * c + c);
    }
};

// In-order team folds without LDS round trips: DPP row_shl:n (lane i reads lane i + n of its
// row; a source beyond the row yields the fold identity) halves the row in four steps, lane 16r
// ending with the in-order fold of row r; rows are combined in order from v_readlane values
// (G = 64) or the row fold is broadcast with row_newbcast:0 (G = 16).  Every result is the
// team's fold, in every lane of the team.
template <int N>
__device__ __forceinline__ uint32_t dpp_shl(uint32_t v, uint32_t identity) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(identity), static_cast<int>(v),
                                                             0x100 + N, 0xf, 0xf, false));
}
__device__ __forceinline__ uint32_t dpp_row_bcast0(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x150, 0xf, 0xf, false));
}
struct OpMin {
    static constexpr float kId = FLT_MAX;
    __device__ static float f(float m, float x) { return rmin(m, x); }
};
struct OpMax {
    static constexpr float kId = FLT_MIN;
    __device__ static float f(float m, float x) { return rmax(m, x); }
};
template <int G, class Op>
__device__ __forceinline__ float team_fold(float v) {
    const uint32_t id = __float_as_uint(Op::kId);
    v = Op::f(v, __uint_as_float(dpp_shl<1>(__float_as_uint(v), id)));
    v = Op::f(v, __uint_as_float(dpp_shl<2>(__float_as_uint(v), id)));
    v = Op::f(v, __uint_as_float(dpp_shl<4>(__float_as_uint(v), id)));
    v = Op::f(v, __uint_as_float(dpp_shl<8>(__float_as_uint(v), id)));
    if (G == 16) return __uint_as_float(dpp_row_bcast0(__float_as_uint(v)));
    const uint32_t u = __float_as_uint(v);
    const float r0 = __uint_as_float(__builtin_amdgcn_readlane(u, 0)), r1 = __uint_as_float(__builtin_amdgcn_readlane(u, 16));
    const float r2 = __uint_as_float(__builtin_amdgcn_readlane(u, 32)), r3 = __uint_as_float(__builtin_amdgcn_readlane(u, 48));
    return Op::f(Op::f(Op::f(r0, r1), r2), r3);
}
template <int G>
__device__ __forceinline__ uint32_t team_sum(uint32_t v) {
    v += dpp_shl<1>(v, 0u);
    v += dpp_shl<2>(v, 0u);
    v += dpp_shl<4>(v, 0u);
    v += dpp_shl<8>(v, 0u);
    if (G == 16) return dpp_row_bcast0(v);
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}
template <int G>
__device__ __forceinline__ Bounds team_fold(const Bounds& B) {
    Bounds R;
    R.l0 = team_fold<G, OpMin>(B.l0); R.l1 = team_fold<G, OpMin>(B.l1); R.l2 = team_fold<G, OpMin>(B.l2);
    R.h0 = team_fold<G, OpMax>(B.h0); R.h1 = team_fold<G, OpMax>(B.h1); R.h2 = team_fold<G, OpMax>(B.h2);
    return R;
}

// Bounds of the triangle boxes at build positions [a, b) (UpdateNodeBounds: a triangle's box
// min(min(v0, v1), v2) grows a node exactly as its three vertices in order do), every lane.
template <int G, class AR>
__device__ __forceinline__ Bounds team_bounds(const Team<G>& tm, const AR& A, const uint32_t* perm, uint32_t a,
                                              uint32_t b) {
    Bounds B;
    uint32_t s, e;
    tm.chunk(a, b - a, s, e);
#pragma unroll 4
    for (uint32_t k = s; k < e; ++k) B.grow(A, perm[k]);
    return team_fold<G>(B);
}

constexpr int kBins = 8, kPlanes = kBins - 1;

// One axis's 8 bins: idxCount and the box of the triangles' vertices, folded in order.
struct Bins {
    float bl[kBins][3], bh[kBins][3];
    uint32_t bc[kBins];
    __device__ void clear() {
#pragma unroll
        for (int q = 0; q < kBins; ++q) {
            bl[q][0] = bl[q][1] = bl[q][2] = FLT_MAX;
            bh[q][0] = bh[q][1] = bh[q][2] = FLT_MIN;
            bc[q] = 0u;
        }
    }
    template <class AR>
    __device__ void add(const AR& A, uint32_t id, int ax, float minBounds, float scale) {
        const float x = (A.c(ax, id) - minBounds) * scale;
        // static_cast<int> of x >= 0 (a NaN x only comes from a NaN vertex: flagged, bin 0)
        int bi = x >= 0.f ? static_cast<int>(fminf(x, 2147483520.f)) : 0;
        bi = kPlanes < bi ? kPlanes : bi;   // std::min(amountOfPlaneBins, binIdx)
        const float lx = A.lx[id], ly = A.ly[id], lz = A.lz[id], hx = A.hx[id], hy = A.hy[id], hz = A.hz[id];
        // branch-free: the other bins see their fold identity (FLT_MAX for a min that starts at
        // FLT_MAX, FLT_MIN for a max that starts at FLT_MIN), which leaves them bit-unchanged;
        // per-bin branches get merged into a pointer select and the bins into scratch memory
#pragma unroll
        for (int q = 0; q < kBins; ++q) {
            const bool h = bi == q;
            bc[q] += h ? 3u : 0u;
            bl[q][0] = rmin(bl[q][0], h ? lx : FLT_MAX);
            bl[q][1] = rmin(bl[q][1], h ? ly : FLT_MAX);
            bl[q][2] = rmin(bl[q][2], h ? lz : FLT_MAX);
            bh[q][0] = rmax(bh[q][0], h ? hx : FLT_MIN);
            bh[q][1] = rmax(bh[q][1], h ? hy : FLT_MIN);
            bh[q][2] = rmax(bh[q][2], h ? hz : FLT_MIN);
        }
    }
    // the plane sweep (DataTypes.h:444-480), AABBs starting at {MaxVector, MinVector}
    __device__ void sweep(int ax, float minBounds, float boundsDifference, float& bestCost, int& axis,
                          float& pos) const {
        float leftArea[kPlanes], rightArea[kPlanes];
        int leftCount[kPlanes], rightCount[kPlanes];
        int leftSum = 0, rightSum = 0;
        float llo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, lhi[3] = {FLT_MIN, FLT_MIN, FLT_MIN};
        float rlo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, rhi[3] = {FLT_MIN, FLT_MIN, FLT_MIN};
#pragma unroll
        for (int i = 0; i < kPlanes; ++i) {
            leftSum += static_cast<int>(bc[i]);
            leftCount[i] = leftSum;
            #pragma unroll
            for (int c = 0; c < 3; ++c) { llo[c] = rmin(llo[c], bl[i][c]); lhi[c] = rmax(lhi[c], bh[i][c]); }
            leftArea[i] = area(llo, lhi);
            rightSum += static_cast<int>(bc[kPlanes - i]);
            rightCount[kPlanes - i - 1] = rightSum;
            #pragma unroll
            for (int c = 0; c < 3; ++c) {
                rlo[c] = rmin(rlo[c], bl[kPlanes - i][c]);
                rhi[c] = rmax(rhi[c], bh[kPlanes - i][c]);
            }
            rightArea[kPlanes - i - 1] = area(rlo, rhi);
        }
        const float step = boundsDifference / kBins;
#pragma unroll
        for (int i = 0; i < kPlanes; ++i) {
            const float planeCost = static_cast<float>(leftCount[i]) * leftArea[i] +
                                    static_cast<float>(rightCount[i]) * rightArea[i];
            if (planeCost < bestCost) {
                axis = ax;
                pos = minBounds + step * static_cast<float>(i + 1);
                bestCost = planeCost;
            }
        }
    }
};

// Centroid bounds of positions [a, b): min from FLT_MAX, max from FLT_MIN (the reference's
// minBounds / maxBounds, DataTypes.h:404-419), the three axes in one fold, every lane.
template <int G, class AR>
__device__ __forceinline__ Bounds team_centroid_bounds(const Team<G>& tm, const AR& A, const uint32_t* perm,
                                                       uint32_t a, uint32_t b) {
    Bounds C;
    uint32_t s, e;
    tm.chunk(a, b - a, s, e);
#pragma unroll 4
    for (uint32_t k = s; k < e; ++k) {
        const uint32_t id = perm[k];
        const float x = A.cx[id], y = A.cy[id], z = A.cz[id];
        C.l0 = rmin(C.l0, x); C.l1 = rmin(C.l1, y); C.l2 = rmin(C.l2, z);
        C.h0 = rmax(C.h0, x); C.h1 = rmax(C.h1, y); C.h2 = rmax(C.h2, z);
    }
    return team_fold<G>(C);
}

// One axis's bins over positions [a, b), every lane.
template <int G, class AR>
__device__ __forceinline__ void team_bins(const Team<G>& tm, const AR& A, const uint32_t* perm, uint32_t a,
                                          uint32_t b, int ax, float minBounds, float scale, Bins& bins) {
    bins.clear();
    uint32_t s, e;
    tm.chunk(a, b - a, s, e);
#pragma unroll 2
    for (uint32_t k = s; k < e; ++k) bins.add(A, perm[k], ax, minBounds, scale);
#pragma unroll
    for (int q = 0; q < kBins; ++q) {
        bins.bc[q] = team_sum<G>(bins.bc[q]);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            bins.bl[q][c] = team_fold<G, OpMin>(bins.bl[q][c]);
            bins.bh[q][c] = team_fold<G, OpMax>(bins.bh[q][c]);
        }
    }
}

// FindBestSplitPlane (DataTypes.h:398-483) for the node at [a, a + n) by one team: the best
// cost (FLT_MAX when no axis is live) with axis / pos, uniform over the team.
template <int G, class AR>
__device__ __forceinline__ float team_best_split(const Team<G>& tm, const AR& A, const uint32_t* perm, uint32_t a,
                                                 uint32_t n, int& axis, float& pos) {
    const Bounds C = team_centroid_bounds(tm, A, perm, a, a + n);
    const float cl[3] = {C.l0, C.l1, C.l2}, ch[3] = {C.h0, C.h1, C.h2};
    float bestCost = FLT_MAX;
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
        const float minBounds = cl[ax];
        const float boundsDifference = ch[ax] - minBounds;
        if (fabsf(boundsDifference) < FLT_EPSILON) continue;
        Bins bins;
        team_bins(tm, A, perm, a, a + n, ax, minBounds, kBins / boundsDifference, bins);
        bins.sweep(ax, minBounds, boundsDifference, bestCost, axis, pos);   // the same in every lane
    }
    return bestCost;
}

// The serial swap loop (DataTypes.h:343-363, in triangle units) on a node of n triangles
// with flags big(q) = !(centroid[axis] < splitPos) examines the left stream q = 0, 1, ...
// and, after each big element, the right stream n-1, n-2, ... until it meets a small one.
// With S small elements in all it ends with i = S, and the left stream covered [0, pL),
// pL = S + big(S) (a big element at S is the meeting point).  Closed form (checked against
// the loop exhaustively on random flag patterns):
//   small q < pL            stays at q
//   m-th big q < pL         -> n-1 (m = 0) or (position of the (m-1)-th right small) - 1
//   m-th small p >= pL      -> position of the m-th left big   (right smalls counted from the end)
//   big p >= pL             -> p - 1
// The ranks of positions [lo, hi) are assigned with the rank bases lbase / rbase (the counts
// of left bigs before lo / right smalls after hi): one team, or one wave of a workgroup.
template <int G, class AR>
__device__ __forceinline__ void team_ranks(const Team<G>& tm, const AR& A, const uint32_t* src, const MeshDev& M,
                                           uint32_t first, uint32_t lo, uint32_t hi, uint32_t pL, int axis,
                                           float pos, uint32_t lbase, uint32_t rbase) {
    auto small = [&](uint32_t q) { return A.c(axis, src[first + q]) < pos; };
    uint32_t carry = lbase;
    const uint32_t lhi = min(hi, pL);
    for (uint32_t base = lo; base < lhi; base += G) {   // left-stream bigs, in order
        const uint32_t q = base + tm.tl;
        const bool b = q < lhi && !small(q);
        const unsigned long long m = tm.ballot(b);
        if (b) {
            const uint32_t r = carry + tm.below(m);
            A.lb[first + r] = q;
            A.rk[first + q] = r;
        }
        carry += __popcll(m);
    }
    carry = rbase;
    const uint32_t rlo = max(lo, pL);
    for (uint32_t top = hi; top > rlo;) {   // right-stream smalls, from the end
        const uint32_t cnt = min(static_cast<uint32_t>(G), top - rlo);
        const bool in = tm.tl < cnt;
        const uint32_t p = in ? top - 1u - tm.tl : 0u;
        const bool sm = in && small(p);
        const unsigned long long m = tm.ballot(sm);
        if (sm) {
            const uint32_t r = carry + tm.below(m);
            A.rs[first + r] = p;
            A.rk[first + p] = r;
        }
        carry += __popcll(m);
        top -= cnt;
    }
}
// Destination of position q once every rank is known.
template <class AR>
__device__ __forceinline__ uint32_t part_dest(const AR& A, uint32_t first, uint32_t n, uint32_t q, uint32_t pL,
                                              bool big) {
    if (q < pL) {
        if (!big) return q;
        const uint32_t m = A.rk[first + q];
        return m == 0u ? n - 1u : static_cast<uint32_t>(A.rs[first + m - 1u]) - 1u;
    }
    return big ? q - 1u : static_cast<uint32_t>(A.lb[first + A.rk[first + q]]);
}
template <int G, class AR>
__device__ __forceinline__ uint32_t team_count_small(const Team<G>& tm, const AR& A, const uint32_t* src,
                                                     uint32_t first, uint32_t lo, uint32_t hi, int axis, float pos) {
    uint32_t S = 0;
    for (uint32_t base = lo; base < hi; base += G) {
        const uint32_t q = base + tm.tl;
        S += __popcll(tm.ballot(q < hi && A.c(axis, src[first + q]) < pos));
    }
    return S;
}
template <int G, class AR>
__device__ __forceinline__ void team_partition(const Team<G>& tm, const AR& A, const uint32_t* src, uint32_t* dst,
                                               const MeshDev& M, uint32_t first, uint32_t n, int axis, float pos,
                                               uint32_t& S_out) {
    const uint32_t S = team_count_small(tm, A, src, first, 0u, n, axis, pos);
    const uint32_t pL = S + ((S < n && !(A.c(axis, src[first + S]) < pos)) ? 1u : 0u);
    team_ranks(tm, A, src, M, first, 0u, n, pL, axis, pos, 0u, 0u);
    __threadfence_block();
    for (uint32_t q = tm.tl; q < n; q += G) {
        const uint32_t id = src[first + q];
        dst[first + part_dest(A, first, n, q, pL, !(A.c(axis, id) < pos))] = id;
    }
    __threadfence_block();
    S_out = S;
}

template <int G>
__device__ __forceinline__ void team_copy(const Team<G>& tm, const uint32_t* src, uint32_t* dst, uint32_t first,
                                          uint32_t n) {
    for (uint32_t q = tm.tl; q < n; q += G) dst[first + q] = src[first + q];
    __threadfence_block();
}

// Node classes by size: huge nodes are processed by the whole workgroup one at a time, large
// ones by a wave, small ones by a 16-lane row, tiny ones by one lane each (a large node of up
// to 2,048 triangles folds up to 32 positions per lane: waves working on different nodes side
// by side beat the serial whole-workgroup path there).
#ifndef RTX_ANIM_HUGE
#define RTX_ANIM_HUGE 2048   // above this a node takes the whole workgroup (512 measured 15 % slower)
#endif
constexpr uint32_t kHugeNode = RTX_ANIM_HUGE, kLargeNode = 64, kTinyNode = 8;
__device__ __forceinline__ uint32_t node_class(uint32_t n) {
    return n > kHugeNode ? 0u : (n > kLargeNode ? 1u : (n > kTinyNode ? 2u : 3u));
}

// Shared state of one build (LDS): per class the node count of the current level and the
// append counter of the next one.
struct Lists {
    uint32_t n[4], next[4], ntmp, depth, err;
};

// Children of a split node: temp ids, and entries in the next level's list of their class.
__device__ __forceinline__ void add_children(const MeshDev& M, Lists& Ls, uint32_t cl, uint32_t t, uint32_t first,
                                             uint32_t n, uint32_t S, uint32_t depth, const float lmn[3],
                                             const float lmx[3], const float rmn[3], const float rmx[3]) {
    const uint32_t c = atomicAdd(&Ls.ntmp, 2u);
    TmpNode a{}, b{};
    for (int q = 0; q < 3; ++q) { a.mn[q] = lmn[q]; a.mx[q] = lmx[q]; b.mn[q] = rmn[q]; b.mx[q] = rmx[q]; }
    a.first = first; a.count = S; a.l = -1; a.depth = depth + 1;
    b.first = first + S; b.count = n - S; b.l = -1; b.depth = depth + 1;
    M.tmp[c] = a;
    M.tmp[c + 1] = b;
    M.tmp[t].l = static_cast<int32_t>(c);
    for (uint32_t h = 0; h < 2; ++h) {
        const uint32_t k = node_class(h ? n - S : S);
        const uint32_t w = atomicAdd(&Ls.next[k], 1u);
        M.lvl[2 * k + (cl ^ 1u)][w] = c + h;
    }
}

// One node by one team of G lanes (a wave, or a 16-lane row).
template <int G, class AR>
__device__ __forceinline__ void team_node(const Team<G>& tm, const AR& A, uint32_t* src, uint32_t* dst,
                                          const MeshDev& M, Lists& Ls, uint32_t cl, uint32_t t, uint32_t depth) {
    const TmpNode X = M.tmp[t];
    const uint32_t n = X.count;
    int axis = 0;
    float pos = 0.f;
    const float splitCost = team_best_split(tm, A, src, X.first, n, axis, pos);
    const float noSplitCost = static_cast<float>(3u * n) * area(X.mn, X.mx);   // CalculateNodeCost
    if (splitCost >= noSplitCost) {
        team_copy(tm, src, dst, X.first, n);
        return;
    }
    uint32_t S = 0;
    team_partition(tm, A, src, dst, M, X.first, n, axis, pos, S);
    if (S == 0u || S == n) {   // leftCount 0 or all: a leaf, with the permutation applied
        team_copy(tm, dst, src, X.first, n);
        return;
    }
    const Bounds Lb = team_bounds(tm, A, dst, X.first, X.first + S);
    const Bounds Rb = team_bounds(tm, A, dst, X.first + S, X.first + n);
    if (tm.tl == 0) {
        float lmn[3], lmx[3], rmn[3], rmx[3];
        Lb.store(lmn, lmx);
        Rb.store(rmn, rmx);
        add_children(M, Ls, cl, t, X.first, n, S, depth, lmn, lmx, rmn, rmx);
    }
}

// Workgroup scratch for a node processed by every wave (huge nodes): per-wave partial folds,
// combined in wave order.
struct WgScratch {
    float b[kAnimWaves][6];                    // bounds / centroid bounds
    float bins[kAnimWaves][kBins * 7];         // one axis's bins: count, lo xyz, hi xyz
    uint32_t cnt[kAnimWaves][2];
};

__device__ __forceinline__ void wg_store_bounds(WgScratch& W, uint32_t wave, const Bounds& B) {
    W.b[wave][0] = B.l0; W.b[wave][1] = B.l1; W.b[wave][2] = B.l2;
    W.b[wave][3] = B.h0; W.b[wave][4] = B.h1; W.b[wave][5] = B.h2;
}
__device__ __forceinline__ Bounds wg_fold_bounds(const WgScratch& W) {   // waves in order
    Bounds B;
#pragma unroll
    for (int w = 0; w < kAnimWaves; ++w) {
        B.l0 = rmin(B.l0, W.b[w][0]); B.l1 = rmin(B.l1, W.b[w][1]); B.l2 = rmin(B.l2, W.b[w][2]);
        B.h0 = rmax(B.h0, W.b[w][3]); B.h1 = rmax(B.h1, W.b[w][4]); B.h2 = rmax(B.h2, W.b[w][5]);
    }
    return B;
}

// One huge node by the whole workgroup: wave w takes the w-th contiguous eighth of the range.
template <class AR>
__device__ void wg_node(const AR& A, uint32_t* src, uint32_t* dst, const MeshDev& M, Lists& Ls, WgScratch& W,
                        uint32_t cl, uint32_t t, uint32_t depth, uint32_t tid) {
    const uint32_t lane = tid & 63u, wave = tid >> 6;
    const Team<64> tm(lane);
    const TmpNode X = M.tmp[t];
    const uint32_t n = X.count, first = X.first;
    const uint32_t per = (n + kAnimWaves - 1u) / kAnimWaves;
    const uint32_t lo = min(n, wave * per), hi = min(n, wave * per + per);   // this wave's eighth
    // centroid bounds
    {
        const Bounds C = team_centroid_bounds(tm, A, src, first + lo, first + hi);
        if (lane == 0) wg_store_bounds(W, wave, C);
    }
    __syncthreads();
    const Bounds C = wg_fold_bounds(W);
    const float cl3[3] = {C.l0, C.l1, C.l2}, ch3[3] = {C.h0, C.h1, C.h2};
    float bestCost = FLT_MAX, pos = 0.f;
    int axis = 0;
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
        const float minBounds = cl3[ax];
        const float boundsDifference = ch3[ax] - minBounds;
        if (fabsf(boundsDifference) < FLT_EPSILON) continue;   // uniform
        Bins bins;
        team_bins(tm, A, src, first + lo, first + hi, ax, minBounds, kBins / boundsDifference, bins);
        __syncthreads();   // the previous axis's partials are consumed
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < kBins; ++q) {
                W.bins[wave][7 * q] = __uint_as_float(bins.bc[q]);
#pragma unroll
                for (int c = 0; c < 3; ++c) { W.bins[wave][7 * q + 1 + c] = bins.bl[q][c]; W.bins[wave][7 * q + 4 + c] = bins.bh[q][c]; }
            }
        }
        __syncthreads();
        Bins all;
        all.clear();
#pragma unroll
        for (int w = 0; w < kAnimWaves; ++w) {
#pragma unroll
            for (int q = 0; q < kBins; ++q) {
                all.bc[q] += __float_as_uint(W.bins[w][7 * q]);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    all.bl[q][c] = rmin(all.bl[q][c], W.bins[w][7 * q + 1 + c]);
                    all.bh[q][c] = rmax(all.bh[q][c], W.bins[w][7 * q + 4 + c]);
                }
            }
        }
        all.sweep(ax, minBounds, boundsDifference, bestCost, axis, pos);
    }
    const float noSplitCost = static_cast<float>(3u * n) * area(X.mn, X.mx);
    if (bestCost >= noSplitCost) {   // uniform: every thread folded the same partials
        for (uint32_t q = tid; q < n; q += kAnimThreads) dst[first + q] = src[first + q];
        return;   // the caller's barrier publishes dst
    }
    // partition: S, then each wave's left bigs / right smalls, rank bases, ranks, scatter
    {
        const uint32_t s = team_count_small(tm, A, src, first, lo, hi, axis, pos);
        if (lane == 0) W.cnt[wave][0] = s;
    }
    __syncthreads();
    uint32_t S = 0;
#pragma unroll
    for (int w = 0; w < kAnimWaves; ++w) S += W.cnt[w][0];
    const uint32_t pL = S + ((S < n && !(A.c(axis, src[first + S]) < pos)) ? 1u : 0u);
    __syncthreads();   // cnt is reused
    {
        uint32_t nl = 0, nr = 0;
        for (uint32_t base = lo; base < hi; base += 64u) {
            const uint32_t q = base + lane;
            const bool in = q < hi;
            const bool sm = in && A.c(axis, src[first + q]) < pos;
            nl += __popcll(tm.ballot(in && q < pL && !sm));
            nr += __popcll(tm.ballot(in && q >= pL && sm));
        }
        if (lane == 0) { W.cnt[wave][0] = nl; W.cnt[wave][1] = nr; }
    }
    __syncthreads();
    uint32_t lbase = 0, rbase = 0;
#pragma unroll
    for (int w = 0; w < kAnimWaves; ++w) {
        if (static_cast<uint32_t>(w) < wave) lbase += W.cnt[w][0];
        if (static_cast<uint32_t>(w) > wave) rbase += W.cnt[w][1];
    }
    team_ranks(tm, A, src, M, first, lo, hi, pL, axis, pos, lbase, rbase);
    __syncthreads();
    for (uint32_t q = tid; q < n; q += kAnimThreads) {
        const uint32_t id = src[first + q];
        dst[first + part_dest(A, first, n, q, pL, !(A.c(axis, id) < pos))] = id;
    }
    __syncthreads();
    if (S == 0u || S == n) {
        for (uint32_t q = tid; q < n; q += kAnimThreads) src[first + q] = dst[first + q];
        return;
    }
    // children's bounds: each wave's part of [first, first + S) and of [first + S, first + n)
    float mn[2][3], mx[2][3];
    for (int h = 0; h < 2; ++h) {
        const uint32_t a0 = h ? S : 0u, a1 = h ? n : S;
        const uint32_t pw = (a1 - a0 + kAnimWaves - 1u) / kAnimWaves;
        const uint32_t l0 = min(a1, a0 + wave * pw), l1 = min(a1, a0 + wave * pw + pw);
        const Bounds B = team_bounds(tm, A, dst, first + l0, first + l1);
        __syncthreads();
        if (lane == 0) wg_store_bounds(W, wave, B);
        __syncthreads();
        wg_fold_bounds(W).store(mn[h], mx[h]);
    }
    if (tid == 0) add_children(M, Ls, cl, t, first, n, S, depth, mn[0], mx[0], mn[1], mx[1]);
}

// One node of at most kTinyNode triangles by ONE lane: the reference's own serial passes
// (bounds folds, bins, sweep, the swap loop itself), in place on `src`, then copied to `dst`
// so that both permutation buffers hold the range.
template <class AR>
__device__ __forceinline__ void lane_node(const AR& A, uint32_t* src, uint32_t* dst, const MeshDev& M, Lists& Ls, uint32_t cl,
                          uint32_t t, uint32_t depth) {
    const TmpNode X = M.tmp[t];
    const uint32_t first = X.first, n = X.count;
    bool leaf = 3u * n <= 8u;
    int axis = 0;
    float pos = 0.f;
    if (!leaf) {
        float cl3[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, ch3[3] = {FLT_MIN, FLT_MIN, FLT_MIN};
#pragma unroll 4
        for (uint32_t k = 0; k < n; ++k) {
            const uint32_t id = src[first + k];
            const float x = A.cx[id], y = A.cy[id], z = A.cz[id];
            cl3[0] = rmin(cl3[0], x); cl3[1] = rmin(cl3[1], y); cl3[2] = rmin(cl3[2], z);
            ch3[0] = rmax(ch3[0], x); ch3[1] = rmax(ch3[1], y); ch3[2] = rmax(ch3[2], z);
        }
        float bestCost = FLT_MAX;
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
            const float minBounds = cl3[ax];
            const float boundsDifference = ch3[ax] - minBounds;
            if (fabsf(boundsDifference) < FLT_EPSILON) continue;
            const float scale = kBins / boundsDifference;
            Bins bins;
            bins.clear();
#pragma unroll 2
            for (uint32_t k = 0; k < n; ++k) bins.add(A, src[first + k], ax, minBounds, scale);
            bins.sweep(ax, minBounds, boundsDifference, bestCost, axis, pos);
        }
        const float noSplitCost = static_cast<float>(3u * n) * area(X.mn, X.mx);   // CalculateNodeCost
        leaf = bestCost >= noSplitCost;
    }
    uint32_t S = n;
    if (!leaf) {   // DataTypes.h:343-363 on this node's range
        int i = 0, j = static_cast<int>(n) - 1;
        while (i <= j) {
            const uint32_t id = src[first + i];
            if (A.c(axis, id) < pos) {
                ++i;
            } else {
                src[first + i] = src[first + j];
                src[first + j] = id;
                --j;
            }
        }
        S = static_cast<uint32_t>(i);
    }
#pragma unroll 4
    for (uint32_t k = 0; k < n; ++k) dst[first + k] = src[first + k];
    if (leaf || S == 0u || S == n) return;
    Bounds L, R;
#pragma unroll 4
    for (uint32_t k = 0; k < S; ++k) L.grow(A, src[first + k]);
#pragma unroll 4
    for (uint32_t k = S; k < n; ++k) R.grow(A, src[first + k]);
    float lmn[3], lmx[3], rmn[3], rmx[3];
    L.store(lmn, lmx);
    R.store(rmn, rmx);
    add_children(M, Ls, cl, t, first, n, S, depth, lmn, lmx, rmn, rmx);
}

// LDS = true: the build arrays live in the workgroup's LDS (every mesh of the launch fits),
// so the compiler sees LDS pointers and emits ds_read / ds_write instead of flat accesses.
template <bool LDS>
__global__ void __launch_bounds__(kAnimThreads) rtx_anim_build(const Launch L) {
    const MeshDev& M = L.meshes[blockIdx.x];
    const float* mat = L.m[blockIdx.x];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t T = M.T, V = M.V;
    const int4* idx = M.idx[L.cur];
    const float4* nrm = M.nrm[L.cur];
    extern __shared__ float s_dyn[];
    __shared__ Lists Ls;
    __shared__ uint32_t s_fr[kMaxAnimParts][3];
    __shared__ uint32_t s_nfr;
    // build arrays: in LDS when every mesh of the launch fits (LDS), else in HBM
    using Scratch = std::conditional_t<LDS, uint16_t, uint32_t>;
    Arr<Scratch> A;
    {
        float* base = LDS ? s_dyn : M.soa;
        A.cx = base; A.cy = base + T; A.cz = base + 2 * T;
        A.lx = base + 3 * T; A.ly = base + 4 * T; A.lz = base + 5 * T;
        A.hx = base + 6 * T; A.hy = base + 7 * T; A.hz = base + 8 * T;
        A.perm[0] = LDS ? reinterpret_cast<uint32_t*>(s_dyn + 9 * T) : M.perm[0];
        A.perm[1] = LDS ? reinterpret_cast<uint32_t*>(s_dyn + 10 * T) : M.perm[1];
        uint16_t* s16 = reinterpret_cast<uint16_t*>(s_dyn + 11 * T);
        A.lb = LDS ? reinterpret_cast<Scratch*>(s16) : reinterpret_cast<Scratch*>(M.lb);
        A.rs = LDS ? reinterpret_cast<Scratch*>(s16 + T) : reinterpret_cast<Scratch*>(M.rs);
        A.rk = LDS ? reinterpret_cast<Scratch*>(s16 + 2 * T) : reinterpret_cast<Scratch*>(M.rk);
    }
    // diagnostic phase stamps (s_memrealtime, 100 MHz): status[8] start, [9] set-up done,
    // [10 + d] level d done, [60] numbered, [61] written, [62] frontier done
    auto stamp = [&](int slot) {
        if (tid == 0) M.status[slot] = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
    };
    stamp(8);
    __shared__ WgScratch W;
    if (tid == 0) {
        for (int q = 0; q < 4; ++q) { Ls.n[q] = 0; Ls.next[q] = 0; }
        Ls.n[node_class(T)] = 1;
        Ls.ntmp = 1; Ls.depth = 0; Ls.err = 0;
    }

    // ---- UpdateTransforms (DataTypes.h:210-230)
    for (uint32_t v = tid; v < V; v += kAnimThreads) {
        const float4 p = M.pos[v];
        const float3 t = xform_point(mat, p.x, p.y, p.z);
        M.tpos[v] = make_float4(t.x, t.y, t.z, 0.f);
    }
    __syncthreads();
    // per triangle: transformed normal (input order), centroid, box
    for (uint32_t k = tid; k < T; k += kAnimThreads) {
        const float4 n = nrm[k];
        const float3 tn = normalized(xform_vector(mat, n.x, n.y, n.z));
        M.tnrm[k] = make_float4(tn.x, tn.y, tn.z, 0.f);
        const int4 i = idx[k];
        const float4 v0 = M.tpos[i.x], v1 = M.tpos[i.y], v2 = M.tpos[i.z];
        if (v0.x != v0.x || v0.y != v0.y || v0.z != v0.z || v1.x != v1.x || v1.y != v1.y || v1.z != v1.z ||
            v2.x != v2.x || v2.y != v2.y || v2.z != v2.z)
            atomicOr(&Ls.err, kErrNaN);
        // (v0 + v1 + v2) * 0.3333f, the reference's centroid (DataTypes.h:348, 411-415, 435)
        A.cx[k] = ((v0.x + v1.x) + v2.x) * 0.3333f;
        A.cy[k] = ((v0.y + v1.y) + v2.y) * 0.3333f;
        A.cz[k] = ((v0.z + v1.z) + v2.z) * 0.3333f;
        A.lx[k] = rmin(rmin(v0.x, v1.x), v2.x); A.ly[k] = rmin(rmin(v0.y, v1.y), v2.y); A.lz[k] = rmin(rmin(v0.z, v1.z), v2.z);
        A.hx[k] = rmax(rmax(v0.x, v1.x), v2.x); A.hy[k] = rmax(rmax(v0.y, v1.y), v2.y); A.hz[k] = rmax(rmax(v0.z, v1.z), v2.z);
        A.perm[0][k] = k;
    }
    __syncthreads();
    // ---- BuildBVH (DataTypes.h:294-308): the root covers every triangle (its bounds: each
    // wave folds its eighth, the eighths are folded in order)
    {
        const Team<64> tm(lane);
        const uint32_t per = (T + kAnimWaves - 1u) / kAnimWaves;
        const Bounds B = team_bounds(tm, A, A.perm[0], min(T, wave * per), min(T, wave * per + per));
        if (lane == 0) wg_store_bounds(W, wave, B);
    }
    __syncthreads();
    if (tid == 0) {
        TmpNode r{};
        wg_fold_bounds(W).store(r.mn, r.mx);
        r.first = 0; r.count = T; r.l = -1; r.depth = 0;
        M.tmp[0] = r;
        M.lvl[2 * node_class(T)][0] = 0;
    }
    __syncthreads();
    stamp(9);
    // ---- Subdivide (DataTypes.h:323-389), one level per iteration, each node by a team
    // sized to it (node_class)
    uint32_t cr = 0, cl = 0;
    for (uint32_t depth = 0;; ++depth) {
        const uint32_t n0 = Ls.n[0], n1 = Ls.n[1], n2 = Ls.n[2], n3 = Ls.n[3];
        if (n0 + n1 + n2 + n3 == 0) break;
        uint32_t* src = cr ? A.perm[1] : A.perm[0];   // (selects: a dynamic index would put A in scratch)
        uint32_t* dst = cr ? A.perm[0] : A.perm[1];
        if (tid == 0 && depth < 12) {   // diagnostics: node count per class at this level
            M.status[64 + 4 * depth] = n0; M.status[65 + 4 * depth] = n1;
            M.status[66 + 4 * depth] = n2; M.status[67 + 4 * depth] = n3;
        }
        for (uint32_t j = 0; j < n0; ++j) {
            wg_node(A, src, dst, M, Ls, W, cl, M.lvl[0 + cl][j], depth, tid);
            __syncthreads();
        }
        if (tid == 0 && depth < 12) M.status[112 + depth] = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
        {
            const Team<64> tm(lane);
            for (uint32_t j = wave; j < n1; j += kAnimWaves) team_node(tm, A, src, dst, M, Ls, cl, M.lvl[2 + cl][j], depth);
        }
        {
            const Team<16> tm(lane);
            constexpr uint32_t kTeams = kAnimThreads / 16;
            for (uint32_t j = tid / 16u; j < n2; j += kTeams) team_node(tm, A, src, dst, M, Ls, cl, M.lvl[4 + cl][j], depth);
        }
        for (uint32_t j = tid; j < n3; j += kAnimThreads) lane_node(A, src, dst, M, Ls, cl, M.lvl[6 + cl][j], depth);
        __syncthreads();
        if (tid == 0) {
            uint32_t any = 0;
            for (int q = 0; q < 4; ++q) { Ls.n[q] = Ls.next[q]; Ls.next[q] = 0; any += Ls.n[q]; }
            if (any) Ls.depth = depth + 1;
            if (depth < 50) M.status[10 + depth] = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
        }
        __syncthreads();
        cr ^= 1u;
        cl ^= 1u;
    }
    // ---- the reference's numbering: split nodes' children pairs in DFS preorder of the splits
    const uint32_t ntmp = Ls.ntmp, maxd = Ls.depth;
    for (int d = static_cast<int>(maxd); d >= 0; --d) {
        for (uint32_t t = tid; t < ntmp; t += kAnimThreads) {
            const TmpNode& X = M.tmp[t];
            if (X.depth != static_cast<uint32_t>(d)) continue;
            M.tmp[t].splits = X.l >= 0 ? 1u + M.tmp[X.l].splits + M.tmp[X.l + 1].splits : 0u;
        }
        __syncthreads();
    }
    if (tid == 0) { M.tmp[0].rank = 0; M.tmp[0].ref = 0; }
    __syncthreads();
    for (uint32_t d = 0; d <= maxd; ++d) {
        for (uint32_t t = tid; t < ntmp; t += kAnimThreads) {
            const TmpNode X = M.tmp[t];
            if (X.depth != d || X.l < 0) continue;
            const uint32_t r = X.rank;
            M.tmp[X.l].ref = 1u + 2u * r;
            M.tmp[X.l + 1].ref = 2u + 2u * r;
            M.tmp[X.l].rank = r + 1u;
            M.tmp[X.l + 1].rank = r + 1u + M.tmp[X.l].splits;
        }
        __syncthreads();
    }
    stamp(60);
    // ---- outputs: the reference's node array (fields the reference writes), the render
    // layout's node records (+ octant copies), the permuted state and triangle records
    const Image& I = L.img;
    for (uint32_t t = tid; t < ntmp; t += kAnimThreads) {
        const TmpNode X = M.tmp[t];
        rtx_bvh_node& R = M.ref[X.ref];
        #pragma unroll
        for (int c = 0; c < 3; ++c) { R.min[c] = X.mn[c]; R.max[c] = X.mx[c]; }
        R.first_idx = 3u * X.first;
        const bool split = X.l >= 0;
        R.idx_count = split ? 0u : 3u * X.count;
        if (split) R.left_node = M.tmp[X.l].ref;
        else if (t == 0) R.left_node = 0u;   // BuildBVH resets the root's leftNode
        const uint32_t link = split ? (M.root + M.tmp[X.l].ref) * 32u : (M.tri0 + X.first) * 64u;
        const float4 a = make_float4(X.mn[0], X.mx[0], X.mn[1], X.mx[1]);
        const float4 b = make_float4(X.mn[2], X.mx[2], fbits(link), fbits(split ? 0u : X.count));
        const size_t slot = static_cast<size_t>(M.root) + X.ref;
        const int copies = I.oct_bytes ? 8 : 1;
        for (int k = 0; k < copies; ++k) {   // copy k stores (hi, lo) on the axes set in k
            float4* dn = reinterpret_cast<float4*>(reinterpret_cast<char*>(I.nodes) + static_cast<size_t>(k) * I.oct_bytes);
            const bool sx = k & 1, sy = k & 2, sz = k & 4;
            dn[2 * slot] = make_float4(sx ? a.y : a.x, sx ? a.x : a.y, sy ? a.w : a.z, sy ? a.z : a.w);
            dn[2 * slot + 1] = make_float4(sz ? b.y : b.x, sz ? b.x : b.y, b.z, b.w);
        }
    }
    const uint32_t* fin = A.perm[0];   // every leaf range is current in both buffers
    int4* idx_out = M.idx[L.cur ^ 1u];
    float4* nrm_out = M.nrm[L.cur ^ 1u];
    for (uint32_t k = tid; k < T; k += kAnimThreads) {
        const uint32_t id = fin[k];
        const int4 i = idx[id];
        const float4 tn = M.tnrm[id];
        idx_out[k] = i;
        nrm_out[k] = nrm[id];
        M.tnrm_out[k] = tn;
        const float4 v0 = M.tpos[i.x], v1 = M.tpos[i.y], v2 = M.tpos[i.z];
        float4* tr = I.tris + 4 * (static_cast<size_t>(M.tri0) + k);
        tr[0] = make_float4(v0.x, v0.y, v0.z, tn.x);
        tr[1] = make_float4(v1.x - v0.x, v1.y - v0.y, v1.z - v0.z, tn.y);   // edge1 (Utils.h:139)
        tr[2] = make_float4(v2.x - v0.x, v2.y - v0.y, v2.z - v0.z, tn.z);   // edge2 (:140)
        tr[3] = make_float4(fbits(M.mat_bits), 0.f, 0.f, 0.f);
    }
    __syncthreads();
    stamp(61);
    // ---- split-rendering frontier (rtx_hip.hip build_parts): split the part with the most
    // triangles (first one on a tie) until part_cap parts or only leaves remain
    if (wave == 0) {
        if (lane == 0) { s_fr[0][0] = 0; s_fr[0][1] = 0; s_fr[0][2] = 0; s_nfr = 1; }
        __builtin_amdgcn_wave_barrier();
        for (;;) {
            const uint32_t nf = s_nfr;
            if (nf >= M.part_cap) break;
            uint32_t key = 0, at = ~0u;   // count + 1 of an eligible entry (0: none), its index
            for (uint32_t k = lane; k < nf; k += 64u) {
                const TmpNode& X = M.tmp[s_fr[k][0]];
                const uint32_t kk = (X.l >= 0 && s_fr[k][2] < 31u) ? X.count + 1u : 0u;
                if (kk > key) { key = kk; at = k; }
            }
            for (uint32_t off = 32; off > 0; off >>= 1) {   // max key, lowest index
                const uint32_t ok = __shfl_xor(key, off), oa = __shfl_xor(at, off);
                if (ok > key || (ok == key && oa < at)) { key = ok; at = oa; }
            }
            if (key == 0u) break;
            const uint32_t e0 = s_fr[at][0], e1 = s_fr[at][1], e2 = s_fr[at][2];
            // entries after `at` move up by one; reads complete before the writes
            uint32_t v0[2], v1[2], v2[2];
            for (int h = 0; h < 2; ++h) {
                const uint32_t k = lane + 64u * h;
                if (k < nf) { v0[h] = s_fr[k][0]; v1[h] = s_fr[k][1]; v2[h] = s_fr[k][2]; }
            }
            __builtin_amdgcn_wave_barrier();
            for (int h = 0; h < 2; ++h) {
                const uint32_t k = lane + 64u * h;
                if (k < nf && k > at) { s_fr[k + 1][0] = v0[h]; s_fr[k + 1][1] = v1[h]; s_fr[k + 1][2] = v2[h]; }
            }
            if (lane == 0) {
                const uint32_t l = static_cast<uint32_t>(M.tmp[e0].l);
                s_fr[at][0] = l; s_fr[at][1] = e1; s_fr[at][2] = e2 + 1u;
                s_fr[at + 1][0] = l + 1u; s_fr[at + 1][1] = e1 | (1u << e2); s_fr[at + 1][2] = e2 + 1u;
                s_nfr = nf + 1u;
            }
            __builtin_amdgcn_wave_barrier();
        }
        const uint32_t nf = s_nfr;
        // A tree deeper than the render kernel's DFS stack must never reach it (its pushes are
        // unchecked): the mesh is disabled in this image — no frontier parts, node count 0, so
        // mesh_traverse / part_traverse skip it — and the update reports kErrDepth.
        const bool too_deep = maxd >= L.depth_limit;
        for (uint32_t k = lane; k < M.part_cap; k += 64u) {
            I.parts[M.part0 + k] = (k < nf && !too_deep) ? make_int4(static_cast<int>(M.mesh),
                                                      static_cast<int>(M.root + M.tmp[s_fr[k][0]].ref),
                                                      static_cast<int>(s_fr[k][1]), static_cast<int>(s_fr[k][2]))
                                          : make_int4(-1, 0, 0, 0);
        }
        if (lane == 0) {
            uint32_t err = Ls.err;
            if (too_deep) err |= kErrDepth;
            M.status[0] = err;
            M.status[1] = maxd;
            M.status[2] = 1u + 2u * M.tmp[0].splits;   // nodesUsed
            // the mesh record's node count (0: disabled, see too_deep)
            I.meshes[M.mesh].y = too_deep ? 0 : static_cast<int>(M.status[2]);
            M.status[3] = nf;
            M.status[62] = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
        }
    }
}

}  // namespace

hipError_t launch_build(const Launch& L, hipStream_t stream) {
    if (L.n == 0) return hipSuccess;
    if (L.lds_bytes == 0) {   // a mesh too large for LDS: every mesh of the launch builds in HBM
        hipLaunchKernelGGL(rtx_anim_build<false>, dim3(L.n), dim3(kAnimThreads), 0, stream, L);
        return hipGetLastError();
    }
    if (L.lds_bytes > 64u * 1024u) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(rtx_anim_build<true>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(L.lds_bytes));
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(rtx_anim_build<true>, dim3(L.n), dim3(kAnimThreads), L.lds_bytes, stream, L);
    return hipGetLastError();
}

}  // namespace rtxa
