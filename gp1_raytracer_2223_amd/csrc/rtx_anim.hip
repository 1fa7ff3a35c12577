// rtx_anim.hip — Scene::Update for animated meshes on the device (see rtx_anim.h).
//
// The reference rebuilds each turning mesh's BVH top-down by binned SAH (DataTypes.h:294-483):
// per node, the centroid bounds, 8 bins per live axis, the 7-plane sweep, the in-place swap
// partition and UpdateNodeBounds of both children.  Here a node is processed by a TEAM of waves
// (16, 8, 4, 2 waves for a big node, one wave per node once a level is wide).  Nodes above
// Launch::cut triangles are split one at a time by a whole workgroup, as tasks of a per-mesh
// queue that 65 workgroups take from (the root by the workgroup that ran the set-up); their
// children below the cut become subtrees, each built level by level by one workgroup.  So the
// build spreads over as many CUs as there are independent nodes, from the root's children on.
//
// Exactness of the folds.  The reference folds with std::min / std::max from FLT_MAX /
// FLT_MIN, keeping the first of equal values; only a signed zero can observe that order.
//   * Bins and centroid bounds feed only the SAH decision: bin boxes enter through
//     AABB::Area = products of (max - min) with max >= FLT_MIN > 0, where (max - (+0)) and
//     (max - (-0)) are the same number, and the centroid minimum through (c - min) and
//     min + step (i + 1), equally blind to the zero's sign.  So they are folded in any order
//     (LDS float atomics, wave reductions): the same VALUES, hence the same decisions.
//   * Node bounds are written to the node array, so their minima keep the reference's first
//     occurrence exactly: an LDS atomic minimum over 64-bit keys (value order with -0 read as
//     +0, then the fold position, the sign riding in the low bit).  Maxima start at FLT_MIN
//     and can never be a zero: any order.
//   * The partition is the swap loop's closed form (derivation at team_ranks), a scatter.
// The output launch numbers the tree as the reference's recursion allocates it (children pairs
// in DFS preorder of the splits) and writes the node array, the render layout and the state.
// Built with the render library's flags (-ffp-contract=off, correctly rounded div/sqrt).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <algorithm>
#include <type_traits>

#include "rtx_anim.h"
#include "rtx_kernels.h"

namespace rtxa {

// Triangles placed in final leaves: the counter the workers stop on (kQDone), and the mark that
// the tree is complete once it reaches T (status word kStComplete, read by rtx_anim_out).
__device__ __forceinline__ void done_add(const MeshDev& M, uint32_t n) {
    const uint32_t o = atomicAdd(&M.q[kQDone], n);
    if (o < M.T && o + n >= M.T) atomicOr(&M.status[kStComplete], 1u);
}
namespace {

__device__ __forceinline__ float rmin(float m, float x) { return (x < m) ? x : m; }   // std::min(m, x)
__device__ __forceinline__ float rmax(float m, float x) { return (m < x) ? x : m; }   // std::max(m, x)
__device__ __forceinline__ float fbits(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t stamp() { return static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime()); }

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
__device__ __forceinline__ float area(float lx, float ly, float lz, float hx, float hy, float hz) {   // AABB::Area
    const float ex = hx - lx, ey = hy - ly, ez = hz - lz;
    return ex * ey + ey * ez + ez * ex;
}

// ---- keys of the first-occurrence minimum (node bounds)
__device__ __forceinline__ uint32_t ord(float v) {   // order-preserving bits of a non-NaN float
    const uint32_t u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
// value (zeros as +0) | fold position | sign: the minimum key is the reference's std::min fold
// result from FLT_MAX (position 0 = the initial value, element p at 1 + p)
__device__ __forceinline__ unsigned long long min_key(float v, uint32_t pos) {
    const float c = (v == 0.f) ? 0.f : v;
    return (static_cast<unsigned long long>(ord(c)) << 32) | (pos << 1) | (__float_as_uint(v) >> 31);
}
__device__ __forceinline__ float min_key_value(unsigned long long k) {
    const float v = unord(static_cast<uint32_t>(k >> 32));
    return (v == 0.f && (k & 1ull)) ? -0.f : v;
}
__device__ __forceinline__ unsigned long long min_key_init() { return min_key(FLT_MAX, 0u); }

// Order-free wave reductions through DPP row shifts (lanes outside the row keep the identity),
// then the rows combined: DPP row broadcasts (lane 15 of rows 0 / 2 into rows 1 / 3, lane 31
// into rows 2 and 3) and lane 63 read back, or (RTX_ANIM_DPP_BCAST=0) the four row results read
// back (values only, see the header).
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp_ctl(uint32_t v, uint32_t identity) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(identity), static_cast<int>(v), CTRL,
                                                             ROWS, 0xf, false));
}
template <int N>
__device__ __forceinline__ uint32_t dpp_shr(uint32_t v, uint32_t identity) {
    return dpp_ctl<0x110 + N>(v, identity);
}
// Batched forms: N independent values per lane reduced together, one DPP step for all of them
// at a time (back-to-back independent DPP moves need no hazard waits; a chain per value did:
// ~7 us per axis of the root's bins).  Order-free.
template <int CTRL, int ROWS, int N>
__device__ __forceinline__ void wred_step_min(float (&v)[N]) {
    float t[N];
#pragma unroll
    for (int i = 0; i < N; ++i) t[i] = __uint_as_float(dpp_ctl<CTRL, ROWS>(__float_as_uint(v[i]), __float_as_uint(FLT_MAX)));
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = fminf(v[i], t[i]);
}
template <int CTRL, int ROWS, int N>
__device__ __forceinline__ void wred_step_max(float (&v)[N]) {
    float t[N];
#pragma unroll
    for (int i = 0; i < N; ++i) t[i] = __uint_as_float(dpp_ctl<CTRL, ROWS>(__float_as_uint(v[i]), __float_as_uint(FLT_MIN)));
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = fmaxf(v[i], t[i]);
}
template <int CTRL, int ROWS, int N>
__device__ __forceinline__ void wred_step_sum(uint32_t (&v)[N]) {
    uint32_t t[N];
#pragma unroll
    for (int i = 0; i < N; ++i) t[i] = dpp_ctl<CTRL, ROWS>(v[i], 0u);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += t[i];
}
template <int CTRL, int ROWS, int N>
__device__ __forceinline__ void wred_step_min64(unsigned long long (&v)[N]) {
    uint32_t lo[N], hi[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        lo[i] = dpp_ctl<CTRL, ROWS>(static_cast<uint32_t>(v[i]), ~0u);
        hi[i] = dpp_ctl<CTRL, ROWS>(static_cast<uint32_t>(v[i] >> 32), ~0u);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const unsigned long long w = (static_cast<unsigned long long>(hi[i]) << 32) | lo[i];
        v[i] = w < v[i] ? w : v[i];
    }
}
// the four row steps (lane 15 of each row then holds the row's fold), then the rows
#define RTX_WRED_ROWS(step, v) step<0x111, 0xf>(v); step<0x112, 0xf>(v); step<0x114, 0xf>(v); step<0x118, 0xf>(v)
#define RTX_WRED_BCAST(step, v) step<0x142, 0xa>(v); step<0x143, 0xc>(v)
__device__ __forceinline__ float rl(float v, int l) { return __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), l)); }
template <int N>
__device__ __forceinline__ void wred_min(float (&v)[N]) {
    RTX_WRED_ROWS(wred_step_min, v);
#if RTX_ANIM_DPP_BCAST
    RTX_WRED_BCAST(wred_step_min, v);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = rl(v[i], 63);
#else
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = fminf(fminf(rl(v[i], 15), rl(v[i], 31)), fminf(rl(v[i], 47), rl(v[i], 63)));
#endif
}
template <int N>
__device__ __forceinline__ void wred_max(float (&v)[N]) {
    RTX_WRED_ROWS(wred_step_max, v);
#if RTX_ANIM_DPP_BCAST
    RTX_WRED_BCAST(wred_step_max, v);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = rl(v[i], 63);
#else
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = fmaxf(fmaxf(rl(v[i], 15), rl(v[i], 31)), fmaxf(rl(v[i], 47), rl(v[i], 63)));
#endif
}
template <int N>
__device__ __forceinline__ void wred_sum(uint32_t (&v)[N]) {
    RTX_WRED_ROWS(wred_step_sum, v);
#if RTX_ANIM_DPP_BCAST
    RTX_WRED_BCAST(wred_step_sum, v);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = __builtin_amdgcn_readlane(v[i], 63);
#else
#pragma unroll
    for (int i = 0; i < N; ++i)
        v[i] = __builtin_amdgcn_readlane(v[i], 15) + __builtin_amdgcn_readlane(v[i], 31) +
               __builtin_amdgcn_readlane(v[i], 47) + __builtin_amdgcn_readlane(v[i], 63);
#endif
}
__device__ __forceinline__ unsigned long long rl64(unsigned long long v, int l) {
    return (static_cast<unsigned long long>(__builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), l)) << 32) |
           __builtin_amdgcn_readlane(static_cast<uint32_t>(v), l);
}
template <int N>
__device__ __forceinline__ void wred_min64(unsigned long long (&v)[N]) {
    RTX_WRED_ROWS(wred_step_min64, v);
#if RTX_ANIM_DPP_BCAST
    RTX_WRED_BCAST(wred_step_min64, v);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = rl64(v[i], 63);
#else
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const unsigned long long r0 = rl64(v[i], 15), r1 = rl64(v[i], 31), r2 = rl64(v[i], 47), r3 = rl64(v[i], 63);
        const unsigned long long a = r0 < r1 ? r0 : r1, b = r2 < r3 ? r2 : r3;
        v[i] = a < b ? a : b;
    }
#endif
}

// Transposing wave reduction of 32 values per lane, index q * 8 + c (c 0: a sum, 1-3: a
// minimum, 4-6: a maximum, 7: unused).  Each step pairs every lane with the lane whose id
// differs in one bit; of its current values the lane keeps one half (the upper when its bit is
// set), sends the other half to its partner and folds what it receives into what it keeps:
// 16 + 8 + 4 + 2 + 1 folds and one exchange of the two 32-lane halves instead of 32 full
// reductions of 15 steps each.  Lane l ends with the wave's fold of value
// q = 2 (l & 1) + ((l >> 1) & 1), c = 4 ((l >> 2) & 1) + 2 ((l >> 3) & 1) + ((l >> 4) & 1)
// (lanes l and l + 32 alike).  Order-free, like the other wave reductions.
__device__ __forceinline__ float fold_c(uint32_t c, float a, float b) {
    return c == 0u ? a + b : (c < 4u ? fminf(a, b) : fmaxf(a, b));
}
template <int X>   // the value of lane l ^ X (X = 1, 2: DPP quad permutes; 4, 8, 16: LDS swizzles)
__device__ __forceinline__ float xchg(float v) {
    const int u = __float_as_int(v);
    if constexpr (X == 1) return __int_as_float(__builtin_amdgcn_mov_dpp(u, 0xB1, 0xf, 0xf, false));   // [1,0,3,2]
    else if constexpr (X == 2) return __int_as_float(__builtin_amdgcn_mov_dpp(u, 0x4E, 0xf, 0xf, false));   // [2,3,0,1]
    else if constexpr (X == 32) return __shfl_xor(v, 32);
    else return __int_as_float(__builtin_amdgcn_ds_swizzle(u, 0x1F | (X << 10)));   // bitmask mode: and 31, xor X
}
template <int X, int N, int V>
__device__ __forceinline__ void tstep(float (&v)[V], uint32_t lane, uint32_t& cbase) {
    constexpr int H = N / 2;
    const bool hi = (lane & static_cast<uint32_t>(X)) != 0u;
    float snd[H], kp[H];
#pragma unroll
    for (int i = 0; i < H; ++i) {
        snd[i] = hi ? v[i] : v[i + H];
        kp[i] = hi ? v[i + H] : v[i];
    }
#pragma unroll
    for (int i = 0; i < H; ++i) snd[i] = xchg<X>(snd[i]);
    if (N <= 8 && hi) cbase += static_cast<uint32_t>(H);   // the kept values' components
#pragma unroll
    for (int i = 0; i < H; ++i) v[i] = fold_c(N > 8 ? static_cast<uint32_t>(i & 7) : cbase + i, kp[i], snd[i]);
}
// V = 64 (eight bins): a sixth halving step across the two 32-lane halves instead of the full
// fold; lane l then holds q = 4 (l & 1) + 2 ((l >> 1) & 1) + ((l >> 2) & 1), c from bits 3-5.
template <int V>
__device__ __forceinline__ float wred_transpose(float (&v)[V], uint32_t lane, uint32_t& q, uint32_t& c) {
    uint32_t cb = 0;
    if constexpr (V == 64) {
        tstep<1, 64>(v, lane, cb);
        tstep<2, 32>(v, lane, cb);
        tstep<4, 16>(v, lane, cb);
        tstep<8, 8>(v, lane, cb);
        tstep<16, 4>(v, lane, cb);
        tstep<32, 2>(v, lane, cb);
        q = 4u * (lane & 1u) + 2u * ((lane >> 1) & 1u) + ((lane >> 2) & 1u);
        c = cb;
        return v[0];
    } else {
        tstep<1, 32>(v, lane, cb);
        tstep<2, 16>(v, lane, cb);
        tstep<4, 8>(v, lane, cb);
        tstep<8, 4>(v, lane, cb);
        tstep<16, 2>(v, lane, cb);
        const float r = fold_c(cb, v[0], __shfl_xor(v[0], 32));
        q = 2u * (lane & 1u) + ((lane >> 1) & 1u);
        c = cb;
        return r;
    }
}

// The build records and permutation of a build region.  Records: centroid (v0 + v1 + v2) *
// 0.3333f and the triangle box min(min(v0, v1), v2) / max(max(v0, v1), v2) — growing a node or
// bin by the box equals growing it by the three vertices in order (first occurrence
// included) — as 9 arrays of `stride` floats by element index.  LDS = true: the region's
// records, permutation buffers and partition scratch are staged in the workgroup's LDS
// (16-bit indices, element = local index, positions relative to pos0); false: HBM
// (MeshDev::soa / perm / lb / rs / rk, element = triangle id, absolute positions).
template <bool LDS>
struct Store {
    using P = std::conditional_t<LDS, uint16_t, uint32_t>;
    P* perm[2];
    P *lb, *rs, *rk;
    const float* rec;
    uint32_t stride, pos0;
    __device__ float c(int ax, uint32_t e) const { return rec[ax * stride + e]; }
    __device__ float lo(int ax, uint32_t e) const { return rec[(3 + ax) * stride + e]; }
    __device__ float hi(int ax, uint32_t e) const { return rec[(6 + ax) * stride + e]; }
};
constexpr uint32_t kLdsBytesTop = 46;    // per element: 9 record floats, 2 + 3 16-bit words
constexpr uint32_t kLdsBytesSub = 50;    // + the element's triangle id
constexpr uint32_t kSubLdsMax = 2816;    // subtrees up to this size build from LDS

constexpr int kBins = 8, kPlanes = kBins - 1;

// Per-team LDS scratch (one node at a time per team).
struct Slot {
    float cb[6];                         // centroid bounds: min xyz, max xyz
    uint32_t bc[3][kBins];               // idxCount per axis and bin
    float bl[3][kBins][3], bh[3][kBins][3];
    unsigned long long cmin[2][3];       // children's node bounds (keys) and maxima
    float cmax[2][3];
    uint32_t wc[kAnimWaves][3];          // per-wave partition counts: smalls, left bigs, right smalls
};

// Shared state of one workgroup's level loop.
struct Level {
    uint32_t K, next, take, maxn, nmaxn;   // nodes this level, appended next-level nodes, wave-task counter, max counts
    uint32_t ids;                          // next temp id
    uint32_t err;
};

// The level lists of a build region (a mesh for the top phase, a subtree's range for launch 2).
struct Region {
    uint32_t* cur;
    uint32_t* nxt;
};

// A team: waves [w0, w0 + k) of the workgroup; lanes tl in [0, 64 k).
struct Team {
    uint32_t k, w0, wt, tl, lane;
};

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
// One wave assigns the ranks of positions [lo, hi) (relative to the node's local first f0),
// given the rank bases lbase / rbase (the counts of left bigs before lo / right smalls after hi).
template <bool LDS>
__device__ __forceinline__ void wave_ranks(const Store<LDS>& St, const typename Store<LDS>::P* src, uint32_t lane,
                                           uint32_t f0, uint32_t lo, uint32_t hi, uint32_t pL, int axis, float pos,
                                           uint32_t lbase, uint32_t rbase) {
    using P = typename Store<LDS>::P;
    auto small = [&](uint32_t q) { return St.c(axis, src[f0 + q]) < pos; };
    const unsigned long long below = (1ull << lane) - 1ull;
    uint32_t carry = lbase;
    const uint32_t lhi = min(hi, pL);
    for (uint32_t base = lo; base < lhi; base += 64u) {   // left-stream bigs, in order
        const uint32_t q = base + lane;
        const bool b = q < lhi && !small(q);
        const unsigned long long m = __ballot(b);
        if (b) {
            const uint32_t r = carry + __popcll(m & below);
            St.lb[f0 + r] = static_cast<P>(q);
            St.rk[f0 + q] = static_cast<P>(r);
        }
        carry += __popcll(m);
    }
    carry = rbase;
    const uint32_t rlo = max(lo, pL);
    for (uint32_t top = hi; top > rlo;) {   // right-stream smalls, from the end
        const uint32_t cnt = min(64u, top - rlo);
        const bool in = lane < cnt;
        const uint32_t p = in ? top - 1u - lane : 0u;
        const bool sm = in && small(p);
        const unsigned long long m = __ballot(sm);
        if (sm) {
            const uint32_t r = carry + __popcll(m & below);
            St.rs[f0 + r] = static_cast<P>(p);
            St.rk[f0 + p] = static_cast<P>(r);
        }
        carry += __popcll(m);
        top -= cnt;
    }
}
// Destination of position q once every rank is known.
template <bool LDS>
__device__ __forceinline__ uint32_t part_dest(const Store<LDS>& St, uint32_t f0, uint32_t n, uint32_t q, uint32_t pL,
                                              bool big) {
    if (q < pL) {
        if (!big) return q;
        const uint32_t m = St.rk[f0 + q];
        return m == 0u ? n - 1u : static_cast<uint32_t>(St.rs[f0 + m - 1u]) - 1u;
    }
    return big ? q - 1u : static_cast<uint32_t>(St.lb[f0 + St.rk[f0 + q]]);
}

// Team synchronisation: a workgroup barrier for multi-wave teams (every wave of the workgroup
// runs the same sequence of barriers), else the wave's own memory ordering.
template <bool MULTI>
__device__ __forceinline__ void tsync() {
    if (MULTI) {
        __syncthreads();
    } else {
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
    }
}

// Node bounds over elements in fold order: a lane's private keys / maxima, then the wave's.
struct BoundAcc {
    unsigned long long k0 = ~0ull, k1 = ~0ull, k2 = ~0ull;
    float m0 = FLT_MIN, m1 = FLT_MIN, m2 = FLT_MIN;
    template <class ST>
    __device__ void add(const ST& St, uint32_t e, uint32_t r) {   // element e at fold position r (>= 1)
        const float a0 = St.lo(0, e), a1 = St.lo(1, e), a2 = St.lo(2, e);
        if (a0 == a0) { const unsigned long long k = min_key(a0, r); k0 = k < k0 ? k : k0; }
        if (a1 == a1) { const unsigned long long k = min_key(a1, r); k1 = k < k1 ? k : k1; }
        if (a2 == a2) { const unsigned long long k = min_key(a2, r); k2 = k < k2 ? k : k2; }
        m0 = fmaxf(m0, St.hi(0, e)); m1 = fmaxf(m1, St.hi(1, e)); m2 = fmaxf(m2, St.hi(2, e));
    }
    __device__ void addv(float a0, float a1, float a2, float h0, float h1, float h2, uint32_t r) {   // from registers
        if (a0 == a0) { const unsigned long long k = min_key(a0, r); k0 = k < k0 ? k : k0; }
        if (a1 == a1) { const unsigned long long k = min_key(a1, r); k1 = k < k1 ? k : k1; }
        if (a2 == a2) { const unsigned long long k = min_key(a2, r); k2 = k < k2 ? k : k2; }
        m0 = fmaxf(m0, h0); m1 = fmaxf(m1, h1); m2 = fmaxf(m2, h2);
    }
    __device__ void wave() {
        unsigned long long k[3] = {k0, k1, k2};
        float m[3] = {m0, m1, m2};
        wred_min64(k);
        wred_max(m);
        k0 = k[0]; k1 = k[1]; k2 = k[2];
        m0 = m[0]; m1 = m[1]; m2 = m[2];
    }
    // into the slot's child c: atomics (several waves) or a plain store (one wave)
    __device__ void put(Slot& sl, int c, bool atomic) const {
        if (atomic) {
            atomicMin(&sl.cmin[c][0], k0); atomicMin(&sl.cmin[c][1], k1); atomicMin(&sl.cmin[c][2], k2);
            atomicMax(&sl.cmax[c][0], m0); atomicMax(&sl.cmax[c][1], m1); atomicMax(&sl.cmax[c][2], m2);
        } else {
            const unsigned long long i = min_key_init();
            sl.cmin[c][0] = k0 < i ? k0 : i; sl.cmin[c][1] = k1 < i ? k1 : i; sl.cmin[c][2] = k2 < i ? k2 : i;
            sl.cmax[c][0] = m0; sl.cmax[c][1] = m1; sl.cmax[c][2] = m2;
        }
    }
};

template <int Q0, int H, class ST, class PT, class SINK>
__device__ __forceinline__ void bins_private_half(const ST& St, const PT* src, uint32_t f0, uint32_t n, uint32_t tl,
                                                  uint32_t nl, uint32_t lane, int ax, float minB, float scale,
                                                  const SINK& sink) {
    // bins Q0 .. Q0 + H - 1 (H = 4: half the registers of all eight)
    uint32_t bc[H];
    float bl[H][3], bh[H][3];
#pragma unroll
    for (int q = 0; q < H; ++q) {
        bc[q] = 0u;
        bl[q][0] = bl[q][1] = bl[q][2] = FLT_MAX;
        bh[q][0] = bh[q][1] = bh[q][2] = FLT_MIN;
    }
    for (uint32_t p = tl; p < n; p += nl) {
        const uint32_t e = src[f0 + p];
        const float x = (St.c(ax, e) - minB) * scale;
        int bi = x >= 0.f ? static_cast<int>(fminf(x, 2147483520.f)) : 0;
        bi = kPlanes < bi ? kPlanes : bi;
        const float l0 = St.lo(0, e), l1 = St.lo(1, e), l2 = St.lo(2, e);
        const float h0 = St.hi(0, e), h1 = St.hi(1, e), h2 = St.hi(2, e);
#pragma unroll
        for (int q = 0; q < H; ++q) {
            const bool h = bi == Q0 + q;
            bc[q] += h ? 3u : 0u;
            bl[q][0] = fminf(bl[q][0], h ? l0 : FLT_MAX);
            bl[q][1] = fminf(bl[q][1], h ? l1 : FLT_MAX);
            bl[q][2] = fminf(bl[q][2], h ? l2 : FLT_MAX);
            bh[q][0] = fmaxf(bh[q][0], h ? h0 : FLT_MIN);
            bh[q][1] = fmaxf(bh[q][1], h ? h1 : FLT_MIN);
            bh[q][2] = fmaxf(bh[q][2], h ? h2 : FLT_MIN);
        }
    }
#if RTX_ANIM_BINS_TRANSPOSE
    float v[8 * H];   // index q * 8 + c: c 0 the count (exact: < 2^24), 1-3 the box minimum, 4-6 its maximum
#pragma unroll
    for (int q = 0; q < H; ++q) {
        v[q * 8] = static_cast<float>(bc[q]);
        v[q * 8 + 1] = bl[q][0]; v[q * 8 + 2] = bl[q][1]; v[q * 8 + 3] = bl[q][2];
        v[q * 8 + 4] = bh[q][0]; v[q * 8 + 5] = bh[q][1]; v[q * 8 + 6] = bh[q][2];
        v[q * 8 + 7] = 0.f;
    }
    uint32_t q, c;
    const float r = wred_transpose<8 * H>(v, lane, q, c);
    if ((H == 8 || lane < 32u) && c < 7u) sink.put1(ax, Q0 + static_cast<int>(q), c, r);
#else
    wred_sum(bc);
    wred_min(reinterpret_cast<float(&)[3 * H]>(bl));
    wred_max(reinterpret_cast<float(&)[3 * H]>(bh));
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < H; ++q) sink.put(ax, Q0 + q, bc[q], bl[q][0], bl[q][1], bl[q][2], bh[q][0], bh[q][1], bh[q][2]);
#endif
}
// One axis's bins over the positions [0, n) a lane visits (tl, tl + nl, ...), folded in
// registers (branch-free: the other bins see their fold identity), then over the wave (DPP),
// then into the slot: atomics (several waves) or plain stores (one wave).  Order-free (see
// the header); used where lanes hold several elements, LDS atomics per element otherwise.
// All eight bins in one pass (the 256-VGPR budget of a 512-thread workgroup; two passes of four
// bins with RTX_ANIM_BIN_PASSES=2: the root's bins 26 -> 23 us).
// Sink of a wave's bins: a slot's bins (the team's, or the wave's own partial record that is
// folded over the team's waves after a barrier — same-address LDS atomics from every wave of a
// team serialised: 40 us a level).
struct SlotSink {
    Slot& sl;
    __device__ void put(int ax, int b, uint32_t c, float a0, float a1, float a2, float b0, float b1, float b2) const {
        sl.bc[ax][b] = c;
        sl.bl[ax][b][0] = a0; sl.bl[ax][b][1] = a1; sl.bl[ax][b][2] = a2;
        sl.bh[ax][b][0] = b0; sl.bh[ax][b][1] = b1; sl.bh[ax][b][2] = b2;
    }
    // one component c (0 the count, 1-3 the minimum, 4-6 the maximum) of bin b
    __device__ void put1(int ax, int b, uint32_t c, float v) const {   // one store, no branches
        uint32_t* const w = c == 0u ? &sl.bc[ax][b]
                                    : reinterpret_cast<uint32_t*>(c < 4u ? &sl.bl[ax][b][c - 1u] : &sl.bh[ax][b][c - 4u]);
        *w = c == 0u ? static_cast<uint32_t>(v) : __float_as_uint(v);
    }
};
template <class ST, class PT, class SINK>
__device__ __forceinline__ void bins_private(const ST& St, const PT* src, uint32_t f0, uint32_t n, uint32_t tl,
                                             uint32_t nl, uint32_t lane, int ax, float minB, float scale,
                                             const SINK& sink) {
#if RTX_ANIM_BIN_PASSES == 1 && RTX_ANIM_BINS_TRANSPOSE
    bins_private_half<0, kBins>(St, src, f0, n, tl, nl, lane, ax, minB, scale, sink);
#else
    bins_private_half<0, kBins / 2>(St, src, f0, n, tl, nl, lane, ax, minB, scale, sink);
    bins_private_half<kBins / 2, kBins / 2>(St, src, f0, n, tl, nl, lane, ax, minB, scale, sink);
#endif
}

// 4. the plane sweep (DataTypes.h:443-480) over the bins in the slot: lane j < 21 evaluates
//    plane j % 7 of axis j / 7; the reference takes the first strictly smaller cost in
//    (axis, plane) order from FLT_MAX.  Returns whether the node splits (at axis, pos).
__device__ __forceinline__ bool plane_sweep(const Slot& sl, uint32_t lane, const bool (&live)[3], const float (&minB)[3],
                                            const float (&bd)[3], uint32_t n, const TmpNode& X, int& axis, float& pos) {
    unsigned long long key = ~0ull;
    const uint32_t j = lane;
    if (j < 3u * kPlanes) {
        const int ax = static_cast<int>(j / kPlanes), i = static_cast<int>(j % kPlanes);
        if (live[ax]) {
            // all eight bins read at once (a fixed loop, no per-lane trip counts); a bin on
            // the other side enters as the fold identity (rmin(m, FLT_MAX) = m, and
            // rmax(m, FLT_MIN) = m for every m >= FLT_MIN, which all maxima are)
            uint32_t bcq[kBins];
            float bq[kBins][6];
#pragma unroll
            for (int q = 0; q < kBins; ++q) {
                bcq[q] = sl.bc[ax][q];
                bq[q][0] = sl.bl[ax][q][0]; bq[q][1] = sl.bl[ax][q][1]; bq[q][2] = sl.bl[ax][q][2];
                bq[q][3] = sl.bh[ax][q][0]; bq[q][4] = sl.bh[ax][q][1]; bq[q][5] = sl.bh[ax][q][2];
            }
            int lc = 0, rc = 0;
            float l0 = FLT_MAX, l1 = FLT_MAX, l2 = FLT_MAX, h0 = FLT_MIN, h1 = FLT_MIN, h2 = FLT_MIN;
#pragma unroll
            for (int q = 0; q < kBins; ++q) {   // leftBox.Grow(bins[q].bounds), q = 0..i
                const bool in = q <= i;
                lc += in ? static_cast<int>(bcq[q]) : 0;
                l0 = rmin(l0, in ? bq[q][0] : FLT_MAX); l1 = rmin(l1, in ? bq[q][1] : FLT_MAX);
                l2 = rmin(l2, in ? bq[q][2] : FLT_MAX);
                h0 = rmax(h0, in ? bq[q][3] : FLT_MIN); h1 = rmax(h1, in ? bq[q][4] : FLT_MIN);
                h2 = rmax(h2, in ? bq[q][5] : FLT_MIN);
            }
            const float la = area(l0, l1, l2, h0, h1, h2);
            l0 = l1 = l2 = FLT_MAX;
            h0 = h1 = h2 = FLT_MIN;
#pragma unroll
            for (int q = kPlanes; q >= 0; --q) {   // rightBox.Grow(bins[q].bounds), q = 7..i+1
                const bool in = q > i;
                rc += in ? static_cast<int>(bcq[q]) : 0;
                l0 = rmin(l0, in ? bq[q][0] : FLT_MAX); l1 = rmin(l1, in ? bq[q][1] : FLT_MAX);
                l2 = rmin(l2, in ? bq[q][2] : FLT_MAX);
                h0 = rmax(h0, in ? bq[q][3] : FLT_MIN); h1 = rmax(h1, in ? bq[q][4] : FLT_MIN);
                h2 = rmax(h2, in ? bq[q][5] : FLT_MIN);
            }
            const float ra = area(l0, l1, l2, h0, h1, h2);
            const float cost = static_cast<float>(lc) * la + static_cast<float>(rc) * ra;
            // candidates: cost < FLT_MAX (NaN never is); ties keep the earlier (axis, plane)
            if (cost < FLT_MAX) key = min_key(cost, j) & ~1ull;
        }
    }
    {
        unsigned long long k1[1] = {key};
        wred_min64(k1);
        key = k1[0];
    }
    float bestCost = FLT_MAX;
    if (key != ~0ull) {
        const uint32_t jb = static_cast<uint32_t>(key) >> 1;
        axis = static_cast<int>(jb / kPlanes);
        const int i = static_cast<int>(jb % kPlanes);
        const float step = bd[axis] / kBins;
        pos = minB[axis] + step * static_cast<float>(i + 1);
        bestCost = min_key_value(key);
    }
    auto u = [](float v) { return __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(v))); };
    const float noSplitCost = static_cast<float>(3u * n) * area(u(X.mn[0]), u(X.mn[1]), u(X.mn[2]), u(X.mx[0]),
                                                                u(X.mx[1]), u(X.mx[2]));
    return !(bestCost >= noSplitCost);   // Subdivide: `if (splitCost >= noSplitCost) return;`
}

// ---- 128-position masks (two ballots) for a one-wave node of at most 128 elements
struct Mask128 {
    unsigned long long w[2];
};
__device__ __forceinline__ uint32_t pop_below(const Mask128& m, uint32_t q) {   // set bits at positions < q
    const unsigned long long b0 = q >= 64u ? ~0ull : ((1ull << q) - 1ull);
    const unsigned long long b1 = q <= 64u ? 0ull : (q >= 128u ? ~0ull : ((1ull << (q - 64u)) - 1ull));
    return static_cast<uint32_t>(__popcll(m.w[0] & b0) + __popcll(m.w[1] & b1));
}
__device__ __forceinline__ uint32_t sel64(unsigned long long m, uint32_t k) {   // position of the k-th set bit (lowest first)
    uint32_t p = 0;
#pragma unroll
    for (uint32_t w = 32; w >= 1u; w >>= 1) {
        const uint32_t c = static_cast<uint32_t>(__popcll(m & ((1ull << w) - 1ull)));
        const bool up = k >= c;
        k = up ? k - c : k;
        m = up ? m >> w : m;
        p = up ? p + w : p;
    }
    return p;
}
__device__ __forceinline__ uint32_t sel128(const Mask128& m, uint32_t k) {
    const uint32_t c0 = static_cast<uint32_t>(__popcll(m.w[0]));
    return k < c0 ? sel64(m.w[0], k) : 64u + sel64(m.w[1], k - c0);
}

// One node of n <= 128 elements by one wave, the elements in registers (positions lane and
// lane + 64): the same decisions and outputs as node_process, without the LDS round trips of
// its element passes.  The partition's closed form (wave_ranks / part_dest) is evaluated on
// the wave's ballot masks: with bigL the big elements left of pL and smallR the small ones
// from pL on, a big q < pL with m = |bigL below q| goes to n - 1 (m = 0) or one before the
// (m - 1)-th element of smallR counted from the top; a small p >= pL with r = |smallR above p|
// goes to the r-th element of bigL; the others stay (q < pL) or move one left (p >= pL).
template <bool LDS>
__device__ __forceinline__ void node_small(const Store<LDS>& St, TmpNode* nodes, uint32_t lane, Slot& sl, Level& Lv,
                                           const Region& rg, uint32_t t, uint32_t b, uint32_t sub, uint32_t n,
                                           uint32_t first, uint32_t depth) {
    using P = typename Store<LDS>::P;
    P* src = b ? St.perm[1] : St.perm[0];
    P* dst = b ? St.perm[0] : St.perm[1];
    const uint32_t f0 = first - St.pos0;
    bool v[2];
    uint32_t e[2];
    float c[2][3], lo[2][3], hi[2][3];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t q = lane + 64u * j;
        v[j] = q < n;
        e[j] = v[j] ? static_cast<uint32_t>(src[f0 + q]) : 0u;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            c[j][a] = v[j] ? St.c(a, e[j]) : 0.f;
            lo[j][a] = v[j] ? St.lo(a, e[j]) : 0.f;
            hi[j][a] = v[j] ? St.hi(a, e[j]) : 0.f;
        }
    }
    if (!(3u * n > 8u)) {   // Subdivide's termination: the range as it is, in both buffers
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (v[j]) dst[f0 + lane + 64u * j] = static_cast<P>(e[j]);
        return;
    }
    // 1. the slot's bins
    if (lane < 3u * kBins) (&sl.bc[0][0])[lane] = 0u;
    for (uint32_t i = lane; i < 3u * kBins * 3u; i += 64u) {
        (&sl.bl[0][0][0])[i] = FLT_MAX;
        (&sl.bh[0][0][0])[i] = FLT_MIN;
    }
    // 2. centroid bounds (DataTypes.h:404-419), order-free
    float mn3[3], mx3[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        mn3[a] = fminf(v[0] ? c[0][a] : FLT_MAX, v[1] ? c[1][a] : FLT_MAX);
        mx3[a] = fmaxf(v[0] ? c[0][a] : FLT_MIN, v[1] ? c[1][a] : FLT_MIN);
    }
    wred_min(mn3);
    wred_max(mx3);
    float minB[3], bd[3], scale[3];
    bool live[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        minB[a] = mn3[a];
        bd[a] = mx3[a] - minB[a];                 // boundsDifference
        live[a] = !(fabsf(bd[a]) < FLT_EPSILON);  // else `continue`
        scale[a] = kBins / bd[a];
    }
    tsync<false>();
    // 3. bins (DataTypes.h:424-440): LDS atomics per element
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (!v[j]) continue;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (!live[a]) continue;
            const float x = (c[j][a] - minB[a]) * scale[a];
            int bi = x >= 0.f ? static_cast<int>(fminf(x, 2147483520.f)) : 0;
            bi = kPlanes < bi ? kPlanes : bi;
            atomicAdd(&sl.bc[a][bi], 3u);
            atomicMin(&sl.bl[a][bi][0], lo[j][0]); atomicMin(&sl.bl[a][bi][1], lo[j][1]); atomicMin(&sl.bl[a][bi][2], lo[j][2]);
            atomicMax(&sl.bh[a][bi][0], hi[j][0]); atomicMax(&sl.bh[a][bi][1], hi[j][1]); atomicMax(&sl.bh[a][bi][2], hi[j][2]);
        }
    }
    tsync<false>();
    // 4. the sweep
    int axis = 0;
    float pos = 0.f;
    const bool split = plane_sweep(sl, lane, live, minB, bd, n, nodes[t], axis, pos);
    if (!split) {   // a leaf: the range as it is, in both buffers
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (v[j]) dst[f0 + lane + 64u * j] = static_cast<P>(e[j]);
        return;
    }
    // 5. the partition on ballot masks
    bool sm[2];
    sm[0] = v[0] && (axis == 0 ? c[0][0] : axis == 1 ? c[0][1] : c[0][2]) < pos;
    sm[1] = v[1] && (axis == 0 ? c[1][0] : axis == 1 ? c[1][1] : c[1][2]) < pos;
    const Mask128 small{{__ballot(sm[0]), __ballot(sm[1])}};
    const Mask128 valid{{__ballot(v[0]), __ballot(v[1])}};
    const uint32_t S = static_cast<uint32_t>(__popcll(small.w[0]) + __popcll(small.w[1]));
    const bool smallS = S < n && ((small.w[S >> 6] >> (S & 63u)) & 1ull);
    const uint32_t pL = S + ((S < n && !smallS) ? 1u : 0u);
    const unsigned long long lt0 = pL >= 64u ? ~0ull : ((1ull << pL) - 1ull);
    const unsigned long long lt1 = pL <= 64u ? 0ull : (pL >= 128u ? ~0ull : ((1ull << (pL - 64u)) - 1ull));
    const Mask128 bigL{{valid.w[0] & ~small.w[0] & lt0, valid.w[1] & ~small.w[1] & lt1}};
    const Mask128 smallR{{small.w[0] & ~lt0, small.w[1] & ~lt1}};
    const uint32_t nR = static_cast<uint32_t>(__popcll(smallR.w[0]) + __popcll(smallR.w[1]));
    const bool kids = S != 0u && S < n;   // (S <= n always; < n also keeps a child count from wrapping)
    uint32_t dpos[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t q = lane + 64u * j;
        uint32_t d = q;
        if (q < pL) {
            if (v[j] && !sm[j]) {
                const uint32_t m = pop_below(bigL, q);
                d = m == 0u ? n - 1u : sel128(smallR, nR - m) - 1u;   // the (m - 1)-th from the top
            }
        } else {
            d = sm[j] ? sel128(bigL, nR - 1u - pop_below(smallR, q)) : q - 1u;   // r = |smallR above q|
        }
        d = d < n ? d : n - 1u;   // (the closed form stays in range; a guard for the stores)
        dpos[j] = d;
        if (v[j]) {
            dst[f0 + d] = static_cast<P>(e[j]);
            if (!kids) src[f0 + d] = static_cast<P>(e[j]);   // leftCount 0 or all: a leaf, both buffers
        }
    }
    if (!kids) return;
    // 6. UpdateNodeBounds of both children (DataTypes.h:310-321) from the registers
    BoundAcc A[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (!v[j]) continue;
        const bool right = dpos[j] >= S;
        const uint32_t r = 1u + (right ? dpos[j] - S : dpos[j]);
        if (right) A[1].addv(lo[j][0], lo[j][1], lo[j][2], hi[j][0], hi[j][1], hi[j][2], r);
        else A[0].addv(lo[j][0], lo[j][1], lo[j][2], hi[j][0], hi[j][1], hi[j][2], r);
    }
    unsigned long long k[6] = {A[0].k0, A[0].k1, A[0].k2, A[1].k0, A[1].k1, A[1].k2};
    float m[6] = {A[0].m0, A[0].m1, A[0].m2, A[1].m0, A[1].m1, A[1].m2};
    wred_min64(k);
    wred_max(m);
    if (lane == 0) {
        const uint32_t cid = atomicAdd(&Lv.ids, 2u);
        const unsigned long long ki = min_key_init();
        TmpNode a{}, bb{};
        for (int q = 0; q < 3; ++q) {
            a.mn[q] = min_key_value(k[q] < ki ? k[q] : ki); a.mx[q] = m[q];
            bb.mn[q] = min_key_value(k[3 + q] < ki ? k[3 + q] : ki); bb.mx[q] = m[3 + q];
        }
        a.first = first; a.count = S; a.l = -1; a.depth = depth + 1; a.parent = static_cast<int32_t>(t); a.sub = sub;
        bb.first = first + S; bb.count = n - S; bb.l = -1; bb.depth = depth + 1; bb.parent = static_cast<int32_t>(t);
        bb.sub = sub;
        nodes[cid] = a;
        nodes[cid + 1] = bb;
        nodes[t].l = static_cast<int32_t>(cid);
        const uint32_t w = atomicAdd(&Lv.next, 2u);
        rg.nxt[w] = cid;
        rg.nxt[w + 1] = cid + 1;
        atomicMax(&Lv.nmaxn, max(S, n - S));
    }
}

// One node (temp id t, or none: `act` false) by one team.  b: the permutation buffer of this
// level (depth parity); the next level's is b ^ 1.  Children are appended to rg.nxt.
template <bool MULTI, bool LDS>
__device__ __forceinline__ void node_process(const MeshDev& M, const Store<LDS>& St, TmpNode* nodes, const Team& tm,
                                             Slot* slots, Level& Lv, const Region& rg, bool act, uint32_t t, uint32_t b,
                                             uint32_t sub) {
    Slot& sl = slots[tm.w0];   // the team's slot; slots[w0 + 1 .. w0 + k - 1] hold partial bins
    auto sl_of = [&](uint32_t wt) -> Slot& { return slots[tm.w0 + wt]; };
    // diagnostics (RTX_ANIM_STEP_STAMPS): step times of the top phase's root (status 63-75)
    // and of subtree 0's root (status 40-52)
    int wbase = -1;
    if (RTX_ANIM_STEP_STAMPS && act) {
        if (sub == kMaxSub && t == 0 && nodes == M.tmp) wbase = 63;
        else if (sub == 0 && (nodes == M.tmp ? t == M.sub[0].root : t == 0)) wbase = 40;
    }
    auto stp = [&](int off) {
        if (RTX_ANIM_STEP_STAMPS && wbase >= 0 && tm.tl == 0) M.status[wbase + off] = stamp();
    };
    stp(0);
    using P = typename Store<LDS>::P;
    P* src = b ? St.perm[1] : St.perm[0];   // (selects: a dynamic index would put St in scratch)
    P* dst = b ? St.perm[0] : St.perm[1];
    const uint32_t nl = 64u * tm.k;
    // register bins when lanes hold several elements (several waves: from RTX_ANIM_PRIV_MULTI
    // elements per 64 lanes, their LDS atomics on one slot serialise)
    const uint32_t priv_min = MULTI ? (nl * RTX_ANIM_PRIV_MULTI) / 64u : 2u * nl;
    // the node's fields are wave-uniform: scalar registers (the VGPRs are the build's budget)
    uint32_t n = 0, first = 0, depth = 0;
    if (act) {
        n = __builtin_amdgcn_readfirstlane(nodes[t].count);
        first = __builtin_amdgcn_readfirstlane(nodes[t].first);
        depth = __builtin_amdgcn_readfirstlane(nodes[t].depth);
    }
    if constexpr (!MULTI) {
        if (RTX_ANIM_SMALL && act && n <= 128u) {   // one wave, elements in registers
            node_small<LDS>(St, nodes, tm.lane, sl, Lv, rg, t, b, sub, n, first, depth);
            return;
        }
    }
    const uint32_t f0 = first - St.pos0;
    // Subdivide's termination (idxCount <= 8) and the teams with no node: nothing but the copy
    const bool work = act && 3u * n > 8u;
    // 1. slot init
    if (work) {
        if (tm.tl < 6) sl.cb[tm.tl] = tm.tl < 3 ? FLT_MAX : FLT_MIN;
        Slot& si = sl_of(RTX_ANIM_BINS_ATOMIC && MULTI ? tm.wt : 0u);   // per-wave copies (atomic bins)
        const uint32_t li = RTX_ANIM_BINS_ATOMIC && MULTI ? tm.lane : tm.tl, ln = RTX_ANIM_BINS_ATOMIC && MULTI ? 64u : nl;
        if (li < 3 * kBins) (&si.bc[0][0])[li] = 0u;
        for (uint32_t i = li; i < 3 * kBins * 3; i += ln) {
            (&si.bl[0][0][0])[i] = FLT_MAX;
            (&si.bh[0][0][0])[i] = FLT_MIN;
        }
        if (MULTI && tm.tl < 6) {
            (&sl.cmin[0][0])[tm.tl] = min_key_init();
            (&sl.cmax[0][0])[tm.tl] = FLT_MIN;
        }
    }
    tsync<MULTI>();
    stp(1);
    // 2. centroid bounds (FindBestSplitPlane's minBounds / maxBounds, DataTypes.h:404-419)
    if (work) {
        float a0 = FLT_MAX, a1 = FLT_MAX, a2 = FLT_MAX, b0 = FLT_MIN, b1 = FLT_MIN, b2 = FLT_MIN;
        for (uint32_t q = tm.tl; q < n; q += nl) {
            const uint32_t e = src[f0 + q];
            const float x = St.c(0, e), y = St.c(1, e), z = St.c(2, e);
            a0 = fminf(a0, x); a1 = fminf(a1, y); a2 = fminf(a2, z);
            b0 = fmaxf(b0, x); b1 = fmaxf(b1, y); b2 = fmaxf(b2, z);
        }
        float mn3[3] = {a0, a1, a2}, mx3[3] = {b0, b1, b2};
        wred_min(mn3);
        wred_max(mx3);
        a0 = mn3[0]; a1 = mn3[1]; a2 = mn3[2];
        b0 = mx3[0]; b1 = mx3[1]; b2 = mx3[2];
        if (tm.lane == 0) {
            if (MULTI) {
                atomicMin(&sl.cb[0], a0); atomicMin(&sl.cb[1], a1); atomicMin(&sl.cb[2], a2);
                atomicMax(&sl.cb[3], b0); atomicMax(&sl.cb[4], b1); atomicMax(&sl.cb[5], b2);
            } else {
                sl.cb[0] = a0; sl.cb[1] = a1; sl.cb[2] = a2; sl.cb[3] = b0; sl.cb[4] = b1; sl.cb[5] = b2;
            }
        }
    }
    tsync<MULTI>();
    stp(2);
    float minB[3] = {0.f, 0.f, 0.f}, bd[3] = {0.f, 0.f, 0.f}, scale[3] = {0.f, 0.f, 0.f};
    bool live[3] = {false, false, false};
    if (work) {
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
            minB[ax] = sl.cb[ax];
            bd[ax] = sl.cb[3 + ax] - minB[ax];                 // boundsDifference
            live[ax] = !(fabsf(bd[ax]) < FLT_EPSILON);          // else `continue`
            scale[ax] = kBins / bd[ax];
        }
        // 3. bins (DataTypes.h:424-440): idxCount += 3 and the box of the three vertices;
        //    in registers when lanes hold several elements, else LDS atomics per element
        if (!RTX_ANIM_BINS_ATOMIC && n > priv_min) {
#pragma unroll
            for (int ax = 0; ax < 3; ++ax) {
                if (!live[ax]) continue;
                // several waves: each its partial bins in its own slot (the team's is slots[w0]),
                // folded below; one wave: straight into the team's slot
                bins_private(St, src, f0, n, tm.tl, nl, tm.lane, ax, minB[ax], scale[ax], SlotSink{sl_of(tm.wt)});
                stp(10 + ax);
            }
        } else for (uint32_t q = tm.tl; q < n; q += nl) {
            const uint32_t e = src[f0 + q];
            const float l0 = St.lo(0, e), l1 = St.lo(1, e), l2 = St.lo(2, e);
            const float h0 = St.hi(0, e), h1 = St.hi(1, e), h2 = St.hi(2, e);
#pragma unroll
            for (int ax = 0; ax < 3; ++ax) {
                if (!live[ax]) continue;
                const float x = (St.c(ax, e) - minB[ax]) * scale[ax];
                // static_cast<int> of x >= 0 (a NaN x only comes from a NaN vertex: flagged, bin 0)
                int bi = x >= 0.f ? static_cast<int>(fminf(x, 2147483520.f)) : 0;
                bi = kPlanes < bi ? kPlanes : bi;   // std::min(amountOfPlaneBins, binIdx)
                Slot& sw = sl_of(RTX_ANIM_BINS_ATOMIC && MULTI ? tm.wt : 0u);   // per-wave copies: folded below
                atomicAdd(&sw.bc[ax][bi], 3u);
                atomicMin(&sw.bl[ax][bi][0], l0); atomicMin(&sw.bl[ax][bi][1], l1); atomicMin(&sw.bl[ax][bi][2], l2);
                atomicMax(&sw.bh[ax][bi][0], h0); atomicMax(&sw.bh[ax][bi][1], h1); atomicMax(&sw.bh[ax][bi][2], h2);
            }
        }
    }
    tsync<MULTI>();
    if (MULTI) {   // the waves' partial bins (slots w0 .. w0 + k - 1), folded in any order (values only)
        if (work && (RTX_ANIM_BINS_ATOMIC || n > priv_min))
            for (uint32_t i = tm.tl; i < static_cast<uint32_t>(3 * kBins * 7); i += nl) {
                const int ax = static_cast<int>(i / (kBins * 7)), b = static_cast<int>((i / 7) % kBins);
                const int c = static_cast<int>(i % 7);
                if (!live[ax]) continue;
                if (c == 0) {
                    uint32_t sum = 0;
                    for (uint32_t k = 0; k < tm.k; ++k) sum += sl_of(k).bc[ax][b];
                    sl.bc[ax][b] = sum;
                } else if (c < 4) {
                    float v = FLT_MAX;
                    for (uint32_t k = 0; k < tm.k; ++k) v = fminf(v, sl_of(k).bl[ax][b][c - 1]);
                    sl.bl[ax][b][c - 1] = v;
                } else {
                    float v = FLT_MIN;
                    for (uint32_t k = 0; k < tm.k; ++k) v = fmaxf(v, sl_of(k).bh[ax][b][c - 4]);
                    sl.bh[ax][b][c - 4] = v;
                }
            }
        tsync<true>();
    }
    stp(3);
    // 4. the plane sweep
    int axis = 0;
    float pos = 0.f;
    bool split = false;
    if (work) split = plane_sweep(sl, tm.lane, live, minB, bd, n, nodes[t], axis, pos);
    // 5. the partition: per-wave blocks of positions in order
    const uint32_t per = (n + tm.k - 1u) / tm.k;
    const uint32_t lo = min(n, tm.wt * per), hi = min(n, tm.wt * per + per);
    auto small = [&](uint32_t q) { return St.c(axis, src[f0 + q]) < pos; };
    uint32_t S = 0, pL = 0;
    if (split) {
        uint32_t s = 0;
        for (uint32_t base = lo; base < hi; base += 64u) {
            const uint32_t q = base + tm.lane;
            s += __popcll(__ballot(q < hi && small(q)));
        }
        if (MULTI && tm.lane == 0) sl.wc[tm.wt][0] = s;
        S = s;
    }
    if (MULTI) {
        tsync<true>();
        stp(4);
        if (split) {
            S = 0;
            for (uint32_t w = 0; w < tm.k; ++w) S += sl.wc[w][0];
        }
    }
    if (split) pL = S + ((S < n && !small(S)) ? 1u : 0u);
    uint32_t lbase = 0, rbase = 0;
    if (split && MULTI) {
        uint32_t cl = 0, cr = 0;
        for (uint32_t base = lo; base < hi; base += 64u) {
            const uint32_t q = base + tm.lane;
            const bool in = q < hi;
            const bool sm = in && small(q);
            cl += __popcll(__ballot(in && q < pL && !sm));
            cr += __popcll(__ballot(in && q >= pL && sm));
        }
        if (tm.lane == 0) { sl.wc[tm.wt][1] = cl; sl.wc[tm.wt][2] = cr; }
    }
    if (MULTI) {
        tsync<true>();
        stp(5);
        if (split)
            for (uint32_t w = 0; w < tm.k; ++w) {
                if (w < tm.wt) lbase += sl.wc[w][1];
                if (w > tm.wt) rbase += sl.wc[w][2];
            }
    }
    if (split) wave_ranks(St, src, tm.lane, f0, lo, hi, pL, axis, pos, lbase, rbase);
    tsync<MULTI>();
    stp(6);
    if (split) {
        for (uint32_t q = tm.tl; q < n; q += nl) {
            const uint32_t e = src[f0 + q];
            dst[f0 + part_dest(St, f0, n, q, pL, !(St.c(axis, e) < pos))] = static_cast<P>(e);
        }
    } else if (act) {
        for (uint32_t q = tm.tl; q < n; q += nl) dst[f0 + q] = src[f0 + q];   // a leaf: both buffers
    }
    tsync<MULTI>();
    stp(7);
    // leftCount 0 or all: a leaf with the permutation applied (both buffers)
    const bool kids = split && S != 0u && S < n;   // (S <= n always; < n also keeps a child count from wrapping)
    if (split && !kids)
        for (uint32_t q = tm.tl; q < n; q += nl) src[f0 + q] = dst[f0 + q];
    // 6. UpdateNodeBounds of both children (DataTypes.h:310-321), positions in the new order
    if (kids) {   // both children in one pass over the node and one batched wave reduction
        BoundAcc A[2];
        for (uint32_t q = tm.tl; q < n; q += nl) {
            const bool right = q >= S;
            const uint32_t e = dst[f0 + q];
            if (right) A[1].add(St, e, 1u + (q - S));
            else A[0].add(St, e, 1u + q);
        }
        stp(13);
        unsigned long long k[6] = {A[0].k0, A[0].k1, A[0].k2, A[1].k0, A[1].k1, A[1].k2};
        float m[6] = {A[0].m0, A[0].m1, A[0].m2, A[1].m0, A[1].m1, A[1].m2};
        wred_min64(k);
        wred_max(m);
        stp(14);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            A[c].k0 = k[3 * c]; A[c].k1 = k[3 * c + 1]; A[c].k2 = k[3 * c + 2];
            A[c].m0 = m[3 * c]; A[c].m1 = m[3 * c + 1]; A[c].m2 = m[3 * c + 2];
        }
        if (tm.lane == 0) { A[0].put(sl, 0, MULTI); A[1].put(sl, 1, MULTI); }
    }
    tsync<MULTI>();
    stp(8);
    if (kids && tm.wt == 0 && tm.lane == 0) {
        const uint32_t c = atomicAdd(&Lv.ids, 2u);
        TmpNode a{}, bb{};
        for (int q = 0; q < 3; ++q) {
            a.mn[q] = min_key_value(sl.cmin[0][q]); a.mx[q] = sl.cmax[0][q];
            bb.mn[q] = min_key_value(sl.cmin[1][q]); bb.mx[q] = sl.cmax[1][q];
        }
        a.first = first; a.count = S; a.l = -1; a.depth = depth + 1; a.parent = static_cast<int32_t>(t); a.sub = sub;
        bb.first = first + S; bb.count = n - S; bb.l = -1; bb.depth = depth + 1; bb.parent = static_cast<int32_t>(t);
        bb.sub = sub;
        nodes[c] = a;
        nodes[c + 1] = bb;
        nodes[t].l = static_cast<int32_t>(c);
        const uint32_t w = atomicAdd(&Lv.next, 2u);
        rg.nxt[w] = c;
        rg.nxt[w + 1] = c + 1;
        atomicMax(&Lv.nmaxn, max(S, n - S));
    }
    if (MULTI) tsync<true>();   // the slot is free for the next level
    stp(9);
}

// The level loop over a region's list (Lv.K nodes in rg.cur) until no level remains or
// max_levels levels are done (rg.cur then lists the next level's Lv.K nodes).  depth: the level
// of the list's nodes.  lvl_base (optional): the first temp id created while processing each
// level (relative to the first).
template <bool LDS>
__device__ __forceinline__ uint32_t build_levels(const MeshDev& M, const Store<LDS>& St, TmpNode* nodes, Level& Lv,
                                                 Slot* slots, Region& rg,
                                 uint32_t depth, uint32_t max_levels, uint32_t sub, uint32_t* lvl_base, uint32_t lvl_cap,
                                 uint32_t* stamps = nullptr, uint32_t nstamps = 0) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t depth0 = depth;
    for (;; ++depth) {
        const uint32_t K = Lv.K;
        if (K == 0) break;
        if (depth - depth0 >= max_levels) break;
        if (lvl_base && tid == 0 && depth - depth0 < lvl_cap) lvl_base[depth - depth0] = Lv.ids;
        const uint32_t b = depth & 1u;
        // team size: 16 / K waves (a power of two), fewer while the nodes are small
        uint32_t k = 1;
        while (2u * k * K <= static_cast<uint32_t>(kAnimWaves)) k *= 2u;
        while (k > 1u && Lv.maxn < RTX_ANIM_TEAM_ELEMS * k) k /= 2u;
        if (k > 1u) {
            const Team tm{k, (wave / k) * k, wave % k, (wave % k) * 64u + lane, lane};
            const uint32_t j = wave / k;
            node_process<true, LDS>(M, St, nodes, tm, slots, Lv, rg, j < K, j < K ? rg.cur[j] : 0u, b, sub);
        } else {
            const Team tm{1u, wave, 0u, lane, lane};
            for (;;) {
                uint32_t j = 0;
                if (lane == 0) j = atomicAdd(&Lv.take, 1u);
                j = __shfl(j, 0);
                if (j >= K) break;
                node_process<false, LDS>(M, St, nodes, tm, slots, Lv, rg, true, rg.cur[j], b, sub);
            }
        }
        __syncthreads();
        if (tid == 0) {
            if (stamps && depth - depth0 < nstamps) stamps[depth - depth0] = stamp();   // diagnostics: level end
            Lv.K = Lv.next;
            Lv.next = 0;
            Lv.take = 0;
            Lv.maxn = Lv.nmaxn;
            Lv.nmaxn = 0;
        }
        uint32_t* tsw = rg.cur;
        rg.cur = rg.nxt;
        rg.nxt = tsw;
        __syncthreads();
    }
    return depth;
}

// ---- the task queue (MeshDev::q; single threads of a workgroup, after a barrier)
// Publish a task: its words, then the entry's epoch with release semantics at agent scope
// (the writes of the whole workgroup before the barrier become visible with it).
__device__ __forceinline__ void push_task(const Launch& L, const MeshDev& M, uint32_t what, uint32_t ids) {
    const uint32_t j = atomicAdd(&M.q[kQHead], 1u);
    if (j >= kQCap) { atomicOr(&M.status[0], kErrCapacity); return; }   // (cannot happen: kQCap bounds the tasks)
    uint32_t* e = M.q + kQEntries + 4u * j;
    e[0] = what;
    e[1] = ids;
    __threadfence();
    __hip_atomic_store(&e[2], L.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
// temp ids r, r + 1 reserved for a node's children: marked unused until the split writes them
__device__ __forceinline__ void reserve_ids(const MeshDev& M, uint32_t r) {
    for (uint32_t i = r; i < r + 2u && i < static_cast<uint32_t>(kMaxTop); ++i) {
        M.tmp[i].parent = -2;
        M.tmp[i].l = -1;
        M.tmp[i].sub = kMaxSub;
        M.tmp[i].count = 0u;
    }
}
// Node t (n triangles, depth d) becomes subtree f: its descendants get 2 n - 2 temp ids
__device__ __forceinline__ void make_subtree(const Launch& L, const MeshDev& M, uint32_t t, uint32_t n, uint32_t d) {
    const uint32_t f = atomicAdd(&M.status[4], 1u);   // < kMaxSub: every subtree root is a distinct id < kMaxTop
    if (f >= static_cast<uint32_t>(kMaxSub)) { atomicOr(&M.status[0], kErrCapacity); return; }   // (guard only)
    const uint32_t base = atomicAdd(&M.q[kQSubIds], n > 1u ? 2u * n - 2u : 0u);
    M.sub[f] = SubRec{t, base, 0u, d};
    M.tmp[t].sub = f;
    push_task(L, M, f, 0u);
}
// After node (n triangles, depth d) was processed: K = 2 children from temp id c, or a leaf.
// A child of 3 n <= 8 indices is a leaf (Subdivide returns at once), a child above the cut a
// split task (ids for its children reserved now), any other a subtree.  `done` counts the
// triangles whose leaves are final: the workers stop when it reaches T.
// keep (optional): the larger child that is itself a split is not queued but returned in
// keep[0] (its reserved ids in keep[1]; ~0u: none) for the calling workgroup to split next.
__device__ __forceinline__ void dispatch_children(const Launch& L, const MeshDev& M, uint32_t n, uint32_t d, uint32_t K,
                                                  uint32_t c0, uint32_t t_start, uint32_t* keep = nullptr) {
    __threadfence();
    const uint32_t k = atomicAdd(&M.status[6], 1u);
    if (k < 4u) {   // diagnostics: the first four splits' size, start and end
        M.status[16 + k] = n;
        M.status[20 + 2 * k] = t_start;
        M.status[21 + 2 * k] = stamp();
    }
    if (K == 0u) {
        atomicMax(&M.status[1], d);
        done_add(M, n);
        return;
    }
    atomicMax(&M.status[1], d + 1u);
    const uint32_t kc = M.tmp[c0].count >= M.tmp[c0 + 1u].count ? c0 : c0 + 1u;   // the larger child
    for (uint32_t c = c0; c < c0 + 2u; ++c) {
        const uint32_t nc = M.tmp[c].count;
        if (3u * nc <= 8u) {
            done_add(M, nc);
            continue;
        }
        if (nc > L.cut) {
            const uint32_t r = atomicAdd(&M.q[kQTop], 2u);
            reserve_ids(M, r);
            if (r + 2u <= static_cast<uint32_t>(kMaxTop)) {
                if (keep && c == kc) {
                    keep[0] = c;
                    keep[1] = r;
                    continue;
                }
                __threadfence();
                push_task(L, M, 0x80000000u | c, r);
                continue;
            }
        }
        make_subtree(L, M, c, nc, d + 1u);
    }
}

// ============================================================ launch 1: set-up + top levels
template <bool LDS>
__device__ __forceinline__ void top_phase(const Launch& L, const MeshDev& M, Level& Lv, Slot* slots, float* dyn,
                                          uint32_t* s_list) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const float* mat = L.m[blockIdx.x];
    const uint32_t T = M.T, V = M.V;
    const int4* idx = M.idx[L.cur];
    const float4* nrm = M.nrm[L.cur];
    float* soa = M.soa;
    Store<LDS> St;
    if (LDS) {
        using P = typename Store<LDS>::P;
        P* p16 = reinterpret_cast<P*>(dyn + 9 * T);
        St = Store<LDS>{{p16, p16 + T}, p16 + 2 * T, p16 + 3 * T, p16 + 4 * T, dyn, T, 0u};
    } else {
        St = Store<LDS>{{reinterpret_cast<typename Store<LDS>::P*>(M.perm[0]),
                         reinterpret_cast<typename Store<LDS>::P*>(M.perm[1])},
                        reinterpret_cast<typename Store<LDS>::P*>(M.lb), reinterpret_cast<typename Store<LDS>::P*>(M.rs),
                        reinterpret_cast<typename Store<LDS>::P*>(M.rk), soa, T, 0u};
    }
    float* rec = const_cast<float*>(St.rec);
    // ---- UpdateTransforms (DataTypes.h:210-230)
    for (uint32_t v0 = tid; v0 < V; v0 += 4u * kAnimThreads) {   // (four vertices per thread at a time)
        float4 p[4];
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j) {
            const uint32_t v = v0 + j * kAnimThreads;
            p[j] = v < V ? M.pos[v] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j) {
            const uint32_t v = v0 + j * kAnimThreads;
            if (v >= V) continue;
            const float3 t = xform_point(mat, p[j].x, p[j].y, p[j].z);
            M.tpos[v] = make_float4(t.x, t.y, t.z, 0.f);
        }
    }
    __syncthreads();
    // per triangle: transformed normal (input order), centroid, box; the identity permutation;
    // the root's bounds over the input order (BuildBVH, DataTypes.h:294-308)
    // (four triangles per thread at a time: their index and vertex loads issued together)
    BoundAcc A;
    constexpr uint32_t kB = 4;
    for (uint32_t k0 = tid; k0 < T; k0 += kB * kAnimThreads) {
        int4 ii[kB];
        float4 nn[kB], v[kB][3];
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
            const uint32_t k = k0 + j * kAnimThreads;
            ii[j] = k < T ? idx[k] : make_int4(0, 0, 0, 0);
            nn[j] = k < T ? nrm[k] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
            const bool in = k0 + j * kAnimThreads < T;
            v[j][0] = in ? M.tpos[ii[j].x] : make_float4(0.f, 0.f, 0.f, 0.f);
            v[j][1] = in ? M.tpos[ii[j].y] : make_float4(0.f, 0.f, 0.f, 0.f);
            v[j][2] = in ? M.tpos[ii[j].z] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
            const uint32_t k = k0 + j * kAnimThreads;
            if (k >= T) continue;
            const float3 tn = normalized(xform_vector(mat, nn[j].x, nn[j].y, nn[j].z));
            M.tnrm[k] = make_float4(tn.x, tn.y, tn.z, 0.f);
            const float4 v0 = v[j][0], v1 = v[j][1], v2 = v[j][2];
            if (v0.x != v0.x || v0.y != v0.y || v0.z != v0.z || v1.x != v1.x || v1.y != v1.y || v1.z != v1.z ||
                v2.x != v2.x || v2.y != v2.y || v2.z != v2.z)
                atomicOr(&Lv.err, kErrNaN);
            // (v0 + v1 + v2) * 0.3333f, the reference's centroid (DataTypes.h:348, 411-415, 435)
            const float r9[9] = {((v0.x + v1.x) + v2.x) * 0.3333f, ((v0.y + v1.y) + v2.y) * 0.3333f,
                                 ((v0.z + v1.z) + v2.z) * 0.3333f,
                                 rmin(rmin(v0.x, v1.x), v2.x), rmin(rmin(v0.y, v1.y), v2.y), rmin(rmin(v0.z, v1.z), v2.z),
                                 rmax(rmax(v0.x, v1.x), v2.x), rmax(rmax(v0.y, v1.y), v2.y), rmax(rmax(v0.z, v1.z), v2.z)};
#pragma unroll
            for (int c = 0; c < 9; ++c) {
                soa[c * T + k] = r9[c];
                if (LDS) rec[c * T + k] = r9[c];
            }
            St.perm[0][k] = static_cast<typename Store<LDS>::P>(k);
            A.addv(r9[3], r9[4], r9[5], r9[6], r9[7], r9[8], 1u + k);
        }
    }
    A.wave();
    Slot& s0 = slots[0];
    if (tid < 3) { s0.cmin[0][tid] = min_key_init(); s0.cmax[0][tid] = FLT_MIN; }
    __syncthreads();
    if (lane == 0) A.put(s0, 0, true);
    __syncthreads();
    if (tid == 0) {
        TmpNode r{};
        for (int q = 0; q < 3; ++q) { r.mn[q] = min_key_value(s0.cmin[0][q]); r.mx[q] = s0.cmax[0][q]; }
        r.first = 0; r.count = T; r.l = -1; r.depth = 0; r.parent = -1; r.sub = kMaxSub;
        M.tmp[0] = r;
        M.status[kStSetup] = stamp();
    }
    __syncthreads();
    // ---- Subdivide (DataTypes.h:323-389): the root's split here, its descendants as tasks
    if (tid == 0) {
        M.status[0] = Lv.err;
        M.status[1] = 0u;
        M.status[4] = 0u;
        M.status[6] = 0u;
        M.status[kStComplete] = 0u;   // before the first task is published (release on push)
        M.status[kStSub0] = 0xffffffffu;
        M.status[kStSubEnd] = 0u;
        M.q[kQSubIds] = kMaxTop;
    }
    if (T > L.cut && !LDS) {   // the root is a task like any node (records and order in HBM)
        __syncthreads();
        if (tid == 0) {
            M.q[kQTop] = 3u;   // the root's children: ids 1 and 2
            reserve_ids(M, 1u);
            M.status[kStTopDone] = stamp();
            __threadfence();
            push_task(L, M, 0x80000000u, 1u);
        }
    } else if (T > L.cut) {   // (LDS: the records are staged by triangle id already)
        if (tid == 0) {
            M.q[kQTop] = 3u;   // the root's children: ids 1 and 2
            reserve_ids(M, 1u);
            Lv.ids = 1u;
            s_list[0] = 0u;
        }
        __syncthreads();
        Region rg{s_list, s_list + 2};
        if constexpr (LDS) {
            // the root, then the larger child while it is a split task, like run_task (records by
            // triangle id, staged for the whole mesh); each node's range in its new order into both
            // buffers
            uint32_t nc = T, dc = 0, fc = 0, ts = M.status[kStSetup];
            uint32_t* keep = s_list + 4;
            for (;;) {
                rg = Region{s_list, s_list + 2};
                build_levels<LDS>(M, St, M.tmp, Lv, slots, rg, dc, 1u, kMaxSub, nullptr, 0u);
                const uint32_t bc = dc & 1u;
                for (uint32_t k = tid; k < nc; k += kAnimThreads) {
                    const uint32_t v = static_cast<uint32_t>(St.perm[bc ^ 1u][fc + k]);
                    M.perm[bc ^ 1u][fc + k] = v;
                    M.perm[bc][fc + k] = v;
                }
                __syncthreads();
                if (tid == 0) {
                    if (dc == 0) M.status[kStTopDone] = stamp();
                    keep[0] = ~0u;
                    dispatch_children(L, M, nc, dc, Lv.K, rg.cur[0], ts, RTX_ANIM_KEEP_CHILD ? keep : nullptr);
                }
                __syncthreads();
                const uint32_t kt = keep[0], kid = keep[1];
                if (!RTX_ANIM_KEEP_CHILD || kt == ~0u) break;
                dc += 1u;
                nc = M.tmp[kt].count;
                fc = M.tmp[kt].first;
                ts = stamp();
                __syncthreads();
                if (tid == 0) {
                    Lv.K = 1; Lv.next = 0; Lv.take = 0; Lv.maxn = nc; Lv.nmaxn = 0; Lv.ids = kid; Lv.err = 0;
                    s_list[0] = kt;
                }
                __syncthreads();
            }
        }
    } else {
        if (LDS)
            for (uint32_t k = tid; k < T; k += kAnimThreads) M.perm[0][k] = k;
        __syncthreads();
        if (tid == 0) {
            M.q[kQTop] = 1u;
            M.status[kStTopDone] = stamp();
            make_subtree(L, M, 0u, T, 0u);
        }
    }
}

// ============================================================ tasks: one workgroup each
// A node of more than Launch::cut triangles (what: bit 31 | temp id; ids: the two reserved for
// its children), split once by the whole workgroup; or subtree `what`, built level by level.
// LDS = true: the records, permutation and partition scratch staged by local element index
// (a subtree also keeps its nodes in an LDS pool under local ids — 0 its root, 1 .. in
// allocation order — with its level lists, written back under temp ids at the end); false:
// everything in HBM.  One call site of the level loop per storage kind keeps the kernel's code
// small (a single wave walking a level runs cold code otherwise).
constexpr uint32_t kSubLevels = 256;
constexpr uint32_t kPoolMax = 700;   // subtrees staged with their node pool: 50 + 128 + 8 bytes per element
template <bool LDS>
__device__ __forceinline__ void run_task(const Launch& L, const MeshDev& M, uint32_t what, uint32_t ids, Level& Lv,
                                         Slot* slots, uint32_t* lvl_base, float* dyn, uint32_t* s_list) {
    const uint32_t tid = threadIdx.x;
    const uint32_t t_start = stamp();
    const bool split = (what & 0x80000000u) != 0u;
    const uint32_t f = split ? static_cast<uint32_t>(kMaxSub) : what;
    SubRec S0{};
    if (!split) S0 = M.sub[f];
    const uint32_t t = split ? (what & 0x7fffffffu) : S0.root;
    const TmpNode X0 = M.tmp[t];
    const uint32_t D = X0.depth, n = X0.count, b = D & 1u, first = X0.first;
    using P = typename Store<LDS>::P;
    Store<LDS> St;
    uint32_t* gmap = nullptr;
    TmpNode* nodes = M.tmp;
    Region rg = split ? Region{s_list, s_list + 2} : Region{M.lvl[0] + first, M.lvl[1] + first};
    uint32_t root = t, ids0 = split ? ids : S0.base;
    if (LDS) {   // stage by local element index
        gmap = reinterpret_cast<uint32_t*>(dyn + 9 * n);
        P* p16 = reinterpret_cast<P*>(gmap + n);
        St = Store<LDS>{{p16, p16 + n}, p16 + 2 * n, p16 + 3 * n, p16 + 4 * n, dyn, n, first};
        for (uint32_t q = tid; q < n; q += kAnimThreads) {
            const uint32_t g = M.perm[b][first + q];
            gmap[q] = g;
#pragma unroll
            for (int c = 0; c < 9; ++c) dyn[c * n + q] = M.soa[c * M.T + g];
            (b ? St.perm[1] : St.perm[0])[q] = static_cast<P>(q);
        }
        if (!split) {
            nodes = reinterpret_cast<TmpNode*>(dyn + ((50u * n + 15u) & ~15u) / 4u);
            uint32_t* lists = reinterpret_cast<uint32_t*>(nodes + (2u * n - 1u));
            rg = Region{lists, lists + n};
            root = 0u;
            ids0 = 1u;
            if (tid == 0) nodes[0] = X0;
        }
    } else {
        St = Store<LDS>{{reinterpret_cast<P*>(M.perm[0]), reinterpret_cast<P*>(M.perm[1])}, reinterpret_cast<P*>(M.lb),
                        reinterpret_cast<P*>(M.rs), reinterpret_cast<P*>(M.rk), M.soa, M.T, 0u};
    }
    if (tid == 0) {
        if (!split) {
            if (f == 0) {   // subtree 0: staged (and the shader clock counter, diagnostics)
                M.status[29] = stamp();
                M.status[60] = static_cast<uint32_t>(__builtin_amdgcn_s_memtime());
            }
            atomicMin(&M.status[kStSub0], stamp());
        }
        Lv.K = 1; Lv.next = 0; Lv.take = 0; Lv.maxn = n; Lv.nmaxn = 0; Lv.ids = ids0; Lv.err = 0;
        rg.cur[0] = root;
    }
    __syncthreads();
    const uint32_t Dend = build_levels<LDS>(M, St, nodes, Lv, slots, rg, D, split ? 1u : ~0u, f,
                                            split ? nullptr : lvl_base, kSubLevels,
                                            (!split && f == 0) ? M.status + 32 : nullptr, 8u);
    if (split) {
        // Split, then keep splitting the larger child in this workgroup while it is a split task
        // (its records are staged here already: positions relative to St.pos0), the other child
        // queued; each node's range in its new order into both buffers (a leaf child's range is
        // final; the next level rewrites the kept child's).
        uint32_t tc = t, nc = n, dc = D, fc = first, ts = t_start;
        uint32_t* keep = s_list + 4;
        for (;;) {
            const uint32_t bc = dc & 1u, f0c = fc - St.pos0;
            const P* dst = bc ? St.perm[0] : St.perm[1];
            uint32_t* hdst = M.perm[bc ^ 1u];
            for (uint32_t q = tid; q < nc; q += kAnimThreads) {
                const uint32_t v = LDS ? gmap[dst[f0c + q]] : hdst[fc + q];
                if (LDS) hdst[fc + q] = v;
                M.perm[bc][fc + q] = v;
            }
            __syncthreads();
            if (tid == 0) {
                keep[0] = ~0u;
                dispatch_children(L, M, nc, dc, Lv.K, rg.cur[0], ts, RTX_ANIM_KEEP_CHILD ? keep : nullptr);
            }
            __syncthreads();
            const uint32_t kt = keep[0], kid = keep[1];
            if (!RTX_ANIM_KEEP_CHILD || kt == ~0u) return;
            tc = kt;
            dc += 1u;
            nc = M.tmp[tc].count;
            fc = M.tmp[tc].first;
            ts = stamp();
            __syncthreads();   // (everyone has read keep[] and the node)
            if (tid == 0) {
                Lv.K = 1; Lv.next = 0; Lv.take = 0; Lv.maxn = nc; Lv.nmaxn = 0; Lv.ids = kid; Lv.err = 0;
                s_list[0] = tc;
            }
            __syncthreads();
            rg = Region{s_list, s_list + 2};
            build_levels<LDS>(M, St, M.tmp, Lv, slots, rg, dc, 1u, kMaxSub, nullptr, 0u);
        }
    }
    if (f == 0 && tid == 0) M.status[30] = stamp();   // subtree 0: levels done
    if (LDS)   // the final order (every leaf range is current in both buffers) as triangle ids
        for (uint32_t q = tid; q < n; q += kAnimThreads) M.perm[0][first + q] = gmap[St.perm[0][q]];
    // levels D .. Dend - 1 hold nodes: level D the root, level D + r (r >= 1) the ids
    // [lvl_base[r - 1], lvl_base[r])
    const uint32_t nlev = Dend - D, idend = Lv.ids;
    const bool ranks_ok = nlev < kSubLevels;
    if (tid == 0 && ranks_ok) lvl_base[nlev] = idend;
    __syncthreads();
    auto lvl_lo = [&](uint32_t r) { return r == 0 ? root : lvl_base[r - 1]; };
    auto lvl_hi = [&](uint32_t r) { return r == 0 ? root + 1u : lvl_base[r]; };
    // split counts bottom-up, then the DFS preorder ranks of the split nodes top-down
    // (relative to the subtree root: its descendants' ranks follow its own)
    if (ranks_ok) {
        for (int r = static_cast<int>(nlev) - 1; r >= 0; --r) {
            for (uint32_t u = lvl_lo(r) + tid; u < lvl_hi(r); u += kAnimThreads) {
                const int32_t l = nodes[u].l;
                nodes[u].splits = l >= 0 ? 1u + nodes[l].splits + nodes[l + 1].splits : 0u;
            }
            __syncthreads();
        }
        if (tid == 0) nodes[root].rank = 0u;
        __syncthreads();
        for (uint32_t r = 0; r < nlev; ++r) {
            for (uint32_t u = lvl_lo(r) + tid; u < lvl_hi(r); u += kAnimThreads) {
                const int32_t l = nodes[u].l;
                if (l < 0) continue;
                const uint32_t rk = nodes[u].rank;
                nodes[l].rank = rk + 1u;
                nodes[l + 1].rank = rk + 1u + nodes[l].splits;
            }
            __syncthreads();
        }
    }
    if (LDS) {   // the pool under temp ids: local 0 is S0.root, local i >= 1 is S0.base + i - 1
        auto gid = [&](int32_t i) -> int32_t {
            return i < 0 ? i : (i == 0 ? static_cast<int32_t>(S0.root) : static_cast<int32_t>(S0.base) + i - 1);
        };
        for (uint32_t i = 1u + tid; i < idend; i += kAnimThreads) {
            TmpNode X = nodes[i];
            X.l = gid(X.l);
            X.parent = gid(X.parent);
            M.tmp[S0.base + i - 1u] = X;
        }
        if (tid == 0) {
            M.tmp[S0.root].l = gid(nodes[0].l);
            M.tmp[S0.root].splits = nodes[0].splits;
            M.tmp[S0.root].rank = nodes[0].rank;
        }
    }
    if (f == 0 && tid == 0) {   // subtree 0: ranks done
        M.status[31] = stamp();
        M.status[61] = static_cast<uint32_t>(__builtin_amdgcn_s_memtime());
    }
    if (tid == 0 && f < 16u) {   // diagnostics: subtrees 0-7 start / end, subtrees 0-15 sizes
        if (f < 8u) { M.status[80 + 2 * f] = t_start; M.status[81 + 2 * f] = stamp(); }
        M.status[96 + f] = n;
    }
    __syncthreads();
    if (tid == 0) {
        M.sub[f].nalloc = idend - ids0;
        M.sub[f].maxd = Dend - 1u;
        if (!ranks_ok) atomicOr(&M.status[0], kErrDepth);
        atomicMax(&M.status[kStSubEnd], stamp());
        __threadfence();
        done_add(M, n);
    }
}

// One kernel: workgroup (mesh, 0) runs the set-up and the root's split, then it and workgroups
// (mesh, 1 .. kWorkers) take tasks from the mesh's queue until every triangle is in a final
// leaf.  A worker takes the next entry index (atomic tail) and waits for its epoch (bounded);
// a task is pushed only by a workgroup that runs, after its writes, so a waiting worker always
// has a running producer (the producers of all meshes come first in dispatch order,
// blockIdx.x fastest).  One launch with the waits in it instead of a kernel per level: a kernel
// boundary cost ~100 us before the next workgroups ran (the idle XCDs' start-up, profiles/r03).
// A waiting worker gives up after Launch::wait_ticks (kWaitTicks = 200 ms of s_memrealtime by
// default, rtx_anim.h): a stuck build reports, never hangs.  (A worker that gives up on a real task
// leaves it unbuilt, so the tree is incomplete: kErrTimeout, and the output launch disables the
// mesh; one that gave up on an index no task takes lost nothing: the output launch sees every
// triangle placed, kStComplete, and keeps the mesh, see rtx_anim_out)
__global__ void __launch_bounds__(kAnimThreads) rtx_anim_build(const Launch L) {
    const MeshDev& M = L.meshes[blockIdx.x];
    extern __shared__ float s_dyn[];
    __shared__ Level Lv;
    __shared__ Slot slots[kAnimWaves];
    __shared__ uint32_t lvl_base[kSubLevels + 1];
    __shared__ uint32_t s_list[8];   // level lists of a split task (4) and its kept child (2)
    __shared__ uint32_t s_task[3];
    const uint32_t tid = threadIdx.x;
    if (M.status[7]) {
        // An earlier update left this mesh's tree incomplete (status word 7, sticky): its order of
        // triangles is no longer the reference's (each build permutes the previous order,
        // DataTypes.h:335-363), so no later update can be exact.  Build nothing; the output launch
        // keeps the mesh disabled and every update reports the error (re-register to recover).
        if (blockIdx.y == 0 && tid == 0) {
            M.status[0] = M.status[7];
            M.status[kStComplete] = 0u;
        }
        return;
    }
    if (blockIdx.y == 0) {
        if (tid == 0) {
            M.status[kStTop0] = stamp();
            M.status[58] = static_cast<uint32_t>(__builtin_amdgcn_s_memtime());   // diagnostics: shader clock
            Lv.K = 1; Lv.next = 0; Lv.take = 0; Lv.maxn = M.T; Lv.nmaxn = 0; Lv.ids = 1; Lv.err = 0;
        }
        __syncthreads();
        if (M.T <= L.top_lds) top_phase<true>(L, M, Lv, slots, s_dyn, s_list);
        else top_phase<false>(L, M, Lv, slots, s_dyn, s_list);
        __syncthreads();
    } else if (tid == 0 && blockIdx.y <= 16u) {
        M.status[111 + blockIdx.y] = stamp();   // diagnostics: workgroup entry (workers 1-16)
    }
    for (;;) {
        if (tid == 0) {
            const uint32_t i = atomicAdd(&M.q[kQTail], 1u);
            const uint32_t* e = M.q + kQEntries + 4u * i;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t go = 0;
            // relaxed polls (an acquire per poll would invalidate this XCD's L2 under the
            // running workgroups), one acquire fence once the entry is seen
            for (;;) {
                if (i < kQCap && __hip_atomic_load(&e[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == L.epoch) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    if ((L.debug & kDbgDropEntry) && i == 0u) {   // tests: lose a real task
                        atomicOr(&M.status[0], kErrTimeout);
                        break;
                    }
                    go = 1;
                    s_task[0] = e[0];
                    s_task[1] = e[1];
                    break;
                }
                if (__hip_atomic_load(&M.q[kQDone], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= M.T) {
                    if (L.debug & kDbgLateTimeout) atomicOr(&M.status[0], kErrTimeout);   // tests
                    break;
                }
                __builtin_amdgcn_s_sleep(RTX_ANIM_POLL_SLEEP);
                if (__builtin_amdgcn_s_memrealtime() - t0 > L.wait_ticks) {
                    atomicOr(&M.status[0], kErrTimeout);
                    break;
                }
            }
            s_task[2] = go;
        }
        __syncthreads();
        const uint32_t what = s_task[0], ids = s_task[1], go = s_task[2];
        __syncthreads();
        if (!go) return;
        const bool split = (what & 0x80000000u) != 0u;
        const uint32_t n = M.tmp[split ? (what & 0x7fffffffu) : M.sub[what].root].count;
        if (L.sub_lds && n <= (split ? kSubLdsMax : kPoolMax))
            run_task<true>(L, M, what, ids, Lv, slots, lvl_base, s_dyn, s_list);
        else
            run_task<false>(L, M, what, ids, Lv, slots, lvl_base, s_dyn, s_list);
        __syncthreads();
    }
}

// ============================================================ launch 3: numbering and output
// The split-rendering frontier of rtx_hip.hip build_parts — split the part with the most
// triangles (the first in frontier order on a tie) while fewer than part_cap parts exist and a
// part is an internal node less than 31 levels deep — and the status words; workgroup
// kOutGroups of the output launch, beside the records.
//
// The greedy's choices are the first part_cap - 1 eligible nodes (internal, depth < 31) in
// (count descending, DFS preorder) order: a child holds strictly fewer triangles than its
// parent (both sides of a split are nonempty), so when a node comes first in that order all its
// ancestors have been split and it is in the frontier, where frontier order is DFS order.  So
// the split set is a threshold selection — every eligible node with count > c*, and of those
// with count == c* the lowest DFS ranks (their parents all have count > c*: at most 2 (m - 1)
// + 1 of them) — found from a histogram of counts.  The parts are the unsplit children of the
// split nodes (the root alone if none), ordered by their root paths read as bit strings.
// Meshes above Launch::frontier_max (<= kFrontierHistMax) triangles keep the serial greedy over HBM.
constexpr uint32_t kFrontierBitWords = (2u * kFrontierHistMax + kMaxTop + 31u) / 32u;
__device__ __forceinline__ void out_frontier(const Launch& L, const MeshDev& M, const uint32_t* s_vbase,
                                             const uint32_t* s_base, const uint32_t* s_rank,
                                             const uint32_t* s_subroot, uint32_t ntop, uint32_t nsub, uint32_t nvirt,
                                             uint32_t maxd, uint32_t nused, uint32_t root_count, int32_t root_l) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t T = M.T, cap = M.part_cap;
    auto tmap = [&](uint32_t v) -> uint32_t {   // virtual index -> temp id (the records' enumeration)
        if (v < ntop) return v;
        uint32_t f = 0, hi = nsub;   // the last subtree whose range starts at or before v
        while (hi - f > 1u) {
            const uint32_t mid = (f + hi) >> 1;
            if (s_vbase[mid] <= v) f = mid;
            else hi = mid;
        }
        return s_base[f] + (v - s_vbase[f]);
    };
    auto rank_abs = [&](uint32_t t, const TmpNode& X) -> uint32_t {
        return t < ntop ? s_rank[t] : s_rank[s_subroot[X.sub]] + X.rank;
    };
    auto ref_of = [&](uint32_t t, const TmpNode& X) -> uint32_t {
        if (t == 0) return 0u;
        const uint32_t p = static_cast<uint32_t>(X.parent);
        const TmpNode P = M.tmp[p];
        return 1u + 2u * rank_abs(p, P) + (t == static_cast<uint32_t>(P.l) + 1u ? 1u : 0u);
    };
    __shared__ uint32_t s_fr[kMaxAnimParts + 1][4];   // parts: temp id, path bits, depth, sort key
    __shared__ uint32_t s_nfr;
    const uint32_t msplit = cap > 0u ? cap - 1u : 0u;   // splits wanted
    if (T <= min(L.frontier_max, kFrontierHistMax)) {
        __shared__ uint32_t s_hist[kFrontierHistMax + 1];
        __shared__ uint32_t s_bits[kFrontierBitWords];   // split set by temp id (< kMaxTop + 2 T)
        __shared__ uint32_t s_wsum[kAnimWaves];
        __shared__ uint32_t s_sel[kMaxAnimParts], s_pidx[kMaxAnimParts], s_dep[kMaxAnimParts], s_path[kMaxAnimParts];
        __shared__ int32_t s_sl[kMaxAnimParts];
        __shared__ uint32_t s_tie[2 * kMaxAnimParts][2];
        __shared__ uint32_t s_nsel, s_ntie, s_cstar, s_take, s_total, s_ncand;
        __shared__ uint32_t s_cand[kFrontierHistMax];   // the eligible nodes (split ones: fewer than T), temp id
        __shared__ uint16_t s_ccnt[kFrontierHistMax];   // and count
        for (uint32_t i = tid; i <= T; i += kAnimThreads) s_hist[i] = 0u;
        for (uint32_t i = tid; i < kFrontierBitWords; i += kAnimThreads) s_bits[i] = 0u;
        if (tid == 0) { s_nsel = 0; s_ntie = 0; s_cstar = ~0u; s_take = 0; s_total = 0; s_ncand = 0; }
        __syncthreads();
        for (uint32_t v = tid; v < nvirt; v += kAnimThreads) {
            const uint32_t t = tmap(v);
            const TmpNode& X = M.tmp[t];
            if (X.l >= 0 && X.depth < 31u) {
                const uint32_t cnt = X.count;
                atomicAdd(&s_hist[cnt], 1u);
                const uint32_t i = atomicAdd(&s_ncand, 1u);
                s_cand[i] = t;
                s_ccnt[i] = static_cast<uint16_t>(cnt);
            }
        }
        __syncthreads();
        // c*: the count where the suffix sums of the histogram reach msplit
        const uint32_t per = (T + 1u + kAnimThreads - 1u) / kAnimThreads;
        const uint32_t b0 = min(T + 1u, tid * per), b1 = min(T + 1u, b0 + per);
        uint32_t own = 0;
        for (uint32_t b = b0; b < b1; ++b) own += s_hist[b];
        uint32_t x = own;   // sum over lanes >= lane of the wave
        for (uint32_t off = 1; off < 64u; off <<= 1) {
            const uint32_t y = __shfl_down(x, off);
            if (lane + off < 64u) x += y;
        }
        if (lane == 0) s_wsum[wave] = x;
        __syncthreads();
        uint32_t run = x - own;   // eligible nodes in the bins above this thread's
        for (uint32_t w = wave + 1u; w < static_cast<uint32_t>(kAnimWaves); ++w) run += s_wsum[w];
        if (tid == 0) s_total = run + own;
        for (uint32_t b = b1; b > b0;) {
            --b;
            const uint32_t h = s_hist[b];
            if (run < msplit && run + h >= msplit) { s_cstar = b; s_take = msplit - run; }
            run += h;
        }
        __syncthreads();
        // every eligible node if there are no more than msplit (c* stays ~0u)
        const uint32_t cstar = s_total <= msplit ? 0u : s_cstar;
        const bool all = s_total <= msplit;
        const uint32_t ncand = s_ncand;
        for (uint32_t v = tid; v < ncand; v += kAnimThreads) {
            const uint32_t t = s_cand[v], cnt = s_ccnt[v];
            if (all || cnt > cstar) {
                s_sel[atomicAdd(&s_nsel, 1u)] = t;
                atomicOr(&s_bits[t >> 5], 1u << (t & 31u));
            } else if (cnt == cstar) {
                const uint32_t i = atomicAdd(&s_ntie, 1u);
                s_tie[i][0] = t;
                s_tie[i][1] = rank_abs(t, M.tmp[t]);
            }
        }
        __syncthreads();
        if (!all) {   // of the ties, the s_take lowest DFS ranks
            const uint32_t nt = s_ntie;
            if (tid < nt) {
                const uint32_t r = s_tie[tid][1];
                uint32_t below = 0;
                for (uint32_t j = 0; j < nt; ++j) below += s_tie[j][1] < r ? 1u : 0u;
                if (below < s_take) {
                    const uint32_t t = s_tie[tid][0];
                    s_sel[atomicAdd(&s_nsel, 1u)] = t;
                    atomicOr(&s_bits[t >> 5], 1u << (t & 31u));
                }
            }
            __syncthreads();
        }
        const uint32_t nsel = s_nsel;
        if (tid < nsel) {   // each split node's parent in the list, depth, left child, side
            const uint32_t t = s_sel[tid];
            const TmpNode X = M.tmp[t];
            uint32_t pi = ~0u;
            for (uint32_t j = 0; j < nsel; ++j)
                if (X.parent >= 0 && s_sel[j] == static_cast<uint32_t>(X.parent)) pi = j;
            const bool right = X.parent >= 0 && t == static_cast<uint32_t>(M.tmp[X.parent].l) + 1u;
            s_pidx[tid] = pi;
            s_dep[tid] = X.depth;
            s_sl[tid] = X.l;
            s_path[tid] = right ? 1u : 0u;   // own side for now
        }
        if (tid == 0) s_nfr = 0;
        __syncthreads();
        uint32_t path = 0;
        if (tid < nsel)   // root path: the side of each split ancestor at its parent's depth
            for (uint32_t p = tid, it = 0; it < 32u && p < nsel && s_dep[p] > 0u; p = s_pidx[p], ++it)   // (bounded)
                path |= s_path[p] << (s_dep[p] - 1u);
        __syncthreads();
        if (tid < nsel) {
            const uint32_t d = s_dep[tid], l = static_cast<uint32_t>(s_sl[tid]);
            for (uint32_t c = 0; c < 2u; ++c) {
                const uint32_t ch = l + c;
                if (s_bits[ch >> 5] & (1u << (ch & 31u))) continue;
                const uint32_t k = atomicAdd(&s_nfr, 1u);
                const uint32_t pb = path | (c << d);
                s_fr[k][0] = ch; s_fr[k][1] = pb; s_fr[k][2] = d + 1u; s_fr[k][3] = __brev(pb);
            }
        }
        if (tid == 0 && nsel == 0) { s_fr[0][0] = 0; s_fr[0][1] = 0; s_fr[0][2] = 0; s_fr[0][3] = 0; s_nfr = 1; }
        __syncthreads();
        // frontier order: the parts' root paths as bit strings (distinct for disjoint subtrees)
        const uint32_t nf = s_nfr;
        uint32_t mine[3] = {0, 0, 0}, pos = 0;
        if (tid < nf) {
            const uint32_t key = s_fr[tid][3];
            for (uint32_t j = 0; j < nf; ++j) pos += s_fr[j][3] < key ? 1u : 0u;
            mine[0] = s_fr[tid][0]; mine[1] = s_fr[tid][1]; mine[2] = s_fr[tid][2];
        }
        __syncthreads();
        if (tid < nf) { s_fr[pos][0] = mine[0]; s_fr[pos][1] = mine[1]; s_fr[pos][2] = mine[2]; }
        __syncthreads();
    } else {
        if (wave != 0) return;
        // the serial greedy: entries (temp id, path bits, depth, count, left child) in frontier order
        __shared__ uint32_t s_fs[kMaxAnimParts + 1][5];
        if (lane == 0) {
            s_fs[0][0] = 0; s_fs[0][1] = 0; s_fs[0][2] = 0; s_fs[0][3] = root_count;
            s_fs[0][4] = static_cast<uint32_t>(root_l);
            s_nfr = 1;
        }
        __builtin_amdgcn_wave_barrier();
        for (;;) {
            const uint32_t nf = s_nfr;
            if (nf >= cap) break;
            uint32_t key = 0, at = ~0u;   // count + 1 of an eligible entry (0: none), its index
            for (uint32_t k = lane; k < nf; k += 64u) {
                const uint32_t kk = (static_cast<int32_t>(s_fs[k][4]) >= 0 && s_fs[k][2] < 31u) ? s_fs[k][3] + 1u : 0u;
                if (kk > key) { key = kk; at = k; }
            }
            for (uint32_t off = 32; off > 0; off >>= 1) {   // max key, lowest index
                const uint32_t ok = __shfl_xor(key, off), oa = __shfl_xor(at, off);
                if (ok > key || (ok == key && oa < at)) { key = ok; at = oa; }
            }
            if (key == 0u) break;
            const uint32_t e1 = s_fs[at][1], e2 = s_fs[at][2], l = s_fs[at][4];
            // entries after `at` move up by one; reads complete before the writes
            uint32_t v[2][5];
            for (int h = 0; h < 2; ++h) {
                const uint32_t k = lane + 64u * h;
                if (k < nf)
                    for (int c = 0; c < 5; ++c) v[h][c] = s_fs[k][c];
            }
            __builtin_amdgcn_wave_barrier();
            for (int h = 0; h < 2; ++h) {
                const uint32_t k = lane + 64u * h;
                if (k < nf && k > at)
                    for (int c = 0; c < 5; ++c) s_fs[k + 1][c] = v[h][c];
            }
            if (lane == 0) {
                const TmpNode A = M.tmp[l], B = M.tmp[l + 1u];
                s_fs[at][0] = l; s_fs[at][1] = e1; s_fs[at][2] = e2 + 1u; s_fs[at][3] = A.count;
                s_fs[at][4] = static_cast<uint32_t>(A.l);
                s_fs[at + 1][0] = l + 1u; s_fs[at + 1][1] = e1 | (1u << e2); s_fs[at + 1][2] = e2 + 1u;
                s_fs[at + 1][3] = B.count; s_fs[at + 1][4] = static_cast<uint32_t>(B.l);
                s_nfr = nf + 1u;
            }
            __builtin_amdgcn_wave_barrier();
        }
        const uint32_t nf = s_nfr;
        for (uint32_t k = lane; k < nf; k += 64u) {
            s_fr[k][0] = s_fs[k][0]; s_fr[k][1] = s_fs[k][1]; s_fr[k][2] = s_fs[k][2];
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (wave != 0) return;
    const Image& I = L.img;
    const uint32_t nf = s_nfr;
    // A tree deeper than the render kernel's DFS stack must never reach it (its pushes are
    // unchecked): the mesh is disabled in this image — no frontier parts, node count 0, so
    // mesh_traverse / part_traverse skip it — and the update reports kErrDepth.
    const bool too_deep = maxd >= L.depth_limit || (M.status[0] & kErrDepth);
    for (uint32_t k = lane; k < M.part_cap; k += 64u) {
        int4 e = make_int4(-1, 0, 0, 0);
        if (k < nf && !too_deep) {
            const uint32_t t = s_fr[k][0];
            const TmpNode X = M.tmp[t];
            e = make_int4(static_cast<int>(M.mesh), static_cast<int>(M.root + ref_of(t, X)), static_cast<int>(s_fr[k][1]),
                          static_cast<int>(s_fr[k][2]));
        }
        I.parts[M.part0 + k] = e;
    }
    if (lane == 0) {
        uint32_t err = M.status[0];
        if (err & kErrTimeout) {   // (complete, or rtx_anim_out would not have come here): spurious
            err &= ~kErrTimeout;
            M.status[kStComplete] |= 2u;
        }
        if (too_deep) err |= kErrDepth;
        const uint32_t used = nused;   // nodesUsed
        M.status[0] = err;
        M.status[1] = maxd;
        M.status[2] = used;
        // the mesh record's node count (0: disabled, see too_deep)
        I.meshes[M.mesh].y = too_deep ? 0 : static_cast<int>(used);
        M.status[3] = nf;
        M.status[5] = ntop;
        // the next update's queue starts empty (every build workgroup has ended: kernel order)
        M.q[kQHead] = 0u;
        M.q[kQTail] = 0u;
        M.q[kQDone] = 0u;
        M.status[kStFrontier] = stamp();
    }
}

__global__ void __launch_bounds__(kAnimThreads) rtx_anim_out(const Launch L) {
    const MeshDev& M = L.meshes[blockIdx.y];
    const uint32_t g = blockIdx.x, tid = threadIdx.x;
    const uint32_t T = M.T;
    // Incomplete: a capacity guard fired, or a worker gave up and not every triangle reached a
    // final leaf (kStComplete: a timeout on an index no task takes loses nothing).  Every workgroup
    // decides alike: kStComplete is final once the build launch has ended, and the frontier
    // workgroup clears the timeout bit only when the tree is complete (then either reading of
    // status word 0 keeps the mesh).
    const uint32_t err0 = M.status[0];
    if ((err0 & kErrCapacity) || ((err0 & kErrTimeout) && !(M.status[kStComplete] & 1u))) {
        // The build left the tree incomplete: none of its numbering, records or frontier is
        // written — their inputs may be stale — and the mesh is disabled in the image (the
        // update's template copy leaves its node region empty): no frontier parts, node count 0,
        // so the render kernel skips it.
        if (g == kOutGroups) {
            for (uint32_t k = tid; k < M.part_cap; k += kAnimThreads) L.img.parts[M.part0 + k] = make_int4(-1, 0, 0, 0);
            if (tid == 0) {
                L.img.meshes[M.mesh].y = 0;
                M.status[7] |= M.status[0] & (kErrTimeout | kErrCapacity);   // sticky: see rtx_anim_build
                M.status[1] = 0u;
                M.status[2] = 0u;
                M.status[3] = 0u;
                M.q[kQHead] = 0u;
                M.q[kQTail] = 0u;
                M.q[kQDone] = 0u;
            }
        }
        return;
    }
    const uint32_t nsub = M.status[4], ntop = min(M.q[kQTop], static_cast<uint32_t>(kMaxTop));
    __shared__ int32_t s_l[kMaxTop];
    __shared__ uint32_t s_split[kMaxTop], s_rank[kMaxTop], s_count[kMaxTop];
    __shared__ uint32_t s_subroot[kMaxSub], s_base[kMaxSub], s_nalloc[kMaxSub], s_smaxd[kMaxSub], s_vbase[kMaxSub + 1];
    __shared__ uint8_t s_isroot[kMaxTop], s_depth[kMaxTop];
    __shared__ uint32_t s_maxd, s_dmax;
    if (g == 0 && tid == 0) M.status[kStOut0] = stamp();
    // ---- the task-split nodes' split counts (bottom-up, subtree roots from their builds) and ranks
    if (tid == 0) { s_maxd = M.status[1]; s_dmax = 0u; }
    __syncthreads();
    for (uint32_t t = tid; t < ntop; t += kAnimThreads) {
        const TmpNode X = M.tmp[t];
        s_l[t] = X.l;
        s_count[t] = X.count;
        s_isroot[t] = X.sub < static_cast<uint32_t>(kMaxSub) ? 1 : 0;
        s_split[t] = s_isroot[t] ? X.splits : 0u;   // a subtree root: its own build's count
        const uint32_t d = X.parent == -2 ? 0u : X.depth;   // (an unused reserved id: no depth)
        s_depth[t] = static_cast<uint8_t>(d);
        atomicMax(&s_dmax, d);
    }
    for (uint32_t f = tid; f < nsub; f += kAnimThreads) {
        const SubRec sr = M.sub[f];
        s_subroot[f] = sr.root; s_base[f] = sr.base; s_nalloc[f] = sr.nalloc; s_smaxd[f] = sr.maxd;
        atomicMax(&s_maxd, sr.maxd);
    }
    __syncthreads();
    // level by level (a task-split node's depth < 256: the build's depth limit)
    const uint32_t dmax = min(s_dmax, 255u);   // (s_depth is 8-bit: task-split nodes are < 256 levels deep)
    for (int d = static_cast<int>(dmax); d >= 0; --d) {
        for (uint32_t t = tid; t < ntop; t += kAnimThreads) {
            const int32_t l = s_l[t];
            if (s_depth[t] == static_cast<uint32_t>(d) && !s_isroot[t])
                s_split[t] = l >= 0 ? 1u + s_split[l] + s_split[l + 1] : 0u;
        }
        __syncthreads();
    }
    if (tid == 0) s_rank[0] = 0u;
    __syncthreads();
    for (uint32_t d = 0; d <= dmax; ++d) {
        for (uint32_t t = tid; t < ntop; t += kAnimThreads) {
            const int32_t l = s_l[t];
            if (s_depth[t] == d && l >= 0 && !s_isroot[t]) {   // a subtree root's children are subtree nodes
                s_rank[l] = s_rank[t] + 1u;
                s_rank[l + 1] = s_rank[t] + 1u + s_split[l];
            }
        }
        __syncthreads();
    }
    // the subtrees' virtual index bases: an exclusive scan of nalloc (one wave, kMaxSub / 64 per lane)
    if (tid < 64u) {
        constexpr uint32_t kPer = (kMaxSub + 63) / 64;
        uint32_t v[kPer], sum = 0;
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const uint32_t f = tid * kPer + i;
            v[i] = f < nsub ? s_nalloc[f] : 0u;
            sum += v[i];
        }
        uint32_t incl = sum;
        for (uint32_t o = 1; o < 64u; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (tid >= o) incl += y;
        }
        uint32_t base = ntop + incl - sum;
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const uint32_t f = tid * kPer + i;
            if (f < nsub) s_vbase[f] = base;
            base += v[i];
            if (f + 1u == nsub) s_vbase[nsub] = base;
        }
        if (nsub == 0u && tid == 0) s_vbase[0] = ntop;
    }
    __syncthreads();
    if (g == kOutGroups && tid == 0) M.status[kStRanks] = stamp();
    // absolute DFS rank of a split node (temp id t)
    auto rank_abs = [&](uint32_t t, const TmpNode& X) -> uint32_t {
        return t < ntop ? s_rank[t] : s_rank[s_subroot[X.sub]] + X.rank;
    };
    // index in the reference's node array: the root 0, the children of the split ranked r at 1 + 2r, 2 + 2r
    auto ref_of = [&](uint32_t t, const TmpNode& X) -> uint32_t {
        if (t == 0) return 0u;
        const uint32_t p = static_cast<uint32_t>(X.parent);
        const TmpNode P = M.tmp[p];
        return 1u + 2u * rank_abs(p, P) + (t == static_cast<uint32_t>(P.l) + 1u ? 1u : 0u);
    };
    const Image& I = L.img;
    const uint32_t nvirt = s_vbase[nsub];
    if (g == kOutGroups) {   // the frontier and the status words, beside the records
        out_frontier(L, M, s_vbase, s_base, s_rank, s_subroot, ntop, nsub, nvirt, s_maxd, 1u + 2u * s_split[0],
                     s_count[0], s_l[0]);
        return;
    }
    const uint32_t stride = kOutGroups * kAnimThreads;
    // ---- the reference's node array (fields the reference writes) and the render records
    for (uint32_t v = g * kAnimThreads + tid; v < nvirt; v += stride) {
        uint32_t t = v;
        if (v >= ntop) {
            uint32_t f = 0, hi = nsub;   // the last subtree whose range starts at or before v
            while (hi - f > 1u) {
                const uint32_t mid = (f + hi) >> 1;
                if (s_vbase[mid] <= v) f = mid;
                else hi = mid;
            }
            t = s_base[f] + (v - s_vbase[f]);
        }
        const TmpNode X = M.tmp[t];
        if (X.parent == -2) continue;   // an id reserved for children of a node that did not split
        const uint32_t ref = ref_of(t, X);
        rtx_bvh_node& R = M.ref[ref];
#pragma unroll
        for (int c = 0; c < 3; ++c) { R.min[c] = X.mn[c]; R.max[c] = X.mx[c]; }
        R.first_idx = 3u * X.first;
        const bool split = X.l >= 0;
        R.idx_count = split ? 0u : 3u * X.count;
        const uint32_t lref = split ? 1u + 2u * rank_abs(t, X) : 0u;
        if (split) R.left_node = lref;
        else if (t == 0) R.left_node = 0u;   // BuildBVH resets the root's leftNode
        const uint32_t link = split ? (M.root + lref) * 32u : (M.tri0 + X.first) * 64u;
        const float4 a = make_float4(X.mn[0], X.mx[0], X.mn[1], X.mx[1]);
        const float4 b = make_float4(X.mn[2], X.mx[2], fbits(link), fbits(split ? 0u : X.count));
        const size_t slot = static_cast<size_t>(M.root) + ref;
        const int copies = I.oct_bytes ? 8 : 1;
        for (int k = 0; k < copies; ++k) {   // copy k stores (hi, lo) on the axes set in k
            float4* dn = reinterpret_cast<float4*>(reinterpret_cast<char*>(I.nodes) + static_cast<size_t>(k) * I.oct_bytes);
            const bool sx = k & 1, sy = k & 2, sz = k & 4;
            dn[2 * slot] = make_float4(sx ? a.y : a.x, sx ? a.x : a.y, sy ? a.w : a.z, sy ? a.z : a.w);
            dn[2 * slot + 1] = make_float4(sz ? b.y : b.x, sz ? b.x : b.y, b.z, b.w);
        }
    }
    // ---- the permuted state and the triangle records
    const uint32_t* fin = M.perm[0];   // every leaf range is current in both buffers
    const int4* idx = M.idx[L.cur];
    const float4* nrm = M.nrm[L.cur];
    int4* idx_out = M.idx[L.cur ^ 1u];
    float4* nrm_out = M.nrm[L.cur ^ 1u];
    for (uint32_t k = g * kAnimThreads + tid; k < T; k += stride) {
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
    if (g == 0 && tid == 0) M.status[57] = stamp();   // workgroup 0: records written
}

}  // namespace

hipError_t launch_build(const Launch& L, hipStream_t stream) {
    if (L.n == 0) return hipSuccess;
    const uint32_t dyn = std::max(L.top_lds * kLdsBytesTop, L.sub_lds ? kSubLdsMax * kLdsBytesSub : 0u);
    if (dyn > 64u * 1024u) {   // dynamic LDS above 64 KB needs the attribute
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(rtx_anim_build),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(dyn));
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(rtx_anim_build, dim3(L.n, 1 + kWorkers), dim3(kAnimThreads), dyn, stream, L);
    hipLaunchKernelGGL(rtx_anim_out, dim3(kOutGroups + 1, L.n), dim3(kAnimThreads), 0, stream, L);
    return hipGetLastError();
}

}  // namespace rtxa
