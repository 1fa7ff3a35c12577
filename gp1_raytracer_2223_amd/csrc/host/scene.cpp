// scene.cpp — host scene model (see scene.h).  Build with -ffp-contract=off.
#include "scene.h"

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <utility>

#include <emmintrin.h>

namespace rtx {

// ---------------------------------------------------------------- TriangleMesh
void TriangleMesh::AppendTriangle(const Vec3& v0, const Vec3& v1, const Vec3& v2) {
    // dae::Triangle(v0, v1, v2) computes its normal (DataTypes.h:85-91), then
    // AppendTriangle pushes 3 fresh vertices + 3 indices + the normal (:158-176).
    const Vec3 normal = Vec3::Cross(v1 - v0, v2 - v0).Normalized();
    int32_t start = static_cast<int32_t>(positions.size());
    positions.push_back(v0); positions.push_back(v1); positions.push_back(v2);
    indices.push_back(start); indices.push_back(start + 1); indices.push_back(start + 2);
    normals.push_back(normal);
}

void TriangleMesh::CalculateNormals() {
    normals.reserve(indices.size() / 3);
    for (size_t idx = 0; idx + 2 < indices.size(); idx += 3) {
        const Vec3& v0 = positions[static_cast<size_t>(indices[idx])];
        const Vec3& v1 = positions[static_cast<size_t>(indices[idx + 1])];
        const Vec3& v2 = positions[static_cast<size_t>(indices[idx + 2])];
        normals.push_back(Vec3::Cross(v1 - v0, v2 - v0).Normalized());
    }
}

void TriangleMesh::UpdateAABB() {
    if (!positions.empty()) {
        minAABB = positions[0]; maxAABB = positions[0];
        for (const auto& p : positions) { minAABB = Vec3::Min(p, minAABB); maxAABB = Vec3::Max(p, maxAABB); }
    }
}

void TriangleMesh::UpdateTransforms() {
    const Mat4 finalTransform = scaleTransform * rotationTransform * translationTransform;
    transformedPositions.clear();
    transformedPositions.reserve(positions.size());
    for (const auto& p : positions) transformedPositions.push_back(finalTransform.TransformPoint(p));
    transformedNormals.clear();
    transformedNormals.reserve(normals.size());
    for (const auto& n : normals) transformedNormals.push_back(finalTransform.TransformVector(n).Normalized());
    BuildBVH();
}

namespace {

// RTX_HOST_BVH=direct: the direct restatement (BuildBVHDirect) instead of the fast builder.
bool UseDirectBuilder() {
    static const bool direct = [] {
        const char* e = std::getenv("RTX_HOST_BVH");
        return e && std::strcmp(e, "direct") == 0;
    }();
    return direct;
}

// Subtree tasks of the fast builder.  A small process-wide pool (at most 8 workers, or
// RTX_HOST_THREADS) that sleeps between builds; a thread waiting for its task helps by
// running queued tasks, so nesting cannot deadlock.
class BuildPool {
public:
    struct Task {
        std::function<void()> fn;
        std::atomic<bool> done{false};
    };
    static BuildPool& Get() {
        static BuildPool* pool = new BuildPool();   // never destroyed: workers may outlive main's statics
        return *pool;
    }
    int Workers() const { return static_cast<int>(threads_.size()); }
    void Submit(Task* t) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(t);
            queued_.fetch_add(1, std::memory_order_release);
        }
        if (sleeping_.load(std::memory_order_acquire)) cv_.notify_one();
    }
    void Wait(Task* t) {
        while (!t->done.load(std::memory_order_acquire))
            if (!RunOne()) std::this_thread::yield();
    }

private:
    BuildPool() {
        unsigned n = std::thread::hardware_concurrency();
        if (const char* e = std::getenv("RTX_HOST_THREADS")) n = static_cast<unsigned>(std::atoi(e));
        n = n > 8 ? 8 : n;
        if (const char* e = std::getenv("RTX_HOST_SPIN_US")) spin_us_ = std::max(0, std::atoi(e));
        for (unsigned k = 1; k < n; ++k) threads_.emplace_back([this] { Loop(); });
        for (auto& th : threads_) th.detach();
    }
    bool RunOne() {
        Task* t = nullptr;
        {
            std::lock_guard<std::mutex> g(mu_);
            if (q_.empty()) return false;
            t = q_.front();
            q_.pop_front();
            queued_.fetch_sub(1, std::memory_order_relaxed);
        }
        t->fn();
        t->done.store(true, std::memory_order_release);
        return true;
    }
    // Workers spin a while on the queue counter before sleeping: during a build the next
    // subtree task is picked up within a microsecond instead of a futex wake-up.  The spin is
    // bounded in TIME (spin_us_ after the last task, RTX_HOST_SPIN_US, default 200 us: well
    // inside one build, shorter than the gap between two animated frames), so idle workers
    // sleep instead of burning the CPU quota the render thread and other ranks share.
    void Loop() {
        using Clock = std::chrono::steady_clock;
        for (;;) {
            Clock::time_point last = Clock::now();
            for (unsigned it = 1;; ++it) {
                if (queued_.load(std::memory_order_acquire) > 0 && RunOne()) {
                    last = Clock::now();
                    continue;
                }
                _mm_pause();
                if ((it & 63u) == 0 && Clock::now() - last > std::chrono::microseconds(spin_us_)) break;
            }
            std::unique_lock<std::mutex> g(mu_);
            sleeping_.fetch_add(1, std::memory_order_acq_rel);
            cv_.wait(g, [this] { return !q_.empty(); });
            sleeping_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    int spin_us_ = 200;
    std::atomic<int> queued_{0}, sleeping_{0};
    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Task*> q_;
};

// std::min(a, b) = (b < a) ? b : a = minps(b, a) per lane; std::max(a, b) = maxps(b, a).
inline __m128 MinRef(__m128 a, __m128 b) { return _mm_min_ps(b, a); }
inline __m128 MaxRef(__m128 a, __m128 b) { return _mm_max_ps(b, a); }
// AABB::Area (e.x * e.y + e.y * e.z + e.z * e.x, summed left to right), e = hi - lo
inline float Area(__m128 lo, __m128 hi) {
    const __m128 e = _mm_sub_ps(hi, lo);
    const __m128 p = _mm_mul_ps(e, _mm_shuffle_ps(e, e, _MM_SHUFFLE(3, 0, 2, 1)));   // (xy, yz, zx, ww)
    const float xy = _mm_cvtss_f32(p), yz = _mm_cvtss_f32(_mm_shuffle_ps(p, p, 1)),
                zx = _mm_cvtss_f32(_mm_shuffle_ps(p, p, 2));
    return xy + yz + zx;
}
inline Vec3 ToVec3(__m128 v) {
    alignas(16) float f[4];
    _mm_store_ps(f, v);
    return {f[0], f[1], f[2]};
}

}  // namespace

void TriangleMesh::BuildBVH() {
    if (nodes.empty() || indices.empty()) return;   // reference: UB / crash (see Scene_W4_TestScene)
    if (!UseDirectBuilder() && BuildBVHFast()) return;
    BuildBVHDirect();
}

// The fast builder takes the same decisions as BuildBVHDirect:
//  * min/max keep the reference's std::min/std::max semantics lane by lane (MinRef/MaxRef),
//    and a triangle's box min(min(v0, v1), v2) grows a node or bin exactly as its three
//    vertices in order would (first-occurrence ties) — as long as no coordinate is NaN,
//    so a mesh with a NaN position takes the direct path;
//  * bin indices, costs and split positions are the same binary32 expressions;
//  * the partition is the reference's swap loop on triangle units (i += 3 / j -= 3 become
//    +-1), applied to (centroid, id) records; the id sequence IS the composed permutation.
bool TriangleMesh::BuildBVHFast() {
    const size_t ntri = indices.size() / 3;
    pt_.resize(ntri);
    box_.resize(ntri);
    for (size_t k = 0; k < ntri; ++k) {
        const Vec3& v0 = transformedPositions[indices[3 * k]];
        const Vec3& v1 = transformedPositions[indices[3 * k + 1]];
        const Vec3& v2 = transformedPositions[indices[3 * k + 2]];
        if (v0.x != v0.x || v0.y != v0.y || v0.z != v0.z || v1.x != v1.x || v1.y != v1.y || v1.z != v1.z ||
            v2.x != v2.x || v2.y != v2.y || v2.z != v2.z)
            return false;
        const Vec3 c = (v0 + v1 + v2) * 0.3333f;
        pt_[k] = {{c.x, c.y, c.z}, static_cast<uint32_t>(k)};
        const Vec3 lo = Vec3::Min(Vec3::Min(v0, v1), v2), hi = Vec3::Max(Vec3::Max(v0, v1), v2);
        box_[k] = {{lo.x, lo.y, lo.z, 0.f}, {hi.x, hi.y, hi.z, 0.f}};
    }
    BVHNode& root = nodes[0];
    root.leftNode = 0;
    root.firstIdx = 0;
    root.idxCount = static_cast<uint32_t>(indices.size());
    nodesUsed = 1;
    tmp_.resize(2 * ntri + 1);
    tmpUsed_ = 1;
    tmp_[0] = {0u, root.idxCount, {}, {}, -1, -1};
    BoundsFast(tmp_[0]);
    SubdivideFast(0);
    root.minAABB = tmp_[0].mn;
    root.maxAABB = tmp_[0].mx;
    Emit(0, 0);
    // apply the composed permutation: slot k now holds the triangle that was at pt_[k].id
    scratchI_.assign(indices.begin(), indices.end());
    scratchN_.assign(normals.begin(), normals.end());
    scratchTN_.assign(transformedNormals.begin(), transformedNormals.end());
    const bool hasN = normals.size() >= ntri, hasTN = transformedNormals.size() >= ntri;
    for (size_t k = 0; k < ntri; ++k) {
        const uint32_t id = pt_[k].id;
        indices[3 * k] = scratchI_[3 * id];
        indices[3 * k + 1] = scratchI_[3 * id + 1];
        indices[3 * k + 2] = scratchI_[3 * id + 2];
        if (hasN) normals[k] = scratchN_[id];
        if (hasTN) transformedNormals[k] = scratchTN_[id];
    }
    return true;
}

void TriangleMesh::BoundsFast(TmpNode& n) const {
    __m128 mn = _mm_set1_ps(FLT_MAX), mx = _mm_set1_ps(FLT_MIN);
    for (uint32_t k = n.first / 3; k < (n.first + n.count) / 3; ++k) {
        const TriBox& b = box_[pt_[k].id];
        mn = MinRef(mn, _mm_load_ps(b.lo));
        mx = MaxRef(mx, _mm_load_ps(b.hi));
    }
    n.mn = ToVec3(mn);
    n.mx = ToVec3(mx);
}

void TriangleMesh::SubdivideFast(uint32_t t) {
    TmpNode& n = tmp_[t];
    if (n.count <= 8) return;
    BVHNode view;
    view.firstIdx = n.first;
    view.idxCount = n.count;
    view.minAABB = n.mn;
    view.maxAABB = n.mx;
    int axis = 0;
    float splitPos = 0.f;
    const float splitCost = FindBestSplitFast(view, axis, splitPos);
    const float noSplitCost = CalculateNodeCost(view);
    if (splitCost >= noSplitCost) return;

    // the reference's partition (DataTypes.h:335-363) in triangle units
    int i = static_cast<int>(n.first / 3);
    int j = static_cast<int>((n.first + n.count) / 3) - 1;
    while (i <= j) {
        if (pt_[i].c[axis] < splitPos) {
            ++i;
        } else {
            std::swap(pt_[i], pt_[j]);
            --j;
        }
    }
    const int leftCount = 3 * i - static_cast<int>(n.first);
    if (leftCount == 0 || static_cast<uint32_t>(leftCount) == n.count) return;

    // A node of n triangles owns the 2n - 1 temp slots from its own: the left subtree the
    // 2nL - 1 after it, the right one the rest.  No shared counter, so subtrees built on
    // different threads never touch one cache line (Emit renumbers in reference order).
    const uint32_t L = t + 1, R = t + 2 * (static_cast<uint32_t>(leftCount) / 3);
    tmp_[L] = {n.first, static_cast<uint32_t>(leftCount), {}, {}, -1, -1};
    tmp_[R] = {static_cast<uint32_t>(3 * i), n.count - static_cast<uint32_t>(leftCount), {}, {}, -1, -1};
    BoundsFast(tmp_[L]);
    BoundsFast(tmp_[R]);
    n.l = static_cast<int32_t>(L);
    n.r = static_cast<int32_t>(R);
    BuildPool& pool = BuildPool::Get();
    static const uint32_t par = [] {   // RTX_HOST_PAR_TRIS: fork subtrees with at least this many triangles a side
        const char* e = std::getenv("RTX_HOST_PAR_TRIS");
        const int v = e ? std::atoi(e) : 128;
        return static_cast<uint32_t>(v > 0 ? v : 128);
    }();
    if (pool.Workers() > 0 && tmp_[L].count >= 3 * par && tmp_[R].count >= 3 * par) {
        BuildPool::Task task;
        task.fn = [this, L] { SubdivideFast(L); };
        pool.Submit(&task);
        SubdivideFast(R);
        pool.Wait(&task);
    } else {
        SubdivideFast(L);
        SubdivideFast(R);
    }
}

// FindBestSplitPlane (DataTypes.h:378-456) over the (centroid, id) records: one SSE pass
// for the three axes' centroid bounds, one for the three axes' bins.
float TriangleMesh::FindBestSplitFast(const BVHNode& node, int& axis, float& splitPos) const {
    float bestCost = FLT_MAX;
    const uint32_t k0 = node.firstIdx / 3, k1 = (node.firstIdx + node.idxCount) / 3;
    __m128 cmn = _mm_set1_ps(FLT_MAX), cmx = _mm_set1_ps(FLT_MIN);
    for (uint32_t k = k0; k < k1; ++k) {
        const __m128 c = _mm_load_ps(pt_[k].c);   // lane 3 (the id) is never read back
        cmn = MinRef(cmn, c);
        cmx = MaxRef(cmx, c);
    }
    alignas(16) float minB[4], maxB[4], scales[4];
    _mm_store_ps(minB, cmn);
    _mm_store_ps(maxB, cmx);
    constexpr int kBins = 8, kPlanes = kBins - 1;
    bool live[3];
    for (int a = 0; a < 3; ++a) {
        const float d = maxB[a] - minB[a];
        live[a] = !(fabsf(d) < FLT_EPSILON);
        scales[a] = live[a] ? kBins / d : 0.f;
    }
    scales[3] = 0.f;
    __m128 blo[3][kBins], bhi[3][kBins];
    uint32_t counts[3][kBins] = {};
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < kBins; ++b) { blo[a][b] = _mm_set1_ps(FLT_MAX); bhi[a][b] = _mm_set1_ps(FLT_MIN); }
    const __m128 vmin = _mm_load_ps(minB), vscale = _mm_load_ps(scales);
    const bool all_live = live[0] && live[1] && live[2];
    for (uint32_t k = k0; k < k1; ++k) {
        // (centroid[axis] - minBounds) * scale, truncated like static_cast<int>
        alignas(16) int32_t bi[4];
        _mm_store_si128(reinterpret_cast<__m128i*>(bi),
                        _mm_cvttps_epi32(_mm_mul_ps(_mm_sub_ps(_mm_load_ps(pt_[k].c), vmin), vscale)));
        const TriBox& tb = box_[pt_[k].id];
        const __m128 lo = _mm_load_ps(tb.lo), hi = _mm_load_ps(tb.hi);
        for (int a = 0; a < 3; ++a) {
            if (!all_live && !live[a]) continue;
            int b = bi[a];
            if (kPlanes < b) b = kPlanes;   // std::min(amountOfPlaneBins, b)
            if (b < 0) b = 0;               // NaN / out of int range: undefined in the reference
            counts[a][b] += 3;
            blo[a][b] = MinRef(blo[a][b], lo);
            bhi[a][b] = MaxRef(bhi[a][b], hi);
        }
    }
    for (int axisIdx = 0; axisIdx < 3; ++axisIdx) {
        if (!live[axisIdx]) continue;
        const float minBounds = minB[axisIdx];
        const float boundsDifference = maxB[axisIdx] - minBounds;
        const uint32_t* binCount = counts[axisIdx];
        // The reference evaluates all 7 planes; only planes right after a non-empty bin with
        // triangles on both sides can be accepted: an empty side has area inf (its box keeps
        // FLT_MAX / FLT_MIN) and 0 * inf = NaN never compares below bestCost, and a plane after
        // an empty bin repeats the previous plane's counts and areas, which the strict < rejects.
        // A bin's box leaves a running box unchanged when the bin is empty (its lo is FLT_MAX,
        // and a running hi never drops below the FLT_MIN it starts from).
        float rightArea[kPlanes];
        int rightCount[kPlanes];
        {
            __m128 rlo = _mm_set1_ps(FLT_MAX), rhi = _mm_set1_ps(FLT_MIN);
            int rightSum = 0;
            for (int j = kPlanes; j >= 1; --j) {   // plane j - 1 has bins j..7 on its right
                if (binCount[j]) {
                    rightSum += binCount[j];
                    rlo = MinRef(rlo, blo[axisIdx][j]);
                    rhi = MaxRef(rhi, bhi[axisIdx][j]);
                }
                rightCount[j - 1] = rightSum;
                if (binCount[j - 1] && rightSum) rightArea[j - 1] = Area(rlo, rhi);
            }
        }
        const float scale = boundsDifference / kBins;
        __m128 llo = _mm_set1_ps(FLT_MAX), lhi = _mm_set1_ps(FLT_MIN);
        int leftSum = 0;
        for (int i = 0; i < kPlanes; ++i) {
            if (!binCount[i]) continue;
            leftSum += binCount[i];
            llo = MinRef(llo, blo[axisIdx][i]);
            lhi = MaxRef(lhi, bhi[axisIdx][i]);
            if (!rightCount[i]) continue;
            const float planeCost = static_cast<float>(leftSum) * Area(llo, lhi) +
                                    static_cast<float>(rightCount[i]) * rightArea[i];
            if (planeCost < bestCost) {
                axis = axisIdx;
                splitPos = minBounds + scale * static_cast<float>(i + 1);
                bestCost = planeCost;
            }
        }
    }
    return bestCost;
}

// Direct restatement: the reference's passes on a per-triangle cache (kept as the
// checked fallback for meshes with NaN coordinates and as RTX_HOST_BVH=direct).
void TriangleMesh::BuildBVHDirect() {
    BVHNode& root = nodes[0];
    root.leftNode = 0;
    root.firstIdx = 0;
    root.idxCount = static_cast<uint32_t>(indices.size());
    nodesUsed = 1;
    tc_.resize(indices.size() / 3);
    for (size_t k = 0; k < tc_.size(); ++k) {
        const Vec3& v0 = transformedPositions[indices[3 * k]];
        const Vec3& v1 = transformedPositions[indices[3 * k + 1]];
        const Vec3& v2 = transformedPositions[indices[3 * k + 2]];
        tc_[k] = {(v0 + v1 + v2) * 0.3333f, v0, v1, v2, Vec3::Min(Vec3::Min(v0, v1), v2), Vec3::Max(Vec3::Max(v0, v1), v2)};
    }
    // build the tree (subtrees in parallel), then number it as the reference's recursive
    // Subdivide would have (DataTypes.h:310-372)
    tmp_.resize(2 * tc_.size() + 1);
    tmpUsed_ = 1;
    tmp_[0] = {0u, root.idxCount, {}, {}, -1, -1};
    Bounds(tmp_[0]);
    SubdivideTmp(0, 0);
    root.minAABB = tmp_[0].mn;
    root.maxAABB = tmp_[0].mx;
    Emit(0, 0);
}

void TriangleMesh::Bounds(TmpNode& n) const {
    Vec3 mn = kMaxVector, mx = kMinVector;
    for (uint32_t k = n.first / 3; k < (n.first + n.count) / 3; ++k) {   // UpdateNodeBounds, index order
        const TriCache& t = tc_[k];
        mn = Vec3::Min(mn, t.v0); mx = Vec3::Max(mx, t.v0);
        mn = Vec3::Min(mn, t.v1); mx = Vec3::Max(mx, t.v1);
        mn = Vec3::Min(mn, t.v2); mx = Vec3::Max(mx, t.v2);
    }
    n.mn = mn;
    n.mx = mx;
}

// Subdivide (DataTypes.h:310-372) on a tree node; touches only its own index range, so
// sibling subtrees run concurrently.
void TriangleMesh::SubdivideTmp(uint32_t t, int depth) {
    TmpNode& n = tmp_[t];
    if (n.count <= 8) return;
    BVHNode view;
    view.firstIdx = n.first;
    view.idxCount = n.count;
    view.minAABB = n.mn;
    view.maxAABB = n.mx;
    int axis = 0;
    float splitPos = 0.f;
    const float splitCost = FindBestSplitPlane(view, axis, splitPos);
    const float noSplitCost = CalculateNodeCost(view);
    if (splitCost >= noSplitCost) return;

    // in-place partition (DataTypes.h:335-363): permutes indices, normals and
    // transformedNormals together
    int i = static_cast<int>(n.first);
    int j = i + static_cast<int>(n.count) - 1;
    while (i <= j) {
        const Vec3& c = tc_[static_cast<uint32_t>(i) / 3].c;
        if (c[axis] < splitPos) {
            i += 3;
        } else {
            std::swap(tc_[i / 3], tc_[(j - 2) / 3]);
            std::swap(normals[i / 3], normals[(j - 2) / 3]);
            std::swap(transformedNormals[i / 3], transformedNormals[(j - 2) / 3]);
            std::swap(indices[i], indices[j - 2]);
            std::swap(indices[i + 1], indices[j - 1]);
            std::swap(indices[i + 2], indices[j]);
            j -= 3;
        }
    }
    const int leftCount = i - static_cast<int>(n.first);
    if (leftCount == 0 || static_cast<uint32_t>(leftCount) == n.count) return;

    const uint32_t L = __atomic_fetch_add(&tmpUsed_, 2u, __ATOMIC_RELAXED), R = L + 1;
    tmp_[L] = {n.first, static_cast<uint32_t>(leftCount), {}, {}, -1, -1};
    tmp_[R] = {static_cast<uint32_t>(i), n.count - static_cast<uint32_t>(leftCount), {}, {}, -1, -1};
    Bounds(tmp_[L]);
    Bounds(tmp_[R]);
    n.l = static_cast<int32_t>(L);
    n.r = static_cast<int32_t>(R);
    // large subtrees: the left one on another thread (its ranges are disjoint from ours)
    if (depth < 3 && tmp_[L].count >= 3 * 256 && tmp_[R].count >= 3 * 256) {
        std::thread th([this, L, depth] { SubdivideTmp(L, depth + 1); });
        SubdivideTmp(R, depth + 1);
        th.join();
    } else {
        SubdivideTmp(L, depth + 1);
        SubdivideTmp(R, depth + 1);
    }
}

// Number the built tree exactly as the reference's recursion allocates it: a split node
// takes the next two slots for its children, then the left subtree is numbered before
// the right one.  Writes the same node fields the reference writes (leaves keep the rest).
void TriangleMesh::Emit(uint32_t t, uint32_t nodeIdx) {
    const TmpNode& n = tmp_[t];
    if (n.l < 0) return;
    const uint32_t L = nodesUsed++, R = nodesUsed++;
    const TmpNode& a = tmp_[static_cast<uint32_t>(n.l)];
    const TmpNode& b = tmp_[static_cast<uint32_t>(n.r)];
    nodes[nodeIdx].leftNode = L;
    nodes[L].firstIdx = a.first;
    nodes[L].idxCount = a.count;
    nodes[R].firstIdx = b.first;
    nodes[R].idxCount = b.count;
    nodes[nodeIdx].idxCount = 0;
    nodes[L].minAABB = a.mn; nodes[L].maxAABB = a.mx;
    nodes[R].minAABB = b.mn; nodes[R].maxAABB = b.mx;
    Emit(static_cast<uint32_t>(n.l), L);
    Emit(static_cast<uint32_t>(n.r), R);
}

float TriangleMesh::CalculateNodeCost(const BVHNode& node) {
    const Vec3 e = node.maxAABB - node.minAABB;
    const float area = e.x * e.y + e.y * e.z + e.z * e.x;
    return static_cast<float>(node.idxCount) * area;
}

// Binned SAH, 8 bins (DataTypes.h:378-456), including the reference's quirks: centroid
// scale 0.3333f, centroid bounds starting at {FLT_MAX, FLT_MIN}, and 0*inf = NaN costs
// for empty sides (never accepted by the strict < comparison).
// Same float operations in the same order per axis as the reference; the three axes share
// one pass over the node's triangles and the centroids come from the build cache.
float TriangleMesh::FindBestSplitPlane(const BVHNode& node, int& axis, float& splitPos) const {
    float bestCost = FLT_MAX;
    const uint32_t k0 = node.firstIdx / 3, k1 = (node.firstIdx + node.idxCount) / 3;
    float minB[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, maxB[3] = {FLT_MIN, FLT_MIN, FLT_MIN};
    for (uint32_t k = k0; k < k1; ++k) {
        const Vec3& c = tc_[k].c;
        for (int a = 0; a < 3; ++a) {
            minB[a] = fmin_ref(minB[a], c[a]);
            maxB[a] = fmax_ref(maxB[a], c[a]);
        }
    }
    constexpr int kBins = 8, kPlanes = kBins - 1;
    AABB bins[3][kBins];
    uint32_t counts[3][kBins] = {};
    float scales[3];
    bool live[3];
    for (int a = 0; a < 3; ++a) {
        const float d = maxB[a] - minB[a];
        live[a] = !(fabsf(d) < FLT_EPSILON);
        scales[a] = kBins / d;
    }
    for (uint32_t k = k0; k < k1; ++k) {
        const TriCache& t = tc_[k];
        for (int a = 0; a < 3; ++a) {
            if (!live[a]) continue;
            const float x = (t.c[a] - minB[a]) * scales[a];
            // static_cast<int> of a NaN (a NaN vertex) is undefined; the reference indexes out of
            // bounds there (x86: INT_MIN).  Such a triangle goes to bin 0 here instead of crashing.
            int b = x >= 0.f ? static_cast<int>(fminf(x, 2147483520.f)) : 0;
            if (kPlanes < b) b = kPlanes;   // std::min(amountOfPlaneBins, b)
            counts[a][b] += 3;
            bins[a][b].minAABB = Vec3::Min(bins[a][b].minAABB, t.lo);
            bins[a][b].maxAABB = Vec3::Max(bins[a][b].maxAABB, t.hi);
        }
    }
    for (int axisIdx = 0; axisIdx < 3; ++axisIdx) {
        if (!live[axisIdx]) continue;
        const float minBounds = minB[axisIdx];
        const float boundsDifference = maxB[axisIdx] - minBounds;
        const AABB* binBounds = bins[axisIdx];
        const uint32_t* binCount = counts[axisIdx];
        float scale;
        float leftArea[kPlanes]{}, rightArea[kPlanes]{};
        int leftCount[kPlanes]{}, rightCount[kPlanes]{};
        int leftSum = 0, rightSum = 0;
        AABB leftBox, rightBox;
        for (int i = 0; i < kPlanes; ++i) {
            leftSum += binCount[i];
            leftCount[i] = leftSum;
            leftBox.Grow(binBounds[i]);
            leftArea[i] = leftBox.Area();
            rightSum += binCount[kPlanes - i];
            rightCount[kPlanes - i - 1] = rightSum;
            rightBox.Grow(binBounds[kPlanes - i]);
            rightArea[kPlanes - i - 1] = rightBox.Area();
        }
        scale = boundsDifference / kBins;
        for (int i = 0; i < kPlanes; ++i) {
            const float planeCost = static_cast<float>(leftCount[i]) * leftArea[i] +
                                    static_cast<float>(rightCount[i]) * rightArea[i];
            if (planeCost < bestCost) {
                axis = axisIdx;
                splitPos = minBounds + scale * static_cast<float>(i + 1);
                bestCost = planeCost;
            }
        }
    }
    return bestCost;
}

// ---------------------------------------------------------------- Camera
void Camera::SetCameraFOV(float degrees) {
    fovAngle = fmax_ref(10.f, fmin_ref(degrees, 175.f));
    fov = tanf(fovAngle * kToRadians / 2.f);
}

void Camera::CalculateCameraToWorld() {
    if (forwardChanged) {
        right = Vec3::Cross(kUnitY, forward).Normalized();
        up = Vec3::Cross(forward, right).Normalized();
        forwardChanged = false;
    }
}

void Camera::CalculateForwardVector() {
    const Mat4 finalRotation = Mat4::Rotation({totalPitch, totalYaw, 0.f});
    forward = finalRotation.TransformVector(kUnitZ);
    forwardChanged = true;
}

rtx_camera Camera::View() const {
    rtx_camera c;
    const Vec3* v[4] = {&origin, &right, &up, &forward};
    float* dst[4] = {c.origin, c.right, c.up, c.forward};
    for (int k = 0; k < 4; ++k) { dst[k][0] = v[k]->x; dst[k][1] = v[k]->y; dst[k][2] = v[k]->z; }
    c.fov = fov;
    return c;
}

// ---------------------------------------------------------------- OBJ
static void FaceNormals(const std::vector<Vec3>& positions, const std::vector<int32_t>& indices,
                        std::vector<Vec3>& normals) {
    // Utils.h:426-448: Cross(v1 - v0, v2 - v0), Normalize()
    for (uint64_t index = 0; index + 2 < indices.size(); index += 3) {
        const uint32_t i0 = static_cast<uint32_t>(indices[index]);
        const uint32_t i1 = static_cast<uint32_t>(indices[index + 1]);
        const uint32_t i2 = static_cast<uint32_t>(indices[index + 2]);
        Vec3 n = Vec3::Cross(positions[i1] - positions[i0], positions[i2] - positions[i0]);
        n.Normalize();
        normals.push_back(n);
    }
}

bool ParseOBJ(const std::string& path, std::vector<Vec3>& positions, std::vector<Vec3>& normals,
              std::vector<int32_t>& indices) {
    // Token stream semantics of Utils.h:377-424: first token of a line selects the
    // command, `f` keeps only the text before the first '/', everything after the
    // three consumed fields is skipped.
    std::ifstream file(path);
    if (!file) return false;
    std::string cmd;
    while (!file.eof()) {
        file >> cmd;
        if (cmd == "v") {
            float x, y, z;
            file >> x >> y >> z;
            positions.push_back({x, y, z});
        } else if (cmd == "f") {
            std::string s0, s1, s2;
            file >> s0 >> s1 >> s2;
            if (s0.empty() || s1.empty() || s2.empty()) continue;
            const float i0 = std::stof(s0.substr(0, s0.find('/')));
            const float i1 = std::stof(s1.substr(0, s1.find('/')));
            const float i2 = std::stof(s2.substr(0, s2.find('/')));
            indices.push_back(static_cast<int32_t>(i0) - 1);
            indices.push_back(static_cast<int32_t>(i1) - 1);
            indices.push_back(static_cast<int32_t>(i2) - 1);
        }
        file.ignore(1000, '\n');
        if (file.eof()) break;
    }
    FaceNormals(positions, indices, normals);
    return true;
}

bool LoadMeshAsset(const std::string& path, std::vector<Vec3>& positions, std::vector<Vec3>& normals,
                   std::vector<int32_t>& indices) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    char magic[4];
    uint32_t nv = 0, ni = 0;
    bool ok = std::fread(magic, 1, 4, f) == 4 && std::memcmp(magic, "RTXM", 4) == 0 &&
              std::fread(&nv, 4, 1, f) == 1 && std::fread(&ni, 4, 1, f) == 1;
    if (ok) {
        std::vector<float> p(3ull * nv);
        std::vector<int32_t> idx(ni);
        ok = std::fread(p.data(), 4, p.size(), f) == p.size() && std::fread(idx.data(), 4, idx.size(), f) == idx.size();
        if (ok) {
            for (uint32_t k = 0; k < nv; ++k) positions.push_back({p[3 * k], p[3 * k + 1], p[3 * k + 2]});
            for (uint32_t k = 0; k < ni; ++k) {
                if (idx[k] < 0 || static_cast<uint32_t>(idx[k]) >= nv) ok = false;
                indices.push_back(idx[k]);
            }
        }
    }
    std::fclose(f);
    if (ok) FaceNormals(positions, indices, normals);
    return ok;
}

bool SaveMeshAsset(const std::string& path, const std::vector<Vec3>& positions, const std::vector<int32_t>& indices) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const uint32_t nv = static_cast<uint32_t>(positions.size()), ni = static_cast<uint32_t>(indices.size());
    bool ok = std::fwrite("RTXM", 1, 4, f) == 4 && std::fwrite(&nv, 4, 1, f) == 1 && std::fwrite(&ni, 4, 1, f) == 1;
    for (const auto& p : positions) ok = ok && std::fwrite(&p.x, 4, 3, f) == 3;
    ok = ok && std::fwrite(indices.data(), 4, indices.size(), f) == indices.size();
    std::fclose(f);
    return ok;
}

// ---------------------------------------------------------------- Scene
rtx_material SolidColor(const Color& c) {
    rtx_material m{}; m.kind = RTX_MAT_SOLID_COLOR; m.color[0] = c.r; m.color[1] = c.g; m.color[2] = c.b; return m;
}
rtx_material Lambert(const Color& c, float kd) {
    rtx_material m = SolidColor(c); m.kind = RTX_MAT_LAMBERT; m.kd = kd; return m;
}
rtx_material LambertPhong(const Color& c, float kd, float ks, float exponent) {
    rtx_material m = SolidColor(c); m.kind = RTX_MAT_LAMBERT_PHONG; m.kd = kd; m.ks = ks; m.exponent = exponent; return m;
}
rtx_material CookTorrance(const Color& albedo, float metalness, float roughness) {
    rtx_material m = SolidColor(albedo); m.kind = RTX_MAT_COOK_TORRANCE; m.metalness = metalness; m.roughness = roughness; return m;
}

namespace colors {
const Color Red{1, 0, 0}, Blue{0, 0, 1}, Green{0, 1, 0}, Yellow{1, 1, 0}, Magenta{1, 0, 1}, White{1, 1, 1};
}

Scene::Scene(std::string assetDir) : m_AssetDir(std::move(assetDir)) {
    m_Materials.push_back(SolidColor({1, 0, 0}));   // Scene.cpp:9-10 default RED
}

uint8_t Scene::AddSphere(const Vec3& o, float radius, uint8_t mat) {
    rtx_sphere s{}; s.origin[0] = o.x; s.origin[1] = o.y; s.origin[2] = o.z; s.radius = radius; s.material = mat;
    m_Spheres.push_back(s);
    return mat;
}
uint8_t Scene::AddPlane(const Vec3& o, const Vec3& n, uint8_t mat) {
    rtx_plane p{};
    p.origin[0] = o.x; p.origin[1] = o.y; p.origin[2] = o.z;
    p.normal[0] = n.x; p.normal[1] = n.y; p.normal[2] = n.z;
    p.material = mat;
    m_Planes.push_back(p);
    return mat;
}
TriangleMesh* Scene::AddTriangleMesh(int32_t cullMode, uint8_t mat) {
    auto m = std::make_unique<TriangleMesh>();
    m->cullMode = cullMode; m->materialIndex = mat;
    m_Meshes.push_back(std::move(m));
    return m_Meshes.back().get();
}
void Scene::AddPointLight(const Vec3& o, float intensity, const Color& c) {
    rtx_light l{};
    l.origin[0] = o.x; l.origin[1] = o.y; l.origin[2] = o.z;
    l.color[0] = c.r; l.color[1] = c.g; l.color[2] = c.b;
    l.intensity = intensity; l.type = RTX_LIGHT_POINT;
    m_Lights.push_back(l);
}
void Scene::AddDirectionalLight(const Vec3& d, float intensity, const Color& c) {
    rtx_light l{};
    l.direction[0] = d.x; l.direction[1] = d.y; l.direction[2] = d.z;
    l.color[0] = c.r; l.color[1] = c.g; l.color[2] = c.b;
    l.intensity = intensity; l.type = RTX_LIGHT_DIRECTIONAL;
    m_Lights.push_back(l);
}
uint8_t Scene::AddMaterial(const rtx_material& m) {
    m_Materials.push_back(m);
    return static_cast<uint8_t>(m_Materials.size() - 1);
}

bool Scene::LoadMesh(TriangleMesh* m, const std::string& stem) {
    // Prefer the committed pre-tokenised asset; fall back to an .obj of the same stem.
    const std::string base = m_AssetDir.empty() ? stem : m_AssetDir + "/" + stem;
    if (LoadMeshAsset(base + ".rtxmesh", m->positions, m->normals, m->indices)) return true;
    if (ParseOBJ(base + ".obj", m->positions, m->normals, m->indices)) return true;
    m_Error = "mesh asset not found: " + base + ".rtxmesh / .obj";
    return false;
}

rtx_scene Scene::View() {
    m_MeshViews.clear();
    for (auto& m : m_Meshes) {
        rtx_mesh v{};
        v.positions = m->transformedPositions.empty() ? nullptr : &m->transformedPositions[0].x;
        v.n_positions = static_cast<uint32_t>(m->transformedPositions.size());
        v.indices = m->indices.data();
        v.n_indices = static_cast<uint32_t>(m->indices.size());
        v.normals = m->transformedNormals.empty() ? nullptr : &m->transformedNormals[0].x;
        v.nodes = reinterpret_cast<const rtx_bvh_node*>(m->nodes.data());
        v.n_nodes = m->nodes.empty() ? 0 : m->nodesUsed;
        v.cull_mode = m->cullMode;
        v.material = m->materialIndex;
        m_MeshViews.push_back(v);
    }
    rtx_scene s{};
    s.spheres = m_Spheres.data(); s.n_spheres = static_cast<uint32_t>(m_Spheres.size());
    s.planes = m_Planes.data(); s.n_planes = static_cast<uint32_t>(m_Planes.size());
    s.meshes = m_MeshViews.data(); s.n_meshes = static_cast<uint32_t>(m_MeshViews.size());
    s.lights = m_Lights.data(); s.n_lights = static_cast<uint32_t>(m_Lights.size());
    s.materials = m_Materials.data(); s.n_materials = static_cast<uint32_t>(m_Materials.size());
    return s;
}

bool Scene::CopyStateFrom(const Scene& o) {
    if (o.m_Meshes.size() != m_Meshes.size() || o.sceneName != sceneName) return false;
    for (size_t i = 0; i < m_Meshes.size(); ++i) {
        const TriangleMesh& a = *o.m_Meshes[i];
        TriangleMesh& b = *m_Meshes[i];
        if (a.positions.size() != b.positions.size() || a.indices.size() != b.indices.size()) return false;
        b.normals = a.normals;
        b.indices = a.indices;
        b.rotationTransform = a.rotationTransform;
        b.translationTransform = a.translationTransform;
        b.scaleTransform = a.scaleTransform;
        b.minAABB = a.minAABB;
        b.maxAABB = a.maxAABB;
        b.nodes = a.nodes;
        b.nodesUsed = a.nodesUsed;
        b.transformedPositions = a.transformedPositions;
        b.transformedNormals = a.transformedNormals;
    }
    m_Camera = o.m_Camera;
    return true;
}

float Scene::SpinYaw(float t) { return (cosf(t) + 1.f) / 2.f * kPi2; }   // Scene.cpp:394

// ---------------------------------------------------------------- catalogue
namespace {

// Scene.cpp:164-184
class SceneW1 final : public Scene {
public:
    using Scene::Scene;
    bool Initialize() override {
        sceneName = "W1";
        constexpr uint8_t red = 0;
        const uint8_t blue = AddMaterial(SolidColor(colors::Blue));
        const uint8_t yellow = AddMaterial(SolidColor(colors::Yellow));
        const uint8_t green = AddMaterial(SolidColor(colors::Green));
        const uint8_t magenta = AddMaterial(SolidColor(colors::Magenta));
        AddSphere({-25.f, 0.f, 100.f}, 50.f, red);
        AddSphere({25.f, 0.f, 100.f}, 50.f, blue);
        AddPlane({-75.f, 0.f, 0.f}, {1.f, 0.f, 0.f}, green);
        AddPlane({75.f, 0.f, 0.f}, {-1.f, 0.f, 0.f}, green);
        AddPlane({0.f, -75.f, 0.f}, {0.f, 1.f, 0.f}, yellow);
        AddPlane({0.f, 75.f, 0.f}, {0.f, -1.f, 0.f}, yellow);
        AddPlane({0.f, 0.f, 125.f}, {0.f, 0.f, -1.f}, magenta);
        return true;
    }
};

// Scene.cpp:188-218
class SceneW2 final : public Scene {
public:
    using Scene::Scene;
    bool Initialize() override {
        sceneName = "W2";
        m_Camera.origin = {0.f, 3.f, -9.f};
        m_Camera.SetCameraFOV(45.f);
        constexpr uint8_t red = 0;
        const uint8_t blue = AddMaterial(SolidColor(colors::Blue));
        const uint8_t yellow = AddMaterial(SolidColor(colors::Yellow));
        const uint8_t green = AddMaterial(SolidColor(colors::Green));
        const uint8_t magenta = AddMaterial(SolidColor(colors::Magenta));
        AddPlane({-5.f, 0.f, 0.f}, {1.f, 0.f, 0.f}, green);
        AddPlane({5.f, 0.f, 0.f}, {-1.f, 0.f, 0.f}, green);
        AddPlane({0.f, 0.f, 0.f}, {0.f, 1.f, 0.f}, yellow);
        AddPlane({0.f, 10.f, 0.f}, {0.f, -1.f, 0.f}, yellow);
        AddPlane({0.f, 0.f, 10.f}, {0.f, 0.f, -1.f}, magenta);
        AddSphere({-1.75f, 1.f, 0.f}, 0.75f, red);
        AddSphere({0.f, 1.f, 0.f}, 0.75f, blue);
        AddSphere({1.75f, 1.f, 0.f}, 0.75f, red);
        AddSphere({-1.75f, 3.f, 0.f}, 0.75f, blue);
        AddSphere({0.f, 3.f, 0.f}, 0.75f, red);
        AddSphere({1.75f, 3.f, 0.f}, 0.75f, blue);
        AddPointLight({0.f, 5.f, -5.f}, 70.f, colors::White);
        return true;
    }
};

// Scene.cpp:223-243
class SceneW3Test final : public Scene {
public:
    using Scene::Scene;
    bool Initialize() override {
        sceneName = "W3_Test";
        m_Camera.origin = {0.f, 1.f, -5.f};
        m_Camera.SetCameraFOV(45.f);
        const uint8_t red = AddMaterial(Lambert(colors::Red, 1.f));
        const uint8_t bluePhong = AddMaterial(LambertPhong(colors::Blue, 1.f, 1.f, 60.f));
        const uint8_t yellow = AddMaterial(Lambert(colors::Yellow, 1.f));
        AddPlane({0.f, 0.f, 0.f}, {0.f, 1.f, 0.f}, yellow);
        AddSphere({-0.75f, 1.f, 0.f}, 1.f, red);
        AddSphere({0.75f, 1.f, 0.f}, 1.f, bluePhong);
        AddPointLight({0.f, 5.f, 5.f}, 25.f, colors::White);
        AddPointLight({0.f, 2.5f, -5.f}, 25.f, colors::White);
        return true;
    }
};

class CatalogueScene : public Scene {
public:
    using Scene::Scene;
protected:
    uint8_t Mat(const rtx_material& m) { return AddMaterial(m); }
    void RoomPlanes(uint8_t mat) {   // the 5 planes shared by W3/W4 (e.g. Scene.cpp:263-267)
        AddPlane({0.f, 0.f, 10.f}, {0.f, 0.f, -1.f}, mat);
        AddPlane({0.f, 0.f, 0.f}, {0.f, 1.f, 0.f}, mat);
        AddPlane({0.f, 10.f, 0.f}, {0.f, -1.f, 0.f}, mat);
        AddPlane({5.f, 0.f, 0.f}, {-1.f, 0.f, 0.f}, mat);
        AddPlane({-5.f, 0.f, 0.f}, {1.f, 0.f, 0.f}, mat);
    }
    void CtMaterials(uint8_t out[6]) {
        const Color metal{0.972f, 0.960f, 0.915f}, plastic{0.75f, 0.75f, 0.75f};
        out[0] = Mat(CookTorrance(metal, 1.f, 1.f));
        out[1] = Mat(CookTorrance(metal, 1.f, 0.6f));
        out[2] = Mat(CookTorrance(metal, 1.f, 0.1f));
        out[3] = Mat(CookTorrance(plastic, 0.f, 1.f));
        out[4] = Mat(CookTorrance(plastic, 0.f, 0.6f));
        out[5] = Mat(CookTorrance(plastic, 0.f, 0.1f));
    }
    void SixSpheres(const uint8_t m[6]) {   // Scene.cpp:273-278
        AddSphere({-1.75f, 1.f, 0.f}, 0.75f, m[0]);
        AddSphere({0.f, 1.f, 0.f}, 0.75f, m[1]);
        AddSphere({1.75f, 1.f, 0.f}, 0.75f, m[2]);
        AddSphere({-1.75f, 3.f, 0.f}, 0.75f, m[3]);
        AddSphere({0.f, 3.f, 0.f}, 0.75f, m[4]);
        AddSphere({1.75f, 3.f, 0.f}, 0.75f, m[5]);
    }
    void ThreeLights() {                    // Scene.cpp:282-284
        AddPointLight({0.f, 5.f, 5.f}, 50.f, Color{1.f, 0.61f, 0.45f});
        AddPointLight({-2.5f, 5.f, -5.f}, 70.f, Color{1.f, 0.8f, 0.45f});
        AddPointLight({2.5f, 2.5f, -5.f}, 50.f, Color{0.34f, 0.47f, 0.68f});
    }
    static float Yaw(float t) { return SpinYaw(t); }
};

// Scene.cpp:245-286
class SceneW3 final : public CatalogueScene {
public:
    using CatalogueScene::CatalogueScene;
    bool Initialize() override {
        sceneName = "W3";
        m_Camera.origin = {0.f, 3.f, -9.f};
        m_Camera.SetCameraFOV(45.f);
        uint8_t ct[6];
        CtMaterials(ct);
        const uint8_t grayBlue = Mat(Lambert({0.49f, 0.57f, 0.57f}, 1.f));
        Mat(LambertPhong(colors::Blue, 0.5f, 0.5f, 3.f));
        Mat(LambertPhong(colors::Blue, 0.5f, 0.5f, 15.f));
        Mat(LambertPhong(colors::Blue, 0.5f, 0.5f, 30.f));
        RoomPlanes(grayBlue);
        SixSpheres(ct);
        ThreeLights();
        return true;
    }
};

// Scene.cpp:289-328 — the reference never allocates pBVHNodes for this scene and
// crashes in BuildBVH (segfault); we refuse it with an error instead.
class SceneW4Test final : public CatalogueScene {
public:
    using CatalogueScene::CatalogueScene;
    bool Initialize() override {
        sceneName = "W4_Test";
        m_Error = "Scene_W4_TestScene is not renderable: the reference never allocates its BVH nodes "
                  "(Scene.cpp:306-310 vs DataTypes.h:231-232) and crashes";
        return false;
    }
};

// Scene.cpp:330-400
class SceneW4Reference final : public CatalogueScene {
public:
    using CatalogueScene::CatalogueScene;
    bool Initialize() override {
        sceneName = "W4_Reference";
        m_Camera.origin = {0.f, 3.f, -9.f};
        m_Camera.SetCameraFOV(45.f);
        uint8_t ct[6];
        CtMaterials(ct);
        const uint8_t grayBlue = Mat(Lambert({0.49f, 0.57f, 0.57f}, 1.f));
        const uint8_t white = Mat(Lambert(colors::White, 1.f));
        RoomPlanes(grayBlue);
        SixSpheres(ct);
        const Vec3 a{-0.75f, 1.5f, 0.f}, b{0.75f, 0.f, 0.f}, c{-0.75f, 0.f, 0.f};
        const int32_t culls[3] = {RTX_CULL_BACK, RTX_CULL_FRONT, RTX_CULL_NONE};
        const float xs[3] = {-1.75f, 0.f, 1.75f};
        for (int k = 0; k < 3; ++k) {
            TriangleMesh* m = AddTriangleMesh(culls[k], white);
            m->AppendTriangle(a, b, c);
            m->Translate({xs[k], 4.5f, 0.f});
            m->AllocateNodes();
            m->UpdateAABB();
            m->UpdateTransforms();
        }
        ThreeLights();
        return true;
    }
    bool Animated() const override { return true; }
    void Update(float t) override {
        const float yaw = Yaw(t);
        for (auto& m : m_Meshes) { m->RotateY(yaw); m->UpdateTransforms(); }
    }
    std::vector<TriangleMesh*> Spinning() override {
        std::vector<TriangleMesh*> v;
        for (auto& m : m_Meshes) v.push_back(m.get());
        return v;
    }
};

// Scene.cpp:402-437
class SceneW4Bunny : public CatalogueScene {
public:
    using CatalogueScene::CatalogueScene;
    bool Initialize() override {
        sceneName = "W4_Bunny";
        m_Camera.origin = {0.f, 3.f, -9.f};
        m_Camera.SetCameraFOV(45.f);
        const uint8_t grayBlue = Mat(Lambert({0.49f, 0.57f, 0.57f}, 1.f));
        const uint8_t white = Mat(Lambert(colors::White, 1.f));
        TriangleMesh* m = AddTriangleMesh(RTX_CULL_BACK, white);
        if (!LoadMesh(m, "lowpoly_bunny2")) return false;
        m->Scale({2.f, 2.f, 2.f});
        m->AllocateNodes();
        m->UpdateAABB();
        m->UpdateTransforms();
        RoomPlanes(grayBlue);
        ThreeLights();
        return true;
    }
    bool Animated() const override { return true; }
    void Update(float t) override {
        m_Meshes[0]->RotateY(Yaw(t));
        m_Meshes[0]->UpdateTransforms();
    }
    std::vector<TriangleMesh*> Spinning() override { return {m_Meshes[0].get()}; }
};

// Bunny + 5 lights at (3.5cos θk, 5.5, 3.5 sin θk − 2), θk = 2πk/5,
// intensity 40, colours cycling the reference trio.
class SceneBunny8Lights final : public SceneW4Bunny {
public:
    using SceneW4Bunny::SceneW4Bunny;
    bool Initialize() override {
        if (!SceneW4Bunny::Initialize()) return false;
        sceneName = "Bunny8Lights";
        const Color trio[3] = {{1.f, 0.61f, 0.45f}, {1.f, 0.8f, 0.45f}, {0.34f, 0.47f, 0.68f}};
        for (int k = 0; k < 5; ++k) {
            const float theta = kPi2 * static_cast<float>(k) / 5.f;
            AddPointLight({3.5f * cosf(theta), 5.5f, 3.5f * sinf(theta) - 2.f}, 40.f, trio[k % 3]);
        }
        return true;
    }
};

// Scene.cpp:439-474
class SceneW4Optional final : public CatalogueScene {
public:
    using CatalogueScene::CatalogueScene;
    bool Initialize() override {
        sceneName = "W4_Optional";
        m_Camera.origin = {0.f, 2.f, -9.f};
        m_Camera.SetCameraFOV(45.f);
        const uint8_t grayBlue = Mat(Lambert({0.49f, 0.57f, 0.57f}, 1.f));
        const uint8_t copper = Mat(CookTorrance({0.72f, 0.254f, 0.055f}, 1.0f, 0.7f));
        TriangleMesh* m = AddTriangleMesh(RTX_CULL_BACK, copper);
        if (!LoadMesh(m, "Assignment3D1")) return false;
        m->Scale({0.03f, 0.03f, 0.03f});
        m->AllocateNodes();
        m->UpdateAABB();
        m->UpdateTransforms();
        RoomPlanes(grayBlue);
        ThreeLights();
        return true;
    }
    bool Animated() const override { return true; }
    void Update(float t) override {
        m_Meshes[0]->RotateY(Yaw(t));
        m_Meshes[0]->UpdateTransforms();
    }
    std::vector<TriangleMesh*> Spinning() override { return {m_Meshes[0].get()}; }
};

// 250 x 200-quad height field = 100,000 triangles over
// x in [-3,3], z in [-1,3], y = 0.3 + 0.5 u, u = (mt19937(42)() >> 8) * 2^-24 per vertex
// (z outer, x inner); back-face culled, Lambert white; Bunny-scene planes and lights.
class SceneSynthetic100k final : public CatalogueScene {
public:
    using CatalogueScene::CatalogueScene;
    bool Initialize() override {
        sceneName = "Synthetic100k";
        m_Camera.origin = {0.f, 3.f, -9.f};
        m_Camera.SetCameraFOV(45.f);
        const uint8_t grayBlue = Mat(Lambert({0.49f, 0.57f, 0.57f}, 1.f));
        const uint8_t white = Mat(Lambert(colors::White, 1.f));
        TriangleMesh* m = AddTriangleMesh(RTX_CULL_BACK, white);
        const int NX = 250, NZ = 200;
        std::mt19937 rng(42);
        for (int j = 0; j <= NZ; ++j) {
            for (int i = 0; i <= NX; ++i) {
                const float u = static_cast<float>(rng() >> 8) * (1.0f / 16777216.0f);
                const float x = -3.0f + (6.0f * static_cast<float>(i)) / 250.0f;
                const float z = -1.0f + (4.0f * static_cast<float>(j)) / 200.0f;
                m->positions.push_back({x, 0.3f + 0.5f * u, z});
            }
        }
        for (int j = 0; j < NZ; ++j) {
            for (int i = 0; i < NX; ++i) {
                const int32_t v00 = j * (NX + 1) + i, v10 = v00 + 1, v01 = v00 + (NX + 1), v11 = v01 + 1;
                const int32_t tri[6] = {v00, v01, v10, v10, v01, v11};
                for (int32_t k : tri) m->indices.push_back(k);
            }
        }
        m->CalculateNormals();
        m->AllocateNodes();
        m->UpdateAABB();
        m->UpdateTransforms();
        RoomPlanes(grayBlue);
        ThreeLights();
        return true;
    }
};

}  // namespace

// ---------------------------------------------------------------- scene files
// Data-driven scenes: a text file, one directive per line, built
// with the same builders, in file order, as the catalogue scenes above are built from
// Scene.cpp.  Grammar (floats by strtof; '#' starts a comment):
//   camera <ox> <oy> <oz> <fov degrees>
//   material solid <r> <g> <b>                        Material_SolidColor
//   material lambert <r> <g> <b> <kd>                 Material_Lambert
//   material lambert_phong <r> <g> <b> <kd> <ks> <exp> Material_LambertPhong
//   material cook_torrance <r> <g> <b> <metal> <rough> Material_CookTorrence
//   sphere <cx> <cy> <cz> <radius> <material>
//   plane <ox> <oy> <oz> <nx> <ny> <nz> <material>
//   mesh <stem> <material> <front|back|none> [scale x y z] [translate x y z] [spin]
//   light point <x> <y> <z> <intensity> <r> <g> <b>
//   light directional <dx> <dy> <dz> <intensity> <r> <g> <b>
// Material indices count from 0 = the scene's built-in red SolidColor (Scene.cpp:9-10);
// the file's materials are 1, 2, ... in order.  A mesh <stem> is <asset dir>/<stem>.rtxmesh
// or .obj (the reference harness reads Resources/<stem>.obj); `spin` meshes rotate in
// Update(t) like the W4 scenes (yaw = (cos t + 1)/2 * 2 pi, Scene.cpp:391-400).
class SceneFile final : public CatalogueScene {
public:
    SceneFile(std::string assetDir, std::string path) : CatalogueScene(std::move(assetDir)), m_Path(std::move(path)) {}
    bool Initialize() override {
        sceneName = "file:" + m_Path;
        std::ifstream in(m_Path);
        if (!in) { m_Error = "cannot open scene file " + m_Path; return false; }
        std::string line;
        int lineNo = 0;
        while (std::getline(in, line)) {
            ++lineNo;
            const size_t hash = line.find('#');
            if (hash != std::string::npos) line.resize(hash);
            std::vector<std::string> tok;
            {
                size_t i = 0;
                while (i < line.size()) {
                    while (i < line.size() && std::isspace(static_cast<unsigned char>(line[i]))) ++i;
                    size_t j = i;
                    while (j < line.size() && !std::isspace(static_cast<unsigned char>(line[j]))) ++j;
                    if (j > i) tok.push_back(line.substr(i, j - i));
                    i = j;
                }
            }
            if (tok.empty()) continue;
            if (!Directive(tok)) {
                m_Error = m_Path + ":" + std::to_string(lineNo) + ": " + (m_Error.empty() ? "bad directive" : m_Error);
                return false;
            }
        }
        return true;
    }
    bool Animated() const override { return !m_Spin.empty(); }
    void Update(float t) override {
        for (TriangleMesh* m : m_Spin) { m->RotateY(Yaw(t)); m->UpdateTransforms(); }
    }
    std::vector<TriangleMesh*> Spinning() override { return m_Spin; }

private:
    static bool F(const std::vector<std::string>& t, size_t i, float& out) {
        if (i >= t.size()) return false;
        char* end = nullptr;
        out = std::strtof(t[i].c_str(), &end);
        return end && *end == 0;
    }
    bool Floats(const std::vector<std::string>& t, size_t i, size_t n, float* out) {
        for (size_t k = 0; k < n; ++k)
            if (!F(t, i + k, out[k])) { m_Error = "expected a number at field " + std::to_string(i + k); return false; }
        return true;
    }
    bool MatIndex(const std::vector<std::string>& t, size_t i, uint8_t& out) {
        float v;
        if (!F(t, i, v) || v < 0.f || v != static_cast<float>(static_cast<int>(v)) ||
            static_cast<size_t>(v) >= m_Materials.size()) {
            m_Error = "material index out of range";
            return false;
        }
        out = static_cast<uint8_t>(v);
        return true;
    }
    bool Directive(const std::vector<std::string>& t) {
        const std::string& d = t[0];
        float v[8];
        if (d == "camera") {
            if (t.size() != 5 || !Floats(t, 1, 4, v)) return false;
            m_Camera.origin = {v[0], v[1], v[2]};
            m_Camera.SetCameraFOV(v[3]);
            return true;
        }
        if (d == "material" && t.size() >= 2) {
            if (m_Materials.size() >= 256) { m_Error = "more than 256 materials"; return false; }
            const std::string& k = t[1];
            if (k == "solid" && t.size() == 5 && Floats(t, 2, 3, v)) { AddMaterial(SolidColor({v[0], v[1], v[2]})); return true; }
            if (k == "lambert" && t.size() == 6 && Floats(t, 2, 4, v)) { AddMaterial(Lambert({v[0], v[1], v[2]}, v[3])); return true; }
            if (k == "lambert_phong" && t.size() == 8 && Floats(t, 2, 6, v)) {
                AddMaterial(LambertPhong({v[0], v[1], v[2]}, v[3], v[4], v[5]));
                return true;
            }
            if (k == "cook_torrance" && t.size() == 7 && Floats(t, 2, 5, v)) {
                AddMaterial(CookTorrance({v[0], v[1], v[2]}, v[3], v[4]));
                return true;
            }
            return false;
        }
        if (d == "sphere") {
            uint8_t m;
            if (t.size() != 6 || !Floats(t, 1, 4, v) || !MatIndex(t, 5, m)) return false;
            AddSphere({v[0], v[1], v[2]}, v[3], m);
            return true;
        }
        if (d == "plane") {
            uint8_t m;
            if (t.size() != 8 || !Floats(t, 1, 6, v) || !MatIndex(t, 7, m)) return false;
            AddPlane({v[0], v[1], v[2]}, {v[3], v[4], v[5]}, m);
            return true;
        }
        if (d == "light" && t.size() == 9 && Floats(t, 2, 7, v)) {
            if (t[1] == "point") { AddPointLight({v[0], v[1], v[2]}, v[3], {v[4], v[5], v[6]}); return true; }
            if (t[1] == "directional") { AddDirectionalLight({v[0], v[1], v[2]}, v[3], {v[4], v[5], v[6]}); return true; }
            return false;
        }
        if (d == "mesh" && t.size() >= 4) {
            uint8_t m;
            if (!MatIndex(t, 2, m)) return false;
            int32_t cull;
            if (t[3] == "front") cull = RTX_CULL_FRONT;
            else if (t[3] == "back") cull = RTX_CULL_BACK;
            else if (t[3] == "none") cull = RTX_CULL_NONE;
            else { m_Error = "cull must be front|back|none"; return false; }
            TriangleMesh* mesh = AddTriangleMesh(cull, m);
            if (!LoadMesh(mesh, t[1])) return false;
            bool spin = false;
            for (size_t i = 4; i < t.size();) {
                if (t[i] == "scale" && Floats(t, i + 1, 3, v)) { mesh->Scale({v[0], v[1], v[2]}); i += 4; }
                else if (t[i] == "translate" && Floats(t, i + 1, 3, v)) { mesh->Translate({v[0], v[1], v[2]}); i += 4; }
                else if (t[i] == "spin") { spin = true; ++i; }
                else { m_Error = "unknown mesh option " + t[i]; return false; }
            }
            mesh->AllocateNodes();   // pBVHNodes = new BVHNode[indices.size()]
            mesh->UpdateAABB();
            mesh->UpdateTransforms();
            if (spin) m_Spin.push_back(mesh);
            return true;
        }
        return false;
    }
    std::string m_Path;
    std::vector<TriangleMesh*> m_Spin;
};

std::unique_ptr<Scene> MakeScene(const std::string& name, const std::string& assetDir) {
    if (name.rfind("file:", 0) == 0) return std::make_unique<SceneFile>(assetDir, name.substr(5));
    std::unique_ptr<Scene> s;
    if (name == "W1") s = std::make_unique<SceneW1>(assetDir);
    else if (name == "W2") s = std::make_unique<SceneW2>(assetDir);
    else if (name == "W3") s = std::make_unique<SceneW3>(assetDir);
    else if (name == "W3_Test") s = std::make_unique<SceneW3Test>(assetDir);
    else if (name == "W4_Test") s = std::make_unique<SceneW4Test>(assetDir);
    else if (name == "W4_Reference") s = std::make_unique<SceneW4Reference>(assetDir);
    else if (name == "W4_Bunny") s = std::make_unique<SceneW4Bunny>(assetDir);
    else if (name == "Bunny8Lights") s = std::make_unique<SceneBunny8Lights>(assetDir);
    else if (name == "W4_Optional") s = std::make_unique<SceneW4Optional>(assetDir);
    else if (name == "Synthetic100k") s = std::make_unique<SceneSynthetic100k>(assetDir);
    return s;
}

}  // namespace rtx
