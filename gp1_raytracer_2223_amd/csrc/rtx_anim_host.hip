// rtx_anim_host.hip — the C-ABI of the device Update (rtx_anim_*, rtx.h): registration of a
// scene's animated meshes with the render context, and each Update's copy of the template image
// plus the rebuild launch (rtx_anim.hip holds the builder's kernels, rtx_anim.h its interface).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rtx_anim.h"
#include "rtx_ctx.h"

using namespace rtxh;

namespace {
inline float4 f4(float x, float y, float z, float w) { return make_float4(x, y, z, w); }
}  // namespace

// ====================================================================== device-side animation
// rtx_anim_* (rtx.h): Scene::Update of animated meshes in HBM (rtx_anim.h).
// Registration uploads the scene once with rebuild-sized regions reserved for the animated
// meshes and keeps that image as a template; an update copies the template into the
// context's next scene image and lets the build kernel overwrite the animated meshes'
// triangle records, node pairs (+ octant copies) and frontier parts.
// Device Update: nodes above this many triangles are split by a whole workgroup as queue
// tasks, smaller ones built as subtrees by one workgroup each (rtx_anim.h)
constexpr uint32_t kAnimCut = 96;

struct rtx_anim {
    int device = 0;
    std::string err;
    std::vector<rtxa::MeshDev> mesh;      // host copies of the device descriptors
    rtxa::MeshDev* d_mesh = nullptr;
    std::vector<void*> allocs;
    char* d_template = nullptr;
    size_t total = 0, tri_off = 0, node_off = 0, part_off = 0, mesh_off = 0;
    uint32_t oct_bytes = 0;
    DevScene dev{};                       // pointers relative to the image base
    bool split_ok = false;
    int spec = 0;
    float room_p0[5] = {};   // rtx_ctx::room_p0 of the registration upload
    std::string sig;
    hipEvent_t ev = nullptr;              // the last update
    // RTX_ANIM_OWN_STREAM=1: the updates run on the anim's own stream (high priority;
    // RTX_ANIM_STREAM_PRIO=normal: default priority) beside the previous frame's render, the
    // context's next render waiting for its event; default: on the context's stream, which
    // measured faster in 4 of 6 animated-loop cases (profiles/r03/anim_benchmark_update_stream.log)
    hipStream_t stream = nullptr;
    bool built = false;
    uint32_t cur = 0;                     // state buffer of the current order
    // rebuilt trees this deep or deeper are disabled in the image (rtxa::Launch::depth_limit);
    // RTX_ANIM_DEPTH_LIMIT lowers it for the tests of that guard
    uint32_t depth_limit = kStackDepth;
    bool reg_fast = false;                // DevScene::tri_fast condition at registration
    bool hbm_only = false;                // RTX_ANIM_HBM=1 at registration: build records in HBM (tests)
    bool serial_frontier = false;         // RTX_ANIM_SERIAL_FRONTIER=1: the frontier's serial greedy for every mesh (tests)
    uint32_t cut = kAnimCut;              // RTX_ANIM_CUT: nodes above this many triangles split as queue tasks
    uint32_t epoch = 0;                   // updates so far (the build's publication flag)
    uint64_t wait_ticks = rtxa::kWaitTicks;   // rtxa::Launch::wait_ticks (RTX_ANIM_WAIT_TICKS: tests of the timeout path)
    uint32_t debug = 0;                       // rtxa::Launch::debug (RTX_ANIM_DEBUG: tests of the timeout path)
    std::vector<double> obj_radius;       // per registered mesh: max |object-space position|
};

namespace {
thread_local std::string g_anim_err;
int afail(rtx_anim* a, int code, const std::string& msg) {
    if (a) a->err = msg; else g_anim_err = msg;
    return code;
}
#define ANIM_TRY(a, call)                                                                    \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess) return afail((a), RTX_E_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
hipError_t anim_alloc(rtx_anim* a, T** p, size_t count) {
    void* q = nullptr;
    const hipError_t e = hipMalloc(&q, count * sizeof(T) + 16);
    if (e == hipSuccess) {
        a->allocs.push_back(q);
        (void)hipMemset(q, 0, count * sizeof(T) + 16);
    }
    *p = static_cast<T*>(q);
    return e;
}

// DevScene pointers as offsets from an image base and back
DevScene rebase(const DevScene& d, const char* from, const char* to) {
    DevScene r = d;
    auto mv = [&](auto& ptr) {
        using P = std::remove_reference_t<decltype(ptr)>;
        ptr = reinterpret_cast<P>(to + (reinterpret_cast<const char*>(ptr) - from));
    };
    mv(r.spheres); mv(r.sphere_mat); mv(r.planes); mv(r.tris); mv(r.nodes); mv(r.meshes); mv(r.lights);
    mv(r.materials); mv(r.parts);
    return r;
}
}  // namespace

extern "C" const char* rtx_anim_last_error(const rtx_anim* a) { return a ? a->err.c_str() : g_anim_err.c_str(); }

extern "C" void rtx_anim_destroy(rtx_anim* a) {
    if (!a) return;
    (void)hipSetDevice(a->device);
    if (a->ev) { (void)hipEventSynchronize(a->ev); (void)hipEventDestroy(a->ev); }
    if (a->stream) { (void)hipStreamSynchronize(a->stream); (void)hipStreamDestroy(a->stream); }
    for (void* p : a->allocs) (void)hipFree(p);
    delete a;
}

extern "C" int rtx_anim_create(rtx_anim** out, rtx_ctx* c, const rtx_scene* s, const int32_t* ids,
                               const rtx_mesh_source* src, uint32_t n) {
    if (!out) return RTX_E_INVALID;
    *out = nullptr;
    g_anim_err.clear();
    if (!c || !s || !ids || !src || n == 0) return afail(nullptr, RTX_E_INVALID, "null argument or no mesh");
    if (join_split(c) != RTX_OK) return afail(nullptr, RTX_E_DEVICE, "joining the last split chain");
    if (n > static_cast<uint32_t>(rtxa::kMaxAnimMeshes)) return afail(nullptr, RTX_E_UNSUPPORTED, "more than 32 animated meshes");
    if (c->split_parts > static_cast<uint32_t>(rtxa::kMaxAnimParts))
        return afail(nullptr, RTX_E_UNSUPPORTED, "frontier target above the device builder's 128 parts");
    std::vector<uint8_t> seen(s->n_meshes, 0);
    for (uint32_t i = 0; i < n; ++i) {
        if (ids[i] < 0 || static_cast<uint32_t>(ids[i]) >= s->n_meshes || seen[ids[i]])
            return afail(nullptr, RTX_E_INVALID, "bad or repeated mesh id");
        seen[ids[i]] = 1;
        const rtx_mesh& m = s->meshes[ids[i]];
        const rtx_mesh_source& q = src[i];
        if (!q.positions || !q.normals || !q.indices || q.n_indices == 0 || q.n_indices % 3 ||
            q.n_indices != m.n_indices || q.n_positions != m.n_positions || !m.nodes || m.n_nodes == 0 ||
            m.n_nodes > q.n_indices)
            return afail(nullptr, RTX_E_INVALID, "mesh source does not match the scene's mesh");
        for (uint32_t k = 0; k < q.n_indices; ++k)
            if (q.indices[k] < 0 || static_cast<uint32_t>(q.indices[k]) >= q.n_positions)
                return afail(nullptr, RTX_E_INVALID, "mesh source index out of range");
        for (uint32_t k = 0; k < 3 * q.n_positions; ++k)
            if (q.positions[k] != q.positions[k]) return afail(nullptr, RTX_E_UNSUPPORTED, "NaN position");
    }
    UploadLayout lay;
    lay.reserve.assign(s->n_meshes, 0);
    for (uint32_t i = 0; i < n; ++i) lay.reserve[ids[i]] = 1;
    lay.tri0.assign(s->n_meshes, 0); lay.root.assign(s->n_meshes, 0);
    lay.part0.assign(s->n_meshes, 0); lay.part_cap.assign(s->n_meshes, 0);
    lay.depth.assign(s->n_meshes, 0);
    int rc = upload_scene(c, s, &lay);
    if (rc != RTX_OK) return afail(nullptr, rc, std::string("upload: ") + c->err);
    if (c->deep_stack) return afail(nullptr, RTX_E_UNSUPPORTED, "scene needs the deep-stack kernel");

    rtx_anim* a = new (std::nothrow) rtx_anim;
    if (!a) return RTX_E_NOMEM;
    a->device = c->device;
    a->hbm_only = std::getenv("RTX_ANIM_HBM") != nullptr;
    a->serial_frontier = std::getenv("RTX_ANIM_SERIAL_FRONTIER") != nullptr;
    if (const char* e = std::getenv("RTX_ANIM_CUT")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 8 && v < (1l << 30)) a->cut = static_cast<uint32_t>(v);
    }
    if (const char* e = std::getenv("RTX_ANIM_WAIT_TICKS")) {
        const long long v = std::strtoll(e, nullptr, 10);
        if (v >= 0) a->wait_ticks = static_cast<uint64_t>(v);
    }
    if (const char* e = std::getenv("RTX_ANIM_DEBUG")) a->debug = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
    if (const char* e = std::getenv("RTX_ANIM_DEPTH_LIMIT")) {
        const int v = std::atoi(e);
        if (v >= 1 && v < kStackDepth) a->depth_limit = static_cast<uint32_t>(v);
    }
    auto bail = [&](int code) { g_anim_err = a->err; rtx_anim_destroy(a); return code; };
#define ANIM_CREATE_TRY(call)                                                                \
    do {                                                                                     \
        const hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) { a->err = std::string(#call) + ": " + hipGetErrorString(e_); return bail(RTX_E_DEVICE); } \
    } while (0)
    ANIM_CREATE_TRY(hipSetDevice(c->device));
    ANIM_CREATE_TRY(hipEventCreateWithFlags(&a->ev, hipEventDisableTiming));
    if (std::getenv("RTX_ANIM_OWN_STREAM") && !std::getenv("RTX_ANIM_SAME_STREAM")) {
        int lo_prio = 0, hi_prio = 0;
        ANIM_CREATE_TRY(hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
        const char* pr = std::getenv("RTX_ANIM_STREAM_PRIO");   // "normal": the default priority (tests)
        ANIM_CREATE_TRY(hipStreamCreateWithPriority(&a->stream, hipStreamNonBlocking,
                                                    pr && std::string(pr) == "normal" ? lo_prio : hi_prio));
    }
    a->total = lay.total;
    a->tri_off = lay.tri_off; a->node_off = lay.node_off; a->part_off = lay.part_off; a->mesh_off = lay.mesh_off;
    a->oct_bytes = lay.oct_bytes;
    ANIM_CREATE_TRY(anim_alloc(a, &a->d_template, a->total));
    // anim_alloc's clears run on the null stream, which the context's non-blocking stream
    // does not wait for: finish them before the template copy is queued
    ANIM_CREATE_TRY(hipDeviceSynchronize());
    const char* base = c->sb[c->sb_cur].d;
    ANIM_CREATE_TRY(hipMemcpyAsync(a->d_template, base, a->total, hipMemcpyDeviceToDevice, c->stream));
    a->dev = rebase(c->dev, base, nullptr);
    // every animated triangle keeps |e1| |e2| within a rounding of its registration value
    // (a rotation): FAST Moller-Trumbore only with a factor-2 margin below its 2^56 bound
    a->dev.tri_fast = lay.max_ee <= 0x1p55 ? 1u : 0u;
    a->reg_fast = a->dev.tri_fast != 0;
    a->split_ok = c->split_ok;
    a->spec = c->scene_spec;
    std::memcpy(a->room_p0, c->room_p0, sizeof a->room_p0);
    a->sig = c->scene_sig;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t id = static_cast<uint32_t>(ids[i]);
        const rtx_mesh& m = s->meshes[id];
        const rtx_mesh_source& q = src[i];
        rtxa::MeshDev d{};
        d.V = q.n_positions;
        d.T = q.n_indices / 3;
        const size_t V = d.V, T = d.T;
        ANIM_CREATE_TRY(anim_alloc(a, const_cast<float4**>(&d.pos), V));
        ANIM_CREATE_TRY(anim_alloc(a, &d.tpos, V));
        for (int k = 0; k < 2; ++k) {
            ANIM_CREATE_TRY(anim_alloc(a, &d.idx[k], T));
            ANIM_CREATE_TRY(anim_alloc(a, &d.nrm[k], T));
        }
        for (int k = 0; k < 2; ++k) ANIM_CREATE_TRY(anim_alloc(a, &d.lvl[k], T));
        ANIM_CREATE_TRY(anim_alloc(a, &d.sub, rtxa::kMaxSub));
        ANIM_CREATE_TRY(anim_alloc(a, &d.tnrm, T));
        ANIM_CREATE_TRY(anim_alloc(a, &d.tnrm_out, T));
        // build records by triangle id and the two permutation buffers
        ANIM_CREATE_TRY(anim_alloc(a, &d.soa, 9 * T));
        ANIM_CREATE_TRY(anim_alloc(a, &d.perm[0], T));
        ANIM_CREATE_TRY(anim_alloc(a, &d.perm[1], T));
        ANIM_CREATE_TRY(anim_alloc(a, &d.lb, T));
        ANIM_CREATE_TRY(anim_alloc(a, &d.rs, T));
        ANIM_CREATE_TRY(anim_alloc(a, &d.rk, T));
        ANIM_CREATE_TRY(anim_alloc(a, &d.tmp, 2 * T + rtxa::kMaxTop));
        ANIM_CREATE_TRY(anim_alloc(a, &d.ref, 3 * T));
        ANIM_CREATE_TRY(anim_alloc(a, &d.status, 128));
        ANIM_CREATE_TRY(anim_alloc(a, &d.q, rtxa::kQWords));
        double rad = 0.0;
        for (size_t k = 0; k < V; ++k) {
            const double x = q.positions[3 * k], y = q.positions[3 * k + 1], z = q.positions[3 * k + 2];
            const double r = std::sqrt(x * x + y * y + z * z);
            rad = (r > rad || r != r) ? r : rad;   // NaN positions are refused above; inf sticks
        }
        a->obj_radius.push_back(rad);
        std::vector<float4> pos(V), nrm(T);
        std::vector<int4> idx(T);
        for (size_t k = 0; k < V; ++k) pos[k] = f4(q.positions[3 * k], q.positions[3 * k + 1], q.positions[3 * k + 2], 0.f);
        for (size_t k = 0; k < T; ++k) {
            nrm[k] = f4(q.normals[3 * k], q.normals[3 * k + 1], q.normals[3 * k + 2], 0.f);
            idx[k] = make_int4(q.indices[3 * k], q.indices[3 * k + 1], q.indices[3 * k + 2], 0);
        }
        ANIM_CREATE_TRY(hipMemcpy(const_cast<float4*>(d.pos), pos.data(), V * 16, hipMemcpyHostToDevice));
        ANIM_CREATE_TRY(hipMemcpy(d.idx[0], idx.data(), T * 16, hipMemcpyHostToDevice));
        ANIM_CREATE_TRY(hipMemcpy(d.nrm[0], nrm.data(), T * 16, hipMemcpyHostToDevice));
        // pBVHNodes persists across builds (a leaf keeps a stale leftNode): start from the scene's
        ANIM_CREATE_TRY(hipMemcpy(d.ref, m.nodes, sizeof(rtx_bvh_node) * m.n_nodes, hipMemcpyHostToDevice));
        d.mat_bits = m.material;
        d.mesh = id;
        d.tri0 = lay.tri0[id];
        d.root = lay.root[id];
        d.part0 = lay.part0[id];
        d.part_cap = c->split_ok ? lay.part_cap[id] : 0u;
        a->mesh.push_back(d);
    }
    ANIM_CREATE_TRY(anim_alloc(a, &a->d_mesh, n));
    ANIM_CREATE_TRY(hipMemcpy(a->d_mesh, a->mesh.data(), n * sizeof(rtxa::MeshDev), hipMemcpyHostToDevice));
    // the template's reserved node slots start empty: an update writes slots [root, root +
    // nodesUsed) and leaves the rest zero, exactly as a host upload of the same state lays it out
    ANIM_CREATE_TRY(hipStreamSynchronize(c->stream));
    for (const rtxa::MeshDev& d : a->mesh)
        for (int k = 0; k < (a->oct_bytes ? 8 : 1); ++k)
            ANIM_CREATE_TRY(hipMemset(a->d_template + a->node_off + static_cast<size_t>(k) * a->oct_bytes +
                                          static_cast<size_t>(d.root) * 32u,
                                      0, static_cast<size_t>(2) * d.T * 32u));
    ANIM_CREATE_TRY(hipDeviceSynchronize());   // every clear and copy above, before any update
#undef ANIM_CREATE_TRY
    *out = a;
    return RTX_OK;
}

extern "C" int rtx_anim_update(rtx_anim* a, rtx_ctx* c, const float* transforms) {
    if (!a || !c || !transforms) return RTX_E_INVALID;
    if (c->device != a->device) return afail(a, RTX_E_INVALID, "context on another device");
    ANIM_TRY(a, hipSetDevice(a->device));
    if (join_split(c) != RTX_OK) return afail(a, RTX_E_DEVICE, "joining the last split chain");
    // the context's next scene image (as rtx_upload_scene picks it)
    const int k = c->sb_cur < 0 ? 0 : (c->sb_cur ^ 1);
    rtx_ctx::SceneBuf& B = c->sb[k];
    if (B.pending) {
        ANIM_TRY(a, hipEventSynchronize(B.done));
        B.pending = false;
    }
    if (a->total > B.cap) {
        (void)hipFree(B.d);
        if (B.h) (void)hipHostFree(B.h);
        B.d = nullptr; B.h = nullptr; B.cap = 0;
        ANIM_TRY(a, hipMalloc(&B.d, a->total));
        ANIM_TRY(a, hipHostMalloc(&B.h, a->total));
        B.cap = a->total;
    }
    // (image B's earlier renders on this context have completed: B.done above)
    hipStream_t s = a->stream ? a->stream : c->stream;
    if (a->built) ANIM_TRY(a, hipStreamWaitEvent(s, a->ev, 0));
    ANIM_TRY(a, hipMemcpyAsync(B.d, a->d_template, a->total, hipMemcpyDeviceToDevice, s));
    rtxa::Launch L{};
    L.meshes = a->d_mesh;
    L.n = static_cast<uint32_t>(a->mesh.size());
    L.cur = a->cur;
    for (uint32_t i = 0; i < L.n; ++i)
        for (int r = 0; r < 4; ++r)
            for (int q = 0; q < 3; ++q) L.m[i][3 * r + q] = transforms[16 * i + 4 * r + q];
    L.img.meshes = reinterpret_cast<int4*>(B.d + a->mesh_off);
    L.img.tris = reinterpret_cast<float4*>(B.d + a->tri_off);
    L.img.nodes = reinterpret_cast<float4*>(B.d + a->node_off);
    L.img.parts = reinterpret_cast<int4*>(B.d + a->part_off);
    L.img.oct_bytes = a->oct_bytes;
    L.depth_limit = a->depth_limit;
    L.top_lds = 0;
    for (const rtxa::MeshDev& d : a->mesh)
        if (d.T <= rtxa::kTopLdsTris) L.top_lds = std::max(L.top_lds, d.T);
    if (a->hbm_only) L.top_lds = 0;
    L.sub_lds = a->hbm_only ? 0u : 1u;
    L.frontier_max = a->serial_frontier ? 0u : rtxa::kFrontierHistMax;
    L.cut = a->cut;
    L.wait_ticks = a->wait_ticks;
    L.debug = a->debug;
    L.epoch = ++a->epoch;
    ANIM_TRY(a, rtxa::launch_build(L, s));
    ANIM_TRY(a, hipEventRecord(a->ev, s));
    if (s != c->stream) ANIM_TRY(a, hipStreamWaitEvent(c->stream, a->ev, 0));   // the next render reads image B
    a->built = true;
    a->cur ^= 1u;
    // the context now renders from image k (the bookkeeping of rtx_upload_scene)
    if (c->sb_cur >= 0) {
        rtx_ctx::SceneBuf& O = c->sb[c->sb_cur];
        HIP_TRY(c, hipEventRecord(O.done, c->stream));
        O.pending = true;
    }
    c->sb_cur = k;
    c->scene_bytes = a->total;
    c->dev = rebase(a->dev, nullptr, B.d);
    // FAST Moller-Trumbore needs |e1| |e2| <= 2^56 for every triangle (DevScene::tri_fast).  The
    // caller's transform is arbitrary (a scale can grow the edges), so bound the rebuilt edges
    // from this transform: |e| <= |v0'| + |v1'| <= 2 (||M||_F R + |t|) for object radius R,
    // 3x3 part M and translation t (1 % for the rounding of the transformed positions),
    // with a factor-2 margin, as at registration.
    bool fast = a->reg_fast;
    for (size_t i = 0; fast && i < a->mesh.size(); ++i) {
        const float* m = transforms + 16 * i;
        double fro = 0.0, tr = 0.0;
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q) fro += double(m[4 * r + q]) * m[4 * r + q];
        for (int q = 0; q < 3; ++q) tr += double(m[12 + q]) * m[12 + q];
        const double e = 2.0 * (std::sqrt(fro) * a->obj_radius[i] + std::sqrt(tr)) * 1.01;
        fast = e * e <= 0x1p55;   // false for NaN / inf too
    }
    c->dev.tri_fast = fast ? 1u : 0u;
    c->deep_stack = false;
    c->hbm_stack = false;
    c->split_ok = a->split_ok;
    c->scene_spec = a->spec;
    std::memcpy(c->room_p0, a->room_p0, sizeof c->room_p0);
    c->has_scene = true;
    ++c->scene_gen;
    c->scene_sig = a->sig;
    return RTX_OK;
}

extern "C" int rtx_anim_status(rtx_anim* a, uint32_t i, uint32_t status[4]) {
    if (!a || !status || i >= a->mesh.size()) return RTX_E_INVALID;
    ANIM_TRY(a, hipSetDevice(a->device));
    if (a->built) ANIM_TRY(a, hipEventSynchronize(a->ev));
    ANIM_TRY(a, hipMemcpy(status, a->mesh[i].status, 16, hipMemcpyDeviceToHost));
    if (status[0])
        return afail(a, RTX_E_UNSUPPORTED,
                     status[0] & rtxa::kErrNaN        ? "NaN vertex in an animated mesh"
                     : status[0] & rtxa::kErrTimeout  ? "device build: a worker timed out waiting for a queue entry (mesh disabled)"
                     : status[0] & rtxa::kErrCapacity ? "device build: task queue or subtree table capacity exceeded (mesh disabled)"
                                                      : "animated BVH too deep for the render stack (mesh disabled)");
    return RTX_OK;
}

// Diagnostics: the last update's 64 status words of registered mesh i (0-3 as
// rtx_anim_status, 8-62 phase stamps of the build at 100 MHz, see rtx_anim.hip).
extern "C" int rtx_anim_stamps(rtx_anim* a, uint32_t i, uint32_t out[128]) {
    if (!a || !out || i >= a->mesh.size()) return RTX_E_INVALID;
    ANIM_TRY(a, hipSetDevice(a->device));
    if (a->built) ANIM_TRY(a, hipEventSynchronize(a->ev));
    ANIM_TRY(a, hipMemcpy(out, a->mesh[i].status, 512, hipMemcpyDeviceToHost));
    return RTX_OK;
}

extern "C" int rtx_anim_download(rtx_anim* a, uint32_t i, float* positions, int32_t* indices, float* normals,
                                 float* tnormals, rtx_bvh_node* nodes) {
    if (!a || i >= a->mesh.size()) return RTX_E_INVALID;
    ANIM_TRY(a, hipSetDevice(a->device));
    if (a->built) ANIM_TRY(a, hipEventSynchronize(a->ev));
    const rtxa::MeshDev& d = a->mesh[i];
    const size_t V = d.V, T = d.T;
    auto get3 = [&](const float4* src, size_t n, float* dst) -> hipError_t {
        std::vector<float4> h(n);
        const hipError_t e = hipMemcpy(h.data(), src, n * 16, hipMemcpyDeviceToHost);
        for (size_t k = 0; k < n; ++k) { dst[3 * k] = h[k].x; dst[3 * k + 1] = h[k].y; dst[3 * k + 2] = h[k].z; }
        return e;
    };
    if (positions) ANIM_TRY(a, get3(d.tpos, V, positions));
    if (normals) ANIM_TRY(a, get3(d.nrm[a->cur], T, normals));
    if (tnormals) ANIM_TRY(a, get3(d.tnrm_out, T, tnormals));
    if (indices) {
        std::vector<int4> h(T);
        ANIM_TRY(a, hipMemcpy(h.data(), d.idx[a->cur], T * 16, hipMemcpyDeviceToHost));
        for (size_t k = 0; k < T; ++k) { indices[3 * k] = h[k].x; indices[3 * k + 1] = h[k].y; indices[3 * k + 2] = h[k].z; }
    }
    if (nodes) ANIM_TRY(a, hipMemcpy(nodes, d.ref, sizeof(rtx_bvh_node) * 3 * T, hipMemcpyDeviceToHost));
    return RTX_OK;
}

