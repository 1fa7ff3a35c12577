// rtx_ctx.h — the render context (rtx_ctx, the opaque handle of include/rtx.h) and the frame
// policies that rtx_policy.hip implements for rtx_hip.hip: the split tuner, the throughput /
// in-flight choice, the frontier refinement and the deferred join of the split chain.  Internal to
// librtx_hip.so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "rtx.h"
#include "rtx_cull.h"
#include "rtx_kernels.h"

using namespace rtxd;

// The two kinds of cull-record tree values (rtx_cull_tris / rtx_cull_nodes in rtx_hip.hip): margin +
// dt per triangle, a box per node slot.  Margins and dt are >= 0 or +inf (never NaN), box bounds never
// NaN either, so the trees' min / max folds are exact in any order.
struct alignas(8) CullMD {
    float m, dt;
};
struct alignas(16) CullBox {
    float lo[3], pad0, hi[3], pad1;
};

struct rtx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    // scene image in HBM (one allocation, 256-B aligned sections)
    // Two scene images (device + pinned staging), alternated by uploads: an upload packs
    // into the image no queued frame reads and copies it asynchronously, so the host can
    // prepare the next animated frame while the GPU renders this one.
    struct SceneBuf {
        char* d = nullptr;
        char* h = nullptr;
        size_t cap = 0;
        hipEvent_t done = nullptr;   // recorded after the last frame that reads this image
        bool pending = false;
        float4* cull = nullptr;      // the image's cull records (DevScene::cull), device only
        size_t cull_cap = 0;
    };
    SceneBuf sb[2];
    int sb_cur = -1;
    size_t scene_bytes = 0;
    std::string scene_sig;   // topology of the uploaded scene (keeps the tile schedule across re-uploads)
    DevScene dev{};
    bool has_scene = false;
    // frame buffer in HBM
    uint32_t* d_px = nullptr;
    float* d_rgb = nullptr;
    size_t px_cap = 0, rgb_cap = 0;
    unsigned long long* d_counters = nullptr;
    // last render
    // cost-ordered tile dispatch
    uint32_t* d_order = nullptr;
    uint32_t* d_order_xcd = nullptr;    // the XCD-affine re-deal of d_order (rtx_sched_xcd)
    bool xcd_order = false;             // RTX_XCD_ORDER=1
    uint32_t* d_cost = nullptr;
    uint32_t* d_saved_cost = nullptr;   // last one-piece cost per tile
    uint32_t* d_hist = nullptr;         // per (class, chunk) tile counts -> slot bases (rtx_sched_*)
    unsigned long long* d_csum = nullptr;   // per chunk cost sums
    unsigned long long* d_thr = nullptr;    // heavy threshold of the measured frame
    uint32_t sched_cap = 0;
    std::string sched_key;
    bool sched_ready = false;
    bool sched_enabled = true;
    uint64_t sched_frame = 0;
    uint64_t scene_gen = 0;
    // split rendering of heavy tiles: double-buffered flag/list sets (the reorder kernel
    // fills the staging set; the host adopts it, with its count, at the next frame)
    uint32_t* d_heavy_flag[2] = {nullptr, nullptr};
    uint32_t* d_heavy_list[2] = {nullptr, nullptr};
    uint32_t* d_heavy_n = nullptr;
    uint32_t* h_heavy_n = nullptr;   // pinned
    hipEvent_t ev_heavy = nullptr;
    hipStream_t split_stream = nullptr;   // split launches run beside the main kernel
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // Throughput mode (prepare): another context of this process on the same device still had a frame
    // in flight when this one was queued (ev_frame, the end of each queued frame; g_frames).  The
    // GPU then interleaves the contexts' frames and a tile's critical path is hidden by the other
    // frames, so the split launches only add work: the measured frames select heavy tiles with at
    // least kThroughputPermille and the tuner (whose timings the other frames distort) waits.
    hipEvent_t ev_frame = nullptr;
    bool in_registry = false;                   // listed in g_frames (its ev_frame is recorded per frame)
    bool concurrent = false;
    bool throughput_off = false;                // RTX_THROUGHPUT=0
    // in flight (kInflightCritPermille): the heaviest tile's one-piece cost measured in the last
    // serialized measurement (cost units), the threshold (RTX_INFLIGHT_CRIT), and whether the last
    // frame rendered one piece because of it
    uint32_t max_cost_serial = 0;
    // deferred join (rtx_ctx::join_pending): the last frame's split chain has not been joined into the
    // frame stream; the next frame's main kernel may start beside it when it repeats the frame exactly
    // (same parameters, cameras, scene image and heavy set: the two write disjoint tiles) — anything
    // else joins first (join_split).  join_*: that frame's identity.
    bool join_pending = false;
    bool join_off = false;                      // RTX_DEFER_JOIN=0
    // frames in flight defer too, except while the in-flight overlap window is timed (RTX_DEFER_INFLIGHT=0: never)
    bool defer_inflight = true;
    rtx_render_params join_p{};
    rtx_camera join_cams[kMaxViews]{};
    int join_views = 0;
    uint64_t join_gen = 0;
    int join_sb = -1;
    const uint32_t* join_heavy = nullptr;
    uint32_t join_heavy_n = 0;
    // the split frames' interval in flight on this context's stream (inflight_onepiece): 0 skipping
    // kInflightWindowSkip frames, 2 timing kInflightWindow frames, 3 waiting for the end event, 4 done
    uint32_t win_state = 0;
    uint32_t win_frames = 0;
    int win_rec = -1;                           // the ev_win slot this frame's end records (-1 none)
    float win_interval_ms = 0.f;
    hipEvent_t ev_win[2] = {};
    uint32_t inflight_crit = kInflightCritPermille;
    bool frame_onepiece = false;
    int heavy_cur = 0;
    uint32_t heavy_n = 0;
    bool heavy_pending = false;
    uint32_t split_mode = 1;         // 0 off, 1 auto, 2 force (RTX_SPLIT=0 / unset / force)
    uint32_t split_slots = 0;        // concurrent render waves on this device
    uint32_t split_permille = kSplitPermille;   // RTX_SPLIT_FACTOR (fixes it: no tuner)
    uint32_t split_min = kSplitMinCost;         // RTX_SPLIT_MIN_US: the least cost (16-cycle units) a split tile has
    // Split-threshold tuner: the frame is max(main kernel, split chain), and the
    // threshold that balances the two is the fastest (Synthetic100k: factor 2.0, W4_Optional 1.5).
    // A measured frame with split tiles times both (ev_tune: fork, main kernel end, chain end); at
    // its adoption the factor the timed set was selected with moves toward the balance, by steps
    // that shrink when the direction flips, until the two are within 4 % or the step is < 1.5 %.
    bool tune_on = true;                        // RTX_SPLIT_TUNE=0 / RTX_SPLIT_FACTOR: off
    bool tune_done = false;
    bool tune_rec = false;                      // the measured frame in flight recorded ev_tune
    uint32_t tune_rec_permille = 0;             // ... and the factor its (current) heavy set was selected with
    uint32_t set_permille[2] = {0, 0};          // per heavy set: the factor the schedule selected it with
    uint32_t tune_steps = 0;
    int tune_dir = 0;
    float tune_step = 1.15f;
    float tune_main_ms = 0.f, tune_chain_ms = 0.f;   // the last timed frame (rtx_split_tune_info)
    float tune_best_span = 0.f;                 // the fastest max(main, chain) seen, and its factor
    uint32_t tune_best_permille = 0;
    hipEvent_t ev_tune[3] = {nullptr, nullptr, nullptr};
    uint32_t sched_period = kSchedPeriod;       // RTX_SCHED_PERIOD (tuning)
    // motion mode (kMotionFrames): frames left, and the previous frame's cameras it compares
    uint32_t motion_left = 0;
    bool frame_motion = false;                  // the frame being prepared / launched is in motion mode
    bool motion_off = false;                    // RTX_MOTION=0: always the static schedule (A/B)
    int prev_views = 0;
    ViewCam prev_cam[kMaxViews] = {};
    uint32_t split_parts = kPartsPerMesh;            // RTX_SPLIT_PARTS (tuning)
    // frontier refinement (kRefineRounds): the current image's parts (host copy of the real entries;
    // the image reserves kMaxParts), its parts section, the round and state (0 waiting for a split
    // frame, 1 measured frame queued, 2 done), frames to wait, the last round's longest part wave
    bool refinable = false;
    bool refine_off = false;                         // RTX_REFINE=0
    // RTX_REFINE_ROUNDS / _SPLITS / _TOP (permille): the kRefine* constants (tuning)
    uint32_t refine_rounds = kRefineRounds, refine_splits = kRefineSplits, refine_top = kRefineTopPermille;
    std::vector<int4> h_parts;
    std::vector<int4> h_parts_base;                  // the upload's frontier (each launch shape starts from it)
    int4* parts_dev = nullptr;
    uint32_t refine_round = 0;
    int refine_state = 2;
    uint32_t refine_wait = 0;
    uint32_t refine_quiet = 0;                       // frames of this shape still to wait
    uint32_t refine_prev_max = 0;
    bool refine_rec = false;
    hipEvent_t ev_refine = nullptr;
    uint32_t* d_part_max = nullptr;
    std::vector<uint32_t> h_part_max;
    bool split_ok = false;           // the uploaded scene admits split rendering
    bool deep_stack = false;         // the uploaded scene needs rtx_render_kernel<..., DEEP = true>
    bool hbm_stack = false;          // ... with its stacks in HBM (HSTK = true): kStackDepthDeep or more levels
    uint32_t max_depth = 0;          // deepest BVH level of the uploaded scene
    uint4* d_hstk = nullptr;         // the HBM stacks (and the instrumented variant's masks), grown on demand
    unsigned long long* d_hstkT = nullptr;
    size_t hstk_entries = 0;
    int scene_spec = 0;              // kSpec* facts of the uploaded scene (kernel specialisation)
    float room_p0[5] = {};           // kSpecRoomPlanes: plane k's origin on axis kRoomAxes[k]
    bool no_spec = false;            // RTX_NO_SPEC=1: always the generic kernel (tests)
    unsigned long long* d_hit_key = nullptr;
    uint32_t* d_occ = nullptr;
    // Light-major frames (FrameArgs::lm_*, DESIGN.md §6, opt-in): lm_mode 0 never (default), 1 auto
    // (RTX_LIGHT_MAJOR=auto: a launch of at most lm_tiles wave tiles, kLmSlotsPercent of the resident
    // wave slots, RTX_LIGHT_MAJOR_TILES), 2 always (RTX_LIGHT_MAJOR=1)
    uint32_t lm_mode = 0;
    uint32_t lm_tiles = 0;
    uint32_t lm_waves = 0;                      // PHASE 5's persistent waves: every resident slot (32 per CU)
    float4* d_lm_rec = nullptr;                 // 2 float4 per tile pixel
    unsigned long long* d_lm_mask = nullptr;    // per (tile, light)
    size_t lm_rec_tiles = 0, lm_mask_cap = 0;
    bool frame_lm = false;                      // the frame being launched is light-major
    // exact cull (DevScene::cull): on for host uploads (RTX_NO_CULL=1: off); the
    // scratch of its record launches (the segment trees of the per-triangle boxes and of each
    // anchor's margins, the slots' boxes, the trees' arrival counters) and the node-slot ranges
    // in the current image
    bool no_cull = false;
    float cull_ratio = 1.5f;              // CullParams (RTX_CULL_RATIO, RTX_CULL_LEAVES: tuning)
    double cull_min_sa = 1.5;             // upload_scene's worth test (RTX_CULL_MIN_SA)
    bool cull_leaves = false;
    // Animated loops re-upload every frame and render it once, so the records are rebuilt per
    // frame.  Round 4's records cost more than a frame and were skipped after two such uploads;
    // the segment-tree records (tens of us) are built for every upload.  RTX_CULL_ANIMATED=0
    // restores the skip (after two consecutive uploads rendered at most once each, until an
    // upload is rendered twice).
    bool cull_animated = true;
    uint32_t renders_since_upload = 0;
    uint32_t short_uploads = 0;
    // An upload in that pattern (the previous upload was rendered at most once too) moves the
    // geometry under a fixed tile schedule as a moving camera does: the next frame starts motion
    // mode when the scene has split tiles (prepare; RTX_MOTION=0 turns both off).
    bool upload_motion = false;
    // The cull's worth estimate (upload_scene: the surface areas of every node's reference box and
    // tight box, tens of us of host time per upload) is reused by the uploads of such a loop for
    // kCullWorthReuse uploads while the scene's counts stay the same: the decision only picks the
    // faster of two exact walks.
    int cull_worth = -1;
    uint32_t cull_worth_age = 0;
    std::string cull_worth_sig;
    CullBox* d_cull_btree = nullptr;      // 2n entries
    CullMD* d_cull_mtree = nullptr;       // 2n entries per anchor of one launch
    size_t cull_mtree_cap = 0;            // entries d_cull_mtree holds
    uint32_t cull_failures = 0;           // record builds that failed (the image then renders unculled)
    uint32_t cull_fail_at = 0, cull_launches = 0;   // RTX_CULL_FAIL=k: the k-th record build fails (tests)
    CullBox* d_cull_nbox = nullptr;       // per node slot of the current image
    uint32_t* d_cull_arrive = nullptr;    // per tree (kCullMaxAnchors margin trees, then the box tree)
    size_t cull_tree_cap = 0, cull_nbox_cap = 0;   // leaves n the trees hold, slots nbox holds
    uint32_t cull_top_lds = kCullTopLds;  // RTX_CULL_TOP_LDS (tests: the global-memory top levels)
    const uint2* cull_rng = nullptr;
    uint32_t cull_nslots = 0, cull_ntris = 0, cull_n = 0;
    float cull_view[kMaxViews][3] = {};   // camera origin each view's records of the current image were made for
    uint32_t cull_view_valid = 0;         // bit v: view v's records are current
    double cull_bmin[3] = {}, cull_bmax[3] = {};   // the meshes' box (a camera anchor's t bound, cull_bt)
    uint64_t cull_updates = 0;            // camera-anchor record launches so far (rtx_cull_info)
    float cull_anchor[kMaxViews + kMaxCullLights][5] = {};   // per record copy: anchor xyz, w, bt (rtx_cull_dump)
    std::vector<std::array<float, 4>> cull_lights;   // the uploaded lights' anchors {origin, T}
    bool cull_boxes_pending = false;      // an upload's boxes and light records wait for its first frame
    rtx_render_params last{};
    int last_views = 1;
    bool last_valid = false, last_rgb = false;
};

namespace rtxh {

inline int fail(rtx_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define HIP_TRY(ctx, call)                                                                  \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail((ctx), RTX_E_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

// The other contexts on c's device with a frame still in flight, and the registry of contexts
// whose frames can be (rtx_ctx::ev_frame, throughput mode).
uint32_t frames_concurrent(rtx_ctx* c);
void frames_note(rtx_ctx* c);
void frames_forget(rtx_ctx* c);
// Layout of an upload whose meshes may reserve rebuild-sized regions (rtx_anim_*): a mesh
// with reserve[i] set owns 2T node slots from its root (the most a rebuild can number) and
// exactly `target` frontier entries (unused ones are {-1, ...}), so a device rebuild can
// rewrite it in place without moving anything else.
struct UploadLayout {
    std::vector<uint8_t> reserve;                            // in, per mesh
    std::vector<uint32_t> tri0, root, part0, part_cap;       // out, per mesh
    std::vector<int> depth;
    double max_ee = 0.0;
    size_t total = 0;
    uint32_t oct_bytes = 0;
    size_t tri_off = 0, node_off = 0, part_off = 0, mesh_off = 0;   // section offsets in the image
};

// Upload a scene into the context's next image (rtx_hip.hip; rtx_upload_scene, and the device
// Update's registration with `lay`).
int upload_scene(rtx_ctx* c, const rtx_scene* s, UploadLayout* lay);

// One step of the split-threshold tuner from a timed frame's main kernel and chain (ms).
void split_tune(rtx_ctx* c, float main_ms, float chain_ms);
// Join the last frame's deferred split chain into the frame stream (rtx_ctx::join_pending).
int join_split(rtx_ctx* c);
// One round of the frontier refinement once its measured frame has completed (rtx_ctx::refine_*).
int refine_round(rtx_ctx* c);
// The heaviest tile's serialized one-piece time over the split frame's serialized span (0 until known).
float inflight_ratio(const rtx_ctx* c);
// Whether a frame in flight, with k frames of this device's contexts at once, renders one piece.
bool inflight_onepiece(rtx_ctx* c, uint32_t k);

}  // namespace rtxh
