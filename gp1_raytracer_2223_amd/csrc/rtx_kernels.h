// rtx_kernels.h — device layout of the uploaded scene and the per-frame launch record.
// Shared by the kernels and the host-side upload code in rtx_hip.hip.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace rtxd {

// Per-wave DFS stack entries in LDS (node index + 64-bit lane mask).  The host checks
// every uploaded BVH's depth against this before accepting the scene.
constexpr int kStackDepth = 64;
// Deep-stack variant (BVH kStackDepth..kStackDepthDeep-1 levels deep): 16 KB of LDS per
// wave for the stack; deeper trees take the variant whose stacks are in HBM (DevScene::hstk).
constexpr int kStackDepthDeep = 1024;
#ifndef RTX_BLOCK_THREADS
#define RTX_BLOCK_THREADS 64
#endif
constexpr int kBlockThreads = RTX_BLOCK_THREADS;   // independent waves, each an 8 x 8 pixel "wave tile"
constexpr int kWavesPerBlock = kBlockThreads / 64;
constexpr int kWaveTile = 8;
constexpr int kReorderThreads = 256;   // rtx_sched_count / rtx_sched_scatter workgroup
constexpr int kSchedChunk = 1024;      // tiles per scheduling workgroup (4 per thread)
constexpr int kScanThreads = 1024;     // rtx_sched_scan (one workgroup)
constexpr int kCostBuckets = 32;
constexpr int kSchedPeriod = 64;      // frames between tile-cost measurements
// A frame whose camera differs from the previous frame's starts (or extends) motion mode for this
// many frames: every frame is measured whose previous measurement has completed (no host wait).
constexpr int kMotionFrames = 64;
constexpr uint32_t kCullWorthReuse = 16;  // animated uploads per cull worth estimate (rtx_ctx::cull_worth)

// Split rendering of heavy tiles: a wave tile whose measured cost exceeds
// kSplitPermille/1000 x (frame cost / concurrent wave slots) is rendered by three extra
// launches in which its BVH traversals are cut into subtree parts run by separate workgroups.
constexpr int kPartsPerMesh = 64;      // target frontier size per mesh BVH (with the exact cull, Synthetic100k
                                       // 1080p: 64 parts 1.00 ms, 128 1.12, 256 1.46; before it 128 beat 64 by 6 %)
constexpr int kMaxParts = 1024;        // all meshes together
// Frontier refinement (rtx_ctx::refine_*): a static scene's split frame is measured per part (its
// longest closest-hit and shadow waves), and the parts whose waves are within kRefineTopPermille /
// 1000 of the longest are cut into their two children (at most kRefineSplits per round, kRefineRounds
// rounds, kRefineQuiet frames after an upload): the chain's critical path is its longest part waves
// (profiles/r06/floor_hist_chain.jsonl), and cutting the few heaviest parts shortens it
// (profiles/r06/part_refine.txt: Synthetic100k share of 8 0.607 -> 0.441-0.473 ms).
constexpr int kPartShards = 16;
constexpr uint32_t kRefineRounds = 3;
constexpr uint32_t kRefineSplits = 8;
constexpr uint32_t kRefineTopPermille = 600;
constexpr uint32_t kRefineQuiet = 32;
// ... and only while the longest part waves (closest hit + shadow) exceed kRefineMinUs: shorter ones
// are not the chain's cost (its launches are), and more parts only add waves (Bunny + 8 lights)
constexpr uint32_t kRefineMinUs = 100;
// ... and than kRefineOverMainPermille / 1000 x the split frame's main kernel (the tuner's last): a
// whole 1080p Synthetic100k frame (main kernel ~0.8 ms, longest part waves ~0.7) is bound by its work,
// and its frames in flight lost throughput to the extra part waves (0.51 -> 0.56 ms per frame)
constexpr uint32_t kRefineOverMainPermille = 1500;
constexpr int kMaxHeavyTiles = 8192;   // heavy wave tiles per frame (hit-key buffer: 64 px each)
// split factor floor while other contexts' frames are in flight (rtx_ctx::ev_frame)
constexpr uint32_t kThroughputPermille = 2600;
// In flight (rtx_ctx::concurrent) a split frame's extra work (the chain's repeated path walks, its
// launches) can cost more than its shorter critical path saves, since the other contexts' frames fill
// the GPU beside a long tile (2 frames in flight, profiles/r06/inflight_split_ab.txt: Bunny + 8 lights
// 4K share of 8 0.067 split / 0.059 ms one piece, W4_Optional share of 8 0.110 / 0.088, Synthetic100k
// share of 8 0.405 / 0.622).  Two frames in flight hide a tile as long as about two frames' time: a
// frame in flight renders one piece when its heaviest tile's one-piece cost (measured serialized) is
// below kInflightCritPermille / 1000 x the split frame's serialized span (the tuner's best, main
// kernel or chain), which holds for the first two and not for Synthetic100k (profiles/r06/
// inflight_crit_ab.txt).  RTX_INFLIGHT_CRIT=f sets the factor (0: split as serialized frames do).
constexpr uint32_t kInflightCritPermille = 1600;
// ... or when split frames in flight do not overlap: k frames in flight at once, their interval on a
// context's stream at least k x the serialized span / kInflightOverlapMin (timed over kInflightWindow
// frames after kInflightWindowSkip; W4_Optional's shares: the chain's work fills the GPU)
constexpr float kInflightOverlapMin = 1.15f;
constexpr uint32_t kInflightWindow = 32;
constexpr uint32_t kInflightWindowSkip = 16;
// 1.5 (v14 sweep, tools/split_sweep.sh): Synthetic100k 4.38 -> 3.51 ms, W4_Optional within
// noise of 2.0; below 1.25 the split overhead outgrows the tail it removes
constexpr int kSplitPermille = 1500;
constexpr int kMaxSplitLights = 32;    // occlusion bits per pixel
// A tile is split only if its cost is also at least kSplitMinUs (in the cost unit, 16 shader cycles at
// 2.4 GHz): a launch with fewer tiles than wave slots (a stripe share) starts every tile at once, and
// there a tile of a few tens of us finishes sooner in one piece than behind the split chain's three
// dependent launches.  Floor sweep (profiles/r06/split_min_sweep.txt, serialized ms, floors 0 / 30 / 60 /
// 100 us): W4_Bunny 1080p share of 8 ranks 0.067 / 0.071 / 0.052 / 0.052, Bunny + 8 lights 4K share of 8
// 0.098 / 0.100 / 0.100 / 0.110, W4_Optional and Synthetic100k (full frames and shares) within 2 %.
constexpr uint32_t kSplitMinUs = 60;
constexpr uint32_t kSplitMinCost = kSplitMinUs * 2400 / 16;
// Kernel specialisation (rtx_render_kernel's SPEC): uniform facts compiled in.
// Bits 0-3: the material kinds the geometry references (bit RTX_MAT_*; none set = any kind).
constexpr int kSpecKindSolid = 1 << 0;
constexpr int kSpecKindLambert = 1 << 1;
constexpr int kSpecKindPhong = 1 << 2;
constexpr int kSpecKindCT = 1 << 3;
constexpr int kSpecKindAll = 15;
constexpr int kSpecPoint = 16;         // every light is a point light
constexpr int kSpecNoSpheres = 32;     // no spheres
constexpr int kSpecCombShadows = 64;   // lighting mode Combined, shadows on
constexpr int kSpecFivePlanes = 128;   // exactly 5 planes (the reference's room: W3, W4, the synthetic scenes)
constexpr int kSpecOneMesh = 256;      // exactly 1 triangle mesh
constexpr int kSpecNoMesh = 512;       // no triangle mesh
// The 5 planes are the reference's room (RoomPlanes, Scene.cpp:263-267): plane k's normal is
// +-1 on axis kRoomAxes[k] and zero elsewhere, and every origin coordinate is finite with
// magnitude <= 2^64.  Then, for a ray with a finite origin, HitTest_Plane's quotient is
// (p0_A - o_A) / d_A whenever the plane can be hit (rtx_hip.hip, room_a).
constexpr int kSpecRoomPlanes = 1024;
constexpr int kRoomAxes[5] = {2, 1, 1, 0, 0};
constexpr int kSpecCullBack = 2048;    // every mesh culls back faces (the cull sign is known)
// The compiled variants, most specific first (the launch takes the first one whose facts hold):
//   0  Lambert only, one back-face-culled mesh, no spheres (W4_Bunny, Synthetic100k, Bunny + 8 lights)
//   1  Lambert + Cook-Torrance, one back-face-culled mesh, no spheres (W4_Optional)
//   2  Lambert + Cook-Torrance, spheres, no mesh (W3)
//   3  Lambert + Cook-Torrance, spheres and meshes (W4_Reference)
//   4  as 3 for five planes of any other arrangement
// all with point lights, 5 planes, Combined lighting + shadows; 0-3 in the room.
constexpr int kSpecCommon = kSpecPoint | kSpecCombShadows | kSpecFivePlanes;
constexpr int kSpecVariants[] = {
    kSpecCommon | kSpecRoomPlanes | kSpecCullBack | kSpecKindLambert | kSpecNoSpheres | kSpecOneMesh,
    kSpecCommon | kSpecRoomPlanes | kSpecCullBack | kSpecKindLambert | kSpecKindCT | kSpecNoSpheres | kSpecOneMesh,
    kSpecCommon | kSpecRoomPlanes | kSpecKindLambert | kSpecKindCT | kSpecNoMesh,
    kSpecCommon | kSpecRoomPlanes | kSpecKindLambert | kSpecKindCT,
    kSpecCommon | kSpecKindLambert | kSpecKindCT,
};

// Work counters (SURVEY §8(d) cost model; same order as the oracle's).
enum Counter {
    kPixels = 0, kSphere, kPlane, kSlab, kTri, kHit, kShadow, kOccluded,
    kShadeBase, kShadeLambert, kShadePhong, kShadeCT,
    // diagnostics (not part of the FLOP model): per-WAVE packet work, counted once per
    // wave by lane 0 — node-pair tests and triangle tests the wave executed
    kWaveNodeTests, kWaveTriTests,
    // the culled walk's counting variant (rtx_count_work_culled): per-lane exact-cull box tests
    kCullTests, kNumCounters
};
constexpr int kModelCounters = 12;

// HBM scene image, every record 16-byte aligned so a wave-uniform index
// becomes one s_load_dwordx4/x8 (scalar cache) instead of 64 vector loads:
//   sphere   1 x float4 {cx, cy, cz, r*r}          + mat u32
//   plane    2 x float4 {ox, oy, oz, mat}, {nx, ny, nz, 0}
//   triangle 4 x float4 {v0, n.x}, {v1-v0, n.y}, {v2-v0, n.z}, {mat}  (BVH leaf order, all meshes)
//   node     2 x float4 {min, link}, {max, tri_count}  link = first tri (leaf) | left node
//   mesh     int4 {first node, n nodes, cull, mat}
//   light    2 x float4 {origin, type}, {color, intensity}
//   material 3 x float4 {kind, rgb}, {kd, ks, exp, metal}, {rough, (rgb*kd)/PI}
struct alignas(64) Tri {
    float4 a, b, c, d;   // {v0, n.x}, {v1-v0, n.y}, {v2-v0, n.z}, {mat, 0, 0, 0}
};

struct DevScene {
    const float4* __restrict__ spheres;
    const uint32_t* __restrict__ sphere_mat;
    const float4* __restrict__ planes;
    const Tri* __restrict__ tris;
    const float4* __restrict__ nodes;
    const int4* __restrict__ meshes;
    const float4* __restrict__ lights;
    const float4* __restrict__ materials;
    // BVH frontier for split rendering: {mesh, node slot, path bits (bit d: right child at
    // depth d+1), depth} — every triangle of every mesh lies under exactly one entry
    const int4* __restrict__ parts;
    uint32_t n_spheres, n_planes, n_meshes, n_lights, n_materials, n_tris, n_nodes, n_parts;
    // every triangle has |e1| * |e2| <= 2^56: with |d| < 2, Moller-Trumbore's determinant
    // stays inside the exact fast-reciprocal domain (rtx_fastdiv.h)
    uint32_t tri_fast;
    // Byte stride between the 8 octant copies of the node array (0: no copies, the octant
    // slab path is off).  Copy k swaps the axes whose bit is set in k (the axes a ray of
    // octant k crosses from hi to lo): per axis it stores (hi, lo) instead of (lo, hi),
    // every (lo, hi) ordered lo <= hi (checked at
    // upload); links, counts and slots are the same in every copy.  Copy 0 is the array
    // the other slab forms read.
    uint32_t oct_bytes;
    // DFS stacks in HBM for a BVH kStackDepthDeep or more levels deep (rtx_render_kernel<...,
    // HSTK = true>): hstk_depth entries per wave, by the wave's index in the launch
    uint4* hstk;
    unsigned long long* hstkT;   // the instrumented variant's tested-lane masks
    uint32_t hstk_depth;
    // Exact cull (rtx_cull.h): per anchor a copy of cull_stride bytes of records at
    // the node slots' byte offsets ({c, E.x}, {E.y, E.z, -, -}: box c +- E); anchor v < kMaxViews =
    // view v's camera, kMaxViews + l = light l, whose shadow rays are culled only up to tmax
    // cull_T[l].  cull_stride 0: off.
    const float4* __restrict__ cull;
    const float* __restrict__ cull_T;
    uint32_t cull_stride;
};

#ifndef RTX_OCT_MAX_BYTES
#define RTX_OCT_MAX_BYTES (size_t(1) << 20)
#endif
constexpr size_t kOctantMaxNodeBytes = RTX_OCT_MAX_BYTES;   // octant node copies only below this (per copy)
constexpr size_t kOctantDeviceMinBytes = size_t(64) << 10;   // from this size copies 1..7 are written on the device
constexpr int kMaxViews = 8;   // views (camera positions) rendered by one launch
constexpr int kMaxCullLights = 32;   // lights with a cull anchor (more: the scene renders without the cull)
// The records' range reductions run over segment trees of the per-triangle values (rtx_cull_tris_*):
// kCullTreeWG leaves per workgroup; the last workgroup of a tree builds the levels above the
// workgroups' roots in LDS when there are at most kCullTopLds of them (else in global memory).
constexpr uint32_t kCullTreeWG = 256;
constexpr uint32_t kCullMaxAnchors = kMaxViews + kMaxCullLights;   // per record launch (after an upload: lights + views)
constexpr uint32_t kCullTopLds = 1024;

struct ViewCam {
    float origin[3];
    float right[3];
    float up[3];
    float forward[3];
    float fov;
    // room planes (kSpecRoomPlanes): p0_A - origin_A per plane, binary32 on the host, and
    // whether all five are 0 or in [2^-60, 2^60] (div_rn's numerator domain, rtx_fastdiv.h)
    float room_a[5];
    uint32_t room_fast;
    float cull_bt;    // the view's camera-anchor cull records: their t bound (CullRay::bt)
};

struct FrameArgs {
    ViewCam cam[kMaxViews];       // the tile's view selects the camera
    uint32_t n_views;             // views in the launch
    float aspect;                 // (float)W / (float)H  (Renderer.cpp:30)
    float inv_width, inv_height;  // RN(1/W), RN(1/H): IEEE divisions on the host
    uint32_t width, height;
    int32_t mode, shadows;
    uint32_t rshift, gshift, bshift, amask;
    uint32_t groups_per_stripe;   // stripe_rows / 8 (0 => whole image)
    uint32_t stripe_first, stripe_step;
    uint32_t tiles_x, tiles_y;    // 8x8 wave tiles per view row / per view column (owned)
    uint32_t n_tiles;             // wave tiles in the launch (all views)
    const uint32_t* __restrict__ order;   // dispatch permutation of the tiles (null = identity)
    uint32_t* __restrict__ cost;          // per-tile cost of this frame (null = not measured)
    // camera in motion (a measured frame of rtx_ctx::motion_left): the split launches add their
    // waves' durations to their tile's cost, which then replaces the tile's saved one-piece cost
    uint32_t part_cost;
    uint32_t* __restrict__ out_px;   // view v at out_px + v * width * height
    float* __restrict__ out_rgb;     // may be null
    unsigned long long* __restrict__ counters;  // COUNT variant only
    unsigned long long* __restrict__ stamps;    // diagnostic RTX_STAMPS builds only (null otherwise)
    unsigned long long* __restrict__ split_stamps;   // diagnostic: per (phase 1/2, part) {sum, max, steps}
    // split rendering (null / unused when no tile is heavy)
    const uint32_t* __restrict__ heavy_flag;    // per tile: non-zero = rendered by the split launches
    const uint32_t* __restrict__ heavy_list;    // split launches: heavy index -> tile
    uint32_t heavy_n;                           // entries of heavy_list in use
    unsigned long long* __restrict__ hit_key;   // per heavy pixel: min {t bits, triangle}
    uint32_t* __restrict__ occ_bits;            // per heavy pixel: bit l = mesh occludes light l
    // split launches of a frame the frontier refinement measures (rtx_ctx::refine_*; else null): per
    // (phase 1/2, part, shard) the longest wave, 16-cycle units (atomicMax; shard = wave % kPartShards)
    uint32_t* __restrict__ part_max;
    // Light-major frame (opt-in): PHASE 4 writes each pixel's hit record, PHASE 5 runs
    // persistent waves over the (tile, light) shadow rays (items in cost order, the light fastest) and
    // publishes each light's occluded lanes, PHASE 6 shades every light in the reference's order.
    uint32_t lm_lights;                         // lights per tile (PHASE 5 items = n_tiles x lm_lights)
    float4* __restrict__ lm_rec;                // per tile pixel: {h, n.x}, {n.y, n.z, mat bits, did}
    unsigned long long* __restrict__ lm_mask;   // per (tile, light): the lanes whose shadow ray is occluded
};

// Light-major frames (opt-in: RTX_LIGHT_MAJOR=1 always, =auto while a launch has at most kLmSlotsPercent /
// 100 wave tiles per resident wave slot, RTX_LIGHT_MAJOR_TILES overrides; default never: each (tile, light)
// item repeats ~200 instructions of set-up for ~200 of shadow walk, measured 1.5x slower than one piece
// at 4K / 8 ranks, profiles/r06), with shadows on and 2..kMaxLmLights lights.
constexpr uint32_t kLmSlotsPercent = 250;
constexpr uint32_t kMaxLmLights = 32;

}  // namespace rtxd
