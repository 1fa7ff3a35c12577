// rtx_anim.h — Scene::Update on the device for animated meshes: the
// interface between the C-ABI (rtx_anim_* in rtx_hip.hip) and the build kernels
// (rtx_anim.hip).  Internal; not part of the installed headers.
//
// Two launches restate, in HBM and bit for bit,
//   TriangleMesh::UpdateTransforms   (source/DataTypes.h:210-236)
//   TriangleMesh::BuildBVH / Subdivide / FindBestSplitPlane / UpdateNodeBounds (:294-483)
// including the in-place swap partition's permutation of indices, normals and
// transformedNormals, which the next Update starts from — and write the result straight
// into a scene image in the render layout of rtx_upload_scene (triangle records, the node
// pairs with their 8 octant copies, the split-rendering frontier):
//   1 rtx_anim_build  workgroup (mesh, 0): transforms, per-triangle build records and the
//                     root's split; then it and kWorkers more workgroups per mesh take tasks
//                     from the mesh's queue (MeshDev::q): a node above Launch::cut triangles
//                     is split by a whole workgroup and its children queued, a smaller one is
//                     a subtree one workgroup builds level by level (then its split counts
//                     and DFS ranks)
//   2 rtx_anim_out    kOutGroups + 1 workgroups per mesh: the reference's numbering, then the
//                   node array, node records, triangle records and permuted state (workgroups
//                   0 .. kOutGroups - 1) beside the split-rendering frontier and the status
//                   words (workgroup kOutGroups)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtx.h"
#include "rtx_variants.h"

namespace rtxa {

constexpr int kAnimThreads = RTX_ANIM_THREADS;   // threads of every build workgroup
constexpr int kAnimWaves = kAnimThreads / 64;
constexpr int kMaxAnimMeshes = 32;               // animated meshes per launch (their matrices travel in the kernel arguments)
constexpr int kMaxAnimParts = 128;               // frontier entries per mesh (kPartsPerMesh)
constexpr int kMaxTop = 256;                     // temp ids of task-split nodes and their children per mesh
constexpr int kMaxSub = kMaxTop;                 // subtrees per mesh (each root is one of those ids)
constexpr int kWorkers = RTX_ANIM_WORKERS;       // task workgroups per mesh besides (mesh, 0)
constexpr int kOutGroups = 16;                   // workgroups per mesh of the output launch
// The task queue of a mesh (MeshDev::q): counters, then entries {what, reserved ids, epoch, -}
// (what: bit 31 set = a node to split, its temp id below; clear = subtree index).  head, tail
// and done are zeroed by the output launch (and at creation); the producer sets the id counters.
enum : uint32_t { kQHead = 0, kQTail = 1, kQTop = 2, kQSubIds = 3, kQDone = 4, kQEntries = 8 };
constexpr uint32_t kQCap = 2 * kMaxTop + kWorkers + 8;   // entries (tasks + the workers' last pops)
constexpr uint32_t kQWords = kQEntries + 4 * kQCap;

// A node of the build tree before the reference's numbering (64 B).
struct alignas(16) TmpNode {
    float mn[3], mx[3];          // UpdateNodeBounds
    uint32_t first, count;       // triangle range, in build positions
    int32_t l;                   // left child's temp id (right = l + 1); -1: leaf
    uint32_t depth;
    uint32_t splits;             // split nodes in the subtree, itself included
    uint32_t rank;               // DFS preorder rank among the split nodes (relative to its subtree root)
    int32_t parent;              // -1 for the root, -2 for a reserved id never used (no split)
    uint32_t sub;                // subtree index (kMaxSub: a task-split node or a leaf child of one)
    uint32_t pad[2];
};

// Per-subtree record written when a node becomes a subtree (make_subtree) and completed by its build.
struct SubRec {
    uint32_t root;               // temp id of the subtree root (a child of a task-split node, or the root)
    uint32_t base;               // first temp id of its descendants (2 n - 2 slots reserved, from kMaxTop on)
    uint32_t nalloc;             // descendants allocated
    uint32_t maxd;               // deepest level reached (absolute depth)
};

struct MeshDev {
    const float4* pos;           // object-space positions (never permuted), V
    float4* tpos;                // transformedPositions, V
    int4* idx[2];                // index triples in the order the last build left them (state), T
    float4* nrm[2];              // object-space normals in that order (state), T
    float4* tnrm;                // transformedNormals in the input order, T
    float4* tnrm_out;            // transformedNormals in the built order, T
    float* soa;                  // build records by triangle id: 9 T floats (centroid xyz, box lo xyz, box hi xyz)
    uint32_t* perm[2];           // build position -> triangle id, T each
    uint32_t* lb;                // partition scratch: left-stream wrong-side positions by rank, T
    uint32_t* rs;                // right-stream ones by rank, T
    uint32_t* rk;                // rank of each position, T
    TmpNode* tmp;                // kMaxTop + 2T: task-split nodes and their children, then subtree ranges
    uint32_t* lvl[2];            // level lists (current / next), T each; a subtree uses [first, first + n)
    SubRec* sub;                 // kMaxSub
    rtx_bvh_node* ref;           // the reference's node array (3T entries, persistent)
    uint32_t* status;            // {error bits, deepest level, nodesUsed, frontier parts, ...} + stamps
    uint32_t* q;                 // the task queue, kQWords
    uint32_t V, T;
    uint32_t mat_bits;           // material index (the triangle record's 4th float4)
    uint32_t mesh;               // mesh index in the scene
    uint32_t tri0;               // first triangle record of the mesh in the scene image
    uint32_t root;               // root node slot (odd) in the scene image
    uint32_t part0, part_cap;    // frontier entries of the mesh in the scene image
};

// status words: 0 error bits, 1 deepest level, 2 nodesUsed, 3 frontier parts, 4 subtrees,
// 5 task-split ids (output launch), 6 tasks split, 7 sticky kErrTimeout / kErrCapacity of an earlier
// update (the mesh stays disabled); 8.. phase stamps (s_memrealtime, 100 MHz, low 32 bits):
// 8 build start, 9 set-up done, 10 root split, 11 first subtree start, 12 last subtree end,
// 13 output start, 14 numbering known (frontier workgroup), 15 frontier done; 16-19 the first
// four task splits' sizes, 20-27 their start / end; 28 completeness: bit 0 = every triangle reached
// a final leaf (the tree is complete), bit 1 = a worker timed out although it was (a spurious
// timeout: reported nowhere else, the mesh stays enabled)
enum : uint32_t { kStTop0 = 8, kStSetup = 9, kStTopDone = 10, kStSub0 = 11, kStSubEnd = 12, kStOut0 = 13,
                  kStRanks = 14, kStFrontier = 15, kStComplete = 28 };

struct Image {                   // sections of the destination scene image
    int4* meshes;                // mesh records {root byte offset, nodesUsed, cull, material}
    float4* tris;
    float4* nodes;
    int4* parts;
    uint32_t oct_bytes;          // byte stride of the 8 octant node copies (0: one copy)
};

struct Launch {
    MeshDev* meshes;             // device array, n entries
    uint32_t n;
    uint32_t cur;                // state buffer (idx / nrm) holding the current order
    float m[kMaxAnimMeshes][12]; // finalTransform: rows data[0..3], xyz each (Matrix.cpp:35-56)
    Image img;
    // A rebuilt tree this many levels deep or deeper would overflow the render kernel's
    // kStackDepth-entry DFS stack: the build then disables the mesh in the image (node count
    // 0, no frontier parts) and reports kErrDepth.  rtxd::kStackDepth; lower only in tests.
    uint32_t depth_limit;
    uint32_t top_lds;            // meshes up to this many triangles split the root from LDS (0: none)
    uint32_t sub_lds;            // tasks and subtrees build from LDS when they fit (0: always from HBM)
    uint32_t epoch;              // this update's number (> 0): tags the queue entries it publishes
    uint32_t cut;                // nodes above this many triangles are split as tasks, smaller ones are subtrees
    uint32_t frontier_max;       // meshes up to this many triangles select the frontier in parallel (else serially)
    uint64_t wait_ticks;         // a worker's wait for a queue entry, s_memrealtime ticks (100 MHz): 200 ms; tests lower it
    uint32_t debug;              // tests only (RTX_ANIM_DEBUG): kDbgDropEntry, kDbgLateTimeout
};
// RTX_ANIM_DEBUG bits (tests of the timeout path): kDbgDropEntry — the worker that takes queue entry
// 0 drops it as if it had timed out before it was published (the tree is then incomplete);
// kDbgLateTimeout — workers that leave because the tree is complete also report a timeout (as a
// worker whose wait ran out just as the last triangles were placed would)
enum : uint32_t { kDbgDropEntry = 1u, kDbgLateTimeout = 2u };
constexpr uint32_t kTopLdsTris = 3136;   // the largest top_lds (rtx_anim.hip's LDS budget)
constexpr uint32_t kFrontierHistMax = 4096;   // the largest frontier_max (the count histogram's bins)

// kErrTimeout: a worker gave up waiting for a queue entry (Launch::wait_ticks); kErrCapacity: a
// task-queue or subtree-table guard fired.  A timeout leaves the tree incomplete only when the entry
// the worker claimed was a real task (published later, then never run); a worker waiting on an
// index no task ever takes gives up harmlessly.  The output launch tells the two apart by whether
// every triangle reached a final leaf (status word kStComplete): an incomplete tree (and any
// capacity error) is not written and the mesh is disabled in the image (no frontier parts, node
// count 0), as for kErrDepth; a complete one is written as usual and the timeout bit is cleared.
enum : uint32_t { kErrNaN = 1u, kErrDepth = 2u, kErrTimeout = 4u, kErrCapacity = 8u };
constexpr uint64_t kWaitTicks = 20000000ull;   // Launch::wait_ticks' default: 200 ms at 100 MHz

hipError_t launch_build(const Launch& L, hipStream_t stream);

}  // namespace rtxa
