// rtx_anim.h — Scene::Update on the device for animated meshes: the
// interface between the C-ABI (rtx_anim_* in rtx_hip.hip) and the build kernel
// (rtx_anim.hip).  Internal; not part of the installed headers.
//
// One workgroup per animated mesh restates, in HBM and bit for bit,
//   TriangleMesh::UpdateTransforms   (source/DataTypes.h:210-236)
//   TriangleMesh::BuildBVH / Subdivide / FindBestSplitPlane / UpdateNodeBounds (:294-483)
// including the in-place swap partition's permutation of indices, normals and
// transformedNormals, which the next Update starts from — and writes the result straight
// into a scene image in the render layout of rtx_upload_scene (triangle records, the node
// pairs with their 8 octant copies, the split-rendering frontier).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtx.h"

namespace rtxa {

constexpr int kAnimThreads = 512;                // one workgroup per mesh
constexpr int kAnimWaves = kAnimThreads / 64;
constexpr int kMaxAnimMeshes = 8;                // animated meshes per launch
constexpr int kMaxAnimParts = 128;               // frontier entries per mesh (kPartsPerMesh)
constexpr int kLdsBytesPerTri = 50;              // 9 build floats, 2 permutation words, 3 16-bit ranks
constexpr int kLdsTris = 3136;                   // meshes up to this size build from LDS (153 KB + 3.6 KB static)

// A node of the build tree before the reference's numbering (64 B).
struct alignas(16) TmpNode {
    float mn[3], mx[3];          // UpdateNodeBounds
    uint32_t first, count;       // triangle range, in build positions
    int32_t l;                   // left child's temp id (right = l + 1); -1: leaf
    uint32_t depth;
    uint32_t splits;             // split nodes in the subtree, itself included
    uint32_t rank;               // DFS preorder rank among the split nodes
    uint32_t ref;                // index in the reference's node array
    uint32_t pad[3];
};

struct MeshDev {
    const float4* pos;           // object-space positions (never permuted), V
    float4* tpos;                // transformedPositions, V
    int4* idx[2];                // index triples in the order the last build left them (state), T
    float4* nrm[2];              // object-space normals in that order (state), T
    float4* tnrm;                // transformedNormals in the input order, T
    float4* tnrm_out;            // transformedNormals in the built order, T
    // Build arrays by triangle id (input order) and the two permutation buffers; used in
    // place of the workgroup's LDS copy when the mesh is too large for it (kLdsTris)
    float* soa;                  // 9 T floats: centroid x, y, z, box lo x, y, z, box hi x, y, z
    uint32_t* perm[2];           // build position -> triangle id, T each
    uint32_t* lb;                // partition scratch: left-stream wrong-side positions by rank, T
    uint32_t* rs;                // right-stream ones by rank, T
    uint32_t* rk;                // rank of each position, T
    TmpNode* tmp;                // 2T
    uint32_t* lvl[8];            // node lists per size class (rtx_anim.hip) x current / next level, T each
    rtx_bvh_node* ref;           // the reference's node array (3T entries, persistent)
    uint32_t* status;            // {error bits, deepest level, nodesUsed, frontier parts}
    uint32_t V, T;
    uint32_t mat_bits;           // material index (the triangle record's 4th float4)
    uint32_t mesh;               // mesh index in the scene
    uint32_t tri0;               // first triangle record of the mesh in the scene image
    uint32_t root;               // root node slot (odd) in the scene image
    uint32_t part0, part_cap;    // frontier entries of the mesh in the scene image
};

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
    uint32_t lds_bytes;          // dynamic LDS per workgroup (meshes that fit build from it)
    // A rebuilt tree this many levels deep or deeper would overflow the render kernel's
    // kStackDepth-entry DFS stack: the build then disables the mesh in the image (node count
    // 0, no frontier parts) and reports kErrDepth.  rtxd::kStackDepth; lower only in tests.
    uint32_t depth_limit;
};

enum : uint32_t { kErrNaN = 1u, kErrDepth = 2u };

hipError_t launch_build(const Launch& L, hipStream_t stream);

}  // namespace rtxa
