// scene.h — the host scene model that feeds the render path (C++, ours).
//
// Mirrors the reference's Scene layer (source/Scene.h, source/DataTypes.h,
// source/Camera.h, Utils::ParseOBJ in source/Utils.h:377-451) closely enough that the
// world-space triangles, the BVH node array and the BVH-permuted triangle order it
// produces are bit-identical to the reference's (checked against oracle goldens in
// tests/test_host_scene.py).  It owns plain std::vectors whose storage the C-ABI view
// (rtx_scene, include/rtx.h) points into.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "rtx.h"
#include "rtx_math.h"

namespace rtx {

// dae::BVHNode (DataTypes.h:43-54) — same 36-byte layout as rtx_bvh_node.
struct BVHNode {
    Vec3 minAABB{kMaxVector};
    Vec3 maxAABB{kMinVector};
    uint32_t firstIdx{0};
    uint32_t idxCount{0};
    uint32_t leftNode{0};
    bool IsLeaf() const { return idxCount > 0; }
};
static_assert(sizeof(BVHNode) == sizeof(rtx_bvh_node), "BVHNode layout");

struct AABB {
    Vec3 minAABB{kMaxVector};
    Vec3 maxAABB{kMinVector};
    void Grow(const Vec3& p) { minAABB = Vec3::Min(minAABB, p); maxAABB = Vec3::Max(maxAABB, p); }
    void Grow(const AABB& b) { minAABB = Vec3::Min(minAABB, b.minAABB); maxAABB = Vec3::Max(maxAABB, b.maxAABB); }
    float Area() const {
        const Vec3 e = maxAABB - minAABB;
        return e.x * e.y + e.y * e.z + e.z * e.x;
    }
};

// dae::TriangleMesh (DataTypes.h:109-519): transforms + binned-SAH BVH build.
struct TriangleMesh {
    std::vector<Vec3> positions, normals;
    std::vector<int32_t> indices;
    uint8_t materialIndex{0};
    int32_t cullMode{RTX_CULL_BACK};
    Mat4 rotationTransform, translationTransform, scaleTransform;
    Vec3 minAABB, maxAABB;
    std::vector<BVHNode> nodes;     // sized like `new BVHNode[indices.size()]`
    uint32_t nodesUsed{1};
    std::vector<Vec3> transformedPositions, transformedNormals;

    void Translate(const Vec3& t) { translationTransform = Mat4::Translation(t); }
    void RotateY(float yaw) { rotationTransform = Mat4::RotationY(yaw); }
    void Scale(const Vec3& s) { scaleTransform = Mat4::Scale(s); }
    void AppendTriangle(const Vec3& v0, const Vec3& v1, const Vec3& v2);  // DataTypes.h:158-176 (ignoreTransformUpdate)
    void CalculateNormals();                                              // :178-195
    void AllocateNodes() { nodes.assign(indices.size(), BVHNode{}); }
    void UpdateAABB();                                                    // :238-250
    void UpdateTransforms();                                              // :210-236
    void BuildBVH();                                                      // :294-308

private:
    // Build tree before numbering: the subtrees are built in parallel, then numbered in
    // the reference's allocation order (children pairs in DFS order of the splits).
    struct TmpNode { uint32_t first, count; Vec3 mn, mx; int32_t l, r; };
    std::vector<TmpNode> tmp_;
    uint32_t tmpUsed_{0};   // bumped with __atomic_fetch_add by the build tasks
    void Bounds(TmpNode& n) const;
    void SubdivideTmp(uint32_t t, int depth);
    void Emit(uint32_t t, uint32_t nodeIdx);
    float FindBestSplitPlane(const BVHNode& node, int& axis, float& splitPos) const;
    static float CalculateNodeCost(const BVHNode& node);
    Vec3 Centroid(uint32_t i) const {
        return (transformedPositions[indices[i]] + transformedPositions[indices[i + 1]] +
                transformedPositions[indices[i + 2]]) * 0.3333f;
    }
    // Build-time cache, permuted with the triangles: centroid (the reference recomputes
    // the same expression at every use, DataTypes.h:348,414,435), the 3 vertices, and the
    // triangle's box (bins grow by it: min/max are exact, so only the sign of a zero
    // could depend on the grouping, and no SAH cost can observe that).
    struct TriCache { Vec3 c, v0, v1, v2, lo, hi; };
    std::vector<TriCache> tc_;
    void BuildBVHDirect();

    // Fast builder (the default; RTX_HOST_BVH=direct selects the one above): the same
    // split decisions from SSE passes over a compact (centroid, triangle id) array that the
    // partition permutes in place; the composed permutation is applied to indices, normals
    // and transformedNormals once at the end, and large subtrees run on a thread pool.
    struct alignas(16) PTri { float c[3]; uint32_t id; };
    struct alignas(16) TriBox { float lo[4], hi[4]; };
    std::vector<PTri> pt_;
    std::vector<TriBox> box_;
    std::vector<int32_t> scratchI_;
    std::vector<Vec3> scratchN_, scratchTN_;
    bool BuildBVHFast();
    void BoundsFast(TmpNode& n) const;
    void SubdivideFast(uint32_t t);
    float FindBestSplitFast(const BVHNode& node, int& axis, float& splitPos) const;
};

// dae::Camera (source/Camera.h): the ray-generation state only (Update is input).
struct Camera {
    Vec3 origin{};
    float fovAngle{90.f};
    float fov{};                     // NOTE: 0 until SetCameraFOV (Camera.h:26)
    Vec3 forward{kUnitZ}, up{kUnitY}, right{kUnitX};
    bool forwardChanged{true};
    float totalPitch{0.f}, totalYaw{0.f};
    void SetCameraFOV(float degrees);                                    // Camera.h:55-59
    void CalculateCameraToWorld();                                       // Camera.h:43-53
    void CalculateForwardVector();                                       // Camera.h:61-66
    rtx_camera View() const;
};

// Utils::ParseOBJ (Utils.h:377-451): `v` and the first field of `f`, face normals.
bool ParseOBJ(const std::string& path, std::vector<Vec3>& positions, std::vector<Vec3>& normals,
              std::vector<int32_t>& indices);
// Same result from the pre-tokenised asset format (.rtxmesh: "RTXM", u32 nV, u32 nI,
// f32 positions[3nV], i32 indices[nI]); normals computed exactly as ParseOBJ does.
bool LoadMeshAsset(const std::string& path, std::vector<Vec3>& positions, std::vector<Vec3>& normals,
                   std::vector<int32_t>& indices);
bool SaveMeshAsset(const std::string& path, const std::vector<Vec3>& positions,
                   const std::vector<int32_t>& indices);

// dae::Scene + the scene catalogue of source/Scene.cpp:163-474 and the two synthetic
// configs of SURVEY §8(d).
class Scene {
public:
    explicit Scene(std::string assetDir);
    virtual ~Scene() = default;
    virtual bool Initialize() = 0;
    virtual void Update(float totalTime) { (void)totalTime; }   // animated meshes only
    virtual bool Animated() const { return false; }             // Update moves geometry
    // The meshes Update(t) turns (RotateY(Yaw(t)) then UpdateTransforms), in mesh order, and
    // that yaw (Scene.cpp:394): the device-side Update (rtx_anim_*) applies the same turn.
    virtual std::vector<TriangleMesh*> Spinning() { return {}; }
    static float SpinYaw(float t);
    Camera& GetCamera() { return m_Camera; }
    const std::string& Name() const { return sceneName; }
    const std::string& Error() const { return m_Error; }

    // Flat C-ABI view pointing into this object's storage (valid until next Update).
    rtx_scene View();
    // Copy the state an Update leaves (every mesh's transforms, world arrays, the BVH-permuted
    // indices and normals, the node array) from `o`, a scene of the same kind: a snapshot of one
    // Update history for a pipelined frame loop.  False when the meshes do not match.
    bool CopyStateFrom(const Scene& o);

    std::vector<rtx_sphere> m_Spheres;
    std::vector<rtx_plane> m_Planes;
    std::vector<std::unique_ptr<TriangleMesh>> m_Meshes;
    std::vector<rtx_light> m_Lights;
    std::vector<rtx_material> m_Materials;

protected:
    std::string sceneName;
    std::string m_AssetDir;
    std::string m_Error;
    Camera m_Camera;
    std::vector<rtx_mesh> m_MeshViews;

    uint8_t AddSphere(const Vec3& origin, float radius, uint8_t mat);
    uint8_t AddPlane(const Vec3& origin, const Vec3& normal, uint8_t mat);
    TriangleMesh* AddTriangleMesh(int32_t cullMode, uint8_t mat);
    void AddPointLight(const Vec3& origin, float intensity, const Color& c);
    void AddDirectionalLight(const Vec3& direction, float intensity, const Color& c);
    uint8_t AddMaterial(const rtx_material& m);
    bool LoadMesh(TriangleMesh* m, const std::string& stem);
};

rtx_material SolidColor(const Color& c);
rtx_material Lambert(const Color& c, float kd);
rtx_material LambertPhong(const Color& c, float kd, float ks, float exponent);
rtx_material CookTorrance(const Color& albedo, float metalness, float roughness);

// Names: W1 W2 W3 W3_Test W4_Test W4_Reference W4_Bunny W4_Optional
//        Synthetic100k Bunny8Lights.   nullptr for an unknown name.
std::unique_ptr<Scene> MakeScene(const std::string& name, const std::string& assetDir);

}  // namespace rtx
