/*
 * rtx_host.h — C-ABI of the host scene library (librtx_host.so, C++): the Scene layer
 * that sits ABOVE the render boundary of rtx.h.  It mirrors the reference's
 * Scene::Initialize / Scene::Update / Scene::GetCamera (source/Scene.h:30-43) for the
 * scene catalogue of source/Scene.cpp:163-474 and flattens a scene into the rtx_scene
 * view that rtx_upload_scene() consumes.
 */
#ifndef RTX_HOST_H_
#define RTX_HOST_H_

#include "rtx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rtx_host_scene rtx_host_scene;

/* Build a catalogue scene (W1, W2, W3, W3_Test, W4_Test, W4_Reference, W4_Bunny,
 * W4_Optional, Synthetic100k, Bunny8Lights) — Scene_*::Initialize() — or, for a name
 * "file:<path>", the scene described by a scene file (text, one directive per line:
 * camera / material / sphere / plane / mesh / light; grammar in csrc/host/scene.cpp and
 * DESIGN.md, examples in scenes/ as *.rtxscene). Mesh assets are looked up in `asset_dir`
 * as <stem>.rtxmesh, then <stem>.obj.  On failure returns an error code and, if
 * err/err_len are given, the reason (for scene files with the line number). */
int rtx_host_scene_create(const char* name, const char* asset_dir, rtx_host_scene** out, char* err,
                          size_t err_len);
void rtx_host_scene_destroy(rtx_host_scene* s);
/* Scene_W4_*::Update minus the SDL camera input: yaw = (cos t + 1)/2 * 2pi on every
 * animated mesh, transforms + BVH rebuilt (source/Scene.cpp:391-400, 431-437, 468-474). */
int rtx_host_scene_update(rtx_host_scene* s, float total_time);
/* Copy the state Update(t) leaves in `src` (meshes' transforms, world positions and normals, the
 * BVH-permuted indices and normals, the node array; the camera) into `dst`, a host scene created
 * with the same name.  The reference's BuildBVH permutes the triangles in place
 * (DataTypes.h:335-363), so a scene's state depends on its whole Update history: a pipelined
 * frame loop updates ONE scene serially and uploads snapshots of it.  RTX_E_INVALID when the
 * scenes differ. */
int rtx_host_scene_copy_state(rtx_host_scene* dst, const rtx_host_scene* src);
/* Flat view (pointers into the scene; valid until the next update/destroy) and the
 * camera after CalculateCameraToWorld(). */
int rtx_host_scene_view(rtx_host_scene* s, rtx_scene* out_scene, rtx_camera* out_camera);
/* 1 if Update(t) moves geometry (the W4 scenes rotate their meshes, Scene.cpp:391-400,
 * 431-437) and the scene must be re-uploaded after it, 0 if not, < 0 on error. */
int rtx_host_scene_animated(const rtx_host_scene* s);
/* Camera controls (Camera.h): origin, fov in degrees (SetCameraFOV), pitch/yaw in
 * radians (CalculateForwardVector). */
int rtx_host_camera_set(rtx_host_scene* s, const float origin[3], float fov_degrees, float pitch, float yaw);

/* Device-side Update (rtx_anim_*, rtx.h).  The meshes Update(t) turns (count returned,
 * ids written up to `capacity`), one mesh's object-space state, and the final transforms
 * Update(t) applies: sets each turning mesh's rotation as Update(t) does and writes
 * scale * rotation * translation (16 floats per turning mesh, Matrix data[4] row-major, at
 * most `capacity` meshes written; the count of turning meshes is returned) WITHOUT rebuilding
 * — the host scene's own geometry is then stale until the next rtx_host_scene_update. */
int rtx_host_scene_spinning(rtx_host_scene* s, int32_t* mesh_ids, uint32_t capacity);
int rtx_host_scene_mesh_source(rtx_host_scene* s, uint32_t mesh, rtx_mesh_source* out);
int rtx_host_scene_transforms(rtx_host_scene* s, float total_time, float* out, uint32_t capacity);

/* Utils::ParseOBJ (source/Utils.h:377-451).  Fills caller buffers when non-NULL and
 * always reports the counts; returns RTX_OK or RTX_E_INVALID (unreadable file). */
int rtx_host_parse_obj(const char* path, float* positions, uint32_t* n_positions, float* normals,
                       int32_t* indices, uint32_t* n_indices, uint32_t capacity_positions,
                       uint32_t capacity_indices);
/* Convert an .obj into the pre-tokenised .rtxmesh asset format. */
int rtx_host_obj_to_asset(const char* obj_path, const char* asset_path);

#ifdef __cplusplus
}
#endif
#endif /* RTX_HOST_H_ */
