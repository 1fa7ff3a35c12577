/*
 * rtx.h — C-ABI drop-in boundary for the per-pixel render loop of
 * JonathanMenschaert/GP1_Raytracer_2223 (`Renderer::Render` → `RenderPixel`).
 *
 * The reference has no plugin API; its seam is `Renderer::Render(Scene*) const`
 * (source/Renderer.h:28, called once per frame from source/main.cpp:91) with the
 * per-pixel body `Renderer::RenderPixel` (source/Renderer.cpp:100-182).  This header
 * replaces that seam with plain C: the caller flattens its Scene into `rtx_scene`
 * (plain pointers + sizes, no C++ or torch types), uploads it once to HBM with
 * `rtx_upload_scene`, then calls `rtx_render` once per frame.
 *
 * Scene records are laid out byte-for-byte like the reference's own value types so a
 * reference Scene can hand its std::vector storage over without repacking:
 *   rtx_sphere   == dae::Sphere   (source/DataTypes.h:13-19,  20 B)
 *   rtx_plane    == dae::Plane    (source/DataTypes.h:21-27,  28 B)
 *   rtx_bvh_node == dae::BVHNode  (source/DataTypes.h:43-54,  36 B)
 *   rtx_light    == dae::Light    (source/DataTypes.h:528-536, 44 B)
 * Materials are polymorphic in the reference (source/Material.h) and are flattened
 * into the tagged `rtx_material`.
 *
 * Error convention: every entry point returns RTX_OK (0) or a negative RTX_E_* code and
 * never throws across the ABI; `rtx_last_error` gives a human-readable reason.  (The
 * reference itself has no error channel: Renderer::Render returns void.)
 *
 * Threading: like Renderer::Render (called only from the main thread), one caller
 * thread per rtx_ctx.  Different contexts (one per GPU) may be driven concurrently.
 *
 * This header is the product boundary: contexts, scene upload, rendering, the host gather, one frame
 * over several GPUs (rtx_group_*) and the device-side Update (rtx_anim_*).  Timing, work counters
 * and the scheduler's / exact cull's internals are in rtx_diag.h; the environment knobs the library
 * reads are listed in INTEGRATION.md (none of them changes a pixel).
 */
#ifndef RTX_H_
#define RTX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTX_ABI_VERSION 2

enum {
    RTX_OK = 0,
    RTX_E_INVALID = -1,   /* bad argument / malformed scene                          */
    RTX_E_DEVICE = -2,    /* HIP runtime error (message in rtx_last_error)           */
    RTX_E_NOMEM = -3,     /* host or device allocation failed                       */
    RTX_E_STATE = -4,     /* e.g. rtx_render before rtx_upload_scene                 */
    RTX_E_UNSUPPORTED = -5
};

/* dae::TriangleCullMode (source/DataTypes.h:29-34), same enumerator order */
enum { RTX_CULL_FRONT = 0, RTX_CULL_BACK = 1, RTX_CULL_NONE = 2 };
/* dae::LightType (source/DataTypes.h:522-526) */
enum { RTX_LIGHT_POINT = 0, RTX_LIGHT_DIRECTIONAL = 1 };
/* Renderer::LightingMode (source/Renderer.h:40-48), same enumerator order */
enum {
    RTX_MODE_OBSERVED_AREA = 0,
    RTX_MODE_RADIANCE = 1,
    RTX_MODE_BRDF = 2,
    RTX_MODE_COMBINED = 3,
    RTX_MODE_COUNT = 4
};
/* Material subclasses of source/Material.h */
enum {
    RTX_MAT_SOLID_COLOR = 0,   /* Material_SolidColor    Material.h:34-48   */
    RTX_MAT_LAMBERT = 1,       /* Material_Lambert       Material.h:54-68   */
    RTX_MAT_LAMBERT_PHONG = 2, /* Material_LambertPhong  Material.h:74-94   */
    RTX_MAT_COOK_TORRANCE = 3  /* Material_CookTorrence  Material.h:99-129  */
};

typedef struct rtx_sphere {
    float origin[3];
    float radius;
    uint8_t material;
    uint8_t _pad[3];
} rtx_sphere;

typedef struct rtx_plane {
    float origin[3];
    float normal[3];
    uint8_t material;
    uint8_t _pad[3];
} rtx_plane;

/* One node of the reference's binned-SAH BVH.  `idx_count` and `first_idx` count
 * INDICES (3 per triangle), leaf iff idx_count > 0, right child = left_node + 1. */
typedef struct rtx_bvh_node {
    float min[3];
    float max[3];
    uint32_t first_idx;
    uint32_t idx_count;
    uint32_t left_node;
} rtx_bvh_node;

/* A TriangleMesh after UpdateTransforms()/BuildBVH() (source/DataTypes.h:109-236):
 * world-space positions, the BVH-permuted index array, per-triangle world normals
 * (transformedNormals, indexed by index/3) and the node array (nodesUsed entries). */
typedef struct rtx_mesh {
    const float* positions;   /* 3 * n_positions floats (transformedPositions) */
    uint32_t n_positions;
    const int32_t* indices;   /* n_indices = 3 * triangles                    */
    uint32_t n_indices;
    const float* normals;     /* 3 * (n_indices / 3) floats (transformedNormals) */
    const rtx_bvh_node* nodes;
    uint32_t n_nodes;
    int32_t cull_mode;        /* RTX_CULL_*                                   */
    uint8_t material;
    uint8_t _pad[3];
} rtx_mesh;

typedef struct rtx_light {
    float origin[3];
    float direction[3];
    float color[3];
    float intensity;
    int32_t type;             /* RTX_LIGHT_* */
} rtx_light;

/* Flattened Material.  Field use per kind:
 *   SOLID_COLOR   : color
 *   LAMBERT       : color (diffuse colour), kd
 *   LAMBERT_PHONG : color, kd, ks, exponent
 *   COOK_TORRANCE : color (albedo), metalness, roughness                         */
typedef struct rtx_material {
    int32_t kind;
    float color[3];
    float kd;
    float ks;
    float exponent;
    float metalness;
    float roughness;
} rtx_material;

typedef struct rtx_scene {
    const rtx_sphere* spheres;     uint32_t n_spheres;
    const rtx_plane* planes;       uint32_t n_planes;
    const rtx_mesh* meshes;        uint32_t n_meshes;
    const rtx_light* lights;       uint32_t n_lights;
    const rtx_material* materials; uint32_t n_materials;
} rtx_scene;

/* Camera after Camera::CalculateCameraToWorld() (source/Camera.h:43-53): the rows of
 * cameraToWorld, the ray origin and fov = tanf(fovAngle*TO_RADIANS/2) (Camera.h:55-59). */
typedef struct rtx_camera {
    float origin[3];
    float right[3];
    float up[3];
    float forward[3];
    float fov;
} rtx_camera;

/* SDL_MapRGB for a palette-less 8-bit-per-channel surface:
 * pixel = r<<rshift | g<<gshift | b<<bshift | amask.  XRGB8888 = {16, 8, 0, 0}. */
typedef struct rtx_pixel_format {
    uint32_t rshift, gshift, bshift, amask;
} rtx_pixel_format;

/* Per-frame parameters (the Renderer's state: m_Width/m_Height, m_CurrentLightingMode,
 * m_ShadowsEnabled — source/Renderer.h:40-61) plus the image partition for multi-GPU:
 * rows are grouped in stripes of `stripe_rows`; this call renders stripe s iff
 * s % stripe_step == stripe_first.  stripe_rows = 0 means "the whole image". */
typedef struct rtx_render_params {
    uint32_t width, height;
    int32_t lighting_mode;        /* RTX_MODE_* (default RTX_MODE_COMBINED) */
    int32_t shadows_enabled;      /* 0/1 (default 1)                         */
    rtx_pixel_format format;
    uint32_t stripe_rows;
    uint32_t stripe_first;
    uint32_t stripe_step;
} rtx_render_params;

typedef struct rtx_ctx rtx_ctx;

/* ---- device context (librtx_hip.so) ------------------------------------------- */
int rtx_abi_version(void);
/* Bind a context to HIP device `device_id` (one context per GPU; one process per GPU
 * is the supported multi-GPU model).  Creates its own non-blocking stream. */
int rtx_create(rtx_ctx** out, int device_id);
void rtx_destroy(rtx_ctx* ctx);
/* Reason for the last error on `ctx`; with ctx == NULL, why the calling thread's last
 * rtx_create failed. */
const char* rtx_last_error(const rtx_ctx* ctx);
/* Copy the caller-owned scene into HBM (device layout of DESIGN.md §3).  The caller
 * may free its arrays afterwards.  Re-call after an animated Scene::Update. */
int rtx_upload_scene(rtx_ctx* ctx, const rtx_scene* scene);
/* Blocking frame render, like Renderer::Render: renders the rows selected by
 * `params` and writes them into the caller's host buffers (row-major, pitch = width
 * pixels; rows this call does not own are left untouched).  out_rgb (3 floats per
 * pixel, post-MaxToOne colour) may be NULL. */
int rtx_render(rtx_ctx* ctx, const rtx_camera* cam, const rtx_render_params* params,
               uint32_t* out_pixels, float* out_rgb);
/* Asynchronous variant for device-resident pipelines: renders into the context's HBM
 * frame buffer on the context stream and returns immediately. */
int rtx_render_async(rtx_ctx* ctx, const rtx_camera* cam, const rtx_render_params* params,
                     int want_rgb);
/* Multi-view batch (one launch): renders n_views (1..8) cameras of the same scene into
 * consecutive frame buffers (view v at offset v*width*height).  With stripes, view v
 * owns the stripes s with s % stripe_step == (stripe_first - v) mod stripe_step, so N
 * ranks with stripe_first = rank and stripe_step = N cover every view exactly once with
 * the same number of rows each (the weak-scaling partition of bench.py). */
int rtx_render_views_async(rtx_ctx* ctx, const rtx_camera* cams, int n_views,
                           const rtx_render_params* params, int want_rgb);
int rtx_synchronize(rtx_ctx* ctx);
/* Copy the context's frame buffer (rows owned by the last render) to host memory. */
int rtx_download(rtx_ctx* ctx, uint32_t* out_pixels, float* out_rgb);
/* Host gather of one partition: queue, on the context stream, the D2H copy
 * of the rows the last render owns into the caller's FULL-FRAME host buffers (row-major,
 * pitch = width; one hipMemcpy2DAsync per view and plane for a striped render) and
 * return.  Rows the context does not own are never written, so several contexts (GPUs,
 * or processes sharing one mapping) can gather disjoint stripes into one frame.  Truly
 * asynchronous only for page-locked memory (rtx_host_register); complete after
 * rtx_synchronize. */
int rtx_gather_async(rtx_ctx* ctx, uint32_t* out_pixels, float* out_rgb);
/* Page-lock caller memory (e.g. a frame shared between the ranks' processes) for every
 * device of the process (hipHostRegister, portable), and undo it. */
int rtx_host_register(rtx_ctx* ctx, void* ptr, size_t bytes);
int rtx_host_unregister(rtx_ctx* ctx, void* ptr);
/* Device pointers of the HBM frame buffer (width*height uint32 / 3*width*height f32).  The
 * frames queued so far are complete in it after rtx_synchronize (a repeated frame may leave
 * its split launches running after rtx_render_async returns, on a stream of its own). */
int rtx_device_buffers(rtx_ctx* ctx, void** d_pixels, void** d_rgb);
/* ---- one frame over several GPUs from one process ------------------
 * The reference's Renderer::Render covers the frame with parallel_for
 * (source/Renderer.cpp:79-85); a group covers it with G render contexts instead.  Rows are
 * dealt in `stripe_rows`-row stripes round robin (member i owns stripe s iff s % G == i);
 * each member has its own host thread and stream, renders its stripes and gathers them
 * straight into the caller's host frame (rtx_gather_async).  rtx_group_render blocks until
 * the whole frame is in out_pixels / out_rgb; the result is bit-identical to one
 * context's rtx_render.  Device ids may repeat (several contexts on one GPU). */
#define RTX_GROUP_MAX 64
typedef struct rtx_group rtx_group;
int rtx_group_create(rtx_group** out, const int* device_ids, int n);
void rtx_group_destroy(rtx_group* group);
/* Reason for the group's last error; with NULL, why this thread's last create failed. */
const char* rtx_group_last_error(const rtx_group* group);
int rtx_group_size(const rtx_group* group);
/* Member i's context (owned by the group), e.g. for rtx_time_frames on its stripes. */
rtx_ctx* rtx_group_context(rtx_group* group, int i);
int rtx_group_upload_scene(rtx_group* group, const rtx_scene* scene);
/* params: stripe_rows = stripe height (multiple of 16; 0 = 16); stripe_step must be 0/1
 * (the group assigns the stripes).  out_pixels: width*height uint32; out_rgb may be NULL. */
int rtx_group_render(rtx_group* group, const rtx_camera* cam, const rtx_render_params* params,
                     uint32_t* out_pixels, float* out_rgb);

/* ---- animated meshes: Scene::Update on the device -------------------
 * Replaces, per animated frame, the host's TriangleMesh::UpdateTransforms + BuildBVH
 * (source/DataTypes.h:210-236, 294-483, called from Scene_W4_*::Update, Scene.cpp:391-400,
 * 431-437, 468-474) followed by rtx_upload_scene: the transform, the reference's binned-SAH
 * rebuild (bit-identical node array and triangle permutation, which the next Update starts
 * from) and the scene image are produced in HBM by one workgroup per mesh. */
/* The object-space state UpdateTransforms starts from: positions (never permuted), the
 * per-triangle normals and the index array in the order the last BuildBVH left them. */
typedef struct rtx_mesh_source {
    const float* positions;   /* 3 * n_positions floats, object space                   */
    uint32_t n_positions;
    const float* normals;     /* 3 per triangle, object space (TriangleMesh::normals)    */
    const int32_t* indices;   /* n_indices = 3 * triangles                               */
    uint32_t n_indices;
} rtx_mesh_source;
typedef struct rtx_anim rtx_anim;
/* Register meshes mesh_ids[0..n) of `scene` (its current flattened state, what
 * rtx_upload_scene takes) as device-animated, with their object-space state src[0..n), and
 * upload the scene to `ctx` with rebuild-sized regions reserved for them.  n <= 32; the
 * meshes must be NaN-free, and the scene must render with the default-depth kernel (BVHs under
 * 64 levels; a rebuilt tree that deep is disabled in the image and reported, see
 * rtx_anim_status). */
int rtx_anim_create(rtx_anim** out, rtx_ctx* ctx, const rtx_scene* scene, const int32_t* mesh_ids,
                    const rtx_mesh_source* src, uint32_t n);
void rtx_anim_destroy(rtx_anim* anim);
/* Reason for the anim's last error; with NULL, why this thread's last create failed. */
const char* rtx_anim_last_error(const rtx_anim* anim);
/* One Update: registered mesh i gets finalTransform = transforms[16 i .. 16 i + 15] (the
 * reference's Matrix, data[0..3] row-major).  Queued on ctx's stream after the previous
 * update (whichever context on the anim's device ran it); frames rendered on ctx afterwards
 * see the new geometry.  Build errors are reported by rtx_anim_status. */
int rtx_anim_update(rtx_anim* anim, rtx_ctx* ctx, const float* transforms);
/* Waits for the last update.  status = {error bits (1: NaN vertex, 2: BVH too deep for the
 * render stack, 4: a build workgroup timed out waiting for a queue task; the frames
 * rendered from it are invalid), deepest level, nodesUsed, frontier parts}; returns
 * RTX_E_UNSUPPORTED when error bits are set. */
int rtx_anim_status(rtx_anim* anim, uint32_t i, uint32_t status[4]);
/* Waits for the last update and copies registered mesh i's state in the reference's own
 * form: transformedPositions (3V), indices (3T), normals (object space, 3T),
 * transformedNormals (3T), the node array pBVHNodes (3T entries).  NULL skips a part. */
int rtx_anim_download(rtx_anim* anim, uint32_t i, float* positions, int32_t* indices, float* normals,
                      float* transformed_normals, rtx_bvh_node* nodes);

#ifdef __cplusplus
}
#endif
#endif /* RTX_H_ */
