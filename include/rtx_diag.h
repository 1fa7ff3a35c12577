/*
 * rtx_diag.h — diagnostics of librtx_hip.so beside the product boundary (rtx.h): timing, the
 * instrumented work counters of the SURVEY §8(d) FLOP model, and the internals of the scheduling
 * and pruning machinery (cost-ordered dispatch, split rendering and its tuner, light-major frames,
 * the exact cull, the device Update's phase stamps).  None of these has a counterpart in the
 * reference's Renderer (source/Renderer.h:17-61); the benchmark (bench.py), the tools and the tests
 * use them.  Same conventions as rtx.h: RTX_OK or a negative RTX_E_* code, nothing throws.
 */
#ifndef RTX_DIAG_H_
#define RTX_DIAG_H_

#include "rtx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Time `iters` back-to-back launches of the render kernel(s) with HIP events recorded
 * on the context stream; writes the mean per-frame device time in ms. */
int rtx_time_frames(rtx_ctx* ctx, const rtx_camera* cam, const rtx_render_params* params,
                    int iters, float* mean_ms);
int rtx_time_views(rtx_ctx* ctx, const rtx_camera* cams, int n_views, const rtx_render_params* params,
                   int iters, float* mean_ms);
/* Bytes of HBM the uploaded scene image occupies. */
int rtx_scene_bytes(const rtx_ctx* ctx, uint64_t* bytes);
/* Diagnostics: copy the context's current scene image (DESIGN.md §2 layout) after its queued
 * work; `bytes` gets the image size (out may be NULL to query it). */
int rtx_scene_image(rtx_ctx* ctx, void* out, size_t capacity, size_t* bytes);
/* Instrumented render: the same traversal with per-ray work counters (12 x uint64, in
 * the order pixels, sphere, plane, slab, tri, hit, shadow, occluded, shade_base,
 * shade_lambert, shade_phong, shade_ct — the SURVEY §8(d) FLOP model).  Not timed. */
int rtx_count_work(rtx_ctx* ctx, const rtx_camera* cam, const rtx_render_params* params,
                   uint64_t* counts12);
/* Same, plus diagnostics appended after the 12 model counters: [12] node-pair tests and
 * [13] triangle tests executed per WAVE (packet work, one count per wave per step). */
int rtx_count_work_ex(rtx_ctx* ctx, const rtx_camera* cam, const rtx_render_params* params,
                      uint64_t* counts, int n_counts);
/* The same counters for the walk the product executes when the scene has exact-cull records
 * (otherwise identical to rtx_count_work_ex): slab [3] and triangle [4] tests the
 * culled, ordered walk performs per lane (a lane in a node's mask is tested against both
 * children), [12]/[13] per-wave steps, and [14] the exact-cull box tests.  One-piece frame (the
 * split launches' extra path tests not included).  Not timed. */
int rtx_count_work_culled(rtx_ctx* ctx, const rtx_camera* cam, const rtx_render_params* params,
                          uint64_t* counts, int n_counts);
/* Split rendering of heavy tiles (no reference counterpart: a scheduling detail of this
 * path).  Tiles whose measured cost exceeds their share of the frame are re-rendered with
 * their BVH traversals cut into `parts` subtree pieces run by separate workgroups; the
 * pixels are identical either way.  Reports the heavy-tile count the next frame will use
 * and the frontier size of the uploaded scene (0 = the scene is rendered unsplit).
 * Environment: RTX_SPLIT=0 disables, RTX_SPLIT=force splits every tile (tests). */
int rtx_split_info(rtx_ctx* ctx, uint32_t* heavy_tiles, uint32_t* parts);
/* Light-major frames (no reference counterpart: a decomposition of the frame's work that never
 * changes a pixel; opt-in, measured slower than one piece): one wave per tile for the
 * primary hits, persistent waves over the (tile, light) shadow rays, one wave per tile shading every
 * light in the reference's order.  Reports whether the last prepared frame was light-major and the
 * largest launch (wave tiles) that is: 0 never (the default), 0xffffffff always (RTX_LIGHT_MAJOR=1),
 * else the threshold of RTX_LIGHT_MAJOR=auto (RTX_LIGHT_MAJOR_TILES). */
int rtx_light_major_info(rtx_ctx* ctx, uint32_t* last_frame, uint32_t* max_tiles);
/* The split threshold's tuner: the current factor (a tile is split when its cost
 * exceeds factor x its share of the frame), the last timed frame's main kernel and split chain
 * (ms, from the fork), and the tuner's state (0 tuning, 1 converged, 2 off: RTX_SPLIT_TUNE=0 or a
 * fixed RTX_SPLIT_FACTOR).  Re-tuned for every new launch shape. */
int rtx_split_tune_info(rtx_ctx* ctx, float* factor, float* main_ms, float* chain_ms, uint32_t* done);
/* Frames in flight: while another context's frame is in flight on the device, a frame
 * whose tiles would split renders one piece when its heaviest tile's serialized one-piece time is
 * below crit_threshold x the split frame's serialized span (the split tuner's best; RTX_INFLIGHT_CRIT,
 * 0: always split as serialized frames do), or when split frames in flight, timed on this context's
 * stream, were found not to overlap.  Reports whether the last prepared frame saw another context's
 * frame in flight, whether it rendered one piece for that, the ratio (heaviest tile / split span; 0
 * until both are measured), the threshold and the split frames' interval in flight (ms, 0 before). */
int rtx_inflight_info(rtx_ctx* ctx, uint32_t* concurrent, uint32_t* onepiece, float* crit, float* crit_threshold,
                      float* split_interval_ms);
/* Exact cull (no reference counterpart: a pruning of the reference's own BVH walk that never
 * changes a pixel).  Reports whether the uploaded scene renders with it (on for
 * host uploads whose reference boxes are inflated enough to pay, see upload_scene) and how
 * many times a camera's records were (re)built.  Environment: RTX_NO_CULL=1 disables;
 * RTX_CULL_MIN_SA, RTX_CULL_RATIO tune the enabling test and the per-node flag (tests). */
int rtx_cull_info(rtx_ctx* ctx, uint32_t* enabled, uint64_t* camera_updates);
/* Diagnostics of the exact cull (tests): waits for the context stream, then copies the current
 * image's records of record copy `anchor` (view v < 8: its camera; 8 + l: light l) — n_slots x
 * 8 floats, {c, E.x}, {E.y, E.z, dt, flag bits} — and their inputs: per slot the triangle range
 * [first, end) (2 x u32), node copy 0 (8 floats per slot), the triangle records (16 floats
 * each: {v0, n.x}, {E1, n.y}, {E2, n.z}, {mat}), and the anchor the copy was last built for
 * (x, y, z, w = 0 camera / tmax bound of a light, bt).  Null pointers are skipped; sizes via
 * *n_slots / *n_tris.  RTX_E_INVALID when the scene has no records. */
int rtx_cull_dump(rtx_ctx* ctx, uint32_t anchor, uint32_t* n_slots, uint32_t* n_tris, float* anchor_p,
                  float* records, uint32_t* ranges, float* nodes, float* tris);
/* Diagnostics of the cost-ordered dispatch (tests): after a measured frame, the dispatch
 * permutation of the first n tiles' slots (`order`) and the one-piece tile costs it was
 * sorted by (`cost`).  *n_tiles = tiles of the current schedule (0 = none measured yet;
 * then nothing is copied). */
int rtx_schedule_state(rtx_ctx* ctx, uint32_t* order, uint32_t* cost, uint32_t n, uint32_t* n_tiles);

/* Diagnostics: 128 status words of the last update of registered mesh i (0-3 as above,
 * 4-6 subtrees / task-split ids / nodes split as tasks, 8-27 phase stamps of the device build
 * at 100 MHz; csrc/rtx_anim.h). */
int rtx_anim_stamps(rtx_anim* anim, uint32_t i, uint32_t out[128]);

#ifdef __cplusplus
}
#endif
#endif /* RTX_DIAG_H_ */
