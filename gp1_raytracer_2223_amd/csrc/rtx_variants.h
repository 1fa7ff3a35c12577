// rtx_variants.h — every compile-time switch of the render kernel and the device Update
// build, in one place.
//
// The product library (build.py) is built with the defaults below plus -DRTX_MIN_WAVES_PER_EU=6.
// The other values exist only for the variant builds of tools/build_variant.py (output under
// gp1_raytracer_2223_amd/lib/exp/, never loaded by the tests, smoke() or bench.py unless
// RTX_HIP_LIB names one): diagnostics that read the kernel from the inside, and ablations that
// time it with one part removed.  Runtime choices (split launches, cull, octant copies, tile
// order) are environment variables read by rtx_create, not switches here;
// the two layout constants RTX_BLOCK_THREADS and RTX_OCT_MAX_BYTES sit in rtx_kernels.h with the
// types they size.
//
// Experiments that lost their A/B were deleted from the kernel rather than kept behind a
// switch; their records stay under profiles/ (profiles/r01/ablate_history.md, profiles/r03/
// ab_*.txt): the plane-skip of primary rays, the touch prefetch of child records, XCD bands
// and XCD runs, the early sphere-loop exit, the unfused triangle test, the non-asm child select;
// round 4: the 128-ray pair kernel and the culled walks' prefetch touches (profiles/r04/); round 5:
// the split grid with the part fastest, a per-group rotation of the XCD dealing and wave priority
// for the heaviest unsplit tiles (profiles/r05/).
#ifndef RTX_VARIANTS_H
#define RTX_VARIANTS_H

// ---- occupancy targets (tuning; product values) ------------------------------------------
// generic kernel: waves per SIMD asked of __launch_bounds__ (build.py passes 6)
#ifndef RTX_MIN_WAVES_PER_EU
#define RTX_MIN_WAVES_PER_EU 1
#endif
// specialised variants with a constant mesh count / the other specialised variants
// (measurements in the comment above rtx_render_kernel)
#ifndef RTX_SPEC_WAVES
#define RTX_SPEC_WAVES 8
#endif
#ifndef RTX_SPEC_WAVES_PARTIAL
#define RTX_SPEC_WAVES_PARTIAL 7
#endif

// ---- formulation choices (product values; the other value is the measured alternative) ----
// shadow-ray walks with cull records visit the child most lanes enter first (1) or left first (0)
#ifndef RTX_CULL_ORDER_ANY
#define RTX_CULL_ORDER_ANY 1
#endif
// split any-hit (PHASE 2): another part's occlusion bit is polled after every leaf, read before the
// leaf's triangle tests so its L2 round trip overlaps them (2, product), after them (1), or never
// (0; the wave then ends only on its own hits).  profiles/r04/ab_occ_poll.txt: 2 is 1-4 % faster
// than 1 on Synthetic100k and its shares, W4_Optional and Bunny + 8 lights at s = 8; 0 is slower.
#ifndef RTX_OCC_POLL
#define RTX_OCC_POLL 2
#endif

// split closest hit (PHASE 1): a part walk starts from the minimum key the pixel's other parts
// have merged so far (1, product: read at the coherence point, the next float above its t) or from
// the sphere/plane scratch t (0).  profiles/r05/ab_p1_shared_key.txt: 1 is ~1 % faster on
// Synthetic100k (0.857 -> 0.847 ms), neutral elsewhere; round 4's version (a plain load) measured
// nothing.
#ifndef RTX_P1_SHARED_T
#define RTX_P1_SHARED_T 1
#endif

// ---- diagnostics (never a product build) -------------------------------------------------
// RTX_STAMPS=1: per-wave {start, end, hw id, node-pair steps, triangle steps, lane-work}
// stamps, read back by rtx_debug_stamps / tools/stamps.py.  RTX_STAMPS_LEAN: the stamps
// with the product walk (timeline only; the step counters stay 0).
#ifndef RTX_STAMPS
#define RTX_STAMPS 0
#endif
#if RTX_STAMPS && !defined(RTX_STAMPS_LEAN)
#define RTX_STAMPS_WALK 1
#else
#define RTX_STAMPS_WALK 0
#endif

// ---- timing ablations (the pixels are WRONG when set; never a product build) -------------
// Each removes one part of the frame's work so tools/ablate.py / tools/cull_ab.py can time the
// rest: primary-ray planes, primary-ray meshes, shadow-ray planes, shadow-ray meshes, lights.
#ifndef RTX_ABL_PPLANE
#define RTX_ABL_PPLANE 0
#endif
#ifndef RTX_ABL_PMESH
#define RTX_ABL_PMESH 0
#endif
#ifndef RTX_ABL_SPLANE
#define RTX_ABL_SPLANE 0
#endif
#ifndef RTX_ABL_SMESH
#define RTX_ABL_SMESH 0
#endif
#ifndef RTX_ABL_LIGHTS
#define RTX_ABL_LIGHTS 0
#endif
// split frames: the main launch alone (the heavy tiles' chain not launched) / the chain alone (the
// main launch skipped on the frames that do not measure tile costs)
#ifndef RTX_ABL_CHAIN
#define RTX_ABL_CHAIN 0
#endif
#ifndef RTX_ABL_MAIN
#define RTX_ABL_MAIN 0
#endif

// ---- device Update build (rtx_anim.hip; opt-in, RTX_ANIM_DEVICE / --device-update) --------
// Shape of the build launch (tuning; product values):
#ifndef RTX_ANIM_THREADS
#define RTX_ANIM_THREADS 512      // threads of every build workgroup
#endif
#ifndef RTX_ANIM_WORKERS
#define RTX_ANIM_WORKERS 64       // task workgroups per mesh besides (mesh, 0)
#endif
#ifndef RTX_ANIM_TEAM_ELEMS
#define RTX_ANIM_TEAM_ELEMS 64u   // a team gets another wave only for this many elements per wave (96: +13 us of timeline, profiles/r03/anim_exp_team*)
#endif
#ifndef RTX_ANIM_POLL_SLEEP
#define RTX_ANIM_POLL_SLEEP 8     // s_sleep units (64 clocks) between a waiting worker's polls
#endif
#ifndef RTX_ANIM_PRIV_MULTI
#define RTX_ANIM_PRIV_MULTI 128   // private-bin threshold in 64ths of an element per lane (128 = two elements per lane)
#endif
// Formulation choices (product values; the other value is the measured alternative, both exact,
// A/B records profiles/r03/anim_exp_*.txt):
#ifndef RTX_ANIM_DPP_BCAST
#define RTX_ANIM_DPP_BCAST 1      // wave reductions: DPP row broadcasts (1) or the four row results read back (0)
#endif
#ifndef RTX_ANIM_KEEP_CHILD
#define RTX_ANIM_KEEP_CHILD 1     // a split task goes on with its larger child instead of queueing it
#endif
#ifndef RTX_ANIM_BIN_PASSES
#define RTX_ANIM_BIN_PASSES 1     // register bins: all eight in one pass (1, 512-thread workgroups) or two halves (2)
#endif
#ifndef RTX_ANIM_BINS_TRANSPOSE
#define RTX_ANIM_BINS_TRANSPOSE 1 // register bins reduced in transposed order
#endif
#ifndef RTX_ANIM_SMALL
#define RTX_ANIM_SMALL 1          // one-wave nodes of up to 128 elements by node_small (0: node_process for all)
#endif
#ifndef RTX_ANIM_BINS_ATOMIC
#define RTX_ANIM_BINS_ATOMIC 0    // experiment: LDS atomics into per-wave bin copies for every node
#endif
// Diagnostics (never a product build):
#ifndef RTX_ANIM_STEP_STAMPS
#define RTX_ANIM_STEP_STAMPS 0    // the root node's step times in status[64..72]
#endif

#endif  // RTX_VARIANTS_H
