/*
 * rt_debug.h — diagnostic exports of librt_amd.so (not part of the drop-in
 * boundary, include/rt.h).
 *
 * The reference has no counterpart: these read back what the acceleration
 * structures cost (bench.py reports them beside the headline number) and
 * self-test the wave primitives the culling relies on.  They never change an
 * image and no product path depends on them; the ABI version of rt.h does not
 * cover them.  Every function returns 0 or a negative RT_E_* code (rt.h).
 */
#ifndef RT_AMD_RT_DEBUG_H
#define RT_AMD_RT_DEBUG_H

#include "rt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Light buffer of the uploaded scene: out[0] built (0/1), out[1] entries,
 * out[2] build ms; then per light j (while 3 + 3j + 2 < n): cells per face
 * edge, uncullable-pair list length, coverage distance dcov. */
int rt_debug_lb_info(rt_ctx*, double* out, int n);

/* Camera buffer of the last build: out[0] current (0/1), out[1] entries,
 * out[2] device ms of the last synchronous build's kernels, out[3] tiles, out[4] inline
 * records (0/1), out[5] host wall ms of the build's enqueue; out[6..9]
 * binning counters: candidate (triangle, tile) pairs tested, lists longer
 * than 256, the longest of them, the entry capacity; out[10] 1 when the
 * candidate pairs passed 2^32 - 1 (no pair tested, every tile flagged to the
 * per-wave path). */
int rt_debug_cb_info(rt_ctx*, double* out, int n);

/* The current camera buffer checked against brute force (every tile with
 * a list against every triangle; synchronous): out[0] tiles whose list is
 * not exactly the triangles passing the camera wave test (or mis-keyed),
 * out[1] passing pairs, out[2] tiles with a list. */
int rt_debug_cb_verify(rt_ctx*, unsigned long long* out3);

/* The last rt_upload_scene's host wall time by part (ms): out[0] records +
 * device copies, out[1] cone / cluster prepasses, out[2] light buffer,
 * out[3] total, out[4..8] the light-buffer build's phases, out[9] (n >= 10) light
 * 0's first light buffer's resolution R (6 R^2 cells; 0 without one). */
int rt_debug_upload_info(rt_ctx*, double* out, int n);

/* The builds' device prefix sum on host counts (n >= 1), in place like its
 * callers: out (n + 1 words) = the exclusive prefixes then the total, both
 * mod 2^32; *total = the 64-bit total. */
int rt_debug_scan(int device, const unsigned* in, unsigned n, unsigned* out, unsigned long long* total);

/* ABI 7: the bounce-ray BVH of the uploaded scene (rt_bvh.h): out[0] built
 * (0/1), out[1] inner nodes, out[2] leaves, out[3] depth (deepest leaf's
 * inner-node path), out[4] host build ms. */
int rt_debug_bvh_info(rt_ctx*, double* out, int n);

/* The last wavefront frame's queue counts (round 6; synchronous): per level
 * L = 0 .. 8, out[3 L] its rays (L >= 1), out[3 L + 1] its parents (nodes
 * that spawned children), out[3 L + 2] its walks finished by the straggler
 * launch.  RT_E_STATE before any wavefront frame. */
int rt_debug_wf_counts(rt_ctx*, unsigned* out, int n);

/* The host BVH build alone, no device (round 6): n triangles of 12 floats
 * (p0, e1, e2, normal); out3 = {depth, inner nodes, leaves}.  The depth is
 * at most 24 (the walk's stack) for every input; RT_E_UNSUPPORTED above
 * 4 x 2^24 triangles (bounce rays then test every triangle). */
int rt_debug_bvh_build(const float* tri12, long long n, int* out3);

/* Bounce-ray closest hits of n arbitrary rays (rays: O.xyz D.xyz per ray),
 * each through the BVH and through every triangle (planes and quadrics
 * too, both ways; synchronous): out_idx / out_t (2 per ray) = [BVH, brute
 * force] winners (file index or -1, t); tally2 = the BVH walk's triangle
 * tests and inner nodes visited, summed.  RT_E_STATE without a BVH. */
int rt_debug_bvh_rays(rt_ctx*, const float* rays, int n, int* out_idx, float* out_t, unsigned long long* tally2);

/* The same rays walked by the wavefront's straggler path — the budgeted
 * serial walk stopped after one step, then the wave-cooperative walk (one
 * wave per ray, a shared LDS stack) — winners into out_idx / out_t (one per
 * ray); compare with rt_debug_bvh_rays' brute force.  RT_E_STATE without a
 * BVH. */
int rt_debug_bvh_rays_wave(rt_ctx*, const float* rays, int n, int* out_idx, float* out_t);

/* Run the wave-primitive self-test (wave min / max / sum, wave cones) over
 * `blocks` workgroups on `device`; *failures = lanes that disagreed. */
int rt_debug_selftest(int device, int blocks, unsigned* failures);

#ifdef RT_PROF
/* Only in a library built with -DRT_PROF (tools/prof_sections.py,
 * tools/prof_tiles.py): per-section shader-clock totals and event counts
 * of the last renders (read and clear), and a per-tile record buffer. */
int rt_debug_prof(unsigned long long* out8);
int rt_debug_prof_events(unsigned long long* out8);
int rt_debug_prof_tiles(unsigned* dev, int ntiles);
#endif

#ifdef __cplusplus
}
#endif
#endif /* RT_AMD_RT_DEBUG_H */
