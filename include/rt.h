/*
 * rt.h — C ABI of the MI355X-native Whitted ray tracer (librt_amd.so).
 *
 * Drop-in boundary for the reference's per-pixel hot path.  The reference
 * (Rodyll/Ray-Tracing-GPU, /root/reference/Projet-INF8702) exposes that path
 * through the CScene singleton (Scene.h:41-70) and chooses the CPU loop or the
 * GL compute shader inside CScene::LancerRayons (Scene.cpp:672) on the global
 * CVar::g_ComputerShadersON (Var.cpp:11).  This header replaces:
 *
 *   rt_scene_*      CScene's host surface: AjusterResolution (Scene.cpp:162),
 *                   AjusterNbRebondsMax / AjusterEnergieMinimale /
 *                   AjusterIndiceRefraction (Scene.cpp:180-217),
 *                   TraiterFichierDeScene (Scene.cpp:231), Initialiser
 *                   (Scene.cpp:140: InitialiserCamera + Pretraitement) and the
 *                   LancerRayons prologue (Scene.cpp:676-679).
 *   rt_create /     CNuanceurCalculProg(path, compile) + activer()
 *   rt_destroy      (NuanceurCalculProg.cpp:57,146) and the GL context.
 *   rt_upload_scene the std140 UBO marshal "General"/"SceneData"
 *                   (Scene.cpp:697-1269) — but file-ordered, unbounded, and
 *                   without the ≤10-per-type cap.
 *   rt_render*      glDispatchCompute(W/16,H/16,1) + glMemoryBarrier
 *                   (Scene.cpp:1307-1310) and, for parity, the CPU loop
 *                   (Scene.cpp:1538-1561) whose float RGB went to
 *                   glTexImage2D(GL_RGBA8, GL_RGB, GL_FLOAT) (Scene.cpp:1562).
 *
 * Conventions: every call returns 0 on success, a negative RT_E* code on
 * failure (the library never exits; see rt_last_error / rt_scene_error).
 * Images are row-major, memory row y = pixel row PixY, row 0 = BOTTOM
 * scanline (GL texture origin, Scene.cpp:1545-1546).  Thread-safe across
 * contexts, not within one.
 */
#ifndef RT_AMD_RT_H
#define RT_AMD_RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 8

enum {
    RT_OK = 0,
    RT_E_ARG = -1,       /* bad argument / null pointer                 */
    RT_E_IO = -2,        /* scene file cannot be opened                 */
    RT_E_PARSE = -3,     /* scene file rejected (see rt_scene_error)    */
    RT_E_STATE = -4,     /* call order violated (e.g. render before upload) */
    RT_E_HIP = -5,       /* HIP runtime error (see rt_last_error)       */
    RT_E_UNSUPPORTED = -6/* e.g. bounce depth beyond the compiled stack */
};

/* Surface kinds, file order is preserved in every array below. */
enum { RT_TRIANGLE = 0, RT_PLANE = 1, RT_QUADRIC = 2 };

/* Post-Pretraitement scene, FILE ORDER (the order of CScene::m_Surfaces).
 * geom[i*12 + …]:
 *   triangle: p0 p1 p2 (9)  normal (3)      — Triangle.h m_Pts / m_Normale
 *   plane   : normal (3) cst (1) 0…         — Plan.h m_Normale / m_Cst
 *   quadric : quad (3) lin (3) mix (3) cst  — Quadrique.h m_Quadratique /
 *                                             m_Lineaire / m_Mixte / m_Cst
 * material[i*10 + …]: r g b Ka Kd Ks shininess Kr Kt ior (ISurface.h:25-41)
 * lights[j*7 + …]   : pos(3) r g b intensity (Lumiere.h:23-27)
 * Caller owns the memory; rt_upload_scene deep-copies to the device. */
typedef struct rt_scene_flat {
    int32_t n_surfaces;
    int32_t n_lights;
    const int32_t* type;
    const float* geom;
    const float* material;
    const float* lights;
} rt_scene_flat;

/* One frame (or one row slab of it, for multi-GPU sharding). */
typedef struct rt_frame {
    float cam_pos[3];     /* CameraDeScene::Position                        */
    float orient[16];     /* CameraDeScene::Orientation, row-major m[4][4]  */
    float half_w, half_h; /* Scene.cpp:676-677                              */
    float inv_w, inv_h;   /* Scene.cpp:678-679                              */
    float background[3];  /* m_CouleurArrierePlan                           */
    int32_t width, height;
    int32_t row_begin, row_end; /* slab [row_begin,row_end) of PixY         */
    int32_t max_bounces;  /* m_NbRebondsMax (0 = the shipped executable)    */
    float min_energy;     /* m_EnergieMinRayon (0.01)                       */
    float scene_ior;      /* m_IndiceRefractionScene (1.0)                  */
    int32_t flags;        /* RT_FLAG_*                                      */
    /* ABI 3, multi-GPU load balance: band_rows > 0 (a
     * multiple of 16) renders cyclic row bands instead of the slab — global
     * bands b = band_index, band_index + band_count, ... of band_rows rows
     * each (band b = rows [b*band_rows, (b+1)*band_rows)), packed in that
     * order into the output; rows >= height are skipped and row_begin /
     * row_end are ignored.  The output then holds rt_band_rows(height,
     * band_rows, band_count, band_index) rows.  band_rows = 0: the slab.   */
    int32_t band_rows;
    int32_t band_count;
    int32_t band_index;
} rt_frame;

#define RT_FLAG_STATS 1   /* count rays / tests into rt_stats (small cost)  */

typedef struct rt_stats {
    uint64_t primary_rays;
    uint64_t bounce_rays;  /* reflected + refracted rays traced            */
    uint64_t shadow_rays;  /* rays sent to ObtenirFiltreDeSurface           */
    uint64_t shadow_tests_skipped; /* shadow tests elided by the exact
                                      all-lanes-opaque early exit           */
    float kernel_ms;       /* last render's kernel time (hipEvent)          */
    int32_t stack_depth;   /* compiled bounce-stack depth that ran          */
    int32_t light_batch;   /* lights sharing one shadow pass in that kernel */
    /* exact ray-primitive tests executed (ABI 2): a test a wave runs counts
       once per lane of the wave, culled tests not at all                    */
    uint64_t triangle_tests;
    uint64_t plane_tests;
    uint64_t quadric_tests;
    /* ABI 7: bounce rays (reflected / refracted, Scene.cpp:1779-1823): their
       exact triangle tests (part of triangle_tests; brute force: every
       triangle per ray) and the BVH inner nodes they visited (RT_OPT_BVH)  */
    uint64_t bounce_triangle_tests;
    uint64_t bvh_nodes_visited;
    char kernel[48];       /* the trace kernel that ran, e.g.
                              "rt_trace_tiny<0,1,37>"                        */
} rt_stats;

/* ------------------------------------------------------------ host scene */
typedef struct rt_scene rt_scene;

int rt_scene_create(rt_scene** out);                          /* CScene::CScene, Scene.cpp:61 */
int rt_scene_set_resolution(rt_scene*, int32_t w, int32_t h);  /* AjusterResolution, Scene.cpp:162 */
int rt_scene_set_max_bounces(rt_scene*, int32_t n);            /* AjusterNbRebondsMax, Scene.cpp:180 */
int rt_scene_set_min_energy(rt_scene*, float e);               /* AjusterEnergieMinimale, Scene.cpp:197 */
int rt_scene_set_scene_ior(rt_scene*, float ior);              /* AjusterIndiceRefraction, Scene.cpp:214 */
int rt_scene_load_file(rt_scene*, const char* path);           /* TraiterFichierDeScene, Scene.cpp:231 */
int rt_scene_prepare(rt_scene*);            /* Initialiser, Scene.cpp:140 (ONCE; not per frame) */
int rt_scene_get_flat(const rt_scene*, rt_scene_flat* out);    /* views into scene-owned arrays */
int rt_scene_get_frame(const rt_scene*, rt_frame* out);        /* full-frame rt_frame */
const char* rt_scene_error(const rt_scene*);
void rt_scene_destroy(rt_scene*);

/* --------------------------------------------------------------- device */
typedef struct rt_ctx rt_ctx;

int rt_create(int32_t hip_device, rt_ctx** out);
int rt_upload_scene(rt_ctx*, const rt_scene_flat*);
/* Synchronous.  rgba8_out: host or device pointer to
 * (row_end-row_begin)*width*4 bytes (or rt_band_rows(...) rows for bands),
 * RGBA8 = GL float->unorm8 of the RGB (clamp to [0,1], round to nearest,
 * alpha 255).  The synchronous renders also (re)build what is kept per
 * camera — the camera buffer of per-tile triangle lists — when the camera
 * (position, orientation, resolution) changed since the last build. */
int rt_render(rt_ctx*, const rt_frame*, uint8_t* rgba8_out);
/* Parity/debug: float RGB exactly as m_InfoPixel (unclamped), 3 floats/px. */
int rt_render_float(rt_ctx*, const rt_frame*, float* rgb_out);
/* Asynchronous, device pointers only, enqueued on `hip_stream` (a hipStream_t;
 * NULL = the HIP null stream, as in every HIP API).  Either output may be
 * NULL.  No host sync.  ABI 5: a new camera's per-camera state — the camera
 * buffer included, where it pays (RT_OPT_CAMERA_BUFFER) — is built on
 * `hip_stream` too; allocation happens only when that state grows (its
 * capacity follows earlier builds' totals, read back without waiting; a tile
 * whose list does not fit this time renders by the per-wave path — the same
 * image either way).
 *
 * Ordering (ABI 4).  The context keeps per-camera state on the device (camera
 * records, cone records, the camera buffer).  Every write of that state is
 * ordered after every render already enqueued on any stream that may read
 * it, and every render after the write that produced its state, with HIP
 * events — the caller needs no host sync between rt_render_async on any
 * number of streams and the synchronous calls, in any order.  A stream
 * passed here must stay alive until the next synchronous call on the context
 * (rt_render*, rt_upload_scene, rt_sync, rt_destroy) returns.
 *
 * hipGraph capture.  When `hip_stream` is capturing, the call records only
 * the trace kernel: the camera state must already be current for the frame
 * (a synchronous render, or rt_prepare_camera, of that camera first), else
 * RT_E_STATE.  A replay renders with the camera state current at replay
 * time, so it is valid while no other camera is rendered on the context; no
 * buffer a captured render references is freed before rt_upload_scene or
 * rt_destroy. */
int rt_render_async(rt_ctx*, const rt_frame*, uint8_t* rgba8_dev, float* rgb_dev, void* hip_stream);
/* ABI 4: a camera path rendered on the device — the headless analogue of
 * the reference's GLUT display loop (Main.cpp:229-250).
 * frames[0..n) (any cameras and sizes) are rendered after the work already
 * on `hip_stream`, and the work enqueued on it afterwards runs after all of
 * them; frame i's RGBA8 goes to rgba8_dev + i * rgba8_stride bytes and/or
 * its float RGB to (char*)rgb_dev + i * rgb_stride.  Frame i prepares its
 * own camera into sequence slot i % 4 (apart from the state the other
 * render calls use) and runs on the context's internal stream i % 4, forked
 * from and joined back into `hip_stream` by events, so up to four
 * consecutive frames are in flight at once; the call needs no host sync (and
 * allocates only when a slot's state grows), and a sequence captured into a hipGraph
 * (the internal streams join the capture) replays exactly whatever was
 * rendered on the context between capture and replay.  A sequence waits for
 * the context's async work on other streams (the slots are shared); a
 * captured one is ordered by its graph's position only.  Shadow rays use the
 * light buffer; camera rays the slot's own camera buffer (ABI 5: built on
 * the frame's stream; inside a capture only into a slot an earlier call
 * sized, else the per-wave culling — the same image).  RT_FLAG_STATS is not
 * accepted here. */
int rt_render_sequence_async(rt_ctx*, const rt_frame* frames, int32_t n, uint8_t* rgba8_dev, size_t rgba8_stride,
                             float* rgb_dev, size_t rgb_stride, void* hip_stream);
/* ABI 4: make the per-camera state (camera records, and the camera buffer
 * where the frame's kernel uses one) current for `frame` without rendering.
 * Synchronous, like rt_render. */
int rt_prepare_camera(rt_ctx*, const rt_frame* frame);
/* ABI 4: wait until everything enqueued through this context (any stream)
 * has finished. */
int rt_sync(rt_ctx*);

/* ABI 4: the CPU backend (the reference's CPU branch of
 * LancerRayons, Scene.cpp:1535-1563, which it chose on
 * CVar::g_ComputerShadersON, Var.cpp:11).  Explicit only: a context made by
 * rt_create_cpu (threads <= 0: all cores; no HIP call is made) takes
 * rt_upload_scene and renders with rt_cpu_render / rt_cpu_render_float into
 * host memory — the HIP path's images, bit for bit, by brute force on host
 * threads.  The HIP render entry points return RT_E_STATE on a CPU context,
 * and rt_create never returns one: a missing GPU is an error, never a switch. */
int rt_create_cpu(int32_t threads, rt_ctx** out);
int rt_cpu_render(rt_ctx*, const rt_frame*, uint8_t* rgba8_out);
int rt_cpu_render_float(rt_ctx*, const rt_frame*, float* rgb_out);

/* ABI 4: context options.  A/B and test switches and tuning knobs; no option
 * changes a single bit of any image.  Upload options take effect at the next
 * rt_upload_scene, launch options at the next render.                      */
enum {
    RT_OPT_LIGHT_BUFFER = 1,    /* upload+launch: shadow rays through the light buffer:
                                   1 every depth-0 scene with opaque triangles (default),
                                   2 only above 1,024 triangles, 0 never (wave culling) */
    RT_OPT_CAMERA_BUFFER = 2,   /* launch: per-camera tile lists: 1 (default) built by
                                   synchronous renders, by an async frame repeating the
                                   previous async frame's camera, and by async / sequence
                                   frames of a new camera where the build pays (more than
                                   1,024 triangles and at least 4 Mpx of output rows);
                                   2 by every frame; 0 never */
    RT_OPT_UNION_PRETEST = 3,   /* launch: small lists' union cone pre-test, 1 (default) / 0 */
    RT_OPT_LB_SCALE = 4,        /* upload: light-buffer cells per cone radius; 0 = auto (4,
                                   at least 128 cells per face edge; 6 above 1,024
                                   triangles); > 0 sets R alone */
    RT_OPT_DCOV_NEAR = 5,       /* upload: big lists' near light-buffer distance, x the
                                   light's farthest triangle; 0 = default (1.25) */
    RT_OPT_CB_INLINE_MAX_MB = 6,/* launch: camera-buffer entries carry inline camera
                                   records while they fit this many MiB (default 0 =
                                   never: the index walk, whose records are staged in
                                   LDS per window; 128 was the round-1 default) */
    RT_OPT_HOST_CHUNK_MB = 7,   /* launch: synchronous renders into host memory render
                                   and copy in row chunks of this many MiB of output,
                                   each copy overlapping the next chunk (default 8;
                                   0 = one kernel, then one copy) */
    RT_OPT_CB_CAPACITY = 8,     /* launch (ABI 5): camera-buffer entries allocated;
                                   0 (default) = sized from earlier builds' totals.  A
                                   tile whose list does not fit renders by the per-wave
                                   path (tests: a small value exercises that path) */
    RT_OPT_BVH = 13,            /* launch (ABI 7): bounce rays of scenes with at least
                                   64 triangles and a reflective or refractive surface
                                   walk the exact BVH built at upload (rt_bvh.h), with
                                   the depth-0 kernels' camera buffer and light-buffer
                                   shadows: 1 (default) / 0 (every triangle per bounce ray) */
    RT_OPT_WAVEFRONT = 14,      /* launch (ABI 7): such frames (RT_OPT_BVH) render their
                                   bounce levels as compacted queues in HBM, one launch
                                   per level then a fold per level (up to 8 levels,
                                   not inside a hipGraph capture or a sequence): 1
                                   (default) / 0 (one kernel, a per-lane DFS stack) */
    RT_OPT_WF_SORT = 15,        /* launch (ABI 8): such wavefront frames order each level's
                                   live rays by counting sorts on the device: bit 0 by
                                   their parent surface's bin (BVH leaf order) and branch
                                   before the BVH walk, bit 1 by their hit surface's bin
                                   before the shading (with bit 2: by the hit point's
                                   light-buffer cell seen from light 0 instead); 0 queue
                                   order; default 1; never changes an image */
    RT_OPT_XCD_DEAL = 16,       /* launch (ABI 8): how the big-list kernels (more than
                                   1,024 triangles) deal 8 x 8 tiles to the 8 XCDs: 1
                                   (default) runs of 8 along a tile row, 2 column stripes
                                   (each XCD walks its own 1/8 of the columns row by row),
                                   3 4 x 2 super-tiles round-robin, 0 hardware order;
                                   never changes an image */
    RT_OPT_XCD_STRIPE = 17,     /* launch (ABI 8): RT_OPT_XCD_DEAL 2's stripe width in tiles,
                                   stripe s on XCD s % 8; 0 (default) one stripe per XCD */
    RT_OPT_LB_UNROLL = 18,      /* launch (ABI 8): depth-0 frames of more than 1,024 triangles
                                   under 4 Mpx of output rows walk the light buffer's
                                   per-lane lists two entries per round: 1 (default) / 0;
                                   never changes an image */
    RT_OPT_WF_OVERLAP = 19,     /* launch (ABI 8): wavefront frames finish each level's
                                   straggling BVH walks and shade their rays on a second
                                   stream while the level's other rays are shaded (one
                                   event fork and join per level): 1 (default) / 0;
                                   never changes an image */
    RT_OPT_LAUNCH_CAMERA = 12   /* launch (ABI 6): depth-0 frames of scenes of 1-20
                                   triangles with light-buffer shadows take their camera
                                   records with the kernel launch — per-triangle camera
                                   values, nearest-hit bounds and tile-mask planes
                                   computed on the host per camera; the trace kernel
                                   computes its tile masks (stored per stream from a
                                   camera's second frame) — so no camera prepass or
                                   camera buffer exists and a moving camera renders
                                   like a static one: 1 (default) / 0 (the device
                                   camera buffer) */
    /* 9-11 (ABI 5: the async camera-state ring, the bounce lane-refill kernel,
       compact light-buffer entries) were measured slower or no faster and are
       removed in ABI 6: rt_set_option returns RT_E_ARG for them.  Their code
       and measurements: profiles/r04/set_aside/. */
};
int rt_set_option(rt_ctx*, int32_t option, double value);
int rt_get_option(rt_ctx*, int32_t option, double* value);
/* ABI 4, upload: the far light-buffer ladder of big lists — rising distance
 * factors (x the light's farthest triangle), n <= 8; n = 0: none; factors =
 * NULL and n < 0: the default 2.5, 6, 16, 64. */
int rt_set_far_ladder(rt_ctx*, const double* factors, int32_t n);
int rt_last_stats(rt_ctx*, rt_stats* out);
const char* rt_last_error(rt_ctx*);
void rt_destroy(rt_ctx*);

int rt_abi_version(void);
/* Output rows of one rank's band set (see rt_frame.band_rows); -1 if invalid. */
int32_t rt_band_rows(int32_t height, int32_t band_rows, int32_t band_count, int32_t band_index);

#ifdef __cplusplus
}
#endif
#endif /* RT_AMD_RT_H */
