/*
 * rt_gather.h — the multi-GPU exchange of the frame (librt_gather.so).
 *
 * SURVEY.md 8(e) / BASELINE.json north_star: frames shard by image row
 * across GPUs "with a single RCCL gather over xGMI at the end".  The
 * reference renders one frame in one process (CScene::LancerRayons,
 * Scene.cpp:672, its CPU loop Scene.cpp:1538-1561, called once from
 * Main.cpp:181) and has no multi-GPU path; this is the exchange that a
 * row-sharded LancerRayons needs: every rank's rendered rows (device memory
 * on its own GPU) land in the root GPU's frame in one fused group of RCCL
 * point-to-point operations (ncclGroupStart, one ncclSend per chunk on the
 * owning rank and the matching ncclRecv on the root, ncclGroupEnd) — on
 * MI355X each peer's chunk crosses its own xGMI link to the root.
 *
 * One process drives all the GPUs (ncclCommInitAll): the library owns one
 * communicator and one stream per rank.  Separate from librt_amd.so so that
 * a process which already has an RCCL (PyTorch's torch.distributed) never
 * loads a second one through the renderer.
 *
 * Status codes are include/rt.h's (RT_OK, RT_E_*); the library never exits.
 */
#ifndef RT_GATHER_H
#define RT_GATHER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_gather rt_gather;

/* One contiguous run of frame bytes: rank `rank`'s device memory `src`
 * (on that rank's GPU) -> byte offset `dst_off` of the root frame.  A rank's
 * row slab is one chunk; a rank's cyclic band set one chunk per band. */
typedef struct rt_gather_chunk {
    int32_t rank;
    const void* src;
    size_t bytes;
    size_t dst_off;
} rt_gather_chunk;

/* Communicator over n distinct HIP devices (rank r = devices[r]; rank 0 is
 * the root).  RT_E_ARG for n <= 0 or a device listed twice (RCCL needs one
 * rank per GPU), RT_E_HIP / RT_E_UNSUPPORTED for device or RCCL failures. */
int rt_gather_create(int32_t n, const int32_t* devices, rt_gather** out);

/* Rank r's stream (a hipStream_t on devices[r]), to enqueue rank r's render
 * on before the gather (rt_render_async), so the gather follows it in order. */
void* rt_gather_stream(rt_gather*, int32_t rank);

/* Enqueue the gather of the chunks into `root_frame` (device memory on the
 * root's GPU, at least max(dst_off + bytes) bytes) as ONE RCCL group on the
 * ranks' streams: no host sync.  The root's own chunks go through RCCL too
 * (a send to itself).  Chunks must not overlap in the root frame. */
int rt_gather_chunks(rt_gather*, int32_t nchunks, const rt_gather_chunk* chunks, void* root_frame);

/* Wait for everything enqueued on the ranks' streams. */
int rt_gather_sync(rt_gather*);

/* RCCL's version (ncclGetVersion), for logs. */
int rt_gather_rccl_version(void);

const char* rt_gather_error(rt_gather*);
void rt_gather_destroy(rt_gather*);

#ifdef __cplusplus
}
#endif
#endif /* RT_GATHER_H */
