// rt_gather.cpp — the frame's RCCL gather (include/rt_gather.h): one process,
// n GPUs, one communicator per rank from ncclCommInitAll, and one fused group
// of point-to-point operations per gather — the root receives every chunk
// (its own by a send to itself), each peer sends its own over its xGMI link.
// the row-sharded frame's single exchange step.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "../../include/rt_gather.h"

struct rt_gather {
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> stream;
    std::string err;
};

#define RT_EXPORT extern "C" __attribute__((visibility("default")))

static int hip_err(rt_gather* g, hipError_t e, const char* what)
{
    g->err = std::string(what) + ": " + hipGetErrorString(e);
    return RT_E_HIP;
}
static int nccl_err(rt_gather* g, ncclResult_t r, const char* what)
{
    g->err = std::string(what) + ": " + ncclGetErrorString(r);
    return RT_E_UNSUPPORTED;
}

RT_EXPORT int rt_gather_rccl_version(void)
{
    int v = 0;
    return ncclGetVersion(&v) == ncclSuccess ? v : -1;
}

RT_EXPORT const char* rt_gather_error(rt_gather* g) { return g ? g->err.c_str() : "null gather"; }

RT_EXPORT void rt_gather_destroy(rt_gather* g)
{
    if (!g) return;
    for (size_t r = 0; r < g->stream.size(); ++r) {
        if (g->stream[r]) {
            (void)hipSetDevice(g->dev[r]);
            (void)hipStreamSynchronize(g->stream[r]);
            (void)hipStreamDestroy(g->stream[r]);
        }
    }
    for (ncclComm_t c : g->comm)
        if (c) ncclCommDestroy(c);
    delete g;
}

RT_EXPORT int rt_gather_create(int32_t n, const int32_t* devices, rt_gather** out)
{
    if (!out) return RT_E_ARG;
    *out = nullptr;
    rt_gather* g = new rt_gather();
    *out = g;
    if (n <= 0 || !devices) {
        g->err = "rt_gather_create: n > 0 devices needed";
        return RT_E_ARG;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        g->err = "no usable HIP device";
        return RT_E_HIP;
    }
    for (int r = 0; r < n; ++r) {
        if (devices[r] < 0 || devices[r] >= ndev) {
            g->err = "rt_gather_create: device " + std::to_string(devices[r]) + " out of range";
            return RT_E_ARG;
        }
        if (std::count(devices, devices + n, devices[r]) > 1) {
            g->err = "rt_gather_create: device " + std::to_string(devices[r]) +
                     " listed twice (RCCL needs one rank per GPU)";
            return RT_E_ARG;
        }
    }
    g->dev.assign(devices, devices + n);
    g->comm.assign((size_t)n, nullptr);
    g->stream.assign((size_t)n, nullptr);
    if (ncclResult_t r = ncclCommInitAll(g->comm.data(), n, g->dev.data()); r != ncclSuccess)
        return nccl_err(g, r, "ncclCommInitAll");
    for (int r = 0; r < n; ++r) {
        if (hipError_t e = hipSetDevice(g->dev[r]); e != hipSuccess) return hip_err(g, e, "hipSetDevice");
        if (hipError_t e = hipStreamCreateWithFlags(&g->stream[r], hipStreamNonBlocking); e != hipSuccess)
            return hip_err(g, e, "hipStreamCreate");
    }
    return RT_OK;
}

RT_EXPORT void* rt_gather_stream(rt_gather* g, int32_t rank)
{
    if (!g || rank < 0 || rank >= (int)g->stream.size()) return nullptr;
    return (void*)g->stream[rank];
}

RT_EXPORT int rt_gather_chunks(rt_gather* g, int32_t nchunks, const rt_gather_chunk* ch, void* root_frame)
{
    if (!g) return RT_E_ARG;
    const int n = (int)g->comm.size();
    if (n == 0 || nchunks < 0 || (nchunks > 0 && (!ch || !root_frame))) {
        g->err = "rt_gather_chunks: bad arguments";
        return RT_E_ARG;
    }
    for (int i = 0; i < nchunks; ++i)
        if (ch[i].rank < 0 || ch[i].rank >= n || (!ch[i].src && ch[i].bytes)) {
            g->err = "rt_gather_chunks: chunk " + std::to_string(i) + " has a bad rank or source";
            return RT_E_ARG;
        }
    // One group: the sends of every rank and the root's receives, so RCCL
    // progresses them together (each peer on its own link to the root).
    if (ncclResult_t r = ncclGroupStart(); r != ncclSuccess) return nccl_err(g, r, "ncclGroupStart");
    ncclResult_t res = ncclSuccess;
    for (int i = 0; i < nchunks && res == ncclSuccess; ++i) {
        if (ch[i].bytes == 0) continue;
        const int r = ch[i].rank;
        res = ncclSend(ch[i].src, ch[i].bytes, ncclUint8, 0, g->comm[r], g->stream[r]);
        if (res == ncclSuccess)
            res = ncclRecv((char*)root_frame + ch[i].dst_off, ch[i].bytes, ncclUint8, r, g->comm[0], g->stream[0]);
    }
    const ncclResult_t end = ncclGroupEnd();
    if (res != ncclSuccess) return nccl_err(g, res, "ncclSend/ncclRecv");
    if (end != ncclSuccess) return nccl_err(g, end, "ncclGroupEnd");
    return RT_OK;
}

RT_EXPORT int rt_gather_sync(rt_gather* g)
{
    if (!g) return RT_E_ARG;
    for (size_t r = 0; r < g->stream.size(); ++r) {
        if (hipError_t e = hipSetDevice(g->dev[r]); e != hipSuccess) return hip_err(g, e, "hipSetDevice");
        if (hipError_t e = hipStreamSynchronize(g->stream[r]); e != hipSuccess)
            return hip_err(g, e, "hipStreamSynchronize");
    }
    return RT_OK;
}
