// rt_main.cpp — headless counterpart of the reference's Main.cpp entry point.
//
//   rt_render <scene.dat> [-x W] [-y H] [-d depth] [-o out.ppm] [-g gpus]
//             [--device first] [--bands] [-n frames] [-s]
//             [--gather rccl|host] [--backend hip|cpu] [--threads N]
//
// Kept from Main.cpp:51-199: argv[1] is the scene file, -x / -y set the
// resolution (default 512x256, Var.cpp:4-5), the same [ETAT]/[ERREUR] log
// lines, and one wall-clock timer around the render (Main.cpp:168-198) — here
// with microsecond resolution (the Linux branch divides tv_usec by 10^6 in
// integer arithmetic, Main.cpp:192-193) and excluding GL set-up.
// Changed: the power-of-two check (Main.cpp:79-84) is advisory only, because
// the render core has no such restriction; there is no GLUT window — the
// frame is written as a binary PPM (top row first) instead; -d sets
// m_NbRebondsMax (default 0 = the shipped executable, whose recursion is
// commented out); -n renders N frames (the scene is prepared once, unlike
// LancerRayons which re-runs Pretraitement); -s prints ray counters.
// Multi-GPU from the command line: -g N renders the frame
// with N contexts, one per GPU from --device on, every context rendering its
// row slab (or, with --bands, its cyclic 16-row bands) into device memory on
// its own GPU, enqueued on its rank's stream; then ONE RCCL gather
// (librt_gather.so, include/rt_gather.h: ncclCommInitAll over the N GPUs, one
// ncclGroupStart / ncclSend / ncclRecv group) brings every part into the root
// GPU's frame over xGMI — the north star's "single RCCL gather" — and the
// frame crosses PCIe once, from the root.  --gather rccl uses it for -g 1 too
// (a send of the root's slab to itself).  With more contexts than GPUs
// (contexts wrapping round onto shared GPUs: RCCL needs one rank per GPU) or
// --gather host, each context renders straight into its part of the host
// frame on a host thread of its own and the parts are assembled in host
// memory — the same partition, without a collective.  --backend cpu renders
// on host threads instead (rt_create_cpu,
// the reference's CPU branch, chosen there by CVar::g_ComputerShadersON):
// the same image, the GPU never touched.
#include <hip/hip_runtime_api.h>

#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt.h"
#include "../../include/rt_gather.h"

static int fail(const char* what, int rc, const char* msg)
{
    std::fprintf(stderr, "[ERREUR]: %s (code %d): %s\n", what, rc, msg ? msg : "");
    return 1;
}

// The frame (memory row 0 = bottom scanline) as a binary PPM, top row first.
static int write_ppm(const char* path, int W, int H, const std::vector<uint8_t>& img)
{
    FILE* f = std::fopen(path, "wb");
    if (!f) return 1;
    std::fprintf(f, "P6\n%d %d\n255\n", W, H);
    for (int y = H - 1; y >= 0; --y)
        for (int x = 0; x < W; ++x) std::fwrite(&img[((size_t)y * W + x) * 4], 1, 3, f);
    std::fclose(f);
    std::printf("[ETAT]: Image ecrite dans %s\n", path);
    return 0;
}

static void print_done(rt_ctx* c0, double total, int frames, int gpus, int band, bool stats)
{
    rt_stats st;
    rt_last_stats(c0, &st);
    std::printf("[ETAT]: Termine! --> Temps total de rendu : %.6f secondes (%d frame(s), %d GPU(s)%s, kernel %.3f ms)\n",
                total, frames, gpus, band ? " bands" : "", st.kernel_ms);
    if (stats)
        std::printf("[STATS]: primary=%llu bounce=%llu shadow=%llu shadow_tests_skipped=%llu stack=%d "
                    "tests: triangle=%llu plane=%llu quadric=%llu (context 0)\n",
                    (unsigned long long)st.primary_rays, (unsigned long long)st.bounce_rays,
                    (unsigned long long)st.shadow_rays, (unsigned long long)st.shadow_tests_skipped,
                    st.stack_depth, (unsigned long long)st.triangle_tests, (unsigned long long)st.plane_tests,
                    (unsigned long long)st.quadric_tests);
}

// librt_gather.so, loaded only by the RCCL path (dlopen next to this
// binary): every other mode — --backend cpu, one GPU, --gather host — runs
// without RCCL present.
struct GatherLib {
    void* h = nullptr;
    int (*create)(int32_t, const int32_t*, rt_gather**) = nullptr;
    void* (*stream)(rt_gather*, int32_t) = nullptr;
    int (*chunks)(rt_gather*, int32_t, const rt_gather_chunk*, void*) = nullptr;
    int (*sync)(rt_gather*) = nullptr;
    int (*version)(void) = nullptr;
    const char* (*error)(rt_gather*) = nullptr;
    void (*destroy)(rt_gather*) = nullptr;
};

static bool load_gather(GatherLib& L, std::string& why)
{
    char exe[4096];
    const ssize_t n = readlink("/proc/self/exe", exe, sizeof exe - 1);
    std::string dir = ".";
    if (n > 0) {
        exe[n] = '\0';
        dir = exe;
        dir = dir.substr(0, dir.find_last_of('/'));
    }
    const std::string path = dir + "/librt_gather.so";
    L.h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!L.h) {
        const char* e = dlerror();
        why = path + ": " + (e ? e : "dlopen failed");
        return false;
    }
    auto sym = [&](const char* name) { return dlsym(L.h, name); };
    L.create = (decltype(L.create))sym("rt_gather_create");
    L.stream = (decltype(L.stream))sym("rt_gather_stream");
    L.chunks = (decltype(L.chunks))sym("rt_gather_chunks");
    L.sync = (decltype(L.sync))sym("rt_gather_sync");
    L.version = (decltype(L.version))sym("rt_gather_rccl_version");
    L.error = (decltype(L.error))sym("rt_gather_error");
    L.destroy = (decltype(L.destroy))sym("rt_gather_destroy");
    if (!L.create || !L.stream || !L.chunks || !L.sync || !L.version || !L.error || !L.destroy) {
        why = path + ": missing rt_gather_* symbols";
        return false;
    }
    return true;
}

// The RCCL path of -g N (N distinct GPUs), pipelined: every rank renders
// frame k into one of two slabs in device memory on its own GPU (on a render
// stream of its own), and frame k's RCCL group — a slab is one chunk, a band
// set one chunk per 16-row band, each landing at its rows of the root GPU's
// frame — runs on the ranks' gather streams while frame k + 1 renders into
// the other slabs; ordering by events only (render k -> gather k on each
// rank; gather k -> render k + 2 into the same slab), one host sync at the
// end.  Reported per frame: the renders (slowest rank, events) and the
// gather (root's gather stream, events), and the wall time of all frames.
static int render_rccl(std::vector<rt_ctx*>& ctx, std::vector<rt_frame>& part,
                       const std::vector<std::vector<uint8_t>>& img, int W, int H, int band, int dev0, int ndev,
                       int frames, bool stats, const char* out, rt_scene* scene)
{
    GatherLib G;
    std::string why;
    if (!load_gather(G, why)) return fail("librt_gather.so", RT_E_UNSUPPORTED, why.c_str());
    const int n = (int)ctx.size();
    std::vector<int32_t> devs((size_t)n);
    for (int r = 0; r < n; ++r) devs[r] = (dev0 + r) % ndev;
    rt_gather* g = nullptr;
    int rc = G.create(n, devs.data(), &g);
    if (rc) return fail("rt_gather_create", rc, G.error(g));
    const size_t rowb = (size_t)W * 4;
    // per rank: two slabs, a render stream, events (render done / gather
    // done per slab, timing pairs per frame)
    std::vector<void*> slab((size_t)2 * n, nullptr);
    std::vector<hipStream_t> rs((size_t)n, nullptr);
    std::vector<hipEvent_t> ev_r((size_t)2 * n, nullptr), ev_g((size_t)2 * n, nullptr);
    std::vector<hipEvent_t> t_r0((size_t)n * frames, nullptr), t_r1((size_t)n * frames, nullptr);
    std::vector<hipEvent_t> t_g0((size_t)frames, nullptr), t_g1((size_t)frames, nullptr);
    void* full = nullptr;
    for (int r = 0; r < n; ++r) {
        (void)hipSetDevice(devs[r]);
        for (int b = 0; b < 2; ++b)
            if (!img[r].empty() && hipMalloc(&slab[2 * r + b], img[r].size()) != hipSuccess)
                return fail("hipMalloc", RT_E_HIP, "slab");
        if (r == 0 && hipMalloc(&full, rowb * H) != hipSuccess) return fail("hipMalloc", RT_E_HIP, "frame");
        if (hipStreamCreateWithFlags(&rs[r], hipStreamNonBlocking) != hipSuccess) return fail("hipStreamCreate", RT_E_HIP, "");
        for (int b = 0; b < 2; ++b) {
            if (hipEventCreateWithFlags(&ev_r[2 * r + b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&ev_g[2 * r + b], hipEventDisableTiming) != hipSuccess)
                return fail("hipEventCreate", RT_E_HIP, "");
        }
        for (int k = 0; k < frames; ++k)
            if (hipEventCreate(&t_r0[(size_t)r * frames + k]) != hipSuccess ||
                hipEventCreate(&t_r1[(size_t)r * frames + k]) != hipSuccess)
                return fail("hipEventCreate", RT_E_HIP, "");
        if (r == 0)
            for (int k = 0; k < frames; ++k)
                if (hipEventCreate(&t_g0[k]) != hipSuccess || hipEventCreate(&t_g1[k]) != hipSuccess)
                    return fail("hipEventCreate", RT_E_HIP, "");
    }
    auto chunks_of = [&](int b) {
        std::vector<rt_gather_chunk> ch;
        for (int r = 0; r < n; ++r) {
            if (img[r].empty()) continue;
            const char* src = (const char*)slab[2 * r + b];
            if (band) {  // packed band j of rank r -> frame rows (j n + r) band ...
                const int q = (int)(img[r].size() / rowb) / band;
                for (int j = 0; j < q; ++j) {
                    const int y0 = (j * n + r) * band, rows = std::min(band, H - y0);
                    if (rows > 0) ch.push_back({r, src + (size_t)j * band * rowb, (size_t)rows * rowb, (size_t)y0 * rowb});
                }
            } else {
                ch.push_back({r, src, img[r].size(), (size_t)part[r].row_begin * rowb});
            }
        }
        return ch;
    };
    const std::vector<rt_gather_chunk> ch[2] = {chunks_of(0), chunks_of(1)};
    size_t gbytes = 0;
    for (const auto& c : ch[0]) gbytes += c.bytes;
    const int ver = G.version();
    std::printf("[ETAT]: gather: RCCL %d.%d.%d, %d rank(s), %zu chunk(s), %.1f MB into GPU %d, pipelined (2 slabs)\n",
                ver / 10000, (ver / 100) % 100, ver % 100, n, ch[0].size(), gbytes / 1e6, devs[0]);
    std::printf("[ETAT]: Lancer de rayons...\n");
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < frames; ++k) {
        const int b = k & 1;
        for (int r = 0; r < n; ++r) {
            if (img[r].empty()) continue;
            (void)hipSetDevice(devs[r]);
            if (k >= 2 && hipStreamWaitEvent(rs[r], ev_g[2 * r + b], 0) != hipSuccess)  // gather k-2 read this slab
                return fail("hipStreamWaitEvent", RT_E_HIP, "");
            (void)hipEventRecord(t_r0[(size_t)r * frames + k], rs[r]);
            if ((rc = rt_render_async(ctx[r], &part[r], (uint8_t*)slab[2 * r + b], nullptr, rs[r])))
                return fail("LancerRayons", rc, rt_last_error(ctx[r]));
            (void)hipEventRecord(t_r1[(size_t)r * frames + k], rs[r]);
            (void)hipEventRecord(ev_r[2 * r + b], rs[r]);
            if (hipStreamWaitEvent((hipStream_t)G.stream(g, r), ev_r[2 * r + b], 0) != hipSuccess)
                return fail("hipStreamWaitEvent", RT_E_HIP, "");
        }
        (void)hipSetDevice(devs[0]);
        // the root's gather stream starts timing once EVERY rank's slab is
        // rendered (its receives wait for them anyway), so the reported
        // gather time is the exchange, not the slowest rank's render
        for (int r = 1; r < n; ++r)
            if (!img[r].empty() && hipStreamWaitEvent((hipStream_t)G.stream(g, 0), ev_r[2 * r + b], 0) != hipSuccess)
                return fail("hipStreamWaitEvent", RT_E_HIP, "");
        (void)hipEventRecord(t_g0[k], (hipStream_t)G.stream(g, 0));
        if ((rc = G.chunks(g, (int32_t)ch[b].size(), ch[b].data(), full)))
            return fail("rt_gather_chunks", rc, G.error(g));
        (void)hipEventRecord(t_g1[k], (hipStream_t)G.stream(g, 0));
        for (int r = 0; r < n; ++r) {
            if (img[r].empty()) continue;
            (void)hipSetDevice(devs[r]);
            (void)hipEventRecord(ev_g[2 * r + b], (hipStream_t)G.stream(g, r));
        }
    }
    if ((rc = G.sync(g))) return fail("rt_gather_sync", rc, G.error(g));
    for (int r = 0; r < n; ++r) {
        (void)hipSetDevice(devs[r]);
        (void)hipStreamSynchronize(rs[r]);
    }
    const double total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    double rsum = 0.0, gsum = 0.0;
    for (int k = 0; k < frames; ++k) {
        float worst = 0.f, gm = 0.f;
        for (int r = 0; r < n; ++r) {
            if (img[r].empty()) continue;
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, t_r0[(size_t)r * frames + k], t_r1[(size_t)r * frames + k]) == hipSuccess)
                worst = std::max(worst, ms);
        }
        (void)hipEventElapsedTime(&gm, t_g0[k], t_g1[k]);
        rsum += worst;
        gsum += gm;
    }
    std::vector<uint8_t> host(rowb * H);
    (void)hipSetDevice(devs[0]);
    if (hipMemcpy(host.data(), full, host.size(), hipMemcpyDeviceToHost) != hipSuccess)
        return fail("hipMemcpy", RT_E_HIP, "frame to host");
    std::printf("[ETAT]: per frame: render %.3f ms (slowest rank), gather %.3f ms (RCCL group of %zu send/recv "
                "pair(s)), wall %.3f ms\n",
                rsum / frames, gsum / frames, ch[0].size(), total * 1e3 / frames);
    print_done(ctx[0], total, frames, n, band, stats);
    if (out && write_ppm(out, W, H, host)) return fail("fopen", -1, out);
    for (int r = 0; r < n; ++r) {
        (void)hipSetDevice(devs[r]);
        for (int b = 0; b < 2; ++b) {
            (void)hipFree(slab[2 * r + b]);
            (void)hipEventDestroy(ev_r[2 * r + b]);
            (void)hipEventDestroy(ev_g[2 * r + b]);
        }
        for (int k = 0; k < frames; ++k) {
            (void)hipEventDestroy(t_r0[(size_t)r * frames + k]);
            (void)hipEventDestroy(t_r1[(size_t)r * frames + k]);
        }
        (void)hipStreamDestroy(rs[r]);
    }
    (void)hipSetDevice(devs[0]);
    for (int k = 0; k < frames; ++k) {
        (void)hipEventDestroy(t_g0[k]);
        (void)hipEventDestroy(t_g1[k]);
    }
    (void)hipFree(full);
    G.destroy(g);
    for (rt_ctx* c : ctx) rt_destroy(c);
    rt_scene_destroy(scene);
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        std::fprintf(stderr, "[ERREUR]: Aucune fichier de scene ne fut passe en argument !\n");
        return 1;
    }
    int W = 512, H = 256, depth = 0, dev0 = 0, frames = 1, gpus = 1, threads = 0;
    bool stats = false, bands = false, cpu = false, dev_given = false, g_given = false;
    int gather = -1;  // -1 auto (RCCL for -g > 1 on distinct GPUs), 0 host, 1 RCCL
    const char* out = nullptr;
    for (int i = 2; i < argc; ++i) {
        if (argv[i][0] != '-') continue;
        auto next = [&](int& v) {
            if (i + 1 < argc) v = std::atoi(argv[++i]);
        };
        if (std::strcmp(argv[i], "--device") == 0) {
            next(dev0);
            dev_given = true;
            continue;
        }
        if (std::strcmp(argv[i], "--bands") == 0) {
            bands = true;
            continue;
        }
        if (std::strcmp(argv[i], "--threads") == 0) {
            next(threads);
            continue;
        }
        if (std::strcmp(argv[i], "--gather") == 0) {
            const char* b = i + 1 < argc ? argv[++i] : "";
            if (std::strcmp(b, "rccl") == 0)
                gather = 1;
            else if (std::strcmp(b, "host") == 0)
                gather = 0;
            else
                return fail("arguments", RT_E_ARG, "--gather is rccl or host");
            continue;
        }
        if (std::strcmp(argv[i], "--backend") == 0) {
            const char* b = i + 1 < argc ? argv[++i] : "";
            if (std::strcmp(b, "cpu") == 0)
                cpu = true;
            else if (std::strcmp(b, "hip") != 0)
                return fail("arguments", RT_E_ARG, "--backend is hip or cpu");
            continue;
        }
        switch (argv[i][1]) {
        case 'x': next(W); break;
        case 'y': next(H); break;
        case 'd': next(depth); break;
        case 'g':
            next(gpus);
            g_given = true;
            break;
        case 'n': next(frames); break;
        case 's': stats = true; break;
        case 'o':
            if (i + 1 < argc) out = argv[++i];
            break;
        }
    }
    if (W <= 0 || H <= 0 || gpus <= 0 || frames <= 0) return fail("arguments", RT_E_ARG, "-x/-y/-g/-n must be > 0");
    // -g was the HIP device index before ABI 3; it is now the GPU count
    if (g_given && !dev_given)
        std::fprintf(stderr, "[NOTE]: -g %d = number of GPUs (from device 0); the device index is --device\n", gpus);
    if (((W - 1) & W) || ((H - 1) & H))
        std::fprintf(stderr, "[ATTENTION]: Resolution %dx%d n'est pas une puissance de deux "
                             "(accepted: the render core has no such restriction)\n", W, H);

    rt_scene* scene = nullptr;
    int rc = rt_scene_create(&scene);
    if (rc) return fail("rt_scene_create", rc, "");
    rt_scene_set_resolution(scene, W, H);
    rt_scene_set_max_bounces(scene, depth);
    std::printf("[ETAT]: Traitement du fichier de donnees de la scene...\n");
    if ((rc = rt_scene_load_file(scene, argv[1]))) return fail("TraiterFichierDeScene", rc, rt_scene_error(scene));
    if ((rc = rt_scene_prepare(scene))) return fail("Initialiser", rc, rt_scene_error(scene));
    rt_scene_flat flat;
    rt_scene_get_flat(scene, &flat);
    rt_frame frame;
    rt_scene_get_frame(scene, &frame);
    if (stats) frame.flags |= RT_FLAG_STATS;

    if (cpu) {  // the CPU backend: one context, host threads
        if (gpus != 1 || bands) return fail("arguments", RT_E_ARG, "-g / --bands are for the hip backend");
        rt_ctx* c = nullptr;
        if ((rc = rt_create_cpu(threads, &c))) return fail("rt_create_cpu", rc, "");
        if ((rc = rt_upload_scene(c, &flat))) return fail("rt_upload_scene", rc, rt_last_error(c));
        std::vector<uint8_t> img((size_t)W * H * 4);
        std::printf("[ETAT]: Lancer de rayons (CPU)...\n");
        double total = 0.0;
        for (int k = 0; k < frames; ++k) {
            const auto t0 = std::chrono::steady_clock::now();
            if ((rc = rt_cpu_render(c, &frame, img.data()))) return fail("LancerRayons", rc, rt_last_error(c));
            total += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
        std::printf("[ETAT]: Termine! --> Temps total de rendu : %.6f secondes (%d frame(s), CPU)\n", total, frames);
        if (out && write_ppm(out, W, H, img)) return fail("fopen", -1, out);
        rt_destroy(c);
        rt_scene_destroy(scene);
        return 0;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail("rt_create", RT_E_HIP, "no HIP device");
    // one context per GPU share; part r = rows of slab r, or band set r
    const int band = bands ? 16 : 0;
    std::vector<rt_ctx*> ctx((size_t)gpus, nullptr);
    std::vector<rt_frame> part((size_t)gpus, frame);
    std::vector<std::vector<uint8_t>> img((size_t)gpus);
    const int slab = (H + gpus - 1) / gpus;
    for (int r = 0; r < gpus; ++r) {
        if ((rc = rt_create((dev0 + r) % ndev, &ctx[r]))) return fail("rt_create", rc, ctx[r] ? rt_last_error(ctx[r]) : "");
        if ((rc = rt_upload_scene(ctx[r], &flat))) return fail("rt_upload_scene", rc, rt_last_error(ctx[r]));
        rt_frame& f = part[r];
        int rows;
        if (band) {
            f.band_rows = band;
            f.band_count = gpus;
            f.band_index = r;
            rows = rt_band_rows(H, band, gpus, r);
        } else {
            f.row_begin = std::min(H, r * slab);
            f.row_end = std::min(H, (r + 1) * slab);
            rows = f.row_end - f.row_begin;
        }
        img[r].resize((size_t)std::max(rows, 0) * W * 4);
    }
    const bool distinct = gpus <= ndev;
    if (gather == 1 && !distinct)
        return fail("arguments", RT_E_ARG, "--gather rccl needs one GPU per context (-g <= the GPU count)");
    if (gather == 1 || (gather == -1 && gpus > 1 && distinct))
        return render_rccl(ctx, part, img, W, H, band, dev0, ndev, frames, stats, out, scene);
    if (gpus > 1)
        std::printf("[ETAT]: gather: host (%d contexts on %d GPU(s)%s)\n", gpus, ndev,
                    distinct ? ", --gather host" : "; RCCL needs one rank per GPU");
    std::printf("[ETAT]: Lancer de rayons...\n");
    double total = 0.0;
    std::vector<int> rcs((size_t)gpus, 0);
    for (int k = 0; k < frames; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        if (gpus == 1) {
            rcs[0] = rt_render(ctx[0], &part[0], img[0].data());
        } else {
            std::vector<std::thread> th;
            for (int r = 0; r < gpus; ++r)
                th.emplace_back([&, r] { rcs[r] = img[r].empty() ? 0 : rt_render(ctx[r], &part[r], img[r].data()); });
            for (auto& t : th) t.join();
        }
        const auto t1 = std::chrono::steady_clock::now();
        for (int r = 0; r < gpus; ++r)
            if (rcs[r]) return fail("LancerRayons", rcs[r], rt_last_error(ctx[r]));
        total += std::chrono::duration<double>(t1 - t0).count();
    }
    // the frame, bottom row first (memory row 0 = bottom scanline)
    std::vector<uint8_t> full((size_t)W * H * 4);
    for (int r = 0; r < gpus; ++r) {
        const size_t rowb = (size_t)W * 4;
        if (band) {
            const int q = (int)(img[r].size() / rowb) / band;
            for (int j = 0; j < q; ++j) {
                const int y0 = (j * gpus + r) * band;
                const int n = std::min(band, H - y0);
                if (n > 0) std::memcpy(&full[(size_t)y0 * rowb], &img[r][(size_t)j * band * rowb], (size_t)n * rowb);
            }
        } else if (!img[r].empty()) {
            std::memcpy(&full[(size_t)part[r].row_begin * rowb], img[r].data(), img[r].size());
        }
    }
    print_done(ctx[0], total, frames, gpus, band, stats);
    if (out && write_ppm(out, W, H, full)) return fail("fopen", -1, out);
    for (rt_ctx* c : ctx) rt_destroy(c);
    rt_scene_destroy(scene);
    return 0;
}
