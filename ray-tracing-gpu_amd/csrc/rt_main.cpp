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

// The RCCL path of -g N (N distinct GPUs): every rank renders its part into
// device memory on its own GPU (rt_render_async on the rank's gather
// stream), then one RCCL group gathers the parts into the root GPU's frame —
// a slab is one chunk, a band set one chunk per 16-row band (each lands at
// its rows of the frame) — and the root's frame is copied to the host once.
// Timed: the whole frame (renders + gather) and, separately, the gather.
static int render_rccl(std::vector<rt_ctx*>& ctx, std::vector<rt_frame>& part,
                       const std::vector<std::vector<uint8_t>>& img, int W, int H, int band, int dev0, int ndev,
                       int frames, bool stats, const char* out, rt_scene* scene)
{
    const int n = (int)ctx.size();
    std::vector<int32_t> devs((size_t)n);
    for (int r = 0; r < n; ++r) devs[r] = (dev0 + r) % ndev;
    rt_gather* g = nullptr;
    int rc = rt_gather_create(n, devs.data(), &g);
    if (rc) return fail("rt_gather_create", rc, rt_gather_error(g));
    const size_t rowb = (size_t)W * 4;
    std::vector<void*> slab((size_t)n, nullptr);
    void* full = nullptr;
    std::vector<rt_gather_chunk> ch;
    for (int r = 0; r < n; ++r) {
        (void)hipSetDevice(devs[r]);
        if (!img[r].empty() && hipMalloc(&slab[r], img[r].size()) != hipSuccess)
            return fail("hipMalloc", RT_E_HIP, "slab");
        if (r == 0 && hipMalloc(&full, rowb * H) != hipSuccess) return fail("hipMalloc", RT_E_HIP, "frame");
        if (img[r].empty()) continue;
        if (band) {  // packed band j of rank r -> frame rows (j n + r) band ...
            const int q = (int)(img[r].size() / rowb) / band;
            for (int j = 0; j < q; ++j) {
                const int y0 = (j * n + r) * band, rows = std::min(band, H - y0);
                if (rows > 0)
                    ch.push_back({r, (const char*)slab[r] + (size_t)j * band * rowb, (size_t)rows * rowb, (size_t)y0 * rowb});
            }
        } else {
            ch.push_back({r, slab[r], img[r].size(), (size_t)part[r].row_begin * rowb});
        }
    }
    size_t gbytes = 0;
    for (const auto& c : ch) gbytes += c.bytes;
    const int ver = rt_gather_rccl_version();
    std::printf("[ETAT]: gather: RCCL %d.%d.%d, %d rank(s), %zu chunk(s), %.1f MB into GPU %d\n", ver / 10000,
                (ver / 100) % 100, ver % 100, n, ch.size(), gbytes / 1e6, devs[0]);
    std::printf("[ETAT]: Lancer de rayons...\n");
    double total = 0.0, gtotal = 0.0;
    for (int k = 0; k < frames; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < n; ++r) {
            if (img[r].empty()) continue;
            if ((rc = rt_render_async(ctx[r], &part[r], (uint8_t*)slab[r], nullptr, rt_gather_stream(g, r))))
                return fail("LancerRayons", rc, rt_last_error(ctx[r]));
        }
        if ((rc = rt_gather_sync(g))) return fail("rt_gather_sync", rc, rt_gather_error(g));
        const auto t1 = std::chrono::steady_clock::now();
        if ((rc = rt_gather_chunks(g, (int32_t)ch.size(), ch.data(), full)))
            return fail("rt_gather_chunks", rc, rt_gather_error(g));
        if ((rc = rt_gather_sync(g))) return fail("rt_gather_sync", rc, rt_gather_error(g));
        const auto t2 = std::chrono::steady_clock::now();
        total += std::chrono::duration<double>(t2 - t0).count();
        gtotal += std::chrono::duration<double>(t2 - t1).count();
    }
    std::vector<uint8_t> host(rowb * H);
    (void)hipSetDevice(devs[0]);
    if (hipMemcpy(host.data(), full, host.size(), hipMemcpyDeviceToHost) != hipSuccess)
        return fail("hipMemcpy", RT_E_HIP, "frame to host");
    std::printf("[ETAT]: gather: %.3f ms per frame (RCCL group of %zu send/recv pair(s))\n", gtotal * 1e3 / frames,
                ch.size());
    print_done(ctx[0], total, frames, n, band, stats);
    if (out && write_ppm(out, W, H, host)) return fail("fopen", -1, out);
    for (int r = 0; r < n; ++r) {
        (void)hipSetDevice(devs[r]);
        (void)hipFree(slab[r]);
    }
    (void)hipSetDevice(devs[0]);
    (void)hipFree(full);
    rt_gather_destroy(g);
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
