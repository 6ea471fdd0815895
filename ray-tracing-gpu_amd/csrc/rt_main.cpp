// rt_main.cpp — headless counterpart of the reference's Main.cpp entry point.
//
//   rt_render <scene.dat> [-x W] [-y H] [-d depth] [-o out.ppm] [-g device]
//             [-n frames] [-s]
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
// commented out), -g picks the HIP device, -n renders N frames (the scene is
// prepared once, unlike LancerRayons which re-runs Pretraitement), -s prints
// ray counters.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/rt.h"

static int fail(const char* what, int rc, const char* msg)
{
    std::fprintf(stderr, "[ERREUR]: %s (code %d): %s\n", what, rc, msg ? msg : "");
    return 1;
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        std::fprintf(stderr, "[ERREUR]: Aucune fichier de scene ne fut passe en argument !\n");
        return 1;
    }
    int W = 512, H = 256, depth = 0, dev = 0, frames = 1;
    bool stats = false;
    const char* out = nullptr;
    for (int i = 2; i < argc; ++i) {
        if (argv[i][0] != '-') continue;
        auto next = [&](int& v) {
            if (i + 1 < argc) v = std::atoi(argv[++i]);
        };
        switch (argv[i][1]) {
        case 'x': next(W); break;
        case 'y': next(H); break;
        case 'd': next(depth); break;
        case 'g': next(dev); break;
        case 'n': next(frames); break;
        case 's': stats = true; break;
        case 'o':
            if (i + 1 < argc) out = argv[++i];
            break;
        }
    }
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

    rt_ctx* ctx = nullptr;
    if ((rc = rt_create(dev, &ctx))) return fail("rt_create", rc, ctx ? rt_last_error(ctx) : "");
    rt_scene_flat flat;
    rt_scene_get_flat(scene, &flat);
    if ((rc = rt_upload_scene(ctx, &flat))) return fail("rt_upload_scene", rc, rt_last_error(ctx));
    rt_frame frame;
    rt_scene_get_frame(scene, &frame);
    if (stats) frame.flags |= RT_FLAG_STATS;

    std::vector<uint8_t> img((size_t)W * H * 4);
    std::printf("[ETAT]: Lancer de rayons...\n");
    double total = 0.0;
    for (int f = 0; f < frames; ++f) {
        const auto t0 = std::chrono::steady_clock::now();
        if ((rc = rt_render(ctx, &frame, img.data()))) return fail("LancerRayons", rc, rt_last_error(ctx));
        const auto t1 = std::chrono::steady_clock::now();
        total += std::chrono::duration<double>(t1 - t0).count();
    }
    rt_stats st;
    rt_last_stats(ctx, &st);
    std::printf("[ETAT]: Termine! --> Temps total de rendu : %.6f secondes (%d frame(s), kernel %.3f ms)\n",
                total, frames, st.kernel_ms);
    if (stats)
        std::printf("[STATS]: primary=%llu bounce=%llu shadow=%llu shadow_tests_skipped=%llu stack=%d "
                    "tests: triangle=%llu plane=%llu quadric=%llu\n",
                    (unsigned long long)st.primary_rays, (unsigned long long)st.bounce_rays,
                    (unsigned long long)st.shadow_rays, (unsigned long long)st.shadow_tests_skipped,
                    st.stack_depth, (unsigned long long)st.triangle_tests, (unsigned long long)st.plane_tests,
                    (unsigned long long)st.quadric_tests);
    if (out) {
        FILE* f = std::fopen(out, "wb");
        if (!f) return fail("fopen", -1, out);
        std::fprintf(f, "P6\n%d %d\n255\n", W, H);
        for (int y = H - 1; y >= 0; --y)  // memory row 0 = bottom scanline
            for (int x = 0; x < W; ++x) std::fwrite(&img[((size_t)y * W + x) * 4], 1, 3, f);
        std::fclose(f);
        std::printf("[ETAT]: Image ecrite dans %s\n", out);
    }
    rt_destroy(ctx);
    rt_scene_destroy(scene);
    return 0;
}
