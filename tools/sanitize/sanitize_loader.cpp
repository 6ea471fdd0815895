// sanitize_loader.cpp — host AddressSanitizer / UBSan run of the code that
// parses untrusted scene text: the product's loader + Pretraitement
// (ray-tracing-gpu_amd/csrc/rt_scene.cpp, through rt.h's rt_scene_* calls)
// and the oracle restatement (oracle/rt_oracle.c, loader + a small render).
// Built by `make -C tools/sanitize` with -fsanitize=address,undefined
// -fno-sanitize-recover=all: any report aborts with a non-zero status.
//
//   sanitize_loader <mutations per file> <scene.dat>...
//
// Every file is loaded as is, then in `mutations` deterministic variants:
// random byte flips, truncations, duplicated and deleted lines, a line of
// >= 80 characters, huge / NaN / negative numbers, out-of-range point
// indices, CR line ends.  Errors are expected and fine (RT_E_PARSE, ...);
// only memory and UB errors fail.
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt.h"

extern "C" {
struct oracle_scene;
int oracle_load(const char* path, int w, int h, int max_bounces, oracle_scene** out);
int oracle_render_window(oracle_scene* S, int row0, int row1, int col0, int col1, float* rgb, int nthreads);
int oracle_counts(oracle_scene* S, int* nsurf, int* nlights);
int oracle_dump(oracle_scene* S, float* surf, float* cam, float* lights);
void oracle_free(oracle_scene* S);
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd()
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static std::string slurp(const char* p)
{
    std::string s;
    FILE* f = std::fopen(p, "rb");
    if (!f) return s;
    char buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    std::fclose(f);
    return s;
}

static std::string mutate(const std::string& src)
{
    std::string s = src;
    static const char* inserts[] = {"1e39", "nan", "-inf", "-2147483648", "99999999999999999999", "0x", "point: 7 1 2 3",
                                    "point: -1 0 0 0", "Poly:", "Quad:", "Plane:", "Lumiere:", "color:", "\r",
                                    "scale: 0 0 0", "rotate: 1e30 -1e30 nan", "specular: 1 -3", "up: 0 0 0"};
    const int ops = 1 + (int)(rnd() % 4);
    for (int k = 0; k < ops; ++k) {
        const size_t at = s.empty() ? 0 : (size_t)(rnd() % s.size());
        switch (rnd() % 7) {
        case 0:  // byte flip
            if (!s.empty()) s[at] = (char)(rnd() & 0xFF);
            break;
        case 1:  // truncate
            s.resize(at);
            break;
        case 2: {  // duplicate a line
            const size_t b = s.rfind('\n', at), e = s.find('\n', at);
            const size_t b0 = b == std::string::npos ? 0 : b + 1, e0 = e == std::string::npos ? s.size() : e + 1;
            s.insert(e0, s.substr(b0, e0 - b0));
            break;
        }
        case 3: {  // delete a line
            const size_t b = s.rfind('\n', at), e = s.find('\n', at);
            const size_t b0 = b == std::string::npos ? 0 : b + 1, e0 = e == std::string::npos ? s.size() : e + 1;
            s.erase(b0, e0 - b0);
            break;
        }
        case 4:  // long line
            s.insert(at, std::string(80 + rnd() % 40, 'x') + "\n");
            break;
        default:  // a token
            s.insert(at, std::string(" ") + inserts[rnd() % (sizeof inserts / sizeof *inserts)] + " ");
            break;
        }
    }
    return s;
}

static int runs = 0, loaded = 0;

static void check(const char* path)
{
    ++runs;
    // the product's host CScene mirror
    rt_scene* sc = nullptr;
    if (rt_scene_create(&sc) == 0) {
        rt_scene_set_resolution(sc, 24, 16);
        rt_scene_set_max_bounces(sc, 2);
        if (rt_scene_load_file(sc, path) == 0 && rt_scene_prepare(sc) == 0) {
            rt_scene_flat fl;
            rt_frame fr;
            if (rt_scene_get_flat(sc, &fl) == 0 && rt_scene_get_frame(sc, &fr) == 0) {
                volatile float acc = 0.f;
                for (int i = 0; i < fl.n_surfaces; ++i) {
                    acc += (float)fl.type[i];
                    for (int k = 0; k < 12; ++k) acc += fl.geom[12 * i + k];
                    for (int k = 0; k < 10; ++k) acc += fl.material[10 * i + k];
                }
                for (int j = 0; j < 7 * fl.n_lights; ++j) acc += fl.lights[j];
                (void)acc;
                ++loaded;
            }
        } else {
            (void)rt_scene_error(sc);
        }
        rt_scene_destroy(sc);
    }
    // the oracle restatement: loader, dump and one 8x8 window
    oracle_scene* o = nullptr;
    if (oracle_load(path, 24, 16, 2, &o) == 0 && o) {
        int ns = 0, nl = 0;
        oracle_counts(o, &ns, &nl);
        if (ns < 4096) {
            std::vector<float> s((size_t)ns * 24 + 1), c(27), l((size_t)nl * 7 + 1);
            oracle_dump(o, s.data(), c.data(), l.data());
            std::vector<float> img(8 * 8 * 3);
            oracle_render_window(o, 4, 12, 8, 16, img.data(), 1);
        }
    }
    if (o) oracle_free(o);
}

int main(int argc, char** argv)
{
    if (argc < 3) {
        std::fprintf(stderr, "usage: sanitize_loader <mutations> <scene.dat>...\n");
        return 2;
    }
    const int muts = std::atoi(argv[1]);
    const char* tmpdir = std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp";
    char tmp[4096];
    std::snprintf(tmp, sizeof tmp, "%s/sanitize_loader_%d.dat", tmpdir, (int)getpid());
    for (int a = 2; a < argc; ++a) {
        check(argv[a]);
        const std::string src = slurp(argv[a]);
        for (int m = 0; m < muts; ++m) {
            const std::string v = mutate(src);
            FILE* f = std::fopen(tmp, "wb");
            if (!f) return 2;
            std::fwrite(v.data(), 1, v.size(), f);
            std::fclose(f);
            check(tmp);
        }
    }
    std::remove(tmp);
    std::printf("sanitize_loader: %d files loaded and rendered, %d parsed by the product, no sanitizer report\n", runs,
                loaded);
    return 0;
}
