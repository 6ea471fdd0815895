// rt_scene.cpp — host CScene mirror: .dat loader, camera, Pretraitement,
// flattening, and the rt_scene_* half of the C ABI (include/rt.h).
//
// Behavioural contract = the reference's, including its quirks (each pinned by
// tests/test_host_scene.py against the oracle and the golden fixtures):
//  * lines are read like istream::getline(Line, 80) (Scene.cpp:251, Scene.h:86):
//    a line of >= 80 characters makes the reference spin forever; we return
//    RT_E_PARSE instead;
//  * CStringUtils::Trim's result is discarded (Scene.cpp:254), so a comment is
//    a line whose first RAW character is '*';
//  * keywords match anywhere in the line (STRING_CHECKFIND, Scene.cpp:39);
//  * the sscanf targets R,G,B,Val0..2 live across lines, so a failed
//    conversion reuses the previous line's value (Scene.cpp:245-246);
//  * generic surface keys win over type-specific ones (Scene.cpp:320-385).
#include "rt_scene.hpp"

#include <cstdio>
#include <cstring>
#include <new>

#pragma clang fp contract(off)

namespace rt {

// ------------------------------------------------------------ Pretraitement
void Surface::Pretraitement()
{
    switch (kind) {
    case SurfaceKind::Triangle: {  // Triangle.cpp:108-113, CalculerNormale :199-204
        for (auto& p : pts) p = p * xform;
        normal = normalize(cross(pts[1] - pts[0], pts[2] - pts[0]));
        break;
    }
    case SurfaceKind::Plane: {  // Plan.cpp:101-114 — the normal goes through the full affine xform
        normal = normalize(normal * xform);
        float p[3] = {0.f, 0.f, 0.f};
        const float n[3] = {normal.x, normal.y, normal.z};
        for (int i = 0; i < 3; ++i)
            if (n[i] != 0) p[i] = -(cst / n[i]);
        const Vec3 pt = make3(p[0], p[1], p[2]) * xform;
        cst = dot(-normal, pt);
        break;
    }
    case SurfaceKind::Quadric: {  // Quadrique.cpp:110-146 (Goldman, Q' = M^-1 Q M^-T)
        const float D = mix.z * 0.5f, E = mix.x * 0.5f, F = mix.y * 0.5f;
        const float G = lin.x * 0.5f, H = lin.y * 0.5f, J = lin.z * 0.5f;
        Mat4 Q{{{quad.x, D, F, G}, {D, quad.y, E, H}, {F, E, quad.z, J}, {G, H, J, cst}}};
        const Mat4 inv = inverse(xform);
        Q = (inv * Q) * transpose(inv);
        quad = make3(Q.m[0][0], Q.m[1][1], Q.m[2][2]);
        cst = Q.m[3][3];
        mix = make3(Q.m[1][2] * 2.0f, Q.m[0][2] * 2.0f, Q.m[0][1] * 2.0f);
        lin = make3(Q.m[0][3] * 2.0f, Q.m[1][3] * 2.0f, Q.m[2][3] * 2.0f);
        break;
    }
    }
}

// Matrice4.h:362-440 — all transforms compose POST: M = M * T.
static void post_rotate(Mat4& m, float rx, float ry, float rz)
{
    Mat4 t = identity4();
    t.m[1][1] = cosf(rx);
    t.m[1][2] = sinf(rx);
    t.m[2][2] = t.m[1][1];
    t.m[2][1] = -t.m[1][2];
    m = m * t;
    t = identity4();
    t.m[0][0] = cosf(ry);
    t.m[0][2] = -sinf(ry);
    t.m[2][2] = t.m[0][0];
    t.m[2][0] = -t.m[0][2];
    m = m * t;
    t = identity4();
    t.m[0][0] = cosf(rz);
    t.m[0][1] = sinf(rz);
    t.m[1][1] = t.m[0][0];
    t.m[1][0] = -t.m[0][1];
    m = m * t;
}
static void post_translate(Mat4& m, float x, float y, float z)
{
    Mat4 t = identity4();
    t.m[3][0] = x;
    t.m[3][1] = y;
    t.m[3][2] = z;
    m = m * t;
}
static void post_scale(Mat4& m, float x, float y, float z)
{
    Mat4 t = identity4();
    t.m[0][0] = x;
    t.m[1][1] = y;
    t.m[2][2] = z;
    m = m * t;
}

// ------------------------------------------------------------------ loader
namespace {
enum class State { Scene, Light, Triangle, Plane, Quadric };

// istream::getline(buf, 80): 0 = got a line, 1 = end of file, -1 = too long.
int read_line(FILE* f, char (&buf)[80], bool& at_eof)
{
    int n = 0;
    for (;;) {
        const int c = std::fgetc(f);
        if (c == EOF) {
            at_eof = true;
            break;
        }
        if (c == '\n') break;
        if (n == 79) return -1;
        buf[n++] = (char)c;
    }
    buf[n] = 0;
    return 0;
}
inline bool has(const char* line, const char* key) { return std::strstr(line, key) != nullptr; }
}  // namespace

int Scene::TraiterFichierDeScene(const char* path)
{
    FILE* f = std::fopen(path, "rb");
    if (!f) {
        error = std::string("cannot open scene file ") + path;
        return RT_E_IO;
    }
    State state = State::Scene;
    Surface* surf = nullptr;
    Light* light = nullptr;
    char line[80];
    char word[80];
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    int R = 0, G = 0, B = 0;
    bool at_eof = false;
    // Objects are appended when created; the reference appends them when the
    // next object keyword (or EOF) arrives, which yields the same order.
    std::vector<Surface> out_s;
    std::vector<Light> out_l;
    auto finish = [&]() {
        if (surf) out_s.push_back(*surf);
        if (light) out_l.push_back(*light);
    };
    Surface cur_s{};
    Light cur_l{};
    while (!at_eof) {
        if (read_line(f, line, at_eof) < 0) {
            std::fclose(f);
            error = "scene line longer than 79 characters: the reference's getline(Line, 80) "
                    "sets failbit and its while(!eof()) loop never ends";
            return RT_E_PARSE;
        }
        if (line[0] == 0 || line[0] == '*') continue;

        State next = state;
        bool is_new = true;
        if (has(line, "Lumiere:")) next = State::Light;
        else if (has(line, "Poly:")) next = State::Triangle;
        else if (has(line, "Plane:")) next = State::Plane;
        else if (has(line, "Quad:")) next = State::Quadric;
        else is_new = false;

        if (is_new) {
            finish();
            surf = nullptr;
            light = nullptr;
            state = next;
            switch (state) {
            case State::Light: cur_l = Light{}; light = &cur_l; break;
            case State::Triangle: cur_s = Surface{SurfaceKind::Triangle}; surf = &cur_s; break;
            case State::Plane: cur_s = Surface{SurfaceKind::Plane}; surf = &cur_s; break;
            case State::Quadric: cur_s = Surface{SurfaceKind::Quadric}; surf = &cur_s; break;
            default: break;
            }
            continue;
        }

        if (surf) {  // Scene.cpp:320-385 generic surface keys
            bool generic = true;
            Material& m = surf->mat;
            if (has(line, "color:")) {
                std::sscanf(line, "%s %i %i %i", word, &R, &G, &B);
                m.color = rgb_from_int(R, G, B);
            } else if (has(line, "ambient:")) {
                std::sscanf(line, "%s %f", word, &v0);
                m.ka = v0;
            } else if (has(line, "diffus:")) {
                std::sscanf(line, "%s %f", word, &v0);
                m.kd = v0;
            } else if (has(line, "specular:")) {
                std::sscanf(line, "%s %f %f", word, &v0, &v1);
                m.ks = v0;
                m.shininess = v1;
            } else if (has(line, "reflect:")) {
                std::sscanf(line, "%s %f", word, &v0);
                m.kr = v0;
            } else if (has(line, "refract:")) {
                std::sscanf(line, "%s %f %f", word, &v0, &v1);
                m.kt = v0;
                m.ior = v1;
            } else if (has(line, "rotate:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                post_rotate(surf->xform, deg2rad(v0), deg2rad(v1), deg2rad(v2));
            } else if (has(line, "translate:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                post_translate(surf->xform, v0, v1, v2);
            } else if (has(line, "scale:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                post_scale(surf->xform, v0, v1, v2);
            } else {
                generic = false;
            }
            if (generic) continue;
        }

        switch (state) {
        case State::Scene:  // Scene.cpp:392-411
            if (has(line, "background:")) {
                std::sscanf(line, "%s %i %i %i", word, &R, &G, &B);
                background = rgb_from_int(R, G, B);
            } else if (has(line, "origin:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                cam_pos = make3(v0, v1, v2);
            } else if (has(line, "eye:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                cam_eye = make3(v0, v1, v2);
            } else if (has(line, "up:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                cam_up = make3(v0, v1, v2);
            }
            break;
        case State::Light:  // Scene.cpp:418-431
            if (has(line, "position:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                light->pos = make3(v0, v1, v2);
            } else if (has(line, "intens:")) {
                std::sscanf(line, "%s %f", word, &v0);
                light->intensity = v0;
            } else if (has(line, "color:")) {
                std::sscanf(line, "%s %i %i %i", word, &R, &G, &B);
                light->color = rgb_from_int(R, G, B);
            }
            break;
        case State::Triangle:  // Scene.cpp:438-443
            if (has(line, "point:")) {
                int idx = -1;
                std::sscanf(line, "%s %i %f %f %f", word, &idx, &v0, &v1, &v2);
                if (idx < 0 || idx > 2) {  // Triangle.h:56 assert
                    std::fclose(f);
                    error = "triangle 'point:' index outside 0..2";
                    return RT_E_PARSE;
                }
                surf->pts[idx] = make3(v0, v1, v2);
            }
            break;
        case State::Plane:  // Scene.cpp:449-458
            if (has(line, "v_linear:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                surf->normal = make3(v0, v1, v2);
            } else if (has(line, "v_const:")) {
                std::sscanf(line, "%s %f", word, &v0);
                surf->cst = v0;
            }
            break;
        case State::Quadric:  // Scene.cpp:464-483
            if (has(line, "v_quad:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                surf->quad = make3(v0, v1, v2);
            } else if (has(line, "v_mixte:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                surf->mix = make3(v0, v1, v2);
            } else if (has(line, "v_linear:")) {
                std::sscanf(line, "%s %f %f %f", word, &v0, &v1, &v2);
                surf->lin = make3(v0, v1, v2);
            } else if (has(line, "v_const:")) {
                std::sscanf(line, "%s %f", word, &v0);
                surf->cst = v0;
            }
            break;
        }
    }
    std::fclose(f);
    finish();  // Scene.cpp:495-496
    surfaces.insert(surfaces.end(), out_s.begin(), out_s.end());
    lights.insert(lights.end(), out_l.begin(), out_l.end());
    loaded = true;
    return RT_OK;
}

// Scene.cpp:624-660
void Scene::InitialiserCamera()
{
    const float kDimFilm = 0.024f;  // Scene.cpp:42 DIM_FILM_CAM
    const float d2 = norm(cam_pos - cam_eye);
    const float y2 = (d2 / (focale * 0.001f) - 1) * kDimFilm;
    angle = (360 * atan2f(y2 * 0.5f, d2)) / kPi;
    const Vec3 N = normalize(cam_pos - cam_eye);
    const Vec3 V = normalize(cam_up - N * dot(cam_up, N));
    const Vec3 U = cross(V, N);
    orientation = Mat4{{{U.x, U.y, U.z, 0.0f}, {V.x, V.y, V.z, 0.0f}, {N.x, N.y, N.z, 0.0f}, {0.0f, 0.0f, 0.0f, 1.0f}}};
}

// Scene.cpp:140-147 Initialiser + the LancerRayons prologue (:676-679).
// The reference runs Pretraitement inside every LancerRayons call, which
// transforms the geometry again on a second frame; here it runs once.
int Scene::Initialiser()
{
    if (!loaded) {
        error = "rt_scene_prepare before rt_scene_load_file";
        return RT_E_STATE;
    }
    if (prepared) return RT_OK;
    if (width <= 0 || height <= 0) {
        error = "resolution not set (rt_scene_set_resolution)";
        return RT_E_ARG;
    }
    InitialiserCamera();
    for (auto& s : surfaces) s.Pretraitement();
    half_h = tanf(deg2rad(angle * 0.5f));
    half_w = ((float)width / height) * half_h;
    inv_w = 1.0f / width;
    inv_h = 1.0f / height;
    prepared = true;
    Flatten();
    return RT_OK;
}

void Scene::Flatten()
{
    const size_t n = surfaces.size();
    flat_type.assign(n, 0);
    flat_geom.assign(n * 12, 0.0f);
    flat_mat.assign(n * 10, 0.0f);
    for (size_t i = 0; i < n; ++i) {
        const Surface& s = surfaces[i];
        flat_type[i] = (int32_t)s.kind;
        float* g = &flat_geom[i * 12];
        switch (s.kind) {
        case SurfaceKind::Triangle:
            for (int k = 0; k < 3; ++k) {
                g[3 * k] = s.pts[k].x;
                g[3 * k + 1] = s.pts[k].y;
                g[3 * k + 2] = s.pts[k].z;
            }
            g[9] = s.normal.x; g[10] = s.normal.y; g[11] = s.normal.z;
            break;
        case SurfaceKind::Plane:
            g[0] = s.normal.x; g[1] = s.normal.y; g[2] = s.normal.z; g[3] = s.cst;
            break;
        case SurfaceKind::Quadric:
            g[0] = s.quad.x; g[1] = s.quad.y; g[2] = s.quad.z;
            g[3] = s.lin.x; g[4] = s.lin.y; g[5] = s.lin.z;
            g[6] = s.mix.x; g[7] = s.mix.y; g[8] = s.mix.z;
            g[9] = s.cst;
            break;
        }
        float* m = &flat_mat[i * 10];
        m[0] = s.mat.color.r; m[1] = s.mat.color.g; m[2] = s.mat.color.b;
        m[3] = s.mat.ka; m[4] = s.mat.kd; m[5] = s.mat.ks; m[6] = s.mat.shininess;
        m[7] = s.mat.kr; m[8] = s.mat.kt; m[9] = s.mat.ior;
    }
    flat_lights.assign(lights.size() * 7, 0.0f);
    for (size_t j = 0; j < lights.size(); ++j) {
        float* l = &flat_lights[j * 7];
        l[0] = lights[j].pos.x; l[1] = lights[j].pos.y; l[2] = lights[j].pos.z;
        l[3] = lights[j].color.r; l[4] = lights[j].color.g; l[5] = lights[j].color.b;
        l[6] = lights[j].intensity;
    }
}

}  // namespace rt

// ------------------------------------------------------------------ C ABI
struct rt_scene {
    rt::Scene s;
};

#define RT_EXPORT extern "C" __attribute__((visibility("default")))

RT_EXPORT int rt_abi_version(void) { return RT_ABI_VERSION; }

RT_EXPORT int32_t rt_band_rows(int32_t height, int32_t band_rows, int32_t band_count, int32_t band_index)
{
    if (height < 0 || band_rows <= 0 || band_rows % 16 != 0 || band_count <= 0 || band_index < 0 ||
        band_index >= band_count)
        return -1;
    const int64_t nb = ((int64_t)height + band_rows - 1) / band_rows;  // bands in the frame
    const int64_t mine = nb > band_index ? (nb - band_index + band_count - 1) / band_count : 0;
    return (int32_t)(mine * band_rows);
}

RT_EXPORT int rt_scene_create(rt_scene** out)
{
    if (!out) return RT_E_ARG;
    *out = new (std::nothrow) rt_scene();
    return *out ? RT_OK : RT_E_ARG;
}
RT_EXPORT void rt_scene_destroy(rt_scene* s) { delete s; }
RT_EXPORT const char* rt_scene_error(const rt_scene* s) { return s ? s->s.error.c_str() : "null scene"; }

RT_EXPORT int rt_scene_set_resolution(rt_scene* s, int32_t w, int32_t h)
{
    if (!s || w <= 0 || h <= 0) return RT_E_ARG;
    if (s->s.prepared && (w != s->s.width || h != s->s.height)) {
        s->s.error = "resolution changed after rt_scene_prepare";
        return RT_E_STATE;
    }
    s->s.width = w;
    s->s.height = h;
    return RT_OK;
}
RT_EXPORT int rt_scene_set_max_bounces(rt_scene* s, int32_t n)
{
    if (!s || n < 0) return RT_E_ARG;
    s->s.max_bounces = n;
    return RT_OK;
}
RT_EXPORT int rt_scene_set_min_energy(rt_scene* s, float e)
{
    if (!s) return RT_E_ARG;
    s->s.min_energy = e;
    return RT_OK;
}
RT_EXPORT int rt_scene_set_scene_ior(rt_scene* s, float ior)
{
    if (!s) return RT_E_ARG;
    s->s.scene_ior = ior;
    return RT_OK;
}
RT_EXPORT int rt_scene_load_file(rt_scene* s, const char* path)
{
    if (!s || !path) return RT_E_ARG;
    if (s->s.prepared) {
        s->s.error = "rt_scene_load_file after rt_scene_prepare";
        return RT_E_STATE;
    }
    return s->s.TraiterFichierDeScene(path);
}
RT_EXPORT int rt_scene_prepare(rt_scene* s)
{
    if (!s) return RT_E_ARG;
    return s->s.Initialiser();
}
RT_EXPORT int rt_scene_get_flat(const rt_scene* s, rt_scene_flat* out)
{
    if (!s || !out) return RT_E_ARG;
    if (!s->s.prepared) return RT_E_STATE;
    out->n_surfaces = (int32_t)s->s.surfaces.size();
    out->n_lights = (int32_t)s->s.lights.size();
    out->type = s->s.flat_type.data();
    out->geom = s->s.flat_geom.data();
    out->material = s->s.flat_mat.data();
    out->lights = s->s.flat_lights.data();
    return RT_OK;
}
RT_EXPORT int rt_scene_get_frame(const rt_scene* s, rt_frame* f)
{
    if (!s || !f) return RT_E_ARG;
    if (!s->s.prepared) return RT_E_STATE;
    const rt::Scene& S = s->s;
    std::memset(f, 0, sizeof *f);
    f->cam_pos[0] = S.cam_pos.x;
    f->cam_pos[1] = S.cam_pos.y;
    f->cam_pos[2] = S.cam_pos.z;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) f->orient[4 * i + j] = S.orientation.m[i][j];
    f->half_w = S.half_w;
    f->half_h = S.half_h;
    f->inv_w = S.inv_w;
    f->inv_h = S.inv_h;
    f->background[0] = S.background.r;
    f->background[1] = S.background.g;
    f->background[2] = S.background.b;
    f->width = S.width;
    f->height = S.height;
    f->row_begin = 0;
    f->row_end = S.height;
    f->max_bounces = S.max_bounces;
    f->min_energy = S.min_energy;
    f->scene_ior = S.scene_ior;
    f->flags = 0;
    return RT_OK;
}
